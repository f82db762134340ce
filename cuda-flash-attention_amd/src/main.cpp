// main.cpp -- the FlashAttention CLI: file in, file out.
//
// Contract of detker/CUDA-Flash-Attention src/main.cpp:14-135:
//   FlashAttention <naive|fa1|fa2> <forward|backward|forward_backward> <fp16|fp32|bf16> <dir/B{b}_H{h}_S{s}_D{d}>
// reads Q.bin K.bin V.bin (+ O.bin logsumexp.bin in backward mode; dO.bin if
// present, else dO = 1), writes O.bin logsumexp.bin and/or dQ.bin dK.bin dV.bin
// into the same directory, and prints the kernel-only time (TimerManager).
// Element counts are size_t here (the reference's int qkv_size caps at 2^31).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dispatcher.h"
#include "timer.h"
#include "utils.h"

int main(int argc, char** argv) {
    ComputeType method;
    ModeType mode;
    ComputeDataType precision;
    char* data_path;
    parse_args(argc, argv, &precision, &method, &mode, &data_path);

    int B, H, S, D;
    parse_config_string(data_path, &B, &H, &S, &D);
    check_method_support(method, mode, precision);

    const size_t n = (size_t)B * H * S * D;
    const size_t nl = (size_t)B * H * S;
    printf("Batch size:    %d\n", B);
    printf("Num heads:     %d\n", H);
    printf("Sequence len:  %d\n", S);
    printf("Head dim:      %d\n", D);

    const bool bwd = mode == ModeType::Backward || mode == ModeType::ForwardBackward;
    std::vector<float> q(n), k(n), v(n), o(n), lse(nl), dout, dq, dk, dv;
    if (bwd) {
        dout.resize(n);
        dq.resize(n);
        dk.resize(n);
        dv.resize(n);
    }
    const std::string dir(data_path);
    auto path = [&](const char* f) { return dir + "/" + f; };

    bool have = file_exists(path("Q.bin").c_str()) && file_exists(path("K.bin").c_str()) &&
                file_exists(path("V.bin").c_str());
    if (mode == ModeType::Backward)
        have = have && file_exists(path("O.bin").c_str()) && file_exists(path("logsumexp.bin").c_str());
    if (!have) ERR("Data files not found.\n");

    printf("Loading data...\n");
    load_binary_file(path("Q.bin").c_str(), q.data(), n);
    load_binary_file(path("K.bin").c_str(), k.data(), n);
    load_binary_file(path("V.bin").c_str(), v.data(), n);
    if (mode == ModeType::Backward) {
        load_binary_file(path("O.bin").c_str(), o.data(), n);
        load_binary_file(path("logsumexp.bin").c_str(), lse.data(), nl);
    }
    if (bwd) {
        if (file_exists(path("dO.bin").c_str())) load_binary_file(path("dO.bin").c_str(), dout.data(), n);
        else std::fill(dout.begin(), dout.end(), 1.0f);  // L = sum(O)  =>  dL/dO = 1
    }
    printf("Data loaded successfully.\n\n");

    // (argv and the input files are checked before the device timer is created, so
    // a bad command line or a missing/short file fails the same way without a GPU)
    TimerManager tm;
    TimerGPU timer_gpu;
    tm.SetTimer(&timer_gpu);
    printf("Running...\n");
    RunFlashAttention(q.data(), k.data(), v.data(), o.data(), lse.data(), bwd ? dout.data() : nullptr,
                      bwd ? dq.data() : nullptr, bwd ? dk.data() : nullptr, bwd ? dv.data() : nullptr, B, H, S, D,
                      precision, method, mode, &tm);
    printf("Kernel execution completed: %.4f seconds.\n\n", tm.TotalElapsedSeconds());

    printf("Saving output...\n");
    if (mode == ModeType::Forward || mode == ModeType::ForwardBackward) {
        save_binary_file(path("O.bin").c_str(), o.data(), n);
        save_binary_file(path("logsumexp.bin").c_str(), lse.data(), nl);
    }
    if (bwd) {
        save_binary_file(path("dQ.bin").c_str(), dq.data(), n);
        save_binary_file(path("dK.bin").c_str(), dk.data(), n);
        save_binary_file(path("dV.bin").c_str(), dv.data(), n);
    }
    printf("Output saved successfully.\n");
    return EXIT_SUCCESS;
}
