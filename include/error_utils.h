// error_utils.h -- error conventions of the reference CLI/host API, on HIP.
// Mirrors detker/CUDA-Flash-Attention include/error_utils.h:6-19: ERR() prints
// errno context and exits; the device-call check prints and exit(1)s; usage()
// prints the argv contract.  (The C ABI in fa2_amd.h returns codes instead.)
#pragma once

#include <cstdio>
#include <cstdlib>

#define ERR(source) (perror(source), fprintf(stderr, "%s:%d\n", __FILE__, __LINE__), exit(EXIT_FAILURE))

#define HIP_CHECK(call)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

inline void usage(char* name) {
    fprintf(stderr,
            "USAGE: %s <computation_method:naive|fa1|fa2> <mode:forward|backward|forward_backward> "
            "<SHM_precision:fp16|fp32|bf16> <data_folder_path>\n",
            name);
    exit(EXIT_FAILURE);
}
