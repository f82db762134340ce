// capi_check.cpp -- host-side checks of csrc/capi.cpp built with AddressSanitizer
// (make -C cuda-flash-attention_amd asan; run by tests/test_asan_cpu.py).
//
// Exercises every C-ABI path that needs no GPU: the shard rule over a grid of
// arguments, argument validation of every entry point (null pointers, bad shapes,
// 32-bit overflow guards, bad precision), the thread-local error string, the
// launch-plan override table under concurrent writers and readers, and the host
// API's error path when no device is visible (it must return a code, free what it
// took and never exit).  Exit status 0 = every check held; ASan aborts on a memory
// error.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fa2_amd.h"

namespace fa2 {
int tune_knob(const char* name, int dflt);
}

static int g_failed = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_failed;                                                   \
        }                                                                 \
    } while (0)

static void shard_rule() {
    for (int total = 0; total <= 70; ++total)
        for (int shards = 1; shards <= 9; ++shards) {
            int next = 0, lo = 1 << 30, hi = -1;
            for (int i = 0; i < shards; ++i) {
                int first = -1, count = -1;
                CHECK(fa2_shard_range(total, shards, i, &first, &count) == FA2_OK);
                CHECK(first == next);  // contiguous, in order
                next = first + count;
                lo = count < lo ? count : lo;
                hi = count > hi ? count : hi;
            }
            CHECK(next == total);  // covers every head once
            CHECK(hi - lo <= 1);   // balanced
        }
    int f = 0, c = 0;
    CHECK(fa2_shard_range(8, 0, 0, &f, &c) == FA2_E_INVALID);
    CHECK(fa2_shard_range(8, 2, 2, &f, &c) == FA2_E_INVALID);
    CHECK(fa2_shard_range(8, 2, -1, &f, &c) == FA2_E_INVALID);
    CHECK(fa2_shard_range(-1, 2, 0, &f, &c) == FA2_E_INVALID);
    CHECK(fa2_shard_range(8, 2, 0, nullptr, &c) == FA2_E_INVALID);
    CHECK(fa2_shard_range(8, 2, 0, &f, nullptr) == FA2_E_INVALID);
    CHECK(std::strlen(fa2_last_error()) > 0);
}

static void validation() {
    std::vector<float> buf(64, 0.f);
    float* p = buf.data();
    // bad shapes / head_dim / precision / null pointers: FA2_E_INVALID before any device call
    CHECK(fa2_forward(p, p, p, p, p, 0, 1, 1, 64, FA2_FP16, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward(p, p, p, p, p, 1, -1, 1, 64, FA2_FP16, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward(p, p, p, p, p, 1, 1, 1, 48, FA2_FP16, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward(p, p, p, p, p, 1, 1, 1, 64, 7, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward(p, nullptr, p, p, p, 1, 1, 1, 64, FA2_FP16, nullptr) == FA2_E_INVALID);
    CHECK(std::string(fa2_last_error()).find("null") != std::string::npos);
    // 32-bit launch-grid guards (products computed in 64 bits, no overflow)
    CHECK(fa2_forward(p, p, p, p, p, 1 << 20, 1 << 10, 1 << 12, 128, FA2_FP32, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward(p, p, p, p, p, 0x7fffffff, 0x7fffffff, 0x7fffffff, 64, FA2_FP32, nullptr) == FA2_E_INVALID);
    CHECK(fa2_delta(p, p, nullptr, 1, 1, 1, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward(p, p, p, p, p, p, p, p, p, nullptr, 1, 1, 8, 64, FA2_FP16, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward(p, p, p, p, p, p, p, p, p, p, 1, 1, 8, 64, -1, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward_dkdv(p, p, p, p, p, p, p, nullptr, 1, 1, 8, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward_dq(p, p, p, p, p, p, nullptr, 1, 1, 8, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward_dq_delta(p, p, p, p, p, p, p, nullptr, 1, 1, 8, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_naive_forward(p, p, p, p, p, nullptr, 1, 1, 8, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_fa1_forward(p, p, p, p, p, nullptr, 1, 1, 8, 64, nullptr) == FA2_E_INVALID);
    CHECK(fa2_forward_host(p, p, p, p, nullptr, 1, 1, 8, 64, FA2_FP16, 1, nullptr) == FA2_E_INVALID);
    CHECK(fa2_backward_host(p, p, p, p, p, p, p, p, nullptr, 1, 1, 8, 64, FA2_FP16, 1, nullptr) == FA2_E_INVALID);
}

// the error string is per thread: a failure on one thread never shows on another
static void thread_local_errors() {
    std::string seen[2];
    std::thread a([&] {
        int f, c;
        fa2_shard_range(1, 0, 0, &f, &c);
        seen[0] = fa2_last_error();
    });
    std::thread b([&] {
        std::vector<float> buf(8);
        fa2_forward(buf.data(), buf.data(), buf.data(), buf.data(), buf.data(), 1, 1, 1, 50, FA2_FP16, nullptr);
        seen[1] = fa2_last_error();
    });
    a.join();
    b.join();
    CHECK(seen[0].find("shard") != std::string::npos);
    CHECK(seen[1].find("head_dim") != std::string::npos);
}

static void tune_table() {
    CHECK(fa2_tune_set(nullptr, 0) == FA2_OK);
    CHECK(fa2::tune_knob("FWD_WAVES", -5) == -5);
    CHECK(fa2_tune_set("", 1) == FA2_E_INVALID);
    CHECK(fa2_tune_set("A_NAME_LONGER_THAN_THIRTY_TWO_CHARS", 1) == FA2_E_INVALID);
    CHECK(fa2_tune_set("FWD_WAVE", 4) == FA2_E_INVALID);  // misspelt: rejected, not stored
    CHECK(fa2::tune_knob("FWD_WAVE", -1) == -1);
    int v = -7;
    CHECK(fa2_tune_get("FWD_WAVES", &v) == 0 && v == -7);
    CHECK(fa2_tune_get("NOT_A_KNOB", &v) == FA2_E_INVALID);
    CHECK(fa2_tune_set("FWD_WAVES", 4) == FA2_OK);
    CHECK(fa2_tune_set("FWD_WAVES", 8) == FA2_OK);  // overwrite, not append
    CHECK(fa2::tune_knob("FWD_WAVES", 0) == 8);
    CHECK(fa2_tune_get("FWD_WAVES", &v) == 1 && v == 8);
    // concurrent writers (every knob, the table grows) and readers
    static const char* const names[] = {"FWD_KS", "DKDV_WAVES", "DKDV_QS", "DQ_WAVES", "DQ_KS", "BWD_FUSED",
                                        "BWD_FQS", "BWD_FKS"};
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([t] {
            for (int i = 0; i < 200; ++i) {
                fa2_tune_set(names[(2 * t + i) % 8], i);
                (void)fa2::tune_knob("FWD_WAVES", 0);
            }
        });
    for (auto& x : th) x.join();
    CHECK(fa2::tune_knob("FWD_WAVES", 0) == 8);
    CHECK(fa2::tune_knob("BWD_FKS", -1) >= 0);
    CHECK(fa2_tune_set(nullptr, 0) == FA2_OK);
    CHECK(fa2::tune_knob("BWD_FKS", -1) == -1);
    CHECK(fa2_tune_get("FWD_WAVES", &v) == 0);
}

// host API with more devices than visible: a code, no exit, nothing leaked
static void host_api_without_devices() {
    const int B = 1, H = 3, S = 37, D = 32;
    const size_t n = (size_t)B * H * S * D, nl = (size_t)B * H * S;
    std::vector<float> q(n, 0.5f), o(n), lse(nl), dq(n), dk(n), dv(n);
    const int visible = fa2_device_count();
    float ms = -1.f;
    CHECK(fa2_forward_host(q.data(), q.data(), q.data(), o.data(), lse.data(), B, H, S, D, FA2_FP16, visible + 1, &ms) !=
          FA2_OK);
    CHECK(fa2_backward_host(q.data(), q.data(), q.data(), q.data(), q.data(), lse.data(), dq.data(), dk.data(),
                            dv.data(), B, H, S, D, FA2_FP32, visible + 2, &ms) != FA2_OK);
    CHECK(std::strlen(fa2_last_error()) > 0);
    CHECK(ms == -1.f);  // untouched on failure
}

int main() {
    CHECK(fa2_version() >= 10000);
    CHECK(fa2_device_count() >= 0);
    shard_rule();
    validation();
    thread_local_errors();
    tune_table();
    host_api_without_devices();
    std::printf("capi_check: %s (%d failed)\n", g_failed ? "FAIL" : "ok", g_failed);
    return g_failed ? 1 : 0;
}
