// dispatcher.h -- runtime head_dim -> template<HEAD_DIM>, then method x precision x mode.
//
// Same entry point and behaviour as detker/CUDA-Flash-Attention
// include/dispatcher.h:220-246 (RunFlashAttention) with its
// FlashAttentionDispatcher (:11-104) and RuntimeDimDispatcher (:107-141):
// head_dim is matched by doubling from 32 (here up to 128); forward_backward runs
// the forward then the backward, O and LSE passing through host memory exactly
// as there (:91-104).  Methods: fa2 (fp32 / fp16 / bf16 tiles, forward and
// backward), fa1 and naive (the comparison baselines, kernels/f-attn.cu and
// kernels/vanilla-attn.cu: fp32 forward only, with the reference's messages and
// exit(1) for the other combinations, :30-47, :74-83).
//
// FA2_NUM_DEVICES=N (environment) shards the B*H heads over N GPUs through the C
// ABI's host API (fa2_amd.h), one host thread per device, no collective.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <utility>

#include "enum_types.h"
#include "f-attn.cuh"
#include "f-attn2.cuh"
#include "vanilla-attn.cuh"
#include "fa2_amd.h"
#include "timer.h"

inline int fa2_env_devices() {
    const char* s = getenv("FA2_NUM_DEVICES");
    const int n = s ? atoi(s) : 1;
    return n < 1 ? 1 : n;
}

// The baselines' unsupported combinations, with the reference's messages
// (dispatcher.h:31-50, 74-83 there).  The dispatcher reaches the same exits; the
// CLI calls this right after argv parsing, before any device work.
inline void check_method_support(ComputeType method, ModeType mode, ComputeDataType prec) {
    if (method == ComputeType::FlashAttention2) return;
    const bool fa1 = method == ComputeType::FlashAttention1;
    if (mode != ModeType::Backward && prec != ComputeDataType::FP32) {
        fprintf(stderr, fa1 ? "Error: Flash Attention 1 FP16 support not implemented\n"
                            : "Error: Vanilla Attention FP16 support not implemented\n");
        exit(EXIT_FAILURE);
    }
    if (mode != ModeType::Forward) {
        fprintf(stderr, fa1 ? "Error: Flash Attention 1 backward pass not implemented\n"
                            : "Error: Vanilla Attention backward pass not implemented\n");
        exit(EXIT_FAILURE);
    }
}

template <int HEAD_DIM>
struct FlashAttentionDispatcher {
    // fa1 / naive forward (fp32 only, as the reference, dispatcher.h:31-50); true if handled
    static bool baseline_forward(const float* Q, const float* K, const float* V, float* O, float* lse, int B, int H,
                                 int S, ComputeDataType prec, ComputeType method, TimerManager* tm) {
        if (method == ComputeType::FlashAttention1) {
            if (prec != ComputeDataType::FP32) {
                fprintf(stderr, "Error: Flash Attention 1 FP16 support not implemented\n");
                exit(EXIT_FAILURE);
            }
            printf("Running Flash Attention 1 Forward (HEAD_DIM=%d)...\n", HEAD_DIM);
            host_flash_attention_forward<HEAD_DIM>(Q, K, V, O, lse, B, S, H, tm);
            return true;
        }
        if (method == ComputeType::Naive) {
            if (prec != ComputeDataType::FP32) {
                fprintf(stderr, "Error: Vanilla Attention FP16 support not implemented\n");
                exit(EXIT_FAILURE);
            }
            printf("Running Vanilla Attention Forward (HEAD_DIM=%d)...\n", HEAD_DIM);
            host_vanilla_attention_forward<HEAD_DIM>(Q, K, V, O, lse, B, S, H, tm);
            return true;
        }
        return false;
    }
    static void require_fa2_backward(ComputeType m) {
        if (m == ComputeType::FlashAttention1) {
            fprintf(stderr, "Error: Flash Attention 1 backward pass not implemented\n");
            exit(EXIT_FAILURE);
        }
        if (m == ComputeType::Naive) {
            fprintf(stderr, "Error: Vanilla Attention backward pass not implemented\n");
            exit(EXIT_FAILURE);
        }
    }
    static void sharded(int rc, float ms, TimerManager* tm) {
        if (rc) {
            fprintf(stderr, "Error: %s\n", fa2_last_error());
            exit(EXIT_FAILURE);
        }
        tm->AddMillis(ms);  // kernel time = max over devices
    }

    static int c_precision(ComputeDataType prec) {
        return prec == ComputeDataType::FP16 ? FA2_FP16 : prec == ComputeDataType::BF16 ? FA2_BF16 : FA2_FP32;
    }

    static void dispatch_forward(const float* Q, const float* K, const float* V, float* O, float* lse, int B, int H,
                                 int S, ComputeDataType prec, ComputeType method, TimerManager* tm) {
        if (baseline_forward(Q, K, V, O, lse, B, H, S, prec, method, tm)) return;
        const int ndev = fa2_env_devices();
        if (ndev > 1) {
            float ms = 0.f;
            const int rc = fa2_forward_host(Q, K, V, O, lse, B, H, S, HEAD_DIM,
                                            c_precision(prec), ndev, &ms);
            sharded(rc, ms, tm);
            return;
        }
        if (prec == ComputeDataType::FP16) {
            printf("Running Flash Attention 2 Forward (HEAD_DIM=%d) with FP16 tiles (MFMA)...\n", HEAD_DIM);
            host_flash_attention2_forward_fp16<HEAD_DIM>(Q, K, V, O, lse, B, S, H, tm);
        } else if (prec == ComputeDataType::BF16) {
            printf("Running Flash Attention 2 Forward (HEAD_DIM=%d) with BF16 tiles (MFMA)...\n", HEAD_DIM);
            host_flash_attention2_forward_bf16<HEAD_DIM>(Q, K, V, O, lse, B, S, H, tm);
        } else {
            printf("Running Flash Attention 2 Forward (HEAD_DIM=%d)...\n", HEAD_DIM);
            host_flash_attention2_forward<HEAD_DIM>(Q, K, V, O, lse, B, S, H, tm);
        }
    }

    static void dispatch_backward(const float* Q, const float* K, const float* V, const float* O, const float* dO,
                                  const float* lse, float* dQ, float* dK, float* dV, int B, int H, int S,
                                  ComputeDataType prec, ComputeType method, TimerManager* tm) {
        require_fa2_backward(method);
        const int ndev = fa2_env_devices();
        if (ndev > 1) {
            float ms = 0.f;
            const int rc = fa2_backward_host(Q, K, V, O, dO, lse, dQ, dK, dV, B, H, S, HEAD_DIM,
                                             c_precision(prec), ndev, &ms);
            sharded(rc, ms, tm);
            return;
        }
        if (prec == ComputeDataType::FP16) {
            printf("Running Flash Attention 2 Backward (HEAD_DIM=%d) with FP16 tiles (MFMA)...\n", HEAD_DIM);
            host_flash_attention2_backward_fp16<HEAD_DIM>(Q, K, V, O, dO, lse, dQ, dK, dV, B, S, H, tm);
        } else if (prec == ComputeDataType::BF16) {
            printf("Running Flash Attention 2 Backward (HEAD_DIM=%d) with BF16 tiles (MFMA)...\n", HEAD_DIM);
            host_flash_attention2_backward_bf16<HEAD_DIM>(Q, K, V, O, dO, lse, dQ, dK, dV, B, S, H, tm);
        } else {
            printf("Running Flash Attention 2 Backward (HEAD_DIM=%d)...\n", HEAD_DIM);
            host_flash_attention2_backward<HEAD_DIM>(Q, K, V, O, dO, lse, dQ, dK, dV, B, S, H, tm);
        }
    }

    static void dispatch_forward_backward(const float* Q, const float* K, const float* V, float* O, float* lse,
                                          const float* dO, float* dQ, float* dK, float* dV, int B, int H, int S,
                                          ComputeDataType prec, ComputeType method, TimerManager* tm) {
        printf("Running Forward+Backward Pass (HEAD_DIM=%d)...\n", HEAD_DIM);
        dispatch_forward(Q, K, V, O, lse, B, H, S, prec, method, tm);
        dispatch_backward(Q, K, V, O, dO, lse, dQ, dK, dV, B, H, S, prec, method, tm);
    }
};

template <int CurrentD, int MaxD>
struct RuntimeDimDispatcher {
    template <typename F>
    static void dispatch(int head_dim, F&& f) {
        if (head_dim == CurrentD) f.template operator()<CurrentD>();
        else RuntimeDimDispatcher<CurrentD * 2, MaxD>::dispatch(head_dim, std::forward<F>(f));
    }
};
template <int MaxD>
struct RuntimeDimDispatcher<MaxD, MaxD> {
    template <typename F>
    static void dispatch(int head_dim, F&& f) {
        if (head_dim == MaxD) {
            f.template operator()<MaxD>();
        } else {
            fprintf(stderr, "Error: Unsupported head dimension %d\n", head_dim);
            exit(EXIT_FAILURE);
        }
    }
};

struct FlashAttentionLaunch {
    const float *Q, *K, *V;
    float *O, *lse;
    const float* dO;
    float *dQ, *dK, *dV;
    int B, H, S;
    ComputeDataType prec;
    ComputeType method;
    ModeType mode;
    TimerManager* tm;
    template <int D>
    void operator()() const {
        using FD = FlashAttentionDispatcher<D>;
        if (mode == ModeType::Forward) FD::dispatch_forward(Q, K, V, O, lse, B, H, S, prec, method, tm);
        else if (mode == ModeType::Backward)
            FD::dispatch_backward(Q, K, V, O, dO, lse, dQ, dK, dV, B, H, S, prec, method, tm);
        else FD::dispatch_forward_backward(Q, K, V, O, lse, dO, dQ, dK, dV, B, H, S, prec, method, tm);
    }
};

inline void RunFlashAttention(const float* Q, const float* K, const float* V, float* O, float* logsumexp,
                              const float* dO, float* dQ, float* dK, float* dV, int batch_size, int num_heads,
                              int seq_len, int head_dim, ComputeDataType compute_data_type, ComputeType compute_method,
                              ModeType mode, TimerManager* tm) {
    static constexpr int MIN_HEAD_DIM = 32;
    static constexpr int MAX_HEAD_DIM = 128;
    FlashAttentionLaunch l{Q, K, V, O, logsumexp, dO, dQ, dK, dV, batch_size, num_heads, seq_len,
                           compute_data_type, compute_method, mode, tm};
    RuntimeDimDispatcher<MIN_HEAD_DIM, MAX_HEAD_DIM>::dispatch(head_dim, l);
}
