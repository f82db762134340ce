// vanilla-attn.cuh -- naive attention forward baseline (the reference's
// kernels/vanilla-attn.cuh:6-17): the S x S score matrix materialised in HBM.
// fp32 only, forward only, as there (include/dispatcher.h:42-50 rejects fp16).
#pragma once

#include "f-attn2.cuh"

template <int head_dim>
void host_vanilla_attention_forward(const float* h_Q, const float* h_K, const float* h_V, float* h_O,
                                    float* h_logsumexp, int batch_size, int seq_len, int num_heads,
                                    TimerManager* tm = nullptr);

namespace fa2 {
// device pointers, async on `stream`; `scores` is [bh,S,S] scratch (ends holding P),
// `lse` [bh,S] may be null
hipError_t launch_vanilla_forward(int D, const float* q, const float* k, const float* v, float* o, float* lse,
                                  float* scores, int bh, int S, hipStream_t stream);
}  // namespace fa2
