// f-attn.cuh -- FlashAttention-1 forward baseline (the reference's kernels/f-attn.cuh:11-22).
// fp32 only, forward only, as there (include/dispatcher.h:31-40 rejects fp16).
// Host buffers, parameter order (B, S, H), synchronous; `logsumexp` receives the FA1
// row sum l (f-attn.cu:167, :200 of the reference), not ln l + m.
#pragma once

#include "f-attn2.cuh"

template <int head_dim>
void host_flash_attention_forward(const float* query, const float* key, const float* value, float* output,
                                  float* logsumexp, int batch_size, int seq_len, int num_heads, TimerManager* tm);

namespace fa2 {
// device pointers, async on `stream`: O [bh,S,D], l and m [bh,S] (m in natural-log units)
hipError_t launch_fa1_forward(int D, const float* q, const float* k, const float* v, float* o, float* l, float* m,
                              int bh, int S, hipStream_t stream);
}  // namespace fa2
