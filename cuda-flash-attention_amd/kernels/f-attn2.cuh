// f-attn2.cuh -- host API of the MI355X-native FA2 forward+backward.
//
// Same four templates, same parameter order (B, S, H!) and same semantics as the
// reference's kernels/f-attn2.cuh:13-71 (detker/CUDA-Flash-Attention):
//   * pointers are HOST buffers owned by the caller, fp32, [B,H,S,D] row-major;
//     logsumexp is [B,H,S] (natural log);
//   * each call allocates device memory, copies in, runs the timed kernels
//     (bracketed by tm->Start()/tm->Stop() like kernel_fa2_optimized.cu:404-410),
//     copies out and frees -- fully synchronous on return;
//   * errors print and exit(1), as CUDA_CHECK does (include/error_utils.h:8-13).
// Explicitly instantiated for head_dim in {32, 64, 128} (the reference stops at 64,
// kernel_fa2_optimized.cu:424-426; BASELINE C4 needs 128).
//
// "_fp16" selects the MFMA path: fp32 in HBM, fp16 tiles in LDS/VGPRs,
// v_mfma_f32_32x32x16_f16 with fp32 accumulation.  The plain names select the
// exact-fp32 path (fp32 tiles, v_mfma_f32_32x32x2_f32).
//
// Below the reference templates sits the device-pointer launch layer (namespace
// fa2) that the C ABI (include/fa2_amd.h) and the templates share.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "error_utils.h"
#include "timer.h"

template <int head_dim>
void host_flash_attention2_forward(const float* query, const float* key, const float* value, float* output,
                                   float* logsumexp, int batch_size, int seq_len, int num_heads, TimerManager* tm);

template <int head_dim>
void host_flash_attention2_backward(const float* query, const float* key, const float* value, const float* output,
                                    const float* deriv_output, const float* logsumexp, float* deriv_query,
                                    float* deriv_key, float* deriv_value, int batch_size, int seq_len, int num_heads,
                                    TimerManager* tm);

template <int head_dim>
void host_flash_attention2_forward_fp16(const float* h_Q, const float* h_K, const float* h_V, float* h_O,
                                        float* h_logsumexp, int batch_size, int seq_len, int num_heads,
                                        TimerManager* tm);

template <int head_dim>
void host_flash_attention2_backward_fp16(const float* query, const float* key, const float* value,
                                         const float* output, const float* deriv_output, const float* logsumexp,
                                         float* deriv_query, float* deriv_key, float* deriv_value, int batch_size,
                                         int seq_len, int num_heads, TimerManager* tm);

// bf16 tiles (the same kernels compiled with -DFA2_TILE_BF16; README "Possible
// Improvements: BF16 precision support"), same semantics as the _fp16 templates
template <int head_dim>
void host_flash_attention2_forward_bf16(const float* h_Q, const float* h_K, const float* h_V, float* h_O,
                                        float* h_logsumexp, int batch_size, int seq_len, int num_heads,
                                        TimerManager* tm);
template <int head_dim>
void host_flash_attention2_backward_bf16(const float* query, const float* key, const float* value,
                                         const float* output, const float* deriv_output, const float* logsumexp,
                                         float* deriv_query, float* deriv_key, float* deriv_value, int batch_size,
                                         int seq_len, int num_heads, TimerManager* tm);

namespace fa2 {

// Device-pointer launch layer.  All pointers are device memory, all launches are
// asynchronous on `stream`, nothing here allocates or synchronises (so a caller
// may capture them into a hipGraph).  `bh` = batch*heads, tensors [bh,S,D].
hipError_t launch_forward_f16(int D, const float* q, const float* k, const float* v, float* o, float* lse, int bh,
                              int S, hipStream_t stream);
hipError_t launch_forward_f32(int D, const float* q, const float* k, const float* v, float* o, float* lse, int bh,
                              int S, hipStream_t stream);
// delta[bh,S] = rowsum(dO * O)  (the reference's D_computation_reduction_kernel)
hipError_t launch_delta(int D, const float* dout, const float* o, float* delta, int bh, int S, hipStream_t stream);
// Backward.  `delta` is caller-provided scratch of bh*S floats (filled here).
// dq/dk/dv are fully overwritten (no pre-zeroing needed, unlike the reference).
hipError_t launch_backward_f16(int D, const float* q, const float* k, const float* v, const float* o,
                               const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                               int bh, int S, hipStream_t stream);
// exact-fp32 backward: the Δ kernel, then one launch whose workgroups take the dK/dV
// role (32 keys each) or the dQ role (32 queries each, S and dP recomputed); no float
// atomics (the reference's dQ atomicAdd, f-attn2-backward.cu:298), bitwise reproducible.
hipError_t launch_backward_f32(int D, const float* q, const float* k, const float* v, const float* o,
                               const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                               int bh, int S, hipStream_t stream);

// individual backward kernels of the fp16 path (bench/profiling hooks)
hipError_t launch_bwd_dkdv_f16(int D, const float* q, const float* k, const float* v, const float* dout,
                               const float* lse, const float* delta, float* dk, float* dv, int bh, int S,
                               hipStream_t stream);
hipError_t launch_bwd_dq_f16(int D, const float* q, const float* k, const float* v, const float* dout,
                             const float* lse, const float* delta, float* dq, int bh, int S, hipStream_t stream);
// dQ with Δ = rowsum(dO * O) computed in its prologue and written to `delta` (the
// dK/dV kernel, launched after it, reads that); replaces launch_delta + dQ
hipError_t launch_bwd_dq_delta_f16(int D, const float* q, const float* k, const float* v, const float* o,
                                   const float* dout, const float* lse, float* delta, float* dq, int bh, int S,
                                   hipStream_t stream);

// Δ given: dK/dV and dQ as ONE launch (two workgroup roles side by side; D <= 64,
// else hipErrorNotSupported)
hipError_t launch_bwd_fused_f16(int D, const float* q, const float* k, const float* v, const float* dout,
                                const float* lse, const float* delta, float* dq, float* dk, float* dv, int bh, int S,
                                hipStream_t stream);

// bf16-tile twins of the *_f16 launchers above (kernels built from the same source)
hipError_t launch_forward_bf16(int D, const float* q, const float* k, const float* v, float* o, float* lse, int bh,
                               int S, hipStream_t stream);
hipError_t launch_backward_bf16(int D, const float* q, const float* k, const float* v, const float* o,
                                const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                                int bh, int S, hipStream_t stream);
hipError_t launch_bwd_dkdv_bf16(int D, const float* q, const float* k, const float* v, const float* dout,
                                const float* lse, const float* delta, float* dk, float* dv, int bh, int S,
                                hipStream_t stream);
hipError_t launch_bwd_dq_bf16(int D, const float* q, const float* k, const float* v, const float* dout,
                              const float* lse, const float* delta, float* dq, int bh, int S, hipStream_t stream);
hipError_t launch_bwd_fused_bf16(int D, const float* q, const float* k, const float* v, const float* dout,
                                 const float* lse, const float* delta, float* dq, float* dk, float* dv, int bh, int S,
                                 hipStream_t stream);
hipError_t launch_bwd_dq_delta_bf16(int D, const float* q, const float* k, const float* v, const float* o,
                                    const float* dout, const float* lse, float* delta, float* dq, int bh, int S,
                                    hipStream_t stream);

inline bool supported_head_dim(int D) { return D == 32 || D == 64 || D == 128; }

// Launch-plan override `name` as set by fa2_tune_set (include/fa2_amd.h), else `dflt`
// (the measured best, what ships).  Never read from the environment: with no override
// set this is one relaxed atomic load.  Tests use it to reach every instance; tools
// use it to A/B plans in one process (tools/kbench.py).
int tune_knob(const char* name, int dflt);

// Waves per workgroup for a grid of `blocks32` 32-row wave units: the largest of
// maxnw, maxnw/2, ..., minnw whose grid still covers every CU of the current device
// (small problems get smaller workgroups, more of them, and waves with their SIMD
// to themselves); maxnw when even that grid fills the chip.
int auto_waves(long blocks32, int maxnw, int minnw = 2);

// Compute units of the current device (cached per device).
int cu_count();

// Device scratch of the split launch plans: one grow-only buffer per (device, stream),
// kept between calls (fa2_host_release frees it).  While `stream` is being captured into
// a graph (a capture must not allocate) the stream's block from an earlier eager call
// moves to the graph, or nullptr when there is none big enough; nullptr too when the
// allocation fails.  The auto plans then fall back to their unsplit form.
void* stream_scratch(hipStream_t stream, size_t bytes);
void stream_scratch_release();

}  // namespace fa2
