/*
 * fa2_amd.h -- C ABI of the MI355X-native FA2 forward+backward (libfa2amd.so).
 *
 * The drop-in boundary for detker/CUDA-Flash-Attention's hot path.  Plain
 * pointers and sizes, no C++ or torch types, so any FFI (ctypes, cgo, JNI,
 * N-API) can bind it; see INTEGRATION.md for the bindings.  Every entry point
 * returns 0 on success or a negative FA2_E* code; fa2_last_error() returns the
 * calling thread's last message.  Nothing here calls exit().
 *
 * Tensor layout everywhere (as in the reference): fp32, [B,H,S,D] row-major for
 * Q, K, V, O, dO, dQ, dK, dV; [B,H,S] for logsumexp (natural log) and delta.
 * head_dim D must be 32, 64 or 128 (the reference instantiates 32 and 64,
 * kernels/kernel_fa2_optimized.cu:424-426; 128 is BASELINE config C4's).
 *
 * `precision` mirrors the reference's ComputeDataType (include/enum_types.h:15-18):
 *   FA2_FP32 -- fp32 tiles, exact-fp32 MFMA (the reference's default .cu files);
 *   FA2_FP16 -- fp16 tiles, MFMA f16 -> fp32 accumulate (the _f16.cu files);
 *   FA2_BF16 -- bf16 tiles, MFMA bf16 -> fp32 accumulate (an extension: the
 *               reference lists BF16 under "Possible Improvements", README.md:504-508).
 */
#ifndef FA2_AMD_H
#define FA2_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { FA2_FP16 = 0, FA2_FP32 = 1, FA2_BF16 = 2 };

enum {
    FA2_OK = 0,
    FA2_E_INVALID = -1,   /* bad shape, head_dim, precision or null pointer */
    FA2_E_DEVICE = -2,    /* HIP runtime / launch failure (see fa2_last_error) */
    FA2_E_NOMEM = -3      /* device allocation failed */
};

/* ---------------------------------------------------------------------------
 * Device-pointer API.  Inputs already resident in HBM; launches are async on
 * `stream` (a hipStream_t, NULL = default stream); nothing allocates or
 * synchronises, so calls are hipGraph-capturable.
 * ------------------------------------------------------------------------- */

/* Forward: O, LSE.  Replaces the device half of host_flash_attention2_forward[_fp16]
 * (kernels/f-attn2.cuh:13-24 / :43-54) and the CuPy launch of
 * flash_attention2_forward_kernel_wrapper (kernel_fa2_optimized.cu:428-444). */
int fa2_forward(const float* q, const float* k, const float* v, float* o, float* lse, int batch, int heads, int seq,
                int head_dim, int precision, void* stream);

/* Δ = rowsum(dO ∘ O).  Replaces D_computation_reduction_kernel(_wrapper)
 * (f-attn2-backward.cu:341-380, :515-528); the output pointer comes last there,
 * first-class here. */
int fa2_delta(const float* dout, const float* o, float* delta, int batch, int heads, int seq, int head_dim,
              void* stream);

/* Backward: dQ, dK, dV (fully overwritten; no pre-zeroing needed).  `delta` is
 * [B,H,S] scratch that receives Δ.  Determinism: results are bitwise reproducible in
 * every precision (no float atomics in any launch plan; the reference adds dQ with
 * fp32 atomics, f-attn2-backward.cu:298, here a dQ workgroup role sums it instead).
 * Replaces the device half of host_flash_attention2_backward[_fp16] (kernels/f-attn2.cuh:26-41 / :56-71) and
 * the CuPy launches of D_computation_reduction_kernel_wrapper +
 * flash_attention2_backward_kernel_wrapper (f-attn2-backward.cu:491-528). */
int fa2_backward(const float* q, const float* k, const float* v, const float* o, const float* dout,
                 const float* lse, float* delta, float* dq, float* dk, float* dv, int batch, int heads, int seq,
                 int head_dim, int precision, void* stream);

/* The two MFMA kernels of the fp16 backward, separately (profiling/bench hooks;
 * fa2_delta + these two compute what fa2_backward with FA2_FP16 does). */
int fa2_backward_dkdv(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                      const float* delta, float* dk, float* dv, int batch, int heads, int seq, int head_dim,
                      void* stream);
int fa2_backward_dq(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                    const float* delta, float* dq, int batch, int heads, int seq, int head_dim, void* stream);
/* dQ with Δ computed in the same kernel (from O and dO) and written to `delta`
 * (B*H*S floats); fa2_backward_dkdv launched after it reads that Δ.  This pair is
 * what fa2_backward runs for FA2_FP16 / FA2_BF16 on grids of at least 8 blocks of 32
 * rows per CU and at D = 128; on smaller grids (D <= 64) it runs ONE launch whose
 * workgroups take the dK/dV or the dQ role side by side (BWD_FUSED; Δ computed inside
 * it below 4 blocks per CU, else fa2_delta first). */
int fa2_backward_dq_delta(const float* q, const float* k, const float* v, const float* o, const float* dout,
                          const float* lse, float* delta, float* dq, int batch, int heads, int seq, int head_dim,
                          void* stream);

/* Comparison baselines, exact fp32, forward only, one workgroup per
 * (b, h) as in the reference.
 *   fa2_naive_forward: the reference's vanilla attention (kernels/vanilla-attn.cu:7-70,
 *     CLI method `naive`): scores [B,H,S,S] materialised in `scores` (left holding P),
 *     O, and LSE (may be NULL; the reference writes none).
 *   fa2_fa1_forward: FlashAttention-1 (kernels/f-attn.cu:18-207, CLI method `fa1`):
 *     O, l (row sum relative to m, the reference's `logsumexp` output) and m. */
int fa2_naive_forward(const float* q, const float* k, const float* v, float* o, float* lse, float* scores, int batch,
                      int heads, int seq, int head_dim, void* stream);
int fa2_fa1_forward(const float* q, const float* k, const float* v, float* o, float* l, float* m, int batch,
                    int heads, int seq, int head_dim, void* stream);

/* ---------------------------------------------------------------------------
 * Host-pointer API: the reference host functions' semantics
 * (kernel_fa2_optimized.cu:350-423, f-attn2-backward.cu:384-485): host buffers
 * in and out, H2D + timed kernels + D2H, synchronous (returns with the outputs
 * in the caller's buffers).  *kernel_ms (may be NULL) receives the hipEvent-timed
 * kernel milliseconds (what TimerManager accumulates; copies excluded).
 *
 * num_devices > 1 shards the B*H heads contiguously over devices 0..n-1, one
 * host thread per device, each copying only its slice (no
 * collective).  *kernel_ms is then the max over devices.
 *
 * Unlike the reference (hipMalloc / hipFree of every tensor per call), the device
 * scratch is kept between calls (one grow-only block per device); each shard runs
 * as a pipeline over head chunks, the H2D of the next chunk and the D2H of the
 * previous one overlapping the current chunk's kernels.  fa2_host_release frees
 * the scratch (the next call allocates it again), and also the per-stream scratch
 * the device-pointer calls keep for their split launch plans (small grids), including
 * the blocks graphs captured from those calls hold; call it with no work of this library
 * in flight and no such graph left to replay.
 * ------------------------------------------------------------------------- */
int fa2_forward_host(const float* q, const float* k, const float* v, float* o, float* lse, int batch, int heads,
                     int seq, int head_dim, int precision, int num_devices, float* kernel_ms);
int fa2_backward_host(const float* q, const float* k, const float* v, const float* o, const float* dout,
                      const float* lse, float* dq, float* dk, float* dv, int batch, int heads, int seq, int head_dim,
                      int precision, int num_devices, float* kernel_ms);

int fa2_host_release(void);

/* Shard helper shared by the C++ and Python drivers: heads [*first, *first+*count)
 * of `total_heads` belong to shard `index` of `shards` (contiguous, balanced). */
int fa2_shard_range(int total_heads, int shards, int index, int* first, int* count);

/* Launch-plan override (tests and tuning tools only; nothing is read from the
 * environment).  fa2_tune_set("DKDV_QS", 2) makes the next launches use that plan
 * where the shape allows it; fa2_tune_set(NULL, 0) clears every override.  Knobs:
 * FWD_HS, FWD_SPLIT, FWD_WAVES, FWD_KS, FWD_NKB, BWD_SPLIT, DKDV_HS, DKDV_WAVES, DKDV_QS, DQ_HS, DQ_WAVES,
 * DQ_KS, BWD_FUSED, BWD_FUSED_DELTA, BWD_FQS, BWD_FKS, BWD_FNW (see the launchers in
 * kernels/; a value that forces a plan the shape cannot take is FA2_E_INVALID at the
 * launch, never a silent fallback), and
 * the test-only HOST_SHARDS_ON_DEVICE0 = 1 (fa2_*_host run every shard on device 0,
 * so an N-way split's head offsets are testable on one GPU) and HOST_CHUNKS (head
 * chunks of the fa2_*_host pipeline; 0 = auto).  Any other name:
 * FA2_E_INVALID.  Process-wide.
 * fa2_tune_get: 1 and *value when `knob` is overridden, 0 when it is not,
 * FA2_E_INVALID for an unknown name. */
int fa2_tune_set(const char* knob, int value);
int fa2_tune_get(const char* knob, int* value);

const char* fa2_last_error(void);
int fa2_version(void); /* MAJOR*10000 + MINOR*100 + PATCH */
/* Hash of the sources and flags this library was built from (16 hex digits):
 * profiles that depend on the kernels' code (rocprofv3 PMC traffic) record it. */
const char* fa2_build_id(void);
int fa2_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* FA2_AMD_H */
