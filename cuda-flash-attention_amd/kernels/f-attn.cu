// f-attn.cu -- FlashAttention-1 forward, fp32, for MI355X (gfx950).  A comparison
// baseline, not the hot path.
//
// Replaces detker/CUDA-Flash-Attention kernels/f-attn.cu: flash_attention_forward_kernel
// (:18-207), host_flash_attention_forward (:209-281, CLI method `fa1`) and the CuPy
// wrapper flash_attention_forward_kernel_wrapper (:283-299, harness kernel "fa1",
// test_flash_attention2.py:315-372: grid B*H, 256 threads).  Same algorithm as the
// reference and the FA1 paper (Dao et al. 2022, Alg. 1): one workgroup per (b, h),
// OUTER loop over 32-key K/V blocks (staged in LDS), INNER loop over 32-row query
// blocks, whose running (O, l, m) live in HBM and are read, updated and written back
// at every K/V block; O is kept normalised, O <- (l e^{m-m'} O + e^{m~-m'} P~V) / l'.
// Outputs as there: O, `logsumexp` = l (the row sum relative to m, not its log;
// f-attn.cu:167, :200) and `maxes` = m.  The running state starts at the first K/V
// block inside the kernel (the reference host pre-fills m = -FLT_MAX, :242-246; the
// harness zero-fills, :325-327 -- either way the same O).
//
// gfx950 shape: waves take query blocks round-robin; S^T = K Q^T and O^T += V^T P^T
// on v_mfma_f32_32x32x2_f32 (exact fp32), keys on the accumulator rows, the query on
// the lane, so row max / sum are 16-register reductions plus one cross-half swap.
//
// Self-contained device code (hiprtc-compilable with -DCUPY_INLINE_COMPILE, C++14).
#ifndef CUPY_INLINE_COMPILE
#include "f-attn.cuh"
#endif

namespace fa2fa1 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define FA1_LOG2E 1.4426950408889634f
#define FA1_LN2 0.6931471805599453f

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
__device__ __forceinline__ float other_half(float x) { return __shfl_xor(x, 32); }

template <int D> struct Fa1Lds {
    static constexpr int LD = D + 4;                 // row pad: conflict-free row / column walks
    static constexpr int FLOATS = 2 * 32 * LD;       // K block, V block
};

// One head.  lm: the `logsumexp` (l) and `maxes` (m) rows of this head.
template <int D>
__device__ void fa1_head(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                         float* __restrict__ O, float* __restrict__ Lrow, float* __restrict__ Mrow, int S,
                         float* smem) {
    constexpr int LD = Fa1Lds<D>::LD;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int nb = (S + 31) / 32;
    const float qscale = FA1_LOG2E / __builtin_sqrtf((float)D);  // scores in the log2 domain
    float* Kt = smem;
    float* Vt = smem + 32 * LD;

    for (int j = 0; j < nb; ++j) {
        // ---- stage K_j, V_j (rows past S as zeros)
        __syncthreads();
        for (int x = tid; x < 32 * (D / 4); x += blockDim.x) {
            const int row = x / (D / 4), c4 = x - row * (D / 4);
            const int key = 32 * j + row;
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
            if (key < S) {
                kv = *reinterpret_cast<const f32x4*>(K + (long)key * D + 4 * c4);
                vv = *reinterpret_cast<const f32x4*>(V + (long)key * D + 4 * c4);
            }
            *reinterpret_cast<f32x4*>(Kt + row * LD + 4 * c4) = kv;
            *reinterpret_cast<f32x4*>(Vt + row * LD + 4 * c4) = vv;
        }
        __syncthreads();

        // ---- every query block against K_j, V_j; state round-trips through HBM
        for (int i = wave; i < nb; i += nw) {
            const int q = 32 * i + r;
            const bool qok = q < S;
            // S^T = K_j Q_i^T; k-slot h of step (m, e) carries feature 8m + 4h + e
            f32x16 sacc;
#pragma unroll
            for (int x = 0; x < 16; ++x) sacc[x] = 0.f;
#pragma unroll 4
            for (int m = 0; m < D / 8; ++m) {
                f32x4 qv = {0.f, 0.f, 0.f, 0.f};
                if (qok) qv = *reinterpret_cast<const f32x4*>(Q + (long)q * D + 8 * m + 4 * h);
                const f32x4 kv = *reinterpret_cast<const f32x4*>(Kt + r * LD + 8 * m + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) sacc = mfma(kv[e], qv[e] * qscale, sacc);
            }
#pragma unroll
            for (int x = 0; x < 16; ++x)
                if (32 * j + acc_row(x, h) >= S) sacc[x] = -__builtin_inff();
            // block row max m~, P~ = exp2(s - m~), row sum l~ (both lane halves)
            float mt = sacc[0];
#pragma unroll
            for (int x = 1; x < 16; ++x) mt = fmaxf(mt, sacc[x]);
            mt = fmaxf(mt, other_half(mt));
            float lt = 0.f;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                sacc[x] = __builtin_amdgcn_exp2f(sacc[x] - mt);
                lt += sacc[x];
            }
            lt += other_half(lt);
            // P~ V_j (the MFMA's two k-slots carry keys acc_row(x, 0) and acc_row(x, 1))
            f32x16 pv[D / 32];
#pragma unroll
            for (int b = 0; b < D / 32; ++b) {
#pragma unroll
                for (int x = 0; x < 16; ++x) pv[b][x] = 0.f;
#pragma unroll
                for (int x = 0; x < 16; ++x) pv[b] = mfma(Vt[acc_row(x, h) * LD + 32 * b + r], sacc[x], pv[b]);
            }
            // previous state (none before the first block)
            float mp = -__builtin_inff(), lp = 0.f;
            if (j > 0 && qok) {
                mp = Mrow[q] * FA1_LOG2E;
                lp = Lrow[q];
            }
            const float mn = fmaxf(mp, mt);
            const float a = (j > 0) ? __builtin_amdgcn_exp2f(mp - mn) * lp : 0.f;
            const float c = __builtin_amdgcn_exp2f(mt - mn);
            const float ln = a + c * lt;
            const float inv = 1.f / ln;
            if (qok) {
                float* orow = O + (long)q * D;
#pragma unroll
                for (int b = 0; b < D / 32; ++b)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        f32x4 prev = {0.f, 0.f, 0.f, 0.f};
                        if (j > 0) prev = *reinterpret_cast<const f32x4*>(orow + 32 * b + 8 * g + 4 * h);
                        f32x4 nv;
#pragma unroll
                        for (int e = 0; e < 4; ++e) nv[e] = (a * prev[e] + c * pv[b][4 * g + e]) * inv;
                        *reinterpret_cast<f32x4*>(orow + 32 * b + 8 * g + 4 * h) = nv;
                    }
                if (h == 0) {
                    Lrow[q] = ln;
                    Mrow[q] = mn * FA1_LN2;
                }
            }
        }
    }
}

template <int D>
__global__ void __launch_bounds__(256)
fa1_fwd_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
               float* __restrict__ O, float* __restrict__ L, float* __restrict__ M, int S) {
    __shared__ __attribute__((aligned(16))) float smem[Fa1Lds<D>::FLOATS];
    const long bh = blockIdx.x;
    const long base = bh * S * D;
    fa1_head<D>(Q + base, K + base, V + base, O + base, L + bh * S, M + bh * S, S, smem);
}

}  // namespace fa2fa1

#ifndef CUPY_INLINE_COMPILE
namespace fa2 {

hipError_t launch_fa1_forward(int D, const float* q, const float* k, const float* v, float* o, float* l, float* m,
                              int bh, int S, hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    switch (D) {
#define FA2_FA1(DD)                                                                                              \
    case DD:                                                                                                     \
        hipLaunchKernelGGL((fa2fa1::fa1_fwd_kernel<DD>), dim3((unsigned)bh), dim3(256), 0, stream, q, k, v, o, l, \
                           m, S);                                                                                 \
        return hipGetLastError();
        FA2_FA1(32) FA2_FA1(64) FA2_FA1(128)
#undef FA2_FA1
        default: return hipErrorInvalidValue;
    }
}

}  // namespace fa2

// Host API with the reference's semantics (f-attn.cu:209-281): host buffers in,
// device alloc + H2D, timed launch, D2H of O and `logsumexp` (= l, as there).
template <int head_dim>
void host_flash_attention_forward(const float* query, const float* key, const float* value, float* output,
                                  float* logsumexp, int batch_size, int seq_len, int num_heads, TimerManager* tm) {
    const size_t n = (size_t)batch_size * num_heads * seq_len * head_dim;
    const size_t nl = (size_t)batch_size * num_heads * seq_len;
    float *dq, *dk, *dv, *dout, *dl, *dm;
    HIP_CHECK(hipMalloc(&dq, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dk, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dv, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dout, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dl, nl * sizeof(float)));
    HIP_CHECK(hipMalloc(&dm, nl * sizeof(float)));
    HIP_CHECK(hipMemcpy(dq, query, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dk, key, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dv, value, n * sizeof(float), hipMemcpyHostToDevice));
    if (tm) tm->Start();
    HIP_CHECK(fa2::launch_fa1_forward(head_dim, dq, dk, dv, dout, dl, dm, batch_size * num_heads, seq_len, nullptr));
    if (tm) tm->Stop();
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(output, dout, n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(logsumexp, dl, nl * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipFree(dq));
    HIP_CHECK(hipFree(dk));
    HIP_CHECK(hipFree(dv));
    HIP_CHECK(hipFree(dout));
    HIP_CHECK(hipFree(dl));
    HIP_CHECK(hipFree(dm));
}
template void host_flash_attention_forward<32>(const float*, const float*, const float*, float*, float*, int, int,
                                               int, TimerManager*);
template void host_flash_attention_forward<64>(const float*, const float*, const float*, float*, float*, int, int,
                                               int, TimerManager*);
template void host_flash_attention_forward<128>(const float*, const float*, const float*, float*, float*, int, int,
                                                int, TimerManager*);
#else
// CuPy face (same symbol as f-attn.cu:283-299): grid B*H, 256 threads, head_dim 64
// as there (the symbol carries no D); `logsumexp` receives l and `maxes` m.
extern "C" __global__ void __launch_bounds__(256)
flash_attention_forward_kernel_wrapper(const float* query, const float* key, const float* value, float* output,
                                       float* logsumexp, float* maxes, int batch_size, int num_heads, int seq_len) {
    (void)batch_size;
    (void)num_heads;
    __shared__ __attribute__((aligned(16))) float smem[fa2fa1::Fa1Lds<64>::FLOATS];
    const long bh = blockIdx.x;
    const long base = bh * seq_len * 64;
    fa2fa1::fa1_head<64>(query + base, key + base, value + base, output + base, logsumexp + bh * seq_len,
                         maxes + bh * seq_len, seq_len, smem);
}
#endif
