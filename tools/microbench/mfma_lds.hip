// mfma_lds.hip -- ceiling of the "LDS fragment -> v_mfma_f32_32x32x16_f16" pattern
// that all three fp16 FA2 kernels are built from, at 8 waves per workgroup
// (2 waves/SIMD), one workgroup per CU, no barriers in the loop.
//
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 mfma_lds.hip -o mfma_lds
//   ./mfma_lds            -> one line per variant: TF/s and MFMA-peak fraction
//
// Variants (MODE):
//   0  MFMA only (A, B in registers)                         -> issue ceiling
//   1  A from ds_read_b128 row fragment, compiler-scheduled
//   2  A from 2 x ds_read_b64_tr_b16, compiler-scheduled
//   3  as 2, A fragments prefetched PF MFMAs ahead (rolling register ring)
//   4  as 1, prefetched PF ahead
//   5  as 2 plus 2 v_exp + 3 VALU per MFMA (softmax-like filler)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16x8 tr8(const _Float16* p0, const _Float16* p1) {
    i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p0);
    i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p1);
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

constexpr int NMF = 16;  // MFMAs per loop iteration per wave (4 accumulators)

template <int MODE, int PF>
__global__ void __launch_bounds__(512) kern(float* out, int iters) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[64 * 64 * 2];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 64 * 64 * 2; i += 512) lds[i] = (_Float16)((i % 7) * 0.01f);
    __syncthreads();
    f16x8 b = {1, 1, 1, 1, 1, 1, 1, 1};
    f16x8 areg = {0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5};
    f32x16 acc[4];
    for (int a = 0; a < 4; ++a)
        for (int i = 0; i < 16; ++i) acc[a][i] = 0.f;
    // per-lane fragment addresses (row / transposed), varied over NMF offsets
    const int rowoff = (lane & 31) * 64 + (lane >> 5) * 8;
    const int g = lane >> 4, i4 = lane & 15;
    const int troff0 = (4 * (g >> 1) + (i4 >> 2)) * 64 + 16 * (g & 1) + 4 * (i4 & 3);
    const int troff1 = troff0 + 8 * 64;
    float x = lane * 0.001f;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
#pragma unroll
            for (int m = 0; m < NMF; ++m) acc[m & 3] = mfma(areg, b, acc[m & 3]);
        } else if (MODE == 1 || MODE == 2 || MODE == 5) {
#pragma unroll
            for (int m = 0; m < NMF; ++m) {
                const int o = (m & 7) * 16 * 64 + (m >> 3) * 32;
                f16x8 a = MODE == 1 ? *reinterpret_cast<const f16x8*>(lds + rowoff + (m & 7) * 8)
                                    : tr8(lds + troff0 + o, lds + troff1 + o);
                acc[m & 3] = mfma(a, b, acc[m & 3]);
                if (MODE == 5) {
                    x = __builtin_amdgcn_exp2f(x * 0.5f) - 0.25f;
                    x = __builtin_amdgcn_exp2f(x * 0.5f) * 0.75f;
                }
            }
        } else {  // 3, 4: explicit prefetch ring of depth PF
            f16x8 ring[PF];
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                const int o = (p & 7) * 16 * 64 + (p >> 3) * 32;
                ring[p] = MODE == 4 ? *reinterpret_cast<const f16x8*>(lds + rowoff + (p & 7) * 8)
                                    : tr8(lds + troff0 + o, lds + troff1 + o);
            }
#pragma unroll
            for (int m = 0; m < NMF; ++m) {
                const f16x8 a = ring[m % PF];
                if (m + PF < NMF) {
                    const int n = m + PF, o = (n & 7) * 16 * 64 + (n >> 3) * 32;
                    ring[m % PF] = MODE == 4 ? *reinterpret_cast<const f16x8*>(lds + rowoff + (n & 7) * 8)
                                             : tr8(lds + troff0 + o, lds + troff1 + o);
                }
                acc[m & 3] = mfma(a, b, acc[m & 3]);
            }
        }
    }
    float s = x;
    for (int a = 0; a < 4; ++a)
        for (int i = 0; i < 16; ++i) s += acc[a][i];
    out[blockIdx.x * 512 + tid] = s;
}

template <int MODE, int PF>
void run(const char* name, float* d, int nblk, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((kern<MODE, PF>), dim3(nblk), dim3(512), 0, 0, d, iters);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL((kern<MODE, PF>), dim3(nblk), dim3(512), 0, 0, d, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double flops = 2.0 * 32 * 32 * 16 * NMF * (double)iters * 8 * nblk;
    const double tf = flops / (best * 1e-3) / 1e12;
    printf("%-40s %8.3f ms  %7.1f TF/s  %.3f of 2.5 PF\n", name, best, tf, tf / 2500.0);
}

int main() {
    float* d;
    const int nblk = 256 * 1;  // one 8-wave workgroup per CU
    (void)hipMalloc(&d, nblk * 512 * sizeof(float));
    const int iters = 2000;
    run<0, 1>("mfma only", d, nblk, iters);
    run<1, 1>("b128 row frag, compiler", d, nblk, iters);
    run<2, 1>("tr_b16 pair frag, compiler", d, nblk, iters);
    run<3, 2>("tr_b16 pair frag, prefetch 2", d, nblk, iters);
    run<3, 4>("tr_b16 pair frag, prefetch 4", d, nblk, iters);
    run<4, 2>("b128 row frag, prefetch 2", d, nblk, iters);
    run<4, 4>("b128 row frag, prefetch 4", d, nblk, iters);
    run<5, 1>("tr pair + 2 exp/MFMA", d, nblk, iters);
    (void)hipFree(d);
    return 0;
}
