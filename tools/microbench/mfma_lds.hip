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
//   7  as 6 with bf16 operands and v_mfma_f32_32x32x16_bf16
//   8  as 6 with v_mfma_f32_16x16x32_f16 (same FLOPs per instruction pair)
//  11  as 9 plus, per 32 KFLOP, 1 independent v_exp + 2 VALU (a dK/dV-like mix)
//  12  as 10 with the same VALU per FLOP
//   9  A from LDS (b128 row fragment) holding random fp16, B random registers, 32x32x16
//  10  as 9 with v_mfma_f32_16x16x32_f16 (2 per slot, equal FLOPs)
//   6  MFMA only, random fp16 operands (8 per-lane register sets, U[0,1) like the
//      bench's inputs): what operand toggling costs at the power cap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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
    if (MODE >= 9) {
        unsigned z = 0x12345u + tid * 7919u;
        for (int i = tid; i < 64 * 64 * 2; i += 512) {
            z ^= z << 13; z ^= z >> 17; z ^= z << 5;
            lds[i] = (_Float16)((z & 0xffff) * (1.f / 65536.f));
        }
    } else {
        for (int i = tid; i < 64 * 64 * 2; i += 512) lds[i] = (_Float16)((i % 7) * 0.01f);
    }
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
    float xs[4] = {lane * 0.001f, lane * 0.002f, lane * 0.003f, lane * 0.004f};
    f16x8 ra[4], rb[4];
    unsigned hs = 0x9e3779b9u * (tid + 1) + blockIdx.x * 0x85ebca6bu;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            hs ^= hs << 13; hs ^= hs >> 17; hs ^= hs << 5;
            ra[s][e] = (_Float16)((hs & 0xffff) * (1.f / 65536.f));
            hs ^= hs << 13; hs ^= hs >> 17; hs ^= hs << 5;
            rb[s][e] = (_Float16)((hs & 0xffff) * (1.f / 65536.f));
        }
    for (int it = 0; it < iters; ++it) {
        if (MODE == 6) {
#pragma unroll
            for (int m = 0; m < NMF; ++m) acc[m & 3] = mfma(ra[m & 3], rb[(m >> 2) & 3], acc[m & 3]);
        } else if (MODE == 7) {
#pragma unroll
            for (int m = 0; m < NMF; ++m)
                acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ra[m & 3]),
                                                                    __builtin_bit_cast(bf16x8, rb[(m >> 2) & 3]),
                                                                    acc[m & 3], 0, 0, 0);
        } else if (MODE == 8) {
            // 16x16x32: half the FLOPs of a 32x32x16; 2 per slot keeps the FLOPs equal
#pragma unroll
            for (int m = 0; m < NMF; ++m)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    f32x4 c4 = {acc[m & 3][4 * u], acc[m & 3][4 * u + 1], acc[m & 3][4 * u + 2], acc[m & 3][4 * u + 3]};
                    c4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[(m + u) & 3], rb[(m >> 2) & 3], c4, 0, 0, 0);
                    acc[m & 3][4 * u] = c4[0]; acc[m & 3][4 * u + 1] = c4[1];
                    acc[m & 3][4 * u + 2] = c4[2]; acc[m & 3][4 * u + 3] = c4[3];
                }
        } else if (MODE == 11 || MODE == 12) {
            const int row16 = (lane & 15) * 64 + (lane >> 4) * 8;
#pragma unroll
            for (int m = 0; m < NMF; ++m) {
                if (MODE == 11) {
                    const f16x8 a = *reinterpret_cast<const f16x8*>(lds + rowoff + (m & 7) * 8 + (m >> 3) * 2048);
                    acc[m & 3] = mfma(a, rb[(m >> 2) & 3], acc[m & 3]);
                } else {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const f16x8 a = *reinterpret_cast<const f16x8*>(lds + row16 + ((2 * m + u) & 15) * 128 + (m >> 3) * 2048);
                        f32x4 c4 = {acc[m & 3][4 * u], acc[m & 3][4 * u + 1], acc[m & 3][4 * u + 2], acc[m & 3][4 * u + 3]};
                        c4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, rb[(m >> 2) & 3], c4, 0, 0, 0);
                        acc[m & 3][4 * u] = c4[0]; acc[m & 3][4 * u + 1] = c4[1];
                        acc[m & 3][4 * u + 2] = c4[2]; acc[m & 3][4 * u + 3] = c4[3];
                    }
                }
                // independent softmax-like filler: one exp and two VALU on a rotating register
                xs[m & 3] = __builtin_amdgcn_exp2f(xs[m & 3] * 0.999f) * 0.5f + 0.25f;
            }
        } else if (MODE == 9) {
#pragma unroll
            for (int m = 0; m < NMF; ++m) {
                const f16x8 a = *reinterpret_cast<const f16x8*>(lds + rowoff + (m & 7) * 8 + (m >> 3) * 2048);
                acc[m & 3] = mfma(a, rb[(m >> 2) & 3], acc[m & 3]);
            }
        } else if (MODE == 10) {
            const int row16 = (lane & 15) * 64 + (lane >> 4) * 8;
#pragma unroll
            for (int m = 0; m < NMF; ++m)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f16x8 a = *reinterpret_cast<const f16x8*>(lds + row16 + (m & 7) * 32 * 0 + ((2 * m + u) & 15) * 1024 / 8 + (m >> 3) * 2048);
                    f32x4 c4 = {acc[m & 3][4 * u], acc[m & 3][4 * u + 1], acc[m & 3][4 * u + 2], acc[m & 3][4 * u + 3]};
                    c4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, rb[(m >> 2) & 3], c4, 0, 0, 0);
                    acc[m & 3][4 * u] = c4[0]; acc[m & 3][4 * u + 1] = c4[1];
                    acc[m & 3][4 * u + 2] = c4[2]; acc[m & 3][4 * u + 3] = c4[3];
                }
        } else if (MODE == 0) {
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
    float s = x + (float)ra[0][0] + (float)rb[0][0] + xs[0] + xs[1] + xs[2] + xs[3];
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

int main(int argc, char** argv) {
    float* d;
    const int nblk = 256 * 1;  // one 8-wave workgroup per CU
    (void)hipMalloc(&d, nblk * 512 * sizeof(float));
    // argv[1] = iterations (default 2000); a large value (e.g. 400000) keeps the chip
    // busy for seconds so clock / power can be sampled at steady state
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    run<0, 1>("mfma only", d, nblk, iters);
    run<1, 1>("b128 row frag, compiler", d, nblk, iters);
    run<2, 1>("tr_b16 pair frag, compiler", d, nblk, iters);
    run<3, 2>("tr_b16 pair frag, prefetch 2", d, nblk, iters);
    run<3, 4>("tr_b16 pair frag, prefetch 4", d, nblk, iters);
    run<4, 2>("b128 row frag, prefetch 2", d, nblk, iters);
    run<4, 4>("b128 row frag, prefetch 4", d, nblk, iters);
    run<5, 1>("tr pair + 2 exp/MFMA", d, nblk, iters);
    run<6, 1>("mfma only, random operands", d, nblk, iters);
    run<7, 1>("mfma only, random bf16 operands", d, nblk, iters);
    run<8, 1>("16x16x32 f16, random operands", d, nblk, iters);
    run<9, 1>("32x32x16, A random LDS b128, B random", d, nblk, iters);
    run<10, 1>("16x16x32, A random LDS b128, B random", d, nblk, iters);
    run<11, 1>("32x32x16 LDS-random + 1 exp 2 valu /32KF", d, nblk, iters);
    run<12, 1>("16x16x32 LDS-random + 1 exp 2 valu /32KF", d, nblk, iters);
    (void)hipFree(d);
    return 0;
}
