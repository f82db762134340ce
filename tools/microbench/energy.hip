// energy.hip -- dynamic energy per wave instruction of the instruction kinds the FA2
// loops are made of, on gfx950 at the power cap question: the C3 kernels all run at
// 1310-1380 W socket power, so their time follows their energy per step.  Each mode
// runs one instruction kind back to back (independent chains, 8 waves per CU, every
// CU busy) for about `secs` seconds; tools/energy_probe.sh samples socket power
// meanwhile.  Energy per instruction = (P_mode - P_sleep) x t / instructions.
//   hipcc --offload-arch=gfx950 -O3 energy.hip -o energy && ./energy <mode> <secs>
// modes: 0 s_sleep (baseline)  1 v_exp_f32  2 v_fma_f32  3 v_pk_mul_f32
//        4 v_cvt_pk_f16_f32  5 ds_read_b128  6 mfma 16x16x32 f16 (random operands)
//        7 mfma 32x32x16 f16 (random operands)  8 v_dot2c_f32_f16  9 ds_read_b64_tr_b16
//        10 global_load_dwordx4 hitting L2 (each workgroup re-reads its own 64 KB)
//        11 global_load_dwordx4 streaming from HBM (a 2 GiB buffer)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr int UNROLL = 8;

__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352d;
    x ^= x >> 15;
    x *= 0x846ca68b;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float rnd(unsigned s) { return (hash(s) & 0xffffff) * (1.f / 16777216.f); }

template <int MODE>
__global__ void __launch_bounds__(512) kern(float* out, int iters, const f32x4* __restrict__ src, long nsrc) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[512 * 8 * 2];
    const int tid = threadIdx.x;
    const unsigned seed = blockIdx.x * 512 + tid;
    float x[UNROLL];
    f32x2 px[UNROLL];
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) {
        x[i] = -rnd(seed * 8 + i) * 4.f;
        px[i] = f32x2{rnd(seed * 16 + i), rnd(seed * 16 + i + 8)};
    }
    for (int i = tid; i < 512 * 8 * 2; i += 512) lds[i] = (_Float16)rnd(i * 7 + 1);
    __syncthreads();
    f16x8 a[2], b[2];  // two random operand sets, alternated (operands change every MFMA, as in the kernels)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[0][j] = (_Float16)rnd(seed * 32 + j);
        b[0][j] = (_Float16)rnd(seed * 32 + 8 + j);
        a[1][j] = (_Float16)rnd(seed * 32 + 16 + j);
        b[1][j] = (_Float16)rnd(seed * 32 + 24 + j);
    }
    f32x4 c4[UNROLL];
    f32x16 c16[2];
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) c4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) c16[i][j] = 0.f;
    f16x8 acc8 = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned pk[UNROLL];
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) pk[i] = 0;
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {
            __builtin_amdgcn_s_sleep(2);
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]) - 4.f;
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) x[i] = __builtin_fmaf(x[i], 0.999f, 0.0001f);
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) px[i] = px[i] * f32x2{0.999f, 1.001f};
        } else if constexpr (MODE == 4) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) {
                const f16x2 h = {(_Float16)x[i], (_Float16)x[(i + 1) % UNROLL]};  // v_cvt_pk_f16_f32
                pk[i] ^= __builtin_bit_cast(unsigned, h);
                x[i] += 1e-7f;
            }
        } else if constexpr (MODE == 5) {
            // 8 ds_read_b128 from fixed conflict-free addresses (asm: not hoisted), one wait
            f32x4 v[UNROLL];
            const unsigned base = (unsigned)(unsigned long)((__attribute__((address_space(3))) _Float16*)lds) + tid * 16;
#pragma unroll
            for (int i = 0; i < UNROLL; ++i)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[i]) : "v"(base), "i"(i * 64) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) pk[i] ^= __builtin_bit_cast(unsigned, v[i][0]);
        } else if constexpr (MODE == 6) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 1], b[i & 1], c4[i], 0, 0, 0);
        } else if constexpr (MODE == 7) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i)
                c16[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(i >> 1) & 1], b[(i >> 1) & 1], c16[i & 1], 0, 0, 0);
        } else if constexpr (MODE == 8) {
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) {
                f16x2 h = {(_Float16)x[i], (_Float16)x[(i + 3) % UNROLL]};
                x[i] = __builtin_amdgcn_fdot2(h, h, x[i], false);
            }
        } else if constexpr (MODE == 9) {
            // 8 ds_read_b64_tr_b16 (asm: not hoisted), one wait
            f32x2 v[UNROLL];
            const unsigned base = (unsigned)(unsigned long)((__attribute__((address_space(3))) _Float16*)lds) + (tid & 63) * 8;
#pragma unroll
            for (int i = 0; i < UNROLL; ++i)
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v[i]) : "v"(base), "i"(i * 512) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) pk[i] ^= __builtin_bit_cast(unsigned, v[i][0]);
        }
        if constexpr (MODE == 10 || MODE == 11) {
            // 8 x 16 B per lane (asm: whole dwordx4 loads, not narrowed), one wait.  MODE 10:
            // this workgroup's own 64 KB window (L2-resident after the first pass); MODE 11:
            // every load a new 16 B of a buffer far larger than L2 + Infinity Cache
            f32x4 v[UNROLL];
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) {
                const long e = MODE == 10 ? (long)blockIdx.x * 4096 + ((tid + 512 * i + it * 64) & 4095)
                                          : ((long)it * 256 * 512 * UNROLL + (long)(i * 256 + blockIdx.x) * 512 + tid) % nsrc;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v[i]) : "v"(src + e) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UNROLL; ++i) pk[i] ^= __builtin_bit_cast(unsigned, v[i][0]);
        }
        if constexpr (MODE == 1 || MODE == 2 || MODE == 4 || MODE == 8)
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                         "+v"(x[7]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < UNROLL; ++i) s += x[i] + px[i][0] + px[i][1] + c4[i][0] + (float)pk[i];
    s += c16[0][0] + c16[1][3] + (float)acc8[0] + (float)acc8[5];
    out[blockIdx.x * 512 + tid] = s;
}

template <int MODE>
double run(float* d, int iters, double secs, int* launches, const f32x4* src, long nsrc) {
    hipLaunchKernelGGL((kern<MODE>), dim3(256), dim3(512), 0, 0, d, 16, src, nsrc);
    const hipError_t e0 = hipGetLastError(), e1 = hipDeviceSynchronize();
    if (e0 != hipSuccess || e1 != hipSuccess) {
        fprintf(stderr, "mode %d: launch %s, sync %s\n", MODE, hipGetErrorString(e0), hipGetErrorString(e1));
        exit(3);
    }
    auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    double el = 0;
    do {
        hipLaunchKernelGGL((kern<MODE>), dim3(256), dim3(512), 0, 0, d, iters, src, nsrc);
        (void)hipDeviceSynchronize();
        ++n;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < secs);
    *launches = n;
    return el;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    const double secs = argc > 2 ? atof(argv[2]) : 4.0;
    const int iters = argc > 3 ? atoi(argv[3]) : 200000;
    float* d;
    if (hipMalloc(&d, 256 * 512 * sizeof(float)) != hipSuccess) return 1;
    const long nsrc = mode == 11 ? (2l << 30) / 16 : 256l * 4096;  // f32x4 elements
    f32x4* src;
    if (hipMalloc(&src, nsrc * 16) != hipSuccess) return 1;
    (void)hipMemset(src, 0x3c, nsrc * 16);
    int n = 0;
    double el = 0;
    switch (mode) {
        case 0: el = run<0>(d, iters, secs, &n, src, nsrc); break;
        case 1: el = run<1>(d, iters, secs, &n, src, nsrc); break;
        case 2: el = run<2>(d, iters, secs, &n, src, nsrc); break;
        case 3: el = run<3>(d, iters, secs, &n, src, nsrc); break;
        case 4: el = run<4>(d, iters, secs, &n, src, nsrc); break;
        case 5: el = run<5>(d, iters, secs, &n, src, nsrc); break;
        case 6: el = run<6>(d, iters, secs, &n, src, nsrc); break;
        case 7: el = run<7>(d, iters, secs, &n, src, nsrc); break;
        case 8: el = run<8>(d, iters, secs, &n, src, nsrc); break;
        case 9: el = run<9>(d, iters, secs, &n, src, nsrc); break;
        case 10: el = run<10>(d, iters, secs, &n, src, nsrc); break;
        case 11: el = run<11>(d, iters, secs, &n, src, nsrc); break;
        default: return 2;
    }
    // wave instructions of the measured kind: 256 WGs x 8 waves x iters x UNROLL per launch
    const double winstr = 256.0 * 8 * iters * (mode == 0 ? 1 : UNROLL) * n;
    printf("{\"mode\": %d, \"seconds\": %.3f, \"launches\": %d, \"wave_instr\": %.4e, \"ns_per_winstr_per_cu\": %.4f}\n",
           mode, el, n, winstr, el * 1e9 / (winstr / 256.0));
    (void)hipFree(d);
    (void)hipFree(src);
    return 0;
}
