// exp_rate.hip -- issue rate of v_exp_f32 vs v_exp_f16 vs v_add_f32 (independent
// chains, 8 waves per CU, every CU busy): is a half-precision exp cheaper to issue?
//   hipcc --offload-arch=gfx950 -O3 exp_rate.hip -o exp_rate && ./exp_rate
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(512) kern(float* out, int iters) {
    float x[8];
    _Float16 hx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = threadIdx.x * 1e-4f + i * 0.01f;
        hx[i] = (_Float16)x[i];
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) x[i] = __builtin_amdgcn_exp2f(x[i]);
            else if (MODE == 1) hx[i] = __builtin_amdgcn_exp2f((float)hx[i]) > 0 ? (_Float16)__builtin_elementwise_exp2((float)hx[i]) : hx[i];
            else if (MODE == 2) hx[i] = __builtin_elementwise_exp2(hx[i]);
            else x[i] = x[i] + 1.0001f;
        }
        if (MODE == 0 || MODE == 3)
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i] + (float)hx[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, float* d, int iters) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((kern<MODE>), dim3(256), dim3(512), 0, 0, d, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((kern<MODE>), dim3(256), dim3(512), 0, 0, d, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    // per SIMD: 2 waves x iters x 8 instructions
    const double cyc_per_instr = ms * 1e-3 * 2.1e9 / (2.0 * iters * 8);
    printf("%-24s %8.3f ms  ~%.2f cycles/instr/SIMD at 2.1 GHz\n", name, ms, cyc_per_instr);
}

int main() {
    float* d;
    (void)hipMalloc(&d, 256 * 512 * sizeof(float));
    const int iters = 200000;
    run<0>("v_exp_f32", d, iters);
    run<2>("v_exp_f16 (elementwise)", d, iters);
    run<3>("v_add_f32", d, iters);
    (void)hipFree(d);
    return 0;
}
