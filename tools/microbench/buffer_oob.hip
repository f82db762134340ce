// Buffer out-of-range behaviour on gfx950 with the descriptor the kernels use
// (stride 0, dword3 0x00020000): does a load past num_records return 0, and is a
// store / atomic past num_records dropped?  Offsets past the range are put in the
// VGPR offset (voffset) or the SGPR offset (soffset).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* buf, int nrec_bytes, int mode, float* out) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, nrec_bytes, 0x00020000);
    const int lane = threadIdx.x;
    // lane l: byte offset 4 * l (the buffer holds 16 floats in range = lanes 0..15)
    if (mode == 0) {  // load, offset in voffset
        out[lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
    } else if (mode == 1) {  // load, offset in soffset (uniform) + small voffset
        out[lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (lane & 15) * 4, (lane >> 4) * 64, 0));
    } else if (mode == 2) {  // store, offset in voffset
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, -1.f), rs, lane * 4, 0, 0);
    } else if (mode == 3) {  // store, offset in soffset
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, -1.f), rs, (lane & 15) * 4, (lane >> 4) * 64, 0);
    } else if (mode == 4) {  // atomic add (int), offset in voffset
        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rs, lane * 4, 0, 0);
    } else if (mode == 5) {  // store at a huge voffset (0x40000000) from lanes >= 16
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, -2.f), rs, lane < 16 ? lane * 4 : 0x40000000 + lane * 4, 0, 0);
    }
}

int main() {
    // floats: 1 GiB + 1 MiB, so that mode 5's stores past the range stay inside the
    // allocation whatever the hardware does with them (no fault)
    const int N = (1 << 28) + (1 << 18);  // the probe's range is the first 16
    float *buf, *out;
    hipMalloc(&buf, N * 4);
    hipMalloc(&out, 64 * 4);
    std::vector<float> h(N), o(64);
    for (int mode = 0; mode < 6; ++mode) {
        for (int i = 0; i < N; ++i) h[i] = (float)(i + 1);
        hipMemcpy(buf, h.data(), N * 4, hipMemcpyHostToDevice);
        hipMemset(out, 0xff, 64 * 4);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, 64, mode, out);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), buf, N * 4, hipMemcpyDeviceToHost);
        hipMemcpy(o.data(), out, 64 * 4, hipMemcpyDeviceToHost);
        int changed_out = 0, first = -1;
        for (int i = 16; i < N; ++i)
            if (h[i] != (float)(i + 1)) { ++changed_out; if (first < 0) first = i; }
        int changed_in = 0;
        for (int i = 0; i < 16; ++i) changed_in += h[i] != (float)(i + 1);
        if (mode <= 1) {
            int zero = 0, mem = 0;
            for (int l = 16; l < 64; ++l) { zero += o[l] == 0.f; mem += o[l] == (float)(l + 1); }
            printf("mode %d load : in-range ok %d; past range: %d lanes read 0, %d read memory\n", mode,
                   o[3] == 4.f, zero, mem);
        } else {
            printf("mode %d %-5s: in-range changed %d/16; words past the range changed %d (first at %d)\n", mode,
                   mode == 4 ? "atom" : "store", changed_in, changed_out, first);
        }
    }
    return 0;
}
