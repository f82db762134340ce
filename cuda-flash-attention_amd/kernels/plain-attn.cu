// plain-attn.cu -- FA2 forward on the vector ALU only (no MFMA), fp32, for MI355X.
// A comparison baseline for the CuPy face only.
//
// Replaces detker/CUDA-Flash-Attention kernels/plain-attn.cu, the harness's
// "fa2-naive" kernel (flash_attention2_forward_kernel_wrapper, :274-289, launched
// by test_flash_attention2.py:374-426: grid B*H*ceil(S/32), 256 threads, head_dim
// 64).  Same FA2 algorithm as the optimised files -- one workgroup per 32 query
// rows, online softmax over 32-key K/V blocks -- written the plain way: every
// product is a scalar v_fma_f32, so against kernel_fa2_optimized.cu (the same math
// on v_mfma_f32_32x32x2_f32) it isolates what the matrix cores buy.  The
// reference compiles this file only for the harness (its CLI never links it), and
// so does this build.
//
// Layout per workgroup: 8 threads per query row (tid = 8 row + part).  Scores:
// thread (row, part) takes keys part, part + 8, part + 16, part + 24 of the block;
// row max / sum are xor-shuffles over the 8 threads of the row; P goes through LDS
// for the P.V step, in which each thread owns D/8 output columns.
//
// Self-contained device code (hiprtc-compilable with -DCUPY_INLINE_COMPILE, C++14).

namespace fa2plain {

template <int D>
__device__ void plain_fa2_block(const float* __restrict__ Q, const float* __restrict__ K,
                                const float* __restrict__ V, float* __restrict__ O, float* __restrict__ LSE, int S,
                                int qb) {
    constexpr int LD = D + 1;  // odd row stride: the 8 threads of a row walk different banks
    __shared__ float qs[32 * LD], ks[32 * LD], vs[32 * LD], ps[32 * 33];
    const int tid = threadIdx.x, row = tid >> 3, part = tid & 7;
    const int q = 32 * qb + row;
    const float scale = 1.f / __builtin_sqrtf((float)D);

    for (int x = tid; x < 32 * D; x += 256) {
        const int rr = x / D, c = x - rr * D;
        qs[rr * LD + c] = (32 * qb + rr < S) ? Q[(long)(32 * qb + rr) * D + c] * scale : 0.f;
    }
    float o[D / 8];
#pragma unroll
    for (int c = 0; c < D / 8; ++c) o[c] = 0.f;
    float m = -__builtin_inff(), l = 0.f;

    const int nb = (S + 31) / 32;
    for (int j = 0; j < nb; ++j) {
        __syncthreads();
        for (int x = tid; x < 32 * D; x += 256) {
            const int rr = x / D, c = x - rr * D;
            const int key = 32 * j + rr;
            ks[rr * LD + c] = key < S ? K[(long)key * D + c] : 0.f;
            vs[rr * LD + c] = key < S ? V[(long)key * D + c] : 0.f;
        }
        __syncthreads();
        float s[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int kk = part + 8 * t;
            float acc = 0.f;
#pragma unroll 16
            for (int c = 0; c < D; ++c) acc = __builtin_fmaf(qs[row * LD + c], ks[kk * LD + c], acc);
            s[t] = (32 * j + kk < S) ? acc : -__builtin_inff();
        }
        float mx = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
#pragma unroll
        for (int o8 = 1; o8 < 8; o8 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o8));
        const float mn = fmaxf(m, mx);
        const float alpha = __expf(m - mn);  // 0 on the first block (m = -inf)
        float rs = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            s[t] = __expf(s[t] - mn);
            rs += s[t];
            ps[row * 33 + part + 8 * t] = s[t];
        }
#pragma unroll
        for (int o8 = 1; o8 < 8; o8 <<= 1) rs += __shfl_xor(rs, o8);
        l = l * alpha + rs;
        m = mn;
        __syncthreads();
#pragma unroll
        for (int c = 0; c < D / 8; ++c) {
            const int col = part + 8 * c;
            float acc = o[c] * alpha;
#pragma unroll 8
            for (int kk = 0; kk < 32; ++kk) acc = __builtin_fmaf(ps[row * 33 + kk], vs[kk * LD + col], acc);
            o[c] = acc;
        }
    }
    if (q < S) {
        const float inv = 1.f / l;
#pragma unroll
        for (int c = 0; c < D / 8; ++c) O[(long)q * D + part + 8 * c] = o[c] * inv;
        if (part == 0) LSE[q] = m + __logf(l);
    }
}

}  // namespace fa2plain

// CuPy face (same symbol and launch as plain-attn.cu:274-289): head_dim 64 as there.
extern "C" __global__ void __launch_bounds__(256)
flash_attention2_forward_kernel_wrapper(const float* query, const float* key, const float* value, float* output,
                                        float* logsumexp, int batch_size, int num_heads, int seq_len) {
    (void)batch_size;
    (void)num_heads;
    const int nqb = (seq_len + 31) / 32;
    const long bh = blockIdx.x / nqb;
    const int qb = blockIdx.x - (int)(bh * nqb);
    const long base = bh * seq_len * 64;
    fa2plain::plain_fa2_block<64>(query + base, key + base, value + base, output + base, logsumexp + bh * seq_len,
                                  seq_len, qb);
}
