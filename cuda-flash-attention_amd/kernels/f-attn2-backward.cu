// f-attn2-backward.cu -- FA2 backward, exact-fp32 path, for MI355X (gfx950).
//
// Replaces detker/CUDA-Flash-Attention kernels/f-attn2-backward.cu
// (flash_attention2_backward_kernel :33-339, D_computation_reduction_kernel
// :341-380, host launcher :384-488, CuPy wrappers :491-528).  Same results:
//   Δ_i = Σ_d dO_id·O_id                              (:341-380)
//   P = exp(QKᵀ/√D − LSE), dV = PᵀdO, dS = P∘(dOVᵀ − Δ)/√D, dK = dSᵀQ, dQ = dS·K.
//
// The reference adds dQ into a pre-zeroed buffer with global fp32 atomics from every
// 32-key workgroup (:269-301, zeroing at :427-429 / harness :546-548).  Here dQ has
// no atomics and needs no pre-zeroing: a workgroup in the dQ ROLE owns 32 query
// rows and walks all keys (recomputing S and dP for them), so every dQ element is
// summed in one fixed order inside one workgroup and written once.  Results are
// bitwise reproducible and no cross-workgroup read-modify-write of dQ exists.  (r03's
// zero-then-atomics design lost one key block's dQ once on a driver box; DESIGN.md §3
// "Exact-fp32 path" records what the evidence does and does not establish about why.)
//
// Roles (both on v_mfma_f32_32x32x2_f32, exact fp32 products, fp32 accumulation):
//   dK/dV role (4 GEMMs): 32 keys per workgroup; the four waves split the query
//     range (wave w takes every 4th 32-row tile of a 128-row Q/dO super-tile staged
//     in LDS) and sum their dKᵀ/dVᵀ register accumulators through LDS at the end.
//     S and dP have the key on the lane, so the P / dS accumulator registers feed
//     dVᵀ += dOᵀP and dKᵀ += QᵀdS directly as B operands.
//   dQ role (3 GEMMs): 32 queries per workgroup; the four waves split the key range
//     (wave w takes every 4th 32-key tile of a 128-key K/V super-tile) and sum their
//     dQᵀ accumulators through LDS.  Sᵀ and dPᵀ have the QUERY on the lane, so the
//     −LSE / −Δ seeds are one lane constant each and the dSᵀ accumulator registers
//     feed dQᵀ += KᵀdSᵀ directly as B operands.
// The library launch (launch_backward_f32) runs the two roles side by side in one
// grid of 2·B·H·⌈S/32⌉ workgroups after the Δ kernel.  The CuPy face keeps the
// harness's grid B·H·⌈S/32⌉ x 256 threads (test_flash_attention2.py:499-535): each
// workgroup runs the dK/dV role for key block i, then the dQ role for query block i.
//
// Self-contained device code (hiprtc -std=c++14 -DCUPY_INLINE_COMPILE).
#ifndef CUPY_INLINE_COMPILE
#include "f-attn2.cuh"
#endif

namespace fa2f32b {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define FA2FB_LOG2E 1.4426950408889634f

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

template <int D>
__device__ __forceinline__ void stage_rows(float* tile, const float* __restrict__ src, int row0, int ROWS, int S,
                                           int tid, float scale) {
    for (int x = tid; x < ROWS * (D / 4); x += 256) {
        const int row = x / (D / 4), c4 = x - row * (D / 4);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (row0 + row < S) v = *reinterpret_cast<const f32x4*>(src + (long)(row0 + row) * D + 4 * c4);
        *reinterpret_cast<f32x4*>(tile + row * (D + 4) + 4 * c4) = v * scale;
    }
}

// stage_rows split in two (guide T14): the loads into registers, issued a compute
// phase ahead of the LDS stores, so the L2/HBM round trip hides under MFMAs.
template <int D, int ROWS>
struct RowStage {
    static constexpr int N = ROWS * (D / 4) / 256;  // f32x4 chunks per thread
    f32x4 v[N];
    __device__ __forceinline__ void load(const float* __restrict__ src, int row0, int S, int tid) {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const int x = tid + 256 * c, row = x / (D / 4), c4 = x - row * (D / 4);
            v[c] = row0 + row < S ? *reinterpret_cast<const f32x4*>(src + (long)(row0 + row) * D + 4 * c4)
                                  : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    __device__ __forceinline__ void store(float* tile, float scale, int tid) const {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const int x = tid + 256 * c, row = x / (D / 4), c4 = x - row * (D / 4);
            *reinterpret_cast<f32x4*>(tile + row * (D + 4) + 4 * c4) = v[c] * scale;
        }
    }
};

// ---------------------------------------------------------------------------
// Δ = rowsum(dO ∘ O).  Reference-geometry body: one row per workgroup, any
// blockDim <= 1024 (the harness uses 64, test_flash_attention2.py:504-506).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void delta_row_body(const float* __restrict__ dO, const float* __restrict__ O, int rows,
                                               int D, float* __restrict__ Dvec) {
    __shared__ float part[16];
    const long row = blockIdx.x;
    if (row >= rows) return;
    float acc = 0.f;
    for (int d = threadIdx.x; d < D; d += blockDim.x) acc += dO[row * D + d] * O[row * D + d];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    const int nw = (blockDim.x + 63) / 64;
    if (nw == 1) {
        if (threadIdx.x == 0) Dvec[row] = acc;
        return;
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += part[w];
        Dvec[row] = s;
    }
}

// Library Δ kernel: D/4 lanes per row (float4 loads), grid-stride over rows.
template <int D>
__global__ void __launch_bounds__(256) fa2_delta_kernel(const float* __restrict__ dO, const float* __restrict__ O,
                                                        float* __restrict__ Dvec, long rows) {
    constexpr int LPR = D / 4;  // lanes per row
    const long stride = (long)gridDim.x * (256 / LPR);
    const int sub = threadIdx.x % LPR;
    for (long row = (long)blockIdx.x * (256 / LPR) + threadIdx.x / LPR; row < rows; row += stride) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(dO + row * D + 4 * sub);
        const f32x4 b = *reinterpret_cast<const f32x4*>(O + row * D + 4 * sub);
        float acc = a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
#pragma unroll
        for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if (sub == 0) Dvec[row] = acc;
    }
}

// ---------------------------------------------------------------------------
// LDS of both roles, in two regions:
//   TR = a 128-row super-tile (Q/dO for dK/dV, K/V for dQ; the 4-wave merge buffer
//        of either role at the end) + the dK/dV role's lse2 / Δ rows;
//   KD = two 32-row tiles (this block's K and V for dK/dV, its Q and dO for dQ).
// ---------------------------------------------------------------------------
template <int D> struct BwdLds {
    static constexpr int LD = D + 4;
    static constexpr int T = 128 * LD;
    static constexpr int ROWS = 2 * 128;
    static constexpr int KV = 32 * LD;
    static constexpr int TR = T + ROWS;
    static constexpr int KD = 2 * KV;
    static constexpr int FLOATS = TR + KD;
};

// dK/dV role: key block `blk` (bh = blk / ⌈S/32⌉), 32 keys, 4 waves over the queries.
template <int D>
__device__ __forceinline__ void dkdv_f32_body(const float* __restrict__ Q, const float* __restrict__ K,
                                              const float* __restrict__ V, const float* __restrict__ dO,
                                              const float* __restrict__ LSE, const float* __restrict__ Delta,
                                              float* __restrict__ dK, float* __restrict__ dV, int BH, int S, int blk,
                                              float* tr_lds, float* kd_lds) {
    constexpr int LD = D + 4;
    constexpr int QS = 128;
    float* T = tr_lds;
    float* lse2 = T + BwdLds<D>::T;
    float* del = lse2 + QS;
    float* Kt = kd_lds;
    float* Vt = Kt + BwdLds<D>::KV;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int nkb = (S + 31) / 32;
    const int bh = blk / nkb, kb = blk - bh * nkb;
    if (bh >= BH) return;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int k0 = kb * 32;
    const float qscale = FA2FB_LOG2E / __builtin_sqrtf((float)D);
    const float dscale = 1.f / __builtin_sqrtf((float)D);

    stage_rows<D>(Kt, K + base, k0, 32, S, tid, 1.f);
    stage_rows<D>(Vt, V + base, k0, 32, S, tid, 1.f);

    f32x16 dka[D / 32], dva[D / 32];
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            dka[b][i] = 0.f;
            dva[b][i] = 0.f;
        }

    // Q and dO super-tiles go HBM -> registers one compute phase before they are
    // needed (RowStage), so each LDS restage costs a barrier pair but no round trip:
    // dO(st) loads during S(st), Q(st + 1) loads during dK(st).  Q(st) is loaded
    // once and stored twice from the same registers: scaled for S, unscaled for dK.
    const int nsuper = (S + QS - 1) / QS;
    RowStage<D, QS> rq, rd;
    float rl = 0.f, rdel = 0.f;  // this thread's LSE / Δ row of the next super-tile (tid < QS)
    auto load_rows = [&](int q0) {
        if (tid < QS) {
            const int qi = q0 + tid;
            rl = qi < S ? LSE[rbase + qi] * FA2FB_LOG2E : __builtin_inff();
            rdel = qi < S ? Delta[rbase + qi] : 0.f;
        }
    };
    rq.load(Q + base, 0, S, tid);
    load_rows(0);
    rq.store(T, qscale, tid);
    if (tid < QS) {
        lse2[tid] = rl;
        del[tid] = rdel;
    }
    __syncthreads();
    for (int st = 0; st < nsuper; ++st) {
        const int q0 = st * QS;
        const int qw = q0 + 32 * wave;  // this wave's 32 query rows
        const bool active = qw < S;
        const bool more = st + 1 < nsuper;
        const float* Tw = T + 32 * wave * LD;
        rd.load(dO + base, q0, S, tid);
        // ---- S = Q K^T (T holds Q scaled), P
        f32x16 p;  // P[q][key]: rows q (registers), col key (lane)
        if (active) {
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = -lse2[32 * wave + acc_row(i, h)];
#pragma unroll
            for (int m = 0; m < D / 8; ++m) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(Tw + r * LD + 8 * m + 4 * h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(Kt + r * LD + 8 * m + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) p = mfma(a[e], b[e], p);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = (k0 + r < S) ? fast_exp2(p[i]) : 0.f;
        }
        // ---- dO
        __syncthreads();
        rd.store(T, 1.f, tid);
        __syncthreads();
        f32x16 ds;
        if (active) {
#pragma unroll
            for (int i = 0; i < 16; ++i) ds[i] = -del[32 * wave + acc_row(i, h)];
#pragma unroll
            for (int m = 0; m < D / 8; ++m) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(Tw + r * LD + 8 * m + 4 * h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(Vt + r * LD + 8 * m + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) ds = mfma(a[e], b[e], ds);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) ds[i] *= p[i];
            // dV^T += dO^T P
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) dva[b] = mfma(Tw[acc_row(i, h) * LD + 32 * b + r], p[i], dva[b]);
        }
        // ---- Q (unscaled, from the same registers) for dK; the next super-tile's row
        // constants (lse2 / del are read only by the S and dP phases, both done)
        if (more) load_rows(q0 + QS);
        __syncthreads();
        rq.store(T, 1.f, tid);
        if (more && tid < QS) {
            lse2[tid] = rl;
            del[tid] = rdel;
        }
        __syncthreads();
        if (more) rq.load(Q + base, q0 + QS, S, tid);
        if (active) {
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) dka[b] = mfma(Tw[acc_row(i, h) * LD + 32 * b + r], ds[i], dka[b]);
        }
        // ---- the next super-tile's Q, scaled
        if (more) {
            __syncthreads();
            rq.store(T, qscale, tid);
            __syncthreads();
        }
    }

    // ---- sum the four waves' dK^T / dV^T through LDS and write rows [k0, k0+32)
    for (int pass = 0; pass < 2; ++pass) {
        __syncthreads();
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x16& a = pass == 0 ? dka[b] : dva[b];
                const f32x4 v = {a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
                *reinterpret_cast<f32x4*>(T + (wave * 32 + r) * LD + 32 * b + 8 * g + 4 * h) = v;
            }
        __syncthreads();
        float* dst = pass == 0 ? dK : dV;
        const float sc = pass == 0 ? dscale : 1.f;
        for (int x = tid; x < 32 * (D / 4); x += 256) {
            const int row = x / (D / 4), c4 = x - row * (D / 4);
            if (k0 + row < S) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int w = 0; w < 4; ++w) acc += *reinterpret_cast<const f32x4*>(T + (w * 32 + row) * LD + 4 * c4);
                *reinterpret_cast<f32x4*>(dst + base + (long)(k0 + row) * D + 4 * c4) = acc * sc;
            }
        }
    }
}

// dQ role: query block `blk` (bh = blk / ⌈S/32⌉), 32 queries, 4 waves over the keys.
// Per 128-key super-tile, one LDS buffer holds V (for dPᵀ) and then K (for Sᵀ and
// dQᵀ): dPᵀ (16 registers) is kept across the restage, so K and V never need LDS
// at the same time.  One RowStage carries K(st) during dPᵀ(st) and V(st + 1)
// during Sᵀ/dQᵀ(st).
template <int D>
__device__ __forceinline__ void dq_f32_body(const float* __restrict__ Q, const float* __restrict__ K,
                                            const float* __restrict__ V, const float* __restrict__ dO,
                                            const float* __restrict__ LSE, const float* __restrict__ Delta,
                                            float* __restrict__ dQ, int BH, int S, int blk, float* t_lds,
                                            float* qd_lds) {
    constexpr int LD = D + 4;
    constexpr int KS = 128;
    float* T = t_lds;
    float* Qt = qd_lds;
    float* Dt = qd_lds + 32 * LD;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int nqb = (S + 31) / 32;
    const int bh = blk / nqb, qb = blk - bh * nqb;
    if (bh >= BH) return;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int q0 = qb * 32;
    const float qscale = FA2FB_LOG2E / __builtin_sqrtf((float)D);
    const float dscale = 1.f / __builtin_sqrtf((float)D);

    stage_rows<D>(Qt, Q + base, q0, 32, S, tid, qscale);
    stage_rows<D>(Dt, dO + base, q0, 32, S, tid, 1.f);
    // this lane's query (column of every accumulator): the −LSE·log2e and −Δ seeds
    const int qi = q0 + r;
    const float nlse = qi < S ? -LSE[rbase + qi] * FA2FB_LOG2E : -__builtin_inff();
    const float ndel = qi < S ? -Delta[rbase + qi] : 0.f;

    f32x16 dqa[D / 32];
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) dqa[b][i] = 0.f;

    const int nsuper = (S + KS - 1) / KS;
    RowStage<D, KS> rs;
    rs.load(V + base, 0, S, tid);
    rs.store(T, 1.f, tid);
    __syncthreads();
    rs.load(K + base, 0, S, tid);
    for (int st = 0; st < nsuper; ++st) {
        const int k0 = st * KS;
        const int kw = k0 + 32 * wave;  // this wave's 32 keys
        const bool active = kw < S;
        const bool more = st + 1 < nsuper;
        const float* Tw = T + 32 * wave * LD;
        // ---- dPᵀ = V dOᵀ − Δ: keys on the registers' rows, queries on the lanes
        f32x16 dp;
        if (active) {
#pragma unroll
            for (int i = 0; i < 16; ++i) dp[i] = ndel;
#pragma unroll
            for (int m = 0; m < D / 8; ++m) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(Tw + r * LD + 8 * m + 4 * h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(Dt + r * LD + 8 * m + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) dp = mfma(a[e], b[e], dp);
            }
        }
        // ---- K over V
        __syncthreads();
        rs.store(T, 1.f, tid);
        __syncthreads();
        if (more) rs.load(V + base, k0 + KS, S, tid);
        if (active) {
            // Sᵀ = K (Q·log2e/√D)ᵀ − LSE·log2e, Pᵀ = exp2, dSᵀ = Pᵀ ∘ dPᵀ
            f32x16 p;
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = nlse;
#pragma unroll
            for (int m = 0; m < D / 8; ++m) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(Tw + r * LD + 8 * m + 4 * h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(Qt + r * LD + 8 * m + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) p = mfma(a[e], b[e], p);
            }
            f32x16 ds;
            if (kw + 32 <= S) {
#pragma unroll
                for (int i = 0; i < 16; ++i) ds[i] = fast_exp2(p[i]) * dp[i];
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) ds[i] = kw + acc_row(i, h) < S ? fast_exp2(p[i]) * dp[i] : 0.f;
            }
            // dQᵀ += Kᵀ dSᵀ: step i takes accumulator register i as B (k = h <-> key acc_row(i, h))
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) dqa[b] = mfma(Tw[acc_row(i, h) * LD + 32 * b + r], ds[i], dqa[b]);
        }
        // ---- the next super-tile's V
        if (more) {
            __syncthreads();
            rs.store(T, 1.f, tid);
            __syncthreads();
            rs.load(K + base, k0 + KS, S, tid);
        }
    }

    // ---- sum the four waves' dQᵀ through LDS and write rows [q0, q0+32)
    __syncthreads();
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 v = {dqa[b][4 * g], dqa[b][4 * g + 1], dqa[b][4 * g + 2], dqa[b][4 * g + 3]};
            *reinterpret_cast<f32x4*>(T + (wave * 32 + r) * LD + 32 * b + 8 * g + 4 * h) = v;
        }
    __syncthreads();
    for (int x = tid; x < 32 * (D / 4); x += 256) {
        const int row = x / (D / 4), c4 = x - row * (D / 4);
        if (q0 + row < S) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int w = 0; w < 4; ++w) acc += *reinterpret_cast<const f32x4*>(T + (w * 32 + row) * LD + 4 * c4);
            *reinterpret_cast<f32x4*>(dQ + base + (long)(q0 + row) * D + 4 * c4) = acc * dscale;
        }
    }
}

// One launch, two roles: workgroups [0, nblk) take the dK/dV role for key block
// blockIdx.x, workgroups [nblk, 2·nblk) the dQ role for query block blockIdx.x − nblk.
template <int D>
__global__ void __launch_bounds__(256)
fa2_bwd_f32_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                   const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
                   float* __restrict__ dQ, float* __restrict__ dK, float* __restrict__ dV, int BH, int S, int nblk) {
    __shared__ __attribute__((aligned(16))) float smem[BwdLds<D>::FLOATS];
    const int blk = blockIdx.x;
    if (blk < nblk)
        dkdv_f32_body<D>(Q, K, V, dO, LSE, Delta, dK, dV, BH, S, blk, smem, smem + BwdLds<D>::TR);
    else
        dq_f32_body<D>(Q, K, V, dO, LSE, Delta, dQ, BH, S, blk - nblk, smem, smem + BwdLds<D>::TR);
}

}  // namespace fa2f32b

#ifndef CUPY_INLINE_COMPILE
namespace fa2 {

namespace {
template <int D>
hipError_t delta_dispatch(const float* dout, const float* o, float* delta, int bh, int S, hipStream_t stream) {
    const long rows = (long)bh * S;
    const long rows_per_block = 256 / (D / 4);
    long grid = (rows + rows_per_block - 1) / rows_per_block;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL((fa2f32b::fa2_delta_kernel<D>), dim3((unsigned)grid), dim3(256), 0, stream, dout, o, delta,
                       rows);
    return hipGetLastError();
}
template <int D>
hipError_t bwd_f32_dispatch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                            const float* delta, float* dq, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    const long nblk = (long)bh * ((S + 31) / 32);
    if (nblk <= 0 || 2 * nblk > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f32b::fa2_bwd_f32_kernel<D>), dim3((unsigned)(2 * nblk)), dim3(256), 0, stream, q, k, v,
                       dout, lse, delta, dq, dk, dv, bh, S, (int)nblk);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_delta(int D, const float* dout, const float* o, float* delta, int bh, int S, hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    switch (D) {
        case 32: return delta_dispatch<32>(dout, o, delta, bh, S, stream);
        case 64: return delta_dispatch<64>(dout, o, delta, bh, S, stream);
        case 128: return delta_dispatch<128>(dout, o, delta, bh, S, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_backward_f32(int D, const float* q, const float* k, const float* v, const float* o,
                               const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                               int bh, int S, hipStream_t stream) {
    if (bh <= 0 || S <= 0 || !supported_head_dim(D)) return hipErrorInvalidValue;
    const hipError_t e = launch_delta(D, dout, o, delta, bh, S, stream);
    if (e != hipSuccess) return e;
    switch (D) {
        case 32: return bwd_f32_dispatch<32>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, stream);
        case 64: return bwd_f32_dispatch<64>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, stream);
        default: return bwd_f32_dispatch<128>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, stream);
    }
}

}  // namespace fa2

// Host API with the reference's semantics (f-attn2-backward.cu:384-485).
template <int head_dim>
void host_flash_attention2_backward(const float* h_Q, const float* h_K, const float* h_V, const float* h_O,
                                    const float* h_dO, const float* h_lse, float* h_dQ, float* h_dK, float* h_dV,
                                    int batch_size, int seq_len, int num_heads, TimerManager* tm) {
    const size_t n = (size_t)batch_size * num_heads * seq_len * head_dim;
    const size_t nl = (size_t)batch_size * num_heads * seq_len;
    float* d[10];
    const size_t sz[10] = {n, n, n, n, n, nl, nl, n, n, n};
    for (int i = 0; i < 10; ++i) HIP_CHECK(hipMalloc(&d[i], sz[i] * sizeof(float)));
    const float* src[6] = {h_Q, h_K, h_V, h_O, h_dO, h_lse};
    for (int i = 0; i < 6; ++i) HIP_CHECK(hipMemcpy(d[i], src[i], sz[i] * sizeof(float), hipMemcpyHostToDevice));
    tm->Start();
    HIP_CHECK(fa2::launch_backward_f32(head_dim, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9],
                                       batch_size * num_heads, seq_len, nullptr));
    tm->Stop();
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(h_dQ, d[7], n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_dK, d[8], n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_dV, d[9], n * sizeof(float), hipMemcpyDeviceToHost));
    for (int i = 0; i < 10; ++i) HIP_CHECK(hipFree(d[i]));
}
#define FA2_INST_BWD32(D)                                                                                    \
    template void host_flash_attention2_backward<D>(const float*, const float*, const float*, const float*, \
                                                    const float*, const float*, float*, float*, float*, int, \
                                                    int, int, TimerManager*);
FA2_INST_BWD32(32)
FA2_INST_BWD32(64)
FA2_INST_BWD32(128)
#else
// CuPy face (test_flash_attention2.py:132-141, 499-535).  The harness hands dQ/dK/dV
// in zeroed; here every element is overwritten.  Grid B·H·⌈S/32⌉: workgroup i runs
// the dK/dV role for key block i, then the dQ role for query block i.
// LDS: the launch adds the harness's dynamic bytes ((32D + 4*32D + 32 + 32*32)*4,
// 45 184 at D=64, :522-527) to this kernel's static bytes, and the sum must stay
// within the 160 KiB a workgroup may own.  Static LDS is therefore sized for
// D <= 64 (53 KB); at D = 128 the 128-row super-tile region moves into the dynamic
// region (86 KB provided there).  The dispatch packet's group_segment_size (static +
// dynamic) is checked first, so an undersized launch writes nothing instead of
// running past its LDS.
__device__ __forceinline__ unsigned fa2_group_segment_bytes() {
    // hsa_kernel_dispatch_packet_t: group_segment_size is the u32 at byte offset 28
    const unsigned char* pkt = (const unsigned char*)__builtin_amdgcn_dispatch_ptr();
    return *(const unsigned*)(pkt + 28);
}

extern "C" __global__ void __launch_bounds__(256)
flash_attention2_backward_kernel_wrapper(const float* query, const float* key, const float* value,
                                         const float* output, const float* d_output, const float* logsumexp,
                                         const float* d, float* d_query, float* d_key, float* d_value,
                                         int batch_size, int num_heads, int seq_len, int head_dim) {
    __shared__ __attribute__((aligned(16))) float smem[fa2f32b::BwdLds<64>::FLOATS];
    extern __shared__ __attribute__((aligned(16))) float dyn[];
    (void)output;
    const int bh = batch_size * num_heads;
    const int blk = blockIdx.x;
    const unsigned have = fa2_group_segment_bytes();
    if (head_dim == 64) {
        float* kd = smem + fa2f32b::BwdLds<64>::TR;
        fa2f32b::dkdv_f32_body<64>(query, key, value, d_output, logsumexp, d, d_key, d_value, bh, seq_len, blk, smem,
                                   kd);
        __syncthreads();
        fa2f32b::dq_f32_body<64>(query, key, value, d_output, logsumexp, d, d_query, bh, seq_len, blk, smem, kd);
    } else if (head_dim == 32) {
        float* kd = smem + fa2f32b::BwdLds<32>::TR;
        fa2f32b::dkdv_f32_body<32>(query, key, value, d_output, logsumexp, d, d_key, d_value, bh, seq_len, blk, smem,
                                   kd);
        __syncthreads();
        fa2f32b::dq_f32_body<32>(query, key, value, d_output, logsumexp, d, d_query, bh, seq_len, blk, smem, kd);
    } else if (head_dim == 128) {
        if (have < sizeof(smem) + 4u * fa2f32b::BwdLds<128>::TR) return;
        static_assert(fa2f32b::BwdLds<128>::KD <= fa2f32b::BwdLds<64>::FLOATS, "KD region must fit the static LDS");
        fa2f32b::dkdv_f32_body<128>(query, key, value, d_output, logsumexp, d, d_key, d_value, bh, seq_len, blk, dyn,
                                    smem);
        __syncthreads();
        fa2f32b::dq_f32_body<128>(query, key, value, d_output, logsumexp, d, d_query, bh, seq_len, blk, dyn, smem);
    }
}

// Note the output pointer comes last, as in the reference (f-attn2-backward.cu:515-528).
extern "C" __global__ void D_computation_reduction_kernel_wrapper(const float* d_output, const float* output,
                                                                  int batch_size, int num_heads, int seq_len,
                                                                  int head_dim, float* d) {
    fa2f32b::delta_row_body(d_output, output, batch_size * num_heads * seq_len, head_dim, d);
}
#endif  // CUPY_INLINE_COMPILE
