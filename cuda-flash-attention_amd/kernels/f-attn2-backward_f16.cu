// f-attn2-backward_f16.cu -- FA2 backward, fp16-tile MFMA path, for MI355X (gfx950).
//
// Replaces detker/CUDA-Flash-Attention kernels/f-attn2-backward_f16.cu
// (flash_attention2_backward_kernel_fp16 :34-330, D kernel :332-371, host
// launcher :375-474, CuPy wrappers :477-514).  Same math as the reference
// backward (f-attn2-backward.cu:119-338):
//   P  = exp(Q Kᵀ/√D − LSE)           (recomputed, :151-184)
//   dV = Pᵀ dO                        (:218-240)
//   dS = P ∘ (dO Vᵀ − Δ),  Δ = rowsum(dO∘O)   (:242-267, :341-380)
//   dQ = dS K / √D                    (:269-301, atomics there)
//   dK = dSᵀ Q / √D                   (:303-323)
//
// MI355X design: two MFMA kernels instead of one kernel
// with ~B·H·S²·D/32 global fp32 atomics (the chip-wide fp32 atomic rate,
// ≈1.3 TB/s, would bound the whole backward):
//   * fa2_bwd_dkdv_f16: one wave = 32 keys whose K, V fragments stay in VGPRs
//     and whose dKᵀ, dVᵀ accumulate in registers; the workgroup streams 64-row
//     Q/dO blocks through LDS.  S and dP are computed with the key on the lane,
//     their accumulators start at −LSE·log2e and −Δ (row constants as initial
//     accumulator), and the packed P / dS accumulators are directly the B
//     operands of dVᵀ += dOᵀP and dKᵀ += QᵀdS (dOᵀ, Qᵀ via ds_read_b64_tr_b16).
//   * fa2_bwd_dq_f16: one wave = 32 queries (Q, dO fragments in VGPRs) streaming
//     64-key K/V tiles; Sᵀ and dPᵀ with the query on the lane, dQᵀ += Kᵀ dSᵀ.
//   Deterministic (no atomics), dq/dk/dv fully written (no memsets).
//
// Self-contained device code (hiprtc-compilable with -DCUPY_INLINE_COMPILE, C++14).
#ifndef CUPY_INLINE_COMPILE
#include "f-attn2.cuh"
#endif

#ifdef FA2_TILE_BF16
#define fa2f16b fa2bf16b
#define FA2_TILE_LAUNCH(x) x##_bf16
#define FA2_TILE_HOST(x) x##_bf16
#else
#define FA2_TILE_LAUNCH(x) x##_f16
#define FA2_TILE_HOST(x) x##_fp16
#endif

namespace fa2f16b {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

#define FA2B_LOG2E 1.4426950408889634f

// Tile element type.  The default build stores fp16 tiles.  The same source compiled
// with -DFA2_TILE_BF16 (Makefile: *_bf16.o, namespace fa2bf16b, launchers *_bf16)
// keeps bf16 bits in the same 16-bit containers -- LDS images and fragments are only
// moved (ds_read_b128 / ds_read_b64_tr_b16 are type-blind), never computed on,
// except by the conversion below and the MFMA -- and runs the bf16 MFMA.
#ifdef FA2_TILE_BF16
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ _Float16 to_tile(float x) { return __builtin_bit_cast(_Float16, (__bf16)x); }
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}
#else
__device__ __forceinline__ _Float16 to_tile(float x) { return (_Float16)x; }
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
#endif
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// dS = P * (dP - Δ) for a pair of scores, as tile values.  fp16 tiles: the product
// of the already-packed fp16 P and the packed (dP - Δ) (v_cvt_pk + v_pk_mul_f16: one
// issue per score fewer than two f32 products and a conversion); bf16 tiles: the f32
// products, rounded once.
typedef _Float16 tile2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ tile2 ds_pair(float p0, float p1, float d0, float d1, _Float16 ph0, _Float16 ph1) {
#ifndef FA2_TILE_BF16
    (void)p0;
    (void)p1;
    return tile2{ph0, ph1} * tile2{(_Float16)d0, (_Float16)d1};
#else
    (void)ph0;
    (void)ph1;
    return tile2{to_tile(p0 * d0), to_tile(p1 * d1)};
#endif
}

template <int D> struct Swz;
// XOR swizzle of the 16-byte chunk index of LDS row r, searched (tools/lds_swizzle.py,
// `swz_shipped`) to make ds_read_b128 row fragments and ds_read_b64_tr_b16 transposed
// fragments bank-conflict-free for both the 32x32x16 and the 16x16x32 operand maps
// (r01's first swizzle, searched for 32x32x16 only, left the 16x16x32 row reads 2-way:
// 27-36 % extra LDS cycles in dK/dV and dQ).  Reads row bits 0..3 only (fragment
// offsets are shifted by whole 16-row blocks).
template <> struct Swz<32> {
    static __device__ __forceinline__ int f(int r) { return ((r >> 2) & 1) | ((((r >> 2) ^ (r >> 3)) & 1) << 1); }
};
template <> struct Swz<64> {
    static __device__ __forceinline__ int f(int r) {
        return ((r >> 1) & 1) | ((((r >> 1) ^ (r >> 2)) & 1) << 1) | ((((r >> 1) ^ (r >> 3)) & 1) << 2);
    }
};
template <> struct Swz<128> {
    static __device__ __forceinline__ int f(int r) {
        return (r & 1) | (((r >> 1) & 1) << 1) | (((r ^ (r >> 2)) & 1) << 2) | (((r ^ (r >> 1) ^ (r >> 3)) & 1) << 3);
    }
};
template <int D>
__device__ __forceinline__ int tile_off(int row, int col) {
    return row * D + (((col >> 3) ^ Swz<D>::f(row)) << 3) + (col & 7);
}
__device__ __forceinline__ f16x8 lds_row8(const _Float16* p) { return *reinterpret_cast<const f16x8*>(p); }
__device__ __forceinline__ i16x4 lds_tr4(const _Float16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p));
}
__device__ __forceinline__ f16x8 cat4(i16x4 a, i16x4 b) {
    i16x8 c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(f16x8, c);
}
__device__ __forceinline__ f16x8 to_f16x8(f32x4 a, f32x4 b, float s) {
    f16x8 r;
    r[0] = to_tile(a[0] * s); r[1] = to_tile(a[1] * s); r[2] = to_tile(a[2] * s); r[3] = to_tile(a[3] * s);
    r[4] = to_tile(b[0] * s); r[5] = to_tile(b[1] * s); r[6] = to_tile(b[2] * s); r[7] = to_tile(b[3] * s);
    return r;
}
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, rr = nwg & 7, xcd = orig & 7, idx = orig >> 3;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
}
// fragment of 8 consecutive fp32 (row `row` of a [S][D] tensor, cols c..c+7) as fp16
__device__ __forceinline__ f16x8 load_frag(const float* __restrict__ p, bool valid, float s) {
    if (!valid) return f16x8{0, 0, 0, 0, 0, 0, 0, 0};
    const f32x4* v = reinterpret_cast<const f32x4*>(p);
    return to_f16x8(v[0], v[1], s);
}

// Per-lane LDS element offsets into a swizzled [rows][D] fp16 tile.  The swizzle
// only reads row bits 0..3, so one set serves every 32-row block and 16-row
// sub-step (those add row*D constants the compiler folds into ds_read offsets).
template <int D>
struct FragOffsets {
    int row[D / 16];    // A operand from rows: row lane&31, k-chunk 2t + lane>>5
    int tr[D / 32][2];  // transposed operand (tr_operand), rows +0 and +8
    __device__ __forceinline__ void init(int lane) {
        const int r = lane & 31, h = lane >> 5, g = lane >> 4, i = lane & 15;
#pragma unroll
        for (int t = 0; t < D / 16; ++t) row[t] = tile_off<D>(r, 16 * t + 8 * h);
        const int rt = 4 * (g >> 1) + (i >> 2), ct = 16 * (g & 1) + 4 * (i & 3);
#pragma unroll
        for (int b = 0; b < D / 32; ++b) {
            tr[b][0] = tile_off<D>(rt, 32 * b + ct);
            tr[b][1] = tile_off<D>(rt + 8, 32 * b + ct);
        }
    }
    // A operand, k over rows r0 .. r0+15 of the tile (r0 multiple of 16), columns 32b..32b+31
    __device__ __forceinline__ f16x8 trop(const _Float16* tile, int r0, int b) const {
        return cat4(lds_tr4(tile + tr[b][0] + r0 * D), lds_tr4(tile + tr[b][1] + r0 * D));
    }
    // A operand, rows r0 + (lane&31), k-chunk t
    __device__ __forceinline__ f16x8 rowop(const _Float16* tile, int r0, int t) const {
        return lds_row8(tile + row[t] + r0 * D);
    }
};

// Buffer descriptor over one head's [S][D] fp32 rows: the hardware range check
// returns zeros for rows >= S, so ragged tiles need no guards.  Built from
// wave-uniform values only (readfirstlane), so no waterfall loops (guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const float* base, int S, int D) {
    const unsigned long long a = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane(S * D * 4);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes,
                                             0x00020000);
}
__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

// Register-staged tile loader: ROWS x D fp32 rows of one head's [S][D] tensor ->
// fp16 swizzled LDS, CPT chunks (8 floats) per thread, byte offsets computed once;
// buffer loads take the tile origin as a scalar offset (no per-load VALU).
template <int D, int ROWS, int NT>
struct TileStager {
    static constexpr int CPR = D / 8;
    static constexpr int CHUNKS = ROWS * CPR;
    static constexpr int CPT = (CHUNKS + NT - 1) / NT;
    static constexpr bool EXACT = CHUNKS % NT == 0;
    f32x4 r[CPT][2];
    int voff[CPT], loff[CPT];
    __amdgpu_buffer_rsrc_t rs;
    bool on = true;  // wave-uniform: this wave takes part in the staging

    __device__ __forceinline__ void init(const float* head_base, int S, int tid) {
        rs = head_rsrc(head_base, S, D);
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int x = tid + c * NT;
            const int row = x / CPR, ch = x % CPR;
            voff[c] = (EXACT || x < CHUNKS) ? (row * D + ch * 8) * 4 : 0x7ffffff0;  // inactive: out of range
            loff[c] = row * D + ((ch ^ Swz<D>::f(row)) << 3);
        }
    }
    // rows [row0, row0 + ROWS); rows >= S read as zeros
    __device__ __forceinline__ void load(int row0) {
        if (!on) return;
        const int soff = row0 * D * 4;
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            r[c][0] = buf_load4(rs, voff[c], soff);
            r[c][1] = buf_load4(rs, voff[c] + 16, soff);
        }
    }
    __device__ __forceinline__ void store(_Float16* tile, float scale, int tid) const {
        if (!on) return;
#pragma unroll
        for (int c = 0; c < CPT; ++c)
            if (EXACT || tid + c * NT < CHUNKS)
                *reinterpret_cast<f16x8*>(tile + loff[c]) = to_f16x8(r[c][0], r[c][1], scale);
    }
};

// Row-coalesced prologue / epilogue.  A workgroup's stationary
// operand block (K and V for dK/dV, Q and dO for dQ) is one contiguous HBM range:
// it is loaded whole rows at a time into the (still idle) LDS tile buffers as scaled
// fp16 and read back as B fragments, instead of every lane fetching 16-B pieces of
// its own row (32 rows per instruction).  Results leave through a wave-private LDS
// stage as whole 128-B row segments.


// Δ = rowsum(dO ∘ O) of a staged block's rows, from the row-coalesced registers of
// its dO and O stagers: the CPR threads that hold one row's chunks are consecutive
// lanes, reduced with xor shuffles.  Δ goes to `delta_lds` (this workgroup's rows)
// and to HBM for the dK/dV kernel.
// NEG: -Δ into `delta_lds` (the dP accumulators' initial value); delta_out may be null.
template <int D, int ROWS, int NT, bool NEG = false>
__device__ __forceinline__ void delta_rows(const TileStager<D, ROWS, NT>& a, const TileStager<D, ROWS, NT>& o, int S,
                                           int row0, float* delta_lds, float* __restrict__ delta_out, int tid) {
    using TS = TileStager<D, ROWS, NT>;
#pragma unroll
    for (int c = 0; c < TS::CPT; ++c) {
        const int x = tid + c * NT;
        const f32x4 p0 = a.r[c][0] * o.r[c][0], p1 = a.r[c][1] * o.r[c][1];
        float d = ((p0[0] + p0[1]) + (p0[2] + p0[3])) + ((p1[0] + p1[1]) + (p1[2] + p1[3]));
#pragma unroll
        for (int off = TS::CPR / 2; off > 0; off >>= 1) d += __shfl_xor(d, off);
        const int row = x / TS::CPR;
        if ((TS::EXACT || x < TS::CHUNKS) && x % TS::CPR == 0) {
            delta_lds[row] = NEG ? -d : d;
            if (delta_out && row0 + row < S) delta_out[row0 + row] = d;
        }
    }
}

// a wave's 32 x D accumulator block (row d = 32b + (i&3) + 8(i>>2) + 4h of the
// transposed result, column = lane & 31 = output row) -> rows [0, rows_valid) of dst
template <int D>
__device__ __forceinline__ void store_block_rows(float (*os)[36], const f32x16 (&acc)[D / 32], float scale,
                                                 float* __restrict__ dst, int rows_valid, int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int b = 0; b < D / 32; ++b) {
#pragma unroll
        for (int i = 0; i < 16; ++i) os[r][(i & 3) + 8 * (i >> 2) + 4 * h] = acc[b][i] * scale;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int row = 8 * s4 + (lane >> 3), c4 = (lane & 7) * 4;
            const f32x4 v = *reinterpret_cast<const f32x4*>(&os[row][c4]);
            if (row < rows_valid) *reinterpret_cast<f32x4*>(dst + (long)row * D + 32 * b + c4) = v;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// dK, dV:  grid BH * ceil(S / (32*NW)), block 64*NW
// ---------------------------------------------------------------------------
template <int D, int KB>
struct DkdvState {
    // KB blocks of 32 keys per wave: B operands (this lane's key rows of K, scaled, and V)
    f16x8 kf[KB][D / 16], vf[KB][D / 16];
    f32x16 dka[KB][D / 32], dva[KB][D / 32];
};

// One 64-query step for the wave's KB x 32 keys: S = Q K^T and dP = dO V^T with the
// key on the lane (their accumulators start at -LSE*log2e and -Delta), P = exp2(S),
// dS = P*(dP - Delta), then dV^T += dO^T P and dK^T += Q^T dS with P / dS packed as
// B operands.  Every LDS fragment (Q / dO rows, dO^T / Q^T columns) feeds KB MFMAs.
template <int D, int KB, typename Mid>
__device__ __forceinline__ void dkdv_step(DkdvState<D, KB>& st, const _Float16* Qs, const _Float16* dOs,
                                          const float* nlse2, const float* ndel, const FragOffsets<D>& fo, int h,
                                          Mid&& mid) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        if (qb == 1) mid();  // between the two query blocks (staging loads, FA2_DKDV_LP)
        // accumulator rows: query qb*32 + (i&3) + 8*(i>>2) + 4h ; col: key (lane)
        f32x16 init_s, init_d;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(nlse2 + qb * 32 + 8 * g + 4 * h);
            const f32x4 dv = *reinterpret_cast<const f32x4*>(ndel + qb * 32 + 8 * g + 4 * h);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                init_s[4 * g + e] = lv[e];
                init_d[4 * g + e] = dv[e];
            }
        }
        f32x16 sa[KB], da[KB];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            sa[kb] = init_s;
            da[kb] = init_d;
        }
#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
            const f16x8 qa = fo.rowop(Qs, qb * 32, t), da_op = fo.rowop(dOs, qb * 32, t);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                sa[kb] = mfma(qa, st.kf[kb][t], sa[kb]);
                da[kb] = mfma(da_op, st.vf[kb][t], da[kb]);
            }
        }
        f16x8 pf[KB][2], dsf[KB][2];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = fast_exp2(sa[kb][i]);
                pf[kb][i >> 3][i & 7] = to_tile(p);
                dsf[kb][i >> 3][i & 7] = to_tile(p * da[kb][i]);
            }
        // dV^T += dO^T P ; dK^T += Q^T dS over this query block's 32 rows
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const f16x8 a_do = fo.trop(dOs, qb * 32 + 16 * s, b), a_q = fo.trop(Qs, qb * 32 + 16 * s, b);
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) {
                    st.dva[kb][b] = mfma(a_do, pf[kb][s], st.dva[kb][b]);
                    st.dka[kb][b] = mfma(a_q, dsf[kb][s], st.dka[kb][b]);
                }
            }
    }
}

// Staging of the next Q/dO step in the dK/dV kernel is done by waves 0-3 only: stamps
// showed waves 4-7 (which lose VALU arbitration to their SIMD partners) ~15 % slower
// per step and the first half idling at the barrier (r01).  The dQ kernel's waves 4-7
// run at s_setprio 1 (MI355X_MICROARCH §Two waves per SIMD, item 4: +1 %); its next-step
// K/V loads are issued on the last step too (rows past S read as zeros through the
// range-checked descriptor, no memory traffic), which removed 8 v_mov_b64 of
// staging-register phi copies per step (+0.7 % at C3, +8.8 % at D = 128).
#define FA2_DKDV_SW 4

// ---- dK, dV on v_mfma_f32_16x16x32 ----------------------------------------------
// Same algorithm and data flow as dkdv_step; the wave's 32 keys are two 16-key
// blocks nb.  Measured at the power cap on random data (tools/microbench/mfma_lds.hip):
// 16x16x32 delivers 16 % more FLOPs per joule than 32x32x16 (it reads and writes a
// quarter of the accumulator per instruction for half the FLOPs), +9 % with a
// dK/dV-like exp/VALU mix beside it.
// Operand maps (lane l, g = l >> 4): A[m = l & 15][k = 8g + j], B[k = 8g + j][n = l & 15],
// C[m = 4g + i][n = l & 15].
//   S / dP (m = query, n = key, k = d): A = Q / dO rows (row reads), B = K / V
//     fragments in VGPRs; accumulators start at -lse2 / -delta of rows 4g + i.
//   dV^T / dK^T (m = d, n = key, k = query): B = P / dS packed from the two query
//     blocks mb: k-slot 8g + j <-> query 16 (j >> 2) + 4g + (j & 3); A = dO^T / Q^T
//     by two 4-row transposed reads (rows 4g.. and 16 + 4g.., columns 16 md..).
template <int D>
struct DkdvState16 {
    f16x8 kf[2][D / 32], vf[2][D / 32];  // [nb][ks]: K / V[key 16 nb + (l&15)][d 32 ks + 8g ..]
    f32x4 dka[D / 16][2], dva[D / 16][2];  // [md][nb]: C[d 16 md + 4g + i][key 16 nb + (l&15)]
};

template <int D>
struct FragOffsets16 {
    int row[D / 32];   // row read: row (l & 15), columns 32 ks + 8g .. +7
    int tr[D / 16][2];  // transposed read of block md: rows 4g + q / 16 + 4g + q, columns 16 md + 4p
    __device__ __forceinline__ void init(int lane) {
        const int i = lane & 15, g = lane >> 4, q = i >> 2, p4 = i & 3;
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) row[ks] = tile_off<D>(i, 32 * ks + 8 * g);
#pragma unroll
        for (int md = 0; md < D / 16; ++md) {
            tr[md][0] = tile_off<D>(4 * g + q, 16 * md + 4 * p4);
            tr[md][1] = tile_off<D>(16 + 4 * g + q, 16 * md + 4 * p4);
        }
    }
    // move every offset by o halves (a wave's fixed tile inside a multi-tile image)
    __device__ __forceinline__ void shift(int o) {
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) row[ks] += o;
#pragma unroll
        for (int md = 0; md < D / 16; ++md) {
            tr[md][0] += o;
            tr[md][1] += o;
        }
    }
    // A operand: rows r0 + (l & 15), k-step ks over columns
    __device__ __forceinline__ f16x8 rowop(const _Float16* tile, int r0, int ks) const {
        return lds_row8(tile + row[ks] + r0 * D);
    }
    // A operand (transposed): columns 16 md .. +15 on m, the 32 rows r0 .. r0+31 on k
    // in the packed order 16 (j >> 2) + 4g + (j & 3)
    __device__ __forceinline__ f16x8 trop(const _Float16* tile, int r0, int md) const {
        return cat4(lds_tr4(tile + tr[md][0] + r0 * D), lds_tr4(tile + tr[md][1] + r0 * D));
    }
};

// LLVM scheduling strategies (__builtin_amdgcn_iglp_opt) for the unsplit dK/dV and dQ
// kernels' step bodies at D = 64; -1 = the default scheduler.  r03, in-process A/Bs
// (`profiles/r03/ab/iglp/`): strategy 0 on dK/dV -1.3 % at C3 in three runs (step -0.6 %,
// C5 and B2_H8_S4096 -0.5 %), +12 % slower at D = 32 (so D = 64 only); strategies 1-3
// and any strategy on dQ within +-0.8 %.
constexpr int kIglpDkdv = 0, kIglpDq = -1;
// ... and for the fused small-grid backward: strategy 2 took B2_H8_S512 15.8 -> 15.3 us
// (dO = ones) and 15.6 -> 15.1 (N(0,1)), S = 1024 fwd + bwd -1.5 %, B4_H8_S512, D = 32
// and S = 2048 +-0; strategy 1 lost 4 % at S = 512.  Per role: the dK/dV role needs it
// with split queries (S = 512: 16.0 us without), and with unsplit queries (4-8 blocks per
// CU) strategy 0 is better (B2_H8_S2048 64.4 -> 62.7 us); the dQ role +-1 % either way.
constexpr int kIglpFused = 2;
template <int D, int IGLP = -1, typename Mid>
__device__ __forceinline__ void dkdv_step16(DkdvState16<D>& st, const _Float16* Qs, const _Float16* dOs,
                                            const float* nlse2, const float* ndel, const FragOffsets16<D>& fo,
                                            int g, Mid&& mid) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        if (qb == 1) mid();
        if constexpr (IGLP >= 0) __builtin_amdgcn_iglp_opt(IGLP);  // LLVM scheduling strategy for the region
        f32x4 sa[2][2], da[2][2];  // [mb][nb]
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(nlse2 + qb * 32 + 16 * mb + 4 * g);
            const f32x4 dv = *reinterpret_cast<const f32x4*>(ndel + qb * 32 + 16 * mb + 4 * g);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                sa[mb][nb] = lv;
                da[mb][nb] = dv;
            }
        }
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks)
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                const f16x8 qa = fo.rowop(Qs, qb * 32 + 16 * mb, ks), doa = fo.rowop(dOs, qb * 32 + 16 * mb, ks);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    sa[mb][nb] = mfma16(qa, st.kf[nb][ks], sa[mb][nb]);
                    da[mb][nb] = mfma16(doa, st.vf[nb][ks], da[mb][nb]);
                }
            }
        f16x8 pf[2], dsf[2];  // [nb], k-slot j <-> query 16 (j >> 2) + 4g + (j & 3)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const float sv0 = sa[j >> 2][nb][j & 3], dv0 = da[j >> 2][nb][j & 3];
                const float sv1 = sa[j >> 2][nb][(j & 3) + 1], dv1 = da[j >> 2][nb][(j & 3) + 1];
                const float p0 = fast_exp2(sv0), p1 = fast_exp2(sv1);
                pf[nb][j] = to_tile(p0);
                pf[nb][j + 1] = to_tile(p1);
                const tile2 d2 = ds_pair(p0, p1, dv0, dv1, pf[nb][j], pf[nb][j + 1]);
                dsf[nb][j] = d2[0];
                dsf[nb][j + 1] = d2[1];
            }
#pragma unroll
        for (int md = 0; md < D / 16; ++md) {
            const f16x8 a_do = fo.trop(dOs, qb * 32, md), a_q = fo.trop(Qs, qb * 32, md);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                st.dva[md][nb] = mfma16(a_do, pf[nb], st.dva[md][nb]);
                st.dka[md][nb] = mfma16(a_q, dsf[nb], st.dka[md][nb]);
            }
        }
    }
}

// a wave's 32 keys x D results (16x16 accumulator layout) through its LDS stage,
// stored as whole 128-B row segments
template <int D>
__device__ __forceinline__ void store_block_rows16(float (*os)[36], const f32x4 (&acc)[D / 16][2], float scale,
                                                   float* __restrict__ dst, int rows_valid, int lane) {
    const int i16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int b = 0; b < D / 32; ++b) {
#pragma unroll
        for (int mh = 0; mh < 2; ++mh)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const f32x4 v = acc[2 * b + mh][nb] * scale;
                *reinterpret_cast<f32x4*>(&os[16 * nb + i16][16 * mh + 4 * g]) = v;
            }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int row = 8 * s4 + (lane >> 3), c4 = (lane & 7) * 4;
            const f32x4 v = *reinterpret_cast<const f32x4*>(&os[row][c4]);
            if (row < rows_valid) *reinterpret_cast<f32x4*>(dst + (long)row * D + 32 * b + c4) = v;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// KB x 32 keys per wave, NW waves: grid BH * ceil(S / (32*KB*NK)), block 64*NW.
// QS > 1 (small grids; 16x16x32 path): the query range is split over QS wave groups
// of NK = NW / QS waves.  Wave w keeps keys of slot w % NK and takes query tiles
// it·QS + w / NK; each step stages QS tiles.  After the loop the groups' dKᵀ / dVᵀ
// are summed in LDS in group order (deterministic) and group 0 stores.
// The workgroup's LDS: [buf][Q | dO][QS] fp16 tiles (or the query-split merge
// records), [buf][-lse2 | -delta][QS] fp32 rows, the per-wave result stage.  Carved
// from one block so the fused backward kernel can overlay it with the dQ role's.
template <int D, int NW, int KB, int QS>
struct DkdvLds {
    static constexpr int QT = 64, TILE = QT * D, NK = NW / QS;
    // query-split merge records: per wave of groups 1..QS-1, dKᵀ and dVᵀ (D floats per lane)
    static constexpr int MERGE = QS > 1 ? 2 * (QS - 1) * NK * D * 64 : 0;  // in halves
    // OVL: the prologue's K and V blocks side by side, loaded together with the first
    // Q/dO step (small grids, where the prologue's round trips are exposed; on the
    // unsplit C3 grid it measured -1.2 %)
    static constexpr bool OVL = QS > 1;
    static constexpr int KV = OVL ? 2 * 32 * KB * NK * D : 0;
    static constexpr int SMEM0 = 2 * 2 * QS * TILE > MERGE ? 2 * 2 * QS * TILE : MERGE;
    static constexpr int SMEM = KV > SMEM0 ? KV : SMEM0;  // halves
    static constexpr int ROWS = 2 * SMEM;                 // byte offsets
    static constexpr int OSTAGE = ROWS + 2 * 2 * QS * QT * 4;
    static constexpr int BYTES = OSTAGE + NK * 32 * 36 * 4;
};

// One workgroup of the dK/dV kernel; `bid` is its (XCD-remapped) block number over
// the BH * ceil(S / (KPW * NK)) key blocks.
// DEL: Δ = rowsum(dO ∘ O) of every staged step computed here from O rows staged
// beside dO (no Delta input: the fused small-grid launch, whose dQ role writes Δ).
template <int D, int NW, int KB = 1, bool M16 = false, int QS = 1, bool DEL = false, int IGLP = -1>
__device__ __forceinline__ void dkdv_body(char* __restrict__ lds, int bid, const float* __restrict__ Q,
                                          const float* __restrict__ K, const float* __restrict__ V,
                                          const float* __restrict__ dO, const float* __restrict__ LSE,
                                          const float* __restrict__ Delta, float* __restrict__ dK,
                                          float* __restrict__ dV, int S, const float* __restrict__ O = nullptr) {
    using L = DkdvLds<D, NW, KB, QS>;
    constexpr int QT = L::QT;  // query rows per step
    constexpr int NT = 64 * NW;
    constexpr int TILE = L::TILE;
    constexpr int KPW = 32 * KB;  // keys per wave
    static_assert(QS == 1 || (M16 && 2 * QS <= NW), "query split: 16x16x32, 2 QS row waves");
    constexpr int NK = L::NK;  // key waves (QS > 1: waves w, w + NK, ... share keys)
    _Float16* smem = reinterpret_cast<_Float16*>(lds);
    float(*rows)[2][QS * QT] = reinterpret_cast<float(*)[2][QS * QT]>(lds + L::ROWS);
    float(*ostage)[32][36] = reinterpret_cast<float(*)[32][36]>(lds + L::OSTAGE);  // per-wave result stage

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
    const int wave = QS > 1 ? (tid >> 6) % NK : tid >> 6;  // key slot of the wave
    const int qg = QS > 1 ? __builtin_amdgcn_readfirstlane((tid >> 6) / NK) : 0;  // query group
    const int nkb = (S + KPW * NK - 1) / (KPW * NK);
    const int bh = bid / nkb, kblk = bid - bh * nkb;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int key0 = kblk * KPW * NK + wave * KPW;  // this wave's first key
    const float kscale = FA2B_LOG2E / __builtin_sqrtf((float)D);

    DkdvState<D, KB> st;
    FragOffsets<D> fo;
    fo.init(lane);
    // 16x16x32 path (M16): its own state / offsets; the unused set is dead code
    static_assert(!M16 || KB == 1, "16x16x32 dK/dV: 32 keys per wave");
    DkdvState16<D> st16;
    FragOffsets16<D> fo16;
    const int g16 = lane >> 4;
    if constexpr (M16) fo16.init(lane);
    // Prologue.  L::OVL: the K and V blocks and the first Q/dO step are loaded in one
    // go (one HBM round trip instead of three), K and V side by side in the LDS block;
    // else K, then V, each through the Q/dO buffers.
    static_assert(KPW * NK <= 4 * QT, "K / V block fits the Q/dO buffers");
    const int kblock0 = kblk * KPW * NK;
    _Float16* const vblk = L::OVL ? smem + KPW * NK * D : smem;
    auto read_k = [&] {
        if constexpr (M16) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) st16.kf[nb][ks] = fo16.rowop(smem, wave * KPW + 16 * nb, ks);
        } else {
#pragma unroll
            for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                for (int t = 0; t < D / 16; ++t) st.kf[kb][t] = fo.rowop(smem, wave * KPW + kb * 32, t);
        }
    };
    auto read_v = [&] {
        if constexpr (M16) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) st16.vf[nb][ks] = fo16.rowop(vblk, wave * KPW + 16 * nb, ks);
        } else {
#pragma unroll
            for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                for (int t = 0; t < D / 16; ++t) st.vf[kb][t] = fo.rowop(vblk, wave * KPW + kb * 32, t);
        }
    };
    TileStager<D, KPW * NK, NT> kst, vst;
    kst.init(K + base, S, tid);
    vst.init(V + base, S, tid);
    kst.load(kblock0);
    if constexpr (!L::OVL) {
        kst.store(smem, kscale, tid);
        __syncthreads();
        read_k();
        __syncthreads();
    }
    vst.load(kblock0);
    if constexpr (!L::OVL) {
        vst.store(smem, 1.f, tid);
        __syncthreads();
        read_v();
        __syncthreads();
    }
    if constexpr (M16) {
#pragma unroll
        for (int md = 0; md < D / 16; ++md)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                st16.dka[md][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
                st16.dva[md][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
    } else {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    st.dka[kb][b][i] = 0.f;
                    st.dva[kb][b][i] = 0.f;
                }
    }

    // next-step staging by the first SW waves (FA2_DKDV_SW, above); DEL stages O too,
    // by every wave (at 8 waves x QS = 2 the 4-wave staging registers spilled ~290 VGPRs)
    constexpr int SW = DEL ? NW : FA2_DKDV_SW < NW ? FA2_DKDV_SW : NW;
    constexpr int NS = 64 * SW;
    const int wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool stg = wave_u < SW;
    TileStager<D, QT * QS, NS> qs, dos, os;
    qs.init(Q + base, S, tid);
    dos.init(dO + base, S, tid);
    if constexpr (DEL) os.init(O + base, S, tid);
    // Row constants of the staged step: wave 0 carries LSE, wave 1 carries Delta
    // (QT == 64 == one wave).  Loaded raw by a range-checked buffer load (rows >= S
    // read 0) and only scaled / negated / masked at store time, so nothing waits on
    // the load before the step's MFMAs (a guarded global load there made the
    // compiler drain vmcnt -- the K/V staging loads too -- at every step start).
    // (QS > 1: waves 0..QS-1 carry the LSE rows of the step's QS tiles, waves
    // QS..2QS-1 the Delta rows)
    static_assert(QT == 64, "one wave per row vector");
    const __amdgpu_buffer_rsrc_t rs_lse = head_rsrc(LSE + rbase, S, 1);
    const __amdgpu_buffer_rsrc_t rs_del = head_rsrc(Delta + rbase, S, 1);
    float rowraw = 0.f;
    int rowq = 0;
    const int rw = wave_u % QS;  // which of the step's tiles this wave's row vector is
    auto load_rows = [&](int q0) {
        q0 += rw * QT;
        rowq = q0 + lane;
        if (wave_u < QS) rowraw = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_lse, lane * 4, q0 * 4, 0));
        else if (!DEL && wave_u < 2 * QS)
            rowraw = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_del, lane * 4, q0 * 4, 0));
    };
    auto store_rows = [&](int buf) {
        // stored negated: they are the initial accumulators of S and dP
        if (wave_u < QS) rows[buf][0][rw * QT + lane] = rowq < S ? -rowraw * FA2B_LOG2E : -__builtin_inff();
        else if (!DEL && wave_u < 2 * QS) rows[buf][1][rw * QT + lane] = -rowraw;
    };
    // the next step's global loads go out between the step's two query blocks (issued
    // all at once right after the barrier they queue on the texture unit: r01)
    auto load_next = [&](int it) {
        if (stg) {
            qs.load(it * QS * QT);
            dos.load(it * QS * QT);
            if constexpr (DEL) os.load(it * QS * QT);
        }
        load_rows(it * QS * QT);
    };
    auto store_step = [&](_Float16* qdst, _Float16* ddst, int rbuf, int step) {
        if (stg) {
            qs.store(qdst, 1.f, tid);
            dos.store(ddst, 1.f, tid);
            if constexpr (DEL)
                delta_rows<D, QT * QS, NS, true>(dos, os, S, step * QS * QT, rows[rbuf][1], nullptr, tid);
        }
        store_rows(rbuf);
    };
    const int nqt = (S + QT - 1) / QT;  // query tiles
    const int nsteps = (nqt + QS - 1) / QS;
    if (stg) {
        qs.load(0);
        dos.load(0);
        if constexpr (DEL) os.load(0);
    }
    load_rows(0);
    if constexpr (L::OVL) {
        kst.store(smem, kscale, tid);
        vst.store(vblk, 1.f, tid);
        __syncthreads();
        read_k();
        read_v();
        __syncthreads();
    }
    store_step(smem, smem + QS * TILE, 0, 0);
    __syncthreads();
    // the group's tile within each staged image: folded into the per-lane offsets
    if (QS > 1) fo16.shift(qg * TILE);
    const int rq = qg * QT;  // the group's row constants

    // one staged step: the group's tile (the next step's loads inside it)
    auto run_step = [&](const _Float16* Qb, const _Float16* dOb, const float* r0, const float* r1, int itc,
                        auto&& mid) {
        if constexpr (M16) {
            const bool live = QS == 1 || itc * QS + qg < nqt;  // wave-uniform
            if (!live) mid();
            else dkdv_step16<D, IGLP>(st16, Qb, dOb, r0 + rq, r1 + rq, fo16, g16, mid);
        } else {
            dkdv_step<D, KB>(st, Qb, dOb, r0, r1, fo, h, mid);
        }
    };
    for (int it = 0; it < nsteps; it += 2) {
        {
            const bool more = it + 1 < nsteps;
            run_step(smem, smem + QS * TILE, rows[0][0], rows[0][1], it, [&] { if (more) load_next(it + 1); });
            if (more) store_step(smem + 2 * QS * TILE, smem + 3 * QS * TILE, 1, it + 1);
            __syncthreads();
        }
        if (it + 1 < nsteps) {
            const bool more = it + 2 < nsteps;
            run_step(smem + 2 * QS * TILE, smem + 3 * QS * TILE, rows[1][0], rows[1][1], it + 1,
                     [&] { if (more) load_next(it + 2); });
            if (more) store_step(smem, smem + QS * TILE, 0, it + 2);
            __syncthreads();
        }
    }

    if constexpr (QS > 1) {
        // query-split merge (the loop ended on a barrier: the tile buffers are free);
        // lane-linear records, summed in group order
        float* mg = reinterpret_cast<float*>(smem);
        if (qg > 0) {
            float* rec = mg + ((qg - 1) * NK + wave) * D * 64;
#pragma unroll
            for (int md = 0; md < D / 16; ++md)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        rec[((md * 2 + nb) * 4 + i) * 64 + lane] = st16.dka[md][nb][i];
                        rec[(D / 2 + (md * 2 + nb) * 4 + i) * 64 + lane] = st16.dva[md][nb][i];
                    }
        }
        __syncthreads();
        if (qg > 0) return;  // no workgroup barrier follows
#pragma unroll
        for (int g = 1; g < QS; ++g) {
            const float* rec = mg + ((g - 1) * NK + wave) * D * 64;
#pragma unroll
            for (int md = 0; md < D / 16; ++md)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        st16.dka[md][nb][i] += rec[((md * 2 + nb) * 4 + i) * 64 + lane];
                        st16.dva[md][nb][i] += rec[(D / 2 + (md * 2 + nb) * 4 + i) * 64 + lane];
                    }
        }
    }
    const float dscale = 1.f / __builtin_sqrtf((float)D);
    if constexpr (M16) {
        store_block_rows16<D>(ostage[wave], st16.dka, dscale, dK + base + (long)key0 * D, S - key0, lane);
        store_block_rows16<D>(ostage[wave], st16.dva, 1.f, dV + base + (long)key0 * D, S - key0, lane);
    } else {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int k0r = key0 + kb * 32;
            store_block_rows<D>(ostage[wave], st.dka[kb], dscale, dK + base + (long)k0r * D, S - k0r, lane);
            store_block_rows<D>(ostage[wave], st.dva[kb], 1.f, dV + base + (long)k0r * D, S - k0r, lane);
        }
    }
}

template <int D, int NW, int KB = 1, bool M16 = false, int QS = 1>
__global__ void __launch_bounds__(64 * NW)
fa2_bwd_dkdv_f16_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                        const float* __restrict__ dO, const float* __restrict__ LSE,
                        const float* __restrict__ Delta, float* __restrict__ dK, float* __restrict__ dV, int S) {
    __shared__ __attribute__((aligned(16))) char lds[DkdvLds<D, NW, KB, QS>::BYTES];
    // the unsplit instances (full grids: C3, C5, long S) under an LLVM scheduling strategy
    dkdv_body<D, NW, KB, M16, QS, false, QS == 1 && D == 64 ? kIglpDkdv : -1>(lds, xcd_remap(blockIdx.x, gridDim.x),
                                                                                 Q, K, V, dO, LSE, Delta, dK, dV, S);
}

// ---------------------------------------------------------------------------
// dQ:  grid BH * ceil(S / (32*NW)), block 64*NW
// ---------------------------------------------------------------------------
template <int D>
struct DqState {
    f16x8 qf[D / 16], df[D / 16];  // B operands: this lane's query row of Q (scaled) and dO
    f32x16 dqa[D / 32];
    f32x16 nlse2, ndel;            // loop-invariant initial accumulators: -lse2, -delta (per lane)
};

// One (32*NKB)-key tile: S^T = K Q^T and dP^T = V dO^T with the query on the lane,
// dS^T = P^T*(dP^T - Delta), dQ^T += K^T dS^T (K^T through ds_read_b64_tr_b16).
template <int D, bool MASK, int NKB, typename Mid>
__device__ __forceinline__ void dq_tile(DqState<D>& st, const _Float16* Ks, const _Float16* Vs,
                                        const FragOffsets<D>& fo, int k0, int S, int h, Mid&& mid) {
    f16x8 dsf[NKB][2];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        if (NKB > 1 && kb == 1) mid();  // between the two key blocks (the next tile's loads)
        // rows: key k0 + kb*32 + (i&3) + 8*(i>>2) + 4h ; col: query (lane)
        f32x16 sa = st.nlse2, da = st.ndel;
#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
            sa = mfma(fo.rowop(Ks, kb * 32, t), st.qf[t], sa);
            da = mfma(fo.rowop(Vs, kb * 32, t), st.df[t], da);
        }
        if (NKB == 1) mid();  // after the tile's S / dP MFMAs
        if (MASK) {  // ragged last tile only
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (k0 + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h >= S) sa[i] = -__builtin_inff();
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) dsf[kb][i >> 3][i & 7] = to_tile(fast_exp2(sa[i]) * da[i]);
    }
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int s = 0; s < 2; ++s) st.dqa[b] = mfma(fo.trop(Ks, kb * 32 + 16 * s, b), dsf[kb][s], st.dqa[b]);
}

// ---- dQ on v_mfma_f32_16x16x32, maps as in dkdv_step16:
//   S^T / dP^T (m = key, n = query, k = d): A = K / V rows of the tile (row reads),
//     B = Q / dO fragments in VGPRs; accumulators start at the lane's -lse2 / -delta.
//   dQ^T (m = d, n = query, k = key): B = dS^T packed k-slot j <-> key
//     16 (j >> 2) + 4g + (j & 3) of each 32-key half; A = K^T by transposed reads.
template <int D>
struct DqState16 {
    f16x8 qf[2][D / 32], df[2][D / 32];  // [nb][ks]: Q (scaled) / dO[query 16 nb + (l&15)][d 32 ks + 8g ..]
    f32x4 dqa[D / 16][2];                // [md][nb]
    f32x4 nlse2[2], ndel[2];             // [nb]: splats of the lane's -lse2 / -delta
};

template <int D, bool MASK, int NKB, int IGLP = -1, typename Mid>
__device__ __forceinline__ void dq_tile16(DqState16<D>& st, const _Float16* Ks, const _Float16* Vs,
                                          const FragOffsets16<D>& fo, int k0, int S, int g, Mid&& mid) {
    f16x8 dsf[NKB][2];  // [32-key half kb][nb]
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        if (NKB > 1 && kb == 1) mid();  // the next tile's loads between the two 32-key halves
        if constexpr (IGLP >= 0) __builtin_amdgcn_iglp_opt(IGLP);  // LLVM scheduling strategy for the region
        f32x4 sa[2][2], da[2][2];  // [mbl][nb]: keys k0 + 32 kb + 16 mbl + 4g + i
#pragma unroll
        for (int mbl = 0; mbl < 2; ++mbl)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                sa[mbl][nb] = st.nlse2[nb];
                da[mbl][nb] = st.ndel[nb];
            }
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks)
#pragma unroll
            for (int mbl = 0; mbl < 2; ++mbl) {
                const f16x8 ka = fo.rowop(Ks, 32 * kb + 16 * mbl, ks), va = fo.rowop(Vs, 32 * kb + 16 * mbl, ks);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    sa[mbl][nb] = mfma16(ka, st.qf[nb][ks], sa[mbl][nb]);
                    da[mbl][nb] = mfma16(va, st.df[nb][ks], da[mbl][nb]);
                }
            }
        if (MASK) {  // ragged last tile only
#pragma unroll
            for (int mbl = 0; mbl < 2; ++mbl)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (k0 + 32 * kb + 16 * mbl + 4 * g + i >= S) sa[mbl][nb][i] = -__builtin_inff();
        }
        if (NKB == 1) mid();  // 32-key tiles: after the tile's S / dP MFMAs
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                dsf[kb][nb][j] = to_tile(fast_exp2(sa[j >> 2][nb][j & 3]) * da[j >> 2][nb][j & 3]);
    }
#pragma unroll
    for (int md = 0; md < D / 16; ++md)
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const f16x8 a = fo.trop(Ks, 32 * kb, md);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) st.dqa[md][nb] = mfma16(a, dsf[kb][nb], st.dqa[md][nb]);
        }
}

// DELTA: Δ is computed here (from O, fused into the dO prologue) and written to
// `Delta` for the dK/dV kernel, which then runs after this one.
// NKB 32-key blocks per K/V tile (1 for D = 128 at 8 waves: fewer registers).
// KS > 1 (small grids; 16x16x32 path): the key range is split over KS wave groups of
// NQ = NW / KS waves.  Wave w keeps query rows of slot w % NQ and takes K/V tiles
// j·KS + w / NQ; each step stages KS tiles.  After the loop the groups' dQᵀ are
// summed in LDS in group order (deterministic) and group 0 stores.
// The workgroup's LDS: [buf][K | V][KS] tiles (at least one Q block for the coalesced
// prologue, and the key-split merge records), the per-wave dQ stage, the block's Δ.
template <int D, int NW, bool DELTA, int NKB, int KS>
struct DqLds {
    static constexpr int KT = 32 * NKB, TILE = KT * D, NQ = NW / KS;
    // key-split merge records: per wave of groups 1..KS-1, dQᵀ (D / 2 floats per lane)
    static constexpr int MERGE = KS > 1 ? 2 * (KS - 1) * NQ * (D / 2) * 64 : 0;  // in halves
    // OVL: the prologue's Q and dO blocks behind the first K/V buffer, loaded together
    // with the first K/V step (small grids and D = 128, where the prologue's round
    // trips are exposed; on the unsplit C3 grid it measured -1.7 %)
    static constexpr bool OVL = KS > 1 || D == 128;
    static constexpr int QD = OVL ? 2 * KS * TILE + 2 * 32 * NQ * D : 32 * NQ * D;
    static constexpr int RING = 4 * KS * TILE;
    static constexpr int SMEM0 = RING > QD ? RING : QD;
    static constexpr int SMEM = SMEM0 > MERGE ? SMEM0 : MERGE;  // halves
    static constexpr int OSTAGE = 2 * SMEM;                     // byte offsets
    static constexpr int DBLK = OSTAGE + NQ * 32 * 36 * 4;
    static constexpr int BYTES = DBLK + (DELTA ? 32 * NQ : 1) * 4;
};

// One workgroup of the dQ kernel; `bid` is its (XCD-remapped) block number over the
// BH * ceil(S / (32 * NQ)) query blocks.
template <int D, int NW, bool DELTA = false, int NKB = 2, bool M16 = false, int KS = 1, int IGLP = -1>
__device__ __forceinline__ void dq_body(char* __restrict__ lds, int bid, const float* __restrict__ Q,
                                        const float* __restrict__ K, const float* __restrict__ V,
                                        const float* __restrict__ dO, const float* __restrict__ LSE,
                                        float* __restrict__ Delta, float* __restrict__ dQ, int S,
                                        const float* __restrict__ O) {
    using L = DqLds<D, NW, DELTA, NKB, KS>;
    constexpr int V0 = KS * L::TILE;  // first V buffer
    constexpr int KT = L::KT;
    constexpr int NT = 64 * NW;
    constexpr int TILE = L::TILE;
    static_assert(KS == 1 || (M16 && NW % KS == 0), "key split: 16x16x32");
    constexpr int NQ = L::NQ;  // query waves (KS > 1: waves w, w + NQ, ... share rows)
    _Float16* smem = reinterpret_cast<_Float16*>(lds);
    float(*ostage)[32][36] = reinterpret_cast<float(*)[32][36]>(lds + L::OSTAGE);  // per-wave dQ stage
    float* delta_blk = reinterpret_cast<float*>(lds + L::DBLK);

    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = KS > 1 ? (tid >> 6) % NQ : tid >> 6;  // query slot of the wave
    const int kg = KS > 1 ? __builtin_amdgcn_readfirstlane((tid >> 6) / NQ) : 0;  // key group
    const int nqb = (S + 32 * NQ - 1) / (32 * NQ);
    const int bh = bid / nqb, qb = bid - bh * nqb;
    const long base = (long)bh * S * D;
    const int q = qb * 32 * NQ + wave * 32 + r;
    const bool qvalid = q < S;
    const float qscale = FA2B_LOG2E / __builtin_sqrtf((float)D);

    DqState<D> st;
    FragOffsets<D> fo;
    fo.init(lane);
    DqState16<D> st16;
    FragOffsets16<D> fo16;
    const int g16 = lane >> 4, i16 = lane & 15;
    if constexpr (M16) fo16.init(lane);
    constexpr int SW = NW;  // K/V staging by every wave (by waves 0-3 only: no gain, r01)
    TileStager<D, KT * KS, 64 * SW> ks, vs;
    ks.init(K + base, S, tid);
    vs.init(V + base, S, tid);
    // Staging flag compile-time true at D = 128 (all waves stage): the runtime flag's
    // branches around the loads left 34 v_mov_b64 of staging-register copies there (dQ
    // +11.8 % without).  At D <= 64 the runtime flag stays: with it gone the compiler
    // schedules the mid-tile loads differently and dQ ran 4.5 % slower at C3.
    ks.on = vs.on = (SW == NW && D > 64) || __builtin_amdgcn_readfirstlane(tid >> 6) < SW;
    const int ntiles = (S + KT - 1) / KT;
    const int last_ragged = (S % KT) ? ntiles - 1 : -1;  // the one tile that needs key masking
    const int nsteps = (ntiles + KS - 1) / KS;
    // Prologue.  L::OVL: the Q and dO blocks (and O for Δ) and the first K/V step are
    // loaded in one go (one HBM round trip instead of three), Q and dO in the second
    // K/V buffer, which the first loop step restages only after the barrier below;
    // else Q, then dO, then the first K/V step, each a round trip.
    constexpr bool OVL = L::OVL;
    _Float16* const qblk = OVL ? smem + 2 * KS * TILE : smem;
    _Float16* const dblk = OVL ? qblk + 32 * NQ * D : smem;
    auto read_q = [&] {
        if constexpr (M16) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) st16.qf[nb][ks] = fo16.rowop(qblk, wave * 32 + 16 * nb, ks);
        } else {
#pragma unroll
            for (int t = 0; t < D / 16; ++t) st.qf[t] = fo.rowop(qblk, wave * 32, t);
        }
    };
    auto read_d = [&] {
        if constexpr (M16) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int ks = 0; ks < D / 32; ++ks) st16.df[nb][ks] = fo16.rowop(dblk, wave * 32 + 16 * nb, ks);
        } else {
#pragma unroll
            for (int t = 0; t < D / 16; ++t) st.df[t] = fo.rowop(dblk, wave * 32, t);
        }
    };
    {
        using TS = TileStager<D, 32 * NQ, NT>;
        TS qst, dst, ost;
        qst.init(Q + base, S, tid);
        dst.init(dO + base, S, tid);
        qst.load(qb * 32 * NQ);
        if constexpr (!OVL) {
            qst.store(qblk, qscale, tid);
            __syncthreads();
            read_q();
            __syncthreads();
        }
        dst.load(qb * 32 * NQ);
        if (DELTA) {
            ost.init(O + base, S, tid);
            ost.load(qb * 32 * NQ);
        }
        if constexpr (OVL) {
            ks.load(0);
            vs.load(0);
            qst.store(qblk, qscale, tid);
        }
        dst.store(dblk, 1.f, tid);
        if (DELTA) delta_rows<D, 32 * NQ, NT>(dst, ost, S, qb * 32 * NQ, delta_blk, Delta + (long)bh * S, tid);
        if constexpr (OVL) {
            ks.store(smem, 1.f, tid);
            vs.store(smem + V0, 1.f, tid);
        }
        __syncthreads();
        if constexpr (OVL) read_q();
        read_d();
        if constexpr (!OVL) __syncthreads();
    }
    {
        const float nl = qvalid ? -LSE[(long)bh * S + q] * FA2B_LOG2E : -__builtin_inff();
        const float nd = !qvalid ? 0.f : DELTA ? -delta_blk[wave * 32 + r] : -Delta[(long)bh * S + q];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            st.nlse2[i] = nl;
            st.ndel[i] = nd;
        }
    }
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) st.dqa[b][i] = 0.f;
    if constexpr (M16) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int qn = qb * 32 * NQ + wave * 32 + 16 * nb + i16;
            const bool ok = qn < S;
            const float nl = ok ? -LSE[(long)bh * S + qn] * FA2B_LOG2E : -__builtin_inff();
            const float nd = !ok ? 0.f : DELTA ? -delta_blk[wave * 32 + 16 * nb + i16] : -Delta[(long)bh * S + qn];
            st16.nlse2[nb] = f32x4{nl, nl, nl, nl};
            st16.ndel[nb] = f32x4{nd, nd, nd, nd};
        }
#pragma unroll
        for (int md = 0; md < D / 16; ++md)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) st16.dqa[md][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (NW == 8 && __builtin_amdgcn_readfirstlane(tid >> 6) >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (!L::OVL) {
        ks.load(0);
        vs.load(0);
        ks.store(smem, 1.f, tid);
        vs.store(smem + V0, 1.f, tid);
    }
    __syncthreads();
    // the group's tile within each staged image: folded into the per-lane offsets
    if (KS > 1) fo16.shift(kg * TILE);

    for (int j = 0; j < nsteps; j += 2) {
        {
            const bool more = j + 1 < nsteps;
            const int jj = j * KS + kg;             // this wave's tile
            const bool live = KS == 1 || jj < ntiles;  // wave-uniform
            auto ld = [&] {
                ks.load((j + 1) * KS * KT);
                vs.load((j + 1) * KS * KT);
            };
            auto mid = [&] { ld(); };  // also on the last step (see FA2_DKDV_SW's note)
            if constexpr (M16) {
                if (!live) mid();
                else if (jj == last_ragged)
                    dq_tile16<D, true, NKB, IGLP>(st16, smem, smem + KS * TILE, fo16, jj * KT, S, g16, mid);
                else dq_tile16<D, false, NKB, IGLP>(st16, smem, smem + KS * TILE, fo16, jj * KT, S, g16, mid);
            } else {
                if (j == last_ragged) dq_tile<D, true, NKB>(st, smem, smem + TILE, fo, j * KT, S, h, mid);
                else dq_tile<D, false, NKB>(st, smem, smem + TILE, fo, j * KT, S, h, mid);
            }
            if (more) {
                ks.store(smem + 2 * KS * TILE, 1.f, tid);
                vs.store(smem + 3 * KS * TILE, 1.f, tid);
            }
            __syncthreads();
        }
        if (j + 1 < nsteps) {
            const bool more = j + 2 < nsteps;
            const int jj = (j + 1) * KS + kg;
            const bool live = KS == 1 || jj < ntiles;
            auto ld = [&] {
                ks.load((j + 2) * KS * KT);
                vs.load((j + 2) * KS * KT);
            };
            auto mid = [&] { ld(); };  // also on the last step (see FA2_DKDV_SW's note)
            if constexpr (M16) {
                if (!live) mid();
                else if (jj == last_ragged)
                    dq_tile16<D, true, NKB, IGLP>(st16, smem + 2 * KS * TILE, smem + 3 * KS * TILE, fo16, jj * KT, S, g16,
                                                  mid);
                else dq_tile16<D, false, NKB, IGLP>(st16, smem + 2 * KS * TILE, smem + 3 * KS * TILE, fo16, jj * KT, S,
                                                    g16, mid);
            } else {
                if (j + 1 == last_ragged)
                    dq_tile<D, true, NKB>(st, smem + 2 * TILE, smem + 3 * TILE, fo, (j + 1) * KT, S, h, mid);
                else dq_tile<D, false, NKB>(st, smem + 2 * TILE, smem + 3 * TILE, fo, (j + 1) * KT, S, h, mid);
            }
            if (more) {
                ks.store(smem, 1.f, tid);
                vs.store(smem + KS * TILE, 1.f, tid);
            }
            __syncthreads();
        }
    }

    if constexpr (KS > 1) {
        // key-split merge (the loop ended on a barrier: the tile buffers are free);
        // lane-linear records, summed in group order
        float* mg = reinterpret_cast<float*>(smem);
        if (kg > 0) {
            float* rec = mg + ((kg - 1) * NQ + wave) * (D / 2) * 64;
#pragma unroll
            for (int md = 0; md < D / 16; ++md)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) rec[((md * 2 + nb) * 4 + i) * 64 + lane] = st16.dqa[md][nb][i];
        }
        __syncthreads();
        if (kg > 0) return;  // no workgroup barrier follows
#pragma unroll
        for (int g = 1; g < KS; ++g) {
            const float* rec = mg + ((g - 1) * NQ + wave) * (D / 2) * 64;
#pragma unroll
            for (int md = 0; md < D / 16; ++md)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) st16.dqa[md][nb][i] += rec[((md * 2 + nb) * 4 + i) * 64 + lane];
        }
    }
    {
        const int q0w = qb * 32 * NQ + wave * 32;
        if constexpr (M16)
            store_block_rows16<D>(ostage[wave], st16.dqa, 1.f / __builtin_sqrtf((float)D), dQ + base + (long)q0w * D,
                                  S - q0w, lane);
        else
            store_block_rows<D>(ostage[wave], st.dqa, 1.f / __builtin_sqrtf((float)D), dQ + base + (long)q0w * D,
                                S - q0w, lane);
    }
}

#ifndef CUPY_INLINE_COMPILE
// ---------------------------------------------------------------------------
// Hand-scheduled dQ (D = 64; S % 64 == 0, S >= 128), r05.
// ---------------------------------------------------------------------------
// One workgroup = 4 waves = 256 query rows, one wave per SIMD; each wave keeps 64 query
// rows as two 32-row chains of two 16-row blocks on the lane (Q, dO fragments and dQᵀ
// accumulators in AGPRs; every product on v_mfma_f32_16x16x32) and streams
// the head's 64-key K/V tiles through LDS.  Per tile four MFMA phases alternate the
// chains: Sᵀ and dPᵀ of one chain while the other chain's dS is formed in the MFMA gaps,
// then that chain's dQᵀ += Kᵀ dSᵀ.  The tile loop is the generated inline-asm block of
// fa2_bwd_dq_hs.inc (gen/gen_bwd_dq.py); this kernel stages the Q and dO blocks, computes
// Δ = rowsum(dO ∘ O) from the staged rows (O given: written out for the dK/dV kernel) or
// reads it, hands the asm the lane-constant seeds -LSE·log2e and -Δ, and stores the dQ
// rows it leaves (unscaled fp32) in an LDS stage.  Every dQ element is summed in one fixed
// order: bitwise reproducible, no atomics (the reference: f-attn2-backward_f16.cu:240-301).
}  // namespace fa2f16b
#include "fa2_bwd_dq_hs.inc"
namespace fa2f16b {

template <int D>
__global__ void __launch_bounds__(256, 1)
fa2_bwd_dq_hs_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                     const float* __restrict__ dO, const float* __restrict__ LSE, float* __restrict__ Delta,
                     float* __restrict__ dQ, int S, const float* __restrict__ O, int P, float* __restrict__ part) {
    static_assert(D == 64, "hand-scheduled dQ: D = 64");
    constexpr int KT = 64, TB = KT * D, OST = D + 4;
    __shared__ __attribute__((aligned(16))) _Float16 smem[FA2_DQ_LDS_D64 / 2];
    __shared__ float rowc[2][256];  // -LSE*log2e and Δ of the block's rows

    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nqb = (S + 255) / 256;
    // workgroup -> (head, key chunk, query block); P = 1: the whole key range.  P > 1
    // (the split backward): keys [kc L, kc L + L), the dQ part goes to
    // part + ((kc BH + bh) S + row) D and chunk 0 writes Δ
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = bid % nqb, bc = bid / nqb;
    const int bh = bc / P, kc = bc - bh * P;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int qrow0 = qb * 256;
    const int L = S / P;
    const long kbase = base + (long)kc * L * D;
    float* dst_rows = P > 1 ? part + ((long)kc * (gridDim.x / (P * nqb)) + bh) * S * D : dQ + base;

    // Q block (scaled by log2(e)/sqrt(D)) -> LDS [4TB, 8TB) halves; dO block -> [8TB, 12TB)
    {
        TileStager<D, 256, 256> qst;
        qst.init(Q + base, S, tid);
        qst.load(qrow0);
        qst.store(smem + 4 * TB, FA2B_LOG2E / __builtin_sqrtf((float)D), tid);
    }
    {
        TileStager<D, 256, 256> dst;
        dst.init(dO + base, S, tid);
        dst.load(qrow0);
        if (O) {
            TileStager<D, 256, 256> ost;
            ost.init(O + base, S, tid);
            ost.load(qrow0);
            delta_rows<D, 256, 256>(dst, ost, S, qrow0, rowc[1], kc == 0 ? Delta + rbase : nullptr, tid);
        }
        dst.store(smem + 8 * TB, 1.f, tid);
    }
    {
        const int q = qrow0 + tid;
        rowc[0][tid] = q < S ? -LSE[rbase + q] * FA2B_LOG2E : -__builtin_inff();
        if (!O) rowc[1][tid] = q < S ? Delta[rbase + q] : 0.f;
    }
    TileStager<D, KT, 256> ks, vs;
    ks.init(K + kbase, L, tid);
    vs.init(V + kbase, L, tid);
    ks.load(0);
    vs.load(0);
    ks.store(smem, 1.f, tid);
    vs.store(smem + 2 * TB, 1.f, tid);
    __syncthreads();

    // per-lane LDS byte offsets of the row and transposed fragment reads (16x16x32 maps)
    FragOffsets16<D> fo;
    fo.init(lane);
    int hs_ka[D / 32], hs_kt[D / 16][2], hs_vo[D / 32];
#pragma unroll
    for (int t = 0; t < D / 32; ++t) hs_ka[t] = fo.row[t] * 2;
#pragma unroll
    for (int b = 0; b < D / 16; ++b) {
        hs_kt[b][0] = fo.tr[b][0] * 2;
        hs_kt[b][1] = fo.tr[b][1] * 2;
    }
#pragma unroll
    for (int c = 0; c < D / 32; ++c) hs_vo[c] = ks.voff[c];
    const int hs_lo = ks.loff[0] * 2;
    // the dQ stage address (row l & 15 of each 16-row block, columns 4 (l >> 4) ..) and the
    // lane-constant seeds -LSE·log2e, -Δ of the lane's row in each 16-row block
    const int g16 = lane >> 4, i16 = lane & 15;
    const int hs_sa = ((wave * 64 + r) * OST + 4 * h) * 4;  // (row l & 31, columns 4 (l >> 5): 'stamps' builds)
    const int hs_oa = ((wave * 64 + i16) * OST + 4 * g16) * 4;
    (void)hs_sa;
    float hs_nl[4], hs_nd[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int row = wave * 64 + 16 * c + i16;
        hs_nl[c] = rowc[0][row];
        hs_nd[c] = -rowc[1][row];
    }
    const __amdgpu_buffer_rsrc_t hs_rsk = ks.rs, hs_rsv = vs.rs;
    const int hs_qb = __builtin_amdgcn_readfirstlane(4 * TB * 2 + wave * 64 * D * 2);
    const int hs_db = __builtin_amdgcn_readfirstlane(8 * TB * 2 + wave * 64 * D * 2);
    int hs_cnt = __builtin_amdgcn_readfirstlane(L / KT - 1);
    int hs_goff = __builtin_amdgcn_readfirstlane(KT * D * 4);
#ifdef FA2_TILE_BF16
    asm volatile(FA2_DQ_ASM_D64_BF16 : FA2_DQ_OUTPUTS_D64 : FA2_DQ_INPUTS_D64 : FA2_DQ_CLOBBERS_D64);
#else
    asm volatile(FA2_DQ_ASM_D64_F16 : FA2_DQ_OUTPUTS_D64 : FA2_DQ_INPUTS_D64 : FA2_DQ_CLOBBERS_D64);
#endif
    // dQ rows [wave*64 + c*32 + q][OST] (unscaled) -> HBM as whole rows, times 1/sqrt(D)
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    const float dscale = 1.f / __builtin_sqrtf((float)D);
    const float* os = reinterpret_cast<const float*>(smem);
#pragma unroll 4
    for (int rr = 0; rr < 64; rr += RPI) {
        const int row = wave * 64 + rr + lane / LPR, c4 = (lane % LPR) * 4;
        const f32x4 v = *reinterpret_cast<const f32x4*>(os + row * OST + c4) * dscale;
        if (qrow0 + row < S) *reinterpret_cast<f32x4*>(dst_rows + (long)(qrow0 + row) * D + c4) = v;
    }
}
// ---------------------------------------------------------------------------
// Hand-scheduled dK/dV (D = 64; S % 64 == 0, S >= 128), r05.
// ---------------------------------------------------------------------------
// One workgroup = 4 waves = 256 keys, one wave per SIMD; each wave keeps 64 keys as two
// 32-key chains (K, V fragments and dKᵀ / dVᵀ accumulators in AGPRs) while the head's
// queries stream in 64-row steps (Q, dO tiles and the -LSE·log2e / -Δ rows) through a
// 3-slot LDS ring.  Per step four MFMA phases alternate the chains: S and dP of one chain
// while the other chain's P and dS are formed in the MFMA gaps, then that chain's
// dVᵀ += dOᵀ P and dKᵀ += Qᵀ dS.  The loop is the generated inline-asm block of
// fa2_bwd_dkdv_hs.inc (gen/gen_bwd_dkdv.py).  This kernel stages the K block (scaled by
// log2(e)/sqrt(D)) and the V block for the asm's fragment reads, the first step's tiles
// and row constants, and hands every wave the same staging code: wave 0 loads the next
// step's LSE row, wave 1 its Δ row, waves 2 and 3 a null descriptor into a sink.  dK and
// dV leave through an LDS stage as whole rows (dK times 1/sqrt(D)); every element is
// summed in one fixed order (the reference: f-attn2-backward_f16.cu:170-268).
}  // namespace fa2f16b
#include "fa2_bwd_dkdv_hs.inc"
namespace fa2f16b {

template <int D>
__global__ void __launch_bounds__(256, 1)
fa2_bwd_dkdv_hs_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                       const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ Delta,
                       float* __restrict__ dK, float* __restrict__ dV, int S, int P, float* __restrict__ part) {
    static_assert(D == 64, "hand-scheduled dK/dV: D = 64");
    constexpr int TB = 64 * D, OST = D + 4;
    constexpr int SLOT = FA2_DK_SLOT_D64, RC = FA2_DK_RC_D64, KVB = FA2_DK_KVB_D64;
    __shared__ __attribute__((aligned(16))) char lds[FA2_DK_LDS_D64];
    _Float16* sh = reinterpret_cast<_Float16*>(lds);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nkb = (S + 255) / 256;
    // workgroup -> (head, query chunk, key block); P = 1: every query.  P > 1 (the split
    // backward): queries [qc L, qc L + L), the dK / dV parts go to
    // part + ((qc BH + bh) S + row) D and part + (P BH + qc BH + bh) S D + row D
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = bid % nkb, bc = bid / nkb;
    const int bh = bc / P, qc = bc - bh * P;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int krow0 = kblk * 256;
    const int L = S / P, q0 = qc * L;
    const long BH = gridDim.x / (P * nkb);
    float* dk_rows = P > 1 ? part + ((long)qc * BH + bh) * S * D : dK + base;
    float* dv_rows = P > 1 ? part + ((long)P * BH + (long)qc * BH + bh) * S * D : dV + base;

    // K block (scaled) and V block -> LDS [KVB, KVB + 2 * 256 * D * 2) bytes
    {
        TileStager<D, 256, 256> kst;
        kst.init(K + base, S, tid);
        kst.load(krow0);
        kst.store(sh + KVB / 2, FA2B_LOG2E / __builtin_sqrtf((float)D), tid);
    }
    {
        TileStager<D, 256, 256> vst;
        vst.init(V + base, S, tid);
        vst.load(krow0);
        vst.store(sh + KVB / 2 + 256 * D, 1.f, tid);
    }
    // step 0: Q, dO tiles and the row constants -> slot 0
    TileStager<D, 64, 256> qs, ds;
    qs.init(Q + base + (long)q0 * D, L, tid);
    ds.init(dO + base + (long)q0 * D, L, tid);
    qs.load(0);
    ds.load(0);
    qs.store(sh, 1.f, tid);
    ds.store(sh + TB, 1.f, tid);
    if (tid < 64) {
        float* rc = reinterpret_cast<float*>(lds + RC);
        rc[tid] = tid < L ? -LSE[rbase + q0 + tid] * FA2B_LOG2E : 0.f;
        rc[64 + tid] = tid < L ? -Delta[rbase + q0 + tid] : 0.f;
    }
    __syncthreads();

    // per-lane LDS byte offsets of the row and transposed fragment reads (16x16x32 maps)
    FragOffsets16<D> fo;
    fo.init(lane);
    int hs_ka[D / 32], hs_tr[D / 16][2], hs_vo[D / 32];
#pragma unroll
    for (int t = 0; t < D / 32; ++t) hs_ka[t] = fo.row[t] * 2;
#pragma unroll
    for (int b = 0; b < D / 16; ++b) {
        hs_tr[b][0] = fo.tr[b][0] * 2;
        hs_tr[b][1] = fo.tr[b][1] * 2;
    }
#pragma unroll
    for (int c = 0; c < D / 32; ++c) hs_vo[c] = qs.voff[c];
    const int hs_lo = qs.loff[0] * 2;
    // row-constant tuples: rows 4g .. 4g + 3 of each 16-row block; the dK/dV stage: row
    // l & 15 of each 16-key block, columns 4g ..
    const int g16 = lane >> 4, i16 = lane & 15;
    const int hs_rco = 16 * g16, hs_rvo = 4 * lane;
    const int hs_rcw = (wave < 2 ? 256 * wave : 512) + 4 * lane;
    const int hs_oak = ((wave * 64 + i16) * OST + 4 * g16) * 4, hs_oav = hs_oak + 256 * OST * 4;
    const __amdgpu_buffer_rsrc_t hs_rsq = qs.rs, hs_rsd = ds.rs;
    // the row-constant stream of this wave: LSE (wave 0), Δ (wave 1), nothing (num_records 0)
    const __amdgpu_buffer_rsrc_t hs_rsc =
        head_rsrc(wave == 1 ? Delta + rbase + q0 : LSE + rbase + q0, wave < 2 ? L : 0, 1);
    const float hs_rsm = __builtin_bit_cast(
        float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, wave == 0 ? -FA2B_LOG2E : wave == 1 ? -1.f : 0.f)));
    const int hs_kvb = __builtin_amdgcn_readfirstlane(KVB + wave * 64 * D * 2);
    int hs_cnt = __builtin_amdgcn_readfirstlane(L / 64 - 1);
    int hs_goff = __builtin_amdgcn_readfirstlane(64 * D * 4);
    int hs_roff = __builtin_amdgcn_readfirstlane(64 * 4);
    (void)SLOT;
#ifdef FA2_TILE_BF16
    asm volatile(FA2_DK_ASM_D64_BF16 : FA2_DK_OUTPUTS_D64 : FA2_DK_INPUTS_D64 : FA2_DK_CLOBBERS_D64);
#else
    asm volatile(FA2_DK_ASM_D64_F16 : FA2_DK_OUTPUTS_D64 : FA2_DK_INPUTS_D64 : FA2_DK_CLOBBERS_D64);
#endif
    // dK rows (stage at 0) and dV rows (stage at 256 * OST floats) -> HBM as whole rows
    constexpr int LPR = D / 4, RPI = 64 / LPR;
    const float dscale = 1.f / __builtin_sqrtf((float)D);
    const float* os = reinterpret_cast<const float*>(lds);
#pragma unroll 4
    for (int rr = 0; rr < 64; rr += RPI) {
        const int row = wave * 64 + rr + lane / LPR, c4 = (lane % LPR) * 4;
        const f32x4 vk = *reinterpret_cast<const f32x4*>(os + row * OST + c4) * dscale;
        const f32x4 vv = *reinterpret_cast<const f32x4*>(os + (256 + row) * OST + c4);
        if (krow0 + row < S) {
            *reinterpret_cast<f32x4*>(dk_rows + (long)(krow0 + row) * D + c4) = vk;
            *reinterpret_cast<f32x4*>(dv_rows + (long)(krow0 + row) * D + c4) = vv;
        }
    }
}

// The split backward's reduce: out[t] = sum over the P chunk parts of tensor t (dQ, dK,
// dV; blockIdx.y), in chunk order -- deterministic.  n floats per tensor, 4 per thread.
__global__ void __launch_bounds__(256)
fa2_bwd_split_reduce_kernel(const float* __restrict__ part, int P, long n, float* __restrict__ dq,
                            float* __restrict__ dk, float* __restrict__ dv) {
    const long x = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (x >= n) return;
    const int t = blockIdx.y;
    const float* src = part + (long)t * P * n + x;
    f32x4 acc = *reinterpret_cast<const f32x4*>(src);
    for (int c = 1; c < P; ++c) acc += *reinterpret_cast<const f32x4*>(src + c * n);
    float* out = t == 0 ? dq : t == 1 ? dk : dv;
    *reinterpret_cast<f32x4*>(out + x) = acc;
}
#endif  // CUPY_INLINE_COMPILE

template <int D, int NW, bool DELTA = false, int NKB = 2, bool M16 = false, int KS = 1>
__global__ void __launch_bounds__(64 * NW)
fa2_bwd_dq_f16_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                      const float* __restrict__ dO, const float* __restrict__ LSE, float* __restrict__ Delta,
                      float* __restrict__ dQ, int S, const float* __restrict__ O) {
    __shared__ __attribute__((aligned(16))) char lds[DqLds<D, NW, DELTA, NKB, KS>::BYTES];
    dq_body<D, NW, DELTA, NKB, M16, KS, KS == 1 && D == 64 ? kIglpDq : -1>(
        lds, xcd_remap(blockIdx.x, gridDim.x), Q, K, V, dO, LSE, Delta, dQ, S, O);
}

// dK/dV and dQ in ONE launch (small grids).  Workgroups [0, ndk) take the dK/dV role
// (QS query groups), [ndk, gridDim.x) the dQ role (KS key groups); the two roles
// share nothing, so they run side by side on the chip instead of one kernel after
// the other, and the second launch's ramp-up and tail go away.  Δ comes from a
// prior fa2_delta_kernel (the dQ role cannot hand its fused Δ to the dK/dV role
// without a cross-workgroup wait).  Both roles run NW waves on the 16x16x32 path;
// the LDS block is the larger of the two layouts, registers the larger of the two.
//   DEL (O given): no Δ input at all.  Each role computes Δ = rowsum(dO ∘ O) from O rows
// staged beside the dO rows it stages anyway -- the dQ role in its prologue (and it
// writes Δ out), the dK/dV role per step -- so the launch depends on nothing but the
// forward's outputs: the separate Δ kernel and its launch boundary go away, at the
// price of the dK/dV role's O reads (these grids are latency-bound, not HBM-bound).
template <int D, int NW, int QS, int KS, int NKB, bool DEL = false>
__global__ void __launch_bounds__(64 * NW)
fa2_bwd_fused_f16_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                         const float* __restrict__ dO, const float* __restrict__ LSE, float* __restrict__ Delta,
                         float* __restrict__ dQ, float* __restrict__ dK, float* __restrict__ dV, int S, int ndk,
                         const float* __restrict__ O) {
    constexpr int B1 = DkdvLds<D, NW, 1, QS>::BYTES, B2 = DqLds<D, NW, DEL, NKB, KS>::BYTES;
    __shared__ __attribute__((aligned(16))) char lds[B1 > B2 ? B1 : B2];
    const int b = blockIdx.x;
    if (b < ndk)
        // the dK/dV role with unsplit queries takes the standalone kernel's strategy
        dkdv_body<D, NW, 1, true, QS, DEL, QS == 1 && D == 64 ? kIglpDkdv : kIglpFused>(
            lds, xcd_remap(b, ndk), Q, K, V, dO, LSE, Delta, dK, dV, S, O);
    else
        dq_body<D, NW, DEL, NKB, true, KS, kIglpFused>(lds, xcd_remap(b - ndk, gridDim.x - ndk), Q, K, V, dO, LSE,
                                                           Delta, dQ, S, O);
}

// ---- CuPy face: the reference harness's launch geometry (grid B*H*ceil(S/32),
// block 256, test_flash_attention2.py:499-535 / f-attn2-backward_f16.cu:445),
// fp16 tiles on MFMA.  The reference adds dQ with float atomics from every key block
// (f-attn2-backward_f16.cu:289); here each workgroup i runs two roles in turn, as the
// exact-fp32 face does (f-attn2-backward.cu), and no atomic is issued:
//   1. dK/dV for key block i: 32 keys (B operands K*log2e/sqrt(D) and V in registers);
//      the head's 32-row query tiles are dealt to the 4 waves round-robin; per tile a
//      wave stages Q into its private buffer (S = Q K^T), then dO (dP = dO V^T,
//      dV^T += dO^T P), then Q again (dK^T += Q^T dS); the waves' dK / dV partials are
//      summed in a fixed order through one LDS buffer;
//   2. dQ for query block i: 32 queries (B operands Q*log2e/sqrt(D) and dO in
//      registers, -LSE*log2e and -Delta as lane constants); the head's 32-key tiles
//      are dealt to the waves round-robin; per tile a wave stages K (S^T = K Q^T), V
//      (dP^T = V dO^T), then K again (dQ^T += K^T dS^T, the packed dS^T accumulator as
//      the B operand); the waves' dQ^T partials are summed in wave order and dQ is
//      written once.
// Every output element is therefore written once, in a fixed order: the face is
// bitwise repeatable, and the harness's zero-filled dQ is simply overwritten.
struct CompatLds {
    static constexpr int DMAX = 128;
    static constexpr int BUF = 4 * 32 * DMAX;  // per-wave [32][D] tiles; the [32][D] f32 merge buffer
    static constexpr int HALVES = BUF;
};

template <int D>
__device__ __forceinline__ void bwd_compat_body(const float* __restrict__ Q, const float* __restrict__ K,
                                                const float* __restrict__ V, const float* __restrict__ dO,
                                                const float* __restrict__ LSE, const float* __restrict__ Delta,
                                                float* __restrict__ dQ, float* __restrict__ dK,
                                                float* __restrict__ dV, int BH, int S, _Float16* lds,
                                                float (*rowc)[2][32]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int nkb = (S + 31) / 32;
    const int bh = blockIdx.x / nkb, kb = blockIdx.x - bh * nkb;
    if (bh >= BH) return;
    const long base = (long)bh * S * D;
    const long rbase = (long)bh * S;
    const int k0 = kb * 32, key = k0 + r;
    const bool kvalid = key < S;
    const float kscale = FA2B_LOG2E / __builtin_sqrtf((float)D);
    const float dscale = 1.f / __builtin_sqrtf((float)D);
    _Float16* buf = lds + wave * 32 * D;
    float* acc = reinterpret_cast<float*>(lds);  // [32][D] f32 merge buffer
    FragOffsets<D> fo;
    fo.init(lane);
    // sum the four waves' accumulators ([32 x 32] blocks, d on the rows) in wave order
    // through the merge buffer, then write rows k0.. of dst scaled by sc
    auto merge_store = [&](const f32x16 (&part)[D / 32], float* dst, float sc) {
        for (int w = 0; w < 4; ++w) {
            __syncthreads();
            if (wave == w) {
#pragma unroll
                for (int b = 0; b < D / 32; ++b)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        float* a = acc + r * D + 32 * b + (i & 3) + 8 * (i >> 2) + 4 * h;
                        *a = w == 0 ? part[b][i] : *a + part[b][i];
                    }
            }
        }
        __syncthreads();
        for (int x = tid; x < 32 * D; x += 256) {
            const int row = x / D, d = x - row * D;
            if (k0 + row < S) dst[base + (long)(k0 + row) * D + d] = acc[x] * sc;
        }
        __syncthreads();
    };

    // ---- role 1: dK, dV of keys k0 .. k0 + 31
    {
        f16x8 kf[D / 16], vf[D / 16];
#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
            kf[t] = load_frag(K + base + (long)key * D + 16 * t + 8 * h, kvalid, kscale);
            vf[t] = load_frag(V + base + (long)key * D + 16 * t + 8 * h, kvalid, 1.f);
        }
        f32x16 dka[D / 32], dva[D / 32];
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                dka[b][i] = 0.f;
                dva[b][i] = 0.f;
            }
        TileStager<D, 32, 64> qs, ds;
        qs.init(Q + base, S, lane);
        ds.init(dO + base, S, lane);
        const int nqt = (S + 31) / 32;
        for (int j = wave; j < nqt; j += 4) {
            const int q0 = j * 32;
            if (h == 0) {
                const int qi = q0 + r;
                rowc[wave][0][r] = qi < S ? -LSE[rbase + qi] * FA2B_LOG2E : -__builtin_inff();
                rowc[wave][1][r] = qi < S ? -Delta[rbase + qi] : 0.f;
            }
            qs.load(q0);
            qs.store(buf, 1.f, lane);
            f32x16 sa, da;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
                sa[i] = rowc[wave][0][row];
                da[i] = rowc[wave][1][row];
            }
            // rows: query q0 + (i&3) + 8*(i>>2) + 4h ; col: key (lane)
#pragma unroll
            for (int t = 0; t < D / 16; ++t) sa = mfma(fo.rowop(buf, 0, t), kf[t], sa);
            ds.load(q0);
            ds.store(buf, 1.f, lane);
#pragma unroll
            for (int t = 0; t < D / 16; ++t) da = mfma(fo.rowop(buf, 0, t), vf[t], da);
            f16x8 pf[2], dsf[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = kvalid ? fast_exp2(sa[i]) : 0.f;
                pf[i >> 3][i & 7] = to_tile(p);
                dsf[i >> 3][i & 7] = to_tile(p * da[i]);
            }
            // dV^T += dO^T P
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int s = 0; s < 2; ++s) dva[b] = mfma(fo.trop(buf, 16 * s, b), pf[s], dva[b]);
            qs.store(buf, 1.f, lane);  // Q again (still in registers) for dK
            // dK^T += Q^T dS
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int s = 0; s < 2; ++s) dka[b] = mfma(fo.trop(buf, 16 * s, b), dsf[s], dka[b]);
        }
        merge_store(dka, dK, dscale);
        merge_store(dva, dV, 1.f);
    }

    // ---- role 2: dQ of queries k0 .. k0 + 31 (this workgroup's index as a query block)
    {
        const int q = k0 + r;
        const bool qvalid = q < S;
        f16x8 qf[D / 16], of[D / 16];
#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
            qf[t] = load_frag(Q + base + (long)q * D + 16 * t + 8 * h, qvalid, kscale);
            of[t] = load_frag(dO + base + (long)q * D + 16 * t + 8 * h, qvalid, 1.f);
        }
        const float nl = qvalid ? -LSE[rbase + q] * FA2B_LOG2E : -__builtin_inff();
        const float nd = qvalid ? -Delta[rbase + q] : 0.f;
        f32x16 dqa[D / 32];
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) dqa[b][i] = 0.f;
        TileStager<D, 32, 64> kst, vst;
        kst.init(K + base, S, lane);
        vst.init(V + base, S, lane);
        for (int j = wave; j < nkb; j += 4) {
            const int kk0 = j * 32;
            kst.load(kk0);
            kst.store(buf, 1.f, lane);
            f32x16 sa, da;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                sa[i] = nl;
                da[i] = nd;
            }
            // S^T = K Q^T - LSE*log2e: rows key kk0 + (i&3) + 8*(i>>2) + 4h, lane = query
#pragma unroll
            for (int t = 0; t < D / 16; ++t) sa = mfma(fo.rowop(buf, 0, t), qf[t], sa);
            vst.load(kk0);
            vst.store(buf, 1.f, lane);  // after this wave's K reads (in-order LDS within a wave)
            // dP^T = V dO^T - Delta
#pragma unroll
            for (int t = 0; t < D / 16; ++t) da = mfma(fo.rowop(buf, 0, t), of[t], da);
            f16x8 dsf[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool kv = kk0 + (i & 3) + 8 * (i >> 2) + 4 * h < S;
                const float p = kv ? fast_exp2(sa[i]) : 0.f;
                dsf[i >> 3][i & 7] = to_tile(p * da[i]);
            }
            kst.store(buf, 1.f, lane);  // K again (still in registers) for dQ^T += K^T dS^T
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int s = 0; s < 2; ++s) dqa[b] = mfma(fo.trop(buf, 16 * s, b), dsf[s], dqa[b]);
        }
        merge_store(dqa, dQ, dscale);
    }
}

// Δ = rowsum(dO ∘ O), one row per workgroup of any blockDim (the harness uses 64).
__device__ __forceinline__ void delta_row_body(const float* __restrict__ dO, const float* __restrict__ O, long rows,
                                               int D, float* __restrict__ Dvec) {
    __shared__ float part[16];
    const long row = blockIdx.x;
    if (row >= rows) return;
    float acc = 0.f;
    for (int d = threadIdx.x; d < D; d += blockDim.x) acc += dO[row * D + d] * O[row * D + d];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    const int nw = (blockDim.x + 63) / 64;
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += part[w];
        Dvec[row] = s;
    }
}

}  // namespace fa2f16b

#ifndef CUPY_INLINE_COMPILE
namespace fa2 {

namespace {
// dK/dV kernel instances (NW waves x 32 keys; QS query groups).  16x16x32 everywhere
// but the 2-wave instance: at the power cap on random data 16x16x32 delivers 16 %
// more FLOPs per joule than 32x32x16 (+5 % at C3, +4 % at D = 128, +7 % on small
// D = 64 grids); the 2-wave instance keeps 32x32x16.
template <int D, int NW, bool M16 = true, int QS = 1>
hipError_t dkdv_launch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                       const float* delta, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    const long grid = (long)bh * ((S + 32 * (NW / QS) - 1) / (32 * (NW / QS)));
    if (grid <= 0 || grid > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f16b::fa2_bwd_dkdv_f16_kernel<D, NW, 1, M16, QS>), dim3((unsigned)grid), dim3(64 * NW), 0,
                       stream, q, k, v, dout, lse, delta, dk, dv, S);
    return hipGetLastError();
}
// Geometry: 8 waves x 32 keys for D <= 64 (2 waves/SIMD in 256 VGPRs); D = 128 4 x 32
// (more than 256 registers per lane); fewer waves where the grid would leave CUs idle.
// Launch-plan overrides (fa2_tune_set, tests and tools only): DKDV_WAVES, DKDV_QS.
template <int D>
hipError_t dkdv_dispatch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                         const float* delta, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    int nw = tune_knob("DKDV_WAVES", 0);  // 0 = auto_waves over the grid of 32-key wave units
    const long units = (long)bh * ((S + 31) / 32);
    // Query groups per workgroup (0 = auto).  Auto, where 8-wave workgroups of one key
    // block per wave would leave CUs idle: below 8 key blocks per CU QS = 2 at 8 waves;
    // below 4, D = 32 QS = 4 at 8 waves and D = 64 QS = 2 at 4 waves (at QS = 4 its
    // 4-tile staging registers spill).  Measured (B2_H8_D64, r01): S = 512 16.1 -> 12.1
    // us, 1024 29.1 -> 20.8, 2048 53.7 -> 44.3.
    int qs = tune_knob("DKDV_QS", 0);
    // a forced DKDV_HS the plan cannot take (D, or other plan knobs) is an error, never a
    // silent launch of another kernel
    if (tune_knob("DKDV_HS", -1) == 1 && (D != 64 || nw || qs)) return hipErrorInvalidValue;
    if constexpr (D == 64) {
        // hand-scheduled kernel: whole 64-query steps, and a grid of at least one 256-key
        // workgroup per CU.  DKDV_HS (tests and tools): 1 forces it (an error where it
        // cannot serve), 0 disables it.  r06, on 16x16x32 (the r05 32x32x16 form lost inside
        // the step): in one process against the 8-wave kernel, dK/dV -3.1 .. -4.5 % and the
        // fwd + bwd step -1.5 .. -2.1 % at C3, B2_H8_S4096 and B16_H16_S2048, dO = ones and
        // N(0,1) (profiles/r06/dkhs16/)
        const int hs = tune_knob("DKDV_HS", -1);
        const bool fits = S % 64 == 0 && S >= 128;
        if (hs == 1 && !fits) return hipErrorInvalidValue;
        const long hgrid = (long)bh * ((S + 255) / 256);
        if (fits && (hs == 1 || (hs < 0 && nw == 0 && qs == 0 && hgrid >= cu_count()))) {
            if (hgrid > 0x7fffffffL) return hipErrorInvalidValue;
            hipLaunchKernelGGL((fa2f16b::fa2_bwd_dkdv_hs_kernel<D>), dim3((unsigned)hgrid), dim3(256), 0, stream, q, k,
                               v, dout, lse, delta, dk, dv, S, 1, nullptr);
            return hipGetLastError();
        }
    }
    if (qs == 0 && nw == 0 && D <= 64) {
        const int a = auto_waves(units, 8);
        if (a == 4) qs = 2, nw = 8;
        else if (a == 2 && D <= 32) qs = 4, nw = 8;
        else if (a == 2) qs = 2, nw = 4;
    }
    // D = 128: 4 waves on every grid (r04: the 2-wave workgroups auto_waves gave small
    // grids measured slower everywhere, B2_H8 D = 128 dK/dV S = 1500 87.9 -> 73.5 us,
    // 1024 54.3 -> 50.9, 512 29.0 -> 28.1; profiles/r04/d128/)
    if (nw == 0) nw = D <= 64 ? auto_waves(units, 8) : 4;
    if constexpr (D <= 64) {
        if (qs == 2 && nw == 8) return dkdv_launch<D, 8, true, 2>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        if (qs == 2 && nw == 4) return dkdv_launch<D, 4, true, 2>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        if (nw == 8) return dkdv_launch<D, 8>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    }
    if constexpr (D <= 32) {
        if (qs == 4 && nw == 8) return dkdv_launch<D, 8, true, 4>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    }
    if (nw == 2) return dkdv_launch<D, 2, false>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    return dkdv_launch<D, 4>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
}
template <int D, int NW, int NKB = 2, bool M16 = false, int KS = 1>
hipError_t dq_launch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                     float* delta, float* dq, int bh, int S, const float* o, hipStream_t stream) {
    const long grid = (long)bh * ((S + 32 * (NW / KS) - 1) / (32 * (NW / KS)));
    if (grid <= 0 || grid > 0x7fffffffL) return hipErrorInvalidValue;
    if (o)
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_f16_kernel<D, NW, true, NKB, M16, KS>), dim3((unsigned)grid),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, S, o);
    else
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_f16_kernel<D, NW, false, NKB, M16, KS>), dim3((unsigned)grid),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, S, o);
    return hipGetLastError();
}
template <int D>
hipError_t dq_dispatch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                       float* delta, float* dq, int bh, int S, const float* o, hipStream_t stream) {
    // 8 waves (2 per SIMD) for D <= 64; at D = 128 8 waves spill (~120 VGPRs), so 4.
    // Launch-plan overrides (fa2_tune_set, tests and tools only): DQ_WAVES, DQ_KS.
    int nw = tune_knob("DQ_WAVES", 0);  // 0 = auto_waves over the grid of 32-query wave units
    // (D = 128 at 8 waves spills even with 32-key tiles: Q, dO fragments, the -LSE / -Δ
    // seeds and the dQ accumulators alone are 160 VGPRs -- r01)
    // (D = 128 at 8 waves on 16x16x32 with 32-key tiles still spills ~70 VGPRs inside the
    // loop: Q, dO fragments and the dQ accumulators alone take 128)
    const long units = (long)bh * ((S + 31) / 32);
    // Key groups per workgroup (0 = auto).  Auto, at 8 waves: KS = 2
    // below 8 query blocks per CU, KS = 4 below 4 (KS = 4 runs 32-key tiles: 64-key
    // tiles with the 4-tile staging registers spill).  Measured (B2_H8_D64 dQ + Δ,
    // r01): S = 512 17.0 -> 11.4 us, 1024 29.5 -> 15.7, 2048 41.9 -> 36.7.
    int ksp = tune_knob("DQ_KS", 0);
    if (tune_knob("DQ_HS", -1) == 1 && (D != 64 || nw || ksp)) return hipErrorInvalidValue;
    if constexpr (D == 64) {
        // hand-scheduled kernel (r05): whole 64-key tiles, and a grid of at least one
        // 256-row workgroup per CU.  DQ_HS (tests and tools): 1 forces it (an error where it
        // cannot serve), 0 disables it
        const int hs = tune_knob("DQ_HS", -1);
        const bool fits = S % 64 == 0 && S >= 128;
        if (hs == 1 && !fits) return hipErrorInvalidValue;
        const long hgrid = (long)bh * ((S + 255) / 256);
        if (fits && (hs == 1 || (hs < 0 && nw == 0 && ksp == 0 && hgrid >= cu_count()))) {
            if (hgrid > 0x7fffffffL) return hipErrorInvalidValue;
            hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_hs_kernel<D>), dim3((unsigned)hgrid), dim3(256), 0, stream, q, k, v,
                               dout, lse, delta, dq, S, o, 1, nullptr);
            return hipGetLastError();
        }
    }
    if (ksp == 0 && nw == 0 && D <= 64) {
        const int a = auto_waves(units, 8);
        if (a == 4) ksp = 2, nw = 8;
        else if (a == 2) ksp = 4, nw = 8;
    }
    if (nw == 0) nw = auto_waves(units, D <= 64 ? 8 : 4, D <= 64 ? 2 : 4);
    if constexpr (D <= 64) {
        if (ksp == 2 && nw == 8) return dq_launch<D, 8, 2, true, 2>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        if (ksp == 4 && nw == 8) return dq_launch<D, 8, 1, true, 4>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        if (ksp == 2 && nw == 4) return dq_launch<D, 4, 2, true, 2>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        if (ksp == 4 && nw == 4) return dq_launch<D, 4, 1, true, 4>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
    }
    // 16x16x32 (+2.4 % at C3 over 32x32x16) but at 2 waves
    if constexpr (D <= 64) {
        if (nw == 8) return dq_launch<D, 8, 2, true>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        if (nw == 2) return dq_launch<D, 2>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
    }
    return dq_launch<D, 4, 2, true>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
}
}  // namespace

hipError_t FA2_TILE_LAUNCH(launch_bwd_dkdv)(int D, const float* q, const float* k, const float* v, const float* dout,
                               const float* lse, const float* delta, float* dk, float* dv, int bh, int S,
                               hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    switch (D) {
        case 32: return dkdv_dispatch<32>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        case 64: return dkdv_dispatch<64>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        case 128: return dkdv_dispatch<128>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t FA2_TILE_LAUNCH(launch_bwd_dq)(int D, const float* q, const float* k, const float* v, const float* dout,
                             const float* lse, const float* delta, float* dq, int bh, int S, hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    float* dl = const_cast<float*>(delta);  // read only when o == nullptr
    switch (D) {
        case 32: return dq_dispatch<32>(q, k, v, dout, lse, dl, dq, bh, S, nullptr, stream);
        case 64: return dq_dispatch<64>(q, k, v, dout, lse, dl, dq, bh, S, nullptr, stream);
        case 128: return dq_dispatch<128>(q, k, v, dout, lse, dl, dq, bh, S, nullptr, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t FA2_TILE_LAUNCH(launch_bwd_dq_delta)(int D, const float* q, const float* k, const float* v, const float* o,
                                   const float* dout, const float* lse, float* delta, float* dq, int bh, int S,
                                   hipStream_t stream) {
    if (bh <= 0 || S <= 0 || !o) return hipErrorInvalidValue;
    switch (D) {
        case 32: return dq_dispatch<32>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        case 64: return dq_dispatch<64>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        case 128: return dq_dispatch<128>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        default: return hipErrorInvalidValue;
    }
}

namespace {
// o != nullptr: the DEL instance (Δ computed in both roles from O and written to delta)
template <int D, int NW, int QS, int KS, int NKB>
hipError_t fused_launch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                        float* delta, float* dq, float* dk, float* dv, int bh, int S, const float* o,
                        hipStream_t stream) {
    const long ndk = (long)bh * ((S + 32 * (NW / QS) - 1) / (32 * (NW / QS)));
    const long ndq = (long)bh * ((S + 32 * (NW / KS) - 1) / (32 * (NW / KS)));
    if (ndk <= 0 || ndq <= 0 || ndk + ndq > 0x7fffffffL) return hipErrorInvalidValue;
    if (o)
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_fused_f16_kernel<D, NW, QS, KS, NKB, true>), dim3((unsigned)(ndk + ndq)),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, dk, dv, S, (int)ndk, o);
    else
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_fused_f16_kernel<D, NW, QS, KS, NKB>), dim3((unsigned)(ndk + ndq)),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, dk, dv, S, (int)ndk, o);
    return hipGetLastError();
}
// The fused dK/dV + dQ launch for D <= 64, or hipErrorNotSupported (then the caller
// runs the two kernels).  Split factors: below 4 blocks of 32 rows per CU QS = 2 /
// KS = 2, else unsplit.  Overrides (fa2_tune_set): BWD_FQS, BWD_FKS, BWD_FNW.
template <int D>
hipError_t fused_dispatch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                          float* delta, float* dq, float* dk, float* dv, int bh, int S, const float* o,
                          hipStream_t stream) {
    if constexpr (D > 64) {
        return hipErrorNotSupported;
    } else {
        const long units = (long)bh * ((S + 31) / 32);
        const int a = auto_waves(units, 8);
        // below 2 blocks per CU: 4-wave roles, KS = 2 (B2_H8_S512: bwd 16.7 -> 15.7 us;
        // at 2 blocks per CU, B2_H8_S1024, that geometry is 21 % slower than 8 waves)
        const bool tiny = a == 2 && auto_waves(units, 2, 1) == 1;
        // dQ role KS = 2 on every split grid (r02: below 4 blocks per CU KS = 2 beat the
        // r01 choice KS = 4 by 4.6-7.5 % on the fwd + bwd step, B2_H8_S1024 D = 32 / 64,
        // B4_H8_S512, B1_H16_S1024, S = 1000, both dO distributions)
        // With 4-8 blocks per CU both roles run unsplit (r03, with iglp_opt(2) on the
        // fused kernel: B2_H8_S2048 bwd 69.0 -> 64.4 us, dO ~ N(0,1) 72.7 -> 68.0, S = 1500
        // 54.3 -> 48.7, B4_H8_S1024 43.9 -> 39.6, D = 32 S = 2048 44.3 -> 41.6;
        // profiles/r03/ab/froles/); below 4 the split roles stay (S = 1024: 24.6 vs 33.4)
        // r04: the split roles (128 keys / 128 query rows per workgroup: units / 2
        // workgroups) only while their grid fits one round of workgroups; past that the
        // unsplit roles (units / 4) win: B2_H8_S1500 bwd 54.5 -> 47.3 us, B3_H8_S1024
        // 41.0 -> 36.2; B2_H8_S1024 (exactly one round split) keeps the split, 26.2 vs
        // 34.0 unsplit (profiles/r04/bwdr/)
        const bool split = (units + 1) / 2 <= (long)cu_count();
        const int fqs = tune_knob("BWD_FQS", split ? 2 : 1);
        const int fks = tune_knob("BWD_FKS", split ? 2 : 1);
        // waves per workgroup of both roles (8, or 4 for the split pairs; the unsplit
        // roles exist at 8 waves only, so a forced FQS = FKS = 1 on a tiny grid takes 8)
        const int fnw = tune_knob("BWD_FNW", tiny && !(fqs == 1 && fks == 1) ? 4 : 8);
        // an override combination no instance serves is an error, never a silent
        // fallback to the two-kernel plan (an A/B would otherwise time the default)
        const bool forced = tune_knob("BWD_FQS", 0) || tune_knob("BWD_FKS", 0) || tune_knob("BWD_FNW", 0);
        if (fnw != 4 && fnw != 8) return hipErrorInvalidValue;
        if (fqs == 1 && fks == 1) {
            if (fnw != 8) return hipErrorInvalidValue;  // the unsplit roles exist at 8 waves only
            return fused_launch<D, 8, 1, 1, 2>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        }
        if (fnw == 4) {
            if (fqs == 2 && fks == 2)
                return fused_launch<D, 4, 2, 2, 2>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
            if (fqs == 2 && fks == 4)
                return fused_launch<D, 4, 2, 4, 1>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        }
        if (fqs == 2 && fks == 2) return fused_launch<D, 8, 2, 2, 2>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        if (fqs == 2 && fks == 4) return fused_launch<D, 8, 2, 4, 1>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        return forced ? hipErrorInvalidValue : hipErrorNotSupported;
    }
}
}  // namespace

hipError_t FA2_TILE_LAUNCH(launch_bwd_fused)(int D, const float* q, const float* k, const float* v, const float* dout,
                                const float* lse, const float* delta, float* dq, float* dk, float* dv, int bh, int S,
                                hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    float* dl = const_cast<float*>(delta);  // read only (no O given)
    switch (D) {
        case 32: return fused_dispatch<32>(q, k, v, dout, lse, dl, dq, dk, dv, bh, S, nullptr, stream);
        case 64: return fused_dispatch<64>(q, k, v, dout, lse, dl, dq, dk, dv, bh, S, nullptr, stream);
        default: return hipErrorNotSupported;
    }
}

namespace {
// the fused launch with Δ computed inside it from O (written to delta)
hipError_t launch_bwd_fused_delta(int D, const float* q, const float* k, const float* v, const float* o,
                                  const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                                  int bh, int S, hipStream_t stream) {
    switch (D) {
        case 32: return fused_dispatch<32>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        case 64: return fused_dispatch<64>(q, k, v, dout, lse, delta, dq, dk, dv, bh, S, o, stream);
        default: return hipErrorNotSupported;
    }
}
}  // namespace

// The split backward (D = 64, grids below one 256-row workgroup per CU): the
// hand-scheduled dQ kernel on P key chunks (Δ fused, written by chunk 0), the
// hand-scheduled dK/dV kernel on P query chunks, both leaving fp32 parts in the stream's
// scratch block, then one ordered reduce of the three tensors.  BWD_SPLIT (tests and
// tools): P >= 2 forces it (an error where it cannot serve: D, shape, other backward plan
// knobs, or no scratch -- a stream being captured without an earlier eager block),
// 1 disables it, 0 = auto (bwd_split_auto).  hipErrorNotSupported: not this plan.
// Chunks per head for a grid of `g` 256-row blocks: only where the unsplit plans leave
// most CUs idle with long heads (g <= 64 at S >= 4096, g <= 16 at S >= 2048), the most
// chunks (a power of two, at most 8) that keep one workgroup per CU and chunks of at
// least 256 rows.  r06 in-process A/B of fa2_backward (profiles/r06/bsplit/), the
// small-grid plan -> split: B1_H2_S4096 88.2 -> 59.6 us (P = 8), B1_H4_S4096 92.9 -> 87.9
// (4), B1_H2_S8192 177.9 -> 149.7 (4), B1_H2_S2048 42.9 -> 37.4 (8); B1_H4_S2048 ties,
// B1_H8_S4096 / B1_H8_S2048 / B2_H8_S2048 lose 1-40 % (three fp32 part tensors and the
// reduce grow with the workgroups; the fused small-grid plan does no recompute).
static int bwd_split_auto(long g, int S) {
    if (!(S >= 4096 && g <= 64) && !(S >= 2048 && g <= 16)) return 1;
    const long ncu = cu_count();
    int P = 1;
    while (P < 8 && g * (2 * P) <= ncu && S % (64 * 2 * P) == 0 && S / (2 * P) >= 256) P *= 2;
    return P;
}
static hipError_t bwd_split_plan(int D, const float* q, const float* k, const float* v, const float* o, const float* dout,
                          const float* lse, float* delta, float* dq, float* dk, float* dv, int bh, int S,
                          hipStream_t stream) {
    const int split = tune_knob("BWD_SPLIT", 0);
    if (split < 0) return hipErrorInvalidValue;
    if (split == 1) return hipErrorNotSupported;
    const bool fits = D == 64 && bh > 0 && S % 64 == 0 && S >= 128;
    const bool forced_other = tune_knob("BWD_FUSED", -1) >= 0 || tune_knob("DQ_HS", -1) >= 0 ||
                              tune_knob("DKDV_HS", -1) >= 0 || tune_knob("DQ_WAVES", 0) || tune_knob("DQ_KS", 0) ||
                              tune_knob("DKDV_WAVES", 0) || tune_knob("DKDV_QS", 0);
    if (split >= 2 && (!fits || forced_other || S % (64 * split) || S / split < 128)) return hipErrorInvalidValue;
    const long g = fits ? (long)bh * ((S + 255) / 256) : 0;
    const int P = split >= 2 ? split : (fits && !forced_other && g < cu_count()) ? bwd_split_auto(g, S) : 1;
    if (P < 2) return hipErrorNotSupported;
    const long n = (long)bh * S * D;
    float* part = static_cast<float*>(stream_scratch(stream, sizeof(float) * 3 * P * (size_t)n));
    if (!part) return split >= 2 ? hipErrorInvalidValue : hipErrorNotSupported;
    const long grid = g * P;
    if (grid > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_hs_kernel<64>), dim3((unsigned)grid), dim3(256), 0, stream, q, k, v, dout,
                       lse, delta, dq, S, o, P, part);
    hipLaunchKernelGGL((fa2f16b::fa2_bwd_dkdv_hs_kernel<64>), dim3((unsigned)grid), dim3(256), 0, stream, q, k, v,
                       dout, lse, delta, dk, dv, S, P, part + (long)P * n);
    hipLaunchKernelGGL(fa2f16b::fa2_bwd_split_reduce_kernel, dim3((unsigned)((n / 4 + 255) / 256), 3), dim3(256), 0,
                       stream, part, P, n, dq, dk, dv);
    return hipGetLastError();
}

// Override BWD_FUSED (fa2_tune_set): 1 = Δ kernel, then dK/dV and dQ in one launch (D <= 64);
// 0 = Δ fused into the dQ kernel's prologue (which stages dO anyway), then dK/dV,
// which reads it; -1 (default) = 1 on grids of fewer than 8 blocks of 32 rows per
// CU.  Measured (fwd + bwd step, B2_H8_D64, r01): S = 512 31.1 -> 27.0 us, 1024
// 50.1 -> 48.2, 2048 108.7 -> 106.0; S = 4096 282 -> 286 and C3 +-0 (so unfused).
hipError_t FA2_TILE_LAUNCH(launch_backward)(int D, const float* q, const float* k, const float* v, const float* o,
                               const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv,
                               int bh, int S, hipStream_t stream) {
    {
        const hipError_t e = bwd_split_plan(D, q, k, v, o, dout, lse, delta, dq, dk, dv, bh, S, stream);
        if (e != hipErrorNotSupported) return e;
    }
    int fused = tune_knob("BWD_FUSED", -1);
    if (fused < 0) fused = bh > 0 && S > 0 && auto_waves((long)bh * ((S + 31) / 32), 8) < 8;
    if (D <= 64 && bh > 0 && S > 0 && fused == 1) {
        // the fused launch has no hand-scheduled roles: forcing one is an error
        if (tune_knob("DQ_HS", -1) == 1 || tune_knob("DKDV_HS", -1) == 1) return hipErrorInvalidValue;
        // Δ inside the fused launch below 4 blocks of 32 rows per CU (override
        // BWD_FUSED_DELTA; 0 = the separate Δ kernel first).  Measured (B2_H8_D64 fwd +
        // bwd, r02): S = 512 29.9 -> 26.7 us, S = 1024 45.0 -> 40.8; at S = 2048 (4
        // blocks per CU) the dK/dV role's O reads cost more than the Δ kernel (+4 %).
        const int dfl = auto_waves((long)bh * ((S + 31) / 32), 8) <= 2;
        if (tune_knob("BWD_FUSED_DELTA", dfl)) {
            const hipError_t e = launch_bwd_fused_delta(D, q, k, v, o, dout, lse, delta, dq, dk, dv, bh, S, stream);
            if (e != hipErrorNotSupported) return e;
        }
        hipError_t e = launch_delta(D, dout, o, delta, bh, S, stream);
        if (e != hipSuccess) return e;
        e = FA2_TILE_LAUNCH(launch_bwd_fused)(D, q, k, v, dout, lse, delta, dq, dk, dv, bh, S, stream);
        if (e != hipErrorNotSupported) return e;
    }
    hipError_t e = FA2_TILE_LAUNCH(launch_bwd_dq_delta)(D, q, k, v, o, dout, lse, delta, dq, bh, S, stream);
    if (e != hipSuccess) return e;
    return FA2_TILE_LAUNCH(launch_bwd_dkdv)(D, q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
}

}  // namespace fa2

// Host API with the reference's semantics (f-attn2-backward_f16.cu:375-474).
template <int head_dim>
void FA2_TILE_HOST(host_flash_attention2_backward)(const float* h_Q, const float* h_K, const float* h_V, const float* h_O,
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
    HIP_CHECK(fa2::FA2_TILE_LAUNCH(launch_backward)(head_dim, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9],
                                       batch_size * num_heads, seq_len, nullptr));
    tm->Stop();
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(h_dQ, d[7], n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_dK, d[8], n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_dV, d[9], n * sizeof(float), hipMemcpyDeviceToHost));
    for (int i = 0; i < 10; ++i) HIP_CHECK(hipFree(d[i]));
}
#define FA2_INST_BWD16(D)                                                                                         \
    template void FA2_TILE_HOST(host_flash_attention2_backward)<D>(const float*, const float*, const float*, const float*, \
                                                         const float*, const float*, float*, float*, float*, int, \
                                                         int, int, TimerManager*);
FA2_INST_BWD16(32)
FA2_INST_BWD16(64)
FA2_INST_BWD16(128)
#else
// CuPy face (same symbols as f-attn2-backward_f16.cu:477-514).  dQ, dK, dV are
// overwritten (the harness zero-fills them for the reference's atomics; nothing here
// adds into them).  head_dim is honoured (32, 64, 128).  Static LDS is 32 KB, so the
// harness's dynamic bytes ((32D + 4*32D + 32 + 32*32)*4, 45 184 at D = 64, 86 144 at
// D = 128) still fit in the 160 KiB of a workgroup.
extern "C" __global__ void __launch_bounds__(256)
flash_attention2_backward_kernel_wrapper(const float* query, const float* key, const float* value,
                                         const float* output, const float* d_output, const float* logsumexp,
                                         const float* d, float* d_query, float* d_key, float* d_value,
                                         int batch_size, int num_heads, int seq_len, int head_dim) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[fa2f16b::CompatLds::HALVES];
    __shared__ float rowc[4][2][32];
    const int bh = batch_size * num_heads;
    (void)output;
    if (head_dim == 64)
        fa2f16b::bwd_compat_body<64>(query, key, value, d_output, logsumexp, d, d_query, d_key, d_value, bh, seq_len,
                                     lds, rowc);
    else if (head_dim == 32)
        fa2f16b::bwd_compat_body<32>(query, key, value, d_output, logsumexp, d, d_query, d_key, d_value, bh, seq_len,
                                     lds, rowc);
    else if (head_dim == 128)
        fa2f16b::bwd_compat_body<128>(query, key, value, d_output, logsumexp, d, d_query, d_key, d_value, bh,
                                      seq_len, lds, rowc);
}

extern "C" __global__ void D_computation_reduction_kernel_wrapper(const float* d_output, const float* output,
                                                                  int batch_size, int num_heads, int seq_len,
                                                                  int head_dim, float* d) {
    fa2f16b::delta_row_body(d_output, output, (long)batch_size * num_heads * seq_len, head_dim, d);
}
#endif  // CUPY_INLINE_COMPILE
