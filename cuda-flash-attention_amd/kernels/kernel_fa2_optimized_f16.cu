// kernel_fa2_optimized_f16.cu -- FA2 forward, fp16-tile MFMA path, for MI355X (gfx950).
//
// Replaces detker/CUDA-Flash-Attention kernels/kernel_fa2_optimized_f16.cu
// (flash_attention2_forward_kernel_fp16, :20-350; host launcher :353-430; CuPy
// wrapper :432-448).  Same math: O = softmax(Q Kᵀ/√D) V, LSE = ln Σ exp + max,
// fp32 tensors in HBM; the tiles live in fp16 and both contractions run on
// v_mfma_f32_32x32x16_f16 with fp32 accumulation (the reference does scalar
// fp32 FMAs on __half LDS tiles).
//
// Design:
//   * one wave = 32 query rows; a workgroup = NW waves sharing 64-key K/V tiles;
//   * S is computed transposed, Sᵀ = K·Qᵀ, so each lane owns one query and 32 of
//     the tile's 64 keys in registers: the row max needs one cross-half
//     exchange, the row sum none until the epilogue;
//   * the Sᵀ accumulator, packed to fp16, IS the B operand of Oᵀ += Vᵀ·Pᵀ (no
//     LDS round trip for P); Vᵀ comes from the row-major V tile through
//     ds_read_b64_tr_b16;
//   * Q is pre-scaled by log2(e)/√D so p = exp2(s - m) is one v_exp_f32;
//   * K/V tiles: fp32 HBM -> registers (issued before the MFMAs of the previous
//     tile) -> fp16 -> XOR-swizzled LDS, double-buffered, one barrier per tile;
//   * blockIdx is remapped so all query blocks of one head share an XCD's L2.
//
// This file is self-contained device code so that it also compiles from source
// text under hiprtc with -DCUPY_INLINE_COMPILE (the reference harness's
// cp.RawModule path, test_flash_attention2.py:113-126), C++14 only.
#ifndef CUPY_INLINE_COMPILE
#include "f-attn2.cuh"
#endif

#ifdef FA2_TILE_BF16
#define fa2f16 fa2bf16
#define FA2_TILE_LAUNCH(x) x##_bf16
#define FA2_TILE_HOST(x) x##_bf16
#else
#define FA2_TILE_LAUNCH(x) x##_f16
#define FA2_TILE_HOST(x) x##_fp16
#endif
namespace fa2f16 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

#define FA2_LOG2E 1.4426950408889634f
#define FA2_LN2 0.6931471805599453f

// Tile element type.  The default build stores fp16 tiles.  The same source compiled
// with -DFA2_TILE_BF16 (Makefile: *_bf16.o, namespace fa2bf16, launchers *_bf16)
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
// sum of a packed pair of tile values plus c (v_dot2_f32_bf16 against ones)
__device__ __forceinline__ float pair_sum(_Float16 a, _Float16 b, float c) {
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const s16x2 v = {__builtin_bit_cast(short, a), __builtin_bit_cast(short, b)};
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, v), bf16x2{(__bf16)1.f, (__bf16)1.f}, c, false);
}
#else
__device__ __forceinline__ _Float16 to_tile(float x) { return (_Float16)x; }
// sum of a packed pair of tile values plus c (v_dot2_f32_f16 against ones)
__device__ __forceinline__ float pair_sum(_Float16 a, _Float16 b, float c) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2(f16x2{a, b}, f16x2{(_Float16)1.f, (_Float16)1.f}, c, false);
}
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
#endif

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// XOR swizzle of the 16-byte chunk index of LDS row r (fp16 rows of D halves).
// Chosen by search (tools/lds_swizzle.py, `swz_old`) so that the 32x32x16 access
// kinds are bank-conflict-free: ds_read_b128 row fragments (lane -> row) and
// ds_read_b64_tr_b16 transposed fragments.  The backward file's swizzle is also
// conflict-free for the 16x16x32 maps its default kernels use; this forward's
// default kernel is 32x32x16 (a 16x16x32 forward's row reads are 2-way here).  f reads
// row bits 0..3 only: fragment offsets are computed once per lane and shifted by
// whole 16-row blocks (FragOffsets*::rowop / trop add r0 * D).
template <int D> struct Swz;
template <> struct Swz<32> {
    static __device__ __forceinline__ int f(int r) { return ((r >> 2) & 1) | (((r >> 3) & 1) << 1); }
};
template <> struct Swz<64> {
    static __device__ __forceinline__ int f(int r) {
        return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | ((((r >> 1) ^ (r >> 3)) & 1) << 2);
    }
};
template <> struct Swz<128> {
    static __device__ __forceinline__ int f(int r) {
        return (r & 1) | (((r >> 1) & 1) << 1) | (((r ^ (r >> 2)) & 1) << 2) | ((((r >> 1) ^ (r >> 3)) & 1) << 3);
    }
};

// element offset (in halves) of (row, col) in a swizzled [rows][D] fp16 tile
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

// Bijective XCD-aware remap (guide T1): consecutive logical blocks land on one XCD.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, rr = nwg & 7, xcd = orig & 7, idx = orig >> 3;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
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
    // move every offset by o halves (a wave's fixed tile inside a multi-tile image)
    __device__ __forceinline__ void shift(int o) {
#pragma unroll
        for (int t = 0; t < D / 16; ++t) row[t] += o;
#pragma unroll
        for (int b = 0; b < D / 32; ++b) {
            tr[b][0] += o;
            tr[b][1] += o;
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

    __device__ __forceinline__ void set_head(const float* head_base, int S) { rs = head_rsrc(head_base, S, D); }
    __device__ __forceinline__ void init(const float* head_base, int S, int tid) {
        set_head(head_base, S);
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

__device__ __forceinline__ float xor32_max(float x) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Online-softmax state of one wave: 32 query rows (one per lane pair), O^T
// accumulator (d on the rows), running max m (log2 domain), four partial row sums
// (four short dependency chains per tile, not one of 32), and nm = -m broadcast
// over 16 registers: the initial value of every S^T accumulator, so the QK^T
// MFMAs produce s - m directly (no per-score v_sub).
template <int D>
struct FwdState {
    f16x8 qf[D / 16];
    f32x16 oacc[D / 32];
    f32x16 nm;
    float m;
    float l[4];
};

// Lazy rescale (guide T13) without a per-tile row max: m is the row max of the
// first tile and moves only when a tile's scores could overflow.  The common path
// computes p = exp2(s - m) and the tile's row sum straight away; a half-row sum
// above 2^13 (or inf / NaN) sends the whole wave to the slow path, which takes the
// row max, moves m, rescales l and O and recomputes the tile.  Every p the common
// path keeps is therefore <= 2^13: exact-range fp16 for the PV operand.  The
// library kernel's tile loop runs the common path only; a block where any wave saw
// such a sum is redone from its first tile by the loop with the slow path.
#define FA2_TILE_SUM_MAX 8192.0f

// LLVM scheduling strategy (__builtin_amdgcn_iglp_opt) for the QK^T and PV regions at
// D = 128; -1 = the default scheduler.  r03 in-process A/Bs (`profiles/r03/ab/figlp/`):
// strategy 0 took C4 (B8_H16_S4096_D128) 1.2-1.5 % faster in two runs, D = 128 at S = 2048
// +-0; at D = 64 every strategy (0-3) lost 5 % at C3, so D = 64 keeps the default.
constexpr int kFwdIglp = 0;

// -m as one opaque 16-register tuple: without the empty asm the compiler
// rematerialises the splat with 16 v_mov before every QK^T chain.
__device__ __forceinline__ f32x16 splat16(float x) {
    f32x16 v = x;
    asm volatile("" : "+v"(v));
    return v;
}

// S^T of one 64-key tile for the wave's MQ query groups (keys on registers, query
// on the lane), relative to m.  Each K fragment read from LDS feeds MQ MFMAs.
// SEED: the chain starts from -m (scores relative to m); otherwise from 0 and the
// softmax subtracts m per score (32-key tiles at D = 128, 16 registers fewer).
template <int D, int MQ, int NKB = 2, bool SEED = true>
__device__ __forceinline__ void fwd_qk(f32x16 (&s)[MQ][NKB], const FwdState<D> (&st)[MQ], const _Float16* Ks,
                                       const FragOffsets<D>& fo) {
    if constexpr (D == 128) __builtin_amdgcn_iglp_opt(kFwdIglp);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        const f16x8 a0 = fo.rowop(Ks, kb * 32, 0);
        const f32x16 zero = {};
#pragma unroll
        for (int g = 0; g < MQ; ++g) s[g][kb] = mfma(a0, st[g].qf[0], SEED ? st[g].nm : zero);
#pragma unroll
        for (int t = 1; t < D / 16; ++t) {
            const f16x8 a = fo.rowop(Ks, kb * 32, t);
#pragma unroll
            for (int g = 0; g < MQ; ++g) s[g][kb] = mfma(a, st[g].qf[t], s[g][kb]);
        }
    }
}

// Row max of a 16*NKB-score register tile as four independent max3 chains.
template <int NKB>
__device__ __forceinline__ float tile_max(const f32x16 (&t)[NKB]) {
    float c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c[k] = fmaxf(t[0][k], t[0][k + 4]);
        c[k] = fmaxf(fmaxf(c[k], t[0][k + 8]), t[0][k + 12]);
#pragma unroll
        for (int kb = 1; kb < NKB; ++kb) {
            c[k] = fmaxf(fmaxf(c[k], t[kb][k]), t[kb][k + 4]);
            c[k] = fmaxf(fmaxf(c[k], t[kb][k + 8]), t[kb][k + 12]);
        }
    }
    return fmaxf(fmaxf(c[0], c[1]), fmaxf(c[2], c[3]));
}

// p = exp2(s - m - sh) of the tile, packed to fp16, with its four partial row sums:
// v_dot2 of the packed tile values against ones (one issue per two scores, and l
// sums exactly the P the PV MFMAs multiply; scalar f32 adds cost one issue per score,
// and float2 chains (v_pk_add_f32) spilled 15 VGPRs at C3 -- r01)
template <bool SHIFT, int NKB = 2>
__device__ __forceinline__ void fwd_exp(const f32x16 (&sacc)[NKB], float sh, f16x8 (&pf)[NKB][2], float (&ls)[4]) {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) pf[kb][i >> 3][i & 7] = to_tile(fast_exp2(SHIFT ? sacc[kb][i] - sh : sacc[kb][i]));
#pragma unroll
    for (int c = 0; c < 4; ++c) ls[c] = 0.f;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = (kb * 8 + j) & 3;
            ls[c] = pair_sum(pf[kb][j >> 2][2 * (j & 3)], pf[kb][j >> 2][2 * (j & 3) + 1], ls[c]);
        }
}

// Online softmax of one tile for the wave's MQ query groups (sacc = s - m) and
// O^T += V^T P^T with the packed scores as the B operand (each V^T fragment feeds MQ
// MFMAs).  first: the wave's first tile (m := its row max).  One slow-path decision
// for all groups keeps the tile a single basic block on the common path.
template <int D, int MQ, bool MASK, int NKB = 2, bool SEED = true>
__device__ __forceinline__ void fwd_softmax_pv(FwdState<D> (&st)[MQ], f32x16 (&sacc)[MQ][NKB], const _Float16* Vs,
                                               const FragOffsets<D>& fo, int k0, int S, int h, bool first) {
    if (MASK) {  // ragged last tile only
#pragma unroll
        for (int g = 0; g < MQ; ++g)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (k0 + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h >= S) sacc[g][kb][i] = -__builtin_inff();
    }
    f16x8 pf[MQ][NKB][2];
    float ls[MQ][4];
    // l += tile sums, O^T += V^T P^T.  Issued inside each branch: joining the paths
    // before it made the register allocator copy O and l on the common path (r01 ISA
    // audit: 29 v_mov per 64-key tile at D = 64; 32 v_mov_b64 + 5 v_mov_b32 per 32-key
    // tile at D = 128); joined after it, the merged values are MFMA results.
    auto accumulate = [&]() {
        if constexpr (D == 128) __builtin_amdgcn_iglp_opt(kFwdIglp);
#pragma unroll
        for (int g = 0; g < MQ; ++g)
#pragma unroll
            for (int c = 0; c < 4; ++c) st[g].l[c] += ls[g][c];
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const f16x8 v = fo.trop(Vs, kb * 32 + 16 * s, b);
#pragma unroll
                    for (int g = 0; g < MQ; ++g) st[g].oacc[b] = mfma(v, pf[g][kb][s], st[g].oacc[b]);
                }
    };
    bool slow = first;
    if (!first) {
        bool bad = false;
#pragma unroll
        for (int g = 0; g < MQ; ++g) {
            fwd_exp<!SEED, NKB>(sacc[g], st[g].m, pf[g], ls[g]);
            const float ts = (ls[g][0] + ls[g][1]) + (ls[g][2] + ls[g][3]);
            bad = bad || !(ts <= FA2_TILE_SUM_MAX);
        }
        slow = __any(bad);
    }
    if (slow) {
#pragma unroll
        for (int g = 0; g < MQ; ++g) {
            const float mx = xor32_max(tile_max<NKB>(sacc[g])) - (SEED ? 0.f : st[g].m);
            const float d = first ? mx : fmaxf(mx, 0.f);
            const float alpha = first ? 0.f : fast_exp2(-d);
            st[g].m += d;
#pragma unroll
            for (int c = 0; c < 4; ++c) st[g].l[c] *= alpha;
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) st[g].oacc[b][i] *= alpha;
            if (SEED) st[g].nm = splat16(-st[g].m);
            fwd_exp<true, NKB>(sacc[g], SEED ? d : st[g].m, pf[g], ls[g]);
        }
        accumulate();
    } else {
        accumulate();
    }
}

// The common-path tile alone (unsplit forward loop): p = exp2(s - m) against the row's current
// m, the tile sums and O^T += V^T P^T, with no rescale branch (no register joins in the
// tile loop).  Returns whether a half-row sum left [0, 2^13] (or went inf / NaN) in any
// lane; the caller then redoes the whole query block with the rescaling loop.
template <int D, int MQ, bool MASK, int NKB = 2, bool SEED = true>
__device__ __forceinline__ bool fwd_softmax_pv_fast(FwdState<D> (&st)[MQ], f32x16 (&sacc)[MQ][NKB], const _Float16* Vs,
                                                    const FragOffsets<D>& fo, int k0, int S, int h) {
    if (MASK) {
#pragma unroll
        for (int g = 0; g < MQ; ++g)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (k0 + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h >= S) sacc[g][kb][i] = -__builtin_inff();
    }
    f16x8 pf[MQ][NKB][2];
    float ls[MQ][4];
    bool bad = false;
#pragma unroll
    for (int g = 0; g < MQ; ++g) {
        fwd_exp<!SEED, NKB>(sacc[g], st[g].m, pf[g], ls[g]);
        const float ts = (ls[g][0] + ls[g][1]) + (ls[g][2] + ls[g][3]);
        bad = bad || !(ts <= FA2_TILE_SUM_MAX);
    }
#pragma unroll
    for (int g = 0; g < MQ; ++g)
#pragma unroll
        for (int c = 0; c < 4; ++c) st[g].l[c] += ls[g][c];
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const f16x8 v = fo.trop(Vs, kb * 32 + 16 * s2, b);
#pragma unroll
                for (int g = 0; g < MQ; ++g) st[g].oacc[b] = mfma(v, pf[g][kb][s2], st[g].oacc[b]);
            }
    return bad;
}

template <int M>
struct MaskTag {
    static constexpr int value = M;
};

template <int D, bool SEED = true>
__device__ __forceinline__ void fwd_init(FwdState<D>& st, const float* Q, long base, int q, int S, int h) {
    const float qscale = FA2_LOG2E / __builtin_sqrtf((float)D);
    // Q fragments (B operand of S^T = K Q^T): lane holds Q[q][16t + 8h + 0..7]
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
        if (q < S) {
            const f32x4* p = reinterpret_cast<const f32x4*>(Q + base + (long)q * D + 16 * t + 8 * h);
            st.qf[t] = to_f16x8(p[0], p[1], qscale);
        } else {
            st.qf[t] = f16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) st.oacc[b][i] = 0.f;
    if (SEED) st.nm = splat16(0.f);
    st.m = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) st.l[c] = 0.f;
}

template <int D>
__device__ __forceinline__ void fwd_store(const FwdState<D>& st, float* O, float* LSE, long base, long lrow, int q,
                                          int S, int h) {
    const float lt = xor32_sum((st.l[0] + st.l[1]) + (st.l[2] + st.l[3]));
    const float inv = 1.f / lt;
    if (q < S) {
        float* orow = O + base + (long)q * D;
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f32x4 v = {st.oacc[b][4 * g] * inv, st.oacc[b][4 * g + 1] * inv, st.oacc[b][4 * g + 2] * inv,
                           st.oacc[b][4 * g + 3] * inv};
                *reinterpret_cast<f32x4*>(orow + 32 * b + 8 * g + 4 * h) = v;
            }
        if (h == 0) LSE[lrow + q] = st.m * FA2_LN2 + __logf(lt);
    }
}

// Grid: BH * ceil(S / (32*NW)) workgroups of 64*NW threads (NW waves x 32 queries).
// (A persistent variant that walks several query blocks per workgroup, with the
// next block's Q prefetched by LDS-DMA and K/V streamed across block seams, cut
// the per-block fixed cost from ~20 to ~16 us at C3 but ran the tile loop ~8 %
// slower back-to-back, a net loss on the bench step -- r01)
//
// The next tile's global loads are issued after the tile's QK^T MFMAs (guide T14:
// issued at the tile start, the eight waves' loads queue on the texture unit and
// stall every wave), its LDS stores after the softmax; Q is loaded and O stored as
// whole rows through LDS (prologue / epilogue).  Waves 4-7 of an 8-wave workgroup
// run at s_setprio 1 for the whole loop (the second-dispatched half loses VALU
// arbitration by age; MI355X_MICROARCH §Two waves per SIMD, item 4: +0.9 %).
//
// NKB 32-key blocks per KV tile (2: 64-key tiles; 1: 32-key tiles, fewer registers
// for D = 128 at 8 waves).

// KS > 1 (small grids): the key range is split over KS wave groups of NQ = NW / KS
// waves.  Wave w handles query rows of slot w % NQ against tiles j·KS + w / NQ;
// each step stages KS tiles.  The groups' (m, l, O) meet in LDS after the loop
// (O = Σ_g 2^(m_g - m) O_g, l likewise) and group 0 stores.  That puts NW waves on
// NQ · 32 query rows, so a grid of few query blocks still covers every SIMD twice.
template <int D, int NW, int NKB = 2, int KS = 1>
__global__ void __launch_bounds__(64 * NW)
fa2_fwd_f16_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                   float* __restrict__ O, float* __restrict__ LSE, int S) {
    constexpr int MQ = 1;            // query groups per wave (2 measured -30 % at D = 32/64: r01)
    constexpr bool SEED = NKB == 2;  // -m seed for 64-key tiles; 32-key tiles subtract m
    constexpr int KT = 32 * NKB;  // keys per tile
    constexpr int NT = 64 * NW;
    constexpr int TILE = KT * D;
    constexpr int QW = 32 * MQ;  // query rows per wave
    static_assert(NW % KS == 0, "key split");
    constexpr int NQ = NW / KS;  // query waves (KS > 1: waves w, w + NQ, ... share rows)
    // key-split merge records: per wave of groups 1..KS-1, O (D/2 floats per lane), m, l
    constexpr int MREC = (D / 2 + 2) * 64;
    constexpr int MERGE = KS > 1 ? 2 * (KS - 1) * NQ * MREC : 0;  // in halves
    // [buf][K | V][KS] tiles; at least one Q block (coalesced prologue) and the merge
    // OVL: the prologue's Q block behind the first K/V buffer, loaded with the first step
    constexpr bool OVL = KS > 1;
    constexpr int QB = (OVL ? 2 * KS * TILE : 0) + 32 * MQ * NQ * D;
    constexpr int SMEM0 = 4 * KS * TILE > QB ? 4 * KS * TILE : QB;
    constexpr int SMEM = SMEM0 > MERGE ? SMEM0 : MERGE;
    __shared__ __attribute__((aligned(16))) _Float16 smem[SMEM];
    __shared__ __attribute__((aligned(16))) float ostage[NQ][32][36];  // per-wave O block stage

    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = KS > 1 ? (tid >> 6) % NQ : tid >> 6;  // query slot of the wave
    const int kg = KS > 1 ? __builtin_amdgcn_readfirstlane((tid >> 6) / NQ) : 0;  // key group
    const int nqb = (S + QW * NQ - 1) / (QW * NQ);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = bid / nqb, qb = bid - bh * nqb;
    const long base = (long)bh * S * D;
    const int q0 = qb * QW * NQ + wave * QW + r;

    FwdState<D> st[MQ];
    FragOffsets<D> fo;
    fo.init(lane);
    // (KS > 1: a step stages KS consecutive tiles as one [KS * KT][D] image per tensor)
    TileStager<D, KT * KS, NT> ks, vs;
    ks.init(K + base, S, tid);
    vs.init(V + base, S, tid);
    const int ntiles = (S + KT - 1) / KT;
    const int last_ragged = (S % KT) ? ntiles - 1 : -1;  // the one tile that needs key masking
    const int nsteps = (ntiles + KS - 1) / KS;
    // Q block (32*NQ rows, one contiguous HBM range) loaded row-coalesced, converted
    // and scaled into LDS, then read back as this wave's B fragments: 1 KB per load
    // instruction instead of 32 rows x 32 B per-lane pieces.  OVL (key split: small
    // grids, where the prologue's round trips are exposed): its loads and the first K/V
    // step's go out together, Q behind the first K/V buffer; else Q first, through the
    // (still idle) K/V buffers.
    {
        _Float16* const qblk = OVL ? smem + 2 * KS * TILE : smem;
        TileStager<D, 32 * MQ * NQ, NT> qst;
        qst.init(Q + base, S, tid);
        qst.load(qb * QW * NQ);
        if constexpr (OVL) {
            ks.load(0);
            vs.load(0);
        }
        qst.store(qblk, FA2_LOG2E / __builtin_sqrtf((float)D), tid);
        if constexpr (OVL) {
            ks.store(smem, 1.f, tid);
            vs.store(smem + KS * TILE, 1.f, tid);
        }
        __syncthreads();
        fwd_init<D, SEED>(st[0], nullptr, 0, S, S, h);  // state only (q >= S: no Q read)
#pragma unroll
        for (int t = 0; t < D / 16; ++t) st[0].qf[t] = fo.rowop(qblk, wave * QW, t);
        __syncthreads();  // every wave has its Q fragments before their buffer is restaged
    }
    // the group's tile within each staged image: folded into the per-lane offsets, so
    // every LDS read keeps a compile-time tile base
    if (KS > 1) fo.shift(kg * TILE);
    if constexpr (!OVL) {
        ks.load(0);
        vs.load(0);
        ks.store(smem, 1.f, tid);
        vs.store(smem + KS * TILE, 1.f, tid);
        __syncthreads();
    }

    if (NW == 8 && __builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
    // one staged step out of the current buffers; the next step's loads after QK^T.
    // redo (wave-uniform): false for a wave that only stages and keeps its state (the
    // restart below recomputes just the waves that saw a spike)
    auto step = [&](const _Float16* Kc, const _Float16* Vc, _Float16* Kn, _Float16* Vn, int j, bool more,
                    bool redo = true) __attribute__((always_inline)) {
        const int jj = j * KS + kg;                          // this wave's tile
        const bool live = (KS == 1 || jj < ntiles) && redo;  // wave-uniform (KS > 1: ragged tail)
        f32x16 sacc[MQ][NKB];
        if (live) fwd_qk<D, MQ, NKB, SEED>(sacc, st, Kc, fo);
        if (more) {
            ks.load((j + 1) * KS * KT);
            vs.load((j + 1) * KS * KT);
        }
        if (live) {
            if (jj == last_ragged) fwd_softmax_pv<D, MQ, true, NKB, SEED>(st, sacc, Vc, fo, jj * KT, S, h, j == 0);
            else fwd_softmax_pv<D, MQ, false, NKB, SEED>(st, sacc, Vc, fo, jj * KT, S, h, j == 0);
        }
        if (more) {
            ks.store(Kn, 1.f, tid);
            vs.store(Vn, 1.f, tid);
        }
        __syncthreads();
    };
    // two steps per trip so every LDS buffer offset is a compile-time immediate
    auto robust_loop = [&](bool redo) __attribute__((always_inline)) {
        for (int j = 0; j < nsteps; j += 2) {
            step(smem, smem + KS * TILE, smem + 2 * KS * TILE, smem + 3 * KS * TILE, j, j + 1 < nsteps, redo);
            if (j + 1 < nsteps)
                step(smem + 2 * KS * TILE, smem + 3 * KS * TILE, smem, smem + KS * TILE, j + 1, j + 2 < nsteps, redo);
        }
    };
    // Tile 0 (each key group's first) sets m (the rescaling step); tiles 1.. run the
    // branch-free common path and only note a sum out of range; if any wave noted one,
    // the whole workgroup restarts the block with the rescaling loop (late score spikes
    // only).  Without the rescale branch in the loop the register allocator keeps O, l
    // and -m in place: r03, in-process A/Bs (profiles/r03/ab/fast/): forward -1.2 ..
    // -1.9 % at C3, C4, C5 and B2_H8_S4096; key-split grids (B2_H8, S = 512 - 2048)
    // fwd + bwd step -1 .. -2 %.
    constexpr bool FWD_FAST = true;
    if constexpr (FWD_FAST) {
        // mt: MaskTag<0>: full tiles only (no masked copy of the tile body to join with,
        // which left ~20 register copies per tile at D = 64); MaskTag<1>: the ragged
        // last tile masked where it comes up
        auto stepf = [&](auto mt, const _Float16* Kc, const _Float16* Vc, _Float16* Kn, _Float16* Vn, int j,
                         bool more) __attribute__((always_inline)) {
            constexpr bool RAG = decltype(mt)::value != 0;
            const int jj = j * KS + kg;                // this wave's tile
            // wave-uniform (KS > 1: ragged tail); full steps (MaskTag<0>) have every group live
            const bool live = KS == 1 || !RAG || jj < ntiles;
            f32x16 sacc[MQ][NKB];
            if (live) fwd_qk<D, MQ, NKB, SEED>(sacc, st, Kc, fo);
            if (more) {
                ks.load((j + 1) * KS * KT);
                vs.load((j + 1) * KS * KT);
            }
            bool b = false;
            if constexpr (RAG) {
                if (live)
                    b = jj == last_ragged ? fwd_softmax_pv_fast<D, MQ, true, NKB, SEED>(st, sacc, Vc, fo, jj * KT, S, h)
                                          : fwd_softmax_pv_fast<D, MQ, false, NKB, SEED>(st, sacc, Vc, fo, jj * KT, S, h);
            } else {
                if (live) b = fwd_softmax_pv_fast<D, MQ, false, NKB, SEED>(st, sacc, Vc, fo, jj * KT, S, h);
            }
            if (more) {
                ks.store(Kn, 1.f, tid);
                vs.store(Vn, 1.f, tid);
            }
            __syncthreads();
            return b;
        };
        step(smem, smem + KS * TILE, smem + 2 * KS * TILE, smem + 3 * KS * TILE, 0, 1 < nsteps);
        // D <= 64: the ragged last tile's step (always the last one) runs after the loop
        // (r03 A/B: B2_H8 fwd S = 512 -7 %, S = 1024 -5 %, C3 -1.2 %); D = 128 keeps it
        // in the loop (peeled, its 32-key-tile loop ran 5.8 % slower at C4)
        constexpr bool PEEL = D <= 64;
        using LoopTag = MaskTag<PEEL ? 0 : 1>;
        // (KS > 1: also a last step where some key group has no tile)
        const int jend = PEEL && (last_ragged >= 0 || ntiles % KS != 0) && nsteps > 1 ? nsteps - 1 : nsteps;
        bool bad = false;
        for (int j = 1; j < jend; j += 2) {
            bad = stepf(LoopTag{}, smem + 2 * KS * TILE, smem + 3 * KS * TILE, smem, smem + KS * TILE, j,
                        j + 1 < nsteps) ||
                  bad;
            if (j + 1 < jend)
                bad = stepf(LoopTag{}, smem, smem + KS * TILE, smem + 2 * KS * TILE, smem + 3 * KS * TILE, j + 1,
                            j + 2 < nsteps) ||
                      bad;
        }
        if (jend < nsteps) {  // j = nsteps - 1 >= 1: its buffers by parity (odd: the second pair)
            _Float16* const kc = (jend & 1) ? smem + 2 * KS * TILE : smem;
            bad = stepf(MaskTag<1>{}, kc, kc + KS * TILE, smem, smem, jend, false) || bad;
        }
        if (__syncthreads_or(bad)) {
            // every wave restages; only the waves that saw a spike reset and recompute (the
            // others' O, l and m never left range and stand as they are)
            const bool redo = __builtin_amdgcn_readfirstlane(__any(bad) ? 1 : 0) != 0;
            if (redo) {
#pragma unroll
                for (int b = 0; b < D / 32; ++b)
#pragma unroll
                    for (int i = 0; i < 16; ++i) st[0].oacc[b][i] = 0.f;  // state only: the Q fragments stay
                if (SEED) st[0].nm = splat16(0.f);
                st[0].m = 0.f;
#pragma unroll
                for (int c = 0; c < 4; ++c) st[0].l[c] = 0.f;
            }
            ks.load(0);
            vs.load(0);
            ks.store(smem, 1.f, tid);
            vs.store(smem + KS * TILE, 1.f, tid);
            __syncthreads();
            robust_loop(redo);
        }
    } else {
        robust_loop(true);
    }
    if constexpr (KS > 1) {
        // Key-split merge (the loop ended on a barrier: the tile buffers are free).
        // Records are lane-linear ([value][lane]), so writes and reads are conflict-free;
        // a group that got no tile (kg >= ntiles) reports m = -inf, weight 0.
        float* mg = reinterpret_cast<float*>(smem);
        if (kg > 0) {
            float* rec = mg + ((kg - 1) * NQ + wave) * MREC;
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) rec[(16 * b + i) * 64 + lane] = st[0].oacc[b][i];
            rec[(D / 2) * 64 + lane] = kg < ntiles ? st[0].m : -__builtin_inff();
            rec[(D / 2 + 1) * 64 + lane] = (st[0].l[0] + st[0].l[1]) + (st[0].l[2] + st[0].l[3]);
        }
        __syncthreads();
        if (kg > 0) return;  // no workgroup barrier follows
        float l = (st[0].l[0] + st[0].l[1]) + (st[0].l[2] + st[0].l[3]);
#pragma unroll
        for (int g = 1; g < KS; ++g) {
            const float* rec = mg + ((g - 1) * NQ + wave) * MREC;
            const float mo = rec[(D / 2) * 64 + lane];
            const float mx = fmaxf(st[0].m, mo);
            const float a = fast_exp2(st[0].m - mx), ao = fast_exp2(mo - mx);
#pragma unroll
            for (int b = 0; b < D / 32; ++b)
#pragma unroll
                for (int i = 0; i < 16; ++i) st[0].oacc[b][i] = st[0].oacc[b][i] * a + rec[(16 * b + i) * 64 + lane] * ao;
            l = l * a + rec[(D / 2 + 1) * 64 + lane] * ao;
            st[0].m = mx;
        }
        st[0].l[0] = l;
        st[0].l[1] = st[0].l[2] = st[0].l[3] = 0.f;
    }
    // O through a wave-private LDS stage, one 32x32 block at a time, stored as whole
    // 128-B row segments (8 rows per instruction) instead of 16-B pieces of 32 rows
    {
        const float lt = xor32_sum((st[0].l[0] + st[0].l[1]) + (st[0].l[2] + st[0].l[3]));
        const float inv = 1.f / lt;
        const int qrow0 = qb * QW * NQ + wave * QW;  // first row of this wave
        float(*os)[36] = ostage[wave];
#pragma unroll
        for (int b = 0; b < D / 32; ++b) {
#pragma unroll
            for (int i = 0; i < 16; ++i) os[r][(i & 3) + 8 * (i >> 2) + 4 * h] = st[0].oacc[b][i] * inv;
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int row = 8 * s4 + (lane >> 3), c4 = (lane & 7) * 4;
                const f32x4 v = *reinterpret_cast<const f32x4*>(&os[row][c4]);
                if (qrow0 + row < S) *reinterpret_cast<f32x4*>(O + base + (long)(qrow0 + row) * D + 32 * b + c4) = v;
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (h == 0 && q0 < S) LSE[(long)bh * S + q0] = st[0].m * FA2_LN2 + __logf(lt);
    }
}

#ifndef CUPY_INLINE_COMPILE
// ---------------------------------------------------------------------------
// Hand-scheduled forward (D = 64, 128; S % 64 == 0, S >= 128), r05.
// ---------------------------------------------------------------------------
// One workgroup = 4 waves = 256 query rows, one wave per SIMD with the whole register
// file; each wave keeps 64 query rows as two 32-row chains and runs, per 64-key tile,
// four MFMA phases with the other chain's softmax placed in their gaps (QKᵀ of A |
// softmax of B, PV of B | softmax of A, QKᵀ of B | softmax of A, PV of A | softmax of
// B).  The tile loop is the generated inline-asm block of fa2_fwd_hs.inc
// (gen/gen_fwd_hs.py: register map, gap schedule, counted waits, hazard states); this
// kernel stages the Q block and the first K/V tile, hands the asm its per-lane LDS
// offsets, staging offsets and buffer descriptors, and finishes with the O rows the
// asm leaves (unnormalised, fp32) in an LDS stage.  Same results as the reference's
// flash_attention2_forward_kernel_fp16 (kernel_fa2_optimized_f16.cu:97-330): the m
// reference point is the first tile's row max, every later tile's half-row sums are
// checked against 2^13 (fp16 range of P), and a block where any was out of range (or
// NaN) is recomputed by the robust compiler-scheduled loop below.
}  // namespace fa2f16
#include "fa2_fwd_hs.inc"
namespace fa2f16 {

// Split partials (KSPLIT = P > 1 key chunks of L = S / P keys per head): chunk c of head
// bh leaves, per query row, its unnormalised O row at part + ((c*BH + bh)*S + row)*D and
// (m, l) -- the chunk's row reference (log2 units) and row sum -- at
// part + P*BH*S*D + ((c*BH + bh)*S + row)*2; fa2_fwd_merge_kernel combines them.
template <int D>
__device__ __forceinline__ void fwd_store_part(const FwdState<D>& st, float* part_o, float* part_ml, int q, int S,
                                               int h) {
    const float lt = xor32_sum((st.l[0] + st.l[1]) + (st.l[2] + st.l[3]));
    if (q < S) {
        float* orow = part_o + (long)q * D;
#pragma unroll
        for (int b = 0; b < D / 32; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f32x4 v = {st.oacc[b][4 * g], st.oacc[b][4 * g + 1], st.oacc[b][4 * g + 2], st.oacc[b][4 * g + 3]};
                *reinterpret_cast<f32x4*>(orow + 32 * b + 8 * g + 4 * h) = v;
            }
        if (h == 0) *reinterpret_cast<float2*>(part_ml + 2L * q) = make_float2(st.m, lt);
    }
}

template <int D>
__global__ void __launch_bounds__(256, 1)
fa2_fwd_hs_kernel(const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
                  float* __restrict__ O, float* __restrict__ LSE, int S, int P, float* __restrict__ part) {
    static_assert(D == 64 || D == 128, "hand-scheduled forward: D = 64 or 128");
    constexpr int KT = 64, TB = KT * D;  // halves per tile image
    constexpr int OST = D + 4;           // O stage row stride (floats), as in the generator
    constexpr int LDSB = D == 64 ? FA2_HS_LDS_D64 : FA2_HS_LDS_D128;
    __shared__ __attribute__((aligned(16))) _Float16 smem[LDSB / 2];
    __shared__ float invl[256];

    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nqb = (S + 255) / 256;
    // workgroup -> (head, key chunk, query block): the query blocks of one chunk are
    // consecutive, so after the XCD remap they share one L2's copy of the chunk's K/V
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = bid % nqb, bc = bid / nqb;
    const int bh = bc / P, kc = bc - bh * P;
    const long base = (long)bh * S * D;
    const int qrow0 = qb * 256;
    const int L = S / P;            // keys of this workgroup's chunk (S itself when P = 1)
    const long kbase = base + (long)kc * L * D;
    // P > 1: this chunk's partial rows (see fwd_store_part)
    const long prow = ((long)kc * (gridDim.x / (P * nqb)) + bh) * S;
    float* part_o = P > 1 ? part + prow * D : nullptr;
    float* part_ml = P > 1 ? part + (long)gridDim.x / nqb * S * D + prow * 2 : nullptr;

    // Q block (256 rows, scaled by log2(e)/sqrt(D)) -> LDS [4TB, 8TB) halves; K(0), V(0)
    // -> slot 0 of the K and V rings ([0, TB) and [2TB, 3TB))
    TileStager<D, KT, 256> ks, vs;
    ks.init(K + kbase, L, tid);
    vs.init(V + kbase, L, tid);
    {
        TileStager<D, 256, 256> qst;
        qst.init(Q + base, S, tid);
        qst.load(qrow0);
        ks.load(0);
        vs.load(0);
        qst.store(smem + 4 * TB, FA2_LOG2E / __builtin_sqrtf((float)D), tid);
        ks.store(smem, 1.f, tid);
        vs.store(smem + 2 * TB, 1.f, tid);
    }
    __syncthreads();

    FragOffsets<D> fo;
    fo.init(lane);
    int hs_ka[D / 16], hs_va[D / 32][2], hs_vo[D / 32];
#pragma unroll
    for (int t = 0; t < D / 16; ++t) hs_ka[t] = fo.row[t] * 2;
#pragma unroll
    for (int b = 0; b < D / 32; ++b) {
        hs_va[b][0] = fo.tr[b][0] * 2;
        hs_va[b][1] = fo.tr[b][1] * 2;
    }
#pragma unroll
    for (int c = 0; c < D / 32; ++c) hs_vo[c] = ks.voff[c];
    const int hs_lo = ks.loff[0] * 2;
    const int hs_oa = ((wave * 64 + r) * OST + 4 * h) * 4;
    const __amdgpu_buffer_rsrc_t hs_rsk = ks.rs, hs_rsv = vs.rs;
    const int hs_qb = __builtin_amdgcn_readfirstlane(4 * TB * 2 + wave * 64 * D * 2);
    int hs_cnt = __builtin_amdgcn_readfirstlane(L / KT - 1);
    int hs_goff = __builtin_amdgcn_readfirstlane(KT * D * 4);
    float hs_m0, hs_m1, hs_l0, hs_l1;
    unsigned long long hs_flag;
    if constexpr (D == 64) {
#ifdef FA2_TILE_BF16
        asm volatile(FA2_HS_ASM_D64_BF16 : FA2_HS_OUTPUTS_D64 : FA2_HS_INPUTS_D64 : FA2_HS_CLOBBERS_D64);
#else
        asm volatile(FA2_HS_ASM_D64_F16 : FA2_HS_OUTPUTS_D64 : FA2_HS_INPUTS_D64 : FA2_HS_CLOBBERS_D64);
#endif
    } else {
#ifdef FA2_TILE_BF16
        asm volatile(FA2_HS_ASM_D128_BF16 : FA2_HS_OUTPUTS_D128 : FA2_HS_INPUTS_D128 : FA2_HS_CLOBBERS_D128);
#else
        asm volatile(FA2_HS_ASM_D128_F16 : FA2_HS_OUTPUTS_D128 : FA2_HS_INPUTS_D128 : FA2_HS_CLOBBERS_D128);
#endif
    }

    // hs_flag is a scalar (wave-uniform): this wave saw a half-row sum out of range
    const bool wave_bad = hs_flag != 0;
    const bool any_bad = __syncthreads_or(wave_bad);
    if (!wave_bad && P > 1) {
        // a key chunk's partial: the unnormalised O rows from the stage, (m, l) per row
        const float lt0 = xor32_sum(hs_l0), lt1 = xor32_sum(hs_l1);
        const int q0 = qrow0 + wave * 64 + r;
        if (h == 0) {
            if (q0 < S) *reinterpret_cast<float2*>(part_ml + 2L * q0) = make_float2(hs_m0, lt0);
            if (q0 + 32 < S) *reinterpret_cast<float2*>(part_ml + 2L * (q0 + 32)) = make_float2(hs_m1, lt1);
        }
        constexpr int LPR = D / 4, RPI = 64 / LPR;
        const float* os = reinterpret_cast<const float*>(smem);
#pragma unroll 4
        for (int rr = 0; rr < 64; rr += RPI) {
            const int row = wave * 64 + rr + lane / LPR, c4 = (lane % LPR) * 4;
            const f32x4 v = *reinterpret_cast<const f32x4*>(os + row * OST + c4);
            if (qrow0 + row < S) *reinterpret_cast<f32x4*>(part_o + (long)(qrow0 + row) * D + c4) = v;
        }
    } else if (!wave_bad) {
        // O rows [wave*64 + c*32 + q][OST] (unnormalised) are in the stage; l is per lane
        // half: the xor-32 sum is the row's total
        const float lt0 = xor32_sum(hs_l0), lt1 = xor32_sum(hs_l1);
        if (h == 0) {
            invl[wave * 64 + r] = 1.f / lt0;
            invl[wave * 64 + 32 + r] = 1.f / lt1;
            const int q0 = qrow0 + wave * 64 + r;
            if (q0 < S) LSE[(long)bh * S + q0] = hs_m0 * FA2_LN2 + __logf(lt0);
            if (q0 + 32 < S) LSE[(long)bh * S + q0 + 32] = hs_m1 * FA2_LN2 + __logf(lt1);
        }
        __builtin_amdgcn_wave_barrier();
        // whole rows: D/4 lanes per row, 16-B pieces
        constexpr int LPR = D / 4, RPI = 64 / LPR;
        const float* os = reinterpret_cast<const float*>(smem);
#pragma unroll 4
        for (int rr = 0; rr < 64; rr += RPI) {
            const int row = wave * 64 + rr + lane / LPR, c4 = (lane % LPR) * 4;
            const f32x4 v = *reinterpret_cast<const f32x4*>(os + row * OST + c4) * invl[row];
            if (qrow0 + row < S) *reinterpret_cast<f32x4*>(O + base + (long)(qrow0 + row) * D + c4) = v;
        }
    }
    if (!any_bad) return;
    // Robust path (a late score spike in some wave's rows): only the flagged waves
    // recompute, both chains in ONE pass over the head's K/V with the rescaling loop
    // (first tile sets m, later tiles move it when their sums leave range); the other
    // waves have stored their rows above and only help stage the tiles.  The barrier
    // keeps the restaging from overwriting an O stage another wave still reads.
    __syncthreads();
    FwdState<D> st[2];
    const int q = qrow0 + wave * 64 + r;
    if (wave_bad) {
        fwd_init<D>(st[0], Q, base, q, S, h);
        fwd_init<D>(st[1], Q, base, q + 32, S, h);
    }
    const int ntiles = L / KT;
#pragma unroll 1
    for (int j = 0; j < ntiles; ++j) {
        ks.load(j * KT);
        vs.load(j * KT);
        if (j) __syncthreads();  // the previous tile's reads are done
        ks.store(smem, 1.f, tid);
        vs.store(smem + TB, 1.f, tid);
        __syncthreads();
        if (wave_bad) {
            f32x16 sacc[2][2];
            fwd_qk<D, 2, 2, true>(sacc, st, smem, fo);
            fwd_softmax_pv<D, 2, false, 2, true>(st, sacc, smem + TB, fo, j * KT, L, h, j == 0);
        }
    }
    if (wave_bad && P > 1) {
        fwd_store_part<D>(st[0], part_o, part_ml, q, S, h);
        fwd_store_part<D>(st[1], part_o, part_ml, q + 32, S, h);
    } else if (wave_bad) {
        fwd_store<D>(st[0], O, LSE, base, (long)bh * S, q, S, h);
        fwd_store<D>(st[1], O, LSE, base, (long)bh * S, q + 32, S, h);
    }
}

// Merge of the P key-chunk partials of fa2_fwd_hs_kernel (layout at fwd_store_part), in
// chunk order (deterministic): M = max m_c, w_c = 2^(m_c - M), O = sum w_c O_c / sum w_c l_c,
// LSE = M ln 2 + ln(sum w_c l_c).  One thread per 4 columns of a row.
template <int D>
__global__ void __launch_bounds__(256)
fa2_fwd_merge_kernel(const float* __restrict__ part, int P, long rows, float* __restrict__ O,
                     float* __restrict__ LSE) {
    constexpr int C4 = D / 4;
    const long x = (long)blockIdx.x * 256 + threadIdx.x;
    if (x >= rows * C4) return;
    const long row = x / C4;
    const int c4 = (int)(x - row * C4) * 4;
    const float2* ml = reinterpret_cast<const float2*>(part + (long)P * rows * D);
    float M = -__builtin_inff();
    for (int c = 0; c < P; ++c) M = fmaxf(M, ml[c * rows + row].x);
    float l = 0.f;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < P; ++c) {
        const float2 e = ml[c * rows + row];
        const float w = exp2f(e.x - M);
        l += w * e.y;
        o += w * *reinterpret_cast<const f32x4*>(part + (c * rows + row) * D + c4);
    }
    *reinterpret_cast<f32x4*>(O + row * D + c4) = o * (1.f / l);
    if (c4 == 0) LSE[row] = M * FA2_LN2 + __logf(l);
}
#endif  // CUPY_INLINE_COMPILE

// ---- CuPy face: the reference harness's launch geometry (grid B*H*ceil(S/32),
// block 256, test_flash_attention2.py:278-281 / kernel_fa2_optimized_f16.cu:401),
// fp16 tiles on MFMA like the library kernel.  A workgroup owns 32 query rows;
// its 64-key tiles are dealt to the 4 waves round-robin (tile j to wave j % 4).
// Each wave stages K, then V, of its tile into a private LDS buffer (LDS order
// within one wave needs no barrier), so the loop has no workgroup barrier; the
// four partial (m, l, O) states are merged through LDS at the end.
template <int D>
__device__ __forceinline__ void fwd_compat_body(const float* __restrict__ Q, const float* __restrict__ K,
                                                const float* __restrict__ V, float* __restrict__ O,
                                                float* __restrict__ LSE, int BH, int S, _Float16* lds,
                                                float (*mrg)[4][32]) {
    constexpr int KT = 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int nqb = (S + 31) / 32;
    const int bh = blockIdx.x / nqb, qb = blockIdx.x - bh * nqb;
    if (bh >= BH) return;
    const long base = (long)bh * S * D;
    const int q = qb * 32 + r;
    _Float16* buf = lds + wave * KT * D;

    FwdState<D> st[1];
    fwd_init<D>(st[0], Q, base, q, S, h);
    FragOffsets<D> fo;
    fo.init(lane);
    TileStager<D, KT, 64> ks, vs;
    ks.init(K + base, S, lane);
    vs.init(V + base, S, lane);
    const int nt = (S + KT - 1) / KT;
    for (int j = wave; j < nt; j += 4) {
        ks.load(j * KT);
        ks.store(buf, 1.f, lane);
        f32x16 sacc[1][2];
        fwd_qk<D, 1>(sacc, st, buf, fo);
        vs.load(j * KT);
        vs.store(buf, 1.f, lane);  // after this wave's K reads (in-order LDS within a wave)
        if ((j + 1) * KT > S) fwd_softmax_pv<D, 1, true>(st, sacc, buf, fo, j * KT, S, h, j == wave);
        else fwd_softmax_pv<D, 1, false>(st, sacc, buf, fo, j * KT, S, h, j == wave);
    }
    // merge: O = sum_w 2^(m_w - M) O_w / sum_w 2^(m_w - M) l_w, M = max_w m_w
    const float lw = xor32_sum((st[0].l[0] + st[0].l[1]) + (st[0].l[2] + st[0].l[3]));
    __syncthreads();
    float* ow = reinterpret_cast<float*>(lds) + wave * 32 * D;  // [q][d] fp32 per wave
#pragma unroll
    for (int b = 0; b < D / 32; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) ow[r * D + 32 * b + (i & 3) + 8 * (i >> 2) + 4 * h] = st[0].oacc[b][i];
    if (h == 0) {
        mrg[0][wave][r] = wave < nt ? st[0].m : -__builtin_inff();
        mrg[1][wave][r] = lw;
    }
    __syncthreads();
    const float* of = reinterpret_cast<const float*>(lds);
    for (int x = tid; x < 32 * D; x += 256) {
        const int row = x / D, d = x - row * D;
        if (qb * 32 + row >= S) continue;
        const float M = fmaxf(fmaxf(mrg[0][0][row], mrg[0][1][row]), fmaxf(mrg[0][2][row], mrg[0][3][row]));
        float num = 0.f, den = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const float c = fast_exp2(mrg[0][w][row] - M);
            num += c * of[(w * 32 + row) * D + d];
            den += c * mrg[1][w][row];
        }
        O[base + (long)(qb * 32 + row) * D + d] = num / den;
        if (d == 0) LSE[(long)bh * S + qb * 32 + row] = M * FA2_LN2 + __logf(den);
    }
}

}  // namespace fa2f16

#ifndef CUPY_INLINE_COMPILE
namespace fa2 {

// KS > 1: NW / KS query waves per workgroup (D = 64: 32-key tiles -- with 64-key
// tiles the KS-tile staging registers spill)
// nkb_req: a FWD_NKB override (0 = none); an instance of other tiles is an error, never
// a silent launch of the plan the override asked to leave
template <int D, int NW, int KS = 1, int NKB = (KS == 1 || D <= 32 ? 2 : 1)>
static hipError_t fwd_f16_launch(const float* q, const float* k, const float* v, float* o, float* lse, int bh, int S,
                                 hipStream_t stream, int nkb_req) {
    if (nkb_req && nkb_req != NKB) return hipErrorInvalidValue;
    const int nqb = (S + 32 * (NW / KS) - 1) / (32 * (NW / KS));
    const long grid = (long)bh * nqb;
    if (grid <= 0 || grid > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f16::fa2_fwd_f16_kernel<D, NW, NKB, KS>), dim3((unsigned)grid), dim3(64 * NW), 0, stream, q, k,
                       v, o, lse, S);
    return hipGetLastError();
}

// P > 1: each head's keys in P chunks of S / P (a multiple of 64, >= 128) on their own
// workgroups, partials in `part` (P * bh * S * (D + 2) floats), then the merge pass
template <int D>
static hipError_t fwd_hs_launch(const float* q, const float* k, const float* v, float* o, float* lse, int bh, int S,
                                hipStream_t stream, int P = 1, float* part = nullptr) {
    if (P < 1 || S % (64 * P) || S / P < 128 || (P > 1 && !part)) return hipErrorInvalidValue;
    const long grid = (long)bh * ((S + 255) / 256) * P;
    if (grid <= 0 || grid > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f16::fa2_fwd_hs_kernel<D>), dim3((unsigned)grid), dim3(256), 0, stream, q, k, v, o, lse, S,
                       P, part);
    if (P == 1) return hipGetLastError();
    const long rows = (long)bh * S, threads = rows * (D / 4);
    hipLaunchKernelGGL((fa2f16::fa2_fwd_merge_kernel<D>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       stream, part, P, rows, o, lse);
    return hipGetLastError();
}

// Key chunks per head for a grid of `g` 256-row workgroups that leaves CUs idle: the
// most chunks (a power of two, at most 4) that keep the grid within one workgroup per
// CU and chunks of at least 1024 keys (D = 64) / 256 keys (D = 128), for heads of at
// least 4096 / 1024 keys; 1 where no split applies.  r06 in-process A/B of the forward
// (profiles/r06/split/), unsplit small-grid plan -> split:
//   D = 64:  B1_H2_S4096 38.2 -> 26.9 us (P = 4), B1_H4_S4096 39.7 -> 34.2 (4),
//            B1_H2_S8192 74.3 -> 46.0 (4); P = 2 (B1_H8_S4096) and S = 2048 at 4-16 heads
//            tie or lose 3-20 % (the merge pass and the partial rows' traffic grow with
//            the workgroups while the unsplit workgroups stream only 2048 keys);
//   D = 128: the small-grid plans are weaker (4 / 8 waves of ~400 VGPRs): B1_H2_S1024
//            31.8 -> 20.0 (4), B1_H2_S2048 57.6 -> 27.5 (4), B1_H8_S2048 59.8 -> 37.2 (4),
//            B2_H8_S2048 66.9 -> 51.1 (2), B1_H8_S4096 124.7 -> 78.2 (2), B2_H8_S1024
//            33.8 -> 30.8 (4); S = 512 loses (19.0 -> 20.9).
static int fwd_split_auto(int D, long g, int S) {
    // D = 64 also at S >= 2048 on grids of <= 16 blocks (2 heads): 20.1 -> 17.9 us at
    // B1_H2_S2048 (P = 4), where the split backward runs too (§6 of DESIGN.md)
    const bool tiny = D == 64 && S >= 2048 && g <= 16;
    const int min_s = D == 128 ? 1024 : 4096, min_chunk = D == 128 ? 256 : tiny ? 512 : 1024;
    if (S < min_s && !tiny) return 1;
    const long ncu = cu_count();
    int P = 1;
    while (P < 4 && g * (2 * P) <= ncu && S % (64 * 2 * P) == 0 && S / (2 * P) >= min_chunk) P *= 2;
    return D == 64 && P < 4 ? 1 : P;
}

template <int D>
static hipError_t fwd_f16_dispatch(const float* q, const float* k, const float* v, float* o, float* lse, int bh, int S,
                                   hipStream_t stream) {
    if constexpr (D == 64 || D == 128) {
        // hand-scheduled kernel (r05): full 64-key tiles only, and a grid of at least one
        // 256-row workgroup per CU (smaller grids keep the key-split plans below).
        // FWD_HS (tests and tools): 1 forces it (an error where it cannot serve), 0 disables it.
        // (Its 16x16x32 form lost in r05: C3 +3.6 %, B2_H8_S4096 +4.7 %, C4 +0.8 %, in-process,
        // profiles/r05/fwd16/: the forward is issue-bound and 16x16x32 halves the issue room
        // per MFMA cycle)
        const int hs = tune_knob("FWD_HS", -1);
        const bool fits = S % 64 == 0 && S >= 128;
        const bool forced_other = tune_knob("FWD_WAVES", 0) || tune_knob("FWD_KS", 0) || tune_knob("FWD_NKB", 0);
        // a forced FWD_HS the plan cannot take (shape, or other plan knobs) is an error
        if (hs == 1 && (!fits || forced_other)) return hipErrorInvalidValue;
        const long g = (long)bh * ((S + 255) / 256);
        // FWD_SPLIT (tests and tools): P >= 2 forces P key chunks per head on the
        // hand-scheduled kernel (an error where it cannot serve: shape, other plan knobs,
        // FWD_HS = 0, or no scratch -- a stream being captured), 1 disables the split,
        // 0 = auto (grids below one workgroup per CU, fwd_split_auto)
        const int split = tune_knob("FWD_SPLIT", 0);
        if (split < 0) return hipErrorInvalidValue;
        if (split >= 2 && (!fits || forced_other || hs == 0 || S % (64 * split) || S / split < 128))
            return hipErrorInvalidValue;
        int P = split >= 2 ? split : 1;
        if (split == 0 && fits && hs < 0 && !forced_other && g < cu_count()) P = fwd_split_auto(D, g, S);
        if (P > 1) {
            float* part = static_cast<float*>(stream_scratch(stream, sizeof(float) * P * (size_t)bh * S * (D + 2)));
            if (part) return fwd_hs_launch<D>(q, k, v, o, lse, bh, S, stream, P, part);
            if (split >= 2) return hipErrorInvalidValue;
        }
        if (fits && (hs == 1 || (hs < 0 && !forced_other && g >= cu_count())))
            return fwd_hs_launch<D>(q, k, v, o, lse, bh, S, stream);
    } else {
        // no hand-scheduled kernel at this D
        if (tune_knob("FWD_HS", -1) == 1 || tune_knob("FWD_SPLIT", 0) >= 2) return hipErrorInvalidValue;
    }
    // 8 waves (2 per SIMD) where the registers allow it; D = 128 runs 4 waves of
    // ~400 VGPRs (8 would spill and exceed the LDS budget with the Q stages)
    // (MQ = 2, two 32-row query groups per wave at 4 waves / 1 per SIMD, measured
    // 30 % slower than 8 waves x 1 group at D = 32 and 64 -- r01)
    // Launch-plan overrides (fa2_tune_set, tests and tools only): FWD_WAVES (0 = auto_waves
    // over the grid of 32-query wave units), FWD_KS.
    const long units = (long)bh * ((S + 31) / 32);
    int nw = tune_knob("FWD_WAVES", 0);
    // Key groups per workgroup (0 = auto).  Small grids split the key range over wave
    // groups instead of shrinking the workgroup (r01, B2_H8_D64 fwd: S = 512 12.4 -> 9.9
    // us, S = 1024 21.4 -> 15.4; r02: KS = 2 at 8 waves on B2_H8_S2048, step 100.6 ->
    // 99.3 us); r04 picks the split by workgroup rounds (below).
    int ks = tune_knob("FWD_KS", 0);
    // FWD_NKB (0 = auto): 32-key (1) or 64-key (2) tiles of a key-split plan
    int nkb = tune_knob("FWD_NKB", 0);
    if (nkb < 0 || nkb > 2) return hipErrorInvalidValue;
    if (ks == 0 && nw == 0 && D <= 64 && units < 8L * cu_count()) {
        // D <= 64 on fewer than 8 blocks of 32 rows per CU: the fewest query rows per
        // workgroup whose grid still runs in ONE round of workgroups (one per CU; every
        // workgroup streams its head's whole K/V, so a second round costs a whole
        // workgroup time): 32 rows (4 waves, KS = 4), 64 (8 waves, KS = 4), 128 (8
        // waves, KS = 2), else the unsplit 256-row plan.  r04 (in-process A/B,
        // profiles/r04/nkb/): B2_H8_S1500 fwd 31.5 -> 19.1 us (the previous rule took
        // KS = 4 on 64 rows: 376 workgroups, two rounds); S = 512 / 1024 / 2048 and
        // B4_H8_S1024 pick the plans they had.  D = 32 (which ran unsplit 4-wave
        // workgroups at 4-8 blocks per CU): S = 1500 20.0 -> 14.4 us, S = 2048 21.1 ->
        // 17.5, S = 3000 38.3 -> 37.6 (profiles/r04/d32/).
        const long ncu = cu_count();
        if (units <= ncu) {
            ks = 4, nw = 4;
        } else if ((units + 1) / 2 <= ncu) {
            ks = 4, nw = 8;
        } else if ((units + 3) / 4 <= ncu) {
            ks = 2, nw = 8;
        } else {
            nw = 8;
        }
    }
    // D = 128 on small grids: 4 waves up to one 32-row block per CU, else 8 -- fewer,
    // larger workgroups than auto_waves' 2-wave ones, each streaming its head's K/V once
    // for more rows (r04, B2_H8 D = 128 fwd: S = 512 21.0 -> 19.2 us, 1024 37.5 -> 32.9,
    // 1500 56.7 -> 47.0, 2048 65.9 -> 61.8; profiles/r04/d128/)
    if (ks == 0 && nw == 0 && D == 128 && units < 8L * cu_count()) nw = units <= cu_count() ? 4 : 8;
    if (nw == 0) nw = auto_waves(units, 8);
    if constexpr (D <= 64) {
        // KS = 2 at 8 waves on 64-key tiles (D = 64, r04: 249 VGPRs, no spill; twice the
        // MFMAs per barrier of the 32-key tiles): B2_H8_S2048 fwd 29.6 -> 25.4 us, step
        // 99.1 -> 95.7; B4_H8_S1024 fwd 18.1 -> 15.8; S = 1500 22.3 -> 19.1
        // (profiles/r04/nkb/).  KS = 4 keeps 32-key tiles at 8 waves (64-key tiles spill).
        if (ks == 2 && nw == 8 && nkb != 1) return fwd_f16_launch<D, 8, 2, 2>(q, k, v, o, lse, bh, S, stream, nkb);
        if (ks == 2 && nw == 8) return fwd_f16_launch<D, 8, 2, 1>(q, k, v, o, lse, bh, S, stream, nkb);
        if (ks == 4 && nw == 4 && nkb == 2) return fwd_f16_launch<D, 4, 4, 2>(q, k, v, o, lse, bh, S, stream, nkb);
        if (ks == 4 && nw == 8) return fwd_f16_launch<D, 8, 4>(q, k, v, o, lse, bh, S, stream, nkb);
        if (ks == 4 && nw == 4) return fwd_f16_launch<D, 4, 4>(q, k, v, o, lse, bh, S, stream, nkb);
        if (ks == 2 && nw == 4) return fwd_f16_launch<D, 4, 2>(q, k, v, o, lse, bh, S, stream, nkb);
    }
    if constexpr (D <= 64) {
        if (nw == 8) return fwd_f16_launch<D, 8>(q, k, v, o, lse, bh, S, stream, nkb);
    } else {
        // D = 128 at 8 waves only with 32-key tiles (64-key tiles spill)
        if (nw == 8) return fwd_f16_launch<D, 8, 1, 1>(q, k, v, o, lse, bh, S, stream, nkb);
    }
    if (nw == 2) return fwd_f16_launch<D, 2>(q, k, v, o, lse, bh, S, stream, nkb);
    return fwd_f16_launch<D, 4>(q, k, v, o, lse, bh, S, stream, nkb);
}

hipError_t FA2_TILE_LAUNCH(launch_forward)(int D, const float* q, const float* k, const float* v, float* o, float* lse, int bh,
                              int S, hipStream_t stream) {
    if (bh <= 0 || S <= 0) return hipErrorInvalidValue;
    switch (D) {
        case 32: return fwd_f16_dispatch<32>(q, k, v, o, lse, bh, S, stream);
        case 64: return fwd_f16_dispatch<64>(q, k, v, o, lse, bh, S, stream);
        case 128: return fwd_f16_dispatch<128>(q, k, v, o, lse, bh, S, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace fa2

// Host API with the reference's semantics (kernel_fa2_optimized_f16.cu:353-430):
// host buffers in, device alloc + H2D, timed launch, D2H, free.
template <int head_dim>
void FA2_TILE_HOST(host_flash_attention2_forward)(const float* h_Q, const float* h_K, const float* h_V, float* h_O,
                                        float* h_logsumexp, int batch_size, int seq_len, int num_heads,
                                        TimerManager* tm) {
    const size_t n = (size_t)batch_size * num_heads * seq_len * head_dim;
    const size_t nl = (size_t)batch_size * num_heads * seq_len;
    float *dq, *dk, *dv, *dout, *dl;
    HIP_CHECK(hipMalloc(&dq, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dk, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dv, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dout, n * sizeof(float)));
    HIP_CHECK(hipMalloc(&dl, nl * sizeof(float)));
    HIP_CHECK(hipMemcpy(dq, h_Q, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dk, h_K, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dv, h_V, n * sizeof(float), hipMemcpyHostToDevice));
    tm->Start();
    HIP_CHECK(fa2::FA2_TILE_LAUNCH(launch_forward)(head_dim, dq, dk, dv, dout, dl, batch_size * num_heads, seq_len, nullptr));
    tm->Stop();
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy(h_O, dout, n * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(h_logsumexp, dl, nl * sizeof(float), hipMemcpyDeviceToHost));
    HIP_CHECK(hipFree(dq));
    HIP_CHECK(hipFree(dk));
    HIP_CHECK(hipFree(dv));
    HIP_CHECK(hipFree(dout));
    HIP_CHECK(hipFree(dl));
}
template void FA2_TILE_HOST(host_flash_attention2_forward)<32>(const float*, const float*, const float*, float*, float*, int,
                                                     int, int, TimerManager*);
template void FA2_TILE_HOST(host_flash_attention2_forward)<64>(const float*, const float*, const float*, float*, float*, int,
                                                     int, int, TimerManager*);
template void FA2_TILE_HOST(host_flash_attention2_forward)<128>(const float*, const float*, const float*, float*, float*, int,
                                                      int, int, TimerManager*);
#else
// CuPy face (same symbol as kernel_fa2_optimized_f16.cu:432-448).  The reference
// hard-wires D = 64 here; head_dim is honoured instead (32, 64, 128).  Static LDS
// is 64 KB, so the harness's dynamic bytes ((3*32*D + 32*32 + 3*32)*4) still fit
// inside the 160 KiB a workgroup may own at every supported D.
extern "C" __global__ void __launch_bounds__(256)
flash_attention2_forward_kernel_wrapper(const float* query, const float* key, const float* value, float* output,
                                        float* logsumexp, const int batch_size, const int num_heads,
                                        const int seq_len, const int head_dim) {
    __shared__ __attribute__((aligned(16))) _Float16 lds[4 * 64 * 128];
    __shared__ float mrg[2][4][32];
    const int bh = batch_size * num_heads;
    if (head_dim == 64)
        fa2f16::fwd_compat_body<64>(query, key, value, output, logsumexp, bh, seq_len, lds, mrg);
    else if (head_dim == 32)
        fa2f16::fwd_compat_body<32>(query, key, value, output, logsumexp, bh, seq_len, lds, mrg);
    else if (head_dim == 128)
        fa2f16::fwd_compat_body<128>(query, key, value, output, logsumexp, bh, seq_len, lds, mrg);
}
#endif  // CUPY_INLINE_COMPILE
