import re
p = 'cuda-flash-attention_amd/kernels/f-attn2-backward_f16.cu'
s = open(p).read()


def rep(a, b, count=1):
    global s
    n = s.count(a)
    if n != count:
        raise SystemExit(f"pattern found {n}x (want {count}): {a[:80]!r}")
    s = s.replace(a, b)


def cut(a, b, keep_b=True):
    """remove from the start of a up to (not including) b"""
    global s
    i = s.index(a)
    j = s.index(b, i)
    s = s[:i] + s[j:]


rep('''#include "f-attn2.cuh"
#ifdef FA2_STAMPS
#include <cstdio>
#include <vector>
#endif
#endif''', '''#include "f-attn2.cuh"
#endif''')
# FA2_DS_PK: the packed form is the fp16 build's only form
rep('''// dS = P * (dP - Δ) for a pair of scores, as tile values.  FA2_DS_PK (fp16 tiles):
// the product of the already-packed fp16 P and the packed (dP - Δ) (v_cvt_pk +
// v_pk_mul_f16: one issue per score fewer than two f32 products and a conversion);
// else the f32 products, rounded once.
#ifndef FA2_DS_PK
#define FA2_DS_PK 1
#endif''', '''// dS = P * (dP - Δ) for a pair of scores, as tile values.  fp16 tiles: the product
// of the already-packed fp16 P and the packed (dP - Δ) (v_cvt_pk + v_pk_mul_f16: one
// issue per score fewer than two f32 products and a conversion); bf16 tiles: the f32
// products, rounded once.''')
rep('#if FA2_DS_PK && !defined(FA2_TILE_BF16)', '#ifndef FA2_TILE_BF16')
# FA2_BWD_COAL is always on
rep('''// Row-coalesced prologue / epilogue (FA2_BWD_COAL).''', '''// Row-coalesced prologue / epilogue.''')
rep('''#ifndef FA2_BWD_COAL
#define FA2_BWD_COAL 1
#endif
''', '')

# ---- dkdv_step (32x32x16): no ablations
rep('''// ABL (timing ablations only, tools/kbench.py; results are wrong when set):
//   2 = no softmax VALU, 8 = no dV/dK MFMAs, 16 = no S/dP MFMAs
template <int D, int KB, int ABL = 0, typename Mid>''', '''template <int D, int KB, typename Mid>''')
rep('''        if (!(ABL & 16)) {
#pragma unroll
            for (int t = 0; t < D / 16; ++t) {
                const f16x8 qa = fo.rowop(Qs, qb * 32, t), da_op = fo.rowop(dOs, qb * 32, t);
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) {
                    sa[kb] = mfma(qa, st.kf[kb][t], sa[kb]);
                    da[kb] = mfma(da_op, st.vf[kb][t], da[kb]);
                }
            }
        }''', '''#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
            const f16x8 qa = fo.rowop(Qs, qb * 32, t), da_op = fo.rowop(dOs, qb * 32, t);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                sa[kb] = mfma(qa, st.kf[kb][t], sa[kb]);
                da[kb] = mfma(da_op, st.vf[kb][t], da[kb]);
            }
        }''')
rep('''            for (int i = 0; i < 16; ++i) {
                if (ABL & 2) {
                    pf[kb][i >> 3][i & 7] = to_tile(sa[kb][i]);
                    dsf[kb][i >> 3][i & 7] = to_tile(da[kb][i]);
                } else {
                    const float p = fast_exp2(sa[kb][i]);
                    pf[kb][i >> 3][i & 7] = to_tile(p);
                    dsf[kb][i >> 3][i & 7] = to_tile(p * da[kb][i]);
                }
            }
        if (ABL & 8) {
#pragma unroll
            for (int kb = 0; kb < KB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) asm volatile("" ::"v"(pf[kb][s]), "v"(dsf[kb][s]));
            continue;
        }''', '''            for (int i = 0; i < 16; ++i) {
                const float p = fast_exp2(sa[kb][i]);
                pf[kb][i >> 3][i & 7] = to_tile(p);
                dsf[kb][i >> 3][i & 7] = to_tile(p * da[kb][i]);
            }''')
# tuning macros fixed at their measured defaults
cut('#ifndef FA2_DKDV_LP\n', '// ---- dK, dV on v_mfma_f32_16x16x32')
rep('// ---- dK, dV on v_mfma_f32_16x16x32 (FA2_TUNE_DKDV_MF=16) ------------------------',
    '''// Staging of the next Q/dO step in the dK/dV kernel is done by waves 0-3 only: stamps
// showed waves 4-7 (which lose VALU arbitration to their SIMD partners) ~15 % slower
// per step and the first half idling at the barrier (r01).  The dQ kernel's waves 4-7
// run at s_setprio 1 (MI355X_MICROARCH §Two waves per SIMD, item 4: +1 %); its next-step
// K/V loads are issued on the last step too (rows past S read as zeros through the
// range-checked descriptor, no memory traffic), which removed 8 v_mov_b64 of
// staging-register phi copies per step (+0.7 % at C3, +8.8 % at D = 128).
#define FA2_DKDV_SW 4

// ---- dK, dV on v_mfma_f32_16x16x32 ----------------------------------------------''')
# ---- dkdv_step16
rep('''template <int D, int ABL = 0, typename Mid>
__device__ __forceinline__ void dkdv_step16(''', '''template <int D, typename Mid>
__device__ __forceinline__ void dkdv_step16(''')
rep('''        if (!(ABL & 16)) {
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
        }''', '''#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks)
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                const f16x8 qa = fo.rowop(Qs, qb * 32 + 16 * mb, ks), doa = fo.rowop(dOs, qb * 32 + 16 * mb, ks);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    sa[mb][nb] = mfma16(qa, st.kf[nb][ks], sa[mb][nb]);
                    da[mb][nb] = mfma16(doa, st.vf[nb][ks], da[mb][nb]);
                }
            }''')
rep('''                const float sv1 = sa[j >> 2][nb][(j & 3) + 1], dv1 = da[j >> 2][nb][(j & 3) + 1];
                if (ABL & 2) {
                    pf[nb][j] = to_tile(sv0);
                    pf[nb][j + 1] = to_tile(sv1);
                    dsf[nb][j] = to_tile(dv0);
                    dsf[nb][j + 1] = to_tile(dv1);
                } else {
                    const float p0 = fast_exp2(sv0), p1 = fast_exp2(sv1);
                    pf[nb][j] = to_tile(p0);
                    pf[nb][j + 1] = to_tile(p1);
                    const tile2 d2 = ds_pair(p0, p1, dv0, dv1, pf[nb][j], pf[nb][j + 1]);
                    dsf[nb][j] = d2[0];
                    dsf[nb][j + 1] = d2[1];
                }
            }
        if (ABL & 8) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) asm volatile("" ::"v"(pf[nb]), "v"(dsf[nb]));
            continue;
        }''', '''                const float sv1 = sa[j >> 2][nb][(j & 3) + 1], dv1 = da[j >> 2][nb][(j & 3) + 1];
                const float p0 = fast_exp2(sv0), p1 = fast_exp2(sv1);
                pf[nb][j] = to_tile(p0);
                pf[nb][j + 1] = to_tile(p1);
                const tile2 d2 = ds_pair(p0, p1, dv0, dv1, pf[nb][j], pf[nb][j + 1]);
                dsf[nb][j] = d2[0];
                dsf[nb][j + 1] = d2[1];
            }''')
# software-pipelined variant (rejected: -2..-5 %)
cut('// FA2_DKDV_PIPE: the two 32-query blocks of a step software-pipelined', '// a wave\'s 32 keys x D results (16x16 accumulator layout)')
open(p, 'w').write(s)
print("stage1 ok")
