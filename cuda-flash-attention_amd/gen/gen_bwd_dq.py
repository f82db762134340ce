#!/usr/bin/env python3
"""Generator of the hand-scheduled FA2 backward dQ tile loop for gfx950 (MI355X), D = 64.

Writes ../kernels/fa2_bwd_dq_hs.inc: the inline-asm body of `fa2_bwd_dq_hs_kernel<64>`
(f-attn2-backward_f16.cu), between its C++ prologue (Q and dO blocks, the first K/V tile,
-LSE*log2e and -Delta per row) and its C++ epilogue (dQ rows from an LDS stage, scaled
by 1/sqrt(D)).  The math is the dQ part of the reference's backward
(kernels/f-attn2-backward_f16.cu:240-301): P = exp(Q K^T / sqrt(D) - LSE),
dS = P o (dO V^T - Delta), dQ = dS K / sqrt(D) -- summed here in one fixed order per
query row (no atomics), the three products per tile on MFMA:

  * one workgroup = 4 waves = 256 query rows, ONE wave per SIMD; each wave holds 64 query
    rows as two 32-row chains A and B, with Q and dO fragments and the dQ^T accumulators
    in AGPRs for the whole key loop;
  * per 64-key tile four phases, each one MFMA chain with the other chain's VALU placed in
    its gaps (gen_fwd_hs.py's structure, with S^T and dP^T together as the first chain):
        P1  S^T, dP^T of A (tile j)   | dS of B (tile j-1), three quarters
        P2  dQ^T of B (tile j-1)      | dS of A (tile j),   the first quarter
        P3  S^T, dP^T of B (tile j)   | dS of A (tile j),   three quarters   -> barrier
        P4  dQ^T of A (tile j)        | dS of B (tile j),   the first quarter
  * S^T = K Q^T starts from -LSE*log2e and dP^T = V dO^T from -Delta (lane-constant splats:
    the query is on the lane), so P = exp2(acc) and dS = P * acc, one v_exp and one v_mul
    per score; dS is packed to fp16/bf16 in place and IS the B operand of
    dQ^T += K^T dS^T (K^T through ds_read_b64_tr_b16 of the K tile);
  * K and V tiles: fp32 HBM -> registers -> fp16/bf16 -> swizzled LDS, one tile ahead;
  * all on v_mfma_f32_16x16x32 (r05: 5-6 % faster than the same loop on 32x32x16 at C3 and
    B2_H8_S4096 in-process, profiles/r05/dq16/ -- less energy per FLOP at the power cap,
    where the kernel runs), on the operand maps:

  A[m = l & 15][k = 8g + j], B[k = 8g + j][n = l & 15], C[m = 4g + i][n = l & 15]  (g = l >> 4)

  * S^T / dP^T tiles [16 keys][16 queries]: A = K / V row fragments (rows 16 kb + (l & 15),
    columns 32 ks + 8g), B = Q / dO fragments of the wave's query block (query on the lane);
    the first MFMA of each tile starts from the -LSE*log2e / -Delta splat of its query block;
  * dQ^T[16 d][16 q] += K^T dS^T over 32 keys per MFMA: B = the packed dS of two key blocks,
    k-slot 8g + j <-> key 16 (j >> 2) + 4g + (j & 3) of the 32; A = K^T by two 4-row
    transposed reads (rows 4g.. and 16 + 4g.., columns 16 db ..) in the same key order.

16x16x32 reads and writes a quarter of the accumulator per instruction for half the FLOPs,
and the splat seeds are 4 registers per 16-query block.

Register map (D = 64; c chain, qb its 16-row query blocks, kb 16-key blocks, ks / s 32-steps):
  AGPR  dQ^T[c][db][qb] a[32c + 8db + 4qb]   Q[c][qb][ks] a[64 + 16c + 8qb + 4ks]
        dO[c][qb][ks]   a[96 + ...]           K^T[db][s] a[128 + 4(2db + s)]
        K rows[kb][ks]  a[160 + 4(2kb + ks)]  V rows[kb][ks] a[192 + 4(2kb + ks)]
  VGPR  S^T[c][qb][kb]  v[32c + 16qb + 4kb]   dP^T v[64 + ...]
        -LSE splat[c][qb] v[128 + 4(2c + qb)] -Delta splat v[144 + ...]  staging v[160..191]

Usage: python3 gen_bwd_dq.py [--check]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import asmgen  # noqa: E402
from asmgen import Ins, R, ablate, ablate_waits, fix_hazards, insert_waits, rng, rtxt, schedule_phase, stamp, tagged, thirds, valu  # noqa: E402,E501

KT = 64
ROWS = 256
# dS groups per chain and tile: (qb, s) = 8 scores of each lane (key blocks 2s, 2s+1 of
# query block qb); the first part (in the short dQ phase) takes one group, the rest three
PART1 = [(0, 0)]
PART2 = [(0, 1), (1, 0), (1, 1)]


class Cfg:
    def __init__(self, D, bf16):
        assert D == 64
        self.D, self.bf16 = D, bf16
        self.KS = D // 32  # 32-column steps of a row fragment
        self.NDB = D // 16  # 16-row blocks of dQ^T
        self.exp_per_gap = 1
        self.min_cap = 12  # 16-cycle MFMAs: about half the 32x32x16 gap's issue room
        self.TBB = KT * D * 2
        self.OST = D + 4
        self.mf = "v_mfma_f32_16x16x32_bf16" if bf16 else "v_mfma_f32_16x16x32_f16"
        self.cvt = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.nvgpr, self.nagpr = 192, 224
        self.SV = self.nvgpr
        if "stamps" in asmgen.ABL:
            self.nvgpr += 2

    # AGPRs
    def O(self, c, db, qb):
        return 32 * c + 8 * db + 4 * qb

    def Q(self, c, qb, ks):
        return 64 + 16 * c + 8 * qb + 4 * ks

    def dO(self, c, qb, ks):
        return 96 + 16 * c + 8 * qb + 4 * ks

    def Kt(self, db, s):
        return 128 + 4 * (2 * db + s)

    def Kr(self, kb, ks):
        return 160 + 4 * (2 * kb + ks)

    def Vr(self, kb, ks):
        return 192 + 4 * (2 * kb + ks)

    # VGPRs
    def S(self, c, qb, kb, i=0):
        return 32 * c + 16 * qb + 4 * kb + i

    def dP(self, c, qb, kb, i=0):
        return 64 + 32 * c + 16 * qb + 4 * kb + i

    def NL(self, c, qb):
        return 128 + 4 * (2 * c + qb)

    def ND(self, c, qb):
        return 144 + 4 * (2 * c + qb)

    def stg(self, tensor, cc):
        return 160 + 8 * (tensor * 2 + cc)

    def koff(self, slot):
        return slot * self.TBB

    def voff(self, slot):
        return (2 + slot) * self.TBB

    @property
    def lds_bytes(self):
        return max(4 * self.TBB + 2 * ROWS * self.D * 2, ROWS * self.OST * 4)


def mfma(cfg, dst, a, b, c, c_is_zero=False):
    rd = R(rng(a[0], a[1], 4), "A") + R(rng(b[0], b[1], 4), "B")
    if not c_is_zero:
        rd += R(rng(c[0], c[1], 4), "C")
    ctxt = "0" if c_is_zero else rtxt(c[0], c[1], 4)
    return Ins(f"{cfg.mf} {rtxt(dst[0], dst[1], 4)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {ctxt}", "mfma",
               rd, rng(dst[0], dst[1], 4))


def row_reads(cfg, slot, tensor):
    """the 8 row fragments (kb, ks) of the K (tensor 0) or V (1) tile in `slot` -> AGPRs"""
    out = []
    base = cfg.koff(slot) if tensor == 0 else cfg.voff(slot)
    for kb in range(4):
        for ks in range(cfg.KS):
            d = cfg.Kr(kb, ks) if tensor == 0 else cfg.Vr(kb, ks)
            out.append(Ins(f"ds_read_b128 {rtxt('a', d, 4)}, %[ka{ks}] offset:{base + kb * 16 * cfg.D * 2}", "dsr",
                           [], rng("a", d, 4)))
    return tagged("lds", out)


def ktr_reads(cfg, db, s, slot, earliest=0):
    off = cfg.koff(slot) + s * 32 * cfg.D * 2
    d = cfg.Kt(db, s)
    return tagged("lds", [
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d, 2)}, %[kt{db}_0] offset:{off}", "dsr", [], rng("a", d, 2),
            earliest=earliest),
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d + 2, 2)}, %[kt{db}_1] offset:{off}", "dsr", [], rng("a", d + 2, 2),
            earliest=earliest)])


def sdp_mfmas(cfg, c):
    """S^T and dP^T tiles of chain c, group (qb, s) by group in PART1 + PART2 order (the first
    part's dS needs its tiles first)"""
    out = []
    for qb, s in PART1 + PART2:
        for kb in (2 * s, 2 * s + 1):
            for which in range(2):
                for ks in range(cfg.KS):
                    if which == 0:
                        dst, a, b, seed = cfg.S(c, qb, kb), cfg.Kr(kb, ks), cfg.Q(c, qb, ks), cfg.NL(c, qb)
                    else:
                        dst, a, b, seed = cfg.dP(c, qb, kb), cfg.Vr(kb, ks), cfg.dO(c, qb, ks), cfg.ND(c, qb)
                    cc = ("v", seed) if ks == 0 else ("v", dst)
                    out.append(mfma(cfg, ("v", dst), ("a", a), ("a", b), cc))
    return out


def dq_mfmas(cfg, c, first=False):
    """dQ^T[c][db][qb] += K^T[db][s] dS^T[c][qb][s]"""
    out = []
    for db in range(cfg.NDB):
        for s in range(2):
            for qb in range(2):
                z = first and s == 0
                out.append(mfma(cfg, ("a", cfg.O(c, db, qb)), ("a", cfg.Kt(db, s)), ("v", cfg.S(c, qb, 2 * s)),
                                ("a", cfg.O(c, db, qb)), c_is_zero=z))
    return out


def ds_part(cfg, c, groups):
    """dS of the given groups (qb, s) of chain c: exp2, * dP', packed in place"""
    out = []
    for qb, s in groups:
        base, dbase = cfg.S(c, qb, 2 * s), cfg.dP(c, qb, 2 * s)
        for i in range(8):
            r = base + i
            out.append(valu(f"v_exp_f32 v{r}, v{r}", [f"v{r}"], [f"v{r}"], kind="exp"))
        for i in range(8):
            r, d = base + i, dbase + i
            out.append(valu(f"v_mul_f32 v{r}, v{r}, v{d}", [f"v{r}", f"v{d}"], [f"v{r}"]))
        for ii in range(4):
            d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
    return tagged("sm", out)


def staging_loads(cfg, tensor):
    rs = "%[rsk]" if tensor == 0 else "%[rsv]"
    out = []
    for cc in range(2):
        base = cfg.stg(tensor, cc)
        for h in range(2):
            off = f" offset:{16 * h}" if h else ""
            out.append(Ins(f"buffer_load_dwordx4 {rtxt('v', base + 4 * h, 4)}, %[vo{cc}], {rs}, %[goff] offen{off}",
                           "vmem", R(["s:goff"]), rng("v", base + 4 * h, 4)))
    return tagged("stg", out)


def goff_inc(cfg):
    return tagged("stg", [Ins(f"s_add_u32 %[goff], %[goff], {KT * cfg.D * 4}", "salu", R(["s:goff"]),
                              ["s:goff", "scc"])])[0]


def staging_convert(cfg, tensor, slot):
    out = []
    toff = cfg.koff(slot) if tensor == 0 else cfg.voff(slot)
    rows_per_chunk_step = 256 // (cfg.D // 8)
    for cc in range(2):
        base = cfg.stg(tensor, cc)
        for ii in range(4):
            d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
        out.append(Ins(f"ds_write_b128 %[lo], {rtxt('v', base, 4)} offset:{toff + cc * rows_per_chunk_step * cfg.D * 2}",
                       "dsw", R(rng("v", base, 4)), []))
    return tagged("stg", out)


def kt_all(cfg, slot):
    out = []
    for db in range(cfg.NDB):
        for s in range(2):
            out += ktr_reads(cfg, db, s, slot)
    return out


def body(cfg, p, log):
    q = 1 - p
    seq = []
    conv = staging_convert(cfg, 0, q)
    for ins in conv:
        ins.earliest = 8
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 0), [ds_part(cfg, 1, PART2), conv], f"P1.{p}", log)
    seq += stamp(cfg.SV)
    # staging loads of tile j+2: K (regs free since P1's convert) then V (free since P2's),
    # spread over P2, P3, P4
    if "nospread" in asmgen.ABL:
        ld = (staging_loads(cfg, 0), [], staging_loads(cfg, 1))
    else:
        ld = thirds(staging_loads(cfg, 0) + staging_loads(cfg, 1))
    seq += schedule_phase(cfg, dq_mfmas(cfg, 1), [ds_part(cfg, 0, PART1), staging_convert(cfg, 1, q),
                                                  list(ld[0])], f"P2.{p}", log)
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 1), [ds_part(cfg, 0, PART2), kt_all(cfg, p), list(ld[1])], f"P3.{p}", log)
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    seq += stamp(cfg.SV)
    seq.append(tagged("bar", [Ins("s_barrier", "bar")])[0])
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, dq_mfmas(cfg, 0), [ds_part(cfg, 1, PART1), row_reads(cfg, q, 0) + row_reads(cfg, q, 1),
                                                  list(ld[2]) + [goff_inc(cfg)]], f"P4.{p}", log)
    return seq


def prologue(cfg):
    D = cfg.D
    seq = [Ins("s_mov_b32 s98, 0", "salu", [], ["s98"])] if "stamps" in asmgen.ABL else []
    seq += stamp(cfg.SV)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    # Q and dO fragments of the wave's 4 query blocks (blocks in LDS at %[qb] / %[db])
    for ks in range(cfg.KS):
        seq.append(valu(f"v_add_u32 v{ks}, %[qb], %[ka{ks}]", [], [f"v{ks}"]))
        seq.append(valu(f"v_add_u32 v{2 + ks}, %[db], %[ka{ks}]", [], [f"v{2 + ks}"]))
    for c in range(2):
        for qb in range(2):
            for ks in range(cfg.KS):
                off = (32 * c + 16 * qb) * D * 2
                seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.Q(c, qb, ks), 4)}, v{ks} offset:{off}", "dsr",
                               R([f"v{ks}"]), rng("a", cfg.Q(c, qb, ks), 4)))
                seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.dO(c, qb, ks), 4)}, v{2 + ks} offset:{off}", "dsr",
                               R([f"v{2 + ks}"]), rng("a", cfg.dO(c, qb, ks), 4)))
    seq += row_reads(cfg, 0, 0) + row_reads(cfg, 0, 1)
    # the seeds: -LSE*log2e and -Delta of the lane's query row in each 16-row block
    for c in range(2):
        for qb in range(2):
            for i in range(4):
                seq.append(valu(f"v_mov_b32 v{cfg.NL(c, qb) + i}, %[nl{2 * c + qb}]", [], [f"v{cfg.NL(c, qb) + i}"]))
                seq.append(valu(f"v_mov_b32 v{cfg.ND(c, qb) + i}, %[nd{2 * c + qb}]", [], [f"v{cfg.ND(c, qb) + i}"]))
    seq += sdp_mfmas(cfg, 0) + sdp_mfmas(cfg, 1)
    seq += ds_part(cfg, 0, PART1) + ds_part(cfg, 0, PART2) + ds_part(cfg, 1, PART1)
    seq += kt_all(cfg, 0)
    for db in range(cfg.NDB):
        for qb in range(2):
            for i in range(4):
                r = cfg.O(1, db, qb) + i
                seq.append(valu(f"v_accvgpr_write_b32 a{r}, 0", [], [f"a{r}"]))
    seq += dq_mfmas(cfg, 0, first=True)
    seq += staging_convert(cfg, 0, 1) + staging_convert(cfg, 1, 1)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    seq += [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_barrier", "bar")]
    seq += row_reads(cfg, 1, 0) + row_reads(cfg, 1, 1)
    seq += stamp(cfg.SV)
    return seq


def epilogue(cfg):
    seq = [Ins("s_waitcnt vmcnt(0) lgkmcnt(0)", "wait")]
    seq += stamp(cfg.SV)
    seq += ds_part(cfg, 1, PART2)
    seq += dq_mfmas(cfg, 1)
    seq.append(Ins("s_barrier", "bar"))
    # dQ^T[c][db][qb] reg i: d = 16 db + 4g + i, query 32c + 16qb + (l & 15) -> stage row, 4 columns
    for c in range(2):
        for db in range(cfg.NDB):
            for qb in range(2):
                r = cfg.O(c, db, qb)
                off = ((32 * c + 16 * qb) * cfg.OST + 16 * db) * 4
                seq.append(Ins(f"ds_write_b128 %[oa], {rtxt('a', r, 4)} offset:{off}", "dsw", R(rng("a", r, 4)), []))
    if "stamps" in asmgen.ABL:
        # the stamps through %[sa], the 32x32 build's stage address (row l & 31, column
        # 4 (l >> 5) + 2), so tools/stamps_hs.py decodes both builds alike
        seq += stamp(cfg.SV)
        sv, sc = cfg.SV, cfg.SV + 1
        seq += [Ins("s_nop 4", "nop"),
                valu(f"v_and_b32 v{sv}, 0xffffff, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_cvt_f32_u32 v{sv}, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_mov_b32 v{sc}, s98", [], [f"v{sc}"]),
                valu(f"v_cvt_f32_u32 v{sc}, v{sc}", [f"v{sc}"], [f"v{sc}"]),
                Ins("s_nop 4", "nop"),
                Ins(f"ds_write_b32 %[sa], v{sv} offset:8", "dsw", R([f"v{sv}"]), []),
                Ins(f"ds_write_b32 %[sa], v{sc} offset:12", "dsw", R([f"v{sc}"]), [])]
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    return seq


def build(cfg):
    log = [f"dQ D={cfg.D} {'bf16' if cfg.bf16 else 'fp16'}: {cfg.nvgpr} VGPRs + {cfg.nagpr} AGPRs in asm, "
           f"LDS {cfg.lds_bytes} B"]
    pro, b1, b0, epi = prologue(cfg), ablate(body(cfg, 1, log)), ablate(body(cfg, 0, log)), epilogue(cfg)
    empty = ((), ())
    pro, st_p = insert_waits(pro, empty)
    b1, st_1 = insert_waits(b1, st_p)
    b0, st_0 = insert_waits(b0, st_1)
    assert asmgen.ABL or st_0 == st_p, "loop-carried wait state differs between the prologue exit and the loop back edge"
    epi, _ = insert_waits(epi, empty)
    b1, b0 = ablate_waits(b1), ablate_waits(b0)
    b1 = b1 + [Ins("s_sub_u32 %[cnt], %[cnt], 1", "salu", R(["s:cnt"]), ["s:cnt", "scc"]),
               Ins("s_cmp_eq_u32 %[cnt], 0", "salu", R(["s:cnt"]), ["scc"]),
               Ins("s_cbranch_scc1 FA2DQ_EPI_%=", "branch", R(["scc"]))]
    b0 = b0 + [Ins("s_sub_u32 %[cnt], %[cnt], 1", "salu", R(["s:cnt"]), ["s:cnt", "scc"]),
               Ins("s_cmp_lg_u32 %[cnt], 0", "salu", R(["s:cnt"]), ["scc"]),
               Ins("s_cbranch_scc1 FA2DQ_LOOP_%=", "branch", R(["scc"]))]
    for _ in range(3):
        pro = fix_hazards(pro, [[]])
        b1 = fix_hazards(b1, [pro[-40:], b0[-40:]])
        b0 = fix_hazards(b0, [b1[-40:]])
        epi = fix_hazards(epi, [b1[-40:], b0[-40:]])
    lines = [i.text for i in pro] + ["FA2DQ_LOOP_%=:"] + [i.text for i in b1] + [i.text for i in b0] + \
            ["FA2DQ_EPI_%=:"] + [i.text for i in epi]
    nm = sum(1 for i in b1 + b0 if i.kind == "mfma")
    nv = sum(1 for i in b1 + b0 if i.kind in ("valu", "exp"))
    nn = sum(int(i.text.split()[1]) + 1 for i in b1 + b0 if i.kind == "nop")
    log.append(f"  loop (2 tiles): {nm} MFMA, {nv} VALU ({nv / max(nm, 1):.2f} per MFMA), {nn} nop wait states, "
               f"{len(b1) + len(b0)} instructions")
    return lines, log


def operands(cfg):
    outs = ['[cnt] "+s"(hs_cnt)', '[goff] "+s"(hs_goff)']
    ins = [f'[ka{ks}] "v"(hs_ka[{ks}])' for ks in range(cfg.KS)]
    ins += [f'[kt{db}_{k}] "v"(hs_kt[{db}][{k}])' for db in range(cfg.NDB) for k in range(2)]
    ins += [f'[vo{c}] "v"(hs_vo[{c}])' for c in range(2)]
    ins += [f'[nl{i}] "v"(hs_nl[{i}])' for i in range(4)] + [f'[nd{i}] "v"(hs_nd[{i}])' for i in range(4)]
    ins += ['[lo] "v"(hs_lo)', '[oa] "v"(hs_oa)', '[rsk] "s"(hs_rsk)', '[rsv] "s"(hs_rsv)', '[qb] "s"(hs_qb)',
            '[db] "s"(hs_db)']
    if "stamps" in asmgen.ABL:
        ins.append('[sa] "v"(hs_sa)')
    clob = [f'"v{i}"' for i in range(cfg.nvgpr)] + [f'"a{i}"' for i in range(cfg.nagpr)] + ['"vcc"', '"scc"', '"memory"']
    if "stamps" in asmgen.ABL:
        clob += asmgen.STAMP_CLOBBERS
    return outs, ins, clob


def emit():
    here = os.path.dirname(os.path.abspath(__file__))
    out = ["// Generated by cuda-flash-attention_amd/gen/gen_bwd_dq.py -- do not edit.",
           "// Hand-scheduled dQ tile loop of fa2_bwd_dq_hs_kernel<D> (f-attn2-backward_f16.cu).",
           "#pragma once", ""]
    logs = []
    for bf16 in (False, True):
        cfg = Cfg(64, bf16)
        lines, log = build(cfg)
        logs += log
        out.append(f"#define FA2_DQ_ASM_D64_{'BF16' if bf16 else 'F16'} \\")
        out += [f'    "{ln}\\n\\t" \\' for ln in lines]
        out.append('    ""')
        out.append("")
    cfg = Cfg(64, False)
    o, i, c = operands(cfg)
    out.append("#define FA2_DQ_OUTPUTS_D64 " + ", ".join(o))
    out.append("#define FA2_DQ_INPUTS_D64 " + ", ".join(i))
    out.append("#define FA2_DQ_CLOBBERS_D64 " + ", ".join(c))
    out.append(f"#define FA2_DQ_LDS_D64 {cfg.lds_bytes}")
    out.append("")
    out = ["// " + ln for ln in logs] + out
    text = "\n".join(out) + "\n"
    path = os.path.join(here, "..", "kernels", "fa2_bwd_dq_hs.inc")
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
    if "--check" in sys.argv:
        cur = open(path).read() if os.path.exists(path) else ""
        if cur != text:
            print("fa2_bwd_dq_hs.inc is stale: run gen/gen_bwd_dq.py")
            sys.exit(1)
        return
    with open(path, "w") as f:
        f.write(text)
    print("\n".join(logs))


if __name__ == "__main__":
    asmgen.parse_abl(sys.argv)
    emit()
