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
        P1  S^T, dP^T of A (tile j)   | dS of B (tile j-1), scores 8..31
        P2  dQ^T of B (tile j-1)      | dS of A (tile j),   scores 0..7
        P3  S^T, dP^T of B (tile j)   | dS of A (tile j),   scores 8..31   -> barrier
        P4  dQ^T of A (tile j)        | dS of B (tile j),   scores 0..7
    (the dS work is split 8 / 24 of each lane's 32 scores so the short dQ phases, 8 MFMAs, and
    the long ones, 16, carry issue in proportion);
  * S^T = K Q^T starts from -LSE*log2e and dP^T = V dO^T from -Delta (lane-constant splats:
    the query is on the lane), so P = exp2(acc) and dS = P * acc, one v_exp and one v_mul
    per score; dS is packed to fp16/bf16 in place and IS the B operand of
    dQ^T += K^T dS^T (K^T through ds_read_b64_tr_b16 of the K tile);
  * K and V tiles: fp32 HBM -> registers -> fp16/bf16 -> swizzled LDS, one tile ahead.

Register map (D = 64):
  AGPR  dQ^T[c][b]  a[16(2c+b)]    Q[c][t] a[64+4(4c+t)]   dO[c][t] a[96+4(4c+t)]
        K^T frags   a[128+4i]      K rows  a[160+4f]       V rows   a[192+4f]
  VGPR  S^T[c][kb]  v[32c+16kb]    dP^T[c][kb] v[64+32c+16kb]
        -LSE splat  v[128+16c]     -Delta splat v[160+16c]   staging v[192..223]

Usage: python3 gen_bwd_dq.py [--check]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import asmgen  # noqa: E402
from asmgen import Ins, R, ablate, ablate_waits, fix_hazards, insert_waits, rng, rtxt, schedule_phase, stamp, tagged, valu  # noqa: E402,E501

KT = 64
ROWS = 256
# dS work per chain and tile = 4 groups of 8 scores (kb, first score); the first part (in the
# short dQ phase) takes one group, the second part (in the long S^T/dP^T phase) three
PART1 = [(0, 0)]
PART2 = [(0, 8), (1, 0), (1, 8)]


class Cfg:
    def __init__(self, D, bf16):
        assert D == 64
        self.D, self.bf16 = D, bf16
        self.NB, self.NTQ, self.CPT = D // 32, D // 16, D // 32
        self.NF = 4 * self.NB  # K^T fragments per tile (dQ A operands)
        self.NKF = 2 * self.NTQ  # K / V row fragments per tile
        self.exp_per_gap = 2
        self.TBB = KT * D * 2
        self.OST = D + 4
        self.mf = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvt = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.nvgpr, self.nagpr = 224, 224
        self.SV = self.nvgpr  # 'stamps' timing builds: the stamp register (and one more)
        if "stamps" in asmgen.ABL:
            self.nvgpr += 2

    # AGPRs
    def O(self, c, b):
        return 16 * (2 * c + b)

    def Q(self, c, t):
        return 64 + 4 * (4 * c + t)

    def dO(self, c, t):
        return 96 + 4 * (4 * c + t)

    def Kt(self, i):
        return 128 + 4 * i

    def Kr(self, f):
        return 160 + 4 * f

    def Vr(self, f):
        return 192 + 4 * f

    # VGPRs
    def S(self, c, kb, i=0):
        return 32 * c + 16 * kb + i

    def dP(self, c, kb, i=0):
        return 64 + 32 * c + 16 * kb + i

    def NL(self, c):
        return 128 + 16 * c

    def ND(self, c):
        return 160 + 16 * c

    def stg(self, tensor, cc):
        return 192 + 8 * (tensor * self.CPT + cc)

    def koff(self, slot):
        return slot * self.TBB

    def voff(self, slot):
        return (2 + slot) * self.TBB

    @property
    def lds_bytes(self):
        # K, V slots + Q block + dO block; the dQ stage reuses the front after a barrier
        return max(4 * self.TBB + 2 * ROWS * self.D * 2, ROWS * self.OST * 4)

    def ktr_addr(self, i):
        b, kb, s = i // 4, (i // 2) % 2, i % 2
        return b, (kb * 32 + 16 * s) * self.D * 2


def mfma(cfg, dst, a, b, c, c_is_zero=False):
    rd = R(rng(a[0], a[1], 4), "A") + R(rng(b[0], b[1], 4), "B")
    if not c_is_zero:
        rd += R(rng(c[0], c[1], 16), "C")
    ctxt = "0" if c_is_zero else rtxt(c[0], c[1], 16)
    return Ins(f"{cfg.mf} {rtxt(dst[0], dst[1], 16)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {ctxt}", "mfma",
               rd, rng(dst[0], dst[1], 16))


def row_reads(cfg, slot, tensor):
    """the 8 row fragments (kb, t) of the K (tensor 0) or V (1) tile in `slot` -> AGPRs"""
    out = []
    base = cfg.koff(slot) if tensor == 0 else cfg.voff(slot)
    for f in range(cfg.NKF):
        kb, t = f // cfg.NTQ, f % cfg.NTQ
        d = cfg.Kr(f) if tensor == 0 else cfg.Vr(f)
        out.append(Ins(f"ds_read_b128 {rtxt('a', d, 4)}, %[ka{t}] offset:{base + kb * 32 * cfg.D * 2}", "dsr", [],
                       rng("a", d, 4)))
    return tagged("lds", out)


def ktr_reads(cfg, i, slot, earliest=0):
    b, off = cfg.ktr_addr(i)
    off += cfg.koff(slot)
    d = cfg.Kt(i)
    return tagged("lds", [
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d, 2)}, %[kt{b}_0] offset:{off}", "dsr", [], rng("a", d, 2),
            earliest=earliest),
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d + 2, 2)}, %[kt{b}_1] offset:{off}", "dsr", [], rng("a", d + 2, 2),
            earliest=earliest)])


def sdp_mfmas(cfg, c, zero_seed=False):
    """S^T[c] = K Q^T - LSE*log2e and dP^T[c] = V dO^T - Delta, kb = 0 first (dS part 1 needs it)"""
    out = []
    for kb in range(2):
        for which in range(2):
            for t in range(cfg.NTQ):
                f = kb * cfg.NTQ + t
                if which == 0:
                    dst, a, b, seed = cfg.S(c, kb), cfg.Kr(f), cfg.Q(c, t), cfg.NL(c)
                else:
                    dst, a, b, seed = cfg.dP(c, kb), cfg.Vr(f), cfg.dO(c, t), cfg.ND(c)
                cc = ("v", seed) if t == 0 else ("v", dst)
                out.append(mfma(cfg, ("v", dst), ("a", a), ("a", b), cc))
    return out


def dq_mfmas(cfg, c, first=False):
    """dQ^T[c][b] += K^T dS^T[c]: b-major, so K^T slot i is free after MFMA i"""
    out = []
    for b in range(cfg.NB):
        for kb in range(2):
            for s in range(2):
                i = b * 4 + kb * 2 + s
                z = first and kb == 0 and s == 0
                out.append(mfma(cfg, ("a", cfg.O(c, b)), ("a", cfg.Kt(i)), ("v", cfg.S(c, kb, 8 * s)),
                                ("a", cfg.O(c, b)), c_is_zero=z))
    return out


def ds_part(cfg, c, groups):
    """dS of the given 8-score groups (kb, first score) of chain c: exp2, * dP', packed in place
    (per group: exps and products first, then the 4 packs)"""
    out = []
    for kb, g0 in groups:
        for i in range(g0, g0 + 8):
            s = cfg.S(c, kb, i)
            out.append(valu(f"v_exp_f32 v{s}, v{s}", [f"v{s}"], [f"v{s}"], kind="exp"))
        for i in range(g0, g0 + 8):
            s, d = cfg.S(c, kb, i), cfg.dP(c, kb, i)
            out.append(valu(f"v_mul_f32 v{s}, v{s}, v{d}", [f"v{s}", f"v{d}"], [f"v{s}"]))
        for ii in range(4):
            d, a, b = cfg.S(c, kb, g0 + ii), cfg.S(c, kb, g0 + 2 * ii), cfg.S(c, kb, g0 + 2 * ii + 1)
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
    return tagged("sm", out)


def staging_loads(cfg, tensor):
    rs = "%[rsk]" if tensor == 0 else "%[rsv]"
    out = []
    for cc in range(cfg.CPT):
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
    for cc in range(cfg.CPT):
        base = cfg.stg(tensor, cc)
        for ii in range(4):
            d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
        out.append(Ins(f"ds_write_b128 %[lo], {rtxt('v', base, 4)} offset:{toff + cc * rows_per_chunk_step * cfg.D * 2}",
                       "dsw", R(rng("v", base, 4)), []))
    return tagged("stg", out)


def body(cfg, p, log):
    q = 1 - p
    seq = []
    conv = staging_convert(cfg, 0, q)
    for ins in conv:
        ins.earliest = 4
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 0), [ds_part(cfg, 1, PART2), conv], f"P1.{p}", log)
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, dq_mfmas(cfg, 1), [ds_part(cfg, 0, PART1), staging_convert(cfg, 1, q),
                                                  staging_loads(cfg, 0)], f"P2.{p}", log)
    seq += stamp(cfg.SV)
    kt = []
    for i in range(cfg.NF):
        kt += ktr_reads(cfg, i, p)
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 1), [ds_part(cfg, 0, PART2), kt], f"P3.{p}", log)
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    seq += stamp(cfg.SV)
    seq.append(tagged("bar", [Ins("s_barrier", "bar")])[0])
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, dq_mfmas(cfg, 0), [ds_part(cfg, 1, PART1), row_reads(cfg, q, 0) + row_reads(cfg, q, 1),
                                                  staging_loads(cfg, 1) + [goff_inc(cfg)]], f"P4.{p}", log)
    return seq


def prologue(cfg):
    D, NTQ = cfg.D, cfg.NTQ
    seq = [Ins("s_mov_b32 s98, 0", "salu", [], ["s98"])] if "stamps" in asmgen.ABL else []
    seq += stamp(cfg.SV)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    # Q and dO fragments of both chains (blocks in LDS at %[qb] / %[db] + this wave's rows)
    for t in range(NTQ):
        seq.append(valu(f"v_add_u32 v{t}, %[qb], %[ka{t}]", [], [f"v{t}"]))
        seq.append(valu(f"v_add_u32 v{4 + t}, %[db], %[ka{t}]", [], [f"v{4 + t}"]))
    for c in range(2):
        for t in range(NTQ):
            seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.Q(c, t), 4)}, v{t} offset:{c * 32 * D * 2}", "dsr",
                           R([f"v{t}"]), rng("a", cfg.Q(c, t), 4)))
            seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.dO(c, t), 4)}, v{4 + t} offset:{c * 32 * D * 2}", "dsr",
                           R([f"v{4 + t}"]), rng("a", cfg.dO(c, t), 4)))
    seq += row_reads(cfg, 0, 0) + row_reads(cfg, 0, 1)
    # the lane-constant seeds: -LSE*log2e and -Delta of this lane's row in each chain
    for c in range(2):
        for i in range(16):
            seq.append(valu(f"v_mov_b32 v{cfg.NL(c) + i}, %[nl{c}]", [], [f"v{cfg.NL(c) + i}"]))
            seq.append(valu(f"v_mov_b32 v{cfg.ND(c) + i}, %[nd{c}]", [], [f"v{cfg.ND(c) + i}"]))
    seq += sdp_mfmas(cfg, 0) + sdp_mfmas(cfg, 1)
    seq += ds_part(cfg, 0, PART1) + ds_part(cfg, 0, PART2) + ds_part(cfg, 1, PART1)
    for i in range(cfg.NF):
        seq += ktr_reads(cfg, i, 0)
    for b in range(cfg.NB):
        for i in range(16):
            r = cfg.O(1, b) + i
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
    for c in range(2):
        for b in range(cfg.NB):
            for g in range(4):
                r = cfg.O(c, b) + 4 * g
                off = (c * 32 * cfg.OST + 32 * b + 8 * g) * 4
                seq.append(Ins(f"ds_write_b128 %[oa], {rtxt('a', r, 4)} offset:{off}", "dsw", R(rng("a", r, 4)), []))
    if "stamps" in asmgen.ABL:
        # the stamps into stage columns 2 / 6, the count into 3 / 7 (gen_fwd_hs.py's layout)
        seq += stamp(cfg.SV)
        sv, sc = cfg.SV, cfg.SV + 1
        seq += [Ins("s_nop 4", "nop"),
                valu(f"v_and_b32 v{sv}, 0xffffff, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_cvt_f32_u32 v{sv}, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_mov_b32 v{sc}, s98", [], [f"v{sc}"]),
                valu(f"v_cvt_f32_u32 v{sc}, v{sc}", [f"v{sc}"], [f"v{sc}"]),
                Ins("s_nop 4", "nop"),
                Ins(f"ds_write_b32 %[oa], v{sv} offset:8", "dsw", R([f"v{sv}"]), []),
                Ins(f"ds_write_b32 %[oa], v{sc} offset:12", "dsw", R([f"v{sc}"]), [])]
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
    ins = [f'[ka{t}] "v"(hs_ka[{t}])' for t in range(cfg.NTQ)]
    ins += [f'[kt{b}_{k}] "v"(hs_kt[{b}][{k}])' for b in range(cfg.NB) for k in range(2)]
    ins += [f'[vo{c}] "v"(hs_vo[{c}])' for c in range(cfg.CPT)]
    ins += ['[lo] "v"(hs_lo)', '[oa] "v"(hs_oa)', '[nl0] "v"(hs_nl0)', '[nl1] "v"(hs_nl1)', '[nd0] "v"(hs_nd0)',
            '[nd1] "v"(hs_nd1)', '[rsk] "s"(hs_rsk)', '[rsv] "s"(hs_rsv)', '[qb] "s"(hs_qb)', '[db] "s"(hs_db)']
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
