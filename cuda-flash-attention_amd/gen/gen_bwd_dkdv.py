#!/usr/bin/env python3
"""Generator of the hand-scheduled FA2 backward dK/dV loop for gfx950 (MI355X), D = 64.

Writes ../kernels/fa2_bwd_dkdv_hs.inc: the inline-asm body of `fa2_bwd_dkdv_hs_kernel<64>`
(f-attn2-backward_f16.cu), between its C++ prologue (the workgroup's K block, scaled by
log2(e)/sqrt(D), and V block; the first 64-query step's Q, dO and row constants) and its
C++ epilogue (dK, dV rows from an LDS stage; dK times 1/sqrt(D)).  The math is the dK/dV
part of the reference's backward (kernels/f-attn2-backward_f16.cu:170-268):
P = exp(Q K^T / sqrt(D) - LSE), dV = P^T dO, dS = P o (dO V^T - Delta), dK = dS^T Q / sqrt(D):

  * one workgroup = 4 waves = 256 keys, ONE wave per SIMD; each wave holds 64 keys (four
    16-key blocks nb): their K and V fragments and dK^T / dV^T accumulators sit in AGPRs
    for the whole query loop;
  * the head's queries stream in 64-row steps (Q and dO as fp16/bf16 tiles, -LSE*log2e and
    -Delta rows) through a 3-slot LDS ring, one barrier per step.  The step's two 32-row
    query blocks are the two chains A and B (every transposed dO^T / Q^T fragment and
    every row-constant tuple is read once per step, by the one chain it belongs to); per
    step four phases:
        P1  S, dP of A (step j)        | P, dS of B (step j-1), key blocks 2, 3
        P2  dV^T, dK^T of B (step j-1)| P, dS of A (step j),   key blocks 0, 1
        P3  S, dP of B (step j)        | P, dS of A (step j),   key blocks 2, 3   -> barrier
        P4  dV^T, dK^T of A (step j)  | P, dS of B (step j),   key blocks 0, 1
  * S = Q K^T starts from -LSE*log2e and dP = dO V^T from -Delta (4-register row-constant
    tuples read from LDS: the query is on the accumulator rows), so P = exp2(acc) and
    dS = P * acc; P and dS are packed in place and ARE the B operands of dV^T += dO^T P
    and dK^T += Q^T dS (dO^T, Q^T through ds_read_b64_tr_b16 into an 8-fragment ring);
  * Q and dO rows: fp32 HBM -> registers -> fp16/bf16 -> swizzled LDS two steps ahead of
    their use; the row constants by one dword load per lane of waves 0 (LSE) and 1 (Delta).
  * every product on v_mfma_f32_16x16x32 (r06; the r05 form of this loop ran 32x32x16 and
    measured level with the compiler-scheduled 8-wave kernel: its MFMAs cost 15 % more
    energy per FLOP at the power cap, where the kernel runs), on the operand maps
      A[m = l & 15][k = 8g + j], B[k = 8g + j][n = l & 15], C[m = 4g + i][n = l & 15]  (g = l >> 4):
    S / dP [16 queries mb][16 keys nb]: A = Q / dO rows 32 qb + 16 mb + (l & 15) (row
    reads), B = K / V fragments of key 16 nb + (l & 15); dV^T / dK^T [16 d md][16 keys nb]
    over the chain's 32 queries per MFMA: B = the packed P / dS of the chain's two query
    blocks, k-slot 8g + j <-> query 16 (j >> 2) + 4g + (j & 3); A = dO^T / Q^T by two 4-row
    transposed reads (rows 4g.. and 16 + 4g.., columns 16 md ..) in the same query order.

Register map (D = 64; qb the chain, mb its 16-query blocks, nb 16-key blocks, md 16-d blocks):
  AGPR  dK^T[md][nb] a[4(4md + nb)]   dV^T[md][nb] a[64 + 4(4md + nb)]
        K[nb][ks] a[128 + 4(2nb + ks)] V[nb][ks] a[160 + 4(2nb + ks)]
        Q rows[qb][mb][ks] a[192 + 4(4qb + 2mb + ks)]   dO rows a[224 + ...]
  VGPR  S[qb][nb][mb] v[32qb + 8nb + 4mb]  dP v[64 + ...]   (the two mb tuples of a key block
        adjacent: packed in place into the key block's 4-register B operand)
        seeds v[128 + 16qb + 8which + 4mb] (-LSE*log2e, -Delta tuples of each chain)
        trop ring v[160..191] (a chain's 8 dO^T / Q^T fragments)   staging v[192..223]  row const v[224]

Usage: python3 gen_bwd_dkdv.py [--check]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import asmgen  # noqa: E402
from asmgen import Ins, R, ablate, ablate_waits, fix_hazards, insert_waits, insert_waits_multi, rng, rtxt, schedule_phase, tagged, thirds, valu  # noqa: E402,E501

QT = 64  # queries per step
KEYS = 256  # keys per workgroup


class Cfg:
    def __init__(self, D, bf16):
        assert D == 64
        self.D, self.bf16 = D, bf16
        self.KS, self.NMD, self.NB, self.CPT = D // 32, D // 16, 4, D // 32
        self.exp_per_gap = 1
        # per-gap filler budget floor, 16-cycle MFMAs: 8 (r06 A/B, profiles/r06/dksched/: step -0.2 .. -0.7 %
        # against 12 in all six C3 / B2_H8_S4096 / B16_H16_S2048 cases, 16 +0.1 .. +1.2 %; 6, 4 and
        # 2 v_exp per gap within +-0.3 %, profiles/r06/sched2/)
        self.min_cap = 8
        self.TBB = QT * D * 2  # one 16-bit [64][D] tile
        # a slot: Q, dO tiles + row constants -LSE*log2e, -Delta (and a 256-B sink that waves
        # 2 and 3 write: every wave runs the same staging code)
        self.SLOT = 2 * self.TBB + 768
        self.RC = 2 * self.TBB  # row constants inside a slot
        self.KVB = 3 * self.SLOT  # K block, then V block (256 rows each)
        self.OST = D + 4
        self.mf = "v_mfma_f32_16x16x32_bf16" if bf16 else "v_mfma_f32_16x16x32_f16"
        self.cvt = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        # fp16: dS = P * dP' on the packed 16-bit halves (v_pk_mul_f16): P and dP' packed
        # first, one multiply per two products; bf16 multiplies in fp32 ('pkmul32': fp16 too)
        self.pkmul = not bf16 and "pkmul32" not in asmgen.ABL
        self.nvgpr, self.nagpr = 226, 256

    # AGPRs
    def dK(self, md, nb):
        return 4 * (4 * md + nb)

    def dV(self, md, nb):
        return 64 + 4 * (4 * md + nb)

    def Kf(self, nb, ks):
        return 128 + 4 * (2 * nb + ks)

    def Vf(self, nb, ks):
        return 160 + 4 * (2 * nb + ks)

    def Qr(self, qb, mb, ks):
        return 192 + 4 * (4 * qb + 2 * mb + ks)

    def dOr(self, qb, mb, ks):
        return 224 + 4 * (4 * qb + 2 * mb + ks)

    # VGPRs
    def S(self, qb, nb, mb=0, i=0):
        return 32 * qb + 8 * nb + 4 * mb + i

    def dP(self, qb, nb, mb=0, i=0):
        return 64 + 32 * qb + 8 * nb + 4 * mb + i

    def seed(self, qb, which, mb):
        return 128 + 16 * qb + 8 * which + 4 * mb

    def tr(self, k):
        return 160 + 4 * k

    def stg(self, tensor, cc):
        return 192 + 8 * (tensor * self.CPT + cc)

    RCV = 224

    @property
    def lds_bytes(self):
        stage = 2 * KEYS * self.OST * 4
        return max(self.KVB + 2 * KEYS * self.D * 2, stage)


def mfma(cfg, dst, a, b, c, c_is_zero=False):
    rd = R(rng(a[0], a[1], 4), "A") + R(rng(b[0], b[1], 4), "B")
    if not c_is_zero:
        rd += R(rng(c[0], c[1], 4), "C")
    ctxt = "0" if c_is_zero else rtxt(c[0], c[1], 4)
    return Ins(f"{cfg.mf} {rtxt(dst[0], dst[1], 4)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {ctxt}", "mfma",
               rd, rng(dst[0], dst[1], 4))


# ---- LDS reads --------------------------------------------------------------------------
def rowop_reads(cfg, slot):
    """Q and dO row fragments (qb, mb, ks) of the step in `slot` -> AGPRs (A operands of S, dP);
    chain A's first (chain B's S, dP of the step before may still be reading theirs)"""
    out = []
    for qb in range(2):
        for tensor in range(2):
            for mb in range(2):
                for ks in range(cfg.KS):
                    d = cfg.Qr(qb, mb, ks) if tensor == 0 else cfg.dOr(qb, mb, ks)
                    off = slot * cfg.SLOT + tensor * cfg.TBB + (32 * qb + 16 * mb) * cfg.D * 2
                    out.append(Ins(f"ds_read_b128 {rtxt('a', d, 4)}, %[ka{ks}] offset:{off}", "dsr", [],
                                   rng("a", d, 4), earliest=qb))
    return tagged("lds", out)


def seed_reads(cfg, slot, which, qb, earliest=0, deadline=None):
    """row-constant tuples (which 0: -LSE*log2e, 1: -Delta) of chain qb: register i of the
    tuple of query block mb holds row 32 qb + 16 mb + 4g + i"""
    out = []
    for mb in range(2):
        off = slot * cfg.SLOT + cfg.RC + which * 256 + (32 * qb + 16 * mb) * 4
        d = cfg.seed(qb, which, mb)
        out.append(Ins(f"ds_read_b128 {rtxt('v', d, 4)}, %[rco] offset:{off}", "dsr", [], rng("v", d, 4),
                       earliest=earliest, deadline=deadline))
    return tagged("lds", out)


def trop_frag(k):
    """the k-th A operand of a chain's dV^T / dK^T phase: (tensor 0: dO^T, 1: Q^T; md)"""
    return k // 4, k % 4


def trop_reads(cfg, slot, qb, k, earliest=0, deadline=None):
    tensor, md = trop_frag(k)
    tt = 1 if tensor == 0 else 0  # LDS tile: 0 = Q, 1 = dO
    off = slot * cfg.SLOT + tt * cfg.TBB + 32 * qb * cfg.D * 2
    d = cfg.tr(k)
    return tagged("lds", [
        Ins(f"ds_read_b64_tr_b16 {rtxt('v', d, 2)}, %[tr{md}_0] offset:{off}", "dsr", [], rng("v", d, 2),
            earliest=earliest, deadline=deadline),
        Ins(f"ds_read_b64_tr_b16 {rtxt('v', d + 2, 2)}, %[tr{md}_1] offset:{off}", "dsr", [], rng("v", d + 2, 2),
            earliest=earliest, deadline=deadline)])


# ---- MFMA chains -------------------------------------------------------------------------
def sdp_mfmas(cfg, qb):
    """chain qb: S[qb][nb][mb] = Q K^T - LSE*log2e, dP = dO V^T - Delta; key blocks 0, 1 first
    (their P, dS are the next phase's filler)"""
    out = []
    for nb in range(cfg.NB):
        for mb in range(2):
            for which in range(2):
                for ks in range(cfg.KS):
                    if which == 0:
                        dst, a, b = cfg.S(qb, nb, mb), cfg.Qr(qb, mb, ks), cfg.Kf(nb, ks)
                    else:
                        dst, a, b = cfg.dP(qb, nb, mb), cfg.dOr(qb, mb, ks), cfg.Vf(nb, ks)
                    cc = ("v", cfg.seed(qb, which, mb)) if ks == 0 else ("v", dst)
                    out.append(mfma(cfg, ("v", dst), ("a", a), ("a", b), cc))
    return out


def dkdv_mfmas(cfg, qb, first=False):
    """chain qb's share: dV^T[md][nb] += dO^T P[qb][nb], dK^T[md][nb] += Q^T dS[qb][nb]; trop
    ring fragment k feeds the four key blocks back to back"""
    out = []
    for k in range(8):
        tensor, md = trop_frag(k)
        for nb in range(cfg.NB):
            acc = cfg.dV(md, nb) if tensor == 0 else cfg.dK(md, nb)
            src = cfg.S(qb, nb) if tensor == 0 else cfg.dP(qb, nb)
            out.append(mfma(cfg, ("a", acc), ("v", cfg.tr(k)), ("v", src), ("a", acc), c_is_zero=first))
    return out


# ---- VALU ---------------------------------------------------------------------------------
def pds_part(cfg, qb, half):
    """P = exp2(S) and dS = P * dP' of key blocks 2 half, 2 half + 1 of chain qb, packed in
    place (register 2ii of the pair (2ii, 2ii + 1) -> ii: the B operand order above)"""
    out = []
    for nb in (2 * half, 2 * half + 1):
        sb, db = cfg.S(qb, nb), cfg.dP(qb, nb)
        for i in range(8):
            out.append(valu(f"v_exp_f32 v{sb + i}, v{sb + i}", [f"v{sb + i}"], [f"v{sb + i}"], kind="exp"))
        if cfg.pkmul:
            for base in (sb, db):
                for ii in range(4):
                    d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
                    out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
            for ii in range(4):
                r, d = sb + ii, db + ii
                out.append(valu(f"v_pk_mul_f16 v{d}, v{d}, v{r}", [f"v{d}", f"v{r}"], [f"v{d}"]))
            continue
        for i in range(8):
            r, d = sb + i, db + i
            out.append(valu(f"v_mul_f32 v{d}, v{d}, v{r}", [f"v{d}", f"v{r}"], [f"v{d}"]))
        for base in (sb, db):
            for ii in range(4):
                d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
                out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
    return tagged("sm", out)


# ---- staging --------------------------------------------------------------------------
def staging_loads(cfg):
    out = []
    for tensor, rs in ((0, "%[rsq]"), (1, "%[rsd]")):
        for cc in range(cfg.CPT):
            base = cfg.stg(tensor, cc)
            for h in range(2):
                off = f" offset:{16 * h}" if h else ""
                out.append(Ins(f"buffer_load_dwordx4 {rtxt('v', base + 4 * h, 4)}, %[vo{cc}], {rs}, %[goff] offen{off}",
                               "vmem", R(["s:goff"]), rng("v", base + 4 * h, 4)))
    out.append(Ins(f"buffer_load_dword v{cfg.RCV}, %[rvo], %[rsc], %[roff] offen", "vmem", R(["s:roff"]),
                   [f"v{cfg.RCV}"]))
    out.append(Ins(f"s_add_u32 %[goff], %[goff], {QT * cfg.D * 4}", "salu", R(["s:goff"]), ["s:goff", "scc"]))
    out.append(Ins(f"s_add_u32 %[roff], %[roff], {QT * 4}", "salu", R(["s:roff"]), ["s:roff", "scc"]))
    return tagged("stg", out)


def staging_convert(cfg, slot):
    out = []
    step = 256 // (cfg.D // 8)
    for tensor in range(2):
        for cc in range(cfg.CPT):
            base = cfg.stg(tensor, cc)
            for ii in range(4):
                d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
                out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
            off = slot * cfg.SLOT + tensor * cfg.TBB + cc * step * cfg.D * 2
            out.append(Ins(f"ds_write_b128 %[lo], {rtxt('v', base, 4)} offset:{off}", "dsw", R(rng("v", base, 4)), []))
    r = cfg.RCV
    out.append(valu(f"v_mul_f32 v{r}, %[rsm], v{r}", [f"v{r}"], [f"v{r}"]))
    out.append(Ins(f"ds_write_b32 %[rcw], v{r} offset:{slot * cfg.SLOT + cfg.RC}", "dsw", R([f"v{r}"]), []))
    return tagged("stg", out)


# ---- program ---------------------------------------------------------------------------
def body(cfg, j3, log):
    """one 64-query step j with j % 3 == j3: its tiles in slot j3; step j+1 staged into (j3+1)%3;
    chain B's dV/dK of step j-1 read slot (j3+2)%3"""
    s, n, pv = j3, (j3 + 1) % 3, (j3 + 2) % 3
    seq = []
    # P1: S, dP of A | P, dS of B (j-1) key blocks 2, 3; stage step j+1; B's (j-1) trop frags
    #     for P2 (the ring is free once P4's first MFMAs have read A's)
    pre = []
    for k in range(8):
        pre += trop_reads(cfg, pv, 1, k, earliest=2)
    conv = staging_convert(cfg, n)
    for i in conv:
        i.earliest = 2
    # the staging convert in P2 (the lightest phase: 47 fillers against P1's 78) and the next
    # step's loads over P3, P4: step -0.6 .. +0.1 % (5 of 6 cases <= 0), kernel -0.2 .. -1.8 %
    # in one process (profiles/r06/convp2/); 'convp1' keeps the old placement
    convp2 = "convp1" not in asmgen.ABL
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 0), [pds_part(cfg, 1, 1)] + ([] if convp2 else [conv]) + [pre],
                          f"P1.{j3}", log)
    # P2: dV, dK of B (j-1) | P, dS of A key blocks 0, 1; B's seeds for P3; loads of step j+2
    #     (staging registers free since P1's convert) spread over P2, P3, P4, the offset adds
    #     after the last of them
    sd = seed_reads(cfg, s, 0, 1) + seed_reads(cfg, s, 1, 1)
    stl = staging_loads(cfg)
    if "nospread" in asmgen.ABL:
        ld = (stl, [], [])
    elif convp2:
        h = (len(stl) - 2 + 1) // 2
        ld = ([], stl[:h], stl[h:])
        for i in conv:
            i.earliest = 0
    else:
        ld = thirds(stl[:-2])
        ld = (ld[0], ld[1], ld[2] + stl[-2:])
    seq += schedule_phase(cfg, dkdv_mfmas(cfg, 1), [pds_part(cfg, 0, 0), sd] + ([conv] if convp2 else []) + [list(ld[0])],
                          f"P2.{j3}", log)
    # P3: S, dP of B | P, dS of A key blocks 2, 3; A's trop frags for P4 (the ring is free
    #     after P2)
    pre = []
    for k in range(8):
        pre += trop_reads(cfg, s, 0, k, earliest=2)
    seq += schedule_phase(cfg, sdp_mfmas(cfg, 1), [pds_part(cfg, 0, 1), pre, list(ld[1])], f"P3.{j3}", log)
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    seq.append(tagged("bar", [Ins("s_barrier", "bar")])[0])
    # P4: dV, dK of A | P, dS of B key blocks 0, 1; Q/dO rows and A's seeds of step j+1
    #     (staged before the barrier by every wave)
    nxt = rowop_reads(cfg, n) + seed_reads(cfg, n, 0, 0, earliest=2) + seed_reads(cfg, n, 1, 0, earliest=2)
    seq += schedule_phase(cfg, dkdv_mfmas(cfg, 0), [pds_part(cfg, 1, 0), nxt, list(ld[2])], f"P4.{j3}", log)
    return seq


def prologue(cfg):
    """step 0 serially (both chains' S, dP; A's P, dS and dV, dK -- whose MFMAs start every
    accumulator from zero; B's key blocks 0, 1), step 1 staged"""
    D = cfg.D
    seq = staging_loads(cfg)  # step 1
    # K and V fragments of the wave's 64 keys from the workgroup's K / V blocks (%[kvb]: this
    # wave's rows)
    for ks in range(cfg.KS):
        seq.append(valu(f"v_add_u32 v{ks}, %[kvb], %[ka{ks}]", [], [f"v{ks}"]))
    for nb in range(cfg.NB):
        for ks in range(cfg.KS):
            seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.Kf(nb, ks), 4)}, v{ks} offset:{nb * 16 * D * 2}", "dsr",
                           R([f"v{ks}"]), rng("a", cfg.Kf(nb, ks), 4)))
            seq.append(Ins(f"ds_read_b128 {rtxt('a', cfg.Vf(nb, ks), 4)}, v{ks} offset:{KEYS * D * 2 + nb * 16 * D * 2}",
                           "dsr", R([f"v{ks}"]), rng("a", cfg.Vf(nb, ks), 4)))
    seq += rowop_reads(cfg, 0)
    for qb in range(2):
        seq += seed_reads(cfg, 0, 0, qb) + seed_reads(cfg, 0, 1, qb)
        seq += sdp_mfmas(cfg, qb)
    seq += pds_part(cfg, 0, 0) + pds_part(cfg, 0, 1) + pds_part(cfg, 1, 0)
    mf = dkdv_mfmas(cfg, 0, first=True)
    for k in range(8):
        seq += trop_reads(cfg, 0, 0, k)
        seq += mf[4 * k:4 * k + 4]
    seq += staging_convert(cfg, 1)
    seq += staging_loads(cfg)  # step 2
    seq += [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_barrier", "bar")]
    seq += rowop_reads(cfg, 1) + seed_reads(cfg, 1, 0, 0) + seed_reads(cfg, 1, 1, 0)
    return seq


def epilogue(cfg, last_slot_expr):
    """after the last step: B's key blocks 2, 3, its dV, dK; stage dK^T, dV^T (last slot: the
    body that exits passes its slot)"""
    seq = [Ins("s_waitcnt vmcnt(0) lgkmcnt(0)", "wait")]
    seq += pds_part(cfg, 1, 1)
    mf = dkdv_mfmas(cfg, 1)
    for k in range(8):
        seq += trop_reads(cfg, last_slot_expr, 1, k)
        seq += mf[4 * k:4 * k + 4]
    seq.append(Ins("s_barrier", "bar"))
    # dK^T[md][nb] register i: d = 16 md + 4g + i of key 16 nb + (l & 15) -> stage row, 4 columns
    for tensor, op in ((0, "%[oak]"), (1, "%[oav]")):
        for md in range(cfg.NMD):
            for nb in range(cfg.NB):
                r = cfg.dK(md, nb) if tensor == 0 else cfg.dV(md, nb)
                off = (16 * nb * cfg.OST + 16 * md) * 4
                seq.append(Ins(f"ds_write_b128 {op}, {rtxt('a', r, 4)} offset:{off}", "dsw", R(rng("a", r, 4)), []))
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    return seq


def build(cfg):
    log = [f"dK/dV D={cfg.D} {'bf16' if cfg.bf16 else 'fp16'}: {cfg.nvgpr} VGPRs + {cfg.nagpr} AGPRs in asm, "
           f"LDS {cfg.lds_bytes} B"]
    pro = prologue(cfg)
    bodies = [ablate(body(cfg, j3, log)) for j3 in (1, 2, 0)]
    empty = ((), ())
    pro, st = insert_waits(pro, empty)
    # the loop head is entered from the prologue and from the back edge: iterate the set of
    # possible wait states there to a fixed point, waits valid for all of them
    heads = [st]
    for _ in range(8):
        done, cur = [], heads
        for b in bodies:
            b2, cur = insert_waits_multi(b, cur)
            done.append(b2)
        new = [x for x in cur if x not in heads]
        if not new or asmgen.ABL:
            break
        heads = heads + new
    else:
        raise AssertionError("loop-carried wait states do not converge")
    done = [ablate_waits(b) for b in done]
    # three epilogues: the last step's slot is that of the body that exits
    epis = []
    for j3 in (1, 2, 0):
        e, _ = insert_waits(epilogue(cfg, j3), empty)
        epis.append(e)
    ctl = lambda lab, cmp: [Ins("s_sub_u32 %[cnt], %[cnt], 1", "salu", R(["s:cnt"]), ["s:cnt", "scc"]),
                            Ins(f"{cmp} %[cnt], 0", "salu", R(["s:cnt"]), ["scc"]),
                            Ins(f"s_cbranch_scc1 {lab}", "branch", R(["scc"]))]
    done[0] += ctl("FA2DK_EPI1_%=", "s_cmp_eq_u32")
    done[1] += ctl("FA2DK_EPI2_%=", "s_cmp_eq_u32")
    done[2] += ctl("FA2DK_LOOP_%=", "s_cmp_lg_u32") + [Ins("s_branch FA2DK_EPI0_%=", "branch")]
    for _ in range(3):
        pro = fix_hazards(pro, [[]])
        done[0] = fix_hazards(done[0], [pro[-40:], done[2][-40:]])
        done[1] = fix_hazards(done[1], [done[0][-40:]])
        done[2] = fix_hazards(done[2], [done[1][-40:]])
        for k in range(3):
            epis[k] = fix_hazards(epis[k], [done[k][-40:]])
    lines = [i.text for i in pro] + ["FA2DK_LOOP_%=:"]
    for k in range(3):
        lines += [i.text for i in done[k]]
    for k, lab in enumerate(("FA2DK_EPI1_%=", "FA2DK_EPI2_%=", "FA2DK_EPI0_%=")):
        lines += [lab + ":"] + [i.text for i in epis[k]]
        if k < 2:
            lines.append("s_branch FA2DK_END_%=")
    lines.append("FA2DK_END_%=:")
    allb = done[0] + done[1] + done[2]
    nm = sum(1 for i in allb if i.kind == "mfma")
    nv = sum(1 for i in allb if i.kind in ("valu", "exp"))
    nl = sum(1 for i in allb if i.kind == "dsr")
    nn = sum(int(i.text.split()[1]) + 1 for i in allb if i.kind == "nop")
    log.append(f"  loop (3 steps): {nm} MFMA, {nv} VALU ({nv / max(nm, 1):.2f} per MFMA), {nl} LDS reads "
               f"({nl / max(nm, 1):.2f} per MFMA), {nn} nop wait states, {len(allb)} instructions")
    return lines, log


def operands(cfg):
    outs = ['[cnt] "+s"(hs_cnt)', '[goff] "+s"(hs_goff)', '[roff] "+s"(hs_roff)']
    ins = [f'[ka{ks}] "v"(hs_ka[{ks}])' for ks in range(cfg.KS)]
    ins += [f'[tr{md}_{k}] "v"(hs_tr[{md}][{k}])' for md in range(cfg.NMD) for k in range(2)]
    ins += [f'[vo{c}] "v"(hs_vo[{c}])' for c in range(cfg.CPT)]
    ins += ['[lo] "v"(hs_lo)', '[rco] "v"(hs_rco)', '[rvo] "v"(hs_rvo)', '[rcw] "v"(hs_rcw)', '[oak] "v"(hs_oak)',
            '[oav] "v"(hs_oav)', '[rsq] "s"(hs_rsq)', '[rsd] "s"(hs_rsd)', '[rsc] "s"(hs_rsc)', '[rsm] "s"(hs_rsm)',
            '[kvb] "s"(hs_kvb)']
    clob = [f'"v{i}"' for i in range(cfg.nvgpr)] + [f'"a{i}"' for i in range(cfg.nagpr)] + ['"vcc"', '"scc"', '"memory"']
    return outs, ins, clob


def emit():
    here = os.path.dirname(os.path.abspath(__file__))
    out = ["// Generated by cuda-flash-attention_amd/gen/gen_bwd_dkdv.py -- do not edit.",
           "// Hand-scheduled dK/dV loop of fa2_bwd_dkdv_hs_kernel<D> (f-attn2-backward_f16.cu).",
           "#pragma once", ""]
    logs = []
    for bf16 in (False, True):
        cfg = Cfg(64, bf16)
        lines, log = build(cfg)
        logs += log
        out.append(f"#define FA2_DK_ASM_D64_{'BF16' if bf16 else 'F16'} \\")
        out += [f'    "{ln}\\n\\t" \\' for ln in lines]
        out.append('    ""')
        out.append("")
    cfg = Cfg(64, False)
    o, i, c = operands(cfg)
    out.append("#define FA2_DK_OUTPUTS_D64 " + ", ".join(o))
    out.append("#define FA2_DK_INPUTS_D64 " + ", ".join(i))
    out.append("#define FA2_DK_CLOBBERS_D64 " + ", ".join(c))
    out.append(f"#define FA2_DK_LDS_D64 {cfg.lds_bytes}")
    out.append(f"#define FA2_DK_SLOT_D64 {cfg.SLOT}")
    out.append(f"#define FA2_DK_RC_D64 {cfg.RC}")
    out.append(f"#define FA2_DK_KVB_D64 {cfg.KVB}")
    out.append("")
    out = ["// " + ln for ln in logs] + out
    text = "\n".join(out) + "\n"
    path = os.path.join(here, "..", "kernels", "fa2_bwd_dkdv_hs.inc")
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
    if "--check" in sys.argv:
        cur = open(path).read() if os.path.exists(path) else ""
        if cur != text:
            print("fa2_bwd_dkdv_hs.inc is stale: run gen/gen_bwd_dkdv.py")
            sys.exit(1)
        return
    with open(path, "w") as f:
        f.write(text)
    print("\n".join(logs))


if __name__ == "__main__":
    asmgen.parse_abl(sys.argv)
    emit()
