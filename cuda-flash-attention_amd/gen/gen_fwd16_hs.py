#!/usr/bin/env python3
"""Generator of the hand-scheduled forward tile loop on v_mfma_f32_16x16x32 (gfx950).

Writes ../kernels/fa2_fwd16_hs.inc: the inline-asm body of `fa2_fwd_hs_kernel<D, true>`
(kernel_fa2_optimized_f16.cu), D = 64 and 128.  Same algorithm, workgroup shape, phases,
staging and restart guard as gen_fwd_hs.py (the 32x32x16 form; its docstring has the
structure), on the 16x16x32 operand maps

  A[m = l & 15][k = 8g + j], B[k = 8g + j][n = l & 15], C[m = 4g + i][n = l & 15]  (g = l >> 4):

  * each wave's 64 query rows are four 16-row blocks on the lane (l & 15); chain c holds
    blocks 2c and 2c + 1 (qb = 0, 1);
  * S^T tiles [16 keys][16 queries]: A = K row fragments (rows 16 kb + (l & 15), columns
    32 ks + 8g), B = the chain's Q fragments; the first MFMA of a tile starts from the -m
    splat of its query block (4 registers);
  * O^T[16 d][16 q] += V^T P^T over 32 keys per MFMA: B = the packed P of two key blocks
    (k-slot 8g + j <-> key 16 (j >> 2) + 4g + (j & 3)), A = V^T by two 4-row transposed
    reads (rows 4g.. and 16 + 4g.., columns 16 db ..) in the same key order;
  * each lane sums its own keys of a row (16 of the tile's 64); the four lane groups g of
    a row meet in the epilogue (and once in the prologue, for the first tile's row max).

16x16x32 reads and writes a quarter of the accumulator per instruction for half the FLOPs:
less energy per FLOP at the power cap, where the kernels run.

Register map (D = head dim, KS = D/32, NDB = D/16):
  AGPR  O^T[c][db][qb]  a[4 (2 NDB c + 2 db + qb)]    Q[c][qb][ks] a[16 NDB + 4 (2 KS c + KS qb + ks)]
        V^T frags       a[16 NDB + 16 KS + 4 i]
  VGPR  S^T[c][qb][kb]  v[32c + 16qb + 4kb]    -m splat[c][qb] v[64 + 4 (2c + qb)]
        K ring          v[80 + 4r], r < 8      staging v[112 ...]   misc (m, l, partial sums)

Usage: python3 gen_fwd16_hs.py [--check]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import asmgen  # noqa: E402
from asmgen import Ins, R, ablate, ablate_waits, fix_hazards, insert_waits, rng, rtxt, schedule_phase, stamp, tagged, valu  # noqa: E402,E501

KT = 64  # keys per tile
SUM_MAX_BITS = 0x46000000  # 8192.0f: tile-sum guard (FA2_TILE_SUM_MAX)


class Cfg:
    def __init__(self, D, bf16):
        self.D, self.bf16 = D, bf16
        self.KS, self.NDB, self.CPT = D // 32, D // 16, D // 32
        self.NKF = 4 * self.KS  # K row fragments per tile: (kb, ks)
        self.NVF = 2 * self.NDB  # V^T fragments per tile: (db, s)
        self.ring = 8
        self.keep_k = self.NKF <= self.ring
        self.QB = 16 * self.NDB
        self.VB = self.QB + 16 * self.KS
        self.nagpr = self.VB + 4 * self.NVF
        self.STG = 112
        self.MB = self.STG + 16 * self.CPT
        self.nvgpr = self.MB + 20
        self.SV = self.nvgpr
        if "stamps" in asmgen.ABL:
            self.nvgpr += 2
        self.TBB = KT * D * 2
        self.OST = D + 4
        self.mf = "v_mfma_f32_16x16x32_bf16" if bf16 else "v_mfma_f32_16x16x32_f16"
        self.cvt = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.exp_per_gap = 1
        self.min_cap = 12

    # AGPRs
    def O(self, c, db, qb):
        return 4 * (2 * self.NDB * c + 2 * db + qb)

    def Q(self, c, qb, ks):
        return self.QB + 4 * (2 * self.KS * c + self.KS * qb + ks)

    def Vf(self, i):
        return self.VB + 4 * i

    # VGPRs
    def S(self, c, qb, kb, i=0):
        return 32 * c + 16 * qb + 4 * kb + i

    def NM(self, c, qb):
        return 64 + 4 * (2 * c + qb)

    def Kr(self, r):
        return 80 + 4 * r

    def stg(self, tensor, cc):
        return self.STG + 8 * (tensor * self.CPT + cc)

    def m(self, c, qb):
        return self.MB + 2 * c + qb

    def l(self, c, qb):
        return self.MB + 4 + 2 * c + qb

    def T(self, c, qb, k):
        return self.MB + 8 + 4 * c + 2 * qb + k

    def ts(self, c):
        return self.MB + 16 + c

    def tmp(self, k):
        return self.MB + 18 + k

    # LDS byte offsets
    def koff(self, slot):
        return slot * self.TBB

    def voff(self, slot):
        return (2 + slot) * self.TBB

    @property
    def lds_bytes(self):
        return max(8 * self.TBB, 256 * self.OST * 4)


# ---------------------------------------------------------------------------------------
# instruction builders
# ---------------------------------------------------------------------------------------
def mfma(cfg, dst, a, b, c, c_is_zero=False):
    rd = R(rng(a[0], a[1], 4), "A") + R(rng(b[0], b[1], 4), "B")
    if not c_is_zero:
        rd += R(rng(c[0], c[1], 4), "C")
    ctxt = "0" if c_is_zero else rtxt(c[0], c[1], 4)
    return Ins(f"{cfg.mf} {rtxt(dst[0], dst[1], 4)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {ctxt}", "mfma",
               rd, rng(dst[0], dst[1], 4))


def kfrag(cfg, f):
    """K row fragment f of a tile: (kb, ks)"""
    return f // cfg.KS, f % cfg.KS


def kfrag_read(cfg, f, slot, dst):
    kb, ks = kfrag(cfg, f)
    off = cfg.koff(slot) + kb * 16 * cfg.D * 2
    return tagged("lds", [Ins(f"ds_read_b128 {rtxt('v', dst, 4)}, %[ka{ks}] offset:{off}", "dsr", [], rng("v", dst, 4))])[0]


def vfrag_reads(cfg, i, slot, earliest=0):
    db, s = i // 2, i % 2
    off = cfg.voff(slot) + s * 32 * cfg.D * 2
    d = cfg.Vf(i)
    return tagged("lds", [
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d, 2)}, %[va{db}_0] offset:{off}", "dsr", [], rng("a", d, 2),
            earliest=earliest),
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d + 2, 2)}, %[va{db}_1] offset:{off}", "dsr", [], rng("a", d + 2, 2),
            earliest=earliest),
    ])


def qk_mfmas(cfg, c, kreg, zero=False):
    """S^T[c][qb][kb] = K Q^T[c][qb] - m[c][qb]: key-block-major, so half 0 (kb 0, 1) finishes
    first and K fragment (kb, ks) is free after its second use"""
    out = []
    for kb in range(4):
        for qb in range(2):
            for ks in range(cfg.KS):
                f = kb * cfg.KS + ks
                if zero:
                    cc, z = ("v", cfg.S(c, qb, kb)), ks == 0
                else:
                    cc, z = (("v", cfg.NM(c, qb)) if ks == 0 else ("v", cfg.S(c, qb, kb))), False
                out.append(mfma(cfg, ("v", cfg.S(c, qb, kb)), ("v", kreg(f)), ("a", cfg.Q(c, qb, ks)), cc, c_is_zero=z))
    return out


def pv_mfmas(cfg, c, first=False):
    """O^T[c][db][qb] += V^T[db][s] P^T[c][qb][s]: V^T slot i = 2 db + s is free after its two MFMAs"""
    out = []
    for db in range(cfg.NDB):
        for s in range(2):
            for qb in range(2):
                z = first and s == 0
                out.append(mfma(cfg, ("a", cfg.O(c, db, qb)), ("a", cfg.Vf(2 * db + s)), ("v", cfg.S(c, qb, 2 * s)),
                                ("a", cfg.O(c, db, qb)), c_is_zero=z))
    return out


def softmax_part(cfg, c, s, final):
    """exp2 of key half s (key blocks 2s, 2s+1: 8 scores of each of the lane's two rows), the
    rows' partial sums (round robin over the four partial registers), packed in place"""
    out = []
    base = [cfg.S(c, qb, 2 * s) for qb in range(2)]
    for qb in range(2):
        for e in range(8):
            r = base[qb] + e
            out.append(valu(f"v_exp_f32 v{r}, v{r}", [f"v{r}"], [f"v{r}"], kind="exp"))
    adds = []
    if s == 0:
        for k in range(2):
            for qb in range(2):
                T, a, b = cfg.T(c, qb, k), base[qb] + 2 * k, base[qb] + 2 * k + 1
                adds.append(valu(f"v_add_f32 v{T}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{T}"]))
        rest = [4, 5, 6, 7]
    else:
        rest = list(range(8))
    # element e of row qb goes to partial k = (e >> 1) & 1
    for j in range(len(rest)):
        for qb in range(2):
            e = rest[j]
            k = (e >> 1) & 1
            T, r = cfg.T(c, qb, k), base[qb] + e
            adds.append(valu(f"v_add_f32 v{T}, v{T}, v{r}", [f"v{T}", f"v{r}"], [f"v{T}"]))
    out += _interleave_adds(adds)
    for qb in range(2):
        for ii in range(4):
            d, a, b = base[qb] + ii, base[qb] + 2 * ii, base[qb] + 2 * ii + 1
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
    tagged("sm", out)
    if final:
        t0, t1, ts = cfg.tmp(0), cfg.tmp(1), cfg.ts(c)
        fin = [valu(f"v_add_f32 v{t0}, v{cfg.T(c, 0, 0)}, v{cfg.T(c, 0, 1)}", [f"v{cfg.T(c, 0, 0)}", f"v{cfg.T(c, 0, 1)}"],
                    [f"v{t0}"]),
               valu(f"v_add_f32 v{t1}, v{cfg.T(c, 1, 0)}, v{cfg.T(c, 1, 1)}", [f"v{cfg.T(c, 1, 0)}", f"v{cfg.T(c, 1, 1)}"],
                    [f"v{t1}"]),
               valu(f"v_add_f32 v{cfg.l(c, 0)}, v{cfg.l(c, 0)}, v{t0}", [f"v{cfg.l(c, 0)}", f"v{t0}"], [f"v{cfg.l(c, 0)}"]),
               valu(f"v_add_f32 v{cfg.l(c, 1)}, v{cfg.l(c, 1)}, v{t1}", [f"v{cfg.l(c, 1)}", f"v{t1}"], [f"v{cfg.l(c, 1)}"]),
               valu(f"v_add_f32 v{ts}, v{t0}, v{t1}", [f"v{t0}", f"v{t1}"], [f"v{ts}"]),
               # NaN or a lane's tile sum above 2^13 -> the block is recomputed by the robust path
               valu(f"v_cmp_nge_f32 vcc, {SUM_MAX_BITS:#x}, v{ts}", [f"v{ts}"], ["vcc"])]
        out += tagged("sm", fin)
        flag = Ins("s_or_b64 %[flg], %[flg], vcc", "salu", R(["vcc", "s:flg"]), ["s:flg"])
        flag.tag = "flag"
        out.append(flag)
    return out


def _interleave_adds(adds):
    """keep consecutive adds off the same partial register where the stream allows it"""
    out, pending = [], list(adds)
    while pending:
        last = out[-1].wr[0] if out else None
        pick = next((k for k, a in enumerate(pending) if a.wr[0] != last and
                     all(a.wr[0] != b.wr[0] for b in pending[:k])), 0)
        out.append(pending.pop(pick))
    return out


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
    return tagged("stg", [Ins(f"s_add_u32 %[goff], %[goff], {KT * cfg.D * 4}", "salu", R(["s:goff"]), ["s:goff", "scc"])])[0]


def staging_convert(cfg, tensor, slot):
    out = []
    toff = cfg.koff(slot) if tensor == 0 else cfg.voff(slot)
    rows_per_chunk_step = 256 // (cfg.D // 8)
    for cc in range(cfg.CPT):
        base = cfg.stg(tensor, cc)
        for ii in range(4):
            d, a, b = base + ii, base + 2 * ii, base + 2 * ii + 1
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
        off = toff + cc * rows_per_chunk_step * cfg.D * 2
        out.append(Ins(f"ds_write_b128 %[lo], {rtxt('v', base, 4)} offset:{off}", "dsw", R(rng("v", base, 4)), []))
    return tagged("stg", out)


# ---------------------------------------------------------------------------------------
# program pieces
# ---------------------------------------------------------------------------------------
def kring_reads(cfg, slot):
    """D = 128: K fragments 8.. into the ring slots of fragments 0..7 once the last MFMA
    reading the old fragment has issued, a few MFMAs before the first one reading the new"""
    use = lambda f, qb: (f // cfg.KS) * 2 * cfg.KS + qb * cfg.KS + f % cfg.KS  # qk_mfmas order
    out = []
    for f in range(cfg.ring, cfg.NKF):
        r = f - cfg.ring
        ins = kfrag_read(cfg, f, slot, cfg.Kr(r))
        ins.earliest, ins.deadline = use(r, 1) + 1, use(f, 0) - 3
        assert ins.earliest <= ins.deadline
        out.append(ins)
    return out


def body(cfg, p, log):
    """one 64-key tile j with parity p: K/V of tile j in slot p; tile j+1 staged into 1-p"""
    q = 1 - p
    NKF = cfg.NKF
    ring = lambda f: cfg.Kr(f % cfg.ring)
    seq = []
    # P1: QK^T of chain A (tile j) | softmax B (j-1) second half, K fragments 8.. (D=128), stage K(j+1)
    kreads = [] if cfg.keep_k else kring_reads(cfg, p)
    conv = staging_convert(cfg, 0, q)
    for ins in conv:
        ins.earliest = len(qk_mfmas(cfg, 0, ring)) // 4
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, qk_mfmas(cfg, 0, ring), [softmax_part(cfg, 1, 1, True), kreads, conv], f"P1.{p}", log)
    seq += stamp(cfg.SV)
    # P2: PV of chain B (tile j-1) | softmax A (j) first half, V(j+1) staged, K(j+2) loads,
    #     K re-read 0..7 (D=128), first V(j) fragments into freed V slots
    nsplit = cfg.NVF // 4 if cfg.D > 64 else 0
    vre = []
    for i in range(nsplit):
        vre += vfrag_reads(cfg, i, p, earliest=2 * i + 2)
    rer = [] if cfg.keep_k else [kfrag_read(cfg, f, p, cfg.Kr(f)) for f in range(cfg.ring)]
    seq += schedule_phase(cfg, pv_mfmas(cfg, 1), [softmax_part(cfg, 0, 0, False), staging_convert(cfg, 1, q),
                                                  staging_loads(cfg, 0), rer, vre], f"P2.{p}", log)
    seq += stamp(cfg.SV)
    # P3: QK^T of chain B (tile j) | softmax A (j) second half, K fragments 8.. (D=128), rest of V(j)
    kreads = [] if cfg.keep_k else kring_reads(cfg, p)
    vre = []
    for i in range(nsplit, cfg.NVF):
        vre += vfrag_reads(cfg, i, p)
    seq += schedule_phase(cfg, qk_mfmas(cfg, 1, ring), [softmax_part(cfg, 0, 1, True), kreads, vre], f"P3.{p}", log)
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    seq += stamp(cfg.SV)
    seq.append(tagged("bar", [Ins("s_barrier", "bar")])[0])
    seq += stamp(cfg.SV)
    # P4: PV of chain A (tile j) | softmax B (j) first half, K(j+1) fragment prefetch, V(j+2) loads
    pre = [kfrag_read(cfg, f, q, cfg.Kr(f)) for f in range(min(cfg.ring, NKF))]
    seq += schedule_phase(cfg, pv_mfmas(cfg, 0), [softmax_part(cfg, 1, 0, False), pre,
                                                  staging_loads(cfg, 1) + [goff_inc(cfg)]], f"P4.{p}", log)
    return seq


def lane_group_max(cfg, m):
    """m = max over the four lane groups g of each row (lanes l, l ^ 16, l ^ 32, l ^ 48)"""
    t0, t1 = cfg.tmp(0), cfg.tmp(1)
    out = []
    for sw in ("v_permlane16_swap_b32", "v_permlane32_swap_b32"):
        out.append(valu(f"v_mov_b32 v{t0}, v{m}", [f"v{m}"], [f"v{t0}"]))
        out.append(valu(f"v_mov_b32 v{t1}, v{m}", [f"v{m}"], [f"v{t1}"]))
        out.append(valu(f"{sw} v{t0}, v{t1}", [f"v{t0}", f"v{t1}"], [f"v{t0}", f"v{t1}"]))
        out.append(valu(f"v_max_f32 v{m}, v{t0}, v{t1}", [f"v{t0}", f"v{t1}"], [f"v{m}"]))
    return out


def prologue(cfg):
    D, NKF = cfg.D, cfg.NKF
    seq = [Ins("s_mov_b32 s98, 0", "salu", [], ["s98"])] if "stamps" in asmgen.ABL else []
    seq += stamp(cfg.SV)
    seq += [Ins("s_mov_b64 %[flg], 0", "salu", [], ["s:flg"])]
    for c in range(2):
        for qb in range(2):
            seq.append(valu(f"v_mov_b32 v{cfg.l(c, qb)}, 0", [], [f"v{cfg.l(c, qb)}"]))
    # tile 1 loads (K then V)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    # Q fragments of both chains -> AGPRs (Q block in LDS at %[qb] + this wave's rows)
    for ks in range(cfg.KS):
        seq.append(valu(f"v_add_u32 v{ks}, %[qb], %[ka{ks}]", [], [f"v{ks}"]))
    for c in range(2):
        for qb in range(2):
            for ks in range(cfg.KS):
                d = cfg.Q(c, qb, ks)
                seq.append(Ins(f"ds_read_b128 {rtxt('a', d, 4)}, v{ks} offset:{(32 * c + 16 * qb) * D * 2}", "dsr",
                               R([f"v{ks}"]), rng("a", d, 4)))
    # S^T of tile 0 for both chains (no -m seed yet): K fragments in ring passes of 8
    ring = lambda f: cfg.Kr(f % cfg.ring)
    mf = qk_mfmas(cfg, 0, ring, zero=True), qk_mfmas(cfg, 1, ring, zero=True)
    per_pass = cfg.ring // cfg.KS  # key blocks per ring pass
    for p0 in range(0, 4, per_pass):
        for f in range(p0 * cfg.KS, (p0 + per_pass) * cfg.KS):
            seq.append(kfrag_read(cfg, f, 0, ring(f)))
        for c in range(2):
            n = 2 * cfg.KS  # MFMAs per key block and chain
            seq += mf[c][p0 * n:(p0 + per_pass) * n]
    # row max per (chain, query block): the lane's 16 scores, then across the lane groups
    for c in range(2):
        for qb in range(2):
            m = cfg.m(c, qb)
            regs = [cfg.S(c, qb, kb, i) for kb in range(4) for i in range(4)]
            seq.append(valu(f"v_max3_f32 v{m}, v{regs[0]}, v{regs[1]}, v{regs[2]}", [f"v{r}" for r in regs[:3]],
                            [f"v{m}"]))
            k = 3
            while k + 1 < len(regs):
                seq.append(valu(f"v_max3_f32 v{m}, v{m}, v{regs[k]}, v{regs[k + 1]}",
                                [f"v{m}", f"v{regs[k]}", f"v{regs[k + 1]}"], [f"v{m}"]))
                k += 2
            if k < len(regs):
                seq.append(valu(f"v_max_f32 v{m}, v{m}, v{regs[k]}", [f"v{m}", f"v{regs[k]}"], [f"v{m}"]))
            seq += lane_group_max(cfg, m)
    # -m splats (the QK^T seeds) and s - m of tile 0
    for c in range(2):
        for qb in range(2):
            m, nm = cfg.m(c, qb), cfg.NM(c, qb)
            seq.append(valu(f"v_sub_f32 v{nm}, 0, v{m}", [f"v{m}"], [f"v{nm}"]))
            for i in range(1, 4):
                seq.append(valu(f"v_mov_b32 v{nm + i}, v{nm}", [f"v{nm}"], [f"v{nm + i}"]))
            for kb in range(4):
                for i in range(4):
                    r = cfg.S(c, qb, kb, i)
                    seq.append(valu(f"v_sub_f32 v{r}, v{r}, v{m}", [f"v{r}", f"v{m}"], [f"v{r}"]))
    seq += softmax_part(cfg, 0, 0, False) + softmax_part(cfg, 0, 1, True) + softmax_part(cfg, 1, 0, False)
    # V(0) fragments, O[B] = 0, PV of chain A (tile 0)
    for i in range(cfg.NVF):
        seq += vfrag_reads(cfg, i, 0)
    for db in range(cfg.NDB):
        for qb in range(2):
            for i in range(4):
                r = cfg.O(1, db, qb) + i
                seq.append(valu(f"v_accvgpr_write_b32 a{r}, 0", [], [f"a{r}"]))
    seq += pv_mfmas(cfg, 0, first=True)
    # tile 1 -> slot 1, tile 2 loads, barrier, K(1) fragment prefetch
    seq += staging_convert(cfg, 0, 1) + staging_convert(cfg, 1, 1)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    seq += [Ins("s_waitcnt lgkmcnt(0)", "wait"), Ins("s_barrier", "bar")]
    seq += [kfrag_read(cfg, f, 1, cfg.Kr(f)) for f in range(min(cfg.ring, NKF))]
    seq += stamp(cfg.SV)
    return seq


def epilogue(cfg):
    seq = [Ins("s_waitcnt vmcnt(0) lgkmcnt(0)", "wait")]
    seq += stamp(cfg.SV)
    seq += softmax_part(cfg, 1, 1, True)
    seq += pv_mfmas(cfg, 1)
    # every wave is done with the tile slots before the O stage overwrites them
    seq.append(Ins("s_barrier", "bar"))
    # O^T[c][db][qb] reg i: d = 16 db + 4g + i, query 32c + 16qb + (l & 15): 4 columns of a stage row
    for c in range(2):
        for db in range(cfg.NDB):
            for qb in range(2):
                r = cfg.O(c, db, qb)
                off = ((32 * c + 16 * qb) * cfg.OST + 16 * db) * 4
                seq.append(Ins(f"ds_write_b128 %[oa], {rtxt('a', r, 4)} offset:{off}", "dsw", R(rng("a", r, 4)), []))
    for c in range(2):
        for qb in range(2):
            i = 2 * c + qb
            seq.append(valu(f"v_mov_b32 %[om{i}], v{cfg.m(c, qb)}", [f"v{cfg.m(c, qb)}"], []))
            seq.append(valu(f"v_mov_b32 %[ol{i}], v{cfg.l(c, qb)}", [f"v{cfg.l(c, qb)}"], []))
    if "stamps" in asmgen.ABL:
        # the stamps through %[sa] (the 32x32 build's stage address: row l & 31, column
        # 4 (l >> 5) + 2), so tools/stamps_hs.py decodes both builds alike; l = 1/4 per
        # lane group, so the epilogue stores the stage as is
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
        seq += [valu(f"v_mov_b32 %[ol{i}], 0.25", [], []) for i in range(4)]
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    return seq


# ---------------------------------------------------------------------------------------
# whole program
# ---------------------------------------------------------------------------------------
def build(cfg):
    log = [f"D={cfg.D} {'bf16' if cfg.bf16 else 'fp16'} (16x16x32): {cfg.nvgpr} VGPRs + {cfg.nagpr} AGPRs in asm, "
           f"LDS {cfg.lds_bytes} B"]
    pro = prologue(cfg)
    b1 = ablate(body(cfg, 1, log))
    b0 = ablate(body(cfg, 0, log))
    epi = epilogue(cfg)
    empty = ((), ())
    pro, st_p = insert_waits(pro, empty)
    b1, st_1 = insert_waits(b1, st_p)
    b0, st_0 = insert_waits(b0, st_1)
    assert asmgen.ABL or st_0 == st_p, "loop-carried wait state differs between the prologue exit and the loop back edge"
    epi, _ = insert_waits(epi, ((), ()))  # starts with a full drain
    b1, b0 = ablate_waits(b1), ablate_waits(b0)
    loop_ctl1 = [Ins("s_sub_u32 %[cnt], %[cnt], 1", "salu", R(["s:cnt"]), ["s:cnt", "scc"]),
                 Ins("s_cmp_eq_u32 %[cnt], 0", "salu", R(["s:cnt"]), ["scc"]),
                 Ins("s_cbranch_scc1 FA2HS_EPI_%=", "branch", R(["scc"]))]
    loop_ctl0 = [Ins("s_sub_u32 %[cnt], %[cnt], 1", "salu", R(["s:cnt"]), ["s:cnt", "scc"]),
                 Ins("s_cmp_lg_u32 %[cnt], 0", "salu", R(["s:cnt"]), ["scc"]),
                 Ins("s_cbranch_scc1 FA2HS_LOOP_%=", "branch", R(["scc"]))]
    b1 = b1 + loop_ctl1
    b0 = b0 + loop_ctl0
    for _ in range(3):
        pro = fix_hazards(pro, [[]])
        b1 = fix_hazards(b1, [pro[-40:], b0[-40:]])
        b0 = fix_hazards(b0, [b1[-40:]])
        epi = fix_hazards(epi, [b1[-40:], b0[-40:]])
    lines = [i.text for i in pro] + ["FA2HS_LOOP_%=:"] + [i.text for i in b1] + [i.text for i in b0] + \
            ["FA2HS_EPI_%=:"] + [i.text for i in epi]
    nm = sum(1 for i in b1 + b0 if i.kind == "mfma")
    nv = sum(1 for i in b1 + b0 if i.kind in ("valu", "exp"))
    nn = sum(int(i.text.split()[1]) + 1 for i in b1 + b0 if i.kind == "nop")
    log.append(f"  loop (2 tiles): {nm} MFMA, {nv} VALU ({nv / max(nm, 1):.2f} per MFMA), {nn} nop wait states, "
               f"{len(b1) + len(b0)} instructions")
    return lines, log


def operands(cfg):
    outs = [f'[om{i}] "=&v"(hs_m[{i}])' for i in range(4)] + [f'[ol{i}] "=&v"(hs_l[{i}])' for i in range(4)]
    outs += ['[flg] "=&s"(hs_flag)', '[cnt] "+s"(hs_cnt)', '[goff] "+s"(hs_goff)']
    ins = [f'[ka{ks}] "v"(hs_ka[{ks}])' for ks in range(cfg.KS)]
    ins += [f'[va{db}_{k}] "v"(hs_va[{db}][{k}])' for db in range(cfg.NDB) for k in range(2)]
    ins += [f'[vo{c}] "v"(hs_vo[{c}])' for c in range(cfg.CPT)]
    ins += ['[lo] "v"(hs_lo)', '[oa] "v"(hs_oa)', '[rsk] "s"(hs_rsk)', '[rsv] "s"(hs_rsv)', '[qb] "s"(hs_qb)']
    if "stamps" in asmgen.ABL:
        ins.append('[sa] "v"(hs_sa)')
    clob = [f'"v{i}"' for i in range(cfg.nvgpr)] + [f'"a{i}"' for i in range(cfg.nagpr)] + ['"vcc"', '"scc"', '"memory"']
    if "stamps" in asmgen.ABL:
        clob += asmgen.STAMP_CLOBBERS
    return outs, ins, clob


def emit():
    here = os.path.dirname(os.path.abspath(__file__))
    out = ["// Generated by cuda-flash-attention_amd/gen/gen_fwd16_hs.py -- do not edit.",
           "// Hand-scheduled 16x16x32 forward tile loop of fa2_fwd_hs_kernel<D, true> (kernel_fa2_optimized_f16.cu).",
           "#pragma once", ""]
    logs = []
    for D in (64, 128):
        for bf16 in (False, True):
            cfg = Cfg(D, bf16)
            lines, log = build(cfg)
            logs += log
            tag = f"D{D}_{'BF16' if bf16 else 'F16'}"
            out.append(f"#define FA2_HS16_ASM_{tag} \\")
            out += [f'    "{ln}\\n\\t" \\' for ln in lines]
            out.append('    ""')
            out.append("")
        cfg = Cfg(D, False)
        o, i, c = operands(cfg)
        out.append(f"#define FA2_HS16_OUTPUTS_D{D} " + ", ".join(o))
        out.append(f"#define FA2_HS16_INPUTS_D{D} " + ", ".join(i))
        out.append(f"#define FA2_HS16_CLOBBERS_D{D} " + ", ".join(c))
        out.append(f"#define FA2_HS16_LDS_D{D} {cfg.lds_bytes}")
        out.append("")
    out = ["// " + ln for ln in logs] + out
    text = "\n".join(out) + "\n"
    path = os.path.join(here, "..", "kernels", "fa2_fwd16_hs.inc")
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
    if "--check" in sys.argv:
        cur = open(path).read() if os.path.exists(path) else ""
        if cur != text:
            print("fa2_fwd16_hs.inc is stale: run gen/gen_fwd16_hs.py")
            sys.exit(1)
        return
    with open(path, "w") as f:
        f.write(text)
    print("\n".join(logs))


if __name__ == "__main__":
    asmgen.parse_abl(sys.argv)
    emit()
