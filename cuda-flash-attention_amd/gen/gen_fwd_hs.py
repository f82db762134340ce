#!/usr/bin/env python3
"""Generator of the hand-scheduled FA2 forward tile loop for gfx950 (MI355X).

Writes ../kernels/fa2_fwd_hs.inc: one inline-asm body per (head_dim, tile type) that the
kernel `fa2_fwd_hs_kernel<D>` (kernel_fa2_optimized_f16.cu) runs between its C++
prologue (Q block and the first K/V tile staged into LDS) and its C++ epilogue (O rows
normalised and stored from an LDS stage, LSE).  It is the forward of the reference's
`flash_attention2_forward_kernel_fp16` (kernels/kernel_fa2_optimized_f16.cu:97-330):
S = Q Kᵀ / √D, online softmax, O += P V, LSE -- on a different structure:

  * one workgroup = 4 waves = 256 query rows, ONE wave per SIMD with the whole
    512-register file; each wave holds 64 query rows as two 32-row chains A and B
    (cdna_hip_programming.md, attention forward "4-wave, one-wave-per-SIMD");
  * per 64-key tile the wave runs four phases, each one MFMA chain with the other
    chain's softmax placed in its gaps:
        P1  QKᵀ of A (tile j)   | softmax of B (tile j-1), second half
        P2  PV   of B (tile j-1)| softmax of A (tile j),   first half
        P3  QKᵀ of B (tile j)   | softmax of A (tile j),   second half   -> barrier
        P4  PV   of A (tile j)  | softmax of B (tile j),   first half
    so the matrix pipe is never waiting for the exponentials of the chain it works on;
  * every filler (exp, cvt, add, LDS fragment read, staging load / convert / LDS write)
    is assigned to an MFMA gap by the list scheduler below, with per-gap issue budgets
    and at most EXP_PER_GAP v_exp per gap; waits are counted (s_waitcnt lgkmcnt / vmcnt
    with the exact count of younger operations) and hazard wait states are inserted
    from the gfx950 rules (MFMA 8-pass result -> any other reader 12 states, VALU ->
    MFMA operand 2, transcendental -> VALU 1);
  * K and V tiles are fp32 in HBM (the reference's layout): staged one tile ahead through
    registers (buffer loads with a hardware range check) -> fp16/bf16 -> XOR-swizzled LDS
    (the swizzle of kernel_fa2_optimized_f16.cu, conflict-free for both fragment reads);
  * m (row reference, log2 units) is the first tile's row max and moves only through the
    robust C++ path: every tile's half-row sums are checked against 2^13 (the fp16 range
    guard of the library's other forward kernels); a flagged block is recomputed.

Register map (per wave, D = head dim, NB = D/32, NTQ = D/16, CPT = D/32):
  AGPR  O[c][b]      a[16(c*NB+b)]            output accumulators (C = D in AGPRs)
        Q[c][t]      a[32NB + 4(c*NTQ+t)]     Q fragments (B operand of Sᵀ = K Qᵀ)
        Vf[i]        a[32NB+8NTQ + 4i]        Vᵀ fragments of one tile (A operand of PV)
  VGPR  S[c][kb]     v[32c + 16kb]            Sᵀ accumulators; exps and packed P in place
        NM[c]        v[64 + 16c]              -m splat: the C operand of each QKᵀ chain
        Kf ring      v[96 + 4r], r < ring     K fragments (A operand of QKᵀ); 8 slots, 12 at D = 128
        staging      v[96 + 4 ring ...]       fp32 K then V rows of the next tile
        misc         m, l, tile partial sums, temporaries

Usage: python3 gen_fwd_hs.py [--check]   (--check: verify the .inc is up to date)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import asmgen  # noqa: E402
from asmgen import Ins, R, ablate, ablate_waits, fix_hazards, insert_waits, rng, rtxt, schedule_phase, stamp, tagged, thirds, valu  # noqa: E402,E501

KT = 64  # keys per tile
NWAVE = 4
ROWS = 64 * NWAVE  # query rows per workgroup
SUM_MAX_BITS = 0x46000000  # 8192.0f: half-row tile-sum guard (FA2_TILE_SUM_MAX)


# ---------------------------------------------------------------------------------------
# configuration and register map
# ---------------------------------------------------------------------------------------
class Cfg:
    def __init__(self, D, bf16):
        self.D, self.bf16 = D, bf16
        self.NB, self.NTQ, self.CPT = D // 32, D // 16, D // 32
        self.NF = 4 * self.NB  # V fragments per tile
        self.NKF = 2 * self.NTQ  # K fragments per tile
        # K fragment ring slots.  D = 128 (16 fragments per tile): 12 slots, so chain B's QKᵀ
        # re-reads only the 4 fragments chain A's overflow reads overwrote (20 b128 fragment
        # reads per tile instead of 32); the 'ring8' build keeps the r05 ring of 8
        self.ring = 12 if D == 128 and "ring8" not in asmgen.ABL else 8
        self.keep_k = self.NKF <= self.ring  # D = 64: all K fragments stay for both QKᵀ
        # overflow fragments per tile; 'big ring' order when they fit half a key block
        self.ovf = self.NKF - self.ring
        self.bigring = not self.keep_k and self.ovf <= self.NTQ // 2
        self.QB = 32 * self.NB
        self.VB = self.QB + 8 * self.NTQ
        self.nagpr = self.VB + 4 * self.NF
        self.STG = 96 + 4 * self.ring
        self.MB = self.STG + 16 * self.CPT
        self.nvgpr = self.MB + 16
        self.SV = self.nvgpr  # 'stamps' timing builds: the stamp register (and one more)
        if "stamps" in asmgen.ABL:
            self.nvgpr += 2
        self.TBB = KT * D * 2  # bytes of one fp16 tile image
        self.OST = D + 4  # O stage row stride (floats)
        self.mf = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvt = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        # D = 128 (r05 A/B, C4 / B2_H16_S4096 / B4_H16_S2048: -1.2 / -0.9 / -1.2 % in one
        # process, profiles/r05/d128/): up to 3 v_exp per gap, and the next tile's staging
        # loads spread over P2-P4 (asmgen.thirds) instead of K in P2 and V in P4; D = 64
        # measured +0.4..0.8 % with either and keeps 2 and the bunched loads
        self.exp_per_gap = 2 if D <= 64 else 3
        self.spread = D == 128
        # D = 128: per-gap issue budget from 16 cycles (was 24): C4 -0.4 %, B2_H16_S4096
        # -0.4 %, B4_H16_S2048 -0.6 % in one process (profiles/r05/d128b/, 'cap16')
        if D == 128:
            self.min_cap = 16
        # fp16 tiles: the row sums add the packed 16-bit P (v_pk_add_f16, two sums per add,
        # issued like v_add_f32) into four packed partials per chain and tile, then one fp32
        # add per lane half: 19 instructions per chain and tile instead of 40.  Five 16-bit
        # roundings on sums of at most 16 P; bf16 (8-bit mantissa) keeps fp32 adds, as does
        # the 'vsum' build
        self.pksum = not bf16 and "vsum" not in asmgen.ABL

    # AGPRs
    def O(self, c, b):
        return 16 * (c * self.NB + b)

    def Q(self, c, t):
        return self.QB + 4 * (c * self.NTQ + t)

    def Vf(self, i):
        return self.VB + 4 * i

    # VGPRs
    def S(self, c, kb, i=0):
        return 32 * c + 16 * kb + i

    def NM(self, c):
        return 64 + 16 * c

    def Kr(self, r):
        return 96 + 4 * r

    def stg(self, tensor, cc):
        return self.STG + 8 * (tensor * self.CPT + cc)

    def m(self, c):
        return self.MB + c

    def l(self, c):
        return self.MB + 2 + c

    def T(self, c, k):
        return self.MB + 4 + 4 * c + k

    def ts(self, c):
        return self.MB + 12 + c

    def tmp(self, k):
        return self.MB + 14 + k

    # LDS byte offsets
    def koff(self, slot):
        return slot * self.TBB

    def voff(self, slot):
        return (2 + slot) * self.TBB

    @property
    def lds_bytes(self):
        return max(8 * self.TBB, ROWS * self.OST * 4)

    def vfrag_addr(self, i):
        b, kb, s = i // 4, (i // 2) % 2, i % 2
        return b, (kb * 32 + 16 * s) * self.D * 2


# ---------------------------------------------------------------------------------------
# instruction builders
# ---------------------------------------------------------------------------------------
def mfma(cfg, dst, a, b, c, c_is_zero=False):
    """dst/c: ('v'|'a', base) 16-reg tuples; a/b: ('v'|'a', base) 4-reg tuples"""
    rd = R(rng(a[0], a[1], 4), "A") + R(rng(b[0], b[1], 4), "B")
    if not c_is_zero:
        rd += R(rng(c[0], c[1], 16), "C")
    ctxt = "0" if c_is_zero else rtxt(c[0], c[1], 16)
    text = f"{cfg.mf} {rtxt(dst[0], dst[1], 16)}, {rtxt(a[0], a[1], 4)}, {rtxt(b[0], b[1], 4)}, {ctxt}"
    return Ins(text, "mfma", rd, rng(dst[0], dst[1], 16))


def kfrag_read(cfg, f, slot, dst):
    kb, t = f // cfg.NTQ, f % cfg.NTQ
    off = cfg.koff(slot) + kb * 32 * cfg.D * 2
    return tagged("lds", [Ins(f"ds_read_b128 {rtxt('v', dst, 4)}, %[ka{t}] offset:{off}", "dsr", [], rng("v", dst, 4))])[0]


def vfrag_reads(cfg, i, slot, earliest=0):
    b, off = cfg.vfrag_addr(i)
    off += cfg.voff(slot)
    d = cfg.Vf(i)
    return tagged("lds", [
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d, 2)}, %[va{b}_0] offset:{off}", "dsr", [], rng("a", d, 2),
            earliest=earliest),
        Ins(f"ds_read_b64_tr_b16 {rtxt('a', d + 2, 2)}, %[va{b}_1] offset:{off}", "dsr", [], rng("a", d + 2, 2),
            earliest=earliest),
    ])


def qk_mfmas(cfg, c, kreg, order=None):
    """Sᵀ[c] = K Qᵀ[c] - m[c]: kb-major chains (kb = 0 finishes first), or the (kb, t)
    `order` given; the first MFMA of each kb takes the -m splat as its C operand"""
    order = order or [(kb, t) for kb in range(2) for t in range(cfg.NTQ)]
    out, seeded = [], set()
    for kb, t in order:
        f = kb * cfg.NTQ + t
        cc = ("v", cfg.S(c, kb)) if kb in seeded else ("v", cfg.NM(c))
        seeded.add(kb)
        out.append(mfma(cfg, ("v", cfg.S(c, kb)), ("v", kreg(f)), ("a", cfg.Q(c, t)), cc))
    return out


def bigring_b(cfg):
    """chain B's QKᵀ order and fragment registers with the big ring (ovf = x overflow
    fragments): chain A's P1 put fragments ring.. into slots 0..x-1, so B runs kb 0 from
    t = x, then kb 1's fragments still in their slots, then kb 0's first x fragments
    re-read into the slots of kb 0's first x (free after B's first x MFMAs), then the
    overflow fragments; kb 0 still finishes 4 MFMAs before the phase ends"""
    x, NTQ = cfg.ovf, cfg.NTQ
    order = [(0, t) for t in range(x, NTQ)] + [(1, t) for t in range(NTQ - x)] + \
            [(0, t) for t in range(x)] + [(1, t) for t in range(NTQ - x, NTQ)]

    def kreg(f):
        if f < x:
            return cfg.Kr(x + f)
        return cfg.Kr(f - cfg.ring) if f >= cfg.ring else cfg.Kr(f)
    # re-read i: into slot x + i after B's MFMA i used it, before B's MFMA 2(NTQ - x) + i
    windows = [(i, i + 1, 2 * (NTQ - x) + i - 3) for i in range(x)]
    return order, kreg, windows


def qk_mfmas_zero(cfg, c, kreg):
    out = []
    for kb in range(2):
        for t in range(cfg.NTQ):
            f = kb * cfg.NTQ + t
            out.append(mfma(cfg, ("v", cfg.S(c, kb)), ("v", kreg(f)), ("a", cfg.Q(c, t)), ("v", cfg.S(c, kb)),
                            c_is_zero=(t == 0)))
    return out


def pv_mfmas(cfg, c, first=False):
    """Oᵀ[c][b] += Vᵀ Pᵀ[c]: b-major, so Vf slot i is free after MFMA i"""
    out = []
    for b in range(cfg.NB):
        for kb in range(2):
            for s in range(2):
                i = b * 4 + kb * 2 + s
                z = first and kb == 0 and s == 0
                out.append(mfma(cfg, ("a", cfg.O(c, b)), ("a", cfg.Vf(i)), ("v", cfg.S(c, kb, 8 * s)),
                                ("a", cfg.O(c, b)), c_is_zero=z))
    return out


def softmax_part(cfg, c, kb, final):
    """exp2 of the 16 scores of half kb (in place), partial row sums, pack to 16-bit P (in place)"""
    out = []
    S = lambda i: cfg.S(c, kb, i)
    T = [cfg.T(c, k) for k in range(4)]
    for s in range(2):
        for i in range(8 * s, 8 * s + 8):
            out.append(valu(f"v_exp_f32 v{S(i)}, v{S(i)}", [f"v{S(i)}"], [f"v{S(i)}"], kind="exp"))
        if cfg.pksum:
            for ii in range(4):
                d, a, b = S(8 * s + ii), S(8 * s + 2 * ii), S(8 * s + 2 * ii + 1)
                out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
            # packed partials: T0, T1 from half 0's first group, T2, T3 from its second;
            # half 1 adds one packed P into each
            p = [S(8 * s + ii) for ii in range(4)]
            if kb == 0:
                for k, (x, y) in enumerate(((p[0], p[1]), (p[2], p[3]))):
                    t = T[2 * s + k]
                    out.append(valu(f"v_pk_add_f16 v{t}, v{x}, v{y}", [f"v{x}", f"v{y}"], [f"v{t}"]))
            else:
                for k in range(4):
                    t = T[k]
                    out.append(valu(f"v_pk_add_f16 v{t}, v{t}, v{p[k]}", [f"v{t}", f"v{p[k]}"], [f"v{t}"]))
            continue
        if kb == 0 and s == 0:
            for k in range(4):
                out.append(valu(f"v_add_f32 v{T[k]}, v{S(k)}, v{S(k + 4)}", [f"v{S(k)}", f"v{S(k + 4)}"], [f"v{T[k]}"]))
        elif "addrr" in asmgen.ABL:
            # the same sums in the same order per partial, round robin over the partials
            for e0 in (0, 4):
                for k in range(4):
                    e = 8 * s + k + e0
                    out.append(valu(f"v_add_f32 v{T[k]}, v{T[k]}, v{S(e)}", [f"v{T[k]}", f"v{S(e)}"], [f"v{T[k]}"]))
        else:
            for k in range(4):
                for e in (8 * s + k, 8 * s + k + 4):
                    out.append(valu(f"v_add_f32 v{T[k]}, v{T[k]}, v{S(e)}", [f"v{T[k]}", f"v{S(e)}"], [f"v{T[k]}"]))
        for ii in range(4):
            d, a, b = S(8 * s + ii), S(8 * s + 2 * ii), S(8 * s + 2 * ii + 1)
            out.append(valu(f"{cfg.cvt} v{d}, v{a}, v{b}", [f"v{a}", f"v{b}"], [f"v{d}"]))
    tagged("sm", out)
    if final:
        ts = cfg.ts(c)
        n0 = len(out)
        if cfg.pksum:
            t1 = cfg.tmp(0) if c == 0 else cfg.tmp(1)
            out.append(valu(f"v_pk_add_f16 v{T[0]}, v{T[0]}, v{T[1]}", [f"v{T[0]}", f"v{T[1]}"], [f"v{T[0]}"]))
            out.append(valu(f"v_pk_add_f16 v{T[2]}, v{T[2]}, v{T[3]}", [f"v{T[2]}", f"v{T[3]}"], [f"v{T[2]}"]))
            out.append(valu(f"v_pk_add_f16 v{T[0]}, v{T[0]}, v{T[2]}", [f"v{T[0]}", f"v{T[2]}"], [f"v{T[0]}"]))
            out.append(valu(f"v_cvt_f32_f16_e32 v{ts}, v{T[0]}", [f"v{T[0]}"], [f"v{ts}"]))
            out.append(valu(f"v_cvt_f32_f16_sdwa v{t1}, v{T[0]} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1",
                            [f"v{T[0]}"], [f"v{t1}"]))
            out.append(valu(f"v_add_f32 v{ts}, v{ts}, v{t1}", [f"v{ts}", f"v{t1}"], [f"v{ts}"]))
        else:
            out.append(valu(f"v_add_f32 v{T[0]}, v{T[0]}, v{T[1]}", [f"v{T[0]}", f"v{T[1]}"], [f"v{T[0]}"]))
            out.append(valu(f"v_add_f32 v{T[2]}, v{T[2]}, v{T[3]}", [f"v{T[2]}", f"v{T[3]}"], [f"v{T[2]}"]))
            out.append(valu(f"v_add_f32 v{ts}, v{T[0]}, v{T[2]}", [f"v{T[0]}", f"v{T[2]}"], [f"v{ts}"]))
        out.append(valu(f"v_add_f32 v{cfg.l(c)}, v{cfg.l(c)}, v{ts}", [f"v{cfg.l(c)}", f"v{ts}"], [f"v{cfg.l(c)}"]))
        # NaN or a half-row sum above 2^13 -> the block is recomputed by the robust path
        out.append(valu(f"v_cmp_nge_f32 vcc, {SUM_MAX_BITS:#x}, v{ts}", [f"v{ts}"], ["vcc"]))  # !(2^13 >= ts)
        out.append(Ins("s_or_b64 %[flg], %[flg], vcc", "salu", R(["vcc", "s:flg"]), ["s:flg"]))
        out[n0:-1] = tagged("sm", out[n0:-1])
        out[-1].tag = "flag"
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
def body(cfg, p, log):
    """one 64-key tile j with parity p: K/V of tile j in slot p; tile j+1 staged into 1-p"""
    q = 1 - p
    NKF, NTQ = cfg.NKF, cfg.NTQ
    # staging loads of tile j+2: K in P2 and V in P4 (D = 64), or spread over P2-P4 (D = 128)
    ld = thirds(staging_loads(cfg, 0) + staging_loads(cfg, 1)) if cfg.spread else \
        (staging_loads(cfg, 0), [], staging_loads(cfg, 1))
    ring = lambda f: cfg.Kr(f % cfg.ring)
    seq = []
    # P1: QKᵀ of chain A (tile j) | softmax B (j-1) second half, K fragments 8.. (D=128), stage K(j+1)
    kreads = []
    if not cfg.keep_k:
        for f in range(cfg.ring, NKF):
            r = f - cfg.ring
            ins = kfrag_read(cfg, f, p, cfg.Kr(r))
            ins.earliest, ins.deadline = r + 1, f - 3
            kreads.append(ins)
    conv = staging_convert(cfg, 0, q)
    for ins in conv:
        ins.earliest = len(qk_mfmas(cfg, 0, ring)) // 4
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, qk_mfmas(cfg, 0, ring), [softmax_part(cfg, 1, 1, True), kreads, conv], f"P1.{p}", log)
    seq += stamp(cfg.SV)
    # P2: PV of chain B (tile j-1) | softmax A (j) first half, V(j+1) staged, K(j+2) loads,
    #     K re-read 0..7 (D = 128, ring of 8), first V(j) fragments into freed Vf slots
    nsplit = cfg.NF // 4 if cfg.D > 64 else 0
    vre = []
    for i in range(nsplit):
        vre += vfrag_reads(cfg, i, p, earliest=i + 2)
    rer = [] if cfg.keep_k or cfg.bigring else [kfrag_read(cfg, f, p, cfg.Kr(f)) for f in range(cfg.ring)]
    seq += schedule_phase(cfg, pv_mfmas(cfg, 1), [softmax_part(cfg, 0, 0, False), staging_convert(cfg, 1, q),
                                                  ld[0], rer, vre], f"P2.{p}", log)
    # P3: QKᵀ of chain B (tile j) | softmax A (j) second half, K re-reads (D = 128), rest of V(j)
    kreads = []
    order_b, kreg_b = None, ring
    if cfg.bigring:
        order_b, kreg_b, windows = bigring_b(cfg)
        for f, lo, hi in windows:
            ins = kfrag_read(cfg, f, p, kreg_b(f))
            ins.earliest, ins.deadline = lo, hi
            kreads.append(ins)
    elif not cfg.keep_k:
        for f in range(cfg.ring, NKF):
            r = f - cfg.ring
            ins = kfrag_read(cfg, f, p, cfg.Kr(r))
            ins.earliest, ins.deadline = r + 1, f - 3
            kreads.append(ins)
    vre = []
    for i in range(nsplit, cfg.NF):
        vre += vfrag_reads(cfg, i, p)
    seq += stamp(cfg.SV)
    seq += schedule_phase(cfg, qk_mfmas(cfg, 1, kreg_b, order_b), [softmax_part(cfg, 0, 1, True), kreads, vre,
                                                                   list(ld[1])], f"P3.{p}", log)
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    seq += stamp(cfg.SV)
    seq.append(Ins("s_barrier", "bar"))
    seq += stamp(cfg.SV)
    # P4: PV of chain A (tile j) | softmax B (j) first half, K(j+1) fragment prefetch, V(j+2) loads
    pre = [kfrag_read(cfg, f, q, cfg.Kr(f)) for f in range(min(cfg.ring, NKF))]
    seq += schedule_phase(cfg, pv_mfmas(cfg, 0), [softmax_part(cfg, 1, 0, False), pre,
                                                  list(ld[2]) + [goff_inc(cfg)]], f"P4.{p}", log)
    return seq


def prologue(cfg):
    D, NTQ, NKF = cfg.D, cfg.NTQ, cfg.NKF
    seq = [Ins("s_mov_b32 s98, 0", "salu", [], ["s98"])] if "stamps" in asmgen.ABL else []
    seq += stamp(cfg.SV)
    seq += [Ins("s_mov_b64 %[flg], 0", "salu", [], ["s:flg"]),
           valu(f"v_mov_b32 v{cfg.l(0)}, 0", [], [f"v{cfg.l(0)}"]),
           valu(f"v_mov_b32 v{cfg.l(1)}, 0", [], [f"v{cfg.l(1)}"])]
    # tile 1 loads (K then V)
    seq += staging_loads(cfg, 0) + staging_loads(cfg, 1) + [goff_inc(cfg)]
    # Q fragments of both chains -> AGPRs (Q block in LDS at %[qb] + this wave's rows)
    for t in range(NTQ):
        seq.append(valu(f"v_add_u32 v{t}, %[qb], %[ka{t}]", [], [f"v{t}"]))
    for c in range(2):
        for t in range(NTQ):
            d = cfg.Q(c, t)
            seq.append(Ins(f"ds_read_b128 {rtxt('a', d, 4)}, v{t} offset:{c * 32 * D * 2}", "dsr", R([f"v{t}"]),
                           rng("a", d, 4)))
    # K(0) fragments: ring slots, then (D = 128) the NM registers as spare slots
    kreg0 = lambda f: cfg.Kr(f) if f < cfg.ring else 64 + 4 * (f - cfg.ring)
    for f in range(NKF):
        seq.append(kfrag_read(cfg, f, 0, kreg0(f)))
    # Sᵀ of tile 0 for both chains (no -m seed yet)
    seq += qk_mfmas_zero(cfg, 0, kreg0) + qk_mfmas_zero(cfg, 1, kreg0)
    # row max per chain -> m; the two lane halves hold the two key halves: xor-32 max
    for c in range(2):
        m = cfg.m(c)
        regs = [cfg.S(c, kb, i) for kb in range(2) for i in range(16)]
        seq.append(valu(f"v_max3_f32 v{m}, v{regs[0]}, v{regs[1]}, v{regs[2]}", [f"v{r}" for r in regs[:3]], [f"v{m}"]))
        k = 3
        while k + 1 < len(regs):
            seq.append(valu(f"v_max3_f32 v{m}, v{m}, v{regs[k]}, v{regs[k + 1]}", [f"v{m}", f"v{regs[k]}", f"v{regs[k + 1]}"],
                            [f"v{m}"]))
            k += 2
        if k < len(regs):
            seq.append(valu(f"v_max_f32 v{m}, v{m}, v{regs[k]}", [f"v{m}", f"v{regs[k]}"], [f"v{m}"]))
        t0, t1 = cfg.tmp(0), cfg.tmp(1)
        seq.append(valu(f"v_mov_b32 v{t0}, v{m}", [f"v{m}"], [f"v{t0}"]))
        seq.append(valu(f"v_mov_b32 v{t1}, v{m}", [f"v{m}"], [f"v{t1}"]))
        seq.append(valu(f"v_permlane32_swap_b32 v{t0}, v{t1}", [f"v{t0}", f"v{t1}"], [f"v{t0}", f"v{t1}"]))
        seq.append(valu(f"v_max_f32 v{m}, v{t0}, v{t1}", [f"v{t0}", f"v{t1}"], [f"v{m}"]))
    # -m splats (the QKᵀ seeds) and s - m of tile 0
    for c in range(2):
        m, nm = cfg.m(c), cfg.NM(c)
        seq.append(valu(f"v_sub_f32 v{nm}, 0, v{m}", [f"v{m}"], [f"v{nm}"]))
        for i in range(1, 16):
            seq.append(valu(f"v_mov_b32 v{nm + i}, v{nm}", [f"v{nm}"], [f"v{nm + i}"]))
        for kb in range(2):
            for i in range(16):
                r = cfg.S(c, kb, i)
                seq.append(valu(f"v_sub_f32 v{r}, v{r}, v{m}", [f"v{r}", f"v{m}"], [f"v{r}"]))
    seq += softmax_part(cfg, 0, 0, False) + softmax_part(cfg, 0, 1, True) + softmax_part(cfg, 1, 0, False)
    # V(0) fragments, O[B] = 0, PV of chain A (tile 0)
    for i in range(cfg.NF):
        seq += vfrag_reads(cfg, i, 0)
    for b in range(cfg.NB):
        for i in range(16):
            r = cfg.O(1, b) + i
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
    D = cfg.D
    seq = [Ins("s_waitcnt vmcnt(0) lgkmcnt(0)", "wait")]
    seq += stamp(cfg.SV)
    seq += softmax_part(cfg, 1, 1, True)
    seq += pv_mfmas(cfg, 1)
    # every wave is done with the tile slots before the O stage overwrites them
    seq.append(Ins("s_barrier", "bar"))
    for c in range(2):
        for b in range(cfg.NB):
            for g in range(4):
                r = cfg.O(c, b) + 4 * g
                off = (c * 32 * cfg.OST + 32 * b + 8 * g) * 4
                seq.append(Ins(f"ds_write_b128 %[oa], {rtxt('a', r, 4)} offset:{off}", "dsw", R(rng("a", r, 4)), []))
    for c in range(2):
        seq.append(valu(f"v_mov_b32 %[om{c}], v{cfg.m(c)}", [f"v{cfg.m(c)}"], []))
        seq.append(valu(f"v_mov_b32 %[ol{c}], v{cfg.l(c)}", [f"v{cfg.l(c)}"], []))
    if "stamps" in asmgen.ABL:
        # the stamps into O columns 2 / 6 of the wave's rows r (lanes r / 32 + r) and the stamp
        # count into columns 3 / 7; l = 1/2 per lane half, so the epilogue stores the stage as is
        seq += stamp(cfg.SV)
        sv, sc = cfg.SV, cfg.SV + 1
        seq += [Ins("s_nop 4", "nop"),
                valu(f"v_and_b32 v{sv}, 0xffffff, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_cvt_f32_u32 v{sv}, v{sv}", [f"v{sv}"], [f"v{sv}"]),
                valu(f"v_mov_b32 v{sc}, s98", [], [f"v{sc}"]),
                valu(f"v_cvt_f32_u32 v{sc}, v{sc}", [f"v{sc}"], [f"v{sc}"]),
                Ins("s_nop 4", "nop"),
                Ins(f"ds_write_b32 %[oa], v{sv} offset:8", "dsw", R([f"v{sv}"]), []),
                Ins(f"ds_write_b32 %[oa], v{sc} offset:12", "dsw", R([f"v{sc}"]), []),
                valu("v_mov_b32 %[ol0], 0.5", [], []), valu("v_mov_b32 %[ol1], 0.5", [], [])]
    seq.append(Ins("s_waitcnt lgkmcnt(0)", "wait"))
    return seq


# ---------------------------------------------------------------------------------------
# whole program
# ---------------------------------------------------------------------------------------
def build(cfg):
    log = [f"D={cfg.D} {'bf16' if cfg.bf16 else 'fp16'}: {cfg.nvgpr} VGPRs + {cfg.nagpr} AGPRs in asm, "
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
    outs = ['[om0] "=&v"(hs_m0)', '[om1] "=&v"(hs_m1)', '[ol0] "=&v"(hs_l0)', '[ol1] "=&v"(hs_l1)',
            '[flg] "=&s"(hs_flag)', '[cnt] "+s"(hs_cnt)', '[goff] "+s"(hs_goff)']
    ins = [f'[ka{t}] "v"(hs_ka[{t}])' for t in range(cfg.NTQ)]
    ins += [f'[va{b}_{k}] "v"(hs_va[{b}][{k}])' for b in range(cfg.NB) for k in range(2)]
    ins += [f'[vo{c}] "v"(hs_vo[{c}])' for c in range(cfg.CPT)]
    ins += ['[lo] "v"(hs_lo)', '[oa] "v"(hs_oa)', '[rsk] "s"(hs_rsk)', '[rsv] "s"(hs_rsv)', '[qb] "s"(hs_qb)']
    clob = [f'"v{i}"' for i in range(cfg.nvgpr)] + [f'"a{i}"' for i in range(cfg.nagpr)] + ['"vcc"', '"scc"', '"memory"']
    if "stamps" in asmgen.ABL:
        clob += asmgen.STAMP_CLOBBERS
    return outs, ins, clob


def emit():
    here = os.path.dirname(os.path.abspath(__file__))
    out = ["// Generated by cuda-flash-attention_amd/gen/gen_fwd_hs.py -- do not edit.",
           "// Hand-scheduled forward tile loop of fa2_fwd_hs_kernel<D> (kernel_fa2_optimized_f16.cu).",
           "#pragma once", ""]
    logs = []
    for D in (64, 128):
        for bf16 in (False, True):
            cfg = Cfg(D, bf16)
            lines, log = build(cfg)
            logs += log
            tag = f"D{D}_{'BF16' if bf16 else 'F16'}"
            out.append(f"#define FA2_HS_ASM_{tag} \\")
            out += [f'    "{ln}\\n\\t" \\' for ln in lines]
            out.append('    ""')
            out.append("")
        cfg = Cfg(D, False)
        o, i, c = operands(cfg)
        out.append(f"#define FA2_HS_OUTPUTS_D{D} " + ", ".join(o))
        out.append(f"#define FA2_HS_INPUTS_D{D} " + ", ".join(i))
        out.append(f"#define FA2_HS_CLOBBERS_D{D} " + ", ".join(c))
        out.append(f"#define FA2_HS_LDS_D{D} {cfg.lds_bytes}")
        out.append("")
    out = ["// " + ln for ln in logs] + out
    text = "\n".join(out) + "\n"
    path = os.path.join(here, "..", "kernels", "fa2_fwd_hs.inc")
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
    if "--check" in sys.argv:
        cur = open(path).read() if os.path.exists(path) else ""
        if cur != text:
            print("fa2_fwd_hs.inc is stale: run gen/gen_fwd_hs.py")
            sys.exit(1)
        return
    with open(path, "w") as f:
        f.write(text)
    print("\n".join(logs))


if __name__ == "__main__":
    asmgen.parse_abl(sys.argv)
    emit()
