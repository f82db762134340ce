"""Shared machinery of the inline-asm generators (gen_fwd_hs.py, gen_bwd_*.py), gfx950.

  Ins              one instruction: text, class, registers read (with MFMA operand role) and
                   written, issue cost, placement window (earliest / deadline MFMA gap)
  schedule_phase   list scheduler: the filler streams of a phase into its MFMA gaps, with a
                   per-gap issue budget and at most `exp_per_gap` v_exp per gap
  insert_waits     exact counted s_waitcnt lgkmcnt / vmcnt before every consumer of an
                   outstanding ds_read / buffer_load (in-order retirement)
  fix_hazards      s_nop wait states from the gfx950 rules: MFMA result -> any other reader
                   or writer (8-pass 32x32x16: 12 states, 4-pass 16x16x32: 8), VALU -> MFMA
                   operand 2, transcendental -> VALU 1, VALU -> permlane 2, permlane -> VALU 2
"""


class Ins:
    """One instruction: text, class, registers read (with MFMA operand role) and written."""

    __slots__ = ("text", "kind", "rd", "wr", "cost", "earliest", "deadline", "trans", "perm", "tag")

    def __init__(self, text, kind, rd=(), wr=(), cost=None, earliest=0, deadline=None):
        self.text = text
        self.kind = kind  # mfma valu exp dsr dsw vmem salu wait nop bar label branch
        self.rd = list(rd)  # list of (reg, role)
        self.wr = list(wr)
        self.earliest = earliest
        self.deadline = deadline
        self.trans = kind == "exp"
        self.perm = text.startswith("v_permlane")
        self.tag = ""
        if cost is None:
            cost = {"mfma": 8, "exp": 8, "valu": 4, "dsr": 4, "dsw": 8, "vmem": 4, "salu": 2, "wait": 0,
                    "nop": 4, "bar": 4, "label": 0, "branch": 4}[kind]
        self.cost = cost

    def ws(self):
        """wait states this instruction provides to a later hazard consumer"""
        if self.kind == "label":
            return 0
        if self.kind == "nop":
            return int(self.text.split()[1]) + 1
        return 1


def tagged(tag, seq):
    for i in seq:
        i.tag = tag
    return seq


def rng(p, base, n):
    return [f"{p}{base + i}" for i in range(n)]


def rtxt(p, base, n):
    return f"{p}{base}" if n == 1 else f"{p}[{base}:{base + n - 1}]"


def R(regs, role="x"):
    return [(r, role) for r in regs]


def valu(text, rd, wr, kind="valu"):
    return Ins(text, kind, R(rd), wr)


def thirds(seq):
    """seq in three consecutive chunks of near-equal length (staging loads spread over three
    phases: bunched into one 8-MFMA phase they ask for ~64 B/clk per CU, the texture unit's
    whole rate, and the issuing waves wait; the 'nospread' build keeps the old placement)"""
    n = len(seq)
    a, b = -(-n // 3), -(-2 * n // 3)
    return seq[:a], seq[a:b], seq[b:]


def schedule_phase(cfg, mfmas, streams, name, log):
    """cfg: any object with exp_per_gap"""
    nM = len(mfmas)
    streams = [s for s in streams if s]
    pos = [0] * len(streams)
    tot = [max(1, sum(i.cost for i in s)) for s in streams]
    done = [0] * len(streams)
    total = sum(sum(i.cost for i in s) for s in streams)
    # exact-result schedule A/Bs: 'epgN' at most N v_exp per gap, 'capN' minimum gap budget N
    epg, mcap = cfg.exp_per_gap, getattr(cfg, "min_cap", 24)
    for a in ABL:
        if a.startswith("epg"):
            epg = int(a[3:])
        elif a.startswith("cap"):
            mcap = int(a[3:])
    cap = max(mcap, -(-total // max(1, nM)))
    out = []
    for g in range(nM + 1):
        used = 0
        nexp = 0
        while True:
            cands = [k for k, s in enumerate(streams) if pos[k] < len(s) and s[pos[k]].earliest <= g]
            if not cands:
                break
            forced = [k for k in cands if streams[k][pos[k]].deadline is not None and streams[k][pos[k]].deadline <= g]
            if forced:
                k = min(forced, key=lambda k: streams[k][pos[k]].deadline)
            else:
                if g < nM and used >= cap:
                    break
                ok = [k for k in cands if g == nM or not (streams[k][pos[k]].kind == "exp" and nexp >= epg)]
                if not ok:
                    break
                k = min(ok, key=lambda k: (done[k] / tot[k], k))
            ins = streams[k][pos[k]]
            pos[k] += 1
            done[k] += ins.cost
            used += ins.cost
            nexp += ins.kind == "exp"
            out.append(ins)
        if g < nM:
            out.append(mfmas[g])
    for k, s in enumerate(streams):
        assert pos[k] == len(s), f"{name}: stream {k} not drained"
    nexp = sum(1 for s in streams for i in s if i.kind == "exp")
    nfill = sum(len(s) for s in streams)
    log.append(f"  {name:4s}: {nM:2d} MFMA, {nfill:3d} fillers ({nexp} exp), filler issue {total:4d} cyc, "
               f"cap/gap {cap}, est. {max(32 * nM, total + 8 * nM)} cyc")
    return out


def regs_of(ins):
    return {r for r, _ in ins.rd} | set(ins.wr)


def insert_waits(seq, state):
    """state: (lgkm list, vm list) of outstanding ops as frozensets of written regs"""
    out, ends = insert_waits_multi(seq, [state])
    return out, ends[0]


def insert_waits_multi(seq, states):
    """counted waits valid for every entry state in `states` (each (lgkm, vm) as above): before
    each consumer the smallest count any state needs; returns (seq, exit states)"""
    sts = [[list(st[0]), list(st[1])] for st in states]
    out = []

    def retire(q, n):
        return q[len(q) - n:] if n < len(q) else q

    for ins in seq:
        if ins.kind == "wait":
            t = ins.text
            for st in sts:
                if "lgkmcnt(" in t:
                    st[0] = retire(st[0], int(t.split("lgkmcnt(")[1].split(")")[0]))
                if "vmcnt(" in t:
                    st[1] = retire(st[1], int(t.split("vmcnt(")[1].split(")")[0]))
            out.append(ins)
            continue
        touched = regs_of(ins)
        nl = nv = None
        for st in sts:
            for idx, e in enumerate(st[0]):
                if e & touched:
                    n = len(st[0]) - idx - 1
                    nl = n if nl is None else min(nl, n)
            for idx, e in enumerate(st[1]):
                if e & touched:
                    n = len(st[1]) - idx - 1
                    nv = n if nv is None else min(nv, n)
        parts = []
        if nv is not None:
            nv = min(nv, 63)
            parts.append(f"vmcnt({nv})")
        if nl is not None:
            nl = min(nl, 15)
            parts.append(f"lgkmcnt({nl})")
        for st in sts:
            if nv is not None:
                st[1] = retire(st[1], nv) if nv else []
            if nl is not None:
                st[0] = retire(st[0], nl) if nl else []
        if parts:
            out.append(Ins("s_waitcnt " + " ".join(parts), "wait"))
        out.append(ins)
        for st in sts:
            if ins.kind in ("dsr", "dsw"):
                st[0].append(frozenset(ins.wr))
            elif ins.kind == "vmem":
                st[1].append(frozenset(ins.wr))
    return out, [(tuple(st[0]), tuple(st[1])) for st in sts]


def mfma_result_ws(ins):
    """wait states after an MFMA before another instruction may read or write its result
    (gfx950: passes + 4; the chained accumulate into the same registers needs none)"""
    return 8 if "16x16x32" in ins.text else 12


def hazard_need(prev, cur):
    """wait states cur needs after prev (0 if none)"""
    need = 0
    pw = set(prev.wr)
    if not pw:
        return 0
    if prev.kind == "mfma":
        for r, role in cur.rd:
            if r in pw:
                if cur.kind == "mfma" and role == "C" and set(cur.wr) == pw:
                    continue  # accumulate chain: back-to-back
                need = max(need, mfma_result_ws(prev))
        if set(cur.wr) & pw and not (cur.kind == "mfma" and set(cur.wr) == pw):
            need = max(need, mfma_result_ws(prev))
        return need
    if prev.kind in ("valu", "exp"):
        rd = {r for r, _ in cur.rd}
        hit = rd & pw
        if not hit:
            return 0
        if cur.kind == "mfma" or cur.perm:
            need = max(need, 2)
        if prev.trans and cur.kind in ("valu", "exp") and not cur.trans:
            need = max(need, 1)
        if prev.perm:
            need = max(need, 2)
        if "vcc" in hit and cur.kind == "salu":
            need = max(need, 1)
        return need
    if prev.kind == "salu":
        if {r for r, _ in cur.rd} & pw and cur.kind == "vmem":
            return 1
    return 0


def fix_hazards(block, preds):
    """insert s_nop into block so every consumer has its wait states after every producer,
    with each predecessor tail in preds as possible history"""
    out = []
    for ins in block:
        need = 0
        for hist in preds:
            h = hist + out
            dist = 0
            for prev in reversed(h):
                if dist > 24:
                    break
                n = hazard_need(prev, ins)
                if n > dist:
                    need = max(need, n - dist)
                dist += prev.ws()
        while need > 0:
            k = min(need, 16)
            out.append(Ins(f"s_nop {k - 1}", "nop"))
            need -= k
        out.append(ins)
    return out


ABL = set()  # timing-only ablations (--abl a,b --out file): results are invalid, never the product .inc
EXACT_ABL = {"addrr", "nospread", "vsum", "pkmul32", "convp1"}  # variants that keep the product's results (and its flag)


def ablate(seq):
    """drop the loop-body instructions the active ablations name"""
    if not {a for a in ABL - EXACT_ABL if not a.startswith(("epg", "cap"))}:
        return seq
    out = []
    for i in seq:
        if i.tag == "flag":
            continue
        if ("nobar" in ABL and i.kind == "bar") or ("nostage" in ABL and i.tag == "stg") or \
                ("nolds" in ABL and i.tag == "lds") or ("nosm" in ABL and i.tag == "sm") or \
                ("noexp" in ABL and i.kind == "exp") or ("nomfma" in ABL and i.kind == "mfma") or \
                ("nowait" in ABL and i.kind == "wait"):
            continue
        out.append(i)
    return out


def stamp(sv):
    """'stamps' timing builds: s_memtime into lane s98 of v{sv} (s98 counts the stamps; the
    drain keeps the counted waits exact around the scalar-memory return); not a product path"""
    if "stamps" not in ABL:
        return []
    return [Ins("s_memtime s[96:97]", "salu", [], ["s96", "s97"]), Ins("s_waitcnt lgkmcnt(0)", "wait"),
            Ins("s_mov_b32 m0, s98", "salu", R(["s98"]), ["m0"]), Ins("s_nop 4", "nop"),
            Ins(f"v_writelane_b32 v{sv}, s96, m0", "valu", R(["s96", "m0"]), [f"v{sv}"]),
            Ins("s_add_u32 s98, s98, 1", "salu", R(["s98"]), ["s98", "scc"])]


STAMP_CLOBBERS = ['"s96"', '"s97"', '"s98"', '"m0"']


def parse_abl(argv):
    if "--abl" in argv:
        ABL.update(argv[argv.index("--abl") + 1].split(","))
        assert "--out" in argv, "ablation builds write elsewhere (--out): never the product .inc"


def ablate_waits(seq):
    """the 'nowait' ablation: no counted waits inside the loop bodies (a timing probe only)"""
    return [i for i in seq if not ("nowait" in ABL and i.kind == "wait")] if ABL else seq
