#!/usr/bin/env python3
"""isa_mix.py -- instruction mix per basic block of one kernel in a hipcc --save-temps .s

    python tools/isa_mix.py <file.s> <kernel-substring> [--top N] [--dump BB]

Classes: mfma, exp (transcendental), valu, salu, ds_read, ds_write, vmem, wait, barrier, other.
VALU issue cycles use MI355X_MICROARCH.md's prices (exp 8, other VALU 4, MFMA 8 of 32)."""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "exp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_write"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 8
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(kern) + r"\S*:", l))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        blocks[cur].append(s)
    if dump:
        print("\n".join(blocks[dump]))
        return
    rows = []
    for bb, ins in blocks.items():
        c = Counter(classify(i.split()[0]) for i in ins)
        valu_cyc = 4 * c["valu"] + 8 * c["exp"] + 8 * c["mfma"]
        rows.append((c["mfma"], bb, c, valu_cyc, len(ins)))
    rows.sort(key=lambda r: -r[0])
    for n, bb, c, cyc, tot in rows[:top]:
        print(f"{bb:14s} n={tot:4d} mfma={c['mfma']:3d} valu={c['valu']:4d} exp={c['exp']:3d} salu={c['salu']:3d} "
              f"dsr={c['ds_read']:3d} dsw={c['ds_write']:3d} vmem={c['vmem']:3d} wait={c['wait']:3d} bar={c['barrier']} "
              f"issue_cyc={cyc:5d} mfma_pipe_cyc={32 * c['mfma']:5d}")


if __name__ == "__main__":
    main()
