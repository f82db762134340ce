#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel.

Per kernel: mean counter value per dispatch; derived figures:
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
      (FETCH_SIZE, WRITE_SIZE in KiB; on gfx950 FETCH_SIZE reports exactly half of
       a wide coalesced streaming read -- MI355X_MICROARCH.md §HBM -- hence x2)
  lds_conflict_frac    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  mfma_busy_frac       = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * CUs)   [approx]
Writes <dir>/pmc_summary.json and, with --commit, profiles/pmc_summary.json
(read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(fa2_\w+?_kernel|flash_attention2_\w+|D_computation\w+|fa2_delta_kernel)", name)
    if not m:
        return None
    base = m.group(1)
    t = re.search(r"<([0-9a-z, ]+)>", name)
    return base + ("<" + t.group(1).replace(" ", "") + ">" if t else "")


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters": m}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            e["hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        if m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("SQ_INSTS_MFMA"):
            e["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"]
            e["lds_per_mfma"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"]
        if m.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            e["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    e[c.lower() + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
        out[k] = e
    meta = os.environ.get("PMC_META")
    if meta:
        out["_meta"] = json.loads(meta)
    text = json.dumps(out, indent=1, sort_keys=True)
    with open(os.path.join(d, "pmc_summary.json"), "w") as f:
        f.write(text)
    for k, e in out.items():
        if k.startswith("_"):
            continue
        print(k)
        for n, v in sorted(e.items()):
            if n != "counters":
                print(f"   {n:28s} {v:.4g}")
        for n, v in sorted(e["counters"].items()):
            print(f"   . {n:26s} {v:.6g}")


if __name__ == "__main__":
    main()
