#!/usr/bin/env python3
"""Segment shares of the ping-pong forward loop from a stamp build
(tools/build_variant.sh stamps -DFA2_PP_STAMPS): R1 / barrier 1 / R2 / barrier 2
per tile, prologue and whole-wave cycles, medians over the waves of one launch."""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    import torch
    import fa2amd
    lib_path = sys.argv[1]
    B, H, S, D = (int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4,16,2048,64").split(","))
    fa2amd.use_library(lib_path)
    fa2amd.tune_set("FWD_PP", 1)
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.rand(B, H, S, D, generator=g).cuda() for _ in range(3))
    for _ in range(50):
        fa2amd.forward(q, k, v, "fp16")
    torch.cuda.synchronize()
    nw = B * H * ((S + 255) // 256) * 4
    buf = (ctypes.c_ulonglong * (nw * 8))()
    L = ctypes.CDLL(lib_path)
    rc = L.fa2_debug_pp_stamps(buf, nw * 8)
    assert rc == 0, rc
    rows = [list(buf[i * 8:(i + 1) * 8]) for i in range(nw)]
    names = ["R1", "bar1", "R2", "bar2", "prologue", "total", "iters"]
    med = {n: statistics.median(r[i] for r in rows) for i, n in enumerate(names)}
    it = med["iters"]
    print(f"shape B{B}_H{H}_S{S}_D{D}, {nw} waves, iters {it}")
    loop = sum(med[n] for n in ("R1", "bar1", "R2", "bar2"))
    for n in ("R1", "bar1", "R2", "bar2"):
        print(f"  {n:6s} {med[n] / it:8.0f} cyc/tile  {100 * med[n] / loop:5.1f} % of loop")
    print(f"  loop   {loop / it:8.0f} cyc/tile; prologue {med['prologue']:.0f}; total {med['total']:.0f}; "
          f"epilogue+rest {med['total'] - med['prologue'] - loop:.0f}")


if __name__ == "__main__":
    main()
