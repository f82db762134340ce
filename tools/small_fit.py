#!/usr/bin/env python3
"""Fixed cost vs per-step cost of the small-grid kernels (DESIGN §4 "Small grids").

At a constant count of 32-row units (B·H·S/32 = 256 by default: the B2_H8_S512 grid)
the launch plan, the grid and the workgroup count stay the same while S -- and with
it the number of loop steps per workgroup -- grows.  A straight-line fit of the time
per call against S splits it into the part every call pays whatever its length
(launch boundary, prologue round trips, epilogue, merge) and the part each step adds.

  python tools/small_fit.py [--units 256] [--plan fixed|auto]

Times are events over back-to-back calls (what a caller looping over small shapes
sees, boundaries included), medians over interleaved rounds."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--units", type=int, default=256)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--plan", choices=["fixed", "auto"], default="fixed")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch
    import fa2amd

    dev = torch.device("cuda", 0)
    D = args.D
    shapes = []
    for S in (128, 256, 512, 1024, 2048):
        bh = args.units * 32 // S
        if bh >= 1:
            shapes.append((bh, S))
    if args.plan == "fixed":  # the S = 512 auto plans, forced on every shape
        knobs = {"FWD_KS": 4, "FWD_WAVES": 4, "BWD_FUSED": 1, "BWD_FUSED_DELTA": 1, "BWD_FNW": 4, "BWD_FQS": 2,
                 "BWD_FKS": 2}
        for k, v in knobs.items():
            fa2amd.tune_set(k, v)
    data = {}
    for bh, S in shapes:
        g = torch.Generator().manual_seed(1)
        q, k, v = (torch.rand(1, bh, S, D, generator=g).to(dev) for _ in range(3))
        do = torch.ones_like(q)
        o, lse = fa2amd.forward(q, k, v, "fp16")
        dl = torch.empty_like(lse)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
        data[(bh, S)] = {
            "fwd": lambda q=q, k=k, v=v, o=o, lse=lse: fa2amd.forward(q, k, v, "fp16", out=o, lse=lse),
            "bwd": lambda q=q, k=k, v=v, o=o, do=do, lse=lse, dq=dq, dk=dk, dv=dv, dl=dl: fa2amd.backward(
                q, k, v, o, do, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl),
        }
        data[(bh, S)]["step"] = (lambda f=data[(bh, S)]["fwd"], b=data[(bh, S)]["bwd"]: (f(), b()))
    # reference: back-to-back launches of a trivial kernel (the Δ kernel on one row)
    t1 = torch.ones(1, 1, 1, D, device=dev)
    tiny_out = torch.empty(1, 1, 1, device=dev)
    data[(0, 0)] = {"tiny": lambda: fa2amd.delta(t1, t1, out=tiny_out)}
    res = {}
    for _ in range(args.rounds):
        for key, calls in data.items():
            for kn, f in calls.items():
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                e1.synchronize()
                res.setdefault((kn, key), []).append(e0.elapsed_time(e1) / args.iters * 1e3)
    out = {"units": args.units, "D": D, "plan": args.plan, "rows": [], "fit": {}}
    tiny = statistics.median(res[("tiny", (0, 0))])
    out["tiny_kernel_us"] = round(tiny, 2)
    print(f"trivial kernel back to back: {tiny:.2f} us per launch")
    del data[(0, 0)]
    for kn in ("fwd", "bwd", "step"):
        xs, ys = [], []
        for (bh, S) in data:
            us = statistics.median(res[(kn, (bh, S))])
            out["rows"].append({"kernel": kn, "bh": bh, "S": S, "us": round(us, 2)})
            xs.append(S)
            ys.append(us)
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        a = my - b * mx
        out["fit"][kn] = {"fixed_us": round(a, 2), "us_per_1k_rows_of_S": round(b * 1000, 2)}
        print(f"{kn:5s} " + " ".join(f"S={S}:{statistics.median(res[(kn, (bh, S))]):6.2f}" for bh, S in data)
              + f"   fit: {a:6.2f} us + {b * 1000:6.2f} us per 1k rows", flush=True)
    fa2amd.tune_set(None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
