#!/usr/bin/env python3
"""Max-abs errors of the fp16 / bf16 / fp32 tile paths against the oracle (calibrates
the tolerances written in tests/test_gpu_*.py).  GPU only.

    python tests/precision_errors.py [--full] [--json out.json]

Small shapes (both input generators, dO ~ N(0,1)) always; --full adds the BASELINE
configurations at full size against the threaded C oracle (oracle/fa2_oracle.c): C3
(B4_H16_S2048_D64, harness inputs, dO = ones and dO ~ N(0,1) seed 43, every head) and C4
(B8_H16_S4096_D128 forward, every head), one row per tensor -- the table DESIGN.md §5
records for the shipped build's rounding points.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-flash-attention_amd"))
import fa2amd  # noqa: E402
from oracle import c_oracle, fa2_oracle as fo  # noqa: E402


def err(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def threads():
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, n or min(len(os.sched_getaffinity(0)), 32))


def small():
    shapes = [(1, 2, 100, 64), (2, 2, 256, 32), (1, 2, 200, 128), (2, 8, 512, 64), (1, 4, 2048, 64)]
    for B, H, S, D in shapes:
        for inputs in ("harness", "cli"):
            q, k, v = fo.harness_inputs(B, H, S, D) if inputs == "harness" else fo.cli_inputs(B, H, S, D, seed=7)
            do = np.random.RandomState(8).randn(B, H, S, D).astype(np.float32)
            eo, el = fo.attention_forward(q, k, v)
            edq, edk, edv, _ = fo.attention_backward(q, k, v, do)
            tq, tk, tv, tdo = (torch.from_numpy(x).cuda() for x in (q, k, v, do))
            row = [f"B{B}_H{H}_S{S}_D{D} {inputs:7s}"]
            for prec in ("fp32", "fp16", "bf16"):
                o, lse = fa2amd.forward(tq, tk, tv, prec)
                dq, dk, dv = fa2amd.backward(tq, tk, tv, o, tdo, lse, prec)
                torch.cuda.synchronize()
                g = max(err(x.cpu().numpy(), e) / max(1.0, float(np.abs(e).max()))
                        for x, e in ((dq, edq), (dk, edk), (dv, edv)))
                row.append(f"{prec}: o {err(o.cpu().numpy(), eo):.2e} lse {err(lse.cpu().numpy(), el):.2e} "
                           f"grad/scale {g:.2e}")
            print(" | ".join(row), flush=True)


def full():
    """per-tensor max-abs at C3 (both gradients) and C4 (forward), with max|ref| beside it"""
    nt = threads()
    rows = []
    B, H, S, D = 4, 16, 2048, 64
    q, k, v = fo.harness_inputs(B, H, S, D)
    eo, el = c_oracle.forward(q, k, v, nt)
    grads = {"ones": np.ones_like(q),
             "randn43": torch.randn(B, H, S, D, generator=torch.Generator().manual_seed(43)).numpy()}
    exp = {name: c_oracle.backward(q, k, v, eo, do, el, nt) for name, do in grads.items()}
    tq, tk, tv = (torch.from_numpy(x).cuda() for x in (q, k, v))
    for prec in ("fp16", "bf16"):
        o, lse = fa2amd.forward(tq, tk, tv, prec)
        torch.cuda.synchronize()
        fw = {"O": (err(o.cpu().numpy(), eo), float(np.abs(eo).max())),
              "LSE": (err(lse.cpu().numpy(), el), float(np.abs(el).max()))}
        for name, do in grads.items():
            dq, dk, dv = fa2amd.backward(tq, tk, tv, o, torch.from_numpy(do).cuda(), lse, prec)
            torch.cuda.synchronize()
            row = {"config": "C3 B4_H16_S2048_D64", "precision": prec, "dO": name}
            for t, (a, b) in fw.items():
                row[t] = a
            for t, got, e in zip(("dQ", "dK", "dV"), (dq, dk, dv), exp[name]):
                row[t] = err(got.cpu().numpy(), e)
                row[t + "_refmax"] = float(np.abs(e).max())
            rows.append(row)
            print(json.dumps(row), flush=True)
    del tq, tk, tv
    torch.cuda.empty_cache()
    B, H, S, D = 8, 16, 4096, 128
    q, k, v = fo.harness_inputs(B, H, S, D)
    eo, el = c_oracle.forward(q, k, v, nt)
    tq, tk, tv = (torch.from_numpy(x).cuda() for x in (q, k, v))
    for prec in ("fp16", "bf16"):
        o, lse = fa2amd.forward(tq, tk, tv, prec)
        torch.cuda.synchronize()
        row = {"config": "C4 B8_H16_S4096_D128 (forward)", "precision": prec, "dO": "-",
               "O": err(o.cpu().numpy(), eo), "LSE": err(lse.cpu().numpy(), el)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    return rows


def main():
    fa2amd.lib()
    if "--full" not in sys.argv:
        small()
        return
    rows = full()
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump({"build_id": fa2amd.build_id(), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
