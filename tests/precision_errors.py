#!/usr/bin/env python3
"""Max-abs errors of the fp16 / bf16 / fp32 tile paths against the oracle (calibrates
the tolerances written in tests/test_gpu_parity.py).  GPU only.

    python tests/precision_errors.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-flash-attention_amd"))
import fa2amd  # noqa: E402
from oracle import fa2_oracle as fo  # noqa: E402


def err(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def main():
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


if __name__ == "__main__":
    main()
