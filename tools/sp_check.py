#!/usr/bin/env python3
"""Quick single-pass backward check across library builds (GPU): for each --lib, BWD_SP=1
against the same build's two-kernel plan (BWD_SP=0) on a few shapes, and repeated calls
bitwise equal.  Bisecting tool for kernel variants (tools/build_variant.sh).

  python tools/sp_check.py --lib a/libfa2amd.so --lib b/libfa2amd.so
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--shape", action="append", default=[])
    args = ap.parse_args()
    import torch
    import fa2amd

    libs = args.lib or [fa2amd.LIB_PATH]
    shapes = [tuple(int(x) for x in s.split(",")) for s in args.shape] or [(1, 1, 1000, 64), (4, 16, 2048, 64),
                                                                         (2, 2, 300, 64), (1, 2, 1100, 64)]
    dev = torch.device("cuda", 0)
    bad = 0
    for lp in libs:
        fa2amd.use_library(lp)
        for (B, H, S, D) in shapes:
            g = torch.Generator().manual_seed(S)
            q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
            do = torch.randn(B, H, S, D, generator=g).to(dev)
            fa2amd.tune_set(None)
            o, lse = fa2amd.forward(q, k, v, "fp16")
            ref = fa2amd.backward(q, k, v, o, do, lse, "fp16")
            fa2amd.tune_set("BWD_SP", 1)
            a = fa2amd.backward(q, k, v, o, do, lse, "fp16")
            b = fa2amd.backward(q, k, v, o, do, lse, "fp16")
            torch.cuda.synchronize()
            msg = []
            for name, x, y, z in zip(("dq", "dk", "dv"), a, b, ref):
                err = float((x - z).abs().max())
                tol = 1e-2 * max(1.0, float(z.abs().max()))
                det = torch.equal(x, y)
                if err >= tol or not det or not torch.isfinite(x).all():
                    bad += 1
                    nrow = int(((x - z).abs().amax(-1) > tol).sum())
                    msg.append(f"{name}: err {err:.3g} rows {nrow} det {det}")
            print(f"{os.path.basename(os.path.dirname(lp)) or lp} B{B}_H{H}_S{S}_D{D}: {'OK' if not msg else '; '.join(msg)}")
    fa2amd.tune_set(None)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
