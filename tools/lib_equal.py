#!/usr/bin/env python3
"""Check that alternate libfa2amd.so builds (tools/build_variant.sh: scheduling-only
changes) produce bitwise the same fp16-tile outputs as the default build.

  python tools/lib_equal.py <variant.so> [...] [--shape B,H,S,D]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--shape", action="append", default=None)
    args = ap.parse_args()
    import torch
    import fa2amd

    shapes = args.shape or ["4,16,2048,64", "1,2,300,64", "2,3,65,32", "1,2,1000,128"]
    default = fa2amd.LIB_PATH
    fa2amd.lib()
    bad = 0
    for sh in shapes:
        B, H, S, D = (int(x) for x in sh.split(","))
        g = torch.Generator().manual_seed(3)
        q, k, v, do = (torch.randn(B, H, S, D, generator=g).cuda() for _ in range(4))
        outs = {}
        for path in [default] + args.libs:
            fa2amd.use_library(path)
            o, lse = fa2amd.forward(q, k, v, "fp16")
            dq, dk, dv = fa2amd.backward(q, k, v, o, do, lse, "fp16")
            torch.cuda.synchronize()
            outs[path] = [t.clone() for t in (o, lse, dq, dk, dv)]
        ref = outs[default]
        for path in args.libs:
            same = [torch.equal(a, b) for a, b in zip(ref, outs[path])]
            diff = [float((a - b).abs().max()) for a, b in zip(ref, outs[path])]
            print(sh, os.path.basename(os.path.dirname(path)) or path, "o lse dq dk dv equal:", same,
                  "max abs diff:", ["%.2e" % d for d in diff])
            bad += not all(same)
    fa2amd.use_library(default)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
