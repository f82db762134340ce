#!/usr/bin/env python3
"""A/B library builds on the exact-fp32 path in ONE process (interleaved rounds,
medians), and the max difference of their outputs -- tools/kbench.py covers the fp16
kernels, this one fa2_forward / fa2_backward with FA2_FP32.

  python tools/kbench_fp32.py --lib cuda-flash-attention_amd/lib/libfa2amd.so \
      --lib cuda-flash-attention_amd/variants/old/libfa2amd.so --shape 2,8,512,64 --shape 8,16,2048,64
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", required=True, help="library builds to A/B (repeatable)")
    ap.add_argument("--shape", action="append", default=None, help="B,H,S,D (repeatable)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    import fa2amd

    dev = torch.device("cuda", 0)
    for shape in args.shape or ["2,8,512,64"]:
        B, H, S, D = (int(x) for x in shape.split(","))
        g = torch.Generator().manual_seed(1)
        q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
        do = torch.randn(B, H, S, D, generator=g).to(dev)
        times, outs = {}, {}
        for _ in range(args.rounds):
            for lib in args.lib:
                fa2amd.use_library(lib)
                o, lse = fa2amd.forward(q, k, v, "fp32")
                for kind, f in (("fwd", lambda: fa2amd.forward(q, k, v, "fp32")),
                                ("bwd", lambda: fa2amd.backward(q, k, v, o, do, lse, "fp32"))):
                    f()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        out = f()
                    e1.record()
                    e1.synchronize()
                    times.setdefault((lib, kind), []).append(e0.elapsed_time(e1) / args.iters)
                    outs[(lib, kind)] = [x.clone() for x in out]
        for kind in ("fwd", "bwd"):
            base = outs[(args.lib[0], kind)]
            for lib in args.lib:
                diff = max(float((x - y).abs().max()) for x, y in zip(outs[(lib, kind)], base))
                print(f"{shape} {kind} {lib}: median {statistics.median(times[(lib, kind)]):.4f} ms, "
                      f"max |diff| vs first {diff:.2e}", flush=True)


if __name__ == "__main__":
    main()
