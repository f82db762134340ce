#!/usr/bin/env python3
"""Host-side cost of one fa2amd.forward / fa2amd.backward call (GPU box): the Python
checks, the stream lookup, the ctypes call and the launch, each timed over N calls
on a tiny shape whose kernels finish faster than the host issues them.

  python tools/host_overhead.py [--shape 2,8,128,64] [--n 2000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="2,8,128,64")
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import fa2amd

    B, H, S, D = (int(x) for x in args.shape.split(","))
    dev = torch.device("cuda", 0)
    q, k, v, do = (torch.rand(B, H, S, D, device=dev) for _ in range(4))
    o, lse = fa2amd.forward(q, k, v, "fp16")
    dq, dk, dv, dl = tuple(torch.empty_like(q) for _ in range(3)) + (torch.empty(B, H, S, device=dev),)
    L = fa2amd.lib()
    st = fa2amd._stream(None, dev)
    fptrs = fa2amd._ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (o, "out", 4), (lse, "lse", 3)), B, H, S, D, dev)
    bnamed = ((q, "q", 4), (k, "k", 4), (v, "v", 4), (o, "o", 4), (do, "dout", 4), (lse, "lse", 3), (dl, "delta", 3),
              (dq, "dq", 4), (dk, "dk", 4), (dv, "dv", 4))
    bptrs = fa2amd._ptrs(bnamed, B, H, S, D, dev)
    cases = {
        "fa2amd.forward": lambda: fa2amd.forward(q, k, v, "fp16", out=o, lse=lse),
        "fa2amd.backward": lambda: fa2amd.backward(q, k, v, o, do, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl),
        "checks (5 tensors)": lambda: fa2amd._ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (o, "out", 4),
                                                    (lse, "lse", 3)), B, H, S, D, dev),
        "checks (10 tensors)": lambda: fa2amd._ptrs(bnamed, B, H, S, D, dev),
        "stream lookup": lambda: fa2amd._stream(None, dev),
        "ctypes fa2_forward": lambda: L.fa2_forward(*fptrs, B, H, S, D, fa2amd.FA2_FP16, st),
        "ctypes fa2_backward": lambda: L.fa2_backward(*bptrs, B, H, S, D, fa2amd.FA2_FP16, st),
    }
    for name, f in cases.items():
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.n):
            f()
            if i % 64 == 63:
                torch.cuda.synchronize()  # keep the queue short
        torch.cuda.synchronize()
        print(f"{name:24s} {(time.perf_counter() - t0) / args.n * 1e6:8.2f} us per call", flush=True)


if __name__ == "__main__":
    main()
