#!/usr/bin/env python3
"""Diagnose the single-pass backward at one shape: N calls of fa2_backward_ws with
the kernels serialized (run under AMD_SERIALIZE_KERNEL=3), synchronising after each
call, then compare with the two-kernel plan."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    import torch
    import fa2amd
    B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,16,2048,64").split(","))
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dist = sys.argv[4] if len(sys.argv) > 4 else "ones"
    nored = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(42)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    if dist == "ones":
        do = torch.ones(B, H, S, D, device=dev)
    elif dist == "ones_cpu":
        do = torch.ones(B, H, S, D).to(dev)
    elif dist == "randn_dev":
        do = torch.randn(B, H, S, D, device=dev)
    else:
        do = torch.randn(B, H, S, D, generator=g).to(dev)
    o, lse = fa2amd.forward(q, k, v, "fp16")
    ref = fa2amd.backward(q, k, v, o, do, lse, "fp16")
    torch.cuda.synchronize()
    print("two-kernel ok", flush=True)
    fa2amd.tune_set("BWD_SP", kind)
    if nored:
        fa2amd.tune_set("BWD_SP_NORED", 1)
    print("workspace", fa2amd.workspace_size(B, H, S, D), flush=True)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    dl = torch.empty(B, H, S, device=dev)
    for i in range(n):
        fa2amd.backward(q, k, v, o, do, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl)
        torch.cuda.synchronize()
        print("call", i, "ok", flush=True)
    for name, a, b in zip("dq dk dv".split(), (dq, dk, dv), ref):
        print(name, float((a - b).abs().max()), float(b.abs().max()), flush=True)


if __name__ == "__main__":
    main()
