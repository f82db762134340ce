#!/usr/bin/env python3
"""A/B kernel variants in ONE process (guide §5.4 rule 24): interleaved rounds,
median and min per variant.  Variants are launch-plan overrides (fa2_tune_set,
include/fa2_amd.h) or alternate library builds.

  python tools/kbench.py --shape 4,16,2048,64 --kernel fwd --variant FWD_WAVES=4 --variant FWD_WAVES=8
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4,16,2048,64")
    ap.add_argument("--kernel", action="append", default=None, help="fwd|dkdv|dq|delta|bwd|step (repeatable)")
    ap.add_argument("--variant", action="append", default=[], help="KNOB=V[,KNOB=V] (repeatable)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", action="append", default=[], help="alternate libfa2amd.so builds to A/B (repeatable)")
    ap.add_argument("--do", choices=["randn", "ones"], default="randn", help="dO distribution (bench.py uses ones)")
    ap.add_argument("--inputs", choices=["rand", "spike"], default="rand",
                    help="Q/K/V U[0,1) as the harness draws them, or with one late spiking key")
    ap.add_argument("--precision", choices=["fp16", "bf16", "fp32"], default="fp16",
                    help="tile precision of the fwd / bwd / stepb calls")
    args = ap.parse_args()
    import torch
    import fa2amd

    B, H, S, D = (int(x) for x in args.shape.split(","))
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(42)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    if args.inputs == "spike":
        # a late key whose scores sit ~2^18 above the first tile's row max: every query
        # block's branch-free forward loop notes it and redoes the block with the
        # rescaling loop (the worst case of the restart, kernel_fa2_optimized_f16.cu)
        k[:, :, -1, :] = 4.0
    do = torch.randn(B, H, S, D, generator=g).to(dev) if args.do == "randn" else torch.ones(B, H, S, D, device=dev)
    P = args.precision
    o, lse = fa2amd.forward(q, k, v, P)
    dl = fa2amd.delta(do, o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    flops = {"fwd": 4.0, "dkdv": 8.0, "dq": 2.0, "dqd": 2.0, "delta": 0.0, "bwd": 10.0, "step": 14.0, "stepb": 14.0,
             "step3": 14.0, "step2s": 14.0, "step2r": 14.0}
    s2 = torch.cuda.Stream(device=dev)

    def two_stream_step(dkdv_first):
        """fwd, delta, then dK/dV and dQ concurrently on two streams (joined)."""
        cur = torch.cuda.current_stream(dev)
        fa2amd.forward(q, k, v, "fp16", out=o, lse=lse, stream=cur)
        fa2amd.delta(do, o, out=dl, stream=cur)
        ev = torch.cuda.Event()
        ev.record(cur)
        s2.wait_event(ev)
        if dkdv_first:
            fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv, stream=s2)
            fa2amd.backward_dq(q, k, v, do, lse, dl, dq, stream=cur)
        else:
            fa2amd.backward_dq(q, k, v, do, lse, dl, dq, stream=s2)
            fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv, stream=cur)
        ev2 = torch.cuda.Event()
        ev2.record(s2)
        cur.wait_event(ev2)
    calls = {
        "fwd": lambda: fa2amd.forward(q, k, v, P, out=o, lse=lse),
        "dkdv": lambda: fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv),
        "dq": lambda: fa2amd.backward_dq(q, k, v, do, lse, dl, dq),
        "delta": lambda: fa2amd.delta(do, o, out=dl),
        "bwd": lambda: fa2amd.backward(q, k, v, o, do, lse, P, dq=dq, dk=dk, dv=dv, delta_buf=dl),
        # one bench.py step: fwd, delta, dK/dV, dQ in stream order
        "step": lambda: (fa2amd.forward(q, k, v, "fp16", out=o, lse=lse),
                         fa2amd.backward_dq_delta(q, k, v, o, do, lse, dl, dq),
                         fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv)),
        "dqd": lambda: fa2amd.backward_dq_delta(q, k, v, o, do, lse, dl, dq),
        # fwd + fa2_backward (whatever launch plan launch_backward picks, e.g. BWD_FUSED)
        "stepb": lambda: (fa2amd.forward(q, k, v, P, out=o, lse=lse),
                          fa2amd.backward(q, k, v, o, do, lse, P, dq=dq, dk=dk, dv=dv, delta_buf=dl)),
        # dK/dV and dQ on two streams after a separate delta kernel
        "step2s": lambda: two_stream_step(True),
        "step2r": lambda: two_stream_step(False),
        # the pre-fusion order: separate delta kernel, dK/dV, dQ
        "step3": lambda: (fa2amd.forward(q, k, v, "fp16", out=o, lse=lse), fa2amd.delta(do, o, out=dl),
                          fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv),
                          fa2amd.backward_dq(q, k, v, do, lse, dl, dq)),
    }
    # the bench step captured once into a HIP graph and replayed
    graph = None
    if "stepg" in (args.kernel or []):
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            calls["step"]()  # warm (lazy init outside the capture)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                calls["step"]()
        torch.cuda.current_stream(dev).wait_stream(side)
        calls["stepg"] = graph.replay
        flops["stepg"] = 14.0
    kernels = args.kernel or ["fwd", "dkdv", "dq"]
    variants = args.variant or [""]
    libs = args.lib or [None]
    if args.lib:
        variants = [f"lib={l}" + ("," + v if v else "") for l in libs for v in (args.variant or [""])]

    def setenv(var):
        if var.startswith("lib="):
            path, _, var = var[4:].partition(",")
            fa2amd.use_library(path)
        fa2amd.tune_set(None)
        for kv in filter(None, var.split(",")):
            if kv.startswith("lib="):
                continue
            kk, vv = kv.split("=")
            fa2amd.tune_set(kk, int(vv))

    res = {(kn, var): [] for kn in kernels for var in variants}
    for r in range(args.rounds):
        for var in variants:
            setenv(var)
            for kn in kernels:
                f = calls[kn]
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                e1.synchronize()
                res[(kn, var)].append(e0.elapsed_time(e1) / args.iters)
    out = []
    for (kn, var), ts in res.items():
        med, mn = statistics.median(ts), min(ts)
        tf = flops[kn] * B * H * S * S * D / (med * 1e-3) / 1e12
        out.append({"kernel": kn, "variant": var or "default", "median_ms": round(med, 4), "min_ms": round(mn, 4),
                    "tflops_alg": round(tf, 1)})
        print(f"{kn:6s} {var or 'default':28s} median {med:8.4f} ms  min {mn:8.4f}  {tf:7.1f} TF(alg)")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
