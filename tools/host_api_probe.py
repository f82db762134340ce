#!/usr/bin/env python3
"""Wall time of the host-pointer API (fa2_forward_host, fa2_backward_host) per call at
C3 and C5 on this box's GPUs, for several head-chunk counts (HOST_CHUNKS); with
--shards-on-device0 N also C5 split N ways with every shard on device 0."""
import argparse
import json
import os
import resource
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def timed(fa2amd, shape, ndev, runs):
    B, H, S, D = shape
    g = np.random.default_rng(1)
    q, k, v = (g.random(shape, dtype=np.float32) for _ in range(3))
    do = np.ones_like(q)
    o, lse = np.empty_like(q), np.empty((B, H, S), np.float32)
    dq, dk, dv = np.empty_like(q), np.empty_like(q), np.empty_like(q)
    tf, tb, cpu = [], [], []
    cpu_s = lambda: (lambda r: r.ru_utime + r.ru_stime)(resource.getrusage(resource.RUSAGE_SELF))
    for i in range(runs + 1):
        c0 = cpu_s()
        t0 = time.perf_counter()
        fa2amd.forward_host(q, k, v, "fp16", num_devices=ndev, out=o, lse=lse)
        t1 = time.perf_counter()
        fa2amd.backward_host(q, k, v, o, do, lse, "fp16", num_devices=ndev, dq=dq, dk=dk, dv=dv)
        t2 = time.perf_counter()
        c1 = cpu_s()
        if i:
            tf.append(t1 - t0)
            tb.append(t2 - t1)
            cpu.append(c1 - c0)
    fb = 4 * B * H * S * (4 * D + 1)
    bb = 4 * B * H * S * (8 * D + 1)
    f, b = statistics.median(tf), statistics.median(tb)
    return {"fwd_ms": round(f * 1e3, 2), "fwd_gbps": round(fb / f / 1e9, 1), "bwd_ms": round(b * 1e3, 2),
            "bwd_gbps": round(bb / b / 1e9, 1),
            # host CPU seconds (user + system, all threads, getrusage) per fwd + bwd pair
            "cpu_ms_per_pair": round(statistics.median(cpu) * 1e3, 2),
            "cpu_over_wall": round(statistics.median(cpu) / (f + b), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards-on-device0", type=int, default=0)
    ap.add_argument("--lib", default=None, help="library build to load instead of the in-tree one")
    ap.add_argument("--c5-only", action="store_true")
    ap.add_argument("--runs", type=int, default=2, help="timed fwd + bwd pairs per C5 entry (medians)")
    args = ap.parse_args()
    import fa2amd
    if args.lib:
        fa2amd.use_library(args.lib)

    out = {}
    for ch in () if args.c5_only else (1, 2, 4, 0):
        fa2amd.tune_set("HOST_CHUNKS", ch)
        out[f"c3_chunks{ch or 'auto'}"] = timed(fa2amd, (4, 16, 2048, 64), 1, 4)
    fa2amd.tune_set(None)
    out["c5_auto"] = timed(fa2amd, (64, 16, 2048, 64), 1, args.runs)
    if args.shards_on_device0:
        fa2amd.tune_set("HOST_SHARDS_ON_DEVICE0", 1)
        out[f"c5_{args.shards_on_device0}shards_dev0"] = timed(fa2amd, (64, 16, 2048, 64), args.shards_on_device0, args.runs)
    fa2amd.tune_set(None)
    fa2amd.host_release()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
