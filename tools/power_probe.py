#!/usr/bin/env python3
"""Socket power, GFX clock and energy per call of each kernel running alone in a long
loop (is a kernel at the power cap?  then its time follows its energy, not its stalls).

  python tools/power_probe.py --shape 4,16,2048,64 --kernel fwd --kernel dqd --kernel dkdv --seconds 4
  python tools/power_probe.py --kernel dqd --variant DQ_HS=0 --variant DQ_HS=1

A background thread samples `amd-smi metric -p -c` every ~0.2 s while the kernel loop
runs; the first 0.6 s of each loop (clock ramp) are discarded.  Energy per call =
median socket power x median call time (events over 50-call batches)."""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def sample(stop, out):
    while not stop.is_set():
        t = time.perf_counter()
        try:
            r = subprocess.run(["amd-smi", "metric", "-g", "0", "-p", "-c"], capture_output=True, text=True,
                               timeout=5).stdout
        except Exception:
            r = ""
        p = re.search(r"SOCKET_POWER:\s*([\d.]+)\s*W", r)
        c = re.search(r"GFX_0:\s*\n\s*CLK:\s*([\d.]+)\s*MHz", r)
        if p and c:
            out.append((t, float(p.group(1)), float(c.group(1))))
        time.sleep(0.15)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4,16,2048,64")
    ap.add_argument("--kernel", action="append", default=None, help="fwd|dqd|dkdv|step")
    ap.add_argument("--variant", action="append", default=[], help="KNOB=V[,KNOB=V] (repeatable)")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--do", choices=["ones", "randn"], default="ones")
    args = ap.parse_args()
    import torch
    import fa2amd

    B, H, S, D = (int(x) for x in args.shape.split(","))
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(42)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    do = torch.randn(B, H, S, D, generator=g).to(dev) if args.do == "randn" else torch.ones(B, H, S, D, device=dev)
    o, lse = fa2amd.forward(q, k, v, "fp16")
    dl = fa2amd.delta(do, o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    calls = {
        "fwd": lambda: fa2amd.forward(q, k, v, "fp16", out=o, lse=lse),
        "dqd": lambda: fa2amd.backward_dq_delta(q, k, v, o, do, lse, dl, dq),
        "dkdv": lambda: fa2amd.backward_dkdv(q, k, v, do, lse, dl, dk, dv),
        "step": lambda: (fa2amd.forward(q, k, v, "fp16", out=o, lse=lse),
                         fa2amd.backward(q, k, v, o, do, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl)),
    }
    res = []
    for var in args.variant or [""]:
        fa2amd.tune_set(None)
        for kv in filter(None, var.split(",")):
            kk, vv = kv.split("=")
            fa2amd.tune_set(kk, int(vv))
        for kn in args.kernel or ["fwd", "dqd", "dkdv"]:
            f = calls[kn]
            samples, stop = [], threading.Event()
            th = threading.Thread(target=sample, args=(stop, samples))
            th.start()
            t0 = time.perf_counter()
            times = []
            while time.perf_counter() - t0 < args.seconds:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    f()
                e1.record()
                e1.synchronize()
                if time.perf_counter() - t0 > 0.6:
                    times.append(e0.elapsed_time(e1) / 50)
            t1 = time.perf_counter()
            stop.set()
            th.join()
            sm = [(p, c) for (t, p, c) in samples if t0 + 0.6 < t < t1]
            pw = statistics.median([p for p, _ in sm]) if sm else None
            ck = statistics.median([c for _, c in sm]) if sm else None
            ms = statistics.median(times)
            row = {"kernel": kn, "variant": var or "default", "ms": round(ms, 4), "socket_w": pw, "gfx_mhz": ck,
                   "mj_per_call": round(pw * ms, 3) if pw else None, "samples": len(sm)}
            res.append(row)
            print(json.dumps(row), flush=True)
            time.sleep(1.0)  # cool down between loops
    print(json.dumps(res))


if __name__ == "__main__":
    main()
