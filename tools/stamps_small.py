#!/usr/bin/env python3
"""Where a small-grid forward's time goes, per workgroup.

Loads a -DFA2_STAMPS build (tools/build_variant.sh stamps -DFA2_STAMPS): thread 0 of each
forward workgroup records s_memrealtime (100 MHz) at phase boundaries and writes the
stamps over its block's first O row.  Phases: 0 entry, 1 Q + first K/V step in LDS,
2 Q fragments in registers, 3 first step done, 4 loop done, 5 key-split merge done,
6 O / LSE stores issued, 7 those stores complete.  Printed per shape: the spread of
workgroup entry times (dispatch ramp), the median of each phase, the span from the
first entry to the last store completion, and the event-timed kernel for comparison.

  python tools/stamps_small.py --lib cuda-flash-attention_amd/variants/stamps/libfa2amd.so"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))

PHASES = ["prologue (Q + K/V step 0)", "Q fragments", "first step", "rest of loop", "merge", "O/LSE store issue",
          "store drain"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--shape", action="append", default=None)
    args = ap.parse_args()
    import torch
    import fa2amd
    fa2amd.use_library(args.lib)
    dev = torch.device("cuda", 0)
    out = {}
    for sh in args.shape or ["2,8,128,64", "2,8,512,64", "2,8,1024,64", "2,8,2048,64", "4,16,2048,64"]:
        B, H, S, D = (int(x) for x in sh.split(","))
        g = torch.Generator().manual_seed(1)
        q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
        o, lse = fa2amd.forward(q, k, v, "fp16")
        for _ in range(20):
            fa2amd.forward(q, k, v, "fp16", out=o, lse=lse)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fa2amd.forward(q, k, v, "fp16", out=o, lse=lse)
        e1.record()
        e1.synchronize()
        ev_us = e0.elapsed_time(e1) / 20 * 1e3
        o.fill_(0.5)
        fa2amd.forward(q, k, v, "fp16", out=o, lse=lse)
        torch.cuda.synchronize()
        st = o.reshape(-1, D)[:, :16].contiguous().view(torch.int64).cpu()  # rows x 8 stamps
        ok = (st[:, 0] > 0) & (st[:, 0] < 10**17)
        for i in range(1, 8):
            ok &= st[:, i] >= st[:, i - 1]
        st = st[ok].double() * 0.01  # ticks of 10 ns -> us
        n = st.shape[0]
        t0 = st[:, 0].min().item()
        entry = (st[:, 0] - t0)
        ph = {PHASES[i]: round(statistics.median((st[:, i + 1] - st[:, i]).tolist()), 3) for i in range(7)}
        rec = {"workgroups": n, "event_us": round(ev_us, 2), "span_us": round(st[:, 7].max().item() - t0, 2),
               "entry_spread_us": round(entry.max().item(), 2), "entry_median_us": round(entry.median().item(), 2),
               "wg_median_us": round(statistics.median((st[:, 7] - st[:, 0]).tolist()), 2),
               "last_done_minus_last_entry_us": round(st[:, 7].max().item() - st[:, 0].max().item(), 2),
               "phase_median_us": ph}
        out[sh] = rec
        print(sh, json.dumps(rec), flush=True)
    # the fused small-grid backward: per workgroup entry and completion, by role
    import ctypes
    import time
    import numpy as np
    lib = fa2amd.lib()
    lib.fa2_bwd_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((65536, 4), np.uint64)
    for sh in args.shape or ["2,8,128,64", "2,8,512,64", "2,8,1024,64", "2,8,2048,64"]:
        B, H, S, D = (int(x) for x in sh.split(","))
        g = torch.Generator().manual_seed(1)
        q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
        do = torch.ones_like(q)
        o, lse = fa2amd.forward(q, k, v, "fp16")
        dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
        dl = torch.empty_like(lse)
        call = lambda: fa2amd.backward(q, k, v, o, do, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl)
        for _ in range(20):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        e1.synchronize()
        ev_us = e0.elapsed_time(e1) / 20 * 1e3
        time.sleep(0.02)
        call()
        torch.cuda.synchronize()
        assert lib.fa2_bwd_stamps_read(buf.ctypes.data, buf.nbytes) == 0
        t = buf.astype(np.float64)
        last = t[:, 0].max()
        sel = (t[:, 0] > last - 1e5) & (t[:, 1] >= t[:, 0])  # the last call: within 1 ms (ticks of 10 ns)
        t = t[sel]
        t0 = t[:, 0].min()
        rec = {"workgroups": int(sel.sum()), "event_us": round(ev_us, 2),
               "span_us": round((t[:, 1].max() - t0) * 0.01, 2),
               "entry_spread_us": round((t[:, 0].max() - t0) * 0.01, 2)}
        for role, name in ((0, "dkdv"), (1, "dq")):
            r = t[t[:, 2] == role]
            if len(r):
                rec[name] = {"n": len(r), "dur_median_us": round(float(np.median(r[:, 1] - r[:, 0])) * 0.01, 2),
                             "dur_max_us": round(float((r[:, 1] - r[:, 0]).max()) * 0.01, 2),
                             "entry_median_us": round(float(np.median(r[:, 0] - t0)) * 0.01, 2),
                             "done_max_us": round(float((r[:, 1] - t0).max()) * 0.01, 2)}
        out["bwd_" + sh] = rec
        print("bwd", sh, json.dumps(rec), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
