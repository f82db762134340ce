#!/usr/bin/env python3
"""Who reduced each dQ step of the single-pass backward (BWD_SP=1): reads the
workspace counters after a call.  Per (head, query step, wave) the counter ends at
NKB + 1 when the step's owner reduced it in the loop, and at NKB + 0x10000 when the
head's last workgroup swept it (kernels/f-attn2-backward_f16.cu, SpWs layout).

  python tools/sp_probe.py --shape 4,16,2048,64
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4,16,2048,64")
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--lib", default=None, help="another build of libfa2amd.so (e.g. an SP_STAMPS variant)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import fa2amd

    B, H, S, D = (int(x) for x in args.shape.split(","))
    if args.lib:
        fa2amd.use_library(args.lib)
    fa2amd.tune_set("BWD_SP", 1)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    do = torch.ones_like(q)
    o, lse = fa2amd.forward(q, k, v, "fp16")
    nb = fa2amd.backward_workspace_size(B, H, S, D, "fp16")
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    nqs, nkb, md = (S + 63) // 64, (S + 255) // 256, D // 32
    hpart = (nqs + 1) * nkb * 8 * md * 1024
    per_head = nqs * 8 + 8
    for c in range(args.calls):
        fa2amd.backward(q, k, v, o, do, lse, "fp16", workspace=ws)
        torch.cuda.synchronize()
        cnt = ws[B * H * hpart:].view(torch.int32).cpu().numpy().astype(np.int64).reshape(B * H, per_head)
        steps = cnt[:, : nqs * 8].reshape(B * H, nqs, 8)
        swept = steps >= 0x10000
        owner = steps == nkb + 1
        other = ~(swept | owner)
        print(f"call {c}: heads {B * H} steps {nqs} nkb {nkb}: owner {owner.mean():.3f} swept {swept.mean():.3f} "
              f"other {other.mean():.3f}; head-done counts {sorted(set(cnt[:, nqs * 8].tolist()))}")
        print("  swept fraction by step:", " ".join(f"{x:.2f}" for x in swept.mean(axis=(0, 2))))
        if args.stamps:  # SP_STAMPS build: per wave [store_step wait, tick, barrier, loop] cycles in its junk slot
            parts = ws[: B * H * hpart].view(B * H, nqs + 1, md, nkb, 8, 1024)
            junk = parts[:, nqs, 0].contiguous().view(torch.int64).cpu().numpy().reshape(B * H, nkb, 8, 128)[..., :4]
            tot = junk[..., 3].astype(np.float64)
            print("  stamps (share of loop): wait %.3f tick %.3f barrier %.3f; loop %.0f cycles/step"
                  % tuple([float((junk[..., i] / tot).mean()) for i in range(3)] + [float(tot.mean() / nqs)]))


if __name__ == "__main__":
    main()
