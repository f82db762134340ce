#!/usr/bin/env python3
"""Phase stamps of the hand-scheduled forward loop (a 'stamps' timing build:
tools/abl_build.sh fw_stamps:fwd:stamps).  The build's asm records s_memtime (shader
clock) into lane k % 64 of one VGPR at every stamp k and leaves the 64 lanes (low 24 bits,
as floats) in O columns 2 / 6 of each wave's rows, the stamp count in columns 3 / 7.
Stamps: 0 entry, 1 loop entry, then per tile P1 start, P2 start, P3 start, barrier
reached (after the lgkmcnt(0) drain), barrier left; epilogue start, end.

  python tools/stamps_hs.py --lib cuda-flash-attention_amd/abl/fw_stamps/libfa2amd.so --shape 4,16,2048,64
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--shape", action="append", default=[])
    ap.add_argument("--kernel", choices=["fwd", "dq"], default="fwd")
    a = ap.parse_args()
    import torch
    import fa2amd

    fa2amd.use_library(os.path.join(ROOT, a.lib) if not os.path.isabs(a.lib) else a.lib)
    fa2amd.tune_set("FWD_HS", 1)
    fa2amd.tune_set("DQ_HS", 1)
    names = ["P1 (QK A | sm B)", "P2 (PV B | sm A)", "P3 (QK B | sm A) + drain", "barrier wait", "P4 (PV A | sm B)"]
    if a.kernel != "fwd":
        names = ["P1 (SdP A | dS B)", "P2 (dQ B | dS A)", "P3 (SdP B | dS A) + drain", "barrier wait",
                 "P4 (dQ A | dS B)"]
    for shp in a.shape or ["4,16,2048,64"]:
        B, H, S, D = (int(x) for x in shp.split(","))
        g = torch.Generator().manual_seed(1)
        q, k, v = (torch.rand(B, H, S, D, generator=g).cuda() for _ in range(3))
        if a.kernel == "fwd":
            for _ in range(5):
                o, lse = fa2amd.forward(q, k, v, "fp16")
            torch.cuda.synchronize()
            O = o.cpu().numpy().reshape(B * H, S // 256, 4, 64, D)
        else:
            o, lse = fa2amd.forward(q, k, v, "fp16")
            do = torch.randn(B, H, S, D, generator=g).cuda()
            dl, dq = torch.empty_like(lse), torch.empty_like(q)
            for _ in range(5):
                fa2amd.backward_dq_delta(q, k, v, o, do, lse, dl, dq)
            torch.cuda.synchronize()
            O = (dq.cpu().numpy() * np.sqrt(D)).reshape(B * H, S // 256, 4, 64, D)  # the epilogue's 1/sqrt(D)
        st = np.concatenate([O[..., :32, 2], O[..., :32, 6]], axis=-1).astype(np.int64)  # [bh, qb, wave, lane]
        N = int(O[0, 0, 0, 0, 3])
        nt = S // 64
        # lane L holds stamp index k = the largest k < N with k % 64 == L
        ks = np.array([max(kk for kk in range(N) if kk % 64 == L) if L < N else -1 for L in range(64)])
        order = np.argsort(ks)
        ks_sorted = ks[order]
        t = st[..., order]
        d = np.diff(t, axis=-1) % (1 << 24)  # cycles between consecutive stamps
        valid = ks_sorted[1:] >= 0
        per = {i: [] for i in range(5)}
        epi = []
        for j, kk in enumerate(ks_sorted[:-1]):
            if not valid[j] or kk < 2:
                continue
            if kk >= 2 + 5 * (nt - 1):
                epi.append(d[..., j].ravel())
                continue
            per[(kk - 2) % 5].append(d[..., j].ravel())
        print(f"shape {shp}: {B * H * (S // 256)} workgroups, {nt} tiles, {N} stamps")
        tot = 0
        for i in range(5):
            if per[i]:
                x = np.concatenate(per[i])
                tot += np.median(x)
                print(f"  {names[i]:28s} median {np.median(x):7.0f} cyc  p10 {np.percentile(x, 10):7.0f}  p90 {np.percentile(x, 90):7.0f}")
        print(f"  {'tile (sum of medians)':28s} {tot:7.0f} cyc")
        if epi:
            x = np.concatenate(epi)
            print(f"  {'epilogue':28s} median {np.median(x):7.0f} cyc")


if __name__ == "__main__":
    main()
