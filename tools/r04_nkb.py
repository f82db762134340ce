#!/usr/bin/env python3
"""FWD_NKB=2 (key-split forward on 64-key tiles) vs the shipped 32-key tiles: max |diff|
against an fp64 torch reference and bitwise repeatability, over ragged / spiking shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))
import torch  # noqa: E402
import fa2amd  # noqa: E402

dev = torch.device("cuda", 0)
for (B, H, S, D, spike) in [(2, 8, 2048, 64, False), (2, 8, 2000, 64, False), (2, 8, 1900, 64, True),
                            (4, 8, 1024, 64, False), (1, 16, 1500, 64, True), (2, 8, 2048, 32, False)]:
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    if spike:
        k[:, :, -3, :] = 3.0
        k[:, :, 70, :] = 2.0
    res = {}
    for nkb in (0, 2):
        fa2amd.tune_set(None)
        fa2amd.tune_set("FWD_KS", 2)
        fa2amd.tune_set("FWD_WAVES", 8)
        if nkb:
            fa2amd.tune_set("FWD_NKB", nkb)
        o, l = fa2amd.forward(q, k, v, "fp16")
        o2, l2 = fa2amd.forward(q, k, v, "fp16")
        res[nkb] = (o, l, bool(torch.equal(o, o2) and torch.equal(l, l2)))
    fa2amd.tune_set(None)
    torch.cuda.synchronize()
    hs = slice(0, 2)
    s = (q[:, hs].double() @ k[:, hs].double().transpose(-1, -2)) / D ** 0.5
    ref = torch.softmax(s, -1) @ v[:, hs].double()
    lref = torch.logsumexp(s, -1)
    line = f"B{B}_H{H}_S{S}_D{D} spike={spike}:"
    for nkb, (o, l, rep) in res.items():
        line += (f"  nkb{nkb}: o {(o[:, hs].double() - ref).abs().max().item():.2e} lse "
                 f"{(l[:, hs].double() - lref).abs().max().item():.2e} rep {rep}")
    print(line, flush=True)
