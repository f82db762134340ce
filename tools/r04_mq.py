#!/usr/bin/env python3
"""FWD_MQ=2 (two 32-row query groups per wave, 512 rows per workgroup, 32-key tiles)
against the default forward: max |diff| vs the default plan and vs an fp32 torch
reference on a few shapes (incl. ragged S and a late score spike)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-flash-attention_amd"))
import torch  # noqa: E402
import fa2amd  # noqa: E402

dev = torch.device("cuda", 0)
for (B, H, S, D, spike) in [(1, 2, 1000, 64, False), (4, 16, 2048, 64, False), (1, 2, 777, 32, False),
                            (1, 4, 1500, 64, True), (2, 8, 4096, 64, False)]:
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    if spike:
        k[:, :, -1, :] = 4.0
    fa2amd.tune_set(None)
    o0, l0 = fa2amd.forward(q, k, v, "fp16")
    fa2amd.tune_set("FWD_MQ", 2)
    o1, l1 = fa2amd.forward(q, k, v, "fp16")
    o2, l2 = fa2amd.forward(q, k, v, "fp16")
    fa2amd.tune_set(None)
    torch.cuda.synchronize()
    hq = slice(0, 1)
    s = (q[:, hq].double() @ k[:, hq].double().transpose(-1, -2)) / D ** 0.5
    ref = torch.softmax(s, -1) @ v[:, hq].double()
    lref = torch.logsumexp(s, -1)
    print(f"B{B}_H{H}_S{S}_D{D} spike={spike}: |o1-o0| {(o1-o0).abs().max().item():.3e} |l1-l0| "
          f"{(l1-l0).abs().max().item():.3e}  repeat-equal {bool(torch.equal(o1, o2) and torch.equal(l1, l2))}  "
          f"vs fp64 head0: mq2 {(o1[:, hq].double()-ref).abs().max().item():.3e} default "
          f"{(o0[:, hq].double()-ref).abs().max().item():.3e} lse {(l1[:, hq].double()-lref).abs().max().item():.3e}",
          flush=True)
