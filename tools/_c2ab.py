import sys, os, statistics, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-flash-attention_amd"))
import fa2amd
dev = torch.device("cuda", 0)
libs = ["cuda-flash-attention_amd/lib/libfa2amd.so", "cuda-flash-attention_amd/variants/head/libfa2amd.so"]
for shape in ["2,8,512,64", "8,16,2048,64", "2,8,512,32", "2,8,512,128", "2,4,1000,64"]:
    B, H, S, D = (int(x) for x in shape.split(","))
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
    do = torch.randn(B, H, S, D, generator=g).to(dev)
    res = {}
    outs = {}
    for r in range(5):
        for L in libs:
            fa2amd.use_library(L)
            for kind in ("fwd", "bwd"):
                o, lse = fa2amd.forward(q, k, v, "fp32")
                f = (lambda: fa2amd.forward(q, k, v, "fp32")) if kind == "fwd" else (lambda: fa2amd.backward(q, k, v, o, do, lse, "fp32"))
                f(); torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10): out = f()
                e1.record(); e1.synchronize()
                res.setdefault((L, kind), []).append(e0.elapsed_time(e1) / 10)
                outs[(L, kind)] = [x.clone() for x in out]
    for kind in ("fwd", "bwd"):
        a, b = outs[(libs[0], kind)], outs[(libs[1], kind)]
        diff = max(float((x - y).abs().max()) for x, y in zip(a, b))
        print(shape, kind, "new %.4f ms" % statistics.median(res[(libs[0], kind)]), "head %.4f ms" % statistics.median(res[(libs[1], kind)]), "maxdiff %.2e" % diff, flush=True)
