import sys, os, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-flash-attention_amd"))
import fa2amd
dev = torch.device("cuda", 0)
B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,8,512,64").split(","))
g = torch.Generator().manual_seed(1)
q, k, v = (torch.rand(B, H, S, D, generator=g).to(dev) for _ in range(3))
do = torch.ones_like(q)
for i in range(200):
    o, lse = fa2amd.forward(q, k, v, "fp32")
    dq, dk, dv = fa2amd.backward(q, k, v, o, do, lse, "fp32")
torch.cuda.synchronize()
