"""Multi-process (gloo, world_size 2) CPU tests of the B*H shard path used by the
host API and bench.py: every rank takes the contiguous head range
fa2amd.shard_range gives it, computes it (here with the CPU oracle, standing in for
one GPU), and the slices reassemble into the unsharded result.  No collective is on
the data path; gather is used only by the test to check the assembly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import fa2amd
from oracle import fa2_oracle as fo


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, H, S, D, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q, k, v = fo.harness_inputs(B, H, S, D)
        do = np.random.RandomState(5).randn(B, H, S, D).astype(np.float32)
        first, count = fa2amd.shard_range(B * H, world, rank)
        sl = slice(first, first + count)
        flat = lambda x: x.reshape(B * H, S, D)[sl][None]
        o, lse = fo.attention_forward(flat(q), flat(k), flat(v))
        dq, dk, dv, _ = fo.attention_backward(flat(q), flat(k), flat(v), flat(do))
        # equal-size shards here (B*H divisible), so all_gather of fixed shapes works
        parts = {}
        for name, t in (("o", o), ("lse", lse), ("dq", dq), ("dk", dk), ("dv", dv)):
            buf = [torch.empty_like(torch.from_numpy(t)) for _ in range(world)]
            dist.all_gather(buf, torch.from_numpy(np.ascontiguousarray(t)))
            parts[name] = torch.cat([b[0] for b in buf]).numpy()
        # barrier + max-over-ranks exactly as bench.py times a step
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            np.savez(os.path.join(out_dir, "parts.npz"), tmax=t.numpy(), **parts)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B,H", [(2, 2), (1, 4)])
def test_two_rank_head_shards_reassemble(tmp_path, B, H):
    S, D, world = 40, 32, 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, B, H, S, D, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "parts.npz")
    q, k, v = fo.harness_inputs(B, H, S, D)
    do = np.random.RandomState(5).randn(B, H, S, D).astype(np.float32)
    eo, el = fo.attention_forward(q, k, v)
    edq, edk, edv, _ = fo.attention_backward(q, k, v, do)
    np.testing.assert_allclose(got["o"].reshape(eo.shape), eo, atol=1e-6)
    np.testing.assert_allclose(got["lse"].reshape(el.shape), el, atol=1e-6)
    for n, e in (("dq", edq), ("dk", edk), ("dv", edv)):
        np.testing.assert_allclose(got[n].reshape(e.shape), e, atol=1e-6)
    assert float(got["tmax"][0]) == 2.0


@pytest.mark.parametrize("total,world", [(64, 1), (64, 2), (64, 8), (1024, 8), (100, 3)])
def test_bench_shard_covers_all_heads(total, world):
    """bench.py --workload c5 splits B*H with fa2amd.shard_range: disjoint, complete, balanced."""
    seen, sizes = [], []
    for r in range(world):
        f, c = fa2amd.shard_range(total, world, r)
        seen.extend(range(f, f + c))
        sizes.append(c)
    assert seen == list(range(total))
    assert max(sizes) - min(sizes) <= 1


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` with no launcher starts two ranks itself (before any
    GPU call) on the north star's C5 strong-scaling split; --dry-run keeps it to the
    rank plumbing (gloo barrier + max over ranks), so it runs on CPU."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "bh-shard2"
    assert line["scaling"] == "strong"
    assert line["config"]["workload"].startswith("B64_H16_S2048_D64")
    assert line["heads_rank0"] == 512
