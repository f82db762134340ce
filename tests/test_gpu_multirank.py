"""The N > 1 path with the HIP kernels doing the work: world_size-2 ranks
(gloo, one process each, both on cuda:0 of the one-GPU box, as bench.py's rehearsal
runs them) each take the contiguous head range fa2amd.shard_range gives them, run the
fp16 forward and backward on their slice through the C ABI, and the reassembled slices
must match the oracle on the whole tensor.  Uneven splits (5 heads over 2 ranks) and a
ragged S are included.  No collective on the data path; the test gathers only to check."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import fa2_oracle as fo

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(B, H, S, D, grad):
    q, k, v = fo.harness_inputs(B, H, S, D)
    if grad == "ones":  # the reference harness's backward (test_flash_attention2.py:220-232)
        do = np.ones((B, H, S, D), np.float32)
    else:
        do = np.random.RandomState(11).randn(B, H, S, D).astype(np.float32)
    return q, k, v, do


def _worker(rank, world, port, B, H, S, D, grad, out_dir):
    import fa2amd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        q, k, v, do = _inputs(B, H, S, D, grad)
        first, count = fa2amd.shard_range(B * H, world, rank)
        sl = slice(first, first + count)
        part = lambda x: torch.from_numpy(np.ascontiguousarray(x.reshape(B * H, S, D)[sl][None])).to(dev)
        tq, tk, tv, tdo = part(q), part(k), part(v), part(do)
        o, lse = fa2amd.forward(tq, tk, tv, "fp16")
        dq, dk, dv = fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")
        torch.cuda.synchronize(dev)
        mine = {n: t.cpu().numpy()[0] for n, t in (("o", o), ("lse", lse), ("dq", dq), ("dk", dk), ("dv", dv))}
        got = [None] * world
        dist.all_gather_object(got, (first, count, mine))
        if rank == 0:
            full = {}
            for n in mine:
                full[n] = np.concatenate([g[2][n] for g in sorted(got, key=lambda g: g[0])])
            assert sum(g[1] for g in got) == B * H
            np.savez(os.path.join(out_dir, "parts.npz"), **full)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grad", ["ones", "randn"])
@pytest.mark.parametrize("B,H,S,D", [(2, 3, 300, 64), (1, 5, 129, 32)])
def test_two_ranks_run_their_head_shards_on_the_gpu(tmp_path, B, H, S, D, grad):
    """dO = ones: the harness's rule, max-abs over the whole tensor with dQ, dK, dV
    concatenated, un-scaled (test_flash_attention2.py:930-935, 1018-1020); dO ~ N(0,1):
    each gradient within 1e-2 of max(1, max|ref|)."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), B, H, S, D, grad, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "parts.npz")
    q, k, v, do = _inputs(B, H, S, D, grad)
    eo, el = fo.attention_forward(q, k, v)
    edq, edk, edv, _ = fo.attention_backward(q, k, v, do)
    for n, e in (("o", eo), ("lse", el)):
        g = got[n].reshape(e.shape)
        assert np.isfinite(g).all(), n
        assert float(np.abs(g - e).max()) < 1e-2, n
    grads = (("dq", edq), ("dk", edk), ("dv", edv))
    for n, e in grads:
        assert np.isfinite(got[n]).all(), n
    if grad == "ones":
        g = np.concatenate([got[n].ravel() for n, _ in grads])
        e = np.concatenate([e.ravel() for _, e in grads])
        assert float(np.abs(g - e).max()) < 1e-2
    else:
        for n, e in grads:
            g = got[n].reshape(e.shape)
            assert float(np.abs(g - e).max()) < 1e-2 * max(1.0, float(np.abs(e).max())), n
