"""CPU checks of the generated (hand-scheduled) tile loops, no GPU needed.

gen/asmsim.py executes the inline asm the generators wrote (kernels/fa2_*_hs.inc) lane
by lane: MFMA lane layouts, ds_read_b64_tr_b16, buffer range checks, and the counted
waits (reading a register whose load no wait has retired fails the run).  Its results
are compared with a float64 numpy restatement of the same block inside the simulator
(the north star's tolerances: 1e-2 fp16, 2e-2 bf16).  Cases: both head dims and tile
types of the forward, the restart flag on a late score spike, and the dQ / dK/dV loops
on several loop exits (S / 64 mod the unroll) and a second block.
"""
import os
import subprocess
import sys

import pytest

GEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-flash-attention_amd", "gen")


def sim(*args):
    r = subprocess.run([sys.executable, os.path.join(GEN, "asmsim.py"), *args], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("D,S,bf16", [(64, 256, False), (64, 320, True), (128, 192, False), (128, 256, True)])
def test_forward_loop(D, S, bf16):
    out = sim("--kernel", "fwd", "--D", str(D), "--S", str(S), *(["--bf16"] if bf16 else []))
    assert "restart flag False" in out


@pytest.mark.parametrize("D", [64, 128])
def test_forward_loop_flags_a_late_spike(D):
    """a late key far above the first tile's row max must raise the restart flag"""
    assert "restart flag True" in sim("--kernel", "fwd", "--D", str(D), "--S", "256", "--spike")


@pytest.mark.parametrize("S,block,bf16", [(128, 0, False), (192, 0, False), (256, 0, True), (320, 0, False),
                                          (512, 1, False)])
def test_dq_loop(S, block, bf16):
    sim("--kernel", "dq", "--D", "64", "--S", str(S), "--block", str(block), *(["--bf16"] if bf16 else []))


@pytest.mark.parametrize("S,block,bf16", [(128, 0, False), (192, 0, False), (256, 0, False), (320, 0, True), (384, 0, False),
                                          (512, 1, False)])
def test_dkdv_loop(S, block, bf16):
    sim("--kernel", "dkdv", "--D", "64", "--S", str(S), "--block", str(block), *(["--bf16"] if bf16 else []))


@pytest.mark.parametrize("gen", ["gen_fwd_hs.py", "gen_bwd_dq.py", "gen_bwd_dkdv.py"])
def test_generated_loops_are_current(gen):
    """each committed kernels/*.inc is what its generator writes from its current source"""
    r = subprocess.run([sys.executable, os.path.join(GEN, gen), "--check"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
