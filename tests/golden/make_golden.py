"""Generate the golden vectors in tests/golden/ FROM THE REFERENCE ITSELF.

Run once, in the build container (where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own Python code read-only -- nothing from it is
copied into this repository; only its numeric outputs are saved:

* ``test_flash_attention2.py`` (detker/CUDA-Flash-Attention) after stubbing the
  two modules this container lacks (``seaborn``, used only for plots, and
  ``cupy``, whose absence makes the module ``sys.exit``).
  Functions called unbound, as pure-torch CPU code:
    - ``FlashAttention2Tester.generate_test_data``   (test_flash_attention2.py:177-195)
    - ``FlashAttention2Tester.compute_reference``    (:197-208)
    - ``FlashAttention2Tester.compute_reference_backward`` (:220-232, dO = ones)
  The LSE is the harness's own formula (:917-921), evaluated here with torch.
  For a random upstream gradient (dO ~ N(0,1), seed 43) the same
  ``compute_reference`` graph is back-propagated with ``O.backward(dO)``.
* ``generate_test_data.generate_test_data`` (generate_test_data.py:6-50),
  writing Q.bin/K.bin/V.bin into a temp dir, which are read back.

Outputs: one ``<case>.npz`` per small case (inputs + O, LSE, Δ, dQ, dK, dV for
dO = ones and for dO random) and ``manifest.json`` with SHA-256 digests of the
inputs/outputs of the two BASELINE configs too large to commit (C1
B2_H8_S512_D64 and C3 B4_H16_S2048_D64, harness distribution, seed 42).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    for name in ("seaborn", "cupy", "cupy.cuda", "cupy.cuda.compiler"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["cupy"].cuda = sys.modules["cupy.cuda"]
    sys.modules["cupy.cuda"].compiler = sys.modules["cupy.cuda.compiler"]
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import test_flash_attention2 as harness  # noqa: E402
    import generate_test_data as gen  # noqa: E402
    return harness, gen


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _lse(torch, q, k):
    # test_flash_attention2.py:917-921, verbatim math
    d = q.shape[-1]
    s = torch.matmul(q, k.transpose(-2, -1)) / np.sqrt(d)
    mx = torch.max(s, dim=-1, keepdim=True)[0]
    return (mx.squeeze(-1) + torch.log(torch.sum(torch.exp(s - mx), dim=-1))).numpy()


def _outputs(harness, torch, q, k, v, do=None):
    T = harness.FlashAttention2Tester
    Q = torch.from_numpy(q.copy()).requires_grad_(True)
    K = torch.from_numpy(k.copy()).requires_grad_(True)
    V = torch.from_numpy(v.copy()).requires_grad_(True)
    O = T.compute_reference(None, Q, K, V)
    if do is None:
        grads = T.compute_reference_backward(None, O, Q, K, V)
        do = np.ones_like(q)
    else:
        O.backward(torch.from_numpy(do))
        grads = {"dQ": Q.grad.clone(), "dK": K.grad.clone(), "dV": V.grad.clone()}
    o = O.detach().numpy()
    with torch.no_grad():
        lse = _lse(torch, Q.detach(), K.detach())
    delta = (do.astype(np.float64) * o.astype(np.float64)).sum(-1).astype(np.float32)
    return o, lse.astype(np.float32), delta, grads["dQ"].numpy(), grads["dK"].numpy(), grads["dV"].numpy()


def main():
    import torch

    harness, gen = _import_reference()
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    cases = [
        # name, B, H, S, D, distribution
        ("harness_B1_H1_S128_D64", 1, 1, 128, 64, "harness"),   # Small-1
        ("harness_B2_H2_S100_D64", 2, 2, 100, 64, "harness"),   # Edge-NonPowerOf2 shape class
        ("harness_B2_H2_S32_D64", 2, 2, 32, 64, "harness"),     # Edge-SmallSeq shape class
        ("harness_B1_H2_S64_D32", 1, 2, 64, 32, "harness"),     # D=32 (reference instantiates 32/64)
        ("harness_B1_H1_S256_D128", 1, 1, 256, 128, "harness"), # D=128 (BASELINE C4 head dim)
        ("harness_B1_H1_S77_D128", 1, 1, 77, 128, "harness"),   # ragged S at D=128
        ("cli_B1_H2_S64_D64", 1, 2, 64, 64, "cli"),             # generate_test_data.py randn
        ("cli_B1_H1_S100_D32", 1, 1, 100, 32, "cli"),
    ]
    manifest = {"generator": "tests/golden/make_golden.py", "reference": REF, "cases": {}, "digests": {}}
    for name, B, H, S, D, dist in cases:
        if dist == "harness":
            cfg = harness.TestConfig(name, B, H, S, D)
            Q, K, V = harness.FlashAttention2Tester.generate_test_data(None, cfg)
            q, k, v = Q.numpy(), K.numpy(), V.numpy()
        else:
            with tempfile.TemporaryDirectory() as tmp:
                path = gen.generate_test_data(B, H, S, D, output_dir=tmp, seed=42)
                q, k, v = (np.fromfile(os.path.join(path, f"{t}.bin"), dtype=np.float32).reshape(B, H, S, D)
                           for t in "QKV")
        o1, lse, dl1, dq1, dk1, dv1 = _outputs(harness, torch, q, k, v)
        do_r = np.random.RandomState(43).randn(B, H, S, D).astype(np.float32)
        o2, _, dl2, dq2, dk2, dv2 = _outputs(harness, torch, q, k, v, do_r)
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            q=q, k=k, v=v, o=o1, lse=lse,
            delta_ones=dl1, dq_ones=dq1, dk_ones=dk1, dv_ones=dv1,
            do_rand=do_r, delta_rand=dl2, dq_rand=dq2, dk_rand=dk2, dv_rand=dv2,
        )
        manifest["cases"][name] = {"B": B, "H": H, "S": S, "D": D, "dist": dist, "seed": 42, "do_rand_seed": 43}
        print("wrote", name)
    # large BASELINE configs: digests only (harness distribution, seed 42)
    for name, B, H, S, D, outputs in (("C1_B2_H8_S512_D64", 2, 8, 512, 64, True),
                                       ("C3_B4_H16_S2048_D64", 4, 16, 2048, 64, False)):
        cfg = harness.TestConfig(name, B, H, S, D)
        Q, K, V = harness.FlashAttention2Tester.generate_test_data(None, cfg)
        ent = {"B": B, "H": H, "S": S, "D": D, "sha256_q": _sha(Q.numpy()), "sha256_k": _sha(K.numpy()),
               "sha256_v": _sha(V.numpy())}
        if outputs:
            o, lse, _, dq, dk, dv = _outputs(harness, torch, Q.numpy(), K.numpy(), V.numpy())
            ent.update({"o_sum": float(o.astype(np.float64).sum()), "lse_sum": float(lse.astype(np.float64).sum()),
                        "lse_min": float(lse.min()), "lse_max": float(lse.max()),
                        "dq_absmax": float(np.abs(dq).max()), "dk_absmax": float(np.abs(dk).max()),
                        "dv_sum": float(dv.astype(np.float64).sum())})
        manifest["digests"][name] = ent
        print("digest", name)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
