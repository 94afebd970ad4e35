"""The bench's CPU baseline (oracle/torch_cpu.py: the reference's label algorithm vectorised in
PyTorch on the host cores) against the reference's own outputs: fed the fixture's injected noise
(tests/golden/make_golden.py draw order: terminal normals, s-uniforms, integral normals), it
reproduces the golden labels to fp64 rounding."""
import math

import numpy as np
import pytest
import torch

from golden_util import load, state_dict
from gpu_util import product_equation, product_module
from oracle import philox as px
from oracle import torch_cpu as TC


@pytest.mark.parametrize("name", ["cha_mlp16_K4", "cha_mlp64x3_K50", "ou_mlp16_K2", "ou_pis32_K2", "cha_zero_K2",
                                  "gbm_mlp16_sdgd_K2"])
def test_torch_cpu_baseline_matches_reference_fixture(name):
    f = load(name)
    eq = product_equation(f)
    net = product_module(f, eq).double()
    net.load_state_dict({k: torch.as_tensor(v, dtype=torch.float64) for k, v in state_dict(f).items()})
    n, M, K = int(f["n"]), int(f["M"]), int(f["K"])
    seed, epoch, pb = int(f["seed"]), int(f["epoch"]), int(f["point_base"])
    ii = (pb + np.arange(n))[:, None]
    mm = np.arange(M)[None, :]
    S_T = sum(px.normals(px.TAG_TERM, epoch, seed, ii, mm, k, eq.nx) for k in range(K))
    S_s = sum(px.normals(px.TAG_INT, epoch, seed, ii, mm, k, eq.nx) for k in range(K))
    U = px.uniforms(px.TAG_S, epoch, seed, ii, mm, open_low=True).reshape(n * M, 1)
    noise = [torch.from_numpy(a) for a in ((S_T / math.sqrt(K)).reshape(n * M, eq.nx), U,
                                           (S_s / math.sqrt(K)).reshape(n * M, eq.nx))]
    v = int(f.get("v", 0))
    if v > 0:  # SDGD indices (make_golden.py draw 7)
        noise.append(torch.from_numpy(px.randint_idx(px.TAG_SDGD, epoch, seed, ii, mm, v, eq.nx).reshape(n * M, v)
                                      .astype(np.int64)))
    y = TC.labels_reference_algorithm(eq, net, torch.from_numpy(f["tx"]), M, None, noise=noise, v=v or None)
    ref = f["y"]
    assert np.linalg.norm(y.detach().numpy() - ref) / np.linalg.norm(ref) < 1e-11


@pytest.mark.parametrize("name", ["gbm_hess_mlp16_K2", "gbm_hess_mlp32x3_K4", "gbm_hess_zero_K2"])
def test_torch_cpu_hessian_labels_match_reference_fixture(name):
    """The Malliavin Hessian labels (the reference's _double estimators, full-Hessian get_f) fed the
    fixture's draws in make_golden.py's order (terminal half-steps, N1, s, integral half-steps, N2)."""
    f = load(name)
    eq = product_equation(f)
    net = product_module(f, eq).double()
    net.load_state_dict({k: torch.as_tensor(v, dtype=torch.float64) for k, v in state_dict(f).items()})
    n, M, K = int(f["n"]), int(f["M"]), int(f["K"])
    seed, epoch, pb = int(f["seed"]), int(f["epoch"]), int(f["point_base"])
    nx = eq.nx
    ii = (pb + np.arange(n))[:, None]
    mm = np.arange(M)[None, :]
    S_T = sum(px.normals(px.TAG_TERM, epoch, seed, ii, mm, k, nx) for k in range(K)).reshape(n * M, nx)
    S_s = sum(px.normals(px.TAG_INT, epoch, seed, ii, mm, k, nx) for k in range(K)).reshape(n * M, nx)
    half = 1.0 / math.sqrt(2 * K)
    noise = [S_T * half, S_T * half, px.normals(px.TAG_HTERM, epoch, seed, ii, mm, 0, nx).reshape(n * M, nx),
             px.uniforms(px.TAG_S, epoch, seed, ii, mm, open_low=True).reshape(n * M, 1), S_s * half, S_s * half,
             px.normals(px.TAG_HINT, epoch, seed, ii, mm, 0, nx).reshape(n * M, nx)]
    noise = [torch.from_numpy(np.ascontiguousarray(a)) for a in noise]
    y = TC.labels_hessians_reference_algorithm(eq, net, torch.from_numpy(f["tx"]), M, None, noise=noise)
    ref = f["y"]
    assert np.linalg.norm(y.detach().numpy() - ref) / np.linalg.norm(ref) < 1e-11


def test_host_cores_is_positive():
    assert TC.host_cores() >= 1 and isinstance(TC.cpu_model(), str)
