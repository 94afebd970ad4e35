"""Tanh hidden activations in the fused label kernels: torch.nn.Tanh is the
reference's default NETWORK.ACTIVATIONS (picard/config.py:61; construct_mlp, picard/solution.py:
123-135).  The Tanh k_paths family (dpi_paths_*_tanh.hip, csrc/dpi_device.h Act<DPI_ACT_TANH>)
against the reference's own labels (tests/golden/*tanh*.npz, made by tests/golden/make_golden.py)
and against the fp64 oracle in both MFMA modes (exact fp32 and the default fp16-split), plus
networks whose widths the kernels are not compiled for (zero-padded to the next compiled width).
Tolerance: rel-L2 <= 1e-4 on the value column and the gradient (and Hessian) block."""
import numpy as np
import pytest
import torch

import deeppicarditeration_amd as dpi
from deeppicarditeration_amd import _lib as L
from oracle import dpi_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(params=["f32", "auto"])
def mode(request):
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_F32 if request.param == "f32" else L.DPI_GEMM_AUTO), "prec")
    yield request.param
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "prec")


def _oracle_mlp(m, acts):
    lin = [l for l in m if isinstance(l, torch.nn.Linear)]
    return O.MLP([l.weight.detach().double().numpy() for l in lin], [l.bias.detach().double().numpy() for l in lin], acts)


def _parts(y, ref):
    y = np.asarray(y, np.float64)
    r = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))  # noqa: E731
    return {"value": r(y[:, :1], ref[:, :1]), "grad": r(y[:, 1:101], ref[:, 1:101]),
            "hess": r(y[:, 101:], ref[:, 101:]) if y.shape[1] > 101 else 0.0}


TANH_GOLDENS = ["cha_mlp16_tanh_K2", "cha_mlp128x4_tanh_K3", "ou_mlp64x2_tanh_K2", "gbm_mlp64x3_tanh_sdgd_K2",
                "gbm_mlp16_tanh_full_K1", "td_cha_mlp32_tanh_K2", "gbm_hess_mlp32x3_tanh_K2"]


@pytest.mark.parametrize("case", TANH_GOLDENS)
def test_tanh_goldens_both_modes(case, mode):
    from golden_util import load
    from gpu_util import generator, product_equation, product_module
    f = load(case)
    assert [str(a) for a in f["acts"]] == ["Tanh"] * len(f["neurons"])
    eq = product_equation(f)
    net = product_module(f, eq)
    assert isinstance(net[1], torch.nn.Tanh)
    gen = generator(f, eq, net)
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    pb = int(f["point_base"])
    if bool(f["hessians"]):
        y = gen.generate_with_gradients_and_hessians(tx, point_base=pb)
    else:
        y = gen.generate_with_gradients(tx, point_base=pb)
    p = _parts(y.cpu().numpy(), f["y"])
    print(case, mode, p)
    assert max(p.values()) < TOL, p


@pytest.mark.parametrize("kind", ["cha128x4_K50", "ou64x3", "gbm64x3_sdgd_K20"])
def test_tanh_networks_vs_oracle(kind, mode):
    torch.manual_seed(21)
    if kind.startswith("cha"):
        eq, oeq, widths, M, K, v = dpi.Cha(100, 1.0, 5.0, 1.0), O.Cha(100, 1.0, 5.0, 1.0), [128] * 4, 512, 50, 0
    elif kind.startswith("ou"):
        eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
        widths, M, K, v = [64] * 3, 256, 10, 0
    else:
        eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
        oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
        widths, M, K, v = [64] * 3, 128, 20, 100
    net = dpi.construct_mlp(101, 1, widths, ["Tanh"] * len(widths), None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=3, epoch=1,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": v}} if v else None)
    tx, y = gen.sample_with_gradients(3)
    ref = O.labels_grad(oeq, _oracle_mlp(net, ["Tanh"] * len(widths)), tx.cpu().double().numpy(), M, K, 3, 1, 0, v=v)
    p = _parts(y.cpu().numpy(), ref)
    print(kind, mode, p)
    assert max(p.values()) < TOL, p


def test_tanh_hessian_labels_vs_oracle(mode):
    """Malliavin Hessian labels with a 3 x 64 Tanh network (tanh'' in the full-Hessian f)."""
    torch.manual_seed(22)
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    net = dpi.construct_mlp(101, 1, [64] * 3, ["Tanh"] * 3, None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                  n_estimate_integral=256, n_euler_steps=5, seed=4, epoch=2)
    tx, y = gen.sample_with_gradients_and_hessians(2)
    ref = O.labels_grad_hess(oeq, _oracle_mlp(net, ["Tanh"] * 3), tx.cpu().double().numpy(), 256, 5, 4, 2, 0)
    p = _parts(y.cpu().numpy(), ref)
    print("tanh hessian labels", mode, p)
    assert max(p.values()) < TOL, p


@pytest.mark.parametrize("widths,act", [([10, 10], "Tanh"), ([100, 50, 20], "ELU"), ([40, 40], "Tanh"),
                                        ([128, 96, 128, 128], "Tanh")])
def test_uncompiled_widths_are_zero_padded(widths, act, mode):
    """Any hidden widths <= 128 (e.g. the reference's default NEURONS [10, 10] with Tanh): the host
    zero-pads the layers to the smallest compiled width; the labels equal the oracle's on the
    unpadded network."""
    torch.manual_seed(23)
    eq, oeq = dpi.Cha(100, 1.0, 5.0, 1.0), O.Cha(100, 1.0, 5.0, 1.0)
    net = dpi.construct_mlp(101, 1, widths, [act] * len(widths), None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=4, seed=5)
    tx, y = gen.sample_with_gradients(3)
    ref = O.labels_grad(oeq, _oracle_mlp(net, [act] * len(widths)), tx.cpu().double().numpy(), 128, 4, 5, 1, 0)
    p = _parts(y.cpu().numpy(), ref)
    assert max(p.values()) < TOL, p


def test_mixed_or_other_activations_raise():
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    for acts in (["Tanh", "ELU"], ["ReLU", "ReLU"]):
        net = dpi.construct_mlp(101, 1, [32, 32], acts, None)
        with pytest.raises(NotImplementedError, match="all-ELU or all-Tanh"):
            dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", n_estimate_terminal=64, n_estimate_integral=64)
