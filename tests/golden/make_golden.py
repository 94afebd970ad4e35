"""Generate the golden label vectors under tests/golden/ from the REFERENCE implementation.

Runs only in the build container (needs /root/reference, read-only).  It imports the
reference's hot-path modules (picard.config/utils/equations/data/solution) with tiny
stand-ins for the third-party modules absent from this image (yacs, lightning, h5py,
tensorboardX, wandb) and with picard/__init__.py bypassed, then injects the
oracle's Philox noise in the reference's exact draw order:

  1 rand(n,1) t  | 2 [OU] randn(n,nx) x0 | 3 randn_like(x) | 4 randn_like (R,nx) terminal
  5 rand_like (R,1) s | 6 randn_like (R,nx) integral | 7 [SDGD] randint(0,nx,(R,v))

Terminal/integral normals are the aggregated K-step noise xi_eff = sum_k xi_k / sqrt(K), so
the reference's one-jump path equals the K-step Euler–Maruyama endpoint.  Outputs (inputs,
weights, expected labels — data only) are written as .npz fixtures.

Usage:  python tests/golden/make_golden.py
"""
import importlib
import math
import os
import shutil
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE))
from oracle import philox as px  # noqa: E402


from ref_stubs import install_stubs  # noqa: E402

CfgNode = install_stubs(REF / "picard")
eqs = importlib.import_module("picard.equations")
data = importlib.import_module("picard.data")
sols = importlib.import_module("picard.solution")


class NoiseQueue:
    """Replace torch's RNG entry points with pops from a queue (shape-checked)."""

    def __init__(self, items):
        self.items = list(items)
        self.orig = {}

    def _pop(self, kind, shape):
        k, arr = self.items.pop(0)
        assert k == kind, f"draw order mismatch: expected {k}, reference asked for {kind}"
        assert tuple(arr.shape) == tuple(shape), f"{kind}: shape {arr.shape} vs {shape}"
        return torch.as_tensor(arr)

    def __enter__(self):
        self.orig = {n: getattr(torch, n) for n in ("rand", "randn", "randn_like", "rand_like", "randint")}
        q = self

        def rand(*size, **kw):
            size = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list)) else size
            return q._pop("rand", size).to(torch.get_default_dtype())

        def randn(*size, **kw):
            size = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list)) else size
            return q._pop("randn", size).to(torch.get_default_dtype())

        def randn_like(x, **kw):
            return q._pop("randn", x.shape).to(x.dtype)

        def rand_like(x, **kw):
            return q._pop("rand", x.shape).to(x.dtype)

        def randint(low, high, size, **kw):
            return q._pop("randint", size).to(torch.int64)

        torch.rand, torch.randn, torch.randn_like, torch.rand_like, torch.randint = (
            rand, randn, randn_like, rand_like, randint)
        return self

    def __exit__(self, *a):
        for n, f in self.orig.items():
            setattr(torch, n, f)
        assert not self.items, f"{len(self.items)} injected draws unused"


def noise_items(eq_name, nx, n, M, K, seed, epoch, point_base, v, t_factors=0, MT=None):
    """M = n_estimate_integral, MT = n_estimate_terminal (default M): the terminal draw (#4) has
    n MT rows, the integral ones n M."""
    MT = M if MT is None else MT
    i = point_base + np.arange(n)
    if t_factors:  # sample_t (data.py:149-159): torch.rand(n, N - i + 1)
        items = [("rand", px.uniforms_seq(px.TAG_T, epoch, seed, i, 0, t_factors))]
    else:
        items = [("rand", px.uniforms(px.TAG_T, epoch, seed, i, 0)[:, None])]
    if eq_name == "OUProcessEquation":
        items.append(("randn", px.normals(px.TAG_X0, epoch, seed, i, 0, 0, nx)))
    items.append(("randn", px.normals(px.TAG_X, epoch, seed, i, 0, 0, nx)))
    ii = i[:, None]
    mm = np.arange(M)[None, :]
    S_T = sum(px.normals(px.TAG_TERM, epoch, seed, ii, np.arange(MT)[None, :], k, nx) for k in range(K))
    S_s = sum(px.normals(px.TAG_INT, epoch, seed, ii, mm, k, nx) for k in range(K))
    items.append(("randn", (S_T / math.sqrt(K)).reshape(n * MT, nx)))
    items.append(("rand", px.uniforms(px.TAG_S, epoch, seed, ii, mm, open_low=True).reshape(n * M, 1)))
    items.append(("randn", (S_s / math.sqrt(K)).reshape(n * M, nx)))
    if v > 0:
        items.append(("randint", px.randint_idx(px.TAG_SDGD, epoch, seed, ii, mm, v, nx).reshape(n * M, v)))
    return items


def noise_items_hess(nx, n, M, K, seed, epoch, point_base, MT=None):
    """Draw order of sample_with_gradients_and_hessians (picard/data.py:225-237) for a GBM
    equation: t | x | terminal dW1, dW2 (two half-steps), N1 | s, integral dW1, dW2, N2.  Each
    pair of half-step normals is injected as S / sqrt(2K) twice, so the two half-steps sum to the
    K-step endpoint x + a sqrt((tau - t)/K) S.  Terminal draws n MT rows (n_estimate_terminal,
    :1164), integral ones n M (:845)."""
    MT = M if MT is None else MT
    i = point_base + np.arange(n)
    items = [("rand", px.uniforms(px.TAG_T, epoch, seed, i, 0)[:, None]),
             ("randn", px.normals(px.TAG_X, epoch, seed, i, 0, 0, nx))]
    ii = i[:, None]
    mm = np.arange(M)[None, :]
    mt = np.arange(MT)[None, :]
    S_T = sum(px.normals(px.TAG_TERM, epoch, seed, ii, mt, k, nx) for k in range(K)).reshape(n * MT, nx)
    S_s = sum(px.normals(px.TAG_INT, epoch, seed, ii, mm, k, nx) for k in range(K)).reshape(n * M, nx)
    half = 1.0 / math.sqrt(2 * K)
    items += [("randn", S_T * half), ("randn", S_T * half),
              ("randn", px.normals(px.TAG_HTERM, epoch, seed, ii, mt, 0, nx).reshape(n * MT, nx)),
              ("rand", px.uniforms(px.TAG_S, epoch, seed, ii, mm, open_low=True).reshape(n * M, 1)),
              ("randn", S_s * half), ("randn", S_s * half),
              ("randn", px.normals(px.TAG_HINT, epoch, seed, ii, mm, 0, nx).reshape(n * M, nx))]
    return items


def make_equation(name, kw, workdir):
    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        return getattr(eqs, name)(**kw)
    finally:
        os.chdir(cwd)


def prepare_workdir():
    wd = Path(tempfile.mkdtemp(prefix="dpi_golden_"))
    for f in (REF / "scripts/fully_nonlinear/case_1").glob("*.pt"):
        shutil.copy(f, wd / f.name)
    for f in (REF / "scripts/hjb").glob("*.pt"):
        shutil.copy(f, wd / f.name)
    # finding 8: var file is not shipped; it is deterministic var_scale * I
    torch.save(torch.stack([2.0 * torch.eye(100, dtype=torch.float64) for _ in range(5)]),
               wd / "var_100d_ms=1.0_vs=2.0_5.pt")
    return wd


def state_dict_np(module):
    return {k: v.detach().cpu().numpy() for k, v in module.state_dict().items()}


def run_case(name, eq_name, eq_kw, net_kind, net_kw, n, M, K, seed, epoch=0, point_base=0, v=0,
             init_seed=0, workdir=None, zero=False, weight_scale=1.0, hessians=False, delta_t=0.0, picard_N=1,
             picard_i=1, t_uniform=True, homog=None, MT=None):
    torch.set_default_dtype(torch.float64)
    eq = make_equation(eq_name, eq_kw, workdir)
    torch.manual_seed(init_seed)
    if zero:
        net = sols.ZeroSolution(1)
    elif net_kind == "mlp":
        net = sols.construct_mlp(1 + eq.nx, 1, net_kw["neurons"],
                                 [net_kw.get("act", "ELU")] * len(net_kw["neurons"]), None)
    else:
        net = sols.PISGradNet(hidden_shapes=net_kw["neurons"], dim=eq.nx, g0=eq.g, T=eq.T)
    if weight_scale != 1.0:
        with torch.no_grad():
            for p in net.parameters():
                p.mul_(weight_scale)
    if homog is not None:  # the network's first layer x s, its other hidden biases x s, its output weights x 1/s:
        # about the same function with every hidden activation ~s times smaller (tools/probe_small.py)
        seq = net.nn_module if net_kind == "pis" else net
        lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
        with torch.no_grad():
            lin[0].weight.mul_(homog)
            for m in lin[:-1]:
                m.bias.mul_(homog)
            lin[-1].weight.mul_(1.0 / homog)
    if net_kind == "pis" and not zero:
        with torch.no_grad():  # a non-trivial learnable phase
            net.timestep_phase.copy_(0.1 * torch.randn(1, 64))
    hess = CfgNode({"method": "SDGD" if v > 0 else None, "kwargs": CfgNode({"v": v} if v > 0 else {})})
    gen = data.OnlineDataGenerator(
        eq, net, picard_N, picard_i, device="cpu", t_always_uniform=t_uniform,
        n_estimate_terminal=M if MT is None else MT,
        n_estimate_integral=M, hessian_approximation=hess, sample_bound=None,
        estimate_terminal="OU_ByGx", estimate_integral="OU_Simple", estimate_delta_t=delta_t)
    if hessians:
        items = noise_items_hess(eq.nx, n, M, K, seed, epoch, point_base, MT)
        with NoiseQueue(items):
            tx, y = gen.sample_with_gradients_and_hessians(n)
    else:
        t_factors = 0 if t_uniform else picard_N - picard_i + 1
        items = noise_items(eq_name, eq.nx, n, M, K, seed, epoch, point_base, v, t_factors, MT)
        with NoiseQueue(items):
            tx, y = gen.sample_with_gradients(n)
    out = {
        "case": name, "eq": eq_name, "net": "zero" if zero else net_kind, "n": n, "M": M, "K": K,
        "MT": M if MT is None else MT,
        "seed": np.uint64(seed), "epoch": epoch, "point_base": point_base, "v": v, "hessians": hessians,
        "delta_t": delta_t, "t_factors": 0 if (t_uniform or hessians) else picard_N - picard_i + 1,
        "tx": tx.numpy(), "y": y.detach().numpy(),
    }
    for k, val in eq_kw.items():
        out[f"eqkw_{k}"] = val
    if not zero:
        for k, val in state_dict_np(net).items():
            out[f"sd_{k}"] = val
        out["neurons"] = np.asarray(net_kw["neurons"])
        if net_kind == "mlp":
            out["acts"] = np.asarray([net_kw.get("act", "ELU")] * len(net_kw["neurons"]))
    if eq_name == "OUProcessEquation":
        out["gmm_mean"] = eq.mean.numpy()
        out["gmm_var"] = torch.diagonal(eq.var, dim1=1, dim2=2).numpy()
        out["gmm_pi"] = eq.pi.numpy()
    if eq_name == "GBMEquationComplexExact":
        out["gbm_w"] = eq.w.numpy()
        out["gbm_v"] = eq.v.numpy()
    np.savez_compressed(HERE / f"{name}.npz", **out)
    print(f"{name}: tx {tx.shape} y {y.shape} |y|={float(y.norm()):.4g}")


def main(only=None):
    wd = prepare_workdir()
    global run_case
    if only:  # regenerate a subset: python make_golden.py <prefix>
        _rc = run_case

        def run_case(name, *a, **k):  # noqa: F811
            if name.startswith(only):
                _rc(name, *a, **k)
    cha = {"nx": 100, "alpha": 1.0, "k": 5.0, "T": 1.0}
    ou = {"nx": 100, "alpha": 1.0, "T": 1.0, "num_components": 5, "mean_scale": 1.0,
          "var_scale": 2.0, "alpha_scale": 4.0}
    gbm = {"nx": 100, "alpha": 1.0, "T": 1.0}
    # Burgers: small MLP, several K; full-width 4x128 (config 1 network) at K=20; zero net
    run_case("cha_mlp16_K1", "Cha", cha, "mlp", {"neurons": [16, 16]}, 4, 64, 1, 20250725, workdir=wd)
    run_case("cha_mlp16_K4", "Cha", cha, "mlp", {"neurons": [16, 16]}, 4, 64, 4, 7, epoch=3, point_base=100, workdir=wd)
    run_case("cha_mlp128x4_K20", "Cha", cha, "mlp", {"neurons": [128] * 4}, 3, 64, 20, 20250725, workdir=wd)
    run_case("cha_zero_K2", "Cha", cha, "mlp", {"neurons": [8]}, 3, 64, 2, 11, workdir=wd, zero=True)
    run_case("cha_mlp64x3_K50", "Cha", cha, "mlp", {"neurons": [64] * 3}, 2, 128, 50, 1, epoch=7, workdir=wd)
    # HJB: OU + GMM, PISGradNet (reduced width), zero net (iteration 1)
    run_case("ou_pis32_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 3, 64, 2, 2, workdir=wd)
    run_case("ou_mlp16_K2", "OUProcessEquation", ou, "mlp", {"neurons": [16, 16]}, 3, 64, 2, 5, workdir=wd)
    run_case("ou_mlp128x4_K3", "OUProcessEquation", ou, "mlp", {"neurons": [128] * 4}, 2, 64, 3, 9, workdir=wd)
    run_case("ou_zero_K1", "OUProcessEquation", ou, "mlp", {"neurons": [8]}, 3, 64, 1, 2, workdir=wd, zero=True)
    # range / precision stress of the fp16-split default: every network parameter scaled by 8 and 32
    run_case("cha_mlp128x4_ws8_K3", "Cha", cha, "mlp", {"neurons": [128] * 4}, 2, 64, 3, 41, workdir=wd,
             weight_scale=8.0)
    run_case("cha_mlp128x4_ws32_K3", "Cha", cha, "mlp", {"neurons": [128] * 4}, 2, 64, 3, 42, workdir=wd,
             weight_scale=32.0)
    run_case("ou_pis32_ws8_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 2, 64, 2, 43, workdir=wd,
             weight_scale=8.0)
    run_case("ou_pis32_ws32_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 2, 64, 2, 44, workdir=wd,
             weight_scale=32.0)
    # small magnitudes in the split storage: every parameter x 1/16 and x 1/256
    # ("wsd"), and the network rescaled so every hidden activation is ~1/256 as large ("homog")
    for s, tag in ((1 / 16, "wsd16"), (1 / 256, "wsd256")):
        run_case(f"ou_pis32_{tag}_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 2, 64, 2, 61, workdir=wd,
                 weight_scale=s)
        run_case(f"gbm_mlp16_sdgd_{tag}_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16, 16]}, 2, 64, 2,
                 62, v=100, workdir=wd, weight_scale=s)
        run_case(f"gbm_mlp64x3_sdgd_{tag}_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [64] * 3}, 2, 64, 2,
                 63, v=100, workdir=wd, weight_scale=s)
        run_case(f"gbm_hess_mlp32x3_{tag}_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [32] * 3}, 2, 64, 2,
                 64, workdir=wd, weight_scale=s, hessians=True)
    run_case("ou_pis32_homog256_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 2, 64, 2, 65, workdir=wd,
             homog=1 / 256)
    run_case("gbm_mlp64x3_sdgd_homog256_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [64] * 3}, 2, 64, 2,
             66, v=100, workdir=wd, homog=1 / 256)
    run_case("gbm_hess_mlp32x3_homog256_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [32] * 3}, 2, 64, 2,
             67, workdir=wd, homog=1 / 256, hessians=True)
    run_case("cha_mlp128x4_homog256_K3", "Cha", cha, "mlp", {"neurons": [128] * 4}, 2, 64, 3, 68, workdir=wd,
             homog=1 / 256)
    # n_estimate_terminal != n_estimate_integral (data.py:444 / :460, :1164 / :845): terminal over MT paths
    run_case("cha_mlp16_MT2x_K2", "Cha", cha, "mlp", {"neurons": [16, 16]}, 3, 64, 2, 71, workdir=wd, MT=128)
    run_case("ou_pis32_MTh_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 2, 128, 2, 72, workdir=wd,
             MT=64)
    run_case("gbm_mlp64x3_sdgd_MT2x_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [64] * 3}, 2, 64, 2, 73,
             v=100, workdir=wd, MT=128)
    run_case("gbm_hess_mlp32x3_MT2x_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [32] * 3}, 2, 64, 2, 74,
             workdir=wd, hessians=True, MT=128)
    run_case("gbm_hess_mlp16_MTh_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16]}, 2, 128, 2, 75,
             workdir=wd, hessians=True, MT=64)
    # Fully-nonlinear case_1 (GBM): SDGD v=100 and full-Hessian (v=0), MLP 3x16
    run_case("gbm_mlp16_sdgd_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16, 16]}, 3, 64, 2, 3,
             v=100, workdir=wd)
    run_case("gbm_mlp16_full_K1", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16]}, 2, 64, 1, 4,
             workdir=wd)
    # Malliavin Hessian labels (generate_with_gradients_and_hessians), full-Hessian f
    run_case("gbm_hess_mlp16_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16]}, 2, 64, 2, 6,
             epoch=1, workdir=wd, hessians=True)
    run_case("gbm_hess_mlp32x3_K4", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [32] * 3}, 2, 128, 4, 8,
             epoch=2, point_base=5, workdir=wd, hessians=True)
    run_case("gbm_hess_zero_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [8]}, 2, 64, 2, 9,
             workdir=wd, zero=True, hessians=True)
    # TD estimators (DATA.ESTIMATE_DELTA_T > 0, data.py:1209-1213): points on both sides of
    # t + delta_t = T (n = 8 points, t ~ U(0.01, 0.99))
    run_case("td_cha_mlp16_K2", "Cha", cha, "mlp", {"neurons": [16, 16]}, 8, 64, 2, 21, workdir=wd, delta_t=0.3)
    run_case("td_cha_mlp64x3_K5", "Cha", cha, "mlp", {"neurons": [64] * 3}, 6, 64, 5, 22, epoch=2, workdir=wd,
             delta_t=0.45)
    run_case("td_cha_zero_K1", "Cha", cha, "mlp", {"neurons": [8]}, 6, 64, 1, 23, workdir=wd, zero=True, delta_t=0.2)
    run_case("td_ou_mlp32_K3", "OUProcessEquation", ou, "mlp", {"neurons": [32, 32]}, 6, 64, 3, 24, workdir=wd,
             delta_t=0.35)
    run_case("td_gbm_mlp16_sdgd_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16]}, 6, 64, 2, 25,
             v=100, workdir=wd, delta_t=0.4)
    run_case("td_ou_pis32_K2", "OUProcessEquation", ou, "pis", {"neurons": [32, 32]}, 6, 64, 2, 26, workdir=wd,
             delta_t=0.55)
    # sample_t (t_always_uniform: false, data.py:149-159): t = T (1 - prod of N - i + 1 uniforms)
    run_case("tprod_cha_mlp16_K2", "Cha", cha, "mlp", {"neurons": [16, 16]}, 6, 64, 2, 31, workdir=wd,
             picard_N=5, picard_i=2, t_uniform=False)
    run_case("tprod_ou_mlp16_K2", "OUProcessEquation", ou, "mlp", {"neurons": [16, 16]}, 5, 64, 2, 32, epoch=4,
             workdir=wd, picard_N=3, picard_i=3, t_uniform=False)
    run_case("tprod_gbm_mlp16_sdgd_K1", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16]}, 5, 64, 1, 33,
             v=100, workdir=wd, picard_N=9, picard_i=3, t_uniform=False)
    # torch.nn.Tanh hidden layers (the reference's default NETWORK.ACTIVATIONS, picard/config.py:61)
    run_case("cha_mlp16_tanh_K2", "Cha", cha, "mlp", {"neurons": [16, 16], "act": "Tanh"}, 4, 64, 2, 51, workdir=wd)
    run_case("cha_mlp128x4_tanh_K3", "Cha", cha, "mlp", {"neurons": [128] * 4, "act": "Tanh"}, 2, 64, 3, 52,
             epoch=1, workdir=wd)
    run_case("ou_mlp64x2_tanh_K2", "OUProcessEquation", ou, "mlp", {"neurons": [64, 64], "act": "Tanh"}, 3, 64, 2,
             53, workdir=wd)
    run_case("gbm_mlp64x3_tanh_sdgd_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [64] * 3, "act": "Tanh"},
             2, 64, 2, 54, v=100, workdir=wd)
    run_case("gbm_mlp16_tanh_full_K1", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [16, 16], "act": "Tanh"},
             2, 64, 1, 55, workdir=wd)
    run_case("gbm_hess_mlp32x3_tanh_K2", "GBMEquationComplexExact", gbm, "mlp", {"neurons": [32] * 3, "act": "Tanh"},
             2, 64, 2, 56, workdir=wd, hessians=True)
    run_case("td_cha_mlp32_tanh_K2", "Cha", cha, "mlp", {"neurons": [32, 32], "act": "Tanh"}, 6, 64, 2, 57,
             workdir=wd, delta_t=0.35)
    # state dimensions above 128 (the wide first-order instances, nx <= 256; equations.py takes any nx)
    cha200 = {**cha, "nx": 200}
    cha256 = {**cha, "nx": 256}
    run_case("wide_cha200_mlp64x3_K2", "Cha", cha200, "mlp", {"neurons": [64] * 3}, 2, 64, 2, 81, workdir=wd)
    run_case("wide_cha256_mlp128x4_tanh_K2", "Cha", cha256, "mlp", {"neurons": [128] * 4, "act": "Tanh"}, 2, 64, 2,
             82, epoch=1, workdir=wd)
    run_case("wide_cha256_mlp16_K2", "Cha", cha256, "mlp", {"neurons": [16, 16]}, 2, 64, 2, 83, workdir=wd)
    run_case("wide_cha256_zero_K1", "Cha", cha256, "mlp", {"neurons": [8]}, 2, 64, 1, 84, workdir=wd, zero=True)
    run_case("wide_ou200_mlp32x2_K2", "OUProcessEquation", {**ou, "nx": 200}, "mlp", {"neurons": [32, 32]}, 2, 64, 2,
             85, workdir=wd)
    run_case("wide_ou256_mlp128x4_K2", "OUProcessEquation", {**ou, "nx": 256}, "mlp", {"neurons": [128] * 4}, 2, 64,
             2, 86, workdir=wd)
    run_case("wide_gbm200_mlp64x3_sdgd_K2", "GBMEquationComplexExact", {**gbm, "nx": 200}, "mlp", {"neurons": [64] * 3},
             2, 64, 2, 87, v=100, workdir=wd)
    run_case("wide_gbm256_mlp32x2_tanh_sdgd_K2", "GBMEquationComplexExact", {**gbm, "nx": 256}, "mlp",
             {"neurons": [32, 32], "act": "Tanh"}, 2, 64, 2, 88, v=200, workdir=wd)
    run_case("wide_gbm256_mlp16_full_K1", "GBMEquationComplexExact", {**gbm, "nx": 256}, "mlp", {"neurons": [16, 16]},
             2, 64, 1, 89, workdir=wd)
    shutil.rmtree(wd)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
