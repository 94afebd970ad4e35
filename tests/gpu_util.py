"""Shared helpers for the GPU parity tests: build the product objects from golden fixtures."""
import numpy as np
import torch

import deeppicarditeration_amd as dpi
from golden_util import acts, delta_t, m_terminal, state_dict, t_factors


def product_equation(f):
    eq = str(f["eq"])
    if eq == "Cha":
        return dpi.Cha(int(f["eqkw_nx"]), float(f["eqkw_alpha"]), float(f["eqkw_k"]), float(f["eqkw_T"]))
    if eq == "OUProcessEquation":
        # the reference ships its GMM files for nx = 100 only; at other nx it drew new parameters
        # (equations.py:533-544), which the fixture holds
        gmm = {} if int(f["eqkw_nx"]) == 100 else dict(mean=f["gmm_mean"], var=f["gmm_var"], pi=f["gmm_pi"])
        e = dpi.OUProcessEquation(nx=int(f["eqkw_nx"]), T=float(f["eqkw_T"]), alpha=float(f["eqkw_alpha"]),
                                  num_components=int(f["eqkw_num_components"]), mean_scale=float(f["eqkw_mean_scale"]),
                                  var_scale=float(f["eqkw_var_scale"]), alpha_scale=float(f["eqkw_alpha_scale"]),
                                  **gmm)
        assert np.allclose(e.mean.numpy(), f["gmm_mean"]) and np.allclose(e.pi.numpy(), f["gmm_pi"])
        return e
    if eq == "GBMEquationComplexExact":
        # the reference ships w / v for nx = 100 only; at other nx it drew them (equations.py:408-420)
        wv = {} if int(f["eqkw_nx"]) == 100 else dict(w=f["gbm_w"], v=f["gbm_v"])
        return dpi.GBMEquationComplexExact(int(f["eqkw_nx"]), float(f["eqkw_alpha"]), float(f["eqkw_T"]), **wv)
    raise ValueError(eq)


def product_module(f, eq):
    kind = str(f["net"])
    if kind == "zero":
        return dpi.ZeroSolution(1)
    sd = {k: torch.as_tensor(v).float() for k, v in state_dict(f).items()}
    if kind == "mlp":
        neurons = [int(v) for v in f["neurons"]]
        m = dpi.construct_mlp(1 + eq.nx, 1, neurons, acts(f, len(neurons)), None)
        m.load_state_dict(sd)
        return m
    m = dpi.PISGradNet(hidden_shapes=[int(v) for v in f["neurons"]], dim=eq.nx, g0=eq.g, T=eq.T)
    m.load_state_dict(sd)
    return m


def generator(f, eq, module, M=None, K=None):
    """The fixture's generator; M overrides both estimator counts (else the fixture's
    n_estimate_integral M and n_estimate_terminal MT)."""
    MT = m_terminal(f) if M is None else M
    M = int(f["M"]) if M is None else M
    v = int(f["v"])
    hess = {"method": "SDGD", "kwargs": {"v": v}} if v > 0 else None
    R = t_factors(f)  # sample_t fixtures: a Picard (N, i) with N - i + 1 = R
    return dpi.OnlineDataGenerator(eq, module, R if R else 1, 1, device="cuda:0", t_always_uniform=R == 0,
                                   n_estimate_terminal=MT,
                                   n_estimate_integral=M, n_euler_steps=int(f["K"]) if K is None else K,
                                   seed=int(f["seed"]), epoch=int(f["epoch"]), hessian_approximation=hess,
                                   estimate_delta_t=delta_t(f))


def rel_l2_parts(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)

    def r(x, y):
        return float(np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-300))

    return {"value": r(a[:, :1], b[:, :1]), "grad": r(a[:, 1:], b[:, 1:]), "all": r(a, b)}
