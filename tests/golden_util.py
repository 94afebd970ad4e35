"""Helpers: load golden fixtures (tests/golden/*.npz) into oracle objects."""
from pathlib import Path

import numpy as np

from oracle import dpi_oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def load(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    return {k: z[k] for k in z.files}


def _is_hess(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    return "hessians" in z.files and bool(z["hessians"])


_ALL = sorted(p.stem for p in GOLDEN.glob("*.npz"))
CASES = [c for c in _ALL if not _is_hess(c)]       # sample_with_gradients fixtures
HESS_CASES = [c for c in _ALL if _is_hess(c)]      # sample_with_gradients_and_hessians fixtures


def t_factors(f):
    """0: sample_t_always_uniform; R = N - i + 1: sample_t's product of R uniforms (tprod_* fixtures)."""
    return int(f["t_factors"]) if "t_factors" in f else 0


def m_terminal(f):
    """n_estimate_terminal of a fixture (M, its n_estimate_integral, unless the fixture names it)."""
    return int(f["MT"]) if "MT" in f else int(f["M"])


def delta_t(f):
    """DATA.ESTIMATE_DELTA_T of a fixture (0 = the plain estimators; TD fixtures td_*)."""
    return float(f["delta_t"]) if "delta_t" in f else 0.0


def oracle_equation(f):
    eq = str(f["eq"])
    if eq == "Cha":
        return O.Cha(int(f["eqkw_nx"]), float(f["eqkw_alpha"]), float(f["eqkw_k"]), float(f["eqkw_T"]))
    if eq == "OUProcessEquation":
        return O.OUProcessEquation(int(f["eqkw_nx"]), f["gmm_mean"], f["gmm_var"], f["gmm_pi"],
                                   alpha=float(f["eqkw_alpha"]), T=float(f["eqkw_T"]),
                                   alpha_scale=float(f["eqkw_alpha_scale"]))
    if eq == "GBMEquationComplexExact":
        return O.GBMEquationComplexExact(int(f["eqkw_nx"]), f["gbm_w"], f["gbm_v"],
                                         alpha=float(f["eqkw_alpha"]), T=float(f["eqkw_T"]))
    raise ValueError(eq)


def acts(f, n_hidden):
    """The hidden activations of an MLP fixture (ELU unless the fixture names them)."""
    return [str(a) for a in f["acts"]] if "acts" in f else ["ELU"] * n_hidden


def state_dict(f):
    return {k[3:]: f[k] for k in f if k.startswith("sd_")}


def oracle_net(f, eq):
    kind = str(f["net"])
    if kind == "zero":
        return O.ZeroNet()
    sd = state_dict(f)
    if kind == "mlp":
        idx = sorted({int(k.split(".")[0]) for k in sd})
        Ws = [sd[f"{i}.weight"] for i in idx]
        bs = [sd[f"{i}.bias"] for i in idx]
        return O.MLP(Ws, bs, acts(f, len(Ws) - 1))
    return O.PISGradNet(sd, eq, T=eq.T)
