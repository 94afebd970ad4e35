"""Range / precision probe of the fp16-split MFMA paths: labels with every network parameter scaled
by s (weight_scale of tests/golden/make_golden.py) against the fp64 oracle, both GEMM modes.
Prints one JSON line per case (tool, not a test)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402
from oracle import dpi_oracle as O  # noqa: E402


def rel(a, b):
    import numpy as np
    r = lambda x, y: float(np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-300))  # noqa: E731
    return {"value": r(a[:, :1], b[:, :1]), "grad": r(a[:, 1:], b[:, 1:])}


def mlp_case(eqname, widths, scale, mode, M=256, K=10, v=0):
    torch.manual_seed(3)
    if eqname == "cha":
        eq, oeq = dpi.Cha(100, 1.0, 5.0, 1.0), O.Cha(100, 1.0, 5.0, 1.0)
    else:
        eq = dpi.GBMEquationComplexExact(100)
        oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    net = dpi.construct_mlp(101, 1, widths, ["ELU"] * len(widths), None)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(scale)
    L.check(L.load().dpi_set_gemm_precision(mode), "prec")
    hess = {"method": "SDGD", "kwargs": {"v": v}} if v else None
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1, hessian_approximation=hess)
    tx, y = gen.sample_with_gradients(2)
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU"] * (len(lin) - 1))
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), M, K, 1, 1, 0, v=v)
    yy = y.cpu().double().numpy()
    return {"net": f"{eqname}-mlp{widths}", "scale": scale, "mode": mode, "finite": bool(torch.isfinite(y).all()),
            "max_abs_label": float(abs(ref).max()), **rel(yy, ref)}


def pis_case(width, scale, mode, M=128, K=10):
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(7)
    net = dpi.PISGradNet(hidden_shapes=[width] * 4, dim=100, g0=eq.g, T=1.0)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(scale)
        net.timestep_phase.copy_(0.1 * torch.randn(1, 64))
    L.check(L.load().dpi_set_gemm_precision(mode), "prec")
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=2)
    tx, y = gen.sample_with_gradients(2)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), M, K, 2, 1, 0)
    return {"net": f"ou-pis{width}x4", "scale": scale, "mode": mode, "finite": bool(torch.isfinite(y).all()),
            "max_abs_label": float(abs(ref).max()), **rel(y.cpu().double().numpy(), ref)}


if __name__ == "__main__":
    for scale in (1.0, 1 / 32, 4.0, 8.0, 16.0, 32.0):
        for mode in (L.DPI_GEMM_AUTO, L.DPI_GEMM_F32):
            for case in (lambda: mlp_case("cha", [128] * 4, scale, mode), lambda: mlp_case("gbm", [64] * 3, scale, mode, v=100),
                         lambda: pis_case(512, scale, mode)):
                try:
                    print(json.dumps(case()), flush=True)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"scale": scale, "mode": mode, "error": str(e)[:200]}), flush=True)
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "prec")
