"""Small-magnitude probe of the fp16-split MFMA paths: labels of networks whose
parameters are scaled DOWN, against the fp64 oracle, in both GEMM modes.

  all      every parameter x s (activations and cotangents shrink)
  interior hidden layers x s (weights and biases), output weights x s^-L: the labels keep their
           size while every stored activation is ~s times smaller (ill-conditioned: fp32 loses too)
  homog    first layer x s, the other hidden biases x s, output weights x 1/s: every hidden
           activation ~s times smaller, the network ~the same function (the split's hard case)

Prints one JSON line per case (tool, not a test)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402
from oracle import dpi_oracle as O  # noqa: E402


def rel(a, b, hess=False):
    r = lambda x, y: float(np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-300))  # noqa: E731
    out = {"value": r(a[:, :1], b[:, :1]), "grad": r(a[:, 1:101], b[:, 1:101])}
    if hess:
        out["hess"] = r(a[:, 101:], b[:, 101:])
    return out


def scale_seq(lin, s, how):
    with torch.no_grad():
        if how == "all":
            for m in lin:
                m.weight.mul_(s)
                m.bias.mul_(s)
        elif how == "homog":
            lin[0].weight.mul_(s)
            lin[0].bias.mul_(s)
            for m in lin[1:-1]:
                m.bias.mul_(s)
            lin[-1].weight.mul_(1.0 / s)
        else:  # interior
            for m in lin[:-1]:
                m.weight.mul_(s)
                m.bias.mul_(s)
            lin[-1].weight.mul_(s ** -(len(lin) - 1))


def mlp_case(eqname, widths, s, how, mode, M=256, K=10, v=0, hess=False):
    torch.manual_seed(3)
    if eqname == "cha":
        eq, oeq = dpi.Cha(100, 1.0, 5.0, 1.0), O.Cha(100, 1.0, 5.0, 1.0)
    else:
        eq = dpi.GBMEquationComplexExact(100)
        oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    net = dpi.construct_mlp(101, 1, widths, ["ELU"] * len(widths), None)
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    scale_seq(lin, s, how)
    L.check(L.load().dpi_set_gemm_precision(mode), "prec")
    hap = {"method": "SDGD", "kwargs": {"v": v}} if v else None
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1, hessian_approximation=hap)
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU"] * (len(lin) - 1))
    if hess:
        tx, y = gen.sample_with_gradients_and_hessians(2)
        ref = O.labels_grad_hess(oeq, onet, tx.cpu().double().numpy(), M, K, 1, 1, 0)
    else:
        tx, y = gen.sample_with_gradients(2)
        ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), M, K, 1, 1, 0, v=v)
    return {"net": f"{eqname}-mlp{widths}" + ("-hess" if hess else ""), "scale": s, "how": how, "mode": mode,
            "finite": bool(torch.isfinite(y).all()), "max_abs_label": float(abs(ref).max()),
            **rel(y.cpu().double().numpy(), ref, hess)}


def pis_case(s, how, mode, M=128, K=10):
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(7)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    with torch.no_grad():
        net.timestep_phase.copy_(0.1 * torch.randn(1, 64))
        if how == "all":
            for p in net.parameters():
                if p is not net.timestep_phase:
                    p.mul_(s)
        elif how == "tenc":  # the time embedding part of nn_module's input small
            for m in net.t_encoder:
                if isinstance(m, torch.nn.Linear):
                    m.weight.mul_(s)
                    m.bias.mul_(s)
        else:
            scale_seq([m for m in net.nn_module if isinstance(m, torch.nn.Linear)], s, how)
    L.check(L.load().dpi_set_gemm_precision(mode), "prec")
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=2)
    tx, y = gen.sample_with_gradients(2)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), M, K, 2, 1, 0)
    return {"net": "ou-pis512x4", "scale": s, "how": how, "mode": mode, "finite": bool(torch.isfinite(y).all()),
            "max_abs_label": float(abs(ref).max()), **rel(y.cpu().double().numpy(), ref)}


if __name__ == "__main__":
    only = sys.argv[1] if len(sys.argv) > 1 else ""  # case prefix (pis, gbm, hess, cha)
    hows = sys.argv[2].split(",") if len(sys.argv) > 2 else None  # scalings to run
    cases = []
    for s, how in ((1 / 16, "homog"), (1 / 256, "homog"), (1 / 4096, "homog"), (1.0, "all"), (1 / 16, "all"),
                   (1 / 256, "all"), (1 / 16, "interior"), (1 / 256, "interior")):
        if hows and how not in hows:
            continue
        cases += [("pis", lambda mode, s=s, how=how: pis_case(s, how, mode)),
                  ("gbm", lambda mode, s=s, how=how: mlp_case("gbm", [64] * 3, s, how, mode, v=100)),
                  ("hess", lambda mode, s=s, how=how: mlp_case("gbm", [64] * 3, s, how, mode, hess=True)),
                  ("cha", lambda mode, s=s, how=how: mlp_case("cha", [128] * 4, s, how, mode))]
    cases += [("pis", lambda mode: pis_case(1 / 256, "tenc", mode))]
    for name, fn in cases:
        if only and not name.startswith(only):
            continue
        for mode in (L.DPI_GEMM_AUTO, L.DPI_GEMM_F32):
            try:
                print(json.dumps(fn(mode)), flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"case": name, "mode": mode, "error": str(e)[:300]}), flush=True)
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "prec")
