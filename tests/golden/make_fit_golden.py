"""Golden vectors for the outer fit from the REFERENCE's training steps.

Runs only in the build container (needs /root/reference, read-only; the module stand-ins and the
package bypass are make_golden.py's).  For each case it builds the reference's `PicardSolution`
(construct_mlp value network) in fp64, wraps it exactly as `PicardRunner.get_solution` does
(picard_iteration.py:113-118 -> PicardSolutionGradientWrapper / PicardSolutionGradientHessianWrapper
.construct_solution, solution_jac.py:112-136), and runs S optimizer steps of its `training_step`
(solution.py:74-81, solution_jac.py:167-213, :219-259) on fixed batches, with the optimizer the
reference configures (torch.optim.<cls>(**kwargs), solution.py:94-97).  Stored: the case
configuration, initial weights, batches, the per-step losses and the final weights (data only).

Usage:  python tests/golden/make_fit_golden.py
"""
import importlib
import json
import random
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as mg  # noqa: E402  (installs the stand-ins, imports the reference)

sj = importlib.import_module("picard.solution_jac")
CfgNode = mg.CfgNode

CASES = {
    # name: (nx, neurons, beta, scaler (cls, kwargs) | None, loss-fn clip | None, supervise, NUM_HESS_SAMPLES)
    "fit_grad_fixed": (100, [16, 16], 0.5, ("FixedLossScaler", {"fixed_weight": 0.1}), None, "gradient", -1),
    "fit_grad_clip_simple": (100, [16, 16], 1.0, ("SimpleLossScaler", {}), 0.1, "gradient", -1),
    "fit_grad_dimension": (100, [16, 16], 0.0, ("DimensionLossScaler", {}), None, "gradient", -1),
    "fit_grad_default_scaler": (100, [16, 16], 0.5, None, None, "gradient", -1),
    "fit_value_zero_weight": (100, [16, 16], 2.0, ("FixedLossScaler", {"fixed_weight": 0.0}), 0.2, "gradient", -1),
    "fit_value_only": (100, [16, 16], 0.5, None, None, "value", -1),
    "fit_hess_full": (6, [8, 8], 0.5, ("FixedHessianLossScaler", {"fixed_gradient_weight": 0.1,
                                                                   "fixed_hessian_weight": 0.01}), None, "hessian", -1),
    "fit_hess_sampled": (6, [8, 8], 0.0, ("FixedHessianLossScaler", {"fixed_gradient_weight": 0.3,
                                                                      "fixed_hessian_weight": 0.05}), 0.5, "hessian", 10),
}
S, B, LR, HESS_SEED = 4, 32, 1e-2, 7


def train_cfg(beta, scaler, clip, n_hess):
    return CfgNode({
        "LOSS": CfgNode({
            "beta": beta,
            "SCALER": CfgNode({"cls": scaler[0] if scaler else None, "kwargs": CfgNode(scaler[1] if scaler else {})}),
            "FN": CfgNode({"cls": "LossFnLinearClip" if clip is not None else None,
                           "kwargs": CfgNode({"clip": clip} if clip is not None else {})}),
            "use_aux_loss": False, "weight_aux_loss": 0.1}),
        "NUM_HESS_SAMPLES": n_hess,
        "OPTIMIZER": CfgNode({"cls": "Adam", "kwargs": CfgNode({"lr": LR})}),
    })


def run(name):
    nx, neurons, beta, scaler, clip, sup, n_hess = CASES[name]
    torch.set_default_dtype(torch.float64)
    eq = mg.eqs.Cha(nx, 1.0, 5.0, 1.0)
    tcfg = train_cfg(beta, scaler, clip, n_hess)
    ncfg = CfgNode({"TYPE": "Value", "PISGRADNET": False, "NEURONS": neurons, "ACTIVATIONS": ["ELU"] * len(neurons),
                    "BOUND": None})
    torch.manual_seed(sum(map(ord, name)))
    plain = mg.sols.PicardSolution(eq, ncfg, tcfg)

    class Runner:  # the parts of PicardRunner construct_solution reads
        def get_solution_plain(self):
            return plain

    if sup == "hessian":
        model = sj.PicardSolutionGradientHessianWrapper.construct_solution(Runner())
    elif sup == "gradient":
        model = sj.PicardSolutionGradientWrapper.construct_solution(Runner())
    else:
        model = plain
    init = {k: v.detach().clone().numpy() for k, v in plain.model.state_dict().items()}
    width = 1 + nx + (nx * nx if sup == "hessian" else 0)
    g = torch.Generator().manual_seed(11)
    tx = torch.cat([torch.rand(S, B, 1, generator=g), torch.randn(S, B, nx, generator=g)], -1)
    y = 0.5 * torch.randn(S, B, width, generator=g)
    opt = torch.optim.Adam(model.parameters(), lr=LR)
    random.seed(HESS_SEED)
    losses = []
    for s in range(S):
        loss = model.training_step((tx[s], y[s]), s)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    final = {k: v.detach().numpy() for k, v in plain.model.state_dict().items()}
    cfg = {"nx": nx, "neurons": neurons, "beta": beta, "scaler": scaler, "clip": clip, "supervise": sup,
           "num_hess_samples": n_hess, "lr": LR, "hess_seed": HESS_SEED,
           "wrapped": type(model).__name__}
    out = {"cfg": np.array(json.dumps(cfg)), "tx": tx.numpy(), "y": y.numpy(), "losses": np.array(losses)}
    out.update({f"init.{k}": v for k, v in init.items()})
    out.update({f"final.{k}": v for k, v in final.items()})
    np.savez_compressed(HERE / "fit" / f"{name}.npz", **out)
    print(name, cfg["wrapped"], losses)


if __name__ == "__main__":
    for n in (sys.argv[1:] or CASES):
        run(n)
