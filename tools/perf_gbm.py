"""GBM (configs[4]) label_moments phase timings on one GPU: 3x64 MLP vs ZeroSolution, K = 50 / 1,
SDGD v = 100 / 0 (full-Hessian trace), terminal / integral / both (interleaved rounds, median)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402
from tools.perf_probe import bench  # noqa: E402

M, N = 1024, 64


def make(net_kind, K, v):
    torch.manual_seed(0)
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = dpi.ZeroSolution() if net_kind == "zero" else dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    ha = {"method": "SDGD", "kwargs": {"v": v}} if v else None
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1, hessian_approximation=ha)
    tx, _ = gen.sample_t_and_x(N, point_base=0)
    ws = gen.point_baseline(tx)
    return gen, tx, ws


def main():
    cases = [(net, K, v, fl, nm) for net in ("zero", "mlp") for K in (1, 50) for v in (100,)
             for fl, nm in ((L.DPI_BOTH, "both"), (L.DPI_TERMINAL, "term"), (L.DPI_INTEGRAL, "int"))]
    objs, res = {}, {c: [] for c in cases}
    for _ in range(3):
        for c in cases:
            key = c[:3]
            if key not in objs:
                objs[key] = make(*key)
            res[c].append(bench(*objs[key], c[3], M=M))
    for c in cases:
        v = sorted(res[c])
        print(f"net={c[0]:5s} K={c[1]:3d} v={c[2]:3d} {c[4]:5s} {v[1]*1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
