"""Ablation timings of dpi_label_moments on one GPU (interleaved rounds in one process)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402


def make(net_kind, K, M=4096, n=16):
    torch.manual_seed(0)
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    if net_kind == "zero":
        net = dpi.ZeroSolution()
    else:
        w = [int(v) for v in net_kind.split("x")]
        net = dpi.construct_mlp(101, 1, [w[0]] * w[1], ["ELU"] * w[1], None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    ws = gen.point_baseline(tx)
    return gen, tx, ws


def bench(gen, tx, ws, flags, M=4096, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        gen.label_moments(tx, 0, M, 0, M, flags, ws)
    e0.record()
    for _ in range(reps):
        gen.label_moments(tx, 0, M, 0, M, flags, ws)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    cases = []
    for net in ["zero", "128x4"]:
        for K in [1, 10, 50]:
            for fl, nm in [(L.DPI_BOTH, "both"), (L.DPI_TERMINAL, "term"), (L.DPI_INTEGRAL, "int")]:
                cases.append((net, K, fl, nm))
    objs = {}
    res = {c: [] for c in cases}
    for rnd in range(3):
        for c in cases:
            net, K, fl, nm = c
            if (net, K) not in objs:
                objs[(net, K)] = make(net, K)
            res[c].append(bench(*objs[(net, K)], fl))
    for c in cases:
        v = sorted(res[c])
        ms = v[len(v) // 2]
        print(f"net={c[0]:6s} K={c[1]:3d} {c[3]:5s}  {ms*1e3:8.1f} us   {16*4096/ms/1e3:.3e} path-labels/s")


if __name__ == "__main__":
    main()
