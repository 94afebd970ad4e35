"""Ablation of k_paths variants on the Burgers bench workload (interleaved rounds, one process):
DPI_ORDER phase-order policy x fused-MLP precision (DPI_GEMM_F32 / DPI_GEMM_AUTO = fp16-split).
usage: perf_order.py [order:mode ...]   e.g. 0:0 0:2 4:2"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.perf_probe import bench, make  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402


def main():
    variants = [tuple(int(x) for x in v.split(":")) for v in (sys.argv[1:] or ["0:0", "0:2", "4:0", "4:2"])]
    lib = L.load()
    objs = make("128x4", int(os.environ.get("PERF_K", "50")))
    gen, tx, ws = objs
    res = {v: [] for v in variants}
    moms = {}
    for rnd in range(5):
        for v in variants:
            os.environ["DPI_ORDER"] = str(v[0])
            L.check(lib.dpi_set_gemm_precision(v[1]), "gemm")
            res[v].append(bench(*objs, L.DPI_BOTH))
            moms[v] = gen.label_moments(tx, 0, 4096, 0, 4096, L.DPI_BOTH, ws).clone()
    base = moms[variants[0]]
    for v in variants:
        t = sorted(res[v])
        d = (moms[v] - base).norm() / base.norm()
        print(f"order={v[0]} gemm={v[1]}  median {t[len(t)//2]*1e3:7.1f} us  min {t[0]*1e3:7.1f} us  "
              f"{16*4096/(t[len(t)//2]*1e-3):.3e} path-labels/s  rel-diff vs first {float(d):.2e}", flush=True)


if __name__ == "__main__":
    main()
