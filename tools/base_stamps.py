"""Per-phase time of the per-point baseline launch (k_baseline) from s_memtime stamps.

Needs the stamp variant:
    python tools/build_variant.py bstamps --units dpi_paths_cha.hip,dpi_paths_gbm.hip -DDPI_BASE_STAMPS
then  DPI_HIP_LIB=tools/variants/libdpi_bstamps.so python tools/base_stamps.py
Stamps (thread 0 of each block, after the barrier that closes a phase): 0 start, 1 point loaded /
sampled, 2 g(x), 3 GBM exact-solution terms, 4 forward layers, 5 value (Cha) / adjoints (GBM),
6 adjoint chain (Cha) / tangent init (GBM), 7-8 tangent layers (GBM), 10 end; inside the second
mat-vec: 11 start, 12 slice loads + fma done (part stored), 13 after its barrier, 14 owner sum done.  Prints the median
cycles of each interval over the launch's blocks for the bench workloads' shapes."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

NB, NEV = 512, 16


def read(lib, unit):
    buf = np.zeros(NB * NEV, dtype=np.uint64)
    fn = getattr(lib, f"dpi_debug_base_stamps_{unit}")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    return buf.reshape(NB, NEV).astype(np.int64)


def report(name, st, n, evs):
    st = st[:n]
    print(f"== {name}: {n} blocks")
    tot = st[:, evs[-1]] - st[:, evs[0]]
    print(f"  block lifetime median {np.median(tot):8.0f} cycles  (p10 {np.percentile(tot, 10):.0f}, "
          f"p90 {np.percentile(tot, 90):.0f})")
    for a, b in zip(evs[:-1], evs[1:]):
        d = st[:, b] - st[:, a]
        print(f"  {a:2d} -> {b:2d}  median {np.median(d):8.0f}  ({np.median(d) / np.median(tot):5.1%})")
    t0 = st[:, evs[0]]
    print("  block start spread:", np.percentile(t0 - t0.min(), [0, 50, 100]).astype(int),
          " launch span:", int(st[:, evs[-1]].max() - t0.min()))


def main():
    torch.manual_seed(0)
    lib = L.load()
    # Burgers (bench default): Cha 100-d, MLP 101-128x4-1, 1024 points sampled inside the launch
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = dpi.construct_mlp(101, 1, [128] * 4, ["ELU"] * 4, None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                  n_estimate_integral=64, n_euler_steps=50, seed=1)
    n = 1024
    ws = torch.empty(gen.workspace_bytes(n, 64), dtype=torch.uint8, device="cuda:0")
    for _ in range(20):
        gen.sample_points_baseline(n, 0, ws)
    st = read(lib, "cha")
    report("Burgers k_baseline<Cha> with in-block sampling (n = 1024)", st, min(n, NB), [0, 1, 2, 4, 5, 6, 10])
    report("  its second mat-vec (layer 2): loads + fma + part store / barrier / owner sum", st, min(n, NB),
           [11, 12, 13, 14])
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    for _ in range(20):
        gen.point_baseline(tx, ws=ws)
    report("Burgers k_baseline<Cha>, points given (n = 1024)", read(lib, "cha"), min(n, NB), [0, 1, 2, 4, 5, 6, 10])
    # GBM (bench gbm / gbm_hess): 101-64x3-1, 64 points
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=1024,
                                  n_estimate_integral=1024, n_euler_steps=50, seed=1,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    n = 64
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    for _ in range(20):
        gen.point_baseline(tx)
    report("GBM k_baseline (n = 64)", read(lib, "gbm"), n, [0, 1, 2, 3, 4, 5, 6, 7, 8, 10])


if __name__ == "__main__":
    main()
