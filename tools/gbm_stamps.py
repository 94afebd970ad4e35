"""Per-phase time of the GBM network launch (k_paths<GBM, 64, 3, split>) from s_memtime stamps.

Needs the stamp variant:  python tools/build_variant.py stamps --units dpi_paths_gbm.hip -DDPI_GBM_STAMPS
then  DPI_HIP_LIB=tools/variants/libdpi_stamps.so python tools/gbm_stamps.py
Events per wave: 0 start, 1 rollouts done, 2 terminal finish (barrier), 3 sweep start (forward,
adjoint, per-path direction lists done), 4 sweep done, 5 integrand + barrier, 6 end (phase 3 and
the fused reduce).  Prints the median cycles of each interval over the launch's waves, and the
block-level spread of start times (how the 1,024 blocks fill the CUs)."""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

NB, NW, NEV = 1024, 4, 8


def main():
    torch.manual_seed(0)
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    M, n = 1024, 64
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=50, seed=1,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    ws = gen.point_baseline(tx)
    for _ in range(20):
        gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    torch.cuda.synchronize()
    lib = L.load()
    buf = np.zeros(NB * NW * NEV * 2, dtype=np.uint64)
    fn = lib.dpi_debug_gbm_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(NB, NW, NEV, 2)[:, :, :, 0].astype(np.int64)
    names = ["rollouts", "terminal finish", "fwd+adj+lists", "sweep", "integrand rest", "phase 3 + reduce"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6)]
    tot = np.median(st[:, :, 6] - st[:, :, 0])
    print(f"wave lifetime: median {tot:.0f} cycles")
    for nm, (a, b) in zip(names, pairs):
        d = (st[:, :, b] - st[:, :, a]).ravel()
        print(f"{nm:18s} median {np.median(d):9.0f}  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}"
              f"  ({np.median(d) / tot:.1%})")
    t0 = st[:, 0, 0]
    print("block start spread (cycles from the first):", np.percentile(t0 - t0.min(), [0, 25, 50, 75, 100]).astype(int))
    print("launch span:", int(st[:, :, 6].max() - t0.min()), "cycles")


if __name__ == "__main__":
    main()
