"""Host-side cost of one bench step (GBM workload): wall time per call with and without syncs."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import deeppicarditeration_amd as dpi  # noqa: E402
from deeppicarditeration_amd.sharding import ShardedLabeler  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "gbm"]
eq, net = bench._make(wl, dpi)
hess = {"method": "SDGD", "kwargs": {"v": wl["sdgd"]}} if wl["sdgd"] else None
gen = dpi.OnlineDataGenerator(eq, net, 80, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=wl["m_per_gpu"],
                              n_estimate_integral=wl["m_per_gpu"], n_euler_steps=wl["K"], seed=1,
                              hessian_approximation=hess)
lab = ShardedLabeler(gen)
for _ in range(5):
    tx, pb = gen.sample_t_and_x(wl["points"])
    lab.labels(tx, pb)
torch.cuda.synchronize()
for rnd in range(3):
    th = {"sample": 0.0, "labels": 0.0}
    t0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        tx, pb = gen.sample_t_and_x(wl["points"])
        b = time.perf_counter()
        lab.labels(tx, pb)
        c = time.perf_counter()
        th["sample"] += b - a
        th["labels"] += c - b
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"wall/step {dt/20*1e3:.3f} ms  host sample {th['sample']/20*1e3:.3f} ms  host labels {th['labels']/20*1e3:.3f} ms",
          flush=True)
