"""Benchmark of the DPI label-generation hot path on MI355X (BASELINE.json metric).

One step = one `sample_with_gradients` pass over one synthetic batch: Philox point sampling,
per-point baseline, the fused K-step rollout + u / grad u + label-moment kernel, (for N > 1) the
RCCL all-gather of per-rank label moments and their fixed-order reduction, finalize.

Workload (N = 1): BASELINE configs[1] — Burgers (Cha, nx = 100, k = 5, T = 1), 4x128 ELU MLP
(random init, torch.manual_seed(0)), 16 points x M = 4096 MC paths = 65,536 path-labels,
K = 50 Euler–Maruyama steps.  For N GPUs (weak scaling, BASELINE configs[3] pattern) each rank
owns MC indices [r*4096, (r+1)*4096) of the same 16 points (global M = 4096 N), and the label
moments are combined with one all-gather over RCCL + dpi_moments_reduce.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

N_POINTS = 16
M_PER_GPU = 4096
K_STEPS = 50
NX = 100
WIDTHS = [128, 128, 128, 128]
# algorithmic FLOP per path-label, SURVEY.md §8(d) (Burgers 4x128: MLP fwd 62,208 MAC + input-grad
# 62,080 MAC + EM 2 K nx + misc)
FLOP_PER_PATH_LABEL = 2.72e5
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix = vector peak
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-paths", type=int, default=512, help="MC paths per point in the CPU sample")
    return ap.parse_args()


def cpu_baseline(sample_paths):
    """Time the CPU oracle (oracle/: numpy fp64 restatement) on a bounded sample of the same
    workload: 1 point x `sample_paths` paths x K = 50, same network."""
    from oracle import dpi_oracle as O
    import numpy as np
    import deeppicarditeration_amd as dpi
    torch.manual_seed(0)
    net = dpi.construct_mlp(1 + NX, 1, WIDTHS, ["ELU"] * 4, None)
    lin = [l for l in net if isinstance(l, torch.nn.Linear)]
    onet = O.MLP([l.weight.detach().double().numpy() for l in lin], [l.bias.detach().double().numpy() for l in lin],
                 ["ELU"] * 4)
    oeq = O.Cha(NX, 1.0, 5.0, 1.0)
    tx = O.sample_points(oeq, 1, seed=1)
    t0 = time.perf_counter()
    O.labels_grad(oeq, onet, tx, sample_paths, K_STEPS, 1, 0, 0, m_chunk=sample_paths)
    dt = time.perf_counter() - t0
    cores = 1  # numpy elementwise Philox/Box–Muller runs on one thread
    return {"value": sample_paths / dt, "unit": "path-labels/s", "cores": cores, "kind": "port",
            "sample": f"oracle/dpi_oracle.py labels_grad, fp64 numpy, 1 point x {sample_paths} paths x K={K_STEPS}, "
                      f"{dt:.1f} s on {platform.processor() or platform.machine()} (os.cpu_count={os.cpu_count()})"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from deeppicarditeration_amd.sharding import ShardedLabeler

    torch.manual_seed(0)
    eq = dpi.Cha(NX, 1.0, 5.0, 1.0)
    net = dpi.construct_mlp(1 + NX, 1, WIDTHS, ["ELU"] * 4, None)
    M = M_PER_GPU * world
    gen = dpi.OnlineDataGenerator(eq, net, 80, 1, device=dev, t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K_STEPS, seed=1)
    labeler = ShardedLabeler(gen, rank=rank, world=world, group=None if dist is None else dist.group.WORLD)

    # path-kernel timing with events on the stream the kernels run on (torch's current stream)
    ev = []

    def step():
        tx, pb = gen.sample_t_and_x(N_POINTS)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        y = labeler.labels(tx, pb, on_moments_begin=lambda: e0.record(), on_moments_end=lambda: e1.record())
        ev.append((e0, e1))
        return y

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    k_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    if dist:
        t = torch.tensor([dt, k_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, k_ms = float(t[0]), float(t[1])
    assert torch.isfinite(y).all()
    path_labels_per_step = N_POINTS * M  # all ranks together
    value = path_labels_per_step * args.steps / dt
    if rank == 0:
        per_launch_units = N_POINTS * M_PER_GPU
        achieved = FLOP_PER_PATH_LABEL * per_launch_units / (k_ms * 1e-3) / 1e12
        traffic = None
        tf = ROOT / "profiles" / "traffic_burgers_cfg2.json"
        if tf.exists():
            traffic = json.loads(tf.read_text()).get("hbm_bytes_per_launch")
        out = {
            "metric": "SDE-path labels/sec (100-d, 50 Euler steps); rel-L2 vs ref <= 1e-4 (tests/test_gpu_parity.py)",
            "value": value,
            "unit": "path-labels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox-sampled collocation points; random-init 4x128 ELU MLP, torch.manual_seed(0))",
            "config": {"workload": "Burgers 100d T=1 (Cha k=5), 16 points x 4096 MC paths per GPU, K=50 EM steps, "
                                   "MLP 101-128x4-1 ELU (BASELINE configs[1]; N>1: MC-sharded, configs[3] pattern)",
                       "points": N_POINTS, "mc_paths_per_gpu": M_PER_GPU, "euler_steps": K_STEPS, "nx": NX,
                       "parallelism": f"mc-shard{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_FP32_TFLOPS, "traffic": traffic,
                         "kernel": "k_paths (+ its 2 small block-reduce kernels) per dpi_label_moments call",
                         "kernel_ms": k_ms, "flop_per_path_label": FLOP_PER_PATH_LABEL},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_paths)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
