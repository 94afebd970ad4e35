"""Benchmark of the DPI label-generation hot path on MI355X (BASELINE.json metric).

One step = one `sample_with_gradients` pass over one synthetic batch: Philox point sampling,
per-point baseline, the fused K-step rollout + u / grad u + label-moment kernel, (for N > 1) the
RCCL all-gather of per-rank label moments and their fixed-order reduction, finalize.

Workload (N = 1, default): BASELINE configs[1] — Burgers (Cha, nx = 100, k = 5, T = 1), 4x128 ELU
MLP (random init, torch.manual_seed(0)), 16 points x M = 4096 MC paths = 65,536 path-labels,
K = 50 Euler–Maruyama steps.  N > 1 (default): BASELINE configs[3] — Burgers, 512 points x 4096 MC
paths = 2M path-labels per step in total (strong scaling), rank r owning MC indices
[r 4096/N, (r+1) 4096/N) of the same 512 points, label moments combined with one all-gather over
RCCL + dpi_moments_reduce (`--workload burgers_cfg3` runs the same at N = 1; `--workload burgers`
at N > 1 is the weak-scaling variant, 4096 paths per GPU).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rehearsal of the N > 1 path on ONE GPU (RCCL refuses two ranks on one device):
DPI_BENCH_BACKEND=gloo DPI_BENCH_SHARE_GPU=1 with torch.distributed.run --nproc-per-node 2 runs both
ranks on cuda:0 with the gloo process group; everything above init_process_group — the sharding,
ShardedLabeler's two-phase begin/end with its asynchronous all_gather_into_tensor, the timing
all-reduce — is the code the RCCL run executes.
"""
import argparse
import ctypes
import json
import os
import re
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

NX = 100
PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix = vector peak (v_mfma_f32_16x16x4_f32)
PEAK_F16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense MFMA peak
# fp16-split MFMA (include/dpi.h DPI_GEMM_F16X3, the default): one fp32 product = 3 f16 products
PEAK_SPLIT_TFLOPS = PEAK_F16_TFLOPS / 3.0
PEAK_HBM_GBS = 8000.0
N_SIMD = 1024          # 256 CUs x 4 SIMDs
PEAK_CLOCK_GHZ = 2.4   # MI355X peak engine clock (MI355X_MICROARCH.md)
# workloads = BASELINE.json configs; FLOP per path-label from SURVEY.md §8(d), except GBM, whose
# kernel runs a cheaper algorithm than §8(d) assumes (adjoint + first-order tangents instead of
# second-order forward mode): there the FLOPs it executes are counted.
# "peak": the MFMA the kernel's network evaluation runs on.
WORKLOADS = {
    "burgers": dict(cfg="configs[1]", eq="Cha", widths=[128] * 4, points=16, m_per_gpu=4096, K=50, sdgd=0,
                    flop=2.72e5, peak="split", kernel="k_paths_fb<Cha,128,4,split>: per-point baseline, rollouts, network and label reduce in one launch per sample_with_gradients call (N > 1: k_baseline + k_paths<Cha,128,4,split>)", desc="Burgers 100d T=1 (Cha k=5), 16 points x 4096 MC paths per GPU, K=50 EM steps, "
                                      "MLP 101-128x4-1 ELU (BASELINE configs[1]; N>1: MC-sharded, configs[3] pattern)"),
    "burgers_cfg3": dict(cfg="configs[3]", eq="Cha", widths=[128] * 4, points=512, m_total=4096, K=50, sdgd=0,
                         flop=2.72e5, peak="split", scaling="strong",
                         kernel="k_paths<Cha,128,4,split> + k_reduce per dpi_label_moments call",
                         desc="Burgers 100d T=1 (Cha k=5), 512 points x 4096 MC paths = 2,097,152 path-labels per step "
                              "in total, MC-sharded 4096/N paths per GPU, K=50 EM steps, MLP 101-128x4-1 ELU, one RCCL "
                              "all-gather of label moments + canonical tree reduce (BASELINE configs[3])"),
    "hjb": dict(cfg="configs[2]", eq="OUProcessEquation", widths=[512] * 4, pis=True, points=64, m_per_gpu=4096, K=50,
                sdgd=0, flop=3.73e6, peak="split", kernel="k_pis_rollout + k_pis_time + k_pis_net (the fp16-split "
                                                           "nn_module VJP chain in one launch) + k_pis_final + "
                                                           "k_reduce per dpi_label_moments call",
                desc="HJB 100d T=1 (OUProcessEquation + 5-component GMM), 64 points x 4096 MC paths per GPU, K=50, "
                     "PISGradNet 4x512 (fp16-split MFMA pipeline: forward + VJP chain in one k_pis_net launch) (BASELINE configs[2])"),
    "gbm_hess": dict(cfg="configs[4] stretch (Malliavin Hessian labels)", eq="GBMEquationComplexExact", widths=[64] * 3,
                     points=64, m_per_gpu=1024, K=50, sdgd=0, hess=True, flop=5.14e6, peak="split",
                     kernel="k_paths<GBM,64,3,hessians> + k_reduce + k_reduce_hess per dpi_label_moments_hessians call",
                     desc="Fully-nonlinear case_1 100d (GBM), generate_with_gradients_and_hessians: labels "
                          "(u, u_x, u_xx) = 1 + 100 + 10,000 wide, full-Hessian f at 3 points per path, 64 points x "
                          "1024 MC paths per GPU, K=50, MLP 101-64x3-1 ELU"),
    # not a BASELINE config: the state dimension above 128 (the wide first-order instances)
    "burgers_nx256": dict(cfg="configs[1] shape at nx = 256 (not a BASELINE config)", eq="Cha", nx=256,
                          widths=[128] * 4, points=16, m_per_gpu=4096, K=50, sdgd=0, flop=3.52e5, peak="split",
                          kernel="k_paths<Cha,128,4,split,nx<=256> (one workgroup per CU) after k_baseline",
                          desc="Burgers 256d T=1 (Cha k=5), 16 points x 4096 MC paths per GPU, K=50 EM steps, "
                               "MLP 257-128x4-1 ELU"),
    "gbm": dict(cfg="configs[4]", eq="GBMEquationComplexExact", widths=[64] * 3, points=64, m_per_gpu=1024, K=50,
                sdgd=100, flop=1.68e6, survey_flop=3.36e6, peak="split",
                kernel="k_paths<GBM,64,3> + k_reduce per dpi_label_moments call",
                desc="Fully-nonlinear case_1 100d (GBM, SDGD v=100), 64 points x 1024 MC paths per GPU, K=50, "
                     "MLP 101-64x3-1 ELU (BASELINE configs[4])"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prewarm-s", type=float, default=0.3, help="untimed steps for this long before the warmup")
    ap.add_argument("--cpu-sample-paths", type=int, default=512, help="MC paths per point in the CPU sample")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="default: burgers (configs[1]) at N = 1, burgers_cfg3 (configs[3], 2M paths MC-sharded "
                         "over the N GPUs) at N > 1")
    ap.add_argument("--pipelined", action="store_true", help="two-phase labels also at N = 1 (default: N > 1 only)")
    ap.add_argument("--prepare", action="store_true", help="two-phase labels with the next batch's sampling and "
                                                           "baseline on a low-priority side stream, the path "
                                                           "kernels on a high-priority stream")
    ap.add_argument("--no-prepare", action="store_true", help="one stream (overrides --prepare and the hjb default)")
    ap.add_argument("--range-check", choices=("step", "region", "off"), default="region",
                    help="the product's range guard (data.RangeGroup) inside the timed region: 'region' (default) = "
                         "one group over the timed steps, verified before the clock stops, as picard train's "
                         "LabelBuffer.fill checks one Picard iteration's labels; 'step' = one group per step, "
                         "verified one step behind, as the dataset surface checks each label buffer; 'off' = "
                         "unguarded (finiteness asserted afterwards)")
    ap.add_argument("--no-fp32-pass", action="store_true", help="skip the untimed exact-fp32 comparison pass")
    return ap.parse_args()


def _make(wl, dpi):
    nx = wl.get("nx", NX)
    torch.manual_seed(0)
    if wl["eq"] == "Cha":
        eq = dpi.Cha(nx, 1.0, 5.0, 1.0)
    elif wl["eq"] == "OUProcessEquation":
        eq = dpi.OUProcessEquation(nx=nx, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
    else:
        eq = dpi.GBMEquationComplexExact(nx, 1.0, 1.0)
    if wl.get("pis"):
        net = dpi.PISGradNet(hidden_shapes=wl["widths"], dim=nx, g0=eq.g, T=1.0)
    else:
        net = dpi.construct_mlp(1 + nx, 1, wl["widths"], ["ELU"] * len(wl["widths"]), None)
    return eq, net


def _oracle_objects(wl, eq, net):
    """The CPU oracle's equation and network for a workload (fp64 numpy, oracle/dpi_oracle.py)."""
    from oracle import dpi_oracle as O
    nx = wl.get("nx", NX)
    if wl["eq"] == "Cha":
        oeq = O.Cha(nx, 1.0, 5.0, 1.0)
    elif wl["eq"] == "OUProcessEquation":
        oeq = O.OUProcessEquation(nx, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    else:
        oeq = O.GBMEquationComplexExact(nx, eq.w.numpy(), eq.v.numpy())
    if wl.get("pis"):
        onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    else:
        lin = [m for m in net if isinstance(m, torch.nn.Linear)]
        onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                     ["ELU"] * (len(lin) - 1))
    return oeq, onet


def live_parity(wl, eq, net, tx, pb, y, M):
    """rel-L2 of the first point of the first timed batch against the fp64 oracle on the same
    counters (all M paths, K steps): value column and gradient block (and Hessian block)."""
    import numpy as np
    from oracle import dpi_oracle as O
    oeq, onet = _oracle_objects(wl, eq, net)
    nx = wl.get("nx", NX)
    t0 = time.perf_counter()
    txr = tx[:1].double().cpu().numpy()
    if wl.get("hess"):
        ref = O.labels_grad_hess(oeq, onet, txr, M, wl["K"], 1, 1, pb, m_chunk=256)
    else:
        ref = O.labels_grad(oeq, onet, txr, M, wl["K"], 1, 1, pb, v=wl["sdgd"], m_chunk=512)
    got = y[:1].double().cpu().numpy()
    r = lambda a, b: float(np.linalg.norm(a - b) / np.linalg.norm(b))  # noqa: E731
    out = {"value": r(got[:, :1], ref[:, :1]), "grad": r(got[:, 1:1 + nx], ref[:, 1:1 + nx])}
    if wl.get("hess"):
        out["hessian"] = r(got[:, 1 + nx:], ref[:, 1 + nx:])
    out.update(tolerance=1e-4, what=f"first point of the first timed batch (point index {pb}), {M} paths x "
                                    f"K={wl['K']} vs the fp64 oracle (oracle/dpi_oracle.py) on the same Philox counters",
               oracle_s=round(time.perf_counter() - t0, 2))
    return out


def cpu_baseline(wl, sample_paths, target_s=6.0):
    """The reference's label algorithm on the host cores (oracle/torch_cpu.py: estimate_terminal_
    with_gradients + estimate_integral_with_gradients vectorised in PyTorch, pinned to the
    reference's outputs by tests/test_cpu_baseline.py), same equation / network / M, in fp32 and
    fp64 on all the CPUs this process may use (GBM: the SDGD branch of get_f, one autograd pass per
    sampled index as in the reference; the Malliavin Hessian labels: the _double estimators with the
    full-Hessian get_f, one autograd pass per state dimension)."""
    import deeppicarditeration_amd as dpi
    from oracle import torch_cpu as TC
    eq, net = _make(wl, dpi)
    cores = TC.host_cores()
    model = TC.cpu_model()
    if wl["eq"] in ("Cha", "OUProcessEquation", "GBMEquationComplexExact"):
        from oracle import dpi_oracle as O
        oeq, _ = _oracle_objects(wl, eq, net)

        def points(n, base):
            return torch.from_numpy(O.sample_points(oeq, n, seed=1, point_base=base))
        M = wl.get("m_per_gpu", wl.get("m_total"))
        res = {}
        for dt, name in ((torch.float32, "fp32"), (torch.float64, "fp64")):
            v, pts, secs, th = TC.time_reference_algorithm(eq, net, points, M, dt, target_s=target_s,
                                                           points_per_call=1 if (wl.get("pis") or wl.get("sdgd")
                                                                                 or wl.get("hess")) else 4,
                                                           threads=cores, v=wl.get("sdgd") or None,
                                                           hessians=bool(wl.get("hess")))
            res[name] = {"value": v, "points": pts, "seconds": round(secs, 2)}
        return {"value": res["fp32"]["value"], "unit": "path-labels/s", "cores": cores, "kind": "port",
                "dtype": "fp32", "fp64": res["fp64"]["value"], "cpu": model,
                "sample": (f"oracle/torch_cpu.py: the reference's _double Hessian estimators (data.py:823-897, "
                           f"1153-1201; two half-steps per path, full-Hessian f by autograd) in PyTorch on "
                           if wl.get("hess") else
                           f"oracle/torch_cpu.py: the reference's estimators (data.py:471-527, 899-926; one Gaussian "
                           f"jump per path, autograd grad u{' and SDGD u_ii' if wl.get('sdgd') else ''}) in PyTorch on ") +
                          f"{cores} host threads, {M} paths per point; "
                          f"fp32 {res['fp32']['points']} points in {res['fp32']['seconds']} s, fp64 "
                          f"{res['fp64']['points']} points in {res['fp64']['seconds']} s"}
    from oracle import dpi_oracle as O
    from threadpoolctl import threadpool_limits
    oeq, onet = _oracle_objects(wl, eq, net)
    done, pts = 0, 0
    t0 = time.perf_counter()
    with threadpool_limits(limits=1):  # the restatement is a scalar port: one thread, BLAS included
        while True:
            tx = O.sample_points(oeq, 1, seed=1, point_base=pts)
            if wl.get("hess"):
                O.labels_grad_hess(oeq, onet, tx, sample_paths, wl["K"], 1, 0, pts, m_chunk=min(sample_paths, 256))
            else:
                O.labels_grad(oeq, onet, tx, sample_paths, wl["K"], 1, 0, pts, v=wl["sdgd"],
                              m_chunk=min(sample_paths, 256))
            done += sample_paths
            pts += 1
            dt = time.perf_counter() - t0
            if dt >= target_s:
                break
    return {"value": done / dt, "unit": "path-labels/s", "cores": 1, "kind": "port", "dtype": "fp64", "cpu": model,
            "sample": f"oracle/dpi_oracle.py labels_grad, fp64 numpy, 1 thread, {pts} point(s) x {sample_paths} "
                      f"paths x K={wl['K']} of this workload, {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    backend = os.environ.get("DPI_BENCH_BACKEND", "nccl")  # "gloo": the one-GPU rehearsal (module docstring)
    share = os.environ.get("DPI_BENCH_SHARE_GPU", "0") == "1"
    dev = torch.device(f"cuda:{0 if share else local}")
    torch.cuda.set_device(dev)
    # PISGradNet workloads: the next batch's sampling and baseline run on a low-priority side stream
    # while this batch's GEMM chain runs on a high-priority one (HJB 6.19 -> 5.92 ms/step).  Not for
    # the fused-kernel workloads, whose one path launch the side work would slow.
    if args.workload is None:
        args.workload = "burgers" if world == 1 else "burgers_cfg3"
    # PISGradNet (hjb): the next batch's rollout runs on the side stream beside this batch's k_pis_net,
    # one wave per SIMD (k_pis_rollout_shared) — the default for that workload
    # GBM (configs[4], first-order labels): the next batch's noise sums (k_noise_shared, one wave per
    # SIMD) beside this batch's network launch — 0.768 -> 0.735 ms/step (profiles/r05d_bench_gbm_*)
    # (GBM Hessian labels: `--prepare` stages the next batch's noise sums the same way — bitwise the same
    # labels but slower, 1.88-1.94 against 1.74-1.75 ms/step one-stream, profiles/r06s_hessab; not the default)
    args.prepare = (args.prepare or bool(WORKLOADS[args.workload].get("pis") or args.workload == "gbm")) \
        and not args.no_prepare
    if args.prepare and os.environ.get("DPI_BENCH_MAIN_PRIORITY", "high") == "high":
        lo, hi = torch.cuda.Stream.priority_range()
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=hi))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from deeppicarditeration_amd.sharding import ShardedLabeler

    wl = WORKLOADS[args.workload]
    N_POINTS, K_STEPS = wl["points"], wl["K"]
    if "m_total" in wl:  # strong scaling: the configs[3] total MC width split over the ranks
        M = wl["m_total"]
        if M % (64 * world):
            raise SystemExit(f"{args.workload}: M = {M} is not a multiple of 64 x {world} ranks")
        M_PER_GPU = M // world
    else:  # weak scaling: every rank owns m_per_gpu MC indices of the same points
        M_PER_GPU = wl["m_per_gpu"]
        M = M_PER_GPU * world
    FLOP_PER_PATH_LABEL = wl["flop"]
    eq, net = _make(wl, dpi)
    hess = {"method": "SDGD", "kwargs": {"v": wl["sdgd"]}} if wl["sdgd"] else None
    gen = dpi.OnlineDataGenerator(eq, net, 80, 1, device=dev, t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K_STEPS, seed=1, hessian_approximation=hess)
    # The product's range guard (OnlineDataGenerator.range_check, on by default) runs inside the timed
    # region: each step's label calls form a RangeGroup (their reductions flag into the group's slot of
    # the net's host-visible status ring), verified one step behind — an event wait for work the GPU
    # finished while it runs the next step, then a host read of the slot.
    gen.range_check = args.range_check != "off"
    # PISGradNet under the prepare schedule: each prepare() samples the next batch's points ahead
    labeler = ShardedLabeler(gen, rank=rank, world=world, group=None if dist is None else dist.group.WORLD,
                             sample_ahead=bool(wl.get("pis")) and os.environ.get("DPI_BENCH_SAMPLE_AHEAD", "1") == "1")

    # path-kernel timing: the library's launch timers (dpi_launch_timer_arm) put HIP start / stop
    # events on the timed launch's own dispatch packet (hipExtLaunchKernel) — k_paths / k_paths_fb,
    # or k_pis_net for PISGradNet — so kernel_ms is that launch's duration, not a window of the
    # stream that holds a cross-stream wait or the marker packets of torch events
    ev = []
    tlib = L.load()

    def arm_timer():
        slot = len(ev) % L.DPI_LAUNCH_TIMERS
        L.check(tlib.dpi_launch_timer_arm(slot), "dpi_launch_timer_arm")
        ev.append(slot)

    def timer_ms(slot):
        ms = ctypes.c_float()
        L.check(tlib.dpi_launch_timer_ms(slot, ctypes.byref(ms)), "dpi_launch_timer_ms")
        return ms.value

    # N > 1: two-phase labels, so step i's RCCL all-gather (on RCCL's stream) overlaps step i+1's
    # kernels; every step's full work (sampling, moments, gather, reduce, finalize) still runs
    # inside the timed region (the pipeline is drained before it starts and at its end).
    pipelined = (world > 1 or args.pipelined or args.prepare) and not wl.get("hess")
    pending = []

    # (tx, point_base) of every begun batch, in order; the labels come out in the same order.  The
    # first timed batch's points and labels are kept for the parity check after the timed region.
    begun, capture = [], {}

    def finish(handle):
        y = handle[1] if isinstance(handle[0], str) else labeler.end(handle)
        tx_, pb_ = begun.pop(0)
        if capture.get("armed") and "y" not in capture:
            capture.update(tx=tx_, pb=pb_, y=y)
        return y

    # The path launch of every EV_EVERY-th step is timed: events on the dispatch packet at that rate
    # cost nothing measurable (same-box A/B, profiles/r06i_ab), while timing every launch added
    # 8-35 us per step (r06k)
    EV_EVERY = 4
    nstep = [0]

    def step():
        sampled = nstep[0] % EV_EVERY == 0
        nstep[0] += 1
        rec0 = arm_timer if sampled else None
        rec1 = None
        if args.prepare and pipelined:  # next batch's sampling + baseline on a low-priority side stream
            prep = labeler.prepare(N_POINTS)
            begun.append(prep[:2])
            pending.append(labeler.begin(prepared=prep, on_moments_begin=rec0, on_moments_end=rec1))
            return finish(pending.pop(0)) if len(pending) > 1 else None
        if wl.get("hess") and args.prepare:  # the next batch's points, baseline and noise sums on the side stream
            prep = labeler.prepare(N_POINTS, hessians=True)
            begun.append(prep[:2])
            pending.append(("hess", labeler.labels_hessians(prepared=prep, on_moments_begin=rec0, on_moments_end=rec1)))
            return finish(pending.pop(0))
        if not wl.get("hess") and not pipelined:  # one rank: sampling inside the path launch (one launch)
            tx, pb, y = labeler.sample_labels(N_POINTS, on_moments_begin=rec0, on_moments_end=rec1)
            begun.append((tx, pb))
            pending.append(("done", y))
            return finish(pending.pop(0))
        tx, pb = gen.sample_t_and_x(N_POINTS)
        begun.append((tx, pb))
        if wl.get("hess"):
            pending.append(("hess", labeler.labels_hessians(tx, pb, on_moments_begin=rec0, on_moments_end=rec1)))
            y = finish(pending.pop(0))
        elif pipelined:
            pending.append(labeler.begin(tx, pb, on_moments_begin=rec0, on_moments_end=rec1))
            y = finish(pending.pop(0)) if len(pending) > 1 else None
        else:
            pending.append(("done", labeler.labels(tx, pb, on_moments_begin=rec0, on_moments_end=rec1)))
            y = finish(pending.pop(0))
        return y

    # RangeGroups of the steps not yet verified ("step": one per step, verified one step behind;
    # "region": one over a whole phase, verified after its drain)
    groups = []
    region = [None]
    raw_step = step

    def step():
        if args.range_check != "step":
            return raw_step()
        with gen.deferred_range_check() as grp:
            y = raw_step()
        groups.append(grp)
        if len(groups) > 2:  # the group before the previous one: its batches have all ended
            groups.pop(0).verify()
        return y

    def open_region():
        if args.range_check == "region":
            region[0] = gen.deferred_range_check()

    def drain():
        y = None
        while pending:
            y = finish(pending.pop(0))
        if region[0] is not None:
            region[0].close()
            groups.append(region[0])
            region[0] = None
        while groups:
            groups.pop(0).verify()
        return y

    # Clock ramp: the GPU needs ~10 ms of load to leave its idle clocks, which a 20-step run at
    # ~0.4 ms/step would otherwise spend mostly in.  Run untimed steps for PREWARM_S seconds of
    # wall time first (steady state is what a Picard run sees: it generates labels for minutes),
    # then the W warmup steps of the contract.
    prewarm = 0
    t_pw = time.perf_counter()
    open_region()
    while True:
        for _ in range(16):
            step()
        prewarm += 16
        torch.cuda.synchronize()
        go = torch.tensor([1.0 if time.perf_counter() - t_pw < args.prewarm_s else 0.0], device=dev)
        if dist:  # every rank runs the same number of steps (each step holds a collective)
            dist.broadcast(go, src=0)
        if go.item() == 0.0:
            break
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    ev.clear()
    nstep[0] = 0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    capture["armed"] = True
    t0 = time.perf_counter()
    open_region()
    for _ in range(args.steps):
        y = step()
    y2 = drain()  # every pending batch ended and every range group verified, inside the timed region
    y = y2 if pipelined else y
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    k_ms = sum(timer_ms(slot) for slot in ev) / len(ev)
    if dist:
        t = torch.tensor([dt, k_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, k_ms = float(t[0]), float(t[1])
    assert torch.isfinite(y).all()
    parity = live_parity(wl, eq, net, capture["tx"], capture["pb"], capture["y"], M) if rank == 0 else None
    if rank == 0 and world > 1:
        # the sharded labels against ONE call over all M paths of the same batch on this GPU (after
        # the timed region): bit-identical when M / (64 N) is a power of two
        one = ShardedLabeler(gen, rank=0, world=1)
        y1 = (one.labels_hessians if wl.get("hess") else one.labels)(capture["tx"], capture["pb"])
        parity["bit_identical_to_single_call"] = bool(torch.equal(y1, capture["y"]))
        parity["max_abs_diff_to_single_call"] = float((y1 - capture["y"]).abs().max())
    # Noise floor of the same launch (untimed, after the timed region): the identical rollout with
    # u = 0 (ZeroSolution: same Philox streams, same K-step EM, no network), i.e. the
    # Philox4x32-10 + Box-Muller VALU issue the noise contract fixes.
    # What the fp16-split MFMA buys: the same schedule with this net on exact-fp32 MFMA
    # (dpi_net_set_precision, = DPI_GEMM=f32), untimed by the contract's clock, after the timed region
    exact_fp32_ms = None
    if not args.no_fp32_pass and os.environ.get("DPI_GEMM", "") != "f32":
        gen.net.set_precision(L.DPI_GEMM_F32)
        for _ in range(2):
            step()
        drain()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        n32 = max(4, min(args.steps, 10))
        tf = time.perf_counter()
        open_region()
        for _ in range(n32):
            step()
        drain()
        torch.cuda.synchronize()
        exact_fp32_ms = (time.perf_counter() - tf) / n32 * 1e3
        if dist:
            t = torch.tensor([exact_fp32_ms], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            exact_fp32_ms = float(t[0])
        gen.net.set_precision(-1)
    floor_ms = None
    if rank == 0 and not wl.get("pis") and not wl.get("hess") and "m_total" not in wl:
        gen0 = dpi.OnlineDataGenerator(eq, dpi.ZeroSolution(1), 80, 1, device=dev, t_always_uniform=True,
                                       n_estimate_terminal=M_PER_GPU, n_estimate_integral=M_PER_GPU,
                                       n_euler_steps=K_STEPS, seed=1, hessian_approximation=hess)
        tx0, pb0 = gen0.sample_t_and_x(N_POINTS)
        ws0 = gen0.point_baseline(tx0)
        fl = []
        for it in range(8):
            slot = it % L.DPI_LAUNCH_TIMERS
            L.check(tlib.dpi_launch_timer_arm(slot), "dpi_launch_timer_arm")
            gen0.label_moments(tx0, pb0, M_PER_GPU, 0, M_PER_GPU, L.DPI_BOTH, ws0)
            fl.append(slot)
        torch.cuda.synchronize()
        floor_ms = sum(timer_ms(slot) for slot in fl[2:]) / len(fl[2:])
    path_labels_per_step = N_POINTS * M  # all ranks together
    value = path_labels_per_step * args.steps / dt
    if rank == 0:
        per_launch_units = N_POINTS * M_PER_GPU
        achieved = FLOP_PER_PATH_LABEL * per_launch_units / (k_ms * 1e-3) / 1e12
        if wl["peak"] == "split":
            peak = PEAK_SPLIT_TFLOPS
            peak_basis = ("fp32-equivalent peak of the fp16-split MFMA the network runs on: 2.5 PFLOP/s dense f16 "
                          "(v_mfma_f32_16x16x32_f16) / 3 f16 products per fp32 product")
        else:
            peak = PEAK_FP32_TFLOPS
            peak_basis = "fp32 MFMA (v_mfma_f32_16x16x4_f32) = fp32 vector peak"
        mfma = {"achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                "peak_basis": peak_basis, "flop_per_path_label": FLOP_PER_PATH_LABEL}
        # the fused kernels are VALU-issue bound (Philox4x32-10 + Box-Muller of the 2 K nx normals per
        # path-label): their roofline is the VALU issue of the 1024 SIMDs at the 2.4 GHz
        # peak clock.  Busy cycles per launch come from the PMC pass of this command
        # (profiles/valu_<workload>.json; the kernel's instruction stream is fixed, so they are a constant
        # of the launch); the launch time is measured live.
        valu = None
        # per-launch PMC figures are measured per workload and rank count (a configs[3] rank's launch
        # at N GPUs is 512 points x 4096/N paths): profiles/<kind>_<workload>[_n<N>].json
        prof_tag = args.workload + (f"_n{world}" if "m_total" in wl and world > 1 else "")
        vf = ROOT / "profiles" / f"valu_{prof_tag}.json"
        scale, busy_note = 1.0, ""
        if not vf.exists() and prof_tag != args.workload:
            # no PMC pass at this rank count: the N = 1 launch's busy cycles scaled by the path
            # count (a rank's launch is the same kernel over M_PER_GPU / M of the paths, whole
            # 64-path workgroups, so its VALU issue is proportional)
            vf = ROOT / "profiles" / f"valu_{args.workload}.json"
            scale = M_PER_GPU / M
            busy_note = f", scaled by this rank's share of the paths ({M_PER_GPU}/{M})"
        if vf.exists() and not wl.get("pis"):
            kern = json.loads(vf.read_text())["kernels"]
            # k_paths<KIND, H, L, ZERO, SPLIT, HESS, TD, ACT>: the network launch, not the u = 0 twin
            # (k_paths_fb<KIND, H, L, ZERO, SPLIT, ACT>: the one-launch sample_with_gradients, base blocks included)
            net_k = [v for k, v in kern.items()
                     if re.search(r"k_paths(_fb)?<", k) and k.split("<", 1)[1].rstrip(">").split(", ")[3] != "true"]
            top = max(net_k, key=lambda v: v["dispatches"])
            busy = top["valu_busy_cycles_per_simd"] * scale
            # the GBM prepare schedule: the next batch's noise sums (k_noise_shared, prepare stream) issue
            # on the same SIMDs during the network launch — their VALU issue per call counts too
            noise_k = [v for k, v in kern.items() if "k_noise_shared<" in k]
            if noise_k:
                busy += sum(v["valu_busy_cycles_per_simd"] * v["dispatches"] for v in noise_k) / top["dispatches"] * scale
                busy_note += ", plus the prepare stream's k_noise_shared issue per call (it runs inside the launch)"
            valu = {"achieved": busy * N_SIMD / (k_ms * 1e-3) / 1e12, "peak": N_SIMD * PEAK_CLOCK_GHZ * 1e9 / 1e12,
                    "unit": "T VALU-busy SIMD-cycles/s", "valu_busy_cycles_per_simd": busy,
                    "busy_source": f"profile_derived: {vf.relative_to(ROOT)} (SQ_ACTIVE_INST_VALU x 4 / "
                                   f"1024 SIMDs per launch){busy_note}"}
            valu["frac"] = valu["achieved"] / valu["peak"]
        traffic = None
        tf = ROOT / "profiles" / f"traffic_{prof_tag}.json"
        if tf.exists():
            traffic = json.loads(tf.read_text()).get("hbm_bytes_per_launch")
        ms_step = dt / args.steps * 1e3
        hbm = None
        if traffic is not None:
            # HBM bytes of one label call (PMC) against the 8 TB/s peak, over the live step time and over
            # the live launch time of the measured launches
            hbm = {"bytes_per_call": traffic, "GB_per_s": traffic / (ms_step * 1e-3) / 1e9,
                   "GB_per_s_kernel": traffic / (k_ms * 1e-3) / 1e9, "peak_GB_per_s": PEAK_HBM_GBS}
            hbm["frac_of_8TBs"] = hbm["GB_per_s"] / PEAK_HBM_GBS
            hbm["frac_of_8TBs_kernel"] = hbm["GB_per_s_kernel"] / PEAK_HBM_GBS
        out = {
            "metric": "SDE-path labels/sec (100-d, 50 Euler steps) per GPU; rel-L2 vs ref",
            "value": value,
            "unit": "path-labels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": wl.get("scaling", "weak"),
            "vs_baseline": None,
            "dtype": "f32",
            "workload_key": args.workload,
            "data": "synthetic (Philox-sampled collocation points; random-init ELU MLP, torch.manual_seed(0))",
            "config": {"workload": wl["desc"], "baseline_config": wl["cfg"],
                       "points": N_POINTS, "mc_paths_per_gpu": M_PER_GPU, "euler_steps": K_STEPS, "nx": wl.get("nx", NX),
                       "parallelism": f"mc-shard{world}", "per_gpu_value": value / world,
                       "arithmetic": ("fp32 noise / Euler-Maruyama / label moments; network "
                                      + ("on exact-fp32 MFMA" if os.environ.get("DPI_GEMM", "") == "f32" else
                                         "GEMMs on fp16x3-split MFMA (x = hi + lo, hi*hi + hi*lo + lo*hi into one "
                                         "fp32 accumulator, DESIGN.md §2.2)")),
                       "process_group": None if dist is None else backend + (" (ranks share cuda:0)" if share else ""),
                       "schedule": ("two-phase, next batch prepared on a side stream" if args.prepare and pipelined
                                    else "next batch's points, baseline and noise sums prepared on a side stream"
                                    if args.prepare and wl.get("hess")
                                    else "two-phase (all-gather overlapped)" if pipelined else "one labels() call"),
                       "prewarm_steps": prewarm,
                       "range_check": args.range_check != "off",
                       "range_check_mode": {"step": "one RangeGroup per step, verified one step behind (the dataset "
                                                    "surface's per-buffer check)",
                                            "region": "one RangeGroup over the timed steps (picard train's "
                                                      "LabelBuffer.fill)",
                                            "off": "unguarded"}[args.range_check],
                       "value_is": ("whole-job total over all N GPUs (the bench contract); the per-GPU figure the "
                                    "metric names is per_gpu_value"),
                       "rel_l2_vs_ref": parity},
            "roofline": {"bound": "valu" if valu else "mfma", **({k: valu[k] for k in ("achieved", "peak", "unit", "frac")}
                                                                  if valu else
                                                                  {k: mfma[k] for k in ("achieved", "peak", "unit", "frac")}),
                         "traffic": traffic,
                         "traffic_source": (f"profile_derived: profiles/traffic_{prof_tag}.json (rocprofv3 PMC "
                                            "FETCH_SIZE / WRITE_SIZE passes of this bench command, HBM bytes per "
                                            "label call)") if traffic is not None else None,
                         "hbm": hbm,
                         "kernel": wl["kernel"], "kernel_ms": k_ms,
                         "valu": valu, "mfma": mfma},
        }
        if "survey_flop" in wl:
            out["roofline"]["mfma"]["survey_flop_per_path_label"] = wl["survey_flop"]
        out["roofline"]["exact_fp32_ms"] = exact_fp32_ms
        if exact_fp32_ms is not None:
            out["roofline"]["exact_fp32"] = {
                "what": "ms/step of the same schedule with the network on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, "
                        "dpi_net_set_precision = DPI_GEMM=f32), untimed passes after the timed region",
                "ms_per_step": exact_fp32_ms, "split_speedup": exact_fp32_ms / ms_step}
        if floor_ms is not None:
            out["roofline"]["noise_floor"] = {
                "what": "same launch with u = 0 (ZeroSolution): Philox4x32-10 + Box-Muller + K-step EM only, the "
                        "VALU-issue floor of the noise contract (2 x K x nx normals per path-label)",
                "kernel_ms": floor_ms, "frac": floor_ms / k_ms}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(wl, args.cpu_sample_paths if wl["eq"] == "Cha" else 64)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
