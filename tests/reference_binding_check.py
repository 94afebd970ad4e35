"""Drives the reference's REAL data module — picard/data.py's PicardDataModule with
integration/picard-hip-backend.patch applied to a scratch copy of /root/reference/picard — through
the binding (`DATA.BACKEND: hip`), on the CPU of the build container.  Run by
tests/test_reference_binding.py in a subprocess (it installs module stand-ins and a fake CUDA
memory API, which must not leak into the test process); it prints one JSON line per scenario.

What is real: every line of PicardDataModule (get_data_generator's tuple return, get_dataset_details,
the NEW_SAMPLING probe GPUMemoryTracker.estimate_largest_data_points and its OOM handling,
estimate_n_buffer_per_worker, the CacheToMemoryWrapper re-batching, wrap_dataset's isinstance
assertions, initialize_dataset's isinstance chain, train_dataloader), the reference's equation
objects and networks, and this package's binding, generator class, datasets and caches.
What stands in: the label call (no GPU here) — `RecordingGenerator` returns index-coded rows and
records every call — and CUDA's memory-statistics API, modelled from the workspace the fused kernel
really allocates per point (dpi_workspace_bytes: 64-path blocks x 256-float slab rows).  Label
values are checked on the GPU by tests/test_gpu_dataset.py against the label call itself.
"""
import importlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
REF = Path(os.environ.get("DPI_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests" / "golden"))

HBM = 288 * 2 ** 30


class FakeCudaMemory:
    """torch.cuda's memory statistics as GPUMemoryTracker reads them (picard/memory.py:19-86)."""

    def __init__(self):
        self.current = 0
        self.peak = 0

    def use(self, nbytes):  # a transient allocation of one label call (workspace + outputs)
        self.peak = max(self.peak, self.current + nbytes)

    def install(self):
        c = torch.cuda
        c.is_available = lambda: True
        c.reset_peak_memory_stats = lambda *a, **k: setattr(self, "peak", self.current)
        c.max_memory_allocated = lambda *a, **k: self.peak
        c.memory_allocated = lambda *a, **k: self.current
        c.memory_reserved = lambda *a, **k: self.current
        c.mem_get_info = lambda *a, **k: (HBM - self.current, HBM)
        c.empty_cache = lambda *a, **k: None


FAKE = FakeCudaMemory()


def patched_reference(tmp):
    shutil.copytree(REF / "picard", tmp / "picard")
    subprocess.run(["patch", "-p1", "-s", "-i", str(REPO / "integration" / "picard-hip-backend.patch")], cwd=tmp,
                   check=True)
    from ref_stubs import install_stubs
    FAKE.install()  # before picard.memory binds reset_peak_memory_stats / max_memory_allocated
    install_stubs(tmp / "picard")
    return {m: importlib.import_module(f"picard.{m}") for m in ("config", "equations", "data", "solution")}


def make_recording_generator(OnlineDataGenerator):
    class RecordingGenerator(OnlineDataGenerator):
        """OnlineDataGenerator with the label call replaced by index-coded rows (no GPU): row r of
        the batch drawn at point counter pb is tx = (pb + r, ...), y = 2 tx + 1 (and a Hessian block)."""

        def __init__(self, equation, solution, N, i, *, device, n_euler_steps, seed, max_points_per_call,
                     label_dtype, **kw):
            self.equation, self.solution, self.N, self.i = equation, solution, N, i
            self._device = torch.device(device)
            self.K, self.seed, self.kw = n_euler_steps, seed, kw
            self.max_points_per_call, self.label_dtype = max_points_per_call, label_dtype
            self.n_estimate_integral = int(kw.get("n_estimate_integral", 1))
            self.point_base = 0
            self.calls = []
            self._range_check = False  # no label kernels here, so no range guard (data.RangeGroup)

        def _rows(self, n, width):
            M = self.n_estimate_integral
            FAKE.use(n * ((M // 64) * 256 * 4 + 3 * width * 4))  # dpi_workspace_bytes + tx, y, moments
            pb = self.point_base
            self.point_base += n
            self.calls.append([pb, n])
            idx = torch.arange(pb, pb + n, dtype=torch.float64)
            tx = torch.cat([idx[:, None], idx[:, None] + torch.arange(self.equation.nx)], 1)  # exact in fp32
            y = torch.cat([2 * tx + 1, torch.zeros(n, width - tx.shape[1], dtype=torch.float64) + idx[:, None]], 1)
            return self._out(tx.float(), y.float())

        def sample_with_gradients(self, n):
            return self._rows(n, 1 + self.equation.nx)

        def sample_with_gradients_and_hessians(self, n):
            return self._rows(n, 1 + self.equation.nx + self.equation.nx ** 2)

    return RecordingGenerator


def data_cfg(R, **over):
    """The reference's DATA defaults (patched picard/config.py) overlaid with a YAML's DATA keys."""
    d = R["config"]._C.DATA
    cfg = type(d)(dict(d))
    for k, v in over.items():
        cfg[k] = v
    return cfg


def run(R, tmp, name, eq, net, dcfg, batch_size, epochs, gradients=True, hessians=False):
    from deeppicarditeration_amd import picard_binding as B
    from deeppicarditeration_amd.data import OnlineDataGenerator
    Rec = make_recording_generator(OnlineDataGenerator)
    orig = B.hip_online_data_generator
    B.hip_online_data_generator = lambda kws, cfg, base=None: orig(kws, cfg, base=base, generator_cls=Rec)
    FAKE.current = FAKE.peak = 0
    try:
        if MODE == "reference":
            dm = R["data"].PicardDataModule(equation=eq, solution=net, N=80, i=1, data_cfg=dcfg,
                                             batch_size=batch_size, exp_dir=tmp / name, do_multi_epochs=epochs > 1,
                                             generate_gradients=gradients, generate_hessians=hessians)
            base = R["data"]._OnlineDataGenerator
        else:
            import picard_datamodule as S
            dcfg = S.reference_data_cfg(**{k: v for k, v in dcfg.items()})
            dm = S.PicardDataModuleStandIn(equation=eq, solution=net, N=80, i=1, data_cfg=dcfg, batch_size=batch_size,
                                           exp_dir=tmp / name, do_multi_epochs=epochs > 1,
                                           generate_gradients=gradients, generate_hessians=hessians)
            base = S._OnlineDataGenerator
        gen = dm.data_generator
        out = {"scenario": name, "is_reference_OnlineDataGenerator": isinstance(gen, base),
               "is_hip_OnlineDataGenerator": isinstance(gen, OnlineDataGenerator),
               "data_dir": None if dm.data_dir is None else str(dm.data_dir.relative_to(tmp)),
               "equation": type(gen.equation).__module__ + "." + type(gen.equation).__name__,
               "max_points_per_call": gen.max_points_per_call, "K": gen.K, "seed": gen.seed,
               "label_dtype": str(gen.label_dtype), "generator_kwargs": sorted(gen.kw)}
        loader = dm.train_dataloader()
        out["dataset_size_info_args"] = list(dm.dataset_size_info_args)
        out["dataset_type"] = type(loader.dataset).__module__ + "." + type(loader.dataset).__name__
        n_probe_calls = len(gen.calls)
        epochs_out = []
        for _ in range(epochs):
            epochs_out.append([[float(b[0][0, 0]), float(b[0][-1, 0]), list(b[0].shape), list(b[1].shape),
                                str(b[1].dtype),
                                bool(torch.equal(b[1][:, :b[0].shape[1]], 2 * b[0] + 1))] for b in loader])
        out["calls"] = gen.calls
        out["n_calls_before_iteration"] = n_probe_calls
        out["epochs"] = epochs_out
        out["active_data_size"] = dm.active_data_size
        if dm.data_dir is not None:
            out["files"] = sorted(p.name for p in (tmp / name).rglob("*.h5"))
        return out
    finally:
        B.hip_online_data_generator = orig


MODE = "reference"


def main():
    global MODE
    MODE = sys.argv[1] if len(sys.argv) > 1 else "reference"
    assert MODE in ("reference", "standin")
    sys.path.insert(0, str(REPO / "tests"))
    tmp = Path(tempfile.mkdtemp(prefix="refbind_"))
    try:
        R = patched_reference(tmp)
        # parameter files the reference loads from the CWD (equations.py:410-411, 530-532)
        os.chdir(tmp)
        for f in (REF / "scripts" / "fully_nonlinear" / "case_1").glob("*.pt"):
            shutil.copy(f, tmp / f.name)
        for f in (REF / "scripts" / "hjb").glob("*.pt"):
            shutil.copy(f, tmp / f.name)
        torch.save(torch.stack([2.0 * torch.eye(100, dtype=torch.float64)] * 5), tmp / "var_100d_ms=1.0_vs=2.0_5.pt")
        torch.set_default_dtype(torch.float64)  # apply_cfg with DATA.FLOAT: double (config.py:194-195)
        eqs, sols = R["equations"], R["solution"]
        cha = eqs.Cha(nx=100, alpha=1.0, k=5.0, T=1.0)
        mlp = sols.construct_mlp(101, 1, [128] * 4, ["ELU"] * 4, None)
        kw = R["config"]._C.DATA.kwargs.__class__
        # scripts/burgers/base_100d_T1.0_w0.0_0.yaml:16-33 (+ DATA.BACKEND hip)
        burgers = dict(FLOAT="double", DATA_SIZE=4096, NEW_SAMPLING=True, N_WORKERS=0, PREFETCH_FACTOR=None,
                       PRELOAD=True, BACKEND="hip",
                       kwargs=kw({"t_always_uniform": True, "n_estimate_terminal": 4096, "n_estimate_integral": 4096}))
        mem = R["config"]._C.DATA.MEMORY.__class__({"RESERVED": 0.0, "REDUCE_FACTOR": 1.0, "REUSE": 2})
        results = [run(R, tmp, "burgers_yaml", cha, mlp, data_cfg(R, MEMORY=mem, **burgers), 512, 16)]
        # the same with DATA.SAVE: the label file goes through the CacheToMemoryWrapper's saver
        results.append(run(R, tmp, "burgers_save", cha, sols.ZeroSolution(1),
                           data_cfg(R, MEMORY=mem, **{**burgers, "DATA_SIZE": 2048, "SAVE": True}), 512, 2))
        # NEW_SAMPLING false with N_BUFFER: one streaming epoch, no cache (initialize_dataset's first branch)
        results.append(run(R, tmp, "n_buffer_stream", cha, mlp,
                           data_cfg(R, MEMORY=mem, **{**burgers, "NEW_SAMPLING": False, "N_BUFFER": 2,
                                                      "PRELOAD": False}), 512, 1))
        # NEW_SAMPLING false, N_BUFFER unset, DATA_SIZE above the cap: the binding refuses up front
        try:
            run(R, tmp, "n_buffer_unset", cha, mlp,
                data_cfg(R, MEMORY=mem, **{**burgers, "NEW_SAMPLING": False, "DATA_SIZE": 32768, "PRELOAD": False}),
                512, 1)
            results.append({"scenario": "n_buffer_unset", "error": None})
        except ValueError as e:
            results.append({"scenario": "n_buffer_unset", "error": str(e)[:120]})
        # the reference's default DATA.N_WORKERS 1 (picard/config.py:75): the loader runs without worker
        # processes under DATA.BACKEND hip and yields N_WORKERS 0's batches (compare burgers_yaml)
        import warnings
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            r = run(R, tmp, "n_workers_default", cha, mlp, data_cfg(R, MEMORY=mem, **{**burgers, "N_WORKERS": 1}),
                    512, 16)
        r["warnings"] = [str(w.message)[:160] for w in caught if "N_WORKERS" in str(w.message)]
        results.append(r)
        # GBM case_1 with Hessian supervision (scripts/fully_nonlinear/case_1/base_100d_T1.0_w0.0_nov_0.yaml)
        gbm = eqs.GBMEquationComplexExact(nx=100, alpha=1.0, T=1.0)
        gnet = sols.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
        hess = R["config"]._C.DATA.HESSIAN_APPROXIMATION
        results.append(run(R, tmp, "gbm_hessians", gbm, gnet,
                           data_cfg(R, MEMORY=mem, **{**burgers, "DATA_SIZE": 1024, "HESSIAN_APPROXIMATION": hess,
                                                      "kwargs": kw({"t_always_uniform": True, "n_estimate_terminal": 1024,
                                                                    "n_estimate_integral": 1024})}),
                           256, 2, hessians=True))
        # equation conversion: the reference objects' parameters reach the device plugin unchanged
        from deeppicarditeration_amd.equations import from_reference
        ou = eqs.OUProcessEquation(nx=100, T=1.0, alpha=1.0, theta=1.0, mu=0.0, num_components=5, mean_scale=1.0,
                                   var_scale=2.0, alpha_scale=4.0)
        c_cha, c_gbm, c_ou = from_reference(cha), from_reference(gbm), from_reference(ou)
        f = lambda a: float(torch.as_tensor(a))  # noqa: E731
        results.append({"scenario": "equations",
                        "cha": [c_cha.nx, f(c_cha.alpha), f(c_cha.k), f(cha.k), c_cha.T],
                        "gbm_w_equal": bool(torch.equal(c_gbm.w, gbm.w.double())),
                        "gbm_v_equal": bool(torch.equal(c_gbm.v, gbm.v.double())),
                        "ou_mean_equal": bool(torch.equal(c_ou.mean, ou.mean.double())),
                        "ou_pi_equal": bool(torch.equal(c_ou.pi, ou.pi.double())),
                        "ou_var_equal": bool(torch.equal(c_ou.var, torch.diagonal(ou.var.double(), dim1=-2, dim2=-1))),
                        "ou_scalars": [c_ou.theta, c_ou.mu, f(c_ou.alpha), c_ou.alpha_scale, c_ou.num_components]})
        for r in results:
            print("@@RESULT " + json.dumps(r), flush=True)
    finally:
        os.chdir("/")
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
