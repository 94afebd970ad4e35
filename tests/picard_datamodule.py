"""A restatement of the reference's `PicardDataModule` data path (picard/data.py:1411-1780) with
integration/picard-hip-backend.patch applied, and of the memory probe it runs
(`GPUMemoryTracker`, picard/memory.py:19-208), so the GPU box — where the reference does not
exist — can drive the drop-in exactly as the reference's data module drives it.  Method by method
it follows the reference's control flow, including every `isinstance` check (against the names
the patch's import swap binds: this package's dataset classes), the `_OnlineDataGenerator`
assertion of `wrap_dataset`, both branches of `get_dataset_size_info_args` (NEW_SAMPLING probe /
estimate_n_buffer_per_worker), the CacheToMemoryWrapper re-batching and `DATA.SAVE`.  Lightning
(the module's base class) and DataLoader worker processes are left out: every shipped YAML sets
N_WORKERS 0.

Pinned to the real module: tests/test_reference_binding.py runs this restatement and the
reference's own PicardDataModule (patched copy, in the build container) on the same scenarios and
requires identical generator calls, dataset sizes, wrappers and batches.  Test infrastructure only.
"""
import dataclasses
import gc
from collections import namedtuple
from math import ceil

import numpy as np
import psutil
import torch
from torch.utils.data import DataLoader, TensorDataset

# the patch's import swap (picard/data.py:31-37)
from deeppicarditeration_amd.dataset import CacheToFileWrapper, CacheToMemoryWrapper, IterableDatasetWithInternalBatch
from deeppicarditeration_amd.h5 import H5Saver


class DataGenerator:
    """picard/data.py:53-85 (only what the module reads)."""
    do_internal_batching = True


class _OnlineDataGenerator(DataGenerator):
    """Stand-in for the reference class the patched get_data_generator passes as `base`; its
    constructor never runs (the binding's class puts the HIP generator first in the MRO)."""


class AttrDict(dict):
    """yacs CfgNode as the module reads it (attribute access)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def float_np(name):
    return np.float64 if str(name).lower() in ("double", "float64", "f64", "64") else np.float32


def float_bytes(name):
    return 8 if float_np(name) is np.float64 else 4


def divisors(n):
    return [d for d in range(1, int(n) + 1) if n % d == 0]


# ---------------------------------------------------------------------------- picard/memory.py
@dataclasses.dataclass
class GPUMemoryReport:
    peak_allocated: int = 0
    enabled: bool = dataclasses.field(default_factory=torch.cuda.is_available)

    def start(self):
        if self.enabled:
            torch.cuda.reset_peak_memory_stats()
            self.peak_allocated = torch.cuda.max_memory_allocated()

    def end(self):
        if self.enabled:
            return (torch.cuda.max_memory_allocated() - self.peak_allocated) / 1024 / 1024


class GPUMemoryTracker:
    EstimationResult = namedtuple("EstimationResult", ["peak_memory_usage", "n_buffer", "batch_size",
                                                       "n_data_per_sample"])
    calls = []  # (what, args, fitted) of every probe trial, for the tests

    @staticmethod
    def get_memory_available():
        free = torch.cuda.mem_get_info()[0] / 1024 / 1024
        return free + (torch.cuda.memory_reserved() - torch.cuda.memory_allocated()) / 1024 / 1024

    @staticmethod
    def get_memory_allocated_by_torch():
        return torch.cuda.memory_allocated() / 1024 / 1024

    @staticmethod
    def try_dataset(dataset_fn, *args):
        try:
            for _ in dataset_fn(*args):
                pass
            ok = True
        except torch.cuda.OutOfMemoryError:
            ok = False
        GPUMemoryTracker.calls.append(("try", args, ok))
        gc.collect()
        torch.cuda.empty_cache()
        return ok

    @classmethod
    def estimate_largest_data_points(cls, dataset_fn, reserved_memory=None, n_data_per_sample_init=1024):
        """memory.py:116-171."""
        rep = GPUMemoryReport()
        reserved_memory = reserved_memory or 0.0
        n = n_data_per_sample_init
        while True:  # phase 1: a size that fits
            rep.start()
            if cls.try_dataset(dataset_fn, n * 2, 1, n):
                used = rep.end()
                break
            n //= 2
            if n == 0:
                raise RuntimeError("Cannot sample each a single data point!")
        step = 0.1
        n_ok, used_ok = n, used
        available = cls.get_memory_available() - reserved_memory
        n = round(n * available / used)
        failed_once = False
        while True:  # phase 2: grow to the memory, back off 10 % per failure
            rep.start()
            ok = cls.try_dataset(dataset_fn, n * 2, 1, n)
            used = rep.end()
            ok = ok and used < available
            if ok:
                used_ok, n_ok = used, n
                if failed_once:
                    return cls.EstimationResult(used_ok, 0, 0, n_ok)
                n = max(round(n * available / used), round(n * (1 + step)))
            else:
                failed_once = True
                n = round(n * (1 - step))
                if n <= n_ok:
                    return cls.EstimationResult(used, 0, 0, n)

    @classmethod
    def estimate_memory_usage(cls, dataset_fn, batch_size, initial_n_buffer_to_try=16.0):
        """memory.py:174-208."""
        rep = GPUMemoryReport()
        n_buffer = initial_n_buffer_to_try
        n_batches = round(n_buffer * 2)
        while True:
            rep.start()
            if cls.try_dataset(dataset_fn, n_batches * batch_size, n_buffer, batch_size):
                return cls.EstimationResult(rep.end(), n_buffer, batch_size, round(n_buffer * batch_size))
            n_batches = max(round(n_batches / 2), 1)
            n_buffer = n_buffer / 2


# ---------------------------------------------------------------------------- picard/data.py
class PicardDataModuleStandIn:
    def __init__(self, equation, solution, N, i, data_cfg, batch_size, exp_dir=None, generate_gradients=False,
                 generate_hessians=False, do_multi_epochs=False, dataset_size_info_args=None, device="cuda"):
        """data.py:1412-1463."""
        self.batch_size = batch_size
        self.equation = equation
        self.data_cfg = data_cfg
        self.generate_gradients = generate_gradients
        self.generate_hessians = generate_hessians
        self._device = torch.device(device)
        self.do_multi_epochs = do_multi_epochs
        self.data_dim_input, self.data_name_input = 1 + equation.nx, "tx"
        self.data_dim, self.data_name = 1, "u"
        self.data_generator, self.data_dir = self.get_data_generator(exp_dir, N, i, solution)
        self.active_data_size = self.data_cfg.DATA_SIZE
        self.dataset_size_info_args = dataset_size_info_args

    def get_data_generator(self, exp_dir, N, i, solution):
        """data.py:1465-1496 as patched: the HIP branch of DATA.BACKEND."""
        if self.data_cfg.SAVE or self.do_multi_epochs or self.data_cfg.PRELOAD:
            assert exp_dir is not None
            data_dir = exp_dir / f"data_iter_{i}"
            data_dir.mkdir(parents=True, exist_ok=True)
        else:
            data_dir = None
        kws = dict(equation=self.equation, solution=solution, N=N, i=i, device=self._device, **self.data_cfg.kwargs)
        if self.data_cfg.HESSIAN_APPROXIMATION is not None:
            kws["hessian_approximation"] = self.data_cfg.HESSIAN_APPROXIMATION
        if self.data_cfg.SAMPLE_BOUND is not None:
            kws["sample_bound"] = self.data_cfg.SAMPLE_BOUND
        kws["estimate_terminal"] = self.data_cfg.ESTIMATE_TERMINAL
        kws["estimate_integral"] = self.data_cfg.ESTIMATE_INTEGRAL
        kws["estimate_delta_t"] = self.data_cfg.ESTIMATE_DELTA_T
        assert self.data_cfg.BACKEND == "hip"
        from deeppicarditeration_amd import picard_binding
        return picard_binding.hip_online_data_generator(kws, self.data_cfg, base=_OnlineDataGenerator), data_dir

    def initialize_dataset(self, dataset, worker_id, num_workers):
        """data.py:1510-1540."""
        n = self.active_data_size // num_workers
        h5_config = tuple()
        if self.data_cfg.SAVE:
            h5_config = (self.data_dir / f"split_{worker_id:02d}.h5", n, [self.data_dim_input, self.data_dim],
                         [self.data_name_input, self.data_name], float_np(self.data_cfg.FLOAT))
        if isinstance(dataset, IterableDatasetWithInternalBatch):
            dataset.set_size(n)
            if self.data_cfg.SAVE:
                dataset.attach_saver(H5Saver(*h5_config))
        elif isinstance(dataset, TensorDataset):
            raise NotImplementedError("TensorDataset is not supported for now!")
        elif isinstance(dataset, CacheToFileWrapper):
            dataset.init(*h5_config, preload=self.data_cfg.PRELOAD)
        elif isinstance(dataset, CacheToMemoryWrapper):
            if self.data_cfg.SAVE:
                dataset.enable_save_to_file(h5_config)
            dataset.init(n, [1 + self.equation.nx, self.data_dim], preload=self.data_cfg.PRELOAD)
        else:
            raise NotImplementedError(f"Unknown dataset type {type(dataset)}, multi-processing is not supported")

    def estimate_n_buffer_per_worker(self, dataset_fn):
        """data.py:1551-1618."""
        mem = self.data_cfg.MEMORY
        if self.data_cfg.N_BUFFER is not None and abs(self.data_cfg.N_BUFFER) > 1e-5:
            return self.data_cfg.N_BUFFER
        n_worker = max(self.data_cfg.N_WORKERS, 1)
        total = self.active_data_size // self.batch_size // n_worker
        assert total * self.batch_size * n_worker == self.active_data_size
        if self.data_cfg.N_BUFFER == 0:
            return total
        est = GPUMemoryTracker.estimate_memory_usage(dataset_fn, batch_size=self.batch_size)
        mb, n_buffer = est.peak_memory_usage, est.n_buffer
        avail = GPUMemoryTracker.get_memory_available() - GPUMemoryTracker.get_memory_allocated_by_torch() * (
            n_worker - 1) - (mem.RESERVED or 0.0)
        maximal = min(avail / n_worker / (mb / n_buffer) / mem.REDUCE_FACTOR, total)
        if maximal < 1:
            n_buffer_per_worker = None
            for calls in divisors(round(self.batch_size)):
                if calls >= 1 / maximal:
                    n_buffer_per_worker = 1 / calls
                    n_iter = total / n_buffer_per_worker
                    if abs(round(n_iter) - n_iter) < 1e-5:
                        break
            assert n_buffer_per_worker is not None
        else:
            least = ceil(total / maximal)
            n_buffer_per_worker = 1
            for d in divisors(round(total)):
                if d >= least:
                    n_buffer_per_worker = total // d
                    break
        return n_buffer_per_worker

    def get_dataset_details(self):
        """data.py:1620-1661 (every entry is read, as there)."""
        f = [k for k, on in (("exact", self.data_cfg.EXACT), ("gradient", self.generate_gradients),
                             ("hessian", self.generate_hessians)) if on]
        g, nx = self.data_generator, self.equation.nx
        D = namedtuple("Details", ["dataset_fn", "data_dim", "data_name"])
        return {"exact+gradient": D(g.dataset_exact_with_gradients, 1 + nx, "u_ux"),
                "exact+gradient+hessian": D(g.dataset_exact_with_gradients_and_hessians, 1 + nx + nx ** 2, "u_ux_uh"),
                "exact": D(g.dataset_exact, 1, "u"),
                "gradient": D(g.dataset_with_gradients, 1 + nx, "u_ux"),
                "gradient+hessian": D(g.dataset_with_gradients_and_hessians, 1 + nx + nx ** 2, "u_ux_uh"),
                "": D(g.dataset, 1, "u")}["+".join(f)]

    def get_dataset_size_info_args(self, dataset_fn):
        """data.py:1663-1712."""
        if self.dataset_size_info_args is not None:
            self.active_data_size = self.dataset_size_info_args[0]
            return self.dataset_size_info_args
        if not self.data_cfg.NEW_SAMPLING:
            return (self.active_data_size, self.estimate_n_buffer_per_worker(dataset_fn), self.batch_size)
        assert self.data_cfg.N_WORKERS <= 1
        est = GPUMemoryTracker.estimate_largest_data_points(dataset_fn, self.data_cfg.MEMORY.RESERVED,
                                                            n_data_per_sample_init=min(1024, self.data_cfg.DATA_SIZE))
        per = round(est.n_data_per_sample / self.data_cfg.MEMORY.REDUCE_FACTOR)
        requested = self.data_cfg.DATA_SIZE
        times = ceil(requested / per)
        per_keep = ceil(requested / times)
        self.active_data_size = times * per_keep
        return (self.active_data_size, 1, per_keep)

    def get_dataset_and_set_data_info(self):
        """data.py:1714-1733."""
        dataset_fn, self.data_dim, self.data_name = self.get_dataset_details()
        self.dataset_size_info_args = self.get_dataset_size_info_args(dataset_fn)
        dataset = dataset_fn(*self.dataset_size_info_args)
        if self.dataset_size_info_args[-1] != self.batch_size:
            if not self.is_memory_enough():
                raise RuntimeError("Memory is not enough to sample the whole dataset")
            dataset = CacheToMemoryWrapper(dataset, batch_size=self.batch_size, drop_last=True,
                                           shuffle=self.data_cfg.SHUFFLE)
        return dataset

    def is_memory_enough(self):
        """data.py:1735-1744."""
        need = self.active_data_size * (self.data_dim_input + self.data_dim) * float_bytes(self.data_cfg.FLOAT)
        return psutil.virtual_memory().available - 2 ** 30 > need

    def wrap_dataset(self, dataset):
        """data.py:1746-1760."""
        if isinstance(dataset, CacheToMemoryWrapper):
            return dataset
        if self.do_multi_epochs or self.data_cfg.PRELOAD:
            assert isinstance(self.data_generator, _OnlineDataGenerator)
            assert isinstance(dataset, IterableDatasetWithInternalBatch)
            if self.is_memory_enough():
                return CacheToMemoryWrapper(dataset, shuffle=self.data_cfg.SHUFFLE)
            assert not self.data_cfg.SHUFFLE
            return CacheToFileWrapper(dataset)
        return dataset

    def train_dataloader(self):
        """data.py:1762-1780 as patched: DATA.BACKEND hip builds the loader without worker processes."""
        dataset = self.wrap_dataset(self.get_dataset_and_set_data_info())
        self.initialize_dataset(dataset, 0, 1)
        return DataLoader(dataset, batch_size=None if self.data_generator.do_internal_batching else self.batch_size,
                          num_workers=0)


def reference_data_cfg(**over):
    """The reference's DATA defaults (picard/config.py:69-102 + the patch's keys) with overrides."""
    cfg = AttrDict(SAVE=False, ONLINE=True, TRAIN_FILE="", N_WORKERS=1, DATA_SIZE=2048 * 5000, NEW_SAMPLING=False,
                   N_BUFFER=None, RESERVED_MEMORY=None,
                   MEMORY=AttrDict(RESERVED=None, REDUCE_FACTOR=1.0, REUSE=9999999), PREFETCH_FACTOR=None,
                   DEVICE=None, FLOAT="float", EXACT=False, SHUFFLE=None, PRELOAD=False, PRELOAD_N_WORKERS=None,
                   HESSIAN_APPROXIMATION=AttrDict(method=None, kwargs=AttrDict()), SAMPLE_BOUND=None,
                   ESTIMATE_TERMINAL="OU_ByGx", ESTIMATE_INTEGRAL="OU_Simple", ESTIMATE_DELTA_T=0.0,
                   kwargs=AttrDict(), BACKEND="torch", SEED=0, EULER_STEPS=50, POINTS_PER_CALL=16384)
    for k, v in over.items():
        cfg[k] = AttrDict(v) if isinstance(v, dict) and not isinstance(v, AttrDict) else v
    return cfg


# scripts/burgers/base_100d_T1.0_w0.0_0.yaml:16-33 (DATA) + TRAIN.BATCH_SIZE 512, N_EPOCHS 16
BURGERS_YAML_DATA = dict(FLOAT="double", DATA_SIZE=4096, NEW_SAMPLING=True, N_WORKERS=0, PREFETCH_FACTOR=None,
                         PRELOAD=True, BACKEND="hip", MEMORY=dict(RESERVED=0.0, REDUCE_FACTOR=1.0, REUSE=2),
                         kwargs=dict(t_always_uniform=True, n_estimate_terminal=4096, n_estimate_integral=4096))
