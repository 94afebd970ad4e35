"""The reference-side binding: what the reference's own `PicardDataModule` (picard/data.py:1411-1780)
calls to put the MI355X label path behind it.  INTEGRATION.md §1 shows the lines a maintainer
changes in the reference; this module is everything those lines call.

The data module keeps its code paths:
- `get_data_generator` (data.py:1465-1496) builds `kws` as it does and, under `DATA.BACKEND: hip`,
  passes them to `hip_online_data_generator(kws, self.data_cfg, base=_OnlineDataGenerator)`; it
  still returns `(data_generator, data_dir)`;
- the generator is an instance of the reference's `_OnlineDataGenerator` (the class is derived from
  the `base` the caller passes), so `wrap_dataset`'s assertion (data.py:1750) holds;
- its datasets are `deeppicarditeration_amd.dataset.IterableDatasetWithInternalBatch`, and with the
  import swap of data.py:31-37 the module's `isinstance` chains (data.py:1522-1540, 1747-1751) and
  its `CacheToMemoryWrapper` / `CacheToFileWrapper` / `H5Saver` are this package's (labels cached
  in HBM);
- `NEW_SAMPLING: true` (every shipped DPI YAML; data.py:1687-1699) runs the reference's memory
  probe `GPUMemoryTracker.estimate_largest_data_points` unchanged.  The fused kernel needs almost no
  memory per point, so left alone the probe would grow the calls until HBM is full (hundreds of
  seconds of labels per trial).  The generator refuses datasets whose calls exceed
  `DATA.POINTS_PER_CALL` (default 16,384) with torch.cuda.OutOfMemoryError — the exception the probe
  reads as "does not fit" (memory.py:95-102) — so the probe settles within 10 % of the cap.

The reference itself is never imported here; `base` is whatever class the caller passes.
"""
import warnings

import torch

from .data import OnlineDataGenerator
from .equations import from_reference

DEFAULT_POINTS_PER_CALL = 16384

_CLASSES = {}


def generator_class(base=None, impl=OnlineDataGenerator):
    """`impl` (OnlineDataGenerator), or a subclass of it and of `base` (the reference's
    `_OnlineDataGenerator`), cached per (base, impl).  This package's methods come first in the MRO,
    so every call the data module makes lands on the HIP path; the base contributes only its type."""
    if base is None or issubclass(impl, base):
        return impl
    cls = _CLASSES.get((base, impl))
    if cls is None:
        cls = type(impl.__name__, (impl, base), {"__module__": __name__, "__doc__": impl.__doc__})
        _CLASSES[(base, impl)] = cls
    return cls


def _cfg_get(cfg, key, default):
    if cfg is None:
        return default
    if hasattr(cfg, "get"):
        v = cfg.get(key, default)
    else:
        v = getattr(cfg, key, default)
    return default if v is None else v


class HipWorkersNote(UserWarning):
    """DATA.N_WORKERS > 0 under DATA.BACKEND hip: the loader runs without worker processes."""


def hip_online_data_generator(kws, data_cfg=None, base=None, generator_cls=None):
    """The HIP generator for the `kws` PicardDataModule.get_data_generator builds (data.py:1474-1488:
    equation, solution, N, i, device, **DATA.kwargs, hessian_approximation, sample_bound,
    estimate_terminal / estimate_integral / estimate_delta_t).  From `data_cfg` (the module's
    DATA node): EULER_STEPS (default 50), SEED (default 0), POINTS_PER_CALL (the per-call cap,
    default 16,384).  The reference equation object is converted by class name
    (`equations.from_reference`); the solution network is uploaded once, as the reference freezes
    it (data.py:409-412).  `generator_cls`: a subclass of OnlineDataGenerator to instantiate instead
    (tests)."""
    kw = dict(kws)
    equation = from_reference(kw.pop("equation"))
    solution, N, i = kw.pop("solution"), kw.pop("N"), kw.pop("i")
    device = kw.pop("device", "cuda")
    cap = int(_cfg_get(data_cfg, "POINTS_PER_CALL", DEFAULT_POINTS_PER_CALL))
    workers = [int(_cfg_get(data_cfg, k, 0) or 0) for k in ("N_WORKERS", "PRELOAD_N_WORKERS")]
    if max(workers) > 0:
        # the reference's default is DATA.N_WORKERS 1 (picard/config.py:75): its DataLoader would run the
        # dataset in worker processes (data.py:1768-1779).  The HIP labels come from one fused kernel per
        # call on this process's stream (device handles of this process), so the patched
        # train_dataloader builds the loader with no workers for DATA.BACKEND hip; the batches are the
        # ones N_WORKERS 0 draws (counter-based noise: worker processes would only move them)
        warnings.warn(f"DATA.BACKEND hip labels in the training process: DATA.N_WORKERS {workers[0]} "
                      f"(PRELOAD_N_WORKERS {workers[1]}) runs as N_WORKERS 0", HipWorkersNote, stacklevel=2)
    data_size = _cfg_get(data_cfg, "DATA_SIZE", None)
    n_buffer = _cfg_get(data_cfg, "N_BUFFER", None)
    if data_cfg is not None and not _cfg_get(data_cfg, "NEW_SAMPLING", False) and n_buffer in (None, 0) \
            and data_size is not None and int(data_size) > cap:
        # estimate_n_buffer_per_worker (data.py:1551-1618) extrapolates the buffer from the memory one
        # probe used; with almost no memory per point it picks the whole DATA_SIZE per call, which the
        # cap would then refuse outside the probe's try/except
        raise ValueError(f"DATA.NEW_SAMPLING false with DATA.N_BUFFER {n_buffer!r} would generate all "
                         f"{data_size} points in one call, above DATA.POINTS_PER_CALL = {cap}: set DATA.N_BUFFER "
                         f"(batches per call) or NEW_SAMPLING true")
    cls = generator_class(base, generator_cls or OnlineDataGenerator)
    return cls(equation, solution, N, i, device=device, n_euler_steps=int(_cfg_get(data_cfg, "EULER_STEPS", 50)),
               seed=int(_cfg_get(data_cfg, "SEED", 0)), max_points_per_call=cap,
               label_dtype=label_dtype(_cfg_get(data_cfg, "FLOAT", None)), **kw)


def label_dtype(float_name):
    """DATA.FLOAT (the names of picard/config.py:131-144) -> the dtype the data module's networks run
    in; None: torch's default dtype, which the reference's apply_cfg sets from DATA.FLOAT."""
    if float_name is None:
        return torch.get_default_dtype()
    if isinstance(float_name, torch.dtype) and float_name in (torch.float32, torch.float64):
        return float_name
    name = str(float_name).lower()
    if name in ("double", "float64", "f64", "64"):
        return torch.float64
    if name in ("float", "float32", "f32", "single", "32"):
        return torch.float32
    raise ValueError(f"DATA.FLOAT {float_name!r}: float or double")
