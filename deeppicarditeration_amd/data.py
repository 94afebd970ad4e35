"""DPI label generation on MI355X — the drop-in for the reference's
`OnlineDataGenerator` (picard/data.py:369-1223) behind the `batch_data_generator` boundary
(`IterableDatasetWithInternalBatch`, picard/dataset.py:27, :112).

Same constructor arguments and method names as the reference; every label is computed by
the HIP kernels of libdpi_hip.so through the C-ABI (include/dpi.h).  There is no eager /
CPU fallback: a missing library or an unsupported configuration raises.

Differences from the reference, by design:
- noise is counter-based Philox4x32-10 keyed by (seed, epoch = Picard iteration, point index,
  MC index, EM step) instead of torch's unseeded global RNG (the reference sets no seed), so
  labels are reproducible and independent of how paths are split over GPUs;
- each forward path is a K-step Euler–Maruyama rollout (`n_euler_steps`, default 50); for the
  zero-drift SDE of every shipped equation this equals the reference's one-jump sampler in
  distribution, and pathwise when the reference is fed xi_eff = sum_k xi_k / sqrt(K);
- tensors are fp32 on the GPU (the YAMLs say DATA.FLOAT: double; parity is measured against
  the fp64 reference, tests/test_gpu_parity.py).

`estimate_delta_t > 0` selects the reference's TD estimators (data.py:1209-1213) on the device
(every network kind).
"""
import warnings
from typing import Union

import torch

from . import _lib
from .dataset import IterableDatasetWithInternalBatch
from .equations import Equation, OUProcessEquation, SimpleDiffusionEquation, SimpleDiffusionEquationWithHessian
from .solution import DeviceNet

# paths one label call takes (include/dpi.h DPI_PATHS_PER_CALL_MAX); more run as several calls
PATHS_PER_CALL_MAX = _lib.DPI_PATHS_PER_CALL_MAX


def _ptr(t):
    return _lib.c_void_p(t.data_ptr())


def _stream(device):
    return _lib.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def new_workspace(nbytes, device):
    """A label-call workspace (uint8).  The caching allocator may hand out a freed workspace's
    address: the library's host-side records of that address (a baseline's fused-reduce tag, an
    unconsumed prepare) are dropped (dpi_workspace_forget), so they cannot vouch for the new one."""
    ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if ws.is_cuda:
        _lib.check(_lib.load().dpi_workspace_forget(_ptr(ws), ws.numel()), "dpi_workspace_forget")
    return ws


class SplitRangeWarning(RuntimeWarning):
    """A network's fp16-split evaluation left fp16's range: its labels are recomputed, and the
    generator's later calls made, with exact-fp32 MFMA (DPI_GEMM_F32) for that network."""


# include/dpi.h status ring: slot 0 serves the immediate (per-call) check, UNCHECKED_SLOT collects the
# flags of calls made with range_check off (never read), the others are handed to RangeGroups
IMMEDIATE_SLOT = 0
UNCHECKED_SLOT = _lib.DPI_STATUS_SLOTS - 1


def _check_handoff(flag):
    """DPI_STATUS_HANDOFF: a one-launch sample_with_gradients path block never saw its point's
    baseline (an internal failure, not a range problem): no fp32 repair, an error."""
    if flag & _lib.DPI_STATUS_HANDOFF:
        raise _lib.DPIError("fused baseline hand-off timed out in dpi_sample_with_gradients (DPI_FUSED_BASE=0 "
                            "runs the two-launch form)")


class RangeGroup:
    """The range guard of a group of label calls, checked once for the whole group instead of with
    a stream synchronisation per call (include/dpi.h dpi_net_status_slot / _peek).

    Every call run through the group is enqueued with the group's own slot of the net's
    host-visible status ring selected, so its reductions flag into that slot and nowhere else.
    `close()` records an event after the group's last call; `verify()` waits for that event — by
    then the caller has usually enqueued the next group, so the GPU does not idle — reads the slot
    from host memory and, if a label came out non-finite, switches the net to exact fp32 and
    recomputes every registered call of the group (same points, same counters) into the tensors
    it returned: the labels are final once verify() has returned, and a consumer that reads them
    only after that never sees an unguarded label (IterableDatasetWithInternalBatch yields a buffer
    only after its group verified; runner.LabelBuffer and bench.py verify before they use them).
    A flag in exact fp32 raises DPIError, as the per-call guard does.  Multi-rank callers pass
    `reduce_flag` (ShardedLabeler): the flag is MAX-reduced over the ranks, so every rank repairs
    the same calls.  The reference's call (picard/data.py:211-223) has no such check: it computes
    in fp64, where the fp16 split cannot overflow."""

    def __init__(self, gen, slot):
        self.gen = gen
        self.slot = slot
        self.calls = []  # (repair callable, returned output) in call order
        self.reduce_flag = None
        self.event = None
        self.open = True
        self.done = False

    def run(self, fn):
        """Enqueue fn() with this group's slot selected (no registration)."""
        gen = self.gen
        prev = gen._slot
        gen._select_slot(self.slot)
        try:
            return fn()
        finally:
            gen._select_slot(prev)

    def register(self, repair, out, reduce_flag=None):
        """`out` (a tensor or a tuple of tensors) is final after verify(); repair() recomputes it."""
        if self.done:
            raise RuntimeError("RangeGroup.register() after verify()")
        self.calls.append((repair, out))
        if reduce_flag is not None:
            self.reduce_flag = reduce_flag
        return out

    def enqueue(self, call, reduce_flag=None):
        return self.register(call, self.run(call), reduce_flag)

    def close(self):
        """End of the group's enqueueing: an event after its last call on the current stream."""
        if self.open:
            self.open = False
            if self.gen._scope is self:
                self.gen._scope = None
            self.event = torch.cuda.Event()
            self.event.record(torch.cuda.current_stream(self.gen.device))

    def verify(self):
        """Wait for the group's work, check its slot, repair its calls if flagged; returns the flag."""
        if self.done:
            return 0
        self.close()
        self.event.synchronize()
        st = _lib.c_int(0)
        _lib.check(self.gen.lib.dpi_net_status_peek(self.gen.net.handle, self.slot, _lib.ctypes.byref(st)),
                   "dpi_net_status_peek")
        flag = st.value
        if self.reduce_flag is not None:
            flag = self.reduce_flag(flag)
        self.done = True
        self.gen._release_slot(self.slot)
        _check_handoff(flag)
        if flag & _lib.DPI_STATUS_NONFINITE:
            self.gen._repair(self.calls, self.reduce_flag)
        self.calls = []
        return flag

    def discard(self):
        """Give the slot back without checking (the group's outputs are dropped unread)."""
        if not self.done:
            self.close()
            self.event.synchronize()
            self.done = True
            self.calls = []
            self.gen._release_slot(self.slot)

    def __del__(self):
        # a group dropped unverified gives its slot back once its kernels are done (an event after
        # its last call, checked lazily by the next deferred_range_check()): a later group taking the
        # slot earlier could see this group's flag and recompute its own labels in fp32 for nothing
        try:
            if not self.done:
                self.done = True
                self.close()
                self.gen._release_slot_after(self.slot, self.event)
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


class _NoGroup:
    """What deferred_range_check() returns with range_check off: runs calls unchecked."""
    calls = ()

    def run(self, fn):
        return fn()

    def register(self, repair, out, reduce_flag=None):
        return out

    def enqueue(self, call, reduce_flag=None):
        return call()

    def close(self):
        pass

    def verify(self):
        return 0

    def discard(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _copy_into(dst, src):
    if isinstance(dst, (tuple, list)):
        for d, s_ in zip(dst, src):
            _copy_into(d, s_)
    elif isinstance(dst, torch.Tensor) and dst is not src:
        dst.copy_(src)


def _hessian_approximation(cfg):
    """DATA.HESSIAN_APPROXIMATION ({method, kwargs: {v}}; config.py:99-101) -> (method, v)."""
    if cfg is None:
        return None, 0
    get = (lambda k, d=None: cfg.get(k, d)) if isinstance(cfg, dict) else (lambda k, d=None: getattr(cfg, k, d))
    method = get("method")
    if method is None:
        return None, 0
    kw = get("kwargs") or {}
    v = kw.get("v") if isinstance(kw, dict) else getattr(kw, "v", None)
    if v is None or not (1 <= int(v) <= 255):
        raise ValueError(f"SDGD needs 1 <= v <= 255 (got {v})")
    return method, int(v)


class OnlineDataGenerator:
    """picard/data.py:369-431 (constructor), :211-223 / :1208-1218 (label entry points)."""

    do_internal_batching = True

    def __init__(self, equation: Equation, solution: torch.nn.Module, N: int, i: int, *,
                 device: Union[str, torch.device] = "cuda", t_always_uniform=False, n_estimate_terminal=1,
                 n_estimate_integral=1, hessian_approximation=None, sample_bound=None, estimate_terminal="OU_ByGx",
                 estimate_integral="OU_Simple", estimate_delta_t=0.0, n_euler_steps: int = 50, seed: int = 0,
                 epoch: int = None, max_points_per_call: int = None, label_dtype: torch.dtype = torch.float32):
        if not (isinstance(equation, SimpleDiffusionEquation) or isinstance(equation, OUProcessEquation)):
            raise AssertionError("Currently only SimpleDiffusionEquation and OUProcessEquation are supported")  # :426-429
        if equation.nu != 1:
            raise AssertionError("Currently only nu=1 is supported")
        self.estimate_delta_t = float(estimate_delta_t or 0.0)
        if self.estimate_delta_t < 0:
            raise ValueError(f"estimate_delta_t must be >= 0 (got {estimate_delta_t})")
        method, sdgd_v = _hessian_approximation(hessian_approximation)
        if method is not None:  # data.py:115-123
            if method not in equation.supported_approximate_methods:
                raise AssertionError(f"Current equation does not support the method {method}")
            if method != "SDGD":
                raise NotImplementedError(f"hessian approximation {method!r}")
        self.equation = equation
        self.solution = solution
        self.N, self.i = N, i
        # t sampler (data.py:109-112): sample_t_always_uniform, or sample_t's product of N - i + 1 uniforms
        self.t_factors = 0 if t_always_uniform else int(N) - int(i) + 1
        if not 0 <= self.t_factors <= 4096:
            raise ValueError(f"sample_t needs 1 <= N - i + 1 <= 4096 (N={N}, i={i})")
        self.T = float(equation.T)
        self._device = torch.device(device)
        if self._device.type != "cuda":
            raise ValueError("the HIP label generator runs on a GPU device ('cuda' on ROCm)")
        self.n_estimate_terminal = int(n_estimate_terminal)
        self.n_estimate_integral = int(n_estimate_integral)
        for m in (self.n_estimate_terminal, self.n_estimate_integral):
            if m % _lib.DPI_PATH_BLOCK:
                raise ValueError(f"Monte-Carlo sample counts must be multiples of {_lib.DPI_PATH_BLOCK} (got {m})")
        self.sample_bound = float("inf") if sample_bound is None else float(sample_bound)
        self.estimate_terminal_type = estimate_terminal
        self.estimate_integral_type = estimate_integral
        # data.py:134-137
        self.eps = 0.01 if ("ByGx" in (estimate_terminal or "") or "Joint" in (estimate_integral or "")) else 0.0
        self.K = int(n_euler_steps)
        if self.K < 1:
            raise ValueError("n_euler_steps must be >= 1")
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.epoch = int(i if epoch is None else epoch) & 0xFFFFFF
        self.point_base = 0
        self.lib = _lib.load()
        for p in solution.parameters():  # data.py:409-412
            p.requires_grad = False
        solution.eval()
        self.net = DeviceNet.from_module(solution, 1 + equation.nx)
        self.problem = equation.dpi_problem()
        self.sdgd_v = sdgd_v
        self._configure_problem()
        self._ws = None
        # Range guard of the label calls (include/dpi.h dpi_net_status): after each call the net's
        # status word says whether a label came out non-finite from finite weights — the network
        # evaluation overflowed fp16 (split storage) or fp32.  Split: the call is recomputed in
        # exact fp32 and the net stays fp32 (SplitRangeWarning); fp32 already: DPIError.  Never a
        # silent inf / NaN label.  A direct call is checked at once (one stream synchronisation);
        # calls inside deferred_range_check() — the label buffers of the dataset surface, picard train
        # and bench.py — are checked once per group, one group behind (RangeGroup).  False skips it.
        self._range_check = True
        self._slot = IMMEDIATE_SLOT
        self._scope = None  # the RangeGroup that label calls are deferred into (deferred_range_check)
        self._free_slots = list(range(UNCHECKED_SLOT - 1, IMMEDIATE_SLOT, -1))
        self._pending_slots = []  # (slot, event) of groups dropped unverified, until their kernels are done
        self._fp32_fallback = False
        # Points per generator call of the dataset surface (None: unbounded).  The reference sizes
        # its calls by probing GPU memory (picard/memory.py:95-171): a dataset whose calls exceed
        # this cap raises torch.cuda.OutOfMemoryError, which those probes read as "does not fit",
        # so NEW_SAMPLING settles at the cap instead of at a size only HBM capacity bounds.
        self.max_points_per_call = None if max_points_per_call is None else int(max_points_per_call)
        # dtype of the (tx, labels) the sample_* surface returns: labels are computed in fp32; a
        # data module running DATA.FLOAT: double (picard/config.py:194-200 sets the default dtype, so
        # its networks are fp64) receives them cast exactly to fp64
        if label_dtype not in (torch.float32, torch.float64):
            raise ValueError(f"label_dtype must be float32 or float64 (got {label_dtype})")
        self.label_dtype = label_dtype

    @property
    def range_check(self):
        return self._range_check

    @range_check.setter
    def range_check(self, on):
        self._range_check = bool(on)
        if self._scope is None:
            self._select_slot(IMMEDIATE_SLOT if self._range_check else UNCHECKED_SLOT)

    def _select_slot(self, slot, clear=False):
        if slot != self._slot or clear:
            _lib.check(self.lib.dpi_net_status_slot(self.net.handle, slot, 1 if clear else 0), "dpi_net_status_slot")
            self._slot = slot

    def _release_slot(self, slot):
        self._free_slots.append(slot)

    def _release_slot_after(self, slot, event):
        """`slot` returns to the free list once `event` (the dropped group's last call) completed."""
        self._pending_slots.append((slot, event))

    def _reclaim_slots(self):
        """Pending slots whose groups' kernels are done go back to the free list (no wait), or, with
        no free slot left, the oldest pending one after its event."""
        keep = []
        for slot, ev in self._pending_slots:
            (self._free_slots.append(slot) if ev is None or ev.query() else keep.append((slot, ev)))
        self._pending_slots = keep
        if not self._free_slots and self._pending_slots:
            slot, ev = self._pending_slots.pop(0)
            ev.synchronize()
            self._free_slots.append(slot)

    def deferred_range_check(self):
        """A RangeGroup that this generator's guarded label calls are deferred into until it is
        closed (use as a context manager, or call close()); verify() it before reading its labels.
        Groups may be closed and still pending while the next one is open (one-ahead pipelines)."""
        if not self._range_check or torch.cuda.is_current_stream_capturing():
            return _NoGroup()
        if self._scope is not None:
            raise RuntimeError("deferred_range_check(): a group is already open on this generator")
        self._reclaim_slots()
        if not self._free_slots:
            raise RuntimeError(f"deferred_range_check(): all {UNCHECKED_SLOT - 1} status slots belong to groups that "
                               "were not verified")
        slot = self._free_slots.pop()
        _lib.check(self.lib.dpi_net_status_slot(self.net.handle, slot, 1), "dpi_net_status_slot")
        _lib.check(self.lib.dpi_net_status_slot(self.net.handle, self._slot, 0), "dpi_net_status_slot")
        g = RangeGroup(self, slot)
        self._scope = g
        return g

    def _repair(self, calls, reduce_flag=None):
        """A group's label came out non-finite: exact fp32 for this net, then every registered call
        again (same points and counters, each checked at once — a call that overflows fp32 too raises
        DPIError) into the outputs it returned.  A group may hold calls enqueued in split mode before
        an earlier group's repair switched the net, so fp32 here only means "from now on"."""
        if not self._fp32_fallback:
            warnings.warn("the fp16-split evaluation of this network left fp16's range (|activation| > 65504); its "
                          "labels are recomputed, and this generator's later calls run, with exact-fp32 MFMA",
                          SplitRangeWarning, stacklevel=3)
            self.use_fp32()
        for repair, out in calls:
            _copy_into(out, self._guarded(repair, reduce_flag, defer=False))

    def __getstate__(self):
        # DataLoader worker processes (DATA.N_WORKERS > 0, picard/data.py:1768-1779) would pickle the
        # generator: its problem / network handles are device state of this process
        raise TypeError("the HIP OnlineDataGenerator holds device handles of this process and cannot move to "
                        "DataLoader worker processes: set DATA.N_WORKERS 0")

    def _configure_problem(self):
        """The device problem handle belongs to the equation and may be shared by several
        generators: (re)apply this generator's estimator settings before each label call."""
        if self.equation.has_hessian_term:
            _lib.check(self.lib.dpi_problem_set_hessian_approximation(self.problem, self.sdgd_v),
                       "dpi_problem_set_hessian_approximation")
        # TD estimators (data.py:1209-1213); 0 = the plain estimators
        _lib.check(self.lib.dpi_problem_set_estimate_delta_t(self.problem, self.estimate_delta_t),
                   "dpi_problem_set_estimate_delta_t")

    @property
    def device(self):
        return self._device

    def to(self, device):
        """data.py:139-143, :433-436.  The labels are computed where the network weights were
        uploaded; moving the generator to another device is not supported."""
        d = torch.device(device)
        if d.type != self._device.type or (d.index is not None and self._device.index is not None
                                           and d.index != self._device.index):
            raise NotImplementedError(f"the generator's device handle lives on {self._device}")
        return self

    # ------------------------------------------------------------------ buffers
    def _workspace(self, n, M, hessians=False):
        need = self.lib.dpi_workspace_bytes(self.problem, self.net.handle, n, M)
        if hessians:
            need = max(need, self.lib.dpi_workspace_bytes_hessians(self.problem, self.net.handle, n, M))
        if self._ws is None or self._ws.numel() < need:
            self._ws = new_workspace(need, self._device)
        return self._ws

    def _take_points(self, n):
        base = self.point_base
        self.point_base = (self.point_base + n) & 0xFFFFFFFF
        return base

    # ------------------------------------------------------------------ reference entry points
    def sample_t_and_x(self, n_batch, point_base=None):
        """t_sampler + equation.sample_x (data.py:149-167, :211-217): tx (n, 1+nx)."""
        tx = torch.empty(n_batch, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
        pb = self._take_points(n_batch) if point_base is None else point_base
        _lib.check(self.lib.dpi_sample_points_t(self.problem, n_batch, self.seed, self.epoch, pb, self.eps,
                                                self.t_factors, _ptr(tx), _stream(self._device)), "dpi_sample_points_t")
        return tx, pb

    def _out(self, tx, y):
        if self.label_dtype == torch.float32:
            return tx, y
        return tx.to(self.label_dtype), y.to(self.label_dtype)

    def sample_with_gradients(self, n_batch):
        """data.py:211-223: (tx, clip(u_ux)) with u_ux (n, 1+nx).  One C-ABI call where it fits
        (dpi_sample_with_gradients: for first-order Cha / OU labels one launch, the per-point
        baseline beside the rollouts and the label reduce in the path launch); tx and labels are
        bitwise those of the separate calls."""
        MT, MI = self.n_estimate_terminal, self.n_estimate_integral
        if MT == MI and MT <= PATHS_PER_CALL_MAX:
            pb = self._take_points(n_batch)
            return self._guarded(lambda: self._out(*self.sample_generate(n_batch, pb)))
        tx, pb = self.sample_t_and_x(n_batch)
        return self._guarded(lambda: self._out(tx, self._generate_once(tx, pb, _lib.DPI_BOTH)))

    def sample_generate(self, n_batch, point_base, bound=None, on_moments_begin=None, on_moments_end=None):
        """Points at counters [point_base, point_base + n) and their clipped labels (no range guard):
        (tx, y) from dpi_sample_with_gradients — for first-order Cha / OU labels one launch (n
        baseline workgroups ahead of the path workgroups, the label reduce in each point's last path
        workgroup), otherwise the sampling inside the baseline launch, then the path launch;
        last_moments as _generate.  on_moments_*: called around the call (bench timing)."""
        n, F = n_batch, 1 + self.equation.nx
        M = self.n_estimate_integral
        ws = self._workspace(n, M)
        tx = torch.empty(n, F, dtype=torch.float32, device=self._device)
        y = torch.empty(n, F, dtype=torch.float32, device=self._device)
        mom = torch.empty(n, 2, F, dtype=torch.float32, device=self._device)
        b = self.sample_bound if bound is None else bound
        self._configure_problem()
        if on_moments_begin:
            on_moments_begin()
        _lib.check(self.lib.dpi_sample_with_gradients(self.problem, self.net.handle, n, M, self.K, self.seed,
                                                      self.epoch, point_base, self.eps, self.t_factors,
                                                      _lib.DPI_BOTH, b, _ptr(tx), _ptr(y), _ptr(mom), _ptr(ws),
                                                      ws.numel(), _stream(self._device)),
                   "dpi_sample_with_gradients")
        if on_moments_end:
            on_moments_end()
        self.last_moments = mom
        return tx, y

    def sample_points_baseline(self, n_batch, point_base, ws, out=None):
        """Points at counters [point_base, point_base + n) sampled inside the per-point baseline
        launch (dpi_sample_points_baseline) into ws (uint8, >= workspace_bytes): tx (n, 1+nx), bitwise
        sample_t_and_x's, and the baseline point_baseline would leave in ws.  out: the (n, 1+nx) fp32
        tensor to write tx into."""
        n, F = n_batch, 1 + self.equation.nx
        if ws.numel() < self.workspace_bytes(n, max(self.n_estimate_terminal, self.n_estimate_integral)):
            raise ValueError("workspace too small")
        tx = torch.empty(n, F, dtype=torch.float32, device=self._device) if out is None else out
        if tx.shape != (n, F) or tx.dtype != torch.float32 or not tx.is_contiguous() or tx.device.type != "cuda":
            raise ValueError("out must be a contiguous (n, 1+nx) fp32 GPU tensor")
        self._configure_problem()
        _lib.check(self.lib.dpi_sample_points_baseline(self.problem, self.net.handle, n, self.seed, self.epoch,
                                                       point_base, self.eps, self.t_factors, _ptr(tx), _ptr(ws),
                                                       ws.numel(), _stream(self._device)), "dpi_sample_points_baseline")
        return tx

    def sample_with_gradients_and_hessians(self, n_batch):
        """data.py:225-237: (tx, clip(u_ux_uxx)) with u_ux_uxx (n, 1 + nx + nx^2)."""
        tx, pb = self.sample_t_and_x(n_batch)
        return self._guarded(lambda: self._out(tx, self._generate_hess_once(tx, pb, self.sample_bound)))

    def generate_with_gradients_and_hessians(self, tx, point_base=None):
        """data.py:1220-1223: Malliavin-weight Hessian labels (no clip), (n, 1 + nx + nx^2)."""
        pb = self._take_points(tx.shape[0]) if point_base is None else point_base
        return self._generate_hess(self._as_points(tx), pb, float("inf"))

    def generate_with_gradients(self, tx, point_base=None):
        """data.py:1208-1218: terminal + integral estimators at given points (no clip)."""
        pb = self._take_points(tx.shape[0]) if point_base is None else point_base
        return self._generate(self._as_points(tx), pb, _lib.DPI_BOTH, bound=float("inf"))

    def estimate_terminal_with_gradients(self, tx, point_base=None):
        """data.py:899-926."""
        pb = self._take_points(tx.shape[0]) if point_base is None else point_base
        return self._generate(self._as_points(tx), pb, _lib.DPI_TERMINAL, bound=float("inf"))

    def estimate_integral_with_gradients(self, tx, point_base=None):
        """data.py:471-527."""
        pb = self._take_points(tx.shape[0]) if point_base is None else point_base
        return self._generate(self._as_points(tx), pb, _lib.DPI_INTEGRAL, bound=float("inf"))

    def generate(self, tx, point_base=None):
        """data.py:1203-1206: value-only labels, E g(X_T) + E int f(s, X_s, u) ds.  The reference's
        value-only integral calls `equation.f(s, X, u)`, which every equation whose nonlinearity
        reads the gradient or the Hessian defines as raising (equations.py:262-263, :369-370,
        :575-576); so does this one, at call time."""
        if self.equation.has_gradient_term or self.equation.has_hessian_term:
            self.equation.f(None, None, None)  # raises the reference's NotImplementedError
        raise NotImplementedError(f"{type(self.equation).__name__}: the device path has no value-only estimator")

    def sample(self, n_batch):
        """data.py:196-209: (tx, clip(u)) with u (n, 1)."""
        tx, pb = self.sample_t_and_x(n_batch)
        u = self.generate(tx, pb)
        return self._out(tx, torch.clamp(u, -self.sample_bound, self.sample_bound))

    # ------------------------------------------------------------------ exact labels (closed form)
    def _t_x(self, n_batch):
        tx, _ = self.sample_t_and_x(n_batch)
        return tx, tx[:, :1], tx[:, 1:]

    def sample_exact(self, n_batch):
        """data.py:239-250: (tx, u*(t, x))."""
        tx, t, x = self._t_x(n_batch)
        with torch.no_grad():
            return self._out(tx, self.equation.exact_solution(t, x).to(tx))

    def sample_exact_with_gradients(self, n_batch):
        """data.py:252-263: (tx, [u*, grad u*])."""
        tx, t, x = self._t_x(n_batch)
        with torch.no_grad():
            u, ux = self.equation.u_u_x(t, x)
        return self._out(tx, torch.cat([u.to(tx), ux.to(tx)], -1))

    def sample_exact_with_gradients_and_hessians(self, n_batch):
        """data.py:265-283: (tx, [u*, grad u*, Hess u*]) — equations with a Hessian term only."""
        if not isinstance(self.equation, SimpleDiffusionEquationWithHessian):
            raise AssertionError("exact Hessian labels need a SimpleDiffusionEquationWithHessian (data.py:274)")
        tx, t, x = self._t_x(n_batch)
        with torch.no_grad():
            u, ux, uh = self.equation.u_u_x_u_hessian(t, x)
        return self._out(tx, torch.cat([u.to(tx), ux.to(tx), uh.reshape(u.shape[0], -1).to(tx)], -1))

    # ------------------------------------------------------------------ datasets (data.py:285-335)
    def _dataset(self, n_total, n_batch_buffer, batch_size, sampler, guard=True):
        ds = IterableDatasetWithInternalBatch(n_total, n_batch_buffer, batch_size, sampler,
                                              range_guard=self if guard else None)
        cap = self.max_points_per_call
        if cap is not None and ds._n_samples_each_call > cap:
            raise torch.cuda.OutOfMemoryError(
                f"{ds._n_samples_each_call} points per generator call (n_batch_buffer {n_batch_buffer} x batch_size "
                f"{batch_size}) exceed the generator's max_points_per_call = {cap} (DATA.POINTS_PER_CALL)")
        return ds

    def dataset(self, n_total, n_batch_buffer, batch_size):
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample)

    def dataset_with_gradients(self, n_total, n_batch_buffer, batch_size):
        """The boundary: the buffered iterable dataset over sample_with_gradients."""
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample_with_gradients)

    def dataset_with_gradients_and_hessians(self, n_total, n_batch_buffer, batch_size):
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample_with_gradients_and_hessians)

    def dataset_exact(self, n_total, n_batch_buffer, batch_size):
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample_exact, guard=False)

    def dataset_exact_with_gradients(self, n_total, n_batch_buffer, batch_size):
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample_exact_with_gradients, guard=False)

    def dataset_exact_with_gradients_and_hessians(self, n_total, n_batch_buffer, batch_size):
        return self._dataset(n_total, n_batch_buffer, batch_size, self.sample_exact_with_gradients_and_hessians, guard=False)

    # ------------------------------------------------------------------ moments (sharding building blocks)
    def workspace_bytes(self, n, M, hessians=False, prepared=False):
        """Device workspace (bytes) of n points x M paths; prepared: for label_prepare and the
        DPI_PREPARED label_moments call it feeds (include/dpi.h dpi_workspace_bytes_prepared)."""
        fn = self.lib.dpi_workspace_bytes_prepared if prepared else self.lib.dpi_workspace_bytes
        need = fn(self.problem, self.net.handle, n, M)
        if hessians:
            fh = self.lib.dpi_workspace_bytes_hessians_prepared if prepared else self.lib.dpi_workspace_bytes_hessians
            need = max(need, fh(self.problem, self.net.handle, n, M))
        return need

    def point_baseline(self, tx, hessians=False, ws=None):
        """Per-point baseline into the generator's workspace, or into `ws` (uint8, >= workspace_bytes)."""
        n = tx.shape[0]
        M = max(self.n_estimate_terminal, self.n_estimate_integral)
        if ws is None:
            ws = self._workspace(n, M, hessians)
        elif ws.numel() < self.workspace_bytes(n, M, hessians):
            raise ValueError("workspace too small")
        _lib.check(self.lib.dpi_point_baseline(self.problem, self.net.handle, _ptr(tx), n, _ptr(ws), ws.numel(),
                                               _stream(self._device)), "dpi_point_baseline")
        return ws

    def _pieces(self, m_begin, m_end, flags=0):
        """[m_begin, m_end) cut into ranges one C-ABI call takes (at most PATHS_PER_CALL_MAX paths)."""
        if m_end - m_begin <= PATHS_PER_CALL_MAX:
            return [(m_begin, m_end)]
        if flags & _lib.DPI_PREPARED:
            raise ValueError(f"a prepared label call covers at most {PATHS_PER_CALL_MAX} paths")
        return [(a, min(a + PATHS_PER_CALL_MAX, m_end)) for a in range(m_begin, m_end, PATHS_PER_CALL_MAX)]

    def label_moments(self, tx, point_base, M, m_begin, m_end, flags, ws):
        """Sum / sum-of-squares of per-path contributions over m in [m_begin, m_end): (n, 2, 1+nx).
        More than PATHS_PER_CALL_MAX paths run as several calls combined by moments_reduce."""
        pieces = self._pieces(m_begin, m_end, flags)
        if len(pieces) > 1:
            return self.moments_reduce(torch.stack([self._label_moments(tx, point_base, M, a, b, flags, ws)
                                                    for a, b in pieces]))
        return self._label_moments(tx, point_base, M, m_begin, m_end, flags, ws)

    def _label_moments(self, tx, point_base, M, m_begin, m_end, flags, ws):
        n = tx.shape[0]
        mom = torch.empty(n, 2, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
        self._configure_problem()
        _lib.check(self.lib.dpi_label_moments(self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed,
                                              self.epoch, point_base, m_begin, m_end, flags, _ptr(mom), _ptr(ws),
                                              ws.numel(), _stream(self._device)), "dpi_label_moments")
        return mom

    def label_moments_finalize(self, tx, point_base, M, flags, ws, bound=None):
        """label_moments over all of [0, M) and finalize in the same reduce launch -> (y, moments)."""
        n = tx.shape[0]
        mom = torch.empty(n, 2, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
        y = torch.empty(n, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
        b = self.sample_bound if bound is None else bound
        self._configure_problem()
        _lib.check(self.lib.dpi_label_moments_finalize(self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed,
                                                       self.epoch, point_base, flags, b, _ptr(y), _ptr(mom), _ptr(ws),
                                                       ws.numel(), _stream(self._device)),
                   "dpi_label_moments_finalize")
        return y, mom

    def label_prepare(self, tx, point_base, M, m_begin, m_end, flags, ws):
        """First half of label_moments that needs no network evaluation of this batch (PISGradNet:
        the first path chunk's rollout; a no-op otherwise), so it can run on a side stream under the
        previous batch's network work.  The matching label_moments call passes flags | DPI_PREPARED."""
        n = tx.shape[0]
        self._configure_problem()
        _lib.check(self.lib.dpi_label_prepare(self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed,
                                              self.epoch, point_base, m_begin, m_end, flags, _ptr(ws), ws.numel(),
                                              _stream(self._device)), "dpi_label_prepare")

    def finalize(self, moments, M, flags, ws, bound=None):
        n = moments.shape[0]
        y = torch.empty(n, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
        b = self.sample_bound if bound is None else bound
        _lib.check(self.lib.dpi_label_finalize(self.problem, _ptr(moments), n, M, flags, b, _ptr(y), _ptr(ws),
                                               ws.numel(), _stream(self._device)), "dpi_label_finalize")
        return y

    def label_moments_hessians(self, tx, point_base, M, m_begin, m_end, ws, flags=_lib.DPI_BOTH):
        """Hessian-label sums over m in [m_begin, m_end): moments (n, 2, 1+nx), Hessian sums (n, nx^2),
        of the estimators `flags` selects (DPI_TERMINAL / DPI_INTEGRAL / both).  More than
        PATHS_PER_CALL_MAX paths run as several calls combined by sums_reduce."""
        pieces = self._pieces(m_begin, m_end, flags)
        if len(pieces) > 1:
            parts = [self._label_moments_hessians(tx, point_base, M, a, b, ws, flags) for a, b in pieces]
            return (self.sums_reduce(torch.stack([p[0] for p in parts])),
                    self.sums_reduce(torch.stack([p[1] for p in parts])))
        return self._label_moments_hessians(tx, point_base, M, m_begin, m_end, ws, flags)

    def _label_moments_hessians(self, tx, point_base, M, m_begin, m_end, ws, flags=_lib.DPI_BOTH):
        n, nx = tx.shape[0], self.equation.nx
        mom = torch.empty(n, 2, 1 + nx, dtype=torch.float32, device=self._device)
        hs = torch.empty(n, nx * nx, dtype=torch.float32, device=self._device)
        self._configure_problem()
        _lib.check(self.lib.dpi_label_moments_hessians(
            self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed, self.epoch, point_base, m_begin, m_end,
            flags, _ptr(mom), _ptr(hs), _ptr(ws), ws.numel(), _stream(self._device)), "dpi_label_moments_hessians")
        return mom, hs

    def finalize_hessians(self, moments, hsums, M, ws, bound=None, flags=_lib.DPI_BOTH):
        n, nx = moments.shape[0], self.equation.nx
        y = torch.empty(n, 1 + nx + nx * nx, dtype=torch.float32, device=self._device)
        b = self.sample_bound if bound is None else bound
        _lib.check(self.lib.dpi_label_finalize_hessians(self.problem, _ptr(moments), _ptr(hsums), n, M, flags, b,
                                                        _ptr(y), _ptr(ws), ws.numel(), _stream(self._device)),
                   "dpi_label_finalize_hessians")
        return y

    def sums_reduce(self, parts):
        """(G, ...) per-rank sums -> (...), the canonical fixed-order tree over ranks."""
        parts = parts.contiguous()
        out = torch.empty(parts.shape[1:], dtype=parts.dtype, device=parts.device)
        _lib.check(self.lib.dpi_sums_reduce(_ptr(parts), parts.shape[0], out.numel(), _ptr(out), _stream(self._device)),
                   "dpi_sums_reduce")
        return out

    def moments_reduce(self, parts):
        """(G, n, 2, 1+nx) per-rank moments -> (n, 2, 1+nx), fixed pairwise order (parts is scratch)."""
        parts = parts.contiguous()
        G, n = parts.shape[0], parts.shape[1]
        out = torch.empty(parts.shape[1:], dtype=parts.dtype, device=parts.device)
        _lib.check(self.lib.dpi_moments_reduce(_ptr(parts), G, n, self.equation.nx, _ptr(out), _stream(self._device)),
                   "dpi_moments_reduce")
        return out

    # ------------------------------------------------------------------ internals
    def range_status(self, clear=True):
        """DPI_STATUS_* bits of the selected status slot (the immediate one outside a group) set by the
        label calls on this generator's net since the last clear (synchronises the stream)."""
        return self.net.status(_stream(self._device), clear)

    def _guarded(self, call, reduce_flag=None, defer=True):
        """Run a label call under the range guard.  Inside deferred_range_check() the call is
        registered with the open RangeGroup (checked at its verify()); otherwise it runs with the
        immediate slot selected and is checked at once: on a DPI_STATUS_NONFINITE flag the net
        switches to exact fp32 and the call runs again (same points and counters), or DPIError if
        it already ran in fp32.  reduce_flag: the multi-rank MAX of a flag (ShardedLabeler)."""
        if not self._range_check:
            return call()
        # no check inside a hipGraph capture (a synchronisation there would invalidate the capture);
        # the flag stays set and the next checked call on this net reports it
        if torch.cuda.is_current_stream_capturing():
            return call()
        if defer and self._scope is not None:
            return self._scope.enqueue(call, reduce_flag)
        prev = self._slot
        self._select_slot(IMMEDIATE_SLOT)
        try:
            y = call()
            flag = self.range_status()
        finally:
            self._select_slot(prev)
        if reduce_flag is not None:
            flag = reduce_flag(flag)
        _check_handoff(flag)
        if not flag & _lib.DPI_STATUS_NONFINITE:
            return y
        if self._fp32_fallback:
            raise _lib.DPIError("label call gave non-finite labels from a network with finite parameters in exact "
                                "fp32: the network's values exceed fp32's range")
        warnings.warn("the fp16-split evaluation of this network left fp16's range (|activation| > 65504); its "
                      "labels are recomputed, and this generator's later calls run, with exact-fp32 MFMA",
                      SplitRangeWarning, stacklevel=3)
        self.use_fp32()
        return self._guarded(call, reduce_flag, defer=False)

    def use_fp32(self):
        """Evaluate this generator's network with exact-fp32 MFMA from now on (dpi_net_set_precision)."""
        self.net.set_precision(_lib.DPI_GEMM_F32)
        self._fp32_fallback = True

    def _generate_hess(self, tx, pb, bound):
        return self._guarded(lambda: self._generate_hess_once(tx, pb, bound))

    def _generate_hess_once(self, tx, pb, bound):
        MT, MI = self.n_estimate_terminal, self.n_estimate_integral
        if MT != MI:  # the terminal estimators over MT paths + the integral ones over MI (data.py:1164, :845)
            ws = self.point_baseline(tx, hessians=True)
            parts = [self.finalize_hessians(*self.label_moments_hessians(tx, pb, M, 0, M, ws, f), M, ws,
                                            float("inf"), f)
                     for M, f in ((MT, _lib.DPI_TERMINAL), (MI, _lib.DPI_INTEGRAL))]
            b = self.sample_bound if bound is None else bound
            return torch.clamp(parts[0] + parts[1], -b, b)
        n, nx, M = tx.shape[0], self.equation.nx, self.n_estimate_integral
        if M > PATHS_PER_CALL_MAX:  # several calls: baseline, per-range sums, one finalize
            ws = self.point_baseline(tx, hessians=True)
            mom, hs = self.label_moments_hessians(tx, pb, M, 0, M, ws)
            return self.finalize_hessians(mom, hs, M, ws, bound)
        need = self.lib.dpi_workspace_bytes_hessians(self.problem, self.net.handle, n, M)
        if self._ws is None or self._ws.numel() < need:
            self._ws = new_workspace(need, self._device)
        y = torch.empty(n, 1 + nx + nx * nx, dtype=torch.float32, device=self._device)
        self._configure_problem()
        _lib.check(self.lib.dpi_generate_with_gradients_and_hessians(
            self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed, self.epoch, pb, bound, _ptr(y),
            _ptr(self._ws), self._ws.numel(), _stream(self._device)), "dpi_generate_with_gradients_and_hessians")
        return y


    def _as_points(self, tx):
        if tx.device != self._device or tx.dtype != torch.float32 or not tx.is_contiguous():
            tx = tx.to(device=self._device, dtype=torch.float32).contiguous()
        return tx

    def _generate(self, tx, pb, flags, bound=None):
        return self._guarded(lambda: self._generate_once(tx, pb, flags, bound))

    def _generate_once(self, tx, pb, flags, bound=None):
        MT, MI = self.n_estimate_terminal, self.n_estimate_integral
        if (MT == MI or flags != _lib.DPI_BOTH) and max(MT, MI) <= PATHS_PER_CALL_MAX:
            # one C-ABI call: baseline + fused rollout/label kernel + block reduce/finalize
            M = MT if flags == _lib.DPI_TERMINAL else MI
            n = tx.shape[0]
            ws = self._workspace(n, max(MT, MI))
            y = torch.empty(n, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
            self.last_moments = torch.empty(n, 2, 1 + self.equation.nx, dtype=torch.float32, device=self._device)
            b = self.sample_bound if bound is None else bound
            self._configure_problem()
            _lib.check(self.lib.dpi_generate_with_gradients(
                self.problem, self.net.handle, _ptr(tx), n, M, self.K, self.seed, self.epoch, pb, flags, b, _ptr(y),
                _ptr(self.last_moments), _ptr(ws), ws.numel(), _stream(self._device)), "dpi_generate_with_gradients")
            return y
        ws = self.point_baseline(tx)
        if MT == MI or flags != _lib.DPI_BOTH:  # one estimator set over more paths than one call takes
            M = MT if flags == _lib.DPI_TERMINAL else MI
            self.last_moments = self.label_moments(tx, pb, M, 0, M, flags, ws)
            return self.finalize(self.last_moments, M, flags, ws, bound)
        yT = self.finalize(self.label_moments(tx, pb, MT, 0, MT, _lib.DPI_TERMINAL, ws), MT, _lib.DPI_TERMINAL, ws,
                           float("inf"))
        yI = self.finalize(self.label_moments(tx, pb, MI, 0, MI, _lib.DPI_INTEGRAL, ws), MI, _lib.DPI_INTEGRAL, ws,
                           float("inf"))
        b = self.sample_bound if bound is None else bound
        return torch.clamp(yT + yI, -b, b)
