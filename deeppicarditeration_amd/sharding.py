"""Monte-Carlo sharding of the label path across GPUs (one process per GPU, torch.distributed
over RCCL/xGMI).

Every path-label is independent and a label is a mean over MC indices m, so rank r of G owns
m in [r M/G, (r+1) M/G) for all points.  Noise counters are global (seed, epoch, point, m, step),
so each path sees the same noise for any G, and the collocation points are sampled identically
on every rank from the same counters (no broadcast).  The one exchange is an all-gather of the
per-rank label moments (n, 2, 1+nx) fp32 — 2 x 16 x 101 x 4 B = 12.9 kB per rank at config 2,
414 kB in total at config 4 — followed by dpi_moments_reduce, the same fixed pairwise tree the
kernel uses over 64-path blocks.  With M/(64 G) a power of two the labels are bit-identical for
G = 1, 2, 4, 8.  (The reference has no collective: SURVEY.md §2 rows 18-19.)
"""
import warnings

import torch


_WARNED = set()


class ShardBitIdentityWarning(UserWarning):
    """M / (64 G) is not a power of two: the labels are correct Monte-Carlo means, but the rank
    sums no longer split the single-call block tree at a power-of-two boundary, so they can differ
    from the one-GPU labels in the last bits."""


class ShardedLabeler:
    def __init__(self, gen, rank=0, world=1, group=None, sample_ahead=False):
        """sample_ahead (PISGradNet, prepare()): each prepare() also samples the NEXT batch's points,
        on a stream of their own, so the next prepare's rollout does not wait for a sampling launch
        on the side stream's critical path.  The batches get the same point ranges in the same
        order (under the generator's seed and epoch at the prepare() that samples them; a batch
        sampled ahead under another seed or epoch than the next prepare()'s is dropped and that
        prepare samples afresh); the points sampled ahead of the last prepare() are skipped — the
        generator's point counter stays one batch further on, which later draws see as a shift of
        their point indices."""
        self.gen = gen
        self.rank = rank
        self.world = world
        self.group = group
        self.sample_ahead = sample_ahead
        self._ahead = None

    def shard(self, M):
        blk = 64
        if M % (blk * self.world):
            raise ValueError(f"M={M} must be a multiple of 64 x world ({self.world})")
        per = M // self.world
        nb = per // blk
        if self.world > 1 and nb & (nb - 1):
            key = (M, self.world)
            if key not in _WARNED:
                _WARNED.add(key)
                warnings.warn(f"M={M} over {self.world} ranks gives {nb} 64-path blocks per rank, not a power of two: "
                              "labels will not be bit-identical to the single-GPU labels (the canonical tree splits "
                              "only at power-of-two block counts)", ShardBitIdentityWarning, stacklevel=2)
        return self.rank * per, (self.rank + 1) * per

    def estimator_sets(self, flags=None):
        """[(M, flags)] of this generator's label passes: one pass over M paths when
        n_estimate_terminal == n_estimate_integral (or one estimator is asked for), else a
        DPI_TERMINAL pass over n_estimate_terminal paths and a DPI_INTEGRAL pass over
        n_estimate_integral paths, whose labels add (picard/data.py:1208-1218; the counts
        :444, :460, :845, :1164).  Each pass shards its own M across the ranks."""
        from . import _lib
        flags = _lib.DPI_BOTH if flags is None else flags
        MT, MI = self.gen.n_estimate_terminal, self.gen.n_estimate_integral
        if MT == MI or flags != _lib.DPI_BOTH:
            return [(MT if flags == _lib.DPI_TERMINAL else MI, flags)]
        return [(MT, _lib.DPI_TERMINAL), (MI, _lib.DPI_INTEGRAL)]

    def _bound(self):
        return getattr(self.gen, "sample_bound", float("inf"))

    def _add_clip(self, ys):
        """Labels of the estimator passes -> their sum, clipped like the reference (data.py:222)."""
        if len(ys) == 1:
            return ys[0]
        b = self._bound()
        return torch.clamp(ys[0] + ys[1], -b, b)

    def gather_moments(self, mom):
        if self.world == 1:
            return mom
        import torch.distributed as dist
        mom = mom.contiguous()
        flat = torch.empty((self.world * mom.shape[0],) + tuple(mom.shape[1:]), dtype=mom.dtype, device=mom.device)
        dist.all_gather_into_tensor(flat, mom, group=self.group)  # rank-major concatenation
        return self.gen.moments_reduce(flat.view((self.world,) + tuple(mom.shape)))

    def _gather_stacked(self, parts, reduce, async_op=False):
        """One all-gather of this rank's per-pass tensors (same shape), stacked; -> (flat, work)
        for _reduce_stacked (async) or the per-pass rank-reduced tensors."""
        import torch.distributed as dist
        x = torch.stack([p.contiguous() for p in parts]).contiguous()
        flat = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        work = dist.all_gather_into_tensor(flat.view((self.world * x.shape[0],) + tuple(x.shape[1:])), x,
                                           group=self.group, async_op=async_op)
        if async_op:
            return flat, work
        return [reduce(flat[:, k]) for k in range(len(parts))]

    def gather_sums(self, x):
        """All-gather per-rank sums (any shape) and reduce them in canonical rank order."""
        if self.world == 1:
            return x
        import torch.distributed as dist
        x = x.contiguous()
        flat = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(flat, x, group=self.group)
        return self.gen.sums_reduce(flat.view((self.world,) + tuple(x.shape)))

    def _reduce_flag(self, flag):
        """A range-guard flag of this rank -> the MAX over all ranks (every rank repairs together)."""
        if self.world == 1:
            return flag
        import torch.distributed as dist
        # a device tensor under RCCL and under gloo alike (gloo stages it through the host), so the
        # one-GPU gloo rehearsal runs the RCCL branch's code
        t = torch.tensor([float(flag)], device=getattr(self.gen, "device", "cpu"))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def _guarded(self, call):
        """The generator's range guard (OnlineDataGenerator._guarded) across ranks: any rank's flag
        is every rank's (a one-word MAX all-reduce), so all ranks recompute in fp32 together; inside
        the generator's deferred_range_check() the call joins the open RangeGroup."""
        g = getattr(self.gen, "_guarded", None)
        return call() if g is None else g(call, reduce_flag=self._reduce_flag)

    def labels_hessians(self, tx=None, point_base=None, on_moments_begin=None, on_moments_end=None, prepared=None):
        """Hessian labels of tx, or of the batch prepare(n, hessians=True) returned (`prepared`: its
        points, baseline and staged noise sums; the labels are bitwise those of the unprepared call).
        A range-guard repair reruns the batch unprepared."""
        if prepared is not None:
            tx, point_base = prepared[0], prepared[1]
        state = {"prep": prepared}

        def call():
            prep, state["prep"] = state["prep"], None
            return self._labels_hessians(tx, point_base, on_moments_begin, on_moments_end, prep)
        return self._guarded(call)

    def _labels_hessians(self, tx, point_base, on_moments_begin=None, on_moments_end=None, prepared=None):
        """generate_with_gradients_and_hessians for tx with this rank's MC shard (n, 1 + nx + nx^2);
        identical on every rank.  Exchange: the (n, 2, 1+nx) moments and (n, nx^2) Hessian sums (of
        both estimator passes when n_estimate_terminal != n_estimate_integral)."""
        from . import _lib
        sets = self.estimator_sets()
        kflags = 0
        if prepared is not None:
            _, _, ws, ready, slot, _, staged = prepared
            torch.cuda.current_stream(self.gen.device).wait_event(ready)
            if staged:
                kflags = _lib.DPI_PREPARED
        else:
            ws = self.gen.point_baseline(tx, hessians=True)
        if on_moments_begin:
            on_moments_begin()
        if len(sets) == 1:
            M = sets[0][0]
            mom, hs = self.gen.label_moments_hessians(tx, point_base, M, *self.shard(M), ws,
                                                      flags=_lib.DPI_BOTH | kflags)
            if on_moments_end:
                on_moments_end()
            y = self.gen.finalize_hessians(self.gather_sums(mom), self.gather_sums(hs), M, ws)
            self._release_prepared(prepared)
            return y
        sums = [self.gen.label_moments_hessians(tx, point_base, M, *self.shard(M), ws, flags=f) for M, f in sets]
        if on_moments_end:
            on_moments_end()
        if self.world > 1:
            moms = self._gather_stacked([m for m, _ in sums], self.gen.sums_reduce)
            hss = self._gather_stacked([h for _, h in sums], self.gen.sums_reduce)
            sums = list(zip(moms, hss))
        y = self._add_clip([self.gen.finalize_hessians(mom, hs, M, ws, bound=float("inf"), flags=f)
                            for (mom, hs), (M, f) in zip(sums, sets)])
        self._release_prepared(prepared)
        return y

    def _release_prepared(self, prepared):
        """prepare() may refill a prepared batch's workspace once the work enqueued on it has run."""
        if prepared is None:
            return
        slot = prepared[4]
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(self.gen.device))
        self._prep_free[slot] = done
        self._prep_busy[slot] = False

    # ------------------------------------------------------------------ two-phase (pipelined) labels
    def prepare(self, n, flags=None, hessians=False):
        """Sample the next batch's points, their per-point baseline and (PISGradNet) the first path
        chunk's rollout on a side stream, into one of three workspaces, so they run while the
        current stream still executes the previous batch's moments: the baseline is a handful of
        latency-bound blocks that otherwise serialise between two path launches, and the VALU-bound
        rollout fits on each CU beside a k_gemm_x3 block of the previous batch's MFMA-bound GEMM
        chain.  Returns the handle for begin(prepared=...), or, with hessians=True (workspaces sized
        for the Hessian labels), for labels_hessians(prepared=...)."""
        from . import _lib
        flags = _lib.DPI_BOTH if flags is None else flags
        gen = self.gen
        cur = torch.cuda.current_stream(gen.device)
        sets = self.estimator_sets(flags)
        M = max(m for m, _ in sets)
        # unequal estimator counts run two label passes in begin(): their points and baseline are
        # prepared here, the passes themselves are not staged
        staged = len(sets) == 1
        need = gen.workspace_bytes(n, M, hessians=hessians, prepared=True)
        if getattr(self, "_prep_ws", None) is None or self._prep_ws[0].numel() < need:
            torch.cuda.synchronize(gen.device)  # a resized pool must not alias in-flight work
            self._side = torch.cuda.Stream(device=gen.device)
            from .data import new_workspace
            self._prep_ws = [new_workspace(need, gen.device) for _ in range(3)]
            self._prep_free, self._prep_next, self._prep_busy = [None] * 3, 0, [False] * 3
        k = self._prep_next
        if self._prep_busy[k]:
            raise RuntimeError("prepare(): all three workspaces hold batches whose end() has not run")
        self._prep_next = (k + 1) % 3
        self._prep_busy[k] = True
        ws = self._prep_ws[k]
        # PISGradNet only: its points need no workspace (the baseline lives in the label call)
        pis = str(getattr(getattr(gen, "net", None), "desc", "")).startswith("pisgrad")
        ahead, self._ahead = self._ahead, None
        if ahead is not None and ahead[:3] != (n, getattr(gen, "seed", None), getattr(gen, "epoch", None)):
            ahead = None  # another batch size, seed or epoch (Picard iteration): those points are skipped
        with torch.cuda.stream(self._side):
            if self._prep_free[k] is not None:  # the batch that last used this workspace is finalized
                self._side.wait_event(self._prep_free[k])
            m0, m1 = self.shard(M)
            if ahead is not None:
                tx, pb, ev = ahead[3:]
                self._side.wait_event(ev)
                tx.record_stream(self._side)
                if staged:
                    gen.label_prepare(tx, pb, M, m0, m1, flags, ws)
            elif pis or not staged or not hasattr(gen, "sample_points_baseline"):  # the staged rollout reads the points
                if hasattr(gen, "sample_points_baseline"):  # one launch: the sampling inside the baseline's
                    pb = gen._take_points(n)
                    tx = gen.sample_points_baseline(n, pb, ws)
                else:
                    tx, pb = gen.sample_t_and_x(n)
                    gen.point_baseline(tx, ws=ws)
                if staged:
                    gen.label_prepare(tx, pb, M, m0, m1, flags, ws)
            else:
                # fused-kernel nets: the staged part (GBM: the noise sums, dpi_label_prepare) needs no
                # points, so it is enqueued first and starts beside the previous batch's path launch;
                # the sampling + baseline launch follows it on this stream
                pb = gen._take_points(n)
                tx = torch.empty(n, 1 + gen.equation.nx, dtype=torch.float32, device=gen.device)
                gen.label_prepare(tx, pb, M, m0, m1, flags, ws)
                gen.sample_points_baseline(n, pb, ws, out=tx)
            ready = torch.cuda.Event()
            ready.record(self._side)
        tx.record_stream(cur)
        if self.sample_ahead and pis:
            if getattr(self, "_samp", None) is None:
                self._samp = torch.cuda.Stream(device=gen.device)
            with torch.cuda.stream(self._samp):
                pb2 = gen._take_points(n)
                tx2, _ = gen.sample_t_and_x(n, point_base=pb2)
                ev2 = torch.cuda.Event()
                ev2.record(self._samp)
            self._ahead = (n, getattr(gen, "seed", None), getattr(gen, "epoch", None), tx2, pb2, ev2)
        return tx, pb, ws, ready, k, flags, staged

    def begin(self, tx=None, point_base=None, flags=None, on_moments_begin=None, on_moments_end=None,
              prepared=None):
        """First half of labels(): this rank's moments and, for world > 1, an asynchronous
        all-gather of them (RCCL runs on its own stream, so the caller can enqueue the next batch's
        kernels while it is in flight).  Two workspaces alternate (three with prepare()), so one
        batch may be pending while the next begins.  Returns the handle end() turns into labels."""
        from . import _lib
        slot = wslot = None
        kflags = None
        grp = self._range_group()
        if prepared is not None:
            tx, point_base, ws, ready, slot, pflags, staged = prepared
            if flags is not None and flags != pflags:
                raise ValueError(f"begin(flags={flags}) on a batch prepared with flags={pflags}")
            flags = pflags
            if staged:
                kflags = flags | _lib.DPI_PREPARED
            torch.cuda.current_stream(self.gen.device).wait_event(ready)
        sets = self.estimator_sets(flags)
        M = max(m for m, _ in sets)
        if prepared is None:
            n = tx.shape[0]
            need = self.gen.workspace_bytes(n, M)
            if not hasattr(self, "_ws_pool") or self._ws_pool[0].numel() < need:
                if any(getattr(self, "_ws_busy", ())):
                    raise RuntimeError("begin(): cannot resize the workspaces while a batch is pending")
                dev = getattr(tx, "device", "cpu")
                from .data import new_workspace
                self._ws_pool = [new_workspace(need, dev) for _ in range(2)]
                self._ws_next, self._ws_busy = 0, [False, False]
            wslot = self._ws_next
            if self._ws_busy[wslot]:
                raise RuntimeError("begin(): two batches are already pending; end() one before beginning another")
            self._ws_busy[wslot] = True
            ws = self._ws_pool[wslot]
            self._ws_next ^= 1
            self.gen.point_baseline(tx, ws=ws)
        flags = _lib.DPI_BOTH if flags is None else flags
        repair = (tx, point_base, flags)  # end() registers labels(tx, point_base, flags) as the repair
        if on_moments_begin:
            on_moments_begin()
        if self.world == 1:  # one rank: the labels come out of the moments' reduce launch
            if len(sets) == 1:
                y, _ = grp.run(lambda: self.gen.label_moments_finalize(tx, point_base, M,
                                                                       flags if kflags is None else kflags, ws))
            else:
                y = grp.run(lambda: self._add_clip([self.gen.label_moments_finalize(tx, point_base, m, f, ws,
                                                                                    bound=float("inf"))[0]
                                                    for m, f in sets]))
            if on_moments_end:
                on_moments_end()
            return (None, y, None, sets, slot, wslot, grp, repair)  # ws None: y final (end() recycles)
        moms = [grp.run(lambda m=m, f=f: self.gen.label_moments(tx, point_base, m, *self.shard(m),
                                                                f if kflags is None else kflags, ws))
                for m, f in sets]
        if on_moments_end:
            on_moments_end()
        flat, work = self._gather_stacked(moms, None, async_op=True)
        return (ws, flat, work, sets, slot, wslot, grp, repair)

    def _pipeline_pending(self):
        return any(getattr(self, "_ws_busy", ())) or any(getattr(self, "_prep_busy", ()))

    def _range_group(self):
        """The RangeGroup a pipelined batch's reductions flag into: the generator's open
        deferred_range_check() group if there is one, else this labeler's pipeline group, opened by
        the first begin() after the last check and verified by pipeline_range_check()."""
        gen = self.gen
        if not hasattr(gen, "deferred_range_check"):
            from .data import _NoGroup
            return _NoGroup()
        if gen._scope is not None:
            return gen._scope
        pg = getattr(self, "_pipe_group", None)
        if pg is None:
            pg = gen.deferred_range_check()
            if gen._scope is pg:  # not the open scope: begin() selects its slot around each enqueue
                gen._scope = None
            self._pipe_group = pg
        return pg

    def pipeline_range_check(self):
        """The range guard of the pipelined path (prepare/begin/end) outside a generator group:
        once every pending batch has ended, verify the pipeline's RangeGroup (one event wait and a
        host read of its status slot; a MAX across ranks) — a flagged pipeline has its batches
        recomputed in exact fp32 into the labels end() returned (SplitRangeWarning), or raises
        DPIError if the net already ran in fp32.  Returns the flag."""
        if self._pipeline_pending():
            raise RuntimeError("pipeline_range_check(): end() every pending batch first")
        pg, self._pipe_group = getattr(self, "_pipe_group", None), None
        if pg is None:
            return 0
        pg.reduce_flag = self._reduce_flag
        return pg.verify()

    def end(self, pending):
        """Second half: wait for the all-gather, canonical reduce, finalize -> y (n, 1+nx)."""
        ws, flat, work, sets, slot, wslot, grp, (tx, point_base, rflags) = pending
        if ws is None:  # one rank: begin() already finalized
            y = flat
        else:
            work.wait()  # the current stream waits for RCCL's, not the host
            bound = None if len(sets) == 1 else float("inf")
            y = self._add_clip([self.gen.finalize(self.gen.moments_reduce(flat[:, k]), m, f, ws, bound=bound)
                                for k, (m, f) in enumerate(sets)])
        if slot is not None:  # prepare() may refill this workspace once the finalize has run
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.gen.device))
            self._prep_free[slot] = done
            self._prep_busy[slot] = False
        if wslot is not None:  # stream order makes the next user of this workspace run after finalize
            self._ws_busy[wslot] = False
        # final once the group verifies: a flagged batch is recomputed by the unpipelined labels()
        return grp.register(lambda: self._labels(tx, point_base, rflags), y, self._reduce_flag)

    def labels(self, tx, point_base, flags=None, on_moments_begin=None, on_moments_end=None):
        """generate_with_gradients for tx with this rank's MC shard; identical y on every rank
        (range-guarded like the generator's calls when gen.range_check)."""
        return self._guarded(lambda: self._labels(tx, point_base, flags, on_moments_begin, on_moments_end))

    def _labels(self, tx, point_base, flags=None, on_moments_begin=None, on_moments_end=None):
        sets = self.estimator_sets(flags)
        ws = self.gen.point_baseline(tx)
        if on_moments_begin:
            on_moments_begin()
        bound = None if len(sets) == 1 else float("inf")  # two passes: clip their sum, not each
        if self.world == 1:  # one rank: the labels come out of the moments' reduce launch
            ys = [self.gen.label_moments_finalize(tx, point_base, m, f, ws, bound=bound)[0] for m, f in sets]
            if on_moments_end:
                on_moments_end()
            return self._add_clip(ys)
        moms = [self.gen.label_moments(tx, point_base, m, *self.shard(m), f, ws) for m, f in sets]
        if on_moments_end:
            on_moments_end()
        moms = self._gather_stacked(moms, self.gen.moments_reduce)
        return self._add_clip([self.gen.finalize(mom, m, f, ws, bound=bound) for mom, (m, f) in zip(moms, sets)])

    # ------------------------------------------------------------------ batch_data_generator surface
    def sample_labels(self, n_batch, on_moments_begin=None, on_moments_end=None):
        """(tx, point_base, labels) for the next n_batch points: for one rank the generator's
        two-launch dpi_sample_with_gradients (range-guarded like labels()), else sampling + labels()."""
        gen = self.gen
        if self.world == 1 and hasattr(gen, "sample_generate") and \
                gen.n_estimate_terminal == gen.n_estimate_integral and gen.n_estimate_integral <= 65536:
            pb = gen._take_points(n_batch)
            tx, y = self._guarded(lambda: gen.sample_generate(n_batch, pb, on_moments_begin=on_moments_begin,
                                                              on_moments_end=on_moments_end))
            return tx, pb, y
        tx, pb = gen.sample_t_and_x(n_batch)
        return tx, pb, self.labels(tx, pb, on_moments_begin=on_moments_begin, on_moments_end=on_moments_end)

    def sample_with_gradients(self, n_batch):
        """OnlineDataGenerator.sample_with_gradients with this rank's MC shard: every rank draws the
        same points (same counters) and returns the same (tx, clip(u_ux))."""
        tx, _, y = self.sample_labels(n_batch)
        return tx, y

    def sample_with_gradients_and_hessians(self, n_batch):
        tx, pb = self.gen.sample_t_and_x(n_batch)
        return tx, self.labels_hessians(tx, pb)
