"""`picard train` on MI355X: the reference's Picard loop (picard/picard_iteration.py:120-307) with
the label generation replaced by the HIP path and the labels kept on the device.

Per Picard iteration i:
  1. labels: `LabelBuffer` fills DATA_SIZE (tx, u_ux) rows on the GPU with
     `OnlineDataGenerator.sample_with_gradients` calls of DATA.POINTS_PER_CALL points — the
     reference's CPU `InMemorySaver` round trip (picard/data_saver.py:69-83) and its OOM-probing
     memory tracker (picard/memory.py) are not needed: the fused kernel never materialises n*M
     tensors;
  2. fit: N_EPOCHS of shuffled mini-batches, value loss weighted by exp(beta t)
     (picard/solution.py:75-82), plus the gradient loss of PicardSolutionGradientWrapper with a
     FixedLossScaler (picard/solution_jac.py:71-82, 167-213) when its weight > 0, or — with
     TRAIN.SUPERVISE_HESSIAN — gradient + Hessian losses of PicardSolutionGradientHessianWrapper with
     a FixedHessianLossScaler (solution_jac.py:85-109, 219-259) on Malliavin Hessian labels;
  3. checkpoint model_{i}.pt; the trained network becomes the next iteration's u.
Iteration 1 uses ZeroSolution (picard_iteration.py:182).
"""
import json
import pathlib
import shutil
import time
import warnings

import torch

from . import equations as eqs
from .config import CfgNode
from .data import OnlineDataGenerator
from .dataset import TensorDatasetBuiltInShuffle
from .fit import build_objective, make_optimizer, train_steps
from .sharding import ShardedLabeler
from .solution import PISGradNet, ZeroSolution, construct_mlp


class LabelBuffer:
    """Device-resident (tx, y) label store for one Picard iteration, filled by DATA_SIZE / POINTS_PER_CALL
    calls of a batch_data_generator `sample(n) -> (tx, y)` (a generator's sample_with_gradients /
    sample_with_gradients_and_hessians / sample_exact_*, or a ShardedLabeler's).

    `guard` (the OnlineDataGenerator behind `sample`): the calls of one fill form one RangeGroup of
    its range guard, checked once when the fill is done (data.RangeGroup) instead of with a stream
    synchronisation after every call."""

    def __init__(self, sample, n_total, points_per_call, guard=None):
        self.sample = sample
        self.n_total = int(n_total)
        self.ppc = max(1, min(int(points_per_call), self.n_total))
        self.guard = guard

    def fill(self):
        txs, ys = [], []
        done = 0
        grp = self.guard.deferred_range_check() if hasattr(self.guard, "deferred_range_check") else None
        try:
            while done < self.n_total:
                n = min(self.ppc, self.n_total - done)
                tx, y = self.sample(n)
                txs.append(tx)
                ys.append(y)
                done += n
        except BaseException:
            if grp is not None:
                grp.discard()
            raise
        if grp is not None:
            grp.close()
        if grp is not None:
            grp.verify()  # before the concatenation: a repair rewrites the calls' own outputs
        return torch.cat(txs), torch.cat(ys)


def eval_metrics(u, u_exact, ux=None, ux_exact=None, uxx=None, uxx_exact=None):
    """EvalCallback.on_validation_epoch_start (picard/utils.py:404-475): MSE / rRMSE / rMAE / MArE of
    u, and with gradients (EVAL.TEST_GRAD) / Hessians (EVAL.TEST_HESSIAN) the per-dimension
    relative errors averaged over dimensions (suffix g / h).  numpy fp64 arrays."""
    import numpy as np
    # An exact value of 0 (e.g. the off-diagonal Hessian entries of a separable exact solution) makes
    # the MArE terms inf or nan, exactly as the reference's numpy expressions do; the metric keeps that
    # value (the reference logs it as is), without numpy's RuntimeWarning on every evaluation.
    with np.errstate(divide="ignore", invalid="ignore"):
        return _eval_metrics(np, u, u_exact, ux, ux_exact, uxx, uxx_exact)


def _eval_metrics(np, u, u_exact, ux, ux_exact, uxx, uxx_exact):
    err = np.abs(u - u_exact)
    m = {"MSE": float(np.sqrt((err ** 2).mean())), "rRMSE": float(np.sqrt((err ** 2).sum()) / np.sqrt((u_exact ** 2).sum())),
         "rMAE": float(err.sum() / np.abs(u_exact).sum()), "MArE": float((err / np.abs(u_exact)).mean())}
    for tag, a, b in (("g", ux, ux_exact), ("h", uxx, uxx_exact)):
        if a is None:
            continue
        e = np.abs(a - b)
        m.update({f"MSE{tag}": float(np.sqrt((e ** 2).mean(0)).mean()),
                  f"rRMSE{tag}": float((np.sqrt((e ** 2).sum(0)) / np.sqrt((b ** 2).sum(0))).mean()),
                  f"rMAE{tag}": float((e.sum(0) / np.abs(b).sum(0)).mean()),
                  f"MArE{tag}": float((e / np.abs(b)).mean())})
    return m


class PicardRunner:
    def __init__(self, cfg: CfgNode, device="cuda", rank=0, world=1, group=None):
        """rank / world > 1: one process per GPU in a torch.distributed job (RCCL on the GPU).
        Every rank generates the labels of its Monte-Carlo shard (ShardedLabeler: one all-gather of
        label moments per call, identical labels on every rank); rank 0 fits, writes the checkpoint,
        history and label files, and broadcasts the fitted weights, so every rank starts the next
        Picard iteration from the same u."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.rank, self.world, self.group = int(rank), int(world), group
        self.exp_dir = pathlib.Path(cfg.NAME)
        err = None
        if self.rank == 0:
            try:
                if self.exp_dir.exists() and any(self.exp_dir.iterdir()):
                    if not cfg.FORCE:
                        raise FileExistsError(f"Experiment directory {self.exp_dir} already exists.")
                    shutil.rmtree(self.exp_dir)
                self.exp_dir.mkdir(parents=True, exist_ok=True)
                (self.exp_dir / "config.yaml").write_text(cfg.dump())
            except Exception as e:  # noqa: BLE001 — re-raised below, after every rank knows
                err = e
        self._agree(err, "experiment directory setup")
        if str(cfg.DATA.FLOAT).lower() in ("double", "float64"):  # picard/config.py:194-200
            warnings.warn("DATA.FLOAT: double — the device label path computes in fp32 (labels within the "
                          "north star's rel-L2 <= 1e-4 of the fp64 reference, DESIGN.md); the fit and the "
                          "label files follow DATA.FLOAT", stacklevel=2)
        if cfg.METHOD.cls != "Picard":  # Diffusion / PINN / FullyNonlinearSolver baselines: out of scope
            raise NotImplementedError(f"METHOD.cls={cfg.METHOD.cls}: only the DPI (Picard) method is built")
        if cfg.PICARD.FORMULA == "TwoLayer":
            raise NotImplementedError("PICARD.FORMULA=TwoLayer is out of scope")
        self.equation = getattr(eqs, cfg.EQUATION.cls)(**cfg.EQUATION.kwargs)  # picard_iteration.py:90-92
        self.supervise_gradient = bool(cfg.TRAIN.SUPERVISE_GRADIENT or self.equation.has_gradient_term)
        self.supervise_hessian = bool(cfg.TRAIN.SUPERVISE_HESSIAN)  # picard_iteration.py:160, :114
        if cfg.NETWORK.TYPE != "Value":
            raise NotImplementedError("NETWORK.TYPE must be 'Value' for the device label path")
        self.N = cfg.PICARD.N
        self.i = 0
        self.u_current = ZeroSolution(1)
        self.history = []

    def _agree(self, err, what):
        """Multi-rank jobs: every rank learns whether any rank failed `what` before the next
        collective, so a failure on rank 0 alone (existing experiment directory, an exception in the
        fit) ends every rank with an error instead of leaving the others blocked in the label
        all-gather or the weight broadcast until the process-group timeout."""
        if self.world > 1:
            import torch.distributed as dist
            dev = "cpu" if dist.get_backend(self.group) == "gloo" else self.device
            flag = torch.tensor([0.0 if err is None else 1.0], device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            if err is None and float(flag) > 0:
                raise RuntimeError(f"{what} failed on another rank; stopping this rank")
        if err is not None:
            raise err

    # ------------------------------------------------------------------ networks
    def new_network(self):
        c = self.cfg.NETWORK
        if c.PISGRADNET:  # picard/solution.py:313-316
            net = PISGradNet(hidden_shapes=list(c.NEURONS), dim=self.equation.nx, g0=self.equation.g, T=self.equation.T)
        else:
            net = construct_mlp(1 + self.equation.nx, 1, list(c.NEURONS), list(c.ACTIVATIONS), c.BOUND)
        return net.to(self.device)

    def checkpoint_path(self, i):
        return self.exp_dir / f"model_{i}.pt"

    # ------------------------------------------------------------------ labels
    def make_generator(self, solution, **overrides):
        """PicardDataModule.get_data_generator (picard/data.py:1465-1496) on the device path."""
        d = self.cfg.DATA
        kw = dict(dict(d.kwargs), hessian_approximation=d.HESSIAN_APPROXIMATION, sample_bound=d.SAMPLE_BOUND,
                  estimate_terminal=d.ESTIMATE_TERMINAL, estimate_integral=d.ESTIMATE_INTEGRAL,
                  estimate_delta_t=d.ESTIMATE_DELTA_T, n_euler_steps=d.EULER_STEPS, seed=d.SEED)
        kw.update(overrides)
        return OnlineDataGenerator(self.equation, solution, self.N, self.i, device=self.device, **kw)

    def label_sampler(self, gen):
        """The batch_data_generator get_dataset_details would pick (data.py:1620-1661): exact labels
        under DATA.EXACT, Monte-Carlo labels otherwise (MC-sharded over the ranks when world > 1)."""
        hess = self.supervise_hessian
        if self.cfg.DATA.EXACT:
            return gen.sample_exact_with_gradients_and_hessians if hess else gen.sample_exact_with_gradients
        src = gen
        if self.world > 1:
            src = ShardedLabeler(gen, self.rank, self.world, self.group)
        return src.sample_with_gradients_and_hessians if hess else src.sample_with_gradients

    def labels(self):
        gen = self.make_generator(self.u_current)
        d = self.cfg.DATA
        return LabelBuffer(self.label_sampler(gen), d.DATA_SIZE, d.POINTS_PER_CALL, guard=gen).fill()

    # ------------------------------------------------------------------ fit
    def fit(self, net, tx, y):
        """TRAIN.N_EPOCHS passes over the labels in BATCH_SIZE batches with the objective the
        reference's solution wrapper computes (fit.build_objective; losses pinned against the
        reference's training steps by tests/test_fit_golden.py).  As in the reference's data
        module, the first epoch takes the labels in the order they were drawn and later epochs
        replay the in-memory cache, shuffled when DATA.SHUFFLE is set (dataset.py:203-255)."""
        t = self.cfg.TRAIN
        objective, self.fit_kind = build_objective(t, self.equation.nx, self.supervise_gradient,
                                                   self.supervise_hessian)
        opt, sched = make_optimizer(net.parameters(), t.OPTIMIZER)
        n = tx.shape[0]
        bs = int(t.BATCH_SIZE) if t.BATCH_SIZE else n
        # When the training batch differs from the generation batch (points per generator call), the
        # reference re-batches through CacheToMemoryWrapper(batch_size, drop_last=True,
        # shuffle=SHUFFLE) and preloads it (picard/data.py:1718-1731), so even the first epoch comes
        # from the cache: shuffled under DATA.SHUFFLE and without the partial last batch.  Otherwise
        # the first epoch streams in draw order and later epochs replay the cache (data.py:1746-1760).
        rebatched = bs != min(int(self.cfg.DATA.POINTS_PER_CALL), n)
        shuffle = bool(self.cfg.DATA.SHUFFLE)
        losses = []
        for epoch in range(int(t.N_EPOCHS)):
            batches = TensorDatasetBuiltInShuffle(tx, y, batch_size=bs, drop_last=rebatched,
                                                  shuffle=shuffle and (epoch > 0 or rebatched))
            losses.append(train_steps(net, objective, opt, batches, sched))
        losses = torch.cat(losses) if losses else torch.empty(0)
        return float(losses[-1]) if losses.numel() else float("nan")

    # ------------------------------------------------------------------ eval
    def evaluate(self, net, n_points=None):
        """EvalCallback (picard/utils.py:329-478): at t = linspace(0, T, n) and x = equation.sample_x(t)
        (seeded per iteration), u of the network vs the exact solution; with EVAL.TEST_GRAD the
        gradient errors and with EVAL.TEST_HESSIAN the Hessian errors (at most 256 points for the
        nx^2 Hessians).  Returns the metrics dict, or {} when the equation has no exact solution."""
        import numpy as np
        ev = self.cfg.EVAL
        n = int(n_points or ev.L2_N_POINTS)
        eq = self.equation
        with torch.random.fork_rng(devices=[]):
            torch.manual_seed(int(self.cfg.DATA.SEED) * 7919 + self.i)
            t = torch.linspace(0.0, float(eq.T), n, dtype=torch.float64).reshape(n, 1)
            x = eq.sample_x(t).to(torch.float64)
        try:
            u_exact = eq.exact_solution(t, x)
        except (NotImplementedError, AttributeError):
            return {}
        dt = next(net.parameters()).dtype if any(True for _ in net.parameters()) else torch.float32
        tx = torch.cat([t, x], -1).to(device=self.device, dtype=dt)
        grads = bool(ev.TEST_GRAD)
        with torch.enable_grad() if grads else torch.no_grad():
            if grads:
                tx.requires_grad_(True)
            u = net(tx)
            ux = torch.autograd.grad(u.sum(), tx)[0][:, 1:] if grads else None
        out = {"u": u.detach().double().cpu().numpy(), "u_exact": u_exact.numpy()}
        if grads:
            out.update(ux=ux.double().cpu().numpy(), ux_exact=eq.u_x(t, x).detach().numpy())
            if ev.TEST_HESSIAN and hasattr(eq, "u_hessian"):
                k = min(n, 256)
                h = torch.func.vmap(torch.func.hessian(lambda z: net(z[None])[0, 0]))(tx[:k].detach())
                out.update(uxx=h[:, 1:, 1:].reshape(k, -1).double().cpu().numpy(),
                           uxx_exact=eq.u_hessian(t[:k], x[:k]).reshape(k, -1).numpy())
        m = eval_metrics(out["u"], out["u_exact"], out.get("ux"), out.get("ux_exact"))
        if "uxx" in out:
            m.update({k: v for k, v in eval_metrics(out["u"][:1], out["u_exact"][:1], out["uxx"],
                                                    out["uxx_exact"]).items() if k.endswith("h")})
        return m

    def save_labels(self, tx, y):
        """The reference's label file for this iteration: datasets `tx` and `u_ux` (`u_ux_uh` with
        Hessian labels) of DATA.FLOAT, one file for the one label producer (worker 0)."""
        import numpy as np
        from .h5 import H5Saver, data_file
        name = "u_ux_uh" if self.supervise_hessian else "u_ux"
        dtype = np.float64 if str(self.cfg.DATA.FLOAT).lower() in ("double", "float64") else np.float32
        saver = H5Saver(data_file(self.exp_dir, self.i, 0), tx.shape[0], [tx.shape[1], y.shape[1]], ["tx", name],
                        dtype)
        saver.save([tx, y], tx.shape[0])
        saver.close()

    # ------------------------------------------------------------------ loop
    def run_one(self):
        self.i += 1
        sync = (lambda: torch.cuda.synchronize(self.device)) if self.device.type == "cuda" else (lambda: None)
        sync()
        t0 = time.perf_counter()
        tx, y = self.labels()
        sync()
        t_labels = time.perf_counter() - t0
        net = self.new_network()
        rec = None
        err = None
        if self.rank == 0:
            try:
                rec = self._fit_and_record(net, tx, y, t_labels)
            except Exception as e:  # noqa: BLE001 — re-raised by _agree on this rank
                err = e
        self._agree(err, f"Picard iteration {self.i} (fit / checkpoint / evaluation on rank 0)")
        if self.world > 1:  # every rank continues from rank 0's fit
            import torch.distributed as dist
            for v in net.state_dict().values():
                dist.broadcast(v, src=0, group=self.group)
        self.u_current = net  # frozen by the next OnlineDataGenerator (data.py:409-412)
        return True

    def _fit_and_record(self, net, tx, y, t_labels):
        if self.cfg.DATA.SAVE:  # data_iter_{i}/split_00.h5 (picard/data.py:1510-1525, data_saver.py:24-56)
            self.save_labels(tx, y)
        if self.cfg.NETWORK.RELOAD and self.i > 1:  # picard_iteration.py:249-251
            net.load_state_dict(torch.load(self.checkpoint_path(self.i - 1), weights_only=True))
        t1 = time.perf_counter()
        loss = self.fit(net, tx, y)
        t_fit = time.perf_counter() - t1
        torch.save(net.state_dict(), self.checkpoint_path(self.i))
        metrics = self.evaluate(net)
        M = int(dict(self.cfg.DATA.kwargs).get("n_estimate_integral", 1))
        n = int(tx.shape[0])
        rec = {"iter": self.i, "labels": n, "label_s": t_labels, "labels_per_s": n / t_labels,
               "path_labels_per_s": None if self.cfg.DATA.EXACT else n * M / t_labels, "ranks": self.world,
               "fit_s": t_fit, "fit": self.fit_kind, "loss": loss, "rel_l2_u": metrics.get("rRMSE"), **metrics}
        self.history.append(rec)
        with open(self.exp_dir / "history.jsonl", "a") as f:
            f.write(json.dumps(rec) + "\n")
        print(json.dumps(rec), flush=True)
        return rec

    def run(self):
        for _ in range(self.N):
            if not self.run_one():
                break
        return self.history
