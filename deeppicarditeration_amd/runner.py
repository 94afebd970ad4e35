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

import torch

from . import equations as eqs
from .config import CfgNode
from .data import OnlineDataGenerator
from .solution import PISGradNet, ZeroSolution, construct_mlp


class LabelBuffer:
    """Device-resident (tx, y) label store for one Picard iteration; y is (u, u_x) or, with
    hessians=True, (u, u_x, u_xx) of generate_with_gradients_and_hessians (data.py:225-237)."""

    def __init__(self, gen, n_total, points_per_call, hessians=False):
        self.gen = gen
        self.n_total = int(n_total)
        self.ppc = max(1, min(int(points_per_call), self.n_total))
        self.sample = gen.sample_with_gradients_and_hessians if hessians else gen.sample_with_gradients

    def fill(self):
        txs, ys = [], []
        done = 0
        while done < self.n_total:
            n = min(self.ppc, self.n_total - done)
            tx, y = self.sample(n)
            txs.append(tx)
            ys.append(y)
            done += n
        return torch.cat(txs), torch.cat(ys)


class PicardRunner:
    def __init__(self, cfg: CfgNode, device="cuda"):
        self.cfg = cfg
        self.device = torch.device(device)
        self.exp_dir = pathlib.Path(cfg.NAME)
        if self.exp_dir.exists() and any(self.exp_dir.iterdir()):
            if not cfg.FORCE:
                raise FileExistsError(f"Experiment directory {self.exp_dir} already exists.")
            shutil.rmtree(self.exp_dir)
        self.exp_dir.mkdir(parents=True, exist_ok=True)
        (self.exp_dir / "config.yaml").write_text(cfg.dump())
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
    def labels(self):
        d = self.cfg.DATA
        kw = dict(d.kwargs)
        gen = OnlineDataGenerator(
            self.equation, self.u_current, self.N, self.i, device=self.device, **kw,
            hessian_approximation=d.HESSIAN_APPROXIMATION, sample_bound=d.SAMPLE_BOUND,
            estimate_terminal=d.ESTIMATE_TERMINAL, estimate_integral=d.ESTIMATE_INTEGRAL,
            estimate_delta_t=d.ESTIMATE_DELTA_T, n_euler_steps=d.EULER_STEPS, seed=d.SEED)
        return LabelBuffer(gen, d.DATA_SIZE, d.POINTS_PER_CALL, hessians=self.supervise_hessian).fill()

    # ------------------------------------------------------------------ fit
    def fit(self, net, tx, y):
        t = self.cfg.TRAIN
        opt = getattr(torch.optim, t.OPTIMIZER.cls)(net.parameters(), **dict(t.OPTIMIZER.kwargs))
        beta = float(t.LOSS.beta)
        loss_fn = torch.square
        if t.LOSS.FN.cls is not None:  # LossFnLinearClip (solution.py:22-33)
            clip = float(t.LOSS.FN.kwargs["clip"])
            loss_fn = lambda x: torch.where(x.abs() < clip, x * x, 2 * clip * x.abs() - clip ** 2)  # noqa: E731
        gw, hw = 0.0, 0.0
        kw = t.LOSS.SCALER.kwargs
        if self.supervise_hessian:  # FixedHessianLossScaler (solution_jac.py:85-109)
            if t.LOSS.SCALER.cls != "FixedHessianLossScaler":
                raise NotImplementedError("SUPERVISE_HESSIAN needs LOSS.SCALER.cls = FixedHessianLossScaler")
            gw, hw = float(kw["fixed_gradient_weight"]), float(kw["fixed_hessian_weight"])
        elif self.supervise_gradient and t.LOSS.SCALER.cls == "FixedLossScaler":
            gw = float(kw.get("fixed_weight", 0.0))
        elif self.supervise_gradient and t.LOSS.SCALER.cls is not None:
            raise NotImplementedError(f"loss scaler {t.LOSS.SCALER.cls}")
        nx = self.equation.nx
        n_hess_samples = int(t.NUM_HESS_SAMPLES)
        hess_fn = None
        if self.supervise_hessian:  # vmap(hessian(forward)) (solution_jac.py:128)
            hess_fn = torch.func.vmap(torch.func.hessian(lambda z: net(z[None])[0, 0]))
        n = tx.shape[0]
        bs = int(t.BATCH_SIZE) if t.BATCH_SIZE else n
        last = float("nan")
        for _ in range(int(t.N_EPOCHS)):
            perm = torch.randperm(n, device=tx.device)
            for b0 in range(0, n, bs):
                idx = perm[b0:b0 + bs]
                xb, yb = tx[idx].detach(), y[idx]
                w = torch.exp(xb[:, :1] * beta)
                if self.supervise_hessian:  # PicardSolutionGradientHessianWrapper (solution_jac.py:219-259)
                    xb.requires_grad_(True)
                    u = net(xb)
                    ux = torch.autograd.grad(u.sum(), xb, create_graph=True)[0][:, 1:]
                    uh = hess_fn(xb)[:, 1:, 1:].reshape(xb.shape[0], nx * nx)
                    diff = uh - yb[:, 1 + nx:]
                    if n_hess_samples > 0:
                        idx_h = torch.randperm(nx * nx, device=xb.device)[:n_hess_samples]
                        diff = diff[:, idx_h]
                    v_loss = torch.mean(w * loss_fn(u - yb[:, :1]))
                    g_loss = torch.mean(w * loss_fn(ux - yb[:, 1:1 + nx]), dim=0).sum()
                    h_loss = torch.mean(w * loss_fn(diff), dim=0).sum()
                    loss = v_loss + gw * g_loss + hw * h_loss
                elif gw > 1e-9:  # PicardSolutionGradientWrapper (solution_jac.py:167-213)
                    xb.requires_grad_(True)
                    u = net(xb)
                    ux = torch.autograd.grad(u.sum(), xb, create_graph=True)[0][:, 1:]
                    v_loss = torch.mean(w * loss_fn(u - yb[:, :1]))
                    g_loss = torch.mean(w * loss_fn(ux - yb[:, 1:1 + nx]), dim=0).sum()
                    loss = v_loss + gw * g_loss
                else:  # PicardBaseSolution.training_step (solution.py:75-82)
                    loss = torch.mean(w * loss_fn(net(xb) - yb[:, :1]))
                opt.zero_grad(set_to_none=True)
                loss.backward()
                opt.step()
                last = float(loss.detach())
        return last

    # ------------------------------------------------------------------ eval
    def evaluate(self, net, n_points=None):
        """rel-L2 of u against the exact solution on freshly sampled points (utils.py:410-476)."""
        n = int(n_points or min(self.cfg.EVAL.L2_N_POINTS, 4096))
        gen = OnlineDataGenerator(self.equation, ZeroSolution(1), self.N, self.i, device=self.device,
                                  t_always_uniform=True, n_estimate_terminal=64, n_estimate_integral=64,
                                  n_euler_steps=1, seed=self.cfg.DATA.SEED + 7919, epoch=0xFFFFFF - self.i)
        tx, _ = gen.sample_t_and_x(n)
        t, x = tx[:, :1].double().cpu(), tx[:, 1:].double().cpu()
        try:
            exact = self.equation.exact_solution(t, x)
        except (NotImplementedError, AttributeError):
            return None
        with torch.no_grad():
            u = net(tx).double().cpu()
        return float(torch.linalg.norm(u - exact) / torch.linalg.norm(exact))

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
        t0 = time.perf_counter()
        tx, y = self.labels()
        torch.cuda.synchronize(self.device)
        t_labels = time.perf_counter() - t0
        if self.cfg.DATA.SAVE:  # data_iter_{i}/split_00.h5 (picard/data.py:1510-1525, data_saver.py:24-56)
            self.save_labels(tx, y)
        net = self.new_network()
        if self.cfg.NETWORK.RELOAD and self.i > 1:  # picard_iteration.py:249-251
            net.load_state_dict(torch.load(self.checkpoint_path(self.i - 1), weights_only=True))
        t1 = time.perf_counter()
        loss = self.fit(net, tx, y)
        t_fit = time.perf_counter() - t1
        torch.save(net.state_dict(), self.checkpoint_path(self.i))
        rel = self.evaluate(net)
        rec = {"iter": self.i, "labels": int(tx.shape[0]), "label_s": t_labels, "fit_s": t_fit, "loss": loss,
               "rel_l2_u": rel}
        self.history.append(rec)
        with open(self.exp_dir / "history.jsonl", "a") as f:
            f.write(json.dumps(rec) + "\n")
        print(json.dumps(rec), flush=True)
        self.u_current = net  # frozen by the next OnlineDataGenerator (data.py:409-412)
        return True

    def run(self):
        for _ in range(self.N):
            if not self.run_one():
                break
        return self.history
