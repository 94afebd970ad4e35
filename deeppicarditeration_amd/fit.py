"""The outer fit's objectives — what the reference's solution wrappers compute per training batch
(SURVEY.md §8f rank 3).  PyTorch-ROCm, not HIP: the fit consumes the device-resident labels.

- `value_objective`: PicardBaseSolution.training_step (picard/solution.py:74-81), the exp(beta t)
  weighted value loss;
- `gradient_objective`: PicardSolutionGradientWrapper.training_step (picard/solution_jac.py:167-213)
  for a value network (output_dim 1): value loss plus the per-dimension gradient losses, combined
  by a loss scaler;
- `gradient_hessian_objective`: PicardSolutionGradientHessianWrapper.training_step
  (solution_jac.py:219-259), plus the Hessian losses (all nx^2 entries, or NUM_HESS_SAMPLES of them
  drawn with `random.sample` as there);
- the loss scalers of solution_jac.py:13-109 and LossFnLinearClip (solution.py:22-33);
- `build_objective`: the wrapper choice of PicardRunner.get_solution (picard_iteration.py:113-118)
  and PicardSolutionGradientWrapper.construct_solution / __init__ (solution_jac.py:112-136).

Each objective is `f(net, tx, y) -> (loss (1,), info dict)`; `net` maps tx (B, 1+nx) -> (B, 1).
"""
import random

import torch


class LossFnLinearClip(torch.nn.Module):
    """solution.py:22-33: x^2 inside |x| < clip, continued linearly (C^1) outside."""

    def __init__(self, clip: float):
        super().__init__()
        self.clip = torch.scalar_tensor(clip)

    def forward(self, x):
        c = self.clip.to(x)
        return torch.where(torch.abs(x) < c, torch.square(x), 2 * c * torch.abs(x) - c ** 2)


def make_loss_fn(fn_cfg):
    """TRAIN.LOSS.FN (solution.py:62-68): None -> square, otherwise LossFnLinearClip(kwargs.clip)."""
    if fn_cfg is None or fn_cfg.get("cls") is None:
        return torch.square
    return LossFnLinearClip(float(fn_cfg["kwargs"]["clip"]))


class LossScaler:
    """solution_jac.py:13-36.  `scale` combines (v_loss (1,), g_loss (nx,)); `scale_g_h` also
    h_loss (nx^2 or NUM_HESS_SAMPLES,).  Both return (total (1,), info)."""

    registry = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        LossScaler.registry[cls.__name__] = cls

    @classmethod
    def get_class(cls, name):
        try:
            return cls.registry[name]
        except KeyError:
            raise ValueError(f"unknown loss scaler {name!r} (known: {sorted(cls.registry)})") from None

    def scale(self, v_loss, g_loss_multi_dim):
        raise NotImplementedError(f"{type(self).__name__} does not scale value + gradient losses")

    def scale_g_h(self, v_loss, g_loss_multi_dim, h_loss_multi_dim):
        raise NotImplementedError(f"{type(self).__name__} does not scale value + gradient + Hessian losses")


class SimpleLossScaler(LossScaler):
    """solution_jac.py:39-50: one weight a = clamp(v / sum g, 0, 1e3).  As there, the summed
    gradient loss is formed under no_grad too, so it adds to the reported loss but not to the
    parameter gradient (kept for parity; tests/golden/fit_grad_clip_simple.npz pins it)."""

    def scale(self, v_loss, g_loss_multi_dim):
        with torch.no_grad():
            g_loss = torch.sum(g_loss_multi_dim, keepdim=True, dim=-1)
            a = torch.clamp(v_loss / g_loss, min=0.0, max=1e3)
        return v_loss + a * g_loss, {"train_gradient_loss(unscaled)": g_loss, "train_gradient_loss_scaling_factor": a}


class DimensionLossScaler(LossScaler):
    """solution_jac.py:53-68: a weight per dimension, a_d = clamp(v / g_d, 0, 1e3)."""

    def scale(self, v_loss, g_loss_multi_dim):
        with torch.no_grad():
            a = torch.clamp(v_loss / g_loss_multi_dim, min=0.0, max=1e3)
            mean_a = torch.mean(a, dim=0)
        g_loss = torch.sum(a * g_loss_multi_dim, keepdim=True, dim=-1)
        return v_loss + g_loss, {"train_gradient_loss(unscaled)": g_loss, "train_gradient_loss_scaling_factor": mean_a}


class FixedLossScaler(LossScaler):
    """solution_jac.py:71-82."""

    def __init__(self, fixed_weight: float):
        self.fixed_weight = fixed_weight

    def scale(self, v_loss, g_loss_multi_dim):
        g_loss = torch.sum(g_loss_multi_dim, keepdim=True, dim=-1)
        return v_loss + self.fixed_weight * g_loss, {"train_gradient_loss(unscaled)": g_loss}

    def __str__(self):
        return f"FixedLossScaler(fixed_weight={self.fixed_weight})"


class FixedHessianLossScaler(LossScaler):
    """solution_jac.py:85-109."""

    def __init__(self, fixed_gradient_weight: float, fixed_hessian_weight: float):
        self.fixed_gradient_weight = fixed_gradient_weight
        self.fixed_hessian_weight = fixed_hessian_weight

    def scale_g_h(self, v_loss, g_loss_multi_dim, h_loss_multi_dim):
        g_loss = torch.sum(g_loss_multi_dim, keepdim=True, dim=-1)
        h_loss = torch.sum(h_loss_multi_dim, keepdim=True, dim=-1)
        return (v_loss + self.fixed_gradient_weight * g_loss + self.fixed_hessian_weight * h_loss,
                {"train_gradient_loss(unscaled)": g_loss, "train_hessian_loss(unscaled)": h_loss})

    def __str__(self):
        return (f"FixedHessianLossScaler(fixed_gradient_weight={self.fixed_gradient_weight},"
                f" fixed_hessian_weight={self.fixed_hessian_weight})")


def _weight(tx, beta):
    return torch.exp(torch.narrow(tx, -1, 0, 1) * beta)


def _u_and_grad(net, tx):
    """u (B, 1) and d u / d tx (B, 1+nx) — the per-row Jacobian of a value network (the reference's
    vmap(jacrev(forward)), solution_jac.py:121), as one reverse pass over the batch sum with the
    graph kept for the parameter gradient."""
    tx = tx.detach().requires_grad_(True)
    with torch.enable_grad():
        u = net(tx)
        (u_tx,) = torch.autograd.grad(u.sum(), tx, create_graph=True)
    return u, u_tx


def value_objective(beta, loss_fn):
    def objective(net, tx, y):
        loss = torch.mean(_weight(tx, beta) * loss_fn(net(tx) - y[:, :1]), dim=0)
        return loss, {}
    return objective


def gradient_objective(beta, loss_fn, scaler, nx):
    def objective(net, tx, y):
        u, u_tx = _u_and_grad(net, tx)
        w = _weight(tx, beta)
        v_loss = torch.mean(w * loss_fn(u - y[:, :1]), dim=0)
        g_loss = torch.mean(w * loss_fn(u_tx[:, 1:] - y[:, 1:1 + nx]), dim=0)
        loss, info = scaler.scale(v_loss, g_loss)
        info["train_value_loss"] = v_loss
        return loss, info
    return objective


def gradient_hessian_objective(beta, loss_fn, scaler, nx, num_hess_samples=-1):
    def objective(net, tx, y):
        u, u_tx = _u_and_grad(net, tx)
        w = _weight(tx, beta)
        v_loss = torch.mean(w * loss_fn(u - y[:, :1]), dim=0)
        g_loss = torch.mean(w * loss_fn(u_tx[:, 1:] - y[:, 1:1 + nx]), dim=0)
        hess = torch.func.vmap(torch.func.hessian(lambda z: net(z[None])[0, 0]))(tx)  # (B, 1+nx, 1+nx)
        diff = hess[:, 1:, 1:].reshape(tx.shape[0], nx * nx) - y[:, 1 + nx:1 + nx + nx * nx]
        if num_hess_samples > 0:  # solution_jac.py:246-249 (python's global `random`, as there)
            idx = torch.tensor(random.sample(range(nx * nx), num_hess_samples), dtype=torch.long, device=y.device)
            diff = torch.index_select(diff, 1, idx)
        h_loss = torch.mean(w * loss_fn(diff), dim=0)
        loss, info = scaler.scale_g_h(v_loss, g_loss, h_loss)
        info["train_value_loss"] = v_loss
        return loss, info
    return objective


def make_scaler(scaler_cfg):
    """solution_jac.py:132-136: no SCALER.cls means FixedLossScaler(1.0)."""
    if scaler_cfg is None or scaler_cfg.get("cls") is None:
        return FixedLossScaler(1.0)
    return LossScaler.get_class(scaler_cfg["cls"])(**dict(scaler_cfg.get("kwargs") or {}))


def build_objective(train_cfg, nx, supervise_gradient, supervise_hessian):
    """PicardRunner.get_solution (picard_iteration.py:113-118) + the wrappers' construct_solution
    (solution_jac.py:112-119): returns (objective, kind) with kind in {"value", "gradient",
    "gradient_hessian"}.  A FixedLossScaler of weight <= 1e-9 falls back to the plain value fit."""
    loss_cfg = train_cfg["LOSS"]
    beta = float(loss_cfg["beta"])
    loss_fn = make_loss_fn(loss_cfg.get("FN"))
    if not (supervise_gradient or supervise_hessian):
        return value_objective(beta, loss_fn), "value"
    if loss_cfg.get("use_aux_loss"):
        raise NotImplementedError("TRAIN.LOSS.use_aux_loss applies to ValueGradient networks only")
    scaler = make_scaler(loss_cfg.get("SCALER"))
    if isinstance(scaler, FixedLossScaler) and scaler.fixed_weight <= 1e-9:
        return value_objective(beta, loss_fn), "value"
    if supervise_hessian:
        n_h = int(train_cfg.get("NUM_HESS_SAMPLES", -1) or -1)
        if n_h > nx * nx:
            raise AssertionError(f"NUM_HESS_SAMPLES {n_h} > nx^2")
        if not isinstance(scaler, FixedHessianLossScaler):
            raise NotImplementedError(f"{scaler} has no scale_g_h: SUPERVISE_HESSIAN needs FixedHessianLossScaler")
        return gradient_hessian_objective(beta, loss_fn, scaler, nx, n_h), "gradient_hessian"
    return gradient_objective(beta, loss_fn, scaler, nx), "gradient"


def make_optimizer(params, opt_cfg):
    """PicardBaseSolution.configure_optimizers (solution.py:94-126): torch.optim.<cls>(**kwargs) and
    an optional per-step torch.optim.lr_scheduler.<cls> (ReduceLROnPlateau: patience 512 unless
    given, stepped on the training loss)."""
    opt = getattr(torch.optim, opt_cfg["cls"])(params, **dict(opt_cfg.get("kwargs") or {}))
    sched_cfg = opt_cfg.get("SCHEDULER") or {}
    sched = None
    if sched_cfg.get("cls") is not None:
        cls = getattr(torch.optim.lr_scheduler, sched_cfg["cls"])
        kws = {"patience": 512} if cls is torch.optim.lr_scheduler.ReduceLROnPlateau else {}
        kws.update(dict(sched_cfg.get("kwargs") or {}))
        sched = cls(opt, **kws)
    return opt, sched


def train_steps(net, objective, opt, batches, sched=None):
    """One optimizer step per (tx, y) batch, in the order Lightning's automatic optimisation runs
    them (training_step, zero_grad, backward, step, then the step-interval scheduler); returns the
    per-step losses as a device tensor (no host synchronisation per step)."""
    losses = []
    for tx, y in batches:
        loss, _ = objective(net, tx, y)
        opt.zero_grad()
        loss.sum().backward()
        opt.step()
        if sched is not None:
            if isinstance(sched, torch.optim.lr_scheduler.ReduceLROnPlateau):
                sched.step(loss.detach().sum())
            else:
                sched.step()
        losses.append(loss.detach().reshape(()))
    return torch.stack(losses) if losses else torch.empty(0)
