"""CPU baseline for bench.py (test / measurement infrastructure, never on the product path): the
reference's own label algorithm, vectorised in PyTorch on the host cores, as the reference runs it
on a CPU — `estimate_terminal_with_gradients` (picard/data.py:899-926) + `estimate_integral_with_
gradients` (:471-527) with `get_f` (:1226-1325): for ff(t, x, u, grad u) equations (Cha,
OUProcessEquation) u and grad u of the network by autograd; for the Hessian-term equation
(GBMEquationComplexExact) the SDGD branch of get_f (:1273-1303) — per path v indices drawn with
randint (:501), one autograd pass per index for u_ii, the baseline's whole diagonal (arange indices)
gathered per path.  One Gaussian jump per path (the reference's sampler, equations.py:217-230), the
per-point baseline f(t, x) evaluated once and repeated.

The equations and networks are the torch modules of deeppicarditeration_amd (the plugin interface),
evaluated on the CPU in fp32 or fp64; the noise is torch's CPU generator (as in the reference).
"""
import math
import os
import time

import torch


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota when one is set
    (a GPU box's share of a large host is a quota, not a smaller affinity mask)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def _u_grad(net, s, X):
    sx = torch.cat([s, X], -1).requires_grad_(True)
    with torch.enable_grad():
        u = net(sx)
        (g,) = torch.autograd.grad(u.sum(), sx, allow_unused=True) if u.requires_grad else (None,)
    if g is None:  # ZeroSolution: grad u := 0 (utils.py:80-94)
        g = torch.zeros_like(sx)
    return u.detach(), g[:, 1:]


def _u_grad_sdgd(net, s, X, idx):
    """u, grad u and u_ii at the columns idx (R, v) (get_f's SDGD loop, data.py:1273-1294; one
    autograd pass per index with create_graph as there)."""
    X = X.detach().requires_grad_(True)
    with torch.enable_grad():
        u = net(torch.cat([s, X], -1))
        (ux,) = torch.autograd.grad(u.sum(), X, create_graph=True, retain_graph=True)
        uii = torch.zeros(idx.shape, dtype=X.dtype)
        for i in range(idx.shape[1]):
            ai = idx[:, i:i + 1]
            (h,) = torch.autograd.grad(torch.gather(ux, 1, ai), X, grad_outputs=torch.ones_like(ai, dtype=X.dtype),
                                       create_graph=True, retain_graph=True)
            uii[:, i] = torch.gather(h, 1, ai).squeeze(1).detach()
    return u.detach(), ux.detach(), uii


def labels_reference_algorithm(eq, net, tx, M, gen, noise=None, v=None):
    """(n, 1+nx) labels for points tx (n, 1+nx), M paths each, in tx's dtype.  `noise` = (xi (R, nx),
    U (R, 1), zeta (R, nx)[, SDGD indices (R, v)]), R = n M, replaces the path draws (tests pin the
    algorithm against the reference's golden outputs this way).  v: SDGD samples per path for a
    Hessian-term equation (default nx)."""
    n, nx = tx.shape[0], eq.nx
    dt = tx.dtype
    T = float(eq.T)
    a = math.sqrt(float(eq.alpha))
    t = tx[:, :1].repeat_interleave(M, 0)
    x = tx[:, 1:].repeat_interleave(M, 0)
    ones = torch.ones(n * M, 1, dtype=dt)
    # terminal estimator (data.py:899-926)
    xi = torch.randn(n * M, nx, generator=gen, dtype=dt) if noise is None else noise[0]
    tau = torch.sqrt(T - t)
    gx = eq.g(tx[:, 1:])
    c = (eq.g(x + tau * a * xi) - gx.repeat_interleave(M, 0)) * torch.cat([ones, xi / tau / a], -1)
    y = c.view(n, M, 1 + nx).mean(1)
    y[:, :1] += gx
    # integral estimator (data.py:471-527, generate_sx_for_integral :350-366)
    U = torch.rand(n * M, 1, generator=gen, dtype=dt) if noise is None else noise[1]
    s = U * (T - t) + t
    zeta = torch.randn(n * M, nx, generator=gen, dtype=dt) if noise is None else noise[2]
    sig = torch.sqrt(s - t)
    Xs = x + sig * a * zeta
    if getattr(eq, "has_hessian_term", False):
        v = nx if v is None else v
        idx = torch.randint(0, nx, (n * M, v), generator=gen) if noise is None else noise[3]
        u, _, uii = _u_grad_sdgd(net, s, Xs, idx)
        f = eq.ffi(s, Xs, u, uii)
        # baseline (get_f with baseline_repeat, :1279-1302): the whole diagonal once per point,
        # repeated and gathered at each path's indices
        ub, _, uiib = _u_grad_sdgd(net, tx[:, :1], tx[:, 1:], torch.arange(nx).repeat(n, 1))
        fb = eq.ffi(t, x, ub.repeat_interleave(M, 0), torch.gather(uiib.repeat_interleave(M, 0), 1, idx))
    else:
        u, ux = _u_grad(net, s, Xs)
        f = eq.ff(s, Xs, u, ux)
        ub, uxb = _u_grad(net, tx[:, :1], tx[:, 1:])  # baseline once per point (get_f baseline_repeat)
        fb = eq.ff(tx[:, :1], tx[:, 1:], ub, uxb).repeat_interleave(M, 0)
    c = (T - t) * (f - fb) * torch.cat([ones, zeta / sig / a], -1)
    c[:, :1] += fb * (T - t)
    return y + c.view(n, M, 1 + nx).mean(1)


def _f_full_hessian(eq, net, s, X):
    """f with the full Hessian of u (get_f without a Hessian approximation, data.py:1259-1272: one
    autograd pass per state dimension, create_graph as there; ZeroSolution: zero derivatives)."""
    X = X.detach().requires_grad_(True)
    nx = X.shape[1]
    with torch.enable_grad():
        u = net(torch.cat([s, X], -1))
        ux = torch.autograd.grad(u.sum(), X, create_graph=True, allow_unused=True)[0] if u.requires_grad else None
        if ux is None:
            ux = torch.zeros_like(X)
            hess = torch.zeros(X.shape[0], nx, nx, dtype=X.dtype)
        else:
            hess = torch.zeros(X.shape[0], nx, nx, dtype=X.dtype)
            for i in range(nx):
                (h,) = torch.autograd.grad(ux[:, i], X, grad_outputs=torch.ones_like(ux[:, i]), create_graph=True)
                hess[:, i, :] = h.detach()
    return eq.ffh(s, X.detach(), u.detach(), ux.detach(), hess)


def labels_hessians_reference_algorithm(eq, net, tx, M, gen, noise=None):
    """(n, 1+nx+nx^2) Malliavin Hessian labels of generate_with_gradients_and_hessians: the terminal
    (data.py:1153-1201) and integral (:823-897) _double estimators, each with its two half-step
    rollout, for an equation with a full-Hessian nonlinearity (GBMEquationComplexExact).  `noise` =
    (terminal dW1, dW2, N1, U, integral dW1, dW2, N2), R = n M rows each (make_golden.py's draw order)."""
    n, nx = tx.shape[0], eq.nx
    dt = tx.dtype
    T = float(eq.T)
    a = math.sqrt(float(eq.alpha))
    R = n * M
    draw = iter(noise) if noise is not None else None

    def rn():
        return next(draw) if draw is not None else torch.randn(R, nx, generator=gen, dtype=dt)

    t = tx[:, :1].repeat_interleave(M, 0)
    x = tx[:, 1:].repeat_interleave(M, 0)
    ones = torch.ones(R, 1, dtype=dt)
    eye = torch.eye(nx, dtype=dt)
    # terminal
    t_mid = (T + t) / 2
    Xm = x + torch.sqrt(t_mid - t) * a * rn()
    XT = Xm + torch.sqrt(T - t_mid) * a * rn()
    Y = (XT - x) / torch.sqrt(T - t) / a / torch.sqrt(T - t)
    g_single = eq.g(tx[:, 1:])
    g = g_single.repeat_interleave(M, 0)
    term = ((eq.g(XT) - g) * torch.cat([ones, Y], -1)).view(n, M, -1).mean(1)
    term[:, :1] += g_single
    W1 = torch.sqrt(T - t) * rn()
    dg = (eq.g(x + a * W1) + eq.g(x - a * W1) - 2 * g) / 2 / (T - t)
    p1 = ((dg / (T - t)).unsqueeze(-1) * torch.einsum("ij,ik->ijk", W1, W1)).view(n, M, -1).mean(1)
    p2 = dg.view(n, M, 1).mean(1, keepdim=True) * eye.reshape(1, 1, nx * nx)
    term_h = p1 - p2.view(n, -1)
    # integral
    U = next(draw) if draw is not None else torch.rand(R, 1, generator=gen, dtype=dt)
    s = U * (T - t) + t + 0.0001
    sm = (s + t) / 2
    Xm = x + torch.sqrt(sm - t) * a * rn()
    Xs = Xm + torch.sqrt(s - sm) * a * rn()
    Ys = (Xs - x) / torch.sqrt(s - t) / a / torch.sqrt(s - t)
    fb_single = _f_full_hessian(eq, net, tx[:, :1], tx[:, 1:])
    fb = fb_single.repeat_interleave(M, 0)
    tt = tx[:, :1]
    intg = ((T - t) * (_f_full_hessian(eq, net, s, Xs) - fb) * torch.cat([ones, Ys], -1)).view(n, M, -1).mean(1)
    intg[:, :1] += fb_single * (T - tt)
    W2 = torch.sqrt(s - t) * rn()
    df = (_f_full_hessian(eq, net, s, x + a * W2) + _f_full_hessian(eq, net, s, x - a * W2) - 2 * fb) / 2 / (s - t)
    p1 = ((df / (s - t)).unsqueeze(-1) * torch.einsum("ij,ik->ijk", W2, W2)).view(n, M, -1).mean(1)
    p2 = df.view(n, M, 1).mean(1, keepdim=True) * eye.reshape(1, 1, nx * nx)
    intg_h = (p1 - p2.view(n, -1)) * (T - tt)
    return torch.cat([term + intg, term_h + intg_h], -1)


def time_reference_algorithm(eq, net, sample_points, M, dtype, target_s=8.0, points_per_call=4, threads=None, v=None,
                             hessians=False):
    """path-labels/s of labels_reference_algorithm on `threads` host threads for ~target_s seconds."""
    threads = threads or host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    net = net.to(dtype)
    gen = torch.Generator().manual_seed(0)
    done = calls = 0
    try:
        label = ((lambda tx: labels_hessians_reference_algorithm(eq, net, tx, M, gen)) if hessians
                 else (lambda tx: labels_reference_algorithm(eq, net, tx, M, gen, v=v)))
        label(sample_points(points_per_call, 0).to(dtype))  # warm-up
        t0 = time.perf_counter()
        while True:
            tx = sample_points(points_per_call, calls * points_per_call).to(dtype)
            # (no finiteness check: in fp32 the reference's s - t rounds to 0 for tiny U, giving inf)
            label(tx)
            done += points_per_call * M
            calls += 1
            dt = time.perf_counter() - t0
            if dt >= target_s:
                break
    finally:
        torch.set_num_threads(prev)
    return done / dt, calls * points_per_call, dt, threads
