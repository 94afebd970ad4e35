"""TEST INFRASTRUCTURE ONLY — CPU oracle for the DPI label-generation hot path.

A numpy (fp64 by default) restatement of the reference estimator, used by `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg as the checker. It is never
imported by the product package (`deeppicarditeration_amd/`), which fails loudly when its
HIP library is missing.

Pinned by the golden vectors in `tests/golden/` (generated from the reference itself with
injected Philox noise by `tests/golden/make_golden.py`) — see tests/test_oracle_golden.py.

Reference map (all paths relative to /root/reference):
  sample_points         picard/data.py:211-223 (sample_with_gradients), :161-167 (t sampler),
                        picard/equations.py:118-124, :217-230 (sample_x / sample_x_ts)
  terminal estimator    picard/data.py:899-926 (estimate_terminal_with_gradients)
  integral estimator    picard/data.py:471-527 (estimate_integral_with_gradients), :350-366
  TD estimators         picard/data.py:1209-1213 (ESTIMATE_DELTA_T > 0): :934-952
                        (estimate_terminal_with_gradients_td), :529-575 (..._integral_..._td)
  get_f                 picard/data.py:1226-1325
  Cha                   picard/equations.py:266-338
  OUProcessEquation     picard/equations.py:489-714 + picard/utils.py:792-880 (GMM)
  GBMEquationComplexExact picard/equations.py:388-486
  construct_mlp         picard/solution.py:123-135 ; PISGradNet picard/solution.py:138-289
  ZeroSolution          picard/solution.py:330-337 (u = 0, grad u := 0, data.py:1316)

The EM rollout: the reference draws ONE Gaussian jump per path (equations.py:225); the north
star asks for K Euler–Maruyama steps.  For the zero-drift SDE dX = sqrt(alpha) dW of every
shipped equation, the K-step endpoint is x + sqrt(alpha) * sqrt(h) * sum_k xi_k (h = (tau-t)/K),
which equals the reference's jump when it is fed xi_eff = sum_k xi_k / sqrt(K).
"""
import math

import numpy as np

from . import philox as px

EPS_T = 0.01  # picard/data.py:134-135 (default ESTIMATE_TERMINAL "OU_ByGx" contains "ByGx")


# ----------------------------------------------------------------------------- equations
class Cha:
    """picard/equations.py:266-338 (Burgers-type, k' = k/sqrt(nx))."""

    has_gradient_term = True
    has_hessian_term = False

    def __init__(self, nx, alpha, k=1.0, T=1.0):
        self.nx, self.alpha, self.T = nx, float(alpha), float(T)
        self.alpha_sqrt = math.sqrt(self.alpha)
        self.k = k / math.sqrt(nx)                      # :285
        self.alpha_d = self.alpha * nx
        self.k_alpha_d = self.k * self.alpha_d
        self.k_alpha_d_2 = 2 * self.k_alpha_d
        self.k2_alpha_d = self.k * self.k_alpha_d

    def sample_x0(self, n, **kw):                       # :334-335
        return np.zeros((n, self.nx))

    def g(self, x):                                     # :304-305
        return 1.0 / (1.0 + np.exp(-(self.T + self.k * x.sum(-1, keepdims=True))))

    def ff(self, t, x, y, ux):                          # :199-200 -> :297-302
        z = self.alpha_sqrt * ux
        return self.alpha_sqrt * (self.k * y - (2 + self.k2_alpha_d) / self.k_alpha_d_2) * z.sum(-1, keepdims=True)

    def exact(self, t, x):                              # :318-319
        return 1.0 / (1.0 + np.exp(-(t + self.k * x.sum(-1, keepdims=True))))

    def exact_grad(self, t, x):                         # :325-327
        u = self.exact(t, x)
        return np.ones_like(x) * (self.k * u * (1 - u))


class OUProcessEquation:
    """picard/equations.py:489-714; g = -log GMM(x) with diagonal covariances (utils.py:852-880)."""

    has_gradient_term = True
    has_hessian_term = False

    def __init__(self, nx, mean, var_diag, pi, alpha=1.0, T=1.0, theta=1.0, mu=0.0, alpha_scale=4.0):
        self.nx, self.alpha, self.T = nx, float(alpha), float(T)
        self.alpha_sqrt = math.sqrt(self.alpha)
        self.theta, self.mu = float(theta), float(mu)
        self.d = float(nx)
        self.mean = np.asarray(mean, np.float64)          # (K, nx)
        self.var = np.asarray(var_diag, np.float64)       # (K, nx)
        self.pi = np.asarray(pi, np.float64)              # (K,)
        self.alpha_init = alpha_scale * self.alpha        # :554
        self.log_2pi = math.log(2 * math.pi)
        self.norm = -0.5 * (nx * self.log_2pi + np.log(np.prod(self.var, axis=1)))  # utils.py:870

    def sample_x0(self, n, z=None):                      # :612-614, :710-711 ; utils.py:785-789
        return math.sqrt(self.alpha_init) * z

    def log_prob(self, x):
        diff = x[:, None, :] - self.mean[None]
        e = -0.5 * np.einsum("bkn,kn->bk", diff ** 2, 1.0 / self.var)
        lp = np.log(self.pi)[None] + self.norm[None] + e
        mx = lp.max(1, keepdims=True)
        return (mx + np.log(np.exp(lp - mx).sum(1, keepdims=True)))

    def grad_log_prob(self, x):                          # utils.py:882-914
        diff = x[:, None, :] - self.mean[None]
        e = -0.5 * np.einsum("bkn,kn->bk", diff ** 2, 1.0 / self.var)
        lp = np.log(self.pi)[None] + self.norm[None] + e
        mx = lp.max(1, keepdims=True)
        w = np.exp(lp - mx)
        w = w / w.sum(1, keepdims=True)
        return np.einsum("bk,bkn->bn", w, -diff / self.var[None])

    def g(self, x):                                      # :592-593
        return -self.log_prob(x)

    def ff(self, t, x, y, z):                            # :660-666 (z = grad u, unscaled)
        F = self.theta * (self.mu - x)
        return (-(F * z).sum(-1, keepdims=True) - self.alpha / 2 * (z ** 2).sum(-1, keepdims=True)
                - self.d * self.theta * np.ones_like(y))


class GBMEquationComplexExact:
    """picard/equations.py:388-486 (fully-nonlinear case_1); w (2, 1+nx), v (2, 1)."""

    has_gradient_term = True
    has_hessian_term = True

    def __init__(self, nx, w, v, alpha=1.0, T=1.0):
        self.nx, self.alpha, self.T = nx, float(alpha), float(T)
        self.alpha_sqrt = math.sqrt(self.alpha)
        self.d = float(nx)
        self.w = np.asarray(w, np.float64)
        self.v = np.asarray(v, np.float64)

    def sample_x0(self, n, **kw):                        # :485-486
        return np.zeros((n, self.nx))

    def _arg(self, t, x):
        t = np.broadcast_to(np.asarray(t, np.float64).reshape(-1, 1), (x.shape[0], 1))
        return np.concatenate([t, x], -1) @ self.w.T      # (B, 2)

    def exact(self, t, x):                               # :427-430
        return np.sin(self._arg(t, x)) @ self.v

    def g(self, x):                                      # :422-423
        return self.exact(self.T, x)

    def u_t(self, t, x):                                 # :432-434
        return np.cos(self._arg(t, x)) @ (self.v * self.w[:, 0:1])

    def laplacian(self, t, x):                           # :452-455
        return -np.sin(self._arg(t, x)) @ (self.v * (self.w[:, 1:] ** 2).sum(-1, keepdims=True))

    def hess_diag(self, t, x):                           # diag of :444-449
        return -np.sin(self._arg(t, x)) @ (self.v * self.w[:, 1:] ** 2)   # (B, nx)

    def ffi(self, t, x, u, u_ii):                        # :457-466
        lap = self.d * u_ii.mean(-1, keepdims=True)
        nonlin = self.d * np.abs(u_ii).mean(-1, keepdims=True)
        return (0.5 * (1.0 - self.alpha) * lap + 0.25 * nonlin - self.u_t(t, x)
                - 0.5 * self.laplacian(t, x) - 0.25 * np.abs(self.hess_diag(t, x)).sum(-1, keepdims=True))


# ----------------------------------------------------------------------------- networks
def _act(name, z):
    if name == "ELU":
        a = np.where(z > 0, z, np.expm1(np.minimum(z, 0)))
        d1 = np.where(z > 0, 1.0, np.exp(np.minimum(z, 0)))
        d2 = np.where(z > 0, 0.0, np.exp(np.minimum(z, 0)))
    elif name == "Tanh":
        a = np.tanh(z)
        d1 = 1 - a * a
        d2 = -2 * a * d1
    else:
        raise ValueError(name)
    return a, d1, d2


class MLP:
    """construct_mlp (picard/solution.py:123-135): Linear->act ... ->Linear; weights (out, in)."""

    def __init__(self, weights, biases, acts):
        self.W = [np.asarray(w, np.float64) for w in weights]
        self.b = [np.asarray(b, np.float64) for b in biases]
        self.acts = list(acts)

    def value_grad(self, tx, need_hdiag=False):
        """u (B,1), grad wrt input (B, 1+nx), optional diag of the x-Hessian (B, nx)."""
        a = tx
        d1s = []
        d2s = []
        hs = []
        for W, b, act in zip(self.W[:-1], self.b[:-1], self.acts):
            z = a @ W.T + b
            a, d1, d2 = _act(act, z)
            d1s.append(d1)
            d2s.append(d2)
            hs.append(a)
        u = a @ self.W[-1].T + self.b[-1]
        delta = np.broadcast_to(self.W[-1][0], a.shape).copy()
        for l in range(len(d1s) - 1, -1, -1):
            delta = (delta * d1s[l]) @ self.W[l]
        hd = None
        if need_hdiag:
            # forward-mode second order along each x-direction e_d (columns 1..nx of the input)
            B = tx.shape[0]
            dz = np.broadcast_to(self.W[0][:, 1:][None], (B,) + self.W[0][:, 1:].shape)  # (B,H,nx)
            d2z = np.zeros_like(dz)
            for l in range(len(d1s)):
                if l > 0:
                    dz = np.einsum("oh,bhn->bon", self.W[l], da)
                    d2z = np.einsum("oh,bhn->bon", self.W[l], d2a)
                da = d1s[l][:, :, None] * dz
                d2a = d2s[l][:, :, None] * dz * dz + d1s[l][:, :, None] * d2z
            hd = np.einsum("oh,bhn->bon", self.W[-1], d2a)[:, 0, :]
        return u, delta, hd


class ZeroNet:
    """ZeroSolution (picard/solution.py:330-337): u = 0; autograd gives None -> zeros (data.py:1316)."""

    def value_grad(self, tx, need_hdiag=False):
        B, F = tx.shape
        return np.zeros((B, 1)), np.zeros((B, F)), (np.zeros((B, F - 1)) if need_hdiag else None)


class PISGradNet:
    """picard/solution.py:138-289.  Parameters given as a dict of numpy arrays with the
    reference state-dict names (timestep_phase, timestep_coeff, t_encoder.{0,2}.*,
    smooth_net.{0,2,..}.*, nn_module.{0,2,..}.*); g0 = the equation's g (and its gradient)."""

    def __init__(self, sd, eq, T=1.0):
        self.sd = {k: np.asarray(v, np.float64) for k, v in sd.items()}
        self.eq = eq
        self.T = float(T)
        self.t_enc = self._layers("t_encoder")
        self.smooth = self._layers("smooth_net")
        self.nn = self._layers("nn_module")

    def _layers(self, prefix):
        idx = sorted({int(k.split(".")[1]) for k in self.sd if k.startswith(prefix + ".")})
        return [(self.sd[f"{prefix}.{i}.weight"], self.sd[f"{prefix}.{i}.bias"]) for i in idx]

    def _emb(self, lbd):
        arg = self.sd["timestep_coeff"] * lbd + self.sd["timestep_phase"]   # :226
        return np.concatenate([np.sin(arg), np.cos(arg)], -1)

    @staticmethod
    def _seq(layers, a, act_last=False):
        for li, (W, b) in enumerate(layers):
            a = a @ W.T + b
            if li < len(layers) - 1 or act_last:
                a = _act("ELU", a)[0]
        return a

    def value_grad(self, tx, need_hdiag=False):
        lbd = self.T - tx[:, 0:1]                                           # :273
        x = tx[:, 1:]
        smooth = (self._seq(self.smooth, self._emb(lbd))[:, 0:1]
                  - self._seq(self.smooth, self._emb(np.zeros_like(lbd)))[:, 0:1])  # :236-254
        t_emb = self._seq(self.t_enc, self._emb(lbd))                       # :279-280
        a = np.concatenate([t_emb, x], -1)
        d1s = []
        for li, (W, b) in enumerate(self.nn):
            z = a @ W.T + b
            if li < len(self.nn) - 1:
                a, d1, _ = _act("ELU", z)
                d1s.append(d1)
            else:
                a = z
        net_out = a
        sp = (net_out * x).sum(-1, keepdims=True)
        decay = np.exp(-0.5 * lbd)
        res = self.eq.g(decay * x)
        u = smooth * sp + (1.0 - smooth) * res
        # grad_x: smooth * (J^T x + net_out) + (1 - smooth) * decay * grad g0(decay x)
        delta = x @ self.nn[-1][0]
        for l in range(len(d1s) - 1, -1, -1):
            delta = delta * d1s[l]
            delta = delta @ self.nn[l][0]
        jx = delta[:, t_emb.shape[1]:]
        gres = -self.eq.grad_log_prob(decay * x) * decay
        gx = smooth * (jx + net_out) + (1.0 - smooth) * gres
        grad = np.concatenate([np.zeros_like(lbd), gx], -1)  # d/dt not needed on the label path
        return u, grad, None


# ----------------------------------------------------------------------------- sampling
def sample_points(eq, n, seed, epoch=0, point_base=0, eps=EPS_T, t_factors=0):
    """Draws 1-3 of sample_with_gradients (picard/data.py:211-223).  t_factors = 0:
    sample_t_always_uniform (:161-167); t_factors = R = N - i + 1: sample_t (:149-159),
    t = T (1 - prod of R uniforms), multiplied left to right."""
    i = point_base + np.arange(n)
    if t_factors:
        u = px.uniforms_seq(px.TAG_T, epoch, seed, i, 0, t_factors)
        prod = np.ones(n)
        for r in range(t_factors):
            prod = prod * u[:, r]
        t = (eq.T * (1 - prod))[:, None]                                    # data.py:157-159
    else:
        u = px.uniforms(px.TAG_T, epoch, seed, i, 0)
        t = ((eq.T - 2 * eps) * (1 - u) + eps)[:, None]                      # data.py:166-167
    if isinstance(eq, OUProcessEquation):
        x0 = eq.sample_x0(n, z=px.normals(px.TAG_X0, epoch, seed, i, 0, 0, eq.nx))
    else:
        x0 = eq.sample_x0(n)
    xi = px.normals(px.TAG_X, epoch, seed, i, 0, 0, eq.nx)
    x = x0 + np.sqrt(t) * eq.alpha_sqrt * xi                               # equations.py:225-226
    return np.concatenate([t, x], -1)


def path_noise(eq, i_glob, m, K, seed, epoch, v=0):
    """Per-path noise for one point: summed EM normals S_T, S_s (len(m), nx), U_s, SDGD idx."""
    S_T = np.zeros((len(m), eq.nx))
    S_s = np.zeros((len(m), eq.nx))
    for k in range(K):  # sequential EM accumulation, step by step
        S_T += px.normals(px.TAG_TERM, epoch, seed, i_glob, m, k, eq.nx)
        S_s += px.normals(px.TAG_INT, epoch, seed, i_glob, m, k, eq.nx)
    U = px.uniforms(px.TAG_S, epoch, seed, i_glob, m, open_low=True)
    idx = px.randint_idx(px.TAG_SDGD, epoch, seed, i_glob, m, v, eq.nx) if v > 0 else None
    return S_T, S_s, U, idx


def _f_and_extras(eq, net, s, X, sdgd_idx=None, base_hdiag=None):
    """get_f (picard/data.py:1226-1325) for the three shipped equations."""
    tx = np.concatenate([s, X], -1)
    need_h = eq.has_hessian_term
    u, grad, hd = net.value_grad(tx, need_hdiag=need_h)
    ux = grad[:, 1:]
    if not eq.has_hessian_term:
        return eq.ff(s, X, u, ux), hd
    # SDGD (data.py:1273-1303): u_ii at the sampled indices
    if base_hdiag is not None:
        uii = np.take_along_axis(base_hdiag, sdgd_idx, 1)
    elif sdgd_idx is not None:
        uii = np.take_along_axis(hd, sdgd_idx, 1)
    else:
        uii = hd  # full Hessian diagonal (hessian_approximation off; data.py:1262-1272)
    return eq.ffi(s, X, u, uii), hd


def td_horizon(eq, t, delta_t):
    """t_next - t and whether the terminal value comes from u (t_next < T) for the TD estimators:
    t_next = clip(t + delta_t, max=T) (picard/data.py:539, :940); delta_t = 0 is the plain
    estimator (horizon T - t, terminal value g)."""
    if delta_t > 0 and t + delta_t < eq.T:
        return delta_t, True
    return eq.T - t, False


def labels_grad(eq, net, tx, M, K, seed, epoch=0, point_base=0, v=0, m_chunk=1024,
                return_parts=False, delta_t=0.0, MT=None):
    """generate_with_gradients (picard/data.py:1208-1218) with K-step EM paths.

    Returns y (n, 1+nx) = terminal + integral.  v > 0 enables SDGD indices (GBM).
    delta_t > 0 selects the TD estimators (data.py:1209-1213): horizon t_next = min(t + delta_t, T)
    instead of T, terminal value u(t_next, X) where t_next < T (data.py:934-952, :529-575).
    M is n_estimate_integral (data.py:460); MT = n_estimate_terminal (:444, default M): the terminal
    estimator averages paths m < MT, the integral one m < M."""
    MT = M if MT is None else MT
    MI, M = M, max(M, MT)
    tx = np.asarray(tx, np.float64)
    n = tx.shape[0]
    nx = eq.nx
    T = eq.T
    a = eq.alpha_sqrt
    term = np.zeros((n, 1 + nx))
    integ = np.zeros((n, 1 + nx))
    for r in range(n):
        ig = point_base + r
        t = tx[r, 0]
        x = tx[r:r + 1, 1:]
        hmt, td_u = td_horizon(eq, t, delta_t)
        # per-point baselines
        g_x = eq.g(x)[0, 0]
        if eq.has_hessian_term:
            _, _, hd_b = net.value_grad(tx[r:r + 1], need_hdiag=True)
        else:
            hd_b = None
        fb_plain = None
        if not eq.has_hessian_term:
            fb_plain = _f_and_extras(eq, net, np.array([[t]]), x)[0][0, 0]
        for m0 in range(0, M, m_chunk):
            m = np.arange(m0, min(M, m0 + m_chunk))
            S_T, S_s, U, idx = path_noise(eq, ig, m, K, seed, epoch, v)
            kt, ki = m < MT, m < MI
            S_T, S_s, U = S_T[kt], S_s[ki], U[ki]
            idx = idx[ki] if idx is not None else None
            mt, m = m[kt], m[ki]
            if len(mt):  # terminal (data.py:899-926; TD :934-952)
                hT = hmt / K
                W_T = math.sqrt(hT) * S_T
                XT = x + a * W_T
                Y = W_T / hmt / a
                if td_u:
                    c = net.value_grad(np.concatenate([np.full((len(mt), 1), t + delta_t), XT], -1))[0] - g_x
                else:
                    c = (eq.g(XT) - g_x)
                term[r, 0] += c.sum()
                term[r, 1:] += (c * Y).sum(0)
            if not len(m):
                continue
            # integral (data.py:471-527, 350-366; TD :529-575)
            s = (U * hmt + t)[:, None]
            W_s = np.sqrt((s - t) / K) * S_s
            Xs = x + a * W_s
            Ys = W_s / (s - t) / a
            if eq.has_hessian_term:
                f, _ = _f_and_extras(eq, net, s, Xs, sdgd_idx=idx)
                xb = np.repeat(x, len(m), 0)
                fb, _ = _f_and_extras(eq, net, np.full((len(m), 1), t), xb, sdgd_idx=idx,
                                      base_hdiag=(np.repeat(hd_b, len(m), 0) if idx is not None else None))
            else:
                f, _ = _f_and_extras(eq, net, s, Xs)
                fb = np.full((len(m), 1), fb_plain)
            cI = hmt * (f - fb)
            integ[r, 0] += cI.sum() + (fb * hmt).sum()
            integ[r, 1:] += (cI * Ys).sum(0)
        term[r] /= MT
        integ[r] /= MI
        term[r, 0] += g_x
    y = term + integ
    if return_parts:
        return y, term, integ
    return y


S_HESS_OFFSET = 1e-4  # picard/data.py:848: s = U (T - t) + t + 0.0001 in the Hessian estimator


def labels_grad_hess(eq, net, tx, M, K, seed, epoch=0, point_base=0, m_chunk=512, return_parts=False, MT=None):
    """generate_with_gradients_and_hessians (picard/data.py:1220-1223) with K-step EM paths:
    estimate_terminal_with_gradients_and_hessians_double (:1153-1201) +
    estimate_integral_with_gradients_and_hessians_double (:823-897).

    The value / gradient columns are the first-order estimators with the reference's two
    half-steps (their sum is the K-step endpoint) and Y without the extra 1/sqrt(alpha) of the
    first-order terminal estimator (:1175-1178, :851-864); f is evaluated with the FULL Hessian
    diagonal (get_f without hessian_approximation_ctx, :1262-1272).  Hessian block (Malliavin
    weights, antithetic second differences):
        H = mean_m[ dg_m (N1 N1^T - I) + (T - t) df_m (N2 N2^T - I) ]
        dg = (g(x + a sqrt(T-t) N1) + g(x - ...) - 2 g(x)) / 2 / (T - t)
        df = (f(s, x + a sqrt(s-t) N2) + f(s, x - ...) - 2 f(t, x)) / 2 / (s - t)
    with fresh normals N1 (tag HTERM), N2 (tag HINT).  Returns y (n, 1 + nx + nx^2).
    M = n_estimate_integral (:845), MT = n_estimate_terminal (:1164, default M)."""
    MT = M if MT is None else MT
    MI, M = M, max(M, MT)
    tx = np.asarray(tx, np.float64)
    n, nx, T, a = tx.shape[0], eq.nx, eq.T, eq.alpha_sqrt
    term = np.zeros((n, 1 + nx))
    integ = np.zeros((n, 1 + nx))
    hT = np.zeros((n, nx, nx))
    hI = np.zeros((n, nx, nx))
    eye = np.eye(nx)
    for r in range(n):
        ig = point_base + r
        t = tx[r, 0]
        x = tx[r:r + 1, 1:]
        g_x = eq.g(x)[0, 0]
        f_b = _f_and_extras(eq, net, np.array([[t]]), x)[0][0, 0]
        for m0 in range(0, M, m_chunk):
            m = np.arange(m0, min(M, m0 + m_chunk))
            S_T, S_s, U, _ = path_noise(eq, ig, m, K, seed, epoch)
            kt, ki = m < MT, m < MI
            S_T, S_s, U = S_T[kt], S_s[ki], U[ki]
            N1 = px.normals(px.TAG_HTERM, epoch, seed, ig, m[kt], 0, nx)
            N2 = px.normals(px.TAG_HINT, epoch, seed, ig, m[ki], 0, nx)
            B = int(ki.sum())
            if kt.any():  # terminal, value / gradient (:1166-1183)
                W_T = math.sqrt((T - t) / K) * S_T
                c = eq.g(x + a * W_T) - g_x
                term[r, 0] += c.sum()
                term[r, 1:] += (c * W_T / (T - t)).sum(0)
                # terminal Hessian (:1185-1199)
                W1 = math.sqrt(T - t) * N1
                dg = (eq.g(x + a * W1) + eq.g(x - a * W1) - 2 * g_x) / 2 / (T - t)          # (B, 1)
                hT[r] += np.einsum("b,bi,bj->ij", dg[:, 0], N1, N1) - dg.sum() * eye
            if not B:
                continue
            # integral, value / gradient (:846-866)
            s = (U * (T - t) + t + S_HESS_OFFSET)[:, None]
            W_s = np.sqrt((s - t) / K) * S_s
            f = _f_and_extras(eq, net, s, x + a * W_s)[0]
            cI = (T - t) * (f - f_b)
            integ[r, 0] += cI.sum() + B * f_b * (T - t)
            integ[r, 1:] += (cI * W_s / (s - t)).sum(0)
            # integral Hessian (:869-881)
            W2 = np.sqrt(s - t) * N2
            fp = _f_and_extras(eq, net, s, x + a * W2)[0]
            fm = _f_and_extras(eq, net, s, x - a * W2)[0]
            df = (fp + fm - 2 * f_b) / 2 / (s - t)                                       # (B, 1)
            hI[r] += (T - t) * (np.einsum("b,bi,bj->ij", df[:, 0], N2, N2) - df.sum() * eye)
        term[r] /= MT
        integ[r] /= MI
        hT[r] /= MT
        hI[r] /= MI
        term[r, 0] += g_x
    y = np.concatenate([term + integ, (hT + hI).reshape(n, nx * nx)], -1)
    if return_parts:
        return y, np.concatenate([term, hT.reshape(n, -1)], -1), np.concatenate([integ, hI.reshape(n, -1)], -1)
    return y


def sample_with_gradients(eq, net, n, M, K, seed, epoch=0, point_base=0, v=0, sample_bound=np.inf, delta_t=0.0,
                          t_factors=0, MT=None):
    """picard/data.py:211-223: (tx, clip(y))."""
    tx = sample_points(eq, n, seed, epoch, point_base, t_factors=t_factors)
    y = labels_grad(eq, net, tx, M, K, seed, epoch, point_base, v, delta_t=delta_t, MT=MT)
    return tx, np.clip(y, -sample_bound, sample_bound)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def rel_l2_parts(a, b):
    return {"value": rel_l2(a[:, :1], b[:, :1]), "grad": rel_l2(a[:, 1:], b[:, 1:]), "all": rel_l2(a, b)}


# ----------------------------------------------------------------------------- moments (sharding)
def path_contributions(eq, net, tx_row, ig, m, K, seed, epoch=0, delta_t=0.0, flags=3):
    """Per-path contribution rows c (len(m), 1+nx) whose mean (+ g(x) in column 0) is the label
    (picard/data.py:923-925, :523-526; TD :947-951, :570-574), for one point and MC indices m.
    flags (DPI_TERMINAL = 1 | DPI_INTEGRAL = 2): the estimators included."""
    t = float(tx_row[0])
    x = np.asarray(tx_row[1:], np.float64)[None]
    a = eq.alpha_sqrt
    hmt, td_u = td_horizon(eq, t, delta_t)
    g_x = eq.g(x)[0, 0]
    fb = _f_and_extras(eq, net, np.array([[t]]), x)[0][0, 0]
    S_T, S_s, U, _ = path_noise(eq, ig, np.asarray(m), K, seed, epoch)
    W_T = math.sqrt(hmt / K) * S_T
    Y = W_T / hmt / a
    if td_u:
        cT = net.value_grad(np.concatenate([np.full((len(m), 1), t + delta_t), x + a * W_T], -1))[0] - g_x
    else:
        cT = eq.g(x + a * W_T) - g_x
    s = (U * hmt + t)[:, None]
    W_s = np.sqrt((s - t) / K) * S_s
    f, _ = _f_and_extras(eq, net, s, x + a * W_s)
    cI = hmt * (f - fb)
    Ys = W_s / (s - t) / a
    if not flags & 1:
        cT = 0 * cT
    if not flags & 2:
        cI, fb = 0 * cI, 0.0
    c = np.concatenate([cT + cI + fb * hmt, cT * Y + cI * Ys], -1)
    return c, g_x


def path_contributions_hess(eq, net, tx_row, ig, m, K, seed, epoch=0, flags=3):
    """Per-path rows of the Hessian-label estimator (labels_grad_hess): value/gradient c
    (len(m), 1+nx), Hessian h (len(m), nx*nx) whose means (+ g(x) in c[:, 0]) are the label.
    flags (DPI_TERMINAL = 1 | DPI_INTEGRAL = 2): the estimators included."""
    t = float(tx_row[0])
    x = np.asarray(tx_row[1:], np.float64)[None]
    T, a, nx = eq.T, eq.alpha_sqrt, eq.nx
    m = np.asarray(m)
    g_x = eq.g(x)[0, 0]
    f_b = _f_and_extras(eq, net, np.array([[t]]), x)[0][0, 0]
    S_T, S_s, U, _ = path_noise(eq, ig, m, K, seed, epoch)
    N1 = px.normals(px.TAG_HTERM, epoch, seed, ig, m, 0, nx)
    N2 = px.normals(px.TAG_HINT, epoch, seed, ig, m, 0, nx)
    W_T = math.sqrt((T - t) / K) * S_T
    cT = eq.g(x + a * W_T) - g_x
    s = (U * (T - t) + t + S_HESS_OFFSET)[:, None]
    W_s = np.sqrt((s - t) / K) * S_s
    cI = (T - t) * (_f_and_extras(eq, net, s, x + a * W_s)[0] - f_b)
    kT, kI = float(flags & 1 != 0), float(flags & 2 != 0)
    cT, cI = kT * cT, kI * cI
    c = np.concatenate([cT + cI + kI * f_b * (T - t), cT * W_T / (T - t) + cI * W_s / (s - t)], -1)
    W1 = math.sqrt(T - t) * N1
    aT = ((eq.g(x + a * W1) + eq.g(x - a * W1) - 2 * g_x) / 2 / (T - t))[:, 0]
    W2 = np.sqrt(s - t) * N2
    fp = _f_and_extras(eq, net, s, x + a * W2)[0]
    fm = _f_and_extras(eq, net, s, x - a * W2)[0]
    aI = (T - t) * ((fp + fm - 2 * f_b) / 2 / (s - t))[:, 0]
    h = (kT * aT[:, None, None] * (N1[:, :, None] * N1[:, None, :] - np.eye(nx))
         + kI * aI[:, None, None] * (N2[:, :, None] * N2[:, None, :] - np.eye(nx)))
    return c, h.reshape(len(m), nx * nx), g_x


def tree_sum_f32(values):
    """The device's canonical fixed-order sum (csrc/dpi_kernels.hip tree_sum): zero-pad to a
    power of two >= 64 and add as a perfect binary tree in index order, in fp32.  values: (cnt, ...)."""
    v = np.asarray(values, np.float32)
    p2 = 64
    while p2 < v.shape[0]:
        p2 *= 2
    pad = np.zeros((p2 - v.shape[0],) + v.shape[1:], np.float32)
    v = np.concatenate([v, pad], 0)
    while v.shape[0] > 1:
        v = (v[0::2] + v[1::2]).astype(np.float32)
    return v[0]
