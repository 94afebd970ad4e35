"""Problem plugins — the reference's `picard/equations.py` interface, kept by name and argument
meaning so YAML `EQUATION.cls` / `EQUATION.kwargs` resolve the same way
(`getattr(equations, cls)(**kwargs)`, picard/picard_iteration.py:90-92).

Each class exposes the reference's attributes/methods used around the label path (nx, nu, T,
alpha, alpha_sqrt, has_*_term, g, g_x, f/ff/fff/ffi/ffh, exact solutions, sample_x0/sample_x
for evaluation) as torch code, and `dpi_problem()` — the compiled device plugin the HIP label
kernels run (include/dpi.h dpi_problem_create_*).  The torch methods are the plugin API for
the outer fit / evaluation; labels are never computed through them.
"""
import math
from pathlib import Path

import numpy as np
import torch

from . import _lib

_DATA = Path(__file__).resolve().parent / "problem_data"


def _load_param(ref_name, packaged_name):
    """Reference loads problem parameters from the CWD (equations.py:410-411, :530-532); keep
    that precedence (safe loader), then fall back to the packaged copy of the shipped file."""
    p = Path(ref_name)
    if p.exists():
        return torch.load(p, weights_only=True).to(torch.float64)
    q = _DATA / packaged_name
    if q.exists():
        return torch.from_numpy(np.load(q, allow_pickle=False)).to(torch.float64)
    raise FileNotFoundError(f"{ref_name} not found in CWD and no packaged copy {packaged_name}")


class _DeviceProblem:
    def __init__(self, handle):
        self.handle = handle

    def __del__(self):
        try:
            _lib.load().dpi_problem_destroy(self.handle)
        except Exception:
            pass


class Equation:
    """picard/equations.py:63-184."""

    has_gradient_term = None
    has_laplacian_term = None
    has_hessian_term = None
    num_v_samples = None
    supported_approximate_methods = tuple()

    def __init__(self, T: float = 1, nx: int = 1):
        self.T = T
        self.nx = nx
        self.nu = 1
        self._dev = None
        self._device = torch.device("cpu")

    @property
    def device(self):
        return self._device

    def to(self, *, device):
        self._device = torch.device(device)
        return self

    def sample_x0(self, n: int):
        return torch.randn(n, self.nx, device=self._device)

    def sample_x(self, t: torch.Tensor):  # equations.py:118-119
        return self.sample_x_ts(torch.zeros_like(t), t, self.sample_x0(len(t)))

    def dpi_problem(self):
        """Compiled device plugin handle (created once)."""
        if self._dev is None:
            self._dev = _DeviceProblem(self._create_device_problem(_lib.load()))
        return self._dev.handle

    def _create_device_problem(self, lib):
        raise NotImplementedError(f"{type(self).__name__} has no device plugin in this build")


class DiffusionEquation(Equation):
    """Sigma = sqrt(alpha) I (equations.py:187-206)."""

    def __init__(self, *, alpha: float = 1.0, **kwargs):
        super().__init__(**kwargs)
        self.alpha = torch.scalar_tensor(alpha, dtype=torch.float64)
        self.alpha_sqrt = torch.sqrt(self.alpha)

    def ff(self, t, x, y, w):
        return self.fff(t, x, y, self.alpha_sqrt * w)


class SimpleDiffusionEquation(DiffusionEquation):
    """mu = 0: dX = sqrt(alpha) dW (equations.py:209-230)."""

    def sample_x_ts(self, t, s, x, return_dW=False):
        dW = torch.randn_like(x)
        x_next = x + torch.sqrt(s - t) * self.alpha_sqrt.to(x) * dW
        return (x_next, dW) if return_dW else x_next


class SimpleDiffusionEquationWithZ(SimpleDiffusionEquation):
    has_gradient_term = True
    has_laplacian_term = False
    has_hessian_term = False

    def f(self, t, x, y):
        raise NotImplementedError("The equation has dependence on z, use fff or ff instead.")


class Cha(SimpleDiffusionEquationWithZ):
    """Burgers-type equation (equations.py:266-338):
        u_t + alpha/2 u_xx + [alpha k u - 1/(k d) - alpha k/2] sum_i u_{x_i} = 0,  g = sigmoid(T + k sum x)
    with k' = k / sqrt(nx); exact solution sigmoid(t + k' sum x)."""

    def __init__(self, nx: int, alpha: float, k=1.0, T: float = 1.0):
        super().__init__(nx=nx, alpha=alpha, T=T)
        self.k_raw = float(k)
        self.k = torch.scalar_tensor(k / np.sqrt(self.nx), dtype=torch.float64)
        self.alpha_d = self.alpha * self.nx
        self.k_alpha_d = self.k * self.alpha_d
        self.k_alpha_d_2 = self.k_alpha_d * 2
        self.k2_alpha_d = self.k * self.k_alpha_d

    def fff(self, t, x, y, z):
        c = (2 + self.k2_alpha_d) / self.k_alpha_d_2
        return self.alpha_sqrt.to(y) * (self.k.to(y) * y - c.to(y)) * torch.sum(z, dim=-1, keepdim=True)

    def g(self, x):
        return torch.sigmoid(self.T + self.k.to(x) * torch.sum(x, dim=-1, keepdim=True))

    def g_x(self, x):
        s = self.g(x)
        return self.k.to(x) * s * (1 - s)

    def exact_solution(self, t, x):
        return torch.sigmoid(t + self.k.to(x) * torch.sum(x, dim=-1, keepdim=True))

    def u_x(self, t, x):
        uu = self.exact_solution(t, x)
        return torch.ones_like(x) * (self.k.to(x) * uu * (1 - uu))

    def u_u_x(self, t, x):
        u = self.exact_solution(t, x)
        return u, torch.ones_like(x) * (self.k.to(x) * u * (1 - u))

    def sample_x0(self, n: int):
        return torch.zeros(n, self.nx, device=self._device)

    def ffh(self, t, x, u, u_x, hess_u):
        return self.ff(t, x, u, u_x)

    def _create_device_problem(self, lib):
        h = _lib.c_void_p()
        _lib.check(lib.dpi_problem_create_cha(self.nx, float(self.alpha), self.k_raw, float(self.T), h),
                   "dpi_problem_create_cha")
        return h


class GaussianMixtureDiagonalCovariance:
    """utils.py:792-914 (diagonal covariances; log-sum-exp over components)."""

    def __init__(self, means, var_diag, weights):
        self.means = means
        self.var_diag = var_diag
        self.weights = weights
        self.dim = means.shape[-1]
        self.log_2pi = math.log(2.0 * math.pi)
        self.log_weights = torch.log(weights)
        self.cov_invs = 1.0 / var_diag
        self.norm = -0.5 * (self.dim * self.log_2pi + torch.log(var_diag).sum(-1))

    def _lp(self, x):
        diff = x.unsqueeze(-2) - self.means.to(x)
        e = -0.5 * torch.einsum("bkn,kn->bk", diff ** 2, self.cov_invs.to(x))
        return self.log_weights.to(x) + self.norm.to(x) + e, diff

    def log_prob(self, x):
        lp, _ = self._lp(x)
        return torch.logsumexp(lp, dim=-1, keepdim=True)

    def grad_log_prob(self, x):
        lp, diff = self._lp(x)
        w = torch.softmax(lp, dim=-1)
        return torch.einsum("bk,bkn->bn", w, -diff * self.cov_invs.to(x))


class ComplexDiffusionEquation(DiffusionEquation):
    """Sigma = sqrt(alpha) I, drift F enters only through ff (equations.py:489-596); the forward
    sampler has no drift (equations.py:560-573) — and neither does the HIP rollout."""

    has_gradient_term = True
    has_laplacian_term = False
    has_hessian_term = False

    def __init__(self, nx, T, theta: float = 1.0, mu: float = 0.0, alpha: float = 1.0, num_components=2,
                 mean_scale=1.0, var_scale=2.0, alpha_scale=4.0, mean=None, var=None, pi=None, **kwargs):
        """mean (K, nx), var (K, nx) diagonals, pi (K): the mixture's parameters when given (the
        reference-side binding passes the reference equation's own tensors); otherwise loaded as the
        reference loads them (equations.py:525-544)."""
        super().__init__(nx=nx, T=T, alpha=alpha, **kwargs)
        self.theta = float(theta)
        self.mu = float(mu)
        self.d = float(nx)
        self.num_components = num_components
        tag = f"{nx}d_ms={mean_scale}_vs={var_scale}_{num_components}"
        f64 = lambda a: torch.as_tensor(a).detach().cpu().to(torch.float64)  # noqa: E731
        self.mean = f64(mean) if mean is not None else _load_param(f"mean_{tag}.pt", f"mean_{tag}.npy")
        self.pi = f64(pi) if pi is not None else _load_param(f"pi_{tag}.pt", f"pi_{tag}.npy")
        if var is not None:
            self.var = f64(var)
        else:
            try:
                self.var = torch.diagonal(_load_param(f"var_{tag}.pt", f"var_{tag}.npy"), dim1=-2, dim2=-1)
            except FileNotFoundError:  # SURVEY.md finding 8: var = var_scale * I (equations.py:539)
                self.var = var_scale * torch.ones(num_components, nx, dtype=torch.float64)
        if self.mean.shape != (num_components, nx) or self.var.shape != (num_components, nx) or \
                self.pi.shape != (num_components,):
            raise ValueError("GMM parameters: mean and var (num_components, nx), pi (num_components,)")
        self.gmm_calc = GaussianMixtureDiagonalCovariance(self.mean, self.var, self.pi)
        self.alpha_scale = float(alpha_scale)
        self.alpha_init = alpha_scale * float(alpha)

    def sample_x_ts(self, t, s, x, return_dW=False):
        dW = torch.randn_like(x)
        x_next = x + torch.sqrt(s - t) * self.alpha_sqrt.to(x) * dW
        return (x_next, dW) if return_dW else x_next

    def f(self, t, x, y):  # equations.py:575-576
        raise NotImplementedError("The equation has dependence on z, use fff or ff instead.")

    def fff(self, t, x, y, z):
        return self.ff(t, x, y, self.alpha_sqrt.to(z) * z)

    def g(self, x):
        return -self.gmm_calc.log_prob(x)

    def g_x(self, x):
        return -self.gmm_calc.grad_log_prob(x)

    def sample_x0(self, n: int):
        return math.sqrt(self.alpha_init) * torch.randn(n, self.nx, device=self._device)


class OUProcessEquation(ComplexDiffusionEquation):
    """HJB with OU drift in the nonlinearity (equations.py:599-714):
        ff(t, x, y, z) = -theta (mu - x) . z - alpha/2 |z|^2 - d theta     (z = grad u)."""

    def F(self, t, x, y, z):
        return self.theta * (self.mu - x)

    def ff(self, t, x, y, z):
        return (-(self.F(t, x, y, z) * z).sum(-1, keepdim=True) - float(self.alpha) / 2 * (z ** 2).sum(-1, keepdim=True)
                - self.d * self.theta * torch.ones_like(y))

    def ffh(self, t, x, u, u_x, hess_u):
        return self.ff(t, x, u, u_x)

    def get_gmm_t(self, t):  # equations.py:638-648 (OU transition of each component)
        et = math.exp(-self.theta * float(t))
        means = self.mu + (self.mean - self.mu) * et
        var = self.var * et ** 2 + (float(self.alpha) / (2 * self.theta)) * (1 - et ** 2)
        return GaussianMixtureDiagonalCovariance(means, var, self.pi)

    def _gmm_rows(self, t, x):
        """Per-row GMM of the OU transition over T - t (get_gmm_t for every row at once):
        component log-densities (n, K) and the scaled residuals diff/var (n, K, nx)."""
        lam = (self.T - torch.as_tensor(t, dtype=x.dtype, device=x.device).reshape(-1, 1)).unsqueeze(-1)  # (n,1,1)
        et = torch.exp(-self.theta * lam)
        means = self.mu + (self.mean.to(x) - self.mu) * et                                    # (n,K,nx)
        var = self.var.to(x) * et ** 2 + (float(self.alpha) / (2 * self.theta)) * (1 - et ** 2)
        diff = x.unsqueeze(-2) - means
        lp = (torch.log(self.pi.to(x)) - 0.5 * (self.nx * math.log(2.0 * math.pi) + torch.log(var).sum(-1))
              - 0.5 * (diff ** 2 / var).sum(-1))
        return lp, diff / var

    def exact_solution(self, t, x):
        """equations.py:650-652: -log of the OU-transported mixture at (T - t, x), row by row."""
        lp, _ = self._gmm_rows(t, x)
        return -torch.logsumexp(lp, dim=-1, keepdim=True)

    def u_x(self, t, x):
        """equations.py:668-681 (autograd there): grad_x of -log sum_k pi_k N_k = sum_k w_k (x - m_k)/v_k."""
        lp, r = self._gmm_rows(t, x)
        return torch.einsum("nk,nkd->nd", torch.softmax(lp, dim=-1), r)

    def u_u_x(self, t, x):  # equations.py:697-700
        lp, r = self._gmm_rows(t, x)
        return -torch.logsumexp(lp, dim=-1, keepdim=True), torch.einsum("nk,nkd->nd", torch.softmax(lp, dim=-1), r)

    def _create_device_problem(self, lib):
        h = _lib.c_void_p()
        m = np.ascontiguousarray(self.mean.numpy(), np.float64)
        v = np.ascontiguousarray(self.var.numpy(), np.float64)
        p = np.ascontiguousarray(self.pi.numpy(), np.float64)
        dp = _lib.P(_lib.c_double)
        _lib.check(lib.dpi_problem_create_ou(self.nx, float(self.alpha), float(self.T), self.theta, self.mu,
                                             self.alpha_scale, self.num_components, m.ctypes.data_as(dp),
                                             v.ctypes.data_as(dp), p.ctypes.data_as(dp), h),
                   "dpi_problem_create_ou")
        return h


class SimpleDiffusionEquationWithHessian(SimpleDiffusionEquation):
    has_gradient_term = True
    has_laplacian_term = False
    has_hessian_term = True

    def f(self, t, x, y):  # equations.py:369-370
        raise NotImplementedError("The equation has dependence on z and hessian, use ffh instead.")


class GBMEquationComplexExact(SimpleDiffusionEquationWithHessian):
    """Fully-nonlinear case (equations.py:388-486): u* = sum_k v_k sin(w_k . [t, x])."""

    supported_approximate_methods = ("SDGD",)

    def __init__(self, nx: int, alpha: float = 1.0, T: float = 1.0, case: str = "case_1", w=None, v=None):
        """w (nodes, 1 + nx), v (nodes, 1): given (the reference-side binding passes the reference
        equation's tensors), or loaded as the reference loads them (equations.py:408-419)."""
        super().__init__(nx=nx, alpha=alpha, T=T)
        self.d = float(nx)
        f64 = lambda a: torch.as_tensor(a).detach().cpu().to(torch.float64)  # noqa: E731
        self.w = f64(w) if w is not None else _load_param(f"gbm_2nodes_w_{nx}d.pt", f"gbm_2nodes_w_{nx}d_{case}.npy")
        self.v = f64(v) if v is not None else _load_param(f"gbm_2nodes_v_{nx}d.pt", f"gbm_2nodes_v_{nx}d_{case}.npy")

    def _arg(self, t, x):
        t = torch.as_tensor(t, dtype=x.dtype, device=x.device) * torch.ones(x.shape[0], 1, dtype=x.dtype,
                                                                              device=x.device)
        return torch.cat([t, x], -1) @ self.w.to(x).t()

    def exact_solution(self, t, x):
        return torch.sin(self._arg(t, x)) @ self.v.to(x)

    def g(self, x):
        return self.exact_solution(self.T, x)

    def u_t(self, t, x):
        return torch.cos(self._arg(t, x)) @ (self.v * self.w[:, 0:1]).to(x)

    def u_x(self, t, x):
        return torch.cos(self._arg(t, x)) @ (self.v * self.w[:, 1:]).to(x)

    def g_x(self, x):
        return self.u_x(self.T, x)

    def laplacian(self, t, x):
        return -torch.sin(self._arg(t, x)) @ (self.v * (self.w[:, 1:] ** 2).sum(-1, keepdim=True)).to(x)

    def u_u_x(self, t, x):  # equations.py:440-443
        return self.exact_solution(t, x), self.u_x(t, x)

    def u_hessian(self, t, x):
        """equations.py:445-450: -sum_k v_k w_k w_k^T sin(w_k . [t, x]), (n, nx, nx)."""
        wx = self.w[:, 1:].to(x)
        return torch.einsum("nk,kij->nij", -torch.sin(self._arg(t, x)),
                            self.v.to(x).reshape(-1, 1, 1) * wx.unsqueeze(2) * wx.unsqueeze(1))

    def u_u_x_u_hessian(self, t, x):  # equations.py:381-385
        return self.exact_solution(t, x), self.u_x(t, x), self.u_hessian(t, x)

    def hess_diag(self, t, x):
        return -torch.sin(self._arg(t, x)) @ (self.v * self.w[:, 1:] ** 2).to(x)

    def ffh(self, t, x, u, u_x, hess_u):  # equations.py:476-478 (full Hessian: its diagonal)
        return self.ffi(t, x, u, torch.diagonal(hess_u, dim1=1, dim2=2))

    def ffi(self, t, x, u, u_ii):
        lap = self.d * u_ii.mean(-1, keepdim=True)
        nonlin = self.d * u_ii.abs().mean(-1, keepdim=True)
        return (0.5 * (1.0 - float(self.alpha)) * lap + 0.25 * nonlin - self.u_t(t, x) - 0.5 * self.laplacian(t, x)
                - 0.25 * self.hess_diag(t, x).abs().sum(-1, keepdim=True))

    def sample_x0(self, n: int):
        return torch.zeros(n, self.nx, device=self._device)

    def _create_device_problem(self, lib):
        h = _lib.c_void_p()
        w = np.ascontiguousarray(self.w.numpy(), np.float64)
        v = np.ascontiguousarray(self.v.numpy().reshape(-1), np.float64)
        dp = _lib.P(_lib.c_double)
        _lib.check(lib.dpi_problem_create_gbm(self.nx, float(self.alpha), float(self.T), w.shape[0],
                                              w.ctypes.data_as(dp), v.ctypes.data_as(dp), h),
                   "dpi_problem_create_gbm")
        return h


def from_reference(eq) -> Equation:
    """The device-backed equation for a reference `picard.equations` object (the reference-side
    binding receives the data module's own equation, picard/data.py:1474-1481): same class name,
    parameters read from the object — Cha (nx, alpha, k = k' sqrt(nx), T; equations.py:283-290),
    OUProcessEquation (nx, T, theta, mu, alpha, alpha_scale = alpha_init / alpha, the GMM's mean /
    var / pi tensors; equations.py:503-558, 609-619), GBMEquationComplexExact (nx, alpha, T, w, v;
    equations.py:403-419).  An equation of this package is returned as is; any other class raises."""
    if isinstance(eq, Equation):
        return eq
    name = type(eq).__name__
    f = lambda a: float(torch.as_tensor(a))  # noqa: E731
    if name == "Cha":
        return Cha(nx=int(eq.nx), alpha=f(eq.alpha), k=f(eq.k) * math.sqrt(int(eq.nx)), T=f(eq.T))
    if name == "OUProcessEquation":
        var = torch.as_tensor(eq.var).detach().cpu().to(torch.float64)
        if var.dim() == 3:  # (K, nx, nx) covariance matrices (equations.py:539): diagonal mixtures only
            diag = torch.diagonal(var, dim1=-2, dim2=-1)
            if not torch.equal(var, torch.diag_embed(diag)):
                raise NotImplementedError("OUProcessEquation with non-diagonal GMM covariances")
            var = diag
        return OUProcessEquation(nx=int(eq.nx), T=f(eq.T), theta=f(eq.theta), mu=f(eq.mu), alpha=f(eq.alpha),
                                 num_components=int(eq.num_components), alpha_scale=f(eq.alpha_init) / f(eq.alpha),
                                 mean=eq.mean, var=var, pi=eq.pi)
    if name == "GBMEquationComplexExact":
        return GBMEquationComplexExact(nx=int(eq.nx), alpha=f(eq.alpha), T=f(eq.T), w=eq.w, v=eq.v)
    raise NotImplementedError(f"{name}: no device plugin in this build (Cha, OUProcessEquation, "
                              "GBMEquationComplexExact)")
