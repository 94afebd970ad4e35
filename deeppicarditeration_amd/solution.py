"""Networks u(t, x) evaluated on the label path (picard/solution.py) and their upload to the
HIP label kernels (include/dpi.h dpi_net_create_*).

`construct_mlp`, `ZeroSolution` and `PISGradNet` keep the reference's module structure and
state-dict names, so a checkpointed reference network loads unchanged; `DeviceNet.from_module`
packs it (state-dict order) into a device handle once per Picard iteration.
"""
from typing import Optional

import numpy as np
import torch

from . import _lib


def construct_mlp(n_in: int, n_out: int, n_neurons: list, activations: list, bound: Optional[float]):
    """picard/solution.py:123-135."""
    assert len(n_neurons) == len(activations)
    layers = []
    dims = [n_in] + list(n_neurons)
    for i in range(len(activations)):
        layers.append(torch.nn.Linear(dims[i], dims[i + 1]))
        layers.append(getattr(torch.nn, activations[i])())
    layers.append(torch.nn.Linear(dims[-1], n_out))
    if bound is not None:
        assert bound > 0
        layers.append(torch.nn.Hardtanh(-bound, bound))
    return torch.nn.Sequential(*layers)


class ZeroFunction(torch.autograd.Function):
    """picard/utils.py:80-94: zeros of shape (B, 1), no gradient wrt the input."""

    @staticmethod
    def forward(ctx, *args, **kwargs):
        tx = args[0]
        return torch.zeros(tx.size(0), 1, device=tx.device, dtype=tx.dtype)

    @staticmethod
    def backward(ctx, *grad_output):
        return None


class ZeroSolution(torch.nn.Module):
    """picard/solution.py:330-337 — the iteration-1 'previous iterate'."""

    def __init__(self, output_dim: int = 1):
        super().__init__()
        self.output_dim = output_dim

    def forward(self, tx):
        return ZeroFunction.apply(tx).expand(-1, self.output_dim)


class PISGradNet(torch.nn.Module):
    """picard/solution.py:138-289 (same submodule names / state dict)."""

    def __init__(self, hidden_shapes: list, dim: int, g0, T=1.0):
        super().__init__()
        self.hidden_shapes = hidden_shapes
        self.n_layers = len(hidden_shapes)
        self.dim = dim
        self.act = torch.nn.ELU()
        self.channels = 64
        self.timestep_phase = torch.nn.Parameter(torch.zeros(1, self.channels))
        self.register_buffer("timestep_coeff", torch.linspace(0.1, 100.0, steps=self.channels).unsqueeze(0))
        self.t_encoder = torch.nn.Sequential(torch.nn.Linear(2 * self.channels, self.channels), self.act,
                                             torch.nn.Linear(self.channels, self.channels))
        layers = [torch.nn.Linear(2 * self.channels, self.channels)]
        for _ in range(self.n_layers):
            layers += [self.act, torch.nn.Linear(self.channels, self.channels)]
        layers += [self.act, torch.nn.Linear(self.channels, dim)]
        self.smooth_net = torch.nn.Sequential(*layers)
        net = []
        in_dim = self.dim + self.channels
        for hs in hidden_shapes:
            net += [torch.nn.Linear(in_dim, hs), self.act]
            in_dim = hs
        net.append(torch.nn.Linear(in_dim, self.dim))
        self.nn_module = torch.nn.Sequential(*net)
        self.g0 = g0
        self.T = T

    def get_pis_timestep_embedding(self, lbd):
        arg = self.timestep_coeff * lbd + self.timestep_phase
        return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)

    def smoothing_function(self, lbd):
        if lbd.ndim == 1:
            lbd = lbd.unsqueeze(-1)
        out_lbd = self.smooth_net(self.get_pis_timestep_embedding(lbd))
        out_zero = self.smooth_net(self.get_pis_timestep_embedding(torch.zeros_like(lbd)))
        return out_lbd[..., 0:1] - out_zero[..., 0:1]

    def forward(self, tx):
        lbd, x = tx[..., 0:1], tx[..., 1:]
        lbd = self.T - lbd
        smooth = self.smoothing_function(lbd)
        t_emb = self.t_encoder(self.get_pis_timestep_embedding(lbd))
        net_out = self.nn_module(torch.cat([t_emb, x], dim=-1))
        sp_out = torch.sum(net_out * x, dim=-1, keepdim=True)
        residual = self.g0(torch.exp(-0.5 * lbd) * x)
        return smooth * sp_out + (1.0 - smooth) * residual


def _unwrap(module):
    """The network inside the reference's solution wrappers: PicardSolution keeps it in `.model`
    (picard/solution.py:313-325), PicardSolutionGradientWrapper / ...HessianWrapper keep the
    PicardSolution in `.solution` (picard/solution_jac.py:124-126, 219-226)."""
    while True:
        inner = getattr(module, "model", None)
        if not isinstance(inner, torch.nn.Module):
            inner = getattr(module, "solution", None)
        if not isinstance(inner, torch.nn.Module):
            return module
        module = inner


class DeviceNet:
    """A network uploaded to the label kernels (owns a dpi_net handle)."""

    def __init__(self, handle, desc):
        self.handle = handle
        self.desc = desc

    def __del__(self):
        try:
            _lib.load().dpi_net_destroy(self.handle)
        except Exception:
            pass

    def set_precision(self, mode):
        """Per-network GEMM precision (include/dpi.h dpi_net_set_precision; -1 = process-wide)."""
        _lib.check(_lib.load().dpi_net_set_precision(self.handle, int(mode)), "dpi_net_set_precision")

    def status(self, stream, clear=True):
        """The sticky DPI_STATUS_* word of the label reductions on this net (synchronises `stream`)."""
        v = _lib.c_int(0)
        _lib.check(_lib.load().dpi_net_status(self.handle, 1 if clear else 0, stream, _lib.ctypes.byref(v)),
                   "dpi_net_status")
        return v.value

    @classmethod
    def from_module(cls, module, n_in: int):
        lib = _lib.load()
        m = _unwrap(module)
        h = _lib.c_void_p()
        if isinstance(m, ZeroSolution) or type(m).__name__ == "ZeroSolution":
            _lib.check(lib.dpi_net_create_zero(h), "dpi_net_create_zero")
            return cls(h, "zero")
        if isinstance(m, torch.nn.Sequential):
            lin = [l for l in m if isinstance(l, torch.nn.Linear)]
            acts = [type(l).__name__ for l in m if not isinstance(l, torch.nn.Linear)]
            # construct_mlp's activations (picard/solution.py:123-135): the label kernels are compiled
            # for ELU (alpha = 1) and Tanh, the same one in every hidden layer
            act_code = {"ELU": _lib.DPI_ACT_ELU, "Tanh": _lib.DPI_ACT_TANH}.get(acts[0] if acts else "ELU")
            if act_code is None or any(a != acts[0] for a in acts):
                raise NotImplementedError(f"MLP activations {acts}: the label kernels are compiled for all-ELU or "
                                          "all-Tanh hidden layers")
            if any(l.alpha != 1.0 for l in m if isinstance(l, torch.nn.ELU)):
                raise NotImplementedError("ELU alpha != 1")
            if lin[-1].out_features != 1:
                raise NotImplementedError("network output_dim != 1 (Value networks only)")
            if lin[0].in_features != n_in:
                raise ValueError(f"network input {lin[0].in_features} != 1 + nx = {n_in}")
            widths = [l.out_features for l in lin[:-1]]
            flat = np.concatenate([np.concatenate([l.weight.detach().cpu().double().numpy().ravel(),
                                                   l.bias.detach().cpu().double().numpy().ravel()]) for l in lin])
            flat = np.ascontiguousarray(flat, np.float32)
            w = (_lib.c_int * len(widths))(*widths)
            _lib.check(lib.dpi_net_create_mlp(n_in, len(widths), w, act_code,
                                              flat.ctypes.data_as(_lib.P(_lib.c_float)), flat.size, h),
                       "dpi_net_create_mlp")
            return cls(h, f"mlp{widths}" + ("" if act_code == _lib.DPI_ACT_ELU else "-tanh"))
        if isinstance(m, PISGradNet) or type(m).__name__ == "PISGradNet":
            return cls._from_pisgrad(lib, m, n_in)
        raise NotImplementedError(f"network type {type(m).__name__} has no device implementation in this build")

    @classmethod
    def _from_pisgrad(cls, lib, m, n_in):
        """PISGradNet -> dpi_net_create_pisgrad (state-dict order, solution.py:160-205)."""
        nx = n_in - 1
        if m.dim != nx or m.channels != 64:
            raise ValueError("PISGradNet dim/channels mismatch")
        g0_owner = getattr(m.g0, "__self__", None)
        if g0_owner is None or type(g0_owner).__name__ != "OUProcessEquation":
            raise NotImplementedError("PISGradNet on the device needs g0 = OUProcessEquation.g (as PicardSolution builds it)")
        sd = m.state_dict()
        L = len(m.hidden_shapes)
        names = ["timestep_phase", "timestep_coeff", "t_encoder.0.weight", "t_encoder.0.bias", "t_encoder.2.weight",
                 "t_encoder.2.bias"]
        names += [f"smooth_net.{2 * j}.{w}" for j in range(L + 2) for w in ("weight", "bias")]
        names += [f"nn_module.{2 * l}.{w}" for l in range(L + 1) for w in ("weight", "bias")]
        flat = np.ascontiguousarray(np.concatenate([sd[k].detach().cpu().double().numpy().ravel() for k in names]),
                                    np.float32)
        hidden = (_lib.c_int * L)(*[int(h) for h in m.hidden_shapes])
        h = _lib.c_void_p()
        _lib.check(lib.dpi_net_create_pisgrad(nx, L, hidden, float(m.T), flat.ctypes.data_as(_lib.P(_lib.c_float)),
                                              flat.size, h), "dpi_net_create_pisgrad")
        return cls(h, f"pisgrad{list(m.hidden_shapes)}")
