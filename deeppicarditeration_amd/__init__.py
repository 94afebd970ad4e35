"""MI355X-native DPI label-generation hot path (Deep Picard Iteration, arXiv 2409.08526).

Drop-in for the reference's `picard.data.OnlineDataGenerator` label path: Philox noise,
K-step Euler–Maruyama rollouts, u / grad u of the previous iterate and the terminal +
f-integral accumulation run in hand-written HIP kernels for gfx950 (libdpi_hip.so, C-ABI in
include/dpi.h), called through ctypes.  PyTorch-ROCm provides device memory, streams and
torch.distributed (RCCL) only.
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401
from .equations import Cha, GBMEquationComplexExact, OUProcessEquation  # noqa: F401
from .solution import DeviceNet, PISGradNet, ZeroSolution, construct_mlp  # noqa: F401
from .data import OnlineDataGenerator  # noqa: F401
