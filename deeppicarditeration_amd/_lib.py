"""ctypes binding of libdpi_hip.so (the C-ABI declared in include/dpi.h).

There is no fallback: if the library is missing or fails to load, every label call raises.
"""
import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DPI_HIP_LIB", _HERE / "libdpi_hip.so"))

# constants mirrored from include/dpi.h (checked against the header by tests/test_capi.py)
DPI_ABI_VERSION = 7
DPI_LAUNCH_TIMERS = 256  # include/dpi.h
DPI_OK, DPI_ERR_ARG, DPI_ERR_UNSUPPORTED, DPI_ERR_HIP, DPI_ERR_WORKSPACE = 0, -1, -2, -3, -4
DPI_TAG_T, DPI_TAG_X0, DPI_TAG_X, DPI_TAG_TERM, DPI_TAG_S, DPI_TAG_INT, DPI_TAG_SDGD, DPI_TAG_HTERM, DPI_TAG_HINT = range(1, 10)
DPI_EQ_CHA, DPI_EQ_OU, DPI_EQ_GBM = 1, 2, 3
DPI_ACT_ELU, DPI_ACT_TANH = 1, 2
DPI_TERMINAL, DPI_INTEGRAL, DPI_BOTH = 1, 2, 3
DPI_PREPARED = 4  # dpi_label_moments: dpi_label_prepare already ran with the same arguments
DPI_PATH_BLOCK = 64
DPI_PATHS_PER_CALL_MAX = 1024 * DPI_PATH_BLOCK
DPI_GEMM_F32, DPI_GEMM_F16X3, DPI_GEMM_AUTO = 0, 1, 2
DPI_STATUS_NONFINITE = 1
DPI_STATUS_HANDOFF = 2
DPI_STATUS_SLOTS = 64

c_int, c_double, c_float, c_size_t, c_void_p, c_uint32, c_uint64 = (
    ctypes.c_int, ctypes.c_double, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64)
P = ctypes.POINTER

# name -> (restype, argtypes); the exact exported surface of include/dpi.h
SIGNATURES = {
    "dpi_abi_version": (c_int, []),
    "dpi_last_error": (c_int, [ctypes.c_char_p, c_size_t]),
    "dpi_problem_create_cha": (c_int, [c_int, c_double, c_double, c_double, P(c_void_p)]),
    "dpi_problem_create_ou": (c_int, [c_int, c_double, c_double, c_double, c_double, c_double, c_int,
                                      P(c_double), P(c_double), P(c_double), P(c_void_p)]),
    "dpi_problem_create_gbm": (c_int, [c_int, c_double, c_double, c_int, P(c_double), P(c_double), P(c_void_p)]),
    "dpi_problem_set_hessian_approximation": (c_int, [c_void_p, c_int]),
    "dpi_problem_set_estimate_delta_t": (c_int, [c_void_p, c_double]),
    "dpi_problem_destroy": (c_int, [c_void_p]),
    "dpi_net_create_zero": (c_int, [P(c_void_p)]),
    "dpi_net_create_mlp": (c_int, [c_int, c_int, P(c_int), c_int, P(c_float), c_size_t, P(c_void_p)]),
    "dpi_net_create_pisgrad": (c_int, [c_int, c_int, P(c_int), c_double, P(c_float), c_size_t, P(c_void_p)]),
    "dpi_net_destroy": (c_int, [c_void_p]),
    "dpi_set_gemm_precision": (c_int, [c_int]),
    "dpi_net_set_precision": (c_int, [c_void_p, c_int]),
    "dpi_net_status": (c_int, [c_void_p, c_int, c_void_p, P(c_int)]),
    "dpi_net_status_slot": (c_int, [c_void_p, c_int, c_int]),
    "dpi_net_status_peek": (c_int, [c_void_p, c_int, P(c_int)]),
    "dpi_build_id": (c_int, [ctypes.c_char_p, c_size_t]),
    "dpi_launch_timer_arm": (c_int, [c_int]),
    "dpi_launch_timer_ms": (c_int, [c_int, P(ctypes.c_float)]),
    "dpi_workspace_bytes": (c_size_t, [c_void_p, c_void_p, c_int, c_int]),
    "dpi_workspace_bytes_prepared": (c_size_t, [c_void_p, c_void_p, c_int, c_int]),
    "dpi_sample_points": (c_int, [c_void_p, c_int, c_uint64, c_uint32, c_uint32, c_float, c_void_p, c_void_p]),
    "dpi_sample_points_t": (c_int, [c_void_p, c_int, c_uint64, c_uint32, c_uint32, c_float, c_int, c_void_p,
                                    c_void_p]),
    "dpi_point_baseline": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "dpi_label_moments": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32, c_uint32,
                                  c_int, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "dpi_label_moments_finalize": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32,
                                           c_uint32, c_int, c_float, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "dpi_label_prepare": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32, c_uint32,
                                  c_int, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "dpi_moments_reduce": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "dpi_label_finalize": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_size_t,
                                   c_void_p]),
    "dpi_generate_with_gradients": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32,
                                            c_uint32, c_int, c_float, c_void_p, c_void_p, c_void_p, c_size_t,
                                            c_void_p]),
    "dpi_sample_with_gradients": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32, c_uint32,
                                          c_float, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_size_t, c_void_p]),
    "dpi_sample_points_baseline": (c_int, [c_void_p, c_void_p, c_int, c_uint64, c_uint32, c_uint32, c_float, c_int,
                                           c_void_p, c_void_p, c_size_t, c_void_p]),
    "dpi_workspace_bytes_hessians": (c_size_t, [c_void_p, c_void_p, c_int, c_int]),
    "dpi_workspace_bytes_hessians_prepared": (c_size_t, [c_void_p, c_void_p, c_int, c_int]),
    "dpi_workspace_forget": (c_int, [c_void_p, c_size_t]),
    "dpi_label_moments_hessians": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64, c_uint32,
                                           c_uint32, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p]),
    "dpi_label_finalize_hessians": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p,
                                            c_void_p, c_size_t, c_void_p]),
    "dpi_sums_reduce": (c_int, [c_void_p, c_int, c_size_t, c_void_p, c_void_p]),
    "dpi_generate_with_gradients_and_hessians": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_uint64,
                                                         c_uint32, c_uint32, c_float, c_void_p, c_void_p, c_size_t,
                                                         c_void_p]),
}

_lib = None


class DPIError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and return the library; raises DPIError if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise DPIError(f"libdpi_hip.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; "
                       f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dpi_abi_version() != DPI_ABI_VERSION:
        raise DPIError(f"ABI mismatch: library {lib.dpi_abi_version()} != {DPI_ABI_VERSION}")
    check_build_id(lib, p)
    if path is None:
        _lib = lib
    return lib


def build_id(lib):
    buf = ctypes.create_string_buffer(80)
    lib.dpi_build_id(buf, 80)
    return buf.value.decode()


def check_build_id(lib, path):
    """The in-tree library must have been built from the tree's sources (build.source_hash): a
    library built from other sources would run kernels the tests and the bench do not describe.
    Skipped for an explicit DPI_HIP_LIB (A/B variants, tools/build_variant.py) and where the
    sources are absent."""
    if "DPI_HIP_LIB" in os.environ or Path(path).resolve() != (_HERE / "libdpi_hip.so").resolve():
        return
    from . import build as B
    if not B.CSRC.is_dir():
        return
    want, got = B.source_hash(), build_id(lib)
    if got != want:
        raise DPIError(f"{path} was built from other sources (build id {got[:12]}, tree {want[:12]}): rebuild it with "
                       "`python -m deeppicarditeration_amd.build` (hipcc --offload-arch=gfx950; `--force` rebuilds every "
                       "object)")


def last_error(lib=None):
    lib = lib or load()
    buf = ctypes.create_string_buffer(512)
    lib.dpi_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise DPIError(f"{what} failed ({rc}): {last_error()}")
