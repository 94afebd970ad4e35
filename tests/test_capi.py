"""The C-ABI library builds, loads on a host without a GPU, and exports exactly the symbols
include/dpi.h declares; the ctypes mirror's constants equal the header's."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "dpi.h"


def _header_functions():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"^\s*(?:int|size_t)\s+(dpi_\w+)\s*\(", txt, flags=re.M))


def _header_defines():
    return {k: int(v.strip("()")) for k, v in re.findall(r"#define\s+(DPI_\w+)\s+(\(?-?\d+\)?)", HEADER.read_text())}


def test_header_and_ctypes_agree():
    from deeppicarditeration_amd import _lib
    assert _header_functions() == set(_lib.SIGNATURES)
    for k, v in _header_defines().items():
        assert getattr(_lib, k) == v, k


def test_library_loads_and_exports_every_symbol():
    from deeppicarditeration_amd import _lib
    from deeppicarditeration_amd.build import OUT, build
    build()
    lib = _lib.load()
    assert lib.dpi_abi_version() == _lib.DPI_ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", str(OUT)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dpi_\w+)", out))
    assert _header_functions() <= exported


def test_host_side_argument_errors_without_gpu():
    import ctypes
    from deeppicarditeration_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.dpi_problem_create_cha(0, 1.0, 5.0, 1.0, h) == _lib.DPI_ERR_ARG
    assert "cha" in _lib.last_error()
    # the compiled state-dimension caps are named refusals (include/dpi.h): 256 for
    # the problems and MLP nets (the wide first-order instances), 128 for PISGradNet, the Hessian
    # labels and the TD estimators (tests/test_gpu_wide.py)
    assert lib.dpi_problem_create_cha(257, 1.0, 5.0, 1.0, h) == _lib.DPI_ERR_UNSUPPORTED
    assert "256" in _lib.last_error()
    assert lib.dpi_net_create_mlp(258, 2, (ctypes.c_int * 2)(16, 16), _lib.DPI_ACT_ELU,
                                  (ctypes.c_float * 1)(), 1, ctypes.byref(ctypes.c_void_p())) == _lib.DPI_ERR_UNSUPPORTED
    assert "256" in _lib.last_error()
    w = (ctypes.c_double * (2 * 258))()
    v = (ctypes.c_double * 2)(1.0, 1.0)
    assert lib.dpi_problem_create_gbm(257, 1.0, 1.0, 2, w, v, h) == _lib.DPI_ERR_UNSUPPORTED
    assert "256" in _lib.last_error()
    # activations: ELU and Tanh only
    assert lib.dpi_net_create_mlp(101, 2, (ctypes.c_int * 2)(16, 16), 3, (ctypes.c_float * 1)(), 1,
                                  ctypes.byref(ctypes.c_void_p())) == _lib.DPI_ERR_UNSUPPORTED
    assert lib.dpi_problem_create_cha(100, 1.0, 5.0, 1.0, h) == 0
    n = ctypes.c_void_p()
    assert lib.dpi_net_create_zero(n) == 0
    assert lib.dpi_workspace_bytes(h, n, 16, 4096) > 0
    # label call argument validation happens before any device work
    rc = lib.dpi_label_moments(h, n, ctypes.c_void_p(16), 4, 4096, 50, 1, 0, 0, 0, 100, 3, ctypes.c_void_p(16),
                               ctypes.c_void_p(16), 1 << 30, None)
    assert rc == _lib.DPI_ERR_ARG and "multiple of 64" in _lib.last_error()
    # n = 0 is an empty batch: scalar checks only, NULL data pointers accepted, nothing launched
    assert lib.dpi_sample_points(h, 0, 1, 0, 0, 1e-3, None, None) == 0
    assert lib.dpi_point_baseline(h, n, None, 0, None, 0, None) == 0
    assert lib.dpi_generate_with_gradients(h, n, None, 0, 4096, 50, 1, 0, 0, 3, 1e9, None, None, None, 0, None) == 0
    assert lib.dpi_label_finalize(h, None, 0, 4096, 3, 1e9, None, None, 0, None) == 0
    assert lib.dpi_sample_points(h, -1, 1, 0, 0, 1e-3, None, None) == _lib.DPI_ERR_ARG
    assert lib.dpi_generate_with_gradients(h, n, None, -1, 4096, 50, 1, 0, 0, 3, 1e9, None, None, None, 0,
                                           None) == _lib.DPI_ERR_ARG
    # estimator / precision settings validate their arguments
    assert lib.dpi_problem_set_estimate_delta_t(h, -0.1) == _lib.DPI_ERR_ARG
    assert lib.dpi_problem_set_estimate_delta_t(h, float("nan")) == _lib.DPI_ERR_ARG
    assert lib.dpi_problem_set_estimate_delta_t(h, 0.25) == 0 and lib.dpi_problem_set_estimate_delta_t(h, 0.0) == 0
    assert lib.dpi_problem_set_hessian_approximation(h, 256) == _lib.DPI_ERR_ARG
    assert lib.dpi_set_gemm_precision(7) == _lib.DPI_ERR_ARG
    assert lib.dpi_net_set_precision(None, 0) == _lib.DPI_ERR_ARG
    st = _lib.c_int(0)
    assert lib.dpi_net_status(None, 1, None, _lib.ctypes.byref(st)) == _lib.DPI_ERR_ARG
    # the status ring: slot range checked; a zero net has no words (reads 0, host only)
    assert lib.dpi_net_status_slot(n, _lib.DPI_STATUS_SLOTS, 1) == _lib.DPI_ERR_ARG
    assert lib.dpi_net_status_slot(n, -1, 0) == _lib.DPI_ERR_ARG
    assert lib.dpi_net_status_slot(n, 5, 1) == 0
    st.value = 7
    assert lib.dpi_net_status_peek(n, 5, _lib.ctypes.byref(st)) == 0 and st.value == 0
    assert lib.dpi_net_status_peek(n, 64, _lib.ctypes.byref(st)) == _lib.DPI_ERR_ARG
    assert lib.dpi_net_destroy(n) == 0 and lib.dpi_problem_destroy(h) == 0


def test_product_fails_loudly_without_library(tmp_path, monkeypatch):
    from deeppicarditeration_amd import _lib
    with pytest.raises(_lib.DPIError):
        _lib.load(tmp_path / "missing.so")


def test_library_is_built_from_this_tree():
    """The .so embeds the SHA-256 of the sources it was built from (dpi_build_id); the in-tree
    library must match the tree (build.needs_build compares the same hash, not mtimes)."""
    from deeppicarditeration_amd import _lib, build as B
    lib = _lib.load()
    assert _lib.build_id(lib) == B.source_hash()
    assert not B.needs_build()
    assert B.embedded_id() == B.source_hash()


def test_stale_library_needs_build_whatever_the_side_file_says(monkeypatch):
    """a checkout that changes csrc leaves the old .so in place; needs_build() reads
    the id embedded in the .so, so a stale library is rebuilt even if a .buildid file says
    otherwise."""
    from deeppicarditeration_amd import build as B
    monkeypatch.setattr(B, "source_hash", lambda: "0" * 64)
    assert B.needs_build()


def test_load_refuses_a_library_built_from_other_sources(monkeypatch):
    from deeppicarditeration_amd import _lib, build as B
    lib = _lib.load()
    monkeypatch.delenv("DPI_HIP_LIB", raising=False)
    monkeypatch.setattr(B, "source_hash", lambda: "0" * 64)
    with pytest.raises(_lib.DPIError, match="other sources"):
        _lib.check_build_id(lib, B.OUT)
    # an explicit DPI_HIP_LIB (an A/B variant) is the caller's choice: not checked
    monkeypatch.setenv("DPI_HIP_LIB", str(B.OUT))
    _lib.check_build_id(lib, B.OUT)


def test_workspace_forget_is_host_only():
    """dpi_workspace_forget drops host-side records only (no device work): callable without a GPU on
    any range, including one that holds no record, and on an empty one."""
    import ctypes

    from deeppicarditeration_amd import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(4096)
    assert lib.dpi_workspace_forget(ctypes.cast(buf, ctypes.c_void_p), 4096) == 0
    assert lib.dpi_workspace_forget(None, 0) == 0
