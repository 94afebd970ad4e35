"""The PISGradNet pipeline's ablation switches give bitwise-identical labels: the split GEMM on 128 x 128
tiles (k_gemm_x3h, the default) or on 256 x 128 tiles (DPI_X3_TILE=256), the latter with or without its
staged DELU epilogue operands (DPI_X3_STAGE), and 4 or 2 Philox chains per rollout wave
(DPI_PIS_UNROLL).  Every per-output product and sum runs in the same order in all of them.  The
switches are read once per process, so each variant labels the same batch in a process of its own;
3 points x 1024 paths + 3 baseline rows also leave a partial last m-tile (waves wholly past M)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[2])
import deeppicarditeration_amd as dpi
eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                           alpha_scale=4.0)
torch.manual_seed(7)
net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=1024,
                              n_estimate_integral=1024, n_euler_steps=10, seed=3, epoch=1)
tx, y = gen.sample_with_gradients(3)
torch.cuda.synchronize()
np.save(sys.argv[1], y.cpu().numpy())
"""


def _labels(tmp_path, name, **env):
    out = str(tmp_path / f"{name}.npy")
    e = dict(os.environ)
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([sys.executable, "-c", SCRIPT, out, ROOT], env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(out)


def test_pisgradnet_ablation_switches_are_bitwise_equal(tmp_path):
    ref = _labels(tmp_path, "default")
    assert np.isfinite(ref).all()
    for name, env in [("tile256", {"DPI_X3_TILE": 256}),
                      ("tile256_nostage", {"DPI_X3_TILE": 256, "DPI_X3_STAGE": 0}),
                      ("unroll2", {"DPI_PIS_UNROLL": 2})]:
        y = _labels(tmp_path, name, **env)
        assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), (name, np.abs(y - ref).max())
