"""k_paths launches for PMC passes: the bench network (4x128, K=50 and K=1) under the fp32 and the
fp16-split fused MLP, plus the RNG-only kernel (ZeroSolution, K=50)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.perf_probe import make  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

lib = L.load()
for net, K, mode in (("zero", 50, 2), ("128x4", 50, 0), ("128x4", 50, 2), ("128x4", 1, 0), ("128x4", 1, 2)):
    L.check(lib.dpi_set_gemm_precision(mode), "gemm")
    gen, tx, ws = make(net, K)
    for _ in range(2):
        gen.label_moments(tx, 0, 4096, 0, 4096, L.DPI_BOTH, ws)
    torch.cuda.synchronize()
    print(net, K, mode, "done", flush=True)
