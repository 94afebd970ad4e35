"""Three k_paths launches for PMC passes: RNG only (ZeroSolution, K=50), full (4x128, K=50),
MLP-dominated (4x128, K=1).  Each variant is a separate kernel instantiation or launch."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.perf_probe import make  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

for net, K in (("zero", 50), ("128x4", 50), ("128x4", 1)):
    gen, tx, ws = make(net, K)
    for _ in range(3):
        gen.label_moments(tx, 0, 4096, 0, 4096, L.DPI_BOTH, ws)
    torch.cuda.synchronize()
    print(net, K, "done", flush=True)
