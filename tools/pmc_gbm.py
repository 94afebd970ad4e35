"""GBM integral-estimator launches (K = 1: network phase dominated; K = 50) for PMC passes."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.perf_gbm import M, make  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

for net, K in (("zero", 1), ("mlp", 1), ("mlp", 50)):
    gen, tx, ws = make(net, K, 100)
    for _ in range(2):
        gen.label_moments(tx, 0, M, 0, M, L.DPI_INTEGRAL, ws)
    torch.cuda.synchronize()
    print(net, K, "done", flush=True)
