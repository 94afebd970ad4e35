"""Why does k_paths take longer inside the bench step than back to back?  Time label_moments
(a) back to back on fixed points, (b) inside full steps (sample + baseline + moments + finalize),
(c) back to back on fresh points (sample + baseline outside the timed kernel pair)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.perf_probe import make  # noqa: E402
from deeppicarditeration_amd import _lib as L  # noqa: E402

gen, tx, ws = make("128x4", 50)
M = 4096


def ev():
    return torch.cuda.Event(enable_timing=True)


def mode_a(reps=20):
    for _ in range(3):
        gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    a, b = ev(), ev()
    a.record()
    for _ in range(reps):
        gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def mode_b(reps=20, sync_between=False):
    times = []
    for r in range(reps + 3):
        t2, pb = gen.sample_t_and_x(16)
        w2 = gen.point_baseline(t2)
        if sync_between:
            torch.cuda.synchronize()
        a, b = ev(), ev()
        a.record()
        mom = gen.label_moments(t2, pb, M, 0, M, L.DPI_BOTH, w2)
        b.record()
        gen.finalize(mom, M, L.DPI_BOTH, w2)
        times.append((a, b))
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in times[3:]]
    return sorted(t)[len(t) // 2]


for rnd in range(3):
    print(f"round {rnd}: fixed back-to-back {mode_a()*1e3:.1f} us | in-step {mode_b()*1e3:.1f} us | "
          f"in-step synced {mode_b(sync_between=True)*1e3:.1f} us", flush=True)
