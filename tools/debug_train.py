import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from test_gpu_train import CHA
from deeppicarditeration_amd.config import load_cfg
from deeppicarditeration_amd.runner import PicardRunner

Path("gpurun_out/dbg").mkdir(parents=True, exist_ok=True)
Path("gpurun_out/dbg/cha.yaml").write_text(CHA.format(name="gpurun_out/dbg/run"))
r = PicardRunner(load_cfg("gpurun_out/dbg/cha.yaml"))
r.i = 1
d = r.cfg.DATA
from deeppicarditeration_amd.data import OnlineDataGenerator
for ppc in (384, 1024, 128):
    gen = OnlineDataGenerator(r.equation, r.u_current, r.N, r.i, device=r.device, **dict(d.kwargs),
                              hessian_approximation=d.HESSIAN_APPROXIMATION, sample_bound=d.SAMPLE_BOUND,
                              estimate_terminal=d.ESTIMATE_TERMINAL, estimate_integral=d.ESTIMATE_INTEGRAL,
                              estimate_delta_t=d.ESTIMATE_DELTA_T, n_euler_steps=d.EULER_STEPS, seed=d.SEED)
    print("gen", ppc, gen.K, gen.seed, gen.epoch, gen.eps, gen.sample_bound, gen.n_estimate_terminal, flush=True)
    done = 0
    while done < 1024:
        n = min(ppc, 1024 - done)
        pb = gen.point_base
        tx, y = gen.sample_with_gradients(n)
        bad = (~torch.isfinite(y)).any(dim=1)
        mom = gen.last_moments
        print(" call pb", pb, "n", n, "bad", int(bad.sum()), flush=True)
        if bad.any():
            k = int(bad.nonzero()[0])
            print("  row", k, "tx", tx[k].tolist())
            print("  y", y[k].tolist())
            print("  mom", mom[k].tolist())
        done += n
