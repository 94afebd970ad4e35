"""`picard train` across ranks on CPU (gloo, world_size 2): every rank generates the labels of its
Monte-Carlo shard through ShardedLabeler, rank 0 fits and broadcasts, and both ranks must hold the
single-rank labels bit for bit and the same network afterwards.  The per-rank label moments come
from the oracle (as in test_sharding.py), standing in for the HIP kernel; everything else — the
runner, the sampler wiring, the all-gather, the fit, the broadcast — is the product code."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_sharding import OracleGen, _problem

CFG = """NAME: {name}
EQUATION:
  cls: Cha
  kwargs: {{nx: 100, alpha: 1.0, k: 5.0, T: 1.0}}
PICARD: {{N: 2}}
FORCE: true
DATA:
  DATA_SIZE: 6
  POINTS_PER_CALL: 3
  kwargs: {{t_always_uniform: true, n_estimate_terminal: 512, n_estimate_integral: 512}}
TRAIN:
  N_EPOCHS: 2
  BATCH_SIZE: 4
  LOSS: {{SCALER: {{cls: FixedLossScaler, kwargs: {{fixed_weight: 0.1}}}}}}
NETWORK:
  NEURONS: [8, 8]
  ACTIVATIONS: [ELU, ELU]
  BOUND: None
EVAL: {{L2_N_POINTS: 16}}
"""


class OracleSampleGen(OracleGen):
    """OracleGen plus the sampler of OnlineDataGenerator (point counters advance per call)."""

    def __init__(self, eq, net):
        super().__init__(eq, net)
        self.point_base = 0

    def sample_t_and_x(self, n):
        from oracle import dpi_oracle as O
        pb = self.point_base
        self.point_base += n
        return torch.from_numpy(O.sample_points(self.eq, n, seed=7, point_base=pb)).float(), pb

    def sample_with_gradients(self, n):  # single rank: the whole MC range in one shard
        from deeppicarditeration_amd.sharding import ShardedLabeler
        return ShardedLabeler(self, 0, 1).sample_with_gradients(n)


def _runner(tmp, rank, world):
    from deeppicarditeration_amd.config import load_cfg
    from deeppicarditeration_amd.runner import PicardRunner
    f = os.path.join(tmp, "cfg.yaml")
    if rank == 0:
        with open(f, "w") as fh:
            fh.write(CFG.format(name=os.path.join(tmp, f"run{world}")))
    if world > 1:
        dist.barrier()

    class R(PicardRunner):
        def make_generator(self, solution, **kw):
            eq, net, _ = _problem()
            return OracleSampleGen(eq, net)

    torch.manual_seed(rank)  # different initial weights per rank: the broadcast must equalise them
    return R(load_cfg(f), device="cpu", rank=rank, world=world)


def _worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=60))
    r = _runner(tmp, rank, world)
    labels = []
    for _ in range(2):
        r.i += 1
        labels.append(r.labels())
        r.i -= 1
        r.run_one()
    sd = {k: v.numpy().copy() for k, v in r.u_current.state_dict().items()}
    q.put((rank, [(a.numpy(), b.numpy()) for a, b in labels], sd, len(r.history)))
    dist.destroy_process_group()


def test_two_rank_picard_train_labels_and_weights(tmp_path):
    ref = _runner(str(tmp_path), 0, 1)
    ref.i = 1
    tx1, y1 = ref.labels()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (lab, sd, nh) for r, lab, sd, nh in (q.get(timeout=180) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r][0][0][0].tobytes() == tx1.numpy().tobytes()
        assert res[r][0][0][1].tobytes() == y1.numpy().tobytes()
    assert res[0][2] == 2 and res[1][2] == 0  # only rank 0 fits and logs
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k
    assert (tmp_path / "run2" / "model_2.pt").exists()


def _worker_fail(rank, world, port, tmp, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=120))
    try:
        if mode == "exists":
            if rank == 0:
                d = os.path.join(tmp, f"run{world}")
                os.makedirs(d, exist_ok=True)
                open(os.path.join(d, "keep"), "w").close()
            dist.barrier()
            from deeppicarditeration_amd.config import load_cfg
            from deeppicarditeration_amd.runner import PicardRunner
            f = os.path.join(tmp, "cfg.yaml")
            if rank == 0:
                with open(f, "w") as fh:
                    fh.write(CFG.format(name=os.path.join(tmp, f"run{world}")).replace("FORCE: true", "FORCE: false"))
            dist.barrier()
            PicardRunner(load_cfg(f), device="cpu", rank=rank, world=world)
        else:
            r = _runner(tmp, rank, world)

            def boom(*a, **k):
                raise ValueError("fit exploded")
            r.fit = boom
            r.run_one()
        q.put((rank, "no error"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, type(e).__name__))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["exists", "fit"])
def test_rank0_failure_stops_every_rank(tmp_path, mode):
    """A failure on rank 0 alone (existing experiment directory without FORCE; an exception in the
    fit) ends every rank with an error before the next collective, instead of leaving the other
    ranks blocked in a collective until the process-group timeout (120 s here)."""
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + os.getpid() % 100 + (0 if mode == "exists" else 100)
    t0 = time.time()
    procs = [ctx.Process(target=_worker_fail, args=(r, 2, port, str(tmp_path), mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert time.time() - t0 < 100
    assert res[0] == ("FileExistsError" if mode == "exists" else "ValueError")
    assert res[1] == "RuntimeError"


def test_fit_rebatching_matches_cache_to_memory_wrapper(tmp_path, monkeypatch):
    """BATCH_SIZE != points per generator call: the reference re-batches through
    CacheToMemoryWrapper(batch_size, drop_last=True, shuffle=SHUFFLE) from the first epoch
    (picard/data.py:1718-1731); equal sizes stream epoch 0 in draw order (data.py:1746-1760)."""
    from deeppicarditeration_amd import runner as R
    seen = []

    def fake_train_steps(net, objective, opt, batches, sched):
        seen.append((batches.batch_size, batches.drop_last, batches.shuffle, len(batches)))
        return torch.zeros(len(batches))
    monkeypatch.setattr(R, "train_steps", fake_train_steps)
    r = _runner(str(tmp_path), 0, 1)
    tx, y = torch.zeros(6, 101), torch.zeros(6, 101)
    r.cfg = load_cfg_with(r, ["DATA.SHUFFLE", "True"])
    r.fit(r.new_network(), tx, y)  # BATCH_SIZE 4, POINTS_PER_CALL 3, 2 epochs
    assert seen == [(4, True, True, 1), (4, True, True, 1)]
    seen.clear()
    r.cfg = load_cfg_with(r, ["DATA.SHUFFLE", "True", "TRAIN.BATCH_SIZE", "3"])
    r.fit(r.new_network(), tx, y)
    assert seen == [(3, False, False, 2), (3, False, True, 2)]


def load_cfg_with(r, overrides):
    from deeppicarditeration_amd.config import load_cfg
    f = r.exp_dir.parent / "cfg.yaml"
    return load_cfg(str(f), overrides)
