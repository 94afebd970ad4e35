"""Multi-rank label sharding (deeppicarditeration_amd/sharding.py) on CPU with the gloo backend:
world_size 2 ranks split the MC indices, all-gather their moments and reduce them with the
canonical tree; the labels must equal the single-rank result bit for bit.  The per-rank moment
computation is the oracle (fp64 contributions -> fp32 64-path blocks -> canonical tree), standing
in for dpi_label_moments, so this checks the sharding logic and collective, not the kernel."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dpi_oracle as O

NX, M, K, N = 100, 512, 3, 3


def _problem():
    rng = np.random.default_rng(0)
    eq = O.Cha(NX, 1.0, 5.0, 1.0)
    W = [rng.normal(0, 0.1, (16, NX + 1)), rng.normal(0, 0.25, (16, 16)), rng.normal(0, 0.25, (1, 16))]
    b = [rng.normal(0, 0.1, 16), rng.normal(0, 0.1, 16), rng.normal(0, 0.1, 1)]
    net = O.MLP(W, b, ["ELU", "ELU"])
    tx = O.sample_points(eq, N, seed=7)
    return eq, net, tx


class OracleGen:
    """Stands in for OnlineDataGenerator's moment building blocks (same method names)."""

    def __init__(self, eq, net):
        self.eq, self.net = eq, net
        self.n_estimate_terminal = self.n_estimate_integral = M
        self.gx = None

    def point_baseline(self, tx, ws=None):
        return tx if ws is None else ws

    def workspace_bytes(self, n, M_):
        return 8

    def label_moments(self, tx, point_base, M_, m0, m1, flags, ws):
        out = np.zeros((tx.shape[0], 2, NX + 1), np.float32)
        gx = []
        for r in range(tx.shape[0]):
            c, g = O.path_contributions(self.eq, self.net, tx[r], point_base + r, np.arange(m0, m1), K, 7,
                                        flags=flags & 3)
            gx.append(g)
            blocks = c.reshape(-1, 64, NX + 1)
            s1 = np.stack([O.tree_sum_f32(bk.astype(np.float32)) for bk in blocks])  # per-block sums
            s2 = np.stack([O.tree_sum_f32((bk.astype(np.float32)) ** 2) for bk in blocks])
            out[r, 0] = O.tree_sum_f32(s1)
            out[r, 1] = O.tree_sum_f32(s2)
        self.gx = np.array(gx)
        return torch.from_numpy(out)

    def moments_reduce(self, parts):
        return torch.from_numpy(O.tree_sum_f32(parts.numpy()))

    def finalize(self, mom, M_, flags, ws, bound=None):
        y = mom[:, 0].numpy() / M_
        if flags & 1:  # the terminal estimator adds g(x) (data.py:925)
            y[:, 0] += self.gx
        return torch.from_numpy(y)

    def label_moments_finalize(self, tx, point_base, M_, flags, ws, bound=None):
        """The single-rank call (dpi_label_moments_finalize): all of [0, M), finalized."""
        mom = self.label_moments(tx, point_base, M_, 0, M_, flags, ws)
        return self.finalize(mom, M_, flags, ws), mom


class OracleGenTwoPhase(OracleGen):
    """For begin()/end(): g(x) per batch is recomputed at finalize (the device path keeps it in the
    batch's own workspace)."""

    def finalize(self, mom, M_, flags, ws, bound=None):
        y = mom[:, 0].numpy() / M_
        if flags & 1:
            y[:, 0] += self.eq.g(self._tx[:, 1:])[:, 0]
        return torch.from_numpy(y)

    def label_moments(self, tx, point_base, M_, m0, m1, flags, ws):
        self._tx = np.asarray(tx)
        return super().label_moments(tx, point_base, M_, m0, m1, flags, ws)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    lab = ShardedLabeler(OracleGen(eq, net), rank=rank, world=world)
    y = lab.labels(tx, 0)
    q.put((rank, y.numpy()))
    dist.destroy_process_group()


def _worker_two_phase(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    lab = ShardedLabeler(OracleGenTwoPhase(eq, net), rank=rank, world=world)
    # the bench's pipeline: batch b + 1 begins (moments, async all-gather) before batch b ends
    pa = lab.begin(tx, 0)
    pb = lab.begin(tx, 100)
    ya = lab.end(pa)
    yb = lab.end(pb)
    q.put((rank, ya.numpy(), yb.numpy()))
    dist.destroy_process_group()


def test_two_rank_gloo_two_phase_pipeline_equals_labels():
    """ShardedLabeler.begin/end (async all-gather, two batches in flight) give the same labels,
    bit for bit, as the single-rank labels() of each batch."""
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    single_a = ShardedLabeler(OracleGen(eq, net), 0, 1).labels(tx, 0).numpy()
    single_b = ShardedLabeler(OracleGen(eq, net), 0, 1).labels(tx, 100).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_two_phase, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (a, b) for r, a, b in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert res[r][0].tobytes() == single_a.tobytes()
        assert res[r][1].tobytes() == single_b.tobytes()


def test_begin_refuses_a_third_pending_batch():
    """Two workspaces alternate: a third begin() before any end() would overwrite a pending
    batch's per-point baseline, so it raises; after one end() the pipeline continues."""
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    lab = ShardedLabeler(OracleGenTwoPhase(eq, net), 0, 1)
    pa = lab.begin(tx, 0)
    pb = lab.begin(tx, 100)
    with pytest.raises(RuntimeError, match="pending"):
        lab.begin(tx, 200)
    lab.end(pa)
    pc = lab.begin(tx, 200)
    lab.end(pb)
    lab.end(pc)


def test_shard_ranges():
    from deeppicarditeration_amd.sharding import ShardedLabeler
    assert [ShardedLabeler(None, r, 4).shard(4096) for r in range(4)] == [(0, 1024), (1024, 2048), (2048, 3072),
                                                                           (3072, 4096)]
    with pytest.raises(ValueError):
        ShardedLabeler(None, 0, 3).shard(4096)


def test_two_rank_gloo_labels_equal_single_rank():
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    single = ShardedLabeler(OracleGen(eq, net), 0, 1).labels(tx, 0).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0].tobytes() == res[1].tobytes()
    assert res[0].tobytes() == single.tobytes()
    # and the labels are the oracle's labels (to fp32 summation error)
    ref = O.labels_grad(eq, net, tx, M, K, 7)
    assert O.rel_l2(single, ref) < 1e-5


# ----------------------------------------------------------------------------- Hessian labels
MH, KH, NH = 256, 2, 2


def _problem_hess():
    from pathlib import Path
    d = Path(__file__).resolve().parents[1] / "deeppicarditeration_amd" / "problem_data"
    eq = O.GBMEquationComplexExact(NX, np.load(d / "gbm_2nodes_w_100d_case_1.npy"),
                                   np.load(d / "gbm_2nodes_v_100d_case_1.npy"))
    rng = np.random.default_rng(1)
    net = O.MLP([rng.normal(0, 0.1, (16, NX + 1)), rng.normal(0, 0.25, (1, 16))],
                [rng.normal(0, 0.1, 16), rng.normal(0, 0.1, 1)], ["ELU"])
    return eq, net, O.sample_points(eq, NH, seed=9)


class OracleGenHess:
    """Stands in for the Hessian-label building blocks of OnlineDataGenerator."""

    def __init__(self, eq, net):
        self.eq, self.net = eq, net
        self.n_estimate_terminal = self.n_estimate_integral = MH
        self.gx = None

    def point_baseline(self, tx, hessians=False):
        assert hessians
        return tx

    def label_moments_hessians(self, tx, point_base, M_, m0, m1, ws, flags=3):
        n = tx.shape[0]
        mom = np.zeros((n, 2, NX + 1), np.float32)
        hs = np.zeros((n, NX * NX), np.float32)
        gx = []
        for r in range(n):
            c, h, g = O.path_contributions_hess(self.eq, self.net, tx[r], point_base + r, np.arange(m0, m1), KH, 9,
                                                flags=flags)
            gx.append(g)
            cb, hb = c.reshape(-1, 64, NX + 1), h.reshape(-1, 64, NX * NX)
            mom[r, 0] = O.tree_sum_f32(np.stack([O.tree_sum_f32(b.astype(np.float32)) for b in cb]))
            mom[r, 1] = O.tree_sum_f32(np.stack([O.tree_sum_f32(b.astype(np.float32) ** 2) for b in cb]))
            hs[r] = O.tree_sum_f32(np.stack([O.tree_sum_f32(b.astype(np.float32)) for b in hb]))
        self.gx = np.array(gx)
        return torch.from_numpy(mom), torch.from_numpy(hs)

    def sums_reduce(self, parts):
        return torch.from_numpy(O.tree_sum_f32(parts.numpy()))

    def finalize_hessians(self, mom, hs, M_, ws, bound=None, flags=3):
        y = mom[:, 0].numpy() / M_
        if flags & 1:
            y[:, 0] += self.gx
        return torch.from_numpy(np.concatenate([y, hs.numpy() / M_], -1))


def _worker_hess(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem_hess()
    y = ShardedLabeler(OracleGenHess(eq, net), rank=rank, world=world).labels_hessians(tx, 0)
    q.put((rank, y.numpy()))
    dist.destroy_process_group()


def test_two_rank_gloo_hessian_labels_equal_single_rank():
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem_hess()
    single = ShardedLabeler(OracleGenHess(eq, net), 0, 1).labels_hessians(tx, 0).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_hess, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0].tobytes() == res[1].tobytes() == single.tobytes()
    ref = O.labels_grad_hess(eq, net, tx, MH, KH, 9)
    assert O.rel_l2(single, ref) < 1e-5


def test_four_rank_gloo_labels_equal_single_rank():
    """A 4-rank rehearsal of the N = 4 bench layout (M = 512 -> 128 MC indices per rank): every rank's
    labels equal the single-rank labels bit for bit (M / (64 G) = 2, a power of two)."""
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    single = ShardedLabeler(OracleGen(eq, net), 0, 1).labels(tx, 0).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(4):
        assert res[r].tobytes() == single.tobytes(), r


def _worker_non_pow2(rank, world, port, q):
    """M = 384 over 2 ranks: 3 blocks of 64 paths per rank (not a power of two)."""
    import warnings
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeppicarditeration_amd.sharding import ShardBitIdentityWarning, ShardedLabeler
    eq, net, tx = _problem()
    gen = OracleGen(eq, net)
    gen.n_estimate_terminal = gen.n_estimate_integral = 384
    lab = ShardedLabeler(gen, rank=rank, world=world)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        y = lab.labels(tx, 0)
    q.put((rank, y.numpy(), [issubclass(x.category, ShardBitIdentityWarning) for x in w]))
    dist.destroy_process_group()


def test_two_rank_gloo_non_power_of_two_blocks_warns():
    """M / (64 G) not a power of two: every rank warns that the labels lose bit-identity with the
    single-GPU call, and the labels still agree with it to fp32 rounding."""
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    g1 = OracleGen(eq, net)
    g1.n_estimate_terminal = g1.n_estimate_integral = 384
    single = ShardedLabeler(g1, 0, 1).labels(tx, 0).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_non_pow2, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (y, w) for r, y, w in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        y, w = res[r]
        assert any(w), f"rank {r} did not warn"
        np.testing.assert_allclose(y, single, rtol=1e-5, atol=1e-6)


def test_power_of_two_shards_do_not_warn():
    import warnings
    from deeppicarditeration_amd.sharding import ShardedLabeler
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        for G in (1, 2, 4, 8):
            for r in range(G):
                ShardedLabeler(None, r, G).shard(4096)


# ------------------------------------------- n_estimate_terminal != n_estimate_integral
MT2, MI2 = 256, 128  # the terminal estimator over twice the integral's paths


def _worker_unequal(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    g = OracleGenTwoPhase(eq, net)
    g.n_estimate_terminal, g.n_estimate_integral = MT2, MI2
    lab = ShardedLabeler(g, rank=rank, world=world)
    y = lab.labels(tx, 0).numpy()
    pa = lab.begin(tx, 0)
    pb = lab.begin(tx, 100)
    ya, yb = lab.end(pa).numpy(), lab.end(pb).numpy()
    eqh, neth, txh = _problem_hess()
    gh = OracleGenHess(eqh, neth)
    gh.n_estimate_terminal, gh.n_estimate_integral = 2 * MH, MH
    yh = ShardedLabeler(gh, rank=rank, world=world).labels_hessians(txh, 0).numpy()
    q.put((rank, y, ya, yb, yh))
    dist.destroy_process_group()


def test_two_rank_gloo_unequal_estimator_counts():
    """n_estimate_terminal = 2 n_estimate_integral: each estimator pass shards its own M over the
    ranks (one all-gather of both passes' moments); labels(), the begin()/end() pipeline and the
    Hessian labels equal the single-rank labels bit for bit on every rank, and the oracle's labels
    with separate counts (labels_grad / labels_grad_hess MT=) to fp32 summation error."""
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, tx = _problem()
    g1 = OracleGenTwoPhase(eq, net)
    g1.n_estimate_terminal, g1.n_estimate_integral = MT2, MI2
    single = ShardedLabeler(g1, 0, 1).labels(tx, 0).numpy()
    single_b = ShardedLabeler(g1, 0, 1).labels(tx, 100).numpy()
    eqh, neth, txh = _problem_hess()
    gh = OracleGenHess(eqh, neth)
    gh.n_estimate_terminal, gh.n_estimate_integral = 2 * MH, MH
    single_h = ShardedLabeler(gh, 0, 1).labels_hessians(txh, 0).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_unequal, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        y, ya, yb, yh = res[r]
        assert y.tobytes() == single.tobytes() and ya.tobytes() == single.tobytes(), r
        assert yb.tobytes() == single_b.tobytes(), r
        assert yh.tobytes() == single_h.tobytes(), r
    assert O.rel_l2(single, O.labels_grad(eq, net, tx, MI2, K, 7, MT=MT2)) < 1e-5
    assert O.rel_l2(single_h, O.labels_grad_hess(eqh, neth, txh, MH, KH, 9, MT=2 * MH)) < 1e-5


def test_estimator_sets():
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq, net, _ = _problem()
    g = OracleGen(eq, net)
    assert ShardedLabeler(g).estimator_sets() == [(M, 3)]
    g.n_estimate_terminal = 2 * M
    assert ShardedLabeler(g).estimator_sets() == [(2 * M, 1), (M, 2)]
    assert ShardedLabeler(g).estimator_sets(1) == [(2 * M, 1)]
    assert ShardedLabeler(g).estimator_sets(2) == [(M, 2)]
