"""The generator surface the reference's data module reads (picard/data.py:53-85, :285-335,
:1620-1661) and the buffered dataset semantics of picard/dataset.py:20-137, on CPU.

The label calls are replaced by a counter generator (row r of the k-th point drawn carries the
value k), so these tests check the buffering, ordering, saver and wrapper logic, not the kernel —
tests/test_gpu_dataset.py drives the same objects with the HIP generator."""
import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader

from deeppicarditeration_amd import dataset as D
from deeppicarditeration_amd.data import OnlineDataGenerator
from picard_datamodule import PicardDataModuleStandIn, reference_data_cfg

NX = 3


class CountingGenerator:
    """batch_data_generator stand-in: rows numbered in draw order; y = 10 * row index."""

    def __init__(self):
        self.next = 0
        self.calls = []

    def __call__(self, n):
        self.calls.append(n)
        r = torch.arange(self.next, self.next + n, dtype=torch.float64)
        self.next += n
        return r[:, None].repeat(1, 1 + NX), 10 * r[:, None]


@pytest.mark.parametrize("nbuf, bs, plan", [(4, 8, (4, 32, 1, 32)), (1, 8, (1, 8, 1, 8)), (2.0000001, 8, (2, 16, 1, 16)),
                                            (0.25, 8, (1, 8, 4, 2)), (0.5, 6, (1, 6, 2, 3))])
def test_buffer_plan_matches_reference_rules(nbuf, bs, plan):
    assert D.buffer_plan(nbuf, bs) == plan


@pytest.mark.parametrize("nbuf, bs", [(0.3, 8), (0.25, 6), (1.5, 8), (0, 8), (-2, 8)])
def test_buffer_plan_rejects_what_the_reference_rejects(nbuf, bs):
    with pytest.raises(AssertionError):
        D.buffer_plan(nbuf, bs)


@pytest.mark.parametrize("nbuf", [3, 0.25])
def test_batches_come_out_in_draw_order(nbuf):
    gen = CountingGenerator()
    ds = D.IterableDatasetWithInternalBatch(96, nbuf, 8, gen)
    assert len(ds) == 12
    batches = list(ds)
    assert len(batches) == 12
    x = torch.cat([b[0] for b in batches])
    y = torch.cat([b[1] for b in batches])
    assert torch.equal(x[:, 0], torch.arange(96, dtype=torch.float64)) and torch.equal(y[:, 0], 10 * x[:, 0])
    assert all(b[0].shape == (8, 1 + NX) for b in batches)
    assert gen.calls == ([24] * 4 if nbuf == 3 else [2] * 48)


class _GuardedCounting(CountingGenerator):
    """CountingGenerator with the range-guard surface the dataset uses: a point counter (the
    generator's point_base) and deferred_range_check() groups that record verify / discard."""

    class _Group:
        def __init__(self, log):
            self.log = log

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def verify(self):
            self.log.append("verify")
            return 0

        def discard(self):
            self.log.append("discard")

    def __init__(self):
        super().__init__()
        self.log = []

    @property
    def point_base(self):
        return self.next

    @point_base.setter
    def point_base(self, v):
        self.next = v

    def deferred_range_check(self):
        return self._Group(self.log)


def test_guarded_dataset_abandoned_early_rewinds_the_drawn_ahead_buffer():
    """with a range guard the dataset draws buffer k+1 before it yields buffer k; a
    consumer that stops early leaves that buffer unread — it is discarded and the generator's point
    counter handed back, so the next draw starts where an unguarded dataset's would."""
    import itertools
    gen = _GuardedCounting()
    ds = D.IterableDatasetWithInternalBatch(96, 2, 8, gen, range_guard=gen)  # 6 buffers of 16 points
    got = list(itertools.islice(iter(ds), 3))  # buffer 0 and half of buffer 1
    assert torch.equal(torch.cat([b[0] for b in got])[:, 0], torch.arange(24, dtype=torch.float64))
    assert gen.point_base == 32 and gen.log[-1] == "discard"  # buffer 2 (points 32-47) drawn ahead, given back
    full = list(ds)  # a complete pass afterwards continues at 32, every buffer verified
    assert torch.equal(torch.cat([b[0] for b in full])[:, 0], torch.arange(32, 128, dtype=torch.float64))
    assert gen.log.count("verify") == 2 + 6


def test_size_must_be_a_multiple_of_the_buffer():
    with pytest.raises(AssertionError):
        D.IterableDatasetWithInternalBatch(100, 3, 8, CountingGenerator())
    ds = D.IterableDatasetWithInternalBatch(48, 3, 8, CountingGenerator())
    ds.set_size(96)
    assert len(ds) == 12
    with pytest.raises(AssertionError):
        ds.set_size(50)


def test_saver_records_every_buffer_and_closes():
    gen = CountingGenerator()
    ds = D.IterableDatasetWithInternalBatch(64, 2, 8, gen)
    saver = D.DeviceMemorySaver(64, [1 + NX, 1])
    closed = []
    saver.close = lambda: closed.append(True)
    ds.attach_saver(saver)
    with pytest.raises(AssertionError):
        ds.attach_saver(saver)
    got = list(ds)
    assert closed == [True] and saver.position == 64
    assert torch.equal(saver.data[0], torch.cat([b[0] for b in got]))
    with pytest.raises(ValueError):
        D.DeviceMemorySaver(8, [1]).create_torch_dataset(4)


def test_cache_to_memory_first_pass_streams_then_replays_the_cache():
    gen = CountingGenerator()
    w = D.CacheToMemoryWrapper(D.IterableDatasetWithInternalBatch(64, 2, 8, gen), shuffle=True, drop_last=True)
    w.init(64, [1 + NX, 1])
    first = torch.cat([b[0] for b in w])
    assert len(gen.calls) == 4
    second = list(w)
    assert len(gen.calls) == 4  # no new labels
    assert len(second) == len(w) == 8
    rows = torch.cat([b[0] for b in second])
    assert torch.equal(torch.sort(rows[:, 0]).values, first[:, 0])
    assert torch.equal(torch.cat([b[1] for b in second])[:, 0], 10 * rows[:, 0])  # pairs stay together


def test_cache_to_memory_with_a_different_batch_size_preloads():
    gen = CountingGenerator()
    w = D.CacheToMemoryWrapper(D.IterableDatasetWithInternalBatch(64, 2, 8, gen), batch_size=16, drop_last=True)
    w.init(64, [1 + NX, 1])
    assert len(gen.calls) == 4 and len(w) == 4
    b = list(w)
    assert [x.shape[0] for x, _ in b] == [16] * 4 and torch.equal(b[0][0][:, 0], torch.arange(16, dtype=torch.float64))


def test_dataloader_with_internal_batching():
    ds = D.IterableDatasetWithInternalBatch(32, 2, 8, CountingGenerator())
    batches = list(DataLoader(ds, batch_size=None, num_workers=0))
    assert len(batches) == 4 and batches[3][0][0, 0] == 24


class _SurfaceOnly(OnlineDataGenerator):
    """The class's own methods on an instance that never touches the device."""

    def __init__(self, equation):
        self.equation = equation
        self.max_points_per_call = None


def test_get_dataset_details_reads_the_whole_generator_surface():
    """picard/data.py:1620-1661 builds a dict of ALL six dataset methods before choosing one."""
    from deeppicarditeration_amd.equations import Cha
    g = _SurfaceOnly(Cha(NX, 1.0, 5.0, 1.0))
    assert g.do_internal_batching is True
    for exact, grad, hess, name, dim in [(False, True, False, "u_ux", 1 + NX), (False, True, True, "u_ux_uh", 1 + NX + NX * NX),
                                         (True, True, False, "u_ux", 1 + NX), (True, False, False, "u", 1),
                                         (False, False, False, "u", 1), (True, True, True, "u_ux_uh", 1 + NX + NX * NX)]:
        dm = PicardDataModuleStandIn.__new__(PicardDataModuleStandIn)  # no generator construction
        dm.data_generator, dm.equation, dm.data_cfg = g, g.equation, reference_data_cfg(EXACT=exact)
        dm.generate_gradients, dm.generate_hessians = grad, hess
        fn, d, nm = dm.get_dataset_details()
        assert (d, nm) == (dim, name)
        ds = fn(64, 2, 8)  # building the dataset draws nothing
        assert isinstance(ds, D.IterableDatasetWithInternalBatch) and len(ds) == 8


def test_value_only_labels_raise_like_the_reference():
    """The reference's value-only estimator calls equation.f, which raises for equations whose
    nonlinearity reads the gradient (equations.py:262-263)."""
    from deeppicarditeration_amd.equations import Cha
    g = _SurfaceOnly(Cha(NX, 1.0, 5.0, 1.0))
    with pytest.raises(NotImplementedError, match="dependence on z"):
        g.generate(torch.zeros(2, 1 + NX))


def test_exact_labels_match_closed_forms():
    """Exact-label equations used by dataset_exact*: OU u, grad u vs autograd of the per-row GMM
    (equations.py:650-700), GBM Hessian vs autograd (equations.py:445-450)."""
    from deeppicarditeration_amd.equations import GBMEquationComplexExact, OUProcessEquation
    torch.manual_seed(0)
    ou = OUProcessEquation(nx=100, T=1.0, num_components=5, mean_scale=1.0, var_scale=2.0)
    t = torch.rand(5, 1, dtype=torch.float64)
    x = 2 * torch.randn(5, 100, dtype=torch.float64)
    u, ux = ou.u_u_x(t, x)
    for r in range(5):
        xr = x[r:r + 1].clone().requires_grad_(True)
        ur = -ou.get_gmm_t(ou.T - float(t[r])).log_prob(xr)
        (gr,) = torch.autograd.grad(ur.sum(), xr)
        assert torch.allclose(ur.detach(), u[r:r + 1], rtol=1e-12, atol=1e-12)
        assert torch.allclose(gr, ux[r:r + 1], rtol=1e-10, atol=1e-12)
    gbm = GBMEquationComplexExact(100)
    u, ux, uh = gbm.u_u_x_u_hessian(t, x)
    xr = x[:1].clone().requires_grad_(True)
    H = torch.autograd.functional.hessian(lambda z: gbm.exact_solution(t[:1], z).sum(), xr)[0, :, 0, :]
    assert torch.allclose(H, uh[0], rtol=1e-10, atol=1e-12)
    assert torch.allclose(ux, gbm.u_x(t, x)) and uh.shape == (5, 100, 100)
    assert np.allclose(torch.diagonal(uh, dim1=1, dim2=2).numpy(), gbm.hess_diag(t, x).numpy())
