"""The reference's data-module path (picard/data.py:1620-1780, picard/dataset.py) driven with the HIP
generator: every batch that comes out of `dataset_with_gradients` must equal the label call on
the same points and counters, the in-memory cache must replay exactly those labels from HBM, and
the exact-label datasets must equal the closed forms."""
import numpy as np
import pytest
import torch

import deeppicarditeration_amd as dpi
from deeppicarditeration_amd import dataset as D
from deeppicarditeration_amd.h5 import read_dataset

pytestmark = pytest.mark.gpu

NX, M, K = 100, 64, 4


def _gen(eq=None, net=None, hess=None, seed=5):
    eq = eq or dpi.Cha(NX, 1.0, 5.0, 1.0)
    if net is None:
        torch.manual_seed(0)
        net = dpi.construct_mlp(1 + NX, 1, [32, 32], ["ELU", "ELU"], None)
    return dpi.OnlineDataGenerator(eq, net, 4, 2, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                   n_estimate_integral=M, n_euler_steps=K, seed=seed, hessian_approximation=hess)


@pytest.mark.parametrize("nbuf, per_call", [(2, 64), (0.5, 16)])
def test_dataset_with_gradients_batches_equal_the_label_calls(nbuf, per_call):
    gen, ref = _gen(), _gen()
    ds = gen.dataset_with_gradients(128, nbuf, 32)
    batches = list(ds)
    assert len(batches) == len(ds) == 4
    tx = torch.cat([b[0] for b in batches])
    y = torch.cat([b[1] for b in batches])
    assert tx.is_cuda and y.is_cuda and y.shape == (128, 1 + NX)
    for c in range(128 // per_call):
        rows = slice(c * per_call, (c + 1) * per_call)
        tx_ref, pb = ref.sample_t_and_x(per_call)
        assert pb == c * per_call
        assert torch.equal(tx[rows], tx_ref)
        assert torch.equal(y[rows], ref.generate_with_gradients(tx_ref, point_base=pb))


class _Recording(dpi.OnlineDataGenerator):
    """The HIP generator, recording (point_base, n, tx, y) of every sample_with_gradients call."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.calls = []

    def sample_with_gradients(self, n):
        pb = self.point_base
        tx, y = super().sample_with_gradients(n)
        self.calls.append((pb, n, tx, y))
        return tx, y


def _standin(monkeypatch, tmp_path, net, epochs, batch_size=512, **data):
    """The stand-in of the reference's data module (tests/picard_datamodule.py, pinned to the real
    module by tests/test_reference_binding.py) over the binding, with the recording generator."""
    from deeppicarditeration_amd import picard_binding as B
    from picard_datamodule import PicardDataModuleStandIn, reference_data_cfg
    orig = B.hip_online_data_generator
    monkeypatch.setattr(B, "hip_online_data_generator",
                        lambda kws, cfg, base=None: orig(kws, cfg, base=base, generator_cls=_Recording))
    return PicardDataModuleStandIn(equation=dpi.Cha(NX, 1.0, 5.0, 1.0), solution=net, N=80, i=1,
                                   data_cfg=reference_data_cfg(**data), batch_size=batch_size, exp_dir=tmp_path,
                                   do_multi_epochs=epochs > 1, generate_gradients=True, device="cuda:0")


def _expected(net, calls, M_, K_=50):
    """Every recorded call recomputed by a fresh generator on the same points and counters."""
    ref = dpi.OnlineDataGenerator(dpi.Cha(NX, 1.0, 5.0, 1.0), net, 80, 1, device="cuda:0", t_always_uniform=True,
                                  n_estimate_terminal=M_, n_estimate_integral=M_, n_euler_steps=K_, seed=0)
    out = []
    for pb, n, tx, y in calls:
        tx_ref, _ = ref.sample_t_and_x(n, point_base=pb)
        y_ref = ref.generate_with_gradients(tx_ref, point_base=pb)
        assert torch.equal(tx.float(), tx_ref) and torch.equal(y.float(), y_ref)
        out.append((tx_ref, y_ref))
    return out


def test_shipped_burgers_yaml_through_the_reference_data_module(monkeypatch, tmp_path):
    """INTEGRATION.md §1 end to end on the GPU with the shipped Burgers YAML's DATA / TRAIN keys
    (scripts/burgers/base_100d_T1.0_w0.0_0.yaml: NEW_SAMPLING, PRELOAD, N_EPOCHS 16, DATA_SIZE 4096,
    BATCH_SIZE 512, M 4096, K 50, FLOAT double): the memory probe settles at the per-call cap, the
    CacheToMemoryWrapper re-batches one 4096-point call, and every batch of all 16 epochs equals
    the label call on the same points and counters, bit for bit (cast exactly to fp64)."""
    from picard_datamodule import BURGERS_YAML_DATA
    torch.manual_seed(0)
    net = dpi.construct_mlp(1 + NX, 1, [128] * 4, ["ELU"] * 4, None)
    dm = _standin(monkeypatch, tmp_path, net, 16, **BURGERS_YAML_DATA)
    assert dm.data_dir == tmp_path / "data_iter_1"
    loader = dm.train_dataloader()
    gen = dm.data_generator
    assert dm.dataset_size_info_args == (4096, 1, 4096)
    assert [c[1] for c in gen.calls[:2]] == [1024, 1024] and 0.9 * 16384 < gen.calls[2][1] <= 16384
    assert len(gen.calls) == 5 and gen.calls[4][1] == 4096
    exp = _expected(net, gen.calls[4:], 4096)
    tx_all, y_all = exp[0]
    for epoch in range(16):
        batches = list(loader)
        assert len(batches) == 8
        for b, (tx, y) in enumerate(batches):
            rows = slice(512 * b, 512 * (b + 1))
            assert tx.dtype == y.dtype == torch.float64 and tx.is_cuda
            assert torch.equal(tx, tx_all[rows].double()) and torch.equal(y, y_all[rows].double()), (epoch, b)
    assert len(gen.calls) == 5  # later epochs replay the HBM cache


def test_data_module_streaming_shuffled_cache_and_label_file(monkeypatch, tmp_path):
    """NEW_SAMPLING false with N_BUFFER 2 (two 128-batches per call), SHUFFLE, SAVE, 3 epochs: DATA.SAVE
    makes the cache preload (dataset.py:229-231), so every epoch replays the HBM cache shuffled, and
    the label file holds the labels in generation order."""
    torch.manual_seed(0)
    net = dpi.construct_mlp(1 + NX, 1, [32, 32], ["ELU", "ELU"], None)
    dm = _standin(monkeypatch, tmp_path, net, 3, batch_size=128, FLOAT="float", DATA_SIZE=1024, N_WORKERS=0,
                  N_BUFFER=2, SHUFFLE=True, SAVE=True, BACKEND="hip", EULER_STEPS=K,
                  kwargs=dict(t_always_uniform=True, n_estimate_terminal=M, n_estimate_integral=M))
    loader = dm.train_dataloader()
    gen = dm.data_generator
    assert [c[1] for c in gen.calls] == [256] * 4
    exp = _expected(net, gen.calls, M, K)
    tx1, y1 = torch.cat([e[0] for e in exp]), torch.cat([e[1] for e in exp])
    o1 = torch.argsort(tx1[:, 0])
    orders = []
    for _ in range(3):
        batches = list(loader)
        assert len(batches) == 8
        tx2, y2 = torch.cat([b[0] for b in batches]), torch.cat([b[1] for b in batches])
        o2 = torch.argsort(tx2[:, 0])
        assert torch.equal(tx1[o1], tx2[o2]) and torch.equal(y1[o1], y2[o2])
        orders.append(o2)
    assert not torch.equal(orders[0], orders[1])  # shuffled per pass
    assert len(gen.calls) == 4
    ftx = read_dataset(tmp_path / "data_iter_1" / "split_00.h5", "tx")
    fy = read_dataset(tmp_path / "data_iter_1" / "split_00.h5", "u_ux")
    assert np.array_equal(ftx, tx1.cpu().numpy()) and np.array_equal(fy, y1.cpu().numpy())


def test_exact_datasets_equal_the_closed_forms():
    gbm = dpi.GBMEquationComplexExact(NX)
    gen = _gen(eq=gbm, hess={"method": "SDGD", "kwargs": {"v": 100}})
    tx, y = next(iter(gen.dataset_exact_with_gradients(64, 1, 64)))
    t, x = tx[:, :1].double().cpu(), tx[:, 1:].double().cpu()
    u, ux = gbm.u_u_x(t, x)
    assert torch.allclose(y.double().cpu(), torch.cat([u, ux], -1), rtol=1e-5, atol=1e-6)
    tx, y = next(iter(gen.dataset_exact_with_gradients_and_hessians(8, 1, 8)))
    u, ux, uh = gbm.u_u_x_u_hessian(tx[:, :1].double().cpu(), tx[:, 1:].double().cpu())
    assert y.shape == (8, 1 + NX + NX * NX)
    assert torch.allclose(y[:, 1 + NX:].double().cpu(), uh.reshape(8, -1), rtol=1e-5, atol=1e-6)
    tx, y = next(iter(gen.dataset_exact(16, 1, 16)))
    assert y.shape == (16, 1)
    with pytest.raises(NotImplementedError):
        next(iter(gen.dataset(16, 1, 16)))


def test_dataset_with_gradients_and_hessians_batches_equal_the_label_calls():
    gbm = dpi.GBMEquationComplexExact(NX)
    torch.manual_seed(1)
    net = dpi.construct_mlp(1 + NX, 1, [16, 16], ["ELU", "ELU"], None)
    hess = {"method": "SDGD", "kwargs": {"v": 100}}
    gen, ref = _gen(gbm, net, hess), _gen(gbm, net, hess)
    b = list(gen.dataset_with_gradients_and_hessians(8, 1, 4))
    assert len(b) == 2 and b[0][1].shape == (4, 1 + NX + NX * NX)
    tx_ref, pb = ref.sample_t_and_x(8)
    assert torch.equal(torch.cat([x for x, _ in b]), tx_ref)
    assert torch.equal(torch.cat([y for _, y in b]), ref.generate_with_gradients_and_hessians(tx_ref, point_base=pb))


def test_sample_bound_clip_matches_oracle():
    """A finite DATA.SAMPLE_BOUND clips the labels (data.py:222) — bound chosen inside the label range."""
    from oracle import dpi_oracle as O
    eq = dpi.Cha(NX, 1.0, 5.0, 1.0)
    torch.manual_seed(0)
    net = dpi.construct_mlp(1 + NX, 1, [32, 32], ["ELU", "ELU"], None)
    free = _gen(eq, net)
    tx, y = free.sample_with_gradients(16)
    bound = float(torch.quantile(y.abs().flatten(), 0.5))
    gen = dpi.OnlineDataGenerator(eq, net, 4, 2, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=5, sample_bound=bound)
    tx2, yc = gen.sample_with_gradients(16)
    assert torch.equal(tx, tx2)
    assert torch.equal(yc, torch.clamp(y, -bound, bound))
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU", "ELU"])
    ref = np.clip(O.labels_grad(O.Cha(NX, 1.0, 5.0, 1.0), onet, tx.cpu().double().numpy(), M, K, 5, 2, 0), -bound, bound)
    err = np.linalg.norm(yc.cpu().double().numpy() - ref) / np.linalg.norm(ref)
    assert err < 1e-4, err
    assert float(yc.abs().max()) <= bound


def test_nan_labels_survive_the_clip():
    """torch.clip keeps NaN (data.py:222); a divergent network must not come out as +-bound."""
    eq = dpi.Cha(NX, 1.0, 5.0, 1.0)
    torch.manual_seed(0)
    net = dpi.construct_mlp(1 + NX, 1, [32, 32], ["ELU", "ELU"], None)
    with torch.no_grad():
        net[-1].bias.fill_(float("nan"))
    gen = dpi.OnlineDataGenerator(eq, net, 4, 2, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=5, sample_bound=0.5)
    _, y = gen.sample_with_gradients(4)
    assert bool(torch.isnan(y).all()), y
