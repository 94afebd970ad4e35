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
from picard_datamodule import PicardDataModuleStandIn

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


def test_datamodule_multi_epoch_cache_and_label_file(tmp_path):
    """Stand-in PicardDataModule: gradient supervision, multi-epoch in-memory cache, DATA.SAVE."""
    gen = _gen()
    dm = PicardDataModuleStandIn(gen, NX, data_size=128, batch_size=32, n_batch_buffer=2, multi_epochs=True,
                                 shuffle=True, save_path=tmp_path / "split_00.h5")
    loader = dm.train_dataloader()
    first = list(loader)
    second = list(loader)
    assert len(first) == len(second) == 4
    tx1 = torch.cat([b[0] for b in first])
    y1 = torch.cat([b[1] for b in first])
    tx2 = torch.cat([b[0] for b in second])
    y2 = torch.cat([b[1] for b in second])
    assert tx2.is_cuda and gen.point_base == 128  # the second epoch drew no new points
    order1, order2 = torch.argsort(tx1[:, 0]), torch.argsort(tx2[:, 0])
    assert torch.equal(tx1[order1], tx2[order2]) and torch.equal(y1[order1], y2[order2])
    ftx = read_dataset(tmp_path / "split_00.h5", "tx")
    fy = read_dataset(tmp_path / "split_00.h5", "u_ux")
    of = np.argsort(ftx[:, 0], kind="stable")
    assert np.array_equal(ftx[of], tx1[order1].cpu().numpy()) and np.array_equal(fy[of], y1[order1].cpu().numpy())


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
