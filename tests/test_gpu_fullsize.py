"""Full BASELINE sizes for the PISGradNet and SDGD workloads (the Burgers ones are in
test_gpu_parity.py): HJB configs[2] (64 points x 4096 paths, K = 50, PISGradNet 4x512 — one
262,144-row chunk through the GEMM pipeline) and GBM configs[4] (64 points x 1024 paths, K = 50,
SDGD v = 100).  Checks: bitwise-reproducible moments, 2 / 4 / 8 MC shards reduced with
dpi_moments_reduce equal to the single call bit for bit, and the first and last point within the
north star's rel-L2 1e-4 of the fp64 oracle on the same counters."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    import deeppicarditeration_amd._lib as L
    L.load()


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _check(gen, oeq, onet, n, M, K, v=0):
    from deeppicarditeration_amd import _lib as L
    from oracle import dpi_oracle as O
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    ws = gen.point_baseline(tx)
    full = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    again = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    assert torch.equal(full, again)
    for G in (2, 4, 8):
        parts = torch.stack([gen.label_moments(tx, 0, M, r * M // G, (r + 1) * M // G, L.DPI_BOTH, ws)
                             for r in range(G)]).contiguous()
        assert torch.equal(gen.moments_reduce(parts), full), G
    y = gen.finalize(full, M, L.DPI_BOTH, ws).cpu().double().numpy()
    assert np.isfinite(y).all()
    txh = tx.cpu().double().numpy()
    for i in (0, n - 1):
        ref = O.labels_grad(oeq, onet, txh[i:i + 1], M, K, 1, 1, i, v=v, m_chunk=512)
        ev, eg = _rel(y[i:i + 1, :1], ref[:, :1]), _rel(y[i:i + 1, 1:], ref[:, 1:])
        print(f"point {i}: value {ev:.2e} grad {eg:.2e}")
        assert ev < TOL and eg < TOL, (i, ev, eg)


def test_hjb_config2_full_size():
    import deeppicarditeration_amd as dpi
    from oracle import dpi_oracle as O
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(0)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    n, M, K = 64, 4096, 50
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    _check(gen, oeq, onet, n, M, K)


def test_gbm_config4_full_size():
    import deeppicarditeration_amd as dpi
    from oracle import dpi_oracle as O
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    torch.manual_seed(3)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    n, M, K, v = 64, 1024, 50, 100
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": v}})
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU"] * 3)
    _check(gen, O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy()), onet, n, M, K, v=v)


def test_gbm_hessian_labels_config4_full_size():
    """Malliavin-weight Hessian labels (generate_with_gradients_and_hessians, picard/data.py:1220-1223;
    _double estimators :823-897, :1153-1201) at BASELINE configs[4] size: 64 points x 1024 paths,
    K = 50, 3 x 64 ELU network.  Bitwise-reproducible sums, 2 / 4 / 8 MC shards + dpi_sums_reduce
    equal to the single call bit for bit, moments + finalize equal to the one-call labels, and the
    first and last point (value, gradient and the 100 x 100 Hessian block) within rel-L2 1e-4 of
    the fp64 oracle on the same counters."""
    import deeppicarditeration_amd as dpi
    from oracle import dpi_oracle as O
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    torch.manual_seed(3)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    n, M, K = 64, 1024, 50
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    ws = gen.point_baseline(tx, hessians=True)
    mom, hs = gen.label_moments_hessians(tx, 0, M, 0, M, ws)
    mom2, hs2 = gen.label_moments_hessians(tx, 0, M, 0, M, ws)
    assert torch.equal(mom, mom2) and torch.equal(hs, hs2)
    for G in (2, 4, 8):
        parts = [gen.label_moments_hessians(tx, 0, M, r * M // G, (r + 1) * M // G, ws) for r in range(G)]
        assert torch.equal(gen.sums_reduce(torch.stack([p[0] for p in parts])), mom), G
        assert torch.equal(gen.sums_reduce(torch.stack([p[1] for p in parts])), hs), G
    y = gen.finalize_hessians(mom, hs, M, ws, bound=float("inf"))
    assert torch.equal(y, gen.generate_with_gradients_and_hessians(tx, point_base=0))
    y = y.cpu().double().numpy()
    assert np.isfinite(y).all() and y.shape == (n, 1 + 100 + 100 * 100)
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU"] * 3)
    oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    txh = tx.cpu().double().numpy()
    for i in (0, n - 1):
        ref = O.labels_grad_hess(oeq, onet, txh[i:i + 1], M, K, 1, 1, i, m_chunk=256)
        ev, eg, eh = (_rel(y[i:i + 1, :1], ref[:, :1]), _rel(y[i:i + 1, 1:101], ref[:, 1:101]),
                      _rel(y[i:i + 1, 101:], ref[:, 101:]))
        print(f"point {i}: value {ev:.2e} grad {eg:.2e} hessian {eh:.2e}")
        assert ev < TOL and eg < TOL and eh < TOL, (i, ev, eg, eh)


def test_hjb_two_pipeline_chunks_equal_separate_calls():
    """More (point, path-block) pairs than one PISGradNet pipeline chunk holds (66 points x 4096 paths
    = 4,224 pairs > DPI_PIS_CHUNK's 4,096): the second chunk's rows (points 64 and 65) run a second
    rollout -> GEMM chain -> final pass, with the baseline rows of all 66 points riding in the first
    chunk.  A row's result does not depend on where it sits in a chunk, so the two-chunk call equals
    the one-chunk calls over points 0-63 and 64-65 (same global point indices) bit for bit; the
    last point matches the fp64 oracle."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from oracle import dpi_oracle as O
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(0)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    n, M, K = 66, 4096, 50
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    full = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, gen.point_baseline(tx))
    a = tx[:64].contiguous()
    b = tx[64:].contiguous()
    part_a = gen.label_moments(a, 0, M, 0, M, L.DPI_BOTH, gen.point_baseline(a))
    part_b = gen.label_moments(b, 64, M, 0, M, L.DPI_BOTH, gen.point_baseline(b))
    assert torch.equal(full[:64], part_a)
    assert torch.equal(full[64:], part_b)
    ws = gen.point_baseline(tx)
    y = gen.finalize(gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws), M, L.DPI_BOTH, ws).cpu().double().numpy()
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    txh = tx.cpu().double().numpy()
    ref = O.labels_grad(oeq, onet, txh[n - 1:n], M, K, 1, 1, n - 1, m_chunk=512)
    ev, eg = _rel(y[n - 1:n, :1], ref[:, :1]), _rel(y[n - 1:n, 1:], ref[:, 1:])
    print(f"point {n - 1} (second chunk): value {ev:.2e} grad {eg:.2e}")
    assert ev < TOL and eg < TOL, (ev, eg)


@pytest.mark.parametrize("n,M", [(64, 4096), (3, 128)])
def test_hjb_fused_chain_equals_layer_wise_chain(n, M, monkeypatch):
    """k_pis_net (the VJP chain in one launch, activations in LDS) against the nine k_gemm_x3h
    launches it replaces (DPI_PIS_FUSED=0): the same products in the same order, so the moments and
    the labels are bitwise equal — at the configs[2] size (262,208 rows, 4,097 full 64-row tiles) and
    at 387 rows (a partial last tile)."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(0)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=8, seed=5)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    out = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("DPI_PIS_FUSED", fused)
        ws = gen.point_baseline(tx)
        mom = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
        out[fused] = (mom, gen.finalize(mom, M, L.DPI_BOTH, ws))
    assert torch.isfinite(out["1"][1]).all()
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])


def test_gbm_hessian_labels_unequal_counts_full_size():
    """n_estimate_terminal = 2,048 != n_estimate_integral = 1,024 (picard/data.py:1164 vs :845) at
    configs[4]'s 64 points, K = 50, 3 x 64 ELU: a DPI_TERMINAL pass over 2,048 paths plus a
    DPI_INTEGRAL pass over 1,024 (dpi_label_moments_hessians flags); the first and last point's value,
    gradient and Hessian blocks within rel-L2 1e-4 of the fp64 oracle with separate counts, and
    the sharded labeler's 2 / 4 MC shards of each pass reduce to the same labels bit for bit."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from oracle import dpi_oracle as O
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    torch.manual_seed(3)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    n, MT, MI, K = 64, 2048, 1024, 50
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=MT,
                                  n_estimate_integral=MI, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    y = gen.generate_with_gradients_and_hessians(tx, point_base=0)
    assert torch.equal(y, gen.generate_with_gradients_and_hessians(tx, point_base=0))
    ws = gen.point_baseline(tx, hessians=True)
    for G in (2, 4):  # each pass's MC range in G shards, reduced per pass, as ShardedLabeler does
        ys = []
        for M, f in ((MT, L.DPI_TERMINAL), (MI, L.DPI_INTEGRAL)):
            parts = [gen.label_moments_hessians(tx, 0, M, r * M // G, (r + 1) * M // G, ws, f) for r in range(G)]
            mom = gen.sums_reduce(torch.stack([p[0] for p in parts]))
            hs = gen.sums_reduce(torch.stack([p[1] for p in parts]))
            ys.append(gen.finalize_hessians(mom, hs, M, ws, float("inf"), f))
        assert torch.equal(ys[0] + ys[1], y), G
    y = y.cpu().double().numpy()
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin],
                 ["ELU"] * 3)
    oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    txh = tx.cpu().double().numpy()
    for i in (0, n - 1):
        ref = O.labels_grad_hess(oeq, onet, txh[i:i + 1], MI, K, 1, 1, i, m_chunk=256, MT=MT)
        ev, eg, eh = (_rel(y[i:i + 1, :1], ref[:, :1]), _rel(y[i:i + 1, 1:101], ref[:, 1:101]),
                      _rel(y[i:i + 1, 101:], ref[:, 101:]))
        print(f"point {i}: value {ev:.2e} grad {eg:.2e} hessian {eh:.2e}")
        assert ev < TOL and eg < TOL and eh < TOL, (i, ev, eg, eh)


def test_sharded_labeler_unequal_counts_equal_generator():
    """ShardedLabeler (one rank) with n_estimate_terminal = 2 n_estimate_integral: labels(), the
    prepare/begin/end pipeline and labels_hessians equal the generator's own labels bit for bit."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd.sharding import ShardedLabeler
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    torch.manual_seed(5)
    net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=512,
                                  n_estimate_integral=256, n_euler_steps=4, seed=2,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    lab = ShardedLabeler(gen)
    tx, pb = gen.sample_t_and_x(5)
    y = gen.generate_with_gradients(tx, point_base=pb)
    assert torch.equal(lab.labels(tx, pb), y)
    prep = lab.prepare(5)
    txp, pbp = prep[0], prep[1]
    yp = lab.end(lab.begin(prepared=prep))
    assert torch.equal(yp, gen.generate_with_gradients(txp, point_base=pbp))
    assert torch.equal(lab.labels_hessians(tx, pb), gen.generate_with_gradients_and_hessians(tx, point_base=pb))
