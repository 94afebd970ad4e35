"""GPU parity of the HIP label path (libdpi_hip.so via the C-ABI) against
(a) the reference's own outputs (golden fixtures, fp64 reference with injected Philox noise) and
(b) the CPU oracle (fp64 numpy restatement) on the same seeded inputs.

Tolerance (north star): rel-L2 <= 1e-4 of the fp32 HIP labels vs the fp64 reference, measured
separately on the value column and the gradient block.  Expected ~1e-7 (fp32 rounding).
"""
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
    L.load()  # fail loudly if the HIP library is missing


from golden_util import CASES, delta_t, load, oracle_equation, oracle_net, t_factors  # noqa: E402
from gpu_util import generator, product_equation, product_module, rel_l2_parts  # noqa: E402
from oracle import dpi_oracle as O  # noqa: E402

SUPPORTED = [c for c in CASES if "_ws" not in c]  # weight-scaled fixtures: tests/test_gpu_range.py, both modes


@pytest.mark.parametrize("case", SUPPORTED)
def test_golden_reference_parity(case):
    f = load(case)
    eq = product_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    y = gen.generate_with_gradients(tx, point_base=int(f["point_base"])).cpu().numpy()
    parts = rel_l2_parts(y, f["y"])
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("case", ["cha_mlp16_K4", "ou_mlp16_K2", "tprod_cha_mlp16_K2", "tprod_gbm_mlp16_sdgd_K1"])
def test_sample_points_match_oracle(case):
    f = load(case)
    eq = product_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    n = 257
    tx, _ = gen.sample_t_and_x(n, point_base=int(f["point_base"]))
    ref = O.sample_points(oracle_equation(f), n, int(f["seed"]), int(f["epoch"]), int(f["point_base"]),
                          t_factors=t_factors(f))
    tx = tx.cpu().double().numpy()
    # fp32 t: one rounding for the uniform sampler, one per factor for sample_t's product
    np.testing.assert_allclose(tx[:, 0], ref[:, 0], rtol=2e-6 if t_factors(f) else 2e-7, atol=1e-7)
    np.testing.assert_allclose(tx[:, 1:], ref[:, 1:], rtol=0, atol=2e-5)
    # the golden fixture's points came from the same contract
    np.testing.assert_allclose(tx[: int(f["n"])], f["tx"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("N,i", [(1, 1), (5, 2), (9, 3), (80, 1)])
def test_product_t_sampler_matches_oracle(N, i):
    """sample_t (t_always_uniform: false, data.py:149-159): t = T (1 - prod of N - i + 1 uniforms)
    from the same Philox stream as the uniform sampler, x sampled at that t."""
    import deeppicarditeration_amd as dpi
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    gen = dpi.OnlineDataGenerator(eq, dpi.ZeroSolution(1), N, i, device="cuda:0", t_always_uniform=False,
                                  n_estimate_terminal=64, n_estimate_integral=64, n_euler_steps=1, seed=77, epoch=5)
    n = 257
    tx, _ = gen.sample_t_and_x(n, point_base=1000)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    ref = O.sample_points(oeq, n, 77, 5, 1000, t_factors=N - i + 1)
    tx = tx.cpu().double().numpy()
    np.testing.assert_allclose(tx[:, 0], ref[:, 0], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(tx[:, 1:], ref[:, 1:], rtol=0, atol=5e-5)
    assert (tx[:, 0] > 0).all() and (tx[:, 0] <= 1.0).all()


@pytest.mark.parametrize("case", ["cha_mlp16_K4", "ou_mlp16_K2", "gbm_mlp16_sdgd_K2"])
def test_terminal_and_integral_estimators(case):
    f = load(case)
    eq = product_equation(f)
    net = product_module(f, eq)
    oeq = oracle_equation(f)
    onet = oracle_net(f, oeq)
    gen = generator(f, eq, net)
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    pb = int(f["point_base"])
    yT = gen.estimate_terminal_with_gradients(tx, point_base=pb).cpu().numpy()
    yI = gen.estimate_integral_with_gradients(tx, point_base=pb).cpu().numpy()
    _, rT, rI = O.labels_grad(oeq, onet, f["tx"], int(f["M"]), int(f["K"]), int(f["seed"]), int(f["epoch"]), pb,
                              v=int(f["v"]), return_parts=True)
    pT, pI = rel_l2_parts(yT, rT), rel_l2_parts(yI, rI)
    assert pT["value"] < TOL and pT["grad"] < TOL, pT
    assert pI["value"] < TOL and pI["grad"] < TOL, pI


@pytest.mark.parametrize("case", ["td_cha_mlp16_K2", "td_ou_mlp32_K3", "td_gbm_mlp16_sdgd_K2", "td_cha_zero_K1"])
def test_td_terminal_and_integral_estimators(case):
    """TD estimators (ESTIMATE_DELTA_T > 0): estimate_terminal_with_gradients_td (data.py:934-952)
    and estimate_integral_with_gradients_td (:529-575) separately vs the oracle."""
    f = load(case)
    eq = product_equation(f)
    oeq = oracle_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    pb = int(f["point_base"])
    yT = gen.estimate_terminal_with_gradients(tx, point_base=pb).cpu().numpy()
    yI = gen.estimate_integral_with_gradients(tx, point_base=pb).cpu().numpy()
    _, rT, rI = O.labels_grad(oeq, oracle_net(f, oeq), f["tx"], int(f["M"]), int(f["K"]), int(f["seed"]),
                              int(f["epoch"]), pb, v=int(f["v"]), return_parts=True, delta_t=delta_t(f))
    pT, pI = rel_l2_parts(yT, rT), rel_l2_parts(yI, rI)
    assert pT["value"] < TOL and pT["grad"] < TOL, pT
    assert pI["value"] < TOL and pI["grad"] < TOL, pI


@pytest.mark.parametrize("gemm_mode", [0, 1])
def test_td_pisgradnet_config3_network_vs_oracle(gemm_mode):
    """TD estimators with PISGradNet 4x512 (config-3 network): terminal stage (rollout to t_next,
    forward GEMM chain, u(t_next, X)) then the integral stage, vs the oracle; fp32 and
    fp16-split GEMMs."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    L.check(L.load().dpi_set_gemm_precision(gemm_mode), "gemm precision")
    try:
        eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        torch.manual_seed(3)
        net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
        M, K, n, dt = 128, 10, 8, 0.4
        gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                      n_estimate_integral=M, n_euler_steps=K, seed=2, estimate_delta_t=dt)
        tx, _ = gen.sample_t_and_x(n, point_base=0)
        t = tx[:, 0].cpu().numpy()
        assert (t + dt < 1).any() and (t + dt >= 1).any()
        y = gen.generate_with_gradients(tx, point_base=0).cpu().numpy()
    finally:
        L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "gemm precision")
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), M, K, 2, 1, 0, delta_t=dt)
    parts = rel_l2_parts(y, ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_td_generator_does_not_leak_into_shared_problem():
    """Two generators on one equation object (one device problem handle), TD and plain: each
    call applies its own estimator settings."""
    f = load("cha_mlp16_K4")
    eq = product_equation(f)
    net = product_module(f, eq)
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    plain = generator(f, eq, net)
    y0 = plain.generate_with_gradients(tx, point_base=int(f["point_base"])).cpu()
    import deeppicarditeration_amd as dpi
    td = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                 n_estimate_integral=64, n_euler_steps=int(f["K"]), seed=int(f["seed"]),
                                 epoch=int(f["epoch"]), estimate_delta_t=0.1)
    y_td = td.generate_with_gradients(tx, point_base=int(f["point_base"])).cpu()
    y1 = plain.generate_with_gradients(tx, point_base=int(f["point_base"])).cpu()
    assert torch.equal(y0, y1)
    assert not torch.equal(y0, y_td)


def _random_mlp(eq, widths, seed):
    import deeppicarditeration_amd as dpi
    torch.manual_seed(seed)
    return dpi.construct_mlp(1 + eq.nx, 1, widths, ["ELU"] * len(widths), None)


def _oracle_mlp(m):
    lin = [l for l in m if isinstance(l, torch.nn.Linear)]
    return O.MLP([l.weight.detach().double().numpy() for l in lin], [l.bias.detach().double().numpy() for l in lin],
                 ["ELU"] * (len(lin) - 1))


@pytest.fixture(params=["f32", "auto"])
def mlp_precision(request):
    """Fused-MLP MFMA precision: exact fp32 or the default fp16-split (include/dpi.h DPI_GEMM_*)."""
    from deeppicarditeration_amd import _lib as L
    mode = L.DPI_GEMM_F32 if request.param == "f32" else L.DPI_GEMM_AUTO
    L.check(L.load().dpi_set_gemm_precision(mode), "gemm precision")
    yield request.param
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "gemm precision")


def test_burgers_full_network_K50_vs_oracle(mlp_precision):
    """Config-2 network (4x128 ELU) and K = 50 at a size the fp64 oracle finishes quickly."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = _random_mlp(eq, [128] * 4, 3)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=512,
                                  n_estimate_integral=512, n_euler_steps=50, seed=1, epoch=0)
    tx, y = gen.sample_with_gradients(3)
    oeq = O.Cha(100, 1.0, 5.0, 1.0)
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 512, 50, 1, 0, 0)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    print("mlp precision", mlp_precision, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_td_burgers_full_network_K50_vs_oracle(mlp_precision):
    """TD estimators with the config-2 network (4x128 ELU), K = 50: the split / fp32 fused MLP
    evaluates u(t_next, X) on the terminal noise, then u, grad u on the integral noise."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = _random_mlp(eq, [128] * 4, 0)
    M, K, n, dt = 128, 50, 8, 0.25
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1, estimate_delta_t=dt)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    t = tx[:, 0].cpu().numpy()
    assert (t + dt < 1).any() and (t + dt >= 1).any()  # t = 0.81, 0.06, 0.18, 0.87, ...
    y = gen.generate_with_gradients(tx, point_base=0).cpu().numpy()
    ref = O.labels_grad(O.Cha(100, 1.0, 5.0, 1.0), _oracle_mlp(net), tx.cpu().double().numpy(), M, K, 1, 1, 0,
                        delta_t=dt)
    parts = rel_l2_parts(y, ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("net_kind", ["zero", "mlp"])
def test_tiny_s_minus_t_regression(net_kind):
    """Point 520 of (seed 0, epoch 1) has a path with U = O(2^-24) at t = 0.933: fp32 s - t rounds
    to 0 there, which once turned Y_s into inf and the gradient labels into -inf / NaN.  The
    kernels use s - t = U (T - t); the label must be finite and match the fp64 oracle."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(8, 1.0, 5.0, 1.0)
    net = dpi.ZeroSolution(1) if net_kind == "zero" else _random_mlp(eq, [32, 32], 5)
    gen = dpi.OnlineDataGenerator(eq, net, 3, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=1024,
                                  n_estimate_integral=1024, n_euler_steps=4, seed=0, epoch=1)
    tx, pb = gen.sample_t_and_x(1, point_base=520)
    assert abs(float(tx[0, 0]) - 0.9333475) < 1e-6
    y = gen.generate_with_gradients(tx, point_base=pb)
    assert torch.isfinite(y).all()
    oeq = O.Cha(8, 1.0, 5.0, 1.0)
    onet = O.ZeroNet() if net_kind == "zero" else _oracle_mlp(net)
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), 1024, 4, 0, 1, 520)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("nx", [1, 7, 80, 96, 113, 128])
def test_dimension_edges_vs_oracle(nx, mlp_precision):
    """Ragged and maximal state dimensions: a partial last 4-dim block (7, 113), a split layer-1 row of
    three 32-column chunks (80, 96: padded to four, the LDS swizzle needs 1, 2 or 4), the 8th block of
    a wave (nx > 112 takes the per-column reduction path) and nx = NXP_MAX = 128."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(nx, 1.0, 5.0, 1.0)
    net = _random_mlp(eq, [64, 64], 11)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=3, seed=4, epoch=3)
    tx, y = gen.sample_with_gradients(3)
    oeq = O.Cha(nx, 1.0, 5.0, 1.0)
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 128, 3, 4, 3, 0)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_hjb_ou_mlp_vs_oracle(mlp_precision):
    import deeppicarditeration_amd as dpi
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    net = _random_mlp(eq, [64] * 3, 4)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                  n_estimate_integral=256, n_euler_steps=10, seed=2, epoch=5)
    tx, y = gen.sample_with_gradients(3)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 256, 10, 2, 5, 0)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_gbm_config5_network_sdgd_vs_oracle(mlp_precision):
    """Config-5 network (3x64 ELU), SDGD v = 100, K = 50, against the fp64 oracle; the tangent
    sweep on the fp16-split MFMA (mlp_hdiag_split) and on the fp32 MFMA (mlp_hdiag)."""
    import deeppicarditeration_amd as dpi
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = _random_mlp(eq, [64] * 3, 6)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=50, seed=3, epoch=2,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    tx, y = gen.sample_with_gradients(2)
    oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 128, 50, 3, 2, 0, v=100)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    print("gbm sdgd, mlp precision", mlp_precision, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("gemm_mode", [0, 1])
def test_hjb_pisgradnet_config3_network_vs_oracle(gemm_mode):
    """Config-3 network: PISGradNet 4 x 512 (MFMA pipeline, fp32 layer-wise GEMMs and the fp16-split k_pis_net chain),
    OU + GMM, K = 20."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    L.check(L.load().dpi_set_gemm_precision(gemm_mode), "gemm precision")
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    torch.manual_seed(7)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    with torch.no_grad():
        net.timestep_phase.copy_(0.1 * torch.randn(1, 64))
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=20, seed=2, epoch=1)
    tx, y = gen.sample_with_gradients(2)
    oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
    onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), 128, 20, 2, 1, 0)
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "gemm precision")
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    print("gemm mode", gemm_mode, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("delta_t", [0.0, 0.3])
def test_full_size_determinism_and_shard_invariance(delta_t):
    """BASELINE config 2 size (16 x 4096 paths, K = 50): bitwise-reproducible labels, and moments
    computed as two MC shards + dpi_moments_reduce equal the single call bit for bit; also with the
    TD estimators (delta_t = 0.3)."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = _random_mlp(eq, [128] * 4, 5)
    M = 4096
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=50, seed=1, estimate_delta_t=delta_t)
    tx, _ = gen.sample_t_and_x(16, point_base=0)
    ws = gen.point_baseline(tx)
    full = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    again = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    assert torch.equal(full, again)
    for G in (2, 4, 8):
        parts = torch.stack([gen.label_moments(tx, 0, M, r * M // G, (r + 1) * M // G, L.DPI_BOTH, ws)
                             for r in range(G)]).contiguous()
        out = torch.empty_like(full)
        L.check(gen.lib.dpi_moments_reduce(L.c_void_p(parts.data_ptr()), G, 16, 100, L.c_void_p(out.data_ptr()),
                                           L.c_void_p(torch.cuda.current_stream().cuda_stream)), "moments_reduce")
        assert torch.equal(out, full), G
    y = gen.finalize(full, M, L.DPI_BOTH, ws)
    assert torch.isfinite(y).all()
    # linearity: terminal + integral estimators == joint estimator (to fp32 rounding)
    yT = gen.finalize(gen.label_moments(tx, 0, M, 0, M, L.DPI_TERMINAL, ws), M, L.DPI_TERMINAL, ws)
    yI = gen.finalize(gen.label_moments(tx, 0, M, 0, M, L.DPI_INTEGRAL, ws), M, L.DPI_INTEGRAL, ws)
    torch.testing.assert_close(yT + yI, y, rtol=1e-5, atol=1e-5)


def test_config4_burgers_2M_paths_sharded_8_ways():
    """BASELINE configs[3] shape: Burgers, 512 points x 4096 MC paths (2,097,152 path-labels),
    K = 50, MC-sharded 8 ways (512 paths per shard, as on 8 GPUs): the 8 shard moments reduced
    with dpi_moments_reduce equal the single call bit for bit, and two of the points (first and
    last) match the fp64 oracle."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = _random_mlp(eq, [128] * 4, 0)
    n, M, G, K = 512, 4096, 8, 50
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(n, point_base=0)
    ws = gen.point_baseline(tx)
    full = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    parts = torch.stack([gen.label_moments(tx, 0, M, r * M // G, (r + 1) * M // G, L.DPI_BOTH, ws)
                         for r in range(G)]).contiguous()
    red = gen.moments_reduce(parts)
    assert torch.equal(red, full)
    y = gen.finalize(full, M, L.DPI_BOTH, ws).cpu().numpy()
    assert np.isfinite(y).all()
    oeq, onet = O.Cha(100, 1.0, 5.0, 1.0), _oracle_mlp(net)
    txh = tx.cpu().double().numpy()
    for i in (0, n - 1):
        ref = O.labels_grad(oeq, onet, txh[i:i + 1], M, K, 1, 1, i)
        parts_i = rel_l2_parts(y[i:i + 1], ref)
        assert parts_i["value"] < TOL and parts_i["grad"] < TOL, (i, parts_i)


def test_unsupported_configurations_fail_loudly():
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd._lib import DPIError
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    with pytest.raises(NotImplementedError):  # activations other than ELU / Tanh (tests/test_gpu_tanh.py)
        dpi.OnlineDataGenerator(eq, dpi.construct_mlp(101, 1, [16], ["Softplus"], None), 1, 1, device="cuda:0",
                                t_always_uniform=True, n_estimate_terminal=64, n_estimate_integral=64)
    with pytest.raises(ValueError):
        dpi.OnlineDataGenerator(eq, dpi.ZeroSolution(), 1, 1, device="cuda:0", t_always_uniform=True,
                                n_estimate_terminal=100, n_estimate_integral=100)
    with pytest.raises(DPIError):  # GBM keeps all weights in LDS: hidden width <= 64
        dpi.OnlineDataGenerator(dpi.GBMEquationComplexExact(100), dpi.construct_mlp(101, 1, [128] * 2, ["ELU"] * 2, None),
                                1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                n_estimate_integral=64).sample_with_gradients(2)


# ----------------------------------------------------------------------------- Hessian labels
from golden_util import HESS_CASES  # noqa: E402


def _blocks(y, nx):
    return {"value": (slice(None), slice(0, 1)), "grad": (slice(None), slice(1, 1 + nx)),
            "hess": (slice(None), slice(1 + nx, None))}


@pytest.mark.parametrize("case", HESS_CASES)
def test_hessian_labels_golden_reference_parity(case):
    """generate_with_gradients_and_hessians (picard/data.py:1220-1223) on the GPU vs the
    reference's own output on the same noise (tests/golden/make_golden.py), per block."""
    f = load(case)
    eq = product_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    y = gen.generate_with_gradients_and_hessians(tx, point_base=int(f["point_base"])).cpu().numpy()
    nx = eq.nx
    assert y.shape == f["y"].shape
    for name, sl in _blocks(y, nx).items():
        r = O.rel_l2(y[sl], f["y"][sl])
        assert r < TOL, (name, r)


def test_hessian_labels_config5_network_vs_oracle(mlp_precision):
    """Config-5 network (3 x 64 ELU), K = 10, M = 256, against the fp64 oracle (fp16-split and fp32
    tangent sweeps); the Hessian block is symmetric by construction."""
    import deeppicarditeration_amd as dpi
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = _random_mlp(eq, [64] * 3, 12)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                  n_estimate_integral=256, n_euler_steps=10, seed=13, epoch=4,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    tx, y = gen.sample_with_gradients_and_hessians(2)
    oeq = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy())
    ref = O.labels_grad_hess(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 256, 10, 13, 4, 0)
    y = y.cpu().numpy()
    for name, sl in _blocks(y, 100).items():
        r = O.rel_l2(y[sl], ref[sl])
        assert r < TOL, (name, r)
    h = y[:, 101:].reshape(2, 100, 100)
    assert np.array_equal(h, np.transpose(h, (0, 2, 1)))


def test_hessian_labels_need_gbm():
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd._lib import DPIError
    eq = dpi.Cha(10, 1.0, 5.0, 1.0)
    gen = dpi.OnlineDataGenerator(eq, dpi.ZeroSolution(1), 1, 1, device="cuda:0", t_always_uniform=True,
                                  n_estimate_terminal=64, n_estimate_integral=64, n_euler_steps=2)
    with pytest.raises(DPIError):
        gen.sample_with_gradients_and_hessians(2)


def test_hessian_labels_shard_invariance_and_determinism():
    """Config-5 network, 8 points x 1024 paths: Hessian labels are bitwise reproducible, the
    MC-sharded sums (G = 2, 4, 8) + dpi_sums_reduce equal the single call bit for bit, and
    moments + finalize equal the one-call generate_with_gradients_and_hessians."""
    import deeppicarditeration_amd as dpi
    eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
    net = _random_mlp(eq, [64] * 3, 14)
    M = 1024
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=8, seed=3, epoch=2)
    tx, _ = gen.sample_t_and_x(8, point_base=0)
    ws = gen.point_baseline(tx, hessians=True)
    mom, hs = gen.label_moments_hessians(tx, 0, M, 0, M, ws)
    mom2, hs2 = gen.label_moments_hessians(tx, 0, M, 0, M, ws)
    assert torch.equal(mom, mom2) and torch.equal(hs, hs2)
    for G in (2, 4, 8):
        parts = [gen.label_moments_hessians(tx, 0, M, r * M // G, (r + 1) * M // G, ws) for r in range(G)]
        assert torch.equal(gen.sums_reduce(torch.stack([p[0] for p in parts])), mom), G
        assert torch.equal(gen.sums_reduce(torch.stack([p[1] for p in parts])), hs), G
    y = gen.finalize_hessians(mom, hs, M, ws, bound=float("inf"))
    y1 = gen.generate_with_gradients_and_hessians(tx, point_base=0)
    assert torch.equal(y, y1)


@pytest.mark.parametrize("kind", ["cha_mlp", "ou_pis", "gbm_hess"])
def test_empty_and_single_point_batches(kind):
    """Edge batches: n = 0 returns empty label blocks without launching (and without moving the
    point counter); n = 1 (a one-point grid, a single-row PIS chunk) matches the oracle."""
    import deeppicarditeration_amd as dpi
    torch.manual_seed(5)
    kw = dict(device="cuda:0", t_always_uniform=True, n_estimate_terminal=128, n_estimate_integral=128,
              n_euler_steps=6, seed=9, epoch=1)
    if kind == "cha_mlp":
        eq = dpi.Cha(100, 1.0, 5.0, 1.0)
        net = _random_mlp(eq, [128] * 4, 5)
        oeq, onet = O.Cha(100, 1.0, 5.0, 1.0), _oracle_mlp(net)
    elif kind == "ou_pis":
        eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
        oeq = O.OUProcessEquation(100, eq.mean.numpy(), eq.var.numpy(), eq.pi.numpy(), alpha_scale=4.0)
        onet = O.PISGradNet({k: v.detach().double().numpy() for k, v in net.state_dict().items()}, oeq, T=1.0)
    else:
        eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
        net = _random_mlp(eq, [64] * 3, 5)
        oeq, onet = O.GBMEquationComplexExact(100, eq.w.numpy(), eq.v.numpy()), _oracle_mlp(net)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, **kw)
    nx, hess = eq.nx, kind == "gbm_hess"
    width = 1 + nx + (nx * nx if hess else 0)
    pb0 = gen.point_base
    if hess:
        tx0, y0 = gen.sample_with_gradients_and_hessians(0)
    else:
        tx0, y0 = gen.sample_with_gradients(0)
    assert tuple(tx0.shape) == (0, 1 + nx) and tuple(y0.shape) == (0, width) and y0.is_cuda
    assert gen.point_base == pb0
    empty = torch.empty(0, 1 + nx, device="cuda:0")
    y0 = gen.generate_with_gradients_and_hessians(empty) if hess else gen.generate_with_gradients(empty)
    assert tuple(y0.shape) == (0, width)
    torch.cuda.synchronize()

    tx, _ = gen.sample_t_and_x(1, point_base=17)
    if hess:
        y = gen.generate_with_gradients_and_hessians(tx, point_base=17).cpu().numpy()
        ref = O.labels_grad_hess(oeq, onet, tx.cpu().double().numpy(), 128, 6, 9, 1, 17)
    else:
        y = gen.generate_with_gradients(tx, point_base=17).cpu().numpy()
        ref = O.labels_grad(oeq, onet, tx.cpu().double().numpy(), 128, 6, 9, 1, 17)
    parts = rel_l2_parts(y, ref)
    print(kind, parts)
    assert all(v < TOL for v in parts.values()), parts


@pytest.mark.parametrize("kind", ["cha_mlp", "ou_pis", "gbm_hess"])
def test_label_call_captures_into_a_hip_graph(kind):
    """include/dpi.h: label calls are stream-ordered, allocate nothing and never synchronise, so a
    whole call (baseline, rollout / GEMM chain, reduce, finalize) captures into a hipGraph
    (torch.cuda.graph) whose replays reproduce the eager labels bit for bit."""
    import deeppicarditeration_amd as dpi
    torch.manual_seed(8)
    kw = dict(device="cuda:0", t_always_uniform=True, n_estimate_terminal=128, n_estimate_integral=128,
              n_euler_steps=5, seed=12, epoch=2)
    if kind == "cha_mlp":
        eq = dpi.Cha(100, 1.0, 5.0, 1.0)
        net = _random_mlp(eq, [128] * 4, 8)
    elif kind == "ou_pis":
        eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
    else:
        eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
        net = _random_mlp(eq, [64] * 3, 8)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, **kw)
    call = gen.generate_with_gradients_and_hessians if kind == "gbm_hess" else gen.generate_with_gradients
    tx, _ = gen.sample_t_and_x(6, point_base=40)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eager = call(tx, point_base=40).clone()  # also sizes the workspace before capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = call(tx, point_base=40)
    for _ in range(3):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, eager)


@pytest.mark.parametrize("kind", ["cha_mlp", "ou_pis", "gbm_sdgd", "gbm_sdgd_tanh", "gbm_full_f32"])
def test_side_stream_preparation_equals_labels(kind):
    """bench.py's pipeline: ShardedLabeler.prepare (sampling + per-point baseline on a side stream,
    three rotating workspaces) -> begin -> end, with one batch in flight, gives every batch's labels
    bit for bit as the one-stream labels() call on the same points."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd.sharding import ShardedLabeler

    def make():
        torch.manual_seed(4)
        hess = None
        if kind == "cha_mlp":
            eq = dpi.Cha(100, 1.0, 5.0, 1.0)
            net = _random_mlp(eq, [128] * 4, 4)
        elif kind.startswith("gbm"):  # the noise sums staged by k_noise_shared (dpi_label_prepare)
            eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
            torch.manual_seed(4)
            net = dpi.construct_mlp(101, 1, [64] * 3, ["Tanh" if kind.endswith("tanh") else "ELU"] * 3, None)
            hess = None if kind == "gbm_full_f32" else {"method": "SDGD", "kwargs": {"v": 100}}
        else:
            eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                       alpha_scale=4.0)
            net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=100, g0=eq.g, T=1.0)
        gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True,
                                      n_estimate_terminal=256, n_estimate_integral=256, n_euler_steps=6, seed=3,
                                      hessian_approximation=hess)
        if kind.endswith("f32"):
            gen.net.set_precision(0)
        return gen

    lab, ref = ShardedLabeler(make()), ShardedLabeler(make())
    got, pending = [], []
    for _ in range(7):
        pending.append(lab.begin(prepared=lab.prepare(16)))
        if len(pending) > 1:
            got.append(lab.end(pending.pop(0)))
    got.append(lab.end(pending.pop(0)))
    torch.cuda.synchronize()
    for y in got:
        tx, pb = ref.gen.sample_t_and_x(16)
        assert torch.equal(y, ref.labels(tx, pb))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["split", "f32"])
def test_side_stream_preparation_equals_hessian_labels(precision):
    """bench.py --workload gbm_hess: ShardedLabeler.prepare(n, hessians=True) (sampling, per-point
    baseline and the k_noise_shared noise sums on a side stream, two batches prepared ahead) ->
    labels_hessians(prepared=...) gives every batch's Hessian labels bit for bit as the unprepared
    call on the same points (the staged sums are the path launch's own, same counters and order)."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd.sharding import ShardedLabeler

    def make():
        eq = dpi.GBMEquationComplexExact(100, 1.0, 1.0)
        torch.manual_seed(4)
        net = dpi.construct_mlp(101, 1, [64] * 3, ["ELU"] * 3, None)
        gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                      n_estimate_integral=256, n_euler_steps=6, seed=3)
        if precision == "f32":
            gen.net.set_precision(0)
        return gen

    lab, ref = ShardedLabeler(make()), ShardedLabeler(make())
    got, prep = [], lab.prepare(8, hessians=True)
    for _ in range(5):
        nxt = lab.prepare(8, hessians=True)
        got.append(lab.labels_hessians(prepared=prep))
        prep = nxt
    got.append(lab.labels_hessians(prepared=prep))
    torch.cuda.synchronize()
    for y in got:
        tx, pb = ref.gen.sample_t_and_x(8)
        assert torch.equal(y, ref.labels_hessians(tx, pb))


@pytest.mark.gpu
def test_prepared_moments_check_the_prepare_call():
    """include/dpi.h DPI_PREPARED contract: a prepared moments call whose points, counters or MC
    range differ from the dpi_label_prepare call on its workspace, or that has no prepare (a second
    prepared call consumes nothing), fails with DPI_ERR_ARG instead of returning labels built from
    another batch's rollout; the matching call succeeds."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    torch.manual_seed(4)
    eq = dpi.OUProcessEquation(nx=100, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    net = dpi.PISGradNet(hidden_shapes=[32] * 2, dim=100, g0=eq.g, T=1.0)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=3, seed=3)
    tx, pb = gen.sample_t_and_x(4)
    ws = gen.point_baseline(tx)
    gen.label_prepare(tx, pb, 128, 0, 128, L.DPI_BOTH, ws)
    with pytest.raises(RuntimeError, match="DPI_PREPARED"):
        gen.label_moments(tx, pb + 1, 128, 0, 128, L.DPI_BOTH | L.DPI_PREPARED, ws)
    gen.label_prepare(tx, pb, 128, 0, 128, L.DPI_BOTH, ws)
    mom = gen.label_moments(tx, pb, 128, 0, 128, L.DPI_BOTH | L.DPI_PREPARED, ws)
    with pytest.raises(RuntimeError, match="DPI_PREPARED"):  # consumed
        gen.label_moments(tx, pb, 128, 0, 128, L.DPI_BOTH | L.DPI_PREPARED, ws)
    ref = gen.label_moments(tx, pb, 128, 0, 128, L.DPI_BOTH, gen.point_baseline(tx))
    torch.cuda.synchronize()
    assert torch.equal(mom, ref)


@pytest.mark.parametrize("hessians", [False, True])
def test_more_paths_than_one_call_takes(hessians):
    """M = 131,072 > DPI_PATHS_PER_CALL_MAX: the generator runs two label calls over [0, 65536) and
    [65536, 131072) and combines them (moments_reduce / sums_reduce), so reference-sized settings
    beyond one call's 1,024 path blocks work; the labels match the fp64 oracle on the same counters."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from oracle import dpi_oracle as O
    M, K = 2 * L.DPI_PATHS_PER_CALL_MAX, 4
    # (the fp64 Hessian oracle over 131,072 paths: 4 dimensions and a 2 x 16 network keep it to seconds)
    nx = 4 if hessians else 100
    if hessians:
        torch.manual_seed(3)
        eq = dpi.GBMEquationComplexExact(nx, 1.0, 1.0, w=0.3 * torch.randn(2, nx + 1), v=torch.randn(2, 1))
        net = dpi.construct_mlp(nx + 1, 1, [16] * 2, ["ELU"] * 2, None)
        oeq = O.GBMEquationComplexExact(nx, eq.w.numpy(), eq.v.numpy())
        act = ["ELU"] * 2
    else:
        eq = dpi.Cha(nx=100, T=1.0, k=5.0, alpha=1.0)
        torch.manual_seed(0)
        net = dpi.construct_mlp(101, 1, [32] * 2, ["ELU"] * 2, None)
        oeq = O.Cha(100, 1.0, 5.0, 1.0)
        act = ["ELU"] * 2
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=K, seed=1)
    tx, _ = gen.sample_t_and_x(1, point_base=0)
    y = (gen.generate_with_gradients_and_hessians(tx, point_base=0) if hessians
         else gen.generate_with_gradients(tx, point_base=0)).cpu().double().numpy()
    lin = [m for m in net if isinstance(m, torch.nn.Linear)]
    onet = O.MLP([m.weight.detach().double().numpy() for m in lin], [m.bias.detach().double().numpy() for m in lin], act)
    txh = tx.cpu().double().numpy()
    ref = (O.labels_grad_hess(oeq, onet, txh, M, K, 1, 1, 0, m_chunk=4096) if hessians
           else O.labels_grad(oeq, onet, txh, M, K, 1, 1, 0, m_chunk=4096))
    def rel(a, b):
        return float(np.linalg.norm(a - b) / np.linalg.norm(b))
    ev, eg = rel(y[:, :1], ref[:, :1]), rel(y[:, 1:nx + 1], ref[:, 1:nx + 1])
    print(f"M = {M}: value {ev:.2e} grad {eg:.2e}")
    assert ev < 1e-4 and eg < 1e-4
    if hessians:
        eh = rel(y[:, nx + 1:], ref[:, nx + 1:])
        print(f"hessian {eh:.2e}")
        assert eh < 1e-4
