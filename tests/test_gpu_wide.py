"""State dimensions above 128: the wide first-order instances (Cha / OU / GBM, nx <= NXW_MAX = 256,
one workgroup per CU) against the reference's own labels (tests/golden/wide_*,
made by tests/golden/make_golden.py from picard/data.py at nx = 200 and 256) and against the fp64
oracle, in both MFMA modes; and the refusals that remain (TD estimators, Hessian labels, PISGradNet
above 128).  Reference: every equation takes any nx (picard/equations.py:266-338, 388-486, 599-714)."""
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


from golden_util import CASES, load  # noqa: E402
from gpu_util import generator, product_equation, product_module, rel_l2_parts  # noqa: E402
from oracle import dpi_oracle as O  # noqa: E402

WIDE = [c for c in CASES if c.startswith("wide_")]


@pytest.fixture(params=["f32", "auto"])
def precision(request):
    from deeppicarditeration_amd import _lib as L
    mode = L.DPI_GEMM_F32 if request.param == "f32" else L.DPI_GEMM_AUTO
    L.check(L.load().dpi_set_gemm_precision(mode), "gemm precision")
    yield request.param
    L.check(L.load().dpi_set_gemm_precision(L.DPI_GEMM_AUTO), "gemm precision")


def test_wide_fixtures_cover_200_and_256():
    nxs = {int(load(c)["eqkw_nx"]) for c in WIDE}
    eqs = {str(load(c)["eq"]) for c in WIDE}
    assert {200, 256} <= nxs and {"Cha", "OUProcessEquation", "GBMEquationComplexExact"} <= eqs


@pytest.mark.parametrize("case", WIDE)
def test_wide_golden_reference_parity(case, precision):
    f = load(case)
    eq = product_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    tx = torch.as_tensor(f["tx"], dtype=torch.float32, device="cuda:0")
    y = gen.generate_with_gradients(tx, point_base=int(f["point_base"])).cpu().numpy()
    parts = rel_l2_parts(y, f["y"])
    print(case, precision, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("case", ["wide_cha256_mlp128x4_tanh_K2", "wide_ou200_mlp32x2_K2"])
def test_wide_sample_with_gradients_matches_the_reference_draws(case):
    """The points (draws 1-3) and labels of one sample_with_gradients call at nx > 128."""
    f = load(case)
    eq = product_equation(f)
    gen = generator(f, eq, product_module(f, eq))
    tx, y = gen.sample_with_gradients(int(f["n"]))
    assert np.allclose(tx.cpu().numpy(), f["tx"], rtol=0, atol=2e-5)
    parts = rel_l2_parts(y.cpu().numpy(), f["y"])
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def _mlp(eq, widths, seed, act="ELU"):
    import deeppicarditeration_amd as dpi
    torch.manual_seed(seed)
    return dpi.construct_mlp(1 + eq.nx, 1, widths, [act] * len(widths), None)


def _oracle_mlp(m, act="ELU"):
    lin = [l for l in m if isinstance(l, torch.nn.Linear)]
    return O.MLP([l.weight.detach().double().numpy() for l in lin], [l.bias.detach().double().numpy() for l in lin],
                 [act] * (len(lin) - 1))


@pytest.mark.parametrize("nx", [129, 144, 200, 255, 256])
def test_wide_dimension_edges_vs_oracle(nx, precision):
    """Ragged wide dimensions: just past the two-workgroup cap (129), a partial 32-column split
    chunk (144 = 4.5 chunks), a partial 4-dim block (255) and the cap itself (256); Cha, 2 x 64 ELU."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(nx, 1.0, 5.0, 1.0)
    net = _mlp(eq, [64, 64], 11)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=3, seed=4, epoch=3)
    tx, y = gen.sample_with_gradients(3)
    ref = O.labels_grad(O.Cha(nx, 1.0, 5.0, 1.0), _oracle_mlp(net), tx.cpu().double().numpy(), 128, 3, 4, 3, 0)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("act", ["ELU", "Tanh"])
def test_wide_burgers_256d_config_network_k50_vs_oracle(act, precision):
    """The configs[1] network shape (4 x 128) at nx = 256, K = 50, 2,048 paths, against the oracle."""
    import deeppicarditeration_amd as dpi
    eq = dpi.Cha(256, 1.0, 5.0, 1.0)
    net = _mlp(eq, [128] * 4, 5, act)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=2048,
                                  n_estimate_integral=2048, n_euler_steps=50, seed=9, epoch=1)
    tx, y = gen.sample_with_gradients(2)
    ref = O.labels_grad(O.Cha(256, 1.0, 5.0, 1.0), _oracle_mlp(net, act), tx.cpu().double().numpy(), 2048, 50, 9, 1, 0,
                        m_chunk=512)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    print(act, precision, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_wide_ou_gmm_vs_oracle(precision):
    import deeppicarditeration_amd as dpi
    rng = np.random.default_rng(3)
    K, nx = 5, 240
    mean, var, pi = rng.uniform(-1, 1, (K, nx)), np.full((K, nx), 2.0), rng.uniform(0.1, 1, K)
    pi = pi / pi.sum()
    eq = dpi.OUProcessEquation(nx=nx, T=1.0, alpha=1.0, num_components=K, mean=mean, var=var, pi=pi, alpha_scale=4.0)
    net = _mlp(eq, [128] * 3, 7)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                  n_estimate_integral=256, n_euler_steps=10, seed=2, epoch=5)
    tx, y = gen.sample_with_gradients(3)
    oeq = O.OUProcessEquation(nx, mean, var, pi, alpha_scale=4.0)
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 256, 10, 2, 5, 0)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


@pytest.mark.parametrize("v", [100, 0])
def test_wide_gbm_config5_network_vs_oracle(v, precision):
    """The configs[4] network (3 x 64 ELU) at nx = 240, K = 20: SDGD v = 100 (the per-path direction
    lists, 64-bit list masks) and the exact diagonal (v = 0: all 240 directions), against the oracle."""
    import deeppicarditeration_amd as dpi
    rng = np.random.default_rng(5)
    nx = 240
    w = rng.standard_normal((2, 1 + nx)) / np.sqrt(nx)
    w[:, 0] = 1.0
    vv = rng.standard_normal((2, 1))
    eq = dpi.GBMEquationComplexExact(nx, 1.0, 1.0, w=w, v=vv)
    net = _mlp(eq, [64] * 3, 6)
    hess = {"method": "SDGD", "kwargs": {"v": v}} if v else None
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=20, seed=3, epoch=2, hessian_approximation=hess)
    tx, y = gen.sample_with_gradients(2)
    oeq = O.GBMEquationComplexExact(nx, eq.w.numpy(), eq.v.numpy())
    ref = O.labels_grad(oeq, _oracle_mlp(net), tx.cpu().double().numpy(), 128, 20, 3, 2, 0, v=v)
    parts = rel_l2_parts(y.cpu().numpy(), ref)
    print("gbm wide", v, precision, parts)
    assert parts["value"] < TOL and parts["grad"] < TOL, parts


def test_wide_gbm_prepared_equals_plain():
    """The GBM prepare schedule (noise sums staged by k_noise_shared on the side stream) at nx = 200:
    bitwise the unprepared labels."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd.sharding import ShardedLabeler
    rng = np.random.default_rng(8)
    nx = 200
    w = rng.standard_normal((2, 1 + nx)) / np.sqrt(nx)
    w[:, 0] = 1.0
    eq = dpi.GBMEquationComplexExact(nx, 1.0, 1.0, w=w, v=rng.standard_normal((2, 1)))
    net = _mlp(eq, [64] * 3, 9)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=1024,
                                  n_estimate_integral=1024, n_euler_steps=5, seed=4,
                                  hessian_approximation={"method": "SDGD", "kwargs": {"v": 100}})
    lab = ShardedLabeler(gen, rank=0, world=1)
    prep = lab.prepare(8)
    tx, pb = prep[:2]
    y_prep = lab.end(lab.begin(prepared=prep))
    y_plain = ShardedLabeler(gen, rank=0, world=1).labels(tx, pb)
    assert torch.equal(y_prep, y_plain)


def test_wide_labels_are_shard_invariant():
    """4,096 paths as 2 and 4 MC shards reduce to the one-call moments bit for bit (M / 64 G a power
    of two), as on 2 / 4 GPUs; the labels are bitwise reproducible."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    eq = dpi.Cha(200, 1.0, 5.0, 1.0)
    net = _mlp(eq, [128] * 2, 12)
    M = 4096
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=5, seed=1)
    tx, _ = gen.sample_t_and_x(4, point_base=0)
    ws = gen.point_baseline(tx)
    full = gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws)
    assert torch.equal(full, gen.label_moments(tx, 0, M, 0, M, L.DPI_BOTH, ws))
    for G in (2, 4):
        parts = torch.stack([gen.label_moments(tx, 0, M, r * M // G, (r + 1) * M // G, L.DPI_BOTH, ws)
                             for r in range(G)]).contiguous()
        out = torch.empty_like(full)
        L.check(gen.lib.dpi_moments_reduce(L.c_void_p(parts.data_ptr()), G, 4, 200, L.c_void_p(out.data_ptr()),
                                           L.c_void_p(torch.cuda.current_stream().cuda_stream)), "moments_reduce")
        assert torch.equal(out, full), G


def test_wide_refusals_name_the_cap():
    """What stays at nx <= 128: the TD estimators, the Malliavin Hessian labels and PISGradNet (named
    refusals)."""
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd._lib import DPIError
    eq = dpi.Cha(200, 1.0, 5.0, 1.0)
    net = _mlp(eq, [32, 32], 1)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                  n_estimate_integral=64, n_euler_steps=2, seed=1, estimate_delta_t=0.3)
    with pytest.raises((DPIError, NotImplementedError), match="128"):
        gen.sample_with_gradients(2)
    g = dpi.GBMEquationComplexExact(200, 1.0, 1.0, w=np.full((2, 201), 0.1), v=np.ones((2, 1)))
    gen = dpi.OnlineDataGenerator(g, _mlp(g, [32, 32], 2), 1, 1, device="cuda:0", t_always_uniform=True,
                                  n_estimate_terminal=64, n_estimate_integral=64, n_euler_steps=2, seed=1)
    with pytest.raises((DPIError, NotImplementedError), match="128"):
        gen.sample_with_gradients_and_hessians(2)
    o = dpi.OUProcessEquation(nx=200, T=1.0, alpha=1.0, num_components=2, mean=np.zeros((2, 200)),
                              var=np.full((2, 200), 2.0), pi=np.full(2, 0.5))
    pis = dpi.PISGradNet(hidden_shapes=[32, 32], dim=200, g0=o.g, T=1.0)
    with pytest.raises((DPIError, NotImplementedError), match="128"):
        dpi.OnlineDataGenerator(o, pis, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                n_estimate_integral=64, n_euler_steps=2, seed=1).sample_with_gradients(2)
