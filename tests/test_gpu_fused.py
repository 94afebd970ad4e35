"""sample_with_gradients in fewer launches against the separate launches they replace —
k_sample_points, k_baseline, k_paths, k_reduce — bit for bit (reference picard/data.py:211-223):
the one-launch form (round 6, k_paths_fb: base workgroups ahead of the path workgroups, an in-launch
hand-off per point) and the two-launch form (round 4, DPI_FUSED_BASE=0: the points sampled inside
the baseline launch, dpi_sample_points_baseline), both with the label reduce inside the path launch
(k_paths' last block per point, DPI_FUSED_REDUCE)."""
import pytest
import torch

import deeppicarditeration_amd as dpi
from deeppicarditeration_amd import _lib as L
from deeppicarditeration_amd.sharding import ShardedLabeler

pytestmark = pytest.mark.gpu

NX = 100


def _make(kind, M, K, t_uniform=True, seed=7):
    torch.manual_seed(0)
    hess = None
    if kind in ("cha", "zero"):
        eq, widths = dpi.Cha(NX, 1.0, 5.0, 1.0), [128] * 4
    elif kind == "ou":
        eq = dpi.OUProcessEquation(nx=NX, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        widths = [64, 64]
    else:
        eq, widths = dpi.GBMEquationComplexExact(NX, 1.0, 1.0), [64] * 3
        hess = {"method": "SDGD", "kwargs": {"v": 100}}
    net = dpi.construct_mlp(1 + NX, 1, widths, ["ELU"] * len(widths), None) if kind != "zero" else dpi.ZeroSolution(1)
    return dpi.OnlineDataGenerator(eq, net, 10, 3, device="cuda:0", t_always_uniform=t_uniform, n_estimate_terminal=M,
                                   n_estimate_integral=M, n_euler_steps=K, seed=seed, hessian_approximation=hess)


def _separate(gen, n, pb):
    """k_sample_points, then k_baseline + k_paths + k_reduce (DPI_FUSED_REDUCE=0)."""
    tx, _ = gen.sample_t_and_x(n, point_base=pb)
    ws = gen.point_baseline(tx)
    y, mom = gen.label_moments_finalize(tx, pb, gen.n_estimate_integral, L.DPI_BOTH, ws)
    return tx, y, mom


@pytest.mark.parametrize("kind,n,M,K,t_uniform", [("cha", 16, 4096, 50, True), ("cha", 5, 192, 3, False),
                                                  ("gbm", 8, 1024, 4, True), ("ou", 3, 128, 4, True),
                                                  ("zero", 4, 64, 2, True)])
@pytest.mark.parametrize("fused_base", ["1", "0"])
def test_two_launch_sample_with_gradients_is_bitwise_the_separate_launches(kind, n, M, K, t_uniform, fused_base,
                                                                           monkeypatch):
    """fused_base "1": one launch for Cha / OU / zero nets (GBM keeps two); "0": two launches."""
    gen = _make(kind, M, K, t_uniform)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "0")
    tx0, y0, mom0 = _separate(gen, n, 40)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    monkeypatch.setenv("DPI_FUSED_BASE", fused_base)
    tx1, y1 = gen.sample_generate(n, 40)
    mom1 = gen.last_moments
    torch.cuda.synchronize()
    assert torch.equal(tx0, tx1)
    assert torch.equal(mom0, mom1)
    assert torch.equal(y0, y1)
    assert torch.isfinite(y1).all()


@pytest.mark.parametrize("n,M", [(512, 128), (64, 4096), (1, 64), (300, 1024)])
def test_one_launch_many_points(n, M, monkeypatch):
    """k_paths_fb with many hand-offs: more base workgroups than one round of the grid holds (512
    points), a point per 64 path workgroups (64 x 4096), one point, a ragged count."""
    gen = _make("cha", M, 3)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "0")
    tx0, y0, mom0 = _separate(gen, n, 11)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    tx1, y1 = gen.sample_generate(n, 11)
    torch.cuda.synchronize()
    assert torch.equal(tx0, tx1)
    assert torch.equal(mom0, gen.last_moments)
    assert torch.equal(y0, y1)


def test_one_launch_repeated_on_one_workspace_and_leaves_the_baseline(monkeypatch):
    """Three one-launch calls on one workspace (each its own hand-off sequence number, so the words
    the previous call left never match) give the same points and labels; afterwards the workspace
    holds the baseline dpi_point_baseline leaves, so a label call on it matches too."""
    gen = _make("cha", 1024, 3)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    outs = [gen.sample_generate(6, 5) for _ in range(3)]
    for tx, y in outs[1:]:
        assert torch.equal(tx, outs[0][0]) and torch.equal(y, outs[0][1])
    ws = gen._workspace(6, 1024)
    y2, _ = gen.label_moments_finalize(outs[0][0], 5, 1024, L.DPI_BOTH, ws)
    assert torch.equal(y2, outs[0][1])


@pytest.mark.parametrize("variant", ["fp32", "tanh", "td", "ou128x4", "h16"])
def test_nets_without_the_one_launch_form_keep_two_launches(variant, monkeypatch):
    """Exact-fp32 mode, Tanh nets, the TD estimators, OU with a 4 x 128 net and 16-wide nets have no
    k_paths_fb instance: the call runs two launches and still equals the separate launches."""
    torch.manual_seed(0)
    eq = dpi.Cha(NX, 1.0, 5.0, 1.0)
    if variant == "ou128x4":
        eq = dpi.OUProcessEquation(nx=NX, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
    act = "Tanh" if variant == "tanh" else "ELU"
    widths = [128] * 4 if variant == "ou128x4" else [16, 16] if variant == "h16" else [64, 64]
    net = dpi.construct_mlp(1 + NX, 1, widths, [act] * len(widths), None)
    gen = dpi.OnlineDataGenerator(eq, net, 10, 3, device="cuda:0", t_always_uniform=True, n_estimate_terminal=256,
                                  n_estimate_integral=256, n_euler_steps=3, seed=7,
                                  estimate_delta_t=0.25 if variant == "td" else None)
    if variant == "fp32":
        gen.use_fp32()
    monkeypatch.setenv("DPI_FUSED_REDUCE", "0")
    tx0, y0, mom0 = _separate(gen, 5, 2)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    tx1, y1 = gen.sample_generate(5, 2)
    assert torch.equal(tx0, tx1) and torch.equal(y0, y1) and torch.equal(mom0, gen.last_moments)


def test_fused_reduce_repeated_calls_reuse_the_tickets(monkeypatch):
    """The tickets reset themselves: three calls on one workspace (one baseline) equal fresh ones."""
    gen = _make("cha", 1024, 2)
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    tx, _ = gen.sample_t_and_x(6, point_base=3)
    ws = gen.point_baseline(tx)
    outs = [gen.label_moments_finalize(tx, 3, 1024, L.DPI_BOTH, ws)[0] for _ in range(3)]
    monkeypatch.setenv("DPI_FUSED_REDUCE", "0")
    ref = gen.label_moments_finalize(tx, 3, 1024, L.DPI_BOTH, ws)[0]
    for y in outs:
        assert torch.equal(y, ref)


def test_sharded_moments_with_the_fused_reduce_equal_the_single_call(monkeypatch):
    """Two MC shards of 2048 paths (32 blocks each, fused reduce) combined by the rank tree equal one
    4096-path call (64 blocks) bit for bit."""
    monkeypatch.setenv("DPI_FUSED_REDUCE", "1")
    gen = _make("cha", 4096, 3)
    tx, pb = gen.sample_t_and_x(4, point_base=0)
    ws = gen.point_baseline(tx)
    parts = torch.stack([gen.label_moments(tx, pb, 4096, r * 2048, (r + 1) * 2048, L.DPI_BOTH, ws) for r in range(2)])
    two = gen.moments_reduce(parts)
    one = gen.label_moments(tx, pb, 4096, 0, 4096, L.DPI_BOTH, ws)
    assert torch.equal(one, two)


def test_generator_and_labeler_surfaces_use_the_two_launch_path():
    """sample_with_gradients of the generator and of a one-rank ShardedLabeler: same points, same
    labels as the separate launches."""
    a, b, c = _make("cha", 512, 3), _make("cha", 512, 3), _make("cha", 512, 3)
    tx_a, y_a = a.sample_with_gradients(8)
    tx_b, y_b = ShardedLabeler(b).sample_with_gradients(8)
    tx_c, y_c, _ = _separate(c, 8, 0)
    assert torch.equal(tx_a, tx_c) and torch.equal(tx_b, tx_c)
    assert torch.equal(y_a, y_c) and torch.equal(y_b, y_c)


def test_prepare_with_points_sampled_ahead_equals_labels():
    """ShardedLabeler(sample_ahead=True) (PISGradNet, the bench's HJB schedule): every prepared batch
    gets the next consecutive point range, and its labels equal labels() on the same points."""
    torch.manual_seed(0)
    eq = dpi.OUProcessEquation(nx=NX, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=NX, g0=eq.g, T=1.0)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=128,
                                  n_estimate_integral=128, n_euler_steps=4, seed=5)
    lab = ShardedLabeler(gen, sample_ahead=True)
    got = []
    for _ in range(3):
        prep = lab.prepare(3)
        got.append((prep[0], prep[1], lab.end(lab.begin(prepared=prep))))
    torch.cuda.synchronize()
    ref = ShardedLabeler(gen)
    for b, (tx, pb, y) in enumerate(got):
        assert pb == got[0][1] + 3 * b
        tx0, _ = gen.sample_t_and_x(3, point_base=pb)
        assert torch.equal(tx, tx0)
        assert torch.equal(y, ref.labels(tx, pb))


def test_points_sampled_ahead_under_another_epoch_are_dropped():
    """A batch sampled ahead under the generator's previous epoch (a new Picard iteration reusing
    the labeler) is not used: the next prepare() samples its points afresh under the new epoch."""
    torch.manual_seed(0)
    eq = dpi.OUProcessEquation(nx=NX, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                               alpha_scale=4.0)
    net = dpi.PISGradNet(hidden_shapes=[512] * 2, dim=NX, g0=eq.g, T=1.0)
    gen = dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=64,
                                  n_estimate_integral=64, n_euler_steps=2, seed=5)
    lab = ShardedLabeler(gen, sample_ahead=True)
    prep = lab.prepare(2)
    lab.end(lab.begin(prepared=prep))
    gen.epoch += 1
    prep = lab.prepare(2)
    tx, pb = prep[0], prep[1]
    y = lab.end(lab.begin(prepared=prep))
    tx0, _ = gen.sample_t_and_x(2, point_base=pb)
    assert torch.equal(tx, tx0)
    assert torch.equal(y, ShardedLabeler(gen).labels(tx, pb))


def test_fused_label_call_without_a_baseline_on_its_workspace_fails():
    """The fused reduce counts blocks on tickets the baseline launch zeroes: a label call on a
    workspace no baseline of these points was enqueued on fails (DPI_ERR_ARG) instead of running a
    reduce that never fires."""
    gen = _make("cha", 256, 2)
    tx, pb = gen.sample_t_and_x(3, point_base=0)
    # an address no earlier workspace of this process started at (an odd offset into a fresh block)
    odd = 7 * 4096 + 256
    ws = torch.empty(gen.workspace_bytes(3, 256) + odd, dtype=torch.uint8, device="cuda:0")[odd:]
    with pytest.raises(L.DPIError, match="baseline"):
        gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, ws)
    gen.point_baseline(tx, ws=ws)
    y, _ = gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, ws)
    assert torch.isfinite(y).all()


@pytest.mark.gpu
def test_a_reused_workspace_address_loses_its_baseline_tag():
    """the fused reduce's baseline tag is keyed on the workspace address, which the
    caching allocator hands out again.  dpi_workspace_forget (called by new_workspace on every
    workspace the package allocates) drops the old records, so a label call on the new workspace
    without its own baseline fails again."""
    from deeppicarditeration_amd.data import new_workspace
    gen = _make("cha", 256, 2)
    tx, pb = gen.sample_t_and_x(3, point_base=0)
    odd = 11 * 4096 + 512
    ws = torch.empty(gen.workspace_bytes(3, 256) + odd, dtype=torch.uint8, device="cuda:0")[odd:]
    gen.point_baseline(tx, ws=ws)
    y, _ = gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, ws)
    torch.cuda.synchronize()
    L.check(L.load().dpi_workspace_forget(L.c_void_p(ws.data_ptr()), ws.numel()), "dpi_workspace_forget")
    with pytest.raises(L.DPIError, match="baseline"):
        gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, ws)
    fresh = new_workspace(gen.workspace_bytes(3, 256), "cuda:0")
    with pytest.raises(L.DPIError, match="baseline"):
        gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, fresh)
    gen.point_baseline(tx, ws=fresh)
    assert torch.equal(gen.label_moments_finalize(tx, pb, 256, L.DPI_BOTH, fresh)[0], y)
