"""No label call writes outside the buffers it is given (the round-4 k_pis_net
row saves once landed up to 1 MB past the workspace, DESIGN.md §2.4 "Partial tiles").

Every workspace-using C-ABI entry point runs on buffers carved from one allocation in which each
buffer it writes (workspace, moments, Hessian sums, labels) is followed by a 4 MB canary of 0xA5,
at partial-tile shapes (point counts that leave a partial 64-row / 128-row tile, shards with
m_begin > 0); every canary must come back untouched and every output finite.  Run once after each
kernel change, never in a loop."""
import ctypes

import pytest
import torch

import deeppicarditeration_amd as dpi
from deeppicarditeration_amd import _lib as L

pytestmark = pytest.mark.gpu

NX = 100
CANARY = 4 << 20
MAGIC = 0xA5


class Carved:
    """Named buffers in one uint8 allocation, each followed by a CANARY-byte guard band."""

    def __init__(self, **sizes):
        self.off, o = {}, 0
        for k, b in sizes.items():
            b = (int(b) + 255) & ~255
            self.off[k] = (o, b)
            o += b + CANARY
        self.buf = torch.full((o,), MAGIC, dtype=torch.uint8, device="cuda:0")

    def u8(self, k):
        o, b = self.off[k]
        return self.buf[o:o + b]

    def f32(self, k, *shape):
        o, _ = self.off[k]
        n = 1
        for s in shape:
            n *= s
        return self.buf[o:o + 4 * n].view(torch.float32).view(*shape)

    def ptr(self, k):
        return ctypes.c_void_p(self.u8(k).data_ptr())

    def nbytes(self, k):
        return self.off[k][1]

    def check(self):
        torch.cuda.synchronize()
        for k, (o, b) in self.off.items():
            band = self.buf[o + b:o + b + CANARY]
            assert bool((band == MAGIC).all()), f"canary after {k!r} overwritten"


def _gen(kind, M, K=3, delta_t=0.0, widths=None):
    torch.manual_seed(0)
    hess = None
    if kind == "cha":
        eq = dpi.Cha(NX, 1.0, 5.0, 1.0)
        net = dpi.construct_mlp(1 + NX, 1, widths or [128] * 4, ["ELU"] * len(widths or [128] * 4), None)
    elif kind in ("gbm", "gbm_sdgd"):
        eq = dpi.GBMEquationComplexExact(NX, 1.0, 1.0)
        net = dpi.construct_mlp(1 + NX, 1, [64] * 3, ["ELU"] * 3, None)
        if kind == "gbm_sdgd":
            hess = {"method": "SDGD", "kwargs": {"v": 100}}
    else:
        eq = dpi.OUProcessEquation(nx=NX, T=1.0, alpha=1.0, num_components=5, mean_scale=1.0, var_scale=2.0,
                                   alpha_scale=4.0)
        net = dpi.PISGradNet(hidden_shapes=[512] * 4, dim=NX, g0=eq.g, T=1.0)
    return dpi.OnlineDataGenerator(eq, net, 1, 1, device="cuda:0", t_always_uniform=True, n_estimate_terminal=M,
                                   n_estimate_integral=M, n_euler_steps=K, seed=5, hessian_approximation=hess,
                                   estimate_delta_t=delta_t)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _first_order(gen, n, M, m0, m1, flags=L.DPI_BOTH, finalize=True, prepared=False):
    F = 1 + NX
    need = gen.workspace_bytes(n, M, prepared=prepared)  # prepared: + the staged noise sums (GBM)
    c = Carved(ws=need, mom=n * 2 * F * 4, y=n * F * 4)
    tx, pb = gen.sample_t_and_x(n, point_base=11)
    gen.point_baseline(tx, ws=c.u8("ws"))
    lib, p, h = gen.lib, gen.problem, gen.net.handle
    args = (p, h, ctypes.c_void_p(tx.data_ptr()), n, M, gen.K, gen.seed, gen.epoch, pb)
    if prepared:
        L.check(lib.dpi_label_prepare(*args, m0, m1, flags, c.ptr("ws"), c.nbytes("ws"), _stream()), "prepare")
        flags |= L.DPI_PREPARED
    if finalize:
        assert (m0, m1) == (0, M)
        L.check(lib.dpi_label_moments_finalize(*args, flags, float("inf"), c.ptr("y"), c.ptr("mom"), c.ptr("ws"),
                                               c.nbytes("ws"), _stream()), "moments_finalize")
    else:
        L.check(lib.dpi_label_moments(*args, m0, m1, flags, c.ptr("mom"), c.ptr("ws"), c.nbytes("ws"), _stream()),
                "moments")
    c.check()
    assert torch.isfinite(c.f32("mom", n, 2, F)).all()
    if finalize:
        assert torch.isfinite(c.f32("y", n, F)).all()


# (kind, n points, M paths, [m_begin, m_end), estimator flags, finalize?, prepared?, TD horizon)
FIRST_ORDER = {
    "cha_fused_partial": ("cha", 3, 192, 0, 192, L.DPI_BOTH, True, False, 0.0),
    "cha_shard_m0": ("cha", 5, 512, 128, 320, L.DPI_BOTH, False, False, 0.0),
    "cha_more_than_64_blocks": ("cha", 2, 8192, 0, 8192, L.DPI_BOTH, True, False, 0.0),
    "cha_terminal_only": ("cha", 3, 128, 0, 128, L.DPI_TERMINAL, True, False, 0.0),
    "cha_h16": ("cha16", 7, 64, 0, 64, L.DPI_BOTH, True, False, 0.0),
    "cha_td": ("cha", 3, 192, 0, 192, L.DPI_BOTH, True, False, 0.3),
    "gbm_sdgd": ("gbm_sdgd", 3, 192, 0, 192, L.DPI_BOTH, True, False, 0.0),
    "gbm_sdgd_shard": ("gbm_sdgd", 3, 256, 64, 192, L.DPI_BOTH, False, False, 0.0),
    "gbm_td": ("gbm_sdgd", 2, 128, 0, 128, L.DPI_BOTH, True, False, 0.4),
    # the noise sums staged by dpi_label_prepare (k_noise_shared) into the workspace, then read
    "gbm_prepared": ("gbm_sdgd", 3, 192, 0, 192, L.DPI_BOTH, True, True, 0.0),
    "gbm_prepared_shard": ("gbm_sdgd", 5, 256, 64, 192, L.DPI_BOTH, False, True, 0.0),
    "pis_partial_tile": ("pis", 3, 64, 0, 64, L.DPI_BOTH, True, False, 0.0),
    "pis_shard_m0": ("pis", 3, 256, 64, 192, L.DPI_BOTH, False, False, 0.0),
    "pis_prepared": ("pis", 5, 128, 0, 128, L.DPI_BOTH, True, True, 0.0),
    "pis_td": ("pis", 3, 128, 0, 128, L.DPI_BOTH, True, False, 0.3),
    # 65 points x 64 path blocks = 4,160 path sets: two pipeline chunks (4,096 per chunk), the first
    # with the 65 baseline rows (a partial 64-row tile)
    "pis_two_chunks": ("pis", 65, 4096, 0, 4096, L.DPI_BOTH, True, False, 0.0),
}


@pytest.mark.parametrize("case", sorted(FIRST_ORDER))
@pytest.mark.parametrize("mode", ["auto", "f32"])
def test_first_order_calls_write_nothing_outside_their_buffers(case, mode):
    kind, n, M, m0, m1, flags, fin, prep, dt = FIRST_ORDER[case]
    if mode == "f32" and case in ("pis_two_chunks", "cha_more_than_64_blocks"):
        pytest.skip("one precision suffices for the large shapes")
    widths = [16] if kind == "cha16" else None
    gen = _gen("cha" if kind == "cha16" else kind, M, delta_t=dt, widths=widths)
    if mode == "f32":
        gen.net.set_precision(L.DPI_GEMM_F32)
    _first_order(gen, n, M, m0, m1, flags, fin, prep)


@pytest.mark.parametrize("n,M,m0,m1,flags", [(3, 192, 0, 192, L.DPI_BOTH), (5, 256, 64, 192, L.DPI_BOTH),
                                             (2, 8192, 0, 8192, L.DPI_BOTH), (3, 128, 0, 128, L.DPI_TERMINAL),
                                             (3, 192, 64, 192, L.DPI_INTEGRAL)])
def test_hessian_label_calls_write_nothing_outside_their_buffers(n, M, m0, m1, flags):
    """dpi_label_moments_hessians + dpi_label_finalize_hessians (a shard with m_begin > 0, more than
    64 path blocks: the wave-per-column reduce, one estimator alone: the unequal-count passes), and
    the one-call dpi_generate_with_gradients_and_hessians."""
    gen = _gen("gbm", M)
    F, C = 1 + NX, NX * NX
    need = max(gen.workspace_bytes(n, M, hessians=True), gen.workspace_bytes(n, M))
    c = Carved(ws=need, mom=n * 2 * F * 4, hs=n * C * 4, y=n * (F + C) * 4, y1=n * (F + C) * 4)
    tx, pb = gen.sample_t_and_x(n, point_base=3)
    gen.point_baseline(tx, hessians=True, ws=c.u8("ws"))
    lib, p, h = gen.lib, gen.problem, gen.net.handle
    txp = ctypes.c_void_p(tx.data_ptr())
    L.check(lib.dpi_label_moments_hessians(p, h, txp, n, M, gen.K, gen.seed, gen.epoch, pb, m0, m1, flags,
                                           c.ptr("mom"), c.ptr("hs"), c.ptr("ws"), c.nbytes("ws"), _stream()),
            "moments_hessians")
    L.check(lib.dpi_label_finalize_hessians(p, c.ptr("mom"), c.ptr("hs"), n, M, flags, float("inf"), c.ptr("y"),
                                            c.ptr("ws"), c.nbytes("ws"), _stream()), "finalize_hessians")
    if (m0, m1) == (0, M) and flags == L.DPI_BOTH:
        L.check(lib.dpi_generate_with_gradients_and_hessians(p, h, txp, n, M, gen.K, gen.seed, gen.epoch, pb,
                                                             float("inf"), c.ptr("y1"), c.ptr("ws"), c.nbytes("ws"),
                                                             _stream()), "generate_hessians")
    c.check()
    assert torch.isfinite(c.f32("y", n, F + C)).all()
    if (m0, m1) == (0, M) and flags == L.DPI_BOTH:
        assert torch.equal(c.f32("y", n, F + C), c.f32("y1", n, F + C))


@pytest.mark.parametrize("kind,n,M", [("cha", 5, 192), ("gbm_sdgd", 3, 128), ("pis", 3, 64)])
def test_sample_with_gradients_writes_nothing_outside_its_buffers(kind, n, M):
    """dpi_sample_with_gradients (points + labels in one C-ABI call; tx is written too)."""
    gen = _gen(kind, M)
    F = 1 + NX
    c = Carved(ws=gen.workspace_bytes(n, M), tx=n * F * 4, mom=n * 2 * F * 4, y=n * F * 4)
    L.check(gen.lib.dpi_sample_with_gradients(gen.problem, gen.net.handle, n, M, gen.K, gen.seed, gen.epoch, 9, 0.01, 0,
                                              L.DPI_BOTH, float("inf"), c.ptr("tx"), c.ptr("y"), c.ptr("mom"),
                                              c.ptr("ws"), c.nbytes("ws"), _stream()), "sample_with_gradients")
    c.check()
    assert torch.isfinite(c.f32("y", n, F)).all()
