"""Register / scratch gate on the built library's gfx950 code objects (amdhsa.kernels metadata; no GPU).

Counted `s_waitcnt vmcnt(N)` waits (dpi_gemm.h's LDS-DMA rings) are exact only while the compiler
adds no vector-memory instruction of its own between the counted ones — and a VGPR spill is
exactly that (scratch accesses count as vector memory).  So every kernel must come out with no VGPR
spill and no private (scratch) segment, and the co-residency plans need their register ceilings:

| kernel | ceiling | why |
|---|---|---|
| k_pis_net | 232 (VGPR + AGPR) | two waves per SIMD leave 48 registers for a one-wave k_pis_rollout_shared block of the next batch |
| k_pis_rollout_shared | 48 | that rollout wave (2 x 232 + 48 = 512, a SIMD's register file) |
| k_pis_rollout | 64 | the full-occupancy rollout (eight waves per SIMD) |
| k_gemm_x3h | 224 | two 4-wave blocks per CU plus a rollout wave (the layer-wise chain) |
| k_paths (first-order, 256-thread blocks) | 256 | two workgroups per CU |

No exception: the exact-fp32 OU 4x128 MLP instance that spilled 4 VGPRs through round 5 runs at one
workgroup per CU (dpi_device.h k_paths_wgs) instead.
"""
import pytest

from deeppicarditeration_amd.build import build, kernel_resources

ALLOWED_SPILL = set()

CEILINGS = {"dpi::k_pis_net<": 232, "dpi::k_pis_rollout_shared<": 48, "dpi::k_pis_rollout<": 64,
            "dpi::k_gemm_x3h<": 224}


@pytest.fixture(scope="module")
def kernels():
    return kernel_resources(build(verbose=False))


def test_every_kernel_is_found(kernels):
    names = [k["name"] for k in kernels]
    for fam in ("dpi::k_pis_net<", "dpi::k_pis_rollout<", "dpi::k_gemm_x3h<", "dpi::k_gemm_x3<", "dpi::k_paths<",
                "dpi::k_paths_fb<", "dpi::k_reduce", "dpi::k_baseline<", "dpi::k_baseline_gbm<"):
        assert any(fam in n for n in names), fam


def test_no_vgpr_spill_and_no_scratch(kernels):
    bad = [(k["name"], k["vgpr_spill_count"], k["private_segment_fixed_size"]) for k in kernels
           if (k["vgpr_spill_count"] or k["private_segment_fixed_size"]) and k["name"] not in ALLOWED_SPILL]
    assert not bad, bad


def test_no_dynamic_stack(kernels):
    assert all(k.get("uses_dynamic_stack") == "false" for k in kernels)


def test_register_ceilings(kernels):
    over = [(k["name"], k["vgpr_count"], cap) for k in kernels for fam, cap in CEILINGS.items()
            if fam in k["name"] and k["vgpr_count"] > cap]
    assert not over, over


def test_rollout_wave_fits_beside_k_pis_net(kernels):
    """The co-residency the prepare schedule relies on: on one SIMD, two k_pis_net waves (one
    512-thread block per CU) and one shared-rollout wave, in 8-register allocation granules."""
    g = lambda r: (r + 7) // 8 * 8  # noqa: E731
    net = max(k["vgpr_count"] for k in kernels if "dpi::k_pis_net<" in k["name"])
    roll = max(k["vgpr_count"] for k in kernels if "dpi::k_pis_rollout_shared<" in k["name"])
    assert 2 * g(net) + g(roll) <= 512, (net, roll)


def test_counted_wait_kernels_spill_nothing(kernels):
    """The kernels whose source holds counted vmcnt immediates (dpi_gemm.h) — checked by name so a
    future allow-list entry cannot cover them."""
    for k in kernels:
        if "dpi::k_gemm_x3" in k["name"]:
            assert k["vgpr_spill_count"] == 0 and k["private_segment_fixed_size"] == 0, k["name"]
