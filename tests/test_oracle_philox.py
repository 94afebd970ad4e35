"""Philox4x32-10 known-answer tests (Random123 kat_vectors; rocRAND engine cross-check)."""
import numpy as np

from oracle import philox as px


def _hex(ws):
    return [int(w) for w in ws]


def test_random123_kat():
    assert _hex(px.philox4x32_10(0, 0, 0, 0, 0)) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert _hex(px.philox4x32_10(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF)) == [
        0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert _hex(px.philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, (0x299F31D0 << 32) | 0xA4093822)) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_rocrand_engine_kat():
    # rocrand_device::philox4x32_10_engine(seed=0x123456789abcdef0, subsequence=5, offset=0).next4() x2,
    # host-compiled from /opt/rocm/include/rocrand/rocrand_philox4x32_10.h in this image.
    seed = 0x123456789ABCDEF0
    assert _hex(px.philox4x32_10(0, 0, 5, 0, seed)) == [0xAEAD3422, 0x70BBC61F, 0xC86A83D9, 0x27D55ADD]
    assert _hex(px.philox4x32_10(1, 0, 5, 0, seed)) == [0x72F03C2C, 0xFA2F013F, 0x91EBB87F, 0xD6219286]


def test_normals_moments_and_independence():
    z = px.normals(px.TAG_TERM, 0, 1, np.arange(4)[:, None], np.arange(2048)[None, :], 0, 100)
    assert z.shape == (4, 2048, 100)
    assert abs(z.mean()) < 5e-3 and abs(z.std() - 1) < 5e-3
    z2 = px.normals(px.TAG_INT, 0, 1, np.arange(4)[:, None], np.arange(2048)[None, :], 0, 100)
    assert abs(np.corrcoef(z.ravel(), z2.ravel())[0, 1]) < 5e-3


def test_uniform_ranges():
    w = np.array([0, 0xFF, 0xFFFFFFFF], dtype=np.uint32)
    assert px.uniform_co(w).tolist() == [0.0, 0.0, 1.0 - 2.0 ** -24]
    assert px.uniform_oc(w).tolist() == [2.0 ** -24, 2.0 ** -24, 1.0]


def test_randint_range():
    idx = px.randint_idx(px.TAG_SDGD, 0, 9, np.arange(8)[:, None], np.arange(64)[None, :], 100, 100)
    assert idx.shape == (8, 64, 100) and idx.min() >= 0 and idx.max() < 100
    assert len(np.unique(idx)) == 100
