"""TEST INFRASTRUCTURE ONLY — CPU oracle, never shipped, never on the product path.

Philox4x32-10 counter-based generator (Salmon et al., SC'11 / Random123), restated in
numpy uint64 arithmetic, plus the DPI noise contract shared with the HIP kernels
(`deeppicarditeration_amd/csrc/dpi_rng.h`, `include/dpi.h`).

The reference (`/root/reference/picard`) draws its noise from torch's unseeded global RNG
(`picard/equations.py:225` randn_like, `picard/data.py:166` rand, `picard/data.py:359`
rand_like, `picard/data.py:501` randint). It pins no generator, so the oracle fixes one:
Philox4x32-10 with the counter layout below, pinned against the Random123 / rocRAND
known-answer vectors (tests/test_oracle_philox.py) — rocRAND's host-compiled engine
(`/opt/rocm/include/rocrand/rocrand_philox4x32_10.h`) produced the same words here.

Counter layout (one Philox call = 4 uint32 words = 4 normals or 4 uniforms):
    c0 = k * NB + j      (EM step k, dim-block j = dims 4j..4j+3, NB = ceil(nx/4))
    c1 = m               (global Monte-Carlo index)
    c2 = i               (global point index = point_base + row)
    c3 = tag | epoch<<8  (stream tag, 24-bit epoch e.g. the Picard iteration)
    key = (seed & 0xffffffff, seed >> 32)
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)

# Stream tags (c3 low byte).  Must equal DPI_TAG_* in include/dpi.h.
TAG_T = 1      # t ~ U            (picard/data.py:166)
TAG_X0 = 2     # OU x0 ~ N(0,4I)  (picard/utils.py:785-789)
TAG_X = 3      # x | x0 normals   (picard/equations.py:225 via sample_x, :118-119)
TAG_TERM = 4   # terminal path    (picard/data.py:914 -> equations.py:225)
TAG_S = 5      # s ~ U[t,T]       (picard/data.py:359)
TAG_INT = 6    # integral path    (picard/data.py:360 -> equations.py:225)
TAG_SDGD = 7   # SDGD indices     (picard/data.py:501)
TAG_HTERM = 8  # Malliavin W1     (picard/data.py:1186)
TAG_HINT = 9   # Malliavin W2     (picard/data.py:870)

TWO_M24 = 1.0 / 16777216.0


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10. c* are broadcastable integer arrays (< 2**32)."""
    c0, c1, c2, c3 = np.broadcast_arrays(*(np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3)))
    c0, c1, c2, c3 = (c.copy() for c in (c0, c1, c2, c3))
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    for r in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def c3_word(tag, epoch):
    return (int(tag) & 0xFF) | ((int(epoch) & 0xFFFFFF) << 8)


def uniform_co(w):
    """[0,1) from the top 24 bits (exact in fp32)."""
    return (np.asarray(w, np.uint32) >> np.uint32(8)).astype(np.float64) * TWO_M24


def uniform_oc(w):
    """(0,1] from the top 24 bits (exact in fp32); avoids log(0) and s == t."""
    return ((np.asarray(w, np.uint32) >> np.uint32(8)).astype(np.float64) + 1.0) * TWO_M24


TWO_M23 = 1.0 / 8388608.0


def box_muller(wa, wb):
    """Two normals from two words (Box–Muller on 23-bit uniforms, csrc/dpi_rng.h):
    u1 = 1 - (wa & 0x7fffff) 2^-23 in (0,1], u2 = (wb & 0x7fffff) 2^-23 in [0,1);
    r = sqrt(-2 ln u1), (r cos 2pi u2, r sin 2pi u2)."""
    u1 = 1.0 - (np.asarray(wa, np.uint32) & np.uint32(0x7FFFFF)).astype(np.float64) * TWO_M23
    u2 = (np.asarray(wb, np.uint32) & np.uint32(0x7FFFFF)).astype(np.float64) * TWO_M23
    r = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * np.pi * u2
    return r * np.cos(ang), r * np.sin(ang)


def normals_block(words):
    """4 Philox words -> 4 normals, in dim order (4j, 4j+1, 4j+2, 4j+3)."""
    w0, w1, w2, w3 = words
    z0, z1 = box_muller(w0, w1)
    z2, z3 = box_muller(w2, w3)
    return np.stack([z0, z1, z2, z3], axis=-1)


def normals(tag, epoch, seed, i, m, k, nx):
    """Normals for points i, MC indices m, EM steps k (broadcast), all nx dims.

    Returns array of shape broadcast(i, m, k) + (nx,).
    """
    nb = (nx + 3) // 4
    i, m, k = np.broadcast_arrays(np.asarray(i, np.int64), np.asarray(m, np.int64), np.asarray(k, np.int64))
    j = np.arange(nb, dtype=np.int64)
    shp = i.shape
    c0 = k[..., None] * nb + j
    words = philox4x32_10(c0, m[..., None], i[..., None], c3_word(tag, epoch), seed)
    z = normals_block(words)  # shp + (nb, 4)
    return z.reshape(shp + (nb * 4,))[..., :nx]


def uniforms(tag, epoch, seed, i, m, open_low=False):
    """One uniform per (i, m) from word 0 of counter (0, m, i, c3)."""
    i, m = np.broadcast_arrays(np.asarray(i, np.int64), np.asarray(m, np.int64))
    w0, _, _, _ = philox4x32_10(0, m, i, c3_word(tag, epoch), seed)
    return uniform_oc(w0) if open_low else uniform_co(w0)


def uniforms_seq(tag, epoch, seed, i, m, R):
    """R uniforms [0, 1) per (i, m): word r&3 of counter (r>>2, m, i, c3); r = 0 is uniforms()."""
    i, m = np.broadcast_arrays(np.asarray(i, np.int64), np.asarray(m, np.int64))
    r = np.arange(R, dtype=np.int64)
    words = philox4x32_10(r >> 2, m[..., None], i[..., None], c3_word(tag, epoch), seed)
    w = np.stack(words, axis=-1)  # shape + (R, 4)
    return uniform_co(w[..., r, r & 3])


def randint_idx(tag, epoch, seed, i, m, v, high):
    """v indices in [0, high) per (i, m): word q&3 of counter (q>>2, m, i, c3), idx = (w*high)>>32."""
    i, m = np.broadcast_arrays(np.asarray(i, np.int64), np.asarray(m, np.int64))
    q = np.arange(v, dtype=np.int64)
    words = philox4x32_10(q >> 2, m[..., None], i[..., None], c3_word(tag, epoch), seed)
    w = np.stack(words, axis=-1)  # shape + (v, 4)
    sel = w[..., q, q & 3]
    return ((sel.astype(np.uint64) * np.uint64(high)) >> np.uint64(32)).astype(np.int64)
