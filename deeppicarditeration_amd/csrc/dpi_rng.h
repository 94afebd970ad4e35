// Counter-based noise for the DPI label path (gfx950).
//
// Philox4x32-10 (Salmon et al. SC'11; the generator behind rocRAND/cuRAND philox) with the
// DPI counter contract of include/dpi.h:
//     c0 = k*NB + j   (EM step k, dim-block j = dims 4j..4j+3, NB = ceil(nx/4))
//     c1 = m          (global Monte-Carlo index)
//     c2 = i          (global point index)
//     c3 = tag | epoch << 8
//     key = seed (lo, hi)
// Every lane of a wave shares (k, j, i, tag) while it works on one dim-block, so the first
// round's two products and half of the second round's are wave-uniform and land on the
// scalar unit; the rest is one v_mad_u64_u32 per product.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpi {

struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;  // one v_mad_u64_u32 (quarter rate) each
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    // 3-input XOR in one v_bitop3_b32 (CDNA4; truth table 0x96) — gfx950 has no v_xor3_b32
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// [0,1) and (0,1] from the top 24 bits: exact in fp32, identical to oracle/philox.py.
__device__ __forceinline__ float u01_co(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float u01_oc(uint32_t w) { return (float)((w >> 8) + 1u) * (1.0f / 16777216.0f); }

// Box–Muller normals.  The 23 low bits of a word become the mantissa of a float in [1,2)
// with one v_and_or_b32:  u1 = 2 - F(wa) = 1 - (wa & 0x7fffff) 2^-23 in (0,1],
// F(wb) = 1 + (wb & 0x7fffff) 2^-23.
// v_log_f32 is log2 and v_sin/v_cos take revolutions (sin 2pi(1+u) = sin 2pi u), so
//     z0 = BM_SCALE * sqrt(-log2 u1) * cos(2pi u2),   z1 = ... * sin(2pi u2),
// BM_SCALE = sqrt(2 ln 2).  box_muller_raw() omits BM_SCALE: the K-step rollout sums raw
// normals and applies the constant once per dimension.
constexpr float BM_SCALE = 1.1774100225154747f;  // sqrt(2 ln 2)

__device__ __forceinline__ float mant_1_2(uint32_t w) {
  return __uint_as_float((w & 0x007FFFFFu) | 0x3F800000u);  // v_and_or_b32
}

__device__ __forceinline__ void box_muller_raw(uint32_t wa, uint32_t wb, float& z0, float& z1) {
  const float u1 = 2.0f - mant_1_2(wa);
  const float rev = mant_1_2(wb);
  const float r = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(rev);
  z1 = r * __builtin_amdgcn_sinf(rev);
}

struct f4 {
  float a, b, c, d;
};

__device__ __forceinline__ f4 normals4_raw(u32x4 w) {
  f4 z;
  box_muller_raw(w.x, w.y, z.a, z.b);
  box_muller_raw(w.z, w.w, z.c, z.d);
  return z;
}

__device__ __forceinline__ f4 normals4(u32x4 w) {
  f4 z = normals4_raw(w);
  z.a *= BM_SCALE;
  z.b *= BM_SCALE;
  z.c *= BM_SCALE;
  z.d *= BM_SCALE;
  return z;
}

}  // namespace dpi
