// Counter-based noise for the DPI label path (gfx950).
//
// Philox4x32-10 (Salmon et al. SC'11; the generator behind rocRAND/cuRAND philox) with the
// DPI counter contract of include/dpi.h:
//     c0 = k*NB + j   (EM step k, dim-block j = dims 4j..4j+3, NB = ceil(nx/4))
//     c1 = m          (global Monte-Carlo index)
//     c2 = i          (global point index)
//     c3 = tag | epoch << 8
//     key = seed (lo, hi)
// Every lane of a wave shares (k, j, i, tag) while it works on one dim-block, so round 1's two
// products and one product each of rounds 2 and 3 are wave-uniform and land on the scalar unit
// (philox4x32_10_wu, below); the rest is one v_mad_u64_u32 per product.
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

// The same generator for a wave whose counter words c0, c2, c3 (and key) are wave-uniform and only
// c1 = m differs per lane — every rollout loop of the label path.  Which words stay uniform, round by
// round (p0 = M0 c0, p1 = M1 c2; c0' = hi p1 ^ c1 ^ k0, c1' = lo p1, c2' = hi p0 ^ c3 ^ k1, c3' = lo p0):
//   round 1: p0, p1 uniform           -> c0' per lane; c1', c2', c3' uniform
//   round 2: p1 uniform, p0 per lane  -> c0', c1' uniform; c2', c3' per lane
//   round 3: p0 uniform, p1 per lane  -> c3' uniform; the rest per lane, and from round 4 on all.
// readfirstlane pins the uniform words to SGPRs, so their products (s_mul_hi_u32 / s_mul_i32) and
// XORs run on the scalar unit: 16 v_mad_u64_u32 and 18 VALU XORs per call instead of 18 and 19 —
// left to itself the compiler moved only one product and turned two others into v_mul_hi_u32 +
// v_mul_lo_u32 pairs.  Bitwise the words of philox4x32_10.
__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ u32x4 philox4x32_10_wu(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                   uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  c0 = wave_uniform(c0), c2 = wave_uniform(c2), c3 = wave_uniform(c3);
  k0 = wave_uniform(k0), k1 = wave_uniform(k1);
  // round 1
  uint32_t a0 = c1 ^ wave_uniform(__umulhi(M1, c2) ^ k0);  // per lane
  uint32_t a1 = M1 * c2;                                   // uniform
  uint32_t a2 = wave_uniform(__umulhi(M0, c0) ^ c3 ^ k1);  // uniform
  uint32_t a3 = M0 * c0;                                   // uniform
  k0 += W0, k1 += W1;
  // round 2
  const uint64_t q0 = (uint64_t)M0 * a0;                   // per lane
  c0 = wave_uniform(__umulhi(M1, a2) ^ a1 ^ k0);           // uniform
  c1 = M1 * a2;                                            // uniform
  c2 = (uint32_t)(q0 >> 32) ^ wave_uniform(a3 ^ k1);       // per lane
  c3 = (uint32_t)q0;                                       // per lane
  k0 += W0, k1 += W1;
  // round 3
  const uint64_t q1 = (uint64_t)M1 * c2;                   // per lane
  a0 = (uint32_t)(q1 >> 32) ^ wave_uniform(c1 ^ k0);
  a1 = (uint32_t)q1;
  a2 = c3 ^ wave_uniform(__umulhi(M0, c0) ^ k1);
  a3 = M0 * c0;                                            // uniform
  k0 += W0, k1 += W1;
  c0 = a0, c1 = a1, c2 = a2, c3 = a3;
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c0;
    const uint64_t p1 = (uint64_t)M1 * c2;
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += W0;
    k1 += W1;
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

// Sum of a dim-block's K raw normal quadruples (the K-step Euler-Maruyama rollout of one 4-dim block;
// counter word c0 = k nb + j), in k order.  philox4x32_10_wu's readfirstlane makes the loop body
// convergent, which the compiler will not unroll by a runtime trip count: the loop is unrolled by
// hand, UNR independent Philox chains per iteration and a remainder loop, summing in the same order.
// WU = false: the plain philox4x32_10 (for kernels whose register budget the scalar form's extra live
// values would overflow: the wide nx <= 256 instances, the GBM TD kernel, the shared PIS rollout wave).
template <int UNR, bool WU = true>
__device__ __forceinline__ void noise_sums(int K, int nb, int j, uint32_t m, uint32_t ig, uint32_t c3, uint32_t k0,
                                           uint32_t k1, float& s0, float& s1, float& s2, float& s3) {
  if constexpr (WU) {
    auto step = [&](int k) {
      const f4 z = normals4_raw(philox4x32_10_wu((uint32_t)(k * nb + j), m, ig, c3, k0, k1));
      s0 += z.a;
      s1 += z.b;
      s2 += z.c;
      s3 += z.d;
    };
    int k = 0;
    for (; k + UNR <= K; k += UNR) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) step(k + u);
    }
    for (; k < K; ++k) step(k);
  } else {  // the compiler's own unroll (the round-5 loop)
#pragma unroll UNR
    for (int k = 0; k < K; ++k) {
      const f4 z = normals4_raw(philox4x32_10((uint32_t)(k * nb + j), m, ig, c3, k0, k1));
      s0 += z.a;
      s1 += z.b;
      s2 += z.c;
      s3 += z.d;
    }
  }
}

}  // namespace dpi
