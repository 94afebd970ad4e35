// Microbenchmark of the split-storage PISGradNet GEMM (dpi_gemm.h k_gemm_x3) and experimental
// variants, at the HJB pipeline's shape (R = 32768 paths, 512 x 512, fp16-split).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_gemm tools/ubench_gemm.hip
// Prints us / launch and effective TF/s (3 f16 MFMA products per fp32 product) per variant, and
// the max relative difference of each variant's output against the product kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../deeppicarditeration_amd/csrc/dpi_gemm.h"

using namespace dpi;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

// packed split of 8 values (pairs): hi = RNE fp16, lo = RNE fp16((x - hi) 2^11)
__device__ __forceinline__ void put8_pk(uint32_t* g, const f2v (&v)[4]) {
  u32x4_t h, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const h2v hi = __builtin_convertvector(v[p], h2v);
    const f2v hf = __builtin_convertvector(hi, f2v);
    const f2v r = (v[p] - hf) * 2048.0f;
    const h2v lo = __builtin_convertvector(r, h2v);
    h[p] = __builtin_bit_cast(uint32_t, hi);
    l[p] = __builtin_bit_cast(uint32_t, lo);
  }
  reinterpret_cast<u32x4_t*>(g)[0] = h;
  reinterpret_cast<u32x4_t*>(g)[1] = l;
}
__device__ __forceinline__ void get8_pk(const uint32_t* g, f2v (&v)[4]) {
  const u32x4_t h = reinterpret_cast<const u32x4_t*>(g)[0], l = reinterpret_cast<const u32x4_t*>(g)[1];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f2v hf = __builtin_convertvector(__builtin_bit_cast(h2v, h[p]), f2v);
    const f2v lf = __builtin_convertvector(__builtin_bit_cast(h2v, l[p]), f2v);
    v[p] = lf * (1.0f / 2048.0f) + hf;
  }
}
__device__ __forceinline__ f2v elu2(f2v z) {
  const f2v zl = z * 1.4426950408889634f;
  const f2v ex = {__builtin_amdgcn_exp2f(zl.x), __builtin_amdgcn_exp2f(zl.y)};
  const f2v em = ex - 1.0f;
  return f2v{z.x > 0.f ? z.x : em.x, z.y > 0.f ? z.y : em.y};
}

// granule swizzle of LDS row r (8 granules of 16 B): position = granule ^ swz(r).  VAR bit 2: the
// ds_read_b128 lane groups {0-3,12-15,20-27}, ... (MI355X_MICROARCH.md LDS table) mix rows il in
// {0..3, 12..15} with ql = q and rows {4..11} with ql = q ^ 1: flipping bit 1 of the swizzle on
// rows 4..11 (mod 16) makes each group's 16 reads hit 16 distinct 4-bank slots.
template <int VAR>
__device__ __forceinline__ int swz(int r) {
  if constexpr (VAR & 4)
    return ((r >> 1) & 7) ^ ((((r + 4) >> 3) & 1) << 1);
  else
    return (r >> 1) & 7;
}

// VAR bit 0: no epilogue (checksum only); bit 1: packed epilogue + bias-initialised accumulators
template <int EPI, int NT, int VAR>
__global__ __launch_bounds__(X3_THREADS, 1) void k_x3v(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                       const float* __restrict__ X, int ldx, float* __restrict__ OUT,
                                                       int ldc, const float* __restrict__ bias,
                                                       const float* __restrict__ AUX, int ldaux) {
  constexpr int BN = 32 * NT, BM = X3_BM, STAGE = (BN + BM) * 32, NWAVE = X3_THREADS / 64;
  constexpr int NINS = (BN + BM) / 8, PER_WAVE = NINS / NWAVE;
  __shared__ uint32_t sm[X3_STAGES * STAGE];
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = Kp >> 5;
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);
  auto issue = [&](int u) {
    uint32_t* dst = sm + (u % X3_STAGES) * STAGE;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int g = (lane & 7) ^ swz<VAR>(r);
      const uint32_t* src;
      if (r < BN)
        src = W + (size_t)(n0 + r) * Kp + 32 * u + 4 * g;
      else if constexpr (VAR & 8)  // L2-resident X (256 rows shared by every block)
        src = Xw + (size_t)((r - BN) & 255) * ldx + 32 * u + 4 * g;
      else
        src = Xw + (size_t)min(m0 + r - BN, M - 1) * ldx + 32 * u + 4 * g;
      if constexpr (VAR & 32) continue;  // no DMA
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = swz<VAR>(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  constexpr bool BI = (VAR & 2) && EPI != EPI_DELU;
  f4v hh[NT][4], xx[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f4v b0 = {0.f, 0.f, 0.f, 0.f};
    if (BI && bias) {  // tile t: n = n0 + 16 (wn NT + t) + 4 ql + r
      const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + 16 * (wn * NT + t) + 4 * ql);
      b0 = f4v{bb.x, bb.y, bb.z, bb.w};
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      hh[t][b] = b0;
      xx[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
    }
  }
  issue(0);
  if (nk > 1) issue(1);
  for (int u = 0; u < nk; ++u) {
    if (u + 1 < nk) {
      if constexpr (PER_WAVE == 6)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (u + 2 < nk) issue(u + 2);
    const uint32_t* buf = sm + (u % X3_STAGES) * STAGE;
    h8 ah[NT], al[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[t], al[t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      h8 bh, bl;
      frag(buf, BN + wm * 64 + 16 * b + il, bh, bl);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr (VAR & 16) {  // no MFMA: consume the fragments with one VALU op
          hh[t][b][0] += (float)(ah[t][0] + bh[0] + al[t][1] + bl[1]);
          continue;
        }
        hh[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[t], bh, hh[t][b], 0, 0, 0);
        xx[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[t], bl, xx[t][b], 0, 0, 0);
        xx[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[t], bh, xx[t][b], 0, 0, 0);
      }
    }
  }
  if constexpr (VAR & 1) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < 4; ++b) s += hh[t][b][0] + hh[t][b][1] + hh[t][b][2] + hh[t][b][3] + xx[t][b][0];
    OUT[(size_t)(m0 + tid % BM) * ldc + (n0 >> 5) * 32 + (tid / BM)] = s;
    return;
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wm * 64 + 16 * b + il;
    if (m >= M) continue;
    uint32_t* orow = reinterpret_cast<uint32_t*>(OUT + (size_t)m * ldc);
    const uint32_t* arow = reinterpret_cast<const uint32_t*>(AUX + (size_t)m * ldaux);
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      const int U = (n0 >> 5) + wn * (NT / 2) + c;
      if constexpr (VAR & 2) {
        f2v v[4];  // pairs (j = 2p, 2p + 1): j < 4 from tile 2c, j >= 4 from tile 2c + 1
        v[0] = f2v{xx[2 * c][b][0], xx[2 * c][b][1]} * (1.0f / 2048.0f) + f2v{hh[2 * c][b][0], hh[2 * c][b][1]};
        v[1] = f2v{xx[2 * c][b][2], xx[2 * c][b][3]} * (1.0f / 2048.0f) + f2v{hh[2 * c][b][2], hh[2 * c][b][3]};
        v[2] = f2v{xx[2 * c + 1][b][0], xx[2 * c + 1][b][1]} * (1.0f / 2048.0f) +
               f2v{hh[2 * c + 1][b][0], hh[2 * c + 1][b][1]};
        v[3] = f2v{xx[2 * c + 1][b][2], xx[2 * c + 1][b][3]} * (1.0f / 2048.0f) +
               f2v{hh[2 * c + 1][b][2], hh[2 * c + 1][b][3]};
        if constexpr (EPI == EPI_BIAS_ELU) {
#pragma unroll
          for (int p = 0; p < 4; ++p) v[p] = elu2(v[p]);
        } else if constexpr (EPI == EPI_DELU) {
          f2v a[4];
          get8_pk(arow + 32 * U + 8 * ql, a);
#pragma unroll
          for (int p = 0; p < 4; ++p) v[p] = v[p] * f2v{fminf(a[p].x, 0.f), fminf(a[p].y, 0.f)} + v[p];
        }
        put8_pk(orow + 32 * U + 8 * ql, v);
      } else {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = fmaf(xx[2 * c][b][r], 1.0f / 2048.0f, hh[2 * c][b][r]);
          v[4 + r] = fmaf(xx[2 * c + 1][b][r], 1.0f / 2048.0f, hh[2 * c + 1][b][r]);
        }
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
          if (bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
            const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 16 + 4 * ql);
            v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
            v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
          }
          if (EPI == EPI_BIAS_ELU)
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f;
        } else {
          float a[8];
          x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : a[j] + 1.0f;
        }
        x3_put8(OUT + (size_t)m * ldc, 0, U, ql, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// W2: split storage with UNSCALED lo (x = hi + lo, lo = fp16(x - hi)) and weights prescaled by 2^ws,
// so hi.hi + hi.lo + lo.hi accumulate into ONE accumulator (64 registers per wave instead of 128).
// The freed registers double-buffer the fragments: chunk u + 1's fragments are read from LDS
// during chunk u's MFMAs.  The slot of chunk u is refilled (DMA of chunk u + 3) as soon as every
// wave holds chunk u's fragments.  8 waves (2 per SIMD), block 256 m x 128 n, wave 64 m x 64 n.
__device__ __forceinline__ void put8_u(uint32_t* g, const float (&v)[8]) {
  u32x4_t h, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t hw = 0, lw = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float x = v[2 * p + e];
      const _Float16 hi = (_Float16)x;
      const _Float16 lo = (_Float16)(x - (float)hi);
      hw |= (uint32_t)__builtin_bit_cast(uint16_t, hi) << (16 * e);
      lw |= (uint32_t)__builtin_bit_cast(uint16_t, lo) << (16 * e);
    }
    h[p] = hw;
    l[p] = lw;
  }
  reinterpret_cast<u32x4_t*>(g)[0] = h;
  reinterpret_cast<u32x4_t*>(g)[1] = l;
}
__device__ __forceinline__ void get8_u(const uint32_t* g, float (&v)[8]) {
  const u32x4_t h = reinterpret_cast<const u32x4_t*>(g)[0], l = reinterpret_cast<const u32x4_t*>(g)[1];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t hw = h[j >> 1], lw = l[j >> 1];
    const _Float16 a = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? hw >> 16 : hw & 0xFFFFu));
    const _Float16 b = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? lw >> 16 : lw & 0xFFFFu));
    v[j] = (float)a + (float)b;
  }
}

template <int EPI, int VAR>
__global__ __launch_bounds__(X3_THREADS, 1) void k_x3u(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                       float wscale, const float* __restrict__ X, int ldx,
                                                       float* __restrict__ OUT, int ldc, const float* __restrict__ bias,
                                                       const float* __restrict__ AUX, int ldaux) {
  constexpr int NT = 4, BN = 32 * NT, BM = X3_BM, STAGE = (BN + BM) * 32, NWAVE = X3_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;  // 6
  __shared__ uint32_t sm[3 * STAGE];
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  uint64_t rt_entry = 0;
  if constexpr (VAR & 1024) rt_entry = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = Kp >> 5;
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);
  auto issue = [&](int u) {
    uint32_t* dst = sm + (u % 3) * STAGE;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int g = (lane & 7) ^ swz<4>(r);
      const uint32_t* src;
      if (r < BN)
        src = W + (size_t)(n0 + r) * Kp + 32 * u + 4 * g;
      else
        src = Xw + (size_t)min(m0 + r - BN, M - 1) * ldx + 32 * u + 4 * g;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = swz<4>(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + (u % 3) * STAGE;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(buf, BN + wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  issue(0);
  if (nk > 1) issue(1);
  if ((VAR & 128) || nk > 2) issue(min(2, nk - 1));
  if ((VAR & 128) || nk > 2)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (nk > 1)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  load(0, std::integral_constant<int, 0>{});
  uint64_t tw_lgkm = 0, tw_vm = 0, tw_bar = 0, tw_iss = 0, tw_mma = 0, tstart = 0;
  auto stamp = [&]() -> uint64_t {
    if constexpr (VAR & 64) return __builtin_readcyclecounter();
    return 0;
  };
  tstart = stamp();
  auto step = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    if (u + 1 < nk) {
      const uint64_t a0 = stamp();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of chunk u have landed
      const uint64_t a1 = stamp();
      if (u + 2 < nk)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // own DMA of chunk u + 1 landed
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t a2 = stamp();
      __builtin_amdgcn_s_barrier();  // chunk u + 1 published; slot u % 3 free
      const uint64_t a3 = stamp();
      if (u + 3 < nk) issue(u + 3);
      load(u + 1, std::integral_constant<int, F ^ 1>{});
      const uint64_t a4 = stamp();
      tw_lgkm += a1 - a0, tw_vm += a2 - a1, tw_bar += a3 - a2, tw_iss += a4 - a3;
    }
    const uint64_t b0 = stamp();
    mma(Fc);
    tw_mma += stamp() - b0;
  };
  uint64_t clk0 = 0, rt0 = 0;
  if constexpr (VAR & 1024) {  // in-kernel clock: s_memtime / s_memrealtime around the main loop
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (VAR & 128) {
    // branch-free steady state (nk even): the DMA of chunk min(u + 3, nk - 1) is issued every
    // iteration (the tail re-fetches the last chunk into free slots) so every wait is the same
    // vmcnt(6); fragment reads of chunk u + 1 interleave with chunk u's MFMAs (1 read : 3 MFMA).
    auto body = [&](int u, auto Fc) {
      constexpr int F = decltype(Fc)::value;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to the compiler's waitcnt model
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue(min(u + 3, nk - 1));
      load(u + 1, std::integral_constant<int, F ^ 1>{});
      mma(Fc);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
      }
    };
    for (int u = 0; u + 2 < nk; u += 2) {
      body(u, std::integral_constant<int, 0>{});
      body(u + 1, std::integral_constant<int, 1>{});
    }
    body(nk - 2, std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mma(std::integral_constant<int, 1>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int u = 0; u < nk; u += 2) {
      step(u, std::integral_constant<int, 0>{});
      if (u + 1 < nk) step(u + 1, std::integral_constant<int, 1>{});
    }
  }
  uint64_t clk1 = 0, rt1 = 0;
  if constexpr (VAR & 1024) {
    clk1 = __builtin_amdgcn_s_memtime();
    rt1 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (VAR & 64) {
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
    const uint64_t tend = stamp();
    if (lane == 0) {
      unsigned long long* st = reinterpret_cast<unsigned long long*>(const_cast<float*>(AUX)) + 8 * (blockIdx.x * 8 + wv);
      st[0] = tw_lgkm, st[1] = tw_vm, st[2] = tw_bar, st[3] = tw_iss, st[4] = tw_mma, st[5] = tend - tstart;
    }
  }
  if constexpr (VAR & 1) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < 4; ++b) s += acc[t][b][0] + acc[t][b][1] + acc[t][b][2] + acc[t][b][3];
    OUT[(size_t)(m0 + tid % BM) * ldc + (n0 >> 5) * 32 + (tid / BM)] = s;
    return;
  }
  const uint64_t e0 = stamp();
  if constexpr (VAR & 256) {  // epilogue stores only: raw accumulator bits, no VALU
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = m0 + wm * 64 + 16 * b + il;
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        u32x4_t* g = reinterpret_cast<u32x4_t*>(reinterpret_cast<uint32_t*>(OUT + (size_t)m * ldc) + 32 * U + 8 * ql);
        g[0] = __builtin_bit_cast(u32x4_t, acc[2 * c][b]);
        g[1] = __builtin_bit_cast(u32x4_t, acc[2 * c + 1][b]);
      }
    }
    return;
  }
  if constexpr (VAR & 4096) {  // packed epilogue (ELU): v_pk_fma scale+bias, v_pk_mul log2e, pairs split
    typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = m0 + wm * 64 + 16 * b + il;
      if (m >= M) continue;
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 16 + 4 * ql);
        const f2v bb[4] = {{b0.x, b0.y}, {b0.z, b0.w}, {b1.x, b1.y}, {b1.z, b1.w}};
        const f2v ws2 = {wscale, wscale};
        u32x4_t hv, lv;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const auto& a = acc[2 * c + (p >> 1)][b];
          const f2v x = {a[2 * (p & 1)], a[2 * (p & 1) + 1]};
          f2v v = x * ws2 + bb[p];
          const f2v tl = v * 1.4426950408889634f;
          const f2v em = f2v{__builtin_amdgcn_exp2f(tl.x), __builtin_amdgcn_exp2f(tl.y)} - 1.0f;
          v = f2v{v.x > 0.f ? v.x : em.x, v.y > 0.f ? v.y : em.y};
          const hh2 h = __builtin_convertvector(v, hh2);
          const hh2 l = __builtin_convertvector(v - __builtin_convertvector(h, f2v), hh2);
          hv[p] = __builtin_bit_cast(uint32_t, h);
          lv[p] = __builtin_bit_cast(uint32_t, l);
        }
        u32x4_t* g = reinterpret_cast<u32x4_t*>(reinterpret_cast<uint32_t*>(OUT + (size_t)m * ldc) + 32 * U + 8 * ql);
        g[0] = hv;
        g[1] = lv;
      }
    }
    return;
  }
  if constexpr (VAR & 512) {  // epilogue VALU only: full math, one store per thread
    float sink = 0.f;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * c][b][r] * wscale;
          v[4 + r] = acc[2 * c + 1][b][r] * wscale;
        }
        const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 16 + 4 * ql);
        v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
        v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f;
        u32x4_t h, l;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          uint32_t hw = 0, lw = 0;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float x = v[2 * p + e];
            const _Float16 hi = (_Float16)x;
            const _Float16 lo = (_Float16)(x - (float)hi);
            hw |= (uint32_t)__builtin_bit_cast(uint16_t, hi) << (16 * e);
            lw |= (uint32_t)__builtin_bit_cast(uint16_t, lo) << (16 * e);
          }
          h[p] = hw;
          l[p] = lw;
        }
        sink += __uint_as_float(h[0] ^ h[1] ^ h[2] ^ h[3] ^ l[0] ^ l[1] ^ l[2] ^ l[3]);
      }
    }
    OUT[(size_t)(m0 + tid % BM) * ldc + (n0 >> 5) * 32 + (tid / BM)] = sink;
    return;
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wm * 64 + 16 * b + il;
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      const int U = (n0 >> 5) + wn * (NT / 2) + c;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * c][b][r] * wscale;
        v[4 + r] = acc[2 * c + 1][b][r] * wscale;
      }
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
        if (bias) {
          const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
          const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 16 + 4 * ql);
          v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
          v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
        }
        if (EPI == EPI_BIAS_ELU)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f;
      } else {
        float a[8];
        get8_u(reinterpret_cast<const uint32_t*>(AUX + (size_t)m * ldaux) + 32 * U + 8 * ql, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : a[j] + 1.0f;
      }
      put8_u(reinterpret_cast<uint32_t*>(OUT + (size_t)m * ldc) + 32 * U + 8 * ql, v);
    }
  }
  if constexpr (VAR & 1024) {  // per-block timeline (wave 0): entry, loop start/end, epilogue end, hardware ids
    const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      unsigned long long* st = reinterpret_cast<unsigned long long*>(const_cast<float*>(AUX)) + 8 * blockIdx.x;
      st[0] = clk1 - clk0;
      st[1] = rt1 - rt0;
      st[2] = rt_entry, st[3] = rt0, st[4] = rt1, st[5] = rt_end;
      st[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      st[7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    }
  }
}

__global__ void k_convert_u(const float* in, float* out, int rows, int Kp, int ld, float scale) {
  // old split (lo scaled 2^11) -> unscaled-lo split of scale * x
  const int m = blockIdx.x;
  if (m >= rows) return;
  for (int idx = threadIdx.x; idx < (Kp / 32) * 4; idx += blockDim.x) {
    const int u = idx >> 2, q = idx & 3;
    float v[8];
    x3_get8(in + (size_t)m * ld, 0, u, q, v);
    for (int j = 0; j < 8; ++j) v[j] *= scale;
    put8_u(reinterpret_cast<uint32_t*>(out + (size_t)m * ld) + 32 * u + 8 * q, v);
  }
}

// Measured negative result (kept for the record): the persistent form below is bitwise equal to
// k_gemm_x3 but slower (262,144 rows: 575-605 vs 460-510 us; 32,768 rows: 84 vs 63 us) - the
// tile-boundary stall it removes was not where the non-loop time goes, and its epilogue spills.
namespace dpi {
// Persistent form of k_gemm_x3: gridDim.x (a multiple of 8, at most one block per CU) blocks walk
// the tiles v = blockIdx.x + j gridDim.x (the same XCD-aware remap of v), and the LDS ring and the
// fragment double buffer run across tile boundaries: the next tile's first chunks are in flight
// while this tile's last chunks multiply and its epilogue stores, so no tile pays the prologue's
// memory latency or waits for a block slot.  Same products in the same order as k_gemm_x3 (bitwise
// equal outputs).  Requires nk = Kp / 32 even.
template <int EPI, int NT>
__global__ __launch_bounds__(X3_THREADS, 1) void k_gemm_x3p(int M, int Kp, int n_ntiles, int n_tiles,
                                                            const uint32_t* __restrict__ W, float wscale,
                                                            const float* __restrict__ X, int ldx,
                                                            float* __restrict__ OUT, int ldc,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ AUX, int ldaux) {
  static_assert(NT == 2 || NT == 4, "wave n-tiles");
  constexpr int BN = 32 * NT, BM = X3_BM, STAGE = (BN + BM) * 32, NWAVE = X3_THREADS / 64;
  constexpr int NINS = (BN + BM) / 8, PER_WAVE = NINS / NWAVE;
  static_assert(NINS % NWAVE == 0 && (PER_WAVE == 6 || PER_WAVE == 5), "DMA split / vmcnt immediates");
  __shared__ uint32_t sm[X3_STAGES * STAGE];
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int G = gridDim.x, bid = blockIdx.x;
  if (bid >= n_tiles) return;  // block-uniform
  const int my_tiles = (n_tiles - 1 - bid) / G + 1;
  const int nk = Kp >> 5, total = my_tiles * nk;
  const int q8 = n_tiles >> 3, r8 = n_tiles & 7;
  auto tile_of = [&](int j) {
    const int v = bid + j * G, xcd = v & 7, loc = v >> 3;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  };
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);

  auto issue = [&](int g, int slot) {  // global chunk g = j nk + c of this block's tile sequence
    const int j = g / nk, c = g - j * nk, t = tile_of(j);
    const int mt = t / n_ntiles, m0 = mt * BM, n0 = (t - mt * n_ntiles) * BN;
    uint32_t* dst = sm + slot * STAGE;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int gr = (lane & 7) ^ x3_swz(r);
      const uint32_t* src;
      if (r < BN)
        src = W + (size_t)(n0 + r) * Kp + 32 * c + 4 * gr;
      else
        src = Xw + (size_t)min(m0 + r - BN, M - 1) * ldx + 32 * c + 4 * gr;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  auto vm_wait = [&]() {
    if constexpr (PER_WAVE == 6)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  };
  f4v acc[NT][4];
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * STAGE;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(buf, BN + wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  auto body = [&](int g, auto Fc) {  // g + 1 < total
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    vm_wait();
    __builtin_amdgcn_s_barrier();
    issue(min(g + 3, total - 1), g % X3_STAGES);
    load((g + 1) % X3_STAGES, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
#pragma unroll
    for (int i = 0; i < 2 * (NT + 4); ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * NT * 4 / (2 * (NT + 4)), 0);
    }
  };
  issue(0, 0);
  issue(min(1, total - 1), 1);
  issue(min(2, total - 1), 2);
  if constexpr (PER_WAVE == 6)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  load(0, std::integral_constant<int, 0>{});
  int g = 0;
  for (int j = 0; j < my_tiles; ++j) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
    const bool last = j + 1 == my_tiles;
    const int gend = g + nk - 2;  // the tile's last pair starts here
    for (; g < gend; g += 2) {
      body(g, std::integral_constant<int, 0>{});
      body(g + 1, std::integral_constant<int, 1>{});
    }
    body(g, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (!last) {  // chunk g + 1 without reading chunk g + 2 yet: the epilogue runs with one fragment set dead
      vm_wait();
      __builtin_amdgcn_s_barrier();
      issue(min(g + 4, total - 1), (g + 1) % X3_STAGES);
      mma(std::integral_constant<int, 1>{});
    } else {
      mma(std::integral_constant<int, 1>{});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int t = tile_of(j);
    const int mt = t / n_ntiles, m0 = mt * BM, n0 = (t - mt * n_ntiles) * BN;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = m0 + wm * 64 + 16 * b + il;
      if (m >= M) continue;
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * c][b][r] * wscale;
          v[4 + r] = acc[2 * c + 1][b][r] * wscale;
        }
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
          if (bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
            const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 16 + 4 * ql);
            v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
            v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
          }
          if (EPI == EPI_BIAS_ELU)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] = v[jj] > 0.f ? v[jj] : __expf(v[jj]) - 1.0f;
        } else {
          float a[8];
          x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) v[jj] *= a[jj] > 0.f ? 1.0f : a[jj] + 1.0f;
        }
        x3_put8(OUT + (size_t)m * ldc, 0, U, ql, v);
      }
    }
    if (!last) load((g + 2) % X3_STAGES, std::integral_constant<int, 0>{});  // the next tile's first chunk
    g += 2;
  }
}

}  // namespace dpi

// in-kernel clock of the main loop (MI355X_MICROARCH.md DVFS item 6): the stamped variant runs
// back to back for ~2 s, then the last launch's per-block (memtime, realtime) deltas give the clock
// and the loop's cycles; MFMA share = 16 cycles x MFMAs per SIMD / loop cycles.
template <int EPI, int VAR>
void clock_u(const char* name, int M, int Kp, int Np, const uint32_t* W, float ws, const float* X, float* OUT,
             const float* bias, float* STAMP) {
  const int nnt = Np / 128, nmt = (M + X3_BM - 1) / X3_BM;
  dim3 grid(nnt * nmt), block(X3_THREADS);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int iters = 0;
  float ms = 0.f;
  CK(hipEventRecord(e0));
  while (ms < 2000.f) {
    for (int i = 0; i < 64; ++i)
      hipLaunchKernelGGL((k_x3u<EPI, VAR>), grid, block, 0, 0, M, Kp, nnt, W, ws, X, Kp, OUT, Np, bias, STAMP, Np);
    iters += 64;
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  std::vector<unsigned long long> st(8 * grid.x);
  CK(hipMemcpy(st.data(), STAMP, st.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> clk, cyc, pro, loop, epi, tot, gap;
  std::vector<std::tuple<unsigned long long, unsigned long long, unsigned long long, unsigned>> ev;
  for (unsigned b = 0; b < grid.x; ++b) {
    const unsigned long long* q = &st[8 * b];
    clk.push_back((double)q[0] / (double)q[1] * 100.0);  // MHz
    cyc.push_back((double)q[0]);
    pro.push_back((q[3] - q[2]) * 10.0), loop.push_back((q[4] - q[3]) * 10.0), epi.push_back((q[5] - q[4]) * 10.0);
    tot.push_back((q[5] - q[2]) * 10.0);  // ns (100 MHz realtime)
    const unsigned long long hw = q[6];
    const unsigned long long cu = (q[7] << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
    ev.emplace_back(cu, q[2], q[5], b);
  }
  std::sort(ev.begin(), ev.end());
  for (size_t i = 1; i < ev.size(); ++i)
    if (std::get<0>(ev[i]) == std::get<0>(ev[i - 1]))
      gap.push_back(((double)std::get<1>(ev[i]) - (double)std::get<2>(ev[i - 1])) * 10.0);
  for (auto* v : {&clk, &cyc, &pro, &loop, &epi, &tot, &gap}) std::sort(v->begin(), v->end());
  auto med = [](const std::vector<double>& v) { return v.empty() ? 0.0 : v[v.size() / 2]; };
  std::printf("  per block (median, ns): prologue %.0f  loop %.0f  epilogue %.0f  entry->end %.0f  same-CU gap %.0f "
              "(%zu gaps)\n", med(pro), med(loop), med(epi), med(tot), med(gap), gap.size());
  const double mfma_cyc = 16.0 * 3.0 * 4.0 * 4.0 * (Kp / 32) * 2.0;  // per SIMD: 2 waves x nk x 48 MFMAs x 16
  std::printf("%-34s %8.2f us/launch  clock %.0f MHz (median over blocks)  loop %.0f cycles  MFMA share %.2f\n",
              name, ms * 1e3f / iters, clk[clk.size() / 2], cyc[cyc.size() / 2], mfma_cyc / cyc[cyc.size() / 2]);
}

template <int EPI, int VAR>
void report_u(const char* name, int M, int Kp, int Np, const uint32_t* W, float ws, const float* X, float* OUT,
              float* REF, const float* bias, const float* AUX) {
  const int nnt = Np / 128, nmt = (M + X3_BM - 1) / X3_BM;
  dim3 grid(nnt * nmt), block(X3_THREADS);
  hipLaunchKernelGGL((k_x3u<EPI, VAR>), grid, block, 0, 0, M, Kp, nnt, W, ws, X, Kp, OUT, Np, bias, AUX, Np);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((k_x3u<EPI, VAR>), grid, block, 0, 0, M, Kp, nnt, W, ws, X, Kp, OUT, Np, bias, AUX, Np);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const float us = ms * 1e3f / iters;
  const double tf = 2.0 * 3.0 * M * (double)Kp * Np / (us * 1e-6) / 1e12;
  double maxrel = 0.0, maxref = 0.0;
  if (!(VAR & 1)) {
    std::vector<float> a((size_t)M * Np), b((size_t)M * Np);
    CK(hipMemcpy(a.data(), OUT, a.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), REF, b.size() * 4, hipMemcpyDeviceToHost));
    for (size_t r = 0; r < (size_t)M; r += 61)
      for (int c = 0; c < Np; ++c) {
        const int u = c >> 5, w = c & 31, q = (w >> 2) & 3, j = (w & 3) + 4 * (w >> 4);
        auto dec = [&](const std::vector<float>& v, double lsc) {
          const uint32_t* row = reinterpret_cast<const uint32_t*>(v.data() + r * Np);
          const uint32_t hw = row[32 * u + 8 * q + (j >> 1)], lw = row[32 * u + 8 * q + 4 + (j >> 1)];
          const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? hw >> 16 : hw & 0xFFFF));
          const _Float16 l = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? lw >> 16 : lw & 0xFFFF));
          return (double)(float)h + (double)(float)l * lsc;
        };
        const double x = dec(a, 1.0), y = dec(b, 1.0);
        maxrel = std::fmax(maxrel, std::fabs(x - y));
        maxref = std::fmax(maxref, std::fabs(y));
      }
  }
  std::printf("%-34s M=%6d K=%4d N=%4d  %8.2f us  %7.1f TF/s(eff f16)  max|diff| %.2e of max|ref| %.2e\n", name, M,
              Kp, Np, us, tf, maxrel, maxref);
}

__global__ void k_fill(float* rows, int M, int Kp, int ld, uint32_t seed, float scale) {
  // split-fill rows[m][0:Kp] with pseudo-random values in (-scale, scale)
  const int m = blockIdx.x, tid = threadIdx.x;
  if (m >= M) return;
  for (int idx = tid; idx < (Kp / 32) * 4; idx += blockDim.x) {
    const int u = idx >> 2, q = idx & 3;
    float v[8];
    for (int j = 0; j < 8; ++j) {
      uint32_t h = (uint32_t)m * 2654435761u ^ (uint32_t)(idx * 8 + j) * 2246822519u ^ seed;
      h ^= h >> 15;
      h *= 2654435761u;
      h ^= h >> 13;
      v[j] = scale * ((float)(h >> 8) * (1.0f / 8388608.0f) - 1.0f);
    }
    x3_put8(rows + (size_t)m * ld, 0, u, q, v);
  }
}

template <int EPI, int NT, int VAR>
float run(int M, int Kp, int Np, const uint32_t* W, const float* X, float* OUT, const float* bias, const float* AUX,
          int iters) {
  const int nnt = Np / (32 * NT), nmt = (M + X3_BM - 1) / X3_BM;
  dim3 grid(nnt * nmt), block(X3_THREADS);
  hipLaunchKernelGGL((k_x3v<EPI, NT, VAR>), grid, block, 0, 0, M, Kp, nnt, W, X, Kp, OUT, Np, bias, AUX, Np);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((k_x3v<EPI, NT, VAR>), grid, block, 0, 0, M, Kp, nnt, W, X, Kp, OUT, Np, bias, AUX, Np);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

template <int EPI, int NT, int VAR>
void report(const char* name, int M, int Kp, int Np, const uint32_t* W, const float* X, float* OUT, float* REF,
            const float* bias, const float* AUX) {
  const float us = run<EPI, NT, VAR>(M, Kp, Np, W, X, OUT, bias, AUX, 50);
  const double tf = 2.0 * 3.0 * M * (double)Kp * Np / (us * 1e-6) / 1e12;
  double maxrel = 0.0;
  if (!(VAR & 1)) {
    std::vector<float> a((size_t)M * Np), b((size_t)M * Np);
    CK(hipMemcpy(a.data(), OUT, a.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), REF, b.size() * 4, hipMemcpyDeviceToHost));
    // compare decoded values: treat each word pair as split storage via the host decode
    for (size_t r = 0; r < (size_t)M; r += 97)
      for (int c = 0; c < Np; ++c) {
        auto dec = [&](const std::vector<float>& v) {
          const uint32_t* row = reinterpret_cast<const uint32_t*>(v.data() + r * Np);
          const int u = c >> 5, w = c & 31, q = (w >> 2) & 3, j = (w & 3) + 4 * (w >> 4);
          const uint32_t hw = row[32 * u + 8 * q + (j >> 1)], lw = row[32 * u + 8 * q + 4 + (j >> 1)];
          const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? hw >> 16 : hw & 0xFFFF));
          const _Float16 l = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? lw >> 16 : lw & 0xFFFF));
          return (double)(float)h + (double)(float)l / 2048.0;
        };
        const double x = dec(a), y = dec(b);
        maxrel = std::fmax(maxrel, std::fabs(x - y) / (std::fabs(y) + 1e-3));
      }
  }
  std::printf("%-34s M=%6d K=%4d N=%4d  %8.2f us  %7.1f TF/s(eff f16)  maxrel vs product %.2e\n", name, M, Kp, Np, us,
              tf, maxrel);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 32768, Kp = 512, Np = 512;
  uint32_t* W;
  float *X, *OUT, *REF, *AUX, *bias;
  CK(hipMalloc(&W, (size_t)Np * Kp * 4));
  CK(hipMalloc(&X, (size_t)M * Kp * 4));
  CK(hipMalloc(&AUX, (size_t)M * Np * 4));
  CK(hipMalloc(&OUT, (size_t)M * Np * 4));
  CK(hipMalloc(&REF, (size_t)M * Np * 4));
  CK(hipMalloc(&bias, Np * 4));
  float* STAMP;
  CK(hipMalloc(&STAMP, (size_t)(M / X3_BM + 1) * (Np / 128) * 64));
  hipLaunchKernelGGL(k_fill, dim3(Np), dim3(128), 0, 0, reinterpret_cast<float*>(W), Np, Kp, Kp, 7u, 0.05f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, X, M, Kp, Kp, 11u, 1.0f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, AUX, M, Np, Np, 13u, 1.5f);
  uint32_t* WU;
  float *XU, *AUXU;
  CK(hipMalloc(&WU, (size_t)Np * Kp * 4));
  CK(hipMalloc(&XU, (size_t)M * Kp * 4));
  CK(hipMalloc(&AUXU, (size_t)M * Np * 4));
  hipLaunchKernelGGL(k_convert_u, dim3(Np), dim3(128), 0, 0, reinterpret_cast<float*>(W), reinterpret_cast<float*>(WU),
                     Np, Kp, Kp, 16.0f);
  hipLaunchKernelGGL(k_convert_u, dim3(M), dim3(128), 0, 0, X, XU, M, Kp, Kp, 1.0f);
  hipLaunchKernelGGL(k_convert_u, dim3(M), dim3(128), 0, 0, AUX, AUXU, M, Np, Np, 1.0f);
  std::vector<float> hb(Np);
  for (int i = 0; i < Np; ++i) hb[i] = 0.01f * (float)((i * 37) % 17 - 8);
  CK(hipMemcpy(bias, hb.data(), Np * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  // reference outputs: the product kernel (dpi_gemm.h, unscaled-lo split, weights prescaled 2^4)
  const int nnt = Np / 128, nmt = M / X3_BM;
  auto prod = [&](int epi, int iters, float* dst = nullptr) {
    if (!dst) dst = REF;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) {
      if (epi == 1)
        hipLaunchKernelGGL((k_gemm_x3<EPI_BIAS_ELU, 4>), dim3(nnt * nmt), dim3(X3_THREADS), 0, 0, M, Kp, nnt, WU,
                           1.0f / 16.0f, XU, Kp, XU, Kp, Kp / 32, dst, Np, bias, AUXU, Np);
      else
        hipLaunchKernelGGL((k_gemm_x3<EPI_DELU, 4>), dim3(nnt * nmt), dim3(X3_THREADS), 0, 0, M, Kp, nnt, WU,
                           1.0f / 16.0f, XU, Kp, XU, Kp, Kp / 32, dst, Np, nullptr, AUXU, Np);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / iters;
  };
  auto prodp = [&](int epi, int iters, float* dst) {
    const int nt = nnt * nmt, G = std::min(nt, 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) {
      if (epi == 1)
        hipLaunchKernelGGL((k_gemm_x3p<EPI_BIAS_ELU, 4>), dim3(G), dim3(X3_THREADS), 0, 0, M, Kp, nnt, nt, WU,
                           1.0f / 16.0f, XU, Kp, dst, Np, bias, AUXU, Np);
      else
        hipLaunchKernelGGL((k_gemm_x3p<EPI_DELU, 4>), dim3(G), dim3(X3_THREADS), 0, 0, M, Kp, nnt, nt, WU,
                           1.0f / 16.0f, XU, Kp, dst, Np, nullptr, AUXU, Np);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / iters;
  };
  auto cmp = [&](const char* name, float us) {
    std::vector<float> a((size_t)M * Np), b((size_t)M * Np);
    CK(hipMemcpy(a.data(), OUT, a.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), REF, b.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i) bad += (std::memcmp(&a[i], &b[i], 4) != 0);
    std::printf("%s %8.2f us  %7.1f TF/s(eff f16)  words differing from k_gemm_x3: %zu\n", name, us,
                2.0 * 3.0 * M * (double)Kp * Np / (us * 1e-6) / 1e12, bad);
  };
  for (int epi = 1; epi <= 2; ++epi) {
    prod(epi, 1, REF);
    CK(hipMemset(OUT, 0, (size_t)M * Np * 4));
    prodp(epi, 1, OUT);
    CK(hipDeviceSynchronize());
    cmp(epi == 1 ? "elu  persistent k_gemm_x3p (-> OUT)" : "delu persistent k_gemm_x3p (-> OUT)", prodp(epi, 50, OUT));
    std::printf("%s product k_gemm_x3 (-> OUT)       %8.2f us\n", epi == 1 ? "elu " : "delu", prod(epi, 50, OUT));
    std::printf("%s persistent again (-> OUT)        %8.2f us\n", epi == 1 ? "elu " : "delu", prodp(epi, 50, OUT));
  }
  for (int epi = 1; epi <= 2; ++epi) {
    prod(epi, 1);
    const float us = prod(epi, 50);
    std::printf("%s product k_gemm_x3               %8.2f us  %7.1f TF/s(eff f16)\n", epi == 1 ? "elu " : "delu", us,
                2.0 * 3.0 * M * (double)Kp * Np / (us * 1e-6) / 1e12);
    prod(epi, 1);  // REF = product output
    if (epi == 1) {
      report<EPI_BIAS_ELU, 4, 1>("elu  v1 (old loop, no epilogue)", M, Kp, Np, W, X, OUT, REF, bias, AUX);
      report_u<EPI_BIAS_ELU, 128>("elu  W3 (ubench copy)", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF, bias, AUXU);
      report_u<EPI_BIAS_ELU, 129>("elu  W3 no epilogue", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF, bias, AUXU);
      report_u<EPI_BIAS_ELU, 128 + 4096>("elu  W3 packed epilogue", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF, bias,
                                         AUXU);
      report_u<EPI_BIAS_ELU, 128>("elu  W3 (again)", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF, bias, AUXU);
      report_u<EPI_BIAS_ELU, 128 + 4096>("elu  W3 packed epilogue (again)", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF,
                                         bias, AUXU);
      clock_u<EPI_BIAS_ELU, 128 + 1024>("elu  W3 + clock stamps", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, bias, STAMP);
      report_u<EPI_BIAS_ELU, 128 + 256>("elu  W3 epilogue = stores only", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF,
                                        bias, AUXU);
      report_u<EPI_BIAS_ELU, 128 + 512>("elu  W3 epilogue = VALU only", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF,
                                        bias, AUXU);
    } else {
      report_u<EPI_DELU, 128>("delu W3 (ubench copy)", M, Kp, Np, WU, 1.0f / 16.0f, XU, OUT, REF, nullptr, AUXU);
    }
    const float us2 = prod(epi, 50);
    std::printf("%s product k_gemm_x3 (again)       %8.2f us\n", epi == 1 ? "elu " : "delu", us2);
    const float us3 = prod(epi, 50, OUT);
    std::printf("%s product k_gemm_x3 (-> OUT)      %8.2f us\n", epi == 1 ? "elu " : "delu", us3);
  }
  std::printf("done\n");
  return 0;
}
