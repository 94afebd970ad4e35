// Batched-path GEMM for networks too wide to keep on chip (PISGradNet, 4 x 512):
//     C[m][n] (ldc) = epi( sum_k A[m][k] (lda) * B[n][k] (ldb) )          (both operands K-contiguous)
// m runs over Monte-Carlo paths (hundreds of thousands), n over output units, k over inputs.
// v_mfma_f32_16x16x4_f32 (exact fp32), 128 x 128 workgroup tile, 4 waves as 2 x 2 with 64 x 64 per
// wave (4 x 4 MFMA tiles, 64 accumulator registers), BK = 16 staged through double-buffered LDS
// in k-major layout ([k][m], row stride 144 floats: the two 16-lane k-rows of a fragment read hit
// disjoint bank halves).  Global loads of step s+1 are issued before the MFMAs of step s.
// Epilogues fuse what the layer needs: +bias, ELU, or x elu'(saved activation) for the backward.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace dpi {

enum GemmEpi : int { EPI_BIAS = 0, EPI_BIAS_ELU = 1, EPI_DELU = 2 };

constexpr int GBM_ = 128, GBN_ = 128, GBK_ = 16, GLD_ = 144;

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(int M, int N, int K, const float* __restrict__ A, int lda,
                                                    const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                    int ldc, const float* __restrict__ bias,
                                                    const float* __restrict__ aux, int ldaux) {
  __shared__ float As[2][GBK_ * GLD_];
  __shared__ float Bs[2][GBK_ * GLD_];
  typedef float floatx4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * GBM_, n0 = blockIdx.y * GBN_;
  const int il = lane & 15, ql = lane >> 4;
  // staging map: 2 float4 of A and of B per thread per k-step
  const int srow = tid >> 2, sk = (tid & 3) * 4;
  float4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = srow + 64 * h;
      const int gm = m0 + r, gn = n0 + r, gk = k0 + sk;
      float4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
      if (gm < M) {  // lda, ldb, ldc and the k offsets are multiples of 4 floats; bases 16-B aligned
        const float* p = A + (size_t)gm * lda + gk;
        if (gk + 3 < K) {
          va = *reinterpret_cast<const float4*>(p);
        } else {
          if (gk < K) va.x = p[0];
          if (gk + 1 < K) va.y = p[1];
          if (gk + 2 < K) va.z = p[2];
        }
      }
      if (gn < N) {
        const float* p = B + (size_t)gn * ldb + gk;
        if (gk + 3 < K) {
          vb = *reinterpret_cast<const float4*>(p);
        } else {
          if (gk < K) vb.x = p[0];
          if (gk + 1 < K) vb.y = p[1];
          if (gk + 2 < K) vb.z = p[2];
        }
      }
      ra[h] = va;
      rb[h] = vb;
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = srow + 64 * h;
      float* a = As[buf] + sk * GLD_ + r;
      a[0] = ra[h].x;
      a[GLD_] = ra[h].y;
      a[2 * GLD_] = ra[h].z;
      a[3 * GLD_] = ra[h].w;
      float* b = Bs[buf] + sk * GLD_ + r;
      b[0] = rb[h].x;
      b[GLD_] = rb[h].y;
      b[2 * GLD_] = rb[h].z;
      b[3 * GLD_] = rb[h].w;
    }
  };
  floatx4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + GBK_ - 1) / GBK_;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload((ks + 1) * GBK_);
#pragma unroll
    for (int kk = 0; kk < GBK_; kk += 4) {
      float fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        fa[t] = As[cur][(kk + ql) * GLD_ + wm * 64 + t * 16 + il];
        fb[t] = Bs[cur][(kk + ql) * GLD_ + wn * 64 + t * 16 + il];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    if (ks + 1 < nk) {
      lstore(cur ^ 1);
      __syncthreads();
    }
  }
  // epilogue: acc[a][b] lane (ql, il) holds C[m = tile a row 4ql + r][n = tile b col il]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int n = n0 + wn * 64 + b * 16 + il;
      if (n >= N) continue;
      const float bn = (EPI == EPI_DELU || bias == nullptr) ? 0.f : bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + a * 16 + 4 * ql + r;
        if (m >= M) continue;
        float v = acc[a][b][r];
        if (EPI == EPI_BIAS) {
          v += bn;
        } else if (EPI == EPI_BIAS_ELU) {
          v += bn;
          v = v > 0.f ? v : __expf(v) - 1.0f;
        } else {
          const float s = aux[(size_t)m * ldaux + n];
          v *= s > 0.f ? 1.0f : s + 1.0f;
        }
        C[(size_t)m * ldc + n] = v;
      }
    }
}

}  // namespace dpi

namespace dpi {

// ---------------------------------------------------------------------------------------------
// Split-storage GEMM (the PISGradNet pipeline's default): every operand and result lives in HBM
// already split, x = hi + lo with hi = fp16(x), lo = fp16(x - hi) (lo unscaled), in the fragment
// order of mlp_tile_split — per row, chunk u of 32 logical columns is 4 granule pairs (q = 0..3)
// of 8 hi then 8 lo halves holding columns 32u + 4q + (j & 3) + 16 (j >> 2).  That order is what
// a lane of group q holds in the 16x16 C layout of n-tiles 2u, 2u+1, so the epilogue stores whole
// 32-B granule pairs and the next GEMM reads them as MFMA operands with no conversion.  The main
// loop is LDS-DMA + ds_read_b128 + v_mfma_f32_16x16x32_f16, three products hi hi + hi lo + lo hi
// accumulated into ONE fp32 accumulator (lo unscaled; relative error ~2^-22 where the residual is
// an fp16 normal).  The weights are stored prescaled by a power of two 2^s (host, per matrix:
// max |2^s W| in [0.5, 1)) so their residuals stay in fp16's normal range; the epilogue multiplies
// by wscale = 2^-s (exact).  The activations and cotangents are stored prescaled too, by a power
// of two 2^e per operand and network (dpi_kernels.hip x3_exponent: rms ~4, so their residuals stay
// normal whatever the network's scale): wscale also carries the input's 2^-e (and, for EPI_DELU,
// the output's 2^e), EPI_BIAS_ELU multiplies its output by oscale = 2^e, and EPI_DELU reads the
// saved activation as a 2^-e = ascale.
//     OUT[m][n] = epi( wscale sum_k W'[n][k] X[m][k] ),  m = path (M rows), n = unit (Np, % 32), k (Kp, % 32)
// W': (Np, Kp) packed split (Kp words per row); X rows at X + m ldx (Kp words); OUT / AUX rows at
// + m ldc / + m ldaux (Np words).  MFMA A = W tile (rows n), B = X tile (columns m).
// Block: BM = 256 paths x BN = 32 NT units, 8 waves as 4 (m) x 2 (n), wave tile 64 m x 16 NT n
// (16 NT accumulator registers).  LDS: a ring of 3 slots of (BN + BM) rows x 128 B (one 32-deep
// chunk); granule g of row r sits at g ^ swz(r), chosen for the ds_read_b128 lane groups.
// Pipeline (branch-free steady state): at iteration u every wave holds chunk u's fragments in
// registers; it retires its own reads (lgkmcnt) and its LDS-DMA of chunk u + 1 (counted vmcnt),
// a raw s_barrier publishes chunk u + 1 and frees chunk u's slot, the DMA of chunk u + 3 (clamped
// to the last chunk) goes into that slot, and the fragment reads of chunk u + 1 interleave with
// chunk u's MFMAs (1 ds_read : 3 MFMA).  Never __syncthreads(): its vmcnt(0) would drain the ring.
// 144 KB (NT = 4): 1 block / CU, 2 waves per SIMD.  Blocks are mapped XCD-aware: the n-tiles of
// one m-tile run back to back on one XCD, so the X tile is fetched from HBM once.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float x3_join(uint32_t hw, uint32_t lw, int half) {
  const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)(half ? hw >> 16 : hw & 0xFFFFu));
  const _Float16 l = __builtin_bit_cast(_Float16, (uint16_t)(half ? lw >> 16 : lw & 0xFFFFu));
  return (float)h + (float)l;
}
// value of logical column c of a split region starting at word `reg` of a row
__device__ __forceinline__ float x3_get(const float* row, int reg, int c) {
  const int u = c >> 5, w = c & 31, q = (w >> 2) & 3, j = (w & 3) + 4 * (w >> 4);
  const uint32_t* g = reinterpret_cast<const uint32_t*>(row + reg) + 32 * u + 8 * q;
  return x3_join(g[j >> 1], g[4 + (j >> 1)], j & 1);
}
// the 8 values of granule pair (u, q): v[j] = column 32u + 4q + (j & 3) + 16 (j >> 2)
__device__ __forceinline__ void x3_get8(const float* row, int reg, int u, int q, float (&v)[8]) {
  const u32x4_t* g = reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint32_t*>(row + reg) + 32 * u + 8 * q);
  const u32x4_t h = g[0], l = g[1];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = x3_join(h[j >> 1], l[j >> 1], j & 1);
}
__device__ __forceinline__ void x3_put8(float* row, int reg, int u, int q, const float (&v)[8]) {
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
  u32x4_t* g = reinterpret_cast<u32x4_t*>(reinterpret_cast<uint32_t*>(row + reg) + 32 * u + 8 * q);
  g[0] = h;
  g[1] = l;
}

// LDS granule swizzle of ring row r (8 granules of 16 B per 128-B row): granule g sits at
// g ^ x3_swz(r).  ds_read_b128 serves a wave in the lane groups {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31}, {32-35, 44-47, 52-59}, {36-43, 48-51, 60-63} (MI355X_MICROARCH.md, LDS):
// each group mixes fragment rows il in {0..3, 12..15} of lane group q with rows {4..11} of group
// q ^ 1.  (r >> 1) & 7 spreads a group's 8 rows of one parity over 8 slots; flipping bit 1 on rows
// 4..11 (mod 16) separates the two halves, so the 16 reads of every group hit 16 distinct 4-bank
// slots.  Fragment rows are 16-aligned plus il, so the pattern holds for every tile.
__device__ __forceinline__ int x3_swz(int r) { return ((r >> 1) & 7) ^ ((((r + 4) >> 3) & 1) << 1); }

constexpr int X3_BM = 256, X3_STAGES = 3, X3_THREADS = 512;

// Two-source K: chunks c >= nk1 of the X operand come from X2 (chunk c - nk1, row stride ldx2), so
// [X | X2] . W^T runs as one GEMM (nk1 = Kp / 32 for a single source).
// VAR (schedule experiments, tools/ubench_x3.hip; 0 = product): bit 0 s_setprio 1 for waves 4-7,
// bit 1 fragment reads front-loaded into the first 2/3 of the MFMAs, bit 2 the DMA issue interleaved
// with the first MFMAs.
// XCD-aware bijective remap (dispatch puts block b on XCD b % 8): the n-tiles of one m-tile run
// back to back on one XCD
// The nwg % 8 blocks past 8 (nwg / 8) — dispatched last — take the LAST tiles, i.e. the chunk's
// partial m-tile (its n-tiles are the launch's final round, cheap with dead waves skipped), instead
// of giving XCDs 0..r8-1 one full tile more than the others.
__device__ __forceinline__ int x3_tile_of_block() {
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3;
  return loc < q8 ? xcd * q8 + loc : 8 * q8 + xcd;
}

template <int NT>
struct X3Lds {
  static constexpr int BN = 32 * NT, STAGE = (BN + X3_BM) * 32;
  uint32_t sm[X3_STAGES * STAGE + BN];  // the ring, then the block's n-tile of the bias
};

// One 256 x BN output tile (rows m0.., units n0..) of the split GEMM, the whole K loop and the
// epilogue; `sm` is the block's LDS ring (free on entry, free again on return).
template <int EPI, int NT, int VAR>
__device__ __forceinline__ void x3_tile(uint32_t* __restrict__ sm, int m0, int n0, int M, int Kp,
                                        const uint32_t* __restrict__ W, float wscale, const float* __restrict__ X,
                                        int ldx, const float* __restrict__ X2, int ldx2, int nk1,
                                        float* __restrict__ OUT, int ldc, const float* __restrict__ bias,
                                        const float* __restrict__ AUX, int ldaux, float oscale, float ascale,
                                        int stage_aux = 1) {
  static_assert(NT == 2 || NT == 4, "wave n-tiles");
  constexpr int BN = 32 * NT, BM = X3_BM, STAGE = (BN + BM) * 32, NWAVE = X3_THREADS / 64;
  constexpr int NINS = (BN + BM) / 8, PER_WAVE = NINS / NWAVE;  // DMA wave-instructions per chunk
  static_assert(NINS % NWAVE == 0 && (PER_WAVE == 6 || PER_WAVE == 5), "DMA split / vmcnt immediates");
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);
  const uint32_t* X2w = reinterpret_cast<const uint32_t*>(X2);

  // LDS-DMA of chunk c into ring slot `slot`: wave-instruction w fills rows 8w..8w+7 (128 B each)
  // lane-linearly; lane i fetches the granule that belongs at position i & 7 of its row.
  auto issue = [&](int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;  // wave-uniform source select
    const uint32_t* xb = one ? Xw + 32 * c : X2w + 32 * (c - nk1);
    const int ld = one ? ldx : ldx2;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int g = (lane & 7) ^ x3_swz(r);
      const uint32_t* src;
      if (r < BN)
        src = W + (size_t)(n0 + r) * Kp + 32 * c + 4 * g;
      else
        src = xb + (size_t)min(m0 + r - BN, M - 1) * ld + 4 * g;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  };
  // DELU epilogue operand staging (NT = 4, nk >= 3): the two DMA slots that the last two load
  // steps would refill with clamped duplicates of the last chunk take this tile's saved activations
  // instead — per wave its 64 rows x 2 output chunks (256 B per row), rows 0-23 in the slot freed at
  // step nk - 3 and rows 24-47 in the slot freed at step nk - 2 (6 DMA instructions per wave each, as
  // many as the duplicates they replace, so every counted wait stays exact); rows 48-63 go straight
  // to registers after the last MFMAs and land while rows 0-47 are processed.  Row rho's 16 granules
  // sit at position g ^ (rho & 15): the epilogue's ds_read_b128 lane groups hit 16 distinct slots.
  constexpr bool AUXC = EPI == EPI_DELU && NT == 4 && PER_WAVE == 6;
  const bool aux_lds = AUXC && nk >= 3 && stage_aux;
  auto issue_aux = [&](int part, int slot) {
    uint32_t* dst = sm + slot * STAGE + wv * 1536;
    const int U0 = (n0 >> 5) + wn * 2;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      int rho = 24 * part + 4 * k + (lane >> 4);
      asm volatile("" : "+v"(rho));  // computed here, not hoisted out of the K loop
      const int gs = (lane & 15) ^ (rho & 15);
      const int mrow = min(m0 + wm * 64 + rho, M - 1);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(AUX) + (size_t)mrow * ldaux + 32 * U0 + 4 * gs;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * k), 16, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  auto vm_wait = [&]() {  // all but this wave's youngest chunk of DMA retired
    if constexpr (PER_WAVE == 6)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  };

  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];  // fragments, double-buffered across chunks
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
  // iteration u (u + 1 < nk): chunk u in register set F, chunk u + 1 -> set F ^ 1
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): chunk u's reads landed (visible to the compiler)
    vm_wait();                           // own DMA of chunk u + 1 landed
    __builtin_amdgcn_s_barrier();        // chunk u + 1 published; chunk u's slot free
    if (AUXC && aux_lds && u + 3 >= nk)
      issue_aux(u + 3 - nk, u % X3_STAGES);
    else
      issue(min(u + 3, nk - 1), u % X3_STAGES);
    load((u + 1) % X3_STAGES, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;  // ds_reads and MFMAs per chunk
    if constexpr (VAR & 4) {  // the DMA wave-instructions between the first MFMAs
#pragma unroll
      for (int i = 0; i < PER_WAVE; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM read (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
    if constexpr (VAR & 2) {  // all reads within the first 2/3 of the MFMAs, then the rest of the MFMAs
#pragma unroll
      for (int i = 0; i < NRD; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, (2 * NMF / 3 - ((VAR & 4) ? PER_WAVE : 0)) / NRD, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NRD; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
        __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);  // then MFMAs
      }
    }
  };
  if constexpr (VAR & 1)
    if (wv >= 4) __builtin_amdgcn_s_setprio(1);
  // above any co-resident wave of another kernel (the prepare stream's rollout): the
  // GEMM's issue comes first, the VALU-bound rollout takes the cycles the GEMM leaves
  if constexpr (!(VAR & 1)) __builtin_amdgcn_s_setprio(2);
  // the bias of the block's n-tile goes to LDS with the prologue (older than every DMA, so the
  // chunk-0 wait covers it): the epilogue then reads it without a global round trip
  // (VAR bit 3: the epilogue's global bias loads instead — the ablation of tools/ubench_x3.hip)
  constexpr bool LDS_BIAS = !(VAR & 8);
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + X3_STAGES * STAGE);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (LDS_BIAS && has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  // prologue: chunks 0, 1, 2 (clamped) in flight; publish chunk 0 and read it
  issue(0, 0);
  issue(min(1, nk - 1), 1);
  issue(min(2, nk - 1), 2);
  if constexpr (PER_WAVE == 6)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  if (LDS_BIAS && has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {
    // every row of this wave lies past M (the chunk's partial last m-tile): no MFMAs, fragment reads
    // or stores — its share of each chunk's DMA (the same instructions the live waves' loop issues,
    // so the staged epilogue regions stay intact) and the same barriers, then done; the wave's SIMD
    // partner runs its MFMAs alone
    for (int u = 0; u + 1 < nk; ++u) {
      vm_wait();
      __builtin_amdgcn_s_barrier();
      if (AUXC && aux_lds && u + 3 >= nk)
        issue_aux(u + 3 - nk, u % X3_STAGES);
      else
        issue(min(u + 3, nk - 1), u % X3_STAGES);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {  // nk even: one more load step, the last chunk lands in set 1
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {  // nk odd: the last chunk is in set 0
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  u32x4_t a3h[2], a3l[2];  // staged DELU epilogue: saved activations of rows 48-63
  if (AUXC && aux_lds) {
    asm volatile("" ::: "memory");  // these loads stay after the staging DMAs
    const int mrow = min(m0 + wm * 64 + 48 + il, M - 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const u32x4_t* g = reinterpret_cast<const u32x4_t*>(reinterpret_cast<const uint32_t*>(AUX) + (size_t)mrow * ldaux +
                                                        32 * ((n0 >> 5) + wn * 2 + c) + 8 * ql);
      a3h[c] = g[0];
      a3l[c] = g[1];
    }
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this wave's staged rows 0-47 landed
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail DMAs land before the slot memory is released
  }

  // epilogue: lane (il, ql) of m-tile b holds OUT[m = m0 + 64 wm + 16 b + il][n = 16 T + 4 ql + r]
  // for the wave's n-tiles T; tiles (2c, 2c+1) form granule pair ql of output chunk U.
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wm * 64 + 16 * b + il;
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      const int U = (n0 >> 5) + wn * (NT / 2) + c;
      float v[8];
      // scale and bias as explicit FMAs (no contraction left to the compiler), so k_pis_net's
      // epilogue reproduces these outputs bit for bit
      float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if ((EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && has_bias) {
        const int o = 32 * (wn * (NT / 2) + c) + 4 * ql;  // = 32 U + 4 ql - n0
        const float* bsrc = LDS_BIAS ? sbias + o : bias + 32 * U + 4 * ql;
        const float4 b0 = *reinterpret_cast<const float4*>(bsrc);
        const float4 b1 = *reinterpret_cast<const float4*>(bsrc + 16);
        bb[0] = b0.x, bb[1] = b0.y, bb[2] = b0.z, bb[3] = b0.w;
        bb[4] = b1.x, bb[5] = b1.y, bb[6] = b1.z, bb[7] = b1.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = __builtin_fmaf(acc[2 * c][b][r], wscale, bb[r]);
        v[4 + r] = __builtin_fmaf(acc[2 * c + 1][b][r], wscale, bb[4 + r]);
      }
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
        if (EPI == EPI_BIAS_ELU)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f) * oscale;
      } else {
        float a[8];
        if (AUXC && aux_lds) {
          u32x4_t h, l;
          if (b < 3) {  // staged in LDS: row rho of part rho / 24
            const int rho = 16 * b + il, part = rho >= 24 ? 1 : 0;
            const uint32_t* rb = sm + ((nk - 3 + part) % X3_STAGES) * STAGE + wv * 1536 + 64 * (rho - 24 * part);
            const int gh = 8 * c + 2 * ql;
            h = *reinterpret_cast<const u32x4_t*>(rb + 4 * (gh ^ (rho & 15)));
            l = *reinterpret_cast<const u32x4_t*>(rb + 4 * ((gh + 1) ^ (rho & 15)));
          } else {
            h = a3h[c];
            l = a3l[c];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = x3_join(h[j >> 1], l[j >> 1], j & 1);
        } else {
          x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : fmaf(a[j], ascale, 1.0f);
      }
      x3_put8(OUT + (size_t)m * ldc, 0, U, ql, v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_gemm_x3h: the same split GEMM on a 128 x 128 block tile with 4 waves (64 x 64 each, the product's
// wave tile) and a 2-slot ring of 32 KB chunks, so two blocks share a CU (2 x 64.5 KB of LDS, one wave
// per SIMD each) and one block's prologue and epilogue run under the other's main loop, at 4/3 the
// L2 -> LDS bytes per MFMA of the 256 x 128 tile.  Per output the same products in the same order:
// bitwise equal to k_gemm_x3.  (tools/ubench_x3.hip "half" mode.)
constexpr int X3H_BM = 128, X3H_THREADS = 256;
struct X3HLds {
  static constexpr int BN = 128, STAGE = (BN + X3H_BM) * 32;
  uint32_t sm[2 * STAGE + BN];
};

template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3h(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux, float oscale,
                                                             float ascale) {
  constexpr int NT = 4, BN = 128, BM = X3H_BM, STAGE = X3HLds::STAGE, NWAVE = X3H_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;  // 8 DMA wave-instructions per chunk
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ X3HLds lds;
  uint32_t* sm = lds.sm;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  // LDS-DMA in buffer form (r03f): the wave id made provably uniform, so each DMA's LDS destination
  // is scalar (m0 from SALU alone), and each lane's row offset fixed in a VGPR with the chunk's
  // column offset in soffset — no per-DMA VALU address arithmetic or readfirstlane.  Bitwise equal;
  // 567-573 -> 528-536 us (ELU), 600-609 -> 579-592 us (DELU) at 262,144 x 512 x 512
  // (profiles/r03f_ubench_x3hb.txt).  The resources start at the block's own tiles (W rows n0..,
  // X rows m0..), so the 32-bit offsets stay small whatever the row stride of the activation
  // workspace (thousands of words: the whole chain's row) or M.
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int mrows = min(BM, M - m0);  // >= 1: the grid holds only tiles with rows
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(W + (size_t)n0 * Kp, (size_t)BN * Kp * 4);
  const __amdgpu_buffer_rsrc_t rx = tile_rsrc(X + (size_t)m0 * ldx, (size_t)mrows * ldx * 4);
  const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc(X2 + (size_t)m0 * ldx2, (size_t)mrows * ldx2 * 4);
  // wave-instruction k fills rows 8w..8w+7, w = 4k + wave: k < 4 the W tile, k >= 4 the X tile
  int vw[PER_WAVE / 2], vx[PER_WAVE / 2], vx2[PER_WAVE / 2];
#pragma unroll
  for (int k = 0; k < PER_WAVE; ++k) {
    const int w = k * NWAVE + wv;
    const int r = 8 * w + (lane >> 3);
    const int g = (lane & 7) ^ x3_swz(r);
    if (k < PER_WAVE / 2) {
      vw[k] = r * Kp * 4 + 16 * g;
    } else {
      const int xr = min(r - BN, mrows - 1);  // rows past M load the last row
      vx[k - PER_WAVE / 2] = xr * ldx * 4 + 16 * g;
      vx2[k - PER_WAVE / 2] = xr * ldx2 * 4 + 16 * g;
    }
  }
  auto issue = [&](int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;  // two-source K as in x3_tile
    const int sx = one ? 128 * c : 128 * (c - nk1);
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      __attribute__((address_space(3))) void* d =
          (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (k < PER_WAVE / 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, d, 16, vw[k], 128 * c, 0, 0);
      else if (one)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx[k - PER_WAVE / 2], sx, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx2, d, 16, vx2[k - PER_WAVE / 2], sx, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
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
  // iteration u (u + 1 < nk): chunk u in set F; the DMA of chunk u + 1 (issued one iteration ago) is
  // this wave's only outstanding one; chunk u + 2 goes into chunk u's slot
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + 2 < nk) issue(u + 2, u & 1);
    load((u + 1) & 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + 2 * STAGE);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  __builtin_amdgcn_s_setprio(2);
  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {  // rows past M: DMA share and barriers only
    for (int u = 0; u + 1 < nk; ++u) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (u + 2 < nk) issue(u + 2, u & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wm * 64 + 16 * b + il;
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      const int U = (n0 >> 5) + wn * (NT / 2) + c;
      float v[8];
      // scale and bias as explicit FMAs (as x3_tile)
      float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if ((EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && has_bias) {
        const float* bsrc = sbias + 32 * (wn * (NT / 2) + c) + 4 * ql;
        const float4 b0 = *reinterpret_cast<const float4*>(bsrc);
        const float4 b1 = *reinterpret_cast<const float4*>(bsrc + 16);
        bb[0] = b0.x, bb[1] = b0.y, bb[2] = b0.z, bb[3] = b0.w;
        bb[4] = b1.x, bb[5] = b1.y, bb[6] = b1.z, bb[7] = b1.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = __builtin_fmaf(acc[2 * c][b][r], wscale, bb[r]);
        v[4 + r] = __builtin_fmaf(acc[2 * c + 1][b][r], wscale, bb[4 + r]);
      }
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
        if (EPI == EPI_BIAS_ELU)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f) * oscale;
      } else {
        float a[8];
        x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : fmaf(a[j], ascale, 1.0f);
      }
      x3_put8(OUT + (size_t)m * ldc, 0, U, ql, v);
    }
  }
}

template <int EPI, int NT, int VAR = 0>
__global__ __launch_bounds__(X3_THREADS, 1) void k_gemm_x3(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                           float wscale, const float* __restrict__ X, int ldx,
                                                           const float* __restrict__ X2, int ldx2, int nk1,
                                                           float* __restrict__ OUT, int ldc,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ AUX, int ldaux, float oscale,
                                                           float ascale, int stage_aux) {
  __shared__ X3Lds<NT> lds;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  x3_tile<EPI, NT, VAR>(lds.sm, mt * X3_BM, nt * 32 * NT, M, Kp, W, wscale, X, ldx, X2, ldx2, nk1, OUT, ldc, bias, AUX,
                        ldaux, oscale, ascale, stage_aux);
}



}  // namespace dpi
