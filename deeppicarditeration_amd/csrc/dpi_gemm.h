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
// fp16-split variant: x = hi + 2^-11 lo with hi = fp16(x), lo = fp16((x - hi) 2^11), so
//     x y = hi_x hi_y + 2^-11 (hi_x lo_y + lo_x hi_y) + O(2^-22 |x y|)
// — three v_mfma_f32_16x16x32_f16 (16 cycles each, K = 32) replace eight v_mfma_f32_16x16x4_f32
// (32 cycles, K = 4): 5.3x fewer matrix-pipe cycles at ~2.4e-7 relative error per product, fp32
// accumulation.  Operands are split once while staging global -> LDS into [row][k] fp16 images
// (row stride 40 halves) so each MFMA fragment is one ds_read_b128.  Valid while |x| < 65504.
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));

constexpr int HBK_ = 32, HLD_ = 40;  // K per stage, LDS row stride in halves

__device__ __forceinline__ void split4(float4 v, half4_t& hi, half4_t& lo) {
  const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 h = (_Float16)x[e];
    hi[e] = h;
    lo[e] = (_Float16)((x[e] - (float)h) * 2048.0f);
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void k_gemm_nt_f16x3(int M, int N, int K, const float* __restrict__ A, int lda,
                                                          const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                          int ldc, const float* __restrict__ bias,
                                                          const float* __restrict__ aux, int ldaux) {
  __shared__ _Float16 sm[2][4][GBM_ * HLD_];  // [buf][A hi, A lo, B hi, B lo][row][k]
  typedef float floatx4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * GBM_, n0 = blockIdx.y * GBN_;
  const int il = lane & 15, ql = lane >> 4;
  // staging: 128 rows x 32 k = 1024 float4 per operand -> 4 per thread; thread covers k4 = tid & 7
  const int sk = (tid & 7) * 4, srow = tid >> 3;  // rows srow + 32 h, h = 0..3
  float4 ra[4], rb[4];
  auto ld4 = [&](const float* base, int ld, int rows_total, int r, int gk) {
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < rows_total) {
      const float* p = base + (size_t)r * ld + gk;
      if (gk + 3 < K) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        if (gk < K) v.x = p[0];
        if (gk + 1 < K) v.y = p[1];
        if (gk + 2 < K) v.z = p[2];
      }
    }
    return v;
  };
  auto gload = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      ra[h] = ld4(A, lda, M, m0 + srow + 32 * h, k0 + sk);
      rb[h] = ld4(B, ldb, N, n0 + srow + 32 * h, k0 + sk);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int off = (srow + 32 * h) * HLD_ + sk;
      half4_t hi, lo;
      split4(ra[h], hi, lo);
      *reinterpret_cast<half4_t*>(&sm[buf][0][off]) = hi;
      *reinterpret_cast<half4_t*>(&sm[buf][1][off]) = lo;
      split4(rb[h], hi, lo);
      *reinterpret_cast<half4_t*>(&sm[buf][2][off]) = hi;
      *reinterpret_cast<half4_t*>(&sm[buf][3][off]) = lo;
    }
  };
  floatx4_t hh[4][4], xx[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) hh[a][b] = xx[a][b] = floatx4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + HBK_ - 1) / HBK_;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload((ks + 1) * HBK_);
    half8_t ah[4], al[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int off = (wm * 64 + a * 16 + il) * HLD_ + 8 * ql;
      ah[a] = *reinterpret_cast<const half8_t*>(&sm[cur][0][off]);
      al[a] = *reinterpret_cast<const half8_t*>(&sm[cur][1][off]);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int off = (wn * 64 + b * 16 + il) * HLD_ + 8 * ql;
      const half8_t bh = *reinterpret_cast<const half8_t*>(&sm[cur][2][off]);
      const half8_t bl = *reinterpret_cast<const half8_t*>(&sm[cur][3][off]);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        hh[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh, hh[a][b], 0, 0, 0);
        xx[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl, xx[a][b], 0, 0, 0);
        xx[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh, xx[a][b], 0, 0, 0);
      }
    }
    if (ks + 1 < nk) {  // buffer cur ^ 1 was last read in step ks - 1, which ended in a barrier
      lstore(cur ^ 1);
      __syncthreads();
    }
  }
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
        float v = fmaf(xx[a][b][r], 1.0f / 2048.0f, hh[a][b][r]);
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
