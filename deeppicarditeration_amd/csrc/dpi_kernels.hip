// MI355X (gfx950) kernels of the DPI label-generation hot path + the C-ABI of include/dpi.h.
//
// One workgroup (256 threads = 4 waves) owns one collocation point i and 64 consecutive
// Monte-Carlo indices m.  Per workgroup:
//   phase 1  (VALU)  Philox4x32-10 + Box–Muller noise, K-step Euler–Maruyama rollout of the
//                    terminal path (t -> T) and the integral path (t -> s), 100 dims each.
//                    Lane = path; a wave owns whole 4-dim blocks, so Philox counters other
//                    than m are wave-uniform.  Terminal sums stay in registers, integral
//                    sums go to LDS as the MFMA B operand; g(X_T) statistics are reduced
//                    over waves in fixed order.
//   phase 2  (MFMA)  u(s, X_s) and its input gradient for the 64 paths: the MLP as
//                    v_mfma_f32_16x16x4_f32 tiles, hidden x paths orientation (wave = 16
//                    paths), activations kept in registers as the next layer's B operand,
//                    weights staged through LDS 32 rows at a time, backward via the
//                    transposed weights.  X_s = x + c_p S is never formed: layer 1 is
//                    z = (W1x x + b1) + W1t s + c_p (W1x S).
//   phase 3          per-path contributions (g(X_T)-g(x))(1,Y_T) + (T-t)(f-f_b)(1,Y_s)
//                    reduced over the 64 lanes into a per-(point, block) partial slab.
// A pairwise reduce kernel then sums the blocks in a fixed tree (bit-reproducible; equal
// for any split of the blocks over GPUs aligned to powers of two) and a finalize kernel
// divides by M, adds g(x) and clips (picard/data.py:924-926, :525-526, :222).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <type_traits>
#include <algorithm>
#include <string>
#include <vector>

#include "../../include/dpi.h"
#include "dpi_eq.h"
#include "dpi_rng.h"

namespace dpi {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int P = DPI_PATH_BLOCK;  // 64 paths per workgroup
constexpr int NTH = 256;           // threads per workgroup
constexpr int SS = P + 4;          // LDS row stride of the [dim][path] noise tile (bank-conflict free)
constexpr int WST = 136;           // LDS row stride of a staged weight chunk (WST/4 = 2 mod 4)
constexpr int NXP_MAX = 128;       // max padded state dimension
constexpr int HMAX = 128;

struct NetDev {
  int kind;  // 0 zero, 1 mlp
  int H, L, nxp;
  const float* W1x;   // (H, nxp)   W1[:, 1:]
  const float* w1t;   // (H)        W1[:, 0]
  const float* b1;    // (H)
  const float* c1;    // (H)        sum_d W1[h, 1+d]
  const float* W1xT;  // (nxp, H)
  const float* W[4];  // (H, H) hidden layer l = 1..L-1
  const float* WT[4];
  const float* b[4];
  const float* wout;  // (H)
  float bout;
  // fp16-split copies (x = hi + 2^-11 lo) in MFMA fragment order, see pack_split():
  int nxp32;                 // nx padded to 32
  const uint32_t* W1xS;      // (H, nxp32)
  const uint32_t* W1xTS;     // (nxp32, H)
  const uint32_t* WS[4];     // (H, H)
  const uint32_t* WTS[4];
};

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float elu(float z) { return z > 0.f ? z : __expf(z) - 1.0f; }
__device__ __forceinline__ float delu_from_a(float a) { return a > 0.f ? 1.0f : a + 1.0f; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// gfx950 cross-half / cross-row lane swaps (VALU, no LDS): for the pair (a, b) the two results
// sum to [a_lo + a_hi | b_lo + b_hi] (halves of 32 lanes) resp. the same over rows of 16 lanes.
__device__ __forceinline__ float swap32_sum(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_sum(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// sum over the 4 lane groups (lanes j, j+16, j+32, j+48) of the MFMA C layout
__device__ __forceinline__ float qsum(float v) {
  v = swap32_sum(v, v);
  return swap16_sum(v, v);
}
// Column sums of a 64 x 64 block: v[c] is lane l's value of column c; on return lane l holds the
// sum over all 64 lanes of column l.  A halving butterfly: at level m = 32, 16, ..., 1 a lane
// keeps the lower half of its columns if (lane & m) == 0, else the upper half, and adds its
// partner's copy of the kept half — 63 exchanges for 64 columns instead of 6 per column.  The
// summation order of every column is fixed (independent of which block or rank runs it).
template <int M>
__device__ __forceinline__ float dpp_take(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), M, 0xF, 0xF, false));
}
__device__ __forceinline__ float column_sums64(float (&v)[64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = swap32_sum(v[j], v[j + 32]);
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = swap16_sum(v[j], v[j + 16]);
  // within rows of 16: partners by row_mirror (i <-> 15 - i), row_half_mirror (i <-> 7 - i),
  // quad_perm [2,3,0,1] and [1,0,3,2]; the side is the lane bit m in every case
#define DPI_BFLY(MASK, H, CTRL)                                  \
  _Pragma("unroll") for (int j = 0; j < H; ++j) {                \
    const bool up = (lane & MASK) != 0;                          \
    const float keep = up ? v[j + H] : v[j];                     \
    const float send = up ? v[j] : v[j + H];                     \
    v[j] = keep + dpp_take<CTRL>(send);                          \
  }
  DPI_BFLY(8, 8, 0x140)
  DPI_BFLY(4, 4, 0x141)
  DPI_BFLY(2, 2, 0x4E)
  DPI_BFLY(1, 1, 0xB1)
#undef DPI_BFLY
  return v[0];
}

// Stage rows [r0, r0 + nrows) of a row-major global matrix with ncol floats per row
// (ncol % 4 == 0) into LDS rows of stride WST.
__device__ __forceinline__ void stage_rows(const float* __restrict__ g, int ncol, int r0, int nrows, float* wsh) {
  const int nf4 = ncol >> 2;
  for (int idx = threadIdx.x; idx < nrows * nf4; idx += NTH) {
    const int r = idx / nf4, c = idx - r * nf4;
    const float4 v = *reinterpret_cast<const float4*>(g + (size_t)(r0 + r) * ncol + 4 * c);
    *reinterpret_cast<float4*>(wsh + r * WST + 4 * c) = v;
  }
}

// ---------------- fp16-split MFMA (v_mfma_f32_16x16x32_f16, three products per fp32 product)
// x = hi + 2^-11 lo with hi = fp16(x), lo = fp16((x - hi) 2^11): a (x) b = hi_a hi_b + 2^-11 (hi_a lo_b
// + lo_a hi_b) + O(2^-22 |a b|).  Split matrices are packed per row as chunks of 32 columns; chunk
// u holds, for each lane group q = 0..3, 8 hi then 8 lo halves of columns
// k(q, j) = 32u + 4q + (j & 3) + 16 (j >> 2), j = 0..7 — exactly the columns whose activations a
// lane of group q holds in the 16x16 C layout of tiles 2u and 2u+1, so activations become the B
// operand without any data movement.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32v4 __attribute__((ext_vector_type(4)));
constexpr float SPLIT_LO = 2048.0f, SPLIT_INV = 1.0f / 2048.0f;

__device__ __forceinline__ floatx4 mfma16(half8 a, half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void split8(const float (&x)[8], half8& hi, half8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)x[j];
    hi[j] = h;
    lo[j] = (_Float16)((x[j] - (float)h) * SPLIT_LO);
  }
}
// B operand of chunk u from activation tiles 2u, 2u+1 held in the C layout.
__device__ __forceinline__ void split_act(const float (&t0)[4], const float (&t1)[4], half8& hi, half8& lo) {
  const float x[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  split8(x, hi, lo);
}
// Split chunks sit in LDS unpadded (C words per row, as LDS-DMA writes 1 KiB lane-linear per wave
// instruction) with the 16-B granules of row r XOR-swizzled: granule g is stored at g ^ (r & m),
// m = min(15, C/4 - 1).  The 16 lanes of each ds_read_b128 lane group then hit distinct banks.
__device__ __forceinline__ int split_swz(int C) { return C >= 64 ? 15 : (C >> 2) - 1; }
__device__ __forceinline__ void load_a_split(const uint32_t* wsh, int C, int row, int u, int q, half8& ah,
                                             half8& al) {
  const int m = split_swz(C), g = 8 * u + 2 * q, x = row & m;
  const uint32_t* rp = wsh + row * C;
  ah = __builtin_bit_cast(half8, *reinterpret_cast<const u32v4*>(rp + 4 * (g ^ x)));
  al = __builtin_bit_cast(half8, *reinterpret_cast<const u32v4*>(rp + 4 * ((g + 1) ^ x)));
}
// 32 output rows (tiles T0, T0+1) of W B for a staged 32-row chunk; B pre-split per chunk u.
template <int NU>
__device__ __forceinline__ void split_rows32(const uint32_t* wsh, int C, int jj, int qq, const half8 (&bh)[NU],
                                             const half8 (&bl)[NU], floatx4 (&out)[2]) {
  floatx4 am[2], ac[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) am[t] = ac[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      half8 ah, al;
      load_a_split(wsh, C, 16 * t + jj, u, qq, ah, al);
      am[t] = mfma16(ah, bh[u], am[t]);
      ac[t] = mfma16(ah, bl[u], ac[t]);
      ac[t] = mfma16(al, bh[u], ac[t]);
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) out[t][r] = fmaf(ac[t][r], SPLIT_INV, am[t][r]);
}

}  // namespace dpi
#include "dpi_gemm.h"
#include "dpi_pis.h"
namespace dpi {

// LDS layout (floats) shared by the baseline and path kernels.
struct Lds {
  float S[NXP_MAX * SS];   // [dim][path] integral noise sums (path kernel) / x tile (baseline)
  float W[2 * 32 * HMAX];  // weight chunk: f32 rows of stride WST, or two split chunks (LDS-DMA ring)
  float vec[4 * HMAX];     // base0 | w1t | wout | c1
  float bh[4 * HMAX];      // hidden-layer biases
  float xsh[NXP_MAX];      // point x (path kernel) / zeros (baseline)
  float gst[4 * P * NSG];  // per-wave partial g statistics
  float tau[P], cmul[P], bsh[P];
};

// ------------------------------------------------------------------------------ MLP tile
// u and gradient terms for the 16 paths of this wave (path column pp = 16*wave + (lane&15)).
// Inputs (all in LDS): S tile [d][p], xsh (X_d = xsh[d] + cmul_p * S[d][p]), tau (time input),
// cmul, vec[0:H] = base0 (layer-1 bias incl. W1x x), vec[H:2H] = w1t, vec[2H:3H] = wout,
// vec[3H:4H] = c1, bh[l*H:(l+1)*H] = biases of hidden layers l >= 1.
// If bx_out != nullptr (baseline mode) writes b1 + W1x S (per path) to bx_out[pp*bstride + h].
template <int KIND, int H, int L, class SH>
__device__ __forceinline__ void mlp_tile(const EqDev& e, const NetDev& net, SH& sh, int nxt, float& u_out,
                                         float& gsum_out, float& gA_out, float& gB_out, float* bx_out,
                                         int bstride, int n_valid_paths) {
  constexpr int HT = H / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane & 15, qq = lane >> 4;
  const int pp = 16 * wv + jj;
  const float tau = sh.tau[pp];
  const float cm = sh.cmul[pp];
  float act[L][HT][4];

  // ---------------- layer 1: z = base0 + w1t*tau + cmul * (W1x S)
#pragma unroll
  for (int T0 = 0; T0 < HT; T0 += 2) {
    const int nr = (HT - T0) >= 2 ? 32 : 16;
    __syncthreads();
    stage_rows(net.W1x, net.nxp, 16 * T0, nr, sh.W);
    __syncthreads();
#pragma unroll
    for (int T2 = 0; T2 < 2; ++T2) {
      const int T = T0 + T2;
      if (T < HT) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* wrow = sh.W + (16 * T2 + jj) * WST + 4 * qq;
        for (int t = 0; t < nxt; ++t) {
          const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
          const float* bc = sh.S + (16 * t + 4 * qq) * SS + pp;
          acc = mfma4(a.x, bc[0], acc);
          acc = mfma4(a.y, bc[SS], acc);
          acc = mfma4(a.z, bc[2 * SS], acc);
          acc = mfma4(a.w, bc[3 * SS], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * T + 4 * qq + r;
          const float z = fmaf(cm, acc[r], fmaf(sh.vec[H + h], tau, sh.vec[h]));
          act[0][T][r] = elu(z);
          if (bx_out && pp < n_valid_paths) bx_out[(size_t)pp * bstride + h] = sh.vec[h] + acc[r];
        }
      }
    }
  }
  // ---------------- hidden layers
#pragma unroll
  for (int l = 1; l < L; ++l) {
#pragma unroll
    for (int T0 = 0; T0 < HT; T0 += 2) {
      const int nr = (HT - T0) >= 2 ? 32 : 16;
      __syncthreads();
      stage_rows(net.W[l], H, 16 * T0, nr, sh.W);
      __syncthreads();
#pragma unroll
      for (int T2 = 0; T2 < 2; ++T2) {
        const int T = T0 + T2;
        if (T < HT) {
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* wrow = sh.W + (16 * T2 + jj) * WST + 4 * qq;
#pragma unroll
          for (int t = 0; t < HT; ++t) {
            const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
            acc = mfma4(a.x, act[l - 1][t][0], acc);
            acc = mfma4(a.y, act[l - 1][t][1], acc);
            acc = mfma4(a.z, act[l - 1][t][2], acc);
            acc = mfma4(a.w, act[l - 1][t][3], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = 16 * T + 4 * qq + r;
            act[l][T][r] = elu(acc[r] + sh.bh[l * H + h]);
          }
        }
      }
    }
  }
  // ---------------- output u = wout . a_L + bout ; delta_L = wout * elu'(a_L)
  float up = 0.f;
#pragma unroll
  for (int T = 0; T < HT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * T + 4 * qq + r;
      const float w = sh.vec[2 * H + h];
      up = fmaf(w, act[L - 1][T][r], up);
      act[L - 1][T][r] = w * delu_from_a(act[L - 1][T][r]);
    }
  u_out = qsum(up) + net.bout;
  // ---------------- backward through hidden layers: delta_l = (W_{l+1}^T delta_{l+1}) * elu'(a_l)
#pragma unroll
  for (int l = L - 2; l >= 0; --l) {
#pragma unroll
    for (int T0 = 0; T0 < HT; T0 += 2) {
      const int nr = (HT - T0) >= 2 ? 32 : 16;
      __syncthreads();
      stage_rows(net.WT[l + 1], H, 16 * T0, nr, sh.W);
      __syncthreads();
#pragma unroll
      for (int T2 = 0; T2 < 2; ++T2) {
        const int T = T0 + T2;
        if (T < HT) {
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* wrow = sh.W + (16 * T2 + jj) * WST + 4 * qq;
#pragma unroll
          for (int t = 0; t < HT; ++t) {
            const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
            acc = mfma4(a.x, act[l + 1][t][0], acc);
            acc = mfma4(a.y, act[l + 1][t][1], acc);
            acc = mfma4(a.z, act[l + 1][t][2], acc);
            acc = mfma4(a.w, act[l + 1][t][3], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) act[l][T][r] = acc[r] * delu_from_a(act[l][T][r]);
        }
      }
    }
  }
  // ---------------- input gradient
  if (!Eq<KIND>::GRAD_FULL) {
    float gp = 0.f;
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) gp = fmaf(sh.vec[3 * H + 16 * T + 4 * qq + r], act[0][T][r], gp);
    gsum_out = qsum(gp);
    gA_out = gB_out = 0.f;
  } else {
    float A = 0.f, B = 0.f;
    for (int T0 = 0; T0 < nxt; T0 += 2) {
      const int nr = (nxt - T0) >= 2 ? 32 : 16;
      __syncthreads();
      stage_rows(net.W1xT, H, 16 * T0, nr, sh.W);
      __syncthreads();
#pragma unroll
      for (int T2 = 0; T2 < 2; ++T2) {
        const int T = T0 + T2;
        if (T < nxt) {
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* wrow = sh.W + (16 * T2 + jj) * WST + 4 * qq;
#pragma unroll
          for (int t = 0; t < HT; ++t) {
            const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
            acc = mfma4(a.x, act[0][t][0], acc);
            acc = mfma4(a.y, act[0][t][1], acc);
            acc = mfma4(a.z, act[0][t][2], acc);
            acc = mfma4(a.w, act[0][t][3], acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int d = 16 * T + 4 * qq + r;
            if (d < e.nx) {
              const float X = fmaf(cm, sh.S[d * SS + pp], sh.xsh[d]);
              Eq<KIND>::gacc(e, d, X, acc[r], A, B);
            }
          }
        }
      }
    }
    gA_out = qsum(A);
    gB_out = qsum(B);
    gsum_out = 0.f;
  }
}

// Weight-chunk stream of the split MLP: every 32-row chunk of every matrix, in use order, is
// copied global -> LDS by LDS-DMA one chunk ahead into a two-slot ring (the copy overlaps the
// MFMAs of the current chunk; no registers, one barrier per chunk).
// Chunk index -> (matrix, C, row offset): layer 1 (W1x), hidden layers (W_l), backward
// (W_{l+1}^T, l = L-2..0), then — GRAD_FULL only — the input gradient (W1x^T).
template <int H, int L>
struct SplitStream {
  static constexpr int NT = H / 32;  // chunks per H-row matrix
  const NetDev& net;
  int C1, n1, nT1, total;
  __device__ SplitStream(const NetDev& n, bool grad_full) : net(n) {
    C1 = n.nxp32;
    n1 = NT;                               // layer-1 chunks (H output rows)
    nT1 = C1 / 32;                         // W1x^T chunks (C1 output rows)
    total = n1 + 2 * (L - 1) * NT + (grad_full ? nT1 : 0);
  }
  __device__ __forceinline__ void desc(int idx, const uint32_t*& g, int& C, int& r0) const {
    if (idx < n1) {
      g = net.W1xS, C = C1, r0 = 32 * idx;
      return;
    }
    idx -= n1;
    if (idx < (L - 1) * NT) {
      g = net.WS[1 + idx / NT], C = H, r0 = 32 * (idx % NT);
      return;
    }
    idx -= (L - 1) * NT;
    if (idx < (L - 1) * NT) {
      g = net.WTS[L - 1 - idx / NT], C = H, r0 = 32 * (idx % NT);
      return;
    }
    idx -= (L - 1) * NT;
    g = net.W1xTS, C = H, r0 = 32 * idx;
  }
  // LDS-DMA of chunk idx into ring slot idx & 1: wave-instruction w writes LDS granules
  // [64 w, 64 w + 64) lane-linearly; lane i's source is the granule that belongs there.
  __device__ __forceinline__ void issue(int idx, uint32_t* ring) const {
    if (idx >= total) return;
    const uint32_t* g;
    int C, r0;
    desc(idx, g, C, r0);
    uint32_t* dst = ring + (idx & 1) * (32 * HMAX);
    const int gpr = C >> 2, m = split_swz(C), lane = threadIdx.x & 63;
    for (int w = threadIdx.x >> 6; w < (C >> 3); w += NTH / 64) {
      const int G = 64 * w + lane, r = G / gpr, gs = (G - r * gpr) ^ (r & m);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(g + (size_t)(r0 + r) * C + 4 * gs),
          (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  }
  // One barrier per chunk: it retires this wave's DMA of chunk idx (vmcnt(0) before s_barrier)
  // and every wave's reads of chunk idx - 1, whose slot then receives chunk idx + 1.
  __device__ __forceinline__ const uint32_t* enter(int idx, uint32_t* ring, int& C) const {
    const uint32_t* g;
    int r0;
    desc(idx, g, C, r0);
    __syncthreads();
    issue(idx + 1, ring);
    return ring + (idx & 1) * (32 * HMAX);
  }
};

// mlp_tile on the fp16-split MFMA (H % 32 == 0): same inputs, outputs and tile layout; each
// 16x16x4 f32 chain becomes 16x16x32 f16 chunks (3 MFMAs per 32-wide chunk instead of 8), the
// weights come pre-split from NetDev::*S, the activations are split in registers.
template <int KIND, int H, int L, class SH>
__device__ __forceinline__ void mlp_tile_split(const EqDev& e, const NetDev& net, SH& sh, float& u_out,
                                               float& gsum_out, float& gA_out, float& gB_out) {
  static_assert(H % 32 == 0, "split MLP needs H % 32 == 0");
  constexpr int HT = H / 16, NU = H / 32;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane & 15, qq = lane >> 4;
  const int pp = 16 * wv + jj;
  const float tau = sh.tau[pp];
  const float cm = sh.cmul[pp];
  uint32_t* wsh = reinterpret_cast<uint32_t*>(sh.W);
  SplitStream<H, L> ss(net, Eq<KIND>::GRAD_FULL);
  const int nu1 = ss.C1 >> 5;
  int chunk = 0;
  ss.issue(0, wsh);
  float act[L][HT][4];
  half8 bh[NU], bl[NU];

  // ---------------- layer 1: z = base0 + w1t*tau + cmul * (W1x S)
  half8 xh[NXP_MAX / 32], xl[NXP_MAX / 32];  // the noise tile as B operand, split once
#pragma unroll
  for (int u = 0; u < NXP_MAX / 32; ++u) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = u < nu1 ? sh.S[(32 * u + 4 * qq + (j & 3) + 16 * (j >> 2)) * SS + pp] : 0.f;
    split8(x, xh[u], xl[u]);
  }
#pragma unroll
  for (int T0 = 0; T0 < HT; T0 += 2) {
    int C;
    const uint32_t* wch = ss.enter(chunk++, wsh, C);
    floatx4 am[2], ac[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) am[t] = ac[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NXP_MAX / 32; ++u) {
      if (u < nu1) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          half8 ah, al;
          load_a_split(wch, C, 16 * t + jj, u, qq, ah, al);
          am[t] = mfma16(ah, xh[u], am[t]);
          ac[t] = mfma16(ah, xl[u], ac[t]);
          ac[t] = mfma16(al, xh[u], ac[t]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * (T0 + t) + 4 * qq + r;
        const float acc = fmaf(ac[t][r], SPLIT_INV, am[t][r]);
        act[0][T0 + t][r] = elu(fmaf(cm, acc, fmaf(sh.vec[H + h], tau, sh.vec[h])));
      }
  }
  // ---------------- hidden layers
#pragma unroll
  for (int l = 1; l < L; ++l) {
#pragma unroll
    for (int u = 0; u < NU; ++u) split_act(act[l - 1][2 * u], act[l - 1][2 * u + 1], bh[u], bl[u]);
#pragma unroll
    for (int T0 = 0; T0 < HT; T0 += 2) {
      int C;
      const uint32_t* wch = ss.enter(chunk++, wsh, C);
      floatx4 o[2];
      split_rows32<NU>(wch, C, jj, qq, bh, bl, o);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) act[l][T0 + t][r] = elu(o[t][r] + sh.bh[l * H + 16 * (T0 + t) + 4 * qq + r]);
    }
  }
  // ---------------- output u = wout . a_L + bout ; delta_L = wout * elu'(a_L)
  float up = 0.f;
#pragma unroll
  for (int T = 0; T < HT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * T + 4 * qq + r;
      const float w = sh.vec[2 * H + h];
      up = fmaf(w, act[L - 1][T][r], up);
      act[L - 1][T][r] = w * delu_from_a(act[L - 1][T][r]);
    }
  u_out = qsum(up) + net.bout;
  // ---------------- backward through hidden layers: delta_l = (W_{l+1}^T delta_{l+1}) * elu'(a_l)
#pragma unroll
  for (int l = L - 2; l >= 0; --l) {
#pragma unroll
    for (int u = 0; u < NU; ++u) split_act(act[l + 1][2 * u], act[l + 1][2 * u + 1], bh[u], bl[u]);
#pragma unroll
    for (int T0 = 0; T0 < HT; T0 += 2) {
      int C;
      const uint32_t* wch = ss.enter(chunk++, wsh, C);
      floatx4 o[2];
      split_rows32<NU>(wch, C, jj, qq, bh, bl, o);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) act[l][T0 + t][r] = o[t][r] * delu_from_a(act[l][T0 + t][r]);
    }
  }
  // ---------------- input gradient
  if (!Eq<KIND>::GRAD_FULL) {
    float gp = 0.f;
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) gp = fmaf(sh.vec[3 * H + 16 * T + 4 * qq + r], act[0][T][r], gp);
    gsum_out = qsum(gp);
    gA_out = gB_out = 0.f;
  } else {
#pragma unroll
    for (int u = 0; u < NU; ++u) split_act(act[0][2 * u], act[0][2 * u + 1], bh[u], bl[u]);
    float A = 0.f, B = 0.f;
    for (int T0 = 0; T0 < (ss.C1 >> 4); T0 += 2) {
      int C;
      const uint32_t* wch = ss.enter(chunk++, wsh, C);
      floatx4 o[2];
      split_rows32<NU>(wch, C, jj, qq, bh, bl, o);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = 16 * (T0 + t) + 4 * qq + r;
          if (d < e.nx) {
            const float X = fmaf(cm, sh.S[d * SS + pp], sh.xsh[d]);
            Eq<KIND>::gacc(e, d, X, o[t][r], A, B);
          }
        }
    }
    gA_out = qsum(A);
    gB_out = qsum(B);
    gsum_out = 0.f;
  }
}

// LDS of the fully-nonlinear (GBM) path kernel: every weight matrix stays resident for the
// 100-direction tangent sweep.  H <= 64, L <= 4.
template <int H>
struct LdsGbm {
  static constexpr int WXS = NXP_MAX + 8;  // W1x row stride (WXS/4 = 2 mod 4)
  static constexpr int WHS = H + 8;        // hidden row stride
  float S[NXP_MAX * SS];
  float W1x[H * WXS];
  float Wh[3][H * WHS];
  float vec[4 * HMAX];
  float bh[4 * HMAX];
  float xsh[NXP_MAX];
  float hb[NXP_MAX];
  float gst[4 * P * NSG];
  float fst[4 * P * NSG];
  float wx[NSG];
  float tau[P], cmul[P], bsh[P], fbp[P];
  float smt[P];                    // Hessian labels: s - t per path
  unsigned char cnt[NXP_MAX * P];  // SDGD index histogram [d][path]
};

__device__ __forceinline__ float d2elu_from_a(float a) { return a > 0.f ? 0.f : a + 1.0f; }

// Diagonal of the x-Hessian of u at (s, X_s) for this wave's 16 paths, contracted with the
// path's SDGD index histogram: s1 = sum_d cnt[d] u_dd, s2 = sum_d cnt[d] |u_dd|.
// Uses u_dd = sum_l < lam_l, elu''(z_l) * zdot_l^2 >, with lam_l = du/da_l (one backward pass)
// and zdot_l = dz_l/dx_d (first-order tangents only): half the MACs of second-order
// forward mode.  All GEMMs are v_mfma_f32_16x16x4_f32 in the hidden x path orientation.
template <int H, int L>
__device__ __forceinline__ void mlp_hdiag(const EqDev& e, const NetDev& net, LdsGbm<H>& sh, int nxt, float& s1_out,
                                          float& s2_out) {
  constexpr int HT = H / 16;
  constexpr int WXS = LdsGbm<H>::WXS, WHS = LdsGbm<H>::WHS;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane & 15, qq = lane >> 4;
  const int pp = 16 * wv + jj;
  const float tau = sh.tau[pp];
  const float cm = sh.cmul[pp];
  float act[L][HT][4];
  float lam[L][HT][4];
  // forward
#pragma unroll
  for (int T = 0; T < HT; ++T) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = sh.W1x + (16 * T + jj) * WXS + 4 * qq;
    for (int t = 0; t < nxt; ++t) {
      const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
      const float* bc = sh.S + (16 * t + 4 * qq) * SS + pp;
      acc = mfma4(a.x, bc[0], acc);
      acc = mfma4(a.y, bc[SS], acc);
      acc = mfma4(a.z, bc[2 * SS], acc);
      acc = mfma4(a.w, bc[3 * SS], acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * T + 4 * qq + r;
      act[0][T][r] = elu(fmaf(cm, acc[r], fmaf(sh.vec[H + h], tau, sh.vec[h])));
    }
  }
#pragma unroll
  for (int l = 1; l < L; ++l) {
#pragma unroll
    for (int T = 0; T < HT; ++T) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* wrow = sh.Wh[l - 1] + (16 * T + jj) * WHS + 4 * qq;
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
        acc = mfma4(a.x, act[l - 1][t][0], acc);
        acc = mfma4(a.y, act[l - 1][t][1], acc);
        acc = mfma4(a.z, act[l - 1][t][2], acc);
        acc = mfma4(a.w, act[l - 1][t][3], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) act[l][T][r] = elu(acc[r] + sh.bh[l * H + 16 * T + 4 * qq + r]);
    }
  }
  // adjoints lam_l = du/da_l
#pragma unroll
  for (int T = 0; T < HT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) lam[L - 1][T][r] = sh.vec[2 * H + 16 * T + 4 * qq + r];
#pragma unroll
  for (int l = L - 2; l >= 0; --l) {
    float Bm[HT][4];
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) Bm[t][r] = delu_from_a(act[l + 1][t][r]) * lam[l + 1][t][r];
#pragma unroll
    for (int T = 0; T < HT; ++T) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)  // A[i][k] = W_{l+1}[k][i]: column 16T+jj, row 16t+4qq+r
          acc = mfma4(sh.Wh[l][(16 * t + 4 * qq + r) * WHS + 16 * T + jj], Bm[t][r], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) lam[l][T][r] = acc[r];
    }
  }
  // tangent sweep over the state dimensions
  float s1 = 0.f, s2 = 0.f;
  for (int d = 0; d < e.nx; ++d) {
    float z[HT][4];
    float term = 0.f;
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        z[T][r] = sh.W1x[(16 * T + 4 * qq + r) * WXS + d];
        term = fmaf(lam[0][T][r] * d2elu_from_a(act[0][T][r]), z[T][r] * z[T][r], term);
      }
#pragma unroll
    for (int l = 1; l < L; ++l) {
      float Bm[HT][4];
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Bm[t][r] = delu_from_a(act[l - 1][t][r]) * z[t][r];
#pragma unroll
      for (int T = 0; T < HT; ++T) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* wrow = sh.Wh[l - 1] + (16 * T + jj) * WHS + 4 * qq;
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
          acc = mfma4(a.x, Bm[t][0], acc);
          acc = mfma4(a.y, Bm[t][1], acc);
          acc = mfma4(a.z, Bm[t][2], acc);
          acc = mfma4(a.w, Bm[t][3], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          z[T][r] = acc[r];
          term = fmaf(lam[l][T][r] * d2elu_from_a(act[l][T][r]), acc[r] * acc[r], term);
        }
      }
    }
    const float ud = qsum(term);
    const float c = (float)sh.cnt[d * P + pp];
    s1 = fmaf(c, ud, s1);
    s2 = fmaf(c, fabsf(ud), s2);
  }
  s1_out = s1;
  s2_out = s2;
}

// ------------------------------------------------------------------------------ kernels
// Draws 1-3 (picard/data.py:161-167, equations.py:118-124/:217-230, utils.py:785-789).
template <int KIND>
__global__ void k_sample_points(EqDev e, int n, uint32_t k0, uint32_t k1, uint32_t c3t, uint32_t c3x0,
                                uint32_t c3x, uint32_t point_base, float eps, float alpha_init_sqrt, float* tx) {
  const int nb = (e.nx + 3) >> 2;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = gid / nb, j = gid - i * nb;
  if (i >= n) return;
  const uint32_t ig = point_base + (uint32_t)i;
  const float U = u01_co(philox4x32_10(0u, 0u, ig, c3t, k0, k1).x);
  const float t = (e.T - 2.f * eps) * (1.f - U) + eps;
  float* row = tx + (size_t)i * (1 + e.nx);
  if (j == 0) row[0] = t;
  const f4 z = normals4(philox4x32_10((uint32_t)j, 0u, ig, c3x, k0, k1));
  f4 z0 = {0.f, 0.f, 0.f, 0.f};
  if (KIND == DPI_EQ_OU) {
    z0 = normals4(philox4x32_10((uint32_t)j, 0u, ig, c3x0, k0, k1));
    z0.a *= alpha_init_sqrt;
    z0.b *= alpha_init_sqrt;
    z0.c *= alpha_init_sqrt;
    z0.d *= alpha_init_sqrt;
  }
  const float sc = sqrtf(t) * e.asq;
  const float zz[4] = {z.a, z.b, z.c, z.d};
  const float xx[4] = {z0.a, z0.b, z0.c, z0.d};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int d = 4 * j + q;
    if (d < e.nx) row[1 + d] = fmaf(sc, zz[q], xx[q]);
  }
}

// Block-wide sum over 256 threads (result on every thread); red: >= 4 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

constexpr int NTHB = 1024;  // baseline workgroup: 16 waves
__device__ __forceinline__ float block_sum_b(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float a = 0.f;
  for (int w = 0; w < NTHB / 64; ++w) a += red[w];
  return a;
}

// Baseline per point (one workgroup per point): g(x), the state-dependent part of
// f(t, x, u, grad u) and bx = b1 + W1[:,1:] x (picard/data.py:918-920 g_single, :506-518
// f_baseline).  A latency-bound handful of points: 1024 threads per point split every mat-vec
// over k-slices (weights read coalesced through the transposed copies), no LDS staging.
template <int KIND, bool ZERO>
__global__ __launch_bounds__(NTHB) void k_baseline(EqDev e, NetDev net, const float* __restrict__ tx, int n,
                                                  float* __restrict__ gx, float* __restrict__ fb,
                                                  float* __restrict__ bx, float* __restrict__ hb) {
  __shared__ float xs[NXP_MAX];
  __shared__ float act[4][HMAX];
  __shared__ float dbuf[2][HMAX];
  __shared__ float red[NTHB / 64];
  const int i = blockIdx.x, tid = threadIdx.x;
  const int nx = e.nx, F = 1 + nx;
  const float* row = tx + (size_t)i * F;
  const float t = row[0];
  for (int d = tid; d < NXP_MAX; d += NTHB) xs[d] = d < nx ? row[1 + d] : 0.f;
  __syncthreads();
  // g(x): per-thread dims, then per-statistic block sums in fixed order (one barrier pair)
  {
    __shared__ float redn[NTHB / 64][NSG];
    float st[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) st[c] = 0.f;
    for (int d = tid; d < nx; d += NTHB) Eq<KIND>::gstat(e, d, xs[d], st);
#pragma unroll
    for (int c = 0; c < NSG; ++c) st[c] = wave_sum(st[c]);
    if ((tid & 63) == 0)
#pragma unroll
      for (int c = 0; c < NSG; ++c) redn[tid >> 6][c] = st[c];
    __syncthreads();
    if (tid == 0) {
#pragma unroll
      for (int c = 0; c < NSG; ++c) {
        float a = 0.f;
        for (int w = 0; w < NTHB / 64; ++w) a += redn[w][c];
        st[c] = a;
      }
      gx[i] = Eq<KIND>::gfin(e, st);
    }
  }
  float Cb = 0.f;
  if constexpr (KIND == DPI_EQ_GBM) {
    // exact-solution part of ffi at (t, x) (equations.py:457-466)
    float arg[NSG], sn[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      float v = 0.f;
      if (c < e.nodes)
        for (int d = tid; d < nx; d += NTHB) v = fmaf(e.gw[c * F + 1 + d], xs[d], v);
      v = block_sum_b(v, red);
      arg[c] = c < e.nodes ? fmaf(e.gw[c * F], t, v) : 0.f;
      sn[c] = __sinf(arg[c]);
    }
    const float ah = block_sum_b(Eq<KIND>::abs_hess_partial(e, sn, tid, NTHB), red);
    Cb = Eq<KIND>::exact_scalar_terms(e, arg) - 0.25f * ah;
    if (ZERO) {
      for (int d = tid; d < NXP_MAX; d += NTHB) hb[(size_t)i * NXP_MAX + d] = 0.f;
      if (tid == 0) fb[i] = Cb;
      return;
    }
  }
  if (ZERO) {
    if (tid == 0) fb[i] = Eq<KIND>::ffv(e, 0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int H = net.H, L = net.L, nxp = net.nxp;
  // Mat-vecs y[h] = sum_k Wt[k][h] v[k] (Wt row-major (K, H), coalesced in h): thread tid takes
  // unit h = tid % H and the k-slice tid / H of NTHB / H slices (<= 16 values, all loads issued
  // before the first FMA: one memory latency per layer); the slices are added in fixed order by
  // the unit's owner.
  __shared__ float part[NTHB];
  auto matvec = [&](const float* __restrict__ Wt, const float* v, int K) -> float {
    const int h = tid % H, ns = NTHB / H, sl = tid / H;
    const int kc = (K + ns - 1) / ns, k0 = sl * kc, k1 = min(K, k0 + kc);  // kc <= 16
    float w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = k0 + j < k1 ? Wt[(size_t)(k0 + j) * H + h] : 0.f;  // all loads in flight
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      if (k0 + j < k1) a0 = fmaf(w[j], v[k0 + j], a0);
      if (k0 + j + 1 < k1) a1 = fmaf(w[j + 1], v[k0 + j + 1], a1);
    }
    part[tid] = a0 + a1;
    __syncthreads();
    float y = 0.f;
    if (tid < H)
      for (int j = 0; j < ns; ++j) y += part[j * H + tid];
    return y;  // valid for tid < H; the caller's barrier precedes the next use of part
  };
  // layer 1
  {
    const float acc = matvec(net.W1xT, xs, nx);
    if (tid < H) {
      bx[(size_t)i * H + tid] = net.b1[tid] + acc;
      act[0][tid] = elu(fmaf(net.w1t[tid], t, net.b1[tid] + acc));
    }
    __syncthreads();
  }
  for (int l = 1; l < L; ++l) {
    const float acc = matvec(net.WT[l], act[l - 1], H);
    if (tid < H) act[l][tid] = elu(acc + net.b[l][tid]);
    __syncthreads();
  }
  if constexpr (KIND == DPI_EQ_GBM) {
    // Hessian diagonal at (t, x): adjoints lam_l = du/da_l, then one thread per state dimension
    // runs its first-order tangent chain (column-major in LDS) and contracts with lam_l * elu''.
    __shared__ float lamb[4][HMAX];
    __shared__ float ztb[2][64][NXP_MAX];
    if (tid < H) lamb[L - 1][tid] = net.wout[tid];
    __syncthreads();
    for (int l = L - 2; l >= 0; --l) {
      if (tid < H) {
        const float* w = net.W[l + 1];
        float acc = 0.f;
        for (int h = 0; h < H; ++h) acc = fmaf(w[(size_t)h * H + tid], delu_from_a(act[l + 1][h]) * lamb[l + 1][h], acc);
        lamb[l][tid] = acc;
      }
      __syncthreads();
    }
    // Tangent sweep as an LDS mat-mat per layer: thread (d = tid % 128, hg = tid / 128) owns the
    // rows h = hg, hg + 8, ... of the tangent Z_l[h][d] = sum_k W_l[h][k] elu'(a_{l-1}[k]) Z_{l-1}[k][d].
    __shared__ float wsc[64 * 65];
    __shared__ float udp[8][NXP_MAX];
    const int d = tid % NXP_MAX, hg = tid / NXP_MAX;  // NTHB = 8 x NXP_MAX
    float ud = 0.f;
    for (int h = hg; h < H; h += 8) {
      const float z = d < nx ? net.W1x[(size_t)h * nxp + d] : 0.f;
      ztb[0][h][d] = z;
      ud = fmaf(lamb[0][h] * d2elu_from_a(act[0][h]), z * z, ud);
    }
    int cz = 0;
    for (int l = 1; l < L; ++l) {
      for (int q = tid; q < H * H; q += NTHB) {
        const int h = q / H, k = q - h * H;
        wsc[h * 65 + k] = net.W[l][q] * delu_from_a(act[l - 1][k]);
      }
      __syncthreads();  // wsc and Z_{l-1} complete
      for (int h = hg; h < H; h += 8) {
        float z = 0.f;
        for (int k = 0; k < H; ++k) z = fmaf(wsc[h * 65 + k], ztb[cz][k][d], z);
        ztb[cz ^ 1][h][d] = z;
        ud = fmaf(lamb[l][h] * d2elu_from_a(act[l][h]), z * z, ud);
      }
      cz ^= 1;
      __syncthreads();  // before wsc is overwritten
    }
    udp[hg][d] = ud;
    __syncthreads();
    if (tid < NXP_MAX) {
      float a = 0.f;
      for (int g = 0; g < 8; ++g) a += udp[g][tid];
      hb[(size_t)i * NXP_MAX + tid] = tid < nx ? a : 0.f;
    }
    if (tid == 0) fb[i] = Cb;
    return;
  }
  const float u = block_sum_b(tid < H ? net.wout[tid] * act[L - 1][tid] : 0.f, red) + net.bout;
  int cur = 0;
  if (tid < H) dbuf[0][tid] = net.wout[tid] * delu_from_a(act[L - 1][tid]);
  __syncthreads();
  for (int l = L - 2; l >= 0; --l) {
    // W_{l+1} (H_out, H_in) row-major is the transposed operand of this mat-vec
    const float acc = matvec(net.W[l + 1], dbuf[cur], H);
    if (tid < H) dbuf[cur ^ 1][tid] = acc * delu_from_a(act[l][tid]);
    cur ^= 1;
    __syncthreads();
  }
  float gs = 0.f, gA = 0.f, gB = 0.f;
  if (!Eq<KIND>::GRAD_FULL) {
    gs = block_sum_b(tid < H ? net.c1[tid] * dbuf[cur][tid] : 0.f, red);
  } else {
    float A = 0.f, B = 0.f;
    for (int d = tid; d < nx; d += NTHB) {
      float z = 0.f;
      for (int k = 0; k < H; ++k) z = fmaf(net.W1x[(size_t)k * nxp + d], dbuf[cur][k], z);
      Eq<KIND>::gacc(e, d, xs[d], z, A, B);
    }
    gA = block_sum_b(A, red);
    gB = block_sum_b(B, red);
  }
  if (tid == 0) fb[i] = Eq<KIND>::ffv(e, u, gs, gA, gB);  // state-dependent part
}

struct PathArgs {
  const float* tx;
  const float* gx;
  const float* fb;
  const float* bx;
  const float* hb;  // GBM: baseline Hessian diagonal [n][NXP_MAX]
  float* partial;
  int n, nbp, m_begin, K, flags;
  uint32_t k0, k1, c3t, c3s, c3i, c3q, point_base;
  int order;  // phase order policy (k_paths)
  int split;  // fused MLP on the fp16-split MFMA
  float* hpart;            // Hessian labels: block sums [n][nbp][nx*nx]
  uint32_t c3h1, c3h2;     // Hessian labels: Malliavin normal streams (tags HTERM, HINT)
};

// ------------------------------------------------------------------------------ Hessian labels
// Malliavin-weight Hessian block of generate_with_gradients_and_hessians (picard/data.py:1220-1223;
// terminal :1185-1199, integral :869-881), per 64-path block, after phase 3 of k_paths:
//   H_blk = sum_p [ aI_p (N2 N2^T - I) + aT_p (N1 N1^T - I) ]
//   aI = (T-t) (f(s, x + a sqrt(s-t) N2) + f(s, x - ...) - 2 f_b) / 2 / (s-t)     (full Hessian f)
//   aT = (g(x + a sqrt(T-t) N1) + g(x - ...) - 2 g(x)) / 2 / (T-t)
// N1, N2: fresh normals (tags HTERM / HINT, k = 0), written into the noise tile in turn; the
// outer-product sums are (nx x 64) (64 x nx) products on v_mfma_f32_16x16x4_f32 over the upper
// triangle of 16 x 16 tiles (wave w owns tiles w, w+4, ...), mirrored on store.
template <int H, int L>
__device__ __forceinline__ void hess_accum(LdsGbm<H>& sh, const float* wgt, int NT, floatx4 (&acc)[9]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, jj = lane & 15, qq = lane >> 4;
  const int ntiles = NT * (NT + 1) / 2;
#pragma unroll
  for (int sl = 0; sl < 9; ++sl) {
    const int q = wv + 4 * sl;
    if (q < ntiles) {
      int I = 0, r = q;
      while (r >= NT - I) {
        r -= NT - I;
        ++I;
      }
      const int J = I + r;
      const float* ra = sh.S + (16 * I + jj) * SS + qq;
      const float* rb = sh.S + (16 * J + jj) * SS + qq;
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[sl] = mfma4(ra[4 * t] * wgt[4 * t + qq], rb[4 * t], acc[sl]);
    }
  }
}

template <int KIND, int H, int L, bool ZERO>
__device__ __forceinline__ void hess_block(const EqDev& e, const NetDev& net, const PathArgs& a, LdsGbm<H>& sh,
                                           int i, int blk, uint32_t ig, uint32_t m, float s, float smt, float tmt,
                                           float g_x, int nxp) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, jj = lane & 15, qq = lane >> 4, pp = 16 * wv + jj;
  const int nx = e.nx, F = 1 + nx, nb = (nx + 3) >> 2, NT = nxp / 16;
  // f at (s, x + cmul S) with the full Hessian diagonal (get_f without SDGD, data.py:1262-1272);
  // valid in the lanes of group qq == 0 for path pp
  auto f_eval = [&]() -> float {
    float s1 = 0.f, s2 = 0.f;
    if (!ZERO) mlp_hdiag<H, L>(e, net, sh, nxp / 16, s1, s2);
    const float c1 = 0.5f * (1.0f - e.alpha), c2 = 0.25f;
    float arg[NSG], sn[NSG];
    const float spp = sh.tau[pp], cpp = sh.cmul[pp];
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      arg[c] = 0.f;
      if (c < e.nodes) {
        const float ws = ((sh.fst[(0 * P + pp) * NSG + c] + sh.fst[(1 * P + pp) * NSG + c]) +
                          sh.fst[(2 * P + pp) * NSG + c]) + sh.fst[(3 * P + pp) * NSG + c];
        arg[c] = fmaf(e.gw[c * F], spp, fmaf(cpp, ws, sh.wx[c]));
      }
      sn[c] = __sinf(arg[c]);
    }
    const float ah = qsum(Eq<KIND>::abs_hess_partial(e, sn, qq, 4));
    return c1 * s1 + c2 * s2 + Eq<KIND>::exact_scalar_terms(e, arg) - 0.25f * ah;
  };
  float* wgt = sh.bsh;  // per-path weights of the current outer-product term
  floatx4 acc[9];
#pragma unroll
  for (int sl = 0; sl < 9; ++sl) acc[sl] = floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- integral term: N2 -> noise tile, w . N2 for the exact-solution terms
  __syncthreads();  // phase 3 is done with the integral noise tile
  {
    float fs[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) fs[c] = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = wv + 4 * c;
      if (j < nb) {
        const f4 z = normals4(philox4x32_10((uint32_t)j, m, ig, a.c3h2, a.k0, a.k1));
        const float zz[4] = {z.a, z.b, z.c, z.d};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = 4 * j + q;
          const float v = d < nx ? zz[q] : 0.f;
          sh.S[d * SS + lane] = v;
          if (d < nx)
#pragma unroll
            for (int c2 = 0; c2 < NSG; ++c2)
              if (c2 < e.nodes) fs[c2] = fmaf(e.gw[c2 * F + 1 + d], v, fs[c2]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NSG; ++c) sh.fst[(wv * P + lane) * NSG + c] = fs[c];
  }
  const float cw = e.asq * sqrtf(smt);
  if (wv == 0) {
    sh.cmul[lane] = cw;
    sh.smt[lane] = smt;
  }
  __syncthreads();
  const float fplus = f_eval();
  __syncthreads();
  if (wv == 0) sh.cmul[lane] = -cw;
  __syncthreads();
  const float fminus = f_eval();
  const float fbp = sh.fbp[pp];
  if (qq == 0) wgt[pp] = tmt * ((fplus + fminus - 2.f * fbp) * 0.5f / sh.smt[pp]);  // path pp, not this lane's
  __syncthreads();
  const float aI = wgt[lane];  // lane = path
  hess_accum<H, L>(sh, wgt, NT, acc);

  // ---- terminal term: N1 -> noise tile, g(x +- a sqrt(T-t) N1)
  __syncthreads();  // every wave is done reading N2 and the weights
  float gp[NSG], gm[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) gp[c] = gm[c] = 0.f;
  const float cw1 = e.asq * sqrtf(tmt);
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int j = wv + 4 * c;
    if (j < nb) {
      const f4 z = normals4(philox4x32_10((uint32_t)j, m, ig, a.c3h1, a.k0, a.k1));
      const float zz[4] = {z.a, z.b, z.c, z.d};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * j + q;
        const float v = d < nx ? zz[q] : 0.f;
        sh.S[d * SS + lane] = v;
        if (d < nx) {
          Eq<KIND>::gstat(e, d, fmaf(cw1, v, sh.xsh[d]), gp);
          Eq<KIND>::gstat(e, d, fmaf(-cw1, v, sh.xsh[d]), gm);
        }
      }
    }
  }
  auto wave_stats = [&](float (&st)[NSG]) -> float {  // g from the 4 waves' partial statistics
#pragma unroll
    for (int c = 0; c < NSG; ++c) sh.gst[(wv * P + lane) * NSG + c] = st[c];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      st[c] = ((sh.gst[(0 * P + lane) * NSG + c] + sh.gst[(1 * P + lane) * NSG + c]) +
               sh.gst[(2 * P + lane) * NSG + c]) + sh.gst[(3 * P + lane) * NSG + c];
    __syncthreads();
    return Eq<KIND>::gfin(e, st);
  };
  const float gplus = wave_stats(gp);
  const float gminus = wave_stats(gm);
  const float aT = (gplus + gminus - 2.f * g_x) * 0.5f / tmt;
  if (wv == 0) wgt[lane] = aT;
  __syncthreads();
  hess_accum<H, L>(sh, wgt, NT, acc);

  // ---- identity part, store (upper tiles mirrored)
  const float dsum = wave_sum(aI + aT);
  float* out = a.hpart + ((size_t)i * a.nbp + blk) * (size_t)nx * nx;
  const int ntiles = NT * (NT + 1) / 2;
#pragma unroll
  for (int sl = 0; sl < 9; ++sl) {
    const int q = wv + 4 * sl;
    if (q < ntiles) {
      int I = 0, r = q;
      while (r >= NT - I) {
        r -= NT - I;
        ++I;
      }
      const int J = I + r;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int d1 = 16 * I + 4 * qq + rr, d2 = 16 * J + jj;
        if (d1 < nx && d2 < nx && d1 <= d2) {  // upper triangle, mirrored: exactly symmetric labels
          const float v = acc[sl][rr] - (d1 == d2 ? dsum : 0.f);
          out[(size_t)d1 * nx + d2] = v;
          if (d1 != d2) out[(size_t)d2 * nx + d1] = v;
        }
      }
    }
  }
}

// One workgroup = (point i, 64 consecutive MC indices).  See the file header.
template <int KIND, int H, int L, bool ZERO, bool SPLIT, bool HESS = false>
__global__ __launch_bounds__(256, KIND == DPI_EQ_GBM ? 1 : 2) void k_paths(EqDev e, NetDev net, PathArgs a) {
  static_assert(!HESS || KIND == DPI_EQ_GBM, "Hessian labels: GBM (SimpleDiffusionEquationWithHessian) only");
  constexpr bool GBM = KIND == DPI_EQ_GBM;
  using SH = std::conditional_t<GBM, LdsGbm<H>, Lds>;
  __shared__ SH sh;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = blockIdx.x / a.nbp, blk = blockIdx.x - i * a.nbp;
  const uint32_t ig = a.point_base + (uint32_t)i;
  const uint32_t m = (uint32_t)(a.m_begin + P * blk + lane);
  const int nx = e.nx, F = 1 + nx;
  const int nb = (nx + 3) >> 2;
  const int nxp = ZERO ? ((nx + 15) & ~15) : net.nxp;
  const bool TERM = a.flags & DPI_TERMINAL, INTG = a.flags & DPI_INTEGRAL;
  const float* txr = a.tx + (size_t)i * F;
  const float t = txr[0];
  const float tmt = e.T - t;
  const float g_x = a.gx[i], f_b = a.fb[i];
  const float Kf = (float)a.K;

  for (int d = tid; d < nxp; d += NTH) sh.xsh[d] = d < nx ? txr[1 + d] : 0.f;
  const int nxpz = (nxp + 31) & ~31;  // the split MLP reads 32-row chunks
  for (int idx = tid; idx < (nxpz - 4 * nb) * P; idx += NTH) {  // zero pad rows of the noise tile
    const int d = 4 * nb + idx / P, p = idx % P;
    sh.S[d * SS + p] = 0.f;
  }
  if (!ZERO) {
    for (int h = tid; h < H; h += NTH) {
      sh.vec[h] = a.bx[(size_t)i * H + h];  // b1 + W1x x (from k_baseline)
      sh.vec[H + h] = net.w1t[h];
      sh.vec[2 * H + h] = net.wout[h];
      sh.vec[3 * H + h] = net.c1[h];
    }
    for (int l = 1; l < L; ++l)
      for (int h = tid; h < H; h += NTH) sh.bh[l * H + h] = net.b[l][h];
  }
  if constexpr (GBM) {
    if (!ZERO) {  // all weights resident for the tangent sweep
      constexpr int WXS = LdsGbm<H>::WXS, WHS = LdsGbm<H>::WHS;
      for (int idx = tid; idx < H * nxp; idx += NTH) {
        const int h = idx / nxp, d = idx - h * nxp;
        sh.W1x[h * WXS + d] = net.W1x[idx];
      }
      for (int l = 1; l < L; ++l)
        for (int idx = tid; idx < H * H; idx += NTH) {
          const int h = idx / H, k = idx - h * H;
          sh.Wh[l - 1][h * WHS + k] = net.W[l][idx];
        }
    }
    for (int d = tid; d < nxp; d += NTH) sh.hb[d] = d < nx ? a.hb[(size_t)i * NXP_MAX + d] : 0.f;
    for (int idx = tid; idx < nxp * P / 4; idx += NTH) reinterpret_cast<uint32_t*>(sh.cnt)[idx] = 0u;
    if (wv == 0) {  // w_k . x for this point
#pragma unroll
      for (int c = 0; c < NSG; ++c) {
        float v = 0.f;
        if (c < e.nodes)
          for (int d = lane; d < nx; d += 64) v = fmaf(e.gw[c * F + 1 + d], txr[1 + d], v);
        v = wave_sum(v);
        if (lane == 0) sh.wx[c] = v;
      }
    }
  }
  // s ~ U(t, T] for this lane's path (data.py:359); integral/terminal step multipliers
  const float U = u01_oc(philox4x32_10(0u, m, ig, a.c3s, a.k0, a.k1).x);
  // Hessian labels: s = U (T - t) + t + 1e-4 (data.py:848) and Y without the first-order
  // terminal estimator's extra 1/sqrt(alpha) (data.py:1175-1178, :851-864)
  const float smt = U * tmt + (HESS ? 1e-4f : 0.f);  // not s - t: that rounds to 0 in fp32 for U < ulp(t) / tmt
  const float s = HESS ? t + smt : fmaf(U, tmt, t);
  const float ya = HESS ? 1.f : e.asq;
  const float cI = e.asq * sqrtf(smt / Kf);            // X_s = x + cI * sum_k xi_k
  const float yI = 1.0f / (sqrtf(Kf * smt) * ya);      // Y_s = yI * sum_k xi_k   (data.py:520)
  const float cT = e.asq * sqrtf(tmt / Kf);
  const float yT = 1.0f / (sqrtf(Kf * tmt) * ya);      // Y_T (data.py:917)
  if (wv == 0) {
    sh.tau[lane] = s;
    sh.cmul[lane] = cI;
  }
  __syncthreads();  // xsh ready

  // ---------------- phase 1: K-step Euler–Maruyama rollouts
  float ST[8][4];
  float gst[NSG], fst[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) gst[c] = fst[c] = 0.f;
  if constexpr (GBM) {
    // SDGD indices (data.py:497-502): v draws in [0, nx) with replacement -> histogram cnt[d][path]
    if (INTG && wv == 1) {  // one wave owns the histogram (wave 1 has 12 rollout blocks, not 13)
      if (e.sdgd_v > 0) {
        for (int q0 = 0; q0 < e.sdgd_v; q0 += 4) {
          const u32x4 w = philox4x32_10((uint32_t)(q0 >> 2), m, ig, a.c3q, a.k0, a.k1);
          const uint32_t ws4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (q0 + r < e.sdgd_v) {
              const int idx = (int)(((uint64_t)ws4[r] * (uint32_t)nx) >> 32);
              sh.cnt[idx * P + lane] += 1;
            }
        }
      } else {
        for (int d = 0; d < nx; ++d) sh.cnt[d * P + lane] = 1;  // exact diagonal: every d once
      }
    }
  }
  auto terminal_rollout = [&]() {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = wv + 4 * c;  // terminal dim-blocks of this wave
      ST[c][0] = ST[c][1] = ST[c][2] = ST[c][3] = 0.f;
      if (TERM && j < nb) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        for (int k = 0; k < a.K; ++k) {
          const f4 z = normals4_raw(philox4x32_10((uint32_t)(k * nb + j), m, ig, a.c3t, a.k0, a.k1));
          s0 += z.a;
          s1 += z.b;
          s2 += z.c;
          s3 += z.d;
        }
        ST[c][0] = s0 * BM_SCALE;
        ST[c][1] = s1 * BM_SCALE;
        ST[c][2] = s2 * BM_SCALE;
        ST[c][3] = s3 * BM_SCALE;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = 4 * j + q;
          if (d < nx) Eq<KIND>::gstat(e, d, fmaf(cT, ST[c][q], sh.xsh[d]), gst);
        }
      }
    }
  };
  auto integral_rollout = [&]() {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = (3 - wv) + 4 * c;  // integral dim-blocks of this wave (balances 13/12/12/13)
      if (j < nb) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        if (INTG) {
          for (int k = 0; k < a.K; ++k) {
            const f4 z = normals4_raw(philox4x32_10((uint32_t)(k * nb + j), m, ig, a.c3i, a.k0, a.k1));
            s0 += z.a;
            s1 += z.b;
            s2 += z.c;
            s3 += z.d;
          }
        }
        const float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = 4 * j + q;
          sh.S[d * SS + lane] = d < nx ? sv[q] : 0.f;
          if constexpr (GBM) {  // w_k . S for the exact-solution terms at X_s = x + cI S
            if (d < nx) {
#pragma unroll
              for (int c = 0; c < NSG; ++c)
                if (c < e.nodes) fst[c] = fmaf(e.gw[c * F + 1 + d], sv[q], fst[c]);
            }
          }
        }
      }
    }
  };
  // g(X_T) statistics over the 4 waves in fixed order; the barrier also publishes S / fst
  auto terminal_finish = [&]() -> float {
#pragma unroll
    for (int c = 0; c < NSG; ++c) sh.gst[(wv * P + lane) * NSG + c] = gst[c];
    if constexpr (GBM) {
#pragma unroll
      for (int c = 0; c < NSG; ++c) sh.fst[(wv * P + lane) * NSG + c] = fst[c];
    }
    __syncthreads();
    float gT = 0.f;
    if (TERM) {
#pragma unroll
      for (int c = 0; c < NSG; ++c)
        gst[c] = ((sh.gst[(0 * P + lane) * NSG + c] + sh.gst[(1 * P + lane) * NSG + c]) +
                  sh.gst[(2 * P + lane) * NSG + c]) + sh.gst[(3 * P + lane) * NSG + c];
      gT = Eq<KIND>::gfin(e, gst);
    }
    return TERM ? gT - g_x : 0.f;  // (g(X_T) - g(x)) (data.py:923)
  };

  // ---------------- phase 2: u, grad u (or the SDGD Hessian diagonal) at (s, X_s) and f -> bsh
  auto integrand = [&]() {
    if constexpr (!GBM) {
      float u = 0.f, gs = 0.f, gA = 0.f, gB = 0.f;
      if (!ZERO && INTG) {
        if constexpr (SPLIT)
          mlp_tile_split<KIND, H, L>(e, net, sh, u, gs, gA, gB);
        else
          mlp_tile<KIND, H, L>(e, net, sh, nxp / 16, u, gs, gA, gB, nullptr, 0, P);
      }
      const int pp = 16 * wv + (lane & 15);
      if ((lane >> 4) == 0) sh.bsh[pp] = INTG ? tmt * (Eq<KIND>::ffv(e, u, gs, gA, gB) - f_b) : 0.f;
    } else {
      // ffi (equations.py:457-466) with u_ii from SDGD (data.py:1273-1303); the baseline f_b
      // gathers the point's Hessian diagonal at this path's indices (data.py:1293-1302).
      const int jj = lane & 15, qq = lane >> 4, pp = 16 * wv + jj;
      float s1 = 0.f, s2 = 0.f;
      if (!ZERO && INTG) mlp_hdiag<H, L>(e, net, sh, nxp / 16, s1, s2);
      const float vv = (float)(e.sdgd_v > 0 ? e.sdgd_v : nx);
      const float c1 = 0.5f * (1.0f - e.alpha) * (float)nx / vv, c2 = 0.25f * (float)nx / vv;
      float arg[NSG], sn[NSG];
      const float spp = sh.tau[pp], cpp = sh.cmul[pp];
#pragma unroll
      for (int c = 0; c < NSG; ++c) {
        arg[c] = 0.f;
        if (c < e.nodes) {
          const float ws = ((sh.fst[(0 * P + pp) * NSG + c] + sh.fst[(1 * P + pp) * NSG + c]) +
                            sh.fst[(2 * P + pp) * NSG + c]) + sh.fst[(3 * P + pp) * NSG + c];
          arg[c] = fmaf(e.gw[c * F], spp, fmaf(cpp, ws, sh.wx[c]));
        }
        sn[c] = __sinf(arg[c]);
      }
      const float ah = qsum(Eq<KIND>::abs_hess_partial(e, sn, qq, 4));
      float b1 = 0.f, b2 = 0.f;  // baseline Hessian diagonal gathered at this path's indices
      for (int d = qq; d < nx; d += 4) {
        const float c = (float)sh.cnt[d * P + pp], h = sh.hb[d];
        b1 = fmaf(c, h, b1);
        b2 = fmaf(c, fabsf(h), b2);
      }
      b1 = qsum(b1);
      b2 = qsum(b2);
      const float f = c1 * s1 + c2 * s2 + Eq<KIND>::exact_scalar_terms(e, arg) - 0.25f * ah;
      const float fbp = f_b + c1 * b1 + c2 * b2;
      if (qq == 0) {
        sh.bsh[pp] = INTG ? tmt * (f - fbp) : 0.f;
        sh.fbp[pp] = fbp;
      }
    }
  };

  // Phase order.  Two workgroups share a CU; if both run their MFMA phase at the same time the
  // matrix pipe idles during the (longer) VALU rollouts.  Workgroups on the "terminal last"
  // order run the MLP between the integral and the terminal rollout, so a co-resident pair in
  // opposite orders overlaps one's MFMA phase with the other's VALU phase.  The results do not
  // depend on the order (same counters, same per-lane arithmetic).
  bool tlast = false;
  if constexpr (SPLIT) {
    tlast = true;  // measured faster, and the terminal sums are not live across the MLP (no spills)
  } else if constexpr (!GBM) {
    if (a.order == 1) tlast = (__builtin_amdgcn_s_getreg((3 << 11) | (16 << 6) | 4) & 1) != 0;  // HW_ID.TG_ID
    else if (a.order == 2) tlast = (blockIdx.x & 1) != 0;
    else if (a.order == 3) tlast = ((blockIdx.x >> 8) & 1) != 0;
    else if (a.order == 4) tlast = true;
  }
  float ap;
  if (!tlast) {
    terminal_rollout();
    integral_rollout();
    ap = terminal_finish();
    integrand();
    __syncthreads();
  } else {
    integral_rollout();
    __syncthreads();
    integrand();
    terminal_rollout();
    ap = terminal_finish();  // its barrier also publishes bsh
  }

  // ---------------- phase 3: per-path contributions -> per-block partial slab
  const float bp = sh.bsh[lane];
  // partial slab layout [point][2F][block]: the reduce kernel reads each column's blocks contiguously
  float* out = a.partial + (size_t)i * 2 * F * a.nbp + blk;
  const int nbs = a.nbp;
  // per-block sums of c and c^2 for this wave's columns: 2 per owned dim (d = 4 (wv + 4c) + q,
  // column 8c + 2q + {0: sum, 1: sum of squares}) and, on wave 0, the value column (56, 57)
  const float aY = ap * yT, bY = bp * yI;
  float col[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) col[c] = 0.f;
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    const int j = wv + 4 * c;
    if (j < nb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * j + q;
        const float v = d < nx ? fmaf(aY, ST[c][q], bY * sh.S[d * SS + lane]) : 0.f;
        col[8 * c + 2 * q] = v;
        col[8 * c + 2 * q + 1] = v * v;
      }
    }
  }
  if (wv == 0) {
    float fbt;
    if constexpr (GBM)
      fbt = sh.fbp[lane];
    else
      fbt = f_b + Eq<KIND>::ffc(e);
    const float c0 = ap + bp + (INTG ? fbt * tmt : 0.f);
    col[56] = c0;
    col[57] = c0 * c0;
  }
  const float tot = column_sums64(col);
  {
    const int c = lane >> 3, q = (lane >> 1) & 3, sq = lane & 1;
    const int d = 4 * (wv + 4 * c) + q;
    if (lane < 56) {
      if (wv + 4 * c < nb && d < nx) out[(size_t)(sq * F + 1 + d) * nbs] = tot;
    } else if (wv == 0 && lane < 58) {
      out[(size_t)(sq * F) * nbs] = tot;
    }
  }
  if (wv + 28 < nb) {  // nx > 112: the eighth dim-block of this wave, one column at a time
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 4 * (wv + 28) + q;
      if (d < nx) {
        const float v = fmaf(aY, ST[7][q], bY * sh.S[d * SS + lane]);
        const float s1 = wave_sum(v), s2 = wave_sum(v * v);
        if (lane == 0) {
          out[(size_t)(1 + d) * nbs] = s1;
          out[(size_t)(F + 1 + d) * nbs] = s2;
        }
      }
    }
  }
  if constexpr (HESS) hess_block<KIND, H, L, ZERO>(e, net, a, sh, i, blk, ig, m, s, smt, tmt, g_x, nxp);
}

// Canonical fixed-order sum of `cnt` values (stride `stride`): zero-pad to a power of two
// P2 >= 64 and add as a perfect binary tree in index order.  One wave per column: each lane
// first sums its q = P2/64 consecutive values pairwise in registers, then the 64 lane values
// are combined by an xor butterfly, whose every level adds aligned neighbours — the same tree.
// Splitting the values over G ranks (G and cnt powers of two) and combining the rank results
// with the same function therefore reproduces the single-call sum bit for bit.
__device__ __forceinline__ float tree_sum(const float* __restrict__ p, int cnt, size_t stride) {
  const int lane = threadIdx.x & 63;
  int p2 = 64;
  while (p2 < cnt) p2 <<= 1;
  const int q = p2 >> 6;  // values per lane (<= 16)
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int b = lane * q + j;
    v[j] = (j < q && b < cnt) ? p[(size_t)b * stride] : 0.f;
  }
#pragma unroll
  for (int w = 1; w < 16; w <<= 1)
#pragma unroll
    for (int j = 0; j < 16; j += 2 * w)
      if (j + w < q) v[j] = v[j] + v[j + w];
  float s = v[0];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float other = __shfl_xor(s, o, 64);
    s = (lane & o) ? other + s : s + other;  // always (left + right): identical on both lanes
  }
  return s;
}

// partial [n][2F][nbp] -> moments [n][2F] (and, if y != nullptr, the finalized labels).
__global__ __launch_bounds__(256) void k_reduce(const float* __restrict__ partial, int n, int F, int nbp,
                                                float* __restrict__ moments, const float* __restrict__ gx,
                                                float invM, int add_g, float bound, float* __restrict__ y,
                                                int ystride) {
  const int i = blockIdx.x;
  const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (c >= 2 * F) return;
  const float s = tree_sum(partial + ((size_t)i * 2 * F + c) * nbp, nbp, 1);
  if ((threadIdx.x & 63) == 0) {
    moments[(size_t)i * 2 * F + c] = s;
    if (y && c < F) {
      float v = s * invM;
      if (c == 0 && add_g) v += gx[i];
      y[(size_t)i * ystride + c] = fminf(fmaxf(v, -bound), bound);
    }
  }
}

// Hessian block sums [n][nbp][C] -> y[:, off:off+C] = clip(sum / M): one wave per (point, column),
// the canonical tree over blocks.
__global__ __launch_bounds__(256) void k_reduce_hess(const float* __restrict__ hpart, int n, int C, int nbp,
                                                     float* __restrict__ hsum, float invM, float bound,
                                                     float* __restrict__ y, int ystride, int yoff) {
  const int i = blockIdx.y;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const float s = tree_sum(hpart + (size_t)i * nbp * C + c, nbp, (size_t)C);
  if ((threadIdx.x & 63) == 0) {
    if (hsum) hsum[(size_t)i * C + c] = s;
    if (y) y[(size_t)i * ystride + yoff + c] = fminf(fmaxf(s * invM, -bound), bound);
  }
}

// Hessian sums (n, C) -> y[:, off:off+C] = clip(sum / M)
__global__ void k_finalize_hess(const float* __restrict__ hsum, int n, int C, float invM, float bound,
                                float* __restrict__ y, int ystride, int yoff) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)n * C) return;
  const size_t i = gid / C, c = gid - i * C;
  y[i * ystride + yoff + c] = fminf(fmaxf(hsum[gid] * invM, -bound), bound);
}

// parts [G][len] -> out [len]
__global__ __launch_bounds__(256) void k_reduce_parts(const float* __restrict__ parts, int G, int len,
                                                      float* __restrict__ out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= len) return;
  const float s = tree_sum(parts + c, G, (size_t)len);
  if ((threadIdx.x & 63) == 0) out[c] = s;
}

__global__ void k_finalize_y(const float* moments, const float* gx, int n, int F, float invM, int add_g,
                             float bound, float* y, int ystride) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * F) return;
  const int i = gid / F, c = gid - i * F;
  float v = moments[(size_t)i * 2 * F + c] * invM;
  if (c == 0 && add_g) v += gx[i];
  y[(size_t)i * ystride + c] = fminf(fmaxf(v, -bound), bound);
}

__global__ void k_finalize(const float* moments, const float* gx, int n, int F, float invM, int add_g, float bound,
                           float* y) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * F) return;
  const int i = gid / F, c = gid - i * F;
  float v = moments[(size_t)i * 2 * F + c] * invM;
  if (c == 0 && add_g) v += gx[i];
  y[gid] = fminf(fmaxf(v, -bound), bound);
}

}  // namespace dpi

// ================================================================================ C-ABI
using namespace dpi;

struct dpi_problem_s {
  EqDev e;
  float alpha_init_sqrt;
  std::vector<void*> dev;
};

struct dpi_net_s {
  NetDev d;        // d.kind: 0 zero, 1 mlp, 2 PISGradNet
  NetPisDev pis;
  void* blob = nullptr;
  int n_in = 0;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t _e = (x);                                                                             \
    if (_e != hipSuccess) return fail(DPI_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename T>
static int upload(dpi_problem_s* p, const std::vector<T>& v, const T** out) {
  void* d = nullptr;
  HIPCHK(hipMalloc(&d, v.size() * sizeof(T) + 16));
  HIPCHK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  p->dev.push_back(d);
  *out = reinterpret_cast<const T*>(d);
  return 0;
}

// Append an R x C (C % 32 == 0) matrix in the fp16-split fragment order of mlp_tile_split:
// row r, chunk u, lane group q: 8 hi halves then 8 lo halves of columns 32u + 4q + (j & 3) + 16 (j >> 2).
// Returns the offset (in 4-byte words) into `blob`.
template <class F>
static size_t pack_split(std::vector<float>& blob, int R, int C, F at) {
  const size_t off = blob.size();
  blob.resize(off + (size_t)R * C, 0.f);
  _Float16* dst = reinterpret_cast<_Float16*>(blob.data() + off);
  for (int r = 0; r < R; ++r)
    for (int u = 0; u < C / 32; ++u)
      for (int q = 0; q < 4; ++q) {
        _Float16* g = dst + ((size_t)r * C + 32 * u + 8 * q) * 2;  // 16 halves = 8 words
        for (int j = 0; j < 8; ++j) {
          const float x = at(r, 32 * u + 4 * q + (j & 3) + 16 * (j >> 2));
          const _Float16 h = (_Float16)x;
          g[j] = h;
          g[8 + j] = (_Float16)((x - (float)h) * 2048.0f);
        }
      }
  return off;
}

extern "C" {

int dpi_abi_version(void) { return DPI_ABI_VERSION; }

int dpi_last_error(char* buf, size_t len) {
  if (buf && len) {
    std::strncpy(buf, g_err.c_str(), len - 1);
    buf[len - 1] = 0;
  }
  return (int)g_err.size();
}

int dpi_problem_destroy(dpi_problem p);

static dpi_problem_s* new_problem(int kind, int nx, double alpha, double T) {
  auto* p = new dpi_problem_s();
  std::memset(&p->e, 0, sizeof(p->e));
  p->e.kind = kind;
  p->e.nx = nx;
  p->e.T = (float)T;
  p->e.alpha = (float)alpha;
  p->e.asq = (float)std::sqrt(alpha);
  p->alpha_init_sqrt = 0.f;
  return p;
}

int dpi_problem_create_cha(int nx, double alpha, double k, double T, dpi_problem* out) {
  if (!out || nx < 1 || nx > NXP_MAX || !(alpha > 0)) return fail(DPI_ERR_ARG, "cha: bad arguments");
  auto* p = new_problem(DPI_EQ_CHA, nx, alpha, T);
  const double kp = k / std::sqrt((double)nx);  // equations.py:285
  const double k_alpha_d = kp * alpha * nx;
  p->e.cha_k = (float)kp;
  p->e.cha_C = (float)((2.0 + kp * k_alpha_d) / (2.0 * k_alpha_d));
  *out = p;
  return 0;
}

int dpi_problem_create_ou(int nx, double alpha, double T, double theta, double mu, double alpha_scale, int n_comp,
                          const double* mean, const double* var_diag, const double* pi, dpi_problem* out) {
  if (!out || nx < 1 || nx > NXP_MAX || n_comp < 1 || n_comp > NSG || !mean || !var_diag || !pi)
    return fail(DPI_ERR_ARG, "ou: bad arguments (1 <= n_comp <= 8, nx <= 128)");
  auto* p = new_problem(DPI_EQ_OU, nx, alpha, T);
  p->e.ou_theta = (float)theta;
  p->e.ou_mu = (float)mu;
  p->e.ou_d = (float)nx;
  p->e.ncomp = n_comp;
  p->alpha_init_sqrt = (float)std::sqrt(alpha_scale * alpha);
  std::vector<float> m(n_comp * nx), iv(n_comp * nx), lc(n_comp);
  const double log2pi = std::log(2.0 * M_PI);
  for (int c = 0; c < n_comp; ++c) {
    double logdet = 0;
    for (int d = 0; d < nx; ++d) {
      m[c * nx + d] = (float)mean[c * nx + d];
      iv[c * nx + d] = (float)(1.0 / var_diag[c * nx + d]);
      logdet += std::log(var_diag[c * nx + d]);
    }
    lc[c] = (float)(std::log(pi[c]) - 0.5 * (nx * log2pi + logdet));
  }
  int rc;
  if ((rc = upload(p, m, &p->e.mean)) || (rc = upload(p, iv, &p->e.ivar)) || (rc = upload(p, lc, &p->e.logc))) {
    delete p;
    return rc;
  }
  *out = p;
  return 0;
}

int dpi_problem_create_gbm(int nx, double alpha, double T, int n_nodes, const double* w, const double* v,
                           dpi_problem* out) {
  if (!out || nx < 1 || nx > NXP_MAX || n_nodes < 1 || n_nodes > NSG || !w || !v)
    return fail(DPI_ERR_ARG, "gbm: bad arguments (1 <= n_nodes <= 8, nx <= 128)");
  auto* p = new_problem(DPI_EQ_GBM, nx, alpha, T);
  p->e.nodes = n_nodes;
  const int F = 1 + nx;
  std::vector<float> gw((size_t)n_nodes * F), gv(n_nodes), wsq(n_nodes), wv2((size_t)n_nodes * nx);
  for (int c = 0; c < n_nodes; ++c) {
    double sq = 0;
    for (int d = 0; d < F; ++d) gw[(size_t)c * F + d] = (float)w[(size_t)c * F + d];
    for (int d = 0; d < nx; ++d) {
      const double wd = w[(size_t)c * F + 1 + d];
      sq += wd * wd;
      wv2[(size_t)c * nx + d] = (float)(v[c] * wd * wd);
    }
    gv[c] = (float)v[c];
    wsq[c] = (float)sq;
  }
  int rc;
  if ((rc = upload(p, gw, &p->e.gw)) || (rc = upload(p, gv, &p->e.gv)) || (rc = upload(p, wsq, &p->e.gwsq)) ||
      (rc = upload(p, wv2, &p->e.gwv2))) {
    dpi_problem_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

int dpi_problem_set_hessian_approximation(dpi_problem p, int sdgd_v) {
  if (!p || sdgd_v < 0 || sdgd_v > 255) return fail(DPI_ERR_ARG, "hessian approximation: 0 <= v <= 255");
  p->e.sdgd_v = sdgd_v;
  return 0;
}

int dpi_problem_destroy(dpi_problem p) {
  if (!p) return 0;
  for (void* d : p->dev) (void)hipFree(d);
  delete p;
  return 0;
}

int dpi_net_create_zero(dpi_net* out) {
  if (!out) return fail(DPI_ERR_ARG, "null out");
  auto* n = new dpi_net_s();
  std::memset(&n->d, 0, sizeof(n->d));
  n->d.kind = 0;
  *out = n;
  return 0;
}

int dpi_net_create_mlp(int n_in, int n_hidden, const int* widths, int act, const float* params, size_t n_params,
                       dpi_net* out) {
  if (!out || !widths || !params || n_in < 2 || n_in - 1 > NXP_MAX || n_hidden < 1 || n_hidden > 4)
    return fail(DPI_ERR_ARG, "mlp: bad arguments");
  if (act != DPI_ACT_ELU) return fail(DPI_ERR_UNSUPPORTED, "mlp: only ELU activations are supported");
  const int H = widths[0];
  for (int l = 1; l < n_hidden; ++l)
    if (widths[l] != H) return fail(DPI_ERR_UNSUPPORTED, "mlp: hidden widths must be equal");
  if (!(H == 16 || H == 32 || H == 64 || H == 128)) return fail(DPI_ERR_UNSUPPORTED, "mlp: width must be 16/32/64/128");
  const int nx = n_in - 1, nxp = (nx + 15) & ~15, L = n_hidden;
  const size_t expect = (size_t)H * n_in + H + (size_t)(L - 1) * (H * H + H) + H + 1;
  if (n_params != expect) return fail(DPI_ERR_ARG, "mlp: parameter count mismatch");
  // host-side repack
  std::vector<float> blob;
  auto take = [&](size_t cnt) {
    size_t off = blob.size();
    blob.resize(off + ((cnt + 3) & ~size_t(3)), 0.f);
    return off;
  };
  const float* W0 = params;
  const float* b0 = W0 + (size_t)H * n_in;
  const size_t oW1x = take((size_t)H * nxp), ow1t = take(H), ob1 = take(H), oc1 = take(H), oW1xT = take((size_t)nxp * H);
  for (int h = 0; h < H; ++h) {
    double cs = 0;
    for (int d = 0; d < nx; ++d) {
      const float w = W0[(size_t)h * n_in + 1 + d];
      blob[oW1x + (size_t)h * nxp + d] = w;
      blob[oW1xT + (size_t)d * H + h] = w;
      cs += w;
    }
    blob[ow1t + h] = W0[(size_t)h * n_in];
    blob[ob1 + h] = b0[h];
    blob[oc1 + h] = (float)cs;
  }
  const float* cur = b0 + H;
  size_t oW[4] = {0}, oWT[4] = {0}, ob[4] = {0};
  for (int l = 1; l < L; ++l) {
    oW[l] = take((size_t)H * H);
    oWT[l] = take((size_t)H * H);
    ob[l] = take(H);
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < H; ++c) {
        blob[oW[l] + (size_t)r * H + c] = cur[(size_t)r * H + c];
        blob[oWT[l] + (size_t)c * H + r] = cur[(size_t)r * H + c];
      }
    cur += (size_t)H * H;
    for (int h = 0; h < H; ++h) blob[ob[l] + h] = cur[h];
    cur += H;
  }
  const size_t owout = take(H);
  for (int h = 0; h < H; ++h) blob[owout + h] = cur[h];
  const float bout = cur[H];
  // fp16-split copies for the split MFMA path (H % 32 == 0)
  const int nxp32 = (nx + 31) & ~31;
  size_t oW1xS = 0, oW1xTS = 0, oWS[4] = {0}, oWTS[4] = {0};
  if (H % 32 == 0) {
    auto Wx = [&](int h, int d) { return d < nx ? W0[(size_t)h * n_in + 1 + d] : 0.f; };
    oW1xS = pack_split(blob, H, nxp32, Wx);
    oW1xTS = pack_split(blob, nxp32, H, [&](int d, int h) { return Wx(h, d); });
    for (int l = 1; l < L; ++l) {
      const float* Wl = blob.data() + oW[l];
      std::vector<float> Wc(Wl, Wl + (size_t)H * H);
      oWS[l] = pack_split(blob, H, H, [&](int r, int c) { return Wc[(size_t)r * H + c]; });
      oWTS[l] = pack_split(blob, H, H, [&](int r, int c) { return Wc[(size_t)c * H + r]; });
    }
  }
  auto* n = new dpi_net_s();
  std::memset(&n->d, 0, sizeof(n->d));
  void* d = nullptr;
  if (hipMalloc(&d, blob.size() * sizeof(float)) != hipSuccess) {
    delete n;
    return fail(DPI_ERR_HIP, "mlp: hipMalloc failed");
  }
  if (hipMemcpy(d, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    delete n;
    return fail(DPI_ERR_HIP, "mlp: hipMemcpy failed");
  }
  const float* base = reinterpret_cast<const float*>(d);
  n->blob = d;
  n->n_in = n_in;
  n->d.kind = 1;
  n->d.H = H;
  n->d.L = L;
  n->d.nxp = nxp;
  n->d.W1x = base + oW1x;
  n->d.w1t = base + ow1t;
  n->d.b1 = base + ob1;
  n->d.c1 = base + oc1;
  n->d.W1xT = base + oW1xT;
  for (int l = 1; l < L; ++l) {
    n->d.W[l] = base + oW[l];
    n->d.WT[l] = base + oWT[l];
    n->d.b[l] = base + ob[l];
  }
  n->d.wout = base + owout;
  n->d.bout = bout;
  n->d.nxp32 = nxp32;
  if (H % 32 == 0) {
    auto u32 = [&](size_t off) { return reinterpret_cast<const uint32_t*>(base + off); };
    n->d.W1xS = u32(oW1xS);
    n->d.W1xTS = u32(oW1xTS);
    for (int l = 1; l < L; ++l) {
      n->d.WS[l] = u32(oWS[l]);
      n->d.WTS[l] = u32(oWTS[l]);
    }
  }
  *out = n;
  return 0;
}

int dpi_net_create_pisgrad(int nx, int n_hidden, const int* hidden, double T, const float* params, size_t n_params,
                           dpi_net* out) {
  if (!out || !hidden || !params || nx < 1 || nx > NXP_MAX || n_hidden < 1 || n_hidden > 4)
    return fail(DPI_ERR_ARG, "pisgrad: bad arguments (1 <= n_hidden <= 4, nx <= 128)");
  for (int l = 0; l < n_hidden; ++l)
    if (hidden[l] < 4 || hidden[l] > 1024 || (hidden[l] % 4)) return fail(DPI_ERR_ARG, "pisgrad: hidden widths % 4");
  const int C = PIS_CH, nsm = n_hidden, L = n_hidden, IN = C + nx;
  // expected parameter count in state-dict order (solution.py:160-205)
  size_t expect = 2 * C + (size_t)C * 2 * C + C + (size_t)C * C + C;   // phase, coeff, t_encoder
  expect += (size_t)C * 2 * C + C + (size_t)nsm * (C * C + C) + (size_t)nx * C + nx;  // smooth_net
  int in = IN;
  for (int l = 0; l < L; ++l) {
    expect += (size_t)hidden[l] * in + hidden[l];
    in = hidden[l];
  }
  expect += (size_t)nx * in + nx;
  if (n_params != expect) return fail(DPI_ERR_ARG, "pisgrad: parameter count mismatch");
  const float* q = params;
  auto take_src = [&](size_t cnt) {
    const float* r = q;
    q += cnt;
    return r;
  };
  std::vector<float> blob;
  auto put = [&](const float* src, size_t cnt) {
    size_t off = blob.size();
    blob.resize(off + ((cnt + 3) & ~size_t(3)), 0.f);
    std::memcpy(blob.data() + off, src, cnt * sizeof(float));
    return off;
  };
  auto putT = [&](const float* src, int rows, int cols, int c0, int nc) {  // (src[:, c0:c0+nc])^T
    size_t off = blob.size();
    blob.resize(off + (((size_t)nc * rows + 3) & ~size_t(3)), 0.f);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < nc; ++c) blob[off + (size_t)c * rows + r] = src[(size_t)r * cols + c0 + c];
    return off;
  };
  const float* phase = take_src(C);
  const float* coeff = take_src(C);
  const float* te0 = take_src((size_t)C * 2 * C);
  const float* te0b = take_src(C);
  const float* te2 = take_src((size_t)C * C);
  const float* te2b = take_src(C);
  const float* sn0 = take_src((size_t)C * 2 * C);
  const float* sn0b = take_src(C);
  const float *snw[4], *snbw[4];
  for (int j = 0; j < nsm; ++j) {
    snw[j] = take_src((size_t)C * C);
    snbw[j] = take_src(C);
  }
  const float* snl = take_src((size_t)nx * C);
  const float* snlb = take_src(nx);
  const float *nnw[5], *nnbw[5];
  int ins[5];
  in = IN;
  for (int l = 0; l <= L; ++l) {
    const int o = l < L ? hidden[l] : nx;
    nnw[l] = take_src((size_t)o * in);
    nnbw[l] = take_src(o);
    ins[l] = in;
    in = o;
  }
  // smooth0 = smooth_net(emb(0))[0] in double on the host
  double smooth0;
  {
    std::vector<double> e(2 * C), h(C), h2(C);
    for (int j = 0; j < C; ++j) {
      e[j] = std::sin((double)phase[j]);
      e[C + j] = std::cos((double)phase[j]);
    }
    auto elu_d = [](double z) { return z > 0 ? z : std::expm1(z); };
    for (int o = 0; o < C; ++o) {
      double a = sn0b[o];
      for (int k = 0; k < 2 * C; ++k) a += (double)sn0[(size_t)o * 2 * C + k] * e[k];
      h[o] = a;
    }
    for (int j = 0; j < nsm; ++j) {
      for (int o = 0; o < C; ++o) {
        double a = snbw[j][o];
        for (int k = 0; k < C; ++k) a += (double)snw[j][(size_t)o * C + k] * elu_d(h[k]);
        h2[o] = a;
      }
      h.swap(h2);
    }
    double a = snlb[0];
    for (int k = 0; k < C; ++k) a += (double)snl[k] * elu_d(h[k]);
    smooth0 = a;
  }
  NetPisDev pd;
  std::memset(&pd, 0, sizeof(pd));
  size_t o_phase = put(phase, C), o_coeff = put(coeff, C), o_te0 = put(te0, (size_t)C * 2 * C), o_te0b = put(te0b, C),
         o_te2 = put(te2, (size_t)C * C), o_te2b = put(te2b, C), o_sn0 = put(sn0, (size_t)C * 2 * C),
         o_sn0b = put(sn0b, C), o_snl = put(snl, C), o_snlb = put(snlb, 1);
  size_t o_sn[4], o_snb[4], o_nn[5], o_nnb[5], o_nnT[5];
  for (int j = 0; j < nsm; ++j) {
    o_sn[j] = put(snw[j], (size_t)C * C);
    o_snb[j] = put(snbw[j], C);
  }
  for (int l = 0; l <= L; ++l) {
    const int o = l < L ? hidden[l] : nx;
    o_nn[l] = put(nnw[l], (size_t)o * ins[l]);
    o_nnb[l] = put(nnbw[l], o);
    o_nnT[l] = l == 0 ? putT(nnw[0], hidden[0], ins[0], C, nx) : putT(nnw[l], o, ins[l], 0, ins[l]);
  }
  auto* n = new dpi_net_s();
  std::memset(&n->d, 0, sizeof(n->d));
  void* d = nullptr;
  if (hipMalloc(&d, blob.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(d, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    if (d) (void)hipFree(d);
    delete n;
    return fail(DPI_ERR_HIP, "pisgrad: device upload failed");
  }
  const float* base = reinterpret_cast<const float*>(d);
  pd.nx = nx;
  pd.L = L;
  pd.nsm = nsm;
  for (int l = 0; l < L; ++l) pd.h[l] = hidden[l];
  pd.T = (float)T;
  pd.smooth0 = (float)smooth0;
  pd.phase = base + o_phase;
  pd.coeff = base + o_coeff;
  pd.te0 = base + o_te0;
  pd.te0b = base + o_te0b;
  pd.te2 = base + o_te2;
  pd.te2b = base + o_te2b;
  pd.sn0 = base + o_sn0;
  pd.sn0b = base + o_sn0b;
  for (int j = 0; j < nsm; ++j) {
    pd.sn[j] = base + o_sn[j];
    pd.snb[j] = base + o_snb[j];
  }
  pd.snlast = base + o_snl;
  pd.snlastb = base + o_snlb;
  for (int l = 0; l <= L; ++l) {
    pd.nn[l] = base + o_nn[l];
    pd.nnb[l] = base + o_nnb[l];
    pd.nnT[l] = base + o_nnT[l];
  }
  n->blob = d;
  n->n_in = 1 + nx;
  n->d.kind = 2;
  n->pis = pd;
  *out = n;
  return 0;
}

int dpi_net_destroy(dpi_net net) {
  if (!net) return 0;
  if (net->blob) (void)hipFree(net->blob);
  delete net;
  return 0;
}

}  // extern "C"

// PISGradNet pipeline rows (floats per path) and chunking
static PisRows pis_rows_layout(const NetPisDev& pd) {
  auto r4 = [](int x) { return (x + 3) & ~3; };
  int hmax = 0;
  for (int l = 0; l < pd.L; ++l) hmax = std::max(hmax, pd.h[l]);
  PisRows L;
  int o = 0;
  L.E = o;
  o += 2 * PIS_CH;
  L.T1 = o;
  o += PIS_CH;
  L.IN = o;
  o += r4(PIS_CH + pd.nx);
  L.H0 = o;
  o += PIS_CH;
  L.H1 = o;
  o += PIS_CH;
  for (int l = 0; l < 4; ++l) {
    L.A[l] = o;
    o += l < pd.L ? r4(pd.h[l]) : 0;
  }
  L.NO = o;
  o += r4(pd.nx);
  L.D0 = o;
  o += r4(hmax);
  L.D1 = o;
  o += r4(hmax);
  L.GX = o;
  o += r4(pd.nx);
  L.SS = o;
  o += r4(pd.nx);
  L.ST = o;
  o += r4(pd.nx);
  L.SC = o;
  o += 4;
  L.stride = o;
  return L;
}
constexpr int PIS_CHUNK_WG = 512;  // (point, 64-path block) pairs per pipeline chunk = 32,768 rows

// Workspace: gx[n] | fb[n] | bx[n][H] | hb[n][128] | [PIS rows] | partial[n][2F][nbp]  (256-B aligned)
struct WsLayout {
  size_t gx, fb, bx, hb, rows, partial, total;
  int rows_cap;
};
static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
static WsLayout ws_layout(dpi_net net, int n, int M, int F) {
  WsLayout w;
  const int H = (net && net->d.kind == 1) ? net->d.H : 0;
  const size_t nbp = (size_t)(M + P - 1) / P;
  w.gx = 0;
  w.fb = al256((size_t)n * 4);
  w.bx = w.fb + al256((size_t)n * 4);
  w.hb = w.bx + al256((size_t)n * H * 4);
  w.rows = w.hb + al256((size_t)n * NXP_MAX * 4);
  w.rows_cap = 0;
  size_t rows_bytes = 0;
  if (net && net->d.kind == 2) {
    const size_t need = std::max((size_t)n, (size_t)n * nbp * P);
    w.rows_cap = (int)std::min(need, (size_t)PIS_CHUNK_WG * P);
    w.rows_cap = std::max(w.rows_cap, (int)std::min((size_t)n, (size_t)PIS_CHUNK_WG * P));
    rows_bytes = al256((size_t)w.rows_cap * pis_rows_layout(net->pis).stride * 4);
  }
  w.partial = w.rows + rows_bytes;
  w.total = w.partial + (size_t)n * nbp * 2 * F * 4;
  return w;
}

// GEMM precision: exact-fp32 MFMA by default; DPI_GEMM=f16x3 selects the fp16-split kernel
// (same speed today: both are load-latency bound).
static int g_gemm_mode = -1;  // -1: from the environment; DPI_GEMM_* of include/dpi.h
static int gemm_mode() {
  if (g_gemm_mode < 0) {
    const char* e = std::getenv("DPI_GEMM");
    g_gemm_mode = !e ? DPI_GEMM_AUTO : std::strcmp(e, "f16x3") == 0 ? DPI_GEMM_F16X3
                                   : std::strcmp(e, "f32") == 0   ? DPI_GEMM_F32
                                                                  : DPI_GEMM_AUTO;
  }
  return g_gemm_mode;
}
static bool gemm_f32() { return gemm_mode() != DPI_GEMM_F16X3; }  // PISGradNet GEMM pipeline
static bool mlp_split() { return gemm_mode() != DPI_GEMM_F32; }   // fused MLP of k_paths

extern "C" int dpi_set_gemm_precision(int mode) {
  if (mode != DPI_GEMM_F32 && mode != DPI_GEMM_F16X3 && mode != DPI_GEMM_AUTO)
    return fail(DPI_ERR_ARG, "gemm precision: 0 = fp32, 1 = fp16-split, 2 = auto");
  g_gemm_mode = mode;
  return 0;
}

static void gemm(int epi, int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                 const float* bias, const float* aux, int ldaux, hipStream_t st) {
  dim3 grid((M + GBM_ - 1) / GBM_, (N + GBN_ - 1) / GBN_), block(256);
  if (!gemm_f32()) {
    if (epi == EPI_BIAS)
      hipLaunchKernelGGL(k_gemm_nt_f16x3<EPI_BIAS>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux,
                         ldaux);
    else if (epi == EPI_BIAS_ELU)
      hipLaunchKernelGGL(k_gemm_nt_f16x3<EPI_BIAS_ELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux,
                         ldaux);
    else
      hipLaunchKernelGGL(k_gemm_nt_f16x3<EPI_DELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux,
                         ldaux);
    return;
  }
  if (epi == EPI_BIAS)
    hipLaunchKernelGGL(k_gemm_nt<EPI_BIAS>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
  else if (epi == EPI_BIAS_ELU)
    hipLaunchKernelGGL(k_gemm_nt<EPI_BIAS_ELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
  else
    hipLaunchKernelGGL(k_gemm_nt<EPI_DELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
}

// PISGradNet forward + VJP over R rows (solution.py:256-289); returns the row layout with H0 pointing
// at the last smooth_net activation.
static PisRows pis_chain(const NetPisDev& pd, float* rows, int R, hipStream_t st) {
  PisRows L = pis_rows_layout(pd);
  const int ld = L.stride, C = PIS_CH, nx = pd.nx;
  // t_encoder -> IN[:, 0:64]
  gemm(EPI_BIAS_ELU, R, C, 2 * C, rows + L.E, ld, pd.te0, 2 * C, rows + L.T1, ld, pd.te0b, nullptr, 0, st);
  gemm(EPI_BIAS, R, C, C, rows + L.T1, ld, pd.te2, C, rows + L.IN, ld, pd.te2b, nullptr, 0, st);
  // smooth_net hidden activations (elu applied on store: each is consumed through an ELU)
  int hs = L.H0, ho = L.H1;
  gemm(EPI_BIAS_ELU, R, C, 2 * C, rows + L.E, ld, pd.sn0, 2 * C, rows + hs, ld, pd.sn0b, nullptr, 0, st);
  for (int j = 0; j < pd.nsm; ++j) {
    gemm(EPI_BIAS_ELU, R, C, C, rows + hs, ld, pd.sn[j], C, rows + ho, ld, pd.snb[j], nullptr, 0, st);
    std::swap(hs, ho);
  }
  // nn_module forward
  int in = C + nx;
  const float* a = rows + L.IN;
  for (int l = 0; l < pd.L; ++l) {
    gemm(EPI_BIAS_ELU, R, pd.h[l], in, a, ld, pd.nn[l], in, rows + L.A[l], ld, pd.nnb[l], nullptr, 0, st);
    a = rows + L.A[l];
    in = pd.h[l];
  }
  gemm(EPI_BIAS, R, nx, in, a, ld, pd.nn[pd.L], in, rows + L.NO, ld, pd.nnb[pd.L], nullptr, 0, st);
  // VJP with cotangent X on net_out: D_{L-1} = (X nn_L) * elu'(A_{L-1}), ..., GX = D_0 nn_0[:, 64:]
  int dcur = L.D0, dnext = L.D1;
  gemm(EPI_DELU, R, pd.h[pd.L - 1], nx, rows + L.IN + PIS_IN_OFF, ld, pd.nnT[pd.L], nx, rows + dcur, ld, nullptr,
       rows + L.A[pd.L - 1], ld, st);
  for (int l = pd.L - 1; l >= 1; --l) {
    gemm(EPI_DELU, R, pd.h[l - 1], pd.h[l], rows + dcur, ld, pd.nnT[l], pd.h[l], rows + dnext, ld, nullptr,
         rows + L.A[l - 1], ld, st);
    std::swap(dcur, dnext);
  }
  gemm(EPI_BIAS, R, nx, pd.h[0], rows + dcur, ld, pd.nnT[0], pd.h[0], rows + L.GX, ld, nullptr, nullptr, 0, st);
  L.H0 = hs;
  return L;
}

extern "C" size_t dpi_workspace_bytes(dpi_problem p, dpi_net net, int n, int M) {
  if (!p || n < 0 || M < 0) return 0;
  return ws_layout(net, n, M, 1 + p->e.nx).total;
}

extern "C" int dpi_sample_points(dpi_problem p, int n, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                      float* tx, void* stream) {
  if (!p || !tx || n < 0 || epoch > 0xFFFFFFu) return fail(DPI_ERR_ARG, "sample_points: bad arguments");
  if (n == 0) return 0;
  const int nb = (p->e.nx + 3) >> 2;
  const int total = n * nb;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t c3t = DPI_TAG_T | (epoch << 8), c3x0 = DPI_TAG_X0 | (epoch << 8), c3x = DPI_TAG_X | (epoch << 8);
  dim3 grid((total + 255) / 256), block(256);
  hipStream_t st = (hipStream_t)stream;
  switch (p->e.kind) {
    case DPI_EQ_CHA:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_CHA>, grid, block, 0, st, p->e, n, k0, k1, c3t, c3x0, c3x, point_base,
                         eps, p->alpha_init_sqrt, tx);
      break;
    case DPI_EQ_OU:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_OU>, grid, block, 0, st, p->e, n, k0, k1, c3t, c3x0, c3x, point_base,
                         eps, p->alpha_init_sqrt, tx);
      break;
    case DPI_EQ_GBM:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_GBM>, grid, block, 0, st, p->e, n, k0, k1, c3t, c3x0, c3x, point_base,
                         eps, p->alpha_init_sqrt, tx);
      break;
    default:
      return fail(DPI_ERR_UNSUPPORTED, "sample_points: equation kind");
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// ---- dispatch over (equation, network shape)
struct Launch {
  bool baseline;
  const float* tx;
  int n;
  float *gx, *fb, *bx, *hb;
  const PathArgs* a;
  int nblocks;
  hipStream_t st;
  bool hess = false;  // k_paths in Hessian-label mode (GBM only)
};

template <int KIND, int H, int L, bool Z>
static void do_launch(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  if (q.baseline)
    hipLaunchKernelGGL((k_baseline<KIND, Z>), dim3(q.n), dim3(NTHB), 0, q.st, p->e, net->d, q.tx, q.n, q.gx, q.fb,
                       q.bx, q.hb);
  else if (q.hess) {
    if constexpr (KIND == DPI_EQ_GBM) {
      EqDev e2 = p->e;
      e2.sdgd_v = 0;  // the Hessian estimators evaluate f with the full Hessian (data.py:856, :1262-1272)
      hipLaunchKernelGGL((k_paths<KIND, H, L, Z, false, true>), dim3(q.nblocks), dim3(NTH), 0, q.st, e2, net->d,
                         *q.a);
    }
  } else if constexpr (!Z && KIND != DPI_EQ_GBM && H % 32 == 0) {
    if (q.a->split)
      hipLaunchKernelGGL((k_paths<KIND, H, L, Z, true>), dim3(q.nblocks), dim3(NTH), 0, q.st, p->e, net->d, *q.a);
    else
      hipLaunchKernelGGL((k_paths<KIND, H, L, Z, false>), dim3(q.nblocks), dim3(NTH), 0, q.st, p->e, net->d, *q.a);
  } else
    hipLaunchKernelGGL((k_paths<KIND, H, L, Z, false>), dim3(q.nblocks), dim3(NTH), 0, q.st, p->e, net->d, *q.a);
}

template <int KIND>
static bool dispatch(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  if (net->d.kind == 0) {
    do_launch<KIND, 16, 1, true>(p, net, q);
    return true;
  }
  const int H = net->d.H, L = net->d.L;
  if (q.baseline) {  // the baseline kernel is shape-generic
    if (KIND == DPI_EQ_GBM && H > 64) return false;
    do_launch<KIND, 16, 1, false>(p, net, q);
    return true;
  }
  if constexpr (KIND == DPI_EQ_GBM) {  // all weights LDS-resident: H <= 64
#define DPI_SHAPE(HH, LL)                      \
  if (H == HH && L == LL) {                    \
    do_launch<KIND, HH, LL, false>(p, net, q); \
    return true;                               \
  }
    DPI_SHAPE(64, 3)
    DPI_SHAPE(64, 2)
    DPI_SHAPE(32, 2)
    DPI_SHAPE(32, 3)
    DPI_SHAPE(16, 1)
    DPI_SHAPE(16, 2)
    DPI_SHAPE(16, 3)
    return false;
  } else {
    DPI_SHAPE(128, 4)
    DPI_SHAPE(128, 3)
    DPI_SHAPE(128, 2)
    DPI_SHAPE(64, 3)
    DPI_SHAPE(64, 2)
    DPI_SHAPE(32, 2)
    DPI_SHAPE(16, 1)
    DPI_SHAPE(16, 2)
    DPI_SHAPE(16, 3)
#undef DPI_SHAPE
    return false;
  }
}

static bool dispatch_any(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  switch (p->e.kind) {
    case DPI_EQ_CHA:
      return dispatch<DPI_EQ_CHA>(p, net, q);
    case DPI_EQ_OU:
      return dispatch<DPI_EQ_OU>(p, net, q);
    case DPI_EQ_GBM:
      return dispatch<DPI_EQ_GBM>(p, net, q);
    default:
      return false;
  }
}

static int check_pair(dpi_problem p, dpi_net net);
extern "C" {
static int check_pair(dpi_problem p, dpi_net net) {
  if (!p || !net) return fail(DPI_ERR_ARG, "null problem or net");
  if (net->d.kind && net->n_in != 1 + p->e.nx) return fail(DPI_ERR_ARG, "net input width != 1 + nx");
  if (net->d.kind && net->d.nxp > NXP_MAX) return fail(DPI_ERR_ARG, "nx too large");
  return 0;
}

static int pis_check(dpi_problem p) {
  if (p->e.kind != DPI_EQ_OU)
    return fail(DPI_ERR_UNSUPPORTED, "PISGradNet device net needs OUProcessEquation (its g0 is the problem's GMM g)");
  return 0;
}

static int pis_baseline(dpi_problem p, dpi_net net, const float* tx, int n, const WsLayout& w, char* b,
                        hipStream_t st) {
  int rc = pis_check(p);
  if (rc) return rc;
  float *gx = (float*)(b + w.gx), *fb = (float*)(b + w.fb), *rows = (float*)(b + w.rows);
  // g(x) (k_baseline's zero-net instance also writes a placeholder f_b, overwritten below)
  hipLaunchKernelGGL((k_baseline<DPI_EQ_OU, true>), dim3(n), dim3(NTHB), 0, st, p->e, net->d, tx, n, gx, fb,
                     (float*)(b + w.bx), (float*)(b + w.hb));
  const int F = 1 + p->e.nx;
  const PisRows L = pis_rows_layout(net->pis);
  for (int i0 = 0; i0 < n; i0 += w.rows_cap) {
    const int R = std::min(w.rows_cap, n - i0);
    hipLaunchKernelGGL(k_pis_points, dim3(R), dim3(64), 0, st, p->e.nx, net->pis, tx + (size_t)i0 * F, R, rows, L);
    const PisRows Lc = pis_chain(net->pis, rows, R, st);
    hipLaunchKernelGGL(k_pis_base_final<DPI_EQ_OU>, dim3((R + 15) / 16), dim3(64), 0, st, p->e, net->pis, rows, Lc,
                       R, fb + i0);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

static int pis_paths(dpi_problem p, dpi_net net, const float* tx, int n, int K, const PathArgs& a, const WsLayout& w,
                     char* b, hipStream_t st) {
  int rc = pis_check(p);
  if (rc) return rc;
  float* rows = (float*)(b + w.rows);
  const PisRows L = pis_rows_layout(net->pis);
  const int G = n * a.nbp, GC = std::max(1, w.rows_cap / P);
  for (int g0 = 0; g0 < G; g0 += GC) {
    const int g = std::min(GC, G - g0);
    hipLaunchKernelGGL(k_pis_rollout<DPI_EQ_OU>, dim3(g), dim3(NTH), 0, st, p->e, net->pis, tx, g0, a.nbp, a.m_begin,
                       K, a.flags, a.k0, a.k1, a.c3t, a.c3s, a.c3i, a.point_base, a.gx, rows, L);
    const PisRows Lc = pis_chain(net->pis, rows, g * P, st);
    hipLaunchKernelGGL(k_pis_final<DPI_EQ_OU>, dim3(g), dim3(NTH), 0, st, p->e, net->pis, tx, g0, a.nbp, K, a.flags,
                       a.fb, rows, Lc, a.partial);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_point_baseline(dpi_problem p, dpi_net net, const float* tx, int n, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (!tx || !ws || n < 0) return fail(DPI_ERR_ARG, "point_baseline: bad arguments");
  if (n == 0) return 0;
  const WsLayout w = ws_layout(net, n, 0, 1 + p->e.nx);
  if (ws_bytes < w.partial) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  char* b = (char*)ws;
  if (net->d.kind == 2) return pis_baseline(p, net, tx, n, w, b, (hipStream_t)stream);
  Launch q{true, tx, n, (float*)(b + w.gx), (float*)(b + w.fb), (float*)(b + w.bx), (float*)(b + w.hb), nullptr, 0,
           (hipStream_t)stream};
  if (!dispatch_any(p, net, q)) return fail(DPI_ERR_UNSUPPORTED, "point_baseline: unsupported equation/network shape");
  HIPCHK(hipGetLastError());
  return 0;
}

// k_paths phase order policy (see the kernel); DPI_ORDER overrides for ablations.
static int path_order() {
  const char* e = std::getenv("DPI_ORDER");
  return e ? std::atoi(e) : 0;
}

static int moments_impl(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                        uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                        void* ws, size_t ws_bytes, void* stream, float* y, float bound) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (!tx || !ws || !moments || n < 0 || K < 1 || M < 1 || m_begin < 0 || m_end > M || m_end <= m_begin ||
      (m_begin % P) || (m_end % P) || !(flags & DPI_BOTH) || (flags & ~DPI_BOTH) || epoch > 0xFFFFFFu)
    return fail(DPI_ERR_ARG, "label_moments: bad arguments (m range multiple of 64 within [0, M], K >= 1)");
  if (n == 0) return 0;
  const int F = 1 + p->e.nx;
  const int nbp = (m_end - m_begin) / P;
  if (nbp > 1024) return fail(DPI_ERR_ARG, "label_moments: at most 1024 x 64 paths per call");
  const WsLayout w = ws_layout(net, n, M, F);
  if (ws_bytes < w.total) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  char* b = (char*)ws;
  float* partial = (float*)(b + w.partial);
  PathArgs a;
  a.tx = tx;
  a.gx = (const float*)(b + w.gx);
  a.fb = (const float*)(b + w.fb);
  a.bx = (const float*)(b + w.bx);
  a.hb = (const float*)(b + w.hb);
  a.partial = partial;
  a.n = n;
  a.nbp = nbp;
  a.m_begin = m_begin;
  a.K = K;
  a.flags = flags;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.c3t = DPI_TAG_TERM | (epoch << 8);
  a.c3s = DPI_TAG_S | (epoch << 8);
  a.c3i = DPI_TAG_INT | (epoch << 8);
  a.c3q = DPI_TAG_SDGD | (epoch << 8);
  a.point_base = point_base;
  a.order = path_order();
  a.split = mlp_split() ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  if (net->d.kind == 2) {
    if ((rc = pis_paths(p, net, tx, n, K, a, w, b, st))) return rc;
  } else {
    Launch q{false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, &a, n * nbp, st};
    if (!dispatch_any(p, net, q))
      return fail(DPI_ERR_UNSUPPORTED, "label_moments: unsupported equation/network shape");
  }
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_reduce, dim3(n, (2 * F + 3) / 4), dim3(256), 0, st, partial, n, F, nbp, moments,
                     (const float*)(b + w.gx), 1.0f / (float)M, (flags & DPI_TERMINAL) ? 1 : 0, bound, y, F);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_label_moments(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed, uint32_t epoch,
                      uint32_t point_base, int m_begin, int m_end, int flags, float* moments, void* ws,
                      size_t ws_bytes, void* stream) {
  return moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, moments, ws, ws_bytes,
                      stream, nullptr, 0.f);
}

int dpi_moments_reduce(float* parts, int n_parts, int n, int nx, float* out, void* stream) {
  if (!parts || !out || n_parts < 1 || n < 0 || nx < 1) return fail(DPI_ERR_ARG, "moments_reduce: bad arguments");
  if (n == 0) return 0;
  if (n_parts > 1024) return fail(DPI_ERR_ARG, "moments_reduce: at most 1024 parts");
  const int len = n * 2 * (1 + nx);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_reduce_parts, dim3((len + 3) / 4), dim3(256), 0, st, (const float*)parts, n_parts, len, out);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_sums_reduce(const float* parts, int n_parts, size_t len, float* out, void* stream) {
  if (!parts || !out || n_parts < 1 || n_parts > 1024 || len > 0x7fffffffu)
    return fail(DPI_ERR_ARG, "sums_reduce: bad arguments (1 <= n_parts <= 1024)");
  if (len == 0) return 0;
  hipLaunchKernelGGL(k_reduce_parts, dim3((unsigned)((len + 3) / 4)), dim3(256), 0, (hipStream_t)stream, parts,
                     n_parts, (int)len, out);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_label_finalize(dpi_problem p, const float* moments, int n, int M, int flags, float sample_bound, float* y,
                       const void* ws, size_t ws_bytes, void* stream) {
  if (!p || !moments || !y || !ws || n < 0 || M < 1 || ws_bytes < (size_t)n * 4)
    return fail(DPI_ERR_ARG, "label_finalize: bad arguments");
  if (n == 0) return 0;
  const int F = 1 + p->e.nx;
  hipLaunchKernelGGL(k_finalize, dim3((n * F + 255) / 256), dim3(256), 0, (hipStream_t)stream, moments,
                     (const float*)ws, n, F, 1.0f / (float)M, (flags & DPI_TERMINAL) ? 1 : 0, sample_bound, y);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_generate_with_gradients(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                                uint32_t epoch, uint32_t point_base, int flags, float sample_bound, float* y,
                                float* moments, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (n == 0) return 0;
  const int F = 1 + p->e.nx;
  const WsLayout w = ws_layout(net, n, M, F);
  if (!ws || ws_bytes < w.total) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  if (!moments) return fail(DPI_ERR_ARG, "generate_with_gradients: moments buffer (n*2*(1+nx) floats) required");
  if ((rc = dpi_point_baseline(p, net, tx, n, ws, ws_bytes, stream))) return rc;
  if (!y) return fail(DPI_ERR_ARG, "generate_with_gradients: null y");
  // moments and labels come out of the same block-reduce launch
  return moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, flags, moments, ws, ws_bytes, stream, y,
                      sample_bound);
}

// ---- Malliavin Hessian labels (generate_with_gradients_and_hessians)
static size_t hess_extra(int n, int M, int nx, size_t* moff) {
  const size_t nbp = (size_t)(M + P - 1) / P;
  *moff = al256((size_t)n * nbp * nx * nx * 4);  // Hessian block sums, then the moments
  return *moff + al256((size_t)n * 2 * (1 + nx) * 4);
}

size_t dpi_workspace_bytes_hessians(dpi_problem p, dpi_net net, int n, int M) {
  if (!p || n < 0 || M < 0) return 0;
  size_t moff;
  return al256(ws_layout(net, n, M, 1 + p->e.nx).total) + hess_extra(n, M, p->e.nx, &moff);
}

static int hess_moments_impl(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                             uint32_t epoch, uint32_t point_base, int m_begin, int m_end, float* moments, float* hsum,
                             void* ws, size_t ws_bytes, void* stream, float* y, float bound) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (p->e.kind != DPI_EQ_GBM)
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels need a SimpleDiffusionEquationWithHessian (GBMEquationComplexExact)");
  if (net->d.kind == 2) return fail(DPI_ERR_UNSUPPORTED, "Hessian labels: MLP or ZeroSolution networks only");
  if (!tx || !ws || !moments || n < 0 || K < 1 || M < 1 || m_begin < 0 || m_end > M || m_end <= m_begin ||
      (m_begin % P) || (m_end % P) || epoch > 0xFFFFFFu)
    return fail(DPI_ERR_ARG, "Hessian labels: bad arguments (m range multiple of 64 within [0, M], K >= 1)");
  if (n == 0) return 0;
  const int nx = p->e.nx, F = 1 + nx, C = nx * nx, nbp = (m_end - m_begin) / P;
  if (nbp > 1024) return fail(DPI_ERR_ARG, "Hessian labels: at most 1024 x 64 paths per call");
  const WsLayout w = ws_layout(net, n, M, F);
  size_t moff;
  const size_t base = al256(w.total), need = base + hess_extra(n, M, nx, &moff);
  if (ws_bytes < need) return fail(DPI_ERR_WORKSPACE, "workspace too small (dpi_workspace_bytes_hessians)");
  char* b = (char*)ws;
  PathArgs a;
  std::memset(&a, 0, sizeof(a));
  a.tx = tx;
  a.gx = (const float*)(b + w.gx);
  a.fb = (const float*)(b + w.fb);
  a.bx = (const float*)(b + w.bx);
  a.hb = (const float*)(b + w.hb);
  a.partial = (float*)(b + w.partial);
  a.n = n;
  a.nbp = nbp;
  a.m_begin = m_begin;
  a.K = K;
  a.flags = DPI_BOTH;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.c3t = DPI_TAG_TERM | (epoch << 8);
  a.c3s = DPI_TAG_S | (epoch << 8);
  a.c3i = DPI_TAG_INT | (epoch << 8);
  a.c3q = DPI_TAG_SDGD | (epoch << 8);
  a.c3h1 = DPI_TAG_HTERM | (epoch << 8);
  a.c3h2 = DPI_TAG_HINT | (epoch << 8);
  a.point_base = point_base;
  a.hpart = (float*)(b + base);
  hipStream_t st = (hipStream_t)stream;
  Launch q{false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, &a, n * nbp, st};
  q.hess = true;
  if (!dispatch_any(p, net, q))
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels: unsupported network shape (GBM: width <= 64)");
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_reduce, dim3(n, (2 * F + 3) / 4), dim3(256), 0, st, a.partial, n, F, nbp, moments, a.gx,
                     1.0f / (float)M, 1, bound, y, F + C);
  hipLaunchKernelGGL(k_reduce_hess, dim3((C + 3) / 4, n), dim3(256), 0, st, a.hpart, n, C, nbp, hsum,
                     1.0f / (float)M, bound, y, F + C, F);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_label_moments_hessians(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                               uint32_t epoch, uint32_t point_base, int m_begin, int m_end, float* moments,
                               float* hessian_sums, void* ws, size_t ws_bytes, void* stream) {
  if (!hessian_sums) return fail(DPI_ERR_ARG, "label_moments_hessians: null hessian_sums");
  return hess_moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, moments, hessian_sums, ws,
                           ws_bytes, stream, nullptr, 0.f);
}

int dpi_label_finalize_hessians(dpi_problem p, const float* moments, const float* hessian_sums, int n, int M,
                                float sample_bound, float* y, void* ws, size_t ws_bytes, void* stream) {
  if (!p || !moments || !hessian_sums || !y || !ws || n < 0 || M < 1)
    return fail(DPI_ERR_ARG, "label_finalize_hessians: bad arguments");
  if (n == 0) return 0;
  const int nx = p->e.nx, F = 1 + nx, C = nx * nx;
  if (ws_bytes < (size_t)n * 4) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const float* gx = (const float*)ws;  // WsLayout: gx at offset 0 (written by dpi_point_baseline)
  hipLaunchKernelGGL(k_finalize_y, dim3((n * F + 255) / 256), dim3(256), 0, st, moments, gx, n, F, 1.0f / (float)M,
                     1, sample_bound, y, F + C);
  const size_t tot = (size_t)n * C;
  hipLaunchKernelGGL(k_finalize_hess, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, hessian_sums, n, C,
                     1.0f / (float)M, sample_bound, y, F + C, F);
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_generate_with_gradients_and_hessians(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K,
                                             uint64_t seed, uint32_t epoch, uint32_t point_base, float sample_bound,
                                             float* y, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (!y || M < P || (M % P) || M > 1024 * P)
    return fail(DPI_ERR_ARG, "generate_with_gradients_and_hessians: bad arguments (M multiple of 64, <= 65536)");
  if (n == 0) return 0;
  if (p->e.kind != DPI_EQ_GBM)
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels need a SimpleDiffusionEquationWithHessian (GBMEquationComplexExact)");
  if ((rc = dpi_point_baseline(p, net, tx, n, ws, ws_bytes, stream))) return rc;
  const WsLayout w = ws_layout(net, n, M, 1 + p->e.nx);
  size_t moff;
  hess_extra(n, M, p->e.nx, &moff);
  float* moments = (float*)((char*)ws + al256(w.total) + moff);
  return hess_moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, moments, nullptr, ws, ws_bytes, stream,
                           y, sample_bound);
}

}  // extern "C"
