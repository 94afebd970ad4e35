// MI355X (gfx950) device code of the DPI label-generation hot path (kernels as templates; the
// C-ABI host code is dpi_kernels.hip, the k_paths instantiations dpi_paths_*.hip).
#pragma once
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
#ifndef DPI_NOISE_UNROLL_FO
// independent Philox chains per wave in the first-order k_paths noise loops: 4 (r03ag same-box A/B,
// 3 pairs: Burgers 0.3763-0.3777 -> 0.3740-0.3760 ms/step, configs[3] 10.354 -> 10.303; still 252 VGPRs)
#define DPI_NOISE_UNROLL_FO 4
#endif
#ifndef DPI_NOISE_UNROLL_GBM
// the same for GBM's one-wave-per-SIMD k_paths (the sweep sets its register count, so the rollout
// may hold more chains): 2 -> 4 r03aj (k_paths 783 -> 773 us), 4 -> 8 r04o (same-box A/B, 2 pairs:
// 742 -> 738-740 us; 376 VGPRs either way)
#define DPI_NOISE_UNROLL_GBM 8
#endif
#ifndef DPI_GBM_WAGPR
#define DPI_GBM_WAGPR 1
#endif
// the GBM network launch's wave index through readfirstlane (paths_body; an A/B knob)
#ifndef DPI_WV_UNIFORM_GBM
#define DPI_WV_UNIFORM_GBM 0
#endif
#ifndef DPI_NOISE_UNROLL_HESS
// the Hessian-label k_paths: 1 -> 4 r04o (same-box A/B, 2 pairs: 1.747 -> 1.719 ms/step)
#define DPI_NOISE_UNROLL_HESS 4
#endif
constexpr int NXP_MAX = 128;       // max padded state dimension of the two-workgroups-per-CU path kernels
// max state dimension of the wide first-order instances (Cha / OU, one workgroup per CU: the noise
// tile of 256 dims x 64 paths is 70 KB of LDS; dpi_paths_wide_*.hip)
constexpr int NXW_MAX = 256;
constexpr int HBS = NXW_MAX;  // row stride of the GBM baseline Hessian diagonal in the workspace (hb[n][HBS])
constexpr int HMAX = 128;

struct NetDev {
  int kind;  // 0 zero, 1 mlp
  int H, L, nxp;
  int act;   // DPI_ACT_* of every hidden layer (k_paths: the ACT template parameter, k_baseline: read here)
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
  // hidden layers for the split tangent sweep (mlp_hdiag_split): lo unscaled, prescaled by
  // 2^s (max |2^s W| in [0.5, 1)), wus = 2^-s (pack_split_x3)
  const uint32_t* WU[4];     // (H, H)
  float wus[4];
  // mlp_hdiag_split's operand scales (powers of two from the host's calibration pass,
  // dpi_kernels.hip x3_exponent): hsa[l] = store scale of a_l as the forward B operand of layer l + 1,
  // hsc[l] = wus[l] / hsa[l - 1]; tangent z'_l (the raw accumulator) = z_l / hzs[l], the operand of
  // layer l + 1 = act'(a_l) hbs[l] z'_l
  float hsa[4], hsc[4], hzs[4], hbs[4];
};

// ------------------------------------------------------------------------------ helpers
__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float elu(float z) { return z > 0.f ? z : __expf(z) - 1.0f; }
__device__ __forceinline__ float delu_from_a(float a) { return a > 0.f ? 1.0f : a + 1.0f; }

// tanh for the network activations (torch.nn.Tanh): 1 - 2 / (e^{2z} + 1) — v_exp_f32 + v_rcp_f32,
// four VALU operations and no extra live registers; saturates to +-1 (e^{2z} = inf or 0).  Its error
// is absolute (~1e-7 near z = 0, where 1 - x cancels), as is ELU's e^z - 1 on the same hardware.
__device__ __forceinline__ float tanh_act(float z) {
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * z)), 1.0f);
}

// The MLP activations of construct_mlp (picard/solution.py:123-135) the kernels are compiled for:
// f(z), and the first and second derivatives expressed through the activation value a = f(z)
// (what the backward passes and the Hessian-diagonal sweeps hold).
template <int ACT>
struct Act;
template <>
struct Act<DPI_ACT_ELU> {  // ELU(alpha = 1)
  static __device__ __forceinline__ float f(float z) { return elu(z); }
  static __device__ __forceinline__ float d(float a) { return delu_from_a(a); }
  static __device__ __forceinline__ float d2(float a) { return a > 0.f ? 0.f : a + 1.0f; }
};
template <>
struct Act<DPI_ACT_TANH> {  // tanh' = 1 - a^2, tanh'' = -2 a (1 - a^2)
  static __device__ __forceinline__ float f(float z) { return tanh_act(z); }
  static __device__ __forceinline__ float d(float a) { return fmaf(-a, a, 1.0f); }
  static __device__ __forceinline__ float d2(float a) { return -2.0f * a * fmaf(-a, a, 1.0f); }
};
// Runtime selection for the shape-generic, latency-bound per-point baseline (k_baseline).
__device__ __forceinline__ float act_f(int act, float z) {
  return act == DPI_ACT_TANH ? Act<DPI_ACT_TANH>::f(z) : Act<DPI_ACT_ELU>::f(z);
}
__device__ __forceinline__ float act_d(int act, float a) {
  return act == DPI_ACT_TANH ? Act<DPI_ACT_TANH>::d(a) : Act<DPI_ACT_ELU>::d(a);
}
__device__ __forceinline__ float act_d2(int act, float a) {
  return act == DPI_ACT_TANH ? Act<DPI_ACT_TANH>::d2(a) : Act<DPI_ACT_ELU>::d2(a);
}

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
typedef float f32x2 __attribute__((ext_vector_type(2)));
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

// LDS layout (floats) of the first-order path kernels for state dimensions up to NXW.
template <int NXW_>
struct LdsT {
  static constexpr int NXW = NXW_;
  float S[NXW * SS];       // [dim][path] integral noise sums
  float W[2 * 32 * HMAX];  // weight chunk: f32 rows of stride WST, or two split chunks (LDS-DMA ring)
  float vec[4 * HMAX];     // base0 | w1t | wout | c1
  float bh[4 * HMAX];      // hidden-layer biases
  float xsh[NXW];          // point x
  float gst[4 * P * NSG];  // per-wave partial g statistics
  float tau[P], cmul[P], bsh[P];
};
using Lds = LdsT<NXP_MAX>;

// ------------------------------------------------------------------------------ MLP tile
// u and gradient terms for the 16 paths of this wave (path column pp = 16*wave + (lane&15)).
// Inputs (all in LDS): S tile [d][p], xsh (X_d = xsh[d] + cmul_p * S[d][p]), tau (time input),
// cmul, vec[0:H] = base0 (layer-1 bias incl. W1x x), vec[H:2H] = w1t, vec[2H:3H] = wout,
// vec[3H:4H] = c1, bh[l*H:(l+1)*H] = biases of hidden layers l >= 1.
// If bx_out != nullptr (baseline mode) writes b1 + W1x S (per path) to bx_out[pp*bstride + h].
template <int KIND, int H, int L, int ACT, class SH>
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
  if constexpr (SH::NXW > NXP_MAX) {  // wide instances: W1x staged in column blocks of 128
#pragma unroll
    for (int T0 = 0; T0 < HT; T0 += 2) {
      const int nr = (HT - T0) >= 2 ? 32 : 16;
      floatx4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      for (int cb = 0; 128 * cb < net.nxp; ++cb) {
        const int ncb = min(128, net.nxp - 128 * cb), nf4 = ncb >> 2;
        __syncthreads();
        for (int idx = threadIdx.x; idx < nr * nf4; idx += NTH) {
          const int r = idx / nf4, c = idx - r * nf4;
          *reinterpret_cast<float4*>(sh.W + r * WST + 4 * c) =
              *reinterpret_cast<const float4*>(net.W1x + (size_t)(16 * T0 + r) * net.nxp + 128 * cb + 4 * c);
        }
        __syncthreads();
#pragma unroll
        for (int T2 = 0; T2 < 2; ++T2) {
          if (T0 + T2 < HT) {
            const float* wrow = sh.W + (16 * T2 + jj) * WST + 4 * qq;
            for (int t = 0; t < (ncb >> 4); ++t) {
              const float4 a = *reinterpret_cast<const float4*>(wrow + 16 * t);
              const float* bc = sh.S + (128 * cb + 16 * t + 4 * qq) * SS + pp;
              acc[T2] = mfma4(a.x, bc[0], acc[T2]);
              acc[T2] = mfma4(a.y, bc[SS], acc[T2]);
              acc[T2] = mfma4(a.z, bc[2 * SS], acc[T2]);
              acc[T2] = mfma4(a.w, bc[3 * SS], acc[T2]);
            }
          }
        }
      }
#pragma unroll
      for (int T2 = 0; T2 < 2; ++T2) {
        const int T = T0 + T2;
        if (T < HT) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int h = 16 * T + 4 * qq + r;
            const float z = fmaf(cm, acc[T2][r], fmaf(sh.vec[H + h], tau, sh.vec[h]));
            act[0][T][r] = Act<ACT>::f(z);
          }
        }
      }
    }
  } else {
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
          act[0][T][r] = Act<ACT>::f(z);
          if (bx_out && pp < n_valid_paths) bx_out[(size_t)pp * bstride + h] = sh.vec[h] + acc[r];
        }
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
            act[l][T][r] = Act<ACT>::f(acc[r] + sh.bh[l * H + h]);
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
      act[L - 1][T][r] = w * Act<ACT>::d(act[L - 1][T][r]);
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
          for (int r = 0; r < 4; ++r) act[l][T][r] = acc[r] * Act<ACT>::d(act[l][T][r]);
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
// NXW > 128 (the wide instances): a layer-1 chunk of 32 rows is split into column sub-chunks of
// 128 words (the ring slot's width), nc1 per row pair, in column order.
template <int H, int L, int NXW = NXP_MAX>
struct SplitStream {
  static constexpr int NT = H / 32;  // chunks per H-row matrix
  static constexpr int NCW = NXW / 128;  // layer-1 column sub-chunks per 32-row chunk, at most
  const NetDev& net;
  int C1, nc1, n1, nT1, total;
  __device__ SplitStream(const NetDev& n, bool grad_full) : net(n) {
    C1 = n.nxp32;
    nc1 = NCW == 1 ? 1 : (C1 + 127) >> 7;
    n1 = NT * nc1;                         // layer-1 chunks (H output rows)
    nT1 = C1 / 32;                         // W1x^T chunks (C1 output rows)
    total = n1 + 2 * (L - 1) * NT + (grad_full ? nT1 : 0);
  }
  // chunk idx: source g (first word of its first row), LDS row width C, source row stride Cg, first row r0
  __device__ __forceinline__ void desc(int idx, const uint32_t*& g, int& C, int& Cg, int& r0) const {
    Cg = 0;
    if (idx < n1) {
      if constexpr (NCW == 1) {
        g = net.W1xS, C = C1, r0 = 32 * idx;
      } else {
        const int pr = idx / nc1, kc = idx - pr * nc1;
        g = net.W1xS + 128 * kc, C = min(128, C1 - 128 * kc), Cg = C1, r0 = 32 * pr;
      }
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
  __device__ __forceinline__ void desc(int idx, const uint32_t*& g, int& C, int& r0) const {
    int Cg;
    desc(idx, g, C, Cg, r0);
  }
  // LDS-DMA of chunk idx into ring slot idx & 1: wave-instruction w writes LDS granules
  // [64 w, 64 w + 64) lane-linearly; lane i's source is the granule that belongs there.
  __device__ __forceinline__ void issue(int idx, uint32_t* ring) const {
    if (idx >= total) return;
    const uint32_t* g;
    int C, Cg, r0;
    desc(idx, g, C, Cg, r0);
    if (NCW == 1 || Cg == 0) Cg = C;
    uint32_t* dst = ring + (idx & 1) * (32 * HMAX);
    const int gpr = C >> 2, m = split_swz(C), lane = threadIdx.x & 63;
    for (int w = threadIdx.x >> 6; w < (C >> 3); w += NTH / 64) {
      const int G = 64 * w + lane, r = G / gpr, gs = (G - r * gpr) ^ (r & m);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(g + (size_t)(r0 + r) * Cg + 4 * gs),
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
template <int KIND, int H, int L, int ACT, class SH>
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
  constexpr int NXW = SH::NXW;
  SplitStream<H, L, NXW> ss(net, Eq<KIND>::GRAD_FULL);
  const int nu1 = ss.C1 >> 5;
  int chunk = 0;
  ss.issue(0, wsh);
  float act[L][HT][4];
  half8 bh[NU], bl[NU];

  // ---------------- layer 1: z = base0 + w1t*tau + cmul * (W1x S)
  half8 xh[NXW / 32], xl[NXW / 32];  // the noise tile as B operand, split once
#pragma unroll
  for (int u = 0; u < NXW / 32; ++u) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = u < nu1 ? sh.S[(32 * u + 4 * qq + (j & 3) + 16 * (j >> 2)) * SS + pp] : 0.f;
    split8(x, xh[u], xl[u]);
  }
#pragma unroll
  for (int T0 = 0; T0 < HT; T0 += 2) {
    floatx4 am[2], ac[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) am[t] = ac[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NXW / 128; ++kc) {  // column sub-chunks of 128 words (one for NXW = 128)
      if (kc == 0 || 128 * kc < ss.C1) {
        int C;
        const uint32_t* wch = ss.enter(chunk++, wsh, C);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (4 * kc + u < nu1) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              half8 ah, al;
              load_a_split(wch, C, 16 * t + jj, u, qq, ah, al);
              am[t] = mfma16(ah, xh[4 * kc + u], am[t]);
              ac[t] = mfma16(ah, xl[4 * kc + u], ac[t]);
              ac[t] = mfma16(al, xh[4 * kc + u], ac[t]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * (T0 + t) + 4 * qq + r;
        const float acc = fmaf(ac[t][r], SPLIT_INV, am[t][r]);
        act[0][T0 + t][r] = Act<ACT>::f(fmaf(cm, acc, fmaf(sh.vec[H + h], tau, sh.vec[h])));
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
        for (int r = 0; r < 4; ++r) act[l][T0 + t][r] = Act<ACT>::f(o[t][r] + sh.bh[l * H + 16 * (T0 + t) + 4 * qq + r]);
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
      act[L - 1][T][r] = w * Act<ACT>::d(act[L - 1][T][r]);
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
        for (int r = 0; r < 4; ++r) act[l][T0 + t][r] = o[t][r] * Act<ACT>::d(act[l][T0 + t][r]);
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
// 100-direction tangent sweep.  H <= 64, L <= 4.  Wide instances (NXW = NXW_MAX, nx <= 256): the
// 256-row noise tile leaves no room for W1x (it is read from L2: layer 0's A operand and the sweep's
// z_0 = W1x[:, d] as a row of W1x^T) and the hidden weights are resident for L <= 3.
template <int H, int NXW_ = NXP_MAX>
struct LdsGbm {
  static constexpr int NXW = NXW_;
  static constexpr bool W1X_LDS = NXW == NXP_MAX;
  static constexpr int WXS = NXP_MAX + 8;  // W1x row stride (WXS/4 = 2 mod 4)
  static constexpr int WHS = H + 8;        // hidden row stride
  static constexpr int NWH = W1X_LDS ? 3 : 2;
  float S[NXW * SS];
  float W1x[W1X_LDS ? H * WXS : 4];
  float Wh[NWH][H * WHS];
  float vec[4 * HMAX];
  float bh[4 * HMAX];
  float xsh[NXW];
  float hb[NXW];
  float gst[4 * P * NSG];
  float fst[4 * P * NSG];
  float wx[NSG];
  float tau[P], cmul[P], bsh[P], fbp[P];
  float smt[P];                    // Hessian labels: s - t per path
  unsigned char cnt[NXW * P];      // SDGD index histogram [d][path]
  // SDGD: each path's distinct sampled directions in increasing order (mlp_hdiag_split's sweep;
  // H >= 32 only — the u = 0 and H = 16 instances keep their LDS under 80 KB, two blocks per CU)
  static constexpr int DLCAP = H >= 32 ? 96 : 1;
  unsigned char dl[P * DLCAP];
};

// Row h of W1x from the GBM LDS image (stride WXS) or, in the wide instances, from L2 (stride nxp).
template <int H, int NXW>
__device__ __forceinline__ const float* gbm_w1x_row(const LdsGbm<H, NXW>& sh, const NetDev& net, int h) {
  if constexpr (LdsGbm<H, NXW>::W1X_LDS)
    return sh.W1x + h * LdsGbm<H, NXW>::WXS;
  else
    return net.W1x + (size_t)h * net.nxp;
}
// z_0 = W1x[:, d] for this lane's units 16 T + 4 qq + r (LDS column reads, or one 16-B row chunk of
// W1x^T per T in the wide instances)
template <int H, int NXW>
__device__ __forceinline__ void gbm_w1x_col(const LdsGbm<H, NXW>& sh, const NetDev& net, int d, int qq,
                                            float (&z)[H / 16][4]) {
#pragma unroll
  for (int T = 0; T < H / 16; ++T) {
    if constexpr (LdsGbm<H, NXW>::W1X_LDS) {
#pragma unroll
      for (int r = 0; r < 4; ++r) z[T][r] = sh.W1x[(16 * T + 4 * qq + r) * LdsGbm<H, NXW>::WXS + d];
    } else {
      const float4 v = *reinterpret_cast<const float4*>(net.W1xT + (size_t)d * H + 16 * T + 4 * qq);
      z[T][0] = v.x, z[T][1] = v.y, z[T][2] = v.z, z[T][3] = v.w;
    }
  }
}

// Diagonal of the x-Hessian of u at (s, X_s) for this wave's 16 paths, contracted with the
// path's SDGD index histogram: s1 = sum_d cnt[d] u_dd, s2 = sum_d cnt[d] |u_dd|.
// Uses u_dd = sum_l < lam_l, elu''(z_l) * zdot_l^2 >, with lam_l = du/da_l (one backward pass)
// and zdot_l = dz_l/dx_d (first-order tangents only): half the MACs of second-order
// forward mode.  All GEMMs are v_mfma_f32_16x16x4_f32 in the hidden x path orientation.
template <int H, int L, int ACT, int NXW>
__device__ __forceinline__ void mlp_hdiag(const EqDev& e, const NetDev& net, LdsGbm<H, NXW>& sh, int nxt, float& s1_out,
                                          float& s2_out) {
  constexpr int HT = H / 16;
  constexpr int WHS = LdsGbm<H, NXW>::WHS;
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
    const float* wrow = gbm_w1x_row(sh, net, 16 * T + jj) + 4 * qq;
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
      act[0][T][r] = Act<ACT>::f(fmaf(cm, acc[r], fmaf(sh.vec[H + h], tau, sh.vec[h])));
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
      for (int r = 0; r < 4; ++r) act[l][T][r] = Act<ACT>::f(acc[r] + sh.bh[l * H + 16 * T + 4 * qq + r]);
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
      for (int r = 0; r < 4; ++r) Bm[t][r] = Act<ACT>::d(act[l + 1][t][r]) * lam[l + 1][t][r];
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
    gbm_w1x_col(sh, net, d, qq, z);
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) term = fmaf(lam[0][T][r] * Act<ACT>::d2(act[0][T][r]), z[T][r] * z[T][r], term);
#pragma unroll
    for (int l = 1; l < L; ++l) {
      float Bm[HT][4];
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) Bm[t][r] = Act<ACT>::d(act[l - 1][t][r]) * z[t][r];
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
          term = fmaf(lam[l][T][r] * Act<ACT>::d2(act[l][T][r]), acc[r] * acc[r], term);
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

// mlp_hdiag on the fp16-split MFMA (H % 32 == 0): same inputs and outputs.  The hidden layers'
// split weights (NetDev::WU: lo unscaled, matrix prescaled by 2^s) are loaded ONCE into registers
// as MFMA A fragments (2 (L - 1) (H / 16) (H / 32) half8: 128 VGPRs at H = 64, L = 3) and reused by
// the forward pass and by every direction of the tangent sweep, which then runs without LDS
// traffic: per direction and layer (H/16)(H/32) x 3 v_mfma_f32_16x16x32_f16 (hi hi + hi lo + lo hi
// into one accumulator) instead of (H/16)(H/4) v_mfma_f32_16x16x4_f32.  B operands are split in
// registers with the same unscaled-lo convention, prescaled by a power of two so their residuals
// stay fp16-normal; every scale is a power of two folded into per-unit constants computed once
// (ELU' x scale for the next layer's operand, lam elu'' / scale^2 for the squared tangents), so a
// direction costs per element one multiply, the split and one FMA.  Layer 0 (the noise tile
// through W1x) and z_0 = W1x[:, d] stay fp32 from LDS; the adjoint reads the transposed split
// weights (WTS) from L2 once.
__device__ __forceinline__ void split8u(const float (&x)[8], half8& hi, half8& lo) {
  typedef _Float16 half2v __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2 x2 = {x[j], x[j + 1]};
    const half2v h = __builtin_convertvector(x2, half2v);
    const half2v l = __builtin_convertvector(x2 - __builtin_convertvector(h, f32x2), half2v);
    hi[j] = h.x, hi[j + 1] = h.y;
    lo[j] = l.x, lo[j + 1] = l.y;
  }
}
template <int H, int L, int ACT, int NXW>
__device__ __forceinline__ void mlp_hdiag_split(const EqDev& e, const NetDev& net, LdsGbm<H, NXW>& sh, int nxt,
                                                float& s1_out, float& s2_out) {
  static_assert(H % 32 == 0, "split hdiag needs H % 32 == 0");
  constexpr int HT = H / 16, NU = H / 32, LH = L > 1 ? L - 1 : 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane & 15, qq = lane >> 4;
  const int pp = 16 * wv + jj;
  const float tau = sh.tau[pp];
  const float cm = sh.cmul[pp];
  auto afrag = [&](const uint32_t* W, int row, int u, half8& ah, half8& al) {  // global, fragment order
    const uint32_t* rp = W + (size_t)row * H + 4 * (8 * u + 2 * qq);
    ah = __builtin_bit_cast(half8, *reinterpret_cast<const u32v4*>(rp));
    al = __builtin_bit_cast(half8, *reinterpret_cast<const u32v4*>(rp + 4));
  };
  half8 wh[LH][HT][NU], wl[LH][HT][NU];
#pragma unroll
  for (int l = 1; l < L; ++l)
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int u = 0; u < NU; ++u) afrag(net.WU[l], 16 * T + jj, u, wh[l - 1][T][u], wl[l - 1][T][u]);
#if DPI_GBM_WAGPR
  // the resident weight fragments pinned to AGPRs (MFMA reads its A operand from either file), so
  // more of the sweep's accumulators stay in VGPRs: GBM k_paths 742 -> 735-736 us, Hessian labels
  // unchanged (same-box pairs, r04t; DPI_GBM_WAGPR=0 builds without)
#pragma unroll
  for (int l = 1; l < L; ++l)
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int u = 0; u < NU; ++u) asm volatile("" : "+a"(wh[l - 1][T][u]), "+a"(wl[l - 1][T][u]));
#endif
  // B operand (C layout, HT tiles x 4) x scale -> split halves per 32-wide chunk
  auto split_b = [&](const float (&x)[HT][4], const float (&f)[HT][4], half8 (&bh)[NU], half8 (&bl)[NU]) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f32x2 a = f32x2{f[2 * u][r], f[2 * u][r + 1]} * f32x2{x[2 * u][r], x[2 * u][r + 1]};
        const f32x2 b = f32x2{f[2 * u + 1][r], f[2 * u + 1][r + 1]} * f32x2{x[2 * u + 1][r], x[2 * u + 1][r + 1]};
        v[r] = a.x, v[r + 1] = a.y, v[4 + r] = b.x, v[5 + r] = b.y;
      }
      split8u(v, bh[u], bl[u]);
    }
  };
  // o = W'_l B (one accumulator per tile; tile-inner order between dependent products)
  auto wmul = [&](int l, const half8 (&bh)[NU], const half8 (&bl)[NU], floatx4 (&o)[HT]) {
#pragma unroll
    for (int T = 0; T < HT; ++T) o[T] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NU; ++u) {
#pragma unroll
      for (int T = 0; T < HT; ++T) o[T] = mfma16(wh[l - 1][T][u], bh[u], o[T]);
#pragma unroll
      for (int T = 0; T < HT; ++T) o[T] = mfma16(wh[l - 1][T][u], bl[u], o[T]);
#pragma unroll
      for (int T = 0; T < HT; ++T) o[T] = mfma16(wl[l - 1][T][u], bh[u], o[T]);
    }
  };
  float act[L][HT][4];
  float lam[L][HT][4];
  // forward, layer 0: fp32 MFMA over the noise tile (once per path)
#pragma unroll
  for (int T = 0; T < HT; ++T) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = gbm_w1x_row(sh, net, 16 * T + jj) + 4 * qq;
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
      act[0][T][r] = Act<ACT>::f(fmaf(cm, acc[r], fmaf(sh.vec[H + h], tau, sh.vec[h])));
    }
  }
  // hidden layers: B = SA a_{l-1} (SA = hsa[l - 1]), o = 2^s SA W a -> a_l = Act<ACT>::f(o wus / SA + b)
  {
#pragma unroll
    for (int l = 1; l < L; ++l) {
      float ones[HT][4];
#pragma unroll
      for (int T = 0; T < HT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) ones[T][r] = net.hsa[l - 1];
      half8 bh[NU], bl[NU];
      split_b(act[l - 1], ones, bh, bl);
      floatx4 o[HT];
      wmul(l, bh, bl, o);
      const float sc = net.hsc[l];
#pragma unroll
      for (int T = 0; T < HT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) act[l][T][r] = Act<ACT>::f(fmaf(o[T][r], sc, sh.bh[l * H + 16 * T + 4 * qq + r]));
    }
  }
  // adjoints lam_l = du/da_l: lam_l = W_{l+1}^T (elu'(a_{l+1}) lam_{l+1})  (scaled-lo WTS, once per path)
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
      for (int r = 0; r < 4; ++r) Bm[t][r] = Act<ACT>::d(act[l + 1][t][r]) * lam[l + 1][t][r];
    half8 bh[NU], bl[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) split_act(Bm[2 * u], Bm[2 * u + 1], bh[u], bl[u]);
#pragma unroll
    for (int T = 0; T < HT; ++T) {
      floatx4 am = {0.f, 0.f, 0.f, 0.f}, ac = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        half8 ah, al;
        afrag(net.WTS[l + 1], 16 * T + jj, u, ah, al);
        am = mfma16(ah, bh[u], am);
        ac = mfma16(ah, bl[u], ac);
        ac = mfma16(al, bh[u], ac);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) lam[l][T][r] = fmaf(ac[r], SPLIT_INV, am[r]);
    }
  }
  // per-unit constants of the sweep.  Tangent of layer l >= 1 is held as z'_l = (SB_{l-1} / wus_l) z_l
  // (the raw accumulator; SB_l = 2^eb[l], the tangent operand's store scale); the next operand is
  // SB_l elu'(a_l) z_l = (elu'(a_l) wus_l SB_l / SB_{l-1}) z'_l = (elu'(a_l) hbs_l) z'_l, and
  // lam_l elu''(a_l) z_l^2 = (lam_l elu''(a_l) hzs_l^2) z'_l^2, hzs_l = wus_l / SB_{l-1}.
  float fz[L > 1 ? L - 1 : 1][HT][4];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float zs = net.hzs[l];
    const float bs = net.hbs[l];
#pragma unroll
    for (int T = 0; T < HT; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lam[l][T][r] *= Act<ACT>::d2(act[l][T][r]) * (zs * zs);
        if (l < L - 1) fz[l][T][r] = Act<ACT>::d(act[l][T][r]) * bs;
      }
  }
  // tangent sweep over the state dimensions.  The lam z^2 terms accumulate in register pairs
  // (v_pk_mul_f32 + v_pk_fma_f32: one VALU issue per unit instead of two).
  float s1 = 0.f, s2 = 0.f;
  // z_0 = W1x[:, d] of the next direction is read from LDS while this direction's MFMAs run: two
  // register sets, the direction loop unrolled by 2 so they swap roles without copies
  auto ldz = [&](int d, float (&zz)[HT][4]) { gbm_w1x_col(sh, net, d, qq, zz); };
  // one direction: z (in) is clobbered; zn receives z_0 of direction dn; counted: weight cnt (else 0)
  auto direction = [&](int d, float (&z)[HT][4], float (&zn)[HT][4], int dn, bool counted) {
    f32x2 term2 = {0.f, 0.f};
    auto acc_terms = [&](const float (&lm)[HT][4], const float (&zz)[HT][4]) {
#pragma unroll
      for (int T = 0; T < HT; ++T)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 z2 = {zz[T][r], zz[T][r + 1]}, l2 = {lm[T][r], lm[T][r + 1]};
          term2 = (l2 * z2) * z2 + term2;
        }
    };
    ldz(dn, zn);
    acc_terms(lam[0], z);
#pragma unroll
    for (int l = 1; l < L; ++l) {
      half8 bh[NU], bl[NU];
      split_b(z, fz[l - 1], bh, bl);
      floatx4 o[HT];
      wmul(l, bh, bl, o);
#pragma unroll
      for (int T = 0; T < HT; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[T][r] = o[T][r];
      acc_terms(lam[l], z);
    }
    const float ud = qsum(term2.x + term2.y);
    const float c = counted ? (float)sh.cnt[d * P + pp] : 0.f;
    s1 = fmaf(c, ud, s1);
    s2 = fmaf(c, fabsf(ud), s2);
  };
  float za[HT][4], zb[HT][4];
  // SDGD (v draws with replacement, data.py:497-502) leaves about 37 % of the directions of a path
  // unsampled (count 0): the sweep then runs over each path's own distinct directions, in
  // increasing order — the MFMA batch of 16 paths needs no common direction, only per-lane
  // z_0 = W1x[:, d_p] — for max over the wave's paths of their distinct counts (about 70 of 100 at
  // v = nx = 100).  A path's padding slots repeat its last direction with weight 0, which leaves
  // s1, s2 exactly as the full sweep's fmaf(0, u_dd, s) steps do: the labels are bitwise the
  // full sweep's.  The exact diagonal (sdgd_v = 0) and paths with more than DLCAP distinct
  // directions take the full sweep.
  int ndp = e.nx, kmax = e.nx;
  bool lists = false;
  if (e.sdgd_v > 0) {
    constexpr int DLCAP = LdsGbm<H, NXW>::DLCAP;
    // the path's four lanes build its list together: lane qq scans dims [qq dq, (qq + 1) dq) (all
    // its histogram bytes read at once), places its sampled dims after the lower quarters' counts
    // (a prefix over the path's lanes jj + 16 q), so the list is in increasing order
    constexpr int QD = NXW / 4;
    using MaskT = std::conditional_t<(QD > 32), unsigned long long, uint32_t>;
    const int dq = (e.nx + 3) >> 2, d0 = qq * dq;
    MaskT mq = 0;
#pragma unroll
    for (int i = 0; i < QD; ++i)
      if (i < dq && d0 + i < e.nx && sh.cnt[(d0 + i) * P + pp]) mq |= (MaskT)1 << i;
    int cq;
    if constexpr (QD > 32)
      cq = __popcll(mq);
    else
      cq = __popc(mq);
    int base = 0;
    ndp = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int v = __shfl(cq, jj + 16 * q, 64);
      base += q < qq ? v : 0;
      ndp += v;
    }
    for (int k = base; mq; ++k) {
      int b;
      if constexpr (QD > 32)
        b = __builtin_ctzll(mq);
      else
        b = __builtin_ctz(mq);
      mq &= mq - 1;
      if (k < DLCAP) sh.dl[pp * DLCAP + k] = (unsigned char)(d0 + b);
    }
    // the list of path pp is written by its four lanes and read by them: LDS operations of one wave
    // complete in order; the asm keeps the compiler from hoisting the reads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    kmax = ndp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) kmax = max(kmax, __shfl_xor(kmax, o, 64));
    lists = kmax <= DLCAP;
  }
  if (lists) {
    constexpr int DLCAP = LdsGbm<H, NXW>::DLCAP;
    auto dir = [&](int k) { return (int)sh.dl[pp * DLCAP + min(k, ndp - 1)]; };
    int k = 0, dk = dir(0);
    ldz(dk, za);
    for (; k + 1 < kmax; k += 2) {
      const int d1 = dir(k + 1), d2 = dir(k + 2);
      direction(dk, za, zb, d1, k < ndp);
      direction(d1, zb, za, d2, k + 1 < ndp);
      dk = d2;
    }
    if (k < kmax) direction(dk, za, zb, dk, k < ndp);
  } else {
    ldz(0, za);
    int d = 0;
    for (; d + 1 < e.nx; d += 2) {
      direction(d, za, zb, d + 1, true);
      direction(d + 1, zb, za, d + 2 < e.nx ? d + 2 : d + 1, true);
    }
    if (d < e.nx) direction(d, za, zb, d, true);
  }
  s1_out = s1;
  s2_out = s2;
}

// u(tau, x + cmul S) for this wave's 16 paths with every weight LDS-resident (GBM layout):
// the forward half of mlp_hdiag.  The TD terminal value (data.py:941-942).
template <int H, int L, int ACT, int NXW>
__device__ __forceinline__ float mlp_value_res(const NetDev& net, LdsGbm<H, NXW>& sh, int nxt) {
  constexpr int HT = H / 16;
  constexpr int WHS = LdsGbm<H>::WHS;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane & 15, qq = lane >> 4;
  const int pp = 16 * wv + jj;
  const float tau = sh.tau[pp];
  const float cm = sh.cmul[pp];
  float act[L][HT][4];
#pragma unroll
  for (int T = 0; T < HT; ++T) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = gbm_w1x_row(sh, net, 16 * T + jj) + 4 * qq;
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
      act[0][T][r] = Act<ACT>::f(fmaf(cm, acc[r], fmaf(sh.vec[H + h], tau, sh.vec[h])));
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
      for (int r = 0; r < 4; ++r) act[l][T][r] = Act<ACT>::f(acc[r] + sh.bh[l * H + 16 * T + 4 * qq + r]);
    }
  }
  float up = 0.f;
#pragma unroll
  for (int T = 0; T < HT; ++T)
#pragma unroll
    for (int r = 0; r < 4; ++r) up = fmaf(sh.vec[2 * H + 16 * T + 4 * qq + r], act[L - 1][T][r], up);
  return qsum(up) + net.bout;
}

// ------------------------------------------------------------------------------ kernels
// Draws 1-3 (picard/data.py:161-167, equations.py:118-124/:217-230, utils.py:785-789).
struct SampleSpec {  // k_baseline's in-block sampling of its point (dpi_sample_with_gradients); tx == null: off
  float* tx;
  uint32_t k0, k1, c3t, c3x0, c3x, point_base;
  float eps, alpha_init_sqrt;
  int t_factors;
};
__device__ __forceinline__ float sample_point_t(const EqDev& e, const SampleSpec& s, uint32_t ig) {
  if (s.t_factors == 0) {  // sample_t_always_uniform (data.py:161-167)
    const float U = u01_co(philox4x32_10(0u, 0u, ig, s.c3t, s.k0, s.k1).x);
    return (e.T - 2.f * s.eps) * (1.f - U) + s.eps;
  }
  // sample_t (data.py:149-159): T (1 - prod of t_factors uniforms), left to right
  float prod = 1.f;
  for (int r0 = 0; r0 < s.t_factors; r0 += 4) {
    const auto w = philox4x32_10((uint32_t)(r0 >> 2), 0u, ig, s.c3t, s.k0, s.k1);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    for (int q = 0; q < 4 && r0 + q < s.t_factors; ++q) prod *= u01_co(ws[q]);
  }
  return e.T * (1.f - prod);
}
// x dims 4 j .. 4 j + 3 of point ig at time t
template <int KIND>
__device__ __forceinline__ void sample_point_x4(const EqDev& e, const SampleSpec& s, uint32_t ig, int j, float t,
                                                float (&x)[4]) {
  const f4 z = normals4(philox4x32_10((uint32_t)j, 0u, ig, s.c3x, s.k0, s.k1));
  f4 z0 = {0.f, 0.f, 0.f, 0.f};
  if (KIND == DPI_EQ_OU) {
    z0 = normals4(philox4x32_10((uint32_t)j, 0u, ig, s.c3x0, s.k0, s.k1));
    z0.a *= s.alpha_init_sqrt;
    z0.b *= s.alpha_init_sqrt;
    z0.c *= s.alpha_init_sqrt;
    z0.d *= s.alpha_init_sqrt;
  }
  const float sc = sqrtf(t) * e.asq;
  x[0] = fmaf(sc, z.a, z0.a);
  x[1] = fmaf(sc, z.b, z0.b);
  x[2] = fmaf(sc, z.c, z0.c);
  x[3] = fmaf(sc, z.d, z0.d);
}

template <int KIND>
__global__ void k_sample_points(EqDev e, int n, SampleSpec s) {
  const int nb = (e.nx + 3) >> 2;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = gid / nb, j = gid - i * nb;
  if (i >= n) return;
  const uint32_t ig = s.point_base + (uint32_t)i;
  const float t = sample_point_t(e, s, ig);
  float* row = s.tx + (size_t)i * (1 + e.nx);
  if (j == 0) row[0] = t;
  float x[4];
  sample_point_x4<KIND>(e, s, ig, j, t, x);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int d = 4 * j + q;
    if (d < e.nx) row[1 + d] = x[q];
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

constexpr int NTHB = 1024;  // GBM baseline workgroup: 16 waves (the Hessian-diagonal sweep)
constexpr int NTB = 256;    // Cha / OU baseline workgroup: k_baseline, and k_paths' fused base blocks
// Block-wide sum over NT threads in wave order (result on every thread); red: >= NT / 64 floats of LDS.
template <int NT>
__device__ __forceinline__ float block_sum_n(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float a = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) a += red[w];
  return a;
}

// Mat-vec of the per-point baseline, y[h] = sum_k Wt[k][h] v[k] (Wt row-major (K, H), H in {16, 32,
// 64, 128}, coalesced in h), over a block of NT threads: thread tid takes the 4 units 4 g .. 4 g + 3,
// g = tid % (H / 4), and the k-slice tid / (H / 4) of NT / (H / 4) slices (<= 4096 / NT k per slice),
// one 16-B load per k, all in flight before the first FMA (the r05 stamps had unit-per-thread slice
// loads at ~22 B/clk into the CU, profiles/r05q_base_stamps_matvec.txt); the wave's slices of a unit
// (lanes g + (H / 4) s) are added by lane swaps (their xor tree over s), the waves' partials in wave
// order by the unit's owner — a fixed order.  Returns y[tid] for tid < H; the caller's barrier
// precedes the next use of part.
template <int NT>
__device__ __forceinline__ float base_matvec(const float* __restrict__ Wt, const float* v, int K, int H,
                                             float (*part)[HMAX]) {
  constexpr int KCM = HMAX * HMAX / 4 / NT;  // max k per slice
  const int tid = threadIdx.x;
  const int G4 = H >> 2, g = tid % G4, sl = tid / G4, ns = NT / G4;
  const int kc = (K + ns - 1) / ns, k0 = sl * kc;
  float4 w[KCM];
#pragma unroll
  for (int j = 0; j < KCM; ++j)  // all loads in flight
    w[j] = (j < kc && k0 + j < K) ? *reinterpret_cast<const float4*>(Wt + (size_t)(k0 + j) * H + 4 * g)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < KCM; ++j)
    if (j < kc && k0 + j < K) {
      const float vk = v[k0 + j];
      a[0] = fmaf(w[j].x, vk, a[0]);
      a[1] = fmaf(w[j].y, vk, a[1]);
      a[2] = fmaf(w[j].z, vk, a[2]);
      a[3] = fmaf(w[j].w, vk, a[3]);
    }
  // lanes g + G4 s of this wave hold the same units: sum them over the lane bits >= log2(G4)
  for (int o = G4; o < 64; o <<= 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] += __shfl_xor(a[r], o, 64);
  if ((tid & 63) < G4) *reinterpret_cast<float4*>(&part[tid >> 6][4 * g]) = make_float4(a[0], a[1], a[2], a[3]);
  __syncthreads();
  float y = 0.f;
  if (tid < H)
#pragma unroll
    for (int j = 0; j < NT / 64; ++j) y += part[j][tid];
  return y;
}
// The same mat-vec for K up to NXW_MAX (a wide layer 1): each slice's k in passes of KCM, in order.
template <int NT>
__device__ __forceinline__ float base_matvec_wide(const float* __restrict__ Wt, const float* v, int K, int H,
                                               float (*part)[HMAX]) {
  constexpr int KCM = HMAX * HMAX / 4 / NT;
  const int tid = threadIdx.x;
  const int G4 = H >> 2, g = tid % G4, sl = tid / G4, ns = NT / G4;
  const int kc = (K + ns - 1) / ns, k0 = sl * kc;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < kc; kb += KCM) {
    float4 w[KCM];
#pragma unroll
    for (int j = 0; j < KCM; ++j)
      w[j] = (kb + j < kc && k0 + kb + j < K) ? *reinterpret_cast<const float4*>(Wt + (size_t)(k0 + kb + j) * H + 4 * g)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < KCM; ++j)
      if (kb + j < kc && k0 + kb + j < K) {
        const float vk = v[k0 + kb + j];
        a[0] = fmaf(w[j].x, vk, a[0]);
        a[1] = fmaf(w[j].y, vk, a[1]);
        a[2] = fmaf(w[j].z, vk, a[2]);
        a[3] = fmaf(w[j].w, vk, a[3]);
      }
  }
  for (int o = G4; o < 64; o <<= 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] += __shfl_xor(a[r], o, 64);
  if ((tid & 63) < G4) *reinterpret_cast<float4*>(&part[tid >> 6][4 * g]) = make_float4(a[0], a[1], a[2], a[3]);
  __syncthreads();
  float y = 0.f;
  if (tid < H)
#pragma unroll
    for (int j = 0; j < NT / 64; ++j) y += part[j][tid];
  return y;
}

// Per-point baseline scratch: k_baseline's LDS, and an overlay of the path LDS in k_paths' fused
// base blocks (a workgroup runs one role).
template <int NT>
struct BaseLds {
  __attribute__((aligned(16))) float part[NT / 64][HMAX];
  float xs[NXW_MAX];
  float act[4][HMAX];
  float dbuf[2][HMAX];
  float red[NT / 64];
  float redn[NT / 64][NSG];
  float ts;
};

// The fused launch's per-point baseline record: [g(x), f_b, pad to 32][bx: HMAX], 640 B, so no
// 128-B line holds values of two points (each point's values are handed off on their own).
constexpr int BREC = 32 + HMAX;

// Baseline of point i over a block of NT threads (Cha / OU; GBM: k_baseline_gbm): g(x), the
// state-dependent part of f(t, x, u, grad u) and bx = b1 + W1[:,1:] x (picard/data.py:918-920
// g_single, :506-518 f_baseline).  A latency-bound chain of block-wide mat-vecs (weights read
// coalesced through the transposed copies).  smp.tx != null: the block first samples its point
// (draws 1-3, k_sample_points' arithmetic) into smp.tx and its LDS copy; tickets != null: zero the
// point's ticket of the fused label reduce; rec != null: the values also go to the point's record.
// WIDE: also nx > 128 (k_baseline; the fused launch's base blocks serve nx <= 128 only and keep
// round 5's code)
template <int KIND, bool ZERO, int NT, bool WIDE = true>
__device__ __forceinline__ void base_point(const EqDev& e, const NetDev& net, const float* __restrict__ tx, int i,
                                           float* __restrict__ gx, float* __restrict__ fb, float* __restrict__ bx,
                                           float* __restrict__ rec, const SampleSpec& smp, int* __restrict__ tickets,
                                           BaseLds<NT>& bs) {
  static_assert(KIND != DPI_EQ_GBM, "GBM: k_baseline_gbm");
  static_assert(NT >= NXP_MAX && NT % 64 == 0, "one thread per padded state dimension");
  const int tid = threadIdx.x;
  const int nx = e.nx, F = 1 + nx;
  float* const r = rec ? rec + (size_t)i * BREC : nullptr;
  if (tickets && tid == 0) tickets[i] = 0;
  if (smp.tx) {
    const uint32_t ig = smp.point_base + (uint32_t)i;
    const int nb = (nx + 3) >> 2;
    float* row = smp.tx + (size_t)i * F;
    if (tid < nb) {
      const float tt = sample_point_t(e, smp, ig);
      if (tid == 0) {
        row[0] = tt;
        bs.ts = tt;
      }
      float x[4];
      sample_point_x4<KIND>(e, smp, ig, tid, tt, x);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * tid + q;
        if (d < nx) row[1 + d] = x[q];
        bs.xs[d] = d < nx ? x[q] : 0.f;
      }
    } else if (4 * nb <= tid && tid < NXP_MAX) {
      bs.xs[tid] = 0.f;
    }
  } else {
    const float* row = tx + (size_t)i * F;
    if (tid == 0) bs.ts = row[0];
    if (tid < NXP_MAX) bs.xs[tid] = tid < nx ? row[1 + tid] : 0.f;
    if (WIDE && nx > NXP_MAX)  // wide problems: the rest of x (only dims < nx are read)
      for (int d = NXP_MAX + tid; d < nx; d += NT) bs.xs[d] = row[1 + d];
  }
  __syncthreads();
  const float t = bs.ts;
  // g(x): per-thread dims, then per-statistic block sums in wave order (one barrier pair)
  {
    float st[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) st[c] = 0.f;
    for (int d = tid; d < nx; d += NT) Eq<KIND>::gstat(e, d, bs.xs[d], st);
#pragma unroll
    for (int c = 0; c < NSG; ++c) st[c] = wave_sum(st[c]);
    if ((tid & 63) == 0)
#pragma unroll
      for (int c = 0; c < NSG; ++c) bs.redn[tid >> 6][c] = st[c];
    __syncthreads();
    if (tid == 0) {
#pragma unroll
      for (int c = 0; c < NSG; ++c) {
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) a += bs.redn[w][c];
        st[c] = a;
      }
      const float g = Eq<KIND>::gfin(e, st);
      gx[i] = g;
      if (r) r[0] = g;
    }
  }
  if (ZERO) {
    if (tid == 0) {
      const float f = Eq<KIND>::ffv(e, 0.f, 0.f, 0.f, 0.f);
      fb[i] = f;
      if (r) r[1] = f;
    }
    return;
  }
  const int H = net.H, L = net.L, nxp = net.nxp;
  // layer 1
  {
    const float acc = (!WIDE || nx <= NXP_MAX) ? base_matvec<NT>(net.W1xT, bs.xs, nx, H, bs.part)
                                               : base_matvec_wide<NT>(net.W1xT, bs.xs, nx, H, bs.part);
    if (tid < H) {
      const float v = net.b1[tid] + acc;
      bx[(size_t)i * H + tid] = v;
      if (r) r[32 + tid] = v;
      bs.act[0][tid] = act_f(net.act, fmaf(net.w1t[tid], t, v));
    }
    __syncthreads();
  }
  for (int l = 1; l < L; ++l) {
    const float acc = base_matvec<NT>(net.WT[l], bs.act[l - 1], H, H, bs.part);
    if (tid < H) bs.act[l][tid] = act_f(net.act, acc + net.b[l][tid]);
    __syncthreads();
  }
  const float u = block_sum_n<NT>(tid < H ? net.wout[tid] * bs.act[L - 1][tid] : 0.f, bs.red) + net.bout;
  int cur = 0;
  if (tid < H) bs.dbuf[0][tid] = net.wout[tid] * act_d(net.act, bs.act[L - 1][tid]);
  __syncthreads();
  for (int l = L - 2; l >= 0; --l) {
    // W_{l+1} (H_out, H_in) row-major is the transposed operand of this mat-vec
    const float acc = base_matvec<NT>(net.W[l + 1], bs.dbuf[cur], H, H, bs.part);
    if (tid < H) bs.dbuf[cur ^ 1][tid] = acc * act_d(net.act, bs.act[l][tid]);
    cur ^= 1;
    __syncthreads();
  }
  float gs = 0.f, gA = 0.f, gB = 0.f;
  if (!Eq<KIND>::GRAD_FULL) {
    gs = block_sum_n<NT>(tid < H ? net.c1[tid] * bs.dbuf[cur][tid] : 0.f, bs.red);
  } else {
    float A = 0.f, B = 0.f;
    for (int d = tid; d < nx; d += NT) {
      float z = 0.f;
      for (int k = 0; k < H; ++k) z = fmaf(net.W1x[(size_t)k * nxp + d], bs.dbuf[cur][k], z);
      Eq<KIND>::gacc(e, d, bs.xs[d], z, A, B);
    }
    gA = block_sum_n<NT>(A, bs.red);
    gB = block_sum_n<NT>(B, bs.red);
  }
  if (tid == 0) {
    const float f = Eq<KIND>::ffv(e, u, gs, gA, gB);  // state-dependent part
    fb[i] = f;
    if (r) r[1] = f;
  }
}

// Per-point baseline launch (Cha / OU): one NTB-thread workgroup per point.
template <int KIND, bool ZERO>
__global__ __launch_bounds__(NTB) void k_baseline(EqDev e, NetDev net, const float* __restrict__ tx, int n,
                                                 float* __restrict__ gx, float* __restrict__ fb,
                                                 float* __restrict__ bx, SampleSpec smp, int* __restrict__ tickets) {
  __shared__ BaseLds<NTB> bs;
  (void)n;
  base_point<KIND, ZERO, NTB>(e, net, tx, blockIdx.x, gx, fb, bx, nullptr, smp, tickets, bs);
}

// GBM per-point baseline (one 1024-thread workgroup per point): g(x), the exact-solution part of
// ffi at (t, x) (equations.py:457-466), bx = b1 + W1[:,1:] x and the network's Hessian diagonal at
// (t, x) for the SDGD baseline gather (data.py:1293-1302).  smp / tickets as base_point.
// NXW = NXW_MAX: the wide instance (nx <= 256), whose tangent sweep runs once per 128 columns.
template <bool ZERO, int NXW = NXP_MAX>
__global__ __launch_bounds__(NTHB) void k_baseline_gbm(EqDev e, NetDev net, const float* __restrict__ tx, int n,
                                                      float* __restrict__ gx, float* __restrict__ fb,
                                                      float* __restrict__ bx, float* __restrict__ hb, SampleSpec smp,
                                                      int* __restrict__ tickets) {
  constexpr int KIND = DPI_EQ_GBM;
  __shared__ float xs[NXW];
  __shared__ float act[4][HMAX];
  __shared__ float red[NTHB / 64];
  __shared__ float ts;
  (void)n;
  const int i = blockIdx.x, tid = threadIdx.x;
  const int nx = e.nx, F = 1 + nx;
  if (tickets && tid == 0) tickets[i] = 0;
  if (smp.tx) {
    const uint32_t ig = smp.point_base + (uint32_t)i;
    const int nb = (nx + 3) >> 2;
    float* row = smp.tx + (size_t)i * F;
    if (tid < nb) {
      const float tt = sample_point_t(e, smp, ig);
      if (tid == 0) {
        row[0] = tt;
        ts = tt;
      }
      float x[4];
      sample_point_x4<KIND>(e, smp, ig, tid, tt, x);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * tid + q;
        if (d < nx) row[1 + d] = x[q];
        xs[d] = d < nx ? x[q] : 0.f;
      }
    } else if (4 * nb <= tid && tid < NXW) {
      xs[tid] = 0.f;
    }
  } else {
    const float* row = tx + (size_t)i * F;
    if (tid == 0) ts = row[0];
    for (int d = tid; d < NXW; d += NTHB) xs[d] = d < nx ? row[1 + d] : 0.f;
  }
  __syncthreads();
  const float t = ts;
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
  // exact-solution part of ffi at (t, x) (equations.py:457-466); the NSG dot products w_c . x
  // reduced together (one barrier pair instead of one per component, each sum in block_sum_n's order)
  float arg[NSG], sn[NSG];
  {
    __shared__ float redw[NTHB / 64][NSG];
    float v[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      v[c] = 0.f;
      if (c < e.nodes)
        for (int d = tid; d < nx; d += NTHB) v[c] = fmaf(e.gw[c * F + 1 + d], xs[d], v[c]);
      v[c] = wave_sum(v[c]);
    }
    __syncthreads();
    if ((tid & 63) == 0)
#pragma unroll
      for (int c = 0; c < NSG; ++c) redw[tid >> 6][c] = v[c];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      float a = 0.f;
      for (int w = 0; w < NTHB / 64; ++w) a += redw[w][c];
      arg[c] = c < e.nodes ? fmaf(e.gw[c * F], t, a) : 0.f;
      sn[c] = __sinf(arg[c]);
    }
  }
  const float ah = block_sum_n<NTHB>(Eq<KIND>::abs_hess_partial(e, sn, tid, NTHB), red);
  const float Cb = Eq<KIND>::exact_scalar_terms(e, arg) - 0.25f * ah;
  if (ZERO) {
    for (int d = tid; d < NXW; d += NTHB) hb[(size_t)i * HBS + d] = 0.f;
    if (tid == 0) fb[i] = Cb;
    return;
  }
  const int H = net.H, L = net.L, nxp = net.nxp;
  __shared__ __attribute__((aligned(16))) float part[NTHB / 64][HMAX];
  // layer 1
  {
    const float acc = base_matvec<NTHB>(net.W1xT, xs, nx, H, part);
    if (tid < H) {
      bx[(size_t)i * H + tid] = net.b1[tid] + acc;
      act[0][tid] = act_f(net.act, fmaf(net.w1t[tid], t, net.b1[tid] + acc));
    }
    __syncthreads();
  }
  for (int l = 1; l < L; ++l) {
    const float acc = base_matvec<NTHB>(net.WT[l], act[l - 1], H, H, part);
    if (tid < H) act[l][tid] = act_f(net.act, acc + net.b[l][tid]);
    __syncthreads();
  }
  // Hessian diagonal at (t, x): adjoints lam_l = du/da_l, then one thread per state dimension
  // runs its first-order tangent chain (column-major in LDS) and contracts with lam_l * elu''.
  __shared__ float lamb[4][HMAX];
  __shared__ float cb[HMAX];
  __shared__ __attribute__((aligned(16))) float ztb[2][64][NXP_MAX];
  if (tid < H) lamb[L - 1][tid] = net.wout[tid];
  __syncthreads();
  // adjoints: lam_l = W_{l+1}^T (elu'(a_{l+1}) * lam_{l+1}), a k-sliced mat-vec over the block with
  // every weight load in flight (W_{l+1} row-major (H_out, H_in) is its transposed operand)
  for (int l = L - 2; l >= 0; --l) {
    if (tid < H) cb[tid] = act_d(net.act, act[l + 1][tid]) * lamb[l + 1][tid];
    __syncthreads();
    const float acc = base_matvec<NTHB>(net.W[l + 1], cb, H, H, part);
    if (tid < H) lamb[l][tid] = acc;
    __syncthreads();
  }
  // Tangent sweep as an LDS mat-mat per layer, Z_l[h][d] = sum_k W_l[h][k] elu'(a_{l-1}[k])
  // Z_{l-1}[k][d]: thread t < 512 owns rows h = hg + 16 j (j < H / 16 <= 4) and columns
  // d = 4 dg .. 4 dg + 3 (hg = t / 32, dg = t % 32), 16 accumulators.  k runs outermost in steps
  // of 4: per step one float4 of Z per k and one broadcast float4 of scaled weights per row, a
  // third of the LDS return bytes of the column-per-thread form, which was bound by them (2.4 MB
  // per layer; 22 K cycles of the launch's 87 K, tools/base_stamps.py r05j).  Every output is the
  // same k-ascending fma chain as before; only the row grouping of the u_dd partials changed.
  __shared__ __attribute__((aligned(16))) float wsc[64 * 64];
  __shared__ float udp[16][NXP_MAX];
  const bool sw = tid < 512;
  const int dg = tid & 31, hg = (tid >> 5) & 15, RJ = (H + 15) >> 4;
  // columns c0 .. c0 + 127 of the diagonal per pass (one pass for NXW = 128)
#pragma unroll 1
  for (int c0 = 0; c0 < NXW; c0 += NXP_MAX) {
  if (NXW > NXP_MAX && c0 >= nx) break;
  float ud[4] = {0.f, 0.f, 0.f, 0.f};
  if (sw) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = hg + 16 * j;
      if (j < RJ && h < H) {
        float z[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = c0 + 4 * dg + q;
          z[q] = d < nx ? net.W1x[(size_t)h * nxp + d] : 0.f;
        }
        *reinterpret_cast<float4*>(&ztb[0][h][4 * dg]) = make_float4(z[0], z[1], z[2], z[3]);
        const float c = lamb[0][h] * act_d2(net.act, act[0][h]);
#pragma unroll
        for (int q = 0; q < 4; ++q) ud[q] = fmaf(c, z[q] * z[q], ud[q]);
      }
    }
  }
  int cz = 0;
  const int H4 = H & ~3;
  for (int l = 1; l < L; ++l) {
    for (int q = tid; q < H * H; q += NTHB) {
      const int h = q / H, k = q - h * H;
      wsc[h * 64 + k] = net.W[l][q] * act_d(net.act, act[l - 1][k]);
    }
    __syncthreads();  // wsc and Z_{l-1} complete
    if (sw) {
      float z[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) z[j][q] = 0.f;
#pragma unroll 1
      for (int k = 0; k < H4; k += 4) {
        const float4 z0 = *reinterpret_cast<const float4*>(&ztb[cz][k][4 * dg]);
        const float4 z1 = *reinterpret_cast<const float4*>(&ztb[cz][k + 1][4 * dg]);
        const float4 z2 = *reinterpret_cast<const float4*>(&ztb[cz][k + 2][4 * dg]);
        const float4 z3 = *reinterpret_cast<const float4*>(&ztb[cz][k + 3][4 * dg]);
        const float a0[4] = {z0.x, z0.y, z0.z, z0.w}, a1[4] = {z1.x, z1.y, z1.z, z1.w};
        const float a2[4] = {z2.x, z2.y, z2.z, z2.w}, a3[4] = {z3.x, z3.y, z3.z, z3.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < RJ && hg + 16 * j < H) {
            const float4 w = *reinterpret_cast<const float4*>(&wsc[(hg + 16 * j) * 64 + k]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
              z[j][q] = fmaf(w.w, a3[q], fmaf(w.z, a2[q], fmaf(w.y, a1[q], fmaf(w.x, a0[q], z[j][q]))));
          }
      }
      for (int k = H4; k < H; ++k) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < RJ && hg + 16 * j < H)
#pragma unroll
            for (int q = 0; q < 4; ++q) z[j][q] = fmaf(wsc[(hg + 16 * j) * 64 + k], ztb[cz][k][4 * dg + q], z[j][q]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = hg + 16 * j;
        if (j < RJ && h < H) {
          *reinterpret_cast<float4*>(&ztb[cz ^ 1][h][4 * dg]) = make_float4(z[j][0], z[j][1], z[j][2], z[j][3]);
          const float c = lamb[l][h] * act_d2(net.act, act[l][h]);
#pragma unroll
          for (int q = 0; q < 4; ++q) ud[q] = fmaf(c, z[j][q] * z[j][q], ud[q]);
        }
      }
    }
    cz ^= 1;
    __syncthreads();  // before wsc is overwritten
  }
  if (sw)
#pragma unroll
    for (int q = 0; q < 4; ++q) udp[hg][4 * dg + q] = ud[q];
  __syncthreads();
  if (tid < NXP_MAX) {
    float a = 0.f;
    for (int g = 0; g < 16; ++g) a += udp[g][tid];
    hb[(size_t)i * HBS + c0 + tid] = c0 + tid < nx ? a : 0.f;
  }
  if (NXW > NXP_MAX) __syncthreads();  // udp and ztb are reused by the next pass
  }
  if (tid == 0) fb[i] = Cb;
}

struct PathArgs {
  const float* tx;
  const float* gx;
  const float* fb;
  const float* bx;
  const float* hb;  // GBM: baseline Hessian diagonal [n][HBS]
  float* partial;
  int n, nbp, m_begin, K, flags;
  uint32_t k0, k1, c3t, c3s, c3i, c3q, point_base;
  int order;  // phase order policy (k_paths)
  int split;  // fused MLP on the fp16-split MFMA
  // Hessian labels: every block's sums as packed upper-triangle 16 x 16 tiles,
  // hpart [n][nbp][NT (NT + 1) / 2][256] (hess_store)
  float* hpart;
  uint32_t c3h1, c3h2;     // Hessian labels: Malliavin normal streams (tags HTERM, HINT)
  // DATA.ESTIMATE_DELTA_T (data.py:1209-1213): > 0 selects the TD estimators (k_paths<.., TD>),
  // horizon t_next = min(t + td_dt, T), terminal value u(t_next, X) where t_next < T
  float td_dt;
  // fused label reduce (tickets != null; first-order labels, nbp <= 64): the last block of a point
  // reduces its nbp slab rows in k_reduce's canonical tree and writes moments / labels (rd_*: the
  // arguments k_reduce would take)
  int* tickets;
  float* rd_moments;
  float* rd_y;
  int* rd_status;
  float rd_invM, rd_bound;
  int rd_add_g;
  // GBM prepared calls (dpi_label_prepare): the noise sums of phase 1, already rolled out by
  // k_noise_shared beside the previous batch's path launch, [n][nbp][2 (terminal, integral)][4 nb][P]
  const float* noise;
};

// The fused per-point baseline of k_paths_fb (dpi_sample_with_gradients as one launch: first-order
// Cha / OU labels of MLP and zero nets, no TD), an argument of that kernel only: blocks
// [0, nbase) run base_point for point blockIdx.x into rec and publish it on ready[i]; the path
// blocks (blockIdx.x - nbase) draw their point themselves (smp: bitwise the base block's draws) and
// wait for its record before they need it (base_poll, base_load).
struct FusedBase {
  int nbase;
  float* rec;                 // [n][BREC]
  unsigned long long* ready;  // [n]: (seq << 32) | ~seq once point i's record is out
  uint32_t ready_seq;
  SampleSpec smp;
};

// Fused baseline hand-off (MI355X_MICROARCH.md's producer / consumer forms): every storing wave
// waits for its stores, a workgroup barrier, then one lane's agent-scope release and a relaxed
// agent-scope store of the point's hand-off word.
__device__ __forceinline__ unsigned long long ready_word(uint32_t seq) {
  return ((unsigned long long)seq << 32) | (unsigned long long)(~seq);
}
__device__ __forceinline__ void base_publish(const FusedBase& fb, int i) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(fb.ready + i, ready_word(fb.ready_seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// Consumer: one lane polls (relaxed agent-scope loads, s_sleep between) and runs one agent-scope
// acquire (base_poll); a workgroup barrier the caller places after it; then every load of the record
// (base_ok() says whether it came).  The poll is bounded (about half a second): a record that never
// comes flags DPI_STATUS_HANDOFF and the point's labels NaN.
constexpr int BASE_SPIN_MAX = 1 << 20;
__device__ __forceinline__ int& base_ok() {
  __shared__ int ok;
  return ok;
}
__device__ __forceinline__ void base_poll(const FusedBase& fb, const PathArgs& a, int i) {
  if (threadIdx.x == 0) {
    const unsigned long long want = ready_word(fb.ready_seq);
    int it = 0;
    while (__hip_atomic_load(fb.ready + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want &&
           ++it < BASE_SPIN_MAX)
      __builtin_amdgcn_s_sleep(8);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool ok = it < BASE_SPIN_MAX;
    base_ok() = ok;
    if (!ok && a.rd_status) *(volatile int*)a.rd_status = DPI_STATUS_HANDOFF | DPI_STATUS_NONFINITE;
  }
}
// A wave-uniform float into a scalar register (the builtin is int-typed: pass the bits)
__device__ __forceinline__ float uniform_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
// A record value as a vector load (a uniform address would otherwise be a scalar-cache load, which
// the acquire does not refresh)
__device__ __forceinline__ float rec_load(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Noise sums of a (point, block, estimator part, wave slice) task: exactly the K-step loops of
// k_paths' terminal / integral rollouts (same counters, same sequential sum per dimension, the same
// BM_SCALE product), so a path launch that reads them is bitwise the one that rolls out itself.
template <int UNR>
__device__ __forceinline__ void noise_task(const PathArgs& a, int nb, int t) {
  const int lane = threadIdx.x & 63;
  const int blkg = t >> 3, part = (t >> 2) & 1, wq = t & 3;  // 8 tasks per (point, block)
  const int i = blkg / a.nbp, blk = blkg - i * a.nbp;
  const uint32_t ig = a.point_base + (uint32_t)i;
  const uint32_t m = (uint32_t)(a.m_begin + P * blk + lane);
  const uint32_t c3 = part ? a.c3i : a.c3t;
  float* out = const_cast<float*>(a.noise) + ((size_t)blkg * 2 + part) * (4 * nb) * P + lane;
  if (!(a.flags & (part ? DPI_INTEGRAL : DPI_TERMINAL))) return;
  for (int j = wq; j < nb; j += 4) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    noise_sums<UNR>(a.K, nb, j, m, ig, c3, a.k0, a.k1, s0, s1, s2, s3);
    out[(4 * j + 0) * P] = s0 * BM_SCALE;
    out[(4 * j + 1) * P] = s1 * BM_SCALE;
    out[(4 * j + 2) * P] = s2 * BM_SCALE;
    out[(4 * j + 3) * P] = s3 * BM_SCALE;
  }
}

// The prepare stream's noise pre-pass for the GBM path launch (dpi_label_prepare): a work queue of
// the 8 n nbp one-wave tasks served by at most `waves` waves per SIMD, the pattern of
// k_pis_rollout_shared: the first waves of the launch on a SIMD claim it (per-SIMD word keyed by
// HW_ID and XCC_ID, zeroed with the queue counter before the launch) and take tasks until the queue
// is empty, every other wave leaves at once.  <= 48 registers and no LDS, so one such wave fits on
// each SIMD beside a k_paths<GBM> wave (<= 464 registers, 162 KB of LDS per CU) of the previous
// batch and issues VALU work in the slots its tangent sweep leaves idle.  Every wave reaches the
// exit: a claimed wave ends when the queue counter passes ntask.
#ifndef DPI_NOISE_SHARED_UNR
#define DPI_NOISE_SHARED_UNR 4
#endif
template <int UNR>
__global__ __launch_bounds__(64, 8) __attribute__((amdgpu_num_vgpr(24))) void k_noise_shared(PathArgs a, int nb,
                                                                                         int ntask, int* queue,
                                                                                         int* claim, int waves) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);         // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;  // HW_REG_XCC_ID
  const unsigned slot = (xcc << 10) | (((hw >> 8) & 0xffu) << 2) | ((hw >> 4) & 3u);
  const int lane = threadIdx.x & 63;
  int old = 0;
  if (lane == 0) old = atomicAdd(claim + slot, 1);
  if (__builtin_amdgcn_readfirstlane(old) >= waves) return;
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= ntask) break;
    noise_task<UNR>(a, nb, t);
  }
}

// ------------------------------------------------------------------------------ Hessian labels
// Malliavin-weight Hessian block of generate_with_gradients_and_hessians (picard/data.py:1220-1223;
// terminal :1185-1199, integral :869-881), per 64-path block, after phase 3 of k_paths:
//   H_blk = sum_p [ aI_p (N2 N2^T - I) + aT_p (N1 N1^T - I) ]
//   aI = (T-t) (f(s, x + a sqrt(s-t) N2) + f(s, x - ...) - 2 f_b) / 2 / (s-t)     (full Hessian f)
//   aT = (g(x + a sqrt(T-t) N1) + g(x - ...) - 2 g(x)) / 2 / (T-t)
// N1, N2: fresh normals (tags HTERM / HINT, k = 0), written into the noise tile in turn; the
// outer-product sums are (nx x 64) (64 x nx) products on v_mfma_f32_16x16x4_f32 over the upper
// triangle of 16 x 16 tiles (wave w owns tiles w, w+4, ...), mirrored on store.
// A block's Hessian sums out as packed upper-triangle tiles (the lower triangle is the mirror):
// tile q's element (r, c) at q 256 + (r & 3) 64 + (r >> 2) 16 + c, one 256-B run per store
// instruction — 28 tiles, 28 KB per block at nx = 100 against 40 KB for the full square.
__device__ __forceinline__ void hess_store(const PathArgs& a, const floatx4 (&acc)[9], int NT) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ntiles = NT * (NT + 1) / 2;
  float* out = a.hpart + (size_t)blockIdx.x * ntiles * 256;
#pragma unroll
  for (int sl = 0; sl < 9; ++sl) {
    const int q = wv + 4 * sl;
    if (q < ntiles)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) out[q * 256 + rr * 64 + lane] = acc[sl][rr];
  }
}

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

template <int KIND, int H, int L, bool ZERO, bool SPLIT, int ACT>
__device__ __forceinline__ void hess_block(const EqDev& e, const NetDev& net, const PathArgs& a, LdsGbm<H>& sh,
                                           int i, int blk, uint32_t ig, uint32_t m, float s, float smt, float tmt,
                                           float g_x, int nxp) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, jj = lane & 15, qq = lane >> 4, pp = 16 * wv + jj;
  const int nx = e.nx, F = 1 + nx, nb = (nx + 3) >> 2, NT = nxp / 16;
  // f at (s, x + cmul S) with the full Hessian diagonal (get_f without SDGD, data.py:1262-1272);
  // valid in the lanes of group qq == 0 for path pp
  auto f_eval = [&]() -> float {
    float s1 = 0.f, s2 = 0.f;
    if constexpr (!ZERO) {
      if constexpr (SPLIT)
        mlp_hdiag_split<H, L, ACT>(e, net, sh, nxp / 16, s1, s2);
      else
        mlp_hdiag<H, L, ACT>(e, net, sh, nxp / 16, s1, s2);
    }
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
  // a.flags selects the estimators (workgroup-uniform): a call over n_estimate_terminal paths with
  // DPI_TERMINAL and one over n_estimate_integral paths with DPI_INTEGRAL make the labels of unequal
  // sample counts (data.py:845 vs :1164), each with its own identity part
  const bool TERM = a.flags & DPI_TERMINAL, INTG = a.flags & DPI_INTEGRAL;
  float aI = 0.f, aT = 0.f;

  // ---- integral term: N2 -> noise tile, w . N2 for the exact-solution terms
  __syncthreads();  // phase 3 is done with the integral noise tile
  if (INTG) {
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
  aI = wgt[lane];  // lane = path
  hess_accum<H, L>(sh, wgt, NT, acc);
  }

  // ---- terminal term: N1 -> noise tile, g(x +- a sqrt(T-t) N1)
  if (TERM) {
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
  aT = (gplus + gminus - 2.f * g_x) * 0.5f / tmt;
  if (wv == 0) wgt[lane] = aT;
  __syncthreads();
  hess_accum<H, L>(sh, wgt, NT, acc);
  }

  // ---- identity part
  const float dsum = wave_sum(aI + aT);
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
        if (d1 == d2) acc[sl][rr] -= dsum;
      }
    }
  }
  hess_store(a, acc, NT);
}


// One workgroup = (point i, 64 consecutive MC indices).  See the file header.
// TD: the TD estimators (ESTIMATE_DELTA_T > 0, data.py:1209-1213, :934-952, :529-575): every
// T - t below becomes the horizon t_next - t, and where t_next = t + dt < T (workgroup-uniform:
// one point per workgroup) the terminal value is u(t_next, X_{t_next}), evaluated by the same MLP
// tile on the terminal noise before the integral rollout takes the noise tile.
// The label reduce of one point inside k_paths (a.tickets != null; nbp <= 64), replacing the
// k_reduce launch: every block publishes its slab row (each storing wave waits for its stores, a
// workgroup barrier, one lane's agent-scope release, then an agent-scope add to the point's
// ticket — MI355X_MICROARCH.md's producer form); the block whose add returns nbp - 1 acquires
// (agent scope) and reduces the point's nbp rows, one thread per column over the 64 zero-padded
// leaves as a perfect binary tree in block order — for nbp <= 64 exactly tree_sum's order, so the
// moments and labels are bitwise k_reduce's — then finalizes (/M, + g(x), clip) and zeroes the
// ticket for the next call (k_baseline zeroes it too).
// rec != null (k_paths_fb): g(x) from the point's baseline record
__device__ __forceinline__ void fused_reduce(const PathArgs& a, int i, int F, const float* rec) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores complete
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(a.tickets + i, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int is_last = prev == a.nbp - 1;
    if (is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last = is_last;
  }
  __syncthreads();
  if (!last) return;
  const int R = slab_row(F), nbp = a.nbp;
  const float* base = a.partial + (size_t)i * nbp * R;
  for (int c = threadIdx.x; c < 2 * F; c += NTH) {
    // the 64-leaf tree as four 16-leaf subtrees, (q0 + q1) + (q2 + q3): the same additions in the
    // same order, a quarter of the live registers (the tail runs inside the path kernel)
    float q[4];
#pragma unroll 1
    for (int h = 0; h < 4; ++h) {
      float v[16];
#pragma unroll
      for (int b = 0; b < 16; ++b) v[b] = 16 * h + b < nbp ? base[(size_t)(16 * h + b) * R + c] : 0.f;
#pragma unroll
      for (int w = 1; w < 16; w <<= 1)
#pragma unroll
        for (int b = 0; b < 16; b += 2 * w) v[b] = v[b] + v[b + w];
      q[h] = v[0];
    }
    const float sum = (q[0] + q[1]) + (q[2] + q[3]);
    if (c < F && a.rd_status && !__builtin_isfinite(sum)) *(volatile int*)a.rd_status = DPI_STATUS_NONFINITE;
    a.rd_moments[(size_t)i * 2 * F + c] = sum;
    if (a.rd_y && c < F) {
      float y = sum * a.rd_invM;
      if (c == 0 && a.rd_add_g) y += rec ? rec_load(rec + (size_t)i * BREC) : a.gx[i];
      a.rd_y[(size_t)i * F + c] = y != y ? y : fminf(fmaxf(y, -a.rd_bound), a.rd_bound);  // torch.clip
    }
  }
  if (threadIdx.x == 0) a.tickets[i] = 0;
}

// The path launch: one workgroup per (point, 64-path block).
// Two workgroups per CU (256 registers per wave) except GBM / TD (one: their LDS) and the exact-fp32
// OU 4 x 128 instance — the range guard's fallback for OU MLP nets — whose GMM statistics beside
// the 128 fp32 activation registers spilled 4 VGPRs at 256: it runs at one workgroup per CU instead.
// Wide instances (NXW > NXP_MAX): one (their 70 KB noise tile).
template <int KIND, int H, int L, bool SPLIT, bool TD, int NXW = NXP_MAX>
constexpr int k_paths_wgs() {
  return (KIND == DPI_EQ_GBM || TD || NXW > NXP_MAX || (KIND == DPI_EQ_OU && !SPLIT && H == 128 && L == 4)) ? 1 : 2;
}
// The path launch body; FBT: the one-launch sample_with_gradients form (k_paths_fb), whose first
// fb.nbase blocks are the points' base blocks — a kernel of its own, so the plain k_paths keeps its
// register allocation (the hand-off's arguments live across the whole kernel).
// NXW: the state-dimension cap of the instance (NXP_MAX; NXW_MAX for the wide first-order instances)
template <int KIND, int H, int L, bool ZERO, bool SPLIT, bool HESS, bool TD, int ACT, bool FBT, int NXW = NXP_MAX>
__device__ __forceinline__ void paths_body(const EqDev& e, const NetDev& net, const PathArgs& a, const FusedBase& fb) {
  static_assert(!HESS || KIND == DPI_EQ_GBM, "Hessian labels: GBM (SimpleDiffusionEquationWithHessian) only");
  static_assert(!(HESS && TD), "the Hessian-label estimators have no TD variant (data.py:1220-1223)");
  static_assert(NXW == NXP_MAX || (!HESS && !TD && !FBT && NXW % 128 == 0 && NXW <= NXW_MAX),
                "wide instances: first-order labels, no TD, no fused baseline");
  static_assert(!(KIND == DPI_EQ_GBM && NXW > NXP_MAX) || L <= 3, "wide GBM instances: the hidden weights of L <= 3");
  using SH = std::conditional_t<KIND == DPI_EQ_GBM, LdsGbm<H, NXW>, LdsT<NXW>>;
  constexpr int NBW = NXW / 16;  // dim-blocks of 4 per wave (4 waves)
  __shared__ SH sh;
  constexpr bool GBM = KIND == DPI_EQ_GBM;
  // fused baseline (k_paths_fb): the first fb.nbase blocks are the points' base blocks
  constexpr bool FBC = FBT && !GBM && !HESS && !TD;
  static_assert(FBC || !FBT, "the fused baseline: first-order Cha / OU labels, no TD");
  constexpr bool FB = FBC;
  if constexpr (FBC) {
    static_assert(sizeof(BaseLds<NTH>) <= sizeof(SH), "base blocks overlay the path LDS");
    if ((int)blockIdx.x < fb.nbase) {
      base_point<KIND, ZERO, NTH, false>(e, net, a.tx, blockIdx.x, const_cast<float*>(a.gx), const_cast<float*>(a.fb),
                                  const_cast<float*>(a.bx), fb.rec, fb.smp, a.tickets,
                                  *reinterpret_cast<BaseLds<NTH>*>(&sh));
      base_publish(fb, blockIdx.x);
      return;
    }
  }
  const unsigned bid = blockIdx.x - (FB ? (unsigned)fb.nbase : 0u);
  const int i = bid / a.nbp;
  const int blk = bid - i * a.nbp;
  // independent Philox chains per wave in the noise loops (2 vs 1: 2 % on the one- and two-wave-per-SIMD
  // kernels; 4 vs 2, round 3: 0.5 % first-order, 1.2 % GBM; round 4: GBM 8, Hessian labels 4)
  // (the u = 0 GBM instance keeps 4: at 8 its own allocation grew and the noise-floor launch ran
  // 801 K -> 1,077 K cycles, profiles/r04s_pmc / valu_gbm.json)
  constexpr int NOISE_UNROLL = HESS ? DPI_NOISE_UNROLL_HESS
                               : GBM ? (ZERO ? 4 : DPI_NOISE_UNROLL_GBM)
                                     : DPI_NOISE_UNROLL_FO;
  constexpr bool NOISE_WU = false;  // the plain philox4x32_10 (see wv below)
  // The wave index as the compiler sees it: divergent (tid >> 6), so the dim-block indices j and the
  // Philox counter words c0 = k nb + j live in VGPRs.  Made uniform (readfirstlane) with the
  // scalar-unit Philox (philox4x32_10_wu), the noise loop issues 195 instead of 216 VALU instructions
  // per 4 calls but 61 SALU more, and two waves per SIMD then issue slower: Burgers 0.360 -> 0.388
  // ms/step, Hessian labels 1.750 -> 1.784 (same-box A/B, profiles/r06o_ab); kept for the one-wave
  // k_noise_shared only.  DPI_WV_UNIFORM_GBM: the A/B knob for the GBM network launch.
  constexpr bool WV_UNIFORM = DPI_WV_UNIFORM_GBM && GBM && !HESS && !TD && NXW == NXP_MAX;
  const int tid = threadIdx.x, lane = tid & 63, wv = WV_UNIFORM ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const uint32_t ig = a.point_base + (uint32_t)i;
  const uint32_t m = (uint32_t)(a.m_begin + P * blk + lane);
  const int nx = e.nx, F = 1 + nx;
  const int nb = (nx + 3) >> 2;
  const int nxp = ZERO ? ((nx + 15) & ~15) : net.nxp;
  const bool TERM = a.flags & DPI_TERMINAL, INTG = a.flags & DPI_INTEGRAL;
  const float* txr = a.tx + (size_t)i * F;
  // fused baseline: the block draws its point itself (the base block's draws, bitwise)
  // (uniform: kept scalar, as the loaded t is)
  const float t = FB ? uniform_f(sample_point_t(e, fb.smp, ig)) : txr[0];
  // horizon: T - t, or for TD t_next - t = dt where t_next = t + dt < T (data.py:539, :940)
  bool td_u = false;
  float tmt = e.T - t;
  if constexpr (TD) {
    td_u = t + a.td_dt < e.T;
    if (td_u) tmt = a.td_dt;
  }
  float g_x = 0.f, f_b = 0.f;  // fused baseline: from the point's record (base_load)
  if (!FB) {
    g_x = a.gx[i];
    f_b = a.fb[i];
  }
  const float Kf = (float)a.K;
  // GBM prepared calls: phase 1's noise sums come from k_noise_shared (a wave-uniform branch)
  const bool PRE = GBM && !TD && a.noise != nullptr;  // first-order and Hessian labels

  if (FB) {
    if (tid < nb) {
      float x[4];
      sample_point_x4<KIND>(e, fb.smp, ig, tid, t, x);
#pragma unroll
      for (int q = 0; q < 4; ++q) sh.xsh[4 * tid + q] = 4 * tid + q < nx ? x[q] : 0.f;
    }
    for (int d = 4 * nb + tid; d < nxp; d += NTH) sh.xsh[d] = 0.f;
  } else {
    for (int d = tid; d < nxp; d += NTH) sh.xsh[d] = d < nx ? txr[1 + d] : 0.f;
  }
  // the split MLP reads the tile's first nxp32 rows (32-row chunks; the host pads nxp with it when
  // it rounds a 96-word chunk up to 128, so this bound covers them)
  const int nxpz = (nxp + 31) & ~31;
  for (int idx = tid; idx < (nxpz - 4 * nb) * P; idx += NTH) {  // zero pad rows of the noise tile
    const int d = 4 * nb + idx / P, p = idx % P;
    sh.S[d * SS + p] = 0.f;
  }
  if (!ZERO) {
    for (int h = tid; h < H; h += NTH) {
      if (!FB) sh.vec[h] = a.bx[(size_t)i * H + h];  // b1 + W1x x (from k_baseline; fused: base_load)
      sh.vec[H + h] = net.w1t[h];
      sh.vec[2 * H + h] = net.wout[h];
      sh.vec[3 * H + h] = net.c1[h];
    }
    for (int l = 1; l < L; ++l)
      for (int h = tid; h < H; h += NTH) sh.bh[l * H + h] = net.b[l][h];
  }
  if constexpr (GBM) {
    if (!ZERO) {  // all weights resident for the tangent sweep (wide instances: W1x from L2)
      [[maybe_unused]] constexpr int WXS = SH::WXS;
      constexpr int WHS = SH::WHS;
      if constexpr (SH::W1X_LDS)
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
    for (int d = tid; d < nxp; d += NTH) sh.hb[d] = d < nx ? a.hb[(size_t)i * HBS + d] : 0.f;
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
  float ST[NBW][4];
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
    for (int c = 0; c < NBW; ++c) {
      const int j = wv + 4 * c;  // terminal dim-blocks of this wave
      ST[c][0] = ST[c][1] = ST[c][2] = ST[c][3] = 0.f;
      if (TERM && j < nb) {
        if (PRE) {  // rolled out by k_noise_shared (GBM prepared calls)
          const float* np = a.noise + ((size_t)(i * a.nbp + blk) * 2) * (4 * nb) * P + lane;
#pragma unroll
          for (int q = 0; q < 4; ++q) ST[c][q] = np[(4 * j + q) * P];
        } else {
          float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
          noise_sums<NOISE_UNROLL, NOISE_WU>(a.K, nb, j, m, ig, a.c3t, a.k0, a.k1, s0, s1, s2, s3);
          ST[c][0] = s0 * BM_SCALE;
          ST[c][1] = s1 * BM_SCALE;
          ST[c][2] = s2 * BM_SCALE;
          ST[c][3] = s3 * BM_SCALE;
        }
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
    for (int c = 0; c < NBW; ++c) {
      const int j = (3 - wv) + 4 * c;  // integral dim-blocks of this wave (balances 13/12/12/13)
      if (j < nb) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        if (INTG && !PRE) {
          noise_sums<NOISE_UNROLL, NOISE_WU>(a.K, nb, j, m, ig, a.c3i, a.k0, a.k1, s0, s1, s2, s3);
        }
        float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
        if (INTG && PRE) {  // rolled out by k_noise_shared (GBM prepared calls)
          const float* np = a.noise + ((size_t)(i * a.nbp + blk) * 2 + 1) * (4 * nb) * P + lane;
#pragma unroll
          for (int q = 0; q < 4; ++q) sv[q] = np[(4 * j + q) * P];
        }
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
          mlp_tile_split<KIND, H, L, ACT>(e, net, sh, u, gs, gA, gB);
        else
          mlp_tile<KIND, H, L, ACT>(e, net, sh, nxp / 16, u, gs, gA, gB, nullptr, 0, P);
      }
      const int pp = 16 * wv + (lane & 15);
      if ((lane >> 4) == 0) sh.bsh[pp] = INTG ? tmt * (Eq<KIND>::ffv(e, u, gs, gA, gB) - f_b) : 0.f;
    } else {
      // ffi (equations.py:457-466) with u_ii from SDGD (data.py:1273-1303); the baseline f_b
      // gathers the point's Hessian diagonal at this path's indices (data.py:1293-1302).
      const int jj = lane & 15, qq = lane >> 4, pp = 16 * wv + jj;
      float s1 = 0.f, s2 = 0.f;
      if constexpr (!ZERO) {
        if (INTG) {
          if constexpr (SPLIT)
            mlp_hdiag_split<H, L, ACT>(e, net, sh, nxp / 16, s1, s2);
          else
            mlp_hdiag<H, L, ACT>(e, net, sh, nxp / 16, s1, s2);
        }
      }
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
  if constexpr (TD) {
    tlast = false;  // the terminal MLP needs the noise tile before the integral rollout
  } else if constexpr (SPLIT && !GBM) {
    tlast = true;  // measured faster, and the terminal sums are not live across the MLP (no spills)
  } else if constexpr (!GBM) {
    if (a.order == 1) tlast = (__builtin_amdgcn_s_getreg((3 << 11) | (16 << 6) | 4) & 1) != 0;  // HW_ID.TG_ID
    else if (a.order == 2) tlast = (bid & 1) != 0;
    else if (a.order == 3) tlast = ((bid >> 8) & 1) != 0;
    else if (a.order == 4) tlast = true;
  }
  // TD terminal value u(t_next, x + cT S_T) (data.py:941-942), per lane = path
  [[maybe_unused]] auto terminal_value_td = [&]() -> float {
#pragma unroll
    for (int c = 0; c < NBW; ++c) {
      const int j = wv + 4 * c;
      if (j < nb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = 4 * j + q;
          sh.S[d * SS + lane] = d < nx ? ST[c][q] : 0.f;
        }
    }
    if (wv == 0) {
      sh.tau[lane] = t + a.td_dt;
      sh.cmul[lane] = cT;
    }
    __syncthreads();
    float u = 0.f;
    if constexpr (!ZERO) {
      if constexpr (GBM) {
        u = mlp_value_res<H, L, ACT>(net, sh, nxp / 16);
      } else {
        float gs, gA, gB;
        if constexpr (SPLIT)
          mlp_tile_split<KIND, H, L, ACT>(e, net, sh, u, gs, gA, gB);
        else
          mlp_tile<KIND, H, L, ACT>(e, net, sh, nxp / 16, u, gs, gA, gB, nullptr, 0, P);
      }
    }
    const int pp = 16 * wv + (lane & 15);
    if ((lane >> 4) == 0) sh.bsh[pp] = u;
    __syncthreads();
    const float uT = sh.bsh[lane];
    if (wv == 0) {
      sh.tau[lane] = s;
      sh.cmul[lane] = cI;
    }
    // the integral rollout's writes into S are published by terminal_finish's barrier
    return uT;
  };
  // fused baseline: the point's record, before the first use of g(x), f_b or bx.  base_poll runs on
  // lane 0 ahead of a workgroup barrier (in the terminal-last order the one after the integral
  // rollout, so the acquire overlaps the waves still rolling out); base_load after it.
  auto base_poll_ = [&]() {
    if constexpr (FBC) base_poll(fb, a, i);
  };
  auto base_load = [&]() {
    if constexpr (FBC) {
      const bool ok = base_ok() != 0;
      const float* r = fb.rec + (size_t)i * BREC;
      g_x = uniform_f(ok ? rec_load(r) : __builtin_nanf(""));  // uniform: scalar
      f_b = uniform_f(ok ? rec_load(r + 1) : __builtin_nanf(""));
      if (!ZERO) {
        for (int h = tid; h < H; h += NTH) sh.vec[h] = r[32 + h];
        __syncthreads();
      }
    }
  };
  float ap;
  if constexpr (TD) {
    terminal_rollout();
    float uT = 0.f;
    if (td_u && TERM) uT = terminal_value_td();
    integral_rollout();
    ap = terminal_finish();
    if (td_u) ap = TERM ? uT - g_x : 0.f;  // (u(t_next, X) - g(x)) (data.py:942, :947)
    integrand();
    __syncthreads();
  } else if (!tlast) {
    terminal_rollout();
    integral_rollout();
    if constexpr (FBC) {
      base_poll_();
      __syncthreads();
      base_load();
    }
    ap = terminal_finish();
    integrand();
    __syncthreads();
  } else {
    integral_rollout();
    base_poll_();
    __syncthreads();
    base_load();
    integrand();
    terminal_rollout();
    ap = terminal_finish();  // its barrier also publishes bsh
  }

  // ---------------- phase 3: per-path contributions -> per-block partial slab
  const float bp = sh.bsh[lane];
  // partial slab layout [point][block][slab_row(F)]: this workgroup's 2F sums are one contiguous,
  // 128-B aligned row, so every HBM line of the slab is written from a single XCD (a column-major
  // [point][2F][block] slab had the blocks of one line written from all eight XCDs' L2s, each
  // writing its dirty bytes back separately: 7.8x the slab in WRITE_SIZE)
  float* out = a.partial + ((size_t)i * a.nbp + blk) * slab_row(F);
  // per-block sums of c and c^2 for this wave's columns: 2 per owned dim (d = 4 (wv + 4c) + q,
  // column 8c + 2q + {0: sum, 1: sum of squares}) and, on wave 0, the value column (56, 57)
  const float aY = ap * yT, bY = bp * yI;
  if constexpr (NXW == NXP_MAX) {
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
        if (wv + 4 * c < nb && d < nx) out[sq * F + 1 + d] = tot;
      } else if (wv == 0 && lane < 58) {
        out[sq * F] = tot;
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
            out[1 + d] = s1;
            out[F + 1 + d] = s2;
          }
        }
      }
    }
  } else {
    // wide instances: this wave's NBW dim-blocks in groups of 7 (56 columns), the value column with
    // the first group; one column_sums64 per group
#pragma unroll
    for (int g0 = 0; g0 < NBW; g0 += 7) {
      float col[64];
#pragma unroll
      for (int c = 0; c < 64; ++c) col[c] = 0.f;
#pragma unroll
      for (int c = 0; c < 7; ++c) {
        const int j = wv + 4 * (g0 + c);
        if (g0 + c < NBW && j < nb) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int d = 4 * j + q;
            const float v = d < nx ? fmaf(aY, ST[g0 + c < NBW ? g0 + c : 0][q], bY * sh.S[d * SS + lane]) : 0.f;
            col[8 * c + 2 * q] = v;
            col[8 * c + 2 * q + 1] = v * v;
          }
        }
      }
      if (g0 == 0 && wv == 0) {
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
      const int c = lane >> 3, q = (lane >> 1) & 3, sq = lane & 1;
      const int j = wv + 4 * (g0 + c), d = 4 * j + q;
      if (lane < 56) {
        if (g0 + c < NBW && j < nb && d < nx) out[sq * F + 1 + d] = tot;
      } else if (g0 == 0 && wv == 0 && lane < 58) {
        out[sq * F] = tot;
      }
    }
  }
  if constexpr (HESS) {
    hess_block<KIND, H, L, ZERO, SPLIT, ACT>(e, net, a, sh, i, blk, ig, m, s, smt, tmt, g_x, nxp);
  } else {
    if (a.tickets) fused_reduce(a, i, F, FB ? fb.rec : nullptr);
  }
}

template <int KIND, int H, int L, bool ZERO, bool SPLIT, bool HESS = false, bool TD = false, int ACT = DPI_ACT_ELU,
          int NXW = NXP_MAX>
__global__ __launch_bounds__(256, (k_paths_wgs<KIND, H, L, SPLIT, TD, NXW>())) void k_paths(EqDev e, NetDev net, PathArgs a) {
  paths_body<KIND, H, L, ZERO, SPLIT, HESS, TD, ACT, false, NXW>(e, net, a, FusedBase{});
}
// The one-launch dpi_sample_with_gradients: fb.nbase base blocks ahead of the path blocks.
template <int KIND, int H, int L, bool ZERO, bool SPLIT, int ACT = DPI_ACT_ELU>
__global__ __launch_bounds__(256, (k_paths_wgs<KIND, H, L, SPLIT, false>())) void k_paths_fb(EqDev e, NetDev net,
                                                                                            PathArgs a, FusedBase fb) {
  paths_body<KIND, H, L, ZERO, SPLIT, false, false, ACT, true>(e, net, a, fb);
}

}  // namespace dpi
