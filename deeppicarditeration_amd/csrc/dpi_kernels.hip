// C-ABI of include/dpi.h (libdpi_hip.so): problem / network handles, the PISGradNet pipeline
// host code, label moments, reduce and finalize kernels.  Device code: dpi_device.h; the per
// equation k_paths instantiations: dpi_paths_{cha,ou,gbm}.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <type_traits>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dpi.h"
#include "dpi_eq.h"
#include "dpi_rng.h"

#include "dpi_dispatch.h"
#include "dpi_pisnet.h"

namespace dpi {

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

// partial [n][nbp][slab_row(F)] -> moments [n][2F] (and, if y != nullptr, the finalized labels).
// torch.clip of the reference (data.py:222): NaN stays NaN (fmaxf alone would return -bound).
__device__ __forceinline__ float clip_label(float v, float bound) {
  return v != v ? v : fminf(fmaxf(v, -bound), bound);
}

// Range guard: a label sum that is not finite while the network's parameters are (status != null
// only then) means the network evaluation left its number format — fp16's 65,504 in the split
// storage of the PISGradNet pipeline, or fp32's range — where the fp64 reference would not.  The
// lane stores DPI_STATUS_NONFINITE into the net's sticky status word (a plain vector store: any
// number of writers store the same value); the host reads it with dpi_net_status.
__device__ __forceinline__ void flag_nonfinite(int* status, float s) {
  if (status && !__builtin_isfinite(s)) *(volatile int*)status = DPI_STATUS_NONFINITE;
}

__global__ __launch_bounds__(256) void k_reduce(const float* __restrict__ partial, int n, int F, int nbp,
                                                float* __restrict__ moments, const float* __restrict__ gx,
                                                float invM, int add_g, float bound, float* __restrict__ y,
                                                int ystride, int* status) {
  // a wave per (point, column): reading the slab's lines from several XCDs costs only duplicate
  // fetches of a 0.9 MB slab, while one workgroup per point serialised the columns (14 vs 4.4 us)
  const int i = blockIdx.x, R = slab_row(F);
  const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (c >= 2 * F) return;
  const float s = tree_sum(partial + (size_t)i * nbp * R + c, nbp, (size_t)R);
  if ((threadIdx.x & 63) == 0) {
    if (c < F) flag_nonfinite(status, s);  // the label sums (a sum of squares may overflow alone)
    moments[(size_t)i * 2 * F + c] = s;
    if (y && c < F) {
      float v = s * invM;
      if (c == 0 && add_g) v += gx[i];
      y[(size_t)i * ystride + c] = clip_label(v, bound);
    }
  }
}

// Offset of Hessian element (d1, d2) in one packed group sum of k_paths' Hessian labels
// (hess_store): upper-triangle 16 x 16 tiles of an NT x NT tiling in row order, tile element
// (r, c) at (r & 3) 64 + (r >> 2) 16 + c; (d1, d2) and (d2, d1) read the same word (symmetric labels).
__device__ __forceinline__ int hess_packed_off(int d1, int d2, int NT) {
  const int a = min(d1, d2), b = max(d1, d2);
  const int I = a >> 4, J = b >> 4, r = a & 15, c = b & 15;
  const int q = I * NT - ((I * (I - 1)) >> 1) + (J - I);
  return q * 256 + (r & 3) * 64 + (r >> 2) * 16 + c;
}

// tree_sum's canonical order in ONE thread: the perfect binary tree, left + right at every level,
// over cnt values zero-padded to P2 = max(64, 2^ceil(log2 cnt)) leaves — bitwise tree_sum's result
// (and every power-of-two sharding of the leaves still reproduces it).  Up to 64 leaves the tree
// runs unrolled in registers; beyond, as a binary counter over the leaves (level l holds the left
// subtree of 2^l leaves until its right sibling completes).
__device__ __forceinline__ float thread_tree(const float* __restrict__ p, int cnt, size_t stride) {
  if (cnt <= 64) {
    float v[64];
#pragma unroll
    for (int b = 0; b < 64; ++b) v[b] = b < cnt ? p[(size_t)b * stride] : 0.f;
#pragma unroll
    for (int w = 1; w < 64; w <<= 1)
#pragma unroll
      for (int b = 0; b < 64; b += 2 * w) v[b] = v[b] + v[b + w];
    return v[0];
  }
  int p2 = 64;
  while (p2 < cnt) p2 <<= 1;
  float st[16], x = 0.f;
#pragma unroll
  for (int l = 0; l < 16; ++l) st[l] = 0.f;
#pragma unroll 4
  for (int b = 0; b < p2; ++b) {
    x = b < cnt ? p[(size_t)b * stride] : 0.f;
    bool carry = true;
#pragma unroll
    for (int l = 0; l < 16; ++l)
      if (carry) {
        if ((b >> l) & 1) {
          x = st[l] + x;
        } else {
          st[l] = x;
          carry = false;
        }
      }
  }
  return x;  // the last leaf's carry reached the root
}

// Hessian block sums [n][nbp][TC] (packed upper-triangle tiles, hess_packed_off) -> hsum [n][nx*nx]
// and y[:, off:off+C] = clip(sum / M).  One thread per packed word: consecutive threads read
// consecutive words of every block (each word read once), sum them in the canonical tree over the
// blocks (thread_tree = tree_sum's order), and store the result at (d1, d2) and (d2, d1) (the
// diagonal tiles' lower halves are skipped: (d1, d2) and (d2, d1) take the upper element, as
// hess_packed_off maps them).  Workgroups are mapped XCD-major: workgroup b runs on XCD b % 8, and an
// XCD's workgroups take whole points (bpp workgroups each), so a point's transposed stores merge
// in one L2 instead of leaving eight XCDs as partial lines.
__global__ __launch_bounds__(256) void k_reduce_hess(const float* __restrict__ hpart, int n, int nx, int NT, int nbp,
                                                     int bpp, float* __restrict__ hsum, float invM, float bound,
                                                     float* __restrict__ y, int ystride, int yoff, int* status) {
  const int TC = NT * (NT + 1) / 2 * 256, C = nx * nx;
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int i = (k / bpp) * 8 + xcd, w = (k % bpp) * 256 + threadIdx.x;
  if (i >= n || w >= TC) return;
  const int q = w >> 8, e = w & 255, r = ((e >> 4) & 3) * 4 + (e >> 6), c = e & 15;
  int I = 0, rq = q;
  while (rq >= NT - I) {
    rq -= NT - I;
    ++I;
  }
  const int J = I + rq, d1 = 16 * I + r, d2 = 16 * J + c;
  if (d1 >= nx || d2 >= nx || (I == J && r > c)) return;
  const float s = thread_tree(hpart + (size_t)i * nbp * TC + w, nbp, (size_t)TC);
  flag_nonfinite(status, s);
  const float v = clip_label(s * invM, bound);
  const size_t o1 = (size_t)d1 * nx + d2, o2 = (size_t)d2 * nx + d1;
  if (hsum) {
    hsum[(size_t)i * C + o1] = s;
    hsum[(size_t)i * C + o2] = s;
  }
  if (y) {
    y[(size_t)i * ystride + yoff + o1] = v;
    y[(size_t)i * ystride + yoff + o2] = v;
  }
}

// Hessian sums (n, C) -> y[:, off:off+C] = clip(sum / M)
__global__ void k_finalize_hess(const float* __restrict__ hsum, int n, int C, float invM, float bound,
                                float* __restrict__ y, int ystride, int yoff) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)n * C) return;
  const size_t i = gid / C, c = gid - i * C;
  y[i * ystride + yoff + c] = clip_label(hsum[gid] * invM, bound);
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
  y[(size_t)i * ystride + c] = clip_label(v, bound);
}

__global__ void k_finalize(const float* moments, const float* gx, int n, int F, float invM, int add_g, float bound,
                           float* y) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * F) return;
  const int i = gid / F, c = gid - i * F;
  float v = moments[(size_t)i * 2 * F + c] * invM;
  if (c == 0 && add_g) v += gx[i];
  y[gid] = clip_label(v, bound);
}

}  // namespace dpi

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

// The same fragment order for the split-storage GEMM (k_gemm_x3, dpi_gemm.h): x' = 2^s x with
// max |x'| in [0.5, 1), hi = fp16(x'), lo = fp16(x' - hi) (unscaled).  *wscale = 2^-s.

// Fragment-major copy of a packed split matrix (R rows of C words, R % 16 == 0, C % 32 == 0) for
// k_pis_net: block (T, c) of 512 words = lane l's hi granule (row 16 T + l % 16, words
// 32 c + 8 (l / 16) .. + 3) at 4 l, then its lo granule (the next 4 words) at 256 + 4 l.
static size_t pack_frag_major(std::vector<float>& blob, size_t src, int R, int C) {
  blob.resize((blob.size() + 31) & ~size_t(31), 0.f);
  const size_t off = blob.size();
  blob.resize(off + (size_t)R * C, 0.f);
  const int nc = C / 32;
  for (int T = 0; T < R / 16; ++T)
    for (int c = 0; c < nc; ++c)
      for (int h = 0; h < 2; ++h)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 4; ++j)
            blob[off + (((size_t)T * nc + c) * 2 + h) * 256 + 4 * l + j] =
                blob[src + (size_t)(16 * T + (l & 15)) * C + 32 * c + 8 * (l >> 4) + 4 * h + j];
  return off;
}

template <class F>
static size_t pack_split_x3(std::vector<float>& blob, int R, int C, F at, float* wscale) {
  float mx = 0.f;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) mx = std::max(mx, std::fabs(at(r, c)));
  int e = 0;
  if (mx > 0.f) (void)std::frexp(mx, &e);  // mx = f 2^e, f in [0.5, 1)
  const float sc = std::ldexp(1.0f, -e);
  *wscale = std::ldexp(1.0f, e);
  const size_t off = blob.size();
  blob.resize(off + (size_t)R * C, 0.f);
  _Float16* dst = reinterpret_cast<_Float16*>(blob.data() + off);
  for (int r = 0; r < R; ++r)
    for (int u = 0; u < C / 32; ++u)
      for (int q = 0; q < 4; ++q) {
        _Float16* g = dst + ((size_t)r * C + 32 * u + 8 * q) * 2;  // 16 halves = 8 words
        for (int j = 0; j < 8; ++j) {
          const float x = at(r, 32 * u + 4 * q + (j & 3) + 16 * (j >> 2)) * sc;
          const _Float16 h = (_Float16)x;
          g[j] = h;
          g[8 + j] = (_Float16)(x - (float)h);
        }
      }
  return off;
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

// ---------------------------------------------------------------- operand exponents (split storage)
// A value stored split with an unscaled residual, hi = fp16(v), lo = fp16(v - hi) (the x3 convention
// of k_gemm_x3 / k_pis_net / k_pis_time and of the GBM tangent sweep), keeps fp32's relative precision
// only while lo is an fp16 normal (|v| >~ 2^-2); below that its error is absolute, ~2^-25.  A network
// with small weights makes every activation (or cotangent, or tangent) of a layer small, and the
// products that read them then lose precision that exact fp32 keeps (tools/probe_small.py "homog").
// So every such operand is stored as 2^e v, e per operand and network, chosen on the host from a
// calibration pass of the network itself (double precision, fixed synthetic inputs) so that the
// operand's rms is ~4: per element fp32-class down to ~rms/16, 2^14 of headroom above the rms before
// fp16 overflows (the range guard's case).  The consuming product folds 2^-e into its weight scale,
// so the arithmetic is a power of two per operand — exact.
static int x3_exponent(double sumsq, double count) {
  if (!(count > 0) || !(sumsq > 0) || !std::isfinite(sumsq)) return 0;
  const int e = 2 - (int)std::lround(0.5 * std::log2(sumsq / count));
  return std::min(std::max(e, -40), 40);
}
// fixed-seed N(0, 1) calibration inputs (splitmix64 + Box-Muller; host only, not a label draw)
struct CalNormal {
  uint64_t s = 0x9E3779B97F4A7C15ull;
  double u01() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return ((double)((z ^ (z >> 31)) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
  }
  double operator()() { return std::sqrt(-2.0 * std::log(u01())) * std::cos(6.283185307179586 * u01()); }
};
constexpr int CAL_ROWS = 16;
static double cal_act(int act, double z) { return act == DPI_ACT_TANH ? std::tanh(z) : (z > 0 ? z : std::expm1(z)); }
static double cal_dact(int act, double a) { return act == DPI_ACT_TANH ? 1.0 - a * a : (a > 0 ? 1.0 : a + 1.0); }
// y = W x + b (W row-major (o, in)); b may be null
static void cal_affine(const float* W, const float* b, int o, int in, const double* x, double* y) {
  for (int r = 0; r < o; ++r) {
    double a = b ? (double)b[r] : 0.0;
    const float* w = W + (size_t)r * in;
    for (int k = 0; k < in; ++k) a += (double)w[k] * x[k];
    y[r] = a;
  }
}
// y = W^T x (W row-major (o, in), x of length o)
static void cal_affine_t(const float* W, int o, int in, const double* x, double* y) {
  for (int k = 0; k < in; ++k) y[k] = 0.0;
  for (int r = 0; r < o; ++r) {
    const float* w = W + (size_t)r * in;
    for (int k = 0; k < in; ++k) y[k] += (double)w[k] * x[r];
  }
}

// PISGradNet's operand exponents: t_encoder's hidden layer (te) and output (temb), the operand of
// smooth_net block j (sn[j]), nn_module's activations A_l (a[l]) and VJP cotangents D_l (d[l]).
// Calibration rows: lambda evenly over (0, T), X ~ N(0, 4 I) (the OU/HJB state scale, x ~ N(0, (4 + t) I)).
struct PisExps {
  int te, temb, sn[4], a[4], d[4];
};
static PisExps pis_calibrate(int nx, int L, const int* hidden, double T, const float* phase, const float* coeff,
                             const float* te0, const float* te0b, const float* te2, const float* te2b, const float* sn0,
                             const float* sn0b, const float* const* snw, const float* const* snbw, int nsm,
                             const float* const* nnw, const float* const* nnbw, const int* ins) {
  const int C = PIS_CH;
  double s_te = 0, s_temb = 0, s_sn[4] = {0, 0, 0, 0}, s_a[4] = {0, 0, 0, 0}, s_d[4] = {0, 0, 0, 0};
  int hmax = C;
  for (int l = 0; l < L; ++l) hmax = std::max(hmax, hidden[l]);
  std::vector<double> e(2 * C), h(C), h2(C), in0(C + nx), A[4], D(hmax), D2(hmax);
  for (int l = 0; l < L; ++l) A[l].assign(hidden[l], 0.0);
  CalNormal nrm;
  auto sq = [](const std::vector<double>& v, int n) {
    double s = 0;
    for (int k = 0; k < n; ++k) s += v[k] * v[k];
    return s;
  };
  for (int r = 0; r < CAL_ROWS; ++r) {
    const double lbd = T * (r + 0.5) / CAL_ROWS;
    for (int j = 0; j < C; ++j) {
      const double a = (double)coeff[j] * lbd + (double)phase[j];
      e[j] = std::sin(a);
      e[C + j] = std::cos(a);
    }
    cal_affine(te0, te0b, C, 2 * C, e.data(), h.data());
    for (int k = 0; k < C; ++k) h[k] = cal_act(DPI_ACT_ELU, h[k]);
    s_te += sq(h, C);
    cal_affine(te2, te2b, C, C, h.data(), in0.data());
    for (int k = 0; k < C; ++k) s_temb += in0[k] * in0[k];
    cal_affine(sn0, sn0b, C, 2 * C, e.data(), h.data());
    for (int j = 0; j < nsm; ++j) {
      for (int k = 0; k < C; ++k) h[k] = cal_act(DPI_ACT_ELU, h[k]);
      s_sn[j] += sq(h, C);
      cal_affine(snw[j], snbw[j], C, C, h.data(), h2.data());
      h.swap(h2);
    }
    for (int d = 0; d < nx; ++d) in0[C + d] = 2.0 * nrm();
    const double* x = in0.data();
    for (int l = 0; l < L; ++l) {
      cal_affine(nnw[l], nnbw[l], hidden[l], ins[l], x, A[l].data());
      for (int k = 0; k < hidden[l]; ++k) A[l][k] = cal_act(DPI_ACT_ELU, A[l][k]);
      s_a[l] += sq(A[l], hidden[l]);
      x = A[l].data();
    }
    // VJP with cotangent X on net_out: D_{L-1} = (nn_L^T X) elu'(A_{L-1}), D_{l-1} = (nn_l^T D_l) elu'(A_{l-1})
    cal_affine_t(nnw[L], nx, ins[L], in0.data() + C, D.data());
    for (int l = L - 1; l >= 0; --l) {
      for (int k = 0; k < hidden[l]; ++k) D[k] *= cal_dact(DPI_ACT_ELU, A[l][k]);
      s_d[l] += sq(D, hidden[l]);
      if (l > 0) {
        cal_affine_t(nnw[l], hidden[l], ins[l], D.data(), D2.data());
        D.swap(D2);
      }
    }
  }
  PisExps x;
  x.te = x3_exponent(s_te, (double)CAL_ROWS * C);
  x.temb = x3_exponent(s_temb, (double)CAL_ROWS * C);
  for (int j = 0; j < 4; ++j) x.sn[j] = j < nsm ? x3_exponent(s_sn[j], (double)CAL_ROWS * C) : 0;
  for (int l = 0; l < 4; ++l) {
    x.a[l] = l < L ? x3_exponent(s_a[l], (double)CAL_ROWS * hidden[l]) : 0;
    x.d[l] = l < L ? x3_exponent(s_d[l], (double)CAL_ROWS * hidden[l]) : 0;
  }
  return x;
}

// The MLP tangent sweep's operand exponents (mlp_hdiag_split): activations a_l (the forward's B
// operands of layers l + 1) and tangent operands act'(a_l) z_l, z_0 = W1x[:, d] over every direction d
// (z_{l+1} = W_{l+1} (act'(a_l) z_l)).  Calibration rows: t evenly over (0, T), x ~ N(0, I).
static void mlp_calibrate(int nx, int H, int L, int act, const float* W0, const float* b0, const float* const* W,
                          const float* const* b, int* ea, int* eb) {
  const int n_in = 1 + nx;
  double sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  std::vector<double> x(n_in), a[4], z((size_t)H * nx), zn((size_t)H * nx);
  for (int l = 0; l < L; ++l) a[l].assign(H, 0.0);
  CalNormal nrm;
  for (int r = 0; r < CAL_ROWS; ++r) {
    x[0] = (r + 0.5) / CAL_ROWS;
    for (int d = 0; d < nx; ++d) x[1 + d] = nrm();
    cal_affine(W0, b0, H, n_in, x.data(), a[0].data());
    for (int k = 0; k < H; ++k) a[0][k] = cal_act(act, a[0][k]);
    for (int l = 1; l < L; ++l) {
      cal_affine(W[l], b[l], H, H, a[l - 1].data(), a[l].data());
      for (int k = 0; k < H; ++k) a[l][k] = cal_act(act, a[l][k]);
    }
    for (int l = 0; l + 1 < L; ++l)
      for (int k = 0; k < H; ++k) sa[l] += a[l][k] * a[l][k];
    if (r >= 4) continue;  // the tangents (H^2 nx per layer) from the first 4 rows
    // tangents of every direction at once: z[h][d]
    for (int h = 0; h < H; ++h)
      for (int d = 0; d < nx; ++d) z[(size_t)h * nx + d] = W0[(size_t)h * n_in + 1 + d];
    for (int l = 0; l + 1 < L; ++l) {
      for (int h = 0; h < H; ++h) {
        const double f = cal_dact(act, a[l][h]);
        for (int d = 0; d < nx; ++d) {
          z[(size_t)h * nx + d] *= f;
          sb[l] += z[(size_t)h * nx + d] * z[(size_t)h * nx + d];
        }
      }
      std::fill(zn.begin(), zn.end(), 0.0);
      for (int o = 0; o < H; ++o)
        for (int k = 0; k < H; ++k) {
          const double w = W[l + 1][(size_t)o * H + k];
          if (w != 0.0)
            for (int d = 0; d < nx; ++d) zn[(size_t)o * nx + d] += w * z[(size_t)k * nx + d];
        }
      z.swap(zn);
    }
  }
  for (int l = 0; l < 4; ++l) {
    ea[l] = l + 1 < L ? x3_exponent(sa[l], (double)CAL_ROWS * H) : 0;
    eb[l] = l + 1 < L ? x3_exponent(sb[l], 4.0 * H * nx) : 0;
  }
}

extern "C" {

int dpi_abi_version(void) { return DPI_ABI_VERSION; }

// ---- launch timers (dpi_launch_timer_*): start / stop events recorded on the timed path
// launch's own dispatch packet
struct LaunchTimer {
  hipEvent_t t0 = nullptr, t1 = nullptr;
  bool recorded = false;
};
static LaunchTimer g_timers[DPI_LAUNCH_TIMERS];
static std::mutex g_timer_mu;
static thread_local int g_timer_armed = -1;

int dpi_launch_timer_arm(int slot) {
  if (slot < 0 || slot >= DPI_LAUNCH_TIMERS) return fail(DPI_ERR_ARG, "launch_timer_arm: slot out of range");
  std::lock_guard<std::mutex> lk(g_timer_mu);
  LaunchTimer& t = g_timers[slot];
  if (!t.t0) {
    HIPCHK(hipEventCreate(&t.t0));
    HIPCHK(hipEventCreate(&t.t1));
  }
  t.recorded = false;
  g_timer_armed = slot;
  return 0;
}

int dpi_launch_timer_ms(int slot, float* ms) {
  if (slot < 0 || slot >= DPI_LAUNCH_TIMERS || !ms) return fail(DPI_ERR_ARG, "launch_timer_ms: bad arguments");
  LaunchTimer& t = g_timers[slot];
  if (!t.recorded) return fail(DPI_ERR_ARG, "launch_timer_ms: no launch recorded on this slot since it was armed");
  HIPCHK(hipEventSynchronize(t.t1));
  HIPCHK(hipEventElapsedTime(ms, t.t0, t.t1));
  return 0;
}

// The armed timer's events for the path launch about to be enqueued (and disarm), or nulls.
static void take_timer(hipEvent_t& t0, hipEvent_t& t1) {
  t0 = t1 = nullptr;
  if (g_timer_armed < 0) return;
  LaunchTimer& t = g_timers[g_timer_armed];
  g_timer_armed = -1;
  t0 = t.t0;
  t1 = t.t1;
  t.recorded = true;
}


int dpi_last_error(char* buf, size_t len) {
  if (buf && len) {
    std::strncpy(buf, g_err.c_str(), len - 1);
    buf[len - 1] = 0;
  }
  return (int)g_err.size();
}

int dpi_problem_destroy(dpi_problem p);
int dpi_net_destroy(dpi_net net);
}
static void prep_tags_drop(const void* owner);  // dpi_label_prepare's records naming a destroyed handle
extern "C" {

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
  if (nx > NXW_MAX) return fail(DPI_ERR_UNSUPPORTED, "cha: nx exceeds the compiled maximum state dimension 256 (NXW_MAX)");
  if (!out || nx < 1 || !(alpha > 0)) return fail(DPI_ERR_ARG, "cha: bad arguments");
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
  if (nx > NXW_MAX) return fail(DPI_ERR_UNSUPPORTED, "ou: nx exceeds the compiled maximum state dimension 256 (NXW_MAX)");
  if (!out || nx < 1 || n_comp < 1 || n_comp > NSG || !mean || !var_diag || !pi)
    return fail(DPI_ERR_ARG, "ou: bad arguments (1 <= n_comp <= 8, nx <= 256)");
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
  if (nx > NXW_MAX) return fail(DPI_ERR_UNSUPPORTED, "gbm: nx exceeds the compiled maximum state dimension 256 (NXW_MAX)");
  if (!out || nx < 1 || n_nodes < 1 || n_nodes > NSG || !w || !v)
    return fail(DPI_ERR_ARG, "gbm: bad arguments (1 <= n_nodes <= 8, nx <= 256)");
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

int dpi_problem_set_estimate_delta_t(dpi_problem p, double delta_t) {
  if (!p || !(delta_t >= 0.0) || !(delta_t < 1e30)) return fail(DPI_ERR_ARG, "estimate_delta_t: 0 <= dt < inf");
  p->td_dt = (float)delta_t;
  return 0;
}

int dpi_problem_destroy(dpi_problem p) {
  if (!p) return 0;
  prep_tags_drop(p);
  for (void* d : p->dev) (void)hipFree(d);
  delete p;
  return 0;
}

// The net's ring of sticky status words (DPI_STATUS_*), zeroed, in host-visible memory the kernels
// write with a vector store and the host reads without a HIP call; and whether every parameter is
// finite.
static int net_init_status(dpi_net_s* n, const float* params, size_t n_params) {
  n->finite = true;
  for (size_t i = 0; i < n_params; ++i)
    if (!std::isfinite(params[i])) {
      n->finite = false;
      break;
    }
  const size_t bytes = (size_t)DPI_STATUS_SLOTS * STATUS_STRIDE * sizeof(int);
  void* h = nullptr;
  HIPCHK(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h, 0, bytes);
  n->status_host = (int*)h;
  void* d = nullptr;
  HIPCHK(hipHostGetDevicePointer(&d, h, 0));
  n->status = (int*)d;
  n->slot = 0;
  return 0;
}

static volatile int* status_word(dpi_net net, int slot) {
  return (volatile int*)(net->status_host + (size_t)slot * STATUS_STRIDE);
}

int dpi_net_create_zero(dpi_net* out) {
  if (!out) return fail(DPI_ERR_ARG, "null out");
  auto* n = new dpi_net_s();
  std::memset(&n->d, 0, sizeof(n->d));
  n->d.kind = 0;  // u = 0 cannot overflow: no status word (creation stays host-only)
  *out = n;
  return 0;
}

int dpi_net_set_precision(dpi_net net, int mode) {
  if (!net || mode < -1 || mode > DPI_GEMM_AUTO) return fail(DPI_ERR_ARG, "net_set_precision: bad arguments");
  net->precision = mode;
  return 0;
}

int dpi_net_status(dpi_net net, int clear, void* stream, int* status) {
  if (!net || !status) return fail(DPI_ERR_ARG, "net_status: bad arguments");
  int v = 0;
  if (net->status_host) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    v = *status_word(net, net->slot);
    if (clear && v) *status_word(net, net->slot) = 0;
  }
  *status = v;
  return 0;
}

int dpi_net_status_slot(dpi_net net, int slot, int clear) {
  if (!net || slot < 0 || slot >= DPI_STATUS_SLOTS) return fail(DPI_ERR_ARG, "net_status_slot: bad arguments");
  net->slot = slot;
  if (clear && net->status_host) *status_word(net, slot) = 0;
  return 0;
}

int dpi_net_status_peek(dpi_net net, int slot, int* status) {
  if (!net || !status || slot < 0 || slot >= DPI_STATUS_SLOTS)
    return fail(DPI_ERR_ARG, "net_status_peek: bad arguments");
  *status = net->status_host ? *status_word(net, slot) : 0;
  return 0;
}

int dpi_net_create_mlp(int n_in, int n_hidden, const int* widths, int act, const float* params, size_t n_params,
                       dpi_net* out) {
  if (n_in - 1 > NXW_MAX)
    return fail(DPI_ERR_UNSUPPORTED, "mlp: nx = n_in - 1 exceeds the compiled maximum state dimension 256 (NXW_MAX)");
  if (!out || !widths || !params || n_in < 2 || n_hidden < 1 || n_hidden > 4)
    return fail(DPI_ERR_ARG, "mlp: bad arguments");
  if (act != DPI_ACT_ELU && act != DPI_ACT_TANH)
    return fail(DPI_ERR_UNSUPPORTED, "mlp: activations must be DPI_ACT_ELU or DPI_ACT_TANH");
  // Any hidden widths up to 128: the layers are zero-padded to the smallest compiled width H in
  // {16, 32, 64, 128} that holds the widest one.  A padded unit has zero weights and bias in and
  // zero weights out, so its activation (ELU(0) = tanh(0) = 0) and every gradient through it add
  // exact zeros: the labels are those of the unpadded network.
  int wmax = 0;
  size_t expect = 0;
  for (int l = 0; l < n_hidden; ++l) {
    if (widths[l] < 1 || widths[l] > HMAX) return fail(DPI_ERR_UNSUPPORTED, "mlp: hidden widths must be in [1, 128]");
    wmax = std::max(wmax, widths[l]);
    expect += (size_t)widths[l] * ((l ? widths[l - 1] : n_in) + 1);
  }
  expect += (size_t)widths[n_hidden - 1] + 1;
  if (n_params != expect) return fail(DPI_ERR_ARG, "mlp: parameter count mismatch");
  const float* const given = params;  // the finiteness scan (range guard) reads the caller's values
  const int H = wmax <= 16 ? 16 : wmax <= 32 ? 32 : wmax <= 64 ? 64 : 128;
  const int nx = n_in - 1, L = n_hidden;
  // nx padded to 16 (the fp32 weight images) and to 32 (the split ones).  The split layer-1 rows are
  // LDS chunks of at most 128 words whose 16-B granules are XOR-swizzled by row (split_swz): a closed
  // permutation only for 8, 16 or 32 granules per row, so a chunk of 96 words (nx in 65..96, or
  // 193..224 in the wide instances) is padded to 128 with zero columns — and nxp with it, so the path
  // kernels zero those rows of their noise tile (and the fp32 images carry the same zero columns)
  int nxp = (nx + 15) & ~15, nxp32 = (nx + 31) & ~31;
  if ((nxp32 & 127) == 96) nxp = nxp32 = nxp32 + 32;
  std::vector<float> padded;
  bool same = true;
  for (int l = 0; l < n_hidden; ++l) same = same && widths[l] == H;
  if (!same) {  // re-lay the parameters out as the equal-width-H network
    padded.assign((size_t)H * n_in + H + (size_t)(L - 1) * (H * H + H) + H + 1, 0.f);
    const float* src = params;
    float* dst = padded.data();
    int win = n_in, wpad_in = n_in;
    for (int l = 0; l < L; ++l) {
      const int w = widths[l];
      for (int r = 0; r < w; ++r)
        for (int c = 0; c < win; ++c) dst[(size_t)r * wpad_in + c] = src[(size_t)r * win + c];
      src += (size_t)w * win;
      dst += (size_t)H * wpad_in;
      for (int r = 0; r < w; ++r) dst[r] = src[r];
      src += w;
      dst += H;
      win = w;
      wpad_in = H;
    }
    for (int c = 0; c < win; ++c) dst[c] = src[c];
    dst[H] = src[win];
    params = padded.data();
  }
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
  size_t oW1xS = 0, oW1xTS = 0, oWS[4] = {0}, oWTS[4] = {0}, oWU[4] = {0};
  float wus[4] = {1.f, 1.f, 1.f, 1.f};
  int ea[4] = {0, 0, 0, 0}, eb[4] = {0, 0, 0, 0};  // mlp_hdiag_split's operand exponents
  if (H % 32 == 0) {
    auto Wx = [&](int h, int d) { return d < nx ? W0[(size_t)h * n_in + 1 + d] : 0.f; };
    oW1xS = pack_split(blob, H, nxp32, Wx);
    oW1xTS = pack_split(blob, nxp32, H, [&](int d, int h) { return Wx(h, d); });
    for (int l = 1; l < L; ++l) {
      const float* Wl = blob.data() + oW[l];
      std::vector<float> Wc(Wl, Wl + (size_t)H * H);
      oWS[l] = pack_split(blob, H, H, [&](int r, int c) { return Wc[(size_t)r * H + c]; });
      oWTS[l] = pack_split(blob, H, H, [&](int r, int c) { return Wc[(size_t)c * H + r]; });
      oWU[l] = pack_split_x3(blob, H, H, [&](int r, int c) { return Wc[(size_t)r * H + c]; }, &wus[l]);
    }
    const float *Wl[4] = {nullptr, nullptr, nullptr, nullptr}, *bl[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int l = 1; l < L; ++l) Wl[l] = blob.data() + oW[l], bl[l] = blob.data() + ob[l];
    mlp_calibrate(nx, H, L, act, W0, b0, Wl, bl, ea, eb);
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
  n->d.act = act;
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
      n->d.WU[l] = u32(oWU[l]);
      n->d.wus[l] = wus[l];
    }
    // mlp_hdiag_split: forward operand of layer l + 1 = 2^ea[l] a_l, tangent operand = 2^eb[l] act'(a_l) z_l
    for (int l = 0; l < L; ++l) {
      n->d.hsa[l] = std::ldexp(1.0f, ea[l]);
      if (l >= 1) n->d.hsc[l] = std::ldexp(wus[l], -ea[l - 1]);
      n->d.hzs[l] = l == 0 ? 1.0f : std::ldexp(wus[l], -eb[l - 1]);
      n->d.hbs[l] = l == 0 ? std::ldexp(1.0f, eb[0]) : std::ldexp(wus[l], eb[l] - eb[l - 1]);
    }
  }
  if (int rc = net_init_status(n, given, n_params)) {
    dpi_net_destroy(n);
    return rc;
  }
  *out = n;
  return 0;
}

int dpi_net_create_pisgrad(int nx, int n_hidden, const int* hidden, double T, const float* params, size_t n_params,
                           dpi_net* out) {
  if (nx > NXP_MAX)
    return fail(DPI_ERR_UNSUPPORTED, "pisgrad: nx exceeds the compiled maximum state dimension 128 (NXP_MAX)");
  if (!out || !hidden || !params || nx < 1 || n_hidden < 1 || n_hidden > 4)
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
  const PisExps ex =
      pis_calibrate(nx, L, hidden, T, phase, coeff, te0, te0b, te2, te2b, sn0, sn0b, snw, snbw, nsm, nnw, nnbw, ins);
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
  // split-storage copies (k_gemm_x3): output dims padded to 64 (hp_l, NOP), input dims to 32
  // (INP = IN's width, NXK = the x part of IN), zero fill, 128-B aligned rows
  auto r64 = [](int x) { return (x + 63) & ~63; };
  const int INP = (C + nx + 31) & ~31, NXK = (nx + 31) & ~31, NOP = r64(nx);
  int hp[4];
  for (int l = 0; l < L; ++l) hp[l] = r64(hidden[l]);
  size_t s_te0, s_te2, s_sn0, s_sn[4] = {0}, s_nn[5] = {0}, s_nnT[5] = {0}, s_nnbP[5] = {0}, s_gxno = 0;
  size_t s_nnF[5] = {0}, s_nnTF[5] = {0}, s_gxnoF = 0;
  float w_te0 = 1.f, w_te2 = 1.f, w_sn0 = 1.f, w_sn[4] = {1.f, 1.f, 1.f, 1.f}, w_nn[5], w_nnT[5], w_gxno = 1.f;
  {
    auto align = [&]() { blob.resize((blob.size() + 31) & ~size_t(31), 0.f); };
    auto packm = [&](const float* src, int rows, int cols, int Np, int Kp, bool trans, float* ws) {
      align();
      return pack_split_x3(blob, Np, Kp, [&](int r, int c) {
        if (trans) return (c < rows && r < cols) ? src[(size_t)c * cols + r] : 0.f;  // (src^T)[r][c]
        return (r < rows && c < cols) ? src[(size_t)r * cols + c] : 0.f;
      }, ws);
    };
    // every product's weight scale carries its stored input's 2^-e (x3_exponent); the VJP's also
    // its output's 2^e (EPI_DELU stores (acc ws) elu'(A))
    s_te0 = packm(te0, C, 2 * C, C, 2 * C, false, &w_te0);
    s_te2 = packm(te2, C, C, C, C, false, &w_te2);
    w_te2 = std::ldexp(w_te2, -ex.te);
    s_sn0 = packm(sn0, C, 2 * C, C, 2 * C, false, &w_sn0);
    for (int j = 0; j < nsm; ++j) {
      s_sn[j] = packm(snw[j], C, C, C, C, false, &w_sn[j]);
      w_sn[j] = std::ldexp(w_sn[j], -ex.sn[j]);
    }
    // forward: nn[0] (h0 x (64 + nx)), nn[l] (h_l x h_{l-1}), nn[L] (nx x h_{L-1}); nn[0]'s t_emb
    // columns carry t_emb's 2^-e (IN holds [2^e t_emb | X], two operands in one K)
    {
      align();
      const float* w0 = nnw[0];
      const int in0 = ins[0], h0 = hidden[0];
      s_nn[0] = pack_split_x3(blob, hp[0], INP, [&](int r, int c) {
        if (r >= h0 || c >= in0) return 0.f;
        return c < C ? std::ldexp(w0[(size_t)r * in0 + c], -ex.temb) : w0[(size_t)r * in0 + c];
      }, &w_nn[0]);
    }
    for (int l = 1; l < L; ++l) {
      s_nn[l] = packm(nnw[l], hidden[l], ins[l], hp[l], hp[l - 1], false, &w_nn[l]);
      w_nn[l] = std::ldexp(w_nn[l], -ex.a[l - 1]);
    }
    s_nn[L] = packm(nnw[L], nx, ins[L], NOP, hp[L - 1], false, &w_nn[L]);
    w_nn[L] = std::ldexp(w_nn[L], -ex.a[L - 1]);
    // VJP: nnT[L] = nn[L]^T (h_{L-1} x nx), nnT[l] = nn[l]^T, nnT[0] = nn[0][:, 64:]^T (nx x h0)
    s_nnT[L] = packm(nnw[L], nx, ins[L], hp[L - 1], NXK, true, &w_nnT[L]);
    w_nnT[L] = std::ldexp(w_nnT[L], ex.d[L - 1]);
    for (int l = 1; l < L; ++l) {
      s_nnT[l] = packm(nnw[l], hidden[l], ins[l], hp[l - 1], hp[l], true, &w_nnT[l]);
      w_nnT[l] = std::ldexp(w_nnT[l], ex.d[l - 1] - ex.d[l]);
    }
    {
      align();
      const float* w0 = nnw[0];
      const int in0 = ins[0], h0 = hidden[0];
      s_nnT[0] = pack_split_x3(blob, NOP, hp[0], [&](int d, int h) {
        return (d < nx && h < h0) ? w0[(size_t)h * in0 + C + d] : 0.f;
      }, &w_nnT[0]);
    }
    {  // [nnT[0] | nn[L]]: row d, columns h < hp0 from nn[0][h][64 + d], then nn[L][d][k]
      align();
      const float *w0 = nnw[0], *wl = nnw[L];
      const int in0 = ins[0], h0 = hidden[0], inl = ins[L];
      // K order [A_{L-1} | D_0]: k_pis_net forms the A_{L-1} half while A_{L-1} is still in LDS
      // (the two halves' columns carry 2^-e of A_{L-1} resp. D_0)
      s_gxno = pack_split_x3(blob, NOP, hp[L - 1] + hp[0], [&](int d, int k) {
        if (d >= nx) return 0.f;
        if (k < hp[L - 1]) return k < inl ? std::ldexp(wl[(size_t)d * inl + k], -ex.a[L - 1]) : 0.f;
        k -= hp[L - 1];
        return k < h0 ? std::ldexp(w0[(size_t)k * in0 + C + d], -ex.d[0]) : 0.f;
      }, &w_gxno);
    }
    for (int l = 0; l <= L; ++l) {
      s_nnF[l] = pack_frag_major(blob, s_nn[l], l < L ? hp[l] : NOP, l == 0 ? INP : hp[l - 1]);
      s_nnTF[l] = pack_frag_major(blob, s_nnT[l], l == 0 ? NOP : hp[l - 1], l == 0 ? hp[0] : l == L ? NXK : hp[l]);
    }
    s_gxnoF = pack_frag_major(blob, s_gxno, NOP, hp[L - 1] + hp[0]);
    for (int l = 0; l <= L; ++l) {
      const int o = l < L ? hidden[l] : nx, op = l < L ? hp[l] : NOP;
      align();
      s_nnbP[l] = blob.size();
      blob.resize(blob.size() + op, 0.f);
      for (int k = 0; k < o; ++k) blob[s_nnbP[l] + k] = nnbw[l][k];
    }
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
  {
    auto u32 = [&](size_t off) { return reinterpret_cast<const uint32_t*>(base + off); };
    pd.te0S = u32(s_te0);
    pd.te2S = u32(s_te2);
    pd.sn0S = u32(s_sn0);
    pd.te0W = w_te0, pd.te2W = w_te2, pd.sn0W = w_sn0;
    for (int j = 0; j < nsm; ++j) pd.snS[j] = u32(s_sn[j]), pd.snW[j] = w_sn[j];
    pd.gxnoS = u32(s_gxno);
    pd.gxnoF = u32(s_gxnoF);
    pd.gxnoW = w_gxno;
    pd.xs_te = std::ldexp(1.0f, ex.te);
    pd.xs_temb = std::ldexp(1.0f, ex.temb);
    for (int j = 0; j < 4; ++j) pd.xs_sn[j] = std::ldexp(1.0f, ex.sn[j]);
    for (int l = 0; l < 4; ++l) {
      pd.nnO[l] = std::ldexp(1.0f, ex.a[l]);
      pd.nnA[l] = std::ldexp(1.0f, -ex.a[l]);
    }
    for (int l = 0; l <= L; ++l) {
      pd.nnS[l] = u32(s_nn[l]);
      pd.nnTS[l] = u32(s_nnT[l]);
      pd.nnF[l] = u32(s_nnF[l]);
      pd.nnTF[l] = u32(s_nnTF[l]);
      pd.nnW[l] = w_nn[l];
      pd.nnTW[l] = w_nnT[l];
      pd.nnbP[l] = base + s_nnbP[l];
    }
  }
  n->blob = d;
  n->n_in = 1 + nx;
  n->d.kind = 2;
  n->pis = pd;
  if (int rc = net_init_status(n, params, n_params)) {
    dpi_net_destroy(n);
    return rc;
  }
  *out = n;
  return 0;
}

int dpi_net_destroy(dpi_net net) {
  if (!net) return 0;
  prep_tags_drop(net);
  if (net->blob) (void)hipFree(net->blob);
  if (net->status_host) (void)hipHostFree(net->status_host);
  delete net;
  return 0;
}

}  // extern "C"

// PISGradNet pipeline rows (floats per path) and chunking.  x3: split-storage regions, every
// offset a multiple of 32 floats (128 B, one granule-pair chunk); GEMM-output widths (hidden
// units, the nx-wide NO / GX) padded to 64, the IN region to 32.
static PisRows pis_rows_layout(const NetPisDev& pd, bool x3) {
  auto r4 = [](int x) { return (x + 3) & ~3; };
  auto rw = [&](int x) { return x3 ? (x + 63) & ~63 : r4(x); };
  int hmax = 0;
  for (int l = 0; l < pd.L; ++l) hmax = std::max(hmax, pd.h[l]);
  PisRows L;
  int o = 0;
  L.E = o;
  o += 2 * PIS_CH;
  L.T1 = o;
  o += PIS_CH;
  L.IN = o;
  L.INP = x3 ? (PIS_CH + pd.nx + 31) & ~31 : r4(PIS_CH + pd.nx);
  o += L.INP;
  L.H0 = o;
  o += PIS_CH;
  L.H1 = o;
  o += PIS_CH;
  for (int l = 0; l < 4; ++l) {
    L.A[l] = o;
    o += l < pd.L ? rw(pd.h[l]) : 0;
  }
  L.NO = o;
  o += rw(pd.nx);
  L.D0 = o;
  o += rw(hmax);
  L.D1 = o;
  o += rw(hmax);
  L.GX = o;
  o += rw(pd.nx);
  L.SS = o;
  o += rw(pd.nx);
  L.ST = o;
  o += rw(pd.nx);
  L.SC = o;  // s, cI, TD u(t_next), s - t, [split: network time input, smooth]; from PIS_GST the
             // rollout parts' terminal GMM statistics
  o += rw(PIS_GST + PIS_PARTS * NSG);
  L.stride = o;
  return L;
}
// (point, 64-path block) pairs per pipeline chunk.  Default 4096 = 262,144 rows (4 GB of rows
// for PISGradNet 4x512 — HBM is 288 GB): every GEMM of the chain is one launch of 4096
// workgroups, so launch gaps and the last-round tail are amortised.  Measured on HJB configs[2]
// (ms/step): 256 -> 8.57, 512 -> 6.93, 1024 -> 6.41, 4096 -> 6.36.  DPI_PIS_CHUNK overrides.
static int pis_chunk_wg() {
  static const int v = [] {
    const char* e = std::getenv("DPI_PIS_CHUNK");
    const int x = e ? std::atoi(e) : 4096;
    return x >= 1 ? x : 4096;
  }();
  return v;
}

// Workspace: gx[n] | fb[n] | bx[n][H] | hb[n][HBS = 256] | tickets[n] | rec[n][BREC] | ready[n] |
// [PIS rows] | partial[n][nbp][slab_row] | ...  (256-B aligned)
struct WsLayout {
  size_t gx, fb, bx, hb, tk, rec, ready, rows, partial, rq, noise, nq, total;
  int rows_cap;
};
static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
// GBM MLP nets stage their noise sums on the prepare stream (dpi_label_prepare -> k_noise_shared;
// DPI_GBM_PREP=0 disables it): the workspace then holds them, [n][nbp][2][4 nb][P] floats.
static bool gbm_noise_prep(dpi_problem p, dpi_net net) {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_GBM_PREP");
    v = (!e || std::atoi(e) != 0) ? 1 : 0;
  }
  return v && p && net && net->d.kind == 1 && p->e.kind == DPI_EQ_GBM;
}
static WsLayout ws_layout(dpi_net net, int n, int M, int F, bool noise = false) {
  WsLayout w;
  const int H = (net && net->d.kind == 1) ? net->d.H : 0;
  const size_t nbp = (size_t)(M + P - 1) / P;
  w.gx = 0;
  w.fb = al256((size_t)n * 4);
  w.bx = w.fb + al256((size_t)n * 4);
  w.hb = w.bx + al256((size_t)n * H * 4);
  w.tk = w.hb + al256((size_t)n * HBS * 4);  // the fused reduce's per-point tickets (k_paths)
  // the one-launch dpi_sample_with_gradients' per-point baseline records and hand-off words
  w.rec = w.tk + al256((size_t)n * 4);
  w.ready = w.rec + al256((size_t)n * BREC * 4);
  w.rows = w.ready + al256((size_t)n * 8);
  w.rows_cap = 0;
  size_t rows_bytes = 0;
  if (net && net->d.kind == 2) {
    // a chunk of path rows plus the n per-point baseline rows, which ride in the first chunk's chain
    w.rows_cap = (int)std::min((size_t)n * nbp * P, (size_t)pis_chunk_wg() * P) + n;
    const int stride = std::max(pis_rows_layout(net->pis, false).stride, pis_rows_layout(net->pis, true).stride);
    rows_bytes = al256((size_t)w.rows_cap * stride * 4);
  }
  w.partial = w.rows + rows_bytes;
  w.rq = w.partial + al256((size_t)n * nbp * slab_row(F) * 4);
  // PISGradNet: the shared rollout's queue counter (256 B) and per-SIMD claim words
  w.noise = w.rq + ((net && net->d.kind == 2) ? 256 + (size_t)PIS_CLAIM_SLOTS * 4 : 0);
  const size_t nb4 = (size_t)((F - 1 + 3) / 4) * 4;
  w.nq = w.noise + (noise ? al256((size_t)n * nbp * 2 * nb4 * P * 4) : 0);
  // k_noise_shared's queue counter (256 B) and per-SIMD claim words
  w.total = w.nq + (noise ? 256 + (size_t)PIS_CLAIM_SLOTS * 4 : 0);
  return w;
}

// GEMM precision (include/dpi.h DPI_GEMM_*): AUTO (default) and F16X3 run the fp16-split MFMA
// everywhere — the fused MLP of k_paths and the PISGradNet pipeline in split storage
// (k_gemm_x3); F32 runs exact-fp32 MFMA (mlp_tile, k_gemm_nt) for ablation.  DPI_GEMM=f32|f16x3
// sets the initial mode.
static int g_gemm_mode = -1;  // -1: from the environment
static int gemm_mode() {
  if (g_gemm_mode < 0) {
    const char* e = std::getenv("DPI_GEMM");
    g_gemm_mode = !e ? DPI_GEMM_AUTO : std::strcmp(e, "f16x3") == 0 ? DPI_GEMM_F16X3
                                   : std::strcmp(e, "f32") == 0   ? DPI_GEMM_F32
                                                                  : DPI_GEMM_AUTO;
  }
  return g_gemm_mode;
}
static int net_mode(dpi_net net) { return (net && net->precision >= 0) ? net->precision : gemm_mode(); }
static bool mlp_split(dpi_net net) { return net_mode(net) != DPI_GEMM_F32; }
static bool pis_x3(dpi_net net) { return net_mode(net) != DPI_GEMM_F32; }
static int* net_status(dpi_net net) {
  return (net && net->finite && net->status) ? net->status + (size_t)net->slot * STATUS_STRIDE : nullptr;
}

extern "C" int dpi_set_gemm_precision(int mode) {
  if (mode != DPI_GEMM_F32 && mode != DPI_GEMM_F16X3 && mode != DPI_GEMM_AUTO)
    return fail(DPI_ERR_ARG, "gemm precision: 0 = fp32, 1 = fp16-split, 2 = auto");
  g_gemm_mode = mode;
  return 0;
}

static void gemm(int epi, int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                 const float* bias, const float* aux, int ldaux, hipStream_t st) {
  dim3 grid((M + GBM_ - 1) / GBM_, (N + GBN_ - 1) / GBN_), block(256);
  if (epi == EPI_BIAS)
    hipLaunchKernelGGL(k_gemm_nt<EPI_BIAS>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
  else if (epi == EPI_BIAS_ELU)
    hipLaunchKernelGGL(k_gemm_nt<EPI_BIAS_ELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
  else
    hipLaunchKernelGGL(k_gemm_nt<EPI_DELU>, grid, block, 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux);
}

static int cu_count() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    ncu = std::max(1, ncu);
  }
  return ncu;
}

// DELU epilogue operands staged through the ring's last two DMA slots (k_gemm_x3); DPI_X3_STAGE=0
// loads them in the epilogue instead (ablation).
static int x3_stage_aux() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_X3_STAGE");
    v = e ? (std::atoi(e) != 0) : 1;
  }
  return v;
}

// Block tile of the NT = 4 split GEMMs: 128 (default, k_gemm_x3h: two blocks per CU) or 256
// (DPI_X3_TILE=256: k_gemm_x3, one 8-wave block per CU with the staged DELU epilogue).
static int x3_tile_rows() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_X3_TILE");
    v = (e && std::atoi(e) == 256) ? 256 : 128;
  }
  return v;
}

// Split-storage GEMM: OUT (M x Np) = epi(X (M x Kp) W^T), all split (Np, Kp multiples of 32).
template <int NT>
static void gemm_x3_nt(int epi, int M, int Kp, int Np, const uint32_t* W, float ws, const float* X, int ldx,
                       const float* X2, int ldx2, int k1, float* OUT, int ldc, const float* bias, const float* aux,
                       int ldaux, float os, float as, hipStream_t st) {
  const int nnt = Np / (32 * NT), nmt = (M + X3_BM - 1) / X3_BM, nk1 = k1 / 32;
  if constexpr (NT == 4) {
    if (x3_tile_rows() == 128) {
      const int nmh = (M + X3H_BM - 1) / X3H_BM;
      dim3 gh(nnt * nmh), bh(X3H_THREADS);
      if (epi == EPI_BIAS)
        hipLaunchKernelGGL(k_gemm_x3h<EPI_BIAS>, gh, bh, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1, OUT, ldc, bias,
                           aux, ldaux, os, as);
      else if (epi == EPI_BIAS_ELU)
        hipLaunchKernelGGL(k_gemm_x3h<EPI_BIAS_ELU>, gh, bh, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1, OUT, ldc,
                           bias, aux, ldaux, os, as);
      else
        hipLaunchKernelGGL(k_gemm_x3h<EPI_DELU>, gh, bh, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1, OUT, ldc, bias,
                           aux, ldaux, os, as);
      return;
    }
  }
  dim3 grid(nnt * nmt), block(X3_THREADS);
  if (epi == EPI_BIAS)
    hipLaunchKernelGGL((k_gemm_x3<EPI_BIAS, NT>), grid, block, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1, OUT,
                       ldc, bias, aux, ldaux, os, as, 0);
  else if (epi == EPI_BIAS_ELU)
    hipLaunchKernelGGL((k_gemm_x3<EPI_BIAS_ELU, NT>), grid, block, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1,
                       OUT, ldc, bias, aux, ldaux, os, as, 0);
  else
    hipLaunchKernelGGL((k_gemm_x3<EPI_DELU, NT>), grid, block, 0, st, M, Kp, nnt, W, ws, X, ldx, X2, ldx2, nk1, OUT,
                       ldc, bias, aux, ldaux, os, as, x3_stage_aux());
}
// ws: the weight matrix's scale 2^-s (pack_split_x3) with the operand exponents folded in; os / as:
// the ELU output's store scale / the DELU operand's read scale (dpi_gemm.h).  X2 != nullptr: K
// columns [k1, Kp) come from X2.
static void gemm_x3(int epi, int M, int Kp, int Np, const uint32_t* W, float ws, const float* X, int ldx, float* OUT,
                    int ldc, const float* bias, const float* aux, int ldaux, float os, float as, hipStream_t st,
                    const float* X2 = nullptr, int ldx2 = 0, int k1 = 0) {  // Np % 64 == 0, Kp % 32 == 0
  if (!X2) X2 = X, ldx2 = ldx, k1 = Kp;
  if (Np % 128 == 0)
    gemm_x3_nt<4>(epi, M, Kp, Np, W, ws, X, ldx, X2, ldx2, k1, OUT, ldc, bias, aux, ldaux, os, as, st);
  else
    gemm_x3_nt<2>(epi, M, Kp, Np, W, ws, X, ldx, X2, ldx2, k1, OUT, ldc, bias, aux, ldaux, os, as, st);
}

// k_pis_net (the fused split VJP chain) by default; DPI_PIS_FUSED=0 selects the layer-wise
// k_gemm_x3h chain (read per call, so one process can compare both).
static bool pis_fused_on() {
  const char* e = std::getenv("DPI_PIS_FUSED");
  return !e || std::atoi(e) != 0;
}
// k_pis_net's shapes: 1-4 hidden layers of 512 units, nx <= 128 (X in <= 4 chunks, GX 64 or 128 wide)
static bool pis_fused_fits(const NetPisDev& pd, const PisRows& L) {
  if (pd.L < 1 || pd.L > 4) return false;
  for (int l = 0; l < pd.L; ++l)
    if (pd.h[l] != PN_H) return false;
  const int nxk = L.INP / 32 - 2, nop = (pd.nx + 63) & ~63;
  return nxk >= 1 && nxk <= PN_XC && (nop == 64 || nop == 128);
}

// The PISGradNet chain of pis_chain in split storage (every width padded to 32; the x part of IN
// starts at its chunk 2 = word 64).
static PisRows pis_chain_x3(const NetPisDev& pd, float* rows, int R, hipStream_t st, bool vjp = true) {
  PisRows L = pis_rows_layout(pd, true);
  auto r64 = [](int x) { return (x + 63) & ~63; };
  const int ld = L.stride, NXK = (pd.nx + 31) & ~31, NOP = r64(pd.nx);
  // t_encoder -> IN[:, 0:64] and smooth -> SC + 5 in one launch (one block per CU: 144 KB of weights in LDS)
  if (R > 0) {
    const int ncu = cu_count();
    const int blocks = std::max(1, std::min(ncu, (R + 16 * (PT_THREADS / 64) - 1) / (16 * (PT_THREADS / 64))));
    hipLaunchKernelGGL(k_pis_time<4>, dim3(blocks), dim3(PT_THREADS), 0, st, pd, rows, L, R);
  }
  // the VJP chain as one launch with the activations in LDS (dpi_pisnet.h), where the shape fits
  if (vjp && R > 0 && pis_fused_on() && pis_fused_fits(pd, L)) {
    const dim3 grid((R + PN_BM - 1) / PN_BM), block(PN_THREADS);
    // DPI_PIS_NT: 2 (default) non-temporal row loads, plain stores; 1 both non-temporal; 0 neither
    const char* e = std::getenv("DPI_PIS_NT");
    const int ntm = e ? (std::atoi(e) == 1 ? 3 : std::atoi(e) == 0 ? 0 : 1) : 1;
    hipEvent_t t0, t1;
    take_timer(t0, t1);
    auto launch = [&](auto ntc, auto nlc) {
      hipExtLaunchKernelGGL((k_pis_net<decltype(ntc)::value, decltype(nlc)::value>), grid, block, 0, st, t0, t1, 0, pd,
                            rows, L, R);
    };
    auto by_depth = [&](auto ntc) {
      switch (pd.L) {
        case 1: launch(ntc, std::integral_constant<int, 1>{}); break;
        case 2: launch(ntc, std::integral_constant<int, 2>{}); break;
        case 3: launch(ntc, std::integral_constant<int, 3>{}); break;
        default: launch(ntc, std::integral_constant<int, 4>{}); break;
      }
    };
    if (ntm == 1)
      by_depth(std::integral_constant<int, 1>{});
    else if (ntm == 3)
      by_depth(std::integral_constant<int, 3>{});
    else
      by_depth(std::integral_constant<int, 0>{});
    return L;
  }
  int Kp = L.INP;
  const float* a = rows + L.IN;
  for (int l = 0; l < pd.L; ++l) {
    const int Np = r64(pd.h[l]);
    gemm_x3(EPI_BIAS_ELU, R, Kp, Np, pd.nnS[l], pd.nnW[l], a, ld, rows + L.A[l], ld, pd.nnbP[l], nullptr, 0, pd.nnO[l],
            1.0f, st);
    a = rows + L.A[l];
    Kp = Np;
  }
  if (!vjp) {  // forward only (TD terminal value): net_out
    gemm_x3(EPI_BIAS, R, Kp, NOP, pd.nnS[pd.L], pd.nnW[pd.L], a, ld, rows + L.NO, ld, pd.nnbP[pd.L], nullptr, 0, 1.0f, 1.0f,
            st);
    return L;
  }
  // VJP: the x part of IN starts at its chunk 2 (word 64).  (Fusing this product into the last
  // forward layer's launch, elu' read back from the tile the block had just stored, measured no
  // faster: 828 us against 487 + 335 us.)
  int dcur = L.D0, dnext = L.D1;
  gemm_x3(EPI_DELU, R, NXK, r64(pd.h[pd.L - 1]), pd.nnTS[pd.L], pd.nnTW[pd.L], rows + L.IN + 2 * 32, ld, rows + dcur, ld,
          nullptr, rows + L.A[pd.L - 1], ld, 1.0f, pd.nnA[pd.L - 1], st);
  for (int l = pd.L - 1; l >= 1; --l) {
    gemm_x3(EPI_DELU, R, r64(pd.h[l]), r64(pd.h[l - 1]), pd.nnTS[l], pd.nnTW[l], rows + dcur, ld, rows + dnext, ld, nullptr,
            rows + L.A[l - 1], ld, 1.0f, pd.nnA[l - 1], st);
    std::swap(dcur, dnext);
  }
  // GX = net_out + J^T X = [A_{L-1} | D_0] . [nn[L] | nnT[0]]^T + b_L: one GEMM with K = h_{L-1} + h_0,
  // the A_{L-1} chunks first (k_pis_net's order; k_pis_final and k_pis_base_final only need the sum)
  gemm_x3(EPI_BIAS, R, Kp + r64(pd.h[0]), NOP, pd.gxnoS, pd.gxnoW, rows + L.A[pd.L - 1], ld, rows + L.GX, ld,
          pd.nnbP[pd.L], nullptr, 0, 1.0f, 1.0f, st, rows + dcur, ld, Kp);
  return L;
}

// PISGradNet forward + VJP over R rows (solution.py:256-289); returns the row layout with H0 pointing
// at the last smooth_net activation.
static PisRows pis_chain(const NetPisDev& pd, float* rows, int R, hipStream_t st, bool vjp = true) {
  PisRows L = pis_rows_layout(pd, false);
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
  L.H0 = hs;
  if (!vjp) return L;
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
// + the staged noise sums of a GBM MLP net's prepared calls (the last region of the layout, so a
// plain call's offsets are the same)
extern "C" size_t dpi_workspace_bytes_prepared(dpi_problem p, dpi_net net, int n, int M) {
  if (!p || n < 0 || M < 0) return 0;
  return ws_layout(net, n, M, 1 + p->e.nx, gbm_noise_prep(p, net)).total;
}

// the counters of draws 1-3 (k_sample_points, k_baseline's in-block sampling)
static SampleSpec sample_spec(dpi_problem p, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                              int t_factors, float* tx) {
  SampleSpec s;
  s.tx = tx;
  s.k0 = (uint32_t)seed;
  s.k1 = (uint32_t)(seed >> 32);
  s.c3t = DPI_TAG_T | (epoch << 8);
  s.c3x0 = DPI_TAG_X0 | (epoch << 8);
  s.c3x = DPI_TAG_X | (epoch << 8);
  s.point_base = point_base;
  s.eps = eps;
  s.alpha_init_sqrt = p->alpha_init_sqrt;
  s.t_factors = t_factors;
  return s;
}

extern "C" int dpi_sample_points(dpi_problem p, int n, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                      float* tx, void* stream) {
  return dpi_sample_points_t(p, n, seed, epoch, point_base, eps, 0, tx, stream);
}

extern "C" int dpi_sample_points_t(dpi_problem p, int n, uint64_t seed, uint32_t epoch, uint32_t point_base, float eps,
                                   int t_factors, float* tx, void* stream) {
  if (!p || (!tx && n) || n < 0 || epoch > 0xFFFFFFu || t_factors < 0 || t_factors > 4096)
    return fail(DPI_ERR_ARG, "sample_points: bad arguments (t_factors in [0, 4096])");
  if (n == 0) return 0;
  const int nb = (p->e.nx + 3) >> 2;
  const int total = n * nb;
  const SampleSpec s = sample_spec(p, seed, epoch, point_base, eps, t_factors, tx);
  dim3 grid((total + 255) / 256), block(256);
  hipStream_t st = (hipStream_t)stream;
  switch (p->e.kind) {
    case DPI_EQ_CHA:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_CHA>, grid, block, 0, st, p->e, n, s);
      break;
    case DPI_EQ_OU:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_OU>, grid, block, 0, st, p->e, n, s);
      break;
    case DPI_EQ_GBM:
      hipLaunchKernelGGL(k_sample_points<DPI_EQ_GBM>, grid, block, 0, st, p->e, n, s);
      break;
    default:
      return fail(DPI_ERR_UNSUPPORTED, "sample_points: equation kind");
  }
  HIPCHK(hipGetLastError());
  return 0;
}

static bool dispatch_any(const dpi_problem_s* p, const dpi_net_s* net, const Launch& q) {
  if (q.fbase) {  // k_paths_fb (fused_base_ok)
    switch (p->e.kind) {
      case DPI_EQ_CHA:
        return dispatch_fb_cha(p, net, q);
      case DPI_EQ_OU:
        return dispatch_fb_ou(p, net, q);
      default:
        return false;
    }
  }
  const bool td = q.td && !q.baseline && !q.hess;
  if (p->e.nx > NXP_MAX && !q.baseline) {  // the wide first-order units (nx <= NXW_MAX; Cha / OU)
    if (td || q.hess) return false;
    const bool tanh = net->d.kind == 1 && net->d.act == DPI_ACT_TANH;
    switch (p->e.kind) {
      case DPI_EQ_CHA:
        return tanh ? dispatch_wide_cha_tanh(p, net, q) : dispatch_wide_cha(p, net, q);
      case DPI_EQ_OU:
        return tanh ? dispatch_wide_ou_tanh(p, net, q) : dispatch_wide_ou(p, net, q);
      case DPI_EQ_GBM:
        return tanh ? dispatch_wide_gbm_tanh(p, net, q) : dispatch_wide_gbm(p, net, q);
      default:
        return false;
    }
  }
  if (net->d.kind == 1 && net->d.act == DPI_ACT_TANH && !q.baseline) {  // the Tanh k_paths units
    switch (p->e.kind) {
      case DPI_EQ_CHA:
        return td ? dispatch_td_cha_tanh(p, net, q) : dispatch_cha_tanh(p, net, q);
      case DPI_EQ_OU:
        return td ? dispatch_td_ou_tanh(p, net, q) : dispatch_ou_tanh(p, net, q);
      case DPI_EQ_GBM:
        return td ? dispatch_td_gbm_tanh(p, net, q) : dispatch_gbm_tanh(p, net, q);
      default:
        return false;
    }
  }
  switch (p->e.kind) {
    case DPI_EQ_CHA:
      return td ? dispatch_td_cha(p, net, q) : dispatch_cha(p, net, q);
    case DPI_EQ_OU:
      return td ? dispatch_td_ou(p, net, q) : dispatch_ou(p, net, q);
    case DPI_EQ_GBM:
      return td ? dispatch_td_gbm(p, net, q) : dispatch_gbm(p, net, q);
    default:
      return false;
  }
}

static int check_pair(dpi_problem p, dpi_net net);
extern "C" {
static int check_pair(dpi_problem p, dpi_net net) {
  if (!p || !net) return fail(DPI_ERR_ARG, "null problem or net");
  if (net->d.kind && net->n_in != 1 + p->e.nx) return fail(DPI_ERR_ARG, "net input width != 1 + nx");
  if (net->d.kind && net->d.nxp > NXW_MAX) return fail(DPI_ERR_ARG, "nx too large");
  if (p->e.nx > NXP_MAX && net->d.kind == 2)
    return fail(DPI_ERR_UNSUPPORTED, "PISGradNet: nx exceeds the compiled maximum state dimension 128 (NXP_MAX)");
  return 0;
}

static int pis_check(dpi_problem p) {
  if (p->e.kind != DPI_EQ_OU)
    return fail(DPI_ERR_UNSUPPORTED, "PISGradNet device net needs OUProcessEquation (its g0 is the problem's GMM g)");
  return 0;
}

// PISGradNet: nothing to launch.  The per-point f_b = f(t, x, u, grad u) needs the whole
// PISGradNet chain, so its n rows ride in the first path chunk's chain, and g(x) is formed beside it
// in k_pis_base_final (pis_paths): every label call computes both before k_pis_final and the reduce
// read them, and the prepare stream's rollout needs neither.
static int pis_baseline(dpi_problem p) { return pis_check(p); }

// Independent Philox chains per wave in the PISGradNet rollout: 4 (default; 61 VGPRs) or 2
// (DPI_PIS_UNROLL=2; 47 VGPRs, room beside the 256 x 128 GEMM's blocks).
static int pis_rollout_unroll() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_PIS_UNROLL");
    v = (e && std::atoi(e) == 2) ? 2 : 4;
  }
  return v;
}

// Prepare-stream rollout in grids of DPI_PIS_PREP_PER_CU path sets per CU (0 / unset: one grid).
// Round 3's k_gemm_x3 chain needed bounded grids (3 per CU) so the rollout did not pack whole CUs;
// the one-wave rollout beside k_pis_net runs as one grid by default.
static int pis_prep_per_cu() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_PIS_PREP_PER_CU");
    v = e ? std::max(0, std::min(64, std::atoi(e))) : 0;
  }
  return v;
}

// The prepare stream's rollout as the per-SIMD-capped work queue (k_pis_rollout_shared), launched
// with DPI_PIS_PREP_SHARED (default 2) waves per SIMD more than it keeps; 0: the plain grid.
static int pis_prep_shared() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("DPI_PIS_PREP_SHARED");
    v = e ? std::max(0, std::min(8, std::atoi(e))) : 2;
  }
  return v;
}

// Path sets of a prepared chunk the prepare stream rolls out: DPI_PIS_PREP_FRAC (default 0.92) of
// them; the shared rollout beside k_pis_net runs at about a third of its stand-alone rate, so the
// rest goes to the prepared call's head at full occupancy (r04f trace: the prepare-stream rollout
// of the whole chunk, 4.07 ms, outlasted the 3.75 ms chain it hid under).  Round 6 sweeps on two
// boxes (profiles/r06x, r06y; 60 steps, two runs each): f = 0.88 3.738 / 3.752 and 3.798 / 3.806
// ms/step against 0.92's 3.763 / 3.774 and 3.831 / 3.827 (0.82: 3.797 / 3.810; 0.96, 1.0, 0.76 slower).
static int pis_prep_sets(int g) {
  static double f = -1.0;
  if (f < 0.0) {
    const char* e = std::getenv("DPI_PIS_PREP_FRAC");
    f = e ? std::max(0.0, std::min(1.0, std::atof(e))) : 0.88;
  }
  return std::max(0, std::min(g, (int)(f * g + 0.5)));
}

// prepared: dpi_label_prepare already ran the first chunk's rollout and baseline rows (same
// arguments, same workspace); prepare_only: run just those (dpi_label_prepare).
static int pis_paths(dpi_problem p, dpi_net net, const float* tx, int n, int K, const PathArgs& a, const WsLayout& w,
                     char* b, hipStream_t st, bool prepared = false, bool prepare_only = false) {
  int rc = pis_check(p);
  if (rc) return rc;
  float* rows = (float*)(b + w.rows);
  float* fb = (float*)(b + w.fb);
  const bool x3 = pis_x3(net);
  const PisRows L = pis_rows_layout(net->pis, x3);
  const int G = n * a.nbp, GC = std::max(1, (w.rows_cap - n) / P);
  const float dt = a.td_dt;
  // TD estimators: a terminal stage (rollout to t_next, forward chain, a_p = u(t_next, X) - g(x))
  // before the integral stage; the plain estimators run both paths in one rollout.
  // The first chunk's integral chain also carries the n baseline rows (t_i, x_i) after its g P path
  // rows: f_b comes out of the same GEMM launches (row results do not depend on where a row sits in
  // the chunk) and lands before k_pis_final reads it.
  auto chunk = [&](auto x3c, int g0, int g) {
    constexpr bool X3 = decltype(x3c)::value;
    auto chain = [&](bool vjp, int R) {
      return X3 ? pis_chain_x3(net->pis, rows, R, st, vjp) : pis_chain(net->pis, rows, R, st, vjp);
    };
    // path sets [0, gprep) of a prepared first chunk roll out on the prepare stream (beside the
    // previous batch's chain), the rest [gprep, g) at full occupancy at the head of the prepared
    // call, so the two streams' critical paths balance (DPI_PIS_PREP_FRAC)
    const int gprep = (prepare_only || prepared) ? pis_prep_sets(g) : g;
    auto rollout = [&](int stage, int gbeg = 0) {
      if constexpr (X3) {  // (k_pis_net, which it hides under, exists for the split rows only)
        if (prepare_only && pis_prep_shared()) {
          // the prepare stream: at most one rollout wave per SIMD beside the previous batch's chain
          int* rq = (int*)(b + w.rq);
          (void)hipMemsetAsync(rq, 0, 256 + (size_t)PIS_CLAIM_SLOTS * 4, st);
          hipLaunchKernelGGL((k_pis_rollout_shared<DPI_EQ_OU, true>), dim3(4 * cu_count() * (1 + pis_prep_shared())),
                             dim3(P), 0, st, p->e, net->pis, tx, g0, a.nbp, a.m_begin, K, a.flags, a.k0, a.k1, a.c3t,
                             a.c3s, a.c3i, a.point_base, rows, L, stage, dt, 0, 2 * PIS_PARTS * gprep, rq, rq + 64,
                             1);
          return;
        }
      }
      const int gend = prepare_only ? gprep : g;
      int step = gend - gbeg;
      if (prepare_only && pis_prep_per_cu() > 0) step = pis_prep_per_cu() * cu_count();
      for (int bx0 = gbeg; bx0 < gend; bx0 += step) {  // two one-wave blocks (terminal, integral) per path set
        const dim3 grid(2 * PIS_PARTS * std::min(step, gend - bx0)), block(P);  // (path, dim part) tasks
        if (pis_rollout_unroll() == 4)
          hipLaunchKernelGGL((k_pis_rollout<DPI_EQ_OU, X3, 4>), grid, block, 0, st, p->e, net->pis, tx, g0, a.nbp,
                             a.m_begin, K, a.flags, a.k0, a.k1, a.c3t, a.c3s, a.c3i, a.point_base, rows, L, stage,
                             dt, bx0);
        else
          hipLaunchKernelGGL((k_pis_rollout<DPI_EQ_OU, X3, 2>), grid, block, 0, st, p->e, net->pis, tx, g0, a.nbp,
                             a.m_begin, K, a.flags, a.k0, a.k1, a.c3t, a.c3s, a.c3i, a.point_base, rows, L, stage,
                             dt, bx0);
      }
    };
    const bool base = g0 == 0;
    float* brows = rows + (size_t)g * P * L.stride;
    if (dt > 0.f) {
      rollout(PIS_TD_TERM);
      if (a.flags & DPI_TERMINAL) {
        const PisRows Lt = chain(false, g * P);
        hipLaunchKernelGGL((k_pis_tvalue<DPI_EQ_OU, X3>), dim3(g), dim3(256), 0, st, p->e, net->pis, tx, g0, a.nbp,
                           rows, Lt, g * P, dt);
      }
      rollout(PIS_TD_INT);
    } else if (!(prepared && base)) {
      rollout(PIS_BOTH);
    } else if (gprep < g) {
      rollout(PIS_BOTH, gprep);  // the prepared chunk's remaining path sets
    }
    if (base && !(prepared && dt == 0.f))
      hipLaunchKernelGGL(k_pis_points<X3>, dim3(n), dim3(64), 0, st, p->e.nx, net->pis, tx, n, brows, L);
    if (prepare_only) return;
    const PisRows Lc = chain(true, g * P + (base ? n : 0));
    if (base)
      hipLaunchKernelGGL((k_pis_base_final<DPI_EQ_OU, X3>), dim3((n + 63) / 64), dim3(256), 0, st, p->e, net->pis,
                         tx, brows, Lc, n, fb, (float*)(b + w.gx));
    hipLaunchKernelGGL((k_pis_final<DPI_EQ_OU, X3>), dim3(g), dim3(NTH), 0, st, p->e, net->pis, tx, g0, a.nbp, K,
                       a.flags, fb, a.gx, rows, Lc, a.partial, dt);
  };
  for (int g0 = 0; g0 < G; g0 += GC) {
    const int g = std::min(GC, G - g0);
    if (x3)
      chunk(std::true_type{}, g0, g);
    else
      chunk(std::false_type{}, g0, g);
    if (prepare_only) break;  // the first chunk only
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// The fused reduce (k_paths' last block per point) counts blocks on per-point tickets that the
// baseline launch zeroes and the last block resets.  The host records which workspaces had a
// baseline of how many points enqueued on them, and a fused label call on a workspace without one
// fails instead of running a reduce whose tickets hold garbage (it would never fire and leave the
// labels unwritten).
static std::mutex g_base_mu;
static std::unordered_map<const void*, int>& base_tags() {
  static std::unordered_map<const void*, int> m;
  return m;
}
static void base_tag_set(const void* ws, int n) {
  std::lock_guard<std::mutex> g(g_base_mu);
  base_tags()[ws] = n;
}
static bool base_tag_ok(const void* ws, int n) {
  std::lock_guard<std::mutex> g(g_base_mu);
  auto it = base_tags().find(ws);
  return it != base_tags().end() && it->second == n;
}

int dpi_point_baseline(dpi_problem p, dpi_net net, const float* tx, int n, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (n < 0 || (n && (!tx || !ws))) return fail(DPI_ERR_ARG, "point_baseline: bad arguments");
  if (n == 0) return 0;
  const WsLayout w = ws_layout(net, n, 0, 1 + p->e.nx);
  if (ws_bytes < w.partial) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  char* b = (char*)ws;
  if (net->d.kind == 2) return pis_baseline(p);
  Launch q{true, tx, n, (float*)(b + w.gx), (float*)(b + w.fb), (float*)(b + w.bx), (float*)(b + w.hb), nullptr, 0,
           (hipStream_t)stream};
  q.tickets = (int*)(b + w.tk);
  if (!dispatch_any(p, net, q)) return fail(DPI_ERR_UNSUPPORTED, "point_baseline: unsupported equation/network shape");
  HIPCHK(hipGetLastError());
  base_tag_set(ws, n);
  return 0;
}

// The label reduce inside k_paths (fused_reduce) for first-order labels with <= 64 path blocks per
// point: one launch fewer per label call.  DPI_FUSED_REDUCE=0 keeps the separate k_reduce launch.
static bool fused_reduce_on() {  // read per call, so one process can compare both
  const char* e = std::getenv("DPI_FUSED_REDUCE");
  return !e || std::atoi(e) != 0;
}

// k_paths phase order policy (see the kernel); DPI_ORDER overrides for ablations.
static int path_order() {
  const char* e = std::getenv("DPI_ORDER");
  return e ? std::atoi(e) : 0;
}

// Validates a label-moments call and fills its PathArgs (shared by dpi_label_moments and
// dpi_label_prepare).  Returns 0, or the error; *w receives the workspace layout.
static int label_args(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                      uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, bool need_moments,
                      const float* moments, void* ws, size_t ws_bytes, WsLayout* w, PathArgs* pa) {
  const bool prepared = !need_moments || (flags & DPI_PREPARED);  // dpi_label_prepare, or its prepared call
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (n < 0 || (n && (!tx || !ws || (need_moments && !moments))) || K < 1 || M < 1 || m_begin < 0 || m_end > M ||
      m_end <= m_begin || (m_begin % P) || (m_end % P) || !(flags & DPI_BOTH) || (flags & ~(DPI_BOTH | DPI_PREPARED)) ||
      epoch > 0xFFFFFFu)
    return fail(DPI_ERR_ARG, "label_moments: bad arguments (m range multiple of 64 within [0, M], K >= 1)");
  if (n == 0) return 0;
  const int F = 1 + p->e.nx;
  const int nbp = (m_end - m_begin) / P;
  if (nbp > DPI_PATHS_PER_CALL_MAX / P) return fail(DPI_ERR_ARG, "label_moments: at most DPI_PATHS_PER_CALL_MAX paths per call");
  // the noise staging region only for dpi_label_prepare and the DPI_PREPARED call it feeds
  *w = ws_layout(net, n, M, F, prepared && gbm_noise_prep(p, net));
  if (ws_bytes < w->total)
    return fail(DPI_ERR_WORKSPACE, prepared ? "workspace too small (prepared calls: dpi_workspace_bytes_prepared)"
                                            : "workspace too small");
  char* b = (char*)ws;
  PathArgs& a = *pa;
  std::memset(&a, 0, sizeof(a));
  a.tx = tx;
  a.gx = (const float*)(b + w->gx);
  a.fb = (const float*)(b + w->fb);
  a.bx = (const float*)(b + w->bx);
  a.hb = (const float*)(b + w->hb);
  a.partial = (float*)(b + w->partial);
  a.n = n;
  a.nbp = nbp;
  a.m_begin = m_begin;
  a.K = K;
  a.flags = flags & DPI_BOTH;
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.c3t = DPI_TAG_TERM | (epoch << 8);
  a.c3s = DPI_TAG_S | (epoch << 8);
  a.c3i = DPI_TAG_INT | (epoch << 8);
  a.c3q = DPI_TAG_SDGD | (epoch << 8);
  a.point_base = point_base;
  a.order = path_order();
  a.split = mlp_split(net) ? 1 : 0;
  a.td_dt = p->td_dt;
  return 0;
}

static bool stages_prepare(dpi_problem p, dpi_net net);
static int moments_impl(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                        uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                        void* ws, size_t ws_bytes, void* stream, float* y, float bound) {
  WsLayout w;
  PathArgs a;
  int rc = label_args(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, true, moments, ws, ws_bytes,
                      &w, &a);
  if (rc || n == 0) return rc;
  const int F = 1 + p->e.nx, nbp = a.nbp;
  char* b = (char*)ws;
  float* partial = a.partial;
  hipStream_t st = (hipStream_t)stream;
  if (net->d.kind == 2) {
    if ((rc = pis_paths(p, net, tx, n, K, a, w, b, st, (flags & DPI_PREPARED) != 0))) return rc;
  } else {
    Launch q{false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, &a, n * nbp, st};
    q.td = p->td_dt > 0.f;
    if (q.td && p->e.nx > NXP_MAX)
      return fail(DPI_ERR_UNSUPPORTED, "label_moments: the TD estimators (ESTIMATE_DELTA_T > 0) are compiled for "
                                       "nx <= 128 (NXP_MAX)");
    take_timer(q.t0, q.t1);
    if ((flags & DPI_PREPARED) && stages_prepare(p, net)) a.noise = (const float*)(b + w.noise);
    if (nbp <= 64 && fused_reduce_on()) {  // k_paths' last block per point reduces and finalizes
      if (!base_tag_ok(ws, n))
        return fail(DPI_ERR_ARG, "label_moments: no dpi_point_baseline / dpi_sample_points_baseline of these n points "
                                 "was enqueued on this workspace (the fused reduce's tickets are zeroed there)");
      a.tickets = (int*)(b + w.tk);
      a.rd_moments = moments;
      a.rd_y = y;
      a.rd_status = net_status(net);
      a.rd_invM = 1.0f / (float)M;
      a.rd_bound = bound;
      a.rd_add_g = (flags & DPI_TERMINAL) ? 1 : 0;
    }
    if (!dispatch_any(p, net, q))
      return fail(DPI_ERR_UNSUPPORTED, "label_moments: unsupported equation/network shape");
    if (a.tickets) {
      HIPCHK(hipGetLastError());
      return 0;
    }
  }
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_reduce, dim3(n, (2 * F + 3) / 4), dim3(256), 0, st, partial, n, F, nbp, moments,
                     (const float*)(b + w.gx), 1.0f / (float)M, (flags & DPI_TERMINAL) ? 1 : 0, bound, y, F,
                     net_status(net));
  HIPCHK(hipGetLastError());
  return 0;
}

// The one-launch dpi_sample_with_gradients (DPI_FUSED_BASE=0: two launches; read per call).
static bool fused_base_on() {
  const char* e = std::getenv("DPI_FUSED_BASE");
  return !e || std::atoi(e) != 0;
}
// The nets and problems k_paths_fb is instantiated for (dpi_dispatch.h fused_base_shape):
// first-order Cha / OU labels without TD, of zero nets or ELU MLP nets in the fp16-split mode
// (H % 32 == 0, the fused-MLP instances; not OU 4 x 128); the rest runs the two-launch form.
static bool fused_base_ok(dpi_problem p, dpi_net net) {
  if (p->e.kind == DPI_EQ_GBM || p->td_dt > 0.f || p->e.nx > NXP_MAX) return false;
  if (net->d.kind == 0) return true;
  const int H = net->d.H, L = net->d.L;
  return net->d.kind == 1 && net->d.act == DPI_ACT_ELU && H % 32 == 0 && mlp_split(net) &&
         !(p->e.kind == DPI_EQ_OU && H == 128 && L == 4);
}
// Hand-off sequence numbers: one per fused launch, process-wide, never 0, so a hand-off word left
// in a workspace by an earlier launch (or never written) does not match this launch's.
static std::atomic<uint32_t> g_ready_seq{0};
static uint32_t next_ready_seq() {
  uint32_t s;
  do s = g_ready_seq.fetch_add(1, std::memory_order_relaxed) + 1u;
  while (s == 0u);
  return s;
}

// sample_with_gradients (picard/data.py:211-223) as one call.  First-order Cha / OU labels of MLP
// and zero nets (no TD; <= 64 path blocks per point, so the label reduce runs in the path launch):
// ONE k_paths launch of n base blocks (base_point: the point's draws 1-3, g(x), f_b, bx; published
// per point) ahead of the n nbp path blocks, which draw their point themselves, roll out, and wait
// for the point's record only before its first use — the baseline's latency-bound chain runs beside
// the rollouts instead of ahead of them.  Otherwise the points' draws inside the baseline launch
// (k_baseline with SampleSpec), then the rollout / label kernel.  PISGradNet:
// dpi_sample_points_t + dpi_generate_with_gradients.
int dpi_sample_with_gradients(dpi_problem p, dpi_net net, int n, int M, int K, uint64_t seed, uint32_t epoch,
                              uint32_t point_base, float eps, int t_factors, int flags, float sample_bound, float* tx,
                              float* y, float* moments, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (n < 0 || M < 1 || K < 1 || epoch > 0xFFFFFFu || t_factors < 0 || t_factors > 4096)
    return fail(DPI_ERR_ARG, "sample_with_gradients: bad arguments (n >= 0, M, K >= 1, t_factors in [0, 4096])");
  if (n == 0) return 0;
  if (!tx || !y || !moments) return fail(DPI_ERR_ARG, "sample_with_gradients: null tx, y or moments");
  const int F = 1 + p->e.nx;
  const WsLayout w = ws_layout(net, n, M, F);
  if (!ws || ws_bytes < w.total) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  if (net->d.kind == 2) {
    if ((rc = dpi_sample_points_t(p, n, seed, epoch, point_base, eps, t_factors, tx, stream))) return rc;
    return dpi_generate_with_gradients(p, net, tx, n, M, K, seed, epoch, point_base, flags, sample_bound, y, moments, ws,
                                       ws_bytes, stream);
  }
  if (fused_base_ok(p, net) && M % P == 0 && M / P <= 64 && fused_reduce_on() && fused_base_on()) {
    WsLayout wl;
    PathArgs a;
    if ((rc = label_args(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, flags, true, moments, ws, ws_bytes, &wl,
                         &a)))
      return rc;
    char* b = (char*)ws;
    a.tickets = (int*)(b + wl.tk);
    a.rd_moments = moments;
    a.rd_y = y;
    a.rd_status = net_status(net);
    a.rd_invM = 1.0f / (float)M;
    a.rd_bound = sample_bound;
    a.rd_add_g = (flags & DPI_TERMINAL) ? 1 : 0;
    FusedBase fb{};
    fb.nbase = n;
    fb.rec = (float*)(b + wl.rec);
    fb.ready = (unsigned long long*)(b + wl.ready);
    fb.ready_seq = next_ready_seq();
    fb.smp = sample_spec(p, seed, epoch, point_base, eps, t_factors, tx);
    Launch q{false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, &a, n + n * a.nbp, (hipStream_t)stream};
    q.fbase = &fb;
    take_timer(q.t0, q.t1);
    if (!dispatch_any(p, net, q))
      return fail(DPI_ERR_UNSUPPORTED, "sample_with_gradients: unsupported equation/network shape");
    HIPCHK(hipGetLastError());
    base_tag_set(ws, n);  // the base blocks zeroed the tickets and left the baseline in ws
    return 0;
  }
  if ((rc = dpi_sample_points_baseline(p, net, n, seed, epoch, point_base, eps, t_factors, tx, ws, ws_bytes, stream)))
    return rc;
  return moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, flags, moments, ws, ws_bytes, stream, y,
                      sample_bound);
}

// The points (dpi_sample_points_t's draws) and their baseline (dpi_point_baseline) in ONE launch
// for MLP / zero networks: each baseline workgroup samples its own point first.
int dpi_sample_points_baseline(dpi_problem p, dpi_net net, int n, uint64_t seed, uint32_t epoch, uint32_t point_base,
                               float eps, int t_factors, float* tx, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (n < 0 || (n && (!tx || !ws)) || epoch > 0xFFFFFFu || t_factors < 0 || t_factors > 4096)
    return fail(DPI_ERR_ARG, "sample_points_baseline: bad arguments (t_factors in [0, 4096])");
  if (n == 0) return 0;
  if (net->d.kind == 2) {
    if ((rc = dpi_sample_points_t(p, n, seed, epoch, point_base, eps, t_factors, tx, stream))) return rc;
    return dpi_point_baseline(p, net, tx, n, ws, ws_bytes, stream);
  }
  const WsLayout w = ws_layout(net, n, 0, 1 + p->e.nx);
  if (ws_bytes < w.partial) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  char* b = (char*)ws;
  Launch q{true, tx, n, (float*)(b + w.gx), (float*)(b + w.fb), (float*)(b + w.bx), (float*)(b + w.hb), nullptr, 0,
           (hipStream_t)stream};
  q.smp = sample_spec(p, seed, epoch, point_base, eps, t_factors, tx);
  q.tickets = (int*)(b + w.tk);
  if (!dispatch_any(p, net, q))
    return fail(DPI_ERR_UNSUPPORTED, "sample_points_baseline: unsupported equation/network shape");
  HIPCHK(hipGetLastError());
  base_tag_set(ws, n);
  return 0;
}

// The DPI_PREPARED contract: a prepared label-moments call trusts that dpi_label_prepare staged
// the first chunk in the same workspace with the same arguments.  dpi_label_prepare records the
// arguments per workspace (host side: no device read, no sync); the prepared call must match them
// and consumes the record, so a mismatched or repeated call fails with DPI_ERR_ARG instead of
// producing labels from another batch's rollout.
// The tag also records the GEMM mode the rows were staged under (split and fp32 rows differ in
// layout): a precision switch between prepare and the prepared call fails instead of reading rows
// laid out the other way.
struct PrepTag {
  const void *p, *net, *tx;
  int n, M, K, m_begin, m_end, flags, mode;
  uint64_t seed;
  uint32_t epoch, point_base;
  size_t ws_bytes;
  bool operator==(const PrepTag& o) const {
    return p == o.p && net == o.net && tx == o.tx && n == o.n && M == o.M && K == o.K && m_begin == o.m_begin &&
           m_end == o.m_end && flags == o.flags && mode == o.mode && seed == o.seed && epoch == o.epoch &&
           point_base == o.point_base && ws_bytes == o.ws_bytes;
  }
};
static std::mutex g_prep_mu;
static std::unordered_map<const void*, PrepTag>& prep_tags() {
  static std::unordered_map<const void*, PrepTag> m;
  return m;
}

static void prep_tags_drop(const void* owner) {
  std::lock_guard<std::mutex> g(g_prep_mu);
  for (auto it = prep_tags().begin(); it != prep_tags().end();)
    it = (it->second.p == owner || it->second.net == owner) ? prep_tags().erase(it) : std::next(it);
}

extern "C" int dpi_workspace_forget(const void* ws, size_t ws_bytes) {
  const char *lo = (const char*)ws, *hi = lo + ws_bytes;
  auto inside = [&](const void* a) { return (const char*)a >= lo && (const char*)a < hi; };
  {
    std::lock_guard<std::mutex> g(g_base_mu);
    for (auto it = base_tags().begin(); it != base_tags().end();) it = inside(it->first) ? base_tags().erase(it) : std::next(it);
  }
  std::lock_guard<std::mutex> g(g_prep_mu);
  for (auto it = prep_tags().begin(); it != prep_tags().end();) it = inside(it->first) ? prep_tags().erase(it) : std::next(it);
  return 0;
}

static bool stages_prepare(dpi_problem p, dpi_net net) {
  return (net->d.kind == 2 || gbm_noise_prep(p, net)) && !(p->td_dt > 0.f);
}

int dpi_label_prepare(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed, uint32_t epoch,
                      uint32_t point_base, int m_begin, int m_end, int flags, void* ws, size_t ws_bytes, void* stream) {
  WsLayout w;
  PathArgs a;
  int rc = label_args(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags & DPI_BOTH, false, nullptr,
                      ws, ws_bytes, &w, &a);
  if (rc || n == 0) return rc;
  if (!stages_prepare(p, net)) return 0;  // nothing to stage: the fused path kernels do it all
  {
    std::lock_guard<std::mutex> g(g_prep_mu);
    prep_tags()[ws] =
        PrepTag{p, net, tx, n, M, K, m_begin, m_end, flags & DPI_BOTH, pis_x3(net) ? 1 : 0, seed, epoch, point_base, ws_bytes};
  }
  if (net->d.kind == 1) {  // GBM: phase 1's noise sums, one wave per SIMD beside the previous path launch
    char* b = (char*)ws;
    hipStream_t st = (hipStream_t)stream;
    int* nq = (int*)(b + w.nq);
    HIPCHK(hipMemsetAsync(nq, 0, 256 + (size_t)PIS_CLAIM_SLOTS * 4, st));
    a.noise = (const float*)(b + w.noise);
    const int nb = (p->e.nx + 3) / 4;
    hipLaunchKernelGGL(k_noise_shared<DPI_NOISE_SHARED_UNR>, dim3(4 * cu_count() * 3), dim3(P), 0, st, a, nb,
                       n * a.nbp * 8, nq, nq + 64, 1);
    HIPCHK(hipGetLastError());
    return 0;
  }
  return pis_paths(p, net, tx, n, K, a, w, (char*)ws, (hipStream_t)stream, false, true);
}

static int check_prepared(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                          uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, void* ws,
                          size_t ws_bytes) {
  if (!(flags & DPI_PREPARED)) {
    // an unprepared call restages this workspace: a tag left from an unconsumed prepare no longer
    // describes its rows
    std::lock_guard<std::mutex> g(g_prep_mu);
    prep_tags().erase(ws);
    return 0;
  }
  if (n == 0 || !p || !net || !stages_prepare(p, net)) return 0;
  const PrepTag want{p, net, tx, n, M, K, m_begin, m_end, flags & DPI_BOTH, pis_x3(net) ? 1 : 0, seed, epoch, point_base,
                     ws_bytes};
  std::lock_guard<std::mutex> g(g_prep_mu);
  auto it = prep_tags().find(ws);
  if (it == prep_tags().end())
    return fail(DPI_ERR_ARG, "label_moments: DPI_PREPARED without a dpi_label_prepare on this workspace");
  const bool same = it->second == want;
  prep_tags().erase(it);
  if (!same)
    return fail(DPI_ERR_ARG, "label_moments: DPI_PREPARED arguments differ from the dpi_label_prepare call on this "
                             "workspace (points, counters, MC range, flags, GEMM precision or workspace size)");
  return 0;
}

int dpi_label_moments(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed, uint32_t epoch,
                      uint32_t point_base, int m_begin, int m_end, int flags, float* moments, void* ws,
                      size_t ws_bytes, void* stream) {
  int rc = check_prepared(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, ws, ws_bytes);
  if (rc) return rc;
  return moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, moments, ws, ws_bytes,
                      stream, nullptr, 0.f);
}

int dpi_label_moments_finalize(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                               uint32_t epoch, uint32_t point_base, int flags, float sample_bound, float* y,
                               float* moments, void* ws, size_t ws_bytes, void* stream) {
  if (n > 0 && !y) return fail(DPI_ERR_ARG, "label_moments_finalize: null y");
  int rc = check_prepared(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, flags, ws, ws_bytes);
  if (rc) return rc;
  return moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, flags, moments, ws, ws_bytes, stream, y,
                      sample_bound);
}

int dpi_moments_reduce(float* parts, int n_parts, int n, int nx, float* out, void* stream) {
  if (n < 0 || (n && (!parts || !out)) || n_parts < 1 || nx < 1) return fail(DPI_ERR_ARG, "moments_reduce: bad arguments");
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
  if (!p || n < 0 || (n && (!moments || !y || !ws)) || M < 1 || ws_bytes < (size_t)n * 4)
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
  if (n < 0 || M < 1 || K < 1) return fail(DPI_ERR_ARG, "generate_with_gradients: bad arguments (n >= 0, M, K >= 1)");
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
static int hess_tiles(int nx) {
  const int NT = (nx + 15) / 16;
  return NT * (NT + 1) / 2;
}
// [packed block sums n x nbp x TC | moments]
static size_t hess_extra(int n, int M, int nx, size_t* moff) {
  const int nbp = (M + P - 1) / P;
  *moff = al256((size_t)n * nbp * hess_tiles(nx) * 256 * 4);
  return *moff + al256((size_t)n * 2 * (1 + nx) * 4);
}

size_t dpi_workspace_bytes_hessians(dpi_problem p, dpi_net net, int n, int M) {
  if (!p || n < 0 || M < 0) return 0;
  size_t moff;
  return al256(ws_layout(net, n, M, 1 + p->e.nx).total) + hess_extra(n, M, p->e.nx, &moff);
}
// the same with the GBM noise staging region (dpi_label_prepare + a DPI_PREPARED Hessian-label call)
size_t dpi_workspace_bytes_hessians_prepared(dpi_problem p, dpi_net net, int n, int M) {
  if (!p || n < 0 || M < 0) return 0;
  size_t moff;
  return al256(ws_layout(net, n, M, 1 + p->e.nx, gbm_noise_prep(p, net)).total) + hess_extra(n, M, p->e.nx, &moff);
}

static int hess_moments_impl(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                             uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                             float* hsum, void* ws, size_t ws_bytes, void* stream, float* y, float bound) {
  int rc = check_pair(p, net);
  if (rc) return rc;
  if (p->e.kind != DPI_EQ_GBM)
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels need a SimpleDiffusionEquationWithHessian (GBMEquationComplexExact)");
  if (net->d.kind == 2) return fail(DPI_ERR_UNSUPPORTED, "Hessian labels: MLP or ZeroSolution networks only");
  if (n < 0 || (n && (!tx || !ws || !moments)) || K < 1 || M < 1 || m_begin < 0 || m_end > M || m_end <= m_begin ||
      (m_begin % P) || (m_end % P) || epoch > 0xFFFFFFu || !(flags & DPI_BOTH) || (flags & ~(DPI_BOTH | DPI_PREPARED)))
    return fail(DPI_ERR_ARG, "Hessian labels: bad arguments (m range multiple of 64 within [0, M], K >= 1, flags in "
                             "DPI_TERMINAL | DPI_INTEGRAL | DPI_PREPARED)");
  if (n == 0) return 0;
  const int nx = p->e.nx, F = 1 + nx, C = nx * nx, nbp = (m_end - m_begin) / P;
  if (nbp > DPI_PATHS_PER_CALL_MAX / P) return fail(DPI_ERR_ARG, "Hessian labels: at most DPI_PATHS_PER_CALL_MAX paths per call");
  // a prepared call (GBM): the terminal / integral noise sums were staged by dpi_label_prepare's
  // k_noise_shared in the prepared layout's noise region — the same counters and summation order as
  // the path launch's own rollout, so the labels are bitwise the unprepared call's
  const bool staged = (flags & DPI_PREPARED) && gbm_noise_prep(p, net);
  const WsLayout w = ws_layout(net, n, M, F, staged);
  size_t moff;
  const size_t base = al256(w.total), need = base + hess_extra(n, M, nx, &moff);
  if (ws_bytes < need)
    return fail(DPI_ERR_WORKSPACE, staged ? "workspace too small (dpi_workspace_bytes_hessians_prepared)"
                                          : "workspace too small (dpi_workspace_bytes_hessians)");
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
  a.flags = flags & DPI_BOTH;
  if (staged) a.noise = (const float*)(b + w.noise);
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  a.c3t = DPI_TAG_TERM | (epoch << 8);
  a.c3s = DPI_TAG_S | (epoch << 8);
  a.c3i = DPI_TAG_INT | (epoch << 8);
  a.c3q = DPI_TAG_SDGD | (epoch << 8);
  a.c3h1 = DPI_TAG_HTERM | (epoch << 8);
  a.c3h2 = DPI_TAG_HINT | (epoch << 8);
  a.split = mlp_split(net) ? 1 : 0;  // fp16-split tangent sweeps (mlp_hdiag_split) unless DPI_GEMM_F32
  a.point_base = point_base;
  a.hpart = (float*)(b + base);
  const int NT = (nx + 15) / 16;
  hipStream_t st = (hipStream_t)stream;
  if (p->e.nx > NXP_MAX)
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels: compiled for nx <= 128 (NXP_MAX)");
  Launch q{false, nullptr, 0, nullptr, nullptr, nullptr, nullptr, &a, n * nbp, st};
  q.hess = true;
  take_timer(q.t0, q.t1);
  if (!dispatch_any(p, net, q))
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels: unsupported network shape (GBM: width <= 64)");
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_reduce, dim3(n, (2 * F + 3) / 4), dim3(256), 0, st, a.partial, n, F, nbp, moments, a.gx,
                     1.0f / (float)M, (flags & DPI_TERMINAL) ? 1 : 0, bound, y, F + C, net_status(net));
  const int bpp = hess_tiles(nx);  // 256 packed words per workgroup: one 16 x 16 tile
  hipLaunchKernelGGL(k_reduce_hess, dim3((unsigned)((n + 7) / 8) * 8 * bpp), dim3(256), 0, st, a.hpart, n, nx, NT, nbp,
                     bpp, hsum, 1.0f / (float)M, bound, y, F + C, F, net_status(net));
  HIPCHK(hipGetLastError());
  return 0;
}

int dpi_label_moments_hessians(dpi_problem p, dpi_net net, const float* tx, int n, int M, int K, uint64_t seed,
                               uint32_t epoch, uint32_t point_base, int m_begin, int m_end, int flags, float* moments,
                               float* hessian_sums, void* ws, size_t ws_bytes, void* stream) {
  if (!hessian_sums) return fail(DPI_ERR_ARG, "label_moments_hessians: null hessian_sums");
  int rc = check_prepared(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, ws, ws_bytes);
  if (rc) return rc;
  return hess_moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, m_begin, m_end, flags, moments, hessian_sums,
                           ws, ws_bytes, stream, nullptr, 0.f);
}

int dpi_label_finalize_hessians(dpi_problem p, const float* moments, const float* hessian_sums, int n, int M, int flags,
                                float sample_bound, float* y, void* ws, size_t ws_bytes, void* stream) {
  if (!p || n < 0 || (n && (!moments || !hessian_sums || !y || !ws)) || M < 1 || !(flags & DPI_BOTH) ||
      (flags & ~DPI_BOTH))
    return fail(DPI_ERR_ARG, "label_finalize_hessians: bad arguments");
  if (n == 0) return 0;
  const int nx = p->e.nx, F = 1 + nx, C = nx * nx;
  if (ws_bytes < (size_t)n * 4) return fail(DPI_ERR_WORKSPACE, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const float* gx = (const float*)ws;  // WsLayout: gx at offset 0 (written by dpi_point_baseline)
  hipLaunchKernelGGL(k_finalize_y, dim3((n * F + 255) / 256), dim3(256), 0, st, moments, gx, n, F, 1.0f / (float)M,
                     (flags & DPI_TERMINAL) ? 1 : 0, sample_bound, y, F + C);
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
  if (n < 0 || (!y && n) || M < P || (M % P) || M > 1024 * P)
    return fail(DPI_ERR_ARG, "generate_with_gradients_and_hessians: bad arguments (M multiple of 64, <= 65536)");
  if (n == 0) return 0;
  if (p->e.kind != DPI_EQ_GBM)
    return fail(DPI_ERR_UNSUPPORTED, "Hessian labels need a SimpleDiffusionEquationWithHessian (GBMEquationComplexExact)");
  if ((rc = dpi_point_baseline(p, net, tx, n, ws, ws_bytes, stream))) return rc;
  const WsLayout w = ws_layout(net, n, M, 1 + p->e.nx);
  size_t moff;
  hess_extra(n, M, p->e.nx, &moff);
  float* moments = (float*)((char*)ws + al256(w.total) + moff);
  return hess_moments_impl(p, net, tx, n, M, K, seed, epoch, point_base, 0, M, DPI_BOTH, moments, nullptr, ws, ws_bytes,
                           stream, y, sample_bound);
}

}  // extern "C"
