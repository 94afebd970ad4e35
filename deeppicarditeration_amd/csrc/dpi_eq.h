// Equation plugins as device functors (picard/equations.py problem API, compiled).
//
// The terminal payoff g and the nonlinearity f of every shipped equation are written as
//   g(X) = G(sum_d phi_c(d, X_d))  (a few separable per-path statistics + a scalar finish),
//   f(s, X, u, grad u) from u, sum_d grad_d u, sum_d (X_d - mu) grad_d u, sum_d (grad_d u)^2,
// so a path's dims can be spread over lanes/waves and combined by fixed-order reductions.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/dpi.h"

namespace dpi {

// Row length (floats) of the per-(point, 64-path block) partial slab: the 2F column sums (c, c^2)
// rounded up to 128 B, so the rows of different workgroups never share an HBM line.
__host__ __device__ constexpr int slab_row(int F) { return (2 * F + 31) & ~31; }


constexpr int NSG = 8;  // max per-path g statistics (OU mixture components)

struct EqDev {
  int kind, nx;
  float T, alpha, asq;  // asq = sqrt(alpha)
  // Cha (equations.py:266-338): k' = k / sqrt(nx); ff(w) = alpha (k' y - C) sum w
  float cha_k, cha_C;
  // OUProcessEquation (equations.py:599-714)
  float ou_theta, ou_mu, ou_d;
  int ncomp;
  const float* mean;  // (ncomp, nx)
  const float* ivar;  // (ncomp, nx) 1/var
  const float* logc;  // (ncomp) log pi_k - 0.5 (nx log 2pi + log det_k)   (utils.py:862-876)
  // GBMEquationComplexExact (equations.py:388-486)
  int nodes;
  const float* gw;   // (nodes, 1+nx)
  const float* gv;   // (nodes)
  const float* gwsq; // (nodes) sum_d w_{k,1+d}^2
  const float* gwv2; // (nodes, nx) v_k w_{k,1+d}^2   (diag of the exact Hessian, :444-449)
  // Hessian approximation (DATA.HESSIAN_APPROXIMATION): sdgd_v > 0 = SDGD with v indices
  // drawn with replacement (data.py:497-502), 0 = exact diagonal (data.py:1262-1272)
  int sdgd_v;
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <int KIND>
struct Eq;

// ------------------------------------------------------------------------------ Cha
template <>
struct Eq<DPI_EQ_CHA> {
  static constexpr int GRAD_FULL = 0;  // fff only needs sum_d z_d (equations.py:297-302)
  __device__ static __forceinline__ void gstat(const EqDev& e, int d, float X, float* st) { st[0] += X; }
  __device__ static __forceinline__ float gfin(const EqDev& e, const float* st) {
    return sigmoidf_(e.T + e.cha_k * st[0]);  // equations.py:304-305
  }
  __device__ static __forceinline__ void gacc(const EqDev& e, int d, float X, float z, float& A, float& B) {}
  // f = ffv + ffc: the state-independent constant is kept apart so f - f_b never cancels it in fp32
  __device__ static __forceinline__ float ffv(const EqDev& e, float u, float gsum, float A, float B) {
    return e.alpha * (e.cha_k * u - e.cha_C) * gsum;  // ff(w) = fff(sqrt(alpha) w), :199-200
  }
  __device__ static __forceinline__ float ffc(const EqDev& e) { return 0.f; }
};

// ------------------------------------------------------------------------------ OU (HJB)
template <>
struct Eq<DPI_EQ_OU> {
  static constexpr int GRAD_FULL = 1;
  __device__ static __forceinline__ void gstat(const EqDev& e, int d, float X, float* st) {
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      if (c < e.ncomp) {
        const float df = X - e.mean[c * e.nx + d];
        st[c] = fmaf(df * df, e.ivar[c * e.nx + d], st[c]);
      }
    }
  }
  __device__ static __forceinline__ float gfin(const EqDev& e, const float* st) {
    // g = -log sum_k exp(logc_k - 0.5 st_k)    (equations.py:592-593, utils.py:852-880)
    float lp[NSG];
    float mx = -3.0e38f;
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      lp[c] = (c < e.ncomp) ? e.logc[c] - 0.5f * st[c] : -3.0e38f;
      mx = fmaxf(mx, lp[c]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.ncomp) s += __expf(lp[c] - mx);
    return -(mx + __logf(s));
  }
  __device__ static __forceinline__ void gacc(const EqDev& e, int d, float X, float z, float& A, float& B) {
    A = fmaf(X - e.ou_mu, z, A);
    B = fmaf(z, z, B);
  }
  // -(theta (mu - x)) . z - alpha/2 |z|^2 - d theta    (equations.py:660-666) = ffv + ffc
  __device__ static __forceinline__ float ffv(const EqDev& e, float u, float gsum, float A, float B) {
    return e.ou_theta * A - 0.5f * e.alpha * B;
  }
  __device__ static __forceinline__ float ffc(const EqDev& e) { return -e.ou_d * e.ou_theta; }
};

// ------------------------------------------------------------------------------ GBM (fully nonlinear)
template <>
struct Eq<DPI_EQ_GBM> {
  static constexpr int GRAD_FULL = 0;
  // g(X) = sum_k v_k sin(w_k0 T + sum_d w_{k,1+d} X_d)   (equations.py:422-430)
  __device__ static __forceinline__ void gstat(const EqDev& e, int d, float X, float* st) {
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.nodes) st[c] = fmaf(e.gw[c * (1 + e.nx) + 1 + d], X, st[c]);
  }
  __device__ static __forceinline__ float gfin(const EqDev& e, const float* st) {
    float g = 0.f;
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.nodes) g = fmaf(e.gv[c], __sinf(fmaf(e.gw[c * (1 + e.nx)], e.T, st[c])), g);
    return g;
  }
  __device__ static __forceinline__ void gacc(const EqDev& e, int d, float X, float z, float& A, float& B) {}
  __device__ static __forceinline__ float ffv(const EqDev& e, float u, float gsum, float A, float B) { return 0.f; }
  __device__ static __forceinline__ float ffc(const EqDev& e) { return 0.f; }
  // exact-solution part of ffi at (s, X) given arg_k = w_k . [s, X]: -u*_t - 1/2 lap u* (:457-466);
  // the -1/4 sum_d |H*_dd| part needs a pass over d (see gbm_abs_hess_partial).
  __device__ static __forceinline__ float exact_scalar_terms(const EqDev& e, const float* arg) {
    float r = 0.f;
#pragma unroll
    for (int c = 0; c < NSG; ++c) {
      if (c < e.nodes) {
        const float sn = __sinf(arg[c]), cs = __cosf(arg[c]);
        r -= e.gv[c] * e.gw[c * (1 + e.nx)] * cs;    // -u*_t
        r += 0.5f * e.gv[c] * e.gwsq[c] * sn;        // -1/2 lap u* = +1/2 sum v |w|^2 sin
      }
    }
    return r;
  }
  // sum over d in [d0, d1) step ds of |H*_dd| = |sum_k v_k w_kd^2 sin(arg_k)|
  __device__ static __forceinline__ float abs_hess_partial(const EqDev& e, const float* sn, int d0, int ds) {
    float r = 0.f;
    for (int d = d0; d < e.nx; d += ds) {
      float h = 0.f;
#pragma unroll
      for (int c = 0; c < NSG; ++c)
        if (c < e.nodes) h = fmaf(e.gwv2[c * e.nx + d], sn[c], h);
      r += fabsf(h);
    }
    return r;
  }
};

}  // namespace dpi
