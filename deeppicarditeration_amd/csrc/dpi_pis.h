// PISGradNet (picard/solution.py:138-289) on the label path, for the OU/HJB problem (config 3).
//
// The 4 x 512 network neither fits in LDS nor keeps per-path activations in registers, so the
// label path becomes a pipeline over a chunk of R paths (R = rows of every buffer below):
//   k_pis_rollout   Philox + K-step EM for both paths (as k_paths phase 1), g(X_T) -> a_p;
//                   writes IN[r] = [.. 64 t_emb slots .., X_s], S_T[r], S_s[r], E[r] = emb(T - s),
//                   per-path scalars;
//   k_gemm_nt x 15  t_encoder, smooth_net, nn_module forward, and the vector-Jacobian product of
//                   nn_module with cotangent X_s (dpi_gemm.h), activations in HBM (fp32);
//   k_pis_final     smooth, grad_x u = smooth (J^T X + net_out) + (1 - smooth) e^{-l/2} grad g0,
//                   f = ffv, b_p, per-path label contributions -> partial slab (fixed-order sums).
// The per-point baseline runs the same GEMM chain on the n points (k_pis_points, k_pis_base_final).
#pragma once
#include <hip/hip_runtime.h>

#include "dpi_eq.h"
#include "dpi_rng.h"

namespace dpi {

constexpr int PIS_CH = 64;        // timestep channels (solution.py:165)
constexpr int PIS_IN_OFF = PIS_CH;  // X occupies IN[:, 64 : 64 + nx]

struct NetPisDev {
  int nx, L, nsm;   // hidden layers of nn_module, smooth_net hidden blocks
  int h[4];         // hidden widths
  float T, smooth0; // smooth_net(emb(0))[0], host-precomputed
  const float* phase;  // (64)
  const float* coeff;  // (64)
  const float *te0, *te0b, *te2, *te2b;               // t_encoder (64x128), (64x64)
  const float *sn0, *sn0b;                            // smooth_net.0 (64x128)
  const float* sn[4];                                 // smooth_net hidden (64x64)
  const float* snb[4];
  const float *snlast, *snlastb;                      // row 0 of smooth_net's last layer (64), bias[0]
  const float* nn[5];                                 // nn_module weights (h_l x in_l), nn[L] = out (nx x h_L)
  const float* nnb[5];
  const float* nnT[5];                                // transposes for the VJP: nnT[l] = nn[l]^T, nnT[0] = x-part^T
  // split-storage pipeline (k_gemm_x3): the same matrices packed split, output dims (rows)
  // zero-padded to multiples of 64 and input dims (columns) to multiples of 32; nnbP = the nn
  // biases padded alike
  const uint32_t *te0S, *te2S, *sn0S, *snS[4];
  const uint32_t *nnS[5], *nnTS[5];
  const float* nnbP[5];
  // k_gemm_x3 weight scales 2^-s (each split matrix is stored prescaled by 2^s)
  float te0W, te2W, sn0W, snW[4], nnW[5], nnTW[5];
};

__device__ __forceinline__ void pis_embed(const NetPisDev& pn, float lbd, float* out /* stride 1 */, int j) {
  // emb(lbd)[j] = sin(c_j lbd + phi_j), emb[64 + j] = cos(...)   (solution.py:215-234)
  const float a = fmaf(pn.coeff[j], lbd, pn.phase[j]);
  float sn, cs;
  sincosf(a, &sn, &cs);
  out[j] = sn;
  out[PIS_CH + j] = cs;
}

// granule pair (u, q) of the split embedding region: columns c = 32u + 4q + (j & 3) + 16 (j >> 2),
// sin for c < 64, cos of channel c - 64 above
__device__ __forceinline__ void pis_embed8(const NetPisDev& pn, float lbd, int u, int q, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = 32 * u + 4 * q + (j & 3) + 16 * (j >> 2), ch = c & (PIS_CH - 1);
    float sn, cs;
    sincosf(fmaf(pn.coeff[ch], lbd, pn.phase[ch]), &sn, &cs);
    v[j] = c < PIS_CH ? sn : cs;
  }
}

// Workspace rows of the pipeline (floats per row); every offset a multiple of 4 (fp32 storage) or
// of 32 (split storage, where E/T1/IN/H0/H1/A/NO/D/GX hold split regions and INP = IN's width).
struct PisRows {
  int E, T1, IN, H0, H1, A[4], NO, D0, D1, GX, SS, ST, SC, stride, INP;
};

// Per-path rollout for the PIS pipeline (phase 1 of k_paths, outputs to global rows).
// Block = (point, 64-path block) number g0 + blockIdx.x; row r = blockIdx.x * 64 + lane.
// TD estimators (td_dt > 0, data.py:934-952, :529-575): horizon t_next - t instead of T - t, run
// in two stages — stage PIS_TD_TERM rolls out the terminal path and writes the network input
// rows at (t_next, X_{t_next}) (the forward chain and k_pis_tvalue then replace a_p by
// u(t_next, X) - g(x) where t_next < T), stage PIS_TD_INT the integral path (ST and a_p kept).
enum PisStage : int { PIS_BOTH = 0, PIS_TD_TERM = 1, PIS_TD_INT = 2 };

__device__ __forceinline__ float pis_horizon(const EqDev& e, float t, float td_dt, bool& td_u) {
  td_u = td_dt > 0.f && t + td_dt < e.T;
  return td_u ? td_dt : e.T - t;
}

template <int KIND, bool X3>
__global__ __launch_bounds__(256) void k_pis_rollout(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0,
                                                     int nbp, int m_begin, int K, int flags, uint32_t k0,
                                                     uint32_t k1, uint32_t c3t, uint32_t c3s, uint32_t c3i,
                                                     uint32_t point_base, const float* __restrict__ gx,
                                                     float* __restrict__ rows, PisRows L, int stage, float td_dt) {
  __shared__ float xsh[NXP_MAX];
  __shared__ float gsts[4 * P * NSG];
  __shared__ float xs3[X3 ? P * (NXP_MAX + 1) : 1];  // split mode: X_s staged [path][dim]
  __shared__ float ssh[X3 ? P : 1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = g0 + blockIdx.x;  // (point, block) in point-major order
  const int i = g / nbp, blk = g - i * nbp;
  const uint32_t ig = point_base + (uint32_t)i;
  const uint32_t m = (uint32_t)(m_begin + P * blk + lane);
  const int nx = e.nx, F = 1 + nx, nb = (nx + 3) >> 2;
  const bool TERM = flags & DPI_TERMINAL, INTG = flags & DPI_INTEGRAL;
  const bool do_term = stage != PIS_TD_INT, do_int = stage != PIS_TD_TERM;
  const float* txr = tx + (size_t)i * F;
  const float t = txr[0], Kf = (float)K;
  bool td_u;
  const float tmt = pis_horizon(e, t, td_dt, td_u);
  for (int d = tid; d < NXP_MAX; d += NTH) xsh[d] = d < nx ? txr[1 + d] : 0.f;
  const size_t r = (size_t)blockIdx.x * P + lane;
  float* row = rows + r * L.stride;
  const float U = u01_oc(philox4x32_10(0u, m, ig, c3s, k0, k1).x);
  const float s = fmaf(U, tmt, t);
  const float smt = U * tmt;  // not s - t: that rounds to 0 in fp32 for U < ulp(t) / tmt
  const float cI = e.asq * sqrtf(smt / Kf);
  const float cT = e.asq * sqrtf(tmt / Kf);
  __syncthreads();
  float gst[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) gst[c] = 0.f;
  for (int j = wv; do_term && j < nb; j += 4) {  // terminal path
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (TERM)
      for (int k = 0; k < K; ++k) {
        const f4 z = normals4_raw(philox4x32_10((uint32_t)(k * nb + j), m, ig, c3t, k0, k1));
        s0 += z.a;
        s1 += z.b;
        s2 += z.c;
        s3 += z.d;
      }
    const float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 4 * j + q;
      if (d < nx) {
        row[L.ST + d] = sv[q];
        if (TERM) Eq<KIND>::gstat(e, d, fmaf(cT, sv[q], xsh[d]), gst);
        if (stage == PIS_TD_TERM) {  // network input X_{t_next}
          if (X3)
            xs3[lane * (NXP_MAX + 1) + d] = fmaf(cT, sv[q], xsh[d]);
          else
            row[L.IN + PIS_IN_OFF + d] = fmaf(cT, sv[q], xsh[d]);
        }
      }
    }
  }
  for (int j = 3 - wv; do_int && j < nb; j += 4) {  // integral path
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (INTG)
      for (int k = 0; k < K; ++k) {
        const f4 z = normals4_raw(philox4x32_10((uint32_t)(k * nb + j), m, ig, c3i, k0, k1));
        s0 += z.a;
        s1 += z.b;
        s2 += z.c;
        s3 += z.d;
      }
    const float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 4 * j + q;
      if (d < nx) {
        row[L.SS + d] = sv[q];
        if (X3)
          xs3[lane * (NXP_MAX + 1) + d] = fmaf(cI, sv[q], xsh[d]);
        else
          row[L.IN + PIS_IN_OFF + d] = fmaf(cI, sv[q], xsh[d]);  // X_s
      }
    }
  }
  // time embedding of lambda = T - s (each wave writes 16 of the 64 channels); the TD terminal
  // stage evaluates the network at t_next
  const float tin = stage == PIS_TD_TERM ? t + td_dt : s;
  if (!X3)
    for (int j = wv; j < PIS_CH; j += 4) pis_embed(pn, pn.T - tin, row + L.E, j);
  else if (wv == 0)
    ssh[lane] = tin;
#pragma unroll
  for (int c = 0; c < NSG; ++c) gsts[(wv * P + lane) * NSG + c] = gst[c];
  __syncthreads();
  if (wv == 0) {
    float gT = 0.f;
    if (TERM && do_term) {
#pragma unroll
      for (int c = 0; c < NSG; ++c)
        gst[c] = ((gsts[(0 * P + lane) * NSG + c] + gsts[(1 * P + lane) * NSG + c]) + gsts[(2 * P + lane) * NSG + c]) +
                 gsts[(3 * P + lane) * NSG + c];
      gT = Eq<KIND>::gfin(e, gst);
    }
    if (do_int) {
      row[L.SC + 0] = s;
      row[L.SC + 1] = cI;
      row[L.SC + 3] = smt;
    }
    if (do_term) row[L.SC + 2] = TERM ? gT - gx[i] : 0.f;  // a_p = g(X_T) - g(x)
  }
  if constexpr (X3) {  // split rows, whole 32-B granule pairs: X_s -> IN chunks 2.., emb -> E
    const int nxc = L.INP / 32 - 2;
    float* rb = rows + (size_t)blockIdx.x * P * L.stride;
    for (int idx = tid; idx < P * nxc * 4; idx += NTH) {
      const int p = idx / (nxc * 4), uq = idx - p * (nxc * 4), u = uq >> 2, q = uq & 3;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 32 * u + 4 * q + (j & 3) + 16 * (j >> 2);
        v[j] = d < nx ? xs3[p * (NXP_MAX + 1) + d] : 0.f;
      }
      x3_put8(rb + (size_t)p * L.stride, L.IN, 2 + u, q, v);
    }
    for (int idx = tid; idx < P * 16; idx += NTH) {
      const int p = idx >> 4, u = (idx >> 2) & 3, q = idx & 3;
      float v[8];
      pis_embed8(pn, pn.T - ssh[p], u, q, v);
      x3_put8(rb + (size_t)p * L.stride, L.E, u, q, v);
    }
  }
}

// Baseline rows: IN[i] = [.., x], E[i] = emb(T - t), SC = (t, 1, 0, 0).
template <bool X3>
__global__ void k_pis_points(int nx, NetPisDev pn, const float* __restrict__ tx, int n, float* __restrict__ rows,
                             PisRows L) {
  const int i = blockIdx.x, tid = threadIdx.x;
  if (i >= n) return;
  const float* txr = tx + (size_t)i * (1 + nx);
  float* row = rows + (size_t)i * L.stride;
  if constexpr (X3) {
    const int nxc = L.INP / 32 - 2;
    for (int idx = tid; idx < nxc * 4; idx += blockDim.x) {
      const int u = idx >> 2, q = idx & 3;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 32 * u + 4 * q + (j & 3) + 16 * (j >> 2);
        v[j] = d < nx ? txr[1 + d] : 0.f;
      }
      x3_put8(row, L.IN, 2 + u, q, v);
    }
    for (int idx = tid; idx < 16; idx += blockDim.x) {
      float v[8];
      pis_embed8(pn, pn.T - txr[0], idx >> 2, idx & 3, v);
      x3_put8(row, L.E, idx >> 2, idx & 3, v);
    }
  } else {
    for (int d = tid; d < nx; d += blockDim.x) row[L.IN + PIS_IN_OFF + d] = txr[1 + d];
    for (int j = tid; j < PIS_CH; j += blockDim.x) pis_embed(pn, pn.T - txr[0], row + L.E, j);
  }
  if (tid == 0) {
    row[L.SC + 0] = txr[0];
    row[L.SC + 1] = 1.f;
    row[L.SC + 2] = 0.f;
    row[L.SC + 3] = 0.f;
  }
}

// GMM parameters staged in LDS per workgroup (the per-dimension gathers of pis_z_stats would
// otherwise be ~1,000 vector loads per thread): gm[0] = means, gm[1] = inverse variances,
// [component][dim], zero beyond nx.
struct PisGmmLds {
  float m[NSG][NXP_MAX];
  float iv[NSG][NXP_MAX];
};
__device__ __forceinline__ void pis_stage_gmm(const EqDev& e, PisGmmLds& g) {
  for (int idx = threadIdx.x; idx < NSG * NXP_MAX; idx += blockDim.x) {
    const int c = idx / NXP_MAX, d = idx - c * NXP_MAX;
    const bool ok = c < e.ncomp && d < e.nx;
    g.m[c][d] = ok ? e.mean[c * e.nx + d] : 0.f;
    g.iv[c][d] = ok ? e.ivar[c * e.nx + d] : 0.f;
  }
}

// grad_x u for one row, reduced into the OU statistics A = sum (X - mu) z, B = sum z^2.
// 4 threads per row (consecutive lanes, q = 0..3).  fp32 rows: dims d = q, q+4, ...; split rows:
// the dims of granule pairs (u, q) — d = 32u + 4q + (j & 3) + 16 (j >> 2) — read 32 B at a time,
// all of this thread's row data loaded into registers in one batch before the two GMM passes.
template <bool X3>
__device__ __forceinline__ void pis_z_stats(const EqDev& e, const NetPisDev& pn, const PisGmmLds& g, const float* row,
                                            const PisRows& L, float lbd, int q, float& A_out, float& B_out,
                                            float& smooth_out) {
  const int nx = e.nx;
  constexpr int NXC = NXP_MAX / 32;
  // smooth = smooth_net(emb(lbd))[0] - smooth_net(emb(0))[0]  (solution.py:236-254)
  float sr = 0.f;
  float xs[NXC][8], js[NXC][8];  // X_d and (J^T X + net_out)_d of this thread's dims
  int nxc = 0;
  if constexpr (X3) {
    nxc = L.INP / 32 - 2;
    float hv[PIS_CH / 32][8];
#pragma unroll
    for (int u = 0; u < PIS_CH / 32; ++u) x3_get8(row, L.H0, u, q, hv[u]);
#pragma unroll
    for (int u = 0; u < NXC; ++u) {
      if (u < nxc) {
        float gv[8], nv[8];
        x3_get8(row, L.IN, 2 + u, q, xs[u]);
        x3_get8(row, L.GX, u, q, gv);
        x3_get8(row, L.NO, u, q, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) js[u][j] = gv[j] + nv[j];
      }
    }
#pragma unroll
    for (int u = 0; u < PIS_CH / 32; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) sr = fmaf(pn.snlast[32 * u + 4 * q + (j & 3) + 16 * (j >> 2)], hv[u][j], sr);
  } else {
    for (int k = q; k < PIS_CH; k += 4) sr = fmaf(pn.snlast[k], row[L.H0 + k], sr);
  }
  sr += __shfl_xor(sr, 1, 64);
  sr += __shfl_xor(sr, 2, 64);
  const float smooth = sr + pn.snlastb[0] - pn.smooth0;
  const float decay = __expf(-0.5f * lbd);
  // visit(d, X_d, (J^T X + net_out)_d) over this thread's dims
  auto for_dims = [&](auto&& visit) {
    if constexpr (X3) {
#pragma unroll
      for (int u = 0; u < NXC; ++u) {
        if (u < nxc) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int d = 32 * u + 4 * q + (j & 3) + 16 * (j >> 2);
            if (d < nx) visit(d, xs[u][j], js[u][j]);
          }
        }
      }
    } else {
      const float* X = row + L.IN + PIS_IN_OFF;
      for (int d = q; d < nx; d += 4) visit(d, X[d], row[L.GX + d] + row[L.NO + d]);
    }
  };
  // GMM responsibilities at y = decay * X  (g0 = -log p, grad g0(y) = sum_k w_k (y - mu_k) / var_k)
  float st[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) st[c] = 0.f;
  for_dims([&](int d, float Xd, float) {
    const float y = decay * Xd;
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.ncomp) {
        const float df = y - g.m[c][d];
        st[c] = fmaf(df * df, g.iv[c][d], st[c]);
      }
  });
  float lp[NSG], mx = -3.0e38f;
#pragma unroll
  for (int c = 0; c < NSG; ++c) {
    st[c] += __shfl_xor(st[c], 1, 64);
    st[c] += __shfl_xor(st[c], 2, 64);
    lp[c] = c < e.ncomp ? e.logc[c] - 0.5f * st[c] : -3.0e38f;
    mx = fmaxf(mx, lp[c]);
  }
  float w[NSG], ws = 0.f;
#pragma unroll
  for (int c = 0; c < NSG; ++c) {
    w[c] = c < e.ncomp ? __expf(lp[c] - mx) : 0.f;
    ws += w[c];
  }
  const float iws = 1.0f / ws;
#pragma unroll
  for (int c = 0; c < NSG; ++c) w[c] *= iws;
  float A = 0.f, B = 0.f;
  for_dims([&](int d, float Xd, float jn) {
    const float y = decay * Xd;
    float gg = 0.f;
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.ncomp) gg = fmaf(w[c], (y - g.m[c][d]) * g.iv[c][d], gg);
    const float z = smooth * jn + (1.0f - smooth) * decay * gg;
    A = fmaf(Xd - e.ou_mu, z, A);
    B = fmaf(z, z, B);
  });
  A += __shfl_xor(A, 1, 64);
  A += __shfl_xor(A, 2, 64);
  B += __shfl_xor(B, 1, 64);
  B += __shfl_xor(B, 2, 64);
  A_out = A;
  B_out = B;
  smooth_out = smooth;
}

// Baseline f_b (state part) and nothing else: one 64-thread block per 16 points.
template <int KIND, bool X3>
__global__ __launch_bounds__(64) void k_pis_base_final(EqDev e, NetPisDev pn, const float* __restrict__ rows, PisRows L, int n,
                                 float* __restrict__ fb) {
  __shared__ PisGmmLds gmm;
  pis_stage_gmm(e, gmm);
  __syncthreads();
  const int i = blockIdx.x * 16 + (threadIdx.x >> 2), q = threadIdx.x & 3;
  const int ic = min(i, n - 1);
  const float* row = rows + (size_t)ic * L.stride;
  float A, B, sm;
  pis_z_stats<X3>(e, pn, gmm, row, L, pn.T - row[L.SC + 0], q, A, B, sm);
  if (i < n && q == 0) fb[i] = Eq<KIND>::ffv(e, 0.f, 0.f, A, B);
}

// TD terminal value (data.py:941-942): for the rows of points with t + td_dt < T, after the
// forward chain on (t_next, X_{t_next}) rows, a_p = u(t_next, X) - g(x) with
// u = smooth (net_out . X) + (1 - smooth) g0(e^{-lambda/2} X), lambda = T - t_next
// (solution.py:256-289).  4 threads per row.
template <int KIND, bool X3>
__global__ void k_pis_tvalue(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0, int nbp,
                             const float* __restrict__ gx, float* __restrict__ rows, PisRows L, int nrows,
                             float td_dt) {
  const int r = blockIdx.x * 64 + (threadIdx.x >> 2), q = threadIdx.x & 3;
  const int rc = min(r, nrows - 1);
  const int g = g0 + rc / P, i = g / nbp;
  const int nx = e.nx;
  const float t = tx[(size_t)i * (1 + nx)];
  bool td_u;
  (void)pis_horizon(e, t, td_dt, td_u);
  float* row = rows + (size_t)rc * L.stride;
  const float lbd = pn.T - (t + td_dt);
  // smooth (as pis_z_stats)
  float sr = 0.f;
  if constexpr (X3) {
#pragma unroll
    for (int u = 0; u < PIS_CH / 32; ++u) {
      float v[8];
      x3_get8(row, L.H0, u, q, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) sr = fmaf(pn.snlast[32 * u + 4 * q + (j & 3) + 16 * (j >> 2)], v[j], sr);
    }
  } else {
    for (int k = q; k < PIS_CH; k += 4) sr = fmaf(pn.snlast[k], row[L.H0 + k], sr);
  }
  sr += __shfl_xor(sr, 1, 64);
  sr += __shfl_xor(sr, 2, 64);
  const float smooth = sr + pn.snlastb[0] - pn.smooth0;
  const float decay = __expf(-0.5f * lbd);
  float sp = 0.f, st[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) st[c] = 0.f;
  auto visit = [&](int d, float Xd, float nod) {
    sp = fmaf(nod, Xd, sp);
    const float y = decay * Xd;
#pragma unroll
    for (int c = 0; c < NSG; ++c)
      if (c < e.ncomp) {
        const float df = y - e.mean[c * nx + d];
        st[c] = fmaf(df * df, e.ivar[c * nx + d], st[c]);
      }
  };
  if constexpr (X3) {
    const int nxc = L.INP / 32 - 2;
    for (int u = 0; u < nxc; ++u) {
      float xv[8], nv[8];
      x3_get8(row, L.IN, 2 + u, q, xv);
      x3_get8(row, L.NO, u, q, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = 32 * u + 4 * q + (j & 3) + 16 * (j >> 2);
        if (d < nx) visit(d, xv[j], nv[j]);
      }
    }
  } else {
    for (int d = q; d < nx; d += 4) visit(d, row[L.IN + PIS_IN_OFF + d], row[L.NO + d]);
  }
  sp += __shfl_xor(sp, 1, 64);
  sp += __shfl_xor(sp, 2, 64);
  float lp[NSG], mx = -3.0e38f;
#pragma unroll
  for (int c = 0; c < NSG; ++c) {
    st[c] += __shfl_xor(st[c], 1, 64);
    st[c] += __shfl_xor(st[c], 2, 64);
    lp[c] = c < e.ncomp ? e.logc[c] - 0.5f * st[c] : -3.0e38f;
    mx = fmaxf(mx, lp[c]);
  }
  float ws = 0.f;
#pragma unroll
  for (int c = 0; c < NSG; ++c) ws += c < e.ncomp ? __expf(lp[c] - mx) : 0.f;
  const float g0v = -(mx + __logf(ws));  // g0 = -log p (equations.py:592-593)
  const float u = smooth * sp + (1.0f - smooth) * g0v;
  if (r < nrows && q == 0 && td_u) row[L.SC + 2] = u - gx[i];
}

// Per-path f, b_p and label contributions for one (point, 64-path block) -> partial slab.
template <int KIND, bool X3>
__global__ __launch_bounds__(256) void k_pis_final(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0,
                                                   int nbp, int K, int flags, const float* __restrict__ fbv,
                                                   const float* __restrict__ rows, PisRows L,
                                                   float* __restrict__ partial, float td_dt) {
  __shared__ float cs[2][P][NXP_MAX + 4];  // per-path contributions and their squares: [path][col]
  __shared__ PisGmmLds gmm;
  pis_stage_gmm(e, gmm);
  __syncthreads();
  const int tid = threadIdx.x;
  const int g = g0 + blockIdx.x;
  const int i = g / nbp, b = g - i * nbp;
  const int nx = e.nx, F = 1 + nx;
  const bool TERM = flags & DPI_TERMINAL, INTG = flags & DPI_INTEGRAL;
  const float t = tx[(size_t)i * F], Kf = (float)K;
  bool td_u;
  const float tmt = pis_horizon(e, t, td_dt, td_u);  // horizon (TD: t_next - t)
  const float f_b = fbv[i];
  const int p = tid >> 2, q = tid & 3;
  const float* row = rows + ((size_t)blockIdx.x * P + p) * L.stride;
  const float s = row[L.SC + 0], ap = row[L.SC + 2], smt = row[L.SC + 3];
  float A, B, sm;
  pis_z_stats<X3>(e, pn, gmm, row, L, pn.T - s, q, A, B, sm);
  const float bp = INTG ? tmt * (Eq<KIND>::ffv(e, 0.f, 0.f, A, B) - f_b) : 0.f;
  const float yT = 1.0f / (sqrtf(Kf * tmt) * e.asq), yI = 1.0f / (sqrtf(Kf * smt) * e.asq);
  if (q == 0) {
    const float c0 = ap + bp + (INTG ? (f_b + Eq<KIND>::ffc(e)) * tmt : 0.f);
    cs[0][p][0] = c0;
    cs[1][p][0] = c0 * c0;
  }
  const float aY = ap * yT, bY = bp * yI;
  for (int d = q; d < nx; d += 4) {
    const float v = fmaf(aY, row[L.ST + d], bY * row[L.SS + d]);
    cs[0][p][1 + d] = v;
    cs[1][p][1 + d] = v * v;
  }
  __syncthreads();
  // fixed-order (pairwise) sum over the 64 paths of each column
  float* out = partial + ((size_t)i * nbp + b) * slab_row(F);  // [point][block][slab_row(F)]
  for (int c = tid; c < 2 * F; c += NTH) {
    const int mom = c >= F, col = c - mom * F;
    float v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = cs[mom][k][col];
#pragma unroll
    for (int w = 1; w < P; w <<= 1)
#pragma unroll
      for (int k = 0; k < P; k += 2 * w) v[k] += v[k + w];
    out[c] = v[0];
  }
}

}  // namespace dpi
