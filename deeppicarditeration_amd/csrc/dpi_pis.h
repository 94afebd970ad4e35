// PISGradNet (picard/solution.py:138-289) on the label path, for the OU/HJB problem (config 3).
//
// The 4 x 512 network neither fits in LDS nor keeps per-path activations in registers, so the
// label path becomes a pipeline over a chunk of R paths (R = rows of every buffer below):
//   k_pis_rollout   Philox + K-step EM for both paths (as k_paths phase 1), g(X_T) -> a_p;
//                   writes IN[r] = [.. 64 t_emb slots .., X_s], S_T[r], S_s[r], per-path scalars
//                   (fp32 rows: also E[r] = emb(T - s));
//   k_pis_time      (split rows) t_encoder -> IN[:, 0:64] and smooth, weights in LDS, activations
//                   in registers (fp32 rows: 7 k_gemm_nt launches through E / T1 / H0 / H1);
//   k_gemm_x3 x 10  nn_module forward and the vector-Jacobian product of nn_module with cotangent
//                   X_s (dpi_gemm.h), activations in HBM;
//   k_pis_final     smooth, grad_x u = smooth (J^T X + net_out) + (1 - smooth) e^{-l/2} grad g0,
//                   f = ffv, b_p, per-path label contributions -> partial slab (fixed-order sums).
// The n per-point baseline rows ride in the first chunk's chain (k_pis_points, k_pis_base_final).
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
  // [nn[L] | nnT[0]] ((nx -> 64) x (h_{L-1} + h_0)): net_out + J^T X = [A_{L-1} | D_0] . this^T + b_L
  const uint32_t* gxnoS;
  // fragment-major copies for k_pis_net (dpi_pisnet.h): per 16-row tile T and 32-deep chunk c a
  // 2 KB block, the 64 lanes' hi granules (lane l: row 16 T + l % 16, granule pair l / 16) then
  // their lo granules, so each weight-fragment load is one contiguous 1 KB (8 whole lines)
  const uint32_t *nnF[5], *nnTF[5], *gxnoF;
  // k_gemm_x3 weight scales 2^-s (each split matrix is stored prescaled by 2^s), times the operand
  // exponents of the stored inputs (2^-e) and, for the VJP products, of the output (2^e)
  float te0W, te2W, sn0W, snW[4], nnW[5], nnTW[5], gxnoW;
  // operand exponents (dpi_kernels.hip x3_exponent): the store scale 2^e of every split operand the
  // network's products read — k_pis_time's t_encoder hidden layer (xs_te), its output, IN[:, 0:64]
  // (xs_temb), the operand of smooth_net block j (xs_sn[j]); nn_module's A_l (nnO[l]; read back by
  // elu' as nnA[l] = 2^-e).  X (IN[:, 64:]) and GX / NO are stored unscaled.
  float xs_te, xs_temb, xs_sn[4], nnO[4], nnA[4];
};

__device__ __forceinline__ void pis_embed(const NetPisDev& pn, float lbd, float* out /* stride 1 */, int j) {
  // emb(lbd)[j] = sin(c_j lbd + phi_j), emb[64 + j] = cos(...)   (solution.py:215-234)
  const float a = fmaf(pn.coeff[j], lbd, pn.phase[j]);
  float sn, cs;
  sincosf(a, &sn, &cs);
  out[j] = sn;
  out[PIS_CH + j] = cs;
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

// Dims 4j..4j+3 of a split region starting at word `reg` of a row (a 32-column chunk u = j / 8 holds
// granule pair q = j % 4 of half h = (j % 8) / 4): 2 hi words and 2 lo words at once.
__device__ __forceinline__ void x3_put4(float* row, int reg, int j, const float (&v)[4]) {
  const int u = j >> 3, q = j & 3, h = (j >> 2) & 1;
  uint32_t hw[2], lw[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const _Float16 h0 = (_Float16)v[2 * p], h1 = (_Float16)v[2 * p + 1];
    const _Float16 l0 = (_Float16)(v[2 * p] - (float)h0), l1 = (_Float16)(v[2 * p + 1] - (float)h1);
    hw[p] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    lw[p] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  }
  uint32_t* g = reinterpret_cast<uint32_t*>(row + reg) + 32 * u + 8 * q + 2 * h;
  *reinterpret_cast<uint2*>(g) = make_uint2(hw[0], hw[1]);
  *reinterpret_cast<uint2*>(g + 4) = make_uint2(lw[0], lw[1]);
}

// v[0..3] of dims d0 .. d0 + 3 as one 16-B store (dims >= nx as 0): a row's noise-sum region is
// written in whole granules, not four 4-B pieces per dim-block (lane = row, so a wave's store
// instruction touches 64 rows; fewer, larger pieces per line reach HBM as fewer partial writes)
__device__ __forceinline__ void pis_put4(float* dst, const float (&v)[4], int d0, int nx) {
  *reinterpret_cast<float4*>(dst) = make_float4(v[0], d0 + 1 < nx ? v[1] : 0.f, d0 + 2 < nx ? v[2] : 0.f,
                                                d0 + 3 < nx ? v[3] : 0.f);
}

// The rollout of one (point, 64-path block) path set, ONE of its two paths and ONE of PIS_PARTS
// dim-block ranges, by one wave (lane = path, no LDS): task 2 PIS_PARTS g' + 2 q + 0 rolls out
// dims [4 nbq q, 4 nbq (q + 1)) of the terminal path t -> T (S_T and that range's GMM statistics of
// X_T, partial sums in SC + PIS_GST + NSG q), task 2 PIS_PARTS g' + 2 q + 1 the same dims of the
// integral path t -> s (S_s, X_s -> the network input rows; part 0 also s and its scalars).  A
// part is a quarter of a path's noise, so a rollout with fewer tasks than SIMDs (the prepared
// call's head) finishes in a quarter of a one-wave rollout's latency.  The point's x and the GMM
// parameters are wave-uniform (scalar loads), each lane's noise sums run over k in order (the sum
// of dimension d is the same sequence of adds whatever wave owns d), and no wave waits for another;
// k_pis_final combines the terminal statistics as (q0 + q1) + (q2 + q3).  Block = one wave, so a
// rollout wave fits on any SIMD with 48 free registers — beside the previous batch's k_pis_net
// block on the prepare stream (dpi_label_prepare).
constexpr int PIS_PARTS = 4;
constexpr int PIS_GST = 8;  // SC + PIS_GST + NSG q: terminal GMM statistics of part q
// WU: the scalar-unit Philox (philox4x32_10_wu; DPI_PIS_WU=1).  Off: the one-stream rollout measured
// even (HJB 3.711 / 3.714 vs 3.729 / 3.712 ms/step, r06o_ab) and under the shared wave's 48-register cap
// the scalar form spilled 9 VGPRs.
#ifndef DPI_PIS_WU
#define DPI_PIS_WU 0
#endif
#ifndef DPI_PIS_SHARED_WU  // the same for the shared rollout wave (an A/B knob; at 4 chains it spills)
#define DPI_PIS_SHARED_WU 0
#endif
template <int KIND, bool X3, int UNR, bool WU = DPI_PIS_WU>
__device__ __forceinline__ void pis_rollout_wave(const EqDev& e, const NetPisDev& pn, const float* __restrict__ tx,
                                                 int g0, int nbp, int m_begin, int K, int flags, uint32_t k0,
                                                 uint32_t k1, uint32_t c3t, uint32_t c3s, uint32_t c3i,
                                                 uint32_t point_base, float* __restrict__ rows, const PisRows& L,
                                                 int stage, float td_dt, int bx, int task) {
  const bool integral = task & 1;
  const int part = task >> 1;
  const int lane = threadIdx.x & 63;
  const int g = g0 + bx;  // (point, block) in point-major order
  const int i = g / nbp, blk = g - i * nbp;
  const uint32_t ig = point_base + (uint32_t)i;
  const uint32_t m = (uint32_t)(m_begin + P * blk + lane);
  const int nx = e.nx, F = 1 + nx, nb = (nx + 3) >> 2;
  const int nbq = (nb + PIS_PARTS - 1) / PIS_PARTS, j0 = part * nbq, j1 = min(nb, j0 + nbq);
  const bool TERM = flags & DPI_TERMINAL, INTG = flags & DPI_INTEGRAL;
  if (integral ? stage == PIS_TD_TERM : stage == PIS_TD_INT) return;
  const float* txr = tx + (size_t)i * F;
  const float t = txr[0], Kf = (float)K;
  bool td_u;
  const float tmt = pis_horizon(e, t, td_dt, td_u);
  float* row = rows + ((size_t)bx * P + lane) * L.stride;
  const bool last = part == PIS_PARTS - 1;
  if (!integral) {  // terminal path
    const float cT = e.asq * sqrtf(tmt / Kf);
    float gst[NSG];
#pragma unroll
    for (int c = 0; c < NSG; ++c) gst[c] = 0.f;
    for (int j = j0; j < j1; ++j) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      if (TERM) noise_sums<UNR, WU>(K, nb, j, m, ig, c3t, k0, k1, s0, s1, s2, s3);
      const float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
      float xv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = 4 * j + q;
        xv[q] = d < nx ? fmaf(cT, sv[q], txr[1 + d]) : 0.f;
        if (d < nx) {
          if (TERM) Eq<KIND>::gstat(e, d, xv[q], gst);
          if (!X3 && stage == PIS_TD_TERM) row[L.IN + PIS_IN_OFF + d] = xv[q];  // network input X_{t_next}
        }
      }
      // one 16-B store per dim-block (the region holds round_up(nx, 4) floats; its padding gets 0)
      pis_put4(row + L.ST + 4 * j, sv, 4 * j, nx);
      if (X3 && stage == PIS_TD_TERM) x3_put4(row, L.IN + 64, j, xv);
    }
    if (stage == PIS_TD_TERM) {  // the network at (t_next, X_{t_next}): time input and zero padding
      if (X3) {
        if (last)
          for (int j = nb; j < (L.INP - 64) / 4; ++j) {
            const float z[4] = {0.f, 0.f, 0.f, 0.f};
            x3_put4(row, L.IN + 64, j, z);
          }
        if (part == 0) row[L.SC + 4] = t + td_dt;  // k_pis_time evaluates the time networks at T - tin
      } else if (part == 0) {
        for (int j = 0; j < PIS_CH; ++j) pis_embed(pn, pn.T - (t + td_dt), row + L.E, j);
      }
    }
    if (TERM)  // this part's statistics of g(X_T); k_pis_final forms a_p = g(X_T) - g(x)
#pragma unroll
      for (int c = 0; c < NSG; ++c) row[L.SC + PIS_GST + NSG * part + c] = gst[c];
    return;
  }
  // integral path
  const float U = u01_oc(philox4x32_10(0u, m, ig, c3s, k0, k1).x);
  const float s = fmaf(U, tmt, t);
  const float smt = U * tmt;  // not s - t: that rounds to 0 in fp32 for U < ulp(t) / tmt
  const float cI = e.asq * sqrtf(smt / Kf);
  for (int j = j0; j < j1; ++j) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (INTG) noise_sums<UNR, WU>(K, nb, j, m, ig, c3i, k0, k1, s0, s1, s2, s3);
    const float sv[4] = {s0 * BM_SCALE, s1 * BM_SCALE, s2 * BM_SCALE, s3 * BM_SCALE};
    float xv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = 4 * j + q;
      xv[q] = d < nx ? fmaf(cI, sv[q], txr[1 + d]) : 0.f;  // X_s
      if (d < nx && !X3) row[L.IN + PIS_IN_OFF + d] = xv[q];
    }
    pis_put4(row + L.SS + 4 * j, sv, 4 * j, nx);
    if (X3) x3_put4(row, L.IN + 64, j, xv);
  }
  if (X3) {  // the zero padding of the x part (dims nx .. INP - 64) of IN; the time input
    if (last)
      for (int j = nb; j < (L.INP - 64) / 4; ++j) {
        const float z[4] = {0.f, 0.f, 0.f, 0.f};
        x3_put4(row, L.IN + 64, j, z);
      }
    if (part == 0) row[L.SC + 4] = s;  // k_pis_time evaluates the time networks at T - s
  } else if (part == 0) {
    for (int j = 0; j < PIS_CH; ++j) pis_embed(pn, pn.T - s, row + L.E, j);
  }
  if (part == 0) {
    row[L.SC + 0] = s;
    row[L.SC + 1] = cI;
    row[L.SC + 3] = smt;
  }
}

// Tasks 2 PIS_PARTS (bx0 + b) .. of the chunk: one 64-thread block per task.  UNR independent
// Philox chains per wave in the noise loops, <= 64 VGPRs.
template <int KIND, bool X3, int UNR = 4>
__global__ __launch_bounds__(64, 8) void k_pis_rollout(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0,
                                                    int nbp, int m_begin, int K, int flags, uint32_t k0, uint32_t k1,
                                                    uint32_t c3t, uint32_t c3s, uint32_t c3i, uint32_t point_base,
                                                    float* __restrict__ rows, PisRows L, int stage, float td_dt,
                                                    int bx0) {
  pis_rollout_wave<KIND, X3, UNR>(e, pn, tx, g0, nbp, m_begin, K, flags, k0, k1, c3t, c3s, c3i, point_base, rows, L,
                                  stage, td_dt, bx0 + (int)(blockIdx.x / (2 * PIS_PARTS)),
                                  (int)(blockIdx.x % (2 * PIS_PARTS)));
}

// The prepare stream's rollout (dpi_label_prepare), beside the previous batch's k_pis_net: a
// work queue of the 2 g one-wave tasks served by at most one wave per SIMD.  Left to the dispatcher,
// the next batch's rollout waves fill every register a finishing k_pis_net block frees (up to nine
// 56-VGPR waves per SIMD) and the next k_pis_net block waits for them: the chain stretched from 2.9
// to 4.0 ms while the rollout ran at nearly its stand-alone speed (r04a) — zero-sum.  Here the first
// wave of the launch on a SIMD (claim word per SIMD, keyed by HW_ID's SE / SH / CU / SIMD fields and
// the XCC id; zeroed with the queue counter before the launch) takes tasks until the queue is
// empty; every other wave leaves at once.  A SIMD then holds two k_pis_net waves (<= 232 registers
// each) and one rollout wave (<= 48): the chain keeps its CU, and the rollout fills the VALU issue
// slots the feed-bound chain leaves idle.  Every wave reaches the exit: a claimed wave ends when the
// queue counter passes ntask, an unclaimed one immediately.
constexpr int PIS_CLAIM_SLOTS = 8 * 256 * 4;  // XCC x (SE, SH, CU) x SIMD
template <int KIND, bool X3, int UNR>
__device__ __forceinline__ void pis_rollout_shared_body(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0, int nbp,
                                                            int m_begin, int K, int flags, uint32_t k0,
                                                           uint32_t k1, uint32_t c3t, uint32_t c3s, uint32_t c3i,
                                                           uint32_t point_base, float* __restrict__ rows, PisRows L,
                                                           int stage, float td_dt,
                                                           int bx0, int ntask, int* __restrict__ queue,
                                                           int* __restrict__ claim, int waves) {
#ifdef DPI_PIS_SHARED_PRIO  // measurement knob: the rollout wave's issue priority (k_pis_net runs at 2)
  __builtin_amdgcn_s_setprio(DPI_PIS_SHARED_PRIO);
#endif
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);         // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;  // HW_REG_XCC_ID
  const unsigned slot = (xcc << 10) | (((hw >> 8) & 0xffu) << 2) | ((hw >> 4) & 3u);
  const int lane = threadIdx.x & 63;
  int old = 0;
  if (lane == 0) old = atomicAdd(claim + slot, 1);
  // (lane 0's values made wave-uniform scalars: the task's indices then live in SGPRs)
  if (__builtin_amdgcn_readfirstlane(old) >= waves) return;  // this SIMD already runs `waves` rollout waves
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(queue, 1);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= ntask) break;
    pis_rollout_wave<KIND, X3, UNR, DPI_PIS_SHARED_WU>(e, pn, tx, g0, nbp, m_begin, K, flags, k0, k1, c3t, c3s, c3i, point_base, rows, L,
                                    stage, td_dt, bx0 + t / (2 * PIS_PARTS), t % (2 * PIS_PARTS));
  }
}

#define DPI_PIS_SHARED_ARGS                                                                                         \
  EqDev e, NetPisDev pn, const float *__restrict__ tx, int g0, int nbp, int m_begin, int K, int flags, uint32_t k0,  \
      uint32_t k1, uint32_t c3t, uint32_t c3s, uint32_t c3i, uint32_t point_base, float *__restrict__ rows,         \
      PisRows L, int stage, float td_dt, int bx0, int ntask, int *__restrict__ queue, int *__restrict__ claim,      \
      int waves
#define DPI_PIS_SHARED_CALL \
  e, pn, tx, g0, nbp, m_begin, K, flags, k0, k1, c3t, c3s, c3i, point_base, rows, L, stage, td_dt, bx0, ntask, queue, claim, waves
// one wave per SIMD: 4 Philox chains per wave, <= 48 registers (beside two 232-register k_pis_net waves)
#ifndef DPI_PIS_SHARED_VGPR_HALF
#define DPI_PIS_SHARED_VGPR_HALF 24  // 48 registers
#endif
#ifndef DPI_PIS_SHARED_UNR
#define DPI_PIS_SHARED_UNR 4
#endif
template <int KIND, bool X3>
__global__ __launch_bounds__(64, 8) __attribute__((amdgpu_num_vgpr(DPI_PIS_SHARED_VGPR_HALF))) void k_pis_rollout_shared(
    DPI_PIS_SHARED_ARGS) {
  pis_rollout_shared_body<KIND, X3, DPI_PIS_SHARED_UNR>(DPI_PIS_SHARED_CALL);
}
#undef DPI_PIS_SHARED_ARGS
#undef DPI_PIS_SHARED_CALL

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
    if (tid == 0) row[L.SC + 4] = txr[0];
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

// ---------------------------------------------------------------------------------------------
// The time networks of PISGradNet in one launch (split storage): per row lambda = T - tin (tin in
// SC + 4), emb(lambda) -> t_encoder -> IN[:, 0:64] (split), smooth_net -> smooth (SC + 5), with
// smooth = smooth_net(emb(lambda))[0] - smooth_net(emb(0))[0] (solution.py:236-254, 268-274).
// Both networks are 64 channels wide and take one scalar per row, so all their weights (te0, te2,
// sn0, sn[0..nsm), 144 KB split for nsm = 4) sit in LDS for the whole launch and every layer's
// activations stay in registers: hidden x path orientation (the units are the MFMA rows, a wave
// owns 16 paths, the C layout of unit tiles 2u, 2u+1 is the next layer's B operand chunk u, as in
// mlp_tile_split), three f16 products per fp32 product into one accumulator (the x3 convention of
// k_gemm_x3: lo unscaled, weights prescaled by 2^s).  Replaces the 7 GEMM launches of the time
// networks (and their E / T1 / H0 / H1 round trips through HBM).
// LDS image of a split matrix with Kp words per row (Kp % 64 == 0): logical granule G of row r at
// (G & ~15) | ((G ^ r) & 15) — every row starts at bank 0, and XOR with the row's low 4 bits gives
// the 16 lanes of each ds_read_b128 lane group 16 distinct 16-B slots.
constexpr int PT_THREADS = 768;  // 12 waves: 3 per SIMD at <= 168 VGPRs
__device__ __forceinline__ int pt_word(int r, int Kp, int G) { return r * Kp + 4 * ((G & ~15) | ((G ^ r) & 15)); }

template <int NSM_MAX>  // LDS holds smooth_net blocks 0..NSM_MAX-1
__global__ __launch_bounds__(PT_THREADS, 1) void k_pis_time(NetPisDev pn, float* __restrict__ rows, PisRows L, int R) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  constexpr int C = PIS_CH, W2 = C * 2 * C, W1 = C * C;  // words of a 64 x 128 / 64 x 64 split matrix
  __shared__ uint32_t wl[2 * W2 + (1 + NSM_MAX) * W1];   // te0 | sn0 | te2 | sn[0..nsm)
  __shared__ float cph[2 * C];                           // coeff | phase
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, jj = lane & 15, qq = lane >> 4;
  const int nsm = min(pn.nsm, NSM_MAX);
  __builtin_amdgcn_s_setprio(2);  // critical path, above a co-resident prepare-stream rollout wave
  auto stage = [&](const uint32_t* src, int off, int Kp) {
    const int ng = C * Kp / 4;
    for (int idx = tid; idx < ng; idx += PT_THREADS) {
      const int r = idx / (Kp / 4), G = idx - r * (Kp / 4);
      *reinterpret_cast<u32x4_t*>(wl + off + pt_word(r, Kp, G)) =
          *reinterpret_cast<const u32x4_t*>(src + (size_t)r * Kp + 4 * G);
    }
  };
  stage(pn.te0S, 0, 2 * C);
  stage(pn.sn0S, W2, 2 * C);
  stage(pn.te2S, 2 * W2, C);
  for (int j = 0; j < nsm; ++j) stage(pn.snS[j], 2 * W2 + (1 + j) * W1, C);
  if (tid < C) {
    cph[tid] = pn.coeff[tid];
    cph[C + tid] = pn.phase[tid];
  }
  __syncthreads();

  // acc[T] += W (64 x 32 NU) . B for this wave's 16 paths; B chunk u = (bh[u], bl[u])
  auto layer = [&](int off, auto NUc, const h8* bh, const h8* bl, f4v (&acc)[4]) {
    constexpr int NU = decltype(NUc)::value, Kp = 32 * NU;
#pragma unroll
    for (int T = 0; T < 4; ++T) acc[T] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        const int r = 16 * T + jj;
        const h8 ah = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(wl + off + pt_word(r, Kp, 8 * u + 2 * qq)));
        const h8 al = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(wl + off + pt_word(r, Kp, 8 * u + 2 * qq + 1)));
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[u], acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[u], acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[u], acc[T], 0, 0, 0);
      }
  };
  // x3 split of 8 values (lo unscaled)
  auto split = [&](const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const _Float16 h = (_Float16)v[j];
      hi[j] = h;
      lo[j] = (_Float16)(v[j] - (float)h);
    }
  };
  // activations (C layout, unit 16 T + 4 qq + r) x the operand's store scale xs -> B chunks u = 0, 1
  // (units 32 u + 4 qq + (j & 3) + 16 (j >> 2))
  auto to_b = [&](const float (&a)[4][4], float xs, h8 (&bh)[2], h8 (&bl)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = a[2 * u + (j >> 2)][j & 3] * xs;
      split(v, bh[u], bl[u]);
    }
  };
  auto epi = [&](const f4v (&acc)[4], float ws, const float* bias, bool act, float (&a)[4][4]) {
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = fmaf(acc[T][r], ws, bias[16 * T + 4 * qq + r]);
        a[T][r] = act ? (z > 0.f ? z : __expf(z) - 1.0f) : z;
      }
  };

  const int ntiles = (R + 15) >> 4, nwaves = gridDim.x * (PT_THREADS / 64);
  for (int tile = blockIdx.x * (PT_THREADS / 64) + wv; tile < ntiles; tile += nwaves) {
    // the LDS weights are loop-invariant: keep the compiler from hoisting every fragment read of
    // the tile loop into registers (it would need ~600 VGPRs)
    asm volatile("" ::: "memory");
    const int pr = min(16 * tile + jj, R - 1);
    float* row = rows + (size_t)pr * L.stride;
    const float lbd = pn.T - row[L.SC + 4];
    // emb(lambda) as the B operand: chunks 0, 1 = sin, 2, 3 = cos of channels 32 u + 4 qq + (j & 3) + 16 (j >> 2)
    h8 eh[4], el[4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float sv[8], cv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ch = 32 * u + 4 * qq + (j & 3) + 16 * (j >> 2);
        sincosf(fmaf(cph[ch], lbd, cph[C + ch]), &sv[j], &cv[j]);
      }
      split(sv, eh[u], el[u]);
      split(cv, eh[2 + u], el[2 + u]);
    }
    f4v acc[4];
    float a[4][4];
    h8 bh[2], bl[2];
    // t_encoder: Linear(128, 64), ELU, Linear(64, 64) -> IN[:, 0:64]
    layer(0, std::integral_constant<int, 4>{}, eh, el, acc);
    epi(acc, pn.te0W, pn.te0b, true, a);
    to_b(a, pn.xs_te, bh, bl);
    layer(2 * W2, std::integral_constant<int, 2>{}, bh, bl, acc);
    epi(acc, pn.te2W, pn.te2b, false, a);
    if (16 * tile + jj < R) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a[2 * u + (j >> 2)][j & 3] * pn.xs_temb;
        x3_put8(row, L.IN, u, qq, v);
      }
    }
    // smooth_net: Linear(128, 64), nsm x (ELU, Linear(64, 64)), ELU, row 0 of Linear(64, dim)
    layer(W2, std::integral_constant<int, 4>{}, eh, el, acc);
    epi(acc, pn.sn0W, pn.sn0b, true, a);
    for (int j = 0; j < nsm; ++j) {
      to_b(a, pn.xs_sn[j], bh, bl);
      layer(2 * W2 + (1 + j) * W1, std::integral_constant<int, 2>{}, bh, bl, acc);
      epi(acc, pn.snW[j], pn.snb[j], true, a);
    }
    float sr = 0.f;
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int r = 0; r < 4; ++r) sr = fmaf(pn.snlast[16 * T + 4 * qq + r], a[T][r], sr);
    sr += __shfl_xor(sr, 16, 64);
    sr += __shfl_xor(sr, 32, 64);
    if (qq == 0 && 16 * tile + jj < R) row[L.SC + 5] = sr + pn.snlastb[0] - pn.smooth0;
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
#pragma unroll
    for (int u = 0; u < NXC; ++u) {
      if (u < nxc) {
        x3_get8(row, L.IN, 2 + u, q, xs[u]);
        x3_get8(row, L.GX, u, q, js[u]);  // split chain: GX = J^T X + net_out in one GEMM
      }
    }
  } else {
    for (int k = q; k < PIS_CH; k += 4) sr = fmaf(pn.snlast[k], row[L.H0 + k], sr);
  }
  sr += __shfl_xor(sr, 1, 64);
  sr += __shfl_xor(sr, 2, 64);
  // split rows: smooth from k_pis_time
  const float smooth = X3 ? row[L.SC + 5] : sr + pn.snlastb[0] - pn.smooth0;
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

// Baseline f_b (state part) and g(x) of the n points: one 256-thread block per 64 points (4
// threads per point; a latency chain, so the GMM staging is spread over all 256 threads).  g(x) is
// formed here, inside the label call, rather than by a baseline launch before the rollout: the
// rollout writes g(X_T) and k_pis_final subtracts g(x), so the prepare stream's rollout of the next
// batch depends on nothing but its points.  Lane q sums the GMM statistics of dims d = q mod 4 in
// ascending d, then the quad combines them as (q0 + q1) + (q2 + q3).
template <int KIND, bool X3>
__global__ __launch_bounds__(256) void k_pis_base_final(EqDev e, NetPisDev pn, const float* __restrict__ tx,
                                                        const float* __restrict__ rows, PisRows L, int n,
                                                        float* __restrict__ fb, float* __restrict__ gx) {
  __shared__ PisGmmLds gmm;
  __builtin_amdgcn_s_setprio(2);
  pis_stage_gmm(e, gmm);
  __syncthreads();
  const int i = blockIdx.x * 64 + (threadIdx.x >> 2), q = threadIdx.x & 3;
  const int ic = min(i, n - 1);
  const float* row = rows + (size_t)ic * L.stride;
  float A, B, sm;
  pis_z_stats<X3>(e, pn, gmm, row, L, pn.T - row[L.SC + 0], q, A, B, sm);
  if (i < n && q == 0) fb[i] = Eq<KIND>::ffv(e, 0.f, 0.f, A, B);
  const int nx = e.nx;
  const float* xr = tx + (size_t)ic * (1 + nx) + 1;
  float st[NSG];
#pragma unroll
  for (int c = 0; c < NSG; ++c) st[c] = 0.f;
  for (int d = q; d < nx; d += 4) Eq<KIND>::gstat(e, d, xr[d], st);
#pragma unroll
  for (int c = 0; c < NSG; ++c) {
    st[c] += __shfl_xor(st[c], 1, 64);
    st[c] += __shfl_xor(st[c], 2, 64);
  }
  if (i < n && q == 0) gx[i] = Eq<KIND>::gfin(e, st);
}

// TD terminal value (data.py:941-942): for the rows of points with t + td_dt < T, after the
// forward chain on (t_next, X_{t_next}) rows, u(t_next, X) into SC + 2 (k_pis_final forms
// a_p = u - g(x), as it does for the rollout's g(X_T)), with
// u = smooth (net_out . X) + (1 - smooth) g0(e^{-lambda/2} X), lambda = T - t_next
// (solution.py:256-289).  4 threads per row.
template <int KIND, bool X3>
__global__ void k_pis_tvalue(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0, int nbp,
                             float* __restrict__ rows, PisRows L, int nrows, float td_dt) {
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
  if constexpr (!X3)
    for (int k = q; k < PIS_CH; k += 4) sr = fmaf(pn.snlast[k], row[L.H0 + k], sr);
  sr += __shfl_xor(sr, 1, 64);
  sr += __shfl_xor(sr, 2, 64);
  const float smooth = X3 ? row[L.SC + 5] : sr + pn.snlastb[0] - pn.smooth0;  // split: from k_pis_time
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
  if (r < nrows && q == 0 && td_u) row[L.SC + 2] = u;
}

// Per-path f, b_p and label contributions for one (point, 64-path block) -> partial slab.
template <int KIND, bool X3>
__global__ __launch_bounds__(256) void k_pis_final(EqDev e, NetPisDev pn, const float* __restrict__ tx, int g0,
                                                   int nbp, int K, int flags, const float* __restrict__ fbv,
                                                   const float* __restrict__ gxv, const float* __restrict__ rows,
                                                   PisRows L, float* __restrict__ partial, float td_dt) {
  __shared__ float part[4][4][64];  // per-wave 16-path column sums: [wave][q][value]
  __shared__ float vsum[4][2];      // per-wave sums of the value column and its square
  __shared__ PisGmmLds gmm;
  // the label call's critical path: above a co-resident prepare-stream rollout wave (as the GEMMs)
  __builtin_amdgcn_s_setprio(2);
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
  // a_p = g(X_T) - g(x), g(X_T) from the rollout parts' statistics combined as (q0 + q1) + (q2 + q3)
  // (TD: u(t_next, X) - g(x) where t_next < T, u from k_pis_tvalue)
  float ap = 0.f;
  if (TERM) {
    float gv;
    if (td_u) {
      gv = row[L.SC + 2];
    } else {
      static_assert(PIS_PARTS == 4, "the fixed combine order below");
      float st[NSG];
      const float* gp = row + L.SC + PIS_GST;
#pragma unroll
      for (int c = 0; c < NSG; ++c)
        st[c] = (gp[c] + gp[NSG + c]) + (gp[2 * NSG + c] + gp[3 * NSG + c]);
      gv = Eq<KIND>::gfin(e, st);
    }
    ap = gv - gxv[i];
  }
  const float s = row[L.SC + 0], smt = row[L.SC + 3];
  float A, B, sm;
  pis_z_stats<X3>(e, pn, gmm, row, L, pn.T - s, q, A, B, sm);
  const float bp = INTG ? tmt * (Eq<KIND>::ffv(e, 0.f, 0.f, A, B) - f_b) : 0.f;
  const float yT = 1.0f / (sqrtf(Kf * tmt) * e.asq), yI = 1.0f / (sqrtf(Kf * smt) * e.asq);
  // this row's contributions: v[2k + mom] for dim d = 16 (k >> 2) + 4 q + (k & 3) (k < 32: nx <= 128),
  // the value column (lane group q = 0) apart.  The noise sums come in 16-B loads: the 4 lanes of a
  // row read 64 contiguous bytes per instruction (8 + 8 loads per lane instead of 32 + 32 single floats)
  static_assert(NXP_MAX <= 128, "dims per lane group");
  float v[64];
  const float aY = ap * yT, bY = bp * yI;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int d0 = 16 * kk + 4 * q;
    float4 st4 = make_float4(0.f, 0.f, 0.f, 0.f), ss4 = st4;
    if (d0 < nx) {  // the regions hold round_up(nx, 4) floats: a quad never leaves its region
      st4 = *reinterpret_cast<const float4*>(row + L.ST + d0);
      ss4 = *reinterpret_cast<const float4*>(row + L.SS + d0);
    }
    const float sts[4] = {st4.x, st4.y, st4.z, st4.w}, sss[4] = {ss4.x, ss4.y, ss4.z, ss4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * kk + j;
      const float c = d0 + j < nx ? fmaf(aY, sts[j], bY * sss[j]) : 0.f;
      v[2 * k] = c;
      v[2 * k + 1] = c * c;
    }
  }
  float c0 = q == 0 ? ap + bp + (INTG ? (f_b + Eq<KIND>::ffc(e)) * tmt : 0.f) : 0.f, c0s = c0 * c0;
  // sum over the wave's 16 rows (lane = 4 row + q) by a halving butterfly on lane bits 5..2: at bit
  // m a lane keeps the half of its values selected by that bit and adds its partner's copy, so lane
  // (row r, q) ends with values 4r .. 4r + 3 summed over the 16 rows of lane group q.  Bits 5 and 4
  // (48 of the 60 exchanges) are the gfx950 VALU lane swaps (v_permlane32/16_swap, no LDS
  // crossbar); every sum is the same pair of operands as an xor exchange, so bitwise unchanged.
  const int lane = tid & 63, wv = tid >> 6;
  c0 = qsum(c0);  // the value column over the same lane bits (5, 4 here; 3, 2 below)
  c0s = qsum(c0s);
#pragma unroll
  for (int bit = 3; bit >= 2; --bit) {
    c0 += __shfl_xor(c0, 1 << bit, 64);
    c0s += __shfl_xor(c0s, 1 << bit, 64);
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = swap32_sum(v[j], v[j + 32]);
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = swap16_sum(v[j], v[j + 16]);
#define DPI_HALVE(BIT, H)                                          \
  _Pragma("unroll") for (int j = 0; j < H; ++j) {                  \
    const bool up = (lane >> BIT) & 1;                             \
    const float keep = up ? v[j + H] : v[j];                       \
    const float send = up ? v[j] : v[j + H];                       \
    v[j] = keep + __shfl_xor(send, 1 << BIT, 64);                  \
  }
  DPI_HALVE(3, 8)
  DPI_HALVE(2, 4)
#undef DPI_HALVE
#pragma unroll
  for (int j = 0; j < 4; ++j) part[wv][q][4 * (lane >> 2) + j] = v[j];
  if (lane == 0) {
    vsum[wv][0] = c0;
    vsum[wv][1] = c0s;
  }
  __syncthreads();
  // the four waves' sums, (w0 + w1) + (w2 + w3): a fixed order independent of rank and chunk
  float* out = partial + ((size_t)i * nbp + b) * slab_row(F);  // [point][block][slab_row(F)]
  {
    const int qq = tid >> 6, j = tid & 63, k = j >> 1, mom = j & 1, d = 16 * (k >> 2) + 4 * qq + (k & 3);
    const float sum = (part[0][qq][j] + part[1][qq][j]) + (part[2][qq][j] + part[3][qq][j]);
    if (d < nx) out[mom * F + 1 + d] = sum;
    if (tid < 2) out[tid * F] = (vsum[0][tid] + vsum[1][tid]) + (vsum[2][tid] + vsum[3][tid]);
  }
}

}  // namespace dpi
