// Schedule experiments on the product split-storage GEMM (dpi_gemm.h k_gemm_x3<EPI, 4, VAR>) at the
// HJB pipeline's size (R = 262,144 paths, 512 x 512, fp16-split): us per launch, effective TF/s
// (3 f16 products per fp32 product: 833 TF/s peak) and the number of output words that differ
// from VAR = 0 (0 = the schedule change is bitwise neutral).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_x3 tools/ubench_x3.hip
//   tools/ubench_x3 [M] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <vector>

#include "../deeppicarditeration_amd/csrc/dpi_device.h"


// =============================================================================================
// Negative result kept for the record (round 2): k_gemm_x4, a 256 x 256 block tile with one wave
// per SIMD owning 128 x 128 (256 AGPR accumulators), X in a 3-slot and W in a 2-slot LDS ring
// (160 KB).  Bitwise equal to k_gemm_x3 (the same products per output in the same order) but not
// faster at R = 262,144: 614 / 667 us (ELU / DELU) against the product's 556 / 622 us with the
// builtin MFMAs (the register allocator ping-pongs accumulators through v_accvgpr moves once they
// are pinned to AGPRs; unpinned it spills), and the in-place inline-asm MFMA form (550 / 614 us)
// races — the compiler's hazard recognizer does not see inline-asm MFMAs, and 4 % of the outputs
// came out wrong.  One wave per SIMD also leaves every barrier's and every fragment reload's
// latency exposed.  The 2-wave 256 x 128 product kernel stays.
namespace dpi {
// ---------------------------------------------------------------------------------------------
// k_gemm_x4: the same split-storage GEMM as k_gemm_x3 (same operands, epilogues and, per output,
// the same products in the same order — bitwise equal outputs) on a 256 x 256 block tile with ONE
// wave per SIMD owning 128 m x 128 n (8 x 8 MFMA tiles, 256 accumulator registers).
// Why: k_gemm_x3's 256 x 128 tile moves 48 KB of L2 -> LDS per 32-deep chunk for 1,536 MFMA
// cycles per SIMD (62 GB/s per CU at 2 GHz), the rate the XCD L2 feeds LDS-DMA at, so its main
// loop keeps the matrix pipes 71 % busy (PMC: MFMA busy 41 % of the launch with the prologue and
// epilogue).  256 x 256 moves 64 KB per 3,072 MFMA cycles per SIMD (2/3 of the bytes per MFMA).
// LDS: X (path rows) in a 3-slot ring (their first n-tile comes from HBM), W in a 2-slot ring
// (always L2-hot): 5 x 32 KB = 160 KB.  Fragments: A (W rows) double-buffered across chunks, B (X
// rows) single-buffered — B of m-tile b is reloaded from chunk u + 1 as soon as chunk u's 24
// MFMAs on it have issued.
constexpr int X4_BM = 256, X4_BN = 256, X4_THREADS = 256, X4_XS = 3, X4_WS = 2;

template <int EPI, int DBG = 0>
__global__ __launch_bounds__(X4_THREADS, 1) void k_gemm_x4(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                           float wscale, const float* __restrict__ X, int ldx,
                                                           const float* __restrict__ X2, int ldx2, int nk1,
                                                           float* __restrict__ OUT, int ldc,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ AUX, int ldaux) {
  constexpr int SLOT = 256 * 32;  // words: 256 rows x 128 B
  __shared__ uint32_t xs[X4_XS * SLOT];
  __shared__ uint32_t ws[X4_WS * SLOT];
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, loc = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int m0 = mt * X4_BM, n0 = nt * X4_BN;
  const int nk = Kp >> 5;
  const uint32_t* Xw = reinterpret_cast<const uint32_t*>(X);
  const uint32_t* X2w = reinterpret_cast<const uint32_t*>(X2);

  // LDS-DMA of 256 rows x 128 B: wave-instruction k of this wave fills rows r = 32 k + r0,
  // r0 = 8 wv + lane / 8; x3_swz(32 k + r0) = x3_swz(r0), so a lane's source offset within its row
  // block is the same for every k: one 32-bit VGPR offset per lane and uniform (SGPR) row-block
  // bases, instead of 16 live 64-bit addresses.
  const int r0 = 8 * wv + (lane >> 3), g0 = (lane & 7) ^ x3_swz(r0);
  const uint32_t w_off = (uint32_t)(r0 * Kp + 4 * g0) * 4u;  // bytes
  const bool full_m = m0 + X4_BM <= M;
  auto dma = [&](const void* src, uint32_t* dst) __attribute__((always_inline)) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };
  auto issue_w = [&](int c, int slot) __attribute__((always_inline)) {
    uint32_t* dst = ws + slot * SLOT + 256 * wv;
    const char* base = reinterpret_cast<const char*>(W + (size_t)n0 * Kp + 32 * c);
#pragma unroll
    for (int k = 0; k < 8; ++k) dma(base + (size_t)32 * k * Kp * 4 + w_off, dst + 1024 * k);
  };
  auto issue_x = [&](int c, int slot) __attribute__((always_inline)) {
    uint32_t* dst = xs + slot * SLOT + 256 * wv;
    const bool one = c < nk1;  // wave-uniform source select (no branches in the DMA issue)
    const uint32_t* xb = one ? Xw + 32 * c : X2w + 32 * (c - nk1);
    const int ld = one ? ldx : ldx2;
    if (full_m && !(DBG & 1)) {
      const char* base = reinterpret_cast<const char*>(xb + (size_t)m0 * ld);
      const uint32_t off = (uint32_t)(r0 * ld + 4 * g0) * 4u;
#pragma unroll
      for (int k = 0; k < 8; ++k) dma(base + (size_t)32 * k * ld * 4 + off, dst + 1024 * k);
    } else {  // the last m-tile: rows past M re-read row M - 1
#pragma unroll
      for (int k = 0; k < 8; ++k) dma(xb + (size_t)min(m0 + 32 * k + r0, M - 1) * ld + 4 * g0, dst + 1024 * k);
    }
  };
  // fragment rows are 16-aligned + il, and x3_swz(16 j + il) = x3_swz(il): a lane's two granule
  // offsets within a 16-row tile are the same for every tile (one VGPR each, tiles by immediates)
  const int swl = x3_swz(il);
  const int fo_h = il * 32 + 4 * ((2 * ql) ^ swl), fo_l = il * 32 + 4 * ((2 * ql + 1) ^ swl);
  auto frag = [&](const uint32_t* buf, int row16, h8& h, h8& l) __attribute__((always_inline)) {
    if constexpr (DBG & 2) {
      const int row = row16 + il, sw = x3_swz(row);
      const uint32_t* rp = buf + row * 32;
      h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ sw)));
      l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ sw)));
    } else {
      const uint32_t* rp = buf + row16 * 32;  // row16: the tile's first row (wave-uniform)
      h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + fo_h));
      l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + fo_l));
    }
  };

  f4v acc[8][8];  // [n-tile t][m-tile b]
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  // A of n-tiles 0-3 double-buffered across chunks (aL[F]), of n-tiles 4-7 single (aH); B single
  h8 alh[2][4], all_[2][4], ahh[4], ahl[4], bh[8], bl[8];
  // The 256 accumulators live in the AGPR file and the fragments in VGPRs ("+a" / "v" inline
  // MFMAs, accumulated in place): with the builtin the register allocator mixes fragments into
  // AGPRs and spills, and pinning the builtin's result makes it ping-pong accumulators through
  // v_accvgpr moves.  Dependent MFMAs on one accumulator issue back to back (srcC = dst); the
  // fragment reloads come long after the MFMAs that read those VGPRs (LDS latency); the epilogue's
  // AGPR reads wait behind explicit s_nops.
  auto mma = [&](int t, int b, const h8& xh, const h8& xl) __attribute__((always_inline)) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[t][b]) : "v"(xh), "v"(bh[b]));
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[t][b]) : "v"(xh), "v"(bl[b]));
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[t][b]) : "v"(xl), "v"(bh[b]));
  };
  // chunk u's MFMAs with chunk u + 1's fragments read behind them: B[b] once m-tile b is done,
  // aL[F ^ 1][b] during m-tiles b = 0..3, aH during the last m-tile (after its n-tiles 4-7)
  auto step = [&](int u, auto Fc, bool next) __attribute__((always_inline)) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* wb = ws + ((u + 1) % X4_WS) * SLOT;
    const uint32_t* xb = xs + ((u + 1) % X4_XS) * SLOT;
    if constexpr (DBG & 4) {  // debug: all MFMAs, then all reads
#pragma unroll
      for (int b = 0; b < 8; ++b) {
#pragma unroll
        for (int t = 0; t < 4; ++t) mma(t, b, alh[F][t], all_[F][t]);
#pragma unroll
        for (int t = 4; t < 8; ++t) mma(t, b, ahh[t - 4], ahl[t - 4]);
      }
      if (next)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          frag(xb, 128 * wm + 16 * b, bh[b], bl[b]);
          if (b < 4)
            frag(wb, 128 * wn + 16 * b, alh[F ^ 1][b], all_[F ^ 1][b]);
          else
            frag(wb, 128 * wn + 16 * b, ahh[b - 4], ahl[b - 4]);
        }
      return;
    }
#pragma unroll
    for (int b = 0; b < 7; ++b) {
#pragma unroll
      for (int t = 0; t < 4; ++t) mma(t, b, alh[F][t], all_[F][t]);
#pragma unroll
      for (int t = 4; t < 8; ++t) mma(t, b, ahh[t - 4], ahl[t - 4]);
      if (next) {
        frag(xb, 128 * wm + 16 * b, bh[b], bl[b]);
        if (b < 4) frag(wb, 128 * wn + 16 * b, alh[F ^ 1][b], all_[F ^ 1][b]);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep each reload behind the MFMAs that free its registers
    }
#pragma unroll
    for (int t = 4; t < 8; ++t) mma(t, 7, ahh[t - 4], ahl[t - 4]);
    __builtin_amdgcn_sched_barrier(0);
    if (next)
#pragma unroll
      for (int t = 4; t < 8; ++t) frag(wb, 128 * wn + 16 * t, ahh[t - 4], ahl[t - 4]);
#pragma unroll
    for (int t = 0; t < 4; ++t) mma(t, 7, alh[F][t], all_[F][t]);
    __builtin_amdgcn_sched_barrier(0);
    if (next) frag(xb, 128 * wm + 16 * 7, bh[7], bl[7]);
    __builtin_amdgcn_sched_barrier(0);
  };
  // iteration u (u + 1 < nk): publish chunk u + 1, refill the slots chunk u used, multiply chunk u
  auto body = [&](int u, auto Fc) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);                 // lgkmcnt(0): chunk u's fragments landed
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own DMA of chunk u + 1 landed (X(u + 2) may fly)
    __builtin_amdgcn_s_barrier();
    issue_w(min(u + 2, nk - 1), u % X4_WS);
    issue_x(min(u + 3, nk - 1), u % X4_XS);
    step(u, Fc, true);
  };
  // prologue: W0 X0 X1 W1 X2 in flight; chunk 0 published and read
  issue_w(0, 0);
  issue_x(0, 0);
  issue_x(min(1, nk - 1), 1);
  issue_w(min(1, nk - 1), 1);
  issue_x(min(2, nk - 1), 2);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (DBG & 8) {  // debug: dump X slot 0 and W slot 0 of block 0 after the prologue
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (blockIdx.x == 0)
      for (int i = tid; i < 5 * SLOT; i += X4_THREADS)
        reinterpret_cast<uint32_t*>(OUT)[i] = i < 3 * SLOT ? xs[i] : ws[i - 3 * SLOT];
    return;
  }
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b < 4)
      frag(ws, 128 * wn + 16 * b, alh[0][b], all_[0][b]);
    else
      frag(ws, 128 * wn + 16 * b, ahh[b - 4], ahl[b - 4]);
    frag(xs, 128 * wm + 16 * b, bh[b], bl[b]);
  }
  // nk even (host-checked): pairs of chunks, the last pair's second chunk without reads — one
  // loop and no branches around it, so the accumulators never meet at a join
  for (int u = 0; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  body(nk - 2, std::integral_constant<int, 0>{});
  __builtin_amdgcn_s_waitcnt(0xC07F);
  step(nk - 1, std::integral_constant<int, 1>{}, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail DMAs land before the LDS is released
  // the last MFMAs' results (16x16x32 f16: 8 passes) before any AGPR read
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int b = 0; b < 8; ++b) asm volatile("" : "+a"(acc[t][b]));  // every AGPR read stays behind the nops

  // epilogue: lane (il, ql) of m-tile b holds OUT[m = m0 + 128 wm + 16 b + il][n = n0 + 128 wn + 16 t + 4 ql + r]
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const int m = m0 + 128 * wm + 16 * b + il;
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int U = (n0 >> 5) + 4 * wn + c;
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
        x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : a[j] + 1.0f;
      }
      x3_put8(OUT + (size_t)m * ldc, 0, U, ql, v);
    }
  }
}

}  // namespace dpi


// Persistent walk of the product tile body (x3_tile), G blocks (one per CU), block b takes the
// virtual blocks v = b + j G through the same XCD remap as the product; STAG > 0: blocks whose
// in-XCD index is odd (STAG = 2) or = 1, 2, 3 mod 4 (STAG = 4) first sleep that fraction of a tile
// (TILE_CYC cycles), so that the CUs' epilogue store bursts do not all coincide.
namespace dpi {
template <int EPI, int STAG>
__global__ __launch_bounds__(X3_THREADS, 1) void k_gemm_x3s(int M, int Kp, int n_ntiles, int n_tiles,
                                                            const uint32_t* __restrict__ W, float wscale,
                                                            const float* __restrict__ X, int ldx, float* __restrict__ OUT,
                                                            int ldc, const float* __restrict__ bias,
                                                            const float* __restrict__ AUX, int ldaux, int tile_cyc) {
  __shared__ X3Lds<4> lds;
  const int G = gridDim.x, b = blockIdx.x;
  if (STAG > 0) {
    const int ph = (b >> 3) % STAG;
    const long long until = (long long)tile_cyc * ph / STAG;
    const long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < until) __builtin_amdgcn_s_sleep(32);
  }
  const int q8 = n_tiles >> 3, r8 = n_tiles & 7;
  for (int v = b; v < n_tiles; v += G) {
    const int xcd = v & 7, loc = v >> 3;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    x3_tile<EPI, 4, 0>(lds.sm, mt * X3_BM, nt * 128, M, Kp, W, wscale, X, ldx, X, ldx, Kp >> 5, OUT, ldc,
                       EPI == EPI_DELU ? nullptr : bias, AUX, ldaux);
    __syncthreads();
  }
}
}  // namespace dpi

using namespace dpi;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void k_fill(float* rows, int M, int Kp, int ld, uint32_t seed, float scale) {
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

static int g_stage = 1;  // DELU epilogue operands staged through the ring (k_gemm_x3 stage_aux)

struct Bufs {
  int M, Kp, Np;
  uint32_t* W;
  float *X, *AUX, *OUT, *REF, *bias;
};

// VAR 100+: k_gemm_x4 (256 x 256 tile, one wave per SIMD); VAR 200 + STAG: persistent x3_tile walk
template <int EPI, int VAR>
static void launch(const Bufs& b, float* out) {
  if constexpr (VAR >= 200) {
    const int nnt = b.Np / 128, nmt = (b.M + X3_BM - 1) / X3_BM;
    hipLaunchKernelGGL((k_gemm_x3s<EPI, VAR - 200>), dim3(256), dim3(X3_THREADS), 0, 0, b.M, b.Kp, nnt, nnt * nmt, b.W,
                       1.0f / 16.0f, b.X, b.Kp, out, b.Np, b.bias, b.AUX, b.Np, 27000 * 2);
  } else if constexpr (VAR >= 100) {
    const int nnt = b.Np / X4_BN, nmt = (b.M + X4_BM - 1) / X4_BM;
    hipLaunchKernelGGL((k_gemm_x4<EPI, VAR - 100>), dim3(nnt * nmt), dim3(X4_THREADS), 0, 0, b.M, b.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, b.Kp, b.X, b.Kp, b.Kp / 32, out, b.Np, EPI == EPI_DELU ? nullptr : b.bias, b.AUX, b.Np);
  } else {
    const int nnt = b.Np / 128, nmt = (b.M + X3_BM - 1) / X3_BM;
    hipLaunchKernelGGL((k_gemm_x3<EPI, 4, VAR>), dim3(nnt * nmt), dim3(X3_THREADS), 0, 0, b.M, b.Kp, nnt, b.W,
                       1.0f / 16.0f, b.X, b.Kp, b.X, b.Kp, b.Kp / 32, out, b.Np, EPI == EPI_DELU ? nullptr : b.bias,
                       b.AUX, b.Np, g_stage);
  }
}

template <int EPI, int VAR>
static void run(const char* name, const Bufs& b, int iters) {
  launch<EPI, VAR>(b, b.OUT);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch<EPI, VAR>(b, b.OUT);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters;
  std::vector<uint32_t> a((size_t)b.M * b.Np), r((size_t)b.M * b.Np);
  CK(hipMemcpy(a.data(), b.OUT, a.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), b.REF, r.size() * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  int hist[16][16] = {};  // [row % 256 / 16][word % 512 / 32] of differing words
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i] != r[i]) {
      ++bad;
      ++hist[(i / b.Np) % 256 / 16][(i % b.Np) / 32];
    }
  if (bad && VAR == 100 && false) {
    int h32[32] = {};
    int shown = 0;
    for (size_t i = 0; i < a.size(); ++i)
      if (a[i] != r[i]) {
        ++h32[i % 32];
        if (shown < 6) {
          std::printf("  row %zu word %zu: %08x vs %08x\n", i / b.Np, i % b.Np, a[i], r[i]);
          ++shown;
        }
      }
    for (int x = 0; x < 32; ++x) std::printf(" %d", h32[x]);
    std::printf("\n");
    // which REF rows / columns do x4's bad rows hold?  compare word 0..31 of bad row against all REF rows < 512
    for (int row = 0; row < 48; ++row) {
      bool rowbad = false;
      for (int w = 0; w < b.Np; ++w) rowbad |= a[(size_t)row * b.Np + w] != r[(size_t)row * b.Np + w];
      if (!rowbad) continue;
      int match = -1, nmatch = 0;
      for (int rr = 0; rr < 512; ++rr) {
        int eq = 0;
        for (int w = 0; w < 32; ++w) eq += a[(size_t)row * b.Np + w] == r[(size_t)rr * b.Np + w];
        if (eq > nmatch) nmatch = eq, match = rr;
      }
      std::printf("  bad row %d: best REF row %d (%d of 32 words equal)\n", row, match, nmatch);
    }
  }
  std::printf("%-4s VAR %2d %-40s %8.1f us  %6.1f TF/s(split-eff)  differing words %zu\n",
              EPI == EPI_DELU ? "delu" : "elu", VAR, name, us, 2.0 * b.M * (double)b.Kp * b.Np / (us * 1e-6) / 1e12,
              bad);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  Bufs b;
  b.M = argc > 1 ? std::atoi(argv[1]) : 262144;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
  b.Kp = 512;
  b.Np = 512;
  CK(hipMalloc(&b.W, (size_t)b.Np * b.Kp * 4));
  CK(hipMalloc(&b.X, (size_t)b.M * b.Kp * 4));
  CK(hipMalloc(&b.AUX, (size_t)b.M * b.Np * 4));
  CK(hipMalloc(&b.OUT, (size_t)b.M * b.Np * 4));
  CK(hipMalloc(&b.REF, (size_t)b.M * b.Np * 4));
  CK(hipMalloc(&b.bias, b.Np * 4));
  hipLaunchKernelGGL(k_fill, dim3(b.Np), dim3(128), 0, 0, reinterpret_cast<float*>(b.W), b.Np, b.Kp, b.Kp, 7u, 0.8f);
  hipLaunchKernelGGL(k_fill, dim3(b.M), dim3(128), 0, 0, b.X, b.M, b.Kp, b.Kp, 11u, 1.0f);
  hipLaunchKernelGGL(k_fill, dim3(b.M), dim3(128), 0, 0, b.AUX, b.M, b.Np, b.Np, 13u, 1.5f);
  std::vector<float> hb(b.Np);
  for (int i = 0; i < b.Np; ++i) hb[i] = 0.01f * (float)((i * 37) % 17 - 8);
  CK(hipMemcpy(b.bias, hb.data(), b.Np * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());

  if (argc > 3 && std::strcmp(argv[3], "lds") == 0) {  // debug: LDS image after the prologue
    launch<EPI_BIAS_ELU, 108>(b, b.OUT);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> img(5 * 256 * 32), xw((size_t)256 * b.Kp), hw((size_t)256 * b.Kp);
    CK(hipMemcpy(img.data(), b.OUT, img.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(xw.data(), b.X, xw.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hw.data(), b.W, hw.size() * 4, hipMemcpyDeviceToHost));
    // block 0's tile after the XCD remap: tile 0 = m-tile 0, n-tile 0; X slots hold chunks 0, 1, 2, W slots 0, 1
    auto swz = [](int r) { return ((r >> 1) & 7) ^ ((((r + 4) >> 3) & 1) << 1); };
    for (int sl = 0; sl < 5; ++sl) {
      const bool isx = sl < 3;
      const int chunk = isx ? sl : sl - 3;
      const std::vector<uint32_t>& src = isx ? xw : hw;
      int bad = 0;
      for (int r = 0; r < 256; ++r)
        for (int p = 0; p < 8; ++p)
          for (int j = 0; j < 4; ++j) {
            const uint32_t got = img[sl * 8192 + r * 32 + 4 * p + j];
            const uint32_t want = src[(size_t)r * b.Kp + 32 * chunk + 4 * (p ^ swz(r)) + j];
            if (got != want && bad++ < 3) std::printf("  slot %d row %d pos %d word %d: got %08x want %08x\n", sl, r, p, j, got, want);
          }
      std::printf("slot %d (%s chunk %d) mismatches: %d\n", sl, isx ? "X" : "W", chunk, bad);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "cpu") == 0) {  // debug: x4 and product vs a CPU GEMM (BIAS epilogue, no bias)
    std::vector<uint32_t> hw((size_t)b.Np * b.Kp), hx((size_t)256 * b.Kp), o4((size_t)256 * b.Np), o3((size_t)256 * b.Np);
    CK(hipMemcpy(hw.data(), b.W, hw.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hx.data(), b.X, hx.size() * 4, hipMemcpyDeviceToHost));
    Bufs s1 = b;
    s1.M = 256;
    s1.bias = nullptr;
    launch<EPI_BIAS, 100>(s1, b.OUT);
    launch<EPI_BIAS, 0>(s1, b.REF);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o4.data(), b.OUT, o4.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o3.data(), b.REF, o3.size() * 4, hipMemcpyDeviceToHost));
    auto dec = [](const uint32_t* row, int c) {
      const int u = c >> 5, w = c & 31, q = (w >> 2) & 3, j = (w & 3) + 4 * (w >> 4);
      const uint32_t hw_ = row[32 * u + 8 * q + (j >> 1)], lw = row[32 * u + 8 * q + 4 + (j >> 1)];
      const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? hw_ >> 16 : hw_ & 0xFFFF));
      const _Float16 l = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? lw >> 16 : lw & 0xFFFF));
      return (double)(float)h + (double)(float)l;
    };
    for (int m : {0, 1, 14, 15, 16, 17, 31}) {
      double e4 = 0, e3 = 0;
      for (int n = 0; n < 64; ++n) {
        double ref = 0;
        for (int k = 0; k < b.Kp; ++k) ref += dec(&hw[(size_t)n * b.Kp], k) * dec(&hx[(size_t)m * b.Kp], k);
        ref /= 16.0;
        e4 = std::max(e4, std::fabs(dec(&o4[(size_t)m * b.Np], n) - ref));
        e3 = std::max(e3, std::fabs(dec(&o3[(size_t)m * b.Np], n) - ref));
      }
      std::printf("row %2d: max|x4 - cpu| %.3e  max|product - cpu| %.3e\n", m, e4, e3);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "stag") == 0) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(b.OUT, 0, (size_t)b.M * b.Np * 4));
      launch<EPI_BIAS_ELU, 0>(b, b.REF);
      run<EPI_BIAS_ELU, 0>("product", b, iters);
      run<EPI_BIAS_ELU, 200>("persistent x3_tile walk", b, iters);
      run<EPI_BIAS_ELU, 202>("persistent, 2-phase stagger", b, iters);
      run<EPI_BIAS_ELU, 204>("persistent, 4-phase stagger", b, iters);
      CK(hipMemset(b.OUT, 0, (size_t)b.M * b.Np * 4));
      launch<EPI_DELU, 0>(b, b.REF);
      run<EPI_DELU, 0>("product", b, iters);
      run<EPI_DELU, 200>("persistent x3_tile walk", b, iters);
      run<EPI_DELU, 202>("persistent, 2-phase stagger", b, iters);
      run<EPI_DELU, 204>("persistent, 4-phase stagger", b, iters);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "x4") == 0) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(b.OUT, 0, (size_t)b.M * b.Np * 4));
      launch<EPI_BIAS_ELU, 0>(b, b.REF);
      run<EPI_BIAS_ELU, 0>("product", b, iters);
      run<EPI_BIAS_ELU, 100>("k_gemm_x4 256x256, 1 wave/SIMD", b, iters);

      launch<EPI_DELU, 0>(b, b.REF);
      run<EPI_DELU, 0>("product", b, iters);
      run<EPI_DELU, 100>("k_gemm_x4 256x256, 1 wave/SIMD", b, iters);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "half") == 0) {  // 128 x 128 tile, two blocks per CU (k_gemm_x3h)
    for (int rep = 0; rep < 2; ++rep) {
      for (int e = 0; e < 2; ++e) {
        const int nnt = b.Np / 128, nmt = (b.M + X3H_BM - 1) / X3H_BM;
        if (e == 0) {
          launch<EPI_BIAS_ELU, 0>(b, b.REF);
          run<EPI_BIAS_ELU, 0>("product 256 x 128", b, iters);
        } else {
          launch<EPI_DELU, 0>(b, b.REF);
          run<EPI_DELU, 0>("product 256 x 128", b, iters);
        }
        CK(hipMemset(b.OUT, 0, (size_t)b.M * b.Np * 4));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto go = [&]() {
          if (e == 0)
            hipLaunchKernelGGL(k_gemm_x3h<EPI_BIAS_ELU>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, b.M, b.Kp, nnt, b.W,
                               1.0f / 16.0f, b.X, b.Kp, b.X, b.Kp, b.Kp / 32, b.OUT, b.Np, b.bias, b.AUX, b.Np);
          else
            hipLaunchKernelGGL(k_gemm_x3h<EPI_DELU>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, b.M, b.Kp, nnt, b.W,
                               1.0f / 16.0f, b.X, b.Kp, b.X, b.Kp, b.Kp / 32, b.OUT, b.Np, nullptr, b.AUX, b.Np);
        };
        go();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < iters; ++i) go();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<uint32_t> a((size_t)b.M * b.Np), r((size_t)b.M * b.Np);
        CK(hipMemcpy(a.data(), b.OUT, a.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), b.REF, r.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < a.size(); ++i) bad += a[i] != r[i];
        std::printf("%-4s x3h 128 x 128, 2 blocks/CU %26s %8.1f us  differing words %zu\n", e == 0 ? "elu" : "delu", "",
                    ms * 1e3 / iters, bad);
        std::fflush(stdout);
      }
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "bias") == 0) {  // ELU: bias staged in LDS (product) vs epilogue loads (VAR 8)
    for (int rep = 0; rep < 3; ++rep) {
      launch<EPI_BIAS_ELU, 0>(b, b.REF);
      run<EPI_BIAS_ELU, 8>("ELU bias: epilogue global loads", b, iters);
      CK(hipMemset(b.OUT, 0, (size_t)b.M * b.Np * 4));
      run<EPI_BIAS_ELU, 0>("ELU bias: staged in LDS", b, iters);
    }
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "stage") == 0) {  // DELU: staged epilogue operands vs epilogue loads
    // K 512 / 128 are the HJB chain's; 96 and 160 (odd chunk counts) and a partial last m-tile
    // (M % 256 != 0) cover the staging's other branches
    const int M0 = b.M;
    for (int kp : {512, 128, 96, 160}) {
      b.Kp = kp;
      for (int m : {M0, M0 - 192}) {
        b.M = m;
        for (int rep = 0; rep < (kp >= 128 && m == M0 ? 2 : 1); ++rep) {
          char n0[64], n1[64];
          std::snprintf(n0, sizeof n0, "K %d M %d epilogue loads", kp, m);
          std::snprintf(n1, sizeof n1, "K %d M %d staged", kp, m);
          g_stage = 0;
          launch<EPI_DELU, 0>(b, b.REF);
          run<EPI_DELU, 0>(n0, b, iters);
          g_stage = 1;
          CK(hipMemset(b.OUT, 0, (size_t)M0 * b.Np * 4));
          run<EPI_DELU, 0>(n1, b, iters);
        }
      }
    }
    b.M = M0;
    return 0;
  }
  if (argc > 3 && std::strcmp(argv[3], "prod") == 0) {  // profiling: the product kernels only
    launch<EPI_BIAS_ELU, 0>(b, b.REF);
    run<EPI_BIAS_ELU, 0>("product", b, iters);
    launch<EPI_DELU, 0>(b, b.REF);
    run<EPI_DELU, 0>("product", b, iters);
    return 0;
  }
  launch<EPI_BIAS_ELU, 0>(b, b.REF);
  CK(hipDeviceSynchronize());
  run<EPI_BIAS_ELU, 0>("product", b, iters);
  run<EPI_BIAS_ELU, 1>("setprio 1 for waves 4-7", b, iters);
  run<EPI_BIAS_ELU, 2>("reads front-loaded", b, iters);
  run<EPI_BIAS_ELU, 4>("DMA issue among the first MFMAs", b, iters);
  run<EPI_BIAS_ELU, 6>("front-loaded + DMA interleave", b, iters);
  run<EPI_BIAS_ELU, 7>("all three", b, iters);
  run<EPI_BIAS_ELU, 0>("product (again)", b, iters);

  launch<EPI_DELU, 0>(b, b.REF);
  CK(hipDeviceSynchronize());
  run<EPI_DELU, 0>("product", b, iters);
  run<EPI_DELU, 1>("setprio 1 for waves 4-7", b, iters);
  run<EPI_DELU, 2>("reads front-loaded", b, iters);
  run<EPI_DELU, 4>("DMA issue among the first MFMAs", b, iters);
  run<EPI_DELU, 6>("front-loaded + DMA interleave", b, iters);
  run<EPI_DELU, 7>("all three", b, iters);
  run<EPI_DELU, 0>("product (again)", b, iters);
  std::printf("done\n");
  return 0;
}
