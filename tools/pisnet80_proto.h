// Measured and not kept (r03aa): k_pis_net with 80 rows per block (no X image;
// X and A_{L-1} reloaded into the one 160 KB image).  Two weight sets: bitwise equal, slower than
// the 64-row kernel; three sets spill.  Not built.
// k_pis_net: the whole split-storage PISGradNet nn_module chain of pis_chain_x3 (solution.py:256-289)
// in ONE launch, 80 rows per block, with the 512-wide activations held in LDS across layers.
//
// pis_chain_x3 runs the chain as 9 k_gemm_x3h launches; between launches every 512-wide activation
// and cotangent makes an HBM round trip (13 GB per HJB label call) and every launch pays its tiles'
// prologues and epilogues.  Here a block takes 80 rows through
//   forward   A_l = elu(W_l A_{l-1} + b_l)                       l = 0 .. L-1  (A_{-1} = IN)
//   VJP       D_{L-1} = (nnT[L] X) * elu'(A_{L-1}),  D_{l-1} = (nnT[l] D_l) * elu'(A_{l-1})
//   output    GX = [D_0 | A_{L-1}] . [nnT[0] | nn[L]]^T + b_L
// with the current operand (at most 512 wide) in a 160 KB LDS image: 80 rows x 16 chunks, chunk-major,
// each 32-deep chunk an 80-row slab laid out like a k_gemm_x3h ring slot.  One block (8 waves, 2 per
// SIMD) per CU.  Only A_0 .. A_{L-1} go to HBM (the VJP's elu' operands and the second half of GX's
// K), and GX; the inputs IN and X = IN[:, 64:] are read from the rollout's rows.
//
// What bounds it: every weight fragment comes from L2 (the chain's 7 MB of fragment-major weights
// are shared by all blocks) and one block re-reads all of them per tile, so the L2 -> CU bytes per
// MFMA fall with the rows a block holds — 80, the most whose 512-wide split activation (2 KB per
// row) fits the LDS.  Wave w owns units 64 w .. 64 w + 63 of every 512-wide product: its weight
// rows are private, so the MFMA A operands come straight into registers as buffer loads (1 KB
// contiguous per instruction, two chunks ahead); the B operands are the shared LDS image.  Per chunk
// and output the same three products in the same order as k_gemm_x3h (hi.hi, hi.lo, lo.hi into one
// accumulator), the same epilogue arithmetic and the same split on store, so every row's GX is
// bitwise equal to the layer-wise chain (tests/test_gpu_fullsize.py).
#pragma once

namespace dpi {

constexpr int PN_BM = 80, PN_NB = PN_BM / 16, PN_THREADS = 512;
constexpr int PN_SLAB = PN_BM * 32;           // words per 32-deep chunk slab
constexpr int PN_H = 512, PN_HC = PN_H / 32;  // hidden width and its chunks
constexpr int PN_XC = 4;                      // chunks of the x part of IN (nx <= 128)

struct PnLds {
  uint32_t act[PN_HC * PN_SLAB];  // 160 KB: the current operand
};

typedef _Float16 pn_h8 __attribute__((ext_vector_type(8)));
typedef float pn_f4 __attribute__((ext_vector_type(4)));

// LDS writes retired, then the workgroup barrier; the memory clobber keeps the compiler from moving
// LDS accesses across it.  (Not __syncthreads(): its vmcnt(0) would also wait for the weight loads
// and HBM stores in flight.)
__device__ __forceinline__ void pn_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pn_rsrc(const void* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// split x = hi + lo of the 8 values of one granule pair (x3_put8's arithmetic)
__device__ __forceinline__ void pn_split8(const float (&v)[8], u32x4_t& h, u32x4_t& l) {
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
}

// row traffic (IN, the saved activations) with the non-temporal hint when NTS, so these streams
// through L2 evict less of the chain's weights (r03y: 1-2 % faster)
template <bool NTS>
__device__ __forceinline__ u32x4_t pn_ld(const u32x4_t* p) {
  if constexpr (NTS) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NTS>
__device__ __forceinline__ void pn_st(u32x4_t* p, u32x4_t v) {
  if constexpr (NTS)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Weight fragment register sets of pn_gemm (NT <= 4 unit tiles): three, rotating.
#ifndef PN_NS
#define PN_NS 3
#endif
struct PnW {
  pn_h8 ah[PN_NS][4], al[PN_NS][4];
};
// set S <- chunk c of tiles T0 .. T0 + NT - 1 of a fragment-major matrix (pack_frag_major) with nkw
// chunks per row behind rw: lane l's 16 B of each 1 KB block (one VGPR offset for every load; tile,
// chunk and hi / lo ride in the scalar offset)
template <int NT, int S>
__device__ __forceinline__ void pn_ldw(PnW& w, __amdgpu_buffer_rsrc_t rw, int vo, int T0, int nkw, int c) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int so = ((T0 + t) * nkw + c) * 2048;
    w.ah[S][t] = __builtin_bit_cast(pn_h8, __builtin_amdgcn_raw_buffer_load_b128(rw, vo, so, 0));
    w.al[S][t] = __builtin_bit_cast(pn_h8, __builtin_amdgcn_raw_buffer_load_b128(rw, vo, so + 1024, 0));
  }
}
// a product's first two chunks into sets 0 and 1 — issued ahead of pn_gemm, under the previous
// product's epilogue and barriers
template <int NT>
__device__ __forceinline__ void pn_pre(PnW& w, __amdgpu_buffer_rsrc_t rw, int vo, int T0, int nkw, int c0, int nk) {
  pn_ldw<NT, 0>(w, rw, vo, T0, nkw, c0);
  pn_ldw<NT, 1>(w, rw, vo, T0, nkw, c0 + min(1, nk - 1));
}

// acc[t][b] += sum over chunks c < nk of W[tile T0 + t][chunk c0 + c] . act chunk c [rows 16 b + il],
// sets 0 and 1 already holding chunks c0, c0 + 1 (pn_pre).  The weights run two chunks ahead in
// the three sets (the loop unrolled by three, branch-free: loads past the last chunk repeat it), so
// a load has two chunks of MFMAs to arrive from L2.  The B fragments (LDS) of path tile b + 1 are
// read while tile b's MFMAs run.  Rows 16 b + il share x3_swz, so two LDS addresses serve every
// path tile.  Per output the products of k_gemm_x3h in its order: hi.hi, hi.lo, lo.hi per chunk.
template <int NT, int NB>
__device__ __forceinline__ void pn_gemm(pn_f4 (&acc)[NT][NB], PnW& w, __amdgpu_buffer_rsrc_t rw, int vo, int T0, int nkw,
                                        int c0, int nk, const uint32_t* act, int il, int ql) {
  const int sw = x3_swz(il);  // = x3_swz(16 b + il)
  const int oh = il * 32 + 4 * ((2 * ql) ^ sw), ol = il * 32 + 4 * ((2 * ql + 1) ^ sw);
  auto ldw = [&](int c, auto Sc) { pn_ldw<NT, decltype(Sc)::value>(w, rw, vo, T0, nkw, c0 + min(c, nk - 1)); };
  auto mm = [&](int c, auto Sc) {
    constexpr int S = decltype(Sc)::value;
    const uint32_t* s = act + c * PN_SLAB;
    pn_h8 bh[2], bl[2];
    bh[0] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + oh));
    bl[0] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + ol));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b + 1 < NB) {
        bh[(b + 1) & 1] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + oh + 512 * (b + 1)));
        bl[(b + 1) & 1] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + ol + 512 * (b + 1)));
      }
      __builtin_amdgcn_sched_barrier(0);  // (keeps the reads one path tile ahead, not all hoisted)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.ah[S][t], bh[b & 1], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.ah[S][t], bl[b & 1], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.al[S][t], bh[b & 1], acc[t][b], 0, 0, 0);
      }
    }
  };
  constexpr std::integral_constant<int, 0> I0{};
  constexpr std::integral_constant<int, 1> I1{};
  // sched_barrier(0): the scheduler keeps each load group where it is written (left alone it sinks
  // every load next to its first use to shorten live ranges)
  int c = 0;
  if constexpr (PN_NS == 2) {  // one chunk ahead in two sets
#pragma unroll 1
    for (; c + 2 <= nk; c += 2) {
      mm(c, I0);
      __builtin_amdgcn_sched_barrier(0);
      ldw(c + 2, I0);
      __builtin_amdgcn_sched_barrier(0);
      mm(c + 1, I1);
      __builtin_amdgcn_sched_barrier(0);
      ldw(c + 3, I1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c < nk) mm(c, I0);
  } else {  // two chunks ahead in three sets
    constexpr std::integral_constant<int, 2> I2{};
#pragma unroll 1
    for (; c + 3 <= nk; c += 3) {
      ldw(c + 2, I2);
      __builtin_amdgcn_sched_barrier(0);
      mm(c, I0);
      __builtin_amdgcn_sched_barrier(0);
      ldw(c + 3, I0);
      __builtin_amdgcn_sched_barrier(0);
      mm(c + 1, I1);
      __builtin_amdgcn_sched_barrier(0);
      ldw(c + 4, I1);
      __builtin_amdgcn_sched_barrier(0);
      mm(c + 2, I2);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c < nk) mm(c, I0);
    if (c + 1 < nk) mm(c + 1, I1);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int NT, int NB>
__device__ __forceinline__ void pn_zero(pn_f4 (&acc)[NT][NB]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[t][b] = pn_f4{0.f, 0.f, 0.f, 0.f};
}

enum { PN_ELU = 0, PN_DELU = 1 };

// R rows from rows (stride L.stride); grid = ceil(R / 80) blocks.  nopt = NOP / 16 GX unit tiles
// (4 or 8; host-checked), one per wave.
template <bool NTS>
__global__ __launch_bounds__(PN_THREADS, 1) void k_pis_net(NetPisDev pd, float* __restrict__ rows, PisRows L, int R) {
  __shared__ PnLds lds;
  uint32_t* const act = lds.act;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 15, ql = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * PN_BM, mrows = min(PN_BM, R - m0);
  const size_t ld = (size_t)L.stride;
  const int nxk = L.INP / 32 - 2;            // chunks of X (1 .. PN_XC)
  const int nopt = ((pd.nx + 63) & ~63) / 16;  // GX unit tiles
  float* const rbase = rows + (size_t)m0 * ld;
  // above any co-resident wave of another kernel, as the layer-wise GEMMs
  __builtin_amdgcn_s_setprio(2);
  // chunks [c0, c0 + n) of a split row region -> act chunks 0 .. n - 1 (rows past R load the last row)
  auto fill = [&](int reg, int c0, int n, auto NMAX) {  // n <= NMAX chunks
    constexpr int PER = PN_BM * 8, NK = (decltype(NMAX)::value * PER + PN_THREADS - 1) / PN_THREADS;
    u32x4_t v[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int i = tid + k * PN_THREADS, c = i / PER, r = (i >> 3) % PN_BM;
      if (c < n)
        v[k] = pn_ld<NTS>(reinterpret_cast<const u32x4_t*>(
            reinterpret_cast<const uint32_t*>(rbase + (size_t)min(r, mrows - 1) * ld + reg) + 32 * (c0 + c) + 4 * (i & 7)));
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int i = tid + k * PN_THREADS, c = i / PER, r = (i >> 3) % PN_BM;
      if (c < n) *reinterpret_cast<u32x4_t*>(act + c * PN_SLAB + r * 32 + 4 * ((i & 7) ^ x3_swz(r))) = v[k];
    }
  };

  // the 512-wide products: wave wv owns units 64 wv .. 64 wv + 63 (4 unit tiles) of all 80 rows
  pn_f4 acc[4][PN_NB];
  PnW w;
  const int vo = 16 * lane;
  // a fragment-major weight matrix of `rows_` rows and Kp words per row
  auto wsrc = [&](const uint32_t* W, int rows_, int Kp) { return pn_rsrc(W, (size_t)rows_ * Kp * 4); };
  constexpr int KG = 2 * PN_H;  // GX's K: [D_0 | A_{L-1}]
  const __amdgpu_buffer_rsrc_t rg = wsrc(pd.gxnoF, 16 * nopt, KG);
  // the next product's first two weight chunks, issued before the current epilogue
  auto pre_fwd = [&](int l) {
    if (l == 0)
      pn_pre<4>(w, wsrc(pd.nnF[0], PN_H, L.INP), vo, 4 * wv, L.INP / 32, 0, 2 + nxk);
    else
      pn_pre<4>(w, wsrc(pd.nnF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC);
  };
  auto pre_vjp = [&](int l) {  // D_{l-1} = (nnT[l] D_l) * elu'(A_{l-1}); l == L: from X
    if (l == pd.L)
      pn_pre<4>(w, wsrc(pd.nnTF[l], PN_H, 32 * nxk), vo, 4 * wv, nxk, 0, nxk);
    else
      pn_pre<4>(w, wsrc(pd.nnTF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC);
  };
  auto pre_gx = [&](int c0) { pn_pre<1>(w, rg, vo, min(wv, nopt - 1), KG / 32, c0, PN_HC); };

  // epilogue of a 512-wide product, in two halves: values -> split words in registers (and the HBM
  // copy) before the barrier that releases the layer input, the LDS stores after it.  Lane (il, ql)
  // of path tile b holds units 64 wv + 16 t + 4 ql + r of row 16 b + il; unit tiles (2 c, 2 c + 1)
  // form granule pair ql of chunk U = 2 wv + c.
  u32x4_t eh[PN_NB][2], el[PN_NB][2];
  u32x4_t xh[PN_NB][2], xl[PN_NB][2];  // elu' operands of the VJP epilogues
  auto lds_at = [&](int b, int c, int hl) {
    const int m = 16 * b + il;
    return reinterpret_cast<u32x4_t*>(act + (2 * wv + c) * PN_SLAB + m * 32 + 4 * ((2 * ql + hl) ^ x3_swz(m)));
  };
  auto aux_load = [&](int reg) {  // this lane's own granules of a saved activation
#pragma unroll
    for (int b = 0; b < PN_NB; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const u32x4_t* g = reinterpret_cast<const u32x4_t*>(
            reinterpret_cast<const uint32_t*>(rbase + (size_t)min(16 * b + il, mrows - 1) * ld + reg) + 32 * (2 * wv + c) +
            8 * ql);
        xh[b][c] = pn_ld<NTS>(g);
        xl[b][c] = pn_ld<NTS>(g + 1);
      }
  };
  auto epi_values = [&](int kind, float ws, const float* bias, int save_reg) {
#pragma unroll
    for (int b = 0; b < PN_NB; ++b) {
      const int m = 16 * b + il;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int U = 2 * wv + c;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * c][b][r] * ws;
          v[4 + r] = acc[2 * c + 1][b][r] * ws;
        }
        if (kind == PN_ELU) {
          const float4 b0 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql);
          const float4 b1 = *reinterpret_cast<const float4*>(bias + 32 * U + 4 * ql + 16);
          v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
          v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = x3_join(xh[b][c][j >> 1], xl[b][c][j >> 1], j & 1);
            v[j] *= a > 0.f ? 1.0f : a + 1.0f;
          }
        }
        pn_split8(v, eh[b][c], el[b][c]);
        if (save_reg >= 0 && m < mrows) {
          u32x4_t* g = reinterpret_cast<u32x4_t*>(reinterpret_cast<uint32_t*>(rbase + (size_t)m * ld + save_reg) + 32 * U +
                                                  8 * ql);
          pn_st<NTS>(g, eh[b][c]);
          pn_st<NTS>(g + 1, el[b][c]);
        }
      }
    }
  };
  auto epi_store = [&]() {
#pragma unroll
    for (int b = 0; b < PN_NB; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        *lds_at(b, c, 0) = eh[b][c];
        *lds_at(b, c, 1) = el[b][c];
      }
  };

  pre_fwd(0);
  constexpr std::integral_constant<int, 2 + PN_XC> IN_MAX{};
  constexpr std::integral_constant<int, PN_HC> H_MAX{};
  fill(L.IN, 0, 2 + nxk, IN_MAX);  // IN: the time embedding (chunks 0, 1) and X
  pn_barrier();

  // forward
  for (int l = 0; l < pd.L; ++l) {
    pn_zero(acc);
    if (l == 0)
      pn_gemm<4, PN_NB>(acc, w, wsrc(pd.nnF[0], PN_H, L.INP), vo, 4 * wv, L.INP / 32, 0, 2 + nxk, act, il, ql);
    else
      pn_gemm<4, PN_NB>(acc, w, wsrc(pd.nnF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC, act, il, ql);
    if (l + 1 < pd.L)
      pre_fwd(l + 1);
    else
      pre_vjp(pd.L);
    epi_values(PN_ELU, pd.nnW[l], pd.nnbP[l], L.A[l]);
    pn_barrier();  // every wave's reads of the layer input are done
    epi_store();
    pn_barrier();
  }
  // the forward's HBM stores of A_0 .. A_{L-1} complete before any wave reads them back (A_{l-1}
  // by the lane that stored it, A_{L-1} by every wave for GX)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // VJP: D_{L-1} from X (reloaded into act chunks 0 ..) and elu'(A_{L-1}) (HBM)
  for (int l = pd.L; l >= 1; --l) {
    pn_zero(acc);
    if (l == pd.L) {  // (every wave is past the forward's last barrier: act is free)
      fill(L.IN, 2, nxk, IN_MAX);
      pn_barrier();
      pn_gemm<4, PN_NB>(acc, w, wsrc(pd.nnTF[l], PN_H, 32 * nxk), vo, 4 * wv, nxk, 0, nxk, act, il, ql);
    } else {
      pn_gemm<4, PN_NB>(acc, w, wsrc(pd.nnTF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC, act, il, ql);
    }
    // elu'(A_{l-1}), then the next weights (after the values: acc, the elu' operands and two weight
    // sets together would not fit the 256 registers)
    aux_load(L.A[l - 1]);
    epi_values(PN_DELU, pd.nnTW[l], nullptr, -1);
    if (l > 1)
      pre_vjp(l - 1);
    else
      pre_gx(0);
    pn_barrier();
    epi_store();
    pn_barrier();
  }
  // GX = [D_0 | A_{L-1}] . gxno^T + b_L (K = 1,024: D_0 from act, then A_{L-1} reloaded into act);
  // wave wv < nopt takes unit tile wv for all 80 rows
  {
    pn_f4 ag[1][PN_NB];
    pn_zero(ag);
    const bool live = wv < nopt;
    if (live) pn_gemm<1, PN_NB>(ag, w, rg, vo, wv, KG / 32, 0, PN_HC, act, il, ql);
    pre_gx(PN_HC);
    pn_barrier();
    fill(L.A[pd.L - 1], 0, PN_HC, H_MAX);
    pn_barrier();
    if (live) pn_gemm<1, PN_NB>(ag, w, rg, vo, wv, KG / 32, PN_HC, PN_HC, act, il, ql);
    pn_barrier();  // act free: GX's fp32 values go through it (row m: 128 floats)
    float* gx = reinterpret_cast<float*>(act);
    if (live) {
      const float* bias = pd.nnbP[pd.L] + 16 * wv + 4 * ql;
#pragma unroll
      for (int b = 0; b < PN_NB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = ag[0][b][r] * pd.gxnoW;  // k_gemm_x3h's EPI_BIAS arithmetic
          v += bias[r];
          gx[(16 * b + il) * 128 + 16 * wv + 4 * ql + r] = v;
        }
    }
    pn_barrier();
    // row m, chunk U, granule pair q: the values of units 32 U + 4 q + (j & 3) + 16 (j >> 2)
    for (int i = tid; i < PN_BM * (nopt / 2) * 4; i += PN_THREADS) {
      const int q = i & 3, U = (i >> 2) % (nopt / 2), m = (i >> 2) / (nopt / 2);
      if (m >= mrows) continue;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gx[m * 128 + 32 * U + 4 * q + (j & 3) + 16 * (j >> 2)];
      x3_put8(rbase + (size_t)m * ld, L.GX, U, q, v);
    }
  }
}

}  // namespace dpi
