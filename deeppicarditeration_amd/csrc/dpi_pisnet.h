// k_pis_net: the whole split-storage PISGradNet nn_module chain of pis_chain_x3 (solution.py:256-289)
// in ONE launch, 64 rows per block, with the 512-wide activations held in LDS across layers.
//
// pis_chain_x3 runs the chain as 9 k_gemm_x3h launches; between launches every 512-wide activation
// and cotangent makes an HBM round trip (13 GB per HJB label call, profiles/traffic_hjb.json) and
// every launch pays its tiles' prologues and epilogues.  Here a block takes 64 rows through
//   forward   A_l = elu(W_l A_{l-1} + b_l)                       l = 0 .. L-1  (A_{-1} = IN)
//   VJP       D_{L-1} = (nnT[L] X) * elu'(A_{L-1}),  D_{l-1} = (nnT[l] D_l) * elu'(A_{l-1})
//   output    GX = [A_{L-1} | D_0] . [nn[L] | nnT[0]]^T + b_L
// with the current 512-wide operand in a 128 KB LDS image (64 rows x 16 chunks, chunk-major so each
// 32-deep chunk is a 64-row slab laid out like a k_gemm_x3h ring slot) and the x part of IN in a
// 32 KB image: 160 KB, one block (8 waves, 2 per SIMD) per CU.  GX's A_{L-1} half is formed while
// A_{L-1} is the LDS image and its fp32 partial sums wait in the X image; only A_0 .. A_{L-2} (the
// VJP's elu' operands) and GX go to HBM.
//
// Wave w owns units 64 w .. 64 w + 63 of every 512-wide product: its weight rows are private, so the
// MFMA A operands come straight from global (L2-resident: 1 MB per layer shared by every block) into
// registers as buffer loads, one chunk ahead; the B operands (the 64 rows) are the shared LDS image.
// Per chunk and output the same three products in the same order as k_gemm_x3h (hi.hi, hi.lo,
// lo.hi into one accumulator), the same epilogue arithmetic and the same split on store, so every
// row's GX is bitwise equal to the layer-wise chain (tests/test_gpu_parity.py).
#pragma once

namespace dpi {

constexpr int PN_BM = 64, PN_THREADS = 512, PN_SLAB = PN_BM * 32;  // words per 32-deep chunk slab
constexpr int PN_H = 512, PN_HC = PN_H / 32;                       // hidden width and its chunks
constexpr int PN_XC = 4;                                           // chunks of the x part of IN (nx <= 128)

struct PnLds {
  uint32_t act[PN_HC * PN_SLAB];  // 128 KB: the current 512-wide operand
  uint32_t xs[PN_XC * PN_SLAB];   // 32 KB: X = IN[:, 64:]
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

// fragment (hi, lo) of row `row` of a slab, lane group ql (x3_swz-swizzled granules, as k_gemm_x3h)
__device__ __forceinline__ void pn_frag(const uint32_t* slab, int row, int ql, pn_h8& h, pn_h8& l) {
  const int s = x3_swz(row);
  const uint32_t* rp = slab + row * 32;
  h = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
  l = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
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

// Weight fragment register sets of pn_gemm (NT <= 4 unit tiles), rotating: PN_WSETS = 3 keeps the
// weights two chunks ahead, 2 one chunk ahead (32 registers fewer).
#ifndef DPI_PN_WSETS
#define DPI_PN_WSETS 3
#endif
constexpr int PN_WSETS = DPI_PN_WSETS;
static_assert(PN_WSETS == 2 || PN_WSETS == 3, "weight register sets");
struct PnW {
  pn_h8 ah[PN_WSETS][4], al[PN_WSETS][4];
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

// acc[t][b] += sum over chunks c < nk of W[tile T0 + t][chunk c0 + c] . slab(c)[rows p0 + 16 b + il],
// sets 0 and 1 already holding chunks c0, c0 + 1 (pn_pre).  The weights run two chunks ahead in
// the three sets (the loop unrolled by three, branch-free: loads past the last chunk repeat it), so
// a load has two chunks of MFMAs to arrive from L2; the B fragments (LDS) are read per chunk just
// before its MFMAs.  Rows p0 + 16 b + il share x3_swz, so two LDS addresses serve every path tile.
// Per output the products of k_gemm_x3h in its order: hi.hi, hi.lo, lo.hi per chunk.
template <int NT, int NB, class Slab>
__device__ __forceinline__ void pn_gemm(pn_f4 (&acc)[NT][NB], PnW& w, __amdgpu_buffer_rsrc_t rw, int vo, int T0, int nkw,
                                        int c0, int nk, int p0, int il, int ql, Slab slab) {
  const int sw = x3_swz(il);  // = x3_swz(p0 + 16 b + il): p0 % 16 == 0
  const int oh = (p0 + il) * 32 + 4 * ((2 * ql) ^ sw), ol = (p0 + il) * 32 + 4 * ((2 * ql + 1) ^ sw);
  auto ldw = [&](int c, auto Sc) { pn_ldw<NT, decltype(Sc)::value>(w, rw, vo, T0, nkw, c0 + min(c, nk - 1)); };
  // B fragments two path tiles at a time: tile b + 2's pair is read while tile b's MFMAs run
  auto mm = [&](int c, auto Sc) {
    constexpr int S = decltype(Sc)::value;
    const uint32_t* s = slab(c);
    pn_h8 bh[2], bl[2];
    auto ldb = [&](int b) {
      bh[b & 1] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + oh + 512 * b));
      bl[b & 1] = __builtin_bit_cast(pn_h8, *reinterpret_cast<const u32x4_t*>(s + ol + 512 * b));
    };
    ldb(0);
    if (NB > 1) ldb(1);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.ah[S][t], bh[b & 1], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.ah[S][t], bl[b & 1], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.al[S][t], bh[b & 1], acc[t][b], 0, 0, 0);
      }
      if (b + 2 < NB) ldb(b + 2);
    }
  };
  constexpr std::integral_constant<int, 0> I0{};
  constexpr std::integral_constant<int, 1> I1{};
  constexpr std::integral_constant<int, 2> I2{};
  // sched_barrier(0): the scheduler keeps each load group where it is written (left alone it sinks
  // every load next to its first use to shorten live ranges)
  int c = 0;
  if constexpr (PN_WSETS == 3) {
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
  } else {
#pragma unroll 1
    for (; c + 2 <= nk; c += 2) {
      mm(c, I0);
      __builtin_amdgcn_sched_barrier(0);
      if (c + 2 < nk) ldw(c + 2, I0);
      __builtin_amdgcn_sched_barrier(0);
      mm(c + 1, I1);
      __builtin_amdgcn_sched_barrier(0);
      if (c + 3 < nk) ldw(c + 3, I1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c < nk) mm(c, I0);
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

enum { PN_ELU = 0, PN_DELU_LDS = 1, PN_DELU_HBM = 2 };

// Row traffic (IN, the saved activations, GX) goes through a buffer resource based at the block's
// first row and sized to its valid rows: rows past R read as zeros and their stores are dropped, so
// the partial last tile needs no clamped addresses, and every access is one 32-bit lane offset
// (holding the whole row offset: the range check ignores the scalar offset) plus a wave-uniform
// scalar offset for the columns (no 64-bit per-lane pointers held across the layers).  NTM: the
// non-temporal hint (cache policy nt) on the row loads (bit 0), so the row streams through L2 do
// not evict the chain's weights (7 MB, shared by every block of the XCD), and on the row stores
// (bit 1).  Stores without it: a lane's two 16-B stores of a 32-B granule pair merge in L2 before
// write-back; with it they leave as partial-line writes (k_pis_net's HBM writes per HJB label call
// 2.69 GB with, 1.84 GB without, against 1.88 GB of rows written, r04i).
template <int NTM>
__device__ __forceinline__ u32x4_t pn_ld(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, (NTM & 1) ? 2 : 0));
}
template <int NTM>
__device__ __forceinline__ void pn_st(__amdgpu_buffer_rsrc_t r, int vo, int so, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r, vo,
                                         so, (NTM & 2) ? 2 : 0);
}

// R rows from rows (stride L.stride); grid = ceil(R / 64) blocks.  NTM: the non-temporal hints
// (DPI_PIS_NT: 2 = loads only, the default; 1 = loads and stores; 0 = none).  At most 232 registers per wave (VGPRs + AGPRs; the
// 160 KB of LDS leave none for another block): a one-wave k_pis_rollout_shared block of the next
// batch (<= 48 VGPRs, no LDS) fits on every SIMD beside the two k_pis_net waves (2 x 232 + 48 =
// 512).  (On gfx950 amdgpu_num_vgpr(N) caps the unified VGPR + AGPR file at 2 N: 116 -> 232; at 224
// the allocator spilled one to five values whatever the code shape.)
#ifndef DPI_PN_VGPR_HALF
#define DPI_PN_VGPR_HALF 116  // 232 registers
#endif
template <int NTM, int NL>
__global__ __launch_bounds__(PN_THREADS, 1) __attribute__((amdgpu_num_vgpr(DPI_PN_VGPR_HALF))) void k_pis_net(NetPisDev pd,
                                                                                                 float* __restrict__ rows,
                                                                                                 PisRows L, int R) {
  // NL = pd.L hidden layers (host-dispatched): a template parameter, so the layer loops unroll
  __shared__ PnLds lds;
  const int tid = threadIdx.x, lane = tid & 63, il = lane & 15, ql = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * PN_BM, mrows = min(PN_BM, R - m0);
  const int ldb = L.stride * 4;  // row stride in bytes
  const int nxk = L.INP / 32 - 2;  // chunks of X (1 .. PN_XC; host-checked)
  float* const rbase = rows + (size_t)m0 * L.stride;
  const __amdgpu_buffer_rsrc_t rr = pn_rsrc(rbase, (size_t)mrows * ldb);
  // above any co-resident wave of another kernel, as the layer-wise GEMMs
  __builtin_amdgcn_s_setprio(2);
  auto act = [&](int c) -> uint32_t* { return lds.act + c * PN_SLAB; };
  auto xsl = [&](int c) -> uint32_t* { return lds.xs + c * PN_SLAB; };
  // whole row regions: thread tid moves granule tid & 7 of tile row tid >> 3 in each chunk
  const int gr = tid >> 3, gg = tid & 7;
  const int vrow = gr * ldb + 16 * gg;                        // + scalar 4 (reg + 32 c)
  auto gdst = [&](uint32_t* slab) { return reinterpret_cast<u32x4_t*>(slab + gr * 32 + 4 * (gg ^ x3_swz(gr))); };
  // a lane's own granule pairs of the 512-wide regions: row 16 b + il, chunk 2 wv + c, pair ql
  // A buffer instruction's range check covers the VGPR (+ immediate) offset but not the scalar one,
  // so a row past R must be past num_records in the VGPR part alone: with 16 b ldb in the scalar
  // offset, rows 16 b + il >= mrows of a partial tile with il < mrows would pass the check and land
  // past the chunk's rows.  The scalar offset carries only the region and chunk columns (< a row).
  // So path tile b gets a resource of its own, based at its row 16 b and sized to its valid rows
  // (scalar registers only), and the lane offset il ldb + 32 ql is the same for every tile.
  const int vown = il * ldb + 32 * ql;                        // + scalar 4 reg + 128 (2 wv + c)
  auto rown = [&](int b) {
    return pn_rsrc(rbase + (size_t)(16 * b) * L.stride, (size_t)max(0, mrows - 16 * b) * ldb);
  };
  auto sown = [&](int reg, int c) { return 4 * reg + 128 * (2 * wv + c); };

  // the 512-wide products: wave wv owns units 64 wv .. 64 wv + 63 (4 unit tiles) of all 64 rows
  pn_f4 acc[4][4];
  PnW w;
  const int vo = 16 * lane;
  // a fragment-major weight matrix of `rows_` rows and Kp words per row
  auto wsrc = [&](const uint32_t* W, int rows_, int Kp) { return pn_rsrc(W, (size_t)rows_ * Kp * 4); };
  constexpr int KG = 2 * PN_H;                  // GX's K: [D_0 | A_{L-1}]
  const int nopt = ((pd.nx + 63) & ~63) / 16;  // GX unit tiles (4 or 8)
  const __amdgpu_buffer_rsrc_t rg = wsrc(pd.gxnoF, 16 * nopt, KG);
  // the next product's first two weight chunks, issued before the current epilogue
  auto pre_fwd = [&](int l) {
    if (l == 0)
      pn_pre<4>(w, wsrc(pd.nnF[0], PN_H, L.INP), vo, 4 * wv, L.INP / 32, 0, 2 + nxk);
    else
      pn_pre<4>(w, wsrc(pd.nnF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC);
  };
  auto pre_vjp = [&](int l) {  // D_{l-1} = (nnT[l] D_l) * elu'(A_{l-1}); l == L: from X
    if (l == NL)
      pn_pre<4>(w, wsrc(pd.nnTF[l], PN_H, 32 * nxk), vo, 4 * wv, nxk, 0, nxk);
    else
      pn_pre<4>(w, wsrc(pd.nnTF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC);
  };
  auto pre_gx = [&](int c0) { pn_pre<1>(w, rg, vo, min(wv, nopt - 1), KG / 32, c0, PN_HC); };

  // epilogue of a 512-wide product, one (path tile b, chunk c) at a time after the barrier that
  // releases the layer input: values -> split words -> the HBM copy and the LDS image.  Lane (il, ql)
  // of path tile b holds units 64 wv + 16 t + 4 ql + r of row 16 b + il; unit tiles (2 c, 2 c + 1)
  // form granule pair ql of chunk U = 2 wv + c.  xh / xl: elu'(A) operands from HBM (kind
  // PN_DELU_HBM); PN_DELU_LDS reads them from the lane's own granules of the image it overwrites.
  auto lds_at = [&](int b, int c, int hl) {
    const int m = 16 * b + il;
    return reinterpret_cast<u32x4_t*>(act(2 * wv + c) + m * 32 + 4 * ((2 * ql + hl) ^ x3_swz(m)));
  };
  // os: the output's store scale 2^e (PN_ELU), as: the saved activation's read scale 2^-e (PN_DELU_*),
  // the operand exponents of dpi_gemm.h (k_gemm_x3h's oscale / ascale)
  auto epilogue = [&](int kind, float ws, const float* bias, int save_reg, float os, float as,
                      const u32x4_t (&xh)[4][2], const u32x4_t (&xl)[4][2]) {
    const __amdgpu_buffer_rsrc_t rb = pn_rsrc(bias, 4 * PN_H);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int U = 2 * wv + c;
        float v[8];
        if (kind == PN_ELU) {  // k_gemm_x3h's EPI_BIAS_ELU arithmetic: fma(acc, 2^-s, bias), then ELU
          // (a float vector, indexed: clang's __builtin_bit_cast of a vector ELEMENT reads element 0)
          const pn_f4 b0 = __builtin_bit_cast(pn_f4, __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * ql, 128 * U, 0));
          const pn_f4 b1 = __builtin_bit_cast(pn_f4, __builtin_amdgcn_raw_buffer_load_b128(rb, 16 * ql, 128 * U + 64, 0));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = __builtin_fmaf(acc[2 * c][b][r], ws, b0[r]);
            v[4 + r] = __builtin_fmaf(acc[2 * c + 1][b][r], ws, b1[r]);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f) * os;
        } else {  // EPI_DELU: (acc 2^-s) elu'(A)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = __builtin_fmaf(acc[2 * c][b][r], ws, 0.f);
            v[4 + r] = __builtin_fmaf(acc[2 * c + 1][b][r], ws, 0.f);
          }
          u32x4_t ah, al;
          if (kind == PN_DELU_LDS) {
            ah = *lds_at(b, c, 0);
            al = *lds_at(b, c, 1);
          } else {
            ah = xh[b][c];
            al = xl[b][c];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float a = x3_join(ah[j >> 1], al[j >> 1], j & 1);
            v[j] *= a > 0.f ? 1.0f : fmaf(a, as, 1.0f);
          }
        }
        u32x4_t eh, el;
        pn_split8(v, eh, el);
        if (save_reg >= 0) {  // rows past R: dropped by the buffer's range check
          pn_st<NTM>(rown(b), vown, sown(save_reg, c), eh);
          pn_st<NTM>(rown(b), vown, sown(save_reg, c) + 16, el);
        }
        *lds_at(b, c, 0) = eh;
        *lds_at(b, c, 1) = el;
      }
    }
  };
  u32x4_t xh[4][2], xl[4][2];  // elu' operands of the PN_DELU_HBM epilogues

  pre_fwd(0);
  // IN: the time embedding (chunks 0, 1) -> act, X (chunks 2 ..) -> xs
  {
    u32x4_t v[2 + PN_XC];
#pragma unroll
    for (int c = 0; c < 2 + PN_XC; ++c)
      if (c < 2 + nxk) v[c] = pn_ld<NTM>(rr, vrow, 4 * (L.IN + 32 * c));
#pragma unroll
    for (int c = 0; c < 2 + PN_XC; ++c)
      if (c < 2 + nxk) *gdst(c < 2 ? act(c) : xsl(c - 2)) = v[c];
  }
  pn_barrier();

  // forward
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    pn_zero(acc);
    if (l == 0)
      pn_gemm<4, 4>(acc, w, wsrc(pd.nnF[0], PN_H, L.INP), vo, 4 * wv, L.INP / 32, 0, 2 + nxk, 0, il, ql,
                    [&](int c) { return c < 2 ? act(c) : xsl(c - 2); });
    else
      pn_gemm<4, 4>(acc, w, wsrc(pd.nnF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC, 0, il, ql, act);
    if (l + 1 < NL)
      pre_fwd(l + 1);
    else
      pre_vjp(NL);
    pn_barrier();  // every wave's reads of the layer input are done
    // A_{L-1} stays in LDS only: GX's A_{L-1} half is formed below and elu'(A_{L-1}) read from the image
    epilogue(PN_ELU, pd.nnW[l], pd.nnbP[l], l + 1 < NL ? L.A[l] : -1, pd.nnO[l], 1.0f, xh, xl);
    pn_barrier();
  }
  // VJP: D_{L-1} from X (xs) and elu'(A_{L-1}) (act: each wave reads and overwrites only its own
  // granules).  Between its product and its epilogue, while act still holds A_{L-1}, GX's A_{L-1}
  // half (chunks 0 .. 15 of K): wave wv < nopt takes unit tile wv of all 64 rows, and its fp32
  // partial sums wait in the X image (free once every wave's product has read X) at the words the
  // same lane later writes GX to, so the accumulation order is the layer-wise GEMM's [A_{L-1} | D_0]
  // and nothing leaves the CU.
  float* const gxs = reinterpret_cast<float*>(lds.xs);  // row m: 128 fp32
  {
    pn_zero(acc);
    pn_gemm<4, 4>(acc, w, wsrc(pd.nnTF[NL], PN_H, 32 * nxk), vo, 4 * wv, nxk, 0, nxk, 0, il, ql, xsl);
    pre_gx(0);
    pn_f4 ag[1][4];
    pn_zero(ag);
    if (wv < nopt) pn_gemm<1, 4>(ag, w, rg, vo, wv, KG / 32, 0, PN_HC, 0, il, ql, act);
    // the forward's HBM stores of A_0 .. A_{L-2} complete (each read back below by the lane that
    // stored it)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (NL > 1)
      pre_vjp(NL - 1);
    else
      pre_gx(PN_HC);
    pn_barrier();  // every wave is done with X and with all of A_{L-1}
    if (wv < nopt)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        *reinterpret_cast<pn_f4*>(gxs + (16 * b + il) * 128 + 16 * wv + 4 * ql) = ag[0][b];
    epilogue(PN_DELU_LDS, pd.nnTW[NL], nullptr, -1, 1.0f, pd.nnA[NL - 1], xh, xl);
    pn_barrier();
  }
#pragma unroll
  for (int l = NL - 1; l >= 1; --l) {
    pn_zero(acc);
    pn_gemm<4, 4>(acc, w, wsrc(pd.nnTF[l], PN_H, PN_H), vo, 4 * wv, PN_HC, 0, PN_HC, 0, il, ql, act);
    // elu'(A_{l-1}): this lane's own HBM copy, issued before the next weights
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        xh[b][c] = pn_ld<NTM>(rown(b), vown, sown(L.A[l - 1], c));
        xl[b][c] = pn_ld<NTM>(rown(b), vown, sown(L.A[l - 1], c) + 16);
      }
    if (l > 1)
      pre_vjp(l - 1);
    else
      pre_gx(PN_HC);
    pn_barrier();
    epilogue(PN_DELU_HBM, pd.nnTW[l], nullptr, -1, 1.0f, pd.nnA[l - 1], xh, xl);
    pn_barrier();
  }
  // GX = [A_{L-1} | D_0] . gxno^T + b_L (K = 1,024): the A_{L-1} half's partial sums back from the
  // X image, then the D_0 half from act.  Wave wv < nopt takes unit tile wv for all 64 rows, so each
  // weight fragment is read once per block; the two tiles of a granule pair then meet in the X image
  // (free since D_{L-1}) as fp32.
  {
    // the lane's (il, ql) again from the hardware lane count: keeping them live across the whole
    // chain cost the register allocator a spill at the 224-register cap
    int lid;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
    const int il = lid & 15, ql = lid >> 4;
    const bool live = wv < nopt;
    float* gx = gxs;
    if (live) {
      pn_f4 ag[1][4];
#pragma unroll
      for (int b = 0; b < 4; ++b) ag[0][b] = *reinterpret_cast<const pn_f4*>(gx + (16 * b + il) * 128 + 16 * wv + 4 * ql);
      pn_gemm<1, 4>(ag, w, rg, vo, wv, KG / 32, PN_HC, PN_HC, 0, il, ql, act);
      const float* bias = pd.nnbP[NL] + 16 * wv + 4 * ql;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = __builtin_fmaf(ag[0][b][r], pd.gxnoW, bias[r]);  // k_gemm_x3h's EPI_BIAS arithmetic
          gx[(16 * b + il) * 128 + 16 * wv + 4 * ql + r] = v;
        }
    }
    pn_barrier();
    // row m, chunk U, granule pair q: units 32 U + 4 q + (j & 3) + 16 (j >> 2)
    const int nu = nopt / 2;
    for (int i = tid; i < PN_BM * nu * 4; i += PN_THREADS) {
      const int q = i & 3, U = (i >> 2) % nu, m = (i >> 2) / nu;
      if (m >= mrows) continue;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gx[m * 128 + 32 * U + 4 * q + (j & 3) + 16 * (j >> 2)];
      x3_put8(rbase + (size_t)m * L.stride, L.GX, U, q, v);
    }
  }
}

}  // namespace dpi
