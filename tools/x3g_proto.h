// k_gemm_x3g (prototype, tools/ubench_x3g.hip): the split GEMM of k_gemm_x3h on the same 128 x 128
// block tile (4 waves of 64 x 64, two blocks per CU), with only W through LDS.
//   - W (the A operand, 128 unit rows x 128 B per 32-deep chunk) goes through an LDS-DMA ring of
//     XD + 2 slots of 16 KB, XD + 1 chunks ahead;
//   - each wave's X fragments (its 64 path rows; lane (il, ql) of m-tile b needs the 32 contiguous
//     bytes of granule pair ql of row 16 b + il) are loaded from global straight into registers, XD
//     chunks ahead, in the fragment order the MFMA takes (the split storage's order): no LDS write, no
//     ds_read for X.
// Per CU and chunk that halves the LDS traffic (32 KB of DMA writes + 64 KB of ds_read_b128 instead
// of 64 + 128 KB) and keeps up to XD + 1 chunks of loads in flight instead of one.  The two waves
// (wn = 0, 1) that share an m-row range load the same X bytes; the second is served by the CU's L1.
// The same products per output in the same order as k_gemm_x3h: bitwise equal outputs.
// NEGATIVE RESULT (r03f): 40 % slower than k_gemm_x3h (tools/ubench_x3g.hip header); kept for the
// record, not used by the product.
#pragma once

namespace dpi {

constexpr int X3G_THREADS = 256;

template <int XD>
struct X3GLds {
  static constexpr int WS = XD + 2, SLOT = 128 * 32;
  uint32_t sm[WS * SLOT + 128];  // the W ring, then the block's n-tile of the bias
};

template <int EPI, int XD>
__global__ __launch_bounds__(X3G_THREADS, 2) void k_gemm_x3g(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  // XD = 2 exceeds 256 VGPRs: spill code copies the inline-asm load destinations before the counted
  // wait retires them (wrong results; one GPU fault in r03f)
  static_assert(XD == 1, "X look-ahead: XD = 1 only");
  constexpr int NT = 4, BN = 128, BM = 128, WS = X3GLds<XD>::WS, SLOT = X3GLds<XD>::SLOT, NXS = XD + 1;
  constexpr int NWAVE = X3G_THREADS / 64, PER_WAVE = BN / 8 / NWAVE;  // 4 W DMA wave-instructions per chunk
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ X3GLds<XD> lds;
  uint32_t* sm = lds.sm;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;

  auto issue_w = [&](int c, int slot) {
    uint32_t* dst = sm + slot * SLOT;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int g = (lane & 7) ^ x3_swz(r);
      const uint32_t* src = W + (size_t)(n0 + r) * Kp + 32 * c + 4 * g;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + 256 * w), 16, 0, 0);
    }
  };
  // X fragments by buffer loads in inline asm, so the compiler's wait model (which turns to
  // vmcnt(0) once VGPR loads and LDS-DMA are both outstanding) never sees them: the counted waits
  // below are the only ones, and the fragments pass through them ("+v") before any MFMA reads them.
  // One resource per source; the lane's row offsets in VGPRs (rows past M clamped to row M - 1), the
  // chunk's column offset in the scalar offset.
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  auto rsrc = [&](const float* base, int ld) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    return i32x4{(int)(uint32_t)a, (int)(uint32_t)(a >> 32) & 0xFFFF,
                 (int)min((size_t)M * ld * 4, (size_t)0x7FFFFFFF), 0x00020000};
  };
  const i32x4 rx = rsrc(X, ldx), rx2 = rsrc(X2, ldx2);
  int xoff[4], xoff2[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int row = min(m0 + wm * 64 + 16 * b + il, M - 1);
    xoff[b] = row * ldx * 4 + 32 * ql;
    xoff2[b] = row * ldx2 * 4 + 32 * ql;
  }

  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT];      // W fragments, double-buffered across chunks (LDS)
  u32x4_t xh[NXS][4], xl[NXS][4];  // X fragments, XD + 1 chunks (global -> registers)

  auto load_x = [&](int c, auto Sc) {
    constexpr int S = decltype(Sc)::value;
    const bool one = c < nk1;  // wave-uniform source select (two-source K as in x3_tile)
    const int soff = one ? 128 * c : 128 * (c - nk1);
    const i32x4 r = one ? rx : rx2;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int vo = one ? xoff[b] : xoff2[b];
      u32x4_t h, l;
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(h) : "v"(vo), "s"(r), "s"(soff));
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:16" : "=v"(l) : "v"(vo), "s"(r), "s"(soff));
      xh[S][b] = h;
      xl[S][b] = l;
    }
  };
  auto read_w = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * SLOT;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = wn * 16 * NT + 16 * t + il, s = x3_swz(row);
      const uint32_t* rp = buf + row * 32;
      ah[F][t] = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
      al[F][t] = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
    }
  };
  auto mma = [&](auto Fc, auto Sc) {
    constexpr int F = decltype(Fc)::value, S = decltype(Sc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const h8 bh = __builtin_bit_cast(h8, xh[S][b]), bl = __builtin_bit_cast(h8, xl[S][b]);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh, acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl, acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh, acc[t][b], 0, 0, 0);
      }
    }
  };
  // Counted waits.  Iteration v issues the group G(v) = {X(v + XD): 8 loads, W(v + WS - 1): 4 DMA};
  // iteration u needs X(u) (in G(u - XD)) and W(u + 1) (in G(u + 2 - WS) = G(u - XD)): all but the
  // XD - 1 youngest groups retired.
  // ... and X(u)'s registers pass through the wait.  N: the youngest VMEM operations that may stay
  // outstanding (the body: 12 = one group when XD = 2; the prologue: 8 = X(1))
  auto vm_wait = [&](auto Sc, auto Nc) {
    constexpr int S = decltype(Sc)::value, N = decltype(Nc)::value;
    u32x4_t h0 = xh[S][0], h1 = xh[S][1], h2 = xh[S][2], h3 = xh[S][3];
    u32x4_t l0 = xl[S][0], l1 = xl[S][1], l2 = xl[S][2], l3 = xl[S][3];
#define X3G_TIES "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3)
    if constexpr (N == 0)
      asm volatile("s_waitcnt vmcnt(0)" : X3G_TIES::"memory");
    else if constexpr (N == 8)
      asm volatile("s_waitcnt vmcnt(8)" : X3G_TIES::"memory");
    else
      asm volatile("s_waitcnt vmcnt(12)" : X3G_TIES::"memory");
    xh[S][0] = h0, xh[S][1] = h1, xh[S][2] = h2, xh[S][3] = h3;
    xl[S][0] = l0, xl[S][1] = l1, xl[S][2] = l2, xl[S][3] = l3;
#undef X3G_TIES
  };
  // iteration u: chunk u's W fragments in set F, its X fragments in set S
  auto body = [&](int u, auto Fc, auto Sc) {
    constexpr int F = decltype(Fc)::value, S = decltype(Sc)::value;
    __builtin_amdgcn_sched_barrier(0);  // the previous body's MFMAs stay in front of this wait
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): chunk u's W fragment reads landed
    vm_wait(Sc, std::integral_constant<int, XD == 1 ? 0 : 12>{});
    __builtin_amdgcn_s_barrier();  // W(u + 1) published; chunk u - 1's slot free
    load_x(min(u + XD, nk - 1), std::integral_constant<int, (S + XD) % NXS>{});
    issue_w(min(u + WS - 1, nk - 1), (u + WS - 1) % WS);
    read_w((u + 1) % WS, std::integral_constant<int, F ^ 1>{});
    mma(Fc, Sc);
    // the loads go out first (program order); the 8 fragment reads one per 4 MFMAs
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
  };

  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + WS * SLOT);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  __builtin_amdgcn_s_setprio(2);
  const bool live = m0 + wm * 64 < M;  // wave-uniform: a wave whose rows all lie past M does no MFMAs
  // prologue: W(0 .. WS - 2) and X(0 .. XD - 1) (chunks clamped); wait for W(0), W(1), X(0)
#pragma unroll
  for (int c = 0; c < WS - 1; ++c) issue_w(min(c, nk - 1), c);
  if (live) {
    load_x(0, std::integral_constant<int, 0>{});
    if constexpr (XD == 2) load_x(min(1, nk - 1), std::integral_constant<int, 1>{});
    // W(0), W(1), X(0) landed (X(1) may be outstanding): the body's wait, for set 0
    vm_wait(std::integral_constant<int, 0>{}, std::integral_constant<int, XD == 1 ? 0 : 8>{});
  } else {
    if constexpr (XD == 2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (!live) {  // this wave's DMA share and every barrier, nothing else
    for (int u = 0; u < nk; ++u) {
      if constexpr (XD == 2)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue_w(min(u + WS - 1, nk - 1), (u + WS - 1) % WS);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  read_w(0, std::integral_constant<int, 0>{});
  // the register sets' period L = lcm(2, NXS) bodies: a branch-free main loop (a conditional body
  // would let the compiler sink the X loads of the body before it into its block, next to their
  // MFMAs), then the nk % L remaining bodies
  constexpr int L = XD == 1 ? 2 : 6;
  auto bodies = [&](int u0, auto Jc) {
    constexpr int J = decltype(Jc)::value;
    body(u0 + J, std::integral_constant<int, J % 2>{}, std::integral_constant<int, J % NXS>{});
  };
  int u = 0;
  for (; u + L <= nk; u += L) {
    bodies(u, std::integral_constant<int, 0>{});
    bodies(u, std::integral_constant<int, 1>{});
    if constexpr (L == 6) {
      bodies(u, std::integral_constant<int, 2>{});
      bodies(u, std::integral_constant<int, 3>{});
      bodies(u, std::integral_constant<int, 4>{});
      bodies(u, std::integral_constant<int, 5>{});
    }
  }
  const int rem = nk - u;
  if (rem > 0) bodies(u, std::integral_constant<int, 0>{});
  if constexpr (L == 6) {
    if (rem > 1) bodies(u, std::integral_constant<int, 1>{});
    if (rem > 2) bodies(u, std::integral_constant<int, 2>{});
    if (rem > 3) bodies(u, std::integral_constant<int, 3>{});
    if (rem > 4) bodies(u, std::integral_constant<int, 4>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail loads land before the slots are released
  __builtin_amdgcn_s_waitcnt(0xC07F);

  // epilogue (as k_gemm_x3h): lane (il, ql) of m-tile b holds OUT[m0 + 64 wm + 16 b + il][16 T + 4 ql + r]
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int m = m0 + wm * 64 + 16 * b + il;
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      const int U = (n0 >> 5) + wn * (NT / 2) + c;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * c][b][r] * wscale;
        v[4 + r] = acc[2 * c + 1][b][r] * wscale;
      }
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
        if (has_bias) {
          const float* bsrc = sbias + 32 * (wn * (NT / 2) + c) + 4 * ql;
          const float4 b0 = *reinterpret_cast<const float4*>(bsrc);
          const float4 b1 = *reinterpret_cast<const float4*>(bsrc + 16);
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
