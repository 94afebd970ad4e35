// k_gemm_x3q (prototype, tools/ubench_x3h.hip): k_gemm_x3h with split rings — the X tile (paths,
// streamed from HBM on first touch) through a 3-slot LDS-DMA ring, two chunks ahead, the W tile
// (L2-hot weights) through a 2-slot ring, one chunk ahead: 5 x 16 KB = 80 KB per block, so two
// blocks still share a CU (160 KB).  The n-tile's bias comes from global memory in the epilogue
// (no LDS left for it).  Same products per output in the same order: bitwise equal to k_gemm_x3h.
#pragma once

namespace dpi {

template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3q(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  constexpr int NT = 4, BN = 128, BM = X3H_BM, SLOT = 128 * 32, NWAVE = X3H_THREADS / 64;
  constexpr int PW = BN / 8 / NWAVE;  // 4 DMA wave-instructions per tile and chunk
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ uint32_t sm[5 * SLOT];  // W slots 0, 1; X slots 2, 3, 4
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int mrows = min(BM, M - m0);
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(W + (size_t)n0 * Kp, (size_t)BN * Kp * 4);
  const __amdgpu_buffer_rsrc_t rx = tile_rsrc(X + (size_t)m0 * ldx, (size_t)mrows * ldx * 4);
  const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc(X2 + (size_t)m0 * ldx2, (size_t)mrows * ldx2 * 4);
  // wave-instruction k of a tile fills its rows 8w..8w+7, w = 4k + wave
  int vw[PW], vx[PW], vx2[PW];
#pragma unroll
  for (int k = 0; k < PW; ++k) {
    const int w = k * NWAVE + wv;
    const int r = 8 * w + (lane >> 3);
    const int g = (lane & 7) ^ x3_swz(r);
    vw[k] = r * Kp * 4 + 16 * g;
    const int xr = min(r, mrows - 1);
    vx[k] = xr * ldx * 4 + 16 * g;
    vx2[k] = xr * ldx2 * 4 + 16 * g;
  }
  auto issue_w = [&](int c) {
    uint32_t* dst = sm + (c & 1) * SLOT;
#pragma unroll
    for (int k = 0; k < PW; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu)), 16, vw[k], 128 * c, 0, 0);
  };
  auto issue_x = [&](int c) {
    uint32_t* dst = sm + (2 + c % 3) * SLOT;
    const bool one = c < nk1;
    const int sx = one ? 128 * c : 128 * (c - nk1);
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      __attribute__((address_space(3))) void* d = (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (one)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx[k], sx, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx2, d, 16, vx2[k], sx, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int c, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* wb = sm + (c & 1) * SLOT;
    const uint32_t* xb = sm + (2 + c % 3) * SLOT;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(wb, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(xb, wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  // Iteration v issues the group G(v) = [W(v + 2) if it exists, X(v + 3) if it exists] into the
  // slots chunk v leaves (its fragments were read during iteration v - 1).  Iteration u needs
  // W(u + 1) (first half of G(u - 1)) and X(u + 1) (in G(u - 2)): all but this wave's X(u + 2)
  // pieces retired — vmcnt(4) while G(u - 1) holds an X chunk (u + 2 < nk), vmcnt(0) after.
  auto vm_wait = [&](int u) {
    if (u + 2 < nk)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto issue_group = [&](int v) {
    if (v + 2 < nk) issue_w(v + 2);
    if (v + 3 < nk) issue_x(v + 3);
  };
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    vm_wait(u);
    __builtin_amdgcn_s_barrier();
    issue_group(u);
    load(u + 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  __builtin_amdgcn_s_setprio(2);
  // prologue: [W(0) X(0)] [W(1) X(1)] [X(2)]; chunk 0 and 1 landed, X(2) may be outstanding
  issue_w(0);
  issue_x(0);
  if (nk > 1) {
    issue_w(1);
    issue_x(1);
  }
  if (nk > 2) {
    issue_x(2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {  // rows past M: DMA share and barriers only
    for (int u = 0; u + 1 < nk; ++u) {
      vm_wait(u);
      __builtin_amdgcn_s_barrier();
      issue_group(u);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
          const float* bsrc = bias + 32 * U + 4 * ql;
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

// k_gemm_x3hs: the product k_gemm_x3h with s_memtime stamps per wave (diagnostic only): entry,
// after the prologue, after the main loop, exit; cycles spent in the per-chunk wait + barrier.
template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3hs(unsigned long long* __restrict__ stamps, int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  constexpr int NT = 4, BN = 128, BM = X3H_BM, STAGE = X3HLds::STAGE, NWAVE = X3H_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;  // 8 DMA wave-instructions per chunk
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ X3HLds lds;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long twait = 0;
  uint32_t* sm = lds.sm;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  // LDS-DMA in buffer form (r03f): the wave id made provably uniform, so each DMA's LDS destination
  // is scalar (m0 from SALU alone), and each lane's row offset fixed in a VGPR with the chunk's
  // column offset in soffset — no per-DMA VALU address arithmetic or readfirstlane.  Bitwise equal;
  // 567-573 -> 528-536 us (ELU), 600-609 -> 579-592 us (DELU) at 262,144 x 512 x 512
  // (profiles/r03f_ubench_x3hb.txt).  The resources start at the block's own tiles (W rows n0..,
  // X rows m0..), so the 32-bit offsets stay small whatever the row stride of the activation
  // workspace (thousands of words: the whole chain's row) or M.
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int mrows = min(BM, M - m0);  // >= 1: the grid holds only tiles with rows
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(W + (size_t)n0 * Kp, (size_t)BN * Kp * 4);
  const __amdgpu_buffer_rsrc_t rx = tile_rsrc(X + (size_t)m0 * ldx, (size_t)mrows * ldx * 4);
  const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc(X2 + (size_t)m0 * ldx2, (size_t)mrows * ldx2 * 4);
  // wave-instruction k fills rows 8w..8w+7, w = 4k + wave: k < 4 the W tile, k >= 4 the X tile
  int vw[PER_WAVE / 2], vx[PER_WAVE / 2], vx2[PER_WAVE / 2];
#pragma unroll
  for (int k = 0; k < PER_WAVE; ++k) {
    const int w = k * NWAVE + wv;
    const int r = 8 * w + (lane >> 3);
    const int g = (lane & 7) ^ x3_swz(r);
    if (k < PER_WAVE / 2) {
      vw[k] = r * Kp * 4 + 16 * g;
    } else {
      const int xr = min(r - BN, mrows - 1);  // rows past M load the last row
      vx[k - PER_WAVE / 2] = xr * ldx * 4 + 16 * g;
      vx2[k - PER_WAVE / 2] = xr * ldx2 * 4 + 16 * g;
    }
  }
  auto issue = [&](int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;  // two-source K as in x3_tile
    const int sx = one ? 128 * c : 128 * (c - nk1);
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      __attribute__((address_space(3))) void* d =
          (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (k < PER_WAVE / 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, d, 16, vw[k], 128 * c, 0, 0);
      else if (one)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx[k - PER_WAVE / 2], sx, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx2, d, 16, vx2[k - PER_WAVE / 2], sx, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  unsigned long long tvm = 0;
  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * STAGE;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(buf, BN + wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  // iteration u (u + 1 < nk): chunk u in set F; the DMA of chunk u + 1 (issued one iteration ago) is
  // this wave's only outstanding one; chunk u + 2 goes into chunk u's slot
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const unsigned long long ta = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long tb = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_barrier();
    twait += __builtin_amdgcn_s_memtime() - ta;
    tvm += tb - ta;
    if (u + 2 < nk) issue(u + 2, u & 1);
    load((u + 1) & 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + 2 * STAGE);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  __builtin_amdgcn_s_setprio(2);
  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {  // rows past M: DMA share and barriers only
    for (int u = 0; u + 1 < nk; ++u) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (u + 2 < nk) issue(u + 2, u & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
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
  const unsigned long long t3 = __builtin_amdgcn_s_memtime();
  const unsigned long long r3 = __builtin_amdgcn_s_memrealtime();
  unsigned hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  if (lane == 0) {
    unsigned long long* o = stamps + ((size_t)blockIdx.x * 4 + wv) * 8;
    o[0] = t0; o[1] = t1; o[2] = t2; o[3] = t3; o[4] = twait; o[5] = tvm; o[6] = hwid; o[7] = r3 - r0;
  }
}

// the split of x3_put8 into registers: granule pair (hi, lo) of the 8 values
__device__ __forceinline__ void x3_split8(const float (&v)[8], u32x4_t& h, u32x4_t& l) {
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

// k_gemm_x3e: the product k_gemm_x3h with the epilogue's stores staged through LDS (see below).
template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3e(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  constexpr int NT = 4, BN = 128, BM = X3H_BM, STAGE = X3HLds::STAGE, NWAVE = X3H_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;  // 8 DMA wave-instructions per chunk
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ X3HLds lds;
  uint32_t* sm = lds.sm;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  // LDS-DMA in buffer form (r03f): the wave id made provably uniform, so each DMA's LDS destination
  // is scalar (m0 from SALU alone), and each lane's row offset fixed in a VGPR with the chunk's
  // column offset in soffset — no per-DMA VALU address arithmetic or readfirstlane.  Bitwise equal;
  // 567-573 -> 528-536 us (ELU), 600-609 -> 579-592 us (DELU) at 262,144 x 512 x 512
  // (profiles/r03f_ubench_x3hb.txt).  The resources start at the block's own tiles (W rows n0..,
  // X rows m0..), so the 32-bit offsets stay small whatever the row stride of the activation
  // workspace (thousands of words: the whole chain's row) or M.
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int mrows = min(BM, M - m0);  // >= 1: the grid holds only tiles with rows
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(W + (size_t)n0 * Kp, (size_t)BN * Kp * 4);
  const __amdgpu_buffer_rsrc_t rx = tile_rsrc(X + (size_t)m0 * ldx, (size_t)mrows * ldx * 4);
  const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc(X2 + (size_t)m0 * ldx2, (size_t)mrows * ldx2 * 4);
  // wave-instruction k fills rows 8w..8w+7, w = 4k + wave: k < 4 the W tile, k >= 4 the X tile
  int vw[PER_WAVE / 2], vx[PER_WAVE / 2], vx2[PER_WAVE / 2];
#pragma unroll
  for (int k = 0; k < PER_WAVE; ++k) {
    const int w = k * NWAVE + wv;
    const int r = 8 * w + (lane >> 3);
    const int g = (lane & 7) ^ x3_swz(r);
    if (k < PER_WAVE / 2) {
      vw[k] = r * Kp * 4 + 16 * g;
    } else {
      const int xr = min(r - BN, mrows - 1);  // rows past M load the last row
      vx[k - PER_WAVE / 2] = xr * ldx * 4 + 16 * g;
      vx2[k - PER_WAVE / 2] = xr * ldx2 * 4 + 16 * g;
    }
  }
  auto issue = [&](int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;  // two-source K as in x3_tile
    const int sx = one ? 128 * c : 128 * (c - nk1);
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      __attribute__((address_space(3))) void* d =
          (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (k < PER_WAVE / 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, d, 16, vw[k], 128 * c, 0, 0);
      else if (one)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx[k - PER_WAVE / 2], sx, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx2, d, 16, vx2[k - PER_WAVE / 2], sx, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  f4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * STAGE;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(buf, BN + wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  // iteration u (u + 1 < nk): chunk u in set F; the DMA of chunk u + 1 (issued one iteration ago) is
  // this wave's only outstanding one; chunk u + 2 goes into chunk u's slot
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + 2 < nk) issue(u + 2, u & 1);
    load((u + 1) & 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + 2 * STAGE);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  __builtin_amdgcn_s_setprio(2);
  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {  // rows past M: DMA share and barriers only
    for (int u = 0; u + 1 < nk; ++u) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (u + 2 < nk) issue(u + 2, u & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // epilogue through LDS: the slot chunk nk - 2 used (free: every wave retired its reads of it before
  // the last loop barrier; for nk = 1 never written) takes each wave's outputs, 32 rows x 256 B per
  // pass (8 KB per wave), granules XOR-swizzled by row; then every store instruction writes 4 rows x
  // 256 contiguous bytes (16 lanes per row) instead of 16 rows x 4 scattered 16-B pieces.
  uint32_t* stg = sm + (nk & 1) * STAGE + wv * 2048;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int b = 2 * pass + bb;
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        const int m = m0 + wm * 64 + 16 * b + il;
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
          x3_get8(AUX + (size_t)min(m, M - 1) * ldaux, 0, U, ql, a);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= a[j] > 0.f ? 1.0f : a[j] + 1.0f;
        }
        const int rho = 16 * bb + il, gh = 8 * c + 2 * ql;
        u32x4_t* rowp = reinterpret_cast<u32x4_t*>(stg + rho * 64);
        x3_split8(v, rowp[gh ^ (rho & 15)], rowp[(gh + 1) ^ (rho & 15)]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rho = 4 * j + (lane >> 4), gg = lane & 15;
      const int m = m0 + wm * 64 + 32 * pass + rho;
      const u32x4_t val = reinterpret_cast<const u32x4_t*>(stg + rho * 64)[gg ^ (rho & 15)];
      if (m < M)
        *reinterpret_cast<u32x4_t*>(reinterpret_cast<uint32_t*>(OUT + (size_t)m * ldc) + 32 * ((n0 >> 5) + wn * (NT / 2)) +
                                    4 * gg) = val;
    }
  }
}

}  // namespace dpi

namespace dpi {
// k_gemm_x3t: k_gemm_x3h on v_mfma_f32_32x32x16_f16 — twice the MACs per instruction at the same 8
// cycles of held issue, so the partner wave's VALU / DMA / ds_read issue gets 3 of every 4 cycles
// instead of 1 of 2.  Same 128 x 128 tile, 4 waves of 64 x 64 (2 x 2 tiles of 32 x 32), same
// buffer-form LDS-DMA ring; the LDS image is swizzled for this kernel's fragment reads (lane l reads
// row l % 32, granule pair 2 s + l / 32 for k-step s): granule g of row r sits at g ^ ((r >> 1) & 7),
// which gives each ds_read_b128 lane group 16 distinct (row parity, 16-B slot) pairs.  Output lane l,
// register r of tile (N, Mt): path m = 32 Mt + l % 32, unit 32 N + 8 (r / 4) + 4 (l / 32) + r % 4 —
// granule pairs q = l / 32 (r = 0-3, 8-11) and q = 2 + l / 32 (r = 4-7, 12-15) of one row, whole.
// Not bitwise equal to the 16x16x32 chain (16-deep partial products).
__device__ __forceinline__ int x3t_swz(int r) { return (r >> 1) & 7; }

template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3t(int M, int Kp, int n_ntiles, const uint32_t* __restrict__ W,
                                                             float wscale, const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  constexpr int BN = 128, BM = X3H_BM, STAGE = X3HLds::STAGE, NWAVE = X3H_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f16v __attribute__((ext_vector_type(16)));
  __shared__ X3HLds lds;
  uint32_t* sm = lds.sm;
  const int tile = x3_tile_of_block(), mt = tile / n_ntiles, ntl = tile - mt * n_ntiles;
  const int m0 = mt * BM, n0 = ntl * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int i32 = lane & 31, g2 = lane >> 5;
  const int nk = Kp >> 5;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int mrows = min(BM, M - m0);
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = tile_rsrc(W + (size_t)n0 * Kp, (size_t)BN * Kp * 4);
  const __amdgpu_buffer_rsrc_t rx = tile_rsrc(X + (size_t)m0 * ldx, (size_t)mrows * ldx * 4);
  const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc(X2 + (size_t)m0 * ldx2, (size_t)mrows * ldx2 * 4);
  int vw[PER_WAVE / 2], vx[PER_WAVE / 2], vx2[PER_WAVE / 2];
#pragma unroll
  for (int k = 0; k < PER_WAVE; ++k) {
    const int w = k * NWAVE + wv;
    const int r = 8 * w + (lane >> 3);
    const int g = (lane & 7) ^ x3t_swz(r);
    if (k < PER_WAVE / 2) {
      vw[k] = r * Kp * 4 + 16 * g;
    } else {
      const int xr = min(r - BN, mrows - 1);
      vx[k - PER_WAVE / 2] = xr * ldx * 4 + 16 * g;
      vx2[k - PER_WAVE / 2] = xr * ldx2 * 4 + 16 * g;
    }
  }
  auto issue = [&](int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;
    const int sx = one ? 128 * c : 128 * (c - nk1);
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      __attribute__((address_space(3))) void* d =
          (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (k < PER_WAVE / 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, d, 16, vw[k], 128 * c, 0, 0);
      else if (one)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, d, 16, vx[k - PER_WAVE / 2], sx, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx2, d, 16, vx2[k - PER_WAVE / 2], sx, 0, 0);
    }
  };
  // fragment of LDS row `row`, k-step s: granule pair q = 2 s + l / 32 (hi granule 2q, lo 2q + 1)
  auto frag = [&](const uint32_t* buf, int row, int s, h8& h, h8& l) {
    const int sw = x3t_swz(row), q = 2 * s + g2;
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * q) ^ sw)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * q + 1) ^ sw)));
  };
  f16v acc[2][2];  // [N][Mt]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  h8 ah[2][2][2], al[2][2][2], bh[2][2][2], bl[2][2][2];  // [set][tile][k-step]
  auto load = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int t = 0; t < 2; ++t) frag(buf, wn * 64 + 32 * t + i32, s, ah[F][t][s], al[F][t][s]);
#pragma unroll
      for (int t = 0; t < 2; ++t) frag(buf, BN + wm * 64 + 32 * t + i32, s, bh[F][t][s], bl[F][t][s]);
    }
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[F][a][s], bh[F][b][s], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[F][a][s], bl[F][b][s], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[F][a][s], bh[F][b][s], acc[a][b], 0, 0, 0);
        }
  };
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + 2 < nk) issue(u + 2, u & 1);
    load((u + 1) & 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // 16 ds_reads among 24 MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  float* sbias = reinterpret_cast<float*>(sm + 2 * STAGE);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
  __builtin_amdgcn_s_setprio(2);
  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(sbias + 4 * tid) = bv;
  __builtin_amdgcn_s_barrier();
  if (m0 + wm * 64 >= M) {
    for (int u = 0; u + 1 < nk; ++u) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (u + 2 < nk) issue(u + 2, u & 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  load(0, std::integral_constant<int, 0>{});
  int u = 0;
  for (; u + 2 < nk; u += 2) {
    body(u, std::integral_constant<int, 0>{});
    body(u + 1, std::integral_constant<int, 1>{});
  }
  if (u + 1 < nk) {
    body(u, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 1>{});
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    mma(std::integral_constant<int, 0>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // epilogue: tile (a, b) lane l holds OUT[m0 + 64 wm + 32 b + l % 32][n0 + 64 wn + 32 a + col(r)]
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int m = m0 + wm * 64 + 32 * b + i32;
    if (m >= M) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int U = (n0 >> 5) + wn * 2 + a;
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // granule pair q = 2 h + l / 32: registers 4h..4h+3 and 8+4h..8+4h+3
        const int q = 2 * h + g2;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[a][b][4 * h + r] * wscale;
          v[4 + r] = acc[a][b][8 + 4 * h + r] * wscale;
        }
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
          if (has_bias) {
            const float* bsrc = sbias + 32 * (wn * 2 + a) + 4 * q;
            const float4 b0 = *reinterpret_cast<const float4*>(bsrc);
            const float4 b1 = *reinterpret_cast<const float4*>(bsrc + 16);
            v[0] += b0.x, v[1] += b0.y, v[2] += b0.z, v[3] += b0.w;
            v[4] += b1.x, v[5] += b1.y, v[6] += b1.z, v[7] += b1.w;
          }
          if (EPI == EPI_BIAS_ELU)
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : __expf(v[j]) - 1.0f;
        } else {
          float av[8];
          x3_get8(AUX + (size_t)m * ldaux, 0, U, q, av);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= av[j] > 0.f ? 1.0f : av[j] + 1.0f;
        }
        x3_put8(OUT + (size_t)m * ldc, 0, U, q, v);
      }
    }
  }
}
}  // namespace dpi

namespace dpi {
// k_gemm_x3p: persistent k_gemm_x3h.  Two blocks per CU walk the tiles (virtual block v = b + k nb
// takes the tile x3_tile_of_block would give block v of an ntiles-wide grid, so a block stays on
// its XCD's tile range); between two tiles the next tile's chunks 0 and 1 are DMA'd into the ring
// (both slots are free once every wave has read the last chunk) before the current tile's epilogue,
// so the next tile's first wait is covered by the epilogue.  The bias double-buffers in LDS.  Waves
// whose rows lie past M compute on the clamped last row (their stores are masked), so every wave
// runs the same instruction stream and barriers.  Same products per output in the same order as
// k_gemm_x3h: bitwise equal.
// per-tile DMA state of k_gemm_x3p: the tile's base pointers and byte counts, the lane's offsets
struct X3pTileDma {
  const uint32_t* wb;
  const float *xb, *x2b;
  int xbytes, x2bytes;
  int vw[4], vx[4], vx2[4];
};
__device__ __forceinline__ int x3p_tile(int v, int ntiles) {
  const int xcd = v & 7, loc = v >> 3, q8 = ntiles >> 3;
  return loc < q8 ? xcd * q8 + loc : 8 * q8 + xcd;
}

template <int EPI>
__global__ __launch_bounds__(X3H_THREADS, 2) void k_gemm_x3p(int M, int Kp, int n_ntiles, int ntiles,
                                                             const uint32_t* __restrict__ W, float wscale,
                                                             const float* __restrict__ X, int ldx,
                                                             const float* __restrict__ X2, int ldx2, int nk1,
                                                             float* __restrict__ OUT, int ldc,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ AUX, int ldaux) {
  constexpr int NT = 4, BN = 128, BM = X3H_BM, STAGE = X3HLds::STAGE, NWAVE = X3H_THREADS / 64;
  constexpr int PER_WAVE = (BN + BM) / 8 / NWAVE;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f4v __attribute__((ext_vector_type(4)));
  __shared__ uint32_t sm[2 * STAGE + 2 * BN];  // the ring, then two bias slots
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wm = wv >> 1, wn = wv & 1;
  const int il = lane & 15, ql = lane >> 4;
  const int nk = Kp >> 5;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int nb = gridDim.x;
  auto tile_rsrc = [](const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  // per-tile DMA state: resources based at the tile, lane offsets (rows clamped to the tile's rows)
  auto setup = [&](int t, X3pTileDma& d) {
    const int mt = t / n_ntiles, m0 = mt * BM, n0 = (t - mt * n_ntiles) * BN;
    const int mrows = min(BM, M - m0);
    d.wb = W + (size_t)n0 * Kp;
    d.xb = X + (size_t)m0 * ldx;
    d.x2b = X2 + (size_t)m0 * ldx2;
    d.xbytes = mrows * ldx * 4;
    d.x2bytes = mrows * ldx2 * 4;
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      const int w = k * NWAVE + wv;
      const int r = 8 * w + (lane >> 3);
      const int g = (lane & 7) ^ x3_swz(r);
      if (k < PER_WAVE / 2) {
        d.vw[k] = r * Kp * 4 + 16 * g;
      } else {
        const int xr = min(r - BN, mrows - 1);
        d.vx[k - PER_WAVE / 2] = xr * ldx * 4 + 16 * g;
        d.vx2[k - PER_WAVE / 2] = xr * ldx2 * 4 + 16 * g;
      }
    }
  };
  auto issue = [&](const X3pTileDma& d, int c, int slot) {
    uint32_t* dst = sm + slot * STAGE;
    const bool one = c < nk1;
    const int sx = one ? 128 * c : 128 * (c - nk1);
    const __amdgpu_buffer_rsrc_t rw = tile_rsrc(d.wb, (size_t)BN * Kp * 4);
    const __amdgpu_buffer_rsrc_t rx = one ? tile_rsrc(d.xb, d.xbytes) : tile_rsrc(d.x2b, d.x2bytes);
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
      __attribute__((address_space(3))) void* p =
          (__attribute__((address_space(3))) void*)(dst + 256 * (k * NWAVE + wvu));
      if (k < PER_WAVE / 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, p, 16, d.vw[k], 128 * c, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, p, 16, one ? d.vx[k - PER_WAVE / 2] : d.vx2[k - PER_WAVE / 2],
                                                 sx, 0, 0);
    }
  };
  auto frag = [&](const uint32_t* buf, int row, h8& h, h8& l) {
    const int s = x3_swz(row);
    const uint32_t* rp = buf + row * 32;
    h = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql) ^ s)));
    l = __builtin_bit_cast(h8, *reinterpret_cast<const u32x4_t*>(rp + 4 * ((2 * ql + 1) ^ s)));
  };
  f4v acc[NT][4];
  h8 ah[2][NT], al[2][NT], bh[2][4], bl[2][4];
  auto load = [&](int slot, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    const uint32_t* buf = sm + slot * STAGE;
#pragma unroll
    for (int t = 0; t < NT; ++t) frag(buf, wn * 16 * NT + 16 * t + il, ah[F][t], al[F][t]);
#pragma unroll
    for (int b = 0; b < 4; ++b) frag(buf, BN + wm * 64 + 16 * b + il, bh[F][b], bl[F][b]);
  };
  auto mma = [&](auto Fc) {
    constexpr int F = decltype(Fc)::value;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bh[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[F][t], bl[F][b], acc[t][b], 0, 0, 0);
        acc[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[F][t], bh[F][b], acc[t][b], 0, 0, 0);
      }
  };
  X3pTileDma cur;
  auto body = [&](int u, auto Fc) {
    constexpr int F = decltype(Fc)::value;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + 2 < nk) issue(cur, u + 2, u & 1);
    load((u + 1) & 1, std::integral_constant<int, F ^ 1>{});
    mma(Fc);
    constexpr int NRD = 2 * (NT + 4), NMF = 3 * NT * 4;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMF / NRD, 0);
    }
  };
  const bool has_bias = (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) && bias != nullptr;
  __builtin_amdgcn_s_setprio(2);
  int v = blockIdx.x;
  if (v >= ntiles) return;  // (the host launches at most ntiles blocks)
  int tile = x3p_tile(v, ntiles);
  setup(tile, cur);
  // first tile's prologue: bias slot 0, chunks 0 and 1
  {
    const int n0 = (tile % n_ntiles) * BN;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (has_bias && tid < BN / 4) bv = *reinterpret_cast<const float4*>(bias + n0 + 4 * tid);
    issue(cur, 0, 0);
    if (nk > 1) issue(cur, 1, 1);
    if (has_bias && tid < BN / 4) *reinterpret_cast<float4*>(reinterpret_cast<float*>(sm + 2 * STAGE) + 4 * tid) = bv;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  for (int k = 0;; ++k) {
    const int mt = tile / n_ntiles, m0 = mt * BM, n0 = (tile - mt * n_ntiles) * BN;
    const float* sbias = reinterpret_cast<const float*>(sm + 2 * STAGE) + (k & 1) * BN;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[t][b] = f4v{0.f, 0.f, 0.f, 0.f};
    load(0, std::integral_constant<int, 0>{});
    int u = 0;
    for (; u + 2 < nk; u += 2) {
      body(u, std::integral_constant<int, 0>{});
      body(u + 1, std::integral_constant<int, 1>{});
    }
    if (u + 1 < nk) {
      body(u, std::integral_constant<int, 0>{});
      __builtin_amdgcn_s_waitcnt(0xC07F);
      mma(std::integral_constant<int, 1>{});
    } else {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      mma(std::integral_constant<int, 0>{});
    }
    // every wave's fragment reads of both slots retired: the ring is free for the next tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int vn = v + nb;
    const bool more = vn < ntiles;
    int tile_n = tile;
    if (more) {
      tile_n = x3p_tile(vn, ntiles);
      setup(tile_n, cur);
      issue(cur, 0, 0);
      if (nk > 1) issue(cur, 1, 1);
      if (has_bias && tid < BN / 4) {
        const int nn0 = (tile_n % n_ntiles) * BN;
        const float4 bv = *reinterpret_cast<const float4*>(bias + nn0 + 4 * tid);
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(sm + 2 * STAGE) + ((k + 1) & 1) * BN + 4 * tid) = bv;
      }
    }
    // epilogue of this tile (as k_gemm_x3h), under the next tile's first DMA
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = m0 + wm * 64 + 16 * b + il;
      if (m >= M) continue;
#pragma unroll
      for (int c = 0; c < NT / 2; ++c) {
        const int U = (n0 >> 5) + wn * (NT / 2) + c;
        float vv[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          vv[r] = acc[2 * c][b][r] * wscale;
          vv[4 + r] = acc[2 * c + 1][b][r] * wscale;
        }
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_ELU) {
          if (has_bias) {
            const float* bsrc = sbias + 32 * (wn * (NT / 2) + c) + 4 * ql;
            const float4 b0 = *reinterpret_cast<const float4*>(bsrc);
            const float4 b1 = *reinterpret_cast<const float4*>(bsrc + 16);
            vv[0] += b0.x, vv[1] += b0.y, vv[2] += b0.z, vv[3] += b0.w;
            vv[4] += b1.x, vv[5] += b1.y, vv[6] += b1.z, vv[7] += b1.w;
          }
          if (EPI == EPI_BIAS_ELU)
#pragma unroll
            for (int j = 0; j < 8; ++j) vv[j] = vv[j] > 0.f ? vv[j] : __expf(vv[j]) - 1.0f;
        } else {
          float a[8];
          x3_get8(AUX + (size_t)m * ldaux, 0, U, ql, a);
#pragma unroll
          for (int j = 0; j < 8; ++j) vv[j] *= a[j] > 0.f ? 1.0f : a[j] + 1.0f;
        }
        x3_put8(OUT + (size_t)m * ldc, 0, U, ql, vv);
      }
    }
    if (!more) break;
    // the next tile's chunks 0 and 1 and its bias landed; every wave is past this tile's epilogue
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    v = vn;
    tile = tile_n;
  }
}
}  // namespace dpi
