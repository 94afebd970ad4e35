// A/B microbenchmark of the 512-wide split GEMMs: k_gemm_x3h (128 x 128 tile, two blocks per CU,
// buffer-form LDS-DMA since r03f) against k_gemm_x3 (256 x 128, pointer-form LDS-DMA), whose
// products per output run in the same order, so the outputs must be bitwise equal; the harness
// counts differing words.  Shapes: the HJB chain's 262,144 x 512 x 512 (ELU, DELU), a partial last
// m-tile, K = 128 / 96 (short and odd chunk counts), K = 1,024 from two sources, one chunk, and a
// 2,304-word row stride (the activation workspace's: row offsets past 2^31 bytes).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_x3h tools/ubench_x3h.hip
//   tools/ubench_x3h [M] [iters]
//
// Record (r03f, profiles/r03f_ubench_x3g.txt, r03f_ubench_x3hb.txt):
//  - buffer-form DMA in k_gemm_x3h (scalar LDS destinations: the wave id through readfirstlane;
//    fixed per-lane row offsets, the chunk's column in soffset): bitwise equal, ELU 567-573 ->
//    528-536 us, DELU 600-609 -> 579-592 us, K 128 261 -> 250 / 320 -> 307 us;
//  - k_gemm_x3g, X fragments loaded from global straight into registers (W alone through a deeper
//    LDS-DMA ring): bitwise equal but 763-793 us (ELU) / 809-834 us (DELU).  A fragment load
//    touches 16 rows x 4 half-lines per wave-instruction (the DMA: 8 rows x 1 line) and both waves
//    of an m-range load the same bytes — 4x the vector-L1 line accesses for X.  Its inline-asm
//    loads (the compiler's own waits fell to vmcnt(0) with VGPR loads and LDS-DMA both in flight)
//    faulted the GPU twice (XD = 2 spilling, then K = 96 with a partial m-tile): removed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cmath>

#include "../deeppicarditeration_amd/csrc/dpi_device.h"
#include "x3q_proto.h"

using namespace dpi;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
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

struct Case {
  int M, Kp, Np, nk1;  // K = Kp: chunks < nk1 from X (row stride ldx), the rest from X2
  int ldx, ldx2;
  int ldaux = 512;  // AUX rows (DELU operand), Np = 512 words unless the workspace's stride
};

struct Bufs {
  uint32_t* W;
  float *X, *X2, *AUX, *OUT, *REF, *bias;
};

// kind 0: k_gemm_x3 (256 x 128 tile, pointer-form LDS-DMA: the reference for bitwise equality),
// 1: k_gemm_x3h (128 x 128, two blocks per CU, buffer-form LDS-DMA since r03f), 2: k_gemm_x3q
// (tools/x3q_proto.h: x3h with a 3-slot X ring, X two chunks ahead)
template <int EPI>
static void launch(int kind, const Case& c, const Bufs& b, float* out) {
  const float* bias = EPI == EPI_DELU ? nullptr : b.bias;
  const int nnt = c.Np / 128;
  if (kind == 0) {
    const int nmt = (c.M + X3_BM - 1) / X3_BM;
    hipLaunchKernelGGL((k_gemm_x3<EPI, 4>), dim3(nnt * nmt), dim3(X3_THREADS), 0, 0, c.M, c.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux, 0);
  } else if (kind == 1) {
    const int nmt = (c.M + X3H_BM - 1) / X3H_BM;
    hipLaunchKernelGGL(k_gemm_x3h<EPI>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, c.M, c.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux);
  } else if (kind == 5) {
    const int nmt = (c.M + X3H_BM - 1) / X3H_BM, ntiles = nnt * nmt;
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nb = std::min(ntiles, 2 * ncu);
    hipLaunchKernelGGL(k_gemm_x3p<EPI>, dim3(nb), dim3(X3H_THREADS), 0, 0, c.M, c.Kp, nnt, ntiles, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux);
  } else if (kind == 4) {
    const int nmt = (c.M + X3H_BM - 1) / X3H_BM;
    hipLaunchKernelGGL(k_gemm_x3t<EPI>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, c.M, c.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux);
  } else if (kind == 3) {
    const int nmt = (c.M + X3H_BM - 1) / X3H_BM;
    hipLaunchKernelGGL(k_gemm_x3e<EPI>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, c.M, c.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux);
  } else {
    const int nmt = (c.M + X3H_BM - 1) / X3H_BM;
    hipLaunchKernelGGL(k_gemm_x3q<EPI>, dim3(nnt * nmt), dim3(X3H_THREADS), 0, 0, c.M, c.Kp, nnt, b.W, 1.0f / 16.0f,
                       b.X, c.ldx, b.X2, c.ldx2, c.nk1, out, c.Np, bias, b.AUX, c.ldaux);
  }
}

template <int EPI>
static double timed(int kind, const Case& c, const Bufs& b, int iters) {
  launch<EPI>(kind, c, b, b.OUT);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch<EPI>(kind, c, b, b.OUT);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / iters;
}

// decoded (hi + lo) outputs: max |out - ref| / max |ref| over the whole output
static double max_rel(const Case& c, const Bufs& b) {
  std::vector<uint32_t> a((size_t)c.M * c.Np), r((size_t)c.M * c.Np);
  CK(hipMemcpy(a.data(), b.OUT, a.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), b.REF, r.size() * 4, hipMemcpyDeviceToHost));
  auto dec = [](const uint32_t* row, int col) {
    const int u = col >> 5, w = col & 31, q = (w >> 2) & 3, j = (w & 3) + 4 * (w >> 4);
    const uint32_t hw = row[32 * u + 8 * q + (j >> 1)], lw = row[32 * u + 8 * q + 4 + (j >> 1)];
    const _Float16 h = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? hw >> 16 : hw & 0xFFFF));
    const _Float16 l = __builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? lw >> 16 : lw & 0xFFFF));
    return (double)(float)h + (double)(float)l;
  };
  double md = 0, mr = 0;
  for (int m = 0; m < c.M; ++m)
    for (int n = 0; n < c.Np; ++n) {
      const double x = dec(&a[(size_t)m * c.Np], n), y = dec(&r[(size_t)m * c.Np], n);
      md = std::max(md, std::fabs(x - y));
      mr = std::max(mr, std::fabs(y));
    }
  return md / mr;
}

static size_t differing(const Case& c, const Bufs& b) {
  std::vector<uint32_t> a((size_t)c.M * c.Np), r((size_t)c.M * c.Np);
  CK(hipMemcpy(a.data(), b.OUT, a.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.data(), b.REF, r.size() * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < a.size(); ++i) bad += a[i] != r[i];
  return bad;
}

template <int EPI>
static void compare(const char* name, const Case& c, const Bufs& b, int iters, int reps) {
  CK(hipMemset(b.REF, 0, (size_t)c.M * c.Np * 4));
  launch<EPI>(0, c, b, b.REF);
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < reps; ++rep)
    for (int kind : {1, 5}) {
      CK(hipMemset(b.OUT, 0xFF, (size_t)c.M * c.Np * 4));
      const double us = timed<EPI>(kind, c, b, iters);
      const size_t bad = differing(c, b);
      const double rel = (kind == 4 || (kind == 5 && bad)) ? max_rel(c, b) : 0.0;
      std::printf("%-5s %-34s %-10s %8.1f us  %6.1f TF/s(split-eff)  differing words %zu  max rel diff %.2e\n",
                  EPI == EPI_DELU ? "delu" : "elu", name,
                  kind == 0 ? "x3 (256)" : kind == 1 ? "x3h" : kind == 2 ? "x3q" : kind == 3 ? "x3e" : kind == 4 ? "x3t 32x32" : "x3p persist", us,
                  2.0 * c.M * (double)c.Kp * c.Np / (us * 1e-6) / 1e12, bad, rel);
      std::fflush(stdout);
    }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 262144;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
  const int KMAX = 1024, NP = 512;
  Bufs b;
  CK(hipMalloc(&b.W, (size_t)NP * KMAX * 4));
  CK(hipMalloc(&b.X, (size_t)M * 512 * 4));
  CK(hipMalloc(&b.X2, (size_t)M * 512 * 4));
  CK(hipMalloc(&b.AUX, (size_t)M * NP * 4));
  CK(hipMalloc(&b.OUT, (size_t)M * NP * 4));
  CK(hipMalloc(&b.REF, (size_t)M * NP * 4));
  CK(hipMalloc(&b.bias, NP * 4));
  hipLaunchKernelGGL(k_fill, dim3(NP), dim3(128), 0, 0, reinterpret_cast<float*>(b.W), NP, KMAX, KMAX, 7u, 0.8f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, b.X, M, 512, 512, 11u, 1.0f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, b.X2, M, 512, 512, 17u, 1.0f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, b.AUX, M, NP, NP, 13u, 1.5f);
  std::vector<float> hb(NP);
  for (int i = 0; i < NP; ++i) hb[i] = 0.01f * (float)((i * 37) % 17 - 8);
  CK(hipMemcpy(b.bias, hb.data(), NP * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());

  // the W image is (NP x KMAX); a case with Kp < KMAX reads its first Kp words per row as a
  // (NP x Kp) matrix, which is what the kernels take (row stride Kp)
  if (argc > 3 && std::strcmp(argv[3], "stamp") == 0) {  // per-wave s_memtime stamps of k_gemm_x3hs
    const int nmt = (M + X3H_BM - 1) / X3H_BM, nnt = NP / 128, nb = nmt * nnt;
    unsigned long long* st;
    CK(hipMalloc(&st, (size_t)nb * 4 * 8 * 8));
    for (int e = 0; e < 2; ++e) {
      CK(hipMemset(st, 0, (size_t)nb * 4 * 8 * 8));
      for (int rep = 0; rep < 30; ++rep) {
        if (e == 0)
          hipLaunchKernelGGL(k_gemm_x3hs<EPI_BIAS_ELU>, dim3(nb), dim3(X3H_THREADS), 0, 0, st, M, 512, nnt, b.W,
                             1.0f / 16.0f, b.X, 512, b.X, 512, 16, b.OUT, NP, b.bias, b.AUX, NP);
        else
          hipLaunchKernelGGL(k_gemm_x3hs<EPI_DELU>, dim3(nb), dim3(X3H_THREADS), 0, 0, st, M, 512, nnt, b.W,
                             1.0f / 16.0f, b.X, 512, b.X, 512, 16, b.OUT, NP, nullptr, b.AUX, NP);
      }
      CK(hipDeviceSynchronize());
      std::vector<unsigned long long> h((size_t)nb * 4 * 8);
      CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long tmin = ~0ull, tmax = 0;
      double pro = 0, loop = 0, epi = 0, wait = 0, vm = 0, rt = 0, cyc = 0;
      size_t nw = 0;
      for (size_t w = 0; w < (size_t)nb * 4; ++w) {
        const unsigned long long* o = &h[w * 8];
        if (!o[0]) continue;
        ++nw;
        tmin = std::min(tmin, o[0]);
        tmax = std::max(tmax, o[3]);
        pro += o[1] - o[0];
        loop += o[2] - o[1];
        epi += o[3] - o[2];
        wait += o[4];
        vm += o[5];
        rt += o[7];
        cyc += o[3] - o[0];
      }
      std::printf("in-kernel clock %.3f GHz (s_memtime / s_memrealtime at 100 MHz, mean over waves)\n",
                  cyc / rt * 0.1);
      std::printf("%s: %zu live waves; launch span %.0f cycles; per wave: prologue %.0f, main loop %.0f (of it "
                  "wait+barrier %.0f, vmcnt %.0f), epilogue %.0f cycles; MFMA issue per wave 12288 cycles\n",
                  e == 0 ? "elu" : "delu", nw, (double)(tmax - tmin), pro / nw, loop / nw, wait / nw, vm / nw,
                  epi / nw);
      // block lifetimes in order of start on one CU: the first 6 blocks' (start, end) relative to launch start
      std::printf("  first blocks (start, after prologue, after loop, end) - launch start:\n");
      for (int blk = 0; blk < 6; ++blk) {
        const unsigned long long* o = &h[(size_t)blk * 4 * 8];
        std::printf("   block %d hwid %08llx: %llu %llu %llu %llu\n", blk, o[6], o[0] - tmin, o[1] - tmin, o[2] - tmin,
                    o[3] - tmin);
      }
      std::fflush(stdout);
    }
    return 0;
  }
  const Case full{M, 512, NP, 16, 512, 512};
  compare<EPI_BIAS_ELU>("262144x512x512", full, b, iters, 3);
  compare<EPI_DELU>("262144x512x512", full, b, iters, 3);
  const Case part{M - 64, 512, NP, 16, 512, 512};
  compare<EPI_BIAS_ELU>("partial m-tile (M - 64)", part, b, iters, 1);
  const Case k128{M, 128, NP, 4, 512, 512};
  compare<EPI_BIAS_ELU>("K 128", k128, b, iters, 1);
  compare<EPI_DELU>("K 128", k128, b, iters, 1);
  const Case k96{M - 192, 96, NP, 3, 512, 512};
  compare<EPI_BIAS_ELU>("K 96, M - 192", k96, b, iters, 1);
  const Case k1024{M, 1024, NP, 16, 512, 512};
  compare<EPI_BIAS_ELU>("K 1024 two-source", k1024, b, iters, 1);
  const Case k32{M, 32, NP, 1, 512, 512};
  compare<EPI_BIAS_ELU>("K 32 (one chunk)", k32, b, iters, 1);
  // the activation workspace's row stride: X and AUX rows 2,304 words apart (M x 2,304 x 4 B > 2 GiB)
  const int LDW = 2304;
  float* Xw;
  CK(hipMalloc(&Xw, (size_t)M * LDW * 4));
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, Xw + 1024, M, 512, LDW, 19u, 1.0f);
  hipLaunchKernelGGL(k_fill, dim3(M), dim3(128), 0, 0, Xw + 1536, M, 512, LDW, 23u, 1.5f);
  Bufs bw = b;
  bw.X = Xw + 1024;
  bw.X2 = Xw + 1024;
  bw.AUX = Xw + 1536;
  const Case wide{M - 64, 512, NP, 16, LDW, LDW, LDW};
  compare<EPI_BIAS_ELU>("row stride 2304, M - 64", wide, bw, iters, 1);
  compare<EPI_DELU>("row stride 2304, M - 64", wide, bw, iters, 1);
  CK(hipFree(Xw));
  return 0;
}
