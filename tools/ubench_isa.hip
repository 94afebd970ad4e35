// Instruction-rate microbenchmark (gfx950): cycles per wave-instruction for the RNG's building blocks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N 4096
template <int OP>
__global__ void k(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3u + 1, a2 = a0 * 5u + 7, a3 = a0 * 7u + 9;
  uint32_t b0 = a0 + 11, b1 = a1 + 13, b2 = a2 + 17, b3 = a3 + 19;
  float f0 = (float)a0 * 1e-9f + 0.5f, f1 = f0 + 0.1f, f2 = f0 + 0.2f, f3 = f0 + 0.3f;
  unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    if (OP == 0) {  // v_mad_u64_u32 (4 independent chains)
      uint64_t p0 = (uint64_t)a0 * 0xD2511F53u, p1 = (uint64_t)a1 * 0xCD9E8D57u, p2 = (uint64_t)a2 * 0xD2511F53u, p3 = (uint64_t)a3 * 0xCD9E8D57u;
      a0 = (uint32_t)(p0 >> 32) ^ (uint32_t)p0; a1 = (uint32_t)(p1 >> 32) ^ (uint32_t)p1;
      a2 = (uint32_t)(p2 >> 32) ^ (uint32_t)p2; a3 = (uint32_t)(p3 >> 32) ^ (uint32_t)p3;
    } else if (OP == 1) {  // v_mul_hi_u32
      a0 = __umulhi(a0, 0xD2511F53u) + b0; a1 = __umulhi(a1, 0xCD9E8D57u) + b1;
      a2 = __umulhi(a2, 0xD2511F53u) + b2; a3 = __umulhi(a3, 0xCD9E8D57u) + b3;
    } else if (OP == 2) {  // v_mul_lo_u32
      a0 = a0 * b0 + 1; a1 = a1 * b1 + 1; a2 = a2 * b2 + 1; a3 = a3 * b3 + 1;
    } else if (OP == 3) {  // xor
      a0 ^= b1; a1 ^= b2; a2 ^= b3; a3 ^= b0; b0 ^= a1; b1 ^= a2; b2 ^= a3; b3 ^= a0;
    } else if (OP == 4) {  // transcendental
      f0 = __builtin_amdgcn_logf(f0); f1 = __builtin_amdgcn_sinf(f1); f2 = __builtin_amdgcn_sqrtf(f2); f3 = __builtin_amdgcn_cosf(f3);
    } else if (OP == 5) {  // fma
      f0 = fmaf(f0, 1.0001f, 0.5f); f1 = fmaf(f1, 1.0001f, 0.5f); f2 = fmaf(f2, 1.0001f, 0.5f); f3 = fmaf(f3, 1.0001f, 0.5f);
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3 ^ __float_as_uint(f0 + f1 + f2 + f3);
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
template <int OP>
void run(const char* name, int per_iter, int blocks, int threads) {
  uint32_t* o; unsigned long long* c; hipMalloc(&o, blocks * threads * 4); hipMalloc(&c, 8);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, o, 1u, c);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, o, 1u, c);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  double waves = (double)blocks * threads / 64.0;
  double instr = waves * N * per_iter;  // wave-instructions of the op
  printf("%-10s blocks=%5d thr=%4d  wave0 cycles/instr=%.2f   chip: %.3e wave-instr/s = %.2f wave-instr/clk/CU @2.4GHz\n",
         name, blocks, threads, (double)cy / (N * per_iter), instr / (ms * 1e-3), instr / (ms * 1e-3) / 256 / 2.4e9);
  hipFree(o); hipFree(c);
}
int main() {
  for (int occ : {1, 2, 4}) {
    int blocks = 256 * occ, thr = 256;
    run<0>("mad_u64", 4, blocks, thr);
    run<1>("mul_hi", 4, blocks, thr);
    run<2>("mul_lo", 4, blocks, thr);
    run<3>("xor", 8, blocks, thr);
    run<4>("transc", 4, blocks, thr);
    run<5>("fma", 4, blocks, thr);
  }
  return 0;
}
