// VALU issue cost of 64-bit vs 32-bit variable shifts on gfx950 (one wave per
// SIMD and four, independent chains): for choosing the line-word width of
// the fan march (csrc/mc_env_kernel.hip fan_pair).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void k(uint64_t* out, int iters, uint32_t sh0) {
  uint64_t a[8];
  uint32_t b[8];
  for (int j = 0; j < 8; ++j) {
    a[j] = 0x9E3779B97F4A7C15ull * (threadIdx.x + 1 + j);
    b[j] = (uint32_t)a[j];
  }
  uint32_t sh = (sh0 + threadIdx.x) & 63;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (MODE == 0) a[j] = (a[j] >> sh) ^ a[(j + 1) & 7];                       // 64-bit shift + 64-bit xor
      else if constexpr (MODE == 1) b[j] = (b[j] >> (sh & 31)) ^ b[(j + 1) & 7];           // 32-bit shift + xor
      else {  // 6 bits out of a 64-bit word by alignbit
        const uint32_t lo = (uint32_t)a[j], hi = (uint32_t)(a[j] >> 32);
        const uint32_t v = sh < 32 ? __builtin_amdgcn_alignbit(hi, lo, sh) : (hi >> (sh - 32));
        b[j] = (v & 63u) ^ b[(j + 1) & 7];
        a[j] ^= b[j];
      }
    }
    asm volatile("" ::: "memory");
  }
  uint64_t r = 0;
  for (int j = 0; j < 8; ++j) r ^= a[j] ^ b[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  uint64_t* out;
  hipMalloc(&out, 1024 * 1024 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int wps : {1, 4}) {
    const int blocks = 256 * 4 * wps;  // 64-thread blocks: wps waves per SIMD on 256 CUs
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, out, iters, 5u);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, out, iters, 5u);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, out, iters, 5u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep) printf("waves/SIMD %d mode %d (%s): %.3f ms, %.3f ns per wave-op-pair\n", wps, mode,
                        mode == 0 ? "64-bit shift+xor" : mode == 1 ? "32-bit shift+xor" : "alignbit 6 bits",
                        ms, ms * 1e6 / ((double)iters * 8 * wps));
      }
    }
  }
  return 0;
}
