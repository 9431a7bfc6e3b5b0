// Workgroup-granularity probe: 2048 waves of an env-kernel-like chain (a
// dependent global round trip, ~VALU_N dependent VALU ops, LDS round trips,
// stores), dispatched as 2048 x 64, 1024 x 128 or 512 x 256 threads.  Waves
// never synchronise with each other (each owns its LDS slice), as the env
// kernel's env slots.  Prints us per launch (hipGraph of back-to-back
// launches).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NT, int VALU_N>
__global__ __launch_bounds__(NT) void k_chain(const uint32_t* __restrict__ p, uint32_t* __restrict__ q) {
  __shared__ uint32_t lds[NT * 24];
  const int w = (int)(blockIdx.x * (NT / 64) + threadIdx.x / 64);  // global wave
  const int lane = threadIdx.x & 63;
  uint32_t* my = lds + (threadIdx.x / 64) * 64 * 24;
  const uint32_t i0 = p[w * 64 + lane];                   // round trip 1
  const uint32_t v = p[((i0 & 0xFFFF) + w * 64 + lane) & 0xFFFFF];  // round trip 2 (dependent)
  uint32_t x = v ^ (uint32_t)lane;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int k = 0; k < VALU_N / 4; ++k) x = (x << 1) ^ (x >> 3) ^ (uint32_t)k;
    my[lane * 24 + r] = x;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local LDS ordering only
    x += my[((lane + 1) & 63) * 24 + r];
  }
  q[w * 64 + lane] = x;
}

template <int NT>
static float timeit(hipStream_t st, const uint32_t* p, uint32_t* q, int n) {
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL((k_chain<NT, 1000>), dim3(2048 * 64 / NT), dim3(NT), 0, st, p, q);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st); hipStreamSynchronize(st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, st); hipGraphLaunch(ge, st); hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / n;
}

int main() {
  hipStream_t st; CK(hipStreamCreate(&st));
  uint32_t *p, *q; CK(hipMalloc(&p, 4 << 20)); CK(hipMalloc(&q, 4 << 20)); CK(hipMemset(p, 0, 4 << 20));
  for (int rep = 0; rep < 2; ++rep)
    printf("2048 waves: WG 64 %.2f us, WG 128 %.2f us, WG 256 %.2f us, WG 512 %.2f us\n", timeit<64>(st, p, q, 300),
           timeit<128>(st, p, q, 300), timeit<256>(st, p, q, 300), timeit<512>(st, p, q, 300));
  return 0;
}
