// Launch-floor probe: back-to-back launches of tiny kernels whose only work
// is reading their arguments and one dependent global round trip, with a
// small argument block vs a ~400-byte by-value struct (like mc::State).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

struct Big { int64_t a[50]; const int* p; int* q; };

__global__ void k_empty() {}
__global__ void k_small(const int* p, int* q) { if (threadIdx.x == 0) q[blockIdx.x] = p[blockIdx.x] + 1; }
__global__ void k_big(Big b) { if (threadIdx.x == 0) b.q[blockIdx.x] = b.p[blockIdx.x] + (int)b.a[49]; }
__global__ void k_chain2(const int* p, int* q) {  // two dependent loads
  if (threadIdx.x == 0) { int i = p[blockIdx.x]; q[blockIdx.x] = p[(i & 1023) + 1024] + 1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <typename F>
static float timeit(F launch, hipStream_t st, int n) {
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) launch();
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
  int *p, *q; CK(hipMalloc(&p, 1 << 20)); CK(hipMalloc(&q, 1 << 20)); CK(hipMemset(p, 0, 1 << 20));
  Big b = {}; b.p = p; b.q = q; b.a[49] = 3;
  const int n = 500;
  for (int blocks : {1, 2048}) {
    printf("blocks %4d: empty %.2f us, small-arg %.2f us, 400B-arg %.2f us, 2 dependent loads %.2f us\n", blocks,
           timeit([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(64), 0, st); }, st, n),
           timeit([&] { hipLaunchKernelGGL(k_small, dim3(blocks), dim3(64), 0, st, p, q); }, st, n),
           timeit([&] { hipLaunchKernelGGL(k_big, dim3(blocks), dim3(64), 0, st, b); }, st, n),
           timeit([&] { hipLaunchKernelGGL(k_chain2, dim3(blocks), dim3(64), 0, st, p, q); }, st, n));
  }
  return 0;
}
