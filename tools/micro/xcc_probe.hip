// Does a workgroup land on the same XCD in consecutive launches of one kernel?
// Launches a 2048-workgroup kernel (the C2 env kernel's grid) several times and
// records HW_REG_XCC_ID per workgroup; prints how many workgroups changed XCD
// between launches, and the implied round-robin offset (xcc - b) mod 8.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void probe(int* out, int launch) {
  if (threadIdx.x == 0) {
    int xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID (id 20), offset 0, size 4
    out[launch * gridDim.x + blockIdx.x] = xcc & 0xF;
  }
}

int main() {
  const int G = 2048, L = 6;
  int* d;
  hipMalloc(&d, G * L * sizeof(int));
  for (int l = 0; l < L; ++l) hipLaunchKernelGGL(probe, dim3(G), dim3(64), 0, 0, d, l);
  hipDeviceSynchronize();
  std::vector<int> h(G * L);
  hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost);
  for (int l = 0; l < L; ++l) {
    int changed = 0, hist[8] = {0};
    for (int b = 0; b < G; ++b) {
      if (l && h[l * G + b] != h[(l - 1) * G + b]) ++changed;
      hist[((h[l * G + b] - b) % 8 + 8) % 8]++;
    }
    printf("launch %d: changed vs previous %d / %d; offset histogram", l, changed, G);
    for (int k = 0; k < 8; ++k) printf(" %d", hist[k]);
    printf("\n");
  }
  return 0;
}
