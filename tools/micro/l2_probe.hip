// Does data written by one kernel launch stay in the XCD's L2 for the next
// launch (workgroup b lands on XCD b % 8 in every launch: xcc_probe.hip)?
// writer: workgroup b writes its own 4 KiB slice; reader (next launch): the
// same workgroup reads the same slice.  Profile with
//   rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -- ./l2_probe
// and compare the reader's hit rate with a reader whose workgroups read
// another XCD's slice (shift 1).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void writer(uint4* buf, int rep) {
  uint4* p = buf + (size_t)blockIdx.x * 256;  // 4 KiB per workgroup
  for (int i = threadIdx.x; i < 256; i += 64) p[i] = make_uint4(rep, blockIdx.x, i, 7);
}

__global__ void reader(const uint4* buf, uint4* sink, int shift) {
  const int b = (blockIdx.x + shift) % gridDim.x;
  const uint4* p = buf + (size_t)b * 256;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i = threadIdx.x; i < 256; i += 64) {
    uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0xdeadbeef) sink[blockIdx.x] = acc;
}

__global__ void reader_same(const uint4* buf, uint4* sink) {  // shift 0, separate name for the trace
  const uint4* p = buf + (size_t)blockIdx.x * 256;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i = threadIdx.x; i < 256; i += 64) {
    uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0xdeadbeef) sink[blockIdx.x] = acc;
}

int main() {
  const int G = 2048;  // 8 MiB written: 1 MiB per XCD, fits its 4 MiB L2
  uint4 *buf, *sink;
  hipMalloc(&buf, (size_t)G * 4096);
  hipMalloc(&sink, (size_t)G * 16);
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(writer, dim3(G), dim3(64), 0, 0, buf, rep);
    hipLaunchKernelGGL(reader_same, dim3(G), dim3(64), 0, 0, buf, sink);
    hipLaunchKernelGGL(writer, dim3(G), dim3(64), 0, 0, buf, rep);
    hipLaunchKernelGGL(reader, dim3(G), dim3(64), 0, 0, buf, sink, 1);
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
