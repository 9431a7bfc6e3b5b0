// FETCH_SIZE / WRITE_SIZE calibration for the env kernel's access shapes
// (MI355X_MICROARCH.md § HBM: the x2 FETCH_SIZE factor is
// established only for 16-B/lane coalesced streaming reads).
//
// Each kernel touches a byte count known exactly on the host; the host
// writes those counts to the JSON named by argv[1].  Profile with separate
// passes (tools/gpu_fetch_calib.sh):
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_probe known.json
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- ./fetch_probe known.json
// and join with tools/fetch_calib.py.  Every buffer is far larger than the
// 256 MiB Infinity Cache and every kernel runs after a flush kernel that
// streams 1 GiB through the caches.
//
// Read shapes:
//   stream16   16 B per lane, contiguous (the guide's calibrated case)
//   line_word  one 8-B word per 128-B line (a lane per line)
//   half_line  8 lanes x 8 B = the first 64 B of each 128-B line
//   full_line8 16 lanes x 8 B = a whole 128-B line in 8-B words
//   tile_window the env kernel's staging: 16 lanes per agent map read the
//              4 x 4 tiles (8 B each) of a window at a random tile offset in
//              the map's 4 x 4-tile 128-B blocks (include/marlcov.h layout),
//              C5 geometry: 518 x 518 maps (17 x 17 blocks), one map per
//              agent, 131,072 maps (4.8 GB); known = 128 B x distinct blocks
// Write shapes:
//   w_full_line8  16 lanes x 8 B = whole lines
//   w_line_word   one 8-B word per line
//   w_tile_window the tile_window pattern as stores (the merge's write-back)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

__global__ void flush(const uint4* p, size_t n, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x9e3779b9u) sink[0] = acc;
}

__global__ void stream16(const uint4* p, size_t n, uint4* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x9e3779b9u) sink[1] = acc;
}

// `per` lanes per line, lane k reads word k of its line
__global__ void words_of_lines(const uint64_t* p, size_t nlines, int per, uint64_t* sink) {
  uint64_t acc = 0;
  const size_t nl = nlines * (size_t)per;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nl; i += (size_t)gridDim.x * blockDim.x) {
    const size_t line = i / per, k = i % per;
    acc ^= p[line * 16 + k];
  }
  if (acc == 0x9e3779b97f4a7c15ull) sink[2] = acc;
}

__global__ void w_words_of_lines(uint64_t* p, size_t nlines, int per) {
  const size_t nl = nlines * (size_t)per;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nl; i += (size_t)gridDim.x * blockDim.x) {
    const size_t line = i / per, k = i % per;
    p[line * 16 + k] = i;
  }
}

// tile index of tile (ti, tj) in a map of tcs block columns (marlcov.h)
__device__ __forceinline__ size_t tile_index(int ti, int tj, int tcs) {
  return ((size_t)(ti >> 2) * tcs + (tj >> 2)) * 16 + (ti & 3) * 4 + (tj & 3);
}

__global__ void tile_window(const uint64_t* maps, const int2* org, int nmaps, int trs, int tcs, uint64_t* sink) {
  uint64_t acc = 0;
  const size_t mw = (size_t)trs * tcs * 16;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)nmaps * 16;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i >> 4;
    const int j = (int)(i & 15);
    const int2 o = org[m];
    acc ^= maps[m * mw + tile_index(o.x + (j >> 2), o.y + (j & 3), tcs)];
  }
  if (acc == 0x9e3779b97f4a7c15ull) sink[3] = acc;
}

__global__ void w_tile_window(uint64_t* maps, const int2* org, int nmaps, int trs, int tcs) {
  const size_t mw = (size_t)trs * tcs * 16;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)nmaps * 16;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i >> 4;
    const int j = (int)(i & 15);
    const int2 o = org[m];
    maps[m * mw + tile_index(o.x + (j >> 2), o.y + (j & 3), tcs)] = i;
  }
}

int main(int argc, char** argv) {
  const char* known_path = argc > 1 ? argv[1] : "fetch_probe_known.json";
  const size_t big = (size_t)1 << 30;  // 1 GiB per buffer
  uint4 *a, *f, *sink;
  CHECK(hipMalloc(&a, big));
  CHECK(hipMalloc(&f, big));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(a, 1, big));
  CHECK(hipMemset(f, 2, big));
  const dim3 G(4096), T(256);
  auto do_flush = [&] { hipLaunchKernelGGL(flush, G, T, 0, 0, f, big / 16, sink); };

  // C5 geometry maps: 518 x 518 cells -> 65 tile rows -> 17 x 17 blocks
  const int TRS = 17, TCS = 17, TR = 65, TC = 65, TW = 4;
  const int NMAPS = 131072;
  const size_t mw = (size_t)TRS * TCS * 16;
  uint64_t* maps;
  CHECK(hipMalloc(&maps, (size_t)NMAPS * mw * 8));
  CHECK(hipMemset(maps, 3, (size_t)NMAPS * mw * 8));
  std::vector<int2> org(NMAPS);
  std::mt19937 rng(12345);
  size_t lines = 0;
  for (int m = 0; m < NMAPS; ++m) {
    org[m].x = (int)(rng() % (TR - TW + 1));
    org[m].y = (int)(rng() % (TC - TW + 1));
    const int br = ((org[m].x + TW - 1) >> 2) - (org[m].x >> 2) + 1;
    const int bc = ((org[m].y + TW - 1) >> 2) - (org[m].y >> 2) + 1;
    lines += (size_t)br * bc;
  }
  int2* dorg;
  CHECK(hipMalloc(&dorg, NMAPS * sizeof(int2)));
  CHECK(hipMemcpy(dorg, org.data(), NMAPS * sizeof(int2), hipMemcpyHostToDevice));

  const size_t nl = big / 128;  // lines in a 1 GiB buffer
  const uint64_t* a64 = reinterpret_cast<const uint64_t*>(a);
  uint64_t* w64 = reinterpret_cast<uint64_t*>(f);
  uint64_t* s64 = reinterpret_cast<uint64_t*>(sink);

  // each probe twice (the second dispatch of a name is the one read: warm TLB)
  for (int rep = 0; rep < 2; ++rep) {
    do_flush();
    hipLaunchKernelGGL(stream16, G, T, 0, 0, a, big / 16, sink);
    do_flush();
    hipLaunchKernelGGL(words_of_lines, G, T, 0, 0, a64, nl, 1, s64);  // line_word
    do_flush();
    hipLaunchKernelGGL(words_of_lines, G, T, 0, 0, a64, nl, 8, s64);  // half_line
    do_flush();
    hipLaunchKernelGGL(words_of_lines, G, T, 0, 0, a64, nl, 16, s64);  // full_line8
    do_flush();
    hipLaunchKernelGGL(tile_window, G, T, 0, 0, maps, dorg, NMAPS, TRS, TCS, s64);
    do_flush();
    hipLaunchKernelGGL(w_words_of_lines, G, T, 0, 0, w64, nl, 16);  // w_full_line8
    do_flush();
    hipLaunchKernelGGL(w_words_of_lines, G, T, 0, 0, w64, nl, 1);  // w_line_word
    do_flush();
    hipLaunchKernelGGL(w_tile_window, G, T, 0, 0, maps, dorg, NMAPS, TRS, TCS);
  }
  CHECK(hipDeviceSynchronize());
  FILE* fp = fopen(known_path, "w");
  if (!fp) return 1;
  // dispatch order per rep (names as rocprofv3 prints them are matched by
  // tools/fetch_calib.py in this order)
  fprintf(fp,
          "{\"order\": [\"stream16\", \"line_word\", \"half_line\", \"full_line8\", \"tile_window\", "
          "\"w_full_line8\", \"w_line_word\", \"w_tile_window\"],\n"
          " \"read_bytes_used\": {\"stream16\": %zu, \"line_word\": %zu, \"half_line\": %zu, \"full_line8\": %zu, "
          "\"tile_window\": %zu},\n"
          " \"lines_touched\": {\"stream16\": %zu, \"line_word\": %zu, \"half_line\": %zu, \"full_line8\": %zu, "
          "\"tile_window\": %zu, \"w_full_line8\": %zu, \"w_line_word\": %zu, \"w_tile_window\": %zu},\n"
          " \"write_bytes_used\": {\"w_full_line8\": %zu, \"w_line_word\": %zu, \"w_tile_window\": %zu},\n"
          " \"tile_window_geometry\": {\"maps\": %d, \"tile_rows\": %d, \"block_rows\": %d, \"window_tiles\": %d, "
          "\"map_bytes\": %zu}}\n",
          big, nl * 8, nl * 64, nl * 128, (size_t)NMAPS * 16 * 8, big / 128, nl, nl, nl, lines, nl, nl, lines,
          nl * 128, nl * 8, (size_t)NMAPS * 16 * 8, NMAPS, TR, TRS, TW, mw * 8);
  fclose(fp);
  printf("fetch_probe done: tile_window lines %zu (%.2f per map)\n", lines, (double)lines / NMAPS);
  return 0;
}
