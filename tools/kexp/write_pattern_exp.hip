// Does the row pass's store pattern cost write bandwidth?  The headline row pass writes 64 KiB per 32-row tile as one
// 64-B segment per class into a class-major [1000][65536] u16 scratch (PMC: 97 % of the write requests are 64 B,
// profiles/pmc_headline_r4.json).  Same bytes, same grid (2048 blocks x 512 threads, XCD-aware tile order), three
// layouts:
//   A  64-B segments, class-major (production);
//   B  128-B segments, class-pair-major (codes of classes 2k / 2k+1 interleaved per row: full lines per tile);
//   C  each block's 64 KiB contiguous (tile-major: the write floor of this traffic).
// Build: hipcc -O3 --offload-arch=gfx950 tools/kexp/write_pattern_exp.hip -o build/write_pattern_exp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int kThreads = 512;
constexpr int kC = 1000;
constexpr int64_t kRows = 65536;
constexpr int kTileRows = 32;
constexpr int64_t kTiles = kRows / kTileRows;  // 2048

__device__ __forceinline__ int64_t xcd_tile(int64_t b) {
  const int64_t per = (kTiles + 7) / 8;
  return (b % 8) * per + b / 8;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) write_kernel(uint4* __restrict__ out, uint32_t salt) {
  const int64_t tile = xcd_tile(blockIdx.x);
  // 64 KiB per block = 4096 16-B pieces, 8 per thread
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int idx = threadIdx.x + k * kThreads;  // piece of this tile
    const uint4 v = make_uint4(idx ^ salt, (uint32_t)tile, 0x3F003F00u, 0x12345678u);
    if (idx >= kC * 4) continue;  // 1000 classes x 4 pieces
    int64_t off;  // in 16-B units
    if (MODE == 0) {  // class c = idx / 4, piece g = idx % 4: c * (131072 B / 16) + tile * 4 + g
      const int c = idx / 4, g = idx % 4;
      off = (int64_t)c * (kRows * 2 / 16) + tile * 4 + g;
    } else if (MODE == 1) {  // class pair k = idx / 8, piece g = idx % 8: k * (262144 B / 16) + tile * 8 + g
      const int kk = idx / 8, g = idx % 8;
      off = (int64_t)kk * (kRows * 4 / 16) + tile * 8 + g;
    } else {  // contiguous 64 000 B per tile
      off = tile * (kC * 4) + idx;
    }
    out[off] = v;
  }
}

template <typename F>
float time_us(F f, int iters = 50) {
  for (int i = 0; i < 5; ++i) f(i);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f(i);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main() {
  const size_t bytes = (size_t)kC * kRows * 2 + (1 << 20);
  uint4* out;
  CK(hipMalloc(&out, bytes));
  const float tA = time_us([&](int i) { hipLaunchKernelGGL(write_kernel<0>, (int)kTiles, kThreads, 0, 0, out, (uint32_t)i); });
  const float tB = time_us([&](int i) { hipLaunchKernelGGL(write_kernel<1>, (int)kTiles, kThreads, 0, 0, out, (uint32_t)i); });
  const float tC = time_us([&](int i) { hipLaunchKernelGGL(write_kernel<2>, (int)kTiles, kThreads, 0, 0, out, (uint32_t)i); });
  CK(hipDeviceSynchronize());
  const double mb = (double)kC * kRows * 2 / 1e6;
  printf("{\"MB\": %.1f, \"A_64B_class_major_us\": %.2f, \"B_128B_pair_major_us\": %.2f, \"C_contiguous_us\": %.2f, \"A_TBps\": %.2f, "
         "\"B_TBps\": %.2f, \"C_TBps\": %.2f}\n", mb, tA, tB, tC, mb / tA, mb / tB, mb / tC);
  return 0;
}
