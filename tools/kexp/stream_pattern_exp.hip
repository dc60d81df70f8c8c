// Does the class pass's access pattern cap its read bandwidth?  131 MB of codes, read three ways (no other work):
//   grid      : grid-stride 16-B loads (STREAM style: at any time the chip reads one narrow address band)
//   blocklocal: one workgroup per class, 1000 x 128 KiB contiguous regions read concurrently (the class pass)
//   blocklocal_db: the same with the next step's loads in flight while the current ones are consumed
// Build: hipcc -O3 --offload-arch=gfx950 tools/kexp/stream_pattern_exp.hip -o build/kexp_r5/stream_pattern_exp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(256) grid_read(const uint4* __restrict__ a, int64_t nv, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += 4 * stride) {
    uint4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = i + u * stride < nv ? a[i + u * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

template <int U, int NT>
__global__ void __launch_bounds__(NT) block_read(const uint4* __restrict__ a, int64_t per_block, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint4* col = a + blockIdx.x * per_block;
  for (int64_t cb = 0; cb < per_block; cb += U * NT) {
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = col[cb + threadIdx.x + u * NT];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

template <int U, int NT>
__global__ void __launch_bounds__(NT) block_read_db(const uint4* __restrict__ a, int64_t per_block, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint4* col = a + blockIdx.x * per_block;
  uint4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = col[threadIdx.x + u * NT];
  for (int64_t cb = 0; cb < per_block; cb += 2 * U * NT) {
    const bool m1 = cb + U * NT < per_block, m2 = cb + 2 * U * NT < per_block;
    if (m1) {
#pragma unroll
      for (int u = 0; u < U; ++u) y[u] = col[cb + U * NT + threadIdx.x + u * NT];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    if (!m1) break;
    if (m2) {
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = col[cb + 2 * U * NT + threadIdx.x + u * NT];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= y[u].x ^ y[u].y ^ y[u].z ^ y[u].w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

template <typename F>
float time_us(F f, int iters = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main() {
  const int C = 1000;
  const int64_t per = 8192;  // 16-B vectors per class (65536 rows of 2-B codes)
  const int64_t nv = per * C;
  uint4* a; uint32_t* out;
  CK(hipMalloc(&a, nv * 16)); CK(hipMalloc(&out, 4096 * 4));
  CK(hipMemset(a, 1, nv * 16));
  printf("{\"MB\": %.1f", nv * 16 / 1e6);
  printf(", \"grid_1024x256\": %.2f", time_us([&] { hipLaunchKernelGGL(grid_read, 1024, 256, 0, 0, a, nv, out); }));
  printf(", \"grid_2048x256\": %.2f", time_us([&] { hipLaunchKernelGGL(grid_read, 2048, 256, 0, 0, a, nv, out); }));
  printf(", \"block_512_u8\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read<8, 512>), C, 512, 32784, 0, a, per, out); }));
  printf(", \"block_512_u8_nolds\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read<8, 512>), C, 512, 0, 0, a, per, out); }));
  printf(", \"block_512_u4\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read<4, 512>), C, 512, 32784, 0, a, per, out); }));
  printf(", \"block_512_db4\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read_db<4, 512>), C, 512, 32784, 0, a, per, out); }));
  printf(", \"block_256_db4_half\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read_db<4, 256>), 2 * C, 256, 16400, 0, a, per / 2, out); }));
  printf(", \"block_1024_u8\": %.2f", time_us([&] { hipLaunchKernelGGL((block_read<8, 1024>), C, 1024, 65568, 0, a, per, out); }));
  printf("}\n");
  return 0;
}
