// Do 16-B global loads at 2-byte-aligned addresses return the right bytes on gfx950, and what do they cost?
// (C % 8 != 0 multiclass rows start at 2-byte granularity: C = 1001 row r begins 2 (r % 8) bytes past a 16-B boundary;
// the round-4 route padded every row with a copy.)  Reads a 131 MB u16 buffer as rows of C = 1001 elements with one
// 16-B load per 8 elements at the row's own (misaligned) address, checks every loaded element against the expected
// pattern, and times the sweep against the same sweep over 1008-element (aligned) rows.  Also the raw-buffer form
// (make_buffer_rsrc + raw_buffer_load with num_records = buffer bytes: past-the-end lanes read 0) at the same offsets.
// Build: hipcc -O3 --offload-arch=gfx950 tools/kexp/unaligned_load_exp.hip -o build/kexp_r5/unaligned_load_exp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(err_), __FILE__, __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint16_t pattern(int64_t i) { return static_cast<uint16_t>((i * 2654435761ull) >> 7); }

__global__ void fill(uint16_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = pattern(i);
}

// one wave per row; lane l loads elements [8l, 8l + 8) of the row (global_load_dwordx4 at the row's own address)
template <int MODE>
__global__ void __launch_bounds__(256) sweep(const uint16_t* __restrict__ p, int64_t rows, int C, int64_t total, int* bad, uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (row >= rows) return;
  const int nvec = (C + 7) / 8;
  uint32_t acc = 0;
  int errs = 0;
  for (int v = lane; v < nvec; v += 64) {
    const int64_t e0 = row * C + 8 * v;
    uint4 w;
    if constexpr (MODE == 0) {
      if (e0 + 8 > total) continue;  // (the plain form needs the caller to keep the tail in bounds)
      w = *reinterpret_cast<const uint4*>(p + e0);
    } else {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p), 0, static_cast<int>(total * 2), 0x00020000);
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(e0 * 2), 0, 0);
      w = make_uint4(x.x, x.y, x.z, x.w);
    }
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
    for (int k = 0; k < 8; ++k) {
      const int64_t e = e0 + k;
      if (8 * v + k >= C) break;
      const uint16_t got = static_cast<uint16_t>(d[k >> 1] >> (16 * (k & 1)));
      if (e < total && got != pattern(e)) ++errs;
      acc += got;
    }
  }
  if (errs) atomicAdd(bad, errs);
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const int64_t rows = 65536;
  const int Cs[2] = {1001, 1008};
  const int64_t total = rows * 1008;
  uint16_t* p;
  CK(hipMalloc(&p, total * 2));
  int* bad;
  uint32_t* sink;
  CK(hipMalloc(&bad, 4));
  CK(hipMalloc(&sink, 4));
  hipLaunchKernelGGL(fill, 4096, 256, 0, 0, p, total);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("{");
  for (int mode = 0; mode < 2; ++mode) {
    for (int ci = 0; ci < 2; ++ci) {
      const int C = Cs[ci];
      const int64_t tot = rows * C;
      CK(hipMemset(bad, 0, 4));
      const int grid = static_cast<int>((rows * 64 + 255) / 256);
      float best = 1e9f;
      for (int it = 0; it < 12; ++it) {
        CK(hipEventRecord(a));
        if (mode == 0) hipLaunchKernelGGL(sweep<0>, grid, 256, 0, 0, p, rows, C, tot, bad, sink);
        else hipLaunchKernelGGL(sweep<1>, grid, 256, 0, 0, p, rows, C, tot, bad, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it >= 2 && ms < best) best = ms;
      }
      int h = 0;
      CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
      printf("%s\"%s_C%d\": {\"us\": %.2f, \"TBps\": %.3f, \"bad_elements\": %d}", (mode || ci) ? ", " : "", mode ? "buffer" : "global", C,
             best * 1e3f, tot * 2 / (best * 1e-3) / 1e12, h / 12);
    }
  }
  printf("}\n");
  return 0;
}
