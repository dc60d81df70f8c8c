// Experiment: the headline class pass with software-pipelined code loads (the next iteration's 16-B vectors are in
// flight while the current ones are counted) and a sweep of vectors per iteration, against the production
// class_hist_u16_kernel on the production row pass's codes.  PMC of the production pass (profiles/pmc_headline_r4.json):
// LDS bank-conflict cycles ~45 % of its LDS time, code reads ~3 TB/s; both phases alternate per block.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/classpass_pipe_exp.hip -o build/classpass_pipe_exp
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

namespace tmx {
template <int NT>
__device__ __forceinline__ void flush_u16x(uint32_t* __restrict__ s_w, int64_t* __restrict__ neg_hist, int& lo, int& hi) {
  for (int w = threadIdx.x; w < kCodes / 2; w += NT) {
    uint32_t v = s_w[w];
    if (w == kTrashBin / 2) v &= 0xFFFFu;
    if (v) {
      const uint32_t a = v & 0xFFFFu, b = v >> 16;
      if (a) { neg_hist[2 * w] += a; lo = min(lo, 2 * w); hi = max(hi, 2 * w); }
      if (b) { neg_hist[2 * w + 1] += b; lo = min(lo, 2 * w + 1); hi = max(hi, 2 * w + 1); }
      s_w[w] = 0u;
    }
  }
}

template <int U>
__device__ __forceinline__ void count_vecs(const uint4 (&w)[U], uint32_t* __restrict__ s_w, int64_t* __restrict__ pos_hist, int& lo, int& hi) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t parts[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
      const uint32_t bin = (x & 0x8000u) ? (uint32_t)kTrashBin : (x & 0x3FFFu);
      atomicAdd(&s_w[bin >> 1], 1u << ((bin & 1u) << 4));
    }
    const uint32_t anypos = (parts[0] | parts[1] | parts[2] | parts[3]) & 0x40004000u;
    if (__builtin_expect(__ballot(anypos != 0) != 0, 0) && anypos != 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
        if ((x & 0xC000u) == 0x4000u) {
          atomicSub(&s_w[(x & 0x3FFFu) >> 1], 1u << ((x & 1u) << 4));
          atomic_add_i64(pos_hist + (x & 0x3FFFu), 1);
          lo = min(lo, (int)(x & 0x3FFFu));
          hi = max(hi, (int)(x & 0x3FFFu));
        }
      }
    }
  }
}

// one class per block; iterations of U vectors per thread, next iteration's loads issued before counting
template <int NT, int U>
__global__ void __launch_bounds__(NT) class_pipe_kernel(const uint16_t* __restrict__ codes, int64_t n_pad, int64_t* __restrict__ hist,
                                                        int* __restrict__ code_range) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_w[];
  const int c = blockIdx.x;
  uint4* s4 = reinterpret_cast<uint4*>(s_w);
  for (int i = threadIdx.x; i < kCodes / 8; i += NT) s4[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  int64_t* neg_hist = hist + ((int64_t)c * 2) * kCodes;
  int64_t* pos_hist = hist + ((int64_t)c * 2 + 1) * kCodes;
  const uint4* col = reinterpret_cast<const uint4*>(codes + (int64_t)c * n_pad);
  const int64_t nv = n_pad / 8;
  constexpr int64_t kChunkV = kClassChunk / 8;
  const uint4 pad = make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);
  int lo = kCodes, hi = -1;
  for (int64_t cb = 0; cb < nv; cb += kChunkV) {
    const int64_t ce = cb + kChunkV < nv ? cb + kChunkV : nv;
    uint4 a[U], b[U];
    int64_t v = cb + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = (v + u * NT < ce) ? col[v + u * NT] : pad;
    for (; v < ce; v += 2 * U * NT) {
      const int64_t vn = v + U * NT;
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = (vn + u * NT < ce) ? col[vn + u * NT] : pad;
      count_vecs<U>(a, s_w, pos_hist, lo, hi);
      if (vn >= ce) break;
      const int64_t vm = vn + U * NT;
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = (vm + u * NT < ce) ? col[vm + u * NT] : pad;
      count_vecs<U>(b, s_w, pos_hist, lo, hi);
    }
    __syncthreads();
    flush_u16x<NT>(s_w, neg_hist, lo, hi);
    __syncthreads();
  }
  lo = wave_min_i32(lo);
  hi = wave_max_i32(hi);
  if ((threadIdx.x & (kWave - 1)) == 0 && hi >= 0) {
    atomicMin(code_range + 2 * c, lo);
    atomicMax(code_range + 2 * c + 1, hi);
  }
}
}  // namespace tmx
__global__ void init_logits(__hip_bfloat16* x, int64_t total, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    uint32_t g = (uint32_t)(i >> 32) * 2654435761u ^ h;
    g ^= g >> 16; g *= 0x7feb352du; g ^= g >> 15;
    float u = ((h & 0xFFFF) + (h >> 16) + (g & 0xFFFF) + (g >> 16)) / 65536.f - 2.f;
    x[i] = __float2bfloat16(1.7f * u);
  }
}
__global__ void init_target(int64_t* t, int64_t n, int C, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    t[i] = h % C;
  }
}
__global__ void reset_range(int* r, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) { r[2 * c] = kCodes; r[2 * c + 1] = -1; }
}

template <typename F>
float time_us(F f, int iters = 20) {
  for (int i = 0; i < 3; ++i) f(i);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f(i);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 65536;
  const int C = argc > 2 ? atoi(argv[2]) : 1000;
  const int64_t n_pad = (N + kTileRows - 1) / kTileRows * kTileRows;
  const int64_t ntiles = n_pad / kTileRows;
  const size_t xbytes = (size_t)N * C * 2, cbytes = (size_t)C * n_pad * 2, hbytes = (size_t)C * 2 * kCodes * 8;
  const int NB = 4;
  std::vector<__hip_bfloat16*> xs(NB);
  for (int k = 0; k < NB; ++k) { CK(hipMalloc(&xs[k], xbytes)); hipLaunchKernelGGL(init_logits, 4096, 256, 0, 0, xs[k], N * C, 1234u + k); }
  int64_t *t, *cm, *histA, *histB;
  uint32_t* codes;
  int *mode, *err, *rows, *state, *rA, *rB;
  CK(hipMalloc(&t, N * 8)); hipLaunchKernelGGL(init_target, 256, 256, 0, 0, t, N, C, 7u);
  CK(hipMalloc(&cm, (size_t)C * C * 8)); CK(hipMalloc(&codes, cbytes)); CK(hipMalloc(&histA, hbytes)); CK(hipMalloc(&histB, hbytes));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&rows, 2 * N * 4)); CK(hipMalloc(&state, 24));
  CK(hipMalloc(&rA, C * 8)); CK(hipMalloc(&rB, C * 8));
  CK(hipMemset(state, 0, 24)); CK(hipMemset(cm, 0, (size_t)C * C * 8));
  int hm[2] = {1, 0}; CK(hipMemcpy(mode, hm, 8, hipMemcpyHostToDevice));
  const int grid1 = (int)((ntiles + 7) / 8 * 8);
  const size_t shm = (size_t)1024 * kSlots * 4;
  auto row = [&](const __hip_bfloat16* x) {
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 2, false>), grid1, kRowThreads, shm, 0, x, t, N, C, C, mode, -1, false,
                       codes, n_pad, cm, err, true, rows, state);
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, true, 2, false>), std::min(grid1, 128), kRowThreads, shm, 0, x, t, N, C, C, mode, -1,
                       false, codes, n_pad, cm, err, false, rows, state);
  };
  auto clsA = [&](const __hip_bfloat16* x) {
    hipLaunchKernelGGL((class_hist_u16_kernel<__hip_bfloat16>), C, kClassThreadsU16, kCodes * 2, 0, (const uint16_t*)codes, n_pad,
                       1, histA, x, C, t, N, mode, true, rows, state, (int64_t*)nullptr, rA, mode, (int64_t*)nullptr, (int*)nullptr);
  };
  auto clsB = [&](int variant) {
    switch (variant) {
      case 0: hipLaunchKernelGGL((class_pipe_kernel<512, 4>), C, 512, kCodes * 2, 0, (const uint16_t*)codes, n_pad, histB, rB); break;
      case 1: hipLaunchKernelGGL((class_pipe_kernel<512, 2>), C, 512, kCodes * 2, 0, (const uint16_t*)codes, n_pad, histB, rB); break;
      case 2: hipLaunchKernelGGL((class_pipe_kernel<256, 4>), C, 256, kCodes * 2, 0, (const uint16_t*)codes, n_pad, histB, rB); break;
      default: hipLaunchKernelGGL((class_pipe_kernel<256, 8>), C, 256, kCodes * 2, 0, (const uint16_t*)codes, n_pad, histB, rB); break;
    }
  };
  printf("{\"N\": %lld, \"C\": %d", (long long)N, C);
  for (int variant = 0; variant < 4; ++variant) {
    CK(hipMemset(histA, 0, hbytes)); CK(hipMemset(histB, 0, hbytes));
    hipLaunchKernelGGL(reset_range, (C + 255) / 256, 256, 0, 0, rA, C); hipLaunchKernelGGL(reset_range, (C + 255) / 256, 256, 0, 0, rB, C);
    for (int k = 0; k < 3; ++k) { row(xs[k]); clsA(xs[k]); clsB(variant); }
    CK(hipDeviceSynchronize());
    std::vector<int64_t> ha(hbytes / 8), hb(hbytes / 8);
    std::vector<int> ra(2 * C), rb(2 * C);
    CK(hipMemcpy(ha.data(), histA, hbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(hb.data(), histB, hbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ra.data(), rA, 8 * C, hipMemcpyDeviceToHost)); CK(hipMemcpy(rb.data(), rB, 8 * C, hipMemcpyDeviceToHost));
    int64_t hd = 0, rd = 0;
    for (size_t i = 0; i < ha.size(); ++i) hd += ha[i] != hb[i];
    for (int i = 0; i < 2 * C; ++i) rd += ra[i] != rb[i];
    const float tv = time_us([&](int) { clsB(variant); });
    const float sv = time_us([&](int i) { row(xs[i % NB]); clsB(variant); });
    printf(", \"v%d\": {\"hist_diffs\": %lld, \"range_diffs\": %lld, \"class_us\": %.2f, \"seq_us\": %.2f}", variant, (long long)hd, (long long)rd, tv, sv);
  }
  const float tA = time_us([&](int i) { clsA(xs[i % NB]); });
  const float sA = time_us([&](int i) { row(xs[i % NB]); clsA(xs[i % NB]); });
  printf(", \"prod_class_us\": %.2f, \"prod_seq_us\": %.2f, \"variants\": \"v0 512x4 pipelined, v1 512x2, v2 256x4, v3 256x8\"}\n", tA, sA);
  return 0;
}
