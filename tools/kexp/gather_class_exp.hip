// Experiment: the headline multiclass exact-histogram update WITHOUT the class-major codes round trip.
//   pass 1 (row stats)   — per row: max and the exp-sum of the softmax (the production row pass's exact sequence:
//                          row_stat, exp_nonpos2, wave_sum_uniform), stored as {max, sum, 1/sum}; the batch's
//                          softmax witness (any score outside [0, 1]) as a device flag — no speculation, no FIXUP.
//                          Plain (allocating) loads, so the logits stay in the 256-MiB Infinity Cache for pass 2.
//   pass 2 (class group) — one workgroup per group of K classes: every row's K consecutive scores (8 B at K = 4) are
//                          gathered, turned into the same bf16 softmax codes (exp_nonpos2, div_rn2, pack_rne2) and
//                          counted into K u16-packed LDS histograms (K x 32 KiB); positives straight to global.
// Production (two-pass with a 131-MB class-major scratch): row pass 62 us + FIXUP 4.5 us + class pass 44 us.
// Validated here against the production kernels on the same batches (identical int64 histograms and code ranges).
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/gather_class_exp.hip -o build/gather_class_exp
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

namespace tmx {

// ---- pass 1: row statistics (one wave per row pair, packed fp32 pair math as in row_tile_compute) ----------------
constexpr int kStatThreads = 256;
template <typename T>
__global__ void __launch_bounds__(kStatThreads) row_stats_kernel(const T* __restrict__ preds, int64_t n, int C, int ld,
                                                                 float4* __restrict__ stats, int* __restrict__ witness) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nvec = ld / 8;
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  const int lq = lo_ok ? lane : nvec - 1;
  const int hq = hi_ok ? lane + kWave : nvec - 1;
  const int64_t pairs = (n + 1) / 2;
  bool saw = false;
  for (int64_t pr = (int64_t)blockIdx.x * (kStatThreads / kWave) + wave; pr < pairs; pr += (int64_t)gridDim.x * (kStatThreads / kWave)) {
    const int64_t r0 = 2 * pr, r1 = min(2 * pr + 1, n - 1);
    const uint4* a = reinterpret_cast<const uint4*>(preds + r0 * ld);
    const uint4* b = reinterpret_cast<const uint4*>(preds + r1 * ld);
    uint4 wa[2], wb[2];
    wa[0] = a[lq]; wa[1] = a[hq]; wb[0] = b[lq]; wb[1] = b[hq];
    RowStat<2> ra, rb;
    row_stat<T, 2>(wa, lo_ok, hi_ok, ra);
    row_stat<T, 2>(wb, lo_ok, hi_ok, rb);
    f32x2 acc = {0.f, 0.f};
    const f32x2 mx2 = {ra.mx, rb.mx};
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = acc + exp_nonpos2(f32x2{ra.v[j], rb.v[j]} - mx2);
    const float sa = wave_sum_uniform(acc.x), sb = wave_sum_uniform(acc.y);
    saw = saw || ra.mx > 1.f || rb.mx > 1.f || wave_min_uniform(__builtin_fminf(ra.mn, rb.mn)) < 0.f;
    if (lane == 0) {
      stats[r0] = make_float4(ra.mx, sa, 1.f / sa, 0.f);
      if (r1 != r0) stats[r1] = make_float4(rb.mx, sb, 1.f / sb, 0.f);
    }
  }
  if (saw && lane == 0) atomicOr(witness, 1);
}

// ---- pass 2: K classes per workgroup ----------------------------------------------------------------------------
template <int K, int NT, int U>
__global__ void __launch_bounds__(NT) gather_hist_kernel(const __hip_bfloat16* __restrict__ preds, const int64_t* __restrict__ target,
                                                         const float4* __restrict__ stats, int64_t n, int C, int ld,
                                                         const int* __restrict__ witness, int64_t* __restrict__ hist,
                                                         int* __restrict__ code_range) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_w[];  // [K][kCodes / 2] u16 pairs
  const int c0 = blockIdx.x * K;
  uint4* s4 = reinterpret_cast<uint4*>(s_w);
  for (int i = threadIdx.x; i < K * kCodes / 8; i += NT) s4[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const bool softmax = *witness != 0;
  int lo[K], hi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { lo[k] = kCodes; hi[k] = -1; }
  static_assert(K == 4, "8-byte gathers");
  for (int64_t cb = 0; cb < n; cb += kClassChunk) {
    const int64_t ce = cb + kClassChunk < n ? cb + kClassChunk : n;
    for (int64_t r = cb + threadIdx.x; r < ce; r += U * NT) {
      uint2 w[U];
      float4 st[U];
      int64_t tv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = min(r + u * NT, ce - 1);
        w[u] = *reinterpret_cast<const uint2*>(preds + rr * ld + c0);
        st[u] = stats[rr];
        tv[u] = target[rr];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * NT >= ce) break;
        uint32_t codes[2];
        if (softmax) {
          const float v0 = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(w[u].x & 0xFFFFu)));
          const float v1 = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(w[u].x >> 16)));
          const float v2 = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(w[u].y & 0xFFFFu)));
          const float v3 = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(w[u].y >> 16)));
          const f32x2 m2 = {st[u].x, st[u].x}, s2 = {st[u].y, st[u].y}, i2 = {st[u].z, st[u].z};
          codes[0] = pack_rne2<__hip_bfloat16>(div_rn2(exp_nonpos2(f32x2{v0, v1} - m2), s2, i2));
          codes[1] = pack_rne2<__hip_bfloat16>(div_rn2(exp_nonpos2(f32x2{v2, v3} - m2), s2, i2));
        } else {
          codes[0] = raw_code<__hip_bfloat16>(w[u].x & 0xFFFFu) | (raw_code<__hip_bfloat16>(w[u].x >> 16) << 16);
          codes[1] = raw_code<__hip_bfloat16>(w[u].y & 0xFFFFu) | (raw_code<__hip_bfloat16>(w[u].y >> 16) << 16);
        }
        const int64_t t = tv[u];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const uint32_t x = (k & 1) ? (codes[k >> 1] >> 16) : (codes[k >> 1] & 0xFFFFu);
          const uint32_t bin = (x & 0x8000u) ? (uint32_t)kTrashBin : (x & 0x3FFFu);
          if (t == c0 + k) {
            atomic_add_i64(hist + ((int64_t)(c0 + k) * 2 + 1) * kCodes + bin, 1);
            lo[k] = min(lo[k], (int)bin);
            hi[k] = max(hi[k], (int)bin);
          } else {
            atomicAdd(&s_w[k * (kCodes / 2) + (bin >> 1)], 1u << ((bin & 1u) << 4));
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int64_t* neg = hist + ((int64_t)(c0 + k) * 2) * kCodes;
      for (int wd = threadIdx.x; wd < kCodes / 2; wd += NT) {
        uint32_t v = s_w[k * (kCodes / 2) + wd];
        if (wd == kTrashBin / 2) v &= 0xFFFFu;
        if (v) {
          const uint32_t a = v & 0xFFFFu, b = v >> 16;
          if (a) { neg[2 * wd] += a; lo[k] = min(lo[k], 2 * wd); hi[k] = max(hi[k], 2 * wd); }
          if (b) { neg[2 * wd + 1] += b; lo[k] = min(lo[k], 2 * wd + 1); hi[k] = max(hi[k], 2 * wd + 1); }
          s_w[k * (kCodes / 2) + wd] = 0u;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int l = wave_min_i32(lo[k]), h = wave_max_i32(hi[k]);
    if ((threadIdx.x & (kWave - 1)) == 0 && h >= 0) {
      atomicMin(code_range + 2 * (c0 + k), l);
      atomicMax(code_range + 2 * (c0 + k) + 1, h);
    }
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
  if (C % 8 != 0 || C > 1024 || C <= 512) { printf("C must be a multiple of 8 in (512, 1024]\n"); return 1; }
  const int64_t n_pad = (N + kTileRows - 1) / kTileRows * kTileRows;
  const int64_t ntiles = n_pad / kTileRows;
  const size_t xbytes = (size_t)N * C * 2, cbytes = (size_t)C * n_pad * 2, hbytes = (size_t)C * 2 * kCodes * 8;
  const int NB = 4;
  std::vector<__hip_bfloat16*> xs(NB);
  for (int k = 0; k < NB; ++k) { CK(hipMalloc(&xs[k], xbytes)); hipLaunchKernelGGL(init_logits, 4096, 256, 0, 0, xs[k], N * C, 1234u + k); }
  int64_t *t, *cm, *histA, *histB;
  uint32_t* codes;
  float4* stats;
  int *mode, *err, *rows, *state, *rA, *rB, *wit;
  CK(hipMalloc(&t, N * 8)); hipLaunchKernelGGL(init_target, 256, 256, 0, 0, t, N, C, 7u);
  CK(hipMalloc(&cm, (size_t)C * C * 8)); CK(hipMalloc(&codes, cbytes)); CK(hipMalloc(&histA, hbytes)); CK(hipMalloc(&histB, hbytes));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&rows, 2 * N * 4)); CK(hipMalloc(&state, 24));
  CK(hipMalloc(&rA, C * 8)); CK(hipMalloc(&rB, C * 8)); CK(hipMalloc(&stats, N * 16)); CK(hipMalloc(&wit, 4));
  CK(hipMemset(state, 0, 24)); CK(hipMemset(cm, 0, (size_t)C * C * 8)); CK(hipMemset(wit, 0, 4));
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
    int splits = 1;
    while ((int64_t)C * splits < 512 && n_pad / (8 * (splits * 2)) >= 1024) splits *= 2;
    hipLaunchKernelGGL((class_hist_u16_kernel<__hip_bfloat16>), C * splits, kClassThreadsU16, kCodes * 2, 0, (const uint16_t*)codes, n_pad,
                       splits, histA, x, C, t, N, mode, true, rows, state, (int64_t*)nullptr, rA, mode, (int64_t*)nullptr, (int*)nullptr);
  };
  const int stat_grid = 2048;
  auto p1 = [&](const __hip_bfloat16* x) {
    CK(hipMemsetAsync(wit, 0, 4, 0));
    hipLaunchKernelGGL(row_stats_kernel<__hip_bfloat16>, stat_grid, kStatThreads, 0, 0, x, N, C, C, stats, wit);
  };
  auto p2 = [&](const __hip_bfloat16* x, int variant) {
    if (variant == 0)
      hipLaunchKernelGGL((gather_hist_kernel<4, 1024, 4>), C / 4, 1024, 4 * kCodes * 2, 0, x, t, stats, N, C, C, wit, histB, rB);
    else
      hipLaunchKernelGGL((gather_hist_kernel<4, 512, 8>), C / 4, 512, 4 * kCodes * 2, 0, x, t, stats, N, C, C, wit, histB, rB);
  };
  CK(hipFuncSetAttribute((const void*)gather_hist_kernel<4, 1024, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kCodes * 2));
  CK(hipFuncSetAttribute((const void*)gather_hist_kernel<4, 512, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kCodes * 2));
  // correctness: 3 batches accumulated by both designs
  CK(hipMemset(histA, 0, hbytes)); CK(hipMemset(histB, 0, hbytes));
  hipLaunchKernelGGL(reset_range, (C + 255) / 256, 256, 0, 0, rA, C); hipLaunchKernelGGL(reset_range, (C + 255) / 256, 256, 0, 0, rB, C);
  for (int k = 0; k < 3; ++k) { row(xs[k]); clsA(xs[k]); p1(xs[k]); p2(xs[k], k == 1); }
  CK(hipDeviceSynchronize());
  std::vector<int64_t> ha(hbytes / 8), hb(hbytes / 8);
  std::vector<int> ra(2 * C), rb(2 * C);
  CK(hipMemcpy(ha.data(), histA, hbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(hb.data(), histB, hbytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ra.data(), rA, 8 * C, hipMemcpyDeviceToHost)); CK(hipMemcpy(rb.data(), rB, 8 * C, hipMemcpyDeviceToHost));
  int64_t hd = 0, rd = 0, tot = 0, pos = 0;
  for (size_t i = 0; i < ha.size(); ++i) { hd += ha[i] != hb[i]; tot += ha[i]; if ((i / kCodes) & 1) pos += ha[i]; }
  for (int i = 0; i < 2 * C; ++i) rd += ra[i] != rb[i];
  printf("{\"N\": %lld, \"C\": %d, \"hist_diffs\": %lld, \"range_diffs\": %lld, \"counts\": %lld, \"positives\": %lld", (long long)N, C,
         (long long)hd, (long long)rd, (long long)tot, (long long)pos);
  const float tRow = time_us([&](int i) { row(xs[i % NB]); });
  const float tCls = time_us([&](int i) { clsA(xs[i % NB]); });
  const float tProd = time_us([&](int i) { row(xs[i % NB]); clsA(xs[i % NB]); });
  const float tP1 = time_us([&](int i) { p1(xs[i % NB]); });
  const float tP2a = time_us([&](int i) { p2(xs[i % NB], 0); });
  const float tP2b = time_us([&](int i) { p2(xs[i % NB], 1); });
  const float tNewA = time_us([&](int i) { p1(xs[i % NB]); p2(xs[i % NB], 0); });
  const float tNewB = time_us([&](int i) { p1(xs[i % NB]); p2(xs[i % NB], 1); });
  printf(", \"prod_row_plus_fixup_us\": %.2f, \"prod_class_us\": %.2f, \"prod_seq_us\": %.2f, \"p1_stats_us\": %.2f, \"p2_1024x4_us\": %.2f, "
         "\"p2_512x8_us\": %.2f, \"new_seq_1024x4_us\": %.2f, \"new_seq_512x8_us\": %.2f}\n",
         tRow, tCls, tProd, tP1, tP2a, tP2b, tNewA, tNewB);
  return 0;
}
