// Standalone ablation harness for the exact-histogram kernels (no torch): times mc_codes_kernel variants with
// parts switched off, class_hist_kernel, and range_flag16_kernel on logits vs probabilities.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/curve_hist_exp.hip -o build/curve_hist_exp
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }

template <typename F>
float time_us(F f, int iters = 20) {
  for (int i = 0; i < 3; ++i) f();
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
  const int64_t N = 65536; const int C = 1000;
  std::vector<uint16_t> h(N * C), hp(N * C);
  std::vector<int64_t> ht(N);
  srand(1);
  for (int64_t i = 0; i < N * C; ++i) {
    float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
    float g = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    h[i] = f2bf(g);
    hp[i] = f2bf(u1);
  }
  for (int64_t i = 0; i < N; ++i) ht[i] = rand() % C;
  __hip_bfloat16 *d, *dp; int64_t *dt, *hist, *cm; int *mode, *err, *flag; uint32_t* codes;
  const int64_t n_pad = (N + kTileRows - 1) / kTileRows * kTileRows;
  CK(hipMalloc(&d, N * C * 2)); CK(hipMalloc(&dp, N * C * 2)); CK(hipMalloc(&dt, N * 8));
  CK(hipMalloc(&hist, (int64_t)C * 2 * kCodes * 8)); CK(hipMalloc(&cm, (int64_t)C * C * 8));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&flag, 4)); CK(hipMalloc(&codes, (int64_t)C * n_pad * 2));
  CK(hipMemcpy(d, h.data(), N * C * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dp, hp.data(), N * C * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(hist, 0, (int64_t)C * 2 * kCodes * 8)); CK(hipMemset(cm, 0, (int64_t)C * C * 8));
  int hm[2] = {1, 0};
  CK(hipMemcpy(mode, hm, 8, hipMemcpyHostToDevice));
  const int64_t ntiles = n_pad / kTileRows;
  const int grid = (int)std::min<int64_t>(ntiles, 256 * 2);
  const size_t shm = (size_t)C * (kTileRows / 2) * 4;
#define RUN_MC(ABL) time_us([&] { hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, ABL>), grid, kA_Threads, shm, 0, d, dt, N, C, mode, -1, false, codes, n_pad, cm, err, false); })
  float t_full = RUN_MC(0);
  float t_nostore = RUN_MC(kAblNoStore);
  float t_nonorm = RUN_MC(kAblNoNorm);
  float t_nolds = RUN_MC(kAblNoLds | kAblNoStore);
  float t_min = RUN_MC(kAblNoLds | kAblNoStore | kAblNoNorm);
  float t_rec = time_us([&] { hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 0>), grid, kA_Threads, shm, 0, d, dt, N, C, mode, -1, false, codes, n_pad, cm, err, true); });
  float t_fix = time_us([&] { hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, true, 0>), grid, kA_Threads, shm, 0, d, dt, N, C, mode, -1, false, codes, n_pad, cm, err, false); });
  float t_hist = time_us([&] { hipLaunchKernelGGL(class_hist_kernel, C, 512, kCodes * 4, 0, (const uint16_t*)codes, n_pad, 1, hist, (int*)nullptr); });
  const int64_t nvec = N * C / 8;
  float t_rf_logit = time_us([&] { CK(hipMemsetAsync(flag, 0, 4)); hipLaunchKernelGGL(range_flag16_kernel<__hip_bfloat16>, 2048, 256, 0, 0, (const uint4*)d, nvec, (const uint16_t*)d, 0, flag); });
  float t_rf_prob = time_us([&] { CK(hipMemsetAsync(flag, 0, 4)); hipLaunchKernelGGL(range_flag16_kernel<__hip_bfloat16>, 2048, 256, 0, 0, (const uint4*)dp, nvec, (const uint16_t*)dp, 0, flag); });
  float t_memset = time_us([&] { CK(hipMemsetAsync(flag, 0, 4)); });
  CK(hipDeviceSynchronize());
  printf("{\"mc_codes_full_us\": %.1f, \"mc_codes_record_mode_us\": %.1f, \"mc_codes_fixup_noop_us\": %.1f, \"mc_codes_no_store_us\": %.1f, \"mc_codes_no_norm_us\": %.1f, "
         "\"mc_codes_no_lds_no_store_us\": %.1f, \"mc_codes_loads_argmax_only_us\": %.1f, \"class_hist_us\": %.1f, "
         "\"range_flag_logits_us\": %.1f, \"range_flag_probs_us\": %.1f, \"memset4_us\": %.1f}\n",
         t_full, t_rec, t_fix, t_nostore, t_nonorm, t_nolds, t_min, t_hist, t_rf_logit, t_rf_prob, t_memset);
  return 0;
}
