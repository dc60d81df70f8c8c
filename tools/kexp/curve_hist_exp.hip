// Standalone harness for the exact-histogram kernels (no torch).  Checks the library row pass (mc_codes_kernel +
// mc_slow_rows_kernel) against the previous one-wave-per-row design (tools/kexp/curve_hist_v2_ref.h) on logits, logits with
// NaN / inf / all -inf / tied rows, ignore_index rows, probabilities and a mis-speculated mode (FIXUP path), then
// times both row passes and the class pass.  Codes may differ only where v2's reciprocal product and the library's
// correctly rounded quotient round to different 16-bit values (|diff| = 1 code); the confusion matrix is exact.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/curve_hist_exp.hip -o build/curve_hist_exp
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "curve_hist_kernels.h"
#include "curve_hist_v2_ref.h"

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

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 65536;
  const int C = argc > 2 ? atoi(argv[2]) : 1000;
  if (C % 8 != 0 || C > 1024 || C <= 512) { printf("{\"error\": \"harness covers 512 < C <= 1024, C %% 8 == 0\"}\n"); return 1; }
  const int64_t n_pad = (N + kTileRows - 1) / kTileRows * kTileRows;
  std::vector<uint16_t> h(N * C), hp(N * C);
  std::vector<int64_t> ht(N), hti(N);
  srand(1);
  for (int64_t i = 0; i < N * C; ++i) {
    float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
    float g = sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
    h[i] = f2bf(2.f * g);
    hp[i] = f2bf(u1);
  }
  for (int64_t i = 0; i < N; ++i) { ht[i] = rand() % C; hti[i] = (i % 7 == 3) ? -100 : ht[i]; }
  std::vector<uint16_t> hn = h, hpn = hp;
  for (int64_t r = 5; r < N; r += 997) hn[r * C + (r % C)] = 0x7FC0;                          // NaN
  for (int64_t r = 11; r < N; r += 1999) hn[r * C + ((r * 7) % C)] = 0x7F80;                  // +inf
  for (int64_t r = 13; r < N; r += 2999) hn[r * C + ((r * 3) % C)] = 0xFF80;                  // one -inf (finite max)
  for (int64_t r = 17; r < N; r += 4001) for (int c = 0; c < C; ++c) hn[r * C + c] = 0xFF80;  // all -inf
  for (int64_t r = 23; r < N; r += 503) hn[r * C + 3] = hn[r * C + 1] = 0x4300;               // tie at the max (128.0)
  for (int64_t r = 7; r < N; r += 1511) hpn[r * C + (r % C)] = 0x7FC0;                        // NaN among probabilities
  __hip_bfloat16 *d, *dp, *dn, *dpn; int64_t *dt, *dti, *hist, *cm2, *cm6; int *mode, *err, *slow_rows, *slow_cnt;
  uint32_t *codes2, *codes6;
  const size_t cbytes = (size_t)C * n_pad * 2, xbytes = (size_t)N * C * 2;
  CK(hipMalloc(&d, xbytes)); CK(hipMalloc(&dp, xbytes)); CK(hipMalloc(&dn, xbytes)); CK(hipMalloc(&dpn, xbytes));
  CK(hipMalloc(&dt, N * 8)); CK(hipMalloc(&dti, N * 8));
  CK(hipMalloc(&hist, (int64_t)C * 2 * kCodes * 8)); CK(hipMalloc(&cm2, (int64_t)C * C * 8)); CK(hipMalloc(&cm6, (int64_t)C * C * 8));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&codes2, cbytes)); CK(hipMalloc(&codes6, cbytes));
  CK(hipMalloc(&slow_rows, 2 * N * 4)); CK(hipMalloc(&slow_cnt, 8));
  CK(hipMemcpy(d, h.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dp, hp.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dn, hn.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dpn, hpn.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), N * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dti, hti.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(slow_cnt, 0, 8));

  const int grid2 = (int)std::min<int64_t>(n_pad / tmx_ref::kTileRows, 256 * 2);
  const size_t shm2 = (size_t)C * (tmx_ref::kTileRows / 2) * 4;
  const int grid6 = (int)((n_pad / kTileRows + 7) / 8 * 8);
  const size_t shm6 = (size_t)1024 * kSlots * 4;
  CK(hipFuncSetAttribute((const void*)mc_codes_kernel<__hip_bfloat16, false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm6));
  CK(hipFuncSetAttribute((const void*)mc_codes_kernel<__hip_bfloat16, true, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm6));
  auto set_mode = [&](int m0) { int hm[2] = {m0, 0}; CK(hipMemcpy(mode, hm, 8, hipMemcpyHostToDevice)); };
  auto run2 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    hipLaunchKernelGGL((tmx_ref::mc_codes_kernel<__hip_bfloat16, false, 0>), grid2, tmx_ref::kA_Threads, shm2, 0, x, t, N, C, mode,
                       -100, ign, codes2, n_pad, cm2, err, false);
  };
  auto row6 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign, bool rec) {
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 2>), grid6, kRowThreads, shm6, 0, x, t, N, C, mode, -100, ign,
                       codes6, n_pad, cm6, err, rec, slow_rows, slow_cnt);
  };
  // full library sequence: row pass, FIXUP row pass (no-op unless the speculation was wrong), slow rows
  auto run6 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    row6(x, t, ign, true);
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, true, 2>), std::min(grid6, 512), kRowThreads, shm6, 0, x, t, N, C, mode, -100, ign,
                       codes6, n_pad, cm6, err, false, slow_rows, slow_cnt);
    hipLaunchKernelGGL(mc_slow_rows_kernel<__hip_bfloat16>, 64, 256, 0, 0, x, t, N, C, mode, true, (uint16_t*)codes6, n_pad,
                       cm6, slow_rows, slow_cnt);
  };
  auto reset_counts = [&] { CK(hipMemsetAsync(slow_cnt, 0, 8)); };

  printf("{\"N\": %lld, \"C\": %d", (long long)N, C);
  struct Case { const char* name; const __hip_bfloat16* x; const int64_t* t; bool ign; int true_mode; int spec_mode; };
  Case cases[] = {{"logits", d, dt, false, 1, 1}, {"logits_nan_inf_ties", dn, dt, false, 1, 1}, {"logits_ignore", dn, dti, true, 1, 1},
                  {"probs", dp, dt, false, 0, 0}, {"probs_nan", dpn, dt, false, 1, 0}, {"logits_misspeculated", dn, dti, true, 1, 0},
                  {"probs_misspeculated", dp, dt, false, 0, 1}};
  std::vector<uint16_t> c2(cbytes / 2), c6(cbytes / 2);
  std::vector<int64_t> m2(C * C), m6(C * C);
  for (const Case& cs : cases) {
    CK(hipMemset(codes2, 0xAB, cbytes)); CK(hipMemset(codes6, 0xCD, cbytes));
    CK(hipMemset(cm2, 0, (size_t)C * C * 8)); CK(hipMemset(cm6, 0, (size_t)C * C * 8));
    set_mode(cs.true_mode);
    run2(cs.x, cs.t, cs.ign);
    CK(hipDeviceSynchronize());
    set_mode(cs.spec_mode);
    CK(hipMemset(slow_cnt, 0, 8));
    run6(cs.x, cs.t, cs.ign);
    CK(hipDeviceSynchronize());
    int hm[2], hc[2]; CK(hipMemcpy(hm, mode, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(hc, slow_cnt, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c2.data(), codes2, cbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(c6.data(), codes6, cbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m2.data(), cm2, (size_t)C * C * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(m6.data(), cm6, (size_t)C * C * 8, hipMemcpyDeviceToHost));
    int64_t diff = 0, diff_gt1 = 0, flagdiff = 0, cmdiff = 0;
    for (int c = 0; c < C; ++c)
      for (int64_t r = 0; r < N; ++r) {
        const uint16_t a = c2[c * n_pad + r], b = c6[c * n_pad + r];
        if (a == b || ((a & 0x8000) && (b & 0x8000))) continue;  // both skipped: equivalent
        ++diff;
        if ((a & 0xC000) != (b & 0xC000)) ++flagdiff;
        else if (std::abs((int)(a & 0x3FFF) - (int)(b & 0x3FFF)) > 1) ++diff_gt1;
      }
    for (int64_t i = 0; i < (int64_t)C * C; ++i) cmdiff += m2[i] != m6[i];
    printf(", \"%s\": {\"code_diffs\": %lld, \"code_diffs_gt1\": %lld, \"flag_diffs\": %lld, \"confmat_diffs\": %lld, \"verdict\": %d, "
           "\"slow_rows\": [%d, %d]}",
           cs.name, (long long)diff, (long long)diff_gt1, (long long)flagdiff, (long long)cmdiff, hm[1], hc[0], hc[1]);
  }
  // timing (logits, correct speculation).  The library resets the slow-row counts in the class pass.
  set_mode(1);
  float t2 = time_us([&] { run2(d, dt, false); });
  float t6 = time_us([&] { reset_counts(); row6(d, dt, false, false); });
  float t6r = time_us([&] { reset_counts(); row6(d, dt, false, true); });
  float t6seq = time_us([&] { reset_counts(); run6(d, dt, false); });
  float t_ms = time_us([&] { reset_counts(); });
  set_mode(0);
  float t2p = time_us([&] { run2(dp, dt, false); });
  float t6p = time_us([&] { reset_counts(); row6(dp, dt, false, false); });
  float t_hist = time_us([&] {
    hipLaunchKernelGGL(class_hist_kernel, C, 512, kCodes * 4, 0, (const uint16_t*)codes6, n_pad, 1, hist, (int*)nullptr, (int*)nullptr); });
  CK(hipDeviceSynchronize());
  printf(", \"v2_rowpass_logits_us\": %.1f, \"rowpass_logits_us\": %.1f, \"rowpass_logits_record_us\": %.1f, "
         "\"rowpass_seq_incl_fixup_slow_us\": %.1f, \"memset_us\": %.1f, \"v2_rowpass_probs_us\": %.1f, \"rowpass_probs_us\": %.1f, "
         "\"class_hist_us\": %.1f, \"rowpass_gbps\": %.0f}\n",
         t2, t6 - t_ms, t6r - t_ms, t6seq - t_ms, t_ms, t2p, t6p - t_ms, t_hist, (double)(xbytes + cbytes) / ((t6 - t_ms) * 1e3));
  return 0;
}
