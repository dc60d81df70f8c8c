// Standalone harness for the exact-histogram kernels (no torch).  Runs the library sequence (mc_codes_kernel, its
// FIXUP launch, class_hist_kernel — which also finishes NaN / inf rows) against the previous one-wave-per-row row
// pass (tools/kexp/curve_hist_v2_ref.h) followed by the same class pass, on logits, logits with NaN / inf / all -inf
// / tied rows, ignore_index rows, probabilities (with and without NaN) and mis-speculated modes (FIXUP path), then
// times the kernels.  Histograms may differ only where v2's reciprocal product and the library's correctly rounded
// quotient round to neighbouring 16-bit codes; the confusion matrix is exact except all -inf rows, which v2 did
// not count and torch.argmax (and the library) put in class 0.
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
  __hip_bfloat16 *d, *dp, *dn, *dpn; int64_t *dt, *dti, *hist2, *hist6, *cm2, *cm6; int *mode, *mode2, *err, *slow_rows, *state, *state2;
  uint32_t *codes2, *codes6;
  const size_t cbytes = (size_t)C * n_pad * 2, xbytes = (size_t)N * C * 2, hbytes = (size_t)C * 2 * kCodes * 8;
  CK(hipMalloc(&d, xbytes)); CK(hipMalloc(&dp, xbytes)); CK(hipMalloc(&dn, xbytes)); CK(hipMalloc(&dpn, xbytes));
  CK(hipMalloc(&dt, N * 8)); CK(hipMalloc(&dti, N * 8));
  CK(hipMalloc(&hist2, hbytes)); CK(hipMalloc(&hist6, hbytes)); CK(hipMalloc(&cm2, (int64_t)C * C * 8)); CK(hipMalloc(&cm6, (int64_t)C * C * 8));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&mode2, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&codes2, cbytes)); CK(hipMalloc(&codes6, cbytes));
  CK(hipMalloc(&slow_rows, 2 * N * 4)); CK(hipMalloc(&state, 24)); CK(hipMalloc(&state2, 24));
  CK(hipMemcpy(d, h.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dp, hp.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dn, hn.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dpn, hpn.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), N * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dti, hti.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(state, 0, 24)); CK(hipMemset(state2, 0, 24));

  const int grid2 = (int)std::min<int64_t>(n_pad / tmx_ref::kTileRows, 256 * 2);
  const size_t shm2 = (size_t)C * (tmx_ref::kTileRows / 2) * 4;
  const int grid6 = (int)((n_pad / kTileRows + 7) / 8 * 8);
  const size_t shm6 = (size_t)1024 * kSlots * 4;
  auto set_mode = [&](int* m, int m0) { int hm[2] = {m0, 0}; CK(hipMemcpy(m, hm, 8, hipMemcpyHostToDevice)); };
  auto row6 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign, bool rec) {
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 2, false>), grid6, kRowThreads, shm6, 0, x, t, N, C, C, mode, -100, ign,
                       codes6, n_pad, cm6, err, rec, slow_rows, state);
  };
  auto fix6 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, true, 2, false>), std::min(grid6, 128), kRowThreads, shm6, 0, x, t, N, C, C, mode, -100, ign,
                       codes6, n_pad, cm6, err, false, slow_rows, state);
  };
  auto class6 = [&](const __hip_bfloat16* x, const int64_t* t, bool spec) {
    hipLaunchKernelGGL((class_hist_kernel<__hip_bfloat16, false>), C, kClassThreads, kCodes * 4, 0, (const uint16_t*)codes6, n_pad, 1, hist6,
                       x, C, t, N, mode, spec, slow_rows, state, cm6, (int*)nullptr, spec ? mode : (int*)nullptr);
  };
  // reference: v2 row pass (mode given), then the same class pass with no rare-row list
  auto ref2 = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    hipLaunchKernelGGL((tmx_ref::mc_codes_kernel<__hip_bfloat16, false, 0>), grid2, tmx_ref::kA_Threads, shm2, 0, x, t, N, C, mode2,
                       -100, ign, codes2, n_pad, cm2, err, false);
    hipLaunchKernelGGL((class_hist_kernel<__hip_bfloat16, false>), C, kClassThreads, kCodes * 4, 0, (const uint16_t*)codes2, n_pad, 1, hist2,
                       x, C, t, N, mode2, false, slow_rows, state2, (int64_t*)nullptr, (int*)nullptr, (int*)nullptr);
  };

  printf("{\"N\": %lld, \"C\": %d", (long long)N, C);
  struct Case { const char* name; const __hip_bfloat16* x; const int64_t* t; bool ign; int true_mode; int spec_mode; };
  Case cases[] = {{"logits", d, dt, false, 1, 1}, {"logits_nan_inf_ties", dn, dt, false, 1, 1}, {"logits_ignore", dn, dti, true, 1, 1},
                  {"probs", dp, dt, false, 0, 0}, {"probs_nan", dpn, dt, false, 1, 0}, {"logits_misspeculated", dn, dti, true, 1, 0},
                  {"probs_misspeculated", dp, dt, false, 0, 1}};
  std::vector<int64_t> h2(hbytes / 8), h6(hbytes / 8), m2(C * C), m6(C * C);
  for (const Case& cs : cases) {
    CK(hipMemset(hist2, 0, hbytes)); CK(hipMemset(hist6, 0, hbytes));
    CK(hipMemset(cm2, 0, (size_t)C * C * 8)); CK(hipMemset(cm6, 0, (size_t)C * C * 8));
    set_mode(mode2, cs.true_mode);
    ref2(cs.x, cs.t, cs.ign);
    set_mode(mode, cs.spec_mode);
    row6(cs.x, cs.t, cs.ign, true);
    fix6(cs.x, cs.t, cs.ign);
    CK(hipDeviceSynchronize());
    int hm[2], hs[3]; CK(hipMemcpy(hm, mode, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(hs, state, 12, hipMemcpyDeviceToHost));
    const int verdict = hm[1];
    class6(cs.x, cs.t, true);
    CK(hipDeviceSynchronize());
    int hm2[2], hs2[3]; CK(hipMemcpy(hm2, mode, 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(hs2, state, 12, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), hist2, hbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(h6.data(), hist6, hbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m2.data(), cm2, (size_t)C * C * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(m6.data(), cm6, (size_t)C * C * 8, hipMemcpyDeviceToHost));
    int64_t l1 = 0, far = 0, tot2 = 0, tot6 = 0, cmdiff = 0;
    for (int c = 0; c < C; ++c)
      for (int s = 0; s < 2; ++s)
        for (int k = 0; k < kCodes; ++k) {
          const int64_t a = h2[((int64_t)c * 2 + s) * kCodes + k], b = h6[((int64_t)c * 2 + s) * kCodes + k];
          tot2 += a; tot6 += b;
          if (a == b) continue;
          l1 += std::llabs(a - b);
          // a moved code lands in a neighbouring bin: the difference must be matched within +-1 bin
          const int64_t lo = k > 0 ? h6[((int64_t)c * 2 + s) * kCodes + k - 1] - h2[((int64_t)c * 2 + s) * kCodes + k - 1] : 0;
          const int64_t hi = k + 1 < kCodes ? h6[((int64_t)c * 2 + s) * kCodes + k + 1] - h2[((int64_t)c * 2 + s) * kCodes + k + 1] : 0;
          if (lo == 0 && hi == 0) ++far;
        }
    for (int64_t i = 0; i < (int64_t)C * C; ++i) cmdiff += m2[i] != m6[i];
    printf(", \"%s\": {\"hist_l1\": %lld, \"hist_isolated_diffs\": %lld, \"counts\": [%lld, %lld], \"confmat_diffs\": %lld, "
           "\"verdict\": %d, \"rare_rows\": [%d, %d], \"after_class_pass\": {\"mode\": [%d, %d], \"state\": [%d, %d, %d]}}",
           cs.name, (long long)l1, (long long)far, (long long)tot2, (long long)tot6, (long long)cmdiff, verdict, hs[0], hs[1],
           hm2[0], hm2[1], hs2[0], hs2[1], hs2[2]);
  }
  // timing (logits, correct speculation)
  set_mode(mode, 1);
  set_mode(mode2, 1);
  float t2 = time_us([&] {
    hipLaunchKernelGGL((tmx_ref::mc_codes_kernel<__hip_bfloat16, false, 0>), grid2, tmx_ref::kA_Threads, shm2, 0, d, dt, N, C, mode2,
                       -100, false, codes2, n_pad, cm2, err, false); });
  float t6 = time_us([&] { row6(d, dt, false, false); });
  float t6r = time_us([&] { row6(d, dt, false, true); });
  float tfix = time_us([&] { fix6(d, dt, false); });
  float tcls = time_us([&] { class6(d, dt, true); });
  float tseq = time_us([&] { row6(d, dt, false, true); fix6(d, dt, false); class6(d, dt, true); });
  set_mode(mode, 0);
  set_mode(mode2, 0);
  float t2p = time_us([&] {
    hipLaunchKernelGGL((tmx_ref::mc_codes_kernel<__hip_bfloat16, false, 0>), grid2, tmx_ref::kA_Threads, shm2, 0, dp, dt, N, C, mode2,
                       -100, false, codes2, n_pad, cm2, err, false); });
  float t6p = time_us([&] { row6(dp, dt, false, false); });
  CK(hipDeviceSynchronize());
  printf(", \"v2_rowpass_logits_us\": %.1f, \"rowpass_logits_us\": %.1f, \"rowpass_logits_record_us\": %.1f, \"fixup_noop_us\": %.1f, "
         "\"class_pass_us\": %.1f, \"update_sequence_us\": %.1f, \"v2_rowpass_probs_us\": %.1f, \"rowpass_probs_us\": %.1f, "
         "\"rowpass_gbps\": %.0f}\n",
         t2, t6, t6r, tfix, tcls, tseq, t2p, t6p, (double)(xbytes + cbytes) / (t6 * 1e3));
  return 0;
}
