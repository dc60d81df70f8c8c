// Standalone harness for the single-launch persistent multiclass histogram update (csrc/curve_persist.h) against
// the two-pass library sequence (row pass, FIXUP, class pass of csrc/curve_hist_kernels.h), no torch.
// Both compute the same codes with the same arithmetic, so histograms, confusion matrices, code ranges, verdicts and
// the rolled mode words must be IDENTICAL on every case (logits, NaN / inf / tied rows, ignore_index, probabilities
// with and without NaN, both mis-speculations); then both are timed on a pool of 4 distinct batches (cold inputs, as
// bench.py cycles them).
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc -I tools/kexp tools/kexp/persist_exp.hip -o build/persist_exp
// Run:   build/persist_exp [N] [C]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "curve_persist.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 65536;
  const int C = argc > 2 ? atoi(argv[2]) : 1000;
  if (C % 8 != 0 || C > 1024 || C <= 512) { printf("{\"error\": \"harness covers 512 < C <= 1024, C %% 8 == 0\"}\n"); return 1; }
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int tpw_min = argc > 3 ? atoi(argv[3]) : 1;
  const PersistPlan pl = persist_plan(N, C, cus, tpw_min);
  if (!pl.ok) { printf("{\"error\": \"no persistent plan\"}\n"); return 1; }
  auto kprod = mc_persist_producer<__hip_bfloat16, 2>;
  auto kcons = mc_persist_consumer<__hip_bfloat16>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kcons), hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPConsumerLds));
  int nb = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kcons, kCThreads, kPConsumerLds));
  if (nb < 1) { printf("{\"error\": \"consumer kernel does not fit a CU\"}\n"); return 1; }
  hipStream_t side;
  hipEvent_t evA, evB;
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&evA, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&evB, hipEventDisableTiming));

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
  for (int64_t r = 5; r < N; r += 997) hn[r * C + (r % C)] = 0x7FC0;
  for (int64_t r = 11; r < N; r += 1999) hn[r * C + ((r * 7) % C)] = 0x7F80;
  for (int64_t r = 13; r < N; r += 2999) hn[r * C + ((r * 3) % C)] = 0xFF80;
  for (int64_t r = 17; r < N; r += 4001) for (int c = 0; c < C; ++c) hn[r * C + c] = 0xFF80;
  for (int64_t r = 23; r < N; r += 503) hn[r * C + 3] = hn[r * C + 1] = 0x4300;
  for (int64_t r = 7; r < N; r += 1511) hpn[r * C + (r % C)] = 0x7FC0;
  // one class with a constant score in every row: its negative bin holds N - (#positives) counts (u16 wrap path)
  std::vector<uint16_t> hc = hp;
  for (int64_t r = 0; r < N; ++r) hc[r * C + 7] = 0x3F00;  // 0.5

  const size_t xbytes = (size_t)N * C * 2, hbytes = (size_t)C * 2 * kCodes * 8, cbytes = (size_t)C * n_pad * 2;
  __hip_bfloat16 *d, *dp, *dn, *dpn, *dc;
  int64_t *dt, *dti, *histA, *histB, *cmA, *cmB;
  int *msA, *msB, *err, *rowsA, *rowsB, *crA, *crB;
  uint32_t *codesA, *codesB;
  uint16_t* pos;
  long long* prof = nullptr;
  const int PW = 4 * kPMaxChunks + 4;
  CK(hipMalloc(&d, xbytes)); CK(hipMalloc(&dp, xbytes)); CK(hipMalloc(&dn, xbytes)); CK(hipMalloc(&dpn, xbytes)); CK(hipMalloc(&dc, xbytes));
  CK(hipMalloc(&dt, N * 8)); CK(hipMalloc(&dti, N * 8));
  CK(hipMalloc(&histA, hbytes)); CK(hipMalloc(&histB, hbytes)); CK(hipMalloc(&cmA, (size_t)C * C * 8)); CK(hipMalloc(&cmB, (size_t)C * C * 8));
  CK(hipMalloc(&msA, 512)); CK(hipMalloc(&msB, 512)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&rowsA, 2 * N * 4)); CK(hipMalloc(&rowsB, 2 * N * 4));
  CK(hipMalloc(&crA, C * 8)); CK(hipMalloc(&crB, C * 8)); CK(hipMalloc(&codesA, cbytes)); CK(hipMalloc(&codesB, cbytes)); CK(hipMalloc(&pos, N * 2));
  CK(hipMemcpy(d, h.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dp, hp.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dn, hn.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dpn, hpn.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, hc.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), N * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dti, hti.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(msA, 0, 512)); CK(hipMemset(msB, 0, 512)); CK(hipMemset(err, 0, 4));

  const int grid6 = (int)((n_pad / kTileRows + 7) / 8 * 8);
  const size_t shm6 = (size_t)1024 * kSlots * 4;
  // two-pass sequence (library): mode_state A = {mode[2], state[6]}
  auto seq = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 2, false>), grid6, kRowThreads, shm6, 0, x, t, N, C, C, msA, -100, ign,
                       codesA, n_pad, cmA, err, true, rowsA, msA + 2);
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, true, 2, false>), std::min(grid6, 128), kRowThreads, shm6, 0, x, t, N, C, C, msA,
                       -100, ign, codesA, n_pad, cmA, err, false, rowsA, msA + 2);
    hipLaunchKernelGGL((class_hist_kernel<__hip_bfloat16, false>), C, kClassThreads, kCodes * 4, 0, (const uint16_t*)codesA, n_pad, 1,
                       histA, x, C, t, N, msA, true, rowsA, msA + 2, cmA, crA, msA);
  };
  auto per = [&](const __hip_bfloat16* x, const int64_t* t, bool ign) {
    PersistArgs a;
    a.preds = x; a.target = t; a.n = N; a.n_pad = n_pad; a.C = C; a.k = pl.k; a.G = pl.G; a.nchunks = pl.nchunks; a.tpw = pl.tpw;
    a.mode = msB; a.state = msB + 2; a.ctrl = msB + 8; a.ignore_index = -100; a.has_ignore = ign; a.codes = codesB; a.hist = histB;
    a.confmat = cmB; a.err = err; a.slow_rows = rowsB; a.code_range = crB; a.pos_code = pos; a.prof = prof;
    // consumer on the main (null) stream, producer on a side stream: they share every CU
    CK(hipEventRecord(evA, 0));
    CK(hipStreamWaitEvent(side, evA, 0));
    hipLaunchKernelGGL(kcons, pl.G, kCThreads, kPConsumerLds, 0, a);
    hipLaunchKernelGGL(kprod, pl.G, kPThreads, kPProducerLds, side, a);
    CK(hipEventRecord(evB, side));
    CK(hipStreamWaitEvent(0, evB, 0));
  };
  auto set_mode = [&](int* m, int m0) { int hm[2] = {m0, 0}; CK(hipMemcpy(m, hm, 8, hipMemcpyHostToDevice)); };
  auto reset_range = [&](int* cr) {
    std::vector<int> v(2 * C);
    for (int c = 0; c < C; ++c) { v[2 * c] = kCodes; v[2 * c + 1] = -1; }
    CK(hipMemcpy(cr, v.data(), C * 8, hipMemcpyHostToDevice));
  };

  printf("{\"N\": %lld, \"C\": %d, \"G\": %d, \"k\": %d, \"nchunks\": %d, \"tpw\": %d, \"lds\": [%zu, %zu]", (long long)N, C, pl.G,
         pl.k, pl.nchunks, pl.tpw, kPConsumerLds, kPProducerLds);
  struct Case { const char* name; const __hip_bfloat16* x; const int64_t* t; bool ign; int spec_mode; };
  Case cases[] = {{"logits", d, dt, false, 1}, {"logits_nan_inf_ties", dn, dt, false, 1}, {"logits_ignore", dn, dti, true, 1},
                  {"probs", dp, dt, false, 0}, {"probs_nan", dpn, dt, false, 0}, {"logits_misspeculated", dn, dti, true, 0},
                  {"probs_misspeculated", dp, dt, false, 1}, {"probs_const_class", dc, dt, false, 0}};
  std::vector<int64_t> hA(hbytes / 8), hB(hbytes / 8), mA(C * C), mB(C * C);
  std::vector<int> rA(2 * C), rB(2 * C);
  int all_ok = 1;
  for (const Case& cs : cases) {
    CK(hipMemset(histA, 0, hbytes)); CK(hipMemset(histB, 0, hbytes));
    CK(hipMemset(cmA, 0, (size_t)C * C * 8)); CK(hipMemset(cmB, 0, (size_t)C * C * 8));
    reset_range(crA); reset_range(crB);
    set_mode(msA, cs.spec_mode); set_mode(msB, cs.spec_mode);
    for (int rep = 0; rep < 2; ++rep) {  // twice: the second launch sees the rolled mode and the reset counters
      seq(cs.x, cs.t, cs.ign);
      per(cs.x, cs.t, cs.ign);
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hA.data(), histA, hbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(hB.data(), histB, hbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(mA.data(), cmA, (size_t)C * C * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(mB.data(), cmB, (size_t)C * C * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rA.data(), crA, C * 8, hipMemcpyDeviceToHost)); CK(hipMemcpy(rB.data(), crB, C * 8, hipMemcpyDeviceToHost));
    int wA[8], wB[8 + kPCtrlWords];
    CK(hipMemcpy(wA, msA, 32, hipMemcpyDeviceToHost)); CK(hipMemcpy(wB, msB, (8 + kPCtrlWords) * 4, hipMemcpyDeviceToHost));
    int64_t hd = 0, cd = 0, rd = 0, tot = 0;
    for (size_t i = 0; i < hA.size(); ++i) { hd += hA[i] != hB[i]; tot += hB[i]; }
    for (size_t i = 0; i < mA.size(); ++i) cd += mA[i] != mB[i];
    for (int i = 0; i < 2 * C; ++i) rd += rA[i] != rB[i];
    int ctrl_dirty = 0;
    for (int i = 0; i < kPCtrlWords; ++i) ctrl_dirty += (i != kPCtrlTimeout) && wB[8 + i] != 0;
    const bool ok = hd == 0 && cd == 0 && rd == 0 && wA[0] == wB[0] && wA[1] == wB[1] && wB[2] == 0 && wB[3] == 0 && ctrl_dirty == 0 &&
                    wB[8 + kPCtrlTimeout] == 0;
    all_ok &= ok;
    printf(", \"%s\": {\"hist_diffs\": %lld, \"confmat_diffs\": %lld, \"range_diffs\": %lld, \"total\": %lld, \"mode_seq\": [%d, %d], "
           "\"mode_persist\": [%d, %d], \"counts_persist\": [%d, %d], \"ctrl_dirty\": %d, \"timeout\": %d, \"ok\": %s}",
           cs.name, (long long)hd, (long long)cd, (long long)rd, (long long)tot, wA[0], wA[1], wB[0], wB[1], wB[2], wB[3], ctrl_dirty,
           wB[8 + kPCtrlTimeout], ok ? "true" : "false");
    fflush(stdout);
  }
  // timing on a pool of 4 distinct logits batches (correct speculation)
  __hip_bfloat16* pool[4] = {d, dn, dp, dc};
  CK(hipMemcpy(dn, h.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dp, h.data(), xbytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, h.data(), xbytes, hipMemcpyHostToDevice));
  set_mode(msA, 1); set_mode(msB, 1);
  auto time_us = [&](auto f, int iters) {
    for (int i = 0; i < 4; ++i) f(i);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) f(i);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / iters;
  };
  const float t_seq = time_us([&](int i) { seq(pool[i & 3], dt, false); }, 40);
  const float t_per = time_us([&](int i) { per(pool[i & 3], dt, false); }, 40);
  const float t_per_warm = time_us([&](int) { per(d, dt, false); }, 40);
  // one profiled launch: per-chunk phase times averaged over workgroups (100 MHz wall clock -> us)
  CK(hipMalloc(&prof, (size_t)pl.G * PW * 8));
  CK(hipMemset(prof, 0, (size_t)pl.G * PW * 8));
  per(pool[0], dt, false);
  CK(hipDeviceSynchronize());
  std::vector<long long> hpf((size_t)pl.G * PW);
  CK(hipMemcpy(hpf.data(), prof, hpf.size() * 8, hipMemcpyDeviceToHost));
  long long t0 = hpf[0];
  for (int g = 0; g < pl.G; ++g) t0 = std::min(t0, hpf[(size_t)g * PW]);
  printf(", \"phases_us\": [");
  for (int s = 0; s < pl.nchunks; ++s) {
    double ps = 0, pe = 0, we = 0, ce = 0, pemax = 0, cemax = 0;
    for (int g = 0; g < pl.G; ++g) {
      const long long* q = &hpf[(size_t)g * PW + 4 * s];
      ps += (q[0] - t0) / 100.0; pe += (q[1] - t0) / 100.0; we += (q[2] - t0) / 100.0; ce += (q[3] - t0) / 100.0;
      pemax = std::max(pemax, (q[1] - t0) / 100.0); cemax = std::max(cemax, (q[3] - t0) / 100.0);
    }
    printf("%s{\"prod_start\": %.1f, \"prod_end\": %.1f, \"prod_end_max\": %.1f, \"wait_end\": %.1f, \"cons_end\": %.1f, \"cons_end_max\": %.1f}",
           s ? ", " : "", ps / pl.G, pe / pl.G, pemax, we / pl.G, ce / pl.G, cemax);
  }
  double e0 = 0, e1 = 0;
  for (int g = 0; g < pl.G; ++g) { e0 += (hpf[(size_t)g * PW + 4 * kPMaxChunks] - t0) / 100.0; e1 = std::max(e1, (hpf[(size_t)g * PW + 4 * kPMaxChunks + 1] - t0) / 100.0); }
  printf("]");
#if TMX_PERSIST_TILE_PROF
  printf(", \"tiles_us\": [");
  for (int j = 0; j < pl.tpw && j < kPMaxChunks; ++j) {
    double w0 = 0, c1 = 0, s2 = 0;
    for (int g = 0; g < pl.G; ++g) {
      const long long* q = &hpf[(size_t)g * PW + 4 * j];
      w0 += (q[0] - t0) / 100.0; c1 += (q[1] - q[0]) / 100.0; s2 += (q[2] - q[1]) / 100.0;
    }
    printf("%s{\"loads_done\": %.2f, \"codes\": %.2f, \"store_tile\": %.2f}", j ? ", " : "", w0 / pl.G, c1 / pl.G, s2 / pl.G);
  }
  printf("]");
#endif
  printf(", \"end_start_avg\": %.1f, \"end_done_max\": %.1f", e0 / pl.G, e1);
  int wB[8 + kPCtrlWords];
  CK(hipMemcpy(wB, msB, (8 + kPCtrlWords) * 4, hipMemcpyDeviceToHost));
  printf(", \"two_pass_us\": %.1f, \"persist_us\": %.1f, \"persist_same_batch_us\": %.1f, \"timeout_after_timing\": %d, \"all_ok\": %s}\n",
         t_seq, t_per, t_per_warm, wB[8 + kPCtrlTimeout], all_ok ? "true" : "false");
  return 0;
}
