// Headline update, sequential vs overlapped (round 5): the row pass of batch k+1 (VALU-heavy, ~4 TB/s) on one stream
// while the class pass of batch k (memory / LDS-bound) runs on a second stream, with two code scratches.  The class
// pass's 32 KiB workgroups fit beside two 64 KiB row-pass workgroups on a CU (160 KiB of LDS).  Measures the time per
// update of each schedule over 40 updates (4 distinct logit batches cycled), and checks the accumulated histograms of
// the two schedules are identical.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/overlap_exp.hip -o build/kexp_r5/overlap_exp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }

// the library row pass with a VGPR cap (ROWCAP waves per SIMD): a class-pass wave then fits on a SIMD beside four
// row-pass waves (512 VGPRs per SIMD lane)
#ifndef ROWCAP
#define ROWCAP 4
#endif
__global__ void __launch_bounds__(kRowThreads) __attribute__((amdgpu_waves_per_eu(ROWCAP))) row_capped(
    const __hip_bfloat16* __restrict__ preds, const int64_t* __restrict__ target, int64_t n, int C, int ld, int* __restrict__ mode,
    int64_t ignore_index, bool has_ignore, uint32_t* __restrict__ codes, int64_t n_pad, int64_t* __restrict__ confmat, int* __restrict__ err,
    bool record_mode, int* __restrict__ slow_rows, int* __restrict__ slow_count, float4* __restrict__ row_stats) {
  mc_codes_block<__hip_bfloat16, false, 2, false>(blockIdx.x, gridDim.x, preds, target, n, C, ld, mode, ignore_index, has_ignore, codes, n_pad,
                                                  confmat, err, record_mode, slow_rows, slow_count, row_stats);
}

int main(int argc, char** argv) {
  const int64_t N = 65536;
  const int C = 1000;
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  const int64_t n_pad = N;
  const int NB = 4;
  std::vector<uint16_t> h(N * C);
  std::vector<int64_t> ht(N);
  __hip_bfloat16* dx[NB];
  int64_t* dt[NB];
  const size_t xbytes = (size_t)N * C * 2, cbytes = (size_t)C * n_pad * 2, hbytes = (size_t)C * 2 * kCodes * 8;
  srand(5);
  for (int b = 0; b < NB; ++b) {
    for (int64_t i = 0; i < N * C; ++i) {
      float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
      h[i] = f2bf(2.f * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2));
    }
    for (int64_t i = 0; i < N; ++i) ht[i] = rand() % C;
    CK(hipMalloc(&dx[b], xbytes)); CK(hipMalloc(&dt[b], N * 8));
    CK(hipMemcpy(dx[b], h.data(), xbytes, hipMemcpyHostToDevice)); CK(hipMemcpy(dt[b], ht.data(), N * 8, hipMemcpyHostToDevice));
  }
  uint32_t* codes[2]; int* rows[2]; int* state[2]; int* mode[2];
  for (int s = 0; s < 2; ++s) {
    CK(hipMalloc(&codes[s], cbytes)); CK(hipMalloc(&rows[s], 2 * N * 4)); CK(hipMalloc(&state[s], 24)); CK(hipMalloc(&mode[s], 8));
    CK(hipMemset(state[s], 0, 24));
    int hm[2] = {1, 1};
    CK(hipMemcpy(mode[s], hm, 8, hipMemcpyHostToDevice));
  }
  int64_t *histS, *histO, *cmS, *cmO; int *rngS, *rngO, *err;
  CK(hipMalloc(&histS, hbytes)); CK(hipMalloc(&histO, hbytes)); CK(hipMalloc(&cmS, (size_t)C * C * 8)); CK(hipMalloc(&cmO, (size_t)C * C * 8));
  CK(hipMalloc(&rngS, C * 8)); CK(hipMalloc(&rngO, C * 8)); CK(hipMalloc(&err, 4));
  const int grid = (int)((n_pad / kTileRows + 7) / 8 * 8);
  const size_t shm = (size_t)1024 * kSlots * 4;
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  std::vector<hipEvent_t> rowDone(iters + 8), clsDone(iters + 8);
  for (auto& ev : rowDone) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : clsDone) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  auto row = [&](int i, hipStream_t s, int slot) {
    hipLaunchKernelGGL(row_capped, grid, kRowThreads, shm, s, dx[i % NB], dt[i % NB], N, C, C,
                       mode[slot], -100, false, codes[slot], n_pad, i % 2 ? cmO : cmS, err, false, rows[slot], state[slot], (float4*)nullptr);
  };
  auto cls = [&](int i, hipStream_t s, int slot, int64_t* hist, int* rng) {
    hipLaunchKernelGGL((class_hist_hi_kernel<__hip_bfloat16>), C, kClassThreadsU16, kHiLdsBytes, s, (const uint16_t*)codes[slot], n_pad, 1,
                       hist, dx[i % NB], C, dt[i % NB], N, mode[slot], false, rows[slot], state[slot], (int64_t*)nullptr, rng,
                       (int*)nullptr, (int64_t*)nullptr, (int*)nullptr, (const float4*)nullptr);
  };
  auto reset = [&] {
    CK(hipMemset(histS, 0, hbytes)); CK(hipMemset(histO, 0, hbytes));
    std::vector<int> r(2 * C);
    for (int c = 0; c < C; ++c) { r[2 * c] = kCodes; r[2 * c + 1] = -1; }
    CK(hipMemcpy(rngS, r.data(), C * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(rngO, r.data(), C * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
  };
  auto seq = [&](int n) {
    for (int i = 0; i < n; ++i) { row(i, sa, 0); cls(i, sa, 0, histS, rngS); }
  };
  auto ovl = [&](int n) {
    for (int i = 0; i < n; ++i) {
      const int slot = i & 1;
      if (i >= 2) CK(hipStreamWaitEvent(sa, clsDone[i - 2], 0));  // the class pass that read this scratch is done
      row(i, sa, slot);
      CK(hipEventRecord(rowDone[i], sa));
      CK(hipStreamWaitEvent(sb, rowDone[i], 0));
      cls(i, sb, slot, histO, rngO);
      CK(hipEventRecord(clsDone[i], sb));
    }
    CK(hipStreamWaitEvent(sa, clsDone[n - 1], 0));
  };
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  auto timed = [&](auto f) {
    reset();
    f(4);  // warm-up
    CK(hipDeviceSynchronize());
    reset();
    CK(hipEventRecord(t0, sa));
    f(iters);
    CK(hipEventRecord(t1, sa));
    CK(hipEventSynchronize(t1));
    float ms; CK(hipEventElapsedTime(&ms, t0, t1));
    return ms * 1000.f / iters;
  };
  float ts[3], to[3];
  for (int r = 0; r < 3; ++r) { ts[r] = timed(seq); to[r] = timed(ovl); }
  reset();
  seq(iters);
  ovl(iters);
  CK(hipDeviceSynchronize());
  std::vector<int64_t> a(hbytes / 8), b(hbytes / 8);
  CK(hipMemcpy(a.data(), histS, hbytes, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), histO, hbytes, hipMemcpyDeviceToHost));
  int64_t diffs = 0, tot = 0;
  for (size_t i = 0; i < a.size(); ++i) { diffs += a[i] != b[i]; tot += a[i]; }
  printf("{\"iters\": %d, \"seq_us_per_update\": [%.2f, %.2f, %.2f], \"overlap_us_per_update\": [%.2f, %.2f, %.2f], \"hist_diffs\": %lld, "
         "\"total_counts\": %lld}\n", iters, ts[0], ts[1], ts[2], to[0], to[1], to[2], (long long)diffs, (long long)tot);
  return diffs == 0 ? 0 : 3;
}
