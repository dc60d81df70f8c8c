// Row pass with positive booking (round 5): time the library row pass (lean softmax tile) with and without the
// PosSink booking, built with -DTMX_POS_ABL=0/1/2 for the ablations (1: no global booking, 2: no range words).
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc [-DTMX_POS_ABL=k] tools/kexp/rowpass_pos_exp.hip -o build/kexp_r5/rowpass_pos_exp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }

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
  const int64_t N = 65536;
  const int C = 1000;
  std::vector<uint16_t> h(N * C);
  std::vector<int64_t> ht(N);
  srand(9);
  for (int64_t i = 0; i < N * C; ++i) {
    float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
    h[i] = f2bf(2.f * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2));
  }
  for (int64_t i = 0; i < N; ++i) ht[i] = rand() % C;
  __hip_bfloat16* dx; int64_t *dt, *hist, *cm; uint32_t* codes; int *mode, *rows, *state, *err, *rng; float4* stats;
  CK(hipMalloc(&dx, N * C * 2)); CK(hipMalloc(&dt, N * 8)); CK(hipMalloc(&codes, (size_t)C * N * 2));
  CK(hipMalloc(&hist, (size_t)C * 2 * kCodes * 8)); CK(hipMalloc(&cm, (size_t)C * C * 8)); CK(hipMalloc(&mode, 8)); CK(hipMalloc(&rows, 2 * N * 4));
  CK(hipMalloc(&state, 24)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&rng, C * 8)); CK(hipMalloc(&stats, N * 16));
  CK(hipMemcpy(dx, h.data(), N * C * 2, hipMemcpyHostToDevice)); CK(hipMemcpy(dt, ht.data(), N * 8, hipMemcpyHostToDevice));
  int hm[2] = {1, 1};
  CK(hipMemcpy(mode, hm, 8, hipMemcpyHostToDevice)); CK(hipMemset(state, 0, 24)); CK(hipMemset(hist, 0, (size_t)C * 2 * kCodes * 8));
  std::vector<int> r(2 * C);
  for (int c = 0; c < C; ++c) { r[2 * c] = kCodes; r[2 * c + 1] = -1; }
  CK(hipMemcpy(rng, r.data(), C * 8, hipMemcpyHostToDevice));
  const int grid = (int)((N / kTileRows + 7) / 8 * 8);
  const size_t shm = (size_t)1024 * kSlots * 4;
  auto run = [&](bool book) {
    const PosSink pos = book ? PosSink{hist, nullptr, rng, nullptr} : PosSink{};
    hipLaunchKernelGGL((mc_codes_kernel<__hip_bfloat16, false, 2, false>), grid, kRowThreads, shm, 0, dx, dt, N, C, C, mode, -100, false,
                       codes, N, cm, err, true, rows, state, stats, pos);
  };
  float a = 0, b = 0;
  for (int rep = 0; rep < 3; ++rep) { a += time_us([&] { run(false); }); b += time_us([&] { run(true); }); }
  printf("{\"abl\": %d, \"rowpass_us\": {\"flag\": %.2f, \"book\": %.2f}}\n", TMX_POS_ABL, a / 3, b / 3);
  return 0;
}
