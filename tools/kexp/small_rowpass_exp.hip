// (Variant C/D kernel removed from the header after this experiment: not faster.)
// Small-class row pass (C <= 16, one lane per row) at 1M x 10 bf16 logits: the production one-wave-workgroup kernel
// (8192 workgroups of 64 threads, profiles/pmc_small_class_c10_r3.json: 43 us for 21 MB in + 21 MB out) against
// (B) the same without the end-of-block mode-witness atomic and (C, D) four independent waves per 256-thread
// workgroup (wave-level ordering only; 4x fewer workgroups).  Codes and confusion-matrix partials must agree.
// Build: hipcc -O3 --offload-arch=gfx950 -I csrc tools/kexp/small_rowpass_exp.hip -o build/small_rowpass_exp
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "curve_hist_kernels.h"

using namespace tmx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

__global__ void init_logits(__hip_bfloat16* x, int64_t total, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    float u = ((h & 0xFFFF) + (h >> 16)) / 65536.f - 1.f;
    x[i] = __float2bfloat16(2.5f * u);
  }
}
__global__ void init_target(int64_t* t, int64_t n, int C, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    t[i] = h % C;
  }
}

template <typename F>
float time_us(F f, int iters = 30) {
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
  const int64_t N = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int C = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t n_pad = (N + kSmallRows - 1) / kSmallRows * kSmallRows;
  const int64_t ntiles = n_pad / kSmallRows;
  __hip_bfloat16* x;
  int64_t *t, *cm;
  uint16_t *codesA, *codesC;
  uint32_t *pcmA, *pcmC;
  int *mode, *err, *rows, *state;
  CK(hipMalloc(&x, N * C * 2)); hipLaunchKernelGGL(init_logits, 4096, 256, 0, 0, x, N * C, 99u);
  CK(hipMalloc(&t, N * 8)); hipLaunchKernelGGL(init_target, 256, 256, 0, 0, t, N, C, 7u);
  CK(hipMalloc(&cm, C * C * 8)); CK(hipMalloc(&codesA, C * n_pad * 2)); CK(hipMalloc(&codesC, C * n_pad * 2));
  const int gridA = (int)std::min<int64_t>(ntiles, 8192), gridC = 2048, gridD = 1024;
  CK(hipMalloc(&pcmA, (size_t)gridA * C * C * 4)); CK(hipMalloc(&pcmC, (size_t)gridA * C * C * 4));
  CK(hipMalloc(&mode, 8)); CK(hipMalloc(&err, 4)); CK(hipMalloc(&rows, 2 * N * 4)); CK(hipMalloc(&state, 8));
  CK(hipMemset(mode, 0, 8)); CK(hipMemset(state, 0, 8)); CK(hipMemset(err, 0, 4));
  int m1[2] = {1, 0}; CK(hipMemcpy(mode, m1, 8, hipMemcpyHostToDevice));
  const size_t shmA = (size_t)kSmallRows * C * 2 + (size_t)C * C * 4, shmC = 4 * (size_t)kSmallRows * C * 2 + (size_t)C * C * 4;
  auto A = [&](bool rec) {
    hipLaunchKernelGGL((mc_codes_small_kernel<__hip_bfloat16, 1, false>), gridA, kSmallRows, shmA, 0, x, t, N, C, mode, -1, false, codesA,
                       n_pad, cm, err, rec, rows, state, pcmA);
  };
  auto Cw = [&](int grid) {
    hipLaunchKernelGGL((mc_codes_small_w4_kernel<__hip_bfloat16, 1, false>), grid, 256, shmC, 0, x, t, N, C, mode, -1, false, codesC,
                       n_pad, cm, err, true, rows, state, pcmC);
  };
  A(true); Cw(gridC);
  CK(hipDeviceSynchronize());
  std::vector<uint16_t> ca(C * n_pad), cc(C * n_pad);
  CK(hipMemcpy(ca.data(), codesA, C * n_pad * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(cc.data(), codesC, C * n_pad * 2, hipMemcpyDeviceToHost));
  int64_t cd = 0;
  for (size_t i = 0; i < ca.size(); ++i) cd += ca[i] != cc[i];
  std::vector<uint32_t> pa((size_t)gridA * C * C), pc((size_t)gridC * C * C);
  CK(hipMemcpy(pa.data(), pcmA, pa.size() * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(pc.data(), pcmC, pc.size() * 4, hipMemcpyDeviceToHost));
  std::vector<int64_t> sa(C * C, 0), sc(C * C, 0);
  for (size_t i = 0; i < pa.size(); ++i) sa[i % (C * C)] += pa[i];
  for (size_t i = 0; i < pc.size(); ++i) sc[i % (C * C)] += pc[i];
  int64_t md = 0, tot = 0;
  for (int i = 0; i < C * C; ++i) { md += sa[i] != sc[i]; tot += sa[i]; }
  const float tA = time_us([&](int) { A(true); });
  const float tB = time_us([&](int) { A(false); });
  const float tC = time_us([&](int) { Cw(gridC); });
  const float tD = time_us([&](int) { Cw(gridD); });
  printf("{\"N\": %lld, \"C\": %d, \"code_diffs\": %lld, \"confmat_diffs\": %lld, \"confmat_total\": %lld, \"A_prod_us\": %.2f, "
         "\"B_no_mode_atomic_us\": %.2f, \"C_w4_2048_us\": %.2f, \"D_w4_1024_us\": %.2f}\n",
         (long long)N, C, (long long)cd, (long long)md, (long long)tot, tA, tB, tC, tD);
  return 0;
}
