// Expected mutual information (K30) for adjusted mutual information, fp64 on gfx950.
//
// Reference: functional/clustering/adjusted_mutual_info_score.py:64-121 (sklearn's _expected_mutual_info_fast port):
// a triple Python loop over (row cluster i, column cluster j, n_ij), one scalar tensor op per term.  Here one 64-lane
// wave owns a (i, j) pair and its lanes stride over n_ij in [max(1, a_i + b_j - N), min(a_i, b_j)]; each term is
//     n_ij / N * (log(N n_ij) - log a_i - log b_j)
//       * exp(lgamma(a_i+1) + lgamma(b_j+1) + lgamma(N-a_i+1) + lgamma(N-b_j+1) - lgamma(N+1)
//             - lgamma(n_ij+1) - lgamma(a_i-n_ij+1) - lgamma(b_j-n_ij+1) - lgamma(N-a_i-b_j+n_ij+1)).
// The pair sums land in a [R * K] buffer that the host reduces in a fixed order (deterministic result).
#include "common.h"

namespace tmx {
namespace {

constexpr int kEmiBlock = 256;

__global__ __launch_bounds__(kEmiBlock) void emi_kernel(const double* __restrict__ a, const double* __restrict__ b, int R, int K,
                                                        double n, double* __restrict__ pair_sum) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t pairs = (int64_t)R * K;
  const int64_t waves = (int64_t)gridDim.x * (kEmiBlock / kWave);
  const double lg_n1 = lgamma(n + 1.0), log_n = log(n);
  for (int64_t pq = (int64_t)blockIdx.x * (kEmiBlock / kWave) + threadIdx.x / kWave; pq < pairs; pq += waves) {
    const double ai = a[pq / K], bj = b[pq % K];
    const double lo = fmax(1.0, ai + bj - n), hi = fmin(ai, bj);
    const double fixed = lgamma(ai + 1.0) + lgamma(bj + 1.0) + lgamma(n - ai + 1.0) + lgamma(n - bj + 1.0) - lg_n1;
    const double lab = log(ai) + log(bj);
    double s = 0.0;
    for (double nij = lo + lane; nij <= hi; nij += kWave) {
      const double gln = fixed - lgamma(nij + 1.0) - lgamma(ai - nij + 1.0) - lgamma(bj - nij + 1.0) - lgamma(n - ai - bj + nij + 1.0);
      s += nij / n * (log_n + log(nij) - lab) * exp(gln);
    }
    s = wave_sum(s);
    if (lane == 0) pair_sum[pq] = s;
  }
}

}  // namespace

// a: fp64 [R] row marginals, b: fp64 [K] column marginals; returns the fp64 EMI scalar
at::Tensor expected_mutual_info(const at::Tensor& a, const at::Tensor& b, double n_samples) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kDouble && b.scalar_type() == at::kDouble,
              "expected_mutual_info: fp64 marginals on the GPU");
  TORCH_CHECK(a.dim() == 1 && b.dim() == 1 && a.is_contiguous() && b.is_contiguous(), "expected_mutual_info: 1-D marginals");
  c10::DeviceGuard guard(a.device());
  const int R = static_cast<int>(a.numel()), K = static_cast<int>(b.numel());
  auto pair_sum = at::zeros({(int64_t)R * K}, a.options());
  if ((int64_t)R * K > 0) {
    const int64_t need = ((int64_t)R * K + kEmiBlock / kWave - 1) / (kEmiBlock / kWave);
    const int grid = static_cast<int>(std::min<int64_t>(need, 256 * 16));
    hipLaunchKernelGGL(emi_kernel, grid, kEmiBlock, 0, stream(), a.data_ptr<double>(), b.data_ptr<double>(), R, K, n_samples,
                       pair_sum.data_ptr<double>());
    TMX_LAUNCH_CHECK();
  }
  return pair_sum.sum();
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("expected_mutual_info(Tensor a, Tensor b, float n_samples) -> Tensor"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("expected_mutual_info", &tmx::expected_mutual_info); }
