// Host-side audio kernels: Levinson Toeplitz solver (CPU twin of csrc/audio.hip) and a batched Hungarian
// assignment solver for permutation-invariant training (replaces scipy's
// linear_sum_assignment, parallel over the batch).
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <cmath>
#include <limits>
#include <vector>

namespace tmx {
namespace {

void levinson(const double* rs, const double* bs, int64_t L, double* x) {
  std::vector<double> r(L), y(L, 0.0);
  const double r0 = rs[0];
  for (int64_t i = 0; i < L; ++i) {
    r[i] = rs[i] / r0;
    x[i] = 0.0;
  }
  double beta = 1.0, alpha = L > 1 ? -r[1] : 0.0;
  x[0] = bs[0] / r0;
  if (L > 1) y[0] = -r[1];
  for (int64_t k = 1; k < L; ++k) {
    beta = (1.0 - alpha * alpha) * beta;
    double s = 0.0;
    for (int64_t i = 0; i < k; ++i) s += r[i + 1] * x[k - 1 - i];
    const double mu = (bs[k] / r0 - s) / beta;
    for (int64_t i = 0; i < k; ++i) x[i] += mu * y[k - 1 - i];
    x[k] = mu;
    if (k < L - 1) {
      s = 0.0;
      for (int64_t i = 0; i < k; ++i) s += r[i + 1] * y[k - 1 - i];
      alpha = (-r[k + 1] - s) / beta;
      for (int64_t i = 0; i < (k + 1) / 2; ++i) {
        const int64_t j = k - 1 - i;
        const double yi = y[i], yj = y[j];
        if (i == j) {
          y[i] = yi + alpha * yi;
        } else {
          y[i] = yi + alpha * yj;
          y[j] = yj + alpha * yi;
        }
      }
      y[k] = alpha;
    }
  }
}

// Hungarian algorithm (shortest augmenting path with potentials), minimising cost; n x n, O(n^3).
// Returns col_of_row.
std::vector<int64_t> hungarian(const double* cost, int64_t n) {
  const double inf = std::numeric_limits<double>::infinity();
  std::vector<double> u(n + 1, 0.0), v(n + 1, 0.0), minv(n + 1);
  std::vector<int64_t> p(n + 1, 0), way(n + 1, 0);
  std::vector<char> used(n + 1);
  for (int64_t i = 1; i <= n; ++i) {
    p[0] = i;
    int64_t j0 = 0;
    std::fill(minv.begin(), minv.end(), inf);
    std::fill(used.begin(), used.end(), 0);
    do {
      used[j0] = 1;
      const int64_t i0 = p[j0];
      double delta = inf;
      int64_t j1 = 0;
      for (int64_t j = 1; j <= n; ++j) {
        if (used[j]) continue;
        const double cur = cost[(i0 - 1) * n + (j - 1)] - u[i0] - v[j];
        if (cur < minv[j]) {
          minv[j] = cur;
          way[j] = j0;
        }
        if (minv[j] < delta) {
          delta = minv[j];
          j1 = j;
        }
      }
      for (int64_t j = 0; j <= n; ++j) {
        if (used[j]) {
          u[p[j]] += delta;
          v[j] -= delta;
        } else {
          minv[j] -= delta;
        }
      }
      j0 = j1;
    } while (p[j0] != 0);
    do {
      const int64_t j1 = way[j0];
      p[j0] = p[j1];
      j0 = j1;
    } while (j0);
  }
  std::vector<int64_t> col_of_row(n);
  for (int64_t j = 1; j <= n; ++j) col_of_row[p[j] - 1] = j - 1;
  return col_of_row;
}

}  // namespace

at::Tensor toeplitz_solve_cpu(const at::Tensor& r_in, const at::Tensor& b_in) {
  TORCH_CHECK(r_in.sizes() == b_in.sizes(), "toeplitz_solve: r and b must have the same shape");
  const int64_t L = r_in.size(-1);
  auto r = r_in.to(at::kDouble).reshape({-1, L}).contiguous();
  auto b = b_in.to(at::kDouble).reshape({-1, L}).contiguous();
  auto x = at::empty_like(b);
  const double* pr = r.data_ptr<double>();
  const double* pb = b.data_ptr<double>();
  double* px = x.data_ptr<double>();
  at::parallel_for(0, r.size(0), 1, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) levinson(pr + i * L, pb + i * L, L, px + i * L);
  });
  return x.reshape(b_in.sizes());
}

// metric [B, S, S] (rows = target speaker, cols = predicted speaker) -> perm [B, S] (pred index for each target),
// maximising (or minimising) the summed metric.
at::Tensor linear_assignment(const at::Tensor& metric, bool maximize) {
  TORCH_CHECK(metric.dim() == 3 && metric.size(1) == metric.size(2), "linear_assignment: expected [B, S, S]");
  // NaN = worst score, +-inf = large finite (an all-infinite row would otherwise leave no finite slack to augment on)
  constexpr double kBig = 1e150;
  auto m = at::nan_to_num(metric.detach().to(at::kCPU).to(at::kDouble), maximize ? -kBig : kBig, kBig, -kBig).contiguous();
  const int64_t B = m.size(0), S = m.size(1);
  auto out = at::empty({B, S}, at::kLong);
  const double* pm = m.data_ptr<double>();
  int64_t* po = out.data_ptr<int64_t>();
  at::parallel_for(0, B, 8, [&](int64_t s, int64_t e) {
    std::vector<double> cost(S * S);
    for (int64_t b = s; b < e; ++b) {
      for (int64_t k = 0; k < S * S; ++k) cost[k] = maximize ? -pm[b * S * S + k] : pm[b * S * S + k];
      const auto col = hungarian(cost.data(), S);
      for (int64_t i = 0; i < S; ++i) po[b * S + i] = col[i];
    }
  });
  return out.to(metric.device());
}

at::Tensor iir_filter_cpu(const at::Tensor& x_in, const at::Tensor& b_in, const at::Tensor& a_in) {
  TORCH_CHECK(x_in.dim() == 2 && b_in.dim() == 2 && a_in.sizes() == b_in.sizes() && b_in.size(0) == x_in.size(0),
              "iir_filter: expected x [C, T], b / a [C, K]");
  auto x = x_in.to(at::kDouble).contiguous();
  auto b = b_in.to(at::kDouble).contiguous();
  auto a = a_in.to(at::kDouble).contiguous();
  const int64_t C = x.size(0), T = x.size(1), K = b.size(1);
  auto y = at::empty_like(x);
  const double* px = x.data_ptr<double>();
  const double* pb = b.data_ptr<double>();
  const double* pa = a.data_ptr<double>();
  double* py = y.data_ptr<double>();
  at::parallel_for(0, C, 1, [&](int64_t s, int64_t e) {
    std::vector<double> bb(K), aa(K);
    for (int64_t c = s; c < e; ++c) {
      const double a0 = pa[c * K];
      for (int64_t k = 0; k < K; ++k) {
        bb[k] = pb[c * K + k] / a0;
        aa[k] = pa[c * K + k] / a0;
      }
      const double* xc = px + c * T;
      double* yc = py + c * T;
      for (int64_t n = 0; n < T; ++n) {
        double acc = 0.0;
        for (int64_t k = 0; k < K && k <= n; ++k) acc += bb[k] * xc[n - k];
        for (int64_t k = 1; k < K && k <= n; ++k) acc -= aa[k] * yc[n - k];
        yc[n] = acc;
      }
    }
  });
  return y;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("toeplitz_solve(Tensor r, Tensor b) -> Tensor");
  m.def("linear_assignment(Tensor metric, bool maximize) -> Tensor");
  m.def("iir_filter(Tensor x, Tensor b, Tensor a) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CPU, m) {
  m.impl("toeplitz_solve", &tmx::toeplitz_solve_cpu);
  m.impl("iir_filter", &tmx::iir_filter_cpu);
}

TORCH_LIBRARY_IMPL(tmx, CompositeExplicitAutograd, m) { m.impl("linear_assignment", &tmx::linear_assignment); }
