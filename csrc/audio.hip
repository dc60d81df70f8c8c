// Symmetric Toeplitz solver for SDR: Levinson recursion, O(L²) per system instead of the
// reference's O(L³) dense `torch.linalg.solve` on an explicitly built L×L Toeplitz matrix.
//
// T x = b with T = toeplitz(r[0..L-1]) (symmetric, positive definite: an autocorrelation), fp64.
// GPU: one 256-thread block per system; r, b, x and the Durbin vector y live in LDS (L ≤ 2048 → ≤ 48 KB of the
// 160 KB LDS), and every recursion step is two block-wide dot products (64-wide wave shuffles + LDS) and two
// parallel vector updates.  Host: the same recursion in C++ (csrc/audio_host.cpp), parallel over systems.
#include "common.h"

namespace tmx {

constexpr int kLevThreads = 256;
constexpr int kLevMaxL = 2048;  // 3·L fp64 in LDS ≤ 48 KB per block

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kLevThreads / kWave; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(kLevThreads) void levinson_kernel(const double* __restrict__ R, const double* __restrict__ B, int64_t L,
                                                              double* __restrict__ X) {
  extern __shared__ double smem[];
  double* r = smem;          // normalised off-diagonals r[1..L-1] / r[0]
  double* x = r + L;
  double* y = x + L;
  __shared__ double red[kLevThreads / kWave];
  const int64_t sys = blockIdx.x;
  const double* rs = R + sys * L;
  const double* bs = B + sys * L;
  const double r0 = rs[0];
  for (int64_t i = threadIdx.x; i < L; i += kLevThreads) {
    r[i] = rs[i] / r0;
    x[i] = 0.0;
    y[i] = 0.0;
  }
  __syncthreads();
  // 0-based translation of the classic Levinson recursion (unit diagonal)
  double beta = 1.0;
  double alpha = L > 1 ? -r[1] : 0.0;
  if (threadIdx.x == 0) {
    x[0] = bs[0] / r0;
    if (L > 1) y[0] = -r[1];
  }
  __syncthreads();
  for (int64_t k = 1; k < L; ++k) {
    beta = (1.0 - alpha * alpha) * beta;
    // mu = (b[k] - Σ_{i<k} r[i+1] x[k-1-i]) / beta
    double part = 0.0;
    for (int64_t i = threadIdx.x; i < k; i += kLevThreads) part += r[i + 1] * x[k - 1 - i];
    const double mu = (bs[k] / r0 - block_sum(part, red)) / beta;
    for (int64_t i = threadIdx.x; i < k; i += kLevThreads) x[i] += mu * y[k - 1 - i];
    if (threadIdx.x == 0) x[k] = mu;
    __syncthreads();
    if (k < L - 1) {
      part = 0.0;
      for (int64_t i = threadIdx.x; i < k; i += kLevThreads) part += r[i + 1] * y[k - 1 - i];
      alpha = (-r[k + 1] - block_sum(part, red)) / beta;
      // y[i], y[k-1-i] updated as a pair (the update reads the mirrored element)
      for (int64_t i = threadIdx.x; i < (k + 1) / 2; i += kLevThreads) {
        const int64_t j = k - 1 - i;
        const double yi = y[i], yj = y[j];
        if (i == j) {
          y[i] = yi + alpha * yi;
        } else {
          y[i] = yi + alpha * yj;
          y[j] = yj + alpha * yi;
        }
      }
      if (threadIdx.x == 0) y[k] = alpha;
      __syncthreads();
    }
  }
  for (int64_t i = threadIdx.x; i < L; i += kLevThreads) X[sys * L + i] = x[i];
}

at::Tensor toeplitz_solve_cuda(const at::Tensor& r_in, const at::Tensor& b_in) {
  TORCH_CHECK(r_in.is_cuda() && b_in.is_cuda(), "toeplitz_solve: expected GPU tensors");
  TORCH_CHECK(r_in.sizes() == b_in.sizes(), "toeplitz_solve: r and b must have the same shape");
  const at::DeviceGuard guard(r_in.device());
  const int64_t L = r_in.size(-1);
  TORCH_CHECK(L >= 1 && L <= kLevMaxL, "toeplitz_solve: filter length must be in [1, ", kLevMaxL, "]");
  auto r = r_in.to(at::kDouble).reshape({-1, L}).contiguous();
  auto b = b_in.to(at::kDouble).reshape({-1, L}).contiguous();
  auto x = at::empty_like(b);
  const int64_t n = r.size(0);
  if (n == 0) return x.reshape(b_in.sizes());
  const size_t shmem = static_cast<size_t>(3 * L) * sizeof(double);
  hipLaunchKernelGGL(levinson_kernel, dim3(static_cast<unsigned>(n)), dim3(kLevThreads), shmem, stream(), r.data_ptr<double>(),
                     b.data_ptr<double>(), L, x.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return x.reshape(b_in.sizes());
}

// ---------------------------------------------------------------------------------------------------------------
// Per-channel IIR filter (SRMR gammatone and modulation filterbanks): direct form
//   y[n] = (Σ_k b[k] x[n-k] - Σ_{k≥1} a[k] y[n-k]) / a[0]
// One thread per channel walks time sequentially; the signal is laid out time-major [T, C] so a wave's 64
// channels read and write 64 consecutive fp64 values per step (coalesced).  Filter order ≤ 8.
constexpr int kIirMaxOrder = 8;

__global__ __launch_bounds__(256) void iir_kernel(const double* __restrict__ x, const double* __restrict__ b, const double* __restrict__ a,
                                                 int64_t C, int64_t T, int K, double* __restrict__ y) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double bb[kIirMaxOrder], aa[kIirMaxOrder], xh[kIirMaxOrder], yh[kIirMaxOrder];
  const double a0 = a[c * K];
  for (int k = 0; k < K; ++k) {
    bb[k] = b[c * K + k] / a0;
    aa[k] = a[c * K + k] / a0;
    xh[k] = 0.0;
    yh[k] = 0.0;
  }
  for (int64_t n = 0; n < T; ++n) {
    for (int k = K - 1; k > 0; --k) xh[k] = xh[k - 1];
    xh[0] = x[n * C + c];
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += bb[k] * xh[k];
    for (int k = 1; k < K; ++k) acc -= aa[k] * yh[k - 1];
    for (int k = K - 1; k > 0; --k) yh[k] = yh[k - 1];
    yh[0] = acc;
    y[n * C + c] = acc;
  }
}

// x [C, T] fp64, b / a [C, K] -> y [C, T]
at::Tensor iir_filter_cuda(const at::Tensor& x_in, const at::Tensor& b_in, const at::Tensor& a_in) {
  TORCH_CHECK(x_in.is_cuda(), "iir_filter: expected GPU tensors");
  TORCH_CHECK(x_in.dim() == 2 && b_in.dim() == 2 && a_in.sizes() == b_in.sizes() && b_in.size(0) == x_in.size(0),
              "iir_filter: expected x [C, T], b / a [C, K]");
  const int K = static_cast<int>(b_in.size(1));
  TORCH_CHECK(K >= 1 && K <= kIirMaxOrder, "iir_filter: filter length must be in [1, ", kIirMaxOrder, "]");
  const at::DeviceGuard guard(x_in.device());
  auto xt = x_in.to(at::kDouble).t().contiguous();  // [T, C]
  auto b = b_in.to(x_in.device()).to(at::kDouble).contiguous();
  auto a = a_in.to(x_in.device()).to(at::kDouble).contiguous();
  const int64_t C = x_in.size(0), T = x_in.size(1);
  auto yt = at::empty_like(xt);
  if (C == 0 || T == 0) return yt.t().contiguous();
  hipLaunchKernelGGL(iir_kernel, dim3(static_cast<unsigned>((C + 255) / 256)), dim3(256), 0, stream(), xt.data_ptr<double>(),
                     b.data_ptr<double>(), a.data_ptr<double>(), C, T, K, yt.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return yt.t().contiguous();
}

// ---- batched Hungarian assignment for PIT ------------------------------------------------
// One 64-lane workgroup per [S, S] problem (S <= 64): the shortest-augmenting-path Hungarian of the host solver
// (audio_host.cpp ``hungarian``) with the column loop spread over the lanes — lane l owns column l + 1 (its potential
// v, slack minv and used flag in registers), the row potentials u, the matching p and the path ``way`` live in LDS,
// and the per-step arg-min over the free columns is a wave reduction of (slack, column) pairs, lowest column on ties
// (the host loop's strict ``<``).  Same fp64 operations in the same order, so the same assignment as the host solver.
constexpr int kHunLanes = 64;

__global__ __launch_bounds__(kHunLanes) void hungarian_kernel(const double* __restrict__ metric, int S, bool maximize,
                                                              int64_t* __restrict__ col_of_row) {
  __shared__ double u[kHunLanes + 1];
  __shared__ int p[kHunLanes + 1];
  __shared__ int way[kHunLanes + 1];
  const int lane = threadIdx.x;
  const int j = lane + 1;  // column owned by this lane (1-based, column 0 is the virtual root)
  const bool valid = j <= S;
  const double* cost = metric + static_cast<int64_t>(blockIdx.x) * S * S;
  const double inf = __builtin_huge_val();
  for (int k = lane; k <= S; k += kHunLanes) {
    u[k] = 0.0;
    p[k] = 0;
    way[k] = 0;
  }
  double v = 0.0;
  __syncthreads();
  for (int i = 1; i <= S; ++i) {
    if (lane == 0) p[0] = i;
    double minv = inf;
    bool used = false;
    int j0 = 0;
    __syncthreads();
    while (true) {
      if (j == j0) used = true;
      const int i0 = p[j0];
      const double ui0 = u[i0];
      const bool open = valid && !used;
      if (open) {
        const double c = cost[(i0 - 1) * S + lane];
        const double cur = (maximize ? -c : c) - ui0 - v;
        if (cur < minv) {
          minv = cur;
          way[j] = j0;
        }
      }
      // arg-min of the free columns' slack, lowest column on ties
      double best = open ? minv : inf;
      int bj = open ? j : kHunLanes + 1;
#pragma unroll
      for (int off = kHunLanes / 2; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off, kHunLanes);
        const int oj = __shfl_xor(bj, off, kHunLanes);
        if (ob < best || (ob == best && oj < bj)) {
          best = ob;
          bj = oj;
        }
      }
      if (bj > S) break;  // unreachable for finite costs (the wrapper sanitises them): never index past the arrays
      const double delta = best;
      const int j1 = bj;
      __syncthreads();  // every lane has read u[i0] / p[j0] before the potentials move
      if (valid) {
        if (used) {
          u[p[j]] += delta;
          v -= delta;
        } else {
          minv -= delta;
        }
      }
      if (lane == 0) u[p[0]] += delta;  // the root column is always in the tree
      __syncthreads();
      j0 = j1;
      if (p[j0] == 0) break;
    }
    if (lane == 0) {  // augment along the alternating path
      do {
        const int j1 = way[j0];
        p[j0] = p[j1];
        j0 = j1;
      } while (j0);
    }
    __syncthreads();
  }
  if (valid && p[j] >= 1) col_of_row[static_cast<int64_t>(blockIdx.x) * S + (p[j] - 1)] = j - 1;
}

// metric [B, S, S] on the GPU (rows = target speaker, cols = predicted speaker) -> perm [B, S] int64, maximising
// (or minimising) the summed metric; no host round trip.
at::Tensor linear_assignment_gpu(const at::Tensor& metric, bool maximize) {
  TORCH_CHECK(metric.is_cuda() && metric.dim() == 3 && metric.size(1) == metric.size(2), "linear_assignment_gpu: expected GPU [B, S, S]");
  const int64_t B = metric.size(0), S = metric.size(1);
  TORCH_CHECK(S >= 1 && S <= kHunLanes, "linear_assignment_gpu: 1 <= S <= ", kHunLanes);
  const at::DeviceGuard guard(metric.device());
  // finite costs keep every augmenting step well defined: NaN is the worst score, +-inf a large finite one (as the host)
  constexpr double kBig = 1e150;
  auto m = at::nan_to_num(metric.detach().to(at::kDouble), maximize ? -kBig : kBig, kBig, -kBig).contiguous();
  auto out = at::zeros({B, S}, metric.options().dtype(at::kLong));
  if (B == 0) return out;
  TORCH_CHECK(B < (int64_t{1} << 31), "linear_assignment_gpu: too many problems");
  hipLaunchKernelGGL(hungarian_kernel, dim3(static_cast<unsigned>(B)), dim3(kHunLanes), 0, stream(), m.data_ptr<double>(),
                     static_cast<int>(S), maximize, out.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("linear_assignment_gpu(Tensor metric, bool maximize) -> Tensor"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("toeplitz_solve", &tmx::toeplitz_solve_cuda);
  m.impl("iir_filter", &tmx::iir_filter_cuda);
  m.impl("linear_assignment_gpu", &tmx::linear_assignment_gpu);
}
