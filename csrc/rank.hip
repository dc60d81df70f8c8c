// Rank-statistics kernels for gfx950 (regression: Spearman K15, Kendall K14).
//
//   rank_average      ties-averaged 1-based ranks of D sorted rows in one launch: every sorted position finds its run
//                     of equal values with two binary searches (no cumsum / bincount / scatter chain) and writes
//                     rank[idx] = (first + last + 2) / 2.  Reference: functional/regression/spearman.py:41-61 (a
//                     Python loop over every repeated value).
//   count_inversions  #{i < j : y_i > y_j} of a double vector by bottom-up merge levels.  One workgroup sorts and
//                     counts each 1024-element tile in LDS (levels 1..512, ping-pong buffers); every higher level
//                     is one launch in which each element finds its merged position with one binary search in the
//                     other half (left: #right < v, right: #left <= v; the right element's inversions are the left
//                     elements > v).  Reference: functional/regression/kendall.py:101-163 (O(n^2) pair masks, or
//                     scipy's merge sort on the host).
#include "common.h"

namespace tmx {
namespace {

constexpr int kTile = 1024;
constexpr int kTileThreads = 256;

template <typename T>
__global__ __launch_bounds__(256) void rank_average_kernel(const T* __restrict__ srt, const int64_t* __restrict__ idx, int64_t n,
                                                          int64_t D, T* __restrict__ rank) {
  const int64_t total = n * D;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = g / n, i = g % n;
    const T* row = srt + d * n;
    const T v = row[i];
    // first position of the run (lower bound of v) and one past its last (upper bound)
    int64_t lo = 0, hi = i;
    while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (row[m] < v) lo = m + 1; else hi = m; }
    const int64_t first = lo;
    lo = i + 1; hi = n;
    while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (row[m] <= v) lo = m + 1; else hi = m; }
    const int64_t last = lo - 1;
    rank[d * n + idx[d * n + i]] = static_cast<T>(static_cast<double>(first + last + 2) * 0.5);
  }
}

// #{k in [0, len) : a[k] < v} (strict) or <= v
template <bool STRICT>
__device__ __forceinline__ int64_t bound(const double* a, int64_t len, double v) {
  int64_t lo = 0, hi = len;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (STRICT ? a[m] < v : a[m] <= v) lo = m + 1;
    else hi = m;
  }
  return lo;
}

__device__ __forceinline__ void block_add_count(long long c, unsigned long long* out) {
  __shared__ long long s_c[kTileThreads / kWave];
  c = wave_sum(c);
  if ((threadIdx.x & (kWave - 1)) == 0) s_c[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < kTileThreads / kWave; ++w) t += s_c[w];
    if (t) atomicAdd(out, static_cast<unsigned long long>(t));
  }
}

// levels 1 .. kTile/2 of one tile inside LDS; the sorted tile is written back in place
__global__ __launch_bounds__(kTileThreads) void inv_tile_kernel(double* __restrict__ buf, unsigned long long* __restrict__ count) {
  __shared__ double s[2][kTile];
  double* base = buf + (int64_t)blockIdx.x * kTile;
  for (int k = threadIdx.x; k < kTile; k += kTileThreads) s[0][k] = base[k];
  __syncthreads();
  long long inv = 0;
  int cur = 0;
  for (int b = 1; b < kTile; b <<= 1) {
    for (int k = threadIdx.x; k < kTile; k += kTileThreads) {
      const int pair = k & ~(2 * b - 1), off = k & (b - 1);
      const double v = s[cur][k];
      int pos;
      if ((k & b) == 0) {  // left half element: left predecessors + right elements strictly smaller
        pos = off + static_cast<int>(bound<true>(&s[cur][pair + b], b, v));
      } else {             // right: right predecessors + left elements <= v; the others are inversions
        const int le = static_cast<int>(bound<false>(&s[cur][pair], b, v));
        inv += b - le;
        pos = off + le;
      }
      s[cur ^ 1][pair + pos] = v;
    }
    __syncthreads();
    cur ^= 1;
  }
  for (int k = threadIdx.x; k < kTile; k += kTileThreads) base[k] = s[cur][k];
  block_add_count(inv, count);
}

__global__ __launch_bounds__(kTileThreads) void inv_level_kernel(const double* __restrict__ in, double* __restrict__ out, int64_t size,
                                                                 int64_t b, unsigned long long* __restrict__ count) {
  long long inv = 0;
  for (int64_t k = (int64_t)blockIdx.x * kTileThreads + threadIdx.x; k < size; k += (int64_t)gridDim.x * kTileThreads) {
    const int64_t pair = k & ~(2 * b - 1), off = k & (b - 1);
    const double v = in[k];
    int64_t pos;
    if ((k & b) == 0) {
      pos = off + bound<true>(in + pair + b, b, v);
    } else {
      const int64_t le = bound<false>(in + pair, b, v);
      inv += b - le;
      pos = off + le;
    }
    out[pair + pos] = v;
  }
  block_add_count(inv, count);
}

}  // namespace

// srt / idx: [D, n] (each row sorted ascending, idx = the sort's permutation); returns ranks [D, n] in srt's dtype
at::Tensor rank_average(const at::Tensor& srt, const at::Tensor& idx) {
  TORCH_CHECK(srt.is_cuda() && srt.dim() == 2 && srt.is_contiguous(), "rank_average: sorted rows [D, n] on the GPU");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.sizes() == srt.sizes() && idx.is_contiguous(), "rank_average: int64 permutation");
  c10::DeviceGuard guard(srt.device());
  auto rank = at::empty_like(srt);
  const int64_t D = srt.size(0), n = srt.size(1);
  if (D * n == 0) return rank;
  const int grid = grid_for(D * n, 256, 256 * 16);
  if (srt.scalar_type() == at::kDouble)
    hipLaunchKernelGGL(rank_average_kernel<double>, grid, 256, 0, stream(), srt.data_ptr<double>(), idx.data_ptr<int64_t>(), n, D, rank.data_ptr<double>());
  else if (srt.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(rank_average_kernel<float>, grid, 256, 0, stream(), srt.data_ptr<float>(), idx.data_ptr<int64_t>(), n, D, rank.data_ptr<float>());
  else
    TORCH_CHECK(false, "rank_average: float32 / float64 rows");
  TMX_LAUNCH_CHECK();
  return rank;
}

// int64 scalar #{i < j : y_i > y_j}
at::Tensor count_inversions(const at::Tensor& y) {
  TORCH_CHECK(y.is_cuda() && y.dim() == 1, "count_inversions: 1-D GPU tensor");
  c10::DeviceGuard guard(y.device());
  const int64_t n = y.numel();
  auto count = at::zeros({1}, y.options().dtype(at::kLong));
  if (n < 2) return count.reshape({});
  int64_t size = kTile;
  while (size < n) size <<= 1;
  auto a = at::full({size}, INFINITY, y.options().dtype(at::kDouble));
  a.narrow(0, 0, n).copy_(y);
  auto b = at::empty_like(a);
  auto* cnt = reinterpret_cast<unsigned long long*>(count.data_ptr<int64_t>());
  hipLaunchKernelGGL(inv_tile_kernel, static_cast<int>(size / kTile), kTileThreads, 0, stream(), a.data_ptr<double>(), cnt);
  TMX_LAUNCH_CHECK();
  double* in = a.data_ptr<double>();
  double* out = b.data_ptr<double>();
  for (int64_t half = kTile; half < size; half <<= 1) {
    const int grid = grid_for(size, kTileThreads, 256 * 16);
    hipLaunchKernelGGL(inv_level_kernel, grid, kTileThreads, 0, stream(), in, out, size, half, cnt);
    TMX_LAUNCH_CHECK();
    std::swap(in, out);
  }
  return count.reshape({});
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("rank_average(Tensor srt, Tensor idx) -> Tensor");
  m.def("count_inversions(Tensor y) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("rank_average", &tmx::rank_average);
  m.impl("count_inversions", &tmx::count_inversions);
}
