// Macro-averaged curves (K7): the sum over C ragged per-class curves of their piecewise-linear interpolation at
// every query point, in one launch.
//
// Reference: functional/classification/roc.py:187-196 / precision_recall_curve.py:587-596 loop over classes in
// Python, each iteration an O(M x K) broadcast compare in ``utilities/compute.py:134-157 interp``.  Here one thread
// owns a query point and walks the classes in order (the same fp32 accumulation order as the per-class loop):
// segment j = #(xp_c <= x) - 1 from a binary search in the class's sorted copy, clamped to [0, K_c - 2];
// slope = (fp[j+1] - fp[j]) / (xp[j+1] - xp[j]) with a zero denominator treated as 1 (``_safe_divide``),
// value = slope * x + (fp[j] - slope * xp[j]) with separate roundings (no FMA contraction), as the tensor expression.
#include "common.h"

namespace tmx {
namespace {

__global__ __launch_bounds__(256) void macro_interp_kernel(const float* __restrict__ x, int64_t M, const float* __restrict__ xp,
                                                           const float* __restrict__ fp, const float* __restrict__ xs,
                                                           const int64_t* __restrict__ off, int C, float* __restrict__ out) {
#pragma clang fp contract(off)
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    const float xv = x[m];
    float acc = 0.f;
    for (int c = 0; c < C; ++c) {
      const int64_t s = off[c], L = off[c + 1] - s;
      if (L < 2) {
        if (L == 1) acc = acc + fp[s];
        continue;
      }
      int64_t lo = 0, hi = L;  // #(xp_c <= xv)
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (xs[s + mid] <= xv) lo = mid + 1;
        else hi = mid;
      }
      int64_t j = lo - 1;
      j = j < 0 ? 0 : (j > L - 2 ? L - 2 : j);
      float dx = xp[s + j + 1] - xp[s + j];
      dx = dx == 0.f ? 1.f : dx;
      const float slope = (fp[s + j + 1] - fp[s + j]) / dx;
      const float intercept = fp[s + j] - slope * xp[s + j];
      const float v = slope * xv;
      acc = acc + (v + intercept);
    }
    out[m] = acc;
  }
}

}  // namespace

// x [M] query points; xp / fp [L] concatenated curves with class offsets off [C + 1]; xs = xp sorted within each
// class.  Returns the fp32 sum over classes of interp_c(x) (the caller divides by C).
at::Tensor macro_interp(const at::Tensor& x, const at::Tensor& xp, const at::Tensor& fp, const at::Tensor& xs, const at::Tensor& off) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && xp.scalar_type() == at::kFloat && fp.scalar_type() == at::kFloat &&
                  xs.scalar_type() == at::kFloat, "macro_interp: fp32 GPU tensors");
  TORCH_CHECK(off.scalar_type() == at::kLong && off.dim() == 1 && off.numel() >= 1, "macro_interp: int64 offsets [C + 1]");
  TORCH_CHECK(xp.numel() == fp.numel() && xs.numel() == xp.numel(), "macro_interp: curve lengths");
  c10::DeviceGuard guard(x.device());
  auto xc = x.contiguous(), xpc = xp.contiguous(), fpc = fp.contiguous(), xsc = xs.contiguous(), oc = off.contiguous();
  const int64_t M = xc.numel();
  auto out = at::empty({M}, xc.options());
  if (M == 0) return out;
  hipLaunchKernelGGL(macro_interp_kernel, grid_for(M, 256, 256 * 16), 256, 0, stream(), xc.data_ptr<float>(), M, xpc.data_ptr<float>(),
                     fpc.data_ptr<float>(), xsc.data_ptr<float>(), oc.data_ptr<int64_t>(), static_cast<int>(oc.numel() - 1),
                     out.data_ptr<float>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("macro_interp(Tensor x, Tensor xp, Tensor fp, Tensor xs, Tensor off) -> Tensor"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("macro_interp", &tmx::macro_interp); }
