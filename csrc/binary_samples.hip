// Binary fp32 / fp64 exact-curve samples on the GPU (reference `_binary_precision_recall_curve_format` +
// `_binary_precision_recall_curve_tensor_validation`, TF/functional/classification/precision_recall_curve.py:140-185,
// and the sample-list update of `BinaryPrecisionRecallCurve.update`, TF/classification/precision_recall_curve.py:160-170).
//
// The reference update is: target value check (two compares, an AND and an `any` = 4 kernels and a host sync), an
// `all(0 <= p <= 1)` test (another host sync) and `sigmoid` when it fails.  Here:
//   * binary_target_check — ONE streaming read of the target (16-B loads) that ORs the deferred-validation flag;
//   * range_flag (classification.hip) — the "any score outside [0, 1]" device flag, early-exit for logits;
//   * sigmoid_if          — one streaming pass writing sigmoid(p) when the flag is set, p otherwise (no host sync).
// At 16.7M samples with int64 targets that is ~60 us of HBM traffic instead of ~200 us of ATen kernels.
//
//   * count_eq_capped     — number of target == value, allowed to stop early once it exceeds `cap` (the anchored
//                           curve route of _curve_engine.anchored_scores only needs "more than ANCHOR_MAX_POS?").
#include "common.h"

namespace tmx {

template <typename TT>
__device__ __forceinline__ bool not01(TT v) {
  return v != TT(0) && v != TT(1);
}

template <typename TT>
__global__ void __launch_bounds__(256) binary_target_check_kernel(const TT* __restrict__ t, int64_t n, int* __restrict__ err) {
  constexpr int V = 16 / sizeof(TT);
  const int64_t nvec = n / V;
  const uint4* tv = reinterpret_cast<const uint4*>(t);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  bool bad = false;
  int64_t i = i0;
  for (; i + 3 * stride < nvec; i += 4 * stride) {  // four 16-B loads in flight
    uint4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = tv[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const TT* e = reinterpret_cast<const TT*>(&q[u]);
#pragma unroll
      for (int k = 0; k < V; ++k) bad |= not01(e[k]);
    }
  }
  for (; i < nvec; i += stride) {
    const uint4 q = tv[i];
    const TT* e = reinterpret_cast<const TT*>(&q);
#pragma unroll
    for (int k = 0; k < V; ++k) bad |= not01(e[k]);
  }
  for (int64_t j = nvec * V + i0; j < n; j += stride) bad |= not01(t[j]);
  if (__ballot(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(err, 1);
}

// torch.sigmoid's formula in the operand's opmath type (1 / (1 + exp(-x))); bit-identical results are checked
// against torch.sigmoid in tests/test_binary_samples_gpu.py
__device__ __forceinline__ float sig(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ double sig(double x) { return 1.0 / (1.0 + exp(-x)); }

template <typename T>
__global__ void __launch_bounds__(256) sigmoid_if_kernel(const T* __restrict__ x, int64_t n, const int* __restrict__ flag,
                                                         T* __restrict__ out) {
  constexpr int V = 16 / sizeof(T);
  const bool on = *flag != 0;
  const int64_t nvec = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  uint4* ov = reinterpret_cast<uint4*>(out);
  int64_t i = i0;
  for (; i + stride < nvec; i += 2 * stride) {
    uint4 q[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) q[u] = xv[i + u * stride];
    if (on) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        T* e = reinterpret_cast<T*>(&q[u]);
#pragma unroll
        for (int k = 0; k < V; ++k) e[k] = sig(e[k]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) ov[i + u * stride] = q[u];
  }
  for (; i < nvec; i += stride) {
    uint4 q = xv[i];
    if (on) {
      T* e = reinterpret_cast<T*>(&q);
#pragma unroll
      for (int k = 0; k < V; ++k) e[k] = sig(e[k]);
    }
    ov[i] = q;
  }
  for (int64_t j = nvec * V + i0; j < n; j += stride) out[j] = on ? sig(x[j]) : x[j];
}

at::Tensor range_flag(const at::Tensor& x_);  // classification.hip

static bool aligned16(const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// preds: float32 / float64 GPU tensor (any shape, flattened); target: integer tensor of the same numel.
// Returns the formatted scores [n] (sigmoid applied iff any score is outside [0, 1] or NaN).  err (int32[1]): ORed
// with 1 when a target value is not 0 / 1.
at::Tensor binary_samples_format(const at::Tensor& preds_, const at::Tensor& target_, const c10::optional<at::Tensor>& err) {
  TORCH_CHECK(preds_.is_cuda() && (preds_.scalar_type() == at::kFloat || preds_.scalar_type() == at::kDouble),
              "binary_samples_format: float32 / float64 scores on the GPU");
  TORCH_CHECK(target_.device() == preds_.device() && target_.numel() == preds_.numel(), "binary_samples_format: target like preds");
  const c10::DeviceGuard guard(preds_.device());
  auto preds = preds_.reshape(-1).contiguous();
  auto target = target_.reshape(-1).contiguous();
  const int64_t n = preds.numel();
  auto out = at::empty({n}, preds.options());
  if (n == 0) return out;
  const int block = 256;
  if (err.has_value() && target.scalar_type() != at::kBool) {
    TORCH_CHECK(err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "binary_samples_format: int32 device flag");
    auto tt = aligned16(target) ? target : target.clone();
    const int64_t per = 16 / tt.element_size();
    const int grid = grid_for(std::max<int64_t>((n / per + 3) / 4, 1), block, 2048);
    switch (tt.scalar_type()) {
      case at::kLong: hipLaunchKernelGGL(binary_target_check_kernel<int64_t>, grid, block, 0, stream(), tt.data_ptr<int64_t>(), n, err->data_ptr<int>()); break;
      case at::kInt: hipLaunchKernelGGL(binary_target_check_kernel<int32_t>, grid, block, 0, stream(), tt.data_ptr<int32_t>(), n, err->data_ptr<int>()); break;
      case at::kShort: hipLaunchKernelGGL(binary_target_check_kernel<int16_t>, grid, block, 0, stream(), tt.data_ptr<int16_t>(), n, err->data_ptr<int>()); break;
      case at::kChar: hipLaunchKernelGGL(binary_target_check_kernel<int8_t>, grid, block, 0, stream(), tt.data_ptr<int8_t>(), n, err->data_ptr<int>()); break;
      case at::kByte: hipLaunchKernelGGL(binary_target_check_kernel<uint8_t>, grid, block, 0, stream(), tt.data_ptr<uint8_t>(), n, err->data_ptr<int>()); break;
      default: TORCH_CHECK(false, "binary_samples_format: integer target expected, got ", tt.scalar_type());
    }
    TMX_LAUNCH_CHECK();
  }
  const auto flag = range_flag(preds);
  auto src = aligned16(preds) ? preds : preds.clone();
  const int64_t per = 16 / src.element_size();
  const int grid = grid_for(std::max<int64_t>((n / per + 1) / 2, 1), block, 2048);
  if (src.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(sigmoid_if_kernel<float>, grid, block, 0, stream(), src.data_ptr<float>(), n, flag.data_ptr<int>(), out.data_ptr<float>());
  else
    hipLaunchKernelGGL(sigmoid_if_kernel<double>, grid, block, 0, stream(), src.data_ptr<double>(), n, flag.data_ptr<int>(), out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

// count of target == value, capped: a one-block probe counts the head (64K elements) first; the main pass over the
// rest leaves at once when the probe already exceeded the cap (balanced labels: ~1 us of reading instead of the whole
// target), else counts with one atomic per wave at its end (an atomic per wave per iteration cost 107 us at 16.7M)
template <typename TT>
__global__ void __launch_bounds__(256) count_eq_kernel(const TT* __restrict__ t, int64_t n, TT value, long long cap,
                                                       unsigned long long* __restrict__ count) {
  if (cap >= 0 && static_cast<long long>(__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) > cap) return;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  unsigned int c = 0;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    TT v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = t[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) c += v[u] == value ? 1u : 0u;
  }
  for (; i < n; i += stride) c += t[i] == value ? 1u : 0u;
  const long long w = wave_sum(static_cast<long long>(c));
  if (w && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(count, static_cast<unsigned long long>(w));
}

template <typename TT>
static void count_eq_launch(const TT* t, int64_t n, TT value, int64_t cap, unsigned long long* c) {
  const int64_t head = std::min<int64_t>(n, 65536);
  // 32 probe blocks (one block walking 64K int64 serially took 34 us: latency, not bandwidth)
  hipLaunchKernelGGL(count_eq_kernel<TT>, static_cast<int>(std::min<int64_t>(32, (head + 2047) / 2048)), 256, 0, stream(), t, head, value, -1ll, c);
  if (n > head) {
    const int grid = grid_for(std::max<int64_t>((n - head + 3) / 4, 1), 256, 2048);
    hipLaunchKernelGGL(count_eq_kernel<TT>, grid, 256, 0, stream(), t + head, n - head, value, static_cast<long long>(cap), c);
  }
  TMX_LAUNCH_CHECK();
}

at::Tensor count_eq_capped(const at::Tensor& target_, int64_t value, int64_t cap) {
  TORCH_CHECK(target_.is_cuda(), "count_eq_capped: GPU tensor");
  const c10::DeviceGuard guard(target_.device());
  auto t = target_.reshape(-1).contiguous();
  auto count = at::zeros({1}, t.options().dtype(at::kLong));
  const int64_t n = t.numel();
  if (n == 0) return count;
  auto* c = reinterpret_cast<unsigned long long*>(count.data_ptr<int64_t>());
  switch (t.scalar_type()) {
    case at::kLong: count_eq_launch<int64_t>(t.data_ptr<int64_t>(), n, value, cap, c); break;
    case at::kInt: count_eq_launch<int32_t>(t.data_ptr<int32_t>(), n, static_cast<int32_t>(value), cap, c); break;
    case at::kByte: count_eq_launch<uint8_t>(t.data_ptr<uint8_t>(), n, static_cast<uint8_t>(value), cap, c); break;
    case at::kBool: count_eq_launch<uint8_t>(reinterpret_cast<const uint8_t*>(t.data_ptr<bool>()), n, static_cast<uint8_t>(value), cap, c); break;
    default: {
      auto tl = t.to(at::kLong);
      count_eq_launch<int64_t>(tl.data_ptr<int64_t>(), n, value, cap, c);
    }
  }
  return count;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("binary_samples_format(Tensor preds, Tensor target, Tensor(a!)? err=None) -> Tensor");
  m.def("count_eq_capped(Tensor target, int value, int cap) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("binary_samples_format", &tmx::binary_samples_format);
  m.impl("count_eq_capped", &tmx::count_eq_capped);
}
