// Fused token negative log-likelihood for Perplexity.
//
// nll[r] = logsumexp(x[r, :]) - x[r, target[r]]   (0 for ignored rows)
//
// The reference materialises softmax(x) and then an [N, N] gather (`probs[:, target].diagonal()`).  Here one
// 256-thread block streams a row once with an online (max, scaled-sum) pair per thread — one exp per element —
// merges the pairs with 64-wide wave shuffles and LDS, and reads the target logit directly: HBM traffic is one
// pass over the logits, nothing else is materialised.  16-byte vector loads when the row is aligned.
#include "common.h"

namespace tmx {

constexpr int kNllThreads = 256;

template <typename A>
struct MaxSum {
  A m, s;
};

template <typename A>
__device__ __forceinline__ void ms_push(MaxSum<A>& a, A x) {
  if (x == -INFINITY) return;  // fully masked logit: contributes exp(-inf) = 0
  if (x > a.m) {
    a.s = a.s * exp(a.m - x) + A(1);
    a.m = x;
  } else {
    a.s += exp(x - a.m);
  }
}

template <typename A>
__device__ __forceinline__ MaxSum<A> ms_merge(MaxSum<A> a, MaxSum<A> b) {
  if (b.m == -INFINITY) return a;
  if (a.m == -INFINITY) return b;
  const A m = a.m > b.m ? a.m : b.m;
  return {m, a.s * exp(a.m - m) + b.s * exp(b.m - m)};
}

template <typename T> struct NllAcc { using type = float; };
template <> struct NllAcc<double> { using type = double; };

template <typename T, typename A>
__device__ __forceinline__ A load_acc(const T* p, int64_t i) {
  if constexpr (std::is_same<T, double>::value) return p[i];
  else return static_cast<A>(to_f32<T>(p[i]));
}

template <typename T>
__global__ __launch_bounds__(kNllThreads) void token_nll_kernel(const T* __restrict__ x, const int64_t* __restrict__ target, int64_t V,
                                                                int64_t ignore, bool has_ignore, typename NllAcc<T>::type* __restrict__ out) {
  using A = typename NllAcc<T>::type;
  const int64_t row = blockIdx.x;
  const int64_t t = target[row];
  if (has_ignore && t == ignore) {
    if (threadIdx.x == 0) out[row] = A(0);
    return;
  }
  if (t < 0 || t >= V) {  // out-of-range class id: poison the row instead of reading out of bounds
    if (threadIdx.x == 0) out[row] = NAN;
    return;
  }
  const T* xr = x + row * V;
  MaxSum<A> acc{-INFINITY, A(0)};
  constexpr int kVec = 16 / sizeof(T);
  const bool aligned = (reinterpret_cast<uintptr_t>(xr) % 16 == 0);
  int64_t done = 0;
  if (aligned && kVec > 1) {
    const int64_t nvec = V / kVec;
    struct alignas(16) Pack { T v[kVec]; };
    const Pack* xp = reinterpret_cast<const Pack*>(xr);
    for (int64_t i = threadIdx.x; i < nvec; i += kNllThreads) {
      const Pack pk = xp[i];
#pragma unroll
      for (int k = 0; k < kVec; ++k) {
        A v;
        if constexpr (std::is_same<T, double>::value) v = pk.v[k];
        else v = static_cast<A>(to_f32<T>(pk.v[k]));
        ms_push(acc, v);
      }
    }
    done = nvec * kVec;
  }
  for (int64_t i = done + threadIdx.x; i < V; i += kNllThreads) ms_push(acc, load_acc<T, A>(xr, i));
  // wave merge
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    MaxSum<A> o{__shfl_xor(acc.m, off, kWave), __shfl_xor(acc.s, off, kWave)};
    acc = ms_merge(acc, o);
  }
  __shared__ A sm[kNllThreads / kWave], ss[kNllThreads / kWave];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) {
    sm[wave] = acc.m;
    ss[wave] = acc.s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MaxSum<A> tot{sm[0], ss[0]};
    for (int w = 1; w < kNllThreads / kWave; ++w) tot = ms_merge(tot, MaxSum<A>{sm[w], ss[w]});
    const A xt = load_acc<T, A>(xr, t);
    out[row] = (tot.m + log(tot.s)) - xt;
  }
}

// logits [N, V] (any float dtype), target [N] int64 -> nll [N] (fp32, or fp64 for fp64 logits)
at::Tensor token_nll(const at::Tensor& logits_in, const at::Tensor& target_in, int64_t ignore_index, bool has_ignore) {
  TORCH_CHECK(logits_in.is_cuda() && target_in.is_cuda(), "token_nll: expected GPU tensors");
  TORCH_CHECK(logits_in.dim() == 2 && target_in.dim() == 1 && target_in.size(0) == logits_in.size(0), "token_nll: expected [N,V] / [N]");
  TORCH_CHECK(target_in.scalar_type() == at::kLong, "token_nll: target must be int64");
  const at::DeviceGuard guard(logits_in.device());
  auto logits = logits_in.contiguous();
  auto target = target_in.contiguous();
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V > 0, "token_nll: empty vocabulary");
  auto out = at::empty({N}, logits.options().dtype(logits.scalar_type() == at::kDouble ? at::kDouble : at::kFloat));
  if (N == 0) return out;
  TMX_DISPATCH_FLOAT(logits.scalar_type(), "token_nll", [&] {
    using A = typename NllAcc<scalar_t>::type;
    hipLaunchKernelGGL(token_nll_kernel<scalar_t>, dim3(static_cast<unsigned>(N)), dim3(kNllThreads), 0, stream(),
                       reinterpret_cast<const scalar_t*>(logits.data_ptr()), target.data_ptr<int64_t>(), V, ignore_index, has_ignore,
                       out.data_ptr<A>());
  });
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("token_nll(Tensor logits, Tensor target, int ignore_index, bool has_ignore) -> Tensor"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("token_nll", &tmx::token_nll); }
