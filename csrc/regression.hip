// Regression map-reduce kernels for gfx950.
//
// One pass over (preds, target) [N, D] produces, per output column, the eight fp64 sums every regression metric
// of the framework is built from:
//   0 Σp   1 Σt   2 Σp²   3 Σt²   4 Σp·t   5 Σ(p−t)²   6 Σ|p−t|   7 Σ op(p, t)
// where `op` is a compile-time selected elementwise error (MAPE / SMAPE / MSLE / log-cosh / Minkowski / |t| /
// Tweedie).  MSE, MAE, R2, RSE, explained variance, Pearson/Concordance moments, cosine pieces, WMAPE, ... all read
// their state increments from this table, so a MetricCollection of regression metrics costs one HBM read.
//
// Mapping (CDNA4, 64-wide waves): a block is 4 waves; blockIdx.y picks a 64-column tile of width W; a wave packs
// R = 64 / W consecutive rows so every lane issues a coalesced load (D == 1 → 64 rows per wave instruction).
// Elementwise math runs in fp32 for ≤32-bit inputs (same rounding as the eager reference ops) and fp64 for fp64;
// accumulation is always fp64.  Each block reduces its lanes per column through LDS and writes one partial row;
// the partials are summed with a deterministic torch reduction (no float atomics → bitwise reproducible).
#include "common.h"

namespace tmx {

enum RegOp : int {
  kOpNone = 0,
  kOpAPE = 1,        // |p-t| / max(|t|, eps)
  kOpSAPE = 2,       // 2 |p-t| / max(|t|+|p|, eps)
  kOpSLE = 3,        // (log1p p - log1p t)^2
  kOpLogCosh = 4,    // log((e^d + e^-d) / 2)
  kOpMinkowski = 5,  // |p-t|^param
  kOpAbsT = 6,       // |t|
  kOpTweedie = 7,    // Tweedie deviance, power = param
};

constexpr int kRegCh = 8;
constexpr int kRegBlock = 256;

template <typename C> __device__ __forceinline__ C xlogy_(C x, C y) { return x == C(0) ? C(0) : x * log(y); }

template <int OP, typename C>
__device__ __forceinline__ C reg_op(C p, C t, C param, C eps) {
  C d = p - t;
  if constexpr (OP == kOpAPE) {
    return fabs(d) / fmax(fabs(t), eps);
  } else if constexpr (OP == kOpSAPE) {
    return C(2) * (fabs(d) / fmax(fabs(t) + fabs(p), eps));
  } else if constexpr (OP == kOpSLE) {
    C e = log1p(p) - log1p(t);
    return e * e;
  } else if constexpr (OP == kOpLogCosh) {
    return log((exp(d) + exp(-d)) / C(2));
  } else if constexpr (OP == kOpMinkowski) {
    return pow(fabs(d), param);
  } else if constexpr (OP == kOpAbsT) {
    return fabs(t);
  } else if constexpr (OP == kOpTweedie) {
    if (param == C(0)) return (t - p) * (t - p);
    if (param == C(1)) return C(2) * (xlogy_(t, t / p) + p - t);
    if (param == C(2)) return C(2) * (log(p / t) + t / p - C(1));
    C term1 = pow(fmax(t, C(0)), C(2) - param) / ((C(1) - param) * (C(2) - param));
    C term2 = t * pow(p, C(1) - param) / (C(1) - param);
    C term3 = pow(p, C(2) - param) / (C(2) - param);
    return C(2) * (term1 - term2 + term3);
  } else {
    return C(0);
  }
}

template <typename T> struct CompT { using type = float; };
template <> struct CompT<double> { using type = double; };

template <typename T> __device__ __forceinline__ typename CompT<T>::type load_c(const T* p, int64_t i) {
  if constexpr (std::is_same<T, double>::value) return p[i];
  else return to_f32<T>(p[i]);
}

// partial: [gridDim.x, 8, D] fp64
template <typename T, int OP>
__global__ __launch_bounds__(kRegBlock) void regression_sums_kernel(const T* __restrict__ preds, const T* __restrict__ target,
                                                                    int64_t N, int D, double param_d, double* __restrict__ partial) {
  using C = typename CompT<T>::type;
  const C param = static_cast<C>(param_d);
  const C eps = static_cast<C>(1.17e-06);
  const int col0 = blockIdx.y * kWave;
  const int W = min(kWave, D - col0);
  const int R = kWave / W;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int k = lane / W;            // packed row within the wave
  const int c = lane - k * W;        // column within the tile
  const bool active = k < R;

  double acc[kRegCh];
#pragma unroll
  for (int i = 0; i < kRegCh; ++i) acc[i] = 0.0;

  if (active) {
    const int64_t rows_per_iter = static_cast<int64_t>(gridDim.x) * 4 * R;
    int64_t row = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * R + k;
    const int col = col0 + c;
#pragma unroll 2
    for (; row < N; row += rows_per_iter) {
      const int64_t off = row * D + col;
      C p = load_c(preds, off);
      C t = load_c(target, off);
      C d = p - t;
      acc[0] += static_cast<double>(p);
      acc[1] += static_cast<double>(t);
      acc[2] += static_cast<double>(p * p);
      acc[3] += static_cast<double>(t * t);
      acc[4] += static_cast<double>(p * t);
      acc[5] += static_cast<double>(d * d);
      acc[6] += static_cast<double>(fabs(d));
      if constexpr (OP != kOpNone) acc[7] += static_cast<double>(reg_op<OP, C>(p, t, param, eps));
    }
  }

  // block reduction per column: lanes (wave, k, c) with the same c hold partials of the same column
  __shared__ double lds[kRegCh][kRegBlock];
#pragma unroll
  for (int i = 0; i < kRegCh; ++i) lds[i][threadIdx.x] = active ? acc[i] : 0.0;
  __syncthreads();
  // thread (ch, c) sums 4 * R entries: one per (wave, k)
  for (int idx = threadIdx.x; idx < kRegCh * W; idx += kRegBlock) {
    const int ch = idx / W;
    const int cc = idx - ch * W;
    double s = 0.0;
    for (int w = 0; w < 4; ++w)
      for (int kk = 0; kk < R; ++kk) s += lds[ch][w * kWave + kk * W + cc];
    partial[(static_cast<int64_t>(blockIdx.x) * kRegCh + ch) * D + col0 + cc] = s;
  }
}

template <typename T>
void launch_regression_sums(const at::Tensor& preds, const at::Tensor& target, int64_t N, int D, int op, double param,
                            at::Tensor& partial, dim3 grid) {
  const auto* p = reinterpret_cast<const T*>(preds.data_ptr());
  const auto* t = reinterpret_cast<const T*>(target.data_ptr());
  double* out = partial.data_ptr<double>();
  switch (op) {
#define TMX_REG_CASE(OPV)                                                                                  \
  case OPV:                                                                                                \
    hipLaunchKernelGGL((regression_sums_kernel<T, OPV>), grid, kRegBlock, 0, stream(), p, t, N, D, param, out); \
    break;
    TMX_REG_CASE(kOpNone)
    TMX_REG_CASE(kOpAPE)
    TMX_REG_CASE(kOpSAPE)
    TMX_REG_CASE(kOpSLE)
    TMX_REG_CASE(kOpLogCosh)
    TMX_REG_CASE(kOpMinkowski)
    TMX_REG_CASE(kOpAbsT)
    TMX_REG_CASE(kOpTweedie)
#undef TMX_REG_CASE
    default:
      break;
  }
}

// Returns fp64 [8, D].
at::Tensor regression_sums(const at::Tensor& preds_in, const at::Tensor& target_in, int64_t op, double param) {
  TORCH_CHECK(preds_in.is_cuda() && target_in.is_cuda(), "regression_sums: expected GPU tensors");
  TORCH_CHECK(preds_in.sizes() == target_in.sizes(), "regression_sums: shape mismatch ", preds_in.sizes(), " vs ",
              target_in.sizes());
  TORCH_CHECK(preds_in.dim() == 2, "regression_sums: expected [N, D] inputs");
  TORCH_CHECK(preds_in.scalar_type() == target_in.scalar_type(), "regression_sums: dtype mismatch");
  TORCH_CHECK(op >= 0 && op <= kOpTweedie, "regression_sums: unknown op ", op);
  const at::DeviceGuard guard(preds_in.device());
  auto preds = preds_in.contiguous();
  auto target = target_in.contiguous();
  const int64_t N = preds.size(0);
  const int64_t D64 = preds.size(1);
  TORCH_CHECK(D64 >= 1 && D64 <= (1 << 20), "regression_sums: unsupported column count ", D64);
  const int D = static_cast<int>(D64);
  auto opts = preds.options().dtype(at::kDouble);
  if (N == 0) return at::zeros({kRegCh, D64}, opts);

  const int tiles = (D + kWave - 1) / kWave;
  const int W0 = std::min(kWave, D);
  const int rows_per_block = 4 * (kWave / W0);
  int64_t gx = (N + rows_per_block - 1) / rows_per_block;
  // ~8 blocks per CU across 256 CUs, shared among column tiles
  const int64_t max_gx = std::max<int64_t>(1, 2048 / tiles);
  gx = std::min(gx, max_gx);
  auto partial = at::empty({gx, kRegCh, D64}, opts);
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(tiles));

  TMX_DISPATCH_FLOAT(preds.scalar_type(), "regression_sums", [&] {
    launch_regression_sums<scalar_t>(preds, target, N, D, static_cast<int>(op), param, partial, grid);
  });
  TMX_LAUNCH_CHECK();
  return gx == 1 ? partial[0] : partial.sum(0);
}

// Streaming Pearson / concordance moments (reference regression/pearson.py update): the batch's per-block partial
// sums are reduced in a fixed order (bitwise reproducible, like partial.sum(0)) and merged into the states in place
// with the pairwise (Chan et al.) update in fp64 -- one small kernel instead of ~25 ATen ops per update.
template <typename S>
__global__ __launch_bounds__(256) void pearson_merge_kernel(const double* __restrict__ partial, int64_t G, int D, double nb,
                                                            S* __restrict__ mean_x, S* __restrict__ mean_y, S* __restrict__ var_x,
                                                            S* __restrict__ var_y, S* __restrict__ corr_xy, S* __restrict__ n_total) {
  const int d = blockIdx.x;
  __shared__ double red[5][256];
  double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t g = threadIdx.x; g < G; g += blockDim.x)
#pragma unroll
    for (int ch = 0; ch < 5; ++ch) a[ch] += partial[(g * kRegCh + ch) * D + d];
#pragma unroll
  for (int ch = 0; ch < 5; ++ch) red[ch][threadIdx.x] = a[ch];
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int ch = 0; ch < 5; ++ch) red[ch][threadIdx.x] += red[ch][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double s0 = red[0][0], s1 = red[1][0], s2 = red[2][0], s3 = red[3][0], s4 = red[4][0];
  const double mxb = s0 / nb, myb = s1 / nb;
  const double m2x = s2 - s0 * mxb, m2y = s3 - s1 * myb, cxy = s4 - s0 * myb;
  const double n0 = (double)n_total[d];
  const double n = n0 + nb;
  const double mx0 = (double)mean_x[d], my0 = (double)mean_y[d];
  const double dx = mxb - mx0, dy = myb - my0;
  const double w = n0 * nb / n;
  mean_x[d] = (S)(mx0 + dx * (nb / n));
  mean_y[d] = (S)(my0 + dy * (nb / n));
  var_x[d] = (S)((double)var_x[d] + m2x + w * dx * dx);
  var_y[d] = (S)((double)var_y[d] + m2y + w * dy * dy);
  corr_xy[d] = (S)((double)corr_xy[d] + cxy + w * dx * dy);
  n_total[d] = n_total[d] + (S)nb;  // state-dtype add, as `num_prior + num_obs` on the state tensor
}

void pearson_update(const at::Tensor& preds_in, const at::Tensor& target_in, at::Tensor& mean_x, at::Tensor& mean_y,
                    at::Tensor& var_x, at::Tensor& var_y, at::Tensor& corr_xy, at::Tensor& n_total) {
  TORCH_CHECK(preds_in.sizes() == target_in.sizes() && preds_in.dim() == 2, "pearson_update: expected matching [N, D] inputs");
  TORCH_CHECK(preds_in.scalar_type() == target_in.scalar_type(), "pearson_update: dtype mismatch");
  const int64_t N = preds_in.size(0), D64 = preds_in.size(1);
  for (const at::Tensor* st : {&mean_x, &mean_y, &var_x, &var_y, &corr_xy, &n_total}) {
    TORCH_CHECK(st->is_contiguous() && st->numel() == D64 && st->scalar_type() == mean_x.scalar_type() &&
                    (st->scalar_type() == at::kFloat || st->scalar_type() == at::kDouble),
                "pearson_update: states must be contiguous float32/float64 [D] of one dtype");
  }
  if (N == 0) return;
  const at::DeviceGuard guard(preds_in.device());
  auto preds = preds_in.contiguous();
  auto target = target_in.contiguous();
  TORCH_CHECK(D64 >= 1 && D64 <= (1 << 20), "pearson_update: unsupported column count ", D64);
  const int D = static_cast<int>(D64);
  const int tiles = (D + kWave - 1) / kWave;
  const int W0 = std::min(kWave, D);
  const int rows_per_block = 4 * (kWave / W0);
  const int64_t gx = std::min<int64_t>((N + rows_per_block - 1) / rows_per_block, std::max<int64_t>(1, 2048 / tiles));
  auto partial = at::empty({gx, kRegCh, D64}, preds.options().dtype(at::kDouble));
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(tiles));
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "pearson_update", [&] {
    launch_regression_sums<scalar_t>(preds, target, N, D, kOpNone, 0.0, partial, grid);
  });
  if (mean_x.scalar_type() == at::kFloat) {
    hipLaunchKernelGGL(pearson_merge_kernel<float>, D, 256, 0, stream(), partial.data_ptr<double>(), gx, D, (double)N,
                       mean_x.data_ptr<float>(), mean_y.data_ptr<float>(), var_x.data_ptr<float>(), var_y.data_ptr<float>(),
                       corr_xy.data_ptr<float>(), n_total.data_ptr<float>());
  } else {
    hipLaunchKernelGGL(pearson_merge_kernel<double>, D, 256, 0, stream(), partial.data_ptr<double>(), gx, D, (double)N,
                       mean_x.data_ptr<double>(), mean_y.data_ptr<double>(), var_x.data_ptr<double>(), var_y.data_ptr<double>(),
                       corr_xy.data_ptr<double>(), n_total.data_ptr<double>());
  }
  TMX_LAUNCH_CHECK();
}


// Sum-state update in place (MSE / MAE / ... update: ``state += sums[chan].to(out) ; total += n``): the batch's
// per-block partials are reduced in a fixed order (as in pearson_merge_kernel) and added into up to four state
// tensors and the int64 sample counter by ONE small launch -- replacing the ATen partial.sum, select, dtype cast and
// two in-place adds (five launches and their host cost per update).  Rounding follows the eager ops: the fp64 sum is
// cast to the inputs' dtype O, then added in promote(S, O) and stored as the state dtype S.
constexpr int kAccMax = 4;
struct AccArgs {
  void* state[kAccMax];
  int32_t chan[kAccMax];
  int32_t s_double[kAccMax];  // state dtype: 1 = float64, 0 = float32
  int32_t count;
};

template <typename O>
__global__ __launch_bounds__(256) void regression_accumulate_kernel(const double* __restrict__ partial, int64_t G, int D, AccArgs a,
                                                                    int64_t* __restrict__ total, int64_t n_add) {
  const int d = blockIdx.x;
  __shared__ double red[kAccMax][256];
  double v[kAccMax] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t g = threadIdx.x; g < G; g += blockDim.x)
#pragma unroll
    for (int i = 0; i < kAccMax; ++i)
      if (i < a.count) v[i] += partial[(g * kRegCh + a.chan[i]) * D + d];
#pragma unroll
  for (int i = 0; i < kAccMax; ++i) red[i][threadIdx.x] = v[i];
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
#pragma unroll
      for (int i = 0; i < kAccMax; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  for (int i = 0; i < a.count; ++i) {
    const O inc = static_cast<O>(red[i][0]);
    if (a.s_double[i]) {
      double* st = static_cast<double*>(a.state[i]);
      st[d] = st[d] + static_cast<double>(inc);
    } else {
      float* st = static_cast<float*>(a.state[i]);
      if constexpr (sizeof(O) == 8) st[d] = static_cast<float>(static_cast<double>(st[d]) + inc);
      else st[d] = st[d] + inc;
    }
  }
  if (d == 0 && total != nullptr) total[0] += n_add;
}

void regression_accumulate(const at::Tensor& preds_in, const at::Tensor& target_in, int64_t op, double param, c10::IntArrayRef chans,
                           at::TensorList states, const c10::optional<at::Tensor>& total, int64_t n_add) {
  TORCH_CHECK(preds_in.sizes() == target_in.sizes() && preds_in.dim() == 2, "regression_accumulate: expected matching [N, D] inputs");
  TORCH_CHECK(preds_in.scalar_type() == target_in.scalar_type() &&
                  (preds_in.scalar_type() == at::kFloat || preds_in.scalar_type() == at::kDouble),
              "regression_accumulate: float32 / float64 inputs of one dtype");
  TORCH_CHECK(op >= 0 && op <= kOpTweedie, "regression_accumulate: unknown op ", op);
  TORCH_CHECK(chans.size() == states.size() && !states.empty() && states.size() <= kAccMax, "regression_accumulate: 1-4 states");
  const int64_t N = preds_in.size(0), D64 = preds_in.size(1);
  TORCH_CHECK(D64 >= 1 && D64 <= (1 << 20), "regression_accumulate: unsupported column count ", D64);
  AccArgs a{};
  a.count = static_cast<int32_t>(states.size());
  for (size_t i = 0; i < states.size(); ++i) {
    const at::Tensor& st = states[i];
    TORCH_CHECK(st.is_cuda() && st.device() == preds_in.device() && st.is_contiguous() && st.numel() == D64 &&
                    (st.scalar_type() == at::kFloat || st.scalar_type() == at::kDouble),
                "regression_accumulate: states must be contiguous float32/float64 [D] on the inputs' device");
    TORCH_CHECK(chans[i] >= 0 && chans[i] < kRegCh, "regression_accumulate: channel out of range");
    a.state[i] = st.data_ptr();
    a.chan[i] = static_cast<int32_t>(chans[i]);
    a.s_double[i] = st.scalar_type() == at::kDouble;
  }
  int64_t* tot = nullptr;
  if (total.has_value()) {
    TORCH_CHECK(total->is_cuda() && total->device() == preds_in.device() && total->scalar_type() == at::kLong && total->numel() == 1,
                "regression_accumulate: total must be one int64 on the inputs' device");
    tot = total->data_ptr<int64_t>();
  }
  const at::DeviceGuard guard(preds_in.device());
  if (N == 0) {  // nothing to add but the (zero) count
    return;
  }
  auto preds = preds_in.contiguous();
  auto target = target_in.contiguous();
  const int D = static_cast<int>(D64);
  const int tiles = (D + kWave - 1) / kWave;
  const int W0 = std::min(kWave, D);
  const int rows_per_block = 4 * (kWave / W0);
  const int64_t gx = std::min<int64_t>((N + rows_per_block - 1) / rows_per_block, std::max<int64_t>(1, 2048 / tiles));
  auto partial = at::empty({gx, kRegCh, D64}, preds.options().dtype(at::kDouble));
  dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(tiles));
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "regression_accumulate", [&] {
    launch_regression_sums<scalar_t>(preds, target, N, D, static_cast<int>(op), param, partial, grid);
  });
  TMX_LAUNCH_CHECK();
  if (preds.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(regression_accumulate_kernel<float>, D, 256, 0, stream(), partial.data_ptr<double>(), gx, D, a, tot, n_add);
  else
    hipLaunchKernelGGL(regression_accumulate_kernel<double>, D, 256, 0, stream(), partial.data_ptr<double>(), gx, D, a, tot, n_add);
  TMX_LAUNCH_CHECK();
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("regression_sums(Tensor preds, Tensor target, int op, float param) -> Tensor");
  m.def("pearson_update(Tensor preds, Tensor target, Tensor(a!) mean_x, Tensor(b!) mean_y, Tensor(c!) var_x, Tensor(d!) var_y, Tensor(e!) corr_xy, Tensor(f!) n_total) -> ()");
  m.def("regression_accumulate(Tensor preds, Tensor target, int op, float param, int[] chans, Tensor(a!)[] states, Tensor(b!)? total, int n_add) -> ()");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("regression_sums", &tmx::regression_sums);
  m.impl("pearson_update", &tmx::pearson_update);
  m.impl("regression_accumulate", &tmx::regression_accumulate);
}
