// Row-wise classification kernels for gfx950: one 64-lane wave per row, the whole row held in registers
// (C <= 64 * VPT, VPT in {1, 2, 4, 8, 16, 32}), no sort and no [N, C] temporaries.
//
//   topk_stats   (K3)  multiclass stat scores for top_k >= 1 and samplewise averaging.  Reference semantics:
//                      functional/classification/stat_scores.py:363-393 (select_topk one-hot, compare, sum).  The
//                      k best entries are found by k wave arg-max rounds over the register-resident row, each round
//                      restricted to entries ordered after the previous pick — (value desc, index asc), NaN first
//                      as torch.topk orders it — so no exclusion state is kept.  Per row: tp / fn on the target
//                      class, fp on every other pick; tn is derived on the host from the valid-row count.
//   mc_hinge     (K11) multiclass hinge loss (crammer-singer or one-vs-all) with the batch's softmax decision read
//                      from the device range flag; every intermediate rounded to the input dtype, as the reference's
//                      tensor expression computes it (functional/classification/hinge.py:118-140).
//   ml_ranking   (K10) multilabel coverage error / label-ranking AP / ranking loss.  Reference loops over samples
//                      with two torch.unique calls per row (functional/classification/ranking.py:27-33, 113-128)
//                      or an argsort of argsort (:196-217); here each relevant label's counts are one register
//                      sweep of the row with the label's score broadcast from its lane.
#include "common.h"

#include <climits>

namespace tmx {
namespace {

constexpr int kRowBlock = 256;  // 4 waves per workgroup, one row per wave at a time

// strict total order of (value, index) used by torch.topk / argmax: NaN before numbers (NaNs by index), larger values
// first, lower index first among equals.  ``before(a, ia, b, ib)`` = (a, ia) comes before (b, ib).
__device__ __forceinline__ bool before(float a, int ia, float b, int ib) {
  const bool na = a != a, nb = b != b;
  if (na != nb) return na;
  if (na) return ia < ib;
  return a > b || (a == b && ia < ib);
}

template <typename T, int VPT>
__device__ __forceinline__ void load_row(const T* __restrict__ row, int C, int lane, float (&v)[VPT]) {
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int c = lane + j * kWave;
    v[j] = c < C ? to_f32<T>(row[c]) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------------------------- top-k stats
template <typename T, int VPT>
__global__ __launch_bounds__(kRowBlock) void topk_stats_kernel(const T* __restrict__ preds, const int64_t* __restrict__ labels,
                                                              const int64_t* __restrict__ target, int64_t M, int C, int k,
                                                              int64_t ignore_index, bool has_ignore, int64_t X, bool samplewise,
                                                              int64_t* __restrict__ tp, int64_t* __restrict__ fp,
                                                              int64_t* __restrict__ fn, int64_t* __restrict__ nvalid) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t waves = (int64_t)gridDim.x * (kRowBlock / kWave);
  for (int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + threadIdx.x / kWave; r < M; r += waves) {
    const int64_t t = target[r];
    if ((has_ignore && t == ignore_index) || t < 0 || t >= C) continue;  // wave-uniform
    int sel = -1;  // lane j < k holds the j-th pick
    if (labels != nullptr) {
      const int64_t p = labels[r];
      sel = (lane == 0 && p >= 0 && p < C) ? static_cast<int>(p) : -1;
    } else {
      float v[VPT];
      load_row<T, VPT>(preds + r * C, C, lane, v);
      float pv = 0.f;
      int pi = -1;  // the previous pick (unused in round 0)
      for (int round = 0; round < k; ++round) {
        float bv = -INFINITY;
        int bi = INT_MAX;
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
          const int c = lane + j * kWave;
          if (c < C && (round == 0 || before(pv, pi, v[j], c)) && before(v[j], c, bv, bi)) { bv = v[j]; bi = c; }
        }
        wave_argmax(bv, bi);
        if (lane == round) sel = bi;
        pv = bv;
        pi = bi;
      }
    }
    const bool hit = __ballot(sel >= 0 && sel == t) != 0;
    const int64_t base = samplewise ? (r / X) * C : 0;
    if (sel >= 0 && sel != t) atomic_add_i64(fp + base + sel, 1);
    if (lane == 0) {
      atomic_add_i64((hit ? tp : fn) + base + t, 1);
      atomic_add_i64(nvalid + (samplewise ? r / X : 0), 1);
    }
  }
}

// ---------------------------------------------------------------------------------------------------- hinge
// NaN-propagating max (torch.max semantics)
__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || a > b) ? a : b; }
__device__ __forceinline__ float nan_clamp0(float x) { return (x != x || x > 0.f) ? x : 0.f; }

template <typename T, int VPT, bool OVA>
__global__ __launch_bounds__(kRowBlock) void mc_hinge_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                            int64_t N, int C, const int* __restrict__ softmax_flag, bool squared,
                                                            float* __restrict__ partial) {
  __shared__ float s_red[kRowBlock / kWave][OVA ? 64 * VPT : 1];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const bool do_softmax = softmax_flag[0] != 0;
  float acc[OVA ? VPT : 1];
#pragma unroll
  for (int j = 0; j < (OVA ? VPT : 1); ++j) acc[j] = 0.f;
  const int64_t waves = (int64_t)gridDim.x * (kRowBlock / kWave);
  for (int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + wave; r < N; r += waves) {
    const int64_t t = target[r];
    float v[VPT];
    load_row<T, VPT>(preds + r * C, C, lane, v);
    if (do_softmax) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < VPT; ++j) m = nan_max(m, v[j]);
      // NaN-propagating wave max
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = nan_max(m, __shfl_xor(m, off, kWave));
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int c = lane + j * kWave;
        v[j] = c < C ? expf(v[j] - m) : 0.f;
        s += v[j];
      }
      s = wave_sum(s);
#pragma unroll
      for (int j = 0; j < VPT; ++j) v[j] = round_trip<T>(v[j] / s);
    }
    if constexpr (OVA) {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int c = lane + j * kWave;
        if (c < C) {
          const float margin = c == t ? v[j] : -v[j];
          float meas = nan_clamp0(round_trip<T>(1.f - margin));
          if (squared) meas = round_trip<T>(meas * meas);
          acc[j] += meas;
        }
      }
    } else {
      float pl = 0.f, mo = -INFINITY;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int c = lane + j * kWave;
        if (c < C) {
          if (c == t) pl = v[j];
          else mo = nan_max(mo, v[j]);
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mo = nan_max(mo, __shfl_xor(mo, off, kWave));
      const float pt = __shfl(pl, static_cast<int>(t & (kWave - 1)), kWave);  // the lane owning class t
      float meas = nan_clamp0(round_trip<T>(1.f - round_trip<T>(pt - mo)));
      if (squared) meas = round_trip<T>(meas * meas);
      if (lane == 0) acc[0] += meas;
    }
  }
  // deterministic block reduction -> partial[blockIdx][*]
  if constexpr (OVA) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) s_red[wave][lane + j * kWave] = acc[j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += kRowBlock) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kRowBlock / kWave; ++w) s += s_red[w][c];
      partial[(int64_t)blockIdx.x * C + c] = s;
    }
  } else {
    if (lane == 0) s_red[wave][0] = acc[0];
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kRowBlock / kWave; ++w) s += s_red[w][0];
      partial[blockIdx.x] = s;
    }
  }
}

// -------------------------------------------------------------------------------------------------- ranking
// KIND 0: coverage error  (#{l : p_l >= min_l (p_l + g [t_l == 0])}),
// KIND 1: label-ranking AP (mean over relevant j of #{rel i : p_i >= p_j} / #{i : p_i >= p_j}; 1 for degenerate rows),
// KIND 2: ranking loss     ((sum_j #{i : p_i > p_j or (p_i == p_j and i >= j)} - n(n+1)/2) / (n (L - n)); 0 when
//                           degenerate, ``any_valid`` set otherwise).
template <typename T, int VPT, int KIND>
__global__ __launch_bounds__(kRowBlock) void ml_ranking_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                              int64_t N, int L, const float* __restrict__ shift,
                                                              float* __restrict__ out, int* __restrict__ any_valid) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t waves = (int64_t)gridDim.x * (kRowBlock / kWave);
  for (int64_t r = (int64_t)blockIdx.x * (kRowBlock / kWave) + threadIdx.x / kWave; r < N; r += waves) {
    float v[VPT];
    bool rel[VPT];
    load_row<T, VPT>(preds + r * L, L, lane, v);
    int nrel = 0;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = lane + j * kWave;
      rel[j] = c < L && target[r * L + c] == 1;
      nrel += rel[j];
    }
    nrel = static_cast<int>(wave_sum(static_cast<long long>(nrel)));
    if constexpr (KIND == 0) {
      const float g = shift[0];
      float pm = INFINITY;
#pragma unroll
      for (int j = 0; j < VPT; ++j)
        if (lane + j * kWave < L) pm = fminf(pm, rel[j] ? v[j] : round_trip<T>(v[j] + g));
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) pm = fminf(pm, __shfl_xor(pm, off, kWave));
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < VPT; ++j) cnt += (lane + j * kWave < L) && v[j] >= pm;
      cnt = static_cast<int>(wave_sum(static_cast<long long>(cnt)));
      if (lane == 0) out[r] = static_cast<float>(cnt);
    } else {
      const bool degenerate = nrel == 0 || nrel == L;
      if (degenerate) {
        if (lane == 0) out[r] = KIND == 1 ? 1.f : 0.f;
        continue;
      }
      float ratio_sum = 0.f;
      int loss_cnt = 0;
#pragma unroll
      for (int jj = 0; jj < VPT; ++jj) {
        uint64_t mask = __ballot(rel[jj]);
        while (mask) {
          const int b = __builtin_ctzll(mask);
          mask &= mask - 1;
          const float sj = __shfl(v[jj], b, kWave);
          const int idx_j = b + jj * kWave;
          if constexpr (KIND == 1) {
            int packed = 0;  // (#relevant >= sj) << 16 | (#all >= sj)
#pragma unroll
            for (int j = 0; j < VPT; ++j)
              if (lane + j * kWave < L && v[j] >= sj) packed += rel[j] ? 0x10001 : 1;
            packed = static_cast<int>(wave_sum(static_cast<long long>(packed)));
            ratio_sum += static_cast<float>(packed >> 16) / static_cast<float>(packed & 0xFFFF);
          } else {
#pragma unroll
            for (int j = 0; j < VPT; ++j) {
              const int c = lane + j * kWave;
              loss_cnt += c < L && (v[j] > sj || (v[j] == sj && c >= idx_j));
            }
          }
        }
      }
      if constexpr (KIND == 1) {
        if (lane == 0) out[r] = ratio_sum / static_cast<float>(nrel);
      } else {
        const long long tot = wave_sum(static_cast<long long>(loss_cnt));
        if (lane == 0) {
          const float corr = 0.5f * nrel * (nrel + 1);
          out[r] = (static_cast<float>(tot) - corr) / static_cast<float>(nrel * (L - nrel));
          if (any_valid) *any_valid = 1;
        }
      }
    }
  }
}

template <typename F>
void dispatch_vpt(int C, F&& f) {
  if (C <= 64) f(std::integral_constant<int, 1>{});
  else if (C <= 128) f(std::integral_constant<int, 2>{});
  else if (C <= 256) f(std::integral_constant<int, 4>{});
  else if (C <= 512) f(std::integral_constant<int, 8>{});
  else if (C <= 1024) f(std::integral_constant<int, 16>{});
  else if (C <= 2048) f(std::integral_constant<int, 32>{});
  else TORCH_CHECK(false, "row kernels hold at most 2048 classes per row, got ", C);
}

int row_grid(int64_t rows) {
  const int64_t need = (rows + kRowBlock / kWave - 1) / (kRowBlock / kWave);
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(need, 256 * 16)));
}

}  // namespace

// preds: float [M, C] scores (labels = None) or ignored when ``labels`` int64 [M] is given (k == 1).
// Returns (tp, fp, fn, nvalid): [C] x3 + [1] (global) or [S, C] x3 + [S] (samplewise, S = M / X).
std::vector<at::Tensor> topk_stats(const at::Tensor& preds, const c10::optional<at::Tensor>& labels, const at::Tensor& target,
                                   int64_t num_classes, int64_t k, int64_t ignore_index, bool has_ignore, int64_t X,
                                   bool samplewise) {
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.is_contiguous(), "topk_stats: target int64");
  const int64_t M = target.numel();
  const int C = static_cast<int>(num_classes);
  TORCH_CHECK(k >= 1 && k <= C, "topk_stats: k out of range");
  TORCH_CHECK(X >= 1 && M % X == 0, "topk_stats: rows must be a multiple of X");
  const bool use_labels = labels.has_value();
  if (use_labels) {
    TORCH_CHECK(k == 1 && labels->scalar_type() == at::kLong && labels->is_contiguous() && labels->numel() == M,
                "topk_stats: label predictions must be int64 [M] with k == 1");
  } else {
    TORCH_CHECK(preds.dim() == 2 && preds.size(0) == M && preds.size(1) == C && preds.is_contiguous(),
                "topk_stats: preds must be contiguous [M, C]");
  }
  c10::DeviceGuard guard(target.device());
  const int64_t S = samplewise ? M / X : 1;
  auto opts = target.options();
  auto buf = at::zeros({3 * S * C + S}, opts);
  int64_t* b = buf.data_ptr<int64_t>();
  const int grid = row_grid(M);
  if (M > 0) {
    const int64_t* lab = use_labels ? labels->data_ptr<int64_t>() : nullptr;
    auto run = [&](auto vpt) {
      constexpr int V = decltype(vpt)::value;
      TMX_DISPATCH_FLOAT(use_labels ? at::kFloat : preds.scalar_type(), "topk_stats", [&] {
        const scalar_t* p = use_labels ? nullptr : reinterpret_cast<const scalar_t*>(preds.data_ptr());
        hipLaunchKernelGGL((topk_stats_kernel<scalar_t, V>), grid, kRowBlock, 0, stream(), p, lab, target.data_ptr<int64_t>(), M, C,
                           static_cast<int>(k), ignore_index, has_ignore, X, samplewise, b, b + S * C, b + 2 * S * C, b + 3 * S * C);
      });
    };
    if (use_labels) run(std::integral_constant<int, 1>{});
    else dispatch_vpt(C, run);
    TMX_LAUNCH_CHECK();
  }
  std::vector<int64_t> shp = samplewise ? std::vector<int64_t>{S, C} : std::vector<int64_t>{C};
  return {buf.narrow(0, 0, S * C).view(shp), buf.narrow(0, S * C, S * C).view(shp), buf.narrow(0, 2 * S * C, S * C).view(shp),
          buf.narrow(0, 3 * S * C, S)};
}

// fp32 sum over rows of the hinge measures: [] (crammer-singer) or [C] (one-vs-all)
at::Tensor mc_hinge(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& softmax_flag, bool squared, bool one_vs_all) {
  TORCH_CHECK(preds.is_cuda() && preds.dim() == 2 && preds.is_contiguous(), "mc_hinge: preds must be contiguous [N, C] on the GPU");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == preds.size(0), "mc_hinge: target int64 [N]");
  TORCH_CHECK(softmax_flag.scalar_type() == at::kInt && softmax_flag.numel() >= 1, "mc_hinge: int32 flag");
  c10::DeviceGuard guard(preds.device());
  const int64_t N = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  const int grid = std::min(row_grid(N), 1024);
  auto partial = at::zeros({grid, one_vs_all ? C : 1}, preds.options().dtype(at::kFloat));
  if (N > 0) {
    dispatch_vpt(C, [&](auto vpt) {
      constexpr int V = decltype(vpt)::value;
      TMX_DISPATCH_FLOAT(preds.scalar_type(), "mc_hinge", [&] {
        const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
        if (one_vs_all)
          hipLaunchKernelGGL((mc_hinge_kernel<scalar_t, V, true>), grid, kRowBlock, 0, stream(), p, target.data_ptr<int64_t>(), N, C,
                             softmax_flag.data_ptr<int>(), squared, partial.data_ptr<float>());
        else
          hipLaunchKernelGGL((mc_hinge_kernel<scalar_t, V, false>), grid, kRowBlock, 0, stream(), p, target.data_ptr<int64_t>(), N, C,
                             softmax_flag.data_ptr<int>(), squared, partial.data_ptr<float>());
      });
    });
    TMX_LAUNCH_CHECK();
  }
  auto s = partial.sum(0);
  return one_vs_all ? s : s.reshape({});
}

// per-row values [N] fp32 of a multilabel ranking metric; kind 0 coverage (shift = |min| + 10 as fp32 [1]),
// 1 label-ranking AP, 2 ranking loss (``any_valid`` int32 [1] set when a non-degenerate row exists).
at::Tensor ml_ranking(const at::Tensor& preds, const at::Tensor& target, int64_t kind, const c10::optional<at::Tensor>& shift,
                      const c10::optional<at::Tensor>& any_valid) {
  TORCH_CHECK(preds.is_cuda() && preds.dim() == 2 && preds.is_contiguous(), "ml_ranking: preds must be contiguous [N, L] on the GPU");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.sizes() == preds.sizes(), "ml_ranking: target int64 [N, L]");
  TORCH_CHECK(kind >= 0 && kind <= 2, "ml_ranking: kind");
  TORCH_CHECK(kind != 0 || (shift.has_value() && shift->scalar_type() == at::kFloat), "ml_ranking: coverage needs an fp32 shift");
  TORCH_CHECK(preds.size(1) < 65536, "ml_ranking: too many labels");
  c10::DeviceGuard guard(preds.device());
  const int64_t N = preds.size(0);
  const int L = static_cast<int>(preds.size(1));
  auto out = at::empty({N}, preds.options().dtype(at::kFloat));
  if (N == 0) return out;
  const float* sh = kind == 0 ? shift->data_ptr<float>() : nullptr;
  int* av = any_valid.has_value() ? any_valid->data_ptr<int>() : nullptr;
  const int grid = row_grid(N);
  dispatch_vpt(L, [&](auto vpt) {
    constexpr int V = decltype(vpt)::value;
    TMX_DISPATCH_FLOAT(preds.scalar_type(), "ml_ranking", [&] {
      const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
      const int64_t* t = target.data_ptr<int64_t>();
      if (kind == 0) hipLaunchKernelGGL((ml_ranking_kernel<scalar_t, V, 0>), grid, kRowBlock, 0, stream(), p, t, N, L, sh, out.data_ptr<float>(), av);
      else if (kind == 1) hipLaunchKernelGGL((ml_ranking_kernel<scalar_t, V, 1>), grid, kRowBlock, 0, stream(), p, t, N, L, sh, out.data_ptr<float>(), av);
      else hipLaunchKernelGGL((ml_ranking_kernel<scalar_t, V, 2>), grid, kRowBlock, 0, stream(), p, t, N, L, sh, out.data_ptr<float>(), av);
    });
  });
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("topk_stats(Tensor preds, Tensor? labels, Tensor target, int num_classes, int k, int ignore_index, bool has_ignore, int X, bool samplewise) -> Tensor[]");
  m.def("mc_hinge(Tensor preds, Tensor target, Tensor softmax_flag, bool squared, bool one_vs_all) -> Tensor");
  m.def("ml_ranking(Tensor preds, Tensor target, int kind, Tensor? shift=None, Tensor(a!)? any_valid=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("topk_stats", &tmx::topk_stats);
  m.impl("mc_hinge", &tmx::mc_hinge);
  m.impl("ml_ranking", &tmx::ml_ranking);
}
