// Segmented retrieval scoring (K16) for gfx950: one 64-lane wave per query over its documents, already laid out
// contiguously and sorted by descending score (functional/retrieval/_grouped.py ``Grouped``).
//
// Reference: retrieval/base.py:114-141 sorts by query, splits on the host and calls a per-query functional in a Python
// loop (functional/retrieval/{average_precision,reciprocal_rank,precision,recall,fall_out,hit_rate,r_precision,
// ndcg}.py).  Here every statistic those metrics need comes out of two sweeps of the query in 64-document chunks:
//   sweep 1: relevant / non-relevant totals (ballot popcounts);
//   sweep 2: relevant and non-relevant in the top k, the AP numerator (running relevant count from a ballot prefix),
//            the first relevant rank, relevant within the top R (R-precision), the tie-averaged DCG and the ideal DCG.
// Tie-averaged DCG: a document in a run [a, b) of equal scores contributes t * (D[min(b,k)] - D[min(a,k)]) / (b - a),
// D = prefix sums of 1 / log2(p + 2) (a table from the host, fp64); runs are found from the neighbours and, only
// when a neighbour ties, by binary search inside the query (NaN scores are singleton runs).
//
// Output: float64 [Q, 10] = (rel_total, neg_total, rel_in_k, neg_in_k, ap_sum, first_rel (-1 none), rel_in_R, dcg,
// idcg, k).
#include "common.h"

namespace tmx {
namespace {

constexpr int kQBlock = 256;
constexpr int kStats = 10;

template <typename T>
__device__ __forceinline__ int64_t run_first(const T* __restrict__ p, int64_t i, T v) {
  // descending order: first index j <= i with p[j] == v  (p[0 .. i] holds values >= v)
  int64_t lo = 0, hi = i;
  while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (p[m] > v) lo = m + 1; else hi = m; }
  return lo;
}
template <typename T>
__device__ __forceinline__ int64_t run_end(const T* __restrict__ p, int64_t i, int64_t n, T v) {
  int64_t lo = i + 1, hi = n;
  while (lo < hi) { const int64_t m = (lo + hi) >> 1; if (p[m] >= v) lo = m + 1; else hi = m; }
  return lo;
}

template <typename T, typename TT>
__global__ __launch_bounds__(kQBlock) void retrieval_segments_kernel(const T* __restrict__ preds, const TT* __restrict__ target,
                                                                    const TT* __restrict__ ideal, const int64_t* __restrict__ start,
                                                                    const int64_t* __restrict__ sizes, int64_t Q, int64_t top_k,
                                                                    bool adaptive, const double* __restrict__ dtab,
                                                                    double* __restrict__ out) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t waves = (int64_t)gridDim.x * (kQBlock / kWave);
  for (int64_t q = (int64_t)blockIdx.x * (kQBlock / kWave) + threadIdx.x / kWave; q < Q; q += waves) {
    const int64_t s0 = start[q], n = sizes[q];
    const T* p = preds + s0;
    const TT* t = target + s0;
    const int64_t k = top_k < 0 ? n : (adaptive ? min(top_k, n) : top_k);
    // sweep 1: totals
    long long rel_total = 0, neg_total = 0;
    for (int64_t b = 0; b < n; b += kWave) {
      const int64_t i = b + lane;
      const bool valid = i < n;
      const float tv = valid ? static_cast<float>(t[i]) : 0.f;
      rel_total += __popcll(__ballot(valid && tv > 0.f));
      neg_total += __popcll(__ballot(valid && !(tv > 0.f)));
    }
    // sweep 2
    long long rel_k = 0, neg_k = 0, rel_R = 0, carry = 0;
    long long first = -1;
    float ap = 0.f, dcg = 0.f, idcg = 0.f;
    const int64_t kk = min(k, n);
    for (int64_t b = 0; b < n; b += kWave) {
      const int64_t i = b + lane;
      const bool valid = i < n;
      const float tv = valid ? static_cast<float>(t[i]) : 0.f;
      const bool r = valid && tv > 0.f;
      const uint64_t rm = __ballot(r);
      const bool in_k = i < k;
      const uint64_t rk = __ballot(r && in_k);
      rel_k += __popcll(rk);
      neg_k += __popcll(__ballot(valid && !r && in_k));
      rel_R += __popcll(__ballot(r && i < rel_total));
      if (first < 0 && rk) first = b + __builtin_ctzll(rk);
      if (r && in_k) ap += static_cast<float>(carry + __popcll(rm & lt_mask) + 1) / static_cast<float>(i + 1);
      carry += __popcll(rm);
      if (valid && i < kk) {
        // tie run of document i inside the query
        const T v = p[i];
        const bool tie_prev = i > 0 && p[i - 1] == v, tie_next = i + 1 < n && p[i + 1] == v;
        const int64_t a = tie_prev ? run_first(p, i, v) : i;
        const int64_t e = tie_next ? run_end(p, i, n, v) : i + 1;
        const double sd = dtab[min(e, kk)] - dtab[min(a, kk)];
        dcg += tv * static_cast<float>(sd / static_cast<double>(e - a));
        idcg += static_cast<float>(ideal[s0 + i]) * static_cast<float>(dtab[i + 1] - dtab[i]);
      } else if (valid && !(i < kk)) {
        // documents below the cut-off still share the DCG of a run that straddles it
        const T v = p[i];
        if (kk > 0 && p[kk - 1] == v) {
          const int64_t a = run_first(p, i, v);
          const int64_t e = (i + 1 < n && p[i + 1] == v) ? run_end(p, i, n, v) : i + 1;
          const double sd = dtab[min(e, kk)] - dtab[min(a, kk)];
          dcg += tv * static_cast<float>(sd / static_cast<double>(e - a));
        }
      }
    }
    ap = wave_sum(ap);
    dcg = wave_sum(dcg);
    idcg = wave_sum(idcg);
    if (lane == 0) {
      double* o = out + q * kStats;
      o[0] = static_cast<double>(rel_total);
      o[1] = static_cast<double>(neg_total);
      o[2] = static_cast<double>(rel_k);
      o[3] = static_cast<double>(neg_k);
      o[4] = ap;
      o[5] = static_cast<double>(first);
      o[6] = static_cast<double>(rel_R);
      o[7] = dcg;
      o[8] = idcg;
      o[9] = static_cast<double>(k);
    }
  }
}

}  // namespace

at::Tensor retrieval_segments(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& ideal, const at::Tensor& start,
                              const at::Tensor& sizes, int64_t top_k, bool adaptive, const at::Tensor& dtab) {
  TORCH_CHECK(preds.is_cuda() && preds.dim() == 1 && preds.is_contiguous(), "retrieval_segments: 1-D sorted preds on the GPU");
  TORCH_CHECK(target.sizes() == preds.sizes() && ideal.sizes() == preds.sizes() && target.is_contiguous() && ideal.is_contiguous(),
              "retrieval_segments: target / ideal like preds");
  TORCH_CHECK(target.scalar_type() == ideal.scalar_type(), "retrieval_segments: target / ideal dtype");
  TORCH_CHECK(start.scalar_type() == at::kLong && sizes.scalar_type() == at::kLong && start.numel() == sizes.numel(),
              "retrieval_segments: int64 start / sizes");
  TORCH_CHECK(dtab.scalar_type() == at::kDouble && dtab.is_contiguous(), "retrieval_segments: fp64 discount prefix table");
  c10::DeviceGuard guard(preds.device());
  const int64_t Q = start.numel();
  auto out = at::empty({Q, kStats}, preds.options().dtype(at::kDouble));
  if (Q == 0) return out;
  const int grid = grid_for(Q, kQBlock / kWave, 256 * 16);
  auto launch_t = [&](auto tag_p) {
    using PT = decltype(tag_p);
    auto go = [&](auto tag_t) {
      using TT = decltype(tag_t);
      hipLaunchKernelGGL((retrieval_segments_kernel<PT, TT>), grid, kQBlock, 0, stream(), reinterpret_cast<const PT*>(preds.data_ptr()),
                         reinterpret_cast<const TT*>(target.data_ptr()), reinterpret_cast<const TT*>(ideal.data_ptr()),
                         start.data_ptr<int64_t>(), sizes.data_ptr<int64_t>(), Q, top_k, adaptive, dtab.data_ptr<double>(),
                         out.data_ptr<double>());
    };
    switch (target.scalar_type()) {
      case at::kFloat: go(float{}); break;
      case at::kDouble: go(double{}); break;
      case at::kLong: go(int64_t{}); break;
      case at::kInt: go(int32_t{}); break;
      default: TORCH_CHECK(false, "retrieval_segments: target dtype ", target.scalar_type());
    }
  };
  switch (preds.scalar_type()) {
    case at::kFloat: launch_t(float{}); break;
    case at::kDouble: launch_t(double{}); break;
    default: TORCH_CHECK(false, "retrieval_segments: preds must be float32 / float64");
  }
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("retrieval_segments(Tensor preds, Tensor target, Tensor ideal, Tensor start, Tensor sizes, int top_k, bool adaptive, Tensor dtab) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("retrieval_segments", &tmx::retrieval_segments); }
