// GPU twins of the host text kernels that still ran on the CPU (verdict r2 "next" #7):
//
// ``levenshtein_beam_gpu`` — EditDistance's beam-restricted weighted DP (see the kernel below).
//
// ``eed_gpu`` — extended edit distance (reference functional/text/eed.py:116-171).  Each reference row of the DP
// ends with a row-wide arg-min (coverage visits) and an optional long jump that rewrites the whole row, so rows are
// strictly sequential, and inside a row next[i] = min(next[i-1] + deletion, ...) chains the cells: no parallel
// scan reproduces that fp64 rounding (and the arg-min tie order) exactly.  One THREAD therefore runs one pair's DP
// with exactly the host op's operation order (bit-identical results), and the parallelism is across pairs: the two
// DP rows live in a global scratch interleaved by pair (element i of pair t at [i * P + t]), so the lanes of a wave
// walking the same column touch one cache line per 8 pairs.
//
// ``ngram_overlap_gpu`` — clipped n-gram overlap per (hypothesis, reference) pair and order n <= n_order (chrF /
// chrF++ / ROUGE-N; host op ``ngram_overlap`` in text.cpp).  Token ids are remapped to a dense range by the caller,
// so an n-gram of n <= 128 / bits ids packs exactly into a 128-bit key (two u64) and n-grams compare as integers.
// One wave per hypothesis (as ``bleu_stats_gpu``): lane l owns hypothesis positions l + 64 k; per order the wave
// counts each n-gram inside the hypothesis and marks first occurrences (keys broadcast by lane shuffles), then
// streams each reference of the group (wave-uniform loads) counting matches per hypothesis n-gram, and reduces
// sum(min(hyp count, ref count)) over first occurrences.
#include "common.h"

namespace tmx {

// ------------------------------------------------------------------------------------------------------------ EED
__device__ __forceinline__ double dmin(double a, double b) { return b < a ? b : a; }  // std::min(a, b)

__global__ __launch_bounds__(256) void eed_pair_kernel(const int64_t* __restrict__ hyp, const int64_t* __restrict__ hyp_off,
                                                      const int64_t* __restrict__ ref, const int64_t* __restrict__ ref_off,
                                                      int64_t P, int64_t space, double alpha, double rho, double deletion,
                                                      double insertion, double* __restrict__ rows, int32_t* __restrict__ visits,
                                                      int64_t stride_n, double* __restrict__ out) {
  // no mul+add contraction (HIP's default fp-contract=fast would fuse cov * rho + row[n] into one FMA): the host op
  // rounds every operation, and the scores must be bit-identical
#pragma clang fp contract(off)
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= P) return;
  const int64_t* h = hyp + hyp_off[t];
  const int64_t n = hyp_off[t + 1] - hyp_off[t];
  const int64_t* r = ref + ref_off[t];
  const int64_t m = ref_off[t + 1] - ref_off[t];
  double* A = rows;                  // row:  A[i * P + t]
  double* B = rows + stride_n * P;   // next: B[i * P + t]
  for (int64_t i = 0; i <= n; ++i) {
    A[i * P + t] = i == 0 ? 0.0 : 1.0;
    visits[i * P + t] = -1;
  }
  for (int64_t w = 1; w <= m; ++w) {
    const int64_t rc = r[w - 1];
    double prev_next = A[t] + 1.0;  // next[0] = row[0] + 1
    B[t] = prev_next;
    double best = prev_next;
    int64_t mi = 0;
    double row_im1 = A[t];
    for (int64_t i = 1; i <= n; ++i) {
      const double row_i = A[i * P + t];
      const double sub = row_im1 + (h[i - 1] != rc ? 1.0 : 0.0);
      const double v = dmin(dmin(prev_next + deletion, sub), row_i + insertion);
      B[i * P + t] = v;
      if (v < best) {
        best = v;
        mi = i;
      }
      prev_next = v;
      row_im1 = row_i;
    }
    visits[mi * P + t] += 1;
    if (rc == space) {
      const double jump = alpha + best;
      for (int64_t i = 0; i <= n; ++i) B[i * P + t] = dmin(B[i * P + t], jump);
    }
    double* tmp = A;
    A = B;
    B = tmp;
  }
  double cov = 0.0;
  for (int64_t i = 0; i <= n; ++i) {
    const int v = visits[i * P + t];
    cov += v >= 0 ? static_cast<double>(v) : 1.0;
  }
  cov *= rho;
  const double fin = A[n * P + t];
  out[t] = dmin(1.0, (fin + cov) / (static_cast<double>(m) + cov));
}

// hyp / ref: flat int64 codepoints (GPU) + offsets [P + 1] (one pair per (hypothesis, reference)); returns fp64 [P]
at::Tensor eed_gpu(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref, const at::Tensor& ref_off, int64_t space,
                   double alpha, double rho, double deletion, double insertion, int64_t max_hyp_len) {
  for (const at::Tensor* x : {&hyp, &hyp_off, &ref, &ref_off})
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kLong, "eed_gpu: expected int64 GPU tensors");
  TORCH_CHECK(hyp_off.numel() == ref_off.numel(), "eed_gpu: pair count mismatch");
  const c10::DeviceGuard guard(hyp.device());
  const int64_t P = hyp_off.numel() - 1;
  auto out = at::empty({std::max<int64_t>(P, 0)}, hyp.options().dtype(at::kDouble));
  if (P <= 0) return out;
  {  // every pair's DP row must fit its scratch column: checked against the offsets (one small host read)
    auto hc = hyp_off.cpu();
    const int64_t* o = hc.data_ptr<int64_t>();
    int64_t mx = 0;
    for (int64_t k = 0; k < P; ++k) mx = std::max(mx, o[k + 1] - o[k]);
    TORCH_CHECK(mx <= max_hyp_len && mx >= 0, "eed_gpu: a hypothesis is longer than max_hyp_len (", mx, " > ", max_hyp_len, ")");
  }
  const int64_t stride_n = max_hyp_len + 1;
  auto rows = at::empty({2 * stride_n * P}, hyp.options().dtype(at::kDouble));
  auto vis = at::empty({stride_n * P}, hyp.options().dtype(at::kInt));
  const auto h = hyp.contiguous(), ho = hyp_off.contiguous(), r = ref.contiguous(), ro = ref_off.contiguous();
  hipLaunchKernelGGL(eed_pair_kernel, dim3(static_cast<unsigned>((P + 255) / 256)), 256, 0, stream(), h.data_ptr<int64_t>(),
                     ho.data_ptr<int64_t>(), r.data_ptr<int64_t>(), ro.data_ptr<int64_t>(), P, space, alpha, rho, deletion, insertion,
                     rows.data_ptr<double>(), vis.data_ptr<int32_t>(), stride_n, out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

// ------------------------------------------------------------------------------------- beam edit distance (EditDistance)
// Tercom's beam-restricted weighted Levenshtein DP (host op lev_beam in text.cpp; reference functional/text/edit.py ->
// helper._LevenshteinEditDistance): row i only fills the band [max(0, diag - beam), min(m + 1, diag + beam)) around
// diag = floor(i m / n) (the whole row for i = n), every other cell is 1e16.  One thread per pair with one DP row in
// an interleaved global scratch (element j of pair t at [j P + t]); the row keeps the invariant "row i - 1 on its
// band, 1e16 elsewhere": the band only moves right, so after row i the cells of the old band left of the new one
// (and right of it, after the full row 0) are reset.  Integer arithmetic in the host op's order: identical results.
constexpr int64_t kBeamInf = 10000000000000000LL;  // text.cpp kInf
constexpr int64_t kBeamWidth = 25;                  // text.cpp kBeam

__global__ __launch_bounds__(256) void edit_beam_kernel(const int64_t* __restrict__ pred, const int64_t* __restrict__ pred_off,
                                                       const int64_t* __restrict__ ref, const int64_t* __restrict__ ref_off,
                                                       int64_t P, int64_t ins, int64_t del, int64_t sub, int64_t* __restrict__ row,
                                                       int64_t* __restrict__ out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= P) return;
  const int64_t* a = pred + pred_off[t];
  const int64_t n = pred_off[t + 1] - pred_off[t];
  const int64_t* b = ref + ref_off[t];
  const int64_t m = ref_off[t + 1] - ref_off[t];
  auto R = [&](int64_t j) -> int64_t& { return row[j * P + t]; };
  for (int64_t j = 0; j <= m; ++j) R(j) = j * ins;
  const double ratio = n ? static_cast<double>(m) / static_cast<double>(n) : 1.0;
  const int64_t beam = (ratio / 2 > kBeamWidth) ? static_cast<int64_t>(ceil(ratio / 2 + kBeamWidth)) : kBeamWidth;
  int64_t plo = 0, phi = m + 1;  // band of the row held in R
  for (int64_t i = 1; i <= n; ++i) {
    const int64_t diag = static_cast<int64_t>(floor(static_cast<double>(i) * ratio));
    const int64_t lo = diag - beam > 0 ? diag - beam : 0;
    const int64_t hi = (i == n) ? m + 1 : (diag + beam < m + 1 ? diag + beam : m + 1);
    const int64_t ai = a[i - 1];
    int64_t up_left = lo >= 1 ? R(lo - 1) : kBeamInf;  // row i - 1, column j - 1 (not yet overwritten)
    int64_t left = kBeamInf;                            // row i, column j - 1 (outside the band: 1e16)
    for (int64_t j = lo; j < hi; ++j) {
      const int64_t up = R(j);
      int64_t c;
      if (j == 0) {
        c = up + del;
      } else {
        c = kBeamInf;
        const int64_t cs = up_left + (ai == b[j - 1] ? 0 : sub);
        const int64_t cd = up + del;
        const int64_t ci = left + ins;
        if (c > cs) c = cs;
        if (c > cd) c = cd;
        if (c > ci) c = ci;
      }
      R(j) = c;
      up_left = up;
      left = c;
    }
    for (int64_t j = plo; j < lo && j < phi; ++j) R(j) = kBeamInf;
    for (int64_t j = hi > plo ? hi : plo; j < phi; ++j) R(j) = kBeamInf;
    plo = lo;
    phi = hi;
  }
  out[t] = R(m);
}

// pred / ref: flat int64 codepoints (GPU) + offsets [P + 1]; returns int64 [P] distances (insertion / deletion / sub costs)
at::Tensor levenshtein_beam_gpu(const at::Tensor& pred, const at::Tensor& pred_off, const at::Tensor& ref, const at::Tensor& ref_off,
                                int64_t ins, int64_t del, int64_t sub, int64_t max_ref_len) {
  for (const at::Tensor* x : {&pred, &pred_off, &ref, &ref_off})
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kLong, "levenshtein_beam_gpu: expected int64 GPU tensors");
  TORCH_CHECK(pred_off.numel() == ref_off.numel(), "levenshtein_beam_gpu: pair count mismatch");
  const c10::DeviceGuard guard(pred.device());
  const int64_t P = pred_off.numel() - 1;
  auto out = at::empty({std::max<int64_t>(P, 0)}, pred.options());
  if (P <= 0) return out;
  {  // every pair's DP row must fit its scratch column (one small host read of the offsets)
    auto rc = ref_off.cpu();
    const int64_t* o = rc.data_ptr<int64_t>();
    int64_t mx = 0;
    for (int64_t k = 0; k < P; ++k) mx = std::max(mx, o[k + 1] - o[k]);
    TORCH_CHECK(mx <= max_ref_len && mx >= 0, "levenshtein_beam_gpu: a reference is longer than max_ref_len (", mx, " > ", max_ref_len, ")");
  }
  auto row = at::empty({(max_ref_len + 1) * P}, pred.options());
  const auto a = pred.contiguous(), ao = pred_off.contiguous(), b = ref.contiguous(), bo = ref_off.contiguous();
  hipLaunchKernelGGL(edit_beam_kernel, dim3(static_cast<unsigned>((P + 255) / 256)), 256, 0, stream(), a.data_ptr<int64_t>(),
                     ao.data_ptr<int64_t>(), b.data_ptr<int64_t>(), bo.data_ptr<int64_t>(), P, ins, del, sub, row.data_ptr<int64_t>(),
                     out.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  return out;
}

// ------------------------------------------------------------------------------------------------ n-gram overlap
constexpr int kNgSlots = 8;  // hypotheses up to 512 tokens on this path
constexpr int kNgWaves = 4;

struct Key128 {
  uint64_t hi, lo;
};
__device__ __forceinline__ bool key_eq(const Key128& a, const Key128& b) { return a.hi == b.hi && a.lo == b.lo; }

// n-gram starting at pos: ids + 1 (0 = padding) in `bits`-bit fields, first token most significant, across 128 bits
__device__ __forceinline__ Key128 ngram_key128(const int64_t* __restrict__ t, int64_t pos, int n, int bits) {
  Key128 k{0ull, 0ull};
  for (int j = 0; j < n; ++j) {
    const uint64_t v = static_cast<uint64_t>(t[pos + j] + 1);
    k.hi = bits >= 64 ? k.lo : ((k.hi << bits) | (k.lo >> (64 - bits)));
    k.lo = bits >= 64 ? v : ((k.lo << bits) | v);
  }
  return k;
}

__global__ __launch_bounds__(kNgWaves * kWave) void ngram_overlap_wave_kernel(
    const int64_t* __restrict__ hyp, const int64_t* __restrict__ hyp_off, const int64_t* __restrict__ ref,
    const int64_t* __restrict__ ref_off, const int64_t* __restrict__ group_off, int64_t nhyp, int n_order, int bits,
    int64_t* __restrict__ match, int64_t* __restrict__ htot, int64_t* __restrict__ rtot) {
  const int lane = threadIdx.x % kWave;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kNgWaves + threadIdx.x / kWave;
  if (i >= nhyp) return;  // wave-uniform
  const int64_t h0 = hyp_off[i], hl = hyp_off[i + 1] - h0;
  const int64_t g0 = group_off[i], g1 = group_off[i + 1];
  for (int n = 1; n <= n_order; ++n) {
    const int64_t ng = hl - n + 1;
    if (lane == 0) htot[i * n_order + n - 1] = ng > 0 ? ng : 0;
    Key128 key[kNgSlots];
    int cnt[kNgSlots];
    bool first[kNgSlots];
#pragma unroll
    for (int k = 0; k < kNgSlots; ++k) {
      const int64_t p = lane + 64 * k;
      key[k] = p < ng ? ngram_key128(hyp + h0, p, n, bits) : Key128{0ull, 0ull};
      cnt[k] = 0;
      first[k] = true;
    }
    // counts inside the hypothesis + first occurrences
#pragma unroll
    for (int kq = 0; kq < kNgSlots; ++kq) {
      if (64 * kq >= ng) break;
      for (int ql = 0; ql < kWave && 64 * kq + ql < ng; ++ql) {
        const Key128 kv{__shfl(key[kq].hi, ql, kWave), __shfl(key[kq].lo, ql, kWave)};
        const int64_t q = 64 * kq + ql;
#pragma unroll
        for (int k = 0; k < kNgSlots; ++k) {
          const int64_t p = lane + 64 * k;
          if (p < ng && key_eq(key[k], kv)) {
            ++cnt[k];
            if (q < p) first[k] = false;
          }
        }
      }
    }
    for (int64_t r = g0; r < g1; ++r) {
      const int64_t r0 = ref_off[r], rng = ref_off[r + 1] - r0 - n + 1;
      if (lane == 0) rtot[r * n_order + n - 1] = rng > 0 ? rng : 0;
      int cur[kNgSlots];
#pragma unroll
      for (int k = 0; k < kNgSlots; ++k) cur[k] = 0;
      for (int64_t q = 0; q < rng; ++q) {
        const Key128 kr = ngram_key128(ref + r0, q, n, bits);  // wave-uniform loads
#pragma unroll
        for (int k = 0; k < kNgSlots; ++k) cur[k] += key_eq(key[k], kr) ? 1 : 0;
      }
      int clipped = 0;
#pragma unroll
      for (int k = 0; k < kNgSlots; ++k) {
        const int64_t p = lane + 64 * k;
        if (p < ng && first[k]) clipped += min(cnt[k], cur[k]);
      }
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) clipped += __shfl_xor(clipped, off, kWave);
      if (lane == 0) match[r * n_order + n - 1] = clipped;
    }
  }
}

// hyp / ref: dense token ids (GPU int64, < 2^bits - 1), offsets; ref_group_off [nhyp + 1].  Same outputs as the host
// ``ngram_overlap``: match [nref, n_order], hyp_tot [nhyp, n_order], ref_tot [nref, n_order] (int64, on the GPU).
std::tuple<at::Tensor, at::Tensor, at::Tensor> ngram_overlap_gpu(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref,
                                                                 const at::Tensor& ref_off, const at::Tensor& group_off, int64_t n_order,
                                                                 int64_t bits, int64_t max_hyp_len) {
  for (const at::Tensor* x : {&hyp, &hyp_off, &ref, &ref_off, &group_off})
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kLong, "ngram_overlap_gpu: expected int64 GPU tensors");
  TORCH_CHECK(n_order >= 1 && bits >= 1 && bits <= 64 && n_order * bits <= 128, "ngram_overlap_gpu: n_order x bits must fit 128 bits");
  TORCH_CHECK(max_hyp_len <= 64 * kNgSlots, "ngram_overlap_gpu: hypothesis longer than ", 64 * kNgSlots, " tokens");
  TORCH_CHECK(group_off.numel() == hyp_off.numel(), "ngram_overlap_gpu: group offsets must have n + 1 entries");
  const c10::DeviceGuard guard(hyp.device());
  const int64_t nh = hyp_off.numel() - 1, nr = ref_off.numel() - 1;
  {  // hypotheses longer than the slots would silently drop n-grams
    auto hc = hyp_off.cpu();
    const int64_t* o = hc.data_ptr<int64_t>();
    for (int64_t k = 0; k < nh; ++k)
      TORCH_CHECK(o[k + 1] - o[k] <= std::min<int64_t>(max_hyp_len, 64 * kNgSlots), "ngram_overlap_gpu: hypothesis too long");
  }
  auto opts = hyp.options();
  auto match = at::zeros({std::max<int64_t>(nr, 0), n_order}, opts), htot = at::zeros({std::max<int64_t>(nh, 0), n_order}, opts);
  auto rtot = at::zeros({std::max<int64_t>(nr, 0), n_order}, opts);
  if (nh <= 0) return {match, htot, rtot};
  const auto h = hyp.contiguous(), ho = hyp_off.contiguous(), r = ref.contiguous(), ro = ref_off.contiguous(), go = group_off.contiguous();
  const unsigned grid = static_cast<unsigned>((nh + kNgWaves - 1) / kNgWaves);
  hipLaunchKernelGGL(ngram_overlap_wave_kernel, dim3(grid), kNgWaves * kWave, 0, stream(), h.data_ptr<int64_t>(), ho.data_ptr<int64_t>(),
                     r.data_ptr<int64_t>(), ro.data_ptr<int64_t>(), go.data_ptr<int64_t>(), nh, static_cast<int>(n_order),
                     static_cast<int>(bits), match.data_ptr<int64_t>(), htot.data_ptr<int64_t>(), rtot.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  return {match, htot, rtot};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("eed_gpu(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, int space, float alpha, float rho, float deletion, "
        "float insertion, int max_hyp_len) -> Tensor");
  m.def("ngram_overlap_gpu(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, Tensor ref_group_off, int n_order, int bits, "
        "int max_hyp_len) -> (Tensor, Tensor, Tensor)");
  m.def("levenshtein_beam_gpu(Tensor pred, Tensor pred_off, Tensor ref, Tensor ref_off, int ins, int dele, int sub, int max_ref_len) "
        "-> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("eed_gpu", &tmx::eed_gpu);
  m.impl("ngram_overlap_gpu", &tmx::ngram_overlap_gpu);
  m.impl("levenshtein_beam_gpu", &tmx::levenshtein_beam_gpu);
}
