// Batched exact Levenshtein distance and LCS on the GPU for WER / CER / MER / WIL / WIP and ROUGE-L.
//
// The reference runs the edit-distance DP in pure Python per sentence pair (functional/text/helper.py:329-350).
// Here one wave scores one pair with Myers' bit-parallel algorithm in Hyyrö's multi-word form: the reference
// sequence is the bit pattern (64 positions per word, up to kMaxWords words held in lane registers) and the
// prediction is streamed token by token.  For every streamed token the match mask of each pattern word is a single
// wave ballot (lane l compares pattern position 64 k + l), so building Peq costs one instruction instead of a
// hash-map lookup; the column update itself is ~15 wave-uniform 64-bit operations per word with the horizontal
// delta carried from word to word.  Sentences arrive tokenised to int64 ids as a flat buffer + offsets (the same
// packing as the host kernels in text.cpp), so the H2D copy is one buffer per side and the distances stay on the
// device, where the metric states live.
#include "common.h"

namespace tmx {

constexpr int kLevMaxWords = 16;  // reference length <= 1024 tokens on this path
constexpr int kLevWaves = 4;

__global__ __launch_bounds__(kLevWaves * kWave) void levenshtein_wave_kernel(const int64_t* __restrict__ a, const int64_t* __restrict__ a_off,
                                                                            const int64_t* __restrict__ b, const int64_t* __restrict__ b_off,
                                                                            int64_t npairs, int64_t* __restrict__ out) {
  const int lane = threadIdx.x % kWave;
  const int64_t pair = static_cast<int64_t>(blockIdx.x) * kLevWaves + threadIdx.x / kWave;
  if (pair >= npairs) return;  // wave-uniform
  const int64_t a0 = a_off[pair], n = a_off[pair + 1] - a0;
  const int64_t b0 = b_off[pair], m = b_off[pair + 1] - b0;
  if (m == 0 || n == 0) {
    if (lane == 0) out[pair] = m + n;
    return;
  }
  const int words = static_cast<int>((m + 63) / 64);
  // pattern tokens of every word in registers (lane l: position 64 k + l); -1 never equals a token id
  int64_t pat[kLevMaxWords];
#pragma unroll
  for (int k = 0; k < kLevMaxWords; ++k) {
    const int64_t pos = 64 * k + lane;
    pat[k] = (k < words && pos < m) ? b[b0 + pos] : -1;
  }
  uint64_t pv[kLevMaxWords], mv[kLevMaxWords];
#pragma unroll
  for (int k = 0; k < kLevMaxWords; ++k) {
    const int64_t bits = m - 64 * k;
    pv[k] = bits >= 64 ? ~0ull : (bits > 0 ? ((1ull << bits) - 1) : 0ull);
    mv[k] = 0ull;
  }
  const uint64_t last_bit = 1ull << ((m - 1) % 64);
  int64_t score = m;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t c = a[a0 + i];
    int hin = 1;  // global distance: the top row grows by one per column
#pragma unroll
    for (int k = 0; k < kLevMaxWords; ++k) {
      if (k >= words) break;
      uint64_t eq = __ballot(pat[k] == c);
      const uint64_t xv = eq | mv[k];
      if (hin < 0) eq |= 1ull;
      const uint64_t xh = (((eq & pv[k]) + pv[k]) ^ pv[k]) | eq;
      uint64_t ph = mv[k] | ~(xh | pv[k]);
      uint64_t mh = pv[k] & xh;
      const uint64_t high = (k == words - 1) ? last_bit : (1ull << 63);
      int hout = (ph & high) ? 1 : ((mh & high) ? -1 : 0);
      ph <<= 1;
      mh <<= 1;
      if (hin < 0) mh |= 1ull;
      else if (hin > 0) ph |= 1ull;
      pv[k] = mh | ~(xv | ph);
      mv[k] = ph & xv;
      hin = hout;
    }
    score += hin;
  }
  if (lane == 0) out[pair] = score;
}

// Longest common subsequence (ROUGE-L), same layout: one wave per pair, Allison-Dix / Hyyro bit-vector LCS in the
// multi-word form V' = (V + (V & Peq)) | (V & ~Peq) — the match mask of each 64-position pattern word is one ballot,
// the addition's carry ripples from word to word (wave-uniform scalars), LCS = m - popcount(V).
__global__ __launch_bounds__(kLevWaves * kWave) void lcs_wave_kernel(const int64_t* __restrict__ a, const int64_t* __restrict__ a_off,
                                                                    const int64_t* __restrict__ b, const int64_t* __restrict__ b_off,
                                                                    int64_t npairs, int64_t* __restrict__ out) {
  const int lane = threadIdx.x % kWave;
  const int64_t pair = static_cast<int64_t>(blockIdx.x) * kLevWaves + threadIdx.x / kWave;
  if (pair >= npairs) return;  // wave-uniform
  const int64_t a0 = a_off[pair], n = a_off[pair + 1] - a0;
  const int64_t b0 = b_off[pair], m = b_off[pair + 1] - b0;
  if (m == 0 || n == 0) {
    if (lane == 0) out[pair] = 0;
    return;
  }
  const int words = static_cast<int>((m + 63) / 64);
  int64_t pat[kLevMaxWords];
  uint64_t v[kLevMaxWords];
  const uint64_t last = (m % 64) ? ((1ull << (m % 64)) - 1) : ~0ull;
#pragma unroll
  for (int k = 0; k < kLevMaxWords; ++k) {
    const int64_t pos = 64 * k + lane;
    pat[k] = (k < words && pos < m) ? b[b0 + pos] : -1;
    v[k] = k < words - 1 ? ~0ull : (k == words - 1 ? last : 0ull);
  }
  for (int64_t i = 0; i < n; ++i) {
    const int64_t c = a[a0 + i];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < kLevMaxWords; ++k) {
      if (k >= words) break;
      const uint64_t eq = __ballot(pat[k] == c);  // padding positions hold -1: never a token id
      const uint64_t u = v[k] & eq;
      const uint64_t s1 = v[k] + u;
      const uint64_t s2 = s1 + carry;
      carry = (s1 < v[k]) | (s2 < s1);
      v[k] = s2 | (v[k] & ~eq);
    }
  }
  int ones = 0;
#pragma unroll
  for (int k = 0; k < kLevMaxWords; ++k) {
    if (k >= words) break;
    ones += __popcll(k == words - 1 ? (v[k] & last) : v[k]);
  }
  if (lane == 0) out[pair] = m - ones;
}

// BLEU sufficient statistics, one wave per hypothesis: the same outputs as the host op
// ``bleu_stats`` (text.cpp).  An n-gram (n <= 4) of token ids < 65535 packs exactly into 64 bits ((id + 1) per 16-bit
// field), so n-grams compare as integers.  Lane l owns hypothesis positions l + 64 k (k < kBleuSlots); for every
// order n the wave (1) counts each of its n-grams inside the hypothesis and marks first occurrences (the keys are
// broadcast position by position with lane shuffles), (2) streams every reference of the group position by position
// (wave-uniform loads) and keeps, per hypothesis n-gram, the maximum count over the references, and (3) sums
// min(count, max reference count) over first occurrences — the clipped matches — with one wave reduction.
constexpr int kBleuSlots = 4;  // hypotheses up to 256 tokens on this path

__device__ __forceinline__ uint64_t gram_key(const int64_t* __restrict__ t, int64_t pos, int n) {
  uint64_t k = 0;
  for (int j = 0; j < n; ++j) k = (k << 16) | static_cast<uint64_t>(t[pos + j] + 1);
  return k;
}

__global__ __launch_bounds__(kLevWaves * kWave) void bleu_stats_wave_kernel(
    const int64_t* __restrict__ hyp, const int64_t* __restrict__ hyp_off, const int64_t* __restrict__ ref,
    const int64_t* __restrict__ ref_off, const int64_t* __restrict__ group_off, int64_t nhyp, int n_gram,
    double* __restrict__ num, double* __restrict__ den, double* __restrict__ lens) {
  const int lane = threadIdx.x % kWave;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kLevWaves + threadIdx.x / kWave;
  if (i >= nhyp) return;  // wave-uniform
  const int64_t h0 = hyp_off[i], hl = hyp_off[i + 1] - h0;
  const int64_t g0 = group_off[i], g1 = group_off[i + 1];
  if (lane == 0) {  // lengths: hypothesis and closest reference (first minimum), as the host op
    int64_t best_diff = -1, best_len = 0;
    for (int64_t r = g0; r < g1; ++r) {
      const int64_t rl = ref_off[r + 1] - ref_off[r];
      const int64_t d = hl > rl ? hl - rl : rl - hl;
      if (best_diff < 0 || d < best_diff) {
        best_diff = d;
        best_len = rl;
      }
    }
    lens[2 * i] = static_cast<double>(hl);
    lens[2 * i + 1] = static_cast<double>(best_len);
  }
  for (int n = 1; n <= n_gram; ++n) {
    const int64_t ng = hl - n + 1;  // n-grams in the hypothesis
    uint64_t key[kBleuSlots];
    int cnt[kBleuSlots], mx[kBleuSlots], cur[kBleuSlots];
    bool first[kBleuSlots];
#pragma unroll
    for (int k = 0; k < kBleuSlots; ++k) {
      const int64_t p = lane + 64 * k;
      key[k] = p < ng ? gram_key(hyp + h0, p, n) : 0ull;
      cnt[k] = 0;
      mx[k] = 0;
      first[k] = true;
    }
    // (1) counts inside the hypothesis + first occurrences
#pragma unroll
    for (int kq = 0; kq < kBleuSlots; ++kq) {
      if (64 * kq >= ng) break;
      for (int ql = 0; ql < kWave && 64 * kq + ql < ng; ++ql) {
        const uint64_t kqv = __shfl(key[kq], ql, kWave);
        const int64_t q = 64 * kq + ql;
#pragma unroll
        for (int k = 0; k < kBleuSlots; ++k) {
          const int64_t p = lane + 64 * k;
          if (p < ng && key[k] == kqv) {
            ++cnt[k];
            if (q < p) first[k] = false;
          }
        }
      }
    }
    // (2) maximum count over the references
    for (int64_t r = g0; r < g1; ++r) {
      const int64_t r0 = ref_off[r], rng = ref_off[r + 1] - r0 - n + 1;
#pragma unroll
      for (int k = 0; k < kBleuSlots; ++k) cur[k] = 0;
      for (int64_t q = 0; q < rng; ++q) {
        const uint64_t kr = gram_key(ref + r0, q, n);  // wave-uniform loads
#pragma unroll
        for (int k = 0; k < kBleuSlots; ++k) cur[k] += (key[k] == kr) ? 1 : 0;
      }
#pragma unroll
      for (int k = 0; k < kBleuSlots; ++k) mx[k] = max(mx[k], cur[k]);
    }
    // (3) clipped matches over first occurrences, hypothesis n-gram total
    int clipped = 0;
#pragma unroll
    for (int k = 0; k < kBleuSlots; ++k) {
      const int64_t p = lane + 64 * k;
      if (p < ng && first[k]) clipped += min(cnt[k], mx[k]);
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) clipped += __shfl_xor(clipped, off, kWave);
    if (lane == 0) {
      num[i * n_gram + (n - 1)] = static_cast<double>(clipped);
      den[i * n_gram + (n - 1)] = static_cast<double>(ng > 0 ? ng : 0);
    }
  }
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bleu_stats_gpu(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref,
                                                              const at::Tensor& ref_off, const at::Tensor& group_off, int64_t n_gram,
                                                              int64_t max_hyp_len) {
  for (const at::Tensor* t : {&hyp, &hyp_off, &ref, &ref_off, &group_off})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong, "bleu_stats_gpu: expected int64 GPU tensors");
  TORCH_CHECK(n_gram >= 1 && n_gram <= 4, "bleu_stats_gpu: n_gram must be in [1, 4] (exact 64-bit n-gram keys)");
  TORCH_CHECK(max_hyp_len <= 64 * kBleuSlots, "bleu_stats_gpu: hypothesis longer than ", 64 * kBleuSlots, " tokens");
  TORCH_CHECK(group_off.numel() == hyp_off.numel(), "bleu_stats_gpu: group offsets must have n + 1 entries");
  const c10::DeviceGuard guard(hyp.device());
  const int64_t n = hyp_off.numel() - 1;
  auto opts = hyp.options().dtype(at::kDouble);
  auto num = at::zeros({n, n_gram}, opts), den = at::zeros({n, n_gram}, opts), lens = at::zeros({n, 2}, opts);
  if (n <= 0) return {num, den, lens};
  const auto h = hyp.contiguous(), ho = hyp_off.contiguous(), r = ref.contiguous(), ro = ref_off.contiguous(), go = group_off.contiguous();
  const unsigned grid = static_cast<unsigned>((n + kLevWaves - 1) / kLevWaves);
  bleu_stats_wave_kernel<<<grid, kLevWaves * kWave, 0, stream()>>>(h.data_ptr<int64_t>(), ho.data_ptr<int64_t>(), r.data_ptr<int64_t>(),
                                                                   ro.data_ptr<int64_t>(), go.data_ptr<int64_t>(), n, static_cast<int>(n_gram),
                                                                   num.data_ptr<double>(), den.data_ptr<double>(), lens.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return {num, den, lens};
}

// a / b: flat int64 token ids (GPU), a_off / b_off: int64 [n + 1] offsets (GPU).  Returns int64 [n] distances.
at::Tensor levenshtein_gpu(const at::Tensor& a, const at::Tensor& a_off, const at::Tensor& b, const at::Tensor& b_off,
                           int64_t max_ref_len) {
  TORCH_CHECK(a.is_cuda() && a_off.is_cuda() && b.is_cuda() && b_off.is_cuda(), "levenshtein_gpu: expected GPU tensors");
  TORCH_CHECK(a.scalar_type() == at::kLong && b.scalar_type() == at::kLong && a_off.scalar_type() == at::kLong &&
                  b_off.scalar_type() == at::kLong, "levenshtein_gpu: expected int64 ids / offsets");
  TORCH_CHECK(a_off.numel() == b_off.numel() && a_off.numel() >= 1, "levenshtein_gpu: offset length mismatch");
  const c10::DeviceGuard guard(a.device());
  const int64_t n = a_off.numel() - 1;
  auto out = at::empty({n}, a_off.options());
  if (n == 0) return out;
  // the caller packed the sequences on the host and passes the longest reference (no device read here)
  TORCH_CHECK(max_ref_len <= 64 * kLevMaxWords, "levenshtein_gpu: reference longer than ", 64 * kLevMaxWords, " tokens");
  const auto ac = a.contiguous(), bc = b.contiguous(), aoc = a_off.contiguous(), boc = b_off.contiguous();
  const unsigned grid = static_cast<unsigned>((n + kLevWaves - 1) / kLevWaves);
  levenshtein_wave_kernel<<<grid, kLevWaves * kWave, 0, stream()>>>(ac.data_ptr<int64_t>(), aoc.data_ptr<int64_t>(), bc.data_ptr<int64_t>(),
                                                                    boc.data_ptr<int64_t>(), n, out.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  return out;
}

// LCS lengths of the pairs (int64 [n]), same packing / limits as levenshtein_gpu.
at::Tensor lcs_gpu(const at::Tensor& a, const at::Tensor& a_off, const at::Tensor& b, const at::Tensor& b_off, int64_t max_ref_len) {
  TORCH_CHECK(a.is_cuda() && a_off.is_cuda() && b.is_cuda() && b_off.is_cuda(), "lcs_gpu: expected GPU tensors");
  TORCH_CHECK(a.scalar_type() == at::kLong && b.scalar_type() == at::kLong && a_off.scalar_type() == at::kLong &&
                  b_off.scalar_type() == at::kLong, "lcs_gpu: expected int64 ids / offsets");
  TORCH_CHECK(a_off.numel() == b_off.numel() && a_off.numel() >= 1, "lcs_gpu: offset length mismatch");
  const c10::DeviceGuard guard(a.device());
  const int64_t n = a_off.numel() - 1;
  auto out = at::empty({n}, a_off.options());
  if (n == 0) return out;
  TORCH_CHECK(max_ref_len <= 64 * kLevMaxWords, "lcs_gpu: reference longer than ", 64 * kLevMaxWords, " tokens");
  const auto ac = a.contiguous(), bc = b.contiguous(), aoc = a_off.contiguous(), boc = b_off.contiguous();
  const unsigned grid = static_cast<unsigned>((n + kLevWaves - 1) / kLevWaves);
  lcs_wave_kernel<<<grid, kLevWaves * kWave, 0, stream()>>>(ac.data_ptr<int64_t>(), aoc.data_ptr<int64_t>(), bc.data_ptr<int64_t>(),
                                                            boc.data_ptr<int64_t>(), n, out.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("levenshtein_gpu(Tensor a, Tensor a_off, Tensor b, Tensor b_off, int max_ref_len) -> Tensor");
  m.def("lcs_gpu(Tensor a, Tensor a_off, Tensor b, Tensor b_off, int max_ref_len) -> Tensor");
  m.def("bleu_stats_gpu(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, Tensor ref_group_off, int n_gram, int max_hyp_len) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("levenshtein_gpu", &tmx::levenshtein_gpu);
  m.impl("lcs_gpu", &tmx::lcs_gpu);
  m.impl("bleu_stats_gpu", &tmx::bleu_stats_gpu);
}
