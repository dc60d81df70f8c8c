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
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("levenshtein_gpu", &tmx::levenshtein_gpu);
  m.impl("lcs_gpu", &tmx::lcs_gpu);
}
