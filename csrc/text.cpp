// Native string-metric kernels: edit distances, Tercom TER with shifts, extended edit distance.
//
// The reference runs these dynamic programmes in pure Python per sentence pair.  Here sentences arrive already
// tokenised to int64 ids (words or code points) as one flat buffer + offsets, and every pair is scored in C++ in
// parallel (at::parallel_for over pairs):
//   * levenshtein_batch      exact unit-cost Levenshtein (WER / CER / MER / WIL / WIP): Myers' bit-parallel
//                            algorithm when the reference fits one 64-bit word, a two-row DP otherwise;
//   * levenshtein_beam_batch Tercom's beam-restricted weighted DP (EditDistance), same band / tie rules;
//   * ter_batch              full Tercom shift search (candidate enumeration, corner cases, ordering, limits);
//   * eed_batch              character-level extended edit distance with jumps and coverage penalty.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <map>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace tmx {
namespace {

using Seq = std::vector<int64_t>;

struct Flat {
  const int64_t* data;
  const int64_t* off;
  int64_t n;
  Seq get(int64_t i) const { return Seq(data + off[i], data + off[i + 1]); }
  int64_t len(int64_t i) const { return off[i + 1] - off[i]; }
  const int64_t* ptr(int64_t i) const { return data + off[i]; }
};

Flat make_flat(const at::Tensor& data, const at::Tensor& off) {
  TORCH_CHECK(data.device().is_cpu() && off.device().is_cpu(), "text kernels run on host tensors");
  TORCH_CHECK(data.scalar_type() == at::kLong && off.scalar_type() == at::kLong, "expected int64 ids / offsets");
  TORCH_CHECK(data.is_contiguous() && off.is_contiguous(), "expected contiguous ids / offsets");
  return {data.data_ptr<int64_t>(), off.data_ptr<int64_t>(), off.numel() - 1};
}

// ---- exact unit-cost Levenshtein ------------------------------------------------------------------------
int64_t lev_dp(const int64_t* a, int64_t n, const int64_t* b, int64_t m) {
  std::vector<int64_t> prev(m + 1), cur(m + 1);
  for (int64_t j = 0; j <= m; ++j) prev[j] = j;
  for (int64_t i = 1; i <= n; ++i) {
    cur[0] = i;
    for (int64_t j = 1; j <= m; ++j) {
      if (a[i - 1] == b[j - 1]) cur[j] = prev[j - 1];
      else cur[j] = std::min(std::min(prev[j], cur[j - 1]), prev[j - 1]) + 1;
    }
    std::swap(prev, cur);
  }
  return prev[m];
}

// Myers (1999) bit-vector algorithm, pattern b of length m <= 64, text a.
int64_t lev_myers(const int64_t* a, int64_t n, const int64_t* b, int64_t m) {
  if (m == 0) return n;
  std::unordered_map<int64_t, uint64_t> peq;
  peq.reserve(static_cast<size_t>(m) * 2);
  for (int64_t j = 0; j < m; ++j) peq[b[j]] |= (1ull << j);
  uint64_t pv = (m == 64) ? ~0ull : ((1ull << m) - 1), mv = 0;
  const uint64_t last = 1ull << (m - 1);
  int64_t score = m;
  for (int64_t i = 0; i < n; ++i) {
    auto it = peq.find(a[i]);
    const uint64_t eq = it == peq.end() ? 0ull : it->second;
    const uint64_t xv = eq | mv;
    const uint64_t xh = (((eq & pv) + pv) ^ pv) | eq;
    uint64_t ph = mv | ~(xh | pv);
    uint64_t mh = pv & xh;
    if (ph & last) ++score;
    else if (mh & last) --score;
    ph = (ph << 1) | 1ull;
    mh <<= 1;
    pv = mh | ~(xv | ph);
    mv = ph & xv;
  }
  return score;
}

// ---- Tercom beam DP (weighted, with trace) --------------------------------------------------------------
enum Op : uint8_t { kNothing = 0, kSub = 1, kIns = 2, kDel = 3, kUndef = 4 };
constexpr int64_t kInf = 10000000000000000LL;  // 1e16
constexpr int64_t kBeam = 25;

struct BeamDP {
  std::vector<int64_t> cost;
  std::vector<uint8_t> op;
};

// distance from `pred` to `ref`; fills the (n+1)x(m+1) table when `keep` is set (for the trace)
int64_t lev_beam(const int64_t* pred, int64_t n, const int64_t* ref, int64_t m, int64_t ins, int64_t del, int64_t sub,
                 BeamDP* keep) {
  const int64_t W = m + 1;
  std::vector<int64_t> cost((n + 1) * W, kInf);
  std::vector<uint8_t> op((n + 1) * W, kUndef);
  for (int64_t j = 0; j <= m; ++j) {
    cost[j] = j * ins;
    op[j] = kIns;
  }
  const double ratio = n ? static_cast<double>(m) / static_cast<double>(n) : 1.0;
  const int64_t beam = (ratio / 2 > kBeam) ? static_cast<int64_t>(std::ceil(ratio / 2 + kBeam)) : kBeam;
  for (int64_t i = 1; i <= n; ++i) {
    const int64_t diag = static_cast<int64_t>(std::floor(static_cast<double>(i) * ratio));
    const int64_t lo = std::max<int64_t>(0, diag - beam);
    const int64_t hi = (i == n) ? m + 1 : std::min<int64_t>(m + 1, diag + beam);
    for (int64_t j = lo; j < hi; ++j) {
      int64_t* c = &cost[i * W + j];
      uint8_t* o = &op[i * W + j];
      if (j == 0) {
        *c = cost[(i - 1) * W] + del;
        *o = kDel;
        continue;
      }
      const bool same = pred[i - 1] == ref[j - 1];
      const int64_t cs = cost[(i - 1) * W + j - 1] + (same ? 0 : sub);
      const int64_t cd = cost[(i - 1) * W + j] + del;
      const int64_t ci = cost[i * W + j - 1] + ins;
      if (*c > cs) { *c = cs; *o = same ? kNothing : kSub; }
      if (*c > cd) { *c = cd; *o = kDel; }
      if (*c > ci) { *c = ci; *o = kIns; }
    }
  }
  const int64_t d = cost[n * W + m];
  if (keep) {
    keep->cost.swap(cost);
    keep->op.swap(op);
  }
  return d;
}

std::vector<uint8_t> beam_trace(const BeamDP& dp, int64_t n, int64_t m) {
  std::vector<uint8_t> trace;
  const int64_t W = m + 1;
  int64_t i = n, j = m;
  while (i > 0 || j > 0) {
    const uint8_t o = dp.op[i * W + j];
    trace.push_back(o);
    if (o == kSub || o == kNothing) { --i; --j; }
    else if (o == kIns) { --j; }
    else if (o == kDel) { --i; }
    else TORCH_CHECK(false, "ter: undefined edit operation in trace");
  }
  std::reverse(trace.begin(), trace.end());
  return trace;
}

// ---- Tercom shifts ---------------------------------------------------------------------------------------
constexpr int64_t kMaxShiftSize = 10;
constexpr int64_t kMaxShiftDist = 50;
constexpr int64_t kMaxShiftCandidates = 1000;

Seq slice(const Seq& s, int64_t a, int64_t b) {
  const int64_t n = static_cast<int64_t>(s.size());
  a = std::min(std::max<int64_t>(a, 0), n);
  b = std::min(std::max<int64_t>(b, 0), n);
  return b > a ? Seq(s.begin() + a, s.begin() + b) : Seq();
}

void append(Seq& dst, const Seq& src) { dst.insert(dst.end(), src.begin(), src.end()); }

Seq perform_shift(const Seq& w, int64_t start, int64_t length, int64_t target) {
  Seq out;
  out.reserve(w.size());
  if (target < start) {
    append(out, slice(w, 0, target));
    append(out, slice(w, start, start + length));
    append(out, slice(w, target, start));
    append(out, slice(w, start + length, static_cast<int64_t>(w.size())));
  } else if (target > start + length) {
    append(out, slice(w, 0, start));
    append(out, slice(w, start + length, target));
    append(out, slice(w, start, start + length));
    append(out, slice(w, target, static_cast<int64_t>(w.size())));
  } else {
    append(out, slice(w, 0, start));
    append(out, slice(w, start + length, length + target));
    append(out, slice(w, start, start + length));
    append(out, slice(w, length + target, static_cast<int64_t>(w.size())));
  }
  return out;
}

struct Candidate {
  int64_t score, length, neg_start, neg_idx;
  Seq words;
  bool operator>(const Candidate& o) const {
    if (score != o.score) return score > o.score;
    if (length != o.length) return length > o.length;
    if (neg_start != o.neg_start) return neg_start > o.neg_start;
    if (neg_idx != o.neg_idx) return neg_idx > o.neg_idx;
    return words > o.words;
  }
};

// One round of the greedy shift search: returns (delta, shifted words) and advances `checked`.
std::pair<int64_t, Seq> shift_words(const Seq& a, const Seq& b, int64_t& checked) {
  const int64_t n = static_cast<int64_t>(a.size()), m = static_cast<int64_t>(b.size());
  BeamDP dp;
  const int64_t dist = lev_beam(a.data(), n, b.data(), m, 1, 1, 1, &dp);
  std::vector<uint8_t> trace = beam_trace(dp, n, m);
  for (auto& o : trace) o = (o == kIns) ? kDel : (o == kDel ? kIns : o);  // flip: rewrite b into a
  // alignment: reference (b) position -> hypothesis (a) position; error flags per position
  std::vector<int64_t> align(m, -2);
  std::vector<int64_t> b_err, a_err;
  int64_t rp = -1, hp = -1;
  for (uint8_t o : trace) {
    if (o == kNothing || o == kSub) {
      ++hp; ++rp;
      align[rp] = hp;
      b_err.push_back(o == kSub);
      a_err.push_back(o == kSub);
    } else if (o == kIns) {
      ++hp;
      a_err.push_back(1);
    } else {
      ++rp;
      align[rp] = hp;
      b_err.push_back(1);
    }
  }
  auto sum_range = [](const std::vector<int64_t>& v, int64_t s, int64_t e) {
    int64_t t = 0;
    for (int64_t k = std::max<int64_t>(s, 0); k < std::min<int64_t>(e, static_cast<int64_t>(v.size())); ++k) t += v[k];
    return t;
  };
  bool have = false;
  Candidate best{0, 0, 0, 0, {}};
  for (int64_t ps = 0; ps < n; ++ps) {
    for (int64_t ts = 0; ts < m; ++ts) {
      if (std::llabs(ts - ps) > kMaxShiftDist) continue;
      for (int64_t len = 1; len < kMaxShiftSize; ++len) {
        if (a[ps + len - 1] != b[ts + len - 1]) break;
        // candidate (ps, ts, len)
        bool skip = sum_range(a_err, ps, ps + len) == 0 || sum_range(b_err, ts, ts + len) == 0;
        if (!skip) {
          const int64_t al = align[ts];
          skip = ps <= al && al < ps + len;
        }
        if (!skip) {
          int64_t prev_idx = -1;
          for (int64_t off = -1; off < len; ++off) {
            int64_t idx;
            if (ts + off == -1) idx = 0;
            else if (ts + off < m && align[ts + off] != -2) idx = align[ts + off] + 1;
            else break;
            if (idx == prev_idx) continue;
            prev_idx = idx;
            Seq shifted = perform_shift(a, ps, len, idx);
            const int64_t d2 = lev_beam(shifted.data(), static_cast<int64_t>(shifted.size()), b.data(), m, 1, 1, 1, nullptr);
            Candidate c{dist - d2, len, -ps, -idx, std::move(shifted)};
            ++checked;
            if (!have || c > best) {
              best = std::move(c);
              have = true;
            }
          }
          if (checked >= kMaxShiftCandidates) goto done;
        }
        if (ps + len == n || ts + len == m) break;
      }
    }
  }
done:
  if (!have) return {0, a};
  return {best.score, std::move(best.words)};
}

// reference semantics: `a` is shifted towards `b`; empty `b` -> 0 edits
double translation_edit_rate(const Seq& a, const Seq& b) {
  if (b.empty()) return 0.0;
  int64_t shifts = 0, checked = 0;
  Seq cur = a;
  while (true) {
    auto res = shift_words(cur, b, checked);
    if (checked >= kMaxShiftCandidates || res.first <= 0) break;
    ++shifts;
    cur = std::move(res.second);
  }
  const int64_t d = lev_beam(cur.data(), static_cast<int64_t>(cur.size()), b.data(), static_cast<int64_t>(b.size()), 1, 1, 1, nullptr);
  return static_cast<double>(shifts + d);
}

// ---- extended edit distance ------------------------------------------------------------------------------
double eed_pair(const int64_t* hyp, int64_t n, const int64_t* ref, int64_t m, int64_t space, double alpha, double rho,
                double deletion, double insertion) {
  const double inf = std::numeric_limits<double>::infinity();
  std::vector<int64_t> visits(n + 1, -1);
  std::vector<double> row(n + 1, 1.0), next(n + 1, inf);
  row[0] = 0.0;
  for (int64_t w = 1; w <= m; ++w) {
    for (int64_t i = 0; i <= n; ++i) {
      if (i > 0) {
        const double sub = row[i - 1] + (hyp[i - 1] != ref[w - 1] ? 1.0 : 0.0);
        next[i] = std::min(std::min(next[i - 1] + deletion, sub), row[i] + insertion);
      } else {
        next[i] = row[i] + 1.0;
      }
    }
    int64_t mi = 0;
    for (int64_t i = 1; i <= n; ++i)
      if (next[i] < next[mi]) mi = i;
    visits[mi] += 1;
    if (ref[w - 1] == space) {
      const double jump = alpha + next[mi];
      for (auto& x : next) x = std::min(x, jump);
    }
    row.swap(next);
    std::fill(next.begin(), next.end(), inf);
  }
  double cov = 0.0;
  for (int64_t v : visits) cov += (v >= 0 ? static_cast<double>(v) : 1.0);
  cov *= rho;
  return std::min(1.0, (row[n] + cov) / (static_cast<double>(m) + cov));
}

// ---- n-gram statistics (BLEU) ----------------------------------------------------------------------------
struct VecHash {
  size_t operator()(const Seq& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int64_t x : v) {
      h ^= static_cast<uint64_t>(x) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
      h *= 1099511628211ull;
    }
    return static_cast<size_t>(h);
  }
};
using NgramCount = std::unordered_map<Seq, int64_t, VecHash>;

NgramCount count_ngrams(const int64_t* t, int64_t len, int64_t n_gram) {
  NgramCount c;
  for (int64_t n = 1; n <= n_gram; ++n)
    for (int64_t j = 0; j + n <= len; ++j) c[Seq(t + j, t + j + n)] += 1;
  return c;
}

// Packed n-grams (n <= 4, ids < 65535): (id + 1) per 16-bit field, so an n-gram is one exact 64-bit key and its order
// is the number of occupied fields — no per-n-gram allocation (the generic map above allocates a vector per key).
inline int64_t packed_order(uint64_t k) { return (64 - __builtin_clzll(k) + 15) / 16; }

// Sorted (key, count) runs of every packed n-gram (orders 1..n_gram) of t, appended to ``out``.
void packed_runs(const int64_t* t, int64_t len, int64_t n_gram, std::vector<uint64_t>& keys,
                 std::vector<std::pair<uint64_t, int64_t>>& out) {
  keys.clear();
  for (int64_t j = 0; j < len; ++j) {
    uint64_t k = 0;
    for (int64_t n = 1; n <= n_gram && j + n <= len; ++n) {
      k = (k << 16) | static_cast<uint64_t>(t[j + n - 1] + 1);
      keys.push_back(k);
    }
  }
  std::sort(keys.begin(), keys.end());
  for (size_t a = 0; a < keys.size();) {
    size_t b = a + 1;
    while (b < keys.size() && keys[b] == keys[a]) ++b;
    out.emplace_back(keys[a], static_cast<int64_t>(b - a));
    a = b;
  }
}

bool packable(const at::Tensor& a, const at::Tensor& b, int64_t n_gram) {
  if (n_gram > 4) return false;
  for (const at::Tensor* t : {&a, &b})
    if (t->numel() && (t->min().item<int64_t>() < 0 || t->max().item<int64_t>() >= 65535)) return false;
  return true;
}

// ---- longest common subsequence (ROUGE-L) -------------------------------------------------------------------
[[maybe_unused]] int64_t lcs_dp(const int64_t* a, int64_t n, const int64_t* b, int64_t m) {  // O(n m) oracle
  std::vector<int64_t> prev(m + 1, 0), cur(m + 1, 0);
  for (int64_t i = 1; i <= n; ++i) {
    for (int64_t j = 1; j <= m; ++j) cur[j] = (a[i - 1] == b[j - 1]) ? prev[j - 1] + 1 : std::max(prev[j], cur[j - 1]);
    std::swap(prev, cur);
  }
  return prev[m];
}

// Allison-Dix / Hyyro bit-vector LCS with the pattern b (m <= 64) in one word.
int64_t lcs_bits(const int64_t* a, int64_t n, const int64_t* b, int64_t m) {
  if (m == 0 || n == 0) return 0;
  std::unordered_map<int64_t, uint64_t> peq;
  peq.reserve(static_cast<size_t>(m) * 2);
  for (int64_t j = 0; j < m; ++j) peq[b[j]] |= (1ull << j);
  const uint64_t mask = (m == 64) ? ~0ull : ((1ull << m) - 1);
  uint64_t v = mask;
  for (int64_t i = 0; i < n; ++i) {
    auto it = peq.find(a[i]);
    if (it == peq.end()) continue;
    const uint64_t u = v & it->second;
    v = ((v + u) | (v - u)) & mask;
  }
  return m - __builtin_popcountll(v);
}

// Multi-word form (any m): V' = (V + (V & Peq)) | (V & ~Peq) with the addition's carry rippling from word to word
// (V - (V & Peq) = V & ~Peq has no borrows).  O(n * ceil(m / 64)) word operations instead of the O(n * m) DP.
int64_t lcs_bits_multi(const int64_t* a, int64_t n, const int64_t* b, int64_t m) {
  if (m == 0 || n == 0) return 0;
  const int64_t words = (m + 63) / 64;
  std::unordered_map<int64_t, int64_t> row;  // token -> row of the match-mask table
  row.reserve(static_cast<size_t>(m) * 2);
  std::vector<uint64_t> peq;
  for (int64_t j = 0; j < m; ++j) {
    auto it = row.find(b[j]);
    if (it == row.end()) {
      it = row.emplace(b[j], static_cast<int64_t>(peq.size() / words)).first;
      peq.resize(peq.size() + words, 0ull);
    }
    peq[it->second * words + j / 64] |= 1ull << (j % 64);
  }
  std::vector<uint64_t> v(words, ~0ull);
  const uint64_t last = (m % 64) ? ((1ull << (m % 64)) - 1) : ~0ull;
  v[words - 1] = last;
  for (int64_t i = 0; i < n; ++i) {
    auto it = row.find(a[i]);
    if (it == row.end()) continue;
    const uint64_t* pm = peq.data() + it->second * words;
    uint64_t carry = 0;
    for (int64_t k = 0; k < words; ++k) {
      const uint64_t u = v[k] & pm[k];
      const uint64_t s1 = v[k] + u;
      const uint64_t s2 = s1 + carry;
      carry = (s1 < v[k]) | (s2 < s1);
      v[k] = s2 | (v[k] & ~pm[k]);
    }
    v[words - 1] &= last;
  }
  int64_t ones = 0;
  for (int64_t k = 0; k < words; ++k) ones += __builtin_popcountll(v[k]);
  return m - ones;
}

}  // namespace

at::Tensor levenshtein_batch(const at::Tensor& a, const at::Tensor& a_off, const at::Tensor& b, const at::Tensor& b_off) {
  const Flat fa = make_flat(a, a_off), fb = make_flat(b, b_off);
  TORCH_CHECK(fa.n == fb.n, "levenshtein_batch: pair count mismatch");
  auto out = at::empty({fa.n}, at::kLong);
  int64_t* o = out.data_ptr<int64_t>();
  at::parallel_for(0, fa.n, 16, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const int64_t n = fa.len(i), m = fb.len(i);
      o[i] = (m <= 64) ? lev_myers(fa.ptr(i), n, fb.ptr(i), m) : lev_dp(fa.ptr(i), n, fb.ptr(i), m);
    }
  });
  return out;
}

at::Tensor levenshtein_beam_batch(const at::Tensor& pred, const at::Tensor& pred_off, const at::Tensor& ref,
                                  const at::Tensor& ref_off, int64_t ins, int64_t del, int64_t sub) {
  const Flat fp = make_flat(pred, pred_off), fr = make_flat(ref, ref_off);
  TORCH_CHECK(fp.n == fr.n, "levenshtein_beam_batch: pair count mismatch");
  auto out = at::empty({fp.n}, at::kLong);
  int64_t* o = out.data_ptr<int64_t>();
  at::parallel_for(0, fp.n, 4, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) o[i] = lev_beam(fp.ptr(i), fp.len(i), fr.ptr(i), fr.len(i), ins, del, sub, nullptr);
  });
  return out;
}

// hyp [n sentences]; refs [R sentences] grouped per hypothesis by ref_group_off [n + 1].
std::tuple<at::Tensor, at::Tensor> ter_batch(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref,
                                             const at::Tensor& ref_off, const at::Tensor& ref_group_off) {
  const Flat fh = make_flat(hyp, hyp_off), fr = make_flat(ref, ref_off);
  TORCH_CHECK(ref_group_off.numel() == fh.n + 1, "ter_batch: group offsets must have n + 1 entries");
  const auto g = ref_group_off.to(at::kLong).contiguous();
  const int64_t* go = g.data_ptr<int64_t>();
  auto edits = at::empty({fh.n}, at::kDouble), avg_len = at::empty({fh.n}, at::kDouble);
  double* pe = edits.data_ptr<double>();
  double* pl = avg_len.data_ptr<double>();
  at::parallel_for(0, fh.n, 1, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const Seq h = fh.get(i);
      double best = 2e16, tot = 0.0;
      const int64_t r0 = go[i], r1 = go[i + 1];
      for (int64_t r = r0; r < r1; ++r) {
        const Seq t = fr.get(r);
        const double ed = translation_edit_rate(t, h);  // the reference side is shifted towards the hypothesis
        tot += static_cast<double>(t.size());
        if (ed < best) best = ed;
      }
      pe[i] = best;
      pl[i] = r1 > r0 ? tot / static_cast<double>(r1 - r0) : 0.0;
    }
  });
  return {edits, avg_len};
}

at::Tensor eed_batch(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref, const at::Tensor& ref_off,
                     int64_t space, double alpha, double rho, double deletion, double insertion) {
  const Flat fh = make_flat(hyp, hyp_off), fr = make_flat(ref, ref_off);
  TORCH_CHECK(fh.n == fr.n, "eed_batch: pair count mismatch");
  auto out = at::empty({fh.n}, at::kDouble);
  double* o = out.data_ptr<double>();
  at::parallel_for(0, fh.n, 2, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i)
      o[i] = eed_pair(fh.ptr(i), fh.len(i), fr.ptr(i), fr.len(i), space, alpha, rho, deletion, insertion);
  });
  return out;
}

// BLEU sufficient statistics for a batch: per hypothesis, clipped n-gram matches against the union (max count) of
// its references, hypothesis n-gram totals, hypothesis length and closest reference length (first minimum).
std::tuple<at::Tensor, at::Tensor, at::Tensor> bleu_stats(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref,
                                                          const at::Tensor& ref_off, const at::Tensor& ref_group_off, int64_t n_gram) {
  const Flat fh = make_flat(hyp, hyp_off), fr = make_flat(ref, ref_off);
  TORCH_CHECK(ref_group_off.numel() == fh.n + 1, "bleu_stats: group offsets must have n + 1 entries");
  const auto g = ref_group_off.to(at::kLong).contiguous();
  const int64_t* go = g.data_ptr<int64_t>();
  auto num = at::zeros({fh.n, n_gram}, at::kDouble), den = at::zeros({fh.n, n_gram}, at::kDouble);
  auto lens = at::zeros({fh.n, 2}, at::kDouble);
  double* pn = num.data_ptr<double>();
  double* pd = den.data_ptr<double>();
  double* pl = lens.data_ptr<double>();
  if (packable(hyp, ref, n_gram)) {  // sorted packed keys + run-length: no hash-map nodes per n-gram
    at::parallel_for(0, fh.n, 8, [&](int64_t s, int64_t e) {
      std::vector<uint64_t> keys;
      std::vector<std::pair<uint64_t, int64_t>> tgt, runs;
      auto sorted_runs = [&](const int64_t* t, int64_t len, std::vector<std::pair<uint64_t, int64_t>>& out) {
        packed_runs(t, len, n_gram, keys, out);
      };
      for (int64_t i = s; i < e; ++i) {
        const int64_t hl = fh.len(i);
        pl[2 * i] = static_cast<double>(hl);
        int64_t best_diff = -1, best_len = 0;
        tgt.clear();
        for (int64_t r = go[i]; r < go[i + 1]; ++r) {
          const int64_t rl = fr.len(r);
          const int64_t d = std::llabs(hl - rl);
          if (best_diff < 0 || d < best_diff) {
            best_diff = d;
            best_len = rl;
          }
          sorted_runs(fr.ptr(r), rl, tgt);  // appended per reference; max per key below
        }
        pl[2 * i + 1] = static_cast<double>(best_len);
        std::sort(tgt.begin(), tgt.end());  // by key, then count: the last of each key run is its maximum
        runs.clear();
        sorted_runs(fh.ptr(i), hl, runs);
        size_t q = 0;
        for (const auto& kv : runs) {
          const int64_t n = packed_order(kv.first) - 1;
          pd[i * n_gram + n] += static_cast<double>(kv.second);
          while (q < tgt.size() && tgt[q].first < kv.first) ++q;
          size_t last = q;
          while (last < tgt.size() && tgt[last].first == kv.first) ++last;
          if (last > q) pn[i * n_gram + n] += static_cast<double>(std::min(kv.second, tgt[last - 1].second));
          q = last;
        }
      }
    });
    return {num, den, lens};
  }
  at::parallel_for(0, fh.n, 8, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const int64_t hl = fh.len(i);
      pl[2 * i] = static_cast<double>(hl);
      int64_t best_diff = -1, best_len = 0;
      NgramCount tgt;
      for (int64_t r = go[i]; r < go[i + 1]; ++r) {
        const int64_t rl = fr.len(r);
        const int64_t d = std::llabs(hl - rl);
        if (best_diff < 0 || d < best_diff) {
          best_diff = d;
          best_len = rl;
        }
        for (auto& kv : count_ngrams(fr.ptr(r), rl, n_gram)) {
          auto& slot = tgt[kv.first];
          slot = std::max(slot, kv.second);
        }
      }
      pl[2 * i + 1] = static_cast<double>(best_len);
      for (auto& kv : count_ngrams(fh.ptr(i), hl, n_gram)) {
        const int64_t n = static_cast<int64_t>(kv.first.size()) - 1;
        pd[i * n_gram + n] += static_cast<double>(kv.second);
        auto it = tgt.find(kv.first);
        if (it != tgt.end()) pn[i * n_gram + n] += static_cast<double>(std::min(kv.second, it->second));
      }
    }
  });
  return {num, den, lens};
}

// Clipped n-gram overlap of every (hypothesis, reference) pair, per order n = 1..n_order (chrF / chrF++ / ROUGE-N):
// match[r, n-1] = Σ_g min(count_hyp(g), count_ref_r(g)) over n-grams g; hyp_tot / ref_tot = number of n-grams.
std::tuple<at::Tensor, at::Tensor, at::Tensor> ngram_overlap(const at::Tensor& hyp, const at::Tensor& hyp_off, const at::Tensor& ref,
                                                             const at::Tensor& ref_off, const at::Tensor& ref_group_off, int64_t n_order) {
  const Flat fh = make_flat(hyp, hyp_off), fr = make_flat(ref, ref_off);
  TORCH_CHECK(ref_group_off.numel() == fh.n + 1, "ngram_overlap: group offsets must have n + 1 entries");
  const auto g = ref_group_off.to(at::kLong).contiguous();
  const int64_t* go = g.data_ptr<int64_t>();
  auto match = at::zeros({fr.n, n_order}, at::kLong), htot = at::zeros({fh.n, n_order}, at::kLong);
  auto rtot = at::zeros({fr.n, n_order}, at::kLong);
  int64_t* pm = match.data_ptr<int64_t>();
  int64_t* ph = htot.data_ptr<int64_t>();
  int64_t* pr = rtot.data_ptr<int64_t>();
  if (packable(hyp, ref, n_order)) {  // sorted packed runs of both sides, merged per reference
    at::parallel_for(0, fh.n, 4, [&](int64_t s, int64_t e) {
      std::vector<uint64_t> keys;
      std::vector<std::pair<uint64_t, int64_t>> hr, rr;
      for (int64_t i = s; i < e; ++i) {
        const int64_t hl = fh.len(i);
        for (int64_t n = 1; n <= n_order; ++n) ph[i * n_order + n - 1] = std::max<int64_t>(hl - n + 1, 0);
        hr.clear();
        packed_runs(fh.ptr(i), hl, n_order, keys, hr);
        for (int64_t r = go[i]; r < go[i + 1]; ++r) {
          const int64_t rl = fr.len(r);
          for (int64_t n = 1; n <= n_order; ++n) pr[r * n_order + n - 1] = std::max<int64_t>(rl - n + 1, 0);
          rr.clear();
          packed_runs(fr.ptr(r), rl, n_order, keys, rr);
          size_t a = 0, b = 0;
          while (a < hr.size() && b < rr.size()) {
            if (hr[a].first < rr[b].first) ++a;
            else if (rr[b].first < hr[a].first) ++b;
            else {
              pm[r * n_order + packed_order(hr[a].first) - 1] += std::min(hr[a].second, rr[b].second);
              ++a;
              ++b;
            }
          }
        }
      }
    });
    return {match, htot, rtot};
  }
  at::parallel_for(0, fh.n, 4, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const int64_t hl = fh.len(i);
      for (int64_t n = 1; n <= n_order; ++n) ph[i * n_order + n - 1] = std::max<int64_t>(hl - n + 1, 0);
      const NgramCount hc = count_ngrams(fh.ptr(i), hl, n_order);
      for (int64_t r = go[i]; r < go[i + 1]; ++r) {
        const int64_t rl = fr.len(r);
        for (int64_t n = 1; n <= n_order; ++n) pr[r * n_order + n - 1] = std::max<int64_t>(rl - n + 1, 0);
        for (auto& kv : count_ngrams(fr.ptr(r), rl, n_order)) {
          auto it = hc.find(kv.first);
          if (it != hc.end()) pm[r * n_order + static_cast<int64_t>(kv.first.size()) - 1] += std::min(kv.second, it->second);
        }
      }
    }
  });
  return {match, htot, rtot};
}

at::Tensor lcs_batch(const at::Tensor& a, const at::Tensor& a_off, const at::Tensor& b, const at::Tensor& b_off) {
  const Flat fa = make_flat(a, a_off), fb = make_flat(b, b_off);
  TORCH_CHECK(fa.n == fb.n, "lcs_batch: pair count mismatch");
  auto out = at::empty({fa.n}, at::kLong);
  int64_t* o = out.data_ptr<int64_t>();
  at::parallel_for(0, fa.n, 16, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const int64_t n = fa.len(i), m = fb.len(i);
      o[i] = (m <= 64) ? lcs_bits(fa.ptr(i), n, fb.ptr(i), m) : lcs_bits_multi(fa.ptr(i), n, fb.ptr(i), m);
    }
  });
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("levenshtein_batch(Tensor a, Tensor a_off, Tensor b, Tensor b_off) -> Tensor");
  m.def("levenshtein_beam_batch(Tensor pred, Tensor pred_off, Tensor ref, Tensor ref_off, int ins, int dele, int sub) -> Tensor");
  m.def("ter_batch(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, Tensor ref_group_off) -> (Tensor, Tensor)");
  m.def("bleu_stats(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, Tensor ref_group_off, int n_gram) -> (Tensor, Tensor, Tensor)");
  m.def("ngram_overlap(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, Tensor ref_group_off, int n_order) -> (Tensor, Tensor, Tensor)");
  m.def("lcs_batch(Tensor a, Tensor a_off, Tensor b, Tensor b_off) -> Tensor");
  m.def("eed_batch(Tensor hyp, Tensor hyp_off, Tensor ref, Tensor ref_off, int space, float alpha, float rho, float deletion, float insertion) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CompositeExplicitAutograd, m) {
  m.impl("levenshtein_batch", &tmx::levenshtein_batch);
  m.impl("levenshtein_beam_batch", &tmx::levenshtein_beam_batch);
  m.impl("ter_batch", &tmx::ter_batch);
  m.impl("eed_batch", &tmx::eed_batch);
  m.impl("bleu_stats", &tmx::bleu_stats);
  m.impl("ngram_overlap", &tmx::ngram_overlap);
  m.impl("lcs_batch", &tmx::lcs_batch);
}
