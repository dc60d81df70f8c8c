// Host (CPU) exact curve scores: per column of ``preds [N, C]`` the exact AUROC, average precision and the positive /
// negative counts over the distinct-threshold curve -- the reference's ``_binary_clf_curve`` (argsort descending,
// distinct-value ends, cumsum; reference functional/classification/precision_recall_curve.py:28-80) followed by its
// trapezoid AUROC and step AP, without materialising the curve.
//
// Per column: scores become order-preserving unsigned keys (descending), packed with the label bit and sorted by an
// LSD radix sort (8-bit digits; a pass whose digit is constant over the column is skipped -- softmax scores share
// their sign / exponent bytes), then ONE scan over the sorted run accumulates the tie-group areas.  Columns run in
// parallel (at::parallel_for).  Replaces the vectorised torch form (sort + 2 gathers + 3 cumsums + cummax + ~15
// elementwise passes over [N, C] float64 temporaries) on CPU states.
//
// Tie semantics = torch.sort + ``sp[1:] != sp[:-1]``: values equal as floats share a group (-0.0 == +0.0), every NaN is
// its own group and sorts first (torch treats NaN as the largest value), entries with valid == 0 are dropped.
#include <ATen/ATen.h>
#include <ATen/Dispatch.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace tmx {
namespace {

inline uint32_t desc_key32(float f) {
  if (std::isnan(f)) f = std::numeric_limits<float>::quiet_NaN();  // canonical (positive) NaN: sorts first
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t ord = (u & 0x80000000u) ? ~u : (u ^ 0x80000000u);  // ascending order of the float
  return ~ord;                                                        // descending
}
inline float key_value32(uint32_t k) {
  const uint32_t ord = ~k;
  const uint32_t u = (ord & 0x80000000u) ? (ord ^ 0x80000000u) : ~ord;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint64_t desc_key64(double f) {
  if (std::isnan(f)) f = std::numeric_limits<double>::quiet_NaN();
  uint64_t u;
  std::memcpy(&u, &f, 8);
  const uint64_t ord = (u & 0x8000000000000000ull) ? ~u : (u ^ 0x8000000000000000ull);
  return ~ord;
}
inline double key_value64(uint64_t k) {
  const uint64_t ord = ~k;
  const uint64_t u = (ord & 0x8000000000000000ull) ? (ord ^ 0x8000000000000000ull) : ~ord;
  double f;
  std::memcpy(&f, &u, 8);
  return f;
}

// LSD radix sort of 64-bit words by bits [lo_byte * 8, 64) (bytes below lo_byte are payload), 8-bit digits.  All digit
// histograms come from ONE pass over the keys; a digit that is constant over the column is skipped.
void radix_sort(std::vector<uint64_t>& a, std::vector<uint64_t>& tmp, int lo_byte) {
  const size_t n = a.size();
  tmp.resize(n);
  std::vector<uint32_t> hist(static_cast<size_t>(8 - lo_byte) * 256, 0);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t v = a[i];
    for (int b = lo_byte; b < 8; ++b) ++hist[(b - lo_byte) * 256 + ((v >> (8 * b)) & 0xFF)];
  }
  for (int b = lo_byte; b < 8; ++b) {
    uint32_t* cnt = hist.data() + (b - lo_byte) * 256;
    bool trivial = false;
    for (int d = 0; d < 256; ++d)
      if (cnt[d] == n) trivial = true;
    if (trivial) continue;
    uint32_t off = 0;
    for (int d = 0; d < 256; ++d) {
      const uint32_t c = cnt[d];
      cnt[d] = off;
      off += c;
    }
    const int shift = 8 * b;
    for (size_t i = 0; i < n; ++i) tmp[cnt[(a[i] >> shift) & 0xFF]++] = a[i];
    a.swap(tmp);
  }
}

struct Scores {
  double auroc, ap, pos, neg;
};

// scan of a descending run: value(i) gives the score, label(i) the 0/1 label
template <typename V, typename L>
Scores scan(size_t n, V value, L label) {
  int64_t tps = 0, fps = 0, tp_prev = 0, fp_prev = 0;
  double area = 0.0, ap = 0.0;
  for (size_t i = 0; i < n; ++i) {
    if (label(i)) ++tps;
    else ++fps;
    const bool end = i + 1 == n || !(value(i) == value(i + 1));  // NaN != NaN: a group of its own
    if (end) {
      area += static_cast<double>(fps - fp_prev) * static_cast<double>(tps + tp_prev);
      const int64_t tot = tps + fps;
      const double prec = tot > 0 ? static_cast<double>(tps) / static_cast<double>(tot) : 0.0;
      ap += static_cast<double>(tps - tp_prev) * prec;
      tp_prev = tps;
      fp_prev = fps;
    }
  }
  const double P = static_cast<double>(tps), N = static_cast<double>(fps);
  Scores s;
  s.auroc = (tps > 0 && fps > 0) ? area / (2.0 * P * N) : 0.0;
  s.ap = tps > 0 ? ap / P : std::numeric_limits<double>::quiet_NaN();
  s.pos = P;
  s.neg = N;
  return s;
}

}  // namespace

// preds [N, C] (or [N]) floating; labels [N, C] (or [N]) bool / integer 0-1; valid optional, same shape -> [C, 4] f64
at::Tensor curve_scores_host(const at::Tensor& preds_in, const at::Tensor& labels_in, const c10::optional<at::Tensor>& valid_in) {
  TORCH_CHECK(preds_in.device().is_cpu(), "curve_scores_host: CPU tensors only");
  TORCH_CHECK(preds_in.is_floating_point(), "curve_scores_host: floating scores");
  at::Tensor preds = preds_in.dim() == 1 ? preds_in.unsqueeze(1) : preds_in;
  // labels: [N, C] 0/1 (binary / multilabel), or int64 class ids [N] against [N, C] scores (multiclass one-vs-rest:
  // label = target == c, no one-hot matrix)
  const bool class_ids = labels_in.dim() == 1 && preds.dim() == 2 && preds.size(1) > 1 && labels_in.scalar_type() == at::kLong;
  at::Tensor labels = class_ids ? labels_in : (labels_in.dim() == 1 ? labels_in.unsqueeze(1) : labels_in);
  TORCH_CHECK(preds.dim() == 2 && (class_ids ? labels.size(0) == preds.size(0) : labels.sizes() == preds.sizes()),
              "curve_scores_host: preds [N, C] with labels [N, C] (or int64 class ids [N])");
  const int64_t N = preds.size(0), C = preds.size(1);
  if (preds.scalar_type() != at::kDouble) preds = preds.to(at::kFloat);  // 16-bit scores compare as their float values
  const at::Tensor pc = preds.t().contiguous();                           // [C, N]: one contiguous run per column
  const at::Tensor lc = class_ids ? at::Tensor() : labels.t().to(at::kByte).contiguous();
  const at::Tensor ids = class_ids ? labels.contiguous() : at::Tensor();
  at::Tensor vc;
  if (valid_in.has_value()) {
    at::Tensor v = valid_in->dim() == 1 ? valid_in->unsqueeze(1) : *valid_in;
    TORCH_CHECK(v.sizes() == preds.sizes(), "curve_scores_host: valid must match preds");
    vc = v.t().to(at::kByte).contiguous();
  }
  at::Tensor out = at::empty({C, 4}, preds.options().dtype(at::kDouble));
  double* o = out.data_ptr<double>();
  const uint8_t* L = class_ids ? nullptr : lc.data_ptr<uint8_t>();
  const int64_t* IDS = class_ids ? ids.data_ptr<int64_t>() : nullptr;
  const uint8_t* VV = vc.defined() ? vc.data_ptr<uint8_t>() : nullptr;
  const bool f64 = pc.scalar_type() == at::kDouble;
  const float* P32 = f64 ? nullptr : pc.data_ptr<float>();
  const double* P64 = f64 ? pc.data_ptr<double>() : nullptr;
  at::parallel_for(0, C, 1, [&](int64_t c0, int64_t c1) {
    std::vector<uint64_t> a, tmp;
    a.reserve(static_cast<size_t>(N));
    for (int64_t c = c0; c < c1; ++c) {
      const uint8_t* l = L ? L + c * N : nullptr;
      auto lab = [&](int64_t i) -> bool { return l ? l[i] != 0 : IDS[i] == c; };
      const uint8_t* vv = VV ? VV + c * N : nullptr;
      a.clear();
      Scores s;
      if (!f64) {
        const float* p = P32 + c * N;
        for (int64_t i = 0; i < N; ++i) {
          if (vv && !vv[i]) continue;
          a.push_back((static_cast<uint64_t>(desc_key32(p[i])) << 32) | (lab(i) ? 1u : 0u));
        }
        radix_sort(a, tmp, 4);
        s = scan(a.size(), [&](size_t i) { return key_value32(static_cast<uint32_t>(a[i] >> 32)); },
                 [&](size_t i) { return (a[i] & 1u) != 0; });
      } else {
        // fp64: the 64-bit key leaves no room for the label, so the sort carries each entry's index alongside
        const double* p = P64 + c * N;
        std::vector<uint32_t> idx;
        for (int64_t i = 0; i < N; ++i) {
          if (vv && !vv[i]) continue;
          a.push_back(desc_key64(p[i]));
          idx.push_back(static_cast<uint32_t>(i));
        }
        const size_t n = a.size();
        std::vector<uint64_t> ka(a), kt(n);
        std::vector<uint32_t> ia(idx), it(n);
        for (int b = 0; b < 8; ++b) {
          const int shift = 8 * b;
          size_t cnt[256] = {0};
          for (size_t i = 0; i < n; ++i) ++cnt[(ka[i] >> shift) & 0xFF];
          bool trivial = false;
          for (int d = 0; d < 256; ++d)
            if (cnt[d] == n) trivial = true;
          if (trivial) continue;
          size_t off = 0;
          for (int d = 0; d < 256; ++d) {
            const size_t cc = cnt[d];
            cnt[d] = off;
            off += cc;
          }
          for (size_t i = 0; i < n; ++i) {
            const size_t dst = cnt[(ka[i] >> shift) & 0xFF]++;
            kt[dst] = ka[i];
            it[dst] = ia[i];
          }
          ka.swap(kt);
          ia.swap(it);
        }
        s = scan(n, [&](size_t i) { return key_value64(ka[i]); }, [&](size_t i) { return lab(ia[i]); });
      }
      o[4 * c + 0] = s.auroc;
      o[4 * c + 1] = s.ap;
      o[4 * c + 2] = s.pos;
      o[4 * c + 3] = s.neg;
    }
  });
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("curve_scores_host(Tensor preds, Tensor labels, Tensor? valid) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CPU, m) { m.impl("curve_scores_host", &tmx::curve_scores_host); }
