// Host (CPU) twins of the multiclass pair-stream kernels for small CPU batches (BASELINE config 1: MulticlassAccuracy,
// 5 classes, batch 10, gloo).  The reference's CPU update is ~10 ATen calls per batch (unique for validation, argmax,
// bincount of t * C + p, reshape, diag, three sums, four in-place adds) plus a module __setattr__ per state.  Here ONE
// dispatcher call does the eager value check, the arg-max and the in-place accumulation:
//
//   mc_stats_host   : tp / fp / tn / fn (per class, or micro totals) += counts of the (target, arg-max) pairs
//   mc_confmat_host : confmat[t, p] += 1
//
// Semantics = the eager PyTorch paths in ops/classification.py (rows whose target is the ignore index or outside
// [0, C), or whose label pred is outside [0, C), are dropped) and the reference's validation rule
// (reference functional/classification/stat_scores.py:307-314): more distinct target values than C (+1 with an
// ignore index), or more distinct integer preds than C, is an error.  The op validates FIRST and accumulates only when
// the batch passes; it returns {passed, distinct targets, distinct preds} and the caller raises the reference's error
// text.  torch.argmax semantics: the first maximum, a NaN counts as the maximum (first NaN wins).
#include <ATen/ATen.h>
#include <ATen/Dispatch.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace tmx {
namespace {

// distinct values of an int64 stream: bitmap over [0, C] (C = an ignore-index slot may sit outside), sorted vector for
// the rest (rare: out-of-range values)
struct DistinctCounter {
  std::vector<uint8_t> seen;
  std::vector<int64_t> other;
  int64_t count = 0;
  explicit DistinctCounter(int64_t C) : seen(static_cast<size_t>(C), 0) {}
  void add(int64_t v) {
    if (v >= 0 && v < static_cast<int64_t>(seen.size())) {
      if (!seen[v]) {
        seen[v] = 1;
        ++count;
      }
    } else {
      other.push_back(v);
    }
  }
  int64_t total() {
    std::sort(other.begin(), other.end());
    return count + static_cast<int64_t>(std::unique(other.begin(), other.end()) - other.begin());
  }
};

template <typename T>
inline float to_float(T v) {
  return static_cast<float>(v);
}

// labels of the batch: arg-max of float rows [M, C] or the integer preds [M]; int64 out
void labels_of(const at::Tensor& preds, int64_t C, std::vector<int64_t>& out) {
  if (preds.is_floating_point()) {
    TORCH_CHECK(preds.dim() == 2 && preds.size(1) == C, "mc host op: float preds must be [M, C]");
    const at::Tensor p = preds.contiguous();
    const int64_t M = p.size(0);
    out.resize(static_cast<size_t>(M));
    AT_DISPATCH_FLOATING_TYPES_AND2(at::kHalf, at::kBFloat16, p.scalar_type(), "mc_labels_host", [&] {
      const scalar_t* x = p.data_ptr<scalar_t>();
      for (int64_t r = 0; r < M; ++r) {
        const scalar_t* row = x + r * C;
        int64_t best = 0;
        float bv = to_float(row[0]);
        if (!std::isnan(bv)) {
          for (int64_t c = 1; c < C; ++c) {
            const float v = to_float(row[c]);
            if (std::isnan(v)) {
              best = c;
              break;
            }
            if (v > bv) {
              bv = v;
              best = c;
            }
          }
        }
        out[static_cast<size_t>(r)] = best;
      }
    });
  } else {
    const at::Tensor p = preds.reshape(-1).to(at::kLong).contiguous();
    const int64_t* x = p.data_ptr<int64_t>();
    out.assign(x, x + p.numel());
  }
}

void targets_of(const at::Tensor& target, std::vector<int64_t>& out) {
  const at::Tensor t = target.reshape(-1).to(at::kLong).contiguous();
  const int64_t* x = t.data_ptr<int64_t>();
  out.assign(x, x + t.numel());
}

// {passed, distinct targets, distinct integer preds (0 for float preds)}
std::vector<int64_t> validate(const std::vector<int64_t>& t, const std::vector<int64_t>& p, bool float_preds, int64_t C,
                              bool has_ignore) {
  DistinctCounter dt(C + 1);
  for (int64_t v : t) dt.add(v);
  const int64_t nt = dt.total();
  int64_t np = 0;
  if (!float_preds) {
    DistinctCounter dp(C);
    for (int64_t v : p) dp.add(v);
    np = dp.total();
  }
  const bool ok = nt <= (has_ignore ? C + 1 : C) && (float_preds || np <= C);
  return {ok ? 1 : 0, nt, np};
}

void check_state(const at::Tensor& s, const char* what) {
  TORCH_CHECK(s.device().is_cpu() && s.scalar_type() == at::kLong && s.is_contiguous(), what, " must be a contiguous CPU int64 tensor");
}

}  // namespace

std::vector<int64_t> mc_stats_host(const at::Tensor& preds, const at::Tensor& target, int64_t C, at::Tensor& tp, at::Tensor& fp,
                                   at::Tensor& tn, at::Tensor& fn, int64_t ignore_index, bool has_ignore, bool micro,
                                   bool validate_values) {
  TORCH_CHECK(C >= 1, "mc_stats_host: num_classes must be positive");
  for (const at::Tensor* s : {&tp, &fp, &tn, &fn}) check_state(*s, "mc_stats_host: state");
  TORCH_CHECK(tp.numel() == (micro ? 1 : C) && fp.numel() == tp.numel() && tn.numel() == tp.numel() && fn.numel() == tp.numel(),
              "mc_stats_host: states must hold ", micro ? 1 : C, " counters");
  std::vector<int64_t> p, t;
  labels_of(preds, C, p);
  targets_of(target, t);
  TORCH_CHECK(p.size() == t.size(), "mc_stats_host: preds rows and targets differ in count");
  std::vector<int64_t> res{1, 0, 0};
  if (validate_values) {
    res = validate(t, p, preds.is_floating_point(), C, has_ignore);
    if (!res[0]) return res;
  }
  int64_t* TP = tp.data_ptr<int64_t>();
  int64_t* FP = fp.data_ptr<int64_t>();
  int64_t* TN = tn.data_ptr<int64_t>();
  int64_t* FN = fn.data_ptr<int64_t>();
  if (micro) {
    int64_t n = 0, hit = 0;
    for (size_t i = 0; i < t.size(); ++i) {
      const int64_t tv = t[i], pv = p[i];
      if ((has_ignore && tv == ignore_index) || tv < 0 || tv >= C || pv < 0 || pv >= C) continue;
      ++n;
      hit += tv == pv;
    }
    TP[0] += hit;
    FP[0] += n - hit;
    FN[0] += n - hit;
    TN[0] += C * n - (hit + 2 * (n - hit));
    return res;
  }
  // per class: tp_c, fp_c (predicted c, wrong), fn_c (true c, missed); tn_c = n - tp_c - fp_c - fn_c
  int64_t n = 0;
  std::vector<int64_t> dtp(static_cast<size_t>(C), 0), dfp(static_cast<size_t>(C), 0), dfn(static_cast<size_t>(C), 0);
  for (size_t i = 0; i < t.size(); ++i) {
    const int64_t tv = t[i], pv = p[i];
    if ((has_ignore && tv == ignore_index) || tv < 0 || tv >= C || pv < 0 || pv >= C) continue;
    ++n;
    if (tv == pv) {
      ++dtp[tv];
    } else {
      ++dfp[pv];
      ++dfn[tv];
    }
  }
  for (int64_t c = 0; c < C; ++c) {
    TP[c] += dtp[c];
    FP[c] += dfp[c];
    FN[c] += dfn[c];
    TN[c] += n - dtp[c] - dfp[c] - dfn[c];
  }
  return res;
}

std::vector<int64_t> mc_confmat_host(const at::Tensor& preds, const at::Tensor& target, at::Tensor& confmat, int64_t ignore_index,
                                     bool has_ignore, bool validate_values) {
  check_state(confmat, "mc_confmat_host: confmat");
  TORCH_CHECK(confmat.dim() == 2 && confmat.size(0) == confmat.size(1), "mc_confmat_host: confmat must be [C, C]");
  const int64_t C = confmat.size(0);
  std::vector<int64_t> p, t;
  labels_of(preds, C, p);
  targets_of(target, t);
  TORCH_CHECK(p.size() == t.size(), "mc_confmat_host: preds rows and targets differ in count");
  std::vector<int64_t> res{1, 0, 0};
  if (validate_values) {
    res = validate(t, p, preds.is_floating_point(), C, has_ignore);
    if (!res[0]) return res;
  }
  int64_t* cm = confmat.data_ptr<int64_t>();
  for (size_t i = 0; i < t.size(); ++i) {
    const int64_t tv = t[i], pv = p[i];
    if ((has_ignore && tv == ignore_index) || tv < 0 || tv >= C || pv < 0 || pv >= C) continue;
    ++cm[tv * C + pv];
  }
  return res;
}


// ---------------------------------------------------------------------------------------------------------------
// stat_reduce_host: the final reduction of every (tp, fp, tn, fn) metric -- accuracy, precision, recall, F-beta,
// specificity, Hamming distance -- for CPU int64 states in ONE call (functional/classification/_stat_family.py).
// The Python chain (sums, _safe_divide, _adjust_weights_safe_divide) is ~15 ATen calls of a few microseconds each on
// [C]-sized tensors; at BASELINE config 1 (5 classes, batch 10) it was the largest part of a CPU forward().  Same
// float32 operations in the same order as that chain (int64 sums, int64 -> float32 casts, a denominator of 0 read as 1,
// F-beta's (1 + b2) tp + b2 fn + fp in float32), except the final sum over classes of macro / weighted averages, which is
// accumulated in double and rounded once (ATen's vectorised float32 sum may differ in the last bit).
//   kind: 0 accuracy, 1 precision, 2 recall, 3 fbeta, 4 specificity, 5 hamming
//   average: 0 binary (elementwise), 1 micro, 2 macro, 3 weighted, 4 none (elementwise)
// States [C] (global) or [N, C] (samplewise: reductions over the last dim), or any shape for binary.
namespace {

#pragma clang fp contract(off)
inline float sdiv(float num, float den) { return num / (den == 0.f ? 1.f : den); }

inline float stat_score(int kind, bool elementwise_acc, bool multilabel, int64_t tp, int64_t fp, int64_t tn, int64_t fn, float k1, float b2) {
  switch (kind) {
    case 0:
    case 5: {
      const float s = (elementwise_acc || multilabel) ? sdiv(static_cast<float>(tp + tn), static_cast<float>(tp + tn + fp + fn))
                                                      : sdiv(static_cast<float>(tp), static_cast<float>(tp + fn));
      return kind == 0 ? s : 1.f - s;
    }
    case 1: return sdiv(static_cast<float>(tp), static_cast<float>(tp + fp));
    case 2: return sdiv(static_cast<float>(tp), static_cast<float>(tp + fn));
    case 3: {
      const float num = k1 * static_cast<float>(tp);
      const float den = (num + b2 * static_cast<float>(fn)) + static_cast<float>(fp);
      return sdiv(num, den);
    }
    default: return sdiv(static_cast<float>(tn), static_cast<float>(tn + fp));
  }
}

}  // namespace

at::Tensor stat_reduce_host(const at::Tensor& tp_t, const at::Tensor& fp_t, const at::Tensor& tn_t, const at::Tensor& fn_t, int64_t kind,
                            int64_t average, bool multilabel, double beta) {
  TORCH_CHECK(kind >= 0 && kind <= 5 && average >= 0 && average <= 4, "stat_reduce_host: bad kind / average");
  for (const at::Tensor* t : {&tp_t, &fp_t, &tn_t, &fn_t})
    TORCH_CHECK(t->device().is_cpu() && t->scalar_type() == at::kLong && t->sizes() == tp_t.sizes(),
                "stat_reduce_host: int64 CPU states of one shape");
  const at::Tensor tp = tp_t.contiguous(), fp = fp_t.contiguous(), tn = tn_t.contiguous(), fn = fn_t.contiguous();
  const int64_t* a = tp.data_ptr<int64_t>();
  const int64_t* b = fp.data_ptr<int64_t>();
  const int64_t* c = tn.data_ptr<int64_t>();
  const int64_t* d = fn.data_ptr<int64_t>();
  const double b2d = beta * beta;
  const float k1 = static_cast<float>(1.0 + b2d), b2 = static_cast<float>(b2d);
  const auto fopt = at::TensorOptions().dtype(at::kFloat);
  if (average == 0 || average == 4) {  // elementwise
    at::Tensor out = at::empty(tp.sizes(), fopt);
    float* o = out.data_ptr<float>();
    const int64_t n = tp.numel();
    for (int64_t i = 0; i < n; ++i) o[i] = stat_score(static_cast<int>(kind), average == 0, multilabel, a[i], b[i], c[i], d[i], k1, b2);
    return out;
  }
  TORCH_CHECK(tp.dim() <= 2, "stat_reduce_host: micro / macro / weighted need [], [C] or [N, C] states");
  const int64_t C = tp.dim() == 0 ? 1 : tp.size(-1), R = tp.dim() == 2 ? tp.size(0) : 1;
  at::Tensor out = tp.dim() == 2 ? at::empty({R}, fopt) : at::empty({}, fopt);
  float* o = out.data_ptr<float>();
  for (int64_t r = 0; r < R; ++r) {
    const int64_t* ar = a + r * C;
    const int64_t* br = b + r * C;
    const int64_t* cr = c + r * C;
    const int64_t* dr = d + r * C;
    if (average == 1) {  // micro: int64 totals, then the elementwise formula
      int64_t st[4] = {0, 0, 0, 0};
      for (int64_t i = 0; i < C; ++i) {
        st[0] += ar[i];
        st[1] += br[i];
        st[2] += cr[i];
        st[3] += dr[i];
      }
      o[r] = stat_score(static_cast<int>(kind), false, multilabel, st[0], st[1], st[2], st[3], k1, b2);
      continue;
    }
    // macro / weighted: _adjust_weights_safe_divide(score, average, multilabel, tp, fp, fn)
    double acc = 0.0;
    if (average == 3) {
      int64_t ws = 0;
      for (int64_t i = 0; i < C; ++i) ws += ar[i] + dr[i];
      const float den = static_cast<float>(ws == 0 ? 1 : ws);
      for (int64_t i = 0; i < C; ++i) {
        const float sc = stat_score(static_cast<int>(kind), false, multilabel, ar[i], br[i], cr[i], dr[i], k1, b2);
        acc += static_cast<double>((static_cast<float>(ar[i] + dr[i]) * sc) / den);
      }
    } else {
      float wsum = 0.f;
      for (int64_t i = 0; i < C; ++i) wsum += (multilabel || ar[i] + br[i] + dr[i] != 0) ? 1.f : 0.f;
      const float den = wsum == 0.f ? 1.f : wsum;
      for (int64_t i = 0; i < C; ++i) {
        const float w = (multilabel || ar[i] + br[i] + dr[i] != 0) ? 1.f : 0.f;
        const float sc = stat_score(static_cast<int>(kind), false, multilabel, ar[i], br[i], cr[i], dr[i], k1, b2);
        acc += static_cast<double>((w * sc) / den);
      }
    }
    o[r] = static_cast<float>(acc);
  }
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("mc_stats_host(Tensor preds, Tensor target, int num_classes, Tensor(a!) tp, Tensor(b!) fp, Tensor(c!) tn, Tensor(d!) fn, int ignore_index, bool has_ignore, bool micro, bool validate) -> int[]");
  m.def("mc_confmat_host(Tensor preds, Tensor target, Tensor(a!) confmat, int ignore_index, bool has_ignore, bool validate) -> int[]");
  m.def("stat_reduce_host(Tensor tp, Tensor fp, Tensor tn, Tensor fn, int kind, int average, bool multilabel, float beta) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CPU, m) {
  m.impl("mc_stats_host", &tmx::mc_stats_host);
  m.impl("mc_confmat_host", &tmx::mc_confmat_host);
  m.impl("stat_reduce_host", &tmx::stat_reduce_host);
}
