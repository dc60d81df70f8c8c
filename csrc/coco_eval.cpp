// Native COCO-style detection evaluator (behaviour of pycocotools' COCOeval evaluate +
// accumulate, re-implemented in C++ for the framework's MeanAveragePrecision).
//
// Host-side C++ (the matching is a sequential greedy scan per (image, class, area range)); work is spread over
// categories with at::parallel_for.  Inputs are flat CPU tensors with one row per detection / ground-truth box
// (image index + label columns), so the Python side never builds COCO JSON dictionaries.
//
//   * IoU: axis-aligned boxes in xywh (crowd ground truth: intersection / detection area), or a caller-supplied
//     per-image IoU matrix (segmentation masks are intersected on the GPU by the caller).
//   * evaluateImg: detections sorted by score (stable), truncated to maxDets[-1]; ground truth ordered with
//     non-ignored first; greedy matching per IoU threshold preferring non-ignored / non-crowd matches.
//   * accumulate: per (class, area, maxDet) the image results are concatenated in image order, stably sorted
//     by score, cumulative TP/FP, precision envelope and recall-threshold sampling (searchsorted, left).
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <tuple>
#include <vector>

namespace tmx {
namespace {

struct ImgCat {
  std::vector<int64_t> dets;  // detection row ids, sorted by score desc (stable), truncated to max_det
  std::vector<int64_t> gts;   // ground-truth row ids, input order
  std::vector<double> iou;    // [dets x gts] row-major
};

struct EvalImg {
  bool valid = false;
  std::vector<double> scores;        // [D]
  std::vector<uint8_t> matched;      // [T x D]
  std::vector<uint8_t> det_ignore;   // [T x D]
  int64_t num_gt_not_ignored = 0;
};

inline double box_iou(const double* d, const double* g, bool crowd) {
  const double ow = std::min(d[0] + d[2], g[0] + g[2]) - std::max(d[0], g[0]);
  if (ow <= 0) return 0.0;
  const double oh = std::min(d[1] + d[3], g[1] + g[3]) - std::max(d[1], g[1]);
  if (oh <= 0) return 0.0;
  const double inter = ow * oh;
  const double u = crowd ? d[2] * d[3] : d[2] * d[3] + g[2] * g[3] - inter;
  return u > 0 ? inter / u : 0.0;
}

}  // namespace

// Returns (precision [T,R,K,A,M], recall [T,K,A,M], scores [T,R,K,A,M], iou_values [P], iou_index [Q,5]) where the
// iou_index rows are (image, category index, n_det, n_gt, offset) for every evaluated (image, category) pair.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> coco_evaluate(
    const at::Tensor& det_boxes_, const at::Tensor& det_scores_, const at::Tensor& det_labels_, const at::Tensor& det_img_,
    const at::Tensor& det_area_, const at::Tensor& gt_boxes_, const at::Tensor& gt_labels_, const at::Tensor& gt_img_,
    const at::Tensor& gt_crowd_, const at::Tensor& gt_area_, const at::Tensor& cat_ids_, int64_t num_images,
    const at::Tensor& iou_thrs_, const at::Tensor& rec_thrs_, const at::Tensor& max_dets_, const at::Tensor& area_rng_,
    const c10::optional<at::Tensor>& img_iou_, const c10::optional<at::Tensor>& img_iou_offsets_) {
  auto f64 = [](const at::Tensor& t) { return t.to(at::kCPU).to(at::kDouble).contiguous(); };
  auto i64 = [](const at::Tensor& t) { return t.to(at::kCPU).to(at::kLong).contiguous(); };
  const auto det_boxes = f64(det_boxes_), det_scores = f64(det_scores_), det_area = f64(det_area_);
  const auto gt_boxes = f64(gt_boxes_), gt_area = f64(gt_area_);
  const auto det_labels = i64(det_labels_), det_img = i64(det_img_), gt_labels = i64(gt_labels_), gt_img = i64(gt_img_);
  const auto gt_crowd = i64(gt_crowd_), cat_ids = i64(cat_ids_), max_dets = i64(max_dets_);
  const auto iou_thrs = f64(iou_thrs_), rec_thrs = f64(rec_thrs_), area_rng = f64(area_rng_);
  const bool custom_iou = img_iou_.has_value() && img_iou_->defined();
  at::Tensor img_iou, img_iou_off;
  if (custom_iou) {
    img_iou = f64(*img_iou_);
    img_iou_off = i64(*img_iou_offsets_);
  }

  const int64_t Nd = det_scores.numel(), Ng = gt_labels.numel();
  const int64_t K = cat_ids.numel(), T = iou_thrs.numel(), R = rec_thrs.numel(), M = max_dets.numel();
  const int64_t A = area_rng.size(0), I = num_images;
  TORCH_CHECK(M > 0 && T > 0 && R > 0 && A > 0, "coco_evaluate: empty parameter list");
  const double* db = det_boxes.data_ptr<double>();
  const double* ds = det_scores.data_ptr<double>();
  const double* da = det_area.data_ptr<double>();
  const double* gb = gt_boxes.data_ptr<double>();
  const double* ga = gt_area.data_ptr<double>();
  const int64_t* dl = det_labels.data_ptr<int64_t>();
  const int64_t* di = det_img.data_ptr<int64_t>();
  const int64_t* gl = gt_labels.data_ptr<int64_t>();
  const int64_t* gi = gt_img.data_ptr<int64_t>();
  const int64_t* gc = gt_crowd.data_ptr<int64_t>();
  const int64_t* cats = cat_ids.data_ptr<int64_t>();
  const double* thr = iou_thrs.data_ptr<double>();
  const double* rthr = rec_thrs.data_ptr<double>();
  const int64_t* mdet = max_dets.data_ptr<int64_t>();
  const double* arng = area_rng.data_ptr<double>();
  const int64_t max_det_last = mdet[M - 1];

  auto cat_index = [&](int64_t label) -> int64_t {
    const int64_t* it = std::lower_bound(cats, cats + K, label);
    return (it != cats + K && *it == label) ? (it - cats) : -1;
  };

  // per-image row offsets of detections / ground truth (rows of one image are contiguous in input order)
  std::vector<std::vector<int64_t>> det_rows_of_img(I), gt_rows_of_img(I);
  for (int64_t d = 0; d < Nd; ++d) det_rows_of_img[di[d]].push_back(d);
  for (int64_t g = 0; g < Ng; ++g) gt_rows_of_img[gi[g]].push_back(g);

  // ---- group by (image, category), sort detections, IoU ------------------------------------------------
  std::vector<ImgCat> groups(static_cast<size_t>(I * K));
  at::parallel_for(0, I, 1, [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      for (int64_t d : det_rows_of_img[i]) {
        const int64_t k = cat_index(dl[d]);
        if (k >= 0) groups[i * K + k].dets.push_back(d);
      }
      for (int64_t g : gt_rows_of_img[i]) {
        const int64_t k = cat_index(gl[g]);
        if (k >= 0) groups[i * K + k].gts.push_back(g);
      }
      for (int64_t k = 0; k < K; ++k) {
        ImgCat& gc_ = groups[i * K + k];
        std::stable_sort(gc_.dets.begin(), gc_.dets.end(), [&](int64_t a, int64_t b) { return ds[a] > ds[b]; });
        if (static_cast<int64_t>(gc_.dets.size()) > max_det_last) gc_.dets.resize(max_det_last);
        const size_t nd = gc_.dets.size(), ng = gc_.gts.size();
        gc_.iou.assign(nd * ng, 0.0);
        if (nd == 0 || ng == 0) continue;
        if (custom_iou) {
          // per-image matrix over all detections x all ground truths of the image (input order)
          const int64_t off = img_iou_off.data_ptr<int64_t>()[i];
          const int64_t img_ng = static_cast<int64_t>(gt_rows_of_img[i].size());
          const int64_t d0 = det_rows_of_img[i].empty() ? 0 : det_rows_of_img[i][0];
          const int64_t g0 = gt_rows_of_img[i].empty() ? 0 : gt_rows_of_img[i][0];
          const double* mat = img_iou.data_ptr<double>() + off;
          for (size_t a = 0; a < nd; ++a)
            for (size_t b = 0; b < ng; ++b) gc_.iou[a * ng + b] = mat[(gc_.dets[a] - d0) * img_ng + (gc_.gts[b] - g0)];
        } else {
          for (size_t a = 0; a < nd; ++a)
            for (size_t b = 0; b < ng; ++b)
              gc_.iou[a * ng + b] = box_iou(db + 4 * gc_.dets[a], gb + 4 * gc_.gts[b], gc[gc_.gts[b]] != 0);
        }
      }
    }
  });

  // ---- evaluateImg for every (category, area, image) -----------------------------------------------------
  std::vector<EvalImg> evals(static_cast<size_t>(K * A * I));
  at::parallel_for(0, K * A, 1, [&](int64_t ka0, int64_t ka1) {
    std::vector<int64_t> gt_order;
    std::vector<uint8_t> gt_ig, gt_crowd_sorted;
    std::vector<int64_t> gtm;
    for (int64_t ka = ka0; ka < ka1; ++ka) {
      const int64_t k = ka / A, a = ka % A;
      const double lo = arng[2 * a], hi = arng[2 * a + 1];
      for (int64_t i = 0; i < I; ++i) {
        const ImgCat& g = groups[i * K + k];
        const int64_t D = static_cast<int64_t>(g.dets.size()), G = static_cast<int64_t>(g.gts.size());
        EvalImg& e = evals[(k * A + a) * I + i];
        if (D == 0 && G == 0) continue;
        e.valid = true;
        // ground truth: ignore flag, non-ignored first (stable)
        gt_order.resize(G);
        std::iota(gt_order.begin(), gt_order.end(), 0);
        std::vector<uint8_t> ig(G);
        for (int64_t b = 0; b < G; ++b) {
          const int64_t row = g.gts[b];
          ig[b] = (gc[row] != 0 || ga[row] < lo || ga[row] > hi) ? 1 : 0;
        }
        std::stable_sort(gt_order.begin(), gt_order.end(), [&](int64_t x, int64_t y) { return ig[x] < ig[y]; });
        gt_ig.resize(G);
        gt_crowd_sorted.resize(G);
        for (int64_t b = 0; b < G; ++b) {
          gt_ig[b] = ig[gt_order[b]];
          gt_crowd_sorted[b] = gc[g.gts[gt_order[b]]] != 0;
          if (!gt_ig[b]) ++e.num_gt_not_ignored;
        }
        e.scores.resize(D);
        for (int64_t d = 0; d < D; ++d) e.scores[d] = ds[g.dets[d]];
        e.matched.assign(T * D, 0);
        e.det_ignore.assign(T * D, 0);
        gtm.assign(T * G, 0);
        for (int64_t t = 0; t < T; ++t) {
          for (int64_t d = 0; d < D; ++d) {
            double best = std::min(thr[t], 1.0 - 1e-10);
            int64_t m = -1;
            for (int64_t b = 0; b < G; ++b) {
              if (gtm[t * G + b] && !gt_crowd_sorted[b]) continue;
              if (m > -1 && gt_ig[m] == 0 && gt_ig[b] == 1) break;
              const double v = g.iou[d * G + gt_order[b]];
              if (v < best) continue;
              best = v;
              m = b;
            }
            if (m == -1) continue;
            e.det_ignore[t * D + d] = gt_ig[m];
            e.matched[t * D + d] = 1;
            gtm[t * G + m] = 1;
          }
        }
        for (int64_t d = 0; d < D; ++d) {
          const double ar = da[g.dets[d]];
          if (ar < lo || ar > hi)
            for (int64_t t = 0; t < T; ++t)
              if (!e.matched[t * D + d]) e.det_ignore[t * D + d] = 1;
        }
      }
    }
  });

  // ---- accumulate ----------------------------------------------------------------------------------------
  auto precision = at::full({T, R, K, A, M}, -1.0, at::kDouble);
  auto recall = at::full({T, K, A, M}, -1.0, at::kDouble);
  auto scores_out = at::full({T, R, K, A, M}, -1.0, at::kDouble);
  double* P = precision.data_ptr<double>();
  double* Rc = recall.data_ptr<double>();
  double* S = scores_out.data_ptr<double>();
  const double eps = 2.220446049250313e-16;  // np.spacing(1)
  at::parallel_for(0, K * A * M, 1, [&](int64_t q0, int64_t q1) {
    std::vector<double> sc, tp_sum, fp_sum, rc, pr;
    std::vector<uint8_t> mt, ig;
    std::vector<int64_t> order;
    for (int64_t q = q0; q < q1; ++q) {
      const int64_t k = q / (A * M), a = (q / M) % A, m = q % M;
      const int64_t maxd = mdet[m];
      sc.clear();
      int64_t npig = 0;
      bool any = false;
      std::vector<std::pair<int64_t, int64_t>> src;  // (eval index, det index)
      for (int64_t i = 0; i < I; ++i) {
        const EvalImg& e = evals[(k * A + a) * I + i];
        if (!e.valid) continue;
        any = true;
        npig += e.num_gt_not_ignored;
        const int64_t D = static_cast<int64_t>(e.scores.size());
        const int64_t use = std::min<int64_t>(D, maxd);
        for (int64_t d = 0; d < use; ++d) {
          sc.push_back(e.scores[d]);
          src.emplace_back((k * A + a) * I + i, d);
        }
      }
      if (!any || npig == 0) continue;
      const int64_t nd = static_cast<int64_t>(sc.size());
      order.resize(nd);
      std::iota(order.begin(), order.end(), 0);
      std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return sc[x] > sc[y]; });
      for (int64_t t = 0; t < T; ++t) {
        tp_sum.assign(nd, 0.0);
        fp_sum.assign(nd, 0.0);
        double tp = 0, fp = 0;
        for (int64_t j = 0; j < nd; ++j) {
          const auto& s = src[order[j]];
          const EvalImg& e = evals[s.first];
          const int64_t D = static_cast<int64_t>(e.scores.size());
          const bool mtd = e.matched[t * D + s.second];
          const bool igd = e.det_ignore[t * D + s.second];
          if (mtd && !igd) tp += 1;
          if (!mtd && !igd) fp += 1;
          tp_sum[j] = tp;
          fp_sum[j] = fp;
        }
        rc.resize(nd);
        pr.resize(nd);
        for (int64_t j = 0; j < nd; ++j) {
          rc[j] = tp_sum[j] / static_cast<double>(npig);
          pr[j] = tp_sum[j] / (fp_sum[j] + tp_sum[j] + eps);
        }
        Rc[((t * K + k) * A + a) * M + m] = nd ? rc[nd - 1] : 0.0;
        for (int64_t j = nd - 1; j > 0; --j)
          if (pr[j] > pr[j - 1]) pr[j - 1] = pr[j];
        for (int64_t r = 0; r < R; ++r) {
          const int64_t pi = std::lower_bound(rc.begin(), rc.end(), rthr[r]) - rc.begin();
          const int64_t idx = (((t * R + r) * K + k) * A + a) * M + m;
          if (pi < nd) {
            P[idx] = pr[pi];
            S[idx] = sc[order[pi]];
          } else {
            // pycocotools stops filling at the first out-of-range index: the rest stay 0
            for (int64_t rr = r; rr < R; ++rr) {
              const int64_t id2 = (((t * R + rr) * K + k) * A + a) * M + m;
              P[id2] = 0.0;
              S[id2] = 0.0;
            }
            break;
          }
        }
      }
    }
  });

  // ---- IoU export (extended summary) ---------------------------------------------------------------------
  int64_t total = 0, pairs = 0;
  for (int64_t i = 0; i < I; ++i)
    for (int64_t k = 0; k < K; ++k) {
      total += static_cast<int64_t>(groups[i * K + k].iou.size());
      ++pairs;
    }
  auto iou_values = at::empty({total}, at::kDouble);
  auto iou_index = at::empty({pairs, 5}, at::kLong);
  double* iv = iou_values.data_ptr<double>();
  int64_t* ix = iou_index.data_ptr<int64_t>();
  int64_t off = 0, p = 0;
  for (int64_t i = 0; i < I; ++i)
    for (int64_t k = 0; k < K; ++k, ++p) {
      const ImgCat& g = groups[i * K + k];
      std::copy(g.iou.begin(), g.iou.end(), iv + off);
      ix[5 * p + 0] = i;
      ix[5 * p + 1] = k;
      ix[5 * p + 2] = static_cast<int64_t>(g.dets.size());
      ix[5 * p + 3] = static_cast<int64_t>(g.gts.size());
      ix[5 * p + 4] = off;
      off += static_cast<int64_t>(g.iou.size());
    }
  return {precision, recall, scores_out, iou_values, iou_index};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def(
      "coco_evaluate(Tensor det_boxes, Tensor det_scores, Tensor det_labels, Tensor det_img, Tensor det_area, "
      "Tensor gt_boxes, Tensor gt_labels, Tensor gt_img, Tensor gt_crowd, Tensor gt_area, Tensor cat_ids, "
      "int num_images, Tensor iou_thrs, Tensor rec_thrs, Tensor max_dets, Tensor area_rng, Tensor? img_iou, "
      "Tensor? img_iou_offsets) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(tmx, CompositeExplicitAutograd, m) { m.impl("coco_evaluate", &tmx::coco_evaluate); }
