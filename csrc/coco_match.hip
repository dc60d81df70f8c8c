// COCO evaluation on the GPU: pycocotools' evaluateImg + accumulate semantics for
// MeanAveragePrecision, without leaving the device.  Replaces the reference's COCO JSON round trip through
// pycocotools / faster-coco-eval (reference detection/mean_ap.py:501-575, legacy matcher _mean_ap.py:521-649,
// accumulate _mean_ap.py:696-857).  The host C++ evaluator (coco_eval.cpp) stays as the CPU path and as the
// oracle the GPU tests compare against.
//
// Pipeline (all on the metric's device; ATen is only used for the stable orderings):
//   1. detections ordered by (image, class, score desc, input row) with two stable sorts; rank within the
//      (image, class) pair; rows past maxDets[-1] stay in the arrays but are never matched (each pair's detection
//      count is clamped to maxDets[-1]) nor accumulated (maxDet clamped likewise) -- no data-dependent compaction,
//      so no host synchronisation.  Ground truth ordered by (image, class, input row).  The (image, class) pairs are
//      the dense grid image * K + class (no unique() and its host read) unless an IoU export needs sizes anyway.
//   2. coco_match_kernel: one wave per (image, class) pair.  Lane l owns one (IoU threshold t, area range a)
//      combination (l = t * A + a, so T * A <= 64) and runs the sequential greedy match of that combination:
//      non-ignored ground truth first, crowd boxes re-matchable, ties resolved to the later ground truth exactly
//      as pycocotools does.  Detections are visited in lock-step, so each detection's per-combination results
//      are two wave ballots: a 64-bit "matched" mask and a 64-bit "ignored" mask.  Per-lane "gt already matched"
//      bitsets live in LDS.  Non-ignored ground-truth counts per (class, area) are integer atomics.
//   3. detections re-ordered by (class, score desc, image, rank) - the order pycocotools' stable mergesort of the
//      per-image concatenation produces - with stable sorts.
//   4. coco_accumulate_kernel: one wave per (class, area, maxDet, IoU threshold).  A forward ballot pass counts
//      TP / FP / kept detections; a backward pass rebuilds each prefix count from the totals, forms the
//      precision, keeps the running precision envelope (suffix max) in a wave scan, and answers every recall
//      threshold at the detection where the prefix TP first reaches ceil(thr * npig) - the same element
//      np.searchsorted(rc, thr, side="left") finds, computed with the same double arithmetic.
//
// Per-image route (bbox IoU, fp32-exact scores, <= 256 detections and ground truths per image: the module's default
// for COCO-style data, tmx::coco_evaluate_gpu_img): steps 1-2 run as one workgroup per image (coco_image_match_kernel:
// rows staged in LDS, ordered and ranked by 64-bit keys, class runs matched by the image's waves), non-ignored
// ground-truth counts come from an LDS-aggregated kernel, and step 3 sorts the detection rows directly.
//
// Limits of the GPU path (the caller falls back to the C++ evaluator beyond them): T * A <= 64,
// <= 1024 ground-truth boxes per (image, class) pair (a device flag, output 5, read with the caller's results),
// <= 256 recall thresholds.
#include "common.h"

#include <algorithm>
#include <climits>
#include <limits>

namespace tmx {

constexpr int kCocoMaxGt = 1024;               // per (image, class) pair
constexpr int kCocoGtWords = kCocoMaxGt / 32;  // matched bitset words per lane
constexpr int kCocoMaxRec = 256;
constexpr int kCocoMatchWaves = 2;             // waves per block in the match kernel
constexpr int kAccBatch = 8;                   // 64-row chunks in flight per accumulate wave

__device__ __forceinline__ double coco_box_iou(const double* d, const double* g, bool crowd) {
  const double ow = fmin(d[0] + d[2], g[0] + g[2]) - fmax(d[0], g[0]);
  if (ow <= 0) return 0.0;
  const double oh = fmin(d[1] + d[3], g[1] + g[3]) - fmax(d[1], g[1]);
  if (oh <= 0) return 0.0;
  const double inter = ow * oh;
  const double u = crowd ? d[2] * d[3] : d[2] * d[3] + g[2] * g[3] - inter;
  return u > 0 ? inter / u : 0.0;
}

struct CocoPairs {
  const int64_t* det_start;  // [P] first row of the pair in the sorted detection arrays
  const int64_t* det_count;  // [P] (<= maxDets[-1])
  const int64_t* gt_start;   // [P]
  const int64_t* gt_count;   // [P]
  const int64_t* cls;        // [P] class index
  const int64_t* img;        // [P] image index
  const int64_t* iou_off;    // [P] offset of the pair's [nd, ng] block in the exported IoU buffer
};

// custom (segmentation) IoU: per-image [n_det_img, n_gt_img] matrices
struct CocoCustomIoU {
  const double* mats;       // concatenated matrices
  const int64_t* img_off;   // [I] offset of the image's matrix
  const int64_t* img_ng;    // [I] ground-truth count of the image (matrix width)
  const int64_t* det_local; // [sorted dets] row of the detection within its image
  const int64_t* gt_local;  // [sorted gts] row of the ground truth within its image
};

__global__ __launch_bounds__(kCocoMatchWaves * kWave) void coco_match_kernel(
    CocoPairs pairs, int64_t P, const double* __restrict__ dbox, const double* __restrict__ darea,
    const double* __restrict__ gbox, const int64_t* __restrict__ gcrowd, const double* __restrict__ garea,
    const double* __restrict__ iou_thr, int T, const double* __restrict__ area_rng, int A, bool custom,
    CocoCustomIoU cust, bool export_iou, double* __restrict__ iou_out, uint64_t* __restrict__ matched_out,
    uint64_t* __restrict__ ignored_out, int64_t* __restrict__ npig) {
  __shared__ uint32_t gtm_all[kCocoMatchWaves][kCocoGtWords][kWave];  // [word][lane]: conflict-free per word
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int64_t p = static_cast<int64_t>(blockIdx.x) * kCocoMatchWaves + wave;
  if (p >= P) return;  // whole wave leaves together (p is wave-uniform); no block barriers below
  uint32_t(*gtm)[kWave] = gtm_all[wave];
  const int64_t d0 = pairs.det_start[p], nd = pairs.det_count[p];
  const int64_t g0 = pairs.gt_start[p], ng = pairs.gt_count[p];
  const int64_t k = pairs.cls[p];
  if (ng > kCocoMaxGt) return;  // beyond the LDS bitsets: flagged by the host op (the caller reruns on the host)

  auto iou_of = [&](int64_t d, int64_t g) -> double {
    if (custom) {
      const int64_t im = pairs.img[p];
      return cust.mats[cust.img_off[im] + cust.det_local[d0 + d] * cust.img_ng[im] + cust.gt_local[g0 + g]];
    }
    return coco_box_iou(dbox + 4 * (d0 + d), gbox + 4 * (g0 + g), gcrowd[g0 + g] != 0);
  };

  if (export_iou && nd > 0 && ng > 0) {
    const int64_t off = pairs.iou_off[p];
    for (int64_t idx = lane; idx < nd * ng; idx += kWave) iou_out[off + idx] = iou_of(idx / ng, idx % ng);
  }

  const bool active = lane < T * A;
  const int t = active ? lane / A : 0, a = active ? lane % A : 0;
  const double lo = area_rng[2 * a], hi = area_rng[2 * a + 1];
  const double thr = fmin(iou_thr[t], 1.0 - 1e-10);
  const int words = static_cast<int>((ng + 31) / 32);
  for (int w = 0; w < words; ++w) gtm[w][lane] = 0u;

  auto gt_ignored = [&](int64_t g) -> bool {
    const double ar = garea[g0 + g];
    return gcrowd[g0 + g] != 0 || ar < lo || ar > hi;
  };

  if (active && t == 0) {
    int64_t c = 0;
    for (int64_t g = 0; g < ng; ++g) c += gt_ignored(g) ? 0 : 1;
    if (c) atomic_add_i64(npig + k * A + a, c);
  }

  for (int64_t d = 0; d < nd; ++d) {  // wave-uniform trip count
    int64_t m = -1;
    bool m_ig = false;
    if (active && ng > 0) {
      double best = thr;
      // pass 0: non-ignored ground truth in input order; pass 1: ignored ones (only if nothing matched yet,
      // the reference's "break once a non-ignored match exists and the ignored block starts")
      for (int pass = 0; pass < 2 && !(pass == 1 && m >= 0); ++pass) {
        for (int64_t g = 0; g < ng; ++g) {
          const bool ig = gt_ignored(g);
          if (ig != (pass == 1)) continue;
          const bool crowd = gcrowd[g0 + g] != 0;
          if (!crowd && ((gtm[g >> 5][lane] >> (g & 31)) & 1u)) continue;
          const double v = iou_of(d, g);
          if (v < best) continue;
          best = v;
          m = g;
          m_ig = ig;
        }
      }
      if (m >= 0) gtm[m >> 5][lane] |= 1u << (m & 31);
    }
    bool ign = m >= 0 ? m_ig : false;
    if (active && m < 0) {
      const double ar = darea[d0 + d];
      ign = ar < lo || ar > hi;
    }
    const uint64_t mb = __ballot(active && m >= 0);
    const uint64_t ib = __ballot(active && ign);
    if (lane == 0) {
      matched_out[d0 + d] = mb;
      ignored_out[d0 + d] = ib;
    }
  }
}

// One wave per (class k, area a, maxDet m, IoU threshold t).  Arrays are in accumulate order: class segments,
// score descending, ties by (image, rank).  Outputs were pre-filled with -1 by the host.
//
// One forward pass.  pycocotools' interpolated precision at recall threshold r is the suffix maximum of the
// precision curve from the element where the TP count first reaches ctab[r].  That element is a TP, and a suffix that
// starts at a TP has its maximum at a TP (precision falls over false positives and stays flat over ignored rows), so
// only TP precisions matter: the n-th TP's precision goes to bucket b with ctab[b] <= n < ctab[b + 1] (an LDS
// atomicMax on the non-negative double's bits), and p[r] is the maximum of buckets >= r.  No backward pass and no
// per-chunk scan; the division runs only in chunks holding a TP.  Same double arithmetic, so the same values.
// The kernel takes any number of waves per workgroup (acc_wpb: the T waves of one (class, area, maxDet) share a
// workgroup when > 1); dynamic LDS: ctab [R] int64 (shared), then per wave bucket maxima [R] and scores [R].
__global__ __launch_bounds__(1024) void coco_accumulate_kernel(
    const int64_t* __restrict__ seg, int K, int A, int M, int T, int R, const int64_t* __restrict__ max_dets,
    const double* __restrict__ rec_thr, const int32_t* __restrict__ rank, const uint64_t* __restrict__ matched,
    const uint64_t* __restrict__ ignored, const double* __restrict__ score, const int64_t* __restrict__ npig_all,
    double* __restrict__ prec_out, double* __restrict__ rec_out, double* __restrict__ score_out) {
  extern __shared__ int64_t acc_lds[];
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave, wpb = blockDim.x / kWave;
  int64_t* ctab = acc_lds;
  unsigned long long* bmax = reinterpret_cast<unsigned long long*>(acc_lds + R * (1 + 2 * wave));  // (>= +0.0 bits)
  double* s_res = reinterpret_cast<double*>(acc_lds + R * (2 + 2 * wave));
  int64_t q = static_cast<int64_t>(blockIdx.x) * wpb + wave;
  const int t = static_cast<int>(q % T); q /= T;
  const int m = static_cast<int>(q % M); q /= M;
  const int a = static_cast<int>(q % A); q /= A;
  const int k = static_cast<int>(q);
  const int64_t npig = npig_all[k * A + a];
  if (npig == 0) {  // no ground truth for this class / area: -1 everywhere ((k, a) is workgroup-uniform)
    for (int r = lane; r < R; r += kWave) {
      const int64_t idx = (((static_cast<int64_t>(t) * R + r) * K + k) * A + a) * M + m;
      prec_out[idx] = -1.0;
      score_out[idx] = -1.0;
    }
    if (lane == 0) rec_out[((static_cast<int64_t>(t) * K + k) * A + a) * M + m] = -1.0;
    return;
  }
  const int64_t s = seg[k], e = seg[k + 1];
  const int bit = t * A + a;
  const int64_t maxd = max_dets[m];
  const double eps = 2.220446049250313e-16;  // np.spacing(1)

  for (int r = lane; r < R; r += kWave) {
    bmax[r] = 0ull;
    s_res[r] = 0.0;
  }
  // smallest TP count whose recall reaches each threshold (same double arithmetic as rc = tp / npig)
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const double thr = rec_thr[r];
    int64_t c = 0;
    if (thr > 0) {
      double cf = ceil(thr * static_cast<double>(npig));
      c = cf < 0 ? 0 : static_cast<int64_t>(cf);
      while (c > 0 && static_cast<double>(c - 1) / static_cast<double>(npig) >= thr) --c;
      while (static_cast<double>(c) / static_cast<double>(npig) < thr) ++c;
      if (c == 0) c = 1;  // thr > 0 needs at least one true positive
    }
    ctab[r] = c;
  }
  __syncthreads();

  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= this one
  // 32-bit counts (a class segment holds < 2^31 rows: checked by the host) -- the TP branch is the kernel's VALU bill:
  // int64 -> double conversions and an int64 division for the bucket guess cost dozens of instructions each
  const int maxd32 = static_cast<int>(min(maxd, static_cast<int64_t>(INT_MAX)));
  const double guess_scale = static_cast<double>(R - 1) / static_cast<double>(npig);
  int nd = 0, tp_run = 0, fp_run = 0;
  int64_t first = -1;
  for (int64_t base = s; base < e; base += kAccBatch * kWave) {
    bool in[kAccBatch];
    int32_t rk[kAccBatch];
    uint64_t mt[kAccBatch], ig[kAccBatch];
#pragma unroll
    for (int u = 0; u < kAccBatch; ++u) {
      const int64_t j = base + u * kWave + lane;
      in[u] = j < e;
      rk[u] = in[u] ? rank[j] : 0;
      mt[u] = in[u] ? matched[j] : 0ull;
      ig[u] = in[u] ? ignored[j] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kAccBatch; ++u) {
      const bool valid = in[u] && rk[u] < maxd32;
      const bool m1 = (mt[u] >> bit) & 1ull, i1 = (ig[u] >> bit) & 1ull;
      const bool tp = valid && m1 && !i1;
      const uint64_t vb = __ballot(valid), tb = __ballot(tp), fb = __ballot(valid && !m1 && !i1);
      if (first < 0 && vb) first = base + u * kWave + __builtin_ctzll(vb);
      nd += __builtin_popcountll(vb);
      if (tb) {  // (wave-uniform) this chunk holds TPs: their precisions, bucketed by TP count
        if (tp) {
          const int tp_sum = tp_run + __builtin_popcountll(tb & upto);
          const int fp_sum = fp_run + __builtin_popcountll(fb & upto);
          const double tpd = static_cast<double>(tp_sum);
          const double prec = tpd / (static_cast<double>(fp_sum) + tpd + eps);
          // upper_bound(ctab, tp_sum): start where evenly spaced thresholds would put it, then walk (a step or
          // two for the usual linspace; a dependent binary search was the kernel's longest latency chain)
          int lo_r = min(R, static_cast<int>(tpd * guess_scale) + 1);
          while (lo_r < R && ctab[lo_r] <= tp_sum) ++lo_r;
          while (lo_r > 0 && ctab[lo_r - 1] > tp_sum) --lo_r;
          if (lo_r > 0) {
            atomicMax(&bmax[lo_r - 1], static_cast<unsigned long long>(__double_as_longlong(prec)));
            // thresholds whose count is exactly this TP's are answered here: their score
            for (int r = lo_r - 1; r >= 0 && ctab[r] == tp_sum; --r) s_res[r] = score[base + u * kWave + lane];
          }
        }
      }
      tp_run += __builtin_popcountll(tb);
      fp_run += __builtin_popcountll(fb);
    }
  }
  const int64_t rec_idx = ((static_cast<int64_t>(t) * K + k) * A + a) * M + m;
  if (lane == 0) rec_out[rec_idx] = nd ? static_cast<double>(tp_run) / static_cast<double>(npig) : 0.0;
  __syncthreads();
  if (lane == 0) {  // suffix maxima over the buckets; thresholds of count 0 are answered at the first kept row
    double carry = 0.0;
    for (int r = R - 1; r >= 0; --r) {
      carry = fmax(carry, __longlong_as_double(static_cast<long long>(bmax[r])));
      const int64_t c = ctab[r];
      const bool answered = c == 0 ? first >= 0 : c <= tp_run;
      bmax[r] = static_cast<unsigned long long>(__double_as_longlong(answered ? carry : 0.0));
      if (c == 0 && first >= 0) s_res[r] = score[first];
    }
  }
  __syncthreads();
  for (int r = lane; r < R; r += kWave) {
    const int64_t idx = (((static_cast<int64_t>(t) * R + r) * K + k) * A + a) * M + m;
    prec_out[idx] = __longlong_as_double(static_cast<long long>(bmax[r]));
    score_out[idx] = s_res[r];
  }
}

// ---- per-image route (bbox IoU, fp32-exact scores, <= kImgMaxRows detections and ground truths per image) -------
// One workgroup per image replaces step 1's two global sorts, the five searchsorted lookups over the dense
// (image, class) grid, six row gathers and the wave-per-pair match launch (204,800 mostly empty waves at 2560 images
// x 80 classes): the image's rows are staged in LDS once (boxes, areas, crowd flags: the greedy match then never waits
// on a dependent global load), its detections ranked by (class, score desc, row) with an all-pairs count (the order
// the two stable sorts produce), its ground truths by (class, row), and each wave then runs the greedy match of the
// classes it is dealt (one class run per turn, lane = (IoU threshold, area range) as in coco_match_kernel).
// Outputs are per detection row (rank within its (image, class) pair, matched / ignored masks), so step 3 sorts the
// rows directly: a stable sort by (class, score desc) over rows in input order ties on (image, rank) exactly as the
// sorted-order arrays did.  The rank pass also writes one descriptor per class run (sorted start, length, ground-truth
// range), so a wave's turn starts matching at once.  LDS: ~33 KB (four workgroups per CU).
constexpr int kImgThreads = 256;
constexpr int kImgWaves = kImgThreads / kWave;
constexpr int kImgMaxRows = 256;  // detections and ground truths of one image (so <= kCocoMaxGt per pair)
constexpr int kImgGtWords = kImgMaxRows / 32;

__device__ __forceinline__ uint32_t coco_score_okey(float f) {  // fp32 bits -> ascending uint32 (see coco_key_kernel)
  const uint32_t u = f != f ? 0x7FC00000u : (f == 0.f ? 0u : __float_as_uint(f));
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(kImgThreads) void coco_image_match_kernel(
    const int64_t* __restrict__ det_off, const int64_t* __restrict__ gt_off, const double* __restrict__ dbox,
    const float* __restrict__ dscore, const int64_t* __restrict__ dcls, const double* __restrict__ gbox,
    const int64_t* __restrict__ gcls, const int64_t* __restrict__ gcrowd, const double* __restrict__ garea,
    const double* __restrict__ iou_thr, int T, const double* __restrict__ area_rng,
    int A, int64_t max_det_last, int32_t* __restrict__ rank_out, uint64_t* __restrict__ matched_out,
    uint64_t* __restrict__ ignored_out, int64_t* __restrict__ overflow, int probe) {
  __shared__ uint64_t s_dkey[kImgMaxRows];  // class << 32 | ~score key: ascending = (class, score desc)
  __shared__ int16_t s_dord[kImgMaxRows];  // image-local detection at each (class, score desc, row) position
  __shared__ int32_t s_gcls[kImgMaxRows];
  __shared__ int16_t s_gord[kImgMaxRows];  // image-local ground truth at each (class, row) position
  __shared__ double4 s_dbox[kImgMaxRows];  // image rows in input order
  __shared__ double s_darea[kImgMaxRows];
  __shared__ double4 s_gbox[kImgMaxRows];
  __shared__ double s_garea[kImgMaxRows];
  __shared__ uint8_t s_gcrowd[kImgMaxRows];
  __shared__ uint32_t s_gtm[kImgWaves][kImgGtWords][kWave];
  __shared__ int4 s_run[kImgMaxRows];  // (sorted start, detections, first sorted ground truth, ground truths)
  __shared__ int s_nrun;
  const int img = blockIdx.x;
  const int64_t d0 = det_off[img], g0 = gt_off[img];
  const int nd = static_cast<int>(det_off[img + 1] - d0), ng = static_cast<int>(gt_off[img + 1] - g0);
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  if (nd == 0 && ng == 0) return;  // (block-uniform)
  if (nd > kImgMaxRows || ng > kImgMaxRows) {  // past the LDS tables: flagged, the caller reruns elsewhere
    if (tid == 0) overflow[0] = 1;
    return;
  }
  if (tid == 0) s_nrun = 0;
  for (int i = tid; i < nd; i += kImgThreads) {
    s_dkey[i] = (static_cast<uint64_t>(dcls[d0 + i]) << 32) | static_cast<uint64_t>(~coco_score_okey(dscore[d0 + i]));
    const double* b = dbox + 4 * (d0 + i);
    s_dbox[i] = make_double4(b[0], b[1], b[2], b[3]);
    s_darea[i] = b[2] * b[3];  // (bbox route: the detection's area is its box area)
  }
  for (int i = tid; i < ng; i += kImgThreads) {
    s_gcls[i] = static_cast<int32_t>(gcls[g0 + i]);
    const double* b = gbox + 4 * (g0 + i);
    s_gbox[i] = make_double4(b[0], b[1], b[2], b[3]);
    const double ga = garea[g0 + i];
    s_garea[i] = ga > 0 ? ga : b[2] * b[3];  // supplied area, else the box's
    s_gcrowd[i] = gcrowd[g0 + i] != 0;
  }
  __syncthreads();
  // position of each detection in (class, score desc, row) order: one 64-bit key per row (class above the inverted
  // score key), an all-pairs count with one LDS broadcast read per pair
  for (int i = tid; i < nd && !(probe & 2); i += kImgThreads) {
    const uint64_t ki = s_dkey[i];
    int pos = 0;
    for (int j = 0; j < nd; ++j) {
      const uint64_t kj = s_dkey[j];
      pos += kj < ki || (kj == ki && j < i);
    }
    s_dord[pos] = static_cast<int16_t>(i);
  }
  for (int g = tid; g < ng; g += kImgThreads) {
    const int cg = s_gcls[g];
    int pos = 0;
    for (int h = 0; h < ng; ++h) {
      const int ch = s_gcls[h];
      pos += ch < cg || (ch == cg && h < g);
    }
    s_gord[pos] = static_cast<int16_t>(g);
  }
  __syncthreads();
  // rank within the (image, class) pair = distance to the class run's head; heads write the run descriptors
  for (int p = tid; p < nd && !(probe & 2); p += kImgThreads) {
    const int i = s_dord[p];
    const uint32_t c = static_cast<uint32_t>(s_dkey[i] >> 32);
    int head = p;
    while (head > 0 && static_cast<uint32_t>(s_dkey[s_dord[head - 1]] >> 32) == c) --head;
    const int rk = p - head;
    if (rk == 0) {
      int cnt = 1;
      while (p + cnt < nd && static_cast<uint32_t>(s_dkey[s_dord[p + cnt]] >> 32) == c) ++cnt;
      int gb = 0, gc = 0;
      for (int h = 0; h < ng; ++h) {
        const uint32_t ch = static_cast<uint32_t>(s_gcls[h]);
        gb += ch < c;
        gc += ch == c;
      }
      s_run[atomicAdd(&s_nrun, 1)] = make_int4(p, cnt, gb, gc);
    }
    rank_out[d0 + i] = rk;
    if (rk >= max_det_last) {  // past maxDets[-1] in its pair: never matched nor accumulated
      matched_out[d0 + i] = 0ull;
      ignored_out[d0 + i] = 0ull;
    }
  }
  __syncthreads();

  const bool active = lane < T * A;
  const int t = active ? lane / A : 0, a = active ? lane % A : 0;
  const double lo = area_rng[2 * a], hi = area_rng[2 * a + 1];
  const double thr = fmin(iou_thr[t], 1.0 - 1e-10);
  uint32_t(*gtm)[kWave] = s_gtm[wave];
  auto match_run = [&](int4 rd) {  // wave-uniform: the detections of one class run
    const int ps = rd.x, gs = rd.z, ngc = rd.w;
    const int nm = static_cast<int>(min(static_cast<int64_t>(rd.y), max_det_last));
    const int words = (ngc + 31) / 32;
    for (int w = 0; w < words; ++w) gtm[w][lane] = 0u;
    for (int d = 0; d < nm; ++d) {
      const int di = s_dord[ps + d];
      const double4 db4 = s_dbox[di];
      const double db[4] = {db4.x, db4.y, db4.z, db4.w};
      int m = -1;
      bool m_ig = false;
      if (active && ngc > 0) {
        double best = thr;
        for (int pass = 0; pass < 2 && !(pass == 1 && m >= 0); ++pass) {
          for (int g = 0; g < ngc; ++g) {
            const int gi = s_gord[gs + g];
            const bool crowd = s_gcrowd[gi] != 0;
            const double ar = s_garea[gi];
            const bool ig = crowd || ar < lo || ar > hi;
            if (ig != (pass == 1)) continue;
            if (!crowd && ((gtm[g >> 5][lane] >> (g & 31)) & 1u)) continue;
            const double4 gb4 = s_gbox[gi];
            const double gb[4] = {gb4.x, gb4.y, gb4.z, gb4.w};
            const double v = coco_box_iou(db, gb, crowd);
            if (v < best) continue;
            best = v;
            m = g;
            m_ig = ig;
          }
        }
        if (m >= 0) gtm[m >> 5][lane] |= 1u << (m & 31);
      }
      bool ign = m >= 0 ? m_ig : false;
      if (active && m < 0) {
        const double ar = s_darea[di];
        ign = ar < lo || ar > hi;
      }
      const uint64_t mb = __ballot(active && m >= 0);
      const uint64_t ib = __ballot(active && ign);
      if (lane == 0) {
        matched_out[d0 + di] = mb;
        ignored_out[d0 + di] = ib;
      }
    }
  };
  const int nrun = (probe & 4) ? 0 : s_nrun;
  for (int r = wave; r < nrun; r += kImgWaves) match_run(s_run[r]);
}

// non-ignored ground truth per (class, area): npig[k * A + a].  Each workgroup counts into LDS (K * A <= 8192 bins)
// and flushes its non-zero bins (a global atomic per ground truth serialises on the few hot bins of COCO-80 data)
constexpr int kNpigLdsBins = 8192;

__global__ __launch_bounds__(256) void coco_npig_kernel(const int64_t* __restrict__ gcls, const int64_t* __restrict__ gcrowd,
                                                        const double* __restrict__ garea, const double* __restrict__ gbox, int64_t n,
                                                        const double* __restrict__ area_rng, int A, int bins, bool lds,
                                                        int64_t* __restrict__ npig) {
  extern __shared__ unsigned np_lds[];
  if (lds) {
    for (int b = threadIdx.x; b < bins; b += blockDim.x) np_lds[b] = 0u;
    __syncthreads();
  }
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < n;
       g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (gcrowd[g] != 0) continue;
    const double ga = garea[g];
    const double ar = ga > 0 ? ga : gbox[4 * g + 2] * gbox[4 * g + 3];
    const int64_t base = gcls[g] * A;
    for (int a = 0; a < A; ++a) {
      if (ar < area_rng[2 * a] || ar > area_rng[2 * a + 1]) continue;
      if (lds) atomicAdd(np_lds + base + a, 1u);
      else atomic_add_i64(npig + base + a, 1);
    }
  }
  if (lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < bins; b += blockDim.x)
      if (np_lds[b]) atomic_add_i64(npig + b, static_cast<long long>(np_lds[b]));
  }
}

// step 3's arrays in accumulate order (one launch for the four gathers) and the class segment starts seg[K + 1]
__global__ void coco_acc_gather_kernel(const int64_t* __restrict__ acc, int64_t n, const int64_t* __restrict__ cls, int K,
                                       const int32_t* __restrict__ rank, const uint64_t* __restrict__ matched,
                                       const uint64_t* __restrict__ ignored, const float* __restrict__ score,
                                       int32_t* __restrict__ a_rank, uint64_t* __restrict__ a_matched,
                                       uint64_t* __restrict__ a_ignored, double* __restrict__ a_score, int64_t* __restrict__ seg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = acc[i];
  a_rank[i] = rank[r];
  a_matched[i] = matched[r];
  a_ignored[i] = ignored[r];
  a_score[i] = static_cast<double>(score[r]);
  const int64_t c = cls[r];
  const int64_t cp = i == 0 ? -1 : cls[acc[i - 1]];
  for (int64_t k = cp + 1; k <= c && k <= K; ++k) seg[k] = i;
  if (i == n - 1)
    for (int64_t k = c + 1; k <= K; ++k) seg[k] = n;
}

// ---- class discovery (MeanAveragePrecision._get_classes) --------------------------------------------------------
// Presence bitmap of the labels in [0, 65536) (bit v of word v / 32; word 2048 flags a label outside that range) and
// the present ids compacted in ascending order on the device, so the host reads 8 KiB once and the evaluator's class
// ids are already resident (no torch.unique sort + size read, no upload back).
constexpr int kClassWords = 2048;

// Each workgroup builds its own bitmap in LDS (read before the LDS atomic: labels repeat, and the LDS copy is
// coherent inside the workgroup) and flushes only its non-zero words: one global atomic per (workgroup, word).  A
// global atomic per label serialises at L2 on the few words a COCO-80 label set touches (~0.6 ms for 300K labels).
__global__ __launch_bounds__(256) void class_mark_kernel(const int64_t* __restrict__ lab, int64_t n, uint32_t* __restrict__ bm) {
  __shared__ uint32_t s_bm[kClassWords + 1];
  for (int w = threadIdx.x; w <= kClassWords; w += blockDim.x) s_bm[w] = 0u;
  __syncthreads();
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t v = lab[i];
    const int w = (v >= 0 && v < 32 * kClassWords) ? static_cast<int>(v >> 5) : kClassWords;
    const uint32_t bit = w == kClassWords ? 1u : 1u << (v & 31);
    if (!(s_bm[w] & bit)) atomicOr(s_bm + w, bit);
  }
  __syncthreads();
  for (int w = threadIdx.x; w <= kClassWords; w += blockDim.x)
    if (s_bm[w]) atomicOr(bm + w, s_bm[w]);
}

__global__ __launch_bounds__(1024) void class_compact_kernel(const uint32_t* __restrict__ bm, int64_t* __restrict__ ids) {
  __shared__ int s_wave[1024 / kWave];
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  const uint32_t w0 = bm[2 * tid], w1 = bm[2 * tid + 1];  // 1024 threads x 2 words = kClassWords
  const int cnt = __popc(w0) + __popc(w1);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int o = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += o;
  }
  if (lane == kWave - 1) s_wave[wave] = incl;
  __syncthreads();
  int base = incl - cnt;
  for (int w = 0; w < wave; ++w) base += s_wave[w];
  for (int h = 0; h < 2; ++h) {
    uint32_t x = h ? w1 : w0;
    while (x) {
      const int b = __builtin_ctz(x);
      x &= x - 1;
      ids[base++] = static_cast<int64_t>(32 * (2 * tid + h) + b);
    }
  }
}

// COCO summary tables for MeanAveragePrecision._summarize_tables: per (t, k, a, m) cell the sum and count of the valid
// (> -1) precisions over the recall thresholds, and the recall with its validity -- [4][T][K][A][M] fp64 -- plus the
// evaluator's overflow flag as the last word: one launch and one copy into pinned memory instead of ~10 ATen ops.
__global__ void coco_summary_kernel(const double* __restrict__ prec, const double* __restrict__ rec, int64_t T, int64_t kam,
                                    int R, const int64_t* __restrict__ overflow, double* __restrict__ out) {
  const int64_t cells = T * kam;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c == 0) out[4 * cells] = overflow != nullptr ? static_cast<double>(overflow[0]) : 0.0;
  if (c >= cells) return;
  const int64_t t = c / kam, j = c % kam;
  double s = 0.0, n = 0.0;
  for (int r = 0; r < R; ++r) {
    const double p = prec[(t * R + r) * kam + j];
    if (p > -1) {
      s += p;
      n += 1.0;
    }
  }
  const double rv = rec[c];
  out[c] = s;
  out[cells + c] = n;
  out[2 * cells + c] = rv > -1 ? rv : 0.0;
  out[3 * cells + c] = rv > -1 ? 1.0 : 0.0;
}

// ------------------------------------------------------------------------------------------------ host side
namespace {

// waves per accumulate workgroup: one.  T waves of one (class, area, maxDet) per workgroup (sharing the rows through
// L1) measured slower: 216 vs 131 us for COCO-80 x 2560 images (gpurun r7g vs r7f)
int acc_wpb(int64_t /*T*/) { return 1; }
size_t acc_lds_bytes(int64_t T, int64_t R) {
  const size_t bytes = sizeof(int64_t) * static_cast<size_t>(R * (1 + 2 * acc_wpb(T)));
  if (bytes > 65536)  // (up to 67.5 KB at R = 256, T = 16)
    TMX_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&coco_accumulate_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes)));
  return bytes;
}

at::Tensor stable_order(const at::Tensor& key, bool descending) {
  return std::get<1>(at::sort(key, /*stable=*/true, /*dim=*/0, descending));
}

}  // namespace

// (major ascending, fp32 score descending) as ONE int64 key: major << 32 | ~orderkey(score), where orderkey maps fp32
// bits to an ascending uint32 (negatives bit-flipped, positives with the sign bit set).  One stable radix sort on it is
// the reference's stable mergesort by score followed by the stable sort by major -- two merge sorts on doubles before.
__global__ void coco_key_kernel(const int64_t* __restrict__ major, const float* __restrict__ score, int64_t n, int64_t* __restrict__ key) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // -0 sorts with +0 and every NaN with the positive quiet NaN (torch's sort: NaN above +inf), as the double sort did
  const uint32_t k = coco_score_okey(score[i]);
  key[i] = static_cast<int64_t>((static_cast<uint64_t>(major[i]) << 32) | static_cast<uint64_t>(~k));
}

namespace {

// stable order by (major asc, score desc); scores exactly representable in fp32 (fp32 / fp16 / bf16 inputs)
at::Tensor major_score_order(const at::Tensor& major, const at::Tensor& score32) {
  const int64_t n = major.numel();
  auto key = at::empty({n}, major.options());
  if (n > 0) {
    const auto mj = major.contiguous();
    const auto sc = score32.contiguous();
    hipLaunchKernelGGL(coco_key_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), 256, 0, stream(), mj.data_ptr<int64_t>(),
                       sc.data_ptr<float>(), n, key.data_ptr<int64_t>());
    TMX_LAUNCH_CHECK();
  }
  return stable_order(key, false);
}

}  // namespace

// Same contract as the host op tmx::coco_evaluate (coco_eval.cpp), except that class labels come in already
// mapped to class indices (det_cls / gt_cls in [0, K)), every tensor lives on the GPU, and iou_index lists only
// the (image, class) pairs that hold a detection or a ground truth.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> coco_evaluate_gpu(
    const at::Tensor& det_boxes_, const at::Tensor& det_scores_, const at::Tensor& det_cls_, const at::Tensor& det_img_,
    const at::Tensor& det_area_, const at::Tensor& gt_boxes_, const at::Tensor& gt_cls_, const at::Tensor& gt_img_,
    const at::Tensor& gt_crowd_, const at::Tensor& gt_area_, int64_t K, int64_t num_images, const at::Tensor& iou_thrs_,
    const at::Tensor& rec_thrs_, const at::Tensor& max_dets_, const at::Tensor& area_rng_,
    const c10::optional<at::Tensor>& img_iou_, const c10::optional<at::Tensor>& img_iou_offsets_,
    const c10::optional<at::Tensor>& det_local_, const c10::optional<at::Tensor>& gt_local_,
    const c10::optional<at::Tensor>& img_ng_, bool export_iou) {
  TORCH_CHECK(det_scores_.is_cuda(), "coco_evaluate_gpu: expected GPU tensors");
  const c10::DeviceGuard guard(det_scores_.device());
  const auto dev = det_scores_.device();
  auto f64 = [&](const at::Tensor& t) { return t.to(dev, at::kDouble).contiguous(); };
  auto i64 = [&](const at::Tensor& t) { return t.to(dev, at::kLong).contiguous(); };
  const auto det_boxes = f64(det_boxes_).reshape({-1, 4}), det_scores = f64(det_scores_), det_area = f64(det_area_);
  const auto gt_boxes = f64(gt_boxes_).reshape({-1, 4}), gt_area = f64(gt_area_);
  const auto det_cls = i64(det_cls_), det_img = i64(det_img_), gt_cls = i64(gt_cls_), gt_img = i64(gt_img_);
  const auto gt_crowd = i64(gt_crowd_);
  const auto iou_thrs = f64(iou_thrs_), rec_thrs = f64(rec_thrs_), area_rng = f64(area_rng_).reshape({-1, 2});
  const auto max_dets_cpu = max_dets_.to(at::kCPU, at::kLong).contiguous();
  const int64_t T = iou_thrs.numel(), R = rec_thrs.numel(), M = max_dets_cpu.numel(), A = area_rng.size(0);
  TORCH_CHECK(T > 0 && R > 0 && M > 0 && A > 0, "coco_evaluate_gpu: empty parameter list");
  TORCH_CHECK(T * A <= 64, "coco_evaluate_gpu: at most 64 (IoU threshold, area range) combinations");
  TORCH_CHECK(R <= kCocoMaxRec, "coco_evaluate_gpu: at most ", kCocoMaxRec, " recall thresholds");
  const int64_t max_det_last = max_dets_cpu.data_ptr<int64_t>()[M - 1];
  // pycocotools truncates each (image, class) list at maxDets[-1] before accumulating every maxDet
  const auto max_dets = max_dets_cpu.clamp_max(max_det_last).to(dev);
  const bool custom = img_iou_.has_value() && img_iou_->defined();

  // every entry is written by the accumulate kernel (-1 where a class / area has no ground truth)
  auto precision = at::empty({T, R, K, A, M}, det_scores.options());
  auto recall = at::empty({T, K, A, M}, det_scores.options());
  auto scores_out = at::empty({T, R, K, A, M}, det_scores.options());
  auto lopt = det_cls.options();
  auto overflow = at::zeros({1}, lopt);
  if (K == 0) return {precision, recall, scores_out, at::zeros({0}, det_scores.options()), at::zeros({0, 5}, lopt), overflow};

  // ---- 1. orderings ------------------------------------------------------------------------------------
  const auto det_pair = det_img * K + det_cls;
  // fp32-exact scores (fp32 / fp16 / bf16 inputs; pair index < 2^31): one radix sort on a composite key
  const bool key32 = (det_scores_.scalar_type() == at::kFloat || det_scores_.scalar_type() == at::kHalf ||
                      det_scores_.scalar_type() == at::kBFloat16) && num_images * K < (int64_t(1) << 31);
  const auto det_score32 = key32 ? det_scores_.to(dev, at::kFloat).contiguous() : at::Tensor();
  at::Tensor order;
  if (key32) {
    order = major_score_order(det_pair, det_score32);
  } else {
    order = stable_order(det_scores, /*descending=*/true);
    order = order.index_select(0, stable_order(det_pair.index_select(0, order), false));
  }
  const auto det_pair_sorted = det_pair.index_select(0, order);
  const auto first_of_pair = at::searchsorted(det_pair_sorted, det_pair_sorted, /*out_int32=*/false, /*right=*/false);
  const auto d_rank = (at::arange(det_pair_sorted.numel(), lopt) - first_of_pair).to(at::kInt);
  const auto& dsel = order;  // every detection in (image, class, rank) order
  const auto& d_pair = det_pair_sorted;
  const auto gorder = stable_order(gt_img * K + gt_cls, false);
  const auto g_pair = (gt_img * K + gt_cls).index_select(0, gorder);

  // pairs: the dense (image, class) grid -- its size is known on the host -- unless an IoU export (which needs its
  // total size on the host anyway) or a very large grid asks for the occupied pairs only
  const bool dense = !export_iou && num_images * K <= (int64_t(1) << 22);
  const auto pair_keys = dense ? at::arange(num_images * K, lopt) : std::get<0>(at::_unique(at::cat({d_pair, g_pair}), /*sorted=*/true));
  const int64_t P = pair_keys.numel();
  const auto det_start = at::searchsorted(d_pair, pair_keys, false, false);
  const auto det_count = (at::searchsorted(d_pair, pair_keys, false, true) - det_start).clamp_max(max_det_last);
  const auto gt_start = at::searchsorted(g_pair, pair_keys, false, false);
  const auto gt_count = at::searchsorted(g_pair, pair_keys, false, true) - gt_start;
  const auto pair_cls = pair_keys.remainder(K);
  const auto pair_img = pair_keys.div(K, "floor");
  const auto pair_cells = det_count * gt_count;
  const auto iou_off = pair_cells.cumsum(0) - pair_cells;
  if (P > 0) overflow = (gt_count.max() > kCocoMaxGt).to(at::kLong).reshape({1});
  int64_t total_cells = 0;
  if (export_iou && P > 0) {  // one host read: the export size and the per-pair ground-truth limit
    const auto host = at::stack({pair_cells.sum(), gt_count.max()}).cpu();
    total_cells = host.data_ptr<int64_t>()[0];
    TORCH_CHECK(host.data_ptr<int64_t>()[1] <= kCocoMaxGt, "coco_evaluate_gpu: more than ", kCocoMaxGt,
                " ground-truth boxes of one class in one image");
  }

  const auto sd_box = det_boxes.index_select(0, dsel).contiguous();
  const auto sd_area = det_area.index_select(0, dsel).contiguous();
  const auto sd_score = det_scores.index_select(0, dsel).contiguous();
  const auto sg_box = gt_boxes.index_select(0, gorder).contiguous();
  const auto sg_crowd = gt_crowd.index_select(0, gorder).contiguous();
  const auto sg_area = gt_area.index_select(0, gorder).contiguous();
  at::Tensor mats, img_off, img_ng, det_local, gt_local;
  CocoCustomIoU cust{nullptr, nullptr, nullptr, nullptr, nullptr};
  if (custom) {
    mats = f64(*img_iou_);
    img_off = i64(*img_iou_offsets_);
    img_ng = i64(*img_ng_);
    det_local = i64(*det_local_).index_select(0, dsel).contiguous();
    gt_local = i64(*gt_local_).index_select(0, gorder).contiguous();
    cust = {mats.data_ptr<double>(), img_off.data_ptr<int64_t>(), img_ng.data_ptr<int64_t>(), det_local.data_ptr<int64_t>(),
            gt_local.data_ptr<int64_t>()};
  }

  // ---- 2. matching -------------------------------------------------------------------------------------
  const int64_t Nk = dsel.numel();
  auto matched = at::zeros({Nk}, lopt);
  auto ignored = at::zeros({Nk}, lopt);
  auto npig = at::zeros({K * A}, lopt);
  auto iou_values = at::empty({export_iou ? total_cells : 0}, det_scores.options());
  if (P > 0) {
    CocoPairs pairs{det_start.data_ptr<int64_t>(), det_count.data_ptr<int64_t>(), gt_start.data_ptr<int64_t>(),
                    gt_count.data_ptr<int64_t>(), pair_cls.data_ptr<int64_t>(), pair_img.data_ptr<int64_t>(),
                    iou_off.data_ptr<int64_t>()};
    const int blocks = static_cast<int>((P + kCocoMatchWaves - 1) / kCocoMatchWaves);
    coco_match_kernel<<<blocks, kCocoMatchWaves * kWave, 0, stream()>>>(
        pairs, P, sd_box.data_ptr<double>(), sd_area.data_ptr<double>(), sg_box.data_ptr<double>(),
        sg_crowd.data_ptr<int64_t>(), sg_area.data_ptr<double>(), iou_thrs.data_ptr<double>(), static_cast<int>(T),
        area_rng.data_ptr<double>(), static_cast<int>(A), custom, cust, export_iou,
        export_iou ? iou_values.data_ptr<double>() : nullptr, reinterpret_cast<uint64_t*>(matched.data_ptr<int64_t>()),
        reinterpret_cast<uint64_t*>(ignored.data_ptr<int64_t>()), npig.data_ptr<int64_t>());
    TMX_LAUNCH_CHECK();
  }

  // ---- 3. accumulate order: (class, score desc, image, rank) ------------------------------------------
  const auto d_cls = d_pair.remainder(K);
  at::Tensor acc;
  if (key32) {
    acc = major_score_order(d_cls, det_score32.index_select(0, dsel));
  } else {
    acc = stable_order(sd_score, true);
    acc = acc.index_select(0, stable_order(d_cls.index_select(0, acc), false));
  }
  const auto a_rank = d_rank.index_select(0, acc).contiguous();
  const auto a_matched = matched.index_select(0, acc).contiguous();
  const auto a_ignored = ignored.index_select(0, acc).contiguous();
  const auto a_score = sd_score.index_select(0, acc).contiguous();
  const auto seg = at::searchsorted(d_cls.index_select(0, acc).contiguous(), at::arange(K + 1, lopt), false, false);

  // ---- 4. accumulate -----------------------------------------------------------------------------------
  TORCH_CHECK(det_scores.numel() < (int64_t(1) << 31), "COCO evaluator: at most 2^31 - 1 detections");
  const int64_t combos = K * A * M * T;
  coco_accumulate_kernel<<<static_cast<unsigned>(combos / acc_wpb(T)), acc_wpb(T) * kWave, acc_lds_bytes(T, R), stream()>>>(
      seg.data_ptr<int64_t>(), static_cast<int>(K), static_cast<int>(A), static_cast<int>(M), static_cast<int>(T),
      static_cast<int>(R), max_dets.data_ptr<int64_t>(), rec_thrs.data_ptr<double>(), a_rank.data_ptr<int32_t>(),
      reinterpret_cast<const uint64_t*>(a_matched.data_ptr<int64_t>()),
      reinterpret_cast<const uint64_t*>(a_ignored.data_ptr<int64_t>()), a_score.data_ptr<double>(),
      npig.data_ptr<int64_t>(), precision.data_ptr<double>(), recall.data_ptr<double>(), scores_out.data_ptr<double>());
  TMX_LAUNCH_CHECK();

  auto iou_index = at::stack({pair_img, pair_cls, det_count, gt_count, iou_off}, 1);
  return {precision, recall, scores_out, iou_values, iou_index, overflow};
}

// precision [T, R, K, A, M], recall [T, K, A, M] (fp64, device) -> host (pinned) fp64 [4 T K A M + 1]: the summary
// tables, then the overflow flag (0 without one); synchronises the stream (the caller reads the result at once)
at::Tensor coco_summary_tables(const at::Tensor& precision, const at::Tensor& recall, const c10::optional<at::Tensor>& overflow) {
  TORCH_CHECK(precision.is_cuda() && precision.dim() == 5 && recall.dim() == 4, "coco_summary_tables: expected GPU [T,R,K,A,M] / [T,K,A,M]");
  const c10::DeviceGuard guard(precision.device());
  const auto p = precision.to(at::kDouble).contiguous(), r = recall.to(at::kDouble).contiguous();
  const int64_t T = p.size(0), R = p.size(1), kam = p.size(2) * p.size(3) * p.size(4);
  TORCH_CHECK(r.numel() == T * kam, "coco_summary_tables: recall does not match precision");
  const int64_t cells = T * kam;
  auto dev_out = at::empty({4 * cells + 1}, p.options());
  const bool has_ov = overflow.has_value() && overflow->defined();
  const auto ov = has_ov ? overflow->to(at::kLong).contiguous() : at::Tensor();
  coco_summary_kernel<<<static_cast<unsigned>(std::max<int64_t>(1, (cells + 255) / 256)), 256, 0, stream()>>>(
      p.data_ptr<double>(), r.data_ptr<double>(), T, kam, static_cast<int>(R), has_ov ? ov.data_ptr<int64_t>() : nullptr,
      dev_out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  auto host = at::empty({4 * cells + 1}, at::TensorOptions().dtype(at::kDouble).pinned_memory(true));
  TMX_CHECK_HIP(hipMemcpyAsync(host.data_ptr<double>(), dev_out.data_ptr<double>(), sizeof(double) * (4 * cells + 1),
                               hipMemcpyDeviceToHost, stream()));
  TMX_CHECK_HIP(hipStreamSynchronize(stream()));
  return host;
}

// (host bitmap [kClassWords + 1] int32 in pinned memory, read after this op's stream synchronisation; device ids
// [32 * kClassWords] int64 whose first popcount(bitmap) entries are the present ids, ascending)
std::tuple<at::Tensor, at::Tensor> class_presence(const at::Tensor& labels) {
  TORCH_CHECK(labels.is_cuda(), "class_presence: expected a GPU tensor");
  const c10::DeviceGuard guard(labels.device());
  const auto lab = labels.to(at::kLong).contiguous().reshape({-1});
  auto bm = at::zeros({kClassWords + 1}, lab.options().dtype(at::kInt));
  auto ids = at::empty({32 * kClassWords}, lab.options());
  const int64_t n = lab.numel();
  if (n > 0) {
    const int blocks = static_cast<int>(std::min<int64_t>((n + 4095) / 4096, 256));
    class_mark_kernel<<<blocks, 256, 0, stream()>>>(lab.data_ptr<int64_t>(), n, reinterpret_cast<uint32_t*>(bm.data_ptr<int>()));
    TMX_LAUNCH_CHECK();
  }
  class_compact_kernel<<<1, 1024, 0, stream()>>>(reinterpret_cast<const uint32_t*>(bm.data_ptr<int>()), ids.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  auto host = at::empty({kClassWords + 1}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
  TMX_CHECK_HIP(hipMemcpyAsync(host.data_ptr<int>(), bm.data_ptr<int>(), sizeof(int) * (kClassWords + 1),
                               hipMemcpyDeviceToHost, stream()));
  TMX_CHECK_HIP(hipStreamSynchronize(stream()));
  return {host, ids};
}

// The per-image route (coco_image_match_kernel): bbox IoU, scores exactly representable in fp32, no IoU export, at
// most kImgMaxRows detections and ground truths in every image (the caller checks the sizes, which it holds on the
// host).  det_off / gt_off: [I + 1] row offsets of each image in the flat arrays.  Same (precision, recall, scores)
// tables as coco_evaluate_gpu, plus a device flag (output 4) set when an image holds more rows than that (the tables
// are then invalid).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> coco_evaluate_gpu_img(
    const at::Tensor& det_boxes_, const at::Tensor& det_scores_, const at::Tensor& det_cls_, const at::Tensor& det_off_,
    const at::Tensor& gt_boxes_, const at::Tensor& gt_cls_, const at::Tensor& gt_crowd_, const at::Tensor& gt_area_,
    const at::Tensor& gt_off_, int64_t K, const at::Tensor& iou_thrs_, const at::Tensor& rec_thrs_,
    const at::Tensor& max_dets_, const c10::optional<at::Tensor>& max_dets_dev_, const at::Tensor& area_rng_) {
  TORCH_CHECK(det_scores_.is_cuda(), "coco_evaluate_gpu_img: expected GPU tensors");
  const auto st = det_scores_.scalar_type();
  TORCH_CHECK(st == at::kFloat || st == at::kHalf || st == at::kBFloat16, "coco_evaluate_gpu_img: fp32-exact scores only");
  const c10::DeviceGuard guard(det_scores_.device());
  const auto dev = det_scores_.device();
  auto f64 = [&](const at::Tensor& t) { return t.to(dev, at::kDouble).contiguous(); };
  auto i64 = [&](const at::Tensor& t) { return t.to(dev, at::kLong).contiguous(); };
  const auto det_boxes = f64(det_boxes_).reshape({-1, 4});
  const auto gt_boxes = f64(gt_boxes_).reshape({-1, 4}), gt_area = f64(gt_area_);
  const auto det_cls = i64(det_cls_), gt_cls = i64(gt_cls_), gt_crowd = i64(gt_crowd_);
  const auto det_off = i64(det_off_), gt_off = i64(gt_off_);
  const auto score32 = det_scores_.to(dev, at::kFloat).contiguous();
  const auto iou_thrs = f64(iou_thrs_), rec_thrs = f64(rec_thrs_), area_rng = f64(area_rng_).reshape({-1, 2});
  const auto max_dets_cpu = max_dets_.to(at::kCPU, at::kLong).contiguous();
  const int64_t T = iou_thrs.numel(), R = rec_thrs.numel(), M = max_dets_cpu.numel(), A = area_rng.size(0);
  const int64_t I = det_off.numel() - 1, n = det_cls.numel();
  TORCH_CHECK(T > 0 && R > 0 && M > 0 && A > 0, "coco_evaluate_gpu_img: empty parameter list");
  TORCH_CHECK(T * A <= 64, "coco_evaluate_gpu_img: at most 64 (IoU threshold, area range) combinations");
  TORCH_CHECK(R <= kCocoMaxRec, "coco_evaluate_gpu_img: at most ", kCocoMaxRec, " recall thresholds");
  TORCH_CHECK(I >= 0 && gt_off.numel() == I + 1, "coco_evaluate_gpu_img: det_off / gt_off must both hold I + 1 offsets");
  TORCH_CHECK(det_boxes.size(0) == n && score32.numel() == n,
              "coco_evaluate_gpu_img: detection columns differ in length");
  TORCH_CHECK(gt_boxes.size(0) == gt_cls.numel() && gt_crowd.numel() == gt_cls.numel() && gt_area.numel() == gt_cls.numel(),
              "coco_evaluate_gpu_img: ground-truth columns differ in length");
  const int64_t max_det_last = max_dets_cpu.data_ptr<int64_t>()[M - 1];
  // (a device copy of the thresholds from the caller's cache avoids a pageable host-to-device copy per call; the
  // clamp to maxDets[-1] is the identity for the sorted thresholds the module passes)
  const bool dev_md = max_dets_dev_.has_value() && max_dets_dev_->defined() && max_dets_dev_->is_cuda() &&
                      max_dets_dev_->scalar_type() == at::kLong && max_dets_dev_->numel() == M &&
                      std::is_sorted(max_dets_cpu.data_ptr<int64_t>(), max_dets_cpu.data_ptr<int64_t>() + M);
  const auto max_dets = dev_md ? max_dets_dev_->contiguous() : max_dets_cpu.clamp_max(max_det_last).to(dev);
  const auto fopt = det_boxes.options();
  // every entry is written by the accumulate kernel (-1 where a class / area has no ground truth)
  auto precision = at::empty({T, R, K, A, M}, fopt);
  auto recall = at::empty({T, K, A, M}, fopt);
  auto scores_out = at::empty({T, R, K, A, M}, fopt);
  const auto lopt = det_cls.options();
  auto overflow = at::zeros({1}, lopt);
  if (K == 0) return {precision, recall, scores_out, overflow};
  auto npig = at::zeros({K * A}, lopt);
  // one int64 buffer: rank (int32 pairs), matched, ignored, then the accumulate-order copies and seg
  auto work = at::empty({6 * n + K + 1}, lopt);
  int64_t* w = work.data_ptr<int64_t>();
  int32_t* rank = reinterpret_cast<int32_t*>(w);
  uint64_t* matched = reinterpret_cast<uint64_t*>(w + n);
  uint64_t* ignored = reinterpret_cast<uint64_t*>(w + 2 * n);
  int32_t* a_rank = reinterpret_cast<int32_t*>(w + 3 * n);
  uint64_t* a_matched = reinterpret_cast<uint64_t*>(w + 4 * n);
  uint64_t* a_ignored = reinterpret_cast<uint64_t*>(w + 5 * n);
  int64_t* seg = w + 6 * n;
  auto a_score = at::empty({n}, fopt);
  // TMX_COCO_IMG_PROBE (timing probe only, tools/coco_img_probe.py; wrong tables): bit 0 skips the ground-truth
  // counts, bit 1 the rank pass, bit 2 the matching
  const char* probe_env = std::getenv("TMX_COCO_IMG_PROBE");
  const int probe = probe_env != nullptr ? std::atoi(probe_env) : 0;
  if (I > 0) {
    coco_image_match_kernel<<<static_cast<unsigned>(I), kImgThreads, 0, stream()>>>(
        det_off.data_ptr<int64_t>(), gt_off.data_ptr<int64_t>(), det_boxes.data_ptr<double>(), score32.data_ptr<float>(),
        det_cls.data_ptr<int64_t>(), gt_boxes.data_ptr<double>(), gt_cls.data_ptr<int64_t>(),
        gt_crowd.data_ptr<int64_t>(), gt_area.data_ptr<double>(), iou_thrs.data_ptr<double>(), static_cast<int>(T),
        area_rng.data_ptr<double>(), static_cast<int>(A), max_det_last, rank, matched, ignored, overflow.data_ptr<int64_t>(), probe);
    TMX_LAUNCH_CHECK();
  }
  const int64_t n_gt = gt_cls.numel();
  if (n_gt > 0 && !(probe & 1)) {
    const bool lds = K * A <= kNpigLdsBins;
    const int blocks = static_cast<int>(std::min<int64_t>((n_gt + 511) / 512, 256));
    coco_npig_kernel<<<blocks, 256, lds ? sizeof(unsigned) * K * A : 0, stream()>>>(
        gt_cls.data_ptr<int64_t>(), gt_crowd.data_ptr<int64_t>(), gt_area.data_ptr<double>(), gt_boxes.data_ptr<double>(), n_gt,
        area_rng.data_ptr<double>(), static_cast<int>(A), static_cast<int>(K * A), lds, npig.data_ptr<int64_t>());
    TMX_LAUNCH_CHECK();
  }
  if (n == 0) {
    work.narrow(0, 6 * n, K + 1).zero_();
  } else {
    const auto acc = major_score_order(det_cls, score32);
    coco_acc_gather_kernel<<<static_cast<unsigned>((n + 255) / 256), 256, 0, stream()>>>(
        acc.data_ptr<int64_t>(), n, det_cls.data_ptr<int64_t>(), static_cast<int>(K), rank, matched, ignored,
        score32.data_ptr<float>(), a_rank, a_matched, a_ignored, a_score.data_ptr<double>(), seg);
    TMX_LAUNCH_CHECK();
  }
  TORCH_CHECK(n < (int64_t(1) << 31), "coco_evaluate_gpu_img: at most 2^31 - 1 detections");
  const int64_t combos = K * A * M * T;
  coco_accumulate_kernel<<<static_cast<unsigned>(combos / acc_wpb(T)), acc_wpb(T) * kWave, acc_lds_bytes(T, R), stream()>>>(
      seg, static_cast<int>(K), static_cast<int>(A), static_cast<int>(M), static_cast<int>(T), static_cast<int>(R),
      max_dets.data_ptr<int64_t>(), rec_thrs.data_ptr<double>(), a_rank, a_matched, a_ignored, a_score.data_ptr<double>(),
      npig.data_ptr<int64_t>(), precision.data_ptr<double>(), recall.data_ptr<double>(), scores_out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return {precision, recall, scores_out, overflow};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def(
      "coco_evaluate_gpu(Tensor det_boxes, Tensor det_scores, Tensor det_cls, Tensor det_img, Tensor det_area, "
      "Tensor gt_boxes, Tensor gt_cls, Tensor gt_img, Tensor gt_crowd, Tensor gt_area, int num_classes, "
      "int num_images, Tensor iou_thrs, Tensor rec_thrs, Tensor max_dets, Tensor area_rng, Tensor? img_iou, "
      "Tensor? img_iou_offsets, Tensor? det_local, Tensor? gt_local, Tensor? img_ng, bool export_iou) "
      "-> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "coco_evaluate_gpu_img(Tensor det_boxes, Tensor det_scores, Tensor det_cls, Tensor det_off, "
      "Tensor gt_boxes, Tensor gt_cls, Tensor gt_crowd, Tensor gt_area, Tensor gt_off, int num_classes, "
      "Tensor iou_thrs, Tensor rec_thrs, Tensor max_dets, Tensor? max_dets_dev, Tensor area_rng) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("class_presence(Tensor labels) -> (Tensor, Tensor)");
  m.def("coco_summary_tables(Tensor precision, Tensor recall, Tensor? overflow) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("coco_evaluate_gpu", &tmx::coco_evaluate_gpu);
  m.impl("coco_evaluate_gpu_img", &tmx::coco_evaluate_gpu_img);
  m.impl("class_presence", &tmx::class_presence);
  m.impl("coco_summary_tables", &tmx::coco_summary_tables);
}
