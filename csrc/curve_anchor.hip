// Exact AUROC / AP for fp32/fp64 scores without sorting the samples (non-binned curves).
//
// The reference sorts every class's full score column (``_binary_clf_curve``: argsort + cumsum per class,
// functional/classification/precision_recall_curve.py:28-80, called once per class at :558-563).  Both
// summaries only need, for every distinct *positive* score v, how many negatives lie above / at v:
//   AP    = sum_v pos(v) * tp(>=v) / (tp(>=v) + fp(>=v)) / P
//   AUROC = sum_neg [2 * #pos(> x) + #pos(== x)] / (2 P N)      (trapezoidal ROC area with ties)
// When positives are scarce (multiclass one-vs-rest: N / C per class), the positives of a class are the anchor:
//   1. anchor_prepare_kernel (one block per class): gather the class's positive scores, bitonic-sort them in LDS
//      (descending), collapse runs into distinct values + multiplicities.
//   2. anchor_stream_kernel (blocks = classes x row groups): the distinct positive values sit in LDS; the block
//      streams its slice of the class-major score column once (16-B loads) and drops every element into one of
//      2D + 1 slots - "strictly between v_{i-1} and v_i" (gap i) or "equal to v_i" (eq i) - found by binary
//      search in LDS; slot counters are LDS atomics flushed once per block with int64 global atomics.
//   3. anchor_finalize_kernel (one wave per class): positives are removed from the eq slots, and one wave scan
//      over the slots gives tp / fp at every distinct positive value -> AP, and the tie-aware AUROC sum.
// The samples are read once from HBM and never written; nothing is sorted except the (small) positive sets.
// Results agree with the sorted formulation up to fp64 rounding (integer slot counts; fixed reduction order).
#include "common.h"

namespace tmx {

constexpr int kAnchorMaxPos = 8192;  // per class; larger anchor sets take the sort-based path
constexpr int kAnchorThreads = 1024;
constexpr int kAnchorTable = 8192;   // bucket-table entries of the stream kernel (32 KiB)

typedef float AnchorF4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) AnchorF4 GlobalF4;

// monotone uint32 image of a float (-0 == +0 via x + 0; NaN lands outside every finite bucket)
__device__ __forceinline__ uint32_t anchor_order_key(float x) {
  const int i = __float_as_int(x + 0.0f);
  return static_cast<uint32_t>(i ^ ((i >> 31) | static_cast<int>(0x80000000u)));
}

// ------------------------------------------------------------------------------------------- 1. prepare
// pos_off [C+1]: positive rows of class c are pos_rows[pos_off[c] .. pos_off[c+1]).  X is class-major [C, N].
// Writes distinct values (descending) and multiplicities at the class's positive offset, and ndist[c].
struct AnchorChunks {
  const int64_t* base;    // [K] addresses of the class-major chunks (float [C, n_k])
  const int64_t* row_off; // [K+1] first global row of each chunk
  int K;
};

__device__ __forceinline__ float anchor_value(const AnchorChunks& ch, int c, int64_t row) {
  int lo = 0, hi = ch.K - 1;  // last chunk whose first row <= row
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ch.row_off[mid] <= row) lo = mid; else hi = mid - 1;
  }
  const int64_t n = ch.row_off[lo + 1] - ch.row_off[lo];
  return reinterpret_cast<const float*>(ch.base[lo])[static_cast<int64_t>(c) * n + (row - ch.row_off[lo])];
}

__global__ __launch_bounds__(kAnchorThreads) void anchor_prepare_kernel(
    AnchorChunks ch, const int64_t* __restrict__ pos_off, const int64_t* __restrict__ pos_rows,
    float* __restrict__ dvals, int32_t* __restrict__ dcnt, int32_t* __restrict__ ndist) {
  __shared__ float v[kAnchorMaxPos];
  __shared__ int32_t head_scan[kAnchorThreads];
  const int c = blockIdx.x;
  const int64_t p0 = pos_off[c];
  const int n = static_cast<int>(pos_off[c + 1] - p0);
  int pow2 = 1;
  while (pow2 < n) pow2 <<= 1;
  for (int i = threadIdx.x; i < pow2; i += blockDim.x) v[i] = i < n ? anchor_value(ch, c, pos_rows[p0 + i]) : -INFINITY;
  __syncthreads();
  // bitonic sort, descending
  for (int k = 2; k <= pow2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < pow2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const float a = v[i], b = v[l];
          const bool desc = (i & k) == 0;
          if (desc ? (a < b) : (a > b)) {
            v[i] = b;
            v[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // run heads -> distinct index by a block scan over per-thread head counts (each thread owns a contiguous run)
  const int per = (n + blockDim.x - 1) / blockDim.x;
  const int b0 = threadIdx.x * per, b1 = min(n, b0 + per);
  int heads = 0;
  for (int i = b0; i < b1; ++i) heads += (i == 0 || v[i] != v[i - 1]) ? 1 : 0;
  head_scan[threadIdx.x] = heads;
  __syncthreads();
  for (int off = 1; off < blockDim.x; off <<= 1) {  // Hillis-Steele inclusive scan (once per class, cheap)
    const int add = threadIdx.x >= off ? head_scan[threadIdx.x - off] : 0;
    __syncthreads();
    head_scan[threadIdx.x] += add;
    __syncthreads();
  }
  int d = head_scan[threadIdx.x] - heads;  // distinct index of this thread's first head
  for (int i = b0; i < b1; ++i) {
    if (i == 0 || v[i] != v[i - 1]) {
      int e = i + 1;
      while (e < n && v[e] == v[i]) ++e;
      dvals[p0 + d] = v[i];
      dcnt[p0 + d] = e - i;
      ++d;
    }
  }
  if (threadIdx.x == blockDim.x - 1) ndist[c] = head_scan[threadIdx.x];
}

// -------------------------------------------------------------------------------------------- 2. stream
// slot layout of class c (at 2 * pos_off[c] + c in `slots`): [2i] gap above v_i (i = 0..D), [2i+1] equal v_i.
// segs [S, 4] = (chunk base address, chunk rows n_k, first row, last row + 1) - 16-B aligned rows when VEC;
// block (class c, group g) streams segments grp[g] .. grp[g + 1] of column c, so the class table built in LDS
// is amortised over ~N / groups elements
template <bool VEC>
__global__ __launch_bounds__(kAnchorThreads) void anchor_stream_kernel(
    const int64_t* __restrict__ segs, const int64_t* __restrict__ grp, int n_groups, const int64_t* __restrict__ pos_off,
    const float* __restrict__ dvals, const int32_t* __restrict__ ndist, unsigned long long* __restrict__ slots) {
  extern __shared__ unsigned char anchor_lds[];
  const int c = blockIdx.x / n_groups, group = blockIdx.x % n_groups;
  const int D = ndist[c];
  uint32_t* table = reinterpret_cast<uint32_t*>(anchor_lds);  // [kAnchorTable]: first key | key count << 16
  float* keys = reinterpret_cast<float*>(table + kAnchorTable);
  uint32_t* bins = reinterpret_cast<uint32_t*>(keys + D);
  const int nb = 2 * D + 1;
  const int64_t p0 = pos_off[c];
  for (int i = threadIdx.x; i < D; i += blockDim.x) keys[i] = dvals[p0 + i];
  for (int i = threadIdx.x; i < nb; i += blockDim.x) bins[i] = 0u;
  __syncthreads();
  // Bucket table over the keys' range, fine enough that a bucket rarely holds more than one key:
  // bucket(x) = order_key(x) >> shift; entry j describes bucket bmin - 1 + j (entry 0 and entry nt - 1 are the
  // "below every key" / "above every key" sentinels, and every bucket outside the range clamps onto them).
  // An element then needs one table read, at most one key read and a compare; only buckets with >= 2 keys search.
  uint32_t bmin = 0;
  int nt = 1, shift = 8;
  if (D > 0) {
    const uint32_t kmax = anchor_order_key(keys[0]), kmin = anchor_order_key(keys[D - 1]);
    // ~4 table entries per key (most buckets then hold <= 1 key) and never more than the LDS table
    const uint32_t limit = static_cast<uint32_t>(min(kAnchorTable, max(256, 4 * D)));
    while (shift < 31 && (kmax >> shift) - (kmin >> shift) + 3 > limit) ++shift;
    bmin = kmin >> shift;
    nt = static_cast<int>((kmax >> shift) - bmin) + 3;
  }
  auto count_above = [&](int64_t bj) {  // keys with bucket > bj (keys descending -> buckets non-increasing)
    int lo = 0, hi = D;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (static_cast<int64_t>(anchor_order_key(keys[mid]) >> shift) > bj) lo = mid + 1; else hi = mid;
    }
    return static_cast<uint32_t>(lo);
  };
  for (int j = threadIdx.x; j < nt; j += blockDim.x) {
    const int64_t bj = static_cast<int64_t>(bmin) - 1 + j;
    uint32_t first, cnt;
    if (j == 0) {
      first = static_cast<uint32_t>(D); cnt = 0;  // below every key
    } else if (j == nt - 1) {
      first = 0; cnt = 0;                         // above every key
    } else {
      first = count_above(bj);
      cnt = count_above(bj - 1) - first;
    }
    table[j] = first | (cnt << 16);
  }
  __syncthreads();
  // the two open-ended gaps are the hot slots on real data (most negatives below every positive): they are
  // counted in registers and added once per wave, not with per-element LDS atomics
  uint32_t n_above = 0, n_below = 0;
  const int last = nt - 1;
  const int dmax = D > 0 ? D - 1 : 0;

  constexpr int kE = 8;  // elements per thread per round: every phase is issued for all of them before one wait
  auto drop_batch = [&](const float (&x)[kE], int valid) {
    uint32_t ent[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const int d = static_cast<int>(anchor_order_key(x[e]) >> shift) - static_cast<int>(bmin) + 1;
      ent[e] = table[min(max(d, 0), last)];
    }
    float k0[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) k0[e] = keys[min(static_cast<int>(ent[e] & 0xFFFFu), dmax)];
    int slot[kE];
    bool any_deep = false;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      // common case without branches: the bucket holds 0 or 1 keys, or x is not below its first key
      const int first = static_cast<int>(ent[e] & 0xFFFFu);
      const bool gt = ent[e] < 0x10000u || x[e] > k0[e];
      slot[e] = 2 * first + (gt ? 0 : (x[e] == k0[e] ? 1 : 2));
      any_deep |= !gt && x[e] < k0[e] && ent[e] >= 0x20000u;
    }
    if (__ballot(any_deep)) {  // below the first of several keys in one bucket: search the bucket (rare)
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int first = static_cast<int>(ent[e] & 0xFFFFu), cnt = static_cast<int>(ent[e] >> 16);
        if (cnt > 1 && x[e] < k0[e]) {
          int lo = first + 1, hi = first + cnt;
          const int end = hi;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (keys[mid] > x[e]) lo = mid + 1; else hi = mid;
          }
          slot[e] = (lo < end && keys[lo] == x[e]) ? 2 * lo + 1 : 2 * lo;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const bool live = e < valid;
      const bool above = slot[e] == 0, below = slot[e] == 2 * D;
      n_above += (live && above) ? 1u : 0u;
      n_below += (live && below) ? 1u : 0u;
      if (live && !above && !below) atomicAdd(bins + slot[e], 1u);
    }
  };

  for (int64_t sg = grp[group]; sg < grp[group + 1]; ++sg) {
    const int64_t* tl = segs + 4 * sg;
    const int64_t n_k = tl[1], r0 = tl[2], r1 = tl[3];
    const float* col = reinterpret_cast<const float*>(tl[0]) + static_cast<int64_t>(c) * n_k;
    if (VEC) {  // every chunk has n_k % 4 == 0 and segment bounds on multiples of 4; two 16-B loads in flight
      // global (not flat) loads: flat loads count on lgkmcnt too, so every LDS wait would also wait for them
      const GlobalF4* c4 = (const GlobalF4*)(col);  // address-space cast
      const int e4 = static_cast<int>(r1 / 4 - r0 / 4);  // float4s of this segment (< 2^31)
      c4 += r0 / 4;
      const int stride = blockDim.x;
      // software pipeline: the next round's two loads are issued before this round's LDS work
      int i = threadIdx.x;
      AnchorF4 n0, n1;
      if (i < e4) {
        n0 = c4[i];
        n1 = c4[i + stride < e4 ? i + stride : i];  // unconditional load, ignored when out of range
      }
      for (; i < e4; i += 2 * stride) {
        const bool second = i + stride < e4;
        const AnchorF4 q0 = n0, q1 = n1;
        const int nx = i + 2 * stride;
        if (nx < e4) {
          n0 = c4[nx];
          n1 = c4[nx + stride < e4 ? nx + stride : nx];
        }
        const float x[kE] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        drop_batch(x, second ? 8 : 4);
      }
    } else {
      for (int64_t i = r0 + threadIdx.x * kE; i < r1; i += static_cast<int64_t>(blockDim.x) * kE) {
        float x[kE];
#pragma unroll
        for (int e = 0; e < kE; ++e) x[e] = i + e < r1 ? col[i + e] : 0.f;
        drop_batch(x, static_cast<int>(min<int64_t>(kE, r1 - i)));
      }
    }
  }
  // register counts of the open-ended gaps: wave sums, one atomic per wave
  const uint32_t wa = static_cast<uint32_t>(wave_sum(static_cast<long long>(n_above)));
  const uint32_t wb = static_cast<uint32_t>(wave_sum(static_cast<long long>(n_below)));
  if ((threadIdx.x & (kWave - 1)) == 0) {
    if (wa) atomicAdd(bins, wa);
    if (wb) atomicAdd(bins + 2 * D, wb);
  }
  __syncthreads();
  unsigned long long* out = slots + 2 * p0 + c;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const uint32_t v = bins[i];
    if (v) atomicAdd(out + i, static_cast<unsigned long long>(v));
  }
}

// ------------------------------------------------------------------------------------------ 3. finalize
__global__ __launch_bounds__(kWave) void anchor_finalize_kernel(
    int64_t N, const int64_t* __restrict__ pos_off, const int32_t* __restrict__ dcnt, const int32_t* __restrict__ ndist,
    const unsigned long long* __restrict__ slots, double* __restrict__ out) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const int64_t p0 = pos_off[c];
  const int64_t P = pos_off[c + 1] - p0;
  const int D = ndist[c];
  const unsigned long long* sl = slots + 2 * p0 + c;
  const int64_t Nn = N - P;
  // chunked wave scan over distinct positive values (descending): carry = (#pos above, #neg at or above)
  int64_t pos_above = 0, neg_upto = 0;
  double auc2 = 0.0, ap = 0.0;
  for (int base = 0; base <= D; base += kWave) {
    const int i = base + lane;
    int64_t pc = 0, gap = 0, negeq = 0;
    if (i < D) {
      pc = dcnt[p0 + i];
      negeq = static_cast<int64_t>(sl[2 * i + 1]) - pc;
    }
    if (i <= D) gap = static_cast<int64_t>(sl[2 * i]);
    // inclusive scans of pc and (gap + negeq) across the chunk
    int64_t spc = pc, sneg = gap + negeq;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int64_t a = __shfl_up(spc, off, kWave), b = __shfl_up(sneg, off, kWave);
      if (lane >= off) {
        spc += a;
        sneg += b;
      }
    }
    const int64_t cum_pc = pos_above + spc - pc;  // positives strictly above v_i
    const int64_t fp = neg_upto + sneg;           // negatives >= v_i
    const int64_t tp = cum_pc + pc;
    double a2 = static_cast<double>(gap) * 2.0 * static_cast<double>(cum_pc);
    double apc = 0.0;
    if (i < D) {
      a2 += static_cast<double>(negeq) * (2.0 * static_cast<double>(cum_pc) + static_cast<double>(pc));
      apc = static_cast<double>(pc) * static_cast<double>(tp) / static_cast<double>(tp + fp);
    }
    auc2 += wave_sum(a2);
    ap += wave_sum(apc);
    pos_above += __shfl(spc, kWave - 1, kWave);
    neg_upto += __shfl(sneg, kWave - 1, kWave);
  }
  if (lane == 0) {
    const double Pd = static_cast<double>(P), Nd = static_cast<double>(Nn);
    out[4 * c + 0] = (P > 0 && Nn > 0) ? auc2 / (2.0 * Pd * Nd) : 0.0;
    out[4 * c + 1] = P > 0 ? ap / Pd : NAN;
    out[4 * c + 2] = Pd;
    out[4 * c + 3] = Nd;
  }
}

// -------------------------------------------------------------------------------------------------- host
// chunks: class-major fp32 [C, n_k] buffers (the samples of K updates, never concatenated); pos_off: int64 [C+1];
// pos_rows: int64 [P] global rows (over the chunks in order) of class c's positives, grouped by class.
// Returns float64 [C, 4] = (auroc, ap, n_pos, n_neg), the layout of curve_hist_reduce.
at::Tensor anchored_curve_scores(at::TensorList chunks_, const at::Tensor& pos_off_, const at::Tensor& pos_rows_, int64_t max_pos) {
  TORCH_CHECK(!chunks_.empty(), "anchored_curve_scores: no score chunks");
  TORCH_CHECK(max_pos <= kAnchorMaxPos, "anchored_curve_scores: more than ", kAnchorMaxPos, " positives in one class");
  const auto dev = chunks_[0].device();
  TORCH_CHECK(dev.is_cuda(), "anchored_curve_scores: expected GPU score chunks");
  const c10::DeviceGuard guard(dev);
  const int64_t C = chunks_[0].size(0);
  std::vector<at::Tensor> chunks;
  std::vector<int64_t> row_off{0}, bases;
  bool vec = true;
  for (const auto& t : chunks_) {
    TORCH_CHECK(t.dim() == 2 && t.size(0) == C && t.device() == dev, "anchored_curve_scores: chunks must be [C, n_k] on one device");
    chunks.push_back(t.to(at::kFloat).contiguous());
    bases.push_back(reinterpret_cast<int64_t>(chunks.back().data_ptr<float>()));
    row_off.push_back(row_off.back() + t.size(1));
    vec = vec && (t.size(1) % 4 == 0);
  }
  const int64_t N = row_off.back();
  const int K = static_cast<int>(chunks.size());
  const auto lopt = at::TensorOptions().dtype(at::kLong);
  const auto pos_off = pos_off_.to(dev, at::kLong).contiguous();
  const auto pos_rows = pos_rows_.to(dev, at::kLong).contiguous();
  TORCH_CHECK(pos_off.numel() == C + 1, "anchored_curve_scores: pos_off must have C + 1 entries");
  const int64_t Ptot = pos_rows.numel();
  const auto fopt = chunks[0].options();
  auto out = at::empty({C, 4}, fopt.dtype(at::kDouble));
  if (C == 0) return out;

  // groups: ~2048 blocks over (class, group of rows), each group >= 16384 rows (cut at multiples of 4), made of
  // per-chunk segments
  const int64_t target_blocks = 2048;
  const int64_t per_class = std::max<int64_t>(1, (target_blocks + C - 1) / C);
  int64_t piece = std::max<int64_t>(16384, (N + per_class - 1) / per_class);
  piece = (piece + 3) / 4 * 4;
  std::vector<int64_t> segs, grp{0};
  for (int64_t g0 = 0; g0 < N; g0 += piece) {
    const int64_t g1 = std::min(N, g0 + piece);
    for (int k = 0; k < K; ++k) {
      const int64_t a0 = std::max(g0, row_off[k]), a1 = std::min(g1, row_off[k + 1]);
      if (a0 < a1) segs.insert(segs.end(), {bases[k], row_off[k + 1] - row_off[k], a0 - row_off[k], a1 - row_off[k]});
    }
    grp.push_back(static_cast<int64_t>(segs.size() / 4));
  }
  const int n_groups = static_cast<int>(grp.size() - 1);
  // one small host->device copy for the chunk table, the segments and the groups
  std::vector<int64_t> meta(bases);
  meta.insert(meta.end(), row_off.begin(), row_off.end());
  meta.insert(meta.end(), segs.begin(), segs.end());
  meta.insert(meta.end(), grp.begin(), grp.end());
  auto meta_t = at::from_blob(meta.data(), {static_cast<int64_t>(meta.size())}, lopt).to(dev, /*non_blocking=*/false);
  const int64_t* meta_p = meta_t.data_ptr<int64_t>();
  AnchorChunks ch{meta_p, meta_p + K, K};
  const int64_t* segs_p = meta_p + 2 * K + 1;
  const int64_t* grp_p = segs_p + segs.size();

  auto dvals = at::empty({std::max<int64_t>(Ptot, 1)}, fopt);
  auto dcnt = at::empty({std::max<int64_t>(Ptot, 1)}, fopt.dtype(at::kInt));
  auto ndist = at::empty({C}, fopt.dtype(at::kInt));
  auto slots = at::zeros({2 * Ptot + C}, fopt.dtype(at::kLong));
  anchor_prepare_kernel<<<static_cast<unsigned>(C), kAnchorThreads, 0, stream()>>>(
      ch, pos_off.data_ptr<int64_t>(), pos_rows.data_ptr<int64_t>(), dvals.data_ptr<float>(), dcnt.data_ptr<int32_t>(),
      ndist.data_ptr<int32_t>());
  TMX_LAUNCH_CHECK();
  if (n_groups > 0) {
    const size_t lds = sizeof(uint32_t) * kAnchorTable + sizeof(float) * max_pos + sizeof(uint32_t) * (2 * max_pos + 1);
    const unsigned grid = static_cast<unsigned>(C * n_groups);
    const void* fn = vec ? reinterpret_cast<const void*>(&anchor_stream_kernel<true>)
                         : reinterpret_cast<const void*>(&anchor_stream_kernel<false>);
    if (lds > 64 * 1024) TMX_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    if (vec) {
      anchor_stream_kernel<true><<<grid, kAnchorThreads, lds, stream()>>>(
          segs_p, grp_p, n_groups, pos_off.data_ptr<int64_t>(), dvals.data_ptr<float>(), ndist.data_ptr<int32_t>(),
          reinterpret_cast<unsigned long long*>(slots.data_ptr<int64_t>()));
    } else {
      anchor_stream_kernel<false><<<grid, kAnchorThreads, lds, stream()>>>(
          segs_p, grp_p, n_groups, pos_off.data_ptr<int64_t>(), dvals.data_ptr<float>(), ndist.data_ptr<int32_t>(),
          reinterpret_cast<unsigned long long*>(slots.data_ptr<int64_t>()));
    }
    TMX_LAUNCH_CHECK();
  }
  anchor_finalize_kernel<<<static_cast<unsigned>(C), kWave, 0, stream()>>>(
      N, pos_off.data_ptr<int64_t>(), dcnt.data_ptr<int32_t>(), ndist.data_ptr<int32_t>(),
      reinterpret_cast<const unsigned long long*>(slots.data_ptr<int64_t>()), out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

// --------------------------------------------------------------------------- update: softmax -> class-major
// The multiclass update of the fp32 sample state: rows [N, C] (C % 4 == 0, C <= 1024) become class-major
// probabilities [C, N] in one pass - softmax when the batch has any value outside [0, 1] (device flag from
// range_flag, the reference's per-batch rule), identity otherwise.  A 1024-thread block owns 32 rows; each wave
// holds two rows in registers (lane j: columns 4j + 256k, k < 4, 16-B loads), reduces max / sum with wave
// shuffles, then the block transposes 256-column slabs through LDS (row stride 260 floats: 16-B stores, no bank
// conflicts on the transposed reads) so every class column leaves as one full 128-B line per block.
constexpr int kSmRows = 32;
constexpr int kSmThreads = 1024;
constexpr int kSmSlab = 256;
constexpr int kSmLd = kSmSlab + 4;

__global__ __launch_bounds__(kSmThreads) void softmax_colmajor_kernel(const float* __restrict__ x, int64_t N, int C,
                                                                      const int* __restrict__ flag, const int64_t* __restrict__ target,
                                                                      int* __restrict__ err, float* __restrict__ out) {
  __shared__ float tile[kSmRows * kSmLd];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kSmRows;
  const int rows = static_cast<int>(min<int64_t>(kSmRows, N - r0));
  const bool soft = *flag != 0;
  const int C4 = C / 4;
  float4 v[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 2 * wave + h;
    const float4* row = reinterpret_cast<const float4*>(x + (r0 + r) * C);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = lane + 64 * k;
      v[h][k] = (r < rows && j < C4) ? row[j] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
  }
  if (target != nullptr && threadIdx.x < rows) {  // fused target range check (deferred error flag)
    const int64_t tv = target[r0 + threadIdx.x];
    if (tv < 0 || tv >= C) atomicOr(err, 1);
  }
  if (soft) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float m = -INFINITY;
#pragma unroll
      for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fmaxf(v[h][k].x, v[h][k].y), fmaxf(v[h][k].z, v[h][k].w)));
      m = wave_max(m);
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (lane + 64 * k < C4) {
          v[h][k].x = expf(v[h][k].x - m);
          v[h][k].y = expf(v[h][k].y - m);
          v[h][k].z = expf(v[h][k].z - m);
          v[h][k].w = expf(v[h][k].w - m);
          sum += (v[h][k].x + v[h][k].y) + (v[h][k].z + v[h][k].w);
        }
      }
      sum = wave_sum(sum);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[h][k].x /= sum;
        v[h][k].y /= sum;
        v[h][k].z /= sum;
        v[h][k].w /= sum;
      }
    }
  }
  const int tr = threadIdx.x % kSmRows, tc = threadIdx.x / kSmRows;  // transposed reader: row, column group
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (64 * k >= C4) break;  // block-uniform
#pragma unroll
    for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(tile + (2 * wave + h) * kSmLd + 4 * lane) = v[h][k];
    __syncthreads();
    const int cols = min(kSmSlab, C - kSmSlab * k);
    if (tr < rows) {
      for (int cc = tc; cc < cols; cc += kSmThreads / kSmRows)
        out[static_cast<int64_t>(kSmSlab * k + cc) * N + r0 + tr] = tile[tr * kSmLd + cc];
    }
    __syncthreads();
  }
}

at::Tensor range_flag(const at::Tensor& x_);  // classification.hip

at::Tensor softmax_colmajor(const at::Tensor& x_, const c10::optional<at::Tensor>& target_, const c10::optional<at::Tensor>& err_) {
  TORCH_CHECK(x_.is_cuda() && x_.dim() == 2 && x_.scalar_type() == at::kFloat, "softmax_colmajor: expected GPU fp32 [N, C]");
  TORCH_CHECK(x_.size(1) <= 1024 && x_.size(1) % 4 == 0, "softmax_colmajor: C must be a multiple of 4 and <= 1024");
  const c10::DeviceGuard guard(x_.device());
  const auto x = x_.contiguous();
  const int64_t N = x.size(0);
  const int C = static_cast<int>(x.size(1));
  auto out = at::empty({C, N}, x.options());
  if (N == 0 || C == 0) return out;
  at::Tensor target;
  const bool check = target_.has_value() && target_->defined() && err_.has_value() && err_->defined();
  if (check) {
    target = target_->to(at::kLong).contiguous();
    TORCH_CHECK(target.numel() == N && err_->scalar_type() == at::kInt && err_->is_cuda(), "softmax_colmajor: bad target / flag");
  }
  const auto flag = range_flag(x);
  const unsigned grid = static_cast<unsigned>((N + kSmRows - 1) / kSmRows);
  softmax_colmajor_kernel<<<grid, kSmThreads, 0, stream()>>>(x.data_ptr<float>(), N, C, flag.data_ptr<int>(),
                                                             check ? target.data_ptr<int64_t>() : nullptr,
                                                             check ? err_->data_ptr<int>() : nullptr, out.data_ptr<float>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("anchored_curve_scores(Tensor[] chunks, Tensor pos_off, Tensor pos_rows, int max_pos) -> Tensor");
  m.def("softmax_colmajor(Tensor x, Tensor? target=None, Tensor? err_flag=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("anchored_curve_scores", &tmx::anchored_curve_scores);
  m.impl("softmax_colmajor", &tmx::softmax_colmajor);
}
