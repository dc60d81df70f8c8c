// Classification hot paths for gfx950 (SURVEY §2.10 kernels K1, K2, K4, K5, K6, K8).
//
//  * tmx::range_flag          — device-side "any value outside [0,1] (or NaN)" flag; replaces the reference's
//                               host-synchronising `if not torch.all((p>=0)*(p<=1))` (stat_scores.py:104).
//  * tmx::bincount            — LDS-privatised int32 histogram, one int64 global atomic per non-empty bin per
//                               workgroup (replaces the deterministic-mode per-bin Python loop, data.py:194).
//  * tmx::mc_confmat_update   — fused argmax-over-C + (target, pred) histogram into an int64 [C, C] state
//                               (stat_scores.py:405-418, confusion_matrix.py:306-337).  One wave per row for
//                               large C (16-B vector loads), one thread per row for small C; LDS-privatised
//                               confusion matrix when C*C int32 counters fit in 64 KiB.
//  * tmx::mc_stat_scores_update — the same pair stream into per-class tp / fp / tn / fn states in place (no
//                               [C, C] temporary, target/pred range validation folded into device flags).
//  * tmx::binary_stats_update — one-pass tp/fp/tn/fn per label with the sigmoid-if-needed + threshold rule
//                               evaluated in the input dtype (stat_scores.py:95-131, 650-681).
//  * tmx::curve_hist_update   — exact score histogram for 16-bit scores: each (class, label, score-code) is
//                               counted in an int64 [C, 2, 16384] state.  A bf16/fp16 value in [0, 1] has at
//                               most 16257 codes and code order == value order, so this reproduces the
//                               reference's sort-based `_binary_clf_curve` (precision_recall_curve.py:28-80)
//                               exactly, with a fixed-size, all-reducible state instead of a growing `cat` list.
//  * tmx::curve_hist_reduce   — per-class AUROC / AP / positive / negative totals from that histogram: one
//                               workgroup per class, block scan over codes in descending order (K8).
//  * tmx::binned_curve_update — bucketize (binary search over T thresholds in LDS) + per-(class, label,
//                               bucket) histogram, then a suffix scan into the reference's [T, C, 2, 2]
//                               multi-threshold confusion matrix (K5) — O(N*C*log T) instead of O(N*C*T).
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include "common.h"

#include <map>
#include <tuple>
#include <mutex>
#include "curve_hist_kernels.h"

namespace tmx {

// =========================================================================================================
// range flag
// =========================================================================================================
template <typename T>
__global__ void range_flag_kernel(const T* __restrict__ x, int64_t n, int* __restrict__ flag) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = to_f32<T>(x[i]);
    bad |= !(v >= 0.f && v <= 1.f);
  }
  unsigned long long m = __ballot(bad);
  if (m && (threadIdx.x & (kWave - 1)) == 0) atomicOr(flag, 1);
}

// fp32: 16-B loads, four in flight per thread, and an early exit once any wave has found an out-of-range value
// (logits trip the flag in the first few elements, so the remaining blocks read nothing)
__global__ __launch_bounds__(256) void range_flag_f32_kernel(const float4* __restrict__ x, int64_t nvec, const float* __restrict__ tail,
                                                             int ntail, int* __restrict__ flag) {
  auto out = [](float v) { return !(v >= 0.f && v <= 1.f); };
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  bool bad = i < ntail && out(tail[i]);
  for (; i < nvec; i += 4 * stride) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    float4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = i + u * stride < nvec ? x[i + u * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) bad |= out(q[u].x) | out(q[u].y) | out(q[u].z) | out(q[u].w);
    if (__ballot(bad)) break;
  }
  // one store per wave that found something, and only while the flag is still clear (no same-address storm)
  if (__ballot(bad) && (threadIdx.x & (kWave - 1)) == 0 && !__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicOr(flag, 1);
}

at::Tensor range_flag(const at::Tensor& x_) {
  auto x = x_.contiguous();
  auto flag = at::zeros({1}, x.options().dtype(at::kInt));
  const int64_t n = x.numel();
  if (n == 0) return flag;
  const int block = 256;
  const bool aligned = (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0;
  if ((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) && aligned) {
    const int64_t nvec = n / 8;
    const int ntail = static_cast<int>(n - nvec * 8);
    const uint16_t* tail = reinterpret_cast<const uint16_t*>(x.data_ptr()) + nvec * 8;
    const uint4* xv = reinterpret_cast<const uint4*>(x.data_ptr());
    const int grid = grid_for(std::max<int64_t>(nvec, 1), block, 2048);
    if (x.scalar_type() == at::kBFloat16)
      hipLaunchKernelGGL(range_flag16_kernel<__hip_bfloat16>, grid, block, 0, stream(), xv, nvec, tail, ntail, flag.data_ptr<int>());
    else
      hipLaunchKernelGGL(range_flag16_kernel<__half>, grid, block, 0, stream(), xv, nvec, tail, ntail, flag.data_ptr<int>());
  } else if (x.scalar_type() == at::kFloat && aligned) {
    const int64_t nvec = n / 4;
    const int ntail = static_cast<int>(n - nvec * 4);
    const float* tail = x.data_ptr<float>() + nvec * 4;
    // a one-block probe over the head first: for logits it sets the flag and every wave of the main pass leaves
    // after one flag read; probabilities (all in range) are read once in full, without any atomics
    const float4* xv = reinterpret_cast<const float4*>(x.data_ptr<float>());
    const int64_t head = std::min<int64_t>(nvec, 16384);
    // 16 probe blocks: one block reading the 256-KiB head alone took 20 us (latency-bound) on in-range data
    hipLaunchKernelGGL(range_flag_f32_kernel, static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(16, (head + 1023) / 1024))), block, 0,
                       stream(), xv, head, tail, ntail, flag.data_ptr<int>());  // >= 1 block: it also checks the < 4-element tail
    if (nvec > head) {
      const int grid = grid_for(std::max<int64_t>((nvec - head + 3) / 4, 1), block, 2048);
      hipLaunchKernelGGL(range_flag_f32_kernel, grid, block, 0, stream(), xv + head, nvec - head, tail, 0, flag.data_ptr<int>());
    }
  } else {
    TMX_DISPATCH_FLOAT(x.scalar_type(), "range_flag", [&] {
      hipLaunchKernelGGL(range_flag_kernel<scalar_t>, grid_for(n, block), block, 0, stream(),
                         reinterpret_cast<const scalar_t*>(x.data_ptr()), n, flag.data_ptr<int>());
    });
  }
  TMX_LAUNCH_CHECK();
  return flag;
}

// =========================================================================================================
// bincount
// =========================================================================================================
__global__ void bincount_lds_kernel(const int64_t* __restrict__ x, int64_t n, int nbins, int64_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) int s_bins[];
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) s_bins[b] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = x[i];
    if (v >= 0 && v < nbins) atomicAdd(&s_bins[v], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int c = s_bins[b];
    if (c) atomic_add_i64(out + b, c);
  }
}

__global__ void bincount_global_kernel(const int64_t* __restrict__ x, int64_t n, int64_t nbins, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = x[i];
    if (v >= 0 && v < nbins) atomic_add_i64(out + v, 1);
  }
}

at::Tensor bincount(const at::Tensor& x_, int64_t minlength) {
  auto x = x_.contiguous().to(at::kLong);
  auto out = at::zeros({minlength}, x.options().dtype(at::kLong));
  const int64_t n = x.numel();
  if (n == 0 || minlength == 0) return out;
  const int block = 256;
  if (minlength <= 16384) {
    const int grid = grid_for(n, block * 8, 1024);
    hipLaunchKernelGGL(bincount_lds_kernel, grid, block, minlength * sizeof(int), stream(), x.data_ptr<int64_t>(), n,
                       (int)minlength, out.data_ptr<int64_t>());
  } else {
    hipLaunchKernelGGL(bincount_global_kernel, grid_for(n, block), block, 0, stream(), x.data_ptr<int64_t>(), n,
                       minlength, out.data_ptr<int64_t>());
  }
  TMX_LAUNCH_CHECK();
  return out;
}

// =========================================================================================================
// multiclass (target, pred) pair stream: labels or arg-max of scores, accumulated by a policy
//   ConfmatAcc -> int64 [C, C] confusion matrix
//   StatAcc    -> per-class (or micro) tp / fp / tn / fn states, updated in place
// Range validation rides along: a target outside [0, C) that is not the ignore index ORs err_t, an integer
// prediction outside [0, C) ORs err_p (the deferred-validation flags of utilities/validation.py); such rows are
// skipped exactly like the confusion matrix skips them.
// =========================================================================================================
__device__ __forceinline__ void confmat_flush(int* s_cm, int64_t* g_cm, int C) {
  __syncthreads();
  for (int b = threadIdx.x; b < C * C; b += blockDim.x) {
    int c = s_cm[b];
    if (c) atomic_add_i64(g_cm + b, c);
  }
}

// Grid-wide sums of K int64 values with last-workgroup detection, without same-address pile-ups: workgroup b adds
// its values into the 128-B line of group b % 8 (one group per XCD under the round-robin dispatch) and takes that
// line's ticket; the group's last workgroup moves the group sums into the top line and takes the top ticket; the
// last of those sees the grid totals.  Sums are read and reset with atomic exchanges (performed at the coherence
// point, after the adds: every adder waits for its adds (vmcnt 0) before taking a ticket), tickets reset the
// same way, so the table is back to zero when the kernel ends.  Called by ONE thread per workgroup; true in
// exactly one workgroup of the grid.  slots: kGridSlotsWords zeroed int64 words.
constexpr int kGridSlotLine = 16;                    // int64 words per 128-B line
constexpr int kGridSlotsWords = 9 * kGridSlotLine;   // 8 group lines + top line
template <int K>
__device__ bool grid_sum_last(unsigned long long* slots, const long long (&v)[K], long long (&tot)[K]) {
  const unsigned G = gridDim.x, x = blockIdx.x & 7u;
  const unsigned groups = G < 8u ? G : 8u;
  const unsigned gsize = (G - x + 7u) / 8u;
  unsigned long long* line = slots + x * kGridSlotLine;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (v[k]) atomicAdd(line + 1 + k, (unsigned long long)v[k]);
  __builtin_amdgcn_s_waitcnt(0);
  if (atomicAdd(line, 1ull) != gsize - 1u) return false;
  long long gs[K];
#pragma unroll
  for (int k = 0; k < K; ++k) gs[k] = (long long)atomicExch(line + 1 + k, 0ull);
  atomicExch(line, 0ull);
  unsigned long long* top = slots + 8 * kGridSlotLine;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (gs[k]) atomicAdd(top + 1 + k, (unsigned long long)gs[k]);
  __builtin_amdgcn_s_waitcnt(0);
  if (atomicAdd(top, 1ull) != groups - 1u) return false;
#pragma unroll
  for (int k = 0; k < K; ++k) tot[k] = (long long)atomicExch(top + 1 + k, 0ull);
  atomicExch(top, 0ull);
  return true;
}

struct ConfmatAcc {
  int64_t* cm;
  int C;
  bool use_lds;
  // LDS copy only for tiny C: zeroing + flushing C*C words per workgroup costs more than the contention it saves
  static ConfmatAcc make(int64_t* cm, int C) { return {cm, C, C <= 32}; }
  int64_t lds_words() const { return use_lds ? (int64_t)C * C : 0; }
  __host__ size_t lds_bytes() const { return use_lds ? (size_t)C * C * sizeof(int) : 0; }
  __device__ void init(int* s) {
    if (!use_lds) return;
    for (int b = threadIdx.x; b < C * C; b += blockDim.x) s[b] = 0;
    __syncthreads();
  }
  __device__ void add(int* s, int t, int p) {
    const int idx = t * C + p;
    if (use_lds) atomicAdd(&s[idx], 1);
    else atomic_add_i64(cm + idx, 1);
  }
  __device__ void flush(int* s) {
    if (use_lds) confmat_flush(s, cm, C);
  }
};

// tp[t] / fp[p] / fn[t] per valid row, privatised in LDS ([3][C] ints) when they fit.  tn[c] = V - tp - fp - fn
// with V the batch's valid-row count: each block subtracts its (tp + fp + fn)[c] sparsely and contributes its V
// to grid_sum_last; the last block adds the total V to every class, so a batch costs one launch and no
// temporary.  micro: four scalar states, tn += C * V - tp - 2 * fp (every wrong row is one fp and one fn), the
// per-block sums also go through grid_sum_last (4096 blocks x 4 atomics on one line cost ~35 us).
enum StatMode { kStatLds = 0, kStatGlobal = 1, kStatMicro = 2 };

template <int MODE>
struct StatAcc {
  static constexpr bool use_lds = MODE == kStatLds;
  static constexpr bool micro = MODE == kStatMicro;
  int64_t *tp, *fp, *tn, *fn;
  unsigned long long* ticket;
  int C;
  int n_valid, n_tp, n_fp;  // per-thread counters

  static bool lds_fits(int C) { return 3 * (int64_t)C * 4 <= 60 * 1024; }
  __host__ __device__ int base() const { return use_lds ? 3 * C : 0; }
  __host__ size_t lds_bytes() const { return (size_t)(base() + 4) * sizeof(int); }
  int64_t lds_words() const { return base(); }
  __device__ void init(int* s) {
    const int nb = base() + 4;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) s[b] = 0;
    __syncthreads();
  }
  __device__ void add(int* s, int t, int p) {
    ++n_valid;
    if constexpr (micro) {
      if (p == t) ++n_tp;
      else ++n_fp;
    } else if constexpr (use_lds) {
      if (p == t) {
        atomicAdd(&s[t], 1);
      } else {
        atomicAdd(&s[C + p], 1);
        atomicAdd(&s[2 * C + t], 1);
      }
    } else if (p == t) {
      atomic_add_i64(tp + t, 1);
      atomic_add_i64(tn + t, -1);
    } else {
      atomic_add_i64(fp + p, 1);
      atomic_add_i64(fn + t, 1);
      atomic_add_i64(tn + p, -1);
      atomic_add_i64(tn + t, -1);
    }
  }
  __device__ void flush(int* s) {
    const int b0 = base();
    const int lane = threadIdx.x & (kWave - 1);
    const long long v = wave_sum((long long)n_valid);
    const long long wt = micro ? wave_sum((long long)n_tp) : 0;
    const long long wf = micro ? wave_sum((long long)n_fp) : 0;
    if constexpr (use_lds) {
      __shared__ long long s_total;
      __syncthreads();  // every LDS increment of the block is done
      if (lane == 0 && v) atomicAdd(&s[b0], (int)v);
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const int a = s[c], b = s[C + c], d = s[2 * C + c];
        if (a) atomic_add_i64(tp + c, a);
        if (b) atomic_add_i64(fp + c, b);
        if (d) atomic_add_i64(fn + c, d);
        if (a | b | d) atomic_add_i64(tn + c, -(long long)(a + b + d));
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        const long long mine[1] = {s[b0]};
        long long tot[1];
        s_total = grid_sum_last<1>(ticket, mine, tot) ? tot[0] : -1;
      }
      __syncthreads();
      const long long total = s_total;
      if (total > 0)
        for (int c = threadIdx.x; c < C; c += blockDim.x) atomic_add_i64(tn + c, total);
      return;
    }
    // No per-class LDS: no end-of-kernel barrier either (finished waves leave instead of holding their slots at
    // __syncthreads).  Each wave adds its sums to LDS and counts itself done; the block's last wave contributes.
    int done = 0;
    if (lane == 0) {
      if (v) atomicAdd(&s[b0], (int)v);
      if (wt) atomicAdd(&s[b0 + 1], (int)wt);
      if (wf) atomicAdd(&s[b0 + 2], (int)wf);
      done = __hip_atomic_fetch_add(&s[b0 + 3], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    done = __builtin_amdgcn_readfirstlane(done);
    if (done != (int)(blockDim.x / kWave) - 1) return;
    int last = 0;
    long long tot[3] = {0, 0, 0};
    if (lane == 0) {
      if constexpr (micro) {
        const long long mine[3] = {s[b0], s[b0 + 1], s[b0 + 2]};
        last = grid_sum_last<3>(ticket, mine, tot);
      } else {
        const long long mine[1] = {s[b0]};
        long long t1[1];
        last = grid_sum_last<1>(ticket, mine, t1);
        tot[0] = t1[0];
      }
    }
    if (!__builtin_amdgcn_readfirstlane(last)) return;
    if constexpr (micro) {
      if (lane == 0) {
        const long long V = tot[0], T = tot[1], F = tot[2];
        atomic_add_i64(tp, T);
        atomic_add_i64(fp, F);
        atomic_add_i64(fn, F);
        atomic_add_i64(tn, (long long)C * V - T - 2 * F);
      }
    } else {
      const long long total = __shfl(tot[0], 0);
      if (total > 0)
        for (int c = lane; c < C; c += kWave) atomic_add_i64(tn + c, total);
    }
  }
};

struct PairChecks {
  bool bad_t = false, bad_p = false;
  // true when the (target, pred) pair should be accumulated
  __device__ __forceinline__ bool keep(int64_t t, int64_t p, int C, int64_t ignore_index, bool has_ignore) {
    if (p < 0 || p >= C) bad_p = true;
    if (has_ignore && t == ignore_index) return false;
    if (t < 0 || t >= C) {
      bad_t = true;
      return false;
    }
    return p >= 0 && p < C;
  }
  __device__ __forceinline__ void report(int* err_t, int* err_p) const {
    if (bad_t && err_t) atomicOr(err_t, 1);
    if (bad_p && err_p) atomicOr(err_p, 1);
  }
};

template <class Acc>
__global__ void mc_pairs_labels_kernel(const int64_t* __restrict__ preds, const int64_t* __restrict__ target, int64_t n,
                                       int C, int64_t ignore_index, bool has_ignore, Acc acc, int* err_t, int* err_p) {
  extern __shared__ __attribute__((aligned(16))) int s_pairs[];
  acc.init(s_pairs);
  PairChecks chk;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = target[i], p = preds[i];
    if (chk.keep(t, p, C, ignore_index, has_ignore)) acc.add(s_pairs, (int)t, (int)p);
  }
  chk.report(err_t, err_p);
  acc.flush(s_pairs);
}

// one thread per row (small C)
template <typename T, class Acc>
__global__ void mc_pairs_argmax_thread_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n,
                                              int C, int64_t ignore_index, bool has_ignore, Acc acc, int* err_t) {
  extern __shared__ __attribute__((aligned(16))) int s_pairs[];
  acc.init(s_pairs);
  PairChecks chk;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = target[r];
    if (!chk.keep(t, 0, C, ignore_index, has_ignore)) continue;
    const T* row = preds + r * C;
    float best = to_f32<T>(row[0]);
    int bi = 0;
    for (int c = 1; c < C; ++c) {
      float v = to_f32<T>(row[c]);
      if (argmax_better(v, c, best, bi)) { best = v; bi = c; }
    }
    acc.add(s_pairs, (int)t, bi);
  }
  chk.report(err_t, nullptr);
  acc.flush(s_pairs);
}

// one wave per row (large or unaligned C)
template <typename T, class Acc>
__global__ void mc_pairs_argmax_wave_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n,
                                            int C, int64_t ignore_index, bool has_ignore, Acc acc, int* err_t) {
  extern __shared__ __attribute__((aligned(16))) int s_pairs[];
  acc.init(s_pairs);
  PairChecks chk;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t r = wave; r < n; r += nwaves) {
    const int64_t t = target[r];
    if (!chk.keep(t, 0, C, ignore_index, has_ignore)) continue;
    const T* row = preds + r * C;
    float best = -INFINITY;
    int bi = C;  // sentinel larger than any index
    for (int c = lane; c < C; c += kWave) {
      float v = to_f32<T>(row[c]);
      if (argmax_better(v, c, best, bi)) { best = v; bi = c; }
    }
    wave_argmax(best, bi);
    if (lane == 0) acc.add(s_pairs, (int)t, bi);
  }
  chk.report(err_t, nullptr);
  acc.flush(s_pairs);
}

// Vectorised arg-max for aligned rows (C multiple of the 16-B vector width, C <= 64 * VEC * NCH): lane L holds
// classes [VEC * L, VEC * L + VEC) of each 64 * VEC chunk (ascending per lane), every wave keeps 4 rows' 16-B
// loads in flight, NaN-first arg-max semantics of argmax_better / wave_argmax, one pair per row.  (One wave per
// row with scalar 2-B loads: 0.11 ms at 65536 x 1000 bf16.)
template <typename T> struct VecOf { static constexpr int n = 16 / sizeof(T); };

template <typename T> __device__ __forceinline__ float vec_elem(const uint4& w, int k) {
  if constexpr (sizeof(T) == 2) {
    const uint32_t p[4] = {w.x, w.y, w.z, w.w};
    const uint16_t b = (k & 1) ? (p[k >> 1] >> 16) : (p[k >> 1] & 0xFFFFu);
    return to_f32<T>(*reinterpret_cast<const T*>(&b));
  } else if constexpr (sizeof(T) == 4) {
    const uint32_t p[4] = {w.x, w.y, w.z, w.w};
    return __uint_as_float(p[k]);
  } else {
    const uint64_t q = (k == 0) ? ((uint64_t)w.y << 32 | w.x) : ((uint64_t)w.w << 32 | w.z);
    return static_cast<float>(__longlong_as_double(static_cast<long long>(q)));
  }
}

template <typename T, int NCH, class Acc>
__global__ void __launch_bounds__(512) mc_pairs_argmax_vec_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                  int64_t n, int C, int64_t ignore_index, bool has_ignore,
                                                                  Acc acc, int* err_t) {
  constexpr int VEC = VecOf<T>::n;
  constexpr int kRows = 4;
  extern __shared__ __attribute__((aligned(16))) int s_pairs[];
  acc.init(s_pairs);
  PairChecks chk;
  const int lane = threadIdx.x & (kWave - 1);
  const int nvec = C / VEC;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t r0 = wave * kRows; r0 < n; r0 += nwaves * kRows) {
    uint4 w[kRows][NCH];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const uint4* row = reinterpret_cast<const uint4*>(preds + min(r0 + i, n - 1) * C);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int q = lane + kWave * ch;
        w[i][ch] = row[q < nvec ? q : nvec - 1];
      }
    }
    int am[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      // per-chunk max and first position of it; any NaN in the row -> the exact NaN-first shuffle reduction
      float m[NCH];
      int kk[NCH];
      bool nan = false;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const bool active = lane + kWave * ch < nvec;
        float mm = -INFINITY;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const float v = vec_elem<T>(w[i][ch], k);
          nan |= active && v != v;
          mm = __builtin_fmaxf(mm, v);
        }
        int kf = VEC - 1;
#pragma unroll
        for (int k = VEC - 2; k >= 0; --k) kf = vec_elem<T>(w[i][ch], k) == mm ? k : kf;
        m[ch] = active ? mm : -INFINITY;
        kk[ch] = kf;
      }
      if (__ballot(nan)) {
        float best = -INFINITY;
        int bi = C;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int q = lane + kWave * ch;
          if (q >= nvec) continue;
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            const float v = vec_elem<T>(w[i][ch], k);
            const int c = VEC * q + k;
            if (argmax_better(v, c, best, bi)) { best = v; bi = c; }
          }
        }
        wave_argmax(best, bi);
        am[i] = __builtin_amdgcn_readfirstlane(bi);
      } else {
        float mx = m[0];
#pragma unroll
        for (int ch = 1; ch < NCH; ++ch) mx = __builtin_fmaxf(mx, m[ch]);
        mx = wave_max_uniform(mx);
        // lanes own ascending class runs per chunk, so the lowest lane of the first chunk holding the max has the
        // first arg-max (an all -inf row: lane 0, position 0)
        uint64_t b = __ballot(m[0] == mx);
        int ch = 0;
        if constexpr (NCH == 2) {
          if (b == 0) {
            b = __ballot(m[1] == mx);
            ch = 1;
          }
        }
        const int L = __builtin_ctzll(b);
        const int kl = __builtin_amdgcn_readlane(NCH == 2 && ch ? kk[NCH - 1] : kk[0], L);
        am[i] = VEC * (L + kWave * ch) + kl;
      }
    }
    if (lane < kRows) {
      int a = am[0];
#pragma unroll
      for (int i = 1; i < kRows; ++i) a = lane == i ? am[i] : a;
      const int64_t r = r0 + lane;
      if (r < n) {
        const int64_t t = target[r];
        if (chk.keep(t, 0, C, ignore_index, has_ignore)) acc.add(s_pairs, (int)t, a);
      }
    }
  }
  chk.report(err_t, nullptr);
  acc.flush(s_pairs);
}

// Small C (<= 128, any alignment of C): a workgroup streams a contiguous tile of 256 / G rows (tile * C * size
// bytes, a multiple of 16) into LDS with coalesced 16-B loads, then a group of G lanes (C / G <= 16 elements each)
// reduces one row's arg-max from LDS.  Replaces one-thread-per-row scalar loads (20-B stride at C = 10: every load
// instruction touched ten cache lines) and the vector kernel's idle lanes at C = 64 (8 of 64 lanes per row).
template <typename T>
__device__ __forceinline__ void group_argmax(float& v, int& idx, int G) {
  for (int off = 1; off < G; off <<= 1) {
    const float ov = __shfl_xor(v, off, kWave);
    const int oi = __shfl_xor(idx, off, kWave);
    const bool o_nan = ov != ov, s_nan = v != v;
    const bool take = (o_nan && !s_nan) || (o_nan == s_nan && (o_nan ? oi < idx : (ov > v || (ov == v && oi < idx))));
    if (take) { v = ov; idx = oi; }
  }
}

template <typename T, class Acc>
__global__ void __launch_bounds__(1024) mc_pairs_argmax_staged_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                     int64_t n, int C, int glog, int acc_words, int64_t ignore_index,
                                                                     bool has_ignore, Acc acc, int* err_t) {
  extern __shared__ __attribute__((aligned(16))) int s_pairs[];
  acc.init(s_pairs);
  T* s_tile = reinterpret_cast<T*>(s_pairs + acc_words);
  PairChecks chk;
  const int G = 1 << glog;
  const int tile_rows = blockDim.x >> glog;
  const int grp = threadIdx.x >> glog, gl = threadIdx.x & (G - 1);
  const int64_t total_bytes = n * C * (int64_t)sizeof(T);
  const int nchunks = tile_rows * C * (int)sizeof(T) / 16;
  const char* base = reinterpret_cast<const char*>(preds);
  const int64_t ntiles = (n + tile_rows - 1) / tile_rows;
  // each thread moves at most sizeof(T) 16-B chunks per tile (tile <= 16 B x 2048 threads' worth / blockDim); the
  // next tile's chunks and target are loaded into registers while the current tile is reduced from LDS
  constexpr int CH = sizeof(T);
  auto load_chunk = [&](int64_t off) -> uint4 {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (off + 16 <= total_bytes) {
      v = *reinterpret_cast<const uint4*>(base + off);
    } else if (off < total_bytes) {
      // last partial chunk: 16-bit pieces (element sizes are >= 2 B), constant indices so v stays in registers
      const int rem = (int)(total_bytes - off);
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t x = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (4 * j + 2 * h < rem) x |= (uint32_t)*reinterpret_cast<const uint16_t*>(base + off + 4 * j + 2 * h) << (16 * h);
        d[j] = x;
      }
      v = make_uint4(d[0], d[1], d[2], d[3]);
    }
    return v;
  };
  uint4 nxt[CH];
  int64_t t_nxt = 0;
  auto prefetch = [&](int64_t tile) {
    const int64_t off0 = tile * tile_rows * C * (int64_t)sizeof(T);
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int q = threadIdx.x + j * blockDim.x;
      nxt[j] = (q < nchunks && tile < ntiles) ? load_chunk(off0 + 16 * (int64_t)q) : make_uint4(0, 0, 0, 0);
    }
    const int64_t r = tile * tile_rows + grp;
    t_nxt = (gl == 0 && tile < ntiles && r < n) ? target[r] : 0;
  };
  int64_t tile = blockIdx.x;
  if (tile < ntiles) prefetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t r = tile * tile_rows + grp;
    const int64_t t = t_nxt;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int q = threadIdx.x + j * blockDim.x;
      if (q < nchunks) reinterpret_cast<uint4*>(s_tile)[q] = nxt[j];
    }
    __syncthreads();
    prefetch(tile + gridDim.x);
    float best = -INFINITY;
    int bi = C;
    if (r < n) {
      const T* row = s_tile + grp * C;
      for (int c = gl; c < C; c += G) {
        const float v = to_f32<T>(row[c]);
        if (argmax_better(v, c, best, bi)) { best = v; bi = c; }
      }
    }
    group_argmax<T>(best, bi, G);
    if (gl == 0 && r < n && chk.keep(t, 0, C, ignore_index, has_ignore)) acc.add(s_pairs, (int)t, bi);
    __syncthreads();
  }
  chk.report(err_t, nullptr);
  acc.flush(s_pairs);
}

// Dispatch one pair stream.  preds: [N] int64 labels or [N, C] float scores (contiguous).
template <class Acc>
void launch_pairs(const at::Tensor& preds_, const at::Tensor& target, int64_t n, int C, int64_t ignore_index, bool has_ignore,
                  Acc acc, int* err_t, int* err_p) {
  const size_t shm = acc.lds_bytes();
  const int block = 256;
  if (!preds_.is_floating_point()) {
    auto preds = preds_.contiguous().to(at::kLong);
    TORCH_CHECK(preds.numel() == n, "preds/target size mismatch");
    hipLaunchKernelGGL(mc_pairs_labels_kernel<Acc>, grid_for(n, block * 4, 1024), block, shm, stream(), preds.data_ptr<int64_t>(),
                       target.data_ptr<int64_t>(), n, C, ignore_index, has_ignore, acc, err_t, err_p);
    return;
  }
  auto preds = preds_.contiguous();
  TORCH_CHECK(preds.numel() == n * C, "preds must be [N, C] with C classes");
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "mc_pairs", [&] {
    const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
    const int64_t* t = target.data_ptr<int64_t>();
    constexpr int VEC = VecOf<scalar_t>::n;
    const bool aligned = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
    const bool vec_ok = C % VEC == 0 && C > 32 && aligned;
    if (aligned && C <= 128) {
      int glog = 0;
      while ((C + (1 << glog) - 1) >> glog > 16) ++glog;
      const int acc_words = (int)((shm + 15) / 16 * 4);
      // big workgroups (tile <= 16 B x 2048 = 32 KB): 4x fewer per-workgroup flushes than 256 threads
      const int threads = std::min(1024, 2048 / (int)sizeof(scalar_t));
      const int tile_rows = threads >> glog;
      const size_t shm_t = (size_t)acc_words * 4 + (size_t)tile_rows * C * sizeof(scalar_t);
      const int64_t ntiles = (n + tile_rows - 1) / tile_rows;
      const int sgrid = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, std::max<int64_t>(512, ntiles / 2)));
      hipLaunchKernelGGL((mc_pairs_argmax_staged_kernel<scalar_t, Acc>), std::min(sgrid, 2048), threads, shm_t, stream(), p,
                         t, n, C, glog, acc_words, ignore_index, has_ignore, acc, err_t);
    } else if (vec_ok && C <= kWave * VEC) {
      hipLaunchKernelGGL((mc_pairs_argmax_vec_kernel<scalar_t, 1, Acc>), grid_for(n * kWave / 4, 512, 2048), 512, shm,
                         stream(), p, t, n, C, ignore_index, has_ignore, acc, err_t);
    } else if (vec_ok && C <= 2 * kWave * VEC) {
      hipLaunchKernelGGL((mc_pairs_argmax_vec_kernel<scalar_t, 2, Acc>), grid_for(n * kWave / 4, 512, 2048), 512, shm,
                         stream(), p, t, n, C, ignore_index, has_ignore, acc, err_t);
    } else if (C <= 32) {
      hipLaunchKernelGGL((mc_pairs_argmax_thread_kernel<scalar_t, Acc>), grid_for(n, block, 2048), block, shm, stream(), p, t, n,
                         C, ignore_index, has_ignore, acc, err_t);
    } else {
      hipLaunchKernelGGL((mc_pairs_argmax_wave_kernel<scalar_t, Acc>), grid_for(n * kWave, block, 2048), block, shm, stream(), p,
                         t, n, C, ignore_index, has_ignore, acc, err_t);
    }
  });
}

int* flag_ptr(const c10::optional<at::Tensor>& f) {
  if (!f.has_value()) return nullptr;
  TORCH_CHECK(f->scalar_type() == at::kInt && f->numel() >= 1 && f->is_contiguous(), "validation flags must be int32");
  return f->data_ptr<int>();
}

// confmat: int64 [C, C] updated in place.
void mc_confmat_update(const at::Tensor& preds, const at::Tensor& target_, at::Tensor& confmat, int64_t ignore_index,
                       bool has_ignore, const c10::optional<at::Tensor>& err_t, const c10::optional<at::Tensor>& err_p) {
  TORCH_CHECK(confmat.is_contiguous() && confmat.scalar_type() == at::kLong, "confmat must be contiguous int64");
  const int C = static_cast<int>(confmat.size(0));
  auto target = target_.contiguous().to(at::kLong);
  const int64_t n = target.numel();
  if (n == 0) return;
  launch_pairs(preds, target, n, C, ignore_index, has_ignore, ConfmatAcc::make(confmat.data_ptr<int64_t>(), C), flag_ptr(err_t),
               flag_ptr(err_p));
  TMX_LAUNCH_CHECK();
}

// Multiclass stat scores accumulated into the metric states in place: tp / fp / tn / fn int64 [C] (or [1] with
// micro), ticket int64 [1] zero-initialised scratch owned by the caller (returned to zero by every launch).
void mc_stat_scores_update(const at::Tensor& preds, const at::Tensor& target_, int64_t num_classes, at::Tensor& tp,
                           at::Tensor& fp, at::Tensor& tn, at::Tensor& fn, at::Tensor& ticket, int64_t ignore_index,
                           bool has_ignore, bool micro, const c10::optional<at::Tensor>& err_t,
                           const c10::optional<at::Tensor>& err_p) {
  const int64_t want = micro ? 1 : num_classes;
  for (const at::Tensor* s : {&tp, &fp, &tn, &fn})
    TORCH_CHECK(s->is_contiguous() && s->scalar_type() == at::kLong && s->numel() == want, "stat states must be int64 [",
                want, "]");
  TORCH_CHECK(ticket.is_contiguous() && ticket.scalar_type() == at::kLong && ticket.numel() >= kGridSlotsWords,
              "ticket must be a zeroed int64 [", kGridSlotsWords, "] scratch");
  const int C = static_cast<int>(num_classes);
  auto target = target_.contiguous().to(at::kLong);
  const int64_t n = target.numel();
  if (n == 0) return;
  TORCH_CHECK(n < (1ll << 40), "too many rows for one update");
  int64_t* p_tp = tp.data_ptr<int64_t>();
  int64_t* p_fp = fp.data_ptr<int64_t>();
  int64_t* p_tn = tn.data_ptr<int64_t>();
  int64_t* p_fn = fn.data_ptr<int64_t>();
  auto* tk = reinterpret_cast<unsigned long long*>(ticket.data_ptr<int64_t>());
  int* et = flag_ptr(err_t);
  int* ep = flag_ptr(err_p);
  if (micro)
    launch_pairs(preds, target, n, C, ignore_index, has_ignore, StatAcc<kStatMicro>{p_tp, p_fp, p_tn, p_fn, tk, C, 0, 0, 0}, et, ep);
  else if (StatAcc<kStatLds>::lds_fits(C))
    launch_pairs(preds, target, n, C, ignore_index, has_ignore, StatAcc<kStatLds>{p_tp, p_fp, p_tn, p_fn, tk, C, 0, 0, 0}, et, ep);
  else
    launch_pairs(preds, target, n, C, ignore_index, has_ignore, StatAcc<kStatGlobal>{p_tp, p_fp, p_tn, p_fn, tk, C, 0, 0, 0}, et, ep);
  TMX_LAUNCH_CHECK();
}

// =========================================================================================================
// binary / multilabel stat scores: counts[L, 4] = (tp, fp, tn, fn) per label
// preds/target viewed as [N, L, S] (S = flattened extra dims), reduced over N and S.
// =========================================================================================================
template <typename T, bool FLOAT_PREDS>
__global__ void binary_stats_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t N, int L,
                                    int64_t S, float threshold, const int* __restrict__ sigmoid_flag,
                                    int64_t ignore_index, bool has_ignore, int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) int s_cnt[];  // [L][4]
  for (int b = threadIdx.x; b < 4 * L; b += blockDim.x) s_cnt[b] = 0;
  __syncthreads();
  const bool do_sigmoid = FLOAT_PREDS && sigmoid_flag != nullptr && sigmoid_flag[0] != 0;
  const float thr_rt = round_trip<T>(threshold);
  const int64_t total = N * L * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = target[i];
    if (has_ignore && t == ignore_index) continue;
    const int l = static_cast<int>((i / S) % L);
    int p;
    if constexpr (FLOAT_PREDS) {
      float v = to_f32<T>(preds[i]);
      if (do_sigmoid) v = round_trip<T>(1.f / (1.f + expf(-v)));
      p = v > thr_rt ? 1 : 0;
    } else {
      p = static_cast<int>(to_f32<T>(preds[i]) != 0.f);
    }
    // (tp, fp, tn, fn)
    int slot = (t == 1) ? (p ? 0 : 3) : (p ? 1 : 2);
    if (t == 0 || t == 1) atomicAdd(&s_cnt[l * 4 + slot], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < 4 * L; b += blockDim.x) {
    int c = s_cnt[b];
    if (c) atomic_add_i64(counts + b, c);
  }
}

template <bool FLOAT_PREDS>
__global__ void binary_stats_int_kernel(const int64_t* __restrict__ preds, const int64_t* __restrict__ target, int64_t N,
                                        int L, int64_t S, int64_t ignore_index, bool has_ignore, int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) int s_cnt[];
  for (int b = threadIdx.x; b < 4 * L; b += blockDim.x) s_cnt[b] = 0;
  __syncthreads();
  const int64_t total = N * L * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = target[i];
    if (has_ignore && t == ignore_index) continue;
    const int l = static_cast<int>((i / S) % L);
    int p = preds[i] != 0;
    int slot = (t == 1) ? (p ? 0 : 3) : (p ? 1 : 2);
    if (t == 0 || t == 1) atomicAdd(&s_cnt[l * 4 + slot], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < 4 * L; b += blockDim.x) {
    int c = s_cnt[b];
    if (c) atomic_add_i64(counts + b, c);
  }
}

// counts: int64 [L, 4] updated in place.
void binary_stats_update(const at::Tensor& preds_, const at::Tensor& target_, at::Tensor& counts, int64_t num_labels,
                         double threshold, int64_t ignore_index, bool has_ignore) {
  TORCH_CHECK(counts.is_contiguous() && counts.scalar_type() == at::kLong && counts.numel() == 4 * num_labels);
  auto target = target_.contiguous().to(at::kLong);
  const int64_t total = target.numel();
  if (total == 0) return;
  const int64_t N = target.size(0);
  const int L = static_cast<int>(num_labels);
  const int64_t S = total / (N * L);
  TORCH_CHECK(N * L * S == total, "target shape incompatible with num_labels");
  const int block = 256;
  const size_t shm = 4 * L * sizeof(int);
  TORCH_CHECK(shm <= 64 * 1024, "too many labels for binary_stats_update");
  const int grid = grid_for(total, block * 4, 1024);
  if (preds_.is_floating_point()) {
    auto preds = preds_.contiguous();
    auto flag = range_flag(preds);
    TMX_DISPATCH_FLOAT(preds.scalar_type(), "binary_stats_update", [&] {
      hipLaunchKernelGGL((binary_stats_kernel<scalar_t, true>), grid, block, shm, stream(),
                         reinterpret_cast<const scalar_t*>(preds.data_ptr()), target.data_ptr<int64_t>(), N, L, S,
                         (float)threshold, flag.data_ptr<int>(), ignore_index, has_ignore, counts.data_ptr<int64_t>());
    });
  } else {
    auto preds = preds_.contiguous().to(at::kLong);
    hipLaunchKernelGGL((binary_stats_int_kernel<false>), grid, block, shm, stream(), preds.data_ptr<int64_t>(),
                       target.data_ptr<int64_t>(), N, L, S, ignore_index, has_ignore, counts.data_ptr<int64_t>());
  }
  TMX_LAUNCH_CHECK();
}

// =========================================================================================================
// binary / multilabel stat scores in ONE launch, straight into the metric states
// (BinaryStatScores / Accuracy / F1 / ..., Multilabel*; reference stat_scores.py:95-131, 650-681)
//
// The reference decides "sigmoid or not" from the whole batch (any pred outside [0, 1]) before thresholding,
// which used to cost a range-flag pre-pass.  Here every element is thresholded both ways and the workgroups count
// (valid, pos, p_raw, tp_raw, p_sig, tp_sig) per label into a scratch table (L == 1: straight through
// grid_sum_last); the last workgroup reads the table with atomic exchanges (reset in the same op), picks the raw
// or sigmoid counts from the batch-wide out-of-range count, and adds tp / fp / tn / fn into the states.
// Layout: the input is [R, W] with W = L * S columns (label of column j = j / S).  A thread owns one vector of
// VEC consecutive columns for its whole life (grid = nvec * rp threads), so its labels are fixed and its counts
// live in registers; 16-B loads for the scores and for the int64 targets.  L == 1 is a flat stream.
// The value checks of the reference (targets in {0, 1} or ignore_index; label preds in {0, 1}) ride along as
// device flags (deferred validation, utilities/validation.py).
// =========================================================================================================
template <typename T, int N> struct alignas(16) Pack16 { T v[N]; };

struct BinCnt {
  int valid = 0, pos = 0, rp = 0, rtp = 0, sp = 0, stp = 0;
  __device__ void add(int v, int p, int r, int rt, int sg, int st) {
    valid += v; pos += p; rp += r; rtp += rt; sp += sg; stp += st;
  }
  __device__ void get(int (&o)[6]) const { o[0] = valid; o[1] = pos; o[2] = rp; o[3] = rtp; o[4] = sp; o[5] = stp; }
};
// Two 16-bit counts per register (a thread sees < 65536 rows, enforced on the host): the per-column counters of
// the multilabel path are 3 VGPRs per column instead of 6.
struct BinCnt16 {
  uint32_t a = 0, b = 0, c = 0;
  __device__ void add(int v, int p, int r, int rt, int sg, int st) {
    a += (uint32_t)v | ((uint32_t)p << 16); b += (uint32_t)r | ((uint32_t)rt << 16); c += (uint32_t)sg | ((uint32_t)st << 16);
  }
  __device__ void get(int (&o)[6]) const {
    o[0] = a & 0xFFFF; o[1] = a >> 16; o[2] = b & 0xFFFF; o[3] = b >> 16; o[4] = c & 0xFFFF; o[5] = c >> 16;
  }
};

template <typename T> struct BinTraits {
  static constexpr bool kLabel = false;
  using A = float;
  __device__ static A val(T v) { return to_f32<T>(v); }
  __device__ static A sig(A v) { return round_trip<T>(1.f / (1.f + expf(-v))); }
  __device__ static A thr(double t) { return round_trip<T>((float)t); }
};
template <> struct BinTraits<double> {
  static constexpr bool kLabel = false;
  using A = double;
  __device__ static A val(double v) { return v; }
  __device__ static A sig(A v) { return 1.0 / (1.0 + exp(-v)); }
  __device__ static A thr(double t) { return t; }
};
template <> struct BinTraits<int64_t> {
  static constexpr bool kLabel = true;
  using A = int64_t;
  __device__ static A val(int64_t v) { return v; }
  __device__ static A sig(A v) { return v; }
  __device__ static A thr(double) { return 0; }
};

template <typename T, class Cnt>
__device__ __forceinline__ void bin_count(Cnt& c, T x, int64_t t, typename BinTraits<T>::A thr, int64_t ignore_index,
                                          bool has_ignore, bool& oor, bool& bad_t, bool& bad_p) {
  using Tr = BinTraits<T>;
  const auto v = Tr::val(x);
  const bool ign = has_ignore && t == ignore_index;
  const bool tv = t == 0 || t == 1;
  bad_t |= !ign && !tv;
  const int valid = (!ign && tv) ? 1 : 0;
  const int pos = valid & (t == 1 ? 1 : 0);
  int p_raw, p_sig;
  if constexpr (Tr::kLabel) {
    bad_p |= v != 0 && v != 1;
    p_raw = p_sig = v != 0;
  } else {
    oor |= !(v >= 0 && v <= 1);
    p_raw = v > thr;
    p_sig = Tr::sig(v) > thr;
  }
  c.add(valid, pos, valid & p_raw, pos & p_raw, valid & p_sig, pos & p_sig);
}

// Thread mapping: workgroup b = (column group cg = b % cgroups, row group rg = b / cgroups); thread t owns column
// vector cg * CVB + t % CVB and walks rows rg * RL + t / CVB, stepping rgroups * RL (RL = 256 / CVB).  Consecutive
// threads read consecutive 16-B column vectors of a row.  The workgroup's labels are the contiguous range covering
// its columns, so its LDS table and its flush are [nl][6] with nl <= CVB * VEC / S + 1, and a label's scratch row
// receives one flush per row group.  L == 1 is the same mapping with one column vector (a flat stream).
template <typename T, int VEC, bool UNIFORM>
__global__ void __launch_bounds__(256) binary_stats_fused_kernel(
    const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t rows, int nvec, int cvb, int cgroups,
    int64_t rgroups, int64_t tail_start, int64_t total, int L, int64_t S, double threshold, int64_t ignore_index,
    bool has_ignore, int64_t* __restrict__ tp, int64_t* __restrict__ fp, int64_t* __restrict__ tn, int64_t* __restrict__ fn,
    unsigned long long* __restrict__ scratch, int* err_t, int* err_p) {
  extern __shared__ __attribute__((aligned(16))) int s_bin[];  // [nl][6]
  __shared__ int s_oor;
  using Tr = BinTraits<T>;
  const auto thr = Tr::thr(threshold);
  const int cg = (int)(blockIdx.x % cgroups);
  const int64_t rg = blockIdx.x / cgroups;
  const int RL = blockDim.x / cvb;
  const int64_t col_lo = (int64_t)cg * cvb * VEC;
  const int lab_lo = L == 1 ? 0 : (int)(col_lo / S);
  const int lab_hi = L == 1 ? 0 : (int)min<int64_t>(L - 1, (std::min<int64_t>(col_lo + (int64_t)cvb * VEC, (int64_t)nvec * VEC) - 1) / S);
  const int nl = lab_hi - lab_lo + 1;
  for (int b = threadIdx.x; b < 6 * nl; b += blockDim.x) s_bin[b] = 0;
  if (threadIdx.x == 0) s_oor = 0;
  __syncthreads();

  constexpr int NC = UNIFORM ? 1 : VEC;
  using Cnt = std::conditional_t<UNIFORM, BinCnt, BinCnt16>;
  Cnt cnt[NC];
  bool oor = false, bad_t = false, bad_p = false;
  const int cv = cg * cvb + (int)(threadIdx.x % cvb);
  const bool col_ok = cv < nvec && (int)(threadIdx.x / cvb) < RL;
  if (col_ok) {
    using PP = Pack16<T, VEC>;
    using TP = Pack16<int64_t, VEC>;
    auto process = [&](const PP& p, const TP& t) {
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        bin_count<T>(cnt[UNIFORM ? 0 : k], p.v[k], t.v[k], thr, ignore_index, has_ignore, oor, bad_t, bad_p);
    };
    const int64_t step = rgroups * RL;
    int64_t r = rg * RL + threadIdx.x / cvb;
    for (; r + step < rows; r += 2 * step) {
      const int64_t e0 = (r * nvec + cv) * VEC, e1 = ((r + step) * nvec + cv) * VEC;
      const PP p0 = *reinterpret_cast<const PP*>(preds + e0);
      const PP p1 = *reinterpret_cast<const PP*>(preds + e1);
      const TP t0 = *reinterpret_cast<const TP*>(target + e0);
      const TP t1 = *reinterpret_cast<const TP*>(target + e1);
      process(p0, t0);
      process(p1, t1);
    }
    if (r < rows) {
      const int64_t e0 = (r * nvec + cv) * VEC;
      process(*reinterpret_cast<const PP*>(preds + e0), *reinterpret_cast<const TP*>(target + e0));
    }
  }
  // flat-stream tail (L == 1, total not a multiple of VEC)
  if (blockIdx.x == 0 && tail_start + threadIdx.x < total) {
    const int64_t e = tail_start + threadIdx.x;
    bin_count<T>(cnt[0], preds[e], target[e], thr, ignore_index, has_ignore, oor, bad_t, bad_p);
  }
  if (bad_t && err_t) atomicOr(err_t, 1);
  if (bad_p && err_p) atomicOr(err_p, 1);
  if (__ballot(oor) && (threadIdx.x & (kWave - 1)) == 0) s_oor = 1;

  // workgroup reduction.  L == 1: six wave sums -> LDS -> grid_sum_last (no table).  L > 1: the workgroup's
  // [nl][6] LDS table -> scratch[L][6]; grid_sum_last only carries the out-of-range count.
  __shared__ long long s_last[7];
  const bool single = L == 1;
  if (single) {
    int c6[6];
    cnt[0].get(c6);
    int w[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) w[j] = (int)wave_sum((long long)c6[j]);
    if ((threadIdx.x & (kWave - 1)) == 0)
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (w[j]) atomicAdd(&s_bin[j], w[j]);
  } else if (col_ok) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int lab = (int)(((int64_t)cv * VEC + k) / S) - lab_lo;
      int c6[6];
      cnt[k].get(c6);
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (c6[j]) atomicAdd(&s_bin[lab * 6 + j], c6[j]);
    }
  }
  __syncthreads();
  if (!single)
    for (int b = threadIdx.x; b < 6 * nl; b += blockDim.x)
      if (s_bin[b]) atomicAdd(&scratch[lab_lo * 6 + b], (unsigned long long)s_bin[b]);
  __builtin_amdgcn_s_waitcnt(0);  // every thread's table atomics are performed before the workgroup's ticket
  __syncthreads();
  unsigned long long* slots = scratch + (single ? 0 : 6 * (int64_t)L);
  if (threadIdx.x == 0) {
    s_last[6] = -1;
    if (single) {
      const long long mine[7] = {s_bin[0], s_bin[1], s_bin[2], s_bin[3], s_bin[4], s_bin[5], s_oor};
      long long tot[7];
      if (grid_sum_last<7>(slots, mine, tot)) {
#pragma unroll
        for (int j = 0; j < 7; ++j) s_last[j] = tot[j];
      }
    } else {
      const long long mine[1] = {s_oor};
      long long tot[1];
      if (grid_sum_last<1>(slots, mine, tot)) s_last[6] = tot[0];
    }
  }
  __syncthreads();
  if (s_last[6] < 0) return;
  const bool sig = s_last[6] > 0;
  for (int l = threadIdx.x; l < L; l += blockDim.x) {
    long long v[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) v[j] = single ? s_last[j] : (long long)atomicExch(&scratch[l * 6 + j], 0ull);
    const long long ptp = sig ? v[5] : v[3], pp1 = sig ? v[4] : v[2];
    const long long d_fp = pp1 - ptp, d_fn = v[1] - ptp, d_tn = v[0] - v[1] - d_fp;
    if (ptp) atomic_add_i64(tp + l, ptp);
    if (d_fp) atomic_add_i64(fp + l, d_fp);
    if (d_tn) atomic_add_i64(tn + l, d_tn);
    if (d_fn) atomic_add_i64(fn + l, d_fn);
  }
}

template <typename T>
void launch_binary_fused(const T* p, const int64_t* t, int64_t total, int64_t N, int L, int64_t S, double threshold,
                         int64_t ignore_index, bool has_ignore, int64_t* tp, int64_t* fp, int64_t* tn, int64_t* fn,
                         unsigned long long* scratch, int* err_t, int* err_p) {
  constexpr int VEC = 16 / sizeof(T);
  const bool aligned = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(t)) & 15) == 0;
  const int64_t W = (int64_t)L * S;
  const int block = 256;
  auto go = [&](auto vec_c, auto uni_c, int64_t rows, int64_t nvec, int64_t tail_start) {
    constexpr int V = decltype(vec_c)::value;
    constexpr bool U = decltype(uni_c)::value;
    TORCH_CHECK(nvec <= INT32_MAX, "too many columns");
    const int cvb = (int)std::min<int64_t>(nvec, 16);
    const int RL = block / cvb;
    const int64_t cgroups = (nvec + cvb - 1) / cvb;
    TORCH_CHECK(cgroups <= INT32_MAX, "too many column groups");
    // ~1024 workgroups, >= 8 rows per thread when there are that many (fewer table flushes), and fewer than 65536
    // rows per thread for the 16-bit packed counters
    int64_t rgroups = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(1, 1024 / cgroups), rows / ((int64_t)RL * 8)));
    if (L == 1) rgroups = std::max<int64_t>(1, std::min<int64_t>(1024, (rows + RL - 1) / RL));
    rgroups = std::max<int64_t>(rgroups, (rows + (int64_t)RL * 32768 - 1) / ((int64_t)RL * 32768));
    const int64_t grid = cgroups * rgroups;
    TORCH_CHECK(grid <= INT32_MAX, "grid too large");
    const int max_nl = L == 1 ? 1 : (int)std::min<int64_t>(L, (int64_t)cvb * V / S + 2);
    const size_t shm = 6 * (size_t)max_nl * sizeof(int);
    TORCH_CHECK(shm <= 64 * 1024, "label table too large");
    hipLaunchKernelGGL((binary_stats_fused_kernel<T, V, U>), (int)grid, block, shm, stream(), p, t, rows, (int)nvec, cvb,
                       (int)cgroups, rgroups, tail_start, total, L, S, threshold, ignore_index, has_ignore, tp, fp, tn, fn,
                       scratch, err_t, err_p);
  };
  using I1 = std::integral_constant<int, 1>;
  using IV = std::integral_constant<int, VEC>;
  using BT = std::true_type;
  using BF = std::false_type;
  if (L == 1) {
    if (aligned) go(IV{}, BT{}, total / VEC, 1, (total / VEC) * VEC);
    else go(I1{}, BT{}, total, 1, total);
  } else if (aligned && W % VEC == 0) {
    if (S % VEC == 0) go(IV{}, BT{}, N, W / VEC, total);
    else go(IV{}, BF{}, N, W / VEC, total);
  } else {
    go(I1{}, BF{}, N, W, total);
  }
}

// tp / fp / tn / fn: int64 [L] states updated in place; scratch: int64 [6 L + kGridSlotsWords] zeros owned by the
// caller (left at zero by every launch).  preds [N, L, ...] float scores/probabilities or integer labels, target same shape.
void binary_stats_fused(const at::Tensor& preds_, const at::Tensor& target_, at::Tensor& tp, at::Tensor& fp, at::Tensor& tn,
                        at::Tensor& fn, at::Tensor& scratch, int64_t num_labels, double threshold, int64_t ignore_index,
                        bool has_ignore, const c10::optional<at::Tensor>& err_t, const c10::optional<at::Tensor>& err_p) {
  const int L = static_cast<int>(num_labels);
  for (const at::Tensor* s : {&tp, &fp, &tn, &fn})
    TORCH_CHECK(s->is_contiguous() && s->scalar_type() == at::kLong && s->numel() == L, "stat states must be int64 [", L, "]");
  TORCH_CHECK(scratch.is_contiguous() && scratch.scalar_type() == at::kLong &&
                  scratch.numel() >= 6 * (int64_t)L + kGridSlotsWords,
              "scratch must be a zeroed int64 [6 L + ", kGridSlotsWords, "]");
  auto target = target_.contiguous().to(at::kLong);
  const int64_t total = target.numel();
  if (total == 0) return;
  TORCH_CHECK(preds_.numel() == total, "preds/target size mismatch");
  const int64_t N = target.size(0);
  const int64_t S = total / (N * L);
  TORCH_CHECK(N * L * S == total, "target shape incompatible with num_labels");
  auto* sc = reinterpret_cast<unsigned long long*>(scratch.data_ptr<int64_t>());
  int* et = flag_ptr(err_t);
  int* ep = flag_ptr(err_p);
  if (preds_.is_floating_point()) {
    auto preds = preds_.contiguous();
    TMX_DISPATCH_FLOAT(preds.scalar_type(), "binary_stats_fused", [&] {
      launch_binary_fused<scalar_t>(reinterpret_cast<const scalar_t*>(preds.data_ptr()), target.data_ptr<int64_t>(), total, N, L,
                                    S, threshold, ignore_index, has_ignore, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(),
                                    tn.data_ptr<int64_t>(), fn.data_ptr<int64_t>(), sc, et, ep);
    });
  } else {
    auto preds = preds_.contiguous().to(at::kLong);
    launch_binary_fused<int64_t>(preds.data_ptr<int64_t>(), target.data_ptr<int64_t>(), total, N, L, S, threshold,
                                 ignore_index, has_ignore, tp.data_ptr<int64_t>(), fp.data_ptr<int64_t>(), tn.data_ptr<int64_t>(),
                                 fn.data_ptr<int64_t>(), sc, et, ep);
  }
  TMX_LAUNCH_CHECK();
}

// =========================================================================================================
// exact 16-bit score histogram  hist[C][2][kCodes]
// =========================================================================================================
__device__ __forceinline__ void hist_add(int64_t* hist, int64_t c, int label, int code) {
  if (code < 0) return;
  atomic_add_i64(hist + (((c << 1) + label) << kCodeBits) + code, 1);
}

// Multiclass: one wave per row.  Softmax (if flagged) is computed in fp32 and rounded to the input dtype,
// exactly as torch's softmax on a 16-bit tensor stores it; codes are the rounded bit patterns.
// Optionally also accumulates the argmax confusion matrix (fused AUROC + ConfusionMatrix plan).
template <typename T, int VPT>
__global__ void __launch_bounds__(256) curve_hist_mc_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                            int64_t n, int C, const int* __restrict__ softmax_flag,
                                                            int64_t ignore_index, bool has_ignore, int64_t* __restrict__ hist,
                                                            int64_t* __restrict__ confmat, int* __restrict__ err) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  const bool do_softmax = softmax_flag[0] != 0;
  for (int64_t r = wave; r < n; r += nwaves) {
    const int64_t t = target[r];
    if (has_ignore && t == ignore_index) continue;
    if ((t < 0 || t >= C) && err != nullptr && lane == 0) atomicOr(err, 1);
    const T* row = preds + r * C;
    float v[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      int c = lane + j * kWave;
      v[j] = c < C ? to_f32<T>(row[c]) : -INFINITY;
    }
    float m = -INFINITY;
    int am = C;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      int c = lane + j * kWave;
      if (c < C && argmax_better(v[j], c, m, am)) { m = v[j]; am = c; }
    }
    float mx = m;
    int amx = am;
    wave_argmax(mx, amx);
    if (confmat != nullptr && lane == 0 && t >= 0 && t < C && amx < C) atomic_add_i64(confmat + t * C + amx, 1);
    float inv = 1.f;
    if (do_softmax) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        int c = lane + j * kWave;
        if (c < C) { v[j] = expf(v[j] - mx); s += v[j]; }
      }
      s = wave_sum(s);
      inv = s;
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      int c = lane + j * kWave;
      if (c < C) {
        uint16_t b = do_softmax ? round_bits16<T>(v[j] / inv) : bits16<T>(row[c]);
        hist_add(hist, c, c == t ? 1 : 0, score_code<T>(b));
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Small-class row pass (C <= 256): the tile row pass spreads ONE row over a wave (8 classes per lane), so at C = 10
// two lanes of 64 work and a 1M-row update took 0.6 ms.  Here a row gets T = ceil(C / 16) lanes (T in 1..16, at most
// 16 classes per lane) and a block 64 rows (64 T threads):
//   1. the block's rows (64 C contiguous 16-bit scores) are staged into LDS with 16-B loads — no host-side padding
//      copy for C % 8 != 0;
//   2. each lane takes its classes of its row, row statistics by T-lane shuffles: the same rules as row_tile (fp32
//      softmax with expf's instruction sequence and a correctly rounded quotient, RNE to the input dtype; arg-max +
//      confusion matrix; rows with NaN / inf listed for the class pass; probability-mode witness);
//   3. codes go through an LDS image [C][64] to the class-major scratch as 128-B class segments.
// The FIXUP instance redoes the codes of a mis-speculated batch (mode[0] != mode[1]); the class pass is shared.
// ---------------------------------------------------------------------------------------------------------
// The small-class row kernel instance launch_small_rows runs for (TL, C, direct), as a function pointer (occupancy).
template <typename T, bool FIXUP>
static const void* small_rows_kernel(int TL, int C, bool direct) {
#define TMX_SK(...) reinterpret_cast<const void*>(&mc_codes_small_kernel<__VA_ARGS__>)
  if (TL == 1 && C >= 2 && C <= 16) {
    switch (C) {
      case 2: return TMX_SK(T, 1, FIXUP, 2);   case 3: return TMX_SK(T, 1, FIXUP, 3);   case 4: return TMX_SK(T, 1, FIXUP, 4);
      case 5: return TMX_SK(T, 1, FIXUP, 5);   case 6: return TMX_SK(T, 1, FIXUP, 6);   case 7: return TMX_SK(T, 1, FIXUP, 7);
      case 8: return TMX_SK(T, 1, FIXUP, 8);   case 9: return TMX_SK(T, 1, FIXUP, 9);   case 10: return TMX_SK(T, 1, FIXUP, 10);
      case 11: return TMX_SK(T, 1, FIXUP, 11); case 12: return TMX_SK(T, 1, FIXUP, 12); case 13: return TMX_SK(T, 1, FIXUP, 13);
      case 14: return TMX_SK(T, 1, FIXUP, 14); case 15: return TMX_SK(T, 1, FIXUP, 15); default: return TMX_SK(T, 1, FIXUP, 16);
    }
  }
  switch (TL) {
    case 1: return direct ? TMX_SK(T, 1, FIXUP, 0, true) : TMX_SK(T, 1, FIXUP);
    case 2: return direct ? TMX_SK(T, 2, FIXUP, 0, true) : TMX_SK(T, 2, FIXUP);
    case 4: return direct ? TMX_SK(T, 4, FIXUP, 0, true) : TMX_SK(T, 4, FIXUP);
    case 8: return direct ? TMX_SK(T, 8, FIXUP, 0, true) : TMX_SK(T, 8, FIXUP);
    default: return direct ? TMX_SK(T, 16, FIXUP, 0, true) : TMX_SK(T, 16, FIXUP);
  }
#undef TMX_SK
}

// Blocks of the small-class row pass: every resident slot on every CU once (blocks loop over 64-row tiles).  A
// fixed 8192 / TL-block grid left a partial second round at C = 64 (TL = 4: 2048 blocks over 1280 resident slots --
// a third of the chip idle for half the kernel).
template <typename T>
static int small_rows_grid(int TL, int C, bool direct, size_t shm, int64_t ntiles) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, size_t, int>, int> cache;
  const void* k = small_rows_kernel<T, false>(TL, C, direct);
  int dev = 0;
  TMX_CHECK_HIP(hipGetDevice(&dev));
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({k, shm, dev});
    if (it == cache.end()) {
      int nb = 0, cus = 0;
      TMX_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kSmallRows * TL, shm));
      TMX_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      // one lane per row (TL = 1, C <= 16: single-wave blocks): at most 16 blocks per CU -- the 32 resident slots of
      // the occupancy query measured slower (C = 10 / 2 / 16 at 1M rows: 0.043 / 0.047 / 0.052 ms with 4096 blocks
      // against 0.055-0.059 / 0.062 / 0.054 with 8192; tools/small_grid_sweep.sh, profiles/small_class_sweep_r5.json)
      if (TL == 1) nb = std::min(nb, 16);
      it = cache.emplace(std::make_tuple(k, shm, dev), std::max(1, nb) * std::max(1, cus)).first;
    }
    per_cu = it->second;
  }
  static const int grid_cap = [] { const char* v = std::getenv("TMX_SMALL_GRID"); return v ? std::atoi(v) : 0; }();  // A/B knob
  const int64_t want = grid_cap > 0 ? grid_cap / TL : per_cu;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ntiles, want)));
}

template <typename T, bool FIXUP>
void launch_small_rows(int TL, int grid, const T* p, const int64_t* target, int64_t n, int C, int* mode, int64_t ignore_index, bool has_ignore,
                       uint16_t* codes, int64_t n_pad, int64_t* cm, int* err, bool rec, int* srows, int* scount, uint32_t* pcm,
                       float4* row_stats = nullptr) {
  const size_t shm = (size_t)kSmallRows * ((C + 1) & ~1) * sizeof(uint16_t) + (C <= kSmallCmMax ? (size_t)C * C * sizeof(uint32_t) : 0);
  // 16-B aligned rows (C % 8 == 0, aligned base): scores straight into registers, no LDS staging
  const bool direct = C % 8 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
#define TMX_SMALL_CASE(TLV)                                                                                                     \
  case TLV:                                                                                                                      \
    if (direct)                                                                                                                  \
      hipLaunchKernelGGL((mc_codes_small_kernel<T, TLV, FIXUP, 0, true>), grid, kSmallRows * TLV, shm, stream(), p, target, n,  \
                         C, mode, ignore_index, has_ignore, codes, n_pad, cm, err, rec, srows, scount, pcm, row_stats);            \
    else                                                                                                                         \
      hipLaunchKernelGGL((mc_codes_small_kernel<T, TLV, FIXUP>), grid, kSmallRows * TLV, shm, stream(), p, target, n, C, mode, \
                         ignore_index, has_ignore, codes, n_pad, cm, err, rec, srows, scount, pcm, row_stats);                    \
    break;
#define TMX_SMALL_CC(CCV)                                                                                                      \
  case CCV:                                                                                                                      \
    hipLaunchKernelGGL((mc_codes_small_kernel<T, 1, FIXUP, CCV>), grid, kSmallRows, shm, stream(), p, target, n, C, mode,       \
                       ignore_index, has_ignore, codes, n_pad, cm, err, rec, srows, scount, pcm, row_stats);                      \
    break;
  if (TL == 1 && C >= 2 && C <= 16) {  // compile-time class count (no masked value slots)
    switch (C) {
      TMX_SMALL_CC(2) TMX_SMALL_CC(3) TMX_SMALL_CC(4) TMX_SMALL_CC(5) TMX_SMALL_CC(6) TMX_SMALL_CC(7) TMX_SMALL_CC(8) TMX_SMALL_CC(9)
      TMX_SMALL_CC(10) TMX_SMALL_CC(11) TMX_SMALL_CC(12) TMX_SMALL_CC(13) TMX_SMALL_CC(14) TMX_SMALL_CC(15) TMX_SMALL_CC(16)
      default: break;
    }
  } else {
    switch (TL) {
      TMX_SMALL_CASE(1) TMX_SMALL_CASE(2) TMX_SMALL_CASE(4) TMX_SMALL_CASE(8) TMX_SMALL_CASE(16)
      default: TORCH_CHECK(false, "mc_codes_small: unsupported lanes per row");
    }
  }
#undef TMX_SMALL_CC
#undef TMX_SMALL_CASE
  TMX_LAUNCH_CHECK();
}

at::Tensor stream_scratch(const at::TensorOptions& opts, int64_t elems, int kind, bool capturing);
static bool stream_capturing();

// Small-class two-pass route: small row pass (+ FIXUP), then the shared class pass (which finishes rare rows and
// rolls the speculation).  Codes are class-major [C][n_pad], n_pad = 64-row blocks.
template <typename T>
void launch_small_two_pass(const T* p, const int64_t* target, int64_t n, int C, int* mode, int* state, bool speculative,
                           int64_t ignore_index, bool has_ignore, int64_t* hist, int64_t* cm, int* err, const at::TensorOptions& opts,
                           int* code_range, int64_t* batch_hist = nullptr, int* batch_range = nullptr) {
  TORCH_CHECK(n < (int64_t{1} << 31), "curve_hist_update: more than 2^31 rows in one batch");
  const int64_t n_pad = (n + kSmallRows - 1) / kSmallRows * kSmallRows;
  const int64_t ntiles = n_pad / kSmallRows;
  int TL = 1;
  while (TL * kSmallVpt < C) TL *= 2;
  // a block loops over 64-row tiles: ~8-16 waves per CU in flight, and one LDS confusion-matrix flush per block
  // (8192 / TL blocks: up to 32 waves per CU — at 2048 / TL the one-wave blocks of C <= 16 left the CUs at 8 waves and
  // the row pass latency-bound, 40 us for 1M x 10 bf16)
  const size_t shm = (size_t)kSmallRows * ((C + 1) & ~1) * sizeof(uint16_t) + (C <= kSmallCmMax ? (size_t)C * C * sizeof(uint32_t) : 0);
  const int grid = small_rows_grid<T>(TL, C, C % 8 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0, shm, ntiles);
  // class pass: the packed partial-flush pass + reduce launch.  The windowed u32 pass of the headline route
  // (class_hist_hi_kernel; opt-in TMX_SMALL_CLASS_HI=1, C > 16) measured slower here: 127 / 95 / 50 us at C = 64 x 1M,
  // 100 x 262k, 256 x 262k against 51 / 22 / 48 us (few classes concentrate the codes on few bins: LDS atomic
  // contention in its window), gpurun_out r5ar
  static const bool hi_on = std::getenv("TMX_SMALL_CLASS_HI") != nullptr;
  const bool hi_pass = C > 16 && hi_on;
  // confusion-matrix partials per block (C <= 64: at most 16 MiB), summed by a reduce launch: no same-cell atomics
  const bool use_pcm = cm != nullptr && C <= (hi_pass ? kSmallCmMax : 32);
  // per-stream cached scratch (no allocator round trips per update); stream order keeps consecutive updates apart
  const bool capturing = stream_capturing();
  const auto pcm_t = use_pcm ? stream_scratch(opts, (int64_t)grid * C * C, 3, capturing) : at::Tensor();
  uint32_t* pcm = use_pcm ? reinterpret_cast<uint32_t*>(pcm_t.data_ptr()) : nullptr;
  const auto codes = stream_scratch(opts, (int64_t)C * n_pad, 0, capturing);
  const auto slow_rows = stream_scratch(opts, 2 * n, 1, capturing);
  // per-row softmax statistics: a mispredicted batch is refit by the class pass (no FIXUP launch)
  const auto stats = speculative ? stream_scratch(opts, 4 * n, 2, capturing) : at::Tensor();
  float4* rstats = speculative ? reinterpret_cast<float4*>(stats.data_ptr()) : nullptr;
  uint16_t* cptr = reinterpret_cast<uint16_t*>(codes.data_ptr());
  int* srows = slow_rows.data_ptr<int>();
  launch_small_rows<T, false>(TL, grid, p, target, n, C, mode, ignore_index, has_ignore, cptr, n_pad, cm, err, speculative, srows, state,
                              pcm, rstats);
  const int pcm_slices = use_pcm ? std::max(1, std::min(64, grid / 256)) : 0;
  if (hi_pass) {
    // enough (class, split) workgroups for four per CU on every CU; at least 2048 rows per split
    int hsplits = 1;
    while ((int64_t)C * hsplits < 1024 && n_pad / (hsplits * 2) >= 2048) hsplits *= 2;
    hipLaunchKernelGGL((class_hist_hi_kernel<T>), C * hsplits, kClassThreadsU16, kHiLdsBytes, stream(), cptr, n_pad, hsplits, hist, p, C,
                       target, n, mode, speculative, srows, state, cm, code_range, speculative ? mode : nullptr, batch_hist, batch_range,
                       rstats, false);
    TMX_LAUNCH_CHECK();
    if (use_pcm) {
      hipLaunchKernelGGL(class_partial_reduce_kernel, dim3(pcm_slices, C), 256, 0, stream(), nullptr, nullptr, 0, hist, nullptr, nullptr,
                         nullptr, pcm, grid, cm, C, pcm_slices, kCodes / 256 + 1);
      TMX_LAUNCH_CHECK();
    }
    return;
  }
  // Class pass: packed LDS histogram per (class, row split) — with few classes 1 / C of the codes are positives —
  // and a partial flush (plain stores of the occupied range, then one reduce launch) instead of global int64 atomics:
  // every split of a class hits the same few thousand bins.  Splits: enough (class, split) blocks to fill the chip,
  // at least ~8k rows per block (the flush writes up to the occupied range, ~4k words for softmax scores), and at most
  // kClassChunk rows per block so the 16-bit halves never need a mid-stream flush.
  const int64_t nv = n_pad / 8;
  int splits = static_cast<int>(std::max<int64_t>(1, (nv + kClassChunk / 8 - 1) / (kClassChunk / 8)));
  // measured (profiles/small_class_splits_r3.json): the fewest splits the 16-bit halves allow is fastest for every C
  // swept (C = 10, 1M rows: 17 splits 0.065 ms vs 136 splits 0.098 ms); grow only to keep >= 32 blocks for small batches
  while ((int64_t)C * splits < 32 && nv / (splits * 2) >= 1024) splits *= 2;
  static const int forced_splits = [] { const char* v = std::getenv("TMX_SMALL_SPLITS"); return v ? std::atoi(v) : 0; }();
  if (forced_splits > 0) splits = forced_splits;  // experiment knob (tools/mc_small_probe.py sweeps)
  const auto partial = stream_scratch(opts, (int64_t)C * splits * kCodes, 4, capturing);
  const auto prange = stream_scratch(opts, (int64_t)C * splits * 2, 5, capturing);
  uint32_t* pp = reinterpret_cast<uint32_t*>(partial.data_ptr());
  hipLaunchKernelGGL((class_hist_partial_kernel<T>), C * splits, kClassThreads, kCodes * sizeof(uint32_t), stream(), cptr, n_pad, splits,
                     hist, p, C, target, n, mode, speculative, srows, state, cm, code_range, speculative ? mode : nullptr, pp,
                     reinterpret_cast<int*>(prange.data_ptr()), rstats);
  TMX_LAUNCH_CHECK();
  hipLaunchKernelGGL(class_partial_reduce_kernel, dim3(kCodes / 256 + 1 + pcm_slices, C), 256, 0, stream(), pp, prange.data_ptr<int>(),
                     splits, hist, code_range, state, speculative ? mode : nullptr, pcm, grid, cm, C, pcm_slices);
  TMX_LAUNCH_CHECK();
}

// Row pass of the multiclass two-pass route (+ FIXUP and the speculation roll when speculative), into caller-owned
// scratch: ``codes`` int16 [C * n_pad] (class-major), ``slow_rows`` int32 [2 n], ``state`` int32[6] (counts zero).
template <typename T, bool PADDED>
void launch_row_pass(const T* p, const int64_t* target, int64_t n, int C, int ld, int* mode, int* state, bool speculative,
                     int64_t ignore_index, bool has_ignore, int64_t* cm, int* err, uint32_t* cptr, int* srows,
                     bool roll_in_class_pass = false, float4* row_stats = nullptr, PosSink pos = PosSink{}) {
  TORCH_CHECK(n < (int64_t{1} << 31), "curve_hist_update: more than 2^31 rows in one batch");
  const int64_t n_pad = (n + kTileRows - 1) / kTileRows * kTileRows;
  const int64_t ntiles = n_pad / kTileRows;
  const int grid = static_cast<int>((ntiles + 7) / 8 * 8);  // one block per tile (XCD-aware order inside)
  const int fixup_grid = std::min(grid, 128);                // exits at once unless the speculation was wrong
  const size_t shm = (size_t)512 * (C > 512 ? 2 : 1) * kSlots * sizeof(uint32_t);  // 32 / 64 KiB -> 2 blocks per CU
  // with row_stats the class pass refits a mispredicted batch itself: no FIXUP launch
  const bool fixup = speculative && row_stats == nullptr;
  TORCH_CHECK(!fixup || pos.hist == nullptr, "curve row pass: positive booking needs the refit route (row statistics)");
  if (C > 512) {
    hipLaunchKernelGGL((mc_codes_kernel<T, false, 2, PADDED>), grid, kRowThreads, shm, stream(), p, target, n, C, ld, mode, ignore_index,
                       has_ignore, cptr, n_pad, cm, err, speculative, srows, state, row_stats, pos);
    TMX_LAUNCH_CHECK();
    if (fixup) {
      hipLaunchKernelGGL((mc_codes_kernel<T, true, 2, PADDED>), fixup_grid, kRowThreads, shm, stream(), p, target, n, C, ld, mode,
                         ignore_index, has_ignore, cptr, n_pad, cm, err, false, srows, state);
      TMX_LAUNCH_CHECK();
    }
  } else {
    hipLaunchKernelGGL((mc_codes_kernel<T, false, 1, PADDED>), grid, kRowThreads, shm, stream(), p, target, n, C, ld, mode, ignore_index,
                       has_ignore, cptr, n_pad, cm, err, speculative, srows, state, row_stats, pos);
    TMX_LAUNCH_CHECK();
    if (fixup) {
      hipLaunchKernelGGL((mc_codes_kernel<T, true, 1, PADDED>), fixup_grid, kRowThreads, shm, stream(), p, target, n, C, ld, mode,
                         ignore_index, has_ignore, cptr, n_pad, cm, err, false, srows, state);
      TMX_LAUNCH_CHECK();
    }
  }
  if (speculative && !roll_in_class_pass) {
    hipLaunchKernelGGL(mode_roll_kernel, 1, 1, 0, stream(), mode, state + 3);
    TMX_LAUNCH_CHECK();
  }
}

// TMX_CLASS_PASS_U16=1: the round-4 class pass (16-bit-packed LDS bins, positives flagged in the codes) for A/B runs
static bool class_pass_u16() {
  static const bool u16 = [] { const char* v = std::getenv("TMX_CLASS_PASS_U16"); return v != nullptr && v[0] == '1'; }();
  return u16;
}

// Class pass of the multiclass two-pass route.  ``bmode`` = the batch's (used, real) mode pair (state + 3 after a
// speculative row pass, else the pre-pass flag with speculative = false).  ``pos_booked``: the row pass booked the
// positives itself (PosSink) and left their codes skipped.
template <typename T>
void launch_class_pass(const uint32_t* cptr, int64_t n, int C, int ld, const T* p, const int64_t* target, const int* bmode,
                       bool speculative, const int* srows, int* state, int64_t* hist, int64_t* cm, int* code_range,
                       int* roll_mode = nullptr, int64_t* batch_hist = nullptr, int* batch_range = nullptr,
                       const float4* row_stats = nullptr, bool pos_booked = false) {
  const int64_t n_pad = (n + kTileRows - 1) / kTileRows * kTileRows;
  // row splits only when there are too few classes to fill the chip (exclusive-owner flush when splits == 1)
  int splits = 1;
  while ((int64_t)C * splits < 512 && n_pad / (8 * (splits * 2)) >= 1024) splits *= 2;
  // windowed u32 LDS histogram, 512-thread workgroups, four per CU (csrc/curve_hist_kernels.h class_hist_hi_kernel)
  if (!class_pass_u16()) {
    hipLaunchKernelGGL((class_hist_hi_kernel<T>), C * splits, kClassThreadsU16, kHiLdsBytes, stream(),
                       reinterpret_cast<const uint16_t*>(cptr), n_pad, splits, hist, p, ld, target, n, bmode, speculative,
                       srows, state, cm, code_range, roll_mode, batch_hist, batch_range, row_stats, pos_booked);
    TMX_LAUNCH_CHECK();
    return;
  }
  TORCH_CHECK(!pos_booked, "curve class pass: the u16 form needs positives flagged in the codes");
  hipLaunchKernelGGL((class_hist_u16_kernel<T>), C * splits, kClassThreadsU16, kCodes / 2 * sizeof(uint32_t), stream(),
                     reinterpret_cast<const uint16_t*>(cptr), n_pad, splits, hist, p, ld, target, n, bmode, speculative,
                     srows, state, cm, code_range, roll_mode, batch_hist, batch_range, row_stats);
  TMX_LAUNCH_CHECK();
}

// Class-major code scratch of the two-pass route, cached per (device, stream) and grown on demand (never freed).  Taken
// from the caching allocator per update it was re-allocated (hipMalloc, ~200 us of host time) on the first update after
// a compute(), whose temporaries had split the cached block (tools/alloc_probe.py).  Work on one stream is ordered, so
// one buffer per stream is race-free.  Under HIP-graph capture the allocator is used (the graph's private pool).
// ``kind`` 0: int16 class-major codes, 1: int32 rare-row lists, 2: float per-row softmax statistics, 3-5: the
// small-class route's int32 confusion-matrix partials, partial histograms and their ranges (one cache entry per
// (device, stream, kind)).
// ``capturing``: the caller's hipStreamIsCapturing verdict (one runtime query per update, not one per buffer).  The
// returned tensor is the whole cached buffer (no narrow() view per call): callers take its data pointer.
at::Tensor stream_scratch(const at::TensorOptions& opts, int64_t elems, int kind, bool capturing) {
  const auto dt = kind == 0 ? at::kShort : (kind == 2 ? at::kFloat : at::kInt);
  if (capturing) return at::empty({elems}, opts.dtype(dt));
  // At most kMaxScratch (device, stream) entries, least recently used evicted: a buffer goes back to the caching
  // allocator, which only hands it out again on the stream it was allocated on (stream-ordered, so safe).
  constexpr size_t kMaxScratch = 32;
  struct Entry {
    at::Tensor t;
    uint64_t used;
  };
  static std::mutex mu;
  static uint64_t tick = 0;
  static auto* cache = new std::map<std::tuple<int, hipStream_t, int>, Entry>();  // leaked: no teardown-order issue
  std::lock_guard<std::mutex> lock(mu);
  const std::tuple<int, hipStream_t, int> key{static_cast<int>(opts.device().index()), stream(), kind};
  if (cache->find(key) == cache->end() && cache->size() >= kMaxScratch) {
    auto lru = cache->begin();
    for (auto it = cache->begin(); it != cache->end(); ++it)
      if (it->second.used < lru->second.used) lru = it;
    cache->erase(lru);
  }
  Entry& e = (*cache)[key];
  e.used = ++tick;
  if (!e.t.defined() || e.t.numel() < elems) e.t = at::empty({elems}, opts.dtype(dt));
  return e.t;
}

static bool stream_capturing() {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  TMX_CHECK_HIP(hipStreamIsCapturing(stream(), &cap));
  return cap != hipStreamCaptureStatusNone;
}

template <typename T, bool PADDED>
void launch_two_pass(const T* p, const int64_t* target, int64_t n, int C, int ld, int* mode, int* state, bool speculative,
                     int64_t ignore_index, bool has_ignore, int64_t* hist, int64_t* cm, int* err, const at::TensorOptions& opts,
                     int* code_range, int64_t* batch_hist = nullptr, int* batch_range = nullptr) {
  const int64_t n_pad = (n + kTileRows - 1) / kTileRows * kTileRows;
  const bool capturing = stream_capturing();
  const auto codes = stream_scratch(opts, (int64_t)C * n_pad, 0, capturing);
  const auto slow_rows = stream_scratch(opts, 2 * n, 1, capturing);  // written before read (counts live in the state word)
  // per-row softmax statistics (float4 per row, 1 MiB at 65536 rows): the class pass refits a mispredicted batch
  const auto stats = speculative ? stream_scratch(opts, 4 * n, 2, capturing) : at::Tensor();
  float4* rstats = speculative ? reinterpret_cast<float4*>(stats.data_ptr()) : nullptr;
  uint32_t* cptr = reinterpret_cast<uint32_t*>(codes.data_ptr());
  int* srows = slow_rows.data_ptr<int>();
  // single stream: the class pass reads the (used, real) pair straight from ``mode`` and its last workgroup rolls it
  // the row pass books each row's positive itself (class pass: negatives only)
  const bool book = !class_pass_u16() && (rstats != nullptr || !speculative);
  const PosSink pos = book ? PosSink{hist, batch_hist, code_range, batch_range} : PosSink{};
  launch_row_pass<T, PADDED>(p, target, n, C, ld, mode, state, speculative, ignore_index, has_ignore, cm, err, cptr, srows, true, rstats,
                             pos);
  launch_class_pass<T>(cptr, n, C, ld, p, target, mode, speculative, srows, state, hist, cm, code_range, speculative ? mode : nullptr,
                       batch_hist, batch_range, rstats, book);
}

// The row pass alone into caller-owned scratch (class-major codes + rare-row list): the per-element code pin of
// tests/test_ops_gpu.py::test_curve_hist_codes_vs_aten_softmax_same_device reads the codes it writes.
void curve_mc_rowpass(const at::Tensor& preds, const at::Tensor& target, at::Tensor& mode, at::Tensor& state, at::Tensor& codes,
                      at::Tensor& slow_rows, int64_t ignore_index, bool has_ignore, c10::optional<at::Tensor> confmat,
                      c10::optional<at::Tensor> err_flag) {
  TORCH_CHECK(preds.dim() == 2 && preds.is_contiguous() && target.is_contiguous() && target.scalar_type() == at::kLong &&
              target.numel() == preds.size(0), "curve_mc_rowpass: preds [N, C] and int64 target [N], contiguous");
  const int64_t n = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  TORCH_CHECK(C % 8 == 0 && C <= 8 * 2 * kWave && (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0,
              "curve_mc_rowpass: C must be a multiple of 8, <= 1024, preds 16-B aligned");
  const int64_t n_pad = (n + kTileRows - 1) / kTileRows * kTileRows;
  TORCH_CHECK(mode.scalar_type() == at::kInt && mode.numel() == 2 && state.scalar_type() == at::kInt && state.numel() == 6 &&
              codes.scalar_type() == at::kShort && codes.numel() >= (int64_t)C * n_pad && slow_rows.scalar_type() == at::kInt &&
              slow_rows.numel() >= 2 * n, "curve_mc_rowpass: scratch shapes");
  int64_t* cm = nullptr;
  if (confmat.has_value()) {
    TORCH_CHECK(confmat->is_contiguous() && confmat->scalar_type() == at::kLong && confmat->numel() == (int64_t)C * C);
    cm = confmat->data_ptr<int64_t>();
  }
  int* err = err_flag.has_value() ? err_flag->data_ptr<int>() : nullptr;
  if (n == 0) return;
  TMX_DISPATCH_HALF(preds.scalar_type(), "curve_mc_rowpass", [&] {
    launch_row_pass<scalar_t, false>(reinterpret_cast<const scalar_t*>(preds.data_ptr()), target.data_ptr<int64_t>(), n, C, C,
                                     mode.data_ptr<int>(), state.data_ptr<int>(), true, ignore_index, has_ignore, cm, err,
                                     reinterpret_cast<uint32_t*>(codes.data_ptr()), slow_rows.data_ptr<int>());
  });
}

// Binary / multilabel: element-wise (sigmoid if flagged). preds/target viewed as [N, L, S].
template <typename T>
__global__ void curve_hist_ml_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t N, int L,
                                     int64_t S, const int* __restrict__ sigmoid_flag, int64_t ignore_index, bool has_ignore,
                                     int64_t* __restrict__ hist, int* __restrict__ err) {
  const bool do_sigmoid = sigmoid_flag[0] != 0;
  const int64_t total = N * L * S;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = target[i];
    if (has_ignore && t == ignore_index) continue;
    bad |= t != 0 && t != 1;
    const int l = static_cast<int>((i / S) % L);
    uint16_t b;
    if (do_sigmoid) {
      float x = to_f32<T>(preds[i]);
      b = round_bits16<T>(1.f / (1.f + expf(-x)));
    } else {
      b = bits16<T>(preds[i]);
    }
    hist_add(hist, l, t == 1 ? 1 : 0, score_code<T>(b));
  }
  if (bad && err) atomicOr(err, 1);
}

// Binary (single label): one 1024-thread workgroup per CU, a [2][kCodes] u32 histogram privatised in LDS
// (128 KiB), 8 scores + 8 targets per vector step, non-empty bins flushed with one int64 atomic each.  Replaces one
// global 64-bit atomic per score, which for BinaryAUROC lands on a few hundred hot bins of ONE class
// (N = 16.7M bf16: 5.4 ms per update before).  Same sigmoid formula and code rules as curve_hist_ml_kernel.
constexpr int kBinThreads = 1024;

template <typename T>
__device__ __forceinline__ void binary_hist_add(uint32_t* s_h, T p, int64_t t, bool do_sigmoid, int64_t ignore_index,
                                                bool has_ignore, bool& bad) {
  if (has_ignore && t == ignore_index) return;
  bad |= t != 0 && t != 1;
  uint16_t b;
  if (do_sigmoid) {
    const float x = to_f32<T>(p);
    b = round_bits16<T>(1.f / (1.f + expf(-x)));
  } else {
    b = bits16<T>(p);
  }
  const int code = score_code<T>(b);
  if (code < 0) return;
  atomicAdd(&s_h[(t == 1 ? kCodes : 0) + code], 1u);
}

template <typename T>
__global__ void __launch_bounds__(kBinThreads) binary_hist_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                  int64_t total, const int* __restrict__ sigmoid_flag,
                                                                  int64_t ignore_index, bool has_ignore, int64_t* __restrict__ hist,
                                                                  int* __restrict__ err, int* __restrict__ code_range = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // [2][kCodes]: negatives, positives
  bool bad = false;
  uint4* s4 = reinterpret_cast<uint4*>(s_h);
  for (int i = threadIdx.x; i < 2 * kCodes / 4; i += kBinThreads) s4[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const bool do_sigmoid = sigmoid_flag[0] != 0;
  const int64_t nvec = total / 8;
  const uint4* pv = reinterpret_cast<const uint4*>(preds);
  const longlong2* tv = reinterpret_cast<const longlong2*>(target);
  const int64_t stride = (int64_t)gridDim.x * kBinThreads;
  for (int64_t v = blockIdx.x * (int64_t)kBinThreads + threadIdx.x; v < nvec; v += stride) {
    const uint4 w = pv[v];
    longlong2 tt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tt[k] = tv[4 * v + k];
    const uint32_t parts[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint16_t bits = static_cast<uint16_t>((k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu));
      const int64_t t = (k & 1) ? tt[k >> 1].y : tt[k >> 1].x;
      binary_hist_add<T>(s_h, *reinterpret_cast<const T*>(&bits), t, do_sigmoid, ignore_index, has_ignore, bad);
    }
  }
  if (blockIdx.x == 0) {  // tail
    for (int64_t i = nvec * 8 + threadIdx.x; i < total; i += kBinThreads)
      binary_hist_add<T>(s_h, preds[i], target[i], do_sigmoid, ignore_index, has_ignore, bad);
  }
  if (bad && err) atomicOr(err, 1);
  __syncthreads();
  int lo = kCodes, hi = -1;  // occupied code range (compute() reads only [lo, hi]): tracked here, no host-side fill
  for (int i = threadIdx.x; i < 2 * kCodes; i += kBinThreads) {
    const uint32_t cnt = s_h[i];
    if (cnt) {
      atomic_add_i64(hist + i, cnt);
      const int b = i & (kCodes - 1);
      lo = min(lo, b);
      hi = max(hi, b);
    }
  }
  if (code_range != nullptr) {
    lo = wave_min_i32(lo);
    hi = wave_max_i32(hi);
    if ((threadIdx.x & (kWave - 1)) == 0 && hi >= 0) {
      atomicMin(code_range, lo);
      atomicMax(code_range + 1, hi);
    }
  }
}

// hist: int64 [C, 2, kCodes] updated in place.
// task 0 = multiclass (preds [N, C], target [N]); task 1 = binary/multilabel (preds/target [N, L, ...]).
void curve_hist_merge_launch(int64_t* dst, int* dst_range, const int64_t* src, const int* src_range, int C);

// ``batch_hist`` / ``batch_range`` (optional, forward()): the batch's own histogram and code range, zero / empty before
// the call, are produced beside the accumulated ones.  The two-pass routes flush both from the class pass; every other
// route counts into the batch histogram and one merge launch adds its occupied range into ``hist``.
void curve_hist_update_impl(const at::Tensor& preds_, const at::Tensor& target_, at::Tensor& hist, int64_t task, int64_t ignore_index,
                            bool has_ignore, c10::optional<at::Tensor> confmat, c10::optional<at::Tensor> norm_flag,
                            c10::optional<at::Tensor> err_flag, c10::optional<at::Tensor> mode_state, c10::optional<at::Tensor> code_range,
                            int64_t* batch_hist, int* batch_range, bool& dual);

void curve_hist_update(const at::Tensor& preds_, const at::Tensor& target_, at::Tensor& hist, int64_t task,
                       int64_t ignore_index, bool has_ignore, c10::optional<at::Tensor> confmat,
                       c10::optional<at::Tensor> norm_flag, c10::optional<at::Tensor> err_flag,
                       c10::optional<at::Tensor> mode_state, c10::optional<at::Tensor> code_range,
                       c10::optional<at::Tensor> batch_hist, c10::optional<at::Tensor> batch_range) {
  TORCH_CHECK(hist.is_contiguous() && hist.scalar_type() == at::kLong && hist.dim() == 3 && hist.size(1) == 2 &&
              hist.size(2) == kCodes, "hist must be int64 [C, 2, 16384]");
  if (!batch_hist.has_value()) {
    bool dual = false;
    curve_hist_update_impl(preds_, target_, hist, task, ignore_index, has_ignore, confmat, norm_flag, err_flag, mode_state, code_range,
                           nullptr, nullptr, dual);
    return;
  }
  TORCH_CHECK(batch_range.has_value(), "curve_hist_update: batch_hist needs batch_range");
  TORCH_CHECK(batch_hist->is_contiguous() && batch_hist->sizes() == hist.sizes() && batch_hist->scalar_type() == at::kLong &&
              batch_hist->device() == hist.device(), "batch_hist must be int64 like hist");
  TORCH_CHECK(batch_range->scalar_type() == at::kInt && batch_range->numel() == 2 * hist.size(0) && batch_range->is_contiguous() &&
              batch_range->device() == hist.device(), "batch_range must be int32[C, 2] on the histogram's device");
  // dual-flush routes write both histograms; the others are run on the batch histogram (+ its range) and merged
  bool dual = true;
  curve_hist_update_impl(preds_, target_, hist, task, ignore_index, has_ignore, confmat, norm_flag, err_flag, mode_state, code_range,
                         batch_hist->data_ptr<int64_t>(), batch_range->data_ptr<int>(), dual);
  if (!dual) {
    curve_hist_update_impl(preds_, target_, *batch_hist, task, ignore_index, has_ignore, confmat, norm_flag, err_flag, mode_state,
                           batch_range, nullptr, nullptr, dual);
    curve_hist_merge_launch(hist.data_ptr<int64_t>(), code_range.has_value() ? code_range->data_ptr<int>() : nullptr,
                            batch_hist->data_ptr<int64_t>(), batch_range->data_ptr<int>(), static_cast<int>(hist.size(0)));
  }
}

// ``dual`` in: the caller asks for the batch histogram (batch_hist / batch_range non-null); out: false when this route
// cannot write it and nothing was done (the caller reruns on the batch histogram and merges).
void curve_hist_update_impl(const at::Tensor& preds_, const at::Tensor& target_, at::Tensor& hist, int64_t task, int64_t ignore_index,
                            bool has_ignore, c10::optional<at::Tensor> confmat, c10::optional<at::Tensor> norm_flag,
                            c10::optional<at::Tensor> err_flag, c10::optional<at::Tensor> mode_state, c10::optional<at::Tensor> code_range,
                            int64_t* batch_hist, int* batch_range, bool& dual) {
  // code_range (int32[C, 2], optional): the occupied code range [lo, hi] of each class of ``hist``.  The two-pass routes widen it
  // in the class pass; every other route (rare shapes) marks it as the full range, so it is always conservative.
  int* crange = nullptr;
  bool range_tracked = false;
  if (code_range.has_value()) {
    TORCH_CHECK(code_range->scalar_type() == at::kInt && code_range->numel() == 2 * hist.size(0) && code_range->is_contiguous() &&
                code_range->device() == hist.device(), "code_range must be int32[C, 2] on the histogram's device");
    crange = code_range->data_ptr<int>();
  }
  struct RangeGuard {  // on exit, routes that did not track the range widen it to everything
    c10::optional<at::Tensor>& r; bool& tracked;
    ~RangeGuard() {
      if (r.has_value() && !tracked) {
        auto v = r->view({-1, 2});
        v.select(1, 0).fill_(0);
        v.select(1, 1).fill_(kCodes - 1);
      }
    }
  } range_guard{code_range, range_tracked};
  // no dispatcher round trips for inputs that are already contiguous int64 (the hot path: ~1 us of host time each)
  const at::Tensor preds = preds_.is_contiguous() ? preds_ : preds_.contiguous();
  const at::Tensor target = target_.is_contiguous() && target_.scalar_type() == at::kLong ? target_ : target_.contiguous().to(at::kLong);
  const int C = static_cast<int>(hist.size(0));
  const int block = 256;
  // two-pass multiclass route for C <= 1024 (C % 8 != 0: rows read in place at stride C, unaligned loads)
  const bool two_pass_ok = task == 0 && C <= 8 * 2 * kWave &&
                           (C % 8 != 0 || (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0);
  if (batch_hist != nullptr) {
    static const bool small_off_b = std::getenv("TMX_CURVE_SMALL_OFF") != nullptr;
    const bool small_route = task == 0 && !small_off_b && C <= kSmallVpt * 16 && (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0;
    // the small route's windowed class pass (C > 16) fills the batch histogram too
    static const bool small_hi = std::getenv("TMX_SMALL_CLASS_HI") != nullptr;
    const bool small_dual = small_route && C > 16 && small_hi;
    const bool ml_route = task == 1 && C != 1 && C % 8 == 0 && C <= 8 * 2 * kWave && target.dim() >= 1 && target.numel() == target.size(0) * C &&
                          (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(target.data_ptr()) & 15) == 0;
    const bool dual_route = (task == 0 && two_pass_ok && !small_route) || small_dual || ml_route;
    if (!dual_route) {
      dual = false;
      range_tracked = true;  // nothing counted: the range stays as it is
      return;
    }
  }
  // speculative normalisation mode (persistent int32[8] per metric: mode[2], rare-row counts[2], ticket) replaces the
  // range pre-pass; the class pass leaves the counts at zero for the next batch
  const bool speculative = two_pass_ok && mode_state.has_value() && !norm_flag.has_value();
  at::Tensor flag, state;
  int* state_ptr = nullptr;
  if (speculative) {
    TORCH_CHECK(mode_state->scalar_type() == at::kInt && mode_state->numel() >= 8 && mode_state->is_contiguous(),
                "mode_state must be int32[>= 8]");
    flag = *mode_state;
    state_ptr = mode_state->data_ptr<int>() + 2;  // [2:8] of the persistent word (no narrow() view per call)
  } else {
    flag = norm_flag.has_value() ? norm_flag->to(at::kInt).contiguous() : range_flag(preds);
    if (two_pass_ok) {
      state = at::zeros({6}, preds.options().dtype(at::kInt));
      state_ptr = state.data_ptr<int>();
    }
  }
  int64_t* cm = nullptr;
  if (confmat.has_value()) {
    TORCH_CHECK(confmat->is_contiguous() && confmat->scalar_type() == at::kLong && confmat->numel() == (int64_t)C * C);
    cm = confmat->data_ptr<int64_t>();
  }
  int* err = nullptr;
  if (err_flag.has_value()) {
    TORCH_CHECK(err_flag->scalar_type() == at::kInt && err_flag->is_contiguous(), "err_flag must be int32");
    err = err_flag->data_ptr<int>();
  }
  TMX_DISPATCH_HALF(preds.scalar_type(), "curve_hist_update", [&] {
    const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
    if (task == 0) {
      const int64_t n = target.numel();
      if (n == 0) { range_tracked = true; return; }
      TORCH_CHECK(preds.numel() == n * C, "preds must be [N, C]");
      static const bool small_off = std::getenv("TMX_CURVE_SMALL_OFF") != nullptr;  // A/B against the tile row pass
      const bool small_ok = !small_off && C <= kSmallVpt * 16 && (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0;
      if (small_ok) {
        launch_small_two_pass<scalar_t>(p, target.data_ptr<int64_t>(), n, C, flag.data_ptr<int>(), state_ptr, speculative,
                                        ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err, preds.options(), crange,
                                        batch_hist, batch_range);
        range_tracked = true;
        return;
      }
      if (two_pass_ok) {
        if (C % 8 != 0) {
          // rows at stride C read in place with 2-byte-aligned 16-B loads (row_tile_load UNALIGNED); round 4 padded
          // every row to a multiple of 8 with a copy (48 us + 18 us of fill at 65,536 x 1001)
          launch_two_pass<scalar_t, true>(p, target.data_ptr<int64_t>(), n, C, C, flag.data_ptr<int>(), state_ptr, speculative,
                                          ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err, preds.options(), crange, batch_hist,
                                          batch_range);
        } else {
          launch_two_pass<scalar_t, false>(p, target.data_ptr<int64_t>(), n, C, C, flag.data_ptr<int>(), state_ptr,
                                           speculative, ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err, preds.options(),
                                           crange, batch_hist, batch_range);
        }
        range_tracked = true;
        return;
      }
      const int grid = grid_for(n * kWave, block, 4096);
      if (C <= 64 * 4) {
        hipLaunchKernelGGL((curve_hist_mc_kernel<scalar_t, 4>), grid, block, 0, stream(), p, target.data_ptr<int64_t>(), n, C,
                           flag.data_ptr<int>(), ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err);
      } else if (C <= 64 * 16) {
        hipLaunchKernelGGL((curve_hist_mc_kernel<scalar_t, 16>), grid, block, 0, stream(), p, target.data_ptr<int64_t>(), n, C,
                           flag.data_ptr<int>(), ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err);
      } else {
        TORCH_CHECK(C <= 64 * 64, "curve_hist_update: num_classes > 4096 not supported by the exact histogram path");
        hipLaunchKernelGGL((curve_hist_mc_kernel<scalar_t, 64>), grid, block, 0, stream(), p, target.data_ptr<int64_t>(), n, C,
                           flag.data_ptr<int>(), ignore_index, has_ignore, hist.data_ptr<int64_t>(), cm, err);
      }
    } else {
      const int64_t total = target.numel();
      if (total == 0) { range_tracked = true; return; }
      TORCH_CHECK(preds.numel() == total, "preds/target size mismatch");
      const int64_t N = target.size(0);
      const int64_t S = total / (N * C);
      TORCH_CHECK(N * C * S == total, "target shape incompatible with num_labels");
      const bool aligned = (reinterpret_cast<uintptr_t>(preds.data_ptr()) & 15) == 0 &&
                           (reinterpret_cast<uintptr_t>(target.data_ptr()) & 15) == 0;
      if (C == 1 && aligned) {
        static const bool lds_ok = [] {  // > 64 KiB of dynamic LDS needs the attribute (gfx950 has 160 KiB per CU)
          return hipFuncSetAttribute(reinterpret_cast<const void*>(binary_hist_kernel<scalar_t>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kCodes * sizeof(uint32_t)) == hipSuccess;
        }();
        TORCH_CHECK(lds_ok, "binary_hist_kernel: cannot reserve 128 KiB of LDS");
        const int grid = static_cast<int>(std::min<int64_t>(256, (total + 8 * kBinThreads - 1) / (8 * kBinThreads)));
        hipLaunchKernelGGL(binary_hist_kernel<scalar_t>, std::max(grid, 1), kBinThreads, 2 * kCodes * sizeof(uint32_t), stream(), p,
                           target.data_ptr<int64_t>(), total, flag.data_ptr<int>(), ignore_index, has_ignore,
                           hist.data_ptr<int64_t>(), err, crange);
        range_tracked = crange != nullptr;
        return;
      }
      if (S == 1 && C % 8 == 0 && C <= 8 * 2 * kWave && aligned) {
        // multilabel: the multiclass two-pass layout (labels as classes), per-element targets and sigmoid
        const int64_t n_pad = (N + kTileRows - 1) / kTileRows * kTileRows;
        auto codes = at::empty({(int64_t)C * n_pad}, preds.options().dtype(at::kShort));
        auto state = at::zeros({6}, preds.options().dtype(at::kInt));
        const int grid = static_cast<int>((n_pad / kTileRows + 7) / 8 * 8);
        const size_t shm = (size_t)512 * (C > 512 ? 2 : 1) * kSlots * sizeof(uint32_t);
        uint32_t* cptr = reinterpret_cast<uint32_t*>(codes.data_ptr());
        if (C > 512)
          hipLaunchKernelGGL((ml_codes_kernel<scalar_t, 2>), grid, kRowThreads, shm, stream(), p, target.data_ptr<int64_t>(), N, C,
                             flag.data_ptr<int>(), ignore_index, has_ignore, cptr, n_pad, err);
        else
          hipLaunchKernelGGL((ml_codes_kernel<scalar_t, 1>), grid, kRowThreads, shm, stream(), p, target.data_ptr<int64_t>(), N, C,
                             flag.data_ptr<int>(), ignore_index, has_ignore, cptr, n_pad, err);
        TMX_LAUNCH_CHECK();
        int splits = 1;
        while ((int64_t)C * splits < 512 && n_pad / (8 * (splits * 2)) >= 1024) splits *= 2;
        hipLaunchKernelGGL((class_hist_kernel<scalar_t, true>), C * splits, kClassThreads, kCodes * sizeof(uint32_t), stream(),
                           reinterpret_cast<const uint16_t*>(cptr), n_pad, splits, hist.data_ptr<int64_t>(), p, C,
                           target.data_ptr<int64_t>(), N, flag.data_ptr<int>(), false, static_cast<const int*>(nullptr),
                           state.data_ptr<int>(), static_cast<int64_t*>(nullptr), crange, static_cast<int*>(nullptr), batch_hist,
                           batch_range);
        range_tracked = true;
        return;
      }
      hipLaunchKernelGGL(curve_hist_ml_kernel<scalar_t>, grid_for(total, block, 4096), block, 0, stream(), p,
                         target.data_ptr<int64_t>(), N, C, S, flag.data_ptr<int>(), ignore_index, has_ignore,
                         hist.data_ptr<int64_t>(), err);
    }
  });
  TMX_LAUNCH_CHECK();
}

// forward()'s batch histogram: ``dst[c, :, lo..hi] += src[c, :, lo..hi]`` over the source's occupied range per class
// (and the destination range widened), or -- curve_hist_zero -- ``src`` zeroed over that range and the range emptied,
// so the scratch is ready for the next batch, or -- curve_hist_drain -- both in one pass (the update lanes' join).
// One 256-thread workgroup per (class, 4096-code slice): grid.y slices.
constexpr int kMergeThreads = 256;
constexpr int kMergeSlice = 4096;
__global__ void __launch_bounds__(kMergeThreads) curve_hist_merge_kernel(int64_t* __restrict__ dst, int* __restrict__ dst_range,
                                                                         int64_t* __restrict__ src, int* __restrict__ src_range, bool zero) {
  const int c = blockIdx.x;
  const int lo = max(src_range[2 * c], 0), hi = min(src_range[2 * c + 1], kCodes - 1);
  const int s0 = lo + blockIdx.y * kMergeSlice, s1 = min(hi + 1, s0 + kMergeSlice);
  for (int h = 0; h < 2; ++h) {
    int64_t* sp = src + ((int64_t)c * 2 + h) * kCodes;
    int64_t* dp = dst != nullptr ? dst + ((int64_t)c * 2 + h) * kCodes : nullptr;
    for (int i = s0 + threadIdx.x; i < s1; i += kMergeThreads) {
      const int64_t v = sp[i];
      if (v == 0) continue;
      if (dp != nullptr) dp[i] += v;
      if (zero) sp[i] = 0;
    }
  }
  if (blockIdx.y == 0 && threadIdx.x == 0 && hi >= lo) {
    if (dst_range != nullptr) {
      atomicMin(dst_range + 2 * c, lo);
      atomicMax(dst_range + 2 * c + 1, hi);
    }
  }
}

__global__ void curve_range_reset_kernel(int* __restrict__ range, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    range[2 * c] = kCodes;
    range[2 * c + 1] = -1;
  }
}

void curve_hist_merge_launch(int64_t* dst, int* dst_range, const int64_t* src, const int* src_range, int C) {
  if (C == 0) return;
  hipLaunchKernelGGL(curve_hist_merge_kernel, dim3(C, kCodes / kMergeSlice), kMergeThreads, 0, stream(), dst, dst_range,
                     const_cast<int64_t*>(src), const_cast<int*>(src_range), false);
  TMX_LAUNCH_CHECK();
}

void curve_hist_zero(at::Tensor& src, at::Tensor& src_range) {
  TORCH_CHECK(src.is_contiguous() && src.scalar_type() == at::kLong && src.dim() == 3 && src.size(1) == 2 && src.size(2) == kCodes,
              "curve_hist_zero: hist must be int64 [C, 2, 16384]");
  TORCH_CHECK(src_range.scalar_type() == at::kInt && src_range.numel() == 2 * src.size(0) && src_range.is_contiguous() &&
              src_range.device() == src.device(), "curve_hist_zero: range must be int32[C, 2] on the histogram's device");
  const int C = static_cast<int>(src.size(0));
  if (C == 0) return;
  hipLaunchKernelGGL(curve_hist_merge_kernel, dim3(C, kCodes / kMergeSlice), kMergeThreads, 0, stream(), static_cast<int64_t*>(nullptr),
                     static_cast<int*>(nullptr), src.data_ptr<int64_t>(), src_range.data_ptr<int>(), true);
  TMX_LAUNCH_CHECK();
  hipLaunchKernelGGL(curve_range_reset_kernel, (C + 255) / 256, 256, 0, stream(), src_range.data_ptr<int>(), C);
  TMX_LAUNCH_CHECK();
}

// The update lanes' join (classification/precision_recall_curve.py ``_join_lanes``): ``src`` (lane 1's histogram) added
// into ``dst`` (the metric's) over src's occupied range per class, dst's range widened, src zeroed and its range emptied.
void curve_hist_drain(at::Tensor& dst, at::Tensor& dst_range, at::Tensor& src, at::Tensor& src_range) {
  TORCH_CHECK(src.is_contiguous() && src.scalar_type() == at::kLong && src.dim() == 3 && src.size(1) == 2 && src.size(2) == kCodes &&
              dst.is_contiguous() && dst.sizes() == src.sizes() && dst.scalar_type() == at::kLong && dst.device() == src.device(),
              "curve_hist_drain: two int64 [C, 2, 16384] histograms on one device");
  for (const at::Tensor* r : {&src_range, &dst_range})
    TORCH_CHECK(r->scalar_type() == at::kInt && r->numel() == 2 * src.size(0) && r->is_contiguous() && r->device() == src.device(),
                "curve_hist_drain: ranges must be int32[C, 2] on the histograms' device");
  const int C = static_cast<int>(src.size(0));
  if (C == 0) return;
  hipLaunchKernelGGL(curve_hist_merge_kernel, dim3(C, kCodes / kMergeSlice), kMergeThreads, 0, stream(), dst.data_ptr<int64_t>(),
                     dst_range.data_ptr<int>(), src.data_ptr<int64_t>(), src_range.data_ptr<int>(), true);
  TMX_LAUNCH_CHECK();
  hipLaunchKernelGGL(curve_range_reset_kernel, (C + 255) / 256, 256, 0, stream(), src_range.data_ptr<int>(), C);
  TMX_LAUNCH_CHECK();
}

// Per-class reduction of the exact histogram (descending code order), one 256-thread workgroup per class.
//   out[c] = {auroc, average_precision, n_pos, n_neg}
// AUROC = sum_k neg_k * (2*TP_{<k} + pos_k) / (2 * P * N)  (trapezoid over every code; empty codes add 0)
// AP    = sum_k (pos_k / P) * TP_k / (TP_k + FP_k)
// Only the class's occupied code range [lo, hi] (``code_range[c]``, tracked by the class pass) is read, in chunks of 4096 codes
// from the top: thread t owns the 16 consecutive codes of its 128-B aligned segment (two 16-B loads per 32 B of each
// half), one block scan of the per-thread sums gives every thread its TP / FP carry, then each walks its codes.
// Softmax scores of 1000 classes occupy ~3000 codes: one chunk, 53 MB read instead of 262 MB, and 4 small
// workgroups per CU keep every class resident at once (the previous 1024-thread, full-range form took 105 us).
constexpr int kRedThreads = 256;
constexpr int kRedPer = 16;
constexpr int kRedChunk = kRedThreads * kRedPer;

__device__ __forceinline__ long long shfl_up_i64(long long v, int off) {
  int lo = __shfl_up(static_cast<int>(v & 0xFFFFFFFFll), off, kWave);
  int hi = __shfl_up(static_cast<int>(v >> 32), off, kWave);
  return (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo);
}

// CLEAR (forward()'s batch histogram, round 6): every read segment is zeroed behind the read and the class's range
// emptied, so the scratch is ready for the next batch without the separate zero + range-reset launches.
__device__ __forceinline__ void curve_summary_block(const double* __restrict__ sc, int C, double* __restrict__ summary);

template <bool CLEAR = false>
__global__ void __launch_bounds__(kRedThreads) curve_hist_reduce_kernel(const int64_t* __restrict__ hist,
                                                                         const int* __restrict__ code_range,
                                                                         double* __restrict__ out, int* __restrict__ done = nullptr,
                                                                         double* __restrict__ summary = nullptr) {
  constexpr int K = kCodes;
  constexpr int kWaves = kRedThreads / kWave;
  const int c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  int lo = 0, hi = K - 1;
  if (code_range != nullptr) {
    lo = max(code_range[2 * c], 0);
    hi = min(code_range[2 * c + 1], K - 1);
  }
  const int64_t* negh = hist + ((int64_t)c * 2 + 0) * K;
  const int64_t* posh = hist + ((int64_t)c * 2 + 1) * K;
  __shared__ long long s_p[kWaves], s_n[kWaves];
  __shared__ double s_a[kWaves], s_b[kWaves];
  long long carry_p = 0, carry_n = 0;
  double area = 0.0, ap_sum = 0.0;
  if (hi >= lo) {
    const int top = hi | (kRedPer - 1), bottom = lo & ~(kRedPer - 1);  // segment-aligned, still inside [0, K)
    for (int chunk_top = top; chunk_top >= bottom; chunk_top -= kRedChunk) {
      const int seg_hi = chunk_top - kRedPer * tid;
      long long p[kRedPer], n[kRedPer];  // index i = i-th highest owned code
      if (seg_hi >= bottom) {
        const longlong2* negv = reinterpret_cast<const longlong2*>(negh + (seg_hi - (kRedPer - 1)));
        const longlong2* posv = reinterpret_cast<const longlong2*>(posh + (seg_hi - (kRedPer - 1)));
#pragma unroll
        for (int v = 0; v < kRedPer / 2; ++v) {
          const longlong2 a = posv[v], b = negv[v];
          p[kRedPer - 1 - 2 * v] = a.x; p[kRedPer - 2 - 2 * v] = a.y;
          n[kRedPer - 1 - 2 * v] = b.x; n[kRedPer - 2 - 2 * v] = b.y;
        }
        if constexpr (CLEAR) {  // (codes of the aligned segment outside [lo, hi] are zero already)
          longlong2* pw = const_cast<longlong2*>(posv);
          longlong2* nw = const_cast<longlong2*>(negv);
#pragma unroll
          for (int v = 0; v < kRedPer / 2; ++v) {
            pw[v] = make_longlong2(0, 0);
            nw[v] = make_longlong2(0, 0);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < kRedPer; ++i) p[i] = n[i] = 0;
      }
      long long sp = 0, sn = 0;
#pragma unroll
      for (int i = 0; i < kRedPer; ++i) { sp += p[i]; sn += n[i]; }
      long long ip = sp, in = sn;  // inclusive wave scan in thread order (= descending code order)
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const long long tp = shfl_up_i64(ip, off), tn = shfl_up_i64(in, off);
        if (lane >= off) { ip += tp; in += tn; }
      }
      if (lane == kWave - 1) { s_p[wave] = ip; s_n[wave] = in; }
      __syncthreads();
      long long wp = 0, wn = 0, bp = 0, bn = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        if (w < wave) { wp += s_p[w]; wn += s_n[w]; }
        bp += s_p[w];
        bn += s_n[w];
      }
      long long tp = carry_p + wp + ip - sp, fp = carry_n + wn + in - sn;  // positives / negatives above this thread
#pragma unroll
      for (int i = 0; i < kRedPer; ++i) {
        const long long pk = p[i], nk = n[i];
        tp += pk;
        fp += nk;
        area += (double)nk * (double)(2 * (tp - pk) + pk);
        if (pk) ap_sum += (double)pk * ((double)tp / (double)(tp + fp));
      }
      carry_p += bp;
      carry_n += bn;
      __syncthreads();  // s_p / s_n are rewritten by the next chunk
    }
  }
  area = wave_sum(area);
  ap_sum = wave_sum(ap_sum);
  if (lane == 0) { s_a[wave] = area; s_b[wave] = ap_sum; }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < kWaves; ++w) { a += s_a[w]; b += s_b[w]; }
    const long long P = carry_p, N = carry_n;
    out[c * 4 + 0] = (P > 0 && N > 0) ? a / (2.0 * (double)P * (double)N) : 0.0;
    out[c * 4 + 1] = P > 0 ? b / (double)P : NAN;
    out[c * 4 + 2] = (double)P;
    out[c * 4 + 3] = (double)N;
    if constexpr (CLEAR) {  // every thread read lo / hi at the start (the barrier above orders this after them)
      int* cr = const_cast<int*>(code_range);
      cr[2 * c] = K;
      cr[2 * c + 1] = -1;
    }
  }
  if (summary != nullptr) {
    // the last block to finish folds every class's scores into the summary (no second launch): release this
    // block's row of ``out``, count it, and the block that completes the count acquires all rows
    __shared__ bool s_last;
    if (tid == 0) {
      __threadfence();
      s_last = atomicAdd(done, 1) == static_cast<int>(gridDim.x) - 1;
    }
    __syncthreads();
    if (s_last) {
      __threadfence();
      curve_summary_block(out, static_cast<int>(gridDim.x), summary);
      if (tid == 0) *done = 0;  // ready for the next launch (stream order)
    }
  }
}

// Class averages and warning flags of curve_hist_reduce's [C, 4] output in one workgroup (replaces ~20 small ATen
// launches and their tiny tensors in compute()):
//   summary = {any N <= 0, any P <= 0, any auroc NaN, any AP NaN,
//              macro AUROC, weighted AUROC, macro AP, weighted AP}   (NaN classes ignored, weights = P)
constexpr int kSumThreads = 256;
__device__ __forceinline__ void curve_summary_block(const double* __restrict__ sc, int C, double* __restrict__ summary) {
  constexpr int kWaves = kSumThreads / kWave;
  double v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // flags x4 | sum_a, cnt_a, wsum_a, sum_ap, cnt_ap, wsum_ap
  double wa = 0.0, wap = 0.0;                     // weight totals over the non-NaN classes
  for (int c = threadIdx.x; c < C; c += kSumThreads) {
    const double a = sc[c * 4 + 0], ap = sc[c * 4 + 1], P = sc[c * 4 + 2], N = sc[c * 4 + 3];
    v[0] += N <= 0.0;
    v[1] += P <= 0.0;
    const bool na = a != a, nap = ap != ap;
    v[2] += na;
    v[3] += nap;
    if (!na) { v[4] += a; v[5] += 1.0; v[6] += a * P; wa += P; }
    if (!nap) { v[7] += ap; v[8] += 1.0; v[9] += ap * P; wap += P; }
  }
  __shared__ double s[kWaves][12];
#pragma unroll
  for (int i = 0; i < 10; ++i) v[i] = wave_sum(v[i]);
  wa = wave_sum(wa);
  wap = wave_sum(wap);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 10; ++i) s[wave][i] = v[i];
    s[wave][10] = wa;
    s[wave][11] = wap;
  }
  __syncthreads();
  if (wave == 0) {  // lane i < 12 folds quantity i over the waves in parallel, lane 0 gathers the 12 totals
    double acc = 0.0;
    if (lane < 12)
      for (int w = 0; w < kWaves; ++w) acc += s[w][lane];
    double t[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) t[i] = __shfl(acc, i, kWave);
    if (lane != 0) return;
    summary[0] = t[0] > 0;
    summary[1] = t[1] > 0;
    summary[2] = t[2] > 0;
    summary[3] = t[3] > 0;
    summary[4] = t[5] > 0 ? t[4] / t[5] : NAN;
    summary[5] = t[10] > 0 ? t[6] / t[10] : NAN;
    summary[6] = t[8] > 0 ? t[7] / t[8] : NAN;
    summary[7] = t[11] > 0 ? t[9] / t[11] : NAN;
    // float32 copies of the 8 values in the buffer's tail (4 doubles): the metric's float32 result is a view, not a
    // conversion launch
    float* s32 = reinterpret_cast<float*>(summary + 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) s32[i] = static_cast<float>(summary[i]);
  }
}

__global__ void __launch_bounds__(kSumThreads) curve_summary_kernel(const double* __restrict__ sc, int C, double* __restrict__ summary) {
  curve_summary_block(sc, C, summary);
}

// Wave-per-class form of the reduce (round 6): one 64-lane wave per class, four classes per 256-thread block, no LDS
// and no block barriers in the scan -- the block form spends most of its ~13 us on the latency of its two barriers
// per 4096-code chunk with ~70 of 256 threads holding codes (a class's occupied range is ~1-2k codes).  Lane l owns
// kRedWavePer consecutive codes of a 64 * kRedWavePer chunk, walked from the top code down with carried prefix
// counts; the per-element arithmetic (area of the trapezoids, precision at each positive) is the block form's.
constexpr int kRedWavePer = 16;
constexpr int kRedWaveChunk = kWave * kRedWavePer;
constexpr int kRedWaveClasses = kRedThreads / kWave;

template <bool CLEAR = false>
__global__ void __launch_bounds__(kRedThreads) curve_hist_reduce_wave_kernel(const int64_t* __restrict__ hist, const int* __restrict__ code_range,
                                                                              double* __restrict__ out, int C, int* __restrict__ done,
                                                                              double* __restrict__ summary) {
  constexpr int K = kCodes;
  const int lane = threadIdx.x & (kWave - 1);
  const int c = blockIdx.x * kRedWaveClasses + static_cast<int>(threadIdx.x / kWave);
  if (c < C) {
    int lo = 0, hi = K - 1;
    if (code_range != nullptr) {
      lo = max(code_range[2 * c], 0);
      hi = min(code_range[2 * c + 1], K - 1);
    }
    const int64_t* negh = hist + ((int64_t)c * 2 + 0) * K;
    const int64_t* posh = hist + ((int64_t)c * 2 + 1) * K;
    long long carry_p = 0, carry_n = 0;
    double area = 0.0, ap_sum = 0.0;
    if (hi >= lo) {
      const int top = hi | (kRedWavePer - 1), bottom = lo & ~(kRedWavePer - 1);
      for (int chunk_top = top; chunk_top >= bottom; chunk_top -= kRedWaveChunk) {
        const int seg_hi = chunk_top - kRedWavePer * lane;
        long long p[kRedWavePer], n[kRedWavePer];  // index i = i-th highest owned code
        if (seg_hi >= bottom) {
          const longlong2* negv = reinterpret_cast<const longlong2*>(negh + (seg_hi - (kRedWavePer - 1)));
          const longlong2* posv = reinterpret_cast<const longlong2*>(posh + (seg_hi - (kRedWavePer - 1)));
#pragma unroll
          for (int v = 0; v < kRedWavePer / 2; ++v) {
            const longlong2 a = posv[v], b = negv[v];
            p[kRedWavePer - 1 - 2 * v] = a.x; p[kRedWavePer - 2 - 2 * v] = a.y;
            n[kRedWavePer - 1 - 2 * v] = b.x; n[kRedWavePer - 2 - 2 * v] = b.y;
          }
          if constexpr (CLEAR) {  // (codes of the aligned segment outside [lo, hi] are zero already)
            longlong2* pw = const_cast<longlong2*>(posv);
            longlong2* nw = const_cast<longlong2*>(negv);
#pragma unroll
            for (int v = 0; v < kRedWavePer / 2; ++v) {
              pw[v] = make_longlong2(0, 0);
              nw[v] = make_longlong2(0, 0);
            }
          }
        } else {
#pragma unroll
          for (int i = 0; i < kRedWavePer; ++i) p[i] = n[i] = 0;
        }
        long long sp = 0, sn = 0;
#pragma unroll
        for (int i = 0; i < kRedWavePer; ++i) { sp += p[i]; sn += n[i]; }
        long long ip = sp, in = sn;  // inclusive wave scan in lane order (= descending code order)
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
          const long long tp = shfl_up_i64(ip, off), tn = shfl_up_i64(in, off);
          if (lane >= off) { ip += tp; in += tn; }
        }
        long long tp = carry_p + ip - sp, fp = carry_n + in - sn;  // positives / negatives above this lane
#pragma unroll
        for (int i = 0; i < kRedWavePer; ++i) {
          const long long pk = p[i], nk = n[i];
          tp += pk;
          fp += nk;
          area += (double)nk * (double)(2 * (tp - pk) + pk);
          if (pk) ap_sum += (double)pk * ((double)tp / (double)(tp + fp));
        }
        carry_p += __shfl(ip, kWave - 1, kWave);
        carry_n += __shfl(in, kWave - 1, kWave);
      }
    }
    area = wave_sum(area);
    ap_sum = wave_sum(ap_sum);
    if (lane == 0) {
      const long long P = carry_p, N = carry_n;
      out[c * 4 + 0] = (P > 0 && N > 0) ? area / (2.0 * (double)P * (double)N) : 0.0;
      out[c * 4 + 1] = P > 0 ? ap_sum / (double)P : NAN;
      out[c * 4 + 2] = (double)P;
      out[c * 4 + 3] = (double)N;
      if constexpr (CLEAR) {  // every lane read lo / hi at the start (program order within the wave)
        int* cr = const_cast<int*>(code_range);
        cr[2 * c] = K;
        cr[2 * c + 1] = -1;
      }
    }
  }
  if (summary != nullptr) {  // the last block folds the summary (see curve_hist_reduce_kernel)
    __shared__ bool s_last;
    __syncthreads();  // every wave's row of ``out`` is written
    if (threadIdx.x == 0) {
      __threadfence();
      s_last = atomicAdd(done, 1) == static_cast<int>(gridDim.x) - 1;
    }
    __syncthreads();
    if (s_last) {
      __threadfence();
      curve_summary_block(out, C, summary);
      if (threadIdx.x == 0) *done = 0;
    }
  }
}

at::Tensor curve_hist_reduce_impl(const at::Tensor& hist_, c10::optional<at::Tensor> code_range, bool clear) {
  TORCH_CHECK(!clear || (hist_.is_contiguous() && code_range.has_value()), "curve_hist_reduce: clear needs a contiguous histogram and its range");
  auto hist = hist_.contiguous();
  TORCH_CHECK(hist.scalar_type() == at::kLong && hist.dim() == 3 && hist.size(1) == 2 && hist.size(2) == kCodes,
              "curve_hist_reduce: hist must be int64 [C, 2, 16384]");
  const int* cr = nullptr;
  if (code_range.has_value()) {
    TORCH_CHECK(code_range->scalar_type() == at::kInt && code_range->numel() == 2 * hist.size(0) && code_range->is_contiguous() &&
                code_range->device() == hist.device(), "code_range must be int32[C, 2] on the histogram's device");
    cr = code_range->data_ptr<int>();
  }
  const int C = static_cast<int>(hist.size(0));
  auto out = at::empty({C, 4}, hist.options().dtype(at::kDouble));
  if (C == 0) return out;
  static const char* form = std::getenv("TMX_REDUCE_FORM");
  if (!clear && (form == nullptr || std::string(form) == "wave")) {  // the same form as curve_hist_scores (bitwise)
    hipLaunchKernelGGL(curve_hist_reduce_wave_kernel<false>, static_cast<unsigned>((C + kRedWaveClasses - 1) / kRedWaveClasses), kRedThreads, 0,
                       stream(), hist.data_ptr<int64_t>(), cr, out.data_ptr<double>(), C, nullptr, nullptr);
  } else if (clear) {
    hipLaunchKernelGGL(curve_hist_reduce_kernel<true>, C, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr, out.data_ptr<double>());
  } else {
    hipLaunchKernelGGL(curve_hist_reduce_kernel<false>, C, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr, out.data_ptr<double>());
  }
  TMX_LAUNCH_CHECK();
  return out;
}

at::Tensor curve_hist_reduce(const at::Tensor& hist, c10::optional<at::Tensor> code_range) {
  return curve_hist_reduce_impl(hist, code_range, false);
}

at::Tensor curve_summary(const at::Tensor& scores_);

// curve_hist_reduce + curve_summary: (scores [C, 4], summary float64[12]).  Two launches: folding the summary into
// the reduce's last class block (device-wide completion counter) measured 33.7 us against 12.4 + 5.1 us -- every
// block's agent-scope release fence has to write back its XCD's L2 (tests/test_compute_fused_gpu.py keeps the op's
// contract; README round 4).
// a zero-initialised int per (device, stream) for the reduce's last-block count (each launch leaves it at zero again;
// launches on one stream are ordered, so they never share it concurrently)
static int* reduce_done_counter(const at::Device& dev) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> counters;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(static_cast<int>(dev.index()), stream());
  auto it = counters.find(key);
  if (it == counters.end()) it = counters.emplace(key, at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(dev))).first;
  return it->second.data_ptr<int>();
}

// scores [C, 4] and the summary [12] in ONE launch (the last reduce block folds the summary)
std::vector<at::Tensor> curve_hist_scores(const at::Tensor& hist_, c10::optional<at::Tensor> code_range, bool clear) {
  TORCH_CHECK(!clear || (hist_.is_contiguous() && code_range.has_value()), "curve_hist_reduce: clear needs a contiguous histogram and its range");
  auto hist = hist_.contiguous();
  TORCH_CHECK(hist.scalar_type() == at::kLong && hist.dim() == 3 && hist.size(1) == 2 && hist.size(2) == kCodes,
              "curve_hist_reduce: hist must be int64 [C, 2, 16384]");
  const int* cr = nullptr;
  if (code_range.has_value()) {
    TORCH_CHECK(code_range->scalar_type() == at::kInt && code_range->numel() == 2 * hist.size(0) && code_range->is_contiguous() &&
                code_range->device() == hist.device(), "code_range must be int32[C, 2] on the histogram's device");
    cr = code_range->data_ptr<int>();
  }
  const int C = static_cast<int>(hist.size(0));
  auto out = at::empty({C, 4}, hist.options().dtype(at::kDouble));
  if (C == 0) return {out, curve_summary(out)};
  auto summary = at::empty({12}, out.options());
  int* done = reduce_done_counter(hist.device());
  // wave-per-class form for compute()'s reduce (22 vs 31 us with the summary, tools/reduce_bench.py), the block form for
  // forward()'s clearing one (28 vs 22 us: the wave form's zeroing stores serialise behind its loads);
  // profiles/reduce_bench_r6.json.  TMX_REDUCE_FORM=block|wave forces one form.
  static const char* form = std::getenv("TMX_REDUCE_FORM");
  const bool wave_form = !clear && (form == nullptr || std::string(form) == "wave");
  if (wave_form) {
    const unsigned blocks = static_cast<unsigned>((C + kRedWaveClasses - 1) / kRedWaveClasses);
    if (clear)
      hipLaunchKernelGGL(curve_hist_reduce_wave_kernel<true>, blocks, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr,
                         out.data_ptr<double>(), C, done, summary.data_ptr<double>());
    else
      hipLaunchKernelGGL(curve_hist_reduce_wave_kernel<false>, blocks, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr,
                         out.data_ptr<double>(), C, done, summary.data_ptr<double>());
    TMX_LAUNCH_CHECK();
    return {out, summary};
  }
  if (clear) {
    // forward's clearing reduce keeps the summary as its own launch: the last-block fold needs a device-scope release
    // per block (an L2 write-back), which behind 18 MB of zeroing stores cost 57 vs 17 + 5 us (profiles/reduce_bench_r6.json)
    hipLaunchKernelGGL(curve_hist_reduce_kernel<true>, C, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr, out.data_ptr<double>(),
                       nullptr, nullptr);
    TMX_LAUNCH_CHECK();
    return {out, curve_summary(out)};
  } else
    hipLaunchKernelGGL(curve_hist_reduce_kernel<false>, C, kRedThreads, 0, stream(), hist.data_ptr<int64_t>(), cr, out.data_ptr<double>(), done,
                       summary.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return {out, summary};
}

at::Tensor curve_summary(const at::Tensor& scores_) {
  auto scores = scores_.contiguous();
  TORCH_CHECK(scores.scalar_type() == at::kDouble && scores.dim() == 2 && scores.size(1) == 4, "curve_summary: scores must be float64 [C, 4]");
  auto summary = at::empty({12}, scores.options());  // [0, 8) float64 values, [8, 12) the same as 8 float32
  hipLaunchKernelGGL(curve_summary_kernel, 1, kSumThreads, 0, stream(), scores.data_ptr<double>(),
                     static_cast<int>(scores.size(0)), summary.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return summary;
}

// =========================================================================================================
// binned (multi-threshold) curve:  confmat[T, C, 2, 2] += counts
// bucket b(p) = #thresholds <= p  (p >= thr[i]  <=>  i < b(p));  hist[C][2][T+1] then suffix-sum.
// =========================================================================================================
// bucket b(p) = #thresholds <= p.  Thresholds are almost always linspace: guess from the spacing, verify with the
// one or two neighbouring thresholds, and fall back to the binary search for any other spacing (exact either way).
__device__ __forceinline__ int thr_bucket(float p, const float* __restrict__ s_thr, int nT, float t0, float inv_step) {
  if (p != p) return 0;  // NaN: no threshold is <= NaN
  float gf = (p - t0) * inv_step + 1.f;
  gf = fminf(fmaxf(gf, 0.f), (float)nT);
  const int g = (int)gf;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int c = d == 0 ? g : (d == 1 ? g + 1 : g - 1);
    if (c < 0 || c > nT) continue;
    if ((c == 0 || s_thr[c - 1] <= p) && (c == nT || s_thr[c] > p)) return c;
  }
  int lo = 0, hi = nT;  // first index with thr > p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s_thr[mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo;
}

template <typename T, int MODE>  // MODE 0: multiclass rows (softmax), 1: elementwise (sigmoid)
__global__ void binned_hist_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t N, int C,
                                   int64_t S, const float* __restrict__ thr, int nT, const int* __restrict__ flag,
                                   int64_t ignore_index, bool has_ignore, int* __restrict__ hist, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) float s_thr[];
  bool bad = false;
  for (int i = threadIdx.x; i < nT; i += blockDim.x) s_thr[i] = thr[i];
  __syncthreads();
  const bool do_norm = flag[0] != 0;
  const float t0 = s_thr[0];
  const float inv_step = nT > 1 && s_thr[nT - 1] > t0 ? (float)(nT - 1) / (s_thr[nT - 1] - t0) : 0.f;
  auto bucket = [&](float p) { return thr_bucket(p, s_thr, nT, t0, inv_step); };
  if constexpr (MODE == 0) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
    const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
    for (int64_t r = wave; r < N; r += nwaves) {
      const int64_t t = target[r];
      if (has_ignore && t == ignore_index) continue;
      bad |= t < 0 || t >= C;
      const T* row = preds + r * C;
      float mx = -INFINITY, s = 0.f;
      if (do_norm) {
        for (int c = lane; c < C; c += kWave) mx = fmaxf(mx, to_f32<T>(row[c]));
        mx = wave_max(mx);
        for (int c = lane; c < C; c += kWave) s += expf(to_f32<T>(row[c]) - mx);
        s = wave_sum(s);
      }
      for (int c = lane; c < C; c += kWave) {
        float v = to_f32<T>(row[c]);
        if (do_norm) v = round_trip<T>(expf(v - mx) / s);
        int b = bucket(v);
        atomicAdd(hist + ((int64_t)c * 2 + (c == t ? 1 : 0)) * (nT + 1) + b, 1);
      }
    }
  } else {
    const int64_t total = N * C * S;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
      const int64_t t = target[i];
      if (has_ignore && t == ignore_index) continue;
      if (t != 0 && t != 1) {
        bad = true;
        continue;
      }
      const int l = static_cast<int>((i / S) % C);
      float v = to_f32<T>(preds[i]);
      if (do_norm) v = round_trip<T>(1.f / (1.f + expf(-v)));
      int b = bucket(v);
      atomicAdd(hist + ((int64_t)l * 2 + (int)t) * (nT + 1) + b, 1);
    }
  }
  if (bad && err) atomicOr(err, 1);
}

// Element-wise (binary / multilabel) binned histogram with the [C][2][T+1] counts privatised in LDS: one copy per wave
// when they fit (same-address atomics of a wave's lanes then only collide within the wave), else one per block; one
// global atomic per non-empty bin on flush.  The global-atomic form above put every score of a BinaryAUROC on the
// same 2 (T + 1) addresses (16M fp32 scores, T = 100: 9.3 ms per update).
constexpr int kBinnedThreads = 512;

template <typename T>
__global__ void __launch_bounds__(kBinnedThreads) binned_hist_lds_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                         int64_t N, int C, int64_t S, const float* __restrict__ thr,
                                                                         int nT, const int* __restrict__ flag, int64_t ignore_index,
                                                                         bool has_ignore, int copies, int* __restrict__ hist,
                                                                         int* __restrict__ err, bool vec_ok) {
  bool bad = false;
  extern __shared__ __attribute__((aligned(16))) int s_mem[];  // [nT] thresholds as float, then [copies][C][2][nT + 1]
  float* s_thr = reinterpret_cast<float*>(s_mem);
  const int nT4 = (nT + 3) / 4 * 4;
  int* s_hist = s_mem + nT4;
  const int H = C * 2 * (nT + 1);
  for (int i = threadIdx.x; i < nT; i += kBinnedThreads) s_thr[i] = thr[i];
  for (int i = threadIdx.x; i < copies * H; i += kBinnedThreads) s_hist[i] = 0;
  __syncthreads();
  const bool do_norm = flag[0] != 0;
  const float t0 = s_thr[0];
  const float inv_step = nT > 1 && s_thr[nT - 1] > t0 ? (float)(nT - 1) / (s_thr[nT - 1] - t0) : 0.f;
  int* my = s_hist + (int)((threadIdx.x / kWave) % copies) * H;
  const int64_t total = N * C * S;
  int64_t start = 0;
  if (C == 1 && vec_ok) {
    // binary: 16-B loads of scores and targets (one label, so no per-element label arithmetic)
    constexpr int VEC = 16 / sizeof(T);
    using PP = Pack16<T, VEC>;
    using TP = Pack16<int64_t, VEC>;
    const int64_t nv = total / VEC;
    for (int64_t v = blockIdx.x * (int64_t)kBinnedThreads + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBinnedThreads) {
      const PP pv = reinterpret_cast<const PP*>(preds)[v];
      const TP tv = reinterpret_cast<const TP*>(target)[v];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const int64_t t = tv.v[k];
        if (has_ignore && t == ignore_index) continue;
        if (t != 0 && t != 1) {
          bad = true;
          continue;
        }
        float x = to_f32<T>(pv.v[k]);
        if (do_norm) x = round_trip<T>(1.f / (1.f + expf(-x)));
        atomicAdd(my + (int)t * (nT + 1) + thr_bucket(x, s_thr, nT, t0, inv_step), 1);
      }
    }
    start = nv * VEC;  // tail below, by every thread of the grid-stride loop
  }
  for (int64_t i = start + blockIdx.x * (int64_t)kBinnedThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBinnedThreads) {
    const int64_t t = target[i];
    if (has_ignore && t == ignore_index) continue;
    if (t != 0 && t != 1) {
      bad = true;
      continue;
    }
    const int l = static_cast<int>((i / S) % C);
    float v = to_f32<T>(preds[i]);
    if (do_norm) v = round_trip<T>(1.f / (1.f + expf(-v)));
    atomicAdd(my + (l * 2 + (int)t) * (nT + 1) + thr_bucket(v, s_thr, nT, t0, inv_step), 1);
  }
  if (bad && err) atomicOr(err, 1);
  __syncthreads();
  for (int b = threadIdx.x; b < H; b += kBinnedThreads) {
    int cnt = 0;
    for (int k = 0; k < copies; ++k) cnt += s_hist[k * H + b];
    if (cnt) atomicAdd(hist + b, cnt);
  }
}

// confmat[t, c, y, p]: y = target (0/1), p = (score >= thr[t]).  tp=[1][1] fp=[0][1] fn=[1][0] tn=[0][0]
// One workgroup per class: the (nT + 1)-bucket histogram is suffix-summed in LDS (Hillis-Steele over 2 * (nT + 1)
// words), then thread t writes threshold t's four cells.  (A single thread walking the buckets took 41 us.)
__global__ void __launch_bounds__(1024) binned_scan_kernel(const int* __restrict__ hist, int C, int nT, int64_t* __restrict__ confmat) {
  extern __shared__ __attribute__((aligned(16))) long long s_suf[];  // [2][nT + 1] suffix sums, then [2][nT + 1] scratch
  const int c = blockIdx.x;
  const int M = nT + 1;
  long long* a = s_suf;
  long long* b = s_suf + 2 * M;
  for (int i = threadIdx.x; i < 2 * M; i += blockDim.x) a[i] = hist[(int64_t)c * 2 * M + i];
  __syncthreads();
  for (int off = 1; off < M; off <<= 1) {  // suffix sums within each of the two rows
    for (int i = threadIdx.x; i < 2 * M; i += blockDim.x) {
      const int j = i % M;
      b[i] = a[i] + (j + off < M ? a[i + off] : 0);
    }
    __syncthreads();
    long long* tmp = a;
    a = b;
    b = tmp;
  }
  for (int t = threadIdx.x; t < nT; t += blockDim.x) {
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const long long total = a[y * M];
      const long long above = a[y * M + t + 1];  // # with bucket > t  (score >= thr[t])
      int64_t* cell = confmat + ((int64_t)t * C + c) * 4 + y * 2;
      cell[1] += above;          // predicted positive
      cell[0] += total - above;  // predicted negative
    }
  }
}

void binned_curve_update(const at::Tensor& preds_, const at::Tensor& target_, const at::Tensor& thresholds_,
                         at::Tensor& confmat, int64_t task, int64_t ignore_index, bool has_ignore,
                         c10::optional<at::Tensor> norm_flag, c10::optional<at::Tensor> err_flag) {
  int* err = nullptr;
  if (err_flag.has_value()) {
    TORCH_CHECK(err_flag->scalar_type() == at::kInt && err_flag->is_contiguous(), "err_flag must be int32");
    err = err_flag->data_ptr<int>();
  }
  auto preds = preds_.contiguous();
  auto target = target_.contiguous().to(at::kLong);
  auto thr = thresholds_.contiguous().to(at::kFloat);
  const int nT = static_cast<int>(thr.numel());
  TORCH_CHECK(confmat.is_contiguous() && confmat.scalar_type() == at::kLong && confmat.dim() == 4 && confmat.size(0) == nT);
  const int C = static_cast<int>(confmat.size(1));
  auto hist = at::zeros({C, 2, nT + 1}, preds.options().dtype(at::kInt));
  auto flag = norm_flag.has_value() ? norm_flag->to(at::kInt).contiguous() : range_flag(preds);
  const int block = 256;
  const size_t shm = nT * sizeof(float);
  TORCH_CHECK(shm <= 64 * 1024, "too many thresholds");
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "binned_curve_update", [&] {
    const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
    if (task == 0) {
      const int64_t n = target.numel();
      if (n == 0) return;
      hipLaunchKernelGGL((binned_hist_kernel<scalar_t, 0>), grid_for(n * kWave, block, 4096), block, shm, stream(), p,
                         target.data_ptr<int64_t>(), n, C, (int64_t)1, thr.data_ptr<float>(), nT, flag.data_ptr<int>(),
                         ignore_index, has_ignore, hist.data_ptr<int>(), err);
    } else {
      const int64_t total = target.numel();
      if (total == 0) return;
      const int64_t N = target.size(0);
      const int64_t S = total / (N * C);
      const int64_t H = (int64_t)C * 2 * (nT + 1);
      const int64_t thr_ints = (nT + 3) / 4 * 4;
      constexpr int64_t kLdsBudget = 64 * 1024 / sizeof(int);
      if (thr_ints + H <= kLdsBudget) {
        const int copies = static_cast<int>(std::min<int64_t>(kBinnedThreads / kWave, (kLdsBudget - thr_ints) / H));
        const size_t shm_lds = (size_t)(thr_ints + copies * H) * sizeof(int);
        const int grid = static_cast<int>(std::min<int64_t>(1024, (total + kBinnedThreads - 1) / kBinnedThreads));
        hipLaunchKernelGGL(binned_hist_lds_kernel<scalar_t>, std::max(grid, 1), kBinnedThreads, shm_lds, stream(), p,
                           target.data_ptr<int64_t>(), N, C, S, thr.data_ptr<float>(), nT, flag.data_ptr<int>(), ignore_index,
                           has_ignore, copies, hist.data_ptr<int>(), err,
                           ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(target.data_ptr())) & 15) == 0);
        return;
      }
      hipLaunchKernelGGL((binned_hist_kernel<scalar_t, 1>), grid_for(total, block, 4096), block, shm, stream(), p,
                         target.data_ptr<int64_t>(), N, C, S, thr.data_ptr<float>(), nT, flag.data_ptr<int>(), ignore_index,
                         has_ignore, hist.data_ptr<int>(), err);
    }
  });
  TMX_LAUNCH_CHECK();
  const size_t scan_shm = 4 * (size_t)(nT + 1) * sizeof(long long);
  TORCH_CHECK(scan_shm <= 64 * 1024, "binned_curve_update: too many thresholds for the LDS scan");
  hipLaunchKernelGGL(binned_scan_kernel, C, 256, scan_shm, stream(), hist.data_ptr<int>(), C, nT, confmat.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
}

// =========================================================================================================
// calibration error: bins[3, n_bins + 1] (count, sum confidence, sum accuracy) in float64
// bin = bucketize(conf, boundaries, right=True) - 1 (boundaries = torch.linspace(0, 1, n_bins + 1) in fp32): the
// number of boundaries <= conf, minus one; NaN -> the last bin (every comparison false), as torch.bucketize.
// Per-block LDS accumulation (ds_add_f64), one global f64 atomic per bin and channel per block — the reference's
// index_add_ puts every sample on the same n_bins + 1 addresses (3.2 ms per update at 65536 x 1000, most of it
// contended f64 atomics).
// =========================================================================================================
constexpr int kCalThreads = 256;

__device__ __forceinline__ int cal_bin(float conf, const float* __restrict__ s_b, int nb1) {
  int lo = 0, hi = nb1;  // first boundary > conf (NaN: none is <= conf -> lo stays... handled below)
  if (conf != conf) return nb1 - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s_b[mid] <= conf) lo = mid + 1; else hi = mid;
  }
  return lo - 1 < 0 ? nb1 - 1 : lo - 1;  // conf < 0: bucketize gives 0 -> index -1 -> wraps to the last bin
}

__device__ __forceinline__ void cal_flush(const double* __restrict__ s_acc, int nb1, double* __restrict__ bins) {
  for (int i = threadIdx.x; i < 3 * nb1; i += kCalThreads)
    if (s_acc[i] != 0.0) atomicAdd(bins + i, s_acc[i]);
}

// element-wise: conf[N] (any float dtype), acc[N] (any numeric dtype, converted to float)
template <typename T, typename A>
__global__ void __launch_bounds__(kCalThreads) ce_bins_kernel(const T* __restrict__ conf, const A* __restrict__ acc, int64_t n,
                                                             const float* __restrict__ boundaries, int nb1, double* __restrict__ bins) {
  extern __shared__ __attribute__((aligned(16))) double s_acc[];  // [3][nb1], then boundaries
  float* s_b = reinterpret_cast<float*>(s_acc + 3 * nb1);
  for (int i = threadIdx.x; i < 3 * nb1; i += kCalThreads) s_acc[i] = 0.0;
  for (int i = threadIdx.x; i < nb1; i += kCalThreads) s_b[i] = boundaries[i];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)kCalThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kCalThreads) {
    const float c = static_cast<float>(to_f32<T>(conf[i]));
    const int b = cal_bin(c, s_b, nb1);
    atomicAdd(&s_acc[b], 1.0);
    atomicAdd(&s_acc[nb1 + b], (double)c);
    atomicAdd(&s_acc[2 * nb1 + b], (double)static_cast<float>(acc[i]));
  }
  __syncthreads();
  cal_flush(s_acc, nb1, bins);
}

// multiclass, fused: one wave per row of preds[N, C].  Reference semantics (preds.softmax(1) if the batch is not in
// [0, 1], then .max(1)): conf = the largest softmax value rounded to the input dtype = RNE(1 / sum exp(x - max)),
// pred = the FIRST class whose rounded softmax equals it (rounding can tie classes the logits order), correct =
// (pred == target); a row with NaN (or a softmax row with +-inf) gives conf NaN and the first NaN's index.
template <typename T>
__global__ void __launch_bounds__(kCalThreads) mc_calibration_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                    int64_t n, int C, const int* __restrict__ softmax_flag,
                                                                    const float* __restrict__ boundaries, int nb1,
                                                                    double* __restrict__ bins) {
  extern __shared__ __attribute__((aligned(16))) double s_acc[];
  float* s_b = reinterpret_cast<float*>(s_acc + 3 * nb1);
  for (int i = threadIdx.x; i < 3 * nb1; i += kCalThreads) s_acc[i] = 0.0;
  for (int i = threadIdx.x; i < nb1; i += kCalThreads) s_b[i] = boundaries[i];
  __syncthreads();
  const bool do_softmax = softmax_flag[0] != 0;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)kCalThreads + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * kCalThreads / kWave;
  for (int64_t r = wave; r < n; r += nwaves) {
    const T* row = preds + r * C;
    float mx = -INFINITY;
    int first_nan = C, am = C;
    for (int c = lane; c < C; c += kWave) {
      const float v = to_f32<T>(row[c]);
      if (v != v) first_nan = min(first_nan, c);
      else if (am == C || v > mx) { mx = v; am = c; }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) first_nan = min(first_nan, __shfl_xor(first_nan, off, kWave));
    wave_argmax(mx, am);
    float conf;
    int pred;
    if (first_nan < C) {
      conf = NAN;
      pred = do_softmax ? 0 : first_nan;  // softmax of a NaN row is all NaN: max returns index 0
    } else if (!do_softmax) {
      conf = mx;
      pred = am;
    } else if (mx == INFINITY || mx == -INFINITY) {  // inf - inf: the softmax row is NaN everywhere
      conf = NAN;
      pred = 0;
    } else {
      float s = 0.f;
      for (int c = lane; c < C; c += kWave) s += expf(to_f32<T>(row[c]) - mx);
      s = wave_sum(s);
      conf = round_trip<T>(1.f / s);  // exp(0) / s, rounded as torch stores the softmax
      int first = C;
      for (int c = lane; c < C; c += kWave)
        if (round_trip<T>(expf(to_f32<T>(row[c]) - mx) / s) == conf) { first = c; break; }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off, kWave));
      pred = first;
    }
    if (lane == 0) {
      const int b = cal_bin(conf, s_b, nb1);
      atomicAdd(&s_acc[b], 1.0);
      atomicAdd(&s_acc[nb1 + b], (double)conf);
      atomicAdd(&s_acc[2 * nb1 + b], pred == target[r] ? 1.0 : 0.0);
    }
  }
  __syncthreads();
  cal_flush(s_acc, nb1, bins);
}

void ce_bins_update(const at::Tensor& conf_, const at::Tensor& acc_, const at::Tensor& boundaries_, at::Tensor& bins) {
  auto conf = conf_.contiguous().reshape(-1);
  auto acc = acc_.contiguous().reshape(-1);
  auto bnd = boundaries_.contiguous().to(at::kFloat);
  const int nb1 = static_cast<int>(bnd.numel());
  TORCH_CHECK(bins.is_contiguous() && bins.scalar_type() == at::kDouble && bins.numel() == 3 * nb1, "bins must be float64 [3, n_bins + 1]");
  TORCH_CHECK(conf.numel() == acc.numel(), "confidences / accuracies size mismatch");
  const int64_t n = conf.numel();
  if (n == 0) return;
  if (acc.scalar_type() == at::kBool) acc = acc.to(at::kFloat);
  const size_t shm = 3 * nb1 * sizeof(double) + nb1 * sizeof(float);
  TORCH_CHECK(shm <= 64 * 1024, "ce_bins_update: too many bins");
  const int grid = grid_for(n, kCalThreads, 1024);
  TMX_DISPATCH_FLOAT(conf.scalar_type(), "ce_bins_update", [&] {
    using CT = scalar_t;
    const CT* cp = reinterpret_cast<const CT*>(conf.data_ptr());
    switch (acc.scalar_type()) {
      case at::kFloat:
        hipLaunchKernelGGL((ce_bins_kernel<CT, float>), grid, kCalThreads, shm, stream(), cp, acc.data_ptr<float>(), n,
                           bnd.data_ptr<float>(), nb1, bins.data_ptr<double>());
        break;
      case at::kDouble:
        hipLaunchKernelGGL((ce_bins_kernel<CT, double>), grid, kCalThreads, shm, stream(), cp, acc.data_ptr<double>(), n,
                           bnd.data_ptr<float>(), nb1, bins.data_ptr<double>());
        break;
      default: {
        auto a64 = acc.to(at::kLong);
        hipLaunchKernelGGL((ce_bins_kernel<CT, int64_t>), grid, kCalThreads, shm, stream(), cp, a64.data_ptr<int64_t>(), n,
                           bnd.data_ptr<float>(), nb1, bins.data_ptr<double>());
      }
    }
  });
  TMX_LAUNCH_CHECK();
}

// One-pass top-label calibration update straight from the raw [N, C] scores (aligned rows, C a multiple of the
// 16-B vector width, C <= 128 * VEC): 4 rows per wave in flight, DPP max / sum and ballot arg-max as the pair-stream
// kernel.  The reference decides "softmax or not" on the whole (ignore-filtered) batch; here every row is binned
// both ways -- raw (max, first arg-max) and softmax (rounded 1 / sum exp, first index whose rounded softmax equals
// it) -- into a [2][3][nb1] table, and the last workgroup (grid_sum_last carrying the out-of-range row count) adds
// the right half to the bins.  Ignored rows are skipped in-kernel (no boolean-index copy); a target outside
// [0, C) ORs err (deferred validation).
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(0.f, v);
  v += dpp_f32<0x4E>(0.f, v);
  v += dpp_f32<0x141>(0.f, v);
  v += dpp_f32<0x140>(0.f, v);
  v += dpp_f32<0x142, 0xA>(0.f, v);
  v += dpp_f32<0x143, 0xC>(0.f, v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

template <typename T, int NCH>
__global__ void __launch_bounds__(256) mc_calibration_vec_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                 int64_t n, int C, int64_t ignore_index, bool has_ignore,
                                                                 const float* __restrict__ boundaries, int nb1,
                                                                 double* __restrict__ bins, unsigned long long* __restrict__ scratch,
                                                                 int* __restrict__ err) {
  constexpr int VEC = VecOf<T>::n;
  constexpr int kRows = 4;
  extern __shared__ __attribute__((aligned(16))) double s_cal[];  // [2 modes][3][nb1], then boundaries (float)
  float* s_b = reinterpret_cast<float*>(s_cal + 6 * nb1);
  __shared__ int s_oor;
  __shared__ long long s_last;
  for (int i = threadIdx.x; i < 6 * nb1; i += blockDim.x) s_cal[i] = 0.0;
  for (int i = threadIdx.x; i < nb1; i += blockDim.x) s_b[i] = boundaries[i];
  if (threadIdx.x == 0) s_oor = 0;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1);
  const int nvec = C / VEC;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  int oor_rows = 0;
  bool bad_t = false;
  for (int64_t r0 = wave * kRows; r0 < n; r0 += nwaves * kRows) {
    uint4 w[kRows][NCH];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const uint4* row = reinterpret_cast<const uint4*>(preds + min(r0 + i, n - 1) * C);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int q = lane + kWave * ch;
        w[i][ch] = row[q < nvec ? q : nvec - 1];
      }
    }
    int64_t tt[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) tt[i] = target[min(r0 + i, n - 1)];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int64_t t = tt[i];
      if (r0 + i >= n || (has_ignore && t == ignore_index)) continue;  // wave-uniform
      bad_t |= t < 0 || t >= C;
      float m[NCH];
      int kk[NCH];
      bool nan = false, out = false;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const bool active = lane + kWave * ch < nvec;
        float mm = -INFINITY;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const float v = vec_elem<T>(w[i][ch], k);
          nan |= active && v != v;
          out |= active && !(v >= 0.f && v <= 1.f);
          mm = __builtin_fmaxf(mm, v);
        }
        int kf = VEC - 1;
#pragma unroll
        for (int k = VEC - 2; k >= 0; --k) kf = vec_elem<T>(w[i][ch], k) == mm ? k : kf;
        m[ch] = active ? mm : -INFINITY;
        kk[ch] = kf;
      }
      const bool row_nan = __ballot(nan) != 0;
      const bool row_oor = __ballot(out) != 0;
      oor_rows += row_oor ? 1 : 0;
      float mx = m[0];
#pragma unroll
      for (int ch = 1; ch < NCH; ++ch) mx = __builtin_fmaxf(mx, m[ch]);
      mx = wave_max_uniform(mx);
      // raw mode (only chosen when no row of the batch is out of [0, 1], so never for NaN rows)
      uint64_t b = __ballot(m[0] == mx);
      int ch0 = 0;
      if constexpr (NCH == 2) {
        if (b == 0) {
          b = __ballot(m[1] == mx);
          ch0 = 1;
        }
      }
      const int L0 = b ? __builtin_ctzll(b) : 0;
      const int pred_raw = VEC * (L0 + kWave * ch0) + __builtin_amdgcn_readlane(NCH == 2 && ch0 ? kk[NCH - 1] : kk[0], L0);
      const float conf_raw = row_nan ? NAN : mx;
      // softmax mode
      float conf_sm = NAN;
      int pred_sm = 0;
      if (!row_nan && mx != INFINITY && mx != -INFINITY) {
        float sum = 0.f;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const bool active = lane + kWave * ch < nvec;
#pragma unroll
          for (int k = 0; k < VEC; ++k)  // hardware exp2 (~1 ulp, like the summation-order difference to ATen)
            sum += active ? __builtin_amdgcn_exp2f((vec_elem<T>(w[i][ch], k) - mx) * 1.4426950408889634f) : 0.f;
        }
        sum = wave_sum_dpp(sum);
        conf_sm = round_trip<T>(1.f / sum);
        // An element can round to the max's softmax value only if exp(v - max) > 1 - 2^-7 (bf16; tighter for fp16 /
        // fp32), i.e. v > max - 0.0079.  Without such a runner-up the answer is the raw first arg-max.
        bool near = false;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const bool active = lane + kWave * ch < nvec;
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            const float v = vec_elem<T>(w[i][ch], k);
            near |= active && v < mx && v > mx - 0.01f;
          }
        }
        pred_sm = pred_raw;
        if (__ballot(near)) {
          int first[NCH];
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const bool active = lane + kWave * ch < nvec;
            int f = VEC;
#pragma unroll
            for (int k = VEC - 1; k >= 0; --k) {
              const float v = vec_elem<T>(w[i][ch], k);
              if (active && v > mx - 0.01f && round_trip<T>(expf(v - mx) / sum) == conf_sm) f = k;
            }
            first[ch] = f;
          }
          uint64_t bs = __ballot(first[0] < VEC);
          int chs = 0;
          if constexpr (NCH == 2) {
            if (bs == 0) {
              bs = __ballot(first[1] < VEC);
              chs = 1;
            }
          }
          const int Ls = bs ? __builtin_ctzll(bs) : 0;
          pred_sm = VEC * (Ls + kWave * chs) + __builtin_amdgcn_readlane(NCH == 2 && chs ? first[NCH - 1] : first[0], Ls);
        }
      }
      if (lane == 0) {
        const int br = cal_bin(conf_raw, s_b, nb1), bsm = cal_bin(conf_sm, s_b, nb1);
        atomicAdd(&s_cal[br], 1.0);
        atomicAdd(&s_cal[nb1 + br], (double)conf_raw);
        atomicAdd(&s_cal[2 * nb1 + br], pred_raw == t ? 1.0 : 0.0);
        atomicAdd(&s_cal[3 * nb1 + bsm], 1.0);
        atomicAdd(&s_cal[4 * nb1 + bsm], (double)conf_sm);
        atomicAdd(&s_cal[5 * nb1 + bsm], pred_sm == t ? 1.0 : 0.0);
      }
    }
  }
  if (bad_t && lane == 0 && err) atomicOr(err, 1);
  if (lane == 0 && oor_rows) atomicAdd(&s_oor, oor_rows);
  __syncthreads();
  for (int i = threadIdx.x; i < 6 * nb1; i += blockDim.x)
    if (s_cal[i] != 0.0) atomicAdd(reinterpret_cast<double*>(scratch) + i, s_cal[i]);
  __builtin_amdgcn_s_waitcnt(0);  // table atomics performed before this workgroup's ticket
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long mine[1] = {s_oor};
    long long tot[1];
    s_last = grid_sum_last<1>(scratch + 6 * nb1, mine, tot) ? tot[0] : -1;
  }
  __syncthreads();
  if (s_last < 0) return;
  const int mode = s_last > 0 ? 1 : 0;
  for (int i = threadIdx.x; i < 3 * nb1; i += blockDim.x) {
    const double keep = __longlong_as_double((long long)atomicExch(&scratch[mode * 3 * nb1 + i], 0ull));
    atomicExch(&scratch[(1 - mode) * 3 * nb1 + i], 0ull);
    if (keep != 0.0 || keep != keep) atomicAdd(bins + i, keep);
  }
}

// Returns false when the shape / alignment does not qualify (caller falls back to the filtered path).
bool mc_calibration_fused(const at::Tensor& preds, const at::Tensor& target_, const at::Tensor& boundaries_, at::Tensor& bins,
                          at::Tensor& scratch, int64_t ignore_index, bool has_ignore, const c10::optional<at::Tensor>& err_flag) {
  TORCH_CHECK(preds.dim() == 2, "preds must be [N, C]");
  auto target = target_.contiguous().to(at::kLong).reshape(-1);
  auto bnd = boundaries_.contiguous().to(at::kFloat);
  const int nb1 = static_cast<int>(bnd.numel());
  TORCH_CHECK(bins.is_contiguous() && bins.scalar_type() == at::kDouble && bins.numel() == 3 * nb1, "bins must be float64 [3, n_bins + 1]");
  TORCH_CHECK(scratch.is_contiguous() && scratch.scalar_type() == at::kDouble && scratch.numel() >= 6 * nb1 + kGridSlotsWords,
              "scratch must be a zeroed float64 [6 (n_bins + 1) + ", kGridSlotsWords, "]");
  const int64_t n = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  TORCH_CHECK(target.numel() == n, "preds must be [N, C] with target [N]");
  if (!preds.is_contiguous() || !preds.is_floating_point()) return false;
  const size_t shm = 6 * nb1 * sizeof(double) + nb1 * sizeof(float);
  if (shm > 48 * 1024) return false;
  if (n == 0) return true;
  int* err = flag_ptr(err_flag);
  bool done = false;
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "mc_calibration_fused", [&] {
    constexpr int VEC = VecOf<scalar_t>::n;
    const scalar_t* p = reinterpret_cast<const scalar_t*>(preds.data_ptr());
    if (C % VEC != 0 || C < 2 || C > 2 * kWave * VEC || (reinterpret_cast<uintptr_t>(p) & 15) != 0) return;
    auto* sc = reinterpret_cast<unsigned long long*>(scratch.data_ptr<double>());
    const int grid = grid_for(n * kWave / 4, 256, 2048);
    if (C <= kWave * VEC)
      hipLaunchKernelGGL((mc_calibration_vec_kernel<scalar_t, 1>), grid, 256, shm, stream(), p, target.data_ptr<int64_t>(), n, C,
                         ignore_index, has_ignore, bnd.data_ptr<float>(), nb1, bins.data_ptr<double>(), sc, err);
    else
      hipLaunchKernelGGL((mc_calibration_vec_kernel<scalar_t, 2>), grid, 256, shm, stream(), p, target.data_ptr<int64_t>(), n, C,
                         ignore_index, has_ignore, bnd.data_ptr<float>(), nb1, bins.data_ptr<double>(), sc, err);
    done = true;
  });
  TMX_LAUNCH_CHECK();
  return done;
}

void mc_calibration_update(const at::Tensor& preds_, const at::Tensor& target_, const at::Tensor& boundaries_, at::Tensor& bins) {
  auto preds = preds_.contiguous();
  auto target = target_.contiguous().to(at::kLong).reshape(-1);
  auto bnd = boundaries_.contiguous().to(at::kFloat);
  const int nb1 = static_cast<int>(bnd.numel());
  TORCH_CHECK(preds.dim() == 2 && preds.size(0) == target.numel(), "preds must be [N, C] with target [N]");
  TORCH_CHECK(bins.is_contiguous() && bins.scalar_type() == at::kDouble && bins.numel() == 3 * nb1, "bins must be float64 [3, n_bins + 1]");
  const int64_t n = preds.size(0);
  const int C = static_cast<int>(preds.size(1));
  if (n == 0) return;
  auto flag = range_flag(preds);
  const size_t shm = 3 * nb1 * sizeof(double) + nb1 * sizeof(float);
  TORCH_CHECK(shm <= 64 * 1024, "mc_calibration_update: too many bins");
  const int grid = grid_for(n * kWave, kCalThreads, 2048);
  TMX_DISPATCH_FLOAT(preds.scalar_type(), "mc_calibration_update", [&] {
    hipLaunchKernelGGL(mc_calibration_kernel<scalar_t>, grid, kCalThreads, shm, stream(),
                       reinterpret_cast<const scalar_t*>(preds.data_ptr()), target.data_ptr<int64_t>(), n, C,
                       flag.data_ptr<int>(), bnd.data_ptr<float>(), nb1, bins.data_ptr<double>());
  });
  TMX_LAUNCH_CHECK();
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("range_flag(Tensor x) -> Tensor");
  m.def("bincount(Tensor x, int minlength) -> Tensor");
  m.def("mc_confmat_update(Tensor preds, Tensor target, Tensor(a!) confmat, int ignore_index, bool has_ignore, Tensor(b!)? err_t=None, Tensor(c!)? err_p=None) -> ()");
  m.def("mc_stat_scores_update(Tensor preds, Tensor target, int num_classes, Tensor(a!) tp, Tensor(b!) fp, Tensor(c!) tn, Tensor(d!) fn, Tensor(e!) ticket, int ignore_index, bool has_ignore, bool micro, Tensor(f!)? err_t=None, Tensor(g!)? err_p=None) -> ()");
  m.def("binary_stats_fused(Tensor preds, Tensor target, Tensor(a!) tp, Tensor(b!) fp, Tensor(c!) tn, Tensor(d!) fn, Tensor(e!) scratch, int num_labels, float threshold, int ignore_index, bool has_ignore, Tensor(f!)? err_t=None, Tensor(g!)? err_p=None) -> ()");
  m.def("binary_stats_update(Tensor preds, Tensor target, Tensor(a!) counts, int num_labels, float threshold, int ignore_index, bool has_ignore) -> ()");
  m.def("curve_hist_update(Tensor preds, Tensor target, Tensor(a!) hist, int task, int ignore_index, bool has_ignore, Tensor(b!)? confmat, Tensor? norm_flag, Tensor(c!)? err_flag, Tensor(d!)? mode_state, Tensor(e!)? code_range=None, Tensor(f!)? batch_hist=None, Tensor(g!)? batch_range=None) -> ()");
  m.def("curve_hist_zero(Tensor(a!) hist, Tensor(b!) code_range) -> ()");
  m.def("curve_hist_drain(Tensor(a!) dst, Tensor(b!) dst_range, Tensor(c!) src, Tensor(d!) src_range) -> ()");
  m.def("curve_hist_reduce(Tensor hist, Tensor? code_range=None) -> Tensor");
  m.def("curve_summary(Tensor scores) -> Tensor");
  m.def("curve_hist_scores(Tensor(a!) hist, Tensor(b!)? code_range=None, bool clear=False) -> Tensor[]");
  m.def("curve_mc_rowpass(Tensor preds, Tensor target, Tensor(a!) mode, Tensor(b!) state, Tensor(c!) codes, Tensor(d!) slow_rows, int ignore_index, bool has_ignore, Tensor(e!)? confmat, Tensor(f!)? err_flag) -> ()");
  m.def("binned_curve_update(Tensor preds, Tensor target, Tensor thresholds, Tensor(a!) confmat, int task, int ignore_index, bool has_ignore, Tensor? norm_flag, Tensor(b!)? err_flag=None) -> ()");
  m.def("ce_bins_update(Tensor conf, Tensor acc, Tensor boundaries, Tensor(a!) bins) -> ()");
  m.def("mc_calibration_update(Tensor preds, Tensor target, Tensor boundaries, Tensor(a!) bins) -> ()");
  m.def("mc_calibration_fused(Tensor preds, Tensor target, Tensor boundaries, Tensor(a!) bins, Tensor(b!) scratch, int ignore_index, bool has_ignore, Tensor(c!)? err_flag=None) -> bool");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("range_flag", &tmx::range_flag);
  m.impl("bincount", &tmx::bincount);
  m.impl("mc_confmat_update", &tmx::mc_confmat_update);
  m.impl("mc_stat_scores_update", &tmx::mc_stat_scores_update);
  m.impl("binary_stats_update", &tmx::binary_stats_update);
  m.impl("binary_stats_fused", &tmx::binary_stats_fused);
  m.impl("curve_hist_update", &tmx::curve_hist_update);
  m.impl("curve_hist_zero", &tmx::curve_hist_zero);
  m.impl("curve_hist_drain", &tmx::curve_hist_drain);
  m.impl("curve_hist_reduce", &tmx::curve_hist_reduce);
  m.impl("curve_summary", &tmx::curve_summary);
  m.impl("curve_hist_scores", &tmx::curve_hist_scores);
  m.impl("curve_mc_rowpass", &tmx::curve_mc_rowpass);
  m.impl("binned_curve_update", &tmx::binned_curve_update);
  m.impl("ce_bins_update", &tmx::ce_bins_update);
  m.impl("mc_calibration_update", &tmx::mc_calibration_update);
  m.impl("mc_calibration_fused", &tmx::mc_calibration_fused);
}
