// Collection-level fusion of the argmax statistics (SURVEY §7.1 "metrics reading the same inputs share one fused
// kernel"; reference compute groups: collections.py:200-307, which only share *states* of identical metrics).
//
// A MetricCollection that holds several multiclass metrics of the same C / ignore_index reads the [N, C] scores
// once: the row pass (the curve metric's exact-histogram kernel, or the plain argmax pair stream) counts the batch's
// (target, argmax) pairs into a scratch confusion matrix, and confmat_fold turns that one [C, C] delta into every
// member's state update:
//   * confusion-matrix members (ConfusionMatrix; Jaccard / CohenKappa / MCC keep the same state):  confmat += delta
//   * StatScores-family members (Accuracy, Precision, Recall, F-beta, Specificity, Hamming, StatScores; global top-1):
//       tp_c += delta[c, c],  fp_c += colsum_c - tp_c,  fn_c += rowsum_c - tp_c,  tn_c += N_valid - tp_c - fp_c - fn_c
//     (micro: the class sums and tn = C * N_valid - tp - fp - fn, the reference's multiclass micro convention)
// One launch: fold_rows (a block owns a 16-row x 256-column tile: adds it into the confusion-matrix states, the
// diagonal, row and column partial sums, and zeroes the delta for the next batch); the last block to finish folds the
// per-class deltas into every stat member and zeroes the sums.
#include "common.h"

namespace tmx {

constexpr int kFoldMax = 8;  // members per kind handled by one launch
constexpr int kFoldRows = 16;  // 16-row chunks: 4 x 63 blocks at C = 1000
constexpr int kFoldThreads = 256;

struct FoldCms {
  int64_t* p[kFoldMax];
  int n;
};

struct FoldStats {
  int64_t* tp[kFoldMax];
  int64_t* fp[kFoldMax];
  int64_t* tn[kFoldMax];
  int64_t* fn[kFoldMax];
  int micro[kFoldMax];
  int n;
};

// sums layout (int64, zero on entry): [0, C) row sums, [C, 2C) diagonal, [2C, 3C) column sums.
// Block (row chunk of 32, column tile of 256): every thread owns one column of the tile; its 32 loads are issued
// before any use; row partial sums are reduced in the block and added with one atomic per row and tile, column
// partial sums with one atomic per column and row chunk.
__device__ void fold_stats_body(int C, const FoldStats& st, int64_t* __restrict__ sums);

__global__ __launch_bounds__(kFoldThreads) void fold_rows_kernel(int64_t* __restrict__ delta, int C, FoldCms cms, FoldStats st,
                                                                 int64_t* __restrict__ sums) {
  __shared__ long long s_row[kFoldThreads / kWave][kFoldRows];
  const int r0 = blockIdx.y * kFoldRows;
  const int c = blockIdx.x * kFoldThreads + threadIdx.x;
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  long long v[kFoldRows];
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) v[i] = (r0 + i < C && c < C) ? delta[static_cast<int64_t>(r0 + i) * C + c] : 0;
  long long col = 0;
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) {
    if (v[i]) {
      const int64_t idx = static_cast<int64_t>(r0 + i) * C + c;
      // no-return atomics: fire-and-forget adds, so a thread never waits on the latency of a read-modify-write
      for (int m = 0; m < cms.n; ++m) atomic_add_i64(cms.p[m] + idx, v[i]);
      delta[idx] = 0;
      col += v[i];
      if (c == r0 + i) atomic_add_i64(sums + C + c, v[i]);  // atomic: read by another XCD's last workgroup
    }
  }
  if (col) atomic_add_i64(sums + 2 * C + c, col);
#pragma unroll
  for (int i = 0; i < kFoldRows; ++i) {
    const long long t = wave_sum(v[i]);
    if (lane == 0) s_row[wave][i] = t;
  }
  __syncthreads();
  if (threadIdx.x < kFoldRows && r0 + threadIdx.x < C) {
    long long t = 0;
    for (int w = 0; w < kFoldThreads / kWave; ++w) t += s_row[w][threadIdx.x];
    if (t) atomic_add_i64(sums + r0 + threadIdx.x, t);
  }
  if (st.n == 0) return;
  // last workgroup to finish folds the class sums into the stat members (one launch for the whole fold): every
  // thread's sum atomics are performed (vmcnt 0) before the workgroup takes its ticket
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    auto* ticket = reinterpret_cast<unsigned long long*>(sums + 3 * C);
    const unsigned long long nblk = (unsigned long long)gridDim.x * gridDim.y;
    s_last = atomicAdd(ticket, 1ull) == nblk - 1;
    if (s_last) atomicExch(ticket, 0ull);
  }
  __syncthreads();
  if (s_last) fold_stats_body(C, st, sums);
}

// Runs in the last workgroup of fold_rows: every other workgroup's sums are in place (ticket order); they are read
// with atomicExch (coherent read that also re-zeroes the scratch for the next batch).
__device__ void fold_stats_body(int C, const FoldStats& st, int64_t* __restrict__ sums) {
  __shared__ long long s_red[kFoldThreads / kWave][2];
  __shared__ long long s_tot[2];
  auto* u = reinterpret_cast<unsigned long long*>(sums);
  const int lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  // N_valid = sum of row sums (every valid row lands in exactly one row of the delta); micro tp = sum of diagonal
  long long nv = 0, dg = 0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    nv += (long long)__hip_atomic_load(u + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dg += (long long)__hip_atomic_load(u + C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  nv = wave_sum(nv);
  dg = wave_sum(dg);
  if (lane == 0) {
    s_red[wave][0] = nv;
    s_red[wave][1] = dg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long a = 0, b = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x / kWave); ++w) {
      a += s_red[w][0];
      b += s_red[w][1];
    }
    s_tot[0] = a;
    s_tot[1] = b;
  }
  __syncthreads();
  const long long N = s_tot[0], TP = s_tot[1];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const long long rs = (long long)atomicExch(u + c, 0ull), tp = (long long)atomicExch(u + C + c, 0ull),
                    cs = (long long)atomicExch(u + 2 * C + c, 0ull);
    const long long fp = cs - tp, fn = rs - tp, tn = N - tp - fp - fn;
    for (int m = 0; m < st.n; ++m) {
      if (st.micro[m]) continue;
      // exclusive owner per (member, class): no-return atomics, no wait on a read-modify-write
      atomic_add_i64(st.tp[m] + c, tp);
      atomic_add_i64(st.fp[m] + c, fp);
      atomic_add_i64(st.fn[m] + c, fn);
      atomic_add_i64(st.tn[m] + c, tn);
    }
  }
  if (threadIdx.x == 0) {
    const long long fp = N - TP;  // = fn
    for (int m = 0; m < st.n; ++m) {
      if (!st.micro[m]) continue;
      atomic_add_i64(st.tp[m], TP);
      atomic_add_i64(st.fp[m], fp);
      atomic_add_i64(st.fn[m], fp);
      atomic_add_i64(st.tn[m], static_cast<long long>(C) * N - TP - 2 * fp);
    }
  }
}

// delta: int64 [C, C] batch confusion matrix (zeroed on return); cms: confusion-matrix states (+= delta);
// stats: flattened (tp, fp, tn, fn) int64 states per member, micro[m] = 1 for a one-element (micro) state;
// sums: int64 [3 C + 1] zeroed scratch (class sums + ticket; zeroed again on return).
void confmat_fold(at::Tensor& delta, at::TensorList cms, at::TensorList stats, at::IntArrayRef micro, at::Tensor& sums) {
  TORCH_CHECK(delta.is_cuda() && delta.dim() == 2 && delta.size(0) == delta.size(1) && delta.scalar_type() == at::kLong &&
                  delta.is_contiguous(), "confmat_fold: delta must be a contiguous int64 [C, C] GPU tensor");
  const int C = static_cast<int>(delta.size(0));
  TORCH_CHECK(sums.is_contiguous() && sums.scalar_type() == at::kLong && sums.numel() == 3 * static_cast<int64_t>(C) + 1,
              "confmat_fold: sums must be int64 [3 C + 1] (class sums + the workgroup ticket)");
  TORCH_CHECK(static_cast<int64_t>(cms.size()) <= kFoldMax && stats.size() == 4 * micro.size() &&
                  static_cast<int64_t>(micro.size()) <= kFoldMax, "confmat_fold: too many members");
  const c10::DeviceGuard guard(delta.device());
  FoldCms fc{};
  fc.n = static_cast<int>(cms.size());
  for (int m = 0; m < fc.n; ++m) {
    TORCH_CHECK(cms[m].is_contiguous() && cms[m].scalar_type() == at::kLong && cms[m].numel() == delta.numel() &&
                    cms[m].device() == delta.device(), "confmat_fold: confusion-matrix state must be contiguous int64 [C, C]");
    fc.p[m] = cms[m].data_ptr<int64_t>();
  }
  FoldStats fs{};
  fs.n = static_cast<int>(micro.size());
  for (int m = 0; m < fs.n; ++m) {
    fs.micro[m] = micro[m] ? 1 : 0;
    const int64_t want = micro[m] ? 1 : C;
    int64_t** dst[4] = {fs.tp, fs.fp, fs.tn, fs.fn};
    for (int k = 0; k < 4; ++k) {
      const at::Tensor& t = stats[4 * m + k];
      TORCH_CHECK(t.is_contiguous() && t.scalar_type() == at::kLong && t.numel() == want && t.device() == delta.device(),
                  "confmat_fold: stat states must be contiguous int64 of ", want, " elements");
      dst[k][m] = t.data_ptr<int64_t>();
    }
  }
  if (C == 0) return;
  const dim3 grid((C + kFoldThreads - 1) / kFoldThreads, (C + kFoldRows - 1) / kFoldRows);
  fold_rows_kernel<<<grid, kFoldThreads, 0, stream()>>>(delta.data_ptr<int64_t>(), C, fc, fs, sums.data_ptr<int64_t>());
  TMX_LAUNCH_CHECK();
  if (fs.n == 0) sums.zero_();
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("confmat_fold(Tensor(a!) delta, Tensor(b!)[] cms, Tensor(c!)[] stats, int[] micro, Tensor(d!) sums) -> ()");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("confmat_fold", &tmx::confmat_fold); }
