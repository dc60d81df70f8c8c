// ``ter_gpu`` — Tercom translation edit rate on the GPU (host op ``ter_batch`` / translation_edit_rate
// in text.cpp; reference functional/text/ter.py + helper.py _LevenshteinEditDistance / _shift_words).
//
// One wave per (reference, hypothesis) pair (a = the reference words, shifted towards b = the hypothesis words), grid-
// strided over the pairs.  Each greedy round of the shift search:
//   1. lane 0 runs the beam DP with its operation table and walks the trace: alignment, error flags (prefix sums);
//   2. lane 0 enumerates the candidate shifts in the host op's order — (start, target start, length) groups, each
//      group's distinct insertion points — and stops after the group that takes the round's running candidate count
//      to the 1000 limit (the host's `goto done`);
//   3. the 64 lanes evaluate the candidates in parallel (shifted words in a lane-private scratch row, distance-only
//      beam DP with a band-reset single row) and a wave arg-max picks the best by (gain, length, -start, -insertion
//      point) — equal keys mean the same shift, so the host's final tie-break on the words never separates them;
//   4. the round's shift is applied unless the limit was reached or the gain is <= 0.
// Distances are small integers: int32 with a 1e9 "infinity" orders exactly as the host op's int64 1e16.
#include "common.h"

namespace tmx {
namespace {

constexpr int kTerInf = 1000000000;
constexpr int kTerBeam = 25;
constexpr int kTerMaxShiftSize = 10;
constexpr int kTerMaxShiftDist = 50;
constexpr int kTerMaxCandidates = 1000;
constexpr int kTerCandCap = kTerMaxCandidates + kTerMaxShiftSize + 1;  // the last group may overshoot by <= len + 1
enum TerOp : uint8_t { kOpNothing = 0, kOpSub = 1, kOpIns = 2, kOpDel = 3 };

struct TerBeam {
  int64_t beam;
  double ratio;
};
__device__ __forceinline__ TerBeam ter_beam(int n, int m) {
  const double ratio = n ? static_cast<double>(m) / static_cast<double>(n) : 1.0;
  return {(ratio / 2 > kTerBeam) ? static_cast<int64_t>(ceil(ratio / 2 + kTerBeam)) : kTerBeam, ratio};
}
__device__ __forceinline__ void ter_band(const TerBeam& bw, int i, int n, int m, int& lo, int& hi) {
  const int64_t diag = static_cast<int64_t>(floor(static_cast<double>(i) * bw.ratio));
  lo = static_cast<int>(diag - bw.beam > 0 ? diag - bw.beam : 0);
  hi = (i == n) ? m + 1 : static_cast<int>(diag + bw.beam < m + 1 ? diag + bw.beam : m + 1);
}

// distance-only beam DP (unit costs) with one row R[0..m] (row i - 1 on its band, inf elsewhere)
__device__ int ter_dist(const int* __restrict__ a, int n, const int* __restrict__ b, int m, int* __restrict__ R) {
  for (int j = 0; j <= m; ++j) R[j] = j;
  const TerBeam bw = ter_beam(n, m);
  int plo = 0, phi = m + 1;
  for (int i = 1; i <= n; ++i) {
    int lo, hi;
    ter_band(bw, i, n, m, lo, hi);
    const int ai = a[i - 1];
    int up_left = lo >= 1 ? R[lo - 1] : kTerInf, left = kTerInf;
    for (int j = lo; j < hi; ++j) {
      const int up = R[j];
      int c;
      if (j == 0) {
        c = up + 1;
      } else {
        c = kTerInf;
        const int cs = up_left + (ai == b[j - 1] ? 0 : 1), cd = up + 1, ci = left + 1;
        if (c > cs) c = cs;
        if (c > cd) c = cd;
        if (c > ci) c = ci;
      }
      R[j] = c;
      up_left = up;
      left = c;
    }
    for (int j = plo; j < lo && j < phi; ++j) R[j] = kTerInf;
    for (int j = hi > plo ? hi : plo; j < phi; ++j) R[j] = kTerInf;
    plo = lo;
    phi = hi;
  }
  return R[m];
}

// full table DP with operations (host lev_beam with `keep`): cost / op [(n + 1) (m + 1)]
__device__ int ter_dp_table(const int* __restrict__ a, int n, const int* __restrict__ b, int m, int* __restrict__ cost,
                            uint8_t* __restrict__ op) {
  const int W = m + 1;
  for (int k = 0; k < (n + 1) * W; ++k) {
    cost[k] = kTerInf;
    op[k] = 4;
  }
  for (int j = 0; j <= m; ++j) {
    cost[j] = j;
    op[j] = kOpIns;
  }
  const TerBeam bw = ter_beam(n, m);
  for (int i = 1; i <= n; ++i) {
    int lo, hi;
    ter_band(bw, i, n, m, lo, hi);
    for (int j = lo; j < hi; ++j) {
      int& c = cost[i * W + j];
      uint8_t& o = op[i * W + j];
      if (j == 0) {
        c = cost[(i - 1) * W] + 1;
        o = kOpDel;
        continue;
      }
      const bool same = a[i - 1] == b[j - 1];
      const int cs = cost[(i - 1) * W + j - 1] + (same ? 0 : 1);
      const int cd = cost[(i - 1) * W + j] + 1;
      const int ci = cost[i * W + j - 1] + 1;
      if (c > cs) { c = cs; o = same ? kOpNothing : kOpSub; }
      if (c > cd) { c = cd; o = kOpDel; }
      if (c > ci) { c = ci; o = kOpIns; }
    }
  }
  return cost[n * W + m];
}

// host perform_shift with clamped slices
__device__ __forceinline__ void ter_append(int* __restrict__ dst, int& k, const int* __restrict__ w, int n, int s, int e) {
  s = s < 0 ? 0 : (s > n ? n : s);
  e = e < 0 ? 0 : (e > n ? n : e);
  for (int x = s; x < e; ++x) dst[k++] = w[x];
}
__device__ void ter_shift(const int* __restrict__ w, int n, int start, int length, int target, int* __restrict__ out) {
  int k = 0;
  if (target < start) {
    ter_append(out, k, w, n, 0, target);
    ter_append(out, k, w, n, start, start + length);
    ter_append(out, k, w, n, target, start);
    ter_append(out, k, w, n, start + length, n);
  } else if (target > start + length) {
    ter_append(out, k, w, n, 0, start);
    ter_append(out, k, w, n, start + length, target);
    ter_append(out, k, w, n, start, start + length);
    ter_append(out, k, w, n, target, n);
  } else {
    ter_append(out, k, w, n, 0, start);
    ter_append(out, k, w, n, start + length, length + target);
    ter_append(out, k, w, n, start, start + length);
    ter_append(out, k, w, n, length + target, n);
  }
}

// candidate order: larger is better
__device__ __forceinline__ bool ter_better(int s1, int l1, int p1, int i1, int s2, int l2, int p2, int i2) {
  if (s1 != s2) return s1 > s2;
  if (l1 != l2) return l1 > l2;
  if (p1 != p2) return p1 < p2;  // -start larger
  return i1 < i2;                // -idx larger
}

struct TerWaveScratch {
  int* cur;      // [maxA]
  int* dpc;      // [(maxA + 1) (maxB + 1)]
  uint8_t* dpo;  // [(maxA + 1) (maxB + 1)]
  uint8_t* tr;   // [maxA + maxB]
  int* align;    // [maxB]
  int* aerr;     // prefix sums [maxA + 1]
  int* berr;     // prefix sums [maxB + 1]
  int* cand;     // [kTerCandCap][3]: start, length, insertion point
  int* lane_w;   // [64][maxA]
  int* lane_r;   // [64][maxB + 1]
};

}  // namespace

__global__ __launch_bounds__(64) void ter_pair_kernel(const int* __restrict__ A, const int64_t* __restrict__ A_off, const int* __restrict__ B,
                                                     const int64_t* __restrict__ B_off, int64_t P, int maxA, int maxB,
                                                     int* __restrict__ scratch, int64_t per_wave_ints, double* __restrict__ out) {
  const int lane = threadIdx.x;
  int* base = scratch + blockIdx.x * per_wave_ints;
  TerWaveScratch s;
  s.cur = base;
  s.dpc = s.cur + maxA;
  s.align = s.dpc + (maxA + 1) * (maxB + 1);
  s.aerr = s.align + maxB;
  s.berr = s.aerr + maxA + 1;
  s.cand = s.berr + maxB + 1;
  s.lane_w = s.cand + 3 * kTerCandCap;
  s.lane_r = s.lane_w + 64 * maxA;
  s.dpo = reinterpret_cast<uint8_t*>(s.lane_r + 64 * (maxB + 1));
  s.tr = s.dpo + (maxA + 1) * (maxB + 1);
  __shared__ int s_info[4];  // candidates this round, limit reached, round distance

  for (int64_t p = blockIdx.x; p < P; p += gridDim.x) {
    const int n = static_cast<int>(A_off[p + 1] - A_off[p]);
    const int m = static_cast<int>(B_off[p + 1] - B_off[p]);
    const int* b = B + B_off[p];
    if (m == 0) {  // empty hypothesis: 0 edits (host translation_edit_rate)
      if (lane == 0) out[p] = 0.0;
      continue;
    }
    for (int k = lane; k < n; k += 64) s.cur[k] = A[A_off[p] + k];
    __syncthreads();
    int shifts = 0, checked = 0;
    while (true) {
      // 1-2. trace, alignment, candidate enumeration (lane 0)
      if (lane == 0) {
        const int dist = ter_dp_table(s.cur, n, b, m, s.dpc, s.dpo);
        // backward trace, flipped (Ins <-> Del: rewrite b into a), stored forward
        int len = 0, i = n, j = m;
        const int W = m + 1;
        while (i > 0 || j > 0) {
          const uint8_t o = s.dpo[i * W + j];
          s.tr[len++] = o;
          if (o == kOpSub || o == kOpNothing) { --i; --j; }
          else if (o == kOpIns) { --j; }
          else { --i; }  // kOpDel (the beam always reaches (0, 0) through defined cells)
        }
        for (int k = 0; k < m; ++k) s.align[k] = -2;
        int rp = -1, hp = -1, na = 0, nb = 0;
        s.aerr[0] = 0;
        s.berr[0] = 0;
        for (int k = len - 1; k >= 0; --k) {
          uint8_t o = s.tr[k];
          o = o == kOpIns ? kOpDel : (o == kOpDel ? kOpIns : o);
          if (o == kOpNothing || o == kOpSub) {
            ++hp; ++rp;
            s.align[rp] = hp;
            s.berr[nb + 1] = s.berr[nb] + (o == kOpSub); ++nb;
            s.aerr[na + 1] = s.aerr[na] + (o == kOpSub); ++na;
          } else if (o == kOpIns) {
            ++hp;
            s.aerr[na + 1] = s.aerr[na] + 1; ++na;
          } else {
            ++rp;
            s.align[rp] = hp;
            s.berr[nb + 1] = s.berr[nb] + 1; ++nb;
          }
        }
        auto rsum = [&](const int* pre, int cnt, int st, int en) {
          st = st < 0 ? 0 : st;
          en = en > cnt ? cnt : en;
          return en > st ? pre[en] - pre[st] : 0;
        };
        int nc = 0;
        bool limit = false;
        for (int ps = 0; ps < n && !limit; ++ps) {
          for (int ts = 0; ts < m && !limit; ++ts) {
            if (abs(ts - ps) > kTerMaxShiftDist) continue;
            for (int ln = 1; ln < kTerMaxShiftSize; ++ln) {
              if (s.cur[ps + ln - 1] != b[ts + ln - 1]) break;
              bool skip = rsum(s.aerr, na, ps, ps + ln) == 0 || rsum(s.berr, nb, ts, ts + ln) == 0;
              if (!skip) {
                const int al = s.align[ts];
                skip = ps <= al && al < ps + ln;
              }
              if (!skip) {
                int prev_idx = -1;
                for (int off = -1; off < ln; ++off) {
                  int idx;
                  if (ts + off == -1) idx = 0;
                  else if (ts + off < m && s.align[ts + off] != -2) idx = s.align[ts + off] + 1;
                  else break;
                  if (idx == prev_idx) continue;
                  prev_idx = idx;
                  s.cand[3 * nc] = ps;
                  s.cand[3 * nc + 1] = ln;
                  s.cand[3 * nc + 2] = idx;
                  ++nc;
                  ++checked;
                }
                if (checked >= kTerMaxCandidates) { limit = true; break; }
              }
              if (ps + ln == n || ts + ln == m) break;
            }
          }
        }
        s_info[0] = nc;
        s_info[1] = limit ? 1 : 0;
        s_info[2] = dist;
      }
      __syncthreads();
      const int nc = s_info[0], limit = s_info[1], dist = s_info[2];
      // 3. candidates in parallel, wave arg-max
      int bs = -kTerInf, bl = 0, bp = 0, bi = 0;
      bool have = false;
      int* w = s.lane_w + lane * maxA;
      int* R = s.lane_r + lane * (maxB + 1);
      for (int c = lane; c < nc; c += 64) {
        const int ps = s.cand[3 * c], ln = s.cand[3 * c + 1], idx = s.cand[3 * c + 2];
        ter_shift(s.cur, n, ps, ln, idx, w);
        const int gain = dist - ter_dist(w, n, b, m, R);
        if (!have || ter_better(gain, ln, ps, idx, bs, bl, bp, bi)) {
          bs = gain; bl = ln; bp = ps; bi = idx;
          have = true;
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const int os = __shfl_xor(bs, off, 64), ol = __shfl_xor(bl, off, 64), op = __shfl_xor(bp, off, 64),
                  oi = __shfl_xor(bi, off, 64), oh = __shfl_xor(have ? 1 : 0, off, 64);
        if (oh && (!have || ter_better(os, ol, op, oi, bs, bl, bp, bi))) {
          bs = os; bl = ol; bp = op; bi = oi;
          have = true;
        }
      }
      // 4. apply the round's best shift (host: stop when the limit was reached or the gain is not positive)
      if (nc == 0 || limit || bs <= 0) break;
      ++shifts;
      if (lane == 0) {
        ter_shift(s.cur, n, bp, bl, bi, w);
        for (int k = 0; k < n; ++k) s.cur[k] = w[k];
      }
      __syncthreads();
    }
    __syncthreads();
    if (lane == 0) out[p] = static_cast<double>(shifts + ter_dist(s.cur, n, b, m, s.lane_r));
    __syncthreads();
  }
}

// a: flat reference words (int32 ids), b: flat hypothesis words, one pair per (a, b) segment; returns fp64 edits [P]
at::Tensor ter_gpu(const at::Tensor& a, const at::Tensor& a_off, const at::Tensor& b, const at::Tensor& b_off, int64_t max_a, int64_t max_b) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kInt && b.scalar_type() == at::kInt, "ter_gpu: int32 GPU word ids");
  TORCH_CHECK(a_off.is_cuda() && b_off.is_cuda() && a_off.scalar_type() == at::kLong && b_off.scalar_type() == at::kLong,
              "ter_gpu: int64 GPU offsets");
  TORCH_CHECK(a_off.numel() == b_off.numel(), "ter_gpu: pair count mismatch");
  TORCH_CHECK(max_a >= 0 && max_b >= 0 && max_a < 4096 && max_b < 4096, "ter_gpu: sentences up to 4095 words");
  const c10::DeviceGuard guard(a.device());
  const int64_t P = a_off.numel() - 1;
  auto out = at::empty({std::max<int64_t>(P, 0)}, a.options().dtype(at::kDouble));
  if (P <= 0) return out;
  {  // the scratch is sized by max_a / max_b: check them against the offsets (one small host read)
    auto ao = a_off.cpu(), bo = b_off.cpu();
    const int64_t *pa = ao.data_ptr<int64_t>(), *pb = bo.data_ptr<int64_t>();
    for (int64_t k = 0; k < P; ++k)
      TORCH_CHECK(pa[k + 1] - pa[k] <= max_a && pb[k + 1] - pb[k] <= max_b && pa[k + 1] >= pa[k] && pb[k + 1] >= pb[k],
                  "ter_gpu: a sentence is longer than max_a / max_b");
  }
  const int64_t A1 = max_a + 1, B1 = max_b + 1;
  const int64_t tbl = A1 * B1;
  // ints: cur + dp cost + align + prefix sums + candidates + lane rows; bytes after: dp ops + trace (rounded up to ints)
  const int64_t per_wave = max_a + tbl + max_b + A1 + B1 + 3 * kTerCandCap + 64 * max_a + 64 * B1 + (tbl + max_a + max_b + 3) / 4 + 4;
  // resident waves: enough to fill the chip (4 per CU), scratch capped at ~512 MB for long sentences
  const int64_t waves = std::max<int64_t>(1, std::min<int64_t>({P, 1024, (int64_t{128} << 20) / per_wave}));
  auto scratch = at::empty({waves * per_wave}, a.options().dtype(at::kInt));
  const auto ac = a.contiguous(), bc = b.contiguous(), aoc = a_off.contiguous(), boc = b_off.contiguous();
  hipLaunchKernelGGL(ter_pair_kernel, dim3(static_cast<unsigned>(waves)), 64, 0, stream(), ac.data_ptr<int>(), aoc.data_ptr<int64_t>(),
                     bc.data_ptr<int>(), boc.data_ptr<int64_t>(), P, static_cast<int>(max_a), static_cast<int>(max_b),
                     scratch.data_ptr<int>(), per_wave, out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("ter_gpu(Tensor a, Tensor a_off, Tensor b, Tensor b_off, int max_a, int max_b) -> Tensor"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("ter_gpu", &tmx::ter_gpu); }
