// SSIM window kernels (device code only; shared by csrc/image.hip and the standalone harness
// tools/kexp/ssim_mfma_exp.hip).  See image.hip for the op-level documentation.
#pragma once

#include "device_common.h"

namespace tmx {

constexpr int kSsimThreads = 256;

// ------------------------------------------------------------------------------------------------------------
// fp32, W % 4 == 0, 16-B aligned planes (the common case): the same valid-window algorithm, restructured for
// throughput (the one-row-per-barrier kernel above ran at 0.78 TB/s on 256 x 3 x 1024^2):
//   * KS input rows are staged per barrier, prefetched into registers with 16-B loads while the previous group is
//     computed (one barrier per KS rows instead of per row);
//   * (p, t) are interleaved in LDS as float2, so one 8-B LDS read feeds both images, and the moment arithmetic runs
//     on packed fp32 pairs (v_pk_mul / v_pk_add / v_pk_fma): (mu_p, mu_t) and (E[pp], E[tt]) share instructions,
//     ~4 instructions per horizontal tap and 3 per vertical tap instead of 7 and 5;
//   * strips of kRowsV2 output rows per block halve the KS - 1 halo rows' share of the reads.
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kRowsV2 = 128;

// SSE (fused PSNR of a MetricCollection{SSIM, PSNR}): every input pixel is owned by exactly one block (rows
// [y0, y0 + kRowsV2) and columns [x0, x0 + 256), the last strip / column block up to H / W), and its (p - t)^2 is
// added while the block stages it anyway: PSNR needs no second pass over the two images.
template <int KS, bool SSE>
__global__ __launch_bounds__(kSsimThreads, 2) void ssim_v2_kernel(const float* __restrict__ preds, const float* __restrict__ target,
                                                                int H, int W, const float* __restrict__ wx,
                                                                const float* __restrict__ wy, const float* __restrict__ consts,
                                                                double* __restrict__ partial_sim, double* __restrict__ partial_cs,
                                                                double* __restrict__ partial_sse, const int* __restrict__ run_if = nullptr) {
  constexpr int kSeg4 = (kSsimThreads + KS - 1 + 3) / 4;   // float4 columns per staged row segment
  constexpr int kSegF = kSeg4 * 4;
  constexpr int kItems = KS * kSeg4;                       // (row, column quad) items per group
  constexpr int kPer = (kItems + kSsimThreads - 1) / kSsimThreads;
  __shared__ f2 s_pt[2][KS][kSegF];
  __shared__ double red[3][kSsimThreads / kWave];
  // the MFMA kernel's fallback launch (ssim_sums): runs only when that kernel flagged out-of-range inputs
  if (run_if != nullptr && __hip_atomic_load(run_if, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;

  const int Hv = H - KS + 1, Wv = W - KS + 1;
  const int64_t plane = blockIdx.z;
  const int x0 = blockIdx.x * kSsimThreads;
  const int y0 = blockIdx.y * kRowsV2;
  const int tid = threadIdx.x;
  const float* P = preds + plane * static_cast<int64_t>(H) * W;
  const float* Tt = target + plane * static_cast<int64_t>(H) * W;
  const float c1 = consts[0], c2 = consts[1];
  f2 wx2[KS], wy2[KS];  // weights pre-splatted into packed pairs (no per-tap register moves)
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    wx2[k] = f2{wx[k], wx[k]};
    wy2[k] = f2{wy[k], wy[k]};
  }
  const int out_rows = min(kRowsV2, Hv - y0);
  const int in_rows = out_rows + KS - 1;
  const bool col_ok = (x0 + tid) < Wv;

  float4 pre_p[kPer], pre_t[kPer];
  auto fetch = [&](int g) {  // group g = input rows y0 + g KS .. + KS - 1 into registers
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kSsimThreads;
      const int r = e / kSeg4, q = e % kSeg4;
      const int y = y0 + g * KS + r, x = x0 + 4 * q;
      const bool ok = e < kItems && g * KS + r < in_rows && x < W;  // W % 4 == 0: a quad is all in or all out
      const int64_t o = static_cast<int64_t>(y) * W + x;
      pre_p[i] = ok ? *reinterpret_cast<const float4*>(P + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      pre_t[i] = ok ? *reinterpret_cast<const float4*>(Tt + o) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kSsimThreads;
      if (e < kItems) {
        const int r = e / kSeg4, q = e % kSeg4;
        f2* d = &s_pt[buf][r][4 * q];
        d[0] = f2{pre_p[i].x, pre_t[i].x};
        d[1] = f2{pre_p[i].y, pre_t[i].y};
        d[2] = f2{pre_p[i].z, pre_t[i].z};
        d[3] = f2{pre_p[i].w, pre_t[i].w};
      }
    }
  };

  // ring of horizontal sums for the last KS rows: (mu_p, mu_t), (E[pp], E[tt]) packed, E[pt] scalar
  f2 rm[KS], rq[KS];
  float rx[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    rm[k] = f2{0.f, 0.f};
    rq[k] = f2{0.f, 0.f};
    rx[k] = 0.f;
  }
  double acc_sim = 0.0, acc_cs = 0.0, acc_sse = 0.0;
  float f_sim = 0.f, f_cs = 0.f, f_sse = 0.f;
  // owned input pixels (SSE): rows r < own_rows, this thread's column, plus columns 256 .. for the last column block
  const bool last_x = blockIdx.x == gridDim.x - 1, last_y = blockIdx.y == gridDim.y - 1;
  const int own_rows = last_y ? in_rows : out_rows;
  const bool own_col = x0 + tid < W && (last_x || tid < kSsimThreads);
  const bool own_col2 = last_x && tid < KS - 1 && x0 + kSsimThreads + tid < W;
  const int groups = (in_rows + KS - 1) / KS;
  if (groups > 0) {
    fetch(0);
    store(0);
  }
  __syncthreads();
  for (int g = 0; g < groups; ++g) {
    const int buf = g & 1;
    if (g + 1 < groups) fetch(g + 1);  // in flight during this group's arithmetic
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      const int r = g * KS + j;
      if (r < in_rows) {  // block-uniform
        f2 hm = f2{0.f, 0.f}, hq = f2{0.f, 0.f};
        float hx = 0.f;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const f2 v = s_pt[buf][j][tid + k];
          const f2 wv = wx2[k] * v;                        // (w p, w t)
          hm += wv;
          hq = __builtin_elementwise_fma(wv, v, hq);       // (w p p, w t t)
          hx = fmaf(wv.x, v.y, hx);                        // w p t
        }
        rm[j] = hm;
        rq[j] = hq;
        rx[j] = hx;
        if constexpr (SSE) {
          if (r < own_rows) {
            if (own_col) {
              const f2 v = s_pt[buf][j][tid];
              const float d = v.x - v.y;
              f_sse = fmaf(d, d, f_sse);
            }
            if (own_col2) {
              const f2 v = s_pt[buf][j][kSsimThreads + tid];
              const float d = v.x - v.y;
              f_sse = fmaf(d, d, f_sse);
            }
          }
        }
        if (r >= KS - 1 && col_ok) {
          f2 m01 = f2{0.f, 0.f}, m23 = f2{0.f, 0.f};
          float m4 = 0.f;
#pragma unroll
          for (int k = 0; k < KS; ++k) {
            const int slot = (j + 1 + k) % KS;  // oldest first
            m01 = __builtin_elementwise_fma(wy2[k], rm[slot], m01);
            m23 = __builtin_elementwise_fma(wy2[k], rq[slot], m23);
            m4 = fmaf(wy2[k].x, rx[slot], m4);
          }
          const float mu_pp = m01.x * m01.x, mu_tt = m01.y * m01.y, mu_pt = m01.x * m01.y;
          const float upper = 2.f * (m4 - mu_pt) + c2;
          const float lower = (m23.x - mu_pp) + (m23.y - mu_tt) + c2;
          // hardware reciprocals (1 ulp) instead of two IEEE divisions (~10 instructions each)
          const float cs = upper * __builtin_amdgcn_rcpf(lower);
          const float sim = (2.f * mu_pt + c1) * cs * __builtin_amdgcn_rcpf(mu_pp + mu_tt + c1);
          f_sim += sim;  // <= kRowsV2 terms per thread in fp32, folded into fp64 per group
          f_cs += cs;
        }
      }
    }
    acc_sim += static_cast<double>(f_sim);
    acc_cs += static_cast<double>(f_cs);
    acc_sse += static_cast<double>(f_sse);
    f_sim = f_cs = f_sse = 0.f;
    if (g + 1 < groups) {
      store(buf ^ 1);  // the other buffer was last read in group g - 1, before the previous barrier
      __syncthreads();
    }
  }
  acc_sim = wave_sum(acc_sim);
  acc_cs = wave_sum(acc_cs);
  if constexpr (SSE) acc_sse = wave_sum(acc_sse);
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  if (lane == 0) {
    red[0][wave] = acc_sim;
    red[1][wave] = acc_cs;
    red[2][wave] = acc_sse;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0, c = 0.0, e = 0.0;
    for (int w = 0; w < kSsimThreads / kWave; ++w) {
      s += red[0][w];
      c += red[1][w];
      e += red[2][w];
    }
    const int64_t idx = (plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    partial_sim[idx] = s;
    partial_cs[idx] = c;
    if constexpr (SSE) partial_sse[idx] = e;
  }
}


// ------------------------------------------------------------------------------------------------------------
// Round 6: the separable window on the matrix cores (fp32 inputs, KS <= 17, W % 4 == 0, 16-B aligned planes).
//
// Both 1-D passes are banded matrix products on v_mfma_f32_16x16x32_f16, one wave per 16-column output tile, marching
// down a strip of output rows in 16-row steps:
//   horizontal  h[16 rows][16 cols]  = In[16 rows][32 input cols] . Bx[32][16],  Bx[x][c] = w[x - c]  (0 <= x - c < KS)
//   vertical    v[16 rows][16 cols]  = Ay[16][32 h rows] . [h_prev; h_cur][32][16], Ay[i][r] = w[r - i]
// The horizontal result's accumulator layout (lane l: col l & 15, rows 4 (l >> 4) .. + 3) IS the vertical product's
// B operand once the two 16-row tiles are interleaved along K (lane group g takes h rows 4g .. 4g + 3 of the previous
// tile and of the current one as its 8 K slots; Ay is built in that K order): no LDS round trip, no lane movement.
// Exactness: every fp32 operand is split into two fp16 halves, x = hi + lo with hi = RNE16(x), lo = RNE16(x - hi)
// (|x - hi - lo| <= 2^-23 |x|, unbiased), and each product is hi.hi + hi.lo + lo.hi with fp32 accumulation (the
// omitted lo.lo is below 2^-22 of a term): the window moments agree with the fp32 VALU kernel to ~1e-7 relative.
// Four moments, not five: SSIM reads E[p^2] and E[t^2] only through their sum, so one window of (p^2 + t^2) serves.
// fp16's range is met by exact power-of-two scaling: scores are multiplied by alpha = 2^(7 - ceil(log2 data_range)),
// squares by alpha^2 / 256 and the weights by 64, so every fp16 operand stays below 2^13.5 and above the subnormals
// for all but values 2^-21 below the window's largest; SSIM is evaluated in those scaled units with c1, c2 scaled
// alike (SSIM is invariant to the common scale).  A lane that meets a pixel pair with p^2 + t^2 above 2^15 in scaled
// units (|(p, t)| beyond 1.41-2.8 data_range, depending on how far data_range is below a power of two) or a NaN / inf
// sets ``fallback``: the op then runs ssim_v2_kernel for the batch
// (a launch that exits at once otherwise) and takes its sums -- no host synchronisation either way.
// The kernel is VALU-issue bound (SQ_ACTIVE_INST_VALU ~90 % of the wave time, profiles/ssim_mfma_pmc_r6.json): per
// band and lane the work is the scaling / products (packed fp32, two columns per instruction), the fp16 splits
// (three instructions per pair), 24 MFMAs and a packed epilogue over two output rows at a time; interior bands load
// without the edge selects.
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
constexpr int kSsimMfmaWaves = 4;    // independent waves (column tiles) per workgroup
#ifndef TMX_SSIM_DEPTH
#define TMX_SSIM_DEPTH 1  // input bands in flight per wave: 1 (128 VGPRs, 4 waves / SIMD) measured 2.44-2.52 vs 2.69-2.75 ms for 2
#endif
constexpr float kSsimMfmaQBound = 128.f;  // (p^2 + t^2) / 256 in scaled units: |p|, |t| <= 2^7.5 for the fp16 operands

// two fp32 values -> (hi pair, lo pair) of packed fp16: hi = v_cvt_pk_f16_f32 (RNE), lo = RNE16(x - hi) by
// v_fma_mix{lo,hi}_f16 reading hi's f16 halves directly (the fma's exact x - hi, one rounding to f16): three
// instructions per pair instead of five (convert back, packed subtract, convert)
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
  typedef float f2x __attribute__((ext_vector_type(2)));
  typedef _Float16 h2x __attribute__((ext_vector_type(2)));
  const h2x h = __builtin_convertvector(f2x{a, b}, h2x);
  hi = __builtin_bit_cast(uint32_t, h);
  uint32_t l;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hi), "v"(a));
  asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(hi), "v"(b));
  lo = l;
}
template <int N>
__device__ __forceinline__ void split_n(const float* v, uint32_t* hi, uint32_t* lo) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) split_pair(v[2 * k], v[2 * k + 1], hi[k], lo[k]);
}
__device__ __forceinline__ h8_t as_h8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(h8_t, u4_t{a, b, c, d});
}
__device__ __forceinline__ f4_t mfma3(h8_t ahi, h8_t alo, h8_t bhi, h8_t blo, f4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bhi, acc, 0, 0, 0);  // the small terms first
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bhi, acc, 0, 0, 0);
}

// grid: x = ceil(col tiles / 4) (four 16-column tiles per workgroup, one per wave), y = row strips of ``strip`` output
// rows (a multiple of 16), z = planes.  ``consts`` (device, fp32): c1, c2, data_range.
// Partials: fp64 [planes][strips][col tiles] of the SSIM / CS (/ SSE) sums.
template <bool SSE>
__global__ __launch_bounds__(kSsimMfmaWaves * kWave) void ssim_mfma_kernel(
    const float* __restrict__ preds, const float* __restrict__ target, int H, int W, int KS, int strip,
    const float* __restrict__ w, const float* __restrict__ consts, double* __restrict__ part_sim, double* __restrict__ part_cs,
    double* __restrict__ part_sse, int* __restrict__ fallback) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int Hv = H - KS + 1, Wv = W - KS + 1;
  const int ntx = (Wv + 15) / 16;
  const int ct = blockIdx.x * kSsimMfmaWaves + wave;
  if (ct >= ntx) return;  // (no workgroup-level synchronisation below)
  const int64_t plane = blockIdx.z;
  const int c0 = ct * 16;
  const int oy0 = blockIdx.y * strip;
  const int orows = min(strip, Hv - oy0);
  const int nb = (orows + 15) / 16 + 1;  // input bands: one more than output tiles (the KS - 1 halo)
  const float* Pp = preds + plane * static_cast<int64_t>(H) * W;
  const float* Tp = target + plane * static_cast<int64_t>(H) * W;
  const int i16 = lane & 15, g = lane >> 4;
  // alpha = 2^(7 - ceil(log2 D)) (exact power of two; 1 for a degenerate range: the range check then decides)
  const float D = consts[2];
  const float alpha = D > 0.f && D <= 3.0e38f ? __builtin_ldexpf(1.f, 7 - static_cast<int>(__builtin_ceilf(__builtin_log2f(D)))) : 1.f;
  const float U2 = (4096.f * alpha) * (4096.f * alpha);
  const float c1 = consts[0] * U2, c2 = consts[1] * U2;

  // band operands (constants of the launch): Bx[x][c] = 64 w[x - c] for lane (c = i16, x = 8 g + j);
  // Ay[i][r] = 64 w[r - i] for lane (i = i16, K slot 8 g + j = h row r(g, j)).  The vertical B operand is one
  // 4-register tuple per moment whose halves alternate roles band by band (no register moves): even bands write the
  // new h rows into the upper half (K order previous | current, r(g, j) = j < 4 ? 4 g + j : 16 + 4 g + j - 4), odd
  // bands into the lower half (current | previous, the second Ay)
  uint32_t bxh[4], bxl[4], ayh[2][4], ayl[2][4];
  {
    float bx[8], ay0[8], ay1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int dx = 8 * g + j - i16;
      bx[j] = dx >= 0 && dx < KS ? 64.f * w[dx] : 0.f;
      const int r0 = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4), r1 = j < 4 ? 16 + 4 * g + j : 4 * g + (j - 4);
      ay0[j] = r0 - i16 >= 0 && r0 - i16 < KS ? 64.f * w[r0 - i16] : 0.f;
      ay1[j] = r1 - i16 >= 0 && r1 - i16 < KS ? 64.f * w[r1 - i16] : 0.f;
    }
    split_n<8>(bx, bxh, bxl);
    split_n<8>(ay0, ayh[0], ayl[0]);
    split_n<8>(ay1, ayh[1], ayl[1]);
  }
  const h8_t BXH = as_h8(bxh[0], bxh[1], bxh[2], bxh[3]), BXL = as_h8(bxl[0], bxl[1], bxl[2], bxl[3]);
  const h8_t AYH[2] = {as_h8(ayh[0][0], ayh[0][1], ayh[0][2], ayh[0][3]), as_h8(ayh[1][0], ayh[1][1], ayh[1][2], ayh[1][3])};
  const h8_t AYL[2] = {as_h8(ayl[0][0], ayl[0][1], ayl[0][2], ayl[0][3]), as_h8(ayl[1][0], ayl[1][1], ayl[1][2], ayl[1][3])};

  // this lane's input vectors of band b: row oy0 + 16 b + i16, columns c0 + 8 g .. + 7 (W % 4 == 0: whole float4s)
  const int xc = c0 + 8 * g;
  const bool x_ok0 = xc < W, x_ok1 = xc + 4 < W;
  float4 np0, np1, nt0, nt1;  // band b + 2 in flight (fetch)
  float4 cp0, cp1, ct0, ct1;  // band b + 1 (arrived or arriving)
  // every lane loads (a masked lane reads the plane's first vector) and zeroes what lies outside the image: no
  // divergent loads, no stack temporaries for the selects
  auto ld = [](const float* base, int64_t o, bool ok) -> float4 {
    float4 v = *reinterpret_cast<const float4*>(base + (ok ? o : 0));
    v.x = ok ? v.x : 0.f;
    v.y = ok ? v.y : 0.f;
    v.z = ok ? v.z : 0.f;
    v.w = ok ? v.w : 0.f;
    return v;
  };
  const bool cols_in = c0 + 32 <= W;  // every lane's 8 columns inside the image (wave-uniform)
  auto fetch = [&](int b) {
    const int y = oy0 + 16 * b + i16;
    const int64_t o = static_cast<int64_t>(y) * W + xc;
    if (cols_in && oy0 + 16 * b + 16 <= H && b < nb) {  // interior band (uniform): plain loads, no selects
      np0 = *reinterpret_cast<const float4*>(Pp + o);
      np1 = *reinterpret_cast<const float4*>(Pp + o + 4);
      nt0 = *reinterpret_cast<const float4*>(Tp + o);
      nt1 = *reinterpret_cast<const float4*>(Tp + o + 4);
      return;
    }
    const bool y_ok = y < H && b < nb;
    np0 = ld(Pp, o, y_ok && x_ok0);
    np1 = ld(Pp, o + 4, y_ok && x_ok1);
    nt0 = ld(Tp, o, y_ok && x_ok0);
    nt1 = ld(Tp, o + 4, y_ok && x_ok1);
  };
  // SSE ownership: input rows [oy0, oy0 + strip) (the last strip: to H), columns [c0, c0 + 16) (the last tile: to W)
  const bool last_strip = blockIdx.y == gridDim.y - 1, last_tile = ct == ntx - 1;
  const int own_row_end = last_strip ? H : oy0 + strip;
  const bool own_lo = g < 2 || last_tile;

  u4_t vh[4], vl[4];  // per moment: the vertical B operand (h rows of two bands, split), halves alternating
  double acc_sim = 0.0, acc_cs = 0.0, acc_sse = 0.0;
  bool bad = false;
  const f2 c1v = {c1, c1}, c2v = {c2, c2};
#if TMX_SSIM_DEPTH == 2
  // two bands in flight: a band's loads are issued two band computations before its use
  fetch(0);
  cp0 = np0; cp1 = np1; ct0 = nt0; ct1 = nt1;
  fetch(1);
#else
  // one band in flight (16 fewer VGPRs: 4 waves per SIMD instead of 3)
  fetch(0);
#endif
  auto band = [&](const int b, auto par_c) {
    constexpr int par = decltype(par_c)::value;  // b & 1
    // (p, t) pairs of the lane's 8 columns, packed as f2 {p, t}... -- the packed ops below take two columns at once
#if TMX_SSIM_DEPTH == 2
    const f2 P[4] = {f2{cp0.x, cp0.y}, f2{cp0.z, cp0.w}, f2{cp1.x, cp1.y}, f2{cp1.z, cp1.w}};
    const f2 T[4] = {f2{ct0.x, ct0.y}, f2{ct0.z, ct0.w}, f2{ct1.x, ct1.y}, f2{ct1.z, ct1.w}};
    cp0 = np0; cp1 = np1; ct0 = nt0; ct1 = nt1;
    if (b + 2 < nb) fetch(b + 2);
#else
    const f2 P[4] = {f2{np0.x, np0.y}, f2{np0.z, np0.w}, f2{np1.x, np1.y}, f2{np1.z, np1.w}};
    const f2 T[4] = {f2{nt0.x, nt0.y}, f2{nt0.z, nt0.w}, f2{nt1.x, nt1.y}, f2{nt1.z, nt1.w}};
    if (b + 1 < nb) fetch(b + 1);
#endif
    float f_sse = 0.f;
    if constexpr (SSE) {
      const int y = oy0 + 16 * b + i16;
      if (own_lo && y < own_row_end && y < H) {
        f2 e = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f2 d = P[j] - T[j];
          e = __builtin_elementwise_fma(d, d, e);  // (zero-filled columns past W add 0)
        }
        f_sse = e.x + e.y;
      }
    }
    // scaled scores, their range check (NaN-propagating maximum: a NaN / inf fails it) and the four moment inputs
    // in scaled units: p, t, (p^2 + t^2) / 256, p t / 256 (SSIM needs E[p^2] + E[t^2] only as a sum)
    const f2 av = {alpha, alpha}, kv = {0.00390625f, 0.00390625f};
    f2 ps[4], ts[4], qs[4], rs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ps[j] = P[j] * av;
      ts[j] = T[j] * av;
      const f2 tk = ts[j] * kv;
      qs[j] = __builtin_elementwise_fma(ps[j], ps[j] * kv, ts[j] * tk);
      rs[j] = ps[j] * tk;
    }
    // range check on (p^2 + t^2) / 256 <= 128, i.e. p^2 + t^2 <= 2^15 (so |p|, |t| <= 2^7.5); NaN-propagating
    // maximum: a NaN / inf fails it
    auto mx3 = [](float a, float b, float c) { return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c); };
    const float m = mx3(mx3(qs[0].x, qs[0].y, qs[1].x), mx3(qs[1].y, qs[2].x, qs[2].y), __builtin_elementwise_maximum(qs[3].x, qs[3].y));
    bad |= !(m <= kSsimMfmaQBound);
    // per moment: the horizontal pass of this band, its split, and the vertical pass for output tile b - 1 (h rows of
    // bands b - 1 and b) -- one moment's values live at a time
    f4_t v[4];
#pragma unroll
    for (int mo = 0; mo < 4; ++mo) {
      const f2* x = mo == 0 ? ps : mo == 1 ? ts : mo == 2 ? qs : rs;
      uint32_t ah[4], al[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) split_pair(x[j].x, x[j].y, ah[j], al[j]);
      const f4_t hm = mfma3(as_h8(ah[0], ah[1], ah[2], ah[3]), as_h8(al[0], al[1], al[2], al[3]), BXH, BXL, f4_t{0.f, 0.f, 0.f, 0.f});
      uint32_t hh[2], hl[2];
      split_pair(hm[0], hm[1], hh[0], hl[0]);
      split_pair(hm[2], hm[3], hh[1], hl[1]);
      vh[mo][2 - 2 * par] = hh[0]; vh[mo][3 - 2 * par] = hh[1];
      vl[mo][2 - 2 * par] = hl[0]; vl[mo][3 - 2 * par] = hl[1];
      if (b > 0)
        v[mo] = mfma3(AYH[par], AYL[par], __builtin_bit_cast(h8_t, vh[mo]), __builtin_bit_cast(h8_t, vl[mo]), f4_t{0.f, 0.f, 0.f, 0.f});
    }
    f2 s_sim = {0.f, 0.f}, s_cs = {0.f, 0.f};
    if (b > 0) {
      // U-scaled moments: mu = v, E[.] = v * 2^20 (see above); two output rows per packed op
      const int x = c0 + i16;
      const int ybase = 16 * (b - 1) + 4 * g;  // output row (strip-relative) of r = 0
      const bool all_ok = c0 + 16 <= Wv && 16 * (b - 1) + 16 <= orows;  // wave-uniform: no masking
      const f2 e20 = {1048576.f, 1048576.f}, two = {2.f, 2.f};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 mp = {v[0][2 * h], v[0][2 * h + 1]}, mt = {v[1][2 * h], v[1][2 * h + 1]};
        const f2 e2 = f2{v[2][2 * h], v[2][2 * h + 1]} * e20, ept = f2{v[3][2 * h], v[3][2 * h + 1]} * e20;
        const f2 mu_pt = mp * mt;
        const f2 musum = __builtin_elementwise_fma(mp, mp, mt * mt);
        const f2 upper = __builtin_elementwise_fma(two, ept - mu_pt, c2v);
        const f2 lower = (e2 - musum) + c2v;
        const f2 num1 = __builtin_elementwise_fma(two, mu_pt, c1v);
        const f2 den1 = musum + c1v;
        // hardware reciprocals (1 ulp) instead of IEEE divisions
        const f2 cs = upper * f2{__builtin_amdgcn_rcpf(lower.x), __builtin_amdgcn_rcpf(lower.y)};
        f2 sim = num1 * cs * f2{__builtin_amdgcn_rcpf(den1.x), __builtin_amdgcn_rcpf(den1.y)};
        f2 csm = cs;
        if (!all_ok) {
          const bool ok0 = x < Wv && ybase + 2 * h < orows, ok1 = x < Wv && ybase + 2 * h + 1 < orows;
          sim = f2{ok0 ? sim.x : 0.f, ok1 ? sim.y : 0.f};
          csm = f2{ok0 ? cs.x : 0.f, ok1 ? cs.y : 0.f};
        }
        s_sim += sim;
        s_cs += csm;
      }
    }
    acc_sim += static_cast<double>(s_sim.x + s_sim.y);
    acc_cs += static_cast<double>(s_cs.x + s_cs.y);
    acc_sse += static_cast<double>(f_sse);
  };
  for (int b = 0; b < nb; b += 2) {
    band(b, std::integral_constant<int, 0>{});
    if (b + 1 < nb) band(b + 1, std::integral_constant<int, 1>{});
  }
  acc_sim = wave_sum(acc_sim);
  acc_cs = wave_sum(acc_cs);
  if constexpr (SSE) acc_sse = wave_sum(acc_sse);
  if (__ballot(bad) != 0 && lane == 0) __hip_atomic_store(fallback, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0) {
    const int64_t idx = (plane * gridDim.y + blockIdx.y) * ntx + ct;
    part_sim[idx] = acc_sim;
    part_cs[idx] = acc_cs;
    if constexpr (SSE) part_sse[idx] = acc_sse;
  }
}

}  // namespace tmx
