// Exact-histogram curve kernels (device code only; shared by csrc/classification.hip and the standalone
// ablation harness tools/kexp/curve_hist_exp.hip).  See classification.hip for the op-level documentation.
#pragma once

#include <type_traits>

#include "device_common.h"

namespace tmx {

// Bit-level range test: a 16/32-bit float is in [0, 1] iff its pattern is <= bits(1.0) or equals -0.0.
// NaN / negative / >1 patterns all compare above; no float conversion needed.
template <typename T> struct RangeBits;
template <> struct RangeBits<__hip_bfloat16> { static constexpr uint32_t one = 0x3F80, neg0 = 0x8000; };
template <> struct RangeBits<__half> { static constexpr uint32_t one = 0x3C00, neg0 = 0x8000; };

template <typename T>
__device__ __forceinline__ bool bad16(uint32_t b) { return b > RangeBits<T>::one && b != RangeBits<T>::neg0; }

// 16-bit floats: 8 elements per 16-B load (vectorised, Guideline 13).
// The flag only needs ONE witness: blocks poll it (agent-scope relaxed load, served by L2) and stop early, and a
// block that finds a bad value sets it with a single plain store (idempotent) — no same-address atomics, which
// serialise at the memory side when every block of a logits batch finds a witness at once.
template <typename T>
__global__ void range_flag16_kernel(const uint4* __restrict__ xv, int64_t nvec, const uint16_t* __restrict__ tail,
                                    int ntail, int* __restrict__ flag) {
  __shared__ int s_done;
  if (threadIdx.x == 0) s_done = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_done) return;
  bool bad = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < ntail) bad |= bad16<T>(tail[threadIdx.x]);
  for (; i < nvec; i += 4 * stride) {
    uint4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = (i + u * stride < nvec) ? xv[i + u * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t parts[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) bad |= bad16<T>(parts[k] & 0xFFFFu) | bad16<T>(parts[k] >> 16);
    }
    if (__syncthreads_or(bad)) break;
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0 && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kCodeBits = 14;
constexpr int kCodes = 1 << kCodeBits;  // 16384 >= 16257 (bf16 codes in [0,1]) and 15361 (fp16)

template <typename T> __device__ __forceinline__ int score_code(uint16_t b);
template <> __device__ __forceinline__ int score_code<__hip_bfloat16>(uint16_t b) {
  if (b == 0x8000) return 0;       // -0.0 == 0.0
  return b <= 0x3F80 ? b : -1;     // >1, negative or NaN -> dropped
}
template <> __device__ __forceinline__ int score_code<__half>(uint16_t b) {
  if (b == 0x8000) return 0;
  return b <= 0x3C00 ? b : -1;
}

// ---------------------------------------------------------------------------------------------------------
// Two-pass multiclass histogram (C % 8 == 0, C <= 1024):
//   (A) row pass (mc_codes_kernel) — one 512-thread block per 32-row tile, two blocks per CU (64-KiB LDS image,
//       <= 128 VGPRs).  A wave owns 2 row pairs; all four rows are loaded up front (16-B vector loads), then per
//       row: fp32 softmax (if the mode says so) with expf's exact instruction sequence and a correctly rounded
//       quotient, rounded to the input dtype; arg-max (fused confusion matrix); 16-bit code per element (bit 14 =
//       positive label, bit 15 = skip).  The two rows of a pair are packed per dword (v_perm) into an LDS image
//       [512 NG][16 dwords], pair slot XOR-swizzled by class group (conflict-free writes), then stored as 16-B
//       pieces of 64-B segments of a class-major scratch codes[C][n_pad] (XCD-aware tile order).
//   (B) rare rows — a row with NaN / +-inf (torch: NaN arg-max semantics, all-NaN softmax) is appended to a device
//       list by (A) and finished inside (C), keeping (A)'s fast path free of per-element special cases.
//   (C) class pass (class_hist_kernel) — one 1024-thread workgroup per (class, row split): negatives counted in an
//       LDS-privatised u32 histogram (64 KiB), positives straight to global; one int64 RMW per non-empty bin.
// Measured on MI355X, 65536 x 1000 bf16 logits (tools/kexp/curve_hist_exp.hip, profiles/kexp_rowpass.json): row
// pass 63 us vs 129 us for the previous one-wave-per-row design; class pass 32 us.
// ---------------------------------------------------------------------------------------------------------
// Rows per tile (two row pairs per wave): 32 rows -> 512-thread blocks with a 64-KiB LDS image (2 blocks per CU);
// 16 rows -> 256 threads and 32 KiB (4 per CU) was slower.  Compile-time switch for A/B runs.
#ifndef TMX_ROW_TILE_ROWS
#define TMX_ROW_TILE_ROWS 32  // measured: 16-row tiles 70.7 us vs 64.0 us at 65536 x 1000 bf16 (profiles/row_tile_ab_r3.json)
#endif
constexpr int kTileRows = TMX_ROW_TILE_ROWS;
constexpr int kRowThreads = kTileRows * 16;
constexpr int kRowWaves = kRowThreads / kWave;
constexpr int kSlots = kTileRows / 2;  // pair slots = dwords per class per tile (64-B segment of a class row)

template <typename T> __device__ __forceinline__ void unpack8(const uint4& w, float* v);
// bf16 -> fp32 through the type conversion (not a bit shift): the compiler then knows the values are canonical and
// emits plain v_max / v_max3 instead of a canonicalising v_max x, x per element.
template <> __device__ __forceinline__ void unpack8<__hip_bfloat16>(const uint4& w, float* v) {
  const uint32_t p[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(p[k] & 0xFFFFu)));
    v[2 * k + 1] = static_cast<float>(__builtin_bit_cast(__bf16, static_cast<uint16_t>(p[k] >> 16)));
  }
}
template <> __device__ __forceinline__ void unpack8<__half>(const uint4& w, float* v) {
  const uint32_t p[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(p[k] & 0xFFFFu)));
    v[2 * k + 1] = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(p[k] >> 16)));
  }
}
template <typename T> __device__ __forceinline__ uint16_t raw_bits(const uint4& w, int e) {
  const uint32_t p[4] = {w.x, w.y, w.z, w.w};
  return (e & 1) ? (p[e >> 1] >> 16) : (p[e >> 1] & 0xFFFF);
}

// ---- wave reductions: DPP row ops (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror) leave the 16-lane
// row's result in every lane of the row; row_bcast:15 (rows 1,3) and row_bcast:31 (rows 2,3) fold the rows into
// lane 63, read back as a wave-uniform scalar — 6 DPP ops + 1 readlane instead of 6 ds_bpermute round trips.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f32(float old, float src) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROW_MASK, 0xF, false));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i32(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, CTRL, ROW_MASK, 0xF, false);
}
// max / min through order-preserving integer keys (sign-magnitude -> two's complement): integer max has no NaN
// canonicalisation, so each step folds into one v_max_i32_dpp.  Callers pass NaN-free lane values (fmaxf/fminf
// partials drop NaN); -0.0 orders below +0.0, which only matters to == comparisons, where the two are equal.
__device__ __forceinline__ int f32_key(float f) { const int v = __float_as_int(f); return v ^ ((v >> 31) & 0x7FFFFFFF); }
__device__ __forceinline__ float key_f32(int v) { return __int_as_float(v ^ ((v >> 31) & 0x7FFFFFFF)); }
__device__ __forceinline__ float wave_max_uniform(float f) {
  int v = f32_key(f);
  v = max(v, dpp_i32<0xB1>(v, v));
  v = max(v, dpp_i32<0x4E>(v, v));
  v = max(v, dpp_i32<0x141>(v, v));
  v = max(v, dpp_i32<0x140>(v, v));
  v = max(v, dpp_i32<0x142, 0xA>(v, v));
  v = max(v, dpp_i32<0x143, 0xC>(v, v));
  return key_f32(__builtin_amdgcn_readlane(v, 63));
}
__device__ __forceinline__ float wave_min_uniform(float f) {
  int v = f32_key(f);
  v = min(v, dpp_i32<0xB1>(v, v));
  v = min(v, dpp_i32<0x4E>(v, v));
  v = min(v, dpp_i32<0x141>(v, v));
  v = min(v, dpp_i32<0x140>(v, v));
  v = min(v, dpp_i32<0x142, 0xA>(v, v));
  v = min(v, dpp_i32<0x143, 0xC>(v, v));
  return key_f32(__builtin_amdgcn_readlane(v, 63));
}
__device__ __forceinline__ float wave_sum_uniform(float v) {
  v += dpp_f32<0xB1>(0.f, v);
  v += dpp_f32<0x4E>(0.f, v);
  v += dpp_f32<0x141>(0.f, v);
  v += dpp_f32<0x140>(0.f, v);
  v += dpp_f32<0x142, 0xA>(0.f, v);
  v += dpp_f32<0x143, 0xC>(0.f, v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// exp(x) for x <= 0, -inf or NaN: the instruction sequence the compiler emits for expf (2^(x log2e) with a
// split-precision product, v_exp_f32 on the fractional part, ldexp by the rounded integer part, exact 0 below
// -103.97) minus the x > 88.72 -> inf test.  Contraction is off: (ph - e) must be a rounded subtraction.
__device__ __forceinline__ float exp_nonpos(float x) {
#pragma clang fp contract(off)
  const float log2e_hi = __uint_as_float(0x3fb8aa3bu), log2e_lo = __uint_as_float(0x32a5705fu);
  const float ph = x * log2e_hi;
  float pl = __builtin_fmaf(x, log2e_hi, -ph);
  const float e = __builtin_rintf(ph);
  pl = __builtin_fmaf(x, log2e_lo, pl);
  const float r = __builtin_amdgcn_exp2f((ph - e) + pl);
  const float y = __builtin_amdgcn_ldexpf(r, static_cast<int>(e));
  return x < __uint_as_float(0xc2ce8ed0u) ? 0.f : y;
}
// correctly rounded e / s from the reciprocal: q = e r, residual e - q s (exact in fma), one correction step — the
// quotient torch's softmax stores before rounding to 16 bits.
__device__ __forceinline__ float div_rn(float e, float s, float rinv) {
  const float q = e * rinv;
  return __builtin_fmaf(__builtin_fmaf(-q, s, e), rinv, q);
}

// ---- packed (two-row) forms of the above: the row pass handles the rows of a pair together, element j of row a in
// .x and of row b in .y, so every IEEE mul / add / fma of the chain issues as one v_pk_*_f32 (CDNA3/4 packed fp32:
// two results per lane per instruction).  Each component performs exactly the scalar sequence -> bit-identical.
typedef float f32x2 __attribute__((ext_vector_type(2)));

// exp_nonpos for two values.  The x < -103.97 -> 0 select is replaced by clamping the scaled exponent at -151:
// for every x >= -104.66 nothing changes (ph > -151), and below it, or in the window where the scalar form forces
// 0, ldexp(r, e) with e <= -150 and r < 2^(ph - e) lands below half the smallest denormal and rounds to 0 too (the
// reference expf's result).  -inf gives pl = -inf -> exp2 -> 0; NaN still propagates through pl (v_max drops it
// from ph only), so a NaN row keeps its NaN exp-sum.  One v_max replaces a compare + select per element.
__device__ __forceinline__ f32x2 exp_nonpos2(f32x2 x) {
#pragma clang fp contract(off)
  const float hi_s = __uint_as_float(0x3fb8aa3bu), lo_s = __uint_as_float(0x32a5705fu);
  const f32x2 log2e_hi = {hi_s, hi_s}, log2e_lo = {lo_s, lo_s};
  f32x2 ph = x * log2e_hi;
  ph.x = __builtin_fmaxf(ph.x, -151.f);
  ph.y = __builtin_fmaxf(ph.y, -151.f);
  f32x2 pl = __builtin_elementwise_fma(x, log2e_hi, -ph);
  const f32x2 e = {__builtin_rintf(ph.x), __builtin_rintf(ph.y)};
  pl = __builtin_elementwise_fma(x, log2e_lo, pl);
  const f32x2 t = (ph - e) + pl;
  return f32x2{__builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(t.x), static_cast<int>(e.x)),
               __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(t.y), static_cast<int>(e.y))};
}
__device__ __forceinline__ f32x2 div_rn2(f32x2 e, f32x2 s, f32x2 rinv) {
  const f32x2 q = e * rinv;
  return __builtin_elementwise_fma(__builtin_elementwise_fma(-q, s, e), rinv, q);
}

// fp32 word whose high half is the RNE 16-bit rounding (bf16) — packed pairwise with v_perm afterwards.
template <typename T> __device__ __forceinline__ uint32_t rne_word(float f);
template <> __device__ __forceinline__ uint32_t rne_word<__hip_bfloat16>(float f) {
  const uint32_t u = __float_as_uint(f);
  return u + 0x7FFFu + ((u >> 16) & 1u);
}
template <> __device__ __forceinline__ uint32_t rne_word<__half>(float f) { return (uint32_t)round_bits16<__half>(f) << 16; }

// two RNE 16-bit roundings packed into one dword (a low, b high): gfx950's v_cvt_pk_bf16_f32 for bf16 (one
// instruction for what rne_word + v_perm did in five), the rne_word pair for fp16
template <typename T> __device__ __forceinline__ uint32_t pack_rne2(f32x2 q);
template <> __device__ __forceinline__ uint32_t pack_rne2<__hip_bfloat16>(f32x2 q) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(q, bf16x2));
}
template <> __device__ __forceinline__ uint32_t pack_rne2<__half>(f32x2 q) {
  return __builtin_amdgcn_perm(rne_word<__half>(q.y), rne_word<__half>(q.x), 0x07060302u);
}

// exp_nonpos2 for pairs of rows whose every element is within 86 of its maximum (see row_tile_softmax_lean)
__device__ __forceinline__ f32x2 exp_nonpos2_narrow(f32x2 x) {
#pragma clang fp contract(off)
  const float hi_s = __uint_as_float(0x3fb8aa3bu), lo_s = __uint_as_float(0x32a5705fu), magic = 12582912.f;
  const f32x2 log2e_hi = {hi_s, hi_s}, log2e_lo = {lo_s, lo_s}, m2 = {magic, magic};
  const f32x2 ph = x * log2e_hi;
  f32x2 pl = __builtin_elementwise_fma(x, log2e_hi, -ph);
  const f32x2 s = ph + m2;  // low bits: rint(ph)
  const f32x2 e = s - m2;   // rint(ph), exact
  pl = __builtin_elementwise_fma(x, log2e_lo, pl);
  const f32x2 t = (ph - e) + pl;
  const uint32_t ra = __float_as_uint(__builtin_amdgcn_exp2f(t.x)), rb = __float_as_uint(__builtin_amdgcn_exp2f(t.y));
  return f32x2{__uint_as_float(ra + (__float_as_uint(s.x) << 23)), __uint_as_float(rb + (__float_as_uint(s.y) << 23))};
}

// ---- fast softmax with verified quotients (round 6) -----------------------------------------------------------------
// A softmax code is DEFINED as RNE16(div_rn(exp_nonpos(x - max), s)): the correctly rounded quotient of expf's exact
// instruction sequence (what ATen's softmax stores before its 16-bit rounding) by the row sum s.  Since round 6 s is
// the fixed-order sum of FAST exponentials e_f(x) = v_exp_f32(RN(RN(x - max) L)), L = RN(log2 e) -- one multiply and
// one v_exp per element instead of the 9-instruction exact sequence.  e_f(max) = 1 exactly (as ATen's exp(0)); the
// other terms differ from expf's in the last bits only (the fp32 summation order already differs from ATen's).  The
// class pass's refit reads s from row_stats, so every route produces the same codes for one batch.
// The quotient of the common case (bf16, every element within 86 of its row maximum) is taken FAST and VERIFIED:
// with r = 1 / s (correctly rounded) and d = RN(x - max), the exact quotient lies in [e_f r (1 - eps), e_f r (1 + eps)]:
//   |RN(d L) - d log2e| <= 2^-24 |d| log2e (1 + 0.24)   (RN(d L) and L = log2e (1 + 0.24 2^-24))
//     -> |e_f / exp(d) - 1| <= 1.24 2^-24 |d| + v_exp_f32's 1 ulp (2^-23),
//   |exp_nonpos(d) / exp(d) - 1| <= 1 ulp, |r s - 1| <= 2^-24, and the roundings of r (1 -+ eps) <= 2^-24 each,
// so eps = 2^-24 (1.25 (max - lane min) + 8) bounds it (the ulp terms in units of 2^-24: 2 + 2 + 1 + 1).  RNE16 and fp32 rounding are monotone: when
// RNE16(fl(e_f r_lo)) == RNE16(fl(e_f r_hi)) the exact quotient rounds to that same code.  The element pairs where any
// lane is undecided (~7 % of the pair slots of randn logits at C = 1000, 1e-3 of the elements) are collected in a
// wave-uniform bit mask and recomputed with the exact sequence after the pass, patching the LDS image.  Per element
// pair: sum pass sub, mul, 2 v_exp, add; quotient pass 2 mul, 2 conversions, 1 compare -- against ~17 instructions
// for the exact exp + correctly rounded division.  fp16 keeps the exact quotient (its 10-bit codes put 8x as many
// rounding boundaries in the window).
constexpr float kLog2eF = 1.44269502163f;  // RN(log2 e) = 0x3fb8aa3b
#ifndef TMX_FASTQ_RELOAD
#define TMX_FASTQ_RELOAD 1  // the fallback re-reads the scores (1) or keeps the raw vectors in registers (0)
#endif
#ifndef TMX_FASTQ_RECOMPUTE
#define TMX_FASTQ_RECOMPUTE 0  // 1: P keeps the scores and the quotient pass recomputes the fast exps (no reload)
#endif
#ifndef TMX_FASTQ_LDS
#define TMX_FASTQ_LDS 0  // 1: each wave parks its raw rows in the (not yet written) LDS image; codes wait in registers
#endif
__device__ __forceinline__ f32x2 exp_fast2(f32x2 d) {  // d = x - max (<= 0, -inf or NaN)
  const f32x2 t = d * f32x2{kLog2eF, kLog2eF};
  return f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
}
// relative half-width of the verification interval (see above); lane_min: the smallest element this lane holds
__device__ __forceinline__ float fast_eps(float mx, float lane_min) { return (1.25f * (mx - lane_min) + 8.f) * 5.9604645e-8f; }
template <typename T> struct FastQuot : std::false_type {};
template <> struct FastQuot<__hip_bfloat16> : std::true_type {};
// the code pair of (e.x, e.y) from the fast exps, and whether either could round differently from the definition
template <typename T>
__device__ __forceinline__ uint32_t fast_code2(f32x2 e, f32x2 rlo, f32x2 rhi, bool& undecided) {
  const uint32_t lo = pack_rne2<T>(e * rlo), hi = pack_rne2<T>(e * rhi);
  undecided = lo != hi;
  return lo;
}
// the definition, for the exact paths and the fallback
template <typename T>
__device__ __forceinline__ uint32_t exact_code2(f32x2 x, f32x2 mx2, f32x2 s2, f32x2 i2, bool narrow) {
  const f32x2 d = x - mx2;
  return pack_rne2<T>(div_rn2(narrow ? exp_nonpos2_narrow(d) : exp_nonpos2(d), s2, i2));
}

// the 16-bit pattern of a score widened to fp32 (exact: bf16 / fp16 -> fp32 is lossless; NaN payloads may be
// quietened for fp16, and every NaN pattern is a skip code anyway)
template <typename T> __device__ __forceinline__ uint32_t half_bits(float f);
template <> __device__ __forceinline__ uint32_t half_bits<__hip_bfloat16>(float f) { return __float_as_uint(f) >> 16; }
template <> __device__ __forceinline__ uint32_t half_bits<__half>(float f) { return bits16<__half>(__float2half(f)); }

// 16-bit code of a raw score pattern: -0.0 -> 0, [0, 1] -> itself, anything else (negative, > 1, inf, NaN) -> skip
template <typename T> __device__ __forceinline__ uint32_t raw_code(uint32_t b) {
  return b == 0x8000u ? 0u : (b <= RangeBits<T>::one ? b : 0x8000u);
}

// Per-row statistics of one wave's share of a row (16 elements per lane for C <= 1024, 8 for C <= 512).
template <int NG>
struct RowStat {
  float v[8 * NG];
  float mlo, mhi, mx;  // lane maxima of class groups 0 / 1, wave maximum
  float mn, sum;       // lane minimum and lane sum of the valid elements (probability mode / range witness)
};

template <typename T, int NG>
__device__ __forceinline__ void row_stat(const uint4 (&w)[2], bool lo_ok, bool hi_ok, RowStat<NG>& r) {
  unpack8<T>(w[0], r.v);
  if constexpr (NG == 1) {  // C <= 512: lanes >= C / 8 hold a clamped duplicate, not classes
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = lo_ok ? r.v[j] : -INFINITY;
  }
  r.mlo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(r.v[0], r.v[1]), __builtin_fmaxf(r.v[2], r.v[3])),
                          __builtin_fmaxf(__builtin_fmaxf(r.v[4], r.v[5]), __builtin_fmaxf(r.v[6], r.v[7])));
  r.mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(r.v[0], r.v[1]), __builtin_fminf(r.v[2], r.v[3])),
                         __builtin_fminf(__builtin_fminf(r.v[4], r.v[5]), __builtin_fminf(r.v[6], r.v[7])));
  r.sum = ((r.v[0] + r.v[1]) + (r.v[2] + r.v[3])) + ((r.v[4] + r.v[5]) + (r.v[6] + r.v[7]));
  if constexpr (NG == 1) {
    r.mn = lo_ok ? r.mn : INFINITY;
    r.sum = lo_ok ? r.sum : 0.f;
  }
  r.mhi = -INFINITY;
  if constexpr (NG == 2) {
    float u[8];
    unpack8<T>(w[1], u);
    const float mh = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(u[0], u[1]), __builtin_fmaxf(u[2], u[3])),
                                     __builtin_fmaxf(__builtin_fmaxf(u[4], u[5]), __builtin_fmaxf(u[6], u[7])));
    const float nh = __builtin_fminf(__builtin_fminf(__builtin_fminf(u[0], u[1]), __builtin_fminf(u[2], u[3])),
                                     __builtin_fminf(__builtin_fminf(u[4], u[5]), __builtin_fminf(u[6], u[7])));
    const float sh = ((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7]));
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[8 + j] = hi_ok ? u[j] : -INFINITY;  // padding classes never win / add 0 to exp-sums
    r.mhi = hi_ok ? mh : -INFINITY;
    r.mn = hi_ok ? __builtin_fminf(r.mn, nh) : r.mn;
    r.sum = hi_ok ? r.sum + sh : r.sum;
  }
  r.mx = wave_max_uniform(__builtin_fmaxf(r.mlo, r.mhi));
}

// Row statistics for rows padded to a multiple of 8 classes (host-side pad when C % 8 != 0): element k of group g in
// lane L is class 512 g + 8 L + k, valid iff below C — nlo / nhi = valid elements of this lane in groups 0 / 1.
template <typename T, int NG>
__device__ __forceinline__ void row_stat_padded(const uint4 (&w)[2], int nlo, int nhi, RowStat<NG>& r) {
  float u[8 * NG];
  unpack8<T>(w[0], u);
  if constexpr (NG == 2) unpack8<T>(w[1], u + 8);
  float mlo = -INFINITY, mhi = -INFINITY, mn = INFINITY, sum = 0.f;
#pragma unroll
  for (int j = 0; j < 8 * NG; ++j) {
    const bool ok = j < 8 ? j < nlo : j - 8 < nhi;
    r.v[j] = ok ? u[j] : -INFINITY;
    mn = ok ? __builtin_fminf(mn, u[j]) : mn;
    sum += ok ? u[j] : 0.f;
    if (j < 8) mlo = __builtin_fmaxf(mlo, r.v[j]);
    else mhi = __builtin_fmaxf(mhi, r.v[j]);
  }
  r.mlo = mlo;
  r.mhi = mhi;
  r.mn = mn;
  r.sum = sum;
  r.mx = wave_max_uniform(__builtin_fmaxf(r.mlo, r.mhi));
}

// arg-max of a row without NaN / inf: first class (ascending) holding the wave maximum.  Classes of group g, lane L,
// slot k are 512 g + 8 L + k, so the winner is the lowest lane whose group-0 maximum equals mx (else the lowest lane
// of group 1) and the lowest slot of that lane.
// The slot is found with one ballot per slot of the winning (wave-uniform) group and a scalar bit test of lane L —
// one v_cmp per slot instead of a compare + select per element of both groups.
template <int NG>
__device__ __forceinline__ int row_argmax(const RowStat<NG>& r) {
  const uint64_t blo = __ballot(r.mlo == r.mx);
  const int g = blo != 0 ? 0 : 1;
  const uint64_t b = blo != 0 ? blo : __ballot(r.mhi == r.mx);
  const int L = __builtin_ctzll(b | (1ull << 63));
  int k = 7;
  if (NG == 1 || g == 0) {
#pragma unroll
    for (int j = 6; j >= 0; --j)
      if ((__ballot(r.v[j] == r.mx) >> L) & 1ull) k = j;
  } else {
#pragma unroll
    for (int j = 6; j >= 0; --j)
      if ((__ballot(r.v[8 * (NG - 1) + j] == r.mx) >> L) & 1ull) k = j;
  }
  return 512 * g + 8 * L + k;
}

struct SlowRows {
  int* rows;   // [2][n]: list 0 = rows of the speculated-mode pass, list 1 = rows of a FIXUP pass
  int* count;  // [2]
};

// Store one tile's LDS image as 16-B pieces of the class rows of the class-major scratch (compile-time trip count):
// thread -> (class c, 16-B group g of the class's 64-B segment).  Segment dword 4g + i lives at LDS slot
// (4g + i) ^ s (s = class swizzle), i.e. in LDS quad g ^ (s >> 2) at position i ^ (s & 3).
// Code stores of the row pass.  TMX_ROWPASS_NT_STORE=1 builds them as non-temporal (streaming) stores, so the
// class-major codes need not sit dirty in the XCD L2s until the kernel-boundary write-back.
#ifndef TMX_ROWPASS_NT_STORE
#define TMX_ROWPASS_NT_STORE 0
#endif
template <int NG>
__device__ __forceinline__ void store_tile(const uint32_t* __restrict__ s_tile, uint32_t* __restrict__ codes, int C,
                                           int64_t n_pad, int64_t tile) {
  constexpr int kQuads = kSlots / 4;  // 4 x 16 B per class per tile
  const int64_t seg = tile * kSlots;
  const int64_t row_dw = n_pad / 2;
#pragma unroll
  for (int k = 0; k < 512 * NG * kQuads / kRowThreads; ++k) {
    const int idx = threadIdx.x + k * kRowThreads;
    const int c = idx / kQuads, g = idx % kQuads;
    const int sw = (c >> 3) & (kSlots - 1);
    const uint4 w = *reinterpret_cast<const uint4*>(&s_tile[c * kSlots + 4 * (g ^ (sw >> 2))]);
    const int x = sw & 3;
    const uint32_t e0 = x & 1 ? w.y : w.x, e1 = x & 1 ? w.x : w.y, e2 = x & 1 ? w.w : w.z, e3 = x & 1 ? w.z : w.w;
    const uint4 o = x & 2 ? make_uint4(e2, e3, e0, e1) : make_uint4(e0, e1, e2, e3);
    if (c < C) {
#if TMX_ROWPASS_NT_STORE
      using v4u = __attribute__((ext_vector_type(4))) unsigned int;
      v4u v = {o.x, o.y, o.z, o.w};
      __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(&codes[c * row_dw + seg + 4 * g]));
#else
      *reinterpret_cast<uint4*>(&codes[c * row_dw + seg + 4 * g]) = o;
#endif
    }
  }
}

// One 32-row tile of the row pass for a fixed normalisation (SOFTMAX).  Every load is issued up front; stores and
// global atomics come only after the last wait (a VMEM write pending behind a load makes the compiler drain the
// whole queue at the next wait).

// Logit loads of the row pass.  TMX_ROWPASS_NT=1 builds them as non-temporal loads (the logits are read once), so
// they need not displace the class-major codes the class pass reads next from the Infinity Cache.
#ifndef TMX_ROWPASS_NT
#define TMX_ROWPASS_NT 1  // measured: 0.118 vs 0.122 ms per update at 65536 x 1000 bf16 (profiles/rowpass_nt_loads.json)
#endif
__device__ __forceinline__ uint4 stream_load16(const uint4* p) {
#if TMX_ROWPASS_NT
  using v4u = __attribute__((ext_vector_type(4))) unsigned int;
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}

// One tile's loads, issued as one batch (the persistent row pass issues the NEXT tile's batch before computing the
// current one): a wave's two row pairs as 16-B vectors per lane and the int64 targets of its four rows (lanes 0-3).
template <int NG>
struct RowLoads {
  uint4 raw[2][2][2];
  int64_t tv;
};

// UNALIGNED (C % 8 != 0, rows at stride C: round 5, no padding copy): a row starts 2 ((r C) % 8) bytes past a 16-B
// boundary; its full 16-B vectors are loaded at the row's own addresses (gfx950 global loads take any 2-byte
// alignment: tools/kexp/unaligned_load_exp.hip, 0 wrong elements; tools/kexp/unaligned_bw_exp.hip, 4.8 vs 5.5 TB/s
// streaming).  The row's last, partial vector is loaded as the 16 B that END at the row's end -- always inside the
// tensor, the last row included -- and rotated by R = 8 - rem slots into place: slots [0, rem) hold the row's last
// rem scores, slots [rem, 8) the R scores before them (real scores of the row, so maxima, minima and the arg-max --
// lowest lane wins -- are unchanged; the exp-sum skips them).  Lanes past the row's vectors load vector 0.
__device__ __forceinline__ uint4 rotate_slots(uint4 w, int R) {  // slot k <- slot (k + R) mod 8, R wave-uniform
  uint32_t d[4] = {w.x, w.y, w.z, w.w};
  if (R & 4) {  // 2 dwords
    const uint32_t t0 = d[0], t1 = d[1];
    d[0] = d[2]; d[1] = d[3]; d[2] = t0; d[3] = t1;
  }
  if (R & 2) {  // 1 dword
    const uint32_t t0 = d[0];
    d[0] = d[1]; d[1] = d[2]; d[2] = d[3]; d[3] = t0;
  }
  if (R & 1) {  // 2 bytes: dword k = high half of d[k], low half of d[k + 1]
    const uint32_t t0 = d[0];
    d[0] = __builtin_amdgcn_alignbyte(d[1], d[0], 2);
    d[1] = __builtin_amdgcn_alignbyte(d[2], d[1], 2);
    d[2] = __builtin_amdgcn_alignbyte(d[3], d[2], 2);
    d[3] = __builtin_amdgcn_alignbyte(t0, d[3], 2);
  }
  return make_uint4(d[0], d[1], d[2], d[3]);
}
// the row's vectors as loaded by row_tile_load<UNALIGNED>, with the partial vector (last group) rotated into place
template <int NG>
__device__ __forceinline__ void realign_partial(uint4 (&w)[2], int ld) {
  const int lane = threadIdx.x & (kWave - 1);
  const int nvec = (ld + 7) / 8;
  if (lane + kWave * (NG - 1) == nvec - 1) w[NG - 1] = rotate_slots(w[NG - 1], 8 * nvec - ld);
}

template <typename T, int NG, bool UNALIGNED = false>
__device__ __forceinline__ void row_tile_load(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n, int ld,
                                              int64_t tile, RowLoads<NG>& L) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nvec = UNALIGNED ? (ld + 7) / 8 : ld / 8;
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  const int lq = lo_ok ? lane : (UNALIGNED ? 0 : nvec - 1);  // clamped: every load stays inside its row
  const int hq = hi_ok ? lane + kWave : (UNALIGNED ? 0 : nvec - 1);
  auto row0_of = [&](int pp) -> int64_t { return tile * kTileRows + 2 * (wave + pp * kRowWaves); };
  L.tv = target[min(row0_of((lane & 3) >> 1) + (lane & 1), n - 1)];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (UNALIGNED) {
#ifdef TMX_UNALIGNED_TIMING_HACK  // timing experiment only (wrong data): the same loads at 16-B aligned addresses
        const uint16_t* row = reinterpret_cast<const uint16_t*>(preds) + (min(row0_of(pp) + h, n - 1) * ld & ~int64_t{7});
#else
        const uint16_t* row = reinterpret_cast<const uint16_t*>(preds) + min(row0_of(pp) + h, n - 1) * ld;
#endif
        const int R = 8 * nvec - ld;  // 1..7
        // the partial vector lives in the last group: NG == 2 -> the hi group (nvec > 64), NG == 1 -> the lo group
        // (the rotation waits until the vector is consumed -- realign_partial -- so every load is in flight first:
        // rotating here stalled the next rows' loads on this one, +7 us per 65,536 x 1001 row pass)
        if constexpr (NG == 2) {
          L.raw[pp][h][0] = stream_load16(reinterpret_cast<const uint4*>(row + 8 * lq));
          L.raw[pp][h][1] = stream_load16(reinterpret_cast<const uint4*>(row + (hq == nvec - 1 ? ld - 8 : 8 * hq)));
        } else {
          L.raw[pp][h][0] = stream_load16(reinterpret_cast<const uint4*>(row + (lq == nvec - 1 ? ld - 8 : 8 * lq)));
        }
        (void)R;
      } else {
        const uint4* row = reinterpret_cast<const uint4*>(preds + min(row0_of(pp) + h, n - 1) * ld);
        L.raw[pp][h][0] = stream_load16(row + lq);
        if constexpr (NG == 2) L.raw[pp][h][1] = stream_load16(row + hq);
      }
    }
}

// Positive booking by the row pass (round 5).  The row pass knows each row's positive (its target); instead of
// flagging it with bit 14 for the class pass to find (a test of every code there: ~40 % of the class pass's 16-B vectors
// carry one at C = 1000), lane i < 4 of each wave marks its row's positive skipped in the LDS image (a returning
// ds_or) and books the code into the int64 positive bins of the target class and its code range (no-return atomics;
// the tile's barrier waits for LDS only, so nothing waits for them).  Values kept alive across the barrier, or range
// words prefetched at the tile's start, cost ~5 us at this kernel's 128-VGPR edge (profiles/kexp_headline_r5.json).
// The booked code goes to row_stats[r].w (code | 0x10000; 0 = none) so the class pass can take it back when it refits
// a mis-speculated batch.  hist == nullptr: the bit-14 flag as before (test op, FIXUP route, u16 pass).
struct PosSink {
  int64_t* hist;    // [C][2][kCodes]: the positive half of class t is hist + (2 t + 1) kCodes
  int64_t* bhist;   // forward()'s batch histogram or nullptr
  int* range;       // [C][2] occupied code range of hist (nullptr: not tracked)
  int* brange;      // [C][2] of bhist
};

struct PosTake {  // lane i < 4: row i of the wave's four rows
  int64_t r, t;
  uint32_t code;  // code | 0x10000 when booked
  int lo, hi, blo, bhi;
};

// before the tile's barrier (the wave's own image writes are done): mark the positive skipped, keep its code
__device__ __forceinline__ void pos_take(PosTake& pt, uint32_t* __restrict__ s_tile, const bool (&keepv)[4], const int64_t (&tt)[4], int C,
                                         int wave, int64_t row00, int64_t n) {
  const int lane = threadIdx.x & (kWave - 1);
  if (lane >= 4) return;
  const bool k = lane == 0 ? keepv[0] : lane == 1 ? keepv[1] : lane == 2 ? keepv[2] : keepv[3];
  const int64_t t = lane == 0 ? tt[0] : lane == 1 ? tt[1] : lane == 2 ? tt[2] : tt[3];
  const int p = wave + (lane >> 1) * kRowWaves;
  const int half = lane & 1;
  const int64_t r = row00 + 2 * (int64_t)(lane >> 1) * kRowWaves + half;
  if (r >= n || !k || t < 0 || t >= C) return;
  const int idx = (int)t * kSlots + (p ^ ((int)(t >> 3) & (kSlots - 1)));
  const uint32_t code = (atomicOr(&s_tile[idx], 0x8000u << (16 * half)) >> (16 * half)) & 0xFFFFu;
  pt.r = r;
  if (!(code & 0x8000u)) pt.code = code | 0x10000u;  // an out-of-range score (probability mode) counts nowhere
}

// after the tile's barrier and store: the global side of the booking
#ifndef TMX_POS_ABL
#define TMX_POS_ABL 0  // kernel-harness ablation (tools/kexp): 1 no global booking, 2 no range words, 4 no row_stats word,
                       // 8 no bin atomic.  0 in the library.
#endif
__device__ __forceinline__ void pos_book(const PosTake& pt, const PosSink& pos, float4* __restrict__ row_stats) {
  if (pos.hist == nullptr || (threadIdx.x & (kWave - 1)) >= 4 || !(pt.code & 0x10000u)) return;
  if (TMX_POS_ABL & 1) return;
  const int64_t t = pt.t;
  const int code = static_cast<int>(pt.code & 0xFFFFu);
  if (!(TMX_POS_ABL & 8)) atomic_add_i64(pos.hist + (2 * t + 1) * kCodes + code, 1);
  if (pos.bhist != nullptr) atomic_add_i64(pos.bhist + (2 * t + 1) * kCodes + code, 1);
  if (pos.range != nullptr && !(TMX_POS_ABL & 2)) {
    if (code < pt.lo) atomicMin(pos.range + 2 * t, code);
    if (code > pt.hi) atomicMax(pos.range + 2 * t + 1, code);
  }
  if (pos.brange != nullptr) {
    if (code < pt.blo) atomicMin(pos.brange + 2 * t, code);
    if (code > pt.bhi) atomicMax(pos.brange + 2 * t + 1, code);
  }
  if (row_stats != nullptr && !(TMX_POS_ABL & 4)) reinterpret_cast<uint32_t*>(row_stats + pt.r)[3] = pt.code;
}

// Compute half of a tile: codes into the LDS image, confusion matrix / error / rare-row side effects.  The caller
// stores the image (after a barrier).
template <typename T, int NG, bool SOFTMAX, bool FIXUP, bool PADDED>
__device__ __forceinline__ void row_tile_compute(const RowLoads<NG>& L, int64_t n, int C, int ld, int64_t ignore_index, bool has_ignore,
                                                 int64_t* __restrict__ confmat, int* __restrict__ err, bool rec, bool& saw_bad,
                                                 SlowRows slow, uint32_t* __restrict__ s_tile, int64_t tile,
                                                 float4* __restrict__ row_stats, const PosSink& pos, PosTake& ptake) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nvec = PADDED ? (ld + 7) / 8 : ld / 8;
  const int nlo = min(max(C - 8 * lane, 0), 8), nhi = min(max(C - 8 * (lane + kWave), 0), 8);
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  auto row0_of = [&](int pp) -> int64_t { return tile * kTileRows + 2 * (wave + pp * kRowWaves); };
  const int64_t tv = L.tv;
  const auto& raw = L.raw;
  auto target_of = [&](int i) -> int64_t {
    const uint64_t u = static_cast<uint64_t>(tv);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), i);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), i);
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  int64_t tt[4];
  int am[4];
  bool keepv[4], slowv[4], validv[4];
  ptake = PosTake{-1, tv, 0u, kCodes, -1, kCodes, -1};
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int p = wave + pp * kRowWaves;
    const int64_t r0 = row0_of(pp);
    const int64_t ta = target_of(2 * pp), tb = target_of(2 * pp + 1);
    const bool va = r0 < n && !(has_ignore && ta == ignore_index);
    const bool vb = r0 + 1 < n && !(has_ignore && tb == ignore_index);
    RowStat<NG> ra, rb;
    // the row pair's vectors (PADDED = UNALIGNED rows: the partial vector rotated into place)
    uint4 wa[2] = {raw[pp][0][0], raw[pp][0][1]}, wb[2] = {raw[pp][1][0], raw[pp][1][1]};
    if constexpr (PADDED) {
      realign_partial<NG>(wa, ld);
      realign_partial<NG>(wb, ld);
      row_stat_padded<T, NG>(wa, nlo, nhi, ra);
      row_stat_padded<T, NG>(wb, nlo, nhi, rb);
    } else {
      row_stat<T, NG>(wa, lo_ok, hi_ok, ra);
      row_stat<T, NG>(wb, lo_ok, hi_ok, rb);
    }
    bool fa = __builtin_isfinite(ra.mx), fb = __builtin_isfinite(rb.mx);
    const int ama = row_argmax<NG>(ra), amb = row_argmax<NG>(rb);
    float sa = 0.f, sb = 0.f, ia = 0.f, ib = 0.f;
    if constexpr (SOFTMAX) {
      f32x2 acc = {0.f, 0.f};
      const f32x2 mx2 = {ra.mx, rb.mx};
      // the row sums of the fast exps, in the lean form's order (padding slots hold -inf: exp2(-inf) adds +0); then
      // the exact exps (the definition's numerators) replace the scores
#pragma unroll
      for (int j = 0; j < 8 * NG; ++j) {
        const f32x2 d = f32x2{ra.v[j], rb.v[j]} - mx2;
        acc = acc + exp_fast2(d);
        const f32x2 e = exp_nonpos2(d);
        ra.v[j] = e.x;
        rb.v[j] = e.y;
      }
      sa = wave_sum_uniform(acc.x);
      sb = wave_sum_uniform(acc.y);
      ia = 1.f / sa;
      ib = 1.f / sb;
      fa = fa && sa == sa;
      fb = fb && sb == sb;
    } else {
      fa = fa && __builtin_isfinite(wave_sum_uniform(ra.sum));
      fb = fb && __builtin_isfinite(wave_sum_uniform(rb.sum));
      if (row_stats != nullptr) {  // the softmax statistics too, so the class pass can refit a mispredicted batch
        f32x2 acc = {0.f, 0.f};
        const f32x2 mx2 = {ra.mx, rb.mx};
#pragma unroll
        for (int j = 0; j < 8 * NG; ++j) acc = acc + exp_fast2(f32x2{ra.v[j], rb.v[j]} - mx2);
        sa = wave_sum_uniform(acc.x);
        sb = wave_sum_uniform(acc.y);
      }
    }
    if (row_stats != nullptr && lane == 0) {
      // per row: {max, exp-sum, flags (bit 0 = counted row, bit 1 = finite softmax)} for the class pass's refit
      // of a batch whose speculated normalisation mode was wrong (class_hist_block)
      const bool sfa = __builtin_isfinite(ra.mx) && sa == sa, sfb = __builtin_isfinite(rb.mx) && sb == sb;
      if (r0 < n) row_stats[r0] = make_float4(ra.mx, sa, __uint_as_float((va ? 1u : 0u) | (sfa ? 2u : 0u)), 0.f);
      if (r0 + 1 < n) row_stats[r0 + 1] = make_float4(rb.mx, sb, __uint_as_float((vb ? 1u : 0u) | (sfb ? 2u : 0u)), 0.f);
    }
    const bool slow_a = va && !fa, slow_b = vb && !fb;
    if (rec && !saw_bad) {
      saw_bad = slow_a || slow_b || (va && ra.mx > 1.f) || (vb && rb.mx > 1.f);
      if (!saw_bad && (va || vb))
        saw_bad = wave_min_uniform(__builtin_fminf(va ? ra.mn : INFINITY, vb ? rb.mn : INFINITY)) < 0.f;
    }
    const bool ka = va && fa, kb = vb && fb;
    const uint32_t keep = (ka ? 0x0000FFFFu : 0u) | (kb ? 0xFFFF0000u : 0u);
    const uint32_t setm = ~keep & 0x80008000u;
#pragma unroll
    for (int j = 0; j < 8 * NG; ++j) {
      uint32_t packed;
      if constexpr (SOFTMAX) {
        packed = pack_rne2<T>(div_rn2(f32x2{ra.v[j], rb.v[j]}, f32x2{sa, sb}, f32x2{ia, ib}));
      } else {
        const uint32_t ca = raw_code<T>(raw_bits<T>(wa[j >> 3], j & 7));
        const uint32_t cb = raw_code<T>(raw_bits<T>(wb[j >> 3], j & 7));
        packed = ca | (cb << 16);
      }
      const int c = 512 * (j >> 3) + 8 * lane + (j & 7);
      s_tile[c * kSlots + (p ^ (lane & (kSlots - 1)))] = (packed & keep) | setm;
    }
    if (lane == 0 && pos.hist == nullptr) {
      if (ka && ta >= 0 && ta < C) atomicOr(&s_tile[ta * kSlots + (p ^ ((int)(ta >> 3) & (kSlots - 1)))], 0x00004000u);
      if (kb && tb >= 0 && tb < C) atomicOr(&s_tile[tb * kSlots + (p ^ ((int)(tb >> 3) & (kSlots - 1)))], 0x40000000u);
    }
    tt[2 * pp] = ta; tt[2 * pp + 1] = tb;
    am[2 * pp] = ama; am[2 * pp + 1] = amb;
    keepv[2 * pp] = ka; keepv[2 * pp + 1] = kb;
    slowv[2 * pp] = slow_a; slowv[2 * pp + 1] = slow_b;
    validv[2 * pp] = va; validv[2 * pp + 1] = vb;
  }
  if (pos.hist != nullptr) {
    pos_take(ptake, s_tile, keepv, tt, C, wave, row0_of(0), n);
    pos_book(ptake, pos, row_stats);
  }
  // global side effects after every load has been consumed
  if (lane == 0) {
    const int list = FIXUP ? 1 : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t t = tt[i];
      if constexpr (!FIXUP) {
        if (confmat != nullptr && keepv[i] && t >= 0 && t < C && am[i] < C) atomic_add_i64(confmat + t * C + am[i], 1);
        if (err != nullptr && validv[i] && (t < 0 || t >= C)) atomicOr(err, 1);
      }
      if (slowv[i]) slow.rows[list * n + atomicAdd(slow.count + list, 1)] = static_cast<int>(row0_of(i >> 1) + (i & 1));
    }
  }
}

// ---- softmax row tile, lean form (round 5) ----------------------------------------------------------------------------
// The same codes, bit for bit, as row_tile_compute<SOFTMAX> with about 40 % fewer VALU instructions per element
// (profiles/pmc_headline_r4.json: the row pass issued ~22 VALU instructions per logit and was VALU-bound):
//  * the two rows of a pair are unpacked straight into (row a, row b) register pairs, so every v_pk_* operand is
//    already adjacent (no v_mov to build pairs);
//  * padding lanes hold duplicates of the row's last vector (the clamped loads), which change neither a maximum, a
//    minimum, nor the arg-max (the lowest lane wins ties); only the exp-sum must skip them: the lane sum is taken
//    before the padding group is added (one select per row instead of one per element);
//  * exp: when every element of the pair is within 86 of its row maximum (ballot, wave-uniform) the clamp is a no-op,
//    rint(ph) is (ph + 1.5 2^23) - 1.5 2^23 (RNE for |ph| < 2^22) and ldexp(r, e) = bits(r) + (e << 23) exactly (r in
//    [0.7, 1.42], 126 + e >= 2: normal), where e << 23 is the low bits of (ph + 1.5 2^23) shifted by 23 -- one
//    v_lshl_add_u32 for v_rndne + v_cvt_i32 + v_ldexp.  Otherwise (a gap > 86, -inf, or a row that is not finite) the
//    pair takes exp_nonpos2, the reference sequence;
//  * the row minimum is only compared (ballots), never wave-reduced; the probability-mode witnesses are tested only
//    while the block has not seen one (``rec && !saw_bad``), as before.

template <typename T, int NG>
__device__ __forceinline__ void unpack_pair(const uint4& wa, const uint4& wb, f32x2* P) {
  float a[8], b[8];
  unpack8<T>(wa, a);
  unpack8<T>(wb, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) P[j] = f32x2{a[j], b[j]};
}

// IEEE 754-2019 maximum (v_maximum3_f32): a NaN row's maximum is NaN -- not finite, so the row takes the rare-row path
// exactly as with fmaxf's NaN-dropping maximum (whose NaN exp-sum marked it)
__device__ __forceinline__ float max8(const float* v) {
  auto m = [](float a, float b) { return __builtin_elementwise_maximum(a, b); };
  return m(m(m(v[0], v[1]), m(v[2], v[3])), m(m(v[4], v[5]), m(v[6], v[7])));
}
// IEEE 754-2019 minimum (NaN-propagating; gfx950 v_minimum3_f32): fminf's sNaN quieting made the compiler canonicalise
// every element first (v_max x, x).  A NaN minimum fails the narrow test below, which is the safe direction.
__device__ __forceinline__ float min8(const float* v) {
  auto m = [](float a, float b) { return __builtin_elementwise_minimum(a, b); };
  return m(m(m(v[0], v[1]), m(v[2], v[3])), m(m(v[4], v[5]), m(v[6], v[7])));
}

template <typename T, int NG, bool UNALIGNED = false>
__device__ __forceinline__ void row_tile_softmax_lean(const T* __restrict__ preds, const RowLoads<NG>& L, int64_t n, int C, int ld, int64_t ignore_index,
                                                      bool has_ignore, int64_t* __restrict__ confmat, int* __restrict__ err, bool rec,
                                                      bool& saw_bad, SlowRows slow, uint32_t* __restrict__ s_tile, int64_t tile,
                                                      float4* __restrict__ row_stats, const PosSink& pos, PosTake& ptake) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nvec = UNALIGNED ? (ld + 7) / 8 : ld / 8;
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  // UNALIGNED: the lane holding the row's partial last vector counts only its first ``rem`` slots in the exp-sum
  const int rem = ld - 8 * (nvec - 1);
  const int cut_lo = UNALIGNED && lane == nvec - 1 ? rem : 8, cut_hi = UNALIGNED && lane + kWave == nvec - 1 ? rem : 8;
  auto row0_of = [&](int pp) -> int64_t { return tile * kTileRows + 2 * (wave + pp * kRowWaves); };
  const int64_t tv = L.tv;
  auto target_of = [&](int i) -> int64_t {
    const uint64_t u = static_cast<uint64_t>(tv);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), i);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), i);
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  int64_t tt[4];
  int am[4];
  bool keepv[4], slowv[4], validv[4];
  ptake = PosTake{-1, tv, 0u, kCodes, -1, kCodes, -1};
#if TMX_FASTQ_LDS
  // the fallback's scores: every wave parks its four rows in the LDS image region ([row in tile][group][lane] 16-B
  // vectors, exactly the image's size), which nobody writes until the barrier after the pair loop -- the codes wait
  // in registers (cv) meanwhile, so an undecided slot re-reads its scores from LDS instead of global memory
  static_assert(kTileRows * kWave * 16 == 512 * kSlots * 4, "raw rows must fit the code image");
  uint32_t cv[2][8 * NG];
  uint4* const raw_lds = reinterpret_cast<uint4*>(s_tile);
#endif
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int p = wave + pp * kRowWaves;
    const int64_t r0 = row0_of(pp);
    const int64_t ta = target_of(2 * pp), tb = target_of(2 * pp + 1);
    const bool va = r0 < n && !(has_ignore && ta == ignore_index);
    const bool vb = r0 + 1 < n && !(has_ignore && tb == ignore_index);
    f32x2 P[8 * NG];
    float mlo_a, mlo_b, mhi_a = -INFINITY, mhi_b = -INFINITY, mn_a, mn_b;
    uint4 wa[2] = {L.raw[pp][0][0], L.raw[pp][0][1]}, wb[2] = {L.raw[pp][1][0], L.raw[pp][1][1]};
    if constexpr (UNALIGNED) {
      realign_partial<NG>(wa, ld);
      realign_partial<NG>(wb, ld);
    }
#if TMX_FASTQ_LDS
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      raw_lds[((2 * p) * NG + g) * kWave + lane] = wa[g];
      raw_lds[((2 * p + 1) * NG + g) * kWave + lane] = wb[g];
    }
#endif
    {
      float a[8], b[8];
      unpack8<T>(wa[0], a);
      unpack8<T>(wb[0], b);
      mlo_a = max8(a);
      mlo_b = max8(b);
      mn_a = min8(a);
      mn_b = min8(b);
#pragma unroll
      for (int j = 0; j < 8; ++j) P[j] = f32x2{a[j], b[j]};
    }
    if constexpr (NG == 2) {
      float a[8], b[8];
      unpack8<T>(wa[1], a);
      unpack8<T>(wb[1], b);
      mhi_a = max8(a);
      mhi_b = max8(b);
      mn_a = __builtin_fminf(mn_a, min8(a));
      mn_b = __builtin_fminf(mn_b, min8(b));
#pragma unroll
      for (int j = 0; j < 8; ++j) P[8 + j] = f32x2{a[j], b[j]};
    }
    const float mxa = wave_max_uniform(__builtin_fmaxf(mlo_a, mhi_a));
    const float mxb = wave_max_uniform(__builtin_fmaxf(mlo_b, mhi_b));
    // arg-max (row_argmax on the pair layout): lowest lane of the lowest group holding the maximum, lowest slot
    auto argmax = [&](float mlo, float mhi, float mx, bool second) -> int {
      const uint64_t blo = __ballot(mlo == mx);
      const int g = blo != 0 ? 0 : 1;
      const uint64_t bm = blo != 0 ? blo : __ballot(mhi == mx);
      const int Ln = __builtin_ctzll(bm | (1ull << 63));
      int k = 7;
      if (NG == 1 || g == 0) {
#pragma unroll
        for (int j = 6; j >= 0; --j)
          if ((__ballot((second ? P[j].y : P[j].x) == mx) >> Ln) & 1ull) k = j;
      } else {
#pragma unroll
        for (int j = 6; j >= 0; --j)
          if ((__ballot((second ? P[8 * (NG - 1) + j].y : P[8 * (NG - 1) + j].x) == mx) >> Ln) & 1ull) k = j;
      }
      return 512 * g + 8 * Ln + k;
    };
    const int ama = argmax(mlo_a, mhi_a, mxa, false), amb = argmax(mlo_b, mhi_b, mxb, true);
    bool fa = __builtin_isfinite(mxa), fb = __builtin_isfinite(mxb);
    // exp(x - max): the lean sequence when every element of both rows is within 86 of its maximum (wave-uniform)
    const bool narrow = __ballot(!(mxa - mn_a <= 86.f && mxb - mn_b <= 86.f)) == 0;
    const f32x2 mx2 = {mxa, mxb};
    f32x2 acc = {0.f, 0.f}, acc_lo = {0.f, 0.f};
    // the partial vector sits in the last class group (nvec - 1 >= 64 when NG == 2): scale its slots by 0 / 1
    auto counted = [&](f32x2 e, int j) -> f32x2 {
      if constexpr (UNALIGNED
#ifdef TMX_UNALIGNED_NOMASK_HACK  // timing experiment only
                    && false
#endif
      ) {
        if (j >= 8 * (NG - 1)) {
          const float m = (j & 7) < (NG == 2 ? cut_hi : cut_lo) ? 1.f : 0.f;
          return e * f32x2{m, m};
        }
      }
      return e;
    };
    // the row sums of the fast exps; on the fast path (bf16, narrow rows) the exps replace the scores in P, otherwise
    // P keeps the scores for the exact quotients
    const bool fast = FastQuot<T>::value && narrow;
    if (fast && !TMX_FASTQ_RECOMPUTE) {
#pragma unroll
      for (int j = 0; j < 8 * NG; ++j) {
        P[j] = exp_fast2(P[j] - mx2);
        acc = acc + counted(P[j], j);
        if (j == 7) acc_lo = acc;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8 * NG; ++j) {
        acc = acc + counted(exp_fast2(P[j] - mx2), j);
        if (j == 7) acc_lo = acc;
      }
    }
    // padding lanes: the group-1 duplicates (NG == 2) or the whole lane (NG == 1) add nothing to the exp-sum
    if constexpr (NG == 2) acc = hi_ok ? acc : acc_lo;
    else acc = lo_ok ? acc : f32x2{0.f, 0.f};
    const float sa = wave_sum_uniform(acc.x), sb = wave_sum_uniform(acc.y);
    const float ia = 1.f / sa, ib = 1.f / sb;
    fa = fa && sa == sa;
    fb = fb && sb == sb;
    if (row_stats != nullptr && lane == 0) {
      const bool sfa = __builtin_isfinite(mxa) && sa == sa, sfb = __builtin_isfinite(mxb) && sb == sb;
      if (r0 < n) row_stats[r0] = make_float4(mxa, sa, __uint_as_float((va ? 1u : 0u) | (sfa ? 2u : 0u)), 0.f);
      if (r0 + 1 < n) row_stats[r0 + 1] = make_float4(mxb, sb, __uint_as_float((vb ? 1u : 0u) | (sfb ? 2u : 0u)), 0.f);
    }
    const bool slow_a = va && !fa, slow_b = vb && !fb;
    if (rec && !saw_bad) {
      saw_bad = slow_a || slow_b || (va && mxa > 1.f) || (vb && mxb > 1.f);
      if (!saw_bad && (va || vb)) {
        // lanes past the row's vectors hold duplicates: a duplicate's minimum is a real element's
        saw_bad = __ballot((va && mn_a < 0.f) || (vb && mn_b < 0.f)) != 0;
      }
    }
    const bool ka = va && fa, kb = vb && fb;
    const f32x2 s2 = {sa, sb}, i2 = {ia, ib};
    // the pair's codes: fast and verified (bf16, narrow rows), else the exact definition from the scores
    const float ea = fast_eps(mxa, mn_a), eb = fast_eps(mxb, mn_b);
    const f32x2 rlo = {ia - ia * ea, ib - ib * eb}, rhi = {ia + ia * ea, ib + ib * eb};
    const uint32_t keep = (ka ? 0x0000FFFFu : 0u) | (kb ? 0xFFFF0000u : 0u);
    const uint32_t setm = ~keep & 0x80008000u;
    auto raw_pair = [&](int j) -> f32x2 {  // the scores of slot j of both rows (the exact paths: rare)
      const uint16_t a = raw_bits<T>(wa[j >> 3], j & 7), b = raw_bits<T>(wb[j >> 3], j & 7);
      return f32x2{to_f32<T>(__builtin_bit_cast(T, a)), to_f32<T>(__builtin_bit_cast(T, b))};
    };
    auto put = [&](int j, uint32_t code) {
#if TMX_FASTQ_LDS
      cv[pp][j] = (code & keep) | setm;
#else
      const int c = 512 * (j >> 3) + 8 * lane + (j & 7);
      s_tile[c * kSlots + (p ^ (lane & (kSlots - 1)))] = (code & keep) | setm;
#endif
    };
    if (fast) {
      uint32_t redo = 0;  // wave-uniform: slot j has an undecided pair in some lane
#pragma unroll
      for (int j = 0; j < 8 * NG; ++j) {
        bool und;
        put(j, fast_code2<T>(TMX_FASTQ_RECOMPUTE ? exp_fast2(P[j] - mx2) : P[j], rlo, rhi, und));
        redo |= (__ballot(und) != 0 ? 1u : 0u) << j;
      }
#ifdef TMX_FASTQ_NO_REDO  // timing experiment only: codes may differ from the definition
      redo = 0;
#endif
      if (redo != 0) {  // rare: the undecided slots from the definition (same wave, same lanes: LDS order holds)
        if constexpr (TMX_FASTQ_RECOMPUTE) {
#pragma unroll
          for (int j = 0; j < 8 * NG; ++j)
            if ((redo >> j) & 1u) put(j, exact_code2<T>(P[j], mx2, s2, i2, true));
        } else {
#if TMX_FASTQ_LDS
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          wa[g] = raw_lds[((2 * p) * NG + g) * kWave + lane];
          wb[g] = raw_lds[((2 * p + 1) * NG + g) * kWave + lane];
        }
        if constexpr (false) {
#else
        if constexpr (TMX_FASTQ_RELOAD && !UNALIGNED) {
#endif
          // the scores again from memory (the pass's own reads: cache hits) instead of holding them in 16 VGPRs
          const int lq = lo_ok ? lane : nvec - 1, hq = hi_ok ? lane + kWave : nvec - 1;
          const uint4* ra = reinterpret_cast<const uint4*>(preds + min(r0, n - 1) * ld);
          const uint4* rb = reinterpret_cast<const uint4*>(preds + min(r0 + 1, n - 1) * ld);
          wa[0] = ra[lq];
          wb[0] = rb[lq];
          if constexpr (NG == 2) {
            wa[1] = ra[hq];
            wb[1] = rb[hq];
          }
        }
#pragma unroll
        for (int j = 0; j < 8 * NG; ++j)
          if ((redo >> j) & 1u) put(j, exact_code2<T>(raw_pair(j), mx2, s2, i2, true));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8 * NG; ++j) put(j, exact_code2<T>(P[j], mx2, s2, i2, narrow));
    }
    if (!TMX_FASTQ_LDS && lane == 0 && pos.hist == nullptr) {
      if (ka && ta >= 0 && ta < C) atomicOr(&s_tile[ta * kSlots + (p ^ ((int)(ta >> 3) & (kSlots - 1)))], 0x00004000u);
      if (kb && tb >= 0 && tb < C) atomicOr(&s_tile[tb * kSlots + (p ^ ((int)(tb >> 3) & (kSlots - 1)))], 0x40000000u);
    }
    tt[2 * pp] = ta; tt[2 * pp + 1] = tb;
    am[2 * pp] = ama; am[2 * pp + 1] = amb;
    keepv[2 * pp] = ka; keepv[2 * pp + 1] = kb;
    slowv[2 * pp] = slow_a; slowv[2 * pp + 1] = slow_b;
    validv[2 * pp] = va; validv[2 * pp + 1] = vb;
  }
#if TMX_FASTQ_LDS
  __syncthreads();  // every wave is done with its parked rows: the image may overwrite them
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int p = wave + pp * kRowWaves;
#pragma unroll
    for (int j = 0; j < 8 * NG; ++j) {
      const int c = 512 * (j >> 3) + 8 * lane + (j & 7);
      s_tile[c * kSlots + (p ^ (lane & (kSlots - 1)))] = cv[pp][j];
    }
    if (lane == 0 && pos.hist == nullptr) {
      const int64_t ta = tt[2 * pp], tb = tt[2 * pp + 1];
      if (keepv[2 * pp] && ta >= 0 && ta < C) atomicOr(&s_tile[ta * kSlots + (p ^ ((int)(ta >> 3) & (kSlots - 1)))], 0x00004000u);
      if (keepv[2 * pp + 1] && tb >= 0 && tb < C) atomicOr(&s_tile[tb * kSlots + (p ^ ((int)(tb >> 3) & (kSlots - 1)))], 0x40000000u);
    }
  }
#endif
  if (pos.hist != nullptr) {
    pos_take(ptake, s_tile, keepv, tt, C, wave, row0_of(0), n);
    pos_book(ptake, pos, row_stats);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t t = tt[i];
      if (confmat != nullptr && keepv[i] && t >= 0 && t < C && am[i] < C) atomic_add_i64(confmat + t * C + am[i], 1);
      if (err != nullptr && validv[i] && (t < 0 || t >= C)) atomicOr(err, 1);
      if (slowv[i]) slow.rows[atomicAdd(slow.count, 1)] = static_cast<int>(row0_of(i >> 1) + (i & 1));
    }
  }
}

#ifndef TMX_ROWPASS_LEAN
#define TMX_ROWPASS_LEAN 1
#endif

#ifndef TMX_ROW_RAW_BARRIER
#define TMX_ROW_RAW_BARRIER 0  // measured: no difference (profiles/kexp_headline_r5.json)
#endif

template <typename T, int NG, bool SOFTMAX, bool FIXUP, bool PADDED, bool LEAN = (TMX_ROWPASS_LEAN != 0)>
__device__ __forceinline__ void row_tile(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n, int C, int ld,
                                          int64_t ignore_index, bool has_ignore, uint32_t* __restrict__ codes, int64_t n_pad,
                                          int64_t* __restrict__ confmat, int* __restrict__ err, bool rec, bool& saw_bad,
                                          SlowRows slow, uint32_t* __restrict__ s_tile, int64_t tile, float4* __restrict__ row_stats,
                                          PosSink pos = PosSink{}) {
  RowLoads<NG> L;
  row_tile_load<T, NG, PADDED>(preds, target, n, ld, tile, L);  // PADDED: rows of C % 8 != 0 scores at stride C
  PosTake ptake;
  if constexpr (FIXUP) pos = PosSink{};
  if constexpr (LEAN && SOFTMAX && !FIXUP)
    row_tile_softmax_lean<T, NG, PADDED>(preds, L, n, C, ld, ignore_index, has_ignore, confmat, err, rec, saw_bad, slow, s_tile, tile, row_stats, pos,
                                         ptake);
  else
    row_tile_compute<T, NG, SOFTMAX, FIXUP, PADDED>(L, n, C, ld, ignore_index, has_ignore, confmat, err, rec, saw_bad, slow, s_tile, tile,
                                                    row_stats, pos, ptake);
  // the image is complete once every wave's LDS writes are: a bare s_barrier after lgkmcnt(0).  __syncthreads() would
  // also wait (vmcnt(0)) for the global atomics just issued (confusion matrix, positive bins), ~1-2 us per tile
#if TMX_ROW_RAW_BARRIER
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
  store_tile<NG>(s_tile, codes, C, n_pad, tile);
}

// Normalisation mode (softmax if any valid score is outside [0, 1], as the reference decides per batch) is
// *speculated*: ``mode[0]`` is the mode this launch uses (the previous batch's verdict), the kernel records the real
// verdict for this batch in ``mode[1]`` (a plain store of 1 by any block that saw a witness).  A FIXUP launch exits
// at once unless mode[0] != mode[1], in which case it redoes the codes with the real mode (confusion matrix and error
// flags are mode independent and are not touched again).  ``class_hist_kernel`` rolls mode[0] = mode[1].
// Grid: one block per tile for the main launch (blocks stride over tiles, so a FIXUP launch can use a small grid).
template <typename T, bool FIXUP, int NG, bool PADDED>
__device__ __forceinline__ void mc_codes_block(int64_t vb, int64_t vgrid, const T* __restrict__ preds, const int64_t* __restrict__ target,
                                               int64_t n, int C, int ld, int* __restrict__ mode, int64_t ignore_index, bool has_ignore,
                                               uint32_t* __restrict__ codes, int64_t n_pad, int64_t* __restrict__ confmat,
                                               int* __restrict__ err, bool record_mode, int* __restrict__ slow_rows,
                                               int* __restrict__ slow_count, float4* __restrict__ row_stats,
                                               PosSink pos = PosSink{}) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[];  // [512 * NG][kSlots]
  int use_mode;
  if constexpr (FIXUP) {
    // the row pass that wrote mode[1] has completed (stream order, kernel-boundary release/acquire): plain loads
    const int m0 = mode[0];
    const int m1 = mode[1];
    if (m0 == m1) return;
    use_mode = m1;
  } else {
    use_mode = mode[0];
  }
  // XCD-aware tile order: dispatch round-robins blocks over the 8 XCDs (block b -> XCD b % 8), so give each XCD a
  // contiguous run of tiles: tiles 2q and 2q+1 then run on one XCD and the two 64-B halves of every 128-B line of
  // the class-major scratch meet in that XCD's L2 before write-back.
  const int64_t ntiles = (n + kTileRows - 1) / kTileRows;
  const int64_t per_xcd = (ntiles + 7) / 8;
  const bool rec = !FIXUP && record_mode;
  bool saw_bad = false;
  const SlowRows slow{slow_rows, slow_count};
  auto run_tile = [&](int64_t b) {
    const int64_t tile = (b % 8) * per_xcd + b / 8;
    if (tile >= ntiles) return;
    if (use_mode != 0)
      row_tile<T, NG, true, FIXUP, PADDED>(preds, target, n, C, ld, ignore_index, has_ignore, codes, n_pad, confmat, err, rec, saw_bad, slow, s_tile, tile,
                                           row_stats, pos);
    else
      row_tile<T, NG, false, FIXUP, PADDED>(preds, target, n, C, ld, ignore_index, has_ignore, codes, n_pad, confmat, err, rec, saw_bad, slow, s_tile, tile,
                                            row_stats, pos);
  };
  if constexpr (FIXUP) {  // rare: blocks stride over the tiles (small grid, cheap early exit)
    for (int64_t b = vb; b < per_xcd * 8; b += vgrid) {
      run_tile(b);
      __syncthreads();  // the LDS image is rewritten by the next tile of this block
    }
  } else {  // one tile per block: no loop, so nothing of one tile's register state lives across another's
    run_tile(vb);
  }
  if constexpr (!FIXUP) {
    if (record_mode && __syncthreads_or(saw_bad) && threadIdx.x == 0 &&
        __hip_atomic_load(mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
      __hip_atomic_store(mode + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T, bool FIXUP, int NG, bool PADDED>
__global__ void __launch_bounds__(kRowThreads, 4) mc_codes_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                    int64_t n, int C, int ld, int* __restrict__ mode,
                                                                    int64_t ignore_index, bool has_ignore,
                                                                    uint32_t* __restrict__ codes, int64_t n_pad,
                                                                    int64_t* __restrict__ confmat, int* __restrict__ err,
                                                                    bool record_mode, int* __restrict__ slow_rows,
                                                                    int* __restrict__ slow_count, float4* __restrict__ row_stats = nullptr,
                                                                    PosSink pos = PosSink{}) {
  mc_codes_block<T, FIXUP, NG, PADDED>(blockIdx.x, gridDim.x, preds, target, n, C, ld, mode, ignore_index, has_ignore, codes, n_pad,
                                       confmat, err, record_mode, slow_rows, slow_count, row_stats, pos);
}

// Multilabel row pass: the same tile / LDS image / class-major scratch as the multiclass row pass, but every element
// is its own binary problem — code = RNE16(sigmoid(x)) (torch's 1 / (1 + exp(-x)) in fp32) or the raw score when the
// batch is already in [0, 1] (the range pre-pass decides, as in the reference), flags from the element's own target
// (1 -> positive, ignore_index -> skip, anything else -> negative).  Labels play the role of classes; the class
// pass is shared.  Targets are int64 [N, L]: the 8 labels a lane owns per group are one 64-B piece of the row.
template <typename T, int NG>
__device__ __forceinline__ void row_tile_ml(const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n, int L,
                                            bool do_sigmoid, int64_t ignore_index, bool has_ignore,
                                            uint32_t* __restrict__ codes, int64_t n_pad, uint32_t* __restrict__ s_tile,
                                            int64_t tile, int* __restrict__ err) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int nvec = L / 8;
  bool bad = false;
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  const int lq = lo_ok ? lane : nvec - 1;
  const int hq = hi_ok ? lane + kWave : nvec - 1;
  auto row0_of = [&](int pp) -> int64_t { return tile * kTileRows + 2 * (wave + pp * kRowWaves); };
  uint4 raw[2][2][2];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4* row = reinterpret_cast<const uint4*>(preds + min(row0_of(pp) + h, n - 1) * L);
      raw[pp][h][0] = row[lq];
      if constexpr (NG == 2) raw[pp][h][1] = row[hq];
    }
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int p = wave + pp * kRowWaves;
    const int64_t r0 = row0_of(pp);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const bool ok = g == 0 ? lo_ok : hi_ok;
      const int q = g == 0 ? lq : hq;
      uint32_t code[2][8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t r = r0 + h;
        const bool valid = r < n && ok;
        const longlong2* trow = reinterpret_cast<const longlong2*>(target + min(r, n - 1) * L + 8 * q);
        longlong2 tt[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) tt[k] = trow[k];
        const uint4 w = raw[pp][h][g];
        float v[8];
        unpack8<T>(w, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int64_t t = (k & 1) ? tt[k >> 1].y : tt[k >> 1].x;
          const uint32_t b = do_sigmoid ? (uint32_t)round_bits16<T>(1.f / (1.f + expf(-v[k]))) : (uint32_t)raw_bits<T>(w, k);
          uint32_t c16 = raw_code<T>(b);
          bad |= valid && !(has_ignore && t == ignore_index) && t != 0 && t != 1;
          if (!valid || (has_ignore && t == ignore_index)) c16 = 0x8000u;
          else if (t == 1 && !(c16 & 0x8000u)) c16 |= 0x4000u;
          code[h][k] = c16;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = 512 * g + 8 * lane + k;
        s_tile[c * kSlots + (p ^ (lane & (kSlots - 1)))] = code[0][k] | (code[1][k] << 16);
      }
    }
  }
  if (bad && err) atomicOr(err, 1);
  __syncthreads();
  store_tile<NG>(s_tile, codes, L, n_pad, tile);
}

template <typename T, int NG>
__global__ void __launch_bounds__(kRowThreads, 4) ml_codes_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                   int64_t n, int L, const int* __restrict__ sigmoid_flag,
                                                                   int64_t ignore_index, bool has_ignore,
                                                                   uint32_t* __restrict__ codes, int64_t n_pad, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[];  // [512 * NG][kSlots]
  const int64_t ntiles = (n + kTileRows - 1) / kTileRows;
  const int64_t per_xcd = (ntiles + 7) / 8;
  const int64_t b = blockIdx.x;
  const int64_t tile = (b % 8) * per_xcd + b / 8;  // XCD-aware order, as the multiclass row pass
  if (tile >= ntiles) return;
  row_tile_ml<T, NG>(preds, target, n, L, sigmoid_flag[0] != 0, ignore_index, has_ignore, codes, n_pad, s_tile, tile, err);
}

// Class pass: one 1024-thread workgroup per (class, row split), two per CU (64-KiB LDS).
//   PACKED = false (multiclass: positives are 1 / C of the codes): an LDS u32 histogram of the negatives, positives
//            straight to the int64 bins with global atomics.
//   PACKED = true (multilabel: ~half the codes are positive; a global atomic per positive took 287 us at
//            16384 x 1000): both halves in ONE LDS word per code — negatives in the low 16 bits, positives in the high
//            16 bits — one LDS atomic per code, rows consumed in chunks of at most kClassChunk so a 16-bit half cannot
//            overflow.
// Every flush adds the LDS counts to the int64 histogram (plain read-modify-write by the exclusive owner when there
// is one split, atomics otherwise).  Measured at 65536 x 1000 multiclass: 1024 threads 32 us vs 39 us at 512
// and 47-61 us for a variant with a 128-KiB two-array histogram (one block per CU): occupancy beats everything else.
// It also finishes the rare rows of the row pass (NaN / +-inf rows, listed in ``slow_rows``): torch semantics — the
// softmax of such a row is all NaN (every code skipped), in probability mode each score keeps its own code, the
// arg-max is the first NaN else the first maximum.  List 0 (speculated pass): codes unless a FIXUP pass replaced
// them, confusion matrix always; list 1 (FIXUP pass): codes with the corrected mode.
// ``state`` = {count0, count1, ticket, bmode0, bmode1}: the batch's mode pair comes from bmode (written by
// mode_roll_kernel); the last block to finish (ticket) clears the counts for the next batch that uses this state —
// every block has read them by then.
constexpr int kClassThreads = 1024;
// 16-B code vectors in flight per thread per iteration (a 65536-row class is 8 vectors per thread of 1024)
#ifndef TMX_CLASS_UNROLL
#define TMX_CLASS_UNROLL 8
#endif
constexpr int kClassUnroll = TMX_CLASS_UNROLL;
constexpr int kTrashBin = kCodes - 1;  // no valid 16-bit score in [0, 1] maps here (bf16 <= 0x3F80, fp16 <= 0x3C00)
constexpr int64_t kClassChunk = 65528;  // rows per LDS flush: a 16-bit half never overflows (multiple of 8)
// The u16 multiclass pass (split-half layout) counts whole 65536-row chunks: a half can only wrap when all 65536 codes
// of a chunk are one negative code, which the chunk's all-equal test catches and books directly (a 65528-row chunk
// left an 8-row tail and a second flush per class at the headline's 65536 rows: 41 -> 36 us).
constexpr int64_t kClassChunkU16 = 65536;

// ``bneg`` / ``bpos`` (optional): the batch histogram of a forward() call, flushed beside the accumulated one (its bins
// are zero before the batch): a plain store when ``bstore`` (the block's only writer of those bins so far), else atomics.
template <bool PACKED, int NT = kClassThreads>
__device__ __forceinline__ void class_flush(uint32_t* __restrict__ s_h, int64_t* __restrict__ neg_hist,
                                            int64_t* __restrict__ pos_hist, bool exclusive, int& lo, int& hi,
                                            int64_t* __restrict__ bneg = nullptr, int64_t* __restrict__ bpos = nullptr,
                                            bool bstore = false) {
  for (int i = threadIdx.x; i < kCodes; i += NT) {
    const uint32_t w = i == kTrashBin ? 0u : s_h[i];  // the trash bin holds skipped codes (non-PACKED pass)
    if (w) {
      lo = min(lo, i);
      hi = max(hi, i);
      const uint32_t neg = PACKED ? (w & 0xFFFFu) : w, pos = PACKED ? (w >> 16) : 0u;
      if (exclusive) {
        if (neg) neg_hist[i] += neg;
        if (pos) pos_hist[i] += pos;
      } else {
        if (neg) atomic_add_i64(neg_hist + i, neg);
        if (pos) atomic_add_i64(pos_hist + i, pos);
      }
      if (bneg != nullptr) {
        if (bstore) {
          if (neg) bneg[i] = neg;
          if (pos) bpos[i] = pos;
        } else {
          if (neg) atomic_add_i64(bneg + i, neg);
          if (pos) atomic_add_i64(bpos + i, pos);
        }
      }
      s_h[i] = 0u;
    }
  }
}

// 16-bit-packed LDS histogram layout: bin b lives in word (b mod 8192), low half for b < 8192, high half above.  Softmax
// codes cluster in a few binades (bins ~14000-16256), so consecutive codes land in consecutive words -- different LDS
// banks -- instead of sharing one word (the b >> 1 layout put every second pair of lanes on the same address, and
// same-address atomics serialise like bank conflicts).  The trash bin 16383 stays the high half of the last word.
#ifndef TMX_FLUSH_RMW
#define TMX_FLUSH_RMW 0
#endif
__device__ __forceinline__ uint32_t u16_word(uint32_t bin) { return bin & (kCodes / 2 - 1); }
__device__ __forceinline__ uint32_t u16_one(uint32_t bin) { return 1u << ((bin >> (kCodeBits - 1)) << 4); }

// Flush of the 16-bit-packed multiclass histogram (two bins per u32 word; the trash bin is the high half of the last
// word): negatives only (positives went straight to global), same exclusive / atomic and batch-histogram rules.
template <int NT>
__device__ __forceinline__ void class_flush_u16(uint32_t* __restrict__ s_w, int64_t* __restrict__ neg_hist, bool exclusive, int& lo, int& hi,
                                                int64_t* __restrict__ bneg, bool bstore) {
  for (int w = threadIdx.x; w < kCodes / 2; w += NT) {
    uint32_t v = s_w[w];
    if (w == kTrashBin / 2) v &= 0xFFFFu;
    if (v) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t cnt = h ? (v >> 16) : (v & 0xFFFFu);
        if (!cnt) continue;
        const int i = w + h * (kCodes / 2);
        lo = min(lo, i);
        hi = max(hi, i);
#if TMX_FLUSH_RMW
        if (exclusive) neg_hist[i] += cnt;
        else atomic_add_i64(neg_hist + i, cnt);
#else
        // a non-returning atomic even when this block owns the class: the plain += waited on a global load per bin
        (void)exclusive;
        atomic_add_i64(neg_hist + i, cnt);
#endif
        if (bneg != nullptr) {
          if (bstore) bneg[i] = cnt;
          else atomic_add_i64(bneg + i, cnt);
        }
      }
      s_w[w] = 0u;
    }
  }
}

// Partial flush (small-class route): the block's occupied LDS range [blo, bhi] goes to its own slice of a scratch
// [C][splits][kCodes] with plain coalesced stores and the range to ``prange``; class_partial_reduce_kernel then sums
// the splits per bin.  With few classes every split of a class hits the same few thousand bins, and a global int64
// atomic per (split, bin) was the class pass's cost (C = 10, 1M rows: 640 blocks x ~4k bins).
template <int NT>
__device__ __forceinline__ void class_store_partial(const uint32_t* __restrict__ s_h, uint32_t* __restrict__ out,
                                                    int* __restrict__ range, int& lo, int& hi) {
  __shared__ int s_rng[2];
  if (threadIdx.x == 0) {
    s_rng[0] = kCodes;
    s_rng[1] = -1;
  }
  __syncthreads();
  int tlo = kCodes, thi = -1;
  for (int i = threadIdx.x; i < kCodes; i += NT)
    if (s_h[i]) {
      tlo = min(tlo, i);
      thi = max(thi, i);
    }
  tlo = wave_min_i32(tlo);
  thi = wave_max_i32(thi);
  if ((threadIdx.x & (kWave - 1)) == 0 && thi >= 0) {
    atomicMin(&s_rng[0], tlo);
    atomicMax(&s_rng[1], thi);
  }
  __syncthreads();
  const int blo = s_rng[0], bhi = s_rng[1];
  for (int i = blo + static_cast<int>(threadIdx.x); i <= bhi; i += NT) out[i] = s_h[i];
  if (threadIdx.x == 0) {
    range[0] = blo;
    range[1] = bhi;
  }
  lo = min(lo, blo);
  hi = max(hi, bhi);
}

template <typename T, bool PACKED, int NT, bool U16 = false>
__device__ __forceinline__ void class_hist_block(int64_t vb, int64_t vgrid, const uint16_t* __restrict__ codes, int64_t n_pad, int splits,
                                                 int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
                                                 const int64_t* __restrict__ target, int64_t n, const int* __restrict__ bmode,
                                                 bool speculative, const int* __restrict__ slow_rows, int* __restrict__ state,
                                                 int64_t* __restrict__ confmat, int* __restrict__ code_range, int* __restrict__ roll_mode,
                                                 uint32_t* __restrict__ partial = nullptr, int* __restrict__ prange = nullptr,
                                                 int64_t* __restrict__ batch_hist = nullptr, int* __restrict__ batch_range = nullptr,
                                                 const float4* __restrict__ row_stats = nullptr) {
  static_assert(!(PACKED && U16), "the 16-bit-packed histogram is the multiclass form");
  // [kCodes]: neg, or neg (lo 16) | pos (hi 16) (PACKED); U16: [kCodes / 2] words holding bins 2w (lo) and 2w + 1 (hi)
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];
  __shared__ int s_info[4];
  int lo = kCodes, hi = -1;  // occupied code range this thread touched (compute() then scans only that range)
  const int C = static_cast<int>(vgrid / splits);
  const int c = static_cast<int>(vb / splits), sp = static_cast<int>(vb % splits);
  if (threadIdx.x == 0) {  // the row-pass kernels of this batch are complete (stream order / event wait)
    s_info[0] = bmode[0];
    s_info[1] = speculative ? bmode[1] : bmode[0];
    s_info[2] = state[0];
    s_info[3] = state[1];
  }
  uint4* s4 = reinterpret_cast<uint4*>(s_h);
  for (int i = threadIdx.x; i < (U16 ? kCodes / 8 : kCodes / 4); i += NT) s4[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  int64_t* neg_hist = hist + ((int64_t)c * 2) * kCodes;
  int64_t* pos_hist = hist + ((int64_t)c * 2 + 1) * kCodes;
  int64_t* bneg = batch_hist != nullptr ? batch_hist + ((int64_t)c * 2) * kCodes : nullptr;
  int64_t* bpos = batch_hist != nullptr ? batch_hist + ((int64_t)c * 2 + 1) * kCodes : nullptr;
  bool bfirst = true;  // no flush of this block has written the batch bins yet
  const bool exclusive = splits == 1;
  const uint4* col = reinterpret_cast<const uint4*>(codes + (int64_t)c * n_pad);
  const int64_t nv = n_pad / 8;
  const int64_t per = (nv + splits - 1) / splits;
  const int64_t v0 = sp * per, v1 = v0 + per < nv ? v0 + per : nv;
  constexpr int64_t kChunkV = U16 ? kClassChunkU16 / 8 : (PACKED ? kClassChunk / 8 : (int64_t{1} << 62));
  // Refit (multiclass routes, no FIXUP launch): when the speculated normalisation mode of this batch was wrong
  // (rare: the first batch of a metric, or inputs switching between logits and probabilities) the codes were written
  // in the wrong mode, and this class's codes are rebuilt from the scores themselves with the row pass's per-row
  // softmax statistics -- the same instruction sequence as the row pass (exp_nonpos2, div_rn2, pack_rne2), so the
  // same bits.  A strided gather (~0.3 ms for the whole batch) instead of a FIXUP launch on every update (4.5 us).
  const bool refit = speculative && row_stats != nullptr && s_info[0] != s_info[1];
  if (refit) {
    // rewrite this class's own slice of the code scratch (rows [8 v0, 8 v1) of class c belong to this workgroup
    // alone), then count it with the normal loop below
    const int m1 = s_info[1];
    uint16_t* ccol = const_cast<uint16_t*>(codes) + (int64_t)c * n_pad;
    for (int64_t r = v0 * 8 + threadIdx.x; r < v1 * 8; r += NT) {
      uint32_t code = 0x8000u;
      if (r < n) {
        const float4 st = row_stats[r];
        const uint32_t fl = __float_as_uint(st.z);
        const T xv = preds[r * ld + c];
        if (m1 != 0) {
          if ((fl & 3u) == 3u) {  // counted row with a finite softmax (NaN / inf rows: every code skipped)
            const float inv = 1.f / st.y;
            // the packed pair sequence of both row passes (row_tile_compute / mc_codes_small_kernel, round 5)
            const f32x2 e = exp_nonpos2(f32x2{to_f32<T>(xv) - st.x, 0.f});
            code = pack_rne2<T>(div_rn2(f32x2{e.x, 0.f}, f32x2{st.y, 1.f}, f32x2{inv, 1.f})) & 0xFFFFu;
          }
        } else if (fl & 1u) {
          code = raw_code<T>(bits16<T>(xv));
        }
        if (!(code & 0x8000u) && target[r] == c) code |= 0x4000u;
      }
      ccol[r] = static_cast<uint16_t>(code);
    }
    __threadfence();  // the rewritten codes are read back by other waves of this workgroup
    __syncthreads();
  }
  for (int64_t cb = v0; cb < v1; cb += kChunkV) {
    const int64_t ce = cb + kChunkV < v1 ? cb + kChunkV : v1;
    // U16, full 65536-row chunk: OR of every code's difference from the chunk's first code (all equal -> a half may
    // have wrapped, fixed below); a partial chunk cannot reach 65536 in one bin
    static_assert(!U16 || (kClassChunkU16 / 8) % (kClassUnroll * NT) == 0, "a full u16 chunk has no padding vectors");
    const bool full = U16 && ce - cb == kChunkV;
    uint32_t ref2 = 0u, diff = 0u;
    if (full) {
      const uint32_t r0 = col[cb].x & 0xFFFFu;
      ref2 = r0 | (r0 << 16);
    }
    for (int64_t v = cb + threadIdx.x; v < ce; v += kClassUnroll * NT) {
      uint4 w[kClassUnroll];
#pragma unroll
      for (int u = 0; u < kClassUnroll; ++u)
        w[u] = (v + u * NT < ce) ? col[v + u * NT] : make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);
      if (full) {
#pragma unroll
        for (int u = 0; u < kClassUnroll; ++u) diff |= ((w[u].x ^ ref2) | (w[u].y ^ ref2)) | ((w[u].z ^ ref2) | (w[u].w ^ ref2));
      }
#pragma unroll
      for (int u = 0; u < kClassUnroll; ++u) {
        const uint32_t parts[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
        if constexpr (PACKED) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
            if (x & 0x8000u) continue;
            atomicAdd(&s_h[x & 0x3FFFu], (x & 0x4000u) ? 0x10000u : 1u);
          }
        } else {
          // Branch-free common case: every code is counted into the LDS bin of its value (a skip code into the
          // never-used trash bin), positives included; the rare positive (1 / C of the codes) is then moved from the
          // LDS bin to the int64 positive histogram under a wave-uniform test of the whole 16-B word.  Before, every
          // code took a two-level divergent branch (exec-mask save / restore per code).
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
            const uint32_t bin = (x & 0x8000u) ? (uint32_t)kTrashBin : (x & 0x3FFFu);
            if constexpr (U16) atomicAdd(&s_h[u16_word(bin)], u16_one(bin));
            else atomicAdd(&s_h[bin], 1u);
          }
          const uint32_t anypos = (parts[0] | parts[1] | parts[2] | parts[3]) & 0x40004000u;
          if (__builtin_expect(__ballot(anypos != 0) != 0, 0) && anypos != 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
              if ((x & 0xC000u) == 0x4000u) {
                if constexpr (U16) atomicSub(&s_h[u16_word(x & 0x3FFFu)], u16_one(x & 0x3FFFu));
                else atomicSub(&s_h[x & 0x3FFFu], 1u);
                atomic_add_i64(pos_hist + (x & 0x3FFFu), 1);
                if (bpos != nullptr) atomic_add_i64(bpos + (x & 0x3FFFu), 1);
                lo = min(lo, (int)(x & 0x3FFFu));
                hi = max(hi, (int)(x & 0x3FFFu));
              }
            }
          }
        }
      }
    }
    if constexpr (U16) {
      if (full && !__syncthreads_or(diff != 0u)) {
        // every code of the chunk is ref2's: a negative code's count 65536 wrapped its 16-bit half (low half: carried
        // 1 into the high half; high half: carried out) -- undo it in LDS and book the count directly.  Positives
        // (added then subtracted) and the trash bin are exact modulo 2^32.
        const uint32_t x = ref2 & 0xFFFFu;
        if (threadIdx.x == 0 && (x & 0xC000u) == 0u) {
          const uint32_t bin = x & 0x3FFFu;
          if (!(bin >> (kCodeBits - 1))) s_h[u16_word(bin)] -= 0x10000u;
          atomic_add_i64(neg_hist + bin, kChunkV * 8);
          if (bneg != nullptr) atomic_add_i64(bneg + bin, kChunkV * 8);
          lo = min(lo, (int)bin);
          hi = max(hi, (int)bin);
        }
      }
    }
    if (ce < v1) {  // more rows than one chunk: flush before a 16-bit half can overflow
      __syncthreads();
      if constexpr (U16) class_flush_u16<NT>(s_h, neg_hist, exclusive, lo, hi, bneg, exclusive && bfirst);
      else class_flush<PACKED, NT>(s_h, neg_hist, pos_hist, exclusive, lo, hi, bneg, bpos, exclusive && bfirst);
      bfirst = false;
      __syncthreads();
    }
  }
  // rare rows (usually none): this class's code of every listed row (split 0 only), and one row's arg-max per block
  const int m0 = s_info[0], m1 = s_info[1];
  const bool fixed = speculative && m0 != m1;
  const int64_t n0 = s_info[2], n1 = s_info[3];
  if (sp == 0) {
    for (int64_t i = threadIdx.x; i < n0 + n1; i += NT) {
      const int lst = i < n0 ? 0 : 1;
      if (lst == 0 && fixed) continue;
      const int64_t r = slow_rows[lst * n + (lst == 0 ? i : i - n0)];
      if ((lst == 1 ? m1 : m0) != 0) continue;  // softmax of a NaN / inf row: all NaN, every code skipped
      const uint32_t code = raw_code<T>(bits16<T>(preds[r * ld + c]));
      if (code & 0x8000u) continue;
      lo = min(lo, (int)code);
      hi = max(hi, (int)code);
      if (target[r] == c) atomic_add_i64(pos_hist + code, 1);
      else atomic_add_i64(neg_hist + code, 1);
      if (bneg != nullptr) atomic_add_i64((target[r] == c ? bpos : bneg) + code, 1);
    }
  }
  if (confmat != nullptr && threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    for (int64_t i = vb; i < n0; i += vgrid) {
      const int64_t r = slow_rows[i];
      const int64_t t = target[r];
      if (t < 0 || t >= C) continue;
      const T* row = preds + r * ld;
      float best = -INFINITY;
      int bi = C, first_nan = C;
      for (int cc = lane; cc < C; cc += kWave) {
        const float v = to_f32<T>(row[cc]);
        if (v != v) first_nan = min(first_nan, cc);
        else if (bi == C || v > best) { best = v; bi = cc; }  // ascending classes per lane: strict > keeps the first
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) first_nan = min(first_nan, __shfl_xor(first_nan, off, kWave));
      wave_argmax(best, bi);
      const int am = first_nan < C ? first_nan : bi;
      if (lane == 0 && am < C) atomic_add_i64(confmat + t * C + am, 1);
    }
  }
  __syncthreads();
  // rare-row codes went to the int64 bins by atomics: then the last flush must be atomic too
  if (partial != nullptr) class_store_partial<NT>(s_h, partial + vb * kCodes, prange + 2 * vb, lo, hi);
  else if constexpr (U16) class_flush_u16<NT>(s_h, neg_hist, exclusive && n0 + n1 == 0, lo, hi, bneg, exclusive && bfirst && n0 + n1 == 0);
  else class_flush<PACKED, NT>(s_h, neg_hist, pos_hist, exclusive && n0 + n1 == 0, lo, hi, bneg, bpos, exclusive && bfirst && n0 + n1 == 0);
  // partial mode: class_partial_reduce_kernel derives the class ranges from prange and resets / rolls the state
  // (no per-block global atomics on the same few words — with few classes hundreds of blocks share each class);
  // only rare-row codes (tracked in lo / hi here, not in the partial histogram) still go through atomics
  if (partial != nullptr && n0 + n1 == 0) return;
  if (code_range != nullptr || batch_range != nullptr) {  // per-class running range [C][2]: one min / max per wave
    lo = wave_min_i32(lo);
    hi = wave_max_i32(hi);
    if ((threadIdx.x & (kWave - 1)) == 0 && hi >= 0) {
      if (code_range != nullptr) {
        atomicMin(code_range + 2 * c, lo);
        atomicMax(code_range + 2 * c + 1, hi);
      }
      if (batch_range != nullptr) {
        atomicMin(batch_range + 2 * c, lo);
        atomicMax(batch_range + 2 * c + 1, hi);
      }
    }
  }
  if (partial != nullptr) return;
  if (threadIdx.x == 0) {
    // No fence: the only ordering needed is "every block's read of mode / counts happened before the reset", and
    // each block consumed those values (s_info, above) before taking its ticket.  (An agent-scope release here writes
    // back the XCD's L2 once per block: it doubled the kernel's time.)
    if (__hip_atomic_fetch_add(state + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)vgrid - 1) {
      state[0] = state[1] = 0;
      state[2] = 0;
      if (roll_mode != nullptr) {  // speculation roll (every block read the mode pair before its ticket)
        const int m1 = roll_mode[1];
        roll_mode[0] = m1;
        roll_mode[1] = 0;
      }
    }
  }
}

template <typename T, bool PACKED>
__global__ void __launch_bounds__(kClassThreads) class_hist_kernel(const uint16_t* __restrict__ codes, int64_t n_pad, int splits,
                                                                   int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
                                                                   const int64_t* __restrict__ target, int64_t n,
                                                                   const int* __restrict__ bmode, bool speculative,
                                                                   const int* __restrict__ slow_rows, int* __restrict__ state,
                                                                   int64_t* __restrict__ confmat, int* __restrict__ code_range,
                                                                   int* __restrict__ roll_mode, int64_t* __restrict__ batch_hist = nullptr,
                                                                   int* __restrict__ batch_range = nullptr) {
  class_hist_block<T, PACKED, kClassThreads>(blockIdx.x, gridDim.x, codes, n_pad, splits, hist, preds, ld, target, n, bmode, speculative,
                                             slow_rows, state, confmat, code_range, roll_mode, nullptr, nullptr, batch_hist, batch_range);
}

// Multiclass class pass with the 16-bit-packed histogram: 512-thread workgroups with 32 KiB of LDS -> four per CU,
// so the 1000 classes of the headline run in one round (the 1024-thread / 64-KiB form needs two rounds whose load,
// count and flush phases line up across each CU's blocks).  Rows are counted in chunks of at most kClassChunk so a
// 16-bit half never overflows.  Measured at 65536 x 1000 bf16 (tools/kexp/classpass_u16_exp.hip): update sequence
// 116.9 -> 99.6 us, identical histograms and code ranges.
constexpr int kClassThreadsU16 = 512;
template <typename T>
__global__ void __launch_bounds__(kClassThreadsU16) class_hist_u16_kernel(const uint16_t* __restrict__ codes, int64_t n_pad, int splits,
                                                                         int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
                                                                         const int64_t* __restrict__ target, int64_t n,
                                                                         const int* __restrict__ bmode, bool speculative,
                                                                         const int* __restrict__ slow_rows, int* __restrict__ state,
                                                                         int64_t* __restrict__ confmat, int* __restrict__ code_range,
                                                                         int* __restrict__ roll_mode, int64_t* __restrict__ batch_hist,
                                                                         int* __restrict__ batch_range, const float4* __restrict__ row_stats = nullptr) {
  class_hist_block<T, false, kClassThreadsU16, true>(blockIdx.x, gridDim.x, codes, n_pad, splits, hist, preds, ld, target, n, bmode,
                                                     speculative, slow_rows, state, confmat, code_range, roll_mode, nullptr, nullptr,
                                                     batch_hist, batch_range, row_stats);
}

// ---- multiclass class pass, windowed u32 form (round 5) ------------------------------------------------------------
// class_hist_u16_kernel spent ~12 VALU instructions per code (unpack one 16-bit code, route skip codes to the trash bin,
// split the bin into a u16 word and a half, test every code for the positive flag; profiles/pmc_headline_r4.json) and
// with that VALU the pass ran at ~55 % of the read floor; without any of its atomics it still took 36 of its 43 us
// (profiles/kexp_classpass_r5.json).  Here the histogram is one u32 word per bin of a window of 8192 codes, so a count
// is a constant 1 at a byte offset computed for two codes at once:
//   y = min(max(code, 8190), 16382)   (v_pk_max_u16 + v_pk_min_u16: both codes of a dword)
//   offset = 4 y - 32760              (one v_mad_u32_u16 per code, the 16-bit half selected by op_sel)
// Word 0 collects every code <= 8190 (the low bucket: scores below 2^-63, rare), words 1..8190 are bins 8191..16380,
// word 8191 (bin 16381, above every bf16 / fp16 score in [0, 1]: 16256 / 15360) collects skip codes (bit 15) AND positives (bit 14),
// which are booked straight into the int64 positive bins under a wave-uniform test of the whole 16-B vector (1 / C of
// the codes).  A block whose low bucket is not empty re-reads its codes once and counts the window [0, 8190] the same
// way (y = min(code, 8191), word 8191 the trash): exact for any input, one extra pass only for classes holding
// probabilities below 2^-63 (logit gaps above ~43).  Per code: ~2.5 VALU instructions and one ds_add_u32.
constexpr int kHiBase = kCodes / 2 - 2;                     // 8190: word 0 = the low bucket
constexpr int kHiWords = kCodes / 2;                        // 8192 words: bins 8191..16381 at words 1..8191
constexpr int kHiTrash = kHiBase + kHiWords - 1;            // 16381: skip codes and positives (word 8191)
constexpr size_t kHiLdsBytes = (size_t)kHiWords * 4;        // exactly 32 KiB (no other LDS object): the workgroup fits
                                                            // beside two 64-KiB row-pass workgroups on a 160-KiB CU
#ifndef TMX_HI_UNROLL
#define TMX_HI_UNROLL 4
#endif
constexpr int kHiUnroll = TMX_HI_UNROLL;  // 16-B code vectors per thread per step (two steps' worth in registers)

typedef unsigned short hi_u16x2 __attribute__((ext_vector_type(2)));

// count the codes of one 16-B vector into the window (LOW: the [0, 8190] re-pass) -- positives are returned as a
// bit mask (0x40004000 bits of any dword) for the caller's wave-uniform test
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// LDS word at byte offset ``off`` of the dynamic allocation (which starts at LDS address 0 in these kernels: no static
// __shared__ object precedes it), counted by one ds_add_u32 with no base-address arithmetic
#ifndef TMX_CLASS_ABL
#define TMX_CLASS_ABL 0  // kernel-harness ablation (tools/kexp): 1 = no LDS count atomics.  Always 0 in the library.
#endif
__device__ uint32_t g_abl_sink;
__device__ __forceinline__ void lds_inc(uint32_t off) {
#if TMX_CLASS_ABL & 1
  if (off == 0xFFFFFFFFu) g_abl_sink = off;
#else
  __hip_atomic_fetch_add(reinterpret_cast<lds_u32*>(static_cast<size_t>(off)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}

// count the codes of one 16-B vector into the window (LOW: the [0, 8190] re-pass): per dword a saturating v_pk_sub_u16
// and a v_pk_min_u16 give both codes' window indices, two SDWA shifts their byte offsets
template <bool LOW>
__device__ __forceinline__ void hi_count4(const uint4& v) {
  const uint32_t parts[4] = {v.x, v.y, v.z, v.w};
  uint32_t idx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hi_u16x2 c = __builtin_bit_cast(hi_u16x2, parts[k]);
    if constexpr (LOW) c = __builtin_elementwise_min(c, (hi_u16x2){kHiBase + 1, kHiBase + 1});
    else c = __builtin_elementwise_min(__builtin_elementwise_sub_sat(c, (hi_u16x2){kHiBase, kHiBase}),
                                       (hi_u16x2){kHiTrash - kHiBase, kHiTrash - kHiBase});
    idx[k] = __builtin_bit_cast(uint32_t, c);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    lds_inc((idx[k] & 0xFFFFu) << 2);
    lds_inc((idx[k] >> 16) << 2);
  }
}

// Last workgroup of a class-pass launch: reset the batch state words and roll the speculation (every workgroup read
// them before its ticket; class_hist_block)
__device__ __forceinline__ void class_hi_ticket(int* __restrict__ state, int* __restrict__ roll_mode, int64_t vgrid) {
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(state + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)vgrid - 1) {
      state[0] = state[1] = 0;
      state[2] = 0;
      if (roll_mode != nullptr) {
        const int mr = roll_mode[1];
        roll_mode[0] = mr;
        roll_mode[1] = 0;
      }
    }
  }
}

template <typename T, int NT>
__device__ __forceinline__ void class_hist_hi_block(int64_t vb, int64_t vgrid, const uint16_t* __restrict__ codes, int64_t n_pad, int splits,
                                                    int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
                                                    const int64_t* __restrict__ target, int64_t n, const int* __restrict__ bmode,
                                                    bool speculative, const int* __restrict__ slow_rows, int* __restrict__ state,
                                                    int64_t* __restrict__ confmat, int* __restrict__ code_range, int* __restrict__ roll_mode,
                                                    int64_t* __restrict__ batch_hist, int* __restrict__ batch_range,
                                                    const float4* __restrict__ row_stats, bool pos_booked) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];  // [kHiWords] words, at LDS address 0
  int lo = kCodes, hi = -1;
  const int C = static_cast<int>(vgrid / splits);
  const int c = static_cast<int>(vb / splits), sp = static_cast<int>(vb % splits);
  // the row-pass kernels of this batch are complete (stream order); read before this block's ticket (below), so before
  // the last block resets the state words
  const int info_m0 = bmode[0], info_m1 = speculative ? bmode[1] : bmode[0];
  const int info_n0 = state[0], info_n1 = state[1];
  uint4* s4 = reinterpret_cast<uint4*>(s_h);
  for (int i = threadIdx.x; i < kHiWords / 4; i += NT) s4[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  int64_t* neg_hist = hist + ((int64_t)c * 2) * kCodes;
  int64_t* pos_hist = hist + ((int64_t)c * 2 + 1) * kCodes;
  int64_t* bneg = batch_hist != nullptr ? batch_hist + ((int64_t)c * 2) * kCodes : nullptr;
  int64_t* bpos = batch_hist != nullptr ? batch_hist + ((int64_t)c * 2 + 1) * kCodes : nullptr;
  const uint4* col = reinterpret_cast<const uint4*>(codes + (int64_t)c * n_pad);
  const int64_t nv = n_pad / 8;
  const int64_t per = (nv + splits - 1) / splits;
  const int64_t v0 = sp * per, v1 = v0 + per < nv ? v0 + per : nv;
  // refit of a mis-speculated batch (the class_hist_block sequence): this class's codes rebuilt from the scores
  if (speculative && row_stats != nullptr && info_m0 != info_m1) {
    const int m1 = info_m1;
    uint16_t* ccol = const_cast<uint16_t*>(codes) + (int64_t)c * n_pad;
    for (int64_t r = v0 * 8 + threadIdx.x; r < v1 * 8; r += NT) {
      uint32_t code = 0x8000u;
      if (r < n) {
        const float4 st = row_stats[r];
        const uint32_t fl = __float_as_uint(st.z);
        const T xv = preds[r * ld + c];
        if (m1 != 0) {
          if ((fl & 3u) == 3u) {
            const float inv = 1.f / st.y;
            const f32x2 e = exp_nonpos2(f32x2{to_f32<T>(xv) - st.x, 0.f});
            code = pack_rne2<T>(div_rn2(f32x2{e.x, 0.f}, f32x2{st.y, 1.f}, f32x2{inv, 1.f})) & 0xFFFFu;
          }
        } else if (fl & 1u) {
          code = raw_code<T>(bits16<T>(xv));
        }
        if (target[r] == c) {
          if (pos_booked) {
            // the row pass booked this row's positive with the mis-speculated mode's code: take it back, book the
            // refit code, and leave the code skipped for the count below
            const uint32_t booked = __float_as_uint(st.w);
            if (booked & 0x10000u) {
              atomic_add_i64(pos_hist + (booked & 0xFFFFu), -1);
              if (bpos != nullptr) atomic_add_i64(bpos + (booked & 0xFFFFu), -1);
            }
            if (!(code & 0x8000u)) {
              atomic_add_i64(pos_hist + code, 1);
              if (bpos != nullptr) atomic_add_i64(bpos + code, 1);
              lo = min(lo, (int)code);
              hi = max(hi, (int)code);
              code = 0x8000u;
            }
          } else if (!(code & 0x8000u)) {
            code |= 0x4000u;
          }
        }
      }
      ccol[r] = static_cast<uint16_t>(code);
    }
    __threadfence();
    __syncthreads();
  }
  // positives of one vector: int64 bins directly (and the batch bins), range tracked here
  auto book_pos = [&](const uint4& v) {
    const uint32_t parts[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t x = (k & 1) ? (parts[k >> 1] >> 16) : (parts[k >> 1] & 0xFFFFu);
      if ((x & 0xC000u) == 0x4000u) {
        const uint32_t bin = x & 0x3FFFu;
        atomic_add_i64(pos_hist + bin, 1);
        if (bpos != nullptr) atomic_add_i64(bpos + bin, 1);
        lo = min(lo, (int)bin);
        hi = max(hi, (int)bin);
      }
    }
  };
  // Loads run one step ahead (register double buffer of kHiUnroll vectors): the next step's loads are in flight while
  // this step is counted, so a workgroup streams instead of alternating load and count phases.  EXACT: the slice is a
  // whole number of steps (65536-row classes: 4 steps of 4 vectors per thread), no bounds tests.
  constexpr int64_t kStep = (int64_t)kHiUnroll * NT;
  // pos_booked: the row pass booked every positive and left its code skipped -- no per-vector positive test here
  auto stream = [&](auto exact_tag, auto booked_tag) {
    constexpr bool EXACT = decltype(exact_tag)::value;
    constexpr bool BOOKED = decltype(booked_tag)::value;
    auto count_step = [&](const uint4 (&w)[kHiUnroll]) {
#pragma unroll
      for (int u = 0; u < kHiUnroll; ++u) {
        hi_count4<false>(w[u]);
        if constexpr (!BOOKED) {
          const uint32_t anypos = ((w[u].x | w[u].y) | (w[u].z | w[u].w)) & 0x40004000u;
          if (__builtin_expect(__ballot(anypos != 0) != 0, 0) && anypos != 0) book_pos(w[u]);
        }
      }
    };
    auto load = [&](uint4 (&w)[kHiUnroll], int64_t cb) {
#pragma unroll
      for (int u = 0; u < kHiUnroll; ++u) {
        const int64_t v = cb + threadIdx.x + u * NT;
        if constexpr (EXACT) w[u] = col[v];
        else w[u] = v < v1 ? col[v] : make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);
      }
    };
    uint4 a[kHiUnroll], b[kHiUnroll];
    if (v0 >= v1) return;
    load(a, v0);
    for (int64_t cb = v0; cb < v1; cb += 2 * kStep) {
      const bool more1 = cb + kStep < v1, more2 = cb + 2 * kStep < v1;  // block-uniform
      if (more1) load(b, cb + kStep);
      count_step(a);
      if (!more1) break;
      if (more2) load(a, cb + 2 * kStep);
      count_step(b);
    }
  };
  const bool exact = (v1 - v0) % kStep == 0;
  if (pos_booked) {
    if (exact) stream(std::true_type{}, std::true_type{});
    else stream(std::false_type{}, std::true_type{});
  } else {
    if (exact) stream(std::true_type{}, std::false_type{});
    else stream(std::false_type{}, std::false_type{});
  }
  __syncthreads();
  const bool low = s_h[0] != 0u;  // block-uniform
  // rare rows (usually none): before the flushes, which then go by atomics when there are any
  const int m0 = info_m0, m1 = info_m1;
  const bool fixed = speculative && m0 != m1;
  const int64_t n0 = info_n0, n1 = info_n1;
  if (sp == 0) {
    for (int64_t i = threadIdx.x; i < n0 + n1; i += NT) {
      const int lst = i < n0 ? 0 : 1;
      if (lst == 0 && fixed) continue;
      const int64_t r = slow_rows[lst * n + (lst == 0 ? i : i - n0)];
      if ((lst == 1 ? m1 : m0) != 0) continue;
      const uint32_t code = raw_code<T>(bits16<T>(preds[r * ld + c]));
      if (code & 0x8000u) continue;
      lo = min(lo, (int)code);
      hi = max(hi, (int)code);
      if (target[r] == c) atomic_add_i64(pos_hist + code, 1);
      else atomic_add_i64(neg_hist + code, 1);
      if (bneg != nullptr) atomic_add_i64((target[r] == c ? bpos : bneg) + code, 1);
    }
  }
  if (confmat != nullptr && threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    for (int64_t i = vb; i < n0; i += vgrid) {
      const int64_t r = slow_rows[i];
      const int64_t t = target[r];
      if (t < 0 || t >= C) continue;
      const T* row = preds + r * ld;
      float best = -INFINITY;
      int bi = C, first_nan = C;
      for (int cc = lane; cc < C; cc += kWave) {
        const float v = to_f32<T>(row[cc]);
        if (v != v) first_nan = min(first_nan, cc);
        else if (bi == C || v > best) { best = v; bi = cc; }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) first_nan = min(first_nan, __shfl_xor(first_nan, off, kWave));
      wave_argmax(best, bi);
      const int am = first_nan < C ? first_nan : bi;
      if (lane == 0 && am < C) atomic_add_i64(confmat + t * C + am, 1);
    }
  }
  const bool bstore = splits == 1 && n0 + n1 == 0;  // this block is the only writer of its batch bins
  // flush of the upper window: words 1..8190 = bins 8191..16380 (word 0: the low bucket, word 8191: trash)
  for (int w = 1 + threadIdx.x; w < kHiWords - 1; w += NT) {
    const uint32_t cnt = s_h[w];
    if (cnt) {
      const int i = w + kHiBase;
      lo = min(lo, i);
      hi = max(hi, i);
      atomic_add_i64(neg_hist + i, cnt);
      if (bneg != nullptr) {
        if (bstore) bneg[i] = cnt;
        else atomic_add_i64(bneg + i, cnt);
      }
    }
  }
  if (low) {  // codes <= 8190 (probabilities below 2^-63): one more pass over this slice, window [0, 8190]
    __syncthreads();
    for (int i = threadIdx.x; i < kHiWords / 4; i += NT) s4[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (int64_t cb = v0; cb < v1; cb += kStep) {
#pragma unroll
      for (int u = 0; u < kHiUnroll; ++u) {
        const int64_t v = cb + threadIdx.x + u * NT;
        if (v < v1) hi_count4<true>(col[v]);
      }
    }
    __syncthreads();
    for (int w = threadIdx.x; w <= kHiBase; w += NT) {
      const uint32_t cnt = s_h[w];
      if (cnt) {
        lo = min(lo, w);
        hi = max(hi, w);
        atomic_add_i64(neg_hist + w, cnt);
        if (bneg != nullptr) {
          if (bstore) bneg[w] = cnt;
          else atomic_add_i64(bneg + w, cnt);
        }
      }
    }
  }
  if (code_range != nullptr || batch_range != nullptr) {
    lo = wave_min_i32(lo);
    hi = wave_max_i32(hi);
    if ((threadIdx.x & (kWave - 1)) == 0 && hi >= 0) {
      if (code_range != nullptr) {
        atomicMin(code_range + 2 * c, lo);
        atomicMax(code_range + 2 * c + 1, hi);
      }
      if (batch_range != nullptr) {
        atomicMin(batch_range + 2 * c, lo);
        atomicMax(batch_range + 2 * c + 1, hi);
      }
    }
  }
  class_hi_ticket(state, roll_mode, vgrid);
}

// amdgpu_waves_per_eu(8): eight waves per SIMD (four workgroups per CU, all 1000 classes of the headline in one round);
// without it the compiler spent 106 SGPRs and the occupancy fell to 7 waves -- 3 workgroups per CU, a second round for
// the last 232 classes (47 vs 31 us)
template <typename T>
__global__ void __launch_bounds__(kClassThreadsU16) __attribute__((amdgpu_waves_per_eu(8))) class_hist_hi_kernel(const uint16_t* __restrict__ codes, int64_t n_pad, int splits,
                                                                        int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
                                                                        const int64_t* __restrict__ target, int64_t n,
                                                                        const int* __restrict__ bmode, bool speculative,
                                                                        const int* __restrict__ slow_rows, int* __restrict__ state,
                                                                        int64_t* __restrict__ confmat, int* __restrict__ code_range,
                                                                        int* __restrict__ roll_mode, int64_t* __restrict__ batch_hist,
                                                                        int* __restrict__ batch_range, const float4* __restrict__ row_stats = nullptr,
                                                                        bool pos_booked = false) {
  class_hist_hi_block<T, kClassThreadsU16>(blockIdx.x, gridDim.x, codes, n_pad, splits, hist, preds, ld, target, n, bmode, speculative,
                                           slow_rows, state, confmat, code_range, roll_mode, batch_hist, batch_range, row_stats, pos_booked);
}

// Small-class class pass: packed LDS histogram per (class, split), partial flush (class_store_partial).
template <typename T>
__global__ void __launch_bounds__(kClassThreads) class_hist_partial_kernel(
    const uint16_t* __restrict__ codes, int64_t n_pad, int splits, int64_t* __restrict__ hist, const T* __restrict__ preds, int ld,
    const int64_t* __restrict__ target, int64_t n, const int* __restrict__ bmode, bool speculative, const int* __restrict__ slow_rows,
    int* __restrict__ state, int64_t* __restrict__ confmat, int* __restrict__ code_range, int* __restrict__ roll_mode,
    uint32_t* __restrict__ partial, int* __restrict__ prange, const float4* __restrict__ row_stats = nullptr) {
  class_hist_block<T, true, kClassThreads>(blockIdx.x, gridDim.x, codes, n_pad, splits, hist, preds, ld, target, n, bmode, speculative,
                                           slow_rows, state, confmat, code_range, roll_mode, partial, prange, nullptr, nullptr, row_stats);
}

// Sum of the splits' partial packed words per (class, bin) into the int64 histogram: one owner thread per bin, so a
// plain read-modify-write; splits whose range misses the bin are not read.  The extra block column x = kCodes / 256
// does the per-class work the class pass left out: the class's occupied range (min / max over its splits) into
// code_range, the row pass's per-block confusion-matrix partials of row c (pcm [blocks][C][C], C <= 64), and —
// block (x, 0) — the batch's state reset and speculation roll (the class pass has completed: stream order).
__global__ void __launch_bounds__(256) class_partial_reduce_kernel(const uint32_t* __restrict__ partial, const int* __restrict__ prange,
                                                                   int splits, int64_t* __restrict__ hist, int* __restrict__ code_range,
                                                                   int* __restrict__ state, int* __restrict__ roll_mode,
                                                                   const uint32_t* __restrict__ pcm, int pcm_blocks,
                                                                   int64_t* __restrict__ confmat, int C, int pcm_slices,
                                                                   int x_base = 0) {
  const int c = blockIdx.y;
  const int bx = static_cast<int>(blockIdx.x) + x_base;  // x_base = kCodes / 256 + 1: the confusion-matrix blocks only
  if (bx > kCodes / 256) {
    // confusion-matrix row c: slice p of the row pass's per-block partials, 256 / C thread groups stride over the
    // slice's blocks, an LDS fold per cell, one int64 atomic per (slice, cell) — a serial loop over thousands of
    // partials per cell was the reduce launch's cost
    __shared__ uint64_t s_acc[256];
    const int p = bx - (kCodes / 256 + 1);
    const int G = 256 / C, cell = threadIdx.x % C, g = threadIdx.x / C;
    const int per = (pcm_blocks + pcm_slices - 1) / pcm_slices;
    const int b0 = p * per, b1 = min(pcm_blocks, b0 + per);
    uint64_t acc = 0;
    if (g < G)
      for (int b = b0 + g; b < b1; b += G) acc += pcm[((int64_t)b * C + c) * C + cell];
    s_acc[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < C) {
      uint64_t tot = 0;
      for (int q = 0; q < G; ++q) tot += s_acc[q * C + threadIdx.x];
      if (tot) atomic_add_i64(confmat + (int64_t)c * C + threadIdx.x, static_cast<int64_t>(tot));
    }
    return;
  }
  if (bx == kCodes / 256) {
    if (threadIdx.x == 0 && code_range != nullptr) {
      int lo = kCodes, hi = -1;
      for (int s = 0; s < splits; ++s) {
        const int64_t b = (int64_t)c * splits + s;
        lo = min(lo, prange[2 * b]);
        hi = max(hi, prange[2 * b + 1]);
      }
      if (hi >= 0) {
        atomicMin(code_range + 2 * c, lo);
        atomicMax(code_range + 2 * c + 1, hi);
      }
    }
    if (c == 0 && threadIdx.x == 0) {
      state[0] = state[1] = 0;
      state[2] = 0;
      if (roll_mode != nullptr) {
        const int m1 = roll_mode[1];
        roll_mode[0] = m1;
        roll_mode[1] = 0;
      }
    }
    return;
  }
  const int i = bx * 256 + threadIdx.x;
  uint64_t neg = 0, pos = 0;
  const int64_t b0 = (int64_t)c * splits;
  int s = 0;
  for (; s + 8 <= splits; s += 8) {  // 8 splits' words requested before any is summed (one latency, not 8)
    uint32_t w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t b = b0 + s + u;
      w[u] = (i >= prange[2 * b] && i <= prange[2 * b + 1]) ? partial[b * kCodes + i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      neg += w[u] & 0xFFFFu;
      pos += w[u] >> 16;
    }
  }
  for (; s < splits; ++s) {
    const int64_t b = b0 + s;
    if (i >= prange[2 * b] && i <= prange[2 * b + 1]) {
      const uint32_t w = partial[b * kCodes + i];
      neg += w & 0xFFFFu;
      pos += w >> 16;
    }
  }
  // one owner per bin; non-returning atomics instead of a read-modify-write that waits on a global load
  if (neg) atomic_add_i64(hist + (int64_t)c * 2 * kCodes + i, static_cast<int64_t>(neg));
  if (pos) atomic_add_i64(hist + ((int64_t)c * 2 + 1) * kCodes + i, static_cast<int64_t>(pos));
}

// Speculation roll, one thread, in row-pass stream order right after the FIXUP launch (standalone row pass only; the
// update route rolls in the class pass's last workgroup instead, one launch fewer): the batch's (used, real) mode pair
// is snapshotted into ``bmode`` = state[3:5] and the next batch speculates the real one.
__global__ void mode_roll_kernel(int* __restrict__ mode, int* __restrict__ bmode) {
  const int m0 = mode[0], m1 = mode[1];
  bmode[0] = m0;
  bmode[1] = m1;
  mode[0] = m1;
  mode[1] = 0;
}


// ---- small-class row pass (C <= 256): see classification.hip launch_small_two_pass
constexpr int kSmallRows = 64;
constexpr int kSmallVpt = 16;
constexpr int kSmallCmMax = 64;  // LDS-privatised confusion matrix up to 64 x 64 (16 KiB)

// Reductions over aligned groups of TL lanes (TL <= 16) by DPP (quad_perm xor 1, xor 2, row_half_mirror, row_mirror:
// after the first two steps a quad is uniform, so the mirrors pair exactly as xor 4 / xor 8 would -- the same values,
// the same fp32 additions as an xor butterfly) -- no LDS round trip and no per-offset address register, which the
// __shfl_xor form (ds_bpermute) hoisted out of the tile loop: ~20 VGPRs of the small row pass's 126.
template <int TL> __device__ __forceinline__ float grp_max(float v) {
  if constexpr (TL > 1) v = __builtin_fmaxf(v, dpp_f32<0xB1>(v, v));
  if constexpr (TL > 2) v = __builtin_fmaxf(v, dpp_f32<0x4E>(v, v));
  if constexpr (TL > 4) v = __builtin_fmaxf(v, dpp_f32<0x141>(v, v));
  if constexpr (TL > 8) v = __builtin_fmaxf(v, dpp_f32<0x140>(v, v));
  return v;
}
template <int TL> __device__ __forceinline__ float grp_min(float v) {
  if constexpr (TL > 1) v = __builtin_fminf(v, dpp_f32<0xB1>(v, v));
  if constexpr (TL > 2) v = __builtin_fminf(v, dpp_f32<0x4E>(v, v));
  if constexpr (TL > 4) v = __builtin_fminf(v, dpp_f32<0x141>(v, v));
  if constexpr (TL > 8) v = __builtin_fminf(v, dpp_f32<0x140>(v, v));
  return v;
}
template <int TL> __device__ __forceinline__ float grp_sum(float v) {
  if constexpr (TL > 1) v += dpp_f32<0xB1>(v, v);
  if constexpr (TL > 2) v += dpp_f32<0x4E>(v, v);
  if constexpr (TL > 4) v += dpp_f32<0x141>(v, v);
  if constexpr (TL > 8) v += dpp_f32<0x140>(v, v);
  return v;
}
template <int TL> __device__ __forceinline__ int grp_min_i32(int v) {
  if constexpr (TL > 1) v = min(v, dpp_i32<0xB1>(v, v));
  if constexpr (TL > 2) v = min(v, dpp_i32<0x4E>(v, v));
  if constexpr (TL > 4) v = min(v, dpp_i32<0x141>(v, v));
  if constexpr (TL > 8) v = min(v, dpp_i32<0x140>(v, v));
  return v;
}
// value of lane ^ M (M < 32): ds_swizzle in bitmask mode (and 0x1F, xor M), no address register
template <int M> __device__ __forceinline__ uint32_t swz_xor(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), 0x1F | (M << 10)));
}

// CC > 0: the class count as a compile-time constant (C <= 16, one lane per row): the per-lane loops lose their
// runtime class masks (at C = 10 the generic form ran 6 of 16 slots masked, 82 VGPRs and 69 SGPR spills).
// DIRECT (C % 8 == 0, 16-B aligned scores): every lane loads its 16 scores straight into registers (two 16-B loads;
// a row's lanes and consecutive rows are contiguous, so a wave reads one contiguous run) -- no LDS staging.
// Otherwise the block's scores are staged into LDS with 16-B loads and each lane reads its 16 from there.
// Image (round 5): the codes of row pair (2k, 2k+1) and class c are packed into one dword (the lane of the even row
// swaps halves with its partner lane of the odd row: the even lane then holds the even classes of both rows, the odd
// lane the odd classes) at dword c * 32 + ((k + rot(c)) & 31), rot(c) = (c >> 4) * (32 / TL): for one store
// instruction the 64 lanes' (class parity, rotated pair slot) are 64 distinct banks.  The round-4 image took one
// 16-bit write per code at c * 64 + row -- a TL-way bank conflict per store (all lanes of a row 2 KiB apart) on top
// of the two-lanes-per-dword one: the row pass of C = 256 x 262,144 ran 171 us against 59 us for C = 1000 x 65,536.
#ifndef TMX_SMALL_WPE
#define TMX_SMALL_WPE 0
#endif
#if TMX_SMALL_WPE > 0
#define TMX_SMALL_WPE_ATTR __attribute__((amdgpu_waves_per_eu(TMX_SMALL_WPE)))
#else
#define TMX_SMALL_WPE_ATTR
#endif
template <typename T, int TL, bool FIXUP, int CC = 0, bool DIRECT = false>
__global__ void __launch_bounds__(kSmallRows * TL) TMX_SMALL_WPE_ATTR mc_codes_small_kernel(
    const T* __restrict__ preds, const int64_t* __restrict__ target, int64_t n, int C_arg, int* __restrict__ mode, int64_t ignore_index,
    bool has_ignore, uint16_t* __restrict__ codes, int64_t n_pad, int64_t* __restrict__ confmat, int* __restrict__ err,
    bool record_mode, int* __restrict__ slow_rows, int* __restrict__ slow_count, uint32_t* __restrict__ pcm,
    float4* __restrict__ row_stats = nullptr) {
  const int C = CC > 0 ? CC : C_arg;
  constexpr int kVpt = CC > 0 ? CC : kSmallVpt;  // value slots per lane
  constexpr int kPairs = (kVpt + 1) / 2;
  constexpr int kRot = 32 / TL;
  static_assert(!DIRECT || kVpt == kSmallVpt, "direct loads take 16 scores per lane");
  extern __shared__ __attribute__((aligned(16))) uint16_t s_small[];  // staging [64][C] / image [C][32 dwords]; cm [C][C]
  uint32_t* s_img = reinterpret_cast<uint32_t*>(s_small);
  int use_mode;
  if constexpr (FIXUP) {
    const int m0 = mode[0], m1 = mode[1];
    if (m0 == m1) return;
    use_mode = m1;
  } else {
    use_mode = mode[0];
  }
  // C <= 64: the confusion matrix is privatised in LDS (at C = 2 every row's atomic hit one of 4 global words)
  uint32_t* s_cm = reinterpret_cast<uint32_t*>(s_small + kSmallRows * ((C + 1) & ~1));
  const bool lds_cm = !FIXUP && confmat != nullptr && C <= kSmallCmMax;
  if (lds_cm)
    for (int i = threadIdx.x; i < C * C; i += kSmallRows * TL) s_cm[i] = 0u;
  const int64_t ntiles = n_pad / kSmallRows;
  bool bad = false;
  // DIRECT: the next tile's scores (and targets) are loaded into registers before this tile is processed, and the
  // tile's barriers wait for LDS only (s_waitcnt lgkmcnt(0); s_barrier): __syncthreads() also drains vmcnt, which
  // would wait for the prefetch.  The image is the only block-shared state, so the LDS-only barrier is sufficient.
  auto lds_barrier = [&]() {
    if constexpr (DIRECT) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else __syncthreads();
  };
  uint4 nxt[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
  int64_t nxt_t = -1;
  auto prefetch = [&](int64_t tl_) {
    const int lid = static_cast<int>(threadIdx.x);
    const int q_ = lid % TL, lr_ = lid / TL, cb_ = q_ * kVpt;
    const int64_t rr = tl_ * kSmallRows + lr_;
    const bool inr = tl_ < ntiles && rr < n;
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(preds) + rr * C + cb_);
    nxt[0] = make_uint4(0u, 0u, 0u, 0u);
    nxt[1] = make_uint4(0u, 0u, 0u, 0u);
    if (inr && cb_ < C) nxt[0] = stream_load16(src);
    if (inr && cb_ + 8 < C) nxt[1] = stream_load16(src + 1);
    nxt_t = inr ? target[rr] : -1;
  };
  if constexpr (DIRECT) prefetch(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  // lane -> (row, class chunk), opaque per tile: loop-invariant per-slot class indices, slot masks and image addresses
  // hoisted out of the tile loop held ~40 VGPRs and ~30 SGPR spills (the loop body needs ~60 registers)
  int lane_id = static_cast<int>(threadIdx.x);
  asm volatile("" : "+v"(lane_id));
  const int q = lane_id % TL, lr = lane_id / TL;  // lane within the row, row within the block
  const int cb = q * kVpt;
  lds_barrier();  // previous tile's class segments were read from the image
  const int64_t r0 = tile * kSmallRows;
  const int rows = static_cast<int>(min<int64_t>(kSmallRows, n - r0));
  const int64_t r = r0 + lr;
  const bool in_rows = lr < rows;
  // the lane's slots as packed fp32 pairs (2p, 2p + 1); slots past the class count (and rows past n) hold -inf
  f32x2 P[kPairs];
  int64_t t_pref = -1;
  if constexpr (DIRECT) {
    const uint4 w[2] = {nxt[0], nxt[1]};
    t_pref = nxt_t;
    prefetch(tile + gridDim.x);  // in flight while this tile is processed
    const bool ok0 = in_rows && cb < C, ok1 = in_rows && cb + 8 < C;
    float u[16];
    unpack8<T>(w[0], u);
    unpack8<T>(w[1], u + 8);
#pragma unroll
    for (int p = 0; p < kPairs; ++p)
      P[p] = f32x2{(p < 4 ? ok0 : ok1) ? u[2 * p] : -INFINITY, (p < 4 ? ok0 : ok1) ? u[2 * p + 1] : -INFINITY};
  } else {
    // 1. stage the block's scores (byte range [r0 C, (r0 + rows) C) x 2; r0 C x 2 is a multiple of 128 B)
    {
      const int64_t nelem = (int64_t)rows * C;
      const uint16_t* src = reinterpret_cast<const uint16_t*>(preds) + r0 * C;
      const int nvec = static_cast<int>(nelem / 8);
      for (int i = threadIdx.x; i < nvec; i += kSmallRows * TL)
        reinterpret_cast<uint4*>(s_small)[i] = reinterpret_cast<const uint4*>(src)[i];
      for (int i = nvec * 8 + threadIdx.x; i < nelem; i += kSmallRows * TL) s_small[i] = src[i];
    }
    __syncthreads();
    auto at = [&](int j) -> float {
      const int c = cb + j;
      return (j < kVpt && in_rows && c < C) ? to_f32<T>(*reinterpret_cast<const T*>(&s_small[lr * C + c])) : -INFINITY;
    };
#pragma unroll
    for (int p = 0; p < kPairs; ++p) P[p] = f32x2{at(2 * p), at(2 * p + 1)};
  }
  const int64_t t = DIRECT ? t_pref : (in_rows ? target[r] : -1);
  const bool valid = in_rows && !(has_ignore && t == ignore_index);
  // row statistics over the TL lanes of the row (xor shuffles stay inside aligned groups of TL lanes)
  // (masked slots are -inf: neutral for the maximum; excluded from the minimum and the sum).  Slots past the class
  // count exist only in the last lanes of a row when C % 16 != 0 (wave-uniform): otherwise the trees run unmasked.
  const bool masked = (CC > 0 ? (kVpt & 1) != 0 : C % kSmallVpt != 0);
  auto slot = [&](int j) -> float { return (j & 1) ? P[j >> 1].y : P[j >> 1].x; };
  float mx, mn;
  if (!masked) {
    float a[kVpt], b[kVpt];
#pragma unroll
    for (int j = 0; j < kVpt; ++j) a[j] = b[j] = slot(j);
#pragma unroll
    for (int w = 1; w < kVpt; w *= 2)  // balanced trees (v_max3 / v_min3 after the compiler's folding)
#pragma unroll
      for (int j = 0; j + w < kVpt; j += 2 * w) {
        a[j] = __builtin_fmaxf(a[j], a[j + w]);
        b[j] = __builtin_fminf(b[j], b[j + w]);
      }
    mx = a[0];
    mn = b[0];
  } else {
    mx = -INFINITY;
    mn = INFINITY;
#pragma unroll
    for (int j = 0; j < kVpt; ++j) {
      mx = __builtin_fmaxf(mx, slot(j));
      if (cb + j < C) mn = __builtin_fminf(mn, slot(j));
    }
  }
  mx = grp_max<TL>(mx);
  mn = grp_min<TL>(mn);
  bool fin = __builtin_isfinite(mx);
  // arg-max of a finite row (the first class holding the maximum): only for the fused confusion matrix
  int am = C;
  if (!FIXUP && confmat != nullptr) {
#pragma unroll
    for (int j = kVpt - 1; j >= 0; --j)
      if (cb + j < C && slot(j) == mx) am = cb + j;
    am = grp_min_i32<TL>(am);
  }
  // exp / quotient / rounding on the packed pairs (round 5): v_pk_* and v_cvt_pk_bf16_f32 -- per component exactly
  // the scalar sequences (exp_nonpos, div_rn, RNE), bit for bit
  float s = 0.f, inv = 0.f;
  // exp(x - max) of the slots and their row sum; the exps replace the scores in P only in softmax mode (probability
  // mode keeps the scores: they are the codes, the sum only feeds the class pass's refit statistics)
  // round 6: the row sum of the fast exps (csrc/curve_hist_kernels.h fast_code2); the scores stay in P
  const f32x2 m2 = {mx, mx};
  // every valid element of every row of the wave within 86 of its maximum: verified fast quotients (bf16)
  const bool narrow = __ballot(!(mx - mn <= 86.f)) == 0;
  auto exp_sum = [&]() -> float {
    f32x2 acc = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
      f32x2 e = exp_fast2(P[p] - m2);
      if (masked) {
        e.x = cb + 2 * p < C ? e.x : 0.f;
        e.y = cb + 2 * p + 1 < C ? e.y : 0.f;
      }
      acc = acc + e;
    }
    return grp_sum<TL>(acc.x + acc.y);
  };
  // softmax statistics: the codes in softmax mode, the class pass's refit of a mispredicted batch otherwise
  if (use_mode != 0 || row_stats != nullptr) s = exp_sum();
  if (use_mode != 0) {
    inv = 1.f / s;
    fin = fin && s == s;
  } else {
    float sum = 0.f;  // probability mode: a row is counted when its scores' sum is finite (no NaN / inf)
#pragma unroll
    for (int j = 0; j < kVpt; ++j)
      if (cb + j < C) sum += slot(j);
    fin = fin && __builtin_isfinite(grp_sum<TL>(sum));
  }
  if (row_stats != nullptr && q == 0 && in_rows && !FIXUP)
    row_stats[r] = make_float4(mx, s, __uint_as_float((valid ? 1u : 0u) | (__builtin_isfinite(mx) && s == s ? 2u : 0u)), 0.f);
  const bool slow = valid && !fin;
  const bool keep = valid && fin;
  // 3. codes into the image (the staging area is free once every lane holds its values): pack class pairs, swap
  //    halves with the partner row's lane, one dword per (class, row pair)
  uint32_t word[kPairs];
  // softmax codes (quotients in [0, 1] are their own codes, never skipped): the positive's bit 14 is set after the
  // image is written, by one LDS OR per row (below) instead of a compare + select per slot pair
  // (one lane per row -- TL == 1 -- keeps the per-pair select: 64 LDS ORs per wave cost more than its few pairs)
  const bool or_positive = TL > 1 && keep && use_mode != 0;
  if (keep && use_mode != 0) {
    const f32x2 s2 = {s, s}, i2 = {inv, inv};
    const int tl = static_cast<int>(t) - cb;  // the positive's slot in this lane (any value when t is not here)
    const uint32_t tflag = TL > 1 ? 0u : 0x4000u << (16 * (tl & 1));
    const bool fast = FastQuot<T>::value && narrow;
    const float eps = fast_eps(mx, mn);  // (the row minimum bounds this lane's elements too)
    const f32x2 rlo = {inv - inv * eps, inv - inv * eps}, rhi = {inv + inv * eps, inv + inv * eps};
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
      if (fast) {
        bool und;
        word[p] = fast_code2<T>(exp_fast2(P[p] - m2), rlo, rhi, und);
        if (__ballot(und) != 0) word[p] = exact_code2<T>(P[p], m2, s2, i2, true);
      } else {
        word[p] = exact_code2<T>(P[p], m2, s2, i2, false);
      }
      if constexpr (TL == 1) word[p] |= ((tl >> 1) == p && tl >= 0 ? tflag : 0u);
    }
  } else {
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
      uint32_t cw[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int j = 2 * p + e;
        const int c = cb + j;
        uint32_t code = 0x8000u;  // padding rows / absent classes: skipped
        if (j < kVpt && keep && c < C) {
          code = raw_code<T>(half_bits<T>(e ? P[p].y : P[p].x));
          if (c == t && !(code & 0x8000u)) code |= 0x4000u;
        }
        cw[e] = code;
      }
      word[p] = cw[0] | (cw[1] << 16);
    }
  }
  const bool odd_row = (lr & 1) != 0;
  const int k = lr >> 1;
  if constexpr (!DIRECT) __syncthreads();  // every lane has read its scores from the staging area (the image's space)
  // this lane's image dwords: class cb + 2p + odd at dword (cb + 2p + odd) * 32 + ((k + q * kRot) & 31) -- one base
  // address, the pairs at immediate offsets of 64 dwords
  uint32_t* img = s_img + (cb + (odd_row ? 1 : 0)) * 32 + ((k + q * kRot) & 31);
#pragma unroll
  for (int p = 0; p < kPairs; ++p) {
    const uint32_t other = swz_xor<TL>(word[p]);  // the partner row's (even, odd) class pair
    // even row lane: class cb + 2p of rows (2k, 2k+1); odd row lane: class cb + 2p + 1 of rows (2k, 2k+1)
    const uint32_t packed = odd_row ? ((other >> 16) | (word[p] & 0xFFFF0000u)) : ((word[p] & 0xFFFFu) | (other << 16));
    if (2 * p + (odd_row ? 1 : 0) < kVpt && cb + 2 * p + (odd_row ? 1 : 0) < C) img[64 * p] = packed;
  }
  // the positive of a softmax row: bit 14 of its half of dword (t, k), after that dword's write (same wave: LDS
  // operations of one wave complete in order)
  if (q == 0 && or_positive && t >= 0 && t < C)
    atomicOr(&s_img[static_cast<int>(t) * 32 + ((k + static_cast<int>(t >> 4) * kRot) & 31)], 0x4000u << (16 * (lr & 1)));
  if (q == 0 && in_rows) {
    if constexpr (!FIXUP) {
      if (confmat != nullptr && keep && t >= 0 && t < C && am < C) {
        if (lds_cm) atomicAdd(s_cm + t * C + am, 1u);
        else atomic_add_i64(confmat + t * C + am, 1);
      }
      if (err != nullptr && valid && (t < 0 || t >= C)) atomicOr(err, 1);
    }
    if (slow) {
      const int list = FIXUP ? 1 : 0;
      slow_rows[list * n + atomicAdd(slow_count + list, 1)] = static_cast<int>(r);
    }
  }
  if (!FIXUP && record_mode && q == 0) bad = bad || slow || (valid && (mx > 1.f || mn < 0.f));
  lds_barrier();
  // class segments: C rows of 64 codes = 8 x 16 B each (4 rotated dwords = two 8-B LDS reads: rot(c) is even)
  for (int i = threadIdx.x; i < C * 8; i += kSmallRows * TL) {
    const int c = i >> 3, m = i & 7;
    const int base = c * 32, rot = (4 * m + (c >> 4) * kRot) & 31;
    const uint2 a = *reinterpret_cast<const uint2*>(s_img + base + rot);
    const uint2 b = *reinterpret_cast<const uint2*>(s_img + base + ((rot + 2) & 31));
    reinterpret_cast<uint4*>(codes + (int64_t)c * n_pad + r0)[m] = make_uint4(a.x, a.y, b.x, b.y);
  }
  }  // tiles
  if (lds_cm) {  // per-block partial (summed by class_partial_reduce_kernel), else atomics on the few cells
    __syncthreads();
    if (pcm != nullptr)
      for (int i = threadIdx.x; i < C * C; i += kSmallRows * TL) pcm[(int64_t)blockIdx.x * C * C + i] = s_cm[i];
    else
      for (int i = threadIdx.x; i < C * C; i += kSmallRows * TL)
        if (s_cm[i]) atomic_add_i64(confmat + i, s_cm[i]);
  }
  if constexpr (!FIXUP) {
    if (record_mode && __syncthreads_or(bad) && threadIdx.x == 0 &&
        __hip_atomic_load(mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
      __hip_atomic_store(mode + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


}  // namespace tmx
