// v2 row pass (the previous library kernel), kept only as the reference the standalone harness checks the current
// row pass against.  Not compiled into the library.
#pragma once
#include "curve_hist_kernels.h"

namespace tmx_ref {
using namespace tmx;
// ---------------------------------------------------------------------------------------------------------
// Two-pass multiclass histogram (C % 8 == 0, C <= 1024):
//   (A) row pass  — one wave per row pair: 16-B vector loads, fp32 softmax (if flagged) rounded to the input
//       dtype, argmax (fused confusion matrix), 16-bit code per element with flag bits
//       (bit 14 = positive label, bit 15 = skip).  Codes of a 64-row tile are transposed to class-major
//       through an LDS tile [C][32 dwords] (two rows packed per dword), XOR-swizzled by class group so both
//       the scattered writes and the row read-out are bank-conflict free, then stored as 128-B segments of
//       a class-major scratch codes[C][n_pad].
//   (B) class pass — one workgroup per (class, row split): negatives counted in an LDS-privatised u32
//       histogram (64 KiB, two workgroups per CU), positives (1/C of the data) straight to global; one
//       int64 atomic per non-empty bin on flush (consecutive codes -> contiguous atomics).
// Replaces 1 scattered 64-bit global atomic per score (2.8 ms/update at 65536x1000 on MI355X).
// ---------------------------------------------------------------------------------------------------------
constexpr int kTileRows = 32;  // v2 tile   // 16 packed dwords per class -> 64 KiB LDS at C=1024, 2 WGs/CU
constexpr int kA_Threads = 512;


// bf16 -> fp32 through the type conversion (not a bit shift): the compiler then knows the values are canonical and
// emits plain v_max / v_max3 instead of a canonicalising v_max x, x per element.
template <typename T> __device__ __forceinline__ uint16_t raw_bits(const uint4& w, int e) {
  const uint32_t p[4] = {w.x, w.y, w.z, w.w};
  return (e & 1) ? (p[e >> 1] >> 16) : (p[e >> 1] & 0xFFFF);
}

// Ablation switches (standalone harness only; the library instantiates ABL = 0).
constexpr int kAblNoStore = 1;    // skip the class-major scratch store
constexpr int kAblNoNorm = 2;     // skip exp/div (raw codes)
constexpr int kAblNoLds = 4;      // skip the LDS transpose

// Normalisation mode (sigmoid/softmax-if-any-value-outside-[0,1]) is *speculated*: ``mode[0]`` holds the mode
// used by this launch (the previous batch's verdict, or the range_flag pre-pass result), the kernel records the
// real verdict for this batch in ``mode[1]`` (plain store of 1 by any block that saw a witness; only
// non-ignored rows count, as in the reference).  A FIXUP launch of the same kernel exits immediately unless
// mode[0] != mode[1], in which case it recomputes the codes with the real mode (confusion matrix and error
// flags are mode independent and are not touched again).  ``class_hist_kernel`` then rolls the prediction
// forward (mode[0] = mode[1], mode[1] = 0).  Net effect: no separate 131-MB range pass per update.
// RNE fp32 -> 16-bit pattern without NaN special-casing (NaN / out-of-range patterns are rejected by score_code).
template <typename T> __device__ __forceinline__ uint32_t rne16(float f);
template <> __device__ __forceinline__ uint32_t rne16<__hip_bfloat16>(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
template <> __device__ __forceinline__ uint32_t rne16<__half>(float f) { return round_bits16<__half>(f); }

// softmax output code: RNE16(e * (1/s)).  The reciprocal form differs from an IEEE ``e / s`` by <= 1 fp32 ulp,
// i.e. it moves a value across a 16-bit rounding boundary with probability ~2^-16 — the same order as the
// summation-order differences every softmax implementation already has (tests bound the flip rate).
template <typename T> __device__ __forceinline__ uint32_t quot_code(float e, float rinv) { return rne16<T>(e * rinv); }

// LDS tile [C][kSlots] dwords, 2 rows per dword (u16 halves), slot XOR-swizzled by the class group q so the
// per-lane scattered writes are (2-way at most) conflict free and the row read-out is conflict free.
template <int ABL>
__device__ __forceinline__ void lds_put(uint16_t* s_tile16, int c, int C, int q, int p, int h, uint32_t code,
                                       int kSlots = kTileRows / 2) {
  if constexpr (!(ABL & kAblNoLds)) {
    if (c < C) s_tile16[2 * (c * kSlots + (p ^ (q & (kSlots - 1)))) + h] = static_cast<uint16_t>(code);
  } else {
    if (code == 0x1234u) s_tile16[threadIdx.x] = 0;  // keep the computation alive
  }
}

// One row of up to 1024 classes lives in 2 x 16 B per lane: element j of lane -> class 8 * (lane + 64 * (j>>3)) + (j&7).
template <typename T, int ABL>
__device__ __forceinline__ void codes_for_row(const uint4 (&w)[2], int64_t t, bool valid, int C, int nvec, int lane,
                                              bool do_softmax, bool fixup, int64_t* __restrict__ confmat,
                                              int* __restrict__ err, bool& saw_bad, bool record_mode, int h, int p,
                                              uint16_t* __restrict__ s_tile16, int slots = kTileRows / 2) {
  float v[16];
  bool has_nan = false;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = lane + kWave * k;
    const bool ok = valid && q < nvec;
    float tmp[8];
    unpack8<T>(w[k], tmp);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[8 * k + e] = ok ? tmp[e] : -INFINITY;
      has_nan |= ok && (tmp[e] != tmp[e]);
      if (!fixup && record_mode && ok) saw_bad |= bad16<T>(raw_bits<T>(w[k], e));
    }
  }
  float mx = -INFINITY;
  if (!fixup || do_softmax) {
    // lane-local arg-max in increasing class order (strict > keeps the first maximum)
    float m = v[0];
    int am = 8 * lane;
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      const int c = 8 * (lane + kWave * (j >> 3)) + (j & 7);
      if (v[j] > m) { m = v[j]; am = c; }
    }
    if (m == -INFINITY) am = C;  // nothing valid in this lane (or all -inf): never wins a tie
    mx = m;
    int amx = am;
    wave_argmax(mx, amx);
    if (__ballot(has_nan)) {  // rare: torch.argmax returns the first NaN
      int first = C;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int c = 8 * (lane + kWave * (j >> 3)) + (j & 7);
        if (v[j] != v[j] && c < first) first = c;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off, kWave));
      amx = first;
    }
    if (!fixup && valid && confmat != nullptr && lane == 0 && t >= 0 && t < C && amx < C) atomic_add_i64(confmat + t * C + amx, 1);
    if (!fixup && valid && (t < 0 || t >= C) && err != nullptr && lane == 0) atomicOr(err, 1);
  }
  if (do_softmax && !(ABL & kAblNoNorm)) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      v[j] = expf(v[j] - mx);  // -inf (padding) -> 0
      acc += v[j];
    }
    const float s = wave_sum(acc);
    const float rinv = 1.f / s;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = 8 * (lane + kWave * (j >> 3)) + (j & 7);
      uint32_t code = 0x8000u;
      if (valid && c < C) {
        const int sc = score_code<T>(static_cast<uint16_t>(quot_code<T>(v[j], rinv)));
        code = sc < 0 ? 0x8000u : (uint32_t)sc | (c == t ? 0x4000u : 0u);
      }
      lds_put<ABL>(s_tile16, c, C, lane + kWave * (j >> 3), p, h, code, slots);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = 8 * (lane + kWave * (j >> 3)) + (j & 7);
      uint32_t code = 0x8000u;
      if (valid && c < C) {
        const int sc = score_code<T>(raw_bits<T>(w[j >> 3], j & 7));
        code = sc < 0 ? 0x8000u : (uint32_t)sc | (c == t ? 0x4000u : 0u);
      }
      lds_put<ABL>(s_tile16, c, C, lane + kWave * (j >> 3), p, h, code, slots);
    }
  }
}

// Persistent, software-pipelined row pass.  Each wave walks its row pairs (2 per 32-row tile) and always has the
// NEXT pair's 2 x 2 x 16 B loads in flight while it computes the current pair.
template <typename T, bool FIXUP, int ABL = 0>
__global__ void __launch_bounds__(kA_Threads, 4) mc_codes_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target,
                                                                  int64_t n, int C, int* __restrict__ mode,
                                                                  int64_t ignore_index, bool has_ignore,
                                                                  uint32_t* __restrict__ codes, int64_t n_pad,
                                                                  int64_t* __restrict__ confmat, int* __restrict__ err,
                                                                  bool record_mode) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[];  // [C][kTileRows / 2]
  constexpr int kSlots = kTileRows / 2;
  constexpr int kWavesPerBlock = kA_Threads / kWave;
  constexpr int kPairsPerWave = kSlots / kWavesPerBlock;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  int use_mode;
  if constexpr (FIXUP) {
    const int m0 = __hip_atomic_load(mode, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int m1 = __hip_atomic_load(mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (m0 == m1) return;  // speculation was right (the common case): nothing to redo
    use_mode = m1;
  } else {
    use_mode = mode[0];
  }
  const bool do_softmax = use_mode != 0;
  bool saw_bad = false;
  const int nvec = C / 8;
  const int64_t ntiles = (n + kTileRows - 1) / kTileRows;

  // row sequence of this wave inside a tile: local rows {2w, 2w+1, 2w+16, 2w+17, ...} (pairs w, w+8)
  auto local_row = [&](int i) { return 2 * (wave + (i >> 1) * kWavesPerBlock) + (i & 1); };
  constexpr int kRowsPerWave = 2 * kPairsPerWave;
  auto load_row = [&](int64_t tl, int lr, uint4 (&w)[2], int64_t& tv) {
    const int64_t r = tl * kTileRows + lr;
    const bool in = tl < ntiles && r < n;
    tv = in ? target[r] : INT64_MIN;
    const uint4* row = reinterpret_cast<const uint4*>(preds + (in ? r : 0) * C);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = lane + kWave * k;
      w[k] = (in && q < nvec) ? row[q] : make_uint4(0, 0, 0, 0);
    }
  };

  uint4 wcur[2], wnext[2];
  int64_t tcur, tnext;
  int64_t tile = blockIdx.x;
  load_row(tile, local_row(0), wcur, tcur);
  for (; tile < ntiles; tile += gridDim.x) {
#pragma unroll 1
    for (int i = 0; i < kRowsPerWave; ++i) {
      // keep the next row's loads in flight while this row is computed
      if (i + 1 < kRowsPerWave) load_row(tile, local_row(i + 1), wnext, tnext);
      else load_row(tile + gridDim.x, local_row(0), wnext, tnext);
      const bool valid = tcur != INT64_MIN && !(has_ignore && tcur == ignore_index);
      codes_for_row<T, ABL>(wcur, tcur, valid, C, nvec, lane, do_softmax, FIXUP, confmat, err, saw_bad, record_mode,
                            i & 1, wave + (i >> 1) * kWavesPerBlock, reinterpret_cast<uint16_t*>(s_tile));
      tcur = tnext;
      wcur[0] = wnext[0];
      wcur[1] = wnext[1];
    }
    __syncthreads();
    if constexpr (!(ABL & kAblNoStore)) {
      const int64_t seg = tile * (kTileRows / 2);  // dword offset of this tile inside a class row
      const int64_t row_dw = n_pad / 2;
      for (int idx = threadIdx.x; idx < C * kSlots; idx += kA_Threads) {
        const int c = idx / kSlots, d = idx % kSlots;
        const uint32_t wv = s_tile[idx];
        const int p = d ^ ((c >> 3) & (kSlots - 1));
        codes[c * row_dw + seg + p] = wv;
      }
    }
    __syncthreads();
  }
  if constexpr (!FIXUP) {
    if (record_mode && __syncthreads_or(saw_bad) && threadIdx.x == 0 &&
        __hip_atomic_load(mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
      __hip_atomic_store(mode + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


}  // namespace tmx_ref
