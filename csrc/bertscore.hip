// BERTScore greedy matching on matrix cores.
//
// For every sentence pair b:  S_b = P_b · R_bᵀ  (cosine similarities of L2-normalised token embeddings) and the
// metric needs only   rowmax[b, i] = max_j S_b[i, j]   and   colmax[b, j] = max_i S_b[i, j].
// The reference materialises the whole [B, Lp, Lr] similarity tensor (and moves embeddings to the CPU).  Here a
// 256-thread block computes one 64 × 64 tile of S_b with MFMA (4 waves × 2 × 2 tiles of 16 × 16), never writes it,
// and folds it straight into the row / column maxima with 16-lane shuffles + one order-preserving integer
// atomicMax per row / column and tile.
//   * bf16 / fp16 embeddings: v_mfma_f32_16x16x32_{bf16,f16} (K = 32 per instruction, fp32 accumulation);
//   * fp32 embeddings:        v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).
// A and B fragments are both "8 (or 1) consecutive k of one row", i.e. 16-byte loads straight from the row-major
// [tokens, D] embeddings (Rᵀ needs no transpose); tiles are re-read from L2 by neighbouring blocks.
// Grid: (Lr / 64, Lp / 64, B) — tens of thousands of blocks for the BASELINE shape (B = 1024, L = 512).
#include "common.h"

#include <cstdlib>

namespace tmx {

constexpr int kBsTile = 64;
constexpr int kBsThreads = 256;

using bs_frag8 = __attribute__((ext_vector_type(8))) short;
using bs_acc4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ int ordered_bits(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}

__device__ __forceinline__ float from_ordered(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

template <typename T>
__device__ __forceinline__ bs_frag8 load8(const T* base, int64_t row, int64_t rows, int64_t D, int64_t k) {
  // 8 consecutive 16-bit values of row `row` starting at k (zero outside the matrix)
  bs_frag8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row < rows) {
    const T* p = base + row * D + k;
    if ((D & 7) == 0 && k + 8 <= D) {
      v = *reinterpret_cast<const bs_frag8*>(p);
    } else {
      for (int j = 0; j < 8; ++j)
        if (k + j < D) v[j] = *reinterpret_cast<const short*>(p + j);
    }
  }
  return v;
}

using bs_acc16 = __attribute__((ext_vector_type(16))) float;

template <typename T>
__device__ __forceinline__ bs_acc16 mfma32(bs_frag8 a, bs_frag8 b, bs_acc16 c) {
  if constexpr (std::is_same<T, __hip_bfloat16>::value) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_f16(reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(a),
                                                      reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(b), c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ bs_acc4 mfma16(bs_frag8 a, bs_frag8 b, bs_acc4 c) {
  if constexpr (std::is_same<T, __hip_bfloat16>::value) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(a),
                                                      reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(b), c, 0, 0, 0);
}

// Epilogue shared by both paths: acc[mi][ni] is the 16x16 tile at (row0 + 16 mi, col0 + 16 ni) with
// C mapping col = lane & 15, row = (lane >> 4) * 4 + reg.
__device__ __forceinline__ void fold_maxima(const bs_acc4 (&acc)[2][2], int64_t row0, int64_t col0, int64_t Lp, int64_t Lr,
                                            int* __restrict__ rowmax, int* __restrict__ colmax) {
  const int lane = threadIdx.x % kWave;
  // row maxima: over the 16 column lanes and both column fragments
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = -INFINITY;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int64_t col = col0 + 16 * ni + (lane & 15);
        if (col < Lr) v = fmaxf(v, acc[mi][ni][r]);
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
      const int64_t row = row0 + 16 * mi + (lane >> 4) * 4 + r;
      if ((lane & 15) == 0 && row < Lp && v > -INFINITY) atomicMax(rowmax + row, ordered_bits(v));
    }
  }
  // column maxima: over the 4 registers, the 4 lane groups and both row fragments
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    float v = -INFINITY;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row0 + 16 * mi + (lane >> 4) * 4 + r;
        if (row < Lp) v = fmaxf(v, acc[mi][ni][r]);
      }
    v = fmaxf(v, __shfl_xor(v, 16, kWave));
    v = fmaxf(v, __shfl_xor(v, 32, kWave));
    const int64_t col = col0 + 16 * ni + (lane & 15);
    if (lane < 16 && col < Lr && v > -INFINITY) atomicMax(colmax + col, ordered_bits(v));
  }
}

template <typename T>
__global__ __launch_bounds__(kBsThreads) void greedy_match_half_kernel(const T* __restrict__ P, const T* __restrict__ R, int64_t Lp, int64_t Lr,
                                                                       int64_t D, int* __restrict__ rowmax, int* __restrict__ colmax) {
  const int64_t b = blockIdx.z;
  const T* Pb = P + b * Lp * D;
  const T* Rb = R + b * Lr * D;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int64_t row0 = static_cast<int64_t>(blockIdx.y) * kBsTile + (wave >> 1) * 32;
  const int64_t col0 = static_cast<int64_t>(blockIdx.x) * kBsTile + (wave & 1) * 32;
  bs_acc4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = bs_acc4{0.f, 0.f, 0.f, 0.f};
  const int kl = 8 * (lane >> 4);
  for (int64_t k0 = 0; k0 < D; k0 += 32) {
    bs_frag8 a[2], bb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = load8<T>(Pb, row0 + 16 * i + (lane & 15), Lp, D, k0 + kl);
      bb[i] = load8<T>(Rb, col0 + 16 * i + (lane & 15), Lr, D, k0 + kl);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16<T>(a[i], bb[j], acc[i][j]);
  }
  fold_maxima(acc, row0, col0, Lp, Lr, rowmax + b * Lp, colmax + b * Lr);
}

__global__ __launch_bounds__(kBsThreads) void greedy_match_f32_kernel(const float* __restrict__ P, const float* __restrict__ R, int64_t Lp,
                                                                      int64_t Lr, int64_t D, int* __restrict__ rowmax, int* __restrict__ colmax) {
  const int64_t b = blockIdx.z;
  const float* Pb = P + b * Lp * D;
  const float* Rb = R + b * Lr * D;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int64_t row0 = static_cast<int64_t>(blockIdx.y) * kBsTile + (wave >> 1) * 32;
  const int64_t col0 = static_cast<int64_t>(blockIdx.x) * kBsTile + (wave & 1) * 32;
  bs_acc4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = bs_acc4{0.f, 0.f, 0.f, 0.f};
  const int kl = lane >> 4;  // 16x16x4: lane holds A[row lane&15][k = lane>>4], B[k = lane>>4][col lane&15]
  for (int64_t k0 = 0; k0 < D; k0 += 4) {
    const int64_t k = k0 + kl;
    float a[2], bb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t pr = row0 + 16 * i + (lane & 15), rr = col0 + 16 * i + (lane & 15);
      a[i] = (pr < Lp && k < D) ? Pb[pr * D + k] : 0.f;
      bb[i] = (rr < Lr && k < D) ? Rb[rr * D + k] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bb[j], acc[i][j], 0, 0, 0);
  }
  fold_maxima(acc, row0, col0, Lp, Lr, rowmax + b * Lp, colmax + b * Lr);
}

// ----------------------------------------------------------------------------------------- tiled MFMA path
// 128 x 128 output tile per 256-thread block (2 x 2 waves of 64 x 64, 4 x 4 MFMA 16x16x32 tiles each), K staged
// through LDS in 64-wide slices with double buffering: the next slice's 16-B global loads are in flight in
// registers while the current slice feeds 32 MFMAs per wave; one barrier per slice (the 32x32x16 variant of this
// tile measured slower: 394 vs 451 TFLOP/s at the BASELINE shape).  LDS rows are padded to 72
// elements (144 B) so the 16 lanes of every ds_read_b128 group hit 16 distinct 16-B bank slots.  A pair's 16 tiles
// are mapped to one XCD (bijective remap of the 1-D block id), so the pair's P / R rows are re-read from that XCD's
// L2.  The epilogue is the same fold as above (row / column maxima, order-preserving integer atomicMax).
constexpr int kT = 128;          // output tile
constexpr int kTK = 64;          // K slice
constexpr int kTLd = kTK + 8;    // padded LDS row (elements)
constexpr int kTThreads = 256;

template <typename T>
__global__ __launch_bounds__(kTThreads) void greedy_match_tiled_kernel(const T* __restrict__ P, const T* __restrict__ R, int64_t B, int64_t Lp,
                                                                       int64_t Lr, int64_t D, int tiles_m, int tiles_n,
                                                                       int* __restrict__ rowmax, int* __restrict__ colmax) {
  __shared__ __attribute__((aligned(16))) short lds[2][2][kT * kTLd];  // [buffer][A|B][row * kTLd + k]
  // XCD-aware, bijective remap: consecutive tile ids (one pair's tiles) share an XCD
  const int64_t nwg = static_cast<int64_t>(gridDim.x);
  const int64_t orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t per_pair = static_cast<int64_t>(tiles_m) * tiles_n;
  const int64_t b = id / per_pair;
  const int tm = static_cast<int>((id % per_pair) / tiles_n), tn = static_cast<int>(id % tiles_n);
  if (b >= B) return;
  const T* Pb = P + b * Lp * D;
  const T* Rb = R + b * Lr * D;
  const int64_t row0 = static_cast<int64_t>(tm) * kT, col0 = static_cast<int64_t>(tn) * kT;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int wr = wave >> 1, wc = wave & 1;

  // global -> register staging: chunk c = tid + 256 i (i < 4) of a 128 x 64 slice: row c / 8, 16-B column c % 8
  bs_frag8 ra[4], rb[4];
  auto load_slice = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kTThreads * i;
      const int r = c >> 3, kk = (c & 7) * 8;
      const int64_t k = k0 + kk;
      ra[i] = (row0 + r < Lp && k < D) ? *reinterpret_cast<const bs_frag8*>(Pb + (row0 + r) * D + k) : bs_frag8{0, 0, 0, 0, 0, 0, 0, 0};
      rb[i] = (col0 + r < Lr && k < D) ? *reinterpret_cast<const bs_frag8*>(Rb + (col0 + r) * D + k) : bs_frag8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kTThreads * i;
      const int r = c >> 3, kk = (c & 7) * 8;
      *reinterpret_cast<bs_frag8*>(&lds[buf][0][r * kTLd + kk]) = ra[i];
      *reinterpret_cast<bs_frag8*>(&lds[buf][1][r * kTLd + kk]) = rb[i];
    }
  };

  bs_acc4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = bs_acc4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((D + kTK - 1) / kTK);
  load_slice(0);
  store_slice(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load_slice(static_cast<int64_t>(s + 1) * kTK);  // in flight during this slice's MFMAs
    const short* A = lds[buf][0];
    const short* Bt = lds[buf][1];
#pragma unroll
    for (int kh = 0; kh < kTK; kh += 32) {
      bs_frag8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const bs_frag8*>(A + (wr * 64 + 16 * i + fr) * kTLd + kh + fk);
        bf[i] = *reinterpret_cast<const bs_frag8*>(Bt + (wc * 64 + 16 * i + fr) * kTLd + kh + fk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<T>(af[i], bf[j], acc[i][j]);
    }
    if (s + 1 < nk) {
      store_slice(buf ^ 1);  // the other buffer was last read one slice ago, before the previous barrier
    }
    __syncthreads();
  }

  // epilogue: this wave's 64 x 64 block -> row maxima (over its 64 columns) and column maxima (over its 64 rows)
  int* rmax = rowmax + b * Lp;
  int* cmax = colmax + b * Lr;
  const int64_t wrow0 = row0 + wr * 64, wcol0 = col0 + wc * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = wcol0 + 16 * j + fr;
        if (col < Lr) v = fmaxf(v, acc[i][j][r]);
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
      const int64_t row = wrow0 + 16 * i + (lane >> 4) * 4 + r;
      if (fr == 0 && row < Lp && v > -INFINITY) atomicMax(rmax + row, ordered_bits(v));
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = wrow0 + 16 * i + (lane >> 4) * 4 + r;
        if (row < Lp) v = fmaxf(v, acc[i][j][r]);
      }
    v = fmaxf(v, __shfl_xor(v, 16, kWave));
    v = fmaxf(v, __shfl_xor(v, 32, kWave));
    const int64_t col = wcol0 + 16 * j + fr;
    if (lane < 16 && col < Lr && v > -INFINITY) atomicMax(cmax + col, ordered_bits(v));
  }
}

// ------------------------------------------------------------------------------------ 256 x 256 MFMA path
// Same pipeline as the 128 x 128 tile, twice the edge: 8 waves as 4 (M) x 2 (N), each owning a 64 x 128 block
// (4 x 8 MFMA 16x16x32 tiles, 128 accumulator registers), so a 32-deep K step issues 32 MFMAs per 12 ds_read_b128
// (2.7 MFMA per LDS read vs 2.0) and every block streams half the L2 bytes per FLOP.  Double-buffered 64-wide K
// slices with padded rows: 2 x (256 + 256) x 72 x 2 B = 144 KiB of the 160 KiB LDS, one block per CU.
constexpr int kW = 256;
constexpr int kWThreads = 512;

template <typename T>
__global__ __launch_bounds__(kWThreads) void greedy_match_w256_kernel(const T* __restrict__ P, const T* __restrict__ R, int64_t B, int64_t Lp,
                                                                      int64_t Lr, int64_t D, int tiles_m, int tiles_n,
                                                                      int* __restrict__ rowmax, int* __restrict__ colmax) {
  __shared__ __attribute__((aligned(16))) short lds[2][2][kW * kTLd];  // [buffer][A|B][row * kTLd + k]
  const int64_t nwg = static_cast<int64_t>(gridDim.x);
  const int64_t orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t per_pair = static_cast<int64_t>(tiles_m) * tiles_n;
  const int64_t b = id / per_pair;
  const int tm = static_cast<int>((id % per_pair) / tiles_n), tn = static_cast<int>(id % tiles_n);
  if (b >= B) return;
  const T* Pb = P + b * Lp * D;
  const T* Rb = R + b * Lr * D;
  const int64_t row0 = static_cast<int64_t>(tm) * kW, col0 = static_cast<int64_t>(tn) * kW;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int wr = wave >> 1, wc = wave & 1;

  // global -> register staging: chunk c = tid + 512 i (i < 4) of a 256 x 64 slice: row c / 8, 16-B column c % 8
  bs_frag8 ra[4], rb[4];
  auto load_slice = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kWThreads * i;
      const int r = c >> 3, kk = (c & 7) * 8;
      const int64_t k = k0 + kk;
      ra[i] = (row0 + r < Lp && k < D) ? *reinterpret_cast<const bs_frag8*>(Pb + (row0 + r) * D + k) : bs_frag8{0, 0, 0, 0, 0, 0, 0, 0};
      rb[i] = (col0 + r < Lr && k < D) ? *reinterpret_cast<const bs_frag8*>(Rb + (col0 + r) * D + k) : bs_frag8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kWThreads * i;
      const int r = c >> 3, kk = (c & 7) * 8;
      *reinterpret_cast<bs_frag8*>(&lds[buf][0][r * kTLd + kk]) = ra[i];
      *reinterpret_cast<bs_frag8*>(&lds[buf][1][r * kTLd + kk]) = rb[i];
    }
  };

  bs_acc4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = bs_acc4{0.f, 0.f, 0.f, 0.f};

  const int nk = static_cast<int>((D + kTK - 1) / kTK);
  load_slice(0);
  store_slice(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load_slice(static_cast<int64_t>(s + 1) * kTK);  // in flight during this slice's MFMAs
    const short* A = lds[buf][0];
    const short* Bt = lds[buf][1];
#pragma unroll
    for (int kh = 0; kh < kTK; kh += 32) {
      bs_frag8 af[4], bf[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bs_frag8*>(A + (wr * 64 + 16 * i + fr) * kTLd + kh + fk);
#pragma unroll
      for (int j = 0; j < 8; ++j) bf[j] = *reinterpret_cast<const bs_frag8*>(Bt + (wc * 128 + 16 * j + fr) * kTLd + kh + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = mfma16<T>(af[i], bf[j], acc[i][j]);
    }
    if (s + 1 < nk) store_slice(buf ^ 1);  // the other buffer was last read one slice ago, before the previous barrier
    __syncthreads();
  }

  int* rmax = rowmax + b * Lp;
  int* cmax = colmax + b * Lr;
  const int64_t wrow0 = row0 + wr * 64, wcol0 = col0 + wc * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t col = wcol0 + 16 * j + fr;
        if (col < Lr) v = fmaxf(v, acc[i][j][r]);
      }
#pragma unroll
      for (int off = 8; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
      const int64_t row = wrow0 + 16 * i + (lane >> 4) * 4 + r;
      if (fr == 0 && row < Lp && v > -INFINITY) atomicMax(rmax + row, ordered_bits(v));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = wrow0 + 16 * i + (lane >> 4) * 4 + r;
        if (row < Lp) v = fmaxf(v, acc[i][j][r]);
      }
    v = fmaxf(v, __shfl_xor(v, 16, kWave));
    v = fmaxf(v, __shfl_xor(v, 32, kWave));
    const int64_t col = wcol0 + 16 * j + fr;
    if (lane < 16 && col < Lr && v > -INFINITY) atomicMax(cmax + col, ordered_bits(v));
  }
}

// one launch fills both maxima with the ordered encoding of -inf; one launch decodes both in place to fp32 bits
__global__ void bs_fill_kernel(int* __restrict__ a, int64_t na, int* __restrict__ b, int64_t nb, int v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * blockDim.x)
    (i < na ? a[i] : b[i - na]) = v;
}
__global__ void bs_decode_kernel(int* __restrict__ a, int64_t na, int* __restrict__ b, int64_t nb) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * blockDim.x) {
    int* p = i < na ? a + i : b + (i - na);
    const int x = *p;
    *p = x >= 0 ? x : x ^ 0x7fffffff;
  }
}

// P [B, Lp, D], R [B, Lr, D] (same float dtype) -> (rowmax [B, Lp] fp32, colmax [B, Lr] fp32)
std::tuple<at::Tensor, at::Tensor> bert_greedy_match(const at::Tensor& P_in, const at::Tensor& R_in) {
  TORCH_CHECK(P_in.is_cuda() && R_in.is_cuda(), "bert_greedy_match: expected GPU tensors");
  TORCH_CHECK(P_in.dim() == 3 && R_in.dim() == 3 && P_in.size(0) == R_in.size(0) && P_in.size(2) == R_in.size(2),
              "bert_greedy_match: expected [B, Lp, D] and [B, Lr, D]");
  TORCH_CHECK(P_in.scalar_type() == R_in.scalar_type(), "bert_greedy_match: dtype mismatch");
  const at::DeviceGuard guard(P_in.device());
  auto P = P_in.contiguous(), R = R_in.contiguous();
  const int64_t B = P.size(0), Lp = P.size(1), Lr = R.size(1), D = P.size(2);
  TORCH_CHECK(B <= 65535, "bert_greedy_match: at most 65535 pairs per call");
  auto opts = P.options().dtype(at::kInt);
  // order-preserving encoding of -inf as the identity of max
  const int neg_inf_bits = static_cast<int>(0xff800000u ^ 0x7fffffffu);
  auto rowmax = at::empty({B, Lp}, opts);
  auto colmax = at::empty({B, Lr}, opts);
  if (B == 0 || Lp == 0 || Lr == 0) {
    return {rowmax.to(at::kFloat).fill_(-INFINITY), colmax.to(at::kFloat).fill_(-INFINITY)};
  }
  const int64_t n_fill = B * (Lp + Lr);
  hipLaunchKernelGGL(bs_fill_kernel, grid_for(n_fill, 256), 256, 0, stream(), rowmax.data_ptr<int>(), B * Lp, colmax.data_ptr<int>(),
                     B * Lr, neg_inf_bits);
  TMX_LAUNCH_CHECK();
  dim3 grid(static_cast<unsigned>((Lr + kBsTile - 1) / kBsTile), static_cast<unsigned>((Lp + kBsTile - 1) / kBsTile),
            static_cast<unsigned>(B));
  const bool tiled = (P.scalar_type() == at::kBFloat16 || P.scalar_type() == at::kHalf) && D % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(P.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(R.data_ptr()) & 15) == 0;
  // 256-wide tiles when they waste little of the pair (<= 25 % padding); else the 128-wide tile
  const int64_t wm = (Lp + kW - 1) / kW, wn = (Lr + kW - 1) / kW;
  const bool wide = tiled && Lp >= kW && Lr >= kW && 4 * wm * wn * kW * kW <= 5 * Lp * Lr &&
                    std::getenv("TMX_BERT_TILE128") == nullptr;
  if (wide) {
    const int64_t nblocks = B * wm * wn;
    TORCH_CHECK(nblocks < (1ll << 31), "bert_greedy_match: too many tiles");
    if (P.scalar_type() == at::kBFloat16) {
      greedy_match_w256_kernel<__hip_bfloat16><<<static_cast<unsigned>(nblocks), kWThreads, 0, stream()>>>(
          reinterpret_cast<const __hip_bfloat16*>(P.data_ptr()), reinterpret_cast<const __hip_bfloat16*>(R.data_ptr()), B, Lp, Lr, D,
          static_cast<int>(wm), static_cast<int>(wn), rowmax.data_ptr<int>(), colmax.data_ptr<int>());
    } else {
      greedy_match_w256_kernel<__half><<<static_cast<unsigned>(nblocks), kWThreads, 0, stream()>>>(
          reinterpret_cast<const __half*>(P.data_ptr()), reinterpret_cast<const __half*>(R.data_ptr()), B, Lp, Lr, D, static_cast<int>(wm),
          static_cast<int>(wn), rowmax.data_ptr<int>(), colmax.data_ptr<int>());
    }
    TMX_LAUNCH_CHECK();
  } else if (tiled) {
    const int tiles_m = static_cast<int>((Lp + kT - 1) / kT), tiles_n = static_cast<int>((Lr + kT - 1) / kT);
    const int64_t nblocks = B * tiles_m * tiles_n;
    TORCH_CHECK(nblocks < (1ll << 31), "bert_greedy_match: too many tiles");
    if (P.scalar_type() == at::kBFloat16) {
      greedy_match_tiled_kernel<__hip_bfloat16><<<static_cast<unsigned>(nblocks), kTThreads, 0, stream()>>>(
          reinterpret_cast<const __hip_bfloat16*>(P.data_ptr()), reinterpret_cast<const __hip_bfloat16*>(R.data_ptr()), B, Lp, Lr, D,
          tiles_m, tiles_n, rowmax.data_ptr<int>(), colmax.data_ptr<int>());
    } else {
      greedy_match_tiled_kernel<__half><<<static_cast<unsigned>(nblocks), kTThreads, 0, stream()>>>(
          reinterpret_cast<const __half*>(P.data_ptr()), reinterpret_cast<const __half*>(R.data_ptr()), B, Lp, Lr, D, tiles_m, tiles_n,
          rowmax.data_ptr<int>(), colmax.data_ptr<int>());
    }
    TMX_LAUNCH_CHECK();
  } else switch (P.scalar_type()) {
    case at::kBFloat16:
      hipLaunchKernelGGL(greedy_match_half_kernel<__hip_bfloat16>, grid, kBsThreads, 0, stream(),
                         reinterpret_cast<const __hip_bfloat16*>(P.data_ptr()), reinterpret_cast<const __hip_bfloat16*>(R.data_ptr()),
                         Lp, Lr, D, rowmax.data_ptr<int>(), colmax.data_ptr<int>());
      break;
    case at::kHalf:
      hipLaunchKernelGGL(greedy_match_half_kernel<__half>, grid, kBsThreads, 0, stream(), reinterpret_cast<const __half*>(P.data_ptr()),
                         reinterpret_cast<const __half*>(R.data_ptr()), Lp, Lr, D, rowmax.data_ptr<int>(), colmax.data_ptr<int>());
      break;
    case at::kFloat:
      hipLaunchKernelGGL(greedy_match_f32_kernel, grid, kBsThreads, 0, stream(), P.data_ptr<float>(), R.data_ptr<float>(), Lp, Lr, D,
                         rowmax.data_ptr<int>(), colmax.data_ptr<int>());
      break;
    default:
      TORCH_CHECK(false, "bert_greedy_match: unsupported dtype ", P.scalar_type());
  }
  TMX_LAUNCH_CHECK();
  // decode the ordered integers back to fp32 bits in place (one launch for both)
  hipLaunchKernelGGL(bs_decode_kernel, grid_for(n_fill, 256), 256, 0, stream(), rowmax.data_ptr<int>(), B * Lp, colmax.data_ptr<int>(), B * Lr);
  TMX_LAUNCH_CHECK();
  return {rowmax.view(at::kFloat), colmax.view(at::kFloat)};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("bert_greedy_match(Tensor preds_emb, Tensor target_emb) -> (Tensor, Tensor)"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("bert_greedy_match", &tmx::bert_greedy_match); }
