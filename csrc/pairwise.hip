// Pairwise distance / similarity matrices for gfx950: L1 / Lp (VALU) and the GEMM forms (MFMA).
//
// out[i, j] = (Σ_k |x[i,k] - y[j,k]|^p)^(1/p)   (p == 1: Manhattan, no root)
//
// The reference materialises the [N, M, d] broadcast difference (O(N·M·d) memory).  Here a block computes a
// 64×64 output tile with 256 threads (4×4 outputs per thread, register accumulators); x and y tiles of 64 rows ×
// 32 features are staged through LDS (padded rows: conflict-free column reads), so HBM traffic is
// O((N + M)·d·(tiles)) and the inner loop is pure VALU.  Accumulation in `Acc` (fp64 for Minkowski to match the
// reference's fp64 evaluation, fp32 otherwise).
#include "common.h"

namespace tmx {

constexpr int kPwTile = 64;
constexpr int kPwK = 32;
constexpr int kPwThreads = 256;

enum PwMode : int { kPwL1 = 0, kPwL2 = 1, kPwLp = 2 };

template <typename T, typename Acc>
__device__ __forceinline__ Acc pw_load(const T* p, int64_t i) {
  if constexpr (std::is_same<T, double>::value) return static_cast<Acc>(p[i]);
  else return static_cast<Acc>(to_f32<T>(p[i]));
}

template <typename T, typename Acc, int MODE>
__global__ __launch_bounds__(kPwThreads) void pairwise_lp_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                                 int64_t N, int64_t M, int64_t D, double p_d,
                                                                 Acc* __restrict__ out) {
  __shared__ Acc xs[kPwK][kPwTile + 1];
  __shared__ Acc ys[kPwK][kPwTile + 1];
  const Acc p = static_cast<Acc>(p_d);
  const int tx = threadIdx.x & 15;  // column group (y rows)
  const int ty = threadIdx.x >> 4;  // row group (x rows)
  const int64_t row0 = static_cast<int64_t>(blockIdx.y) * kPwTile;
  const int64_t col0 = static_cast<int64_t>(blockIdx.x) * kPwTile;

  Acc acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = Acc(0);

  for (int64_t k0 = 0; k0 < D; k0 += kPwK) {
    // cooperative tile loads: 64 rows x 32 features each for x and y
    for (int e = threadIdx.x; e < kPwTile * kPwK; e += kPwThreads) {
      const int r = e / kPwK;
      const int k = e - r * kPwK;
      const int64_t gk = k0 + k;
      const int64_t gx = row0 + r, gy = col0 + r;
      xs[k][r] = (gx < N && gk < D) ? pw_load<T, Acc>(x, gx * D + gk) : Acc(0);
      ys[k][r] = (gy < M && gk < D) ? pw_load<T, Acc>(y, gy * D + gk) : Acc(0);
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kPwK; ++k) {
      Acc xv[4], yv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) xv[a] = xs[k][ty + 16 * a];
#pragma unroll
      for (int b = 0; b < 4; ++b) yv[b] = ys[k][tx + 16 * b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          Acc d = xv[a] - yv[b];
          if constexpr (MODE == kPwL1) acc[a][b] += fabs(d);
          else if constexpr (MODE == kPwL2) acc[a][b] += d * d;
          else acc[a][b] += pow(fabs(d), p);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int64_t i = row0 + ty + 16 * a;
    if (i >= N) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int64_t j = col0 + tx + 16 * b;
      if (j >= M) continue;
      Acc v = acc[a][b];
      if constexpr (MODE == kPwL2) v = sqrt(v);
      else if constexpr (MODE == kPwLp) v = pow(v, Acc(1) / p);
      out[i * M + j] = v;
    }
  }
}

template <typename T, typename Acc>
void launch_pairwise(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, int mode, double p) {
  const int64_t N = x.size(0), M = y.size(0), D = x.size(1);
  dim3 grid(static_cast<unsigned>((M + kPwTile - 1) / kPwTile), static_cast<unsigned>((N + kPwTile - 1) / kPwTile));
  const auto* xp = reinterpret_cast<const T*>(x.data_ptr());
  const auto* yp = reinterpret_cast<const T*>(y.data_ptr());
  Acc* op = out.data_ptr<Acc>();
  if (mode == kPwL1) hipLaunchKernelGGL((pairwise_lp_kernel<T, Acc, kPwL1>), grid, kPwThreads, 0, stream(), xp, yp, N, M, D, p, op);
  else if (mode == kPwL2) hipLaunchKernelGGL((pairwise_lp_kernel<T, Acc, kPwL2>), grid, kPwThreads, 0, stream(), xp, yp, N, M, D, p, op);
  else hipLaunchKernelGGL((pairwise_lp_kernel<T, Acc, kPwLp>), grid, kPwThreads, 0, stream(), xp, yp, N, M, D, p, op);
}

// Returns [N, M] distances in fp64 when `fp64_acc` else fp32.
at::Tensor pairwise_lp(const at::Tensor& x_in, const at::Tensor& y_in, double p, bool fp64_acc) {
  TORCH_CHECK(x_in.is_cuda() && y_in.is_cuda(), "pairwise_lp: expected GPU tensors");
  TORCH_CHECK(x_in.dim() == 2 && y_in.dim() == 2 && x_in.size(1) == y_in.size(1), "pairwise_lp: expected [N,d] and [M,d]");
  TORCH_CHECK(x_in.scalar_type() == y_in.scalar_type(), "pairwise_lp: dtype mismatch");
  TORCH_CHECK(p >= 1.0, "pairwise_lp: p must be >= 1");
  const at::DeviceGuard guard(x_in.device());
  auto x = x_in.contiguous();
  auto y = y_in.contiguous();
  const int mode = (p == 1.0) ? kPwL1 : (p == 2.0 ? kPwL2 : kPwLp);
  auto out = at::empty({x.size(0), y.size(0)}, x.options().dtype(fp64_acc ? at::kDouble : at::kFloat));
  if (x.size(0) == 0 || y.size(0) == 0) return out;
  if (x.size(1) == 0) return out.zero_();
  TMX_DISPATCH_FLOAT(x.scalar_type(), "pairwise_lp", [&] {
    if (fp64_acc) launch_pairwise<scalar_t, double>(x, y, out, mode, p);
    else launch_pairwise<scalar_t, float>(x, y, out, mode, p);
  });
  TMX_LAUNCH_CHECK();
  return out;
}

// ------------------------------------------------------------------------------ GEMM forms: linear / cosine / euclidean
// out[i, j] = epilogue(x[i] . y[j]) in one kernel (reference ``functional/pairwise/{linear,cosine,euclidean}.py``):
//   linear     x . y                                (fp32 accumulation for fp32 / bf16 / fp16, fp64 for fp64)
//   cosine     x . y * (1/|x|) * (1/|y|)            (the reference normalises the rows first, then runs the GEMM)
//   euclidean  sqrt(T(|x|^2 + |y|^2 - 2 x . y))     (fp64 throughout, as the reference's upcast; rounded to the input
//                                                    dtype before the root, diagonal zeroed before the root)
// The reference runs 4-12 separate ATen kernels and, for euclidean, round-trips the N x M matrix through HBM in fp64
// five times.  Here one 64 x 64 output tile per 256-thread workgroup: 64-row slices of x and y (32 deep for fp32
// accumulation, 16 for fp64) are converted to the accumulation type on the way into LDS (k-major rows padded to 80
// elements: the four 16-lane groups of a fragment read land in disjoint bank ranges), double-buffered with the next
// slice in registers during the MFMAs; each wave owns a 32 x 32 block (2 x 2 MFMA tiles: v_mfma_f32_16x16x4_f32,
// exact fp32 products, or v_mfma_f64_16x16x4_f64).  Row norms are summed from the staging registers (no extra pass),
// the epilogue runs on the accumulators and writes the input dtype once.  Tile ids are remapped so that consecutive
// ids (same x rows) share an XCD and its L2.
enum PgMode : int { kPgLinear = 0, kPgCosine = 1, kPgEuclid = 2, kPgAbsCosMax = 3 };  // 3: MiFID's row max |cos|
constexpr int kPgT = 64, kPgPad = 16, kPgThreads = 256;
// slice depth: 32 (fp32) / 16 (fp64) -- 40 KiB of double-buffered LDS either way, three workgroups per CU
template <typename Acc> constexpr int pg_k() { return std::is_same<Acc, double>::value ? 16 : 32; }

template <typename Acc> struct PgMma;
template <> struct PgMma<float> {
  typedef float V __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ V mma(float a, float b, V c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) * 4 + r; }
};
template <> struct PgMma<double> {
  typedef double V __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ V mma(double a, double b, V c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }  // f64 C/D map
};

template <typename T, typename Acc> __device__ __forceinline__ Acc pg_in(T v) {
  if constexpr (std::is_same<T, double>::value) return static_cast<Acc>(v);
  else return static_cast<Acc>(to_f32<T>(v));
}
// Acc -> output dtype the way ATen's ``.to`` does (double -> float -> 16-bit: c10 rounds through float)
template <typename T, typename Acc> __device__ __forceinline__ T pg_out(Acc v) {
  if constexpr (std::is_same<T, double>::value) return static_cast<double>(v);
  else if constexpr (std::is_same<T, float>::value) return static_cast<float>(v);
  else if constexpr (std::is_same<T, __hip_bfloat16>::value) return __float2bfloat16(static_cast<float>(v));
  else return __float2half(static_cast<float>(v));
}
template <typename T> __device__ __forceinline__ T pg_sqrt(T v) {
  if constexpr (std::is_same<T, double>::value) return sqrt(v);
  else if constexpr (std::is_same<T, float>::value) return sqrtf(v);
  else return pg_out<T, float>(sqrtf(to_f32<T>(v)));
}

// KPT consecutive elements of one row into Acc registers: whole-vector loads when VEC (D % KPT == 0, rows aligned
// to the vector: host check)
template <typename T, typename Acc, int KPT, bool VEC>
__device__ __forceinline__ void pg_load(const T* __restrict__ p, int64_t row, int64_t nrows, int64_t k, int64_t D, Acc (&v)[KPT]) {
  if constexpr (VEC) {
    constexpr int kBytes = KPT * static_cast<int>(sizeof(T));
    constexpr int kVec = kBytes < 16 ? kBytes : 16;
    using W = typename std::conditional<kVec == 16, uint4, uint2>::type;
    constexpr int kPer = kVec / static_cast<int>(sizeof(T));
    if (row < nrows && k < D) {
      const W* q = reinterpret_cast<const W*>(p + row * D + k);
#pragma unroll
      for (int c = 0; c < KPT / kPer; ++c) {
        const W w = q[c];
        const T* e = reinterpret_cast<const T*>(&w);
#pragma unroll
        for (int i = 0; i < kPer; ++i) v[c * kPer + i] = pg_in<T, Acc>(e[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < KPT; ++i) v[i] = Acc(0);
    }
  } else {
#pragma unroll
    for (int i = 0; i < KPT; ++i) v[i] = (row < nrows && k + i < D) ? pg_in<T, Acc>(p[row * D + k + i]) : Acc(0);
  }
}

template <typename T, typename Acc, int MODE, bool VEC>
__global__ __launch_bounds__(kPgThreads) void pairwise_gemm_kernel(const T* __restrict__ x, const T* __restrict__ y, int64_t N, int64_t M,
                                                                   int64_t D, int tiles_n, bool zero_diag, T* __restrict__ out,
                                                                   void* __restrict__ rowmax = nullptr,
                                                                   const int* __restrict__ run_if = nullptr) {
  using Mma = PgMma<Acc>;
  constexpr int kPgK = pg_k<Acc>(), KPT = kPgK / 4;
  __shared__ Acc xs[2][kPgK][kPgT + kPgPad];
  __shared__ Acc ys[2][kPgK][kPgT + kPgPad];
  __shared__ Acc nrm[2][kPgT];
  if (run_if != nullptr && *run_if == 0) return;  // device-side fallback launch (x3 route, non-finite inputs)
  const int64_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t row0 = (id / tiles_n) * kPgT, col0 = (id % tiles_n) * kPgT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int sr = tid >> 2, sk = (tid & 3) * KPT;  // staging: row sr, k [sk, sk + KPT) of the slice
  // two register sets: slices s + 1 and s + 2 in flight while slice s is multiplied
  Acc rx[2][KPT], ry[2][KPT];
  Acc px = Acc(0), py = Acc(0);
  auto load = [&](int64_t k0, Acc (&qx)[KPT], Acc (&qy)[KPT]) {
    pg_load<T, Acc, KPT, VEC>(x, row0 + sr, N, k0 + sk, D, qx);
    pg_load<T, Acc, KPT, VEC>(y, col0 + sr, M, k0 + sk, D, qy);
    if constexpr (MODE != kPgLinear) {
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        px = fma(qx[i], qx[i], px);
        py = fma(qy[i], qy[i], py);
      }
    }
  };
  auto store = [&](int buf, const Acc (&qx)[KPT], const Acc (&qy)[KPT]) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      xs[buf][sk + i][sr] = qx[i];
      ys[buf][sk + i][sr] = qy[i];
    }
  };
  typename Mma::V acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = typename Mma::V{0, 0, 0, 0};
  const int nk = static_cast<int>((D + kPgK - 1) / kPgK);
  load(0, rx[0], ry[0]);
  store(0, rx[0], ry[0]);
  if (nk > 1) load(kPgK, rx[1], ry[1]);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  // nx / ny: the set that held slice s (already in LDS) takes slice s + 2; sx / sy hold slice s + 1
  auto step = [&](int s, Acc (&nx)[KPT], Acc (&ny)[KPT], const Acc (&sx)[KPT], const Acc (&sy)[KPT]) {
    const int buf = s & 1;
    if (s + 2 < nk) load(static_cast<int64_t>(s + 2) * kPgK, nx, ny);
#pragma unroll
    for (int kk = 0; kk < kPgK; kk += 4) {
      Acc a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = xs[buf][kk + fk][wr * 32 + 16 * i + fr];
        b[i] = ys[buf][kk + fk][wc * 32 + 16 * i + fr];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mma::mma(a[i], b[j], acc[i][j]);
    }
    if (s + 1 < nk) store(buf ^ 1, sx, sy);  // that buffer was last read before the previous barrier
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, rx[0], ry[0], rx[1], ry[1]);
    if (s + 1 < nk) step(s + 1, rx[1], ry[1], rx[0], ry[0]);
  }
  if constexpr (MODE != kPgLinear) {
    // four consecutive lanes share a staging row
    px += __shfl_xor(px, 1, kWave);
    px += __shfl_xor(px, 2, kWave);
    py += __shfl_xor(py, 1, kWave);
    py += __shfl_xor(py, 2, kWave);
    if ((tid & 3) == 0) {  // cosine keeps reciprocal norms: the epilogue is two multiplies per output
      nrm[0][sr] = MODE == kPgCosine || MODE == kPgAbsCosMax ? Acc(1) / sqrt(px) : px;
      nrm[1][sr] = MODE == kPgCosine || MODE == kPgAbsCosMax ? Acc(1) / sqrt(py) : py;
    }
    __syncthreads();
  }
  if constexpr (MODE == kPgAbsCosMax) {
    // row maxima of |cos|: the lane's two columns, then the 16 lanes of a row (col = lane & 15 in both C/D maps),
    // one order-preserving integer atomicMax per (row, wave) -- non-negative floats order as their bit patterns
    using Bits = typename std::conditional<std::is_same<Acc, double>::value, unsigned long long, unsigned int>::type;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 32 + 16 * i + Mma::row(lane, r);
        const int64_t gi = row0 + lr;
        Acc mv = Acc(-1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int lc = wc * 32 + 16 * j + fr;
          if (gi < N && col0 + lc < M) mv = fmax(mv, fabs(acc[i][j][r] * nrm[0][lr] * nrm[1][lc]));
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) mv = fmax(mv, __shfl_xor(mv, off, kWave));
        if (fr == 0 && gi < N && mv >= Acc(0)) atomicMax(reinterpret_cast<Bits*>(rowmax) + gi, __builtin_bit_cast(Bits, mv));
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 32 + 16 * i + Mma::row(lane, r), lc = wc * 32 + 16 * j + fr;
        const int64_t gi = row0 + lr, gj = col0 + lc;
        if (gi >= N || gj >= M) continue;
        const Acc v = acc[i][j][r];
        T res;
        if constexpr (MODE == kPgLinear) {
          res = pg_out<T, Acc>(v);
          if (zero_diag && gi == gj) res = pg_out<T, Acc>(Acc(0));
        } else if constexpr (MODE == kPgCosine) {
          res = pg_out<T, Acc>(v * nrm[0][lr] * nrm[1][lc]);
          if (zero_diag && gi == gj) res = pg_out<T, Acc>(Acc(0));
        } else {
          T d = pg_out<T, Acc>((nrm[0][lr] + nrm[1][lc]) - Acc(2) * v);
          if (zero_diag && gi == gj) d = pg_out<T, Acc>(Acc(0));
          res = pg_sqrt<T>(d);
        }
        out[gi * M + gj] = res;
      }
}

// 16-bit inputs, linear / cosine, large outputs: 128 x 128 tiles on v_mfma_f32_16x16x32_{bf16,f16} (exact 16-bit
// products, fp32 accumulation -- what the f32 MFMA path above computes, at 16x its rate).  Four waves, each a 64 x 64
// block of 4 x 4 MFMA tiles; 64-deep K slices of both operands staged row-major in LDS (rows padded to 72 elements:
// the 16 lanes of each ds_read_b128 group land on distinct bank quads), double-buffered with the next slice in
// registers.  Cosine scales by reciprocal fp32 row norms taken by one ATen reduction per operand.
constexpr int kPhT = 128, kPhK = 64, kPhLd = kPhK + 8, kPhThreads = 256;
typedef short ph_frag8 __attribute__((ext_vector_type(8)));
typedef float ph_acc4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ ph_acc4 ph_mma(ph_frag8 a, ph_frag8 b, ph_acc4 c) {
  if constexpr (std::is_same<T, __hip_bfloat16>::value) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(a),
                                                      reinterpret_cast<__attribute__((ext_vector_type(8))) _Float16&>(b), c, 0, 0, 0);
}

template <typename T, int MODE, bool VEC>
__global__ __launch_bounds__(kPhThreads) void pairwise_gemm_h16_kernel(const T* __restrict__ x, const T* __restrict__ y, int64_t N, int64_t M,
                                                                       int64_t D, int tiles_n, bool zero_diag, T* __restrict__ out,
                                                                       const float* __restrict__ xnorm, const float* __restrict__ ynorm) {
  __shared__ __attribute__((aligned(16))) short lds[2][2][kPhT * kPhLd];  // [buffer][x | y][row * kPhLd + k]
  __shared__ float nrm[2][kPhT];
  const int64_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t row0 = (id / tiles_n) * kPhT, col0 = (id % tiles_n) * kPhT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // staging chunk i (< 4): row (tid >> 3) + 32 i, elements [8 (tid & 7), + 8) of the slice
  ph_frag8 rx[4], ry[4];
  auto ld8 = [&](const T* __restrict__ p, int64_t row, int64_t nrows, int64_t k) -> ph_frag8 {
    ph_frag8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row < nrows) {
      if constexpr (VEC) {
        if (k < D) v = *reinterpret_cast<const ph_frag8*>(p + row * D + k);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (k + e < D) v[e] = reinterpret_cast<const short*>(p)[row * D + k + e];
      }
    }
    return v;
  };
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const int64_t k = k0 + 8 * (tid & 7);
      rx[i] = ld8(x, row0 + r, N, k);
      ry[i] = ld8(y, col0 + r, M, k);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i, kk = 8 * (tid & 7);
      *reinterpret_cast<ph_frag8*>(&lds[buf][0][r * kPhLd + kk]) = rx[i];
      *reinterpret_cast<ph_frag8*>(&lds[buf][1][r * kPhLd + kk]) = ry[i];
    }
  };
  ph_acc4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ph_acc4{0.f, 0.f, 0.f, 0.f};
  const int nk = static_cast<int>((D + kPhK - 1) / kPhK);
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load(static_cast<int64_t>(s + 1) * kPhK);
    const short* A = lds[buf][0];
    const short* B = lds[buf][1];
#pragma unroll
    for (int kh = 0; kh < kPhK; kh += 32) {
      ph_frag8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const ph_frag8*>(A + (wr * 64 + 16 * i + fr) * kPhLd + kh + fk);
        bf[i] = *reinterpret_cast<const ph_frag8*>(B + (wc * 64 + 16 * i + fr) * kPhLd + kh + fk);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = ph_mma<T>(af[i], bf[j], acc[i][j]);
    }
    if (s + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  if constexpr (MODE == kPgCosine) {  // reciprocal row norms of the tile (fp32 norms of the inputs, from the host op)
    const int64_t g = tid < kPhT ? row0 + tid : col0 + (tid - kPhT);
    const float nv = tid < kPhT ? (g < N ? xnorm[g] : 1.f) : (g < M ? ynorm[g] : 1.f);
    nrm[tid >> 7][tid & 127] = 1.f / nv;
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 64 + 16 * i + (lane >> 4) * 4 + r, lc = wc * 64 + 16 * j + fr;
        const int64_t gi = row0 + lr, gj = col0 + lc;
        if (gi >= N || gj >= M) continue;
        float v = acc[i][j][r];
        if constexpr (MODE == kPgCosine) v = v * nrm[0][lr] * nrm[1][lc];
        if (zero_diag && gi == gj) v = 0.f;
        out[gi * M + gj] = pg_out<T, float>(v);
      }
}

template <typename T, int MODE>
void launch_pairwise_gemm_h16(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, bool zero_diag) {
  const int64_t N = x.size(0), M = y.size(0), D = x.size(1);
  const int64_t tiles_m = (N + kPhT - 1) / kPhT, tiles_n = (M + kPhT - 1) / kPhT, nwg = tiles_m * tiles_n;
  TORCH_CHECK(nwg < (int64_t(1) << 31), "pairwise_gemm: output too large");
  const auto* xp = reinterpret_cast<const T*>(x.data_ptr());
  const auto* yp = reinterpret_cast<const T*>(y.data_ptr());
  auto* op = reinterpret_cast<T*>(out.data_ptr());
  const bool vec = D % 8 == 0 && reinterpret_cast<uintptr_t>(xp) % 16 == 0 && reinterpret_cast<uintptr_t>(yp) % 16 == 0;
  // cosine: fp32 row norms by one ATen reduction per operand (vector_norm accumulates 16-bit inputs in fp32)
  at::Tensor xn, yn;
  if (MODE == kPgCosine) {
    xn = at::linalg_vector_norm(x, 2, at::IntArrayRef{1}, false, at::kFloat);
    yn = at::linalg_vector_norm(y, 2, at::IntArrayRef{1}, false, at::kFloat);
  }
  const float* xnp = MODE == kPgCosine ? xn.data_ptr<float>() : nullptr;
  const float* ynp = MODE == kPgCosine ? yn.data_ptr<float>() : nullptr;
  if (vec)
    hipLaunchKernelGGL((pairwise_gemm_h16_kernel<T, MODE, true>), dim3(static_cast<unsigned>(nwg)), kPhThreads, 0, stream(), xp, yp, N, M,
                       D, static_cast<int>(tiles_n), zero_diag, op, xnp, ynp);
  else
    hipLaunchKernelGGL((pairwise_gemm_h16_kernel<T, MODE, false>), dim3(static_cast<unsigned>(nwg)), kPhThreads, 0, stream(), xp, yp, N, M,
                       D, static_cast<int>(tiles_n), zero_diag, op, xnp, ynp);
}

// ------------------------------------------------------------------------------------ fp32 on f16 matrix cores (x3)
// fp32 linear / cosine / MiFID row max at large shapes.  gfx950's fp32 MFMA rate is a sixteenth of its f16 rate, and
// hipBLASLt's fp32 GEMM reaches ~110 TFLOP/s there.  Here every fp32 row is split into two f16 planes: t = x·2^s
// (s per row: the row max lands in [2^14, 2^15), so nothing overflows and the planes stay normal for every element
// within 2^-18 of the row max), hi = f16(t), lo = f16(t - hi): hi + lo carries 22 of t's 24 bits.  The dot product
// is hi·hi + hi·lo + lo·hi (three v_mfma_f32_16x16x32_f16 per fragment, exact f16 products, fp32 accumulation);
// the dropped lo·lo term is below 2^-22 of |x||y| -- under fp32's own rounding of a K-deep sum.  The split runs once
// per operand (x3_split_kernel: packed [row][k/32][hi 32 | lo 32] planes, the same bytes as the fp32 input) and the
// GEMM reuses the 16-bit kernel's 128 x 128 tiles: one 64-element LDS row slice holds 32 k of both planes.
// Output: ldexp(acc, -(s_x + s_y)) (linear) or acc · f_x · f_y with f = 1 / |t| (cosine / |cos| row max).
// Non-finite rows (inf / NaN) set a flag; linear mode then reruns the exact fp32 MFMA kernel on device (its run_if).
constexpr int kX3K = 32;  // real k per slice (64 halves: hi | lo)

__global__ __launch_bounds__(256) void x3_split_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t N, int64_t Np,
                                                       int64_t M, int64_t D, int64_t Dp, __half* __restrict__ px, __half* __restrict__ py,
                                                       int* __restrict__ shift, float* __restrict__ finv, int* __restrict__ nonfinite) {
  const int lane = threadIdx.x & 63;
  const int64_t grow = blockIdx.x * 4 + (threadIdx.x >> 6);  // rows [0, Np) of x, then [Np, Np + Mp) of y
  const bool is_x = grow < Np;
  const int64_t row = is_x ? grow : grow - Np, nrows = is_x ? N : M;
  const float* __restrict__ src = is_x ? x : y;
  __half* __restrict__ dst = (is_x ? px : py) + row * 2 * Dp;
  float mx = 0.f;
  if (row < nrows)
    for (int64_t k = lane; k < D; k += 64) mx = fmaxf(mx, fabsf(src[row * D + k]));
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
  const bool fin = mx <= 3.4028235e38f;  // false for inf and NaN (fmaxf drops NaN: checked below per element)
  int e = 0;
  if (fin && mx > 0.f) frexpf(mx, &e);
  const int s = fin && mx > 0.f ? 15 - e : 0;
  float ss = 0.f;
  bool bad = !fin;
  for (int64_t k = lane; k < Dp; k += 64) {
    const float v = (row < nrows && k < D) ? src[row * D + k] : 0.f;
    bad |= v != v;
    const float t = ldexpf(v, s);
    const __half h = __float2half_rn(t);
    const __half l = __float2half_rn(t - __half2float(h));
    ss = fmaf(t, t, ss);
    dst[(k >> 5) * 64 + (k & 31)] = h;
    dst[(k >> 5) * 64 + 32 + (k & 31)] = l;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) ss += __shfl_xor(ss, off, kWave);
  const bool any_bad = __any(bad);
  if (lane == 0) {
    shift[grow] = s;
    finv[grow] = 1.f / sqrtf(ss);
    if (any_bad && row < nrows) nonfinite[0] = 1;
  }
}

// The x3 tile core shared by the pairwise forms, MiFID's row max and KID's polynomial sums: a 128 x 128 block of
// packed-plane dot products on 4 waves (64 x 64 each, 4 x 4 MFMA tiles).  ``xrow(r)`` / ``yrow(r)`` give the packed row
// of tile row r (nullptr: a zero row -- KID's gathered subsets end mid-tile); slices of 32 k (64 halves) are double-
// buffered through LDS with the next slice in registers.
typedef __half X3Lds[2][2][kPhT * kPhLd];
template <bool ZERO_ROWS, typename RowA, typename RowB>
__device__ __forceinline__ void x3_tile_core(RowA xrow, RowB yrow, int nk, X3Lds& lds, ph_acc4 (&acc)[4][4]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const __half* xr[4];
  const __half* yr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xr[i] = xrow((tid >> 3) + 32 * i);
    yr[i] = yrow((tid >> 3) + 32 * i);
  }
  ph_frag8 rx[4], ry[4];
  auto load = [&](int64_t s) {  // slice s: 64 halves = 128 B per row, 8 lanes per row
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t off = s * 64 + 8 * (tid & 7);
      if constexpr (ZERO_ROWS) {
        const ph_frag8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        rx[i] = xr[i] != nullptr ? *reinterpret_cast<const ph_frag8*>(xr[i] + off) : z;
        ry[i] = yr[i] != nullptr ? *reinterpret_cast<const ph_frag8*>(yr[i] + off) : z;
      } else {
        rx[i] = *reinterpret_cast<const ph_frag8*>(xr[i] + off);
        ry[i] = *reinterpret_cast<const ph_frag8*>(yr[i] + off);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i, kk = 8 * (tid & 7);
      *reinterpret_cast<ph_frag8*>(reinterpret_cast<short*>(lds[buf][0]) + r * kPhLd + kk) = rx[i];
      *reinterpret_cast<ph_frag8*>(reinterpret_cast<short*>(lds[buf][1]) + r * kPhLd + kk) = ry[i];
    }
  };
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ph_acc4{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load(s + 1);
    const short* A = reinterpret_cast<const short*>(lds[buf][0]);
    const short* B = reinterpret_cast<const short*>(lds[buf][1]);
    ph_frag8 ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = *reinterpret_cast<const ph_frag8*>(A + (wr * 64 + 16 * i + fr) * kPhLd + fk);
      bh[i] = *reinterpret_cast<const ph_frag8*>(B + (wc * 64 + 16 * i + fr) * kPhLd + fk);
      al[i] = *reinterpret_cast<const ph_frag8*>(A + (wr * 64 + 16 * i + fr) * kPhLd + 32 + fk);
      bl[i] = *reinterpret_cast<const ph_frag8*>(B + (wc * 64 + 16 * i + fr) * kPhLd + 32 + fk);
    }
    // the small terms first: hi·lo and lo·hi, then hi·hi (16 independent accumulators between reuses)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = ph_mma<__half>(ah[i], bl[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = ph_mma<__half>(al[i], bh[j], acc[i][j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = ph_mma<__half>(ah[i], bh[j], acc[i][j]);
    if (s + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
}

template <int MODE>
__global__ __launch_bounds__(kPhThreads, 2) void pairwise_gemm_x3_kernel(const __half* __restrict__ x, const __half* __restrict__ y, int64_t N,
                                                                         int64_t M, int64_t Dp, int tiles_n, bool zero_diag,
                                                                         float* __restrict__ out, const int* __restrict__ xs_shift,
                                                                         const int* __restrict__ ys_shift, const float* __restrict__ xs_f,
                                                                         const float* __restrict__ ys_f) {
  __shared__ __attribute__((aligned(16))) X3Lds lds;  // [buffer][x | y][row * kPhLd + (hi 32 | lo 32)]
  __shared__ float fac[2][kPhT];
  __shared__ int sh[2][kPhT];
  const int64_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int64_t row0 = (id / tiles_n) * kPhT, col0 = (id % tiles_n) * kPhT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane & 15;
  const int64_t ld = 2 * Dp;  // halves per packed row; rows are padded to the tile (zeros), so no bounds checks
  ph_acc4 acc[4][4];
  x3_tile_core<false>([&](int r) { return x + (row0 + r) * ld; }, [&](int r) { return y + (col0 + r) * ld; },
                      static_cast<int>(Dp / kX3K), lds, acc);
  {
    const int64_t g = tid < kPhT ? row0 + tid : col0 + (tid - kPhT);
    fac[tid >> 7][tid & 127] = tid < kPhT ? xs_f[g] : ys_f[g];
    sh[tid >> 7][tid & 127] = tid < kPhT ? xs_shift[g] : ys_shift[g];
    __syncthreads();
  }
  if constexpr (MODE == kPgAbsCosMax) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 64 + 16 * i + (lane >> 4) * 4 + r;
        const int64_t gi = row0 + lr;
        float mv = -1.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int lc = wc * 64 + 16 * j + fr;
          if (col0 + lc < M) mv = fmaxf(mv, fabsf(acc[i][j][r] * fac[0][lr] * fac[1][lc]));
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) mv = fmaxf(mv, __shfl_xor(mv, off, kWave));
        if (fr == 0 && gi < N && mv >= 0.f) atomicMax(reinterpret_cast<unsigned int*>(out) + gi, __float_as_uint(mv));
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 64 + 16 * i + (lane >> 4) * 4 + r, lc = wc * 64 + 16 * j + fr;
        const int64_t gi = row0 + lr, gj = col0 + lc;
        if (gi >= N || gj >= M) continue;
        float v = acc[i][j][r];
        if constexpr (MODE == kPgCosine) v = v * fac[0][lr] * fac[1][lc];
        else v = ldexpf(v, -(sh[0][lr] + sh[1][lc]));
        if (zero_diag && gi == gj) v = 0.f;
        out[gi * M + gj] = v;
      }
}

// x3 route: fp32, >= 256 128 x 128 output tiles (the host decides; see pairwise_gemm / pairwise_abs_cos_rowmax)
inline bool x3_eligible(const at::Tensor& x, const at::Tensor& y) {
  return x.scalar_type() == at::kFloat && ((x.size(0) + kPhT - 1) / kPhT) * ((y.size(0) + kPhT - 1) / kPhT) >= 256 &&
         !std::getenv("TMX_PAIRWISE_X3_OFF");
}

// out: [N, M] fp32 (linear / cosine) or [N] row maxima (kPgAbsCosMax, zero-initialised)
template <int MODE>
void launch_pairwise_gemm_x3(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, bool zero_diag) {
  const int64_t N = x.size(0), M = y.size(0), D = x.size(1);
  const int64_t Np = (N + kPhT - 1) / kPhT * kPhT, Mp = (M + kPhT - 1) / kPhT * kPhT, Dp = (D + kX3K - 1) / kX3K * kX3K;
  const int64_t tiles_n = Mp / kPhT, nwg = (Np / kPhT) * tiles_n;
  TORCH_CHECK(nwg < (int64_t(1) << 31), "pairwise_gemm: output too large");
  auto px = at::empty({Np, 2 * Dp}, x.options().dtype(at::kHalf));
  auto py = at::empty({Mp, 2 * Dp}, x.options().dtype(at::kHalf));
  auto shift = at::empty({Np + Mp}, x.options().dtype(at::kInt));
  auto finv = at::empty({Np + Mp}, x.options());
  auto flag = at::zeros({1}, x.options().dtype(at::kInt));
  const float* xp = x.data_ptr<float>();
  const float* yp = y.data_ptr<float>();
  hipLaunchKernelGGL(x3_split_kernel, dim3(static_cast<unsigned>((Np + Mp) / 4)), 256, 0, stream(), xp, yp, N, Np, M, D, Dp,
                     reinterpret_cast<__half*>(px.data_ptr()), reinterpret_cast<__half*>(py.data_ptr()), shift.data_ptr<int>(),
                     finv.data_ptr<float>(), flag.data_ptr<int>());
  const int* shp = shift.data_ptr<int>();
  const float* fp = finv.data_ptr<float>();
  hipLaunchKernelGGL((pairwise_gemm_x3_kernel<MODE>), dim3(static_cast<unsigned>(nwg)), kPhThreads, 0, stream(),
                     reinterpret_cast<const __half*>(px.data_ptr()), reinterpret_cast<const __half*>(py.data_ptr()), N, M, Dp,
                     static_cast<int>(tiles_n), zero_diag, out.data_ptr<float>(), shp, shp + Np, fp, fp + Np);
  if constexpr (MODE == kPgLinear) {
    // inf / NaN inputs: the exact fp32 kernel redoes the product on device (a no-op grid otherwise)
    const int64_t t64 = (M + kPgT - 1) / kPgT, nwg64 = ((N + kPgT - 1) / kPgT) * t64;
    const bool vec = D % 8 == 0 && reinterpret_cast<uintptr_t>(xp) % 16 == 0 && reinterpret_cast<uintptr_t>(yp) % 16 == 0;
    if (vec)
      hipLaunchKernelGGL((pairwise_gemm_kernel<float, float, kPgLinear, true>), dim3(static_cast<unsigned>(nwg64)), kPgThreads, 0, stream(),
                         xp, yp, N, M, D, static_cast<int>(t64), zero_diag, out.data_ptr<float>(), nullptr, flag.data_ptr<int>());
    else
      hipLaunchKernelGGL((pairwise_gemm_kernel<float, float, kPgLinear, false>), dim3(static_cast<unsigned>(nwg64)), kPgThreads, 0, stream(),
                         xp, yp, N, M, D, static_cast<int>(t64), zero_diag, out.data_ptr<float>(), nullptr, flag.data_ptr<int>());
  }
}

template <typename T, typename Acc, int MODE>
void launch_pairwise_gemm(const at::Tensor& x, const at::Tensor& y, at::Tensor& out, bool zero_diag) {
  const int64_t N = x.size(0), M = y.size(0), D = x.size(1);
  const int64_t tiles_m = (N + kPgT - 1) / kPgT, tiles_n = (M + kPgT - 1) / kPgT;
  const int64_t nwg = tiles_m * tiles_n;
  TORCH_CHECK(nwg < (int64_t(1) << 31) && tiles_n < (int64_t(1) << 31), "pairwise_gemm: output too large");
  const auto* xp = reinterpret_cast<const T*>(x.data_ptr());
  const auto* yp = reinterpret_cast<const T*>(y.data_ptr());
  auto* op = reinterpret_cast<T*>(out.data_ptr());
  constexpr int kpt = pg_k<Acc>() / 4, align = kpt * sizeof(T) < 16 ? kpt * sizeof(T) : 16;
  const bool vec = D % kpt == 0 && reinterpret_cast<uintptr_t>(xp) % align == 0 && reinterpret_cast<uintptr_t>(yp) % align == 0;
  if (vec)
    hipLaunchKernelGGL((pairwise_gemm_kernel<T, Acc, MODE, true>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), xp, yp, N, M, D,
                       static_cast<int>(tiles_n), zero_diag, op);
  else
    hipLaunchKernelGGL((pairwise_gemm_kernel<T, Acc, MODE, false>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), xp, yp, N, M, D,
                       static_cast<int>(tiles_n), zero_diag, op);
}

// ------------------------------------------------------------------------------- KID polynomial MMD sums (K20)
// One launch per subset of the reference's ``poly_mmd`` (``image/kid.py``: three GEMMs f @ gᵀ, then
// (· gamma + coef) ** degree, diagonal and full sums -- about twenty kernels and three m x m matrices per subset).
// Here the three products (real·real, fake·fake, real·fake) are tiles of one grid; rows are gathered through the
// subset index vectors while they are staged (no subset copies), and each tile's epilogue raises its dot products to
// the polynomial and folds them (diagonal left out of the two self terms) into one fp64 atomic per workgroup.
template <typename T, typename Acc, bool VEC>
__global__ __launch_bounds__(kPgThreads) void kid_poly_kernel(const T* __restrict__ real, const T* __restrict__ fake,
                                                              const int64_t* __restrict__ idx_r, const int64_t* __restrict__ idx_f,
                                                              int64_t m, int64_t D, int tiles, int degree, double gamma, double coef,
                                                              double* __restrict__ sums) {
  using Mma = PgMma<Acc>;
  constexpr int kPgK = pg_k<Acc>(), KPT = kPgK / 4;
  __shared__ Acc xs[2][kPgK][kPgT + kPgPad];
  __shared__ Acc ys[2][kPgK][kPgT + kPgPad];
  __shared__ double red[kPgThreads / kWave];
  const int64_t per = static_cast<int64_t>(tiles) * tiles;
  const int64_t sub = blockIdx.x / (3 * per);  // subset
  const int prob = static_cast<int>((blockIdx.x / per) % 3);  // 0: real x real, 1: fake x fake, 2: real x fake
  const int64_t t = blockIdx.x % per;
  const int64_t row0 = (t / tiles) * kPgT, col0 = (t % tiles) * kPgT;
  const T* A = prob == 1 ? fake : real;
  const T* B = prob == 0 ? real : fake;
  const int64_t* ia = (prob == 1 ? idx_f : idx_r) + sub * m;
  const int64_t* ib = (prob == 0 ? idx_r : idx_f) + sub * m;
  sums += 3 * sub;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int sr = tid >> 2, sk = (tid & 3) * KPT;
  const int64_t ra_row = row0 + sr < m ? ia[row0 + sr] : 0, rb_row = col0 + sr < m ? ib[col0 + sr] : 0;
  Acc rx[KPT], ry[KPT];
  auto load = [&](int64_t k0) {
    // a row outside the subset (row0 + sr >= m) loads zeros: nrows = 0 masks it
    pg_load<T, Acc, KPT, VEC>(A, ra_row, row0 + sr < m ? ra_row + 1 : 0, k0 + sk, D, rx);
    pg_load<T, Acc, KPT, VEC>(B, rb_row, col0 + sr < m ? rb_row + 1 : 0, k0 + sk, D, ry);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      xs[buf][sk + i][sr] = rx[i];
      ys[buf][sk + i][sr] = ry[i];
    }
  };
  typename Mma::V acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = typename Mma::V{0, 0, 0, 0};
  const int nk = static_cast<int>((D + kPgK - 1) / kPgK);
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nk; ++s) {
    const int buf = s & 1;
    if (s + 1 < nk) load(static_cast<int64_t>(s + 1) * kPgK);
#pragma unroll
    for (int kk = 0; kk < kPgK; kk += 4) {
      Acc a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = xs[buf][kk + fk][wr * 32 + 16 * i + fr];
        b[i] = ys[buf][kk + fk][wc * 32 + 16 * i + fr];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mma::mma(a[i], b[j], acc[i][j]);
    }
    if (s + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  const Acc g = static_cast<Acc>(gamma), c0 = static_cast<Acc>(coef);
  double part = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gi = row0 + wr * 32 + 16 * i + Mma::row(lane, r), gj = col0 + wc * 32 + 16 * j + fr;
        if (gi >= m || gj >= m || (prob < 2 && gi == gj)) continue;
        const Acc base = acc[i][j][r] * g + c0;  // the reference's (f @ gᵀ * gamma + coef)
        Acc p = base;
        for (int e = 1; e < degree; ++e) p = p * base;  // ** degree (integer degree >= 1)
        part += static_cast<double>(p);
      }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, kWave);
  if (lane == 0) red[wave] = part;
  __syncthreads();
  if (tid == 0) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < kPgThreads / kWave; ++w) tot += red[w];
    atomicAdd(sums + prob, tot);
  }
}

// KID on the x3 core (fp32 features, round 6): the real and fake features are split once (x3_split_kernel), every
// (subset, product, 128 x 128 tile) block gathers its rows through the subset indices into the shared tile core, and
// the epilogue raises ldexp(acc, -(s_i + s_j)) * gamma + coef to the degree and folds one fp64 atomic per block.
__global__ __launch_bounds__(kPhThreads, 2) void kid_poly_x3_kernel(const __half* __restrict__ pr, const __half* __restrict__ pf,
                                                                    const int* __restrict__ sh_r, const int* __restrict__ sh_f,
                                                                    const int64_t* __restrict__ idx_r, const int64_t* __restrict__ idx_f,
                                                                    int64_t m, int64_t Dp, int tiles, int degree, double gamma, double coef,
                                                                    double* __restrict__ sums) {
  __shared__ __attribute__((aligned(16))) X3Lds lds;
  __shared__ int sh[2][kPhT];
  __shared__ double red[kPhThreads / kWave];
  const int64_t per = static_cast<int64_t>(tiles) * tiles;
  const int64_t sub = blockIdx.x / (3 * per);
  const int prob = static_cast<int>((blockIdx.x / per) % 3);  // 0: real x real, 1: fake x fake, 2: real x fake
  const int64_t t = blockIdx.x % per;
  const int64_t row0 = (t / tiles) * kPhT, col0 = (t % tiles) * kPhT;
  const __half* A = prob == 1 ? pf : pr;
  const __half* B = prob == 0 ? pr : pf;
  const int* sa = prob == 1 ? sh_f : sh_r;
  const int* sb = prob == 0 ? sh_r : sh_f;
  const int64_t* ia = (prob == 1 ? idx_f : idx_r) + sub * m;
  const int64_t* ib = (prob == 0 ? idx_r : idx_f) + sub * m;
  const int64_t ld = 2 * Dp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, fr = lane & 15;
  ph_acc4 acc[4][4];
  x3_tile_core<true>([&](int r) -> const __half* { return row0 + r < m ? A + ia[row0 + r] * ld : nullptr; },
                     [&](int r) -> const __half* { return col0 + r < m ? B + ib[col0 + r] * ld : nullptr; },
                     static_cast<int>(Dp / kX3K), lds, acc);
  {
    const int64_t g = tid < kPhT ? row0 + tid : col0 + (tid - kPhT);
    sh[tid >> 7][tid & 127] = g < m ? (tid < kPhT ? sa[ia[g]] : sb[ib[g]]) : 0;
    __syncthreads();
  }
  const float gf = static_cast<float>(gamma), cf = static_cast<float>(coef);
  double part = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 64 + 16 * i + (lane >> 4) * 4 + r, lc = wc * 64 + 16 * j + fr;
        const int64_t gi = row0 + lr, gj = col0 + lc;
        if (gi >= m || gj >= m || (prob < 2 && gi == gj)) continue;
        const float base = ldexpf(acc[i][j][r], -(sh[0][lr] + sh[1][lc])) * gf + cf;  // (f @ gᵀ * gamma + coef)
        float p = base;
        for (int e = 1; e < degree; ++e) p = p * base;
        part += static_cast<double>(p);
      }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, kWave);
  if (lane == 0) red[wave] = part;
  __syncthreads();
  if (tid == 0) {
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < kPhThreads / kWave; ++w) tot += red[w];
    atomicAdd(sums + 3 * sub + prob, tot);
  }
}

// [S, 3] fp64 per subset s: Σ_{i != j} k(r_i, r_j), Σ_{i != j} k(f_i, f_j), Σ k(r_i, f_j) over real[idx_r[s]],
// fake[idx_f[s]] (idx [S, m], or [m] for one subset -> [3]); every subset in one launch
at::Tensor kid_poly_sums(const at::Tensor& real_in, const at::Tensor& fake_in, const at::Tensor& idx_r_in, const at::Tensor& idx_f_in,
                         int64_t degree, double gamma, double coef) {
  TORCH_CHECK(real_in.is_cuda() && fake_in.is_cuda(), "kid_poly_sums: expected GPU features");
  TORCH_CHECK(real_in.dim() == 2 && fake_in.dim() == 2 && real_in.size(1) == fake_in.size(1), "kid_poly_sums: expected [n, d] features");
  TORCH_CHECK(real_in.scalar_type() == fake_in.scalar_type(), "kid_poly_sums: dtype mismatch");
  TORCH_CHECK(degree >= 1, "kid_poly_sums: degree must be >= 1");
  const at::DeviceGuard guard(real_in.device());
  auto real = real_in.contiguous();
  auto fake = fake_in.contiguous();
  // the kernel gathers rows through the indices: bounds are checked on the host before any launch (a device index
  // costs one synchronising copy; KernelInceptionDistance passes host randperm slices, as the reference draws them)
  const at::Tensor hr = idx_r_in.to(at::kCPU, at::kLong).contiguous(), hf = idx_f_in.to(at::kCPU, at::kLong).contiguous();
  if (hr.numel() > 0) {
    TORCH_CHECK(hr.min().item<int64_t>() >= 0 && hr.max().item<int64_t>() < real_in.size(0), "kid_poly_sums: real subset index out of range");
    TORCH_CHECK(hf.min().item<int64_t>() >= 0 && hf.max().item<int64_t>() < fake_in.size(0), "kid_poly_sums: fake subset index out of range");
  }
  auto idx_r = hr.to(real.device());
  auto idx_f = hf.to(real.device());
  TORCH_CHECK(idx_r_in.dim() <= 2 && idx_r_in.sizes() == idx_f_in.sizes(), "kid_poly_sums: index shapes differ");
  const bool batched = idx_r_in.dim() == 2;
  const int64_t S = batched ? idx_r_in.size(0) : 1, m = batched ? idx_r_in.size(1) : idx_r_in.numel(), D = real.size(1);
  auto sums = at::zeros(batched ? at::IntArrayRef{S, 3} : at::IntArrayRef{3}, real.options().dtype(at::kDouble));
  if (m == 0 || D == 0 || S == 0) return sums;
  if (real.scalar_type() == at::kFloat && D >= 256 && !std::getenv("TMX_PAIRWISE_X3_OFF")) {
    // fp32 Inception-depth features: the x3 route (both feature sets split once, 128 x 128 tiles)
    const int64_t Nr = real.size(0), Nf = fake.size(0), Dp = (D + kX3K - 1) / kX3K * kX3K;
    const int64_t Nrp = (Nr + 3) / 4 * 4, Nfp = (Nf + 3) / 4 * 4;
    auto pr = at::empty({Nrp, 2 * Dp}, real.options().dtype(at::kHalf));
    auto pf = at::empty({Nfp, 2 * Dp}, real.options().dtype(at::kHalf));
    auto shift = at::empty({Nrp + Nfp}, real.options().dtype(at::kInt));
    auto finv = at::empty({Nrp + Nfp}, real.options());
    auto flag = at::zeros({1}, real.options().dtype(at::kInt));
    hipLaunchKernelGGL(x3_split_kernel, dim3(static_cast<unsigned>((Nrp + Nfp) / 4)), 256, 0, stream(), real.data_ptr<float>(),
                       fake.data_ptr<float>(), Nr, Nrp, Nf, D, Dp, reinterpret_cast<__half*>(pr.data_ptr()),
                       reinterpret_cast<__half*>(pf.data_ptr()), shift.data_ptr<int>(), finv.data_ptr<float>(), flag.data_ptr<int>());
    TMX_LAUNCH_CHECK();
    const int tiles = static_cast<int>((m + kPhT - 1) / kPhT);
    const int64_t nwg = 3 * S * static_cast<int64_t>(tiles) * tiles;
    TORCH_CHECK(nwg < (int64_t(1) << 31), "kid_poly_sums: subset too large");
    hipLaunchKernelGGL(kid_poly_x3_kernel, dim3(static_cast<unsigned>(nwg)), kPhThreads, 0, stream(),
                       reinterpret_cast<const __half*>(pr.data_ptr()), reinterpret_cast<const __half*>(pf.data_ptr()), shift.data_ptr<int>(),
                       shift.data_ptr<int>() + Nrp, idx_r.data_ptr<int64_t>(), idx_f.data_ptr<int64_t>(), m, Dp, tiles, static_cast<int>(degree),
                       gamma, coef, sums.data_ptr<double>());
    TMX_LAUNCH_CHECK();
    return sums;
  }
  const int tiles = static_cast<int>((m + kPgT - 1) / kPgT);
  const int64_t nwg = 3 * S * static_cast<int64_t>(tiles) * tiles;
  TORCH_CHECK(nwg < (int64_t(1) << 31), "kid_poly_sums: subset too large");
  TMX_DISPATCH_FLOAT(real.scalar_type(), "kid_poly_sums", [&] {
    constexpr bool kF64 = std::is_same<scalar_t, double>::value;
    using Acc = typename std::conditional<kF64, double, float>::type;
    constexpr int kpt = pg_k<Acc>() / 4, align = kpt * sizeof(scalar_t) < 16 ? kpt * sizeof(scalar_t) : 16;
    const auto* rp = reinterpret_cast<const scalar_t*>(real.data_ptr());
    const auto* fp = reinterpret_cast<const scalar_t*>(fake.data_ptr());
    const bool vec = D % kpt == 0 && reinterpret_cast<uintptr_t>(rp) % align == 0 && reinterpret_cast<uintptr_t>(fp) % align == 0;
    if (vec)
      hipLaunchKernelGGL((kid_poly_kernel<scalar_t, Acc, true>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), rp, fp,
                         idx_r.data_ptr<int64_t>(), idx_f.data_ptr<int64_t>(), m, D, tiles, static_cast<int>(degree), gamma, coef,
                         sums.data_ptr<double>());
    else
      hipLaunchKernelGGL((kid_poly_kernel<scalar_t, Acc, false>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), rp, fp,
                         idx_r.data_ptr<int64_t>(), idx_f.data_ptr<int64_t>(), m, D, tiles, static_cast<int>(degree), gamma, coef,
                         sums.data_ptr<double>());
  });
  TMX_LAUNCH_CHECK();
  return sums;
}

// ------------------------------------------------------------------------------- FID moments
// gram += xᵀx and colsum += Σ_b x[b] in fp64 for a feature batch x [B, F] of any float dtype (reference
// ``image/fid.py``: ``features.double()``, ``sum(dim=0)`` and ``cov_sum.addmm(features.t(), features)`` -- a converted
// copy, a new F x F fp64 matrix per update and both triangles computed).  Here one launch, in place: only the tiles
// with tm <= tn of the 64 x 64 tiling are computed (the Gram is symmetric), each by one workgroup on
// v_mfma_f64_16x16x4_f64 from 16-deep batch slices converted to fp64 on the way into LDS (the batch dimension is the
// GEMM's K; the staging layout is the k-major one of the pairwise kernel, reached with row-contiguous loads).  An
// off-diagonal tile adds itself at (tm, tn) and, transposed through LDS for coalesced rows, at (tn, tm); diagonal tiles
// also fold their feature sums.  Every Gram element has exactly one writer: plain read-modify-writes, no atomics.
template <typename T, bool VEC>
__global__ __launch_bounds__(kPgThreads) void fid_gram_kernel(const T* __restrict__ x, int64_t B, int64_t F, int tiles,
                                                              double* __restrict__ gram, double* __restrict__ colsum) {
  using Mma = PgMma<double>;
  constexpr int K = 16, kLd = kPgT + kPgPad, kTld = kPgT + 1;
  static_assert(2 * 2 * K * kLd >= kPgT * kTld, "the transpose tile reuses the staging buffers");
  __shared__ double buf[2 * 2 * K * kLd];
  __shared__ double csum[kPgThreads / kWave][kPgT];
  auto xs = [&](int b, int k, int r) -> double& { return buf[((b * 2 + 0) * K + k) * kLd + r]; };
  auto ys = [&](int b, int k, int r) -> double& { return buf[((b * 2 + 1) * K + k) * kLd + r]; };
  const int64_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  int64_t id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int tm = 0;
  while (id >= tiles - tm) {  // upper-triangular row tm holds tiles - tm tiles (tiles <= 64 for F <= 4096)
    id -= tiles - tm;
    ++tm;
  }
  const int tn = tm + static_cast<int>(id);
  const int64_t f0 = static_cast<int64_t>(tm) * kPgT, g0 = static_cast<int64_t>(tn) * kPgT;
  const bool diag = tm == tn;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int sb = tid >> 4, sf = 4 * (tid & 15);  // staging: batch row sb of the slice, features [sf, sf + 4)
  // two register sets: slices s + 1 and s + 2 are in flight while slice s is multiplied (a batch of a few hundred
  // rows is only ~16 slices, and one slice of prefetch left each slice waiting on its loads)
  double ra[2][4], rb[2][4], cs[4] = {0.0, 0.0, 0.0, 0.0};
  auto load = [&](int64_t b0, double (&pa)[4], double (&pb)[4]) {
    pg_load<T, double, 4, VEC>(x, b0 + sb, B, f0 + sf, F, pa);
    pg_load<T, double, 4, VEC>(x, b0 + sb, B, g0 + sf, F, pb);
    if (diag) {
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[e] += pa[e];
    }
  };
  auto store = [&](int b, const double (&pa)[4], const double (&pb)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xs(b, sb, sf + e) = pa[e];
      ys(b, sb, sf + e) = pb[e];
    }
  };
  typename Mma::V acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = typename Mma::V{0, 0, 0, 0};
  const int nk = static_cast<int>((B + K - 1) / K);
  load(0, ra[0], rb[0]);
  store(0, ra[0], rb[0]);
  if (nk > 1) load(K, ra[1], rb[1]);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  auto step = [&](int s, double (&na)[4], double (&nb)[4], const double (&sa)[4], const double (&sb2)[4]) {
    // na / nb: the set that held slice s (already in LDS) takes slice s + 2; sa / sb2 hold slice s + 1
    const int b = s & 1;
    if (s + 2 < nk) load(static_cast<int64_t>(s + 2) * K, na, nb);
#pragma unroll
    for (int kk = 0; kk < K; kk += 4) {
      double a[2], c[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = xs(b, kk + fk, wr * 32 + 16 * i + fr);
        c[i] = ys(b, kk + fk, wc * 32 + 16 * i + fr);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mma::mma(a[i], c[j], acc[i][j]);
    }
    if (s + 1 < nk) store(b ^ 1, sa, sb2);
    __syncthreads();
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, ra[0], rb[0], ra[1], rb[1]);
    if (s + 1 < nk) step(s + 1, ra[1], rb[1], ra[0], rb[0]);
  }
  // (tm, tn): rows f0 + lr, columns g0 + lc; off-diagonal tiles stage the block for the mirrored (tn, tm) rows
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wr * 32 + 16 * i + Mma::row(lane, r), lc = wc * 32 + 16 * j + fr;
        const double v = acc[i][j][r];
        if (f0 + lr < F && g0 + lc < F) gram[(f0 + lr) * F + g0 + lc] += v;
        if (!diag) buf[lc * kTld + lr] = v;  // transposed: row lc of the mirrored block
      }
  if (!diag) {
    __syncthreads();
    for (int e = tid; e < kPgT * kPgT; e += kPgThreads) {
      const int r = e / kPgT, c = e % kPgT;
      if (g0 + r < F && f0 + c < F) gram[(g0 + r) * F + f0 + c] += buf[r * kTld + c];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // the 16 lanes of a wave sharing sf are 16 apart
      cs[e] += __shfl_xor(cs[e], 16, kWave);
      cs[e] += __shfl_xor(cs[e], 32, kWave);
    }
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[wave][sf + e] = cs[e];
    }
    __syncthreads();
    if (tid < kPgT && f0 + tid < F) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < kPgThreads / kWave; ++w) t += csum[w][tid];
      colsum[f0 + tid] += t;
    }
  }
}

template <typename T>
void launch_fid_gram(const at::Tensor& x, at::Tensor& gram, at::Tensor& colsum) {
  const int64_t B = x.size(0), F = x.size(1);
  const int tiles = static_cast<int>((F + kPgT - 1) / kPgT);
  const int64_t nwg = static_cast<int64_t>(tiles) * (tiles + 1) / 2;
  const auto* xp = reinterpret_cast<const T*>(x.data_ptr());
  constexpr int align = 4 * sizeof(T) < 16 ? 4 * sizeof(T) : 16;
  const bool vec = F % 4 == 0 && reinterpret_cast<uintptr_t>(xp) % align == 0;
  if (vec)
    hipLaunchKernelGGL((fid_gram_kernel<T, true>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), xp, B, F, tiles,
                       gram.data_ptr<double>(), colsum.data_ptr<double>());
  else
    hipLaunchKernelGGL((fid_gram_kernel<T, false>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(), xp, B, F, tiles,
                       gram.data_ptr<double>(), colsum.data_ptr<double>());
}

// gram [F, F] += xᵀx, colsum [F] += Σ_b x[b] (fp64 states; x [B, F] fp32 / fp64 / bf16 / fp16)
void fid_gram_update(const at::Tensor& x_in, at::Tensor gram, at::Tensor colsum) {
  TORCH_CHECK(x_in.is_cuda() && gram.is_cuda() && colsum.is_cuda(), "fid_gram_update: expected GPU tensors");
  TORCH_CHECK(x_in.dim() == 2, "fid_gram_update: expected features [B, F]");
  const int64_t F = x_in.size(1);
  TORCH_CHECK(gram.scalar_type() == at::kDouble && colsum.scalar_type() == at::kDouble, "fid_gram_update: fp64 states expected");
  TORCH_CHECK(gram.dim() == 2 && gram.size(0) == F && gram.size(1) == F && gram.is_contiguous(), "fid_gram_update: gram must be a contiguous [F, F]");
  TORCH_CHECK(colsum.dim() == 1 && colsum.size(0) == F && colsum.is_contiguous(), "fid_gram_update: colsum must be a contiguous [F]");
  TORCH_CHECK(F <= 4096 * 4, "fid_gram_update: too many features");
  TORCH_CHECK(x_in.device() == gram.device() && x_in.device() == colsum.device(), "fid_gram_update: device mismatch");
  const at::DeviceGuard guard(x_in.device());
  if (x_in.size(0) == 0 || F == 0) return;
  auto x = x_in.contiguous();
  TMX_DISPATCH_FLOAT(x.scalar_type(), "fid_gram_update", [&] { launch_fid_gram<scalar_t>(x, gram, colsum); });
  TMX_LAUNCH_CHECK();
}

// MiFID's memorization term: for every row of x the largest |cos| against the rows of y (fp32, fp64 for fp64 inputs),
// without the N x M similarity matrix (reference ``image/mifid.py``: normalise, n1 @ n2ᵀ, abs, min of 1 - |cos|)
at::Tensor pairwise_abs_cos_rowmax(const at::Tensor& x_in, const at::Tensor& y_in) {
  TORCH_CHECK(x_in.is_cuda() && y_in.is_cuda(), "pairwise_abs_cos_rowmax: expected GPU tensors");
  TORCH_CHECK(x_in.dim() == 2 && y_in.dim() == 2 && x_in.size(1) == y_in.size(1), "pairwise_abs_cos_rowmax: expected [N,d] and [M,d]");
  TORCH_CHECK(x_in.scalar_type() == y_in.scalar_type(), "pairwise_abs_cos_rowmax: dtype mismatch");
  TORCH_CHECK(y_in.size(0) > 0 && x_in.size(1) > 0, "pairwise_abs_cos_rowmax: empty operand");
  const at::DeviceGuard guard(x_in.device());
  auto x = x_in.contiguous();
  auto y = y_in.contiguous();
  const bool f64 = x.scalar_type() == at::kDouble;
  auto out = at::zeros({x.size(0)}, x.options().dtype(f64 ? at::kDouble : at::kFloat));
  if (x.size(0) == 0) return out;
  const int64_t N = x.size(0), M = y.size(0), D = x.size(1);
  const int64_t tiles_m = (N + kPgT - 1) / kPgT, tiles_n = (M + kPgT - 1) / kPgT, nwg = tiles_m * tiles_n;
  TORCH_CHECK(nwg < (int64_t(1) << 31), "pairwise_abs_cos_rowmax: too large");
  if (x3_eligible(x, y)) {  // fp32 at large shapes: the f16-split matrix-core route
    launch_pairwise_gemm_x3<kPgAbsCosMax>(x, y, out, false);
    TMX_LAUNCH_CHECK();
    return out;
  }
  TMX_DISPATCH_FLOAT(x.scalar_type(), "pairwise_abs_cos_rowmax", [&] {
    constexpr bool kF64 = std::is_same<scalar_t, double>::value;
    using Acc = typename std::conditional<kF64, double, float>::type;
    constexpr int kpt = pg_k<Acc>() / 4, align = kpt * sizeof(scalar_t) < 16 ? kpt * sizeof(scalar_t) : 16;
    const auto* xp = reinterpret_cast<const scalar_t*>(x.data_ptr());
    const auto* yp = reinterpret_cast<const scalar_t*>(y.data_ptr());
    const bool vec = D % kpt == 0 && reinterpret_cast<uintptr_t>(xp) % align == 0 && reinterpret_cast<uintptr_t>(yp) % align == 0;
    if (vec)
      hipLaunchKernelGGL((pairwise_gemm_kernel<scalar_t, Acc, kPgAbsCosMax, true>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(),
                         xp, yp, N, M, D, static_cast<int>(tiles_n), false, static_cast<scalar_t*>(nullptr), out.data_ptr());
    else
      hipLaunchKernelGGL((pairwise_gemm_kernel<scalar_t, Acc, kPgAbsCosMax, false>), dim3(static_cast<unsigned>(nwg)), kPgThreads, 0, stream(),
                         xp, yp, N, M, D, static_cast<int>(tiles_n), false, static_cast<scalar_t*>(nullptr), out.data_ptr());
  });
  TMX_LAUNCH_CHECK();
  return out;
}

// [N, M] in the input dtype; mode 0 linear, 1 cosine, 2 euclidean (fp64 accumulation, as the reference)
at::Tensor pairwise_gemm(const at::Tensor& x_in, const at::Tensor& y_in, int64_t mode, bool zero_diag) {
  TORCH_CHECK(x_in.is_cuda() && y_in.is_cuda(), "pairwise_gemm: expected GPU tensors");
  TORCH_CHECK(x_in.dim() == 2 && y_in.dim() == 2 && x_in.size(1) == y_in.size(1), "pairwise_gemm: expected [N,d] and [M,d]");
  TORCH_CHECK(x_in.scalar_type() == y_in.scalar_type(), "pairwise_gemm: dtype mismatch");
  TORCH_CHECK(mode >= kPgLinear && mode <= kPgEuclid, "pairwise_gemm: bad mode");
  const at::DeviceGuard guard(x_in.device());
  auto x = x_in.contiguous();
  auto y = y_in.contiguous();
  auto out = at::empty({x.size(0), y.size(0)}, x.options());
  if (x.size(0) == 0 || y.size(0) == 0) return out;
  TMX_DISPATCH_FLOAT(x.scalar_type(), "pairwise_gemm", [&] {
    constexpr bool kF64 = std::is_same<scalar_t, double>::value;
    using AccLC = typename std::conditional<kF64, double, float>::type;
    constexpr bool kH16 = std::is_same<scalar_t, __hip_bfloat16>::value || std::is_same<scalar_t, __half>::value;
    // 16-bit linear / cosine with at least 256 128 x 128 tiles: the 16-bit MFMA kernel
    const bool h16 = kH16 && mode != kPgEuclid && ((x.size(0) + kPhT - 1) / kPhT) * ((y.size(0) + kPhT - 1) / kPhT) >= 256;
    if constexpr (kH16) {
      if (h16) {
        if (mode == kPgLinear) launch_pairwise_gemm_h16<scalar_t, kPgLinear>(x, y, out, zero_diag);
        else launch_pairwise_gemm_h16<scalar_t, kPgCosine>(x, y, out, zero_diag);
        return;
      }
    }
    if constexpr (std::is_same<scalar_t, float>::value) {
      if (mode != kPgEuclid && x3_eligible(x, y)) {  // fp32 at large shapes: the f16-split matrix-core route
        if (mode == kPgLinear) launch_pairwise_gemm_x3<kPgLinear>(x, y, out, zero_diag);
        else launch_pairwise_gemm_x3<kPgCosine>(x, y, out, zero_diag);
        return;
      }
    }
    if (mode == kPgLinear) launch_pairwise_gemm<scalar_t, AccLC, kPgLinear>(x, y, out, zero_diag);
    else if (mode == kPgCosine) launch_pairwise_gemm<scalar_t, AccLC, kPgCosine>(x, y, out, zero_diag);
    else launch_pairwise_gemm<scalar_t, double, kPgEuclid>(x, y, out, zero_diag);
  });
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("pairwise_lp(Tensor x, Tensor y, float p, bool fp64_acc) -> Tensor");
  m.def("pairwise_gemm(Tensor x, Tensor y, int mode, bool zero_diag) -> Tensor");
  m.def("fid_gram_update(Tensor x, Tensor(a!) gram, Tensor(b!) colsum) -> ()");
  m.def("pairwise_abs_cos_rowmax(Tensor x, Tensor y) -> Tensor");
  m.def("kid_poly_sums(Tensor real, Tensor fake, Tensor idx_r, Tensor idx_f, int degree, float gamma, float coef) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("pairwise_lp", &tmx::pairwise_lp);
  m.impl("pairwise_gemm", &tmx::pairwise_gemm);
  m.impl("fid_gram_update", &tmx::fid_gram_update);
  m.impl("kid_poly_sums", &tmx::kid_poly_sums);
  m.impl("pairwise_abs_cos_rowmax", &tmx::pairwise_abs_cos_rowmax);
}
