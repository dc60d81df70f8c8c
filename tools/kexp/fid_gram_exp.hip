// ``fid_moments_update`` — FID's fp64 moment states in one launch (reference image/fid.py:322-338:
// ``features.double()``, ``features.sum(0)``, ``features.t().mm(features)`` — three launches, an fp64 copy of the batch
// and the full D x D GEMM).
//
// The Gram XᵀX is symmetric, so only the upper-triangular 64 x 64 tiles are computed (one wave per tile and batch
// split, 4 x 4 fp64 MFMA 16x16x4 blocks, K = batch rows four at a time), each added into its tile and mirrored into the
// lower one: half the FLOPs of the GEMM.  fp32 features are widened to fp64 in registers (exact); the diagonal-tile
// waves also fold their 64 column sums.  fp64 accumulation order differs from rocBLAS's (~1e-16 relative).
#include "common.h"

namespace tmx {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// 64 x 64 tile per wave (4 x 4 MFMA blocks, 16 accumulators of 4 fp64 = 128 VGPRs), batch rows split into S chunks so
// the upper triangle (T (T + 1) / 2 tiles, T = D / 64) times S fills the chip; partial tiles go out with fp64 atomic
// adds (run-to-run order differences ~1e-16 relative).
__global__ __launch_bounds__(256) void fid_gram_kernel(const float* __restrict__ X, int64_t N, int D, int T, int64_t tiles, int S,
                                                      double* __restrict__ fsum, double* __restrict__ cov) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = blockIdx.x * 4 + threadIdx.x / 64;
  if (wv >= tiles * S) return;
  const int64_t w = wv / S;
  const int split = static_cast<int>(wv % S);
  // w -> (ti, tj), ti <= tj, row-major over the upper triangle of T x T tiles
  int ti = 0;
  int64_t rem = w;
  while (rem >= T - ti) {
    rem -= T - ti;
    ++ti;
  }
  const int tj = ti + static_cast<int>(rem);
  const int r = lane >> 4, c = lane & 15;
  const bool diag = ti == tj;
  f64x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  const float* xi = X + ti * 64 + c;
  const float* xj = X + tj * 64 + c;
  const int64_t per = ((N + S - 1) / S + 3) / 4 * 4;
  const int64_t kb = split * per, ke = kb + per < N ? kb + per : N;
  for (int64_t k0 = kb; k0 < ke; k0 += 4) {
    const int64_t row = k0 + r;
    const bool ok = row < ke;
    double av[4], bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      av[q] = ok ? static_cast<double>(xi[row * D + 16 * q]) : 0.0;
      bv[q] = ok ? static_cast<double>(xj[row * D + 16 * q]) : 0.0;
    }
    // A (16 x 4): lane holds A[c][r] = X[row][i-col c]; B (4 x 16): lane holds B[r][c] = X[row][j-col c]
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[q] += bv[q];
  }
  // D (16 x 16): lane holds D[lane / 16 + 4 e][lane % 16], e = 0..3 (the f64 MFMA interleaves the rows; measured)
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t gi = ti * 64 + a * 16 + r + 4 * e, gj = tj * 64 + b * 16 + c;
        const double v = acc[a][b][e];
        unsafeAtomicAdd(cov + gi * D + gj, v);
        if (!diag) unsafeAtomicAdd(cov + gj * D + gi, v);
      }
  if (diag) {  // column sums of the tile's 64 columns: fold the four row groups of the wave
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cs[q] += __shfl_xor(cs[q], 16, 64);
      cs[q] += __shfl_xor(cs[q], 32, 64);
    }
    if (r == 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) unsafeAtomicAdd(fsum + tj * 64 + 16 * q + c, cs[q]);
  }
}

// features fp32 [N, D] (D % 32 == 0), states fp64 sum [D] and Gram [D, D] updated in place
void fid_moments_update(const at::Tensor& features, at::Tensor fsum, at::Tensor cov) {
  TORCH_CHECK(features.is_cuda() && features.scalar_type() == at::kFloat && features.dim() == 2, "fid_moments_update: fp32 [N, D] GPU features");
  const int64_t N = features.size(0), D = features.size(1);
  TORCH_CHECK(D % 64 == 0 && D > 0, "fid_moments_update: feature size must be a multiple of 64");
  TORCH_CHECK(fsum.is_cuda() && fsum.scalar_type() == at::kDouble && fsum.numel() == D && fsum.is_contiguous(), "fid_moments_update: sum state");
  TORCH_CHECK(cov.is_cuda() && cov.scalar_type() == at::kDouble && cov.numel() == D * D && cov.is_contiguous(), "fid_moments_update: Gram state");
  const c10::DeviceGuard guard(features.device());
  if (N == 0) return;
  const auto x = features.contiguous();
  const int T = static_cast<int>(D / 64);
  const int64_t tiles = static_cast<int64_t>(T) * (T + 1) / 2;
  // batch splits: >= ~2048 waves (8 per CU), each split at least 32 rows
  int S = 1;
  while (tiles * S < 2048 && N / (4 * S) >= 32) S *= 2;
  hipLaunchKernelGGL(fid_gram_kernel, dim3(static_cast<unsigned>((tiles * S + 3) / 4)), 256, 0, stream(), x.data_ptr<float>(), N,
                     static_cast<int>(D), T, tiles, S, fsum.data_ptr<double>(), cov.data_ptr<double>());
  TMX_LAUNCH_CHECK();
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("fid_moments_update(Tensor features, Tensor(a!) fsum, Tensor(b!) cov) -> ()"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("fid_moments_update", &tmx::fid_moments_update); }
