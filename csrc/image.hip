// Fused separable-window SSIM for gfx950.
//
// The reference reflect-pads both images, stacks (p, t, p², t², p·t) into a 5·B-image batch, runs a grouped
// conv2d and crops the padded border.  The cropped region is exactly the set of windows that lie fully inside the
// image, so the per-image SSIM is the mean over all *valid* KS×KS windows and no padding is ever needed.
//
// One block = 256 threads = 256 output columns of one (image, channel) plane and a strip of kRowsPerBlock output
// rows.  Per input row the block stages the row segment (256 + KS − 1 values of p and t) in LDS (double buffered),
// every thread computes the horizontal window sums of the five moments for its column, and keeps the last KS
// horizontal results in a register ring.  The ring is addressed with compile-time indices (row loop unrolled by
// KS), so the vertical pass is pure register FMAs; only the horizontal taps touch LDS.  The SSIM / contrast-
// sensitivity terms of each valid window are reduced per block (wave shuffles + LDS) into one fp64 partial per
// (plane, block) — the output image is never materialised.
#include "common.h"
#include "ssim_kernels.h"

#include <cstdlib>

namespace tmx {

constexpr int kRowsPerBlock = 64;

template <typename T> __device__ __forceinline__ float ld_f(const T* p, int64_t i) { return to_f32<T>(p[i]); }

template <typename T, int KS>
__global__ __launch_bounds__(kSsimThreads) void ssim_valid_kernel(const T* __restrict__ preds, const T* __restrict__ target,
                                                                  int H, int W, const float* __restrict__ wx,
                                                                  const float* __restrict__ wy, const float* __restrict__ consts,
                                                                  double* __restrict__ partial_sim, double* __restrict__ partial_cs) {
  constexpr int kSeg = kSsimThreads + KS - 1;
  __shared__ float sp[2][kSeg];
  __shared__ float st[2][kSeg];
  __shared__ float s_w[KS];
  __shared__ double red[2][kSsimThreads / kWave];

  const int Hv = H - KS + 1, Wv = W - KS + 1;
  const int64_t plane = blockIdx.z;
  const int x0 = blockIdx.x * kSsimThreads;
  const int y0 = blockIdx.y * kRowsPerBlock;
  const int tid = threadIdx.x;
  const T* P = preds + plane * static_cast<int64_t>(H) * W;
  const T* Tt = target + plane * static_cast<int64_t>(H) * W;
  const float c1 = consts[0], c2 = consts[1];
  if (tid < KS) s_w[tid] = wx[tid];

  float wyr[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) wyr[k] = wy[k];

  // ring of horizontal window sums: (mu_p, mu_t, E[pp], E[tt], E[pt]) for the last KS input rows
  float ring[KS][5];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int q = 0; q < 5; ++q) ring[k][q] = 0.f;

  const int out_rows = min(kRowsPerBlock, Hv - y0);
  const int in_rows = out_rows + KS - 1;  // input rows y0 .. y0 + in_rows - 1
  const bool col_ok = (x0 + tid) < Wv;
  double acc_sim = 0.0, acc_cs = 0.0;

  auto stage = [&](int r, int buf) {
    const int64_t row = static_cast<int64_t>(y0 + r) * W;
    for (int i = tid; i < kSeg; i += kSsimThreads) {
      const int x = x0 + i;
      const bool ok = x < W;
      sp[buf][i] = ok ? ld_f(P, row + x) : 0.f;
      st[buf][i] = ok ? ld_f(Tt, row + x) : 0.f;
    }
  };

  if (in_rows > 0) stage(0, 0);
  __syncthreads();

  for (int base = 0; base < in_rows; base += KS) {
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      const int r = base + j;
      if (r < in_rows) {  // uniform across the block
        const int buf = r & 1;
        if (r + 1 < in_rows) stage(r + 1, buf ^ 1);
        // horizontal pass for this thread's column
        float hp = 0.f, ht = 0.f, hpp = 0.f, htt = 0.f, hpt = 0.f;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const float w = s_w[k];
          const float p = sp[buf][tid + k];
          const float t = st[buf][tid + k];
          const float wp = w * p, wt = w * t;
          hp += wp;
          ht += wt;
          hpp = fmaf(wp, p, hpp);
          htt = fmaf(wt, t, htt);
          hpt = fmaf(wp, t, hpt);
        }
        ring[j][0] = hp;
        ring[j][1] = ht;
        ring[j][2] = hpp;
        ring[j][3] = htt;
        ring[j][4] = hpt;
        if (r >= KS - 1 && col_ok) {
          // vertical pass: rows r-KS+1 .. r live in ring[(j+1+k) % KS] (oldest first)
          float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < KS; ++k) {
            const int slot = (j + 1 + k) % KS;
#pragma unroll
            for (int q = 0; q < 5; ++q) m[q] = fmaf(wyr[k], ring[slot][q], m[q]);
          }
          const float mu_pp = m[0] * m[0], mu_tt = m[1] * m[1], mu_pt = m[0] * m[1];
          const float upper = 2.f * (m[4] - mu_pt) + c2;
          const float lower = (m[2] - mu_pp) + (m[3] - mu_tt) + c2;
          const float cs = upper / lower;
          const float sim = (2.f * mu_pt + c1) * upper / ((mu_pp + mu_tt + c1) * lower);
          acc_sim += static_cast<double>(sim);
          acc_cs += static_cast<double>(cs);
        }
        __syncthreads();  // staged row r+1 visible; buffer r free for r+2
      }
    }
  }

  // block reduction of the two sums
  acc_sim = wave_sum(acc_sim);
  acc_cs = wave_sum(acc_cs);
  const int wave = tid / kWave, lane = tid & (kWave - 1);
  if (lane == 0) {
    red[0][wave] = acc_sim;
    red[1][wave] = acc_cs;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0, c = 0.0;
    for (int w = 0; w < kSsimThreads / kWave; ++w) {
      s += red[0][w];
      c += red[1][w];
    }
    const int64_t idx = (plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    partial_sim[idx] = s;
    partial_cs[idx] = c;
  }
}

template <typename T, int KS>
void launch_ssim(const at::Tensor& p, const at::Tensor& t, const at::Tensor& wx, const at::Tensor& wy,
                 const at::Tensor& consts, at::Tensor& ps, at::Tensor& pc, dim3 grid, int H, int W) {
  hipLaunchKernelGGL((ssim_valid_kernel<T, KS>), grid, kSsimThreads, 0, stream(), reinterpret_cast<const T*>(p.data_ptr()),
                     reinterpret_cast<const T*>(t.data_ptr()), H, W, wx.data_ptr<float>(), wy.data_ptr<float>(),
                     consts.data_ptr<float>(), ps.data_ptr<double>(), pc.data_ptr<double>());
}

template <int KS>
void launch_ssim_v2(const at::Tensor& p, const at::Tensor& t, const at::Tensor& wx, const at::Tensor& wy, const at::Tensor& consts,
                    at::Tensor& ps, at::Tensor& pc, double* pe, dim3 grid, int H, int W, const int* run_if = nullptr) {
  if (pe != nullptr)
    hipLaunchKernelGGL((ssim_v2_kernel<KS, true>), grid, kSsimThreads, 0, stream(), p.data_ptr<float>(), t.data_ptr<float>(), H, W,
                       wx.data_ptr<float>(), wy.data_ptr<float>(), consts.data_ptr<float>(), ps.data_ptr<double>(), pc.data_ptr<double>(), pe,
                       run_if);
  else
    hipLaunchKernelGGL((ssim_v2_kernel<KS, false>), grid, kSsimThreads, 0, stream(), p.data_ptr<float>(), t.data_ptr<float>(), H, W,
                       wx.data_ptr<float>(), wy.data_ptr<float>(), consts.data_ptr<float>(), ps.data_ptr<double>(), pc.data_ptr<double>(),
                       nullptr, run_if);
}

// preds/target [P, H, W] planes (P = B*C); wx/wy fp32 [KS] window weights; consts fp32 [2] = (c1, c2) on device, or
// [3] = (c1, c2, data range): the matrix-core kernel (wx == wy).
// Returns fp64 [2, P]: per-plane sums of SSIM and contrast sensitivity over all valid windows.
at::Tensor ssim_sums(const at::Tensor& preds_in, const at::Tensor& target_in, const at::Tensor& wx_in,
                     const at::Tensor& wy_in, const at::Tensor& consts_in, bool with_sse) {
  TORCH_CHECK(preds_in.is_cuda() && target_in.is_cuda(), "ssim_sums: expected GPU tensors");
  TORCH_CHECK(preds_in.dim() == 3 && preds_in.sizes() == target_in.sizes(), "ssim_sums: expected matching [P, H, W]");
  TORCH_CHECK(preds_in.scalar_type() == target_in.scalar_type(), "ssim_sums: dtype mismatch");
  const int64_t KS = wx_in.numel();
  TORCH_CHECK(wy_in.numel() == KS, "ssim_sums: window size mismatch");
  const at::DeviceGuard guard(preds_in.device());
  auto p = preds_in.contiguous();
  auto t = target_in.contiguous();
  auto wx = wx_in.to(at::kFloat).contiguous();
  auto wy = wy_in.to(at::kFloat).contiguous();
  auto consts = consts_in.to(at::kFloat).contiguous();
  const int64_t P = p.size(0), H = p.size(1), W = p.size(2);
  TORCH_CHECK(H >= KS && W >= KS, "ssim_sums: image smaller than the window");
  TORCH_CHECK(P <= 65535, "ssim_sums: too many planes for one launch");
  const int64_t Hv = H - KS + 1, Wv = W - KS + 1;
  static const bool v2_off = std::getenv("TMX_SSIM_V1") != nullptr;  // A/B knob (tools/ssim_bench.py)
  const bool v2 = !v2_off && p.scalar_type() == at::kFloat && W % 4 == 0 && (reinterpret_cast<uintptr_t>(p.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0 && KS % 2 == 1 && KS <= 15;
  const int rows_per_block = v2 ? kRowsV2 : kRowsPerBlock;
  dim3 grid(static_cast<unsigned>((Wv + kSsimThreads - 1) / kSsimThreads),
            static_cast<unsigned>((Hv + rows_per_block - 1) / rows_per_block), static_cast<unsigned>(P));
  auto opts = p.options().dtype(at::kDouble);
  auto ps = at::empty({P, static_cast<int64_t>(grid.y) * grid.x}, opts);
  auto pc = at::empty({P, static_cast<int64_t>(grid.y) * grid.x}, opts);
  auto pe_t = with_sse && v2 ? at::empty({P, static_cast<int64_t>(grid.y) * grid.x}, opts) : at::Tensor();
  double* pe = with_sse && v2 ? pe_t.data_ptr<double>() : nullptr;
  // round 6: the matrix-core kernel (csrc/ssim_kernels.h ssim_mfma_kernel) when the caller passes the data range
  // (consts = c1, c2, D), with ssim_v2_kernel as its device-side fallback for out-of-range data
  static const bool mfma_off = std::getenv("TMX_SSIM_V2") != nullptr;  // A/B knob (tools/ssim_bench.py)
  if (v2 && !mfma_off && consts.numel() >= 3 && KS <= 17) {
    // output rows per workgroup strip (a multiple of 16; each strip re-reads a KS - 1 halo band); 1024 measured fastest
    // of 256 / 512 / 1024 on the 1080p bench config (2.48 / 2.35 / 2.32 ms, tools/kexp/ssim_mfma_exp.hip)
    static const int kStrip = std::getenv("TMX_SSIM_STRIP") ? std::max(16, std::atoi(std::getenv("TMX_SSIM_STRIP")) / 16 * 16) : 1024;
    const int ntx = static_cast<int>((Wv + 15) / 16);
    dim3 mgrid(static_cast<unsigned>((ntx + kSsimMfmaWaves - 1) / kSsimMfmaWaves), static_cast<unsigned>((Hv + kStrip - 1) / kStrip),
               static_cast<unsigned>(P));
    const int64_t nparts = static_cast<int64_t>(mgrid.y) * ntx;
    auto ms = at::empty({P, nparts}, opts), mc = at::empty({P, nparts}, opts);
    auto me = with_sse ? at::empty({P, nparts}, opts) : at::Tensor();
    auto flag = at::zeros({1}, p.options().dtype(at::kInt));
    if (with_sse)
      hipLaunchKernelGGL((ssim_mfma_kernel<true>), mgrid, kSsimMfmaWaves * kWave, 0, stream(), p.data_ptr<float>(), t.data_ptr<float>(),
                         (int)H, (int)W, (int)KS, kStrip, wx.data_ptr<float>(), consts.data_ptr<float>(), ms.data_ptr<double>(),
                         mc.data_ptr<double>(), me.data_ptr<double>(), flag.data_ptr<int>());
    else
      hipLaunchKernelGGL((ssim_mfma_kernel<false>), mgrid, kSsimMfmaWaves * kWave, 0, stream(), p.data_ptr<float>(), t.data_ptr<float>(),
                         (int)H, (int)W, (int)KS, kStrip, wx.data_ptr<float>(), consts.data_ptr<float>(), ms.data_ptr<double>(),
                         mc.data_ptr<double>(), nullptr, flag.data_ptr<int>());
    TMX_LAUNCH_CHECK();
    // the fallback launch: every workgroup exits at its first load unless the kernel above flagged the batch
    switch (KS) {
      case 3: launch_ssim_v2<3>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      case 5: launch_ssim_v2<5>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      case 7: launch_ssim_v2<7>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      case 9: launch_ssim_v2<9>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      case 11: launch_ssim_v2<11>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      case 13: launch_ssim_v2<13>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
      default: launch_ssim_v2<15>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W, flag.data_ptr<int>()); break;
    }
    TMX_LAUNCH_CHECK();
    auto use_v2 = flag.gt(0);
    auto fast = with_sse ? at::stack({ms.sum(1), mc.sum(1), me.sum(1)}) : at::stack({ms.sum(1), mc.sum(1)});
    auto slow = with_sse ? at::stack({ps.sum(1), pc.sum(1), pe_t.sum(1)}) : at::stack({ps.sum(1), pc.sum(1)});
    return at::where(use_v2, slow, fast);
  }
  if (v2) {
    switch (KS) {
      case 3: launch_ssim_v2<3>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      case 5: launch_ssim_v2<5>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      case 7: launch_ssim_v2<7>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      case 9: launch_ssim_v2<9>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      case 11: launch_ssim_v2<11>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      case 13: launch_ssim_v2<13>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
      default: launch_ssim_v2<15>(p, t, wx, wy, consts, ps, pc, pe, grid, H, W); break;
    }
    TMX_LAUNCH_CHECK();
    if (with_sse) return at::stack({ps.sum(1), pc.sum(1), pe_t.sum(1)});
    return at::stack({ps.sum(1), pc.sum(1)});
  }
  TMX_DISPATCH_FLOAT(p.scalar_type(), "ssim_sums", [&] {
    switch (KS) {
      case 3: launch_ssim<scalar_t, 3>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 5: launch_ssim<scalar_t, 5>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 7: launch_ssim<scalar_t, 7>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 9: launch_ssim<scalar_t, 9>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 11: launch_ssim<scalar_t, 11>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 13: launch_ssim<scalar_t, 13>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      case 15: launch_ssim<scalar_t, 15>(p, t, wx, wy, consts, ps, pc, grid, H, W); break;
      default: TORCH_CHECK(false, "ssim_sums: unsupported window size ", KS);
    }
  });
  TMX_LAUNCH_CHECK();
  if (with_sse) {  // (v1 path) SSE by a separate reduction
    auto d = (p.to(at::kDouble) - t.to(at::kDouble));
    return at::stack({ps.sum(1), pc.sum(1), (d * d).sum({1, 2})});
  }
  return at::stack({ps.sum(1), pc.sum(1)});
}

// ------------------------------------------------------------------------------------------------------------
// LPIPS head: per pixel, channel-L2-normalise both feature maps, squared difference, 1×1
// linear layer (C -> 1) and spatial mean — fused into one pass over the two [B, C, H·W] feature tensors.
//   Σ_c w_c (f0_c/a − f1_c/b)² = S00/a² + S11/b² − 2·S01/(a·b),  a² = eps + Σ f0², b² = eps + Σ f1²
// One thread per pixel (coalesced across the spatial index for every channel), five fp32 accumulators; one fp64
// partial per block, summed deterministically on the host side of the op.
// ------------------------------------------------------------------------------------------------------------
constexpr int kLpipsThreads = 256;

template <typename T>
__global__ __launch_bounds__(kLpipsThreads) void lpips_head_kernel(const T* __restrict__ f0, const T* __restrict__ f1,
                                                                   const float* __restrict__ w, int C, int64_t HW,
                                                                   double* __restrict__ partial) {
  const int64_t b = blockIdx.y;
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kLpipsThreads + threadIdx.x;
  double v = 0.0;
  if (s < HW) {
    const T* p0 = f0 + b * C * HW + s;
    const T* p1 = f1 + b * C * HW + s;
    float n0 = 0.f, n1 = 0.f, s00 = 0.f, s11 = 0.f, s01 = 0.f;
    for (int c = 0; c < C; ++c) {
      const float x = to_f32<T>(p0[c * HW]);
      const float y = to_f32<T>(p1[c * HW]);
      const float wc = w[c];
      n0 = fmaf(x, x, n0);
      n1 = fmaf(y, y, n1);
      s00 = fmaf(wc * x, x, s00);
      s11 = fmaf(wc * y, y, s11);
      s01 = fmaf(wc * x, y, s01);
    }
    const float a2 = 1e-8f + n0, b2 = 1e-8f + n1;
    v = static_cast<double>(s00 / a2 + s11 / b2 - 2.f * s01 / (sqrtf(a2) * sqrtf(b2)));
  }
  v = wave_sum(v);
  __shared__ double red[kLpipsThreads / kWave];
  const int wave = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < kLpipsThreads / kWave; ++i) t += red[i];
    partial[b * gridDim.x + blockIdx.x] = t;
  }
}

// channels_last feature maps ([B][H·W][C] in memory, what a channels_last trunk produces): the same sums, each thread
// walking its pixel's C contiguous channels (no layout copy of the feature maps before the head)
template <typename T>
__global__ __launch_bounds__(kLpipsThreads) void lpips_head_nhwc_kernel(const T* __restrict__ f0, const T* __restrict__ f1,
                                                                        const float* __restrict__ w, int C, int64_t HW,
                                                                        double* __restrict__ partial) {
  const int64_t b = blockIdx.y;
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kLpipsThreads + threadIdx.x;
  double v = 0.0;
  if (s < HW) {
    const T* p0 = f0 + (b * HW + s) * C;
    const T* p1 = f1 + (b * HW + s) * C;
    float n0 = 0.f, n1 = 0.f, s00 = 0.f, s11 = 0.f, s01 = 0.f;
    for (int c = 0; c < C; ++c) {
      const float x = to_f32<T>(p0[c]);
      const float y = to_f32<T>(p1[c]);
      const float wc = w[c];
      n0 = fmaf(x, x, n0);
      n1 = fmaf(y, y, n1);
      s00 = fmaf(wc * x, x, s00);
      s11 = fmaf(wc * y, y, s11);
      s01 = fmaf(wc * x, y, s01);
    }
    const float a2 = 1e-8f + n0, b2 = 1e-8f + n1;
    v = static_cast<double>(s00 / a2 + s11 / b2 - 2.f * s01 / (sqrtf(a2) * sqrtf(b2)));
  }
  v = wave_sum(v);
  __shared__ double red[kLpipsThreads / kWave];
  const int wave = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < kLpipsThreads / kWave; ++i) t += red[i];
    partial[b * gridDim.x + blockIdx.x] = t;
  }
}

// channels_last, C % 4 == 0, 16-B aligned: four threads per pixel read adjacent float4s of its channel row (a wave covers
// 16 pixels x 64 B per load instead of 64 pixels x 4 B at stride C), then two xor-shuffle steps combine the four
// partial sums.  (The per-thread walk above ran at 9.4 ms per call on VGG16's first tap: gpurun r7w.)
constexpr int kLpipsPixPerBlock = kLpipsThreads / 4;

__global__ __launch_bounds__(kLpipsThreads) void lpips_head_nhwc4_kernel(const float* __restrict__ f0, const float* __restrict__ f1,
                                                                         const float* __restrict__ w, int C, int64_t HW,
                                                                         double* __restrict__ partial) {
  const int64_t b = blockIdx.y;
  const int q = threadIdx.x & 3;
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kLpipsPixPerBlock + (threadIdx.x >> 2);
  float n0 = 0.f, n1 = 0.f, s00 = 0.f, s11 = 0.f, s01 = 0.f;
  if (s < HW) {
    const float4* p0 = reinterpret_cast<const float4*>(f0 + (b * HW + s) * C);
    const float4* p1 = reinterpret_cast<const float4*>(f1 + (b * HW + s) * C);
    const float4* w4 = reinterpret_cast<const float4*>(w);
    for (int k = q; k < C / 4; k += 4) {
      const float4 x = p0[k], y = p1[k], wc = w4[k];
      n0 = fmaf(x.x, x.x, fmaf(x.y, x.y, fmaf(x.z, x.z, fmaf(x.w, x.w, n0))));
      n1 = fmaf(y.x, y.x, fmaf(y.y, y.y, fmaf(y.z, y.z, fmaf(y.w, y.w, n1))));
      s00 = fmaf(wc.x * x.x, x.x, fmaf(wc.y * x.y, x.y, fmaf(wc.z * x.z, x.z, fmaf(wc.w * x.w, x.w, s00))));
      s11 = fmaf(wc.x * y.x, y.x, fmaf(wc.y * y.y, y.y, fmaf(wc.z * y.z, y.z, fmaf(wc.w * y.w, y.w, s11))));
      s01 = fmaf(wc.x * x.x, y.x, fmaf(wc.y * x.y, y.y, fmaf(wc.z * x.z, y.z, fmaf(wc.w * x.w, y.w, s01))));
    }
  }
#pragma unroll
  for (int off = 1; off < 4; off <<= 1) {  // (every lane takes part: the shuffles stay uniform)
    n0 += __shfl_xor(n0, off, 4);
    n1 += __shfl_xor(n1, off, 4);
    s00 += __shfl_xor(s00, off, 4);
    s11 += __shfl_xor(s11, off, 4);
    s01 += __shfl_xor(s01, off, 4);
  }
  double v = 0.0;
  if (q == 0 && s < HW) {
    const float a2 = 1e-8f + n0, b2 = 1e-8f + n1;
    v = static_cast<double>(s00 / a2 + s11 / b2 - 2.f * s01 / (sqrtf(a2) * sqrtf(b2)));
  }
  v = wave_sum(v);
  __shared__ double red[kLpipsThreads / kWave];
  const int wave = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < kLpipsThreads / kWave; ++i) t += red[i];
    partial[b * gridDim.x + blockIdx.x] = t;
  }
}

// f0/f1 [B, C, H, W]; w [C] (1×1 conv weight). Returns fp64 [B] spatial means of the weighted normalised distance.
at::Tensor lpips_head(const at::Tensor& f0_in, const at::Tensor& f1_in, const at::Tensor& w_in) {
  TORCH_CHECK(f0_in.is_cuda() && f1_in.is_cuda(), "lpips_head: expected GPU tensors");
  TORCH_CHECK(f0_in.dim() == 4 && f0_in.sizes() == f1_in.sizes(), "lpips_head: expected matching [B, C, H, W]");
  TORCH_CHECK(f0_in.scalar_type() == f1_in.scalar_type(), "lpips_head: dtype mismatch");
  TORCH_CHECK(w_in.numel() == f0_in.size(1), "lpips_head: weight / channel mismatch");
  const at::DeviceGuard guard(f0_in.device());
  // channels_last inputs (a channels_last trunk) are read in place by the NHWC kernel
  const bool nhwc = !f0_in.is_contiguous() && f0_in.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    f1_in.is_contiguous(at::MemoryFormat::ChannelsLast);
  auto f0 = nhwc ? f0_in : f0_in.contiguous();
  auto f1 = nhwc ? f1_in : f1_in.contiguous();
  auto w = w_in.reshape(-1).to(at::kFloat).contiguous();
  const int64_t B = f0.size(0), C = f0.size(1), HW = f0.size(2) * f0.size(3);
  auto opts = f0.options().dtype(at::kDouble);
  if (B == 0 || HW == 0) return at::zeros({B}, opts);
  TORCH_CHECK(B <= 65535, "lpips_head: batch too large for one launch");
  const bool nhwc4 = nhwc && f0.scalar_type() == at::kFloat && C % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(f0.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(f1.data_ptr()) & 15) == 0;
  const int64_t per_block = nhwc4 ? kLpipsPixPerBlock : kLpipsThreads;
  dim3 grid(static_cast<unsigned>((HW + per_block - 1) / per_block), static_cast<unsigned>(B));
  auto partial = at::empty({B, static_cast<int64_t>(grid.x)}, opts);
  if (nhwc4) {  // (w is a fresh contiguous fp32 tensor: 16-B aligned)
    hipLaunchKernelGGL(lpips_head_nhwc4_kernel, grid, kLpipsThreads, 0, stream(), f0.data_ptr<float>(), f1.data_ptr<float>(),
                       w.data_ptr<float>(), static_cast<int>(C), HW, partial.data_ptr<double>());
    TMX_LAUNCH_CHECK();
    return partial.sum(1) / static_cast<double>(HW);
  }
  TMX_DISPATCH_FLOAT(f0.scalar_type(), "lpips_head", [&] {
    if (nhwc)
      hipLaunchKernelGGL((lpips_head_nhwc_kernel<scalar_t>), grid, kLpipsThreads, 0, stream(),
                         reinterpret_cast<const scalar_t*>(f0.data_ptr()), reinterpret_cast<const scalar_t*>(f1.data_ptr()),
                         w.data_ptr<float>(), static_cast<int>(C), HW, partial.data_ptr<double>());
    else
      hipLaunchKernelGGL((lpips_head_kernel<scalar_t>), grid, kLpipsThreads, 0, stream(),
                         reinterpret_cast<const scalar_t*>(f0.data_ptr()), reinterpret_cast<const scalar_t*>(f1.data_ptr()),
                         w.data_ptr<float>(), static_cast<int>(C), HW, partial.data_ptr<double>());
  });
  TMX_LAUNCH_CHECK();
  return partial.sum(1) / static_cast<double>(HW);
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("ssim_sums(Tensor preds, Tensor target, Tensor wx, Tensor wy, Tensor consts, bool with_sse=False) -> Tensor");
  m.def("lpips_head(Tensor f0, Tensor f1, Tensor w) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("ssim_sums", &tmx::ssim_sums);
  m.impl("lpips_head", &tmx::lpips_head);
}
