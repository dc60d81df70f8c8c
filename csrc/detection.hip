// Pairwise box-overlap matrices for gfx950: IoU / GIoU / DIoU / CIoU of two xyxy box sets.
//
// One thread per (i, j) output; a block covers a 16 × 64 output tile and stages its 16 + 64 boxes (plus their
// areas) in LDS once, so every box is read from HBM once per tile instead of once per output.  fp32 math with
// the same formulas (and eps = 1e-7 for the distance terms) as the torchvision operators the reference calls.
#include "common.h"

namespace tmx {

constexpr int kBoxTileI = 16;
constexpr int kBoxTileJ = 64;

enum BoxMode : int { kIoU = 0, kGIoU = 1, kDIoU = 2, kCIoU = 3 };

template <int MODE>
__global__ __launch_bounds__(kBoxTileI * kBoxTileJ) void box_pairwise_kernel(const float* __restrict__ b1, const float* __restrict__ b2,
                                                                          int64_t N, int64_t M, float* __restrict__ out) {
  __shared__ float s1[kBoxTileI][4];
  __shared__ float s2[kBoxTileJ][4];
  const int tid = threadIdx.x;
  const int64_t i0 = static_cast<int64_t>(blockIdx.y) * kBoxTileI;
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * kBoxTileJ;
  if (tid < kBoxTileI * 4) {
    const int64_t r = i0 + tid / 4;
    s1[tid / 4][tid % 4] = r < N ? b1[r * 4 + tid % 4] : 0.f;
  }
  if (tid < kBoxTileJ * 4) {
    const int64_t r = j0 + tid / 4;
    s2[tid / 4][tid % 4] = r < M ? b2[r * 4 + tid % 4] : 0.f;
  }
  __syncthreads();
  const int li = tid / kBoxTileJ, lj = tid % kBoxTileJ;
  const int64_t i = i0 + li, j = j0 + lj;
  if (i >= N || j >= M) return;
  const float ax0 = s1[li][0], ay0 = s1[li][1], ax1 = s1[li][2], ay1 = s1[li][3];
  const float bx0 = s2[lj][0], by0 = s2[lj][1], bx1 = s2[lj][2], by1 = s2[lj][3];
  const float area_a = (ax1 - ax0) * (ay1 - ay0);
  const float area_b = (bx1 - bx0) * (by1 - by0);
  const float iw = fmaxf(fminf(ax1, bx1) - fmaxf(ax0, bx0), 0.f);
  const float ih = fmaxf(fminf(ay1, by1) - fmaxf(ay0, by0), 0.f);
  const float inter = iw * ih;
  const float uni = area_a + area_b - inter;
  const float iou = inter / uni;
  float v = iou;
  if constexpr (MODE == kGIoU) {
    const float cw = fmaxf(fmaxf(ax1, bx1) - fminf(ax0, bx0), 0.f);
    const float ch = fmaxf(fmaxf(ay1, by1) - fminf(ay0, by0), 0.f);
    const float area_c = cw * ch;
    v = iou - (area_c - uni) / area_c;
  } else if constexpr (MODE == kDIoU || MODE == kCIoU) {
    const float eps = 1e-7f;
    const float cw = fmaxf(fmaxf(ax1, bx1) - fminf(ax0, bx0), 0.f);
    const float ch = fmaxf(fmaxf(ay1, by1) - fminf(ay0, by0), 0.f);
    const float diag = cw * cw + ch * ch + eps;
    const float dx = (ax0 + ax1) * 0.5f - (bx0 + bx1) * 0.5f;
    const float dy = (ay0 + ay1) * 0.5f - (by0 + by1) * 0.5f;
    v = iou - (dx * dx + dy * dy) / diag;
    if constexpr (MODE == kCIoU) {
      const float at = atanf((ax1 - ax0) / (ay1 - ay0)) - atanf((bx1 - bx0) / (by1 - by0));
      const float vv = (4.f / (3.14159265358979323846f * 3.14159265358979323846f)) * at * at;
      const float alpha = vv / (1.f - iou + vv + eps);
      v = v - alpha * vv;
    }
  }
  out[i * M + j] = v;
}

at::Tensor box_pairwise(const at::Tensor& b1_in, const at::Tensor& b2_in, int64_t mode) {
  TORCH_CHECK(b1_in.is_cuda() && b2_in.is_cuda(), "box_pairwise: expected GPU tensors");
  TORCH_CHECK(b1_in.dim() == 2 && b1_in.size(1) == 4 && b2_in.dim() == 2 && b2_in.size(1) == 4,
              "box_pairwise: expected [N,4] and [M,4] xyxy boxes");
  TORCH_CHECK(mode >= 0 && mode <= 3, "box_pairwise: unknown mode ", mode);
  const at::DeviceGuard guard(b1_in.device());
  auto b1 = b1_in.to(at::kFloat).contiguous();
  auto b2 = b2_in.to(at::kFloat).contiguous();
  const int64_t N = b1.size(0), M = b2.size(0);
  auto out = at::empty({N, M}, b1.options());
  if (N == 0 || M == 0) return out;
  dim3 grid(static_cast<unsigned>((M + kBoxTileJ - 1) / kBoxTileJ), static_cast<unsigned>((N + kBoxTileI - 1) / kBoxTileI));
  const int threads = kBoxTileI * kBoxTileJ;
  switch (mode) {
    case kIoU: hipLaunchKernelGGL(box_pairwise_kernel<kIoU>, grid, threads, 0, stream(), b1.data_ptr<float>(), b2.data_ptr<float>(), N, M, out.data_ptr<float>()); break;
    case kGIoU: hipLaunchKernelGGL(box_pairwise_kernel<kGIoU>, grid, threads, 0, stream(), b1.data_ptr<float>(), b2.data_ptr<float>(), N, M, out.data_ptr<float>()); break;
    case kDIoU: hipLaunchKernelGGL(box_pairwise_kernel<kDIoU>, grid, threads, 0, stream(), b1.data_ptr<float>(), b2.data_ptr<float>(), N, M, out.data_ptr<float>()); break;
    default: hipLaunchKernelGGL(box_pairwise_kernel<kCIoU>, grid, threads, 0, stream(), b1.data_ptr<float>(), b2.data_ptr<float>(), N, M, out.data_ptr<float>()); break;
  }
  TMX_LAUNCH_CHECK();
  return out;
}

// ---------------------------------------------------------------------------------------------------------------
// Bit-packed mask IoU (segmentation mAP).  Masks arrive packed 64 pixels per uint64 word; a block computes a
// 16 × 16 (detection, ground truth) tile, staging 64-word chunks of both row sets in LDS, and every thread
// accumulates popcount(d & g) for one pair.  Exact integer intersections at 1/64 of the bytes of a float matmul.
// Crowd ground truth uses the detection area as the denominator (COCO semantics).
constexpr int kMaskTile = 16;
constexpr int kMaskChunk = 64;

__global__ __launch_bounds__(kMaskTile * kMaskTile) void mask_iou_kernel(const uint64_t* __restrict__ dbits, const uint64_t* __restrict__ gbits,
                                                                         const double* __restrict__ darea, const double* __restrict__ garea,
                                                                         const bool* __restrict__ crowd, int64_t D, int64_t G, int64_t W,
                                                                         double* __restrict__ out) {
  __shared__ uint64_t sd[kMaskTile][kMaskChunk + 1];
  __shared__ uint64_t sg[kMaskTile][kMaskChunk + 1];
  const int tid = threadIdx.x;
  const int ld = tid / kMaskTile, lg = tid % kMaskTile;
  const int64_t d0 = static_cast<int64_t>(blockIdx.y) * kMaskTile;
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * kMaskTile;
  unsigned long long inter = 0;
  for (int64_t w0 = 0; w0 < W; w0 += kMaskChunk) {
    for (int e = tid; e < kMaskTile * kMaskChunk; e += kMaskTile * kMaskTile) {
      const int r = e / kMaskChunk, c = e % kMaskChunk;
      const int64_t w = w0 + c;
      sd[r][c] = (d0 + r < D && w < W) ? dbits[(d0 + r) * W + w] : 0ull;
      sg[r][c] = (g0 + r < G && w < W) ? gbits[(g0 + r) * W + w] : 0ull;
    }
    __syncthreads();
#pragma unroll 8
    for (int c = 0; c < kMaskChunk; ++c) inter += __popcll(sd[ld][c] & sg[lg][c]);
    __syncthreads();
  }
  const int64_t d = d0 + ld, g = g0 + lg;
  if (d >= D || g >= G) return;
  const double i = static_cast<double>(inter);
  const double u = crowd[g] ? darea[d] : darea[d] + garea[g] - i;
  out[d * G + g] = u > 0 ? i / u : 0.0;
}

// dbits [D, W] / gbits [G, W] int64 words; areas fp64; crowd bool [G] -> fp64 [D, G]
at::Tensor mask_iou(const at::Tensor& dbits_in, const at::Tensor& gbits_in, const at::Tensor& darea_in, const at::Tensor& garea_in,
                    const at::Tensor& crowd_in) {
  TORCH_CHECK(dbits_in.is_cuda() && gbits_in.is_cuda(), "mask_iou: expected GPU tensors");
  TORCH_CHECK(dbits_in.scalar_type() == at::kLong && gbits_in.scalar_type() == at::kLong, "mask_iou: expected int64 packed words");
  TORCH_CHECK(dbits_in.dim() == 2 && gbits_in.dim() == 2 && dbits_in.size(1) == gbits_in.size(1), "mask_iou: word count mismatch");
  const int64_t D = dbits_in.size(0), G = gbits_in.size(0), W = dbits_in.size(1);
  TORCH_CHECK(darea_in.numel() == D && garea_in.numel() == G && crowd_in.numel() == G, "mask_iou: area/crowd size mismatch");
  const at::DeviceGuard guard(dbits_in.device());
  auto dbits = dbits_in.contiguous(), gbits = gbits_in.contiguous();
  auto darea = darea_in.to(at::kDouble).contiguous(), garea = garea_in.to(at::kDouble).contiguous();
  auto crowd = crowd_in.to(at::kBool).contiguous();
  auto out = at::zeros({D, G}, dbits.options().dtype(at::kDouble));
  if (D == 0 || G == 0) return out;
  dim3 grid(static_cast<unsigned>((G + kMaskTile - 1) / kMaskTile), static_cast<unsigned>((D + kMaskTile - 1) / kMaskTile));
  hipLaunchKernelGGL(mask_iou_kernel, grid, kMaskTile * kMaskTile, 0, stream(), reinterpret_cast<const uint64_t*>(dbits.data_ptr<int64_t>()),
                     reinterpret_cast<const uint64_t*>(gbits.data_ptr<int64_t>()), darea.data_ptr<double>(), garea.data_ptr<double>(),
                     crowd.data_ptr<bool>(), D, G, W, out.data_ptr<double>());
  TMX_LAUNCH_CHECK();
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("box_pairwise(Tensor boxes1, Tensor boxes2, int mode) -> Tensor");
  m.def("mask_iou(Tensor det_bits, Tensor gt_bits, Tensor det_area, Tensor gt_area, Tensor gt_crowd) -> Tensor");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("box_pairwise", &tmx::box_pairwise);
  m.impl("mask_iou", &tmx::mask_iou);
}
