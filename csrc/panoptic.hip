// Panoptic quality segment keys (K24) for gfx950.
//
// Reference: functional/detection/_panoptic_quality_common.py:231-296 builds Python dicts of (category, instance)
// colours per image and counts pixels with torch.unique over [P, 2] rows.  Here one pass over the pixels of both
// inputs maps every category id to its continuous index (binary search in the sorted id table held in LDS; unmapped
// / void -> k) and packs (image, continuous category, instance) into one order-preserving int64 key
// (16 | 16 | 32 bits), so segment discovery is a 1-D radix unique instead of a lexicographic row sort, and the
// segment's category is read back from its key.  Pixels whose instance id does not fit 32 unsigned bits set a
// flag (the caller then keeps the row-unique path).
#include "common.h"

namespace tmx {
namespace {

constexpr int kPqMaxIds = 4096;

__global__ __launch_bounds__(256) void pq_keys_kernel(const int64_t* __restrict__ preds, const int64_t* __restrict__ target,
                                                      int64_t P, int64_t total, const int64_t* __restrict__ ids,
                                                      const int64_t* __restrict__ cont, int n_ids, int64_t* __restrict__ pkey,
                                                      int64_t* __restrict__ tkey, int* __restrict__ overflow) {
  __shared__ int64_t s_ids[kPqMaxIds];
  __shared__ int s_cont[kPqMaxIds + 1];
  for (int i = threadIdx.x; i < n_ids; i += blockDim.x) {
    s_ids[i] = ids[i];
    s_cont[i] = static_cast<int>(cont[i]);
  }
  if (threadIdx.x == 0) s_cont[n_ids] = static_cast<int>(cont[n_ids]);
  __syncthreads();
  const int k = s_cont[n_ids];
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / P;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int64_t* src = side ? target : preds;
      const int64_t cat = src[2 * i], inst = src[2 * i + 1];
      int lo = 0, hi = n_ids;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_ids[mid] < cat) lo = mid + 1;
        else hi = mid;
      }
      const int ci = (lo < n_ids && s_ids[lo] == cat) ? s_cont[lo] : k;
      bad |= inst < 0 || inst > 0xFFFFFFFFll;
      const int64_t key = (b << 48) | (static_cast<int64_t>(ci) << 32) | (inst & 0xFFFFFFFFll);
      (side ? tkey : pkey)[i] = key;
    }
  }
  if (__ballot(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(overflow, 1);
}

}  // namespace

// preds / target: int64 [B, P, 2] (category, instance) after preprocessing; ids: sorted int64 category ids; cont:
// int64 [n_ids + 1] continuous index per id (+ k for void / unmapped).  Returns (pred keys [B * P], target keys
// [B * P], overflow flag int32 [1]).
std::vector<at::Tensor> panoptic_segment_keys(const at::Tensor& preds, const at::Tensor& target, const at::Tensor& ids,
                                              const at::Tensor& cont) {
  TORCH_CHECK(preds.is_cuda() && preds.scalar_type() == at::kLong && target.scalar_type() == at::kLong && preds.dim() == 3 &&
                  preds.size(2) == 2 && target.sizes() == preds.sizes(), "panoptic_segment_keys: int64 [B, P, 2] inputs");
  TORCH_CHECK(ids.scalar_type() == at::kLong && cont.scalar_type() == at::kLong && cont.numel() == ids.numel() + 1 &&
                  ids.numel() <= kPqMaxIds, "panoptic_segment_keys: id table");
  TORCH_CHECK(preds.size(0) < 32768 && cont.max().item<int64_t>() < 65536, "panoptic_segment_keys: key field widths");
  c10::DeviceGuard guard(preds.device());
  auto p = preds.contiguous(), t = target.contiguous(), ic = ids.contiguous(), cc = cont.contiguous();
  const int64_t B = p.size(0), P = p.size(1), total = B * P;
  auto pkey = at::empty({total}, p.options()), tkey = at::empty({total}, p.options());
  auto overflow = at::zeros({1}, p.options().dtype(at::kInt));
  if (total > 0) {
    hipLaunchKernelGGL(pq_keys_kernel, grid_for(total, 256, 256 * 8), 256, 0, stream(), p.data_ptr<int64_t>(), t.data_ptr<int64_t>(), P,
                       total, ic.data_ptr<int64_t>(), cc.data_ptr<int64_t>(), static_cast<int>(ic.numel()), pkey.data_ptr<int64_t>(),
                       tkey.data_ptr<int64_t>(), overflow.data_ptr<int>());
    TMX_LAUNCH_CHECK();
  }
  return {pkey, tkey, overflow};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("panoptic_segment_keys(Tensor preds, Tensor target, Tensor ids, Tensor cont) -> Tensor[]"); }

TORCH_LIBRARY_IMPL(tmx, CUDA, m) { m.impl("panoptic_segment_keys", &tmx::panoptic_segment_keys); }
