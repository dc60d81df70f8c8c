// Row-list helpers for list-state metrics (host C++, any device).
//
// ``cat_rows(items, width)``: the dim-0 concatenation of per-item tensors (MeanAveragePrecision's per-image boxes /
// scores / labels, reference ``detection/mean_ap.py:458-499``) together with every item's row count, validated in C++:
// every item on one device, of one dtype, 1-d (width 0) or [k, width].  A Python-side check of 512 items x 5 columns
// (shape, dtype and device attribute reads) cost ~1 ms per update; here it is one pass over the item list.
// When the items are consecutive contiguous row blocks of ONE storage -- a batch tensor indexed per image, the usual
// shape of a detection data loader's output -- the result is a view of that storage (no copy, no kernel);
// otherwise one at::cat.  Returns (flat, sizes int64 [n] on the host); empty tensors mean the items are not
// uniform (the caller takes its per-item path, which raises the reference's errors).
#include <ATen/ATen.h>
#include <torch/library.h>

#include <tuple>
#include <vector>

namespace tmx {

std::tuple<at::Tensor, at::Tensor> cat_rows(const std::vector<at::Tensor>& items, int64_t width) {
  auto sizes = at::empty({static_cast<int64_t>(items.size())}, at::kLong);
  const std::tuple<at::Tensor, at::Tensor> refuse = {at::empty({0}), at::empty({0}, at::kLong)};
  if (items.empty()) return refuse;
  int64_t* sz = sizes.data_ptr<int64_t>();
  const at::Tensor& first = items[0];
  const auto dtype = first.scalar_type();
  const auto device = first.device();
  const int64_t want_dim = width > 0 ? 2 : 1;
  const int64_t esize = first.element_size();
  const int64_t row_bytes = (width > 0 ? width : 1) * esize;
  // consecutive row blocks of one storage?
  bool chained = true;
  const void* storage = first.defined() ? first.storage().data() : nullptr;
  const char* next = nullptr;
  int64_t total = 0;
  for (size_t i = 0; i < items.size(); ++i) {
    const at::Tensor& t = items[i];
    if (!t.defined() || t.scalar_type() != dtype || t.device() != device || t.dim() != want_dim || t.requires_grad() ||
        (width > 0 && t.size(1) != width))
      return refuse;
    const int64_t k = t.size(0);
    if (k == 0) return refuse;  // (empty images take the per-item path, as before)
    sz[i] = k;
    total += k;
    if (chained) {
      const char* p = static_cast<const char*>(t.data_ptr());
      chained = t.is_contiguous() && t.storage().data() == storage && (i == 0 || p == next);
      next = p + k * row_bytes;
    }
  }
  if (chained) {
    std::vector<int64_t> shape = {total};
    if (width > 0) shape.push_back(width);
    std::vector<int64_t> stride = {width > 0 ? width : 1};
    if (width > 0) stride.push_back(1);
    return {first.as_strided(shape, stride, first.storage_offset()), sizes};
  }
  return {at::cat(items, 0), sizes};
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("cat_rows(Tensor[] items, int width) -> (Tensor, Tensor)"); }
TORCH_LIBRARY_IMPL(tmx, CompositeExplicitAutograd, m) { m.impl("cat_rows", &tmx::cat_rows); }

// ---------------------------------------------------------------------------------------------------------------
// upload_i64(host, like): a small host int64 tensor on ``like``'s device without waiting for the stream.  A
// ``torch.tensor(list, device=cuda)`` copy from pageable memory blocks the host until every kernel queued before it
// has run (~20 us idle, the whole backlog when the stream is busy); fresh pinned memory per call costs ~60 us.  Here
// one pinned staging buffer per device is reused: its previous copy is waited for by an event (long complete by the
// next call in practice), the values are memcpy'd in, and the device copy is enqueued asynchronously.
#include <hip/hip_runtime.h>
#include <c10/hip/HIPStream.h>

#include <cstring>
#include <mutex>
#include <unordered_map>

namespace tmx {

namespace {
struct Staging {
  void* buf = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
};
}  // namespace

at::Tensor upload_i64(const at::Tensor& host, const at::Tensor& like) {
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == at::kLong, "upload_i64: expected a host int64 tensor");
  auto src = host.contiguous();
  const int64_t n = src.numel();
  auto out = at::empty(src.sizes(), like.options().dtype(at::kLong));
  if (n == 0 || !like.is_cuda()) return like.is_cuda() ? out : src.clone();
  static std::mutex mu;
  static std::unordered_map<int, Staging> stage;
  std::lock_guard<std::mutex> lock(mu);
  const c10::DeviceGuard guard(like.device());
  Staging& st = stage[like.device().index()];
  const size_t bytes = static_cast<size_t>(n) * sizeof(int64_t);
  if (st.pending) {
    C10_HIP_CHECK(hipEventSynchronize(st.done));
    st.pending = false;
  }
  if (st.cap < bytes) {
    if (st.buf != nullptr) C10_HIP_CHECK(hipHostFree(st.buf));
    st.cap = std::max<size_t>(bytes, 1 << 16);
    C10_HIP_CHECK(hipHostMalloc(&st.buf, st.cap, hipHostMallocDefault));
  }
  if (st.done == nullptr) C10_HIP_CHECK(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
  std::memcpy(st.buf, src.data_ptr<int64_t>(), bytes);
  const hipStream_t s = c10::hip::getCurrentHIPStream().stream();
  C10_HIP_CHECK(hipMemcpyAsync(out.data_ptr<int64_t>(), st.buf, bytes, hipMemcpyHostToDevice, s));
  C10_HIP_CHECK(hipEventRecord(st.done, s));
  st.pending = true;
  return out;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) { m.def("upload_i64(Tensor host, Tensor like) -> Tensor"); }
TORCH_LIBRARY_IMPL(tmx, CompositeExplicitAutograd, m) { m.impl("upload_i64", &tmx::upload_i64); }
