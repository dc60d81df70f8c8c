// Host helpers for list-state metrics.  (The per-image column concatenation of MeanAveragePrecision's batched update
// lives in csrc/py_columns.cpp: it reads the Python dicts directly.)
//
// upload_i64(host, like): a small host int64 tensor on ``like``'s device without waiting for the stream.  A
// ``torch.tensor(list, device=cuda)`` copy from pageable memory blocks the host until every kernel queued before it
// has run (~20 us idle, the whole backlog when the stream is busy); fresh pinned memory per call costs ~60 us.  Here
// one pinned staging buffer per device is reused: its previous copy is waited for by an event (long complete by the
// next call in practice), the values are memcpy'd in, and the device copy is enqueued asynchronously.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

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
