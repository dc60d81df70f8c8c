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
