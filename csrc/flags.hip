// One read of every host-side check of a compute() (utilities/validation.py HostCheckBatch): the deferred input
// flags, the degenerate-class warning flags and the NaN-class flags of the averages are small device tensors of
// assorted dtypes.  Converting and concatenating them with ATen took one kernel per flag plus a cat (~10 launches of
// ~4 us each in the headline's compute window); here ONE kernel reads every flag (descriptors passed by value in
// the kernel arguments), writes them as int32 into one buffer and zeroes the flags the caller consumes, then one
// device->host copy into a pinned buffer and a stream synchronisation.
#include "common.h"

#include <mutex>
#include <vector>

namespace tmx {

constexpr int kMaxFlagDescs = 48;

struct FlagDesc {
  const void* ptr;
  int32_t dtype;  // 0 bool/u8, 1 int32, 2 int64, 3 f32, 4 f64, 5 f16, 6 bf16
  int32_t numel;
  int32_t out_off;
  int32_t zero;
};

struct FlagArgs {
  FlagDesc d[kMaxFlagDescs];
  int32_t n;
};

__device__ __forceinline__ int32_t flag_value(const FlagDesc& f, int j) {
  switch (f.dtype) {
    case 0: return static_cast<int32_t>(static_cast<const uint8_t*>(f.ptr)[j]);
    case 1: return static_cast<const int32_t*>(f.ptr)[j];
    case 2: return static_cast<int32_t>(static_cast<const int64_t*>(f.ptr)[j]);
    case 3: return static_cast<int32_t>(static_cast<const float*>(f.ptr)[j]);
    case 4: return static_cast<int32_t>(static_cast<const double*>(f.ptr)[j]);
    case 5: return static_cast<int32_t>(__half2float(static_cast<const __half*>(f.ptr)[j]));
    default: return static_cast<int32_t>(static_cast<float>(static_cast<const __hip_bfloat16*>(f.ptr)[j]));
  }
}

__device__ __forceinline__ void flag_clear(const FlagDesc& f, int j) {
  switch (f.dtype) {
    case 0: static_cast<uint8_t*>(const_cast<void*>(f.ptr))[j] = 0; break;
    case 1: static_cast<int32_t*>(const_cast<void*>(f.ptr))[j] = 0; break;
    case 2: static_cast<int64_t*>(const_cast<void*>(f.ptr))[j] = 0; break;
    case 3: static_cast<float*>(const_cast<void*>(f.ptr))[j] = 0.f; break;
    case 4: static_cast<double*>(const_cast<void*>(f.ptr))[j] = 0.0; break;
    case 5: static_cast<__half*>(const_cast<void*>(f.ptr))[j] = __float2half(0.f); break;
    default: static_cast<__hip_bfloat16*>(const_cast<void*>(f.ptr))[j] = __float2bfloat16(0.f); break;
  }
}

// one wave: lane l walks the flat element list with stride 64; a flag shared by two descriptors (two metrics attached
// to one kernel-written word) is read by both before any clear: all reads, a wave barrier, then the clears
// (read == 0: a clear-only launch, issued after every read launch when the descriptors span several launches)
__global__ void __launch_bounds__(kWave) gather_flags_kernel(FlagArgs args, int32_t read, int32_t* __restrict__ out) {
  if (read) {
    for (int k = 0; k < args.n; ++k) {
      const FlagDesc& f = args.d[k];
      for (int j = threadIdx.x; j < f.numel; j += kWave) out[f.out_off + j] = flag_value(f, j);
    }
    __syncthreads();
  }
  for (int k = 0; k < args.n; ++k) {
    const FlagDesc& f = args.d[k];
    if (!f.zero) continue;
    for (int j = threadIdx.x; j < f.numel; j += kWave) flag_clear(f, j);
  }
}

static int32_t flag_dtype(at::ScalarType t) {
  switch (t) {
    case at::kBool: case at::kByte: return 0;
    case at::kInt: return 1;
    case at::kLong: return 2;
    case at::kFloat: return 3;
    case at::kDouble: return 4;
    case at::kHalf: return 5;
    case at::kBFloat16: return 6;
    default: TORCH_CHECK(false, "gather_flags: unsupported flag dtype ", t);
  }
  return -1;
}

// flags: device tensors on one device (any shape); zero[i]: clear flags[i] after reading it (contiguous flags only).
// Device int32 tensor with every flag's elements in order; one launch per 48 flags, no host synchronisation.
// One launch per 48 flags: every flag's elements, in order, as int32 at out (device-visible memory).  A flag tensor
// may appear twice (two metrics attached to one kernel-written word, or one sink registered for its errors and its
// warnings): within one launch the kernel reads before it clears; when the list spans several launches, the read
// launches clear nothing and clear-only launches follow them, so no descriptor sees a flag another one consumed.
static void launch_gather(at::TensorList flags, c10::IntArrayRef zero, int64_t total, int32_t* out) {
  const at::Device dev = flags[0].device();
  std::vector<at::Tensor> keep;  // contiguous views (a non-contiguous flag is read from a copy; it is never cleared then)
  keep.reserve(flags.size());
  const bool split = flags.size() > static_cast<size_t>(kMaxFlagDescs);
  std::vector<FlagArgs> clears;
  int64_t off = 0;
  size_t i = 0;
  while (i < flags.size()) {
    FlagArgs args{};
    args.n = 0;
    while (i < flags.size() && args.n < kMaxFlagDescs) {
      const at::Tensor& f = flags[i];
      TORCH_CHECK(f.device() == dev, "gather_flags: flags on different devices");
      TORCH_CHECK(f.numel() < (int64_t{1} << 30), "gather_flags: flag too large");
      keep.push_back(f.is_contiguous() ? f : f.contiguous());
      FlagDesc& d = args.d[args.n++];
      d.ptr = keep.back().data_ptr();
      d.dtype = flag_dtype(f.scalar_type());
      d.numel = static_cast<int32_t>(f.numel());
      d.out_off = static_cast<int32_t>(off);
      d.zero = zero[i] != 0 && f.is_contiguous();
      off += f.numel();
      ++i;
    }
    if (split) {
      clears.push_back(args);
      for (int k = 0; k < args.n; ++k) args.d[k].zero = 0;
    }
    hipLaunchKernelGGL(gather_flags_kernel, 1, kWave, 0, stream(), args, 1, out);
    TMX_LAUNCH_CHECK();
  }
  (void)total;
  for (const FlagArgs& c : clears) {
    hipLaunchKernelGGL(gather_flags_kernel, 1, kWave, 0, stream(), c, 0, out);
    TMX_LAUNCH_CHECK();
  }
}

// flags: device tensors on one device (any shape); zero[i]: clear flags[i] after reading it (contiguous flags only).
// Device int32 tensor with every flag's elements in order; one launch per 48 flags, no host synchronisation.
at::Tensor gather_flags_device(at::TensorList flags, c10::IntArrayRef zero) {
  TORCH_CHECK(flags.size() == zero.size(), "gather_flags: one zero entry per flag");
  TORCH_CHECK(!flags.empty(), "gather_flags: no flags");
  int64_t total = 0;
  for (const at::Tensor& f : flags) total += f.numel();
  const at::Device dev = flags[0].device();
  TORCH_CHECK(dev.is_cuda(), "gather_flags: device tensors only");
  const c10::DeviceGuard guard(dev);
  auto out = at::empty({total}, at::TensorOptions().dtype(at::kInt).device(dev));
  if (total == 0) return out;
  launch_gather(flags, zero, total, out.data_ptr<int32_t>());
  return out;
}

// flags[i] |= src[off_i ...] for every flag (the inverse of a zeroing gather: forward() puts the accumulated flags
// back after its batch compute), one launch.
__global__ void __launch_bounds__(kWave) or_flags_kernel(FlagArgs args, const int32_t* __restrict__ src) {
  for (int k = 0; k < args.n; ++k) {
    const FlagDesc& f = args.d[k];
    for (int j = threadIdx.x; j < f.numel; j += kWave) {
      const int32_t v = src[f.out_off + j];
      if (v == 0) continue;
      switch (f.dtype) {
        case 0: static_cast<uint8_t*>(const_cast<void*>(f.ptr))[j] |= static_cast<uint8_t>(v); break;
        case 1: static_cast<int32_t*>(const_cast<void*>(f.ptr))[j] |= v; break;
        case 2: static_cast<int64_t*>(const_cast<void*>(f.ptr))[j] |= v; break;
        default: break;  // float flags are never restored (they are computed, not accumulated)
      }
    }
  }
}

void or_flags(at::TensorList flags, const at::Tensor& src) {
  if (flags.empty()) return;
  const at::Device dev = flags[0].device();
  TORCH_CHECK(dev.is_cuda() && src.device() == dev && src.scalar_type() == at::kInt && src.is_contiguous(),
              "or_flags: int32 source on the flags' device");
  const c10::DeviceGuard guard(dev);
  int64_t off = 0;
  size_t i = 0;
  while (i < flags.size()) {
    FlagArgs args{};
    args.n = 0;
    while (i < flags.size() && args.n < kMaxFlagDescs) {
      const at::Tensor& f = flags[i];
      TORCH_CHECK(f.device() == dev && f.is_contiguous(), "or_flags: contiguous flags on one device");
      FlagDesc& d = args.d[args.n++];
      d.ptr = f.data_ptr();
      d.dtype = flag_dtype(f.scalar_type());
      d.numel = static_cast<int32_t>(f.numel());
      d.out_off = static_cast<int32_t>(off);
      d.zero = 0;
      off += f.numel();
      ++i;
    }
    TORCH_CHECK(off <= src.numel(), "or_flags: source too short");
    hipLaunchKernelGGL(or_flags_kernel, 1, kWave, 0, stream(), args, src.data_ptr<int32_t>());
    TMX_LAUNCH_CHECK();
  }
}

// The same gather written straight into pinned host memory (mapped into the device's address space: no separate
// device->host copy launch), then a stream synchronisation: a CPU int32 tensor.  Falls back to a device buffer + copy
// when the pinned block has no device mapping.
at::Tensor gather_flags(at::TensorList flags, c10::IntArrayRef zero) {
  int64_t total = 0;
  for (const at::Tensor& f : flags) total += f.numel();
  auto host = at::empty({total}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
  if (total == 0) return host;
  TORCH_CHECK(flags.size() == zero.size(), "gather_flags: one zero entry per flag");
  TORCH_CHECK(flags[0].is_cuda(), "gather_flags: device tensors only");
  const c10::DeviceGuard guard(flags[0].device());
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, host.data_ptr(), 0) == hipSuccess && dptr != nullptr) {
    launch_gather(flags, zero, total, static_cast<int32_t*>(dptr));
  } else {
    (void)hipGetLastError();  // clear the failed lookup
    const at::Tensor out = gather_flags_device(flags, zero);
    TMX_CHECK_HIP(hipMemcpyAsync(host.data_ptr<int32_t>(), out.data_ptr<int32_t>(), total * sizeof(int32_t), hipMemcpyDeviceToHost,
                                 stream()));
  }
  TMX_CHECK_HIP(hipStreamSynchronize(stream()));
  return host;
}

// gather_flags without the synchronisation: the caller records an event after it and reads the pinned result once the
// event has completed (forward()'s parked warning flags: no pipeline drain every few dozen forwards)
at::Tensor gather_flags_async(at::TensorList flags, c10::IntArrayRef zero) {
  int64_t total = 0;
  for (const at::Tensor& f : flags) total += f.numel();
  auto host = at::empty({total}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
  if (total == 0) return host;
  TORCH_CHECK(flags.size() == zero.size(), "gather_flags_async: one zero entry per flag");
  TORCH_CHECK(flags[0].is_cuda(), "gather_flags_async: device tensors only");
  const c10::DeviceGuard guard(flags[0].device());
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, host.data_ptr(), 0) == hipSuccess && dptr != nullptr) {
    launch_gather(flags, zero, total, static_cast<int32_t*>(dptr));
  } else {
    (void)hipGetLastError();
    const at::Tensor out = gather_flags_device(flags, zero);
    TMX_CHECK_HIP(hipMemcpyAsync(host.data_ptr<int32_t>(), out.data_ptr<int32_t>(), total * sizeof(int32_t), hipMemcpyDeviceToHost,
                                 stream()));
  }
  return host;
}

}  // namespace tmx

TORCH_LIBRARY_FRAGMENT(tmx, m) {
  m.def("gather_flags_async(Tensor[] flags, int[] zero) -> Tensor");
  m.def("gather_flags(Tensor[] flags, int[] zero) -> Tensor");
  m.def("gather_flags_device(Tensor[] flags, int[] zero) -> Tensor");
  m.def("or_flags(Tensor(a!)[] flags, Tensor src) -> ()");
}

TORCH_LIBRARY_IMPL(tmx, CUDA, m) {
  m.impl("gather_flags", &tmx::gather_flags);
  m.impl("gather_flags_async", &tmx::gather_flags_async);
  m.impl("gather_flags_device", &tmx::gather_flags_device);
  m.impl("or_flags", &tmx::or_flags);
}
