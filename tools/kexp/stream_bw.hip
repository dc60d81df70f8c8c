// STREAM-style HBM / Infinity-Cache bandwidth floor on MI355X (gfx950): the measured ceiling the headline curve
// kernels are compared against (VERDICT r3 "measure the floor").  Standalone, no torch.
//   read      : 16-B vector loads, one wave-reduced word stored per workgroup
//   write     : 16-B vector stores
//   copy      : 16-B load + 16-B store (the row pass's shape: logits in, class-major codes out)
//   copy+read : copy A -> B, then read B (the class pass re-reading the codes the row pass just wrote)
// Each is timed over sizes inside and beyond the 256 MiB Infinity Cache, grid = k * 256 CUs, 20 iterations, after
// 3 warm-up launches.  Rotating buffers (NBUF of them) keep "beyond cache" honest for the streamed operand.
// Build: hipcc -O3 --offload-arch=gfx950 tools/kexp/stream_bw.hip -o build/stream_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const uint4* __restrict__ a, int64_t nv, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += U * stride) {
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * stride;
      if (j < nv) {
        if constexpr (NT) {
          using v4u = __attribute__((ext_vector_type(4))) unsigned int;
          const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a + j));
          w[u] = make_uint4(v.x, v.y, v.z, v.w);
        } else {
          w[u] = a[j];
        }
      } else {
        w[u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;  // keeps the loads alive; practically never stores
}

template <int U>
__global__ void __launch_bounds__(256) write_kernel(uint4* __restrict__ b, int64_t nv, uint32_t seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * stride;
      if (j < nv) b[j] = make_uint4(seed, (uint32_t)j, seed ^ 1u, (uint32_t)(j >> 32));
    }
  }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, int64_t nv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += U * stride) {
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * stride;
      if (j < nv) {
        if constexpr (NT) {
          using v4u = __attribute__((ext_vector_type(4))) unsigned int;
          const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a + j));
          w[u] = make_uint4(v.x, v.y, v.z, v.w);
        } else {
          w[u] = a[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + u * stride;
      if (j < nv) b[j] = make_uint4(w[u].y, w[u].x, w[u].w, w[u].z);
    }
  }
}

template <typename F>
static float time_us(F f, int iters = 20) {
  for (int i = 0; i < 3; ++i) f(i);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f(i);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms * 1000.f / iters;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int64_t sizes[] = {int64_t(131072000), int64_t(262144000), int64_t(1) << 30};  // 131 MB = 65536 x 1000 bf16
  const int NBUF = 4;                                                                 // rotating inputs (like bench.py's pool)
  const int64_t maxb = int64_t(1) << 30;
  std::vector<uint4*> src(NBUF);
  for (int k = 0; k < NBUF; ++k) {
    CK(hipMalloc(&src[k], maxb));
    CK(hipMemset(src[k], k + 1, maxb));
  }
  uint4* dst;
  CK(hipMalloc(&dst, maxb));
  CK(hipMemset(dst, 0, maxb));
  uint32_t* sink;
  CK(hipMalloc(&sink, 1 << 20));
  printf("{\"device\": \"%s\", \"cus\": %d, \"results\": [\n", prop.name, cus);
  bool first = true;
  auto emit = [&](const char* op, int64_t bytes_operand, int64_t moved, int grid_mult, const char* variant, float us) {
    printf("%s  {\"op\": \"%s\", \"variant\": \"%s\", \"operand_MB\": %.1f, \"bytes_moved_MB\": %.1f, \"grid\": %d, \"us\": %.2f, \"TB_s\": %.3f}",
           first ? "" : ",\n", op, variant, bytes_operand / 1e6, moved / 1e6, grid_mult * cus, us, moved / (us * 1e-6) / 1e12);
    first = false;
  };
  for (int64_t bytes : sizes) {
    const int64_t nv = bytes / 16;
    for (int gm : {4, 8, 16}) {
      const int grid = gm * cus;
      float us = time_us([&](int i) { read_kernel<4, false><<<grid, 256>>>(src[i % NBUF], nv, sink); });
      emit("read", bytes, bytes, gm, "rotating-4", us);
      us = time_us([&](int i) { read_kernel<4, true><<<grid, 256>>>(src[i % NBUF], nv, sink); });
      emit("read", bytes, bytes, gm, "rotating-4-nt", us);
      us = time_us([&](int) { read_kernel<4, false><<<grid, 256>>>(src[0], nv, sink); });
      emit("read", bytes, bytes, gm, "same-buffer", us);
      us = time_us([&](int i) { write_kernel<4><<<grid, 256>>>(dst, nv, (uint32_t)i); });
      emit("write", bytes, bytes, gm, "same-buffer", us);
      us = time_us([&](int i) { copy_kernel<4, false><<<grid, 256>>>(src[i % NBUF], dst, nv); });
      emit("copy", bytes, 2 * bytes, gm, "rotating-4", us);
      us = time_us([&](int i) { copy_kernel<4, true><<<grid, 256>>>(src[i % NBUF], dst, nv); });
      emit("copy", bytes, 2 * bytes, gm, "rotating-4-nt-load", us);
      us = time_us([&](int i) {
        copy_kernel<4, true><<<grid, 256>>>(src[i % NBUF], dst, nv);
        read_kernel<4, false><<<grid, 256>>>(dst, nv, sink);
      });
      emit("copy+read", bytes, 3 * bytes, gm, "rotating-4-nt-load", us);
    }
  }
  printf("\n]}\n");
  CK(hipDeviceSynchronize());
  for (auto p : src) CK(hipFree(p));
  CK(hipFree(dst));
  CK(hipFree(sink));
  return 0;
}
