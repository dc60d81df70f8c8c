// How fast does the host learn that the stream's last kernel finished?  (round 5: the headline's compute window ends
// in one flag read -- csrc/flags.hip gather_flags writes the flags into mapped pinned memory, then the host waits.)
// Each trial queues a ~200 us busy kernel then a one-wave "flag" kernel that writes a sequence number into pinned host
// memory; the host then waits by (a) hipStreamSynchronize, (b) hipEventSynchronize, (c) a hipStreamQuery spin,
// (d) spinning on the pinned word (the kernel's store follows a system-scope fence).  The busy kernel's duration is the
// same in every mode, so the median wall differences are the wake-up latency differences.
// Build: hipcc -O3 --offload-arch=gfx950 tools/kexp/sync_latency_exp.hip -o build/kexp_r5/sync_latency_exp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(err_), __FILE__, __LINE__); exit(1); } } while (0)

__global__ void busy_kernel(long long ticks, int* sink) {
  const long long t0 = wall_clock64();
  int acc = 0;
  while (wall_clock64() - t0 < ticks) acc += threadIdx.x;
  if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void flag_kernel(int* host_word, int seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(host_word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 100;
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const int busy_us = argc > 2 ? atoi(argv[2]) : 200;
  const long long ticks = static_cast<long long>(rate_khz) * busy_us / 1000;
  int* sink;
  CK(hipMalloc(&sink, 64));
  int* host_word;
  CK(hipHostMalloc(&host_word, 64, hipHostMallocMapped));
  int* dev_word;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_word), host_word, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names[] = {"stream_sync", "event_sync", "query_spin", "pinned_spin"};
  int seq = 0;
  for (int warm = 0; warm < 5; ++warm) {
    hipLaunchKernelGGL(busy_kernel, 1, 64, 0, s, ticks, sink);
    hipLaunchKernelGGL(flag_kernel, 1, 64, 0, s, dev_word, ++seq);
    CK(hipStreamSynchronize(s));
  }
  printf("{\"busy_us\": %d, \"trials\": %d", busy_us, trials);
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> t;
    for (int k = 0; k < trials; ++k) {
      const int want = ++seq;
      const double t0 = now_us();
      hipLaunchKernelGGL(busy_kernel, 1, 64, 0, s, ticks, sink);
      hipLaunchKernelGGL(flag_kernel, 1, 64, 0, s, dev_word, want);
      if (mode == 0) {
        CK(hipStreamSynchronize(s));
      } else if (mode == 1) {
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
      } else if (mode == 2) {
        while (hipStreamQuery(s) == hipErrorNotReady) {
        }
      } else {
        const double deadline = t0 + 100000.0;
        while (__atomic_load_n(host_word, __ATOMIC_ACQUIRE) != want) {
          if (now_us() > deadline) { printf("\n pinned spin timed out\n"); exit(1); }
        }
      }
      t.push_back(now_us() - t0);
      CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    printf(", \"%s_us_median\": %.1f, \"%s_us_p10\": %.1f", names[mode], t[t.size() / 2], names[mode], t[t.size() / 10]);
  }
  // idle stream: one flag kernel alone
  for (int mode = 0; mode < 4; mode += 3) {
    std::vector<double> t;
    for (int k = 0; k < trials; ++k) {
      const int want = ++seq;
      const double t0 = now_us();
      hipLaunchKernelGGL(flag_kernel, 1, 64, 0, s, dev_word, want);
      if (mode == 0) {
        CK(hipStreamSynchronize(s));
      } else {
        while (__atomic_load_n(host_word, __ATOMIC_ACQUIRE) != want) {
        }
      }
      t.push_back(now_us() - t0);
      CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    printf(", \"idle_%s_us_median\": %.1f", names[mode], t[t.size() / 2]);
  }
  printf("}\n");
  return 0;
}
