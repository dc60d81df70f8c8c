// Device-only helpers shared by every gfx950 kernel (no torch headers: also used by standalone harnesses).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <cstdint>

namespace tmx {

constexpr int kWave = 64;  // CDNA wavefront width


inline int grid_for(int64_t work, int block, int max_blocks = 256 * 8) {
  int64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return static_cast<int>(g);
}


// ---------------------------------------------------------------------------------------------- scalar I/O
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<double>(double v) { return static_cast<float>(v); }
template <> __device__ __forceinline__ float to_f32<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }
template <> __device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }

// Raw 16-bit pattern of an element (only meaningful for 16-bit float types).
template <typename T> __device__ __forceinline__ uint16_t bits16(T v);
template <> __device__ __forceinline__ uint16_t bits16<__hip_bfloat16>(__hip_bfloat16 v) {
  return *reinterpret_cast<const uint16_t*>(&v);
}
template <> __device__ __forceinline__ uint16_t bits16<__half>(__half v) { return *reinterpret_cast<const uint16_t*>(&v); }

// Round an fp32 value to T with round-to-nearest-even and return its bit pattern (16-bit types).
template <typename T> __device__ __forceinline__ uint16_t round_bits16(float v);
template <> __device__ __forceinline__ uint16_t round_bits16<__hip_bfloat16>(float v) {
  __hip_bfloat16 b = __float2bfloat16(v);  // RNE
  return *reinterpret_cast<const uint16_t*>(&b);
}
template <> __device__ __forceinline__ uint16_t round_bits16<__half>(float v) {
  __half h = __float2half_rn(v);
  return *reinterpret_cast<const uint16_t*>(&h);
}

// Round fp32 -> T -> fp32 (emulates torch computing an op in fp32 and storing it in the input dtype).
template <typename T> __device__ __forceinline__ float round_trip(float v) { return v; }
template <> __device__ __forceinline__ float round_trip<__hip_bfloat16>(float v) { return __bfloat162float(__float2bfloat16(v)); }
template <> __device__ __forceinline__ float round_trip<__half>(float v) { return __half2float(__float2half_rn(v)); }

// --------------------------------------------------------------------------------------------- wave ops
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ __forceinline__ long long wave_sum(long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
  return v;
}

// (value, index) arg-max reduction across a wave; ties -> lowest index, NaN counts as +inf-beyond-inf.
__device__ __forceinline__ void wave_argmax(float& v, int& idx) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float ov = __shfl_xor(v, off, kWave);
    int oi = __shfl_xor(idx, off, kWave);
    bool o_nan = ov != ov, s_nan = v != v;
    // NaN beats numbers; between two NaNs (or equal numbers) the lower index wins, so every lane ends with the
    // same (value, index) — the first NaN, as torch.argmax returns
    bool take = (o_nan && !s_nan) || (o_nan == s_nan && (o_nan ? oi < idx : (ov > v || (ov == v && oi < idx))));
    if (take) { v = ov; idx = oi; }
  }
}

__device__ __forceinline__ bool argmax_better(float cand, int ci, float best, int bi) {
  bool c_nan = cand != cand, b_nan = best != best;
  if (c_nan != b_nan) return c_nan;
  return cand > best || (cand == best && ci < bi);
}

__device__ __forceinline__ void atomic_add_i64(int64_t* p, long long v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(v));
}

}  // namespace tmx
