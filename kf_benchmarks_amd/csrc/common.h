// Shared helpers for the kf_benchmarks_amd gfx950 kernels.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC, viewed as a [rows, C] matrix (rows = N*H*W);
//   * element type codes: 0 = fp32, 1 = bf16, 2 = fp16 (must match ops/_native.py);
//   * all entry points are extern "C", take raw device pointers plus the
//     hipStream_t of the caller's current torch stream, and return hipError_t
//     of the launch so the Python side can fail loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KFB_API extern "C" __attribute__((visibility("default")))

namespace kfb {

enum DType : int { F32 = 0, BF16 = 1, F16 = 2 };

// n / d for 0 <= n < 2^31 as a multiply-high and a shift (round-up
// multiplier method): the gather maps divide every chunk's row and k index on
// every K step (conv_f32.hip, the generic igemm_k loader), and a true 32-bit
// division costs tens of VALU instructions.
struct FastDiv {
  unsigned d, mul, shift;
  FastDiv() = default;
  __host__ explicit FastDiv(int dv) : d((unsigned)dv), mul(0), shift(0) {
    while ((1u << shift) < d) ++shift;
    mul = (unsigned)(((1ull << 32) * ((1ull << shift) - d)) / d + 1);
  }
  __device__ __forceinline__ int div(int n) const {
    return (int)((__umulhi((unsigned)n, mul) + (unsigned)n) >> shift);
  }
};

typedef __bf16 bf16;
typedef _Float16 f16;

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

// 16-byte vector of T: the unit every streaming kernel moves per lane.
template <typename T, int N> struct alignas(sizeof(T) * N) Vec { T v[N]; };

template <typename T, int N>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&out)[N]) {
  Vec<T, N> r = *reinterpret_cast<const Vec<T, N>*>(p);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = to_f32(r.v[i]);
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float (&in)[N]) {
  Vec<T, N> r;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = from_f32<T>(in[i]);
  *reinterpret_cast<Vec<T, N>*>(p) = r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Largest vector width (elements) in {8,4,2,1} dividing C.
inline int vec_width(int C) { return (C % 8 == 0) ? 8 : (C % 4 == 0) ? 4 : (C % 2 == 0) ? 2 : 1; }

}  // namespace kfb

// Dispatch a templated launcher over the element type.
#define KFB_DISPATCH_DTYPE(code, T, ...)            \
  switch (code) {                                   \
    case kfb::F32: { typedef float T; __VA_ARGS__; break; } \
    case kfb::BF16: { typedef kfb::bf16 T; __VA_ARGS__; break; } \
    case kfb::F16: { typedef kfb::f16 T; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;           \
  }

#define KFB_DISPATCH_VEC(vw, V, ...)                \
  switch (vw) {                                     \
    case 8: { constexpr int V = 8; __VA_ARGS__; break; } \
    case 4: { constexpr int V = 4; __VA_ARGS__; break; } \
    case 2: { constexpr int V = 2; __VA_ARGS__; break; } \
    default: { constexpr int V = 1; __VA_ARGS__; break; } \
  }
