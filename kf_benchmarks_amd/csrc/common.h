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

#include <atomic>
#include <tuple>
#include <type_traits>
#include <utility>

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

// ---- kernel launches (recorded for the launch tape's raw replay) ---------
// Every kernel of the library is launched through kfb::launch (the
// hipLaunchKernelGGL macro below): the arguments are converted to the
// kernel's parameter types, laid out as hipLaunchKernel's argument table, and
// while the launch tape records an entry point (tape.hip) the launch is also
// appended to that tape op - function, grid, block, LDS bytes, stream and a
// copy of the argument bytes - so a replay can re-issue it with
// hipLaunchKernel directly instead of calling the entry point again.
extern std::atomic<int> g_raw_rec;  // nonzero while a tape op records
void raw_record_launch(const void* fn, dim3 grid, dim3 block, unsigned shm, hipStream_t s,
                       void* const* argv, const size_t* sizes, int n);
void raw_record_memset(void* p, int value, size_t bytes, hipStream_t s);
void raw_taint();  // the op did device work a raw replay cannot repeat

template <typename Tup, size_t... I>
inline void launch_argv(Tup& t, void** argv, size_t* sz, std::index_sequence<I...>) {
  ((argv[I] = (void*)&std::get<I>(t), sz[I] = sizeof(std::tuple_element_t<I, Tup>)), ...);
}

template <typename... P, typename... A>
inline void launch(void (*k)(P...), dim3 grid, dim3 block, size_t shm, hipStream_t s,
                   A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  std::tuple<std::decay_t<P>...> t(static_cast<std::decay_t<P>>(std::forward<A>(a))...);
  constexpr size_t n = sizeof...(P);
  void* argv[n > 0 ? n : 1];
  size_t sz[n > 0 ? n : 1];
  launch_argv(t, argv, sz, std::index_sequence_for<P...>{});
  (void)hipLaunchKernel((const void*)k, grid, block, argv, shm, s);
  if (g_raw_rec.load(std::memory_order_relaxed))
    raw_record_launch((const void*)k, grid, block, (unsigned)shm, s, argv, sz, (int)n);
}

inline hipError_t memset_async(void* p, int value, size_t bytes, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(p, value, bytes, s);
  if (g_raw_rec.load(std::memory_order_relaxed)) raw_record_memset(p, value, bytes, s);
  return e;
}

}  // namespace kfb

#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(k, grid, block, shm, stream, ...) \
  ::kfb::launch(k, dim3(grid), dim3(block), (size_t)(shm), (hipStream_t)(stream), ##__VA_ARGS__)

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
