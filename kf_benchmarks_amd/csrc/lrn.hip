// Local response normalization across channels (tf.nn.lrn semantics) on NHWC.
//
// Replaces the TF/cuDNN LRN of tcb/convnet_builder.py:463-469 (AlexNet
// CIFAR variant, tcb/models/alexnet_model.py):
//
//   s[c]  = bias + alpha * sum_{|c'-c| <= r} x[c']^2
//   y[c]  = x[c] * s[c]^-beta
//   dx[c] = dy[c] * s[c]^-beta
//           - 2 alpha beta x[c] * sum_{|c'-c| <= r} dy[c'] x[c'] s[c']^(-beta-1)
//
// A workgroup owns P whole pixels (P*C contiguous elements): coalesced
// 16-byte loads of the tile into LDS as fp32, then each thread produces
// outputs (pixel, channel) from the channel window in LDS; consecutive
// threads store consecutive elements (coalesced).  Backward stages x, then s and the
// per-element t = dy x s^(-beta-1) so the window sum of t is also an LDS
// read.
#include "common.h"

namespace kfb {

constexpr int LRN_TILE = 2048;  // fp32 elements per staged array

template <typename T>
__device__ __forceinline__ void lrn_load_tile(const T* __restrict__ src, float* dst, long base,
                                              int n) {
  // 16-byte loads when the tile base is 16-byte aligned (C % 8 == 0)
  const bool vec = (base & 7) == 0 && (((uintptr_t)src) & 15) == 0;
  for (int i = threadIdx.x * 8; i < n; i += blockDim.x * 8) {
    if (vec && i + 8 <= n) {
      float v[8];
      load_vec<T, 8>(src + base + i, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) dst[i + k] = v[k];
    } else {
      for (int k = i; k < min(i + 8, n); ++k) dst[k] = (float)src[base + k];
    }
  }
}

__device__ __forceinline__ float lrn_pow(float s, float e) {
  return e == 0.5f ? rsqrtf(s) : (e == 0.75f ? rsqrtf(s) * rsqrtf(sqrtf(s)) : __powf(s, -e));
}

template <typename T>
__global__ void __launch_bounds__(256) lrn_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                 long pixels, int C, int P, int r, float bias,
                                                 float alpha, float beta) {
  __shared__ float xs[LRN_TILE];
  const long p0 = (long)blockIdx.x * P;
  const int np = (int)min((long)P, pixels - p0);
  if (np <= 0) return;
  const int n = np * C;
  const long base = p0 * C;
  lrn_load_tile<T>(x, xs, base, n);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int px = i / C, c = i - px * C;
    const float* row = xs + px * C;
    float sq = 0.f;
    const int lo = max(c - r, 0), hi = min(c + r, C - 1);
    for (int k = lo; k <= hi; ++k) sq += row[k] * row[k];
    y[base + i] = (T)(row[c] * lrn_pow(bias + alpha * sq, beta));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) lrn_bwd_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                 T* __restrict__ dx, long pixels, int C, int P,
                                                 int r, float bias, float alpha, float beta) {
  __shared__ float xs[LRN_TILE];
  __shared__ float ts[LRN_TILE];
  __shared__ float ss[LRN_TILE];
  const long p0 = (long)blockIdx.x * P;
  const int np = (int)min((long)P, pixels - p0);
  if (np <= 0) return;
  const int n = np * C;
  const long base = p0 * C;
  lrn_load_tile<T>(x, xs, base, n);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int px = i / C, c = i - px * C;
    const float* row = xs + px * C;
    float sq = 0.f;
    const int lo = max(c - r, 0), hi = min(c + r, C - 1);
    for (int k = lo; k <= hi; ++k) sq += row[k] * row[k];
    const float s = bias + alpha * sq;
    const float g = (float)dy[base + i];
    ss[i] = s;
    ts[i] = g * row[c] * lrn_pow(s, beta) / s;  // dy x s^(-beta-1)
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int px = i / C, c = i - px * C;
    const float* trow = ts + px * C;
    float acc = 0.f;
    const int lo = max(c - r, 0), hi = min(c + r, C - 1);
    for (int k = lo; k <= hi; ++k) acc += trow[k];
    const float g = (float)dy[base + i];
    dx[base + i] = (T)(g * lrn_pow(ss[i], beta) - 2.f * alpha * beta * xs[i] * acc);
  }
}

}  // namespace kfb

using namespace kfb;

// x, y: NHWC viewed as [pixels][C]; C <= 2048.
KFB_API hipError_t kfb_lrn_fwd(int dtype, const void* x, void* y, long pixels, int C, int r,
                               float bias, float alpha, float beta, hipStream_t stream) {
  if (C <= 0 || C > LRN_TILE) return hipErrorInvalidValue;
  if (pixels <= 0) return hipSuccess;
  const int P = LRN_TILE / C;
  const dim3 grid((unsigned)((pixels + P - 1) / P));
  KFB_DISPATCH_DTYPE(dtype, T,
                     hipLaunchKernelGGL(lrn_fwd_k<T>, grid, dim3(256), 0, stream, (const T*)x,
                                        (T*)y, pixels, C, P, r, bias, alpha, beta));
  return hipGetLastError();
}

KFB_API hipError_t kfb_lrn_bwd(int dtype, const void* x, const void* dy, void* dx, long pixels,
                               int C, int r, float bias, float alpha, float beta,
                               hipStream_t stream) {
  if (C <= 0 || C > LRN_TILE) return hipErrorInvalidValue;
  if (pixels <= 0) return hipSuccess;
  const int P = LRN_TILE / C;
  const dim3 grid((unsigned)((pixels + P - 1) / P));
  KFB_DISPATCH_DTYPE(dtype, T,
                     hipLaunchKernelGGL(lrn_bwd_k<T>, grid, dim3(256), 0, stream, (const T*)x,
                                        (const T*)dy, (T*)dx, pixels, C, P, r, bias, alpha, beta));
  return hipGetLastError();
}
