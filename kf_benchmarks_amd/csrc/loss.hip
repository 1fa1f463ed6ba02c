// Sparse softmax cross-entropy (fwd + bwd) and in-top-k accuracy.
//
// Role of tf.losses.sparse_softmax_cross_entropy + reduce_mean and
// tf.nn.in_top_k in tcb/models/model.py:285-312.  One 256-thread workgroup per
// row (1001 classes -> 4 elements per lane); the forward keeps each row's
// log-sum-exp so the backward is a single streaming pass that needs no second
// reduction: dlogits = (softmax - onehot(label)) * upstream * row_weight.
#include "common.h"

namespace kfb {

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}

template <typename T>
__global__ void __launch_bounds__(256)
xent_fwd_k(const T* __restrict__ logits, const int* __restrict__ labels, int K,
           float* __restrict__ loss, float* __restrict__ lse_out) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const T* lr = logits + row * K;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < K; j += 256) m = fmaxf(m, to_f32(lr[j]));
  m = block_max<256>(m, red);
  float s = 0.f;
  for (int j = threadIdx.x; j < K; j += 256) s += __expf(to_f32(lr[j]) - m);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float lse = m + __logf(s);
    const int lab = labels[row];
    const float tl = (lab >= 0 && lab < K) ? to_f32(lr[lab]) : NAN;
    loss[row] = lse - tl;
    lse_out[row] = lse;
  }
}

// upstream: device scalar d(total)/d(mean loss); scale applied per row (1/N).
template <typename T>
__global__ void __launch_bounds__(256)
xent_bwd_k(const T* __restrict__ logits, const int* __restrict__ labels,
           const float* __restrict__ lse, const float* __restrict__ upstream, float scale, int K,
           T* __restrict__ dlogits) {
  const long row = blockIdx.x;
  const T* lr = logits + row * K;
  T* dr = dlogits + row * K;
  const float l = lse[row];
  const float g = upstream[0] * scale;
  const int lab = labels[row];
  for (int j = threadIdx.x; j < K; j += 256) {
    float p = __expf(to_f32(lr[j]) - l);
    if (j == lab) p -= 1.f;
    dr[j] = from_f32<T>(p * g);
  }
}

// correct[row] = 1 if fewer than k logits exceed the label's logit (TF in_top_k:
// ties at the boundary count as inside).  out1/out5 for k=1 and k=5.
template <typename T>
__global__ void __launch_bounds__(256)
in_top_k_k(const T* __restrict__ logits, const int* __restrict__ labels, int K,
           float* __restrict__ out1, float* __restrict__ out5) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const T* lr = logits + row * K;
  const int lab = labels[row];
  // an out-of-range label (e.g. -1) is never "in the top k" (as xent_fwd_k,
  // which gives it a NaN loss) and reads nothing outside the row
  const float t = (lab >= 0 && lab < K) ? to_f32(lr[lab]) : NAN;
  float cnt = 0.f;
  for (int j = threadIdx.x; j < K; j += 256) cnt += (to_f32(lr[j]) > t) ? 1.f : 0.f;
  cnt = block_sum<256>(cnt, red);
  if (threadIdx.x == 0) {
    const bool finite = isfinite(t);
    out1[row] = (finite && cnt < 1.f) ? 1.f : 0.f;
    out5[row] = (finite && cnt < 5.f) ? 1.f : 0.f;
  }
}

// out[0] = mean(x[0..n)) in one workgroup (fixed summation order: the loss
// a step reports is bitwise reproducible).
__global__ void __launch_bounds__(256) mean_f32_k(const float* __restrict__ x, long n,
                                                  float* __restrict__ out) {
  __shared__ float part[4];
  float s = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((part[0] + part[1]) + (part[2] + part[3])) / (float)n;
}

}  // namespace kfb

using namespace kfb;

KFB_API hipError_t kfb_mean_f32(const float* x, long n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(mean_f32_k, dim3(1), dim3(256), 0, stream, x, n, out);
  return hipGetLastError();
}

KFB_API hipError_t kfb_xent_fwd(int dtype, const void* logits, const int* labels, long N, int K,
                                float* loss, float* lse, hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((xent_fwd_k<T>), dim3(N), dim3(256), 0, stream, (const T*)logits, labels,
                       K, loss, lse);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_xent_bwd(int dtype, const void* logits, const int* labels, const float* lse,
                                const float* upstream, float scale, long N, int K, void* dlogits,
                                hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((xent_bwd_k<T>), dim3(N), dim3(256), 0, stream, (const T*)logits, labels,
                       lse, upstream, scale, K, (T*)dlogits);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_in_top_k(int dtype, const void* logits, const int* labels, long N, int K,
                                float* out1, float* out5, hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((in_top_k_k<T>), dim3(N), dim3(256), 0, stream, (const T*)logits, labels, K,
                       out1, out5);
  });
  return hipGetLastError();
}
