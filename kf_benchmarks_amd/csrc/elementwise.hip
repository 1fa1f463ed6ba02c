// Elementwise / small-reduction kernels for the non-BN layers.
//
//   bias_act_fwd     y = act(x + b)            conv/affine bias + relu
//                                               (tcb/convnet_builder.py:188-213, 311-345)
//   act_bwd_bias     dx = dy * relu'(y); db += colsum(dx)
//   dropout fwd/bwd  counter-based hash RNG: the mask is recomputed from
//                    (seed, index) in the backward, nothing is stored
//                    (tcb/convnet_builder.py:396-406)
//   synthetic_fill   truncated normal(127, 60) images + uniform labels, made on
//                    device (tcb/models/model.py:220-237)
//   add              y = a + b (+relu)
#include "common.h"
#include <cstdlib>

namespace kfb {

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  // lowbias32 (Wellons) - good avalanche, 6 ops.
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float u01(uint32_t seed, uint64_t i, uint32_t stream) {
  uint32_t h = hash_u32((uint32_t)i ^ hash_u32(seed + 0x9e3779b9U * stream) ^
                        hash_u32((uint32_t)(i >> 32) + 0x85ebca6bU));
  return ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T, int V, bool RELU>
__global__ void __launch_bounds__(256)
bias_act_k(const T* __restrict__ x, const float* __restrict__ b, T* __restrict__ y, long nvec,
           int C) {
  const unsigned cv = (unsigned)(C / V);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < (unsigned)nvec;
       i += gridDim.x * blockDim.x) {
    const long e = (long)i * V;
    const int c = (int)(i % cv) * V;
    float v[V];
    load_vec<T, V>(x + e, v);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float o = v[k] + (b ? b[c + k] : 0.f);
      v[k] = RELU ? fmaxf(o, 0.f) : o;
    }
    store_vec<T, V>(y + e, v);
  }
}

// dx = dy * (y > 0) [if RELU]; partial column sums of dx into pbias[blockIdx.x][C].
// Grid: (nslab, nchunk) with a window of 256*V/... like the BN partial kernels:
// each block owns cw channels and a slab of rows.
template <typename T, int V, bool RELU>
__global__ void __launch_bounds__(256)
act_bwd_bias_k(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long rows,
               int C, int cw, int tpr, int rpi, long slab_rows, float* __restrict__ pbias) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int t = tid % tpr, r = tid / tpr;
  const int c0 = blockIdx.y * cw + t * V;
  const bool cok = (c0 < C) && (r < rpi);
  float s[V];
#pragma unroll
  for (int k = 0; k < V; ++k) s[k] = 0.f;
  const long rbeg = (long)blockIdx.x * slab_rows;
  long rend = rbeg + slab_rows;
  if (rend > rows) rend = rows;
  if (cok) {
    for (long row = rbeg + r; row < rend; row += rpi) {
      const long off = row * C + c0;
      float g[V];
      load_vec<T, V>(dy + off, g);
      if (RELU) {
        float yv[V];
        load_vec<T, V>(y + off, yv);
#pragma unroll
        for (int k = 0; k < V; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
        if (dx) store_vec<T, V>(dx + off, g);
      }
#pragma unroll
      for (int k = 0; k < V; ++k) s[k] += g[k];
    }
  }
  if (pbias) {
    if (r < rpi) {
#pragma unroll
      for (int k = 0; k < V; ++k) lds[(r * tpr + t) * V + k] = s[k];
    }
    __syncthreads();
    if (r == 0 && c0 < C) {
      for (int rr = 1; rr < rpi; ++rr)
#pragma unroll
        for (int k = 0; k < V; ++k) s[k] += lds[(rr * tpr + t) * V + k];
#pragma unroll
      for (int k = 0; k < V; ++k) pbias[(long)blockIdx.x * C + c0 + k] = s[k];
    }
  }
}

// out[c] (+)= sum_k p[k][c].  16 channels x 16 slab groups per workgroup:
// each thread strides over the slabs with four independent accumulators,
// then the 16 groups fold through LDS (one thread per channel and slab
// serially took ~0.3 ms per call at 1024 slabs: 4.7 ms of a VGG-16 step).
__global__ void __launch_bounds__(256) colsum_finalize_k(const float* __restrict__ p, int nslab,
                                                         int C, float* __restrict__ out,
                                                         int accumulate) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < C) {
    int k = grp;
    for (; k + 48 < nslab; k += 64) {
      a0 += p[(long)k * C + c];
      a1 += p[(long)(k + 16) * C + c];
      a2 += p[(long)(k + 32) * C + c];
      a3 += p[(long)(k + 48) * C + c];
    }
    for (; k < nslab; k += 16) a0 += p[(long)k * C + c];
  }
  red[grp][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (grp == 0 && c < C) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g][cl];
    out[c] = (accumulate ? out[c] : 0.f) + s;
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
dropout_k(const T* __restrict__ x, T* __restrict__ y, long n, float keep, uint32_t seed) {
  const float inv = 1.f / keep;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float u = u01(seed, (uint64_t)i, 7u);
    y[i] = from_f32<T>(u < keep ? to_f32(x[i]) * inv : 0.f);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
synthetic_images_k(T* __restrict__ x, long n, float mean, float std, uint32_t seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    // Truncated normal (|z| <= 2) by rejection over a few Box-Muller draws.
    float z = 0.f;
    for (uint32_t k = 0; k < 8; ++k) {
      const float u1 = u01(seed, (uint64_t)i, 2 * k + 1), u2 = u01(seed, (uint64_t)i, 2 * k + 2);
      z = sqrtf(-2.f * __logf(u1)) * __cosf(6.28318530718f * u2);
      if (fabsf(z) <= 2.f) break;
      z = 0.f;
    }
    x[i] = from_f32<T>(mean + std * z);
  }
}

// 8 values per thread (one 16-byte store), 32-bit indexing and a per-thread
// hoisted seed hash, cheap enough to re-sample the synthetic batch every
// training step (inside the timed step).  The truncated normal (|z| <= 2) is
// drawn by inversion instead of Box-Muller rejection: z = sqrt(2) *
// erfinv(erf(sqrt(2)) * (2u - 1)) maps one uniform to one value with no
// data-dependent loop (with rejection nearly every wave ran 2-3 rounds of
// log + sqrt + sincos for its few rejected lanes).  erfinv: single-precision
// polynomial in w = -log(1 - x^2) (Giles' central branch; |x| <= erf(sqrt 2)
// keeps w <= 2.42, inside the branch's w < 5 range).
__device__ __forceinline__ float u01h(uint32_t sh, uint32_t i) {
  const uint32_t h = hash_u32(i ^ sh);
  return ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float trunc_normal2(float u) {
  const float x = 0.954499736f * (2.f * u - 1.f);  // erf(sqrt(2)) * (2u - 1)
  float w = -__logf((1.f - x) * (1.f + x)) - 2.5f;
  float p = 2.81022636e-08f;
  p = fmaf(p, w, 3.43273939e-07f);
  p = fmaf(p, w, -3.5233877e-06f);
  p = fmaf(p, w, -4.39150654e-06f);
  p = fmaf(p, w, 0.00021858087f);
  p = fmaf(p, w, -0.00125372503f);
  p = fmaf(p, w, -0.00417768164f);
  p = fmaf(p, w, 0.246640727f);
  p = fmaf(p, w, 1.50140941f);
  const float z = 1.41421356f * p * x;
  return fminf(fmaxf(z, -2.f), 2.f);  // (rounding at the ends)
}

template <typename T>
__global__ void __launch_bounds__(256)
synthetic_images8_k(T* __restrict__ x, unsigned n8, float mean, float std, uint32_t seed) {
  const uint32_t sh = hash_u32(seed + 0x9e3779b9U);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    Vec<T, 8> o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = from_f32<T>(mean + std * trunc_normal2(u01h(sh, i * 8 + k)));
    *reinterpret_cast<Vec<T, 8>*>(x + (long)i * 8) = o;
  }
}

__global__ void __launch_bounds__(256)
synthetic_labels_k(int* __restrict__ y, long n, int maxval, uint32_t seed, uint32_t salt) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    // (24-bit uniforms: maxval above 2^24 leaves some values unreachable)
    int v = (int)(u01(seed, (uint64_t)i, salt) * (float)maxval);
    y[i] = v >= maxval ? maxval - 1 : v;
  }
}

// Uniform [lo, lo + scale) (SSD's synthetic images, boxes, classes and box
// counts); ``salt`` separates the tensors drawn with one per-step seed.
template <typename T>
__global__ void __launch_bounds__(256)
synthetic_uniform_k(T* __restrict__ x, long n, float lo, float scale, uint32_t seed,
                    uint32_t salt) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    x[i] = from_f32<T>(lo + scale * u01(seed, (uint64_t)i, salt));
}

// y = a * b and its backward (da = dy * b, db = dy * a) in one pass: NCF's
// GMF product of the user and item embeddings.
template <typename T>
__global__ void __launch_bounds__(256)
mul_k(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = from_f32<T>(to_f32(a[i]) * to_f32(b[i]));
}

template <typename T>
__global__ void __launch_bounds__(256)
mul_bwd_k(const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ dy,
          T* __restrict__ da, T* __restrict__ db, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float g = to_f32(dy[i]);
    da[i] = from_f32<T>(g * to_f32(b[i]));
    db[i] = from_f32<T>(g * to_f32(a[i]));
  }
}

template <typename T, int V, bool RELU>
__global__ void __launch_bounds__(256)
add_k(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long nvec) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (long)gridDim.x * blockDim.x) {
    float va[V], vb[V];
    load_vec<T, V>(a + i * V, va);
    load_vec<T, V>(b + i * V, vb);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float o = va[k] + vb[k];
      va[k] = RELU ? fmaxf(o, 0.f) : o;
    }
    store_vec<T, V>(y + i * V, va);
  }
}

// Elementwise activations without a bias (KIND 1 = relu6, 2 = tanh); the
// backward reads the forward output: relu6' = 0 < y < 6, tanh' = 1 - y^2.
template <typename T, int V, int KIND>
__global__ void __launch_bounds__(256)
act_fwd_k(const T* __restrict__ x, T* __restrict__ y, long nvec) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (long)gridDim.x * blockDim.x) {
    float v[V];
    load_vec<T, V>(x + i * V, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = KIND == 1 ? fminf(fmaxf(v[k], 0.f), 6.f) : tanhf(v[k]);
    store_vec<T, V>(y + i * V, v);
  }
}

template <typename T, int V, int KIND>
__global__ void __launch_bounds__(256)
act_bwd_k(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long nvec) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
       i += (long)gridDim.x * blockDim.x) {
    float g[V], o[V];
    load_vec<T, V>(dy + i * V, g);
    load_vec<T, V>(y + i * V, o);
#pragma unroll
    for (int k = 0; k < V; ++k)
      g[k] = KIND == 1 ? ((o[k] > 0.f && o[k] < 6.f) ? g[k] : 0.f) : g[k] * (1.f - o[k] * o[k]);
    store_vec<T, V>(dx + i * V, g);
  }
}

static int egrid(long n) {
  long b = (n + 255) / 256;
  if (b > 256L * 16) b = 256L * 16;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace kfb

using namespace kfb;

KFB_API hipError_t kfb_bias_act(int dtype, const void* x, const float* b, void* y, long rows, int C,
                                int relu, hipStream_t stream) {
  const int V = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = rows * C / VV;
      if (relu)
        hipLaunchKernelGGL((bias_act_k<T, VV, true>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)x, b, (T*)y, nvec, C);
      else
        hipLaunchKernelGGL((bias_act_k<T, VV, false>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)x, b, (T*)y, nvec, C);
    });
  });
  return hipGetLastError();
}

// y = act(x) / dx = dy * act'(y) over n elements (n % vec width == 0 is not
// required: the vector width is picked from n), kind 1 = relu6, 2 = tanh.
KFB_API hipError_t kfb_act_fwd(int dtype, const void* x, void* y, long n, int kind,
                               hipStream_t stream) {
  if (kind != 1 && kind != 2) return hipErrorInvalidValue;
  const int V = n % 8 == 0 ? 8 : n % 4 == 0 ? 4 : n % 2 == 0 ? 2 : 1;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = n / VV;
      if (kind == 1)
        hipLaunchKernelGGL((act_fwd_k<T, VV, 1>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)x, (T*)y, nvec);
      else
        hipLaunchKernelGGL((act_fwd_k<T, VV, 2>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)x, (T*)y, nvec);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_act_bwd(int dtype, const void* dy, const void* y, void* dx, long n, int kind,
                               hipStream_t stream) {
  if (kind != 1 && kind != 2) return hipErrorInvalidValue;
  const int V = n % 8 == 0 ? 8 : n % 4 == 0 ? 4 : n % 2 == 0 ? 2 : 1;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = n / VV;
      if (kind == 1)
        hipLaunchKernelGGL((act_bwd_k<T, VV, 1>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)dy, (const T*)y, (T*)dx, nvec);
      else
        hipLaunchKernelGGL((act_bwd_k<T, VV, 2>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)dy, (const T*)y, (T*)dx, nvec);
    });
  });
  return hipGetLastError();
}

KFB_API int kfb_colsum_num_slabs(long rows, int C) {
  const int V = vec_width(C);
  const int cw = C < 256 * V ? C : 256 * V;
  const int tpr = cw / V, rpi = 256 / tpr;
  const int nchunk = ceil_div(C, cw);
  long target = 1024 / nchunk;
  if (target < 1) target = 1;
  long by_work = rows / ((long)rpi * 8);
  if (by_work < 1) by_work = 1;
  long s = target < by_work ? target : by_work;
  return (int)(s > 4096 ? 4096 : s);
}

// relu-backward (if relu) and bias-gradient column sums in one pass.
// dx may alias dy. db (may be null) is written or accumulated.
KFB_API hipError_t kfb_act_bwd_bias(int dtype, const void* dy, const void* y, void* dx, long rows,
                                    int C, int relu, float* pbias, int nslab, float* db,
                                    int accumulate, hipStream_t stream) {
  const int V = vec_width(C);
  // Without a bias gradient the slab count is free: size the grid for the
  // whole tensor (callers pass nslab = 1 there, which left one workgroup per
  // channel chunk streaming every row, ~1.3 ms per NASNet ReLU backward).
  if (!db) nslab = kfb_colsum_num_slabs(rows, C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const int cw = C < 256 * VV ? C : 256 * VV;
      const int tpr = cw / VV, rpi = 256 / tpr;
      const int nchunk = ceil_div(C, cw);
      const long slab_rows = (rows + nslab - 1) / nslab;
      const size_t lds = (size_t)rpi * tpr * VV * sizeof(float);
      dim3 grid(nslab, nchunk);
      float* pb = db ? pbias : nullptr;
      if (relu)
        hipLaunchKernelGGL((act_bwd_bias_k<T, VV, true>), grid, dim3(256), lds, stream,
                           (const T*)dy, (const T*)y, (T*)dx, rows, C, cw, tpr, rpi, slab_rows, pb);
      else
        hipLaunchKernelGGL((act_bwd_bias_k<T, VV, false>), grid, dim3(256), lds, stream,
                           (const T*)dy, (const T*)y, (T*)dx, rows, C, cw, tpr, rpi, slab_rows, pb);
      if (db)
        hipLaunchKernelGGL(colsum_finalize_k, dim3(ceil_div(C, 16)), dim3(256), 0, stream,
                           pbias, nslab, C, db, accumulate);
    });
  });
  return hipGetLastError();
}

// out[c] (+)= sum_k p[k][c]: the bias gradient from the [nslab][C] column
// partials a consumer conv's dgrad epilogue accumulated (fused ReLU/bias
// backward of a conv without BN).
KFB_API hipError_t kfb_slab_colsum(const float* p, int nslab, int C, float* out, int accumulate,
                                   hipStream_t stream) {
  hipLaunchKernelGGL(colsum_finalize_k, dim3(ceil_div(C, 16)), dim3(256), 0, stream, p, nslab, C,
                     out, accumulate);
  return hipGetLastError();
}

KFB_API hipError_t kfb_dropout(int dtype, const void* x, void* y, long n, float keep, uint32_t seed,
                               hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((dropout_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (const T*)x, (T*)y, n,
                       keep, seed);
  });
  return hipGetLastError();
}

// NASNet drop path (tcb/models/nasnet_utils.py drop_path): every sample n of
// x [N][per] is kept with probability kp and scaled by 1/kp, or zeroed:
// y = x * floor(kp + u_n) / kp, u_n uniform from (seed, n).  The backward
// is the same call on dy (same seed, same kp).  kp = 1 is the identity.
template <typename T>
__global__ void __launch_bounds__(256)
drop_path_k(const T* __restrict__ x, T* __restrict__ y, long n, long per, float kp,
            uint32_t seed) {
  const float inv = 1.f / kp;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float u = u01(seed, (uint64_t)(i / per), 11u);
    y[i] = from_f32<T>(floorf(kp + u) * inv * to_f32(x[i]));
  }
}

KFB_API hipError_t kfb_drop_path(int dtype, const void* x, void* y, long n, long per, float kp,
                                 uint32_t seed, hipStream_t stream) {
  if (per <= 0 || !(kp > 0.f)) return hipErrorInvalidValue;
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((drop_path_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (const T*)x, (T*)y,
                       n, per, kp, seed);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_synthetic_images(int dtype, void* x, long n, float mean, float std,
                                        uint32_t seed, hipStream_t stream) {
  const bool vec8 = n % 8 == 0 && n / 8 < (1L << 31) && ((uintptr_t)x & 15) == 0;
  KFB_DISPATCH_DTYPE(dtype, T, {
    if (vec8 && sizeof(T) == 2)
      hipLaunchKernelGGL((synthetic_images8_k<T>), dim3(egrid(n / 8)), dim3(256), 0, stream,
                         (T*)x, (unsigned)(n / 8), mean, std, seed);
    else
      hipLaunchKernelGGL((synthetic_images_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (T*)x, n,
                         mean, std, seed);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_synthetic_labels(int* y, long n, int maxval, uint32_t seed,
                                        hipStream_t stream) {
  hipLaunchKernelGGL(synthetic_labels_k, dim3(egrid(n)), dim3(256), 0, stream, y, n, maxval, seed,
                     99u);
  return hipGetLastError();
}

// Integers uniform in [0, maxval); ``salt`` separates tensors drawn with one
// per-step seed (NCF's users, items and labels).
KFB_API hipError_t kfb_synthetic_ints(int* y, long n, int maxval, uint32_t seed, uint32_t salt,
                                      hipStream_t stream) {
  hipLaunchKernelGGL(synthetic_labels_k, dim3(egrid(n)), dim3(256), 0, stream, y, n, maxval, seed,
                     salt);
  return hipGetLastError();
}

KFB_API hipError_t kfb_synthetic_uniform(int dtype, void* x, long n, float lo, float scale,
                                         uint32_t seed, uint32_t salt, hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((synthetic_uniform_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (T*)x, n,
                       lo, scale, seed, salt);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_mul(int dtype, const void* a, const void* b, void* y, long n,
                           hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((mul_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (const T*)a,
                       (const T*)b, (T*)y, n);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_mul_bwd(int dtype, const void* a, const void* b, const void* dy, void* da,
                               void* db, long n, hipStream_t stream) {
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((mul_bwd_k<T>), dim3(egrid(n)), dim3(256), 0, stream, (const T*)a,
                       (const T*)b, (const T*)dy, (T*)da, (T*)db, n);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_add(int dtype, const void* a, const void* b, void* y, long n, int relu,
                           hipStream_t stream) {
  const int V = (n % 8 == 0) ? 8 : (n % 4 == 0) ? 4 : (n % 2 == 0) ? 2 : 1;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = n / VV;
      if (relu)
        hipLaunchKernelGGL((add_k<T, VV, true>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)a, (const T*)b, (T*)y, nvec);
      else
        hipLaunchKernelGGL((add_k<T, VV, false>), dim3(egrid(nvec)), dim3(256), 0, stream,
                           (const T*)a, (const T*)b, (T*)y, nvec);
    });
  });
  return hipGetLastError();
}

// ---- layout padding for few-channel / odd-width convs (recordable in a
// launch tape, unlike torch's pad): dst [Rp][K][Cp] = src [R][K][C] with zeros
// in the padding (activations: R = 1, K = pixels; weights: R = Cout,
// K = KH*KW).
template <typename T>
__global__ void __launch_bounds__(256)
pad_rkc_k(const T* __restrict__ src, T* __restrict__ dst, long total, int R, int K, int C,
          int Cp) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % Cp);
    const long rk = i / Cp;
    const int r = (int)(rk / K);
    dst[i] = (r < R && c < C) ? src[rk * C + c] : (T)0.f;
  }
}

// dst [R][K][C] (fp32) += src [Rp][K][Cp] over r < R, c < C: a padded conv's
// weight gradient accumulated into the parameter's gradient view
__global__ void __launch_bounds__(256)
unpad_accum_f32_k(const float* __restrict__ src, float* __restrict__ dst, long total, int K,
                  int C, int Cp) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long rk = i / C;
    dst[i] += src[rk * Cp + c];
  }
}

KFB_API hipError_t kfb_pad_rkc(int dtype, const void* src, void* dst, int R, long K, int C, int Rp,
                               int Cp, hipStream_t stream) {
  if (C > Cp || R > Rp) return hipErrorInvalidValue;
  const long total = (long)Rp * K * Cp;
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((pad_rkc_k<T>), dim3(egrid(total)), dim3(256), 0, stream, (const T*)src,
                       (T*)dst, total, R, (int)K, C, Cp);
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_unpad_accum_f32(const float* src, float* dst, int R, long K, int C, int Cp,
                                       hipStream_t stream) {
  const long total = (long)R * K * C;
  hipLaunchKernelGGL(unpad_accum_f32_k, dim3(egrid(total)), dim3(256), 0, stream, src, dst, total,
                     (int)K, C, Cp);
  return hipGetLastError();
}

// dst [R][K][C] = the leading block of src [Rp][K][Cp] (r < R, c < C): the
// inverse of pad_rkc, for a channel-padded conv's output / input gradient
template <typename T>
__global__ void __launch_bounds__(256)
crop_rkc_k(const T* __restrict__ src, T* __restrict__ dst, long total, int K, int C, int Cp) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long rk = i / C;
    dst[i] = src[rk * Cp + c];
  }
}

KFB_API hipError_t kfb_crop_rkc(int dtype, const void* src, void* dst, int R, long K, int C,
                                int Cp, hipStream_t stream) {
  if (C > Cp) return hipErrorInvalidValue;
  const long total = (long)R * K * C;
  if (total == 0) return hipSuccess;
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((crop_rkc_k<T>), dim3(egrid(total)), dim3(256), 0, stream, (const T*)src,
                       (T*)dst, total, (int)K, C, Cp);
  });
  return hipGetLastError();
}

// Conv weight relayouts for the dgrad GEMMs (tcb's conv2d_backprop_input
// filter use): dst[ci][kh][kw][co] = src[co][kh'][kw'][ci] with (kh', kw') =
// (KH-1-kh, KW-1-kw) when flip (stride-1 transposed conv), else (kh, kw);
// a 1x1 conv's case is the plain [Cout][Cin] -> [Cin][Cout] transpose.
template <typename T>
__global__ void __launch_bounds__(256)
wrelayout_k(const T* __restrict__ src, T* __restrict__ dst, int cout, int KH, int KW, int cin,
            int flip) {
  const long total = (long)cout * KH * KW * cin;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    // i indexes dst [ci][kh][kw][co]
    const int co = (int)(i % cout);
    long r = i / cout;
    const int kw = (int)(r % KW);
    r /= KW;
    const int kh = (int)(r % KH);
    const int ci = (int)(r / KH);
    const int sh = flip ? KH - 1 - kh : kh, sw = flip ? KW - 1 - kw : kw;
    dst[i] = src[(((long)co * KH + sh) * KW + sw) * cin + ci];
  }
}

KFB_API hipError_t kfb_wrelayout(int dtype, const void* src, void* dst, int cout, int KH, int KW,
                                 int cin, int flip, hipStream_t stream) {
  const long total = (long)cout * KH * KW * cin;
  if (total == 0) return hipSuccess;
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((wrelayout_k<T>), dim3(egrid(total)), dim3(256), 0, stream, (const T*)src,
                       (T*)dst, cout, KH, KW, cin, flip);
  });
  return hipGetLastError();
}

// Strided / shifted window of an NHWC tensor and its adjoint:
//   adjoint = 0: y[n][oh][ow][c] = x[n][oh*sh + oh0][ow*sw + ow0][c] (0 outside x)
//   adjoint = 1: dx[n][h][w][c] = dy[n][(h-oh0)/sh][(w-ow0)/sw][c] where that
//                is an exact, in-range sample (0 elsewhere): the gradient
// The 1x1 strided average pool of ResNet shortcuts (tcb/convnet_builder.py
// apool with a 1x1 window) and NASNet's one-pixel shift before its second
// factorized-reduction path (tcb/models/nasnet_utils.py
// _factorized_reduction: pad + slice).  V channels per thread.
namespace kfb {
template <typename T, int V>
__global__ void __launch_bounds__(256)
window_k(const T* __restrict__ src, T* __restrict__ dst, long total, int H, int W, int C,
         int OH, int OW, int sh, int sw, int oh0, int ow0, int adjoint) {
  const int CV = C / V;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int cv = (int)(i % CV);
    long r = i / CV;
    Vec<T, V> v;
    bool ok;
    long so;
    if (!adjoint) {  // i indexes y [N][OH][OW][CV]
      const int ow = (int)(r % OW);
      r /= OW;
      const int oh = (int)(r % OH);
      const long n = r / OH;
      const int h = oh * sh + oh0, w = ow * sw + ow0;
      ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      so = ((n * H + h) * W + w) * C + (long)cv * V;
    } else {  // i indexes dx [N][H][W][CV]
      const int w = (int)(r % W);
      r /= W;
      const int h = (int)(r % H);
      const long n = r / H;
      const int hh = h - oh0, ww = w - ow0;
      const int oh = hh / sh, ow = ww / sw;
      ok = hh >= 0 && ww >= 0 && oh * sh == hh && ow * sw == ww && oh < OH && ow < OW;
      so = ((n * OH + oh) * OW + ow) * C + (long)cv * V;
    }
    if (ok) {
      v = *(const Vec<T, V>*)(src + so);
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) v.v[k] = (T)0.f;
    }
    *(Vec<T, V>*)(dst + i * V) = v;
  }
}
}  // namespace kfb

KFB_API hipError_t kfb_window(int dtype, const void* src, void* dst, int N, int H, int W, int C,
                              int OH, int OW, int sh, int sw, int oh0, int ow0, int adjoint,
                              hipStream_t stream) {
  if (sh < 1 || sw < 1) return hipErrorInvalidValue;
  const int V = (C % 8 == 0 && dtype != F32) ? 8 : (C % 4 == 0 ? 4 : 1);
  const long total = (long)N * (adjoint ? (long)H * W : (long)OH * OW) * (C / V);
  if (total == 0) return hipSuccess;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      hipLaunchKernelGGL((kfb::window_k<T, VV>), dim3(egrid(total)), dim3(256), 0, stream,
                         (const T*)src, (T*)dst, total, H, W, C, OH, OW, sh, sw, oh0, ow0,
                         adjoint);
    });
  });
  return hipGetLastError();
}
