// NHWC pooling: max / average (k x k, stride s, explicit pads) and the global
// spatial mean, forward and backward.
//
// Role of cnn.mpool / cnn.apool / cnn.spatial_mean (tcb/convnet_builder.py:215-266,
// 385-394).  Each lane owns V consecutive channels of one pixel (16-byte
// accesses).  Max-pool forward stores the in-window argmax as one byte per
// output element; the backward is a gather (no atomics): every input pixel
// visits the <= ceil(k/s)^2 windows that contain it.  Average pooling divides
// by the number of in-bounds taps (TF 'SAME' semantics).
#include "common.h"

namespace kfb {

struct PoolGeo {
  int N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl;
};

template <typename T, int V>
__global__ void __launch_bounds__(256)
maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, PoolGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.OH * g.OW * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int ow = (int)(p % g.OW); p /= g.OW;
    const int oh = (int)(p % g.OH);
    const int n = (int)(p / g.OH);
    float best[V];
    int bi[V];
#pragma unroll
    for (int k = 0; k < V; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
    for (int a = 0; a < g.kh; ++a) {
      const int h = h0 + a;
      if (h < 0 || h >= g.H) continue;
      for (int b = 0; b < g.kw; ++b) {
        const int w = w0 + b;
        if (w < 0 || w >= g.W) continue;
        float v[V];
        load_vec<T, V>(x + (((long)n * g.H + h) * g.W + w) * g.C + c, v);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (v[k] > best[k]) { best[k] = v[k]; bi[k] = a * g.kw + b; }
      }
    }
    const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c;
    store_vec<T, V>(y + o, best);
    if (idx) {
#pragma unroll
      for (int k = 0; k < V; ++k) idx[o + k] = (uint8_t)bi[k];
    }
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
maxpool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx,
              PoolGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.H * g.W * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int w = (int)(p % g.W); p /= g.W;
    const int h = (int)(p % g.H);
    const int n = (int)(p / g.H);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    // outputs whose window covers h: oh*sh - pt <= h <= oh*sh - pt + kh - 1
    int oh_lo = h + g.pt - g.kh + 1;
    oh_lo = oh_lo <= 0 ? 0 : (oh_lo + g.sh - 1) / g.sh;
    int oh_hi = (h + g.pt) / g.sh;
    if (oh_hi >= g.OH) oh_hi = g.OH - 1;
    int ow_lo = w + g.pl - g.kw + 1;
    ow_lo = ow_lo <= 0 ? 0 : (ow_lo + g.sw - 1) / g.sw;
    int ow_hi = (w + g.pl) / g.sw;
    if (ow_hi >= g.OW) ow_hi = g.OW - 1;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int a = h - (oh * g.sh - g.pt);
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int b = w - (ow * g.sw - g.pl);
        const int pos = a * g.kw + b;
        const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c;
        float d[V];
        load_vec<T, V>(dy + o, d);
#pragma unroll
        for (int k = 0; k < V; ++k)
          if (idx[o + k] == pos) acc[k] += d[k];
      }
    }
    store_vec<T, V>(dx + (((long)n * g.H + h) * g.W + w) * g.C + c, acc);
  }
}

__device__ __forceinline__ int pool_count(const PoolGeo& g, int oh, int ow) {
  const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
  const int h1 = min(h0 + g.kh, g.H), w1 = min(w0 + g.kw, g.W);
  return (h1 - max(h0, 0)) * (w1 - max(w0, 0));
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, PoolGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.OH * g.OW * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int ow = (int)(p % g.OW); p /= g.OW;
    const int oh = (int)(p % g.OH);
    const int n = (int)(p / g.OH);
    float s[V];
#pragma unroll
    for (int k = 0; k < V; ++k) s[k] = 0.f;
    const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
    for (int a = 0; a < g.kh; ++a) {
      const int h = h0 + a;
      if (h < 0 || h >= g.H) continue;
      for (int b = 0; b < g.kw; ++b) {
        const int w = w0 + b;
        if (w < 0 || w >= g.W) continue;
        float v[V];
        load_vec<T, V>(x + (((long)n * g.H + h) * g.W + w) * g.C + c, v);
#pragma unroll
        for (int k = 0; k < V; ++k) s[k] += v[k];
      }
    }
    const float inv = 1.f / (float)pool_count(g, oh, ow);
#pragma unroll
    for (int k = 0; k < V; ++k) s[k] *= inv;
    store_vec<T, V>(y + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c, s);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, PoolGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.H * g.W * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int w = (int)(p % g.W); p /= g.W;
    const int h = (int)(p % g.H);
    const int n = (int)(p / g.H);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    int oh_lo = h + g.pt - g.kh + 1;
    oh_lo = oh_lo <= 0 ? 0 : (oh_lo + g.sh - 1) / g.sh;
    int oh_hi = (h + g.pt) / g.sh;
    if (oh_hi >= g.OH) oh_hi = g.OH - 1;
    int ow_lo = w + g.pl - g.kw + 1;
    ow_lo = ow_lo <= 0 ? 0 : (ow_lo + g.sw - 1) / g.sw;
    int ow_hi = (w + g.pl) / g.sw;
    if (ow_hi >= g.OW) ow_hi = g.OW - 1;
    for (int oh = oh_lo; oh <= oh_hi; ++oh)
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const float inv = 1.f / (float)pool_count(g, oh, ow);
        float d[V];
        load_vec<T, V>(dy + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c, d);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] += d[k] * inv;
      }
    store_vec<T, V>(dx + (((long)n * g.H + h) * g.W + w) * g.C + c, acc);
  }
}

// Global spatial mean: x [N, HW, C] -> y [N, C] (fp32 accumulate).
template <typename T, int V>
__global__ void __launch_bounds__(256)
gap_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int HW, int C) {
  const int cv = C / V;
  const long total = (long)N * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    const int n = (int)(i / cv);
    float s[V];
#pragma unroll
    for (int k = 0; k < V; ++k) s[k] = 0.f;
    const T* base = x + (long)n * HW * C + c;
    for (int p = 0; p < HW; ++p) {
      float v[V];
      load_vec<T, V>(base + (long)p * C, v);
#pragma unroll
      for (int k = 0; k < V; ++k) s[k] += v[k];
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int k = 0; k < V; ++k) s[k] *= inv;
    store_vec<T, V>(y + (long)n * C + c, s);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
gap_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  const int cv = C / V;
  const long total = (long)N * HW * cv;
  const float inv = 1.f / (float)HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    const long np = i / cv;
    const int n = (int)(np / HW);
    float d[V];
    load_vec<T, V>(dy + (long)n * C + c, d);
#pragma unroll
    for (int k = 0; k < V; ++k) d[k] *= inv;
    store_vec<T, V>(dx + np * C + c, d);
  }
}

static int pgrid(long total) {
  long b = (total + 255) / 256;
  if (b > 256L * 16) b = 256L * 16;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace kfb

using namespace kfb;

#define POOL_GEO_ARGS                                                                   \
  PoolGeo g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};                               \
  const int V = vec_width(C);

KFB_API hipError_t kfb_maxpool_fwd(int dtype, const void* x, void* y, uint8_t* idx, int N, int H,
                                   int W, int C, int OH, int OW, int kh, int kw, int sh, int sw,
                                   int pt, int pl, hipStream_t stream) {
  POOL_GEO_ARGS
  if (kh * kw > 255) return hipErrorInvalidValue;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * OH * OW * (C / VV);
      hipLaunchKernelGGL((maxpool_fwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)x, (T*)y, idx, g);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_maxpool_bwd(int dtype, const void* dy, const uint8_t* idx, void* dx, int N,
                                   int H, int W, int C, int OH, int OW, int kh, int kw, int sh,
                                   int sw, int pt, int pl, hipStream_t stream) {
  POOL_GEO_ARGS
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * H * W * (C / VV);
      hipLaunchKernelGGL((maxpool_bwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)dy, idx, (T*)dx, g);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_avgpool_fwd(int dtype, const void* x, void* y, int N, int H, int W, int C,
                                   int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                                   hipStream_t stream) {
  POOL_GEO_ARGS
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * OH * OW * (C / VV);
      hipLaunchKernelGGL((avgpool_fwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)x, (T*)y, g);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_avgpool_bwd(int dtype, const void* dy, void* dx, int N, int H, int W, int C,
                                   int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl,
                                   hipStream_t stream) {
  POOL_GEO_ARGS
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * H * W * (C / VV);
      hipLaunchKernelGGL((avgpool_bwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)dy, (T*)dx, g);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_gap_fwd(int dtype, const void* x, void* y, int N, int HW, int C,
                               hipStream_t stream) {
  const int V = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * (C / VV);
      hipLaunchKernelGGL((gap_fwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)x, (T*)y, N, HW, C);
    });
  });
  return hipGetLastError();
}

KFB_API hipError_t kfb_gap_bwd(int dtype, const void* dy, void* dx, int N, int HW, int C,
                               hipStream_t stream) {
  const int V = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long total = (long)N * HW * (C / VV);
      hipLaunchKernelGGL((gap_bwd_k<T, VV>), dim3(pgrid(total)), dim3(256), 0, stream,
                         (const T*)dy, (T*)dx, N, HW, C);
    });
  });
  return hipGetLastError();
}
