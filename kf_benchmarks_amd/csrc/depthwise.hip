// NHWC depthwise convolution (channel multiplier 1): forward, data gradient
// and filter gradient.  Role of tf.nn.depthwise_conv2d / slim.separable_conv2d
// in MobileNet-v2 and NASNet (tcb/models/mobilenet_conv_blocks.py,
// tcb/models/nasnet_utils.py).
//
// Depthwise convs do ~k*k MACs per loaded element, so they are HBM-bound:
// every lane owns V consecutive channels of one pixel and moves 16-byte
// vectors; the filter [KH][KW][C] (TF layout [KH,KW,C,1]) is read per tap
// through L1/L2.
//   fwd   : y[n,oh,ow,c]  = sum_{a,b} x[n, oh*s-pt+a, ow*s-pl+b, c] * w[a,b,c]
//   dgrad : dx[n,h,w,c]   = sum_{a,b: (h+pt-a)%s==0 ...} dy[n,(h+pt-a)/s,(w+pl-b)/s,c] * w[a,b,c]
//   wgrad : dw[a,b,c]    += sum_{n,oh,ow} dy[n,oh,ow,c] * x[n, oh*s-pt+a, ow*s-pl+b, c]
// wgrad: a workgroup owns one V-channel group and a slice of output pixels;
// its 256 lanes each accumulate KH*KW*V partial sums in registers over a
// strided subset of the slice, reduce through LDS and add the block's sum
// into the fp32 filter gradient with one atomic per element.
#include "common.h"

namespace kfb {

struct DwGeo {
  int N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl;
};

template <typename T, int V>
__global__ void __launch_bounds__(256)
dw_fwd_k(const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y, DwGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.OH * g.OW * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int ow = (int)(p % g.OW);
    p /= g.OW;
    const int oh = (int)(p % g.OH);
    const int n = (int)(p / g.OH);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
    for (int a = 0; a < g.KH; ++a) {
      const int h = h0 + a;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int b = 0; b < g.KW; ++b) {
        const int ww = w0 + b;
        if ((unsigned)ww >= (unsigned)g.W) continue;
        float xv[V], wv[V];
        load_vec<T, V>(x + (((long)n * g.H + h) * g.W + ww) * g.C + c, xv);
        load_vec<T, V>(w + (a * g.KW + b) * g.C + c, wv);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = fmaf(xv[k], wv[k], acc[k]);
      }
    }
    store_vec<T, V>(y + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c, acc);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
dw_dgrad_k(const T* __restrict__ dy, const T* __restrict__ w, T* __restrict__ dx, DwGeo g) {
  const int cv = g.C / V;
  const long total = (long)g.N * g.H * g.W * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    long p = i / cv;
    const int wq = (int)(p % g.W);
    p /= g.W;
    const int h = (int)(p % g.H);
    const int n = (int)(p / g.H);
    float acc[V];
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] = 0.f;
    for (int a = 0; a < g.KH; ++a) {
      const int hh = h + g.pt - a;
      if (hh < 0 || hh % g.sh) continue;
      const int oh = hh / g.sh;
      if (oh >= g.OH) continue;
      for (int b = 0; b < g.KW; ++b) {
        const int ww = wq + g.pl - b;
        if (ww < 0 || ww % g.sw) continue;
        const int ow = ww / g.sw;
        if (ow >= g.OW) continue;
        float dv[V], wv[V];
        load_vec<T, V>(dy + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c, dv);
        load_vec<T, V>(w + (a * g.KW + b) * g.C + c, wv);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[k] = fmaf(dv[k], wv[k], acc[k]);
      }
    }
    store_vec<T, V>(dx + (((long)n * g.H + h) * g.W + wq) * g.C + c, acc);
  }
}

// KMAX taps accumulated per lane in registers (7x7 max).
template <typename T, int V, int KMAX>
__global__ void __launch_bounds__(256)
dw_wgrad_k(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ dw, DwGeo g,
           int pix_per_block) {
  __shared__ float red[256 / 64][KMAX * V];
  const int cv = g.C / V;
  const int cg = blockIdx.y;  // channel group
  const int c = cg * V;
  const long M = (long)g.N * g.OH * g.OW;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = p0 + pix_per_block < M ? p0 + pix_per_block : M;
  const int taps = g.KH * g.KW;
  float acc[KMAX][V];
#pragma unroll
  for (int t = 0; t < KMAX; ++t)
#pragma unroll
    for (int k = 0; k < V; ++k) acc[t][k] = 0.f;
  for (long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const int ow = (int)(p % g.OW);
    const long q = p / g.OW;
    const int oh = (int)(q % g.OH);
    const int n = (int)(q / g.OH);
    float dv[V];
    load_vec<T, V>(dy + p * g.C + c, dv);
    const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
#pragma unroll
    for (int t = 0; t < KMAX; ++t) {
      const int a = t / g.KW, b = t - a * g.KW;
      const int h = h0 + a, ww = w0 + b;
      if (t < taps && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W) {
        float xv[V];
        load_vec<T, V>(x + (((long)n * g.H + h) * g.W + ww) * g.C + c, xv);
#pragma unroll
        for (int k = 0; k < V; ++k) acc[t][k] = fmaf(dv[k], xv[k], acc[t][k]);
      }
    }
  }
  // wave reduce, then across the 4 waves through LDS
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < KMAX; ++t) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float s = wave_sum(acc[t][k]);
      if (lane == 0) red[wid][t * V + k] = s;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < taps * V; e += blockDim.x) {
    const float s = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    const int t = e / V, k = e - t * V;
    if (s != 0.f) atomicAdd(dw + t * g.C + c + k, s);
  }
  (void)cv;
}

inline DwGeo geo(int N, int H, int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                 int pt, int pl) {
  return DwGeo{N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl};
}

inline int grid_for(long work) {
  long b = (work + 255) / 256;
  return (int)(b < 65536 * 8 ? (b > 0 ? b : 1) : 65536 * 8);
}

}  // namespace kfb

using namespace kfb;

KFB_API hipError_t kfb_dw_fwd(int dtype, const void* x, const void* w, void* y, int N, int H, int W,
                              int C, int OH, int OW, int KH, int KW, int sh, int sw, int pt, int pl,
                              hipStream_t stream) {
  const DwGeo g = geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl);
  const int vw = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, KFB_DISPATCH_VEC(vw, V, {
    hipLaunchKernelGGL((dw_fwd_k<T, V>), dim3(grid_for((long)N * OH * OW * (C / V))), dim3(256),
                       0, stream, (const T*)x, (const T*)w, (T*)y, g);
  }));
  return hipGetLastError();
}

KFB_API hipError_t kfb_dw_dgrad(int dtype, const void* dy, const void* w, void* dx, int N, int H,
                                int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                                int pt, int pl, hipStream_t stream) {
  const DwGeo g = geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl);
  const int vw = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, KFB_DISPATCH_VEC(vw, V, {
    hipLaunchKernelGGL((dw_dgrad_k<T, V>), dim3(grid_for((long)N * H * W * (C / V))), dim3(256),
                       0, stream, (const T*)dy, (const T*)w, (T*)dx, g);
  }));
  return hipGetLastError();
}

// dw: fp32 [KH][KW][C], accumulated into (caller zeroes or passes the gradient sink).
KFB_API hipError_t kfb_dw_wgrad(int dtype, const void* dy, const void* x, float* dw, int N, int H,
                                int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                                int pt, int pl, hipStream_t stream) {
  const DwGeo g = geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl);
  if (KH * KW > 49) return hipErrorInvalidValue;
  const long M = (long)N * OH * OW;
  const int vw = C % 4 == 0 ? 4 : (C % 2 == 0 ? 2 : 1);  // 4 channels: KMAX*V registers
  // ~ 2048 blocks in total across channel groups, at least 1024 pixels each
  const int groups = C / vw;
  long blocks_x = (2048 + groups - 1) / groups;
  int ppb = (int)((M + blocks_x - 1) / blocks_x);
  if (ppb < 1024) ppb = 1024;
  blocks_x = (M + ppb - 1) / ppb;
  const dim3 grid((unsigned)blocks_x, (unsigned)groups);
#define DW_WGRAD_LAUNCH(KM)                                                                        \
  KFB_DISPATCH_DTYPE(dtype, T, {                                                            \
    if (vw == 4)                                                                            \
      hipLaunchKernelGGL((dw_wgrad_k<T, 4, KM>), grid, dim3(256), 0, stream, (const T*)dy,  \
                         (const T*)x, dw, g, ppb);                                           \
    else if (vw == 2)                                                                       \
      hipLaunchKernelGGL((dw_wgrad_k<T, 2, KM>), grid, dim3(256), 0, stream, (const T*)dy,  \
                         (const T*)x, dw, g, ppb);                                           \
    else                                                                                    \
      hipLaunchKernelGGL((dw_wgrad_k<T, 1, KM>), grid, dim3(256), 0, stream, (const T*)dy,  \
                         (const T*)x, dw, g, ppb);                                           \
  })
  if (KH * KW <= 9) {
    DW_WGRAD_LAUNCH(9);
  } else if (KH * KW <= 25) {
    DW_WGRAD_LAUNCH(25);
  } else {
    DW_WGRAD_LAUNCH(49);
  }
#undef DW_WGRAD_LAUNCH
  return hipGetLastError();
}
