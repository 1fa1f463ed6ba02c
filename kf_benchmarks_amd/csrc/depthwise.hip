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
// wgrad: see dw_wgrad_k (lanes along the NHWC vector index, taps x V
// partial sums per lane, one LDS reduction and one atomic per element and
// workgroup).
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

// Filter gradient.  Lanes run along the NHWC vector index (pixel-major,
// channel group minor), so a wave's dy / x loads are contiguous runs: with
// cv = C/V channel groups, a workgroup holds cvb = min(cv, 256) groups
// (blockIdx.y picks the chunk) times P = 256/cvb pixel lanes, and every
// thread keeps its channel group while it walks its slice of pixels with
// stride P.  A workgroup covers ROWS filter rows x RW filter columns
// (blockIdx.z picks the group: 3x3 filters in one, larger ones one row of
// <= 7 columns per group, so the accumulators stay at <= 7 x 8 registers
// and there are enough workgroups).  The P pixel lanes of a group are summed through LDS
// one tap at a time and the workgroup adds its sum into the fp32 filter
// gradient (one atomic per element and workgroup).  (The per-pixel-lane
// layout it replaces loaded one 8-byte piece per lane from a different cache
// line: MobileNet-v2's filter gradients took 5.3 of its 14.8 ms step,
// profiles/r13_depthwise.txt.)
template <typename T, int V, int ROWS, int RW>
__global__ void __launch_bounds__(256)
dw_wgrad_k(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ dw, DwGeo g,
           int cvb, int P, int ppb, int ncg, FastDiv fow, FastDiv foh) {
  __shared__ float red[256 * V];
  const int cv = g.C / V;
  const int tid = threadIdx.x;
  const int gl = tid % cvb, q = tid / cvb;
  const int cg = blockIdx.y * cvb + gl;
  const bool active = q < P && cg < cv;
  const int c = cg * V;
  const int row0 = (int)(blockIdx.z / ncg) * ROWS;      // ncg column groups per row group
  const int col0 = (int)(blockIdx.z % ncg) * RW;
  const int M = g.N * g.OH * g.OW;
  const int p0 = blockIdx.x * ppb;
  const int p1 = p0 + ppb < M ? p0 + ppb : M;
  float acc[ROWS * RW][V];
#pragma unroll
  for (int t = 0; t < ROWS * RW; ++t)
#pragma unroll
    for (int k = 0; k < V; ++k) acc[t][k] = 0.f;
  if (active) {
    for (int p = p0 + q; p < p1; p += P) {
      const int r = fow.div(p);
      const int ow = p - r * g.OW;
      const int n = foh.div(r);
      const int oh = r - n * g.OH;
      float dv[V];
      load_vec<T, V>(dy + (long)p * g.C + c, dv);
      const int h0 = oh * g.sh - g.pt + row0, w0 = ow * g.sw - g.pl + col0;
      const T* xn = x + (long)n * g.H * g.W * g.C + c;
#pragma unroll
      for (int a = 0; a < ROWS; ++a) {
        const int h = h0 + a;
        if (row0 + a >= g.KH || (unsigned)h >= (unsigned)g.H) continue;
#pragma unroll
        for (int b = 0; b < RW; ++b) {
          const int ww = w0 + b;
          if (col0 + b < g.KW && (unsigned)ww < (unsigned)g.W) {
            float xv[V];
            load_vec<T, V>(xn + ((long)h * g.W + ww) * g.C, xv);
#pragma unroll
            for (int k = 0; k < V; ++k) acc[a * RW + b][k] = fmaf(dv[k], xv[k], acc[a * RW + b][k]);
          }
        }
      }
    }
  }
  // per tap: the P pixel lanes of each channel group through LDS
#pragma unroll
  for (int t = 0; t < ROWS * RW; ++t) {
    const int a = t / RW, b = t - a * RW;
    if (row0 + a < g.KH && col0 + b < g.KW) {  // uniform over the block
      if (active) {
#pragma unroll
        for (int k = 0; k < V; ++k) red[tid * V + k] = acc[t][k];
      }
      __syncthreads();
      float* dwt = dw + (long)((row0 + a) * g.KW + col0 + b) * g.C;
      for (int e = tid; e < cvb * V; e += 256) {
        const int gl2 = e / V, k = e - gl2 * V;
        const int cg2 = blockIdx.y * cvb + gl2;
        if (cg2 < cv) {
          float s = 0.f;
          for (int qq = 0; qq < P; ++qq) s += red[(qq * cvb + gl2) * V + k];
          if (s != 0.f) atomicAdd(dwt + cg2 * V + k, s);
        }
      }
      __syncthreads();
    }
  }
}

// V channels per lane (<= 8: ROWS * RW * V accumulators <= 72)
template <typename T, int ROWS, int RW>
static void launch_dw_wgrad(int vw, dim3 grid, hipStream_t stream, const void* dy, const void* x,
                            float* dw, const DwGeo& g, int cvb, int P, int ppb, int ncg,
                            FastDiv fow, FastDiv foh) {
  if (vw == 8)
    hipLaunchKernelGGL((dw_wgrad_k<T, 8, ROWS, RW>), grid, dim3(256), 0, stream, (const T*)dy,
                       (const T*)x, dw, g, cvb, P, ppb, ncg, fow, foh);
  else if (vw == 4)
    hipLaunchKernelGGL((dw_wgrad_k<T, 4, ROWS, RW>), grid, dim3(256), 0, stream, (const T*)dy,
                       (const T*)x, dw, g, cvb, P, ppb, ncg, fow, foh);
  else if (vw == 2)
    hipLaunchKernelGGL((dw_wgrad_k<T, 2, ROWS, RW>), grid, dim3(256), 0, stream, (const T*)dy,
                       (const T*)x, dw, g, cvb, P, ppb, ncg, fow, foh);
  else
    hipLaunchKernelGGL((dw_wgrad_k<T, 1, ROWS, RW>), grid, dim3(256), 0, stream, (const T*)dy,
                       (const T*)x, dw, g, cvb, P, ppb, ncg, fow, foh);
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

KFB_API int kfb_get_deterministic();  // (conv_igemm.hip) fixed-order weight-gradient sums

// dw: fp32 [KH][KW][C], accumulated into (caller zeroes or passes the gradient sink).
KFB_API hipError_t kfb_dw_wgrad(int dtype, const void* dy, const void* x, float* dw, int N, int H,
                                int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                                int pt, int pl, hipStream_t stream) {
  const DwGeo g = geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl);
  const long M = (long)N * OH * OW;
  if (KW < 1 || KH < 1 || M >= (1L << 31) - 256 || M <= 0) return hipErrorInvalidValue;
  const int vw = vec_width(C);
  const int cv = C / vw;
  const int cvb = cv < 256 ? cv : 256;
  const int P = 256 / cvb;
  const int chunks = (cv + cvb - 1) / cvb;
  const bool small = KH <= 3 && KW <= 3;       // one group of 3 x 3 taps
  const int rw = small || KW <= 3 ? 3 : KW <= 5 ? 5 : 7;
  const int ncg = small ? 1 : (KW + rw - 1) / rw;  // column groups per filter row
  const int zg = small ? 1 : KH * ncg;             // else one row x rw columns per group
  const int tapsz = small ? 9 : rw;                // taps per workgroup (upper bound)
  // ~2048 workgroups with >= 8 pixel iterations per lane, and <= ~2M atomics
  // per launch (each workgroup adds tapsz * cvb * V) but >= 64 workgroups
  constexpr long kMinIters = 8, kBlocks = 2048, kAtomics = 2L << 20;
  long bx = (M + kMinIters * P - 1) / (kMinIters * P);
  long cap = kBlocks / ((long)chunks * zg);
  const long acap = kAtomics / ((long)tapsz * C * zg);
  if (acap < cap) cap = acap;
  if (cap < 64) cap = 64;
  if (bx > cap) bx = cap;
  if (bx < 1 || kfb_get_deterministic()) bx = 1;  // deterministic: one atomic per element
  long ppb = (M + bx - 1) / bx;
  ppb = (ppb + P - 1) / P * P;
  bx = (M + ppb - 1) / ppb;
  const dim3 grid((unsigned)bx, (unsigned)chunks, (unsigned)zg);
  const FastDiv fow(OW), foh(OH);
#define DW_WGRAD_LAUNCH(ROWS, RW)                                                              \
  KFB_DISPATCH_DTYPE(dtype, T, {                                                               \
    launch_dw_wgrad<T, ROWS, RW>(vw, grid, stream, dy, x, dw, g, cvb, P, (int)ppb, ncg, fow,   \
                                 foh);                                                         \
  })
  if (small) {
    DW_WGRAD_LAUNCH(3, 3);
  } else if (rw == 3) {
    DW_WGRAD_LAUNCH(1, 3);
  } else if (rw == 5) {
    DW_WGRAD_LAUNCH(1, 5);
  } else {
    DW_WGRAD_LAUNCH(1, 7);
  }
#undef DW_WGRAD_LAUNCH
  return hipGetLastError();
}
