// Fused batch-norm (+ residual add) (+ ReLU) forward and backward for NHWC
// activations viewed as [rows, C].
//
// Replaces cuDNN's fused BN as used by tcb/convnet_builder.py:437-461 and the
// ResNet block tail relu(shortcut + bn(conv)) (tcb/models/resnet_model_legacy.py:76-78).
//
// Structure (each phase is one launch, all HBM-streaming with 16-byte lanes):
//   fwd : partial_stats  -> finalize (mean, invstd, running-stat update,
//         per-channel scale/shift) -> apply (y = relu(x*scale+shift [+res]))
//   bwd : partial_grad (sum dy', sum dy'*(x-mean), dy' = relu-masked dy)
//         -> finalize (dgamma, dbeta, dx coefficients) -> apply
//         (dx = dy'*A + x*B + Cc, dres = dy')
// The partial kernels give every block a slab of rows and a window of channels
// so a launch has >= 1024 workgroups on 256 CUs for the ResNet shapes.
#include "common.h"

namespace kfb {

constexpr int BN_THREADS = 512;

struct Geo {
  int cw;    // channels per block window
  int tpr;   // threads per row = cw / V
  int rpi;   // rows per iteration = BN_THREADS / tpr
  int nchunk;
};

template <int V>
static Geo make_geo(int C) {
  Geo g;
  g.cw = C < BN_THREADS * V ? C : BN_THREADS * V;
  g.tpr = g.cw / V;
  g.rpi = BN_THREADS / g.tpr;
  g.nchunk = ceil_div(C, g.cw);
  return g;
}

// Sum of per-lane vectors over the rpi row-lanes of the block: LDS tree
// reduction (row-lane 0 ends with the block totals).
template <int V>
__device__ __forceinline__ void block_row_reduce(float (&a)[V], float (&b)[V], float* lds, int t,
                                                 int r, int tpr, int rpi) {
  // lds layout: [rpi][tpr][V] for a then b.
  const int stride = rpi * tpr * V;
  if (r < rpi) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      lds[(r * tpr + t) * V + i] = a[i];
      lds[stride + (r * tpr + t) * V + i] = b[i];
    }
  }
  __syncthreads();
  int p2 = 1;
  while (p2 * 2 <= rpi) p2 *= 2;
  if (r < rpi - p2) {  // fold the non-power-of-two tail
#pragma unroll
    for (int i = 0; i < V; ++i) {
      lds[(r * tpr + t) * V + i] += lds[((r + p2) * tpr + t) * V + i];
      lds[stride + (r * tpr + t) * V + i] += lds[stride + ((r + p2) * tpr + t) * V + i];
    }
  }
  __syncthreads();
  for (int h = p2 / 2; h > 0; h /= 2) {
    if (r < h) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        lds[(r * tpr + t) * V + i] += lds[((r + h) * tpr + t) * V + i];
        lds[stride + (r * tpr + t) * V + i] += lds[stride + ((r + h) * tpr + t) * V + i];
      }
    }
    __syncthreads();
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      a[i] = lds[t * V + i];
      b[i] = lds[stride + t * V + i];
    }
  }
}

// ---------------------------------------------------------------- forward
template <typename T, int V>
__global__ void __launch_bounds__(BN_THREADS)
bn_partial_stats_k(const T* __restrict__ x, long rows, int C, int cw, int tpr, int rpi,
                   long slab_rows, float* __restrict__ psum, float* __restrict__ psq,
                   const float* __restrict__ kshift) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int t = tid % tpr, r = tid / tpr;
  const int c0 = blockIdx.y * cw + t * V;
  const bool cok = (c0 < C) && (r < rpi);
  float s[V], q[V], k[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { s[i] = 0.f; q[i] = 0.f; k[i] = (kshift && cok) ? kshift[c0 + i] : 0.f; }
  const long rbeg = (long)blockIdx.x * slab_rows;
  long rend = rbeg + slab_rows;
  if (rend > rows) rend = rows;
  if (cok) {
    // 4 rows per iteration, loads first (see bn_partial_grad_k)
    long row = rbeg + r;
    for (; row + 3 * rpi < rend; row += 4 * rpi) {
      float v[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_vec<T, V>(x + (row + u * rpi) * C + c0, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const float e = v[u][i] - k[i];
          s[i] += e;
          q[i] += e * e;
        }
      }
    }
    for (; row < rend; row += rpi) {
      float v[V];
      load_vec<T, V>(x + row * C + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float e = v[i] - k[i];
        s[i] += e;
        q[i] += e * e;
      }
    }
  }
  block_row_reduce<V>(s, q, lds, t, r, tpr, rpi);
  if (r == 0 && c0 < C) {
    float* ps = psum + (long)blockIdx.x * C + c0;
    float* pq = psq + (long)blockIdx.x * C + c0;
#pragma unroll
    for (int i = 0; i < V; ++i) { ps[i] = s[i]; pq[i] = q[i]; }
  }
}

// Slab partials -> per-channel totals.  Block = 64 channels x FOLD_Y slab
// lanes, each lane sums every FOLD_Y-th slab with 4 independent accumulators
// (the fold is latency-bound: the 32 conv-epilogue slots take one round of
// loads), lanes combine through LDS.
constexpr int FOLD_Y = 16;  // slab lanes per channel (blockDim.y of the finalize kernels)

__device__ __forceinline__ void fold_slabs(const float* __restrict__ pa,
                                           const float* __restrict__ pb, int nslab, int C,
                                           int c, double& sa, double& sb) {
  __shared__ double red[2][FOLD_Y][64];
  const int lane = threadIdx.y, cx = threadIdx.x;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int k = lane;
    for (; k + 3 * FOLD_Y < nslab; k += 4 * FOLD_Y) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] += pa[(long)(k + FOLD_Y * u) * C + c];
        b[u] += pb[(long)(k + FOLD_Y * u) * C + c];
      }
    }
    for (; k < nslab; k += FOLD_Y) {
      a[0] += pa[(long)k * C + c];
      b[0] += pb[(long)k * C + c];
    }
  }
  red[0][lane][cx] = (double)a[0] + a[1] + a[2] + a[3];
  red[1][lane][cx] = (double)b[0] + b[1] + b[2] + b[3];
  __syncthreads();
  sa = 0.0;
  sb = 0.0;
#pragma unroll
  for (int l = 0; l < FOLD_Y; ++l) {
    sa += red[0][l][cx];
    sb += red[1][l][cx];
  }
}

__global__ void __launch_bounds__(64 * FOLD_Y)
bn_finalize_stats_k(const float* __restrict__ psum, const float* __restrict__ psq,
                    int nslab, int C, long rows, const float* __restrict__ gamma,
                    const float* __restrict__ beta, float decay, float eps,
                    float* __restrict__ run_mean, float* __restrict__ run_var,
                    float* __restrict__ save_mean, float* __restrict__ save_invstd,
                    float* __restrict__ scale, float* __restrict__ shift,
                    float* __restrict__ kshift) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  double s, q;
  fold_slabs(psum, psq, nslab, C, c, s, q);
  if (threadIdx.y != 0 || c >= C) return;
  // Shifted statistics: the partials are sums of (x - K) and (x - K)^2 with
  // K = kshift[c] (the previous step's batch mean of this BN, 0 at first),
  // so var = E[(x-K)^2] - E[x-K]^2 cancels only |mean - K|^2, not mean^2
  // (the plain E[x^2] - E[x]^2 loses every digit of a channel whose mean is
  // large next to its spread).  This step's mean becomes the next step's K.
  const double n = (double)rows;
  const double k = kshift ? (double)kshift[c] : 0.0;
  const double dm = s / n;
  const double mean = k + dm;
  double var = q / n - dm * dm;
  if (var < 0.0) var = 0.0;
  if (kshift) kshift[c] = (float)mean;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  scale[c] = g * invstd;
  shift[c] = b - (float)mean * g * invstd;
  if (run_mean) {
    const double unbiased = rows > 1 ? var * n / (n - 1.0) : var;
    run_mean[c] = run_mean[c] * decay + (float)mean * (1.f - decay);
    run_var[c] = run_var[c] * decay + (float)unbiased * (1.f - decay);
  }
}

__global__ void bn_infer_coefs_k(int C, const float* __restrict__ gamma,
                                 const float* __restrict__ beta, const float* __restrict__ rm,
                                 const float* __restrict__ rv, float eps, float* __restrict__ scale,
                                 float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  const float sc = g * rsqrtf(rv[c] + eps);
  scale[c] = sc;
  shift[c] = b - rm[c] * sc;
}

// Streaming apply passes.  With a power-of-two channel-vector count cv =
// C/V (every ResNet / VGG width) the grid-stride step is a multiple of cv, so
// each thread's channels never change: the per-channel coefficients are read
// once into registers and the loop carries no modulo; two grid steps are
// loaded before either is computed, doubling the bytes in flight per thread
// (the passes were at 3.5-4.2 TB/s with per-element coefficient loads).
template <int V>
__device__ __forceinline__ void coef_load(const float* __restrict__ p, int c, float (&o)[V]) {
#pragma unroll
  for (int k = 0; k < V; ++k) o[k] = p[c + k];
}

// dx = g*A + x*B + C with one fixed FMA order, so every backward apply kernel
// (launch-finalized or folded) rounds the same way
__device__ __forceinline__ float bwd_fma(float g, float a, float x, float b, float c) {
  return __builtin_fmaf(g, a, __builtin_fmaf(x, b, c));
}

// ReLU bit mask of one 8-channel vector of a 2-byte output: bit k of byte
// mb[i] = act_pass(stored y[8i + k]), from the value as rounded to T, so it
// equals the test a consumer would make on y itself.  A conv dgrad epilogue reads
// this byte (1/16 of y's bytes) instead of y (IgArgs::maskbits).
// ACT: the activation after the BN - 1 ReLU, 2 ReLU6 (MobileNet-v2's
// min(max(y, 0), 6), tcb/models/mobilenet_conv_blocks.py); act_pass is its
// gradient gate on the stored output y (the gradient passes where 0 < y, and
// for ReLU6 y < 6).
template <int ACT>
__device__ __forceinline__ float act_apply(float o) {
  o = fmaxf(o, 0.f);
  if constexpr (ACT == 2) o = fminf(o, 6.f);
  return o;
}
template <int ACT>
__device__ __forceinline__ bool act_pass(float y) {
  if constexpr (ACT == 2) return y > 0.f && y < 6.f;
  return y > 0.f;
}

template <typename T, int V, int ACT = 1>
__device__ __forceinline__ void relu_bits(uint8_t* __restrict__ mb, unsigned i, const float (&v)[V]) {
  if constexpr (V == 8 && sizeof(T) == 2) {
    if (!mb) return;
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < V; ++k) b |= (act_pass<ACT>((float)(T)v[k]) ? 1u : 0u) << k;
    mb[i] = (uint8_t)b;
  }
}

template <typename T, int V, bool RES, int RELU, int U = 0>
__global__ void __launch_bounds__(256)
bn_apply_k(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y, long nvec, int C,
           const float* __restrict__ scale, const float* __restrict__ shift,
           uint8_t* __restrict__ mb) {
  // nvec < 2^31 is checked on the host: 32-bit index math avoids 64-bit division.
  const unsigned cv = (unsigned)(C / V);
  const unsigned n = (unsigned)nvec, stride = gridDim.x * blockDim.x;
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  auto apply = [&](float (&v)[V], const float (&rr)[V], const float (&sc)[V],
                   const float (&sf)[V]) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float o = __builtin_fmaf(v[k], sc[k], sf[k]);
      if (RES) o += rr[k];
      if (RELU) o = act_apply<RELU>(o);
      v[k] = o;
    }
  };
  if constexpr (U > 0) {
    // flat: block b owns vectors [b*256*U, (b+1)*256*U); 256 % cv == 0
    const unsigned base = blockIdx.x * 256u * U + threadIdx.x;
    const int c = (int)(threadIdx.x % cv) * V;
    float sc[V], sf[V], v[U][V], rr[U][V];
    coef_load<V>(scale, c, sc);
    coef_load<V>(shift, c, sf);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        load_vec<T, V>(x + (long)i * V, v[u]);
        if (RES) load_vec<T, V>(res + (long)i * V, rr[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        apply(v[u], rr[u], sc, sf);
        store_vec<T, V>(y + (long)i * V, v[u]);
        if (RELU) relu_bits<T, V, RELU>(mb, i, v[u]);
      }
    }
    return;
  }
  if (stride % cv == 0) {
    const int c = (int)(i0 % cv) * V;
    float sc[V], sf[V];
    coef_load<V>(scale, c, sc);
    coef_load<V>(shift, c, sf);
    unsigned i = i0;
    for (; i + stride < n; i += 2 * stride) {
      float v0[V], v1[V], r0[V], r1[V];
      load_vec<T, V>(x + (long)i * V, v0);
      load_vec<T, V>(x + (long)(i + stride) * V, v1);
      if (RES) {
        load_vec<T, V>(res + (long)i * V, r0);
        load_vec<T, V>(res + (long)(i + stride) * V, r1);
      }
      apply(v0, r0, sc, sf);
      apply(v1, r1, sc, sf);
      store_vec<T, V>(y + (long)i * V, v0);
      store_vec<T, V>(y + (long)(i + stride) * V, v1);
      if (RELU) {
        relu_bits<T, V, RELU>(mb, i, v0);
        relu_bits<T, V, RELU>(mb, i + stride, v1);
      }
    }
    if (i < n) {
      float v0[V], r0[V];
      load_vec<T, V>(x + (long)i * V, v0);
      if (RES) load_vec<T, V>(res + (long)i * V, r0);
      apply(v0, r0, sc, sf);
      store_vec<T, V>(y + (long)i * V, v0);
      if (RELU) relu_bits<T, V, RELU>(mb, i, v0);
    }
    return;
  }
  for (unsigned i = i0; i < n; i += stride) {
    const long e = (long)i * V;
    const int c = (int)(i % cv) * V;
    float v[V], rr[V], sc[V], sf[V];
    load_vec<T, V>(x + e, v);
    if (RES) load_vec<T, V>(res + e, rr);
    coef_load<V>(scale, c, sc);
    coef_load<V>(shift, c, sf);
    apply(v, rr, sc, sf);
    store_vec<T, V>(y + e, v);
    if (RELU) relu_bits<T, V, RELU>(mb, i, v);
  }
}

// y = relu?(x * scale + shift + xr * scale_r + shift_r): a BN whose residual
// is itself a BN output with no ReLU (ResNet v1 projection shortcut,
// tcb/models/resnet_model.py:60-75), applied from both raw inputs so the
// shortcut BN output is never materialized.
template <typename T, int V, bool RELU, int U = 0>
__global__ void __launch_bounds__(256)
bn_apply2_k(const T* __restrict__ x, const T* __restrict__ xr, T* __restrict__ y, long nvec, int C,
            const float* __restrict__ scale, const float* __restrict__ shift,
            const float* __restrict__ scale_r, const float* __restrict__ shift_r,
            uint8_t* __restrict__ mb) {
  const unsigned cv = (unsigned)(C / V);
  const unsigned n = (unsigned)nvec, stride = gridDim.x * blockDim.x;
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  auto apply = [&](float (&v)[V], const float (&r)[V], const float (&a)[V], const float (&b)[V],
                   const float (&ar)[V], const float (&br)[V]) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float o = v[k] * a[k] + b[k] + (r[k] * ar[k] + br[k]);
      if (RELU) o = fmaxf(o, 0.f);
      v[k] = o;
    }
  };
  if constexpr (U > 0) {  // flat (see bn_apply_k)
    const unsigned base = blockIdx.x * 256u * U + threadIdx.x;
    const int c = (int)(threadIdx.x % cv) * V;
    float a[V], b[V], ar[V], br[V], v[U][V], r[U][V];
    coef_load<V>(scale, c, a);
    coef_load<V>(shift, c, b);
    coef_load<V>(scale_r, c, ar);
    coef_load<V>(shift_r, c, br);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        load_vec<T, V>(x + (long)i * V, v[u]);
        load_vec<T, V>(xr + (long)i * V, r[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        apply(v[u], r[u], a, b, ar, br);
        store_vec<T, V>(y + (long)i * V, v[u]);
        if (RELU) relu_bits<T, V>(mb, i, v[u]);
      }
    }
    return;
  }
  if (stride % cv == 0) {
    const int c = (int)(i0 % cv) * V;
    float a[V], b[V], ar[V], br[V];
    coef_load<V>(scale, c, a);
    coef_load<V>(shift, c, b);
    coef_load<V>(scale_r, c, ar);
    coef_load<V>(shift_r, c, br);
    unsigned i = i0;
    for (; i + stride < n; i += 2 * stride) {
      float v0[V], v1[V], r0[V], r1[V];
      load_vec<T, V>(x + (long)i * V, v0);
      load_vec<T, V>(x + (long)(i + stride) * V, v1);
      load_vec<T, V>(xr + (long)i * V, r0);
      load_vec<T, V>(xr + (long)(i + stride) * V, r1);
      apply(v0, r0, a, b, ar, br);
      apply(v1, r1, a, b, ar, br);
      store_vec<T, V>(y + (long)i * V, v0);
      store_vec<T, V>(y + (long)(i + stride) * V, v1);
      if (RELU) {
        relu_bits<T, V>(mb, i, v0);
        relu_bits<T, V>(mb, i + stride, v1);
      }
    }
    if (i < n) {
      float v0[V], r0[V];
      load_vec<T, V>(x + (long)i * V, v0);
      load_vec<T, V>(xr + (long)i * V, r0);
      apply(v0, r0, a, b, ar, br);
      store_vec<T, V>(y + (long)i * V, v0);
      if (RELU) relu_bits<T, V>(mb, i, v0);
    }
    return;
  }
  for (unsigned i = i0; i < n; i += stride) {
    const long e = (long)i * V;
    const int c = (int)(i % cv) * V;
    float v[V], r[V], a[V], b[V], ar[V], br[V];
    load_vec<T, V>(x + e, v);
    load_vec<T, V>(xr + e, r);
    coef_load<V>(scale, c, a);
    coef_load<V>(shift, c, b);
    coef_load<V>(scale_r, c, ar);
    coef_load<V>(shift_r, c, br);
    apply(v, r, a, b, ar, br);
    store_vec<T, V>(y + e, v);
    if (RELU) relu_bits<T, V>(mb, i, v);
  }
}

// ---------------------------------------------------------------- backward
template <typename T, int V, int MASK>
__global__ void __launch_bounds__(BN_THREADS)
bn_partial_grad_k(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x,
                  const float* __restrict__ mean, long rows, int C, int cw, int tpr, int rpi,
                  long slab_rows, float* __restrict__ pdy, float* __restrict__ pdyx) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int t = tid % tpr, r = tid / tpr;
  const int c0 = blockIdx.y * cw + t * V;
  const bool cok = (c0 < C) && (r < rpi);
  float s[V], q[V], m[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { s[i] = 0.f; q[i] = 0.f; m[i] = cok ? mean[c0 + i] : 0.f; }
  const long rbeg = (long)blockIdx.x * slab_rows;
  long rend = rbeg + slab_rows;
  if (rend > rows) rend = rows;
  if (cok) {
    // 4 rows per iteration, every load issued before any is used: one block
    // per CU streams 2-3 tensors, so the loop is latency-bound without the
    // loads of several rows in flight (3.0-3.4 TB/s on the ResNet shapes)
    auto row_acc = [&](const float (&g0)[V], const float (&xv)[V], const float (&yv)[V]) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float g = (!MASK || act_pass<MASK>(yv[i])) ? g0[i] : 0.f;
        s[i] += g;
        q[i] += g * (xv[i] - m[i]);
      }
    };
    long row = rbeg + r;
    for (; row + 3 * rpi < rend; row += 4 * rpi) {
      float g[4][V], xv[4][V], yv[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long off = (row + u * rpi) * C + c0;
        load_vec<T, V>(dy + off, g[u]);
        load_vec<T, V>(x + off, xv[u]);
        if (MASK) load_vec<T, V>(y + off, yv[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) row_acc(g[u], xv[u], yv[u]);
    }
    for (; row < rend; row += rpi) {
      const long off = row * C + c0;
      float g[V], xv[V], yv[V];
      load_vec<T, V>(dy + off, g);
      load_vec<T, V>(x + off, xv);
      if (MASK) load_vec<T, V>(y + off, yv);
      row_acc(g, xv, yv);
    }
  }
  block_row_reduce<V>(s, q, lds, t, r, tpr, rpi);
  if (r == 0 && c0 < C) {
    float* ps = pdy + (long)blockIdx.x * C + c0;
    float* pq = pdyx + (long)blockIdx.x * C + c0;
#pragma unroll
    for (int i = 0; i < V; ++i) { ps[i] = s[i]; pq[i] = q[i]; }
  }
}

// dgamma = invstd * sum(dy'(x-mean)); dbeta = sum(dy').
// dx = dy'*A + x*B + Cc  with A = g*invstd, B = -A*invstd^2*S2/n,
// Cc = -A*S1/n - mean*B.
__global__ void __launch_bounds__(64 * FOLD_Y)
bn_finalize_grad_k(const float* __restrict__ pdy, const float* __restrict__ pdyx,
                   int nslab, int C, long rows, const float* __restrict__ gamma,
                   const float* __restrict__ mean, const float* __restrict__ invstd,
                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                   float* __restrict__ coefA, float* __restrict__ coefB,
                   float* __restrict__ coefC, int accumulate, int s2_over_scale) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  double s1, s2;
  fold_slabs(pdy, pdyx, nslab, C, c, s1, s2);
  if (threadIdx.y != 0 || c >= C) return;
  const float is = invstd[c];
  const float g = gamma ? gamma[c] : 1.f;
  // s2_over_scale: the partials hold sum(dy' (y - beta)) over the BN output y
  // (the stem pool's consumers, see kfb_bn_relu_maxpool_bwd), and
  // x - mean = (y - beta) / (gamma * invstd) where the ReLU passed
  if (s2_over_scale) s2 /= (double)g * (double)is;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)(s2 * is);
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)s1;
  const double n = (double)rows;
  const double A = (double)g * is;
  const double B = -A * (double)is * (double)is * s2 / n;
  coefA[c] = (float)A;
  coefB[c] = (float)B;
  coefC[c] = (float)(-A * s1 / n - (double)mean[c] * B);
}

template <typename T, int V, int MASK, bool DRES, int U = 0>
__global__ void __launch_bounds__(256)
bn_bwd_apply_k(const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x,
               T* __restrict__ dx, T* __restrict__ dres, long nvec, int C,
               const float* __restrict__ A, const float* __restrict__ B,
               const float* __restrict__ Cc) {
  // nvec < 2^31 is checked on the host: 32-bit index math avoids 64-bit division.
  const unsigned cv = (unsigned)(C / V);
  const unsigned n = (unsigned)nvec, stride = gridDim.x * blockDim.x;
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (U > 0) {  // flat (see bn_apply_k)
    const unsigned base = blockIdx.x * 256u * U + threadIdx.x;
    const int c = (int)(threadIdx.x % cv) * V;
    float a[V], b[V], cc[V], g[U][V], xv[U][V], yv[U][V];
    coef_load<V>(A, c, a);
    coef_load<V>(B, c, b);
    coef_load<V>(Cc, c, cc);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        load_vec<T, V>(dy + (long)i * V, g[u]);
        load_vec<T, V>(x + (long)i * V, xv[u]);
        if (MASK) load_vec<T, V>(y + (long)i * V, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        if (MASK) {
#pragma unroll
          for (int k = 0; k < V; ++k) g[u][k] = act_pass<MASK>(yv[u][k]) ? g[u][k] : 0.f;
        }
        if (DRES) store_vec<T, V>(dres + (long)i * V, g[u]);
        float o[V];
#pragma unroll
        for (int k = 0; k < V; ++k) o[k] = bwd_fma(g[u][k], a[k], xv[u][k], b[k], cc[k]);
        store_vec<T, V>(dx + (long)i * V, o);
      }
    }
    return;
  }
  // g <- mask(dy); dres <- g; dx <- g*A + x*B + Cc
  auto step2 = [&](unsigned ia, unsigned ib, bool two, const float (&a)[V], const float (&b)[V],
                   const float (&cc)[V]) {
    float g0[V], g1[V], x0[V], x1[V];
    load_vec<T, V>(dy + (long)ia * V, g0);
    load_vec<T, V>(x + (long)ia * V, x0);
    if (two) {
      load_vec<T, V>(dy + (long)ib * V, g1);
      load_vec<T, V>(x + (long)ib * V, x1);
    }
    if (MASK) {
      float y0[V], y1[V];
      load_vec<T, V>(y + (long)ia * V, y0);
      if (two) load_vec<T, V>(y + (long)ib * V, y1);
#pragma unroll
      for (int k = 0; k < V; ++k) g0[k] = act_pass<MASK>(y0[k]) ? g0[k] : 0.f;
      if (two) {
#pragma unroll
        for (int k = 0; k < V; ++k) g1[k] = act_pass<MASK>(y1[k]) ? g1[k] : 0.f;
      }
    }
    if (DRES) {
      store_vec<T, V>(dres + (long)ia * V, g0);
      if (two) store_vec<T, V>(dres + (long)ib * V, g1);
    }
    float o0[V], o1[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      o0[k] = bwd_fma(g0[k], a[k], x0[k], b[k], cc[k]);
      o1[k] = bwd_fma(g1[k], a[k], x1[k], b[k], cc[k]);
    }
    store_vec<T, V>(dx + (long)ia * V, o0);
    if (two) store_vec<T, V>(dx + (long)ib * V, o1);
  };
  if (stride % cv == 0) {
    const int c = (int)(i0 % cv) * V;
    float a[V], b[V], cc[V];
    coef_load<V>(A, c, a);
    coef_load<V>(B, c, b);
    coef_load<V>(Cc, c, cc);
    unsigned i = i0;
    for (; i + stride < n; i += 2 * stride) step2(i, i + stride, true, a, b, cc);
    if (i < n) step2(i, i, false, a, b, cc);
    return;
  }
  for (unsigned i = i0; i < n; i += stride) {
    const int c = (int)(i % cv) * V;
    float a[V], b[V], cc[V];
    coef_load<V>(A, c, a);
    coef_load<V>(B, c, b);
    coef_load<V>(Cc, c, cc);
    step2(i, i, false, a, b, cc);
  }
}

// ---- backward apply with the gradient finalize folded in ------------------
// In the backward pass a finalize launch sits between the dgrad that summed
// a BN's backward partials and the apply pass that needs its coefficients;
// beside the weight-gradient stream such a 5 us kernel waits for a dispatch
// slot and took 19 us on average in the ResNet-50 bs256 step (38 launches,
// 0.73 ms of the compute stream, profiles/r12_step_timeline.txt).  Here
// each workgroup owns one 64-channel slice and a set of rows: it folds the
// 32 conv-epilogue slots of its 64 channels (2 x 32 x 64 floats, one L2
// round trip) with the arithmetic of fold_slabs + bn_finalize_grad_k, so
// the coefficients are bitwise the finalize launch's, then streams its rows.
// Workgroups of row block 0 write dgamma / dbeta and the coefficient arrays.
// DUAL: the apply of kfb_bn_bwd_dual (the residual branch's coefficients
// come from its own finalize launch: its partials are bn_partial_grad_k's).
constexpr int FS_C = 64;      // channels per slice (8 lanes x 8 channels)
constexpr int FS_SLOTS = 32;  // conv-epilogue slots (IG_SPREAD)

struct BnFoldArgs {
  const float* pdy;
  const float* pdyx;
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* coefA;
  float* coefB;
  float* coefC;
  int accumulate;
};

// FR (with DUAL): the second BN's finalize is folded too, from fr.pdyx and
// the first BN's sum dy' (the dual dgrad epilogue's partials,
// kfb_conv_s1_dgrad_dual); else its coefficients Ar / Br / Cr come from a
// finalize launch.
template <typename T, bool DRES, bool DUAL, bool FR = false>
__global__ void __launch_bounds__(256)
bn_bwd_apply_fold_k(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ xr,
                    T* __restrict__ dx, T* __restrict__ dres, long rows, int C, BnFoldArgs f,
                    const float* __restrict__ Ar, const float* __restrict__ Br,
                    const float* __restrict__ Cr, BnFoldArgs fr) {
  static_assert(FOLD_Y == 16 && FS_SLOTS == 2 * FOLD_Y, "fold order of fold_slabs");
  static_assert(!FR || DUAL, "second-BN fold needs the dual form");
  constexpr int NA = FR ? 3 : 2;  // slot arrays: sum dy', sum dy'(x - mean)[, sum dy'(xr - mean_r)]
  __shared__ double red[NA][FOLD_Y][FS_C];
  __shared__ double tot[NA][FS_C];
  __shared__ float cf[FR ? 6 : 3][FS_C];
  const int t = threadIdx.x;
  const int ns = C / FS_C;
  const int slice = blockIdx.x % ns, rb = blockIdx.x / ns, nrb = gridDim.x / ns;
  const int c0 = slice * FS_C;
  const int q = t & 7;
  const int c = c0 + 8 * q;
  const long step = (long)nrb * 32;
  long r = (long)rb * 32 + (t >> 3);
  // the first two rows' operands are issued before the fold, so their
  // latency overlaps its L2 round trip and LDS reduction
  float g0[8], g1[8], x0[8], x1[8], r0[8], r1[8];
  const bool has0 = r < rows, has1 = r + step < rows;
  if (has0) {
    load_vec<T, 8>(dy + r * C + c, g0);
    load_vec<T, 8>(x + r * C + c, x0);
    if constexpr (DUAL) load_vec<T, 8>(xr + r * C + c, r0);
  }
  if (has1) {
    load_vec<T, 8>(dy + (r + step) * C + c, g1);
    load_vec<T, 8>(x + (r + step) * C + c, x1);
    if constexpr (DUAL) load_vec<T, 8>(xr + (r + step) * C + c, r1);
  }
  {
    // fold_slabs' order for 32 slots: lane l holds float(p[l] + p[l + 16]),
    // the 16 lanes are summed in double in lane order
    const int arr = t >> 7, l = (t >> 3) & 15;
    const float* p = (arr ? f.pdyx : f.pdy) + c0 + 8 * q;
    const float4* lo = (const float4*)(p + (long)l * C);
    const float4* hi = (const float4*)(p + (long)(l + FOLD_Y) * C);
    const float4 a0 = lo[0], a1 = lo[1], b0 = hi[0], b1 = hi[1];
    const float sv[8] = {a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w,
                         a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) red[arr][l][8 * q + k] = (double)sv[k];
  }
  if constexpr (FR) {
    if (t < 128) {  // the second BN's sum dy'(xr - mean_r) slots, same order
      const int l = (t >> 3) & 15;
      const float* p = fr.pdyx + c0 + 8 * q;
      const float4* lo = (const float4*)(p + (long)l * C);
      const float4* hi = (const float4*)(p + (long)(l + FOLD_Y) * C);
      const float4 a0 = lo[0], a1 = lo[1], b0 = hi[0], b1 = hi[1];
      const float sv[8] = {a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w,
                           a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) red[NA - 1][l][8 * q + k] = (double)sv[k];
    }
  }
  __syncthreads();
  if (t < NA * FS_C) {
    const int arr = t >> 6, cc = t & 63;
    double sum = 0.0;
#pragma unroll
    for (int l = 0; l < FOLD_Y; ++l) sum += red[arr][l][cc];
    tot[arr][cc] = sum;
  }
  __syncthreads();
  if (t < FS_C) {
    const int ch = c0 + t;
    const double s1 = tot[0][t], s2 = tot[1][t];
    // (the math of bn_finalize_grad_k)
    const float is = f.invstd[ch];
    const float g = f.gamma ? f.gamma[ch] : 1.f;
    const double n = (double)rows;
    const double A = (double)g * is;
    const double B = -A * (double)is * (double)is * s2 / n;
    const float av = (float)A, bv = (float)B, cv = (float)(-A * s1 / n - (double)f.mean[ch] * B);
    cf[0][t] = av;
    cf[1][t] = bv;
    cf[2][t] = cv;
    if (rb == 0) {
      if (f.dgamma) f.dgamma[ch] = (f.accumulate ? f.dgamma[ch] : 0.f) + (float)(s2 * is);
      if (f.dbeta) f.dbeta[ch] = (f.accumulate ? f.dbeta[ch] : 0.f) + (float)s1;
      f.coefA[ch] = av;
      f.coefB[ch] = bv;
      f.coefC[ch] = cv;
    }
  } else if (FR && t < 2 * FS_C) {
    // the second BN: its sum dy' is the first's (one ReLU-masked dy')
    const int u = t - FS_C, ch = c0 + u;
    const double s1 = tot[0][u], s2 = tot[NA - 1][u];
    const float is = fr.invstd[ch];
    const float g = fr.gamma ? fr.gamma[ch] : 1.f;
    const double n = (double)rows;
    const double A = (double)g * is;
    const double B = -A * (double)is * (double)is * s2 / n;
    const float av = (float)A, bv = (float)B, cv = (float)(-A * s1 / n - (double)fr.mean[ch] * B);
    cf[FR ? 3 : 0][u] = av;
    cf[FR ? 4 : 0][u] = bv;
    cf[FR ? 5 : 0][u] = cv;
    if (rb == 0) {
      if (fr.dgamma) fr.dgamma[ch] = (fr.accumulate ? fr.dgamma[ch] : 0.f) + (float)(s2 * is);
      if (fr.dbeta) fr.dbeta[ch] = (fr.accumulate ? fr.dbeta[ch] : 0.f) + (float)s1;
      fr.coefA[ch] = av;
      fr.coefB[ch] = bv;
      fr.coefC[ch] = cv;
    }
  }
  __syncthreads();
  float a[8], b[8], cc[8], ar[8], br[8], crr[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = cf[0][8 * q + k];
    b[k] = cf[1][8 * q + k];
    cc[k] = cf[2][8 * q + k];
  }
  if constexpr (FR) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ar[k] = cf[FR ? 3 : 0][8 * q + k];
      br[k] = cf[FR ? 4 : 0][8 * q + k];
      crr[k] = cf[FR ? 5 : 0][8 * q + k];
    }
  } else if constexpr (DUAL) {
    coef_load<8>(Ar, c, ar);
    coef_load<8>(Br, c, br);
    coef_load<8>(Cr, c, crr);
  }
  // one row's outputs from its loaded operands
  auto emit = [&](long e, const float (&gv)[8], const float (&xv)[8], const float (&rv)[8]) {
    float o[8];
    if constexpr (DUAL) {
      float o2[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o2[k] = bwd_fma(gv[k], ar[k], rv[k], br[k], crr[k]);
      store_vec<T, 8>(dres + e, o2);
    } else if constexpr (DRES) {
      store_vec<T, 8>(dres + e, gv);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = bwd_fma(gv[k], a[k], xv[k], b[k], cc[k]);
    store_vec<T, 8>(dx + e, o);
  };
  if (!has0) return;
  emit(r * C + c, g0, x0, r0);
  if (!has1) return;
  emit((r + step) * C + c, g1, x1, r1);
  for (r += 2 * step; r < rows; r += 2 * step) {
    // both rows' loads issue before either is used
    const bool two = r + step < rows;
    const long e0 = r * C + c, e1 = (r + step) * C + c;
    load_vec<T, 8>(dy + e0, g0);
    load_vec<T, 8>(x + e0, x0);
    if constexpr (DUAL) load_vec<T, 8>(xr + e0, r0);
    if (two) {
      load_vec<T, 8>(dy + e1, g1);
      load_vec<T, 8>(x + e1, x1);
      if constexpr (DUAL) load_vec<T, 8>(xr + e1, r1);
    }
    emit(e0, g0, x0, r0);
    if (two) emit(e1, g1, x1, r1);
  }
}

template <typename T, int V, int U = 0>
__global__ void __launch_bounds__(256)
bn_bwd_apply2_k(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ xr,
                T* __restrict__ dx, T* __restrict__ dxr, long nvec, int C,
                const float* __restrict__ A, const float* __restrict__ B,
                const float* __restrict__ Cc, const float* __restrict__ Ar,
                const float* __restrict__ Br, const float* __restrict__ Cr) {
  const unsigned cv = (unsigned)(C / V);
  const unsigned n = (unsigned)nvec, stride = gridDim.x * blockDim.x;
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  struct Co { float a[V], b[V], c[V], ar[V], br[V], cr[V]; };
  auto coefs = [&](int c, Co& k) {
    coef_load<V>(A, c, k.a);
    coef_load<V>(B, c, k.b);
    coef_load<V>(Cc, c, k.c);
    coef_load<V>(Ar, c, k.ar);
    coef_load<V>(Br, c, k.br);
    coef_load<V>(Cr, c, k.cr);
  };
  if constexpr (U > 0) {  // flat (see bn_apply_k)
    const unsigned base = blockIdx.x * 256u * U + threadIdx.x;
    Co k;
    coefs((int)(threadIdx.x % cv) * V, k);
    float g[U][V], xv[U][V], rv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        load_vec<T, V>(dy + (long)i * V, g[u]);
        load_vec<T, V>(x + (long)i * V, xv[u]);
        load_vec<T, V>(xr + (long)i * V, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = base + u * 256u;
      if (i < n) {
        float o[V], q[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          o[j] = bwd_fma(g[u][j], k.a[j], xv[u][j], k.b[j], k.c[j]);
          q[j] = bwd_fma(g[u][j], k.ar[j], rv[u][j], k.br[j], k.cr[j]);
        }
        store_vec<T, V>(dx + (long)i * V, o);
        store_vec<T, V>(dxr + (long)i * V, q);
      }
    }
    return;
  }
  auto one = [&](unsigned i, const Co& k) {
    float g[V], xv[V], rv[V], o[V], orr[V];
    load_vec<T, V>(dy + (long)i * V, g);
    load_vec<T, V>(x + (long)i * V, xv);
    load_vec<T, V>(xr + (long)i * V, rv);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      o[j] = bwd_fma(g[j], k.a[j], xv[j], k.b[j], k.c[j]);
      orr[j] = bwd_fma(g[j], k.ar[j], rv[j], k.br[j], k.cr[j]);
    }
    store_vec<T, V>(dx + (long)i * V, o);
    store_vec<T, V>(dxr + (long)i * V, orr);
  };
  if (stride % cv == 0) {
    Co k;
    coefs((int)(i0 % cv) * V, k);
    unsigned i = i0;
    for (; i + stride < n; i += 2 * stride) {
      float g0[V], x0[V], r0[V], g1[V], x1[V], r1[V];
      load_vec<T, V>(dy + (long)i * V, g0);
      load_vec<T, V>(x + (long)i * V, x0);
      load_vec<T, V>(xr + (long)i * V, r0);
      load_vec<T, V>(dy + (long)(i + stride) * V, g1);
      load_vec<T, V>(x + (long)(i + stride) * V, x1);
      load_vec<T, V>(xr + (long)(i + stride) * V, r1);
      float o0[V], q0[V], o1[V], q1[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        o0[j] = bwd_fma(g0[j], k.a[j], x0[j], k.b[j], k.c[j]);
        q0[j] = bwd_fma(g0[j], k.ar[j], r0[j], k.br[j], k.cr[j]);
        o1[j] = bwd_fma(g1[j], k.a[j], x1[j], k.b[j], k.c[j]);
        q1[j] = bwd_fma(g1[j], k.ar[j], r1[j], k.br[j], k.cr[j]);
      }
      store_vec<T, V>(dx + (long)i * V, o0);
      store_vec<T, V>(dxr + (long)i * V, q0);
      store_vec<T, V>(dx + (long)(i + stride) * V, o1);
      store_vec<T, V>(dxr + (long)(i + stride) * V, q1);
    }
    if (i < n) one(i, k);
    return;
  }
  for (unsigned i = i0; i < n; i += stride) {
    Co k;
    coefs((int)(i % cv) * V, k);
    one(i, k);
  }
}

// --------------------------------------------- BN + ReLU + max-pool (stem)
// The ResNet stem tail relu(bn(conv1)) -> maxpool 3x3/2 as one op
// (tcb/models/resnet_model.py:306-312): the forward never materializes the
// 112x112 BN output (it normalizes each window tap on the fly and keeps the
// argmax byte), and the backward never materializes the max-pool gradient
// (each input pixel gathers the pooled gradients that routed to it, ReLU
// masked by the pooled value, in both the partial-sum and the apply pass).
struct BPGeo {
  int N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl;
};

// K3 = true: 3x3 windows with every tap's load issued before the max (taps
// outside the input read a clamped in-range pixel and are masked off); the
// generic loop leaves each load behind a bounds branch.
template <typename T, int V, bool K3 = false>
__global__ void __launch_bounds__(256)
bn_relu_maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ z, uint8_t* __restrict__ idx,
                      const float* __restrict__ scale, const float* __restrict__ shift, BPGeo g) {
  // 32-bit index math (the host checks the element counts < 2^31)
  const unsigned cv = (unsigned)(g.C / V);
  const unsigned total = (unsigned)g.N * g.OH * g.OW * cv;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    unsigned p = i / cv;
    const int ow = (int)(p % (unsigned)g.OW); p /= (unsigned)g.OW;
    const int oh = (int)(p % (unsigned)g.OH);
    const int n = (int)(p / (unsigned)g.OH);
    float sc[V], sf[V], best[V];
    int bi[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      sc[k] = scale[c + k]; sf[k] = shift[c + k]; best[k] = -INFINITY; bi[k] = 0;
    }
    const int h0 = oh * g.sh - g.pt, w0 = ow * g.sw - g.pl;
    if constexpr (K3) {
      float v[9][V];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const int h = min(max(h0 + a, 0), g.H - 1), w = min(max(w0 + b, 0), g.W - 1);
          load_vec<T, V>(x + (((long)n * g.H + h) * g.W + w) * g.C + c, v[a * 3 + b]);
        }
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const bool in = (unsigned)(h0 + a) < (unsigned)g.H && (unsigned)(w0 + b) < (unsigned)g.W;
#pragma unroll
          for (int k = 0; k < V; ++k) {
            const float o = (float)from_f32<T>(fmaxf(v[a * 3 + b][k] * sc[k] + sf[k], 0.f));
            if (in && o > best[k]) { best[k] = o; bi[k] = a * 3 + b; }
          }
        }
    }
    for (int a = 0; !K3 && a < g.kh; ++a) {
      const int h = h0 + a;
      if (h < 0 || h >= g.H) continue;
      for (int b = 0; b < g.kw; ++b) {
        const int w = w0 + b;
        if (w < 0 || w >= g.W) continue;
        float v[V];
        load_vec<T, V>(x + (((long)n * g.H + h) * g.W + w) * g.C + c, v);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          // same bf16 rounding as the unfused BN output the pool would read
          const float o = (float)from_f32<T>(fmaxf(v[k] * sc[k] + sf[k], 0.f));
          if (o > best[k]) { best[k] = o; bi[k] = a * g.kw + b; }
        }
      }
    }
    const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c;
    store_vec<T, V>(z + o, best);
    Vec<uint8_t, V> iv;
#pragma unroll
    // bit 7: the pooled value is 0 (every input <= 0 after the ReLU), so no
    // gradient flows - the backward compares idx with a 0..8 window position
    // and needs no read of the pooled output for the ReLU mask
    for (int k = 0; k < V; ++k) iv.v[k] = (uint8_t)(bi[k] | (best[k] > 0.f ? 0 : 0x80));
    *reinterpret_cast<Vec<uint8_t, V>*>(idx + o) = iv;
  }
}

// Gradient reaching BN-output pixel (n, h, w), channels c..c+V-1: the sum of
// the pooled gradients whose argmax is this pixel, where the pooled value is
// > 0 (ReLU mask: the pooled value IS the ReLU output at the argmax).
template <typename T, int V>
__device__ __forceinline__ void pool_route_grad(const T* __restrict__ dz, const T* __restrict__ z,
                                                const uint8_t* __restrict__ idx, const BPGeo& g,
                                                int n, int h, int w, int c, float (&acc)[V]) {
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
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int a = h - (oh * g.sh - g.pt);
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int pos = a * g.kw + (w - (ow * g.sw - g.pl));
      const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c;
      float d[V];
      load_vec<T, V>(dz + o, d);
      const Vec<uint8_t, V> iv = *reinterpret_cast<const Vec<uint8_t, V>*>(idx + o);
#pragma unroll
      for (int k = 0; k < V; ++k)
        if (iv.v[k] == pos) acc[k] += d[k];  // bit 7 (pooled value 0) never matches
    }
  }
}

// Pass 1: per-slab sums of g and g*(x - mean) (g = routed, masked gradient).
template <typename T, int V>
__global__ void __launch_bounds__(BN_THREADS)
bn_pool_partial_grad_k(const T* __restrict__ dz, const T* __restrict__ z,
                       const uint8_t* __restrict__ idx, const T* __restrict__ x,
                       const float* __restrict__ mean, BPGeo g, long rows, int cw, int tpr,
                       int rpi, long slab_rows, float* __restrict__ pdy, float* __restrict__ pdyx) {
  extern __shared__ float lds[];
  const int C = g.C;
  const int tid = threadIdx.x;
  const int t = tid % tpr, r = tid / tpr;
  const int c0 = blockIdx.y * cw + t * V;
  const bool cok = (c0 < C) && (r < rpi);
  float s[V], q[V], m[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { s[i] = 0.f; q[i] = 0.f; m[i] = cok ? mean[c0 + i] : 0.f; }
  const long rbeg = (long)blockIdx.x * slab_rows;
  long rend = rbeg + slab_rows;
  if (rend > rows) rend = rows;
  if (cok) {
    for (long row = rbeg + r; row < rend; row += rpi) {
      const unsigned ur = (unsigned)row;
      const int w = (int)(ur % (unsigned)g.W);
      const unsigned hn = ur / (unsigned)g.W;
      const int h = (int)(hn % (unsigned)g.H), n = (int)(hn / (unsigned)g.H);
      float gr[V], xv[V];
      pool_route_grad<T, V>(dz, z, idx, g, n, h, w, c0, gr);
      load_vec<T, V>(x + row * C + c0, xv);
#pragma unroll
      for (int i = 0; i < V; ++i) { s[i] += gr[i]; q[i] += gr[i] * (xv[i] - m[i]); }
    }
  }
  block_row_reduce<V>(s, q, lds, t, r, tpr, rpi);
  if (r == 0 && c0 < C) {
    float* ps = pdy + (long)blockIdx.x * C + c0;
    float* pq = pdyx + (long)blockIdx.x * C + c0;
#pragma unroll
    for (int i = 0; i < V; ++i) { ps[i] = s[i]; pq[i] = q[i]; }
  }
}

// Pass 2: dx = g*A + x*B + Cc for every BN input pixel.
template <typename T, int V>
__global__ void __launch_bounds__(256)
bn_pool_bwd_apply_k(const T* __restrict__ dz, const T* __restrict__ z,
                    const uint8_t* __restrict__ idx, const T* __restrict__ x, T* __restrict__ dx,
                    BPGeo g, const float* __restrict__ A, const float* __restrict__ B,
                    const float* __restrict__ Cc) {
  const unsigned cv = (unsigned)(g.C / V);
  const unsigned total = (unsigned)g.N * g.H * g.W * cv;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * V;
    const unsigned row = i / cv;
    const int w = (int)(row % (unsigned)g.W);
    const unsigned hn = row / (unsigned)g.W;
    const int h = (int)(hn % (unsigned)g.H), n = (int)(hn / (unsigned)g.H);
    float gr[V], xv[V], o[V];
    pool_route_grad<T, V>(dz, z, idx, g, n, h, w, c, gr);
    load_vec<T, V>(x + row * g.C + c, xv);
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = gr[k] * A[c + k] + xv[k] * B[c + k] + Cc[c + k];
    store_vec<T, V>(dx + row * g.C + c, o);
  }
}

// 3x3 / stride-2 specialization (the ResNet stem pool).  A thread owns the
// 2x2 block of BN-output pixels (2*oy - pt + a, 2*ox - pl + b), a, b in {0,1},
// for 8 channels: exactly the windows (oy-1|oy, ox-1|ox) can route gradient
// into it, so the thread reads those <= 4 windows once for 4 pixels (the
// generic gather above reads up to 4 windows per pixel) and needs no
// per-window index arithmetic.
template <typename T>
__device__ __forceinline__ void route_block_3s2(const T* __restrict__ dz, const T* __restrict__ z,
                                                const uint8_t* __restrict__ idx, const BPGeo& g,
                                                int n, int oy, int ox, int c,
                                                float (&gr)[2][2][8]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int k = 0; k < 8; ++k) gr[a][b][k] = 0.f;
  // all four windows' loads are issued before any routing (windows outside
  // the pooled grid read a clamped in-range window and are masked off)
  float d[2][2][8];
  Vec<uint8_t, 8> ivs[2][2];
#pragma unroll
  for (int dy = -1; dy <= 0; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 0; ++dx) {
      const int oh = max(oy + dy, 0), ow = max(ox + dx, 0);
      const bool in = (oy + dy) >= 0 && (ox + dx) >= 0 && oh < g.OH && ow < g.OW;
      const long o = (((long)n * g.OH + min(oh, g.OH - 1)) * g.OW + min(ow, g.OW - 1)) * g.C + c;
      load_vec<T, 8>(dz + o, d[dy + 1][dx + 1]);
      ivs[dy + 1][dx + 1] = *reinterpret_cast<const Vec<uint8_t, 8>*>(idx + o);
      if (!in) {
#pragma unroll
        for (int k = 0; k < 8; ++k) ivs[dy + 1][dx + 1].v[k] = 0xff;
      }
    }
#pragma unroll
  for (int dy = -1; dy <= 0; ++dy) {
#pragma unroll
    for (int dx = -1; dx <= 0; ++dx) {
      const Vec<uint8_t, 8> iv = ivs[dy + 1][dx + 1];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int rh = a - 2 * dy;  // row of pixel a inside window oh: 0..3
        if (rh > 2) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int rw = b - 2 * dx;
          if (rw > 2) continue;
          const int pos = rh * 3 + rw;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (iv.v[k] == pos) gr[a][b][k] += d[dy + 1][dx + 1][k];
        }
      }
    }
  }
}

// PASS 0: per-block partial sums of g and g*(x-mean) -> slab blockIdx.x
// (threads of a block share a channel group iff C/8 divides 256).
// PASS 1: dx = g*A + x*B + Cc.
template <typename T, int PASS>
__global__ void __launch_bounds__(256)
bn_pool3s2_k(const T* __restrict__ dz, const T* __restrict__ z, const uint8_t* __restrict__ idx,
             const T* __restrict__ x, T* __restrict__ dx, BPGeo g, int OHo, int OWo,
             const float* __restrict__ mean, float* __restrict__ pdy, float* __restrict__ pdyx,
             const float* __restrict__ A, const float* __restrict__ B,
             const float* __restrict__ Cc) {
  const unsigned cv = (unsigned)(g.C / 8);
  const unsigned total = (unsigned)g.N * OHo * OWo * cv;
  const int c = (int)(threadIdx.x % cv) * 8;  // fixed: the grid stride is a multiple of cv
  float cA[8], cB[8], cC[8], m[8], s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (PASS == 0) { m[k] = mean[c + k]; s[k] = 0.f; q[k] = 0.f; }
    else { cA[k] = A[c + k]; cB[k] = B[c + k]; cC[k] = Cc[c + k]; }
  }
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += gridDim.x * blockDim.x) {
    unsigned p = i / cv;
    const int ox = (int)(p % (unsigned)OWo); p /= (unsigned)OWo;
    const int oy = (int)(p % (unsigned)OHo);
    const int n = (int)(p / (unsigned)OHo);
    // the block's 4 x loads go out first (clamped in-range addresses, masked
    // below), so they fly with the window loads of the routing instead of
    // after it (the partial pass was latency-bound at ~2 TB/s)
    float xb[2][2][8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = min(max(2 * oy - g.pt + a, 0), g.H - 1);
        const int w = min(max(2 * ox - g.pl + b, 0), g.W - 1);
        load_vec<T, 8>(x + (((long)n * g.H + h) * g.W + w) * g.C + c, xb[a][b]);
      }
    float gr[2][2][8];
    route_block_3s2<T>(dz, z, idx, g, n, oy, ox, c, gr);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * oy - g.pt + a;
      if ((unsigned)h >= (unsigned)g.H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * ox - g.pl + b;
        if ((unsigned)w >= (unsigned)g.W) continue;
        const long e = (((long)n * g.H + h) * g.W + w) * g.C + c;
        const float (&xv)[8] = xb[a][b];
        if (PASS == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { s[k] += gr[a][b][k]; q[k] += gr[a][b][k] * (xv[k] - m[k]); }
        } else {
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = bwd_fma(gr[a][b][k], cA[k], xv[k], cB[k], cC[k]);
          store_vec<T, 8>(dx + e, o);
        }
      }
    }
  }
  if (PASS == 0) {
    // fold the 256/cv threads of each channel group: LDS [256][16]
    __shared__ float red[256 * 17];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[threadIdx.x * 17 + k] = s[k];
      red[threadIdx.x * 17 + 8 + k] = q[k];
    }
    __syncthreads();
    if (threadIdx.x < cv * 16) {
      const int grp = threadIdx.x / 16, k = threadIdx.x % 16;
      float acc = 0.f;
      for (int t = grp; t < 256; t += cv) acc += red[t * 17 + k];
      float* dst = (k < 8 ? pdy : pdyx) + (long)blockIdx.x * g.C + grp * 8 + (k & 7);
      *dst = acc;
    }
  }
}

// Flat apply passes: one block per 1024 vectors, all of a thread's 4 loads
// issued before any compute, no grid-stride loop; needs a power-of-two
// channel-vector count dividing 256.  Used for tensors of >= 256 MB (ResNet-50
// bs256 stage 1: 4.3 -> 5.6 TB/s in isolation, +1% on the step); below that
// the grid-stride passes run (isolated rates within +-5%, but the flat grids
// cost ResNet-152 bs128 ~6% beside the weight-gradient stream).
// (mode 1 of the round-2 A/B: flat above the size threshold; 0 = never and
// 2 = every size both lost)
static int bn_flat_mode() { return 1; }

static bool flat_ok(long nvec, int C, int V) {
  const int cv = C / V;
  const int mode = bn_flat_mode();
  const long bytes = nvec * 16;
  // tensors from 64 MB up (was 256 MB: -0.09 and -0.16 ms/step on interleaved ResNet-50 runs,
  // 16 MB no better; profiles/r13_bn_launch_ab.txt)
  return mode > 0 && (mode == 2 || bytes >= (64L << 20)) && cv > 0 && (cv & (cv - 1)) == 0 &&
         256 % cv == 0 && nvec < (1L << 31) - 256L * 8;
}

static int flat_grid(long nvec) { return (int)((nvec + 256L * 4 - 1) / (256L * 4)); }

static int stream_grid(long nvec) {
  long b = (nvec + 255) / 256;
  if (b > 256L * 16) b = 256L * 16;  // grid-stride beyond 16 blocks per CU
  if (b < 1) b = 1;
  return (int)b;
}

static long choose_slabs(long rows, int rpi, int nchunk) {
  // ~2 blocks of 512 threads per CU in total, at most 256 slabs (so the
  // finalize pass stays short) and >= 8 row-iterations per thread.
  long target = 512 / nchunk;
  if (target < 1) target = 1;
  long max_by_work = rows / ((long)rpi * 8);
  if (max_by_work < 1) max_by_work = 1;
  long s = target < max_by_work ? target : max_by_work;
  if (s > 256) s = 256;
  return s;
}

template <typename T, int V, int M, bool R>
static void launch_bwd_apply(int gb, hipStream_t stream, const void* dy, const void* y,
                             const void* x, void* dx, void* dres, long nvec, int C,
                             const float* A, const float* B, const float* Cc) {
  if (flat_ok(nvec, C, V))
    hipLaunchKernelGGL((bn_bwd_apply_k<T, V, M, R, 4>), dim3(flat_grid(nvec)), dim3(256), 0,
                       stream, (const T*)dy, (const T*)y, (const T*)x, (T*)dx, (T*)dres, nvec, C,
                       A, B, Cc);
  else
    hipLaunchKernelGGL((bn_bwd_apply_k<T, V, M, R>), dim3(gb), dim3(256), 0, stream,
                       (const T*)dy, (const T*)y, (const T*)x, (T*)dx, (T*)dres, nvec, C, A, B,
                       Cc);
}

// kfb_bn_set_fold_bwd (tests): the backward apply passes fold their
// conv-epilogue partials (bn_bwd_apply_fold_k) instead of a finalize launch -
// 1 (default): tensors up to 64 MB, 2: every size, 0: never.  On the large tensors the slice layout streams slower
// than the grid-stride / flat passes (every size: ResNet-50 bs256 +0.1
// ms/step; up to 16 or 32 MB: -0.09 ms, profiles/r12_bn_fold_bwd.txt); on
// the small ones the launch it removes waits for a dispatch slot beside the
// weight-gradient stream (ResNet-152 bs32 2,515 -> 2,581-2,606 img/s).
static int g_fold_bwd = 1;

static bool fold_bwd_ok(int V, int nslab, int C, long rows) {
  // up to 64 MB, where the flat passes take over (32 MB: +0.04 ms/step on
  // interleaved runs, profiles/r13_bn_launch_ab.txt; 16 / 32 / 64 / 128 MB
  // measured alike with the flat passes from 256 MB)
  constexpr long max_bytes = 64L << 20;
  return g_fold_bwd && V == 8 && nslab == FS_SLOTS && C % FS_C == 0 && rows > 0 &&
         (g_fold_bwd == 2 || rows * C * 2 <= max_bytes);
}

// kfb_bn_set_fold_r(0) (tests): the dual backward's second BN keeps its
// finalize launch even when its partials could be folded
static int g_fold_r = 1;
static bool fold_r_on() { return g_fold_r != 0; }

static int fold_bwd_grid(long rows, int C) {
  constexpr long target = 1024;  // workgroups (256-thread blocks measured slower)
  const int ns = C / FS_C;
  long nrb = target / ns;
  const long need = (rows + 63) / 64;  // two 32-row groups per iteration
  if (nrb > need) nrb = need;
  if (nrb < 1) nrb = 1;
  return (int)(nrb * ns);
}

template <typename T, int V, bool RES, int RELU>
static void launch_apply(hipStream_t stream, const void* x, const void* res, void* y, long nvec,
                         int C, const float* scale, const float* shift, uint8_t* mb = nullptr) {
  if (flat_ok(nvec, C, V))
    hipLaunchKernelGGL((bn_apply_k<T, V, RES, RELU, 4>), dim3(flat_grid(nvec)), dim3(256), 0,
                       stream, (const T*)x, (const T*)res, (T*)y, nvec, C, scale, shift, mb);
  else
    hipLaunchKernelGGL((bn_apply_k<T, V, RES, RELU>), dim3(stream_grid(nvec)), dim3(256), 0,
                       stream, (const T*)x, (const T*)res, (T*)y, nvec, C, scale, shift, mb);
}

}  // namespace kfb

using namespace kfb;

// Number of slab partial rows the caller must allocate (per output array).
namespace kfb {
hipError_t bn_finalize_stats_launch(const float* psum, const float* psq, int nslab, int C,
                                    long rows, const float* gamma, const float* beta, float decay,
                                    float eps, float* run_mean, float* run_var, float* save_mean,
                                    float* save_invstd, float* scale, float* shift, float* kshift,
                                    hipStream_t stream) {
  hipLaunchKernelGGL(bn_finalize_stats_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, psum,
                     psq, nslab, C, rows, gamma, beta, decay, eps, run_mean, run_var, save_mean,
                     save_invstd, scale, shift, kshift);
  return hipGetLastError();
}

hipError_t bn_finalize_grad_launch(const float* slots, int C, long rows, const float* gamma,
                                   const float* mean, const float* invstd, float* dgamma,
                                   float* dbeta, float* coefA, float* coefB, float* coefC,
                                   int accumulate, hipStream_t stream) {
  constexpr int NSLOT = 32;  // IG_SPREAD
  hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, slots,
                     slots + (long)NSLOT * C, NSLOT, C, rows, gamma, mean, invstd, dgamma, dbeta,
                     coefA, coefB, coefC, accumulate, 0);
  return hipGetLastError();
}
}  // namespace kfb


// test / A/B hook: 1 folds the dual backward's second-BN finalize into the
// apply pass when its partials allow it
KFB_API void kfb_bn_set_fold_r(int on) { kfb::g_fold_r = on ? 1 : 0; }
KFB_API int kfb_bn_get_fold_r() { return kfb::fold_r_on() ? 1 : 0; }

// test / A/B hook: 1 folds the backward gradient finalize into the apply pass
KFB_API void kfb_bn_set_fold_bwd(int mode) { g_fold_bwd = mode; }
KFB_API int kfb_bn_get_fold_bwd() {
  fold_bwd_ok(0, 0, 0, 0);  // (resolves the environment default)
  return g_fold_bwd;
}

KFB_API int kfb_bn_num_slabs(long rows, int C) {
  const int V = vec_width(C);
  int n = 0;
  KFB_DISPATCH_VEC(V, VV, { Geo g = make_geo<VV>(C); n = (int)choose_slabs(rows, g.rpi, g.nchunk); });
  return n;
}

// Forward, training mode. psum/psq: [nslab, C] fp32 scratch.
KFB_API hipError_t kfb_bn_fwd_train(int dtype, const void* x, const void* res, void* y, long rows,
                                    int C, const float* gamma, const float* beta, float decay,
                                    float eps, float* run_mean, float* run_var, float* save_mean,
                                    float* save_invstd, float* scale, float* shift, float* psum,
                                    float* psq, int nslab, int relu, int have_partials,
                                    float* kshift, uint8_t* mbits, hipStream_t stream) {
  // mbits (nullable, 2-byte dtypes with relu): also write y's ReLU bit mask
  // [rows * C / 8] (see relu_bits)
  const int V = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      Geo g = make_geo<VV>(C);
      const long slab_rows = (rows + nslab - 1) / nslab;
      dim3 grid(nslab, g.nchunk);
      const size_t lds = 2 * (size_t)g.rpi * g.tpr * VV * sizeof(float);
      if (!have_partials)  // else the producing conv's epilogue already summed y, y^2
        hipLaunchKernelGGL((bn_partial_stats_k<T, VV>), grid, dim3(BN_THREADS), lds, stream,
                           (const T*)x, rows, C, g.cw, g.tpr, g.rpi, slab_rows, psum, psq,
                           kshift);
      if (have_partials != 2)  // 2: the producing conv's last workgroup finalized (BnFin)
        hipLaunchKernelGGL(bn_finalize_stats_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream,
                           psum, psq, nslab, C, rows, gamma, beta, decay, eps, run_mean, run_var,
                           save_mean, save_invstd, scale, shift, kshift);
      const long nvec = rows * C / VV;
      if (res) {
        if (relu) launch_apply<T, VV, true, 1>(stream, x, res, y, nvec, C, scale, shift, mbits);
        else launch_apply<T, VV, true, 0>(stream, x, res, y, nvec, C, scale, shift);
      } else {
        if (relu == 2) launch_apply<T, VV, false, 2>(stream, x, nullptr, y, nvec, C, scale, shift, mbits);
        else if (relu) launch_apply<T, VV, false, 1>(stream, x, nullptr, y, nvec, C, scale, shift, mbits);
        else launch_apply<T, VV, false, 0>(stream, x, nullptr, y, nvec, C, scale, shift);
      }
    });
  });
  return hipGetLastError();
}

// Forward, training mode, of y = relu?(bn(x) + bn_r(xr)) where both inputs'
// partial sums [nslab][C] were accumulated by the producing convs' epilogues:
// both finalizes (running statistics, scale/shift) and ONE apply pass.
KFB_API hipError_t kfb_bn_fwd_train_dual(
    int dtype, const void* x, const void* xr, void* y, long rows, int C, const float* gamma,
    const float* beta, float decay, float eps, float* run_mean, float* run_var, float* save_mean,
    float* save_invstd, float* scale, float* shift, const float* psum, const float* psq,
    int nslab, const float* gamma_r, const float* beta_r, float decay_r, float eps_r,
    float* run_mean_r, float* run_var_r, float* save_mean_r, float* save_invstd_r,
    float* scale_r, float* shift_r, const float* psum_r, const float* psq_r, int nslab_r,
    int relu, float* kshift, float* kshift_r, uint8_t* mbits, hipStream_t stream) {
  const int V = vec_width(C);
  hipLaunchKernelGGL(bn_finalize_stats_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, psum_r,
                     psq_r, nslab_r, C, rows, gamma_r, beta_r, decay_r, eps_r, run_mean_r,
                     run_var_r, save_mean_r, save_invstd_r, scale_r, shift_r, kshift_r);
  hipLaunchKernelGGL(bn_finalize_stats_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, psum,
                     psq, nslab, C, rows, gamma, beta, decay, eps, run_mean, run_var, save_mean,
                     save_invstd, scale, shift, kshift);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = rows * C / VV;
      const bool flat = flat_ok(nvec, C, VV);
      const int gb = flat ? flat_grid(nvec) : stream_grid(nvec);
      if (relu) {
        if (flat)
          hipLaunchKernelGGL((bn_apply2_k<T, VV, true, 4>), dim3(gb), dim3(256), 0, stream,
                             (const T*)x, (const T*)xr, (T*)y, nvec, C, scale, shift, scale_r,
                             shift_r, mbits);
        else
          hipLaunchKernelGGL((bn_apply2_k<T, VV, true>), dim3(gb), dim3(256), 0, stream,
                             (const T*)x, (const T*)xr, (T*)y, nvec, C, scale, shift, scale_r,
                             shift_r, mbits);
      } else {
        if (flat)
          hipLaunchKernelGGL((bn_apply2_k<T, VV, false, 4>), dim3(gb), dim3(256), 0, stream,
                             (const T*)x, (const T*)xr, (T*)y, nvec, C, scale, shift, scale_r,
                             shift_r, (uint8_t*)nullptr);
        else
          hipLaunchKernelGGL((bn_apply2_k<T, VV, false>), dim3(gb), dim3(256), 0, stream,
                             (const T*)x, (const T*)xr, (T*)y, nvec, C, scale, shift, scale_r,
                             shift_r, (uint8_t*)nullptr);
      }
    });
  });
  return hipGetLastError();
}

// Forward, inference mode (moving statistics).
KFB_API hipError_t kfb_bn_fwd_infer(int dtype, const void* x, const void* res, void* y, long rows,
                                    int C, const float* gamma, const float* beta,
                                    const float* run_mean, const float* run_var, float eps,
                                    float* scale, float* shift, int relu, hipStream_t stream) {
  const int V = vec_width(C);
  hipLaunchKernelGGL(bn_infer_coefs_k, dim3(ceil_div(C, 256)), dim3(256), 0, stream, C, gamma,
                     beta, run_mean, run_var, eps, scale, shift);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      const long nvec = rows * C / VV;
      if (res) {
        if (relu) launch_apply<T, VV, true, 1>(stream, x, res, y, nvec, C, scale, shift);
        else launch_apply<T, VV, true, 0>(stream, x, res, y, nvec, C, scale, shift);
      } else {
        if (relu == 2) launch_apply<T, VV, false, 2>(stream, x, nullptr, y, nvec, C, scale, shift);
        else if (relu) launch_apply<T, VV, false, 1>(stream, x, nullptr, y, nvec, C, scale, shift);
        else launch_apply<T, VV, false, 0>(stream, x, nullptr, y, nvec, C, scale, shift);
      }
    });
  });
  return hipGetLastError();
}

// Backward. y (forward output) supplies the ReLU mask when relu != 0
// (relu 2: ReLU6, no residual).
// dres (may be null) receives the gradient of the residual input.
// dgamma/dbeta are written (accumulate=0) or added to (accumulate=1).
KFB_API hipError_t kfb_bn_bwd(int dtype, const void* dy, const void* y, const void* x, void* dx,
                              void* dres, long rows, int C, const float* gamma,
                              const float* save_mean, const float* save_invstd, float* dgamma,
                              float* dbeta, float* pdy, float* pdyx, int nslab, float* coefA,
                              float* coefB, float* coefC, int relu, int accumulate,
                              int have_partials, hipStream_t stream) {
  const int V = vec_width(C);
  // have_partials: dy arrives already ReLU-masked and its partial sums were
  // produced by the consuming conv's dgrad epilogue.
  if (have_partials) relu = 0;
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      Geo g = make_geo<VV>(C);
      const long slab_rows = (rows + nslab - 1) / nslab;
      dim3 grid(nslab, g.nchunk);
      const size_t lds = 2 * (size_t)g.rpi * g.tpr * VV * sizeof(float);
      if (have_partials) {
      } else if (relu == 2)
        hipLaunchKernelGGL((bn_partial_grad_k<T, VV, 2>), grid, dim3(BN_THREADS), lds, stream,
                           (const T*)dy, (const T*)y, (const T*)x, save_mean, rows, C, g.cw,
                           g.tpr, g.rpi, slab_rows, pdy, pdyx);
      else if (relu)
        hipLaunchKernelGGL((bn_partial_grad_k<T, VV, 1>), grid, dim3(BN_THREADS), lds, stream,
                           (const T*)dy, (const T*)y, (const T*)x, save_mean, rows, C, g.cw,
                           g.tpr, g.rpi, slab_rows, pdy, pdyx);
      else
        hipLaunchKernelGGL((bn_partial_grad_k<T, VV, 0>), grid, dim3(BN_THREADS), lds,
                           stream, (const T*)dy, (const T*)y, (const T*)x, save_mean, rows, C,
                           g.cw, g.tpr, g.rpi, slab_rows, pdy, pdyx);
      const long nvec = rows * C / VV;
      if (have_partials == 1 && fold_bwd_ok(VV, nslab, C, rows)) {
        const BnFoldArgs f{pdy, pdyx, gamma, save_mean, save_invstd, dgamma, dbeta,
                           coefA, coefB, coefC, accumulate};
        const dim3 gf(fold_bwd_grid(rows, C));
        if (dres)
          hipLaunchKernelGGL((bn_bwd_apply_fold_k<T, true, false>), gf, dim3(256), 0, stream,
                             (const T*)dy, (const T*)x, (const T*)nullptr, (T*)dx, (T*)dres, rows,
                             C, f, (const float*)nullptr, (const float*)nullptr,
                             (const float*)nullptr, BnFoldArgs{});
        else
          hipLaunchKernelGGL((bn_bwd_apply_fold_k<T, false, false>), gf, dim3(256), 0, stream,
                             (const T*)dy, (const T*)x, (const T*)nullptr, (T*)dx, (T*)nullptr,
                             rows, C, f, (const float*)nullptr, (const float*)nullptr,
                             (const float*)nullptr, BnFoldArgs{});
        return hipGetLastError();
      }
      if (have_partials != 2)  // 2: the producing dgrad's last workgroup finalized (BnGFin)
        hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream,
                           pdy, pdyx, nslab, C, rows, gamma, save_mean, save_invstd, dgamma, dbeta,
                           coefA, coefB, coefC, accumulate, 0);
      const int gb = stream_grid(nvec);
      if (relu == 2) {  // (ReLU6: never with a residual add)
        launch_bwd_apply<T, VV, 2, false>(gb, stream, dy, y, x, dx, dres, nvec, C, coefA, coefB, coefC);
      } else if (relu) {
        if (dres) launch_bwd_apply<T, VV, 1, true>(gb, stream, dy, y, x, dx, dres, nvec, C, coefA, coefB, coefC);
        else launch_bwd_apply<T, VV, 1, false>(gb, stream, dy, y, x, dx, dres, nvec, C, coefA, coefB, coefC);
      } else {
        if (dres) launch_bwd_apply<T, VV, 0, true>(gb, stream, dy, y, x, dx, dres, nvec, C, coefA, coefB, coefC);
        else launch_bwd_apply<T, VV, 0, false>(gb, stream, dy, y, x, dx, dres, nvec, C, coefA, coefB, coefC);
      }
    });
  });
  return hipGetLastError();
}

// Backward of y = relu(bn(x) + bn_r(xr)) (kfb_bn_fwd_train_dual) when dy
// arrives ReLU-masked with bn's partial sums [nslab][C] already produced by
// the consuming conv's dgrad epilogue: bn_r's partials (one pass over dy, xr,
// unless `partials_r_ready`: the dgrad epilogue summed them too,
// kfb_conv_s1_dgrad_dual, into pdy_r / pdyx_r), both finalizes, and ONE apply
// pass writing dx and dxr.
KFB_API hipError_t kfb_bn_bwd_dual(
    int dtype, const void* dy, const void* x, const void* xr, void* dx, void* dxr, long rows,
    int C, const float* gamma, const float* save_mean, const float* save_invstd, float* dgamma,
    float* dbeta, const float* pdy, const float* pdyx, int nslab, float* coefA, float* coefB,
    float* coefC, int accumulate, const float* gamma_r, const float* save_mean_r,
    const float* save_invstd_r, float* dgamma_r, float* dbeta_r, float* pdy_r, float* pdyx_r,
    int nslab_r, float* coefA_r, float* coefB_r, float* coefC_r, int accumulate_r,
    int partials_r_ready, hipStream_t stream) {
  const int V = vec_width(C);
  KFB_DISPATCH_DTYPE(dtype, T, {
    KFB_DISPATCH_VEC(V, VV, {
      if (!partials_r_ready) {
        Geo g = make_geo<VV>(C);
        const long slab_rows = (rows + nslab_r - 1) / nslab_r;
        const size_t lds = 2 * (size_t)g.rpi * g.tpr * VV * sizeof(float);
        hipLaunchKernelGGL((bn_partial_grad_k<T, VV, false>), dim3(nslab_r, g.nchunk),
                           dim3(BN_THREADS), lds, stream, (const T*)dy, (const T*)nullptr,
                           (const T*)xr, save_mean_r, rows, C, g.cw, g.tpr, g.rpi, slab_rows,
                           pdy_r, pdyx_r);
      }
      const bool fold = fold_bwd_ok(VV, nslab, C, rows);
      if (!fold)
        hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream,
                           pdy, pdyx, nslab, C, rows, gamma, save_mean, save_invstd, dgamma, dbeta,
                           coefA, coefB, coefC, accumulate, 0);
      // both finalizes folded into the apply when the second BN's partials
      // came from the dgrad epilogue in the first BN's slot layout
      const bool fold_r = fold && partials_r_ready && nslab_r == FS_SLOTS && pdy_r == pdy &&
                          fold_r_on();
      if (!fold_r)
        hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream,
                           pdy_r, pdyx_r, nslab_r, C, rows, gamma_r, save_mean_r, save_invstd_r,
                           dgamma_r, dbeta_r, coefA_r, coefB_r, coefC_r, accumulate_r, 0);
      if (fold) {
        const BnFoldArgs f{pdy, pdyx, gamma, save_mean, save_invstd, dgamma, dbeta,
                           coefA, coefB, coefC, accumulate};
        if (fold_r) {
          const BnFoldArgs fr{pdy_r, pdyx_r, gamma_r, save_mean_r, save_invstd_r, dgamma_r,
                              dbeta_r, coefA_r, coefB_r, coefC_r, accumulate_r};
          hipLaunchKernelGGL((bn_bwd_apply_fold_k<T, true, true, true>),
                             dim3(fold_bwd_grid(rows, C)), dim3(256), 0, stream, (const T*)dy,
                             (const T*)x, (const T*)xr, (T*)dx, (T*)dxr, rows, C, f,
                             (const float*)nullptr, (const float*)nullptr,
                             (const float*)nullptr, fr);
        } else {
          hipLaunchKernelGGL((bn_bwd_apply_fold_k<T, true, true>), dim3(fold_bwd_grid(rows, C)),
                             dim3(256), 0, stream, (const T*)dy, (const T*)x, (const T*)xr,
                             (T*)dx, (T*)dxr, rows, C, f, coefA_r, coefB_r, coefC_r,
                             BnFoldArgs{});
        }
        return hipGetLastError();
      }
      const long nvec = rows * C / VV;
      if (flat_ok(nvec, C, VV))
        hipLaunchKernelGGL((bn_bwd_apply2_k<T, VV, 4>), dim3(flat_grid(nvec)), dim3(256), 0,
                           stream, (const T*)dy, (const T*)x, (const T*)xr, (T*)dx, (T*)dxr, nvec,
                           C, coefA, coefB, coefC, coefA_r, coefB_r, coefC_r);
      else
        hipLaunchKernelGGL((bn_bwd_apply2_k<T, VV>), dim3(stream_grid(nvec)), dim3(256), 0,
                           stream, (const T*)dy, (const T*)x, (const T*)xr, (T*)dx, (T*)dxr, nvec,
                           C, coefA, coefB, coefC, coefA_r, coefB_r, coefC_r);
    });
  });
  return hipGetLastError();
}

// Fused stem tail, forward (training): BN statistics come from the producing
// conv's epilogue (psum/psq [nslab][C]); z = maxpool(relu(bn(x))) and the
// per-element argmax bytes idx.  V = 8 (C % 8 == 0) only.
KFB_API hipError_t kfb_bn_relu_maxpool_fwd(int dtype, const void* x, void* z, uint8_t* idx, int N,
                                           int H, int W, int C, int OH, int OW, int kh, int kw,
                                           int sh, int sw, int pt, int pl, const float* gamma,
                                           const float* beta, float decay, float eps,
                                           float* run_mean, float* run_var, float* save_mean,
                                           float* save_invstd, float* scale, float* shift,
                                           float* psum, float* psq, int nslab, float* kshift,
                                           hipStream_t stream) {
  if (C % 8 || kh * kw > 255 || (long)N * H * W * C >= (1L << 31)) return hipErrorInvalidValue;
  const BPGeo g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};
  const long rows = (long)N * H * W;
  hipLaunchKernelGGL(bn_finalize_stats_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, psum, psq,
                     nslab, C, rows, gamma, beta, decay, eps, run_mean, run_var, save_mean,
                     save_invstd, scale, shift, kshift);
  const long total = (long)N * OH * OW * (C / 8);
  KFB_DISPATCH_DTYPE(dtype, T, {
    if (kh == 3 && kw == 3)
      hipLaunchKernelGGL((bn_relu_maxpool_fwd_k<T, 8, true>), dim3(stream_grid(total)), dim3(256),
                         0, stream, (const T*)x, (T*)z, idx, scale, shift, g);
    else
      hipLaunchKernelGGL((bn_relu_maxpool_fwd_k<T, 8>), dim3(stream_grid(total)), dim3(256), 0,
                         stream, (const T*)x, (T*)z, idx, scale, shift, g);
  });
  return hipGetLastError();
}

// Fused stem tail, backward: dx (gradient of the BN input) from the pooled
// gradient dz; dgamma/dbeta written (accumulate=0) or added (accumulate=1).
// pdy/pdyx: [kfb_bn_num_slabs(N*H*W, C)][C] scratch; coef*: [C] scratch.
KFB_API hipError_t kfb_bn_relu_maxpool_bwd(int dtype, const void* dz, const void* z,
                                           const uint8_t* idx, const void* x, void* dx, int N,
                                           int H, int W, int C, int OH, int OW, int kh, int kw,
                                           int sh, int sw, int pt, int pl, const float* gamma,
                                           const float* save_mean, const float* save_invstd,
                                           float* dgamma, float* dbeta, float* pdy, float* pdyx,
                                           int nslab, float* coefA, float* coefB, float* coefC,
                                           int accumulate, int have_partials, hipStream_t stream) {
  // have_partials: pdy / pdyx already hold [nslab][C] slot sums of dz' and
  // dz' (z - beta) over the pooled output z (accumulated by the dgrad epilogue
  // of the convs that consume z, with z's ReLU mask): each window routes its
  // gradient to one BN-output pixel p, whose x_p - mean = (z - beta) /
  // (gamma * invstd), so the partial pass over x is skipped
  if (C % 8 || (long)N * H * W * C >= (1L << 31)) return hipErrorInvalidValue;
  const BPGeo g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};
  const long rows = (long)N * H * W;
  const int cv = C / 8;
  if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && 256 % cv == 0) {
    // 3x3/2 block kernels: nslab blocks for the partial pass (the caller
    // sizes the slabs with kfb_bn_pool_num_slabs)
    const int OHo = (H + pt + 1) / 2, OWo = (W + pl + 1) / 2;
    const long total = (long)N * OHo * OWo * cv;
    if (total >= (1L << 31)) return hipErrorInvalidValue;
    KFB_DISPATCH_DTYPE(dtype, T, {
      if (!have_partials)
        hipLaunchKernelGGL((bn_pool3s2_k<T, 0>), dim3(nslab), dim3(256), 0, stream, (const T*)dz,
                           (const T*)z, idx, (const T*)x, (T*)dx, g, OHo, OWo, save_mean, pdy, pdyx,
                           nullptr, nullptr, nullptr);
      hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, pdy,
                         pdyx, nslab, C, rows, gamma, save_mean, save_invstd, dgamma, dbeta, coefA,
                         coefB, coefC, accumulate, have_partials);
      hipLaunchKernelGGL((bn_pool3s2_k<T, 1>), dim3(stream_grid(total)), dim3(256), 0, stream,
                         (const T*)dz, (const T*)z, idx, (const T*)x, (T*)dx, g, OHo, OWo, nullptr,
                         nullptr, nullptr, coefA, coefB, coefC);
    });
    return hipGetLastError();
  }
  KFB_DISPATCH_DTYPE(dtype, T, {
    Geo gg = make_geo<8>(C);
    const long slab_rows = (rows + nslab - 1) / nslab;
    const size_t lds = 2 * (size_t)gg.rpi * gg.tpr * 8 * sizeof(float);
    if (!have_partials)
      hipLaunchKernelGGL((bn_pool_partial_grad_k<T, 8>), dim3(nslab, gg.nchunk), dim3(BN_THREADS),
                         lds, stream, (const T*)dz, (const T*)z, idx, (const T*)x, save_mean, g,
                         rows, gg.cw, gg.tpr, gg.rpi, slab_rows, pdy, pdyx);
    hipLaunchKernelGGL(bn_finalize_grad_k, dim3(ceil_div(C, 64)), dim3(64, FOLD_Y), 0, stream, pdy,
                       pdyx, nslab, C, rows, gamma, save_mean, save_invstd, dgamma, dbeta, coefA,
                       coefB, coefC, accumulate, have_partials);
    hipLaunchKernelGGL((bn_pool_bwd_apply_k<T, 8>), dim3(stream_grid(rows * C / 8)), dim3(256), 0,
                       stream, (const T*)dz, (const T*)z, idx, (const T*)x, (T*)dx, g, coefA,
                       coefB, coefC);
  });
  return hipGetLastError();
}

// Slab count kfb_bn_relu_maxpool_bwd uses (pdy/pdyx need nslab * C floats).
KFB_API int kfb_bn_pool_num_slabs(int N, int H, int W, int C, int kh, int kw, int sh, int sw) {
  if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && C % 8 == 0 && 256 % (C / 8) == 0)
    return 2048;  // 8 blocks per CU of the latency-bound gather pass
  return kfb_bn_num_slabs((long)N * H * W, C);
}
