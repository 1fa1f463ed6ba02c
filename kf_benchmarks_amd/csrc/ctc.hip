// CTC loss and its gradient on gfx950 (DeepSpeech2's loss:
// tcb/models/experimental/deepspeech.py:360-395, tf.nn.ctc_loss with
// ignore_longer_outputs_than_inputs -> infeasible sequences give loss 0).
//
// Blank = class C-1 (the reference's 28 of 29).  Per sequence b, with the
// blank-extended label l' of length S = 2L+1:
//   alpha_t(s) = lse(alpha_{t-1}(s), alpha_{t-1}(s-1), [alpha_{t-1}(s-2)]) + lp_t(l'_s)
//   beta_t(s)  = lse(beta_{t+1}(s), beta_{t+1}(s+1), [beta_{t+1}(s+2)]) + lp_t(l'_s)
//   loss_b = -lse(alpha_{T-1}(S-1), alpha_{T-1}(S-2))
//   dloss_b/dz_t(c) = softmax_t(c) - sum_{s: l'_s = c} exp(alpha_t(s) + beta_t(s) - lp_t(c) + loss_b)
// with lp = log_softmax(z) over the classes.  One 256-thread workgroup per
// sequence runs both recursions with the state vector double-buffered in LDS
// (one barrier per time step); alpha goes to a [B][T][S] fp32 workspace and
// the beta pass folds the per-class posteriors through LDS float atomics,
// writing the finished gradient row of step t right away.  The gradient is
// computed in the forward (as TF's CTC op does); the backward only scales it.
#include "common.h"

namespace kfb {
namespace ctc {

constexpr int NT = 256;
constexpr int MAXS = 4095;  // 2 * max label length + 1
constexpr int MAXC = 256;
constexpr float NEG = -INFINITY;

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG) return NEG;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

struct Args {
  const void* z;  // logits, element (t, b, c) at t*ldt + b*ldb + c
  long ldt, ldb;
  const int* labels;  // [B][Lmax]
  const int* ilen;    // [B] (already scaled to the logits' time axis)
  const int* llen;    // [B]
  int T, B, C, Lmax;
  float* lp;     // [T][B][C] log_softmax workspace
  float* alpha;  // [B][T][S_max]
  int smax;
  float* loss;   // [B]
  float* grad;   // element (t, b, c) at t*ldt + b*ldb + c (fp32, same strides as z)
};

// lp[row][c] = z - lse(z) for every (t, b) row: one wave per row.
template <typename T>
__global__ void __launch_bounds__(256) log_softmax_k(Args a) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long row = blockIdx.x * 4L + wid;
  if (row >= (long)a.T * a.B) return;
  const int t = (int)(row / a.B), b = (int)(row % a.B);
  const T* z = (const T*)a.z + t * a.ldt + b * a.ldb;
  float m = NEG;
  for (int c = lane; c < a.C; c += 64) m = fmaxf(m, (float)z[c]);
  m = wave_max(m);
  float sum = 0.f;
  for (int c = lane; c < a.C; c += 64) sum += __expf((float)z[c] - m);
  sum = wave_sum(sum);
  const float l = m + __logf(sum);
  for (int c = lane; c < a.C; c += 64) a.lp[row * a.C + c] = (float)z[c] - l;
}

__global__ void __launch_bounds__(NT) ctc_k(Args a) {
  __shared__ int ext[MAXS + 1];
  __shared__ float buf[2][MAXS + 1];
  __shared__ float post[MAXC];
  __shared__ float red[NT / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int C = a.C, blank = C - 1;
  int L = a.llen[b];
  L = L < 0 ? 0 : (L > a.Lmax ? a.Lmax : L);
  int Tb = a.ilen[b];
  Tb = Tb > a.T ? a.T : Tb;
  const int S = 2 * L + 1;
  for (int s = tid; s < S; s += NT) {
    int c = (s & 1) ? a.labels[(long)b * a.Lmax + (s >> 1)] : blank;
    ext[s] = (c < 0 || c >= C) ? blank : c;
  }
  __syncthreads();
  const float* lp = a.lp;
  auto lpt = [&](int t, int c) { return lp[((long)t * a.B + b) * C + c]; };
  float* al = a.alpha + (long)b * a.T * a.smax;
  float logp = NEG;
  if (Tb > 0) {
    // ---- alpha
    for (int s = tid; s < S; s += NT) {
      const float v = s == 0 ? lpt(0, blank) : (s == 1 ? lpt(0, ext[1]) : NEG);
      buf[0][s] = v;
      al[s] = v;
    }
    __syncthreads();
    int cur = 0;
    for (int t = 1; t < Tb; ++t) {
      const float* pv = buf[cur];
      float* nv = buf[cur ^ 1];
      for (int s = tid; s < S; s += NT) {
        float v = pv[s];
        if (s >= 1) v = lse2(v, pv[s - 1]);
        if (s >= 2 && ext[s] != blank && ext[s] != ext[s - 2]) v = lse2(v, pv[s - 2]);
        v = v == NEG ? NEG : v + lpt(t, ext[s]);
        nv[s] = v;
        al[(long)t * a.smax + s] = v;
      }
      cur ^= 1;
      __syncthreads();
    }
    logp = S > 1 ? lse2(buf[cur][S - 1], buf[cur][S - 2]) : buf[cur][S - 1];
  }
  const bool feasible = logp != NEG;
  if (tid == 0) a.loss[b] = feasible ? -logp : 0.f;
  float* g = a.grad;
  // rows past the sequence end (and every row of an infeasible sequence) get zero gradient
  for (int t = feasible ? Tb : 0; t < a.T; ++t)
    for (int c = tid; c < C; c += NT) g[t * a.ldt + b * a.ldb + c] = 0.f;
  if (!feasible) return;
  // ---- beta, with the gradient row of each step
  __syncthreads();
  int cur = 0;
  for (int t = Tb - 1; t >= 0; --t) {
    for (int c = tid; c < C; c += NT) post[c] = 0.f;
    const float* pv = buf[cur];
    float* nv = buf[cur ^ 1];
    __syncthreads();  // post cleared; previous step's nv complete
    for (int s = tid; s < S; s += NT) {
      float v;
      const float l = lpt(t, ext[s]);
      if (t == Tb - 1) {
        v = s >= S - 2 ? l : NEG;
      } else {
        v = pv[s];
        if (s + 1 < S) v = lse2(v, pv[s + 1]);
        if (s + 2 < S && ext[s] != blank && ext[s + 2] != ext[s]) v = lse2(v, pv[s + 2]);
        v = v == NEG ? NEG : v + l;
      }
      nv[s] = v;
      const float av = al[(long)t * a.smax + s];
      if (av != NEG && v != NEG) atomicAdd(&post[ext[s]], __expf(av + v - l - logp));
    }
    __syncthreads();
    for (int c = tid; c < C; c += NT) g[t * a.ldt + b * a.ldb + c] = __expf(lpt(t, c)) - post[c];
    cur ^= 1;
  }
  (void)red;
}

// dz = grad * gloss[b] (gloss: the upstream gradient of each sequence's loss)
template <typename T>
// dz = grad * gloss[b * gstride] * mul (gstride 0: one scalar gradient for
// every sequence, e.g. the backward of the batch-mean loss)
__global__ void __launch_bounds__(256) scale_k(const float* __restrict__ grad,
                                               const float* __restrict__ gloss, T* __restrict__ dz,
                                               long ldt, long ldb, int T_, int B, int C,
                                               int gstride, float mul) {
  const long n = (long)T_ * B * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long r = e / C;
    const int b = (int)(r % B), t = (int)(r / B);
    const long off = t * ldt + b * ldb + c;
    dz[off] = (T)(grad[off] * (gloss[b * gstride] * mul));
  }
}

// Input lengths on the logits' time axis: out = in * num / den (integer
// division, as the reference's length scaling), on the device so a
// recorded step holds no host or torch arithmetic.
__global__ void scale_lengths_k(const int* __restrict__ in, int* __restrict__ out, int n, int num,
                                int den) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int)(((long long)in[i] * num) / den);
}

}  // namespace ctc
}  // namespace kfb

using namespace kfb;

KFB_API int kfb_ctc_max_states() { return ctc::MAXS; }

// Per-sequence CTC loss and its gradient w.r.t. the logits (see top).
// lp: [T*B*C] fp32 workspace; alpha: [B*T*smax] fp32 workspace (smax >= 2*Lmax+1).
KFB_API hipError_t kfb_ctc_loss(int dtype, const void* z, long ldt, long ldb, const int* labels,
                                const int* ilen, const int* llen, int T, int B, int C, int Lmax,
                                float* lp, float* alpha, int smax, float* loss, float* grad,
                                hipStream_t stream) {
  if (C < 2 || C > ctc::MAXC || 2 * Lmax + 1 > ctc::MAXS || smax < 2 * Lmax + 1 || T < 1 || B < 1)
    return hipErrorInvalidValue;
  ctc::Args a{z, ldt, ldb, labels, ilen, llen, T, B, C, Lmax, lp, alpha, smax, loss, grad};
  const unsigned rows = (unsigned)(((long)T * B + 3) / 4);
  KFB_DISPATCH_DTYPE(dtype, T_,
                     hipLaunchKernelGGL(ctc::log_softmax_k<T_>, dim3(rows), dim3(256), 0, stream,
                                        a));
  hipLaunchKernelGGL(ctc::ctc_k, dim3(B), dim3(ctc::NT), 0, stream, a);
  return hipGetLastError();
}

KFB_API hipError_t kfb_ctc_grad_scale(int dtype, const float* grad, const float* gloss, void* dz,
                                      long ldt, long ldb, int T, int B, int C,
                                      hipStream_t stream) {
  const long n = (long)T * B * C;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  KFB_DISPATCH_DTYPE(dtype, T_,
                     hipLaunchKernelGGL(ctc::scale_k<T_>, dim3((unsigned)blocks), dim3(256), 0,
                                        stream, grad, gloss, (T_*)dz, ldt, ldb, T, B, C, 1, 1.f));
  return hipGetLastError();
}

// Backward of mean_b(loss_b): dz = grad * g[0] * inv_count.
KFB_API hipError_t kfb_ctc_grad_scale_mean(int dtype, const float* grad, const float* g, void* dz,
                                           long ldt, long ldb, int T, int B, int C,
                                           float inv_count, hipStream_t stream) {
  const long n = (long)T * B * C;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  KFB_DISPATCH_DTYPE(dtype, T_,
                     hipLaunchKernelGGL(ctc::scale_k<T_>, dim3((unsigned)blocks), dim3(256), 0,
                                        stream, grad, g, (T_*)dz, ldt, ldb, T, B, C, 0,
                                        inv_count));
  return hipGetLastError();
}

KFB_API hipError_t kfb_ctc_scale_lengths(const int* in, int* out, int n, int num, int den,
                                         hipStream_t stream) {
  if (n <= 0 || den <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ctc::scale_lengths_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     in, out, n, num, den);
  return hipGetLastError();
}
