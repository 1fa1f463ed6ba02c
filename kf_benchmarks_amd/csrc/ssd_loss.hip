// SSD300 training loss (tcb/models/ssd_model.py:loss_function, the
// classification term with hard-negative mining and the smooth-L1
// localisation term).  Per image b, anchor a (A = 8732), C = 81 classes,
// logits row x[a] = [4 box deltas | C class logits]:
//
//   ce[a]   = logsumexp_c x[a][4+c] - x[a][4+label[a]]
//   pos[a]  = label[a] > 0,   k_b = min(negs_per_pos * floor(n_b), A)
//   neg[a]  = a is a negative among the k_b largest of ce*(1-pos)
//             (descending; equal values taken in anchor order)
//   loss_b  = (sum_a ce[a] (pos+neg)[a] + sum_pos smoothL1(x[a][:4] - gt[a])) / n_b
//   loss    = mean_b loss_b
//
// Three launches instead of the ~20 (two full argsorts) of the tensor form:
//   1. ssd_rows_k   - grid over all B*A rows: one online-softmax pass per row
//                     (16 lanes per row)
//                     gives lse[i] and v[i] = ce (+ smooth-L1 if positive);
//   2. ssd_select_k - one 1024-lane workgroup per image: the keys
//                     ce*(1-pos) sit in LDS (35 KB) and a 4-pass 8-bit radix
//                     select finds the k-th largest; writes the per-anchor
//                     weight w = pos+neg and the image loss;
//   3. ssd_mean_k   - mean over images.
// Backward (one pass over the elements, bf16/f32 logits in, same dtype out):
//   dx[a][4+c] = g/(B n_b) * w[a] * (softmax(x[a])[c] - [c == label[a]])
//   dx[a][j]   = g/(B n_b) * pos[a] * clamp(x[a][j] - gt[a][j], -1, 1)
// Labels arrive as the model's float32 input column and are truncated like
// the tensor form's .long().
#include "common.h"

namespace kfb {

constexpr int SSD_MAX_ANCHORS = 8960;  // LDS key rows (>= 8732)
constexpr int SSD_SEL_THREADS = 1024;

__device__ __forceinline__ float smooth_l1(float d) {
  const float a = fabsf(d);
  return a < 1.f ? 0.5f * d * d : a - 0.5f;
}

__device__ __forceinline__ int ssd_label(float l, int C, bool* pos) {
  int li = (int)l;
  *pos = li > 0;
  return li < 0 ? 0 : (li >= C ? C - 1 : li);
}

// 16 lanes per row (16 rows per 256-thread workgroup): each lane keeps an
// online (max, sum) over every 16th class logit, the pairs merge across the
// group by shuffles, so a wave reads 4 consecutive rows' bytes together
// (one thread per row strode the rows 4 + C elements apart: uncoalesced).
constexpr int SSD_G = 16;

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  if (mm == -INFINITY) return;  // both empty
  s = s * __expf(m - mm) + s2 * __expf(m2 - mm);
  m = mm;
}

template <typename T>
__global__ void __launch_bounds__(256)
ssd_rows_k(const T* __restrict__ x, const float* __restrict__ gt_loc,
           const float* __restrict__ label, long rows, int C, float* __restrict__ lse_out,
           float* __restrict__ v_out) {
  const int R = 4 + C;
  const int g = threadIdx.x & (SSD_G - 1);
  for (long i = (long)blockIdx.x * (256 / SSD_G) + threadIdx.x / SSD_G; i < rows;
       i += (long)gridDim.x * (256 / SSD_G)) {
    const T* row = x + i * R;
    float m = -INFINITY, sm = 0.f;
    for (int c = g; c < C; c += SSD_G) {
      const float v = (float)row[4 + c];
      if (v > m) {
        sm = sm * __expf(m - v) + 1.f;
        m = v;
      } else {
        sm += __expf(v - m);
      }
    }
    bool pos;
    const int l = ssd_label(label[i], C, &pos);
    float sl = 0.f;
    if (pos && g < 4) sl = smooth_l1((float)row[g] - gt_loc[i * 4 + g]);
#pragma unroll
    for (int o = SSD_G / 2; o > 0; o >>= 1) {
      lse_merge(m, sm, __shfl_xor(m, o, SSD_G), __shfl_xor(sm, o, SSD_G));
      sl += __shfl_xor(sl, o, SSD_G);
    }
    if (g == 0) {
      const float lse = m + __logf(sm);
      lse_out[i] = lse;
      v_out[i] = lse - (float)row[4 + l] + sl;
    }
  }
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < (int)(blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) red[0] = t;
  }
  __syncthreads();
  const float r = red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(SSD_SEL_THREADS)
ssd_select_k(const float* __restrict__ v_in, const float* __restrict__ label,
             const float* __restrict__ num_matched, int A, int C, int negs_per_pos,
             float* __restrict__ w_out, float* __restrict__ loss_img) {
  __shared__ unsigned key[SSD_MAX_ANCHORS];
  __shared__ unsigned hist[256];
  __shared__ unsigned wcnt[SSD_SEL_THREADS / 64];
  __shared__ float red[SSD_SEL_THREADS / 64];
  __shared__ unsigned sel[3];  // prefix, remaining count, running equal count
  const int b = blockIdx.x;
  const float* vb = v_in + (long)b * A;
  const float* lb = label + (long)b * A;
  const float nm = num_matched[b];
  float sum_pos = 0.f;
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    bool pos;
    ssd_label(lb[a], C, &pos);
    const float v = vb[a];
    if (pos) sum_pos += v;
    // ce >= 0 up to rounding: non-negative floats order like their bits
    key[a] = pos ? 0u : __float_as_uint(fmaxf(v, 0.f));
  }
  sum_pos = block_sum(sum_pos, red);  // (its barriers also publish key[])
  const long kk = (long)nm * negs_per_pos;
  const unsigned k = (unsigned)(kk < A ? (kk > 0 ? kk : 0) : A);
  if (threadIdx.x == 0) { sel[0] = 0u; sel[1] = k; sel[2] = 0u; }
  __syncthreads();
  if (k > 0) {
    for (int pass = 3; pass >= 0; --pass) {
      for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0u;
      __syncthreads();
      const unsigned prefix = sel[0];
      const unsigned hi = pass == 3 ? 0u : (0xFFFFFFFFu << (8 * (pass + 1)));
      for (int a = threadIdx.x; a < A; a += blockDim.x) {
        const unsigned v = key[a];
        if ((v & hi) == prefix) atomicAdd(&hist[(v >> (8 * pass)) & 255u], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned rem = sel[1];
        int d = 255;
        for (; d > 0; --d) {  // walk digits from the largest
          if (hist[d] >= rem) break;
          rem -= hist[d];
        }
        sel[0] = prefix | ((unsigned)d << (8 * pass));
        sel[1] = rem;
      }
      __syncthreads();
    }
  }
  // k-th largest key = thr; take every key > thr and the first take_eq keys
  // equal to thr in anchor order.
  const unsigned thr = sel[0], take_eq = k > 0 ? sel[1] : 0u;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float sum_neg = 0.f;
  for (int a0 = 0; a0 < A; a0 += blockDim.x) {
    const int a = a0 + threadIdx.x;
    const bool in = a < A;
    const unsigned v = in ? key[a] : 0u;
    const bool eq = in && k > 0 && v == thr;
    const unsigned long long ball = __ballot(eq);
    if (lane == 0) wcnt[wid] = (unsigned)__popcll(ball);
    __syncthreads();
    unsigned before = sel[2] + (unsigned)__popcll(ball & ((1ull << lane) - 1ull));
    for (int j = 0; j < wid; ++j) before += wcnt[j];
    if (in) {
      bool pos;
      ssd_label(lb[a], C, &pos);
      // Positives never count as hard negatives.  (They tie at key 0, so
      // they could only be reached when k exceeds the number of negatives
      // with a non-zero loss, where the tensor form's unstable argsort
      // picks an arbitrary subset.)
      const bool neg = !pos && k > 0 && (v > thr || (eq && before < take_eq));
      w_out[(long)b * A + a] = (pos || neg) ? 1.f : 0.f;
      if (neg) sum_neg += vb[a];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned t = 0;
      for (int j = 0; j < nw; ++j) t += wcnt[j];
      sel[2] += t;
    }
    __syncthreads();
  }
  sum_neg = block_sum(sum_neg, red);
  if (threadIdx.x == 0) loss_img[b] = (sum_pos + sum_neg) / nm;
}

__global__ void ssd_mean_k(const float* __restrict__ loss_img, int B, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < B; i += 64) s += loss_img[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[0] = s / (float)B;
}

// One thread per logit element (coalesced: consecutive lanes, consecutive
// elements); the per-anchor scalars come from L1.  I: the element index type
// - 32-bit (cheaper divisions) while B*A*(4+C) < 2^31, 64-bit beyond (large
// per-GPU batches, e.g. ~2,900+ images at 81 classes).
template <typename T, typename I>
__global__ void __launch_bounds__(256)
ssd_bwd_k(const T* __restrict__ x, const float* __restrict__ gt_loc,
          const float* __restrict__ label, const float* __restrict__ num_matched,
          const float* __restrict__ lse, const float* __restrict__ w, const float* __restrict__ g,
          int B, int A, int C, T* __restrict__ dx) {
  const I R = 4 + C;
  const I n = (I)B * (I)A * R;
  const float gs = g[0] / (float)B;
  for (I e = (I)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (I)gridDim.x * blockDim.x) {
    const I i = e / R;
    const int c = (int)(e - i * R);
    const float scale = gs / num_matched[i / (I)A];
    bool pos;
    const int l = ssd_label(label[i], C, &pos);
    const float xv = (float)x[e];
    float d;
    if (c >= 4)
      d = w[i] * scale * (__expf(xv - lse[i]) - (c - 4 == l ? 1.f : 0.f));
    else
      d = (pos ? scale : 0.f) * fminf(fmaxf(xv - gt_loc[i * 4 + c], -1.f), 1.f);
    dx[e] = (T)d;
  }
}

inline unsigned row_grid(long rows) {
  long b = (rows + 255) / 256;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace kfb

using namespace kfb;

// work: fp32 scratch of B + 3*B*A floats: loss_img[B] | lse[B*A] | v[B*A] | w[B*A].
KFB_API hipError_t kfb_ssd_loss_fwd(int dtype, const void* x, const float* gt_loc,
                                    const float* label, const float* num_matched, int B, int A,
                                    int C, int negs_per_pos, float* work, float* out,
                                    hipStream_t stream) {
  if (A > SSD_MAX_ANCHORS || A < 1 || B < 1 || C < 1) return hipErrorInvalidValue;
  const long rows = (long)B * A;
  float* loss_img = work;
  float* lse = work + B;
  float* v = lse + rows;
  float* w = v + rows;
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((ssd_rows_k<T>), dim3(row_grid(rows * SSD_G)), dim3(256), 0, stream,
                       (const T*)x, gt_loc, label, rows, C, lse, v);
  });
  hipLaunchKernelGGL(ssd_select_k, dim3(B), dim3(SSD_SEL_THREADS), 0, stream, v, label,
                     num_matched, A, C, negs_per_pos, w, loss_img);
  hipLaunchKernelGGL(ssd_mean_k, dim3(1), dim3(64), 0, stream, loss_img, B, out);
  return hipGetLastError();
}

// g: fp32 [1] upstream gradient of the scalar loss (device).
KFB_API hipError_t kfb_ssd_loss_bwd(int dtype, const void* x, const float* gt_loc,
                                    const float* label, const float* num_matched,
                                    const float* work, const float* g, int B, int A, int C,
                                    void* dx, hipStream_t stream) {
  if (A < 1 || B < 1 || C < 1) return hipErrorInvalidValue;
  const long rows = (long)B * A;
  const bool narrow = rows * (4 + C) < (1L << 31);
  const float* lse = work + B;
  const float* w = lse + 2 * rows;
  KFB_DISPATCH_DTYPE(dtype, T, {
    if (narrow)
      hipLaunchKernelGGL((ssd_bwd_k<T, unsigned>), dim3(row_grid(rows * (4 + C))), dim3(256), 0,
                         stream, (const T*)x, gt_loc, label, num_matched, lse, w, g, B, A, C,
                         (T*)dx);
    else
      hipLaunchKernelGGL((ssd_bwd_k<T, unsigned long long>), dim3(row_grid(rows * (4 + C))),
                         dim3(256), 0, stream, (const T*)x, gt_loc, label, num_matched, lse, w,
                         g, B, A, C, (T*)dx);
  });
  return hipGetLastError();
}
