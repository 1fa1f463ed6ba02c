// Recurrent layers of DeepSpeech2 on gfx950: TF BasicLSTMCell (gates i, j,
// f, o; forget bias 1.0) and the basic tanh RNN cell, one or two directions
// (tcb/models/experimental/deepspeech.py:121-125, :231-270).
//
// The layer is split the way its FLOPs split:
//   * the input projection x . Wx + b of every time step is ONE big GEMM
//     (ops/nn.linear, csrc/gemm.hip) producing gx [T][B][dirs*G*H];
//   * the recurrence runs one launch per time step (both directions in the
//     same launch, blockIdx.z = direction) of a 16-wave kernel that multiplies
//     the 16-unit x (16*NB)-row tile of h_{t-1} . Wh on MFMA (K split over the
//     waves, every load of a wave in flight at once) and applies the cell in
//     its epilogue (gates, c, h never round-trip through a separate
//     elementwise kernel);
//   * the backward step kernel does dh = dout + dG_{t+1} . Wh^T on MFMA with
//     the cell's backward in the epilogue, writing dG_t = d(gx) in place for
//     the input-projection backward; dWh = sum_t h_{t-1}^T dG_t is one GEMM
//     over all steps afterwards (ops/rnn.py).
// The host loops over time steps in C++ (kfb_rnn_fwd / kfb_rnn_bwd), so a
// layer costs one ctypes call, not T.
//
// Layouts (time-major; direction d processes time t = s or T-1-s at step s):
//   gx   [T][B][ldg]  (T)  columns d*G*H + g*H + u        (ldg = dirs*G*H)
//   whT  [dirs][G*H][H] (T)  forward operand (K = H contiguous)
//   wh   [dirs][H][G*H] (T)  backward operand (K = G*H contiguous; TF layout)
//   out  [T][B][dirs*H] (T)  h_t, directions concatenated
//   hp   [dirs][T][B][H] (T) h entering the step at time t (0 for the first)
//   act  [dirs][T][B][G*H] fp32  activated gates (LSTM) / h_t (RNN)
//   cell [dirs][T][B][H] fp32    c_t (LSTM)
//   dc   [2][dirs][B][H] fp32    cell gradient carried between backward steps
#include "common.h"

namespace kfb {
namespace rnn {

typedef __attribute__((ext_vector_type(4))) float v4f;
typedef __attribute__((ext_vector_type(8))) short v8s;

enum Kind : int { LSTM = 0, TANH = 1, GRU = 2 };

// Reduction tiling.  A workgroup of NW = 16 waves owns one 16-unit x
// (16*NB)-row output tile; its waves share the G gate blocks x NW/G K parts
// (wave w: gate w % G, part w / G), so each wave's slice of K is short
// enough (H = 800: 200 deep) that ALL its operand loads are issued before
// its first MFMA: one memory round trip per step instead of one per 4 K
// steps (the step kernels are latency-bound: a few MB of weights, 100-800
// workgroups).  Partial tiles meet in LDS red[w][u][b] and the epilogue
// thread of (b, u) sums its gate's parts.
constexpr int NW = 16;
constexpr int NT = NW * 64;
constexpr int RED_LD = 33;
constexpr int MAXIT = 8;  // MFMA steps whose loads are in flight together

// acc[nb][r] += sum_{k in [kb, ke)} A[i][k] * B[nb*16 + j][k] with
// i = 4*(lane/16) + r, j = lane % 16 (the 16x16 MFMA accumulator layout).
// A: 16 rows (lda), B: up to 16*NB rows (ldb), rows >= brows read as zero.
// Each lane loads one contiguous k-chunk per row per MFMA step: the k order
// inside a step is a permutation, identical for A and B, so the sum is the
// plain dot product.  kb, ke multiples of 8 (16-bit) / 4 (fp32).
template <typename T, int NB>
__device__ __forceinline__ void dot_rows(const T* __restrict__ A, long lda,
                                         const T* __restrict__ Bm, long ldb, int brows, int kb,
                                         int ke, v4f (&acc)[NB]) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const T* pa = A + r16 * lda;
  const T* pb[NB];
  bool bok[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    bok[nb] = nb * 16 + r16 < brows;
    pb[nb] = Bm + (long)(bok[nb] ? nb * 16 + r16 : 0) * ldb;
  }
  if constexpr (sizeof(T) == 2) {
    constexpr int KS = 32;
    for (int k0 = kb; k0 < ke; k0 += MAXIT * KS) {
      v8s av[MAXIT], bv[NB][MAXIT];
#pragma unroll
      for (int it = 0; it < MAXIT; ++it) {
        const int kk = k0 + it * KS + kq * 8;
        const bool kok = kk < ke;
        av[it] = kok ? *(const v8s*)(pa + kk) : v8s{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          bv[nb][it] = (kok && bok[nb]) ? *(const v8s*)(pb[nb] + kk)
                                        : v8s{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int it = 0; it < MAXIT; ++it) {
        if (k0 + it * KS >= ke) break;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          if constexpr (__is_same(T, bf16)) {
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[it], bv[nb][it], acc[nb], 0, 0, 0);
          } else {
            typedef __attribute__((ext_vector_type(8))) _Float16 v8h;
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, av[it]),
                                                             __builtin_bit_cast(v8h, bv[nb][it]),
                                                             acc[nb], 0, 0, 0);
          }
        }
      }
    }
  } else {
    constexpr int KS = 16;
    for (int k0 = kb; k0 < ke; k0 += MAXIT * KS) {
      float4 av[MAXIT], bv[NB][MAXIT];
#pragma unroll
      for (int it = 0; it < MAXIT; ++it) {
        const int kk = k0 + it * KS + kq * 4;
        const bool kok = kk < ke;
        av[it] = kok ? *(const float4*)(pa + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          bv[nb][it] = (kok && bok[nb]) ? *(const float4*)(pb[nb] + kk)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int it = 0; it < MAXIT; ++it) {
        if (k0 + it * KS >= ke) break;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[it].x, bv[nb][it].x, acc[nb], 0, 0, 0);
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[it].y, bv[nb][it].y, acc[nb], 0, 0, 0);
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[it].z, bv[nb][it].z, acc[nb], 0, 0, 0);
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[it].w, bv[nb][it].w, acc[nb], 0, 0, 0);
        }
      }
    }
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

struct Args {
  const void* gx;
  const void* w;  // forward: whT; backward: wh
  void* out;
  void* hp;
  float* act;
  float* cell;
  const void* dout;
  void* dgx;
  float* dc;
  void* rh;    // GRU: r * h_{t-1}  [dirs][T][B][H] (T), the candidate GEMM's operand
  float* dhb;  // GRU backward: dh(t) of the previous step   [2][dirs][B][H]
  float* drh;  // GRU backward: d(r*h)(t) of the previous step [2][dirs][B][H]
  int T, B, H, dirs, ldg;
};

typedef float Red[NW][16][RED_LD];

__device__ __forceinline__ void kpart(int K, int parts, int p, int& kb, int& ke) {
  const int per = ((K + parts - 1) / parts + 7) / 8 * 8;
  kb = min(K, p * per);
  ke = min(K, kb + per);
}

// Wave w's partial product (gate w % G, K part w / G of NW / G) into red[w]:
// gate g's A rows start at A0 + g * gstride.  active = false stores zeros
// (the first step: h_{-1} = 0).
template <typename T, int NB>
__device__ __forceinline__ void wave_partial(const T* A0, long gstride, long lda, const T* Bm,
                                             long ldb, int brows, int K, int G, bool active,
                                             Red& red) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  v4f acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = v4f{0.f, 0.f, 0.f, 0.f};
  if (active) {
    const int g = w % G, p = w / G;
    int kb, ke;
    kpart(K, NW / G, p, kb, ke);
    dot_rows<T, NB>(A0 + g * gstride, lda, Bm, ldb, brows, kb, ke, acc);
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][4 * (lane >> 4) + r][nb * 16 + (lane & 15)] = acc[nb][r];
}

// sum of gate g's K parts at (u, b)
__device__ __forceinline__ float gsum(const Red& red, int g, int G, int ul, int bl) {
  float v = 0.f;
  for (int q = g; q < NW; q += G) v += red[q][ul][bl];
  return v;
}

template <typename T, int G, int NB>
__global__ void __launch_bounds__(NT) rnn_fwd_step_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = G * H;
  const int t = d ? T_ - 1 - s : s;
  const int tprev = d ? t + 1 : t - 1, tnext = d ? t - 1 : t + 1;
  const T* hp = (const T*)a.hp;
  wave_partial<T, NB>((const T*)a.w + ((long)d * GH + u0) * H, (long)H * H, H,
                      hp + (((long)d * T_ + t) * B + b0) * H, H, B - b0, H, G, s > 0, red);
  __syncthreads();
  const T* __restrict__ gx = (const T*)a.gx;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long grow = ((long)t * B + b) * a.ldg + (long)d * GH;
  const long srow = ((long)d * T_ + t) * B + b;  // [dirs][T][B] row
  float pre[G];
#pragma unroll
  for (int g = 0; g < G; ++g) pre[g] = (float)gx[grow + g * H + u] + gsum(red, g, G, ul, bl);
  float h;
  if constexpr (G == 4) {
    const float ig = sigm(pre[0]), jg = tanhf(pre[1]), fg = sigm(pre[2] + 1.0f),
                og = sigm(pre[3]);
    const float cp = s > 0 ? a.cell[((long)d * T_ + tprev) * B * H + (long)b * H + u] : 0.f;
    const float c = cp * fg + ig * jg;
    h = tanhf(c) * og;
    float* ap = a.act + srow * GH + u;
    ap[0] = ig; ap[H] = jg; ap[2 * H] = fg; ap[3 * H] = og;
    a.cell[srow * H + u] = c;
  } else {
    h = tanhf(pre[0]);
    a.act[srow * GH + u] = h;
  }
  const T hv = (T)h;
  ((T*)a.out)[((long)t * B + b) * a.dirs * H + (long)d * H + u] = hv;
  T* hpw = (T*)a.hp;
  if (s == 0) hpw[srow * H + u] = (T)0.f;  // h_{-1} = 0 (read by the dWh GEMM)
  if (s + 1 < T_) hpw[(((long)d * T_ + tnext) * B + b) * H + u] = hv;
}

template <typename T, int G, int NB>
__global__ void __launch_bounds__(NT) rnn_bwd_step_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = G * H;
  const int t = d ? s : T_ - 1 - s;  // reverse of the forward order
  const int tnext = d ? t - 1 : t + 1, tprev = d ? t + 1 : t - 1;
  const bool has_prev = d ? t < T_ - 1 : t > 0;
  // dh_rec[u][b] = sum_n wh[d][u][n] * dG(tnext)[b][n], K = G*H in NW parts
  wave_partial<T, NB>((const T*)a.w + ((long)d * H + u0) * GH, 0, GH,
                      (const T*)a.dgx + ((long)(s > 0 ? tnext : t) * B + b0) * a.ldg +
                          (long)d * GH,
                      a.ldg, B - b0, GH, 1, s > 0, red);
  __syncthreads();
  const T* __restrict__ dout = (const T*)a.dout;
  T* __restrict__ dgx = (T*)a.dgx;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long srow = ((long)d * T_ + t) * B + b;
  const float dh = (float)dout[((long)t * B + b) * a.dirs * H + (long)d * H + u] +
                   gsum(red, 0, 1, ul, bl);
  const long grow = ((long)t * B + b) * a.ldg + (long)d * GH;
  if constexpr (G == 4) {
    const float* ap = a.act + srow * GH + u;
    const float ig = ap[0], jg = ap[H], fg = ap[2 * H], og = ap[3 * H];
    const float c = a.cell[srow * H + u];
    const float cp = has_prev ? a.cell[((long)d * T_ + tprev) * B * H + (long)b * H + u] : 0.f;
    const float tc = tanhf(c);
    const long dci = ((long)d * B + b) * H + u, dcn = (long)a.dirs * B * H;
    float dcv = dh * og * (1.f - tc * tc);
    if (s > 0) dcv += a.dc[(s & 1) * dcn + dci];
    a.dc[((s + 1) & 1) * dcn + dci] = dcv * fg;
    dgx[grow + u] = (T)(dcv * jg * ig * (1.f - ig));
    dgx[grow + H + u] = (T)(dcv * ig * (1.f - jg * jg));
    dgx[grow + 2 * H + u] = (T)(dcv * cp * fg * (1.f - fg));
    dgx[grow + 3 * H + u] = (T)(dh * tc * og * (1.f - og));
  } else {
    const float h = a.act[srow * GH + u];
    dgx[grow + u] = (T)(dh * (1.f - h * h));
  }
}

// ---------------------------------------------------------------- GRU
// TF GRUCell: [r, u] = sigmoid([x, h] Wg + bg); c = tanh([x, r*h] Wc + bc);
// h' = u*h + (1-u)*c.  Columns per direction: r | u | c (G = 3); the
// candidate's recurrent GEMM reads r*h, so a step is two launches: the gate
// kernel (writes r, u and r*h) and the candidate kernel (c and h').
template <typename T, int NB>
__global__ void __launch_bounds__(NT) gru_gate_step_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = 3 * H;
  const int t = d ? T_ - 1 - s : s;
  T* hp = (T*)a.hp;
  wave_partial<T, NB>((const T*)a.w + ((long)d * GH + u0) * H, (long)H * H, H,
                      hp + (((long)d * T_ + t) * B + b0) * H, H, B - b0, H, 2, s > 0, red);
  __syncthreads();
  const T* __restrict__ gx = (const T*)a.gx;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long grow = ((long)t * B + b) * a.ldg + (long)d * GH;
  const long srow = ((long)d * T_ + t) * B + b;
  const float rg = sigm((float)gx[grow + u] + gsum(red, 0, 2, ul, bl));
  const float ug = sigm((float)gx[grow + H + u] + gsum(red, 1, 2, ul, bl));
  const float hprev = s > 0 ? (float)hp[srow * H + u] : 0.f;
  a.act[srow * GH + u] = rg;
  a.act[srow * GH + H + u] = ug;
  ((T*)a.rh)[srow * H + u] = (T)(rg * hprev);
  if (s == 0) hp[srow * H + u] = (T)0.f;
}

template <typename T, int NB>
__global__ void __launch_bounds__(NT) gru_cand_step_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = 3 * H;
  const int t = d ? T_ - 1 - s : s, tnext = d ? t - 1 : t + 1;
  T* hp = (T*)a.hp;
  wave_partial<T, NB>((const T*)a.w + ((long)d * GH + 2 * H + u0) * H, 0, H,
                      (const T*)a.rh + (((long)d * T_ + t) * B + b0) * H, H, B - b0, H, 1, s > 0,
                      red);
  __syncthreads();
  const T* __restrict__ gx = (const T*)a.gx;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long grow = ((long)t * B + b) * a.ldg + (long)d * GH;
  const long srow = ((long)d * T_ + t) * B + b;
  const float c = tanhf((float)gx[grow + 2 * H + u] + gsum(red, 0, 1, ul, bl));
  const float ug = a.act[srow * GH + H + u];
  const float hprev = s > 0 ? (float)hp[srow * H + u] : 0.f;
  const float h = ug * hprev + (1.f - ug) * c;
  a.act[srow * GH + 2 * H + u] = c;
  const T hv = (T)h;
  ((T*)a.out)[((long)t * B + b) * a.dirs * H + (long)d * H + u] = hv;
  if (s + 1 < T_) hp[(((long)d * T_ + tnext) * B + b) * H + u] = hv;
}

// Backward step, part A: dh(t) = dout(t) + u(tn) dh(tn) + r(tn) d(rh)(tn)
// + [dr_pre, du_pre](tn) . Wg^T; then dc_pre(t), du_pre(t).
template <typename T, int NB>
__global__ void __launch_bounds__(NT) gru_bwd_a_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = 3 * H;
  const int t = d ? s : T_ - 1 - s, tnext = d ? t - 1 : t + 1;
  const bool has_prev = d ? t < T_ - 1 : t > 0;
  wave_partial<T, NB>((const T*)a.w + ((long)d * H + u0) * GH, 0, GH,
                      (const T*)a.dgx + ((long)(s > 0 ? tnext : t) * B + b0) * a.ldg +
                          (long)d * GH,
                      a.ldg, B - b0, 2 * H, 1, s > 0, red);
  __syncthreads();
  const T* __restrict__ dout = (const T*)a.dout;
  T* __restrict__ dgx = (T*)a.dgx;
  const long dn = (long)a.dirs * B * H;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long srow = ((long)d * T_ + t) * B + b;
  const long dci = ((long)d * B + b) * H + u;
  float dh = (float)dout[((long)t * B + b) * a.dirs * H + (long)d * H + u] +
             gsum(red, 0, 1, ul, bl);
  if (s > 0) {
    const float* an = a.act + (((long)d * T_ + tnext) * B + b) * GH;
    const long q = ((s + 1) & 1) * dn + dci;
    dh += an[H + u] * a.dhb[q] + an[u] * a.drh[q];
  }
  a.dhb[(s & 1) * dn + dci] = dh;
  const float* ap = a.act + srow * GH;
  const float ug = ap[H + u], c = ap[2 * H + u];
  const float hprev = has_prev ? (float)((const T*)a.hp)[srow * H + u] : 0.f;
  const long grow = ((long)t * B + b) * a.ldg + (long)d * GH;
  dgx[grow + 2 * H + u] = (T)(dh * (1.f - ug) * (1.f - c * c));
  dgx[grow + H + u] = (T)(dh * (hprev - c) * ug * (1.f - ug));
}

// Backward step, part B: d(rh)(t) = dc_pre(t) . Wc^T -> dr_pre(t).
template <typename T, int NB>
__global__ void __launch_bounds__(NT) gru_bwd_b_k(Args a, int s) {
  __shared__ Red red;
  constexpr int BT = 16 * NB;
  const int d = blockIdx.z, u0 = blockIdx.x * 16, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int T_ = a.T, B = a.B, H = a.H, GH = 3 * H;
  const int t = d ? s : T_ - 1 - s;
  const bool has_prev = d ? t < T_ - 1 : t > 0;
  wave_partial<T, NB>((const T*)a.w + ((long)d * H + u0) * GH + 2 * H, 0, GH,
                      (const T*)a.dgx + ((long)t * B + b0) * a.ldg + (long)d * GH + 2 * H, a.ldg,
                      B - b0, H, 1, true, red);
  __syncthreads();
  T* __restrict__ dgx = (T*)a.dgx;
  const long dn = (long)a.dirs * B * H;
  const int ul = tid & 15, bl = tid >> 4;
  const int b = b0 + bl, u = u0 + ul;
  if (bl >= BT || b >= B) return;
  const long srow = ((long)d * T_ + t) * B + b;
  const float drh = gsum(red, 0, 1, ul, bl);
  a.drh[(s & 1) * dn + ((long)d * B + b) * H + u] = drh;
  const float rg = a.act[srow * GH + u];
  const float hprev = has_prev ? (float)((const T*)a.hp)[srow * H + u] : 0.f;
  dgx[((long)t * B + b) * a.ldg + (long)d * GH + u] = (T)(drh * hprev * rg * (1.f - rg));
}

// out[n][c][r] = (T) in[n][r][c]   (batched transpose with cast, 32x32 tiles)
template <typename T>
__global__ void __launch_bounds__(256) transpose_cast_k(const float* __restrict__ in,
                                                        T* __restrict__ out, int R, int C) {
  __shared__ float tile[32][33];
  const long base = (long)blockIdx.z * R * C;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int i = 0; i < 32; i += 8) {
    const int r = r0 + ty + i, c = c0 + tx;
    tile[ty + i][tx] = (r < R && c < C) ? in[base + (long)r * C + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 32; i += 8) {
    const int c = c0 + ty + i, r = r0 + tx;
    if (r < R && c < C) out[base + (long)c * R + r] = (T)tile[tx][ty + i];
  }
}

// out[j][i][:] = in[i][j][:]  ([A][Bd][R] -> [Bd][A][R]); R % V == 0
template <typename T, int V>
__global__ void __launch_bounds__(256) permute01_k(const T* __restrict__ in, T* __restrict__ out,
                                                   int A, int Bd, int R) {
  const int rv = R / V;
  const long n = (long)A * Bd * rv;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % rv);
    const long row = e / rv;  // output row j*A + i
    const int i = (int)(row % A), j = (int)(row / A);
    *(Vec<T, V>*)(out + row * R + c * V) = *(const Vec<T, V>*)(in + ((long)i * Bd + j) * R + c * V);
  }
}

template <typename T, int NB>
static hipError_t fwd_nb(int kind, const Args& a, hipStream_t st) {
  const dim3 grid(a.H / 16, (a.B + 16 * NB - 1) / (16 * NB), a.dirs);
  for (int s = 0; s < a.T; ++s) {
    if (kind == LSTM) {
      hipLaunchKernelGGL((rnn_fwd_step_k<T, 4, NB>), grid, dim3(NT), 0, st, a, s);
    } else if (kind == GRU) {
      hipLaunchKernelGGL((gru_gate_step_k<T, NB>), grid, dim3(NT), 0, st, a, s);
      hipLaunchKernelGGL((gru_cand_step_k<T, NB>), grid, dim3(NT), 0, st, a, s);
    } else {
      hipLaunchKernelGGL((rnn_fwd_step_k<T, 1, NB>), grid, dim3(NT), 0, st, a, s);
    }
  }
  return hipGetLastError();
}

template <typename T, int NB>
static hipError_t bwd_nb(int kind, const Args& a, hipStream_t st) {
  const dim3 grid(a.H / 16, (a.B + 16 * NB - 1) / (16 * NB), a.dirs);
  for (int s = 0; s < a.T; ++s) {
    if (kind == LSTM) {
      hipLaunchKernelGGL((rnn_bwd_step_k<T, 4, NB>), grid, dim3(NT), 0, st, a, s);
    } else if (kind == GRU) {
      hipLaunchKernelGGL((gru_bwd_a_k<T, NB>), grid, dim3(NT), 0, st, a, s);
      hipLaunchKernelGGL((gru_bwd_b_k<T, NB>), grid, dim3(NT), 0, st, a, s);
    } else {
      hipLaunchKernelGGL((rnn_bwd_step_k<T, 1, NB>), grid, dim3(NT), 0, st, a, s);
    }
  }
  return hipGetLastError();
}

// One 16-row batch block per workgroup for batches <= 16 (more workgroups
// on small batches), two otherwise (half the weight re-reads).
template <typename T>
static hipError_t fwd(int kind, const Args& a, hipStream_t st) {
  return a.B <= 16 ? fwd_nb<T, 1>(kind, a, st) : fwd_nb<T, 2>(kind, a, st);
}

template <typename T>
static hipError_t bwd(int kind, const Args& a, hipStream_t st) {
  return a.B <= 16 ? bwd_nb<T, 1>(kind, a, st) : bwd_nb<T, 2>(kind, a, st);
}

}  // namespace rnn
}  // namespace kfb

using namespace kfb;

static int rnn_gates(int kind) { return kind == rnn::LSTM ? 4 : kind == rnn::GRU ? 3 : 1; }

static bool rnn_shape_ok(int kind, int T, int B, int H, int dirs) {
  return (kind == rnn::LSTM || kind == rnn::TANH || kind == rnn::GRU) && T > 0 && B > 0 && H > 0 && H % 16 == 0 &&
         (dirs == 1 || dirs == 2);
}

// Forward recurrence over all T steps (see the layout block at the top).
// rh: GRU only ([dirs][T][B][H] in dtype, kept for the backward).
KFB_API hipError_t kfb_rnn_fwd(int dtype, int kind, const void* gx, const void* whT, void* out,
                               void* hp, float* act, float* cell, void* rh, int T, int B, int H,
                               int dirs, hipStream_t stream) {
  if (!rnn_shape_ok(kind, T, B, H, dirs) || (kind == rnn::LSTM && !cell) ||
      (kind == rnn::GRU && !rh))
    return hipErrorInvalidValue;
  const int G = rnn_gates(kind);
  rnn::Args a{gx, whT, out, hp, act, cell, nullptr, nullptr, nullptr, rh, nullptr, nullptr,
              T, B, H, dirs, dirs * G * H};
  KFB_DISPATCH_DTYPE(dtype, T_, return rnn::fwd<T_>(kind, a, stream));
  return hipSuccess;
}

// Backward recurrence: dgx [T][B][dirs*G*H] (T) receives d(gx); dc (LSTM),
// dhb and drh (GRU) are [2][dirs][B][H] fp32 workspaces; hp is the forward's
// h-entering-each-step tensor (GRU).
KFB_API hipError_t kfb_rnn_bwd(int dtype, int kind, const void* dout, const void* wh,
                               const float* act, const float* cell, const void* hp, void* dgx,
                               float* dc, float* dhb, float* drh, int T, int B, int H, int dirs,
                               hipStream_t stream) {
  if (!rnn_shape_ok(kind, T, B, H, dirs) || (kind == rnn::LSTM && (!cell || !dc)) ||
      (kind == rnn::GRU && (!hp || !dhb || !drh)))
    return hipErrorInvalidValue;
  const int G = rnn_gates(kind);
  rnn::Args a{nullptr, wh, nullptr, (void*)hp, (float*)act, (float*)cell, dout, dgx, dc,
              nullptr, dhb, drh, T, B, H, dirs, dirs * G * H};
  KFB_DISPATCH_DTYPE(dtype, T_, return rnn::bwd<T_>(kind, a, stream));
  return hipSuccess;
}

// out[n] = cast(in[n]^T): in fp32 [nb][R][C] -> out [nb][C][R] in dtype.
KFB_API hipError_t kfb_transpose_cast(int dtype, const float* in, void* out, int nb, int R, int C,
                                      hipStream_t stream) {
  const dim3 grid((C + 31) / 32, (R + 31) / 32, nb);
  KFB_DISPATCH_DTYPE(dtype, T_,
                     hipLaunchKernelGGL(rnn::transpose_cast_k<T_>, grid, dim3(256), 0, stream,
                                        in, (T_*)out, R, C));
  return hipGetLastError();
}

// [A][Bd][R] -> [Bd][A][R] (swap the two leading dims; R contiguous).
KFB_API hipError_t kfb_permute01(int dtype, const void* in, void* out, int A, int Bd, int R,
                                 hipStream_t stream) {
  const int es = dtype == F32 ? 4 : 2;
  const int vw = vec_width(R) * es > 16 ? 16 / es : vec_width(R);
  const long n = (long)A * Bd * (R / vw);
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  KFB_DISPATCH_DTYPE(dtype, T_,
                     KFB_DISPATCH_VEC(vw, V,
                                      hipLaunchKernelGGL((rnn::permute01_k<T_, V>),
                                                         dim3((unsigned)blocks), dim3(256), 0,
                                                         stream, (const T_*)in, (T_*)out, A, Bd,
                                                         R)));
  return hipGetLastError();
}
