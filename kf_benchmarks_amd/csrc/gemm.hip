// MFMA GEMM for affine (fully connected) layers on gfx950.
//
// Replaces the cuBLAS matmul of tcb/convnet_builder.py:311-345 (affine,
// matmul at :336) and its autodiff.  One kernel template computes
//
//     C[m][n] = sum_k P(m, k) * Q(n, k)
//
// where each operand is stored either K-contiguous ("KC": P[m*ldp + k]) or
// K-strided ("KS": P[k*ldp + m]).  With the affine weight in its TF layout
// W[Cin][Cout] (fp32 master, bf16 compute copy) the three GEMMs of a layer
// need no transposed weight copy:
//
//     forward  y [B][Cout] = x [B][Cin]  . W        P = x   (KC), Q = W  (KS)
//     dgrad    dx[B][Cin]  = dy[B][Cout] . W^T      P = dy  (KC), Q = W  (KC)
//     wgrad    dW[Cin][Cout] = x^T . dy             P = x   (KS), Q = dy (KS)
//
// Tiles: 256 threads = 4 waves (2 x 2), 128 x 128 output tile, K step 64
// (fp32: 32), v_mfma_f32_16x16x32_bf16 (fp32: v_mfma_f32_16x16x4_f32, exact
// fp32 products) with the N-side operand as the A matrix so each
// lane's 4 accumulators are 4 consecutive output columns of one row.  Both
// operand tiles go through a double-buffered LDS stage, loaded one K step
// ahead in registers with range-checked buffer loads (out-of-range -> 0).
// A KC image has 128-byte rows (one K step) whose 16-byte chunks are
// XOR-swizzled and is read with ds_read_b128; a 16-bit KS image has 256-byte
// rows (one k, 128 m or n) with 32-byte units XOR-swizzled and is read with
// the hardware transpose ds_read_b64_tr_b16, so the fragment k order is the
// natural one on both kinds and they pair in one MFMA (fp32: see Tr<float>).
//
// Small-batch layers (VGG/AlexNet fc6-8: M = batch <= 512, K up to 25088)
// stream the weight once and have few output tiles, so the forward and
// dgrad split K over workgroups (>= 2 workgroups per CU) into an fp32 slab
// that one elementwise pass reduces, adds the bias, applies the ReLU and
// converts; wgrad (reduction over the batch) writes fp32 straight into the
// flat gradient buffer.
#include "gemm_core.h"

namespace kfb {

namespace gm {

struct Args {
  const void* p;  // M-side operand
  const void* q;  // N-side operand
  int M, N, K, ldp, ldq;
  int pbytes, qbytes;  // byte ranges of p / q (< 2 GiB)
  void* c;             // OUT_T: T [M][ldc]; OUT_F32: float [M][ldc]
  int ldc;
  float* slab;         // OUT_SLAB: [nsplit][M][ldslab]
  int ldslab;
  int kper;            // K per split (multiple of the K step)
  const float* bias;   // OUT_T: [N] or null
  int relu;
  int accumulate;      // OUT_F32: C += result
};

template <typename T, bool PKS, bool QKS, bool PV, bool QV, int OUT>
__global__ void __launch_bounds__(256, 2) gemm_k(Args a) {
  constexpr int TM = TILE / 32, TN = TILE / 32;  // 16-wide subtiles per wave
  constexpr int IMG = img_elems<T>();
  constexpr int BK = Tr<T>::BK;
  __shared__ __attribute__((aligned(16))) T smem[2 * 2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mt = (a.M + TILE - 1) / TILE, nt = (a.N + TILE - 1) / TILE;
  const int tiles = mt * nt;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // tile-major within a split, m fastest: consecutive ids share the N-side
  // (weight) tile on one XCD
  const int split = bid / tiles, tile = bid - split * tiles;
  const int m0 = (tile % mt) * TILE, n0 = (tile / mt) * TILE;
  const int kbeg = split * a.kper;
  const int kend = min(a.K, kbeg + a.kper);

  Loader<T, PKS, PV> lp;
  Loader<T, QKS, QV> lq;
  lp.init(a.p, a.pbytes, a.ldp, a.M, m0, kend, tid);
  lq.init(a.q, a.qbytes, a.ldq, a.N, n0, kend, tid);
  v4f acc[TN][TM];
  const int wn = wid >> 1, wm = wid & 1;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  mainloop<T>(lp, lq, kbeg, nk, smem, acc);

  // acc[i][j][r] = C[m][n + r], m = m0 + wm*64 + j*16 + (lane & 15),
  //                             n = n0 + wn*64 + i*16 + (lane >> 4) * 4
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int m = m0 + wm * (TILE / 2) + j * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wn * (TILE / 2) + i * 16 + (lane >> 4) * 4;
      if (n >= a.N) continue;
      v4f v = acc[i][j];
      if constexpr (OUT == OUT_SLAB) {
        // ldslab is a multiple of 4: columns past N land in the padding
        *(v4f*)(a.slab + ((long)split * a.M + m) * a.ldslab + n) = v;
      } else if constexpr (OUT == OUT_F32) {
        float* c = (float*)a.c + (long)m * a.ldc + n;
        if (n + 3 < a.N && (a.ldc & 3) == 0) {
          if (a.accumulate) {
            const v4f o = *(const v4f*)c;
            v += o;
          }
          *(v4f*)c = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < a.N) c[r] = a.accumulate ? c[r] + v[r] : v[r];
        }
      } else {
        T* c = (T*)a.c + (long)m * a.ldc + n;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = v[r];
          if (a.bias && n + r < a.N) t += a.bias[n + r];
          o[r] = a.relu ? fmaxf(t, 0.f) : t;
        }
        if (n + 3 < a.N && (a.ldc & 3) == 0) {
          Vec<T, 4> w;
#pragma unroll
          for (int r = 0; r < 4; ++r) w.v[r] = (T)o[r];
          *(Vec<T, 4>*)c = w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < a.N) c[r] = (T)o[r];
        }
      }
    }
  }
}

// out[m][n] = act(sum_s slab[s][m][n] + bias[n]) as T; one thread per 4 columns.
template <typename T>
__global__ void __launch_bounds__(256) slab_reduce_k(const float* __restrict__ slab, int nsplit,
                                                     int M, int N, int ldslab,
                                                     const float* __restrict__ bias, int relu,
                                                     T* __restrict__ out, int ldc,
                                                     int accumulate) {
  const int q4 = ldslab >> 2;
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= (long)M * q4) return;
  const int m = (int)(i / q4), n = (int)(i - (long)m * q4) * 4;
  if (n >= N) return;
  const long plane = (long)M * ldslab;
  const float* s = slab + (long)m * ldslab + n;
  v4f acc = *(const v4f*)s;
  for (int k = 1; k < nsplit; ++k) acc += *(const v4f*)(s + k * plane);
  T* c = out + (long)m * ldc + n;
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t = acc[r];
    if (bias && n + r < N) t += bias[n + r];
    if (accumulate && n + r < N) t += (float)c[r];  // (wgrad: fp32 C += result)
    o[r] = relu ? fmaxf(t, 0.f) : t;
  }
  if (n + 3 < N && (ldc & 3) == 0) {
    Vec<T, 4> w;
#pragma unroll
    for (int r = 0; r < 4; ++r) w.v[r] = (T)o[r];
    *(Vec<T, 4>*)c = w;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < N) c[r] = (T)o[r];
  }
}

// Split-K count for an output of M x N with reduction K: >= 2 workgroups
// per CU when the tile count alone does not reach it, >= 4 K steps each.
template <typename T>
inline int choose_split(int M, int N, int K) {
  const int tiles = ((M + TILE - 1) / TILE) * ((N + TILE - 1) / TILE);
  const int nk = (K + Tr<T>::BK - 1) / Tr<T>::BK;
  if (tiles >= 256) return 1;
  int s = (512 + tiles - 1) / tiles;
  const int smax = nk / 4;
  if (s > smax) s = smax;
  return s < 1 ? 1 : s;
}

template <typename T, bool PKS, bool QKS, int OUT>
static void launch(const Args& a, bool pv, bool qv, int nwg, hipStream_t s) {
  const dim3 g(nwg), b(256);
  if (pv && qv) hipLaunchKernelGGL((gemm_k<T, PKS, QKS, true, true, OUT>), g, b, 0, s, a);
  else if (pv) hipLaunchKernelGGL((gemm_k<T, PKS, QKS, true, false, OUT>), g, b, 0, s, a);
  else if (qv) hipLaunchKernelGGL((gemm_k<T, PKS, QKS, false, true, OUT>), g, b, 0, s, a);
  else hipLaunchKernelGGL((gemm_k<T, PKS, QKS, false, false, OUT>), g, b, 0, s, a);
}

template <typename T>
static hipError_t run(int mode, const Args& a0, int nsplit, hipStream_t s) {
  Args a = a0;
  // VEC: 8-element chunks along each operand's contiguous extent are whole
  // and 16-byte aligned
  const bool pks = mode == 2, qks = mode != 1;
  constexpr int E = Tr<T>::EPC;
  const bool pv = a.ldp % E == 0 && (pks ? a.M : a.K) % E == 0;
  const bool qv = a.ldq % E == 0 && (qks ? a.N : a.K) % E == 0;
  const int tiles = ((a.M + TILE - 1) / TILE) * ((a.N + TILE - 1) / TILE);
  if (mode == 2 && nsplit <= 1) {  // wgrad: fp32 output
    a.kper = a.K;
    launch<T, true, true, OUT_F32>(a, pv, qv, tiles, s);
    return hipGetLastError();
  }
  if (nsplit <= 1) {
    a.kper = a.K;
    if (mode == 0) launch<T, false, true, OUT_T>(a, pv, qv, tiles, s);
    else launch<T, false, false, OUT_T>(a, pv, qv, tiles, s);
    return hipGetLastError();
  }
  const int nk = (a.K + Tr<T>::BK - 1) / Tr<T>::BK;
  a.kper = ((nk + nsplit - 1) / nsplit) * Tr<T>::BK;
  nsplit = (a.K + a.kper - 1) / a.kper;
  if (mode == 0) launch<T, false, true, OUT_SLAB>(a, pv, qv, tiles * nsplit, s);
  else if (mode == 1) launch<T, false, false, OUT_SLAB>(a, pv, qv, tiles * nsplit, s);
  else launch<T, true, true, OUT_SLAB>(a, pv, qv, tiles * nsplit, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const long work = (long)a.M * (a.ldslab / 4);
  if (mode == 2)  // the split wgrad's fp32 (+=) output
    hipLaunchKernelGGL(slab_reduce_k<float>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                       s, (const float*)a.slab, nsplit, a.M, a.N, a.ldslab, nullptr, 0,
                       (float*)a.c, a.ldc, a.accumulate);
  else
    hipLaunchKernelGGL(slab_reduce_k<T>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                       (const float*)a.slab, nsplit, a.M, a.N, a.ldslab, a.bias, a.relu, (T*)a.c,
                       a.ldc, 0);
  return hipGetLastError();
}

}  // namespace gm
}  // namespace kfb

using namespace kfb;

// Split count kfb_gemm will use for a GEMM of this output shape and reduction
// (the caller sizes the slab workspace: nsplit * M * round_up(N, 4) floats).
KFB_API int kfb_gemm_splits(int dtype, int M, int N, int K) {
  return dtype == F32 ? gm::choose_split<float>(M, N, K) : gm::choose_split<bf16>(M, N, K);
}

// mode 0: forward  C[M][N] = P[M][K] . Q[K][N]           (P KC, Q KS)  -> T
// mode 1: dgrad    C[M][N] = P[M][K] . Q[N][K]^T         (P KC, Q KC)  -> T
// mode 2: wgrad    C[M][N] = P[K][M]^T . Q[K][N]          (P KS, Q KS)  -> fp32 (+=)
// T outputs get bias[n] (nullable) and an optional ReLU; K is split into
// `slab` (>= nsplit * M * round_up(N, 4) floats) when nsplit > 1 (wgrad: a
// small output over a long batch, e.g. NCF's 256 x 256 layers at batch 2048,
// which unsplit runs 4 workgroups down the whole batch).
KFB_API hipError_t kfb_gemm(int dtype, int mode, const void* p, int ldp, const void* q, int ldq,
                            int M, int N, int K, void* c, int ldc, const float* bias, int relu,
                            int accumulate, float* slab, long slab_elems, int nsplit,
                            hipStream_t stream) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (mode < 0 || mode > 2 || K < 0) return hipErrorInvalidValue;
  const int esz = dtype == F32 ? 4 : 2;
  const long pel = mode == 2 ? (long)K * ldp : (long)M * ldp;
  const long qel = mode == 1 ? (long)N * ldq : (long)K * ldq;
  if (pel * esz >= (1L << 31) || qel * esz >= (1L << 31)) return hipErrorInvalidValue;
  const int ldslab = (N + 3) / 4 * 4;
  if (nsplit > 1 && (slab == nullptr || (long)nsplit * M * ldslab > slab_elems))
    return hipErrorInvalidValue;
  gm::Args a{p, q, M, N, K, ldp, ldq, (int)(pel * esz), (int)(qel * esz), c, ldc, slab,
             ldslab, K, bias, relu, accumulate};
  if (dtype == F32) return gm::run<float>(mode, a, nsplit, stream);
  if (dtype == BF16) return gm::run<bf16>(mode, a, nsplit, stream);
  if (dtype == F16) return gm::run<f16>(mode, a, nsplit, stream);
  return hipErrorInvalidValue;
}
