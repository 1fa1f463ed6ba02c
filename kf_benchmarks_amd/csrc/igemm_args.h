// Arguments of the implicit-GEMM convolution kernels (conv_igemm.hip) and
// of the streaming 3x3 kernel (conv_stream.hip): one launch = one conv
// forward / dgrad / scattered 1x1 GEMM with an optional fused epilogue.
#pragma once
#include "common.h"

namespace kfb {

// BN forward finalize of a conv whose epilogue accumulated the statistics
// (counter == null: off): the last workgroup to finish folds the
// [2][IG_SPREAD][Ncol] slots into mean / invstd, scale / shift, the running
// statistics and the next step's statistics shift - the work of
// bn.hip's bn_finalize_stats_k, without its launch
// (tcb/convnet_builder.py:437-461 batch_norm in training mode).
struct BnFin {
  int* counter;  // zeroed with the statistics slots
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* save_mean;
  float* save_invstd;
  float* scale;
  float* shift;
  float* kshift;  // the shift the partials are centered on (updated to this mean)
  float decay, eps;
  long rows;
};

// BN backward finalize of a dgrad whose epilogue accumulated the producer
// BN's backward partials (counter == null: off): the last workgroup folds the
// [2][IG_SPREAD][Ncol] slots into dgamma / dbeta and the apply coefficients
// dx = dy' * A + x * B + Cc - the work of bn.hip's bn_finalize_grad_k
// without its launch (the BN's saved mean is IgArgs::mean).
struct BnGFin {
  int* counter;  // zeroed with the partial-sum slots
  const float* gamma;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* coefA;
  float* coefB;
  float* coefC;
  int accumulate;  // add into dgamma / dbeta (flat gradient buffer) instead of writing
};

struct IgArgs {
  const void* x;  // gathered operand (NHWC [N,H,W,C])
  const void* w;  // [Ncol][Ktot]
  void* y;        // output rows
  int N, H, W, C;
  int OH, OW;     // GEMM row space (M = N*OH*OW)
  int KH, KW, sh, sw, pt, pl;
  int Ncol, Ktot, M;
  int YH, YW, ys, ldy;  // row m=(img,oh,ow) -> ((img*YH + oh*ys)*YW + ow*ys)*ldy
  // Fused epilogue (optional):
  //   stats != null, mask == null : BN forward statistics of the output,
  //       stats[slot][0][n] += sum y, stats[slot][1][n] += sum y^2
  //   stats != null, xbn != null  : BN backward partials of the *producer* BN
  //       of this conv's input: y' = y * (mask > 0) (mask may be null = no
  //       ReLU), stats[slot][0][n] += sum y', stats[slot][1][n] += sum y'(xbn - mean)
  //   layout [2][IG_SPREAD][Ncol]; slot = pixel-tile index % IG_SPREAD (spreads
  //   the atomics over 32 copies; the BN finalize folds the 32 slots).  Keyed
  //   by the pixel tile, not the workgroup: the pixel tiles of one channel
  //   tile land in distinct slots, so with <= 32 pixel tiles every slot takes
  //   one add and the statistics are bitwise run-to-run deterministic.
  float* stats;
  const void* mask;
  const void* xbn;
  const float* mean;
  // addend != null: y = conv(...) + addend (same layout as y) before the
  // mask / statistics - the gradient other consumers of the conv input
  // already produced (residual / second-branch accumulation).
  const void* addend;
  // mcoef != null (with xbn, mask == null): the producer BN's ReLU mask is
  // recomputed as xbn * scale + shift > 0 (mcoef = [scale | shift], [2][Ncol])
  // instead of read from its output - BNs without a residual add.
  const float* mcoef;
  // Forward epilogue of a conv without BN (VGG / AlexNet / GoogLeNet
  // style): y = act(conv + bias[n]), bias nullable, relu 0/1; never combined
  // with the statistics or the dgrad-style operands.
  const float* bias;
  int relu;
  // FAST path only: byte sizes of x and w (buffer-descriptor range checks)
  int xbytes, wbytes;
  // byte size of the output layout (= that of addend / mask / xbn), or 0 if
  // >= 2 GiB (the epilogue then uses plain loads instead of buffer loads)
  int ybytes;
  // forward statistics only: per-channel shift K (nullable); the partials
  // are sums of (y - K) and (y - K)^2 (see bn_finalize_stats_k)
  const float* kshift;
  // generic (non-FAST) loader: k -> (tap, channel) -> (kh, kw) and the
  // transposed gather's stride divisions as multiply-high divisions
  FastDiv fd_c, fd_kw, fd_sh, fd_sw;
  // stride-2 scatter (ys == 2, YH == 2*OH, YW == 2*OW): every output chunk
  // also writes zeros to the three unsampled pixels of its 2x2 block, so the
  // output needs no separate zero fill
  int zfill;
  // 8-channel geometry (C == 8, KW | 8, KH*KW % 8 == 0; e.g. the stem's
  // pixel-pair conv, csrc/stem.hip): a 64-deep K step spans 8 taps, one
  // 16-byte chunk each, so each lane's chunk kc is its own tap
  // (kh, kw) = (8s + kc) / KW, (8s + kc) % KW of step s; the step advances
  // the rows by 8 / KW (c8_step elements)
  int c8, c8_step;
  // mask != null: 1 = `mask` is the producer BN's ReLU bit mask (bit k of
  // byte e/8 = y[e + k] > 0 for the 8-element chunk starting at element e,
  // written by the BN apply pass, csrc/bn.hip relu_bits) instead of its
  // output y - 1/16 of the bytes for the same test
  int maskbits;
  BnFin fin;
  BnGFin gfin;
  // Streaming 1x1 apply form (conv_s1.hip EPI_APPLY, out != null): the conv
  // output y is recomputed from x and w instead of read back, and the BN
  // apply of its consumer runs in the epilogue:
  //   out = relu?(bf16(y) * bn_scale[n] + bn_shift[n] + addend), y stored too
  //   (ybytes 0: not stored), out_bits = out's ReLU bit mask (nullable)
  void* out;
  const float* bn_scale;
  const float* bn_shift;
  uint8_t* out_bits;
  int outbytes;  // byte size of out (< 2 GiB)
  // Second BN of a dual-BN block output y = relu(bn(x) + bn2(x2))
  // (kfb_bn_fwd_train_dual; conv_s1.hip EPI_DGRAD with the bit mask only):
  // the masked y' is also the output gradient of bn2, whose backward
  // partial stats2[slot][n] += sum y'(xbn2 - mean2) ([IG_SPREAD][Ncol]) the
  // epilogue accumulates beside the first BN's; bn2's sum y' is the first
  // half of `stats`.  xbn2 == null: off.
  const void* xbn2;
  const float* mean2;
  float* stats2;
};

constexpr int IG_BK = 64;
constexpr int IG_SPREAD = 32;

// One channel's finalize from its summed partials (double): the math of
// bn_finalize_stats_k.
__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int c, double s, double q) {
  const double n = (double)f.rows;
  const double k = f.kshift ? (double)f.kshift[c] : 0.0;
  const double dm = s / n;
  const double mean = k + dm;
  double var = q / n - dm * dm;
  if (var < 0.0) var = 0.0;
  if (f.kshift) f.kshift[c] = (float)mean;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float g = f.gamma ? f.gamma[c] : 1.f;
  const float b = f.beta ? f.beta[c] : 0.f;
  f.save_mean[c] = (float)mean;
  f.save_invstd[c] = invstd;
  f.scale[c] = g * invstd;
  f.shift[c] = b - (float)mean * g * invstd;
  if (f.run_mean) {
    const double unbiased = f.rows > 1 ? var * n / (n - 1.0) : var;
    f.run_mean[c] = f.run_mean[c] * f.decay + (float)mean * (1.f - f.decay);
    f.run_var[c] = f.run_var[c] * f.decay + (float)unbiased * (1.f - f.decay);
  }
}

// Called once by every workgroup of the launch, at its very end, after its
// statistics atomics: true in the last one to arrive.  The slots are only
// ever written by float atomics, which execute at the memory side (MI355X
// guide, Global float atomics), so there are no dirty L2 lines to publish:
// a workgroup's vmcnt drain (its atomics acknowledged) orders them before
// its ticket, with no agent release (a buffer_wbl2 per workgroup measured
// +35 % on the 56x56 convs); the last arriver acquires and reads the slots
// with agent-scope loads.  `flag`: one int of the kernel's LDS (dead by now).
__device__ __forceinline__ bool last_arriver(int* counter, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int total = (int)(gridDim.x * gridDim.y * gridDim.z);
    const int prev = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == total - 1;
  }
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return true;
}

// Folds the [2][IG_SPREAD][Ncol] slots of channels 4 g .. 4 g + 3 (after the
// last arriver's acquire): 16 independent 16-byte loads per batch, so the
// serial tail costs four memory round trips per channel group rather than
// one per few slots.
__device__ __forceinline__ void fold_slots4(const IgArgs& a, int g, double (&s)[4],
                                            double (&q)[4]) {
  typedef __attribute__((ext_vector_type(4))) float f4;
#pragma unroll
  for (int j = 0; j < 4; ++j) { s[j] = 0.0; q[j] = 0.0; }
  const f4* p = (const f4*)a.stats + g;
  const long row = a.Ncol / 4;
#pragma unroll
  for (int kb = 0; kb < IG_SPREAD; kb += 8) {
    f4 vs[8], vq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      vs[k] = p[(kb + k) * row];
      vq[k] = p[(IG_SPREAD + kb + k) * row];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] += vs[k][j];
        q[j] += vq[k][j];
      }
  }
}

__device__ __forceinline__ void bn_fin_tail(const IgArgs& a, int* flag) {
  if (!a.fin.counter || !a.stats) return;  // (uniform)
  if (!last_arriver(a.fin.counter, flag)) return;
  for (int g = threadIdx.x; g < a.Ncol / 4; g += blockDim.x) {
    double s[4], q[4];
    fold_slots4(a, g, s, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) bn_fin_channel(a.fin, 4 * g + j, s[j], q[j]);
  }
}

// the dgrad form (bn_finalize_grad_k's math): dgamma = invstd * S2,
// dbeta = S1, A = g * invstd, B = -A * invstd^2 * S2 / n,
// Cc = -A * S1 / n - mean * B
__device__ __forceinline__ void bn_gfin_tail(const IgArgs& a, int* flag) {
  if (!a.gfin.counter || !a.stats) return;  // (uniform)
  if (!last_arriver(a.gfin.counter, flag)) return;
  const double n = (double)a.M;
  for (int g4 = threadIdx.x; g4 < a.Ncol / 4; g4 += blockDim.x) {
    double s[4], q[4];
    fold_slots4(a, g4, s, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * g4 + j;
      const double s1 = s[j], s2 = q[j];
      const float is = a.gfin.invstd[c];
      const float g = a.gfin.gamma ? a.gfin.gamma[c] : 1.f;
      if (a.gfin.dgamma)
        a.gfin.dgamma[c] = (a.gfin.accumulate ? a.gfin.dgamma[c] : 0.f) + (float)(s2 * is);
      if (a.gfin.dbeta)
        a.gfin.dbeta[c] = (a.gfin.accumulate ? a.gfin.dbeta[c] : 0.f) + (float)s1;
      const double A = (double)g * is;
      const double B = -A * (double)is * (double)is * s2 / n;
      a.gfin.coefA[c] = (float)A;
      a.gfin.coefB[c] = (float)B;
      a.gfin.coefC[c] = (float)(-A * s1 / n - (double)a.mean[c] * B);
    }
  }
}

// the tail of a kernel that can carry either finalize
__device__ __forceinline__ void bn_tail(const IgArgs& a, int* flag) {
  if (a.gfin.counter) bn_gfin_tail(a, flag);
  else bn_fin_tail(a, flag);
}

// bn.hip: the separate finalize launches (kernels without the tail)
hipError_t bn_finalize_grad_launch(const float* slots, int C, long rows, const float* gamma,
                                   const float* mean, const float* invstd, float* dgamma,
                                   float* dbeta, float* coefA, float* coefB, float* coefC,
                                   int accumulate, hipStream_t stream);
hipError_t bn_finalize_stats_launch(const float* psum, const float* psq, int nslab, int C,
                                    long rows, const float* gamma, const float* beta, float decay,
                                    float eps, float* run_mean, float* run_var, float* save_mean,
                                    float* save_invstd, float* scale, float* shift, float* kshift,
                                    hipStream_t stream);

// conv_stream.hip: the streaming 3x3 64-channel kernel (IG_ALGO_S3)
bool conv_s3_fits(const IgArgs& a);
hipError_t launch_conv_s3(int dtype, const IgArgs& a, hipStream_t stream);
// conv_s1.hip: the streaming 1x1 64 -> 256-channel kernel (IG_ALGO_S1)
// (ybytes 0 in a statistics-only launch: the output is not stored)
bool conv_s1_fits(const IgArgs& a);
hipError_t launch_conv_s1(int dtype, const IgArgs& a, hipStream_t stream);
// conv_s7.hip: the streaming stem conv (IG_ALGO_S7)
bool conv_s7_fits(const IgArgs& a);
hipError_t launch_conv_s7(int dtype, const IgArgs& a, hipStream_t stream);
// conv_stream.hip: the streaming 3x3 kernel's streaming weight gradient (slab per workgroup + fixed-order fold)
int wgrad_s3_splits(int N, int H, int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                    int pt, int pl, int Ncol);
hipError_t launch_wgrad_s3(int dtype, const void* dy, const void* x, float* dw, int N, int H,
                           int W, int C, int OH, int OW, int KH, int KW, int sh, int sw, int pt,
                           int pl, int Ncol, float* slab, long slab_elems, hipStream_t stream);

}  // namespace kfb
