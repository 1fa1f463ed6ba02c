// Streaming 3x3 convolution for 64-channel layers (ResNet conv2_x: 56x56,
// 64 -> 64, stride 1, SAME padding), forward and stride-1 dgrad, with the
// implicit-GEMM kernels' fused epilogues (BN statistics, ReLU mask / BN
// backward partials, addend).  Replaces the cuDNN conv of
// tcb/convnet_builder.py:107-213 on the shapes of
// tcb/models/resnet_model.py:306-328 (conv2_x bottleneck 3x3).
//
// Why a separate kernel: the tiled igemm kernels (conv_igemm.hip) fetch the
// pixel tile of every one of the 9 taps from L2 again and re-stage it through
// LDS, and keep only one K step of the 64 x 576 weight slab on chip; at 64
// channels that makes them LDS-write bound (profiles/r8_conv3x3_pmc.txt:
// 22.6 % MFMA busy, SQ_WAIT_INST_LDS 29 M cycles).  Here:
//
//  * one persistent 256-thread workgroup per CU, 152 KB of LDS: the whole
//    weight slab (9 taps x 64 x 64 bf16 = 72 KB) is loaded once by LDS-DMA
//    and stays resident;
//  * the input is read exactly once, as a stream: output pixels are indexed
//    in a zero-padded "position" space in which every tap is a constant
//    shift.  The batch is laid out as rows of W+1 positions (column 0 is the
//    zero pad shared by the right edge of one row and the left edge of the
//    next), H+1 rows per image (row 0 of each image is the zero row shared
//    with the image above), so pixel (img, h, w) sits at
//        P = (img*(H+1) + 1 + h) * (W+1) + 1 + w
//    and tap (kh, kw) of output position Q reads input position
//    Q + (kh-1)*(W+1) + (kw-1).  3.5 % of the computed positions are pads
//    (discarded), in exchange every MFMA operand fragment is 32 consecutive
//    positions at every tap;
//  * each workgroup owns a contiguous run of 256-position tiles; the input
//    positions stream through a 640-position LDS ring (5 blocks of 128)
//    filled by LDS-DMA with range-checked buffer loads (a pad position loads
//    zeros), two blocks ahead, one barrier per tile.  Tile t reads blocks
//    2t..2t+2 while blocks 2t+3, 2t+4 land in the slots tile t-1 released;
//  * 4 waves, each a 64-channel x 64-position wave tile of four
//    v_mfma_f32_32x32x16_bf16 accumulators (weights = A, positions = B): one
//    ds_read_b128 per MFMA, half the LDS rate;
//  * ring and weight images are XOR-swizzled by position / channel
//    ((p >> 1) & 7 on the 16-byte chunk): the 16-lane groups of every
//    ds_read_b128 read 16 distinct positions mod 16, so every fragment read
//    is conflict-free at every tap shift;
//  * the epilogue works from registers: v_permlane32_swap pairs turn the
//    32x32 accumulator layout into 8 consecutive channels of one position
//    per lane (one 16-byte store per chunk, no LDS staging); the BN
//    statistics / backward partials accumulate per lane across all the
//    workgroup's tiles and are reduced across lanes once, at the end.
#include "common.h"
#include "igemm_args.h"

#include <mutex>

namespace kfb {
namespace s3 {

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(16))) float v16f;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u_t;

constexpr int CH = 64;              // input and output channels
constexpr int BM = 256;             // output positions per tile (4 waves x 64)
constexpr int BLK = 128;            // positions per ring block
constexpr int NBLK = 5;             // ring blocks
constexpr int RING = BLK * NBLK;    // 640 positions (80 KB)
constexpr int ROWB = CH * 2;        // bytes per position / weight row
constexpr int W_BYTES = 9 * CH * ROWB;     // 73728
constexpr int R_BYTES = RING * ROWB;       // 81920
constexpr int NPRM = 5 * CH;               // kshift | mean | scale | shift | bias
constexpr int LDS_BYTES = W_BYTES + R_BYTES + NPRM * 4;  // 156928

struct Geo {
  int W1, H1;       // W + 1, H + 1
  FastDiv fw1, fh1;
  int Qlo, Qhi;     // output positions [Qlo, Qhi)
  int tiles;        // ceil((Qhi - Qlo) / BM)
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           off, 0, 0, 0);
}

__device__ __forceinline__ void barrier_lds() { asm volatile("s_barrier" ::: "memory"); }

// byte offset of the pixel at padded position P in the NHWC tensor, or -1 for
// a pad position / outside the batch
__device__ __forceinline__ int pix_off(int P, const Geo& g, const IgArgs& a) {
  if (P < 0) return -1;
  const int r = g.fw1.div(P), c = P - r * g.W1;
  const int img = g.fh1.div(r), rr = r - img * g.H1;
  if (c == 0 || rr == 0 || img >= a.N) return -1;
  return ((img * a.H + rr - 1) * a.W + c - 1) * ROWB;
}

__device__ __forceinline__ unsigned f2u(float f) { return __builtin_bit_cast(unsigned, f); }
__device__ __forceinline__ float u2f(unsigned u) { return __builtin_bit_cast(float, u); }

template <typename T>
__device__ __forceinline__ v16f mfma32(v8s a, v8s b, v16f c);
template <>
__device__ __forceinline__ v16f mfma32<bf16>(v8s a, v8s b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ v16f mfma32<f16>(v8s a, v8s b, v16f c) {
  typedef __attribute__((ext_vector_type(8))) _Float16 v8h;
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, a),
                                                __builtin_bit_cast(v8h, b), c, 0, 0, 0);
}

// MODE 0: forward-style epilogue (bias / ReLU / statistics of the output);
// MODE 1: dgrad-style (addend, producer-BN ReLU mask from bits / values /
// recomputed from xbn, BN backward partials).
template <typename T, int MODE>
__global__ void __launch_bounds__(256, 1) conv_s3_k(IgArgs a, Geo g) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const wl = smem;
  char* const ring = smem + W_BYTES;
  float* const prm = (float*)(smem + W_BYTES + R_BYTES);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  const int G = gridDim.x, b = blockIdx.x;
  const int t0 = (int)((long)b * g.tiles / G), t1 = (int)((long)(b + 1) * g.tiles / G);
  const int ntile = t1 - t0;
  if (ntile <= 0) return;  // (workgroup-uniform)
  const int Qa = g.Qlo + t0 * BM;
  const int halo = g.W1 + 1;  // W + 2: the largest tap shift
  const int Pbase = Qa - halo;  // position of stream index 0

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, a.ybytes, 0x00020000);

  // per-channel epilogue parameters
  if (tid < CH) {
    prm[tid] = a.kshift ? a.kshift[tid] : 0.f;
    prm[CH + tid] = (MODE == 1 && a.mean) ? a.mean[tid] : 0.f;
    prm[2 * CH + tid] = (MODE == 1 && a.mcoef) ? a.mcoef[tid] : 0.f;
    prm[3 * CH + tid] = (MODE == 1 && a.mcoef) ? a.mcoef[CH + tid] : 0.f;
    prm[4 * CH + tid] = (MODE == 0 && a.bias) ? a.bias[tid] : 0.f;
  }
  // weight slab: row R = tap * 64 + cout (128 B), chunk-swizzled by cout
#pragma unroll
  for (int q0 = 0; q0 < 9 * CH / 8; q0 += 4) {
    const int q = q0 + wid;
    const int R = q * 8 + (lane >> 3);
    const int tap = R >> 6, co = R & 63;
    const int off = (co * 9 * CH + tap * CH) * 2 + (((lane & 7) ^ ((co >> 1) & 7)) << 4);
    dma16(wrs, wl + q * 1024, off);
  }
  // one ring block: this wave's 32 of its 128 positions, 4 DMA pieces
  auto load_block = [&](int blk) {
    const int slot = blk % NBLK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = blk * BLK + 32 * wid + 8 * i + (lane >> 3);
      const int po = pix_off(Pbase + s, g, a);
      const int off = po < 0 ? -1 : po + (((lane & 7) ^ ((s >> 1) & 7)) << 4);
      dma16(xrs, ring + (slot * BLK + 32 * wid + 8 * i) * ROWB, off);
    }
  };
  load_block(0);
  load_block(1);
  load_block(2);
  wait_vm<0>();
  __syncthreads();

  // statistics / partials: lane-local sums over this workgroup's positions of
  // channels 8c + k, c = 4i + 2a + hh (the channels this lane owns after the
  // epilogue's swaps)
  float s1[2][2][8], s2[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[i][p][k] = 0.f; s2[i][p][k] = 0.f; }
  const bool want_stats = a.stats != nullptr;
  const int fw = (l32 >> 1) & 7;  // weight-row swizzle of this lane's channel rows

  for (int t = 0; t < ntile; ++t) {
    load_block(2 * t + 3);
    load_block(2 * t + 4);
    const int Q0 = Qa + t * BM;
    // this lane's two output positions (subtile j), their pixel offsets
    int po[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int Q = Q0 + 64 * wid + 32 * j + l32;
      po[j] = Q < g.Qhi ? pix_off(Q, g, a) : -1;
    }
    // dgrad-style operands of this tile (in flight during the MFMAs)
    uint4 ad[2][2][2], xb[2][2][2];
    unsigned mk[2][2][2];
    if constexpr (MODE == 1) {
      const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.addend ? a.addend : a.y), (short)0, a.addend ? a.ybytes : 0, 0x00020000);
      const __amdgpu_buffer_rsrc_t xbrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.xbn ? a.xbn : a.y), (short)0, a.xbn ? a.ybytes : 0, 0x00020000);
      const int mlen = a.mask ? (a.maskbits ? a.ybytes / 16 : a.ybytes) : 0;
      const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.mask ? a.mask : a.y), (short)0, mlen, 0x00020000);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const int c = 4 * i + 2 * p + hh;
            const int off = po[j] < 0 ? -1 : po[j] + c * 16;
            ad[j][i][p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ars, off, 0, 0));
            xb[j][i][p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xbrs, off, 0, 0));
            if (a.maskbits)
              mk[j][i][p] = __builtin_amdgcn_raw_buffer_load_b8(mrs, off < 0 ? -1 : off >> 4, 0, 0);
            else {
              const uint4 m = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(mrs, off, 0, 0));
              // one bit per channel: value > 0
              const Vec<T, 8> mv = __builtin_bit_cast(Vec<T, 8>, m);
              unsigned bits = 0;
#pragma unroll
              for (int k = 0; k < 8; ++k) bits |= ((float)mv.v[k] > 0.f ? 1u : 0u) << k;
              mk[j][i][p] = bits;
            }
          }
    }

    v16f acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // stream index of this wave's first position at tap shift 0
    const int sw0 = t * BM + halo + 64 * wid;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      const int shift = (kh - 1) * g.W1 + (kw - 1);
      const int sb = (sw0 + shift) % RING;  // wave-uniform ring slot of lane 0, subtile 0
      int rowb[2], fx[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        unsigned x = (unsigned)(sb + 32 * j + l32);
        x = min(x, x - (unsigned)RING);  // wrap (x < 2 * RING)
        rowb[j] = (int)x * ROWB;
        fx[j] = (x >> 1) & 7;  // == fx[0]: 32 is a multiple of 16
      }
      const char* wrow = wl + (tap * CH + l32) * ROWB;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = 2 * ks + hh;
        v8s af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *(const v8s*)(wrow + i * 32 * ROWB + ((ch ^ fw) << 4));
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = *(const v8s*)(ring + rowb[j] + ((ch ^ fx[j]) << 4));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma32<T>(af[i], bf[j], acc[i][j]);
      }
    }

    // ---- epilogue: acc[i][j] reg 4g + r = channel 32i + 8g + 4hh + r of
    // position 32j + l32; swap groups (2p, 2p+1) across the lane halves so
    // this lane holds channels 8c .. 8c+7, c = 4i + 2p + hh
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool valid = po[j] >= 0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int c = 4 * i + 2 * p + hh;
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane32_swap(f2u(acc[i][j][8 * p + r]),
                                                             f2u(acc[i][j][8 * p + 4 + r]),
                                                             false, false);
            v[r] = u2f(sw[0]);
            v[4 + r] = u2f(sw[1]);
          }
          const float4* pp = (const float4*)prm;
          Vec<T, 8> ov;
          if constexpr (MODE == 0) {
            if (a.bias || a.relu) {
              const float4 b0 = pp[(4 * CH + 8 * c) / 4], b1 = pp[(4 * CH + 8 * c) / 4 + 1];
              const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                v[k] += bb[k];
                if (a.relu) v[k] = fmaxf(v[k], 0.f);
              }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) ov.v[k] = (T)v[k];
            if (want_stats) {
              const float4 k0 = pp[(8 * c) / 4], k1 = pp[(8 * c) / 4 + 1];
              const float kk[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const float d = valid ? (float)ov.v[k] - kk[k] : 0.f;
                s1[i][p][k] += d;
                s2[i][p][k] += d * d;
              }
            }
          } else {
            const Vec<T, 8> av = __builtin_bit_cast(Vec<T, 8>, ad[j][i][p]);
            const Vec<T, 8> xv = __builtin_bit_cast(Vec<T, 8>, xb[j][i][p]);
            const float4 m0 = pp[(CH + 8 * c) / 4], m1 = pp[(CH + 8 * c) / 4 + 1];
            const float mu[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
            float sc[8], sh[8];
            const bool mrec = a.xbn && !a.mask && a.mcoef;
            if (mrec) {
              const float4 c0 = pp[(2 * CH + 8 * c) / 4], c1 = pp[(2 * CH + 8 * c) / 4 + 1];
              const float4 d0 = pp[(3 * CH + 8 * c) / 4], d1 = pp[(3 * CH + 8 * c) / 4 + 1];
              const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
              const float ds[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) { sc[k] = cs[k]; sh[k] = ds[k]; }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              float x = v[k] + (float)av.v[k];  // zero addend when absent
              if (a.xbn) {
                if (a.mask) x = (mk[j][i][p] >> k) & 1u ? x : 0.f;
                else if (mrec) x = (float)xv.v[k] * sc[k] + sh[k] > 0.f ? x : 0.f;
                if (want_stats && valid) {
                  s1[i][p][k] += x;
                  s2[i][p][k] += x * ((float)xv.v[k] - mu[k]);
                }
              } else if (want_stats && valid) {
                s1[i][p][k] += x;
                s2[i][p][k] += x * x;
              }
              ov.v[k] = (T)x;
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, ov), yrs,
                                                 valid ? po[j] + c * 16 : -1, 0, 0);
        }
    }
    // the blocks issued at the top of this tile (older than its 8 stores)
    // landed for every wave; every wave is done reading blocks 2t, 2t+1
    wait_vm<8>();
    barrier_lds();
  }

  if (!want_stats) return;
  // reduce the lane sums over the 32 lanes of each half (same channels),
  // then over the 4 waves through LDS (the ring is free now), then one
  // atomic add per channel into statistics slot blockIdx % IG_SPREAD
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          s1[i][p][k] += __shfl_xor(s1[i][p][k], o, 64);
          s2[i][p][k] += __shfl_xor(s2[i][p][k], o, 64);
        }
      }
  float* red = (float*)ring;  // [wave][stat][64 channels]
  if (l32 == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int ch = 8 * (4 * i + 2 * p + hh) + k;
          red[(wid * 2 + 0) * CH + ch] = s1[i][p][k];
          red[(wid * 2 + 1) * CH + ch] = s2[i][p][k];
        }
  }
  __syncthreads();
  if (tid < 2 * CH) {
    const int st = tid / CH, ch = tid % CH;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + st) * CH + ch];
    atomicAdd(a.stats + ((long)st * IG_SPREAD + b % IG_SPREAD) * CH + ch, v);
  }
}

}  // namespace s3

// Geometry the streaming kernel computes (see file comment).
static bool s3_geometry(int C, int Ncol, int KH, int KW, int sh, int sw, int pt, int pl, int H,
                        int W, int OH, int OW, int YH, int YW, int ys, int ldy) {
  return C == s3::CH && Ncol == s3::CH && KH == 3 && KW == 3 && sh == 1 && sw == 1 && pt == 1 &&
         pl == 1 && OH == H && OW == W && YH == OH && YW == OW && ys == 1 && ldy == Ncol &&
         2 * (W + 2) <= s3::BLK;
}

static int s3_grid_force = 0;  // test hook: fixed grid size (0 = one workgroup per CU)

static int s3_grid(int tiles) {
  if (s3_grid_force > 0) return tiles < s3_grid_force ? tiles : s3_grid_force;
  static std::once_flag once;
  static int cus = 256;
  std::call_once(once, [] {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
      int n = 0;
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
          n > 0)
        cus = n;
    }
  });
  return tiles < cus ? tiles : cus;
}

bool conv_s3_fits(const IgArgs& a) {
  return s3_geometry(a.C, a.Ncol, a.KH, a.KW, a.sh, a.sw, a.pt, a.pl, a.H, a.W, a.OH, a.OW, a.YH,
                     a.YW, a.ys, a.ldy) &&
         a.xbytes > 0 && a.wbytes > 0 && a.ybytes > 0 && !a.zfill && !a.c8 &&
         (long)a.N * (a.H + 1) * (a.W + 1) + 4L * s3::BLK < (1L << 31) &&
         !(a.relu && (a.addend || a.xbn));
}

// Launch for an igemm_k-style argument block (forward / stride-1 dgrad with
// flipped weights) whose geometry conv_s3_fits.
hipError_t launch_conv_s3(int dtype, const IgArgs& a, hipStream_t stream) {
  if (!conv_s3_fits(a)) return hipErrorInvalidValue;
  s3::Geo g;
  g.W1 = a.W + 1;
  g.H1 = a.H + 1;
  g.fw1 = FastDiv(g.W1);
  g.fh1 = FastDiv(g.H1);
  g.Qlo = g.W1;
  g.Qhi = a.N * g.H1 * g.W1;
  g.tiles = (g.Qhi - g.Qlo + s3::BM - 1) / s3::BM;
  const int grid = s3_grid(g.tiles);
  const bool dg = a.addend || a.xbn;
  if (dtype == BF16) {
    if (dg) hipLaunchKernelGGL((s3::conv_s3_k<bf16, 1>), dim3(grid), dim3(256), 0, stream, a, g);
    else hipLaunchKernelGGL((s3::conv_s3_k<bf16, 0>), dim3(grid), dim3(256), 0, stream, a, g);
  } else if (dtype == F16) {
    if (dg) hipLaunchKernelGGL((s3::conv_s3_k<f16, 1>), dim3(grid), dim3(256), 0, stream, a, g);
    else hipLaunchKernelGGL((s3::conv_s3_k<f16, 0>), dim3(grid), dim3(256), 0, stream, a, g);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kfb

KFB_API int kfb_conv_s3_applicable(int C, int Ncol, int KH, int KW, int sh, int sw, int pt, int pl,
                                   int H, int W, int OH, int OW) {
  return kfb::s3_geometry(C, Ncol, KH, KW, sh, sw, pt, pl, H, W, OH, OW, OH, OW, 1, Ncol) ? 1 : 0;
}

// Test hook: run the streaming kernel on at most `grid` workgroups (0 = one
// per CU), so small problems exercise many tiles (and ring wraps) per
// workgroup.
KFB_API void kfb_conv_s3_set_grid(int grid) { kfb::s3_grid_force = grid > 0 ? grid : 0; }
