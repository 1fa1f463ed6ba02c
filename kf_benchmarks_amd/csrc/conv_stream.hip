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
constexpr int LDS_BYTES = W_BYTES + R_BYTES;  // 155648

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
// a pad position / outside the batch (branch-free: selects only)
__device__ __forceinline__ int pix_off(int P, const Geo& g, const IgArgs& a) {
  const int Pc = P < 0 ? 0 : P;
  const int r = g.fw1.div(Pc), c = Pc - r * g.W1;
  const int img = g.fh1.div(r), rr = r - img * g.H1;
  const int off = ((img * a.H + rr - 1) * a.W + c - 1) * ROWB;
  return (P < 0 || c == 0 || rr == 0 || img >= a.N) ? -1 : off;
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

// Epilogue variants (compile time, so the epilogue is branch-free and can be
// scheduled between the next tile's MFMAs):
//   EPI_STATS : forward, BN statistics of the output (sum (y-K), sum (y-K)^2)
//   EPI_ACT   : forward, y = act(conv + bias) (bias / ReLU), no statistics
//   EPI_DGRAD : dX = conv + addend, masked by the producer BN's ReLU
//               (MASK: 0 none, 1 bit mask, 2 mask values, 3 recomputed from
//               xbn * scale + shift), BN backward partials sum dX,
//               sum dX * (xbn - mean) (sum dX^2 without xbn)
enum { EPI_STATS = 0, EPI_ACT = 1, EPI_DGRAD = 2 };

// chunk q of a tile's epilogue (q = 4j + 2i + p): position subtile j, channel
// subtile i, register-group pair p -> this lane's 16-byte chunk c = 4i + 2p + hh
// of position 32j + l32
template <int EPI>
__host__ __device__ constexpr int chunk_tap(int q) {
  // tap of the next tile at which chunk q is finished: from tap 1 on; the
  // dgrad form loads the operands of position subtile j = 0 at the tile
  // start (chunks 0-3 at taps 2-3) and those of j = 1 after tap 1 (chunks
  // 4-7 at taps 5-8), each subtile in its own registers
  return EPI == EPI_DGRAD ? (q < 4 ? 2 + (q >> 1) : q + 1) : q + 1;
}
template <int EPI>
__host__ __device__ constexpr int load_tap(int j) {
  return j == 0 ? -1 : 1;  // dgrad operands of subtile j issued after this tap
}

template <typename T, int EPI, int MASK>
__global__ void __launch_bounds__(256, 1) conv_s3_k(IgArgs a, Geo g) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const wl = smem;
  char* const ring = smem + W_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  const int G = gridDim.x, b = blockIdx.x;
  const int t0 = (int)((long)b * g.tiles / G), t1 = (int)((long)(b + 1) * g.tiles / G);
  const int ntile = t1 - t0;
  if (ntile <= 0) {  // (workgroup-uniform) nothing to compute; still arrives
    bn_tail(a, (int*)smem);
    return;
  }
  const int Qa = g.Qlo + t0 * BM;
  const int halo = g.W1 + 1;    // W + 2: the largest tap shift
  const int Pbase = Qa - halo;  // position of stream index 0

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, a.ybytes, 0x00020000);
  // dgrad-form operands (a null operand gets a zero-size range: reads 0)
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.addend ? a.addend : a.y), (short)0, a.addend ? a.ybytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xbrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.xbn ? a.xbn : a.y), (short)0, a.xbn ? a.ybytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.mask ? a.mask : a.y), (short)0,
      a.mask ? (MASK == 1 ? a.ybytes / 16 : a.ybytes) : 0, 0x00020000);
  const unsigned xbn_mask = a.xbn != nullptr ? ~0u : 0u;  // (wave-uniform)
  const float relu_floor = a.relu ? 0.f : -INFINITY;

  // per-lane channel parameters of the 32 channels this lane finishes:
  // 8c + k, c = 4i + 2p + hh
  float pa[2][2][8], pb[2][2][8], pc[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int ch = 8 * (4 * i + 2 * p + hh) + k;
        if constexpr (EPI == EPI_STATS) pa[i][p][k] = a.kshift ? a.kshift[ch] : 0.f;
        if constexpr (EPI == EPI_ACT) pa[i][p][k] = a.bias ? a.bias[ch] : 0.f;
        if constexpr (EPI == EPI_DGRAD) pa[i][p][k] = a.mean ? a.mean[ch] : 0.f;
        if constexpr (EPI == EPI_DGRAD && MASK == 3) {
          pb[i][p][k] = a.mcoef[ch];
          pc[i][p][k] = a.mcoef[CH + ch];
        }
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

  float s1[2][2][8], s2[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[i][p][k] = 0.f; s2[i][p][k] = 0.f; }
  const int fw = (l32 >> 1) & 7;  // weight-row swizzle of this lane's channel rows
  const char* const wlane = wl + l32 * ROWB;

  // dgrad-form operands of the tile being finished: [position subtile j][q & 3]
  uint4 ad[2][4], xb[2][4];
  unsigned mk[2][4];
  uint4 mv[2][4];
  auto epi_loads = [&](const int (&po)[2], int j) {
    if constexpr (EPI == EPI_DGRAD) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int i = qq >> 1, p = qq & 1;
        const int c = 4 * i + 2 * p + hh;
        const int off = po[j] < 0 ? -1 : po[j] + c * 16;
        ad[j][qq] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ars, off, 0, 0));
        xb[j][qq] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xbrs, off, 0, 0));
        if constexpr (MASK == 1)
          mk[j][qq] = __builtin_amdgcn_raw_buffer_load_b8(mrs, off < 0 ? -1 : off >> 4, 0, 0);
        if constexpr (MASK == 2)
          mv[j][qq] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(mrs, off, 0, 0));
      }
    }
  };

  // finishes chunk q of the tile held in acc (positions po)
  auto epi_chunk = [&](int q, const v16f (&acc)[2][2], const int (&po)[2]) {
    const int j = q >> 2, i = (q >> 1) & 1, p = q & 1;
    const int c = 4 * i + 2 * p + hh;
    const bool valid = po[j] >= 0;
    // selects as bit masks (a ?: on per-lane data becomes an exec-mask
    // branch, which would split the MFMA block the epilogue is scheduled in)
    const unsigned vmask = valid ? ~0u : 0u;
    auto keep_if = [](float x, unsigned m) { return u2f(f2u(x) & m); };
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const auto sw = __builtin_amdgcn_permlane32_swap(f2u(acc[i][j][8 * p + r]),
                                                       f2u(acc[i][j][8 * p + 4 + r]), false,
                                                       false);
      v[r] = u2f(sw[0]);
      v[4 + r] = u2f(sw[1]);
    }
    Vec<T, 8> ov;
    if constexpr (EPI == EPI_STATS) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ov.v[k] = (T)v[k];
        const float d = keep_if(v[k] - pa[i][p][k], vmask);
        s1[i][p][k] += d;
        s2[i][p][k] = fmaf(d, d, s2[i][p][k]);
      }
    } else if constexpr (EPI == EPI_ACT) {
#pragma unroll
      for (int k = 0; k < 8; ++k) ov.v[k] = (T)fmaxf(v[k] + pa[i][p][k], relu_floor);
    } else {
      const Vec<T, 8> av = __builtin_bit_cast(Vec<T, 8>, ad[q >> 2][q & 3]);
      const Vec<T, 8> xv = __builtin_bit_cast(Vec<T, 8>, xb[q >> 2][q & 3]);
      const Vec<T, 8> mvv = __builtin_bit_cast(Vec<T, 8>, mv[q >> 2][q & 3]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float x = v[k] + (float)av.v[k];
        if constexpr (MASK == 1) x = keep_if(x, 0u - ((mk[q >> 2][q & 3] >> k) & 1u));
        if constexpr (MASK == 2) x = keep_if(x, 0u - (unsigned)((float)mvv.v[k] > 0.f));
        if constexpr (MASK == 3)
          x = keep_if(x, 0u - (unsigned)((float)xv.v[k] * pb[i][p][k] + pc[i][p][k] > 0.f));
        const float xd = keep_if(x, vmask);
        s1[i][p][k] += xd;
        // (xbn - mean) with xbn, else x (sum of squares); xbn reads 0 when absent
        const float dx = (float)xv.v[k] - pa[i][p][k];
        s2[i][p][k] = fmaf(xd, u2f((f2u(dx) & xbn_mask) | (f2u(x) & ~xbn_mask)), s2[i][p][k]);
        ov.v[k] = (T)x;
      }
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, ov), yrs,
                                           valid ? po[j] + c * 16 : -1, 0, 0);
  };

  int po_prev[2] = {-1, -1};
  v16f accA[2][2], accB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) { accA[i][j][r] = 0.f; accB[i][j][r] = 0.f; }

  // one tile into acc, finishing the previous tile (accp, po_prev) between its MFMAs
  auto tile = [&](int t, v16f (&acc)[2][2], const v16f (&accp)[2][2]) {
    epi_loads(po_prev, 0);  // (older than the DMAs below: waiting for them skips those)
    load_block(2 * t + 3);
    load_block(2 * t + 4);
    const int Q0 = Qa + t * BM;
    int po[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int Q = Q0 + 64 * wid + 32 * j + l32;
      po[j] = Q < g.Qhi ? pix_off(Q, g, a) : -1;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // stream index of this wave's first position at tap shift 0
    const int sw0 = t * BM + halo + 64 * wid;
    // operand fragments are double-buffered by groups of KG k steps (16 deep
    // each): the reads of group gi + 1 are issued before the MFMAs of group
    // gi.  KG = 4 (a whole tap) for the forward forms; the dgrad form holds
    // its epilogue operands in registers too and uses half taps
    constexpr int KG = EPI == EPI_DGRAD ? 2 : 4;
    constexpr int NG = 36 / KG;
    v8s fa[2][KG][2], fb[2][KG][2];  // [buffer][k step][i / j]
    auto frags = [&](int gi, v8s (&af)[KG][2], v8s (&bf)[KG][2]) {
      const int tap = gi * KG / 4, ks0 = gi * KG % 4;
      const int kh = tap / 3, kw = tap % 3;
      const int sb = (sw0 + (kh - 1) * g.W1 + (kw - 1)) % RING;
      unsigned x0 = (unsigned)(sb + l32), x1 = x0 + 32u;
      x0 = min(x0, x0 - (unsigned)RING);
      x1 = min(x1, x1 - (unsigned)RING);
      const int fx = (x0 >> 1) & 7;  // same for x1 (32 is a multiple of 16)
#pragma unroll
      for (int kk = 0; kk < KG; ++kk) {
        const int ks = ks0 + kk;
        const int cw = ((2 * ks + hh) ^ fw) << 4, cx = ((2 * ks + hh) ^ fx) << 4;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[kk][i] = *(const v8s*)(wlane + (tap * CH + 32 * i) * ROWB + cw);
        bf[kk][0] = *(const v8s*)(ring + (int)x0 * ROWB + cx);
        bf[kk][1] = *(const v8s*)(ring + (int)x1 * ROWB + cx);
      }
    };
    frags(0, fa[0], fb[0]);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      const int cb = gi & 1;
      if (gi + 1 < NG) frags(gi + 1, fa[cb ^ 1], fb[cb ^ 1]);
#pragma unroll
      for (int kk = 0; kk < KG; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = mfma32<T>(fa[cb][kk][i], fb[cb][kk][j], acc[i][j]);
      if ((gi + 1) * KG % 4 == 0) {  // end of a tap
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (chunk_tap<EPI>(q) == (gi * KG / 4)) epi_chunk(q, accp, po_prev);
        if (load_tap<EPI>(1) == gi * KG / 4) epi_loads(po_prev, 1);
      }
    }
    po_prev[0] = po[0];
    po_prev[1] = po[1];
    // this tile's DMAs (older than the previous tile's 8 stores) landed for
    // every wave; every wave is done reading blocks 2t, 2t+1
    wait_vm<8>();
    barrier_lds();
  };

  for (int t = 0; t < ntile; t += 2) {
    tile(t, accA, accB);
    if (t + 1 < ntile) tile(t + 1, accB, accA);
  }
  // the last tile's epilogue
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    epi_loads(po_prev, j);
    if (ntile & 1) {
#pragma unroll
      for (int q = 4 * j; q < 4 * j + 4; ++q) epi_chunk(q, accA, po_prev);
    } else {
#pragma unroll
      for (int q = 4 * j; q < 4 * j + 4; ++q) epi_chunk(q, accB, po_prev);
    }
  }

  if (EPI == EPI_ACT || !a.stats) return;  // (no statistics: no finalize either)
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
  bn_tail(a, (int*)smem);
}

}  // namespace s3

// ---------------------------------------------------------------------------
// Streaming weight gradient of the same 3x3 64 -> 64 conv:
//   dW[co][tap][ci] = sum_Q dy[Q][co] * x[Q + shift(tap)][ci]
// over the output positions Q of the padded position space (dy is zero at
// pad positions: the DMA loads zeros there).  Each persistent workgroup owns
// a run of 256-position tiles, streams x through the same 640-position ring
// as the forward kernel and dy tiles through two 32 KB stages, and keeps its
// whole partial dW (64 x 576 fp32) in accumulators: wave w computes output
// channels 32 (w & 1) .. +32 x input channels 32 (w >> 1) .. +32 for all 9
// taps (nine 32x32 tiles, 144 AGPRs).  The reduction index (positions) is
// the MFMA K: both operands are read column-major with ds_read_b64_tr_b16
// from [position][channel] images whose 16-byte chunks are swizzled by
// c ^ 4 ((p >> 1) & 1), which puts any 4 consecutive positions in 4 distinct
// 64-byte quarters of the bank row (every transposed read conflict-free).
// The workgroup's partial dW goes to its slab; wgrad_reduce_k-style fixed-
// order summation folds the slabs into dW (deterministic).
namespace s3w {

using s3::CH;
using s3::BM;
using s3::BLK;
using s3::NBLK;
using s3::RING;
using s3::ROWB;
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef s3::v8s v8s;
typedef s3::v16f v16f;

constexpr int R_BYTES = RING * ROWB;        // 81920
constexpr int D_BYTES = BM * ROWB;          // 32768 per dy stage
constexpr int LDS_BYTES = R_BYTES + 2 * D_BYTES;  // 147456

__device__ __forceinline__ int swz(int pos, int chunk) {
  return pos * ROWB + ((chunk ^ (((pos >> 1) & 1) << 2)) << 4);
}

__device__ __forceinline__ v4s read_tr(const char* p) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}

template <typename T>
__global__ void __launch_bounds__(256, 1) wgrad_s3_k(const void* dyp, const void* xp,
                                                     float* __restrict__ slab, int N, int H,
                                                     int W, int dybytes, int xbytes, s3::Geo g) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const ring = smem;
  char* const dys = smem + R_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  const int G = gridDim.x, b = blockIdx.x;
  const int t0 = (int)((long)b * g.tiles / G), t1 = (int)((long)(b + 1) * g.tiles / G);
  const int ntile = t1 - t0;
  const int Qa = g.Qlo + t0 * BM;
  const int halo = g.W1 + 1;
  const int Pbase = Qa - halo;
  IgArgs a{};  // pix_off reads N, H, W
  a.N = N;
  a.H = H;
  a.W = W;

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xp, (short)0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void*)dyp, (short)0, dybytes, 0x00020000);

  auto load_block = [&](int blk) {
    const int slot = blk % NBLK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int sp = blk * BLK + 32 * wid + 8 * i + (lane >> 3);
      const int po = s3::pix_off(Pbase + sp, g, a);
      const int off = po < 0 ? -1 : po + (((lane & 7) ^ (((sp >> 1) & 1) << 2)) << 4);
      s3::dma16(xrs, ring + (slot * BLK + 32 * wid + 8 * i) * ROWB, off);
    }
  };
  auto load_dy = [&](int t, int stage) {
    const int Q0 = Qa + t * BM;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int u = 64 * wid + 8 * i + (lane >> 3);
      const int Q = Q0 + u;
      const int po = Q < g.Qhi ? s3::pix_off(Q, g, a) : -1;
      const int off = po < 0 ? -1 : po + (((lane & 7) ^ (((u >> 1) & 1) << 2)) << 4);
      s3::dma16(drs, dys + stage * D_BYTES + (64 * wid + 8 * i) * ROWB, off);
    }
  };

  v16f acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;

  if (ntile > 0) {
    load_block(0);
    load_block(1);
    load_block(2);
    load_dy(0, 0);
    s3::wait_vm<0>();
    __syncthreads();
  }
  // this lane's part of a transposed read: row q of a 4-row block, columns
  // 4p .. 4p+3 of its 16-column group gq
  const int q = (lane & 15) >> 2, pq = lane & 3, gq = (lane >> 4) & 1;
  const int co_col = 32 * (wid & 1) + 16 * gq + 4 * pq;  // dy column (output channel)
  const int ci_col = 32 * (wid >> 1) + 16 * gq + 4 * pq;  // x column (input channel)
  const int co_chunk = co_col >> 3, co_half = (co_col & 7) * 2;   // byte offset in chunk
  const int ci_chunk = ci_col >> 3, ci_half = (ci_col & 7) * 2;

  for (int t = 0; t < ntile; ++t) {
    const int st = t & 1;
    load_block(2 * t + 3);
    load_block(2 * t + 4);
    if (t + 1 < ntile) load_dy(t + 1, st ^ 1);
    const char* dyb = dys + st * D_BYTES;
    const int sw0 = t * BM + halo;  // stream index of the tile's position 0
#pragma unroll 2
    for (int ks = 0; ks < BM / 16; ++ks) {
      // A: dy^T, rows = positions 16 ks + 8 hh + 4 e + q
      v8s af;
      {
        const int u0 = 16 * ks + 8 * hh + q;
        const v4s lo = read_tr(dyb + swz(u0, co_chunk) + co_half);
        const v4s hi = read_tr(dyb + swz(u0 + 4, co_chunk) + co_half);
        af = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3;
        const int sb = (sw0 + 16 * ks + (kh - 1) * g.W1 + (kw - 1)) % RING;  // wave-uniform
        unsigned x0 = (unsigned)(sb + 8 * hh + q), x1 = x0 + 4u;
        x0 = min(x0, x0 - (unsigned)RING);
        x1 = min(x1, x1 - (unsigned)RING);
        const v4s lo = read_tr(ring + swz((int)x0, ci_chunk) + ci_half);
        const v4s hi = read_tr(ring + swz((int)x1, ci_chunk) + ci_half);
        const v8s bf = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[tap] = s3::mfma32<T>(af, bf, acc[tap]);
      }
    }
    // this tile's x blocks and the next tile's dy stage landed for every
    // wave; every wave is done reading blocks 2t, 2t+1 and dy stage st
    s3::wait_vm<0>();
    s3::barrier_lds();
  }

  // partial dW -> slab[b][co][tap][ci] (acc[tap] reg 4gg + r = row co =
  // 32 (w & 1) + 8 gg + 4 hh + r, column ci = 32 (w >> 1) + l32)
  float* const out = slab + (long)b * CH * 9 * CH;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * (wid & 1) + 8 * (r >> 2) + 4 * hh + (r & 3);
      out[(co * 9 + tap) * CH + 32 * (wid >> 1) + l32] = acc[tap][r];
    }
}

}  // namespace s3w

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
         !(a.relu && (a.addend || a.xbn)) && !(a.stats && !(a.addend || a.xbn) && (a.bias || a.relu)) &&
         // producer-BN ReLU mask: none or the bit mask (mask values / the
         // recomputed mask stay on the tiled kernels)
         !(a.xbn && ((a.mask && !a.maskbits) || (!a.mask && a.mcoef)));
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
  // epilogue variant and mask source (see conv_s3_k)
  const int epi = dg ? s3::EPI_DGRAD : (a.stats ? s3::EPI_STATS : s3::EPI_ACT);
  int mask = 0;
  if (dg && a.xbn) {
    if (a.mask) mask = a.maskbits ? 1 : 2;
    else if (a.mcoef) mask = 3;
  }
  if (epi == s3::EPI_STATS && (a.bias || a.relu)) return hipErrorInvalidValue;
#define S3_LAUNCH_CASES(T)                                                                      \
  switch (epi * 4 + mask) {                                                                   \
    case 0: hipLaunchKernelGGL((s3::conv_s3_k<T, 0, 0>), dim3(grid), dim3(256), 0, stream, a, g); break; \
    case 4: hipLaunchKernelGGL((s3::conv_s3_k<T, 1, 0>), dim3(grid), dim3(256), 0, stream, a, g); break; \
    case 8: hipLaunchKernelGGL((s3::conv_s3_k<T, 2, 0>), dim3(grid), dim3(256), 0, stream, a, g); break; \
    case 9: hipLaunchKernelGGL((s3::conv_s3_k<T, 2, 1>), dim3(grid), dim3(256), 0, stream, a, g); break; \
    default: return hipErrorInvalidValue;                                                      \
  }
  if (dtype == BF16) {
    S3_LAUNCH_CASES(bf16)
  } else if (dtype == F16) {
    S3_LAUNCH_CASES(f16)
  } else {
    return hipErrorInvalidValue;
  }
#undef S3_LAUNCH_CASES
  return hipGetLastError();
}

}  // namespace kfb

namespace kfb {
namespace s3w {
// dw[i] += sum_s slab[s][i] in split order (float4 per thread)
__global__ void __launch_bounds__(256) reduce_k(const float4* __restrict__ slab,
                                                float4* __restrict__ dw, int n4, int nsplit) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 acc = dw[i];
  int sp = 0;
  for (; sp + 4 <= nsplit; sp += 4) {
    const float4 v0 = slab[(long)sp * n4 + i], v1 = slab[(long)(sp + 1) * n4 + i];
    const float4 v2 = slab[(long)(sp + 2) * n4 + i], v3 = slab[(long)(sp + 3) * n4 + i];
    acc.x += (v0.x + v1.x) + (v2.x + v3.x);
    acc.y += (v0.y + v1.y) + (v2.y + v3.y);
    acc.z += (v0.z + v1.z) + (v2.z + v3.z);
    acc.w += (v0.w + v1.w) + (v2.w + v3.w);
  }
  for (; sp < nsplit; ++sp) {
    const float4 v = slab[(long)sp * n4 + i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  dw[i] = acc;
}
}  // namespace s3w

static bool s3w_geo(int N, int H, int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                    int pt, int pl, int Ncol, s3::Geo* g) {
  if (!s3_geometry(C, Ncol, KH, KW, sh, sw, pt, pl, H, W, OH, OW, OH, OW, 1, Ncol)) return false;
  if ((long)N * (H + 1) * (W + 1) + 4L * s3::BLK >= (1L << 31)) return false;
  if ((long)N * H * W * C * 2 >= (1L << 31)) return false;
  g->W1 = W + 1;
  g->H1 = H + 1;
  g->fw1 = FastDiv(g->W1);
  g->fh1 = FastDiv(g->H1);
  g->Qlo = g->W1;
  g->Qhi = N * g->H1 * g->W1;
  g->tiles = (g->Qhi - g->Qlo + s3::BM - 1) / s3::BM;
  return true;
}

// Splits (= workgroups, one partial dW slab each) of the streaming wgrad, or
// 0 off its geometry.
int wgrad_s3_splits(int N, int H, int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                    int pt, int pl, int Ncol) {
  s3::Geo g;
  if (!s3w_geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol, &g)) return 0;
  return s3_grid(g.tiles);
}

hipError_t launch_wgrad_s3(int dtype, const void* dy, const void* x, float* dw, int N, int H,
                           int W, int C, int OH, int OW, int KH, int KW, int sh, int sw, int pt,
                           int pl, int Ncol, float* slab, long slab_elems, hipStream_t stream) {
  s3::Geo g;
  if (!s3w_geo(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol, &g)) return hipErrorInvalidValue;
  const int grid = s3_grid(g.tiles);
  const long per = (long)s3::CH * 9 * s3::CH;
  if (!slab || (long)grid * per > slab_elems) return hipErrorInvalidValue;
  const int bytes = (int)((long)N * H * W * C * 2);
  if (dtype == BF16)
    hipLaunchKernelGGL((s3w::wgrad_s3_k<bf16>), dim3(grid), dim3(256), 0, stream, dy, x, slab, N,
                       H, W, bytes, bytes, g);
  else if (dtype == F16)
    hipLaunchKernelGGL((s3w::wgrad_s3_k<f16>), dim3(grid), dim3(256), 0, stream, dy, x, slab, N,
                       H, W, bytes, bytes, g);
  else
    return hipErrorInvalidValue;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int n4 = (int)(per / 4);
  hipLaunchKernelGGL(s3w::reduce_k, dim3((n4 + 255) / 256), dim3(256), 0, stream,
                     (const float4*)slab, (float4*)dw, n4, grid);
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
