// Streaming 1x1 convolution for the memory-bound pointwise layers of the
// ResNet bottleneck (tcb/models/resnet_model.py:306-328): the expanding
// conv c / projection shortcut forward (K -> 4K channels, K = 64 .. 512,
// with the consuming BN's statistics) and conv a's data gradient
// dX[4K] = dY[K] W (with the producer BN's fused backward epilogue:
// residual addend, ReLU bit mask, backward partial sums).
//
// These GEMMs have K <= 512 and outputs 4x wider than their inputs: nearly
// all their time is moving activations, so the kernel is a streaming copy
// with a small MFMA inside, not a tiled GEMM:
//
//  * persistent 256-thread workgroups, one per CU; workgroup r owns an
//    output-channel slice of NS = 4 * WCH channels and a contiguous run of
//    32-pixel tiles (the slices of one pixel run sit on one XCD, so the
//    pixel rows they share are read from HBM once, into that XCD's L2);
//  * each wave keeps its WCH x K weight slice in VGPRs for the whole launch
//    (32 .. 128 registers of MFMA A fragments), so LDS holds only the ring;
//  * every operand of a tile streams into a (D+1)-stage LDS ring by LDS-DMA,
//    D tiles ahead: the pixel rows (32 x K) and, for the data gradient, the
//    epilogue operands (addend, the BN input x_bn, ReLU bits) of the slice;
//    a tile's stores may stay in flight for D tiles (the counted wait covers
//    only the DMAs of the next tile and what came before them); one barrier
//    per tile;
//  * apply form (EPI_APPLY): the conv whose output only a residual BN + ReLU
//    consumes is computed twice - once for the BN statistics with its stores
//    dropped (IgArgs::ybytes 0), once here with the BN apply, residual add and
//    ReLU in the epilogue (the residual streams through the ring like the
//    data gradient's addend); y itself is stored from this pass.  At 56x56
//    64 -> 256 that replaces writing y (411 MB) in one pass and reading it
//    back (411 MB) in the next by a second read of x (103 MB);
//  * the waves finish their WCH x 32 accumulators from registers:
//    v_permlane32_swap pairs give each lane 8 consecutive channels of one
//    pixel, whose epilogue operands it reads from the ring (chunk-swizzled
//    rows: conflict-free) and whose 16 bytes it stores directly; BN
//    statistics / backward partials accumulate per lane across the tiles.
#include "common.h"
#include "igemm_args.h"

#include <cstdlib>
#include <mutex>

namespace kfb {
namespace s1 {

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(16))) float v16f;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u_t;

constexpr int BMP = 32;              // pixels per tile
constexpr int LDS_CAP = 160 * 1024;  // per CU

enum { EPI_STATS = 0, EPI_APPLY = 1, EPI_DGRAD = 2 };

// per input-channel count K: WCH channels per wave (4 waves along channels);
// WPC workgroups per CU share its LDS; DU: the dual-BN data gradient (a third
// epilogue operand, the second BN's input)
template <int K, int EPI, int WPC, bool DU = false>
struct Cfg {
  static constexpr int WCH = K <= 128 ? 64 : 32;
  static constexpr int NS = 4 * WCH;            // channels per workgroup
  static constexpr int CT = WCH / 32;           // 32-channel MFMA tiles per wave
  static constexpr int KS = K / 16;             // 32x32x16 k-steps
  static constexpr int XROW = 2 * K;            // bytes per pixel row of x
  static constexpr int XB = BMP * XROW;         // x tile
  static constexpr int YROW = 2 * NS;           // bytes per pixel row of the slice
  static constexpr int YB = BMP * YROW;         // one epilogue operand tile
  static constexpr int MB = BMP * NS / 8;       // ReLU bits tile
  // (an LDS-DMA writes 4 bytes per lane even for narrower loads: the bits
  // go by 4-byte DMAs, one 256-byte piece per wave; NS = 128 leaves two
  // pieces unused)
  static constexpr int MBA = 1024;              // bits area of a stage
  static constexpr int XD = XB / 4096;          // x DMAs per wave (1 KB each)
  static constexpr int YD = YB / 4096;          // per epilogue operand per wave
  static constexpr bool DG = EPI == EPI_DGRAD;
  static constexpr bool AP = EPI == EPI_APPLY;
  static constexpr int NY = DU ? 3 : 2;         // dgrad operand tiles (addend, x_bn[, x_bn2])
  static constexpr int MOFF = XB + NY * YB;      // the ReLU bits' offset in a dgrad stage
  static constexpr int STB = XB + (DG ? NY * YB + MBA : AP ? YB : 0);  // ring stage
  static constexpr int DMAS = XD + (DG ? NY * YD + 1 : AP ? YD : 0);  // DMAs per wave per tile
  // stores per lane per tile (16-byte y / out stores, out's ReLU-bit bytes;
  // the apply form issues all three even when y / the bits are not kept)
  static constexpr int ST = (AP ? 3 : 1) * 2 * CT;
  // ring stages: what LDS holds, at most 7, and few enough that the counted
  // wait below fits vmcnt (< 64)
  // y staged through LDS (STAGED): each wave writes its 32-pixel x WCH-channel
  // tile into a private region, reads it back as whole 128-byte (WCH 64) /
  // 64-byte (WCH 32) row pieces and stores those: the per-lane 16-byte pieces
  // of 32 pixel rows per store instruction cap the write stream at ~3.1 TB/s,
  // full-line pieces reach ~5.5 (scripts/probes/s1store.hip); where the
  // staging area leaves at least two ring stages (not the apply form)
  static constexpr int STG = 4 * BMP * WCH * 2;
  static constexpr int NSTS = (LDS_CAP / WPC - STG) / STB;
  static constexpr bool STAGED = !AP && NSTS >= 2;
  static constexpr int NST0 = STAGED ? NSTS : LDS_CAP / WPC / STB;
  static constexpr int NSTV = (63 + DMAS) / (ST + DMAS) + 1;
  static constexpr int NST = NST0 < NSTV ? (NST0 > 7 ? 7 : NST0) : (NSTV > 7 ? 7 : NSTV);
  static constexpr int D = NST - 1;             // prefetch distance (tiles)
  static constexpr int WAIT = ST * D + (D - 1) * DMAS;
  static_assert(XD >= 1 && (!(DG || AP) || YD >= 1), "tile split");
  static_assert(MB <= MBA, "bits area");
  static_assert(D >= 1 && WAIT < 64, "pipeline depth");
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
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, void* lds, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4,
                                           off, 0, 0, 0);
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

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(unsigned long)((__attribute__((address_space(3))) const void*)p);
}

// x rows: 16-byte chunk c of pixel row p sits at physical chunk c ^ xsw(p)
// (128-byte rows: two rows per 256-byte bank row; longer rows: one)
template <int K>
__device__ __forceinline__ int xsw(int p) {
  return K == 64 ? (p >> 1) & 7 : p & 15;
}

// MASK (EPI_DGRAD): 0 none, 1 the producer BN's ReLU bit mask, 2 the bit mask
// of a dual-BN output y = relu(bn(x) + bn2(x2)): also bn2's backward partial
// sum y'(x2 - mean2) into IgArgs::stats2 (kfb_conv_s1_dgrad_dual).  FULL: every
// 32-pixel tile is whole (M % 32 == 0, every ResNet batch size that is a
// multiple of 32 / 8 / 2 at 56 / 28 / 14), so the per-element pixel masks of
// the statistics fold away
template <typename T, int K, int EPI, int MASK, int WPC, bool FULL = false>
__global__ void __launch_bounds__(256, WPC) conv_s1_k(IgArgs a, int tiles, int nsl) {
  constexpr bool DU = MASK == 2;
  using C = Cfg<K, EPI, WPC, DU>;
  constexpr int NS = C::NS, CT = C::CT, KS = C::KS, D = C::D, NST = C::NST;
  constexpr int STB = C::STB;
  __shared__ __attribute__((aligned(16))) char ring[NST * STB + (C::STAGED ? C::STG : 0)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  // this wave's staging rows (STAGED): WCH * 2 bytes per pixel, 16-byte chunk
  // j of row r at j ^ sgz(r) (8 lanes of one ds_write / ds_read phase hit 8
  // distinct 16-byte bank groups)
  constexpr int SROW = C::WCH * 2;
  const unsigned stg = lds_addr(ring + NST * STB) + (unsigned)(wid * BMP * SROW);
  auto sgz = [](int r) { return SROW == 128 ? (r & 7) : ((r >> 1) & 3); };
  // XCD-aware placement: r runs over the workgroups of one XCD first
  // (dispatch round-robins blockIdx over the 8 XCDs); the nsl slices of a
  // pixel group are consecutive r
  const int G = gridDim.x, b = blockIdx.x;
  const int r = (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b;
  const int slice = r % nsl, group = r / nsl, ng = G / nsl;
  const int ns0 = slice * NS;
  const int t0 = (int)((long)group * tiles / ng), t1 = (int)((long)(group + 1) * tiles / ng);
  const int ntile = t1 - t0;

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, a.ybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.addend ? a.addend : a.y), (short)0,
      a.addend ? (a.out ? a.outbytes : a.ybytes) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t xbrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.xbn ? a.xbn : a.y), (short)0, a.xbn ? a.ybytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.mask ? a.mask : a.y), (short)0, (a.mask && MASK >= 1) ? a.ybytes / 16 : 0,
      0x00020000);
  const __amdgpu_buffer_rsrc_t x2rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.xbn2 ? a.xbn2 : a.y), (short)0, (DU && a.xbn2) ? a.ybytes : 0, 0x00020000);
  // (the bit mask always comes with the BN input: MASK >= 1 selects x - mean)
  const unsigned xbn_mask = (MASK >= 1 || a.xbn != nullptr) ? ~0u : 0u;
  const int ldy2 = a.Ncol * 2;
  // apply form: out (same layout as y) and its ReLU bits ([M * Ncol / 8])
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.out ? a.out : a.y), (short)0, a.out ? a.outbytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t obrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.out_bits ? (void*)a.out_bits : a.y), (short)0,
      a.out_bits ? a.outbytes / 16 : 0, 0x00020000);

  // this wave's weight slice as MFMA A fragments (rows = output channels
  // ns0 + WCH wid + 32 i + l32, k = 16 ks + 8 hh .. +7), resident in VGPRs
  v8s af[CT][KS];
#pragma unroll
  for (int i = 0; i < CT; ++i) {
    const T* wr = (const T*)a.w + (long)(ns0 + C::WCH * wid + 32 * i + l32) * K + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[i][ks] = *(const v8s*)(wr + 16 * ks);
  }
  // channel parameters of this lane's chunks cc = (WCH/8) w + 4 i + 2 p + hh
  // (the apply form: BN scale in pa, shift in pb)
  float pa[CT][2][8], pb[CT][2][8], pm2[CT][2][8];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int ch = ns0 + 8 * ((C::WCH / 8) * wid + 4 * i + 2 * p + hh) + k;
        if constexpr (EPI == EPI_STATS) pa[i][p][k] = a.kshift ? a.kshift[ch] : 0.f;
        else if constexpr (EPI == EPI_APPLY) {
          pa[i][p][k] = a.bn_scale[ch];
          pb[i][p][k] = a.bn_shift[ch];
        } else pa[i][p][k] = a.mean ? a.mean[ch] : 0.f;
        if constexpr (DU) pm2[i][p][k] = a.mean2[ch];
      }
  // (retire those register loads here, not at their first use inside the
  // tile loop, where the compiler's wait would also drain the ring)
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(af[i][ks]));
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        asm volatile("" ::"v"(pa[i][p][k]));
        if constexpr (EPI == EPI_APPLY) asm volatile("" ::"v"(pb[i][p][k]));
        if constexpr (DU) asm volatile("" ::"v"(pm2[i][p][k]));
      }

  // one tile's operands into ring stage st; the same DMA count in every
  // wave and every iteration (tiles past the end load nothing: offset -1),
  // so one counted wait fits all
  auto load_tile = [&](int t, int st) {
    char* const sb = ring + st * STB;
    const int p0 = (t0 + t) * BMP;
    const int pend = t < ntile ? a.M : 0;
    {  // x: 1 KB = 512 / K pixel rows per DMA, chunk c at c ^ xsw(p)
      constexpr int LPR = K / 8;  // lanes per row
#pragma unroll
      for (int q = 0; q < C::XD; ++q) {
        const int j = wid * C::XD + q;
        const int pl = j * (64 / LPR) + lane / LPR;
        const int p = p0 + pl;
        const int off =
            p < pend ? p * C::XROW + (((lane % LPR) ^ xsw<K>(pl)) << 4) : -1;
        dma16(xrs, sb + j * 1024, off);
      }
    }
    if constexpr (EPI == EPI_APPLY) {
      // residual slice rows (2 NS bytes): chunk c at c ^ (p & 15)
      constexpr int LPR = NS / 8;
#pragma unroll
      for (int q = 0; q < C::YD; ++q) {
        const int j = wid * C::YD + q;
        const int pl = j * (64 / LPR) + lane / LPR;
        const int p = p0 + pl;
        const int off =
            p < pend ? p * ldy2 + ns0 * 2 + (((lane % LPR) ^ (pl & 15)) << 4) : -1;
        dma16(ars, sb + C::XB + j * 1024, off);
      }
    }
    if constexpr (EPI == EPI_DGRAD) {
      // addend / x_bn slice rows (2 NS bytes): chunk c at c ^ (p & 15)
      constexpr int LPR = NS / 8;
#pragma unroll
      for (int q = 0; q < C::YD; ++q) {
        const int j = wid * C::YD + q;
        const int pl = j * (64 / LPR) + lane / LPR;
        const int p = p0 + pl;
        const int off =
            p < pend ? p * ldy2 + ns0 * 2 + (((lane % LPR) ^ (pl & 15)) << 4) : -1;
        dma16(ars, sb + C::XB + j * 1024, off);
        dma16(xbrs, sb + C::XB + C::YB + j * 1024, off);
        if constexpr (DU) dma16(x2rs, sb + C::XB + 2 * C::YB + j * 1024, off);
      }
      // ReLU bits: NS / 8 bytes per pixel, this wave's quarter of the tile
      const int byte = 256 * wid + 4 * lane;
      const int pl = byte / (NS / 8);
      const int p = p0 + pl;
      const int off = (MASK >= 1 && byte < C::MB && p < pend)
                          ? p * (a.Ncol / 8) + ns0 / 8 + byte % (NS / 8) : -1;
      dma4(mrs, sb + C::MOFF + 256 * wid, off);
    }
  };

  float s1[CT][2][8], s2[CT][2][8], s3[CT][2][8];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[i][p][k] = 0.f; s2[i][p][k] = 0.f; s3[i][p][k] = 0.f; }
  const int fx = xsw<K>(l32);
  auto keep_if = [](float x, unsigned m) { return u2f(f2u(x) & m); };

#pragma unroll
  for (int t = 0; t < D; ++t) load_tile(t, t);
  wait_vm<0>();
  __syncthreads();

  int st = 0, sn = D;  // stages of tile t and of tile t + D
  for (int t = 0; t < ntile; ++t) {
    load_tile(t + D, sn);
    const char* const sb = ring + st * STB;
    // ---- WCH channels x 32 pixels per wave
    v16f acc[CT];
#pragma unroll
    for (int i = 0; i < CT; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const v8s bf = *(const v8s*)(sb + l32 * C::XROW + (((2 * ks + hh) ^ fx) << 4));
#pragma unroll
      for (int i = 0; i < CT; ++i) acc[i] = mfma32<T>(af[i][ks], bf, acc[i]);
    }
    // ---- epilogue: acc[i] reg 4g + q = channel WCH w + 32 i + 8 g + 4 hh + q
    // of pixel l32; swap register groups (2p, 2p+1) across the halves: this
    // lane then holds the 8 channels of chunk cc = (WCH/8) w + 4 i + 2 p + hh
    // epilogue operands of this lane's chunks, read from the ring by inline
    // asm: a plain LDS read here makes hipcc wait for every LDS-DMA in
    // flight (it cannot tell the ring stages apart), which would drain the
    // prefetch pipeline each tile
    v8s ea[CT][2], ex[CT][2], ex2[CT][2];
    unsigned em[CT][2];
    if constexpr (EPI == EPI_APPLY) {
#pragma unroll
      for (int i = 0; i < CT; ++i)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int cc = (C::WCH / 8) * wid + 4 * i + 2 * pp + hh;
          const unsigned so = lds_addr(sb + C::XB) + l32 * C::YROW + ((cc ^ (l32 & 15)) << 4);
          asm volatile("ds_read_b128 %0, %1" : "=v"(ea[i][pp]) : "v"(so));
        }
      if constexpr (CT == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ea[0][0]), "+v"(ea[0][1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ea[0][0]), "+v"(ea[0][1]), "+v"(ea[CT - 1][0]), "+v"(ea[CT - 1][1]));
    }
    if constexpr (EPI == EPI_DGRAD) {
#pragma unroll
      for (int i = 0; i < CT; ++i)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int cc = (C::WCH / 8) * wid + 4 * i + 2 * pp + hh;
          const unsigned so = lds_addr(sb + C::XB) + l32 * C::YROW + ((cc ^ (l32 & 15)) << 4);
          asm volatile("ds_read_b128 %0, %1" : "=v"(ea[i][pp]) : "v"(so));
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ex[i][pp]) : "v"(so), "i"(C::YB));
          if constexpr (DU)
            asm volatile("ds_read_b128 %0, %1 offset:%2"
                         : "=v"(ex2[i][pp]) : "v"(so), "i"(2 * C::YB));
          if constexpr (MASK >= 1) {
            const unsigned mo = lds_addr(sb + C::MOFF) + ((l32 * (NS / 8) + cc) & ~1);
            asm volatile("ds_read_u16 %0, %1" : "=v"(em[i][pp]) : "v"(mo));
          } else {
            em[i][pp] = 0xFFu;
          }
        }
      // (the registers pass through the wait: their uses stay behind it)
      if constexpr (DU && CT == 1)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ex2[0][0]), "+v"(ex2[0][1]));
      else if constexpr (DU)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ex2[0][0]), "+v"(ex2[0][1]), "+v"(ex2[CT - 1][0]),
                       "+v"(ex2[CT - 1][1]));
      if constexpr (CT == 1)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ea[0][0]), "+v"(ea[0][1]), "+v"(ex[0][0]), "+v"(ex[0][1]),
                       "+v"(em[0][0]), "+v"(em[0][1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ea[0][0]), "+v"(ea[0][1]), "+v"(ex[0][0]), "+v"(ex[0][1]),
                       "+v"(em[0][0]), "+v"(em[0][1]), "+v"(ea[CT - 1][0]), "+v"(ea[CT - 1][1]),
                       "+v"(ex[CT - 1][0]), "+v"(ex[CT - 1][1]), "+v"(em[CT - 1][0]),
                       "+v"(em[CT - 1][1]));
    }
    const int p = (t0 + t) * BMP + l32;
    const bool valid = p < a.M;
    const unsigned vmask = (FULL || valid) ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < CT; ++i)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int cc = (C::WCH / 8) * wid + 4 * i + 2 * pp + hh;
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(f2u(acc[i][8 * pp + q]),
                                                           f2u(acc[i][8 * pp + 4 + q]), false,
                                                           false);
          v[q] = u2f(sw[0]);
          v[4 + q] = u2f(sw[1]);
        }
        Vec<T, 8> ov;
        if constexpr (EPI == EPI_STATS) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            ov.v[k] = (T)v[k];
            const float d = keep_if(v[k] - pa[i][pp][k], vmask);
            s1[i][pp][k] += d;
            s2[i][pp][k] = fmaf(d, d, s2[i][pp][k]);
          }
        } else if constexpr (EPI == EPI_APPLY) {
          // the BN apply of bn.hip bn_apply_k on the stored (rounded) y
          const Vec<T, 8> rv = __builtin_bit_cast(Vec<T, 8>, ea[i][pp]);
          const float floor_ = a.relu ? 0.f : -INFINITY;
          Vec<T, 8> outv;
          unsigned bits = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            ov.v[k] = (T)v[k];
            float o = (float)ov.v[k] * pa[i][pp][k] + pb[i][pp][k];
            o = fmaxf(o + (float)rv.v[k], floor_);
            outv.v[k] = (T)o;
            bits |= ((float)outv.v[k] > 0.f ? 1u : 0u) << k;
          }
          const int ooff = valid ? p * ldy2 + (ns0 + 8 * cc) * 2 : -1;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, outv), ors, ooff, 0,
                                                 0);
          __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bits, obrs,
                                               valid ? (p * a.Ncol + ns0 + 8 * cc) / 8 : -1, 0, 0);
        } else {
          const Vec<T, 8> av = __builtin_bit_cast(Vec<T, 8>, ea[i][pp]);
          const Vec<T, 8> xv = __builtin_bit_cast(Vec<T, 8>, ex[i][pp]);
          const unsigned mk = MASK >= 1 ? (em[i][pp] >> (8 * (cc & 1))) & 0xFFu : 0xFFu;
          const Vec<T, 8> x2v = __builtin_bit_cast(Vec<T, 8>, DU ? ex2[i][pp] : ex[i][pp]);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float x = v[k] + (float)av.v[k];
            x = keep_if(x, 0u - ((mk >> k) & 1u));
            const float xd = keep_if(x, vmask);
            s1[i][pp][k] += xd;
            const float dx = (float)xv.v[k] - pa[i][pp][k];
            s2[i][pp][k] =
                fmaf(xd, u2f((f2u(dx) & xbn_mask) | (f2u(x) & ~xbn_mask)), s2[i][pp][k]);
            if constexpr (DU)
              s3[i][pp][k] = fmaf(xd, (float)x2v.v[k] - pm2[i][pp][k], s3[i][pp][k]);
            ov.v[k] = (T)x;
          }
        }
        if constexpr (C::STAGED) {
          const int j = 4 * i + 2 * pp + hh;  // chunk within the wave's columns
          const unsigned sa = stg + l32 * SROW + ((j ^ sgz(l32)) << 4);
          asm volatile("ds_write_b128 %0, %1" ::"v"(sa), "v"(__builtin_bit_cast(v4u_t, ov)));
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, ov), yrs,
                                                 valid ? p * ldy2 + (ns0 + 8 * cc) * 2 : -1, 0,
                                                 0);
        }
      }
    if constexpr (C::STAGED) {
      // whole row pieces back out: WCH / 16 stores per lane, as many as the
      // per-lane pieces they replace (the counted ring wait is unchanged)
      constexpr int LPR = SROW / 16;  // lanes per row piece
      constexpr int NQ = C::WCH / 16;
      v4u_t sv[NQ];
      asm volatile("s_waitcnt lgkmcnt(0)");
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r = q * (64 / LPR) + lane / LPR, c = lane % LPR;
        asm volatile("ds_read_b128 %0, %1" : "=v"(sv[q]) : "v"(stg + r * SROW + ((c ^ sgz(r)) << 4)));
      }
      if constexpr (NQ == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(sv[0]), "+v"(sv[NQ - 1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(sv[0]), "+v"(sv[1]), "+v"(sv[2]), "+v"(sv[NQ - 1]));
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r = q * (64 / LPR) + lane / LPR, c = lane % LPR;
        const int pr = (t0 + t) * BMP + r;
        __builtin_amdgcn_raw_buffer_store_b128(
            sv[q], yrs, (FULL || pr < a.M) ? pr * ldy2 + (ns0 + C::WCH * wid + 8 * c) * 2 : -1, 0,
            0);
      }
    }
    // tile t+1's operands landed for every wave (issued in iteration t+1-D;
    // after them: the stores of tiles t+1-D .. t and the DMAs of tiles
    // t+2 .. t+D) and every wave is done reading stage st
    wait_vm<C::WAIT>();
    __builtin_amdgcn_s_barrier();
    st = st == NST - 1 ? 0 : st + 1;
    sn = sn == NST - 1 ? 0 : sn + 1;
  }

  if (a.stats) {
    // lanes with one hh hold the same channels: reduce over the 32 lanes,
    // then one atomic add per channel into statistics slot blockIdx % 32
#pragma unroll
    for (int i = 0; i < CT; ++i)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) {
            s1[i][pp][k] += __shfl_xor(s1[i][pp][k], o, 64);
            s2[i][pp][k] += __shfl_xor(s2[i][pp][k], o, 64);
            if constexpr (DU) s3[i][pp][k] += __shfl_xor(s3[i][pp][k], o, 64);
          }
        }
    if (l32 == 0) {
#pragma unroll
      for (int i = 0; i < CT; ++i)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int ch = ns0 + 8 * ((C::WCH / 8) * wid + 4 * i + 2 * pp + hh) + k;
            atomicAdd(a.stats + (long)(b % IG_SPREAD) * a.Ncol + ch, s1[i][pp][k]);
            atomicAdd(a.stats + (long)(IG_SPREAD + b % IG_SPREAD) * a.Ncol + ch, s2[i][pp][k]);
            if constexpr (DU) atomicAdd(a.stats2 + (long)(b % IG_SPREAD) * a.Ncol + ch, s3[i][pp][k]);
          }
    }
  }
  bn_tail(a, (int*)ring);
}

static int slice_width(int K) { return K <= 128 ? 256 : 128; }

}  // namespace s1

bool conv_s1_fits(const IgArgs& a) {
  const int K = a.C;
  const bool geo = (K == 64 || K == 128 || K == 256 || K == 512) &&
                   a.Ncol % s1::slice_width(K) == 0 && a.KH == 1 && a.KW == 1 && a.sh == 1 &&
                   a.sw == 1 && a.pt == 0 && a.pl == 0 && a.OH == a.H && a.OW == a.W &&
                   a.YH == a.OH && a.YW == a.OW && a.ys == 1 && a.ldy == a.Ncol && !a.zfill &&
                   !a.c8 && a.xbytes > 0 && a.wbytes > 0 && !a.bias;
  if (a.out) {  // apply form: BN apply (+ residual, ReLU) of the recomputed output
    return geo && a.bn_scale && a.bn_shift && a.outbytes > 0 && !a.stats && !a.xbn &&
           !a.mask && !a.mcoef && (a.ybytes == 0 || a.ybytes == a.outbytes);
  }
  const bool dg = a.addend || a.xbn;
  // dual-BN partials: the bit-mask data gradient only
  if (a.xbn2 && !(dg && a.xbn && a.mask && a.maskbits && a.stats && a.stats2 && a.mean2))
    return false;
  return geo && !(dg && a.kshift) && !(!dg && a.mask) && !a.relu &&
         // statistics-only forward (ybytes 0: stores dropped)
         (a.ybytes > 0 || (a.stats && !dg)) &&
         // producer-BN ReLU mask: none or the bit mask
         !(dg && a.xbn && ((a.mask && !a.maskbits) || (!a.mask && a.mcoef))) &&
         !(dg && !a.xbn && a.mask);
}

static int g_s1_grid_force = 0;  // test hook: workgroups per launch (0 = one per CU)

// workgroups per CU: 2 where two fit (LDS ring and registers: the variants
// below 256 VGPR + AGPR at one workgroup per CU) - the second workgroup's
// waves hide the first's MFMA / LDS / epilogue latencies, which one wave per
// SIMD leaves exposed - except the K = 64 data gradient: at one workgroup
// its output stores go through the LDS staging (no room beside two rings),
// 291 -> 279 us at 56x56, ResNet-50 -0.06 ms/step on 4 interleaved pairs
// (profiles/r12_s1_staged_stores.txt)
static int s1_wpc(int K, bool dg) {
  const bool two = dg ? K == 256 : K <= 256;
  return two ? 2 : 1;
}

static int s1_grid(int tiles, int nsl, int wpc) {
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
  int g = g_s1_grid_force > 0 ? g_s1_grid_force : cus * wpc;
  // whole pixel groups (one workgroup per slice each), at most one tile each
  int groups = g / nsl;
  if (groups > tiles) groups = tiles;
  if (groups < 1) groups = 1;
  return groups * nsl;
}

template <typename T, int K, int EPI, int MASK, int WPC>
static void launch_s1_k(const IgArgs& a, int tiles, int nsl, hipStream_t s) {
  if (a.M % s1::BMP == 0)
    hipLaunchKernelGGL((s1::conv_s1_k<T, K, EPI, MASK, WPC, true>), dim3(s1_grid(tiles, nsl, WPC)),
                       dim3(256), 0, s, a, tiles, nsl);
  else
    hipLaunchKernelGGL((s1::conv_s1_k<T, K, EPI, MASK, WPC>), dim3(s1_grid(tiles, nsl, WPC)),
                       dim3(256), 0, s, a, tiles, nsl);
}

template <typename T, int K>
static void launch_s1(const IgArgs& a, int tiles, int nsl, int epi, int mask, hipStream_t s) {
  if (mask == 2) {  // dual-BN partials: three operand tiles per stage, one workgroup per CU
    launch_s1_k<T, K, s1::EPI_DGRAD, 2, 1>(a, tiles, nsl, s);
    return;
  }
  if (s1_wpc(K, epi == s1::EPI_DGRAD) == 2) {
    if constexpr (K <= 256) {
      if (epi == s1::EPI_STATS) launch_s1_k<T, K, s1::EPI_STATS, 0, 2>(a, tiles, nsl, s);
      else if (epi == s1::EPI_APPLY) launch_s1_k<T, K, s1::EPI_APPLY, 0, 2>(a, tiles, nsl, s);
      else if constexpr (K != 128) {
        if (mask) launch_s1_k<T, K, s1::EPI_DGRAD, 1, 2>(a, tiles, nsl, s);
        else launch_s1_k<T, K, s1::EPI_DGRAD, 0, 2>(a, tiles, nsl, s);
      }
      return;
    }
  }
  if (epi == s1::EPI_STATS) launch_s1_k<T, K, s1::EPI_STATS, 0, 1>(a, tiles, nsl, s);
  else if (epi == s1::EPI_APPLY) launch_s1_k<T, K, s1::EPI_APPLY, 0, 1>(a, tiles, nsl, s);
  else if (mask) launch_s1_k<T, K, s1::EPI_DGRAD, 1, 1>(a, tiles, nsl, s);
  else launch_s1_k<T, K, s1::EPI_DGRAD, 0, 1>(a, tiles, nsl, s);
}

template <typename T>
static hipError_t launch_s1_t(const IgArgs& a, hipStream_t s) {
  const int tiles = (a.M + s1::BMP - 1) / s1::BMP;
  const int nsl = a.Ncol / s1::slice_width(a.C);
  const int epi = a.out ? s1::EPI_APPLY : (a.addend || a.xbn) ? s1::EPI_DGRAD : s1::EPI_STATS;
  const int mask = (epi == s1::EPI_DGRAD && a.xbn && a.mask) ? (a.xbn2 ? 2 : 1) : 0;
  switch (a.C) {
    case 64: launch_s1<T, 64>(a, tiles, nsl, epi, mask, s); break;
    case 128: launch_s1<T, 128>(a, tiles, nsl, epi, mask, s); break;
    case 256: launch_s1<T, 256>(a, tiles, nsl, epi, mask, s); break;
    case 512: launch_s1<T, 512>(a, tiles, nsl, epi, mask, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_conv_s1(int dtype, const IgArgs& a, hipStream_t stream) {
  if (!conv_s1_fits(a)) return hipErrorInvalidValue;
  if (dtype == BF16) return launch_s1_t<bf16>(a, stream);
  if (dtype == F16) return launch_s1_t<f16>(a, stream);
  return hipErrorInvalidValue;
}

}  // namespace kfb

KFB_API void kfb_conv_s1_set_grid(int g) { kfb::g_s1_grid_force = g; }

// The apply form (EPI_APPLY): y = conv1x1(x, w) recomputed (NHWC [N,H,W,C] ->
// [N,H,W,Ncol]), stored to y when y != null, and out = relu?(bf16(y) * scale
// + shift + res) (res nullable) with out's ReLU bit mask (bits nullable).
KFB_API hipError_t kfb_conv_s1_apply(int dtype, const void* x, const void* w, void* y, void* out,
                                     const void* res, int N, int H, int W, int C, int Ncol,
                                     const float* scale, const float* shift, int relu,
                                     uint8_t* bits, hipStream_t stream);

// The BN forward (training) of a conv whose output was never stored: the
// statistics were summed by the conv's statistics-only pass (psum / psq
// slots, finalized here unless `finalized`), then one apply-form pass
// recomputes y, stores it (the BN backward reads it) and writes
// out = relu?(bn(y) + res) with its ReLU bit mask.  The two launches of
// kfb_bn_fwd_train's finalize + apply, with y's write moved from the
// conv's first pass into the apply pass and the apply's read of y replaced
// by the conv's 4x smaller input.
KFB_API hipError_t kfb_bn_fwd_train_recompute(
    int dtype, const void* x, const void* w, void* y, void* out, const void* res, int N, int H,
    int W, int C, int Ncol, const float* gamma, const float* beta, float decay, float eps,
    float* run_mean, float* run_var, float* save_mean, float* save_invstd, float* scale,
    float* shift, const float* psum, const float* psq, int nslab, int finalized, float* kshift,
    int relu, uint8_t* bits, hipStream_t stream) {
  if (!finalized) {
    const hipError_t e =
        kfb::bn_finalize_stats_launch(psum, psq, nslab, Ncol, (long)N * H * W, gamma, beta, decay,
                                      eps, run_mean, run_var, save_mean, save_invstd, scale, shift,
                                      kshift, stream);
    if (e != hipSuccess) return e;
  }
  return kfb_conv_s1_apply(dtype, x, w, y, out, res, N, H, W, C, Ncol, scale, shift, relu, bits,
                           stream);
}

KFB_API hipError_t kfb_conv_s1_apply(int dtype, const void* x, const void* w, void* y, void* out,
                                     const void* res, int N, int H, int W, int C, int Ncol,
                                     const float* scale, const float* shift, int relu,
                                     uint8_t* bits, hipStream_t stream) {
  if (C % 8 || Ncol % 8) return hipErrorInvalidValue;
  const long xbytes = (long)N * H * W * C * 2, wbytes = (long)Ncol * C * 2;
  const long obytes = (long)N * H * W * Ncol * 2;
  if (xbytes >= (1L << 31) || obytes >= (1L << 31)) return hipErrorInvalidValue;
  kfb::IgArgs a{};
  a.x = x;
  a.w = w;
  a.y = y ? y : out;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.OH = H;
  a.OW = W;
  a.KH = a.KW = a.sh = a.sw = 1;
  a.Ncol = Ncol;
  a.Ktot = C;
  a.M = N * H * W;
  a.YH = H;
  a.YW = W;
  a.ys = 1;
  a.ldy = Ncol;
  a.addend = res;
  a.relu = relu ? 1 : 0;
  a.xbytes = (int)xbytes;
  a.wbytes = (int)wbytes;
  a.ybytes = y ? (int)obytes : 0;
  a.out = out;
  a.bn_scale = scale;
  a.bn_shift = shift;
  a.out_bits = bits;
  a.outbytes = (int)obytes;
  if (!out || !kfb::conv_s1_fits(a)) return hipErrorInvalidValue;
  return kfb::launch_conv_s1(dtype, a, stream);
}

// Data gradient of a 1x1 stride-1 conv (dX [N,H,W,Ncol] = dY [N,H,W,K] W,
// w = [Ncol][K]) whose input is a dual-BN block output y = relu(bn(x) +
// bn2(x2)) (kfb_bn_fwd_train_dual): the epilogue adds `addend` (nullable),
// applies y's ReLU bit mask and accumulates both BNs' backward partials -
// stats [2][IG_SPREAD][Ncol] (sum y', sum y'(x - mean)) and stats2
// [IG_SPREAD][Ncol] (sum y'(x2 - mean2)), so the dual backward
// (kfb_bn_bwd_dual) needs no partial pass over y' and x2.  Streaming kernel
// geometries only (kfb_conv_s1_applicable); 16-byte aligned pointers.
KFB_API hipError_t kfb_conv_s1_dgrad_dual(int dtype, const void* dy, const void* w, void* dx,
                                          int N, int H, int W, int K, int Ncol, float* stats,
                                          const uint8_t* bits, const void* xbn, const float* mean,
                                          const void* addend, const void* xbn2,
                                          const float* mean2, float* stats2,
                                          hipStream_t stream) {
  if (K % 8 || Ncol % 8 || !stats || !bits || !xbn || !mean || !xbn2 || !mean2 || !stats2)
    return hipErrorInvalidValue;
  const long xbytes = (long)N * H * W * K * 2, wbytes = (long)Ncol * K * 2;
  const long ybytes = (long)N * H * W * Ncol * 2;
  if (xbytes >= (1L << 31) || ybytes >= (1L << 31)) return hipErrorInvalidValue;
  kfb::IgArgs a{};
  a.x = dy;
  a.w = w;
  a.y = dx;
  a.N = N;
  a.H = a.OH = a.YH = H;
  a.W = a.OW = a.YW = W;
  a.C = a.Ktot = K;
  a.KH = a.KW = a.sh = a.sw = a.ys = 1;
  a.Ncol = a.ldy = Ncol;
  a.M = N * H * W;
  a.stats = stats;
  a.mask = bits;
  a.maskbits = 1;
  a.xbn = xbn;
  a.mean = mean;
  a.addend = addend;
  a.xbytes = (int)xbytes;
  a.wbytes = (int)wbytes;
  a.ybytes = (int)ybytes;
  a.xbn2 = xbn2;
  a.mean2 = mean2;
  a.stats2 = stats2;
  if (!kfb::conv_s1_fits(a)) return hipErrorInvalidValue;
  return kfb::launch_conv_s1(dtype, a, stream);
}

KFB_API int kfb_conv_s1_applicable(int C, int Ncol, int KH, int KW, int sh, int sw, int pt, int pl,
                                   int H, int W, int OH, int OW) {
  return (C == 64 || C == 128 || C == 256 || C == 512) &&
                 Ncol % kfb::s1::slice_width(C) == 0 && KH == 1 && KW == 1 && sh == 1 &&
                 sw == 1 && pt == 0 && pl == 0 && OH == H && OW == W
             ? 1
             : 0;
}
