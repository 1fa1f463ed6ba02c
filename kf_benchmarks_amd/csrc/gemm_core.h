// Shared MFMA GEMM core (gfx950): operand images, fragment reads, loaders
// and the double-buffered main loop used by the affine GEMM (gemm.hip) and
// the fp32 implicit-GEMM convolutions (conv_f32.hip).  See gemm.hip for the
// tiling and the two operand layouts (KC / KS).
#pragma once
#include "common.h"

namespace kfb {
namespace gm {

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(4))) float v4f;
typedef __attribute__((ext_vector_type(4))) short v4s;

constexpr int TILE = 128;

enum { OUT_T = 0, OUT_F32 = 1, OUT_SLAB = 2 };


// Per-dtype geometry.  Every operand tile moves in 16-byte chunks of EPC
// elements; a K step is 8 chunks (128 bytes) of each KC row, i.e. 64 k for
// 16-bit types and 32 k for fp32, so both image kinds take 16 KB per
// operand per stage for every dtype.
//   16-bit: v_mfma_f32_16x16x32_{bf16,f16}; fragment = 8 consecutive k.
//   fp32:   v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate);
//           a lane reads 4 consecutive k (one 16-byte KC chunk, or 4 KS
//           rows) and feeds them to 4 MFMAs: MFMA t sums k = 16s + 4g + t
//           over the lane groups g, the same permutation on both operands.
template <typename T> struct Tr {
  static constexpr int EPC = 8, BK = 64;
  static constexpr int KS_ROWS = 64, KS_PITCH = 128;  // KS image: [k][128 cols]
  typedef v8s Frag;
};
template <> struct Tr<float> {
  static constexpr int EPC = 4, BK = 32;
  static constexpr int KS_ROWS = 32, KS_PITCH = 132;  // +4 floats: 4 row groups -> 4 bank quarters
  typedef v4f Frag;
};

template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  static __device__ __forceinline__ v4f run(v8s a, v8s b, v4f c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<f16> {
  static __device__ __forceinline__ v4f run(v8s a, v8s b, v4f c) {
    typedef __attribute__((ext_vector_type(8))) _Float16 v8h;
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a),
                                                  __builtin_bit_cast(v8h, b), c, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  static __device__ __forceinline__ v4f run(v4f a, v4f b, v4f c) {
#pragma unroll
    for (int t = 0; t < 4; ++t) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[t], c, 0, 0, 0);
    return c;
  }
};

// KC image: element offset of 16-byte chunk `chunk` (0..7) of 128-byte row
// `row`, chunks XOR-swizzled by (row >> 1) & 7 (conflict-free 16-lane reads).
template <typename T>
__device__ __forceinline__ int kc_off(int row, int chunk) {
  return row * Tr<T>::BK + ((chunk ^ ((row >> 1) & 7)) * Tr<T>::EPC);
}

// KS image.  16-bit: 256-byte rows (128 elements); 32-byte unit u of row r
// stored at u ^ f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2 (the 8 rows one
// 32-lane half reads land in 8 distinct 32-byte bank windows).  fp32: rows
// of 132 floats (the 4 rows one fragment read touches sit in 4 bank quarters).
template <typename T>
__device__ __forceinline__ int ks_off(int row, int col) {
  if constexpr (sizeof(T) == 4) {
    return row * Tr<T>::KS_PITCH + col;
  } else {
    const int f = (row & 3) | (((row >> 3) & 1) << 2);
    return row * TILE + ((((col >> 4) ^ f) << 4) | (col & 15));
  }
}

__device__ __forceinline__ v4s ds_read_tr(const void* p) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <typename T> struct Bits;
template <> struct Bits<bf16> { typedef unsigned short U; };
template <> struct Bits<f16> { typedef unsigned short U; };
template <> struct Bits<float> { typedef unsigned int U; };

// One operand's per-step loader: 4 chunks of EPC elements per thread.
//   KC: chunk c -> (row c >> 3, k EPC * (c & 7));
//   KS: chunk c -> (k c / (128 / EPC), row EPC * (c % (128 / EPC))).
// VEC: every chunk is fully in or fully out of range and 16-byte aligned
// (the contiguous extent and ld are multiples of EPC): one buffer load.
// Otherwise per-element loads with per-element bounds.
template <typename T, bool KS_, bool VEC>
struct Loader {
  static constexpr bool KS = KS_;
  static constexpr int EPC = Tr<T>::EPC, CPR = TILE / EPC;
  typedef typename Bits<T>::U U;
  __amdgpu_buffer_rsrc_t rs;
  const U* base;
  int ld, rows, r0, kend;
  int cr[4], ck[4];  // chunk row / k offsets (relative to the tile / step)

  __device__ __forceinline__ void init(const void* ptr, int bytes, int ld_, int rows_, int r0_,
                                       int kend_, int tid) {
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)ptr, (short)0, bytes, 0x00020000);
    base = (const U*)ptr;
    ld = ld_;
    rows = rows_;
    r0 = r0_;
    kend = kend_;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * 256;
      if (KS) { ck[i] = c / CPR; cr[i] = (c % CPR) * EPC; }
      else { cr[i] = c >> 3; ck[i] = (c & 7) * EPC; }
    }
  }

  __device__ __forceinline__ void load(uint4 (&r)[4], int k0) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r0 + cr[i], k = k0 + ck[i];
      if constexpr (VEC) {
        const bool ok = row < rows && k < kend;
        const int off = ok ? (KS ? k * ld + row : row * ld + k) * (int)sizeof(T) : -1;
        r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      } else {
        U e[EPC];
#pragma unroll
        for (int j = 0; j < EPC; ++j) {
          const int rr = KS ? row + j : row, kk = KS ? k : k + j;
          const bool ok = rr < rows && kk < kend;
          e[j] = ok ? base[KS ? (long)kk * ld + rr : (long)rr * ld + kk] : (U)0;
        }
        r[i] = __builtin_bit_cast(uint4, e);
      }
    }
  }

  __device__ __forceinline__ void store(const uint4 (&r)[4], T* img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = KS ? ks_off<T>(ck[i], cr[i]) : kc_off<T>(cr[i], ck[i] / EPC);
      *(uint4*)(img + off) = r[i];
    }
  }
};

// Fragment of 16 rows (rbase .. rbase+15) for K substep ks (32 k for 16-bit,
// 16 k for fp32) of lane.
template <typename T, bool KS>
__device__ __forceinline__ typename Tr<T>::Frag frag(const T* img, int rbase, int ks, int lane) {
  const int g = lane >> 4;
  if constexpr (sizeof(T) == 4) {
    if constexpr (KS) {
      const int k0 = ks * 16 + 4 * g, col = rbase + (lane & 15);
      return v4f{img[ks_off<T>(k0, col)], img[ks_off<T>(k0 + 1, col)],
                 img[ks_off<T>(k0 + 2, col)], img[ks_off<T>(k0 + 3, col)]};
    } else {
      return *(const v4f*)(img + kc_off<T>(rbase + (lane & 15), ks * 4 + g));
    }
  } else if constexpr (KS) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int k0 = ks * 32 + 8 * g, col = rbase + 4 * p;
    const v4s lo = ds_read_tr(img + ks_off<T>(k0 + q, col));
    const v4s hi = ds_read_tr(img + ks_off<T>(k0 + 4 + q, col));
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  } else {
    return *(const v8s*)(img + kc_off<T>(rbase + (lane & 15), ks * 4 + g));
  }
}

template <typename T>
constexpr int img_elems() {  // one operand image (KS fp32 rows are padded)
  return sizeof(T) == 4 ? Tr<T>::KS_ROWS * Tr<T>::KS_PITCH : TILE * Tr<T>::BK;
}


// fp32 operands as bf16 pairs: x = hi + lo, hi = bf16(x), lo = bf16(x - hi)
// (both round-to-nearest-even).  8 fp32 values -> the hi and lo fragments of
// one 16x16x32 bf16 MFMA.
__device__ __forceinline__ void split_bf16x2(v4f x0, v4f x1, v8s& hi, v8s& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float f = e < 4 ? x0[e] : x1[e - 4];
    const __bf16 h = (__bf16)f;
    hi[e] = __builtin_bit_cast(short, h);
    lo[e] = __builtin_bit_cast(short, (__bf16)(f - (float)h));
  }
}

// The double-buffered main loop over nk K steps from kbeg: P (M-side) and
// Q (N-side) loaders fill the two operand images of a stage one K step
// ahead in registers; 2 x 2 waves each own a 64 x 64 block of the 128 x 128
// tile (acc[i][j] = columns wn*64 + 16i .., rows wm*64 + 16j ..).
//
// X3 (fp32 only): instead of v_mfma_f32_16x16x4_f32, each pair of 16-k
// substeps runs as three v_mfma_f32_16x16x32_bf16 on the bf16 split of both
// operands, a*b ~ ah*bh + ah*bl + al*bh (the dropped al*bl and the rounding of
// lo leave a relative error ~2^-16 per product; fp32 accumulation).  Lane
// group g supplies k = 4g..4g+3 of substep 0 and of substep 1 as its 8
// consecutive MFMA k: the same permutation on both operands, so the sum
// over k is unchanged.  One bf16 MFMA = 16 cycles vs 32 per 4-k fp32 MFMA:
// 32 k cost 3 x 16 instead of 8 x 32 cycles.
template <typename T, class LP, class LQ, bool X3 = false>
__device__ __forceinline__ void mainloop(LP& lp, LQ& lq, int kbeg, int nk, T* smem,
                                         v4f (&acc)[TILE / 32][TILE / 32]) {
  constexpr int TM = TILE / 32, TN = TILE / 32;
  constexpr int IMG = img_elems<T>();
  constexpr int BK = Tr<T>::BK;
  typedef typename Tr<T>::Frag Frag;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wm = wid & 1;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  uint4 pr[4], qr[4];
  if (nk > 0) {
    lp.load(pr, kbeg);
    lq.load(qr, kbeg);
    lp.store(pr, smem);
    lq.store(qr, smem + IMG);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      lp.load(pr, kbeg + (kt + 1) * BK);
      lq.load(qr, kbeg + (kt + 1) * BK);
    }
    const T* pimg = smem + cur * 2 * IMG;
    const T* qimg = pimg + IMG;
    if constexpr (X3) {
      static_assert(sizeof(T) == 4, "X3 splits fp32 operands");
      v8s ah[TN], al[TN], bh[TM], bl[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int r = wn * (TILE / 2) + i * 16;
        split_bf16x2(frag<T, LQ::KS>(qimg, r, 0, lane), frag<T, LQ::KS>(qimg, r, 1, lane), ah[i],
                     al[i]);
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int r = wm * (TILE / 2) + j * 16;
        split_bf16x2(frag<T, LP::KS>(pimg, r, 0, lane), frag<T, LP::KS>(pimg, r, 1, lane), bh[j],
                     bl[j]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          v4f c = Mfma<bf16>::run(al[i], bh[j], acc[i][j]);
          c = Mfma<bf16>::run(ah[i], bl[j], c);
          acc[i][j] = Mfma<bf16>::run(ah[i], bh[j], c);
        }
    } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      Frag af[TN], bf[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = frag<T, LQ::KS>(qimg, wn * (TILE / 2) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bf[j] = frag<T, LP::KS>(pimg, wm * (TILE / 2) + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bf[j], acc[i][j]);
    }
    }
    if (kt + 1 < nk) {
      T* nimg = smem + (cur ^ 1) * 2 * IMG;
      lp.store(pr, nimg);
      lq.store(qr, nimg + IMG);
    }
    __syncthreads();
  }
}

}  // namespace gm
}  // namespace kfb
