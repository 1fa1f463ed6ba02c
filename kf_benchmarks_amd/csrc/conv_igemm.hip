// Implicit-GEMM NHWC convolution on gfx950 MFMA (bf16/fp16 in, fp32 acc).
//
// Replaces cuDNN conv fwd / bwd-data / bwd-filter (tf.nn.conv2d and its
// autodiff in tcb/convnet_builder.py:107-213).
//
//   fwd   : y[m][n]  = sum_k  X(m,k) * Wt[n][k]      m=(img,oh,ow) n=cout k=(kh,kw,cin)
//   dgrad : dx[m][n] = sum_k dY'(m,k) * Wd[n][k]     m=(img,h,w)   n=cin  k=(kh,kw,cout)
//           ("transposed" gather: dY row (h+pt-kh)/s when divisible), or a
//           plain 1x1 GEMM scattered into every s-th output pixel for
//           strided 1x1 convs (ResNet v1 projection shortcuts).
//   wgrad : dW[n][k] = sum_m  dY[m][n] * X(m,k)      reduction over m = N*OH*OW,
//           split over workgroups, fp32 atomic accumulation.
//
// Tiling (igemm_k): 256 threads = 4 waves in a 2x2 grid; a workgroup computes
// BN(out-channel) x BM(pixel) with v_mfma_f32_16x16x32_bf16, the weight tile
// as the A operand and the pixel tile as the B operand, so each lane's four
// accumulator registers are four consecutive output channels of one pixel
// (one 8-byte store per lane-row).  K advances 64 per step through a
// double-buffered LDS image with 128-byte rows whose 16-byte chunks are
// XOR-swizzled by (row>>1)&7: the ds_read_b128 fragment reads of every
// 16-lane group then hit 16 distinct bank slots (conflict-free).  The global
// loads of step k+1 are issued before the MFMAs of step k.  Workgroup ids
// are remapped so each XCD works on a contiguous run of tiles (L2 reuse of
// the pixel rows across the output-channel tiles).
//
// wgrad_k reads both operands transposed (reduction index m is the row of
// both LDS images) with ds_read_b64_tr_b16; its images use 256-byte rows
// with 32-byte units XOR-swizzled so the 8 rows a 32-lane half reads land in
// 8 distinct 32-byte bank windows.
#include "common.h"
#include "igemm_args.h"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

namespace kfb {

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(4))) float v4f;
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((ext_vector_type(16))) float v16f;

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
// 32x32x16 form: twice the MACs per instruction and ~15% more sustained
// throughput than 16x16x32 on random operands (scripts/probes/mfma_rate.hip:
// 1.79 vs 1.55 PFLOP/s); lane l holds rows 8g + 4(l/32) + r (g, r < 4) of
// column l % 32 of the 32x32 result, and supplies row / column l % 32, K
// elements 8(l/32) .. +8 of each operand.
template <typename T> struct Mfma32;
template <> struct Mfma32<bf16> {
  static __device__ __forceinline__ v16f run(v8s a, v8s b, v16f c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma32<f16> {
  static __device__ __forceinline__ v16f run(v8s a, v8s b, v16f c) {
    typedef __attribute__((ext_vector_type(8))) _Float16 v8h;
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, a),
                                                  __builtin_bit_cast(v8h, b), c, 0, 0, 0);
  }
};


// offset (elements) of chunk kc's tap within step 0 (8-channel geometry) or
// of the 16-byte channel chunk kc (C % 64 == 0)
__device__ __forceinline__ int fast_lane_off(const IgArgs& a, int kc) {
  return a.c8 ? ((kc / a.KW) * a.W + kc % a.KW) * a.C : kc * 8;
}

__device__ __forceinline__ int swz_off(int row, int chunk) {
  // element offset of 16-byte chunk `chunk` (0..7) of 128-byte row `row`
  return row * IG_BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

typedef __attribute__((ext_vector_type(4))) unsigned int v4u;

// Workgroup barrier for LDS traffic only.  __syncthreads() also waits for
// every outstanding global store of the wave (vmcnt(0)); in the epilogue the
// statistics fold runs right after a tile's 16-32 KB of output stores, and
// that wait cost ~2 us per workgroup round on the memory-bound layers.
__device__ __forceinline__ void lds_only_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Shared epilogue of the implicit-GEMM kernels: acc[i][j] holds channels
// n..n+3 of pixel m for each (i, j) 16x16 subtile of the wave's
// (BM/WGM) x (BN/WGN) block; NT threads; smem must hold BM*BN elements (and
// NT*16 floats for the statistics fold).  `pre` runs once the accumulators
// are staged in LDS (they are dead from there on): a multi-tile workgroup
// issues the next tile's first operand loads there, so they are in flight
// while this tile's output stores drain.
struct NoPrefetch {
  __device__ void operator()() const {}
};

// Output-row offset (elements) of GEMM row m in the y layout.
__device__ __forceinline__ long ig_row_offset(const IgArgs& a, int m) {
  if (a.ys == 1 && a.YH == a.OH && a.YW == a.OW) return (long)m * a.ldy;
  const int OHW = a.OH * a.OW;
  const int img = m / OHW, rem = m - img * OHW;
  const int oh = rem / a.OW, ow = rem - oh * a.OW;
  return ((long)(img * a.YH + oh * a.ys) * a.YW + ow * a.ys) * a.ldy;
}

// Range-checked buffer resources of the dgrad-style epilogue operands
// (addend, mask / ReLU bits, xbn); a null operand gets a zero-size range.
struct EpiRsrc {
  __amdgpu_buffer_rsrc_t ad, mk, xb;
};
__device__ __forceinline__ EpiRsrc epi_rsrc(const IgArgs& a) {
  EpiRsrc r;
  r.ad = __builtin_amdgcn_make_buffer_rsrc((void*)(a.addend ? a.addend : a.y), (short)0,
                                           a.addend ? a.ybytes : 0, 0x00020000);
  r.mk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.mask ? a.mask : a.y), (short)0,
      (a.mask && a.xbn) ? (a.maskbits ? a.ybytes / 16 : a.ybytes) : 0, 0x00020000);
  r.xb = __builtin_amdgcn_make_buffer_rsrc((void*)(a.xbn ? a.xbn : a.y), (short)0,
                                           a.xbn ? a.ybytes : 0, 0x00020000);
  return r;
}

// One pass group's epilogue operands (G 16-byte chunks of each of addend,
// mask, xbn, and their byte offsets; -1 = outside the output).
template <int G>
struct EpiOps {
  int offb[G];
  uint4 ad[G], mk[G], xb[G];
};

template <typename T, int BN, int NT, int G>
__device__ __forceinline__ void epi_load(const IgArgs& a, const EpiRsrc& r, int m0, int n0, int g,
                                         EpiOps<G>& e) {
  constexpr int CPR = BN / 8;
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < G; ++q) {
    const int t = tid + (g * G + q) * NT;
    const int m = m0 + t / CPR, n = n0 + (t % CPR) * 8;
    e.offb[q] = (m < a.M && n < a.Ncol) ? (int)((ig_row_offset(a, m) + n) * (long)sizeof(T)) : -1;
    e.ad[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r.ad, e.offb[q], 0, 0));
    if (a.maskbits)  // one byte per 16-byte chunk (offb < 0: out of range, reads 0)
      e.mk[q] = make_uint4(
          __builtin_amdgcn_raw_buffer_load_b8(r.mk, e.offb[q] < 0 ? -1 : e.offb[q] >> 4, 0, 0), 0u,
          0u, 0u);
    else
      e.mk[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r.mk, e.offb[q], 0, 0));
    e.xb[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r.xb, e.offb[q], 0, 0));
  }
}

// Pass-group size of the dgrad-style epilogue of a BM x BN tile on NT threads.
template <int BM, int BN, int NT>
constexpr int epi_group() {
  // the largest of 4 .. 1 passes that divides the tile's pass count
  constexpr int np = BM * (BN / 8) / NT;
  return np % 4 == 0 ? (np > 4 ? 4 : np) : np % 3 == 0 && np > 3 ? 3 : np % 2 == 0 ? 2 : 1;
}

// EARLY: the first pass group's operands were loaded by the kernel before
// its K loop (`early`, valid only when the launch has addend / xbn): their
// latency hides behind the GEMM instead of following it (short-K dgrads,
// where the epilogue's three extra streams are most of the bytes).
// ACC: v4f [BN/WGN/16][BM/WGM/16] (16x16x32 accumulators) or v16f
// [BN/WGN/32][BM/WGM/32] (32x32x16); only the LDS staging differs.
template <typename T, int BM, int BN, int NT, int WGM, int WGN, typename Pre = NoPrefetch,
          bool EXTRAS = true, bool EARLY = false, typename ACC>
__device__ __forceinline__ void ig_epilogue(const IgArgs& a, ACC& acc,
                                            T* smem, int m0, int n0, int wm, int wn,
                                            Pre pre = Pre(),
                                            const EpiOps<epi_group<BM, BN, NT>()>* early = nullptr) {
  constexpr bool M32 = std::is_same<std::decay_t<decltype(acc[0][0])>, v16f>::value;
  constexpr int TN = BN / WGN / 16, TM = BM / WGM / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int OHW = a.OH * a.OW;
  // Epilogue: lane holds channels n..n+3 of pixel m for each (i, j) subtile.
  // Stage the BM x BN tile through LDS (rows = pixels, 16-byte chunks
  // XOR-swizzled by row) so every global store is a full 16-byte lane write
  // and each pixel row goes out as one contiguous BN*2-byte run.
  T* __restrict__ y = (T*)a.y;
  T* cs = smem;  // reuse the operand buffers (the final __syncthreads above retired them)
  constexpr int CPR = BN / 8;  // 16-byte chunks per staged row
  // statistics shift of this thread's 8 channels (forward statistics only:
  // the host passes kshift only without addend / xbn, so the dgrad-style
  // branch - the epilogue's register peak - never holds it); issued before
  // the staging pass so its latency hides behind it
  float kv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int n = n0 + (tid % CPR) * 8 + k;
    kv[k] = (a.kshift && n < a.Ncol) ? a.kshift[n] : 0.f;
  }
  if constexpr (!M32) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int ml = wm * (BM / WGM) + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int nl = wn * (BN / WGN) + i * 16 + (lane >> 4) * 4;
        Vec<T, 4> o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o.v[r] = (T)acc[i][j][r];
        const int chunk = (nl >> 3) ^ (ml & (CPR - 1));
        *reinterpret_cast<Vec<T, 4>*>(cs + ml * BN + chunk * 8 + (nl & 7)) = o;
      }
    }
  } else {
    // 32x32 tiles: register group g of lane l = channels 8g + 4(l/32) .. +3
    // of pixel l % 32
#pragma unroll
    for (int j = 0; j < TM / 2; ++j) {
      const int ml = wm * (BM / WGM) + j * 32 + (lane & 31);
#pragma unroll
      for (int i = 0; i < TN / 2; ++i) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int nl = wn * (BN / WGN) + i * 32 + g * 8 + (lane >> 5) * 4;
          Vec<T, 4> o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o.v[r] = (T)acc[i][j][g * 4 + r];
          const int chunk = (nl >> 3) ^ (ml & (CPR - 1));
          *reinterpret_cast<Vec<T, 4>*>(cs + ml * BN + chunk * 8 + (nl & 7)) = o;
        }
      }
    }
  }
  __syncthreads();
  pre();
  const bool dense = (a.ys == 1 && a.YH == a.OH && a.YW == a.OW);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  // dgrad-style epilogue operands (EXTRAS = false: the kernel is never launched with them)
  const bool extras = EXTRAS && (a.addend || a.xbn);
  // this thread's 8 output channels are fixed (column tid % CPR of every pass)
  float mu[8], msc[8], msh[8];
  const bool mrec = a.xbn && !a.mask && a.mcoef;  // recompute the ReLU mask from xbn
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int n = n0 + (tid % CPR) * 8 + k;
    const bool nok = n < a.Ncol;
    mu[k] = (a.xbn && nok) ? a.mean[n] : 0.f;
    msc[k] = (mrec && nok) ? a.mcoef[n] : 0.f;
    msh[k] = (mrec && nok) ? a.mcoef[a.Ncol + n] : 0.f;
  }
  constexpr int NPASS = BM * CPR / NT;
  auto row_offset = [&](int m) -> long {
    if (dense) return (long)m * a.ldy;
    const int img = m / OHW, rem = m - img * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    return ((long)(img * a.YH + oh * a.ys) * a.YW + ow * a.ys) * a.ldy;
  };
  auto lds_chunk = [&](int t) -> uint4 {
    const int ml = t / CPR, ch = t % CPR;
    return *(const uint4*)(cs + ml * BN + ((ch ^ (ml & (CPR - 1))) * 8));
  };
  // Stores and loads share the in-order vmcnt counter: waiting for a load
  // issued after a store also waits for that store.  So the epilogue issues
  // no global load after its first store: the statistics-only path loads
  // nothing, and the dgrad-style path issues every extra-operand load (as
  // branch-free range-checked buffer loads) before any store.
  if (!extras) {
    const bool bact = a.bias || a.relu;
    float bv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int n = n0 + (tid % CPR) * 8 + k;
      bv[k] = (a.bias && n < a.Ncol) ? a.bias[n] : 0.f;
    }
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int t = tid + p * NT;
      const int m = m0 + t / CPR, n = n0 + (t % CPR) * 8;
      uint4 raw = lds_chunk(t);
      if (bact) {
        Vec<T, 8> tv = __builtin_bit_cast(Vec<T, 8>, raw);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float v = (float)tv.v[k] + bv[k];
          tv.v[k] = (T)(a.relu ? fmaxf(v, 0.f) : v);
        }
        raw = __builtin_bit_cast(uint4, tv);
      }
      if (m < a.M && n < a.Ncol) {
        if (a.stats) {
          const Vec<T, 8> tv = __builtin_bit_cast(Vec<T, 8>, raw);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = (float)tv.v[k] - kv[k];
            s1[k] += v;
            s2[k] += v * v;
          }
        }
        T* yp = y + row_offset(m) + n;
        *(uint4*)yp = raw;
        if (a.zfill) {
          const uint4 z = make_uint4(0, 0, 0, 0);
          *(uint4*)(yp + a.ldy) = z;
          *(uint4*)(yp + (long)a.YW * a.ldy) = z;
          *(uint4*)(yp + (long)(a.YW + 1) * a.ldy) = z;
        }
      }
    }
  } else if (EXTRAS && a.ybytes > 0) {
    const bool mbits = a.maskbits != 0;
    const EpiRsrc rs = epi_rsrc(a);
    // Passes go in groups of G: the extra-operand loads of group g+1 are
    // issued before group g is processed and stored, so they fly meanwhile
    // and a store never precedes the loads it would make wait (loads and
    // stores share the in-order vmcnt).  Small tiles (NPASS <= 4) form one
    // group: every load before any store.  Big tiles keep 2 groups of 3 x G
    // 16-byte operands in registers instead of 3 x NPASS.
    constexpr int G = epi_group<BM, BN, NT>();
    constexpr int NG = NPASS / G;
    static_assert(NPASS % G == 0, "pass groups");
    EpiOps<G> ops[2];
    if constexpr (EARLY) ops[0] = *early;
    else epi_load<T, BN, NT, G>(a, rs, m0, n0, 0, ops[0]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int b = g & 1;
      if (g + 1 < NG) epi_load<T, BN, NT, G>(a, rs, m0, n0, g + 1, ops[b ^ 1]);
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const uint4 raw = lds_chunk(tid + (g * G + q) * NT);
        const Vec<T, 8> tv = __builtin_bit_cast(Vec<T, 8>, raw);
        const Vec<T, 8> av = __builtin_bit_cast(Vec<T, 8>, ops[b].ad[q]);
        const Vec<T, 8> mv = __builtin_bit_cast(Vec<T, 8>, ops[b].mk[q]);
        const Vec<T, 8> xv = __builtin_bit_cast(Vec<T, 8>, ops[b].xb[q]);
        Vec<T, 8> ov;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float v = (float)tv.v[k] + (float)av.v[k];  // zero addend when absent
          if (a.xbn) {
            if (a.mask) {
              if (mbits) v = (ops[b].mk[q].x >> k) & 1u ? v : 0.f;
              else v = (float)mv.v[k] > 0.f ? v : 0.f;
            }
            // same expression as the BN apply (bn_apply_k), so the same sign
            else if (mrec) v = (float)xv.v[k] * msc[k] + msh[k] > 0.f ? v : 0.f;
            s1[k] += v;
            s2[k] += v * ((float)xv.v[k] - mu[k]);
          } else if (a.stats) {
            s1[k] += v;
            s2[k] += v * v;
          }
          ov.v[k] = (T)v;
        }
        if (ops[b].offb[q] >= 0) {
          char* yp = (char*)y + ops[b].offb[q];
          *(uint4*)yp = __builtin_bit_cast(uint4, ov);
          if (a.zfill) {
            const uint4 z = make_uint4(0, 0, 0, 0);
            const long rb = (long)a.ldy * sizeof(T);
            *(uint4*)(yp + rb) = z;
            *(uint4*)(yp + a.YW * rb) = z;
            *(uint4*)(yp + (a.YW + 1) * rb) = z;
          }
        }
      }
    }
  } else if (EXTRAS) {
    // outputs >= 2 GiB: plain loads interleaved with the stores
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int t = tid + p * NT;
      const int m = m0 + t / CPR, n = n0 + (t % CPR) * 8;
      if (m >= a.M || n >= a.Ncol) continue;
      const long off = row_offset(m) + n;
      const Vec<T, 8> tv = __builtin_bit_cast(Vec<T, 8>, lds_chunk(t));
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (float)tv.v[k];
      if (a.addend) {
        const Vec<T, 8> av = *(const Vec<T, 8>*)((const T*)a.addend + off);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += (float)av.v[k];
      }
      if (a.xbn) {
        if (a.mask && a.maskbits) {
          const unsigned mb = ((const uint8_t*)a.mask)[off >> 3];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = (mb >> k) & 1u ? v[k] : 0.f;
        } else if (a.mask) {
          const Vec<T, 8> mv = *(const Vec<T, 8>*)((const T*)a.mask + off);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = (float)mv.v[k] > 0.f ? v[k] : 0.f;
        }
        const Vec<T, 8> xv = *(const Vec<T, 8>*)((const T*)a.xbn + off);
        if (mrec) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = (float)xv.v[k] * msc[k] + msh[k] > 0.f ? v[k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s1[k] += v[k];
          s2[k] += v[k] * ((float)xv.v[k] - mu[k]);
        }
      } else if (a.stats) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s1[k] += v[k] - kv[k];
          s2[k] += (v[k] - kv[k]) * (v[k] - kv[k]);
        }
      }
      Vec<T, 8> ov;
#pragma unroll
      for (int k = 0; k < 8; ++k) ov.v[k] = (T)v[k];
      *(uint4*)(y + off) = __builtin_bit_cast(uint4, ov);
      if (a.zfill) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        *(uint4*)(y + off + a.ldy) = z;
        *(uint4*)(y + off + (long)a.YW * a.ldy) = z;
        *(uint4*)(y + off + (long)(a.YW + 1) * a.ldy) = z;
      }
    }
  }
  if (a.stats) {
    // Fold the per-thread sums of threads sharing a chunk column, then one
    // atomic add per channel per workgroup into a spread slot.  LDS-only
    // barriers: the tile's global stores stay in flight.
    lds_only_barrier();
    float* red = (float*)smem;  // [NT/CPR][CPR][16]
    const int ch = tid % CPR, rg = tid / CPR;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[(rg * CPR + ch) * 16 + k] = s1[k];
      red[(rg * CPR + ch) * 16 + 8 + k] = s2[k];
    }
    lds_only_barrier();
    constexpr int RG = NT / CPR;
    if (tid < CPR * 16) {
      const int c = tid / 16, k = tid % 16;
      float acc2 = 0.f;
      for (int r = 0; r < RG; ++r) acc2 += red[(r * CPR + c) * 16 + k];
      const int n = n0 + c * 8 + (k & 7);
      if (n < a.Ncol) {
        float* dst = a.stats + ((long)(k >> 3) * IG_SPREAD + (m0 / BM) % IG_SPREAD) * a.Ncol + n;
        atomicAdd(dst, acc2);
      }
    }
  }
}

// FAST (forward / stride-1 gather, C % 64 == 0, operands < 2 GiB): every
// 64-deep K step lies inside one filter tap, so the tap (kh, kw) and the
// channel offset advance as wave-uniform scalars; each pixel row carries a
// bitmask of its in-bounds taps, and operands are read with range-checked
// buffer loads (an out-of-range offset returns zeros), so the loads need no
// per-lane branches and no 64-bit address math.
//
// NBUF = 1: one LDS stage (the tile of step kt+1 waits in registers while
// step kt computes).  Half the LDS and <= 128 VGPRs give 4 workgroups per CU
// instead of 2; for the short-K layers (K = 64..128, e.g. the 56x56 1x1
// convs, one or two K steps) the kernel is latency/epilogue bound and the
// doubled occupancy is what hides it.
//
// 64 x 64 tiles (NBUF = 1): <= 96 VGPRs and 16 KB of LDS staging for 5
// workgroups (20 waves) per CU - more loads and stores in flight per CU, for
// the short-K, write-heavy layers (e.g. 1x1 convs with K = 64).

// (EARLY at 128 x 64: the early operands stay live through the K loop; 3
// workgroups per CU, <= 168 VGPRs, no spills)
template <typename T, int BM, int BN, bool TRANS, bool FAST, int NBUF = 2, bool EARLY = false>
__global__ void __launch_bounds__(256, BM * BN <= 4096 ? 5 : (EARLY ? 3 : (NBUF == 1 ? 4 : 2)))
    igemm_k(IgArgs a) {
  constexpr int XC = BM / 32;  // 16-byte X chunks per thread per K step
  constexpr int WC = BN / 32;  // 16-byte W chunks per thread per K step
  constexpr int TM = BM / 32;  // 16-wide pixel subtiles per wave
  constexpr int TN = BN / 32;  // 16-wide channel subtiles per wave
  static_assert(NBUF == 1 || NBUF == 2, "stages");
  static_assert(NBUF * (BM + BN) * IG_BK >= BM * BN, "epilogue staging exceeds LDS");
  __shared__ __attribute__((aligned(16))) T smem[NBUF * (BM + BN) * IG_BK];

  const T* __restrict__ x = (const T*)a.x;
  const T* __restrict__ w = (const T*)a.w;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.Ncol + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int m0 = (bid / ntiles) * BM, n0 = (bid % ntiles) * BN;
  const int kc = tid & 7;  // this thread's 16-byte chunk within a 64-wide K step
  const int OHW = a.OH * a.OW;

  // Per-thread pixel rows of the X tile.
  int xbase[XC], xh[XC], xw[XC];
  bool xok[XC];
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int m = m0 + (tid >> 3) + i * 32;
    xok[i] = m < a.M;
    const int mm = xok[i] ? m : 0;
    const int img = mm / OHW, rem = mm - img * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    xbase[i] = img * a.H * a.W * a.C;
    if (TRANS) { xh[i] = oh + a.pt; xw[i] = ow + a.pl; }
    else { xh[i] = oh * a.sh - a.pt; xw[i] = ow * a.sw - a.pl; }
  }
  const T* wrow[WC];
  bool wok[WC];
#pragma unroll
  for (int i = 0; i < WC; ++i) {
    const int n = n0 + (tid >> 3) + i * 32;
    wok[i] = n < a.Ncol;
    wrow[i] = w + (long)(wok[i] ? n : 0) * a.Ktot;
  }

  // X staging registers come in two sets: the X loads of K step t+2 are
  // issued at the top of step t and written to LDS at the bottom of step
  // t+1, so each has two steps of MFMA work (not one) to cover its latency.
  uint4 xr0[XC], wr0[WC], xr1[XC];
  // ---- FAST-path state
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, a.wbytes, 0x00020000);
  unsigned long long tapmask[XC];
  int xoff[XC], woff[WC];
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      unsigned long long mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw) {
          const bool in = (unsigned)(xh[i] + kh) < (unsigned)a.H &&
                          (unsigned)(xw[i] + kw) < (unsigned)a.W;
          mk |= (unsigned long long)(in && xok[i]) << (kh * a.KW + kw);
        }
      tapmask[i] = a.c8 ? mk >> kc : mk;  // 8-channel: bit 8s = this lane's tap of step s
      xoff[i] = xbase[i] + (xh[i] * a.W + xw[i]) * a.C + fast_lane_off(a, kc);
    }
#pragma unroll
    for (int i = 0; i < WC; ++i) woff[i] = (n0 + (tid >> 3) + i * 32) * a.Ktot + kc * 8;
  }
  // X and W have separate step counters: X runs one K step ahead of W.
  auto load_x = [&](uint4 (&xr)[XC], int kt) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < XC; ++i) {
        const bool ok = (tapmask[i] >> s_tapi) & 1ull;
        const int off = ok ? (xoff[i] + s_tap + s_cc) * (int)sizeof(T) : -1;
        xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      }
      if (a.c8) {
        s_tapi += 8;  // the 8 taps of the next step (lane kc's at bit kc)
        s_tap += a.c8_step;
      } else {
        s_cc += IG_BK;
        if (s_cc == a.C) {
          s_cc = 0;
          ++s_tapi;
          if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
          s_tap = (s_kh * a.W + s_kw) * a.C;
        }
      }
    } else {
      const int k = kt * IG_BK + kc * 8;
      const bool kok = k < a.Ktot;
      const int tap = a.fd_c.div(k), cc = k - tap * a.C;
      const int kh = a.fd_kw.div(tap), kw = tap - kh * a.KW;
#pragma unroll
      for (int i = 0; i < XC; ++i) {
        bool ok = kok && xok[i];
        int hi, wi;
        if (TRANS) {
          const int hh = xh[i] - kh, ww = xw[i] - kw;
          ok = ok && hh >= 0 && ww >= 0;
          hi = a.fd_sh.div(hh); wi = a.fd_sw.div(ww);  // hh, ww >= 0 when ok
          ok = ok && hi * a.sh == hh && wi * a.sw == ww && hi < a.H && wi < a.W;
        } else {
          hi = xh[i] + kh; wi = xw[i] + kw;
          ok = ok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        }
        xr[i] = ok ? *(const uint4*)(x + xbase[i] + (hi * a.W + wi) * a.C + cc)
                   : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto load_w = [&](uint4 (&wr)[WC], int kt) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < WC; ++i)
        wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                             wrs, (woff[i] + s_k) * (int)sizeof(T), 0, 0));
      s_k += IG_BK;
    } else {
      const int k = kt * IG_BK + kc * 8;
      const bool kok = k < a.Ktot;
#pragma unroll
      for (int i = 0; i < WC; ++i)
        wr[i] = (kok && wok[i]) ? *(const uint4*)(wrow[i] + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](const uint4 (&xr)[XC], const uint4 (&wr)[WC], int buf) {
    if constexpr (NBUF == 1) buf = 0;
    T* xs = smem + buf * (BM + BN) * IG_BK;
    T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int i = 0; i < XC; ++i) *(uint4*)(xs + swz_off((tid >> 3) + i * 32, kc)) = xr[i];
#pragma unroll
    for (int i = 0; i < WC; ++i) *(uint4*)(ws + swz_off((tid >> 3) + i * 32, kc)) = wr[i];
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int wn = wid >> 1, wm = wid & 1;
  const int nk = (a.Ktot + IG_BK - 1) / IG_BK;
  auto compute = [&](int buf) {
    if constexpr (NBUF == 1) buf = 0;
    const T* xs = smem + buf * (BM + BN) * IG_BK;
    const T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int ks = 0; ks < IG_BK / 32; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *(const v8s*)(ws + swz_off(wn * (BN / 2) + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / 2) + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
  };
  // The pixel (X) operand is loaded two K steps ahead through two register
  // sets; the weight operand (small, L2-resident) one step ahead through a
  // single set (a second set would spill at 128x128).
  load_x(xr0, 0);
  load_w(wr0, 0);
  // EARLY: the epilogue's first group of extra operands, issued behind the
  // first K step's operand loads (the in-order vmcnt lets the LDS store of
  // those wait for them alone)
  constexpr int EG = epi_group<BM, BN, 256>();
  EpiOps<EG> early;
  if constexpr (EARLY) {
    if (a.ybytes > 0 && (a.addend || a.xbn))
      epi_load<T, BN, 256, EG>(a, epi_rsrc(a), m0, n0, 0, early);
  }
  store(xr0, wr0, 0);
  // Only the FAST 128x128 kernel takes the second X set: the generic gather
  // would spill, and at 128x64 the extra registers cost a workgroup per CU
  // (measured slower).
  constexpr bool DEEP = FAST && BN > 64 && NBUF == 2;
  if constexpr (!DEEP) {
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) { load_x(xr0, kt + 1); load_w(wr0, kt + 1); }
      compute(kt & 1);
      if (kt + 1 < nk) {
        if constexpr (NBUF == 1) __syncthreads();  // every wave done reading the stage
        store(xr0, wr0, (kt + 1) & 1);
      }
      __syncthreads();
    }
  }
  if (DEEP && nk > 1) load_x(xr1, 1);
  if constexpr (DEEP) __syncthreads();
  // LDS buffer (kt & 1) holds step kt; X set 1 holds step kt+1 for even kt, set 0 for odd kt.
  for (int kt = 0; DEEP && kt < nk; kt += 2) {
    if (kt + 1 < nk) load_w(wr0, kt + 1);
    if (kt + 2 < nk) load_x(xr0, kt + 2);
    compute(0);
    if (kt + 1 < nk) store(xr1, wr0, 1);
    __syncthreads();
    if (kt + 1 >= nk) break;
    if (kt + 2 < nk) load_w(wr0, kt + 2);
    if (kt + 3 < nk) load_x(xr1, kt + 3);
    compute(1);
    if (kt + 2 < nk) store(xr0, wr0, 0);
    __syncthreads();
  }

  ig_epilogue<T, BM, BN, 256, 2, 2, NoPrefetch, true, EARLY>(a, acc, smem, m0, n0, wm, wn,
                                                             NoPrefetch(), &early);
  bn_fin_tail(a, (int*)smem);
}

// Multi-tile form of the FAST one-stage igemm_k: each workgroup computes TPW
// consecutive tiles (the channel tiles of one pixel tile, in order).  The
// first operand loads of tile t+1 are issued as soon as tile t's accumulators
// are staged in LDS, so they fly while tile t's output stores drain: the
// short-K write-heavy layers (one K step, then a 4x larger output) no longer
// run their load and store phases back to back in every workgroup.  Forward
// epilogues only (statistics / bias / ReLU): the host never launches it with
// the dgrad-style operands (addend, mask, xbn), whose loads would spill.
template <typename T, int BM, int BN, int TPW>
__global__ void __launch_bounds__(256, BM * BN <= 4096 ? 5 : 4) igemm_mt_k(IgArgs a) {
  constexpr int XC = BM / 32, WC = BN / 32;  // 16-byte X / W chunks per thread per K step
  constexpr int TM = BM / 32, TN = BN / 32;  // 16-wide pixel / channel subtiles per wave
  static_assert(TPW > 1, "one tile per workgroup: igemm_k");
  static_assert((BM + BN) * IG_BK >= BM * BN, "epilogue staging exceeds LDS");
  __shared__ __attribute__((aligned(16))) T smem[(BM + BN) * IG_BK];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.Ncol + BN - 1) / BN;
  const int ntot = mtiles * ntiles;
  const int bid = xcd_remap(blockIdx.x, (ntot + TPW - 1) / TPW);
  const int kc = tid & 7;  // this thread's 16-byte chunk within a 64-wide K step
  const int OHW = a.OH * a.OW;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);

  // per-tile loader state (setup) and the step counters (X and W advance together)
  unsigned long long tapmask[XC];
  int xoff[XC], woff[WC];
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  auto setup = [&](int tile) {
    const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int m = m0 + (tid >> 3) + i * 32;
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      const int img = mm / OHW, rem = mm - img * OHW;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const int xh = oh * a.sh - a.pt, xw = ow * a.sw - a.pl;
      unsigned long long mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw) {
          const bool in = (unsigned)(xh + kh) < (unsigned)a.H && (unsigned)(xw + kw) < (unsigned)a.W;
          mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
        }
      tapmask[i] = mk;
      xoff[i] = img * a.H * a.W * a.C + (xh * a.W + xw) * a.C + kc * 8;
    }
#pragma unroll
    for (int i = 0; i < WC; ++i) woff[i] = (n0 + (tid >> 3) + i * 32) * a.Ktot + kc * 8;
    s_cc = s_kh = s_kw = s_tap = s_tapi = s_k = 0;
  };
  uint4 xr[XC], wr[WC];
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const bool ok = (tapmask[i] >> s_tapi) & 1ull;
      const int off = ok ? (xoff[i] + s_tap + s_cc) * (int)sizeof(T) : -1;
      xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
    s_cc += IG_BK;
    if (s_cc == a.C) {
      s_cc = 0;
      ++s_tapi;
      if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
      s_tap = (s_kh * a.W + s_kw) * a.C;
    }
#pragma unroll
    for (int i = 0; i < WC; ++i)
      wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            wrs, (woff[i] + s_k) * (int)sizeof(T), 0, 0));
    s_k += IG_BK;
  };
  auto store = [&]() {
    T* xs = smem;
    T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int i = 0; i < XC; ++i) *(uint4*)(xs + swz_off((tid >> 3) + i * 32, kc)) = xr[i];
#pragma unroll
    for (int i = 0; i < WC; ++i) *(uint4*)(ws + swz_off((tid >> 3) + i * 32, kc)) = wr[i];
  };
  const int wn = wid >> 1, wm = wid & 1;
  const int nk = a.Ktot / IG_BK;  // FAST geometry: C % 64 == 0
  v4f acc[TN][TM];
  auto compute = [&]() {
    const T* xs = smem;
    const T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int ks = 0; ks < IG_BK / 32; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *(const v8s*)(ws + swz_off(wn * (BN / 2) + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / 2) + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
  };

  setup(bid * TPW);
  load();
#pragma unroll 1
  for (int t = 0; t < TPW; ++t) {
    const int tile = bid * TPW + t;
    if (tile >= ntot) break;  // workgroup-uniform
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    store();
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load();
      compute();
      if (kt + 1 < nk) {
        __syncthreads();  // every wave done reading the stage
        store();
      }
      __syncthreads();
    }
    const bool more = t + 1 < TPW && tile + 1 < ntot;
    auto next = [&]() {
      if (more) {
        setup(tile + 1);
        load();
      }
    };
    ig_epilogue<T, BM, BN, 256, 2, 2, decltype(next), false>(
        a, acc, smem, (tile / ntiles) * BM, (tile % ntiles) * BN, wm, wn, next);
    if (more) __syncthreads();  // the epilogue's LDS reads precede the next tile's store
  }
  bn_fin_tail(a, (int*)smem);
}

// ------------------------------------------------------------ LDS-DMA igemm
// FAST-geometry implicit GEMM whose operand tiles go global -> LDS by
// LDS-DMA (buffer_load_dwordx4 ... lds): no staging registers, no ds_write
// pass, and a 3-stage LDS ring so the loads of K step t+2 are in flight
// while step t computes (counted vmcnt + raw barrier; never vmcnt(0) in the
// loop).  512 threads = 8 waves as WGM (pixels) x WGN (channels); tile
// BM pixels x BN channels; one workgroup per CU (the ring is up to 144 KB).
//
// An LDS-DMA wave-instruction writes 1 KB linearly (lane l -> base + 16 l),
// i.e. 8 rows of the 128-byte-row image; the XOR swizzle of the fragment
// reads (swz_off) is applied on the SOURCE side instead: lane l fetches the
// logical 16-byte chunk (l & 7) ^ ((row >> 1) & 7) of its row.  Out-of-range
// offsets (padding taps, rows past M or Ncol) make the range-checked load
// write zeros into LDS (probed: scripts/probes/glds_oob.hip).
constexpr int GL_STAGES = 3;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // s_waitcnt simm16: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// One LDS-DMA piece: 16 bytes per lane from buffer offset `off` (bytes) to
// LDS base `lds` + 16 * lane.  A plain (non-template) device function: the
// host compilation pass drops a kernel template that names this builtin.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           off, 0, 0, 0);
}

__device__ __forceinline__ void lds_barrier() {
  // raw barrier: __syncthreads() would also drain vmcnt (the ring's DMAs)
  asm volatile("s_barrier" ::: "memory");
}

//
// STAGES = 2 (the "tall" 64-channel tiles, 2 workgroups or one 144 KB
// workgroup per CU): the DMAs of step t+1 are issued right after the barrier
// that retires step t and fly during compute(t); the wait at the top of each
// step is then vmcnt(0) (only that step's DMAs are outstanding).
// Workgroups per CU the register budget is sized for: the 128-row 4-wave
// tiles (48 / 64 KB rings) run 3 / 2 per CU, the rest one.
template <int BM, int BN, int NT>
constexpr int glds_occupancy() {
  return NT == 256 && BM == 128 ? (BN == 64 ? 3 : 2) : 1;
}

// MF32: 32x32x16 MFMAs (wave tiles must be multiples of 32 in both dims)
template <typename T, int BM, int BN, int WGM, int WGN, int STAGES = GL_STAGES,
          bool EXTRAS = true, bool MF32 = false>
__global__ void __launch_bounds__(WGM * WGN * 64, (glds_occupancy<BM, BN, WGM * WGN * 64>()))
    igemm_glds_k(IgArgs a) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int SLAB = NT / 8;  // rows one DMA instruction of every wave covers
  // pixel rows of the LDS tile: BM rounded up to whole DMA slabs (BM = 224:
  // 7 MFMA rows per wave, the slab rows past BM load nothing)
  constexpr int BMA = (BM + SLAB - 1) / SLAB * SLAB;
  static_assert(STAGES == 2 || STAGES == 3, "ring depth");
  static_assert(BN % SLAB == 0 && SLAB % 16 == 0 && BM % (16 * WGM) == 0, "DMA slabs");
  constexpr int TM = BM / WGM / 16, TN = BN / WGN / 16;
  constexpr int XI = BMA / SLAB, WI = BN / SLAB;  // DMA instructions per thread per K step
  constexpr int STAGE = (BMA + BN) * IG_BK;       // elements per ring stage
  static_assert(BM * BN <= STAGES * STAGE, "epilogue staging exceeds the ring");
  __shared__ __attribute__((aligned(16))) T smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.Ncol + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int m0 = (bid / ntiles) * BM, n0 = (bid % ntiles) * BN;
  const int OHW = a.OH * a.OW;
  const int rr = tid >> 3;                       // DMA row within each SLAB-row slab
  const int kc = (lane & 7) ^ ((rr >> 1) & 7);   // logical chunk this lane fetches

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  unsigned long long tapmask[XI];
  int xoff[XI], woff[WI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int m = m0 + i * SLAB + rr;
    const bool ok = m < a.M && (BMA == BM || i * SLAB + rr < BM);
    const int mm = ok ? m : 0;
    const int img = mm / OHW, rem = mm - img * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    const int xh = oh * a.sh - a.pt, xw = ow * a.sw - a.pl;
    unsigned long long mk = 0;
    for (int kh = 0; kh < a.KH; ++kh)
      for (int kw = 0; kw < a.KW; ++kw) {
        const bool in = (unsigned)(xh + kh) < (unsigned)a.H && (unsigned)(xw + kw) < (unsigned)a.W;
        mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
      }
    tapmask[i] = a.c8 ? mk >> kc : mk;  // 8-channel: bit 8s = this lane's tap of step s
    xoff[i] = img * a.H * a.W * a.C + (xh * a.W + xw) * a.C + fast_lane_off(a, kc);
  }
#pragma unroll
  for (int j = 0; j < WI; ++j) woff[j] = (n0 + j * SLAB + rr) * a.Ktot + kc * 8;

  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  auto issue = [&](int stage) {
    T* xs = smem + stage * STAGE;
    T* ws = xs + BMA * IG_BK;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const bool ok = (tapmask[i] >> s_tapi) & 1ull;
      const int off = ok ? (xoff[i] + s_tap + s_cc) * (int)sizeof(T) : -1;
      dma16(xrs, xs + (i * SLAB + wid * 8) * IG_BK, off);
    }
#pragma unroll
    for (int j = 0; j < WI; ++j)
      dma16(wrs, ws + (j * SLAB + wid * 8) * IG_BK, (woff[j] + s_k) * (int)sizeof(T));
    s_k += IG_BK;
    if (a.c8) {
      s_tapi += 8;  // the 8 taps of the next step (lane kc's at bit kc)
      s_tap += a.c8_step;
    } else {
      s_cc += IG_BK;
      if (s_cc == a.C) {
        s_cc = 0;
        ++s_tapi;
        if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
        s_tap = (s_kh * a.W + s_kw) * a.C;
      }
    }
  };

  static_assert(!MF32 || (TN % 2 == 0 && TM % 2 == 0), "32x32 wave tiles");
  constexpr int TN2 = MF32 ? TN / 2 : 1, TM2 = MF32 ? TM / 2 : 1;
  v4f acc[MF32 ? 1 : TN][MF32 ? 1 : TM];
  v16f acc32[TN2][TM2];
#pragma unroll
  for (int i = 0; i < (MF32 ? 1 : TN); ++i)
#pragma unroll
    for (int j = 0; j < (MF32 ? 1 : TM); ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < TN2; ++i)
#pragma unroll
    for (int j = 0; j < TM2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;
  const int wm = wid % WGM, wn = wid / WGM;
  auto compute = [&](int stage) {
    const T* xs = smem + stage * STAGE;
    const T* ws = xs + BMA * IG_BK;
    if constexpr (MF32) {
      // four 16-deep sub-steps; lane l reads chunk 2ks + l/32 of row l % 32
#pragma unroll
      for (int ks = 0; ks < IG_BK / 16; ++ks) {
        const int chunk = ks * 2 + (lane >> 5);
        v8s af[TN2], bfr[TM2];
#pragma unroll
        for (int i = 0; i < TN2; ++i)
          af[i] = *(const v8s*)(ws + swz_off(wn * (BN / WGN) + i * 32 + (lane & 31), chunk));
#pragma unroll
        for (int j = 0; j < TM2; ++j)
          bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / WGM) + j * 32 + (lane & 31), chunk));
#pragma unroll
        for (int i = 0; i < TN2; ++i)
#pragma unroll
          for (int j = 0; j < TM2; ++j) acc32[i][j] = Mfma32<T>::run(af[i], bfr[j], acc32[i][j]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < IG_BK / 32; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
        v8s af[TN], bfr[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i)
          af[i] = *(const v8s*)(ws + swz_off(wn * (BN / WGN) + i * 16 + (lane & 15), chunk));
#pragma unroll
        for (int j = 0; j < TM; ++j)
          bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / WGM) + j * 16 + (lane & 15), chunk));
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
      }
    }
  };

  const int nk = a.Ktot / IG_BK;  // FAST geometry: C % 64 == 0
  issue(0);
  if (STAGES == 3 && nk > 1) issue(1);
  int st = 0;  // stage of step kt
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 3) {
      // retire step kt's DMAs (step kt+1's, issued later, may stay in flight)
      if (kt + 1 < nk) wait_vmcnt<XI + WI>(); else wait_vmcnt<0>();
      lds_barrier();  // every wave's DMAs of step kt landed; stage (kt+2)%3 fully read
      if (kt + 2 < nk) issue(st == 0 ? 2 : st - 1);
      compute(st);  // (s_setprio(1) around it measured no faster)
      st = st == 2 ? 0 : st + 1;
    } else {
      wait_vmcnt<0>();  // step kt's DMAs (the only ones outstanding)
      lds_barrier();    // ... of every wave landed; stage st^1 (step kt-1) fully read
      if (kt + 1 < nk) issue(st ^ 1);
      compute(st);
      st ^= 1;
    }
  }
  __syncthreads();  // all fragment reads done before the epilogue reuses the ring
  if constexpr (MF32)
    ig_epilogue<T, BM, BN, NT, WGM, WGN, NoPrefetch, EXTRAS>(a, acc32, smem, m0, n0, wm, wn);
  else
    ig_epilogue<T, BM, BN, NT, WGM, WGN, NoPrefetch, EXTRAS>(a, acc, smem, m0, n0, wm, wn);
  bn_fin_tail(a, (int*)smem);
}

// Multi-tile form of the 4-wave 2-stage LDS-DMA kernel (128 x 64 / 128 x 128):
// each workgroup computes TPW consecutive tiles.  The epilogue stages its
// output tile in ring stage 1 while the DMAs of the next tile's first K step
// land in stage 0, so the next tile's loads are in flight while this tile's
// stores drain (igemm_mt_k does the same for the register-staged kernel).
template <typename T, int BM, int BN, int TPW>
__global__ void __launch_bounds__(256, (glds_occupancy<BM, BN, 256>()))
    igemm_glds_mt_k(IgArgs a) {
  constexpr int WGM = 2, WGN = 2, NT = 256;
  constexpr int SLAB = NT / 8;  // rows one DMA instruction of every wave covers
  static_assert(BM % SLAB == 0 && BN % SLAB == 0 && SLAB % 16 == 0, "DMA slabs");
  constexpr int TM = BM / WGM / 16, TN = BN / WGN / 16;
  constexpr int XI = BM / SLAB, WI = BN / SLAB;  // DMA instructions per thread per K step
  constexpr int STAGE = (BM + BN) * IG_BK;       // elements per ring stage
  static_assert(BM * BN <= STAGE && NT * 16 * 4 <= STAGE * (int)sizeof(T),
                "epilogue staging / statistics fold exceed one ring stage");
  static_assert(TPW > 1, "one tile per workgroup: igemm_glds_k");
  __shared__ __attribute__((aligned(16))) T smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.Ncol + BN - 1) / BN;
  const int ntot = mtiles * ntiles;
  const int bid = xcd_remap(blockIdx.x, (ntot + TPW - 1) / TPW);
  const int OHW = a.OH * a.OW;
  const int rr = tid >> 3;                       // DMA row within each SLAB-row slab
  const int kc = (lane & 7) ^ ((rr >> 1) & 7);   // logical chunk this lane fetches
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  unsigned long long tapmask[XI];
  int xoff[XI], woff[WI];
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  auto setup = [&](int tile) {
    const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int m = m0 + i * SLAB + rr;
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      const int img = mm / OHW, rem = mm - img * OHW;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const int xh = oh * a.sh - a.pt, xw = ow * a.sw - a.pl;
      unsigned long long mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw) {
          const bool in = (unsigned)(xh + kh) < (unsigned)a.H && (unsigned)(xw + kw) < (unsigned)a.W;
          mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
        }
      tapmask[i] = mk;
      xoff[i] = img * a.H * a.W * a.C + (xh * a.W + xw) * a.C + kc * 8;
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) woff[j] = (n0 + j * SLAB + rr) * a.Ktot + kc * 8;
    s_cc = s_kh = s_kw = s_tap = s_tapi = s_k = 0;
  };
  auto issue = [&](int stage) {
    T* xs = smem + stage * STAGE;
    T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const bool ok = (tapmask[i] >> s_tapi) & 1ull;
      const int off = ok ? (xoff[i] + s_tap + s_cc) * (int)sizeof(T) : -1;
      dma16(xrs, xs + (i * SLAB + wid * 8) * IG_BK, off);
    }
#pragma unroll
    for (int j = 0; j < WI; ++j)
      dma16(wrs, ws + (j * SLAB + wid * 8) * IG_BK, (woff[j] + s_k) * (int)sizeof(T));
    s_k += IG_BK;
    s_cc += IG_BK;
    if (s_cc == a.C) {
      s_cc = 0;
      ++s_tapi;
      if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
      s_tap = (s_kh * a.W + s_kw) * a.C;
    }
  };
  v4f acc[TN][TM];
  const int wm = wid % WGM, wn = wid / WGM;
  auto compute = [&](int stage) {
    const T* xs = smem + stage * STAGE;
    const T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int ks = 0; ks < IG_BK / 32; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *(const v8s*)(ws + swz_off(wn * (BN / WGN) + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / WGM) + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
  };

  const int nk = a.Ktot / IG_BK;  // FAST geometry: C % 64 == 0
  setup(bid * TPW);
  issue(0);
#pragma unroll 1
  for (int t = 0; t < TPW; ++t) {
    const int tile = bid * TPW + t;
    if (tile >= ntot) break;  // workgroup-uniform
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    // step 0 always sits in stage 0 (the previous epilogue staged in stage 1)
    int st = 0;
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt<0>();  // step kt's DMAs (and the previous tile's stores)
      lds_barrier();    // ... of every wave landed; stage st^1 fully read
      if (kt + 1 < nk) issue(st ^ 1);
      compute(st);
      st ^= 1;
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses the ring
    const bool more = t + 1 < TPW && tile + 1 < ntot;
    auto next = [&]() {
      if (more) {
        setup(tile + 1);
        issue(0);
      }
    };
    ig_epilogue<T, BM, BN, NT, WGM, WGN, decltype(next)>(
        a, acc, smem + STAGE, (tile / ntiles) * BM, (tile % ntiles) * BN, wm, wn, next);
  }
  bn_fin_tail(a, (int*)smem);
}

// ------------------------------------------------------------ 8-phase igemm
// 256 x 256 FAST-geometry tile on 8 waves (2 pixel halves x 4 channel
// quarters, 128 x 64 wave tiles) with the K-tile split into four phases of
// 16 MFMAs, one wave-tile quadrant each, and the two pixel-half wave groups
// running one barrier apart: while the waves of one group issue their
// quadrant's fragment reads and LDS-DMA prefetch, the other group's MFMAs
// run on the same SIMDs (a workgroup's waves w and w + 4 share a SIMD), so
// the fragment-read latency and issue slots hide behind the other group's
// matrix work (MI355X guide: the 256^2 8-phase template).
//
// LDS: two K-tile buffers of X [256][64] + W [256][64] (128 KB, one
// workgroup per CU), rows XOR-swizzled as in igemm_glds_k.  Each K-tile is
// moved as four half-tiles, one per phase, for the NEXT K-tile, in the order
// they are consumed: XA (pixel rows of quadrant half 0 of both groups), WA
// (channel rows of quadrant half 0 of every quarter), WB, XB; consumed in
// phases 0, 0, 1, 2.  Every barrier is preceded by vmcnt(4) (vmcnt(0) in the
// last K-tile): a half-tile is read >= 3 phases after its issue, so with the
// groups one barrier apart the two most recent half-tiles (4 DMAs per
// thread) may stay in flight and everything older has landed on every wave
// before the barrier the reader passes.  A buffer is overwritten 4 phases
// after its last read.
template <typename T, bool EXTRAS = true>
__global__ void __launch_bounds__(512, 1) igemm_8p_k(IgArgs a) {
  constexpr int BM = 256, BN = 256, NT = 512;
  constexpr int TM = 8, TN = 4;             // 16-wide pixel / channel subtiles per wave
  constexpr int STAGE = (BM + BN) * IG_BK;  // elements per K-tile buffer
  __shared__ __attribute__((aligned(16))) T smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;  // pixel half, channel quarter
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.Ncol + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int m0 = (bid / ntiles) * BM, n0 = (bid % ntiles) * BN;
  const int OHW = a.OH * a.OW;
  const int kc = (lane & 7) ^ ((tid >> 4) & 7);  // logical 16-byte chunk this lane fetches
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  // DMA slots s = 2 h + i (half h, instruction i): X row i*128 + h*64 + wid*8
  // + lane/8; W 8-row group g = 8 i + wid at (g/4)*64 + h*32 + (g%4)*8
  unsigned long long tapmask[4];
  int xoff[4], woff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int h = s >> 1, i = s & 1;
    const int m = m0 + i * 128 + h * 64 + wid * 8 + (lane >> 3);
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    const int img = mm / OHW, rem = mm - img * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    const int xh = oh * a.sh - a.pt, xw = ow * a.sw - a.pl;
    unsigned long long mk = 0;
    for (int kh = 0; kh < a.KH; ++kh)
      for (int kw = 0; kw < a.KW; ++kw) {
        const bool in = (unsigned)(xh + kh) < (unsigned)a.H && (unsigned)(xw + kw) < (unsigned)a.W;
        mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
      }
    tapmask[s] = mk;
    xoff[s] = img * a.H * a.W * a.C + (xh * a.W + xw) * a.C + kc * 8;
    const int g = i * 8 + wid;
    woff[s] = (n0 + (g >> 2) * 64 + h * 32 + (g & 3) * 8 + (lane >> 3)) * a.Ktot + kc * 8;
  }
  // K state of the K-tile being issued
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  auto advance = [&]() {
    s_k += IG_BK;
    s_cc += IG_BK;
    if (s_cc == a.C) {
      s_cc = 0;
      ++s_tapi;
      if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
      s_tap = (s_kh * a.W + s_kw) * a.C;
    }
  };
  auto issue_x = [&](int h, int buf) {
    T* xs = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int s = h * 2 + i;
      const bool ok = (tapmask[s] >> s_tapi) & 1ull;
      const int off = ok ? (xoff[s] + s_tap + s_cc) * (int)sizeof(T) : -1;
      dma16(xrs, xs + (i * 128 + h * 64 + wid * 8) * IG_BK, off);
    }
  };
  auto issue_w = [&](int h, int buf) {
    T* ws = smem + buf * STAGE + BM * IG_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int g = i * 8 + wid;
      dma16(wrs, ws + ((g >> 2) * 64 + h * 32 + (g & 3) * 8) * IG_BK,
            (woff[h * 2 + i] + s_k) * (int)sizeof(T));
    }
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s xf[4][2], wf0[2][2], wf1[2][2];
  auto read_x = [&](const T* xs, int ph) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        xf[j][ks] = *(const v8s*)(xs + swz_off(wr * 128 + ph * 64 + j * 16 + (lane & 15),
                                               ks * 4 + (lane >> 4)));
  };
  auto read_w = [&](const T* ws, int chh, v8s (&wf)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wf[i][ks] = *(const v8s*)(ws + swz_off(wc * 64 + chh * 32 + i * 16 + (lane & 15),
                                               ks * 4 + (lane >> 4)));
  };
  auto mfma = [&](int ph, int chh, const v8s (&wf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[chh * 2 + i][ph * 4 + j] =
              Mfma<T>::run(wf[i][ks], xf[j][ks], acc[chh * 2 + i][ph * 4 + j]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = a.Ktot / IG_BK;  // FAST geometry: C % 64 == 0
  issue_x(0, 0);
  issue_w(0, 0);
  issue_w(1, 0);
  issue_x(1, 0);
  advance();
  wait_vmcnt<0>();
  barrier();
  if (wr) barrier();  // group 1 runs one barrier behind group 0
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    const bool more = t + 1 < nk;
    const T* xs = smem + b * STAGE;
    const T* ws = xs + BM * IG_BK;
    auto sync = [&]() {
      if (more) wait_vmcnt<4>(); else wait_vmcnt<0>();
      barrier();
    };
    // phase 0: quadrant (pixel half 0, channel half 0)
    read_x(xs, 0);
    read_w(ws, 0, wf0);
    if (more) issue_x(0, b ^ 1);
    sync();
    mfma(0, 0, wf0);
    sync();
    // phase 1: (0, 1)
    read_w(ws, 1, wf1);
    if (more) issue_w(0, b ^ 1);
    sync();
    mfma(0, 1, wf1);
    sync();
    // phase 2: (1, 1)
    read_x(xs, 1);
    if (more) issue_w(1, b ^ 1);
    sync();
    mfma(1, 1, wf1);
    sync();
    // phase 3: (1, 0)
    if (more) {
      issue_x(1, b ^ 1);
      advance();
    }
    sync();
    mfma(1, 0, wf0);
    sync();
  }
  if (!wr) barrier();  // group 0 matches group 1's extra barrier
  __syncthreads();     // every fragment read done before the epilogue reuses the buffers
  ig_epilogue<T, BM, BN, NT, 2, 4, NoPrefetch, EXTRAS>(a, acc, smem, m0, n0, wr, wc);
  bn_fin_tail(a, (int*)smem);
}

// ------------------------------------------------------------ direct-B igemm
// The register-staged and LDS-DMA kernels above stage BOTH operands through
// LDS; with 2x2 wave grids every pixel chunk is written once and read by two
// waves, and the LDS pipe (not the MFMAs) bounds the 64- and 128-channel
// layers (~1.1 KB of LDS traffic per 16x16x32 MFMA at 128x64).  Here only the
// weight tile goes through LDS.  The four waves split the 256-pixel tile
// along M (64 pixels each, 64 output channels), so no pixel chunk is shared
// between waves and each lane loads its B fragments straight from global
// memory in MFMA layout: the 16-byte chunk (lane >> 4) of K sub-step ks of
// pixel (lane & 15) of subtile j - one buffer load per fragment, no LDS
// round trip.  The 64 x 64 weight tile of a K step (8 KB) is double-
// buffered in LDS (one 16-byte chunk per thread, two per step) and read as
// the A fragments.  LDS traffic per MFMA: ~0.3 KB.  B fragments of step k+1
// are loaded (two register sets) while step k computes.
// FAST geometry only (C % 64 == 0: a K step is one tap, 64 channels).
constexpr int DB_BM = 256, DB_BN = 64;

template <typename T>
__global__ void __launch_bounds__(256, 2) igemm_db_k(IgArgs a) {
  __shared__ __attribute__((aligned(16))) T smem[DB_BM * DB_BN];  // 2 A stages, then the epilogue
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mtiles = (a.M + DB_BM - 1) / DB_BM, ntiles = (a.Ncol + DB_BN - 1) / DB_BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int m0 = (bid / ntiles) * DB_BM, n0 = (bid % ntiles) * DB_BN;
  const int OHW = a.OH * a.OW;
  const int kc = lane >> 4;  // this lane's 16-byte chunk of a 32-deep K sub-step
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  // B: this lane's pixel of each of the wave's four 16-pixel subtiles
  int xoff[4];
  unsigned long long tapmask[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wid * 64 + j * 16 + (lane & 15);
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    const int img = mm / OHW, rem = mm - img * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    const int ih = oh * a.sh - a.pt, iw = ow * a.sw - a.pl;
    unsigned long long mk = 0;
    for (int kh = 0; kh < a.KH; ++kh)
      for (int kw = 0; kw < a.KW; ++kw) {
        const bool in = (unsigned)(ih + kh) < (unsigned)a.H && (unsigned)(iw + kw) < (unsigned)a.W;
        mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
      }
    tapmask[j] = mk;
    xoff[j] = img * a.H * a.W * a.C + (ih * a.W + iw) * a.C + kc * 8;
  }
  // A: weight rows n0 + (tid >> 3) and n0 + 32 + (tid >> 3), chunk tid & 7
  const int ar = tid >> 3, ac = tid & 7;
  const int woff0 = (n0 + ar) * a.Ktot + ac * 8, woff1 = (n0 + 32 + ar) * a.Ktot + ac * 8;
  const bool wok0 = n0 + ar < a.Ncol, wok1 = n0 + 32 + ar < a.Ncol;
  int s_k = 0;
  auto load_a = [&](uint4 (&wr)[2]) {
    wr[0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                          wrs, wok0 ? (woff0 + s_k) * (int)sizeof(T) : -1, 0, 0));
    wr[1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                          wrs, wok1 ? (woff1 + s_k) * (int)sizeof(T) : -1, 0, 0));
    s_k += IG_BK;
  };
  auto store_a = [&](const uint4 (&wr)[2], int buf) {
    T* ws = smem + buf * (DB_BN * IG_BK);
    *(uint4*)(ws + swz_off(ar, ac)) = wr[0];
    *(uint4*)(ws + swz_off(ar + 32, ac)) = wr[1];
  };
  // B state: tap (kh, kw), its bit, element offset of the tap, channel block
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0;
  auto load_b = [&](v8s (&br)[4][2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = (tapmask[j] >> s_tapi) & 1ull;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int off = ok ? (xoff[j] + s_tap + s_cc + ks * 32) * (int)sizeof(T) : -1;
        br[j][ks] = __builtin_bit_cast(v8s, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
      }
    }
    s_cc += IG_BK;
    if (s_cc == a.C) {
      s_cc = 0;
      ++s_tapi;
      if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
      s_tap = (s_kh * a.W + s_kw) * a.C;
    }
  };
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const v8s (&br)[4][2], int buf) {
    const T* ws = smem + buf * (DB_BN * IG_BK);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *(const v8s*)(ws + swz_off(i * 16 + (lane & 15), ks * 4 + kc));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::run(af[i], br[j][ks], acc[i][j]);
    }
  };
  const int nk = a.Ktot / IG_BK;
  uint4 wr[2];
  v8s b0[4][2], b1[4][2];
  load_a(wr);
  load_b(b0);
  store_a(wr, 0);
  __syncthreads();
  // step kt: A in LDS stage kt & 1, B in set (kt & 1 ? b1 : b0)
  for (int kt = 0; kt < nk; kt += 2) {
    if (kt + 1 < nk) { load_a(wr); load_b(b1); }
    compute(b0, 0);
    if (kt + 1 < nk) store_a(wr, 1);
    __syncthreads();
    if (kt + 1 >= nk) break;
    if (kt + 2 < nk) { load_a(wr); load_b(b0); }
    compute(b1, 1);
    if (kt + 2 < nk) store_a(wr, 0);
    __syncthreads();
  }
  ig_epilogue<T, DB_BM, DB_BN, 256, 4, 1>(a, acc, smem, m0, n0, wid, 0);
  bn_fin_tail(a, (int*)smem);
}

// ------------------------------------------------------------ stream-K igemm
// Persistent form of the 4-wave 128 x 128 LDS-DMA tile whose workgroups
// share the tail of the tile space along K.  A launch of T tiles on P
// resident workgroups (2 per CU) otherwise ends in a partial round: 784
// tiles (the 14x14 3x3 convs at batch 256) on 512 slots are 1.53 rounds run
// as 2, i.e. 23 % of the chip idles.  Here tiles [0, Tdp) run data-parallel
// (Tdp a multiple of P, tile w + r*P on workgroup w), and the K steps of the
// other Tsk = T - Tdp tiles (P + T % P of them, or all T when T < P) are cut
// into P equal contiguous ranges, one per workgroup, so every workgroup ends
// at the same time.  A tile whose K steps span several workgroups is summed
// by its last-arriving contributor: each contributor stores its fp32 partial
// tile (workspace slot 0 = the tile its range starts in, 1 = the tile it
// ends in; every other tile of a range is whole) with write-through stores,
// waits for them and takes a relaxed agent-scope ticket; the one that draws
// the last ticket acquires (agent scope), sums every contributor's partial in contributor
// order (so the result does not depend on who arrived last), resets the
// ticket for the next launch and runs the ordinary epilogue.  No workgroup
// ever waits for another, so nothing can deadlock whatever else occupies
// the chip (the weight-gradient side stream).  The split sums K in a
// different order than the one-tile kernels: the autotune's candidates no
// longer agree bitwise, only to fp32 rounding.
struct SkArgs {
  float* ws;  // [P][2][128 * 128] partial tiles
  int* cnt;   // [Tsk] tickets, zero between launches
  int T, nk, Tdp;
  long L;     // Tsk * nk: K steps of the stream-K region
  int probe;  // 1 (timing probe only, wrong results): no fix-up
};

// workgroup whose range holds step i of the stream-K region (P ranges of L)
__device__ __forceinline__ int sk_owner(long i, long L, int P) {
  return (int)(((i + 1) * P - 1) / L);
}

template <typename T>
__global__ void __launch_bounds__(256, 2) igemm_sk_k(IgArgs a, SkArgs sk) {
  constexpr int BM = 128, BN = 128, WGM = 2, WGN = 2, NT = 256;
  constexpr int SLAB = NT / 8;
  constexpr int TM = BM / WGM / 16, TN = BN / WGN / 16;
  constexpr int XI = BM / SLAB, WI = BN / SLAB;
  constexpr int STAGE = (BM + BN) * IG_BK;
  static_assert(BM * BN <= STAGE && NT * 16 * 4 <= STAGE * (int)sizeof(T), "epilogue staging");
  __shared__ __attribute__((aligned(16))) T smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int P = gridDim.x;
  const int w = xcd_remap(blockIdx.x, P);  // consecutive ranges share an XCD's L2
  const int ntiles = (a.Ncol + BN - 1) / BN;
  const int OHW = a.OH * a.OW;
  const int rr = tid >> 3;
  const int kc = (lane & 7) ^ ((rr >> 1) & 7);
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.wbytes, 0x00020000);
  unsigned long long tapmask[XI];
  int xoff[XI], woff[WI];
  int s_cc = 0, s_kh = 0, s_kw = 0, s_tap = 0, s_tapi = 0, s_k = 0;
  // operand offsets of `tile` and the K state of step k0
  auto setup = [&](int tile, int k0) {
    const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int m = m0 + i * SLAB + rr;
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      const int img = mm / OHW, rem = mm - img * OHW;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const int xh = oh * a.sh - a.pt, xw = ow * a.sw - a.pl;
      unsigned long long mk = 0;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw) {
          const bool in = (unsigned)(xh + kh) < (unsigned)a.H && (unsigned)(xw + kw) < (unsigned)a.W;
          mk |= (unsigned long long)(in && ok) << (kh * a.KW + kw);
        }
      tapmask[i] = mk;
      xoff[i] = img * a.H * a.W * a.C + (xh * a.W + xw) * a.C + kc * 8;
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) woff[j] = (n0 + j * SLAB + rr) * a.Ktot + kc * 8;
    s_k = k0 * IG_BK;
    s_tapi = s_k / a.C;
    s_cc = s_k - s_tapi * a.C;
    s_kh = s_tapi / a.KW;
    s_kw = s_tapi - s_kh * a.KW;
    s_tap = (s_kh * a.W + s_kw) * a.C;
  };
  auto issue = [&](int stage) {
    T* xs = smem + stage * STAGE;
    T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const bool ok = (tapmask[i] >> s_tapi) & 1ull;
      const int off = ok ? (xoff[i] + s_tap + s_cc) * (int)sizeof(T) : -1;
      dma16(xrs, xs + (i * SLAB + wid * 8) * IG_BK, off);
    }
#pragma unroll
    for (int j = 0; j < WI; ++j)
      dma16(wrs, ws + (j * SLAB + wid * 8) * IG_BK, (woff[j] + s_k) * (int)sizeof(T));
    s_k += IG_BK;
    s_cc += IG_BK;
    if (s_cc == a.C) {
      s_cc = 0;
      ++s_tapi;
      if (++s_kw == a.KW) { s_kw = 0; ++s_kh; }
      s_tap = (s_kh * a.W + s_kw) * a.C;
    }
  };
  v4f acc[TN][TM];
  const int wm = wid % WGM, wn = wid / WGM;
  auto compute = [&](int stage) {
    const T* xs = smem + stage * STAGE;
    const T* ws = xs + BM * IG_BK;
#pragma unroll
    for (int ks = 0; ks < IG_BK / 32; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *(const v8s*)(ws + swz_off(wn * (BN / WGN) + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *(const v8s*)(xs + swz_off(wm * (BM / WGM) + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
  };

  // Work items: the data-parallel tiles w, w + P, ... < Tdp, then the K
  // range [i, e) of the stream-K region cut at tile boundaries.
  int dp = w;
  long si = (long)w * sk.L / P;
  const long se = (long)(w + 1) * sk.L / P;
  auto next_item = [&](int& tile, int& k0, int& k1) -> bool {
    if (dp < sk.Tdp) {
      tile = dp;
      k0 = 0;
      k1 = sk.nk;
      dp += P;
      return true;
    }
    if (si >= se) return false;
    const int tl = (int)(si / sk.nk);
    k0 = (int)(si - (long)tl * sk.nk);
    k1 = (se - si) < (long)(sk.nk - k0) ? k0 + (int)(se - si) : sk.nk;
    tile = sk.Tdp + tl;
    si += k1 - k0;
    return true;
  };

  int tile, k0, k1;
  bool have = next_item(tile, k0, k1);
  if (have) {
    setup(tile, k0);
    issue(0);
  }
  volatile int* flag = (volatile int*)smem;  // stage 0, read before any later DMA lands there
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)sk.ws, (short)0, (int)((long)P * 2 * BM * BN * sizeof(float)), 0x00020000);
#pragma unroll 1
  while (have) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    int st = 0;  // every item's first step sits in stage 0
    for (int kt = k0; kt < k1; ++kt) {
      wait_vmcnt<0>();
      lds_barrier();
      if (kt + 1 < k1) issue(st ^ 1);
      compute(st);
      st ^= 1;
    }
    __syncthreads();  // fragment reads done: the ring is free
    int ntile = 0, nk0 = 0, nk1 = 0;
    const bool more = next_item(ntile, nk0, nk1);
    auto next = [&]() {
      if (more) {
        setup(ntile, nk0);
        issue(0);
      }
    };
    const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
    bool finish = (k0 == 0 && k1 == sk.nk) || sk.probe;
    if (!finish) {
      // partial tile: publish it, and sum the tile if this is the last piece
      const int tl = tile - sk.Tdp;
      const long t0 = (long)tl * sk.nk;
      const int c0 = sk_owner(t0, sk.L, P), c1 = sk_owner(t0 + sk.nk - 1, sk.L, P);
      auto slot_of = [&](int c) -> float* {
        const int first_tile = (int)(((long)c * sk.L / P) / sk.nk);
        return sk.ws + ((long)c * 2 + (first_tile == tl ? 0 : 1)) * (BM * BN);
      };
      // write-through (sc1) stores: visible past this XCD's L2 once waited
      // for, so no release fence (an agent release writes back every dirty
      // line of the L2, this launch's output tiles included)
      const int pbase = (int)((slot_of(w) - sk.ws) * sizeof(float));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[i][j]), wsr,
                                                 pbase + ((i * TM + j) * NT + tid) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int prev =
            __hip_atomic_fetch_add(sk.cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == c1 - c0;
        if (last) {
          __hip_atomic_store(sk.cnt + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
      }
      __syncthreads();
      finish = __builtin_amdgcn_readfirstlane(*flag) != 0;
      lds_barrier();  // every wave has read the flag before stage 0 is reused
      if (finish) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
        for (int c = c0; c <= c1; ++c) {
          const int cbase = (int)((slot_of(c) - sk.ws) * sizeof(float));
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
              acc[i][j] += __builtin_bit_cast(
                  v4f, __builtin_amdgcn_raw_buffer_load_b128(
                           wsr, cbase + ((i * TM + j) * NT + tid) * 16, 0, 16));
        }
      }
    }
    if (finish)
      ig_epilogue<T, BM, BN, NT, WGM, WGN, decltype(next)>(a, acc, smem + STAGE, m0, n0, wm, wn,
                                                           next);
    else
      next();
    tile = ntile;
    k0 = nk0;
    k1 = nk1;
    have = more;
  }
}

// ------------------------------------------------------------------ wgrad
struct WgArgs {
  const void* dy;  // [M][Ncol]  (NHWC output gradient, Ncol = Cout)
  const void* x;   // NHWC input [N,H,W,C]
  float* dw;       // [Ncol][Ktot] fp32, accumulated atomically
  int N, H, W, C;
  int OH, OW;
  int KH, KW, sh, sw, pt, pl;
  int Ncol, Ktot, M;
  int mper;        // rows of m per split
  int dybytes, xbytes;  // GATHER / PLAIN loaders: operand byte sizes (< 2 GiB)
  // slab != null: each split stores its partial dW tile with plain stores to
  // slab[split][Ncol][Ktot] (every element of every split is written) and
  // wgrad_reduce_k folds the slabs into dw; else fp32 atomics into dw.
  float* slab;
  FastDiv fd_ohw, fd_ow;  // WG_GENERIC: the per-step row -> (img, oh, ow)
};

constexpr int WG_BK = 32;  // reduction rows per step (64 measured no faster)
// waves per SIMD the wgrad register budget is sized for: 2 lets the 128x128
// tiles use 134-142 VGPRs (3 workgroups per CU); 4 (<= 128 VGPRs) spills in
// the main loop and measured 2.5x slower on the 1x1 wgrads
// (profiles/r5_wgrad_occupancy_ab.txt)
#define WG_OCC 2
constexpr bool WG_XCD = true;  // XCD-aware workgroup order (r4_wgrad_xcd_ab.txt)

// 256-byte rows (128 elements); 32-byte unit u (0..7) of row r stored at
// u ^ f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2.
__device__ __forceinline__ int tr_off(int row, int col) {
  const int f = (row & 3) | (((row >> 3) & 1) << 2);
  const int u = col >> 4;
  return row * 128 + (((u ^ f) << 4) | (col & 15));
}

template <typename T>
__device__ __forceinline__ v4s ds_read_tr(const T* p) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}

// Loader modes: WG_GENERIC re-derives (img, oh, ow) of every row each step;
// WG_GATHER walks them incrementally (wave-uniform step of WG_BK rows) and
// reads with range-checked buffer loads; WG_PLAIN (1x1, stride 1, no
// padding) reads x rows as a plain [M][C] matrix.  GATHER/PLAIN need both
// operands < 2 GiB.
enum { WG_GENERIC = 0, WG_GATHER = 1, WG_PLAIN = 2 };

template <typename T, int BMC, int BNK, int MODE>
__global__ void __launch_bounds__(256, WG_OCC) wgrad_k(WgArgs a) {
  // BMC = output-channel tile (rows of dW), BNK = k tile (cols of dW); both 128 or 64.
  constexpr int TN = BMC / 32, TM = BNK / 32;
  constexpr int DC = WG_BK * BMC / 8 / 256;  // dy chunks per thread
  constexpr int XC = WG_BK * BNK / 8 / 256;  // x chunks per thread
  __shared__ __attribute__((aligned(16))) T smem[2 * WG_BK * 256];  // [buf][dy 32x128 | x 32x128]

  const T* __restrict__ dy = (const T*)a.dy;
  const T* __restrict__ x = (const T*)a.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ctiles = (a.Ncol + BMC - 1) / BMC, ktiles = (a.Ktot + BNK - 1) / BNK;
  const int tiles = ctiles * ktiles;
  // XCD-aware order: the tiles of one reduction split (which read the same
  // dy rows and overlapping x rows) get consecutive remapped ids, i.e. one
  // XCD and its L2; the hardware's round-robin order spread them over 8 L2s
  // (4-11% L2 hit rate on the 56x56 3x3 wgrad).
  const int bid = WG_XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int c0 = (tile / ktiles) * BMC, k0 = (tile % ktiles) * BNK;
  const int mbeg = split * a.mper;
  const int mend = min(a.M, mbeg + a.mper);
  const int OHW = a.OH * a.OW;

  // Loader geometry: dy rows are m (WG_BK per step), BMC/8 chunks per row.
  constexpr int DCPR = BMC / 8, XCPR = BNK / 8;
  int dcol[DC], drow[DC];
#pragma unroll
  for (int i = 0; i < DC; ++i) {
    const int c = tid + i * 256;
    drow[i] = c / DCPR;
    dcol[i] = (c % DCPR) * 8;
  }
  // x chunks: fixed k per thread (col), row = m
  int xcol[XC], xrow[XC], xtap_h[XC], xtap_w[XC], xcc[XC];
  bool xkok[XC];
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int c = tid + i * 256;
    xrow[i] = c / XCPR;
    xcol[i] = (c % XCPR) * 8;
    const int k = k0 + xcol[i];
    xkok[i] = k < a.Ktot;
    const int tap = k / a.C;
    xcc[i] = k - tap * a.C;
    xtap_h[i] = tap / a.KW;
    xtap_w[i] = tap - xtap_h[i] * a.KW;
  }
  uint4 dr[DC], xr[XC];
  // ---- incremental (GATHER / PLAIN) loader state
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, a.xbytes, 0x00020000);
  int doff[DC], xo[XC], ximg[XC], xoh[XC], xow[XC], xh0[XC], xw0[XC];
  bool dcok[DC];
  int s_m = mbeg;  // first row of the next step to load
  const int dq = WG_BK / a.OW, dr_ = WG_BK - dq * a.OW;
  if constexpr (MODE != WG_GENERIC) {
#pragma unroll
    for (int i = 0; i < DC; ++i) {
      dcok[i] = c0 + dcol[i] < a.Ncol;
      doff[i] = (mbeg + drow[i]) * a.Ncol + c0 + dcol[i];
    }
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int m = mbeg + xrow[i];
      if constexpr (MODE == WG_PLAIN) {
        xo[i] = m * a.C + xcc[i];
      } else {
        ximg[i] = m / OHW;
        const int rem = m - ximg[i] * OHW;
        xoh[i] = rem / a.OW;
        xow[i] = rem - xoh[i] * a.OW;
        xh0[i] = xtap_h[i] - a.pt;
        xw0[i] = xtap_w[i] - a.pl;
      }
    }
  }
  auto load_inc = [&]() {
#pragma unroll
    for (int i = 0; i < DC; ++i) {
      const bool ok = dcok[i] && s_m + drow[i] < mend;
      dr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            drs, ok ? doff[i] * (int)sizeof(T) : -1, 0, 0));
      doff[i] += WG_BK * a.Ncol;
    }
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const bool mok = xkok[i] && s_m + xrow[i] < mend;
      int off;
      if constexpr (MODE == WG_PLAIN) {
        off = mok ? xo[i] * (int)sizeof(T) : -1;
        xo[i] += WG_BK * a.C;
      } else {
        const int hi = xoh[i] * a.sh + xh0[i], wi = xow[i] * a.sw + xw0[i];
        const bool ok = mok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        off = ok ? (((ximg[i] * a.H + hi) * a.W + wi) * a.C + xcc[i]) * (int)sizeof(T) : -1;
        xow[i] += dr_;
        xoh[i] += dq;
        if (xow[i] >= a.OW) { xow[i] -= a.OW; ++xoh[i]; }
        while (xoh[i] >= a.OH) { xoh[i] -= a.OH; ++ximg[i]; }
      }
      xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
    s_m += WG_BK;
  };
  auto load = [&](int mstep) {
    if constexpr (MODE != WG_GENERIC) { load_inc(); return; }
#pragma unroll
    for (int i = 0; i < DC; ++i) {
      const int m = mstep + drow[i];
      const int col = c0 + dcol[i];
      dr[i] = (m < mend && col < a.Ncol) ? *(const uint4*)(dy + (long)m * a.Ncol + col)
                                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int m = mstep + xrow[i];
      bool ok = xkok[i] && m < mend;
      const int mm = ok ? m : 0;
      const int img = a.fd_ohw.div(mm), rem = mm - img * OHW;
      const int oh = a.fd_ow.div(rem), ow = rem - oh * a.OW;
      const int hi = oh * a.sh - a.pt + xtap_h[i], wi = ow * a.sw - a.pl + xtap_w[i];
      ok = ok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      xr[i] = ok ? *(const uint4*)(x + ((long)(img * a.H + hi) * a.W + wi) * a.C + xcc[i])
                 : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
    T* ds = smem + buf * WG_BK * 256;
    T* xs = ds + WG_BK * 128;
#pragma unroll
    for (int i = 0; i < DC; ++i) *(uint4*)(ds + tr_off(drow[i], dcol[i])) = dr[i];
#pragma unroll
    for (int i = 0; i < XC; ++i) *(uint4*)(xs + tr_off(xrow[i], xcol[i])) = xr[i];
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int wn = wid >> 1, wm = wid & 1;
  // Transposed-read addressing: group g = lane>>4 needs rows 8g..8g+7
  // (two reads of 4 rows); lane 4q+p of the group addresses row q, cols 4p..4p+3.
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int nsteps = (mend - mbeg + WG_BK - 1) / WG_BK;
  if (nsteps > 0) {
    load(mbeg);
    store(0);
  }
  __syncthreads();
  int cur = 0;
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) load(mbeg + (s + 1) * WG_BK);
    const T* ds = smem + cur * WG_BK * 256;
    const T* xs = ds + WG_BK * 128;
#pragma unroll
    for (int kk = 0; kk < WG_BK / 32; ++kk) {
      const int r0 = kk * 32 + 8 * g;
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int col = wn * (BMC / 2) + i * 16 + 4 * p;
        v4s lo = ds_read_tr<T>(ds + tr_off(r0 + q, col));
        v4s hi = ds_read_tr<T>(ds + tr_off(r0 + 4 + q, col));
        af[i] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int col = wm * (BNK / 2) + j * 16 + 4 * p;
        v4s lo = ds_read_tr<T>(xs + tr_off(r0 + q, col));
        v4s hi = ds_read_tr<T>(xs + tr_off(r0 + 4 + q, col));
        bfr[j] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
    if (s + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // acc[i][j]: rows (dW output channel) c0 + wn*BMC/2 + i*16 + (lane>>4)*4 + r,
  // col (k) k0 + wm*BNK/2 + j*16 + (lane&15).
  if (a.slab) {
    // Plain-store slab epilogue: stage half the tile (BMC/2 rows x BNK fp32)
    // at a time through LDS so each lane stores 16 contiguous bytes of a row.
    // Float atomics run at the memory side at ~1.3 TB/s (every lane-dword an
    // uncached request); plain 16-byte stores stream at ~6 TB/s.
    constexpr int HR = BMC / 2;              // rows per half (one wave row wn)
    constexpr int LDR = BNK;  // ds_write_b32 rows 4 apart: 2-way, free per the LDS table
    static_assert(HR * LDR * 4 <= (int)sizeof(smem), "slab staging exceeds LDS");
    float* st = (float*)smem;
    float* dst = a.slab + (long)split * a.Ncol * a.Ktot;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (wn == h) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              st[(i * 16 + (lane >> 4) * 4 + r) * LDR + wm * (BNK / 2) + j * 16 + (lane & 15)] =
                  acc[i][j][r];
      }
      __syncthreads();
      constexpr int CPR = BNK / 4;  // float4 chunks per row
#pragma unroll
      for (int t = tid; t < HR * CPR; t += 256) {
        const int row = t / CPR, cc = (t % CPR) * 4;
        const int c = c0 + h * HR + row, k = k0 + cc;
        if (c < a.Ncol && k < a.Ktot)
          *(float4*)(dst + (long)c * a.Ktot + k) = *(const float4*)(st + row * LDR + cc);
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int k = k0 + wm * (BNK / 2) + j * 16 + (lane & 15);
      if (k >= a.Ktot) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + wn * (BMC / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (c < a.Ncol) atomicAdd(a.dw + (long)c * a.Ktot + k, acc[i][j][r]);
      }
    }
}

// LDS-DMA form of wgrad_k (128 x 128 dW tiles, 4 waves of 64 x 64): both
// operand tiles go global -> LDS by buffer_load ... lds into a 2-stage ring
// of 64-row steps (2 x 32 KB, two workgroups per CU), so there is no
// register staging, no ds_write pass and half the barriers per reduction row
// of the register-staged kernel (32-row steps).  The LDS images keep
// wgrad_k's 256-byte rows with XOR-swizzled 32-byte units (tr_off) for the
// transposed fragment reads; the swizzle moves to the source side: a DMA
// wave-instruction fills 4 rows linearly, lane l writing 16-byte chunk l & 15
// of row l >> 4, so it fetches the logical chunk that tr_off maps there.
// Row (l >> 4) & 3 and bit 3 of the row (the wave's 4-row group parity) fix
// that chunk, so each lane's columns (and for 3x3 gathers its filter tap and
// channel) are constant over the whole reduction.
template <typename T, int MODE>
__global__ void __launch_bounds__(256, 2) wgrad_glds_k(WgArgs a) {
  constexpr int BMC = 128, BNK = 128, TN = 4, TM = 4, BK = 64;
  constexpr int STAGE = 2 * BK * 128;  // dy [64][128] + x [64][128] elements
  __shared__ __attribute__((aligned(16))) T smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ctiles = (a.Ncol + BMC - 1) / BMC, ktiles = (a.Ktot + BNK - 1) / BNK;
  const int tiles = ctiles * ktiles;
  const int bid = WG_XCD ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int c0 = (tile / ktiles) * BMC, k0 = (tile % ktiles) * BNK;
  const int mbeg = split * a.mper;
  const int mend = min(a.M, mbeg + a.mper);
  const int OHW = a.OH * a.OW;

  // this lane's logical 8-element column chunk (see above)
  const int lrow = lane >> 4;                                  // row within the 4-row group
  const int f = lrow | (((wid >> 1) & 1) << 2);                // tr_off's f(row)
  const int pc = lane & 15;                                    // physical 16-byte chunk
  const int col = ((((pc >> 1) ^ f) << 4) | ((pc & 1) << 3));  // logical column
  const int n = c0 + col, k = k0 + col;
  const bool nok = n < a.Ncol, kok = k < a.Ktot;
  const int tap = kok ? k / a.C : 0, cc = k - tap * a.C;
  const int kh = tap / a.KW, kw = tap - kh * a.KW;
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  // rows of DMA instruction i (0..3) at step s: mbeg + s*64 + i*16 + wid*4 + lrow
  int doff[4], ximg[4], xoh[4], xow[4], xo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mbeg + i * 16 + wid * 4 + lrow;
    doff[i] = m * a.Ncol + n;
    if constexpr (MODE == WG_PLAIN) {
      xo[i] = m * a.C + cc;
    } else {
      ximg[i] = m / OHW;
      const int rem = m - ximg[i] * OHW;
      xoh[i] = rem / a.OW;
      xow[i] = rem - xoh[i] * a.OW;
    }
  }
  const int dq = BK / a.OW, dr = BK - dq * a.OW;
  int s_m = mbeg;  // first row of the next step to issue
  auto issue = [&](int stage) {
    T* ds = smem + stage * STAGE;
    T* xs = ds + BK * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i * 16 + wid * 4;  // first LDS row of this wave-instruction
      const bool mok = s_m + r + lrow < mend;
      dma16(drs, ds + r * 128, (mok && nok) ? doff[i] * (int)sizeof(T) : -1);
      doff[i] += BK * a.Ncol;
      int off;
      if constexpr (MODE == WG_PLAIN) {
        off = (mok && kok) ? xo[i] * (int)sizeof(T) : -1;
        xo[i] += BK * a.C;
      } else {
        const int hi = xoh[i] * a.sh - a.pt + kh, wi = xow[i] * a.sw - a.pl + kw;
        const bool ok = mok && kok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
        off = ok ? (((ximg[i] * a.H + hi) * a.W + wi) * a.C + cc) * (int)sizeof(T) : -1;
        xow[i] += dr;
        xoh[i] += dq;
        if (xow[i] >= a.OW) { xow[i] -= a.OW; ++xoh[i]; }
        while (xoh[i] >= a.OH) { xoh[i] -= a.OH; ++ximg[i]; }
      }
      dma16(xrs, xs + r * 128, off);
    }
    s_m += BK;
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int wn = wid >> 1, wm = wid & 1;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto compute = [&](int stage) {
    const T* ds = smem + stage * STAGE;
    const T* xs = ds + BK * 128;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int r0 = kk * 32 + 8 * g;
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int cl = wn * (BMC / 2) + i * 16 + 4 * p;
        v4s lo = ds_read_tr<T>(ds + tr_off(r0 + q, cl));
        v4s hi = ds_read_tr<T>(ds + tr_off(r0 + 4 + q, cl));
        af[i] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int cl = wm * (BNK / 2) + j * 16 + 4 * p;
        v4s lo = ds_read_tr<T>(xs + tr_off(r0 + q, cl));
        v4s hi = ds_read_tr<T>(xs + tr_off(r0 + 4 + q, cl));
        bfr[j] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
  };

  const int nsteps = (mend - mbeg + BK - 1) / BK;
  if (nsteps > 0) issue(0);
  int st = 0;
  for (int s = 0; s < nsteps; ++s) {
    wait_vmcnt<0>();  // this step's DMAs (the only ones outstanding)
    lds_barrier();    // ... of every wave landed; stage st^1 (step s-1) fully read
    if (s + 1 < nsteps) issue(st ^ 1);
    compute(st);
    st ^= 1;
  }
  __syncthreads();  // every fragment read done before the epilogue reuses the ring
  // acc[i][j]: dW row c0 + wn*64 + i*16 + (lane>>4)*4 + r, col k0 + wm*64 + j*16 + (lane&15)
  if (a.slab) {
    constexpr int HR = BMC / 2, LDR = BNK;
    static_assert(HR * LDR * 4 <= (int)sizeof(smem), "slab staging exceeds LDS");
    float* stg = (float*)smem;
    float* dst = a.slab + (long)split * a.Ncol * a.Ktot;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (wn == h) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              stg[(i * 16 + (lane >> 4) * 4 + r) * LDR + wm * (BNK / 2) + j * 16 + (lane & 15)] =
                  acc[i][j][r];
      }
      __syncthreads();
      constexpr int CPR = BNK / 4;
#pragma unroll
      for (int t = tid; t < HR * CPR; t += 256) {
        const int row = t / CPR, cq = (t % CPR) * 4;
        const int c = c0 + h * HR + row, kq = k0 + cq;
        if (c < a.Ncol && kq < a.Ktot)
          *(float4*)(dst + (long)c * a.Ktot + kq) = *(const float4*)(stg + row * LDR + cq);
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int kq = k0 + wm * (BNK / 2) + j * 16 + (lane & 15);
      if (kq >= a.Ktot) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + wn * (BMC / 2) + i * 16 + (lane >> 4) * 4 + r;
        if (c < a.Ncol) atomicAdd(a.dw + (long)c * a.Ktot + kq, acc[i][j][r]);
      }
    }
}

// dw[i] += sum_s slab[s][i]   (n4 = elements / 4), one thread per float4.
__global__ void __launch_bounds__(256) wgrad_reduce_k(const float4* __restrict__ slab,
                                                      float4* __restrict__ dw, long n4,
                                                      int nsplit) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 acc = dw[i];
    int s = 0;
    for (; s + 4 <= nsplit; s += 4) {  // four independent loads in flight
      const float4 v0 = slab[(long)s * n4 + i], v1 = slab[(long)(s + 1) * n4 + i];
      const float4 v2 = slab[(long)(s + 2) * n4 + i], v3 = slab[(long)(s + 3) * n4 + i];
      acc.x += (v0.x + v1.x) + (v2.x + v3.x);
      acc.y += (v0.y + v1.y) + (v2.y + v3.y);
      acc.z += (v0.z + v1.z) + (v2.z + v3.z);
      acc.w += (v0.w + v1.w) + (v2.w + v3.w);
    }
    for (; s < nsplit; ++s) {
      const float4 v = slab[(long)s * n4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    dw[i] = acc;
  }
}

// Small dW with many splits: blockIdx.y sums a group of splits for one float
// per thread and adds it atomically (lane-contiguous: one 256-byte run per
// wave-instruction).
__global__ void __launch_bounds__(256) wgrad_reduce_grouped_k(const float* __restrict__ slab,
                                                              float* __restrict__ dw, long n,
                                                              int nsplit) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n) return;
  const int s0 = (int)((long)nsplit * blockIdx.y / gridDim.y);
  const int s1 = (int)((long)nsplit * (blockIdx.y + 1) / gridDim.y);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = s0;
  for (; s + 4 <= s1; s += 4) {
    a0 += slab[(long)s * n + i];
    a1 += slab[(long)(s + 1) * n + i];
    a2 += slab[(long)(s + 2) * n + i];
    a3 += slab[(long)(s + 3) * n + i];
  }
  for (; s < s1; ++s) a0 += slab[(long)s * n + i];
  atomicAdd(dw + i, (a0 + a1) + (a2 + a3));
}

// kfb_set_deterministic(1): weight-gradient slab folds run in one fixed
// order (no grouped atomic fold); for bitwise run-to-run comparisons
static int g_deterministic = 0;

static bool igemm_fast_disabled() { return false; }

template <typename T>
static void launch_glds_tall(const IgArgs& a, bool wide, hipStream_t s) {
  // 64-channel tiles with 64x64 wave tiles and a 2-stage ring: 512 x 64 on 8
  // waves (144 KB, one workgroup per CU) or 256 x 64 on 4 waves (80 KB, two)
  const int nt = (a.Ncol + 63) / 64;
  if (wide)
    hipLaunchKernelGGL((igemm_glds_k<T, 512, 64, 8, 1, 2>), dim3(((a.M + 511) / 512) * nt),
                       dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_glds_k<T, 256, 64, 4, 1, 2>), dim3(((a.M + 255) / 256) * nt),
                       dim3(256), 0, s, a);
}

template <typename T>
static void launch_glds(const IgArgs& a, bool narrow, hipStream_t s) {
  const int mt = (a.M + 255) / 256;
  if (a.Ncol <= 64 || narrow)
    hipLaunchKernelGGL((igemm_glds_k<T, 256, 64, 8, 1>), dim3(mt * ((a.Ncol + 63) / 64)), dim3(512),
                       0, s, a);
  else
    hipLaunchKernelGGL((igemm_glds_k<T, 256, 128, 4, 2>), dim3(mt * ((a.Ncol + 127) / 128)),
                       dim3(512), 0, s, a);
}

// 128-row tiles on 4 waves through a 2-stage LDS-DMA ring: 128 x 64 (48 KB,
// three workgroups per CU, 64 x 32 wave tiles as igemm_k's) or 128 x 128
// (64 KB, two per CU, 64 x 64 wave tiles): no staging registers and no
// ds_write pass (the register-staged igemm_k spends more LDS cycles on its
// ds_write_b128 stores than on its fragment reads)
template <typename T>
static void launch_glds_short(const IgArgs& a, bool wide, bool three, hipStream_t s,
                              bool mf32 = false) {
  const int mt = (a.M + 127) / 128;
  const dim3 g128(mt * ((a.Ncol + 127) / 128)), g64(mt * ((a.Ncol + 63) / 64));
  if (mf32 && wide)
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 128, 2, 2, 2, true, true>), g128, dim3(256), 0, s, a);
  else if (mf32)
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 64, 2, 2, 2, true, true>), g64, dim3(256), 0, s, a);
  else if (wide && three)
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 128, 2, 2, 3>), g128, dim3(256), 0, s, a);
  else if (wide)
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 128, 2, 2, 2>), g128, dim3(256), 0, s, a);
  else if (three)
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 64, 2, 2, 3>), g64, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_glds_k<T, 128, 64, 2, 2, 2>), g64, dim3(256), 0, s, a);
}

// Big-tile LDS-DMA kernels, one 8-wave workgroup per CU with 128 x 64 wave
// tiles (twice the MFMAs per fragment read of the 64 x 64 wave tiles, and
// half the L2 bytes per MFMA of the 256 x 128 workgroup tile): 256 x 256 for
// >= 256 output channels (2 x 64 KB ring), 512 x 128 for 128-channel layers
// (2 x 80 KB ring, the whole 160 KB LDS).
template <typename T>
static void launch_glds_big(const IgArgs& a, bool wide, hipStream_t s, bool mf32 = false) {
  if (mf32)
    hipLaunchKernelGGL((igemm_glds_k<T, 256, 256, 2, 4, 2, true, true>),
                       dim3(((a.M + 255) / 256) * ((a.Ncol + 255) / 256)), dim3(512), 0, s, a);
  else if (wide)
    hipLaunchKernelGGL((igemm_glds_k<T, 256, 256, 2, 4, 2>),
                       dim3(((a.M + 255) / 256) * ((a.Ncol + 255) / 256)), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_glds_k<T, 512, 128, 4, 2, 2>),
                       dim3(((a.M + 511) / 512) * ((a.Ncol + 127) / 128)), dim3(512), 0, s, a);
}

// 224 x 256 tiles on the same 8 waves (7 x 4 MFMA tiles per wave): where M
// is 196 pixels per image (14x14), 224-row tiles give 224 tiles instead of
// 196 256-row ones on 256 CUs - 7/8 of the work per tile with every CU used
template <typename T>
static void launch_glds_224(const IgArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((igemm_glds_k<T, 224, 256, 2, 4, 2>),
                     dim3(((a.M + 223) / 224) * ((a.Ncol + 255) / 256)), dim3(512), 0, s, a);
}

// 448 x 128 (waves 4 x 2 of 112 x 64): for the 128-channel layers, 448 tiles
// at 28x28 batch 256 (1.75 rounds on 256 CUs) where 512 x 128 has 392 (1.53)
template <typename T>
static void launch_glds_448(const IgArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((igemm_glds_k<T, 448, 128, 4, 2, 2>),
                     dim3(((a.M + 447) / 448) * ((a.Ncol + 127) / 128)), dim3(512), 0, s, a);
}

template <typename T>
static void launch_8p(const IgArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((igemm_8p_k<T>), dim3(((a.M + 255) / 256) * ((a.Ncol + 255) / 256)),
                     dim3(512), 0, s, a);
}

// Multi-tile 4-wave LDS-DMA kernels, 2 tiles per workgroup.
template <typename T>
static void launch_glds_mt(const IgArgs& a, bool wide, hipStream_t s) {
  const int mt = (a.M + 127) / 128;
  if (wide)
    hipLaunchKernelGGL((igemm_glds_mt_k<T, 128, 128, 2>), dim3((mt * ((a.Ncol + 127) / 128) + 1) / 2),
                       dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_glds_mt_k<T, 128, 64, 2>), dim3((mt * ((a.Ncol + 63) / 64) + 1) / 2),
                       dim3(256), 0, s, a);
}

// Multi-tile FAST kernels (64-channel tiles: 128 x 64 or 64 x 64; the 128 x
// 128 form spills), forward-style epilogues only.
template <typename T, int BM>
static void launch_mt(const IgArgs& a, int tpw, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + 63) / 64);
  if (tpw == 4)
    hipLaunchKernelGGL((igemm_mt_k<T, BM, 64, 4>), dim3((nwg + 3) / 4), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_mt_k<T, BM, 64, 2>), dim3((nwg + 1) / 2), dim3(256), 0, s, a);
}

// Stream-K launch: P = CUs x resident workgroups, per-(device, stream)
// workspace (partial tiles + tickets) allocated on first use and kept (a
// recorded launch tape replays the same pointers; kernels of one stream run
// in order, so one workspace per stream is never shared by two launches in
// flight).
struct SkWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;
  int P = 0;
};

template <typename T>
static hipError_t launch_sk(const IgArgs& a, hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, SkWorkspace> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  SkWorkspace wsp;
  {
    std::lock_guard<std::mutex> g(mu);
    SkWorkspace& c = cache[{dev, s}];
    if (!c.ws) {
      int cus = 0, per = 0;
      e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (e != hipSuccess) return e;
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, igemm_sk_k<T>, 256, 0);
      if (e != hipSuccess) return e;
      if (per < 1) per = 1;
      const int P = cus * per;
      e = hipMalloc((void**)&c.ws, (size_t)P * 2 * 128 * 128 * sizeof(float));
      if (e != hipSuccess) return e;
      e = hipMalloc((void**)&c.cnt, (size_t)2 * P * sizeof(int));
      if (e != hipSuccess) return e;
      e = kfb::memset_async(c.cnt, 0, (size_t)2 * P * sizeof(int), s);
      if (e != hipSuccess) return e;
      c.P = P;
    }
    wsp = c;
  }
  const int P = wsp.P;
  const int tiles = ((a.M + 127) / 128) * ((a.Ncol + 127) / 128);
  SkArgs sk;
  sk.ws = wsp.ws;
  sk.cnt = wsp.cnt;
  sk.T = tiles;
  sk.nk = a.Ktot / IG_BK;
  // stream-K region: the last partial round plus one full round (or all of
  // a launch smaller than one round); none when the rounds come out even
  const int Tsk = tiles < P ? tiles : (tiles % P == 0 ? 0 : P + tiles % P);
  sk.Tdp = tiles - Tsk;
  sk.L = (long)Tsk * sk.nk;
  const int probe = 0;  // (1: timing probe without the fix-up; 2: + geometry print)
  sk.probe = probe;
  const int grid = (sk.Tdp > 0 || sk.L >= P) ? P : (int)sk.L;
  if (grid < 1) return hipSuccess;
  if (probe >= 2)
    fprintf(stderr, "[sk] P %d tiles %d nk %d Tdp %d L %ld grid %d\n", P, tiles, sk.nk, sk.Tdp, sk.L,
            grid);
  hipLaunchKernelGGL(igemm_sk_k<T>, dim3(grid), dim3(256), 0, s, a, sk);
  return hipGetLastError();
}

template <typename T, int BM, int BN>
static void launch_ig(const IgArgs& a, bool trans, bool fast, hipStream_t s, bool onebuf = false,
                      bool early = false) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + BN - 1) / BN);
  if (early && fast && onebuf)
    hipLaunchKernelGGL((igemm_k<T, BM, BN, false, true, 1, true>), dim3(nwg), dim3(256), 0, s, a);
  else if (early && fast)
    hipLaunchKernelGGL((igemm_k<T, BM, BN, false, true, 2, true>), dim3(nwg), dim3(256), 0, s, a);
  else if (onebuf && fast)
    hipLaunchKernelGGL((igemm_k<T, BM, BN, false, true, 1>), dim3(nwg), dim3(256), 0, s, a);
  else if (trans)
    hipLaunchKernelGGL((igemm_k<T, BM, BN, true, false>), dim3(nwg), dim3(256), 0, s, a);
  else if (fast)
    hipLaunchKernelGGL((igemm_k<T, BM, BN, false, true>), dim3(nwg), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_k<T, BM, BN, false, false>), dim3(nwg), dim3(256), 0, s, a);
}

// Reduction split of a wgrad launch: ~target_blocks workgroups, >= 8 steps
// per workgroup; returns the split count and the rows per split.
static int wgrad_split(int M, int Ktot, int Ncol, int target_blocks, int* mper_out) {
  const int bmc = Ncol <= 64 ? 64 : 128;
  const int tiles = ((Ncol + bmc - 1) / bmc) * ((Ktot + 127) / 128);
  int split = target_blocks > 0 ? target_blocks / tiles : 1024 / tiles;
  const int max_split = (M + WG_BK * 8 - 1) / (WG_BK * 8);
  if (split > max_split) split = max_split;
  if (split < 1) split = 1;
  const int mper = ((M + split - 1) / split + WG_BK - 1) / WG_BK * WG_BK;
  if (mper_out) *mper_out = mper;
  return (M + mper - 1) / mper;
}

template <typename T, int BMC>
static void launch_wg(const WgArgs& a, int mode, dim3 grid, hipStream_t s) {
  if (mode == WG_PLAIN)
    hipLaunchKernelGGL((wgrad_k<T, BMC, 128, WG_PLAIN>), grid, dim3(256), 0, s, a);
  else if (mode == WG_GATHER)
    hipLaunchKernelGGL((wgrad_k<T, BMC, 128, WG_GATHER>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((wgrad_k<T, BMC, 128, WG_GENERIC>), grid, dim3(256), 0, s, a);
}

}  // namespace kfb

using namespace kfb;

// Kernel choice (algo): IG_ALGO_CLASSIC = register-staged 128-tile igemm_k,
// IG_ALGO_GLDS = LDS-DMA ring igemm_glds_k (FAST geometry only; others fall
// back to igemm_k).  The _N64 variants force the 64-channel-wide tile for
// Ncol > 64: twice the workgroups, which pays where 128-wide tiles leave the
// last wave of workgroups mostly empty (small-M stage-4/5 layers: 784 tiles
// on 512 slots is 1.5 waves).  ops/conv_hip.py times the candidates per
// geometry.
//   IG_ALGO_ONEBUF(_N64): FAST igemm_k with one LDS stage (4 workgroups/CU).
//   IG_ALGO_TALL512 / TALL256: igemm_glds_k with 64-channel tiles and 64x64
//   wave tiles (twice the MFMAs per fragment read of the 256x64 8-wave tile).
//   IG_ALGO_SMALL: FAST igemm_k with 64x64 tiles, one LDS stage, 5 workgroups/CU.
//   IG_ALGO_GSHORT64 / GSHORT128 (_3): igemm_glds_k 128x64 / 128x128 on 4 waves,
//   2-stage (3-stage) ring.
//   IG_ALGO_MULTI2 / MULTI4: igemm_mt_k, the 128 x 64 ONEBUF kernel with 2 / 4
//   tiles per workgroup (the next tile's loads overlap this tile's output
//   stores); IG_ALGO_SMALL_MULTI4: 64 x 64 tiles, 4 per workgroup.
//   IG_ALGO_GMULTI64 / GMULTI128: igemm_glds_mt_k, GSHORT64 / GSHORT128 with 2
//   tiles per workgroup (next tile's DMAs land in stage 0 while the epilogue
//   stages in stage 1).  IG_ALGO_SK128: igemm_sk_k, the GSHORT128 tile
//   persistent with the last partial round split along K.  IG_ALGO_G8P:
//   igemm_8p_k, the 256 x 256 tile with the 8-phase staggered schedule.  Forward-style
//   epilogues only: with addend / mask / xbn they fall through to the
//   one-tile kernels.
enum { IG_ALGO_CLASSIC = 1, IG_ALGO_GLDS = 2, IG_ALGO_CLASSIC_N64 = 3, IG_ALGO_GLDS_N64 = 4,
       IG_ALGO_ONEBUF = 5, IG_ALGO_ONEBUF_N64 = 6, IG_ALGO_TALL512 = 7, IG_ALGO_TALL256 = 8,
       IG_ALGO_SMALL = 9, IG_ALGO_GSHORT64 = 10, IG_ALGO_GSHORT128 = 11,
       IG_ALGO_GSHORT64_3 = 12, IG_ALGO_GSHORT128_3 = 13, IG_ALGO_MULTI2 = 14,
       IG_ALGO_MULTI4 = 15, IG_ALGO_SMALL_MULTI4 = 16, IG_ALGO_GMULTI64 = 17,
       IG_ALGO_GMULTI128 = 18, IG_ALGO_GBIG256 = 19, IG_ALGO_GBIG512 = 20,
       IG_ALGO_GENERIC = 21, IG_ALGO_SK128 = 22, IG_ALGO_G8P = 23, IG_ALGO_ONEBUF_E = 24,
       IG_ALGO_ONEBUF_N64_E = 25, IG_ALGO_CLASSIC_N64_E = 26, IG_ALGO_DB = 27,
       IG_ALGO_GBIG256_32 = 28, IG_ALGO_GSHORT128_32 = 29, IG_ALGO_GSHORT64_32 = 30,
       IG_ALGO_S3 = 31, IG_ALGO_S1 = 32, IG_ALGO_S7 = 33, IG_ALGO_GBIG224 = 34,
       IG_ALGO_GBIG448 = 35 };

static bool c8_geometry(int C, int KH, int KW) {
  return C == 8 && (KW == 1 || KW == 2 || KW == 4 || KW == 8) && (KH * KW) % 8 == 0;
}

KFB_API int kfb_conv_igemm_fast(int C, int KH, int KW, int trans) {
  return !trans && (C % IG_BK == 0 || c8_geometry(C, KH, KW)) && KH * KW <= 64 &&
         !igemm_fast_disabled();
}

// Forward conv or dgrad (trans=1) or scattered 1x1 GEMM (ys>1).
// Requirements: C % 8 == 0, Ncol % 4 == 0, 16-byte aligned pointers.
KFB_API hipError_t kfb_conv_igemm(int dtype, const void* x, const void* w, void* y, int N, int H,
                                  int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                                  int pt, int pl, int Ncol, int YH, int YW, int ys, int ldy,
                                  int trans, float* stats, const void* mask, const void* xbn,
                                  const float* mean, const void* addend, const float* mcoef,
                                  const float* bias, int flags, int algo, const float* kshift,
                                  int* fin_counter, const float* fin_gamma,
                                  const float* fin_beta, float* fin_rm, float* fin_rv,
                                  float* fin_mean, float* fin_invstd, float* fin_scale,
                                  float* fin_shift, float fin_decay, float fin_eps,
                                  hipStream_t stream) {
  // fin_counter != null (forward statistics epilogue only): the consuming
  // BN's finalize runs in the last workgroup (BnFin); the BN forward then
  // skips its finalize launch
  // flags: bit 0 = ReLU after the bias (forward epilogue), bit 1 = zero-fill
  // the unsampled pixels of a stride-2 scatter (see IgArgs::zfill), bit 2 =
  // `mask` is a ReLU bit mask (see IgArgs::maskbits), bit 3 = statistics
  // only: the streaming 1x1 kernel (IG_ALGO_S1) sums the output's BN
  // statistics without storing it (its consumer recomputes it,
  // kfb_bn_fwd_train_recompute)
  if (C % 8 || Ncol % 8) return hipErrorInvalidValue;
  const int relu = flags & 1, zfill = (flags >> 1) & 1;
  if (zfill && !(ys == 2 && YH == 2 * OH && YW == 2 * OW)) return hipErrorInvalidValue;
  const long xbytes = (long)N * H * W * C * 2, wbytes = (long)Ncol * KH * KW * C * 2;
  const long ybytes = (long)N * YH * YW * ldy * 2;
  IgArgs a{x, w, y, N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol, KH * KW * C,
           N * OH * OW, YH, YW, ys, ldy, stats, mask, xbn, mean, addend, mcoef, bias, relu,
           (int)(xbytes < (1L << 31) ? xbytes : 0), (int)(wbytes < (1L << 31) ? wbytes : 0),
           (int)(ybytes < (1L << 31) ? ybytes : 0),
           (stats && !xbn && !addend) ? kshift : nullptr,
           FastDiv(C), FastDiv(KW), FastDiv(sh), FastDiv(sw), zfill, 0, 0,
           (mask && ((flags >> 2) & 1)) ? 1 : 0};
  // With a dgrad-style epilogue (xbn != null) the fin_* arguments carry the
  // producer BN's backward finalize instead (BnGFin): fin_gamma = gamma,
  // fin_invstd = its saved invstd, fin_rm / fin_rv = dgamma / dbeta,
  // fin_scale / fin_shift / fin_mean = coefA / coefB / coefC, fin_decay != 0:
  // accumulate into dgamma / dbeta.
  const bool gfin = fin_counter && xbn;
  if (gfin) {
    if (!stats || ys != 1) return hipErrorInvalidValue;
    a.gfin = BnGFin{fin_counter, fin_gamma, fin_invstd, fin_rm, fin_rv, fin_scale, fin_shift,
                    fin_mean, fin_decay != 0.f ? 1 : 0};
  } else if (fin_counter) {
    if (!stats || xbn || addend || ys != 1) return hipErrorInvalidValue;
    a.fin = BnFin{fin_counter, fin_gamma, fin_beta, fin_rm, fin_rv, fin_mean, fin_invstd,
                  fin_scale, fin_shift, const_cast<float*>(kshift), fin_decay, fin_eps,
                  (long)N * OH * OW};
  }
  const bool t = trans != 0;
  // IG_ALGO_GENERIC: the per-chunk division loader (autotune candidate for
  // the 8-channel geometry, where it can beat the FAST tap stepping)
  const bool c8 = !t && C % IG_BK != 0 && c8_geometry(C, KH, KW) && algo != IG_ALGO_GENERIC;
  if (c8) {
    a.c8 = 1;
    a.c8_step = (8 / KW) * W * C;
  }
  const bool fast = !t && (C % IG_BK == 0 || c8) && KH * KW <= 64 && xbytes < (1L << 31) &&
                    wbytes < (1L << 31) && !igemm_fast_disabled() && algo != IG_ALGO_GENERIC;
  // (the early-epilogue forms exist at 128 x 64 only: 128 x 128 spills)
  const bool narrow = algo == IG_ALGO_CLASSIC_N64 || algo == IG_ALGO_GLDS_N64 ||
                      algo == IG_ALGO_ONEBUF_N64 || algo == IG_ALGO_ONEBUF_N64_E ||
                      algo == IG_ALGO_CLASSIC_N64_E || algo == IG_ALGO_ONEBUF_E;
  const bool onebuf = algo == IG_ALGO_ONEBUF || algo == IG_ALGO_ONEBUF_N64 ||
                      algo == IG_ALGO_ONEBUF_E || algo == IG_ALGO_ONEBUF_N64_E;
  // the early-epilogue forms (dgrad-style operands loaded before the K loop)
  const bool early = algo == IG_ALGO_ONEBUF_E || algo == IG_ALGO_ONEBUF_N64_E ||
                     algo == IG_ALGO_CLASSIC_N64_E;
  // IG_ALGO_S3: the streaming 3x3 64-channel kernel (conv_stream.hip); off
  // its geometry the default kernel below runs
  if (algo == IG_ALGO_S3 && fast && !c8 && conv_s3_fits(a)) return launch_conv_s3(dtype, a, stream);
  // IG_ALGO_S1: the streaming 1x1 K -> 4K-channel kernel (conv_s1.hip)
  if ((flags >> 3) & 1) {  // statistics only: S1 with its stores dropped
    if (algo != IG_ALGO_S1 || !stats || xbn || addend || !fast || c8) return hipErrorInvalidValue;
    a.ybytes = 0;
    if (!conv_s1_fits(a)) return hipErrorInvalidValue;
    return launch_conv_s1(dtype, a, stream);
  }
  if (algo == IG_ALGO_S1 && fast && !c8 && conv_s1_fits(a)) return launch_conv_s1(dtype, a, stream);
  // IG_ALGO_S7: the streaming stem conv over the pixel-pair view (conv_s7.hip)
  if (algo == IG_ALGO_S7 && !t && conv_s7_fits(a)) return launch_conv_s7(dtype, a, stream);
  if (gfin) {
    // only the persistent kernels above carry the backward finalize tail:
    // any other kernel runs without it and the finalize is launched after
    a.gfin = BnGFin{};
    const hipError_t e = kfb_conv_igemm(dtype, x, w, y, N, H, W, C, OH, OW, KH, KW, sh, sw, pt,
                                        pl, Ncol, YH, YW, ys, ldy, trans, stats, mask, xbn, mean,
                                        addend, mcoef, bias, flags, algo, kshift, nullptr, nullptr,
                                        nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                        nullptr, 0.f, 0.f, stream);
    if (e != hipSuccess) return e;
    return bn_finalize_grad_launch(stats, Ncol, (long)N * OH * OW, fin_gamma, mean, fin_invstd,
                                   fin_rm, fin_rv, fin_scale, fin_shift, fin_mean,
                                   fin_decay != 0.f ? 1 : 0, stream);
  }
  if ((algo == IG_ALGO_TALL512 || algo == IG_ALGO_TALL256) && fast) {
    if (dtype == BF16) launch_glds_tall<bf16>(a, algo == IG_ALGO_TALL512, stream);
    else if (dtype == F16) launch_glds_tall<f16>(a, algo == IG_ALGO_TALL512, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo >= IG_ALGO_GSHORT64 && algo <= IG_ALGO_GSHORT128_3 && fast) {
    const bool wide = algo == IG_ALGO_GSHORT128 || algo == IG_ALGO_GSHORT128_3;
    const bool three = algo >= IG_ALGO_GSHORT64_3;
    if (dtype == BF16) launch_glds_short<bf16>(a, wide, three, stream);
    else if (dtype == F16) launch_glds_short<f16>(a, wide, three, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo == IG_ALGO_GBIG448 && fast) {
    if (dtype == BF16) launch_glds_448<bf16>(a, stream);
    else if (dtype == F16) launch_glds_448<f16>(a, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo == IG_ALGO_GBIG224 && fast) {
    if (dtype == BF16) launch_glds_224<bf16>(a, stream);
    else if (dtype == F16) launch_glds_224<f16>(a, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if ((algo == IG_ALGO_GBIG256 || algo == IG_ALGO_GBIG512) && fast) {
    if (dtype == BF16) launch_glds_big<bf16>(a, algo == IG_ALGO_GBIG256, stream);
    else if (dtype == F16) launch_glds_big<f16>(a, algo == IG_ALGO_GBIG256, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo == IG_ALGO_G8P && fast && !c8) {
    if (dtype == BF16) launch_8p<bf16>(a, stream);
    else if (dtype == F16) launch_8p<f16>(a, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if ((algo == IG_ALGO_GBIG256_32 || algo == IG_ALGO_GSHORT128_32 || algo == IG_ALGO_GSHORT64_32) &&
      fast) {
    if (algo == IG_ALGO_GBIG256_32) {
      if (dtype == BF16) launch_glds_big<bf16>(a, true, stream, true);
      else if (dtype == F16) launch_glds_big<f16>(a, true, stream, true);
      else return hipErrorInvalidValue;
    } else {
      const bool wide = algo == IG_ALGO_GSHORT128_32;
      if (dtype == BF16) launch_glds_short<bf16>(a, wide, false, stream, true);
      else if (dtype == F16) launch_glds_short<f16>(a, wide, false, stream, true);
      else return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (algo == IG_ALGO_DB && fast && !c8) {
    const int nwg = ((a.M + DB_BM - 1) / DB_BM) * ((a.Ncol + DB_BN - 1) / DB_BN);
    if (dtype == BF16) hipLaunchKernelGGL(igemm_db_k<bf16>, dim3(nwg), dim3(256), 0, stream, a);
    else if (dtype == F16) hipLaunchKernelGGL(igemm_db_k<f16>, dim3(nwg), dim3(256), 0, stream, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo == IG_ALGO_SK128 && fast && !c8) {
    // (no finalize tail in the stream-K kernel: a separate finalize launch)
    hipError_t e = hipErrorInvalidValue;
    if (dtype == BF16) e = launch_sk<bf16>(a, stream);
    if (dtype == F16) e = launch_sk<f16>(a, stream);
    if (e == hipSuccess && a.fin.counter)
      e = bn_finalize_stats_launch(stats, stats + (long)IG_SPREAD * Ncol, IG_SPREAD, Ncol,
                                   a.fin.rows, fin_gamma, fin_beta, fin_decay, fin_eps, fin_rm,
                                   fin_rv, fin_mean, fin_invstd, fin_scale, fin_shift,
                                   const_cast<float*>(kshift), stream);
    return e;
  }
  if ((algo == IG_ALGO_GMULTI64 || algo == IG_ALGO_GMULTI128) && fast && !c8) {
    const bool wide = algo == IG_ALGO_GMULTI128;
    if (dtype == BF16) launch_glds_mt<bf16>(a, wide, stream);
    else if (dtype == F16) launch_glds_mt<f16>(a, wide, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (algo == IG_ALGO_SMALL && fast) {
    if (dtype == BF16) launch_ig<bf16, 64, 64>(a, false, true, stream, true);
    else if (dtype == F16) launch_ig<f16, 64, 64>(a, false, true, stream, true);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if ((algo == IG_ALGO_MULTI2 || algo == IG_ALGO_MULTI4 || algo == IG_ALGO_SMALL_MULTI4) && fast &&
      !addend && !xbn && !mask && !c8) {
    const int tpw = algo == IG_ALGO_MULTI2 ? 2 : 4;
    const bool small = algo == IG_ALGO_SMALL_MULTI4;
    if (dtype == BF16) small ? launch_mt<bf16, 64>(a, tpw, stream) : launch_mt<bf16, 128>(a, tpw, stream);
    else if (dtype == F16) small ? launch_mt<f16, 64>(a, tpw, stream) : launch_mt<f16, 128>(a, tpw, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if ((algo == IG_ALGO_GLDS || algo == IG_ALGO_GLDS_N64) && fast) {
    if (dtype == BF16) launch_glds<bf16>(a, narrow, stream);
    else if (dtype == F16) launch_glds<f16>(a, narrow, stream);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (dtype == BF16) {
    if (Ncol <= 64 || narrow) launch_ig<bf16, 128, 64>(a, t, fast, stream, onebuf, early);
    else launch_ig<bf16, 128, 128>(a, t, fast, stream, onebuf, early);
  } else if (dtype == F16) {
    if (Ncol <= 64 || narrow) launch_ig<f16, 128, 64>(a, t, fast, stream, onebuf, early);
    else launch_ig<f16, 128, 128>(a, t, fast, stream, onebuf, early);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

KFB_API int kfb_conv_stats_spread() { return IG_SPREAD; }

KFB_API void kfb_set_deterministic(int on) { g_deterministic = on ? 1 : 0; }
KFB_API int kfb_get_deterministic() { return g_deterministic; }

// Number of reduction splits kfb_conv_wgrad uses for this geometry (the
// slab workspace needs splits * Ncol * KH*KW*C floats).
KFB_API int kfb_conv_wgrad_splits(int N, int OH, int OW, int KH, int KW, int C, int Ncol,
                                  int target_blocks) {
  if ((target_blocks >> 16) == 2) {  // streaming wgrad: stride 1, SAME (OH == H)
    const int sp = wgrad_s3_splits(N, OH, OW, C, OH, OW, KH, KW, 1, 1, 1, 1, Ncol);
    if (sp > 0) return sp;
  }
  return wgrad_split(N * OH * OW, KH * KW * C, Ncol, target_blocks & 0xFFFF, nullptr);
}

// Weight gradient: dw [Ncol][KH*KW*C] fp32 must be zeroed by the caller.
KFB_API hipError_t kfb_conv_wgrad(int dtype, const void* dy, const void* x, float* dw, int N,
                                  int H, int W, int C, int OH, int OW, int KH, int KW, int sh,
                                  int sw, int pt, int pl, int Ncol, int target_blocks,
                                  float* slab, long slab_elems, hipStream_t stream) {
  if (C % 8 || Ncol % 8) return hipErrorInvalidValue;
  // target_blocks bits 16+: kernel (0 = wgrad_k, 1 = wgrad_glds_k where it applies)
  const int algo = target_blocks >> 16;
  target_blocks &= 0xFFFF;
  // algo 2: the streaming 3x3 64-channel wgrad (conv_stream.hip)
  if (algo == 2 && wgrad_s3_splits(N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol) > 0)
    return launch_wgrad_s3(dtype, dy, x, dw, N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol,
                           slab, slab_elems, stream);
  const long dybytes = (long)N * OH * OW * Ncol * 2, xbytes = (long)N * H * W * C * 2;
  WgArgs a{dy, x, dw, N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Ncol, KH * KW * C,
           N * OH * OW, 0, (int)(dybytes < (1L << 31) ? dybytes : 0),
           (int)(xbytes < (1L << 31) ? xbytes : 0), nullptr, FastDiv(OH * OW), FastDiv(OW)};
  const int bmc = Ncol <= 64 ? 64 : 128;
  const int tiles = ((Ncol + bmc - 1) / bmc) * ((a.Ktot + 127) / 128);
  const int split = wgrad_split(a.M, a.Ktot, Ncol, target_blocks, &a.mper);
  const long per_split = (long)Ncol * a.Ktot;
  if (slab && split > 1 && (long)split * per_split <= slab_elems) a.slab = slab;
  int mode = WG_GENERIC;
  if (dybytes < (1L << 31) && xbytes < (1L << 31) && !igemm_fast_disabled())
    mode = (KH == 1 && KW == 1 && sh == 1 && sw == 1 && pt == 0 && pl == 0 && OH == H && OW == W)
               ? WG_PLAIN : WG_GATHER;
  const dim3 grid(tiles * split);
  if (algo == 1 && mode != WG_GENERIC && bmc == 128 && (dtype == BF16 || dtype == F16)) {
    if (dtype == BF16) {
      if (mode == WG_PLAIN) hipLaunchKernelGGL((wgrad_glds_k<bf16, WG_PLAIN>), grid, dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((wgrad_glds_k<bf16, WG_GATHER>), grid, dim3(256), 0, stream, a);
    } else {
      if (mode == WG_PLAIN) hipLaunchKernelGGL((wgrad_glds_k<f16, WG_PLAIN>), grid, dim3(256), 0, stream, a);
      else hipLaunchKernelGGL((wgrad_glds_k<f16, WG_GATHER>), grid, dim3(256), 0, stream, a);
    }
  } else if (dtype == BF16) {
    if (bmc == 64) launch_wg<bf16, 64>(a, mode, grid, stream);
    else launch_wg<bf16, 128>(a, mode, grid, stream);
  } else if (dtype == F16) {
    if (bmc == 64) launch_wg<f16, 64>(a, mode, grid, stream);
    else launch_wg<f16, 128>(a, mode, grid, stream);
  } else {
    return hipErrorInvalidValue;
  }
  if (a.slab) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const long n4 = per_split / 4;
    if (n4 >= 65536) {
      long blocks = (n4 + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(wgrad_reduce_k, dim3((unsigned)blocks), dim3(256), 0, stream,
                         (const float4*)slab, (float4*)dw, n4, split);
    } else {
      // >= ~1024 workgroups, <= 16 splits per thread
      const long blocks = (per_split + 255) / 256;
      long groups = (1024 + blocks - 1) / blocks;
      if (groups < (split + 15) / 16) groups = (split + 15) / 16;
      if (groups > split) groups = split;
      if (g_deterministic) groups = 1;  // one atomic add per element into zeroed / fixed dW
      hipLaunchKernelGGL(wgrad_reduce_grouped_k, dim3((unsigned)blocks, (unsigned)groups),
                         dim3(256), 0, stream, (const float*)slab, dw, per_split, split);
    }
  }
  return hipGetLastError();
}
