// fp32 implicit-GEMM convolution (forward / dgrad / wgrad) on gfx950
// v_mfma_f32_16x16x4_f32: exact fp32 products with fp32 accumulation, the
// precision of the reference's only published numbers (fp32 cuDNN convs of
// tcb/convnet_builder.py:107-124; default use_fp16=False).
//
// The tiles, LDS images and main loop are the MFMA GEMM core of gemm_core.h
// (128 x 128 tile, 4 waves, 32-deep K steps through double-buffered LDS).
// What is convolution-specific is the operand *gather*: each loader maps a
// (GEMM row, k) pair to an element of the NHWC activation / [Cout][KH][KW]
// [Cin] weight, with zero padding as out-of-range:
//
//   fwd   y [m=(n,oh,ow)][co]       = sum_{k=(kh,kw,ci)} X(m,k)   W[co][k]
//   dgrad dx[m=(n,h,w)][ci]         = sum_{k=(kh,kw,co)} dY'(m,k) W[co][kh][kw][ci]
//         (dY' gathers dy[(h+pt-kh)/s][(w+pl-kw)/s] where divisible)
//   wgrad dW[co][k=(kh,kw,ci)]      = sum_{m=(n,oh,ow)}  dy[m][co] X(m,k)
//         (reduction over all output pixels, split over workgroups,
//          fp32 atomics into the zeroed / accumulating gradient)
//
// With Cin and Cout multiples of 4 every 16-byte chunk a loader moves is
// 4 consecutive channels of one tap (one aligned vector load); otherwise
// (the 3-channel RGB stem) the loaders fetch element by element.
#include "gemm_core.h"

namespace kfb {
namespace cf {

using gm::TILE;
using gm::Tr;
using gm::v4f;

struct Geo {
  int N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Cout;
  FastDiv ohw, ow, hw, w, c, kw, cout, s_h, s_w;
};

// Element offset of operand (row, k), or -1 if it is a zero (padding or
// out of range).  `rows` / `kend` bound the GEMM row and reduction index.
struct FwdX {  // row m = (n, oh, ow), k = (kh, kw, ci) -> x[n][h][w][ci]
  Geo g;
  int rows;
  __device__ __forceinline__ long operator()(int m, int k, int kend) const {
    if (m >= rows || k >= kend) return -1;
    const int ohw = g.OH * g.OW, img = g.ohw.div(m), rem = m - img * ohw;
    const int oh = g.ow.div(rem), ow = rem - oh * g.OW;
    const int tap = g.c.div(k), ci = k - tap * g.C;
    const int kh = g.kw.div(tap), kw = tap - kh * g.KW;
    const int h = oh * g.sh - g.pt + kh, w = ow * g.sw - g.pl + kw;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return -1;
    return ((long)(img * g.H + h) * g.W + w) * g.C + ci;
  }
};

struct FwdW {  // row co, k -> w[co][k]
  int rows, K;
  __device__ __forceinline__ long operator()(int co, int k, int kend) const {
    return (co < rows && k < kend) ? (long)co * K + k : -1;
  }
};

struct DgradDy {  // row m = (n, h, w), k = (kh, kw, co) -> dy[n][oh][ow][co]
  Geo g;
  int rows;
  __device__ __forceinline__ long operator()(int m, int k, int kend) const {
    if (m >= rows || k >= kend) return -1;
    const int hw = g.H * g.W, img = g.hw.div(m), rem = m - img * hw;
    const int h = g.w.div(rem), w = rem - h * g.W;
    const int tap = g.cout.div(k), co = k - tap * g.Cout;
    const int kh = g.kw.div(tap), kw = tap - kh * g.KW;
    const int hn = h + g.pt - kh, wn = w + g.pl - kw;
    if (hn < 0 || wn < 0) return -1;
    const int oh = g.s_h.div(hn), ow = g.s_w.div(wn);
    if (oh * g.sh != hn || ow * g.sw != wn || oh >= g.OH || ow >= g.OW) return -1;
    return ((long)(img * g.OH + oh) * g.OW + ow) * g.Cout + co;
  }
};

struct DgradW {  // row ci, k = (kh, kw, co) -> w[co][kh][kw][ci]
  Geo g;
  __device__ __forceinline__ long operator()(int ci, int k, int kend) const {
    if (ci >= g.C || k >= kend) return -1;
    const int tap = g.cout.div(k), co = k - tap * g.Cout;
    return ((long)co * g.KH * g.KW + tap) * g.C + ci;
  }
};

struct WgradDy {  // row co, k = m -> dy[m][co]
  int Cout;
  __device__ __forceinline__ long operator()(int co, int m, int kend) const {
    return (co < Cout && m < kend) ? (long)m * Cout + co : -1;
  }
};

struct WgradX {  // row n = (kh, kw, ci), k = m = (img, oh, ow) -> x[img][h][w][ci]
  Geo g;
  int K;
  __device__ __forceinline__ long operator()(int n, int m, int kend) const {
    if (n >= K || m >= kend) return -1;
    const int ohw = g.OH * g.OW, img = g.ohw.div(m), rem = m - img * ohw;
    const int oh = g.ow.div(rem), ow = rem - oh * g.OW;
    const int tap = g.c.div(n), ci = n - tap * g.C;
    const int kh = g.kw.div(tap), kw = tap - kh * g.KW;
    const int h = oh * g.sh - g.pt + kh, w = ow * g.sw - g.pl + kw;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return -1;
    return ((long)(img * g.H + h) * g.W + w) * g.C + ci;
  }
};

// A loader over a Map: the chunk assignment and LDS image of gm::Loader, the
// addresses from the map (64-bit, so no operand-size limit).
template <bool KS_, bool VEC, class Map>
struct Gather {
  static constexpr bool KS = KS_;
  static constexpr int EPC = Tr<float>::EPC, CPR = TILE / EPC;
  const float* base;
  Map map;
  int r0, kend;
  int cr[4], ck[4];

  __device__ __forceinline__ void init(const float* p, const Map& m, int r0_, int kend_, int tid) {
    base = p;
    map = m;
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
        const long off = map(row, k, kend);
        r[i] = off >= 0 ? *(const uint4*)(base + off) : make_uint4(0, 0, 0, 0);
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long off = KS ? map(row + j, k, kend) : map(row, k + j, kend);
          e[j] = off >= 0 ? base[off] : 0.f;
        }
        r[i] = __builtin_bit_cast(uint4, e);
      }
    }
  }

  __device__ __forceinline__ void store(const uint4 (&r)[4], float* img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = KS ? gm::ks_off<float>(ck[i], cr[i]) : gm::kc_off<float>(cr[i], ck[i] / EPC);
      *(uint4*)(img + off) = r[i];
    }
  }
};

// C[m][n] tile store (plain or atomic fp32).
__device__ __forceinline__ void store_tile(v4f (&acc)[TILE / 32][TILE / 32], float* out, int ldc,
                                           int M, int Ncol, int m0, int n0, bool atomic) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wn = wid >> 1, wm = wid & 1;
#pragma unroll
  for (int j = 0; j < TILE / 32; ++j) {
    const int m = m0 + wm * (TILE / 2) + j * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < TILE / 32; ++i) {
      const int n = n0 + wn * (TILE / 2) + i * 16 + (lane >> 4) * 4;
      if (n >= Ncol) continue;
      float* c = out + (long)m * ldc + n;
      const v4f v = acc[i][j];
      if (atomic) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < Ncol) atomicAdd(c + r, v[r]);
      } else if (n + 3 < Ncol && (ldc & 3) == 0) {
        *(v4f*)c = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < Ncol) c[r] = v[r];
      }
    }
  }
}

struct Args {
  const float* a;  // fwd: x    dgrad: dy   wgrad: dy
  const float* b;  // fwd: w    dgrad: w    wgrad: x
  float* out;      // fwd: y    dgrad: dx   wgrad: dw (accumulated)
  Geo g;
  int kper;        // wgrad: reduction rows per split
};

__device__ __forceinline__ void tile_of(int M, int Ncol, int& m0, int& n0, int& split) {
  const int mt = (M + TILE - 1) / TILE, nt = (Ncol + TILE - 1) / TILE;
  const int tiles = mt * nt;
  const int bid = gm::xcd_remap(blockIdx.x, gridDim.x);
  split = bid / tiles;
  const int t = bid - split * tiles;
  m0 = (t % mt) * TILE;
  n0 = (t / mt) * TILE;
}

template <bool VEC, bool X3>
__global__ void __launch_bounds__(256, 2) fwd_k(Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * gm::img_elems<float>()];
  const Geo& g = a.g;
  const int M = g.N * g.OH * g.OW, K = g.KH * g.KW * g.C;
  int m0, n0, split;
  tile_of(M, g.Cout, m0, n0, split);
  Gather<false, VEC, FwdX> lp;
  Gather<false, VEC, FwdW> lq;
  lp.init(a.a, FwdX{g, M}, m0, K, threadIdx.x);
  lq.init(a.b, FwdW{g.Cout, K}, n0, K, threadIdx.x);
  v4f acc[TILE / 32][TILE / 32];
  gm::mainloop<float, decltype(lp), decltype(lq), X3>(lp, lq, 0, (K + Tr<float>::BK - 1) / Tr<float>::BK,
                                                       smem, acc);
  store_tile(acc, a.out, g.Cout, M, g.Cout, m0, n0, false);
}

template <bool VEC, bool X3>
__global__ void __launch_bounds__(256, 2) dgrad_k(Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * gm::img_elems<float>()];
  const Geo& g = a.g;
  const int M = g.N * g.H * g.W, K = g.KH * g.KW * g.Cout;
  int m0, n0, split;
  tile_of(M, g.C, m0, n0, split);
  Gather<false, VEC, DgradDy> lp;
  Gather<true, VEC, DgradW> lq;
  lp.init(a.a, DgradDy{g, M}, m0, K, threadIdx.x);
  lq.init(a.b, DgradW{g}, n0, K, threadIdx.x);
  v4f acc[TILE / 32][TILE / 32];
  gm::mainloop<float, decltype(lp), decltype(lq), X3>(lp, lq, 0, (K + Tr<float>::BK - 1) / Tr<float>::BK,
                                                       smem, acc);
  store_tile(acc, a.out, g.C, M, g.C, m0, n0, false);
}

template <bool VEC, bool X3>
__global__ void __launch_bounds__(256, 2) wgrad_k(Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * gm::img_elems<float>()];
  const Geo& g = a.g;
  const int R = g.N * g.OH * g.OW, K = g.KH * g.KW * g.C;
  int m0, n0, split;
  tile_of(g.Cout, K, m0, n0, split);
  const int kbeg = split * a.kper, kend = min(R, kbeg + a.kper);
  Gather<true, VEC, WgradDy> lp;
  Gather<true, VEC, WgradX> lq;
  lp.init(a.a, WgradDy{g.Cout}, m0, kend, threadIdx.x);
  lq.init(a.b, WgradX{g, K}, n0, kend, threadIdx.x);
  v4f acc[TILE / 32][TILE / 32];
  const int nk = kend > kbeg ? (kend - kbeg + Tr<float>::BK - 1) / Tr<float>::BK : 0;
  gm::mainloop<float, decltype(lp), decltype(lq), X3>(lp, lq, kbeg, nk, smem, acc);
  store_tile(acc, a.out, K, g.Cout, K, m0, n0, true);
}

template <bool X3>
static void launch(int mode, bool vec, dim3 grid, const Args& a, hipStream_t s) {
  if (mode == 0) {
    if (vec) hipLaunchKernelGGL((fwd_k<true, X3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fwd_k<false, X3>), grid, dim3(256), 0, s, a);
  } else if (mode == 1) {
    if (vec) hipLaunchKernelGGL((dgrad_k<true, X3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dgrad_k<false, X3>), grid, dim3(256), 0, s, a);
  } else {
    if (vec) hipLaunchKernelGGL((wgrad_k<true, X3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_k<false, X3>), grid, dim3(256), 0, s, a);
  }
}

}  // namespace cf
}  // namespace kfb

using namespace kfb;

// mode 0: y = conv(x, w)            a = x  [N,H,W,C],    b = w [Cout,KH,KW,C], out = y  [N,OH,OW,Cout]
// mode 1: dx = conv^T(dy, w)        a = dy [N,OH,OW,Cout], b = w,              out = dx [N,H,W,C]
// mode 2: dw += wgrad(dy, x)        a = dy,               b = x,              out = dw [Cout,KH,KW,C]
// mode | 8: products as three bf16 MFMAs of the operands' bf16 splits (gm::mainloop X3)
KFB_API hipError_t kfb_conv_f32(int mode, const float* a, const float* b, float* out, int N, int H,
                                int W, int C, int OH, int OW, int KH, int KW, int sh, int sw,
                                int pt, int pl, int Cout, hipStream_t stream) {
  const bool x3 = (mode & 8) != 0;
  mode &= 7;
  cf::Geo g{N, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, Cout,
            FastDiv(OH * OW), FastDiv(OW), FastDiv(H * W), FastDiv(W),
            FastDiv(C), FastDiv(KW), FastDiv(Cout), FastDiv(sh), FastDiv(sw)};
  if ((long)N * H * W >= (1L << 31) || (long)N * OH * OW >= (1L << 31) ||
      (long)KH * KW * (C > Cout ? C : Cout) >= (1L << 31))
    return hipErrorInvalidValue;  // FastDiv range
  cf::Args args{a, b, out, g, 0};
  const bool vec = C % 4 == 0 && Cout % 4 == 0;
  auto tiles = [](long M, long Ncol) {
    return ((M + cf::TILE - 1) / cf::TILE) * ((Ncol + cf::TILE - 1) / cf::TILE);
  };
  dim3 grid;
  if (mode == 0) {
    const long nwg = tiles((long)N * OH * OW, Cout);
    grid = dim3(nwg);
  } else if (mode == 1) {
    const long nwg = tiles((long)N * H * W, C);
    grid = dim3(nwg);
  } else if (mode == 2) {
    const long R = (long)N * OH * OW, K = (long)KH * KW * C;
    const long t = tiles(Cout, K);
    const int bk = cf::Tr<float>::BK;
    const long nk = (R + bk - 1) / bk;
    long split = (1024 + t - 1) / t;  // ~4 workgroups per CU
    if (split > nk / 8) split = nk / 8;  // >= 8 K steps each
    if (split < 1) split = 1;
    args.kper = (int)(((nk + split - 1) / split) * bk);
    split = (R + args.kper - 1) / args.kper;
    grid = dim3(t * split);
  } else {
    return hipErrorInvalidValue;
  }
  if (x3) cf::launch<true>(mode, vec, grid, args, stream);
  else cf::launch<false>(mode, vec, grid, args, stream);
  return hipGetLastError();
}
