// Space-to-depth repack for stride-2 convolutions over few-channel inputs
// (the RGB stem: 7x7/2, 3 -> 64, tcb/models/resnet_model.py:311 with the
// SAME_RESNET padding of tcb/convnet_builder.py:159-183).
//
// A 3-channel NHWC image gives an implicit GEMM only 3 useful elements per
// tap, so the generic kernel pads C to 8 and walks 49 taps of 8 (K = 392 for
// 147 useful).  Instead, for each output row oh and each column pair j the
// repack writes one 64-element "pixel":
//
//   X2[n][oh][j][kh*8 + t*4 + c] = x[n][2*oh - pt + kh][2*j + t - pl][c]
//
// (zero outside the image, for c >= C and for kh >= KH).  The strided conv
// then becomes a stride-1, KW2 = ceil(KW/2)-tap, 64-channel conv over X2 with
// no padding: K = 4*64 = 256 for the 7x7 stem, and the FAST implicit-GEMM
// kernels (C % 64 == 0, wave-uniform tap stepping, LDS-DMA) apply unchanged.
// The weight is repacked to [Cout][1][KW2][64] the same way (host side,
// ops/conv_hip.py), and the weight gradient of the X2 conv maps back by the
// inverse permutation.
#include "common.h"

#include <cstdlib>

namespace kfb {

// One workgroup per output row (n, oh): its KH input rows are read with
// dword loads (all issued before any LDS write: 8 rows x 4 per thread in
// flight) into an LDS copy raw[kh][W*C] (zeros for rows outside the image or
// kh >= KH); every 16-byte output chunk (j, kh) is then gathered from LDS and
// written with one 16-byte store.
constexpr int S2D_ROW_DW = 1024;  // max dwords per input row (host-checked)

template <typename T>
__global__ void __launch_bounds__(256)
s2d_stem_k(const T* __restrict__ x, T* __restrict__ x2, int H, int W, int C, int OH, int OW2,
           int KH, int pt, int pl) {
  __shared__ uint32_t raw[8 * S2D_ROW_DW];
  const int row = blockIdx.x;  // n * OH + oh
  const int n = row / OH, oh = row - n * OH;
  const int rdw = W * C * (int)sizeof(T) / 4;
  const int tid = threadIdx.x;
  uint32_t v[8][4];
#pragma unroll
  for (int kh = 0; kh < 8; ++kh) {
    const int h = 2 * oh - pt + kh;
    const bool ok = kh < KH && (unsigned)h < (unsigned)H;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(x + ((long)n * H + (ok ? h : 0)) * W * C);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int d = tid + it * 256;
      v[kh][it] = (ok && d < rdw) ? src[d] : 0u;
    }
  }
#pragma unroll
  for (int kh = 0; kh < 8; ++kh)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int d = tid + it * 256;
      if (d < rdw) raw[kh * rdw + d] = v[kh][it];
    }
  __syncthreads();
  const T* rt = reinterpret_cast<const T*>(raw);
  const int rel = rdw * 4 / (int)sizeof(T);  // elements per LDS row (= W*C)
  T* dst = x2 + (long)row * OW2 * 64;
  for (int q = tid; q < OW2 * 8; q += 256) {
    const int j = q >> 3, kh = q & 7;
    Vec<T, 8> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int t = e >> 2, c = e & 3;
      const int w = 2 * j + t - pl;
      o.v[e] = (c < C && (unsigned)w < (unsigned)W) ? rt[kh * rel + w * C + c] : (T)0.f;
    }
    *reinterpret_cast<Vec<T, 8>*>(dst + (long)j * 64 + kh * 8) = o;
  }
}

// 16-bit, C == 3 (the RGB stem): LDS row kh holds input pixel w at slot
// w + pl (3 elements per slot, zeros around the image), 2*OW2 slots, so the
// two pixels (2j - pl, 2j + 1 - pl) of output chunk (j, kh) are the 6
// elements at 6j: three aligned dword reads per 16-byte chunk instead of
// eight 2-byte gathers with bounds checks.  Each LDS dword is assembled in
// registers from the (at most two) input dwords holding its two elements, so
// the rows go to LDS in one pass of dword stores (no zero fill, no 2-byte
// stores).  Rows of up to S2D3_Q dwords (host-checked).
constexpr int S2D3_Q = 512;

template <typename T>
__global__ void __launch_bounds__(256)
s2d_stem3_k(const T* __restrict__ x, T* __restrict__ x2, int H, int W, int OH, int OW2, int KH,
            int pt, int pl) {
  static_assert(sizeof(T) == 2, "16-bit elements");
  __shared__ uint32_t raw[8 * S2D3_Q];
  const int row = blockIdx.x;  // n * OH + oh
  const int n = row / OH, oh = row - n * OH;
  const int rp = 3 * OW2;      // LDS dwords per row (2 * OW2 slots of 3 elements)
  const int n3 = 3 * W;        // input elements per row
  const int e0 = 3 * pl;       // element shift of the padded row
  const int tid = threadIdx.x;
  uint32_t w0[8][2], w1[8][2];
#pragma unroll
  for (int kh = 0; kh < 8; ++kh) {
    const int h = 2 * oh - pt + kh;
    const bool okr = kh < KH && (unsigned)h < (unsigned)H;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(x + ((long)n * H + (okr ? h : 0)) * n3);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + it * 256;
      const int i0 = 2 * q - e0, i1 = i0 + 1;
      const bool ok = okr && q < rp;
      w0[kh][it] = (ok && i0 >= 0 && i0 < n3) ? src[i0 >> 1] : 0u;
      w1[kh][it] = (ok && i1 >= 0 && i1 < n3) ? src[i1 >> 1] : 0u;
    }
  }
#pragma unroll
  for (int kh = 0; kh < 8; ++kh)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + it * 256;
      const int i0 = 2 * q - e0;
      const uint32_t lo = (w0[kh][it] >> (16 * (i0 & 1))) & 0xffffu;
      const uint32_t hi = (w1[kh][it] >> (16 * ((i0 + 1) & 1))) & 0xffffu;
      if (q < rp) raw[kh * rp + q] = lo | (hi << 16);
    }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(x2 + (long)row * OW2 * 64);
  for (int q = tid; q < OW2 * 8; q += 256) {
    const int j = q >> 3, kh = q & 7;
    const uint32_t* r = raw + kh * rp + 3 * j;
    const uint32_t d0 = r[0], d1 = r[1], d2 = r[2];
    // [a0 a1 | a2 0 | b0 b1 | b2 0]
    dst[q] = make_uint4(d0, d1 & 0xffffu, (d1 >> 16) | (d2 << 16), d2 >> 16);
  }
}

// ---------------------------------------------------------------- "pairs"
// The stride-2 stem as a plain strided conv over PIXEL PAIRS, with no
// repacked copy of the input: pad the image to 4 channels and by
// (pt, pl) zeros, then view it as [N, Hp, Wp/2, 8] (two adjacent 4-channel
// pixels per 8-channel "pixel").  Output (oh, ow) of the 7x7/2 conv reads
// padded rows 2*oh + kh (kh < 8) and pair columns ow + j (j < 4), i.e. it is
// an 8x4-tap conv with stride (2, 1) and C = 8 over the pair view:
//   y[oh][ow][n] = sum_{kh<8, j<4, t<2, c<4} xp[2oh+kh][2(ow+j)+t][c] *
//                  w2[n][kh][j][t*4+c],   w2[n][kh][j][t*4+c] = w[n][kh][2j+t][c]
// (zero where kh >= KH, 2j+t >= KW or c >= C).  K = 256 as in the s2d repack,
// but the kernels read the 1.4x padded image (108 MB at ResNet-50 bs256)
// instead of writing and re-reading a 4.2x repack (422 MB).
template <typename T>
__global__ void __launch_bounds__(256)
stem_pad_k(const T* __restrict__ x, T* __restrict__ xp, long npix, int H, int W, int C, int Hp,
           int Wp, int pt, int pl) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < npix; i += (long)gridDim.x * 256) {
    const long n = i / ((long)Hp * Wp);
    const int r = (int)(i - n * Hp * Wp);
    const int hp = r / Wp, wp = r - hp * Wp;
    const int h = hp - pt, w = wp - pl;
    Vec<T, 4> o;
    const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    const T* src = x + ((n * H + (in ? h : 0)) * W + (in ? w : 0)) * C;
#pragma unroll
    for (int c = 0; c < 4; ++c) o.v[c] = (in && c < C) ? src[c] : (T)0.f;
    reinterpret_cast<Vec<T, 4>*>(xp)[i] = o;
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
stem_weight_k(const T* __restrict__ w, T* __restrict__ w2, int cout, int KH, int KW, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // [cout][8][4][8]
  if (i >= cout * 256) return;
  const int n = i >> 8, kh = (i >> 5) & 7, j = (i >> 3) & 3, e = i & 7;
  const int kw = 2 * j + (e >> 2), c = e & 3;
  w2[i] = (kh < KH && kw < KW && c < C) ? w[((n * KH + kh) * KW + kw) * C + c] : (T)0.f;
}

// dw [cout][KH][KW][C] (fp32) += the pair-view weight gradient dw2
__global__ void __launch_bounds__(256)
stem_weight_grad_k(const float* __restrict__ dw2, float* __restrict__ dw, int cout, int KH,
                   int KW, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cout * KH * KW * C) return;
  const int c = i % C, kw = (i / C) % KW, kh = (i / (C * KW)) % KH, n = i / (C * KW * KH);
  dw[i] += dw2[(((n * 8 + kh) * 4 + (kw >> 1)) * 8) + (kw & 1) * 4 + c];
}

}  // namespace kfb

using namespace kfb;

// x [N,H,W,C<=4] -> xp [N,Hp,Wp,4] (zero border: rows [pt, pt+H), cols [pl, pl+W))
KFB_API hipError_t kfb_stem_pad(int dtype, const void* x, void* xp, int N, int H, int W, int C,
                                int Hp, int Wp, int pt, int pl, hipStream_t stream) {
  if (C > 4 || dtype == F32) return hipErrorInvalidValue;
  const long npix = (long)N * Hp * Wp;
  long blocks = (npix + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (dtype == BF16)
    hipLaunchKernelGGL((stem_pad_k<bf16>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const bf16*)x, (bf16*)xp, npix, H, W, C, Hp, Wp, pt, pl);
  else
    hipLaunchKernelGGL((stem_pad_k<f16>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       (const f16*)x, (f16*)xp, npix, H, W, C, Hp, Wp, pt, pl);
  return hipGetLastError();
}

// w [cout][KH][KW][C] -> w2 [cout][8][4][8] (KH <= 8, KW <= 8, C <= 4)
KFB_API hipError_t kfb_stem_weight(int dtype, const void* w, void* w2, int cout, int KH, int KW,
                                   int C, hipStream_t stream) {
  if (KH > 8 || KW > 8 || C > 4 || dtype == F32) return hipErrorInvalidValue;
  const int blocks = (cout * 256 + 255) / 256;
  if (dtype == BF16)
    hipLaunchKernelGGL((stem_weight_k<bf16>), dim3(blocks), dim3(256), 0, stream, (const bf16*)w,
                       (bf16*)w2, cout, KH, KW, C);
  else
    hipLaunchKernelGGL((stem_weight_k<f16>), dim3(blocks), dim3(256), 0, stream, (const f16*)w,
                       (f16*)w2, cout, KH, KW, C);
  return hipGetLastError();
}

KFB_API hipError_t kfb_stem_weight_grad(const float* dw2, float* dw, int cout, int KH, int KW,
                                        int C, hipStream_t stream) {
  const int n = cout * KH * KW * C;
  hipLaunchKernelGGL(stem_weight_grad_k, dim3((n + 255) / 256), dim3(256), 0, stream, dw2, dw,
                     cout, KH, KW, C);
  return hipGetLastError();
}

// x [N,H,W,C] (C <= 4) -> x2 [N,OH,OW2,64]; requires KH <= 8.
KFB_API hipError_t kfb_s2d_stem(int dtype, const void* x, void* x2, int N, int H, int W, int C,
                                int OH, int OW2, int KH, int pt, int pl, hipStream_t stream) {
  const int esz = dtype == F32 ? 4 : 2;
  if (C > 4 || KH > 8 || (W * C * esz) % 4 || W * C * esz > 4 * S2D_ROW_DW ||
      ((uintptr_t)x & 3))
    return hipErrorInvalidValue;
  if (C == 3 && esz == 2 && 3 * OW2 <= S2D3_Q) {
    if (dtype == BF16)
      hipLaunchKernelGGL((s2d_stem3_k<bf16>), dim3(N * OH), dim3(256), 0, stream, (const bf16*)x,
                         (bf16*)x2, H, W, OH, OW2, KH, pt, pl);
    else
      hipLaunchKernelGGL((s2d_stem3_k<f16>), dim3(N * OH), dim3(256), 0, stream, (const f16*)x,
                         (f16*)x2, H, W, OH, OW2, KH, pt, pl);
    return hipGetLastError();
  }
  KFB_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((s2d_stem_k<T>), dim3(N * OH), dim3(256), 0, stream, (const T*)x, (T*)x2,
                       H, W, C, OH, OW2, KH, pt, pl);
  });
  return hipGetLastError();
}
