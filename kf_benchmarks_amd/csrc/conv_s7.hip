// Streaming stem convolution: the 7x7 / stride-2 RGB stem of the ImageNet
// models (tcb/models/resnet_model.py:372 conv(64, 7, 7, 2, 2), SAME), run as
// an 8x4-tap stride-(2,1) conv over the padded pixel-pair view of the image
// (csrc/stem.hip kfb_stem_pad: 8 channels = 2 pixels x 4 channels), with the
// consuming BN's statistics in the epilogue.
//
// The tiled implicit GEMM re-reads every input row for each of the 8 tap
// rows through L2 and runs ~100 short workgroups per CU (311 us at batch 256,
// 3.5x its memory bound).  Here one persistent 256-thread workgroup per
// CU owns a band of output rows of one image:
//
//  * the input pair-rows stream through an LDS ring (one output row needs
//    8 input rows, the next output row 2 more), LDS-DMA D output rows ahead;
//    each row's 16 trailing chunks beyond the image stay zero;
//  * each wave keeps the whole 64 x 256 weight matrix as MFMA A fragments in
//    VGPRs (128 registers) and computes 64 channels x 32 output pixels of the
//    row (the 112-pixel row padded to 4 x 32; the fourth wave's upper half is
//    masked), v_mfma_f32_32x32x16 with B fragments read straight from the
//    ring (a 16-byte tap chunk per lane, consecutive pixels = consecutive
//    chunks: conflict-free);
//  * the epilogue is conv_s1.hip's: v_permlane32_swap gives each lane 8
//    consecutive channels of one pixel for a 16-byte store, and the shifted
//    BN statistics accumulate per lane over the band.
#include "common.h"
#include "igemm_args.h"

#include <mutex>

namespace kfb {
namespace s7 {

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(16))) float v16f;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u_t;

constexpr int NC = 64;          // output channels
constexpr int KT = 32;          // taps (8 x 4), 8 channels each: K = 256
constexpr int KS = KT / 2;      // 32x32x16 k-steps (two taps each)
constexpr int OWP = 128;        // output row padded to 4 x 32 pixels
constexpr int ROWB = 2112;      // LDS bytes per input row: 128 chunks by DMA + 4 zero chunks
constexpr int D = 4;            // output rows prefetched ahead
constexpr int RING = 2 * D + 8; // input rows resident
constexpr int LDS_BYTES = RING * ROWB + NC * 4;  // + the statistics shift
constexpr int WAIT = 4 * D + (D - 1);  // counted wait: 4 stores + 1 DMA per wave per row

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, int off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
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

// grid: N images x nb row bands (blockIdx.x = img * nb + band)
template <typename T>
__global__ void __launch_bounds__(256, 1) conv_s7_k(IgArgs a, int nb) {
  __shared__ __attribute__((aligned(16))) char ring[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  const int img = blockIdx.x / nb, band = blockIdx.x - img * nb;
  const int oh0 = (int)((long)band * a.OH / nb), oh1 = (int)((long)(band + 1) * a.OH / nb);
  const int nrow = oh1 - oh0;

  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, a.ybytes, 0x00020000);

  // weights as A fragments: rows = output channel 32 i + l32, k = 16 ks + 8 hh
  v8s af[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const T* wr = (const T*)a.w + (long)(32 * i + l32) * (KT * 8) + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[i][ks] = *(const v8s*)(wr + 16 * ks);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(af[i][ks]));
  // the statistics shift lives in LDS (registers go to the weights)
  float* const kls = (float*)(ring + RING * ROWB);
  if (tid < NC) kls[tid] = a.kshift ? a.kshift[tid] : 0.f;

  // zero every ring row's 4 trailing chunks (never written by the DMAs)
  if (tid < RING * 4) *(v4u_t*)(ring + (tid >> 2) * ROWB + 2048 + (tid & 3) * 16) = v4u_t{0, 0, 0, 0};

  // input row r (of the padded pair image) -> ring slot r % RING; a row is
  // two 1 KB DMAs (128 chunks; chunks past the image width read as zero)
  const long img_off = (long)img * a.H * a.W * 8;  // elements
  // (a row past the band or the image loads zeros - into its own ring slot,
  // which by the ring's size holds no row still being read)
  auto load_row_half = [&](int r, int h, bool want) {
    const int chunk = 64 * h + lane;
    const bool ok = want && r < a.H && chunk < a.W;
    const int off = ok ? (int)((img_off + ((long)r * a.W + chunk) * 8) * sizeof(T)) : -1;
    dma16(xrs, ring + (r % RING) * ROWB + h * 1024, off);
  };
  // the 2 new input rows of output row t of the band: 4 DMAs, one per wave
  auto load_out_row = [&](int t) {
    load_row_half(2 * (oh0 + t) + 6 + (wid >> 1), wid & 1, t < nrow);
  };
  // prologue: input rows 2 oh0 .. 2 (oh0 + D - 1) + 7, i.e. 2D + 6 rows
  for (int q = wid; q < 2 * (2 * D + 6); q += 4) load_row_half(2 * oh0 + (q >> 1), q & 1, true);

  float s1[2][2][8], s2[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[i][p][k] = 0.f; s2[i][p][k] = 0.f; }
  auto keep_if = [](float x, unsigned m) { return u2f(f2u(x) & m); };
  const int ow = 32 * wid + l32;
  const bool pvalid = ow < a.OW;
  const unsigned vmask = pvalid ? ~0u : 0u;
  wait_vm<0>();
  __syncthreads();

  for (int t = 0; t < nrow; ++t) {
    load_out_row(t + D);
    const int oh = oh0 + t;
    v16f acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int tap = 2 * ks + hh, kh = tap >> 2, j = tap & 3;
      const v8s bf = *(const v8s*)(ring + ((2 * oh + kh) % RING) * ROWB + (ow + j) * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i] = mfma32<T>(af[i][ks], bf, acc[i]);
    }
    const long p = ((long)img * a.OH + oh) * a.OW + ow;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int cc = 4 * i + 2 * pp + hh;
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
        float pa[8];
        *(float4*)pa = *(const float4*)(kls + 8 * cc);
        *(float4*)(pa + 4) = *(const float4*)(kls + 8 * cc + 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ov.v[k] = (T)v[k];
          const float d = keep_if(v[k] - pa[k], vmask);
          s1[i][pp][k] += d;
          s2[i][pp][k] = fmaf(d, d, s2[i][pp][k]);
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_t, ov), yrs,
                                               pvalid ? (int)(p * (NC * 2)) + cc * 16 : -1, 0,
                                               0);
      }
    // output row t+1's input rows landed for every wave; row t's reads done
    wait_vm<WAIT>();
    __builtin_amdgcn_s_barrier();
  }

  wait_vm<0>();  // (the tail's zero-DMAs into the ring have landed)
  if (a.stats) {
    // reduce over the 32 lanes of one half, then over the 4 waves (they
    // hold the same channels) through LDS, one atomic pair per channel
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) {
            s1[i][pp][k] += __shfl_xor(s1[i][pp][k], o, 64);
            s2[i][pp][k] += __shfl_xor(s2[i][pp][k], o, 64);
          }
        }
    __syncthreads();
    float* red = (float*)ring;  // [wave][2][64]
    if (l32 == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int ch = 8 * (4 * i + 2 * pp + hh) + k;
            red[wid * 128 + ch] = s1[i][pp][k];
            red[wid * 128 + 64 + ch] = s2[i][pp][k];
          }
    }
    __syncthreads();
    if (tid < 128) {
      const float v = red[tid] + red[128 + tid] + red[256 + tid] + red[384 + tid];
      const int slot = blockIdx.x % IG_SPREAD;
      atomicAdd(a.stats + (long)((tid >> 6) * IG_SPREAD + slot) * NC + (tid & 63), v);
    }
  }
  bn_tail(a, (int*)ring + 1024);
}

}  // namespace s7

bool conv_s7_fits(const IgArgs& a) {
  return a.C == 8 && a.KH == 8 && a.KW == 4 && a.sh == 2 && a.sw == 1 && a.pt == 0 &&
         a.pl == 0 && a.Ncol == s7::NC && a.OW <= s7::OWP && a.W >= a.OW + 3 && a.W <= 128 &&
         a.H >= 2 * (a.OH - 1) + 8 && a.YH == a.OH && a.YW == a.OW && a.ys == 1 &&
         a.ldy == a.Ncol && !a.zfill && !a.bias && !a.relu && !a.mask && !a.xbn && !a.addend &&
         a.xbytes > 0 && a.ybytes > 0;
}

hipError_t launch_conv_s7(int dtype, const IgArgs& a, hipStream_t stream) {
  if (!conv_s7_fits(a)) return hipErrorInvalidValue;
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
  // row bands per image: enough workgroups for every CU, >= 8 rows each
  int nb = (cus + a.N - 1) / a.N;
  if (nb > a.OH / 8) nb = a.OH / 8;
  if (nb < 1) nb = 1;
  const dim3 grid(a.N * nb);
  if (dtype == BF16)
    hipLaunchKernelGGL((s7::conv_s7_k<bf16>), grid, dim3(256), 0, stream, a, nb);
  else if (dtype == F16)
    hipLaunchKernelGGL((s7::conv_s7_k<f16>), grid, dim3(256), 0, stream, a, nb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace kfb

KFB_API int kfb_conv_s7_applicable(int C, int Ncol, int KH, int KW, int sh, int sw, int pt, int pl,
                                   int H, int W, int OH, int OW) {
  return C == 8 && Ncol == kfb::s7::NC && KH == 8 && KW == 4 && sh == 2 && sw == 1 && pt == 0 &&
                 pl == 0 && OW <= kfb::s7::OWP && W >= OW + 3 && W <= 128 &&
                 H >= 2 * (OH - 1) + 8
             ? 1
             : 0;
}
