// GPU half of JPEG reconstruction for the train input pipeline: the host
// threads entropy-decode and ship the quantized 8x8 coefficient blocks of
// each training crop (csrc/runtime/kfb_images.cpp, kfbrt_imgpipe_run_coef);
// here one kernel dequantizes + inverse-DCTs every block into block-linear
// sample planes, and a second one builds each output pixel of the bilinear
// resize from them: four crop pixels, each with fancy-upsampled chroma and
// YCbCr -> RGB (csrc/jpeg_recon.h, bit-exact with libjpeg-turbo's decode).
// The uint8 result feeds csrc/augment.hip (flip, colour distortions, scaling).
//
// Reference: tf.image.decode_jpeg + crop + resize in the reference's input
// graph (tcb/preprocessing.py:192-265).
#include "common.h"

#define KFB_HD __host__ __device__
#include "jpeg_recon.h"

namespace kfb {
namespace jpeg {

constexpr int SPLIT = 8;  // workgroups per (image, component)

// grid (n * 3, SPLIT): one thread per 8x8 block of component blockIdx.x % 3
// of image blockIdx.x / 3.
__global__ void __launch_bounds__(256) idct_k(const int16_t* __restrict__ blocks,
                                              const jpg::Desc* __restrict__ descs,
                                              uint8_t* __restrict__ planes, long nblocks) {
  const int img = blockIdx.x / 3, k = blockIdx.x % 3;
  const jpg::Desc& d = descs[img];
  if (d.mode != jpg::MODE_COEF || k >= d.ncomp) return;
  const jpg::Comp& c = d.c[k];
  const long cnt = (long)c.bh * c.bw;
  if (c.blk < 0 || c.blk + cnt > nblocks) return;  // (host-built; never true)
  for (long i = blockIdx.y * 256L + threadIdx.x; i < cnt; i += SPLIT * 256L) {
    const long b = c.blk + i;
    int16_t coef[64];
    const int4* src = reinterpret_cast<const int4*>(blocks + 64 * b);
#pragma unroll
    for (int v = 0; v < 8; ++v) reinterpret_cast<int4*>(coef)[v] = src[v];
    uint8_t out[64];
    jpg::idct_islow<false>(coef, d.q[k], out);
    int4* dst = reinterpret_cast<int4*>(planes + 64 * b);
#pragma unroll
    for (int v = 0; v < 4; ++v) dst[v] = reinterpret_cast<const int4*>(out)[v];
  }
}

// grid (CROP_GRID, n): the crop of image blockIdx.y reconstructed once, one
// thread per crop pixel (fancy-upsampled chroma + YCbCr -> RGB), into the
// batch's crop-RGB buffer - the resize then reads each source pixel instead
// of rebuilding it for every output pixel that touches it.
constexpr int CROP_GRID = 64;

__global__ void __launch_bounds__(256) crop_rgb_k(const jpg::Desc* __restrict__ descs,
                                                  const uint8_t* __restrict__ planes,
                                                  uint8_t* __restrict__ rgb) {
  const jpg::Desc& d = descs[blockIdx.y];
  if (d.mode != jpg::MODE_COEF || d.rgb_off < 0) return;
  const long area = (long)d.ch * d.cw;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < area; p += CROP_GRID * 256L) {
    const int y = (int)(p / d.cw), x = (int)(p - (long)y * d.cw);
    int px[3];
    jpg::pixel_rgb(planes, d, d.cy + y, d.cx + x, px);
    uint8_t* o = rgb + 3L * (d.rgb_off + p);
    o[0] = (uint8_t)px[0];
    o[1] = (uint8_t)px[1];
    o[2] = (uint8_t)px[2];
  }
}

// grid (ceil(oh * ow / 256), n): one thread per output pixel.
__global__ void __launch_bounds__(256) rgb_k(const jpg::Desc* __restrict__ descs,
                                             const uint8_t* __restrict__ planes,
                                             const uint8_t* __restrict__ crop_rgb,
                                             const uint8_t* __restrict__ host_imgs,
                                             uint8_t* __restrict__ out, int oh, int ow) {
  const int img = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= oh * ow) return;
  const jpg::Desc& d = descs[img];
  uint8_t* o = out + ((long)img * oh * ow + p) * 3;
  if (d.mode != jpg::MODE_COEF) {
    const uint8_t* s = host_imgs ? host_imgs + ((long)d.host_slot * oh * ow + p) * 3 : nullptr;
    o[0] = s ? s[0] : 128;
    o[1] = s ? s[1] : 128;
    o[2] = s ? s[2] : 128;
    return;
  }
  uint8_t px[3];
  if (crop_rgb && d.rgb_off >= 0)
    jpg::resized_from_rgb(crop_rgb, d, oh, ow, p / ow, p % ow, px);
  else
    jpg::resized_pixel(planes, d, oh, ow, p / ow, p % ow, px);
  o[0] = px[0];
  o[1] = px[1];
  o[2] = px[2];
}

}  // namespace jpeg
}  // namespace kfb

using namespace kfb;

KFB_API int kfb_jpeg_desc_bytes() { return (int)sizeof(jpg::Desc); }

// descs [n] (device copy of the host descriptors), blocks [nblocks][64]
// int16, planes [nblocks][64] uint8 scratch, host_imgs [n][oh][ow][3] (the
// MODE_HOST images; nullable when there are none) -> out [n][oh][ow][3].
// crop_rgb (nullable): scratch of 3 x the crops' pixel count (the host's
// kfbrt_imgpipe_run_coef reports it); without it every output pixel
// rebuilds its four source pixels.
KFB_API hipError_t kfb_jpeg_decode(const void* descs, int n, const int16_t* blocks, long nblocks,
                                   uint8_t* planes, uint8_t* crop_rgb, const uint8_t* host_imgs,
                                   int oh, int ow, uint8_t* out, hipStream_t stream) {
  if (n <= 0 || oh <= 0 || ow <= 0 || (long)oh * ow >= (1L << 31) / 3) return hipErrorInvalidValue;
  const jpg::Desc* d = static_cast<const jpg::Desc*>(descs);
  if (nblocks > 0)
    hipLaunchKernelGGL(jpeg::idct_k, dim3((unsigned)n * 3, jpeg::SPLIT), dim3(256), 0, stream,
                       blocks, d, planes, nblocks);
  if (nblocks > 0 && crop_rgb)
    hipLaunchKernelGGL(jpeg::crop_rgb_k, dim3(jpeg::CROP_GRID, (unsigned)n), dim3(256), 0, stream,
                       d, planes, crop_rgb);
  hipLaunchKernelGGL(jpeg::rgb_k, dim3((unsigned)((oh * ow + 255) / 256), (unsigned)n), dim3(256),
                     0, stream, d, planes, (const uint8_t*)crop_rgb, host_imgs, out, oh, ow);
  return hipGetLastError();
}
