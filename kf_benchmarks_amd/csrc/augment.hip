// Training-image augmentation on the device: the colour distortions and the
// final normalisation of the reference's ImageNet train preprocessing
// (tcb/preprocessing.py:268-307 distort_color, :192-265 train_image), applied
// to the whole uint8 batch after its host-to-device copy.
//
// The host threads only decode, crop and resize (PIL, GIL released) and draw
// each image's random parameters in the reference's order; the per-pixel
// float work (brightness, RGB->HSV->RGB saturation/hue, per-image contrast
// around the channel means, clip, [-1, 1] scaling) and the horizontal flip
// run here, on 4x fewer transferred bytes than a float32 batch.
//
// params [N][8] f32: flip, brightness delta, saturation factor, hue delta,
// contrast factor, order (0: brightness, sat/hue, contrast; 1: brightness,
// contrast, sat/hue), distort (0: normalisation only), unused.
//
// Two passes: aug_sums_k folds each image's per-channel sums of the image the
// contrast step sees into AUG_BLOCKS partial slots per image (plain stores,
// no atomics: deterministic); aug_apply_k folds the slots of its image into
// the mean in its prologue and writes the output.
#include "common.h"

namespace kfb {

constexpr int AUG_BLOCKS = 32;  // partial-sum workgroups per image
constexpr int AUG_PARAMS = 8;

struct AugP {
  float flip, bright, sat, hue, contrast, order, distort;
};

__device__ __forceinline__ AugP aug_params(const float* __restrict__ p) {
  AugP a;
  a.flip = p[0];
  a.bright = p[1];
  a.sat = p[2];
  a.hue = p[3];
  a.contrast = p[4];
  a.order = p[5];
  a.distort = p[6];
  return a;
}

// saturation scale + hue shift of one pixel (same arithmetic as the host's
// kfbrt_adjust_sat_hue, csrc/runtime/kfb_runtime.cpp)
__device__ __forceinline__ void sat_hue(float& r, float& g, float& b, float sat, float hue) {
  const float mx = fmaxf(r, fmaxf(g, b));
  const float mn = fminf(r, fminf(g, b));
  const float d = mx - mn;
  const float v = mx;
  float s = mx > 0.f ? d / fmaxf(mx, 1e-12f) : 0.f;
  float h = 0.f;
  if (d > 0.f) {
    const float dd = fmaxf(d, 1e-12f);
    if (mx == r) h = (g - b) / dd;
    else if (mx == g) h = 2.f + (b - r) / dd;
    else h = 4.f + (r - g) / dd;
    h = h / 6.f;
    h -= floorf(h);
  }
  s = fminf(fmaxf(s * sat, 0.f), 1.f);
  h += hue;
  h -= floorf(h);
  const float h6 = h * 6.f;
  const float fl = floorf(h6);
  const int sector = (((int)fl) % 6 + 6) % 6;
  const float f = h6 - fl;
  const float p = v * (1.f - s), q = v * (1.f - s * f), t = v * (1.f - s * (1.f - f));
  switch (sector) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// Per-channel sums of the image the contrast step sees: brightness (+ sat/hue
// for order 0).  grid (AUG_BLOCKS, N), 256 threads.
__global__ void __launch_bounds__(256) aug_sums_k(const uint8_t* __restrict__ src,
                                                  const float* __restrict__ params, int npix,
                                                  float* __restrict__ part) {
  __shared__ float red[3][256];
  const int n = blockIdx.y;
  const AugP a = aug_params(params + (long)n * AUG_PARAMS);
  const uint8_t* img = src + (long)n * npix * 3;
  float sr = 0.f, sg = 0.f, sb = 0.f;
  if (a.distort != 0.f) {
    const bool sh = a.order == 0.f;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < npix; i += AUG_BLOCKS * 256) {
      float r = img[3 * i] * (1.f / 255.f) + a.bright;
      float g = img[3 * i + 1] * (1.f / 255.f) + a.bright;
      float b = img[3 * i + 2] * (1.f / 255.f) + a.bright;
      if (sh) sat_hue(r, g, b, a.sat, a.hue);
      sr += r;
      sg += g;
      sb += b;
    }
  }
  red[0][threadIdx.x] = sr;
  red[1][threadIdx.x] = sg;
  red[2][threadIdx.x] = sb;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h)
#pragma unroll
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[((long)n * AUG_BLOCKS + blockIdx.x) * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// dst[n][y][x][c] = augmented pixel scaled to [-1, 1]; grid (blocks, N),
// 256 threads, one pixel per thread per iteration.
template <typename T>
__global__ void __launch_bounds__(256) aug_apply_k(const uint8_t* __restrict__ src,
                                                   const float* __restrict__ params,
                                                   const float* __restrict__ part, int H, int W,
                                                   T* __restrict__ dst) {
  const int n = blockIdx.y;
  const int npix = H * W;
  const AugP a = aug_params(params + (long)n * AUG_PARAMS);
  float mean[3] = {0.f, 0.f, 0.f};
  if (a.distort != 0.f) {
    for (int k = 0; k < AUG_BLOCKS; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) mean[c] += part[((long)n * AUG_BLOCKS + k) * 3 + c];
#pragma unroll
    for (int c = 0; c < 3; ++c) mean[c] /= (float)npix;
  }
  const uint8_t* img = src + (long)n * npix * 3;
  T* out = dst + (long)n * npix * 3;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < npix; i += gridDim.x * 256) {
    const int y = i / W, x = i - y * W;
    const int si = a.flip != 0.f ? y * W + (W - 1 - x) : i;
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = img[3 * si + c] * (1.f / 255.f);
    if (a.distort != 0.f) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] += a.bright;
      if (a.order == 0.f) {
        sat_hue(v[0], v[1], v[2], a.sat, a.hue);
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (v[c] - mean[c]) * a.contrast + mean[c];
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (v[c] - mean[c]) * a.contrast + mean[c];
        sat_hue(v[0], v[1], v[2], a.sat, a.hue);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = fminf(fmaxf(v[c], 0.f), 1.f);
    }
    // x * 255 / 127.5 - 1 (the reference's normalized_image of [0, 255] pixels)
#pragma unroll
    for (int c = 0; c < 3; ++c) out[3 * i + c] = (T)(v[c] * 2.f - 1.f);
  }
}

}  // namespace kfb

using namespace kfb;

KFB_API int kfb_augment_blocks() { return AUG_BLOCKS; }

// src uint8 [N][H][W][3], params f32 [N][8], part f32 [N][AUG_BLOCKS][3]
// (scratch), dst [N][H][W][3] in dtype.
KFB_API hipError_t kfb_augment(int dtype, const uint8_t* src, const float* params, float* part,
                               int N, int H, int W, void* dst, hipStream_t stream) {
  if (N <= 0 || H <= 0 || W <= 0) return hipSuccess;
  const int npix = H * W;
  hipLaunchKernelGGL(aug_sums_k, dim3(AUG_BLOCKS, N), dim3(256), 0, stream, src, params, npix,
                     part);
  int blocks = (npix + 255) / 256;
  if (blocks > 64) blocks = 64;
  KFB_DISPATCH_DTYPE(dtype, T,
                     hipLaunchKernelGGL((aug_apply_k<T>), dim3(blocks, N), dim3(256), 0, stream,
                                        src, params, part, H, W, (T*)dst));
  return hipGetLastError();
}
