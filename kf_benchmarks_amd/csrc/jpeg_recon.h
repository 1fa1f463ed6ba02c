// JPEG pixel reconstruction from quantized DCT coefficients, shared by the
// device kernels (csrc/jpeg.hip) and the host reference / fallback
// (csrc/runtime/kfb_images.cpp, built with g++: KFB_HD is empty there).
//
// The host threads of the image pipeline only entropy-decode
// (jpeg_read_coefficients) and copy the 8x8 coefficient blocks covering the
// training crop; everything after that - dequantization, the 8x8 inverse
// DCT, chroma upsampling, YCbCr -> RGB and the bilinear resize of the crop -
// runs here, per output pixel, on the GPU.  The integer arithmetic is the
// one libjpeg-turbo uses with its defaults (what TF's decode_jpeg and PIL
// run): the "islow" IDCT (Loeffler-Ligtenberg-Moschytz, 13 fractional bits,
// 2 extra bits between the passes), "fancy" triangle-filter upsampling of
// h2v1 / h2v2 chroma, and the 16-bit fixed-point YCbCr tables, so the
// reconstructed pixels match a full libjpeg-turbo decode bit for bit.
//
// Reference: the reference decodes with tf.image.decode_jpeg and crops /
// resizes in TF ops (tcb/preprocessing.py:192-265).
#pragma once

#include <stdint.h>

#ifndef KFB_HD
#define KFB_HD
#endif

namespace kfb {
namespace jpg {

// Per-component block window of one image: blocks [by0, by0+bh) x
// [bx0, bx0+bw) of the component's coefficient array, stored row-major as
// int16[64] blocks starting at block index `blk` of the batch arena; the
// IDCT writes each block's 8x8 samples to byte 64 * (blk + i) of the plane
// buffer (block-linear layout).
struct Comp {
  int h, v;      // sampling factors
  int by0, bx0;  // window origin (blocks)
  int bh, bw;    // window size (blocks)
  int dw, dh;    // downsampled width / height of the component (samples)
  int blk;       // first block of the window in the batch arena
  int pad;
};

enum { MODE_COEF = 0, MODE_HOST = 1 };

// One image of a batch (host-filled, read by both kernels).
struct Desc {
  int mode;     // MODE_COEF: reconstruct here; MODE_HOST: pixels decoded on the host
  int ncomp;    // 1 (grayscale) or 3 (YCbCr)
  int cy, cx, ch, cw;  // training crop in full-resolution pixels
  int host_slot;       // MODE_HOST: index into the host-decoded image buffer
  int rgb_off;         // MODE_COEF: first pixel of this crop in the batch's crop-RGB buffer
  Comp c[3];
  uint16_t q[3][64];   // dequantization tables, natural order
};

// ------------------------------------------------------------ islow IDCT
constexpr int CONST_BITS = 13, PASS1_BITS = 2;

KFB_HD inline int descale(int64_t x, int n) { return (int)((x + ((int64_t)1 << (n - 1))) >> n); }

KFB_HD inline uint8_t idct_range(int v) {
  // libjpeg's post-IDCT range-limit table (index v & 1023 around centre 128)
  const int k = v & 1023;
  return (uint8_t)(k < 128 ? k + 128 : k < 512 ? 255 : k < 896 ? 0 : k - 896);
}

// One 8x8 block: coef (natural order) x q -> 64 samples (row-major).
// ZERO_TESTS: libjpeg's all-AC-zero column / row shortcuts (exact: they give
// the full computation's values); the device form leaves them out so both
// passes unroll with the workspace in registers.
template <bool ZERO_TESTS = true>
KFB_HD inline void idct_islow(const int16_t* coef, const uint16_t* q, uint8_t* out) {
  int ws[64];
#pragma unroll
  for (int c = 0; c < 8; ++c) {  // pass 1: columns
    const int d0 = coef[c] * (int)q[c], d1 = coef[8 + c] * (int)q[8 + c];
    const int d2 = coef[16 + c] * (int)q[16 + c], d3 = coef[24 + c] * (int)q[24 + c];
    const int d4 = coef[32 + c] * (int)q[32 + c], d5 = coef[40 + c] * (int)q[40 + c];
    const int d6 = coef[48 + c] * (int)q[48 + c], d7 = coef[56 + c] * (int)q[56 + c];
    if (ZERO_TESTS && (d1 | d2 | d3 | d4 | d5 | d6 | d7) == 0) {
      const int dc = d0 * (1 << PASS1_BITS);
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
      continue;
    }
    int64_t z1 = (int64_t)(d2 + d6) * 4433;
    const int64_t tmp2 = z1 + (int64_t)d6 * -15137, tmp3 = z1 + (int64_t)d2 * 6270;
    const int64_t tmp0 = (int64_t)(d0 + d4) << CONST_BITS, tmp1 = (int64_t)(d0 - d4) << CONST_BITS;
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    int64_t o0 = d7, o1 = d5, o2 = d3, o3 = d1;
    z1 = o0 + o3;
    int64_t z2 = o1 + o2, z3 = o0 + o2, z4 = o1 + o3;
    const int64_t z5 = (z3 + z4) * 9633;
    o0 *= 2446; o1 *= 16819; o2 *= 25172; o3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    o0 += z1 + z3; o1 += z2 + z4; o2 += z2 + z3; o3 += z1 + z4;
    constexpr int S = CONST_BITS - PASS1_BITS;
    ws[0 * 8 + c] = descale(t10 + o3, S); ws[7 * 8 + c] = descale(t10 - o3, S);
    ws[1 * 8 + c] = descale(t11 + o2, S); ws[6 * 8 + c] = descale(t11 - o2, S);
    ws[2 * 8 + c] = descale(t12 + o1, S); ws[5 * 8 + c] = descale(t12 - o1, S);
    ws[3 * 8 + c] = descale(t13 + o0, S); ws[4 * 8 + c] = descale(t13 - o0, S);
  }
  constexpr int S2 = CONST_BITS + PASS1_BITS + 3;
#pragma unroll
  for (int r = 0; r < 8; ++r) {  // pass 2: rows
    const int* w = ws + r * 8;
    uint8_t* o = out + r * 8;
    if (ZERO_TESTS && (w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0) {
      const uint8_t v = idct_range(descale(w[0], PASS1_BITS + 3));
      for (int k = 0; k < 8; ++k) o[k] = v;
      continue;
    }
    int64_t z1 = (int64_t)(w[2] + w[6]) * 4433;
    const int64_t tmp2 = z1 + (int64_t)w[6] * -15137, tmp3 = z1 + (int64_t)w[2] * 6270;
    const int64_t tmp0 = (int64_t)(w[0] + w[4]) << CONST_BITS;
    const int64_t tmp1 = (int64_t)(w[0] - w[4]) << CONST_BITS;
    const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    int64_t o0 = w[7], o1 = w[5], o2 = w[3], o3 = w[1];
    z1 = o0 + o3;
    int64_t z2 = o1 + o2, z3 = o0 + o2, z4 = o1 + o3;
    const int64_t z5 = (z3 + z4) * 9633;
    o0 *= 2446; o1 *= 16819; o2 *= 25172; o3 *= 12299;
    z1 *= -7373; z2 *= -20995; z3 *= -16069; z4 *= -3196;
    z3 += z5; z4 += z5;
    o0 += z1 + z3; o1 += z2 + z4; o2 += z2 + z3; o3 += z1 + z4;
    o[0] = idct_range(descale(t10 + o3, S2)); o[7] = idct_range(descale(t10 - o3, S2));
    o[1] = idct_range(descale(t11 + o2, S2)); o[6] = idct_range(descale(t11 - o2, S2));
    o[2] = idct_range(descale(t12 + o1, S2)); o[5] = idct_range(descale(t12 - o1, S2));
    o[3] = idct_range(descale(t13 + o0, S2)); o[4] = idct_range(descale(t13 - o0, S2));
  }
}

// ------------------------------------------------------------ pixels
// Sample (row, col) of component k (component coordinates; inside its window).
KFB_HD inline int sample(const uint8_t* planes, const Comp& c, int row, int col) {
  const int br = (row >> 3) - c.by0, bc = (col >> 3) - c.bx0;
  if ((unsigned)br >= (unsigned)c.bh || (unsigned)bc >= (unsigned)c.bw) return 0;  // (guard)
  return planes[64L * (c.blk + br * c.bw + bc) + ((row & 7) << 3) + (col & 7)];
}

// Chroma sample at full-resolution pixel (py, px), fancy-upsampled.
KFB_HD inline int chroma(const uint8_t* planes, const Comp& c, int hmax, int vmax, int py,
                         int px) {
  const int hr = hmax / c.h, vr = vmax / c.v;
  if (hr == 1 && vr == 1) return sample(planes, c, py, px);
  const int col = px >> (hr - 1), u = px & (hr - 1);
  if (vr == 1) {  // h2v1: (3 * nearer + farther + 1 or 2) >> 2
    const int s = sample(planes, c, py, col);
    if (u == 0) return col == 0 ? s : (3 * s + sample(planes, c, py, col - 1) + 1) >> 2;
    return col == c.dw - 1 ? s : (3 * s + sample(planes, c, py, col + 1) + 2) >> 2;
  }
  // h2v2: vertical 3:1 column sums (rows beyond the image repeat the edge
  // row), then horizontal 3:1 with the +8 / +7 bias of each output parity
  const int row = py >> 1;
  const int rn = (py & 1) ? (row + 1 < c.dh ? row + 1 : row) : (row > 0 ? row - 1 : row);
  auto colsum = [&](int k) { return 3 * sample(planes, c, row, k) + sample(planes, c, rn, k); };
  const int t = colsum(col);
  if (u == 0) return col == 0 ? (4 * t + 8) >> 4 : (3 * t + colsum(col - 1) + 8) >> 4;
  return col == c.dw - 1 ? (4 * t + 7) >> 4 : (3 * t + colsum(col + 1) + 7) >> 4;
}

KFB_HD inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// RGB of full-resolution pixel (py, px).
KFB_HD inline void pixel_rgb(const uint8_t* planes, const Desc& d, int py, int px, int (&rgb)[3]) {
  const int y = sample(planes, d.c[0], py, px);
  if (d.ncomp == 1) {
    rgb[0] = rgb[1] = rgb[2] = y;
    return;
  }
  const int hmax = d.c[0].h, vmax = d.c[0].v;
  const int cb = chroma(planes, d.c[1], hmax, vmax, py, px) - 128;
  const int cr = chroma(planes, d.c[2], hmax, vmax, py, px) - 128;
  // 16-bit fixed point, as libjpeg's ycc -> rgb tables
  const int rr = (91881 * cr + 32768) >> 16;
  const int bb = (116130 * cb + 32768) >> 16;
  const int gg = (-22554 * cb + 32768 - 46802 * cr) >> 16;
  rgb[0] = clamp255(y + rr);
  rgb[1] = clamp255(y + gg);
  rgb[2] = clamp255(y + bb);
}

// Output pixel (i, j) of the oh x ow bilinear resize (half-pixel centres,
// edge clamp) of the crop - the same arithmetic as the host pipeline's
// resize_bilinear.
KFB_HD inline void resized_pixel(const uint8_t* planes, const Desc& d, int oh, int ow, int i, int j,
                                 uint8_t* out3) {
#ifdef __clang__
#pragma clang fp contract(off)  // (the host build has no FMA contraction either)
#endif
  const float fy = (float)d.ch / (float)oh, fx = (float)d.cw / (float)ow;
  float sy = ((float)i + 0.5f) * fy - 0.5f;
  sy = sy < 0.f ? 0.f : sy > (float)(d.ch - 1) ? (float)(d.ch - 1) : sy;
  float sx = ((float)j + 0.5f) * fx - 0.5f;
  sx = sx < 0.f ? 0.f : sx > (float)(d.cw - 1) ? (float)(d.cw - 1) : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + 1 < d.ch ? y0 + 1 : d.ch - 1, x1 = x0 + 1 < d.cw ? x0 + 1 : d.cw - 1;
  const float ay = sy - (float)y0, ax = sx - (float)x0;
  int p00[3], p01[3], p10[3], p11[3];
  pixel_rgb(planes, d, d.cy + y0, d.cx + x0, p00);
  pixel_rgb(planes, d, d.cy + y0, d.cx + x1, p01);
  pixel_rgb(planes, d, d.cy + y1, d.cx + x0, p10);
  pixel_rgb(planes, d, d.cy + y1, d.cx + x1, p11);
  for (int k = 0; k < 3; ++k) {
    const float t = (float)p00[k] + ax * (float)(p01[k] - p00[k]);
    const float b = (float)p10[k] + ax * (float)(p11[k] - p10[k]);
    float v = t + ay * (b - t) + 0.5f;
    v = v < 0.f ? 0.f : v > 255.f ? 255.f : v;
    out3[k] = (uint8_t)v;
  }
}

// resized_pixel over a crop already reconstructed into rgb (the crop's
// [ch][cw][3] pixels from pixel 3 * rgb_off): the same arithmetic, so the
// same bytes.
KFB_HD inline void resized_from_rgb(const uint8_t* rgb, const Desc& d, int oh, int ow, int i,
                                    int j, uint8_t* out3) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  const float fy = (float)d.ch / (float)oh, fx = (float)d.cw / (float)ow;
  float sy = ((float)i + 0.5f) * fy - 0.5f;
  sy = sy < 0.f ? 0.f : sy > (float)(d.ch - 1) ? (float)(d.ch - 1) : sy;
  float sx = ((float)j + 0.5f) * fx - 0.5f;
  sx = sx < 0.f ? 0.f : sx > (float)(d.cw - 1) ? (float)(d.cw - 1) : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + 1 < d.ch ? y0 + 1 : d.ch - 1, x1 = x0 + 1 < d.cw ? x0 + 1 : d.cw - 1;
  const float ay = sy - (float)y0, ax = sx - (float)x0;
  const uint8_t* base = rgb + 3L * d.rgb_off;
  const uint8_t* q00 = base + 3L * ((long)y0 * d.cw + x0);
  const uint8_t* q01 = base + 3L * ((long)y0 * d.cw + x1);
  const uint8_t* q10 = base + 3L * ((long)y1 * d.cw + x0);
  const uint8_t* q11 = base + 3L * ((long)y1 * d.cw + x1);
  for (int k = 0; k < 3; ++k) {
    const int p00 = q00[k], p01 = q01[k], p10 = q10[k], p11 = q11[k];
    const float t = (float)p00 + ax * (float)(p01 - p00);
    const float b = (float)p10 + ax * (float)(p11 - p10);
    float v = t + ay * (b - t) + 0.5f;
    v = v < 0.f ? 0.f : v > 255.f ? 255.f : v;
    out3[k] = (uint8_t)v;
  }
}

}  // namespace jpg
}  // namespace kfb
