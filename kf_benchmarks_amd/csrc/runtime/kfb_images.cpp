// Native host half of the ImageNet train preprocessing: tf.train.Example
// parse -> JPEG decode (DCT-domain downscale when the crop allows) -> random
// bbox crop -> bilinear resize to uint8 [H][W][3], plus the image's
// augmentation parameters (flip, colour-distortion draws) for the device pass
// in csrc/augment.hip.  One call per batch from Python, with the GIL released
// (ctypes), spread over a persistent worker pool: the reference runs this
// stage as TF's parallel input ops (tcb/preprocessing.py:192-265,
// :505-548); a Python thread pool over PIL topped out near 800 images/sec on
// the 16 CPUs of a MI355X box share.
//
// JPEG decoding uses libjpeg through dlopen ("libjpeg.so.9" built against the
// jpeglib.h this file is compiled with; KFB_LIBJPEG overrides the path).
// Without it kfbrt_imgpipe_available() returns 0 and Python keeps its PIL
// path.
#include <dlfcn.h>
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#if defined(KFB_HAVE_JPEGLIB)
extern "C" {
#include <jpeglib.h>
}
#endif

#include "jpeg_recon.h"

#define API extern "C" __attribute__((visibility("default")))

extern "C" long kfbrt_parse_example(const uint8_t* data, size_t n, uint8_t* out, size_t cap);

namespace {

// ------------------------------------------------------------ RNG
struct Rng {  // xoshiro256** seeded by splitmix64
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; ++i) {
      seed += 0x9E3779B97F4A7C15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  double uniform(double a, double b) { return a + (b - a) * uniform(); }
  int64_t integers(int64_t lo, int64_t hi) {  // [lo, hi)
    return hi <= lo ? lo : lo + (int64_t)(next() % (uint64_t)(hi - lo));
  }
};

// ------------------------------------------------------------ Example fields
struct Fields {
  const uint8_t* jpeg = nullptr;
  size_t jpeg_len = 0;
  int64_t label = -1;
  std::vector<float> box[4];  // ymin, xmin, ymax, xmax
};

bool read_fields(const uint8_t* p, const uint8_t* e, Fields& f) {
  static const char* kBox[4] = {"image/object/bbox/ymin", "image/object/bbox/xmin",
                                "image/object/bbox/ymax", "image/object/bbox/xmax"};
  while (p + 4 <= e) {
    uint32_t kl;
    std::memcpy(&kl, p, 4);
    p += 4;
    if ((size_t)(e - p) < kl + 5) return false;
    const char* key = (const char*)p;
    p += kl;
    const uint8_t kind = *p++;
    uint32_t cnt;
    std::memcpy(&cnt, p, 4);
    p += 4;
    auto is = [&](const char* k) { return strlen(k) == kl && std::memcmp(key, k, kl) == 0; };
    if (kind == 1) {
      for (uint32_t i = 0; i < cnt; ++i) {
        if (e - p < 4) return false;
        uint32_t bl;
        std::memcpy(&bl, p, 4);
        p += 4;
        if ((uint32_t)(e - p) < bl) return false;
        if (i == 0 && is("image/encoded")) {
          f.jpeg = p;
          f.jpeg_len = bl;
        }
        p += bl;
      }
    } else if (kind == 2) {
      if ((size_t)(e - p) < (size_t)cnt * 4) return false;
      for (int b = 0; b < 4; ++b)
        if (is(kBox[b])) {
          f.box[b].resize(cnt);
          std::memcpy(f.box[b].data(), p, (size_t)cnt * 4);
        }
      p += (size_t)cnt * 4;
    } else if (kind == 3) {
      if ((size_t)(e - p) < (size_t)cnt * 8) return false;
      if (cnt > 0 && is("image/class/label")) std::memcpy(&f.label, p, 8);
      p += (size_t)cnt * 8;
    }
  }
  return true;
}

// tf.image.sample_distorted_bounding_box (min_object_covered 0.1, aspect
// 0.75-1.33, area 0.05-1.0, 100 attempts, whole image on failure); the same
// procedure as data/preprocessing.py:sample_distorted_bounding_box.
void sample_box(int H, int W, const Fields& f, Rng& rng, int& y, int& x, int& h, int& w) {
  size_t nb = f.box[0].size();
  for (int b = 1; b < 4; ++b) nb = std::min(nb, f.box[b].size());
  const double min_area = 0.05 * H * W, max_area = 1.0 * H * W;
  for (int attempt = 0; attempt < 100; ++attempt) {
    double by0 = 0, bx0 = 0, by1 = H, bx1 = W;
    if (nb > 0) {
      const size_t k = (size_t)rng.integers(0, (int64_t)nb);
      by0 = f.box[0][k] * H;
      bx0 = f.box[1][k] * W;
      by1 = f.box[2][k] * H;
      bx1 = f.box[3][k] * W;
    }
    const double ar = rng.uniform(0.75, 1.33);
    int max_h = (int)std::lround(std::sqrt(max_area / ar));
    if (std::lround(max_h * ar) > W) max_h = (int)((W + 0.5 - 1e-7) / ar);
    max_h = std::min(max_h, H);
    const int min_h = std::min((int)std::lround(std::sqrt(min_area / ar)), max_h);
    if (max_h < 1) continue;
    const int hh = (int)rng.integers(std::max(min_h, 1), max_h + 1);
    const int ww = (int)std::lround(hh * ar);
    if (ww < 1 || ww > W || (double)hh * ww < min_area || (double)hh * ww > max_area) continue;
    const int yy = (int)rng.integers(0, H - hh + 1);
    const int xx = (int)rng.integers(0, W - ww + 1);
    const double iy = std::max(0.0, std::min(by1, (double)(yy + hh)) - std::max(by0, (double)yy));
    const double ix = std::max(0.0, std::min(bx1, (double)(xx + ww)) - std::max(bx0, (double)xx));
    const double barea = std::max((by1 - by0) * (bx1 - bx0), 1e-12);
    if (iy * ix / barea < 0.1) continue;
    y = yy;
    x = xx;
    h = hh;
    w = ww;
    return;
  }
  y = 0;
  x = 0;
  h = H;
  w = W;
}

// bilinear resize (half-pixel centres, edge clamp) of an RGB crop
void resize_bilinear(const uint8_t* src, int sh, int sw, uint8_t* dst, int dh, int dw) {
  const float fy = (float)sh / dh, fx = (float)sw / dw;
  std::vector<int> x0(dw), x1(dw);
  std::vector<float> ax(dw);
  for (int j = 0; j < dw; ++j) {
    float sx = (j + 0.5f) * fx - 0.5f;
    sx = std::min(std::max(sx, 0.f), (float)(sw - 1));
    x0[j] = (int)sx;
    x1[j] = std::min(x0[j] + 1, sw - 1);
    ax[j] = sx - x0[j];
  }
  for (int i = 0; i < dh; ++i) {
    float sy = (i + 0.5f) * fy - 0.5f;
    sy = std::min(std::max(sy, 0.f), (float)(sh - 1));
    const int y0 = (int)sy, y1 = std::min(y0 + 1, sh - 1);
    const float ay = sy - y0;
    const uint8_t* r0 = src + (size_t)y0 * sw * 3;
    const uint8_t* r1 = src + (size_t)y1 * sw * 3;
    uint8_t* o = dst + (size_t)i * dw * 3;
    for (int j = 0; j < dw; ++j) {
      for (int c = 0; c < 3; ++c) {
        const float t = r0[x0[j] * 3 + c] + ax[j] * (r0[x1[j] * 3 + c] - r0[x0[j] * 3 + c]);
        const float b = r1[x0[j] * 3 + c] + ax[j] * (r1[x1[j] * 3 + c] - r1[x0[j] * 3 + c]);
        o[j * 3 + c] = (uint8_t)std::min(255.f, std::max(0.f, t + ay * (b - t) + 0.5f));
      }
    }
  }
}

// ------------------------------------------------------------ libjpeg
#if defined(KFB_HAVE_JPEGLIB)
struct Jpeg {
  bool ok = false;
  struct jpeg_error_mgr* (*std_error)(struct jpeg_error_mgr*) = nullptr;
  void (*create)(j_decompress_ptr, int, size_t) = nullptr;
  void (*mem_src)(j_decompress_ptr, const unsigned char*, unsigned long) = nullptr;
  int (*read_header)(j_decompress_ptr, boolean) = nullptr;
  boolean (*start)(j_decompress_ptr) = nullptr;
  JDIMENSION (*read_scanlines)(j_decompress_ptr, JSAMPARRAY, JDIMENSION) = nullptr;
  void (*abort_)(j_decompress_ptr) = nullptr;
  void (*destroy)(j_decompress_ptr) = nullptr;
  jvirt_barray_ptr* (*read_coefficients)(j_decompress_ptr) = nullptr;  // (optional)
};

Jpeg& jpeg() {
  static Jpeg j;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = getenv("KFB_LIBJPEG");
    void* h = nullptr;
    if (env) h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libjpeg.so.9", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/conda/lib/libjpeg.so.9", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
#define KFB_J(f, n) j.f = (decltype(j.f))dlsym(h, n)
    KFB_J(std_error, "jpeg_std_error");
    KFB_J(create, "jpeg_CreateDecompress");
    KFB_J(mem_src, "jpeg_mem_src");
    KFB_J(read_header, "jpeg_read_header");
    KFB_J(start, "jpeg_start_decompress");
    KFB_J(read_scanlines, "jpeg_read_scanlines");
    KFB_J(abort_, "jpeg_abort_decompress");
    KFB_J(destroy, "jpeg_destroy_decompress");
    KFB_J(read_coefficients, "jpeg_read_coefficients");
#undef KFB_J
    j.ok = j.std_error && j.create && j.mem_src && j.read_header && j.start &&
           j.read_scanlines && j.abort_ && j.destroy;
  });
  return j;
}

struct ErrMgr {
  struct jpeg_error_mgr pub;
  jmp_buf jb;
};

void on_error(j_common_ptr c) { longjmp(reinterpret_cast<ErrMgr*>(c->err)->jb, 1); }
void on_message(j_common_ptr) {}
#endif

struct Config {
  int height, width, distortions, yiq, draft;
};

// One image: 0 on success; on a decode failure the output is mid-grey.
int process(const Config& cfg, const uint8_t* rec, size_t len, uint64_t seed, int position,
            uint8_t* out, float* prm, int32_t* label, std::vector<uint8_t>& scratch,
            std::vector<uint8_t>& crop) {
  const size_t img_bytes = (size_t)cfg.height * cfg.width * 3;
  std::memset(prm, 0, 8 * sizeof(float));
  *label = -1;
  scratch.resize(len + 4096);
  long n = kfbrt_parse_example(rec, len, scratch.data(), scratch.size());
  if (n == -2) {
    scratch.resize(len * 2 + 65536);
    n = kfbrt_parse_example(rec, len, scratch.data(), scratch.size());
  }
  Fields f;
  if (n < 0 || !read_fields(scratch.data(), scratch.data() + n, f) || !f.jpeg) {
    std::memset(out, 128, img_bytes);
    return 1;
  }
  *label = (int32_t)f.label;
  Rng rng(seed);
#if defined(KFB_HAVE_JPEGLIB)
  Jpeg& J = jpeg();
  if (!J.ok) {
    std::memset(out, 128, img_bytes);
    return 1;
  }
  struct jpeg_decompress_struct ci;
  ErrMgr em;
  ci.err = J.std_error(&em.pub);
  em.pub.error_exit = on_error;
  em.pub.output_message = on_message;
  if (setjmp(em.jb)) {
    J.destroy(&ci);
    std::memset(out, 128, img_bytes);
    return 1;
  }
  J.create(&ci, JPEG_LIB_VERSION, sizeof(ci));
  J.mem_src(&ci, f.jpeg, (unsigned long)f.jpeg_len);
  J.read_header(&ci, TRUE);
  const int H0 = (int)ci.image_height, W0 = (int)ci.image_width;
  int y, x, h, w;
  sample_box(H0, W0, f, rng, y, x, h, w);
  const bool flip = rng.uniform() < 0.5;
  int d = 1;
  if (cfg.draft)
    while (d < 8 && w / (2 * d) >= cfg.width && h / (2 * d) >= cfg.height) d *= 2;
  ci.scale_num = 1;
  ci.scale_denom = d;
  ci.out_color_space = JCS_RGB;
  ci.dct_method = JDCT_ISLOW;  // tf.image.decode_jpeg default (tcb sets none)
  J.start(&ci);
  const int OW = (int)ci.output_width, OH = (int)ci.output_height;
  // crop in output (scaled) coordinates
  int cx = (int)((long)x * OW / W0), cy = (int)((long)y * OH / H0);
  int cw = std::max(1, (int)std::lround((double)w * OW / W0));
  int ch = std::max(1, (int)std::lround((double)h * OH / H0));
  cw = std::min(cw, OW - cx);
  ch = std::min(ch, OH - cy);
  // (scratch holds the parsed record, i.e. the JPEG bytes libjpeg is reading)
  thread_local std::vector<uint8_t> rowbuf;
  rowbuf.resize((size_t)OW * 3);
  crop.resize((size_t)cw * ch * 3);
  JSAMPROW row = rowbuf.data();
  while ((int)ci.output_scanline < cy + ch) {
    const int r = (int)ci.output_scanline;
    J.read_scanlines(&ci, &row, 1);
    if (r >= cy) std::memcpy(crop.data() + (size_t)(r - cy) * cw * 3, row + (size_t)cx * 3, (size_t)cw * 3);
  }
  J.abort_(&ci);
  J.destroy(&ci);
  if (cw == cfg.width && ch == cfg.height) std::memcpy(out, crop.data(), img_bytes);
  else resize_bilinear(crop.data(), ch, cw, out, cfg.height, cfg.width);
  prm[0] = flip ? 1.f : 0.f;
  if (cfg.distortions) {
    prm[1] = (float)rng.uniform(-32. / 255., 32. / 255.);
    auto sat_hue = [&]() {
      if (cfg.yiq) {
        prm[3] = (float)rng.uniform(-0.2, 0.2);
        prm[2] = (float)rng.uniform(0.5, 1.5);
      } else {
        prm[2] = (float)rng.uniform(0.5, 1.5);
        prm[3] = (float)rng.uniform(-0.2, 0.2);
      }
    };
    const int order = position % 2;
    if (order == 0) {
      sat_hue();
      prm[4] = (float)rng.uniform(0.5, 1.5);
    } else {
      prm[4] = (float)rng.uniform(0.5, 1.5);
      sat_hue();
    }
    prm[5] = (float)order;
    prm[6] = 1.f;
  }
  return 0;
#else
  (void)position;
  (void)crop;
  std::memset(out, 128, img_bytes);
  return 1;
#endif
}

// ------------------------------------------------------------ coefficients
// The GPU-reconstruction form of process(): the same crop / flip / colour
// draws, but the host only entropy-decodes (jpeg_read_coefficients) and
// copies the coefficient blocks that cover the crop (plus the one-sample
// chroma margin the upsampling filter reads) into the batch arena;
// csrc/jpeg.hip does the rest (jpeg_recon.h).  Layouts the reconstruction
// does not cover (CMYK / RGB-coded / odd sampling / DCT-scaled files) and an
// arena overflow take process() and are marked MODE_HOST.
struct Arena {
  int16_t* blocks = nullptr;  // [cap][64]
  long cap = 0;
  std::atomic<long> next{0};
};

#if defined(KFB_HAVE_JPEGLIB)
// Block window of component `c` covering full-resolution rows [y, y+h) and
// columns [x, x+w) (+ the upsampling margin).
static void comp_window(const jpeg_decompress_struct& ci, int k, int y, int x, int h, int w,
                        kfb::jpg::Comp& c) {
  const jpeg_component_info& cp = ci.comp_info[k];
  const int hmax = ci.max_h_samp_factor, vmax = ci.max_v_samp_factor;
  c.h = cp.h_samp_factor;
  c.v = cp.v_samp_factor;
  c.dw = (int)(((long)ci.image_width * c.h + hmax - 1) / hmax);
  c.dh = (int)(((long)ci.image_height * c.v + vmax - 1) / vmax);
  const int hr = hmax / c.h, vr = vmax / c.v;
  int r0 = y / vr, r1 = (y + h - 1) / vr, c0 = x / hr, c1 = (x + w - 1) / hr;
  if (vr > 1) { r0 -= 1; r1 += 1; }
  if (hr > 1) { c0 -= 1; c1 += 1; }
  r0 = std::max(r0, 0);
  c0 = std::max(c0, 0);
  r1 = std::min(r1, c.dh - 1);
  c1 = std::min(c1, c.dw - 1);
  c.by0 = r0 / 8;
  c.bx0 = c0 / 8;
  c.bh = r1 / 8 - c.by0 + 1;
  c.bw = c1 / 8 - c.bx0 + 1;
  c.pad = 0;
}

static bool coef_layout_ok(const jpeg_decompress_struct& ci) {
  if (ci.block_size != 8 || ci.image_width < 3 || ci.image_height < 1) return false;
  if (ci.num_components == 1) return ci.jpeg_color_space == JCS_GRAYSCALE;
  if (ci.num_components != 3 || ci.jpeg_color_space != JCS_YCbCr) return false;
  const int hmax = ci.max_h_samp_factor, vmax = ci.max_v_samp_factor;
  if (ci.comp_info[0].h_samp_factor != hmax || ci.comp_info[0].v_samp_factor != vmax) return false;
  for (int k = 1; k < 3; ++k) {
    const int h = ci.comp_info[k].h_samp_factor, v = ci.comp_info[k].v_samp_factor;
    if (hmax % h || vmax % v) return false;
    const int hr = hmax / h, vr = vmax / v;
    // (libjpeg-turbo's fancy upsamplers: h1v1, h2v1, h2v2; h1v2 and wider
    // ratios keep the host decode)
    if (!((hr == 1 && vr == 1) || (hr == 2 && vr == 1) || (hr == 2 && vr == 2))) return false;
    if (hr == 2 && (ci.image_width * h + hmax - 1) / hmax <= 2) return false;
  }
  return true;
}
#endif

// 0: packed (MODE_COEF) or decoded on the host (MODE_HOST); 1: failure
// (grey, MODE_HOST).  `host_img`: this image's slot of the host-decoded
// buffer.
int pack(const Config& cfg, const uint8_t* rec, size_t len, uint64_t seed, int position,
         Arena& ar, kfb::jpg::Desc* d, float* prm, int32_t* label, uint8_t* host_img, int slot,
         std::vector<uint8_t>& scratch, std::vector<uint8_t>& crop) {
  std::memset(d, 0, sizeof(*d));
  d->mode = kfb::jpg::MODE_HOST;
  d->host_slot = slot;
#if defined(KFB_HAVE_JPEGLIB)
  Jpeg& J = jpeg();
  if (J.ok && J.read_coefficients) {
    scratch.resize(len + 4096);
    long n = kfbrt_parse_example(rec, len, scratch.data(), scratch.size());
    if (n == -2) {
      scratch.resize(len * 2 + 65536);
      n = kfbrt_parse_example(rec, len, scratch.data(), scratch.size());
    }
    Fields f;
    if (n >= 0 && read_fields(scratch.data(), scratch.data() + n, f) && f.jpeg) {
      struct jpeg_decompress_struct ci;
      ErrMgr em;
      ci.err = J.std_error(&em.pub);
      em.pub.error_exit = on_error;
      em.pub.output_message = on_message;
      bool packed = false;
      if (setjmp(em.jb)) {
        J.destroy(&ci);
        packed = false;
      } else {
        J.create(&ci, JPEG_LIB_VERSION, sizeof(ci));
        J.mem_src(&ci, f.jpeg, (unsigned long)f.jpeg_len);
        J.read_header(&ci, TRUE);
        if (coef_layout_ok(ci)) {
          Rng rng(seed);
          const int H0 = (int)ci.image_height, W0 = (int)ci.image_width;
          int y, x, h, w;
          sample_box(H0, W0, f, rng, y, x, h, w);
          const bool flip = rng.uniform() < 0.5;
          kfb::jpg::Desc& D = *d;
          D.ncomp = ci.num_components;
          D.cy = y;
          D.cx = x;
          D.ch = h;
          D.cw = w;
          long need = 0;
          for (int k = 0; k < D.ncomp; ++k) {
            comp_window(ci, k, y, x, h, w, D.c[k]);
            need += (long)D.c[k].bh * D.c[k].bw;
          }
          const long base = ar.next.fetch_add(need);
          if (base + need <= ar.cap) {
            jvirt_barray_ptr* coefs = J.read_coefficients(&ci);
            long b = base;
            for (int k = 0; k < D.ncomp; ++k) {
              kfb::jpg::Comp& c = D.c[k];
              c.blk = (int)b;
              const JQUANT_TBL* qt = ci.comp_info[k].quant_table;
              for (int i = 0; i < 64; ++i) D.q[k][i] = qt ? qt->quantval[i] : 1;
              for (int r = 0; r < c.bh; ++r) {
                JBLOCKARRAY rows = (*ci.mem->access_virt_barray)(
                    (j_common_ptr)&ci, coefs[k], (JDIMENSION)(c.by0 + r), 1, FALSE);
                std::memcpy(ar.blocks + 64 * b, rows[0][c.bx0], sizeof(JBLOCK) * c.bw);
                b += c.bw;
              }
            }
            static_assert(sizeof(JBLOCK) == 128, "16-bit coefficients");
            D.mode = kfb::jpg::MODE_COEF;
            *label = (int32_t)f.label;
            prm[0] = flip ? 1.f : 0.f;
            if (cfg.distortions) {
              // (the same draws, in the same order, as process())
              std::memset(prm + 1, 0, 7 * sizeof(float));
              prm[1] = (float)rng.uniform(-32. / 255., 32. / 255.);
              auto sat_hue = [&]() {
                if (cfg.yiq) {
                  prm[3] = (float)rng.uniform(-0.2, 0.2);
                  prm[2] = (float)rng.uniform(0.5, 1.5);
                } else {
                  prm[2] = (float)rng.uniform(0.5, 1.5);
                  prm[3] = (float)rng.uniform(-0.2, 0.2);
                }
              };
              const int order = position % 2;
              if (order == 0) {
                sat_hue();
                prm[4] = (float)rng.uniform(0.5, 1.5);
              } else {
                prm[4] = (float)rng.uniform(0.5, 1.5);
                sat_hue();
              }
              prm[5] = (float)order;
              prm[6] = 1.f;
            } else {
              std::memset(prm + 1, 0, 7 * sizeof(float));
            }
            packed = true;
          }
        }
        J.abort_(&ci);
        J.destroy(&ci);
      }
      if (packed) return 0;
    }
  }
#endif
  (void)ar;
  d->mode = kfb::jpg::MODE_HOST;
  d->host_slot = slot;
  return process(cfg, rec, len, seed, position, host_img, prm, label, scratch, crop);
}

// ------------------------------------------------------------ worker pool
struct Pipe {
  Config cfg;
  std::vector<std::thread> threads;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  // current batch
  int n = 0;
  const uint8_t* const* recs = nullptr;
  const size_t* lens = nullptr;
  const uint64_t* seeds = nullptr;
  const int* positions = nullptr;
  uint8_t* images = nullptr;
  float* params = nullptr;
  int32_t* labels = nullptr;
  // coefficient mode (kfbrt_imgpipe_run_coef): descriptors + block arena
  kfb::jpg::Desc* descs = nullptr;
  Arena* arena = nullptr;
  std::atomic<int> next{0}, failed{0}, hosted{0};
  int active = 0;
  long gen = 0;
  bool stop = false;

  void work() {
    std::vector<uint8_t> scratch, crop;
    const size_t img_bytes = (size_t)cfg.height * cfg.width * 3;
    for (int i; (i = next.fetch_add(1)) < n;) {
      if (descs) {
        failed += pack(cfg, recs[i], lens[i], seeds[i], positions[i], *arena, descs + i,
                       params + (size_t)i * 8, labels + i, images + i * img_bytes, i, scratch,
                       crop);
        hosted += descs[i].mode == kfb::jpg::MODE_HOST;
      } else {
        failed += process(cfg, recs[i], lens[i], seeds[i], positions[i], images + i * img_bytes,
                          params + (size_t)i * 8, labels + i, scratch, crop);
      }
    }
  }

  void loop() {
    long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      work();
      {
        std::lock_guard<std::mutex> l(mu);
        if (--active == 0) done_cv.notify_all();
      }
    }
  }
};

}  // namespace

API int kfbrt_imgpipe_available() {
#if defined(KFB_HAVE_JPEGLIB)
  return jpeg().ok ? 1 : 0;
#else
  return 0;
#endif
}

API void* kfbrt_imgpipe_create(int threads, int height, int width, int distortions, int yiq,
                               int draft) {
  Pipe* p = new Pipe();
  p->cfg = Config{height, width, distortions, yiq, draft};
  for (int t = 0; t < std::max(0, threads - 1); ++t) p->threads.emplace_back([p] { p->loop(); });
  return p;
}

// Processes n records into images [n][H][W][3] uint8, params [n][8] f32 and
// labels [n] i32 (per-image seeds and batch positions given); returns the
// number of images that could not be decoded (mid-grey, label from the
// record or -1).  The calling thread works too.
API int kfbrt_imgpipe_run(void* h, int n, const uint8_t* const* recs, const size_t* lens,
                          const uint64_t* seeds, const int* positions, uint8_t* images,
                          float* params, int32_t* labels) {
  Pipe* p = static_cast<Pipe*>(h);
  {
    std::lock_guard<std::mutex> l(p->mu);
    p->n = n;
    p->recs = recs;
    p->lens = lens;
    p->seeds = seeds;
    p->positions = positions;
    p->images = images;
    p->params = params;
    p->labels = labels;
    p->next = 0;
    p->failed = 0;
    p->active = (int)p->threads.size();
    ++p->gen;
  }
  p->cv.notify_all();
  p->work();
  std::unique_lock<std::mutex> l(p->mu);
  p->done_cv.wait(l, [&] { return p->active == 0; });
  return p->failed.load();
}

// Coefficient mode: descs [n] (kfb::jpg::Desc), blocks [cap][64] int16 (the
// batch arena), images [n][H][W][3] for the images decoded on the host
// (MODE_HOST).  out3[0] = arena blocks used, out3[1] = images decoded on the
// host, out2[2] = pixels of the reconstructed crops (the device's crop-RGB
// buffer); returns the failure count as kfbrt_imgpipe_run.
API int kfbrt_imgpipe_run_coef(void* h, int n, const uint8_t* const* recs, const size_t* lens,
                               const uint64_t* seeds, const int* positions, void* descs,
                               int16_t* blocks, long cap, uint8_t* images, float* params,
                               int32_t* labels, long* out2) {
  Pipe* p = static_cast<Pipe*>(h);
  Arena ar;
  ar.blocks = blocks;
  ar.cap = cap;
  {
    std::lock_guard<std::mutex> l(p->mu);
    p->n = n;
    p->recs = recs;
    p->lens = lens;
    p->seeds = seeds;
    p->positions = positions;
    p->images = images;
    p->params = params;
    p->labels = labels;
    p->descs = static_cast<kfb::jpg::Desc*>(descs);
    p->arena = &ar;
    p->next = 0;
    p->failed = 0;
    p->hosted = 0;
    p->active = (int)p->threads.size();
    ++p->gen;
  }
  p->cv.notify_all();
  p->work();
  std::unique_lock<std::mutex> l(p->mu);
  p->done_cv.wait(l, [&] { return p->active == 0; });
  // each reconstructed crop's place in the device's crop-RGB buffer (batch
  // order: deterministic), out2[2] = its size in pixels
  long rgb = 0;
  for (int i = 0; i < n; ++i) {
    kfb::jpg::Desc& d = p->descs[i];
    d.rgb_off = -1;  // (the device rebuilds such a crop per output pixel)
    if (d.mode == kfb::jpg::MODE_COEF && rgb + (long)d.ch * d.cw < (1L << 31) / 3) {
      d.rgb_off = (int)rgb;
      rgb += (long)d.ch * d.cw;
    }
  }
  p->descs = nullptr;
  p->arena = nullptr;
  out2[0] = std::min(ar.next.load(), cap);
  out2[1] = p->hosted.load();
  out2[2] = rgb;
  return p->failed.load();
}

API int kfbrt_jpeg_desc_bytes() { return (int)sizeof(kfb::jpg::Desc); }

// Host reference of csrc/jpeg.hip (tests; and the CPU form of the device
// op): IDCT every arena block, then reconstruct + resize every image to
// out [n][oh][ow][3] (MODE_HOST images are copied from `images`).
API void kfbrt_jpeg_reconstruct(const void* descs, int n, const int16_t* blocks, long nblocks,
                                const uint8_t* images, int oh, int ow, uint8_t* out) {
  const kfb::jpg::Desc* D = static_cast<const kfb::jpg::Desc*>(descs);
  std::vector<uint8_t> planes((size_t)nblocks * 64);
  // block -> (image, component) for the dequantization table
  for (int i = 0; i < n; ++i) {
    if (D[i].mode != kfb::jpg::MODE_COEF) continue;
    for (int k = 0; k < D[i].ncomp; ++k) {
      const kfb::jpg::Comp& c = D[i].c[k];
      for (long b = c.blk; b < c.blk + (long)c.bh * c.bw; ++b)
        kfb::jpg::idct_islow(blocks + 64 * b, D[i].q[k], planes.data() + 64 * b);
    }
  }
  const size_t img = (size_t)oh * ow * 3;
  for (int i = 0; i < n; ++i) {
    uint8_t* o = out + i * img;
    if (D[i].mode != kfb::jpg::MODE_COEF) {
      std::memcpy(o, images + (size_t)D[i].host_slot * img, img);
      continue;
    }
    for (int r = 0; r < oh; ++r)
      for (int c = 0; c < ow; ++c)
        kfb::jpg::resized_pixel(planes.data(), D[i], oh, ow, r, c, o + ((size_t)r * ow + c) * 3);
  }
}

// Test hook: the whole image through the coefficient path (crop = image,
// no resize) into rgb [h][w][3] (cap bytes); returns 0, or -1 when the
// layout is not covered / the buffer is too small / the decode fails.
API int kfbrt_jpeg_decode_coef(const uint8_t* jpeg_bytes, size_t len, uint8_t* rgb, size_t cap,
                               int* hw) {
#if defined(KFB_HAVE_JPEGLIB)
  Jpeg& J = jpeg();
  if (!J.ok || !J.read_coefficients) return -1;
  struct jpeg_decompress_struct ci;
  ErrMgr em;
  ci.err = J.std_error(&em.pub);
  em.pub.error_exit = on_error;
  em.pub.output_message = on_message;
  kfb::jpg::Desc D;
  std::memset(&D, 0, sizeof(D));
  std::vector<int16_t> blocks;
  if (setjmp(em.jb)) {
    J.destroy(&ci);
    return -1;
  }
  J.create(&ci, JPEG_LIB_VERSION, sizeof(ci));
  J.mem_src(&ci, jpeg_bytes, (unsigned long)len);
  J.read_header(&ci, TRUE);
  const int H = (int)ci.image_height, W = (int)ci.image_width;
  if (!coef_layout_ok(ci) || (size_t)H * W * 3 > cap) {
    J.destroy(&ci);
    return -1;
  }
  D.mode = kfb::jpg::MODE_COEF;
  D.ncomp = ci.num_components;
  D.ch = H;
  D.cw = W;
  long total = 0;
  for (int k = 0; k < D.ncomp; ++k) {
    comp_window(ci, k, 0, 0, H, W, D.c[k]);
    D.c[k].blk = (int)total;
    total += (long)D.c[k].bh * D.c[k].bw;
  }
  blocks.resize((size_t)total * 64);
  jvirt_barray_ptr* coefs = J.read_coefficients(&ci);
  for (int k = 0; k < D.ncomp; ++k) {
    const kfb::jpg::Comp& c = D.c[k];
    const JQUANT_TBL* qt = ci.comp_info[k].quant_table;
    for (int i = 0; i < 64; ++i) D.q[k][i] = qt ? qt->quantval[i] : 1;
    for (int r = 0; r < c.bh; ++r) {
      JBLOCKARRAY rows = (*ci.mem->access_virt_barray)((j_common_ptr)&ci, coefs[k],
                                                       (JDIMENSION)(c.by0 + r), 1, FALSE);
      std::memcpy(blocks.data() + 64 * (c.blk + (long)r * c.bw), rows[0][c.bx0],
                  sizeof(JBLOCK) * c.bw);
    }
  }
  J.abort_(&ci);
  J.destroy(&ci);
  std::vector<uint8_t> planes((size_t)total * 64);
  for (int k = 0; k < D.ncomp; ++k)
    for (long b = D.c[k].blk; b < D.c[k].blk + (long)D.c[k].bh * D.c[k].bw; ++b)
      kfb::jpg::idct_islow(blocks.data() + 64 * b, D.q[k], planes.data() + 64 * b);
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      int px[3];
      kfb::jpg::pixel_rgb(planes.data(), D, r, c, px);
      for (int k = 0; k < 3; ++k) rgb[((size_t)r * W + c) * 3 + k] = (uint8_t)px[k];
    }
  hw[0] = H;
  hw[1] = W;
  return 0;
#else
  (void)jpeg_bytes;
  (void)len;
  (void)rgb;
  (void)cap;
  (void)hw;
  return -1;
#endif
}

API void kfbrt_imgpipe_destroy(void* h) {
  Pipe* p = static_cast<Pipe*>(h);
  {
    std::lock_guard<std::mutex> l(p->mu);
    p->stop = true;
  }
  p->cv.notify_all();
  for (auto& t : p->threads) t.join();
  delete p;
}
