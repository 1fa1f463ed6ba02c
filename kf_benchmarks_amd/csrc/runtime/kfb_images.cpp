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
  std::atomic<int> next{0}, failed{0};
  int active = 0;
  long gen = 0;
  bool stop = false;

  void work() {
    std::vector<uint8_t> scratch, crop;
    const size_t img_bytes = (size_t)cfg.height * cfg.width * 3;
    for (int i; (i = next.fetch_add(1)) < n;)
      failed += process(cfg, recs[i], lens[i], seeds[i], positions[i], images + i * img_bytes,
                        params + (size_t)i * 8, labels + i, scratch, crop);
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
