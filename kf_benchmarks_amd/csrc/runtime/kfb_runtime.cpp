// Host-side native runtime for kf_benchmarks_amd (plain C++17, no TF).
//
//  * CRC32C (Castagnoli), slicing-by-8, plus the TF/LevelDB "masked" form.
//  * TFRecord files: framing  [u64 len][u32 masked crc(len)][data][u32 masked crc(data)]
//    reader with CRC verification and a writer (tcb/preprocessing.py reads
//    these through tf.data; tcb/test_data/tfrecord_image_generator.py writes them).
//  * tf.train.Example decoding: Features map -> flat list of (key, kind,
//    bytes/int64/float values) entries, enough for image/encoded,
//    image/class/label, image/object/bbox/* (tcb/preprocessing.py:27-72).
//  * LevelDB-format SSTable ("table") writer and reader, the container of a
//    TF V2 checkpoint's .index file (tensor name -> BundleEntryProto),
//    so checkpoints keep the reference layout model.ckpt-N.{index,data-*}
//    (tcb/benchmark_cnn.py:905-950, 2076-2082, 2374-2378).
//
// Exposed as a C ABI for ctypes (kf_benchmarks_amd/runtime/__init__.py).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <cmath>

#define API extern "C" __attribute__((visibility("default")))

namespace {

// ------------------------------------------------------------------ CRC32C
uint32_t g_table[8][256];
bool g_init = false;

void crc_init() {
  if (g_init) return;
  const uint32_t poly = 0x82F63B78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (int i = 0; i < 256; ++i)
      g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xff];
  g_init = true;
}

uint32_t crc_extend(uint32_t crc, const uint8_t* p, size_t n) {
  crc_init();
  uint32_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = g_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = g_table[7][v & 0xff] ^ g_table[6][(v >> 8) & 0xff] ^ g_table[5][(v >> 16) & 0xff] ^
        g_table[4][(v >> 24) & 0xff] ^ g_table[3][(v >> 32) & 0xff] ^
        g_table[2][(v >> 40) & 0xff] ^ g_table[1][(v >> 48) & 0xff] ^ g_table[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return ~c;
}

inline uint32_t mask_crc(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

// ----------------------------------------------------------------- varints
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back(char((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back(char(v));
}

bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64 && p < end; shift += 7) {
    uint8_t b = *p++;
    v |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

void put_fixed32(std::string& s, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);
  s.append(b, 4);
}

void put_fixed64(std::string& s, uint64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  s.append(b, 8);
}

// --------------------------------------------------------------- TFRecord
struct RecordReader {
  FILE* f = nullptr;
  std::vector<uint8_t> buf;
  int verify = 1;
};

struct RecordWriter {
  FILE* f = nullptr;
};

// ----------------------------------------------------------------- SSTable
// LevelDB block: entries with shared-prefix compression, restart points
// every 16 keys, trailer = [restart offsets u32...][num_restarts u32].
struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  std::string last_key;
  int counter = 0;
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < 16) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(buf, shared);
    put_varint(buf, key.size() - shared);
    put_varint(buf, value.size());
    buf.append(key.data() + shared, key.size() - shared);
    buf.append(value);
    last_key = key;
    ++counter;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(out, r);
    put_fixed32(out, (uint32_t)restarts.size());
    return out;
  }
  bool empty() const { return buf.empty(); }
  size_t size_estimate() const { return buf.size() + restarts.size() * 4 + 4; }
};

const uint64_t kTableMagic = 0xdb4775248b80fb57ull;

// Appends a block + trailer(type 0 = uncompressed, masked crc) and returns its handle.
void write_block(std::string& file, const std::string& contents, uint64_t& off, uint64_t& size) {
  off = file.size();
  size = contents.size();
  file.append(contents);
  const char type = 0;
  uint32_t crc = crc_extend(0, (const uint8_t*)contents.data(), contents.size());
  crc = crc_extend(crc, (const uint8_t*)&type, 1);
  file.push_back(type);
  put_fixed32(file, mask_crc(crc));
}

void encode_handle(std::string& s, uint64_t off, uint64_t size) {
  put_varint(s, off);
  put_varint(s, size);
}

bool parse_block(const uint8_t* data, size_t n,
                 std::vector<std::pair<std::string, std::string>>& out) {
  if (n < 4) return false;
  uint32_t nrest;
  std::memcpy(&nrest, data + n - 4, 4);
  if (4 + 4ull * nrest > n) return false;
  const uint8_t* end = data + n - 4 - 4 * nrest;
  const uint8_t* p = data;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, shared) || !get_varint(p, end, nonshared) ||
        !get_varint(p, end, vlen))
      return false;
    if (shared > key.size() || p + nonshared + vlen > end) return false;
    key.resize(shared);
    key.append((const char*)p, nonshared);
    p += nonshared;
    out.emplace_back(key, std::string((const char*)p, vlen));
    p += vlen;
  }
  return true;
}

struct Table {
  std::vector<std::pair<std::string, std::string>> kv;
};

}  // namespace

// ====================================================================== C ABI
API uint32_t kfbrt_crc32c(const uint8_t* data, size_t n) { return crc_extend(0, data, n); }
API uint32_t kfbrt_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n) {
  return crc_extend(crc, data, n);
}
API uint32_t kfbrt_masked_crc32c(const uint8_t* data, size_t n) {
  return mask_crc(crc_extend(0, data, n));
}

API void* kfbrt_record_reader_open(const char* path, int verify) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return nullptr;
  auto* r = new RecordReader();
  r->f = f;
  r->verify = verify;
  return r;
}

// Returns record length (>=0), -1 at EOF, -2 on a corrupt record.
// The record stays valid until the next call (pointer via *out).
API long kfbrt_record_reader_next(void* h, const uint8_t** out) {
  auto* r = static_cast<RecordReader*>(h);
  uint8_t hdr[12];
  const size_t got = std::fread(hdr, 1, 12, r->f);
  if (got == 0) return -1;
  if (got != 12) return -2;
  uint64_t len;
  uint32_t lcrc;
  std::memcpy(&len, hdr, 8);
  std::memcpy(&lcrc, hdr + 8, 4);
  if (r->verify && mask_crc(crc_extend(0, hdr, 8)) != lcrc) return -2;
  if (len > (1ull << 34)) return -2;
  r->buf.resize(len + 4);
  if (std::fread(r->buf.data(), 1, len + 4, r->f) != len + 4) return -2;
  uint32_t dcrc;
  std::memcpy(&dcrc, r->buf.data() + len, 4);
  if (r->verify && mask_crc(crc_extend(0, r->buf.data(), len)) != dcrc) return -2;
  *out = r->buf.data();
  return (long)len;
}

API void kfbrt_record_reader_close(void* h) {
  auto* r = static_cast<RecordReader*>(h);
  if (r->f) std::fclose(r->f);
  delete r;
}

API void* kfbrt_record_writer_open(const char* path) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return nullptr;
  auto* w = new RecordWriter();
  w->f = f;
  return w;
}

API int kfbrt_record_writer_write(void* h, const uint8_t* data, size_t n) {
  auto* w = static_cast<RecordWriter*>(h);
  uint8_t hdr[12];
  uint64_t len = n;
  std::memcpy(hdr, &len, 8);
  uint32_t c = mask_crc(crc_extend(0, hdr, 8));
  std::memcpy(hdr + 8, &c, 4);
  uint32_t dc = mask_crc(crc_extend(0, data, n));
  if (std::fwrite(hdr, 1, 12, w->f) != 12) return -1;
  if (n && std::fwrite(data, 1, n, w->f) != n) return -1;
  if (std::fwrite(&dc, 1, 4, w->f) != 4) return -1;
  return 0;
}

API void kfbrt_record_writer_close(void* h) {
  auto* w = static_cast<RecordWriter*>(h);
  if (w->f) std::fclose(w->f);
  delete w;
}

// ------------------------------------------------------------- SSTable API
// Build a table from n sorted (key, value) pairs; writes the file at path.
API int kfbrt_table_write(const char* path, int n, const char* const* keys,
                          const size_t* key_lens, const char* const* vals,
                          const size_t* val_lens) {
  std::string file;
  BlockBuilder data, index;
  std::string last_key;
  bool pending = false;
  uint64_t poff = 0, psize = 0;
  for (int i = 0; i < n; ++i) {
    std::string k(keys[i], key_lens[i]);
    if (i > 0 && !(last_key < k)) return -1;  // keys must be strictly increasing
    if (pending) {
      std::string hv;
      encode_handle(hv, poff, psize);
      index.add(last_key, hv);
      pending = false;
    }
    data.add(k, std::string(vals[i], val_lens[i]));
    last_key = k;
    if (data.size_estimate() >= 4096) {
      write_block(file, data.finish(), poff, psize);
      data = BlockBuilder();
      pending = true;
    }
  }
  if (!data.empty()) {
    write_block(file, data.finish(), poff, psize);
    pending = true;
  }
  if (pending) {
    std::string hv;
    encode_handle(hv, poff, psize);
    index.add(last_key, hv);
  }
  uint64_t moff, msize, ioff, isize;
  BlockBuilder meta;
  write_block(file, meta.finish(), moff, msize);
  write_block(file, index.finish(), ioff, isize);
  std::string footer;
  encode_handle(footer, moff, msize);
  encode_handle(footer, ioff, isize);
  footer.resize(40, '\0');
  put_fixed64(footer, kTableMagic);
  file.append(footer);
  FILE* f = std::fopen(path, "wb");
  if (!f) return -2;
  const size_t w = std::fwrite(file.data(), 1, file.size(), f);
  std::fclose(f);
  return w == file.size() ? 0 : -3;
}

// Reads a whole table; returns a handle (nullptr on error, *err set).
API void* kfbrt_table_read(const char* path, int* err) {
  *err = 0;
  FILE* f = std::fopen(path, "rb");
  if (!f) { *err = -1; return nullptr; }
  std::fseek(f, 0, SEEK_END);
  long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> buf(sz > 0 ? sz : 0);
  if (sz > 0 && std::fread(buf.data(), 1, sz, f) != (size_t)sz) { std::fclose(f); *err = -2; return nullptr; }
  std::fclose(f);
  if (sz < 48) { *err = -3; return nullptr; }
  uint64_t magic;
  std::memcpy(&magic, buf.data() + sz - 8, 8);
  if (magic != kTableMagic) { *err = -4; return nullptr; }
  const uint8_t* p = buf.data() + sz - 48;
  const uint8_t* e = buf.data() + sz - 8;
  uint64_t moff, msize, ioff, isize;
  if (!get_varint(p, e, moff) || !get_varint(p, e, msize) || !get_varint(p, e, ioff) ||
      !get_varint(p, e, isize)) { *err = -5; return nullptr; }
  if (ioff + isize + 5 > (uint64_t)sz) { *err = -6; return nullptr; }
  std::vector<std::pair<std::string, std::string>> idx;
  if (!parse_block(buf.data() + ioff, isize, idx)) { *err = -7; return nullptr; }
  auto* t = new Table();
  for (auto& kv : idx) {
    const uint8_t* hp = (const uint8_t*)kv.second.data();
    const uint8_t* he = hp + kv.second.size();
    uint64_t boff, bsize;
    if (!get_varint(hp, he, boff) || !get_varint(hp, he, bsize) ||
        boff + bsize + 5 > (uint64_t)sz) { delete t; *err = -8; return nullptr; }
    uint32_t stored;
    std::memcpy(&stored, buf.data() + boff + bsize + 1, 4);
    uint32_t crc = crc_extend(0, buf.data() + boff, bsize + 1);
    if (mask_crc(crc) != stored) { delete t; *err = -9; return nullptr; }
    if (buf[boff + bsize] != 0) { delete t; *err = -10; return nullptr; }  // compressed block
    if (!parse_block(buf.data() + boff, bsize, t->kv)) { delete t; *err = -11; return nullptr; }
  }
  return t;
}

API int kfbrt_table_size(void* h) { return (int)static_cast<Table*>(h)->kv.size(); }

API void kfbrt_table_entry(void* h, int i, const char** key, size_t* klen, const char** val,
                           size_t* vlen) {
  auto& kv = static_cast<Table*>(h)->kv[i];
  *key = kv.first.data();
  *klen = kv.first.size();
  *val = kv.second.data();
  *vlen = kv.second.size();
}

API void kfbrt_table_free(void* h) { delete static_cast<Table*>(h); }

// ------------------------------------------------------- tf.train.Example
// Decodes Example{features{feature map<string, Feature>}} into a flat
// description written to `out` (caller-allocated, cap bytes):
//   for each feature: [u32 keylen][key][u8 kind 1=bytes 2=float 3=int64][u32 count]
//   then count values: bytes -> [u32 len][data]; float -> f32; int64 -> i64.
// Returns bytes written, or -1 on malformed input, -2 if cap is too small.
namespace {
struct Out {
  uint8_t* p;
  size_t cap, n = 0;
  bool ok = true;
  void put(const void* d, size_t k) {
    if (n + k > cap) { ok = false; return; }
    std::memcpy(p + n, d, k);
    n += k;
  }
  void u32(uint32_t v) { put(&v, 4); }
};

bool skip_field(const uint8_t*& p, const uint8_t* e, uint32_t wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, e, v);
    case 1: if (e - p < 8) return false; p += 8; return true;
    case 2: if (!get_varint(p, e, v) || (uint64_t)(e - p) < v) return false; p += v; return true;
    case 5: if (e - p < 4) return false; p += 4; return true;
    default: return false;
  }
}

bool decode_feature(const uint8_t* p, const uint8_t* e, Out& o) {
  // Feature: oneof bytes_list=1 / float_list=2 / int64_list=3
  while (p < e) {
    uint64_t tag;
    if (!get_varint(p, e, tag)) return false;
    const uint32_t field = tag >> 3, wt = tag & 7;
    if (wt != 2 || field < 1 || field > 3) {
      if (!skip_field(p, e, wt)) return false;
      continue;
    }
    uint64_t len;
    if (!get_varint(p, e, len) || (uint64_t)(e - p) < len) return false;
    const uint8_t* lp = p;
    const uint8_t* le = p + len;
    p = le;
    uint8_t kind = (uint8_t)field;
    // First pass: count values.
    uint32_t count = 0;
    std::vector<std::pair<const uint8_t*, size_t>> bytes_vals;
    std::vector<float> fvals;
    std::vector<int64_t> ivals;
    const uint8_t* q = lp;
    while (q < le) {
      uint64_t t2;
      if (!get_varint(q, le, t2)) return false;
      const uint32_t wt2 = t2 & 7;
      if ((t2 >> 3) != 1) { if (!skip_field(q, le, wt2)) return false; continue; }
      if (kind == 1) {
        uint64_t bl;
        if (wt2 != 2 || !get_varint(q, le, bl) || (uint64_t)(le - q) < bl) return false;
        bytes_vals.emplace_back(q, bl);
        q += bl;
      } else if (kind == 2) {
        if (wt2 == 2) {  // packed
          uint64_t bl;
          if (!get_varint(q, le, bl) || (uint64_t)(le - q) < bl || bl % 4) return false;
          for (uint64_t k = 0; k < bl; k += 4) { float f; std::memcpy(&f, q + k, 4); fvals.push_back(f); }
          q += bl;
        } else if (wt2 == 5) {
          if (le - q < 4) return false;
          float f; std::memcpy(&f, q, 4); fvals.push_back(f); q += 4;
        } else return false;
      } else {
        if (wt2 == 2) {
          uint64_t bl;
          if (!get_varint(q, le, bl) || (uint64_t)(le - q) < bl) return false;
          const uint8_t* pe = q + bl;
          while (q < pe) { uint64_t v; if (!get_varint(q, pe, v)) return false; ivals.push_back((int64_t)v); }
        } else if (wt2 == 0) {
          uint64_t v; if (!get_varint(q, le, v)) return false; ivals.push_back((int64_t)v);
        } else return false;
      }
    }
    count = kind == 1 ? bytes_vals.size() : kind == 2 ? fvals.size() : ivals.size();
    o.put(&kind, 1);
    o.u32(count);
    if (kind == 1) {
      for (auto& bv : bytes_vals) { o.u32((uint32_t)bv.second); o.put(bv.first, bv.second); }
    } else if (kind == 2) {
      o.put(fvals.data(), fvals.size() * 4);
    } else {
      o.put(ivals.data(), ivals.size() * 8);
    }
    return true;
  }
  uint8_t none = 0;
  uint32_t zero = 0;
  o.put(&none, 1);
  o.u32(zero);
  return true;
}
}  // namespace

API long kfbrt_parse_example(const uint8_t* data, size_t n, uint8_t* out, size_t cap) {
  Out o{out, cap};
  const uint8_t* p = data;
  const uint8_t* e = data + n;
  while (p < e) {
    uint64_t tag;
    if (!get_varint(p, e, tag)) return -1;
    if ((tag >> 3) != 1 || (tag & 7) != 2) {  // Example.features = 1
      if (!skip_field(p, e, tag & 7)) return -1;
      continue;
    }
    uint64_t flen;
    if (!get_varint(p, e, flen) || (uint64_t)(e - p) < flen) return -1;
    const uint8_t* fp = p;
    const uint8_t* fe = p + flen;
    p = fe;
    while (fp < fe) {  // Features.feature = 1 (map entry)
      uint64_t t;
      if (!get_varint(fp, fe, t)) return -1;
      if ((t >> 3) != 1 || (t & 7) != 2) { if (!skip_field(fp, fe, t & 7)) return -1; continue; }
      uint64_t elen;
      if (!get_varint(fp, fe, elen) || (uint64_t)(fe - fp) < elen) return -1;
      const uint8_t* ep = fp;
      const uint8_t* ee = fp + elen;
      fp = ee;
      const uint8_t* key = nullptr;
      uint64_t klen = 0;
      const uint8_t* val = nullptr;
      uint64_t vlen = 0;
      while (ep < ee) {
        uint64_t t2;
        if (!get_varint(ep, ee, t2)) return -1;
        if ((t2 & 7) != 2) { if (!skip_field(ep, ee, t2 & 7)) return -1; continue; }
        uint64_t l;
        if (!get_varint(ep, ee, l) || (uint64_t)(ee - ep) < l) return -1;
        if ((t2 >> 3) == 1) { key = ep; klen = l; }
        else if ((t2 >> 3) == 2) { val = ep; vlen = l; }
        ep += l;
      }
      if (!key) continue;
      o.u32((uint32_t)klen);
      o.put(key, klen);
      if (!decode_feature(val ? val : ep, val ? val + vlen : ep, o)) return -1;
    }
  }
  if (!o.ok) return -2;
  return (long)o.n;
}

// ------------------------------------------------------------------ images
// Saturation scale + hue shift of a float RGB image in place (the host
// colour distortion of tcb/preprocessing.py:268-307, tf.image.adjust_saturation
// / adjust_hue): one RGB -> HSV -> RGB pass per pixel, s <- clip(s * sat, 0, 1),
// h <- (h + hue) mod 1.  Called through ctypes, which releases the GIL, so
// the input pipeline's worker threads run it in parallel.
API void kfbrt_adjust_sat_hue(float* img, long npix, float sat, float hue) {
  for (long i = 0; i < npix; ++i) {
    float* px = img + 3 * i;
    const float r = px[0], g = px[1], b = px[2];
    const float mx = std::max(r, std::max(g, b));
    const float mn = std::min(r, std::min(g, b));
    const float d = mx - mn;
    const float v = mx;
    float s = mx > 0.f ? d / std::max(mx, 1e-12f) : 0.f;
    float h = 0.f;
    if (d > 0.f) {
      const float dd = std::max(d, 1e-12f);
      if (mx == r) h = (g - b) / dd;
      else if (mx == g) h = 2.f + (b - r) / dd;
      else h = 4.f + (r - g) / dd;
      h = h / 6.f;
      h -= std::floor(h);
    }
    s = std::min(std::max(s * sat, 0.f), 1.f);
    h += hue;
    h -= std::floor(h);
    const float h6 = h * 6.f;
    const float fl = std::floor(h6);
    const int sector = ((int)fl % 6 + 6) % 6;
    const float f = h6 - fl;
    const float p = v * (1.f - s), q = v * (1.f - s * f), t = v * (1.f - s * (1.f - f));
    float ro, go, bo;
    switch (sector) {
      case 0: ro = v; go = t; bo = p; break;
      case 1: ro = q; go = v; bo = p; break;
      case 2: ro = p; go = v; bo = t; break;
      case 3: ro = p; go = q; bo = v; break;
      case 4: ro = t; go = p; bo = v; break;
      default: ro = v; go = p; bo = q; break;
    }
    px[0] = ro; px[1] = go; px[2] = bo;
  }
}
