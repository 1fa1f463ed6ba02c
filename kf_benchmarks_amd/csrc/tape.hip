// Launch tape: the native step executor.
//
// The reference runs a training step as ONE call into TF's C++ executor
// (sess.run, tcb/benchmark_cnn.py:821).  Here a step is ~450 kernel launches
// whose host-side preparation (autograd, shape logic, epilogue wiring,
// autotune lookups) costs ~20 us each in Python - a ~10 ms/step host floor.
// A tape removes that floor without HIP graphs (whose replay executes the
// nodes of a two-stream step one after another on this stack: 27.9 vs 19.8
// ms/step for ResNet-50 bs256, profiles/r6_graph_env_probe.txt):
//
//   record  one eager step runs normally while every native entry point it
//           calls (kernels, memsets, cross-stream waits) is appended to the
//           tape with its raw arguments (device pointers, shapes, streams);
//   replay  kfb_tape_replay re-issues the recorded calls in order from C++,
//           patching the few per-step scalars (learning rate, RNG seeds)
//           first.  Each call is the same KFB_API function the eager path
//           calls, so kernels, launch shapes and stream assignment (compute
//           stream + weight-gradient side stream, joined by events) are
//           identical and the two streams stay concurrent.
//
// Memory: the recording step allocates from a private pool that nothing
// else allocates from afterwards (ops/tape.py), so every recorded address
// stays valid and owned by the tape.
//
// Calls are made through libffi (the library ctypes itself uses, loaded at
// run time): argument type codes come from the Python-side signature table.
#include "common.h"
#include <hip/hip_ext.h>

#include <dlfcn.h>

#include <chrono>

#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace kfb {
std::atomic<int> g_raw_rec{0};

namespace tape {

// ---- minimal libffi ABI (libffi >= 3.3, x86-64 SysV) -----------------------
struct ffi_type_t {
  size_t size;
  unsigned short alignment;
  unsigned short type;
  ffi_type_t** elements;
};
constexpr int FFI_UNIX64 = 2;
// ffi_cif is { abi, nargs, arg_types, rtype, bytes, flags } on x86-64; the
// buffer is over-sized so a longer layout cannot overflow it.
struct alignas(16) Cif {
  unsigned char raw[128];
};
typedef int (*prep_cif_fn)(void*, int, unsigned, ffi_type_t*, ffi_type_t**);
typedef void (*call_fn)(void*, void (*)(void), void*, void**);

struct Ffi {
  bool ok = false;
  prep_cif_fn prep = nullptr;
  call_fn call = nullptr;
  ffi_type_t *t_sint32 = nullptr, *t_uint32 = nullptr, *t_sint64 = nullptr, *t_ptr = nullptr,
             *t_float = nullptr, *t_uint64 = nullptr;
};

static Ffi& ffi() {
  static Ffi f;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("libffi.so.8", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libffi.so.7", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libffi.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    f.prep = (prep_cif_fn)dlsym(h, "ffi_prep_cif");
    f.call = (call_fn)dlsym(h, "ffi_call");
    f.t_sint32 = (ffi_type_t*)dlsym(h, "ffi_type_sint32");
    f.t_uint32 = (ffi_type_t*)dlsym(h, "ffi_type_uint32");
    f.t_sint64 = (ffi_type_t*)dlsym(h, "ffi_type_sint64");
    f.t_uint64 = (ffi_type_t*)dlsym(h, "ffi_type_uint64");
    f.t_ptr = (ffi_type_t*)dlsym(h, "ffi_type_pointer");
    f.t_float = (ffi_type_t*)dlsym(h, "ffi_type_float");
    f.ok = f.prep && f.call && f.t_sint32 && f.t_uint32 && f.t_sint64 && f.t_uint64 && f.t_ptr &&
           f.t_float;
  });
  return f;
}

// One signature (type string -> prepared call interface), shared by every op
// with that signature.  Type codes: i int32, u uint32, l int64, q uint64 /
// size_t, p pointer, f float.
struct Sig {
  Cif cif;
  std::vector<ffi_type_t*> types;
};

// What an entry point did on the device while it was recorded, for the raw
// replay: kernel launches (function, shape, stream, argument bytes), memsets,
// cross-stream waits and device copies.
struct Raw {
  int kind = 0;  // 0 launch, 1 memset, 2 stream wait, 3 device-to-device copy
  const void* fn = nullptr;
  dim3 grid, block;
  unsigned shm = 0;
  hipStream_t s = nullptr, s2 = nullptr;
  hipEvent_t ev = nullptr;
  std::vector<uint64_t> blob;  // the kernel's argument bytes
  std::vector<void*> argv;     // hipLaunchKernel's table into blob
  void* p = nullptr;
  const void* q = nullptr;
  int value = 0;
  size_t bytes = 0;
  // replay plan (plan_binds): a launch that carries the completion event of
  // the cross-stream wait right after it on its stream, and that wait, which
  // then only enqueues the wait (no event-record marker on the source stream)
  hipEvent_t bind_ev = nullptr;
  bool bound = false;
};

struct Op {
  void (*fn)(void);
  const Sig* sig;
  std::vector<uint64_t> slots;  // one 64-bit slot per argument (value in the low bytes)
  std::vector<void*> argp;      // ffi avalue: &slots[k]
  // raw replay: the recorded device work stands in for the entry point
  // when nothing else happened in it (raw_ok) and no argument is patched
  std::vector<Raw> raw;
  bool tainted = false, patched = false, raw_ok = false;
};

struct Tape {
  std::vector<Op> ops;
  // KFB_TAPE_PROFILE: accumulated host seconds per op over all replays
  std::vector<double> host_s;
  std::unordered_map<std::string, Sig*> sigs;
  ~Tape() {
    for (auto& kv : sigs) delete kv.second;
  }
};

static ffi_type_t* type_of(char c) {
  Ffi& f = ffi();
  switch (c) {
    case 'i': return f.t_sint32;
    case 'u': return f.t_uint32;
    case 'l': return f.t_sint64;
    case 'q': return f.t_uint64;
    case 'p': return f.t_ptr;
    case 'f': return f.t_float;
    default: return nullptr;
  }
}

static const Sig* get_sig(Tape* t, const char* types) {
  auto it = t->sigs.find(types);
  if (it != t->sigs.end()) return it->second;
  Sig* s = new Sig();
  const int n = (int)strlen(types);
  for (int k = 0; k < n; ++k) {
    ffi_type_t* ty = type_of(types[k]);
    if (!ty) {
      delete s;
      return nullptr;
    }
    s->types.push_back(ty);
  }
  memset(&s->cif, 0, sizeof(s->cif));
  if (ffi().prep(&s->cif, FFI_UNIX64, (unsigned)n, ffi().t_sint32, s->types.data()) != 0) {
    delete s;
    return nullptr;
  }
  t->sigs.emplace(types, s);
  return s;
}

// argv points into blob: element moves must keep the buffers where they are
static_assert(std::is_nothrow_move_constructible<Raw>::value, "Raw moves must not copy");
static_assert(std::is_nothrow_move_constructible<Op>::value, "Op moves must not copy");

// the op being recorded (one at a time, by the thread that added it).
// thread_local: another thread launching while an op records (the input
// producer's JPEG / augment kernels) sees no tape and never touches the
// recording thread's ops vector
static thread_local Tape* g_rt = nullptr;
static thread_local int g_rop = -1;

static Op* cur_op() {
  if (!g_rt || g_rop < 0 || g_rop >= (int)g_rt->ops.size()) return nullptr;
  return &g_rt->ops[g_rop];
}

static hipError_t replay_raw(const Raw& r) {
  switch (r.kind) {
    case 0:
      if (r.bind_ev)
        return hipExtLaunchKernel(r.fn, r.grid, r.block, const_cast<void**>(r.argv.data()), r.shm,
                                  r.s, nullptr, r.bind_ev, 0);
      return hipLaunchKernel(r.fn, r.grid, r.block, const_cast<void**>(r.argv.data()), r.shm,
                             r.s);
    case 1: return hipMemsetAsync(r.p, r.value, r.bytes, r.s);
    case 2: {
      const hipError_t e = r.bound ? hipSuccess : hipEventRecord(r.ev, r.s2);
      return e != hipSuccess ? e : hipStreamWaitEvent(r.s, r.ev, 0);
    }
    default: return hipMemcpyAsync(r.p, r.q, r.bytes, hipMemcpyDeviceToDevice, r.s);
  }
}

static const bool g_bind = true;  // (off: every wait replayed as record + wait)

// A cross-stream wait recorded right after a kernel launch on its source
// stream (nothing else issued on that stream in between) is replayed by
// launching that kernel with the wait's event as its completion event
// (hipExtLaunchKernel stopEvent) and enqueueing only the wait: the source
// stream then carries no separate event-record marker, which costs the
// producing stream ~2-3 us per wait (scripts/probes/evgap.hip).  Same
// ordering: the source stream is in order, so the kernel's completion is
// the completion of everything enqueued on it before the wait.  Anything
// else issued on a stream (memset, copy, its own wait, an op replayed
// through its entry point) ends the candidate launch for that stream.
static void plan_binds(Tape* t, bool raw_replay) {
  struct Last {
    hipStream_t s;
    Raw* r;
  };
  std::vector<Last> last;
  auto find = [&](hipStream_t s) -> Raw** {
    for (Last& l : last)
      if (l.s == s) return &l.r;
    return nullptr;
  };
  auto set = [&](hipStream_t s, Raw* r) {
    if (Raw** p = find(s)) *p = r;
    else last.push_back({s, r});
  };
  for (Op& op : t->ops) {
    const bool raw = raw_replay && op.raw_ok && !op.patched;
    for (Raw& r : op.raw) {
      r.bind_ev = nullptr;
      r.bound = false;
    }
    if (!raw) {
      last.clear();  // the entry point may issue anything on any stream
      continue;
    }
    for (Raw& r : op.raw) {
      if (r.kind == 0) {
        set(r.s, &r);
      } else if (r.kind == 2) {
        Raw** p = find(r.s2);
        if (g_bind && p && *p && !(*p)->bind_ev && r.s2 != r.s) {
          (*p)->bind_ev = r.ev;
          r.bound = true;
        }
        if (p) *p = nullptr;  // (one wait per bound launch)
        set(r.s, nullptr);    // a later wait on r.s must also cover this wait
      } else {
        set(r.s, nullptr);
      }
    }
  }
}

}  // namespace tape

void raw_record_launch(const void* fn, dim3 grid, dim3 block, unsigned shm, hipStream_t s,
                       void* const* argv, const size_t* sizes, int n) {
  tape::Op* op = tape::cur_op();
  if (!op) return;
  tape::Raw r;
  r.kind = 0;
  r.fn = fn;
  r.grid = grid;
  r.block = block;
  r.shm = shm;
  r.s = s;
  std::vector<size_t> off(n);
  size_t total = 0;
  for (int i = 0; i < n; ++i) {
    total = (total + 7) & ~(size_t)7;  // (every argument 8-byte aligned in the copy)
    const size_t al = sizes[i] >= 16 ? 16 : 8;
    total = (total + al - 1) & ~(al - 1);
    off[i] = total;
    total += sizes[i];
  }
  r.blob.assign((total + 15) / 8 + 2, 0);
  char* base = (char*)r.blob.data();
  base = (char*)(((uintptr_t)base + 15) & ~(uintptr_t)15);
  r.argv.resize(n);
  for (int i = 0; i < n; ++i) {
    memcpy(base + off[i], argv[i], sizes[i]);
    r.argv[i] = base + off[i];
  }
  op->raw.push_back(std::move(r));  // (vector moves keep blob's storage in place)
}

void raw_record_memset(void* p, int value, size_t bytes, hipStream_t s) {
  tape::Op* op = tape::cur_op();
  if (!op) return;
  tape::Raw r;
  r.kind = 1;
  r.p = p;
  r.value = value;
  r.bytes = bytes;
  r.s = s;
  op->raw.push_back(std::move(r));
}

void raw_taint() {
  tape::Op* op = tape::cur_op();
  if (op) op->tainted = true;
}

}  // namespace kfb

using namespace kfb::tape;

// KFB_TAPE_RAW=0 (or kfb_tape_set_raw(0)): every op replays through its
// entry point instead of its recorded raw launches
static int g_raw_replay = [] {
  const char* e = getenv("KFB_TAPE_RAW");
  return (e && atoi(e) == 0) ? 0 : 1;
}();

KFB_API void kfb_tape_set_raw(int on) { g_raw_replay = on ? 1 : 0; }

KFB_API int kfb_tape_available() { return ffi().ok ? 1 : 0; }

KFB_API void* kfb_tape_new() {
  if (!ffi().ok) return nullptr;
  return new Tape();
}

KFB_API void kfb_tape_free(void* h) { delete (Tape*)h; }

KFB_API int kfb_tape_size(void* h) { return h ? (int)((Tape*)h)->ops.size() : 0; }

// Host seconds spent in each op over all replays so far (KFB_TAPE_PROFILE
// set; zeros otherwise); out has kfb_tape_size entries.
KFB_API int kfb_tape_host_times(void* h, double* out) {
  Tape* t = (Tape*)h;
  if (!t) return -1;
  for (size_t i = 0; i < t->ops.size(); ++i) out[i] = i < t->host_s.size() ? t->host_s[i] : 0.0;
  return 0;
}

// Appends fn(args...) with ``types`` (one code per argument) and the raw
// 64-bit argument slots; returns the op index or -1.
KFB_API int kfb_tape_add(void* h, void* fn, const char* types, const uint64_t* slots, int n) {
  Tape* t = (Tape*)h;
  if (!t || !fn || (int)strlen(types) != n) return -1;
  const Sig* s = get_sig(t, types);
  if (!s) return -1;
  t->ops.emplace_back();
  Op& op = t->ops.back();
  op.fn = (void (*)(void))fn;
  op.sig = s;
  op.slots.assign(slots, slots + n);
  return (int)t->ops.size() - 1;
}

// Overwrites argument ``arg`` of op ``op`` (a per-step scalar).
KFB_API int kfb_tape_patch(void* h, int op, int arg, uint64_t value) {
  Tape* t = (Tape*)h;
  if (!t || op < 0 || op >= (int)t->ops.size() || arg < 0 ||
      arg >= (int)t->ops[op].slots.size())
    return -1;
  t->ops[op].slots[arg] = value;
  t->ops[op].patched = true;  // (a per-step argument: always the entry point)
  return 0;
}

// Brackets the eager execution of a just-added op while recording: its kernel
// launches, memsets, waits and copies are captured (Raw); allow_raw = 0 keeps
// the op on the entry-point call at replay (an entry with host-side effects).
KFB_API int kfb_tape_begin_op(void* h, int op) {
  Tape* t = (Tape*)h;
  if (!t || op < 0 || op >= (int)t->ops.size()) return -1;
  g_rt = t;
  g_rop = op;
  kfb::g_raw_rec.store(1);
  return 0;
}

KFB_API int kfb_tape_end_op(void* h, int op, int allow_raw) {
  Tape* t = (Tape*)h;
  kfb::g_raw_rec.store(0);
  g_rt = nullptr;
  g_rop = -1;
  if (!t || op < 0 || op >= (int)t->ops.size()) return -1;
  Op& o = t->ops[op];
  o.raw_ok = allow_raw && !o.tainted && !o.raw.empty();
  return o.raw_ok ? 1 : 0;
}

// Device operations (launches, memsets, waits, copies) the raw ops re-issue per replay.
KFB_API long kfb_tape_raw_launches(void* h) {
  Tape* t = (Tape*)h;
  if (!t) return -1;
  long n = 0;
  for (const Op& o : t->ops)
    if (o.raw_ok && !o.patched) n += (long)o.raw.size();
  return n;
}

// Number of ops a replay re-issues raw (the rest call their entry point).
KFB_API int kfb_tape_raw_ops(void* h) {
  Tape* t = (Tape*)h;
  if (!t) return -1;
  int n = 0;
  for (const Op& o : t->ops) n += o.raw_ok && !o.patched;
  return n;
}

// Re-issues every recorded call in order: patches first (npatch triples
// op/arg/value), then the calls.  Returns 0, or the first non-zero return
// code; *failed_op receives its index.
KFB_API int kfb_tape_replay(void* h, const int* pop, const int* parg, const uint64_t* pval,
                            int npatch, int* failed_op) {
  Tape* t = (Tape*)h;
  if (!t) return -1;
  for (int k = 0; k < npatch; ++k)
    if (kfb_tape_patch(h, pop[k], parg[k], pval[k]) != 0) return -2;
  plan_binds(t, g_raw_replay != 0);
  call_fn call = ffi().call;
  static const bool prof = getenv("KFB_TAPE_PROFILE") != nullptr;
  if (prof && t->host_s.size() != t->ops.size()) t->host_s.assign(t->ops.size(), 0.0);
  for (size_t i = 0; i < t->ops.size(); ++i) {
    Op& op = t->ops[i];
    if (op.argp.size() != op.slots.size()) {
      op.argp.resize(op.slots.size());
      for (size_t k = 0; k < op.slots.size(); ++k) op.argp[k] = &op.slots[k];
    }
    int64_t rc = 0;  // ffi widens an int return to a full register
    const auto t0 = prof ? std::chrono::steady_clock::now()
                         : std::chrono::steady_clock::time_point();
    if (op.raw_ok && !op.patched && g_raw_replay) {
      for (const Raw& r : op.raw) {
        const hipError_t e = replay_raw(r);
        if (e != hipSuccess) {
          rc = (int64_t)e;
          break;
        }
      }
    } else {
      call((void*)&op.sig->cif, op.fn, &rc, op.argp.data());
    }
    if (prof)
      t->host_s[i] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if ((int)rc != 0) {
      if (failed_op) *failed_op = (int)i;
      return (int)rc;
    }
  }
  return 0;
}

// ---- recordable stream-ordering and memory primitives ----------------------
// (the eager path uses them too, so a recorded step orders its streams with
// exactly the calls the tape replays)

KFB_API hipError_t kfb_event_create(hipEvent_t* ev) {
  return hipEventCreateWithFlags(ev, hipEventDisableTiming);
}

// device_only: the event orders work of two streams of one device and no
// host or other device inspects it, so its record skips the system-scope
// release fence (hipEventDisableSystemFence: ~1.8 us less per wait on the
// producing stream, scripts/probes/evgap.hip)
KFB_API hipError_t kfb_event_create_device(hipEvent_t* ev) {
  return hipEventCreateWithFlags(ev, hipEventDisableTiming | hipEventDisableSystemFence);
}

KFB_API hipError_t kfb_event_destroy(hipEvent_t ev) { return hipEventDestroy(ev); }

// ---- interval timer: pairs of timing events in a ring ----------------------
// The exposed-communication probe (parallel/bucket.py): mark 0 when the
// backward's kernels are done, mark 1 when the compute stream may use the
// reduced gradients.  Both marks are entry-point calls (the kfb_event_ prefix
// keeps a replayed tape on the entry point), so every replayed step records
// into the next slot and the host reads the intervals after the fact.
struct EventTimer {
  std::vector<hipEvent_t> a, b;
  long w = 0;  // next slot to fill (mark 1 advances it)
  long r = 0;  // first slot not yet read
};

KFB_API hipError_t kfb_event_timer_new(int slots, void** out) {
  if (slots <= 0 || !out) return hipErrorInvalidValue;
  EventTimer* t = new EventTimer;
  t->a.resize(slots);
  t->b.resize(slots);
  for (int i = 0; i < slots; ++i) {
    hipError_t e = hipEventCreate(&t->a[i]);
    if (e == hipSuccess) e = hipEventCreate(&t->b[i]);
    if (e != hipSuccess) return e;
  }
  *out = t;
  return hipSuccess;
}

KFB_API hipError_t kfb_event_timer_mark(void* h, int which, hipStream_t s) {
  EventTimer* t = (EventTimer*)h;
  if (!t || (which != 0 && which != 1)) return hipErrorInvalidValue;
  const size_t k = (size_t)(t->w % (long)t->a.size());
  const hipError_t e = hipEventRecord(which == 0 ? t->a[k] : t->b[k], s);
  if (which == 1) t->w += 1;
  return e;
}

// Waits for the intervals recorded since the last read and writes their
// lengths (ms) to out (at most max, the newest ones); returns how many.
KFB_API int kfb_event_timer_read(void* h, float* out, int max) {
  EventTimer* t = (EventTimer*)h;
  if (!t || !out || max <= 0) return -1;
  const long n = (long)t->a.size();
  long r = t->r;
  if (t->w - r > n) r = t->w - n;  // overwritten: keep the newest n
  if (t->w - r > max) r = t->w - max;
  int got = 0;
  for (; r < t->w; ++r) {
    const size_t k = (size_t)(r % n);
    if (hipEventSynchronize(t->b[k]) != hipSuccess) return -1;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t->a[k], t->b[k]) != hipSuccess) ms = 0.f;
    out[got++] = ms > 0.f ? ms : 0.f;
  }
  t->r = t->w;
  return got;
}

KFB_API int kfb_event_timer_free(void* h) {
  EventTimer* t = (EventTimer*)h;
  if (!t) return 0;
  for (size_t i = 0; i < t->a.size(); ++i) {
    hipEventDestroy(t->a[i]);
    hipEventDestroy(t->b[i]);
  }
  delete t;
  return 0;
}

// dst waits for everything enqueued on src so far (ev: scratch event).
KFB_API hipError_t kfb_stream_wait(hipStream_t dst, hipStream_t src, hipEvent_t ev) {
  if (Op* op = cur_op()) {
    Raw r;
    r.kind = 2;
    r.s = dst;
    r.s2 = src;
    r.ev = ev;
    op->raw.push_back(std::move(r));
  }
  hipError_t e = hipEventRecord(ev, src);
  if (e != hipSuccess) return e;
  return hipStreamWaitEvent(dst, ev, 0);
}

KFB_API hipError_t kfb_memset(void* p, int byte, size_t bytes, hipStream_t s) {
  return kfb::memset_async(p, byte, bytes, s);
}

KFB_API hipError_t kfb_memcpy_d2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (Op* op = cur_op()) {
    Raw r;
    r.kind = 3;
    r.p = dst;
    r.q = src;
    r.bytes = bytes;
    r.s = s;
    op->raw.push_back(std::move(r));
  }
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
}

// ---- host-side self test (no GPU): records calls of a probe function with
// every argument type and replays them with a patch
static uint64_t g_probe_sum = 0;
KFB_API int kfb_tape_probe(int a, float b, long c, void* d, unsigned e, int f, float g, long h,
                           int i, int j, float k) {
  g_probe_sum += (uint64_t)(a + (long)(b * 4) + c + (long)(uintptr_t)d + e + f + (long)(g * 4) +
                            h + i + j + (long)(k * 4));
  return a == -7 ? 5 : 0;  // a == -7: report an error
}
KFB_API uint64_t kfb_tape_probe_sum() { return g_probe_sum; }
