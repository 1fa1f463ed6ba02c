// Fused optimizer steps over ONE flat fp32 parameter buffer.
//
// All trainable variables of a model live as views into a single contiguous
// fp32 buffer (and their gradients in a matching flat buffer), so each
// optimizer step is a single streaming launch over ~25.6M (ResNet-50) or
// ~138M (VGG-16) elements instead of one launch per variable.  The same pass
// folds in what the reference does as separate graph ops:
//   * loss-scale unscale            (tcb/benchmark_cnn.py:3110-3120)
//   * L2 weight decay gradient      (tcb/benchmark_cnn.py:3070-3099, grad += wd*w)
//   * gradient clip_by_value        (tcb/benchmark_cnn.py:2787-2794)
//   * the update rule of tf.train.{GradientDescent,Momentum(nesterov),RMSProp,Adam}
//     Optimizer (tcb/benchmark_cnn.py:1172-1190)
//   * the low-precision (bf16/fp16) shadow copy of the weights the kernels read.
// A per-element decay mask (1 byte, optional) excludes variables from L2.
//
// Model averaging (KungFu PairAveraging / SMA, tcb/benchmark_cnn.py:1196-1201)
// is folded into the same pass: with ``mix`` set, w <- mix_a * w + mix_b * mix
// before the update (PairAveraging: (w + w_peer) / 2; SMA: w - alpha (w - avg)),
// gated by a device flag ``mix_ok`` (the peer snapshot's seqlock check, see
// seqlock_check_k); ``wout`` receives a copy of the updated weights (the
// PairAveraging publish slot, the SMA all-reduce buffer), so neither strategy
// runs extra elementwise passes over the model.
#include "common.h"

#include <cstring>

namespace kfb {

enum OptKind : int { SGD = 0, MOMENTUM = 1, RMSPROP = 2, ADAM = 3 };

struct OptArgs {
  float lr;
  float grad_scale;   // multiply raw grads (1/loss_scale, 1/num_replicas, ...)
  float weight_decay; // coefficient on w added to the gradient
  float clip;         // <= 0: no clipping
  float mom;          // momentum / rmsprop momentum
  float b1, b2, eps;  // rmsprop decay in b1; adam betas
  float lr_t;         // adam bias-corrected step size
  int nesterov;
  const float* mix;   // model to average in before the update (nullable)
  float mix_a, mix_b; // w <- mix_a * w + mix_b * mix
  const int* mix_ok;  // nullable; *mix_ok == 0 skips the averaging
  float* wout;        // nullable; receives the updated weights
};

template <int KIND, typename LP>
__global__ void __launch_bounds__(256)
opt_step_k(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ s1,
           float* __restrict__ s2, LP* __restrict__ wlp, const uint8_t* __restrict__ decay_mask,
           long n4, OptArgs a) {
  const bool mix = a.mix && (!a.mix_ok || *a.mix_ok);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    // the L2 term is part of the gradient of the loss the step's forward
    // computed, so it uses those weights, not the averaged ones (KungFu's
    // averaging optimizers assign the average, then apply the gradients)
    const float w0[4] = {wv.x, wv.y, wv.z, wv.w};
    if (mix) {
      const float4 pv = reinterpret_cast<const float4*>(a.mix)[i];
      wv = make_float4(a.mix_a * wv.x + a.mix_b * pv.x, a.mix_a * wv.y + a.mix_b * pv.y,
                       a.mix_a * wv.z + a.mix_b * pv.z, a.mix_a * wv.w + a.mix_b * pv.w);
    }
    float ww[4] = {wv.x, wv.y, wv.z, wv.w};
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float m1[4], m2[4];
    if (KIND != SGD) {
      float4 t = reinterpret_cast<float4*>(s1)[i];
      m1[0] = t.x; m1[1] = t.y; m1[2] = t.z; m1[3] = t.w;
    }
    if (KIND == RMSPROP || KIND == ADAM) {
      float4 t = reinterpret_cast<float4*>(s2)[i];
      m2[0] = t.x; m2[1] = t.y; m2[2] = t.z; m2[3] = t.w;
    }
    uint32_t dm = 0xffffffffu;
    if (decay_mask) dm = reinterpret_cast<const uint32_t*>(decay_mask)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gg[k] * a.grad_scale;
      if ((dm >> (8 * k)) & 0xffu) gk += a.weight_decay * w0[k];
      if (a.clip > 0.f) gk = fminf(fmaxf(gk, -a.clip), a.clip);
      if (KIND == SGD) {
        ww[k] -= a.lr * gk;
      } else if (KIND == MOMENTUM) {
        // tf ApplyMomentum: accum = accum*mu + g; nesterov: var -= lr*(g + mu*accum)
        const float acc = m1[k] * a.mom + gk;
        m1[k] = acc;
        ww[k] -= a.nesterov ? a.lr * (gk + a.mom * acc) : a.lr * acc;
      } else if (KIND == RMSPROP) {
        // tf ApplyRMSProp: ms = ms + (g^2 - ms)(1-decay); mom = mom*mu + lr*g/sqrt(ms+eps)
        const float ms = m2[k] + (gk * gk - m2[k]) * (1.f - a.b1);
        m2[k] = ms;
        const float mo = m1[k] * a.mom + a.lr * gk * rsqrtf(ms + a.eps);
        m1[k] = mo;
        ww[k] -= mo;
      } else {  // ADAM
        const float m = m1[k] + (gk - m1[k]) * (1.f - a.b1);
        const float v = m2[k] + (gk * gk - m2[k]) * (1.f - a.b2);
        m1[k] = m;
        m2[k] = v;
        ww[k] -= a.lr_t * m / (sqrtf(v) + a.eps);
      }
    }
    reinterpret_cast<float4*>(w)[i] = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if (a.wout) reinterpret_cast<float4*>(a.wout)[i] = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if (KIND != SGD)
      reinterpret_cast<float4*>(s1)[i] = make_float4(m1[0], m1[1], m1[2], m1[3]);
    if (KIND == RMSPROP || KIND == ADAM)
      reinterpret_cast<float4*>(s2)[i] = make_float4(m2[0], m2[1], m2[2], m2[3]);
    if (wlp) {
      Vec<LP, 4> o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o.v[k] = (LP)ww[k];
      reinterpret_cast<Vec<LP, 4>*>(wlp)[i] = o;
    }
  }
}

// Seqlock validation of a peer-model snapshot, run on the pull stream right
// after the copy: the snapshot is good iff the peer's sequence word for the
// slot (host memory, mapped for the device) still holds the even value read
// before the copy - a rewrite overlapping the copy makes it odd first and
// leaves it at a larger value.  ok[0] = 1 / 0; torn[0] counts rejections.
__global__ void seqlock_check_k(const long long* seq, long long expect, int* ok, int* torn) {
  const long long v = __hip_atomic_load(seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int good = v == expect;
  ok[0] = good;
  if (!good) atomicAdd(torn, 1);
}

// Non-finite detector for dynamic loss scaling: flag[0] |= any(!isfinite(x)).
__global__ void __launch_bounds__(256)
nonfinite_k(const float* __restrict__ x, long n, int* __restrict__ flag) {
  int bad = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// Sum of squares of a flat buffer (L2 loss reporting): out[0] += sum(x^2)/2.
__global__ void __launch_bounds__(256)
half_sumsq_k(const float* __restrict__ x, long n, float* __restrict__ out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    s += x[i] * x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, 0.5f * s);
}

template <typename LP>
__global__ void __launch_bounds__(256)
cast_f32_k(const float* __restrict__ x, LP* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = (LP)x[i];
}

template <typename LP>
__global__ void __launch_bounds__(256)
cast_to_f32_k(const LP* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    y[i] = (float)x[i];
}

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 256L * 8) b = 256L * 8;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace kfb

using namespace kfb;

// n must be a multiple of 4 (the flat buffer is padded by the allocator).
// lp_dtype: element type of wlp (ignored when wlp is null).
KFB_API hipError_t kfb_opt_step(int kind, float* w, const float* g, float* s1, float* s2, void* wlp,
                                int lp_dtype, const uint8_t* decay_mask, long n, float lr,
                                float grad_scale, float weight_decay, float clip, float mom,
                                float b1, float b2, float eps, float lr_t, int nesterov,
                                const float* mix, float mix_a, float mix_b, const int* mix_ok,
                                float* wout, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  OptArgs a{lr, grad_scale, weight_decay, clip, mom, b1, b2, eps, lr_t, nesterov,
            mix, mix_a, mix_b, mix_ok, wout};
  const long n4 = n / 4;
  const int gb = grid_for(n4);
#define KFB_OPT(K, LP)                                                                      \
  hipLaunchKernelGGL((opt_step_k<K, LP>), dim3(gb), dim3(256), 0, stream, w, g, s1, s2,      \
                     (LP*)wlp, decay_mask, n4, a)
#define KFB_OPT_LP(K)                                  \
  if (!wlp || lp_dtype == F32) KFB_OPT(K, float);      \
  else if (lp_dtype == BF16) KFB_OPT(K, bf16);         \
  else KFB_OPT(K, f16);
  if (!wlp) wlp = nullptr;
  switch (kind) {
    case SGD: { KFB_OPT_LP(SGD); break; }
    case MOMENTUM: { KFB_OPT_LP(MOMENTUM); break; }
    case RMSPROP: { KFB_OPT_LP(RMSPROP); break; }
    case ADAM: { KFB_OPT_LP(ADAM); break; }
    default: return hipErrorInvalidValue;
  }
#undef KFB_OPT_LP
#undef KFB_OPT
  return hipGetLastError();
}

KFB_API hipError_t kfb_nonfinite(const float* x, long n, int* flag, hipStream_t stream) {
  hipLaunchKernelGGL(nonfinite_k, dim3(grid_for(n)), dim3(256), 0, stream, x, n, flag);
  return hipGetLastError();
}

KFB_API hipError_t kfb_half_sumsq(const float* x, long n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(half_sumsq_k, dim3(grid_for(n)), dim3(256), 0, stream, x, n, out);
  return hipGetLastError();
}

KFB_API hipError_t kfb_cast_f32(const float* x, void* y, int dtype, long n, hipStream_t stream) {
  if (dtype == BF16)
    hipLaunchKernelGGL((cast_f32_k<bf16>), dim3(grid_for(n)), dim3(256), 0, stream, x, (bf16*)y, n);
  else if (dtype == F16)
    hipLaunchKernelGGL((cast_f32_k<f16>), dim3(grid_for(n)), dim3(256), 0, stream, x, (f16*)y, n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

KFB_API hipError_t kfb_seqlock_check(const long long* seq, long long expect, int* ok, int* torn,
                                     hipStream_t stream) {
  hipLaunchKernelGGL(seqlock_check_k, dim3(1), dim3(1), 0, stream, seq, expect, ok, torn);
  return hipGetLastError();
}

// Page-locks host memory (e.g. a /dev/shm mapping) for device access;
// *dev receives its device address.
KFB_API hipError_t kfb_host_register(void* p, size_t bytes, void** dev) {
  hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped);
  if (e != hipSuccess) return e;
  return hipHostGetDevicePointer(dev, p, 0);
}

KFB_API hipError_t kfb_host_unregister(void* p) { return hipHostUnregister(p); }

// ---------------------------------------------------------------------------
// Peer model slots over HIP IPC (KungFu PairAveraging, parallel/kungfu.py).
// The exporter publishes the IPC handle of the allocation that holds its
// slots plus the slots' byte offset inside it (the caching allocator hands
// out sub-ranges of larger blocks); the importer opens the handle on ITS OWN
// device (the peer's memory mapped into this device's address space, peer
// access enabled), so no rank ever creates a context on a peer's GPU.

// handle (64 bytes) and the byte offset of p within its allocation
KFB_API hipError_t kfb_ipc_export(void* p, void* handle, long long* offset) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return e;
  void* base = nullptr;
  size_t size = 0;
  e = hipMemGetAddressRange(&base, &size, p);
  if (e != hipSuccess) return e;
  memcpy(handle, &h, sizeof(h));
  *offset = (long long)((char*)p - (char*)base);
  return hipSuccess;
}

KFB_API int kfb_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// Opens a peer's handle on `device` (this rank's own GPU): *base receives the
// mapped base address of the peer allocation.  The calling thread's current
// device is restored.
KFB_API hipError_t kfb_ipc_open(const void* handle, int device, void** base) {
  int prev = -1;
  hipError_t e = hipGetDevice(&prev);
  if (e != hipSuccess) return e;
  if (prev != device && (e = hipSetDevice(device)) != hipSuccess) return e;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  e = hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess);
  if (prev != device) {
    const hipError_t e2 = hipSetDevice(prev);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

KFB_API hipError_t kfb_ipc_close(void* base) { return hipIpcCloseMemHandle(base); }

// Peer access from `device` to `peer` (both physical indices as this process
// sees them); already-enabled counts as success, an impossible pairing as
// hipErrorPeerAccessUnsupported.
KFB_API hipError_t kfb_enable_peer(int device, int peer) {
  if (device == peer) return hipSuccess;
  int can = 0;
  hipError_t e = hipDeviceCanAccessPeer(&can, device, peer);
  if (e != hipSuccess) return e;
  if (!can) return hipErrorPeerAccessUnsupported;
  int prev = -1;
  if ((e = hipGetDevice(&prev)) != hipSuccess) return e;
  if (prev != device && (e = hipSetDevice(device)) != hipSuccess) return e;
  e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    e = hipSuccess;
  }
  if (prev != device) {
    const hipError_t e2 = hipSetDevice(prev);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

// y (fp32) = x (bf16 / fp16): a low-precision gradient wire buffer back into
// the flat fp32 gradient.
KFB_API hipError_t kfb_cast_to_f32(const void* x, int dtype, float* y, long n, hipStream_t stream) {
  if (dtype == BF16)
    hipLaunchKernelGGL((cast_to_f32_k<bf16>), dim3(grid_for(n)), dim3(256), 0, stream,
                       (const bf16*)x, y, n);
  else if (dtype == F16)
    hipLaunchKernelGGL((cast_to_f32_k<f16>), dim3(grid_for(n)), dim3(256), 0, stream,
                       (const f16*)x, y, n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
