// Row gathers and channel concatenation.
//
// * Embedding lookup / gradient (NCF, tcb/models/experimental/
//   official_ncf_model.py via official.recommendation.neumf_model:
//   tf.nn.embedding_lookup and its IndexedSlices gradient): the forward
//   gathers rows of the table; the backward scatter-adds dy rows into the
//   fp32 flat-gradient view of the table (float atomics: several batch rows
//   may name the same table row).
// * Channel concat / split on NHWC activations (tf.concat(axis=3) in the
//   inception / DenseNet / NASNet cells, tcb/convnet_builder.py:347-383):
//   one launch over the output rows for all k inputs, the backward the same
//   walk in the other direction.  A null input is a block of zero channels
//   (channel padding of the CIFAR ResNet option-A shortcut).
#include "common.h"

namespace kfb {

template <typename T, int V>
__global__ void __launch_bounds__(256)
embed_fwd_k(const T* __restrict__ table, const int* __restrict__ idx, T* __restrict__ out, long n,
            int dim, long rows_in_table) {
  const int cv = dim / V;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n * cv;
       i += (long)gridDim.x * blockDim.x) {
    const long b = i / cv;
    const int c = (int)(i - b * cv) * V;
    const long r = idx[b];
    float v[V];
    if (r >= 0 && r < rows_in_table) {
      load_vec<T, V>(table + r * dim + c, v);
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] = 0.f;  // out-of-range ids read zeros
    }
    store_vec<T, V>(out + b * dim + c, v);
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256)
embed_bwd_k(const T* __restrict__ dy, const int* __restrict__ idx, float* __restrict__ grad, long n,
            int dim, long rows_in_table) {
  const int cv = dim / V;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n * cv;
       i += (long)gridDim.x * blockDim.x) {
    const long b = i / cv;
    const int c = (int)(i - b * cv) * V;
    const long r = idx[b];
    if (r < 0 || r >= rows_in_table) continue;
    float g[V];
    load_vec<T, V>(dy + b * dim + c, g);
#pragma unroll
    for (int k = 0; k < V; ++k) atomicAdd(grad + r * dim + c + k, g[k]);
  }
}

// out[r][off_j + c] = in_j[r][c] for every input j (split: the reverse).
// The k <= 16 input pointers and channel offsets travel by value in the
// kernel arguments (no device-side table to upload per call).
constexpr int CAT_MAX = 16;
struct CatArgs {
  void* ptrs[CAT_MAX];
  int offs[CAT_MAX + 1];
  int k;
};

template <typename T, int V, bool SPLIT>
__global__ void __launch_bounds__(256)
concat_k(T* __restrict__ out, CatArgs a, long rows, int ctot) {
  const int cv = ctot / V;
  const long total = rows * cv;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / cv;
    const int c = (int)(i - r * cv) * V;
    int j = 0;
    while (j + 1 < a.k && a.offs[j + 1] <= c) ++j;
    const int cj = a.offs[j + 1] - a.offs[j];
    T* o = out + r * ctot + c;
    if (a.ptrs[j] == nullptr) {  // zero part (channel padding): written as 0, split skips it
      if constexpr (!SPLIT) {
        if constexpr (V == 1) *o = (T)0.f;
        else *reinterpret_cast<Vec<T, V>*>(o) = Vec<T, V>{};
      }
      continue;
    }
    T* p = (T*)a.ptrs[j] + r * cj + (c - a.offs[j]);
    if constexpr (V == 1) {
      if (SPLIT) *p = *o;
      else *o = *p;
    } else {
      typedef Vec<T, V> VT;
      if (SPLIT) *reinterpret_cast<VT*>(p) = *reinterpret_cast<const VT*>(o);
      else *reinterpret_cast<VT*>(o) = *reinterpret_cast<const VT*>(p);
    }
  }
}

inline unsigned gather_grid(long work) {
  long b = (work + 255) / 256;
  if (b > 256L * 16) b = 256L * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace kfb

using namespace kfb;

KFB_API hipError_t kfb_embedding_fwd(int dtype, const void* table, long rows_in_table,
                                     const int* idx, void* out, long n, int dim,
                                     hipStream_t stream) {
  const int V = vec_width(dim);
  KFB_DISPATCH_DTYPE(dtype, T, KFB_DISPATCH_VEC(V, VV, {
    hipLaunchKernelGGL((embed_fwd_k<T, VV>), dim3(gather_grid(n * (dim / VV))), dim3(256), 0,
                       stream, (const T*)table, idx, (T*)out, n, dim, rows_in_table);
  }));
  return hipGetLastError();
}

// grad: fp32 [rows_in_table][dim], accumulated (the caller zeroes it).
KFB_API hipError_t kfb_embedding_bwd(int dtype, const void* dy, const int* idx, float* grad,
                                     long rows_in_table, long n, int dim, hipStream_t stream) {
  const int V = vec_width(dim) > 4 ? 4 : vec_width(dim);
  KFB_DISPATCH_DTYPE(dtype, T, KFB_DISPATCH_VEC(V, VV, {
    hipLaunchKernelGGL((embed_bwd_k<T, VV>), dim3(gather_grid(n * (dim / VV))), dim3(256), 0,
                       stream, (const T*)dy, idx, grad, n, dim, rows_in_table);
  }));
  return hipGetLastError();
}

// split = 0: out[rows][ctot] = concat(ins, channels);  split = 1: the reverse.
// ptrs / offs are HOST arrays (k pointers, k+1 channel offsets), k <= 16;
// vec: every width and pointer allows 16-byte vectors.
KFB_API hipError_t kfb_concat(int dtype, void* out, void* const* ptrs, const int* offs, int k,
                              long rows, int ctot, int vec, int split, hipStream_t stream) {
  if (k < 1 || k > CAT_MAX) return hipErrorInvalidValue;
  CatArgs a{};
  for (int j = 0; j < k; ++j) a.ptrs[j] = ptrs[j];
  for (int j = 0; j <= k; ++j) a.offs[j] = offs[j];
  a.k = k;
  KFB_DISPATCH_DTYPE(dtype, T, {
    constexpr int V = 16 / sizeof(T);
    if (vec) {
      const unsigned g = gather_grid(rows * (ctot / V));
      if (split)
        hipLaunchKernelGGL((concat_k<T, V, true>), dim3(g), dim3(256), 0, stream, (T*)out, a,
                           rows, ctot);
      else
        hipLaunchKernelGGL((concat_k<T, V, false>), dim3(g), dim3(256), 0, stream, (T*)out, a,
                           rows, ctot);
    } else {
      const unsigned g = gather_grid(rows * ctot);
      if (split)
        hipLaunchKernelGGL((concat_k<T, 1, true>), dim3(g), dim3(256), 0, stream, (T*)out, a,
                           rows, ctot);
      else
        hipLaunchKernelGGL((concat_k<T, 1, false>), dim3(g), dim3(256), 0, stream, (T*)out, a,
                           rows, ctot);
    }
  });
  return hipGetLastError();
}

// ----------------------------------------------------- anchor-major heads
// SSD300 prediction heads (tcb/models/ssd_model.py): each head's NHWC
// output [nb][A = H*W][Bd = anchors per pixel][R = 4 or classes] goes to rows
// row0 + j*A + i (anchor-major), columns col0.. of the [nb][rows][ld] logits
// tensor - one launch per head instead of a permute copy plus two concats.
// dir = 1 is the backward: the head's gradient gathered back from dlogits.
namespace kfb {

template <typename T>
__global__ void __launch_bounds__(256)
heads_k(const T* __restrict__ src, T* __restrict__ dst, int nb, int A, int Bd, int R,
        long row0, int col0, long ob, int ld, int dir) {
  const long n = (long)nb * A * Bd * R;
  if (n < (1L << 31) && row0 + (long)Bd * A <= (1L << 31) / ld) {
    // 32-bit index math (every SSD300 head): unsigned divisions are a few
    // instructions, the 64-bit ones a long software sequence per element
    const unsigned n32 = (unsigned)n, uR = R, uBd = Bd, uA = A;
    for (unsigned e = blockIdx.x * 256u + threadIdx.x; e < n32; e += gridDim.x * 256u) {
      unsigned q = e / uR;
      const unsigned r = e - q * uR;
      unsigned q2 = q / uBd;
      const unsigned j = q - q2 * uBd;
      const unsigned b = q2 / uA, i = q2 - b * uA;
      const long o = b * ob + (long)((unsigned)row0 + j * uA + i) * ld + col0 + r;
      if (dir == 0) dst[o] = src[e];
      else dst[e] = src[o];
    }
    return;
  }
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int r = (int)(e % R);
    long q = e / R;
    const int j = (int)(q % Bd);
    q /= Bd;
    const int i = (int)(q % A);
    const int b = (int)(q / A);
    const long o = b * ob + (row0 + (long)j * A + i) * ld + col0 + r;  // logits element
    if (dir == 0) dst[o] = src[e];
    else dst[e] = src[o];
  }
}

}  // namespace kfb

KFB_API hipError_t kfb_ssd_heads(int dtype, const void* src, void* dst, int nb, int A, int Bd,
                                 int R, long row0, int col0, long ob, int ld, int dir,
                                 hipStream_t stream) {
  const long n = (long)nb * A * Bd * R;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  KFB_DISPATCH_DTYPE(dtype, T,
                     hipLaunchKernelGGL(kfb::heads_k<T>, dim3((unsigned)blocks), dim3(256), 0,
                                        stream, (const T*)src, (T*)dst, nb, A, Bd, R, row0, col0,
                                        ob, ld, dir));
  return hipGetLastError();
}
