// Batched conv-weight re-layout for the data-gradient kernels.
//
// dgrad runs as an implicit GEMM whose B operand is the weight with input and
// output channels swapped: Wd[ci][a][b][co] = W[co][a'][b'][ci] with
// (a', b') = (KH-1-a, KW-1-b) for stride-1 convs (the transposed conv is a
// forward conv with the flipped kernel) and (a, b) otherwise.  Instead of one
// permute/flip copy per conv per step, the optimizer's low-precision weight
// buffer is re-laid out for ALL convs in one launch right after the update:
// the host builds a table of 64x64 (co, ci) tiles per tap and every
// workgroup transposes one tile through LDS (coalesced 16-byte reads and
// writes on both sides).
#include "common.h"

namespace kfb {

struct WtItem {  // one 64x64 tile of one tap of one conv
  long src;      // element offset of W[co=0][a=0][b=0][ci=0] in the source buffer
  long dst;      // element offset of Wd[ci=0][0][0][co=0] in the destination buffer
  int cout, cin, kh, kw;
  int a, b, flip;  // destination tap (a, b)
  int co0, ci0;
};

template <typename T>
__global__ void __launch_bounds__(256) wtrans_k(const T* __restrict__ src, T* __restrict__ dst,
                                                const WtItem* __restrict__ items) {
  __shared__ T tile[64][64 + 8];
  const WtItem it = items[blockIdx.x];
  const int sa = it.flip ? it.kh - 1 - it.a : it.a;
  const int sb = it.flip ? it.kw - 1 - it.b : it.b;
  const int taps = it.kh * it.kw;
  // read: rows co (64), 8 ci per lane (16 B)
  const int t = threadIdx.x;
  for (int r = t / 8; r < 64; r += 32) {
    const int co = it.co0 + r, ci = it.ci0 + (t % 8) * 8;
    float v[8];
    if (co < it.cout && ci < it.cin) {
      load_vec<T, 8>(src + it.src + ((long)co * taps + sa * it.kw + sb) * it.cin + ci, v);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[r][(t % 8) * 8 + k] = (T)v[k];
  }
  __syncthreads();
  // write: rows ci (64), 8 co per lane
  for (int r = t / 8; r < 64; r += 32) {
    const int ci = it.ci0 + r, co = it.co0 + (t % 8) * 8;
    if (ci >= it.cin || co >= it.cout) continue;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)tile[(t % 8) * 8 + k][r];
    store_vec<T, 8>(dst + it.dst + ((long)ci * taps + it.a * it.kw + it.b) * it.cout + co, v);
  }
}

}  // namespace kfb

using namespace kfb;

KFB_API int kfb_wtrans_item_bytes() { return (int)sizeof(WtItem); }

// items: device array of n WtItem.  cin and cout must be multiples of 8.
KFB_API hipError_t kfb_weight_transforms(int dtype, const void* src, void* dst, const void* items,
                                         int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (dtype == BF16)
    hipLaunchKernelGGL((wtrans_k<bf16>), dim3(n), dim3(256), 0, stream, (const bf16*)src,
                       (bf16*)dst, (const WtItem*)items);
  else if (dtype == F16)
    hipLaunchKernelGGL((wtrans_k<f16>), dim3(n), dim3(256), 0, stream, (const f16*)src,
                       (f16*)dst, (const WtItem*)items);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
