// Probe: sustained FLOP/s of v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16
// on random (gaussian-like) operands held in registers, 4 independent
// accumulator chains per wave, 8 waves per CU on every CU, 2 s of work per
// form, interleaved A/B/A/B.  Under DVFS the chip's clock depends on the
// switching activity of the operands, so zero-filled operands would overstate
// both forms.
//   build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(8))) short v8s;
typedef __attribute__((ext_vector_type(4))) float v4f;
typedef __attribute__((ext_vector_type(16))) float v16f;

__device__ __forceinline__ short rnd_bf16(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  // bf16 with a random mantissa and exponent in [2^-2, 2^1], random sign
  return (short)(((s >> 16) & 0x807F) | ((125u + ((s >> 8) & 3u)) << 7));
}

template <int FORM>
__global__ void __launch_bounds__(256) mfma_loop(float* out, int iters, unsigned seed) {
  unsigned s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
  v8s a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = rnd_bf16(s);
    b[i] = rnd_bf16(s);
  }
  if constexpr (FORM == 16) {
    v4f c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < iters; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  } else {
    v16f c0 = {}, c1 = {};
    for (int it = 0; it < iters; ++it) {
      // 2 chains of 32x32x16 = the FLOPs of 4 chains of 16x16x32
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[5];
  }
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 2;  // 8 waves per CU
  float* out;
  (void)hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2000000;  // ~0.12 s per launch
  // FLOPs per launch: blocks * 4 waves * iters * 4 (16x16x32) * 16*16*32*2
  const double flop = (double)blocks * 4 * iters * 4 * (16.0 * 16 * 32 * 2);
  for (int round = 0; round < 3; ++round) {
    for (int form : {16, 32}) {
      (void)hipEventRecord(e0);
      if (form == 16) hipLaunchKernelGGL(mfma_loop<16>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u + round);
      else hipLaunchKernelGGL(mfma_loop<32>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u + round);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("round %d  %s  %8.2f ms  %7.1f TFLOP/s\n", round,
             form == 16 ? "16x16x32" : "32x32x16", ms, flop / ms / 1e9);
    }
  }
  (void)hipFree(out);
  return 0;
}
