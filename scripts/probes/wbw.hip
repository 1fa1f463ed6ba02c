// HBM write-bandwidth probe: what a write-heavy streaming kernel can reach.
//   write:  every lane stores 16 B, fully coalesced, grid-stride
//   copy:   16 B load + 16 B store
//   r1w4:   16 B load, 4 x 16 B stores (the 1x1 64->256 expand's traffic mix)
//   w32:    stores in 32-byte pieces at a 512-byte row stride (S1's pattern)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned v4u;

__global__ void k_write(v4u* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = v4u{(unsigned)i, 1, 2, 3};
}
__global__ void k_copy(const v4u* x, v4u* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = x[i];
}
__global__ void k_r1w4(const v4u* x, v4u* y, long n) {  // n = x elements
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    v4u v = x[i];
    long b = (i / 64) * 256 + (i % 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) y[b + 64 * k] = v + k;
  }
}
// rows of 512 B: lane pair (p, h) writes 16 B at row p, chunk 2c + h
__global__ void k_w32(v4u* y, long rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (long r0 = blockIdx.x * 32L; r0 < rows; r0 += gridDim.x * 32L) {
    long p = r0 + (lane & 31);
#pragma unroll
    for (int c = 0; c < 4; ++c) y[p * 32 + 8 * w + 2 * c + (lane >> 5)] = v4u{(unsigned)p, 0, 0, 0};
  }
}

int main() {
  const long bytes = 411L << 20;  // ~ the expand conv's output
  v4u *x, *y;
  hipMalloc(&x, bytes);
  hipMalloc(&y, bytes);
  hipMemset(x, 1, bytes);
  hipMemset(y, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const long n = bytes / 16;
  for (int grid : {1024, 2048, 4096, 8192}) {
    float t[4];
    for (int kind = 0; kind < 4; ++kind) {
      float best = 1e9;
      for (int it = 0; it < 6; ++it) {
        hipEventRecord(a);
        if (kind == 0) k_write<<<grid, 256>>>(y, n);
        if (kind == 1) k_copy<<<grid, 256>>>(x, y, n / 2);
        if (kind == 2) k_r1w4<<<grid, 256>>>(x, y, n / 4);
        if (kind == 3) k_w32<<<grid / 4, 256>>>(y, bytes / 512);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
      }
      t[kind] = best;
    }
    // bytes moved: write = bytes, copy = bytes (n/2 read + n/2 written), r1w4 = bytes*5/4, w32 = bytes
    printf("grid %5d  write %.2f TB/s  copy %.2f TB/s  r1w4 %.2f TB/s  w32 %.2f TB/s\n", grid,
           bytes / t[0] / 1e9, bytes / t[1] / 1e9, bytes * 1.25 / t[2] / 1e9, bytes / t[3] / 1e9);
  }
  return 0;
}
