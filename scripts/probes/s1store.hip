// Store pattern of the streaming 1x1 forward (csrc/conv_s1.hip EPI_STATS) vs
// a fully coalesced one, at its traffic mix: per 32-pixel tile each 256-thread
// workgroup reads a 4 KB input tile and writes a 16 KB output tile (512-byte
// pixel rows, 56x56 64 -> 256 at batch 256: 25088 tiles).
//   s1:   store i of lane (l32, hh) in wave w writes 16 B at row l32, chunk
//         8 w + 2 i + hh (32-byte pieces in 32 rows per instruction)
//   coal: store i writes 16 B at byte 16 (256 i + tid) (1 KB runs)
//   lds:  the s1 fragments written to LDS, read back row-contiguous, stored
//         as coal (the cost of staging the tile through LDS)
//   seg:  store i of wave w writes 16 B at row 8 i + lane / 8, chunk 8 w +
//         lane % 8 (each wave's own 128-byte column: 8 full lines per
//         instruction, a wave-local staging needs no workgroup barrier)
// Persistent grid (workgroups per CU x 256 CUs), grid-stride over tiles.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned v4u;

template <int MODE>
__global__ void __launch_bounds__(256) k_tile(const v4u* __restrict__ x, v4u* __restrict__ y,
                                              int tiles) {
  __shared__ v4u st[1024];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l32 = lane & 31, hh = lane >> 5;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const v4u v = x[(long)t * 256 + tid];
    v4u* yt = y + (long)t * 1024;
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) yt[l32 * 32 + 8 * w + 2 * i + hh] = v + (unsigned)i;
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) yt[256 * i + tid] = v + (unsigned)i;
    } else if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 4; ++i) yt[(8 * i + (lane >> 3)) * 32 + 8 * w + (lane & 7)] = v + (unsigned)i;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) st[l32 * 32 + ((8 * w + 2 * i + hh) ^ (l32 & 31))] = v + (unsigned)i;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 256 * i + tid, r = e >> 5, c = e & 31;
        yt[e] = st[r * 32 + (c ^ (r & 31))];
      }
      __syncthreads();
    }
  }
}

int main() {
  const int tiles = 25088;
  v4u *x, *y;
  hipMalloc(&x, (long)tiles * 4096);
  hipMalloc(&y, (long)tiles * 16384);
  hipMemset(x, 1, (long)tiles * 4096);
  hipMemset(y, 1, (long)tiles * 16384);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = (double)tiles * (4096 + 16384);
  for (int wpc : {1, 2, 4, 8}) {
    const int grid = 256 * wpc;
    float t[4];
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e9;
      for (int it = 0; it < 8; ++it) {
        hipEventRecord(a);
        if (mode == 0) k_tile<0><<<grid, 256>>>(x, y, tiles);
        if (mode == 1) k_tile<1><<<grid, 256>>>(x, y, tiles);
        if (mode == 2) k_tile<2><<<grid, 256>>>(x, y, tiles);
        if (mode == 3) k_tile<3><<<grid, 256>>>(x, y, tiles);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
      }
      t[mode] = best;
    }
    printf("wg/CU %d  s1 %.1f us %.2f TB/s   coal %.1f us %.2f TB/s   lds %.1f us %.2f TB/s   "
           "seg %.1f us %.2f TB/s\n", wpc, t[0] * 1e3, bytes / t[0] / 1e9, t[1] * 1e3,
           bytes / t[1] / 1e9, t[2] * 1e3, bytes / t[2] / 1e9, t[3] * 1e3, bytes / t[3] / 1e9);
  }
  return 0;
}
