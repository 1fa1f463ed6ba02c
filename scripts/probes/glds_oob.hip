// Probe: does buffer_load_dwordx4 ... lds (LDS-DMA) write zeros to LDS for
// an out-of-range lane (offset beyond num_records), like a register load?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void probe(const unsigned* src, unsigned* out, int nbytes) {
  __shared__ __attribute__((aligned(16))) unsigned lds[64 * 4 * 2];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 4 * 2; i += 64) lds[i] = 0xABABABABu;
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, 0x00020000);
  const int off = (lane & 1) ? -1 : lane * 16;  // odd lanes out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, off, 0, 0, 0);
  // second block: global_load_lds with a plain pointer
  __builtin_amdgcn_global_load_lds((const void*)(src + lane * 4), (__attribute__((address_space(3))) void*)(lds + 256), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 64 * 4 * 2; i += 64) out[i] = lds[i];
}

int main() {
  unsigned h[256], o[512];
  for (int i = 0; i < 256; ++i) h[i] = 1000 + i;
  unsigned *d, *dout;
  (void)hipMalloc(&d, sizeof(h)); (void)hipMalloc(&dout, sizeof(o));
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, dout, (int)sizeof(h));
  (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int bad = 0, zeros = 0, stale = 0;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j) {
      unsigned v = o[l * 4 + j];
      if (l & 1) { if (v == 0) ++zeros; else if (v == 0xABABABABu) ++stale; else ++bad; }
      else if (v != 1000u + l * 4 + j) ++bad;
      if (o[256 + l * 4 + j] != 1000u + l * 4 + j) ++bad;
    }
  printf("glds probe: in-range/global mismatches=%d  oob lanes: zero=%d stale=%d (of 128)\n", bad, zeros, stale);
  return bad ? 1 : 0;
}
