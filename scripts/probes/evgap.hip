// Cost of a cross-stream dependency on the producing stream.  Stream A runs
// K1, K2, K1, K2, ... (short compute kernels); after every K1 stream B waits
// for it and runs a tiny K3.  Variants of how the dependency is expressed:
//   none    no cross-stream dependency (B idle)
//   record  hipEventRecord(ev, A) after K1 + hipStreamWaitEvent(B, ev)
//   ext     K1 launched with hipExtLaunchKernel(..., stopEvent = ev) (the
//           event bound to the kernel, no separate marker) + hipStreamWaitEvent
//   *-nsf   the same with events created hipEventDisableSystemFence
//   *-dev   the same with events created hipEventReleaseToDevice
// Printed: us per A-pair (K1 + K2) over REPS pairs, min of 5 rounds.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void work(float* p, int iters) {
  float v = p[blockIdx.x * blockDim.x + threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.5f;
  p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                         \
    }                                                                   \
  } while (0)

int main() {
  const int REPS = 200, G = 1024, B = 256;
  float *p1, *p2, *p3;
  CK(hipMalloc(&p1, G * B * 4));
  CK(hipMalloc(&p2, G * B * 4));
  CK(hipMalloc(&p3, 64 * 4));
  CK(hipMemset(p1, 0, G * B * 4));
  CK(hipMemset(p2, 0, G * B * 4));
  CK(hipMemset(p3, 0, 64 * 4));
  hipStream_t A, Bs;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&Bs, hipStreamNonBlocking));
  hipEvent_t evs[3][REPS];
  const unsigned fl[3] = {0u, (unsigned)hipEventDisableSystemFence, (unsigned)hipEventReleaseToDevice};
  for (int f = 0; f < 3; ++f)
    for (int i = 0; i < REPS; ++i)
      CK(hipEventCreateWithFlags(&evs[f][i], hipEventDisableTiming | fl[f]));
  const char* names[7] = {"none", "record", "ext", "record-nsf", "ext-nsf", "record-dev", "ext-dev"};
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int iters : {200, 2000}) {
    for (int v = 0; v < 7; ++v) {
      const int variant = v == 0 ? 0 : (v % 2 ? 1 : 2);
      hipEvent_t* ev = evs[(v - 1) / 2 < 0 ? 0 : (v - 1) / 2];
      float best = 1e9;
      for (int round = 0; round < 6; ++round) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(t0, A));
        for (int r = 0; r < REPS; ++r) {
          int it = iters;
          void* a1[] = {&p1, &it};
          if (variant == 2) {
            CK(hipExtLaunchKernel((const void*)work, dim3(G), dim3(B), a1, 0, A, nullptr, ev[r], 0));
          } else {
            CK(hipLaunchKernel((const void*)work, dim3(G), dim3(B), a1, 0, A));
            if (variant == 1) CK(hipEventRecord(ev[r], A));
          }
          if (variant > 0) {
            CK(hipStreamWaitEvent(Bs, ev[r], 0));
            int one = 10;
            void* a3[] = {&p3, &one};
            CK(hipLaunchKernel((const void*)work, dim3(1), dim3(64), a3, 0, Bs));
          }
          void* a2[] = {&p2, &it};
          CK(hipLaunchKernel((const void*)work, dim3(G), dim3(B), a2, 0, A));
        }
        CK(hipEventRecord(t1, A));
        CK(hipEventSynchronize(t1));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, t0, t1));
        if (round > 0 && ms < best) best = ms;
      }
      printf("iters %5d  %-10s  %7.2f us per K1+K2 pair\n", iters, names[v], best * 1e3 / REPS);
    }
  }
  return 0;
}
