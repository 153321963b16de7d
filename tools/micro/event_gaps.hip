// event_gaps.hip -- micro-benchmark: the gap between two dependent kernels on one stream when
// the stream also waits on events of other streams (already complete, or not) and records
// timing / non-timing events in between.  Prints the median gap per variant (us).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__global__ void k_spin(uint64_t cycles, uint32_t *out) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  hipStream_t a, b, c;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  uint32_t *d;
  CK(hipMalloc(&d, 64));
  hipEvent_t e1, e2, t1, t2, n1, n2, m0, m1;
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&t1));
  CK(hipEventCreate(&t2));
  CK(hipEventCreateWithFlags(&n1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&n2, hipEventDisableTiming));
  CK(hipEventCreate(&m0));
  CK(hipEventCreate(&m1));
  const uint64_t us = 100;  // wall_clock64 runs at 100 MHz on MI300-class parts
  const char *names[] = {"plain back-to-back", "timing event record between", "non-timing event record between",
                         "wait 1 done event (other stream)", "wait 2 done events", "wait 1 done non-timing event",
                         "wait on event still pending (producer ends first)", "cross-stream handoff (producer on b)"};
  for (int v = 0; v < 8; v++) {
    std::vector<float> gaps;
    for (int rep = 0; rep < 30; rep++) {
      // producer work on b / c that is long finished (variants 3-5) or still running (6)
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, b, 20 * us, d);
      CK(hipEventRecord(e1, b));
      CK(hipEventRecord(n1, b));
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c, 20 * us, d);
      CK(hipEventRecord(e2, c));
      CK(hipStreamSynchronize(b));
      CK(hipStreamSynchronize(c));
      if (v == 6 || v == 7) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, b, (v == 6 ? 300 : 200) * us, d);
        CK(hipEventRecord(e1, b));
      }
      if (v == 7) {
        CK(hipEventRecord(m0, b));  // (unused)
      }
      // measured pair on a: K1 (200 us) ... K2; gap = m1 - m0 brackets minus kernel times
      if (v != 7) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, 200 * us, d);
      CK(hipEventRecord(m0, v == 7 ? b : a));
      if (v == 1) CK(hipEventRecord(t1, a));
      if (v == 2) CK(hipEventRecord(n2, a));
      if (v == 3 || v == 4 || v == 6 || v == 7) CK(hipStreamWaitEvent(a, e1, 0));
      if (v == 4) CK(hipStreamWaitEvent(a, e2, 0));
      if (v == 5) CK(hipStreamWaitEvent(a, n1, 0));
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, 1, d);
      CK(hipEventRecord(m1, a));
      CK(hipStreamSynchronize(a));
      CK(hipStreamSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, m0, m1));
      gaps.push_back(ms * 1000.f);
    }
    std::sort(gaps.begin(), gaps.end());
    const float base = v == 6 ? 100.f : 0.f;  // variant 6: K1 ends 100 us before the producer
    printf("%-52s median %7.1f us  (min %6.1f)\n", names[v], gaps[gaps.size() / 2] - base, gaps[0] - base);
  }
  return 0;
}
