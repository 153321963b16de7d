// valu_peak.hip -- measures the chip-wide issue rate of the integer instructions the
// P-256 kernels are built from (v_mad_u64_u32 rate is undocumented).
// Each lane runs 8 independent chains; grid = 256 CUs x 8 waves.  Prints lane-ops/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ __launch_bounds__(256) void kpeak(uint64_t *out, uint32_t iters, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 7 + seed;
  uint64_t acc[8];
  uint32_t x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = a + j; x[j] = b + 3 * j; }
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) {  // v_mad_u64_u32
        acc[j] = (uint64_t)x[j] * (a + j) + acc[j];
      } else if (OP == 1) {  // v_add_u32 (full-rate reference)
        x[j] = x[j] + (a ^ j) ;
        x[j] = x[j] ^ (b + j);
      } else if (OP == 2) {  // v_mul_hi_u32
        x[j] = __umulhi(x[j], a + j) + j;
      } else {  // add-with-carry pair (v_add_co + v_addc)
        uint32_t c;
        x[j] = __builtin_addc(x[j], a, 0u, &c);
        acc[j] += c;
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j] + x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
double run(uint64_t *d, uint32_t iters, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kpeak<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kpeak<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * 256 * iters * 8 * (OP == 1 ? 2 : 1);
  return ops / (ms * 1e-3);
}

int main() {
  int blocks = 256 * 8;
  uint64_t *d; hipMalloc(&d, blocks * 256 * 8);
  uint32_t it = 20000;
  printf("{\"v_mad_u64_u32_per_s\": %.4g, \"v_add_xor_u32_per_s\": %.4g, \"v_mul_hi_u32_per_s\": %.4g, \"addc_pair_per_s\": %.4g}\n",
         run<0>(d, it, blocks), run<1>(d, it, blocks), run<2>(d, it, blocks), run<3>(d, it, blocks));
  return 0;
}
