// hexcheck.hip -- test helper (not part of libfgv): runs the device txid decoder hex64_words
// (fabric_amd/csrc/fin_dev.h, used by k_fin_rows, k_fin_index_dev and k_bd_fold) on chosen
// offsets of a device buffer, so tests/test_gpu_hexwords.py can pin it against Python's
// bytes.fromhex at every alignment, with bad characters at every position, and on a txid that
// ends at the last byte before the buffer's 64-byte tail padding.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../fabric_amd/csrc/fin_dev.h"

__global__ void k_hexcheck(const uint8_t *buf, const uint32_t *offs, uint32_t k, uint8_t *ok, uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  uint32_t w[8];
  ok[i] = hex64_words(buf + offs[i], w) ? 1 : 0;
  for (int j = 0; j < 8; j++) out[8 * i + j] = w[j];
}

extern "C" int hexcheck_run(const uint8_t *h_buf, size_t n, const uint32_t *offs, size_t k, uint8_t *ok, uint32_t *out) {
  uint8_t *d_buf = nullptr, *d_ok = nullptr;
  uint32_t *d_offs = nullptr, *d_out = nullptr;
  int rc = 0;
  if (hipMalloc(&d_buf, n + 64) != hipSuccess || hipMalloc(&d_offs, k * 4) != hipSuccess ||
      hipMalloc(&d_ok, k) != hipSuccess || hipMalloc(&d_out, k * 32) != hipSuccess)
    rc = -1;
  if (!rc && (hipMemset(d_buf, 0x5a, n + 64) != hipSuccess ||
              hipMemcpy(d_buf, h_buf, n, hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(d_offs, offs, k * 4, hipMemcpyHostToDevice) != hipSuccess))
    rc = -2;
  if (!rc) {
    for (size_t i = 0; i < k; i++)
      if (offs[i] + 64 > n) rc = -3;  // (a span must lie inside the buffer)
  }
  if (!rc) {
    hipLaunchKernelGGL(k_hexcheck, dim3((uint32_t)((k + 63) / 64)), dim3(64), 0, 0, d_buf, d_offs, (uint32_t)k, d_ok, d_out);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(ok, d_ok, k, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(out, d_out, k * 32, hipMemcpyDeviceToHost) != hipSuccess)
      rc = -4;
  }
  hipFree(d_buf);
  hipFree(d_offs);
  hipFree(d_ok);
  hipFree(d_out);
  return rc;
}
