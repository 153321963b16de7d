// der_kernel.hip -- Go-rule DER decode + low-S on the device, one signature per lane, for
// batches already resident in HBM (same fgv_der.h definition the host path uses).
// Replaces bccsp/utils/ecdsa.go:41-65 (UnmarshalECDSASignature) + :82-89 (IsLowS) and the
// empty-signature check of bccsp/sw/impl.go:253-255.
#include "fgv_der.h"
#include "fgv_kernels.h"

__global__ __launch_bounds__(256) void k_der(const uint8_t *__restrict__ sig_buf,
                                             const uint64_t *__restrict__ off,
                                             const uint32_t *__restrict__ len, uint32_t n,
                                             uint8_t *__restrict__ status,
                                             uint32_t *__restrict__ r_limbs,
                                             uint32_t *__restrict__ s_limbs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t r[8], s[8];
  uint8_t code = ST_PENDING;
  const uint32_t L = len[i];
  bool rb = false, sb = false;
  if (L == 0) {
    code = 6;
  } else if (fgv::der_decode_sig(sig_buf + off[i], L, r, s, rb, sb)) {
    code = 2;
  } else if (sb || !fgv::is_low_s(s)) {
    code = 3;
  } else if (rb) {
    // r >= 2^256 -> an out-of-range value (n) so k_prep reports RANGE after the key check
    r[0] = 0xFC632551u; r[1] = 0xF3B9CAC2u; r[2] = 0xA7179E84u; r[3] = 0xBCE6FAADu;
    r[4] = 0xFFFFFFFFu; r[5] = 0xFFFFFFFFu; r[6] = 0x00000000u; r[7] = 0xFFFFFFFFu;
  }
  if (code != ST_PENDING) {
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = s[k] = 0;
  }
  status[i] = code;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r_limbs[(size_t)k * n + i] = r[k];
    s_limbs[(size_t)k * n + i] = s[k];
  }
}
