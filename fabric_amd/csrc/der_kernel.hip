// der_kernel.hip -- Go-rule DER decode + low-S on the device, one signature per lane, for
// batches already resident in HBM (same fgv_der.h definition the host path uses).
// Replaces bccsp/utils/ecdsa.go:41-65 (UnmarshalECDSASignature) + :82-89 (IsLowS) and the
// empty-signature check of bccsp/sw/impl.go:253-255.
#include "fgv_der.h"
#include "fgv_kernels.h"

// Signatures up to DER_STAGE_MAX bytes are first copied into LDS with independent aligned
// dword loads (one memory latency instead of one per parsed byte: the parse is a chain of
// dependent byte reads), then decoded from LDS.  Longer ones are decoded in place.
#define DER_STAGE_MAX 124
#define DER_STAGE_DW 33  // dwords per lane: (3 + DER_STAGE_MAX + 3) / 4 + pad

__global__ __launch_bounds__(256) void k_der(const uint8_t *__restrict__ sig_buf,
                                             const uint64_t *__restrict__ off,
                                             const uint32_t *__restrict__ len, uint32_t n,
                                             const uint32_t *__restrict__ dn,
                                             uint8_t *__restrict__ status,
                                             uint32_t *__restrict__ r_limbs,
                                             uint32_t *__restrict__ s_limbs,
                                             const uint32_t *__restrict__ key_slot) {
  __builtin_amdgcn_s_setprio(3);  // on the verify chain; SHA-256 may be running beside it
  __shared__ uint32_t stage[256 * DER_STAGE_DW];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // n: capacity (the r / s column stride); dn: the item count in device memory (or n)
  if (i >= (dn ? min(n, *dn) : n)) return;
  if (key_slot && (key_slot[i] & KEY_P384_FLAG)) {  // a P-384 identity's signature: k_p384_verify
    status[i] = ST_P384;
#pragma unroll
    for (int k = 0; k < 8; k++) r_limbs[(size_t)k * n + i] = s_limbs[(size_t)k * n + i] = 0;
    return;
  }
  uint32_t r[8], s[8];
  uint8_t code = ST_PENDING;
  const uint32_t L = len[i];
  const uint8_t *src = sig_buf ? sig_buf + off[i] : reinterpret_cast<const uint8_t *>((uintptr_t)off[i]);
  if (L > 0 && L <= DER_STAGE_MAX) {
    // aligned dwords covering [src, src + L); device allocations are >= 4-byte aligned, so
    // the dword holding src starts inside the allocation; the last partial dword is read by
    // bytes (never past src + L)
    const uintptr_t a = (uintptr_t)src, a0 = a & ~(uintptr_t)3, end = a + L;
    const uint32_t nd = (uint32_t)((end - a0 + 3) >> 2);
    uint32_t *dst = stage + threadIdx.x * DER_STAGE_DW;
#pragma unroll
    for (uint32_t d = 0; d < DER_STAGE_DW; d++) {
      const uintptr_t p = a0 + 4 * d;
      if (d >= nd) {
      } else if (p + 4 <= end) {
        dst[d] = *reinterpret_cast<const uint32_t *>(p);
      } else {
        uint32_t w = 0;
        for (uintptr_t q = p; q < end; q++) w |= (uint32_t)(*reinterpret_cast<const uint8_t *>(q)) << (8 * (q - p));
        dst[d] = w;
      }
    }
    src = reinterpret_cast<const uint8_t *>(dst) + (a - a0);
  }
  bool rb = false, sb = false;
  if (L == 0) {
    code = 6;
  } else if (fgv::der_decode_sig(src, L, r, s, rb, sb)) {
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
