// fgv_kernels.h -- shared layout constants and kernel declarations (device + host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Fixed-base comb: 43 windows of 6 bits (signed digits in [-31, 32]), 32 entries/window.
#define WBITS 6
#define NWIN 43
#define TAB_K 32
#define KT_ENTRIES (NWIN * TAB_K)           // 1376 affine points per table
#define KT_BYTES ((size_t)KT_ENTRIES * 64)  // 88,064 bytes per table
#define PREP_B 8                            // items per lane in the batched inversion
#define POINT_THREADS 512
#define ST_PENDING 0xFF

struct apoint_raw {  // affine point, Montgomery limbs (64 B, 16-B aligned)
  uint32_t x[8];
  uint32_t y[8];
};
struct jpoint_raw {  // key-table build scratch: Jacobian point + prefix product
  uint32_t x[8];
  uint32_t y[8];
  uint32_t z[8];
  uint32_t pref[8];
};

__global__ void k_keytab(const uint32_t *qxy, const uint32_t *slots, apoint_raw *tables,
                         jpoint_raw *scratch, uint8_t *key_ok, uint32_t nkeys);
__global__ void k_prep(uint32_t n, uint8_t *status, const uint32_t *key_slot, const uint8_t *key_ok,
                       const uint32_t *r_limbs, const uint32_t *s_limbs, const uint8_t *digests,
                       const uint32_t *dig_idx, int8_t *d1, int8_t *d2, uint32_t *w_scratch);
__global__ void k_point(uint32_t n, uint8_t *status, const uint32_t *key_slot, const apoint_raw *gtab,
                        const apoint_raw *ktab, const int8_t *d1, const int8_t *d2,
                        const uint32_t *r_limbs);
struct ShaJob {  // message = span0 || span1 || span2 (absolute device addresses)
  uint64_t p[3];
  uint32_t n[3];
  uint32_t pad;
};
__global__ void k_sha256_jobs(const ShaJob *jobs, uint32_t n, uint8_t *out);
__global__ void k_sha256(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint32_t n,
                         uint8_t *out);
__global__ void k_der(const uint8_t *sig_buf, const uint64_t *off, const uint32_t *len, uint32_t n,
                      uint8_t *status, uint32_t *r_limbs, uint32_t *s_limbs);
