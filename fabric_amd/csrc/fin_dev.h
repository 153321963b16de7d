// fin_dev.h -- the batch txid table of the device finalize (finalize.hip), shared with
// k_bd_fold, which runs the k_fin_codes step itself for a single-device fused call.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ inline uint64_t fin_hash(const uint32_t *k, uint64_t seed) {
  uint64_t h = seed;
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const uint64_t w = (uint64_t)k[i] | ((uint64_t)k[i + 1] << 32);
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
  }
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 31);
}

// slot of key k in a table whose owners' keys sit in `keys` (32 B per position; the early
// index k_fin_index_dev), or -1
__device__ inline int64_t fin_find_keys(const uint32_t k[8], uint64_t h, const uint32_t *owner, const uint8_t *keys,
                                        uint32_t mask) {
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint32_t s = (uint32_t)(h + probe) & mask;
    const uint32_t o = owner[s];
    if (o == 0) return -1;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(keys + (size_t)(o - 1) * 32);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; i++) eq &= q[i] == k[i];
    if (eq) return s;
  }
  return -1;
}

// k_bd_fold's k_fin_codes step: owner == nullptr = off (the finalize runs it after the fold)
struct FinDev {
  const uint32_t *owner;
  const int32_t *minblk;
  uint32_t *minvalid;
  const uint8_t *keys;
  uint8_t *flags;
  uint32_t *pslot;
  uint32_t mask;
  uint64_t seed;
};
