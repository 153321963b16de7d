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

// The 64 lowercase hex characters at p (any alignment) -> 32 bytes as 8 little-endian words;
// false on any other character.  The 17 aligned dwords covering [p, p + 64) are loaded at once
// (at most 4 bytes past the span: inside the block's >= 64 B tail padding): a byte-at-a-time
// loop with an early exit waited for each load in turn (64 round trips per transaction in
// k_fin_rows / k_fin_index_dev / k_bd_fold).
__device__ inline bool hex64_words(const uint8_t *p, uint32_t out[8]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3u);
  uint32_t raw[17];
#pragma unroll
  for (int i = 0; i < 17; i++) raw[i] = w[i];
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 16; i++) {  // characters 4i .. 4i+3 -> bytes 2i, 2i+1
    const uint32_t x = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
    uint32_t nib[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t c = (x >> (8 * j)) & 0xFFu;
      const uint32_t d = c - (uint32_t)'0', h = c - (uint32_t)'a';
      ok &= (d < 10u) | (h < 6u);
      nib[j] = d < 10u ? d : h + 10u;
    }
    const uint32_t b0 = ((nib[0] << 4) | nib[1]) & 0xFFu, b1 = ((nib[2] << 4) | nib[3]) & 0xFFu;
    if (i & 1) out[i >> 1] |= (b0 << 16) | (b1 << 24);
    else out[i >> 1] = b0 | (b1 << 8);
  }
  return ok;
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
