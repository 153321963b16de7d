// sha256_host.h -- streaming SHA-256 on the host for the block data hash.
//
// The block data hash (protoutil/blockutils.go:76-79, ComputeBlockDataHash) is ONE
// Merkle-Damgard chain over every envelope of the block (~110 MB for a 20k-tx block): no
// intra-message parallelism exists, and a single GPU lane runs one compression per ~2 us,
// i.e. ~30 MB/s, while an x86 core with the SHA extensions does ~1.5-2 GB/s.  So this chain
// runs on host cores (one block per thread, overlapped with the GPU's batch work); the
// per-message hashes of the committer path stay on the GPU (sha256.hip).
//
// SHA-NI path (Intel SHA extensions: sha256rnds2 / sha256msg1 / sha256msg2, FIPS 180-4
// round structure) selected at run time by CPUID; portable scalar path otherwise.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace fgvsha {

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

void compress_scalar(uint32_t st[8], const uint8_t *p, size_t nblk);
void compress_ni(uint32_t st[8], const uint8_t *p, size_t nblk);
bool have_sha_ni();

struct Stream {
  uint32_t st[8];
  uint8_t buf[64];
  size_t fill = 0;
  uint64_t total = 0;
  void (*comp)(uint32_t *, const uint8_t *, size_t);
  Stream() {
    static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(st, IV, sizeof st);
    comp = have_sha_ni() ? compress_ni : compress_scalar;
  }
  void update(const uint8_t *p, size_t n) {
    total += n;
    if (fill) {
      const size_t k = n < 64 - fill ? n : 64 - fill;
      memcpy(buf + fill, p, k);
      fill += k;
      p += k;
      n -= k;
      if (fill < 64) return;
      comp(st, buf, 1);
      fill = 0;
    }
    if (n >= 64) {
      comp(st, p, n / 64);
      p += n & ~(size_t)63;
      n &= 63;
    }
    if (n) {
      memcpy(buf, p, n);
      fill = n;
    }
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    uint8_t pad[72];
    const size_t padn = (fill < 56 ? 56 - fill : 120 - fill);
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    for (int i = 0; i < 8; i++) pad[padn + i] = (uint8_t)(bits >> (56 - 8 * i));
    const uint64_t keep = total;
    update(pad, padn + 8);
    total = keep;
    for (int i = 0; i < 8; i++) {
      out[4 * i] = (uint8_t)(st[i] >> 24);
      out[4 * i + 1] = (uint8_t)(st[i] >> 16);
      out[4 * i + 2] = (uint8_t)(st[i] >> 8);
      out[4 * i + 3] = (uint8_t)st[i];
    }
  }
};

inline void sha256(const uint8_t *p, size_t n, uint8_t out[32]) {
  Stream s;
  s.update(p, n);
  s.final(out);
}

}  // namespace fgvsha
