// sha3_dev.h -- SHA3-256 on the device for MSPs whose SignatureHashFamily is SHA3.
//
// identity.Verify hashes the message with the MSP's hash family (msp/identities.go:170-199,
// getHashOpt :219-227): SHA3 -> bccsp SHA3_256Opts -> the sw CSP's hasher over
// golang.org/x/crypto/sha3.New256 (bccsp/sw/new.go), i.e. FIPS 202 SHA3-256: Keccak-f[1600],
// rate 136 bytes, domain padding 0x06 ... 0x80, the first 32 bytes of the state out.
//
// Used where a SHA3 identity's digest replaces the SHA-256 one: k_sha256_jobs (a job flagged
// SHA3, the host-parse committer) and k_bd_sha3 (the device-parse committer's creator and
// endorsement slots).  One lane per message; SHA3 MSPs are rare, so the lanes read their bytes
// one at a time (any alignment) and no effort goes into sharing a wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fgvsha3 {

__constant__ static const uint64_t RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

__device__ __forceinline__ uint64_t rotl(uint64_t x, int s) { return s ? (x << s) | (x >> (64 - s)) : x; }

// Keccak-f[1600]: theta, rho + pi, chi, iota; a[x + 5 y]
__device__ inline void keccak_f(uint64_t a[25]) {
  // rho offsets and the pi lane order (the standard "pi-then-rho" walk starting from lane 1)
  constexpr int ROT[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
  constexpr int PI[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
#pragma unroll 1
  for (int r = 0; r < 24; r++) {
    uint64_t c[5];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
#pragma unroll
      for (int y = 0; y < 25; y += 5) a[x + y] ^= d;
    }
    uint64_t t = a[1];
#pragma unroll
    for (int i = 0; i < 24; i++) {
      const uint64_t u = a[PI[i]];
      a[PI[i]] = rotl(t, ROT[i]);
      t = u;
    }
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      uint64_t b[5];
#pragma unroll
      for (int x = 0; x < 5; x++) b[x] = a[y + x];
#pragma unroll
      for (int x = 0; x < 5; x++) a[y + x] = b[x] ^ (~b[(x + 1) % 5] & b[(x + 2) % 5]);
    }
    a[0] ^= RC[r];
  }
}

// SHA3-256 of span0 || span1 || span2 (device addresses, any alignment; a span may be empty)
__device__ inline void sha3_256_spans(const uint8_t *const p[3], const uint32_t n[3], uint8_t out[32]) {
  constexpr uint32_t RATE = 136;
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; i++) a[i] = 0;
  uint32_t pos = 0;  // byte position within the current block
  uint64_t lane = 0;
  auto absorb = [&](uint8_t byte) {
    lane |= (uint64_t)byte << (8 * (pos & 7));
    pos++;
    if ((pos & 7) == 0) {
      a[(pos >> 3) - 1] ^= lane;
      lane = 0;
      if (pos == RATE) {
        keccak_f(a);
        pos = 0;
      }
    }
  };
  for (int s = 0; s < 3; s++)
    for (uint32_t i = 0; i < n[s]; i++) absorb(p[s][i]);
  // pad10*1 with the SHA3 domain bits 01: 0x06 at the end of the message, 0x80 in the last
  // byte of the block (one byte 0x86 when they coincide)
  lane |= (uint64_t)0x06 << (8 * (pos & 7));
  a[pos >> 3] ^= lane;
  a[(RATE >> 3) - 1] ^= 0x8000000000000000ull;
  keccak_f(a);
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(a[i] >> (8 * b));
}

}  // namespace fgvsha3
