// sha256_dev.h -- SHA-256 device code shared by sha256.hip (job / arena kernels) and
// blockdev.hip (per-transaction payload hashes): the compression function and a message
// walker over up to three spans that loads the next block while compressing the current one.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__constant__ static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// a ^ b ^ c in one VALU op (gfx950 v_bitop3, truth table 0x96); hipcc emits two v_xor here
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ void sha_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = k + S1 + ch + SHA_K[i] + wi;
    uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    uint32_t mj = (a & b) | (c & (a | b));
    uint32_t t2 = S0 + mj;
    k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// ---------------------------------------------------------------------------------
// k_sha256_jobs: messages that are the concatenation of up to 3 spans, each given by an
// absolute device address (spans point straight into block bytes resident in HBM):
//   creator payload (1 span), nonce||creator (TxID, protoutil/proputils.go:351-360),
//   chdr||shdr||ccpp (proposal hash, protoutil/txutils.go:449-466),
//   prp||endorser (endorsement message, statebased/validator_keylevel.go:246-260).
// A hash is a serial chain of compressions, so a wave's time is its longest message; the
// next block's words are loaded before the current block is compressed (the loads' latency
// hides behind ~1.4k VALU ops).  A word is one unaligned 32-bit load (two aligned loads +
// v_alignbyte) unless it straddles a span boundary or the end (then byte by byte).
struct JobView {
  const uint8_t *p[3];
  uint32_t beg[4];  // span k covers message bytes [beg[k], beg[k+1])
  uint32_t L;
};
__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) {  // unaligned little-endian
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}
// span k's base and start by selects (a dynamically indexed JobView would live in scratch)
__device__ __forceinline__ const uint8_t *span_p(const JobView &v, int k) {
  return k == 0 ? v.p[0] : (k == 1 ? v.p[1] : v.p[2]);
}
__device__ __forceinline__ uint32_t span_beg(const JobView &v, int k) {
  return k == 0 ? 0u : (k == 1 ? v.beg[1] : v.beg[2]);
}
__device__ __forceinline__ uint32_t span_end(const JobView &v, int k) {
  return k == 0 ? v.beg[1] : (k == 1 ? v.beg[2] : v.beg[3]);
}
__device__ __forceinline__ uint32_t job_byte(const JobView &v, uint32_t q) {
  if (q >= v.L) return q == v.L ? 0x80u : 0u;
  const int k = q < v.beg[1] ? 0 : (q < v.beg[2] ? 1 : 2);
  return span_p(v, k)[q - span_beg(v, k)];
}
// big-endian message word at byte offset pos of the padded message (bit length excluded)
__device__ __forceinline__ uint32_t job_word(const JobView &v, uint32_t pos) {
  const int k = pos < v.beg[1] ? 0 : (pos < v.beg[2] ? 1 : 2);
  if (pos + 4 <= span_end(v, k)) return __builtin_bswap32(ld_u32(span_p(v, k) + (pos - span_beg(v, k))));
  if (pos >= v.L + 1) return 0u;
  uint32_t w = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) w = (w << 8) | job_byte(v, pos + q);
  return w;
}
__device__ __forceinline__ void job_block(const JobView &v, uint32_t blk, uint32_t nblk, uint32_t w[16]) {
  const uint32_t s = blk * 64;
#pragma unroll
  for (int k = 0; k < 16; k++) w[k] = job_word(v, s + 4 * k);
  if (blk == nblk - 1) {
    const uint64_t bits = (uint64_t)v.L * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}

// Over-read contract: a message may be read up to 7 bytes past its end (aligned dword loads);
// block arenas carry >= 64 bytes of tail padding.
__device__ __forceinline__ void sha_view(const JobView &v, uint8_t *out) {
  const uint32_t nblk = (v.L + 8) / 64 + 1;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  // a block inside one span is 17 aligned dwords + a byte shift (fetched one block ahead);
  // blocks across a span boundary or holding the padding go word by word
  uint32_t raw[17], sh = 0, w[16];
  bool fast = false;
  auto fetch = [&](uint32_t b) {
    const uint32_t s = b * 64;
    const int k = s < v.beg[1] ? 0 : (s < v.beg[2] ? 1 : 2);
    fast = s + 64 <= span_end(v, k);
    if (fast) {
      // global (not flat) loads: the 17 dwords merge into 4 x dwordx4 + 1 -- a quarter of the
      // per-lane cache-line requests of dword loads, where 64 lanes read 64 scattered messages
      const uintptr_t a = reinterpret_cast<uintptr_t>(span_p(v, k) + (s - span_beg(v, k)));
      const __attribute__((address_space(1))) uint32_t *al =
          reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(a & ~(uintptr_t)3);
      sh = (uint32_t)(a & 3u);
#pragma unroll
      for (int q = 0; q < 17; q++) raw[q] = al[q];
    }
  };
  fetch(0);
#pragma unroll 1
  for (uint32_t blk = 0; blk < nblk; blk++) {
    if (fast) {
#pragma unroll
      for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
    } else {
      job_block(v, blk, nblk, w);
    }
    if (blk + 1 < nblk) fetch(blk + 1);
    sha_compress(h, w);
  }
  uint32_t *o = reinterpret_cast<uint32_t *>(out);
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
}

