// sha256.hip -- batched SHA-256 for gfx950: one message per lane, messages read in place
// from a byte arena (envelope bytes resident in HBM; no gather copy).
// Replaces bccsp/sw/hash.go:29-33 (Go crypto/sha256) for identity.Verify digests
// (msp/identities.go:179) and the TxID / proposal-hash checks (protoutil/proputils.go:354,
// protoutil/txutils.go:458).  Integer VALU only: ~2.7k 32-bit ops per 64-byte block.
#include "fgv_kernels.h"

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

__device__ __forceinline__ void sha_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = k + S1 + ch + SHA_K[i] + wi;
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) | (c & (a | b));
    uint32_t t2 = S0 + mj;
    k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// Arena contract: every message may be over-read by up to 3 bytes past its end for the
// aligned fast path; the host pads the arena by >= 64 bytes.
__global__ __launch_bounds__(256) void k_sha256(const uint8_t *__restrict__ buf,
                                                const uint64_t *__restrict__ off,
                                                const uint32_t *__restrict__ len, uint32_t n,
                                                uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *msg = buf + off[i];
  const uint32_t L = len[i];
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t nfull = L >> 6;
  const uintptr_t base = reinterpret_cast<uintptr_t>(msg);
  const uint32_t *aligned = reinterpret_cast<const uint32_t *>(base & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(base & 3) * 8;
  uint32_t w[16];
#pragma unroll 1
  for (uint32_t blk = 0; blk < nfull; blk++) {
    const uint32_t *p = aligned + blk * 16;
    uint32_t cur = p[0];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t nxt = p[j + 1];
      // bytes at msg+64*blk+4j .. +3, little-endian load -> big-endian word
      uint32_t v = sh ? __builtin_amdgcn_alignbyte(nxt, cur, sh >> 3) : cur;
      w[j] = __builtin_bswap32(v);
      cur = nxt;
    }
    sha_compress(h, w);
  }
  // tail: remaining bytes + 0x80 + zero pad + 64-bit bit length (1 or 2 blocks)
  const uint32_t rem = L & 63;
  const uint32_t ntail = (rem + 9 <= 64) ? 1 : 2;
  const uint8_t *tp = msg + (size_t)nfull * 64;
  const uint64_t bits = (uint64_t)L * 8;
#pragma unroll 1
  for (uint32_t t = 0; t < ntail; t++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t word = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t pos = t * 64 + j * 4 + q;
        uint32_t byte = pos < rem ? tp[pos] : (pos == rem ? 0x80u : 0u);
        word = (word << 8) | byte;
      }
      w[j] = word;
    }
    if (t == ntail - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha_compress(h, w);
  }
  uint32_t *o = reinterpret_cast<uint32_t *>(out + (size_t)i * 32);
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = __builtin_bswap32(h[j]);
}

// ---------------------------------------------------------------------------------
// k_sha256_jobs: messages that are the concatenation of up to 3 spans, each given by an
// absolute device address (spans point straight into block bytes resident in HBM):
//   creator payload (1 span), nonce||creator (TxID, protoutil/proputils.go:351-360),
//   chdr||shdr||ccpp (proposal hash, protoutil/txutils.go:449-466),
//   prp||endorser (endorsement message, statebased/validator_keylevel.go:246-260).
// 64-byte blocks lying inside one span use the aligned dword path; blocks that straddle a
// span boundary or hold the padding are assembled byte by byte.
__device__ __forceinline__ uint32_t job_byte(const ShaJob &j, uint32_t q) {
  if (q < j.n[0]) return reinterpret_cast<const uint8_t *>(j.p[0])[q];
  q -= j.n[0];
  if (q < j.n[1]) return reinterpret_cast<const uint8_t *>(j.p[1])[q];
  q -= j.n[1];
  return reinterpret_cast<const uint8_t *>(j.p[2])[q];
}

__global__ __launch_bounds__(256) void k_sha256_jobs(const ShaJob *__restrict__ jobs, uint32_t n,
                                                     uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ShaJob j = jobs[i];
  const uint32_t L = j.n[0] + j.n[1] + j.n[2];
  const uint32_t nblk = (L + 8) / 64 + 1;
  const uint64_t bits = (uint64_t)L * 8;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t w[16];
  uint32_t cum0 = j.n[0], cum1 = j.n[0] + j.n[1];
#pragma unroll 1
  for (uint32_t blk = 0; blk < nblk; blk++) {
    const uint32_t s = blk * 64, e = s + 64;
    int span = -1;
    uint32_t base = 0;
    if (e <= cum0) { span = 0; base = 0; }
    else if (s >= cum0 && e <= cum1) { span = 1; base = cum0; }
    else if (s >= cum1 && e <= L) { span = 2; base = cum1; }
    if (span >= 0) {
      const uint8_t *msg = reinterpret_cast<const uint8_t *>(j.p[span]) + (s - base);
      const uintptr_t a = reinterpret_cast<uintptr_t>(msg);
      const uint32_t *al = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(a & 3);
      uint32_t cur = al[0];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        uint32_t nxt = (sh || k < 15) ? al[k + 1] : 0u;  // aligned & last word: no over-read
        uint32_t v = sh ? __builtin_amdgcn_alignbyte(nxt, cur, sh) : cur;
        w[k] = __builtin_bswap32(v);
        cur = nxt;
      }
    } else {
#pragma unroll 1
      for (int k = 0; k < 16; k++) {
        uint32_t word = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t pos = s + k * 4 + q;
          const uint32_t byte = pos < L ? job_byte(j, pos) : (pos == L ? 0x80u : 0u);
          word = (word << 8) | byte;
        }
        w[k] = word;
      }
      if (blk == nblk - 1) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
      }
    }
    sha_compress(h, w);
  }
  uint32_t *o = reinterpret_cast<uint32_t *>(out + (size_t)i * 32);
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
}
