// blockdev_sha.hip -- the committer's SHA-256 kernels: k_bd_sha_payload (Envelope.payload,
// the creator signature's digest) and k_bd_sha (every other message of a transaction).  Shared
// helpers: blockdev_dev.h.  Reference: core/common/validation/msgvalidation.go:26-64, 248-320,
// msp/identities.go:179-199 (identity.Verify hashes the message), protoutil/txutils.go:503-534.
#include "sha3_dev.h"
#include "blockdev_dev.h"

// ============================================================ k_bd_sha_payload
// SHA-256(Envelope.payload) of every envelope -- the creator signature's digest
// (msgvalidation.go:26-64 -> msp/identities.go:179), digest slot 0 -- launched on the second
// stream BEFORE the parse: it decodes the Envelope (two fields, the same rules and visitor as
// k_bd_parse) and hashes field 1.  Each payload is its transaction's longest message (~58
// compressions for C2), a serial chain; a batch has far fewer chains (16k) than the chip has
// lanes, so the kernel is bound by ONE chain's latency, not by throughput.  Each chain is
// therefore split over two waves of a workgroup on two SIMDs (64 payloads per workgroup):
//   wave 1 (schedule): loads block b+1 (one block ahead), expands W[0..63] and writes
//                      KW[t] = W[t] + K[t] to LDS (double-buffered, [t/4][lane] x 16 B)
//   wave 0 (rounds):   the 64 rounds of block b from LDS (16 x ds_read_b128)
// one barrier per block.  The rounds wave carries ~950 VALU instructions per compression
// instead of ~1,650 for the whole compression in one lane.
#define PAY_KW_BYTES (2 * 16 * 64 * 16)
__device__ __forceinline__ void pay_view(uint32_t ntx, uint32_t t, const uint32_t *envtab, const uint64_t *bases,
                                         JobView &v, uint32_t &nblk) {
  nblk = 0;
  v.p[0] = v.p[1] = v.p[2] = nullptr;
  v.beg[0] = v.beg[1] = v.beg[2] = v.beg[3] = v.L = 0;
  if (t >= ntx) return;
  const uint32_t *et = envtab + BD_ENV_WORDS * t;
  VTwoBytes env;
  bool ovf = false;
  if (!decode(S{reinterpret_cast<const uint8_t *>(bases[et[0]]) + et[1], et[2]}, env, ovf)) return;
  v.p[0] = v.p[1] = v.p[2] = env.a.p;
  v.beg[1] = v.beg[2] = v.beg[3] = v.L = env.a.n;
  nblk = (v.L + 8) / 64 + 1;
}

__global__ __launch_bounds__(128) void k_bd_sha_payload(uint32_t ntx, const uint32_t *__restrict__ envtab,
                                                        const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                        unsigned long long *__restrict__ nblk_total,
                                                        uint32_t prio) {
  // the longest serial chains of the batch: first in issue order (FGV_PAYLOAD_PRIO)
  if (prio == 3) __builtin_amdgcn_s_setprio(3);
  else __builtin_amdgcn_s_setprio(2);
  __shared__ uint4 KW[2][16][64];  // [buffer][t / 4][lane]: KW[t] = W[t] + K[t] of one block
  const uint32_t lane = threadIdx.x & 63u;
  const bool sched = threadIdx.x >= 64;  // wave-uniform
  const uint32_t t = blockIdx.x * 64 + lane;
  JobView v;
  uint32_t nblk;
  pay_view(ntx, t, envtab, bases, v, nblk);
  uint32_t maxb = nblk;
  for (int off = 32; off > 0; off >>= 1) maxb = max(maxb, (uint32_t)__shfl_xor((int)maxb, off));
  if (sched) {
    // ---- schedule wave: block b's words (fetched one block ahead), expansion, KW to LDS
    uint32_t raw[17], sh = 0;
    bool fast = false;
    auto fetch = [&](uint32_t b) {
      const uint32_t s0 = b * 64;
      const int k = s0 < v.beg[1] ? 0 : (s0 < v.beg[2] ? 1 : 2);
      fast = s0 + 64 <= span_end(v, k);
      if (fast) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(span_p(v, k) + (s0 - span_beg(v, k)));
        const __attribute__((address_space(1))) uint32_t *al =
            reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(a & ~(uintptr_t)3);
        sh = (uint32_t)(a & 3u);
#pragma unroll
        for (int q = 0; q < 17; q++) raw[q] = al[q];
      }
    };
    auto produce = [&](uint32_t b) {
      if (b >= nblk) return;
      uint32_t w[16];
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        job_block(v, b, nblk, w);
      }
      if (b + 1 < nblk) fetch(b + 1);
      uint4 *o = &KW[b & 1][0][lane];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int i = 4 * q + j;
          uint32_t wi;
          if (i < 16) {
            wi = w[i];
          } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
          }
          kw[j] = wi + SHA_K[i];
        }
        o[q * 64] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
      }
    };
    if (nblk) fetch(0);
    produce(0);
    __syncthreads();
#pragma unroll 1
    for (uint32_t b = 0; b < maxb; b++) {
      if (b + 1 < maxb) produce(b + 1);
      __syncthreads();
    }
    return;
  }
  // ---- rounds wave
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  __syncthreads();
#pragma unroll 1
  for (uint32_t b = 0; b < maxb; b++) {
    if (b < nblk) {
      const uint4 *in = &KW[b & 1][0][lane];
      uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint4 x = in[q * 64];
        const uint32_t kw4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
          const uint32_t ch = (e & f) ^ (~e & g);
          const uint32_t t1 = k + S1 + ch + kw4[j];
          const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
          const uint32_t mj = (a & bb) | (c & (a | bb));
          k = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + S0 + mj;
        }
      }
      h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
    }
    __syncthreads();
  }
  if (nblk) {
    uint32_t *o = reinterpret_cast<uint32_t *>(dig + (size_t)t * 32);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
  }
  uint64_t blocks = nblk;
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_total, (unsigned long long)blocks);
}

// ============================================================ k_bd_sha
// Every other SHA-256 message of the batch, hashed speculatively right after the parse on the
// third stream (beside identity resolution and the job counts): all of them are spans the parse
// already found; only WHETHER a digest is consumed is decided later (a hash is pure, so a
// superset of the consumed ones is hashed).  Digest slots (BD_DIG_SLOTS x ntx, slot-major):
//   0                      SHA-256(e.Payload): k_bd_sha_payload (msgvalidation.go:26-64)
//   1 + k (k < BD_MAX_END) SHA-256(prp || endorser_k) (statebased/validator_keylevel.go:246-260)
//   BD_DIG_T               SHA-256(nonce || creator): TxID (protoutil/proputils.go:351-360)
//   BD_DIG_P               SHA-256(chdr || shdr || ccpp): proposal hash (protoutil/txutils.go:449-466)
//   BD_DIG_I               SHA-256(nonce || creator) of the txid index entry (txutils.go:503-534)
// A transaction's endorsement messages share the prefix prp: the SHA-256 state after its H =
// floor(|prp| / 64) whole blocks (the midstate) is the same for all of them.  SHA_GROUP = 3 lanes
// per transaction, 21 transactions per wave:
//   lane 0: prp || endorser_0 in full (its state after block H-1 is the midstate), then the
//           tails (blocks H.. from the midstate) of endorsements 3, 6, ...
//   lane 1: nonce || creator (TxID), then the tails of endorsements 1, 4, ...
//   lane 2: chdr || shdr || ccpp, the index txid message when needed, then the tails 2, 5, ...
// Lanes run in lockstep, one compression per step; at step H every lane of the group copies
// lane 0's state (cross-lane read), so a tail never starts before step H.  For C2 this is ~33
// steps per wave in 750 waves instead of 7 lanes per tx in 1750 -- the prp prefix is hashed once
// instead of once per endorsement, and the waves fit beside the payload hashes on the SIMDs.
#define SHA_GROUP 3u  // lanes per transaction (SHA_GPW groups per wave, blockdev.h; lane 63 idles)
namespace {
// one message (or its tail) of a lane: up to three spans held as scalars (an indexed array of
// span pointers would be placed in scratch)
struct ShaSeg {
  uint64_t a, b, c;    // span addresses
  uint32_t la, lb, lc; // span lengths; message = a || b || c, L = la + lb + lc
  uint32_t b0, nblk;   // blocks [b0, nblk) of the padded message
  uint32_t slot;       // digest slot
  bool mid;            // starts from the midstate (b0 = H)
  bool ok;
};
DEV void seg_set(ShaSeg &g, const uint8_t *base, DSpan x, DSpan y, DSpan z, uint32_t slot) {
  g.a = (uint64_t)(uintptr_t)(base + x.off);
  g.b = (uint64_t)(uintptr_t)(base + y.off);
  g.c = (uint64_t)(uintptr_t)(base + z.off);
  g.la = x.len;
  g.lb = y.len;
  g.lc = z.len;
  g.slot = slot;
  g.ok = true;
}
// segment s of lane r of transaction R (ok = false: the lane's list ended)
DEV ShaSeg lane_seg(const DevTx &R, const uint8_t *base, uint32_t r, uint32_t s, uint32_t H, bool live_t, bool live_p,
                    bool live_i, uint32_t nE) {
  ShaSeg g{};
  const DSpan z{0, 0};
  uint32_t nfull = 0;  // full messages ahead of this lane's tails
  if (r == 0) {
    if (nE > 0) {
      if (s == 0) seg_set(g, base, R.prp, R.end_ser[0], z, 1);
      nfull = 1;
    }
  } else if (r == 1) {
    if (live_t) {
      if (s == 0) seg_set(g, base, R.nonce, R.creator, z, BD_DIG_T);
      nfull = 1;
    }
  } else {
    if (live_p) {
      if (s == nfull) seg_set(g, base, R.chdr, R.act_hdr, R.ccpp, BD_DIG_P);
      nfull++;
    }
    if (live_i) {
      if (s == nfull) seg_set(g, base, R.idx_nonce, R.idx_creator, z, BD_DIG_I);
      nfull++;
    }
  }
  if (!g.ok && s >= nfull) {  // tails: endorsements k = r + 3 j (lane 0 hashed k = 0 in full)
    const uint32_t k = r + SHA_GROUP * (s - nfull + (r == 0 ? 1u : 0u));
    if (k < nE) {
      seg_set(g, base, R.prp, R.end_ser[k], z, 1 + k);
      g.b0 = H;
      g.mid = true;
    }
  }
  if (g.ok) g.nblk = (g.la + g.lb + g.lc + 8) / 64 + 1;
  return g;
}
// choose one of three values by masks (a select chain on a position would be turned into a
// table in scratch indexed by the span number)
DEV uint64_t pick3(bool c0, bool c1, uint64_t x0, uint64_t x1, uint64_t x2) {
  const uint64_t m0 = 0ull - (uint64_t)c0, m1 = (0ull - (uint64_t)c1) & ~m0, m2 = ~(m0 | m1);
  return (x0 & m0) | (x1 & m1) | (x2 & m2);
}
// message byte q (padding: 0x80 at L, zeros after)
DEV uint32_t seg_byte(const ShaSeg &g, uint32_t q) {
  const uint32_t L = g.la + g.lb + g.lc;
  if (q >= L) return q == L ? 0x80u : 0u;
  const bool in_a = q < g.la, in_b = q < g.la + g.lb;
  const uint64_t p = pick3(in_a, in_b, g.a + q, g.b + (q - g.la), g.c + (q - g.la - g.lb));
  return *reinterpret_cast<const uint8_t *>(p);
}
// block `blk` of g: the span holding all 64 bytes (fast: 17 raw dwords + byte shift) or not
DEV void seg_fetch(const ShaSeg &g, uint32_t blk, uint32_t raw[17], uint32_t &sh, bool &fast) {
  const uint32_t s = blk * 64, ab = g.la + g.lb;
  const bool in_a = s + 64 <= g.la, in_b = s >= g.la && s + 64 <= ab;
  fast = in_a || in_b || (s >= ab && s + 64 <= ab + g.lc);
  const uint64_t p = pick3(in_a, in_b, g.a + s, g.b + (s - g.la), g.c + (s - ab));
  if (fast) {
    const __attribute__((address_space(1))) uint32_t *al =
        reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(p & ~(uint64_t)3);
    sh = (uint32_t)(p & 3u);
#pragma unroll
    for (int q = 0; q < 17; q++) raw[q] = al[q];
  }
}
// big-endian message word at byte position pos: one unaligned dword load when the word lies
// inside a span, bytes only when it straddles a span boundary or the end (0x80, then zeros)
DEV uint32_t seg_word(const ShaSeg &g, uint32_t pos) {
  const uint32_t L = g.la + g.lb + g.lc;
  if (pos >= L) return pos == L ? 0x80000000u : 0u;
  const bool in_a = pos < g.la, in_b = pos < g.la + g.lb;
  const uint64_t p = pick3(in_a, in_b, g.a + pos, g.b + (pos - g.la), g.c + (pos - g.la - g.lb));
  const uint32_t room = (uint32_t)pick3(in_a, in_b, g.la - pos, g.la + g.lb - pos, L - pos);
  if (room >= 4) return __builtin_bswap32(ld_u32(reinterpret_cast<const uint8_t *>(p)));
  uint32_t w = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) w = (w << 8) | seg_byte(g, pos + q);
  return w;
}
// a block that is not inside one span (span boundaries, the padding and length)
DEV void seg_block_slow(const ShaSeg &g, uint32_t blk, uint32_t w[16]) {
  const uint32_t s = blk * 64;
#pragma unroll
  for (int k = 0; k < 16; k++) w[k] = seg_word(g, s + 4 * k);
  if (blk == g.nblk - 1) {
    const uint64_t bits = (uint64_t)(g.la + g.lb + g.lc) * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}
}  // namespace

DEV void bd_sha_body(uint32_t ntx, const DevTx *__restrict__ txs, const uint64_t *__restrict__ bases,
                     uint8_t *__restrict__ dig, unsigned long long *__restrict__ nblk_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t grp = lane / SHA_GROUP, r = lane - grp * SHA_GROUP;
  const uint32_t t = blockIdx.x * SHA_GPW + grp;
  const bool in = grp < SHA_GPW && t < ntx;
  uint32_t H = 0, nE = 0;
  bool live_t = false, live_p = false, live_i = false;
  const uint8_t *base = nullptr;
  ShaSeg g;
  g.ok = false;
  if (in) {
    const DevTx &R = txs[t];
    base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
    const bool live = R.pre == C_PENDING;
    live_t = live && R.type == 3;
    live_p = live_t && R.etx == C_VALID;
    live_i = (R.flags & BDF_INDEX_OK) && !(R.flags & BDF_INDEX_FROM_TXID);
    nE = (live_p && R.disp == C_VALID) ? R.nend : 0u;
    H = R.prp.len / 64;
    g = lane_seg(R, base, r, 0, H, live_t, live_p, live_i, nE);
  }
  uint32_t s = 0, blk = g.ok ? g.b0 : 0;
  uint32_t h[8], mid[8];
  const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = mid[k] = IV[k];
  uint64_t blocks = 0;
  uint32_t raw[17], sh = 0, w[16];
  bool fast = false;
  if (g.ok) seg_fetch(g, blk, raw, sh, fast);
  const int src = (int)(grp * SHA_GROUP);  // lane 0 of the group
#pragma unroll 1
  for (uint32_t step = 0;; step++) {
    // the midstate: lane 0's state after its first H blocks (every lane runs the reads)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (uint32_t)__shfl((int)h[k], src);
      if (step == H) mid[k] = v;
    }
    const bool waiting = g.ok && g.mid && step < H;
    if (__ballot(g.ok) == 0ull) break;
    if (g.ok && !waiting) {
      if (blk == g.b0 && g.mid) {
#pragma unroll
        for (int k = 0; k < 8; k++) h[k] = mid[k];
      }
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        seg_block_slow(g, blk, w);
      }
      // the lane's next block (or the next segment's first), fetched while this one compresses
      ShaSeg gn = g;
      uint32_t bn = blk + 1;
      bool next_seg = bn >= g.nblk;
      if (next_seg) {
        gn = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        bn = gn.ok ? gn.b0 : 0;
      }
      if (gn.ok) seg_fetch(gn, bn, raw, sh, fast);
      sha_compress(h, w);
      blocks++;
      if (next_seg) {
        uint32_t *o = reinterpret_cast<uint32_t *>(dig + ((size_t)g.slot * ntx + t) * 32);
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
        g = gn;
        s++;
        if (g.ok && !g.mid) {  // (a tail takes the midstate at its first block)
#pragma unroll
          for (int k = 0; k < 8; k++) h[k] = IV[k];
        }
      }
      blk = bn;
    }
  }
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_out, (unsigned long long)blocks);
}
// ---- the same hashes, each lane's chain split over two waves of a workgroup on two SIMDs
// (k_bd_sha_payload's scheme): wave 1 (schedule) walks the lanes' segments exactly as
// bd_sha_body does, fetches each step's block one step ahead, expands the message schedule and
// writes KW[t] = W[t] + K[t] to LDS (double-buffered, [t/4][lane] x 16 B); wave 0 (rounds) runs
// the 64 rounds from LDS, takes the midstate, writes the digests.  One barrier per step; both
// waves run the same number of steps: a lane's last step is max(full blocks, H) + tail blocks.
DEV uint32_t lane_steps(const DevTx &R, const uint8_t *base, uint32_t r, uint32_t H, bool live_t, bool live_p,
                        bool live_i, uint32_t nE) {
  uint32_t pos = 0;
  for (uint32_t s = 0;; s++) {
    const ShaSeg g = lane_seg(R, base, r, s, H, live_t, live_p, live_i, nE);
    if (!g.ok) return pos;
    if (g.mid && pos < H) pos = H;
    pos += g.nblk - g.b0;
  }
}

DEV void bd_sha_split_body(uint32_t ntx, const DevTx *__restrict__ txs, const uint64_t *__restrict__ bases,
                           uint8_t *__restrict__ dig, unsigned long long *__restrict__ nblk_out) {
  __shared__ uint4 KW[2][16][64];  // [buffer][t / 4][lane]
  const uint32_t lane = threadIdx.x & 63u;
  const bool sched = threadIdx.x >= 64;  // wave-uniform
  const uint32_t grp = lane / SHA_GROUP, r = lane - grp * SHA_GROUP;
  const uint32_t t = blockIdx.x * SHA_GPW + grp;
  const bool in = grp < SHA_GPW && t < ntx;
  uint32_t H = 0, nE = 0, nsteps = 0;
  bool live_t = false, live_p = false, live_i = false;
  const uint8_t *base = nullptr;
  ShaSeg g;
  g.ok = false;
  if (in) {
    const DevTx &R = txs[t];
    base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
    const bool live = R.pre == C_PENDING;
    live_t = live && R.type == 3;
    live_p = live_t && R.etx == C_VALID;
    live_i = (R.flags & BDF_INDEX_OK) && !(R.flags & BDF_INDEX_FROM_TXID);
    nE = (live_p && R.disp == C_VALID) ? R.nend : 0u;
    H = R.prp.len / 64;
    g = lane_seg(R, base, r, 0, H, live_t, live_p, live_i, nE);
    nsteps = lane_steps(R, base, r, H, live_t, live_p, live_i, nE);
  }
  uint32_t maxs = nsteps;
  for (int off = 32; off > 0; off >>= 1) maxs = max(maxs, (uint32_t)__shfl_xor((int)maxs, off));
  uint32_t s = 0, blk = g.ok ? g.b0 : 0;
  if (sched) {
    // ---- schedule wave
    uint32_t raw[17], sh = 0;
    bool fast = false;
    if (g.ok) seg_fetch(g, blk, raw, sh, fast);
    auto produce = [&](uint32_t step) {
      if (!g.ok || (g.mid && step < H)) return;
      uint32_t w[16];
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        seg_block_slow(g, blk, w);
      }
      ShaSeg gn = g;
      uint32_t bn = blk + 1;
      if (bn >= g.nblk) {
        gn = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        bn = gn.ok ? gn.b0 : 0;
        s++;
      }
      if (gn.ok) seg_fetch(gn, bn, raw, sh, fast);
      g = gn;
      blk = bn;
      uint4 *o = &KW[step & 1][0][lane];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int i = 4 * q + j;
          uint32_t wi;
          if (i < 16) {
            wi = w[i];
          } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
          }
          kw[j] = wi + SHA_K[i];
        }
        o[q * 64] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
      }
    };
    if (maxs) produce(0);
    __syncthreads();
#pragma unroll 1
    for (uint32_t step = 0; step < maxs; step++) {
      if (step + 1 < maxs) produce(step + 1);
      __syncthreads();
    }
    return;
  }
  // ---- rounds wave
  const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t h[8], mid[8];
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = mid[k] = IV[k];
  uint64_t blocks = 0;
  const int src = (int)(grp * SHA_GROUP);  // lane 0 of the group
  __syncthreads();
#pragma unroll 1
  for (uint32_t step = 0; step < maxs; step++) {
    // the midstate: lane 0's state after its first H blocks (every lane runs the reads)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (uint32_t)__shfl((int)h[k], src);
      if (step == H) mid[k] = v;
    }
    if (g.ok && !(g.mid && step < H)) {
      if (blk == g.b0 && g.mid) {
#pragma unroll
        for (int k = 0; k < 8; k++) h[k] = mid[k];
      }
      const uint4 *in4 = &KW[step & 1][0][lane];
      uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], gg = h[6], k = h[7];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint4 x = in4[q * 64];
        const uint32_t kw4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
          const uint32_t ch = (e & f) ^ (~e & gg);
          const uint32_t t1 = k + S1 + ch + kw4[j];
          const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
          const uint32_t mj = (a & bb) | (c & (a | bb));
          k = gg; gg = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + S0 + mj;
        }
      }
      h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += gg; h[7] += k;
      blocks++;
      uint32_t bn = blk + 1;
      if (bn >= g.nblk) {
        uint32_t *o = reinterpret_cast<uint32_t *>(dig + ((size_t)g.slot * ntx + t) * 32);
#pragma unroll
        for (int q = 0; q < 8; q++) o[q] = __builtin_bswap32(h[q]);
        g = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        s++;
        bn = g.ok ? g.b0 : 0;
        if (g.ok && !g.mid) {  // (a tail takes the midstate at its first block)
#pragma unroll
          for (int q = 0; q < 8; q++) h[q] = IV[q];
        }
      }
      blk = bn;
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_out, (unsigned long long)blocks);
}
__global__ __launch_bounds__(128) void k_bd_sha2(uint32_t ntx, const DevTx *__restrict__ txs,
                                                 const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                 unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(1);
  bd_sha_split_body(ntx, txs, bases, dig, nblk_out);
}

// k_prep waits for these digests and for the parse -> identities -> counts -> emit -> der ->
// inv chain: the wave priority decides which of the two finishes first (FGV_SHA_PRIO A/B)
__global__ __launch_bounds__(64) void k_bd_sha(uint32_t ntx, const DevTx *__restrict__ txs,
                                               const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                               unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(1);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}
__global__ __launch_bounds__(64) void k_bd_sha_p2(uint32_t ntx, const DevTx *__restrict__ txs,
                                                  const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                  unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(2);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}
__global__ __launch_bounds__(64) void k_bd_sha_p3(uint32_t ntx, const DevTx *__restrict__ txs,
                                                  const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                  unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(3);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}

// SHA3 MSPs (identities.go:170-199, getHashOpt :219-227): once the identities are resolved
// (after k_bd_count), the creator digest (slot 0) and each endorsement digest (slot 1 + k) of an
// identity whose MSP hashes with SHA3 are replaced by SHA3-256 of the same message.  One lane
// per transaction; launched only for a channel that has such identities.
__global__ __launch_bounds__(64) void k_bd_sha3(uint32_t ntx, const DevTx *__restrict__ txs,
                                                const uint64_t *__restrict__ bases, DevChannel ch,
                                                const int32_t *__restrict__ ident, uint8_t *__restrict__ dig) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const DevTx &R = txs[t];
  const int32_t *id = ident + (size_t)t * BD_OCC;
  const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
  const int32_t ci = id[0];
  if (ci >= 0 && ch.idents[ci].hash3) {  // Envelope.payload
    const uint8_t *const p[3] = {base + R.payload.off, base, base};
    const uint32_t n[3] = {R.payload.len, 0u, 0u};
    fgvsha3::sha3_256_spans(p, n, dig + (size_t)t * 32);
  }
  for (uint32_t k = 0; k < R.nend && k < BD_MAX_END; k++) {  // prp || endorser
    const int32_t e = id[1 + k];
    if (e < 0 || !ch.idents[e].hash3) continue;
    const uint8_t *const p[3] = {base + R.prp.off, base + R.end_ser[k].off, base};
    const uint32_t n[3] = {R.prp.len, R.end_ser[k].len, 0u};
    fgvsha3::sha3_256_spans(p, n, dig + ((size_t)(1 + k) * ntx + t) * 32);
  }
}
