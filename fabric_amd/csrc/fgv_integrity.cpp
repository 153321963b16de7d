// fgv_integrity.cpp -- deliver-side block integrity for the committer's input
// (BlockVerificationAssistant.VerifyBlock, common/deliverclient/block_verification.go:243-273):
//   verifyHeader    :311-331  header present; number == last + 1; PreviousHash == SHA-256 of
//                             the last verified header's ASN.1 bytes (when that hash is known)
//   verifyMetadata  :303-309  at least len(BlockMetadataIndex_name) = 5 metadata entries
//   BlockDataHash   protoutil/blockutils.go:69-74 -> VerifyTransactionsAreWellFormed
//                   (:310-350) then ComputeBlockDataHash (:76-79) = SHA-256(concat(Data))
//   DataHash compare :258-263
//   sigVerifierFunc :265-268  (fgv_blocks_verify_signed only) the orderer signatures against the
//                             channel's BlockValidation policy, fgv_block_sig_verdicts in
//                             fgv_block.cpp (GPU verify + the channel model's policy fold)
// and on success the chain state advances to BlockHeaderHash (blockutils.go:48-67: SHA-256
// of DER SEQUENCE{INTEGER number, OCTET STRING previous_hash, OCTET STRING data_hash}).
//
// Placement: the data hash is one sequential SHA-256 chain per block, so blocks
// hash in parallel on host cores with the SHA extensions, one block per thread.
#include <immintrin.h>

#include <atomic>
#include <vector>

#include "fgv_internal.h"
#include "fgv_visitors.h"
#include "pbwire.h"
#include "sha256_host.h"
#include "thread_pool.h"

namespace fgvsha {

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void compress_scalar(uint32_t st[8], const uint8_t *p, size_t nblk) {
  for (; nblk--; p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) |
             p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
      const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
  }
}

// The SHA extensions keep the state as two registers ABEF / CDGH; every 4 rounds consume one
// 128-bit message-schedule word group W[4g..4g+3] (+K), and groups 4..15 are produced by
// msg1 (W[t-16] + s0(W[t-15])), + W[t-7] (alignr of the two previous groups), msg2 (+ s1).
__attribute__((target("sha,sse4.1,ssse3"))) void compress_ni(uint32_t st[8], const uint8_t *p, size_t nblk) {
  const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st));       // A B C D
  __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(st + 4));  // E F G H
  t = _mm_shuffle_epi32(t, 0xB1);                                           // B A D C
  s1 = _mm_shuffle_epi32(s1, 0x1B);                                         // H G F E
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                   // ABEF
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                        // CDGH
  for (; nblk--; p += 64) {
    const __m128i save0 = s0, save1 = s1;
    __m128i m[4];
#pragma unroll
    for (int g = 0; g < 16; g++) {
      __m128i &cur = m[g & 3];
      if (g < 4) {
        cur = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * g)), BSWAP);
      } else {
        const __m128i prev = m[(g + 3) & 3], prev2 = m[(g + 2) & 3];
        cur = _mm_sha256msg1_epu32(cur, m[(g + 1) & 3]);
        cur = _mm_add_epi32(cur, _mm_alignr_epi8(prev, prev2, 4));
        cur = _mm_sha256msg2_epu32(cur, prev);
      }
      __m128i msg = _mm_add_epi32(cur, _mm_loadu_si128(reinterpret_cast<const __m128i *>(K256 + 4 * g)));
      s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
    }
    s0 = _mm_add_epi32(s0, save0);
    s1 = _mm_add_epi32(s1, save1);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);     // F E B A
  s1 = _mm_shuffle_epi32(s1, 0xB1);    // D C H G
  s0 = _mm_blend_epi16(t, s1, 0xF0);   // D C B A
  s1 = _mm_alignr_epi8(s1, t, 8);      // H G F E
  _mm_storeu_si128(reinterpret_cast<__m128i *>(st), s0);
  _mm_storeu_si128(reinterpret_cast<__m128i *>(st + 4), s1);
}

bool have_sha_ni() {
  static const bool v = [] {
    unsigned a, b, c, d;
    __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    const bool sha = (b >> 29) & 1;
    __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(1), "c"(0));
    const bool sse41 = (c >> 19) & 1, ssse3 = (c >> 9) & 1;
    return sha && sse41 && ssse3 && getenv("FGV_NO_SHA_NI") == nullptr;
  }();
  return v;
}

}  // namespace fgvsha

namespace {

using pbw::Span;

// common.Block with the fields VerifyBlock reads (merge semantics of protobuf-go: a repeated
// singular message field decodes every occurrence into the same value)
struct VHdrFields {  // BlockHeader {number = 1, previous_hash = 2, data_hash = 3}
  uint64_t number = 0;
  Span prev, data_hash;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_VARINT : (n == 2 || n == 3) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { number = v; }
  bool on_len(uint32_t n, Span s) { (n == 2 ? prev : data_hash) = s; return true; }
};
struct VMetaCount {  // BlockMetadata {repeated bytes metadata = 1}: count + metadata[SIGNATURES]
  size_t n = 0;
  Span sigs;
  pbw::Kind kind(uint32_t k) { return k == 1 ? pbw::K_REP_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    if (n++ == 0) sigs = s;
    return true;
  }
};
struct VBlockAll {
  bool has_header = false, has_data = false, has_meta = false;
  VHdrFields hdr;
  fgvb::VBlockData data;
  VMetaCount meta;
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { has_header = true; return pbw::decode(s.p, s.n, hdr); }
    if (n == 2) { has_data = true; return pbw::decode(s.p, s.n, data); }
    has_meta = true;
    return pbw::decode(s.p, s.n, meta);
  }
};

// varint of minimal length? (proto.Marshal always emits the minimal form)
static bool rd_min_varint(const uint8_t *&p, const uint8_t *e, uint64_t &v) {
  const uint8_t *s = p;
  if (!pbw::rd_varint(p, e, v)) return false;
  const size_t used = (size_t)(p - s);
  size_t need = 1;
  for (uint64_t x = v; x >= 0x80; x >>= 7) need++;
  return used == need;
}

// VerifyTransactionsAreWellFormed for one envelope (blockutils.go:321-346): proto.Unmarshal
// succeeds, Payload and Signature non-empty, and proto.Marshal(env) reproduces the raw bytes.
// protobuf-go marshals known fields in field order (payload, signature; minimal tag and length
// encodings; empty bytes omitted), then the unknown fields verbatim in their original order.
// So the raw bytes must be: one field-1 record, one field-2 record, then only unknown records
// (a field 1/2 record with another wire type is unknown to the decoder and kept as such).
static bool envelope_well_formed(Span raw) {
  fgvb::VEnvelope env;
  if (!pbw::decode(raw.p, raw.n, env)) return false;           // "is invalid"
  if (env.payload.n == 0 || env.signature.n == 0) return false;  // "no payload" / "no signature"
  const uint8_t *p = raw.p, *e = raw.p + raw.n;
  for (uint32_t want = 1; want <= 2; want++) {  // the two known records, in order
    if (p >= e || *p != (uint8_t)(want << 3 | 2)) return false;
    p++;
    uint64_t l;
    if (!rd_min_varint(p, e, l) || l > (uint64_t)(e - p)) return false;
    const Span &v = want == 1 ? env.payload : env.signature;
    if (p != v.p || l != v.n) return false;  // a later occurrence won: Marshal emits that one only
    p += l;
  }
  while (p < e) {  // unknown records only (decode already validated their wire format)
    uint64_t tag;
    if (!pbw::rd_varint(p, e, tag)) return false;
    const uint64_t num = tag >> 3;
    const int wt = (int)(tag & 7);
    if ((num == 1 || num == 2) && wt == 2) return false;
    if (!pbw::skip_value(p, e, (uint32_t)num, wt)) return false;
  }
  return true;
}

// HasConfigTx (protoutil/commonutils.go:198-230): exactly one envelope whose channel header
// decodes with type CONFIG
static bool has_config_tx(const std::vector<Span> &data) {
  if (data.size() != 1) return false;
  fgvb::VEnvelope env;
  if (!pbw::decode(data[0].p, data[0].n, env)) return false;
  fgvb::VPayload pl;
  if (!pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.present) return false;
  fgvb::VHeader hdr;
  if (!pl.header.decode_into(hdr)) return false;
  fgvb::VChannelHeader ch;
  if (!pbw::decode(hdr.channel_header.p, hdr.channel_header.n, ch)) return false;
  return ch.type == 1;
}

static size_t der_len(uint8_t *o, size_t n) {
  if (n < 128) { o[0] = (uint8_t)n; return 1; }
  uint8_t tmp[8];
  size_t k = 0;
  for (size_t x = n; x; x >>= 8) tmp[k++] = (uint8_t)x;
  o[0] = (uint8_t)(0x80 | k);
  for (size_t i = 0; i < k; i++) o[1 + i] = tmp[k - 1 - i];
  return 1 + k;
}

}  // namespace

// BlockHeaderBytes (protoutil/blockutils.go:48-67): asn1.Marshal of {Number *big.Int,
// PreviousHash, DataHash []byte} -- DER SEQUENCE{INTEGER, OCTET STRING, OCTET STRING}
void fgv_block_header_der(uint64_t number, const uint8_t *prev, size_t prev_n, const uint8_t *dh, size_t dh_n,
                          std::vector<uint8_t> &out) {
  uint8_t integer[10];
  size_t in = 0;
  {  // minimal two's-complement big-endian, positive
    uint8_t be[8];
    for (int i = 0; i < 8; i++) be[i] = (uint8_t)(number >> (56 - 8 * i));
    int s = 0;
    while (s < 7 && be[s] == 0) s++;
    if (be[s] & 0x80) integer[in++] = 0;
    for (int i = s; i < 8; i++) integer[in++] = be[i];
  }
  std::vector<uint8_t> body;
  body.reserve(32 + prev_n + dh_n);
  uint8_t l[9];
  body.push_back(0x02);
  body.insert(body.end(), l, l + der_len(l, in));
  body.insert(body.end(), integer, integer + in);
  body.push_back(0x04);
  body.insert(body.end(), l, l + der_len(l, prev_n));
  if (prev_n) body.insert(body.end(), prev, prev + prev_n);
  body.push_back(0x04);
  body.insert(body.end(), l, l + der_len(l, dh_n));
  if (dh_n) body.insert(body.end(), dh, dh + dh_n);
  out.clear();
  out.reserve(body.size() + 10);
  out.push_back(0x30);
  out.insert(out.end(), l, l + der_len(l, body.size()));
  out.insert(out.end(), body.begin(), body.end());
}

void fgv_block_header_hash(uint64_t number, const uint8_t *prev, size_t prev_n, const uint8_t *dh, size_t dh_n,
                           uint8_t out[32]) {
  std::vector<uint8_t> der;
  fgv_block_header_der(number, prev, prev_n, dh, dh_n, der);
  fgvsha::sha256(der.data(), der.size(), out);
}

// sig: evaluate the orderer signatures (fgv_blocks_verify_signed) after the data hash, as
// VerifyBlock does (block_verification.go:265-268)
static int verify_impl(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                       fgv_chain_state *chain, fgv_block_check *out, bool sig, const char *policy, int bft) {
  if (!out || (nblocks && (!blocks || !lens))) return FGV_EINVAL;  // ctx NULL: one host thread
  if (sig && !ctx) return FGV_EINVAL;
  struct Pre {
    VBlockAll b;
    bool parsed = false;
  };
  std::vector<Pre> pre(nblocks);
  // independent per-block work (decode, well-formedness, data hash, header hash) in parallel
  auto work = [&](size_t i) {
    fgv_block_check &o = out[i];
    memset(&o, 0, sizeof o);
    o.bad_tx = UINT32_MAX;
    Pre &P = pre[i];
    P.parsed = pbw::decode(blocks[i], lens[i], P.b);
    if (!P.parsed) { o.status = FGV_BLK_UNPARSABLE; return; }
    const VBlockAll &B = P.b;
    o.number = B.hdr.number;
    if (B.has_header) fgv_block_header_hash(B.hdr.number, B.hdr.prev.p, B.hdr.prev.n, B.hdr.data_hash.p,
                                            B.hdr.data_hash.n, o.header_hash);
    const std::vector<Span> &d = B.data.data;
    if (!B.has_data || d.empty()) {
      o.status = FGV_BLK_EMPTY;
    } else if (!has_config_tx(d)) {
      for (size_t k = 0; k < d.size(); k++)
        if (!envelope_well_formed(d[k])) {
          o.status = FGV_BLK_TX_MALFORMED;
          o.bad_tx = (uint32_t)k;
          break;
        }
    }
    if (B.has_data) {
      fgvsha::Stream s;
      for (const Span &x : d) s.update(x.p, x.n);
      s.final(o.data_hash);
    }
  };
  if (ctx) {
    // one block per job (each hash chain is sequential) on a pool of its own: concurrent calls
    // (a deliver service verifying the next batches while the committer validates this one) each
    // take a free pool instead of queueing behind one another
    ThreadPool *pool = nullptr;
    {
      std::lock_guard<std::mutex> lk(ctx->integ_mu);
      if (!ctx->integ_free.empty()) {
        pool = ctx->integ_free.back();
        ctx->integ_free.pop_back();
      }
    }
    if (!pool) {
      const char *e = getenv("FGV_HASH_THREADS");
      const int n = e ? atoi(e) : 8;
      pool = new ThreadPool(n > 0 ? (unsigned)n : 1u);
    }
    pool->run(nblocks, work);
    std::lock_guard<std::mutex> lk(ctx->integ_mu);
    ctx->integ_free.push_back(pool);
  } else {
    for (size_t i = 0; i < nblocks; i++) work(i);
  }

  // orderer-signature verdicts of every block that can reach the signature check (speculative:
  // the chain checks come below; verdicts are pure functions of the block and the channel model)
  std::vector<uint8_t> verdict;
  if (sig) {
    std::vector<fgv_sig_block> in(nblocks);
    for (size_t i = 0; i < nblocks; i++) {
      const VBlockAll &B = pre[i].b;
      if (out[i].status != FGV_BLK_OK || !B.has_header || !B.has_meta || B.meta.n < 5) continue;
      if (B.hdr.data_hash.n != 32 || memcmp(B.hdr.data_hash.p, out[i].data_hash, 32) != 0) continue;
      in[i].want = true;
      in[i].meta = B.meta.sigs.p;
      in[i].meta_n = B.meta.sigs.n;
      fgv_block_header_der(B.hdr.number, B.hdr.prev.p, B.hdr.prev.n, B.hdr.data_hash.p, B.hdr.data_hash.n,
                           in[i].hdr_der);
    }
    verdict.assign(nblocks, FGV_SIGV_FAIL);
    const int rc = fgv_block_sig_verdicts(ctx, nblocks, in.data(), policy, bft, verdict.data());
    if (rc) return rc;
  }

  // sequential chain checks in the reference's order; only a verified block advances it
  for (size_t i = 0; i < nblocks; i++) {
    fgv_block_check &o = out[i];
    if (o.status == FGV_BLK_UNPARSABLE) continue;
    const VBlockAll &B = pre[i].b;
    const int32_t body = o.status;  // EMPTY / TX_MALFORMED / 0, decided above
    if (!B.has_header) { o.status = FGV_BLK_NO_HEADER; continue; }
    if (chain && chain->valid) {
      if (B.hdr.number != chain->number + 1) { o.status = FGV_BLK_NUMBER; continue; }
      if (chain->has_hash && (B.hdr.prev.n != 32 || memcmp(B.hdr.prev.p, chain->header_hash, 32) != 0)) {
        o.status = FGV_BLK_PREV_HASH;
        continue;
      }
    }
    if (!B.has_meta || B.meta.n < 5) { o.status = FGV_BLK_METADATA; continue; }
    if (body) { o.status = body; continue; }
    if (B.hdr.data_hash.n != 32 || memcmp(B.hdr.data_hash.p, o.data_hash, 32) != 0) {
      o.status = FGV_BLK_DATA_HASH;
      continue;
    }
    if (sig && verdict[i] != FGV_SIGV_OK) {
      if (verdict[i] == FGV_SIGV_FAIL) {
        o.status = FGV_BLK_SIGNATURES;
        continue;
      }
      // outside the model: the reference decides this block, and with it the chain from here on
      for (size_t k = i; k < nblocks; k++) out[k].status = FGV_BLK_SIG_UNSUPPORTED;
      return FGV_EUNSUPPORTED;
    }
    o.status = FGV_BLK_OK;
    if (chain) {
      chain->valid = 1;
      chain->number = B.hdr.number;
      chain->has_hash = 1;
      memcpy(chain->header_hash, o.header_hash, 32);
    }
  }
  return FGV_OK;
}

extern "C" int fgv_blocks_verify(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                 fgv_chain_state *chain, fgv_block_check *out) {
  return verify_impl(ctx, nblocks, blocks, lens, chain, out, false, nullptr, 0);
}

extern "C" int fgv_blocks_verify_signed(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                                        const size_t *lens, fgv_chain_state *chain, const char *policy, int bft,
                                        fgv_block_check *out) {
  return verify_impl(ctx, nblocks, blocks, lens, chain, out, true, policy, bft);
}

void fgv_integrity_free(fgv_ctx *c) {
  for (ThreadPool *p : c->integ_free) delete p;
  c->integ_free.clear();
}

extern "C" int fgv_sha256_host(const uint8_t *buf, size_t n, uint8_t out[32]) {
  if (!out || (n && !buf)) return FGV_EINVAL;
  fgvsha::sha256(buf, n, out);
  return fgvsha::have_sha_ni() ? 1 : 0;
}
