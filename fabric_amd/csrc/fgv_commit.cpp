// fgv_commit.cpp -- the ledger's block commit hash (libfgv.so, host C++).
//
// kvLedger.addBlockCommitHash (core/ledger/kvledger/kv_ledger.go:806-817) chains every block's
// TRANSACTIONS_FILTER and update batch into a 32-byte commit hash -- the value that turns one
// wrong validation flag into a visible fork.  The update batch bytes are
// deterministicBytesForPubAndHashUpdates (txmgr/update_batch_bytes.go:29-105): the public and
// hashed (private-data) puts and deletes of the block's VALID endorser transactions at
// Height{block, tx} (validation/types.go:81-112, tx_ops.go:17-51; a later transaction's write of
// a key replaces an earlier one), namespaces sorted with "" (channel config) skipped, keys sorted,
// collections sorted, as txmgr.Updates{KVWrite{namespace, collection, key, isDelete, value,
// version_bytes}} (txmgr/updates.proto).  A serial SHA-256 over one short message per block: host
// code (SHA extensions when present), like the block data hash in fgv_integrity.cpp.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_visitors.h"
#include "sha256_host.h"
#include "thread_pool.h"

using namespace fgvb;

namespace {

// One put or delete of a VALID transaction, spans into the block.  The update batch is the
// block's writes sorted by (namespace, public before hashed, collection, key), the last
// transaction's write of a key replacing the earlier ones (tx_ops.go:17-51).
struct WEnt {
  Span ns, coll, key, value;  // value: the put's value (public) or value hash (hashed)
  uint32_t tx;
  bool hashed, del;
};

inline int span_cmp(const Span &a, const Span &b) {  // std::string / Go sort.Strings order (bytewise)
  const size_t m = a.n < b.n ? a.n : b.n;
  const int c = m ? memcmp(a.p, b.p, m) : 0;
  return c ? c : (a.n < b.n ? -1 : a.n > b.n ? 1 : 0);
}
inline bool span_eq(const Span &a, const Span &b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }
inline bool same_key(const WEnt &a, const WEnt &b) {
  return a.hashed == b.hashed && span_eq(a.key, b.key) && span_eq(a.ns, b.ns) && span_eq(a.coll, b.coll);
}

inline size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) v >>= 7, n++;
  return n;
}
inline uint8_t *put_varint(uint8_t *o, uint64_t v) {
  while (v >= 0x80) {
    *o++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *o++ = (uint8_t)v;
  return o;
}
inline size_t field_len(size_t n) { return 1 + varint_len(n) + n; }  // (field numbers < 16: one tag byte)
inline uint8_t *put_bytes(uint8_t *o, uint32_t field, const uint8_t *p, size_t n) {
  *o++ = (uint8_t)(field << 3 | 2);
  o = put_varint(o, n);
  if (n) memcpy(o, p, n);
  return o + n;
}
// common/ledger/util/util.go:32-52 EncodeOrderPreservingVarUint64
inline size_t opv(uint8_t *o, uint64_t n) {
  int i = 0;
  while (i < 8 && ((n >> (56 - 8 * i)) & 0xFF) == 0) i++;
  size_t k = 0;
  o[k++] = (uint8_t)(8 - i);
  for (; i < 8; i++) o[k++] = (uint8_t)(n >> (56 - 8 * i));
  return k;
}

// txmgr.Updates.KVWrite{namespace 1 (on the first write of a namespace), collection 2 (on the
// first write of a collection), key 3, is_delete 4, value 5, version_bytes 6}, as repeated field 1
void kvwrite(std::vector<uint8_t> &out, const Span &ns, const Span &coll, const WEnt &w, uint64_t blk) {
  uint8_t ver[18];
  size_t vl = opv(ver, blk);
  vl += opv(ver + vl, w.tx);
  size_t m = 0;
  if (ns.n) m += field_len(ns.n);
  if (coll.n) m += field_len(coll.n);
  if (w.key.n) m += field_len(w.key.n);
  if (w.del) m += 2;
  else if (w.value.n) m += field_len(w.value.n);
  m += field_len(vl);
  const size_t at = out.size();
  out.resize(at + field_len(m));
  uint8_t *o = out.data() + at;
  *o++ = (uint8_t)(1 << 3 | 2);
  o = put_varint(o, m);
  if (ns.n) o = put_bytes(o, 1, ns.p, ns.n);
  if (coll.n) o = put_bytes(o, 2, coll.p, coll.n);
  if (w.key.n) o = put_bytes(o, 3, w.key.p, w.key.n);
  if (w.del) {
    *o++ = 0x20;  // isDelete = true
    *o++ = 0x01;
  } else if (w.value.n) {
    o = put_bytes(o, 5, w.value.p, w.value.n);
  }
  put_bytes(o, 6, ver, vl);
}

constexpr uint8_t kEmptySha256[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                      0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                      0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

struct TxScratch {
  std::vector<VKVRead> reads;
  std::vector<VKVWrite> writes;
  std::vector<VHashRead> hreads;
  std::vector<VHashWrite> hwrites;
};

// the writes of one VALID transaction (FGV_OK / FGV_EINVAL / FGV_EUNSUPPORTED)
int add_tx(Span d, uint32_t txi, std::vector<WEnt> &out, TxScratch &x) {
  VEnvelope env;
  VPayload pl;
  VHeader hdr;
  VChannelHeader chdr;
  if (!pbw::decode(d.p, d.n, env) || !pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.present ||
      !pl.header.decode_into(hdr) || !pbw::decode(hdr.channel_header.p, hdr.channel_header.n, chdr))
    return FGV_EINVAL;  // cannot be a VALID transaction
  if (chdr.type == 1) return FGV_OK;  // CONFIG: namespace "" only (core/peer/configtx_processor.go:19-39)
  if (chdr.type != 3) return FGV_EUNSUPPORTED;
  VTransaction tx;
  VCcActionPayload cap;
  VPrp prp;
  VCcAction cca;
  VTxRwSet rw;
  if (!pbw::decode(pl.data.p, pl.data.n, tx) || tx.actions.empty() ||
      !pbw::decode(tx.actions[0].payload.p, tx.actions[0].payload.n, cap) || !cap.has_action ||
      !pbw::decode(cap.action.prp.p, cap.action.prp.n, prp) || prp.extension.nil() ||
      !pbw::decode(prp.extension.p, prp.extension.n, cca) || !pbw::decode(cca.results.p, cca.results.n, rw))
    return FGV_EINVAL;
  const size_t mine = out.size();
  for (const VNsRwSet &ns : rw.ns) {
    x.reads.clear();
    x.writes.clear();
    VKVRWSet kv;
    kv.reads = &x.reads;
    kv.writes = &x.writes;
    if (!pbw::decode(ns.rwset.p, ns.rwset.n, kv)) return FGV_EINVAL;
    if (kv.nmeta) return FGV_EUNSUPPORTED;  // metadata: merged values come from the state DB
    for (const VKVWrite &w : x.writes) {
      const bool del = w.is_delete || w.value.n == 0;  // IsKVWriteDelete (rwset_proto_util.go:366-368)
      out.push_back(WEnt{ns.ns, Span(), w.key, del ? Span() : w.value, txi, false, del});
    }
    for (const VCollHashed &c : ns.coll) {
      x.hreads.clear();
      x.hwrites.clear();
      VHashedRWSet h;
      h.reads = &x.hreads;
      h.writes = &x.hwrites;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) return FGV_EINVAL;
      if (h.nmeta) return FGV_EUNSUPPORTED;
      for (const VHashWrite &w : x.hwrites) {  // IsKVWriteHashDelete (rwset_proto_util.go:370-375)
        const bool del = w.is_delete || w.value_hash.n == 0 ||
                         (w.value_hash.n == 32 && memcmp(w.value_hash.p, kEmptySha256, 32) == 0);
        out.push_back(WEnt{ns.ns, c.name, w.key, del ? Span() : w.value_hash, txi, true, del});
      }
    }
  }
  // a key written twice by one transaction: txOps flag arithmetic (tx_ops.go:183-191)
  for (size_t a = mine; a < out.size(); a++)
    for (size_t b = a + 1; b < out.size(); b++)
      if (same_key(out[a], out[b])) return FGV_EUNSUPPORTED;
  return FGV_OK;
}

}  // namespace

// SHA-256 stream over len(flags) || flags || update batch bytes of one block: everything of
// the commit hash but the previous hash, which comes last (kv_ledger.go:806-817)
static int commit_prefix(const uint8_t *block, size_t len, const uint8_t *flags, size_t ntx, uint64_t block_num,
                         fgvsha::Stream &s) {
  VBlock b;
  if (!pbw::decode(block, len, b) || b.data.data.size() != ntx) return FGV_EINVAL;
  std::vector<WEnt> w;
  w.reserve(ntx * 4 + 16);
  TxScratch x;
  for (size_t i = 0; i < ntx; i++) {
    if (flags[i] != 0) continue;
    const int rc = add_tx(b.data.data[i], (uint32_t)i, w, x);
    if (rc) return rc;
  }
  // (namespace, public < hashed, collection, key, tx): the last of each key's run is its update
  std::sort(w.begin(), w.end(), [](const WEnt &p, const WEnt &q) {
    int c = span_cmp(p.ns, q.ns);
    if (c) return c < 0;
    if (p.hashed != q.hashed) return !p.hashed;
    if ((c = span_cmp(p.coll, q.coll))) return c < 0;
    if ((c = span_cmp(p.key, q.key))) return c < 0;
    return p.tx < q.tx;
  });
  std::vector<uint8_t> batch;
  size_t est = 0;
  for (const WEnt &e : w) est += e.ns.n + e.coll.n + e.key.n + e.value.n + 48;
  batch.reserve(est + 256);
  const WEnt *prev = nullptr;  // the last update written
  for (size_t i = 0; i < w.size(); i++) {
    const WEnt &e = w[i];
    if (i + 1 < w.size() && same_key(w[i + 1], e)) continue;  // a later transaction writes this key too
    if (e.ns.n == 0) continue;  // channel config: not part of the hash (update_batch_bytes.go:39-44)
    const bool new_ns = !prev || !span_eq(prev->ns, e.ns);
    const bool new_coll = e.hashed && (new_ns || !prev->hashed || !span_eq(prev->coll, e.coll));
    kvwrite(batch, new_ns ? e.ns : Span(), new_coll ? e.coll : Span(), e, block_num);
    prev = &e;
  }
  uint8_t pre[10];
  const size_t pl = (size_t)(put_varint(pre, ntx) - pre);
  s.update(pre, pl);
  if (ntx) s.update(flags, ntx);
  if (!batch.empty()) s.update(batch.data(), batch.size());
  return FGV_OK;
}

extern "C" int fgv_commit_hash(const uint8_t *block, size_t len, const uint8_t *flags, size_t ntx,
                               uint64_t block_num, const uint8_t *prev, size_t prev_len, uint8_t out[32]) {
  if (!block || !out || (ntx && !flags) || (prev_len && !prev)) return FGV_EINVAL;
  fgvsha::Stream s;
  const int rc = commit_prefix(block, len, flags, ntx, block_num, s);
  if (rc) return rc;
  if (prev_len) s.update(prev, prev_len);
  s.final(out);
  return FGV_OK;
}

// Consecutive blocks: every block's update batch and the SHA-256 of everything before the
// previous hash on host workers in parallel, then the chain -- one last update and the final
// padding per block -- in block order.
extern "C" int fgv_commit_hashes(size_t n, const uint8_t *const *blocks, const size_t *lens,
                                 const uint8_t *const *flags, const size_t *ntx, const uint64_t *block_nums,
                                 const uint8_t *prev, size_t prev_len, uint8_t *out, unsigned threads) {
  if (n && (!blocks || !lens || !flags || !ntx || !block_nums || !out)) return FGV_EINVAL;
  if (prev_len && !prev) return FGV_EINVAL;
  for (size_t b = 0; b < n; b++)
    if (!blocks[b] || (ntx[b] && !flags[b])) return FGV_EINVAL;
  std::vector<fgvsha::Stream> st(n);
  std::vector<int> rc(n, FGV_OK);
  auto one = [&](size_t b) { rc[b] = commit_prefix(blocks[b], lens[b], flags[b], ntx[b], block_nums[b], st[b]); };
  // a persistent pool of min(16, hardware threads) workers, one caller at a time (a pool per call
  // spent ~20 us per thread creation); `threads` = 1 runs on the caller only
  static std::mutex pool_mu;
  static ThreadPool *pool = nullptr;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (threads == 1 || n <= 1) {
    for (size_t b = 0; b < n; b++) one(b);
  } else {
    std::lock_guard<std::mutex> g(pool_mu);
    if (!pool) pool = new ThreadPool(hw - 1);  // (the caller takes jobs too)
    pool->run(n, one);
  }
  for (size_t b = 0; b < n; b++)
    if (rc[b]) return rc[b];
  for (size_t b = 0; b < n; b++) {
    if (b) st[b].update(out + 32 * (b - 1), 32);
    else if (prev_len) st[b].update(prev, prev_len);
    st[b].final(out + 32 * b);
  }
  return FGV_OK;
}
