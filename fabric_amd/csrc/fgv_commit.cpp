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
#include <memory>
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
  uint32_t grp;               // (namespace, hashed, collection) group: its rank after sort_groups
  uint64_t kp;                // the key's first 8 bytes, big-endian, zero-padded (sort prefix)
  bool hashed, del;
};

inline int span_cmp(const Span &a, const Span &b) {  // std::string / Go sort.Strings order (bytewise)
  const size_t m = a.n < b.n ? a.n : b.n;
  const int c = m ? memcmp(a.p, b.p, m) : 0;
  return c ? c : (a.n < b.n ? -1 : a.n > b.n ? 1 : 0);
}
inline bool span_eq(const Span &a, const Span &b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }

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
uint8_t *kvwrite(uint8_t *o, const Span &ns, const Span &coll, const WEnt &w, uint64_t blk) {
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
  return put_bytes(o, 6, ver, vl);
}

constexpr uint8_t kEmptySha256[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                      0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                      0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// KVRWSet / HashedRWSet with the writes captured and the reads and range queries skipped at
// the wire level: a VALID transaction's read set was decoded by the validation that flagged
// it, and the update batch holds writes only
struct VKVWritesOnly {
  uint32_t nmeta = 0;
  std::vector<VKVWrite> *writes = nullptr;
  pbw::Kind kind(uint32_t n) { return (n == 3 || n == 4) ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 4) {
      nmeta++;
      return true;
    }
    VKVWrite w;
    if (!pbw::decode(s.p, s.n, w)) return false;
    writes->push_back(w);
    return true;
  }
};
struct VHashedWritesOnly {
  uint32_t nmeta = 0;
  std::vector<VHashWrite> *writes = nullptr;
  pbw::Kind kind(uint32_t n) { return (n == 2 || n == 3) ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 3) {
      nmeta++;
      return true;
    }
    VHashWrite w;
    if (!pbw::decode(s.p, s.n, w)) return false;
    writes->push_back(w);
    return true;
  }
};

// ChaincodeActionPayload.action.proposal_response_payload alone (the endorsements were
// verified by the validation that flagged the transaction VALID); every occurrence of the
// action merged in order, the last payload winning, as VCcActionPayload
struct VEaPrp {
  Span prp;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    prp = s;
    return true;
  }
};
struct VCapPrp {
  bool has_action = false;
  VEaPrp action;
  pbw::Kind kind(uint32_t n) { return n == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    has_action = true;
    return pbw::decode(s.p, s.n, action);
  }
};

inline uint64_t key_prefix(const Span &k) {
  uint64_t v = 0;
  const size_t m = k.n < 8 ? k.n : 8;
  for (size_t i = 0; i < m; i++) v |= (uint64_t)k.p[i] << (56 - 8 * i);
  return v;
}

struct SortRec {
  uint64_t kp;
  uint32_t grp, i;
};

// per-thread scratch reused across blocks (a fresh ~0.5 MB batch buffer per block cost its
// page faults every call)
struct TxScratch {
  std::vector<VKVWrite> writes;
  std::vector<VHashWrite> hwrites;
  std::vector<WEnt> w;
  std::vector<WEnt> grp;  // one representative entry per (namespace, hashed, collection) group
  std::vector<uint32_t> rank;
  std::vector<SortRec> ix;
  std::vector<uint32_t> dup;  // one transaction's write indices (the twice-written-key check)
  std::unique_ptr<uint8_t[]> batch;
  size_t cap = 0;
  uint32_t last = UINT32_MAX;
  uint32_t group_of(const WEnt &e) {
    if (last < grp.size() && grp[last].hashed == e.hashed && span_eq(grp[last].ns, e.ns) &&
        span_eq(grp[last].coll, e.coll))
      return last;
    for (uint32_t g = 0; g < grp.size(); g++)
      if (grp[g].hashed == e.hashed && span_eq(grp[g].ns, e.ns) && span_eq(grp[g].coll, e.coll)) return last = g;
    grp.push_back(e);
    return last = (uint32_t)(grp.size() - 1);
  }
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
  VCapPrp cap;
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
    x.writes.clear();
    VKVWritesOnly kv;
    kv.writes = &x.writes;
    if (!pbw::decode(ns.rwset.p, ns.rwset.n, kv)) return FGV_EINVAL;
    if (kv.nmeta) return FGV_EUNSUPPORTED;  // metadata: merged values come from the state DB
    for (const VKVWrite &w : x.writes) {
      const bool del = w.is_delete || w.value.n == 0;  // IsKVWriteDelete (rwset_proto_util.go:366-368)
      WEnt e{ns.ns, Span(), w.key, del ? Span() : w.value, txi, 0, key_prefix(w.key), false, del};
      e.grp = x.group_of(e);
      out.push_back(e);
    }
    for (const VCollHashed &c : ns.coll) {
      x.hwrites.clear();
      VHashedWritesOnly h;
      h.writes = &x.hwrites;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) return FGV_EINVAL;
      if (h.nmeta) return FGV_EUNSUPPORTED;
      for (const VHashWrite &w : x.hwrites) {  // IsKVWriteHashDelete (rwset_proto_util.go:370-375)
        const bool del = w.is_delete || w.value_hash.n == 0 ||
                         (w.value_hash.n == 32 && memcmp(w.value_hash.p, kEmptySha256, 32) == 0);
        WEnt e{ns.ns, c.name, w.key, del ? Span() : w.value_hash, txi, 0, key_prefix(w.key), true, del};
        e.grp = x.group_of(e);
        out.push_back(e);
      }
    }
  }
  // a key written twice by one transaction: txOps flag arithmetic (tx_ops.go:183-191).  Pairwise
  // for a handful of writes; otherwise the transaction's writes sorted by (group, prefix, key) and
  // neighbours compared, so a bulk-load transaction stays O(w log w)
  const size_t nw = out.size() - mine;
  if (nw <= 16) {
    for (size_t a = mine; a < out.size(); a++)
      for (size_t b = a + 1; b < out.size(); b++)
        if (out[a].grp == out[b].grp && out[a].kp == out[b].kp && span_eq(out[a].key, out[b].key))
          return FGV_EUNSUPPORTED;
    return FGV_OK;
  }
  std::vector<uint32_t> &o = x.dup;
  o.resize(nw);
  for (uint32_t i = 0; i < nw; i++) o[i] = (uint32_t)(mine + i);
  std::sort(o.begin(), o.end(), [&out](uint32_t a, uint32_t b) {
    if (out[a].grp != out[b].grp) return out[a].grp < out[b].grp;
    if (out[a].kp != out[b].kp) return out[a].kp < out[b].kp;
    return span_cmp(out[a].key, out[b].key) < 0;
  });
  for (size_t i = 1; i < nw; i++) {
    const WEnt &a = out[o[i - 1]], &b = out[o[i]];
    if (a.grp == b.grp && a.kp == b.kp && span_eq(a.key, b.key)) return FGV_EUNSUPPORTED;
  }
  return FGV_OK;
}

}  // namespace

// SHA-256 stream over len(flags) || flags || update batch bytes of one block: everything of
// the commit hash but the previous hash, which comes last (kv_ledger.go:806-817)
static int commit_prefix(const uint8_t *block, size_t len, const uint8_t *flags, size_t ntx, uint64_t block_num,
                         fgvsha::Stream &s) {
  VBlock b;
  if (!pbw::decode(block, len, b) || b.data.data.size() != ntx) return FGV_EINVAL;
  thread_local TxScratch x;
  std::vector<WEnt> &w = x.w;
  w.clear();
  x.grp.clear();
  x.last = UINT32_MAX;
  for (size_t i = 0; i < ntx; i++) {
    if (flags[i] != 0) continue;
    const int rc = add_tx(b.data.data[i], (uint32_t)i, w, x);
    if (rc) return rc;
  }
  // groups in (namespace, public < hashed, collection) order, then each group's keys: the entry
  // order is (group, key, tx) and the last of each key's run is its update
  const size_t ng = x.grp.size();
  std::vector<uint32_t> ord(ng);
  for (uint32_t g = 0; g < ng; g++) ord[g] = g;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t c) {
    const WEnt &p = x.grp[a], &q = x.grp[c];
    int r = span_cmp(p.ns, q.ns);
    if (r) return r < 0;
    if (p.hashed != q.hashed) return !p.hashed;
    return span_cmp(p.coll, q.coll) < 0;
  });
  x.rank.resize(ng);
  for (uint32_t g = 0; g < ng; g++) x.rank[ord[g]] = g;
  // sorted as 16-byte (group rank, key prefix, entry) records -- entries are in transaction
  // order, so the entry index breaks ties as the transaction number would
  std::vector<SortRec> &ix = x.ix;
  ix.resize(w.size());
  for (uint32_t i = 0; i < w.size(); i++) ix[i] = SortRec{w[i].kp, x.rank[w[i].grp], i};
  std::sort(ix.begin(), ix.end(), [&w](const SortRec &p, const SortRec &q) {
    if (p.grp != q.grp) return p.grp < q.grp;
    if (p.kp != q.kp) return p.kp < q.kp;
    const int c = span_cmp(w[p.i].key, w[q.i].key);
    return c ? c < 0 : p.i < q.i;
  });
  size_t est = 0;  // bound: every entry with its namespace and collection, 48 B of tags and lengths
  for (const WEnt &e : w) est += e.ns.n + e.coll.n + e.key.n + e.value.n + 48;
  if (est > x.cap) {
    x.cap = est + est / 4 + 4096;
    x.batch.reset(new uint8_t[x.cap]);
  }
  uint8_t *const b0 = x.batch.get();
  uint8_t *o = b0;
  const WEnt *prev = nullptr;  // the last update written
  for (size_t i = 0; i < ix.size(); i++) {
    const WEnt &e = w[ix[i].i];
    if (i + 1 < ix.size() && ix[i + 1].grp == ix[i].grp && ix[i + 1].kp == ix[i].kp && span_eq(w[ix[i + 1].i].key, e.key))
      continue;  // a later transaction writes this key too
    if (e.ns.n == 0) continue;  // channel config: not part of the hash (update_batch_bytes.go:39-44)
    const bool new_ns = !prev || !span_eq(prev->ns, e.ns);
    const bool new_coll = e.hashed && (new_ns || !prev->hashed || !span_eq(prev->coll, e.coll));
    o = kvwrite(o, new_ns ? e.ns : Span(), new_coll ? e.coll : Span(), e, block_num);
    prev = &e;
  }
  uint8_t pre[10];
  const size_t pl = (size_t)(put_varint(pre, ntx) - pre);
  s.update(pre, pl);
  if (ntx) s.update(flags, ntx);
  if (o != b0) s.update(b0, (size_t)(o - b0));
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
  return fgv_commit_hashes_ub(n, nullptr, nullptr, blocks, lens, flags, ntx, block_nums, prev, prev_len, out, threads);
}

// The same chain with the update-batch bytes given where the device serialised them
// (fgv_mvcc_update_bytes_acquire): such a block's prefix is varint(len(flags)) || flags || bytes,
// one SHA-256 stream; a block without them is decoded as above.
extern "C" int fgv_commit_hashes_ub(size_t n, const uint8_t *const *ub, const size_t *ub_lens,
                                    const uint8_t *const *blocks, const size_t *lens, const uint8_t *const *flags,
                                    const size_t *ntx, const uint64_t *block_nums, const uint8_t *prev,
                                    size_t prev_len, uint8_t *out, unsigned threads) {
  if (n && (!flags || !ntx || !out)) return FGV_EINVAL;
  if (prev_len && !prev) return FGV_EINVAL;
  if (ub && !ub_lens) return FGV_EINVAL;
  for (size_t b = 0; b < n; b++) {
    if (ntx[b] && !flags[b]) return FGV_EINVAL;
    if (!(ub && ub[b]) && (!blocks || !lens || !block_nums || !blocks[b])) return FGV_EINVAL;
  }
  std::vector<fgvsha::Stream> st(n);
  std::vector<int> rc(n, FGV_OK);
  auto one = [&](size_t b) {
    if (ub && ub[b]) {
      uint8_t pre[10];
      st[b].update(pre, (size_t)(put_varint(pre, ntx[b]) - pre));
      if (ntx[b]) st[b].update(flags[b], ntx[b]);
      if (ub_lens[b]) st[b].update(ub[b], ub_lens[b]);
      return;
    }
    rc[b] = commit_prefix(blocks[b], lens[b], flags[b], ntx[b], block_nums[b], st[b]);
  };
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
