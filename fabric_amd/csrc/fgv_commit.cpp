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
#include <map>
#include <thread>
#include <string>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_visitors.h"
#include "sha256_host.h"

using namespace fgvb;

namespace {

struct Val {
  Span value;  // nil: delete
  bool del = false;
  uint64_t blk = 0, tx = 0;
};
using KeyMap = std::map<std::string, Val>;  // std::string order == Go sort.Strings (bytewise)

void put_varint(std::string &o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(uint8_t)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)(uint8_t)v);
}
void put_bytes(std::string &o, uint32_t field, const void *p, size_t n) {
  put_varint(o, (uint64_t)field << 3 | 2);
  put_varint(o, n);
  o.append(static_cast<const char *>(p), n);
}
// common/ledger/util/util.go:32-52 EncodeOrderPreservingVarUint64
void put_opv(std::string &o, uint64_t n) {
  int i = 0;
  while (i < 8 && ((n >> (56 - 8 * i)) & 0xFF) == 0) i++;
  o.push_back((char)(uint8_t)(8 - i));
  for (; i < 8; i++) o.push_back((char)(uint8_t)(n >> (56 - 8 * i)));
}

void kvwrite(std::string &out, const std::string &ns, const std::string &coll, const std::string &key, const Val &v) {
  std::string m;
  if (!ns.empty()) put_bytes(m, 1, ns.data(), ns.size());
  if (!coll.empty()) put_bytes(m, 2, coll.data(), coll.size());
  if (!key.empty()) put_bytes(m, 3, key.data(), key.size());
  if (v.del) {
    m.push_back(0x20);  // isDelete = true
    m.push_back(0x01);
  } else if (v.value.n) {
    put_bytes(m, 5, v.value.p, v.value.n);
  }
  std::string ver;
  put_opv(ver, v.blk);
  put_opv(ver, v.tx);
  put_bytes(m, 6, ver.data(), ver.size());
  put_bytes(out, 1, m.data(), m.size());
}

constexpr uint8_t kEmptySha256[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                      0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                      0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// the update batch of one VALID transaction (FGV_OK / FGV_EINVAL / FGV_EUNSUPPORTED)
int add_tx(Span d, uint64_t blk, uint64_t txi, std::map<std::string, KeyMap> &pub,
           std::map<std::string, std::map<std::string, KeyMap>> &hashed) {
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
  std::vector<VKVRead> reads;
  std::vector<VKVWrite> writes;
  std::vector<VHashRead> hreads;
  std::vector<VHashWrite> hwrites;
  std::map<std::string, int> seen;  // a key written twice by one tx: txOps flag arithmetic
  for (const VNsRwSet &ns : rw.ns) {
    reads.clear();
    writes.clear();
    VKVRWSet kv;
    kv.reads = &reads;
    kv.writes = &writes;
    if (!pbw::decode(ns.rwset.p, ns.rwset.n, kv)) return FGV_EINVAL;
    if (kv.nmeta) return FGV_EUNSUPPORTED;  // metadata: merged values come from the state DB
    const std::string nss = ns.ns.str();
    for (const VKVWrite &w : writes) {
      std::string k = w.key.str();
      if (!seen.emplace(std::string("p") + nss + '\0' + k, 0).second) return FGV_EUNSUPPORTED;
      Val v;
      v.del = w.is_delete || w.value.n == 0;  // IsKVWriteDelete (rwset_proto_util.go:366-368)
      v.value = v.del ? Span() : w.value;
      v.blk = blk;
      v.tx = txi;
      pub[nss][k] = v;
    }
    for (const VCollHashed &c : ns.coll) {
      hreads.clear();
      hwrites.clear();
      VHashedRWSet h;
      h.reads = &hreads;
      h.writes = &hwrites;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) return FGV_EINVAL;
      if (h.nmeta) return FGV_EUNSUPPORTED;
      const std::string cn = c.name.str();
      for (const VHashWrite &w : hwrites) {
        std::string k = w.key.str();
        if (!seen.emplace(std::string("h") + nss + '\0' + cn + '\0' + k, 0).second) return FGV_EUNSUPPORTED;
        Val v;  // IsKVWriteHashDelete (rwset_proto_util.go:370-375)
        v.del = w.is_delete || w.value_hash.n == 0 ||
                (w.value_hash.n == 32 && memcmp(w.value_hash.p, kEmptySha256, 32) == 0);
        v.value = v.del ? Span() : w.value_hash;
        v.blk = blk;
        v.tx = txi;
        hashed[nss][cn][k] = v;
      }
    }
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
  std::map<std::string, KeyMap> pub;
  std::map<std::string, std::map<std::string, KeyMap>> hashed;
  for (size_t i = 0; i < ntx; i++) {
    if (flags[i] != 0) continue;
    const int rc = add_tx(b.data.data[i], block_num, i, pub, hashed);
    if (rc) return rc;
  }
  std::string batch;
  auto pit = pub.begin();
  auto hit = hashed.begin();
  while (pit != pub.end() || hit != hashed.end()) {  // merged, sorted namespace lists
    std::string ns;
    const KeyMap *pk = nullptr;
    const std::map<std::string, KeyMap> *hk = nullptr;
    if (hit == hashed.end() || (pit != pub.end() && pit->first <= hit->first)) {
      ns = pit->first;
      pk = &pit->second;
      if (hit != hashed.end() && hit->first == ns) hk = &(hit++)->second;
      ++pit;
    } else {
      ns = hit->first;
      hk = &(hit++)->second;
    }
    if (ns.empty()) continue;  // channel config: not part of the hash (update_batch_bytes.go:39-44)
    bool first = true;
    if (pk)
      for (const auto &kv : *pk) {
        kvwrite(batch, first ? ns : std::string(), std::string(), kv.first, kv.second);
        first = false;
      }
    if (hk)
      for (const auto &cm : *hk) {
        bool cfirst = true;
        for (const auto &kv : cm.second) {
          kvwrite(batch, first ? ns : std::string(), cfirst ? cm.first : std::string(), kv.first, kv.second);
          first = cfirst = false;
        }
      }
  }
  std::string pre;
  put_varint(pre, ntx);
  s.update(reinterpret_cast<const uint8_t *>(pre.data()), pre.size());
  if (ntx) s.update(flags, ntx);
  s.update(reinterpret_cast<const uint8_t *>(batch.data()), batch.size());
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
  const unsigned nt = std::min<size_t>(n, threads ? threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (nt <= 1) {
    for (size_t b = 0; b < n; b++) one(b);
  } else {
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++)
      th.emplace_back([&] {
        for (size_t b; (b = next.fetch_add(1)) < n;) one(b);
      });
    for (size_t b; (b = next.fetch_add(1)) < n;) one(b);
    for (auto &t : th) t.join();
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
