// fgv_mvcc.cpp -- host side of MVCC validation (libfgv.so): the committed-state table on the
// GPU (a cache of the state DB, rebuilt from it at start -- never authoritative), per-block
// rwset extraction, kernel orchestration (mvcc.hip).
//
// Reference (core/ledger/kvledger/txmgmt): validation/batch_preparer.go:192-286
// (preprocessProtoBlock: skip committer-invalid txs, NIL_TXACTION(16) / INVALID_OTHER_REASON
// (255) on extraction errors), validation/validator.go:81-200 (sequential MVCC, code 11),
// validation/types.go:81-112 + tx_ops.go:17-51 (puts/deletes applied at Height{blk, tx}; a
// later write of the same key wins), statedb/stateleveldb/stateleveldb.go:128-137 (GetVersion),
// internal/version/version.go:82-90 (AreSame: nil == nil).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_internal.h"
#include "fgv_visitors.h"

bool fgv_block_take_presplit(fgv_block_state *S, const uint8_t *block, size_t len, std::vector<Span> &out);

using namespace fgvb;

namespace {

struct MvRead {
  Span ns, key;
  bool has_ver;
  uint64_t blk, txn;
};
struct MvWrite {
  Span ns, key;
  bool del;
};
struct MvTx {
  uint8_t code = 0;  // 0 participates; 16 / 255 decided here; 0xFD unsupported; 0xFF skipped
  bool new_ns = false;             // names a namespace not yet registered (resolved serially)
  std::vector<MvRead> reads;       // (vectors keep their capacity across blocks)
  std::vector<MvWrite> writes;
  std::vector<uint32_t> rns, wns;  // namespace id of each read / write
  std::vector<std::string> hashed_ns;  // ns + "$$h" + coll of the private-data sets read/written
  uint64_t wbytes = 0;
};

constexpr uint8_t MV_UNSUP = 0xFD, MV_SKIP = 0xFF;
// SHA-256("") = rwsetutil.hashOfZeroLengthByteArray (rwset_proto_util.go:370)
constexpr uint8_t kEmptySha256[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                      0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                      0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

// GetActionFromEnvelope + TxRwSet.FromProtoBytes for one committer-valid transaction
void mv_parse(Span d, MvTx &T) {
  T.code = 0;
  T.new_ns = false;
  T.reads.clear();
  T.writes.clear();
  T.wbytes = 0;
  VEnvelope env;
  VPayload pl;
  VHeader hdr;
  VChannelHeader chdr;
  if (!pbw::decode(d.p, d.n, env) || !pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.present ||
      !pl.header.decode_into(hdr) || !pbw::decode(hdr.channel_header.p, hdr.channel_header.n, chdr)) {
    T.code = MV_UNSUP;  // the reference returns an error (channel halt) -- not ours to decide
    return;
  }
  if (chdr.type != 3) {
    T.code = MV_UNSUP;  // CONFIG etc. go through custom tx processors
    return;
  }
  VTransaction tx;
  if (!pbw::decode(pl.data.p, pl.data.n, tx) || tx.actions.empty()) { T.code = 16; return; }
  VCcActionPayload cap;
  if (!pbw::decode(tx.actions[0].payload.p, tx.actions[0].payload.n, cap)) { T.code = 16; return; }
  if (!cap.has_action || cap.action.prp.nil()) { T.code = 16; return; }
  VPrp prp;
  if (!pbw::decode(cap.action.prp.p, cap.action.prp.n, prp) || prp.extension.nil()) { T.code = 16; return; }
  VCcAction cca;
  if (!pbw::decode(prp.extension.p, prp.extension.n, cca)) { T.code = 16; return; }
  VTxRwSet rw;
  if (!pbw::decode(cca.results.p, cca.results.n, rw)) { T.code = 255; return; }
  bool unsup = false;
  static thread_local std::vector<VKVRead> reads;
  static thread_local std::vector<VKVWrite> writes;
  static thread_local std::vector<VHashRead> hreads;
  static thread_local std::vector<VHashWrite> hwrites;
  size_t ncoll = 0;
  for (const VNsRwSet &ns : rw.ns) ncoll += ns.coll.size();
  T.hashed_ns.clear();
  T.hashed_ns.reserve(ncoll);  // spans below point into these strings: no reallocation after this
  for (VNsRwSet &ns : rw.ns) {
    reads.clear();
    writes.clear();
    VKVRWSet kv;
    kv.reads = &reads;
    kv.writes = &writes;
    if (!pbw::decode(ns.rwset.p, ns.rwset.n, kv)) { T.code = 255; return; }
    if (kv.nrq || kv.nmeta) unsup = true;  // phantom checks / metadata writes: not modelled
    for (const VKVRead &r : reads) T.reads.push_back(MvRead{ns.ns, r.key, r.has_ver, r.ver.block, r.ver.tx});
    // IsKVWriteDelete (rwsetutil/rwset_proto_util.go:366-368): is_delete or an empty value
    for (const VKVWrite &w : writes) {
      T.writes.push_back(MvWrite{ns.ns, w.key, w.is_delete || w.value.n == 0});
      T.wbytes += w.key.n;
    }
    // private data: validateKVReadHash (validation/validator.go:272-293) is a point read of the
    // key hash in the hashed-data namespace ns + "$$h" + coll (privacyenabledstate/db.go:355-357)
    for (const VCollHashed &c : ns.coll) {
      hreads.clear();
      hwrites.clear();
      VHashedRWSet h;
      h.reads = &hreads;
      h.writes = &hwrites;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) { T.code = 255; return; }
      if (h.nmeta) unsup = true;  // hashed metadata writes: not modelled
      if (hreads.empty() && hwrites.empty()) continue;
      T.hashed_ns.emplace_back();
      std::string &hn = T.hashed_ns.back();
      hn.reserve(ns.ns.n + 3 + c.name.n);
      hn.append((const char *)ns.ns.p, ns.ns.n).append("$$h").append((const char *)c.name.p, c.name.n);
      const Span hs{(const uint8_t *)hn.data(), (uint32_t)hn.size()};
      for (const VHashRead &r : hreads) T.reads.push_back(MvRead{hs, r.key, r.has_ver, r.ver.block, r.ver.tx});
      // IsKVWriteHashDelete (rwset_proto_util.go:373-375): is_delete, empty value hash, or the
      // hash of the empty string
      for (const VHashWrite &w : hwrites) {
        const bool del = w.is_delete || w.value_hash.n == 0 ||
                         (w.value_hash.n == 32 && memcmp(w.value_hash.p, kEmptySha256, 32) == 0);
        T.writes.push_back(MvWrite{hs, w.key, del});
        T.wbytes += w.key.n;
      }
    }
  }
  if (unsup) T.code = MV_UNSUP;
}

}  // namespace

struct fgv_mvcc_state {
  std::unordered_map<std::string, uint32_t> ns_ids;
  uint64_t cap = 0, mask = 0, nkeys = 0, arena_cap = 0, arena_used = 0;
  DevBuf tbl, arena, top;
  DevBuf reads, writes, rtags, wtags, btbl, wslot, rslot, rbeg, part, bad, st, undec, pend, npend, flags, lbytes, lkeys;
  std::vector<MvTx> txs;
  std::vector<Span> pre_envs;  // envelope spans taken from a pre-split
  HostBuf hreads, hwrites, hmeta;  // pinned staging of the MvKey arrays, rbeg and part
  uint32_t last_rounds = 0;
};

void fgv_mvcc_free(fgv_mvcc_state *M) {
  if (!M) return;
  DevBuf *d[] = {&M->tbl, &M->arena, &M->top, &M->reads, &M->writes, &M->rtags, &M->wtags, &M->btbl, &M->wslot,
                 &M->rslot, &M->rbeg, &M->part, &M->bad, &M->st, &M->undec, &M->pend, &M->npend, &M->flags,
                 &M->lbytes, &M->lkeys};
  for (auto *b : d) b->release();
  M->hreads.release();
  M->hwrites.release();
  M->hmeta.release();
  delete M;
}

// namespace ids of one parsed transaction, read-only on the map (parallel phase): a span equal
// to the previous one reuses its id; an unknown namespace sets new_ns
static void mv_resolve_ns(const fgv_mvcc_state *M, MvTx &T) {
  T.rns.resize(T.reads.size());
  T.wns.resize(T.writes.size());
  Span last{nullptr, 0};
  uint32_t last_id = 0;
  bool have = false;
  auto id_of = [&](const Span &s, uint32_t &id) {
    if (have && s.n == last.n && (s.n == 0 || memcmp(s.p, last.p, s.n) == 0)) {
      id = last_id;
      return true;
    }
    auto it = M->ns_ids.find(s.str());
    if (it == M->ns_ids.end()) return false;
    last = s;
    last_id = id = it->second;
    have = true;
    return true;
  };
  for (size_t k = 0; k < T.reads.size(); k++)
    if (!id_of(T.reads[k].ns, T.rns[k])) T.new_ns = true;
  for (size_t k = 0; k < T.writes.size(); k++)
    if (!id_of(T.writes[k].ns, T.wns[k])) T.new_ns = true;
}

static bool ns_lookup(fgv_mvcc_state *M, const Span &s, bool create, uint32_t &id) {
  const std::string k = s.str();
  auto it = M->ns_ids.find(k);
  if (it != M->ns_ids.end()) {
    id = it->second;
    return true;
  }
  if (!create || M->ns_ids.size() >= 0x7fff) return false;
  id = (uint32_t)M->ns_ids.size();
  M->ns_ids.emplace(k, id);
  return true;
}

static inline dim3 grid_for(size_t n) { return dim3((uint32_t)((n + 255) / 256)); }

extern "C" {

int fgv_statedb_init(fgv_ctx *c, uint64_t slots, uint64_t arena_bytes) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  if (!c->mv) c->mv = new fgv_mvcc_state();
  fgv_mvcc_state *M = c->mv;
  uint64_t cap = 1024;
  while (cap < (slots ? slots : (1ull << 22))) cap <<= 1;
  const uint64_t arena = arena_bytes ? arena_bytes : (64ull << 20);
  if (!M->tbl.ensure(cap * sizeof(StateSlot)) || !M->arena.ensure(arena) || !M->top.ensure(8)) return FGV_ENOMEM;
  M->cap = cap;
  M->mask = cap - 1;
  M->arena_cap = arena;
  M->arena_used = 0;
  M->nkeys = 0;
  M->ns_ids.clear();
  HIP_TRY(hipMemsetAsync(M->tbl.p, 0, cap * sizeof(StateSlot), c->stream));
  HIP_TRY(hipMemsetAsync(M->top.p, 0, 8, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FGV_OK;
}

int fgv_statedb_load(fgv_ctx *c, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                     const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn, size_t n) {
  if (!c || !ns || (n && (!key_buf || !key_off || !key_len || !blk || !txn))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  if (n == 0) return FGV_OK;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  uint32_t nsid;
  if (!ns_lookup(M, Span{reinterpret_cast<const uint8_t *>(ns), (uint32_t)strlen(ns)}, true, nsid))
    return FGV_EUNSUPPORTED;
  if ((M->nkeys + n) * 10 > M->cap * 7) return FGV_ENOMEM;  // keep the load factor <= 0.7
  size_t bytes = 0;
  for (size_t i = 0; i < n; i++) {
    if (key_len[i] > 0xffff) return FGV_EUNSUPPORTED;
    bytes = std::max<size_t>(bytes, key_off[i] + key_len[i]);
  }
  if (M->arena_used + bytes > M->arena_cap) return FGV_ENOMEM;
  if (!M->lbytes.ensure(bytes + 64) || !M->lkeys.ensure(n * sizeof(MvKey)) || !M->wtags.ensure(n * 8))
    return FGV_ENOMEM;
  std::vector<MvKey> keys(n);
  const uint64_t base = (uint64_t)(uintptr_t)M->lbytes.p;
  for (size_t i = 0; i < n; i++) keys[i] = MvKey{base + key_off[i], key_len[i], nsid, 0, 0, blk[i], txn[i]};
  HIP_TRY(hipMemcpyAsync(M->lbytes.p, key_buf, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(M->lkeys.p, keys.data(), n * sizeof(MvKey), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_mv_tags, grid_for(n), dim3(256), 0, c->stream, M->lkeys.as<MvKey>(), (uint32_t)n,
                     M->wtags.as<uint64_t>());
  hipLaunchKernelGGL(k_mv_load, grid_for(n), dim3(256), 0, c->stream, M->lkeys.as<MvKey>(), M->wtags.as<uint64_t>(),
                     (uint32_t)n, M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                     M->top.as<unsigned long long>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  M->nkeys += n;
  M->arena_used += bytes;
  return FGV_OK;
}

static int mvcc_validate(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block, uint64_t block_num,
                         uint8_t *flags, size_t ntx, int commit, const uint8_t *next, size_t next_len);

int fgv_mvcc_validate_block(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block,
                            uint64_t block_num, uint8_t *flags, size_t ntx, int commit) {
  return mvcc_validate(c, block, len, d_block, block_num, flags, ntx, commit, nullptr, 0);
}

int fgv_mvcc_validate_block_next(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block,
                                 uint64_t block_num, uint8_t *flags, size_t ntx, int commit, const uint8_t *next,
                                 size_t next_len) {
  if (next && !next_len) return FGV_EINVAL;
  return mvcc_validate(c, block, len, d_block, block_num, flags, ntx, commit, next, next_len);
}

}  // extern "C"

static int mvcc_validate(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block, uint64_t block_num,
                         uint8_t *flags, size_t ntx, int commit, const uint8_t *next, size_t next_len) {
  if (!c || !block || (ntx && !flags)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  // the block's envelope spans: from fgv_presplit of this block (walked while the previous
  // block validated), else walked here (one dependent load per envelope)
  VBlock blk;
  const bool pre = fgv_block_take_presplit(c->blk, block, len, M->pre_envs);
  if (!pre && !pbw::decode(block, len, blk)) return FGV_EINVAL;
  const std::vector<Span> &envs = pre ? M->pre_envs : blk.data.data;
  if (next) fgv_block_presplit(c->blk, c->device, 1, &next, &next_len, nullptr, nullptr);  // the next block's walk
  if (envs.size() != ntx) return FGV_EINVAL;
  const uint8_t *dblk = d_block;
  if (!dblk) {
    if (!c->blk_arena.ensure(len + 64)) return FGV_ENOMEM;
    HIP_TRY(hipMemcpyAsync(c->blk_arena.p, block, len, hipMemcpyHostToDevice, c->stream));
    dblk = c->blk_arena.as<uint8_t>();
  }
  // --- host: rwsets of committer-valid txs, namespace ids (parallel; the map is read-only)
  M->txs.resize(ntx);
  fgv_parallel_for(c->blk, ntx, [&](size_t i) {
    MvTx &T = M->txs[i];
    if (flags[i] != 0) {
      T.code = MV_SKIP;
      return;
    }
    mv_parse(envs[i], T);
    if (T.code == 0) mv_resolve_ns(M, T);
  });
  // serial: unsupported txs, first sightings of a namespace (rare), read / write offsets
  if (!M->hmeta.ensure((ntx + 1) * 4 * 2 + ntx + 64)) return FGV_ENOMEM;
  uint32_t *rbeg = M->hmeta.as<uint32_t>(), *wbeg = rbeg + ntx + 1;
  uint8_t *part = reinterpret_cast<uint8_t *>(wbeg + ntx + 1);
  size_t nr = 0, nw = 0, wbytes = 0;
  for (size_t i = 0; i < ntx; i++) {
    MvTx &T = M->txs[i];
    rbeg[i] = (uint32_t)nr;
    wbeg[i] = (uint32_t)nw;
    part[i] = 0;
    if (T.code == MV_UNSUP) return FGV_EUNSUPPORTED;
    if (T.code != 0) continue;
    if (T.new_ns) {
      for (size_t k = 0; k < T.reads.size(); k++)
        if (!ns_lookup(M, T.reads[k].ns, true, T.rns[k])) return FGV_EUNSUPPORTED;
      for (size_t k = 0; k < T.writes.size(); k++)
        if (!ns_lookup(M, T.writes[k].ns, true, T.wns[k])) return FGV_EUNSUPPORTED;
    }
    part[i] = 1;
    nr += T.reads.size();
    nw += T.writes.size();
    wbytes += T.wbytes;
  }
  rbeg[ntx] = (uint32_t)nr;
  wbeg[ntx] = (uint32_t)nw;
  // parallel: the MvKey arrays, straight into pinned staging
  if (!M->hreads.ensure(std::max<size_t>(nr, 1) * sizeof(MvKey)) ||
      !M->hwrites.ensure(std::max<size_t>(nw, 1) * sizeof(MvKey)))
    return FGV_ENOMEM;
  MvKey *hr = M->hreads.as<MvKey>(), *hw = M->hwrites.as<MvKey>();
  std::atomic<bool> too_long{false};
  fgv_parallel_for(c->blk, ntx, [&](size_t i) {
    const MvTx &T = M->txs[i];
    if (!part[i]) return;
    const uint64_t base = (uint64_t)(uintptr_t)dblk - (uint64_t)(uintptr_t)block;
    MvKey *r = hr + rbeg[i], *w = hw + wbeg[i];
    for (size_t k = 0; k < T.reads.size(); k++) {
      const MvRead &x = T.reads[k];
      if (x.key.n > 0xffff) too_long = true;
      r[k] = MvKey{base + (uint64_t)(uintptr_t)x.key.p, x.key.n, T.rns[k], (uint32_t)i, x.has_ver ? 1u : 0u, x.blk,
                   x.txn};
    }
    for (size_t k = 0; k < T.writes.size(); k++) {
      const MvWrite &x = T.writes[k];
      if (x.key.n > 0xffff) too_long = true;
      w[k] = MvKey{base + (uint64_t)(uintptr_t)x.key.p, x.key.n, T.wns[k], (uint32_t)i, x.del ? 1u : 0u, 0, 0};
    }
  });
  if (too_long) return FGV_EUNSUPPORTED;
  uint32_t bcap = 1024;
  while (bcap < 2 * nw) bcap <<= 1;
  if (commit && ((M->nkeys + nw) * 10 > M->cap * 7 || M->arena_used + wbytes > M->arena_cap)) return FGV_ENOMEM;
  if (!M->reads.ensure(std::max<size_t>(nr, 1) * sizeof(MvKey)) || !M->writes.ensure(std::max<size_t>(nw, 1) * sizeof(MvKey)) ||
      !M->rtags.ensure(std::max<size_t>(nr, 1) * 8) || !M->wtags.ensure(std::max<size_t>(nw, 1) * 8) ||
      !M->btbl.ensure(bcap * sizeof(BlkSlot)) || !M->wslot.ensure(std::max<size_t>(nw, 1) * 4) ||
      !M->rslot.ensure(std::max<size_t>(nr, 1) * 4) || !M->rbeg.ensure((ntx + 1) * 4) || !M->part.ensure(ntx + 1) ||
      !M->bad.ensure(ntx + 1) || !M->st.ensure(ntx + 1) || !M->undec.ensure(4) || !M->pend.ensure(bcap * 4) ||
      !M->npend.ensure(4) || !M->flags.ensure(ntx + 1))
    return FGV_ENOMEM;
  hipStream_t s = c->stream;
  if (nr) HIP_TRY(hipMemcpyAsync(M->reads.p, hr, nr * sizeof(MvKey), hipMemcpyHostToDevice, s));
  if (nw) HIP_TRY(hipMemcpyAsync(M->writes.p, hw, nw * sizeof(MvKey), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(M->rbeg.p, rbeg, (ntx + 1) * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(M->part.p, part, ntx, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(M->bad.p, 0, ntx + 1, s));
  HIP_TRY(hipMemsetAsync(M->btbl.p, 0, bcap * sizeof(BlkSlot), s));
  HIP_TRY(hipEventRecord(c->ev[0], s));
  if (nr + nw)
    hipLaunchKernelGGL(k_mv_tags2, grid_for(nr + nw), dim3(256), 0, s, M->reads.as<MvKey>(), (uint32_t)nr,
                       M->rtags.as<uint64_t>(), M->writes.as<MvKey>(), (uint32_t)nw, M->wtags.as<uint64_t>());
  if (nr)
    hipLaunchKernelGGL(k_mv_lookup, grid_for(nr), dim3(256), 0, s, M->reads.as<MvKey>(), M->rtags.as<uint64_t>(),
                       (uint32_t)nr, M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(), M->bad.as<uint8_t>());
  HIP_TRY(hipEventRecord(c->ev[1], s));
  if (nw)
    hipLaunchKernelGGL(k_mv_blk_insert, grid_for(nw), dim3(256), 0, s, M->writes.as<MvKey>(), M->wtags.as<uint64_t>(),
                       (uint32_t)nw, M->btbl.as<BlkSlot>(), bcap - 1, M->wslot.as<uint32_t>());
  hipLaunchKernelGGL(k_mv_find_init, grid_for(nr + ntx), dim3(256), 0, s, M->reads.as<MvKey>(), M->rtags.as<uint64_t>(),
                     (uint32_t)nr, M->btbl.as<BlkSlot>(), bcap - 1, M->writes.as<MvKey>(), M->wtags.as<uint64_t>(),
                     M->rslot.as<uint32_t>(), (uint32_t)ntx, M->part.as<uint8_t>(), M->bad.as<uint8_t>(),
                     M->st.as<uint8_t>());
  HIP_TRY(hipGetLastError());
  // fixpoint: two rounds per host check
  uint32_t undec = 1, rounds = 0;
  while (undec) {
    for (int k = 0; k < 2; k++) {
      rounds++;  // round tags start at 1 (the write table was zeroed above)
      hipLaunchKernelGGL(k_mv_min, grid_for(nw ? nw : 1), dim3(256), 0, s, M->writes.as<MvKey>(), M->wslot.as<uint32_t>(),
                         (uint32_t)nw, M->st.as<uint8_t>(), M->btbl.as<BlkSlot>(), rounds, M->undec.as<uint32_t>());
      hipLaunchKernelGGL(k_mv_decide, grid_for(ntx), dim3(256), 0, s, (uint32_t)ntx, M->rbeg.as<uint32_t>(),
                         M->rslot.as<uint32_t>(), M->btbl.as<BlkSlot>(), M->st.as<uint8_t>(), rounds,
                         M->undec.as<uint32_t>());
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&undec, M->undec.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (rounds > 2 * ntx + 4) return FGV_EDEVICE;  // cannot happen: one decision per round at least
  }
  M->last_rounds = rounds;
  hipLaunchKernelGGL(k_mv_flags, grid_for(ntx), dim3(256), 0, s, (uint32_t)ntx, M->part.as<uint8_t>(),
                     M->st.as<uint8_t>(), M->flags.as<uint8_t>());
  std::vector<uint8_t> mv(ntx);
  HIP_TRY(hipMemcpyAsync(mv.data(), M->flags.p, ntx, hipMemcpyDeviceToHost, s));
  if (commit && nw) {
    HIP_TRY(hipMemsetAsync(M->npend.p, 0, 4, s));
    hipLaunchKernelGGL(k_mv_lastwriter, grid_for(nw), dim3(256), 0, s, M->writes.as<MvKey>(), M->wslot.as<uint32_t>(),
                       (uint32_t)nw, M->st.as<uint8_t>(), M->btbl.as<BlkSlot>());
    hipLaunchKernelGGL(k_mv_apply_find, grid_for(bcap), dim3(256), 0, s, M->btbl.as<BlkSlot>(), bcap,
                       M->writes.as<MvKey>(), M->wtags.as<uint64_t>(), M->tbl.as<StateSlot>(), M->mask,
                       M->arena.as<uint8_t>(), block_num, M->pend.as<uint32_t>(), M->npend.as<uint32_t>());
    uint32_t np = 0;
    HIP_TRY(hipMemcpyAsync(&np, M->npend.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (np)
      hipLaunchKernelGGL(k_mv_apply_insert, grid_for(np), dim3(256), 0, s, M->btbl.as<BlkSlot>(), M->pend.as<uint32_t>(),
                         np, M->writes.as<MvKey>(), M->wtags.as<uint64_t>(), M->tbl.as<StateSlot>(), M->mask,
                         M->arena.as<uint8_t>(), M->top.as<unsigned long long>(), block_num);
    HIP_TRY(hipGetLastError());
    M->nkeys += np;
    M->arena_used += wbytes;  // upper bound of the bytes appended
  }
  HIP_TRY(hipEventRecord(c->ev[2], s));
  HIP_TRY(hipStreamSynchronize(s));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_mvcc_lookup = ms;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[2]) == hipSuccess) c->t_mvcc_total = ms;
  c->n_mvcc_reads = nr;
  c->n_mvcc_writes = nw;
  for (size_t i = 0; i < ntx; i++) {
    const MvTx &T = M->txs[i];
    if (T.code == MV_SKIP) continue;
    flags[i] = T.code ? T.code : mv[i];
  }
  return FGV_OK;
}

extern "C" {

int fgv_mvcc_last_stats(fgv_ctx *c, double *lookup_ms, double *total_ms, uint64_t *reads, uint64_t *writes,
                        uint32_t *rounds) {
  if (!c) return FGV_EINVAL;
  if (lookup_ms) *lookup_ms = c->t_mvcc_lookup;
  if (total_ms) *total_ms = c->t_mvcc_total;
  if (reads) *reads = c->n_mvcc_reads;
  if (writes) *writes = c->n_mvcc_writes;
  if (rounds) *rounds = c->mv ? c->mv->last_rounds : 0;
  return FGV_OK;
}

}  // extern "C"
