// fgv_mvcc.cpp -- host side of MVCC validation (libfgv.so): the committed-state table on the
// GPU (a cache of the state DB, loaded from it at start and kept current by commits or by
// fgv_statedb_apply -- never authoritative) and the launch sequence of mvcc.hip.
//
// Per block the host only walks the block data framing (the envelope spans; usually done ahead
// by fgv_presplit / fgv_mvcc_validate_block_next while the previous block validates), sends one
// head copy (envelope table | committer flags | zeroed counters) and reads back one tail copy
// (counters | TRANSACTIONS_FILTER).  rwset extraction, the version checks, the fixpoint and the
// commit run on the device (mvcc.hip).
//
// Reference (core/ledger/kvledger/txmgmt): validation/batch_preparer.go:192-286,
// validation/validator.go:81-293, validation/types.go:81-112 + tx_ops.go:17-51,
// statedb/stateleveldb/stateleveldb.go:128-137 (GetVersion), internal/version/version.go:82-90.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fgv.h"
#include "blockdev.h"
#include "fgv_internal.h"
#include "mvcc_multi.h"
#include "fgv_visitors.h"
#include "sha256_host.h"

bool fgv_block_take_presplit(fgv_block_state *S, const uint8_t *block, size_t len, std::vector<Span> &out);
bool fgv_block_take_presplit_batch(fgv_block_state *S, size_t nb, const uint8_t *const *blocks, const size_t *lens,
                                   const uint32_t **et, const size_t **ntx, const size_t **first);

using namespace fgvb;

namespace {
constexpr uint32_t kRoundsPerEnqueue = 6;  // fixpoint rounds enqueued before the first host check
constexpr uint64_t kMaxArena = 32ull << 30;  // StateSlot.off8 addresses 8-byte units with 32 bits
constexpr size_t kCounterBytes = 256;       // MvCounters, padded (head and tail)
}  // namespace

// per-block device buffers: the single-block path uses set 0, a batch of consecutive blocks
// (fgv_mvcc_validate_blocks) rotates through kSets of them, so the extraction of the next blocks
// runs ahead of the block being checked and committed (blocks 1 .. kSets-1 of a call in one
// launch: mvcc_multi.h)
constexpr int kSets = MVX_MULTI_MAX;
struct MvSet {
  DevBuf head, info, reads, writes, wslot, rslot, bad, st, pend, tail;
  DevBuf xscr;  // k_mvx_extract's per-tx record scratch
  DevBuf blk;   // the block's bytes when the caller gives no device copy (batch path)
  hipEvent_t ev_x = nullptr;     // the block's extraction is done (stream2)
  hipEvent_t ev_free = nullptr;  // the set's last reader on the main stream is done
  void release() {
    DevBuf *d[] = {&head, &info, &reads, &writes, &wslot, &rslot, &bad, &st, &pend, &tail, &xscr, &blk};
    for (auto *b : d) b->release();
    if (ev_x) hipEventDestroy(ev_x);
    if (ev_free) hipEventDestroy(ev_free);
    ev_x = ev_free = nullptr;
  }
};

struct fgv_mvcc_state {
  uint64_t cap = 0, mask = 0, arena_cap = 0;
  uint64_t nkeys = 0, arena_used = 0;  // read back from `top` after every commit / load
  DevBuf tbl, arena, top;              // top: [0] arena bytes used, [1] occupied slots
  DevBuf btbl;
  DevBuf dheads;                       // batch path: every block's head (one copy per call)
  hipEvent_t ev_heads = nullptr;       // batch path: the heads' copy is done (second extraction stream)
  hipEvent_t ev_multi[5] = {};         // batch path: the multi-block extraction groups are done
  MvSet set[kSets];
  DevBuf lrecs, lbytes;                // load / apply staging
  DevBuf qver, qpres, qrange, qout;    // phantom path: lookups and range scans
  HostBuf hhead, htail;
  HostBuf bhead, btail;                // batch path: per-block head / tail regions
  std::vector<Span> pre_envs;          // envelope spans taken from a pre-split
  uint32_t epoch = 0;                  // block-table epoch (BlkSlot.owner)
  uint32_t rg = 0;                     // global fixpoint round tag (BlkSlot.fw_*)
  uint64_t btbl_cap = 0;
  uint32_t last_rounds = 0;
  // batch pass (mvcc_batch): one head / tail per call, the batch write table, blocks staged
  // contiguously when the caller gives no device copies
  DevBuf mbdhead, mbtbl, mbblk, mbrstat;
  HostBuf mbhead, mbtail;
  uint64_t mbtbl_cap = 0;
  uint32_t mb_epoch = 0, mb_rounds = 0;
  // update-batch bytes (fgv_mvcc_set_update_bytes, mvcc_ub.hip): one generation per committing
  // call, two alternating, so a host thread hashes call k's bytes while call k+1 runs
  struct UbGen {
    DevBuf arena, used;      // the serialisation arena and its claim counter
    HostBuf meta;            // UbMeta per block of the call (pinned, written by k_ub_sort)
    HostBuf host;            // the arena, copied back by the first acquire
    HostBuf usedh;           // the claim counter, read back with it
    hipEvent_t kev = nullptr, cev = nullptr;  // the call's serialisation / a copy back is done
    bool copied = false;
    uint64_t ticket = 0;     // the call (0: none)
    uint64_t cap = 0;
    size_t nb = 0;
    int readers = 0;         // fgv_mvcc_update_bytes_acquire holders
  } ub[2];
  DevBuf ub_dmeta, ub_ents;  // one launch's per-block results and sorted entries (k_ub_sort -> k_ub_write)
  bool ub_on = false;
  int ub_cur = -1;           // generation of the call in progress (-1: none)
  uint64_t ub_calls = 0, ub_last = 0;
  std::mutex ub_mu;
  std::condition_variable ub_cv;
  hipStream_t ub_stream = nullptr;    // the batch pass's serialisation
  hipStream_t ub_cp = nullptr;        // the copies back (fgv_mvcc_update_bytes_acquire)
  std::mutex ub_cp_mu;
  hipEvent_t ub_in = nullptr, ub_tail = nullptr;  // (into / the last work queued on ub_stream)
  bool ub_tail_set = false, ub_side = false;
};

void fgv_mvcc_free(fgv_mvcc_state *M) {
  if (!M) return;
  DevBuf *d[] = {&M->tbl, &M->arena, &M->top, &M->btbl, &M->dheads, &M->lrecs, &M->lbytes, &M->qver, &M->qpres, &M->qrange, &M->qout,
                 &M->mbdhead, &M->mbtbl, &M->mbblk, &M->mbrstat};
  for (auto *b : d) b->release();
  for (auto &S : M->set) S.release();
  if (M->ev_heads) hipEventDestroy(M->ev_heads);
  for (hipEvent_t &e : M->ev_multi)
    if (e) hipEventDestroy(e);
  HostBuf *h[] = {&M->hhead, &M->htail, &M->bhead, &M->btail, &M->mbhead, &M->mbtail};
  for (auto *b : h) b->release();
  if (M->ub_stream) hipStreamSynchronize(M->ub_stream);
  if (M->ub_cp) hipStreamSynchronize(M->ub_cp);
  for (auto &G : M->ub) {
    G.arena.release();
    G.used.release();
    G.meta.release();
    G.host.release();
    G.usedh.release();
    if (G.kev) hipEventDestroy(G.kev);
    if (G.cev) hipEventDestroy(G.cev);
  }
  M->ub_dmeta.release();
  M->ub_ents.release();
  if (M->ub_in) hipEventDestroy(M->ub_in);
  if (M->ub_tail) hipEventDestroy(M->ub_tail);
  if (M->ub_stream) hipStreamDestroy(M->ub_stream);
  if (M->ub_cp) hipStreamDestroy(M->ub_cp);
  delete M;
}

static inline dim3 grid_for(size_t n) { return dim3((uint32_t)((n + 255) / 256)); }
static inline dim3 grid_stride(size_t n, uint32_t max_blocks = 2048) {
  const size_t b = (n + 255) / 256;
  return dim3((uint32_t)std::max<size_t>(1, std::min<size_t>(b, max_blocks)));
}

// occupied slots / arena bytes after the last commit or load
static int read_top(fgv_ctx *c, fgv_mvcc_state *M) {
  uint64_t t[2];
  HIP_TRY(hipMemcpyAsync(t, M->top.p, 16, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  M->arena_used = t[0];
  M->nkeys = t[1];
  return FGV_OK;
}

// Host-supplied keys of one flattened namespace, each with a version or a delete:
// fgv_statedb_load (no deletes) and fgv_statedb_apply.  Existing entries are updated in place.
static int upsert_host(fgv_ctx *c, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                       const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn, const uint8_t *is_delete,
                       size_t n) {
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  if (n == 0) return FGV_OK;
  if (n >= 0x7FFFFFFFull) return FGV_EINVAL;
  const size_t nsl = strlen(ns);
  if (nsl > 0xFFFF) return FGV_EUNSUPPORTED;
  // keys of one call must be distinct (phase 2 inserts without compares)
  std::unordered_set<std::string_view> seen;
  seen.reserve(n * 2);
  size_t kb = 0, need = 0;
  for (size_t i = 0; i < n; i++) {
    if (key_len[i] > 0xFFFF || nsl + key_len[i] > 0xFFFF) return FGV_EUNSUPPORTED;
    if (!seen.emplace(reinterpret_cast<const char *>(key_buf + key_off[i]), key_len[i]).second) return FGV_EINVAL;
    kb = std::max<size_t>(kb, key_off[i] + key_len[i]);
    if (!is_delete || !is_delete[i]) need += (nsl + key_len[i] + 7) & ~(size_t)7;
  }
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  int rc = read_top(c, M);
  if (rc) return rc;
  if ((M->nkeys + n) * 10 > M->cap * 7 || M->arena_used + need > M->arena_cap) return FGV_ENOMEM;
  // staging: [ns | key bytes] in lbytes; one record per key (ns_off 0)
  const size_t kofs = (nsl + 7) & ~(size_t)7;
  if (!M->lbytes.ensure(kofs + kb + 64) || !M->lrecs.ensure(n * sizeof(MvRec)) || !M->set[0].pend.ensure(n + 64))
    return FGV_ENOMEM;
  if (kofs + kb > 0xFFFFFFFFull) return FGV_EINVAL;
  std::vector<MvRec> recs(n);
  for (size_t i = 0; i < n; i++) {
    MvRec &r = recs[i];
    memset(&r, 0, sizeof r);
    r.ns_off = 0;
    r.ns_len = (uint16_t)nsl;
    r.key_off = (uint32_t)(kofs + key_off[i]);
    r.key_len = (uint16_t)key_len[i];
    r.flags = (is_delete && is_delete[i]) ? MVR_DELETE : 0;
    r.blk = blk[i];
    r.txn = txn[i];
  }
  hipStream_t s = c->stream;
  uint8_t *lb = M->lbytes.as<uint8_t>();
  if (nsl) HIP_TRY(hipMemcpyAsync(lb, ns, nsl, hipMemcpyHostToDevice, s));
  if (kb) HIP_TRY(hipMemcpyAsync(lb + kofs, key_buf, kb, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(M->lrecs.p, recs.data(), n * sizeof(MvRec), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_mv_tags, grid_for(n), dim3(256), 0, s, lb, M->lrecs.as<MvRec>(), (uint32_t)n);
  hipLaunchKernelGGL(k_mv_upsert_find, grid_stride(n), dim3(256), 0, s, 0u, 0u, (uint32_t)n, lb, M->lrecs.as<MvRec>(),
                     nullptr, nullptr, nullptr, 0u, M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(), 0ull,
                     M->set[0].pend.as<uint8_t>(), nullptr);
  hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(n), dim3(256), 0, s, 0u, 0u, (uint32_t)n, lb,
                     M->lrecs.as<MvRec>(), M->set[0].pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask,
                     M->arena.as<uint8_t>(), M->top.as<unsigned long long>(), 0ull, nullptr, nullptr, nullptr, 0u);
  HIP_TRY(hipGetLastError());
  return read_top(c, M);
}

extern "C" {

int fgv_statedb_init(fgv_ctx *c, uint64_t slots, uint64_t arena_bytes) {
  if (!c) return FGV_EINVAL;
  const uint64_t arena = arena_bytes ? arena_bytes : (64ull << 20);
  if (arena > kMaxArena || slots > (1ull << 40)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  if (!c->mv) c->mv = new fgv_mvcc_state();
  fgv_mvcc_state *M = c->mv;
  uint64_t cap = 1024;
  while (cap < (slots ? slots : (1ull << 22))) cap <<= 1;
  if (!M->tbl.ensure(cap * sizeof(StateSlot) + 64) ||  // (+64: word loads past the last slot's inline key)
      !M->arena.ensure(arena + 64) || !M->top.ensure(64)) return FGV_ENOMEM;
  M->cap = cap;
  M->mask = cap - 1;
  M->arena_cap = arena;
  M->arena_used = 0;
  M->nkeys = 0;
  HIP_TRY(hipMemsetAsync(M->tbl.p, 0, cap * sizeof(StateSlot), c->stream));
  HIP_TRY(hipMemsetAsync(M->top.p, 0, 64, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FGV_OK;
}

int fgv_statedb_load(fgv_ctx *c, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                     const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn, size_t n) {
  if (!c || !ns || (n && (!key_buf || !key_off || !key_len || !blk || !txn))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return upsert_host(c, ns, key_buf, key_off, key_len, blk, txn, nullptr, n);
}

int fgv_statedb_apply(fgv_ctx *c, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                      const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn, const uint8_t *is_delete,
                      size_t n) {
  if (!c || !ns || (n && (!key_buf || !key_off || !key_len || !blk || !txn || !is_delete))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return upsert_host(c, ns, key_buf, key_off, key_len, blk, txn, is_delete, n);
}

int fgv_statedb_stats(fgv_ctx *c, uint64_t *keys, uint64_t *arena_used, uint64_t *slots, uint64_t *arena_cap) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  int rc = read_top(c, M);
  if (rc) return rc;
  if (keys) *keys = M->nkeys;
  if (arena_used) *arena_used = M->arena_used;
  if (slots) *slots = M->cap;
  if (arena_cap) *arena_cap = M->arena_cap;
  return FGV_OK;
}

}  // extern "C"

// ======================================================================= phantom path
// A block with range queries (validator.go:205-244) is validated here, in block order, exactly
// as validateAndPrepareBatch does (validator.go:81-162): per namespace public reads (11), range
// queries (PHANTOM_READ_CONFLICT 12), hashed reads (11); a valid tx's writes enter the update
// batch at Height{block, tx}.  The device pass already classified every transaction (codes 16 /
// 255, committer-invalid skips, unsupported shapes) and located its TxReadWriteSet; the
// committed versions come from the GPU table (k_mv_lookup), the committed keys of each range
// from one scan of it (k_mv_range_scan).  The combined iterator (combined_iterator.go), the raw
// and the merkle-hash validators (rangequery_validator.go, rwsetutil/query_results_helper.go)
// are restated below.
namespace {

using pbw::Kind;
using pbw::K_BYTES;
using pbw::K_MSG;
using pbw::K_NONE;
using pbw::K_REP_BYTES;
using pbw::K_REP_MSG;
using pbw::K_STRING;
using pbw::K_VARINT;

// host visitors with the field rules of mvcc.hip's (the device walked these rwsets cleanly)
struct HVer {
  uint64_t b = 0, t = 0;
  Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : K_NONE; }
  void on_varint(uint32_t n, uint64_t v) { (n == 1 ? b : t) = v; }
  bool on_len(uint32_t, Span) { return true; }
};
struct HRead {
  bool hashed = false;
  Span key;
  bool has_ver = false;
  HVer v;
  Kind kind(uint32_t n) { return n == 1 ? (hashed ? K_BYTES : K_STRING) : n == 2 ? K_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    has_ver = true;
    return pbw::decode(s.p, s.n, v);
  }
};
struct HWrite {
  bool hashed = false;
  Span key, val;
  bool del = false;
  Kind kind(uint32_t n) {
    if (n == 1) return hashed ? K_BYTES : K_STRING;
    if (n == 2) return K_VARINT;
    if (n == 3) return K_BYTES;
    return (hashed && n == 4) ? K_VARINT : K_NONE;
  }
  void on_varint(uint32_t n, uint64_t v) { if (n == 2) del = v != 0; }
  bool on_len(uint32_t n, Span s) { (n == 1 ? key : val) = s; return true; }
};
struct HQReads {
  std::vector<HRead> *out;
  Kind kind(uint32_t n) { return n == 1 ? K_REP_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    HRead r;
    if (!pbw::decode(s.p, s.n, r)) return false;
    out->push_back(r);
    return true;
  }
};
struct HMerk {  // QueryReadsMerkleSummary {max_degree uint32 1, max_level uint32 2, max_level_hashes 3}
  uint32_t degree = 0, level = 0;
  std::vector<Span> hashes;
  Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : n == 3 ? K_REP_BYTES : K_NONE; }
  void on_varint(uint32_t n, uint64_t v) { (n == 1 ? degree : level) = (uint32_t)v; }
  bool on_len(uint32_t, Span s) { hashes.push_back(s); return true; }
};
struct HRQ {  // RangeQueryInfo
  Span start, end;
  bool exhausted = false, raw = false, merk = false;
  std::vector<HRead> reads;
  HMerk m;
  Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_STRING : n == 3 ? K_VARINT : (n == 4 || n == 5) ? K_MSG : K_NONE; }
  void on_varint(uint32_t n, uint64_t v) { if (n == 3) exhausted = v != 0; }
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { start = s; return true; }
    if (n == 2) { end = s; return true; }
    if (n == 4) {
      raw = true;
      HQReads q{&reads};
      return pbw::decode(s.p, s.n, q);
    }
    merk = true;
    return pbw::decode(s.p, s.n, m);
  }
};
struct HMetaEntry {  // KVMetadataEntry {name string 1, value bytes 2}
  Span name, value;
  Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? name : value) = s; return true; }
};
struct HMetaW {  // KVMetadataWrite {key string 1, entries 2} / KVMetadataWriteHash {key_hash bytes 1, entries 2}
  bool hashed = false;
  Span key;
  Span vp;  // the VALIDATION_PARAMETER entry (the last one: statemetadata.Deserialize's map)
  Kind kind(uint32_t n) { return n == 1 ? (hashed ? K_BYTES : K_STRING) : n == 2 ? K_REP_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    HMetaEntry e;
    if (!pbw::decode(s.p, s.n, e)) return false;
    if (e.name.eq("VALIDATION_PARAMETER", 20)) vp = e.value;
    return true;
  }
};
struct HRW {  // KVRWSet / HashedRWSet
  bool hashed = false;
  std::vector<HRead> reads;
  std::vector<HRQ> rqs;
  std::vector<HWrite> writes;
  std::vector<Span> meta;  // keys of the metadata writes
  std::vector<Span> meta_vp;  // their VALIDATION_PARAMETER values (empty: none)
  Kind kind(uint32_t n) { return (n >= 1 && n <= (hashed ? 3u : 4u)) ? K_REP_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) {
      HRead r;
      r.hashed = hashed;
      if (!pbw::decode(s.p, s.n, r)) return false;
      reads.push_back(r);
      return true;
    }
    if (!hashed && n == 2) {
      HRQ q;
      if (!pbw::decode(s.p, s.n, q)) return false;
      rqs.push_back(std::move(q));
      return true;
    }
    if (n == (hashed ? 2u : 3u)) {
      HWrite w;
      w.hashed = hashed;
      if (!pbw::decode(s.p, s.n, w)) return false;
      writes.push_back(w);
      return true;
    }
    HMetaW m;
    m.hashed = hashed;
    if (!pbw::decode(s.p, s.n, m)) return false;
    meta.push_back(m.key);
    meta_vp.push_back(m.vp);
    return true;
  }
};
struct HColl {
  Span name, hashed;
  Kind kind(uint32_t n) { return n == 1 ? K_STRING : (n == 2 || n == 3) ? K_BYTES : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) name = s;
    else if (n == 2) hashed = s;
    return true;
  }
};
struct HNs {
  Span ns, rwset;
  std::vector<HColl> colls;
  Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : n == 3 ? K_REP_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) ns = s;
    else if (n == 2) rwset = s;
    else {
      HColl c;
      if (!pbw::decode(s.p, s.n, c)) return false;
      colls.push_back(c);
    }
    return true;
  }
};
struct HTxRW {
  std::vector<HNs> ns;
  Kind kind(uint32_t n) { return n == 1 ? K_VARINT : n == 2 ? K_REP_MSG : K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    HNs h;
    if (!pbw::decode(s.p, s.n, h)) return false;
    ns.push_back(std::move(h));
    return true;
  }
};

struct Ver {
  uint64_t b = 0, t = 0;
  bool operator==(const Ver &o) const { return b == o.b && t == o.t; }
};
struct Upd {
  Ver v;
  bool del = false;
};
struct TxNs {  // one NsReadWriteSet, decoded
  std::string ns;
  HRW kv;
  std::vector<std::pair<std::string, HRW>> colls;  // flattened hashed ns, hashed rwset
  std::vector<std::string> coll_names;
};
// a change of a key's VALIDATION_PARAMETER in the committed state (fgv_kvmeta_set)
struct KvOp {
  std::string ns, coll, key;
  Span vp;  // empty: none
};
std::string sv(const Span &s) { return std::string(reinterpret_cast<const char *>(s.p), s.n); }
// (namespace, key) as one map key: 4-byte namespace length, namespace, key (keys and hashed
// keys may hold any byte)
std::string flat_key(const std::string &ns, const std::string &key) {
  const uint32_t n = (uint32_t)ns.size();
  std::string o(reinterpret_cast<const char *>(&n), 4);
  return o + ns + key;
}
void split_flat(const std::string &fk, std::string &ns, std::string &key) {
  uint32_t n;
  memcpy(&n, fk.data(), 4);
  ns = fk.substr(4, n);
  key = fk.substr(4 + n);
}

constexpr uint8_t kEmptySha256[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                      0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                      0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
bool is_delete(const HWrite &w) {  // IsKVWriteDelete / IsKVWriteHashDelete
  if (w.del || w.val.n == 0) return true;
  return w.hashed && w.val.n == 32 && memcmp(w.val.p, kEmptySha256, 32) == 0;
}

// ---- merkle summary (rwsetutil/query_results_helper.go)
void put_varint(std::string &o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(uint8_t)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)(uint8_t)v);
}
void put_len(std::string &o, uint32_t field, const std::string &b) {
  put_varint(o, (uint64_t)field << 3 | 2);
  put_varint(o, b.size());
  o += b;
}
using KV = std::pair<std::string, Ver>;
// proto.Marshal(&kvrwset.QueryReads{KvReads}): KVRead{key 1 (omitted when empty), version 2
// (present: NewKVRead of a committed / updated height)}, Version{block_num 1, tx_num 2}
std::string marshal_query_reads(const std::vector<KV> &kvs) {
  std::string out;
  for (const KV &kv : kvs) {
    std::string ver, msg;
    if (kv.second.b) { put_varint(ver, 1 << 3); put_varint(ver, kv.second.b); }
    if (kv.second.t) { put_varint(ver, 2 << 3); put_varint(ver, kv.second.t); }
    if (!kv.first.empty()) put_len(msg, 1, kv.first);
    put_len(msg, 2, ver);
    put_len(out, 1, msg);
  }
  return out;
}
std::string sha(const std::string &b) {
  uint8_t d[32];
  fgvsha::sha256(reinterpret_cast<const uint8_t *>(b.data()), b.size(), d);
  return std::string(reinterpret_cast<const char *>(d), 32);
}
struct Merkle {
  std::map<uint32_t, std::vector<std::string>> tree;
  uint32_t max_level = 1, max_degree;
  explicit Merkle(uint32_t d) : max_degree(d) {}
  static std::string combine(const std::vector<std::string> &hs) {
    std::string b;
    for (const auto &h : hs) b += h;
    return sha(b);
  }
  void update(const std::string &h) {
    tree[1].push_back(h);
    uint32_t level = 1;
    for (;;) {
      auto it = tree.find(level);
      if (it == tree.end() || it->second.size() <= max_degree) return;
      const std::string next = combine(it->second);
      tree.erase(it);
      level++;
      tree[level].push_back(next);
      if (level > max_level) max_level = level;
    }
  }
  void done() {
    uint32_t level = 1;
    while (level < max_level) {
      auto it = tree.find(level);
      if (it == tree.end() || it->second.empty()) {
        level++;
        continue;
      }
      const std::string h = it->second.size() == 1 ? it->second[0] : combine(it->second);
      tree.erase(it);
      level++;
      tree[level].push_back(h);
    }
    auto it = tree.find(max_level);
    if (it != tree.end() && it->second.size() > max_degree) {
      const std::string h = combine(it->second);
      tree.erase(it);
      max_level++;
      tree[max_level] = {h};
    }
  }
  const std::vector<std::string> &top() {
    static const std::vector<std::string> none;
    auto it = tree.find(max_level);
    return it == tree.end() ? none : it->second;
  }
  bool empty() {
    auto it = tree.find(1);
    return max_level == 1 && (it == tree.end() || it->second.empty());
  }
};

// the combined iterator's output for one range query (combined_iterator.go)
std::vector<KV> combined(const std::vector<KV> &db, const std::map<std::string, Upd> *upd, const std::string &start,
                         const std::string &end, bool unbounded, bool include_end, bool end_known, const Upd &end_val) {
  std::vector<KV> out;
  std::map<std::string, Upd>::const_iterator u, ue;
  if (upd) {
    u = start.empty() ? upd->begin() : upd->lower_bound(start);
    ue = unbounded ? upd->end() : upd->lower_bound(end);
    if (!unbounded && !start.empty() && start > end) u = ue;  // SearchStrings: next >= last -> empty
  }
  size_t i = 0;
  const bool has_u = upd != nullptr;
  for (;;) {
    const bool db_left = i < db.size(), u_left = has_u && u != ue;
    if (!db_left && !u_left) break;
    int cmp;
    if (!u_left) cmp = -1;
    else if (!db_left) cmp = 1;
    else cmp = db[i].first < u->first ? -1 : (u->first < db[i].first ? 1 : 0);
    if (cmp < 0) {
      out.push_back(db[i++]);
      continue;
    }
    const std::string &k = u->first;
    const Upd uv = u->second;
    ++u;
    if (cmp == 0) i++;
    if (!uv.del) out.push_back(KV{k, uv.v});
  }
  if (include_end && end_known && !end_val.del) out.push_back(KV{end, end_val.v});
  return out;
}

// rangeQueryResultsValidator / rangeQueryHashValidator: 1 valid, 0 phantom, -1 the reference
// errors out (maxDegree < 2; a raw read without a version dereferences nil)
int rq_validate(const HRQ &q, const std::vector<KV> &res) {
  if (q.merk) {
    if (q.m.degree < 2) return -1;
    Merkle mt(q.m.degree);
    std::vector<KV> pending;
    int last = -1;
    for (const KV &kv : res) {
      pending.push_back(kv);
      if (pending.size() > q.m.degree) {
        mt.update(sha(marshal_query_reads(pending)));
        pending.clear();
      }
      if (mt.max_level < q.m.level) continue;
      const std::vector<std::string> &h = mt.top();
      if (last == (int)h.size() - 1) continue;
      if (h.size() > q.m.hashes.size()) return 0;
      last++;
      if (!q.m.hashes[last].eq(h[last].data(), h[last].size())) return 0;
    }
    if (mt.empty()) return 0;  // Done() -> nil summary: never equal
    if (!pending.empty()) mt.update(sha(marshal_query_reads(pending)));
    mt.done();
    const std::vector<std::string> &h = mt.top();
    if (mt.max_level != q.m.level || h.size() != q.m.hashes.size()) return 0;
    for (size_t k = 0; k < h.size(); k++)
      if (!q.m.hashes[k].eq(h[k].data(), h[k].size())) return 0;
    return 1;
  }
  if (q.reads.empty()) return res.empty() ? 1 : 0;
  size_t j = 0;
  for (const HRead &r : q.reads) {
    if (j >= res.size() || !r.key.eq(res[j].first.data(), res[j].first.size())) return 0;
    if (!r.has_ver) return -1;
    if (!(res[j].second == Ver{r.v.b, r.v.t})) return 0;
    j++;
  }
  return j == res.size() ? 1 : 0;
}

}  // namespace

// Sanitizer probe (tools/sanitize): the phantom path's host decode of one TxReadWriteSet --
// namespaces, KV and hashed rwsets, range queries with their raw reads or merkle summaries --
// and both range-query validators over an empty and a one-result iterator.  No GPU call.
uint64_t fgv_mvcc_parse_probe(const uint8_t *rws, size_t n) {
  HTxRW rw;
  if (!pbw::decode(rws, n, rw)) return 0;
  uint64_t h = 1;
  for (HNs &ns : rw.ns) {
    HRW kv;
    kv.hashed = false;
    if (!pbw::decode(ns.rwset.p, ns.rwset.n, kv)) continue;
    h = h * 31 + kv.reads.size() + 7 * kv.writes.size() + 13 * kv.rqs.size();
    for (const HRQ &q : kv.rqs) {
      const std::vector<KV> none, one{KV{"k", Ver{1, 1}}};
      h = h * 31 + (uint64_t)(rq_validate(q, none) + 2) + 5 * (uint64_t)(rq_validate(q, one) + 2);
    }
    for (const HColl &cl : ns.colls) {
      HRW hr;
      hr.hashed = true;
      if (pbw::decode(cl.hashed.p, cl.hashed.n, hr)) h = h * 31 + hr.reads.size() + 7 * hr.writes.size();
    }
  }
  return h;
}

static int phantom_block(fgv_ctx *c, fgv_mvcc_state *M, const uint8_t *block, uint64_t block_num,
                         const uint8_t *in_flags, uint8_t *flags, size_t ntx, int commit) {
  hipStream_t s = c->stream;
  std::vector<MvTxInfo> info(ntx);
  HIP_TRY(hipMemcpyAsync(info.data(), M->set[0].info.p, ntx * sizeof(MvTxInfo), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  // 1. decode the participating transactions' rwsets
  std::vector<std::vector<TxNs>> txs(ntx);
  for (size_t i = 0; i < ntx; i++) {
    if (info[i].code != 0) continue;
    HTxRW rw;
    if (!pbw::decode(block + info[i].rws_off, info[i].rws_len, rw)) return FGV_EUNSUPPORTED;  // (cannot happen)
    for (HNs &h : rw.ns) {
      TxNs e;
      e.ns = sv(h.ns);
      e.kv.hashed = false;
      if (!pbw::decode(h.rwset.p, h.rwset.n, e.kv)) return FGV_EUNSUPPORTED;
      for (const HColl &cl : h.colls) {
        HRW hr;
        hr.hashed = true;
        if (!pbw::decode(cl.hashed.p, cl.hashed.n, hr)) return FGV_EUNSUPPORTED;
        e.colls.emplace_back(e.ns + "$$h" + sv(cl.name), std::move(hr));
        e.coll_names.push_back(sv(cl.name));
      }
      txs[i].push_back(std::move(e));
    }
  }
  // metadata writes not combined with a KVWrite of the same key in the same tx (those follow
  // the write: upsert+metadata puts, delete+metadata deletes); a key with two metadata writes
  // or two KVWrites (txOps adds the flags: tx_ops.go:183-203) is outside the model
  struct TxMeta {
    bool hashed;
    std::string ns, key;
  };
  std::vector<std::vector<TxMeta>> metas(ntx);
  for (size_t i = 0; i < ntx; i++) {
    std::unordered_set<std::string> written, meta_seen;
    for (const TxNs &e : txs[i]) {
      for (const HWrite &w : e.kv.writes) written.insert(flat_key("p" + e.ns, sv(w.key)));
      for (const auto &cl : e.colls)
        for (const HWrite &w : cl.second.writes) written.insert(flat_key("h" + cl.first, sv(w.key)));
    }
    for (const TxNs &e : txs[i]) {
      for (const Span &k : e.kv.meta) {
        const std::string fk = flat_key("p" + e.ns, sv(k));
        if (!meta_seen.insert(fk).second) return FGV_EUNSUPPORTED;
        if (!written.count(fk)) metas[i].push_back(TxMeta{false, e.ns, sv(k)});
      }
      for (const auto &cl : e.colls)
        for (const Span &k : cl.second.meta) {
          const std::string fk = flat_key("h" + cl.first, sv(k));
          if (!meta_seen.insert(fk).second) return FGV_EUNSUPPORTED;
          if (!written.count(fk)) metas[i].push_back(TxMeta{true, cl.first, sv(k)});
        }
    }
  }
  // 2. committed versions of every point-read key, range end key and metadata-only key;
  // committed keys of every range
  std::unordered_map<std::string, uint32_t> qidx;  // flat key -> lookup index
  std::vector<std::pair<std::string, std::string>> qkeys;
  auto want = [&](const std::string &ns, const std::string &key) {
    const std::string fk = flat_key(ns, key);
    if (qidx.emplace(fk, (uint32_t)qkeys.size()).second) qkeys.emplace_back(ns, key);
  };
  struct RangeQ {
    std::string ns, start, end;
    bool unbounded;
  };
  std::vector<RangeQ> ranges;
  for (size_t i = 0; i < ntx; i++)
    for (const TxNs &e : txs[i]) {
      for (const HRead &r : e.kv.reads) want(e.ns, sv(r.key));
      for (const HRQ &q : e.kv.rqs) {
        ranges.push_back(RangeQ{e.ns, sv(q.start), sv(q.end), q.end.n == 0});
        if (!q.exhausted) want(e.ns, sv(q.end));
      }
      for (const auto &cl : e.colls)
        for (const HRead &r : cl.second.reads) want(cl.first, sv(r.key));
    }
  for (size_t i = 0; i < ntx; i++)
    for (const TxMeta &m : metas[i]) want(m.ns, m.key);
  for (const auto &k : qkeys)
    if (k.first.size() > 0xFFFF || k.second.size() > 0xFFFF || k.first.size() + k.second.size() > 0xFFFF)
      return FGV_EUNSUPPORTED;
  // staging: bytes [ns | key]... then the range bounds; one MvRec per lookup (flattened ns)
  std::string bytes;
  std::vector<MvRec> recs(qkeys.size());
  for (size_t k = 0; k < qkeys.size(); k++) {
    MvRec &r = recs[k];
    memset(&r, 0, sizeof r);
    r.ns_off = (uint32_t)bytes.size();
    r.ns_len = (uint16_t)qkeys[k].first.size();
    bytes += qkeys[k].first;
    r.key_off = (uint32_t)bytes.size();
    r.key_len = (uint16_t)qkeys[k].second.size();
    bytes += qkeys[k].second;
  }
  std::vector<MvRange> rdesc(ranges.size());
  for (size_t k = 0; k < ranges.size(); k++) {
    MvRange &d = rdesc[k];
    memset(&d, 0, sizeof d);
    d.ns_off = (uint32_t)bytes.size();
    d.ns_len = (uint32_t)ranges[k].ns.size();
    bytes += ranges[k].ns;
    d.s_off = (uint32_t)bytes.size();
    d.s_len = (uint32_t)ranges[k].start.size();
    bytes += ranges[k].start;
    d.e_off = (uint32_t)bytes.size();
    d.e_len = (uint32_t)ranges[k].end.size();
    bytes += ranges[k].end;
    d.flags = ranges[k].unbounded ? MVRANGE_UNBOUNDED : 0u;
  }
  if (bytes.size() >= 0xFFFFFFFFull) return FGV_EUNSUPPORTED;
  const size_t nq = qkeys.size();
  if (!M->lbytes.ensure(bytes.size() + 64) || !M->lrecs.ensure((nq + 1) * sizeof(MvRec)) ||
      !M->qver.ensure((nq + 1) * 16) || !M->qpres.ensure(nq + 64) || !M->qrange.ensure((ranges.size() + 1) * sizeof(MvRange)) ||
      !M->qout.ensure(1 << 20) || !M->top.ensure(64))
    return FGV_ENOMEM;
  uint8_t *lb = M->lbytes.as<uint8_t>();
  if (!bytes.empty()) HIP_TRY(hipMemcpyAsync(lb, bytes.data(), bytes.size(), hipMemcpyHostToDevice, s));
  std::vector<uint64_t> qver(2 * nq);
  std::vector<uint8_t> qpres(nq);
  if (nq) {
    HIP_TRY(hipMemcpyAsync(M->lrecs.p, recs.data(), nq * sizeof(MvRec), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_mv_tags, grid_for(nq), dim3(256), 0, s, lb, M->lrecs.as<MvRec>(), (uint32_t)nq);
    hipLaunchKernelGGL(k_mv_lookup, grid_stride(nq), dim3(256), 0, s, (uint32_t)nq, lb, M->lrecs.as<MvRec>(),
                       M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(), M->qver.as<uint64_t>(),
                       M->qpres.as<uint8_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(qver.data(), M->qver.p, nq * 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(qpres.data(), M->qpres.p, nq, hipMemcpyDeviceToHost, s));
  }
  std::vector<std::vector<KV>> scanned(ranges.size());
  if (!ranges.empty()) {
    HIP_TRY(hipMemcpyAsync(M->qrange.p, rdesc.data(), ranges.size() * sizeof(MvRange), hipMemcpyHostToDevice, s));
    unsigned long long *used = reinterpret_cast<unsigned long long *>(M->top.as<uint8_t>() + 32);
    std::vector<uint8_t> out;
    for (int attempt = 0; attempt < 2; attempt++) {
      HIP_TRY(hipMemsetAsync(used, 0, 8, s));
      hipLaunchKernelGGL(k_mv_range_scan, grid_stride(M->cap, 4096), dim3(256), 0, s, M->cap, M->tbl.as<StateSlot>(),
                         M->arena.as<uint8_t>(), (uint32_t)ranges.size(), M->qrange.as<MvRange>(), lb,
                         M->qout.as<uint8_t>(), (uint64_t)M->qout.cap, used);
      HIP_TRY(hipGetLastError());
      unsigned long long u = 0;
      HIP_TRY(hipMemcpyAsync(&u, used, 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      if (u <= M->qout.cap) {
        out.resize(u);
        if (u) HIP_TRY(hipMemcpy(out.data(), M->qout.p, u, hipMemcpyDeviceToHost));
        break;
      }
      if (attempt == 1 || !M->qout.ensure(u + (1 << 20))) return FGV_ENOMEM;
    }
    for (size_t o = 0; o + 24 <= out.size();) {
      uint32_t h[2];
      uint64_t v[2];
      memcpy(h, out.data() + o, 8);
      memcpy(v, out.data() + o + 8, 16);
      if (h[0] >= ranges.size() || o + 24 + h[1] > out.size()) return FGV_EDEVICE;
      scanned[h[0]].push_back(KV{std::string(reinterpret_cast<const char *>(out.data() + o + 24), h[1]), Ver{v[0], v[1]}});
      o += 24 + ((h[1] + 7u) & ~7u);
    }
    for (auto &v : scanned) std::sort(v.begin(), v.end(), [](const KV &a, const KV &b) { return a.first < b.first; });
  }
  HIP_TRY(hipStreamSynchronize(s));
  auto committed = [&](const std::string &ns, const std::string &key, Ver &v) -> bool {
    const uint32_t k = qidx.at(flat_key(ns, key));
    v = Ver{qver[2 * k], qver[2 * k + 1]};
    return qpres[k] != 0;
  };
  // 3. validateAndPrepareBatch, in block order
  std::map<std::string, std::map<std::string, Upd>> pub;  // ns -> key -> update (sorted: range scans)
  std::unordered_map<std::string, Upd> hsh;               // flat hashed ns + key
  auto read_ok = [&](const std::string &ns, const HRead &r, bool hashed) {
    const std::string key = sv(r.key);
    if (hashed) {
      if (hsh.count(flat_key(ns, key))) return false;
    } else {
      auto it = pub.find(ns);
      if (it != pub.end() && it->second.count(key)) return false;
    }
    Ver v;
    const bool present = committed(ns, key, v);
    if (!present || !r.has_ver) return present == r.has_ver;  // version.AreSame (nil <=> absent)
    return v == Ver{r.v.b, r.v.t};
  };
  std::vector<KvOp> kvops;                   // key-level parameter changes, in block order
  std::vector<size_t> rq_base(ntx + 1, 0);  // the first range index of each tx
  for (size_t i = 0; i < ntx; i++) {
    size_t k = 0;
    for (const TxNs &e : txs[i]) k += e.kv.rqs.size();
    rq_base[i + 1] = rq_base[i] + k;
  }
  for (size_t i = 0; i < ntx; i++) {
    size_t rq_at = rq_base[i];
    const uint8_t code = info[i].code;
    if (code == MV_SKIP) { flags[i] = in_flags[i]; continue; }
    if (code != 0) { flags[i] = code; continue; }
    uint8_t verdict = 0;
    for (const TxNs &e : txs[i]) {
      for (const HRead &r : e.kv.reads)
        if (!read_ok(e.ns, r, false)) { verdict = 11; break; }
      if (verdict) break;
      for (const HRQ &q : e.kv.rqs) {
        const size_t ri = rq_at++;
        if (verdict) continue;
        auto pit = pub.find(e.ns);
        const std::string end = sv(q.end);
        Upd ev;
        bool end_known = false;
        if (!q.exhausted) {  // serveEndKeyIfNeeded: updates.Get, else db.GetState
          auto u = pit != pub.end() ? pit->second.find(end) : std::map<std::string, Upd>::const_iterator();
          if (pit != pub.end() && u != pit->second.end()) {
            ev = u->second;
            end_known = true;
          } else {
            Ver v;
            end_known = committed(e.ns, end, v);
            ev = Upd{v, false};
          }
        }
        const std::vector<KV> res = combined(scanned[ri], pit != pub.end() ? &pit->second : nullptr, sv(q.start), end,
                                             q.end.n == 0, !q.exhausted, end_known, ev);
        const int ok = rq_validate(q, res);
        if (ok < 0) return FGV_EUNSUPPORTED;  // the reference returns an error (the peer stops)
        if (!ok) verdict = 12;
      }
      if (verdict) break;
      for (const auto &cl : e.colls) {
        for (const HRead &r : cl.second.reads)
          if (!read_ok(cl.first, r, true)) { verdict = 11; break; }
        if (verdict) break;
      }
      if (verdict) break;
    }
    if (verdict) {
      flags[i] = verdict;
      continue;
    }
    flags[i] = 0;
    // applyWriteSet / prepareTxOps (types.go:81-112, tx_ops.go:17-53): per key, a delete wins,
    // an upsert puts; a metadata-only write puts the key's latest value again -- a new version
    // -- if the key exists (preceding updates, else committed state) and is a no-op otherwise.
    // A key deleted earlier in the block makes the reference panic (PutValAndMetadata(nil)).
    const Ver h{block_num, (uint64_t)i};
    for (const TxNs &e : txs[i]) {
      for (const HWrite &w : e.kv.writes) pub[e.ns][sv(w.key)] = Upd{h, is_delete(w)};
      for (const auto &cl : e.colls)
        for (const HWrite &w : cl.second.writes) hsh[flat_key(cl.first, sv(w.key))] = Upd{h, is_delete(w)};
    }
    for (const TxMeta &m : metas[i]) {
      Upd *prev = nullptr;
      if (m.hashed) {
        auto it = hsh.find(flat_key(m.ns, m.key));
        if (it != hsh.end()) prev = &it->second;
      } else {
        auto it = pub.find(m.ns);
        if (it != pub.end()) {
          auto k = it->second.find(m.key);
          if (k != it->second.end()) prev = &k->second;
        }
      }
      bool exists;
      if (prev) {
        if (prev->del) return FGV_EUNSUPPORTED;
        exists = true;
      } else {
        Ver v;
        exists = committed(m.ns, m.key, v);
      }
      if (!exists) continue;
      if (m.hashed) hsh[flat_key(m.ns, m.key)] = Upd{h, false};
      else pub[m.ns][m.key] = Upd{h, false};
    }
    // the keys' metadata (statedb VALIDATION_PARAMETER, tx_ops.go:17-53 + 97-148): a delete drops
    // it, an upsert keeps it, a metadata write beside an upsert replaces it, a metadata-only
    // write replaces it when the key exists (its update now carries this tx's height)
    for (const TxNs &e : txs[i]) {
      auto track = [&](const std::string &coll, const std::string &fns, const HRW &rw) {
        for (const HWrite &w : rw.writes)
          if (is_delete(w)) kvops.push_back(KvOp{e.ns, coll, sv(w.key), Span{}});
        for (size_t m = 0; m < rw.meta.size(); m++) {
          const HWrite *w = nullptr;
          for (const HWrite &x : rw.writes)
            if (x.key.eq(rw.meta[m])) w = &x;
          if (w) {
            if (!is_delete(*w)) kvops.push_back(KvOp{e.ns, coll, sv(rw.meta[m]), rw.meta_vp[m]});
            continue;
          }
          const std::string key = sv(rw.meta[m]);
          bool ex = false;
          if (rw.hashed) {
            auto it = hsh.find(flat_key(fns, key));
            ex = it != hsh.end() && it->second.v == h;
          } else {
            auto it = pub.find(fns);
            if (it != pub.end()) {
              auto k = it->second.find(key);
              ex = k != it->second.end() && k->second.v == h;
            }
          }
          if (ex) kvops.push_back(KvOp{e.ns, coll, key, rw.meta_vp[m]});
        }
      };
      track("", e.ns, e.kv);
      for (size_t k = 0; k < e.colls.size(); k++) track(e.coll_names[k], e.colls[k].first, e.colls[k].second);
    }
  }
  if (!commit) return FGV_OK;
  // 4. commit the update batch: one upsert per flattened namespace (capacity checked first, so
  // a block is committed whole or not at all)
  std::map<std::string, std::vector<std::pair<std::string, Upd>>> groups;
  for (const auto &nsm : pub)
    for (const auto &kv : nsm.second) groups[nsm.first].emplace_back(kv.first, kv.second);
  for (const auto &kv : hsh) {
    std::string ns, key;
    split_flat(kv.first, ns, key);
    groups[ns].emplace_back(key, kv.second);
  }
  int rc = read_top(c, M);
  if (rc) return rc;
  size_t n_all = 0, need = 0;
  for (const auto &g : groups)
    for (const auto &kv : g.second) {
      n_all++;
      if (!kv.second.del) need += (g.first.size() + kv.first.size() + 7) & ~(size_t)7;
    }
  if ((M->nkeys + n_all) * 10 > M->cap * 7 || M->arena_used + need > M->arena_cap) return FGV_ENOMEM;
  for (const auto &g : groups) {
    std::string kb;
    std::vector<uint64_t> off, blk, txn;
    std::vector<uint32_t> len;
    std::vector<uint8_t> del;
    for (const auto &kv : g.second) {
      off.push_back(kb.size());
      len.push_back((uint32_t)kv.first.size());
      kb += kv.first;
      blk.push_back(kv.second.v.b);
      txn.push_back(kv.second.v.t);
      del.push_back(kv.second.del ? 1 : 0);
    }
    rc = upsert_host(c, g.first.c_str(), reinterpret_cast<const uint8_t *>(kb.data()), off.data(), len.data(), blk.data(),
                     txn.data(), del.data(), g.second.size());
    if (rc) return rc;
  }
  for (const KvOp &o : kvops)
    fgv_block_kvmeta_set(c->blk, o.ns, o.coll, reinterpret_cast<const uint8_t *>(o.key.data()), o.key.size(), o.vp.p,
                         o.vp.n);
  return FGV_OK;
}

// A block committed by the device path (no metadata writes): its valid deletes drop the deleted
// keys' validation parameters
static int kvmeta_deletes(fgv_ctx *c, fgv_mvcc_state *M, const uint8_t *block, const uint8_t *flags, size_t ntx) {
  std::vector<MvTxInfo> info(ntx);
  HIP_TRY(hipMemcpy(info.data(), M->set[0].info.p, ntx * sizeof(MvTxInfo), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < ntx; i++) {
    if (flags[i] != 0 || info[i].code != 0) continue;
    HTxRW rw;
    if (!pbw::decode(block + info[i].rws_off, info[i].rws_len, rw)) continue;
    for (const HNs &n : rw.ns) {
      HRW kv;
      if (!pbw::decode(n.rwset.p, n.rwset.n, kv)) continue;
      const std::string ns = sv(n.ns);
      for (const HWrite &w : kv.writes)
        if (is_delete(w)) fgv_block_kvmeta_set(c->blk, ns, "", w.key.p, w.key.n, nullptr, 0);
      for (const HColl &cl : n.colls) {
        HRW hr;
        hr.hashed = true;
        if (!pbw::decode(cl.hashed.p, cl.hashed.n, hr)) continue;
        for (const HWrite &w : hr.writes)
          if (is_delete(w)) fgv_block_kvmeta_set(c->blk, ns, sv(cl.name), w.key.p, w.key.n, nullptr, 0);
      }
    }
  }
  return FGV_OK;
}

// rounds enqueued before the first host check: one more than the last block needed (a block
// needing more pays one extra synchronisation); FGV_MVX_ROUNDS fixes the count (A/B)
static uint32_t first_rounds(const fgv_mvcc_state *M) {
  static const int fixed_rounds = [] {
    const char *e = getenv("FGV_MVX_ROUNDS");
    return e ? atoi(e) : 0;
  }();
  if (fixed_rounds > 0) return (uint32_t)fixed_rounds;
  return M->last_rounds ? std::min<uint32_t>(std::max<uint32_t>(M->last_rounds + 1, 2), kRoundsPerEnqueue)
                        : kRoundsPerEnqueue;
}
static uint32_t mvx_touch() {
  static const uint32_t touch = [] {
    const char *e = getenv("FGV_MVX_TOUCH");
    return e ? (uint32_t)atoi(e) : 1u;
  }();
  return touch;
}
// k_mvx_extract transactions per workgroup (16 / 32 / 64; FGV_MVX_TPW, A/B).  Measured on MI355X
// (chained C3, two alternating rounds, profiles/round3_ab/mvx_tpw*): 32 -> 60.0 / 63.6 M tx/s,
// 64 -> 54.6 / 55.3, 16 -> 45.8 / 51.1
static uint32_t mvx_tpw() {
  static const uint32_t v = [] {
    const char *e = getenv("FGV_MVX_TPW");
    const uint32_t x = e ? (uint32_t)atoi(e) : 32u;
    return (x == 16u || x == 64u) ? x : 32u;
  }();
  return v;
}
// the first block of a chain is extracted alone on an idle chip (FGV_MVX_TPW0, A/B; default as
// FGV_MVX_TPW)
static uint32_t mvx_tpw0() {
  static const uint32_t v = [] {
    const char *e = getenv("FGV_MVX_TPW0");
    const uint32_t x = e ? (uint32_t)atoi(e) : mvx_tpw();
    return (x == 16u || x == 64u || x == 32u) ? x : mvx_tpw();
  }();
  return v;
}
// FGV_MVCC_SPIN=0: blocking waits (A/B); polled by default -- a block's GPU work is ~0.2 ms, and a
// blocking synchronize's wake-up is a large share of that
// FGV_MVX_ONEWALK (default 1): k_mvx_extract's counting walk also writes every transaction's
// records to a per-tx scratch in global memory and copies them to the claimed ranges, instead of
// walking the (LDS-staged) rwset a second time.  The scratch costs its own write and read back
// (k_mvx_extract_t: 9.7 MB written per C3 block against 6.2 MB with two walks, r6za), but two walks
// measured slower on MI355X (C3, every path, r6zb): 84.4-85.1 M tx/s against 91.2-92.6 M -- on.
// Since r6zk the scratch is in LDS (mvcc.hip FGV_MVX_LDSSCR): one global write per record.
static bool mvx_onewalk() {
  static const bool on = [] {
    const char *e = getenv("FGV_MVX_ONEWALK");
    return !e || atoi(e) != 0;
  }();
  return on;
}
static MvRec *mvx_scr(MvSet &S) { return mvx_onewalk() ? S.xscr.as<MvRec>() : nullptr; }
// bytes of the global per-tx scratch for `ntx` transactions: a token buffer when the scratch is in
// LDS (mvcc.hip FGV_MVX_LDSSCR=1: the kernel only needs to know that a scratch is wanted)
static size_t mvx_scr_bytes(size_t ntx) { return mvx_lds_scratch() ? 64 : ntx * 2 * MVX_SCR * sizeof(MvRec); }

static bool mvcc_spin() {
  static const bool spin = [] {
    const char *e = getenv("FGV_MVCC_SPIN");
    return !e || atoi(e) != 0;
  }();
  return spin;
}

// ----------------------------------------------------------------- update-batch bytes
// A committing call with fgv_mvcc_set_update_bytes on takes generation (calls + 1) & 1: it waits
// for that generation's readers (fgv_mvcc_update_bytes_acquire of the call two back).  Every
// device path of the call launches k_ub_sort + k_ub_write behind its flags (meta entry = the
// block's index in the call): the batch pass on ub_stream, beside its commit kernels (the call
// does not wait for them), the chain and the single-block path in line.  After the call one copy
// brings the arena back on ub_stream; the ticket names the call, and acquire waits for the copy.
// Every MVCC call first fences its stream behind ub_stream (the serialisation reads the records,
// codes and counters the next call overwrites).
static int ub_fence(fgv_ctx *c, fgv_mvcc_state *M) {
  if (M->ub_tail_set) HIP_TRY(hipStreamWaitEvent(c->stream, M->ub_tail, 0));
  return FGV_OK;
}
static int ub_begin(fgv_ctx *c, fgv_mvcc_state *M, size_t nb, const size_t *lens) {
  M->ub_cur = -1;
  M->ub_side = false;
  if (!M->ub_on || nb == 0) return FGV_OK;
  const int gi = (int)((M->ub_calls + 1) & 1);
  auto &G = M->ub[gi];
  {
    std::unique_lock<std::mutex> lk(M->ub_mu);
    M->ub_cv.wait(lk, [&] { return G.readers == 0; });
    G.ticket = 0;
  }
  // arena: 5/4 of the blocks' bytes (an update batch holds the valid writes' keys and values, once
  // each, plus ~30 B of framing per write); a block that does not fit is decoded on the host
  uint64_t cap = 1 << 20;
  for (size_t k = 0; k < nb; k++) cap += lens[k] + lens[k] / 4;
  cap = (cap + 15) & ~(uint64_t)15;
  if (!G.arena.ensure(cap) || !G.used.ensure(64) || !G.usedh.ensure(64) || !G.meta.ensure(nb * sizeof(UbMeta)) ||
      !G.host.ensure(cap) ||
      !M->ub_dmeta.ensure(nb * sizeof(UbBlk)) || !M->ub_ents.ensure(nb * (size_t)UB_MAX * sizeof(UbEnt)))
    return FGV_ENOMEM;
  G.cap = cap;
  UbMeta *m = G.meta.as<UbMeta>();
  for (size_t k = 0; k < nb; k++) m[k] = UbMeta{0, 0, UB_NONE};
  if (!G.kev) HIP_TRY(hipEventCreateWithFlags(&G.kev, hipEventDisableTiming));
  if (!G.cev) HIP_TRY(hipEventCreateWithFlags(&G.cev, hipEventDisableTiming));
  if (!M->ub_in) HIP_TRY(hipEventCreateWithFlags(&M->ub_in, hipEventDisableTiming));
  if (!M->ub_tail) HIP_TRY(hipEventCreateWithFlags(&M->ub_tail, hipEventDisableTiming));
  if (!M->ub_stream) HIP_TRY(hipStreamCreateWithFlags(&M->ub_stream, hipStreamNonBlocking));
  if (!M->ub_cp) HIP_TRY(hipStreamCreateWithFlags(&M->ub_cp, hipStreamNonBlocking));
  // (a copy back of this generation's arena ran inside an acquire that has been released)
  HIP_TRY(hipMemsetAsync(G.used.p, 0, 8, c->stream));
  G.copied = false;
  G.nb = nb;
  M->ub_cur = gi;
  return FGV_OK;
}
// k_ub_sort + k_ub_write for `nb` blocks whose call-level indices start at idx: on stream s (in
// line), or beside it on ub_stream once s's work so far is done (side)
static void ub_launch(hipStream_t s, bool side, fgv_mvcc_state *M, size_t idx, uint32_t nb, const uint8_t *base,
                      const MvRec *writes, const MvTxInfo *info, const uint8_t *st, const MvCounters *c,
                      uint32_t rlast, const uint32_t *bfirst, const uint64_t *bnums, uint32_t ntx0, uint64_t num0) {
  if (M->ub_cur < 0) return;
  auto &G = M->ub[M->ub_cur];
  UbMeta *m = nullptr;
  if (idx + nb > G.nb || hipHostGetDevicePointer(reinterpret_cast<void **>(&m), G.meta.p, 0) != hipSuccess) return;
  hipStream_t q = s;
  if (side) {
    if (hipEventRecord(M->ub_in, s) != hipSuccess || hipStreamWaitEvent(M->ub_stream, M->ub_in, 0) != hipSuccess) return;
    q = M->ub_stream;
  } else if (M->ub_side) {  // (the shared launch scratch: behind the side launch of this call)
    if (hipStreamWaitEvent(s, M->ub_tail, 0) != hipSuccess) return;
  }
  ub_block_launch(q, nb, base, writes, info, st, c, rlast, bfirst, bnums, ntx0, num0, G.arena.as<uint8_t>(), G.cap,
                  G.used.as<unsigned long long>(), m + idx, M->ub_dmeta.as<UbBlk>(), M->ub_ents.as<UbEnt>());
  if (side && hipEventRecord(M->ub_tail, M->ub_stream) == hipSuccess) {
    M->ub_side = true;
    M->ub_tail_set = true;
  }
}
// after the call's last synchronisation: the call's serialisation is named by an event (the side
// launch on ub_stream may still run; the in-line ones are done) and a ticket.  Nothing waits here:
// the first fgv_mvcc_update_bytes_acquire of the ticket copies the claimed arena back (the copy
// engine, exactly the claimed bytes), so the host thread that hashes pays for it, not this call.
static void ub_end(fgv_ctx *c, fgv_mvcc_state *M, bool ok) {
  const int gi = M->ub_cur;
  M->ub_cur = -1;
  if (gi < 0) return;
  auto &G = M->ub[gi];
  if (ok) ok = hipEventRecord(G.kev, M->ub_side ? M->ub_stream : c->stream) == hipSuccess;
  std::lock_guard<std::mutex> lk(M->ub_mu);
  if (!ok) return;  // (ticket stays 0: the caller decodes every block on the host)
  G.ticket = ++M->ub_calls;
  M->ub_last = G.ticket;
}
// the claimed arena of generation G back to its host buffer (once per call)
static int ub_copy_back(fgv_mvcc_state *M, fgv_mvcc_state::UbGen &G) {
  std::lock_guard<std::mutex> lk(M->ub_cp_mu);
  if (G.copied) return FGV_OK;
  HIP_TRY(hipStreamWaitEvent(M->ub_cp, G.kev, 0));
  HIP_TRY(hipMemcpyAsync(G.usedh.p, G.used.p, 8, hipMemcpyDeviceToHost, M->ub_cp));
  HIP_TRY(hipEventRecord(G.cev, M->ub_cp));
  HIP_TRY(hipEventSynchronize(G.cev));
  const uint64_t total = std::min<uint64_t>(*G.usedh.as<uint64_t>(), G.cap);
  if (total) {
    HIP_TRY(hipMemcpyAsync(G.host.p, G.arena.p, total, hipMemcpyDeviceToHost, M->ub_cp));
    HIP_TRY(hipEventRecord(G.cev, M->ub_cp));
    HIP_TRY(hipEventSynchronize(G.cev));
  }
  G.copied = true;
  return FGV_OK;
}

static int mvcc_validate_locked(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block,
                                uint64_t block_num, uint8_t *flags, size_t ntx, int commit, const uint8_t *next,
                                size_t next_len, size_t ub_idx = 0);

static int mvcc_validate(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block, uint64_t block_num,
                         uint8_t *flags, size_t ntx, int commit, const uint8_t *next, size_t next_len) {
  if (!c || !block || (ntx && !flags)) return FGV_EINVAL;
  if (len >= 0xFFFFFFFFull || ntx >= 0x7FFFFFFFull) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_mvcc_state *M = c->mv;
  if (M && hipSetDevice(c->device) == hipSuccess) {
    int rc = ub_fence(c, M);
    if (!rc && commit) rc = ub_begin(c, M, 1, &len);
    if (rc) return rc;
  }
  const int rc = mvcc_validate_locked(c, block, len, d_block, block_num, flags, ntx, commit, next, next_len, 0);
  if (M) ub_end(c, M, rc == FGV_OK);
  return rc;
}

static int mvcc_validate_locked(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block,
                                uint64_t block_num, uint8_t *flags, size_t ntx, int commit, const uint8_t *next,
                                size_t next_len, size_t ub_idx) {
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
  c->n_mvcc_reads = c->n_mvcc_writes = 0;
  M->last_rounds = 0;
  if (ntx == 0) return FGV_OK;
  hipStream_t s = c->stream;
  const uint8_t *dblk = d_block;
  if (!dblk) {
    if (!c->blk_arena.ensure(len + 64)) return FGV_ENOMEM;
    HIP_TRY(hipMemcpyAsync(c->blk_arena.p, block, len, hipMemcpyHostToDevice, s));
    dblk = c->blk_arena.as<uint8_t>();
  }
  // head: envelope table (off, len) | committer flags | counters (zero)
  const size_t et_bytes = (ntx * 8 + 63) & ~(size_t)63, fl_bytes = (ntx + 63) & ~(size_t)63;
  const size_t hbytes = et_bytes + fl_bytes + kCounterBytes;
  // records: a KVRead / KVWrite takes >= 2 bytes of the block -> <= len / 2 of each
  const size_t rcap = len / 2 + 64;
  uint64_t bcap = 1024;
  while (bcap < 2 * rcap) bcap <<= 1;  // >= 2 x the writes any block of this size can hold
  if (!M->hhead.ensure(hbytes) || !M->set[0].head.ensure(hbytes) || !M->set[0].info.ensure(ntx * sizeof(MvTxInfo)) ||
      !M->set[0].reads.ensure(rcap * sizeof(MvRec)) || !M->set[0].writes.ensure(rcap * sizeof(MvRec)) ||
      !M->set[0].wslot.ensure(rcap * 4) || !M->set[0].rslot.ensure(rcap * 4) || !M->set[0].pend.ensure(rcap + 64) ||
      !M->set[0].bad.ensure(ntx + 64) || !M->set[0].st.ensure(ntx + 64) || !M->set[0].tail.ensure(kCounterBytes + ntx + 64) ||
      !M->htail.ensure(kCounterBytes + ntx + 64 + 16))
    return FGV_ENOMEM;
  if (bcap > M->btbl_cap) {  // (re)allocated tables start with epoch 0 everywhere
    M->btbl.release();
    if (!M->btbl.ensure(bcap * sizeof(BlkSlot))) return FGV_ENOMEM;
    HIP_TRY(hipMemsetAsync(M->btbl.p, 0, bcap * sizeof(BlkSlot), s));
    M->btbl_cap = bcap;
    M->epoch = 0;
    M->rg = 0;
  }
  // epoch / round tags only grow; on wrap the table is cleared and they restart
  if (M->epoch == 0xFFFFFFFFu || (uint64_t)M->rg + 4 * (uint64_t)ntx + 1024 > 0xFFFFFFFFull) {
    HIP_TRY(hipMemsetAsync(M->btbl.p, 0, M->btbl_cap * sizeof(BlkSlot), s));
    M->epoch = 0;
    M->rg = 0;
  }
  const uint32_t epoch = ++M->epoch;
  uint8_t *h = M->hhead.as<uint8_t>();
  uint32_t *et = reinterpret_cast<uint32_t *>(h);
  for (size_t i = 0; i < ntx; i++) {
    et[2 * i] = (uint32_t)(envs[i].p - block);
    et[2 * i + 1] = envs[i].n;
  }
  memcpy(h + et_bytes, flags, ntx);
  memset(h + et_bytes + fl_bytes, 0, kCounterBytes);
  uint8_t *dh = M->set[0].head.as<uint8_t>();
  const uint32_t *d_et = reinterpret_cast<const uint32_t *>(dh);
  const uint8_t *d_in = dh + et_bytes;
  MvCounters *d_c = reinterpret_cast<MvCounters *>(dh + et_bytes + fl_bytes);
  MvTxInfo *d_info = M->set[0].info.as<MvTxInfo>();
  MvRec *d_r = M->set[0].reads.as<MvRec>(), *d_w = M->set[0].writes.as<MvRec>();
  BlkSlot *d_b = M->btbl.as<BlkSlot>();
  uint8_t *d_out = M->set[0].tail.as<uint8_t>() + kCounterBytes;
  const uint32_t N = (uint32_t)ntx;
  const size_t top_off = (kCounterBytes + ntx + 7) & ~(size_t)7;  // (in htail, behind the flags)
  HIP_TRY(hipMemcpyAsync(dh, h, hbytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(c->ev[0], s));
  const uint32_t touch = mvx_touch();
  if (mvx_onewalk() && !M->set[0].xscr.ensure(mvx_scr_bytes(ntx))) return FGV_ENOMEM;
  mvx_extract_launch(mvx_tpw(), s, N, dblk, d_et, d_in, d_info, d_r, d_w, d_c, touch, mvx_scr(M->set[0]),
                     M->set[0].bad.as<uint8_t>());
  hipLaunchKernelGGL(k_mvx_prep, grid_stride(rcap), dim3(256), 0, s, dblk, d_r, d_w, d_b, epoch,
                     M->set[0].wslot.as<uint32_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                     M->set[0].bad.as<uint8_t>(), d_c, nullptr);
  HIP_TRY(hipEventRecord(c->ev[1], s));
  const uint32_t rg0 = M->rg;
  hipLaunchKernelGGL(k_mvx_find, grid_stride(rcap + ntx), dim3(256), 0, s, N, dblk, d_r, d_w, d_b, d_b, epoch,
                     M->set[0].wslot.as<uint32_t>(), M->set[0].rslot.as<uint32_t>(), d_info, M->set[0].bad.as<uint8_t>(),
                     M->set[0].st.as<uint8_t>(), rg0 + 1, d_c);
  // fixpoint rounds, enqueued ahead: a round after convergence exits at once
  uint32_t r = 0;
  auto enqueue = [&](uint32_t k) -> int {
    for (uint32_t q = 0; q < k; q++) {
      r++;
      hipLaunchKernelGGL(k_mvx_round, dim3((N + 63) / 64), dim3(64), 0, s, N, r, rg0 + r, d_info,
                         M->set[0].rslot.as<uint32_t>(), M->set[0].wslot.as<uint32_t>(), d_b, M->set[0].st.as<uint8_t>(), d_c);
    }
    hipLaunchKernelGGL(k_mvx_flags, grid_for(ntx), dim3(256), 0, s, N, r, d_in, d_info, M->set[0].st.as<uint8_t>(), d_out,
                       d_c);
    if (commit)  // (self-gated: a launch before convergence reports "not produced", the next decides)
      ub_launch(s, false, M, ub_idx, 1, dblk, d_w, d_info, M->set[0].st.as<uint8_t>(), d_c, r, nullptr, nullptr, N, block_num);
    if (commit) {
      hipLaunchKernelGGL(k_mv_last, grid_stride(rcap), dim3(256), 0, s, r, d_w, M->set[0].wslot.as<uint32_t>(),
                         M->set[0].st.as<uint8_t>(), d_b, epoch, d_c, M->top.as<unsigned long long>(), M->cap, M->arena_cap);
      hipLaunchKernelGGL(k_mv_upsert_find, grid_stride(rcap), dim3(256), 0, s, 1u, r, 0u, dblk, d_w,
                         M->set[0].wslot.as<uint32_t>(), M->set[0].st.as<uint8_t>(), d_b, epoch, M->tbl.as<StateSlot>(), M->mask,
                         M->arena.as<uint8_t>(), block_num, M->set[0].pend.as<uint8_t>(), d_c);
      hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(rcap), dim3(256), 0, s, 1u, r, 0u, dblk, d_w,
                         M->set[0].pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                         M->top.as<unsigned long long>(), block_num, d_c, nullptr, nullptr, 0u);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(M->set[0].tail.p, d_c, sizeof(MvCounters), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemcpyAsync(M->htail.p, M->set[0].tail.p, kCounterBytes + ntx, hipMemcpyDeviceToHost, s));
    // the arena top after the commit rides on the same synchronisation (no second one)
    if (commit) HIP_TRY(hipMemcpyAsync(M->htail.as<uint8_t>() + top_off, M->top.p, 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->ev[2], s));
    HIP_TRY(fgv_stream_wait(s, mvcc_spin()));
    return FGV_OK;
  };
  int rc = enqueue(first_rounds(M));
  if (rc) return rc;
  const MvCounters *hc = M->htail.as<MvCounters>();
  while (!hc->unsup && !hc->done) {  // a longer dependency chain: more rounds
    if (r > 2 * ntx + 8) return FGV_EDEVICE;  // cannot happen: one decision per round at least
    rc = enqueue(std::min<uint32_t>(4 * r, 256));
    if (rc) return rc;
  }
  M->rg = rg0 + r + 2;  // round tags of this block: rg0 + 1 .. rg0 + r + 1
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_mvcc_lookup = ms;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[2]) == hipSuccess) c->t_mvcc_total = ms;
  c->n_mvcc_reads = hc->nr;
  c->n_mvcc_writes = hc->nw;
  M->last_rounds = hc->rounds;
  if (hc->unsup == MV_HOSTPATH) {  // range queries / metadata writes, nothing else outside the model
    c->t_mvcc_total = 0;
    return phantom_block(c, M, block, block_num, flags, flags, ntx, commit);
  }
  if (hc->unsup) return FGV_EUNSUPPORTED;  // nothing was committed
  if (commit) {
    uint64_t t[2];
    memcpy(t, M->htail.as<uint8_t>() + top_off, 16);
    M->arena_used = t[0];
    M->nkeys = t[1];
    if (hc->nomem) return FGV_ENOMEM;  // nothing was committed
  }
  memcpy(flags, M->htail.as<uint8_t>() + kCounterBytes, ntx);
  if (commit && fgv_block_kvmeta_count(c->blk) > 0) return kvmeta_deletes(c, M, block, flags, ntx);
  return FGV_OK;
}

// ======================================================================= consecutive blocks
// fgv_mvcc_validate_blocks: blocks k = first..n-1, validated (and committed) in order exactly as
// one fgv_mvcc_validate_block call per block, but enqueued as ONE device chain with one wait:
//   host   : the framing walks (taken from a pre-split of this very batch -- walked while the
//            previous call's chain ran -- else walked here on the host pool, one block per job)
//            fill the pinned heads (envelope table | flags | zeroed counters) of every block;
//   stream2: ONE copy of all heads, then k_mvx_extract of block after block -- extraction reads
//            no state, so it runs ahead of the chain;
//   stream : per block k_mvx_prep (block k proceeds only when block k-1 was decided and committed
//            on the device, else nothing of it runs: MV_HALT), k_mvx_find, the fixpoint rounds,
//            k_mvx_flags, the commit, and k_mv_tail: codes, counters and arena top land straight
//            in the block's pinned tail region.
// kSets buffer sets rotate; the extraction of block k+kSets waits for block k's chain.  After the
// wait the host takes the blocks in order: the device result of every block before the first one
// the device did not finish (range queries or metadata writes -> the phantom path, a longer
// fixpoint, unsupported, table full) is final; *stop = that block (n when all finished).
// FGV_MVCC_LOG=1: each chain call's host timeline on stderr (profiling aid): microseconds from
// entry to the first record, block 0's launch, the other heads' launches, the end of the
// enqueue, the end of the wait and the return, and since the previous call's return
static bool mvcc_log() {
  static const bool on = getenv("FGV_MVCC_LOG") && atoi(getenv("FGV_MVCC_LOG"));
  return on;
}
static double mvcc_now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int mvcc_chain(fgv_ctx *c, fgv_mvcc_state *M, size_t first, size_t n, const uint8_t *const *blocks,
                      const size_t *lens, const uint8_t *const *d_blocks, const uint64_t *block_nums,
                      uint8_t *const *flags, const size_t *ntx, int commit, size_t *stop, size_t n_next,
                      const uint8_t *const *next_blocks, const size_t *next_lens) {
  *stop = first;
  const size_t nb = n - first;
  static double last_exit = 0;
  double tl[6] = {mvcc_now_us(), 0, 0, 0, 0, 0};
  // per-block sizes and the offsets of their head / tail regions
  std::vector<size_t> hoff(nb + 1, 0), toff(nb + 1, 0);
  size_t max_len = 0;
  for (size_t k = 0; k < nb; k++) {
    const size_t T = ntx[first + k];
    const size_t et_bytes = (T * 8 + 63) & ~(size_t)63, fl_bytes = (T + 63) & ~(size_t)63;
    hoff[k + 1] = hoff[k] + et_bytes + fl_bytes + kCounterBytes;
    toff[k + 1] = toff[k] + ((kCounterBytes + T + 7) & ~(size_t)7) + 64;
    max_len = std::max(max_len, lens[first + k]);
  }
  const size_t rcap = max_len / 2 + 64;
  uint64_t bcap = 1024;
  while (bcap < 2 * rcap) bcap <<= 1;
  if (!M->bhead.ensure(hoff[nb]) || !M->btail.ensure(toff[nb]) || !M->dheads.ensure(hoff[nb])) return FGV_ENOMEM;
  // each buffer set is sized for the blocks that use it (k % kSets == q), not for the call's
  // largest block: a call of many blocks holds up to kSets sets
  const int nsets = (int)std::min<size_t>(kSets, nb);
  std::vector<size_t> qlen(nsets, 0), qntx(nsets, 0);
  for (size_t k = 0; k < nb; k++) {
    qlen[k % kSets] = std::max(qlen[k % kSets], lens[first + k]);
    qntx[k % kSets] = std::max(qntx[k % kSets], ntx[first + k]);
  }
  for (int q = 0; q < nsets; q++) {
    MvSet &S = M->set[q];
    const size_t rq = qlen[q] / 2 + 64, tq = qntx[q];  // (a KVRead / KVWrite takes >= 2 block bytes)
    if (!S.info.ensure(tq * sizeof(MvTxInfo)) || !S.reads.ensure(rq * sizeof(MvRec)) ||
        !S.writes.ensure(rq * sizeof(MvRec)) || !S.wslot.ensure(rq * 4) || !S.rslot.ensure(rq * 4) ||
        !S.pend.ensure(rq + 64) || !S.bad.ensure(tq + 64) || !S.st.ensure(tq + 64) ||
        !S.tail.ensure(kCounterBytes + tq + 64) || (mvx_onewalk() && !S.xscr.ensure(mvx_scr_bytes(tq))))
      return FGV_ENOMEM;
    if (!S.ev_x) HIP_TRY(hipEventCreateWithFlags(&S.ev_x, hipEventDisableTiming));
    if (!S.ev_free) HIP_TRY(hipEventCreateWithFlags(&S.ev_free, hipEventDisableTiming));
  }
  bool need_copy = false;
  for (size_t k = 0; k < nb; k++) need_copy |= !d_blocks || !d_blocks[first + k];
  if (need_copy)
    for (int q = 0; q < nsets; q++)
      if (!M->set[q].blk.ensure(qlen[q] + 64)) return FGV_ENOMEM;
  hipStream_t s = c->stream, sx = c->stream2;
  if (bcap > M->btbl_cap) {  // (re)allocated tables start with epoch 0 everywhere
    M->btbl.release();
    if (!M->btbl.ensure(bcap * sizeof(BlkSlot))) return FGV_ENOMEM;
    HIP_TRY(hipMemsetAsync(M->btbl.p, 0, bcap * sizeof(BlkSlot), s));
    M->btbl_cap = bcap;
    M->epoch = 0;
    M->rg = 0;
  }
  const uint32_t R = first_rounds(M);
  uint64_t rg_need = 1024;
  for (size_t k = 0; k < nb; k++) rg_need += 4 * (uint64_t)ntx[first + k] + R + 2;
  if ((uint64_t)M->epoch + nb >= 0xFFFFFFFFull || (uint64_t)M->rg + rg_need > 0xFFFFFFFFull) {
    HIP_TRY(hipMemsetAsync(M->btbl.p, 0, M->btbl_cap * sizeof(BlkSlot), s));
    M->epoch = 0;
    M->rg = 0;
  }
  // FGV_MVCC_ZC=0: the tails come back by copies (A/B)
  static const bool zc_on = [] {
    const char *e = getenv("FGV_MVCC_ZC");
    return !e || atoi(e) != 0;
  }();
  uint8_t *d_btail = nullptr;
  if (zc_on && hipHostGetDevicePointer(reinterpret_cast<void **>(&d_btail), M->btail.p, 0) != hipSuccess) d_btail = nullptr;
  const bool zc = d_btail != nullptr;
  // the heads: envelope spans from the pre-split of this batch, else the framing walks here (one
  // walk is 0.2-1 ms of dependent loads over a 4 MB block: longer than the block's device work)
  std::vector<uint8_t> walked(nb, 0);
  const uint32_t *pet = nullptr;
  const size_t *pntx = nullptr, *pfirst = nullptr;
  const bool pre = fgv_block_take_presplit_batch(c->blk, nb, blocks + first, lens + first, &pet, &pntx, &pfirst);
  const bool pre0 = !pre && fgv_block_take_presplit(c->blk, blocks[first], lens[first], M->pre_envs);
  auto fill = [&](size_t k) {
    const size_t b = first + k, T = ntx[b];
    const size_t et_bytes = (T * 8 + 63) & ~(size_t)63, fl_bytes = (T + 63) & ~(size_t)63;
    uint8_t *h = M->bhead.as<uint8_t>() + hoff[k];
    uint32_t *et = reinterpret_cast<uint32_t *>(h);
    if (pre) {
      if (pntx[k] != T) return;
      const uint32_t *e = pet + BD_ENV_WORDS * pfirst[k];
      for (size_t i = 0; i < T; i++, e += BD_ENV_WORDS) {
        et[2 * i] = e[1];
        et[2 * i + 1] = e[2];
      }
    } else {
      VBlock vb;
      const std::vector<Span> *envs = nullptr;
      if (k == 0 && pre0) envs = &M->pre_envs;
      else if (pbw::decode(blocks[b], lens[b], vb)) envs = &vb.data.data;
      if (!envs || envs->size() != T) return;
      for (size_t i = 0; i < T; i++) {
        et[2 * i] = (uint32_t)((*envs)[i].p - blocks[b]);
        et[2 * i + 1] = (*envs)[i].n;
      }
    }
    memcpy(h + et_bytes, flags[b], T);
    memset(h + et_bytes + fl_bytes, 0, kCounterBytes);
    walked[k] = 1;
  };
  // block 0's head first, on this thread: its copy and extraction start while the host pool
  // fills the other blocks' heads
  fill(0);
  if (!walked[0]) return FGV_OK;  // (the single-block path reports that block's error)
  // (stream2 starts after whatever the main stream holds: the table reset above, earlier calls)
  tl[1] = mvcc_now_us();
  HIP_TRY(hipEventRecord(c->ev[0], s));
  HIP_TRY(hipStreamWaitEvent(sx, c->ev[0], 0));
  // FGV_MVX_STREAMS=2: extractions alternate over stream2 and stream3, two side by side (A/B).
  // Measured on MI355X (chained C3, alternating): GPU 0.127 / 0.130 ms per block against 0.139 /
  // 0.135 on one stream, but wall 46 / 63 M tx/s against 63 / 69 M (profiles/round3_ab/mvx_xs*):
  // one stream stays the default
  static const int nxs_env = [] {
    const char *e = getenv("FGV_MVX_STREAMS");
    return e ? atoi(e) : 1;
  }();
  const size_t nxs = nxs_env == 2 ? 2 : 1;
  const hipStream_t xs[2] = {sx, c->stream3};
  if (!M->ev_heads) HIP_TRY(hipEventCreateWithFlags(&M->ev_heads, hipEventDisableTiming));
  for (hipEvent_t &e : M->ev_multi)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // FGV_MVX_MULTI=0: one extraction launch per block (A/B).  Else blocks 1 .. m_end-1 are walked
  // on stream3, beside block 0's extraction and chain, in groups of 1, 2, 4, 8 blocks per launch:
  // a lone block's walk (~0.11 ms for 10k tx, one lane per tx) leaves most of the chip idle, a
  // group of n walks in ~0.045 n ms, and the doubling groups finish about when the chain reaches
  // them (MI355X, chained C3, profiles/round5_mvcc_*)
  static const bool multi_on = [] {
    const char *e = getenv("FGV_MVX_MULTI");
    return !e || atoi(e) != 0;
  }();
  size_t m_end = 1;        // blocks [1, m_end) extracted by the group launches
  size_t grp_end[5] = {};  // group g: blocks [grp_end[g-1] or 1, grp_end[g])
  int ngrp = 0;
  uint8_t *dheads = M->dheads.as<uint8_t>();
  HIP_TRY(hipMemcpyAsync(dheads, M->bhead.p, hoff[1], hipMemcpyHostToDevice, sx));
  size_t nq = 1;  // blocks enqueued: up to the first one that is not a block of ntx transactions
  bool rest_sent = nb == 1;
  const uint32_t touch = mvx_touch();
  BlkSlot *d_b = M->btbl.as<BlkSlot>();
  const MvCounters *prev_c = nullptr;
  // FGV_MVCC_FUSE=0: k_mvx_flags + k_mv_last and one k_mv_tail per block (A/B); else the fused
  // k_mvx_flags_last and the tails of the call at its end (mvcc_multi.h)
  static const bool fuse = [] {
    const char *e = getenv("FGV_MVCC_FUSE");
    return !e || atoi(e) != 0;
  }();
  std::vector<const MvCounters *> tails_c;
  std::vector<uint32_t *> tails_h;
  for (size_t k = 0; k < nb; k++) {
    const size_t b = first + k;
    const uint8_t *block = blocks[b];
    const size_t len = lens[b], T = ntx[b];
    MvSet &S = M->set[k % kSets];
    const size_t et_bytes = (T * 8 + 63) & ~(size_t)63, fl_bytes = (T + 63) & ~(size_t)63;
    if (k >= nq) break;
    if (k >= 1 && k < m_end) {  // extracted by a group launch: wait for it at its first block
      for (int g = 0; g < ngrp; g++)
        if (k == (g ? grp_end[g - 1] : 1)) HIP_TRY(hipStreamWaitEvent(s, M->ev_multi[g], 0));
    } else {
    // block k's extraction stream: the set is free once block k-kSets's chain is done
      hipStream_t sxk = xs[k % nxs];
      if (k >= (size_t)kSets) HIP_TRY(hipStreamWaitEvent(sxk, S.ev_free, 0));
      const uint8_t *db = d_blocks ? d_blocks[b] : nullptr;
      if (!db) HIP_TRY(hipMemcpyAsync(S.blk.p, block, len, hipMemcpyHostToDevice, sxk));
      uint8_t *dh = dheads + hoff[k];
      mvx_extract_launch(k == 0 ? mvx_tpw0() : mvx_tpw(), sxk, (uint32_t)T, db ? db : S.blk.as<uint8_t>(),
                         reinterpret_cast<const uint32_t *>(dh), dh + et_bytes, S.info.as<MvTxInfo>(),
                         S.reads.as<MvRec>(), S.writes.as<MvRec>(),
                         reinterpret_cast<MvCounters *>(dh + et_bytes + fl_bytes), touch, mvx_scr(S),
                         S.bad.as<uint8_t>());
      HIP_TRY(hipEventRecord(S.ev_x, sxk));
      // main stream: block k's chain
      HIP_TRY(hipStreamWaitEvent(s, S.ev_x, 0));
    }
    if (k == 0) tl[2] = mvcc_now_us();
    if (k == 0 && !rest_sent) {  // the other heads, once block 0's extraction is on its way
      fgv_parallel_run(c->blk, nb - 1, [&](size_t j) { fill(j + 1); });
      while (nq < nb && walked[nq]) nq++;
      const bool multi = multi_on && nq > 2;
      if (nq > 1) {  // the other heads: on stream3 when the groups start there, else behind block 0
        hipStream_t hs = multi ? xs[1] : sx;
        if (multi) HIP_TRY(hipStreamWaitEvent(hs, c->ev[0], 0));
        HIP_TRY(hipMemcpyAsync(dheads + hoff[1], M->bhead.as<uint8_t>() + hoff[1], hoff[nq] - hoff[1],
                               hipMemcpyHostToDevice, hs));
        if (nxs > 1 || multi) {  // the other extraction stream starts after the heads' copy
          HIP_TRY(hipEventRecord(M->ev_heads, hs));
          HIP_TRY(hipStreamWaitEvent(multi ? sx : xs[1], M->ev_heads, 0));
        }
      }
      if (multi) {
        m_end = std::min(nq, (size_t)kSets);
        const uint32_t tpw = mvx_tpw();
        for (size_t g0 = 1, gs = 1; g0 < m_end && ngrp < 5; g0 += gs, gs *= 2) {
          const size_t g1 = (ngrp == 4) ? m_end : std::min(m_end, g0 + gs);
          MvxJobs J{};
          J.touch = touch;
          uint32_t wgs = 0;
          for (size_t q = g0; q < g1; q++) {
            const size_t bq = first + q, Tq = ntx[bq];
            MvSet &Sq = M->set[q];
            const uint8_t *db = d_blocks ? d_blocks[bq] : nullptr;
            if (!db) {
              HIP_TRY(hipMemcpyAsync(Sq.blk.p, blocks[bq], lens[bq], hipMemcpyHostToDevice, xs[1]));
              db = Sq.blk.as<uint8_t>();
            }
            const size_t etq = (Tq * 8 + 63) & ~(size_t)63, flq = (Tq + 63) & ~(size_t)63;
            uint8_t *dh = dheads + hoff[q];
            MvxJob &j = J.j[J.n++];
            j.base = db;
            j.envtab = reinterpret_cast<const uint32_t *>(dh);
            j.in_flags = dh + etq;
            j.info = Sq.info.as<MvTxInfo>();
            j.reads = Sq.reads.as<MvRec>();
            j.writes = Sq.writes.as<MvRec>();
            j.c = reinterpret_cast<MvCounters *>(dh + etq + flq);
            j.scr = mvx_scr(Sq);
            j.bad = Sq.bad.as<uint8_t>();
            j.ntx = (uint32_t)Tq;
            j.wg0 = wgs;
            wgs += (uint32_t)((Tq + tpw - 1) / tpw);
          }
          if (wgs) mvx_extract_multi_launch(tpw, xs[1], J, wgs);
          HIP_TRY(hipGetLastError());
          HIP_TRY(hipEventRecord(M->ev_multi[ngrp], xs[1]));
          grp_end[ngrp++] = g1;
          if (g1 == m_end) break;
        }
      }
      rest_sent = true;
    }
    if (k == 0) tl[3] = mvcc_now_us();
    // the next call's framing walks start on the pre-split worker as soon as every head of this
    // call is filled (they overwrite the pre-split table the heads were filled from)
    if (k == 0 && n_next) {
      fgv_block_presplit(c->blk, c->device, n_next, next_blocks, next_lens, nullptr, nullptr);
      n_next = 0;
    }
    const uint8_t *dblk = d_blocks && d_blocks[b] ? d_blocks[b] : S.blk.as<uint8_t>();
    uint8_t *dh = dheads + hoff[k];
    const uint8_t *d_in = dh + et_bytes;
    MvCounters *d_c = reinterpret_cast<MvCounters *>(dh + et_bytes + fl_bytes);
    MvTxInfo *d_info = S.info.as<MvTxInfo>();
    MvRec *d_r = S.reads.as<MvRec>(), *d_w = S.writes.as<MvRec>();
    const uint32_t N = (uint32_t)T;
    const uint32_t epoch = ++M->epoch;
    const uint32_t rg0 = M->rg;
    // k_mvx_prep gates the block on block k-1 (prev_c: decided and committed on the device)
    hipLaunchKernelGGL(k_mvx_prep, grid_stride(rcap), dim3(256), 0, s, dblk, d_r, d_w, d_b, epoch,
                       S.wslot.as<uint32_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                       S.bad.as<uint8_t>(), d_c, prev_c);
    hipLaunchKernelGGL(k_mvx_find, grid_stride(rcap + T), dim3(256), 0, s, N, dblk, d_r, d_w, d_b, d_b, epoch,
                       S.wslot.as<uint32_t>(), S.rslot.as<uint32_t>(), d_info, S.bad.as<uint8_t>(), S.st.as<uint8_t>(),
                       rg0 + 1, d_c);
    for (uint32_t r = 1; r <= R; r++)
      hipLaunchKernelGGL(k_mvx_round, dim3((N + 63) / 64), dim3(64), 0, s, N, r, rg0 + r, d_info,
                         S.rslot.as<uint32_t>(), S.wslot.as<uint32_t>(), d_b, S.st.as<uint8_t>(), d_c);
    // zero-copy: the codes, counters and arena top go straight to the block's pinned tail region
    uint8_t *d_out = zc ? d_btail + toff[k] + kCounterBytes : S.tail.as<uint8_t>() + kCounterBytes;
    if (fuse) {
      hipLaunchKernelGGL(k_mvx_flags_last, grid_stride(std::max(rcap, T)), dim3(256), 0, s, N, R, d_in, d_info,
                         S.st.as<uint8_t>(), d_out, d_c, commit ? 1u : 0u, d_w, S.wslot.as<uint32_t>(), d_b, epoch,
                         M->top.as<unsigned long long>(), M->cap, M->arena_cap);
    } else {
      hipLaunchKernelGGL(k_mvx_flags, grid_for(T), dim3(256), 0, s, N, R, d_in, d_info, S.st.as<uint8_t>(), d_out, d_c);
      if (commit)
        hipLaunchKernelGGL(k_mv_last, grid_stride(rcap), dim3(256), 0, s, R, d_w, S.wslot.as<uint32_t>(),
                           S.st.as<uint8_t>(), d_b, epoch, d_c, M->top.as<unsigned long long>(), M->cap, M->arena_cap);
    }
    if (commit) {
      ub_launch(s, false, M, b, 1, dblk, d_w, d_info, S.st.as<uint8_t>(), d_c, R, nullptr, nullptr, N, block_nums[b]);
      hipLaunchKernelGGL(k_mv_upsert_find, grid_stride(rcap), dim3(256), 0, s, 1u, R, 0u, dblk, d_w,
                         S.wslot.as<uint32_t>(), S.st.as<uint8_t>(), d_b, epoch, M->tbl.as<StateSlot>(), M->mask,
                         M->arena.as<uint8_t>(), block_nums[b], S.pend.as<uint8_t>(), d_c);
      hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(rcap), dim3(256), 0, s, 1u, R, 0u, dblk, d_w,
                         S.pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                         M->top.as<unsigned long long>(), block_nums[b], d_c, nullptr, nullptr, 0u);
    }
    HIP_TRY(hipGetLastError());
    uint8_t *ht = M->btail.as<uint8_t>() + toff[k];
    const size_t top_off = (kCounterBytes + T + 7) & ~(size_t)7;
    if (zc && fuse) {
      tails_c.push_back(d_c);
      tails_h.push_back(reinterpret_cast<uint32_t *>(d_btail + toff[k]));
    } else if (zc) {
      uint8_t *dt = d_btail + toff[k];
      hipLaunchKernelGGL(k_mv_tail, dim3(1), dim3(64), 0, s, d_c, M->top.as<unsigned long long>(),
                         reinterpret_cast<uint32_t *>(dt),
                         commit ? reinterpret_cast<unsigned long long *>(dt + top_off) : nullptr);
    } else {
      HIP_TRY(hipMemcpyAsync(S.tail.p, d_c, sizeof(MvCounters), hipMemcpyDeviceToDevice, s));
      HIP_TRY(hipMemcpyAsync(ht, S.tail.p, kCounterBytes + T, hipMemcpyDeviceToHost, s));
      if (commit) HIP_TRY(hipMemcpyAsync(ht + top_off, M->top.p, 16, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipEventRecord(S.ev_free, s));  // the set's last reader of block k is done
    M->rg = rg0 + R + 2;  // round tags of this block: rg0 + 1 .. rg0 + R + 1
    prev_c = d_c;
  }
  // fused mode: every block's counters in one launch per MVX_MULTI_MAX blocks, and the arena top
  // after the last commit once, into the last block's tail (a later block commits nothing after a
  // block the device did not finish, so the final top is the last finished block's)
  const size_t last_top = tails_c.empty() ? 0 : toff[tails_c.size() - 1] +
                                                     ((kCounterBytes + ntx[first + tails_c.size() - 1] + 7) & ~(size_t)7);
  for (size_t q0 = 0; q0 < tails_c.size(); q0 += MVX_MULTI_MAX) {
    MvTails Tl{};
    const size_t q1 = std::min(tails_c.size(), q0 + MVX_MULTI_MAX);
    for (size_t q = q0; q < q1; q++) {
      Tl.c[Tl.n] = tails_c[q];
      Tl.hc[Tl.n++] = tails_h[q];
    }
    hipLaunchKernelGGL(k_mv_tails, dim3(Tl.n), dim3(64), 0, s, Tl, M->top.as<unsigned long long>(),
                       (commit && q1 == tails_c.size()) ? reinterpret_cast<unsigned long long *>(d_btail + last_top)
                                                        : nullptr);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev[2], s));
  // the next batch's framing walks run on the pre-split worker while this chain runs
  if (n_next) fgv_block_presplit(c->blk, c->device, n_next, next_blocks, next_lens, nullptr, nullptr);
  tl[4] = mvcc_now_us();
  HIP_TRY(fgv_stream_wait(s, mvcc_spin()));
  tl[5] = mvcc_now_us();
  float ms = 0;
  c->t_mvcc_lookup = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[2]) == hipSuccess) c->t_mvcc_total = ms / (double)nq;
  c->n_mvcc_reads = c->n_mvcc_writes = 0;
  uint32_t rounds = 0;
  size_t k = 0;
  for (; k < nq; k++) {
    const size_t b = first + k, T = ntx[b];
    const uint8_t *ht = M->btail.as<uint8_t>() + toff[k];
    const MvCounters *hc = reinterpret_cast<const MvCounters *>(ht);
    if (hc->unsup || !hc->done || (commit && hc->nomem)) break;
    memcpy(flags[b], ht + kCounterBytes, T);
    if (commit) {
      uint64_t t[2];
      memcpy(t, tails_c.empty() ? ht + ((kCounterBytes + T + 7) & ~(size_t)7) : M->btail.as<uint8_t>() + last_top, 16);
      M->arena_used = t[0];
      M->nkeys = t[1];
    }
    c->n_mvcc_reads += hc->nr;
    c->n_mvcc_writes += hc->nw;
    rounds = std::max(rounds, hc->rounds);
  }
  if (rounds) M->last_rounds = rounds;
  *stop = first + k;
  if (mvcc_log()) {
    const double t = mvcc_now_us();
    fprintf(stderr, "[fgv] mvcc chain %zu blocks: since last %.0f | ev0 %.0f b0 %.0f rest %.0f enq %.0f wait %.0f ret %.0f us\n",
            nq, last_exit ? tl[0] - last_exit : 0.0, tl[1] - tl[0], tl[2] - tl[0], tl[3] - tl[0], tl[4] - tl[0],
            tl[5] - tl[0], t - tl[0]);
    last_exit = t;
  }
  return FGV_OK;
}

// ======================================================================= batch pass
// Consecutive blocks [first, n) validated as ONE device pass (mvcc.hip "batch pass"): one
// extraction over every transaction of the batch in block order, the write table of the whole
// batch, the fixpoint under the sequential rule restated there (a read checks the last valid
// earlier writer of its key: same block -> conflict, an earlier block -> that writer's height,
// none -> the state before the batch), one commit of each key's last valid writer at its own
// block's height.  Results equal one fgv_mvcc_validate_block call per block.  The blocks' bytes
// must lie within 4 GB of one base (the records' 32-bit offsets): caller device copies that do,
// or host blocks staged here back to back.  Anything the pass does not finish -- unsupported or
// host-path transactions (range queries, metadata writes), a key with more than MB_WR writers, a
// longer fixpoint, a full table -- commits nothing and leaves *stop at `first`: the per-block
// chain then takes the blocks.
static int mvcc_batch(fgv_ctx *c, fgv_mvcc_state *M, size_t first, size_t n, const uint8_t *const *blocks,
                      const size_t *lens, const uint8_t *const *d_blocks, const uint64_t *block_nums,
                      uint8_t *const *flags, const size_t *ntx, int commit, size_t *stop, size_t n_next,
                      const uint8_t *const *next_blocks, const size_t *next_lens) {
  *stop = first;
  const size_t nb = n - first;
  size_t total = 0, bytes = 0;
  for (size_t k = 0; k < nb; k++) total += ntx[first + k], bytes += lens[first + k];
  if (total >= 0x7FFFFFFFull) return FGV_OK;
  // the common base: the caller's device copies when they span < 4 GB, else a staging copy
  const uint8_t *base = nullptr;
  std::vector<uint64_t> boff(nb);
  bool have_dev = d_blocks != nullptr;
  for (size_t k = 0; have_dev && k < nb; k++) have_dev = d_blocks[first + k] != nullptr;
  if (have_dev) {
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (size_t k = 0; k < nb; k++) {
      const uintptr_t a = (uintptr_t)d_blocks[first + k];
      lo = std::min(lo, a);
      hi = std::max(hi, a + lens[first + k] + 64);
    }
    if (hi - lo >= (1ull << 32)) return FGV_OK;  // (the per-block chain)
    base = reinterpret_cast<const uint8_t *>(lo);
    for (size_t k = 0; k < nb; k++) boff[k] = (uintptr_t)d_blocks[first + k] - lo;
  } else {
    uint64_t o = 0;
    for (size_t k = 0; k < nb; k++) {
      boff[k] = o;
      o += (lens[first + k] + 64 + 255) & ~(size_t)255;
    }
    if (o >= (1ull << 32) || !M->mbblk.ensure(o)) return o >= (1ull << 32) ? FGV_OK : FGV_ENOMEM;
    base = M->mbblk.as<uint8_t>();
  }
  // head: envelope table (8 B/tx) | committer flags | counters | block firsts (nb + 1) | numbers
  const size_t et_bytes = (total * 8 + 63) & ~(size_t)63, fl_bytes = (total + 63) & ~(size_t)63;
  const size_t bf_off = et_bytes + fl_bytes + kCounterBytes, bn_off = bf_off + (((nb + 1) * 4 + 63) & ~(size_t)63);
  const size_t hbytes = bn_off + ((nb * 8 + 63) & ~(size_t)63);
  const size_t tbytes = kCounterBytes + ((total + 63) & ~(size_t)63) + 64;
  const size_t rcap = bytes / 2 + 64;
  uint64_t bcap = 1024;
  while (bcap < 2 * rcap) bcap <<= 1;
  MvSet &S = M->set[0];
  if (!M->mbhead.ensure(hbytes) || !M->mbdhead.ensure(hbytes) || !M->mbtail.ensure(tbytes) ||
      !S.info.ensure(total * sizeof(MvTxInfo)) || !S.reads.ensure(rcap * sizeof(MvRec)) ||
      !S.writes.ensure(rcap * sizeof(MvRec)) || !S.wslot.ensure(rcap * 4) || !S.rslot.ensure(rcap * 4) ||
      !S.pend.ensure(rcap + 64) || !S.bad.ensure(total + 64) || !S.st.ensure(total + 64) ||
      (mvx_onewalk() && !S.xscr.ensure(mvx_scr_bytes(total))) || !M->mbrstat.ensure(rcap + 64))
    return FGV_ENOMEM;
  hipStream_t s = c->stream;
  if (bcap > M->mbtbl_cap) {  // (re)allocated: epoch 0 everywhere
    M->mbtbl.release();
    if (!M->mbtbl.ensure(bcap * sizeof(MbSlot))) return FGV_ENOMEM;
    HIP_TRY(hipMemsetAsync(M->mbtbl.p, 0, bcap * sizeof(MbSlot), s));
    M->mbtbl_cap = bcap;
    M->mb_epoch = 0;
  }
  if (M->mb_epoch + 1 >= 0xFFFFFFFFu) {
    HIP_TRY(hipMemsetAsync(M->mbtbl.p, 0, M->mbtbl_cap * sizeof(MbSlot), s));
    M->mb_epoch = 0;
  }
  uint8_t *d_tail = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&d_tail), M->mbtail.p, 0) != hipSuccess) return FGV_OK;
  // envelope spans: the pre-split of this batch, else the framing walks on the host pool
  uint8_t *h = M->mbhead.as<uint8_t>();
  uint32_t *et = reinterpret_cast<uint32_t *>(h);
  uint32_t *bfirst = reinterpret_cast<uint32_t *>(h + bf_off);
  uint64_t *bnums = reinterpret_cast<uint64_t *>(h + bn_off);
  bfirst[0] = 0;
  for (size_t k = 0; k < nb; k++) {
    bfirst[k + 1] = bfirst[k] + (uint32_t)ntx[first + k];
    bnums[k] = block_nums[first + k];
  }
  const uint32_t *pet = nullptr;
  const size_t *pntx = nullptr, *pfirst = nullptr;
  const bool pre = fgv_block_take_presplit_batch(c->blk, nb, blocks + first, lens + first, &pet, &pntx, &pfirst);
  std::vector<uint8_t> ok(nb, 0);
  auto fill = [&](size_t k) {
    const size_t b = first + k, T = ntx[b];
    uint32_t *e_out = et + 2 * (size_t)bfirst[k];
    if (pre) {
      if (pntx[k] != T) return;
      const uint32_t *e = pet + BD_ENV_WORDS * pfirst[k];
      for (size_t i = 0; i < T; i++, e += BD_ENV_WORDS) {
        e_out[2 * i] = (uint32_t)(boff[k] + e[1]);
        e_out[2 * i + 1] = e[2];
      }
    } else {
      VBlock vb;
      if (!pbw::decode(blocks[b], lens[b], vb) || vb.data.data.size() != T) return;
      for (size_t i = 0; i < T; i++) {
        e_out[2 * i] = (uint32_t)(boff[k] + (uint64_t)(vb.data.data[i].p - blocks[b]));
        e_out[2 * i + 1] = vb.data.data[i].n;
      }
    }
    memcpy(h + et_bytes + bfirst[k], flags[b], T);
    ok[k] = 1;
  };
  if (pre) {
    for (size_t k = 0; k < nb; k++) fill(k);
  } else {
    fgv_parallel_run(c->blk, nb, fill);
  }
  for (size_t k = 0; k < nb; k++)
    if (!ok[k]) return FGV_OK;  // (the per-block path reports the block's error)
  memset(h + et_bytes + fl_bytes, 0, kCounterBytes);
  HIP_TRY(hipEventRecord(c->ev[0], s));
  if (!have_dev)
    for (size_t k = 0; k < nb; k++)
      HIP_TRY(hipMemcpyAsync(M->mbblk.as<uint8_t>() + boff[k], blocks[first + k], lens[first + k],
                             hipMemcpyHostToDevice, s));
  uint8_t *dh = M->mbdhead.as<uint8_t>();
  HIP_TRY(hipMemcpyAsync(dh, h, hbytes, hipMemcpyHostToDevice, s));
  const uint32_t *d_et = reinterpret_cast<const uint32_t *>(dh);
  const uint8_t *d_in = dh + et_bytes;
  MvCounters *d_c = reinterpret_cast<MvCounters *>(dh + et_bytes + fl_bytes);
  const uint32_t *d_bf = reinterpret_cast<const uint32_t *>(dh + bf_off);
  const uint64_t *d_bn = reinterpret_cast<const uint64_t *>(dh + bn_off);
  MvTxInfo *d_info = S.info.as<MvTxInfo>();
  MvRec *d_r = S.reads.as<MvRec>(), *d_w = S.writes.as<MvRec>();
  MbSlot *d_b = M->mbtbl.as<MbSlot>();
  const uint32_t N = (uint32_t)total, NB = (uint32_t)nb;
  const uint32_t epoch = ++M->mb_epoch;
  mvx_extract_launch(mvx_tpw(), s, N, base, d_et, d_in, d_info, d_r, d_w, d_c, mvx_touch(), mvx_scr(S),
                     S.bad.as<uint8_t>());
  hipLaunchKernelGGL(k_mvb_prep, grid_stride(2 * rcap), dim3(256), 0, s, base, d_r, d_w, d_b, epoch,
                     S.wslot.as<uint32_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                     M->mbrstat.as<uint8_t>(), d_c);
  hipLaunchKernelGGL(k_mvb_find, grid_stride(2 * rcap + total), dim3(256), 0, s, N, base, d_r, d_w, d_b, epoch,
                     S.wslot.as<uint32_t>(), S.rslot.as<uint32_t>(), d_info, S.st.as<uint8_t>(), d_c);
  // rounds: two more than the last batch needed, at least 6 (FGV_MVB_ROUNDS fixes the count)
  static const uint32_t fixed_rounds = [] {
    const char *e = getenv("FGV_MVB_ROUNDS");
    return e ? (uint32_t)std::max(1, std::min(64, atoi(e))) : 0u;
  }();
  const uint32_t R = fixed_rounds ? fixed_rounds : std::min<uint32_t>(32, std::max<uint32_t>(6, M->mb_rounds + 2));
  for (uint32_t r = 1; r <= R; r++)
    hipLaunchKernelGGL(k_mvb_round, dim3((N + 63) / 64), dim3(64), 0, s, N, r, d_info, d_r, d_w,
                       S.rslot.as<uint32_t>(), M->mbrstat.as<uint8_t>(), d_b, S.st.as<uint8_t>(), d_bf, d_bn, NB, d_c);
  hipLaunchKernelGGL(k_mvx_flags, grid_for(total), dim3(256), 0, s, N, R, d_in, d_info, S.st.as<uint8_t>(),
                     d_tail + kCounterBytes, d_c);
  if (commit)  // (before k_mvb_upsert_find, which stores versions in the write records' value fields)
    ub_launch(s, true, M, first, NB, base, d_w, d_info, S.st.as<uint8_t>(), d_c, R, d_bf, d_bn, 0u, 0ull);
  if (commit) {
    hipLaunchKernelGGL(k_mvb_last, grid_stride(rcap), dim3(256), 0, s, R, d_w, S.wslot.as<uint32_t>(),
                       S.st.as<uint8_t>(), d_b, epoch, d_c, M->top.as<unsigned long long>(), M->cap, M->arena_cap);
    hipLaunchKernelGGL(k_mvb_upsert_find, grid_stride(rcap), dim3(256), 0, s, R, base, d_w, S.wslot.as<uint32_t>(),
                       S.st.as<uint8_t>(), d_b, epoch, M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(), d_bf,
                       d_bn, NB, S.pend.as<uint8_t>(), d_c);
    hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(rcap), dim3(256), 0, s, 2u, R, 0u, base, d_w,
                       S.pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                       M->top.as<unsigned long long>(), 0ull, d_c, d_bf, d_bn, NB);
  }
  const size_t top_off = kCounterBytes + ((total + 63) & ~(size_t)63);
  hipLaunchKernelGGL(k_mv_tail, dim3(1), dim3(64), 0, s, d_c, M->top.as<unsigned long long>(),
                     reinterpret_cast<uint32_t *>(d_tail),
                     commit ? reinterpret_cast<unsigned long long *>(d_tail + top_off) : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev[2], s));
  // the next batch's framing walks run on the pre-split worker meanwhile
  if (n_next) fgv_block_presplit(c->blk, c->device, n_next, next_blocks, next_lens, nullptr, nullptr);
  HIP_TRY(fgv_stream_wait(s, mvcc_spin()));
  const uint8_t *ht = M->mbtail.as<uint8_t>();
  const MvCounters *hc = reinterpret_cast<const MvCounters *>(ht);
  if (hc->unsup || !hc->done || (commit && hc->nomem)) {
    if (!hc->unsup && !hc->done) M->mb_rounds = R;  // (the fixpoint needed more: one more next time)
    return FGV_OK;  // nothing committed: the per-block chain takes the blocks
  }
  for (size_t k = 0; k < nb; k++) memcpy(flags[first + k], ht + kCounterBytes + bfirst[k], ntx[first + k]);
  if (commit) {
    uint64_t t[2];
    memcpy(t, ht + top_off, 16);
    M->arena_used = t[0];
    M->nkeys = t[1];
  }
  float ms = 0;
  c->t_mvcc_lookup = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[2]) == hipSuccess) c->t_mvcc_total = ms / (double)nb;
  c->n_mvcc_reads = hc->nr;
  c->n_mvcc_writes = hc->nw;
  M->mb_rounds = hc->rounds;
  M->last_rounds = hc->rounds;
  *stop = n;
  return FGV_OK;
}

static int mvcc_blocks_run(fgv_ctx *c, fgv_mvcc_state *M, size_t n, const uint8_t *const *blocks, const size_t *lens,
                           const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                           const size_t *ntx, int commit, size_t *n_done, size_t n_next,
                           const uint8_t *const *next_blocks, const size_t *next_lens);
static int mvcc_blocks(fgv_ctx *c, size_t n, const uint8_t *const *blocks, const size_t *lens,
                       const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                       const size_t *ntx, int commit, size_t *n_done, size_t n_next,
                       const uint8_t *const *next_blocks, const size_t *next_lens) {
  if (n_done) *n_done = 0;
  if (!c || (n && (!blocks || !lens || !block_nums || !flags || !ntx))) return FGV_EINVAL;
  for (size_t k = 0; k < n; k++)
    if (!blocks[k] || (ntx[k] && !flags[k]) || lens[k] >= 0xFFFFFFFFull || ntx[k] >= 0x7FFFFFFFull) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  {
    int rc = ub_fence(c, M);
    if (!rc && commit) rc = ub_begin(c, M, n, lens);
    if (rc) return rc;
  }
  const int rc = mvcc_blocks_run(c, M, n, blocks, lens, d_blocks, block_nums, flags, ntx, commit, n_done, n_next,
                                 next_blocks, next_lens);
  ub_end(c, M, rc == FGV_OK || (n_done && *n_done > 0));
  return rc;
}

static int mvcc_blocks_run(fgv_ctx *c, fgv_mvcc_state *M, size_t n, const uint8_t *const *blocks, const size_t *lens,
                           const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                           const size_t *ntx, int commit, size_t *n_done, size_t n_next,
                           const uint8_t *const *next_blocks, const size_t *next_lens) {
  size_t done = 0;
  // FGV_MVCC_CHAIN=0: one single-block call per block (A/B)
  static const bool chain = [] {
    const char *e = getenv("FGV_MVCC_CHAIN");
    return !e || atoi(e) != 0;
  }();
  while (done < n) {
    // key-level state is kept current by the single-block path's host step (kvmeta_deletes); an
    // empty block has no device work
    size_t stop = done;
    if (chain && ntx[done] > 0 && !(commit && fgv_block_kvmeta_count(c->blk) > 0)) {
      size_t end = done;
      while (end < n && ntx[end] > 0) end++;
      // FGV_MVCC_BATCH=0: the per-block chain only (A/B)
      static const bool batch = [] {
        const char *e = getenv("FGV_MVCC_BATCH");
        return !e || atoi(e) != 0;
      }();
      // the batch pass for runs of small blocks, where the per-block chain is launch-bound: its
      // fixpoint rounds grow with the batch's longest chain of dependent outcomes, which large
      // blocks over a dense key space make long (C3, 10 x 10k-tx blocks: 20+ rounds, measured
      // 47 M tx/s through the pass against 63 M chained) -- FGV_MVCC_BATCH_TX = the largest
      // block the pass takes (default 4096 transactions)
      static const size_t batch_tx = [] {
        const char *e = getenv("FGV_MVCC_BATCH_TX");
        return e ? (size_t)atol(e) : (size_t)4096;
      }();
      size_t big = 0;
      for (size_t k = done; k < end; k++) big = std::max(big, ntx[k]);
      if (batch && end - done >= 2 && big <= batch_tx) {
        const int rc = mvcc_batch(c, M, done, end, blocks, lens, d_blocks, block_nums, flags, ntx, commit, &stop,
                                  n_next, next_blocks, next_lens);
        n_next = 0;  // (the next batch is being walked)
        if (rc) return rc;
        if (stop != end) {  // (the blocks again below: behind the pass's serialisation on ub_stream)
          const int rf = ub_fence(c, M);
          if (rf) return rf;
        }
        if (stop == end) {
          done = end;
          if (n_done) *n_done = done;
          if (done == n) break;
          continue;
        }
      }
      const int rc = mvcc_chain(c, M, done, end, blocks, lens, d_blocks, block_nums, flags, ntx, commit, &stop,
                                n_next, next_blocks, next_lens);
      n_next = 0;  // (the next batch is being walked)
      if (rc) {
        if (n_done) *n_done = done;
        return rc;
      }
      done = stop;
      if (n_done) *n_done = done;
      if (done == n) break;
    }
    // the first block the chain did not finish: the single-block path (phantom validators, more
    // rounds, or the error it returns)
    const int rc = mvcc_validate_locked(c, blocks[done], lens[done], d_blocks ? d_blocks[done] : nullptr,
                                        block_nums[done], flags[done], ntx[done], commit, nullptr, 0, done);
    if (rc) return rc;
    done++;
    if (n_done) *n_done = done;
  }
  return FGV_OK;
}

extern "C" {

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

int fgv_mvcc_validate_blocks(fgv_ctx *c, size_t n, const uint8_t *const *blocks, const size_t *lens,
                             const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                             const size_t *ntx, int commit, size_t *n_done) {
  return mvcc_blocks(c, n, blocks, lens, d_blocks, block_nums, flags, ntx, commit, n_done, 0, nullptr, nullptr);
}

int fgv_mvcc_validate_blocks_next(fgv_ctx *c, size_t n, const uint8_t *const *blocks, const size_t *lens,
                                  const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                                  const size_t *ntx, int commit, size_t *n_done, size_t n_next,
                                  const uint8_t *const *next_blocks, const size_t *next_lens) {
  if (n_next && (!next_blocks || !next_lens)) return FGV_EINVAL;
  return mvcc_blocks(c, n, blocks, lens, d_blocks, block_nums, flags, ntx, commit, n_done, n_next, next_blocks,
                     next_lens);
}

int fgv_mvcc_set_update_bytes(fgv_ctx *c, int on) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->mv) return FGV_ESTATE;
  c->mv->ub_on = on != 0;
  return FGV_OK;
}

int fgv_mvcc_last_ticket(fgv_ctx *c, uint64_t *ticket) {
  if (!c || !ticket) return FGV_EINVAL;
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  std::lock_guard<std::mutex> lk(M->ub_mu);
  *ticket = M->ub_last;
  return FGV_OK;
}

int fgv_mvcc_update_bytes_acquire(fgv_ctx *c, uint64_t ticket, size_t n, const uint8_t **bytes, size_t *lens) {
  if (!c || (n && (!bytes || !lens))) return FGV_EINVAL;
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  fgv_mvcc_state::UbGen *G = nullptr;
  {
    std::lock_guard<std::mutex> lk(M->ub_mu);
    for (auto &g : M->ub)
      if (ticket && g.ticket == ticket) G = &g;
    if (!G) return FGV_ESTATE;  // not a call of the last two with update bytes
    if (n > G->nb) return FGV_EINVAL;
    G->readers++;
  }
  hipSetDevice(c->device);
  const int rc = ub_copy_back(M, *G);
  if (rc) {
    fgv_mvcc_update_bytes_release(c, ticket);
    return rc;
  }
  const UbMeta *m = G->meta.as<UbMeta>();
  for (size_t b = 0; b < n; b++) {
    const bool ok = m[b].status == UB_OK && m[b].off + m[b].len <= G->cap;
    bytes[b] = ok ? G->host.as<uint8_t>() + m[b].off : nullptr;
    lens[b] = ok ? m[b].len : 0;
  }
  return FGV_OK;
}

int fgv_mvcc_update_bytes_release(fgv_ctx *c, uint64_t ticket) {
  if (!c) return FGV_EINVAL;
  fgv_mvcc_state *M = c->mv;
  if (!M) return FGV_ESTATE;
  std::lock_guard<std::mutex> lk(M->ub_mu);
  for (auto &g : M->ub)
    if (ticket && g.ticket == ticket && g.readers > 0) {
      g.readers--;
      M->ub_cv.notify_all();
      return FGV_OK;
    }
  return FGV_ESTATE;
}

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
