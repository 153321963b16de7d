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
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_set>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_internal.h"
#include "fgv_visitors.h"

bool fgv_block_take_presplit(fgv_block_state *S, const uint8_t *block, size_t len, std::vector<Span> &out);

using namespace fgvb;

namespace {
constexpr uint32_t kRoundsPerEnqueue = 6;  // fixpoint rounds enqueued before the first host check
constexpr uint64_t kMaxArena = 32ull << 30;  // StateSlot.off8 addresses 8-byte units with 32 bits
constexpr size_t kCounterBytes = 256;       // MvCounters, padded (head and tail)
}  // namespace

struct fgv_mvcc_state {
  uint64_t cap = 0, mask = 0, arena_cap = 0;
  uint64_t nkeys = 0, arena_used = 0;  // read back from `top` after every commit / load
  DevBuf tbl, arena, top;              // top: [0] arena bytes used, [1] occupied slots
  DevBuf head, info, reads, writes, btbl, wslot, rslot, bad, st, pend, tail;
  DevBuf lrecs, lbytes;                // load / apply staging
  HostBuf hhead, htail;
  std::vector<Span> pre_envs;          // envelope spans taken from a pre-split
  uint32_t epoch = 0;                  // block-table epoch (BlkSlot.owner)
  uint32_t rg = 0;                     // global fixpoint round tag (BlkSlot.fw_*)
  uint64_t btbl_cap = 0;
  uint32_t last_rounds = 0;
};

void fgv_mvcc_free(fgv_mvcc_state *M) {
  if (!M) return;
  DevBuf *d[] = {&M->tbl, &M->arena, &M->top, &M->head, &M->info, &M->reads, &M->writes, &M->btbl, &M->wslot,
                 &M->rslot, &M->bad, &M->st, &M->pend, &M->tail, &M->lrecs, &M->lbytes};
  for (auto *b : d) b->release();
  M->hhead.release();
  M->htail.release();
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
  if (!M->lbytes.ensure(kofs + kb + 64) || !M->lrecs.ensure(n * sizeof(MvRec)) || !M->pend.ensure(n + 64))
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
                     M->pend.as<uint8_t>(), nullptr);
  hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(n), dim3(256), 0, s, 0u, 0u, (uint32_t)n, lb,
                     M->lrecs.as<MvRec>(), M->pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask,
                     M->arena.as<uint8_t>(), M->top.as<unsigned long long>(), 0ull, nullptr);
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
  if (!M->tbl.ensure(cap * sizeof(StateSlot)) || !M->arena.ensure(arena) || !M->top.ensure(64)) return FGV_ENOMEM;
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

static int mvcc_validate(fgv_ctx *c, const uint8_t *block, size_t len, const uint8_t *d_block, uint64_t block_num,
                         uint8_t *flags, size_t ntx, int commit, const uint8_t *next, size_t next_len) {
  if (!c || !block || (ntx && !flags)) return FGV_EINVAL;
  if (len >= 0xFFFFFFFFull || ntx >= 0x7FFFFFFFull) return FGV_EINVAL;
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
  if (!M->hhead.ensure(hbytes) || !M->head.ensure(hbytes) || !M->info.ensure(ntx * sizeof(MvTxInfo)) ||
      !M->reads.ensure(rcap * sizeof(MvRec)) || !M->writes.ensure(rcap * sizeof(MvRec)) ||
      !M->wslot.ensure(rcap * 4) || !M->rslot.ensure(rcap * 4) || !M->pend.ensure(rcap + 64) ||
      !M->bad.ensure(ntx + 64) || !M->st.ensure(ntx + 64) || !M->tail.ensure(kCounterBytes + ntx + 64) ||
      !M->htail.ensure(kCounterBytes + ntx + 64))
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
  uint8_t *dh = M->head.as<uint8_t>();
  const uint32_t *d_et = reinterpret_cast<const uint32_t *>(dh);
  const uint8_t *d_in = dh + et_bytes;
  MvCounters *d_c = reinterpret_cast<MvCounters *>(dh + et_bytes + fl_bytes);
  MvTxInfo *d_info = M->info.as<MvTxInfo>();
  MvRec *d_r = M->reads.as<MvRec>(), *d_w = M->writes.as<MvRec>();
  BlkSlot *d_b = M->btbl.as<BlkSlot>();
  uint8_t *d_out = M->tail.as<uint8_t>() + kCounterBytes;
  const uint32_t N = (uint32_t)ntx;
  HIP_TRY(hipMemcpyAsync(dh, h, hbytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(M->bad.p, 0, ntx, s));
  HIP_TRY(hipEventRecord(c->ev[0], s));
  hipLaunchKernelGGL(k_mvx_count, dim3((N + 63) / 64), dim3(64), 0, s, N, dblk, d_et, d_in, d_info, d_c);
  hipLaunchKernelGGL(k_mvx_emit, dim3((N + 63) / 64), dim3(64), 0, s, N, dblk, d_info, d_r, d_w, d_c);
  hipLaunchKernelGGL(k_mvx_prep, grid_stride(rcap), dim3(256), 0, s, dblk, d_r, d_w, d_b, epoch,
                     M->wslot.as<uint32_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                     M->bad.as<uint8_t>(), d_c);
  HIP_TRY(hipEventRecord(c->ev[1], s));
  const uint32_t rg0 = M->rg;
  hipLaunchKernelGGL(k_mvx_find, grid_stride(rcap + ntx), dim3(256), 0, s, N, dblk, d_r, d_w, d_b, d_b, epoch,
                     M->wslot.as<uint32_t>(), M->rslot.as<uint32_t>(), d_info, M->bad.as<uint8_t>(),
                     M->st.as<uint8_t>(), rg0 + 1, d_c);
  // fixpoint rounds, enqueued ahead: a round after convergence exits at once
  uint32_t r = 0;
  auto enqueue = [&](uint32_t k) -> int {
    for (uint32_t q = 0; q < k; q++) {
      r++;
      hipLaunchKernelGGL(k_mvx_round, dim3((N + 63) / 64), dim3(64), 0, s, N, r, rg0 + r, d_info,
                         M->rslot.as<uint32_t>(), M->wslot.as<uint32_t>(), d_b, M->st.as<uint8_t>(), d_c);
    }
    hipLaunchKernelGGL(k_mvx_flags, grid_for(ntx), dim3(256), 0, s, N, r, d_in, d_info, M->st.as<uint8_t>(), d_out,
                       d_c);
    if (commit) {
      hipLaunchKernelGGL(k_mv_last, grid_stride(rcap), dim3(256), 0, s, r, d_w, M->wslot.as<uint32_t>(),
                         M->st.as<uint8_t>(), d_b, epoch, d_c, M->top.as<unsigned long long>(), M->cap, M->arena_cap);
      hipLaunchKernelGGL(k_mv_upsert_find, grid_stride(rcap), dim3(256), 0, s, 1u, r, 0u, dblk, d_w,
                         M->wslot.as<uint32_t>(), M->st.as<uint8_t>(), d_b, epoch, M->tbl.as<StateSlot>(), M->mask,
                         M->arena.as<uint8_t>(), block_num, M->pend.as<uint8_t>(), d_c);
      hipLaunchKernelGGL(k_mv_upsert_insert, grid_stride(rcap), dim3(256), 0, s, 1u, r, 0u, dblk, d_w,
                         M->pend.as<uint8_t>(), M->tbl.as<StateSlot>(), M->mask, M->arena.as<uint8_t>(),
                         M->top.as<unsigned long long>(), block_num, d_c);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(M->tail.p, d_c, sizeof(MvCounters), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemcpyAsync(M->htail.p, M->tail.p, kCounterBytes + ntx, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->ev[2], s));
    HIP_TRY(hipStreamSynchronize(s));
    return FGV_OK;
  };
  int rc = enqueue(kRoundsPerEnqueue);
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
  if (hc->unsup) return FGV_EUNSUPPORTED;  // nothing was committed
  if (commit) {
    rc = read_top(c, M);
    if (rc) return rc;
    if (hc->nomem) return FGV_ENOMEM;  // nothing was committed
  }
  memcpy(flags, M->htail.as<uint8_t>() + kCounterBytes, ntx);
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
