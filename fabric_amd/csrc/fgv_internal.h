// fgv_internal.h -- host-internal interfaces between fgv_host.cpp (context, device buffers,
// kernels) and fgv_block.cpp (block parse / fold).  Not part of the C ABI.
#pragma once
#include <cstdlib>
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include <array>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_kernels.h"

#define FGV_STAT_SUMS 25
struct fgv_block_state;
struct fgv_mvcc_state;
struct fgv_msp_cache;
struct ThreadPool;
namespace fgvb {
struct Channel;
}

namespace fgvh {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {  // pinned staging
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return false;
    cap = want;
    return true;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct KeyHash {
  size_t operator()(const std::array<uint8_t, 64> &k) const {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 64; i += 8) {
      uint64_t w;
      memcpy(&w, k.data() + i, 8);
      h = (h ^ w) * 1099511628211ull;
    }
    return (size_t)h;
  }
};

// big-endian 32 bytes -> 8 little-endian limbs
inline void be32_to_limbs(const uint8_t *b, uint32_t *l) {
  for (int i = 0; i < 8; i++) {
    const uint8_t *p = b + 4 * (7 - i);
    l[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
}

}  // namespace fgvh
using namespace fgvh;

// the finalize's plan for one batch (fgv_host.cpp fin_prepare)
struct FinPlan {
  uint64_t P = 0;
  size_t cap = 0, wn = 0, meta = 0;
};

struct fgv_p384_state;  // p384.hip: the context's P-384 keys and comb tables
struct fgv_ctx {
  fgv_mvcc_state *mv = nullptr;
  fgv_p384_state *p384 = nullptr;
  DevBuf kt_base;     // k_keybase: the window bases of the keys of one k_keytab launch
  DevBuf p384_items;  // fgv_p384_verify_msgs: item columns + signature bytes
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // k_der + k_inv of a block batch, concurrent with SHA-256
  hipStream_t stream3 = nullptr;  // the device-parse committer's non-payload SHA-256 (k_bd_sha)
  hipStream_t streamF = nullptr;  // the device-parse committer's front half (parse, identities, job counts)
  hipEvent_t ev[8] = {};          // 0/1 sha, 2/3 inv, 4/5 prep, 6 point end, 7 fork
  hipEvent_t kev[12] = {};        // per-kernel brackets of the device-parse committer (fgv_last_kernel_times)
  double t_kern[12] = {};
  uint64_t n_pay_blocks = 0;      // SHA-256 compressions of the payload hashes (last block call)
  std::mutex mu;
  // the generator comb, the key tiers (fgv_host.cpp): every key has an id;
  // kmap[id] = its slot in the comb-table cache or KEY_NONE (variable-base kernels)
  DevBuf g_ok;
  DevBuf key_ok;                // [id] the key is a P-256 point
  DevBuf gtab28, ktab28, redo;  // Montgomery-280 comb tables (k_point28); redo: kernel counters
  uint32_t key_slots = 0;       // comb slots (5.2 MB each)
  uint32_t key_ids = 0;         // id capacity
  uint32_t pinned = 0;          // ids [0, pinned): registered keys, for good; then ad-hoc ids up to n_ids
  uint32_t n_ids = 0;
  uint32_t n_vb = 0;            // ids without a comb (the variable-base kernels run when > 0)
  std::unordered_map<std::array<uint8_t, 64>, uint32_t, KeyHash> key_map;  // key -> id
  std::vector<std::array<uint8_t, 64>> id_key;  // id -> key
  std::vector<uint32_t> kmap_h;                 // host mirror of kmap
  std::vector<uint32_t> comb_owner;             // comb slot -> id (KEY_NONE: free)
  std::vector<uint32_t> comb_free;              // free comb slots (popped from the back)
  DevBuf kmap, vbt, vbuse, vbpromo, vblist, vbhand, vbacc, kt_id;
  uint32_t vbt_keys = 0;           // key ids vbt holds rows for (grown by doubling, up to key_ids)
  uint32_t vb_last_items = 0;      // the last read-back batch's variable-base items (k_vb_fin's grid)
  HostBuf h_promo, h_kid;       // the promotion queue read back (k_vb_mul -> streamV copy)
  hipStream_t streamV = nullptr;  // k_vb_mul: beside the hashes (u2 * Q needs no digest)
  hipStream_t streamK = nullptr;  // promotion comb builds (k_keytab + k_kmap_set), not waited on
  hipEvent_t kt_ev = nullptr;     // the last build on streamK (its staging buffers are reused)
  bool kt_busy = false;
  hipEvent_t vb_ev[3] = {};       // 0 the VB list is built (k_inv), 1 k_vb_mul done, 2 queue copied
  hipEvent_t vb_t[2] = {};        // k_vb_mul's bracket on streamV (timed calls)
  double t_vb = 0;                // k_vb_mul ms of the last timed call
  bool vb_timed = false;
  bool vb_pending = false;        // k_vb_mul enqueued: launch_prep_point adds k_vb_fin
  bool vb_copied = false;         // a promotion-queue copy was enqueued (vb_ev[2])
  bool vb_launched = false;       // the last verify stages ran the variable-base kernels
  uint32_t promote_uses = 256;    // variable-base verifies of one key before its comb is built (a 64 MiB
                                  // 17-bit comb repays its build over ~30k verifies: round 6, 64 -> 256)
  uint32_t adhoc_comb_uses = 32;  // uses of an ad-hoc key in one call for a comb
  // FGV_PROMOTE_AT = 1 / 2 / 3 (test knob, tests/test_gpu_concurrency.py): promotions build their
  // tables on the main stream and enqueue k_kmap_set after k_inv / before k_point28 / before
  // k_vb_fin of the consuming batch; kmap_defer = ids whose k_kmap_set is still to be enqueued
  hipEvent_t ext_ev = nullptr;  // fgv_stream_wait_external
  uint32_t promote_at = 0;
  uint32_t kmap_defer = 0;
  uint64_t n_promoted = 0;        // keys promoted to a comb since fgv_init
  uint32_t promote_per_call = 32; // comb builds from the promotion queue per call (FGV_PROMOTE_PER_CALL)
  std::vector<uint32_t> promo_backlog;  // queued ids not built yet (<= VB_BACKLOG_CAP while no comb slot is free)
  bool promote_fixed = false;  // FGV_PROMOTE_PER_CALL given: no scaling by call size
  // per-block outcomes (fgv_set_block_outcomes) and the fallback counters (fgv_unsupported_stats)
  bool block_outcomes = false;
  std::vector<int32_t> blk_status;
  int last_rc = FGV_OK;  // the last validate call's return code (fgv_last_block_status)
  size_t n_final = 0;
  uint64_t unsup_batches = 0, unsup_blocks = 0, unsup_txs = 0;
  // running sums of the per-call diagnostics (fgv_stats_sums): a benchmark reads them once after
  // its timed loop instead of one library call per step inside it
  double stat_sum[FGV_STAT_SUMS] = {};
  std::chrono::steady_clock::time_point t_call_end{};  // end of the last validation call
  double t_gap = 0, t_finish = 0;  // host ms: previous call's end -> first kernel; the finish after its wait
  fgv_block_state *blk = nullptr;
  DevBuf bj_jobs, bj_sigp, bj_sigl, bj_slot, bj_didx, bj_dig, bj_vst, blk_arena;
  HostBuf hb_dig, hb_vst;
  HostBuf hb_jobs, hb_sigp, hb_sigl, hb_slot, hb_didx;  // block-job staging (filled in place)
  // device finalize (finalize.hip)
  DevBuf fz_meta, fz_rowmap, fz_blkof, fz_owner, fz_minblk, fz_minvalid, fz_flags, fz_pslot, fz_res;
  HostBuf hb_fz, hb_fflags, hb_res;
  uint64_t fin_seed = 0;
  // early txid index of a single-device batch (fgv_finalize_early_index): set by the fused
  // validate call before the device enqueue, consumed by its finalize
  bool want_early_fin = false, early_fin = false;
  bool fold_codes = false;  // k_bd_fold ran the finalize's codes step (the finalize runs the rest)
  uint32_t *fold_unsup = nullptr;  // with fold_codes: the batch's flag word (k_fin_dups)
  // with fold_codes: the batch's 64 B of counters in HBM and its pinned host copy; k_fin_dups's last
  // workgroup writes them straight into the mapped host copy (fin_misc_done), no copy kernel
  const uint32_t *fin_misc_src = nullptr;
  uint32_t *fin_misc_dst = nullptr;
  bool fin_misc_done = false;
  bool defer_ahead = false;  // the fused call: the next front half after the finalize is queued
  bool early_fin_on = [] {  // A/B knob FGV_EARLY_FIN=0: the whole finalize after the fold
    const char *e = getenv("FGV_EARLY_FIN");
    return !(e && atoi(e) == 0);
  }();
  hipEvent_t fin_ev = nullptr;
  DevBuf fz_keys;
  uint32_t n_cu = 0;        // compute units (persistent k_point grid)
  uint32_t last_lanes = 0;  // lanes per verify of the last k_point launch
  // per-batch device buffers
  DevBuf kt_q, kt_slot, kt_scratch;
  DevBuf status, slot, r, s, dig, d1, wv, wscr, msg, moff, mlen;
  // pinned staging
  HostBuf h_status, h_slot, h_r, h_s, h_dig, h_kq, h_kslot, h_moff, h_mlen;
  double t_sha = 0, t_prep = 0, t_point = 0, t_keytab = 0;
  uint64_t n_sha_jobs = 0, n_sha_blocks = 0, n_verifies = 0;  // last call
  double t_mvcc_lookup = 0, t_mvcc_total = 0;
  double t_host_parse = 0, t_host_assemble = 0, t_host_device = 0, t_host_fold = 0;
  // the last validate call saw a tx that may change key-level state (a metadata write, a delete
  // of a key holding a parameter): a group with later blocks on another device is unsupported
  bool kl_changes = false;
  FinPlan early_plan;  // the plan fgv_finalize_early_index prepared (its metadata copy may be pending)
  uint64_t n_mvcc_reads = 0, n_mvcc_writes = 0;
  // deliver-side integrity (fgv_integrity.cpp): own host pool, own lock -- runs concurrently
  // with committer calls on the same context
  std::vector<ThreadPool *> integ_free;  // idle host pools (one per concurrent call, created on demand)
  std::mutex integ_mu;
  // device-resident committer path (blockdev.hip)
  bool stage_ran = false;
  hipEvent_t digests_ready = nullptr;  // k_prep waits for it when set (digests from another stream)
  hipEvent_t digests_ready2 = nullptr;  // ... and for this one (a second producing stream)
  bool last_presplit = false;  // the last device-parse call used a fgv_presplit result
  // fgv_validate_shard_dev_next: the batch to pre-split once this call's GPU work is queued
  struct NextBatch {
    size_t n = 0;
    const uint8_t *const *blocks = nullptr;
    const size_t *lens = nullptr;
    const uint32_t *lo = nullptr, *hi = nullptr;
    bool prefetch = false;  // also queue its H2D copy (host-resident batches)
    const uint8_t *const *d_blocks = nullptr;  // its device copy (known: its front half is enqueued ahead)
    hipEvent_t wait = nullptr;                 // ... once this event (the prefetch copy) has fired
  } next;
  bool last_ahead = false;  // the last device-parse call found its front half enqueued ahead
  int ahead_mode = 2;       // fgv_set_ahead: 0 off, 1 after the ECDSA kernels, 2 at once (default), 3 after the fold
  // fgv_set_timing: record the committer's timing-only events (per-kernel device times); each
  // is a timestamp packet on the critical path (~5 us on MI355X), so off by default
  bool timing = false;
  bool spin = false;  // FGV_SPIN=1: poll the committer's final wait (fgv_stream_wait; equal within noise on MI355X)
  bool timing_ran = true;  // the last verify stages recorded their events (read_stage_times)
  // host-resident batches: a ring of device staging arenas.  The running call's batch holds one;
  // batches staged ahead (the pipelined calls' NEXT batch, fgv_prefetch of later ones) hold the
  // others, filled on the copy stream while earlier batches validate
  static constexpr int kStage = 3;
  DevBuf stage[kStage];
  hipEvent_t stage_ev[kStage] = {};  // the slot's last staging copy
  int stage_cur = 0;                 // the slot of the batch the current / last call validated
  hipStream_t copy_stream = nullptr;
  struct Prefetch {
    int slot = 0;
    std::vector<const uint8_t *> src, dev;
    std::vector<size_t> lens;
    bool matches(size_t n, const uint8_t *const *b, const size_t *l) const {
      if (n != src.size()) return false;
      for (size_t i = 0; i < n; i++)
        if (src[i] != b[i] || lens[i] != l[i]) return false;
      return true;
    }
  };
  std::vector<Prefetch> pf;  // staged batches, oldest first (at most kStage - 1)
  uint64_t n_prefetch_hits = 0, h2d_bytes = 0;  // last call: blocks found prefetched / bytes copied in the call
  DevBuf bd_env, bd_bases, bd_tx, bd_ident, bd_jobs, bd_misc;
  HostBuf hb_env, hb_bases, hb_misc;
  double t_bd_split = 0, t_bd_pre = 0, t_bd_fold = 0;
  fgv_msp_cache *msp = nullptr;  // MSP models of the cache-miss path (fgv_msp.cpp)
};
void fgv_integrity_free(fgv_ctx *c);
// P-384 identities (p384.hip): register a key (X || Y big-endian, 96 B) -> its table index, the
// per-item verify launch over a verify list, teardown
int fgv_p384_key_locked(fgv_ctx *c, const uint8_t pub[96], uint32_t *idx);
uint32_t fgv_p384_nkeys(const fgv_ctx *c);
int fgv_p384_launch(fgv_ctx *c, hipStream_t st, uint32_t n, const uint32_t *dn, uint8_t *status, const uint64_t *sigp,
                    const uint32_t *sigl, const uint32_t *slot, const uint32_t *dig_idx, const uint8_t *digests);
void fgv_p384_free(fgv_ctx *c);

// Wait for a stream: polled (hipStreamQuery) when `spin`, else a blocking synchronize.  The
// committer's calls wait ~0.8 ms for their batch; polling returns as soon as the last copy lands
// instead of after the blocking wait's wake-up.
inline hipError_t fgv_stream_wait(hipStream_t s, bool spin) {
  if (!spin) return hipStreamSynchronize(s);
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    __builtin_ia32_pause();
  }
}

#define HIP_TRY(x)                                     \
  do {                                                 \
    if ((x) != hipSuccess) return FGV_EDEVICE;         \
  } while (0)


fgv_block_state *fgv_block_state_new(unsigned threads);
// per-block outcomes of the next validation (fgv_set_block_outcomes): on = per-transaction 0xFD
// codes and a split block instead of a whole-batch FGV_EUNSUPPORTED; split = UINT32_MAX: none
void fgv_block_set_soft(fgv_block_state *S, bool on);
uint32_t fgv_block_split(fgv_block_state *S);
bool fgv_block_soft_unsup(fgv_block_state *S);  // the last soft validation left a transaction undecided
// fgv_validate_shard_dev with per-block outcomes (fgv_group's soft calls): undecided transactions
// carry 0xFD in their records instead of failing the shard; *split = the first block of this
// call's list that must wait for an earlier block's commit (UINT32_MAX: none)
extern "C" int fgv_validate_shard_dev_soft(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                const uint32_t *tx_lo, const uint32_t *tx_hi, void *d_results, size_t results_cap,
                                size_t *ntx, uint32_t *split);
void fgv_block_state_free(fgv_block_state *s);

#include <functional>
void fgv_parallel_for(fgv_block_state *S, size_t n, const std::function<void(size_t)> &f);
// one job per index on the pool (no chunking: for a few long jobs)
void fgv_parallel_run(fgv_block_state *S, size_t n, const std::function<void(size_t)> &f);
void fgv_mvcc_free(fgv_mvcc_state *M);

int fgv_block_set_channel(fgv_block_state *S, const char *name);
int fgv_block_add_identity(fgv_block_state *S, const uint8_t *ser, size_t len, int32_t key_slot,
                           const fgv_identity_info *info);
int fgv_block_define_chaincode(fgv_block_state *S, const char *ns, const char *plugin, const uint8_t *policy,
                               size_t len, uint32_t flags);
int fgv_block_define_collection(fgv_block_state *S, const char *ns, const char *coll, const uint8_t *policy,
                                size_t len);
struct DevTx;
extern "C" int fgv_finalize_early_index(fgv_ctx *c, size_t nblocks, const size_t *ntx, const DevTx *dtx,
                                        const uint64_t *bases,
                             const uint8_t *digests, hipStream_t st);
int fgv_block_kvmeta_set(fgv_block_state *S, const std::string &ns, const std::string &coll, const uint8_t *key,
                         size_t key_len, const uint8_t *vp, size_t vp_len);
size_t fgv_block_kvmeta_count(fgv_block_state *S);
const std::string *fgv_block_kvmeta_get(fgv_block_state *S, const std::string &ns, const std::string &coll,
                                        const uint8_t *key, size_t key_len);
int fgv_block_channel_config(fgv_block_state *S, const uint8_t *config, size_t len);
int fgv_block_declare_msp(fgv_block_state *S, const char *mspid);
int fgv_block_add_txids(fgv_block_state *S, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                        size_t n);
int fgv_block_validate_impl(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                            const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                            const uint32_t *tx_hi, fgv_tx_result *res_out, size_t res_cap, size_t *ntx_out);
long fgv_block_count_txs(const uint8_t *b, size_t n);
// GetOrganizationalUnits of a registered identity (fgv_msp_identity_ous, the MSP cache miss)
int fgv_block_identity_ous(fgv_block_state *S, const uint8_t *ser, size_t len, size_t n, const char *const *ou,
                           const size_t *ou_lens, const uint8_t *const *certifiers, const size_t *cert_lens);
// the key-level batch rule of fgv_block_validate_impl over whole blocks (a group's device ranges
// together): FGV_EUNSUPPORTED when a block may change the parameter of a key a later block writes
// split (per-block outcomes): instead of FGV_EUNSUPPORTED, the first block that must wait for an
// earlier block's commit (UINT32_MAX: none)
int fgv_block_kl_check(fgv_block_state *S, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                       uint32_t *split = nullptr);
int fgv_finalize_impl(size_t nblocks, const size_t *ntx, const fgv_tx_result *res, uint8_t *flags);

// Pinned host staging for one block batch's device jobs (valid until the next reserve).
struct BlockJobs {
  ShaJob *jobs;
  uint64_t *sig_ptr;  // device address of each DER signature (0: empty)
  uint32_t *sig_len, *key_slot, *dig_idx;
};
int fgv_block_jobs_reserve(fgv_ctx *c, size_t nj, size_t nv, BlockJobs *out);
// Device pass: SHA-256 jobs -> digests (all nj), then ECDSA verify jobs whose digest is
// digests[dig_idx[i]] -> vstatus (nv).  Outputs point into pinned host buffers owned by the
// context.  sha_blocks: compressions of the batch (statistics).  Implemented in fgv_host.cpp.
int fgv_run_block_jobs(fgv_ctx *c, size_t nj, size_t nv, uint64_t sha_blocks, const uint8_t **digests,
                       const uint8_t **vstatus);
// device-resident variant: jobs already in c->bj_jobs / c->bj_sigp; results stay in HBM
// dig: the digest buffer (default c->bj_dig)
// dn: the verify count in device memory (nv = capacity, n_est = the host's estimate)
int fgv_run_block_jobs_device(fgv_ctx *c, size_t nj, size_t nv, uint64_t sha_blocks, size_t dig_off = 0,
                              const uint8_t *dig = nullptr, const uint32_t *dn = nullptr, size_t n_est = 0);
// wait for (and forget) a device-parse front half enqueued ahead of its call
void fgv_block_drain(fgv_ctx *c);
// the front half fgv_block_validate_dev_enqueue deferred (c->defer_ahead): launch it, or drop it
void fgv_block_launch_deferred_ahead(fgv_ctx *c, bool launch = true);
void fgv_read_block_job_times(fgv_ctx *c);
int fgv_verify_prefix_dev(fgv_ctx *c, hipStream_t st, size_t cap, const uint32_t *dn, const uint8_t *sigblk,
                          uint8_t *vst, DevBuf &r, DevBuf &s, DevBuf &w, DevBuf &wscr);
int fgv_verify_main_dev(fgv_ctx *c, size_t cap, const uint32_t *dn, size_t n_est, const uint8_t *sigblk, uint8_t *vst,
                        const uint32_t *r, const uint32_t *w, const uint8_t *digests);
int fgv_block_set_parse_mode(fgv_block_state *S, int mode);
int fgv_block_presplit(fgv_block_state *S, int device, size_t nblocks, const uint8_t *const *h_blocks,
                       const size_t *lens, const uint32_t *tx_lo, const uint32_t *tx_hi);
int fgv_block_parse_mode(fgv_block_state *S);
// device-resident committer pass (fgv_block.cpp + blockdev.hip): records -> d_res (HBM).
// Returns FGV_OK, FGV_EUNSUPPORTED, an error, or 1 = "a transaction exceeded a device
// capacity: run the host parser for this batch".
int fgv_block_validate_dev(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                           const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                           const uint32_t *tx_hi, fgv_tx_result *d_res, size_t res_cap, size_t *ntx_out);
// the same in two halves: _enqueue queues the whole batch (no host synchronisation) and returns
// FGV_OK or an error; more work may then be queued on c->stream behind it (the finalize
// kernels); _finish synchronises and returns fgv_block_validate_dev's outcome
int fgv_block_validate_dev_enqueue(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                                   const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                                   const uint32_t *tx_hi, fgv_tx_result *d_res, size_t res_cap, size_t *ntx_out);
int fgv_block_validate_dev_finish(fgv_ctx *c, fgv_block_state *S);

// identity.Verify(msg, sig) of registered identities (pinned key slots), host buffers; the
// caller holds c->mu (fgv_host.cpp)
int fgv_verify_msgs_slots_locked(fgv_ctx *c, const uint8_t *msg_buf, size_t msg_buf_len, const uint64_t *msg_off,
                                 const uint32_t *msg_len, const uint8_t *sig_buf, size_t sig_buf_len,
                                 const uint64_t *sig_off, const uint32_t *sig_len, const uint32_t *slots, size_t n,
                                 uint8_t *status_out);
// BlockHeaderBytes (protoutil/blockutils.go:48-67): ASN.1 DER of {number, previous_hash, data_hash}
void fgv_block_header_der(uint64_t number, const uint8_t *prev, size_t prev_n, const uint8_t *dh, size_t dh_n,
                          std::vector<uint8_t> &out);
// The orderer-signature input of one block (fgv_integrity.cpp -> fgv_block.cpp): the marshalled
// Metadata at metadata[SIGNATURES] and the header's BlockHeaderBytes
struct fgv_sig_block {
  bool want = false;  // evaluate this block (it passed every earlier check that needs no chain)
  const uint8_t *meta = nullptr;
  size_t meta_n = 0;
  std::vector<uint8_t> hdr_der;
};
#define FGV_SIGV_FAIL 0   // the verifier returns an error (policy unsatisfied, malformed metadata)
#define FGV_SIGV_OK 1
#define FGV_SIGV_UNSUP 2  // outside the engine's model: the reference decides
// BlockSignatureVerifier (protoutil/blockutils.go:245-290) + policy.EvaluateSignedData for every
// block with want set; locks c->mu (the channel model, the GPU verify).  policy: a channel policy
// path; bft: the channel runs BFT (identifier headers are then outside the model).
int fgv_block_sig_verdicts(fgv_ctx *c, size_t n, const fgv_sig_block *in, const char *policy, int bft,
                           uint8_t *verdict);

// registered (pinned) P-256 keys -> key ids; c->mu held (fgv_host.cpp).  want_comb[i] (nullable:
// all): the key is expected to be hot (a comb slot while one is free), else it starts on the
// variable-base kernels and is promoted by use
int fgv_keys_register_locked(fgv_ctx *c, const uint8_t *keys, size_t n, uint32_t *slots,
                             const uint8_t *want_comb = nullptr);
// the comb policy of an identity by its role bits (fgv_identity_info.roles): a definite client
// (CLIENT, and none of ADMIN / PEER / ORDERER: a NodeOU classification) signs rarely and starts on
// the variable-base kernels; every other identity (peers, orderers, admins, unknown roles, MSPs
// without NodeOUs) is expected to sign often.  Either way use promotes a key.
inline bool fgv_roles_want_comb(uint32_t roles) {
  if (roles & FGV_ROLES_UNKNOWN) return true;
  const bool client = (roles & (1u << 2)) != 0;
  return !client || (roles & ((1u << 1) | (1u << 3) | (1u << 4))) != 0;
}
// the channel model of a block state (fgv_block.cpp)
fgvb::Channel &fgv_block_channel(fgv_block_state *S);
// the identities a batch names (creators, endorsers) that the registry does not hold but a
// channel MSP may (Channel::lookup == -2), deduplicated (fgv_block.cpp)
void fgv_block_misses(fgv_block_state *S, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                      std::vector<std::string> &out);
// the MSP cache miss (fgv_msp.cpp); c->mu held.  registered: identities added to the registry
int fgv_msp_resolve_locked(fgv_ctx *c, size_t n, const uint8_t *const *ser, const size_t *lens, int *status,
                           size_t *registered);
int fgv_msp_resolve_blocks_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                  size_t *registered);
bool fgv_msp_auto(fgv_ctx *c);  // fgv_set_auto_resolve (default on)
void fgv_msp_cache_free(fgv_ctx *c);

// Sanitizer probes (tools/sanitize/harness.cpp): the host parsers alone, no GPU call
uint64_t fgv_block_parse_probe(const char *channel, const uint8_t *const *ids, const size_t *id_lens, size_t nids,
                               const char *ns, const uint8_t *policy, size_t policy_len, const uint8_t *blk,
                               size_t n);
uint64_t fgv_mvcc_parse_probe(const uint8_t *rws, size_t n);
uint64_t fgv_msp_config_probe(const uint8_t *conf, size_t n);
extern "C" int fgv_x509_probe(const uint8_t *pem, size_t n, char *out, size_t cap);
