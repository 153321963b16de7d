// fgv_block.cpp -- TxValidator.Validate for blocks of endorser transactions (libfgv.so).
//
// One call validates a batch of blocks (signatures of several blocks are verified in one GPU
// pass -- verify bits are pure functions of their inputs, so speculative batching is exact):
//   A. host, parallel over txs: single-pass protobuf parse of every envelope (pbwire.h, Go
//      protobuf-go rules) into a TxRec: every check of the reference that needs no crypto is
//      decided here, and hash / verify jobs are emitted for the rest;
//   B. device: k_sha256_jobs (creator payload, nonce||creator, chdr||shdr||ccpp,
//      prp||endorser -- spans read in place from the block bytes in HBM), k_der, k_prep,
//      k_point over every creator + endorsement signature;
//   C. host, parallel over txs: the reference's code precedence, cauthdsl policy folding over
//      the verify bits, then (serial) markTXIdDuplicates and the txid index across blocks.
//
// Reference (behaviour restated; citations under /root/reference):
//   core/committer/txvalidator/v20/validator.go:180-481, core/common/validation/msgvalidation.go
//   :26-320, plugindispatcher/dispatcher.go:102-302, builtin/v20/validation_logic.go:109-217,
//   statebased/validator_keylevel.go:38-282 + v20.go:105-167, core/policy/application.go:148-163,
//   common/cauthdsl/cauthdsl.go:24-92 + policy.go:86-108, common/policies/policy.go:363-395,
//   msp/identities.go:170-199, protoutil/{proputils.go:198-223,351-370, txutils.go:21-58,449-466,
//   503-534}.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_internal.h"
#include "thread_pool.h"
#include "pbwire.h"

#include "fgv_visitors.h"
#include "fgv_channel.h"
#include "blockdev.h"
#include "fin_dev.h"
#include "sha256_host.h"

// ======================================================================= channel model
// (fgv_channel.h)
namespace fgvb {
// ======================================================================= per-tx records
enum : uint8_t { C_VALID = 0, C_BAD_PAYLOAD = 2, C_BAD_HDR = 3, C_BAD_CREATOR = 4, C_BAD_ETX = 5,
                 C_UNSUP_PAYLOAD = 7, C_BAD_TXID = 8, C_DUP_TXID = 9, C_POLICY = 10,
                 C_BAD_HDR_EXT = 19, C_BAD_RESP = 21, C_BAD_RWSET = 22, C_ILLEGAL_WS = 23,
                 C_INVALID_CC = 25, C_OTHER = 255, C_PENDING = 0xFE, C_UNSUPPORTED = 0xFD };

// extractDependenciesForTx (validator_keylevel.go:184-222): an unmarshal error returns before
// the dependency is signalled (X_FAIL), Actions[0] of none / a nil action panic (X_PANIC)
enum : uint8_t { X_OK = 0, X_FAIL = 1, X_PANIC = 2, X_UNKNOWN = 0xFF };

struct EndRec {
  int ident = -1;
  uint32_t vjob = UINT32_MAX;  // verify job (UINT32_MAX: no verification possible)
  Span endorser, sig;
};

struct TxRec {
  uint8_t pre = C_PENDING;   // decided without crypto (final) or C_PENDING
  int32_t type = 0;
  Span payload, env_sig, nonce, creator, chdr, act_hdr, ccpp, prop_hash, prp, txid;
  int creator_ident = -1;
  uint8_t etx = C_PENDING;   // validateEndorserTransaction structural result (0 ok, 5, unsupported)
  uint8_t disp = C_PENDING;  // Dispatch structural result (0 ok -> policies)
  std::vector<int> policies;  // chaincode policy per written namespace (-1 unknown chaincode)
  std::vector<EndRec> ends;
  uint32_t cjob = UINT32_MAX, txid_job = UINT32_MAX, prop_job = UINT32_MAX, cvjob = UINT32_MAX;
  Span index_txid;         // GetOrComputeTxIDFromEnvelope (txid index): chdr.TxId when non-empty
  bool index_ok = false;   // index entry exists (chdr.TxId, or computed on the device)
  Span idx_nonce, idx_creator;  // for the computed txid when chdr.TxId is empty
  uint32_t index_job = UINT32_MAX;
  // device job counts of this tx, by kind (filled after parsing; see the assembly stage)
  uint8_t n_cj = 0, n_tj = 0, n_pj = 0, n_ij = 0;
  uint16_t n_ej = 0;
  // key-level endorsement (statebased/validator_keylevel.go, vpmanagerimpl.go)
  uint8_t xstat = X_UNKNOWN;  // extractDependenciesForTx outcome (X_OK / X_FAIL / X_PANIC)
  bool has_md = false;        // metadata writes (public or hashed) in some namespace
  bool vw = false;            // some vscc that runs reads a written key (GetValidationParameterForKey)
  bool vany = false;          // some vscc runs (PreValidate)
  bool vpns = false;          // writes a namespace the state holds key-level parameters for
  Span results, ccid;         // ChaincodeAction.results, the invoked chaincode

  void reset() {  // keep the vectors' capacity across calls
    std::vector<int> p = std::move(policies);
    std::vector<EndRec> e = std::move(ends);
    *this = TxRec();
    p.clear();
    e.clear();
    policies = std::move(p);
    ends = std::move(e);
  }
};

}  // namespace fgvb

// ======================================================================= context glue
using namespace fgvb;

// channel model image in HBM for the device-resident path (blockdev.h DevChannel)
struct DevImage {
  DevBuf name, idents, ibytes, itable, ihash, cc, colls, impl, msps, ccb, pol, nodes, kids, subs, prins, iou, committed,
      kvp, kvpb;
  DevChannel ch{};
  bool has_sha3 = false;  // an identity of a SHA3 MSP: the batch runs k_bd_sha3 (fgv_front_launch)
  void release() {
    for (DevBuf *b : {&name, &idents, &ibytes, &itable, &ihash, &cc, &colls, &impl, &msps, &ccb, &pol, &nodes, &kids,
                      &subs, &prins, &iou, &committed, &kvp, &kvpb})
      b->release();
  }
};

// Envelope spans of a batch (the block data framing walk, the only host-side parse of the
// device path) and the envelope table k_bd_parse reads: per transaction (block, offset, len).
struct SplitOut {
  std::vector<uint32_t> lo, hi;
  std::vector<size_t> ntx, first;
  size_t total = 0;
};

// A batch split ahead of its fgv_validate_shard_dev call (fgv_presplit): a peer walks block
// k+1's framing while block k validates.  The result is used only by a call whose batch --
// block addresses, lengths and shard ranges -- is the one split here.  One persistent worker
// thread (a thread start would cost more than the overlap gains).
static int split_batch(ThreadPool &pool, size_t nblocks, const uint8_t *const *h_blocks, const size_t *lens,
                       const uint32_t *tx_lo, const uint32_t *tx_hi, SplitOut &o, HostBuf &et);
// FGV_PRESPLIT_LOG=1: each pre-split walk's duration and each wait for one on stderr (profiling aid)
static bool presplit_log() {
  static const bool on = getenv("FGV_PRESPLIT_LOG") && atoi(getenv("FGV_PRESPLIT_LOG"));
  return on;
}

struct PreSplit {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  bool req = false, done = false, stop = false;
  bool active = false;  // requested and neither used nor discarded (owner thread only)
  int device = 0;
  std::vector<const uint8_t *> blocks;
  std::vector<size_t> lens;
  std::vector<uint32_t> lo_in, hi_in;
  int rc = FGV_OK;
  SplitOut out;
  HostBuf et;  // pinned envelope table, swapped with the context's on use
  std::unique_ptr<ThreadPool> pool;
  bool matches(size_t nb, const uint8_t *const *b, const size_t *l, const uint32_t *lo, const uint32_t *hi) const {
    if (nb != blocks.size() || (lo == nullptr) != lo_in.empty() || (hi == nullptr) != hi_in.empty()) return false;
    for (size_t i = 0; i < nb; i++)
      if (b[i] != blocks[i] || l[i] != lens[i] || (lo && lo[i] != lo_in[i]) || (hi && hi[i] != hi_in[i])) return false;
    return true;
  }
  void worker() {
    bool dev_set = false;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || req; });
      if (stop) return;
      req = false;
      lk.unlock();
      int r = FGV_OK;
      if (!dev_set) r = hipSetDevice(device) == hipSuccess ? FGV_OK : FGV_EDEVICE;  // (pinned staging)
      dev_set = r == FGV_OK;
      const bool log = presplit_log();
      const auto t0 = std::chrono::steady_clock::now();
      if (r == FGV_OK)
        r = split_batch(*pool, blocks.size(), blocks.data(), lens.data(), lo_in.empty() ? nullptr : lo_in.data(),
                        hi_in.empty() ? nullptr : hi_in.data(), out, et);
      if (log)
        fprintf(stderr, "[fgv] pre-split of %zu blocks: %.3f ms\n", blocks.size(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      lk.lock();
      rc = r;
      done = true;
      cv.notify_all();
    }
  }
  void start() {
    if (!th.joinable()) {
      pool.reset(new ThreadPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency()))));
      th = std::thread([this] { worker(); });
    }
    std::lock_guard<std::mutex> lk(mu);
    done = false;
    req = true;
    active = true;
    cv.notify_all();
  }
  bool ready() {  // the requested split is done (no wait)
    std::lock_guard<std::mutex> lk(mu);
    return done;
  }
  void join() {  // wait for the requested split (if any); the result stays readable
    if (!active) return;
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    active = false;
  }
  ~PreSplit() {
    join();
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
      cv.notify_all();
    }
    if (th.joinable()) th.join();
    et.release();
  }
};

// One batch's device-parse state.  There are two: batch k+1's front half (head upload, payload
// and message hashes, parse, identities, job counts -- the side streams) is enqueued while
// batch k's back half (verify jobs, ECDSA, fold -- the main stream) runs.
struct BdSet {
  DevBuf env, tx, ident, jobs, dig;  // env: envelope table | block bases | counters (the head)
  DevBuf klrec, klhead, kldep, kllist;  // key-level records, their buckets, dependencies (blockdev.h KlDev)
  // the batch's verify jobs (k_bd_emit columns), status, r / s / w limbs, k_inv scratch: per set,
  // so that k_bd_emit -> k_der -> k_inv of a batch can run ahead with its front half (vdone)
  DevBuf vsig, vst, vr, vs, vw, vscr;
  bool vdone = false;
  uint32_t prio = 2;  // the front chain's wave priority for this batch (front_launch_a)
  bool emitted = false;  // k_bd_count wrote the verify jobs (FGV_FUSE_EMIT, default): no k_bd_emit
  uint32_t klseq = 0;                   // the bucket tag of the batch this set holds
  KlDev kl{};
  HostBuf head, misc;                // pinned head staging / counters read back
  // 0 start, 1 payload hashes done (stream2), 2 k_bd_sha done (stream3), 3 head uploaded,
  // 4 parse done, 5 k_bd_sha start, 6 counts done, 7 k_bd_ident start (0, 5, 7: timing only),
  // 8 every digest done (stream3, after joining stream2: the back half waits on this one only),
  // 9 the verify prefix done (k_bd_emit, k_der, k_inv)
  hipEvent_t ev[10] = {};
  SplitOut so;
  bool presplit = false;
  bool force_host = false;  // a shard's block prefix writes metadata (host parser)
  const uint32_t *misc_src = nullptr;  // the batch counters in HBM (copied back by the finish)
  bool timed = false;  // its front half recorded the timing-only events
  hipStream_t stream = nullptr;  // the stream its parse / identity / count chain ran on
  size_t eoff = 0, moff = 0;
  uint32_t N = 0;
  // the batch this set holds (the match key of a front half enqueued ahead)
  std::vector<const uint8_t *> hb, db;
  std::vector<size_t> lens;
  std::vector<uint32_t> lo, hi;
  bool has_lo = false, has_hi = false;
  bool matches(size_t nb, const uint8_t *const *h, const size_t *l, const uint8_t *const *d, const uint32_t *lo_,
               const uint32_t *hi_) const {
    if (nb != hb.size() || (lo_ != nullptr) != has_lo || (hi_ != nullptr) != has_hi) return false;
    for (size_t i = 0; i < nb; i++)
      if (h[i] != hb[i] || l[i] != lens[i] || d[i] != db[i] || (lo_ && lo_[i] != lo[i]) || (hi_ && hi_[i] != hi[i]))
        return false;
    return true;
  }
  void release() {
    for (DevBuf *b : {&env, &tx, &ident, &jobs, &dig, &klrec, &klhead, &kldep, &kllist, &vsig, &vst, &vr, &vs, &vw,
                      &vscr})
      b->release();
    head.release();
    misc.release();
    for (auto &e : ev)
      if (e) hipEventDestroy(e);
  }
};

struct fgv_block_state {
  Channel ch;
  ThreadPool pool;
  // the two most recent pre-split requests (fgv_presplit): a call uses the one of its batch and
  // discards those requested before it, so a caller may walk batch k+2 while batch k+1's walk
  // waits for its call (FIFO of requests: pre_ord)
  PreSplit pre[2];
  uint64_t pre_ord[2] = {0, 0};
  uint64_t pre_next = 1;
  // per-call scratch
  std::vector<TxRec> recs;
  // device image of `ch`, rebuilt when the channel model changes (the committed txid table
  // alone when only ledger txids were added)
  DevImage dimg;
  bool dev_dirty = true;
  bool txid_dirty = false;
  int parse_mode = 0;  // 0: device parse (host parser for capacity overflows), 1: host parse
  BdSet set[2];
  int ahead = -1;  // set holding a front half enqueued ahead of its call (-1: none)
  int early = -1;  // set holding phase a of the next batch's front half, queued at the call's top
  double early_ms = 0;  // host time of that phase a
  int prefix_next = -1;  // set whose verify prefix the finish queues on the main stream (prefix_main)
  hipEvent_t done_ev = nullptr;  // the call's own work on the main stream (the finish waits on it)
  bool ahead_deferred = false;  // a front half to launch once the caller's finalize is queued
  fgv_ctx::NextBatch ahead_nx{};
  int ahead_cur = 0;
  int last = 1;    // set of the last call
  int pending = -1;           // set enqueued by _enqueue and not yet finished
  double nv_per_tx = 0;       // verifies per tx of the last batch (lanes-per-verify estimate)
  // per-block outcomes (fgv_set_block_outcomes) of the running call: soft = report instead of
  // failing the batch; split = the first block that must wait for an earlier block's commit
  bool soft = false;
  bool soft_unsup = false;  // the soft call marked some transaction undecided (0xFD)
  uint32_t split = UINT32_MAX;
  uint32_t klseq = 0;         // key-level bucket tags (blockdev.h KlDev::seq), one per front half
  std::chrono::steady_clock::time_point t_enq;
  explicit fgv_block_state(unsigned threads) : pool(threads) {}
  ~fgv_block_state() {
    if (done_ev) hipEventDestroy(done_ev);
    dimg.release();
    set[0].release();
    set[1].release();
  }
};

fgv_block_state *fgv_block_state_new(unsigned threads) { return new fgv_block_state(threads); }
void fgv_block_set_soft(fgv_block_state *S, bool on) {
  S->soft = on;
  S->soft_unsup = false;
  S->split = UINT32_MAX;
}
bool fgv_block_soft_unsup(fgv_block_state *S) { return S->soft_unsup; }
uint32_t fgv_block_split(fgv_block_state *S) { return S->split; }
Channel &fgv_block_channel(fgv_block_state *S) { return S->ch; }
void fgv_parallel_for(fgv_block_state *S, size_t n, const std::function<void(size_t)> &f) {
  S->pool.parallel_for(n, f);
}
void fgv_parallel_run(fgv_block_state *S, size_t n, const std::function<void(size_t)> &f) { S->pool.run(n, f); }
void fgv_block_state_free(fgv_block_state *s) { delete s; }

// ======================================================================= parsing
// metadata writes in a TxReadWriteSet (rwset.FromProtoBytes: any decode error -> none)
static bool rwset_has_md(const Span &results) {
  VTxRwSet rw;
  if (!pbw::decode(results.p, results.n, rw)) return false;
  bool md = false;
  for (size_t k = 0; k < rw.ns.size(); k++) {
    VKVRWSet kv;
    if (!pbw::decode(rw.ns[k].rwset.p, rw.ns[k].rwset.n, kv)) return false;
    md |= kv.nmeta != 0;
    for (const VCollHashed &c : rw.ns[k].coll) {
      VHashedRWSet h;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) return false;
      md |= h.nmeta != 0;
    }
  }
  return md;
}

// extractDependenciesForTx (validator_keylevel.go:184-222) for a tx whose validation walk
// stopped before its ChaincodeAction
static void extract_walk(Span d, TxRec &R) {
  R.xstat = X_FAIL;
  VEnvelope env;
  if (!pbw::decode(d.p, d.n, env)) return;
  VPayload pl;
  VHeader hdr;
  if (!pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.decode_into(hdr)) return;
  VTransaction tx;
  if (!pbw::decode(pl.data.p, pl.data.n, tx)) return;
  if (tx.actions.size() == 0) { R.xstat = X_PANIC; return; }
  VCcActionPayload cap;
  if (!pbw::decode(tx.actions[0].payload.p, tx.actions[0].payload.n, cap)) return;
  if (!cap.has_action) { R.xstat = X_PANIC; return; }
  VPrp prp;
  if (!pbw::decode(cap.action.prp.p, cap.action.prp.n, prp)) return;
  VCcAction cca;
  if (!pbw::decode(prp.extension.p, prp.extension.n, cca)) return;
  R.xstat = X_OK;
  R.results = cca.results;
  R.has_md = rwset_has_md(cca.results);
}

static void parse_tx_flow(const Channel &ch, Span d, TxRec &R);
static void parse_tx(const Channel &ch, Span d, TxRec &R) {
  R.reset();
  parse_tx_flow(ch, d, R);
  if (R.xstat == X_UNKNOWN) extract_walk(d, R);
}

static void parse_tx_flow(const Channel &ch, Span d, TxRec &R) {
  VEnvelope env;
  if (!pbw::decode(d.p, d.n, env)) { R.pre = C_OTHER; return; }
  VPayload pl;
  VHeader hdr;
  if (!pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.decode_into(hdr)) {
    R.pre = C_BAD_PAYLOAD;
    return;
  }
  // txid index value (protoutil.GetOrComputeTxIDFromEnvelope, txutils.go:503-534)
  if (pl.header.present) {
    VChannelHeader c0;
    if (pbw::decode(hdr.channel_header.p, hdr.channel_header.n, c0)) {
      if (c0.tx_id.n) {
        R.index_txid = c0.tx_id;
        R.index_ok = true;
      } else {
        VSignatureHeader s0;
        if (pbw::decode(hdr.signature_header.p, hdr.signature_header.n, s0)) {
          R.index_ok = true;  // computed on the device (ComputeTxID)
          R.idx_nonce = s0.nonce;
          R.idx_creator = s0.creator;
        }
      }
    }
  }
  if (!pl.header.present) { R.pre = C_BAD_HDR; return; }
  VChannelHeader chdr;
  VSignatureHeader shdr;
  if (!pbw::decode(hdr.channel_header.p, hdr.channel_header.n, chdr) ||
      !pbw::decode(hdr.signature_header.p, hdr.signature_header.n, shdr)) {
    R.pre = C_BAD_HDR;
    return;
  }
  if (chdr.type != 3 && chdr.type != 2 && chdr.type != 1) { R.pre = C_BAD_HDR; return; }
  if (chdr.epoch != 0 || shdr.nonce.nil() || shdr.creator.nil()) { R.pre = C_BAD_HDR; return; }
  R.type = chdr.type;
  R.payload = env.payload;
  R.env_sig = env.signature;
  R.nonce = shdr.nonce;
  R.creator = shdr.creator;
  R.chdr = hdr.channel_header;
  R.txid = chdr.tx_id;
  // checkSignatureFromCreator (msgvalidation.go:26-64)
  if (env.signature.nil()) { R.pre = C_BAD_CREATOR; return; }
  if (chdr.channel_id.n == 0) { R.pre = C_UNSUPPORTED; return; }  // peer-local MSP
  if (!chdr.channel_id.eq(ch.name.data(), ch.name.size())) { R.pre = C_BAD_CREATOR; return; }
  // DeserializeIdentity -> Validate -> Verify (msgvalidation.go:26-64)
  R.creator_ident = ch.lookup(shdr.creator);
  if (R.creator_ident == -2) { R.pre = C_UNSUPPORTED; return; }  // unregistered certificate of a channel MSP
  if (R.creator_ident < 0) { R.pre = C_BAD_CREATOR; return; }
  const Ident &ci = ch.idents[R.creator_ident];
  if (!ci.valid || ci.verify_class_tx() == 1) { R.pre = C_BAD_CREATOR; return; }
  if (ci.verify_class_tx() == 2) { R.pre = C_UNSUPPORTED; return; }  // P-384 key
  if (chdr.type != 3) return;  // CONFIG (unsupported) / CONFIG_UPDATE (7) decided in the fold

  // validateEndorserTransaction (msgvalidation.go:165-245)
  R.etx = C_BAD_ETX;
  if (pl.data.nil()) return;
  VTransaction tx;
  if (!pbw::decode(pl.data.p, pl.data.n, tx) || tx.actions.size() != 1) return;
  const VTransactionAction &act = tx.actions[0];
  VSignatureHeader ash;
  if (!pbw::decode(act.header.p, act.header.n, ash) || ash.nonce.nil() || ash.creator.nil()) return;
  VCcActionPayload cap;
  if (!pbw::decode(act.payload.p, act.payload.n, cap)) return;
  if (!cap.has_action) { R.etx = C_UNSUPPORTED; return; }  // reference dereferences nil (panic)
  VPrp prp;
  if (!pbw::decode(cap.action.prp.p, cap.action.prp.n, prp)) return;
  if (cap.ccpp.nil() || act.header.nil()) return;  // GetProposalHash2 nil arguments
  R.etx = C_VALID;
  R.act_hdr = act.header;
  R.ccpp = cap.ccpp;
  R.prop_hash = prp.proposal_hash;
  R.prp = cap.action.prp;

  // Dispatch (dispatcher.go:102-221)
  VHdrExt ext;
  if (!pbw::decode(chdr.extension.p, chdr.extension.n, ext)) { R.disp = C_BAD_HDR_EXT; return; }
  // GetActionFromEnvelope: same bytes as above; failure points re-checked in order
  if (cap.action.prp.nil()) { R.disp = C_BAD_RESP; return; }
  if (prp.extension.nil()) { R.disp = C_BAD_RESP; return; }
  VCcAction cca;
  if (!pbw::decode(prp.extension.p, prp.extension.n, cca)) { R.disp = C_BAD_RESP; return; }
  R.xstat = X_OK;  // (the dependency extraction decodes the same messages)
  R.results = cca.results;
  VTxRwSet rw;
  if (!pbw::decode(cca.results.p, cca.results.n, rw)) { R.disp = C_BAD_RWSET; return; }
  // per namespace: 1 = writes (kv / metadata / collection), 2 = metadata writes, 4 = public
  // writes; the collections with hashed writes (policyCheckerV20 collection EPs)
  pbw::SmallVec<uint8_t, 8> wflags;
  pbw::SmallVec<std::pair<uint32_t, Span>, 8> wcolls;  // (namespace index, collection name)
  for (size_t k = 0; k < rw.ns.size(); k++) {
    VKVRWSet kv;
    if (!pbw::decode(rw.ns[k].rwset.p, rw.ns[k].rwset.n, kv)) { R.disp = C_BAD_RWSET; return; }
    bool coll_writes = false, coll_meta = false;
    for (const VCollHashed &c : rw.ns[k].coll) {
      VHashedRWSet h;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) { R.disp = C_BAD_RWSET; return; }
      if (h.nwrites) wcolls.push_back({(uint32_t)k, c.name});
      coll_writes |= h.nwrites != 0;
      coll_meta |= h.nmeta != 0;
    }
    wflags.push_back((uint8_t)(((kv.nwrites || kv.nmeta || coll_writes || coll_meta) ? 1 : 0) |
                               ((kv.nmeta || coll_meta) ? 2 : 0) | (kv.nwrites ? 4 : 0)));
  }
  for (uint8_t f : wflags) R.has_md |= (f & 2) != 0;
  if (!ext.has_ccid || !cca.has_ccid) { R.disp = C_OTHER; return; }
  const Span ccid = ext.ccid.name;
  R.ccid = ccid;
  if (ccid.n == 0 || !ccid.eq(reinterpret_cast<const char *>(cca.ccid.name.p), cca.ccid.name.n) ||
      cca.ccid.version.n == 0) {
    R.disp = C_INVALID_CC;
    return;
  }
  if (!cca.events.nil()) {
    VCcEvent ev;
    if (!pbw::decode(cca.events.p, cca.events.n, ev) ||
        !ev.chaincode_id.eq(reinterpret_cast<const char *>(ccid.p), ccid.n)) {
      R.disp = C_OTHER;
      return;
    }
  }
  // duplicate namespace -> ILLEGAL_WRITESET (any duplicate: the reference stops at the first)
  pbw::SmallVec<Span, 8> nss;
  for (size_t k = 0; k < rw.ns.size(); k++) nss.push_back(rw.ns[k].ns);
  std::sort(nss.begin(), nss.end());
  for (size_t k = 1; k < nss.size(); k++)
    if (nss[k].eq(nss[k - 1])) { R.disp = C_ILLEGAL_WS; return; }
  // written namespaces + the invoked chaincode
  pbw::SmallVec<Span, 8> wr;
  wr.push_back(ccid);
  for (size_t k = 0; k < rw.ns.size(); k++) {
    if (!(wflags[k] & 1)) continue;
    if (!rw.ns[k].ns.eq(ccid)) wr.push_back(rw.ns[k].ns);
  }
  std::sort(wr.begin(), wr.end());
  R.disp = C_VALID;
  // the policies each namespace's vscc evaluates (statebased/validator_keylevel.go:87-143,
  // v20.go:105-167) when no written key has a key-level parameter and no metadata is written
  // (those txs take the sequential fold): public writes -> the chaincode EP; a collection with
  // hashed writes -> its collection EP (or the chaincode EP; the collection "" is the public
  // path); none of these -> the chaincode EP.  -1: INVALID_CHAINCODE, -2: outside the model.
  auto push = [&](int p) {
    if (std::find(R.policies.begin(), R.policies.end(), p) == R.policies.end()) R.policies.push_back(p);
  };
  for (const Span &ns : wr) {
    auto it = ch.ccs.find(ns.str());
    if (it == ch.ccs.end() || it->second.status == 1) { push(-1); continue; }
    const CCInfo &cc = it->second;
    R.vany = true;
    if (cc.status != 0) { push(-2); continue; }
    int k = -1;
    for (size_t q = 0; q < rw.ns.size(); q++)
      if (rw.ns[q].ns.eq(ns)) { k = (int)q; break; }
    if (k >= 0 && (wflags[k] & 1)) {
      R.vw = true;
      R.vpns |= cc.has_vp;
    }
    bool any = false;
    if (k >= 0 && (wflags[k] & 4)) { push(cc.ep); any = true; }
    for (const auto &wc : wcolls) {
      if ((int)wc.first != k) continue;
      any = true;
      if (wc.second.n == 0) { push(cc.ep); continue; }  // GetStateMetadata + CheckCCEPIfNotChecked(cc, "")
      const std::string coll = wc.second.str();
      if (coll.compare(0, strlen(kImplicitPrefix), kImplicitPrefix) == 0) {
        auto ie = ch.implicit_ep.find(coll.substr(strlen(kImplicitPrefix)));
        push(ie == ch.implicit_ep.end() ? -2 : ie->second);
        continue;
      }
      if (!cc.colls_known) { push(-2); continue; }
      auto ce = cc.colls.find(coll);
      push(ce == cc.colls.end() ? 0 : ce->second < 0 ? cc.ep : ce->second);  // "no such collection" -> reject
    }
    if (!any) push(cc.ep);
  }
  // endorsement signature set (validator_keylevel.go:246-260)
  R.ends.resize(cap.action.ends.size());
  for (size_t k = 0; k < cap.action.ends.size(); k++) {
    EndRec &e = R.ends[k];
    e.endorser = cap.action.ends[k].endorser;
    e.sig = cap.action.ends[k].signature;
    e.ident = ch.lookup(e.endorser);
  }
}

// ======================================================================= policy fold
// cauthdsl greedy evaluation (common/cauthdsl/cauthdsl.go:24-92) over the deduplicated,
// verified signers `ids`: SignedBy takes the first unused signer satisfying the principal;
// NOutOf evaluates every sub-rule on a copy of `used` and keeps the copy when it succeeds.
struct UsedBits {  // <= 64 signers
  uint64_t w = 0;
  bool get(size_t i) const { return (w >> i) & 1; }
  void set(size_t i) { w |= 1ull << i; }
};
struct UsedVec {
  std::vector<uint8_t> v;
  bool get(size_t i) const { return v[i] != 0; }
  void set(size_t i) { v[i] = 1; }
};
static_assert(DPR_ROLE == PR_ROLE && DPR_IDENTITY == PR_IDENTITY && DPR_OU == PR_OU && DPR_NOMINAL == PR_NOMINAL &&
                  DPR_NEVER == PR_NEVER && DPR_UNRESOLVED == PR_UNRESOLVED,
              "device principal kinds");
// SatisfiesPrincipal of one leaf (msp/mspimpl.go:477-660, MSP v1.4.3): 1 / 0 / 2 (unknown)
static int prin_sat(const Prin &p, const Ident &I) {
  switch (p.kind) {
    case PR_ROLE:  // same MSP; MEMBER = Validate, other roles from the MSP layer's role bits
      return I.msp == p.msp && (p.role == 0 ? I.valid : ((I.roles >> p.role) & 1u) != 0);
    case PR_IDENTITY:  // the same sanitized certificate (cert.Raw) of the same MSP, then Validate
      return I.canon == p.canon && I.msp == p.msp && I.valid;
    case PR_OU:  // same MSP, Validate, then one of its (OU, certifier) pairs
      if (I.msp != p.msp || !I.valid) return 0;
      if (!I.ous_known) return 2;
      return std::find(I.ous.begin(), I.ous.end(), p.ou) != I.ous.end();
    case PR_NOMINAL: return 1;
    case PR_UNRESOLVED: return 2;
    default: return 0;
  }
}
// the leaves of one SignedBy principal, in collectPrincipals order: the first error decides
static int principal_sat(const Policy &P, int pr, const Ident &I) {
  int r = 1;
  for (uint32_t k = P.prin_off[pr], e = k + P.prin_cnt[pr]; k < e; k++) {
    const int v = prin_sat(P.prins[k], I);
    if (v == 0) return 0;
    if (v == 2) r = 2;
  }
  return r;
}
template <class U>
static int eval_node(const Policy &P, int node, const int *ids, size_t nids, const Channel &ch, U &used) {
  const PNode &N = P.nodes[node];
  if (N.type == 2) {
    for (size_t i = 0; i < nids; i++) {
      if (used.get(i)) continue;
      const int v = principal_sat(P, N.principal, ch.idents[ids[i]]);
      if (v == 2) return 2;  // (the greedy choice depends on it)
      if (v == 1) {
        used.set(i);
        return 1;
      }
    }
    return 0;
  }
  int32_t verified = 0;
  for (int k : N.kids) {
    U tmp = used;
    const int v = eval_node(P, k, ids, nids, ch, tmp);
    if (v == 2) return 2;
    if (v == 1) {
      verified++;
      used = std::move(tmp);
    }
  }
  return verified >= N.n;
}
// 1 satisfied, 0 not, 2 outside the model
static int eval_policy(const Channel &ch, int pi, const int *ids, size_t nids, int depth = 0) {
  const Policy &P = ch.policies[pi];
  switch (P.kind) {
    case PK_REJECT: return 0;
    case PK_SIG: {
      if (!P.decode_ok || !P.compile_ok) return 0;
      if (P.needs_roles)
        for (size_t i = 0; i < nids; i++)
          if (!ch.idents[ids[i]].roles_known) return 2;
      if (nids <= 64) {
        UsedBits u;
        return eval_node(P, P.root, ids, nids, ch, u);
      }
      UsedVec u;
      u.v.assign(nids, 0);
      return eval_node(P, P.root, ids, nids, ch, u);
    }
    case PK_IMPLICIT: {  // ImplicitMetaPolicy.EvaluateSignedData (implicitmeta.go:69-104)
      if (depth > 0) return 2;
      int ok = 0;
      for (int s : P.subs) {
        const int v = eval_policy(ch, s, ids, nids, depth + 1);
        if (v == 2) return 2;
        ok += v;
      }
      // threshold 0 (no sub-policies, or an unknown rule): `remaining` starts at 0 and every
      // satisfied sub-policy drives it negative, so only "none satisfied" succeeds
      return (P.threshold == 0 ? ok == 0 : ok >= P.threshold) ? 1 : 0;
    }
    default: return 2;
  }
}

// ======================================================================= API
static bool hex32(const Span &s, uint8_t out[32]) {
  if (s.n != 64) return false;
  for (int k = 0; k < 64; k++) {
    const uint8_t ch = s.p[k];
    int v;
    if (ch >= '0' && ch <= '9') v = ch - '0';
    else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
    else return false;  // only lowercase hex can equal a VALID txid (ComputeTxID output)
    if (k & 1) out[k >> 1] |= (uint8_t)v;
    else out[k >> 1] = (uint8_t)(v << 4);
  }
  return true;
}

// device jobs of one parsed tx, by kind (see the assembly stage)
static void count_jobs(const Channel &ch, TxRec &R) {
  if (R.index_ok && R.index_txid.n == 0) R.n_ij = 1;
  if (R.pre != C_PENDING) return;
  R.n_cj = 1;
  if (R.type != 3) return;
  R.n_tj = 1;
  if (R.etx != C_VALID) return;
  R.n_pj = 1;
  if (R.disp != C_VALID) return;
  uint32_t ne = 0;
  for (const EndRec &e : R.ends)
    if (e.ident >= 0 && ch.idents[e.ident].verify_class_tx() == 0) ne++;
  R.n_ej = (uint16_t)std::min<uint32_t>(ne, 0xFFFF);
}

// ======================================================================= key-level endorsement
// KeyLevelValidationParameterManagerImpl's per-block state (vpmanagerimpl.go:113-233), restated
// for a fold in block order: the metadata writers of every key, and each tx's vscc result per
// namespace -- VR_PASS (nil), VR_FAIL, VR_INDET (whether it runs depends on Go map order);
// absent: it never runs, so a later GetValidationParameterForKey waiting on it never returns.
enum : int8_t { VR_FAIL = 0, VR_PASS = 1, VR_INDET = 2 };
static inline std::string_view sv(const Span &s) { return std::string_view(reinterpret_cast<const char *>(s.p), s.n); }
struct SbeBlock {
  std::unordered_map<std::string, std::vector<uint32_t>> deps;  // kvkey -> metadata writers (tx index)
  std::vector<std::vector<std::pair<std::string, int8_t>>> res;  // per tx index of the block
  int result(uint32_t j, std::string_view ns) const {
    if (j >= res.size()) return -1;
    for (const auto &p : res[j])
      if (p.first == ns) return p.second;
    return -1;
  }
};

// ExtractValidationParameterDependency (vpmanagerimpl.go:258-292): the metadata-write keys of
// every namespace; a rwset that does not decode adds none
static void add_deps(const Span &results, uint32_t i, SbeBlock &B) {
  VTxRwSet rw;
  if (!pbw::decode(results.p, results.n, rw)) return;
  std::vector<std::string> keys;
  for (const VNsRwSet &n : rw.ns) {
    std::vector<Span> mk;
    VKVRWSet kv;
    kv.meta_keys = &mk;
    if (!pbw::decode(n.rwset.p, n.rwset.n, kv)) return;
    for (const Span &k : mk) keys.push_back(Channel::kvkey(sv(n.ns), "", sv(k)));
    for (const VCollHashed &c : n.coll) {
      std::vector<Span> hk;
      VHashedRWSet h;
      h.meta_keys = &hk;
      if (!pbw::decode(c.hashed.p, c.hashed.n, h)) return;
      for (const Span &k : hk) keys.push_back(Channel::kvkey(sv(n.ns), sv(c.name), sv(k)));
    }
  }
  for (std::string &k : keys) B.deps[std::move(k)].push_back(i);
}

// The builtin vscc v20 of one namespace (validator_keylevel.go:87-143 over policyCheckerV20,
// v20.go:105-167): per written key -- public writes, public metadata writes, hashed writes,
// hashed metadata writes -- an earlier valid metadata writer fails it (ValidationParameterUpdated-
// Error), else its key-level parameter, else CheckCCEPIfNotChecked; none -> the chaincode EP.
// 1 nil, 0 an error, 2 outside the model.  Every step is evaluated (the reference returns at the
// first error; the outcomes are pure, so the verdict is the same) and a step outside the model
// anywhere makes the tx unsupported, as in the oracle.  `hang`: an earlier tx never signalled
// its dependencies (GetValidationParameterForKey would wait forever).
// touched != null (the parallel first pass): an earlier metadata writer of a key only sets
// *touched -- the tx is folded again in block order once the writers' results are final.
static int sbe_vscc(const Channel &ch, const CCInfo &cc, std::string_view ns, const VNsRwSet *nrw, uint32_t i,
                    const SbeBlock &B, bool hang, const std::function<int(int)> &eval, bool *touched = nullptr) {
  int ok = 1;
  bool some = false, cc_checked = false;
  pbw::SmallVec<Span, 4> colls_checked;
  auto step = [&](const Span &coll, const Span &key) -> bool {  // false: outside the model
    some = true;
    if (hang) return false;
    auto d = B.deps.find(Channel::kvkey(ns, sv(coll), sv(key)));
    bool updated = false;
    if (d != B.deps.end())
      for (uint32_t j : d->second) {
        if (j >= i) continue;
        if (touched) {
          *touched = true;
          continue;
        }
        const int r = B.result(j, ns);
        if (r < 0 || r == VR_INDET) return false;
        updated |= r == VR_PASS;
      }
    if (updated) { ok = 0; return true; }
    const int pi = ch.kv_policy(ns, sv(coll), sv(key));
    if (pi == -3) return false;
    if (pi >= 0) {
      const int v = eval(pi);
      ok &= v;
      return v != 2;
    }
    if (coll.n) {
      for (const Span &c : colls_checked)
        if (c.eq(coll)) return true;
      const std::string cs = coll.str();
      int cp;
      if (cs.compare(0, strlen(kImplicitPrefix), kImplicitPrefix) == 0) {
        auto ie = ch.implicit_ep.find(cs.substr(strlen(kImplicitPrefix)));
        if (ie == ch.implicit_ep.end()) return false;
        cp = ie->second;
      } else {
        if (!cc.colls_known) return false;
        auto ce = cc.colls.find(cs);
        if (ce == cc.colls.end()) { ok = 0; return true; }  // no such collection -> policyErr
        cp = ce->second;
      }
      if (cp >= 0) {
        const int v = eval(cp);
        ok &= v;
        colls_checked.push_back(coll);
        return v != 2;
      }
    }
    if (!cc_checked) {
      const int v = eval(cc.ep);
      ok &= v;
      cc_checked = true;
      return v != 2;
    }
    return true;
  };
  if (nrw) {
    std::vector<VKVWrite> ws;
    std::vector<Span> mk;
    VKVRWSet kv;
    kv.writes = &ws;
    kv.meta_keys = &mk;
    if (!pbw::decode(nrw->rwset.p, nrw->rwset.n, kv)) return 2;  // (decoded by the parse already)
    std::vector<std::vector<VHashWrite>> hw(nrw->coll.size());
    std::vector<std::vector<Span>> hm(nrw->coll.size());
    for (size_t c = 0; c < nrw->coll.size(); c++) {
      VHashedRWSet h;
      h.writes = &hw[c];
      h.meta_keys = &hm[c];
      if (!pbw::decode(nrw->coll[c].hashed.p, nrw->coll[c].hashed.n, h)) return 2;
    }
    const Span pub{};
    for (const VKVWrite &w : ws)
      if (!step(pub, w.key)) return 2;
    for (const Span &k : mk)
      if (!step(pub, k)) return 2;
    for (size_t c = 0; c < nrw->coll.size(); c++)
      for (const VHashWrite &w : hw[c])
        if (!step(nrw->coll[c].name, w.key)) return 2;
    for (size_t c = 0; c < nrw->coll.size(); c++)
      for (const Span &k : hm[c])
        if (!step(nrw->coll[c].name, k)) return 2;
  }
  if (!some) return eval(cc.ep);  // CheckCCEPIfNoEPChecked (FAB-9473)
  return ok;
}

// (oracle keylevel_writes) the kvkeys one tx may change the key-level state of -- its metadata
// writes, its deletes of keys holding a VALIDATION_PARAMETER (tx_ops.go:17-51) -- and every key it
// writes or metadata-writes; nothing when the rwset does not decode
static void kl_keys(const Channel &ch, const Span &results, std::vector<std::string> &changed,
                    std::vector<std::string> &touched) {
  VTxRwSet rw;
  if (!pbw::decode(results.p, results.n, rw)) return;
  std::vector<std::string> c, t;
  for (const VNsRwSet &n : rw.ns) {
    std::vector<VKVWrite> ws;
    std::vector<Span> mk;
    VKVRWSet kv;
    kv.writes = &ws;
    kv.meta_keys = &mk;
    if (!pbw::decode(n.rwset.p, n.rwset.n, kv)) return;
    for (const VKVWrite &w : ws) {
      t.push_back(Channel::kvkey(sv(n.ns), "", sv(w.key)));
      if (w.is_delete && ch.kvmeta.count(t.back())) c.push_back(t.back());
    }
    for (const Span &k : mk) t.push_back(Channel::kvkey(sv(n.ns), "", sv(k))), c.push_back(t.back());
    for (const VCollHashed &cl : n.coll) {
      std::vector<VHashWrite> hw;
      std::vector<Span> hk;
      VHashedRWSet h;
      h.writes = &hw;
      h.meta_keys = &hk;
      if (!pbw::decode(cl.hashed.p, cl.hashed.n, h)) return;
      for (const VHashWrite &w : hw) {
        t.push_back(Channel::kvkey(sv(n.ns), sv(cl.name), sv(w.key)));
        if (w.is_delete && ch.kvmeta.count(t.back())) c.push_back(t.back());
      }
      for (const Span &k : hk) t.push_back(Channel::kvkey(sv(n.ns), sv(cl.name), sv(k))), c.push_back(t.back());
    }
  }
  changed.insert(changed.end(), c.begin(), c.end());
  touched.insert(touched.end(), t.begin(), t.end());
}

// GetOrComputeTxIDFromEnvelope (protoutil/txutils.go:503-534): the txid index entry of one
// envelope (chdr.TxId, or hex(SHA-256(nonce || creator)) when it is empty); false: none
static bool index_entry(const Span &d, std::string &out) {
  VEnvelope env;
  VPayload pl;
  VHeader hdr;
  if (!pbw::decode(d.p, d.n, env) || !pbw::decode(env.payload.p, env.payload.n, pl) || !pl.header.decode_into(hdr) ||
      !pl.header.present)
    return false;
  VChannelHeader c0;
  if (!pbw::decode(hdr.channel_header.p, hdr.channel_header.n, c0)) return false;
  if (c0.tx_id.n) {
    out.assign(reinterpret_cast<const char *>(c0.tx_id.p), c0.tx_id.n);
    return true;
  }
  VSignatureHeader s0;
  if (!pbw::decode(hdr.signature_header.p, hdr.signature_header.n, s0)) return false;
  std::string m(reinterpret_cast<const char *>(s0.nonce.p), s0.nonce.n);
  m.append(reinterpret_cast<const char *>(s0.creator.p), s0.creator.n);
  uint8_t dg[32];
  fgvsha::sha256(reinterpret_cast<const uint8_t *>(m.data()), m.size(), dg);
  static const char HX[] = "0123456789abcdef";
  out.resize(64);
  for (int k = 0; k < 32; k++) out[2 * k] = HX[dg[k] >> 4], out[2 * k + 1] = HX[dg[k] & 15];
  return true;
}

static inline uint32_t sha_blocks(const ShaJob &j) { return (j.n[0] + j.n[1] + j.n[2] + 8) / 64 + 1; }

int fgv_block_validate_impl(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                            const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                            const uint32_t *tx_hi, fgv_tx_result *res_out, size_t res_cap, size_t *ntx_out) {
  Channel &ch = S->ch;
  if (ch.dirty) ch.compile();
  using clk = std::chrono::steady_clock;
  auto t_start = clk::now();
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  // --- block envelopes (shard: transactions [tx_lo[b], tx_hi[b]) of block b)
  std::vector<std::vector<Span>> envs(nblocks);
  std::vector<uint32_t> lo(nblocks), hi(nblocks);
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) {
    if (tx_lo && tx_lo[b] == FGV_SHARD_SKIP) {  // another rank's block: not parsed
      ntx_out[b] = 0;
      lo[b] = hi[b] = 0;
      continue;
    }
    VBlock blk;
    if (!pbw::decode(h_blocks[b], lens[b], blk)) return FGV_EINVAL;  // unparsable block
    envs[b] = std::move(blk.data.data);
    ntx_out[b] = envs[b].size();
    lo[b] = tx_lo ? std::min<uint32_t>(tx_lo[b], (uint32_t)envs[b].size()) : 0;
    hi[b] = tx_hi ? std::min<uint32_t>(tx_hi[b], (uint32_t)envs[b].size()) : (uint32_t)envs[b].size();
    if (hi[b] < lo[b]) hi[b] = lo[b];
    total += hi[b] - lo[b];
  }
  if (total > res_cap) return FGV_EINVAL;
  // Blocks the reference cannot validate (key-level dependency tracking, validator_keylevel.go:
  // 184-241): a tx whose dependency extraction failed before a later tx's vscc reads a written
  // key, or panicked before a later tx's vscc runs.  Per block, the first such tx index; a shard
  // starting inside a block walks the block's earlier transactions too.
  std::vector<uint32_t> xfail(nblocks, UINT32_MAX), xpanic(nblocks, UINT32_MAX);
  bool sequential = false;
  std::vector<std::vector<std::pair<uint32_t, Span>>> pre_md(nblocks);  // prefix metadata writers
  for (size_t b = 0; b < nblocks; b++)
    for (uint32_t i = 0; i < lo[b]; i++) {
      TxRec tmp;
      extract_walk(envs[b][i], tmp);
      if (tmp.xstat == X_FAIL) xfail[b] = std::min(xfail[b], i);
      if (tmp.xstat == X_PANIC) xpanic[b] = std::min(xpanic[b], i);
      if (tmp.has_md) pre_md[b].push_back({i, tmp.results}), sequential = true;
    }
  // Shadow transactions (a shard split inside a block): the metadata writers before
  // this rank's range are validated here too -- parsed, verified and folded in block order like the
  // rank's own, their records dropped -- so a dependent whose writer another rank holds reads that
  // writer's vscc result per namespace (vpmanagerimpl.go:296-355 SetTxValidationResult /
  // GetValidationParameterForKey) instead of staying undecided.  Every writer a shadow depends on
  // is an earlier metadata writer, so the set is closed.  Metadata writers are rare: the extra
  // work is a handful of transactions per split block.
  size_t nshadow = 0;
  for (size_t b = 0; b < nblocks; b++)
    if (hi[b] > lo[b]) nshadow += pre_md[b].size();
  const size_t total_all = total + nshadow;
  std::vector<TxRec> &recs = S->recs;
  if (recs.size() < total_all) recs.resize(total_all);
  std::vector<std::pair<uint32_t, uint32_t>> where(total_all);
  std::vector<uint32_t> outpos(total_all, UINT32_MAX);  // the record's row in res_out (shadows: none)
  for (size_t b = 0, t = 0, r = 0; b < nblocks; b++) {
    if (hi[b] > lo[b])
      for (const auto &pm : pre_md[b]) where[t++] = {(uint32_t)b, pm.first};
    for (size_t i = lo[b]; i < hi[b]; i++) outpos[t] = (uint32_t)r++, where[t++] = {(uint32_t)b, (uint32_t)i};
  }
  std::vector<fgv_tx_result> shadow_res(nshadow ? total_all : 0);
  auto res_at = [&](size_t t) -> fgv_tx_result & { return outpos[t] != UINT32_MAX ? res_out[outpos[t]] : shadow_res[t]; };

  // --- A. parse (every check that needs no crypto) + per-tx device job counts
  S->pool.parallel_for(total_all, [&](size_t t) {
    TxRec &R = recs[t];
    parse_tx(ch, envs[where[t].first][where[t].second], R);
    count_jobs(ch, R);
  });
  c->t_host_parse = ms_since(t_start);
  auto t_asm = clk::now();

  // --- assemble device jobs, grouped by kind so the lanes of a wave hash similar lengths:
  //     sha  [creator payload | nonce||creator | chdr||shdr||ccpp | prp||endorser | index txid]
  //     ecdsa [creator signatures | endorsement signatures]
  // chunked exclusive scan over the per-tx counts, then a parallel fill of pinned buffers
  constexpr size_t CH = 256;
  const size_t nch = (total_all + CH - 1) / CH;
  std::vector<std::array<uint32_t, 5>> cbase(nch + 1);
  S->pool.run(nch, [&](size_t k) {
    std::array<uint32_t, 5> a{};
    for (size_t t = k * CH, e = std::min(total_all, t + CH); t < e; t++) {
      const TxRec &R = recs[t];
      a[0] += R.n_cj; a[1] += R.n_tj; a[2] += R.n_pj; a[3] += R.n_ej; a[4] += R.n_ij;
    }
    cbase[k + 1] = a;
  });
  cbase[0] = {};
  for (size_t k = 0; k < nch; k++)
    for (int q = 0; q < 5; q++) cbase[k + 1][q] += cbase[k][q];
  const std::array<uint32_t, 5> cnt = cbase[nch];
  const uint32_t kbase[5] = {0, cnt[0], cnt[0] + cnt[1], cnt[0] + cnt[1] + cnt[2],
                             cnt[0] + cnt[1] + cnt[2] + cnt[3]};
  const size_t nj = (size_t)kbase[4] + cnt[4], nv = (size_t)cnt[0] + cnt[3];
  BlockJobs J;
  int rc = fgv_block_jobs_reserve(c, nj, nv, &J);
  if (rc) return rc;
  auto dev_addr = [&](size_t b, const Span &s) -> uint64_t {
    return s.n ? (uint64_t)(uintptr_t)d_blocks[b] + (uint64_t)(s.p - h_blocks[b]) : 0;
  };
  std::vector<uint64_t> chunk_blocks(nch, 0);
  S->pool.run(nch, [&](size_t k) {
    uint32_t o[5];
    for (int q = 0; q < 5; q++) o[q] = kbase[q] + cbase[k][q];
    uint32_t ov0 = cbase[k][0], ov3 = cnt[0] + cbase[k][3];
    uint64_t nb = 0;
    auto job = [&](uint32_t idx, size_t b, Span s0, Span s1 = Span(), Span s2 = Span()) {
      ShaJob &j = J.jobs[idx];
      j.p[0] = dev_addr(b, s0); j.n[0] = s0.n;
      j.p[1] = dev_addr(b, s1); j.n[1] = s1.n;
      j.p[2] = dev_addr(b, s2); j.n[2] = s2.n;
      j.pad = 0;
      nb += sha_blocks(j);
    };
    auto verify = [&](uint32_t vi, size_t b, Span sig, int32_t slot, uint32_t dig) {
      J.sig_ptr[vi] = dev_addr(b, sig);
      J.sig_len[vi] = sig.n;
      J.key_slot[vi] = (uint32_t)slot;
      J.dig_idx[vi] = dig;
    };
    for (size_t t = k * CH, e = std::min(total_all, t + CH); t < e; t++) {
      TxRec &R = recs[t];
      const size_t b = where[t].first;
      if (R.n_cj) {
        R.cjob = o[0]++;
        job(R.cjob, b, R.payload);
        if (ch.idents[R.creator_ident].hash3) J.jobs[R.cjob].pad = SHAJOB_SHA3;  // SHA3 MSP
        R.cvjob = ov0++;
        verify(R.cvjob, b, R.env_sig, ch.idents[R.creator_ident].key_slot, R.cjob);
      }
      if (R.n_tj) job(R.txid_job = o[1]++, b, R.nonce, R.creator);
      if (R.n_pj) job(R.prop_job = o[2]++, b, R.chdr, R.act_hdr, R.ccpp);
      if (R.n_ej) {
        uint32_t left = R.n_ej;
        for (EndRec &e2 : R.ends) {
          if (!left) break;
          if (e2.ident < 0 || ch.idents[e2.ident].verify_class_tx() != 0) continue;
          const uint32_t hj = o[3]++;
          job(hj, b, R.prp, e2.endorser);
          if (ch.idents[e2.ident].hash3) J.jobs[hj].pad = SHAJOB_SHA3;
          e2.vjob = ov3++;
          verify(e2.vjob, b, e2.sig, ch.idents[e2.ident].key_slot, hj);
          left--;
        }
      }
      if (R.n_ij) job(R.index_job = o[4]++, b, R.idx_nonce, R.idx_creator);
    }
    chunk_blocks[k] = nb;
  });
  uint64_t nblk = 0;
  for (uint64_t x : chunk_blocks) nblk += x;
  c->t_host_assemble = ms_since(t_asm);

  // --- B. device
  auto t_dev = clk::now();
  const uint8_t *digests = nullptr, *vstatus = nullptr;
  rc = fgv_run_block_jobs(c, nj, nv, nblk, &digests, &vstatus);
  if (rc) return rc;
  c->t_host_device = ms_since(t_dev);
  auto t_fold = clk::now();

  // --- C. fold (code precedence, validator.go:297-453) + result records
  for (size_t t = 0; t < total_all; t++) {
    const TxRec &R = recs[t];
    const size_t b = where[t].first;
    const uint32_t i = where[t].second;
    if (R.xstat == X_FAIL) xfail[b] = std::min(xfail[b], i);
    if (R.xstat == X_PANIC) xpanic[b] = std::min(xpanic[b], i);
    sequential |= R.has_md || R.vpns;
  }
  // key-level endorsement state (a batch with metadata writes or writes to keys with parameters)
  std::vector<SbeBlock> sbe(sequential ? nblocks : 0);
  if (sequential) {
    for (size_t b = 0; b < nblocks; b++) {
      sbe[b].res.resize(hi[b]);
      for (const auto &pm : pre_md[b]) add_deps(pm.second, pm.first, sbe[b]);
    }
    for (size_t t = 0; t < total_all; t++)  // (the shadows were added as prefix writers)
      if (outpos[t] != UINT32_MAX && recs[t].has_md && recs[t].xstat == X_OK)
        add_deps(recs[t].results, where[t].second, sbe[where[t].first]);
  }
  // The batch validates every block against the key-level state committed before it, but the
  // reference commits block k before block k+1's vscc reads GetStateMetadata.  A key whose
  // parameter an earlier block may change (metadata write; delete of a key holding one) and a
  // later block writes: the outcome depends on block k's validity and MVCC -> unsupported (oracle
  // check_keylevel_batch).  Another rank's later block (SKIP) is walked when its bytes are there;
  // an empty placeholder is unknown: a change before it is enough.
  c->kl_changes = false;
  if (sequential) {
    std::vector<std::vector<std::string>> chg(nblocks), tch(nblocks);
    std::vector<uint8_t> unknown(nblocks, 0);
    for (size_t b = 0; b < nblocks; b++) {
      if (tx_lo && tx_lo[b] == FGV_SHARD_SKIP) {
        VBlock blk;
        if (!lens[b] || !pbw::decode(h_blocks[b], lens[b], blk)) {
          unknown[b] = 1;
          continue;
        }
        for (const Span &d : blk.data.data) {
          TxRec tmp;
          extract_walk(d, tmp);
          if (tmp.xstat == X_OK) kl_keys(ch, tmp.results, chg[b], tch[b]);
        }
        continue;
      }
      for (uint32_t i = 0; i < (uint32_t)envs[b].size(); i++) {
        if (i >= lo[b] && i < hi[b]) continue;  // (another rank's transactions of this block)
        TxRec tmp;
        extract_walk(envs[b][i], tmp);
        if (tmp.xstat == X_OK) kl_keys(ch, tmp.results, chg[b], tch[b]);
      }
    }
    for (size_t t = 0; t < total_all; t++)  // (shadows: walked above as other ranks' transactions)
      if (outpos[t] != UINT32_MAX && recs[t].xstat == X_OK) kl_keys(ch, recs[t].results, chg[where[t].first], tch[where[t].first]);
    std::unordered_set<std::string> changed;
    for (size_t b = 0; b < nblocks && b < S->split; b++) {
      if (unknown[b]) {
        if (!changed.empty()) {
          if (!S->soft) return FGV_EUNSUPPORTED;
          S->split = (uint32_t)b;  // (another rank's block whose bytes are not here: it waits)
          break;
        }
        continue;
      }
      bool dep = false;
      for (const std::string &k : tch[b]) dep |= changed.count(k) != 0;
      if (dep) {
        if (!S->soft) return FGV_EUNSUPPORTED;
        S->split = (uint32_t)b;  // per-block outcomes: this block and the later ones wait
        break;
      }
      changed.insert(chg[b].begin(), chg[b].end());
    }
    c->kl_changes = !changed.empty();
  }
  // A metadata writer whose txid an earlier block of the batch indexes is a ledger duplicate in the
  // reference (block k's txids are committed before block k+1 validates), so its vscc never runs
  // and a later dependent waits forever.  The first block indexing each txid (every block the
  // call has bytes for; a block before b without bytes: unknown -> its results are undecided).
  std::unordered_map<std::string, uint32_t> first_index;
  std::vector<uint8_t> index_unknown(nblocks, 0);
  if (sequential && nblocks > 1) {
    std::vector<std::vector<std::string>> keys(nblocks);
    std::vector<uint8_t> nobytes(nblocks, 0);
    S->pool.run(nblocks, [&](size_t b) {
      if (tx_lo && tx_lo[b] == FGV_SHARD_SKIP) {
        VBlock blk;
        if (!lens[b] || !pbw::decode(h_blocks[b], lens[b], blk)) { nobytes[b] = 1; return; }
        std::string k;
        for (const Span &d : blk.data.data)
          if (index_entry(d, k)) keys[b].push_back(k);
        return;
      }
      std::string k;
      for (const Span &d : envs[b])
        if (index_entry(d, k)) keys[b].push_back(k);
    });
    bool unknown = false;
    for (size_t b = 0; b < nblocks; b++) {
      index_unknown[b] = unknown;
      unknown |= nobytes[b] != 0;
      for (std::string &k : keys[b]) first_index.emplace(std::move(k), (uint32_t)b);
    }
  }
  auto batch_dup = [&](const Span &txid, size_t b) {
    auto it = first_index.find(std::string(reinterpret_cast<const char *>(txid.p), txid.n));
    return it != first_index.end() && it->second < b;
  };
  static const char HEX[] = "0123456789abcdef";
  // pass 0: no key-level state (parallel); 1: key-level, every tx in parallel, a tx whose written
  // key has an earlier metadata writer only marked; 2: the marked txs again, in block order
  std::vector<uint8_t> touched(sequential ? total_all : 0, 0);
  std::vector<uint8_t> cfg_blk(nblocks, 0);  // blocks with a CONFIG transaction reaching Apply
  auto fold_one = [&](size_t t, int pass) {
    const TxRec &R = recs[t];
    const size_t b = where[t].first;
    const uint32_t bi = where[t].second;
    uint8_t code;
    bool reached = false;
    if (R.pre != C_PENDING) {
      code = R.pre;
    } else if (vstatus[R.cvjob] != 0) {
      code = C_BAD_CREATOR;
    } else if (R.type == 1) {
      code = C_UNSUPPORTED;  // CONFIG transaction (validator.go:397-420: ChannelResources.Apply)
      cfg_blk[b] = 1;        // per-block outcomes: the later blocks wait for its commit
    } else if (R.type == 2) {
      code = C_UNSUP_PAYLOAD;
    } else {
      // CheckTxID: hex(SHA-256(nonce||creator)) == chdr.TxId
      const uint8_t *d = &digests[(size_t)R.txid_job * 32];
      bool ok = R.txid.n == 64;
      for (int k = 0; ok && k < 32; k++)
        ok = R.txid.p[2 * k] == (uint8_t)HEX[d[k] >> 4] && R.txid.p[2 * k + 1] == (uint8_t)HEX[d[k] & 15];
      if (!ok) {
        code = C_BAD_TXID;
      } else if (R.etx != C_VALID) {
        code = R.etx;
      } else if (R.prop_hash.n != 32 || memcmp(&digests[(size_t)R.prop_job * 32], R.prop_hash.p, 32) != 0) {
        code = C_BAD_ETX;
      } else if ((reached = true, ch.is_committed(R.txid))) {
        code = C_DUP_TXID;  // checkTxIdDupsLedger (initial ledger; batch-earlier blocks: finalize)
      } else if (pass != 0 && batch_dup(R.txid, b)) {
        code = C_DUP_TXID;  // (the finalize marks it too; here its vscc must not run)
      } else if (R.disp != C_VALID) {
        code = R.disp;
      } else if ((R.vany && xpanic[b] < bi) || (R.vw && xfail[b] < bi)) {
        code = C_UNSUPPORTED;  // the reference panics / waits forever (validator_keylevel.go:184-241)
      } else {
        // SignatureSetToValidIdentities (policy.go:363-395): deserialize, dedup, verify; only
        // when some policy is evaluated
        pbw::SmallVec<int, 16> ids;
        bool ids_done = false, ids_unsup = false;
        auto get_ids = [&] {
          if (ids_done) return;
          ids_done = true;
          pbw::SmallVec<uint32_t, 16> seen;
          for (const EndRec &e : R.ends) {
            if (e.ident == -2) { ids_unsup = true; return; }
            if (e.ident < 0) continue;
            const Ident &I = ch.idents[e.ident];
            if (std::find(seen.begin(), seen.end(), I.canon) != seen.end()) continue;
            const int vc = I.verify_class_tx();
            if (vc == 2) { ids_unsup = true; return; }
            if (vc == 1 || e.vjob == UINT32_MAX || vstatus[e.vjob] != 0) continue;
            seen.push_back(I.canon);
            ids.push_back(e.ident);
          }
        };
        bool has25 = false, has10 = false, unsup = false;
        if (pass == 0) {
          for (int pi : R.policies) {
            if (pi == -2) { unsup = true; break; }
            if (pi == -1) { has25 = true; continue; }
            get_ids();
            if (ids_unsup) { unsup = true; break; }
            const int v = eval_policy(ch, pi, ids.data(), ids.size());
            if (v == 2) { unsup = true; break; }
            if (v == 0) has10 = true;
          }
        } else {
          // Dispatch over the written namespaces (dispatcher.go:185-214) with the key-level
          // vscc; each namespace's result is recorded for the block's later transactions
          auto eval = [&](int pi) -> int {
            get_ids();
            return ids_unsup ? 2 : eval_policy(ch, pi, ids.data(), ids.size());
          };
          VTxRwSet rw;
          pbw::decode(R.results.p, R.results.n, rw);  // (decoded by the parse already)
          pbw::SmallVec<Span, 8> wr;
          pbw::SmallVec<int, 8> wk;
          wr.push_back(R.ccid);
          for (size_t k = 0; k < rw.ns.size(); k++) {
            VKVRWSet kv;
            pbw::decode(rw.ns[k].rwset.p, rw.ns[k].rwset.n, kv);
            bool w = kv.nwrites || kv.nmeta;
            for (const VCollHashed &c : rw.ns[k].coll) {
              VHashedRWSet h;
              pbw::decode(c.hashed.p, c.hashed.n, h);
              w |= h.nwrites || h.nmeta;
            }
            if (w && !rw.ns[k].ns.eq(R.ccid)) wr.push_back(rw.ns[k].ns);
          }
          std::sort(wr.begin(), wr.end());
          pbw::SmallVec<int, 8> rs;  // -1 INVALID_CHAINCODE, 0 / 1 vscc result, 2 outside the model
          for (const Span &ns : wr) {
            int k = -1;
            for (size_t q = 0; q < rw.ns.size(); q++)
              if (rw.ns[q].ns.eq(ns)) { k = (int)q; break; }
            auto it = ch.ccs.find(ns.str());
            int r;
            if (it == ch.ccs.end() || it->second.status == 1) r = -1;
            else if (it->second.status != 0) r = 2;
            else {
              bool tch = false;
              r = sbe_vscc(ch, it->second, sv(ns), k >= 0 ? &rw.ns[k] : nullptr, bi, sbe[b], xfail[b] < bi, eval,
                           pass == 1 ? &tch : nullptr);
              if (tch) touched[t] = 1;
            }
            rs.push_back(r);
          }
          sbe[b].res[bi].clear();
          for (size_t q = 0; q < wr.size(); q++) {
            unsup |= rs[q] == 2;
            has25 |= rs[q] == -1;
            has10 |= rs[q] == 0;
          }
          for (size_t q = 0; q < wr.size(); q++) {
            if (rs[q] != 0 && rs[q] != 1) continue;
            bool others = index_unknown[b] != 0;  // (it may be a ledger duplicate: undecided)
            for (size_t o = 0; o < wr.size(); o++) others |= o != q && (rs[o] == -1 || rs[o] == 0);
            sbe[b].res[bi].push_back({wr[q].str(), others ? VR_INDET : (int8_t)rs[q]});
          }
        }
        code = C_VALID;
        if (unsup) code = C_UNSUPPORTED;
        else if (has25 && has10) code = C_UNSUPPORTED;  // Go map order decides the reported code
        else if (has25) code = C_INVALID_CC;
        else if (has10) code = C_POLICY;
      }
    }
    fgv_tx_result &o = res_at(t);
    memset(&o, 0, sizeof o);
    o.code = code;
    if (reached) {  // chdr.TxId == hex(digest): the record carries the digest bytes
      memcpy(o.txid, &digests[(size_t)R.txid_job * 32], 32);
      o.flags |= FGV_TXR_REACHED;
    }
    // txid index entry for later blocks of this batch: chdr.TxId, or when empty
    // ComputeTxID(nonce, creator) (protoutil/txutils.go:503-534)
    if (R.index_ok) {
      if (R.index_txid.n == 0) {
        memcpy(o.index_txid, &digests[(size_t)R.index_job * 32], 32);
        o.flags |= FGV_TXR_INDEXED;
      } else if (hex32(R.index_txid, o.index_txid)) {
        o.flags |= FGV_TXR_INDEXED;
      }
    }
  };
  if (sequential) {  // block order for the txs that read the vscc results of earlier ones
    S->pool.parallel_for(total_all, [&](size_t t) { fold_one(t, 1); });
    for (size_t t = 0; t < total_all; t++)
      if (touched[t]) fold_one(t, 2);
  } else {
    S->pool.parallel_for(total_all, [&](size_t t) { fold_one(t, 0); });
  }
  c->t_host_fold = ms_since(t_fold);
  for (size_t b = 0; b < nblocks; b++)
    if (cfg_blk[b]) {
      S->split = std::min<uint32_t>(S->split, (uint32_t)b + 1);
      break;
    }
  // (from the final codes: a pass-1 verdict of a tx folded again in pass 2 does not count;
  // per-block outcomes: the codes stay, 0xFD marking the undecided transactions)
  for (size_t t = 0; t < total; t++)
    if (res_out[t].code == C_UNSUPPORTED) {
      if (!S->soft) return FGV_EUNSUPPORTED;
      S->soft_unsup = true;
      break;
    }
  return FGV_OK;
}

int fgv_block_kl_check(fgv_block_state *S, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                       uint32_t *split) {
  if (split) *split = UINT32_MAX;
  Channel &ch = S->ch;
  if (ch.dirty) ch.compile();
  std::vector<std::vector<std::string>> chg(nblocks), tch(nblocks);
  std::vector<int> bad(nblocks, 0);
  S->pool.parallel_for(nblocks, [&](size_t b) {
    VBlock blk;
    if (!pbw::decode(blocks[b], lens[b], blk)) { bad[b] = 1; return; }
    for (const Span &d : blk.data.data) {
      TxRec tmp;
      extract_walk(d, tmp);
      if (tmp.xstat == X_OK) kl_keys(ch, tmp.results, chg[b], tch[b]);
    }
  });
  std::unordered_set<std::string> changed;
  for (size_t b = 0; b < nblocks; b++) {
    if (bad[b]) return FGV_EINVAL;
    for (const std::string &k : tch[b])
      if (changed.count(k)) {
        if (!split) return FGV_EUNSUPPORTED;
        *split = (uint32_t)b;  // per-block outcomes: this block and the later ones wait
        return FGV_OK;
      }
    changed.insert(chg[b].begin(), chg[b].end());
  }
  return FGV_OK;
}

// number of transactions of a block (-1 if the block does not decode)
long fgv_block_count_txs(const uint8_t *b, size_t n) {
  VBlock blk;
  if (!pbw::decode(b, n, blk)) return -1;
  return (long)blk.data.data.size();
}

// markTXIdDuplicates + the txid index of earlier blocks of the batch (see fgv.h)
struct Key32Hash {
  size_t operator()(const std::array<uint8_t, 32> &k) const {
    uint64_t h;
    memcpy(&h, k.data(), 8);
    return (size_t)h;
  }
};
int fgv_finalize_impl(size_t nblocks, const size_t *ntx, const fgv_tx_result *res, uint8_t *flags) {
  std::unordered_set<std::array<uint8_t, 32>, Key32Hash> index;
  size_t o = 0;
  for (size_t b = 0; b < nblocks; b++) {
    const size_t n = ntx[b];
    std::array<uint8_t, 32> k;
    for (size_t i = 0; i < n; i++) {
      const fgv_tx_result &r = res[o + i];
      uint8_t code = r.code;
      if (r.flags & FGV_TXR_REACHED) {
        memcpy(k.data(), r.txid, 32);
        if (index.count(k)) code = C_DUP_TXID;  // checkTxIdDupsLedger precedes Dispatch
      }
      flags[o + i] = code;
    }
    std::unordered_set<std::array<uint8_t, 32>, Key32Hash> seen;
    for (size_t i = 0; i < n; i++) {
      if (flags[o + i] != C_VALID) continue;
      memcpy(k.data(), res[o + i].txid, 32);
      if (!seen.insert(k).second) flags[o + i] = C_DUP_TXID;
    }
    for (size_t i = 0; i < n; i++) {
      if (!(res[o + i].flags & FGV_TXR_INDEXED)) continue;
      memcpy(k.data(), res[o + i].index_txid, 32);
      index.insert(k);
    }
    o += n;
  }
  return FGV_OK;
}

// ---- configuration entry points (called from fgv_host.cpp wrappers)
int fgv_block_set_channel(fgv_block_state *S, const char *name) {
  S->dev_dirty = true;
  S->ch.name = name ? name : "";
  return FGV_OK;
}

// key_slot: the P-256 key table slot (or -1); info: key type, hash family, Validate() result,
// role bits and the identity digest (include/fgv.h fgv_identity_info).  Registering the same
// (mspid, id_bytes) again replaces its record.
int fgv_block_add_identity(fgv_block_state *S, const uint8_t *ser, size_t len, int32_t key_slot,
                           const fgv_identity_info *info) {
  VSerializedIdentity sid;
  if (!pbw::decode(ser, len, sid)) return FGV_EINVAL;
  if (info->key_type < FGV_KEY_P256 || info->key_type > FGV_KEY_UNDESERIALIZABLE || info->hash_family > FGV_HASH_SHA3)
    return FGV_EINVAL;
  S->dev_dirty = true;
  Channel &ch = S->ch;
  ch.dirty = true;
  Ident I;
  I.mspid = sid.mspid.str();
  I.id_bytes = sid.id_bytes.str();
  I.kind = (uint8_t)info->key_type;
  I.key_slot = (info->key_type == FGV_KEY_P256 || info->key_type == FGV_KEY_P384) ? key_slot : -1;
  I.hash3 = info->hash_family == FGV_HASH_SHA3;
  I.valid = info->valid != 0;
  I.roles_known = (info->roles & FGV_ROLES_UNKNOWN) == 0;
  I.roles = I.roles_known ? info->roles : 0;
  memcpy(I.digest, info->id_digest, 32);
  if (I.kind == FGV_KEY_P256) memcpy(I.pub, info->pubkey, 64);
  if (I.kind == FGV_KEY_P384) memcpy(I.pub384, info->pubkey_p384, 96);
  std::string canon = I.mspid + std::string(reinterpret_cast<const char *>(info->id_digest), 32);
  auto it = ch.canon_ids.find(canon);
  if (it == ch.canon_ids.end()) it = ch.canon_ids.emplace(canon, (uint32_t)ch.canon_ids.size()).first;
  I.canon = it->second;
  I.msp = ch.intern(I.mspid);
  uint64_t h = hash_bytes(sid.mspid.p, sid.mspid.n);
  h = hash_bytes(sid.id_bytes.p, sid.id_bytes.n, h ^ 0xA5);
  auto range = ch.ident_index.equal_range(h);
  for (auto r = range.first; r != range.second; ++r) {
    Ident &old = ch.idents[r->second];
    if (old.mspid == I.mspid && old.id_bytes == I.id_bytes) {
      old = I;
      return FGV_OK;
    }
  }
  ch.idents.push_back(I);
  ch.ident_index.emplace(h, (uint32_t)ch.idents.size() - 1);
  return FGV_OK;
}

int fgv_block_identity_ous(fgv_block_state *S, const uint8_t *ser, size_t len, size_t n, const char *const *ou,
                           const size_t *ou_lens, const uint8_t *const *certifiers, const size_t *cert_lens) {
  Channel &ch = S->ch;
  VSerializedIdentity sid;
  if (!pbw::decode(ser, len, sid)) return FGV_EINVAL;
  uint64_t h = hash_bytes(sid.mspid.p, sid.mspid.n);
  h = hash_bytes(sid.id_bytes.p, sid.id_bytes.n, h ^ 0xA5);
  auto range = ch.ident_index.equal_range(h);
  for (auto r = range.first; r != range.second; ++r) {
    Ident &I = ch.idents[r->second];
    if (!sid.mspid.eq(I.mspid.data(), I.mspid.size()) || !sid.id_bytes.eq(I.id_bytes.data(), I.id_bytes.size()))
      continue;
    I.ous.clear();
    for (size_t k = 0; k < n; k++)
      I.ous.push_back(ch.ou_intern(std::string_view(reinterpret_cast<const char *>(certifiers[k]), cert_lens[k]),
                                   std::string_view(ou[k], ou_lens[k])));
    I.ous_known = true;
    S->dev_dirty = true;
    ch.dirty = true;
    return FGV_OK;
  }
  return FGV_ESTATE;
}

int fgv_block_define_chaincode(fgv_block_state *S, const char *ns, const char *plugin, const uint8_t *policy,
                               size_t len, uint32_t flags) {
  S->dev_dirty = true;
  S->ch.dirty = true;
  CCDef &d = S->ch.ccdefs[ns];
  d.plugin = plugin;
  d.policy.assign(reinterpret_cast<const char *>(policy), len);
  d.flags = flags;
  d.colls.clear();
  return FGV_OK;
}

int fgv_block_define_collection(fgv_block_state *S, const char *ns, const char *coll, const uint8_t *policy,
                                size_t len) {
  auto it = S->ch.ccdefs.find(ns);
  if (it == S->ch.ccdefs.end()) return FGV_ESTATE;
  S->dev_dirty = true;
  S->ch.dirty = true;
  it->second.flags |= FGV_CC_COLLECTIONS_KNOWN;
  it->second.colls[coll].assign(reinterpret_cast<const char *>(policy), len);
  return FGV_OK;
}

int fgv_block_kvmeta_set(fgv_block_state *S, const std::string &ns, const std::string &coll, const uint8_t *key,
                         size_t key_len, const uint8_t *vp, size_t vp_len) {
  Channel &ch = S->ch;
  const std::string k = Channel::kvkey(ns, coll, std::string(reinterpret_cast<const char *>(key), key_len));
  auto it = ch.kvmeta.find(k);
  if (vp_len == 0) {
    if (it == ch.kvmeta.end()) return FGV_OK;
    ch.kvmeta.erase(it);
    if (--ch.kvmeta_ns[ns] == 0) ch.kvmeta_ns.erase(ns);
  } else if (it == ch.kvmeta.end()) {
    ch.kvmeta.emplace(k, std::string(reinterpret_cast<const char *>(vp), vp_len));
    ch.kvmeta_ns[ns]++;
  } else {
    it->second.assign(reinterpret_cast<const char *>(vp), vp_len);
  }
  S->dev_dirty = true;
  S->ch.dirty = true;
  return FGV_OK;
}

size_t fgv_block_kvmeta_count(fgv_block_state *S) { return S->ch.kvmeta.size(); }

const std::string *fgv_block_kvmeta_get(fgv_block_state *S, const std::string &ns, const std::string &coll,
                                        const uint8_t *key, size_t key_len) {
  auto it = S->ch.kvmeta.find(Channel::kvkey(ns, coll, std::string_view(reinterpret_cast<const char *>(key), key_len)));
  return it == S->ch.kvmeta.end() ? nullptr : &it->second;
}

int fgv_block_channel_config(fgv_block_state *S, const uint8_t *config, size_t len) {
  RawConfig rc;
  if (!parse_channel_config(config, len, rc)) return FGV_EINVAL;
  S->dev_dirty = true;
  S->ch.dirty = true;
  S->ch.config = std::move(rc);
  return FGV_OK;
}

int fgv_block_declare_msp(fgv_block_state *S, const char *mspid) {
  S->dev_dirty = true;
  S->ch.dirty = true;
  S->ch.declared_msps.insert(mspid);
  return FGV_OK;
}

int fgv_block_add_txids(fgv_block_state *S, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                        size_t n) {
  S->txid_dirty = true;
  for (size_t i = 0; i < n; i++) {
    std::string_view v(reinterpret_cast<const char *>(buf + off[i]), len[i]);
    if (S->ch.committed.count(v)) continue;
    S->ch.committed_store.emplace_back(v);
    S->ch.committed.insert(std::string_view(S->ch.committed_store.back()));
  }
  return FGV_OK;
}


// ======================================================================= device-resident path
int fgv_block_set_parse_mode(fgv_block_state *S, int mode) {
  if (mode != 0 && mode != 1) return FGV_EINVAL;
  S->parse_mode = mode;
  return FGV_OK;
}
int fgv_block_parse_mode(fgv_block_state *S) { return S->parse_mode; }

template <class T>
static int upload(DevBuf &b, const std::vector<T> &v) {
  const size_t n = v.size() * sizeof(T);
  if (!b.ensure(n ? n : 16)) return FGV_ENOMEM;
  if (n) HIP_TRY(hipMemcpy(b.p, v.data(), n, hipMemcpyHostToDevice));
  return FGV_OK;
}

static int build_committed(fgv_block_state *S);
// Flatten the channel model into the HBM image the kernels read (blockdev.h).
static int build_dev_image(fgv_block_state *S) {
  const Channel &ch = S->ch;
  DevImage &D = S->dimg;
  int rc;
  std::vector<uint8_t> name(ch.name.begin(), ch.name.end());
  if ((rc = upload(D.name, name))) return rc;
  // identities
  std::vector<DevIdent> idents(ch.idents.size());
  std::vector<int32_t> iou;
  std::vector<uint8_t> ib;
  std::vector<uint64_t> ih(ch.idents.size());
  D.has_sha3 = false;
  for (size_t i = 0; i < ch.idents.size(); i++) {
    const Ident &I = ch.idents[i];
    DevIdent &d = idents[i];
    // both fields start 4-byte aligned (k_bd_ident compares them a word at a time)
    d.msp_off = (uint32_t)ib.size();
    d.msp_len = (uint32_t)I.mspid.size();
    ib.insert(ib.end(), I.mspid.begin(), I.mspid.end());
    ib.resize((ib.size() + 3) & ~(size_t)3, 0);
    d.idb_off = (uint32_t)ib.size();
    d.idb_len = (uint32_t)I.id_bytes.size();
    ib.insert(ib.end(), I.id_bytes.begin(), I.id_bytes.end());
    ib.resize((ib.size() + 3) & ~(size_t)3, 0);
    d.key_slot = I.key_slot;
    d.msp = I.msp;
    d.canon = I.canon;
    d.valid = I.valid ? 1u : 0u;
    d.vclass = I.kind == FGV_KEY_UNDESERIALIZABLE ? 3u : (uint32_t)I.verify_class_tx();
    d.hash3 = (I.hash3 && d.vclass == 0) ? 1u : 0u;
    D.has_sha3 |= d.hash3 != 0;
    d.roles = I.roles;
    d.roles_known = I.roles_known ? 1u : 0u;
    d.ous_known = I.ous_known ? 1u : 0u;
    d.ou_off = (uint32_t)iou.size();
    d.ou_n = (uint32_t)I.ous.size();
    iou.insert(iou.end(), I.ous.begin(), I.ous.end());
    ih[i] = bd_ident_hash(reinterpret_cast<const uint8_t *>(I.mspid.data()), d.msp_len,
                          reinterpret_cast<const uint8_t *>(I.id_bytes.data()), d.idb_len);
  }
  ib.resize(ib.size() + 64, 0);  // word loads may read past the last field
  size_t icap = 16;
  while (icap < 2 * ch.idents.size()) icap <<= 1;
  std::vector<uint32_t> itable(icap, 0);
  for (size_t i = 0; i < ch.idents.size(); i++) {
    uint32_t pos = (uint32_t)ih[i] & (uint32_t)(icap - 1);
    while (itable[pos]) pos = (pos + 1) & (uint32_t)(icap - 1);
    itable[pos] = (uint32_t)i + 1;
  }
  if ((rc = upload(D.idents, idents)) || (rc = upload(D.ibytes, ib)) || (rc = upload(D.itable, itable)) ||
      (rc = upload(D.ihash, ih)) || (rc = upload(D.iou, iou)))
    return rc;
  // chaincodes (+ their collections), implicit collections, channel MSPs -> word tables over
  // one byte arena; policies -> flat node / kid / sub arrays
  std::vector<uint32_t> cc, colls, impl, msps;
  std::vector<uint8_t> ccb;
  auto str = [&](const std::string &x, std::vector<uint32_t> &out) {
    out.push_back((uint32_t)ccb.size());
    out.push_back((uint32_t)x.size());
    ccb.insert(ccb.end(), x.begin(), x.end());
  };
  for (const auto &kv : ch.ccs) {
    const CCInfo &c = kv.second;
    str(kv.first, cc);
    cc.push_back((uint32_t)c.ep);
    cc.push_back(c.status);
    cc.push_back(c.colls_known ? 1u : 0u);
    cc.push_back((uint32_t)(colls.size() / BD_COLL_WORDS));
    cc.push_back((uint32_t)c.colls.size());
    cc.push_back(c.has_vp ? 1u : 0u);
    for (const auto &cl : c.colls) {
      str(cl.first, colls);
      colls.push_back((uint32_t)cl.second);
    }
  }
  for (const auto &kv : ch.implicit_ep) {
    str(kv.first, impl);
    impl.push_back((uint32_t)kv.second);
  }
  for (const auto &kv : ch.msp_ids)
    if (ch.known_msps.count(kv.second)) str(kv.first, msps);
  std::vector<DevPolicy> pol(ch.policies.size());
  std::vector<DevPNode> nodes;
  std::vector<DevPrin> prins;
  std::vector<uint32_t> kids, subs;
  for (size_t p = 0; p < ch.policies.size(); p++) {
    const Policy &P = ch.policies[p];
    const uint32_t nbase = (uint32_t)nodes.size(), pbase = (uint32_t)prins.size();
    for (const Prin &x : P.prins) prins.push_back(DevPrin{x.kind, x.msp, x.role, x.canon, x.ou, 0});
    DevPolicy &d = pol[p];
    d.kind = P.kind == PK_SIG ? DP_SIG : P.kind == PK_IMPLICIT ? DP_IMPLICIT : P.kind == PK_UNSUP ? DP_UNSUP : DP_REJECT;
    d.decode_ok = P.decode_ok;
    d.compile_ok = P.compile_ok;
    d.needs_roles = P.needs_roles;
    d.root = P.root >= 0 ? (int32_t)(nbase + P.root) : -1;
    d.threshold = P.threshold;
    d.sub0 = (uint32_t)subs.size();
    d.nsub = (uint32_t)P.subs.size();
    for (int x : P.subs) subs.push_back((uint32_t)x);
    for (const PNode &N : P.nodes) {
      DevPNode dn;
      dn.type = N.type;
      dn.n = N.n;
      dn.p0 = (N.type == 2) ? pbase + P.prin_off[N.principal] : 0;
      dn.np = (N.type == 2) ? P.prin_cnt[N.principal] : 0;
      dn.kid0 = (uint32_t)kids.size();
      dn.nkids = (uint32_t)N.kids.size();
      for (int k : N.kids) kids.push_back(nbase + (uint32_t)k);
      nodes.push_back(dn);
    }
  }
  ccb.resize(ccb.size() + 64, 0);
  if ((rc = upload(D.cc, cc)) || (rc = upload(D.colls, colls)) || (rc = upload(D.impl, impl)) ||
      (rc = upload(D.msps, msps)) || (rc = upload(D.ccb, ccb)) || (rc = upload(D.pol, pol)) ||
      (rc = upload(D.nodes, nodes)) || (rc = upload(D.kids, kids)) || (rc = upload(D.subs, subs)) ||
      (rc = upload(D.prins, prins)))
    return rc;
  // committed key-level validation parameters (Channel::kvmeta_pi): kvkey = u32 |ns| ns u32
  // |coll| coll key -> slot (blockdev.h DevChannel::kvp)
  std::vector<uint32_t> kvp;
  std::vector<uint8_t> kvpb;
  size_t kcap = 0;
  if (!ch.kvmeta_pi.empty()) {
    kcap = 16;
    while (kcap < 2 * ch.kvmeta_pi.size()) kcap <<= 1;
    kvp.assign(kcap * 8, 0);
    for (const auto &kv : ch.kvmeta_pi) {
      const std::string &k = kv.first;
      uint32_t nl, cl;
      memcpy(&nl, k.data(), 4);
      memcpy(&cl, k.data() + 4 + nl, 4);
      const uint8_t *ns = reinterpret_cast<const uint8_t *>(k.data()) + 4;
      const uint8_t *coll = ns + nl + 4;
      const uint8_t *key = coll + cl;
      const uint32_t kl = (uint32_t)(k.size() - 8 - nl - cl);
      const uint64_t h = bd_kl_hash(ns, nl, coll, cl, key, kl);
      uint32_t pos = (uint32_t)h & (uint32_t)(kcap - 1);
      while (kvp[8 * pos + 7]) pos = (pos + 1) & (uint32_t)(kcap - 1);
      uint32_t *e = &kvp[8 * pos];
      e[0] = (uint32_t)h;
      e[1] = (uint32_t)(h >> 32);
      e[2] = (uint32_t)kvpb.size();
      e[3] = nl;
      e[4] = cl;
      e[5] = kl;
      e[6] = (uint32_t)kv.second;
      e[7] = 1;
      kvpb.insert(kvpb.end(), ns, ns + nl);
      kvpb.insert(kvpb.end(), coll, coll + cl);
      kvpb.insert(kvpb.end(), key, key + kl);
    }
    kvpb.resize(kvpb.size() + 64, 0);
    if ((rc = upload(D.kvp, kvp)) || (rc = upload(D.kvpb, kvpb))) return rc;
  }
  int rc2 = build_committed(S);
  if (rc2) return rc2;
  DevChannel &d = D.ch;
  d.kvp = kcap ? D.kvp.as<uint32_t>() : nullptr;
  d.kvp_bytes = kcap ? D.kvpb.as<uint8_t>() : nullptr;
  d.kvp_mask = kcap ? (uint32_t)(kcap - 1) : 0u;
  d.force_host = ch.policies.size() > 32767 ? 1u : 0u;  // (DevTx::pol is int16)
  d.name = D.name.as<uint8_t>();
  d.name_len = (uint32_t)name.size();
  d.nident = (uint32_t)idents.size();
  d.idents = D.idents.as<DevIdent>();
  d.ident_bytes = D.ibytes.as<uint8_t>();
  d.ident_table = D.itable.as<uint32_t>();
  d.ident_hash = D.ihash.as<uint64_t>();
  d.ident_mask = (uint32_t)(icap - 1);
  d.ncc = (uint32_t)(cc.size() / BD_CC_WORDS);
  d.cc = D.cc.as<uint32_t>();
  d.colls = D.colls.as<uint32_t>();
  d.nimpl = (uint32_t)(impl.size() / BD_COLL_WORDS);
  d.impl = D.impl.as<uint32_t>();
  d.nmsp = (uint32_t)(msps.size() / 2);
  d.msps = D.msps.as<uint32_t>();
  d.cc_bytes = D.ccb.as<uint8_t>();
  d.policies = D.pol.as<DevPolicy>();
  d.nodes = D.nodes.as<DevPNode>();
  d.kids = D.kids.as<uint32_t>();
  d.subs = D.subs.as<uint32_t>();
  d.prins = D.prins.as<DevPrin>();
  d.ident_ous = D.iou.as<int32_t>();
  return FGV_OK;
}

// The committed ledger txids (checkTxIdDupsLedger) as an open-addressing table in HBM.  Read by
// k_bd_fold only, so a front half enqueued ahead never sees it change under it.
static int build_committed(fgv_block_state *S) {
  const Channel &ch = S->ch;
  DevImage &D = S->dimg;
  int rc;
  S->txid_dirty = false;
  // only 64-char lowercase hex can equal a txid that passed CheckTxID
  std::vector<std::array<uint8_t, 32>> keys;
  uint32_t zero = 0;
  for (const std::string_view &v : ch.committed) {
    std::array<uint8_t, 32> k;
    if (!hex32(Span{reinterpret_cast<const uint8_t *>(v.data()), (uint32_t)v.size()}, k.data())) continue;
    bool z = true;
    for (uint8_t x : k) z &= x == 0;
    if (z) zero = 1;
    else keys.push_back(k);
  }
  size_t ccap = 0;
  std::vector<uint8_t> ctab;
  if (!keys.empty()) {
    ccap = 16;
    while (ccap < 2 * keys.size()) ccap <<= 1;
    ctab.assign(ccap * 32, 0);
    for (const auto &k : keys) {
      uint32_t h;
      memcpy(&h, k.data(), 4);
      uint32_t pos = h & (uint32_t)(ccap - 1);
      while (true) {
        uint8_t *e = &ctab[(size_t)pos * 32];
        bool empty = true;
        for (int i = 0; i < 32; i++) empty &= e[i] == 0;
        if (empty) { memcpy(e, k.data(), 32); break; }
        if (memcmp(e, k.data(), 32) == 0) break;
        pos = (pos + 1) & (uint32_t)(ccap - 1);
      }
    }
  }
  if ((rc = upload(D.committed, ctab))) return rc;
  DevChannel &d = D.ch;
  d.committed = ccap ? D.committed.as<uint8_t>() : nullptr;
  d.committed_mask = ccap ? (uint32_t)(ccap - 1) : 0u;
  d.committed_zero = zero;
  return FGV_OK;
}

__global__ void k_bd_parse(uint32_t ntx, const uint32_t *envtab, const uint64_t *bases, DevChannel ch, DevTx *out,
                           uint32_t *flags, uint32_t *xhaz, KlDev kl, uint32_t touch);
void bd_parse_lds_launch(uint32_t tpw, hipStream_t st, uint32_t ntx, const uint32_t *envtab, const uint64_t *bases,
                         const DevChannel &ch, DevTx *out, uint32_t *flags, uint32_t *xhaz, const KlDev &kl,
                         int32_t *ident);
__global__ void k_bd_kl(uint32_t ntx, DevTx *txs, const uint64_t *bases, KlDev kl, uint32_t *flags);
__global__ void k_head_pull(const uint4 *src, uint4 *dst, uint32_t n16);
__global__ void k_bd_ident(uint32_t ntx, const DevTx *txs, const uint64_t *bases, DevChannel ch, int32_t *ident,
                           uint32_t prio);
__global__ void k_bd_count(uint32_t ntx, DevTx *txs, DevChannel ch, const int32_t *ident, DevJobIdx *jobs,
                           uint32_t *totals, uint32_t prio, const uint64_t *bases, BdVerifyCols vc);
__global__ void k_bd_sha(uint32_t ntx, const DevTx *txs, const uint64_t *bases, uint8_t *dig, unsigned long long *nblk);
__global__ void k_bd_sha3(uint32_t ntx, const DevTx *txs, const uint64_t *bases, DevChannel ch, const int32_t *ident,
                          uint8_t *dig);
__global__ void k_bd_sha2(uint32_t ntx, const DevTx *txs, const uint64_t *bases, uint8_t *dig, unsigned long long *nblk);
__global__ void k_bd_sha_p2(uint32_t ntx, const DevTx *txs, const uint64_t *bases, uint8_t *dig,
                            unsigned long long *nblk);
__global__ void k_bd_sha_p3(uint32_t ntx, const DevTx *txs, const uint64_t *bases, uint8_t *dig,
                            unsigned long long *nblk);
__global__ void k_bd_sha_payload(uint32_t ntx, const uint32_t *envtab, const uint64_t *bases, uint8_t *dig,
                                 unsigned long long *nblk, uint32_t prio);
__global__ void k_bd_emit(uint32_t ntx, const DevTx *txs, const uint64_t *bases, DevChannel ch, const int32_t *ident,
                          const DevJobIdx *jobs, const uint32_t *totals, uint64_t *sig_ptr, uint32_t *sig_len,
                          uint32_t *key_slot, uint32_t *dig_idx, uint32_t *nv_out);
__global__ void k_bd_fold(uint32_t ntx, const DevTx *txs, const uint64_t *bases, DevChannel ch, const int32_t *ident,
                          const DevJobIdx *jobs, const uint32_t *totals, const uint8_t *digests,
                          const uint8_t *vstatus, fgv_tx_result *res, uint32_t *flags, const uint32_t *xhaz,
                          FinDev fin, KlDev kl, uint32_t touch);

// The batch head, one H2D copy: envelope table | block base addresses | 64 zero bytes (the
// kernels' counters) | per-block dependency-extraction hazards (blockdev.h) | per-block
// key-level words (KlDev::blk), each part 64-byte aligned.
static size_t head_env_bytes(size_t total) { return (total * 4 * BD_ENV_WORDS + 63) & ~(size_t)63; }
static size_t head_blk_bytes(size_t nblocks) { return (nblocks * 8 + 63) & ~(size_t)63; }
static size_t head_bytes(size_t total, size_t nblocks) {
  return head_env_bytes(total) + 2 * head_blk_bytes(nblocks) + 64 + ((nblocks * 4 * KL_BLK_WORDS + 63) & ~(size_t)63);
}

// host: split each block into envelope spans (tag / length walk of the block data framing)
// and write the envelope table into `et`
static int split_batch(ThreadPool &pool, size_t nblocks, const uint8_t *const *h_blocks, const size_t *lens,
                       const uint32_t *tx_lo, const uint32_t *tx_hi, SplitOut &o, HostBuf &et) {
  std::vector<std::vector<Span>> envs(nblocks);
  std::atomic<bool> bad{false};
  pool.run(nblocks, [&](size_t b) {
    if (tx_lo && tx_lo[b] == FGV_SHARD_SKIP) return;  // another rank's block: not parsed
    VBlock blk;
    if (!pbw::decode(h_blocks[b], lens[b], blk)) { bad = true; return; }
    envs[b] = std::move(blk.data.data);
  });
  if (bad) return FGV_EINVAL;
  o.lo.assign(nblocks, 0);
  o.hi.assign(nblocks, 0);
  o.ntx.assign(nblocks, 0);
  o.first.assign(nblocks, 0);
  o.total = 0;
  for (size_t b = 0; b < nblocks; b++) {
    o.ntx[b] = envs[b].size();  // 0 for a skipped block
    o.lo[b] = tx_lo ? std::min<uint32_t>(tx_lo[b], (uint32_t)envs[b].size()) : 0;
    o.hi[b] = tx_hi ? std::min<uint32_t>(tx_hi[b], (uint32_t)envs[b].size()) : (uint32_t)envs[b].size();
    if (o.hi[b] < o.lo[b]) o.hi[b] = o.lo[b];
    o.first[b] = o.total;
    o.total += o.hi[b] - o.lo[b];
    if (lens[b] > 0xFFFFFFFFull) return FGV_EINVAL;
  }
  if (o.total >= 0x7FFFFFFFull) return FGV_EINVAL;
  if (!et.ensure(head_bytes(o.total, nblocks) + 64)) return FGV_ENOMEM;
  uint32_t *e = et.as<uint32_t>();
  for (size_t b = 0; b < nblocks; b++) {  // writes only (the spans are already known)
    uint32_t *w = e + BD_ENV_WORDS * o.first[b];
    for (uint32_t i = o.lo[b]; i < o.hi[b]; i++, w += BD_ENV_WORDS) {
      w[0] = (uint32_t)b;
      w[1] = (uint32_t)(envs[b][i].p - h_blocks[b]);
      w[2] = envs[b][i].n;
    }
  }
  return FGV_OK;
}

// the pending pre-split of exactly this batch, or null
static PreSplit *pre_find(fgv_block_state *S, size_t nb, const uint8_t *const *b, const size_t *l, const uint32_t *lo,
                          const uint32_t *hi) {
  for (PreSplit &P : S->pre)
    if (P.active && P.matches(nb, b, l, lo, hi)) return &P;
  return nullptr;
}

// discard the pending pre-splits requested before P (every one: P null)
static void pre_discard_older(fgv_block_state *S, const PreSplit *P) {
  const uint64_t ord = P ? S->pre_ord[P - S->pre] : UINT64_MAX;
  for (int i = 0; i < 2; i++)
    if (&S->pre[i] != P && S->pre[i].active && S->pre_ord[i] < ord) S->pre[i].join();
}

int fgv_block_presplit(fgv_block_state *S, int device, size_t nblocks, const uint8_t *const *h_blocks,
                       const size_t *lens, const uint32_t *tx_lo, const uint32_t *tx_hi) {
  // the same batch requested again (the caller's own fgv_presplit earlier, then the call that
  // announces it as its next): the walk already running or done stands
  if (pre_find(S, nblocks, h_blocks, lens, tx_lo, tx_hi)) return FGV_OK;
  // a free slot, else the older request (discarded: nobody used it)
  int i = !S->pre[0].active ? 0 : !S->pre[1].active ? 1 : (S->pre_ord[0] < S->pre_ord[1] ? 0 : 1);
  PreSplit &P = S->pre[i];
  P.join();
  S->pre_ord[i] = S->pre_next++;
  P.device = device;
  P.blocks.assign(h_blocks, h_blocks + nblocks);
  P.lens.assign(lens, lens + nblocks);
  P.lo_in.clear();
  P.hi_in.clear();
  if (tx_lo) P.lo_in.assign(tx_lo, tx_lo + nblocks);
  if (tx_hi) P.hi_in.assign(tx_hi, tx_hi + nblocks);
  P.start();
  return FGV_OK;
}

// MVCC (fgv_mvcc_validate_block): the envelope spans of `block` from a pre-split of exactly
// this one block, if one was requested; a pre-split of another batch is left pending.
bool fgv_block_take_presplit(fgv_block_state *S, const uint8_t *block, size_t len, std::vector<Span> &out) {
  PreSplit *Q = pre_find(S, 1, &block, &len, nullptr, nullptr);
  if (!Q) return false;
  pre_discard_older(S, Q);
  PreSplit &P = *Q;
  P.join();
  if (P.rc != FGV_OK || P.out.ntx.size() != 1) return false;
  const uint32_t *e = P.et.as<uint32_t>();
  out.resize(P.out.total);
  for (size_t i = 0; i < P.out.total; i++, e += BD_ENV_WORDS) out[i] = Span{block + e[1], e[2]};
  return true;
}

// The pre-split of exactly these whole blocks (fgv_mvcc_validate_blocks_next walked them while
// the previous call ran): per block its envelope count, its first row in `et` (BD_ENV_WORDS per
// envelope: block, offset, length).  Valid until the next pre-split.
bool fgv_block_take_presplit_batch(fgv_block_state *S, size_t nb, const uint8_t *const *blocks, const size_t *lens,
                                   const uint32_t **et, const size_t **ntx, const size_t **first) {
  PreSplit *Q = pre_find(S, nb, blocks, lens, nullptr, nullptr);
  if (!Q) return false;
  pre_discard_older(S, Q);
  PreSplit &P = *Q;
  const auto t0 = std::chrono::steady_clock::now();
  P.join();
  if (presplit_log())
    fprintf(stderr, "[fgv] waited %.3f ms for the pre-split of %zu blocks\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), nb);
  if (P.rc != FGV_OK || P.out.ntx.size() != nb) return false;
  *et = P.et.as<uint32_t>();
  *ntx = P.out.ntx.data();
  *first = P.out.first.data();
  return true;
}

// The dependency-extraction hazards of transactions [0, lo) of a block (a shard starting inside
// it): extraction failures, panics, metadata writes.
static void prefix_hazards(const uint8_t *blk, size_t len, uint32_t lo, uint8_t &fail, uint8_t &panic, bool &md) {
  fail = panic = 0;
  md = false;
  VBlock B;
  if (!pbw::decode(blk, len, B)) return;
  for (uint32_t i = 0; i < lo && i < B.data.data.size(); i++) {
    TxRec tmp;
    extract_walk(B.data.data[i], tmp);
    fail |= tmp.xstat == X_FAIL;
    panic |= tmp.xstat == X_PANIC;
    md |= tmp.has_md;
  }
}

// k_bd_emit -> k_der -> k_inv of the batch in set B on stream `st` (its counts are done there):
// the verify stages that need no digest, into the set's own buffers
static int emit_prefix(fgv_ctx *c, fgv_block_state *S, BdSet &B, hipStream_t st) {
  const uint32_t N = B.N;
  const size_t cap = (size_t)N * (1 + BD_MAX_END);
  if (!B.vsig.ensure(cap * 20 + 64) || !B.vst.ensure(cap + 64)) return FGV_ENOMEM;
  uint32_t *misc = reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff);
  const uint64_t *dbs = reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff);
  uint8_t *sp = B.vsig.as<uint8_t>();
  const bool tim = c->timing && B.timed;
  // the verify count the stages read: k_bd_count's creator-kind total when it emitted the jobs
  // (endorsements inside the same range), else k_bd_emit's sum
  const uint32_t *dn = misc + BJ_C;
  if (!B.emitted) {
    if (tim) HIP_TRY(hipEventRecord(c->kev[6], st));
    hipLaunchKernelGGL(k_bd_emit, dim3((N + 255) / 256), dim3(256), 0, st, N, B.tx.as<DevTx>(), dbs, S->dimg.ch,
                       B.ident.as<int32_t>(), B.jobs.as<DevJobIdx>(), misc, reinterpret_cast<uint64_t *>(sp),
                       reinterpret_cast<uint32_t *>(sp + cap * 8), reinterpret_cast<uint32_t *>(sp + cap * 12),
                       reinterpret_cast<uint32_t *>(sp + cap * 16), misc + 10);
    HIP_TRY(hipGetLastError());
    if (tim) HIP_TRY(hipEventRecord(c->kev[7], st));
    dn = misc + 10;
  } else if (tim) {  // (no k_bd_emit: an empty interval, so fgv_last_kernel_times reads recorded events)
    HIP_TRY(hipEventRecord(c->kev[6], st));
    HIP_TRY(hipEventRecord(c->kev[7], st));
  }
  int rc = fgv_verify_prefix_dev(c, st, cap, dn, sp, B.vst.as<uint8_t>(), B.vr, B.vs, B.vw, B.vscr);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(B.ev[9], st));
  B.vdone = true;
  return FGV_OK;
}

// The front-half chain (parse, identities, counts) at wave priority 3, the verify chain's
// (FGV_FRONT_PRIO=2: one below it).  With the front half queued behind the back half (round 4) 3
// measured 0.572-0.575 ms per C2 step against 0.559-0.561 at 2 (r4o), 0.560-0.564 against
// 0.557-0.562 in round 5 (r5fp); with its parse queued at the call's top (front_early, round 5)
// 0.516-0.521 against 0.522-0.541, alternating on one box (r5f3, r5f4): 3 is the default
static uint32_t front_prio_knob() {
  static const uint32_t v = [] {
    const char *e = getenv("FGV_FRONT_PRIO");
    return e && atoi(e) == 2 ? 2u : 3u;
  }();
  return v;
}
// FGV_PARSE_LDS = transactions per workgroup of the LDS-staged walk (see front_launch_a)
static uint32_t parse_lds_knob() {
  static const uint32_t v = [] {
    const char *e = getenv("FGV_PARSE_LDS");
    const uint32_t x = e ? (uint32_t)atoi(e) : 0u;
    return (x == 4u || x == 8u || x == 16u) ? x : 0u;
  }();
  return v;
}
// FGV_PARSE_IDENT=0: k_bd_ident as its own kernel after the LDS-staged parse (A/B); by default
// the parse workgroups resolve their transactions' identities themselves
static bool parse_ident_knob() {
  static const bool v = [] {
    const char *e = getenv("FGV_PARSE_IDENT");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// Front half of a batch into set B, on the side streams: envelope spans (pre-split or walked
// here), head upload, k_bd_sha_payload (stream2), k_bd_parse -> k_bd_ident -> k_bd_count ->
// job counters in device memory (streamF), k_bd_sha (stream3).  `wait` (optional): an event the head
// upload waits for (the H2D copy of host-resident blocks).  Nothing here reads the committed
// txid table (k_bd_fold does), so ledger txids added afterwards never stale it.
// `sf` carries the parse -> identities -> counts chain: the main stream for the call's own batch
// (its back half then follows in order, with no cross-stream hop), c->streamF for a front half
// enqueued ahead beside the current batch's back half.
// k_bd_ident -> k_bd_count of the batch in set B on its parse stream (front_launch_a, or _b with
// FGV_FRONT_COUNTS_B=1)
static int front_counts(fgv_block_state *S, BdSet &B) {
  const uint32_t N = B.N;
  const DevChannel ch = S->dimg.ch;
  hipStream_t sf = B.stream;
  const bool tim = B.timed;
  uint32_t *misc = reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff);
  const uint64_t *dbs = reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff);
  DevTx *dtx = B.tx.as<DevTx>();
  const uint32_t front_prio = B.prio;
  const bool fused_ident = parse_lds_knob() && parse_ident_knob();
  if (tim) HIP_TRY(hipEventRecord(B.ev[7], sf));
  if (!fused_ident)
    hipLaunchKernelGGL(k_bd_ident, dim3((uint32_t)(((uint64_t)N * 16 * BD_ID_PAR + 255) / 256)), dim3(256), 0, sf, N,
                       dtx, dbs, ch, B.ident.as<int32_t>(), front_prio);
  // FGV_FUSE_EMIT=0: k_bd_emit as its own kernel at the head of the back half (A/B); by default
  // k_bd_count writes the verify jobs itself
  static const bool fuse_emit = [] {
    const char *e = getenv("FGV_FUSE_EMIT");
    return !e || atoi(e) != 0;
  }();
  BdVerifyCols vc{nullptr, nullptr, nullptr, nullptr};
  B.emitted = false;
  if (fuse_emit) {
    const size_t cap = (size_t)N * (1 + BD_MAX_END);
    if (!B.vsig.ensure(cap * 20 + 64) || !B.vst.ensure(cap + 64)) return FGV_ENOMEM;
    uint8_t *sp = B.vsig.as<uint8_t>();
    vc = BdVerifyCols{reinterpret_cast<uint64_t *>(sp), reinterpret_cast<uint32_t *>(sp + cap * 8),
                      reinterpret_cast<uint32_t *>(sp + cap * 12), reinterpret_cast<uint32_t *>(sp + cap * 16)};
    B.emitted = true;
  }
  hipLaunchKernelGGL(k_bd_count, dim3((N + 1023) / 1024), dim3(1024), 0, sf, N, dtx, ch, B.ident.as<int32_t>(),
                     B.jobs.as<DevJobIdx>(), misc, front_prio, dbs, vc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(B.ev[6], sf));
  return FGV_OK;
}

// FGV_FRONT_COUNTS_B=1: identities and counts queued with phase b (behind the call's back half)
// instead of right after the parse (A/B)
static bool counts_in_b() {
  static const bool v = [] {
    const char *e = getenv("FGV_FRONT_COUNTS_B");
    return e && atoi(e) != 0;
  }();
  return v;
}

// Two phases (front_launch = both): front_launch_a -- the host part, head upload, k_bd_parse and
// the payload hashes; front_launch_b -- k_bd_sha (stream3), identities and counts.  A call may
// queue phase a of the next batch at its top and phase b behind its own back half (front_early).
static int front_launch_a(fgv_ctx *c, fgv_block_state *S, BdSet &B, size_t nblocks, const uint8_t *const *h_blocks,
                          const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                          const uint32_t *tx_hi, hipStream_t sf, hipEvent_t wait, hipEvent_t wait2) {
  // FGV_FRONT_LOG=1: host time of each phase of the enqueue, one stderr line per call (profiling aid)
  static const bool flog = getenv("FGV_FRONT_LOG") && atoi(getenv("FGV_FRONT_LOG"));
  using fclk = std::chrono::steady_clock;
  const auto ft0 = fclk::now();
  double fts[6] = {};
  auto fmark = [&](int i) {
    if (flog) fts[i] = std::chrono::duration<double, std::micro>(fclk::now() - ft0).count();
  };
  B.vdone = false;
  B.hb.assign(h_blocks, h_blocks + nblocks);
  B.db.assign(d_blocks, d_blocks + nblocks);
  B.lens.assign(lens, lens + nblocks);
  B.has_lo = tx_lo != nullptr;
  B.has_hi = tx_hi != nullptr;
  B.lo.clear();
  B.hi.clear();
  if (tx_lo) B.lo.assign(tx_lo, tx_lo + nblocks);
  if (tx_hi) B.hi.assign(tx_hi, tx_hi + nblocks);
  B.N = 0;
  B.presplit = false;
  for (auto &e : B.ev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  // --- host: the batch's envelope spans, split ahead by fgv_presplit or here
  {
    PreSplit *P = pre_find(S, nblocks, h_blocks, lens, tx_lo, tx_hi);
    pre_discard_older(S, P);  // (requests before this batch's: nobody will use them)
    if (P) {
      P->join();  // (its worker is idle from here on)
      if (P->rc == FGV_OK) {
        B.so = std::move(P->out);
        std::swap(B.head, P->et);  // (B's old head: no copy from it is pending)
        B.presplit = true;
      }
    }
  }
  if (!B.presplit) {
    int rc = split_batch(S->pool, nblocks, h_blocks, lens, tx_lo, tx_hi, B.so, B.head);
    if (rc) return rc;
  }
  fmark(0);
  const size_t total = B.so.total;
  if (total == 0) return FGV_OK;
  const uint32_t N = (uint32_t)total;
  const size_t hbytes = head_bytes(total, nblocks);
  B.eoff = head_env_bytes(total);
  B.moff = B.eoff + ((nblocks * 8 + 63) & ~(size_t)63);
  // (B.head already holds hbytes: split_batch sized it)
  if (!B.misc.ensure(64) || !B.env.ensure(hbytes) || !B.tx.ensure(total * sizeof(DevTx)) ||
      !B.ident.ensure(total * BD_OCC * 4) || !B.jobs.ensure(total * sizeof(DevJobIdx)) ||
      !B.dig.ensure((size_t)N * 32 * BD_DIG_SLOTS + 64))  // k_bd_sha digest slots (blockdev.h), slot-major
    return FGV_ENOMEM;
  uint8_t *head = B.head.as<uint8_t>();  // the envelope table is already in place
  uint64_t *bs = reinterpret_cast<uint64_t *>(head + B.eoff);
  for (size_t b = 0; b < nblocks; b++) bs[b] = (uint64_t)(uintptr_t)d_blocks[b];
  memset(head + B.moff, 0, 64);
  // dependency-extraction hazards: none yet; a shard starting inside a block walks the block's
  // earlier transactions (their metadata writes would need their vscc results: host parser)
  uint32_t *xh = reinterpret_cast<uint32_t *>(head + B.moff + 64);
  B.force_host = false;
  for (size_t b = 0; b < nblocks; b++) {
    xh[2 * b] = xh[2 * b + 1] = UINT32_MAX;
    if (!tx_lo || tx_lo[b] == 0 || tx_lo[b] == FGV_SHARD_SKIP) continue;
    uint8_t fail, panic;
    bool md;
    prefix_hazards(h_blocks[b], lens[b], tx_lo[b], fail, panic, md);
    if (fail) xh[2 * b] = 0;
    if (panic) xh[2 * b + 1] = 0;
    B.force_host |= md;
  }
  // key-level state of the batch (blockdev.h KlDev): per-block words, records chained in buckets
  // tagged with this batch's sequence number (no reset between batches)
  const size_t klb_off = B.moff + 64 + head_blk_bytes(nblocks);
  uint32_t *klw = reinterpret_cast<uint32_t *>(head + klb_off);
  for (size_t b = 0; b < nblocks; b++) {
    klw[KL_BLK_WORDS * b] = (uint32_t)B.so.first[b];
    klw[KL_BLK_WORDS * b + 1] = (uint32_t)(B.so.hi[b] - B.so.lo[b]);
    klw[KL_BLK_WORDS * b + 2] = klw[KL_BLK_WORDS * b + 3] = 0;
  }
  const size_t rcap = 2 * total + 1024;
  size_t hcap = 1024;
  while (hcap < 2 * rcap) hcap <<= 1;
  const size_t hbuf = B.klhead.cap;
  if (!B.klrec.ensure(rcap * sizeof(KlRec)) || !B.klhead.ensure(hcap * 8) ||
      !B.kldep.ensure(total * KL_DEPS * 4) || !B.kllist.ensure(nblocks * KL_MAXDEP * 4))
    return FGV_ENOMEM;
  if (B.klhead.cap != hbuf) HIP_TRY(hipMemsetAsync(B.klhead.p, 0, B.klhead.cap, sf));  // (new memory: no stale tag)
  if (++S->klseq == 0) ++S->klseq;
  B.klseq = S->klseq;
  fmark(1);
  const DevChannel ch = S->dimg.ch;
  B.stream = sf;
  if (wait) HIP_TRY(hipStreamWaitEvent(sf, wait, 0));
  if (wait2) HIP_TRY(hipStreamWaitEvent(sf, wait2, 0));
  // events: ev3 (head uploaded), ev4 (parsed), ev1 (payload digests), ev2 (other digests), ev6
  // (job counts) order the streams; ev0 / ev5 / ev7 only time kernels (fgv_set_timing)
  const bool tim = c->timing;
  B.timed = tim;
  if (tim) HIP_TRY(hipEventRecord(B.ev[0], sf));
  // FGV_HEAD_PULL=1: the GPU reads the head from the pinned host copy (k_head_pull) instead of a
  // copy-engine transfer (A/B)
  static const bool head_pull = [] {
    const char *e = getenv("FGV_HEAD_PULL");
    return e && atoi(e) != 0;
  }();
  const uint4 *hsrc = nullptr;
  if (head_pull && (hbytes & 15) == 0 &&
      hipHostGetDevicePointer(reinterpret_cast<void **>(const_cast<uint4 **>(&hsrc)), head, 0) != hipSuccess)
    hsrc = nullptr;
  if (hsrc) {
    const uint32_t n16 = (uint32_t)(hbytes / 16);
    hipLaunchKernelGGL(k_head_pull, dim3(std::min<uint32_t>((n16 + 255) / 256, 128)), dim3(256), 0, sf, hsrc,
                       B.env.as<uint4>(), n16);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemcpyAsync(B.env.p, head, hbytes, hipMemcpyHostToDevice, sf));
  }
  HIP_TRY(hipEventRecord(B.ev[3], sf));
  fmark(2);
  // [0..5) totals, [5] flags, bytes 24..32 k_bd_sha compressions, 32..40 payload compressions
  uint32_t *misc = reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff);
  const uint32_t *envtab = B.env.as<uint32_t>();
  const uint64_t *dbs = reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff);
  DevTx *dtx = B.tx.as<DevTx>();
  // the payload hashes (the longest serial chains) beside the parse, on the second stream.  Queued
  // after the parse (the front half's critical chain since round 4: its launch is ~15 us earlier);
  // FGV_PAYLOAD_FIRST=1 queues them before it (A/B)
  static const bool payload_first = [] {
    const char *e = getenv("FGV_PAYLOAD_FIRST");
    return e && atoi(e) != 0;
  }();
  auto launch_payload = [&]() -> hipError_t {
    hipError_t e = hipStreamWaitEvent(c->stream2, B.ev[3], 0);
    if (e != hipSuccess) return e;
    // FGV_PAYLOAD_PRIO=3: the payload hashes at the front chain's wave priority (A/B; default 2)
    static const uint32_t pay_prio = [] {
      const char *e = getenv("FGV_PAYLOAD_PRIO");
      return e && atoi(e) == 3 ? 3u : 2u;
    }();
    hipLaunchKernelGGL(k_bd_sha_payload, dim3((N + 63) / 64), dim3(128), 0, c->stream2, N, envtab, dbs,
                       B.dig.as<uint8_t>(), reinterpret_cast<unsigned long long *>(misc + 8), pay_prio);
    return hipEventRecord(B.ev[1], c->stream2);
  };
  if (payload_first) HIP_TRY(launch_payload());
  B.kl = KlDev{B.klrec.as<KlRec>(),
               B.klhead.as<unsigned long long>(),
               (uint32_t)(hcap - 1),
               (uint32_t)rcap,
               B.klseq,
               (!tx_lo && !tx_hi) ? 1u : 0u,
               misc + 11,
               reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + klb_off),
               B.kllist.as<uint32_t>(),
               B.kldep.as<uint32_t>()};
  B.prio = front_prio_knob();
  const uint32_t front_prio = B.prio;
  // every line of each envelope requested before the walk (touch_lines): measured on MI355X (C2,
  // lean harness, one box) 0.665-0.667 ms per step against 0.702-0.724 without
  // (profiles/round3_ab/parse_t*); FGV_PARSE_TOUCH=0 turns it off (A/B)
  static const uint32_t parse_touch = [] {
    const char *e = getenv("FGV_PARSE_TOUCH");
    return e ? (uint32_t)atoi(e) : 1u;
  }();
  // transactions (walking lanes) per workgroup (the LDS arrays stay sized for 64 lanes);
  // FGV_PARSE_LANES = 16 / 32 / 64 (A/B).  Measured on MI355X (C2 lean harness, two alternating
  // rounds, profiles/round3_ab/parse_lanes_*): 64 -> 0.690 / 0.722 ms per step, 32 -> 0.706 /
  // 0.720, 16 -> 0.794 / 0.811: fewer lanes per wave does not shorten the walk; 64 stays
  static const uint32_t parse_lanes = [] {
    const char *e = getenv("FGV_PARSE_LANES");
    const uint32_t v = e ? (uint32_t)atoi(e) : 64u;
    return (v == 16u || v == 32u) ? v : 64u;
  }();
  // FGV_PARSE_LDS = transactions per workgroup of the LDS-staged walk (k_bd_parse_lds: 4, 8 or 16,
  // each envelope copied to LDS before the walk); 0 (default) = the global walk above.  Measured on
  // MI355X (C2 lean harness, one box): 8 per workgroup 1.01 ms per step against 0.67-0.71 for the
  // global walk -- the walk is bound by instruction issue per wave (8 walking lanes of 64), not
  // by the latency of its loads (profiles/round4_ab)
  const uint32_t parse_lds = parse_lds_knob();
  const bool fused_ident = parse_lds && parse_ident_knob();
  if (parse_lds)
    bd_parse_lds_launch(parse_lds, sf, N, envtab, dbs, ch, dtx, misc + 5, misc + 16, B.kl,
                        fused_ident ? B.ident.as<int32_t>() : nullptr);
  else
    hipLaunchKernelGGL(k_bd_parse, dim3((N + parse_lanes - 1) / parse_lanes), dim3(parse_lanes), 0, sf, N, envtab,
                       dbs, ch, dtx, misc + 5, misc + 16, B.kl, parse_touch | (front_prio == 3 ? 0x100u : 0u));
  HIP_TRY(hipEventRecord(B.ev[4], sf));
  if (!payload_first) HIP_TRY(launch_payload());
  B.N = N;
  if (!counts_in_b()) {
    int rc = front_counts(S, B);
    if (rc) return rc;
  }
  fmark(3);
  if (flog)
    fprintf(stderr, "[fgv] front_launch_a us: split %.1f head %.1f upload %.1f parse+payload(+counts) %.1f (N %u, %s)\n",
            fts[0], fts[1] - fts[0], fts[2] - fts[1], fts[3] - fts[2], N, B.presplit ? "presplit" : "walked");
  return FGV_OK;
}

static int front_launch_b(fgv_ctx *c, fgv_block_state *S, BdSet &B, bool prefix) {
  if (B.N == 0) return FGV_OK;
  static const bool flog = getenv("FGV_FRONT_LOG") && atoi(getenv("FGV_FRONT_LOG"));
  const auto ft0 = std::chrono::steady_clock::now();
  const uint32_t N = B.N;
  const DevChannel ch = S->dimg.ch;
  hipStream_t sf = B.stream;
  const bool tim = B.timed;
  uint32_t *misc = reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff);
  const uint64_t *dbs = reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff);
  DevTx *dtx = B.tx.as<DevTx>();
  // every other SHA-256 message is known after the parse: hashed on the third stream while
  // identities and job counts are worked out on this one
  HIP_TRY(hipStreamWaitEvent(c->stream3, B.ev[4], 0));
  if (tim) HIP_TRY(hipEventRecord(B.ev[5], c->stream3));
  static const int sha_prio = [] {
    const char *e = getenv("FGV_SHA_PRIO");
    return e ? atoi(e) : 1;
  }();
  // FGV_SHA_SPLIT=1: the two-wave k_bd_sha2 (schedule wave + rounds wave per chain).  Measured
  // on MI355X with the next batch's front half ahead (profiles/round3_ab/split*): 0.678-0.688 ms
  // per C2 step vs 0.666-0.673 for the one-wave kernel -- beside the other batch's kernels the
  // extra waves and the 32 KB of LDS per workgroup cost more than the shorter chain gains -- so
  // the one-wave kernel is the default.
  static const bool sha_split = [] {
    const char *e = getenv("FGV_SHA_SPLIT");
    return e && atoi(e) != 0;
  }();
  if (sha_split)
    hipLaunchKernelGGL(k_bd_sha2, dim3((N + SHA_GPW - 1) / SHA_GPW), dim3(128), 0, c->stream3, N, dtx, dbs,
                       B.dig.as<uint8_t>(), reinterpret_cast<unsigned long long *>(misc + 6));
  else
    hipLaunchKernelGGL(sha_prio == 3 ? k_bd_sha_p3 : sha_prio == 2 ? k_bd_sha_p2 : k_bd_sha,
                       dim3((N + SHA_GPW - 1) / SHA_GPW), dim3(64), 0,
                       c->stream3, N, dtx, dbs, B.dig.as<uint8_t>(), reinterpret_cast<unsigned long long *>(misc + 6));
  HIP_TRY(hipEventRecord(B.ev[2], c->stream3));
  HIP_TRY(hipStreamWaitEvent(c->stream3, B.ev[1], 0));
  // a channel with SHA3 MSP identities: their digests are replaced once the identities are known
  // (after k_bd_count, below), and the digests join there instead
  const bool sha3 = S->dimg.has_sha3;
  if (!sha3) HIP_TRY(hipEventRecord(B.ev[8], c->stream3));
  if (counts_in_b()) {
    int rc = front_counts(S, B);
    if (rc) return rc;
  }
  if (sha3) {
    HIP_TRY(hipStreamWaitEvent(c->stream3, B.ev[6], 0));
    hipLaunchKernelGGL(k_bd_sha3, dim3((N + 63) / 64), dim3(64), 0, c->stream3, N, dtx, dbs, ch,
                       (const int32_t *)B.ident.as<int32_t>(), B.dig.as<uint8_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(B.ev[8], c->stream3));
  }
  if (flog)
    fprintf(stderr, "[fgv] front_launch_b us: %.1f\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - ft0).count());
  if (prefix) return emit_prefix(c, S, B, sf);
  return FGV_OK;
}

static int front_launch(fgv_ctx *c, fgv_block_state *S, BdSet &B, size_t nblocks, const uint8_t *const *h_blocks,
                        const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                        const uint32_t *tx_hi, hipStream_t sf, hipEvent_t wait, hipEvent_t wait2 = nullptr,
                        bool prefix = false) {
  int rc = front_launch_a(c, S, B, nblocks, h_blocks, lens, d_blocks, tx_lo, tx_hi, sf, wait, wait2);
  if (rc) return rc;
  return front_launch_b(c, S, B, prefix);
}

// Wait for a front half enqueued ahead and forget it (its batch was not the next call's, or
// the channel model is about to change under it).
static void drain_ahead(fgv_ctx *c, fgv_block_state *S) {
  if (S->early >= 0) S->ahead = S->early, S->early = -1;  // (a phase a without its phase b)
  S->prefix_next = -1;
  if (S->ahead < 0) return;
  hipStreamSynchronize(c->stream);  // (a verify prefix queued there by the last finish)
  hipStreamSynchronize(c->streamF);
  hipStreamSynchronize(c->stream2);
  hipStreamSynchronize(c->stream3);
  S->ahead = -1;
}

void fgv_block_drain(fgv_ctx *c) { drain_ahead(c, c->blk); }

// The next batch's front half, ahead of its call, while this back half runs: its device copy is
// known (caller-resident, or being prefetched by the copy stream).
static void launch_ahead(fgv_ctx *c, fgv_block_state *S, const fgv_ctx::NextBatch &nx, int cur, bool fused = false) {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  // Measured on MI355X (C2, 32 x 500-tx batches, fused single-GPU call; DESIGN.md s5,
  // profiles/round3_ab): enqueued at once (2, the default) 0.715-0.724 ms per step against 0.773-
  // 0.799 not ahead (0), in the full default bench and in the lean A/B harness alike; after this
  // batch's ECDSA (1) or after its fold (3) it collides with k_point28 or with the next call's own
  // kernels.  fgv_set_ahead / FGV_AHEAD select a placement (A/B).
  const int ahead_mode = c->ahead_mode;
  if (S->early >= 0 && !(nx.n && nx.d_blocks && ahead_mode)) {
    S->ahead = S->early, S->early = -1;
    drain_ahead(c, S);
  }
  if (nx.n && nx.d_blocks && ahead_mode) {
    BdSet &A = S->set[cur ^ 1];
    // (mode 2 with this batch's verifies on the variable-base kernels, or with the next batch's H2D
    // copy still in flight: after this batch's k_prep, as mode 4 -- C2 churn with the next batch
    // pre-split ahead, lean harness: 1.239 ms per step against 1.377 at once, 1.577 after the
    // ECDSA, 1.664 after the fold, r5pe2; C2 PCIe-inclusive: 1.123 ms against 1.251 at once, r5pcie5)
    static const bool copy_after = [] {  // FGV_COPY_AFTER=0: a copy-pending batch's front half at once (A/B)
      const char *e = getenv("FGV_COPY_AFTER");
      return !e || atoi(e) != 0;
    }();
    const bool vb_now = ahead_mode == 2 && (c->n_vb > 0 || (copy_after && nx.wait)) && c->stage_ran;
    hipEvent_t after = (ahead_mode == 1 && c->stage_ran)               ? c->ev[6]
                       : ((ahead_mode == 4 || vb_now) && c->stage_ran) ? c->ev[5]
                       : ahead_mode == 3                               ? c->kev[9]
                                                                       : nullptr;
    // FGV_PREFIX_AHEAD=1: the next batch's k_bd_emit / k_der / k_inv run ahead with its front
    // half.  Measured on MI355X (C2 lean harness, alternating on one box, profiles/round3_ab/
    // prefix_*): 0.748 / 0.753 ms per step ahead against 0.683 / 0.670 at the call -- beside the
    // current back half they stretch k_point28 more than they shorten the chain -- so off.
    static const bool prefix_ahead = [] {
      const char *e = getenv("FGV_PREFIX_AHEAD");
      return e && atoi(e) != 0;
    }();
    // (with keys on the variable-base kernels the prefix stays in the call: their list and
    // counters belong to one batch at a time)
    const auto tf = clk::now();
    // FGV_PREFIX_MAIN=1 (the fused single-GPU call, without fgv_set_timing): the next batch's
    // k_bd_emit / k_der / k_inv queued on the main stream behind this call's finalize
    // (fgv_block_validate_dev_finish), so they start as soon as its k_fin_dups ends instead of
    // after the host's turnaround to the next call; the finish waits on an event recorded before
    // them.  Measured on MI355X (C2 lean harness, one box, r5pm): 0.546-0.554 ms per step against
    // 0.516-0.522 without -- off (A/B)
    static const bool prefix_main = [] {
      const char *e = getenv("FGV_PREFIX_MAIN");
      return e && atoi(e) != 0;
    }();
    const bool vb_free = c->n_vb == 0 && !c->kt_busy;
    const bool pre = prefix_ahead && vb_free;
    S->prefix_next = -1;
    const bool pmain = !pre && prefix_main && fused && vb_free && !c->timing;
    const bool early = S->early == (cur ^ 1);
    S->early = -1;
    if ((early ? front_launch_b(c, S, A, pre)
               : front_launch(c, S, A, nx.n, nx.blocks, nx.lens, nx.d_blocks, nx.lo, nx.hi, c->streamF, nx.wait,
                              after, pre)) == FGV_OK)
      S->ahead = cur ^ 1, S->prefix_next = pmain ? cur ^ 1 : -1;
    else
      drain_ahead(c, S), S->ahead = -1;  // (the next call starts it again and reports any error)
    c->t_kern[11] = ms_since(tf) + (early ? S->early_ms : 0.0);  // host time to enqueue it (its pre-split join included)
  } else {
    c->t_kern[11] = 0;
  }
}

void fgv_block_launch_deferred_ahead(fgv_ctx *c, bool launch) {
  fgv_block_state *S = c->blk;
  if (!S || !S->ahead_deferred) return;
  S->ahead_deferred = false;
  if (launch) {
    launch_ahead(c, S, S->ahead_nx, S->ahead_cur, true);
  } else {
    if (S->early >= 0) drain_ahead(c, S);  // (phase a queued at the call's top: forgotten)
    c->t_kern[11] = 0;
  }
}

int fgv_block_validate_dev_enqueue(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                                   const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                                   const uint32_t *tx_hi, fgv_tx_result *d_res, size_t res_cap, size_t *ntx_out) {
  using clk = std::chrono::steady_clock;
  S->pending = -1;
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  auto t0 = clk::now();
  fgv_ctx::NextBatch nx = c->next;  // the batch whose front half this call enqueues ahead
  // FGV_PRESPLIT_EARLY=1: the next batch's framing walk starts at the top of the call (A/B against
  // starting it once the first back-half kernels are queued)
  static const bool presplit_early = [] {
    const char *e = getenv("FGV_PRESPLIT_EARLY");
    return e && atoi(e) != 0;
  }();
  if (presplit_early && nx.n) {
    fgv_block_presplit(S, c->device, nx.n, nx.blocks, nx.lens, nx.lo, nx.hi);
    c->next.n = 0;
  }
  if (S->ch.dirty || S->dev_dirty) {
    drain_ahead(c, S);  // (its kernels read the image about to be rebuilt; its results are stale)
    if (S->ch.dirty) S->ch.compile();
    int rc = build_dev_image(S);
    if (rc) return rc;
    S->dev_dirty = false;
  } else if (S->txid_dirty) {
    int rc = build_committed(S);
    if (rc) return rc;
  }
  // --- front half: enqueued by the previous call, or now
  int cur;
  bool ahead_hit = false;
  if (S->ahead >= 0 && S->set[S->ahead].matches(nblocks, h_blocks, lens, d_blocks, tx_lo, tx_hi)) {
    cur = S->ahead;
    ahead_hit = true;
    S->ahead = -1;
  } else {
    drain_ahead(c, S);
    cur = S->last ^ 1;
    int rc = front_launch(c, S, S->set[cur], nblocks, h_blocks, lens, d_blocks, tx_lo, tx_hi, c->stream, nullptr);
    if (rc) return rc;
  }
  S->last = cur;
  BdSet &B = S->set[cur];
  for (size_t b = 0; b < nblocks; b++) ntx_out[b] = B.so.ntx[b];
  c->n_sha_jobs = c->n_sha_blocks = c->n_verifies = 0;
  c->last_presplit = B.presplit;
  c->last_ahead = ahead_hit;
  if (B.so.total > res_cap) return FGV_EINVAL;
  const uint32_t N = B.N;
  if (N == 0) return FGV_OK;
  c->t_host_parse = ms_since(t0);
  auto t1 = clk::now();
  // --- back half on the main stream, enqueued without reading the job counts back: the verify
  // columns are sized for the batch's capacity (a creator + BD_MAX_END endorsements per tx) and
  // k_bd_emit leaves the verify count in device memory (misc[10]) for k_der ... k_point
  const size_t cap = (size_t)N * (1 + BD_MAX_END);
  const size_t n_est = (size_t)((double)N * (S->nv_per_tx > 0 ? S->nv_per_tx : 3.5) + 0.5);
  hipStream_t st = c->stream;
  const DevChannel ch = S->dimg.ch;
  uint32_t *misc = reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff);
  const uint64_t *dbs = reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff);
  DevTx *dtx = B.tx.as<DevTx>();
  int32_t *did = B.ident.as<int32_t>();
  DevJobIdx *dj = B.jobs.as<DevJobIdx>();
  const bool tim = c->timing && B.timed;
  if (B.vdone) {  // k_bd_emit, k_der, k_inv ran ahead with the front half (front_launch prefix)
    HIP_TRY(hipStreamWaitEvent(st, B.ev[9], 0));
  } else {
    if (B.stream != st) HIP_TRY(hipStreamWaitEvent(st, B.ev[6], 0));  // (a front half enqueued ahead)
    int rc = emit_prefix(c, S, B, st);
    if (rc) return rc;
  }
  // host time from the end of the previous validation call to this call's first back-half kernel
  // (the caller's own work between calls included)
  c->t_gap = c->t_call_end.time_since_epoch().count() ? ms_since(c->t_call_end) : 0.0;
  // FGV_FRONT_EARLY (default 1): when the next batch's framing walk is already done (the caller
  // pre-split it with fgv_presplit after the previous call), its head upload, k_bd_parse and
  // payload hashes are queued here, beside this batch's first back-half kernels, instead of behind
  // the whole back half and finalize (~0.1 ms of host enqueue later); the rest of its front half
  // follows where it always did (launch_ahead: front_launch_b)
  static const bool front_early = [] {
    const char *e = getenv("FGV_FRONT_EARLY");
    return !e || atoi(e) != 0;
  }();
  S->early = -1;
  S->early_ms = 0;
  const auto te = clk::now();
  const PreSplit *nxp = nx.n ? pre_find(S, nx.n, nx.blocks, nx.lens, nx.lo, nx.hi) : nullptr;
  // (not while the verifies use the variable-base kernels -- the last call's n_vb: beside them the
  // early parse measured 1.36 ms per C2 churn step against 1.30 without, r5pc)
  if (front_early && nx.n && nx.d_blocks && !nx.wait && c->ahead_mode == 2 && c->n_vb == 0 && nxp &&
      const_cast<PreSplit *>(nxp)->ready()) {
    if (front_launch_a(c, S, S->set[cur ^ 1], nx.n, nx.blocks, nx.lens, nx.d_blocks, nx.lo, nx.hi, c->streamF,
                       nx.wait, nullptr) == FGV_OK) {
      S->early = cur ^ 1;
      S->early_ms = ms_since(te);
    } else {
      S->ahead = cur ^ 1;  // (the next call starts it again and reports any error)
      drain_ahead(c, S);
    }
    c->next.n = 0;  // (its pre-split is used)
  }
  // the next batch's framing walk, on the host worker while this batch's GPU work runs (started
  // once the first kernels of this back half are queued: the GPU gets them a few us sooner)
  if (nx.n && !presplit_early && S->early < 0) {
    fgv_block_presplit(S, c->device, nx.n, nx.blocks, nx.lens, nx.lo, nx.hi);
    c->next.n = 0;
  }
  c->digests_ready = B.ev[8];  // (payload and the other digests, joined on stream3)
  c->digests_ready2 = nullptr;
  int rc = fgv_verify_main_dev(c, cap, B.emitted ? misc + BJ_C : misc + 10, n_est, B.vsig.as<uint8_t>(), B.vst.as<uint8_t>(),
                               B.vr.as<uint32_t>(), B.vw.as<uint32_t>(), B.dig.as<uint8_t>());
  c->digests_ready = c->digests_ready2 = nullptr;
  if (rc) return rc;
  // (the digests were joined before k_prep: the verify stages always run, for the capacity)
  if (tim) HIP_TRY(hipEventRecord(c->kev[8], st));
  // the fused single-device call: its finalize's txid index runs on stream3 after the batch's
  // digests, beside the verify chain (fgv_finalize_early_index).  Enqueued after the verify
  // chain, so the host's plan preparation overlaps the chain's first kernels instead of
  // delaying them (the main stream is idle between two calls until k_bd_emit is queued)
  if (c->want_early_fin && !tx_lo && !tx_hi && B.N) {
    // the key-level dependencies (nothing to do without key-level records), ahead of the index
    hipLaunchKernelGGL(k_bd_kl, dim3((B.N + 255) / 256), dim3(256), 0, c->stream3, B.N, B.tx.as<DevTx>(),
                       reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff), B.kl,
                       reinterpret_cast<uint32_t *>(B.env.as<uint8_t>() + B.moff) + 5);
    int rc = fgv_finalize_early_index(c, nblocks, B.so.ntx.data(), B.tx.as<DevTx>(),
                                      reinterpret_cast<const uint64_t *>(B.env.as<uint8_t>() + B.eoff),
                                      B.dig.as<uint8_t>(), c->stream3);
    if (rc) return rc;
  }
  // the finalize's codes step inside the fold once the early index (stream3) is there
  FinDev fin{};
  c->fold_codes = false;
  if (c->early_fin) {
    HIP_TRY(hipStreamWaitEvent(st, c->fin_ev, 0));
    size_t cap = 1024;
    while (cap < 2 * (size_t)N) cap <<= 1;
    fin = FinDev{c->fz_owner.as<uint32_t>(), c->fz_minblk.as<int32_t>(), c->fz_minvalid.as<uint32_t>(),
                 c->fz_keys.as<uint8_t>(), c->fz_flags.as<uint8_t>(), c->fz_pslot.as<uint32_t>(),
                 (uint32_t)(cap - 1), c->fin_seed};
    c->fold_codes = true;
    c->fold_unsup = misc + 5;  // (k_fin_dups: a first VALID position failed by the key-level walk)
  }
  static const uint32_t fold_touch = [] {
    const char *e = getenv("FGV_FOLD_TOUCH");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  // FGV_FOLD_WG = threads per workgroup of the fold (64 / 128 / 256, default 256; A/B: a lane per
  // transaction, latency-bound, so smaller workgroups spread the same waves over more CUs)
  static const uint32_t fold_wg = [] {
    const char *e = getenv("FGV_FOLD_WG");
    const uint32_t v = e ? (uint32_t)atoi(e) : 256u;
    return (v == 64u || v == 128u) ? v : 256u;
  }();
  hipLaunchKernelGGL(k_bd_fold, dim3((N + fold_wg - 1) / fold_wg), dim3(fold_wg), 0, st, N, dtx, dbs, ch, did, dj, misc,
                     B.dig.as<uint8_t>(), B.vst.as<uint8_t>(), d_res, misc + 5, misc + 16, fin, B.kl,
                     fold_touch);
  HIP_TRY(hipGetLastError());
  if (tim || c->ahead_mode == 3) HIP_TRY(hipEventRecord(c->kev[9], st));  // (ahead mode 3 waits on it)
  // (the counters' D2H is queued by fgv_block_validate_dev_finish, behind whatever the caller
  // queues after the fold -- the finalize -- so it never sits between the fold and the finalize)
  B.misc_src = misc;
  c->fin_misc_src = c->fold_codes ? misc : nullptr;  // (k_fin_dups copies them out: fin_back)
  c->fin_misc_dst = B.misc.as<uint32_t>();
  c->fin_misc_done = false;
  c->t_bd_pre = ms_since(t1);
  c->t_host_assemble = c->t_bd_pre;
  S->t_enq = clk::now();
  // --- the next batch's front half, ahead of its call (launch_ahead).  The fused single-GPU
  // call defers it until its finalize kernels are queued: the host spends ~0.1 ms enqueuing a
  // front half (its pre-split join included), and k_fin_dups queued behind that started ~65 us
  // after the fold it follows (MI355X C2 trace, r4e)
  if (c->defer_ahead) {
    S->ahead_nx = nx;
    S->ahead_cur = cur;
    S->ahead_deferred = true;
  } else {
    launch_ahead(c, S, nx, cur);
  }
  S->pending = cur;
  return FGV_OK;
}

// Wait for the batch enqueued by fgv_block_validate_dev_enqueue (the caller may have enqueued
// more work on c->stream after it, e.g. the finalize kernels) and read its outcome: FGV_OK,
// FGV_EUNSUPPORTED, or 1 = a transaction exceeded a device capacity (run the host parser).
int fgv_block_validate_dev_finish(fgv_ctx *c, fgv_block_state *S) {
  using clk = std::chrono::steady_clock;
  if (S->pending < 0) return FGV_OK;
  BdSet &B = S->set[S->pending];
  S->pending = -1;
  if (B.misc_src && !c->fin_misc_done) HIP_TRY(hipMemcpyAsync(B.misc.p, B.misc_src, 64, hipMemcpyDeviceToHost, c->stream));
  B.misc_src = nullptr;
  c->fin_misc_done = false;
  c->fin_misc_src = nullptr;
  const int pp = S->prefix_next;
  S->prefix_next = -1;
  if (pp >= 0 && S->ahead == pp && S->set[pp].N && !S->set[pp].vdone) {
    // the next batch's verify prefix behind this call's work (prefix_main, launch_ahead)
    if (!S->done_ev) HIP_TRY(hipEventCreateWithFlags(&S->done_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(S->done_ev, c->stream));
    BdSet &A = S->set[pp];
    HIP_TRY(hipStreamWaitEvent(c->stream, A.ev[6], 0));
    if (emit_prefix(c, S, A, c->stream) != FGV_OK) {
      drain_ahead(c, S);  // (the next call starts its batch again)
      A.vdone = false;
    }
    if (c->spin) {
      hipError_t e;
      while ((e = hipEventQuery(S->done_ev)) == hipErrorNotReady) __builtin_ia32_pause();
      HIP_TRY(e);
    } else {
      HIP_TRY(hipEventSynchronize(S->done_ev));
    }
  } else {
    HIP_TRY(fgv_stream_wait(c->stream, c->spin));
  }
  const auto t_woke = clk::now();
  fgv_read_block_job_times(c);
  {  // per-kernel device times (fgv_last_kernel_times)
    auto el = [&](hipEvent_t a, hipEvent_t b) {
      float ms = 0;
      return hipEventElapsedTime(&ms, a, b) == hipSuccess ? (double)ms : 0.0;
    };
    // always (stream-ordering events): payload, parse, k_bd_sha, identities + counts
    c->t_kern[0] = el(B.ev[3], B.ev[1]);  // k_bd_sha_payload
    c->t_kern[1] = el(B.ev[3], B.ev[4]);  // k_bd_parse
    c->t_kern[2] = el(B.timed ? B.ev[5] : B.ev[4], B.ev[2]);  // k_bd_sha
    c->t_kern[3] = el(B.timed ? B.ev[7] : B.ev[4], B.ev[6]);  // k_bd_ident + k_bd_count
    const bool tim = c->timing && B.timed;  // with fgv_set_timing only
    c->t_kern[4] = tim ? el(c->kev[6], c->kev[7]) : 0.0;                     // k_bd_emit
    c->t_kern[5] = tim && c->stage_ran ? el(c->ev[2], c->ev[3]) : 0.0;  // k_der + k_inv
    c->t_kern[6] = tim && c->stage_ran ? el(c->ev[4], c->ev[5]) : 0.0;  // k_prep
    c->t_kern[7] = c->stage_ran ? el(c->ev[5], c->ev[6]) : 0.0;  // k_point28 (+ k_point hand-overs), live
    c->t_kern[8] = tim ? el(c->kev[8], c->kev[9]) : 0.0;               // k_bd_fold
    c->t_kern[9] = tim ? el(B.ev[0], c->kev[9]) : 0.0;                 // the batch, head upload to fold
    c->t_sha = std::max(c->t_kern[0], el(B.ev[3], B.ev[2]));
    (void)hipGetLastError();  // (an interval whose events this call did not record is 0, not a sticky error)
  }
  const uint32_t *hm = B.misc.as<uint32_t>();
  uint64_t nb, np;
  memcpy(&nb, hm + 6, 8);
  memcpy(&np, hm + 8, 8);
  c->n_sha_blocks = nb + np;
  c->n_pay_blocks = np;
  const uint32_t nv = B.emitted ? hm[BJ_C] : hm[10];  // (the fused count: endorsements inside BJ_C)
  c->n_verifies = nv;
  if (B.N) S->nv_per_tx = (double)nv / B.N;  // the next batch's lanes-per-verify estimate
  c->t_host_device = std::chrono::duration<double, std::milli>(clk::now() - S->t_enq).count();
  c->t_host_fold = 0;
  c->t_finish = std::chrono::duration<double, std::milli>(clk::now() - t_woke).count();
  if ((hm[5] & 1u) || B.force_host) return 1;
  // per-block outcomes: the undecided transactions carry 0xFD in the flags, the first block that
  // must wait for an earlier one's commit comes back in word 12 (k_bd_kl)
  if (S->soft) {
    if (hm[5] & 2u) S->soft_unsup = true;
    if (hm[12]) S->split = std::min<uint32_t>(S->split, ~hm[12]);
    return FGV_OK;
  }
  if (hm[5] & 2u) return FGV_EUNSUPPORTED;
  return FGV_OK;
}

int fgv_block_validate_dev(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                           const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                           const uint32_t *tx_hi, fgv_tx_result *d_res, size_t res_cap, size_t *ntx_out) {
  const int rc = fgv_block_validate_dev_enqueue(c, S, nblocks, h_blocks, lens, d_blocks, tx_lo, tx_hi, d_res,
                                                res_cap, ntx_out);
  if (rc) {
    S->pending = -1;
    return rc;
  }
  return fgv_block_validate_dev_finish(c, S);
}

// ======================================================================= orderer signatures
// BlockSignatureVerifier (protoutil/blockutils.go:245-290) for a channel that does not run BFT,
// then policy.EvaluateSignedData of the channel policy it was built with
// (deliverclient/verifier_assembler.go:32-56: /Channel/Orderer/BlockValidation):
//   Metadata = proto.Unmarshal(metadata[SIGNATURES])            error -> fail
//   per MetadataSignature, in order: SignatureHeader unmarshal   error -> fail
//     SignedData{Identity: header.Creator, Signature, Data: md.Value || signature_header ||
//                BlockHeaderBytes(header)}
//   EvaluateSignedData: SignatureSetToValidIdentities (policy.go:363-395: deserialize, dedup on
//   Mspid+Id, verify, in order) feeding the cauthdsl / ImplicitMeta evaluation.
// Under BFT a signature with an empty signature header and an identifier header names a
// consenter by number (blockutils.go:262-273): outside the model -> FGV_SIGV_UNSUP.  Verify bits
// are pure functions of (key, message, signature), so every block's signatures are verified in
// one GPU pass ahead of the sequential fold.
namespace {
struct VMetaSig {  // MetadataSignature {signature_header = 1, signature = 2, identifier_header = 3}
  Span sig_header, signature, id_header;
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    (n == 1 ? sig_header : n == 2 ? signature : id_header) = s;
    return true;
  }
};
struct VMetadata {  // Metadata {value = 1, repeated MetadataSignature signatures = 2}
  Span value;
  std::vector<VMetaSig> sigs;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : n == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) {
      value = s;
      return true;
    }
    VMetaSig m;
    if (!pbw::decode(s.p, s.n, m)) return false;
    sigs.push_back(m);
    return true;
  }
};
struct VMeta0 {  // BlockMetadata: metadata[SIGNATURES]
  bool has = false;
  Span sigs;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_REP_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    if (!has) sigs = s, has = true;
    return true;
  }
};
struct VBlockMeta0 {  // Block: field 3 only
  bool has = false;
  Span sigs;
  pbw::Kind kind(uint32_t n) { return n == 3 ? pbw::K_MSG : (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    VMeta0 m;
    if (!pbw::decode(s.p, s.n, m)) return false;
    if (m.has) has = true, sigs = m.sigs;
    return true;
  }
};
struct SigItem {
  int ident;          // Channel::lookup: index, -1 deserialize error, -2 outside the model
  uint32_t vjob;      // verify job (UINT32_MAX: none)
  Span sig;
};
}  // namespace

// ManagerImpl.GetPolicy on the root manager (policy.go:330-358): index, 0 = reject (absent,
// or not under /Channel/), -1 = no usable channel config
static int channel_policy_index(const Channel &ch, const std::string &path) {
  if (!ch.config.present || ch.config.unsupported) return -1;
  std::string ref = path;
  if (!ref.empty() && ref[0] == '/') {
    static const std::string root = "/Channel/";
    if (ref.compare(0, root.size(), root) != 0) return 0;
    ref = ref.substr(root.size());
  }
  auto it = ch.chan_idx.find(ref);
  return (ref.empty() || it == ch.chan_idx.end()) ? 0 : it->second;
}

int fgv_block_sig_verdicts(fgv_ctx *c, size_t n, const fgv_sig_block *in, const char *policy, int bft,
                           uint8_t *verdict) {
  std::lock_guard<std::mutex> g(c->mu);
  Channel &ch = c->blk->ch;
  if (ch.dirty) ch.compile();
  // orderer identities the registry has not seen: the MSP cache miss first (fgv_msp.cpp)
  if (fgv_msp_auto(c)) {
    std::vector<std::string> miss;
    for (size_t b = 0; b < n; b++) {
      VMetadata md;
      if (!in[b].want || !pbw::decode(in[b].meta, in[b].meta_n, md)) continue;
      for (const VMetaSig &ms : md.sigs) {
        VSignatureHeader sh;
        if (pbw::decode(ms.sig_header.p, ms.sig_header.n, sh) && ch.lookup(sh.creator) == -2)
          miss.push_back(sh.creator.str());
      }
    }
    if (!miss.empty()) {
      std::vector<const uint8_t *> mp(miss.size());
      std::vector<size_t> ml(miss.size());
      std::vector<int> st(miss.size());
      for (size_t i = 0; i < miss.size(); i++) {
        mp[i] = reinterpret_cast<const uint8_t *>(miss[i].data());
        ml[i] = miss[i].size();
      }
      const int rc = fgv_msp_resolve_locked(c, miss.size(), mp.data(), ml.data(), st.data(), nullptr);
      if (rc) return rc;
      if (ch.dirty) ch.compile();
    }
  }
  const int pi = channel_policy_index(ch, policy ? policy : "/Channel/Orderer/BlockValidation");
  // does the evaluation reach SignatureSetToValidIdentities?  A signature policy does; an
  // ImplicitMeta policy does through any signature sub-policy (a rejecting sub-policy never
  // satisfies, so the walk cannot stop before the first signature one); a reject policy never.
  bool reads_ids = false;
  if (pi > 0) {
    const Policy &P = ch.policies[pi];
    reads_ids = P.kind == PK_SIG || P.kind == PK_UNSUP;
    if (P.kind == PK_IMPLICIT)
      for (int s : P.subs) reads_ids |= ch.policies[s].kind != PK_REJECT;
  }
  std::vector<std::vector<SigItem>> items(n);
  std::vector<uint8_t> msgs;
  std::vector<uint64_t> moff, soff;
  std::vector<uint32_t> mlen, slen, slots;
  std::vector<const uint8_t *> sptr;
  for (size_t b = 0; b < n; b++) {
    verdict[b] = FGV_SIGV_FAIL;
    if (!in[b].want) continue;
    if (pi < 0) {
      verdict[b] = FGV_SIGV_UNSUP;
      continue;
    }
    VMetadata md;
    if (!pbw::decode(in[b].meta, in[b].meta_n, md)) continue;  // "error unmarshalling signatures"
    bool bad = false, unsup = false;
    std::vector<SigItem> &its = items[b];
    const size_t m0 = msgs.size(), j0 = moff.size();
    for (const VMetaSig &ms : md.sigs) {
      if (bft && ms.sig_header.n == 0 && ms.id_header.n > 0) {
        unsup = true;
        break;
      }
      VSignatureHeader sh;
      if (!pbw::decode(ms.sig_header.p, ms.sig_header.n, sh)) {
        bad = true;
        break;
      }
      SigItem it{ch.lookup(sh.creator), UINT32_MAX, ms.signature};
      if (it.ident >= 0 && ch.idents[it.ident].verify_class() == 0 && reads_ids) {
        it.vjob = (uint32_t)moff.size();
        moff.push_back(msgs.size());
        msgs.insert(msgs.end(), md.value.p, md.value.p + md.value.n);
        msgs.insert(msgs.end(), ms.sig_header.p, ms.sig_header.p + ms.sig_header.n);
        msgs.insert(msgs.end(), in[b].hdr_der.begin(), in[b].hdr_der.end());
        mlen.push_back((uint32_t)(msgs.size() - moff.back()));
        sptr.push_back(ms.signature.p);
        slen.push_back(ms.signature.n);
        slots.push_back((uint32_t)ch.idents[it.ident].key_slot);
      }
      its.push_back(it);
    }
    if (bad || unsup) {
      verdict[b] = unsup ? FGV_SIGV_UNSUP : FGV_SIGV_FAIL;
      its.clear();
      msgs.resize(m0);
      moff.resize(j0);
      mlen.resize(j0);
      sptr.resize(j0);
      slen.resize(j0);
      slots.resize(j0);
      continue;
    }
    verdict[b] = 0xFF;  // evaluated below
  }
  // one GPU pass over every signature the evaluations may read
  const size_t nv = moff.size();
  std::vector<uint8_t> vst(nv, 1);
  if (nv) {
    std::vector<uint8_t> sigs;
    soff.resize(nv);
    for (size_t j = 0; j < nv; j++) {
      soff[j] = sigs.size();
      sigs.insert(sigs.end(), sptr[j], sptr[j] + slen[j]);
    }
    const int rc = fgv_verify_msgs_slots_locked(c, msgs.data(), msgs.size(), moff.data(), mlen.data(), sigs.data(),
                                                sigs.size(), soff.data(), slen.data(), slots.data(), nv, vst.data());
    if (rc) return rc;
  }
  for (size_t b = 0; b < n; b++) {
    if (verdict[b] != 0xFF) continue;
    pbw::SmallVec<int, 16> ids;
    bool unsup = false;
    if (reads_ids) {
      pbw::SmallVec<uint32_t, 16> seen;
      for (const SigItem &it : items[b]) {
        if (it.ident == -2) { unsup = true; break; }
        if (it.ident < 0) continue;
        const Ident &I = ch.idents[it.ident];
        if (std::find(seen.begin(), seen.end(), I.canon) != seen.end()) continue;
        const int vc = I.verify_class();
        if (vc == 2) { unsup = true; break; }
        if (vc == 1 || it.vjob == UINT32_MAX || vst[it.vjob] != 0) continue;
        seen.push_back(I.canon);
        ids.push_back(it.ident);
      }
    }
    int v = unsup ? 2 : pi == 0 ? 0 : eval_policy(ch, pi, ids.data(), ids.size());
    verdict[b] = v == 2 ? FGV_SIGV_UNSUP : v == 1 ? FGV_SIGV_OK : FGV_SIGV_FAIL;
  }
  return FGV_OK;
}

// ======================================================================= MSP cache misses
void fgv_block_misses(fgv_block_state *S, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                      std::vector<std::string> &out) {
  Channel &ch = S->ch;
  if (ch.dirty) ch.compile();
  std::vector<Span> envs;
  for (size_t b = 0; b < nblocks; b++) {
    VBlock blk;
    if (pbw::decode(blocks[b], lens[b], blk)) envs.insert(envs.end(), blk.data.data.begin(), blk.data.data.end());
  }
  std::vector<std::vector<Span>> per(envs.size());
  S->pool.parallel_for(envs.size(), [&](size_t t) {
    auto add = [&](const Span &id) {
      if (ch.lookup(id) == -2) per[t].push_back(id);
    };
    VEnvelope env;
    VPayload pl;
    VHeader hdr;
    if (!pbw::decode(envs[t].p, envs[t].n, env) || !pbw::decode(env.payload.p, env.payload.n, pl) ||
        !pl.header.decode_into(hdr))
      return;
    VSignatureHeader sh;
    if (pbw::decode(hdr.signature_header.p, hdr.signature_header.n, sh)) add(sh.creator);
    VTransaction tx;
    if (!pbw::decode(pl.data.p, pl.data.n, tx)) return;
    for (const VTransactionAction &act : tx.actions) {
      VCcActionPayload cap;
      if (!pbw::decode(act.payload.p, act.payload.n, cap) || !cap.has_action) continue;
      for (const auto &e : cap.action.ends) add(e.endorser);
    }
  });
  std::unordered_set<std::string_view> seen;
  for (const auto &v : per)
    for (const Span &id : v) {
      const std::string_view k(reinterpret_cast<const char *>(id.p), id.n);
      if (seen.insert(k).second) out.push_back(std::string(k));
    }
  // IDENTITY principals of the compiled policies that name a never-deserialized certificate
  for (const std::string &p : ch.unresolved_principals)
    if (seen.insert(p).second) out.push_back(p);
}

// ======================================================================= sanitizer probe
// The host parser alone, for the CPU sanitizer build (tools/sanitize): every envelope of a
// block through parse_tx + count_jobs against a channel with the given identities (valid P-256,
// key slot 0, roles unknown) and chaincode definition, the policy fold over each transaction's
// resolved endorsers (as if every signature verified), then the block's orderer-signature
// metadata (Metadata / SignatureHeader decode, identity lookup).  No GPU call.  Returns a digest
// of the decided codes (the harness only needs the parse to be memory-safe).
uint64_t fgv_block_parse_probe(const char *channel, const uint8_t *const *ids, const size_t *id_lens, size_t nids,
                               const char *ns, const uint8_t *policy, size_t policy_len, const uint8_t *blk,
                               size_t n) {
  fgv_block_state S(1);
  fgv_block_set_channel(&S, channel);
  fgv_identity_info info{};
  info.key_type = FGV_KEY_P256;
  info.valid = 1;
  info.roles = FGV_ROLES_UNKNOWN;
  for (size_t i = 0; i < nids; i++) {
    for (int k = 0; k < 32; k++) info.id_digest[k] = (uint8_t)(i * 31 + k);
    fgv_block_add_identity(&S, ids[i], id_lens[i], 0, &info);
  }
  if (ns) fgv_block_define_chaincode(&S, ns, "vscc", policy, policy_len, 0);
  if (ns) {  // key-level parameters: the policy bytes as a (maybe untranslatable) envelope
    fgv_block_kvmeta_set(&S, ns, "", reinterpret_cast<const uint8_t *>("k0000001"), 8, policy, policy_len);
    fgv_block_kvmeta_set(&S, ns, "collA", reinterpret_cast<const uint8_t *>("k0000002"), 8, policy, policy_len);
  }
  Channel &ch = S.ch;
  ch.compile();
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&](uint64_t v) { h = (h ^ v) * 0x100000001b3ull; };
  VBlock b;
  if (!pbw::decode(blk, n, b)) return 0;
  TxRec R;
  SbeBlock sb;
  sb.res.resize(b.data.data.size());
  uint32_t i = 0;
  for (const Span &d : b.data.data) {
    parse_tx(ch, d, R);
    count_jobs(ch, R);
    mix(R.pre);
    mix(R.etx);
    mix(R.disp);
    mix(R.n_ej);
    mix(R.xstat);
    if (R.has_md && R.xstat == X_OK) add_deps(R.results, i, sb);
    if (R.disp == C_VALID) {
      pbw::SmallVec<int, 16> ids_ok;
      for (const EndRec &e : R.ends)
        if (e.ident >= 0 && std::find(ids_ok.begin(), ids_ok.end(), e.ident) == ids_ok.end()) ids_ok.push_back(e.ident);
      for (int pi : R.policies)
        if (pi >= 0) mix((uint64_t)eval_policy(ch, pi, ids_ok.data(), ids_ok.size()));
      // the key-level vscc walk of every namespace of the rwset
      VTxRwSet rw;
      if (pbw::decode(R.results.p, R.results.n, rw))
        for (const VNsRwSet &nr : rw.ns) {
          auto it = ch.ccs.find(nr.ns.str());
          if (it == ch.ccs.end() || it->second.status != 0) continue;
          auto eval = [&](int pi) { return eval_policy(ch, pi, ids_ok.data(), ids_ok.size()); };
          const int r = sbe_vscc(ch, it->second, sv(nr.ns), &nr, i, sb, false, eval);
          mix((uint64_t)r);
          if (r == 0 || r == 1) sb.res[i].push_back({nr.ns.str(), (int8_t)r});
        }
    }
    i++;
  }
  // the orderer-signature metadata (fgv_block_sig_verdicts' decode)
  VBlockMeta0 m;
  if (pbw::decode(blk, n, m) && m.has) {
    VMetadata md;
    if (pbw::decode(m.sigs.p, m.sigs.n, md))
      for (const VMetaSig &ms : md.sigs) {
        VSignatureHeader sh;
        if (pbw::decode(ms.sig_header.p, ms.sig_header.n, sh)) mix((uint64_t)(int64_t)ch.lookup(sh.creator));
      }
  }
  return h;
}
