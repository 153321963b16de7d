// fgv_group.cpp -- the committer on several GPUs of one process (fgv_group_*, include/fgv.h).
//
// The multi-GPU protocol of fabric_amd/shard.py (one process per GPU over RCCL) inside the
// library, for a peer that drives all its GPUs from one process through the C ABI (a Go peer
// over cgo): a batch's blocks are split into contiguous ranges of about equal bytes, one per
// device ("block" plan: each device stages, splits and parses only its own blocks); every device
// validates its range on its own host worker (fgv_validate_shard_dev into its own HBM); the
// records (68 B per transaction) are gathered onto the first device with peer copies over xGMI;
// the first device runs the two cross-transaction steps of the reference -- the block-store txid
// index of earlier blocks of the batch (checkTxIdDupsLedger, validator.go:460-481) and
// markTXIdDuplicates (validator.go:279-295) -- as the finalize kernels.  Only the records cross
// the fabric (a gather to one device, not an all-gather: the flags leave from there), and the
// per-device work is TxValidator.Validate's, so results equal fgv_validate_blocks on one GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sched.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "fgv_internal.h"
#include "thread_pool.h"

// RCCL, loaded on first use (fgv_group_set_collective): the library is resolved at run time with
// RTLD_LOCAL so a host process that carries its own RCCL copy (a torch peer, say) keeps it apart
// from ours, and a peer that never asks for the collective never loads it.
namespace {
struct Rccl {
  void *h = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool load() {
    if (h) return true;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
    comm_init_all = reinterpret_cast<decltype(comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    comm_destroy = reinterpret_cast<decltype(comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    all_gather = reinterpret_cast<decltype(all_gather)>(dlsym(h, "ncclAllGather"));
    group_start = reinterpret_cast<decltype(group_start)>(dlsym(h, "ncclGroupStart"));
    group_end = reinterpret_cast<decltype(group_end)>(dlsym(h, "ncclGroupEnd"));
    return comm_init_all && comm_destroy && all_gather && group_start && group_end;
  }
};
Rccl &rccl() {
  static Rccl r;
  return r;
}
std::mutex rccl_mu;  // (one-time load)
}  // namespace

struct fgv_group {
  std::vector<fgv_ctx *> ctx;
  std::vector<int> dev;
  std::vector<DevBuf> res;  // per device: its shard's records (allocated on that device)
  DevBuf gath;              // on device 0: world x rows records
  hipStream_t s0 = nullptr; // device 0: the gather copies
  ThreadPool *pool = nullptr;
  std::mutex mu;
  // per-block outcomes (fgv_group_set_block_outcomes) and those of the last call
  bool soft = false;
  std::vector<int32_t> blk_status;
  size_t n_final = 0;
  int last_rc = FGV_OK;  // the last call's return code
  // FGV_GROUP_COLL_RCCL: one RCCL communicator over the devices, the records all-gathered into
  // every device's HBM on its own stream, the finalize on every device
  int coll = FGV_GROUP_COLL_PEER;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> cs;   // per device: the collective's stream
  std::vector<DevBuf> gathr;     // per device: world x rows records
  std::vector<std::vector<uint8_t>> dflags;  // devices 1..: their finalized flags (checked equal)
};

extern "C" {

int fgv_group_init(const int *devices, size_t ndev, const fgv_config *cfg, fgv_group **out) {
  if (!devices || !ndev || !out || ndev > 64) return FGV_EINVAL;
  *out = nullptr;
  fgv_group *g = new fgv_group();
  // host workers: the process's CPU share split between the devices (unless given)
  unsigned share = 0;
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) share = (unsigned)CPU_COUNT(&cs);
  for (size_t i = 0; i < ndev; i++) {
    fgv_config c = cfg ? *cfg : fgv_config{};
    c.device = devices[i];
    if (c.host_threads == 0 && share) c.host_threads = std::max(2u, std::min(24u, share / (unsigned)ndev));
    fgv_ctx *x = nullptr;
    const int rc = fgv_init(&c, &x);
    if (rc) {
      fgv_group_destroy(g);
      return rc;
    }
    g->ctx.push_back(x);
    g->dev.push_back(devices[i]);
  }
  g->res.resize(ndev);
  if (hipSetDevice(devices[0]) != hipSuccess || hipStreamCreateWithFlags(&g->s0, hipStreamNonBlocking) != hipSuccess) {
    fgv_group_destroy(g);
    return FGV_EDEVICE;
  }
  // peer access from device 0 to the others (xGMI); a device already enabled, or the same
  // device twice, is fine -- the copies work either way
  for (size_t i = 1; i < ndev; i++)
    if (devices[i] != devices[0]) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[0], devices[i]) == hipSuccess && can) {
        const hipError_t e = hipDeviceEnablePeerAccess(devices[i], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      }
    }
  g->pool = new ThreadPool((unsigned)ndev);
  *out = g;
  return FGV_OK;
}

static void coll_release(fgv_group *g) {
  for (size_t i = 0; i < g->comms.size(); i++)
    if (g->comms[i]) rccl().comm_destroy(g->comms[i]);
  g->comms.clear();
  for (size_t i = 0; i < g->cs.size(); i++)
    if (hipSetDevice(g->dev[i]) == hipSuccess) {
      if (g->cs[i]) hipStreamDestroy(g->cs[i]);
      if (i < g->gathr.size()) g->gathr[i].release();
    }
  g->cs.clear();
  g->gathr.clear();
  g->dflags.clear();
  g->coll = FGV_GROUP_COLL_PEER;
}

int fgv_group_set_collective(fgv_group *g, int mode) {
  if (!g || (mode != FGV_GROUP_COLL_PEER && mode != FGV_GROUP_COLL_RCCL)) return FGV_EINVAL;
  std::lock_guard<std::mutex> lk(g->mu);
  if (mode == g->coll) return FGV_OK;
  coll_release(g);
  if (mode == FGV_GROUP_COLL_PEER) return FGV_OK;
  const size_t W = g->ctx.size();
  for (size_t i = 0; i < W; i++)  // (a communicator has one rank per device)
    for (size_t j = i + 1; j < W; j++)
      if (g->dev[i] == g->dev[j]) return FGV_EINVAL;
  {
    std::lock_guard<std::mutex> l2(rccl_mu);
    if (!rccl().load()) return FGV_EDEVICE;
  }
  g->comms.assign(W, nullptr);
  if (rccl().comm_init_all(g->comms.data(), (int)W, g->dev.data()) != ncclSuccess) {
    g->comms.clear();
    return FGV_EDEVICE;
  }
  g->cs.assign(W, nullptr);
  g->gathr.resize(W);
  for (size_t i = 0; i < W; i++)
    if (hipSetDevice(g->dev[i]) != hipSuccess || hipStreamCreateWithFlags(&g->cs[i], hipStreamNonBlocking) != hipSuccess) {
      coll_release(g);
      return FGV_EDEVICE;
    }
  g->coll = FGV_GROUP_COLL_RCCL;
  return FGV_OK;
}

void fgv_group_destroy(fgv_group *g) {
  if (!g) return;
  coll_release(g);
  delete g->pool;
  for (size_t i = 0; i < g->ctx.size(); i++) {
    if (hipSetDevice(g->dev[i]) == hipSuccess) g->res[i].release();
    fgv_destroy(g->ctx[i]);
  }
  if (!g->dev.empty() && hipSetDevice(g->dev[0]) == hipSuccess) {
    g->gath.release();
    if (g->s0) hipStreamDestroy(g->s0);
  }
  delete g;
}

size_t fgv_group_size(const fgv_group *g) { return g ? g->ctx.size() : 0; }

fgv_ctx *fgv_group_ctx(fgv_group *g, size_t i) { return g && i < g->ctx.size() ? g->ctx[i] : nullptr; }

static int group_validate_locked(fgv_group *g, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                 uint8_t *flags, size_t flags_cap, size_t *ntx);
static int group_outcomes(fgv_group *g, size_t nblocks, const size_t *ntx, const uint8_t *flags, bool soft,
                          size_t n_final);

int fgv_group_validate_blocks(fgv_group *g, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                              uint8_t *flags, size_t flags_cap, size_t *ntx) {
  if (!g || (nblocks && (!blocks || !lens || !flags || !ntx))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> lk(g->mu);
  g->blk_status.clear();
  g->n_final = 0;
  return g->last_rc = group_validate_locked(g, nblocks, blocks, lens, flags, flags_cap, ntx);
}

static int group_validate_locked(fgv_group *g, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                 uint8_t *flags, size_t flags_cap, size_t *ntx) {
  const bool soft = g->soft;
  const size_t W = g->ctx.size();
  // The plan.  At least as many blocks as devices: contiguous block ranges of about total/W
  // bytes (a device stages, splits and parses only its own).  Fewer (one block, a short batch):
  // contiguous ranges of the batch's transactions, block-major (shard by
  // transaction index) -- every device stages the blocks its range touches and parses its rows.
  const bool by_tx = nblocks < W;
  std::vector<size_t> b0(W + 1, nblocks);
  std::vector<uint32_t> lo(W * nblocks, FGV_SHARD_SKIP), hi(W * nblocks, FGV_SHARD_SKIP);
  std::vector<size_t> cap(W, 0), nrec(W, 0);
  if (by_tx) {
    std::vector<size_t> nt(nblocks);
    size_t total = 0;
    for (size_t b = 0; b < nblocks; b++) {
      const long k = fgv_block_count_txs(blocks[b], lens[b]);
      if (k < 0) return FGV_EINVAL;
      nt[b] = (size_t)k;
      total += nt[b];
    }
    for (size_t r = 0; r < W; r++) {
      const size_t a = total * r / W, e = total * (r + 1) / W;
      size_t base = 0;
      for (size_t b = 0; b < nblocks; b++) {
        const size_t x = std::max(a, base), y = std::min(e, base + nt[b]);
        if (x < y) {
          lo[r * nblocks + b] = (uint32_t)(x - base);
          hi[r * nblocks + b] = (uint32_t)(y - base);
          nrec[r] += y - x;
        }
        base += nt[b];
      }
      cap[r] = nrec[r];
    }
  } else {
    size_t total = 0;
    for (size_t b = 0; b < nblocks; b++) total += lens[b];
    b0[0] = 0;
    size_t acc = 0, r = 1;
    for (size_t b = 0; b < nblocks && r < W; b++) {
      acc += lens[b];
      while (r < W && acc * W >= total * r) b0[r++] = b + 1;
    }
    // records per device are bounded by its blocks' bytes (an envelope takes >= 2 bytes) and
    // by flags_cap
    for (size_t q = 0; q < W; q++) {
      size_t bytes = 0;
      for (size_t b = b0[q]; b < b0[q + 1]; b++) bytes += lens[b];
      cap[q] = std::min(flags_cap, bytes / 2 + (b0[q + 1] - b0[q]));
    }
  }
  const size_t capmax = *std::max_element(cap.begin(), cap.end());
  std::vector<int> rcs(W, FGV_OK);
  std::vector<uint32_t> split(W, UINT32_MAX);  // per-block outcomes: each device's first waiting block
  std::vector<std::vector<size_t>> ntx_dev(W, std::vector<size_t>(nblocks, 0));
  g->pool->run(W, [&](size_t r) {
    if (by_tx ? nrec[r] == 0 : b0[r + 1] == b0[r]) return;
    if (hipSetDevice(g->dev[r]) != hipSuccess) {
      rcs[r] = FGV_EDEVICE;
      return;
    }
    // (the RCCL all-gather sends the same row count from every device: room for the largest share)
    if (!g->res[r].ensure((g->coll == FGV_GROUP_COLL_RCCL ? capmax : cap[r]) * sizeof(fgv_tx_result) + 64)) {
      rcs[r] = FGV_ENOMEM;
      return;
    }
    // (an identity this device's registry has not seen is resolved inside, MSP cache miss)
    if (soft && by_tx)
      rcs[r] = fgv_validate_shard_dev_soft(g->ctx[r], nblocks, blocks, lens, &lo[r * nblocks], &hi[r * nblocks],
                                           g->res[r].p, cap[r], ntx_dev[r].data(), &split[r]);
    else if (soft)
      rcs[r] = fgv_validate_shard_dev_soft(g->ctx[r], b0[r + 1] - b0[r], blocks + b0[r], lens + b0[r], nullptr,
                                           nullptr, g->res[r].p, cap[r], ntx + b0[r], &split[r]);
    else if (by_tx)
      rcs[r] = fgv_validate_shard_dev(g->ctx[r], nblocks, blocks, lens, nullptr, &lo[r * nblocks], &hi[r * nblocks],
                                      g->res[r].p, cap[r], ntx_dev[r].data());
    else
      rcs[r] = fgv_validate_shard_dev(g->ctx[r], b0[r + 1] - b0[r], blocks + b0[r], lens + b0[r], nullptr, nullptr,
                                      nullptr, g->res[r].p, cap[r], ntx + b0[r]);
  });
  // the first block that waits for an earlier block's commit (per-block outcomes; global index)
  size_t n_final = nblocks;
  for (size_t r = 0; r < W; r++)
    if (split[r] != UINT32_MAX) n_final = std::min(n_final, (by_tx ? 0 : b0[r]) + (size_t)split[r]);
  int unsup = 0;
  for (int rc : rcs) {
    if (rc == FGV_EUNSUPPORTED) unsup = 1;
    else if (rc) return rc;
  }
  if (unsup) return FGV_EUNSUPPORTED;
  if (by_tx) {
    for (size_t b = 0; b < nblocks; b++) {  // (every device with rows saw the full counts)
      ntx[b] = 0;
      for (size_t r = 0; r < W; r++) ntx[b] = std::max(ntx[b], ntx_dev[r][b]);
    }
  } else {
    // a device whose blocks may change key-level state while a later device's blocks were
    // validated against the state before them (fgv_block_validate_impl's batch rule across devices)
    for (size_t r = 0; r + 1 < W; r++)
      if (b0[r + 1] > b0[r] && b0[r + 1] < nblocks && g->ctx[r]->kl_changes) {
        uint32_t ks = UINT32_MAX;  // (the whole batch, host; soft: the first waiting block)
        const int rc = fgv_block_kl_check(g->ctx[0]->blk, nblocks, blocks, lens, soft ? &ks : nullptr);
        if (rc) return rc;
        if (ks != UINT32_MAX) n_final = std::min(n_final, (size_t)ks);
        break;
      }
    for (size_t r = 0; r < W; r++)
      for (size_t b = b0[r]; b < b0[r + 1]; b++) {
        lo[r * nblocks + b] = 0;
        hi[r * nblocks + b] = (uint32_t)ntx[b];
        nrec[r] += ntx[b];
      }
  }
  size_t all = 0, rows = 0;
  for (size_t r = 0; r < W; r++) {
    rows = std::max(rows, nrec[r]);
    all += nrec[r];
  }
  if (all > flags_cap) return FGV_EINVAL;
  if (all == 0) {
    if (soft) {
      g->blk_status.assign(nblocks, FGV_OK);
      g->n_final = n_final;
      for (size_t b = n_final; b < nblocks; b++) g->blk_status[b] = FGV_BLOCK_LATER;
    }
    return FGV_OK;
  }
  if (g->coll == FGV_GROUP_COLL_RCCL) {
    // ncclAllGather of every device's rows (68 B records, rank r's at r x rows, the
    // layout fabric_amd/shard.py's all-gather makes) into every device's HBM over xGMI, then the
    // finalize on every device -- each holds the batch's final flags; device 0's go to the caller
    // and the others' are checked equal to them
    std::vector<int> grc(W, FGV_OK);
    g->pool->run(W, [&](size_t r) {
      if (hipSetDevice(g->dev[r]) != hipSuccess) { grc[r] = FGV_EDEVICE; return; }
      if (g->res[r].cap < rows * sizeof(fgv_tx_result) || !g->gathr[r].ensure(W * rows * sizeof(fgv_tx_result) + 64))
        grc[r] = FGV_ENOMEM;
    });
    for (int rc : grc)
      if (rc) return rc;
    if (rccl().group_start() != ncclSuccess) return FGV_EDEVICE;
    ncclResult_t nr = ncclSuccess;
    for (size_t r = 0; r < W && nr == ncclSuccess; r++) {
      if (hipSetDevice(g->dev[r]) != hipSuccess) { nr = ncclInvalidUsage; break; }
      nr = rccl().all_gather(g->res[r].p, g->gathr[r].p, rows * sizeof(fgv_tx_result), ncclUint8, g->comms[r], g->cs[r]);
    }
    if (rccl().group_end() != ncclSuccess || nr != ncclSuccess) return FGV_EDEVICE;
    g->dflags.resize(W);
    for (size_t r = 1; r < W; r++) g->dflags[r].resize(all);
    g->pool->run(W, [&](size_t r) {
      if (hipSetDevice(g->dev[r]) != hipSuccess || hipStreamSynchronize(g->cs[r]) != hipSuccess) {
        grc[r] = FGV_EDEVICE;
        return;
      }
      grc[r] = fgv_finalize_flags_dev_plan(g->ctx[r], nblocks, ntx, (uint32_t)W, rows, lo.data(), hi.data(),
                                           g->gathr[r].p, r == 0 ? flags : g->dflags[r].data());
    });
    for (int rc : grc)
      if (rc) return rc;
    for (size_t r = 1; r < W; r++)
      if (memcmp(g->dflags[r].data(), flags, all) != 0) return FGV_EDEVICE;  // (devices disagree)
    return group_outcomes(g, nblocks, ntx, flags, soft, n_final);
  }
  // gather onto device 0 (rank r's rows at r x rows), then the finalize there
  if (hipSetDevice(g->dev[0]) != hipSuccess) return FGV_EDEVICE;
  if (!g->gath.ensure(W * rows * sizeof(fgv_tx_result) + 64)) return FGV_ENOMEM;
  uint8_t *dst = g->gath.as<uint8_t>();
  for (size_t r = 0; r < W; r++) {
    if (!nrec[r]) continue;
    HIP_TRY(hipMemcpyPeerAsync(dst + r * rows * sizeof(fgv_tx_result), g->dev[0], g->res[r].p, g->dev[r],
                               nrec[r] * sizeof(fgv_tx_result), g->s0));
  }
  HIP_TRY(hipStreamSynchronize(g->s0));
  const int rc = fgv_finalize_flags_dev_plan(g->ctx[0], nblocks, ntx, (uint32_t)W, rows, lo.data(), hi.data(), dst,
                                             flags);
  if (rc) return rc;
  return group_outcomes(g, nblocks, ntx, flags, soft, n_final);
}

static int group_outcomes(fgv_group *g, size_t nblocks, const size_t *ntx, const uint8_t *flags, bool soft,
                          size_t n_final) {
  if (!soft) return FGV_OK;
  // per-block outcomes (fgv_last_block_status's rules): blocks from n_final on wait; a block with
  // an undecided transaction (0xFD) goes to the reference; the others are final
  g->blk_status.assign(nblocks, FGV_OK);
  g->n_final = n_final;
  size_t o = 0;
  for (size_t b = 0; b < nblocks; o += ntx[b], b++) {
    if (b >= n_final) {
      g->blk_status[b] = FGV_BLOCK_LATER;
      continue;
    }
    for (size_t t = 0; t < ntx[b]; t++)
      if (flags[o + t] == 0xFD) {
        g->blk_status[b] = FGV_EUNSUPPORTED;
        break;
      }
  }
  return FGV_OK;
}

int fgv_group_set_block_outcomes(fgv_group *g, int on) {
  if (!g) return FGV_EINVAL;
  std::lock_guard<std::mutex> lk(g->mu);
  g->soft = on != 0;
  return FGV_OK;
}

int fgv_group_last_block_status(fgv_group *g, int32_t *status, size_t n, size_t *n_final) {
  if (!g || (n && !status)) return FGV_EINVAL;
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->last_rc != FGV_OK) {  // a failed call decided nothing
    for (size_t b = 0; b < n; b++) status[b] = g->last_rc;
    if (n_final) *n_final = 0;
    return g->last_rc;
  }
  for (size_t b = 0; b < n; b++) status[b] = b < g->blk_status.size() ? g->blk_status[b] : FGV_OK;
  if (n_final) *n_final = g->n_final;
  return FGV_OK;
}

int fgv_group_p256_verify_msgs(fgv_group *g, const uint8_t *keys, const uint8_t *msg_buf, size_t msg_buf_len,
                               const uint64_t *msg_off, const uint32_t *msg_len, const uint8_t *sig_buf,
                               size_t sig_buf_len, const uint64_t *sig_off, const uint32_t *sig_len, size_t n,
                               uint8_t *status) {
  if (!g || (n && (!keys || !msg_buf || !msg_off || !msg_len || !sig_buf || !sig_off || !sig_len || !status)))
    return FGV_EINVAL;
  if (n == 0) return FGV_OK;
  std::lock_guard<std::mutex> lk(g->mu);
  const size_t W = g->ctx.size();
  std::vector<int> rcs(W, FGV_OK);
  // item ranges [n r / W, n (r+1) / W); each device gets the byte spans its items reference
  // (rebased offsets), verifies them with its own key cache and writes its slice of `status`
  g->pool->run(W, [&](size_t r) {
    const size_t a = n * r / W, e = n * (r + 1) / W;
    if (a == e) return;
    uint64_t m0 = UINT64_MAX, m1 = 0, s0 = UINT64_MAX, s1 = 0;
    for (size_t i = a; i < e; i++) {
      if (msg_off[i] + msg_len[i] > msg_buf_len || sig_off[i] + sig_len[i] > sig_buf_len) {
        rcs[r] = FGV_EINVAL;
        return;
      }
      m0 = std::min<uint64_t>(m0, msg_off[i]);
      m1 = std::max<uint64_t>(m1, msg_off[i] + msg_len[i]);
      s0 = std::min<uint64_t>(s0, sig_off[i]);
      s1 = std::max<uint64_t>(s1, sig_off[i] + sig_len[i]);
    }
    std::vector<uint64_t> mo(e - a), so(e - a);
    for (size_t i = a; i < e; i++) {
      mo[i - a] = msg_off[i] - m0;
      so[i - a] = sig_off[i] - s0;
    }
    rcs[r] = fgv_p256_verify_msgs(g->ctx[r], keys + 64 * a, msg_buf + m0, m1 - m0, mo.data(), msg_len + a,
                                  sig_buf + s0, s1 - s0, so.data(), sig_len + a, e - a, status + a);
  });
  for (int rc : rcs)
    if (rc) return rc;
  return FGV_OK;
}

}  // extern "C"
