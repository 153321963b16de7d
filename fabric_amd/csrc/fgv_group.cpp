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
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <vector>

#include "fgv_internal.h"
#include "thread_pool.h"

struct fgv_group {
  std::vector<fgv_ctx *> ctx;
  std::vector<int> dev;
  std::vector<DevBuf> res;  // per device: its shard's records (allocated on that device)
  DevBuf gath;              // on device 0: world x rows records
  hipStream_t s0 = nullptr; // device 0: the gather copies
  ThreadPool *pool = nullptr;
  std::mutex mu;
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

void fgv_group_destroy(fgv_group *g) {
  if (!g) return;
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

int fgv_group_validate_blocks(fgv_group *g, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                              uint8_t *flags, size_t flags_cap, size_t *ntx) {
  if (!g || (nblocks && (!blocks || !lens || !flags || !ntx))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> lk(g->mu);
  const size_t W = g->ctx.size();
  // the block plan: contiguous ranges of about total/W bytes (a device may get none)
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) total += lens[b];
  std::vector<size_t> b0(W + 1, nblocks);
  b0[0] = 0;
  {
    size_t acc = 0, r = 1;
    for (size_t b = 0; b < nblocks && r < W; b++) {
      acc += lens[b];
      while (r < W && acc * W >= total * r) b0[r++] = b + 1;
    }
  }
  // records per device are bounded by its blocks' bytes (an envelope takes >= 2 bytes) and
  // by flags_cap
  std::vector<size_t> cap(W, 0);
  for (size_t r = 0; r < W; r++) {
    size_t bytes = 0;
    for (size_t b = b0[r]; b < b0[r + 1]; b++) bytes += lens[b];
    cap[r] = std::min(flags_cap, bytes / 2 + (b0[r + 1] - b0[r]));
  }
  std::vector<int> rcs(W, FGV_OK);
  g->pool->run(W, [&](size_t r) {
    const size_t nb = b0[r + 1] - b0[r];
    if (nb == 0) return;
    if (hipSetDevice(g->dev[r]) != hipSuccess) {
      rcs[r] = FGV_EDEVICE;
      return;
    }
    if (!g->res[r].ensure(cap[r] * sizeof(fgv_tx_result) + 64)) {
      rcs[r] = FGV_ENOMEM;
      return;
    }
    // (an identity this device's registry has not seen is resolved inside, MSP cache miss)
    rcs[r] = fgv_validate_shard_dev(g->ctx[r], nb, blocks + b0[r], lens + b0[r], nullptr, nullptr, nullptr,
                                    g->res[r].p, cap[r], ntx + b0[r]);
  });
  int unsup = 0;
  for (int rc : rcs) {
    if (rc == FGV_EUNSUPPORTED) unsup = 1;
    else if (rc) return rc;
  }
  if (unsup) return FGV_EUNSUPPORTED;
  // a device whose blocks may change key-level state while a later device's blocks were
  // validated against the state before them (fgv_block_validate_impl's batch rule across devices)
  for (size_t r = 0; r + 1 < W; r++)
    if (b0[r + 1] > b0[r] && b0[r + 1] < nblocks && g->ctx[r]->kl_changes) {
      const int rc = fgv_block_kl_check(g->ctx[0]->blk, nblocks, blocks, lens);  // (the whole batch, host)
      if (rc) return rc;
      break;
    }
  size_t all = 0, rows = 0;
  std::vector<size_t> nrec(W, 0);
  for (size_t r = 0; r < W; r++) {
    for (size_t b = b0[r]; b < b0[r + 1]; b++) nrec[r] += ntx[b];
    rows = std::max(rows, nrec[r]);
    all += nrec[r];
  }
  if (all > flags_cap) return FGV_EINVAL;
  if (all == 0) return FGV_OK;
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
  std::vector<uint32_t> lo(W * nblocks, FGV_SHARD_SKIP), hi(W * nblocks, FGV_SHARD_SKIP);
  for (size_t r = 0; r < W; r++)
    for (size_t b = b0[r]; b < b0[r + 1]; b++) {
      lo[r * nblocks + b] = 0;
      hi[r * nblocks + b] = (uint32_t)ntx[b];
    }
  return fgv_finalize_flags_dev_plan(g->ctx[0], nblocks, ntx, (uint32_t)W, rows, lo.data(), hi.data(), dst, flags);
}

}  // extern "C"
