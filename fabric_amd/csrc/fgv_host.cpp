// fgv_host.cpp -- host side of libfgv.so: context, device buffers, key-table cache and
// the BCCSP-shaped batch entry points of include/fgv.h.
//
// Data flow for one verify batch (all device work on ctx->stream):
//   host: Go-rule DER decode + low-S (fgv_der.h), key -> table slot (cache), SoA packing
//   H2D:  status/slot (5 B/item), r,s limbs (64 B/item) [+ digests or message arena]
//   dev:  [k_keytab for keys not yet cached] -> [k_sha256] -> k_prep -> k_point
//   D2H:  status (1 B/item)
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <unordered_map>
#include <vector>

#include "../../include/fgv.h"
#include "fgv_der.h"
#include "fgv_internal.h"
#include "fgv_kernels.h"

static void stats_accumulate(fgv_ctx *c);

// ======================================================================= key tiers
// DESIGN.md s4a.  Every P-256 key the engine verifies against has an id.  Registered keys
// (fgv_keys_register, channel identities, MSP CA keys) hold ids [0, pinned) for good; ad-hoc
// BCCSP keys (fgv_p256_verify_batch / _msgs) take ids after them until the id space is flushed.
// Each id's verifies run on one of two kernel paths:
//   comb -- kmap[id] = a slot of the comb-table cache (5.2 MB per key, built by k_keytab: ~80 us
//           of whole-chip time per key, batched 32 keys per launch): k_point28, 32 mixed
//           additions per verify;
//   VB   -- kmap[id] = KEY_NONE: k_vb_mul / k_vb_fin from the key's coordinates alone (64 B,
//           k_keyprep): 256 doublings + <= 64 additions for u2 * Q, ~9x a comb verify, no build.
// Policy: a key expected to be hot -- fgv_keys_register, an identity with a PEER / ORDERER / ADMIN
// role or unknown roles, an MSP CA key, an ad-hoc key used >= adhoc_comb_uses times in its call --
// takes a comb slot while one is free.  Every other key (client identities, one-off ad-hoc keys)
// starts on VB; k_vb_mul counts its verifies and queues it once they reach promote_uses, and the
// next call builds its comb in a free slot (promote_consume).  A full comb cache never fails a
// batch: the keys stay on VB.  Only the id space (fgv_config.key_ids) can run out.

// Build comb tables for `nk` keys (h_qxy: nk*16 plain limbs) into `tables28` at `h_slots`,
// KT_BUILD_KEYS keys per k_keytab launch (its scratch is KT_ENTRIES Jacobian points per key).
static int build_tables(fgv_ctx *c, const uint32_t *h_qxy, const uint32_t *h_slots, uint32_t nk,
                        apoint_raw *tables, apoint_raw *tables28, uint8_t *ok, hipStream_t st = nullptr) {
  const bool timed = st == nullptr;
  if (!st) st = c->stream;
  const uint32_t per = nk < KT_BUILD_KEYS ? nk : KT_BUILD_KEYS;
  // the scratch at its full size on first use (335 MB): grown build by build, every larger
  // promotion batch would pay a hipFree -- a device-wide synchronisation -- inside a call
  if (!c->kt_q.ensure((size_t)nk * 64) || !c->kt_slot.ensure((size_t)nk * 4) ||
      !c->kt_scratch.ensure((size_t)KT_BUILD_KEYS * KT_ENTRIES * sizeof(jpoint_raw)) ||
      !c->kt_base.ensure((size_t)KT_BUILD_KEYS * NWIN * sizeof(jpoint_raw)))
    return FGV_ENOMEM;
  HIP_TRY(hipMemcpyAsync(c->kt_q.p, h_qxy, (size_t)nk * 64, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(c->kt_slot.p, h_slots, (size_t)nk * 4, hipMemcpyHostToDevice, st));
  if (timed) HIP_TRY(hipEventRecord(c->ev[6], st));
  for (uint32_t k = 0; k < nk; k += per) {
    const uint32_t m = nk - k < per ? nk - k : per;
    const uint32_t threads = m * KT_THREADS_PER_KEY;
    hipLaunchKernelGGL(k_keybase, dim3((m * NWIN + 63) / 64), dim3(64), 0, st, c->kt_q.as<uint32_t>() + 16 * k, m,
                       c->kt_base.as<jpoint_raw>());
    hipLaunchKernelGGL(k_keytab, dim3((threads + 63) / 64), dim3(64), 0, st, c->kt_q.as<uint32_t>() + 16 * k,
                       c->kt_slot.as<uint32_t>() + k, tables, tables28, c->kt_scratch.as<jpoint_raw>(), ok, m,
                       c->kt_base.as<const jpoint_raw>());
    HIP_TRY(hipGetLastError());
  }
  if (timed) HIP_TRY(hipEventRecord(c->ev[7], st));
  return FGV_OK;
}

// comb tables for ids that have none (taken in order while comb slots are free; the rest stay on
// VB).  Synchronises the stream (the staging buffers are reused by the next build).
// The staging buffers of an asynchronous build (streamK) are free again.
static int kt_wait(fgv_ctx *c) {
  if (!c->kt_busy) return FGV_OK;
  HIP_TRY(hipEventSynchronize(c->kt_ev));
  c->kt_busy = false;
  return FGV_OK;
}

static int comb_build(fgv_ctx *c, const std::vector<uint32_t> &ids, bool async = false) {
  int wrc = kt_wait(c);
  if (wrc) return wrc;
  // (distinct ids: a key named twice must not take two slots nor count twice against n_vb)
  std::vector<uint32_t> uniq(ids);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  std::vector<uint32_t> take;
  for (uint32_t id : uniq)
    if (take.size() < c->comb_free.size() && id < c->n_ids && c->kmap_h[id] == KEY_NONE) take.push_back(id);
  if (take.empty()) return FGV_OK;
  const uint32_t nk = (uint32_t)take.size();
  if (!c->h_kq.ensure((size_t)nk * 64) || !c->h_kslot.ensure((size_t)nk * 4) || !c->h_kid.ensure((size_t)nk * 4) ||
      !c->kt_id.ensure((size_t)nk * 4))
    return FGV_ENOMEM;
  uint32_t *kq = c->h_kq.as<uint32_t>(), *ks = c->h_kslot.as<uint32_t>(), *ki = c->h_kid.as<uint32_t>();
  for (uint32_t j = 0; j < nk; j++) {
    const uint32_t id = take[j], slot = c->comb_free.back();
    c->comb_free.pop_back();
    c->comb_owner[slot] = id;
    c->kmap_h[id] = slot;
    c->n_vb--;
    be32_to_limbs(c->id_key[id].data(), kq + 16 * j);
    be32_to_limbs(c->id_key[id].data() + 32, kq + 16 * j + 8);
    ks[j] = slot;
    ki[j] = id;
  }
  if (async && c->promote_at) {  // (test knob: the table now, k_kmap_set at a chosen point later)
    int rc = build_tables(c, kq, ks, nk, nullptr, c->ktab28.as<apoint_raw>(), nullptr, c->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->kt_id.p, ki, (size_t)nk * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->kmap_defer = nk;
    return FGV_OK;
  }
  // async (promotions): on streamK, nobody waits.  A kernel that reads kmap while the build is in
  // flight sees KEY_NONE (variable-base path) or the slot once the table is complete (k_kmap_set
  // runs after k_keytab): kmap only goes from KEY_NONE to a slot outside a flush, and both paths
  // give the same status, so a batch may even see the change between k_inv and k_point28
  hipStream_t st = async ? c->streamK : c->stream;
  int rc = build_tables(c, kq, ks, nk, nullptr, c->ktab28.as<apoint_raw>(), nullptr, async ? st : nullptr);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->kt_id.p, ki, (size_t)nk * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_kmap_set, dim3((nk + 63) / 64), dim3(64), 0, st, c->kt_id.as<uint32_t>(),
                     c->kt_slot.as<uint32_t>(), nk, c->kmap.as<uint32_t>());
  HIP_TRY(hipGetLastError());
  if (async) {
    HIP_TRY(hipEventRecord(c->kt_ev, st));
    c->kt_busy = true;
    return FGV_OK;
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[6], c->ev[7]) == hipSuccess) c->t_keytab += ms;
  return FGV_OK;
}

// FGV_PROMOTE_AT: the deferred k_kmap_set of a promotion, enqueued on `st` at chain point
// `point` (1 after k_inv, 2 before k_point28, 3 before k_vb_fin; 0 whatever the point)
static int kmap_defer_flush(fgv_ctx *c, hipStream_t st, uint32_t point) {
  if (!c->kmap_defer || (point && point != c->promote_at)) return FGV_OK;
  hipLaunchKernelGGL(k_kmap_set, dim3((c->kmap_defer + 63) / 64), dim3(64), 0, st, c->kt_id.as<uint32_t>(),
                     c->kt_slot.as<uint32_t>(), c->kmap_defer, c->kmap.as<uint32_t>());
  c->kmap_defer = 0;
  HIP_TRY(hipGetLastError());
  return FGV_OK;
}

// forget the ad-hoc ids [pinned, n_ids): their comb slots go back to the free list
static int flush_adhoc(fgv_ctx *c) {
  if (c->n_ids == c->pinned) return FGV_OK;
  int wrc = kt_wait(c);  // (a promotion's k_kmap_set must land before the reset below)
  if (wrc) return wrc;
  wrc = kmap_defer_flush(c, c->stream, 0);
  if (wrc) return wrc;
  for (uint32_t id = c->pinned; id < c->n_ids; id++) {
    c->key_map.erase(c->id_key[id]);
    const uint32_t slot = c->kmap_h[id];
    if (slot == KEY_NONE) {
      c->n_vb--;
    } else {
      c->comb_owner[slot] = KEY_NONE;
      c->comb_free.push_back(slot);
      c->kmap_h[id] = KEY_NONE;
    }
  }
  const size_t k = c->n_ids - c->pinned;
  c->promo_backlog.erase(std::remove_if(c->promo_backlog.begin(), c->promo_backlog.end(),
                                        [c](uint32_t id) { return id >= c->pinned; }),
                         c->promo_backlog.end());
  HIP_TRY(hipMemsetAsync(c->kmap.as<uint32_t>() + c->pinned, 0xFF, k * 4, c->stream));
  HIP_TRY(hipMemsetAsync(c->vbuse.as<uint32_t>() + c->pinned, 0, k * 4, c->stream));
  c->n_ids = c->pinned;
  c->id_key.resize(c->n_ids);
  return FGV_OK;
}

// ids for `keys` (distinct, none known yet): coordinates and on-curve bits on the device
// (k_keyprep), then comb tables for those with want[i] (nullable: all) while slots are free.
// Synchronises the stream.
static int ids_new(fgv_ctx *c, const std::vector<std::array<uint8_t, 64>> &keys, const std::vector<uint8_t> *want,
                   uint32_t *ids_out) {
  int wrc = kt_wait(c);  // (the staging buffers below)
  if (wrc) return wrc;
  const uint32_t nk = (uint32_t)keys.size();
  if (nk == 0) return FGV_OK;
  if ((uint64_t)c->n_ids + nk > c->key_ids) return FGV_ENOMEM;
  if (!c->h_kq.ensure((size_t)nk * 64) || !c->h_kid.ensure((size_t)nk * 4) || !c->kt_q.ensure((size_t)nk * 64) ||
      !c->kt_id.ensure((size_t)nk * 4))
    return FGV_ENOMEM;
  // the variable-base tables (60 KB per id) grow by doubling; kernels in flight read the old rows
  if (c->n_ids + nk > c->vbt_keys) {
    const uint32_t want = std::min<uint32_t>(c->key_ids, std::max<uint32_t>({c->n_ids + nk, 2 * c->vbt_keys, 4096u}));
    uint32_t grow = want;
    DevBuf nb;
    if (!nb.ensure((size_t)grow * VBT_WORDS * 4)) {  // (no room to double: exactly what is needed)
      grow = c->n_ids + nk;
      if (!nb.ensure((size_t)grow * VBT_WORDS * 4)) return FGV_ENOMEM;
    }
    HIP_TRY(hipStreamSynchronize(c->streamV));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->vbt_keys) HIP_TRY(hipMemcpy(nb.p, c->vbt.p, (size_t)c->vbt_keys * VBT_WORDS * 4, hipMemcpyDeviceToDevice));
    c->vbt.release();
    c->vbt = nb;
    nb.p = nullptr;
    c->vbt_keys = grow;
  }
  uint32_t *kq = c->h_kq.as<uint32_t>(), *ki = c->h_kid.as<uint32_t>();
  std::vector<uint32_t> comb;
  for (uint32_t j = 0; j < nk; j++) {
    const uint32_t id = c->n_ids++;
    c->key_map.emplace(keys[j], id);
    c->id_key.push_back(keys[j]);
    c->kmap_h[id] = KEY_NONE;
    c->n_vb++;
    be32_to_limbs(keys[j].data(), kq + 16 * j);
    be32_to_limbs(keys[j].data() + 32, kq + 16 * j + 8);
    ki[j] = id;
    ids_out[j] = id;
    if (!want || (*want)[j]) comb.push_back(id);
  }
  HIP_TRY(hipMemcpyAsync(c->kt_q.p, kq, (size_t)nk * 64, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->kt_id.p, ki, (size_t)nk * 4, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_keyprep, dim3((nk * VB_WINS + 63) / 64), dim3(64), 0, c->stream, c->kt_q.as<uint32_t>(),
                     c->kt_id.as<uint32_t>(), nk, c->vbt.as<uint32_t>(), c->key_ok.as<uint8_t>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));  // (the staging is reused by comb_build)
  return comb_build(c, comb);
}

// The promotion queue k_vb_mul filled (copied back on streamV behind it): build combs for the
// queued ids, then empty the queue on the device.  At the start of a call, under c->mu; a copy
// still in flight is left for the next call.
// `st`: the stream this call's k_inv runs on -- the queue's reset is ordered before the k_vb_mul
// that follows it (that kernel waits for an event recorded on `st` after k_inv)
static int promote_consume(fgv_ctx *c, uint32_t items, hipStream_t st) {
  if (c->vb_copied && hipEventQuery(c->vb_ev[2]) == hipSuccess) {  // (a copy in flight: a later call)
    c->vb_copied = false;
    uint32_t *q = c->h_promo.as<uint32_t>();
    c->vb_last_items = q[1];
    const uint32_t np = std::min<uint32_t>(q[0], VB_PROMO_CAP);
    if (np) {
      c->promo_backlog.insert(c->promo_backlog.end(), q + 2, q + 2 + np);
      q[0] = 0;
      HIP_TRY(hipMemsetAsync(c->vbpromo.p, 0, 4, st));
    }
  }
  // a full comb cache keeps the queue (bounded, distinct ids) for slots a flush frees later:
  // k_vb_mul queues a key once, when its count reaches the threshold
  if (c->comb_free.empty()) {
    if (c->promo_backlog.size() > VB_BACKLOG_CAP) {
      std::sort(c->promo_backlog.begin(), c->promo_backlog.end());
      c->promo_backlog.erase(std::unique(c->promo_backlog.begin(), c->promo_backlog.end()), c->promo_backlog.end());
      if (c->promo_backlog.size() > VB_BACKLOG_CAP) c->promo_backlog.resize(VB_BACKLOG_CAP);
    }
    return FGV_OK;
  }
  if (c->promo_backlog.empty()) return FGV_OK;
  // the previous builds still running: leave the queue for a later call (never block the host)
  if (c->kt_busy) {
    if (hipEventQuery(c->kt_ev) != hipSuccess) return FGV_OK;
    c->kt_busy = false;
  }
  // at most promote_per_call builds per call, and about one per 24,000 verify slots of this call (a
  // 17-bit comb is 64 MiB: ~8x a 13-bit one's build, round 6), so a burst of keys reaching the
  // threshold together spreads over calls, and a small call (one block) is not swamped by builds
  // running beside it (FGV_PROMOTE_PER_CALL set: exactly that many, whatever the call's size)
  const size_t per = c->promote_fixed ? c->promote_per_call
                                      : std::max<size_t>(1, std::min<size_t>(c->promote_per_call, items / 24000));
  const size_t take = std::min<size_t>(c->promo_backlog.size(), per);
  std::vector<uint32_t> ids(c->promo_backlog.begin(), c->promo_backlog.begin() + take);
  c->promo_backlog.erase(c->promo_backlog.begin(), c->promo_backlog.begin() + take);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  const uint32_t before = (uint32_t)c->comb_free.size();
  int rc = comb_build(c, ids, true);
  c->n_promoted += before - c->comb_free.size();
  return rc;
}

extern "C" {

const char *fgv_strerror(int code) {
  switch (code) {
    case FGV_OK: return "ok";
    case FGV_EINVAL: return "invalid argument";
    case FGV_EDEVICE: return "HIP device error";
    case FGV_ENOMEM: return "out of memory";
    case FGV_ECOMM: return "communication error";
    case FGV_ESTATE: return "invalid state";
    default: return "unknown error";
  }
}

int fgv_init(const fgv_config *cfg, fgv_ctx **out) {
  if (!out) return FGV_EINVAL;
  *out = nullptr;
  fgv_ctx *c = new (std::nothrow) fgv_ctx();
  if (!c) return FGV_ENOMEM;
  c->device = cfg ? cfg->device : 0;
  c->key_slots = (cfg && cfg->key_slots) ? cfg->key_slots : 256;  // x 64 MiB (KT_BYTES): 16 GiB of comb tables
  c->key_ids = (cfg && cfg->key_ids) ? cfg->key_ids : (1u << 20);
  if (const char *e = getenv("FGV_PROMOTE_USES")) c->promote_uses = (uint32_t)std::max(1, atoi(e));
  if (const char *e = getenv("FGV_ADHOC_COMB")) c->adhoc_comb_uses = (uint32_t)std::max(1, atoi(e));
  if (const char *e = getenv("FGV_PROMOTE_AT")) c->promote_at = (uint32_t)std::max(0, std::min(3, atoi(e)));
  if (const char *e = getenv("FGV_PROMOTE_PER_CALL")) {
    c->promote_per_call = (uint32_t)std::max(1, atoi(e));
    c->promote_fixed = true;
  }
  // host workers: fgv_config.host_threads, else min(24, this process's CPU share) -- 24 measured
  // best on a whole machine (tools/sweep_threads.sh); eight ranks on one node each get their
  // affinity mask's share, not the whole machine
  unsigned share = 0;
  {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) share = (unsigned)CPU_COUNT(&cs);
    if (const char *e = getenv("OMP_NUM_THREADS")) {
      const int v = atoi(e);
      if (v > 0 && (share == 0 || (unsigned)v < share)) share = (unsigned)v;
    }
  }
  const unsigned dflt = share ? std::min(24u, share) : 24u;
  c->blk = fgv_block_state_new((cfg && cfg->host_threads) ? cfg->host_threads : dflt);
  if (const char *e = getenv("FGV_AHEAD")) c->ahead_mode = std::max(0, std::min(4, atoi(e)));
  if (const char *e = getenv("FGV_TIMING")) c->timing = atoi(e) != 0;
  if (const char *e = getenv("FGV_SPIN")) c->spin = atoi(e) != 0;
  auto fail = [&](int e) {
    fgv_destroy(c);
    return e;
  };
  if (hipSetDevice(c->device) != hipSuccess) return fail(FGV_EDEVICE);
  // the main stream carries the latency-critical chain (parse -> identities -> verify jobs ->
  // k_point) at high priority; stream2 fills the rest of the chip with SHA-256 / k_inv.
  // Creation order matters: HIP shares the least-used hardware queue once GPU_MAX_HW_QUEUES (4)
  // queues of a priority exist, and (as we read the traces) the process's first stream holds one.  streamF (the
  // next batch's parse / identities / counts) comes before the copy stream so that it gets a queue
  // of its own: created after it, it shared the first stream's queue and the C2 step measured
  // 0.63-0.65 ms instead of 0.55-0.58 (MI355X).  streamK (comb builds) is
  // CU-masked: a queue of its own.
  {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi) != hipSuccess) return fail(FGV_EDEVICE);
    // FGV_FRONT_RESERVE=k (A/B): the front-half streams (payload, k_bd_sha, parse / identities)
    // leave k CUs per XCD to the main stream, so the back half's short kernels (k_point, fold,
    // dups, emit ...) find CUs while the next batch's front half holds the rest.  CUs 33 x + 8 j
    // (x < 8, j < k): k per XCD whether CU ids run XCD-major or round-robin over the XCDs.
    static const int reserve = [] {
      const char *e = getenv("FGV_FRONT_RESERVE");
      const int v = e ? atoi(e) : 0;
      return v >= 0 && v <= 3 ? v : 0;
    }();
    int ncu0 = 0;
    if (reserve && hipDeviceGetAttribute(&ncu0, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess &&
        ncu0 == 256) {
      uint32_t mask[8];
      for (auto &m : mask) m = 0xFFFFFFFFu;
      for (int x = 0; x < 8; x++)
        for (int j = 0; j < reserve; j++) {
          const int cu = 33 * x + 8 * j;
          mask[cu / 32] &= ~(1u << (cu % 32));
        }
      for (hipStream_t *sp : {&c->stream2, &c->stream3, &c->streamF})
        if (hipExtStreamCreateWithCUMask(sp, 8, mask) != hipSuccess) return fail(FGV_EDEVICE);
    } else {
      if (hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, lo) != hipSuccess) return fail(FGV_EDEVICE);
      if (hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, lo) != hipSuccess) return fail(FGV_EDEVICE);
      if (hipStreamCreateWithPriority(&c->streamF, hipStreamNonBlocking, lo) != hipSuccess) return fail(FGV_EDEVICE);
    }
    if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) return fail(FGV_EDEVICE);
    if (hipStreamCreateWithPriority(&c->streamV, hipStreamNonBlocking, lo) != hipSuccess) return fail(FGV_EDEVICE);
    // streamK (promotion comb builds: one k_keytab launch runs ~2-3 ms whatever its key count)
    // on a CU-masked queue of its own -- CUs i with i % 8 == 7 by default (FGV_KT_CUS=0: an
    // ordinary stream): on a shared hardware queue a build held up every kernel queued behind it
    // (C2 churn 1.90 ms per step with promotions against 0.97 without, r4y)
    static const int kt_cus = [] {
      const char *e = getenv("FGV_KT_CUS");
      return e ? atoi(e) : 1;
    }();
    int ncu_k = 0;
    if (kt_cus && hipDeviceGetAttribute(&ncu_k, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess &&
        ncu_k > 0 && ncu_k % 32 == 0) {
      std::vector<uint32_t> mask((size_t)ncu_k / 32, 0u);
      for (int i = 7; i < ncu_k; i += 8) mask[(size_t)i / 32] |= 1u << (i % 32);
      if (hipExtStreamCreateWithCUMask(&c->streamK, (uint32_t)mask.size(), mask.data()) != hipSuccess)
        return fail(FGV_EDEVICE);
    } else if (hipStreamCreateWithPriority(&c->streamK, hipStreamNonBlocking, lo) != hipSuccess) {
      return fail(FGV_EDEVICE);
    }
    if (hipEventCreateWithFlags(&c->kt_ev, hipEventDisableTiming) != hipSuccess) return fail(FGV_EDEVICE);
  }
  for (auto &e : c->vb_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(FGV_EDEVICE);
  for (auto &e : c->vb_t)
    if (hipEventCreate(&e) != hipSuccess) return fail(FGV_EDEVICE);
  for (auto &e : c->stage_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(FGV_EDEVICE);
  {
    std::random_device rd;  // per-context hash seed of the finalize txid table
    c->fin_seed = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)(uintptr_t)c;
  }
  for (auto &e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(FGV_EDEVICE);
  for (auto &e : c->kev)
    if (hipEventCreate(&e) != hipSuccess) return fail(FGV_EDEVICE);
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || ncu <= 0)
      return fail(FGV_EDEVICE);
    c->n_cu = (uint32_t)ncu;
  }
  if (!c->g_ok.ensure(16) || !c->gtab28.ensure(GT_BYTES) || !c->redo.ensure(64) ||
      !c->ktab28.ensure((size_t)c->key_slots * KT_BYTES) || !c->key_ok.ensure(c->key_ids) ||
      !c->kmap.ensure((size_t)c->key_ids * 4) ||
      !c->vbuse.ensure((size_t)c->key_ids * 4) || !c->vbpromo.ensure((VB_PROMO_CAP + 2) * 4) ||
      !c->h_promo.ensure((VB_PROMO_CAP + 2) * 4))
    return fail(FGV_ENOMEM);
  // key tiers: every id starts without a comb; comb slots free, taken from slot 0 up
  c->kmap_h.assign(c->key_ids, KEY_NONE);
  c->comb_owner.assign(c->key_slots, KEY_NONE);
  c->comb_free.resize(c->key_slots);
  for (uint32_t k = 0; k < c->key_slots; k++) c->comb_free[k] = c->key_slots - 1 - k;
  memset(c->h_promo.p, 0, (VB_PROMO_CAP + 2) * 4);
  if (hipMemset(c->redo.p, 0, 64) != hipSuccess || hipMemset(c->kmap.p, 0xFF, (size_t)c->key_ids * 4) != hipSuccess ||
      hipMemset(c->vbuse.p, 0, (size_t)c->key_ids * 4) != hipSuccess ||
      hipMemset(c->vbpromo.p, 0, (VB_PROMO_CAP + 2) * 4) != hipSuccess ||
      hipMemset(c->key_ok.p, 0, c->key_ids) != hipSuccess)
    return fail(FGV_EDEVICE);
  // generator comb table (k_gtab), built once per context
  {
    DevBuf scr;
    if (!scr.ensure((size_t)GT_THREADS_PER_WIN * GT_CHUNK * sizeof(jpoint_raw))) return fail(FGV_ENOMEM);
    bool ok = true;
    for (uint32_t w = 0; w < NGWIN && ok; w++) {  // one window per launch (the scratch holds one)
      hipLaunchKernelGGL(k_gtab, dim3((GT_THREADS_PER_WIN + 63) / 64), dim3(64), 0, c->stream,
                         c->gtab28.as<apoint_raw>(), scr.as<jpoint_raw>(), w);
      ok = hipGetLastError() == hipSuccess;
    }
    ok = ok && hipStreamSynchronize(c->stream) == hipSuccess;
    scr.release();
    if (!ok) return fail(FGV_EDEVICE);
  }
  *out = c;
  return FGV_OK;
}

void fgv_destroy(fgv_ctx *c) {
  if (!c) return;
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  for (hipStream_t x : {c->stream2, c->stream3, c->streamF, c->streamV, c->streamK})  // (a front half enqueued ahead)
    if (x) hipStreamSynchronize(x);
  DevBuf *d[] = {&c->p384_items, &c->kt_base, &c->stage[0], &c->stage[1], &c->stage[2], &c->bd_env, &c->bd_bases, &c->bd_tx, &c->bd_ident, &c->bd_jobs,
                 &c->bd_misc, &c->g_ok, &c->key_ok, &c->gtab28, &c->ktab28, &c->redo, &c->kt_q, &c->kt_slot, &c->kt_scratch,
                 &c->kmap, &c->vbt, &c->vbuse, &c->vbpromo, &c->vblist, &c->vbhand, &c->vbacc, &c->kt_id,
                 &c->status, &c->slot, &c->r, &c->s, &c->dig, &c->d1, &c->wv, &c->wscr, &c->msg,
                 &c->moff, &c->mlen, &c->bj_jobs, &c->bj_sigp, &c->bj_sigl, &c->bj_slot, &c->bj_didx,
                 &c->bj_dig, &c->bj_vst, &c->blk_arena, &c->fz_meta, &c->fz_rowmap, &c->fz_blkof,
                 &c->fz_owner, &c->fz_minblk, &c->fz_minvalid, &c->fz_flags, &c->fz_pslot, &c->fz_res};
  if (c->blk) fgv_block_state_free(c->blk);
  if (c->mv) fgv_mvcc_free(c->mv);
  fgv_integrity_free(c);
  fgv_msp_cache_free(c);
  fgv_p384_free(c);
  for (auto *b : d) b->release();
  HostBuf *h[] = {&c->h_status, &c->h_slot, &c->h_r, &c->h_s, &c->h_dig, &c->h_kq, &c->h_kslot,
                  &c->h_moff, &c->h_mlen, &c->hb_dig, &c->hb_vst, &c->hb_jobs, &c->hb_sigp,
                  &c->hb_sigl, &c->hb_slot, &c->hb_didx, &c->hb_fz, &c->hb_fflags, &c->hb_res,
                  &c->hb_env, &c->hb_bases, &c->hb_misc, &c->h_promo, &c->h_kid};
  for (auto *b : h) b->release();
  for (auto &e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto &e : c->kev)
    if (e) hipEventDestroy(e);
  if (c->stream) hipStreamDestroy(c->stream);
  if (c->stream2) hipStreamDestroy(c->stream2);
  if (c->stream3) hipStreamDestroy(c->stream3);
  if (c->copy_stream) hipStreamDestroy(c->copy_stream);
  if (c->streamF) hipStreamDestroy(c->streamF);
  if (c->streamK) hipStreamSynchronize(c->streamK), hipStreamDestroy(c->streamK);
  if (c->kt_ev) hipEventDestroy(c->kt_ev);
  if (c->ext_ev) hipEventDestroy(c->ext_ev);
  if (c->streamV) hipStreamDestroy(c->streamV);
  for (auto &e : c->vb_ev)
    if (e) hipEventDestroy(e);
  for (auto &e : c->vb_t)
    if (e) hipEventDestroy(e);
  for (auto e : c->stage_ev)
    if (e) hipEventDestroy(e);
  delete c;
}

int fgv_last_host_timing(fgv_ctx *c, double *parse_ms, double *assemble_ms, double *device_ms, double *fold_ms) {
  if (!c) return FGV_EINVAL;
  if (parse_ms) *parse_ms = c->t_host_parse;
  if (assemble_ms) *assemble_ms = c->t_host_assemble;
  if (device_ms) *device_ms = c->t_host_device;
  if (fold_ms) *fold_ms = c->t_host_fold;
  return FGV_OK;
}

int fgv_last_kernel_times(fgv_ctx *c, double *out, size_t n) {
  if (!c || (n && !out)) return FGV_EINVAL;
  for (size_t i = 0; i < n && i < 12; i++) out[i] = c->t_kern[i];
  for (size_t i = 12; i < n; i++) out[i] = 0;
  if (n > 10) out[10] = (double)c->n_pay_blocks;
  return FGV_OK;
}

int fgv_last_counts(fgv_ctx *c, uint64_t *sha_jobs, uint64_t *sha_blocks, uint64_t *verifies) {
  if (!c) return FGV_EINVAL;
  if (sha_jobs) *sha_jobs = c->n_sha_jobs;
  if (sha_blocks) *sha_blocks = c->n_sha_blocks;
  if (verifies) *verifies = c->n_verifies;
  return FGV_OK;
}

int fgv_last_point_handovers(fgv_ctx *c, uint64_t *handovers) {
  if (!c || !handovers) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  uint32_t n = 0;
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpyAsync(&n, c->redo.p, 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return FGV_EDEVICE;
  *handovers = n;
  return FGV_OK;
}

int fgv_last_vb_timing(fgv_ctx *c, double *vb_mul_ms) {
  if (!c || !vb_mul_ms) return FGV_EINVAL;
  *vb_mul_ms = c->t_vb;
  return FGV_OK;
}

int fgv_last_timing(fgv_ctx *c, double *sha_ms, double *prep_ms, double *point_ms,
                    double *keytab_ms) {
  if (!c) return FGV_EINVAL;
  if (sha_ms) *sha_ms = c->t_sha;
  if (prep_ms) *prep_ms = c->t_prep;
  if (point_ms) *point_ms = c->t_point;
  if (keytab_ms) *keytab_ms = c->t_keytab;
  return FGV_OK;
}

}  // extern "C"

// k_prep + k_point on device-resident SoA inputs (events ev[2..4] bracket them)
// k_inv on stream `st` (events ev[2]/ev[3]); the caller orders it after k_der.
// N: capacity (column stride); dn: device-side item count (nullptr: N items)
static int launch_inv(fgv_ctx *c, hipStream_t st, uint32_t N, const uint32_t *dn, uint8_t *d_status,
                      const uint32_t *d_slot, const uint32_t *d_r, const uint32_t *d_s, DevBuf &w, DevBuf &wscr) {
  uint32_t nl = (N + PREP_B - 1) / PREP_B;
  nl = (nl + INV_THREADS - 1) / INV_THREADS * INV_THREADS;
  if (!wscr.ensure((size_t)PREP_B * 8 * nl * 4) || !w.ensure((size_t)N * 32)) return FGV_ENOMEM;
  const bool tim = c->timing || !dn;  // (host-count callers always time their stages)
  // keys whose variable-base verifies reached the promotion threshold in an earlier call get their
  // comb tables now (stream-ordered before this batch's point kernels read kmap)
  int prc = promote_consume(c, N, st);
  if (prc) return prc;
  // keys without a comb (c->n_vb): k_inv lists their items, k_vb_mul computes u2 * Q for them on
  // streamV -- beside the hashes and k_prep: it needs s^-1, not the digest -- and
  // launch_prep_point's k_vb_fin adds u1 * G once k_prep has run
  // (a promotion still building on streamK: its keys count as comb keys on the host but may read
  // KEY_NONE on the device, so their items still need the variable-base kernels)
  if (c->kt_busy && hipEventQuery(c->kt_ev) == hipSuccess) c->kt_busy = false;
  const bool vb = c->n_vb > 0 || c->kt_busy || c->kmap_defer;
  uint32_t *redo = c->redo.as<uint32_t>();
  if (c->vb_pending) {
    // an earlier call queued k_inv / k_vb_mul but failed before its k_vb_fin (which resets the
    // list counters): wait for that k_vb_mul, then reset them here
    c->vb_pending = false;
    HIP_TRY(hipStreamWaitEvent(st, c->vb_ev[1], 0));
    HIP_TRY(hipMemsetAsync(redo + RD_VB_CNT, 0, 4 * (RD_VB_DONE - RD_VB_CNT + 1), st));
    HIP_TRY(hipMemsetAsync(redo + RD_VB2_CNT, 0, 4 * (RD_VB2_MUL - RD_VB2_CNT + 1), st));
  }
  c->vb_launched = vb;
  if (vb && (!c->vblist.ensure((size_t)N * 4) || !c->vbhand.ensure((size_t)N * 4) ||
             !c->vbacc.ensure((size_t)N * VB_ACC_WORDS * 4)))
    return FGV_ENOMEM;
  if (tim) HIP_TRY(hipEventRecord(c->ev[2], st));
  hipLaunchKernelGGL(k_inv, dim3(nl / INV_THREADS), dim3(INV_THREADS), 0, st, N, dn, d_status, d_slot,
                     c->key_ok.as<uint8_t>(), d_r, d_s, w.as<uint32_t>(), wscr.as<uint32_t>(),
                     vb ? c->kmap.as<uint32_t>() : nullptr, vb ? c->vblist.as<uint32_t>() : nullptr,
                     vb ? redo + RD_VB_CNT : nullptr);
  HIP_TRY(hipGetLastError());
  prc = kmap_defer_flush(c, st, 1);
  if (prc) return prc;
  if (tim) HIP_TRY(hipEventRecord(c->ev[3], st));
  if (vb) {
    HIP_TRY(hipEventRecord(c->vb_ev[0], st));
    HIP_TRY(hipStreamWaitEvent(c->streamV, c->vb_ev[0], 0));
    c->vb_timed = tim;
    if (tim) HIP_TRY(hipEventRecord(c->vb_t[0], c->streamV));
    // FGV_VB_WGS = workgroups per CU (k_vb_mul fits 3 waves per SIMD, k_vb_mul_o4 4; default 2:
    // beside k_point28)
    static const uint32_t vb_wgs = [] {
      const char *e = getenv("FGV_VB_WGS");
      const int v = e ? atoi(e) : 2;
      return (uint32_t)(v >= 1 && v <= 4 ? v : 2);
    }();
    // FGV_VB28=0: the exact radix-2^32 kernel alone (A/B); by default k_vb_mul28 (radix 2^28,
    // incomplete formulas) and the exact kernel over its hand-over list only (empty for honest
    // inputs: it returns at once)
    static const bool vb28 = [] {
      const char *e = getenv("FGV_VB28");
      return !e || atoi(e) != 0;
    }();
    // lanes per item: 16 for a small batch (the previous batch's count up to 8 items per CU: a
    // single block's cold creators are one serial chain per lane, and 16 lanes halve it), else 8
    // (a full batch shares the chip with the hashes and the comb verifies, and 16 lanes add
    // butterfly work).  Measured on MI355X (r5v): C2 churn single-block latency 0.63-0.64 ms
    // with 16 against 0.68 with 8; a C2 churn step (~16k cold items) 1.07 ms with 16 against
    // 1.01-1.03 with 8.  FGV_VB_LANES=8 / 16 fixes it (A/B).
    static const int vb_lanes_env = [] {
      const char *e = getenv("FGV_VB_LANES");
      return e ? atoi(e) : 0;
    }();
    // The 16-lane grid is 4 workgroups per CU (not all resident at once: the items are taken from
    // a work queue, so a late workgroup only finds fewer left).
    const uint32_t wgs16 = 4;
    const bool lanes16 = vb_lanes_env == 16 || (vb_lanes_env != 8 && c->vb_last_items <= 8u * c->n_cu);
    if (vb28) {
      hipLaunchKernelGGL(lanes16 ? k_vb_mul28_16 : k_vb_mul28, dim3((lanes16 ? wgs16 : vb_wgs) * c->n_cu), dim3(VB_THREADS),
                         0, c->streamV, N, d_slot,
                         c->vbt.as<uint32_t>(), d_r, w.as<uint32_t>(), redo, c->vblist.as<uint32_t>(),
                         c->vbacc.as<uint32_t>(), c->vbuse.as<uint32_t>(), c->promote_uses,
                         c->vbpromo.as<uint32_t>(), c->vbhand.as<uint32_t>());
      hipLaunchKernelGGL(k_vb_mul, dim3(VB_HAND_WGS), dim3(VB_THREADS), 0, c->streamV, N, d_slot, c->vbt.as<uint32_t>(),
                         d_r, w.as<uint32_t>(), redo + (RD_VB2_CNT - RD_VB_CNT), redo + RD_VB2_MUL,
                         c->vblist.as<uint32_t>(), c->vbacc.as<uint32_t>(), (uint32_t *)nullptr, 0u,
                         c->vbpromo.as<uint32_t>(), c->vbhand.as<uint32_t>());
    } else {
      hipLaunchKernelGGL(vb_wgs == 4 ? k_vb_mul_o4 : k_vb_mul, dim3(vb_wgs * c->n_cu), dim3(VB_THREADS), 0, c->streamV,
                         N, d_slot, c->vbt.as<uint32_t>(), d_r, w.as<uint32_t>(), redo, redo + RD_VB_MUL,
                         c->vblist.as<uint32_t>(), c->vbacc.as<uint32_t>(), c->vbuse.as<uint32_t>(),
                         c->promote_uses, c->vbpromo.as<uint32_t>(), (const uint32_t *)nullptr);
    }
    HIP_TRY(hipGetLastError());
    if (tim) HIP_TRY(hipEventRecord(c->vb_t[1], c->streamV));
    HIP_TRY(hipEventRecord(c->vb_ev[1], c->streamV));
    // the promotion queue back to the host behind it (read by the next call: promote_consume)
    HIP_TRY(hipMemcpyAsync(c->h_promo.p, c->vbpromo.p, (VB_PROMO_CAP + 2) * 4, hipMemcpyDeviceToHost, c->streamV));
    HIP_TRY(hipEventRecord(c->vb_ev[2], c->streamV));
    c->vb_copied = true;
    c->vb_pending = true;
  }
  return FGV_OK;
}
static int launch_inv(fgv_ctx *c, hipStream_t st, uint32_t N, const uint32_t *dn, uint8_t *d_status,
                      const uint32_t *d_slot, const uint32_t *d_r, const uint32_t *d_s) {
  return launch_inv(c, st, N, dn, d_status, d_slot, d_r, d_s, c->wv, c->wscr);
}

// k_prep + k_point on the main stream, after k_inv (ev[3]) and the digests.  N: capacity;
// dn: device-side item count (nullptr: N), n_est: the host's estimate of it (lanes per verify)
static int launch_prep_point(fgv_ctx *c, uint32_t N, const uint32_t *dn, uint32_t n_est, uint8_t *d_status,
                             const uint32_t *d_slot, const uint32_t *d_r, const uint8_t *d_dig,
                             const uint32_t *d_dig_idx, const uint32_t *d_w = nullptr) {
  if (!d_w) d_w = c->wv.as<uint32_t>();
  if (!c->d1.ensure((size_t)DIG_STRIDE * N)) return FGV_ENOMEM;
  const bool tim = c->timing || !dn;
  if (tim) HIP_TRY(hipStreamWaitEvent(c->stream, c->ev[3], 0));  // (k_inv may run on stream2)
  // the digests' producers, waited on directly (a chained cross-stream event adds ~30 us)
  if (c->digests_ready) HIP_TRY(hipStreamWaitEvent(c->stream, c->digests_ready, 0));
  if (c->digests_ready2) HIP_TRY(hipStreamWaitEvent(c->stream, c->digests_ready2, 0));
  if (tim) HIP_TRY(hipEventRecord(c->ev[4], c->stream));
  // k_point28 (radix-2^28, incomplete formulas) decides every item except those that hit an
  // exceptional addition; k_point (complete formulas) then finishes those, and returns at
  // once when k_point28 counted none.  FGV_POINT_EXACT=1 runs k_point alone (A/B knob).
  static const bool exact_only = [] {
    const char *e = getenv("FGV_POINT_EXACT");
    return e && atoi(e) == 1;
  }();
  uint32_t *redo = exact_only ? nullptr : c->redo.as<uint32_t>();
  hipLaunchKernelGGL(k_prep, dim3((N + 255) / 256), dim3(256), 0, c->stream, N, dn, d_status, d_r,
                     d_w, d_dig, d_dig_idx, c->d1.as<int8_t>(), redo);  // (k_prep zeroes *redo)
  HIP_TRY(hipGetLastError());
  // (k_point28's bracket, always: its device time is read live; ahead mode 4 waits on it)
  HIP_TRY(hipEventRecord(c->ev[5], c->stream));
  // Grid: two POINT_THREADS workgroups per CU (2 waves per SIMD) taking chunks of items from a
  // device counter (k_point*: waves placed late, beside a next batch's front half, take fewer).
  // Lanes per verify L (1, 2, 4, 8):
  // k_point28 is VALU-bound; a wave carries ceil(NTERMS / L) comb terms plus log2(L) tree
  // additions (~1.5 mixed-addition equivalents each).  A SIMD running one wave issues at about
  // half rate (dependent-issue latency), two or more share it at full rate, so the batch time
  // is max(2 x wave, waves-per-SIMD x wave) on the busiest SIMD (measured on MI355X: C2
  // 54k verifies L=1/2/4 = 586/340/393 us, C4 131k = 660/685/790 us).  FGV_POINT_LANES forces L.
  static const int forced = [] {
    const char *e = getenv("FGV_POINT_LANES");
    return e ? atoi(e) : 0;
  }();
  const uint64_t simds = (uint64_t)c->n_cu * 4, slots = (uint64_t)c->n_cu * 2 * (POINT_THREADS / 64);
  uint32_t L = 1;
  double best = 1e30;
  for (uint32_t l = 1, lg = 0; l <= POINT_LANES_MAX; l <<= 1, lg++) {
    const uint64_t waves = ((uint64_t)(dn ? n_est : N) * l + 63) / 64;
    const uint64_t passes = (waves + slots - 1) / slots;  // the persistent grid's passes
    const uint64_t per_simd = std::max<uint64_t>(std::max<uint64_t>((waves + simds - 1) / simds, passes), 2);
    const double cost = (double)per_simd * ((double)((NTERMS + l - 1) / l) + 1.5 * lg);
    if (cost < best - 1e-9) { best = cost; L = l; }
  }
  if (forced >= 1 && forced <= POINT_LANES_MAX) L = (uint32_t)forced;

  int frc = kmap_defer_flush(c, c->stream, 2);
  if (frc) return frc;
  if (redo) {
    hipLaunchKernelGGL(k_point28, dim3(2 * c->n_cu), dim3(POINT_THREADS), 0, c->stream, N, dn, L, d_status, d_slot,
                       c->gtab28.as<apoint_raw>(), c->ktab28.as<apoint_raw>(), c->d1.as<int8_t>(), d_r, redo,
                       c->kmap.as<uint32_t>());
  }
  // (after k_point28 a small grid: honest batches hand nothing over, and an empty launch of 2 x n_cu
  // workgroups waited ~50 us for CUs beside the next batch's front half)
  hipLaunchKernelGGL(k_point, dim3(redo ? POINT_EXACT_WGS : 2 * c->n_cu), dim3(POINT_THREADS), 0, c->stream, N, dn, L,
                     d_status, d_slot,
                     c->gtab28.as<apoint_raw>(), c->ktab28.as<apoint_raw>(), c->d1.as<int8_t>(), d_r, redo,
                     c->kmap.as<uint32_t>());
  c->last_lanes = L;
  HIP_TRY(hipGetLastError());
  if (c->vb_pending) {  // the variable-base items: + u1 * G and the x check, after k_vb_mul (streamV)
    c->vb_pending = false;
    HIP_TRY(hipStreamWaitEvent(c->stream, c->vb_ev[1], 0));
    frc = kmap_defer_flush(c, c->stream, 3);
    if (frc) return frc;
    // the grid follows the last read-back batch's variable-base item count (one item per lane):
    // at least VB_FIN_WGS -- every workgroup ends with an atomic on one counter word, and a 2 x n_cu
    // grid spent ~40 us on those alone with an empty list -- at most 2 x n_cu
    const uint32_t fin_wgs = std::min<uint32_t>(std::max<uint32_t>((c->vb_last_items + 255) / 256, VB_FIN_WGS),
                                                2 * c->n_cu);
    hipLaunchKernelGGL(k_vb_fin, dim3(fin_wgs), dim3(256), 0, c->stream, N, d_status, c->gtab28.as<apoint_raw>(),
                       c->d1.as<int8_t>(), d_r, c->redo.as<uint32_t>(), c->vblist.as<uint32_t>(),
                       c->vbacc.as<uint32_t>());
    HIP_TRY(hipGetLastError());
  }
  frc = kmap_defer_flush(c, c->stream, 0);  // (a point this call did not reach)
  if (frc) return frc;
  HIP_TRY(hipEventRecord(c->ev[6], c->stream));  // (ahead mode 1 waits on it)
  return FGV_OK;
}

static int launch_verify_stages(fgv_ctx *c, uint32_t N, uint8_t *d_status, const uint32_t *d_slot,
                                const uint32_t *d_r, const uint32_t *d_s, const uint8_t *d_dig,
                                const uint32_t *d_dig_idx = nullptr) {
  c->timing_ran = true;
  int rc = launch_inv(c, c->stream, N, nullptr, d_status, d_slot, d_r, d_s);
  if (rc) return rc;
  return launch_prep_point(c, N, nullptr, N, d_status, d_slot, d_r, d_dig, d_dig_idx);
}

static void read_stage_times(fgv_ctx *c, bool ran) {
  float ms = 0;
  c->t_prep = c->t_point = c->t_vb = 0;
  if (!ran || !c->timing_ran) return;
  if (c->vb_launched && c->vb_timed && hipEventElapsedTime(&ms, c->vb_t[0], c->vb_t[1]) == hipSuccess) c->t_vb = ms;
  if (hipEventElapsedTime(&ms, c->ev[2], c->ev[3]) == hipSuccess) c->t_prep = ms;
  if (hipEventElapsedTime(&ms, c->ev[4], c->ev[5]) == hipSuccess) c->t_prep += ms;
  if (hipEventElapsedTime(&ms, c->ev[5], c->ev[6]) == hipSuccess) c->t_point = ms;
}

// ------------------------------------------------------------------ verify core
// Host half of verifyECDSA for item i: Go-rule DER (utils.UnmarshalECDSASignature) + low-S;
// writes r, s (zero unless pending) and returns ST_PENDING when the device must finish it,
// FGV_SIG_* otherwise, or -1 for an offset outside sig_buf.
static int der_prepare(const uint8_t *sig_buf, size_t sig_buf_len, size_t so, size_t sl, uint32_t r[8],
                       uint32_t s[8]) {
  int code = ST_PENDING;
  if (sl == 0) {
    code = FGV_SIG_EMPTY;
  } else if (so > sig_buf_len || sl > sig_buf_len - so) {
    return -1;
  } else {
    bool rb, sb;
    if (fgv::der_decode_sig(sig_buf + so, sl, r, s, rb, sb)) {
      code = FGV_SIG_DER;
    } else if (sb || !fgv::is_low_s(s)) {
      code = FGV_SIG_HIGH_S;
    } else if (rb) {
      // r >= 2^256: force an out-of-range value (n) so the device reports RANGE after
      // the key check, matching ecdsa.Verify's order
      static const uint32_t NL[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                     0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};
      memcpy(r, NL, 32);
    }
  }
  if (code != ST_PENDING) {
    memset(r, 0, 32);
    memset(s, 0, 32);
  }
  return code;
}

// upload the prepared items (status / slot / r / s columns in the host staging buffers) and
// digests, run the device stages for the pending ones, read the statuses back
static int verify_run(fgv_ctx *c, size_t n, size_t pending, const uint8_t *h_digests, bool dev_digests,
                      uint8_t *status_out) {
  uint8_t *st = c->h_status.as<uint8_t>();
  if (!c->status.ensure(n) || !c->slot.ensure(n * 4) || !c->r.ensure(n * 32) ||
      !c->s.ensure(n * 32) || !c->dig.ensure(n * 32))
    return FGV_ENOMEM;
  HIP_TRY(hipMemcpyAsync(c->status.p, st, n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->slot.p, c->h_slot.p, n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->r.p, c->h_r.p, n * 32, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->s.p, c->h_s.p, n * 32, hipMemcpyHostToDevice, c->stream));
  if (!dev_digests) {
    if (!c->h_dig.ensure(n * 32)) return FGV_ENOMEM;
    memcpy(c->h_dig.p, h_digests, n * 32);
    HIP_TRY(hipMemcpyAsync(c->dig.p, c->h_dig.p, n * 32, hipMemcpyHostToDevice, c->stream));
  }
  if (pending) {
    int rc = launch_verify_stages(c, (uint32_t)n, c->status.as<uint8_t>(), c->slot.as<uint32_t>(),
                                  c->r.as<uint32_t>(), c->s.as<uint32_t>(), c->dig.as<uint8_t>());
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpyAsync(st, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  memcpy(status_out, st, n);
  read_stage_times(c, pending != 0);
  return FGV_OK;
}

// digests: host pointer (n*32) or nullptr when ctx->dig already holds device digests.
static int verify_core(fgv_ctx *c, const uint8_t *keys, const uint8_t *sig_buf, size_t sig_buf_len,
                       const uint64_t *sig_off, const uint32_t *sig_len, const uint8_t *h_digests,
                       size_t n, uint8_t *status_out, bool dev_digests) {
  if (n == 0) return FGV_OK;
  if (n > 0x7fffffffu) return FGV_EINVAL;
  if (!c->h_status.ensure(n) || !c->h_slot.ensure(n * 4) || !c->h_r.ensure(n * 32) ||
      !c->h_s.ensure(n * 32))
    return FGV_ENOMEM;
  uint8_t *st = c->h_status.as<uint8_t>();
  uint32_t *slot = c->h_slot.as<uint32_t>(), *R = c->h_r.as<uint32_t>(), *S = c->h_s.as<uint32_t>();

  // 1) host: Go-rule DER + low-S; key -> id (new keys counted, assigned below)
  std::unordered_map<std::array<uint8_t, 64>, uint32_t, KeyHash> fresh;  // new key -> uses in this call
  std::unordered_map<uint32_t, uint32_t> vb_uses;                        // known VB id -> uses in this call
  size_t pending = 0;
  for (size_t i = 0; i < n; i++) {
    uint32_t r[8], s[8];
    const int code = der_prepare(sig_buf, sig_buf_len, sig_off[i], sig_len[i], r, s);
    if (code < 0) return FGV_EINVAL;
    st[i] = (uint8_t)code;
    slot[i] = 0;
    if (code == ST_PENDING) {
      pending++;
      std::array<uint8_t, 64> k;
      memcpy(k.data(), keys + 64 * i, 64);
      auto it = c->key_map.find(k);
      if (it == c->key_map.end()) {
        fresh[k]++;
        slot[i] = KEY_NONE;  // assigned below
      } else {
        slot[i] = it->second;
        if (c->kmap_h[it->second] == KEY_NONE) vb_uses[it->second]++;
      }
    }
    for (int k = 0; k < 8; k++) {
      R[(size_t)k * n + i] = r[k];
      S[(size_t)k * n + i] = s[k];
    }
  }
  // 2) ids for new keys (the ad-hoc ids are flushed when the id space would overflow); a key
  // used adhoc_comb_uses times in this call gets a comb table while slots are free (C4: 16 keys x
  // 8192 uses), a one-off key runs on the variable-base kernels
  c->t_keytab = 0;
  if (!fresh.empty() || !vb_uses.empty()) {
    if ((uint64_t)c->n_ids + fresh.size() > c->key_ids) {
      int rc = flush_adhoc(c);
      if (rc) return rc;
      fresh.clear();
      vb_uses.clear();
      for (size_t i = 0; i < n; i++) {
        if (st[i] != ST_PENDING) continue;
        std::array<uint8_t, 64> k;
        memcpy(k.data(), keys + 64 * i, 64);
        auto it = c->key_map.find(k);
        if (it == c->key_map.end()) {
          fresh[k]++;
          slot[i] = KEY_NONE;
        } else if (c->kmap_h[it->second] == KEY_NONE) {
          vb_uses[it->second]++;
        }
      }
      if ((uint64_t)c->n_ids + fresh.size() > c->key_ids) return FGV_ENOMEM;
    }
    std::vector<std::array<uint8_t, 64>> nk;
    std::vector<uint8_t> want;
    for (auto &kv : fresh) {
      nk.push_back(kv.first);
      want.push_back(kv.second >= c->adhoc_comb_uses);
    }
    std::vector<uint32_t> ids(nk.size());
    int rc = ids_new(c, nk, &want, ids.data());
    if (rc) return rc;
    std::vector<uint32_t> hot;  // known VB keys this call uses often
    for (auto &kv : vb_uses)
      if (kv.second >= c->adhoc_comb_uses) hot.push_back(kv.first);
    rc = comb_build(c, hot);
    if (rc) return rc;
    if (!nk.empty())
      for (size_t i = 0; i < n; i++)
        if (st[i] == ST_PENDING && slot[i] == KEY_NONE) {
          std::array<uint8_t, 64> k;
          memcpy(k.data(), keys + 64 * i, 64);
          slot[i] = c->key_map[k];
        }
  }
  // 3) upload + kernels
  return verify_run(c, n, pending, h_digests, dev_digests, status_out);
}

static int launch_sha(fgv_ctx *c, const uint8_t *d_buf, const uint64_t *d_off,
                      const uint32_t *d_len, size_t n) {
  if (!c->dig.ensure(n * 32)) return FGV_ENOMEM;
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  hipLaunchKernelGGL(k_sha256, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, c->stream, d_buf,
                     d_off, d_len, (uint32_t)n, c->dig.as<uint8_t>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  return FGV_OK;
}

static int sha_core(fgv_ctx *c, const uint8_t *buf, size_t buf_len, const uint64_t *off,
                    const uint32_t *len, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (off[i] > buf_len || len[i] > buf_len - off[i]) return FGV_EINVAL;
  if (!c->msg.ensure(buf_len + 64) || !c->moff.ensure(n * 8) || !c->mlen.ensure(n * 4) ||
      !c->dig.ensure(n * 32))
    return FGV_ENOMEM;
  HIP_TRY(hipMemcpyAsync(c->msg.p, buf, buf_len, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(c->msg.as<uint8_t>() + buf_len, 0, 64, c->stream));
  HIP_TRY(hipMemcpyAsync(c->moff.p, off, n * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->mlen.p, len, n * 4, hipMemcpyHostToDevice, c->stream));
  return launch_sha(c, c->msg.as<uint8_t>(), c->moff.as<uint64_t>(), c->mlen.as<uint32_t>(), n);
}

// identity.Verify(msg, sig) for identities of the channel model (registered key slots), host
// buffers: SHA-256 of the messages and the ECDSA stages on the device.  Caller holds c->mu.
int fgv_verify_msgs_slots_locked(fgv_ctx *c, const uint8_t *msg_buf, size_t msg_buf_len, const uint64_t *msg_off,
                                 const uint32_t *msg_len, const uint8_t *sig_buf, size_t sig_buf_len,
                                 const uint64_t *sig_off, const uint32_t *sig_len, const uint32_t *slots, size_t n,
                                 uint8_t *status_out) {
  if (n == 0) return FGV_OK;
  if (n > 0x7fffffffu) return FGV_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  if (!c->h_status.ensure(n) || !c->h_slot.ensure(n * 4) || !c->h_r.ensure(n * 32) || !c->h_s.ensure(n * 32))
    return FGV_ENOMEM;
  uint8_t *st = c->h_status.as<uint8_t>();
  uint32_t *slot = c->h_slot.as<uint32_t>(), *R = c->h_r.as<uint32_t>(), *S = c->h_s.as<uint32_t>();
  size_t pending = 0;
  for (size_t i = 0; i < n; i++) {
    uint32_t r[8], s[8];
    const int code = der_prepare(sig_buf, sig_buf_len, sig_off[i], sig_len[i], r, s);
    if (code < 0 || slots[i] >= c->pinned) return FGV_EINVAL;  // registered (pinned) keys only
    st[i] = (uint8_t)code;
    slot[i] = code == ST_PENDING ? slots[i] : 0;
    pending += code == ST_PENDING;
    for (int k = 0; k < 8; k++) {
      R[(size_t)k * n + i] = r[k];
      S[(size_t)k * n + i] = s[k];
    }
  }
  int rc = sha_core(c, msg_buf, msg_buf_len, msg_off, msg_len, n);
  if (rc) return rc;
  rc = verify_run(c, n, pending, nullptr, true, status_out);
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  c->t_keytab = 0;
  return rc;
}

extern "C" {

int fgv_sha256_batch(fgv_ctx *c, const uint8_t *buf, size_t buf_len, const uint64_t *off,
                     const uint32_t *len, size_t n, uint8_t *out) {
  if (!c || (n && (!off || !len || !out)) || (buf_len && !buf)) return FGV_EINVAL;
  if (n == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  int rc = sha_core(c, buf, buf_len, off, len, n);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, c->dig.p, n * 32, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  return FGV_OK;
}

int fgv_p256_verify_batch(fgv_ctx *c, const uint8_t *keys, const uint8_t *sig_buf,
                          size_t sig_buf_len, const uint64_t *sig_off, const uint32_t *sig_len,
                          const uint8_t *digests, size_t n, uint8_t *status) {
  if (!c || (n && (!keys || !sig_off || !sig_len || !digests || !status))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  c->t_sha = 0;
  return verify_core(c, keys, sig_buf, sig_buf_len, sig_off, sig_len, digests, n, status, false);
}

// identity.Verify for P-384 keys (bccsp sw ecdsaPublicKeyKeyVerifier over any NIST curve,
// sw/ecdsa.go:41-75): SHA-256 of the messages (k_sha256), the keys registered in the context's
// P-384 table (comb built once per key), then k_p384_verify -- one status byte per item.
int fgv_p384_verify_msgs(fgv_ctx *c, const uint8_t *keys, const uint8_t *msg_buf, size_t msg_buf_len,
                         const uint64_t *msg_off, const uint32_t *msg_len, const uint8_t *sig_buf, size_t sig_buf_len,
                         const uint64_t *sig_off, const uint32_t *sig_len, size_t n, uint8_t *status) {
  if (!c || (n && (!keys || !msg_off || !msg_len || !sig_off || !sig_len || !status))) return FGV_EINVAL;
  if (n == 0) return FGV_OK;
  if (n > 0x3fffffffu) return FGV_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (sig_off[i] > sig_buf_len || sig_len[i] > sig_buf_len - sig_off[i]) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  // the columns k_p384_verify reads: absolute signature addresses, lengths, flagged key slots;
  // digests at index i; status ST_P384 for every item
  std::vector<uint32_t> slots(n);
  for (size_t i = 0; i < n; i++) {
    uint32_t k;
    const int rc = fgv_p384_key_locked(c, keys + 96 * i, &k);
    if (rc) return rc;
    slots[i] = KEY_P384_FLAG | k;
  }
  int rc = sha_core(c, msg_buf, msg_buf_len, msg_off, msg_len, n);
  if (rc) return rc;
  const size_t col = n * 8 + n * 4 + n * 4;
  if (!c->p384_items.ensure(col + sig_buf_len + 64) || !c->status.ensure(n)) return FGV_ENOMEM;
  uint8_t *d = c->p384_items.as<uint8_t>();
  uint8_t *dsig = d + col;
  std::vector<uint64_t> ptr(n);
  std::vector<uint32_t> len(n);
  for (size_t i = 0; i < n; i++) {
    ptr[i] = (uint64_t)(uintptr_t)(dsig + sig_off[i]);
    len[i] = sig_len[i];
  }
  if (sig_buf_len) HIP_TRY(hipMemcpyAsync(dsig, sig_buf, sig_buf_len, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d, ptr.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d + n * 8, len.data(), n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d + n * 12, slots.data(), n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemsetAsync(c->status.p, ST_P384, n, c->stream));
  rc = fgv_p384_launch(c, c->stream, (uint32_t)n, nullptr, c->status.as<uint8_t>(), reinterpret_cast<const uint64_t *>(d),
                       reinterpret_cast<const uint32_t *>(d + n * 8), reinterpret_cast<const uint32_t *>(d + n * 12),
                       nullptr, c->dig.as<uint8_t>());
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FGV_OK;
}

int fgv_p256_verify_msgs(fgv_ctx *c, const uint8_t *keys, const uint8_t *msg_buf,
                         size_t msg_buf_len, const uint64_t *msg_off, const uint32_t *msg_len,
                         const uint8_t *sig_buf, size_t sig_buf_len, const uint64_t *sig_off,
                         const uint32_t *sig_len, size_t n, uint8_t *status) {
  if (!c || (n && (!keys || !msg_off || !msg_len || !sig_off || !sig_len || !status)))
    return FGV_EINVAL;
  if (n == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  int rc = sha_core(c, msg_buf, msg_buf_len, msg_off, msg_len, n);
  if (rc) return rc;
  rc = verify_core(c, keys, sig_buf, sig_buf_len, sig_off, sig_len, nullptr, n, status, true);
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  return rc;
}

int fgv_keys_reset(fgv_ctx *c) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pinned) return FGV_ESTATE;  // identities of the channel model hold ids
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  const int rc = flush_adhoc(c);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FGV_OK;
}

int fgv_key_stats(fgv_ctx *c, uint64_t *ids, uint64_t *comb, uint64_t *vb, uint64_t *promoted,
                  uint64_t *vb_verifies_last) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  int wrc = kt_wait(c);  // (promotions still building count as promoted; their kmap lands first)
  if (wrc) return wrc;
  if (ids) *ids = c->n_ids;
  if (comb) *comb = c->n_ids - c->n_vb;
  if (vb) *vb = c->n_vb;
  if (promoted) *promoted = c->n_promoted;
  if (vb_verifies_last) {  // (k_vb_mul of the last verify stages wrote it; copied back behind it)
    *vb_verifies_last = 0;
    if (c->vb_launched) {
      HIP_TRY(hipEventSynchronize(c->vb_ev[2]));
      *vb_verifies_last = c->h_promo.as<uint32_t>()[1];
    }
  }
  return FGV_OK;
}

static int keys_register_locked(fgv_ctx *c, const uint8_t *keys, size_t n, uint32_t *slots, const uint8_t *want_comb);

int fgv_keys_register(fgv_ctx *c, const uint8_t *keys, size_t n, uint32_t *slots) {
  if (!c || (n && (!keys || !slots))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return keys_register_locked(c, keys, n, slots, nullptr);
}

int fgv_keys_register_tiered(fgv_ctx *c, const uint8_t *keys, size_t n, const uint8_t *hot, uint32_t *slots) {
  if (!c || (n && (!keys || !slots))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return keys_register_locked(c, keys, n, slots, hot);
}

// registered keys are pinned: ad-hoc (BCCSP-path) ids are dropped first so the pinned range
// stays contiguous.  A key registered before keeps its id and tier -- except that a key now
// wanted hot gets a comb if it has none and a slot is free.
static int keys_register_locked(fgv_ctx *c, const uint8_t *keys, size_t n, uint32_t *slots, const uint8_t *want_comb) {
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  c->t_keytab = 0;
  std::vector<std::array<uint8_t, 64>> fresh;
  std::vector<uint8_t> want;
  std::unordered_map<std::array<uint8_t, 64>, uint32_t, KeyHash> seen;  // fresh key -> index
  std::vector<uint32_t> upgrade;
  bool adhoc_hit = false;
  for (size_t i = 0; i < n; i++) {
    std::array<uint8_t, 64> k;
    memcpy(k.data(), keys + 64 * i, 64);
    const bool w = !want_comb || want_comb[i];
    auto it = c->key_map.find(k);
    if (it != c->key_map.end() && it->second < c->pinned) {
      if (w && c->kmap_h[it->second] == KEY_NONE) upgrade.push_back(it->second);
      continue;
    }
    adhoc_hit |= it != c->key_map.end();
    auto sj = seen.find(k);
    if (sj != seen.end()) {
      want[sj->second] |= w;
      continue;
    }
    seen.emplace(k, (uint32_t)fresh.size());
    fresh.push_back(k);
    want.push_back(w);
  }
  if (!fresh.empty() || adhoc_hit) {
    int rc = flush_adhoc(c);
    if (rc) return rc;
    if ((uint64_t)c->pinned + fresh.size() > c->key_ids) return FGV_ENOMEM;
    std::vector<uint32_t> ids(fresh.size());
    rc = ids_new(c, fresh, &want, ids.data());
    if (rc) return rc;
    c->pinned = c->n_ids;
  }
  if (!upgrade.empty()) {
    int rc = comb_build(c, upgrade);
    if (rc) return rc;
  }
  for (size_t i = 0; i < n; i++) {
    std::array<uint8_t, 64> k;
    memcpy(k.data(), keys + 64 * i, 64);
    slots[i] = c->key_map[k];
  }
  return FGV_OK;
}

int fgv_p256_verify_msgs_dev(fgv_ctx *c, const uint8_t *d_msg_buf, const uint64_t *d_msg_off,
                             const uint32_t *d_msg_len, const uint8_t *d_sig_buf,
                             const uint64_t *d_sig_off, const uint32_t *d_sig_len,
                             const uint32_t *d_key_slot, size_t n, uint8_t *d_status) {
  if (!c || (n && (!d_msg_buf || !d_msg_off || !d_msg_len || !d_sig_buf || !d_sig_off ||
                   !d_sig_len || !d_key_slot || !d_status)))
    return FGV_EINVAL;
  if (n == 0) return FGV_OK;
  if (n > 0x7fffffffu) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  const uint32_t N = (uint32_t)n;
  if (!c->r.ensure(n * 32) || !c->s.ensure(n * 32) || !c->dig.ensure(n * 32)) return FGV_ENOMEM;
  // k_sha256 on stream2 beside k_der + k_inv on the main stream (the inverse needs s, not the
  // digest); k_prep waits for the digests.  FGV_SIG_FORK=0: all on one stream (A/B).  C4 on
  // MI355X, alternating: 0.679 / 0.684 ms per 131k against 0.701 / 0.707 (profiles/round3_ab/sig_f*)
  static const bool fork = [] {
    const char *e = getenv("FGV_SIG_FORK");
    return !e || atoi(e) != 0;
  }();
  int rc;
  if (fork) {
    HIP_TRY(hipEventRecord(c->ev[7], c->stream));  // (stream2 after the main stream's earlier work)
    HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev[7], 0));
    HIP_TRY(hipEventRecord(c->ev[0], c->stream2));
    hipLaunchKernelGGL(k_sha256, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, c->stream2, d_msg_buf, d_msg_off,
                       d_msg_len, N, c->dig.as<uint8_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[1], c->stream2));
  } else {
    rc = launch_sha(c, d_msg_buf, d_msg_off, d_msg_len, n);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_der, dim3((N + 255) / 256), dim3(256), 0, c->stream, d_sig_buf, d_sig_off,
                     d_sig_len, N, (const uint32_t *)nullptr, d_status, c->r.as<uint32_t>(), c->s.as<uint32_t>(),
                     (const uint32_t *)nullptr);
  HIP_TRY(hipGetLastError());
  c->timing_ran = true;
  rc = launch_inv(c, c->stream, N, nullptr, d_status, d_key_slot, c->r.as<uint32_t>(), c->s.as<uint32_t>());
  if (rc) return rc;
  if (fork) c->digests_ready = c->ev[1];
  rc = launch_prep_point(c, N, nullptr, N, d_status, d_key_slot, c->r.as<uint32_t>(), c->dig.as<uint8_t>(), nullptr);
  c->digests_ready = nullptr;
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  read_stage_times(c, true);
  c->t_keytab = 0;
  return FGV_OK;
}

}  // extern "C"

int fgv_keys_register_locked(fgv_ctx *c, const uint8_t *keys, size_t n, uint32_t *slots, const uint8_t *want_comb) {
  return keys_register_locked(c, keys, n, slots, want_comb);
}

// ======================================================================= block engine glue
// verify-job arrays share one staging block (one H2D copy): [sig_ptr u64 | sig_len | key_slot
// | dig_idx u32], each of nv entries
static size_t sig_block_bytes(size_t nv) { return nv * 20; }

int fgv_block_jobs_reserve(fgv_ctx *c, size_t nj, size_t nv, BlockJobs *out) {
  if (!c->hb_jobs.ensure(nj * sizeof(ShaJob) + 64) || !c->hb_sigp.ensure(sig_block_bytes(nv) + 64))
    return FGV_ENOMEM;
  out->jobs = c->hb_jobs.as<ShaJob>();
  uint8_t *b = c->hb_sigp.as<uint8_t>();
  out->sig_ptr = reinterpret_cast<uint64_t *>(b);
  out->sig_len = reinterpret_cast<uint32_t *>(b + nv * 8);
  out->key_slot = reinterpret_cast<uint32_t *>(b + nv * 12);
  out->dig_idx = reinterpret_cast<uint32_t *>(b + nv * 16);
  return FGV_OK;
}

int fgv_run_block_jobs(fgv_ctx *c, size_t nj, size_t nv, uint64_t sha_blocks, const uint8_t **digests,
                       const uint8_t **vstatus) {
  c->n_sha_jobs = nj;
  c->n_verifies = nv;
  c->n_sha_blocks = sha_blocks;
  if (!c->hb_dig.ensure(nj * 32 + 64) || !c->hb_vst.ensure(nv + 64)) return FGV_ENOMEM;
  *digests = c->hb_dig.as<uint8_t>();
  *vstatus = c->hb_vst.as<uint8_t>();
  if (nj == 0) return FGV_OK;
  if (!c->bj_jobs.ensure(nj * sizeof(ShaJob)) || !c->bj_dig.ensure(nj * 32)) return FGV_ENOMEM;
  HIP_TRY(hipMemcpyAsync(c->bj_jobs.p, c->hb_jobs.p, nj * sizeof(ShaJob), hipMemcpyHostToDevice, c->stream));
  bool ran = false;
  if (nv) {
    const uint32_t N = (uint32_t)nv;
    if (!c->bj_sigp.ensure(sig_block_bytes(nv)) || !c->bj_vst.ensure(nv) || !c->r.ensure(nv * 32) ||
        !c->s.ensure(nv * 32))
      return FGV_ENOMEM;
    HIP_TRY(hipMemcpyAsync(c->bj_sigp.p, c->hb_sigp.p, sig_block_bytes(nv), hipMemcpyHostToDevice, c->stream));
    uint8_t *dsig = c->bj_sigp.as<uint8_t>();
    const uint64_t *d_sigp = reinterpret_cast<const uint64_t *>(dsig);
    const uint32_t *d_sigl = reinterpret_cast<const uint32_t *>(dsig + nv * 8);
    const uint32_t *d_slot = reinterpret_cast<const uint32_t *>(dsig + nv * 12);
    // DER decode first (short), then fork: s^-1 on stream2 while the SHA-256 jobs run on the
    // main stream (launched together, the SHA workgroups would occupy the CUs first)
    hipLaunchKernelGGL(k_der, dim3((N + 255) / 256), dim3(256), 0, c->stream, (const uint8_t *)nullptr, d_sigp,
                       d_sigl, N, (const uint32_t *)nullptr, c->bj_vst.as<uint8_t>(), c->r.as<uint32_t>(),
                       c->s.as<uint32_t>(), d_slot);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[7], c->stream));
    HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev[7], 0));
    c->timing_ran = true;
    int rc = launch_inv(c, c->stream2, N, nullptr, c->bj_vst.as<uint8_t>(), d_slot, c->r.as<uint32_t>(),
                        c->s.as<uint32_t>());
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  hipLaunchKernelGGL(k_sha256_jobs, dim3((uint32_t)((nj + 255) / 256)), dim3(256), 0, c->stream,
                     c->bj_jobs.as<ShaJob>(), (uint32_t)nj, c->bj_dig.as<uint8_t>());
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  if (nv) {
    const uint32_t N = (uint32_t)nv;
    const uint8_t *dsig = c->bj_sigp.as<uint8_t>();
    int rc = launch_prep_point(c, N, nullptr, N, c->bj_vst.as<uint8_t>(),
                               reinterpret_cast<const uint32_t *>(dsig + nv * 12), c->r.as<uint32_t>(),
                               c->bj_dig.as<uint8_t>(), reinterpret_cast<const uint32_t *>(dsig + nv * 16));
    if (rc) return rc;
    rc = fgv_p384_launch(c, c->stream, N, nullptr, c->bj_vst.as<uint8_t>(), reinterpret_cast<const uint64_t *>(dsig),
                         reinterpret_cast<const uint32_t *>(dsig + nv * 8), reinterpret_cast<const uint32_t *>(dsig + nv * 12),
                         reinterpret_cast<const uint32_t *>(dsig + nv * 16), c->bj_dig.as<uint8_t>());
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->hb_vst.p, c->bj_vst.p, nv, hipMemcpyDeviceToHost, c->stream));
    ran = true;
  }
  HIP_TRY(hipMemcpyAsync(c->hb_dig.p, c->bj_dig.p, nj * 32, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  read_stage_times(c, ran);
  return FGV_OK;
}

// Device-resident variant (blockdev path): the jobs were written by k_bd_emit straight into
// c->bj_jobs / c->bj_sigp (layout of fgv_block_jobs_reserve, columns of stride nv); digests stay
// in c->bj_dig and verify status in c->bj_vst.  Enqueued on c->stream; no host copies, no
// synchronisation.  dn: the verify count in device memory (nv is then the capacity, n_est the
// host's estimate of the count), so the stages need no host round trip after the job counts.
int fgv_run_block_jobs_device(fgv_ctx *c, size_t nj, size_t nv, uint64_t sha_blocks, size_t dig_off,
                              const uint8_t *dig, const uint32_t *dn, size_t n_est) {
  const uint8_t *digs = dig ? dig : c->bj_dig.as<uint8_t>();
  c->n_sha_jobs = nj;
  c->n_verifies = dn ? n_est : nv;
  c->n_sha_blocks = sha_blocks;
  c->timing_ran = c->timing || !dn;
  if (nj == 0 && nv == 0) return FGV_OK;
  bool ran = false;
  if (nv) {
    const uint32_t N = (uint32_t)nv;
    if (!c->r.ensure(nv * 32) || !c->s.ensure(nv * 32)) return FGV_ENOMEM;
    uint8_t *dsig = c->bj_sigp.as<uint8_t>();
    const uint64_t *d_sigp = reinterpret_cast<const uint64_t *>(dsig);
    const uint32_t *d_sigl = reinterpret_cast<const uint32_t *>(dsig + nv * 8);
    const uint32_t *d_slot = reinterpret_cast<const uint32_t *>(dsig + nv * 12);
    hipLaunchKernelGGL(k_der, dim3((N + 255) / 256), dim3(256), 0, c->stream, (const uint8_t *)nullptr, d_sigp,
                       d_sigl, N, dn, c->bj_vst.as<uint8_t>(), c->r.as<uint32_t>(), c->s.as<uint32_t>(), d_slot);
    HIP_TRY(hipGetLastError());
    // k_inv beside the SHA-256 jobs when this call hashes (second stream); the device-parse
    // committer's hashes already run on the second stream (k_bd_sha), so k_inv follows k_der
    hipStream_t ist = c->stream;
    if (nj) {
      ist = c->stream2;
      HIP_TRY(hipEventRecord(c->ev[7], c->stream));
      HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev[7], 0));
    }
    int rc = launch_inv(c, ist, N, dn, c->bj_vst.as<uint8_t>(), d_slot, c->r.as<uint32_t>(), c->s.as<uint32_t>());
    if (rc) return rc;
  }
  if (nj) {  // (the device-parse committer hashes with k_bd_sha instead: nj == 0)
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    hipLaunchKernelGGL(k_sha256_jobs, dim3((uint32_t)((nj + 255) / 256)), dim3(256), 0, c->stream,
                       c->bj_jobs.as<ShaJob>(), (uint32_t)nj, c->bj_dig.as<uint8_t>() + dig_off);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  }
  if (nv) {
    const uint32_t N = (uint32_t)nv;
    const uint8_t *dsig = c->bj_sigp.as<uint8_t>();
    int rc = launch_prep_point(c, N, dn, (uint32_t)std::min(n_est, nv), c->bj_vst.as<uint8_t>(),
                               reinterpret_cast<const uint32_t *>(dsig + nv * 12), c->r.as<uint32_t>(), digs,
                               reinterpret_cast<const uint32_t *>(dsig + nv * 16));
    if (rc) return rc;
    rc = fgv_p384_launch(c, c->stream, N, dn, c->bj_vst.as<uint8_t>(), reinterpret_cast<const uint64_t *>(dsig),
                         reinterpret_cast<const uint32_t *>(dsig + nv * 8), reinterpret_cast<const uint32_t *>(dsig + nv * 12),
                         reinterpret_cast<const uint32_t *>(dsig + nv * 16), digs);
    if (rc) return rc;
    ran = true;
  }
  c->stage_ran = ran;
  return FGV_OK;
}

// The device-parse committer's verify stages over one batch's own buffers (fgv_block.cpp
// BdSet), split in two so that the prefix -- k_der, k_inv: they need only the batch's signature
// list, not the digests -- can be enqueued ahead with the batch's front half, beside the
// previous batch's back half.  sigblk: the k_bd_emit columns (ptr | len | key slot | digest
// index, stride cap); dn: the verify count in device memory.
int fgv_verify_prefix_dev(fgv_ctx *c, hipStream_t st, size_t cap, const uint32_t *dn, const uint8_t *sigblk,
                          uint8_t *vst, DevBuf &r, DevBuf &s, DevBuf &w, DevBuf &wscr) {
  const uint32_t N = (uint32_t)cap;
  if (!r.ensure(cap * 32) || !s.ensure(cap * 32)) return FGV_ENOMEM;
  hipLaunchKernelGGL(k_der, dim3((N + 255) / 256), dim3(256), 0, st, (const uint8_t *)nullptr,
                     reinterpret_cast<const uint64_t *>(sigblk), reinterpret_cast<const uint32_t *>(sigblk + cap * 8), N,
                     dn, vst, r.as<uint32_t>(), s.as<uint32_t>(), reinterpret_cast<const uint32_t *>(sigblk + cap * 12));
  HIP_TRY(hipGetLastError());
  return launch_inv(c, st, N, dn, vst, reinterpret_cast<const uint32_t *>(sigblk + cap * 12), r.as<uint32_t>(),
                    s.as<uint32_t>(), w, wscr);
}
int fgv_verify_main_dev(fgv_ctx *c, size_t cap, const uint32_t *dn, size_t n_est, const uint8_t *sigblk, uint8_t *vst,
                        const uint32_t *r, const uint32_t *w, const uint8_t *digests) {
  c->n_sha_jobs = 0;
  c->n_verifies = n_est;
  c->n_sha_blocks = 0;
  c->timing_ran = c->timing;
  int rc = launch_prep_point(c, (uint32_t)cap, dn, (uint32_t)std::min(n_est, cap), vst,
                             reinterpret_cast<const uint32_t *>(sigblk + cap * 12), r, digests,
                             reinterpret_cast<const uint32_t *>(sigblk + cap * 16), w);
  // (P-384 identities' signatures: their own kernel, same stream, before the fold reads vst)
  if (rc == FGV_OK)
    rc = fgv_p384_launch(c, c->stream, (uint32_t)cap, dn, vst, reinterpret_cast<const uint64_t *>(sigblk),
                         reinterpret_cast<const uint32_t *>(sigblk + cap * 8),
                         reinterpret_cast<const uint32_t *>(sigblk + cap * 12),
                         reinterpret_cast<const uint32_t *>(sigblk + cap * 16), digests);
  c->stage_ran = rc == FGV_OK;
  return rc;
}

// stage times of the last fgv_run_block_jobs_device (after the stream has been synchronised)
void fgv_read_block_job_times(fgv_ctx *c) {
  float ms = 0;
  c->t_sha = 0;
  if (c->n_sha_jobs && hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) c->t_sha = ms;
  read_stage_times(c, c->stage_ran);
}

extern "C" {

int fgv_channel_init(fgv_ctx *c, const char *name) {
  if (!c || !name) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_set_channel(c->blk, name);
}

int fgv_msp_register_identity(fgv_ctx *c, const uint8_t *serialized, size_t len, const fgv_identity_info *info) {
  if (!c || !serialized || !info) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  int32_t slot = -1;
  if (info->key_type == FGV_KEY_P256) {
    uint32_t s;
    const uint8_t want = fgv_roles_want_comb(info->roles) ? 1 : 0;
    int rc = keys_register_locked(c, info->pubkey, 1, &s, &want);
    if (rc) return rc;
    slot = (int32_t)s;
  } else if (info->key_type == FGV_KEY_P384) {
    // verified per item on the GPU (p384.hip) when the key is given; an all-zero key is "not
    // known": the identity stays outside the engine, as before round 6
    bool given = false;
    for (int i = 0; i < 96; i++) given |= info->pubkey_p384[i] != 0;
    if (given) {
      uint32_t k;
      int rc = fgv_p384_key_locked(c, info->pubkey_p384, &k);
      if (rc) return rc;
      slot = (int32_t)(KEY_P384_FLAG | k);
    }
  }
  return fgv_block_add_identity(c->blk, serialized, len, slot, info);
}

int fgv_msp_identity_ous(fgv_ctx *c, const uint8_t *serialized, size_t len, size_t n, const char *const *ou,
                         const size_t *ou_lens, const uint8_t *const *certifiers, const size_t *certifier_lens) {
  if (!c || !serialized || (n && (!ou || !ou_lens || !certifiers || !certifier_lens))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_identity_ous(c->blk, serialized, len, n, ou, ou_lens, certifiers, certifier_lens);
}

int fgv_msp_add_identity(fgv_ctx *c, const uint8_t *serialized, size_t len, const uint8_t *pubkey, int valid,
                         const uint8_t *id_digest) {
  if (!c || !serialized || !id_digest) return FGV_EINVAL;
  fgv_identity_info info{};
  info.key_type = pubkey ? FGV_KEY_P256 : FGV_KEY_OTHER;
  info.hash_family = FGV_HASH_SHA2;
  info.valid = valid != 0;
  info.roles = FGV_ROLES_UNKNOWN;
  if (pubkey) memcpy(info.pubkey, pubkey, 64);
  memcpy(info.id_digest, id_digest, 32);
  return fgv_msp_register_identity(c, serialized, len, &info);
}

int fgv_chaincode_define2(fgv_ctx *c, const char *ns, const char *plugin, const uint8_t *policy, size_t len,
                          uint32_t flags) {
  if (!c || !ns || !plugin || (len && !policy)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_define_chaincode(c->blk, ns, plugin, policy, len, flags);
}

int fgv_chaincode_define(fgv_ctx *c, const char *ns, const uint8_t *policy, size_t len) {
  return fgv_chaincode_define2(c, ns, "vscc", policy, len, 0);
}

int fgv_collection_define(fgv_ctx *c, const char *ns, const char *coll, const uint8_t *policy, size_t len) {
  if (!c || !ns || !coll || (len && !policy)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_define_collection(c->blk, ns, coll, policy, len);
}

int fgv_kvmeta_set(fgv_ctx *c, const char *ns, const char *coll, const uint8_t *key, size_t key_len,
                   const uint8_t *vp, size_t vp_len) {
  if (!c || !ns || (key_len && !key) || (vp_len && !vp)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_kvmeta_set(c->blk, ns, coll ? coll : "", key, key_len, vp, vp_len);
}

int fgv_kvmeta_get(fgv_ctx *c, const char *ns, const char *coll, const uint8_t *key, size_t key_len, uint8_t *buf,
                   size_t cap, size_t *len) {
  if (!c || !ns || !len || (key_len && !key) || (cap && !buf)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  const std::string *v = fgv_block_kvmeta_get(c->blk, ns, coll ? coll : "", key, key_len);
  *len = v ? v->size() : 0;
  if (v && cap) memcpy(buf, v->data(), std::min(cap, v->size()));
  return FGV_OK;
}

size_t fgv_kvmeta_count(fgv_ctx *c) {
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_kvmeta_count(c->blk);
}

int fgv_channel_config(fgv_ctx *c, const uint8_t *config, size_t len) {
  if (!c || (len && !config)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_channel_config(c->blk, config, len);
}

int fgv_msp_declare(fgv_ctx *c, const char *mspid) {
  if (!c || !mspid) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_declare_msp(c->blk, mspid);
}

int fgv_ledger_add_txids(fgv_ctx *c, const uint8_t *buf, const uint64_t *off, const uint32_t *len, size_t n) {
  if (!c || (n && (!buf || !off || !len))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_add_txids(c->blk, buf, off, len, n);
}


// Device finalize over W x rows gathered records (finalize.hip).  Caller holds c->mu and has
// set the device.
// rank_lo / rank_hi (W x nb, FGV_SHARD_SKIP = no rows) or null for the per-block split
// [floor(n r / W), floor(n (r+1) / W)).  The ranks' ranges must tile every block.
// defer: leave the flags' D2H copy (into c->hb_fflags) queued -- the caller synchronises and
// copies them out (fgv_validate_blocks: one synchronisation for validation + finalize).
// Three parts: fin_prepare (host metadata, buffers), fin_front (metadata upload, row map +
// table reset, the txid index) and fin_back (codes, duplicates, flags D2H).  A single-device
// batch runs fin_front early, beside its verify chain (fgv_finalize_early_index).
static int fin_prepare(fgv_ctx *c, size_t nblocks, const size_t *ntx, uint32_t W, size_t rows, const uint32_t *rank_lo,
                       const uint32_t *rank_hi, FinPlan &F) {
  if (W == 0 || (!rank_lo) != (!rank_hi)) return FGV_EINVAL;
  uint64_t P = 0;
  for (size_t b = 0; b < nblocks; b++) P += ntx[b];
  F.P = P;
  if (P == 0) return FGV_OK;
  if (P >= 0x7FFFFFFFull || nblocks >= 0x7FFFFFFFull || rows * W >= 0xFFFFFFFFull) return FGV_EINVAL;
  // host metadata: blk_start (nb+1 u64) | roff (W x nb u32) | lo (W x nb u32) | cnt (W x nb u32)
  const size_t wn = (size_t)W * nblocks;
  const size_t meta = (nblocks + 1) * 8 + 3 * wn * 4;
  if (!c->hb_fz.ensure(meta) || !c->fz_meta.ensure(meta)) return FGV_ENOMEM;
  uint64_t *bstart = c->hb_fz.as<uint64_t>();
  uint32_t *roff = reinterpret_cast<uint32_t *>(bstart + nblocks + 1), *rlo = roff + wn, *rcnt = rlo + wn;
  bstart[0] = 0;
  for (size_t b = 0; b < nblocks; b++) bstart[b + 1] = bstart[b] + ntx[b];
  for (uint32_t r = 0; r < W; r++) {
    uint64_t o = 0;
    for (size_t b = 0; b < nblocks; b++) {
      const size_t k = (size_t)r * nblocks + b;
      const uint64_t n = ntx[b];
      uint64_t lo = (n * r) / W, hi = (n * (r + 1)) / W;
      if (rank_lo) {
        lo = rank_lo[k] == FGV_SHARD_SKIP ? 0 : rank_lo[k];
        hi = rank_lo[k] == FGV_SHARD_SKIP ? 0 : rank_hi[k];
        if (hi < lo || hi > n) return FGV_EINVAL;
      }
      roff[k] = (uint32_t)o;
      rlo[k] = (uint32_t)lo;
      rcnt[k] = (uint32_t)(hi - lo);
      o += hi - lo;
    }
    if (o > rows) return FGV_EINVAL;  // gathered rows cannot hold rank r's shard
  }
  for (size_t b = 0; b < nblocks; b++) {  // the ranges must tile the block
    uint64_t cover = 0;
    for (uint32_t r = 0; r < W; r++) cover += rcnt[(size_t)r * nblocks + b];
    if (cover != ntx[b]) return FGV_EINVAL;
  }
  size_t cap = 1024;
  while (cap < 2 * P) cap <<= 1;
  if (!c->fz_rowmap.ensure(P * 4) || !c->fz_blkof.ensure(P * 4) || !c->fz_owner.ensure(cap * 4) ||
      !c->fz_minblk.ensure(cap * 4) || !c->fz_minvalid.ensure(cap * 4) || !c->fz_flags.ensure(P) ||
      !c->fz_pslot.ensure(P * 4) || !c->hb_fflags.ensure(P))
    return FGV_ENOMEM;
  F.cap = cap;
  F.wn = wn;
  F.meta = meta;
  return FGV_OK;
}
// The finalize front (k_fin_rows, k_fin_index_dev) at wave priority 3, like the verify chain it
// runs beside (the fold waits for it).  C2 lean harness on MI355X, alternating x3: 0.689 / 0.677 /
// 0.655 ms per step against 0.679 / 0.696 / 0.681 at priority 0 (profiles/round3_ab/fp*): a
// small gain at the noise level; FGV_FIN_PRIO=0 turns it off (A/B)
static uint32_t fin_prio() {
  static const uint32_t v = [] {
    const char *e = getenv("FGV_FIN_PRIO");
    return e ? (uint32_t)atoi(e) : 1u;
  }();
  return v;
}
// index from the gathered records (recs != null) or from a single-device batch's parse and
// digests (dtx != null: the owners' keys go to c->fz_keys)
static int fin_front(fgv_ctx *c, hipStream_t st, size_t nblocks, uint32_t W, size_t rows, const FinPlan &F,
                     const uint8_t *d_recs, const DevTx *dtx, const uint64_t *bases, const uint8_t *digests) {
  HIP_TRY(hipMemcpyAsync(c->fz_meta.p, c->hb_fz.p, F.meta, hipMemcpyHostToDevice, st));
  const uint32_t n32 = (uint32_t)F.P, mask = (uint32_t)(F.cap - 1);
  const dim3 grid((n32 + 255) / 256), blk(256);
  const uint64_t *d_bstart = c->fz_meta.as<uint64_t>();
  const uint32_t *d_roff = reinterpret_cast<const uint32_t *>(d_bstart + nblocks + 1);
  // (k_fin_rows also resets the cap-slot txid table)
  hipLaunchKernelGGL(k_fin_rows, dim3((uint32_t)((std::max<size_t>(F.P, F.cap) + 255) / 256)), blk, 0, st, n32,
                     d_bstart, (uint32_t)nblocks, W, (uint32_t)rows, d_roff, d_roff + F.wn, d_roff + 2 * F.wn,
                     c->fz_rowmap.as<uint32_t>(), c->fz_blkof.as<uint32_t>(), (uint32_t)F.cap,
                     c->fz_owner.as<uint32_t>(), c->fz_minblk.as<int32_t>(), c->fz_minvalid.as<uint32_t>(), dtx,
                     bases, digests, dtx ? c->fz_keys.as<uint8_t>() : nullptr, fin_prio());
  if (dtx)
    hipLaunchKernelGGL(k_fin_index_dev, grid, blk, 0, st, n32, dtx, bases, digests, c->fz_keys.as<uint8_t>(),
                       c->fz_owner.as<uint32_t>(), c->fz_minblk.as<int32_t>(), mask, c->fin_seed, fin_prio());
  else
    hipLaunchKernelGGL(k_fin_index, grid, blk, 0, st, n32, d_recs, c->fz_rowmap.as<uint32_t>(),
                       c->fz_blkof.as<uint32_t>(), c->fz_owner.as<uint32_t>(), c->fz_minblk.as<int32_t>(), mask,
                       c->fin_seed);
  HIP_TRY(hipGetLastError());
  return FGV_OK;
}
static int fin_back(fgv_ctx *c, hipStream_t st, const FinPlan &F, const uint8_t *d_recs, const uint8_t *keys,
                    bool codes_done = false) {
  const uint32_t n32 = (uint32_t)F.P, mask = (uint32_t)(F.cap - 1);
  const dim3 grid((n32 + 255) / 256), blk(256);
  if (!codes_done)
    hipLaunchKernelGGL(k_fin_codes, grid, blk, 0, st, n32, d_recs, c->fz_rowmap.as<uint32_t>(),
                     c->fz_blkof.as<uint32_t>(), c->fz_owner.as<uint32_t>(), c->fz_minblk.as<int32_t>(),
                     c->fz_minvalid.as<uint32_t>(), mask, c->fin_seed, c->fz_flags.as<uint8_t>(),
                     c->fz_pslot.as<uint32_t>(), keys);
  // the final flags go straight into the pinned host buffer (mapped): a 16 KB D2H copy behind the
  // last kernel ran as a blit kernel that waited ~50 us for CUs held by the next batch's front
  // half (MI355X C2 trace).  FGV_FLAGS_ZC=0: the copy (A/B)
  static const bool zc_on = [] {
    const char *e = getenv("FGV_FLAGS_ZC");
    return !e || atoi(e) != 0;
  }();
  uint8_t *zc = nullptr;
  if (zc_on && hipHostGetDevicePointer(reinterpret_cast<void **>(&zc), c->hb_fflags.p, 0) != hipSuccess) zc = nullptr;
  // (the fused call: the batch counters ride along, written by the last workgroup)
  uint32_t *mz = nullptr;
  if (zc && codes_done && c->fin_misc_src && c->fin_misc_dst &&
      hipHostGetDevicePointer(reinterpret_cast<void **>(&mz), c->fin_misc_dst, 0) != hipSuccess)
    mz = nullptr;
  hipLaunchKernelGGL(k_fin_dups, grid, blk, 0, st, n32, c->fz_pslot.as<uint32_t>(), c->fz_minvalid.as<uint32_t>(),
                     c->fz_flags.as<uint8_t>(), codes_done ? c->fold_unsup : nullptr, zc,
                     mz ? c->fin_misc_src : nullptr, mz, c->redo.as<uint32_t>() + RD_FIN_DONE);
  c->fin_misc_done = mz != nullptr;
  c->fin_misc_src = nullptr;
  HIP_TRY(hipGetLastError());
  if (!zc) HIP_TRY(hipMemcpyAsync(c->hb_fflags.p, c->fz_flags.p, F.P, hipMemcpyDeviceToHost, st));
  return FGV_OK;
}

// the single-device fused call's finalize front, enqueued on `st` once the batch's digests are
// there (stream order), recorded as c->fin_ev
int fgv_finalize_early_index(fgv_ctx *c, size_t nblocks, const size_t *ntx, const DevTx *dtx, const uint64_t *bases,
                             const uint8_t *digests, hipStream_t st) {
  c->early_fin = false;
  FinPlan F;
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) total += ntx[b];
  int rc = fin_prepare(c, nblocks, ntx, 1, total, nullptr, nullptr, F);
  if (rc || F.P == 0) return rc;
  if (!c->fz_keys.ensure(F.P * 32)) return FGV_ENOMEM;
  if (!c->fin_ev) HIP_TRY(hipEventCreateWithFlags(&c->fin_ev, hipEventDisableTiming));
  rc = fin_front(c, st, nblocks, 1, total, F, nullptr, dtx, bases, digests);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->fin_ev, st));
  c->early_plan = F;
  c->early_fin = true;
  return FGV_OK;
}

static int finalize_dev_core(fgv_ctx *c, size_t nblocks, const size_t *ntx, uint32_t W, size_t rows,
                             const uint8_t *d_recs, uint8_t *flags, const uint32_t *rank_lo = nullptr,
                             const uint32_t *rank_hi = nullptr, bool defer = false) {
  const bool early = c->early_fin, codes_done = c->fold_codes;
  c->early_fin = c->fold_codes = false;
  if (((uintptr_t)d_recs & 3)) return FGV_EINVAL;
  FinPlan F;
  int rc;
  hipStream_t st = c->stream;
  uint64_t P = 0;
  for (size_t b = 0; b < nblocks; b++) P += ntx[b];
  if (early && W == 1 && c->early_plan.P == P) {  // the front ran beside the verify chain (W = 1, rows = P)
    // (its plan is reused: preparing again would rewrite the pinned metadata while the front's
    // copy of it may still be queued)
    F = c->early_plan;
    if (F.P == 0) return FGV_OK;
    HIP_TRY(hipStreamWaitEvent(st, c->fin_ev, 0));
    rc = fin_back(c, st, F, d_recs, c->fz_keys.as<uint8_t>(), codes_done);
  } else {
    if (early) HIP_TRY(hipEventSynchronize(c->fin_ev));  // (its metadata copy reads c->hb_fz)
    rc = fin_prepare(c, nblocks, ntx, W, rows, rank_lo, rank_hi, F);
    if (rc || F.P == 0) return rc;
    rc = fin_front(c, st, nblocks, W, rows, F, d_recs, nullptr, nullptr, nullptr);
    if (!rc) rc = fin_back(c, st, F, d_recs, nullptr);
  }
  if (rc) return rc;
  if (defer) return FGV_OK;
  HIP_TRY(hipStreamSynchronize(st));
  memcpy(flags, c->hb_fflags.p, F.P);
  return FGV_OK;
}

static size_t stage_bytes(size_t nblocks, const size_t *lens) {
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) total += (lens[b] + 64 + 255) & ~(size_t)255;
  return total;
}

// H2D copies of a batch into arena A on stream `st`: blocks that lie back to back in host memory
// (a peer's pinned receive buffer, the bench's batches) travel as ONE copy per run, laid out in
// the arena exactly as in host memory (a kernel reading past a block's end reads the next one's
// bytes), each run followed by >= 64 B of padding; the device addresses go to dev[].  Returns the
// bytes copied.
static int copy_runs(size_t nblocks, const uint8_t *const *blocks, const size_t *lens, uint8_t *A, hipStream_t st,
                     const uint8_t **dev, size_t *copied) {
  size_t o = 0, b = 0;
  *copied = 0;
  while (b < nblocks) {
    size_t e = b + 1, run = lens[b];
    while (e < nblocks && blocks[e] == blocks[e - 1] + lens[e - 1]) run += lens[e++];
    if (run) HIP_TRY(hipMemcpyAsync(A + o, blocks[b], run, hipMemcpyHostToDevice, st));
    for (size_t q = b; q < e; q++) dev[q] = A + o + (size_t)(blocks[q] - blocks[b]);
    *copied += run;
    o += (run + 64 + 255) & ~(size_t)255;
    b = e;
  }
  return FGV_OK;
}

// A staging slot no staged batch holds and the current call's batch does not use (every earlier
// call has completed: each validation call ends synchronised); with none free the oldest staged
// batch is dropped (its front half, if enqueued ahead, is drained first).
static int free_slot(fgv_ctx *c, int avoid) {
  for (;;) {
    for (int q = 0; q < fgv_ctx::kStage; q++) {
      if (q == avoid) continue;
      bool held = false;
      for (const auto &e : c->pf) held |= e.slot == q;
      if (!held) return q;
    }
    fgv_block_drain(c);  // (a front half enqueued ahead may read the arena about to be reused)
    c->pf.erase(c->pf.begin());
  }
}

// Host-resident blocks -> device.  A batch staged ahead (the previous _next / pipelined call's
// NEXT batch, or fgv_prefetch) is already on its way (copy stream): the compute stream waits
// for that copy instead of copying again.
static int stage_blocks(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                        const uint8_t *const *d_blocks, std::vector<const uint8_t *> &dev) {
  dev.resize(nblocks);
  c->n_prefetch_hits = 0;
  c->h2d_bytes = 0;
  if (d_blocks) {
    for (size_t b = 0; b < nblocks; b++) dev[b] = d_blocks[b];
    return FGV_OK;
  }
  for (size_t q = 0; q < c->pf.size(); q++) {
    if (!c->pf[q].matches(nblocks, blocks, lens)) continue;
    const fgv_ctx::Prefetch e = c->pf[q];
    c->pf.erase(c->pf.begin() + (long)q);
    c->stage_cur = e.slot;
    for (size_t b = 0; b < nblocks; b++) dev[b] = e.dev[b];
    c->n_prefetch_hits = nblocks;
    HIP_TRY(hipStreamWaitEvent(c->stream, c->stage_ev[e.slot], 0));
    return FGV_OK;
  }
  // copy now, into a slot no staged batch holds (64 B padding after each block)
  const int slot = free_slot(c, -1);
  DevBuf &A = c->stage[slot];
  if (!A.ensure(stage_bytes(nblocks, lens))) return FGV_ENOMEM;
  HIP_TRY(hipStreamWaitEvent(c->stream, c->stage_ev[slot], 0));  // (a dropped staging copy may still write it)
  size_t copied = 0;
  int rc = copy_runs(nblocks, blocks, lens, A.as<uint8_t>(), c->stream, dev.data(), &copied);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->stage_ev[slot], c->stream));
  c->stage_cur = slot;
  c->h2d_bytes = copied;
  return FGV_OK;
}

// Stage a later batch's H2D copy into a free arena on the copy stream (it overlaps the kernels of
// the batches before it).  Called after stage_blocks of the current batch, or from fgv_prefetch
// between calls.  A batch already staged is not copied again.  -> the staged entry
static int prefetch_blocks(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                           const fgv_ctx::Prefetch **out, bool in_call = true) {
  *out = nullptr;
  if (!nblocks) return FGV_OK;
  for (const auto &e : c->pf)
    if (e.matches(nblocks, blocks, lens)) {
      *out = &e;
      return FGV_OK;
    }
  // (inside a call its own batch's slot is busy; between calls the last call's slot is free)
  const int slot = free_slot(c, in_call ? c->stage_cur : -1);
  DevBuf &A = c->stage[slot];
  if (!A.ensure(stage_bytes(nblocks, lens))) return FGV_ENOMEM;
  fgv_ctx::Prefetch e;
  e.slot = slot;
  e.src.assign(blocks, blocks + nblocks);
  e.lens.assign(lens, lens + nblocks);
  e.dev.resize(nblocks);
  size_t copied = 0;
  int rc = copy_runs(nblocks, blocks, lens, A.as<uint8_t>(), c->copy_stream, e.dev.data(), &copied);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->stage_ev[slot], c->copy_stream));
  c->pf.push_back(std::move(e));
  *out = &c->pf.back();
  return FGV_OK;
}

int fgv_prefetch(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens) {
  if (!c || (nblocks && (!blocks || !lens))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  const fgv_ctx::Prefetch *e = nullptr;
  return prefetch_blocks(c, nblocks, blocks, lens, &e, false);
}

static size_t shard_count(size_t nblocks, const size_t *ntx, const uint32_t *tx_lo, const uint32_t *tx_hi) {
  size_t n = 0;
  for (size_t b = 0; b < nblocks; b++) {
    if (tx_lo && tx_lo[b] == FGV_SHARD_SKIP) continue;
    const size_t lo = tx_lo ? std::min<size_t>(tx_lo[b], ntx[b]) : 0;
    const size_t hi = tx_hi ? std::min<size_t>(tx_hi[b], ntx[b]) : ntx[b];
    if (hi > lo) n += hi - lo;
  }
  return n;
}

int fgv_set_parse_mode(fgv_ctx *c, int mode) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_set_parse_mode(c->blk, mode);
}

// An FGV_EUNSUPPORTED batch whose obstacle may be identities the registry has not seen: resolve
// them through the channel's MSPs (the MSP cache miss, fgv_msp.cpp); true when any was added,
// so that one retry of the batch can help.
static bool resolve_for_retry(fgv_ctx *c, int rc, size_t nblocks, const uint8_t *const *blocks, const size_t *lens) {
  if (rc != FGV_EUNSUPPORTED || !fgv_msp_auto(c)) return false;
  size_t reg = 0;
  return fgv_msp_resolve_blocks_locked(c, nblocks, blocks, lens, &reg) == FGV_OK && reg > 0;
}

static int shard_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                        const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                        fgv_tx_result *results, size_t results_cap, size_t *ntx) {
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  std::vector<const uint8_t *> dev;
  int rc = stage_blocks(c, nblocks, blocks, lens, d_blocks, dev);
  if (rc) return rc;
  if (fgv_block_parse_mode(c->blk) == 0) {
    if (!c->fz_res.ensure(results_cap * sizeof(fgv_tx_result) + 64)) return FGV_ENOMEM;
    rc = fgv_block_validate_dev(c, c->blk, nblocks, blocks, lens, dev.data(), tx_lo, tx_hi,
                                c->fz_res.as<fgv_tx_result>(), results_cap, ntx);
    if (rc != 1) {
      if (rc) return rc;
      const size_t n = shard_count(nblocks, ntx, tx_lo, tx_hi);
      if (n) HIP_TRY(hipMemcpy(results, c->fz_res.p, n * sizeof(fgv_tx_result), hipMemcpyDeviceToHost));
      return FGV_OK;
    }
  }
  return fgv_block_validate_impl(c, c->blk, nblocks, blocks, lens, dev.data(), tx_lo, tx_hi, results,
                                 results_cap, ntx);
}

int fgv_validate_shard(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                       const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                       fgv_tx_result *results, size_t results_cap, size_t *ntx) {
  if (!c || (nblocks && (!blocks || !lens || !ntx || (results_cap && !results)))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  int rc = shard_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, results, results_cap, ntx);
  if (resolve_for_retry(c, rc, nblocks, blocks, lens))
    rc = shard_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, results, results_cap, ntx);
  return rc;
}

static int shard_dev_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                            const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                            void *d_results, size_t results_cap, size_t *ntx) {
  c->kl_changes = false;  // (set by the host-parse path only: plain batches change no key-level state)
  if (nblocks == 0) return FGV_OK;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  std::vector<const uint8_t *> dev;
  int rc = stage_blocks(c, nblocks, blocks, lens, d_blocks, dev);
  if (rc) return rc;
  if (c->next.n && c->next.prefetch) {
    const fgv_ctx::Prefetch *e = nullptr;
    rc = prefetch_blocks(c, c->next.n, c->next.blocks, c->next.lens, &e);
    if (rc) return rc;
    c->next.d_blocks = e->dev.data();  // its front half can be enqueued ahead of its call
    c->next.wait = c->stage_ev[e->slot];
  }
  if (fgv_block_parse_mode(c->blk) == 0) {
    rc = fgv_block_validate_dev(c, c->blk, nblocks, blocks, lens, dev.data(), tx_lo, tx_hi,
                                static_cast<fgv_tx_result *>(d_results), results_cap, ntx);
    if (rc != 1) return rc;
  }
  if (!c->hb_res.ensure(results_cap * sizeof(fgv_tx_result) + 64)) return FGV_ENOMEM;
  fgv_tx_result *res = c->hb_res.as<fgv_tx_result>();
  rc = fgv_block_validate_impl(c, c->blk, nblocks, blocks, lens, dev.data(), tx_lo, tx_hi, res, results_cap, ntx);
  if (rc) return rc;
  const size_t n = shard_count(nblocks, ntx, tx_lo, tx_hi);
  if (n) {
    HIP_TRY(hipMemcpyAsync(d_results, res, n * sizeof(fgv_tx_result), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  return FGV_OK;
}

static int shard_dev_outcomes(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                              const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                              void *d_results, size_t results_cap, size_t *ntx);

int fgv_validate_shard_dev(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                           const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                           void *d_results, size_t results_cap, size_t *ntx) {
  if (!c || (nblocks && (!blocks || !lens || !ntx || (results_cap && !d_results)))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->next = fgv_ctx::NextBatch{};
  if (c->block_outcomes)
    return shard_dev_outcomes(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
  c->blk_status.clear();
  int rc = shard_dev_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
  if (resolve_for_retry(c, rc, nblocks, blocks, lens))
    rc = shard_dev_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
  return c->last_rc = rc;
}

// shard_dev_locked with per-block outcomes on (the caller holds c->mu): undecided transactions keep
// 0xFD in their records; *split = the first block of the call's list that must wait for an earlier
// block's commit (UINT32_MAX: none).  A soft pass that left transactions undecided resolves the
// blocks' identities through the MSP cache-miss path and runs again, as fgv_validate_blocks does.
static int shard_dev_soft_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                 const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                                 void *d_results, size_t results_cap, size_t *ntx, uint32_t *split) {
  bool unsup = false;
  auto run = [&] {
    fgv_block_set_soft(c->blk, true);
    const int r = shard_dev_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
    *split = fgv_block_split(c->blk);
    unsup = fgv_block_soft_unsup(c->blk);
    fgv_block_set_soft(c->blk, false);
    return r;
  };
  int rc = run();
  if (resolve_for_retry(c, rc, nblocks, blocks, lens)) {
    rc = run();
  } else if (rc == FGV_OK && unsup && fgv_msp_auto(c)) {
    // identities a channel MSP may hold (the records stay on the device: the call's blocks)
    size_t reg = 0;
    if (fgv_msp_resolve_blocks_locked(c, nblocks, blocks, lens, &reg) == FGV_OK && reg > 0) rc = run();
  }
  return rc;
}

// the shard calls with fgv_set_block_outcomes on: this rank's statuses (LATER from its split on;
// the caller marks unsupported blocks from the final flags and takes n_final's minimum over ranks)
static int shard_dev_outcomes(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                              const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                              void *d_results, size_t results_cap, size_t *ntx) {
  c->blk_status.clear();
  c->n_final = 0;
  uint32_t sp = UINT32_MAX;
  const int rc = shard_dev_soft_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap,
                                       ntx, &sp);
  c->last_rc = rc;
  if (rc) return rc;
  c->n_final = std::min<size_t>(nblocks, sp);
  c->blk_status.assign(nblocks, FGV_OK);
  for (size_t b = c->n_final; b < nblocks; b++) c->blk_status[b] = FGV_BLOCK_LATER;
  return FGV_OK;
}

int fgv_validate_shard_dev_soft(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                const uint32_t *tx_lo, const uint32_t *tx_hi, void *d_results, size_t results_cap,
                                size_t *ntx, uint32_t *split) {
  if (!c || !split || (nblocks && (!blocks || !lens || !ntx || (results_cap && !d_results)))) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->next = fgv_ctx::NextBatch{};
  return shard_dev_soft_locked(c, nblocks, blocks, lens, nullptr, tx_lo, tx_hi, d_results, results_cap, ntx, split);
}

int fgv_validate_shard_dev_pipelined(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                     const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                                     void *d_results, size_t results_cap, size_t *ntx, size_t next_nblocks,
                                     const uint8_t *const *next_blocks, const size_t *next_lens,
                                     const uint8_t *const *next_d_blocks, const uint32_t *next_lo,
                                     const uint32_t *next_hi) {
  if (!c || (nblocks && (!blocks || !lens || !ntx || (results_cap && !d_results))) ||
      (next_nblocks && (!next_blocks || !next_lens)))
    return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  // a host-resident next batch travels H2D now (copy stream) when this batch is host-resident
  // too; a device-resident one (next_d_blocks) is read in place
  c->next = fgv_ctx::NextBatch{next_nblocks, next_blocks,   next_lens, next_lo, next_hi,
                               !next_d_blocks && !d_blocks, next_d_blocks, nullptr};
  int rc;
  if (c->block_outcomes) {
    rc = shard_dev_outcomes(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
  } else {
    c->blk_status.clear();
    rc = shard_dev_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
    if (resolve_for_retry(c, rc, nblocks, blocks, lens))
      rc = shard_dev_locked(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap, ntx);
    c->last_rc = rc;
  }
  if (rc == FGV_OK) stats_accumulate(c);
  c->t_call_end = std::chrono::steady_clock::now();
  if (c->next.n) {  // not started inside (host-parse path, empty batch, early error): start it now
    fgv_block_presplit(c->blk, c->device, c->next.n, c->next.blocks, c->next.lens, c->next.lo, c->next.hi);
  }
  c->next = fgv_ctx::NextBatch{};
  return rc;
}

int fgv_validate_shard_dev_next(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                                void *d_results, size_t results_cap, size_t *ntx, size_t next_nblocks,
                                const uint8_t *const *next_blocks, const size_t *next_lens, const uint32_t *next_lo,
                                const uint32_t *next_hi) {
  return fgv_validate_shard_dev_pipelined(c, nblocks, blocks, lens, d_blocks, tx_lo, tx_hi, d_results, results_cap,
                                          ntx, next_nblocks, next_blocks, next_lens, nullptr, next_lo, next_hi);
}

int fgv_last_ahead(fgv_ctx *c) { return c && c->last_ahead ? 1 : 0; }

int fgv_set_timing(fgv_ctx *c, int on) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->timing = on != 0;
  return FGV_OK;
}

int fgv_set_ahead(fgv_ctx *c, int mode) {
  if (!c || mode < 0 || mode > 4) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  fgv_block_drain(c);  // (a front half already enqueued ahead is discarded)
  c->ahead_mode = mode;
  return FGV_OK;
}

int fgv_presplit(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens, const uint32_t *tx_lo,
                 const uint32_t *tx_hi) {
  if (!c || (nblocks && (!blocks || !lens))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  return fgv_block_presplit(c->blk, c->device, nblocks, blocks, lens, tx_lo, tx_hi);
}

int fgv_host_alloc(fgv_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return FGV_EINVAL;
  *out = nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? FGV_OK : FGV_ENOMEM;
}

int fgv_stream_wait_external(fgv_ctx *c, void *stream) {
  if (!c) return FGV_EINVAL;  // (stream == NULL: the device's null stream)
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  if (!c->ext_ev) HIP_TRY(hipEventCreateWithFlags(&c->ext_ev, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(c->ext_ev, static_cast<hipStream_t>(stream)));
  HIP_TRY(hipStreamWaitEvent(c->stream, c->ext_ev, 0));
  return FGV_OK;
}

int fgv_dev_alloc(fgv_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return FGV_EINVAL;
  *out = nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  return hipMalloc(out, bytes ? bytes : 1) == hipSuccess ? FGV_OK : FGV_ENOMEM;
}

int fgv_dev_upload(fgv_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return FGV_EINVAL;
  if (!bytes) return FGV_OK;
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? FGV_OK : FGV_EDEVICE;
}

int fgv_dev_free(fgv_ctx *c, void *p) {
  if (!c) return FGV_EINVAL;
  if (!p) return FGV_OK;
  {  // (kernels of this context may still read it)
    std::lock_guard<std::mutex> g(c->mu);
    for (hipStream_t x : {c->stream, c->stream2, c->stream3, c->streamF, c->copy_stream, c->streamV})
      if (x) hipStreamSynchronize(x);
  }
  return hipFree(p) == hipSuccess ? FGV_OK : FGV_EINVAL;
}

int fgv_host_free(fgv_ctx *c, void *p) {
  if (!c) return FGV_EINVAL;
  if (!p) return FGV_OK;
  {  // a prefetch may still read it
    std::lock_guard<std::mutex> g(c->mu);
    if (c->copy_stream) hipStreamSynchronize(c->copy_stream);
  }
  return hipHostFree(p) == hipSuccess ? FGV_OK : FGV_EINVAL;
}

int fgv_last_h2d(fgv_ctx *c, uint64_t *copied_bytes, uint64_t *prefetched_blocks) {
  if (!c) return FGV_EINVAL;
  if (copied_bytes) *copied_bytes = c->h2d_bytes;
  if (prefetched_blocks) *prefetched_blocks = c->n_prefetch_hits;
  return FGV_OK;
}

int fgv_last_presplit(fgv_ctx *c) { return c && c->last_presplit ? 1 : 0; }

int fgv_finalize_flags_dev(fgv_ctx *c, size_t nblocks, const size_t *ntx, uint32_t world, size_t rows_per_rank,
                           const void *d_gathered, uint8_t *flags) {
  if (!c || (nblocks && (!ntx || !flags || !d_gathered))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  return finalize_dev_core(c, nblocks, ntx, world, rows_per_rank, static_cast<const uint8_t *>(d_gathered), flags);
}

int fgv_finalize_flags_dev_plan(fgv_ctx *c, size_t nblocks, const size_t *ntx, uint32_t world, size_t rows_per_rank,
                                const uint32_t *rank_lo, const uint32_t *rank_hi, const void *d_gathered,
                                uint8_t *flags) {
  if (!c || (nblocks && (!ntx || !flags || !d_gathered || !rank_lo || !rank_hi))) return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  return finalize_dev_core(c, nblocks, ntx, world, rows_per_rank, static_cast<const uint8_t *>(d_gathered), flags,
                           rank_lo, rank_hi);
}

int fgv_finalize_flags(size_t nblocks, const size_t *ntx, const fgv_tx_result *results, uint8_t *flags) {
  if (nblocks && (!ntx || !flags)) return FGV_EINVAL;
  return fgv_finalize_impl(nblocks, ntx, results, flags);
}

// the running sums of fgv_stats_sums, after a validation call (layout in include/fgv.h)
static void stats_accumulate(fgv_ctx *c) {
  double *a = c->stat_sum;
  a[0] += 1;
  for (int i = 0; i < 12; i++) a[1 + i] += c->t_kern[i];
  a[13] += (double)c->n_pay_blocks;
  a[14] += (double)c->n_sha_blocks;
  a[15] += (double)c->n_verifies;
  a[16] += c->t_sha;
  a[17] += c->t_prep;
  a[18] += c->t_point;
  a[19] += c->t_host_parse;
  a[20] += c->t_host_assemble;
  a[21] += c->t_host_device;
  a[22] += c->t_host_fold;
  a[23] += c->t_gap;
  a[24] += c->t_finish;
}

// Per-block outcomes of a call validated with fgv_set_block_outcomes on: blocks from `split` on
// wait for the commit of the earlier ones (LATER); a block with an undecided transaction (0xFD) is
// unsupported, the others are final.
static void block_outcomes(fgv_ctx *c, size_t nblocks, const size_t *ntx, const uint8_t *flags, uint32_t split) {
  c->blk_status.assign(nblocks, FGV_OK);
  c->n_final = std::min<size_t>(nblocks, split);
  size_t o = 0;
  for (size_t b = 0; b < nblocks; o += ntx[b], b++) {
    if (b >= c->n_final) {
      c->blk_status[b] = FGV_BLOCK_LATER;
      continue;
    }
    size_t k = 0;
    for (size_t t = 0; t < ntx[b]; t++) k += flags[o + t] == 0xFD;
    if (k) c->blk_status[b] = FGV_EUNSUPPORTED;
  }
}

// undecided transactions of the call's final outcomes (counted once, after any rerun)
static void count_unsup_txs(fgv_ctx *c, size_t nblocks, const size_t *ntx, const uint8_t *flags) {
  size_t o = 0;
  for (size_t b = 0; b < nblocks && b < c->blk_status.size(); o += ntx[b], b++)
    if (c->blk_status[b] == FGV_EUNSUPPORTED)
      for (size_t t = 0; t < ntx[b]; t++) c->unsup_txs += flags[o + t] == 0xFD;
}

// TxValidator.Validate of a batch on one GPU: the device-parse pass and the finalize kernels
// (markTXIdDuplicates + the batch's txid index) are queued back to back and the call waits once.
static int validate_blocks_locked(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                  const uint8_t *const *d_blocks, uint8_t *flags, size_t flags_cap, size_t *ntx) {
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  std::vector<const uint8_t *> dev;
  int rc = stage_blocks(c, nblocks, blocks, lens, d_blocks, dev);
  if (rc) return rc;
  if (c->next.n && c->next.prefetch) {
    const fgv_ctx::Prefetch *e = nullptr;
    rc = prefetch_blocks(c, c->next.n, c->next.blocks, c->next.lens, &e);
    if (rc) return rc;
    c->next.d_blocks = e->dev.data();
    c->next.wait = c->stage_ev[e->slot];
  }
  if (fgv_block_parse_mode(c->blk) == 0) {
    // records: at most one per 2 bytes of block data (an envelope's framing), and flags_cap
    size_t bytes = 0;
    for (size_t b = 0; b < nblocks; b++) bytes += lens[b];
    const size_t bound = std::min(flags_cap, bytes / 2 + nblocks);
    if (!c->fz_res.ensure(bound * sizeof(fgv_tx_result) + 64)) return FGV_ENOMEM;
    c->want_early_fin = c->early_fin_on;
    // (the next batch's front half is queued after this batch's finalize: defer_ahead)
    static const bool defer = [] {
      const char *e = getenv("FGV_DEFER_AHEAD");
      return !e || atoi(e) != 0;
    }();
    c->defer_ahead = defer;
    rc = fgv_block_validate_dev_enqueue(c, c->blk, nblocks, blocks, lens, dev.data(), nullptr, nullptr,
                                        c->fz_res.as<fgv_tx_result>(), bound, ntx);
    c->want_early_fin = false;
    c->defer_ahead = false;
    if (rc) {
      fgv_block_launch_deferred_ahead(c, false);
      fgv_block_validate_dev_finish(c, c->blk);  // (waits for anything already queued)
      c->early_fin = c->fold_codes = false;
      return rc;
    }
    size_t total = 0;
    for (size_t b = 0; b < nblocks; b++) total += ntx[b];
    if (total) rc = finalize_dev_core(c, nblocks, ntx, 1, total, c->fz_res.as<uint8_t>(), flags, nullptr, nullptr, true);
    fgv_block_launch_deferred_ahead(c, rc == FGV_OK);
    const int rv = fgv_block_validate_dev_finish(c, c->blk);
    if (rc) return rc;
    if (rv == FGV_OK) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (total) memcpy(flags, c->hb_fflags.p, total);
      return FGV_OK;
    }
    if (rv != 1) return rv;
    // a transaction exceeded a device capacity: the host parser redoes the batch
  }
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) {
    long k = fgv_block_count_txs(blocks[b], lens[b]);
    if (k < 0) return FGV_EINVAL;
    total += (size_t)k;
  }
  if (total > flags_cap) return FGV_EINVAL;
  if (total == 0) {
    for (size_t b = 0; b < nblocks; b++) ntx[b] = 0;
    return FGV_OK;
  }
  if (!c->hb_res.ensure(total * sizeof(fgv_tx_result) + 64) || !c->fz_res.ensure(total * sizeof(fgv_tx_result)))
    return FGV_ENOMEM;
  fgv_tx_result *res = c->hb_res.as<fgv_tx_result>();
  rc = fgv_block_validate_impl(c, c->blk, nblocks, blocks, lens, dev.data(), nullptr, nullptr, res, total, ntx);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->fz_res.p, res, total * sizeof(fgv_tx_result), hipMemcpyHostToDevice, c->stream));
  return finalize_dev_core(c, nblocks, ntx, 1, total, c->fz_res.as<uint8_t>(), flags);
}

int fgv_validate_blocks(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                        const uint8_t *const *d_blocks, uint8_t *flags, size_t flags_cap, size_t *ntx) {
  return fgv_validate_blocks_pipelined(c, nblocks, blocks, lens, d_blocks, flags, flags_cap, ntx, 0, nullptr,
                                       nullptr, nullptr);
}

int fgv_validate_blocks_pipelined(fgv_ctx *c, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                                  const uint8_t *const *d_blocks, uint8_t *flags, size_t flags_cap, size_t *ntx,
                                  size_t next_nblocks, const uint8_t *const *next_blocks, const size_t *next_lens,
                                  const uint8_t *const *next_d_blocks) {
  if (!c || (nblocks && (!blocks || !lens || !flags || !ntx)) || (next_nblocks && (!next_blocks || !next_lens)))
    return FGV_EINVAL;
  if (nblocks == 0) return FGV_OK;
  std::lock_guard<std::mutex> g(c->mu);
  c->next = fgv_ctx::NextBatch{next_nblocks, next_blocks,   next_lens, nullptr, nullptr,
                               !next_d_blocks && !d_blocks, next_d_blocks, nullptr};
  const bool soft = c->block_outcomes;
  // (a failed call leaves no per-block outcomes of an earlier call behind)
  c->blk_status.clear();
  c->n_final = 0;
  auto run = [&] {
    c->blk_status.clear();
    c->n_final = 0;
    fgv_block_set_soft(c->blk, soft);
    const int r = validate_blocks_locked(c, nblocks, blocks, lens, d_blocks, flags, flags_cap, ntx);
    if (soft && r == FGV_OK) block_outcomes(c, nblocks, ntx, flags, fgv_block_split(c->blk));
    fgv_block_set_soft(c->blk, false);
    return r;
  };
  int rc = run();
  if (resolve_for_retry(c, rc, nblocks, blocks, lens)) {
    rc = run();
  } else if (soft && rc == FGV_OK && fgv_msp_auto(c)) {
    // per-block outcomes: identities a channel MSP may hold, in the unsupported blocks only
    std::vector<const uint8_t *> ub;
    std::vector<size_t> ul;
    for (size_t b = 0; b < nblocks; b++)
      if (c->blk_status[b] == FGV_EUNSUPPORTED) ub.push_back(blocks[b]), ul.push_back(lens[b]);
    size_t reg = 0;
    if (!ub.empty() && fgv_msp_resolve_blocks_locked(c, ub.size(), ub.data(), ul.data(), &reg) == FGV_OK && reg > 0)
      rc = run();
  }
  if (rc == FGV_OK) stats_accumulate(c);
  c->t_call_end = std::chrono::steady_clock::now();
  if (soft && rc == FGV_OK) {
    for (size_t b = 0; b < nblocks; b++) c->unsup_blocks += c->blk_status[b] == FGV_EUNSUPPORTED;
    count_unsup_txs(c, nblocks, ntx, flags);
  } else if (rc == FGV_EUNSUPPORTED) {
    c->unsup_batches++;
    c->unsup_blocks += nblocks;
  }
  if (c->next.n)  // not started inside (host-parse path, empty batch, early error): start it now
    fgv_block_presplit(c->blk, c->device, c->next.n, c->next.blocks, c->next.lens, nullptr, nullptr);
  c->next = fgv_ctx::NextBatch{};
  c->last_rc = rc;
  return rc;
}

int fgv_stats_sums(fgv_ctx *c, double *out, size_t n, int reset) {
  if (!c || (n && !out)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  for (size_t i = 0; i < n; i++) out[i] = i < FGV_STAT_SUMS ? c->stat_sum[i] : 0.0;
  if (reset)
    for (double &x : c->stat_sum) x = 0;
  return FGV_OK;
}

int fgv_set_block_outcomes(fgv_ctx *c, int on) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->block_outcomes = on != 0;
  return FGV_OK;
}

int fgv_last_block_status(fgv_ctx *c, int32_t *status, size_t n, size_t *n_final) {
  if (!c || (n && !status)) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  // a call that failed decided nothing: every status is its return code, and so is ours (ADVICE r5:
  // a caller reading the statuses without the call's code must not see final blocks)
  if (c->last_rc != FGV_OK) {
    for (size_t b = 0; b < n; b++) status[b] = c->last_rc;
    if (n_final) *n_final = 0;
    return c->last_rc;
  }
  for (size_t b = 0; b < n; b++) status[b] = b < c->blk_status.size() ? c->blk_status[b] : FGV_OK;
  if (n_final) *n_final = c->n_final;
  return FGV_OK;
}

int fgv_unsupported_stats(fgv_ctx *c, uint64_t *batches, uint64_t *blocks, uint64_t *txs) {
  if (!c) return FGV_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (batches) *batches = c->unsup_batches;
  if (blocks) *blocks = c->unsup_blocks;
  if (txs) *txs = c->unsup_txs;
  return FGV_OK;
}

}  // extern "C"
