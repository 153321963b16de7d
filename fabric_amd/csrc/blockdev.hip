// blockdev.hip -- the committer's per-transaction work on the GPU (see blockdev.h).
//
// Restates, for device code, the host parser of fgv_block.cpp (parse_tx / count_jobs / the
// assembly loop / the fold) rule for rule; the protobuf rules are those of pbwire.h
// (google.golang.org/protobuf v1.33.0 as vendored by the reference).  Reference behaviour:
//   core/committer/txvalidator/v20/validator.go:297-453 (validateTx precedence),
//   core/common/validation/msgvalidation.go:26-320, plugindispatcher/dispatcher.go:102-302,
//   builtin/v20/validation_logic.go:109-217, statebased/validator_keylevel.go:246-260,
//   common/policies/policy.go:363-395, common/cauthdsl/cauthdsl.go:24-92,
//   protoutil/txutils.go:503-534 (GetOrComputeTxIDFromEnvelope for the txid index).
//
// One thread per transaction (k_bd_parse, k_bd_count, k_bd_emit, k_bd_fold) or per identity
// occurrence (k_bd_ident).  These are byte-walking kernels: latency-bound on dependent loads,
// with every transaction of the batch in flight at once.
//

//
// This unit: k_bd_parse, k_bd_ident, k_bd_count (blockdev_lds.hip: the LDS-staged walk, an A/B
// mode; blockdev_sha.hip: the SHA-256 kernels; blockdev_fold.hip: emit, key-level walk, fold).
#include "blockdev_parse.h"

// Global walk: one lane per transaction, the envelope's lines requested up front (touch).
__global__ __launch_bounds__(PL) void k_bd_parse(uint32_t ntx, const uint32_t *__restrict__ envtab,
                                                 const uint64_t *__restrict__ bases, DevChannel ch,
                                                 DevTx *__restrict__ out, uint32_t *__restrict__ flags,
                                                 uint32_t *__restrict__ xhaz, KlDev kl, uint32_t touch) {
  // front half: below the back half's verify chain (3), above k_bd_sha (1); touch bit 8: at 3
  // (FGV_FRONT_PRIO, A/B)
  if (touch & 0x100u) __builtin_amdgcn_s_setprio(3);
  else __builtin_amdgcn_s_setprio(2);
  touch &= 0xFFu;
  __shared__ ParseLdsT<PL> L;
  const uint32_t lane = threadIdx.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;  // (no barrier below: every lane works on its own LDS column)
  const uint32_t *et = envtab + BD_ENV_WORDS * t;
  const uint32_t blk = et[0];
  const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[blk]);
  const S d{base + et[1], et[2]};
  if (touch) touch_lines(d.p, d.n);  // (A/B: FGV_PARSE_TOUCH)
  parse_one<PL>(t, lane, blk, L, base, d, ch, out, flags, xhaz, kl);
}

__global__ __launch_bounds__(256) void k_bd_ident(uint32_t ntx, const DevTx *__restrict__ txs,
                                                  const uint64_t *__restrict__ bases, DevChannel ch,
                                                  int32_t *__restrict__ ident, uint32_t prio) {
  if (prio == 3) __builtin_amdgcn_s_setprio(3);  // (FGV_FRONT_PRIO, A/B)
  else __builtin_amdgcn_s_setprio(2);  // front-half chain; k_bd_sha fills the SIMDs beside it
  // ID_PAR groups per tx (one wave): group g resolves occurrences g, g + ID_PAR, ... -- a C2
  // transaction's creator and endorsers in one pass instead of one after the other
  const uint32_t grp = (blockIdx.x * blockDim.x + threadIdx.x) / ID_LANES;
  const uint32_t t = grp / ID_PAR, g = grp % ID_PAR;
  const uint32_t l = threadIdx.x % ID_LANES;
  if (t >= ntx) return;  // whole groups exit together
  const DevTx &R = txs[t];
  const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
  const uint32_t nend = R.nend;
  for (uint32_t k = g; k <= nend; k += ID_PAR) {
    // the creator is needed when the parse got past the channel check (pre still pending)
    const DSpan sp = k == 0 ? R.creator : R.end_ser[k - 1];
    const bool want = k == 0 ? (R.pre == C_PENDING && sp.len != 0) : true;
    const int32_t res = want ? ident_lookup(absl(base, sp), ch, l) : -1;
    if (l == 0) ident[(size_t)t * BD_OCC + k] = res;
  }
}

// ============================================================ k_bd_count
// creator decision (msgvalidation.go:26-64: deserialize, Validate, then Verify) + count_jobs
DEV void count_jobs(DevTx &R, const DevChannel &ch, const int32_t *id, DevJobIdx &J);
// Job slots are claimed with ONE atomicAdd per workgroup and kind: a wave-inclusive scan by
// shuffles, the waves' totals scanned in LDS, lane q of the first wave adds kind q's workgroup
// total (all kinds' atomics in flight at once).  Slots of a kind stay grouped; their order
// across workgroups is the atomics' order.  (One atomic per wave and kind, issued one kind after
// the other, made this kernel ~55 us of contended atomics on one cache line.)
// With the verify columns given (vc.sig_ptr != null, the default device path) the kernel also
// does k_bd_emit's work: a transaction's creator and endorsement verifies take ONE contiguous
// range of the BJ_C counter (J.base[BJ_C] = the creator's slot, J.base[BJ_E] = the first
// endorsement's, absolute; totals[BJ_E] stays 0, so totals[BJ_C] is the verify count the
// stages behind read), and the thread writes its verify jobs at once -- one launch fewer on the
// committer's chain.
#define BC_THREADS 1024u
__global__ __launch_bounds__(BC_THREADS) void k_bd_count(uint32_t ntx, DevTx *__restrict__ txs, DevChannel ch,
                                                         const int32_t *__restrict__ ident,
                                                         DevJobIdx *__restrict__ jobs, uint32_t *__restrict__ totals,
                                                         uint32_t prio, const uint64_t *__restrict__ bases,
                                                         BdVerifyCols vc) {
  if (prio == 3) __builtin_amdgcn_s_setprio(3);  // (FGV_FRONT_PRIO, A/B)
  else __builtin_amdgcn_s_setprio(2);  // front-half chain; k_bd_sha fills the SIMDs beside it
  __shared__ uint32_t wtot[BJ_KINDS][BC_THREADS / 64], wbase[BJ_KINDS][BC_THREADS / 64];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool fused = vc.sig_ptr != nullptr;
  DevJobIdx J;
  for (int q = 0; q < BJ_KINDS; q++) J.cnt[q] = J.base[q] = 0;
  if (t < ntx) count_jobs(txs[t], ch, ident + (size_t)t * BD_OCC, J);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t incl[BJ_KINDS];
  for (int q = 0; q < BJ_KINDS; q++) {
    // (fused: the endorsements claim inside the creator kind's range)
    uint32_t v = fused ? (q == BJ_C ? J.cnt[BJ_C] + J.cnt[BJ_E] : q == BJ_E ? 0u : J.cnt[q]) : J.cnt[q];
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)v, d);
      if (lane >= d) v += o;
    }
    incl[q] = v;
    if (lane == 63u) wtot[q][w] = v;
  }
  __syncthreads();
  if (w == 0 && lane < BJ_KINDS) {  // lane q: kind q over the workgroup's waves
    const uint32_t q = lane;
    uint32_t run = 0;
    for (uint32_t k = 0; k < BC_THREADS / 64; k++) {
      const uint32_t x = wtot[q][k];
      wtot[q][k] = run;
      run += x;
    }
    wbase[q][0] = run ? atomicAdd(&totals[q], run) : 0u;
  }
  __syncthreads();
  for (int q = 0; q < BJ_KINDS; q++) J.base[q] = wbase[q][0] + wtot[q][w] + incl[q] - J.cnt[q];
  if (fused) {
    const uint32_t v0 = wbase[BJ_C][0] + wtot[BJ_C][w] + incl[BJ_C] - (J.cnt[BJ_C] + J.cnt[BJ_E]);
    J.base[BJ_C] = v0;
    J.base[BJ_E] = v0 + J.cnt[BJ_C];
  }
  if (t >= ntx) return;
  jobs[t] = J;
  if (!fused) return;
  // k_bd_emit's assembly: verify jobs [creator | its endorsements]; digests are k_bd_sha's slots
  const DevTx &R = txs[t];
  const int32_t *id = ident + (size_t)t * BD_OCC;
  const uint64_t base = bases[R.blk];
  auto verify = [&](uint32_t vi, DSpan sig, int32_t slot, uint32_t dig) {
    vc.sig_ptr[vi] = sig.len ? base + sig.off : 0ull;
    vc.sig_len[vi] = sig.len;
    vc.key_slot[vi] = (uint32_t)slot;
    vc.dig_idx[vi] = dig;
  };
  if (J.cnt[BJ_C]) verify(J.base[BJ_C], R.env_sig, ch.idents[id[0]].key_slot, t);
  if (J.cnt[BJ_E]) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < R.nend && r < J.cnt[BJ_E]; k++) {
      const int32_t e = id[1 + k];
      if (e < 0 || ch.idents[e].vclass != 0) continue;
      verify(J.base[BJ_E] + r, R.end_sig[k], ch.idents[e].key_slot, (1 + k) * ntx + t);
      r++;
    }
  }
}
DEV void count_jobs(DevTx &R, const DevChannel &ch, const int32_t *id, DevJobIdx &J) {
  if (R.pre == C_PENDING) {  // DeserializeIdentity -> Validate -> Verify (msgvalidation.go:26-64)
    const int32_t ci = id[0];
    if (ci == -2) R.pre = C_UNSUPPORTED;
    else if (ci < 0 || !ch.idents[ci].valid || ch.idents[ci].vclass == 1) R.pre = C_BAD_CREATOR;
    else if (ch.idents[ci].vclass != 0) R.pre = C_UNSUPPORTED;  // P-384 key
  }
  if ((R.flags & BDF_INDEX_OK) && !(R.flags & BDF_INDEX_FROM_TXID)) J.cnt[BJ_I] = 1;
  if (R.pre == C_PENDING) {
    J.cnt[BJ_C] = 1;
    if (R.type == 3) {
      J.cnt[BJ_T] = 1;
      if (R.etx == C_VALID) {
        J.cnt[BJ_P] = 1;
        if (R.disp == C_VALID) {
          uint32_t ne = 0;
          for (uint32_t k = 0; k < R.nend; k++) {
            const int32_t e = id[1 + k];
            if (e >= 0 && ch.idents[e].vclass == 0) ne++;
          }
          J.cnt[BJ_E] = ne;
        }
      }
    }
  }
}
