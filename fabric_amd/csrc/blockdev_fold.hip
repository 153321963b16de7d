// blockdev_fold.hip -- the committer's back-half kernels: k_bd_emit (verify job assembly),
// k_bd_kl (key-level dependencies), k_head_pull, k_bd_fold (validateTx precedence, policy
// evaluation, the key-level walk, the finalize codes step).  Shared helpers: blockdev_dev.h.
// Reference: core/committer/txvalidator/v20/validator.go:297-453, common/cauthdsl/cauthdsl.go:24-92,
// common/policies/policy.go:363-395, core/common/validation/statebased/validator_keylevel.go.
#include "blockdev_dev.h"

// ============================================================ k_bd_emit
// the assembly loop: SHA-256 jobs grouped by kind [creator payload | nonce||creator |
// chdr||shdr||ccpp | prp||endorser | index txid], verify jobs [creators | endorsements]
__global__ __launch_bounds__(256) void k_bd_emit(uint32_t ntx, const DevTx *__restrict__ txs,
                                                 const uint64_t *__restrict__ bases, DevChannel ch,
                                                 const int32_t *__restrict__ ident,
                                                 const DevJobIdx *__restrict__ jobs,
                                                 const uint32_t *__restrict__ totals,
                                                 uint64_t *__restrict__ sig_ptr, uint32_t *__restrict__ sig_len,
                                                 uint32_t *__restrict__ key_slot, uint32_t *__restrict__ dig_idx,
                                                 uint32_t *__restrict__ nv_out) {
  __builtin_amdgcn_s_setprio(3);  // latency-critical chain; k_bd_sha fills the SIMDs beside it
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // the verify count, read in device memory by the verify stages enqueued behind this kernel
  if (t == 0) *nv_out = totals[BJ_C] + totals[BJ_E];
  if (t >= ntx) return;
  const DevTx &R = txs[t];
  const DevJobIdx &J = jobs[t];
  const int32_t *id = ident + (size_t)t * BD_OCC;
  const uint64_t base = bases[R.blk];
  auto verify = [&](uint32_t vi, DSpan sig, int32_t slot, uint32_t dig) {
    sig_ptr[vi] = sig.len ? base + sig.off : 0ull;
    sig_len[vi] = sig.len;
    key_slot[vi] = (uint32_t)slot;
    dig_idx[vi] = dig;
  };
  // verify jobs [creators | endorsements]; digests are k_bd_sha's slots
  if (J.cnt[BJ_C]) verify(J.base[BJ_C], R.env_sig, ch.idents[id[0]].key_slot, t);
  if (J.cnt[BJ_E]) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < R.nend && r < J.cnt[BJ_E]; k++) {
      const int32_t e = id[1 + k];
      if (e < 0 || ch.idents[e].vclass != 0) continue;
      verify(totals[BJ_C] + J.base[BJ_E] + r, R.end_sig[k], ch.idents[e].key_slot, (1 + k) * ntx + t);
      r++;
    }
  }
}

// ============================================================ k_bd_fold
namespace {

// cauthdsl greedy evaluation (common/cauthdsl/cauthdsl.go:24-92): SignedBy takes the first
// unused signer satisfying the principal (same MSP; MEMBER = valid, other roles from the role
// bits); NOutOf tries each sub-rule on a copy of `used` and keeps the copy when it succeeds.
// SatisfiesPrincipal of one leaf (fgv_block.cpp prin_sat, MSP v1.4.3): 1 / 0 / 2 (unknown)
DEV int prin_sat(const DevChannel &ch, const DevPrin &p, const DevIdent &I) {
  switch (p.kind) {
    case DPR_ROLE: return I.msp == p.msp && (p.role == 0 ? I.valid != 0 : ((I.roles >> p.role) & 1u) != 0);
    case DPR_IDENTITY: return I.canon == p.canon && I.msp == p.msp && I.valid != 0;
    case DPR_OU: {
      if (I.msp != p.msp || !I.valid) return 0;
      if (!I.ous_known) return 2;
      for (uint32_t k = 0; k < I.ou_n; k++)
        if (ch.ident_ous[I.ou_off + k] == p.ou) return 1;
      return 0;
    }
    case DPR_NOMINAL: return 1;
    case DPR_UNRESOLVED: return 2;
    default: return 0;
  }
}
// the leaves of one SignedBy principal in collectPrincipals order: the first error decides
DEV int principal_sat(const DevChannel &ch, const DevPNode &N, const DevIdent &I) {
  int r = 1;
  for (uint32_t k = 0; k < N.np; k++) {
    const int v = prin_sat(ch, ch.prins[N.p0 + k], I);
    if (v == 0) return 0;
    if (v == 2) r = 2;
  }
  return r;
}
// Iterative DFS; returns -1 on stack overflow, 2 when a principal cannot be decided.
DEV int eval_sig(const DevChannel &ch, const DevPolicy &P, const int32_t *ids, uint32_t nids) {
  struct F {
    uint32_t node, k;
    int32_t verified;
    uint32_t saved;
  };
  F st[16];
  int sp = 0;
  uint32_t used = 0;
  uint32_t node = (uint32_t)P.root;
  int ret = -2;  // -2: descend into `node`; else result of the last finished node (0/1)
  for (;;) {
    if (ret == -2) {
      const DevPNode &N = ch.nodes[node];
      if (N.type == 2) {
        ret = 0;
        for (uint32_t i = 0; i < nids; i++) {
          if ((used >> i) & 1u) continue;
          const int v = principal_sat(ch, N, ch.idents[ids[i]]);
          if (v == 2) return 2;  // (the greedy choice depends on it)
          if (v == 1) {
            used |= 1u << i;
            ret = 1;
            break;
          }
        }
      } else {
        if (sp == 16) return -1;
        st[sp++] = F{node, 0, 0, 0};
        ret = -3;  // start iterating kids
      }
    }
    // ret in {0,1}: a child finished; -3: frame freshly pushed
    if (sp == 0) return ret;
    F &f = st[sp - 1];
    const DevPNode &N = ch.nodes[f.node];
    if (ret >= 0 && f.k > 0) {  // a kid returned
      if (ret == 1) f.verified++;
      else used = f.saved;
    }
    if (f.k < N.nkids) {
      f.saved = used;
      node = ch.kids[N.kid0 + f.k];
      f.k++;
      ret = -2;
      continue;
    }
    ret = f.verified >= N.n ? 1 : 0;
    sp--;
    if (sp == 0) return ret;
  }
}
// 1 satisfied, 0 not, 2 outside the model, -1 device stack overflow (host redo)
DEV int eval_policy(const DevChannel &ch, uint32_t pi, const int32_t *ids, uint32_t nids, int depth) {
  const DevPolicy &P = ch.policies[pi];
  if (P.kind == DP_REJECT) return 0;
  if (P.kind == DP_SIG) {
    if (!P.decode_ok || !P.compile_ok) return 0;
    if (P.needs_roles)
      for (uint32_t i = 0; i < nids; i++)
        if (!ch.idents[ids[i]].roles_known) return 2;
    return eval_sig(ch, P, ids, nids);
  }
  if (P.kind == DP_IMPLICIT && depth == 0) {  // ImplicitMetaPolicy (implicitmeta.go:69-104)
    int32_t ok = 0;
    for (uint32_t q = 0; q < P.nsub; q++) {
      const int v = eval_policy(ch, ch.subs[P.sub0 + q], ids, nids, 1);
      if (v == 2 || v < 0) return v;
      ok += v;
    }
    // threshold 0 (no sub-policies, or an unknown rule): `remaining` starts at 0 and every
    // satisfied sub-policy drives it negative, so only "none satisfied" succeeds
    return (P.threshold == 0 ? ok == 0 : ok >= P.threshold) ? 1 : 0;
  }
  return 2;
}

DEV bool hex32(S s, uint8_t out[32]) {
  if (s.n != 64) return false;
  uint32_t w[8];
  if (hex64_words(s.p, w)) {  // (all loads at once; fin_dev.h)
    for (int k = 0; k < 32; k++) out[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    return true;
  }
  // not all lowercase hex: the byte loop, for the same partial output as the host parser
  for (int k = 0; k < 64; k++) {
    const uint8_t c = s.p[k];
    int v;
    if (c >= '0' && c <= '9') v = c - '0';
    else if (c >= 'a' && c <= 'f') v = c - 'a' + 10;
    else return false;
    if (k & 1) out[k >> 1] |= (uint8_t)v;
    else out[k >> 1] = (uint8_t)(v << 4);
  }
  return true;
}

// d: a 32-byte aligned digest slot; table entries are 32-byte aligned too (word compares)
DEV bool committed(const DevChannel &ch, const uint8_t *d) {
  const uint4 *dv = reinterpret_cast<const uint4 *>(d);
  const uint4 d0 = dv[0], d1 = dv[1];
  if (!(d0.x | d0.y | d0.z | d0.w | d1.x | d1.y | d1.z | d1.w)) return ch.committed_zero != 0;
  if (!ch.committed) return false;
  const uint32_t h = d0.x;  // SHA-256 output: uniform
  for (uint32_t pos = h & ch.committed_mask;; pos = (pos + 1) & ch.committed_mask) {
    const uint4 *ev = reinterpret_cast<const uint4 *>(ch.committed + (size_t)pos * 32);
    const uint4 e0 = ev[0], e1 = ev[1];
    if (!((e0.x ^ d0.x) | (e0.y ^ d0.y) | (e0.z ^ d0.z) | (e0.w ^ d0.w) | (e1.x ^ d1.x) | (e1.y ^ d1.y) |
          (e1.z ^ d1.z) | (e1.w ^ d1.w)))
      return true;
    if (!(e0.x | e0.y | e0.z | e0.w | e1.x | e1.y | e1.z | e1.w)) return false;
  }
}

// the 4 lowercase hex characters of digest bytes 2j and 2j+1, as a little-endian word
DEV uint32_t hex_word(const uint32_t *dw, uint32_t j) {
  const uint32_t two = (dw[j >> 1] >> (16u * (j & 1u))) & 0xFFFFu;
  auto hx = [](uint32_t v) -> uint32_t { return v < 10 ? '0' + v : 'a' + v - 10; };
  return hx((two >> 4) & 15u) | hx(two & 15u) << 8 | hx((two >> 12) & 15u) << 16 | hx((two >> 8) & 15u) << 24;
}

}  // namespace

// ============================================================ k_bd_kl
// Per transaction whose rwset decoded, every written key (oracle keylevel_writes' `touched`)
// against the batch's key-level records (k_bd_parse): a change by an earlier block of the batch
// -> unsupported (flag 2; oracle check_keylevel_batch), and flags[7] = ~(the lowest such block)
// for the per-block outcomes (fgv_set_block_outcomes: blocks from there on are LATER); a metadata write by an earlier
// transaction of its block -> a dependency (validation_parameter_updated): the writer goes to the
// transaction's list and the transaction to its block's dependent list, which k_bd_fold walks in
// block order.  Launched for the fused single-device call only; no records: nothing to do.
// The batch head (envelope table, block bases, counters, key-level words) pulled from the
// host's pinned copy by the GPU itself: 16 B per lane over PCIe, a few microseconds for a
// C2 head, and no copy-engine round trip ahead of the parse (FGV_HEAD_PULL, A/B against the
// hipMemcpyAsync it replaces).
__global__ __launch_bounds__(256) void k_head_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint32_t n16) {
  __builtin_amdgcn_s_setprio(3);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_bd_kl(uint32_t ntx, DevTx *__restrict__ txs,
                                               const uint64_t *__restrict__ bases, KlDev kl,
                                               uint32_t *__restrict__ flags) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx || *kl.cnt == 0) return;
  DevTx &R = txs[t];
  if (!R.results.len) return;
  const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
  uint32_t deps[KL_DEPS];
  uint32_t nd = 0;
  bool over = false, unsup = false;
  auto chk = [&](S ns, S coll, S key, int, bool) {
    const uint64_t h = kl_hash(ns, coll, key);
    const unsigned long long hv = kl.head[(uint32_t)h & kl.hmask];
    if ((uint32_t)(hv >> 32) != kl.seq) return;
    for (uint32_t r = (uint32_t)hv; r;) {
      const KlRec &E = kl.rec[r - 1];
      r = E.next;
      if (E.hash != h || E.blk > R.blk || E.ns_len != ns.n || E.coll_len != coll.n || E.key_len != key.n) continue;
      if (E.blk == R.blk && (E.kind != KL_MD || E.tx >= t)) continue;
      const uint8_t *eb = reinterpret_cast<const uint8_t *>(bases[E.blk]);
      if (!s_eq(S{eb + E.ns_off, ns.n}, ns) || !s_eq(S{eb + E.coll_off, coll.n}, coll) ||
          !s_eq(S{eb + E.key_off, key.n}, key))
        continue;
      if (E.blk < R.blk) {
        unsup = true;
        atomicMax(&flags[7], ~R.blk);  // the first block that must wait for an earlier one's commit
        continue;
      }
      bool seen = false;
      for (uint32_t q = 0; q < nd; q++) seen |= deps[q] == E.tx;
      if (seen) continue;
      if (nd == KL_DEPS) over = true;
      else deps[nd++] = E.tx;
    }
  };
  bool ovf = false;
  if (!tx_keys(absl(base, R.results), chk, ovf) || ovf) over = true;
  if (unsup) atomicOr(flags, 2u);
  if (over) atomicOr(flags, 1u);  // (capacity: host parser)
  if (nd == 0) return;
  for (uint32_t q = 0; q < nd; q++) kl.dep[(size_t)t * KL_DEPS + q] = deps[q];
  R.kln = (uint8_t)nd;
  const uint32_t slot = atomicAdd(&kl.blk[KL_BLK_WORDS * R.blk + 3], 1u);
  if (slot >= KL_MAXDEP) {
    atomicOr(flags, 1u);
    return;
  }
  kl.deplist[(size_t)R.blk * KL_MAXDEP + slot] = t;
}

namespace {
// The dependent transactions of block b in block order (BlockContext.validation_parameter_updated
// restated): once every transaction of the block is folded, each dependent's vscc -- when it
// ran -- fails if an earlier metadata writer's vscc for the namespace returned nil, and cannot be
// decided (the reference waits forever, or Go map order decides) when a writer's never ran or
// ran beside another failing namespace.  A dependent decided here is final before any later one
// reads it.  Codes are the fused finalize's (ledger duplicates of earlier blocks included, before
// markTXIdDuplicates).  Transactions with several vscc namespaces are decided only when the
// answer needs no per-namespace result (a VALID writer); otherwise unsupported.
// a byte another workgroup of this launch wrote (device-coherent load of its word)
DEV uint8_t ld_code(const uint8_t *f, uint32_t i) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(f + (i & ~3u));
  return (uint8_t)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8u * (i & 3u)));
}
__device__ __noinline__ void kl_walk_block(uint32_t b, const DevTx *txs, const KlDev &kl, const FinDev &fin,
                                           fgv_tx_result *res, uint32_t *flags) {
  const uint32_t nd = min(kl.blk[KL_BLK_WORDS * b + 3], (uint32_t)KL_MAXDEP);
  uint32_t list[KL_MAXDEP];
  for (uint32_t i = 0; i < nd; i++) {
    const uint32_t v = kl.deplist[(size_t)b * KL_MAXDEP + i];
    uint32_t j = i;
    for (; j > 0 && list[j - 1] > v; j--) list[j] = list[j - 1];
    list[j] = v;
  }
  for (uint32_t i = 0; i < nd; i++) {
    const uint32_t t = list[i];
    const DevTx &D = txs[t];
    uint8_t code = ld_code(fin.flags, t);
    const bool dfr = code == C_UNSUPPORTED && ld_code(reinterpret_cast<const uint8_t *>(res), (uint32_t)(t * sizeof(fgv_tx_result) + 2));
    const bool ran = code == C_VALID || code == C_POLICY || (D.nwr > 1 && code == C_INVALID_CC) || dfr;
    if (!ran) continue;
    bool upd = false, bad = D.nwr != 1;
    for (uint32_t q = 0; q < D.kln; q++) {
      const uint32_t j = kl.dep[(size_t)t * KL_DEPS + q];
      const uint8_t cj = ld_code(fin.flags, j);
      if (cj == C_VALID) upd = true;              // its vscc of every namespace returned nil
      else if (!(cj == C_POLICY && txs[j].nwr == 1)) bad = true;  // never ran / map order
    }
    if (bad || (dfr && !upd)) {
      code = C_UNSUPPORTED;
      atomicOr(flags, 2u);
    } else if (upd) {
      code = C_POLICY;  // ValidationParameterUpdatedError -> policyErr
    }
    fin.flags[t] = code;
    res[t].code = code;
    res[t].pad[0] = 0;
  }
}
}  // namespace

__global__ __launch_bounds__(256) void k_bd_fold(uint32_t ntx, const DevTx *__restrict__ txs,
                                                 const uint64_t *__restrict__ bases, DevChannel ch,
                                                 const int32_t *__restrict__ ident,
                                                 const DevJobIdx *__restrict__ jobs,
                                                 const uint32_t *__restrict__ totals,
                                                 const uint8_t *__restrict__ digests,
                                                 const uint8_t *__restrict__ vstatus,
                                                 fgv_tx_result *__restrict__ res, uint32_t *__restrict__ flags,
                                                 const uint32_t *__restrict__ xhaz, FinDev fin, KlDev kl,
                                                 uint32_t touch) {
  __builtin_amdgcn_s_setprio(3);  // back half; a next batch's front half may run beside it
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx) return;
  const DevTx &R = txs[t];
  const DevJobIdx &J = jobs[t];
  const int32_t *id = ident + (size_t)t * BD_OCC;
  // digests: k_bd_sha's slots
  const size_t kT = (size_t)BD_DIG_T * ntx + t, kP = (size_t)BD_DIG_P * ntx + t, kI = (size_t)BD_DIG_I * ntx + t;
  if (touch) {  // the lines the fold reads at fixed addresses, all requested at once (FGV_FOLD_TOUCH)
    const uint8_t *dt = reinterpret_cast<const uint8_t *>(&R);
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t o = 0; o < sizeof(DevTx); o += 128) acc ^= *reinterpret_cast<const uint32_t *>(dt + o);
    acc ^= *reinterpret_cast<const uint32_t *>(dt + sizeof(DevTx) - 4);
    acc ^= J.cnt[0] ^ (uint32_t)id[0] ^ *reinterpret_cast<const uint32_t *>(digests + kT * 32) ^
           *reinterpret_cast<const uint32_t *>(digests + kP * 32) ^ *reinterpret_cast<const uint32_t *>(digests + kI * 32);
    asm volatile("" ::"v"(acc));
  }
  const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
  uint8_t code;
  bool reached = false, defer = false;
  const uint8_t *txd = nullptr;
  if (R.pre != C_PENDING) {
    code = R.pre;
  } else if (vstatus[J.base[BJ_C]] != 0) {
    code = C_BAD_CREATOR;
  } else if (R.type == 1) {
    // CONFIG reaching ChannelResources.Apply (validator.go:397-420): the configuration the later
    // blocks validate under changes -- per-block outcomes: they wait (LATER from R.blk + 1)
    code = C_UNSUPPORTED;
    atomicMax(&flags[7], ~(R.blk + 1u));
  } else if (R.type == 2) {
    code = C_UNSUP_PAYLOAD;
  } else {
    txd = digests + kT * 32;
    const S txid = absl(base, R.txid);
    bool ok = txid.n == 64;  // chdr.TxId == hex(SHA-256(nonce || creator)), 16 independent word reads
    if (ok) {
      const uint32_t *dw = reinterpret_cast<const uint32_t *>(txd);
      uint32_t diff = 0;
      for (uint32_t j = 0; j < 16; j++) diff |= ld4(txid.p + 4 * j) ^ hex_word(dw, j);
      ok = diff == 0;
    }
    if (!ok) {
      code = C_BAD_TXID;
    } else if (R.etx != C_VALID) {
      code = R.etx;
    } else {
      const S ph = absl(base, R.prop_hash);
      const uint32_t *pd = reinterpret_cast<const uint32_t *>(digests + kP * 32);
      bool same = ph.n == 32;
      if (same) {
        uint32_t diff = 0;
        for (uint32_t j = 0; j < 8; j++) diff |= ld4(ph.p + 4 * j) ^ pd[j];
        same = diff == 0;
      }
      if (!same) {
        code = C_BAD_ETX;
      } else if ((reached = true, committed(ch, txd))) {
        code = C_DUP_TXID;
      } else if (R.disp != C_VALID) {
        code = R.disp;
      } else if (((R.flags & BDF_VANY) && xhaz[2 * R.blk + 1] <= t) || ((R.flags & BDF_VW) && xhaz[2 * R.blk] <= t)) {
        code = C_UNSUPPORTED;  // the reference panics / waits forever (validator_keylevel.go:184-241)
      } else {
        // SignatureSetToValidIdentities (policy.go:363-395): deserialize, dedup, verify -- when
        // some policy is evaluated
        bool evaluates = false, unsup = false;
        for (uint32_t i = 0; i < R.npol; i++) evaluates |= R.pol[i] >= 0;
        int32_t ids[BD_MAX_END];
        uint32_t seen[BD_MAX_END];
        uint32_t nids = 0, r = 0;
        for (uint32_t k = 0; k < R.nend && evaluates; k++) {
          const int32_t e = id[1 + k];
          if (e == -2) { unsup = true; break; }
          if (e < 0) continue;
          const DevIdent &I = ch.idents[e];
          const bool has_job = I.vclass == 0;
          // (k_bd_count's fused emission leaves totals[BJ_E] at 0 and J.base[BJ_E] absolute; k_bd_emit
          // numbers endorsements after all creators)
          const uint32_t vj = has_job ? (totals[BJ_E] ? totals[0] : 0u) + J.base[BJ_E] + r : 0u;
          if (has_job) r++;
          bool dup = false;
          for (uint32_t q = 0; q < nids; q++) dup |= seen[q] == I.canon;
          if (dup) continue;
          if (I.vclass == 2) { unsup = true; break; }
          if (!has_job || vstatus[vj] != 0) continue;
          seen[nids] = I.canon;
          ids[nids++] = e;
        }
        bool has25 = false, has10 = false, st = false;
        for (uint32_t i = 0; i < R.npol; i++) st |= R.pol[i] == -2;
        code = C_VALID;
        for (uint32_t i = 0; i < R.npol && !unsup; i++) {
          const int pi = R.pol[i];
          if (pi == -2) { unsup = true; break; }
          if (pi < 0) { has25 = true; continue; }
          const int v = eval_policy(ch, (uint32_t)pi, ids, nids, 0);
          if (v < 0) atomicOr(flags, 1u);  // deeper than the device stack: host redo
          if (v == 2) { unsup = true; break; }
          if (v != 1) has10 = true;
        }
        // a dependent transaction whose policies could not be evaluated (an identity or principal
        // outside the model) is decided by the block walk: an updated key fails its vscc before
        // any evaluation matters (validation_parameter_updated)
        defer = unsup && !st && R.kln && kl.on && fin.owner;
        if (unsup) code = C_UNSUPPORTED;
        else if (has25 && has10) code = C_UNSUPPORTED;
        else if (has25) code = C_INVALID_CC;
        else if (has10) code = C_POLICY;
      }
    }
  }
  if (code == C_UNSUPPORTED && !defer) atomicOr(flags, 2u);
  if (fin.owner) {  // k_fin_codes (finalize.hip) for the single-device fused call
    uint32_t slot = 0xFFFFFFFFu;
    uint8_t c2 = code;
    if (reached) {
      uint32_t k[8];
      const uint32_t *dw = reinterpret_cast<const uint32_t *>(txd);
#pragma unroll
      for (int i = 0; i < 8; i++) k[i] = dw[i];
      const int64_t s = fin_find_keys(k, fin_hash(k, fin.seed), fin.owner, fin.keys, fin.mask);
      if (s >= 0) {
        if (fin.minblk[s] < (int32_t)R.blk) c2 = C_DUP_TXID;  // indexed by an earlier block of the batch
        slot = (uint32_t)s;
      }
    }
    if (c2 == C_VALID && slot != 0xFFFFFFFFu) atomicMin(&fin.minvalid[slot], t);
    fin.flags[t] = c2;
    fin.pslot[t] = slot;
  }
  fgv_tx_result o;
  o.code = code;
  o.flags = 0;
  o.pad[0] = defer ? 1 : 0;  // (read by the block walk)
  o.pad[1] = 0;
  for (int k = 0; k < 32; k++) o.txid[k] = o.index_txid[k] = 0;
  if (reached) {
    for (int k = 0; k < 32; k++) o.txid[k] = txd[k];
    o.flags |= FGV_TXR_REACHED;
  }
  if (R.flags & BDF_INDEX_OK) {
    if (!(R.flags & BDF_INDEX_FROM_TXID)) {
      const uint8_t *d = digests + kI * 32;
      for (int k = 0; k < 32; k++) o.index_txid[k] = d[k];
      o.flags |= FGV_TXR_INDEXED;
    } else if (hex32(absl(base, R.index_txid), o.index_txid)) {
      o.flags |= FGV_TXR_INDEXED;
    }
  }
  res[t] = o;
  if (kl.on && *kl.cnt) {  // a batch with key-level changes
    if (!fin.owner) {      // (the ordered walk reads the fused finalize's codes: host parser)
      atomicOr(flags, 1u);
      return;
    }
    __threadfence();
    uint32_t *bw = kl.blk + KL_BLK_WORDS * R.blk;
    if (atomicAdd(&bw[2], 1u) + 1u == bw[1]) {  // the block's last transaction to finish
      __threadfence();
      if (bw[3]) kl_walk_block(R.blk, txs, kl, fin, res, flags);
    }
  }
}
