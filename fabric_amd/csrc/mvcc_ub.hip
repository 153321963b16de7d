// mvcc_ub.hip -- a committed block's update-batch bytes, built on the device from the MVCC write
// records (the input of the ledger's commit hash), so the host keeps only the serial SHA-256.
//
// Reference: core/ledger/kvledger/kv_ledger.go:806-817 (addBlockCommitHash hashes
// varint(len(filter)) || filter || updateBatchBytes || prevCommitHash) and
// core/ledger/kvledger/txmgmt/txmgr/update_batch_bytes.go:29-105
// (deterministicBytesForPubAndHashUpdates): the puts and deletes of the block's VALID
// transactions at Height{block, tx} (validation/types.go:81-112, tx_ops.go:17-51: a later
// transaction's write of a key replaces an earlier one), namespaces sorted with "" skipped, per
// namespace its public writes sorted by key, then each collection (sorted) with its hashed writes
// sorted by key hash; KVWrite{namespace 1 (first write of a namespace), collection 2 (first write of
// a collection), key 3, is_delete 4, value 5, version_bytes 6} as repeated field 1 of
// txmgr.Updates.  Host restatement: fgv_commit.cpp commit_prefix (and oracle/commithash.py).
//
// k_ub_sort: one workgroup (1,024 lanes) per block, everything in LDS:
//   1. gather: the write records of the block's VALID transactions (MvTxInfo.code 0 and the
//      fixpoint's ST_VALID), a block-wide scan of the per-transaction counts;
//   2. groups: (namespace, hashed, collection) found by leader election (the first unassigned
//      entry's group, compared by every lane; a block has a handful), ranked by one lane;
//   3. sort: 64-bit keys (group rank | 7 key bytes after the prefix every key of the block shares)
//      by a bitonic network over up to UB_MAX entries, ties by the full key, then by transaction;
//   4. the last entry of each key's run survives; sizes, a block-wide scan, one arena claim; the
//      survivors' (record, offset, fields) go to the entry list.
// k_ub_write: one wave per listed entry over the whole chip (the byte framing of ~30 B plus the
// key and value per write: the serialisation's bulk, spread over every CU instead of one per block).
// A block that does not fit (more than UB_MAX valid writes, more than UB_GROUPS groups, the arena
// full) reports status UB_NONE: the host decodes that block instead (fgv_commit.cpp).
#include "fgv_kernels.h"
#include "pbwire_dev.h"

using namespace pbd;

#define UB_T 1024u
#define UB_GROUPS 64u   // (namespace, hashed, collection) groups of one block
#define UB_ST_VALID 1   // mvcc.hip ST_VALID: the fixpoint's verdict for a VALID transaction

namespace {

DEV int s_cmp(S a, S b) {  // byte-lexicographic three-way compare
  const uint32_t m = a.n < b.n ? a.n : b.n;
  for (uint32_t i = 0; i < m; i += 4) {
    const uint32_t k = lo_mask(m - i);
    const uint32_t x = __builtin_bswap32(ld4(a.p + i) & k), y = __builtin_bswap32(ld4(b.p + i) & k);
    if (x != y) return x < y ? -1 : 1;
  }
  return a.n < b.n ? -1 : a.n > b.n ? 1 : 0;
}
DEV S ns_of(const uint8_t *base, const MvRec &r) { return S{base + r.ns_off, r.ns_len}; }
DEV S coll_of(const uint8_t *base, const MvRec &r) { return S{base + r.coll_off, r.coll_len}; }
DEV S key_of(const uint8_t *base, const MvRec &r) { return S{base + r.key_off, r.key_len}; }
DEV bool same_group(const uint8_t *base, const MvRec &a, const MvRec &b) {
  if ((a.flags ^ b.flags) & MVR_HASHED) return false;
  if (!s_eq(ns_of(base, a), ns_of(base, b))) return false;
  return !(a.flags & MVR_HASHED) || s_eq(coll_of(base, a), coll_of(base, b));
}
// group order: namespace, public before hashed, collection (update_batch_bytes.go:47-75)
DEV bool group_lt(const uint8_t *base, const MvRec &a, const MvRec &b) {
  const int c = s_cmp(ns_of(base, a), ns_of(base, b));
  if (c) return c < 0;
  const bool ha = a.flags & MVR_HASHED, hb = b.flags & MVR_HASHED;
  if (ha != hb) return !ha;
  return ha && s_cmp(coll_of(base, a), coll_of(base, b)) < 0;
}
DEV uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) v >>= 7, n++;
  return n;
}
DEV uint32_t field_len(uint32_t n) { return 1u + varint_len(n) + n; }
DEV uint32_t opv_len(uint64_t n) {  // EncodeOrderPreservingVarUint64 (common/ledger/util/util.go:32-52)
  uint32_t k = 0;
  while (k < 8 && (n >> (56 - 8 * k) & 0xFF) == 0) k++;
  return 1u + (8u - k);
}
// KVWrite message length (field 1's payload) of entry r with the namespace / collection fields
// present or not
DEV uint32_t kvwrite_len(const uint8_t *base, const MvRec &r, bool with_ns, bool with_coll, uint32_t vl) {
  uint32_t m = 0;
  if (with_ns && r.ns_len) m += field_len(r.ns_len);
  if (with_coll && r.coll_len) m += field_len(r.coll_len);
  if (r.key_len) m += field_len(r.key_len);
  if (r.flags & MVR_DELETE) m += 2;
  else if (r.txn) m += field_len((uint32_t)r.txn);
  return m + field_len(vl);
}

}  // namespace

__global__ __launch_bounds__(UB_T) void k_ub_sort(const uint8_t *__restrict__ base, const MvRec *__restrict__ writes,
                                                  const MvTxInfo *__restrict__ info, const uint8_t *__restrict__ st,
                                                  const MvCounters *__restrict__ c, uint32_t rlast,
                                                  const uint32_t *__restrict__ bfirst, const uint64_t *__restrict__ bnums,
                                                  uint32_t ntx0, uint64_t num0, uint64_t out_cap,
                                                  unsigned long long *__restrict__ used, UbMeta *__restrict__ meta,
                                                  UbBlk *__restrict__ dmeta, UbEnt *__restrict__ ents) {
  __shared__ uint64_t skey[UB_MAX];
  __shared__ uint32_t sidx[UB_MAX];  // record index (skey: the sort key, then the entry's output offset)
  __shared__ uint8_t sgrp[UB_MAX];
  __shared__ uint32_t wsum[UB_T / 64], grep[UB_GROUPS], gfirst[UB_GROUPS];
  __shared__ uint8_t grank[UB_GROUPS], gnewns[UB_GROUPS], gskip[UB_GROUPS];
  __shared__ uint32_t sh_m, sh_lead, sh_ng, sh_bad, sh_lcp, sh_total;
  __shared__ unsigned long long sh_off;
  __builtin_amdgcn_s_setprio(0);  // (beside the commit and the next call's kernels: off their chains)
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t b = blockIdx.x;
  UbMeta *mo = meta + b;
  UbBlk *dm = dmeta + b;
  UbEnt *ent = ents + (size_t)b * UB_MAX;
  if (tid == 0) dm->nent = 0;  // (k_ub_write: nothing of this block unless it finishes below)
  // the fixpoint converged (mvcc.hip converged()): otherwise a later launch of this block decides
  if (c->unsup || !(c->done || c->undec[rlast & 3] == 0)) {
    if (tid == 0) mo->status = UB_NONE;
    return;
  }
  const uint32_t t0 = bfirst ? bfirst[b] : 0u;
  const uint32_t T = bfirst ? bfirst[b + 1] - t0 : ntx0;
  const uint64_t num = bnums ? bnums[b] : num0;
  if (tid == 0) {
    sh_m = 0;
    sh_bad = 0;
    sh_ng = 0;
    sh_lcp = 0xFFFFFFFFu;
    sh_total = 0;
  }
  __syncthreads();
  // 1. gather
  for (uint32_t q0 = 0; q0 < T; q0 += UB_T) {
    const uint32_t t = t0 + q0 + tid;
    uint32_t cnt = 0, wb = 0;
    if (q0 + tid < T && info[t].code == 0 && st[t] == UB_ST_VALID) {
      cnt = info[t].wcnt;
      wb = info[t].wbeg;
    }
    uint32_t v = cnt;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)v, d);
      if (lane >= d) v += o;
    }
    if (lane == 63u) wsum[wv] = v;
    __syncthreads();
    uint32_t pre = sh_m;
    for (uint32_t k = 0; k < wv; k++) pre += wsum[k];
    pre += v - cnt;
    for (uint32_t q = 0; q < cnt; q++)
      if (pre + q < UB_MAX) sidx[pre + q] = wb + q;
    __syncthreads();
    if (tid == UB_T - 1) sh_m = pre + cnt;
    __syncthreads();
  }
  const uint32_t M = sh_m;
  if (M > UB_MAX) {
    if (tid == 0) mo->status = UB_NONE;
    return;
  }
  // 2. groups by leader election
  for (uint32_t i = tid; i < M; i += UB_T) sgrp[i] = 0xFF;
  __syncthreads();
  for (;;) {
    if (tid == 0) sh_lead = 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t i = tid; i < M; i += UB_T)
      if (sgrp[i] == 0xFF) {
        atomicMin(&sh_lead, i);
        break;
      }
    __syncthreads();
    const uint32_t lead = sh_lead, g = sh_ng;
    if (lead == 0xFFFFFFFFu) break;
    if (g == UB_GROUPS) {
      if (tid == 0) sh_bad = 1;
      break;
    }
    const MvRec L = writes[sidx[lead]];
    for (uint32_t i = tid; i < M; i += UB_T)
      if (sgrp[i] == 0xFF && same_group(base, writes[sidx[i]], L)) sgrp[i] = (uint8_t)g;
    if (tid == 0) {
      grep[g] = sidx[lead];
      sh_ng = g + 1;
    }
    __syncthreads();
  }
  __syncthreads();
  if (sh_bad) {
    if (tid == 0) mo->status = UB_NONE;
    return;
  }
  const uint32_t G = sh_ng;
  if (tid == 0) {  // rank the groups (insertion sort of a handful); "" namespaces are skipped
    uint32_t ord[UB_GROUPS];
    for (uint32_t g = 0; g < G; g++) {
      uint32_t j = g;
      while (j > 0 && group_lt(base, writes[grep[g]], writes[grep[ord[j - 1]]])) {
        ord[j] = ord[j - 1];
        j--;
      }
      ord[j] = g;
    }
    int prev = -1;  // the last written group: a group opens its namespace when the namespace differs
    for (uint32_t r = 0; r < G; r++) {
      const uint32_t g = ord[r];
      const MvRec &R = writes[grep[g]];
      grank[g] = (uint8_t)r;
      gskip[g] = R.ns_len == 0;
      gnewns[g] = 0;
      gfirst[g] = 0xFFFFFFFFu;
      if (gskip[g]) continue;
      gnewns[g] = prev < 0 || !s_eq(ns_of(base, R), ns_of(base, writes[grep[prev]]));
      prev = (int)g;
    }
  }
  // common key prefix of the block (every key shares [0, lcp) with entry 0's key, so the 7 bytes
  // after it order the keys as their full compare does, up to ties)
  if (M) {
    const S k0 = key_of(base, writes[sidx[0]]);
    uint32_t my = 0xFFFFFFFFu;
    for (uint32_t i = tid; i < M; i += UB_T) {
      const S k = key_of(base, writes[sidx[i]]);
      uint32_t l = 0;
      const uint32_t m = min(min(k.n, k0.n), 32u);
      while (l < m && k.p[l] == k0.p[l]) l++;
      my = min(my, l);
    }
    atomicMin(&sh_lcp, my);
  }
  __syncthreads();
  const uint32_t lcp = sh_lcp;
  // 3. sort
  uint32_t N = 1;
  while (N < M) N <<= 1;
  for (uint32_t i = tid; i < N; i += UB_T) {
    if (i < M) {
      const MvRec &R = writes[sidx[i]];
      const S k = key_of(base, R);
      uint64_t v = (uint64_t)grank[sgrp[i]] << 56;
      for (uint32_t j = 0; j < 7; j++) v |= (uint64_t)(lcp + j < k.n ? k.p[lcp + j] : 0) << (48 - 8 * j);
      skey[i] = v;
    } else {
      skey[i] = ~0ull;
      sidx[i] = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  // full order of entries a, b (their keys equal): the key past the shared prefix, then the tx
  auto less = [&](uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) -> bool {
    if (ka != kb) return ka < kb;
    if (ia == 0xFFFFFFFFu || ib == 0xFFFFFFFFu) return ia < ib;
    const MvRec &A = writes[ia], &B = writes[ib];
    const S x = key_of(base, A), y = key_of(base, B);
    const int cm = s_cmp(S{x.p + lcp, x.n - lcp}, S{y.p + lcp, y.n - lcp});
    if (cm) return cm < 0;
    return A.tx < B.tx;
  };
  for (uint32_t k = 2; k <= N; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = tid; i < N; i += UB_T) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint64_t ki = skey[i], kl = skey[l];
          const uint32_t ii = sidx[i], il = sidx[l];
          const bool up = (i & k) == 0;
          if (up ? less(kl, il, ki, ii) : less(ki, ii, kl, il)) {
            skey[i] = kl;
            skey[l] = ki;
            sidx[i] = il;
            sidx[l] = ii;
          }
        }
      }
      __syncthreads();
    }
  // 4. survivors (the last of each key's run), their sizes, the group's first survivor
  for (uint32_t i = tid; i < M; i += UB_T) {
    const MvRec &R = writes[sidx[i]];
    bool last = i + 1 == M || skey[i + 1] != skey[i];
    if (!last) {
      const S x = key_of(base, R), y = key_of(base, writes[sidx[i + 1]]);
      last = !s_eq(x, y);
    }
    uint32_t g = 0;
    for (; g < G; g++)  // (the entry's group by its rank: the sort moved the entries)
      if (grank[g] == (uint32_t)(skey[i] >> 56)) break;
    sgrp[i] = (uint8_t)(last && !gskip[g] ? g : 0xFF);
    if (sgrp[i] != 0xFF) atomicMin(&gfirst[g], i);
  }
  __syncthreads();
  // sizes -> offsets (block-wide scan in chunks), written over skey
  uint32_t carry = 0;
  for (uint32_t q0 = 0; q0 < M; q0 += UB_T) {
    const uint32_t i = q0 + tid;
    uint32_t sz = 0;
    if (i < M && sgrp[i] != 0xFF) {
      const MvRec &R = writes[sidx[i]];
      const uint32_t g = sgrp[i];
      const bool first = gfirst[g] == i;
      const uint32_t vl = opv_len(num) + opv_len(R.tx - t0);
      const uint32_t m = kvwrite_len(base, R, first && gnewns[g], first && (R.flags & MVR_HASHED), vl);
      sz = 1u + varint_len(m) + m;
    }
    uint32_t v = sz;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)v, d);
      if (lane >= d) v += o;
    }
    if (lane == 63u) wsum[wv] = v;
    __syncthreads();
    uint32_t pre = carry;
    for (uint32_t k = 0; k < wv; k++) pre += wsum[k];
    pre += v - sz;
    if (i < M) skey[i] = pre;
    uint32_t tot = carry;
    for (uint32_t k = 0; k < UB_T / 64; k++) tot += wsum[k];
    __syncthreads();
    carry = tot;
  }
  if (tid == 0) {
    sh_total = carry;
    const unsigned long long off = atomicAdd(used, (unsigned long long)carry);
    sh_off = off;
    sh_bad = off + carry > out_cap;
  }
  __syncthreads();
  if (sh_bad) {
    if (tid == 0) mo->status = UB_NONE;
    return;
  }
  // the survivors' entries (sorted order) for k_ub_write
  const uint64_t boff = sh_off;
  for (uint32_t i = tid; i < M; i += UB_T) {
    const uint32_t g = sgrp[i];
    if (g == 0xFF) {
      ent[i] = UbEnt{0, 0, 0};
      continue;
    }
    const bool first = gfirst[g] == i;
    const bool hashed = writes[sidx[i]].flags & MVR_HASHED;
    ent[i] = UbEnt{sidx[i], (uint32_t)skey[i],
                   (first && gnewns[g] ? UBE_NS : 0u) | (first && hashed ? UBE_COLL : 0u) | UBE_LIVE};
  }
  if (tid == 0) {
    *dm = UbBlk{boff, sh_total, M, t0, num};
    mo->off = boff;
    mo->len = sh_total;
    mo->status = UB_OK;
  }
}

// One wave per entry: its ~230 bytes written 64 contiguous bytes per store instruction (a lane per
// byte position), the key and value read the same way -- one cache line per wave-wide access
// instead of 64 scattered ones.  The entry's bytes are segments: literal tag / length bytes (at
// most 6 each), the namespace, collection, key and value copied from the block, and the version
// field (tag, length, EncodeOrderPreservingVarUint64 of the block number and of the tx index).
DEV uint32_t lit_put(uint64_t &w, uint32_t tag, uint32_t n) {  // tag || varint(n) into w -> length
  w = tag;
  uint32_t k = 1;
  while (n >= 0x80) {
    w |= (uint64_t)((n & 0x7F) | 0x80) << (8 * k++);
    n >>= 7;
  }
  w |= (uint64_t)n << (8 * k++);
  return k;
}
DEV uint32_t opv_byte(uint64_t n, uint32_t len, uint32_t q) {  // byte q of opv(n) (len = opv_len(n))
  return q == 0 ? len - 1 : (uint32_t)(n >> (8 * (len - 1 - q))) & 0xFF;
}
// waves of the launch: block q of the launch takes UB_WAVES waves, wave j of them entries j, j + UB_WAVES, ...
#define UB_WAVES 256u
__global__ __launch_bounds__(256) void k_ub_write(const uint8_t *__restrict__ base, const MvRec *__restrict__ writes,
                                                  const UbBlk *__restrict__ dmeta, const UbEnt *__restrict__ ents,
                                                  uint8_t *__restrict__ out) {
  __builtin_amdgcn_s_setprio(0);
  constexpr uint32_t WG_PER_BLOCK = UB_WAVES / 4;
  const uint32_t q = blockIdx.x / WG_PER_BLOCK;
  const uint32_t w0 = (blockIdx.x % WG_PER_BLOCK) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const UbBlk B = dmeta[q];
  const uint32_t lnum = opv_len(B.num);
  for (uint32_t i = w0; i < B.nent; i += UB_WAVES) {
    const UbEnt E = ents[(size_t)q * UB_MAX + i];
    if (!(E.flags & UBE_LIVE)) continue;
    const MvRec R = writes[E.rec];
    const bool wns = (E.flags & UBE_NS) && R.ns_len, wcoll = (E.flags & UBE_COLL) && R.coll_len;
    const uint32_t txn = R.tx - B.t0, ltx = opv_len(txn), vl = lnum + ltx;
    const bool del = R.flags & MVR_DELETE, val = !del && R.txn;
    const uint32_t m = kvwrite_len(base, R, wns, wcoll, vl);
    // segments in order: L0 [L1 C1] [L2 C2] [L3 C3] (L4 | L4 C4) V
    uint64_t l0, l1 = 0, l2 = 0, l3 = 0, l4 = 0;
    const uint32_t n0 = lit_put(l0, 0x0A, m);
    const uint32_t n1 = wns ? lit_put(l1, 0x0A, R.ns_len) : 0, c1 = wns ? R.ns_len : 0;
    const uint32_t n2 = wcoll ? lit_put(l2, 0x12, R.coll_len) : 0, c2 = wcoll ? R.coll_len : 0;
    const uint32_t n3 = R.key_len ? lit_put(l3, 0x1A, R.key_len) : 0, c3 = R.key_len;
    uint32_t n4 = 0, c4 = 0;
    if (del) {
      l4 = 0x0120;  // is_delete = true
      n4 = 2;
    } else if (val) {
      n4 = lit_put(l4, 0x2A, (uint32_t)R.txn);
      c4 = (uint32_t)R.txn;
    }
    const uint32_t s1 = n0, s1c = s1 + n1, s2 = s1c + c1, s2c = s2 + n2, s3 = s2c + c2, s3c = s3 + n3;
    const uint32_t s4 = s3c + c3, s4c = s4 + n4, s5 = s4c + c4, sz = s5 + 2 + vl;
    const uint8_t *pns = base + R.ns_off, *pcoll = base + R.coll_off, *pkey = base + R.key_off, *pval = base + R.blk;
    uint8_t *o = out + B.off + E.off;
    for (uint32_t p = lane; p < sz; p += 64) {
      uint32_t v;
      if (p < s1) v = (uint32_t)(l0 >> (8 * p));
      else if (p < s1c) v = (uint32_t)(l1 >> (8 * (p - s1)));
      else if (p < s2) v = pns[p - s1c];
      else if (p < s2c) v = (uint32_t)(l2 >> (8 * (p - s2)));
      else if (p < s3) v = pcoll[p - s2c];
      else if (p < s3c) v = (uint32_t)(l3 >> (8 * (p - s3)));
      else if (p < s4) v = pkey[p - s3c];
      else if (p < s4c) v = (uint32_t)(l4 >> (8 * (p - s4)));
      else if (p < s5) v = pval[p - s4c];
      else {
        const uint32_t r = p - s5;  // version field: 0x32, vl, opv(num), opv(txn)
        v = r == 0 ? 0x32u : r == 1 ? vl : r - 2 < lnum ? opv_byte(B.num, lnum, r - 2) : opv_byte(txn, ltx, r - 2 - lnum);
      }
      o[p] = (uint8_t)v;
    }
  }
}

void ub_block_launch(hipStream_t s, uint32_t nb, const uint8_t *base, const MvRec *writes, const MvTxInfo *info,
                     const uint8_t *st, const MvCounters *c, uint32_t rlast, const uint32_t *bfirst,
                     const uint64_t *bnums, uint32_t ntx0, uint64_t num0, uint8_t *out, uint64_t out_cap,
                     unsigned long long *used, UbMeta *meta, UbBlk *dmeta, UbEnt *ents) {
  hipLaunchKernelGGL(k_ub_sort, dim3(nb), dim3(UB_T), 0, s, base, writes, info, st, c, rlast, bfirst, bnums, ntx0,
                     num0, out_cap, used, meta, dmeta, ents);
  hipLaunchKernelGGL(k_ub_write, dim3(nb * (UB_WAVES / 4)), dim3(256), 0, s, base, writes, dmeta, ents, out);
}
