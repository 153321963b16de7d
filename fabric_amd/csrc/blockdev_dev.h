// blockdev_dev.h -- device-side helpers shared by the committer kernels (blockdev.hip,
// blockdev_sha.hip, blockdev_fold.hip): wire visitors, channel lookups, key-level records.
// Header-only (anonymous namespace / inline): each translation unit compiles its own kernels.
#pragma once
#include <hip/hip_runtime.h>
#include "fin_dev.h"
#include <stdint.h>

#include "../../include/fgv.h"
#include "blockdev.h"
#include "fgv_kernels.h"
#include "sha256_dev.h"
#include "pbwire_dev.h"

using namespace pbd;

namespace {

enum : uint8_t { C_VALID = 0, C_BAD_PAYLOAD = 2, C_BAD_HDR = 3, C_BAD_CREATOR = 4, C_BAD_ETX = 5,
                 C_UNSUP_PAYLOAD = 7, C_BAD_TXID = 8, C_DUP_TXID = 9, C_POLICY = 10,
                 C_BAD_HDR_EXT = 19, C_BAD_RESP = 21, C_BAD_RWSET = 22, C_ILLEGAL_WS = 23,
                 C_INVALID_CC = 25, C_OTHER = 255, C_PENDING = 0xFE, C_UNSUPPORTED = 0xFD };

// rwset: validated in full; the committer needs namespaces and write presence
struct VVersion {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VKVRead {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    VVersion v;
    return decode(s, v, ovf);
  }
};
struct VQueryReads {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) { VKVRead r; return decode(s, r, ovf); }
};
struct VMerkle {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : n == 3 ? K_REP_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VRangeQuery {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_STRING : n == 3 ? K_VARINT : (n == 4 || n == 5) ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 4) { VQueryReads q; return decode(s, q, ovf); }
    if (n == 5) { VMerkle m; return decode(s, m, ovf); }
    return true;
  }
};
struct VKVWrite {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_VARINT : n == 3 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VMetaEntry {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VMetaWrite {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    VMetaEntry e;
    return decode(s, e, ovf);
  }
};
struct VKVRWSet {
  uint32_t nwrites = 0, nmeta = 0;
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= 4) ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { VKVRead r; return decode(s, r, ovf); }
    if (n == 2) { VRangeQuery q; return decode(s, q, ovf); }
    if (n == 3) { nwrites++; VKVWrite w; return decode(s, w, ovf); }
    nmeta++;
    VMetaWrite m;
    return decode(s, m, ovf);
  }
};
struct VHashRead {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    VVersion v;
    return decode(s, v, ovf);
  }
};
struct VHashWrite {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 3) ? K_BYTES : (n == 2 || n == 4) ? K_VARINT : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VHashMeta {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    VMetaEntry e;
    return decode(s, e, ovf);
  }
};
struct VHashedRWSet {
  uint32_t nwrites = 0, nmeta = 0;
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { VHashRead r; return decode(s, r, ovf); }
    if (n == 2) { nwrites++; VHashWrite w; return decode(s, w, ovf); }
    nmeta++;
    VHashMeta m;
    return decode(s, m, ovf);
  }
};
struct VCollHashed {
  S name{nullptr, 0}, hashed{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : (n == 2 || n == 3) ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) name = s;
    else if (n == 2) hashed = s;
    return true;
  }
};
// k_bd_parse keeps its per-transaction arrays in LDS, element k of lane l at [k][l] (field-major,
// lane-minor): in private memory they were ~2 KB of scratch per lane -- HBM-backed reads in the
// middle of a walk that is one long chain of dependent reads.
#define BD_MAX_COLL 8
#define PL 64u  // lanes per k_bd_parse workgroup (global walk)
template <uint32_t W>  // W walking lanes per workgroup
struct ParseLdsT {
  S ns[BD_MAX_NS][W], rwset[BD_MAX_NS][W], msg[BD_MAX_NS][W];  // TxReadWriteSet namespaces
  S wr[BD_MAX_POL][W];   // written namespaces + the invoked chaincode, sorted
  S coll[BD_MAX_COLL][W];  // a namespace's collection hashed rwsets / collection names
  uint8_t cw[BD_MAX_NS][W];
  int16_t pol[BD_MAX_POL][W];
};
// NsReadWriteSet: namespace, rwset bytes, collection hashed rwsets (kept for the second pass)
struct VNsRwSet {
  S ns{nullptr, 0}, rwset{nullptr, 0};
  uint32_t ncoll = 0;
  S *coll_hashed;  // LDS, stride `stride`
  uint32_t stride;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : n == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { ns = s; return true; }
    if (n == 2) { rwset = s; return true; }
    VCollHashed c;
    if (!decode(s, c, ovf)) return false;
    if (ncoll == BD_MAX_COLL) { ovf = true; return false; }
    coll_hashed[stride * ncoll++] = c.hashed;
    return true;
  }
};
template <uint32_t W>
struct VTxRwSet {
  uint32_t nns = 0;
  ParseLdsT<W> *L;
  uint32_t lane;
  // L->ns / rwset / msg (msg: the NsReadWriteSet, collections re-walked); L->cw bit0: a
  // collection has hashed writes, bit1: a collection failed to decode, bit2: a collection has
  // metadata writes
  DEV Kind kind(uint32_t n) { return n == 1 ? K_VARINT : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    VNsRwSet r;
    r.coll_hashed = &L->coll[0][lane];
    r.stride = W;
    if (!decode(s, r, ovf)) return false;
    if (nns == BD_MAX_NS) { ovf = true; return false; }
    L->ns[nns][lane] = r.ns;
    L->rwset[nns][lane] = r.rwset;
    L->msg[nns][lane] = s;
    uint8_t cw = 0;
    for (uint32_t k = 0; k < r.ncoll; k++) {
      VHashedRWSet h;
      if (!decode(L->coll[k][lane], h, ovf)) { cw |= 2; break; }
      if (h.nwrites) cw |= 1;
      if (h.nmeta) cw |= 4;
    }
    L->cw[nns][lane] = cw;
    nns++;
    return true;
  }
};
// the collections of one NsReadWriteSet with hashed writes, in order (their EPs)
struct VNsCollNames {
  S *names;  // LDS, stride `stride`
  uint32_t stride;
  uint32_t n = 0;
  DEV Kind kind(uint32_t f) { return f == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    VCollHashed c;
    if (!decode(s, c, ovf)) return false;
    VHashedRWSet h;
    if (!decode(c.hashed, h, ovf)) return false;
    if (!h.nwrites) return true;
    if (n == BD_MAX_COLL) { ovf = true; return false; }
    names[stride * n++] = c.name;
    return true;
  }
};
DEV DSpan rel(const uint8_t *base, S s);
// ChaincodeEndorsedAction / ChaincodeActionPayload: endorsements written straight to the
// transaction's record (read only for k < nend, set once the parse succeeds)
struct VEndorsedActionOut {
  S prp{nullptr, 0};
  uint32_t nend = 0;
  const uint8_t *base;
  DevTx *o;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { prp = s; return true; }
    VTwoBytes e;
    if (!decode(s, e, ovf)) return false;
    if (nend == BD_MAX_END) { ovf = true; return false; }
    o->end_ser[nend] = rel(base, e.a);
    o->end_sig[nend] = rel(base, e.b);
    nend++;
    return true;
  }
};
struct VCcActionPayloadOut {
  S ccpp{nullptr, 0};
  bool has_action = false;
  VEndorsedActionOut action;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { ccpp = s; return true; }
    has_action = true;
    return decode(s, action, ovf);
  }
};
struct VSerializedIdentity {
  S mspid{nullptr, 0}, id_bytes{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) { (n == 1 ? mspid : id_bytes) = s; return true; }
};

DEV DSpan rel(const uint8_t *base, S s) { return DSpan{s.n ? (uint32_t)(s.p - base) : 0u, s.n}; }
DEV S absl(const uint8_t *base, DSpan d) { return S{base + d.off, d.len}; }

// chaincode definition lookup (lifecycle ValidationInfo): cc table entry or -1
DEV int cc_find(const DevChannel &ch, S ns) {
  for (uint32_t i = 0; i < ch.ncc; i++) {
    const uint32_t *e = ch.cc + BD_CC_WORDS * i;
    if (e[1] == ns.n && s_eq(S{ch.cc_bytes + e[0], e[1]}, ns)) return (int)i;
  }
  return -1;
}
// a word table of (name off, name len, value): value of `name`, or `dflt`
DEV int32_t name_find(const DevChannel &ch, const uint32_t *tab, uint32_t n, S name, int32_t dflt) {
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t *e = tab + BD_COLL_WORDS * i;
    if (e[1] == name.n && s_eq(S{ch.cc_bytes + e[0], e[1]}, name)) return (int32_t)e[2];
  }
  return dflt;
}
DEV bool msp_known(const DevChannel &ch, S mspid) {
  for (uint32_t i = 0; i < ch.nmsp; i++)
    if (ch.msps[2 * i + 1] == mspid.n && s_eq(S{ch.cc_bytes + ch.msps[2 * i], ch.msps[2 * i + 1]}, mspid)) return true;
  return false;
}

// ------------------------------------------------------------ key-level state keys
// == bd_kl_hash (blockdev.h), word loads
DEV uint64_t kl_hash(S ns, S coll, S key) {
  uint64_t h = bd_mix(0x6A09E667F3BCC908ull, ((uint64_t)ns.n << 32) | coll.n);
  h = bd_mix(h, key.n);
  for (uint32_t j = 0; 4u * j < ns.n; j++) h = bd_mix(h, ld4(ns.p + 4u * j) & lo_mask(ns.n - 4u * j));
  for (uint32_t j = 0; 4u * j < coll.n; j++) h = bd_mix(h, ld4(coll.p + 4u * j) & lo_mask(coll.n - 4u * j));
  for (uint32_t j = 0; 4u * j < key.n; j++) h = bd_mix(h, ld4(key.p + 4u * j) & lo_mask(key.n - 4u * j));
  return h;
}
// the committed VALIDATION_PARAMETER of (ns, coll, key): its policy, -3 (it does not unmarshal),
// -1 none (Channel::kv_policy)
DEV int32_t kvp_find(const DevChannel &ch, uint64_t h, S ns, S coll, S key) {
  if (!ch.kvp) return -1;
  for (uint32_t pos = (uint32_t)h & ch.kvp_mask;; pos = (pos + 1) & ch.kvp_mask) {
    const uint32_t *e = ch.kvp + 8u * pos;
    if (!e[7]) return -1;
    if (e[0] == (uint32_t)h && e[1] == (uint32_t)(h >> 32) && e[3] == ns.n && e[4] == coll.n && e[5] == key.n) {
      const uint8_t *a = ch.kvp_bytes + e[2];
      if (s_eq(S{a, ns.n}, ns) && s_eq(S{a + ns.n, coll.n}, coll) && s_eq(S{a + ns.n + coll.n, key.n}, key))
        return (int32_t)e[6];
    }
  }
}

// The written keys of a TxReadWriteSet that decoded in full (DevTx::results; every decode below
// succeeds): f(ns, coll, key, kind, is_delete) for the public writes (kind 0) and metadata writes
// (1) of each namespace, then each collection's hashed writes (0) and hashed metadata writes (1)
// -- validator_keylevel.go:87-143's four lists (the order does not matter to the callers).
struct KWrite {  // KVWrite / KVWriteHash: key (hash) = 1, is_delete = 2
  S key{nullptr, 0};
  bool del = false;
  bool hashed = false;
  DEV Kind kind(uint32_t n) {
    return n == 1 ? (hashed ? K_BYTES : K_STRING) : (n == 2 || (hashed && n == 4)) ? K_VARINT : n == 3 ? K_BYTES : K_NONE;
  }
  DEV void on_varint(uint32_t n, uint64_t v) {
    if (n == 2) del = v != 0;
  }
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) key = s;
    return true;
  }
};
struct KMeta {  // KVMetadataWrite / KVMetadataWriteHash: key (hash) = 1, entries = 2
  S key{nullptr, 0};
  bool hashed = false;
  DEV Kind kind(uint32_t n) { return n == 1 ? (hashed ? K_BYTES : K_STRING) : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) key = s;
    return true;
  }
};
template <class F>
struct KKeys {  // KVRWSet (writes = 3, metadata_writes = 4) or HashedRWSet (2, 3)
  F *f;
  S ns, coll;
  bool hashed;
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= (hashed ? 3u : 4u)) ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == (hashed ? 2u : 3u)) {
      KWrite w;
      w.hashed = hashed;
      if (!decode(s, w, ovf)) return false;
      (*f)(ns, coll, w.key, 0, w.del);
    } else if (n == (hashed ? 3u : 4u)) {
      KMeta m;
      m.hashed = hashed;
      if (!decode(s, m, ovf)) return false;
      (*f)(ns, coll, m.key, 1, false);
    }
    return true;
  }
};
struct KColl {  // CollectionHashedReadWriteSet: collection_name = 1, hashed_rwset = 2
  S name{nullptr, 0}, hashed{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : (n == 2 || n == 3) ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) name = s;
    else if (n == 2) hashed = s;
    return true;
  }
};
template <class F>
struct KColls {  // NsReadWriteSet.collection_hashed_rwset (3), in order
  F *f;
  S ns;
  DEV Kind kind(uint32_t n) { return n == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    KColl c;
    if (!decode(s, c, ovf)) return false;
    KKeys<F> k{f, ns, c.name, true};
    return decode(c.hashed, k, ovf);
  }
};
struct KNs {  // NsReadWriteSet: namespace = 1, rwset = 2 (collections: KColls)
  S ns{nullptr, 0}, rwset{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : n == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) ns = s;
    else if (n == 2) rwset = s;
    return true;
  }
};
// the keys of one NsReadWriteSet message `nsmsg` whose namespace is `ns` and KVRWSet `kv`
template <class F>
DEV bool ns_keys(S ns, S kv, S nsmsg, F &f, bool &ovf) {
  KKeys<F> k{&f, ns, S{nullptr, 0}, false};
  if (!decode(kv, k, ovf)) return false;
  KColls<F> c{&f, ns};
  return decode(nsmsg, c, ovf);
}
template <class F>
struct KTx {  // TxReadWriteSet: ns_rwset = 2
  F *f;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_VARINT : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    KNs n;
    if (!decode(s, n, ovf)) return false;
    return ns_keys(n.ns, n.rwset, s, *f, ovf);
  }
};
template <class F>
DEV bool tx_keys(S results, F &f, bool &ovf) {
  KTx<F> t{&f};
  return decode(results, t, ovf);
}

// a chained record (k_bd_parse): false when the table is full (host parser)
DEV bool kl_insert(const KlDev &kl, const uint8_t *base, uint32_t t, uint32_t blk, uint32_t kind, S ns, S coll, S key) {
  const uint32_t r = atomicAdd(kl.cnt, 1u);
  if (r >= kl.rcap) return false;
  const uint64_t h = kl_hash(ns, coll, key);
  KlRec &R = kl.rec[r];
  R.hash = h;
  R.tx = t;
  R.blk = blk;
  R.kind = kind;
  R.ns_off = (uint32_t)(ns.p - base);
  R.ns_len = ns.n;
  R.coll_off = coll.n ? (uint32_t)(coll.p - base) : 0u;
  R.coll_len = coll.n;
  R.key_off = key.n ? (uint32_t)(key.p - base) : 0u;
  R.key_len = key.n;
  const unsigned long long old =
      atomicExch(&kl.head[(uint32_t)h & kl.hmask], ((unsigned long long)kl.seq << 32) | (r + 1u));
  R.next = (uint32_t)(old >> 32) == kl.seq ? (uint32_t)old : 0u;
  return true;
}

}  // namespace
