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

// ============================================================ k_bd_parse
// ChaincodeEndorsedAction decoded for its errors only (the dependency-extraction walk)
struct VEndorsedActionChk {
  S prp{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { prp = s; return true; }
    VTwoBytes e;
    return decode(s, e, ovf);
  }
};
struct VCcActionPayloadChk {
  bool has_action = false;
  VEndorsedActionChk action;  // every occurrence decoded into it (protobuf merge)
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    has_action = true;
    return decode(s, action, ovf);
  }
};
enum : uint8_t { X_OK = 0, X_FAIL = 1, X_PANIC = 2, X_UNKNOWN = 0xFF };
// metadata writes of a TxReadWriteSet (rwset.FromProtoBytes: a decode error -> none); rw_ok:
// the whole rwset decodes
template <uint32_t W>
DEV bool rwset_md(S results, ParseLdsT<W> &L, uint32_t lane, bool &ovf, bool &rw_ok) {
  rw_ok = false;
  VTxRwSet<W> rw;
  rw.L = &L;
  rw.lane = lane;
  if (!decode(results, rw, ovf)) return false;
  bool md = false;
  for (uint32_t k = 0; k < rw.nns; k++) {
    VKVRWSet kv;
    if (!decode(L.rwset[k][lane], kv, ovf) || (L.cw[k][lane] & 2)) return false;
    md |= kv.nmeta != 0 || (L.cw[k][lane] & 4) != 0;
  }
  rw_ok = true;
  return md;
}
// extractDependenciesForTx (validator_keylevel.go:184-222) for a tx whose validation walk
// stopped before its ChaincodeAction (fgv_block.cpp extract_walk); `results`: the rwset bytes
// when X_OK
template <uint32_t W>
DEV uint8_t extract_walk(S d, ParseLdsT<W> &L, uint32_t lane, bool &md, S &results, bool &rw_ok, bool &ovf) {
  md = false;
  rw_ok = false;
  VTwoBytes env;
  if (!decode(d, env, ovf)) return X_FAIL;
  VPayload pl;
  if (!decode(env.a, pl, ovf)) return X_FAIL;
  VTransaction tx;
  if (!decode(pl.data, tx, ovf)) return X_FAIL;
  if (tx.nact == 0) return X_PANIC;
  VCcActionPayloadChk cap;
  if (!decode(tx.first.b, cap, ovf)) return X_FAIL;
  if (!cap.has_action) return X_PANIC;
  VTwoBytes prp;
  if (!decode(cap.action.prp, prp, ovf)) return X_FAIL;
  VCcAction cca;
  if (!decode(prp.b, cca, ovf)) return X_FAIL;
  results = cca.results;
  md = rwset_md(cca.results, L, lane, ovf, rw_ok);
  return X_OK;
}

// fgv_block.cpp parse_tx, speculatively past the creator lookup (resolved by k_bd_ident;
// k_bd_count applies the creator decision before anything downstream reads the rest).
// Key-level endorsement (kl.on): a namespace with committed VALIDATION_PARAMETERs or with
// metadata writes in this tx resolves its policies key by key (sbe_vscc's steps against the
// committed state), and the tx's metadata writes / deletes of parameter-holding keys go to the
// batch's record table (k_bd_kl).  Without kl.on (a shard of a batch) such a tx sends the batch
// to the host parser (flag 1).  Dependency-extraction failures and panics are recorded per block
// (xhaz).
// One transaction t on lane `lane` (its LDS column of L): `base` maps block offsets to bytes --
// the block in HBM, or a "virtual base" into the LDS copy of the envelope (k_bd_parse_lds), so the
// recorded spans stay block-relative either way; d = the envelope.
template <uint32_t W>
DEV void parse_one(uint32_t t, uint32_t lane, uint32_t blk, ParseLdsT<W> &L, const uint8_t *base, S d,
                   const DevChannel &ch, DevTx *__restrict__ out, uint32_t *__restrict__ flags,
                   uint32_t *__restrict__ xhaz, const KlDev &kl) {
  DevTx &O = out[t];  // endorsements are written straight into it; the rest at the end
  struct {
    uint32_t blk;
    uint8_t pre, etx, disp, flags;
    int32_t type;
    DSpan payload, env_sig, nonce, creator, chdr, act_hdr, ccpp, prop_hash, prp, txid;
    DSpan idx_nonce, idx_creator, index_txid;
    uint8_t npol, nend, nwr;
  } R;
  R.blk = blk;
  R.pre = C_PENDING;
  R.etx = C_PENDING;
  R.disp = C_PENDING;
  R.flags = 0;
  R.type = 0;
  const DSpan z{0, 0};
  R.payload = R.env_sig = R.nonce = R.creator = R.chdr = R.act_hdr = R.ccpp = R.prop_hash = R.prp = R.txid = z;
  R.idx_nonce = R.idx_creator = R.index_txid = z;
  R.npol = 0;
  R.nend = 0;
  R.nwr = 0;
  bool ovf = false;
  uint8_t xs = X_UNKNOWN;
  bool md = false, vpns = false, rw_ok = false;
  S results{nullptr, 0};
  do {
    VTwoBytes env;
    if (!decode(d, env, ovf)) { R.pre = C_OTHER; break; }
    VPayload pl;
    if (!decode(env.a, pl, ovf)) { R.pre = C_BAD_PAYLOAD; break; }
    const VTwoBytes &hdr = pl.hdr;
    // txid index value (GetOrComputeTxIDFromEnvelope)
    if (pl.has_header) {
      VChannelHeader c0;
      if (decode(hdr.a, c0, ovf)) {
        if (c0.tx_id.n) {
          R.index_txid = rel(base, c0.tx_id);
          R.flags |= BDF_INDEX_OK | BDF_INDEX_FROM_TXID;
        } else {
          VTwoBytes s0;
          if (decode(hdr.b, s0, ovf)) {
            R.flags |= BDF_INDEX_OK;
            R.idx_nonce = rel(base, s0.b);
            R.idx_creator = rel(base, s0.a);
          }
        }
      }
    }
    if (!pl.has_header) { R.pre = C_BAD_HDR; break; }
    VChannelHeader chdr;
    VTwoBytes shdr;  // creator, nonce
    if (!decode(hdr.a, chdr, ovf) || !decode(hdr.b, shdr, ovf)) { R.pre = C_BAD_HDR; break; }
    if (chdr.type != 3 && chdr.type != 2 && chdr.type != 1) { R.pre = C_BAD_HDR; break; }
    if (chdr.epoch != 0 || shdr.b.n == 0 || shdr.a.n == 0) { R.pre = C_BAD_HDR; break; }
    R.type = chdr.type;
    R.payload = rel(base, env.a);
    R.env_sig = rel(base, env.b);
    R.nonce = rel(base, shdr.b);
    R.creator = rel(base, shdr.a);
    R.chdr = rel(base, hdr.a);
    R.txid = rel(base, chdr.tx_id);
    if (env.b.n == 0) { R.pre = C_BAD_CREATOR; break; }
    if (chdr.channel_id.n == 0) { R.pre = C_UNSUPPORTED; break; }
    if (!s_eq(chdr.channel_id, S{ch.name, ch.name_len})) { R.pre = C_BAD_CREATOR; break; }
    // creator identity: k_bd_ident / k_bd_count
    if (chdr.type != 3) break;

    // validateEndorserTransaction
    R.etx = C_BAD_ETX;
    if (pl.data.n == 0) break;
    VTransaction tx;
    if (!decode(pl.data, tx, ovf) || tx.nact != 1) break;
    VTwoBytes ash;
    if (!decode(tx.first.a, ash, ovf) || ash.b.n == 0 || ash.a.n == 0) break;
    VCcActionPayloadOut cap;
    cap.action.base = base;
    cap.action.o = &O;
    if (!decode(tx.first.b, cap, ovf)) break;
    if (!cap.has_action) { R.etx = C_UNSUPPORTED; break; }
    VTwoBytes prp;  // proposal_hash, extension
    if (!decode(cap.action.prp, prp, ovf)) break;
    if (cap.ccpp.n == 0 || tx.first.a.n == 0) break;
    R.etx = C_VALID;
    R.act_hdr = rel(base, tx.first.a);
    R.ccpp = rel(base, cap.ccpp);
    R.prop_hash = rel(base, prp.a);
    R.prp = rel(base, cap.action.prp);

    // Dispatch
    VHdrExt ext;
    if (!decode(chdr.extension, ext, ovf)) { R.disp = C_BAD_HDR_EXT; break; }
    if (cap.action.prp.n == 0) { R.disp = C_BAD_RESP; break; }
    if (prp.b.n == 0) { R.disp = C_BAD_RESP; break; }
    VCcAction cca;
    if (!decode(prp.b, cca, ovf)) { R.disp = C_BAD_RESP; break; }
    xs = X_OK;  // (the dependency extraction decodes the same messages)
    results = cca.results;
    VTxRwSet<W> rw;
    rw.L = &L;
    rw.lane = lane;
    if (!decode(cca.results, rw, ovf)) { R.disp = C_BAD_RWSET; break; }
    // per namespace: 1 written (kv / metadata / collections), 2 metadata writes, 4 public writes
    uint8_t wflags[BD_MAX_NS];
    bool bad_rw = false;
    for (uint32_t k = 0; k < rw.nns && !bad_rw; k++) {
      VKVRWSet kv;
      if (!decode(L.rwset[k][lane], kv, ovf) || (L.cw[k][lane] & 2)) { bad_rw = true; break; }
      const uint8_t cw = L.cw[k][lane];
      wflags[k] = (uint8_t)(((kv.nwrites || kv.nmeta || (cw & 5)) ? 1 : 0) | ((kv.nmeta || (cw & 4)) ? 2 : 0) |
                            (kv.nwrites ? 4 : 0));
    }
    if (bad_rw) { R.disp = ovf ? C_UNSUPPORTED : C_BAD_RWSET; break; }
    rw_ok = true;
    for (uint32_t k = 0; k < rw.nns; k++) md |= (wflags[k] & 2) != 0;
    if (!ext.has_ccid || !cca.has_ccid) { R.disp = C_OTHER; break; }
    const S ccid = ext.ccid.name;
    if (ccid.n == 0 || !s_eq(ccid, cca.ccid.name) || cca.ccid.version.n == 0) { R.disp = C_INVALID_CC; break; }
    if (cca.events.n != 0) {
      VCcEvent ev;
      if (!decode(cca.events, ev, ovf) || !s_eq(ev.chaincode_id, ccid)) { R.disp = C_OTHER; break; }
    }
    bool dup = false;
    for (uint32_t a = 0; a < rw.nns && !dup; a++)
      for (uint32_t b = a + 1; b < rw.nns; b++)
        if (s_eq(L.ns[a][lane], L.ns[b][lane])) { dup = true; break; }
    if (dup) { R.disp = C_ILLEGAL_WS; break; }
    // written namespaces + the invoked chaincode, sorted (Go string order)
    uint32_t nwr = 0;
    L.wr[nwr++][lane] = ccid;
    for (uint32_t k = 0; k < rw.nns; k++) {
      if (!(wflags[k] & 1)) continue;
      const S nk = L.ns[k][lane];
      if (!s_eq(nk, ccid)) {
        if (nwr == BD_MAX_POL) { ovf = true; break; }
        L.wr[nwr++][lane] = nk;
      }
    }
    if (ovf) break;
    R.nwr = (uint8_t)nwr;
    for (uint32_t i = 1; i < nwr; i++)  // insertion sort
      for (uint32_t j = i; j > 0 && s_lt(L.wr[j][lane], L.wr[j - 1][lane]); j--) {
        const S tmp = L.wr[j][lane];
        L.wr[j][lane] = L.wr[j - 1][lane];
        L.wr[j - 1][lane] = tmp;
      }
    // the EPs each namespace's vscc evaluates (fgv_block.cpp parse_tx restated): -1
    // INVALID_CHAINCODE, -2 outside the model, else a policy index
    uint32_t np = 0;
    auto push = [&](int32_t p) {
      for (uint32_t q = 0; q < np; q++)
        if (L.pol[q][lane] == p) return;
      if (np == BD_MAX_POL) { ovf = true; return; }
      L.pol[np++][lane] = (int16_t)p;
    };
    for (uint32_t i = 0; i < nwr && !ovf; i++) {
      const S wi = L.wr[i][lane];
      const int ci = cc_find(ch, wi);
      const uint32_t *e = ci >= 0 ? ch.cc + BD_CC_WORDS * ci : nullptr;
      if (!e || e[3] == 1) { push(-1); continue; }
      R.flags |= BDF_VANY;
      if (e[3] != 0) { push(-2); continue; }
      const int32_t ep = (int32_t)e[2];
      int k = -1;
      for (uint32_t q = 0; q < rw.nns; q++)
        if (s_eq(L.ns[q][lane], wi)) { k = (int)q; break; }
      if (k >= 0 && (wflags[k] & 1)) {
        R.flags |= BDF_VW;
        vpns |= e[7] != 0;
      }
      if (kl.on && k >= 0 && (e[7] != 0 || (wflags[k] & 2))) {
        // key by key (fgv_block.cpp sbe_vscc against the committed state; an earlier metadata
        // writer of the block is k_bd_kl's and the fold's): its parameter, else the collection
        // EP once, else the chaincode EP once; no key -> the chaincode EP
        bool some = false, cc_checked = false;
        uint32_t ncc = 0;  // collections whose EP was pushed: L.coll[0 .. ncc)
        auto step = [&](S ns, S coll, S key, int, bool) {
          some = true;
          const int32_t pi = kvp_find(ch, kl_hash(ns, coll, key), ns, coll, key);
          if (pi == -3) { push(-2); return; }  // untranslatable: the reference halts
          if (pi >= 0) { push(pi); return; }
          if (coll.n) {
            for (uint32_t c = 0; c < ncc; c++)
              if (s_eq(L.coll[c][lane], coll)) return;
            int32_t cp;
            const uint32_t pl = 14;  // "_implicit_org_"
            if (coll.n >= pl && ld4(coll.p) == 0x706d695fu && ld4(coll.p + 4) == 0x6963696cu &&
                ld4(coll.p + 8) == 0x726f5f74u && (ld4(coll.p + 12) & 0xFFFFu) == 0x5f67u) {
              cp = name_find(ch, ch.impl, ch.nimpl, S{coll.p + pl, coll.n - pl}, -2);
              if (cp == -2) { push(-2); return; }
            } else {
              if (!e[4]) { push(-2); return; }
              cp = name_find(ch, ch.colls + BD_COLL_WORDS * e[5], e[6], coll, -3);
              if (cp == -3) { push(0); return; }  // no such collection -> policyErr
            }
            if (cp >= 0) {
              push(cp);
              if (ncc < BD_MAX_COLL) L.coll[ncc++][lane] = coll;
              return;
            }
          }
          if (!cc_checked) {
            push(ep);
            cc_checked = true;
          }
        };
        if (!ns_keys(L.ns[k][lane], L.rwset[k][lane], L.msg[k][lane], step, ovf)) ovf = true;
        if (!some) push(ep);
        continue;
      }
      bool any = false;
      if (k >= 0 && (wflags[k] & 4)) { push(ep); any = true; }
      if (k >= 0 && (L.cw[k][lane] & 1)) {
        VNsCollNames cn;
        cn.names = &L.coll[0][lane];
        cn.stride = W;
        if (!decode(L.msg[k][lane], cn, ovf)) break;
        for (uint32_t c = 0; c < cn.n; c++) {
          any = true;
          const S nm = L.coll[c][lane];
          if (nm.n == 0) { push(ep); continue; }  // the collection "": public metadata + the chaincode EP
          const uint32_t pl = 14;  // "_implicit_org_" (core/chaincode/implicitcollection/name.go:24-29)
          if (nm.n >= pl && ld4(nm.p) == 0x706d695fu /* _imp */ && ld4(nm.p + 4) == 0x6963696cu /* lici */ &&
              ld4(nm.p + 8) == 0x726f5f74u /* t_or */ && (ld4(nm.p + 12) & 0xFFFFu) == 0x5f67u /* g_ */) {
            push(name_find(ch, ch.impl, ch.nimpl, S{nm.p + pl, nm.n - pl}, -2));
            continue;
          }
          if (!e[4]) { push(-2); continue; }
          const int32_t cep = name_find(ch, ch.colls + BD_COLL_WORDS * e[5], e[6], nm, -3);
          push(cep == -3 ? 0 : cep < 0 ? ep : cep);  // "no such collection" -> reject
        }
      }
      if (!any) push(ep);
    }
    if (ovf) break;
    R.disp = C_VALID;
    R.npol = (uint8_t)np;
    R.nend = (uint8_t)cap.action.nend;
    for (uint32_t q = 0; q < np; q++) O.pol[q] = L.pol[q][lane];
  } while (0);
  if (xs == X_UNKNOWN && !ovf) xs = extract_walk(d, L, lane, md, results, rw_ok, ovf);
  if (xs == X_FAIL) atomicMin(&xhaz[2 * blk], t + 1);
  if (xs == X_PANIC) atomicMin(&xhaz[2 * blk + 1], t + 1);
  if (!rw_ok || xs != X_OK) results = S{nullptr, 0};
  if (kl.on && !ovf && results.n && (md || ch.kvp)) {
    // ExtractValidationParameterDependency's metadata writes, and the deletes that clear a
    // committed parameter (oracle keylevel_writes: the key-level changes of the batch)
    bool full = false;
    auto rec = [&](S ns, S coll, S key, int kind, bool del) {
      if (kind == 1) full |= !kl_insert(kl, base, t, blk, KL_MD, ns, coll, key);
      else if (del && kvp_find(ch, kl_hash(ns, coll, key), ns, coll, key) != -1)
        full |= !kl_insert(kl, base, t, blk, KL_DEL, ns, coll, key);
    };
    if (!tx_keys(results, rec, ovf) || full) ovf = true;
  }
  if (ovf || ch.force_host || (!kl.on && (md || vpns))) atomicOr(flags, 1u);  // capacity / a shard: host parser
  O.blk = R.blk;
  O.pre = R.pre;
  O.etx = R.etx;
  O.disp = R.disp;
  O.flags = R.flags;
  O.type = R.type;
  O.payload = R.payload;
  O.env_sig = R.env_sig;
  O.nonce = R.nonce;
  O.creator = R.creator;
  O.chdr = R.chdr;
  O.act_hdr = R.act_hdr;
  O.ccpp = R.ccpp;
  O.prop_hash = R.prop_hash;
  O.prp = R.prp;
  O.txid = R.txid;
  O.idx_nonce = R.idx_nonce;
  O.idx_creator = R.idx_creator;
  O.index_txid = R.index_txid;
  O.npol = R.npol;
  O.nend = R.nend;
  O.nwr = R.nwr;
  O.kln = 0;
  O.results = rel(base, results);
}

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

// ============================================================ k_bd_ident
// ID_LANES lanes per (tx, occurrence): occurrence 0 = creator, 1..nend = endorsers.
// Channel::lookup restated: decode SerializedIdentity (mspid UTF-8), hash, probe, exact compare.
// The compare is split over the group's lanes a 32-bit word at a time (block bytes at any
// alignment via v_alignbyte; registry fields are 4-byte aligned), then one ballot.
#define ID_LANES 16u
#define ID_PAR BD_ID_PAR
DEV uint32_t ldu32(const uint8_t *p) {  // unaligned little-endian word (reads the next word too)
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}
DEV uint32_t tail_mask(uint32_t n, uint32_t j) {  // bytes of word j inside [0, n)
  const uint32_t r = n - 4u * j;
  return r >= 4u ? 0xFFFFFFFFu : ((1u << (8u * r)) - 1u);
}
DEV uint64_t ident_hash_dev(S msp, S idb) {  // == bd_ident_hash (blockdev.h), word loads
  uint64_t h = bd_ident_hash_msp(msp.p, msp.n, idb.n);
  const uint32_t T = idb.n < BD_HASH_TAIL ? idb.n : BD_HASH_TAIL;
  const uint8_t *s = idb.p + (idb.n - T);
  for (uint32_t j = 0; 4u * j < T; j++) h = bd_mix(h, ldu32(s + 4u * j) & tail_mask(T, j));
  return bd_mix(h, 0x5A);
}
// every lane of the group calls this with the same spans; `b` is 4-byte aligned
DEV bool group_eq(S a, S b, uint32_t l) {
  if (a.n != b.n) return false;
  uint32_t diff = 0;
  const uint32_t *bw = reinterpret_cast<const uint32_t *>(b.p);
  for (uint32_t j = l; 4u * j < a.n; j += ID_LANES) diff |= (ldu32(a.p + 4u * j) ^ bw[j]) & tail_mask(a.n, j);
  const uint64_t bal = __ballot(diff != 0u);
  const uint32_t lane = threadIdx.x & 63u;
  return ((bal >> (lane & ~(ID_LANES - 1u))) & ((1ull << ID_LANES) - 1ull)) == 0ull;
}
// Channel::lookup of one SerializedIdentity (every lane of a 16-lane group calls it with the same
// span): the registry index, -1 (deserialize error / undeserializable key) or -2 (a certificate of
// a channel MSP that was never registered: outside the engine)
DEV int32_t ident_lookup(S ser, const DevChannel &ch, uint32_t l) {
  VSerializedIdentity sid;
  bool ovf = false;
  if (!decode(ser, sid, ovf)) return -1;
  const uint64_t h = ident_hash_dev(sid.mspid, sid.id_bytes);
  // (an empty registry has no table: every identity of a channel MSP is a miss)
  for (uint32_t pos = (uint32_t)h & ch.ident_mask; ch.nident; pos = (pos + 1) & ch.ident_mask) {
    const uint32_t e = ch.ident_table[pos];
    if (e == 0) break;
    const uint32_t i = e - 1;
    if (ch.ident_hash[i] != h) continue;
    const DevIdent &I = ch.idents[i];
    if (group_eq(sid.mspid, S{ch.ident_bytes + I.msp_off, I.msp_len}, l) &&
        group_eq(sid.id_bytes, S{ch.ident_bytes + I.idb_off, I.idb_len}, l))
      return I.vclass == 3 ? -1 : (int32_t)i;  // undeserializable key: deserialize error
  }
  return msp_known(ch, sid.mspid) ? -2 : -1;
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

// LDS-staged walk: one 64-lane workgroup per TPW transactions.  The wave first copies the
// group's envelopes into LDS -- 16-byte loads of the aligned lines covering [off, off + len + 8)
// (the walk's over-read contract), every line in flight at once -- then lane j walks transaction
// j from LDS through a virtual base, so each of the walk's dependent loads is an LDS access
// instead of a cache round trip (the global walk pays ~0.5-1 us per field).  An envelope larger
// than CAP bytes is walked from global memory.
// ident (nullable): k_bd_ident's work in the same workgroup once the walks are done -- the
// creator and endorser SerializedIdentities of the group's transactions (bytes in LDS when
// staged) resolved against the HBM registry by four 16-lane groups at a time, the 56 lanes the
// walk leaves idle -- so the front half has one kernel fewer on its chain.
template <uint32_t TPW, uint32_t CAP>
__global__ __launch_bounds__(64) void k_bd_parse_lds(uint32_t ntx, const uint32_t *__restrict__ envtab,
                                                     const uint64_t *__restrict__ bases, DevChannel ch,
                                                     DevTx *__restrict__ out, uint32_t *__restrict__ flags,
                                                     uint32_t *__restrict__ xhaz, KlDev kl,
                                                     int32_t *__restrict__ ident) {
  __builtin_amdgcn_s_setprio(2);
  constexpr uint32_t C16 = CAP / 16;  // 16-byte lines per staged envelope
  __shared__ ParseLdsT<TPW> L;
  __shared__ uint4 env[TPW * C16];
  __shared__ uint32_t pre[TPW + 1];
  __shared__ uint64_t src[TPW];  // aligned source line of each staged envelope
  const uint32_t lane = threadIdx.x, t0 = blockIdx.x * TPW;
  uint32_t my = 0;
  if (lane < TPW && t0 + lane < ntx) {
    const uint32_t *et = envtab + BD_ENV_WORDS * (t0 + lane);
    const uint64_t a = bases[et[0]] + et[1];
    const uint64_t a0 = a & ~15ull, a1 = (a + et[2] + 8u + 15u) & ~15ull;
    if (a1 - a0 <= CAP) {
      my = (uint32_t)((a1 - a0) / 16u);
      src[lane] = a0;
    }
  }
  uint32_t v = my;  // inclusive prefix over the TPW lanes (wave scan)
  for (uint32_t dd = 1; dd < TPW; dd <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, dd);
    if (lane >= dd) v += o;
  }
  if (lane < TPW) pre[lane + 1] = v;
  if (lane == 0) pre[0] = 0;
  __syncthreads();
  const uint32_t total = pre[TPW];
  // 8 lines per lane per pass, all loads issued before the first LDS store
  constexpr uint32_t U = 8;
  for (uint32_t i0 = lane; i0 < total; i0 += 64 * U) {
    uint4 val[U];
    uint32_t dst[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t i = i0 + 64 * u;
      dst[u] = 0xFFFFFFFFu;
      if (i < total) {
        uint32_t j = 0;  // the envelope of line i: pre[j] <= i < pre[j + 1]
#pragma unroll
        for (uint32_t b = TPW / 2; b > 0; b >>= 1)
          if (pre[j + b] <= i) j += b;
        const uint32_t k = i - pre[j];
        val[u] = reinterpret_cast<const uint4 *>(src[j])[k];
        dst[u] = j * C16 + k;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (dst[u] != 0xFFFFFFFFu) env[dst[u]] = val[u];
  }
  __syncthreads();
  __shared__ const uint8_t *vbase[TPW];  // each transaction's walk base (LDS virtual base or block)
  __shared__ DSpan occ[TPW][BD_OCC];     // its creator and endorser SerializedIdentity spans
  __shared__ uint32_t nocc[TPW];         // 1 + endorsements (0: no transaction)
  __shared__ uint32_t want0[TPW];        // the creator is needed (the parse got past the channel check)
  const uint32_t t = t0 + lane;
  if (lane < TPW && t < ntx) {
    const uint32_t *et = envtab + BD_ENV_WORDS * t;
    const uint32_t blk = et[0];
    const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[blk]);
    if (my) {  // the virtual base: block offset o -> env + (o - (a0 - block))
      const uint64_t a0 = src[lane];
      base = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(&env[lane * C16]) -
                                               (uintptr_t)(a0 - bases[blk]));
    } else {
      touch_lines(base + et[1], et[2]);
    }
    parse_one<TPW>(t, lane, blk, L, base, S{base + et[1], et[2]}, ch, out, flags, xhaz, kl);
    if (ident) {
      const DevTx &O = out[t];  // (written by this lane)
      const uint32_t ne = O.nend;
      vbase[lane] = base;
      nocc[lane] = 1 + ne;
      want0[lane] = O.pre == C_PENDING && O.creator.len != 0;
      occ[lane][0] = O.creator;
      for (uint32_t k = 0; k < ne; k++) occ[lane][1 + k] = O.end_ser[k];
    }
  } else if (ident && lane < TPW) {
    nocc[lane] = 0;
  }
  if (!ident) return;
  __syncthreads();
  // k_bd_ident's lookups: group g of 16 lanes takes (transaction, occurrence) pairs g, g + 4, ...
  const uint32_t g = lane / ID_LANES, l = lane % ID_LANES;
  for (uint32_t p = g; p < TPW * BD_OCC; p += 64u / ID_LANES) {
    const uint32_t j = p / BD_OCC, k = p % BD_OCC;
    if (k >= nocc[j]) continue;  // (uniform within the group)
    const bool want = k == 0 ? want0[j] != 0 : true;
    const int32_t res = want ? ident_lookup(absl(vbase[j], occ[j][k]), ch, l) : -1;
    if (l == 0) ident[(size_t)(t0 + j) * BD_OCC + k] = res;
  }
}

void bd_parse_lds_launch(uint32_t tpw, hipStream_t st, uint32_t ntx, const uint32_t *envtab, const uint64_t *bases,
                         const DevChannel &ch, DevTx *out, uint32_t *flags, uint32_t *xhaz, const KlDev &kl,
                         int32_t *ident) {
  if (tpw == 16)
    hipLaunchKernelGGL((k_bd_parse_lds<16, 4352>), dim3((ntx + 15) / 16), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
  else if (tpw == 4)
    hipLaunchKernelGGL((k_bd_parse_lds<4, 4352>), dim3((ntx + 3) / 4), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
  else
    hipLaunchKernelGGL((k_bd_parse_lds<8, 4352>), dim3((ntx + 7) / 8), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
}

// ============================================================ k_bd_count
// creator decision (msgvalidation.go:26-64: deserialize, Validate, then Verify) + count_jobs
DEV void count_jobs(DevTx &R, const DevChannel &ch, const int32_t *id, DevJobIdx &J);
// Job slots are claimed with ONE atomicAdd per workgroup and kind: a wave-inclusive scan by
// shuffles, the waves' totals scanned in LDS, lane q of the first wave adds kind q's workgroup
// total (all kinds' atomics in flight at once).  Slots of a kind stay grouped; their order
// across workgroups is the atomics' order.  (One atomic per wave and kind, issued one kind after
// the other, made this kernel ~55 us of contended atomics on one cache line.)
#define BC_THREADS 1024u
__global__ __launch_bounds__(BC_THREADS) void k_bd_count(uint32_t ntx, DevTx *__restrict__ txs, DevChannel ch,
                                                         const int32_t *__restrict__ ident,
                                                         DevJobIdx *__restrict__ jobs, uint32_t *__restrict__ totals,
                                                         uint32_t prio) {
  if (prio == 3) __builtin_amdgcn_s_setprio(3);  // (FGV_FRONT_PRIO, A/B)
  else __builtin_amdgcn_s_setprio(2);  // front-half chain; k_bd_sha fills the SIMDs beside it
  __shared__ uint32_t wtot[BJ_KINDS][BC_THREADS / 64], wbase[BJ_KINDS][BC_THREADS / 64];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  DevJobIdx J;
  for (int q = 0; q < BJ_KINDS; q++) J.cnt[q] = J.base[q] = 0;
  if (t < ntx) count_jobs(txs[t], ch, ident + (size_t)t * BD_OCC, J);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t incl[BJ_KINDS];
  for (int q = 0; q < BJ_KINDS; q++) {
    uint32_t v = J.cnt[q];
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
  if (t < ntx) jobs[t] = J;
}
DEV void count_jobs(DevTx &R, const DevChannel &ch, const int32_t *id, DevJobIdx &J) {
  if (R.pre == C_PENDING) {  // DeserializeIdentity -> Validate -> Verify (msgvalidation.go:26-64)
    const int32_t ci = id[0];
    if (ci == -2) R.pre = C_UNSUPPORTED;
    else if (ci < 0 || !ch.idents[ci].valid || ch.idents[ci].vclass == 1) R.pre = C_BAD_CREATOR;
    else if (ch.idents[ci].vclass != 0) R.pre = C_UNSUPPORTED;  // P-384 key / SHA3 MSP
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

// ============================================================ k_bd_sha_payload
// SHA-256(Envelope.payload) of every envelope -- the creator signature's digest
// (msgvalidation.go:26-64 -> msp/identities.go:179), digest slot 0 -- launched on the second
// stream BEFORE the parse: it decodes the Envelope (two fields, the same rules and visitor as
// k_bd_parse) and hashes field 1.  Each payload is its transaction's longest message (~58
// compressions for C2), a serial chain; a batch has far fewer chains (16k) than the chip has
// lanes, so the kernel is bound by ONE chain's latency, not by throughput.  Each chain is
// therefore split over two waves of a workgroup on two SIMDs (64 payloads per workgroup):
//   wave 1 (schedule): loads block b+1 (one block ahead), expands W[0..63] and writes
//                      KW[t] = W[t] + K[t] to LDS (double-buffered, [t/4][lane] x 16 B)
//   wave 0 (rounds):   the 64 rounds of block b from LDS (16 x ds_read_b128)
// one barrier per block.  The rounds wave carries ~950 VALU instructions per compression
// instead of ~1,650 for the whole compression in one lane.
#define PAY_KW_BYTES (2 * 16 * 64 * 16)
__device__ __forceinline__ void pay_view(uint32_t ntx, uint32_t t, const uint32_t *envtab, const uint64_t *bases,
                                         JobView &v, uint32_t &nblk) {
  nblk = 0;
  v.p[0] = v.p[1] = v.p[2] = nullptr;
  v.beg[0] = v.beg[1] = v.beg[2] = v.beg[3] = v.L = 0;
  if (t >= ntx) return;
  const uint32_t *et = envtab + BD_ENV_WORDS * t;
  VTwoBytes env;
  bool ovf = false;
  if (!decode(S{reinterpret_cast<const uint8_t *>(bases[et[0]]) + et[1], et[2]}, env, ovf)) return;
  v.p[0] = v.p[1] = v.p[2] = env.a.p;
  v.beg[1] = v.beg[2] = v.beg[3] = v.L = env.a.n;
  nblk = (v.L + 8) / 64 + 1;
}

__global__ __launch_bounds__(128) void k_bd_sha_payload(uint32_t ntx, const uint32_t *__restrict__ envtab,
                                                        const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                        unsigned long long *__restrict__ nblk_total) {
  // the longest serial chains of the batch: first in issue order
  __builtin_amdgcn_s_setprio(2);
  __shared__ uint4 KW[2][16][64];  // [buffer][t / 4][lane]: KW[t] = W[t] + K[t] of one block
  const uint32_t lane = threadIdx.x & 63u;
  const bool sched = threadIdx.x >= 64;  // wave-uniform
  const uint32_t t = blockIdx.x * 64 + lane;
  JobView v;
  uint32_t nblk;
  pay_view(ntx, t, envtab, bases, v, nblk);
  uint32_t maxb = nblk;
  for (int off = 32; off > 0; off >>= 1) maxb = max(maxb, (uint32_t)__shfl_xor((int)maxb, off));
  if (sched) {
    // ---- schedule wave: block b's words (fetched one block ahead), expansion, KW to LDS
    uint32_t raw[17], sh = 0;
    bool fast = false;
    auto fetch = [&](uint32_t b) {
      const uint32_t s0 = b * 64;
      const int k = s0 < v.beg[1] ? 0 : (s0 < v.beg[2] ? 1 : 2);
      fast = s0 + 64 <= span_end(v, k);
      if (fast) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(span_p(v, k) + (s0 - span_beg(v, k)));
        const __attribute__((address_space(1))) uint32_t *al =
            reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(a & ~(uintptr_t)3);
        sh = (uint32_t)(a & 3u);
#pragma unroll
        for (int q = 0; q < 17; q++) raw[q] = al[q];
      }
    };
    auto produce = [&](uint32_t b) {
      if (b >= nblk) return;
      uint32_t w[16];
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        job_block(v, b, nblk, w);
      }
      if (b + 1 < nblk) fetch(b + 1);
      uint4 *o = &KW[b & 1][0][lane];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int i = 4 * q + j;
          uint32_t wi;
          if (i < 16) {
            wi = w[i];
          } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
          }
          kw[j] = wi + SHA_K[i];
        }
        o[q * 64] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
      }
    };
    if (nblk) fetch(0);
    produce(0);
    __syncthreads();
#pragma unroll 1
    for (uint32_t b = 0; b < maxb; b++) {
      if (b + 1 < maxb) produce(b + 1);
      __syncthreads();
    }
    return;
  }
  // ---- rounds wave
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  __syncthreads();
#pragma unroll 1
  for (uint32_t b = 0; b < maxb; b++) {
    if (b < nblk) {
      const uint4 *in = &KW[b & 1][0][lane];
      uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint4 x = in[q * 64];
        const uint32_t kw4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
          const uint32_t ch = (e & f) ^ (~e & g);
          const uint32_t t1 = k + S1 + ch + kw4[j];
          const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
          const uint32_t mj = (a & bb) | (c & (a | bb));
          k = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + S0 + mj;
        }
      }
      h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
    }
    __syncthreads();
  }
  if (nblk) {
    uint32_t *o = reinterpret_cast<uint32_t *>(dig + (size_t)t * 32);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
  }
  uint64_t blocks = nblk;
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_total, (unsigned long long)blocks);
}

// ============================================================ k_bd_sha
// Every other SHA-256 message of the batch, hashed speculatively right after the parse on the
// third stream (beside identity resolution and the job counts): all of them are spans the parse
// already found; only WHETHER a digest is consumed is decided later (a hash is pure, so a
// superset of the consumed ones is hashed).  Digest slots (BD_DIG_SLOTS x ntx, slot-major):
//   0                      SHA-256(e.Payload): k_bd_sha_payload (msgvalidation.go:26-64)
//   1 + k (k < BD_MAX_END) SHA-256(prp || endorser_k) (statebased/validator_keylevel.go:246-260)
//   BD_DIG_T               SHA-256(nonce || creator): TxID (protoutil/proputils.go:351-360)
//   BD_DIG_P               SHA-256(chdr || shdr || ccpp): proposal hash (protoutil/txutils.go:449-466)
//   BD_DIG_I               SHA-256(nonce || creator) of the txid index entry (txutils.go:503-534)
// A transaction's endorsement messages share the prefix prp: the SHA-256 state after its H =
// floor(|prp| / 64) whole blocks (the midstate) is the same for all of them.  SHA_GROUP = 3 lanes
// per transaction, 21 transactions per wave:
//   lane 0: prp || endorser_0 in full (its state after block H-1 is the midstate), then the
//           tails (blocks H.. from the midstate) of endorsements 3, 6, ...
//   lane 1: nonce || creator (TxID), then the tails of endorsements 1, 4, ...
//   lane 2: chdr || shdr || ccpp, the index txid message when needed, then the tails 2, 5, ...
// Lanes run in lockstep, one compression per step; at step H every lane of the group copies
// lane 0's state (cross-lane read), so a tail never starts before step H.  For C2 this is ~33
// steps per wave in 750 waves instead of 7 lanes per tx in 1750 -- the prp prefix is hashed once
// instead of once per endorsement, and the waves fit beside the payload hashes on the SIMDs.
#define SHA_GROUP 3u  // lanes per transaction (SHA_GPW groups per wave, blockdev.h; lane 63 idles)
namespace {
// one message (or its tail) of a lane: up to three spans held as scalars (an indexed array of
// span pointers would be placed in scratch)
struct ShaSeg {
  uint64_t a, b, c;    // span addresses
  uint32_t la, lb, lc; // span lengths; message = a || b || c, L = la + lb + lc
  uint32_t b0, nblk;   // blocks [b0, nblk) of the padded message
  uint32_t slot;       // digest slot
  bool mid;            // starts from the midstate (b0 = H)
  bool ok;
};
DEV void seg_set(ShaSeg &g, const uint8_t *base, DSpan x, DSpan y, DSpan z, uint32_t slot) {
  g.a = (uint64_t)(uintptr_t)(base + x.off);
  g.b = (uint64_t)(uintptr_t)(base + y.off);
  g.c = (uint64_t)(uintptr_t)(base + z.off);
  g.la = x.len;
  g.lb = y.len;
  g.lc = z.len;
  g.slot = slot;
  g.ok = true;
}
// segment s of lane r of transaction R (ok = false: the lane's list ended)
DEV ShaSeg lane_seg(const DevTx &R, const uint8_t *base, uint32_t r, uint32_t s, uint32_t H, bool live_t, bool live_p,
                    bool live_i, uint32_t nE) {
  ShaSeg g{};
  const DSpan z{0, 0};
  uint32_t nfull = 0;  // full messages ahead of this lane's tails
  if (r == 0) {
    if (nE > 0) {
      if (s == 0) seg_set(g, base, R.prp, R.end_ser[0], z, 1);
      nfull = 1;
    }
  } else if (r == 1) {
    if (live_t) {
      if (s == 0) seg_set(g, base, R.nonce, R.creator, z, BD_DIG_T);
      nfull = 1;
    }
  } else {
    if (live_p) {
      if (s == nfull) seg_set(g, base, R.chdr, R.act_hdr, R.ccpp, BD_DIG_P);
      nfull++;
    }
    if (live_i) {
      if (s == nfull) seg_set(g, base, R.idx_nonce, R.idx_creator, z, BD_DIG_I);
      nfull++;
    }
  }
  if (!g.ok && s >= nfull) {  // tails: endorsements k = r + 3 j (lane 0 hashed k = 0 in full)
    const uint32_t k = r + SHA_GROUP * (s - nfull + (r == 0 ? 1u : 0u));
    if (k < nE) {
      seg_set(g, base, R.prp, R.end_ser[k], z, 1 + k);
      g.b0 = H;
      g.mid = true;
    }
  }
  if (g.ok) g.nblk = (g.la + g.lb + g.lc + 8) / 64 + 1;
  return g;
}
// choose one of three values by masks (a select chain on a position would be turned into a
// table in scratch indexed by the span number)
DEV uint64_t pick3(bool c0, bool c1, uint64_t x0, uint64_t x1, uint64_t x2) {
  const uint64_t m0 = 0ull - (uint64_t)c0, m1 = (0ull - (uint64_t)c1) & ~m0, m2 = ~(m0 | m1);
  return (x0 & m0) | (x1 & m1) | (x2 & m2);
}
// message byte q (padding: 0x80 at L, zeros after)
DEV uint32_t seg_byte(const ShaSeg &g, uint32_t q) {
  const uint32_t L = g.la + g.lb + g.lc;
  if (q >= L) return q == L ? 0x80u : 0u;
  const bool in_a = q < g.la, in_b = q < g.la + g.lb;
  const uint64_t p = pick3(in_a, in_b, g.a + q, g.b + (q - g.la), g.c + (q - g.la - g.lb));
  return *reinterpret_cast<const uint8_t *>(p);
}
// block `blk` of g: the span holding all 64 bytes (fast: 17 raw dwords + byte shift) or not
DEV void seg_fetch(const ShaSeg &g, uint32_t blk, uint32_t raw[17], uint32_t &sh, bool &fast) {
  const uint32_t s = blk * 64, ab = g.la + g.lb;
  const bool in_a = s + 64 <= g.la, in_b = s >= g.la && s + 64 <= ab;
  fast = in_a || in_b || (s >= ab && s + 64 <= ab + g.lc);
  const uint64_t p = pick3(in_a, in_b, g.a + s, g.b + (s - g.la), g.c + (s - ab));
  if (fast) {
    const __attribute__((address_space(1))) uint32_t *al =
        reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(p & ~(uint64_t)3);
    sh = (uint32_t)(p & 3u);
#pragma unroll
    for (int q = 0; q < 17; q++) raw[q] = al[q];
  }
}
// big-endian message word at byte position pos: one unaligned dword load when the word lies
// inside a span, bytes only when it straddles a span boundary or the end (0x80, then zeros)
DEV uint32_t seg_word(const ShaSeg &g, uint32_t pos) {
  const uint32_t L = g.la + g.lb + g.lc;
  if (pos >= L) return pos == L ? 0x80000000u : 0u;
  const bool in_a = pos < g.la, in_b = pos < g.la + g.lb;
  const uint64_t p = pick3(in_a, in_b, g.a + pos, g.b + (pos - g.la), g.c + (pos - g.la - g.lb));
  const uint32_t room = (uint32_t)pick3(in_a, in_b, g.la - pos, g.la + g.lb - pos, L - pos);
  if (room >= 4) return __builtin_bswap32(ld_u32(reinterpret_cast<const uint8_t *>(p)));
  uint32_t w = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) w = (w << 8) | seg_byte(g, pos + q);
  return w;
}
// a block that is not inside one span (span boundaries, the padding and length)
DEV void seg_block_slow(const ShaSeg &g, uint32_t blk, uint32_t w[16]) {
  const uint32_t s = blk * 64;
#pragma unroll
  for (int k = 0; k < 16; k++) w[k] = seg_word(g, s + 4 * k);
  if (blk == g.nblk - 1) {
    const uint64_t bits = (uint64_t)(g.la + g.lb + g.lc) * 8;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}
}  // namespace

DEV void bd_sha_body(uint32_t ntx, const DevTx *__restrict__ txs, const uint64_t *__restrict__ bases,
                     uint8_t *__restrict__ dig, unsigned long long *__restrict__ nblk_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t grp = lane / SHA_GROUP, r = lane - grp * SHA_GROUP;
  const uint32_t t = blockIdx.x * SHA_GPW + grp;
  const bool in = grp < SHA_GPW && t < ntx;
  uint32_t H = 0, nE = 0;
  bool live_t = false, live_p = false, live_i = false;
  const uint8_t *base = nullptr;
  ShaSeg g;
  g.ok = false;
  if (in) {
    const DevTx &R = txs[t];
    base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
    const bool live = R.pre == C_PENDING;
    live_t = live && R.type == 3;
    live_p = live_t && R.etx == C_VALID;
    live_i = (R.flags & BDF_INDEX_OK) && !(R.flags & BDF_INDEX_FROM_TXID);
    nE = (live_p && R.disp == C_VALID) ? R.nend : 0u;
    H = R.prp.len / 64;
    g = lane_seg(R, base, r, 0, H, live_t, live_p, live_i, nE);
  }
  uint32_t s = 0, blk = g.ok ? g.b0 : 0;
  uint32_t h[8], mid[8];
  const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = mid[k] = IV[k];
  uint64_t blocks = 0;
  uint32_t raw[17], sh = 0, w[16];
  bool fast = false;
  if (g.ok) seg_fetch(g, blk, raw, sh, fast);
  const int src = (int)(grp * SHA_GROUP);  // lane 0 of the group
#pragma unroll 1
  for (uint32_t step = 0;; step++) {
    // the midstate: lane 0's state after its first H blocks (every lane runs the reads)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (uint32_t)__shfl((int)h[k], src);
      if (step == H) mid[k] = v;
    }
    const bool waiting = g.ok && g.mid && step < H;
    if (__ballot(g.ok) == 0ull) break;
    if (g.ok && !waiting) {
      if (blk == g.b0 && g.mid) {
#pragma unroll
        for (int k = 0; k < 8; k++) h[k] = mid[k];
      }
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        seg_block_slow(g, blk, w);
      }
      // the lane's next block (or the next segment's first), fetched while this one compresses
      ShaSeg gn = g;
      uint32_t bn = blk + 1;
      bool next_seg = bn >= g.nblk;
      if (next_seg) {
        gn = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        bn = gn.ok ? gn.b0 : 0;
      }
      if (gn.ok) seg_fetch(gn, bn, raw, sh, fast);
      sha_compress(h, w);
      blocks++;
      if (next_seg) {
        uint32_t *o = reinterpret_cast<uint32_t *>(dig + ((size_t)g.slot * ntx + t) * 32);
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = __builtin_bswap32(h[k]);
        g = gn;
        s++;
        if (g.ok && !g.mid) {  // (a tail takes the midstate at its first block)
#pragma unroll
          for (int k = 0; k < 8; k++) h[k] = IV[k];
        }
      }
      blk = bn;
    }
  }
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_out, (unsigned long long)blocks);
}
// ---- the same hashes, each lane's chain split over two waves of a workgroup on two SIMDs
// (k_bd_sha_payload's scheme): wave 1 (schedule) walks the lanes' segments exactly as
// bd_sha_body does, fetches each step's block one step ahead, expands the message schedule and
// writes KW[t] = W[t] + K[t] to LDS (double-buffered, [t/4][lane] x 16 B); wave 0 (rounds) runs
// the 64 rounds from LDS, takes the midstate, writes the digests.  One barrier per step; both
// waves run the same number of steps: a lane's last step is max(full blocks, H) + tail blocks.
DEV uint32_t lane_steps(const DevTx &R, const uint8_t *base, uint32_t r, uint32_t H, bool live_t, bool live_p,
                        bool live_i, uint32_t nE) {
  uint32_t pos = 0;
  for (uint32_t s = 0;; s++) {
    const ShaSeg g = lane_seg(R, base, r, s, H, live_t, live_p, live_i, nE);
    if (!g.ok) return pos;
    if (g.mid && pos < H) pos = H;
    pos += g.nblk - g.b0;
  }
}

DEV void bd_sha_split_body(uint32_t ntx, const DevTx *__restrict__ txs, const uint64_t *__restrict__ bases,
                           uint8_t *__restrict__ dig, unsigned long long *__restrict__ nblk_out) {
  __shared__ uint4 KW[2][16][64];  // [buffer][t / 4][lane]
  const uint32_t lane = threadIdx.x & 63u;
  const bool sched = threadIdx.x >= 64;  // wave-uniform
  const uint32_t grp = lane / SHA_GROUP, r = lane - grp * SHA_GROUP;
  const uint32_t t = blockIdx.x * SHA_GPW + grp;
  const bool in = grp < SHA_GPW && t < ntx;
  uint32_t H = 0, nE = 0, nsteps = 0;
  bool live_t = false, live_p = false, live_i = false;
  const uint8_t *base = nullptr;
  ShaSeg g;
  g.ok = false;
  if (in) {
    const DevTx &R = txs[t];
    base = reinterpret_cast<const uint8_t *>(bases[R.blk]);
    const bool live = R.pre == C_PENDING;
    live_t = live && R.type == 3;
    live_p = live_t && R.etx == C_VALID;
    live_i = (R.flags & BDF_INDEX_OK) && !(R.flags & BDF_INDEX_FROM_TXID);
    nE = (live_p && R.disp == C_VALID) ? R.nend : 0u;
    H = R.prp.len / 64;
    g = lane_seg(R, base, r, 0, H, live_t, live_p, live_i, nE);
    nsteps = lane_steps(R, base, r, H, live_t, live_p, live_i, nE);
  }
  uint32_t maxs = nsteps;
  for (int off = 32; off > 0; off >>= 1) maxs = max(maxs, (uint32_t)__shfl_xor((int)maxs, off));
  uint32_t s = 0, blk = g.ok ? g.b0 : 0;
  if (sched) {
    // ---- schedule wave
    uint32_t raw[17], sh = 0;
    bool fast = false;
    if (g.ok) seg_fetch(g, blk, raw, sh, fast);
    auto produce = [&](uint32_t step) {
      if (!g.ok || (g.mid && step < H)) return;
      uint32_t w[16];
      if (fast) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh));
      } else {
        seg_block_slow(g, blk, w);
      }
      ShaSeg gn = g;
      uint32_t bn = blk + 1;
      if (bn >= g.nblk) {
        gn = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        bn = gn.ok ? gn.b0 : 0;
        s++;
      }
      if (gn.ok) seg_fetch(gn, bn, raw, sh, fast);
      g = gn;
      blk = bn;
      uint4 *o = &KW[step & 1][0][lane];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int i = 4 * q + j;
          uint32_t wi;
          if (i < 16) {
            wi = w[i];
          } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
          }
          kw[j] = wi + SHA_K[i];
        }
        o[q * 64] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
      }
    };
    if (maxs) produce(0);
    __syncthreads();
#pragma unroll 1
    for (uint32_t step = 0; step < maxs; step++) {
      if (step + 1 < maxs) produce(step + 1);
      __syncthreads();
    }
    return;
  }
  // ---- rounds wave
  const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t h[8], mid[8];
#pragma unroll
  for (int k = 0; k < 8; k++) h[k] = mid[k] = IV[k];
  uint64_t blocks = 0;
  const int src = (int)(grp * SHA_GROUP);  // lane 0 of the group
  __syncthreads();
#pragma unroll 1
  for (uint32_t step = 0; step < maxs; step++) {
    // the midstate: lane 0's state after its first H blocks (every lane runs the reads)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t v = (uint32_t)__shfl((int)h[k], src);
      if (step == H) mid[k] = v;
    }
    if (g.ok && !(g.mid && step < H)) {
      if (blk == g.b0 && g.mid) {
#pragma unroll
        for (int k = 0; k < 8; k++) h[k] = mid[k];
      }
      const uint4 *in4 = &KW[step & 1][0][lane];
      uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], gg = h[6], k = h[7];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const uint4 x = in4[q * 64];
        const uint32_t kw4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
          const uint32_t ch = (e & f) ^ (~e & gg);
          const uint32_t t1 = k + S1 + ch + kw4[j];
          const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
          const uint32_t mj = (a & bb) | (c & (a | bb));
          k = gg; gg = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + S0 + mj;
        }
      }
      h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += gg; h[7] += k;
      blocks++;
      uint32_t bn = blk + 1;
      if (bn >= g.nblk) {
        uint32_t *o = reinterpret_cast<uint32_t *>(dig + ((size_t)g.slot * ntx + t) * 32);
#pragma unroll
        for (int q = 0; q < 8; q++) o[q] = __builtin_bswap32(h[q]);
        g = lane_seg(txs[t], base, r, s + 1, H, live_t, live_p, live_i, nE);
        s++;
        bn = g.ok ? g.b0 : 0;
        if (g.ok && !g.mid) {  // (a tail takes the midstate at its first block)
#pragma unroll
          for (int q = 0; q < 8; q++) h[q] = IV[q];
        }
      }
      blk = bn;
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) blocks += __shfl_down(blocks, off);
  if (lane == 0 && blocks) atomicAdd(nblk_out, (unsigned long long)blocks);
}
__global__ __launch_bounds__(128) void k_bd_sha2(uint32_t ntx, const DevTx *__restrict__ txs,
                                                 const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                 unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(1);
  bd_sha_split_body(ntx, txs, bases, dig, nblk_out);
}

// k_prep waits for these digests and for the parse -> identities -> counts -> emit -> der ->
// inv chain: the wave priority decides which of the two finishes first (FGV_SHA_PRIO A/B)
__global__ __launch_bounds__(64) void k_bd_sha(uint32_t ntx, const DevTx *__restrict__ txs,
                                               const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                               unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(1);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}
__global__ __launch_bounds__(64) void k_bd_sha_p2(uint32_t ntx, const DevTx *__restrict__ txs,
                                                  const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                  unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(2);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}
__global__ __launch_bounds__(64) void k_bd_sha_p3(uint32_t ntx, const DevTx *__restrict__ txs,
                                                  const uint64_t *__restrict__ bases, uint8_t *__restrict__ dig,
                                                  unsigned long long *__restrict__ nblk_out) {
  __builtin_amdgcn_s_setprio(3);
  bd_sha_body(ntx, txs, bases, dig, nblk_out);
}

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
    code = C_UNSUPPORTED;
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
          const uint32_t vj = has_job ? totals[0] + J.base[BJ_E] + r : 0u;
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
