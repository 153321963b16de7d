// mvcc.hip -- MVCC validation of a block on the GPU (gfx950): rwset extraction, the committed
// version check, the intra-block read/write conflict fixpoint and the commit, all on the device.
//
// Reference semantics (core/ledger/kvledger/txmgmt/validation):
//   batch_preparer.go:192-286  preprocessProtoBlock: committer-invalid txs are skipped;
//        GetActionFromEnvelope errors -> NIL_TXACTION(16); rwset unmarshal errors ->
//        INVALID_OTHER_REASON(255)
//   validator.go:81-200        in block order, tx i is MVCC_READ_CONFLICT(11) if a read key was
//        written by an EARLIER VALID tx of the block (updates.Exists) or the committed version
//        differs from the read version (version.AreSame, nil <=> absent)
//   validator.go:246-293       hashed (private-data) reads are point reads of the key hash in
//        ns + "$$h" + coll (privacyenabledstate/db.go:355-357)
//   types.go:81-112, tx_ops.go:17-51  valid write sets enter `updates` at Height{blk, tx};
//        IsKVWriteDelete / IsKVWriteHashDelete (rwsetutil/rwset_proto_util.go:366-375)
//
// Pipeline of one block (one H2D head copy, one D2H tail copy, no host sync in between):
//   k_mvx_extract one lane per tx: envelope -> ... -> TxReadWriteSet walk (pbwire_dev.h rules),
//                 codes 16 / 255 / unsupported, read/write counts, record ranges claimed by
//                 wave-aggregated atomics, then the same walk again by the same lane (cache hits)
//                 writing 48-byte records + 64-bit tags; duplicate writes of one key in one tx
//                 (tx_ops.go:183-191 adds flags: undefined semantics) -> unsupported
//   k_mvx_prep    writes -> block write table (claim by CAS, epoch-tagged: never cleared);
//                 reads  -> committed-state table, static version check
//   k_mvx_find    reads -> write-table slot; initial state per tx + round-1 first writers
//   k_mvx_round   one launch per fixpoint round (enqueued speculatively; a converged round
//                 exits at once): every undecided tx decides from round r's first writers,
//                 every non-invalid tx publishes its writes for round r+1 (double buffered)
//   k_mvx_flags   TRANSACTIONS_FILTER codes
//   k_mv_last / k_mv_upsert_find / k_mv_upsert_insert   commit: the last valid writer of each
//                 key updates or inserts the committed-state entry
//
// Fixpoint (validity is sequential; decided by a monotone fixpoint over per-key first writers):
//   st[i] in {UNDEC, VALID, INVALID}; INVALID initially for static conflicts / parse codes.
//   Round r: fw_cand(k)  = min{ j : st[j] != INVALID, k in W_j },
//            fw_valid(k) = min{ j : st[j] == VALID,   k in W_j };
//            undecided i -> INVALID if some read key k has fw_valid(k) < i,
//                        -> VALID   if every read key k has fw_cand(k) >= i.
//   The lowest undecided tx is always decided, so rounds <= longest alternating chain.
#include "fgv_kernels.h"
#include "mvcc_multi.h"
#include "pbwire_dev.h"

using namespace pbd;

#define ST_UNDEC 0
#define ST_VALID 1
#define ST_INVALID 2
#define FW_INF 0xFFFFFFFFu

// ------------------------------------------------------------------ keys and tags
// A key is (namespace, key bytes); a private-data key's namespace is ns + "$$h" + coll.  The
// tag hashes the flattened namespace, a separator and the key (FNV-1a 64 + a finalizer); the
// committed-state arena stores the flattened namespace followed by the key.
// (bytes in order, read a word at a time: the loads are independent, the FNV chain is ALU)
__device__ __forceinline__ uint64_t th(uint64_t h, const uint8_t *p, uint32_t n) {
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const uint32_t w = ld4(p + i);
    h = (h ^ (w & 0xFFu)) * 0x100000001b3ull;
    h = (h ^ ((w >> 8) & 0xFFu)) * 0x100000001b3ull;
    h = (h ^ ((w >> 16) & 0xFFu)) * 0x100000001b3ull;
    h = (h ^ (w >> 24)) * 0x100000001b3ull;
  }
  for (; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  return h;
}
__device__ __forceinline__ uint64_t th_fin(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h | MV_TAG_OCC;  // never 0 (empty)
}
__device__ __forceinline__ uint64_t rec_tag(const uint8_t *base, const MvRec &r) {
  uint64_t h = th(0xcbf29ce484222325ull, base + r.ns_off, r.ns_len);
  if (r.flags & MVR_HASHED) {
    const uint8_t sep[3] = {'$', '$', 'h'};
    h = th(h, sep, 3);
    h = th(h, base + r.coll_off, r.coll_len);
  }
  h = (h ^ 0xFFu) * 0x100000001b3ull;  // (0xFF never occurs in UTF-8 namespace strings)
  return th_fin(th(h, base + r.key_off, r.key_len));
}
__device__ __forceinline__ uint32_t flat_ns_len(const MvRec &r) {
  return r.ns_len + ((r.flags & MVR_HASHED) ? 3u + r.coll_len : 0u);
}
// a word at a time (ld4: any alignment; block arenas, key staging and the state arena carry
// >= 8 bytes of tail slack)
__device__ __forceinline__ bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
  uint32_t diff = 0;
  for (uint32_t i = 0; i < n; i += 4) diff |= (ld4(a + i) ^ ld4(b + i)) & lo_mask(n - i);
  return diff == 0;
}
// record == committed-state entry (flattened namespace + key at arena offset)
__device__ __forceinline__ bool rec_eq_state(const uint8_t *base, const MvRec &r, const StateSlot &s,
                                             const uint8_t *arena) {
  if (s.ns_len != flat_ns_len(r) || s.key_len != r.key_len) return false;
  // a short key from the slot's own line (MV_INLINE), a longer one from the arena
  const uint8_t *a = (uint32_t)s.ns_len + s.key_len <= MV_INLINE ? s.ik : arena + ((uint64_t)s.off8 << 3);
  if (!bytes_eq(a, base + r.ns_off, r.ns_len)) return false;
  a += r.ns_len;
  if (r.flags & MVR_HASHED) {
    if (a[0] != '$' || a[1] != '$' || a[2] != 'h') return false;
    if (!bytes_eq(a + 3, base + r.coll_off, r.coll_len)) return false;
    a += 3 + r.coll_len;
  }
  return bytes_eq(a, base + r.key_off, r.key_len);
}
// two records of the block name the same key of the same update map: public and hashed updates
// are separate maps in the reference (privacyenabledstate UpdateBatch), so the kind must agree
__device__ __forceinline__ bool rec_eq(const uint8_t *base, const MvRec &a, const MvRec &b) {
  if (a.tag != b.tag || ((a.flags ^ b.flags) & MVR_HASHED) || a.ns_len != b.ns_len || a.key_len != b.key_len)
    return false;
  if ((a.flags & MVR_HASHED) &&
      (a.coll_len != b.coll_len || !bytes_eq(base + a.coll_off, base + b.coll_off, a.coll_len)))
    return false;
  return bytes_eq(base + a.ns_off, base + b.ns_off, a.ns_len) && bytes_eq(base + a.key_off, base + b.key_off, a.key_len);
}

// committed-state probe: slot index or -1
__device__ __forceinline__ int64_t state_find(const StateSlot *tbl, uint64_t mask, const uint8_t *arena,
                                              const uint8_t *base, const MvRec &r) {
  uint64_t idx = r.tag & mask;
  for (uint64_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    const uint64_t t = tbl[idx].tag;
    if (t == 0) return -1;
    if ((t | MV_TAG_PRESENT) == (r.tag | MV_TAG_PRESENT) && rec_eq_state(base, r, tbl[idx], arena)) return (int64_t)idx;
  }
  return -1;
}

// ------------------------------------------------------------------ device rwset walk
namespace {

// record sink: pass 1 counts, pass 2 writes records at the tx's claimed ranges
struct Sink {
  const uint8_t *base;
  MvRec *rout, *wout;  // null: count only
  uint32_t tx, nr, nw;
  uint64_t wbytes;     // arena bytes the writes could need (capacity check of the commit)
  bool big;            // a length exceeds the record fields
  uint32_t kmax = 0xFFFFFFFFu;  // records per kind the outputs hold (the per-tx scratch)
  bool spill = false;           // more than kmax of a kind: the scratch copy is incomplete
  __device__ void rec(MvRec *out, uint32_t k, S ns, bool hashed, S coll, S key, uint32_t flags, uint64_t b,
                      uint64_t t) {
    if (ns.n > 0xFFFF || key.n > 0xFFFF || coll.n > 0xFFFF || ns.n + 3u + coll.n > 0xFFFF) { big = true; return; }
    if (!out) return;
    if (k >= kmax) { spill = true; return; }
    MvRec r;
    r.ns_off = (uint32_t)(ns.p - base);
    r.key_off = (uint32_t)(key.p - base);
    r.coll_off = hashed ? (uint32_t)(coll.p - base) : 0u;
    r.ns_len = (uint16_t)ns.n;
    r.key_len = (uint16_t)key.n;
    r.coll_len = hashed ? (uint16_t)coll.n : 0;
    r.flags = (uint16_t)(flags | (hashed ? MVR_HASHED : 0));
    r.tx = tx;
    r.blk = b;
    r.txn = t;
    r.tag = rec_tag(base, r);
    out[k] = r;
  }
  __device__ void read(S ns, bool hashed, S coll, S key, bool has_ver, uint64_t b, uint64_t t) {
    rec(rout, nr++, ns, hashed, coll, key, has_ver ? MVR_HASVER : 0u, b, t);
  }
  // (a write's blk / txn: its value span -- offset from base, length -- for k_ub_block)
  __device__ void write(S ns, bool hashed, S coll, S key, bool del, S val) {
    rec(wout, nw++, ns, hashed, coll, key, del ? MVR_DELETE : 0u, del ? 0ull : (uint64_t)(val.p - base),
        del ? 0ull : val.n);
    wbytes += ((uint64_t)ns.n + (hashed ? 3u + coll.n : 0u) + key.n + 7u) & ~7ull;
  }
};

struct VVer {  // Version {block_num = 1, tx_num = 2}; occurrences merge
  uint64_t b = 0, t = 0;
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : K_NONE; }
  DEV void on_varint(uint32_t n, uint64_t v) { (n == 1 ? b : t) = v; }
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VRead {  // KVRead {key string = 1, version = 2} / KVReadHash {key_hash bytes = 1, version = 2}
  bool hashed;
  S key{nullptr, 0};
  bool has_ver = false;
  VVer v;
  DEV Kind kind(uint32_t n) { return n == 1 ? (hashed ? K_BYTES : K_STRING) : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { key = s; return true; }
    has_ver = true;
    return decode(s, v, ovf);
  }
};
struct VWrite {  // KVWrite {key string 1, is_delete 2, value 3} / KVWriteHash {key_hash 1, is_delete 2, value_hash 3, is_purge 4}
  bool hashed;
  S key{nullptr, 0}, val{nullptr, 0};
  bool del = false;
  DEV Kind kind(uint32_t n) {
    if (n == 1) return hashed ? K_BYTES : K_STRING;
    if (n == 2) return K_VARINT;
    if (n == 3) return K_BYTES;
    return (hashed && n == 4) ? K_VARINT : K_NONE;
  }
  DEV void on_varint(uint32_t n, uint64_t v) { if (n == 2) del = v != 0; }
  DEV bool on_len(uint32_t n, S s, bool &) { (n == 1 ? key : val) = s; return true; }
};
struct VMetaEnt {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VMetaW {  // KVMetadataWrite {key string 1, entries 2} / KVMetadataWriteHash {key_hash bytes 1, entries 2}
  bool hashed;
  DEV Kind kind(uint32_t n) { return n == 1 ? (hashed ? K_BYTES : K_STRING) : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    VMetaEnt e;
    return decode(s, e, ovf);
  }
};
struct VQReads {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) { VRead r{false}; return decode(s, r, ovf); }
};
struct VMerk {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : n == 3 ? K_REP_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VRQ {  // RangeQueryInfo (validated; phantom checks are outside the model)
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_STRING : n == 3 ? K_VARINT : (n == 4 || n == 5) ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 4) { VQReads q; return decode(s, q, ovf); }
    if (n == 5) { VMerk m; return decode(s, m, ovf); }
    return true;
  }
};
// KVRWSet (hashed = false) or HashedRWSet (hashed = true): reads / writes go to the sink
struct VRW {
  Sink *sk;
  S ns, coll;
  bool hashed;
  bool unsup = false;
  bool host = false;  // range queries / metadata writes: validated here, decided by the host path
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= (hashed ? 3u : 4u)) ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) {
      VRead r{hashed};
      if (!decode(s, r, ovf)) return false;
      sk->read(ns, hashed, coll, r.key, r.has_ver, r.v.b, r.v.t);
      return true;
    }
    if (!hashed && n == 2) { host = true; VRQ q; return decode(s, q, ovf); }  // range query
    if (n == (hashed ? 2u : 3u)) {
      VWrite w{hashed};
      if (!decode(s, w, ovf)) return false;
      bool del = w.del || w.val.n == 0;
      if (hashed && !del && w.val.n == 32) {  // value hash == SHA-256("") (rwset_proto_util.go:370)
        const uint8_t e[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
                               0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
        del = bytes_eq(w.val.p, e, 32);
      }
      sk->write(ns, hashed, coll, w.key, del, w.val);
      return true;
    }
    host = true;  // metadata write (conditional on the key existing: the host path)
    VMetaW m{hashed};
    return decode(s, m, ovf);
  }
};
struct VColl {  // CollectionHashedReadWriteSet {collection_name 1, hashed_rwset 2, pvt_rwset_hash 3}
  S name{nullptr, 0}, hashed{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : (n == 2 || n == 3) ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) {
    if (n == 1) name = s;
    else if (n == 2) hashed = s;
    return true;
  }
};
// NsReadWriteSet pass 1: namespace (last occurrence wins), rwset span; collections validated
struct VNsHdr {
  S ns{nullptr, 0}, rwset{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_STRING : n == 2 ? K_BYTES : n == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) ns = s;
    else if (n == 2) rwset = s;
    else { VColl c; return decode(s, c, ovf); }
    return true;
  }
};
// NsReadWriteSet pass 2: each collection's hashed rwset, in order
struct VNsColls {
  Sink *sk;
  S ns;
  bool fail = false, unsup = false, host = false;
  DEV Kind kind(uint32_t n) { return n == 3 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    VColl c;
    if (!decode(s, c, ovf)) return false;
    VRW h{sk, ns, c.name, true};
    if (!decode(c.hashed, h, ovf)) { fail = true; return true; }
    unsup |= h.unsup;
    host |= h.host;
    return true;
  }
};
// TxReadWriteSet {data_model 1, ns_rwset 2}; decode failures anywhere -> 255 (rwsetutil
// TxRwSet.FromProtoBytes unmarshals every namespace and collection before any check)
struct VTxRW {
  Sink *sk;
  bool fail = false, unsup = false, host = false;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_VARINT : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    VNsHdr h;
    if (!decode(s, h, ovf)) return false;
    VRW kv{sk, h.ns, S{nullptr, 0}, false};
    if (!decode(h.rwset, kv, ovf)) fail = true;
    unsup |= kv.unsup;
    host |= kv.host;
    VNsColls cs{sk, h.ns};
    if (!decode(s, cs, ovf)) return false;
    fail |= cs.fail;
    unsup |= cs.unsup;
    host |= cs.host;
    return true;
  }
};
struct VEndLite {  // ChaincodeEndorsedAction: prp span; endorsements validated only
  S prp{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { prp = s; return true; }
    VTwoBytes e;
    return decode(s, e, ovf);
  }
};
struct VCapLite {
  bool has_action = false;
  VEndLite action;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) return true;
    has_action = true;
    return decode(s, action, ovf);
  }
};

// GetActionFromEnvelope (protoutil/txutils.go) up to ChaincodeAction.results; code or 0
// (a decode that failed on a device capacity -- START_GROUP nesting -- is not a verdict: `ovf`
// turns it into "unsupported")
DEV uint8_t find_results(S d, S &results) {
  bool ovf = false;
  VTwoBytes env;
  VPayload pl;
  VChannelHeader chdr;
  // an unparsable committer-valid envelope / nil header: the reference errors out (halt) --
  // not ours to decide; non-endorser txs go through custom processors
  if (!decode(d, env, ovf) || !decode(env.a, pl, ovf) || !pl.has_header || !decode(pl.hdr.a, chdr, ovf))
    return MV_UNSUP;
  if (chdr.type != 3) return MV_UNSUP;
  VTransaction tx;
  if (!decode(pl.data, tx, ovf) || tx.nact == 0) return ovf ? MV_UNSUP : MV_NIL;
  VCapLite cap;
  if (!decode(tx.first.b, cap, ovf) || !cap.has_action || cap.action.prp.n == 0) return ovf ? MV_UNSUP : MV_NIL;
  VTwoBytes prp;
  if (!decode(cap.action.prp, prp, ovf) || prp.b.n == 0) return ovf ? MV_UNSUP : MV_NIL;
  VCcAction cca;
  if (!decode(prp.b, cca, ovf)) return ovf ? MV_UNSUP : MV_NIL;
  results = cca.results;
  return 0;
}

DEV uint8_t walk_rwset(S results, Sink &sk, bool &host) {
  bool ovf = false;
  VTxRW rw{&sk};
  const bool ok = decode(results, rw, ovf);
  if (ovf) return MV_UNSUP;
  if (!ok || rw.fail) return MV_OTHER;
  if (rw.unsup || sk.big) return MV_UNSUP;
  host = rw.host;
  return 0;
}

// wave-aggregated claim of `cnt` consecutive slots of a counter
DEV uint32_t wave_claim(uint32_t cnt, uint32_t *counter) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t v = cnt;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, d);
    if (lane >= d) v += o;
  }
  uint32_t b = 0;
  if (lane == 63u && v) b = atomicAdd(counter, v);
  b = (uint32_t)__shfl((int)b, 63);
  return b + v - cnt;
}

// the same for a 64-bit counter (every lane of the wave calls it)
DEV uint64_t wave_claim64(uint32_t cnt, unsigned long long *counter) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t v = cnt;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  uint64_t b = 0;
  if (lane == 63u && v) b = atomicAdd(counter, (unsigned long long)v);
  b = __shfl(b, 63);
  return b + v - cnt;
}

DEV uint32_t bmask_of(uint32_t nw) {
  uint32_t cap = 1024;
  while (cap < 2u * nw) cap <<= 1;
  return cap - 1;
}

}  // namespace

// ============================================================ rwset extraction
// One workgroup (one wave) per TPW transactions.  The wave first copies the group's
// envelopes into LDS -- coalesced dword loads, every envelope's lines in flight at once -- then
// lane j walks transaction j's TxReadWriteSet from LDS (pbwire_dev.h rules) through a "virtual
// base" (the LDS copy minus the envelope's block offset), so record offsets stay block-relative
// while every dependent load of the walk is an LDS access instead of a cache / HBM round trip.
// An envelope larger than CAP is walked from global memory (its lines requested up front).
// The counting walk writes the records to the per-tx scratch too, so a tx within it is copied
// instead of walked a second time; record ranges are claimed by wave-aggregated atomics.
// Duplicate writes of one key in one tx (tx_ops.go:183-191 adds flags: undefined semantics)
// -> unsupported.
// touch (global walks only): FGV_MVX_TOUCH=0 turns the up-front line requests off (A/B)
// scr (nullable): per-tx scratch of MVX_SCR reads + MVX_SCR writes
// n 16-byte words, 8 loads issued before their stores (one round trip per pass)
__device__ __forceinline__ void copy16(uint4 *__restrict__ d, const uint4 *__restrict__ s, uint32_t n) {
  for (uint32_t q = 0; q < n; q += 8) {
    uint4 v[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++)
      if (q + u < n) v[u] = s[q + u];
#pragma unroll
    for (uint32_t u = 0; u < 8; u++)
      if (q + u < n) d[q + u] = v[u];
  }
}

// XM (FGV_MVX_LDSSCR, with a scratch requested): 1 = LS, the counting walk's records go to an LDS
// scratch (MVX_SCR of each kind per transaction) and the wave copies them to the claimed ranges
// with coalesced 16-byte stores -- each record is written to global memory once; 0 = the per-tx
// scratch in global memory (`scr`) with the full staging cap (A/B)
template <uint32_t TPW, uint32_t XM>
__device__ __forceinline__ void mvx_extract(uint32_t ntx, const uint8_t *__restrict__ base,
                                            const uint32_t *__restrict__ envtab, const uint8_t *__restrict__ in_flags,
                                            MvTxInfo *__restrict__ info, MvRec *__restrict__ reads,
                                            MvRec *__restrict__ writes, MvCounters *__restrict__ c, uint32_t touch,
                                            MvRec *__restrict__ scr, uint8_t *__restrict__ bad, uint32_t wg) {
  // LDS bytes per transaction (larger envelopes walk global memory): 48 KB per workgroup at 64;
  // halved with the LDS record scratch (24 KB at 32 per workgroup), so that a workgroup still
  // takes 48 KB at 32 (three per CU)
  constexpr bool LS = XM == 1;
  constexpr uint32_t CAP = (TPW == 64 ? 768u : 1536u) / (LS ? 2u : 1u);
  __shared__ uint32_t lds[TPW * (CAP / 4)];
  __shared__ uint32_t pre[TPW + 1], src0[TPW];  // dword prefix of the staged envelopes, source dword
  __shared__ uint4 lscr[LS ? TPW * 2 * MVX_SCR * 3 : 1];  // (LS) per-tx records: MVX_SCR reads, MVX_SCR writes
  __shared__ uint32_t ldst[LS ? 4 * TPW : 1];             // (LS) rbeg, rcnt, wbeg, wcnt of copied txs
  const uint32_t lane = threadIdx.x, t0 = wg * TPW;
  // stage: the dwords covering [off, off + len + 8) of each committer-valid envelope (the walk's
  // over-read contract: up to 7 bytes past a span; block buffers carry >= 64 B of tail padding).
  // Lane j reads transaction j's table entry; then every lane copies dwords of the concatenated
  // envelopes (independent loads, all in flight).
  uint32_t my_nw = 0;
  if (lane < TPW && t0 + lane < ntx && in_flags[t0 + lane] == 0) {
    const uint32_t off = envtab[2 * (t0 + lane)], len = envtab[2 * (t0 + lane) + 1];
    const uint32_t a0 = off & ~3u, nwd = ((off + len + 8u + 3u) & ~3u) / 4u - a0 / 4u;
    if (nwd <= CAP / 4) {
      my_nw = nwd;
      src0[lane] = a0 / 4u;
    }
  }
  // inclusive prefix over the TPW lanes (wave scan)
  uint32_t v = my_nw;
  for (uint32_t d = 1; d < TPW; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, d);
    if (lane >= d) v += o;
  }
  if (lane < TPW) pre[lane + 1] = v;
  if (lane == 0) pre[0] = 0;
  __syncthreads();
  const uint32_t total = pre[TPW];
  const uint32_t *src = reinterpret_cast<const uint32_t *>(base);
  // 8 dwords per lane per pass: all 8 loads are issued before the first LDS store, so a pass
  // costs one memory round trip (a plain loop waited for each load before its store)
  constexpr uint32_t U = 8;
  for (uint32_t i0 = lane; i0 < total; i0 += 64 * U) {
    uint32_t v[U], dst[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t i = i0 + 64 * u;
      dst[u] = 0xFFFFFFFFu;
      if (i < total) {
        uint32_t j = 0;  // the envelope of dword i: pre[j] <= i < pre[j + 1]
#pragma unroll
        for (uint32_t b = TPW / 2; b > 0; b >>= 1)
          if (pre[j + b] <= i) j += b;
        const uint32_t k = i - pre[j];
        v[u] = src[src0[j] + k];
        dst[u] = j * (CAP / 4) + k;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (dst[u] != 0xFFFFFFFFu) lds[dst[u]] = v[u];
  }
  __syncthreads();
  const uint32_t t = lane < TPW ? t0 + lane : ntx;
  uint32_t nr = 0, nw = 0;
  uint64_t wb = 0;
  MvTxInfo I{};
  bool copied = false;
  const uint8_t *vb = base;  // the walk's base: block offsets -> bytes (LDS copy or global)
  if (t < ntx) {
    bad[t] = 0;  // (k_mvx_prep marks static conflicts after this kernel: no separate memset)
    I.code = MV_SKIP;
    if (in_flags[t] == 0) {
      const uint32_t off = envtab[2 * t], len = envtab[2 * t + 1];
      const uint32_t a0 = off & ~3u, nwd = ((off + len + 8u + 3u) & ~3u) / 4u - a0 / 4u;
      if (nwd <= CAP / 4)
        vb = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(lds + lane * (CAP / 4)) - a0);
      else if (touch)
        touch_lines(base + off, len);
      S results{nullptr, 0};
      I.code = find_results(S{vb + off, len}, results);
      if (I.code == 0) {
        MvRec *sr = LS ? reinterpret_cast<MvRec *>(lscr + lane * (2 * MVX_SCR * 3))
                       : scr ? scr + (size_t)t * (2 * MVX_SCR) : nullptr;
        Sink sk{vb, sr, sr ? sr + MVX_SCR : nullptr, t, 0, 0, 0, false};
        sk.kmax = MVX_SCR;
        bool host = false;
        I.code = walk_rwset(results, sk, host);
        I.rws_off = (uint32_t)(results.p - vb);
        I.rws_len = results.n;
        if (I.code == 0) { nr = sk.nr; nw = sk.nw; wb = sk.wbytes; }
        copied = sr && !sk.spill;
        // range queries / metadata writes: the block goes to the host path (fgv_mvcc.cpp),
        // which takes these codes and rwset spans (MV_HOSTPATH stops the device pipeline)
        if (I.code == 0 && host) atomicOr(&c->unsup, MV_HOSTPATH);
      }
      if (I.code == MV_UNSUP) atomicOr(&c->unsup, 1u);
    }
  }
  I.rbeg = wave_claim(nr, &c->nr);
  I.wbeg = wave_claim(nw, &c->nw);
  I.rcnt = nr;
  I.wcnt = nw;
  for (int o = 32; o > 0; o >>= 1) wb += __shfl_down(wb, o);
  if (lane == 0 && wb) atomicAdd(&c->wbytes, (unsigned long long)wb);
  if (LS) {
    // the copied transactions' records, LDS -> their claimed ranges: 16-byte word q of
    // transaction j's scratch on lane (j * 3 * MVX_SCR + q) % 64, consecutive lanes on
    // consecutive words of one range
    const bool cp = t < ntx && I.code == 0 && copied;
    if (lane < TPW) {
      ldst[4 * lane] = I.rbeg;
      ldst[4 * lane + 1] = cp ? I.rcnt * 3 : 0u;
      ldst[4 * lane + 2] = I.wbeg;
      ldst[4 * lane + 3] = cp ? I.wcnt * 3 : 0u;
    }
    __syncthreads();
    constexpr uint32_t Q = 3 * MVX_SCR;
    for (uint32_t u = lane; u < 2 * TPW * Q; u += 64) {
      const uint32_t kind = u / (TPW * Q), v = u - kind * (TPW * Q), j = v / Q, q = v - j * Q;
      if (q < ldst[4 * j + 2 * kind + 1]) {
        uint4 *dst = reinterpret_cast<uint4 *>((kind ? writes : reads) + ldst[4 * j + 2 * kind]);
        dst[q] = lscr[j * (2 * Q) + kind * Q + q];
      }
    }
  }
  if (t >= ntx) return;
  if (I.code == 0) {
    if (LS && copied) {
      // (copied by the wave above)
    } else if (copied) {  // (16-byte copies, 8 loads in flight per pass, instead of a second walk)
      const MvRec *sr = scr + (size_t)t * (2 * MVX_SCR);
      copy16(reinterpret_cast<uint4 *>(reads + I.rbeg), reinterpret_cast<const uint4 *>(sr), I.rcnt * 3);
      copy16(reinterpret_cast<uint4 *>(writes + I.wbeg), reinterpret_cast<const uint4 *>(sr + MVX_SCR), I.wcnt * 3);
    } else {
      Sink sk{vb, reads + I.rbeg, writes + I.wbeg, t, 0, 0, 0, false};
      bool host = false;
      walk_rwset(S{vb + I.rws_off, I.rws_len}, sk, host);
    }
    const MvRec *w = !copied ? writes + I.wbeg
                     : LS    ? reinterpret_cast<const MvRec *>(lscr + lane * (2 * MVX_SCR * 3)) + MVX_SCR
                             : scr + (size_t)t * (2 * MVX_SCR) + MVX_SCR;
    bool dup = false;
    for (uint32_t a = 0; a < I.wcnt && !dup; a++)
      for (uint32_t b = a + 1; b < I.wcnt; b++)
        if (rec_eq(vb, w[a], w[b])) { dup = true; break; }
    if (dup) {
      I.code = MV_UNSUP;
      atomicOr(&c->unsup, 1u);
    }
  }
  info[t] = I;
}
template <uint32_t TPW, uint32_t XM>
__global__ __launch_bounds__(64) void k_mvx_extract_t(uint32_t ntx, const uint8_t *__restrict__ base,
                                                      const uint32_t *__restrict__ envtab,
                                                      const uint8_t *__restrict__ in_flags, MvTxInfo *__restrict__ info,
                                                      MvRec *__restrict__ reads, MvRec *__restrict__ writes,
                                                      MvCounters *__restrict__ c, uint32_t touch, MvRec *__restrict__ scr,
                                                      uint8_t *__restrict__ bad) {
  mvx_extract<TPW, XM>(ntx, base, envtab, in_flags, info, reads, writes, c, touch, scr, bad, blockIdx.x);
}
// several blocks in one launch (mvcc_multi.h): workgroup -> its block by the jobs' wg0
template <uint32_t TPW, uint32_t XM>
__global__ __launch_bounds__(64) void k_mvx_extract_multi(const MvxJobs J) {
  uint32_t q = 0;
  while (q + 1 < J.n && blockIdx.x >= J.j[q + 1].wg0) q++;
  const MvxJob &b = J.j[q];
  mvx_extract<TPW, XM>(b.ntx, b.base, b.envtab, b.in_flags, b.info, b.reads, b.writes, b.c, J.touch, b.scr, b.bad,
                   blockIdx.x - b.wg0);
}
// transactions per workgroup (16 / 32 / 64): host picks (fgv_mvcc.cpp mvx_launch).
// FGV_MVX_LDSSCR (with a scratch requested, FGV_MVX_ONEWALK): 1 (default) the records' scratch
// in LDS, each record written to global memory once (mvx_extract); 0 the per-tx scratch in global
// memory with the full staging cap, at 32 per workgroup whatever FGV_MVX_TPW says (A/B; each
// instantiation of the walk costs minutes of compile).  Measured on MI355X (C3 chained, 10 blocks
// per call, alternating on one box, r6zk): 0 -> 93.2 / 93.4 M tx/s, 1 -> 97.0 / 96.1, and a
// temporary mode with the global scratch and the halved cap 97.6 / 97.4 -- the gain is the
// workgroups' smaller LDS footprint (C3 envelopes are ~430 B), and 1 also drops the scratch's
// global write and read back
static uint32_t mvx_ldsscr() {
  static const uint32_t on = [] {
    const char *e = getenv("FGV_MVX_LDSSCR");
    return e && atoi(e) == 0 ? 0u : 1u;
  }();
  return on;
}
bool mvx_lds_scratch() { return mvx_ldsscr() == 1u; }
template <uint32_t TPW, uint32_t XM>
static void mvx_multi_go(hipStream_t st, const MvxJobs &J, uint32_t wgs) {
  hipLaunchKernelGGL((k_mvx_extract_multi<TPW, XM>), dim3(wgs), dim3(64), 0, st, J);
}
void mvx_extract_multi_launch(uint32_t tpw, hipStream_t st, const MvxJobs &J, uint32_t wgs) {
  const uint32_t ls = J.n && J.j[0].scr ? mvx_ldsscr() : 0u;
  if (ls != 1) mvx_multi_go<32, 0>(st, J, wgs);  // (the A/B mode: 32 per workgroup)
  else if (tpw == 64) mvx_multi_go<64, 1>(st, J, wgs);
  else if (tpw == 32) mvx_multi_go<32, 1>(st, J, wgs);
  else mvx_multi_go<16, 1>(st, J, wgs);
}
template <uint32_t TPW, uint32_t XM>
static void mvx_extract_go(hipStream_t st, uint32_t ntx, const uint8_t *base, const uint32_t *envtab,
                           const uint8_t *in_flags, MvTxInfo *info, MvRec *reads, MvRec *writes, MvCounters *c,
                           uint32_t touch, MvRec *scr, uint8_t *bad) {
  hipLaunchKernelGGL((k_mvx_extract_t<TPW, XM>), dim3((ntx + TPW - 1) / TPW), dim3(64), 0, st, ntx, base, envtab,
                     in_flags, info, reads, writes, c, touch, scr, bad);
}
void mvx_extract_launch(uint32_t tpw, hipStream_t st, uint32_t ntx, const uint8_t *base, const uint32_t *envtab,
                        const uint8_t *in_flags, MvTxInfo *info, MvRec *reads, MvRec *writes, MvCounters *c,
                        uint32_t touch, MvRec *scr, uint8_t *bad) {
  const uint32_t ls = scr ? mvx_ldsscr() : 0u;
  if (ls != 1) mvx_extract_go<32, 0>(st, ntx, base, envtab, in_flags, info, reads, writes, c, touch, scr, bad);
  else if (tpw == 64) mvx_extract_go<64, 1>(st, ntx, base, envtab, in_flags, info, reads, writes, c, touch, scr, bad);
  else if (tpw == 32) mvx_extract_go<32, 1>(st, ntx, base, envtab, in_flags, info, reads, writes, c, touch, scr, bad);
  else mvx_extract_go<16, 1>(st, ntx, base, envtab, in_flags, info, reads, writes, c, touch, scr, bad);
}

// ============================================================ lookups
// writes: claim a block write-table slot (epoch-tagged owner; a slot of an older block is free)
// reads: committed-state probe, static version check (version.AreSame; nil <=> absent)
__global__ __launch_bounds__(256) void k_mvx_prep(const uint8_t *__restrict__ base, const MvRec *__restrict__ reads,
                                                  const MvRec *__restrict__ writes, BlkSlot *__restrict__ btbl,
                                                  uint32_t epoch, uint32_t *__restrict__ wslot,
                                                  const StateSlot *__restrict__ tbl, uint64_t mask,
                                                  const uint8_t *__restrict__ arena, uint8_t *__restrict__ bad,
                                                  MvCounters *__restrict__ c, const MvCounters *__restrict__ prev) {
  // a chain of blocks (fgv_mvcc_validate_blocks): block k runs only when block k-1 was decided
  // and committed on the device; else nothing of it runs (MV_HALT) and the host takes over from
  // the first such block, in block order
  if (prev && (prev->unsup || !prev->done || prev->nomem)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&c->unsup, MV_HALT);
    return;
  }
  const uint32_t nr = c->nr, nw = c->nw, bm = bmask_of(nw);
  if (c->unsup) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr + nw; i += gridDim.x * blockDim.x) {
    if (i < nw) {
      const MvRec w = writes[i];
      const uint64_t mine = ((uint64_t)epoch << 32) | (i + 1);
      uint32_t idx = (uint32_t)w.tag & bm, out = FW_INF;
      for (uint32_t probe = 0; probe <= bm && out == FW_INF; probe++, idx = (idx + 1) & bm) {
        unsigned long long *o = reinterpret_cast<unsigned long long *>(&btbl[idx].owner);
        unsigned long long cur = *reinterpret_cast<volatile unsigned long long *>(o);
        // a slot owned by an older block is free: claim it (at most two tries -- a failed CAS
        // means another write of this block claimed the slot)
        while ((uint32_t)(cur >> 32) != epoch) {
          const unsigned long long prev = atomicCAS(o, cur, (unsigned long long)mine);
          if (prev == cur) { cur = mine; break; }
          cur = prev;
        }
        if (cur == mine || rec_eq(base, writes[(uint32_t)cur - 1], w)) out = idx;
      }
      wslot[i] = out;
    } else {
      const MvRec r = reads[i - nw];
      const int64_t s = state_find(tbl, mask, arena, base, r);
      const bool committed = s >= 0 && (tbl[s].tag & MV_TAG_PRESENT);
      const bool has_ver = (r.flags & MVR_HASVER) != 0;
      bool same;
      if (!committed || !has_ver) same = committed == has_ver;
      else same = tbl[s].blk == r.blk && tbl[s].txn == r.txn;
      if (!same) bad[r.tx] = 1;
    }
  }
}

__device__ __forceinline__ uint64_t fw_enc(uint32_t rg, uint32_t tx) { return ((uint64_t)rg << 32) | (0xFFFFFFFFu - tx); }
__device__ __forceinline__ uint32_t fw_dec(uint64_t v, uint32_t rg) {
  return (uint32_t)(v >> 32) == rg ? 0xFFFFFFFFu - (uint32_t)v : FW_INF;
}
__device__ __forceinline__ void publish(BlkSlot *btbl, const uint32_t *wslot, const MvTxInfo &I, uint32_t t,
                                        uint8_t s, uint32_t rg) {
  if (s == ST_INVALID) return;
  const unsigned long long e = fw_enc(rg, t);
  for (uint32_t w = I.wbeg; w < I.wbeg + I.wcnt; w++) {
    BlkSlot &B = btbl[wslot[w]];
    atomicMax(reinterpret_cast<unsigned long long *>(&B.fw_cand[rg & 1]), e);
    if (s == ST_VALID) atomicMax(reinterpret_cast<unsigned long long *>(&B.fw_valid[rg & 1]), e);
  }
}

// reads -> block write-table slot; tx -> initial state + round-1 first writers (global round rg1)
__global__ __launch_bounds__(256) void k_mvx_find(uint32_t ntx, const uint8_t *__restrict__ base,
                                                  const MvRec *__restrict__ reads, const MvRec *__restrict__ writes,
                                                  const BlkSlot *__restrict__ btbl_r, BlkSlot *__restrict__ btbl,
                                                  uint32_t epoch, const uint32_t *__restrict__ wslot,
                                                  uint32_t *__restrict__ rslot, const MvTxInfo *__restrict__ info,
                                                  const uint8_t *__restrict__ bad, uint8_t *__restrict__ st,
                                                  uint32_t rg1, const MvCounters *__restrict__ c) {
  const uint32_t nr = c->nr, bm = bmask_of(c->nw);
  if (c->unsup) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr + ntx; i += gridDim.x * blockDim.x) {
    if (i < nr) {
      const MvRec r = reads[i];
      uint32_t idx = (uint32_t)r.tag & bm, out = FW_INF;
      for (uint32_t probe = 0; probe <= bm; probe++, idx = (idx + 1) & bm) {
        const uint64_t own = btbl_r[idx].owner;
        if ((uint32_t)(own >> 32) != epoch) break;
        const MvRec &o = writes[(uint32_t)own - 1];
        if (o.tag == r.tag && rec_eq(base, o, r)) { out = idx; break; }
      }
      rslot[i] = out;
    } else {
      const uint32_t t = i - nr;
      const MvTxInfo I = info[t];
      const uint8_t s = (I.code == 0 && !bad[t]) ? ST_UNDEC : ST_INVALID;
      st[t] = s;
      if (I.code == 0) publish(btbl, wslot, I, t, s, rg1);
    }
  }
}

// fixpoint round r (1-based within the block; global round tag rg = rg0 + r)
__global__ __launch_bounds__(64) void k_mvx_round(uint32_t ntx, uint32_t r, uint32_t rg, const MvTxInfo *__restrict__ info,
                                                  const uint32_t *__restrict__ rslot, const uint32_t *__restrict__ wslot,
                                                  BlkSlot *__restrict__ btbl, uint8_t *__restrict__ st,
                                                  MvCounters *__restrict__ c) {
  if (c->done || c->unsup) return;
  if (r > 1 && c->undec[(r - 1) & 3] == 0) {  // round r-1 decided everything
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      c->done = 1;
      c->rounds = r - 1;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) c->undec[(r + 1) & 3] = 0;  // the slot round r+1 counts into
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t und = 0;
  if (t < ntx) {
    uint8_t s = st[t];
    const MvTxInfo I = info[t];
    if (s == ST_UNDEC) {
      bool conflict = false, clear = true;
      for (uint32_t j = I.rbeg; j < I.rbeg + I.rcnt; j++) {
        const uint32_t k = rslot[j];
        if (k == FW_INF) continue;  // key never written in this block
        if (fw_dec(btbl[k].fw_valid[rg & 1], rg) < t) { conflict = true; break; }
        if (fw_dec(btbl[k].fw_cand[rg & 1], rg) < t) clear = false;
      }
      s = conflict ? ST_INVALID : clear ? ST_VALID : ST_UNDEC;
      st[t] = s;
      und = s == ST_UNDEC;
    }
    if (I.code == 0) publish(btbl, wslot, I, t, s, rg + 1);
  }
  for (int off = 32; off > 0; off >>= 1) und += __shfl_down(und, off);
  if ((threadIdx.x & 63u) == 0 && und) atomicAdd(&c->undec[r & 3], und);
}

// the fixpoint has converged after round `rlast` (or earlier)
__device__ __forceinline__ bool converged(const MvCounters *c, uint32_t rlast) {
  return !c->unsup && (c->done || c->undec[rlast & 3] == 0);
}

// TRANSACTIONS_FILTER after MVCC: committer-invalid txs keep their code
__global__ __launch_bounds__(256) void k_mvx_flags(uint32_t ntx, uint32_t rlast, const uint8_t *__restrict__ in_flags,
                                                   const MvTxInfo *__restrict__ info, const uint8_t *__restrict__ st,
                                                   uint8_t *__restrict__ out, MvCounters *__restrict__ c) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (!converged(c, rlast)) return;
  if (t == 0 && !c->done) {
    c->done = 1;
    c->rounds = rlast;
  }
  if (t >= ntx) return;
  const uint8_t code = info[t].code;
  uint8_t f;
  if (code == MV_SKIP) f = in_flags[t];
  else if (code != 0) f = code;
  else f = st[t] == ST_INVALID ? 11 : 0;
  out[t] = f;
}

// the fused flags + last step of a chain block (mvcc_multi.h): k_mvx_flags over ntx, then (commit)
// k_mv_last's capacity check and last-valid-writer election over the block's writes
__global__ __launch_bounds__(256) void k_mvx_flags_last(uint32_t ntx, uint32_t rlast, const uint8_t *__restrict__ in_flags,
                                                        const MvTxInfo *__restrict__ info, const uint8_t *__restrict__ st,
                                                        uint8_t *__restrict__ out, MvCounters *__restrict__ c,
                                                        uint32_t commit, const MvRec *__restrict__ writes,
                                                        const uint32_t *__restrict__ wslot, BlkSlot *__restrict__ btbl,
                                                        uint32_t epoch, const unsigned long long *__restrict__ top,
                                                        uint64_t slots_cap, uint64_t arena_cap) {
  if (!converged(c, rlast)) return;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  if (gid == 0 && !c->done) {
    c->done = 1;
    c->rounds = rlast;
  }
  for (uint32_t t = gid; t < ntx; t += stride) {
    const uint8_t code = info[t].code;
    uint8_t f;
    if (code == MV_SKIP) f = in_flags[t];
    else if (code != 0) f = code;
    else f = st[t] == ST_INVALID ? 11 : 0;
    out[t] = f;
  }
  if (!commit) return;
  const uint32_t nw = c->nw;
  if ((top[1] + nw) * 10 > slots_cap * 7 || top[0] + c->wbytes > arena_cap) {
    if (gid == 0) c->nomem = 1;
    return;
  }
  for (uint32_t i = gid; i < nw; i += stride) {
    const uint32_t tx = writes[i].tx;
    if (st[tx] == ST_VALID)
      atomicMax(reinterpret_cast<unsigned long long *>(&btbl[wslot[i]].last), ((unsigned long long)epoch << 32) | (tx + 1));
  }
}

// ============================================================ commit
// last VALID writer of each key (a key is written at most once per tx: duplicates are
// unsupported), and the capacity check of the whole commit
__global__ __launch_bounds__(256) void k_mv_last(uint32_t rlast, const MvRec *__restrict__ writes,
                                                 const uint32_t *__restrict__ wslot, const uint8_t *__restrict__ st,
                                                 BlkSlot *__restrict__ btbl, uint32_t epoch, MvCounters *__restrict__ c,
                                                 const unsigned long long *__restrict__ top, uint64_t slots_cap,
                                                 uint64_t arena_cap) {
  if (!converged(c, rlast)) return;
  const uint32_t nw = c->nw;
  // load factor <= 0.7 and arena room for every write (upper bounds): else nothing is committed
  if ((top[1] + nw) * 10 > slots_cap * 7 || top[0] + c->wbytes > arena_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) c->nomem = 1;
    return;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
    const uint32_t tx = writes[i].tx;
    if (st[tx] == ST_VALID)
      atomicMax(reinterpret_cast<unsigned long long *>(&btbl[wslot[i]].last), ((unsigned long long)epoch << 32) | (tx + 1));
  }
}

// Upsert phase 1: keys already in the table are updated in place (version, present bit);
// absent, non-deleted keys are marked for phase 2.  mode 1 = block commit (only the last
// valid writer of each key; Height{block_num, tx}); mode 0 = host-supplied batch (every record,
// its own version: fgv_statedb_load / fgv_statedb_apply).
__global__ __launch_bounds__(256) void k_mv_upsert_find(uint32_t mode, uint32_t rlast, uint32_t n_host,
                                                        const uint8_t *__restrict__ base, const MvRec *__restrict__ recs,
                                                        const uint32_t *__restrict__ wslot, const uint8_t *__restrict__ st,
                                                        const BlkSlot *__restrict__ btbl, uint32_t epoch,
                                                        StateSlot *__restrict__ tbl, uint64_t mask,
                                                        const uint8_t *__restrict__ arena, uint64_t block_num,
                                                        uint8_t *__restrict__ pend, const MvCounters *__restrict__ c) {
  uint32_t n = n_host;
  if (mode == 1) {
    if (!converged(c, rlast) || c->nomem) return;
    n = c->nw;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const MvRec w = recs[i];
    uint64_t vb = w.blk, vt = w.txn;
    pend[i] = 0;
    if (mode == 1) {
      if (st[w.tx] != ST_VALID || btbl[wslot[i]].last != (((uint64_t)epoch << 32) | (w.tx + 1))) continue;
      vb = block_num;
      vt = w.tx;
    }
    const bool del = (w.flags & MVR_DELETE) != 0;
    const int64_t s = state_find(tbl, mask, arena, base, w);
    if (s >= 0) {
      tbl[s].blk = vb;
      tbl[s].txn = vt;
      tbl[s].tag = del ? (tbl[s].tag & ~MV_TAG_PRESENT) : (tbl[s].tag | MV_TAG_PRESENT);
    } else if (!del) {
      pend[i] = 1;
    }
  }
}

// Upsert phase 2: claim empty slots for keys known to be absent and distinct (no compares).
// top[0] = arena bytes used, top[1] = occupied slots.
__device__ __forceinline__ uint32_t blk_of(const uint32_t *__restrict__ bfirst, uint32_t nb, uint32_t g);
__global__ __launch_bounds__(256) void k_mv_upsert_insert(uint32_t mode, uint32_t rlast, uint32_t n_host,
                                                          const uint8_t *__restrict__ base, const MvRec *__restrict__ recs,
                                                          const uint8_t *__restrict__ pend, StateSlot *__restrict__ tbl,
                                                          uint64_t mask, uint8_t *__restrict__ arena,
                                                          unsigned long long *__restrict__ top, uint64_t block_num,
                                                          const MvCounters *__restrict__ c, const uint32_t *__restrict__ bfirst,
                                                          const uint64_t *__restrict__ bnums, uint32_t nb) {
  uint32_t n = n_host;
  if (mode >= 1) {  // (mode 2: the batch pass -- its versions are in the records)
    if (!converged(c, rlast) || c->nomem) return;
    n = c->nw;
  }
  // every lane of a wave runs the same iterations, so the arena bytes and the slot count are
  // claimed with one atomic per wave (a per-key atomicAdd on the two counters serialised the
  // kernel on their cache line)
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
    const uint32_t i = i0 + threadIdx.x;
    const bool mine = i < n && pend[i];
    MvRec w{};
    uint32_t fl = 0, need = 0;
    if (mine) {
      w = recs[i];
      fl = flat_ns_len(w);
      need = (fl + w.key_len + 7u) & ~7u;
    }
    const uint64_t off = wave_claim64(need, &top[0]);
    const uint64_t nmine = __popcll(__ballot(mine));
    if ((threadIdx.x & 63u) == 0 && nmine) atomicAdd(&top[1], (unsigned long long)nmine);
    if (!mine) continue;
    // the flattened ns [|| "$$h" || coll] || key, zero-padded to `need`, written a 32-bit word at a
    // time (byte stores cost a memory write each: ~0.7 KB of WRITE_SIZE per key, r4r)
    auto flat_byte = [&](uint32_t j) -> uint32_t {
      if (j < w.ns_len) return base[w.ns_off + j];
      j -= w.ns_len;
      if (w.flags & MVR_HASHED) {
        if (j < 3) return j < 2 ? (uint32_t)'$' : (uint32_t)'h';
        j -= 3;
        if (j < w.coll_len) return base[w.coll_off + j];
        j -= w.coll_len;
      }
      return j < w.key_len ? base[w.key_off + j] : 0u;
    };
    uint32_t *aw = reinterpret_cast<uint32_t *>(arena + off);  // (off: 8-byte aligned)
    for (uint32_t o = 0; o < need; o += 4)
      aw[o / 4] = flat_byte(o) | (flat_byte(o + 1) << 8) | (flat_byte(o + 2) << 16) | (flat_byte(o + 3) << 24);
    const unsigned long long tag = (unsigned long long)(w.tag | MV_TAG_PRESENT);
    uint64_t idx = w.tag & mask;
    for (uint64_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
      if (atomicCAS(reinterpret_cast<unsigned long long *>(&tbl[idx].tag), 0ull, tag) == 0ull) {
        tbl[idx].off8 = (uint32_t)(off >> 3);
        tbl[idx].ns_len = (uint16_t)fl;
        tbl[idx].key_len = w.key_len;
        if (mode == 2) {  // the batch pass: Height{the record's block, its index there}
          const uint32_t b = blk_of(bfirst, nb, w.tx);
          tbl[idx].blk = bnums[b];
          tbl[idx].txn = w.tx - bfirst[b];
        } else {
          tbl[idx].blk = mode == 1 ? block_num : w.blk;
          tbl[idx].txn = mode == 1 ? (uint64_t)w.tx : w.txn;
        }
        if (fl + w.key_len <= MV_INLINE) {  // the inline copy (the arena bytes written above; off
          // is 8-byte aligned), 8-byte words: bytes past the key are never compared
          const uint2 *src = reinterpret_cast<const uint2 *>(arena + off);
          uint2 *dst = reinterpret_cast<uint2 *>(tbl[idx].ik);
          for (uint32_t q = 0; 8 * q < fl + w.key_len; q++) dst[q] = src[q];
        }
        break;
      }
    }
  }
}

// The tail of a block of a chain written straight into pinned host memory (no copy kernels):
// its counters and, after a commit, the arena top (k_mvx_flags wrote the codes there already)
__global__ __launch_bounds__(64) void k_mv_tail(const MvCounters *__restrict__ c, const unsigned long long *__restrict__ top,
                                                uint32_t *__restrict__ hc, unsigned long long *__restrict__ htop) {
  const uint32_t t = threadIdx.x;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(c);
  if (t < sizeof(MvCounters) / 4) hc[t] = w[t];
  if (htop && t < 2) htop[t] = top[t];
  __threadfence_system();
}

// k_mv_tail for several chain blocks (mvcc_multi.h): workgroup q copies block q's counters
__global__ __launch_bounds__(64) void k_mv_tails(const MvTails T, const unsigned long long *__restrict__ top,
                                                 unsigned long long *__restrict__ htop) {
  const uint32_t t = threadIdx.x, q = blockIdx.x;
  if (q < T.n) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(T.c[q]);
    if (t < sizeof(MvCounters) / 4) T.hc[q][t] = w[t];
  }
  if (q == 0 && htop && t < 2) htop[t] = top[t];
  __threadfence_system();
}

// host-supplied key records (load / apply): tags
__global__ __launch_bounds__(256) void k_mv_tags(const uint8_t *__restrict__ base, MvRec *__restrict__ recs, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) recs[i].tag = rec_tag(base, recs[i]);
}

// ============================================================ host phantom path support
// Point lookups of host-given keys (flattened namespace at ns_off, key at key_off of `base`):
// found-and-present flag + committed version.
__global__ __launch_bounds__(256) void k_mv_lookup(uint32_t n, const uint8_t *__restrict__ base,
                                                   const MvRec *__restrict__ recs, const StateSlot *__restrict__ tbl,
                                                   uint64_t mask, const uint8_t *__restrict__ arena,
                                                   uint64_t *__restrict__ ver, uint8_t *__restrict__ present) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int64_t s = state_find(tbl, mask, arena, base, recs[i]);
    const bool p = s >= 0 && (tbl[s].tag & MV_TAG_PRESENT);
    present[i] = p ? 1 : 0;
    ver[2 * i] = p ? tbl[s].blk : 0;
    ver[2 * i + 1] = p ? tbl[s].txn : 0;
  }
}

// GetStateRangeScanIterator without an ordered index: every present committed key is tested
// against the block's ranges (namespace equal, start <= key, key < end unless unbounded) and
// matches are appended as {range, key_len, blk, txn} + key bytes (8-byte padded).  The host
// sorts each range's matches.  *used may exceed cap: the host then grows the buffer and reruns.
DEV bool key_lt(const uint8_t *a, uint32_t an, const uint8_t *b, uint32_t bn) {  // Go string order
  const uint32_t m = an < bn ? an : bn;
  for (uint32_t i = 0; i < m; i++)
    if (a[i] != b[i]) return a[i] < b[i];
  return an < bn;
}
__global__ __launch_bounds__(256) void k_mv_range_scan(uint64_t cap, const StateSlot *__restrict__ tbl,
                                                       const uint8_t *__restrict__ arena, uint32_t nranges,
                                                       const MvRange *__restrict__ ranges,
                                                       const uint8_t *__restrict__ rbytes, uint8_t *__restrict__ out,
                                                       uint64_t out_cap, unsigned long long *__restrict__ used) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
    const StateSlot sl = tbl[i];
    if (!(sl.tag & MV_TAG_OCC) || !(sl.tag & MV_TAG_PRESENT)) continue;
    const uint8_t *a = arena + ((uint64_t)sl.off8 << 3);
    const uint8_t *key = a + sl.ns_len;
    for (uint32_t r = 0; r < nranges; r++) {
      const MvRange R = ranges[r];
      if (R.ns_len != sl.ns_len || !bytes_eq(a, rbytes + R.ns_off, R.ns_len)) continue;
      if (key_lt(key, sl.key_len, rbytes + R.s_off, R.s_len)) continue;
      if (!(R.flags & MVRANGE_UNBOUNDED) && !key_lt(key, sl.key_len, rbytes + R.e_off, R.e_len)) continue;
      const uint64_t sz = 24 + (((uint64_t)sl.key_len + 7) & ~7ull);
      const uint64_t o = atomicAdd(used, (unsigned long long)sz);
      if (o + sz > out_cap) continue;  // counted: the host reruns with room
      uint32_t *h = reinterpret_cast<uint32_t *>(out + o);
      h[0] = r;
      h[1] = sl.key_len;
      uint64_t *v = reinterpret_cast<uint64_t *>(out + o + 8);
      v[0] = sl.blk;
      v[1] = sl.txn;
      for (uint32_t k = 0; k < sl.key_len; k++) out[o + 24 + k] = key[k];
    }
  }
}

// ============================================================ batch pass (consecutive blocks as one)
// fgv_mvcc_validate_blocks over B consecutive blocks whose bytes lie within 4 GB of one base
// (their records then share the block code's 32-bit offsets): ONE extraction, lookup and
// fixpoint over every transaction of the batch in block order (global index g), one commit of
// the batch's last valid writers -- a fixed ~10 launches per call instead of ~14 per block.
//
// The sequential reference rule, restated over the batch (validator.go:81-200, run block after
// block with each block's updates committed before the next -- kv_ledger.go:612-652): a read of
// key K with version V by transaction g is valid iff, with W = the LAST valid writer of K among
// the batch's transactions before g,
//   W in g's own block              -> conflict (updates.Exists);
//   W in an earlier block           -> V == Height{block of W, tx of W} (nil if W deleted K): the
//                                      committed state g's block reads was written by W;
//   no such W                       -> V == the committed version before the batch (nil if absent).
// Fixpoint: a read is decided once no UNDECIDED writer of K sits after the last VALID one before
// g; a transaction is INVALID as soon as one decided read conflicts, VALID once all its reads
// are decided and clear.  The lowest undecided transaction always decides, so rounds <= the
// longest chain of dependent outcomes; the host enqueues a few and falls back to the per-block
// chain when they do not suffice (nothing is committed then).
// The batch's writers of one key are listed in its write-table slot (MB_WR at most; more -> the
// per-block chain, MV_OVF).
__device__ __forceinline__ uint32_t blk_of(const uint32_t *__restrict__ bfirst, uint32_t nb, uint32_t g) {
  uint32_t lo = 0, hi = nb;  // bfirst[lo] <= g < bfirst[hi]
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (bfirst[m] <= g) lo = m;
    else hi = m;
  }
  return lo;
}

// writes: claim the key's batch slot (epoch-tagged owner; the claimer empties its writer list);
// reads: committed-state probe, static version check against the state before the batch
__global__ __launch_bounds__(256) void k_mvb_prep(const uint8_t *__restrict__ base, const MvRec *__restrict__ reads,
                                                  const MvRec *__restrict__ writes, MbSlot *__restrict__ btbl,
                                                  uint32_t epoch, uint32_t *__restrict__ wslot,
                                                  const StateSlot *__restrict__ tbl, uint64_t mask,
                                                  const uint8_t *__restrict__ arena, uint8_t *__restrict__ rstat,
                                                  MvCounters *__restrict__ c) {
  const uint32_t nr = c->nr, nw = c->nw, bm = bmask_of(nw);
  if (c->unsup) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr + nw; i += gridDim.x * blockDim.x) {
    if (i < nw) {
      const MvRec w = writes[i];
      const uint64_t mine = ((uint64_t)epoch << 32) | (i + 1);
      uint32_t idx = (uint32_t)w.tag & bm, out = FW_INF;
      for (uint32_t probe = 0; probe <= bm && out == FW_INF; probe++, idx = (idx + 1) & bm) {
        unsigned long long *o = reinterpret_cast<unsigned long long *>(&btbl[idx].owner);
        unsigned long long cur = *reinterpret_cast<volatile unsigned long long *>(o);
        while ((uint32_t)(cur >> 32) != epoch) {
          const unsigned long long prev = atomicCAS(o, cur, (unsigned long long)mine);
          if (prev == cur) {
            cur = mine;
            btbl[idx].nwr = 0u;  // (the list fills in k_mvb_find, after every claim)
            break;
          }
          cur = prev;
        }
        if (cur == mine || rec_eq(base, writes[(uint32_t)cur - 1], w)) out = idx;
      }
      wslot[i] = out;
    } else {
      const MvRec r = reads[i - nw];
      const int64_t s = state_find(tbl, mask, arena, base, r);
      const bool committed = s >= 0 && (tbl[s].tag & MV_TAG_PRESENT);
      const bool has_ver = (r.flags & MVR_HASVER) != 0;
      bool same;
      if (!committed || !has_ver) same = committed == has_ver;
      else same = tbl[s].blk == r.blk && tbl[s].txn == r.txn;
      rstat[i - nw] = same ? 0 : 1;
    }
  }
}

// writes -> their slot's writer list; reads -> the key's slot (FW_INF: no batch writer);
// transactions -> initial state
__global__ __launch_bounds__(256) void k_mvb_find(uint32_t ntx, const uint8_t *__restrict__ base,
                                                  const MvRec *__restrict__ reads, const MvRec *__restrict__ writes,
                                                  MbSlot *__restrict__ btbl, uint32_t epoch,
                                                  const uint32_t *__restrict__ wslot, uint32_t *__restrict__ rslot,
                                                  const MvTxInfo *__restrict__ info, uint8_t *__restrict__ st,
                                                  MvCounters *__restrict__ c) {
  const uint32_t nr = c->nr, nw = c->nw, bm = bmask_of(nw);
  if (c->unsup) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw + nr + ntx; i += gridDim.x * blockDim.x) {
    if (i < nw) {
      const uint32_t s = wslot[i];
      const uint32_t k = s == FW_INF ? MB_WR : atomicAdd(&btbl[s].nwr, 1u);
      if (k < MB_WR) btbl[s].wr[k] = i;
      else atomicOr(&c->unsup, MV_OVF);  // (a hot key: the per-block chain)
    } else if (i < nw + nr) {
      const MvRec r = reads[i - nw];
      uint32_t idx = (uint32_t)r.tag & bm, out = FW_INF;
      for (uint32_t probe = 0; probe <= bm; probe++, idx = (idx + 1) & bm) {
        const uint64_t own = btbl[idx].owner;
        if ((uint32_t)(own >> 32) != epoch) break;
        const MvRec &o = writes[(uint32_t)own - 1];
        if (o.tag == r.tag && rec_eq(base, o, r)) { out = idx; break; }
      }
      rslot[i - nw] = out;
    } else {
      const uint32_t t = i - nw - nr;
      st[t] = info[t].code == 0 ? ST_UNDEC : ST_INVALID;
    }
  }
}

// Transaction states read by other transactions of the same launch: a plain load may see a state
// decided in this round or not yet (other workgroups, other XCDs' L2s) -- either is correct, the
// rule only ever acts on decided states; an undecided view waits for the next round
__device__ __forceinline__ uint8_t st_ld(const uint8_t *st, uint32_t g) { return st[g]; }
__device__ __forceinline__ void st_set(uint8_t *st, uint32_t g, uint8_t s) { st[g] = s; }

// fixpoint round r (1-based): every undecided transaction evaluates its reads once.  Rounds grow
// with the longest chain of dependent outcomes in the batch -- a read of a key an earlier
// transaction of the batch wrote, whose own validity waits on an earlier one ... -- which is
// short for batches of small blocks (the pass's purpose) and long for a few large blocks over a
// dense key space (C3: ~20 links); the host chooses the per-block chain for those.
// (Re-evaluating inside one launch while other workgroups publish -- device-scope atomic state
// loads, up to 96 passes -- measured slower on MI355X: C3 30.5 M tx/s against 47.3 M, r5e/r5f.)
#define MVB_SPIN 1u
__global__ __launch_bounds__(64) void k_mvb_round(uint32_t ntx, uint32_t r, const MvTxInfo *__restrict__ info,
                                                  const MvRec *__restrict__ reads, const MvRec *__restrict__ writes,
                                                  const uint32_t *__restrict__ rslot, const uint8_t *__restrict__ rstat,
                                                  const MbSlot *__restrict__ btbl, uint8_t *__restrict__ st,
                                                  const uint32_t *__restrict__ bfirst, const uint64_t *__restrict__ bnums,
                                                  uint32_t nb, MvCounters *__restrict__ c) {
  if (c->done || c->unsup) return;
  if (r > 1 && c->undec[(r - 1) & 3] == 0) {  // round r-1 decided everything
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      c->done = 1;
      c->rounds = r - 1;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) c->undec[(r + 1) & 3] = 0;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t und = 0;
  if (g < ntx && st_ld(st, g) == ST_UNDEC) {
    const MvTxInfo I = info[g];
    const uint32_t gb = blk_of(bfirst, nb, g);
    uint8_t s = ST_UNDEC;
    for (uint32_t pass = 0;; pass++) {
      bool conflict = false, open = false;
      for (uint32_t j = I.rbeg; j < I.rbeg + I.rcnt && !conflict; j++) {
        const uint32_t sl = rslot[j];
        int64_t vmax = -1, umax = -1;
        uint32_t vw = 0;
        if (sl != FW_INF) {
          const uint32_t n = min(btbl[sl].nwr, (uint32_t)MB_WR);
          for (uint32_t q = 0; q < n; q++) {
            const uint32_t w = btbl[sl].wr[q];
            const uint32_t gw = writes[w].tx;
            if (gw >= g) continue;
            const uint8_t sw = st_ld(st, gw);
            if (sw == ST_VALID && (int64_t)gw > vmax) { vmax = gw; vw = w; }
            else if (sw == ST_UNDEC && (int64_t)gw > umax) umax = gw;
          }
        }
        if (umax > vmax) { open = true; continue; }  // an undecided later writer decides this read
        if (vmax < 0) {
          conflict = rstat[j] != 0;
          continue;
        }
        const uint32_t wb = blk_of(bfirst, nb, (uint32_t)vmax);
        if (wb == gb) { conflict = true; continue; }  // written earlier in the same block
        const MvRec rd = reads[j];
        const bool has_ver = (rd.flags & MVR_HASVER) != 0;
        if (writes[vw].flags & MVR_DELETE) conflict = has_ver;
        else conflict = !has_ver || rd.blk != bnums[wb] || rd.txn != (uint64_t)((uint32_t)vmax - bfirst[wb]);
      }
      s = conflict ? ST_INVALID : open ? ST_UNDEC : ST_VALID;
      if (s != ST_UNDEC || pass + 1 >= MVB_SPIN) break;
      __builtin_amdgcn_s_sleep(4);
    }
    if (s != ST_UNDEC) st_set(st, g, s);
    und = s == ST_UNDEC;
  }
  for (int off = 32; off > 0; off >>= 1) und += __shfl_down(und, off);
  if ((threadIdx.x & 63u) == 0 && und) atomicAdd(&c->undec[r & 3], und);
}

// commit, part 1: the last VALID writer of each key over the whole batch; capacity check
__global__ __launch_bounds__(256) void k_mvb_last(uint32_t rlast, const MvRec *__restrict__ writes,
                                                  const uint32_t *__restrict__ wslot, const uint8_t *__restrict__ st,
                                                  MbSlot *__restrict__ btbl, uint32_t epoch, MvCounters *__restrict__ c,
                                                  const unsigned long long *__restrict__ top, uint64_t slots_cap,
                                                  uint64_t arena_cap) {
  if (!converged(c, rlast)) return;
  const uint32_t nw = c->nw;
  if ((top[1] + nw) * 10 > slots_cap * 7 || top[0] + c->wbytes > arena_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) c->nomem = 1;
    return;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
    const uint32_t tx = writes[i].tx;
    if (st[tx] == ST_VALID)
      atomicMax(reinterpret_cast<unsigned long long *>(&btbl[wslot[i]].last), ((unsigned long long)epoch << 32) | (tx + 1));
  }
}

// commit, part 2: the last valid writer of each key updates the committed entry in place at
// Height{its block's number, its index in the block}, or is marked for insertion (then
// k_mv_upsert_insert, mode 2, derives the same version from the record's transaction; the records
// stay unchanged -- k_ub_block may be reading their value spans beside these kernels)
__global__ __launch_bounds__(256) void k_mvb_upsert_find(uint32_t rlast, const uint8_t *__restrict__ base,
                                                         const MvRec *__restrict__ recs, const uint32_t *__restrict__ wslot,
                                                         const uint8_t *__restrict__ st, const MbSlot *__restrict__ btbl,
                                                         uint32_t epoch, StateSlot *__restrict__ tbl, uint64_t mask,
                                                         const uint8_t *__restrict__ arena,
                                                         const uint32_t *__restrict__ bfirst,
                                                         const uint64_t *__restrict__ bnums, uint32_t nb,
                                                         uint8_t *__restrict__ pend, const MvCounters *__restrict__ c) {
  if (!converged(c, rlast) || c->nomem) return;
  const uint32_t n = c->nw;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    MvRec w = recs[i];
    pend[i] = 0;
    if (st[w.tx] != ST_VALID || btbl[wslot[i]].last != (((uint64_t)epoch << 32) | (w.tx + 1))) continue;
    const uint32_t b = blk_of(bfirst, nb, w.tx);
    const uint64_t vb = bnums[b], vt = w.tx - bfirst[b];
    const bool del = (w.flags & MVR_DELETE) != 0;
    const int64_t s = state_find(tbl, mask, arena, base, w);
    if (s >= 0) {
      tbl[s].blk = vb;
      tbl[s].txn = vt;
      tbl[s].tag = del ? (tbl[s].tag & ~MV_TAG_PRESENT) : (tbl[s].tag | MV_TAG_PRESENT);
    } else if (!del) {
      pend[i] = 1;
    }
  }
}
