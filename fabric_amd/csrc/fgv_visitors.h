// fgv_visitors.h -- pbwire visitors for the Fabric messages on the committer path (one
// struct per message; field numbers from vendor/github.com/hyperledger/fabric-protos-go,
// SURVEY.md Appendix B).  Shared by the committer (fgv_block.cpp) and MVCC (fgv_mvcc.cpp).
#pragma once
#include <stdint.h>

#include <vector>

#include "pbwire.h"

using pbw::Span;

namespace fgvb {

// ------------------------------------------------------------------ small helpers
// Word-wise 64-bit hash (four independent multiply-rotate lanes over 32-byte strides) -- used
// for the identity index, where serialized identities are ~800 B PEM certificates.  Not
// cryptographic: every hit is confirmed by an exact byte compare.
inline uint64_t hash_bytes(const uint8_t *p, size_t n, uint64_t h = 0x9E3779B97F4A7C15ull) {
  constexpr uint64_t M1 = 0x9E3779B97F4A7C15ull, M2 = 0xC2B2AE3D27D4EB4Full, M3 = 0x165667B19E3779F9ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto ld = [](const uint8_t *q) { uint64_t w; memcpy(&w, q, 8); return w; };
  uint64_t a = h ^ n, b = h + M1, c = h ^ M2, d = h - M3;
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    a = rotl(a + ld(p + i) * M2, 31) * M1;
    b = rotl(b + ld(p + i + 8) * M2, 31) * M1;
    c = rotl(c + ld(p + i + 16) * M2, 31) * M1;
    d = rotl(d + ld(p + i + 24) * M2, 31) * M1;
  }
  uint64_t x = rotl(a, 1) + rotl(b, 7) + rotl(c, 12) + rotl(d, 18);
  for (; i + 8 <= n; i += 8) x = rotl(x ^ (ld(p + i) * M2), 27) * M1 + M3;
  uint64_t t = 0;
  for (int k = 0; i < n; i++, k += 8) t |= (uint64_t)p[i] << k;
  x = (x ^ (t * M2)) * M1;
  x ^= x >> 33;
  x *= M2;
  x ^= x >> 29;
  return x;
}

// ------------------------------------------------------------------ message visitors
struct VEnvelope {
  Span payload, signature;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? payload : signature) = s; return true; }
};
struct VHeader {
  Span channel_header, signature_header;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? channel_header : signature_header) = s; return true; }
};
struct VPayload {
  pbw::MsgField header;
  Span data;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_MSG : n == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) header.add(s); else data = s;
    return true;
  }
};
struct VTimestamp {  // google.protobuf.Timestamp {seconds int64 = 1, nanos int32 = 2}
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span) { return true; }
};
struct VChannelHeader {
  int32_t type = 0;
  uint64_t epoch = 0;
  Span channel_id, tx_id, extension;
  pbw::Kind kind(uint32_t n) {
    switch (n) {
      case 1: case 2: case 6: return pbw::K_VARINT;
      case 3: return pbw::K_MSG;
      case 4: case 5: return pbw::K_STRING;
      case 7: case 8: return pbw::K_BYTES;
      default: return pbw::K_NONE;
    }
  }
  void on_varint(uint32_t n, uint64_t v) {
    if (n == 1) type = pbw::as_int32(v);
    else if (n == 6) epoch = v;
  }
  bool on_len(uint32_t n, Span s) {
    if (n == 3) { VTimestamp t; return pbw::decode(s.p, s.n, t); }
    if (n == 4) channel_id = s;
    else if (n == 5) tx_id = s;
    else if (n == 7) extension = s;
    return true;
  }
};
struct VSignatureHeader {
  Span creator, nonce;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? creator : nonce) = s; return true; }
};
struct VTransactionAction {
  Span header, payload;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? header : payload) = s; return true; }
};
struct VTransaction {
  pbw::SmallVec<VTransactionAction, 2> actions;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    VTransactionAction a;
    if (!pbw::decode(s.p, s.n, a)) return false;
    actions.push_back(a);
    return true;
  }
};
struct VEndorsement {
  Span endorser, signature;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? endorser : signature) = s; return true; }
};
struct VEndorsedAction {
  Span prp;
  pbw::SmallVec<VEndorsement, 8> ends;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : n == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { prp = s; return true; }
    VEndorsement e;
    if (!pbw::decode(s.p, s.n, e)) return false;
    ends.push_back(e);
    return true;
  }
};
struct VCcActionPayload {
  Span ccpp;
  bool has_action = false;
  VEndorsedAction action;  // all occurrences merged in order
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : n == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { ccpp = s; return true; }
    has_action = true;
    return pbw::decode(s.p, s.n, action);
  }
};
struct VPrp {
  Span proposal_hash, extension;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? proposal_hash : extension) = s; return true; }
};
struct VChaincodeID {
  Span path, name, version;
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_STRING : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? path : n == 2 ? name : version) = s; return true; }
};
struct VResponse {
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_VARINT : n == 2 ? pbw::K_STRING : n == 3 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span) { return true; }
};
struct VCcAction {
  Span results, events;
  bool has_ccid = false;
  VChaincodeID ccid;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_BYTES : (n == 3 || n == 4) ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { results = s; return true; }
    if (n == 2) { events = s; return true; }
    if (n == 3) { VResponse r; return pbw::decode(s.p, s.n, r); }
    has_ccid = true;
    return pbw::decode(s.p, s.n, ccid);
  }
};
struct VHdrExt {  // ChaincodeHeaderExtension {chaincode_id = 2}
  bool has_ccid = false;
  VChaincodeID ccid;
  pbw::Kind kind(uint32_t n) { return n == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) { has_ccid = true; return pbw::decode(s.p, s.n, ccid); }
};
struct VCcEvent {
  Span chaincode_id;
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_STRING : n == 4 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { if (n == 1) chaincode_id = s; return true; }
};
// --- rwset (validated in full; the committer only needs namespaces + write presence)
struct VVersion {
  uint64_t block = 0, tx = 0;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t n, uint64_t v) { (n == 1 ? block : tx) = v; }
  bool on_len(uint32_t, Span) { return true; }
};
struct VKVRead {
  Span key;
  bool has_ver = false;
  VVersion ver;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    has_ver = true;
    return pbw::decode(s.p, s.n, ver);
  }
};
struct VQueryReads {
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) { VKVRead r; return pbw::decode(s.p, s.n, r); }
};
struct VMerkle {
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 2) ? pbw::K_VARINT : n == 3 ? pbw::K_REP_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span) { return true; }
};
struct VRangeQuery {
  pbw::Kind kind(uint32_t n) {
    return (n == 1 || n == 2) ? pbw::K_STRING : n == 3 ? pbw::K_VARINT : (n == 4 || n == 5) ? pbw::K_MSG : pbw::K_NONE;
  }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 4) { VQueryReads q; return pbw::decode(s.p, s.n, q); }
    if (n == 5) { VMerkle m; return pbw::decode(s.p, s.n, m); }
    return true;
  }
};
struct VKVWrite {
  Span key, value;
  bool is_delete = false;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_VARINT : n == 3 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { is_delete = v != 0; }
  bool on_len(uint32_t n, Span s) { (n == 1 ? key : value) = s; return true; }
};
struct VMetaEntry {
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span) { return true; }
};
struct VMetaWrite {  // KVMetadataWrite {key string=1, entries=2}
  Span key;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    VMetaEntry e;
    return pbw::decode(s.p, s.n, e);
  }
};
struct VKVRWSet {
  uint32_t nreads = 0, nrq = 0, nwrites = 0, nmeta = 0;
  std::vector<VKVRead> *reads = nullptr;     // optional capture (MVCC)
  std::vector<VKVWrite> *writes = nullptr;
  std::vector<Span> *meta_keys = nullptr;    // optional capture (key-level endorsement)
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 4) ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) {
      VKVRead r;
      if (!pbw::decode(s.p, s.n, r)) return false;
      nreads++;
      if (reads) reads->push_back(r);
      return true;
    }
    if (n == 2) { nrq++; VRangeQuery q; return pbw::decode(s.p, s.n, q); }
    if (n == 3) {
      VKVWrite w;
      if (!pbw::decode(s.p, s.n, w)) return false;
      nwrites++;
      if (writes) writes->push_back(w);
      return true;
    }
    nmeta++;
    VMetaWrite m;
    if (!pbw::decode(s.p, s.n, m)) return false;
    if (meta_keys) meta_keys->push_back(m.key);
    return true;
  }
};
struct VHashRead {  // KVReadHash {key_hash bytes=1, version=2}
  Span key;
  bool has_ver = false;
  VVersion ver;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : n == 2 ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    has_ver = true;
    return pbw::decode(s.p, s.n, ver);
  }
};
struct VHashWrite {  // KVWriteHash {key_hash=1, is_delete=2, value_hash=3, is_purge=4}
  Span key, value_hash;
  bool is_delete = false;
  pbw::Kind kind(uint32_t n) { return (n == 1 || n == 3) ? pbw::K_BYTES : (n == 2 || n == 4) ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t n, uint64_t v) { if (n == 2) is_delete = v != 0; }
  bool on_len(uint32_t n, Span s) { (n == 1 ? key : value_hash) = s; return true; }
};
struct VHashMeta {  // KVMetadataWriteHash {key_hash bytes=1, entries=2}
  Span key;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_BYTES : n == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { key = s; return true; }
    VMetaEntry e;
    return pbw::decode(s.p, s.n, e);
  }
};
struct VHashedRWSet {
  uint32_t nreads = 0, nwrites = 0, nmeta = 0;
  std::vector<VHashRead> *reads = nullptr;  // optional capture (MVCC)
  std::vector<VHashWrite> *writes = nullptr;
  std::vector<Span> *meta_keys = nullptr;   // optional capture (key-level endorsement)
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) {
      nreads++;
      VHashRead r;
      if (!pbw::decode(s.p, s.n, r)) return false;
      if (reads) reads->push_back(r);
      return true;
    }
    if (n == 2) {
      nwrites++;
      VHashWrite w;
      if (!pbw::decode(s.p, s.n, w)) return false;
      if (writes) writes->push_back(w);
      return true;
    }
    nmeta++;
    VHashMeta m;
    if (!pbw::decode(s.p, s.n, m)) return false;
    if (meta_keys) meta_keys->push_back(m.key);
    return true;
  }
};
struct VCollHashed {
  Span name, hashed;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : (n == 2 || n == 3) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) name = s;
    else if (n == 2) hashed = s;
    return true;
  }
};
struct VNsRwSet {
  Span ns, rwset;
  pbw::SmallVec<VCollHashed, 2> coll;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_BYTES : n == 3 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 1) { ns = s; return true; }
    if (n == 2) { rwset = s; return true; }
    VCollHashed c;
    if (!pbw::decode(s.p, s.n, c)) return false;
    coll.push_back(c);
    return true;
  }
};
struct VTxRwSet {
  pbw::SmallVec<VNsRwSet, 4> ns;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_VARINT : n == 2 ? pbw::K_REP_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    VNsRwSet r;
    if (!pbw::decode(s.p, s.n, r)) return false;
    ns.push_back(r);
    return true;
  }
};
struct VSerializedIdentity {
  Span mspid, id_bytes;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) { (n == 1 ? mspid : id_bytes) = s; return true; }
};
struct VBlockData {
  std::vector<Span> data;
  VBlockData() { data.reserve(1024); }
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_REP_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span s) {
    data.push_back(s);
    // the framing walk is a chain of dependent loads (each tag follows the previous envelope's
    // end): over a cold multi-MB block each is a DRAM miss.  Envelopes of a block are of similar
    // size, so the lines where the next 8 tags would be if they were the same size are requested
    // now (two lines each: the guess is off by a few bytes when sizes differ a little)
    const size_t step = (size_t)s.n + 4;
    if (step >= 256)
      for (size_t k = 1; k <= 8; k++) {
        __builtin_prefetch(s.p + s.n + k * step - 32);
        __builtin_prefetch(s.p + s.n + k * step + 32);
      }
    return true;
  }
};
struct VSkipMsg {  // BlockHeader / BlockMetadata: validated, contents unused
  uint32_t rep_bytes_field = 0;
  pbw::Kind kind(uint32_t n) { return n == 1 ? (rep_bytes_field ? pbw::K_REP_BYTES : pbw::K_VARINT) : (n == 2 || n == 3) ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t, Span) { return true; }
};
struct VBlock {
  VBlockData data;
  pbw::Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? pbw::K_MSG : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t) {}
  bool on_len(uint32_t n, Span s) {
    if (n == 2) return pbw::decode(s.p, s.n, data);
    VSkipMsg m;
    m.rep_bytes_field = (n == 3);
    return pbw::decode(s.p, s.n, m);
  }
};

// --- policies
struct VMSPRole {
  Span mspid;
  int32_t role = 0;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_STRING : n == 2 ? pbw::K_VARINT : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { role = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { mspid = s; return true; }
};
struct VPrincipal {
  int32_t cls = 0;
  Span principal;
  pbw::Kind kind(uint32_t n) { return n == 1 ? pbw::K_VARINT : n == 2 ? pbw::K_BYTES : pbw::K_NONE; }
  void on_varint(uint32_t, uint64_t v) { cls = pbw::as_int32(v); }
  bool on_len(uint32_t, Span s) { principal = s; return true; }
};

}  // namespace fgvb

