// blockdev_parse.h -- the per-transaction protobuf walk (parse_one) and the identity lookup
// shared by the global-walk kernels (blockdev.hip) and the LDS-staged walk (blockdev_lds.hip).
#pragma once
#include "blockdev_dev.h"

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
