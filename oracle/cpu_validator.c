/* cpu_validator.c -- TEST / BASELINE INFRASTRUCTURE ONLY (never linked by libfgv.so).
 *
 * A plain-C restatement of the committer's per-transaction validation for endorser
 * transactions, for the CPU baseline of bench.py (cpu_baseline, kind "port"): the same
 * algorithm as oracle/v20.py validate_blocks restricted to the headline workload's shapes --
 * one chaincode whose endorsement policy is OutOf(n, [msp_i.member]), no collections, no
 * key-level parameters, P-256 identities given by the caller's registry.  Anything outside
 * that subset makes the call return 0xFD for the transaction (the bench then reports the
 * baseline as unavailable).  Reference behaviour restated (file:line in /root/reference):
 *   core/committer/txvalidator/v20/validator.go:297-453   validateTx precedence
 *   core/common/validation/msgvalidation.go:26-64, 165-245  creator signature, endorser tx
 *   core/committer/txvalidator/v20/plugindispatcher/dispatcher.go:102-221   Dispatch
 *   core/handlers/validation/builtin/v20/validation_logic.go:185-217 + common/cauthdsl/
 *     cauthdsl.go:24-92 + common/policies/policy.go:363-395   endorsement policy
 *   core/committer/txvalidator/v20/validator.go:279-295, 460-481   txid duplicates
 * Crypto: SHA-256 and ECDSA-P256 (Go DER + low-S front, OpenSSL 3 back-end) from
 * fgv_oracle.c.  Threads validate whole blocks; the cross-block txid index and
 * markTXIdDuplicates run afterwards in block order. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fgv_oracle.h"

enum { C_VALID = 0, C_BAD_PAYLOAD = 2, C_BAD_HDR = 3, C_BAD_CREATOR = 4, C_BAD_ETX = 5, C_UNSUP_PAYLOAD = 7,
       C_BAD_TXID = 8, C_DUP_TXID = 9, C_POLICY = 10, C_BAD_HDR_EXT = 19, C_BAD_RESP = 21, C_BAD_RWSET = 22,
       C_ILLEGAL_WS = 23, C_INVALID_CC = 25, C_OTHER = 255, C_UNSUP = 0xFD };

/* ------------------------------------------------------------ protobuf wire */
typedef struct {
  const uint8_t *p;
  size_t n;
} span;

static int rd_varint(const uint8_t **p, const uint8_t *e, uint64_t *v) {
  uint64_t x = 0;
  for (int i = 0; i < 10; i++) {
    if (*p >= e) return 0;
    const uint8_t c = *(*p)++;
    if (i == 9 && c > 1) return 0;
    x |= (uint64_t)(c & 0x7f) << (7 * i);
    if (c < 0x80) {
      *v = x;
      return 1;
    }
  }
  return 0;
}

/* one field of a message: number, wire type, varint value or length-delimited span */
typedef struct {
  uint32_t num, wt;
  uint64_t v;
  span s;
} field;

static int next_field(const uint8_t **p, const uint8_t *e, field *f) {
  uint64_t tag;
  if (!rd_varint(p, e, &tag)) return 0;
  f->num = (uint32_t)(tag >> 3);
  f->wt = (uint32_t)(tag & 7);
  if (f->num == 0) return 0;
  switch (f->wt) {
    case 0: return rd_varint(p, e, &f->v);
    case 1:
      if (e - *p < 8) return 0;
      *p += 8;
      return 1;
    case 5:
      if (e - *p < 4) return 0;
      *p += 4;
      return 1;
    case 2: {
      uint64_t l;
      if (!rd_varint(p, e, &l) || l > (uint64_t)(e - *p)) return 0;
      f->s.p = *p;
      f->s.n = (size_t)l;
      *p += l;
      return 1;
    }
    default: return 0; /* groups: outside the subset (treated as malformed) */
  }
}

#define FOR_FIELDS(msg, f)                                                              \
  for (const uint8_t *_p = (msg).p, *_e = (msg).p + (msg).n; _p < _e;)                 \
    if (!next_field(&_p, _e, &(f))) goto bad;                                           \
    else

static int sp_eq(span a, span b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }

/* ------------------------------------------------------------ registry (caller's) */
typedef struct {
  const uint8_t *ser_buf;
  const uint64_t *ser_off;
  const uint32_t *ser_len;
  const uint8_t *keys;   /* 64 B per identity: P-256 x || y */
  const int32_t *msp;    /* interned Mspid */
  const int32_t *canon;  /* dedup id (Mspid + Id) */
  const uint8_t *ok;     /* 1: deserializes, validates and verifies with its P-256 key */
  size_t n;
  uint32_t *table;       /* open addressing: index + 1 */
  size_t mask;
  void **eckey;          /* parsed once per identity (oracle_p256_key_new) */
} registry;

static uint64_t fnv(const uint8_t *p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  return h ^ (h >> 29);
}

static int lookup(const registry *R, span ser) {
  for (size_t pos = fnv(ser.p, ser.n) & R->mask;; pos = (pos + 1) & R->mask) {
    const uint32_t e = R->table[pos];
    if (!e) return -1;
    const size_t i = e - 1;
    if (R->ser_len[i] == ser.n && memcmp(R->ser_buf + R->ser_off[i], ser.p, ser.n) == 0) return (int)i;
  }
}

static int verify(const registry *R, int id, span msg, span sig) {
  uint8_t d[32];
  oracle_sha256(msg.p, msg.n, d);
  return oracle_p256_verify_der_key(R->eckey[id], sig.p, sig.n, d, 32) == 0;
}

static void hex64(const uint8_t d[32], char out[64]) {
  static const char H[] = "0123456789abcdef";
  for (int i = 0; i < 32; i++) out[2 * i] = H[d[i] >> 4], out[2 * i + 1] = H[d[i] & 15];
}

typedef struct {
  const registry *R;
  span channel, ccname;
  const int32_t *pol_msp;
  int pol_k, pol_n;
} model;

/* per transaction: code, the txid it reached the ledger check with, its index entry */
typedef struct {
  uint8_t code, reached, indexed;
  char txid[64];
  char index[64];
  uint32_t index_len;
} txout;

/* validateTx for one envelope (C2 subset) */
static void validate_tx(const model *M, span d, txout *o) {
  field f;
  o->code = C_OTHER;
  o->reached = o->indexed = 0;
  span payload = {0}, esig = {0};
  int has_sig = 0;
  FOR_FIELDS(d, f) {
    if (f.num == 1 && f.wt == 2) payload = f.s;
    else if (f.num == 2 && f.wt == 2) esig = f.s, has_sig = 1;
  }
  span hdr = {0}, data = {0};
  int has_hdr = 0;
  {
    const uint8_t *p = payload.p, *e = payload.p + payload.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_PAYLOAD; return; }
      if (f.num == 1 && f.wt == 2) hdr = f.s, has_hdr = 1;
      else if (f.num == 2 && f.wt == 2) data = f.s;
    }
  }
  span chb = {0}, shb = {0};
  {
    const uint8_t *p = hdr.p, *e = hdr.p + hdr.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_PAYLOAD; return; }
      if (f.num == 1 && f.wt == 2) chb = f.s;
      else if (f.num == 2 && f.wt == 2) shb = f.s;
    }
  }
  uint64_t type = 0, epoch = 0;
  span chan = {0}, txid = {0}, ext = {0}, creator = {0}, nonce = {0};
  int c_ok = 1, s_ok = 1;
  {
    const uint8_t *p = chb.p, *e = chb.p + chb.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { c_ok = 0; break; }
      if (f.num == 1 && f.wt == 0) type = f.v;
      else if (f.num == 4 && f.wt == 2) chan = f.s;
      else if (f.num == 5 && f.wt == 2) txid = f.s;
      else if (f.num == 6 && f.wt == 0) epoch = f.v;
      else if (f.num == 7 && f.wt == 2) ext = f.s;
    }
    p = shb.p, e = shb.p + shb.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { s_ok = 0; break; }
      if (f.num == 1 && f.wt == 2) creator = f.s;
      else if (f.num == 2 && f.wt == 2) nonce = f.s;
    }
  }
  /* GetOrComputeTxIDFromEnvelope (the txid index entry) */
  if (has_hdr && c_ok) {
    if (txid.n) {
      if (txid.n <= 64) {
        memcpy(o->index, txid.p, txid.n);
        o->index_len = (uint32_t)txid.n;
        o->indexed = 1;
      } else {
        o->code = C_UNSUP;  /* (outside the subset: long txid strings) */
        return;
      }
    } else if (s_ok) {
      uint8_t *m = malloc(nonce.n + creator.n + 1);
      memcpy(m, nonce.p, nonce.n);
      memcpy(m + nonce.n, creator.p, creator.n);
      uint8_t dg[32];
      oracle_sha256(m, nonce.n + creator.n, dg);
      free(m);
      hex64(dg, o->index);
      o->index_len = 64;
      o->indexed = 1;
    }
  }
  if (!has_hdr) { o->code = C_BAD_HDR; return; }
  if (!c_ok || !s_ok) { o->code = C_BAD_HDR; return; }
  if (type != 3 && type != 2 && type != 1) { o->code = C_BAD_HDR; return; }
  if (epoch != 0 || nonce.n == 0 || creator.n == 0) { o->code = C_BAD_HDR; return; }
  if (!has_sig || esig.n == 0) { o->code = C_BAD_CREATOR; return; }
  if (chan.n == 0) { o->code = C_UNSUP; return; }
  if (!sp_eq(chan, M->channel)) { o->code = C_BAD_CREATOR; return; }
  const int cid = lookup(M->R, creator);
  if (cid < 0 || !M->R->ok[cid]) { o->code = C_BAD_CREATOR; return; }
  if (!verify(M->R, cid, payload, esig)) { o->code = C_BAD_CREATOR; return; }
  if (type != 3) { o->code = C_UNSUP; return; }
  /* CheckTxID */
  {
    uint8_t *m = malloc(nonce.n + creator.n + 1);
    memcpy(m, nonce.p, nonce.n);
    memcpy(m + nonce.n, creator.p, creator.n);
    uint8_t dg[32];
    oracle_sha256(m, nonce.n + creator.n, dg);
    free(m);
    char hx[64];
    hex64(dg, hx);
    if (txid.n != 64 || memcmp(hx, txid.p, 64) != 0) { o->code = C_BAD_TXID; return; }
    memcpy(o->txid, hx, 64);
  }
  /* validateEndorserTransaction */
  span act_hdr = {0}, act_pl = {0};
  int nact = 0;
  if (data.n == 0) { o->code = C_BAD_ETX; return; }
  {
    const uint8_t *p = data.p, *e = data.p + data.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) {
        nact++;
        const uint8_t *q = f.s.p, *qe = f.s.p + f.s.n;
        field g;
        while (q < qe) {
          if (!next_field(&q, qe, &g)) { o->code = C_BAD_ETX; return; }
          if (g.num == 1 && g.wt == 2) act_hdr = g.s;
          else if (g.num == 2 && g.wt == 2) act_pl = g.s;
        }
      }
    }
  }
  if (nact != 1 || act_hdr.n == 0) { o->code = C_BAD_ETX; return; }
  {
    span an = {0}, ac = {0};
    const uint8_t *p = act_hdr.p, *e = act_hdr.p + act_hdr.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) ac = f.s;
      else if (f.num == 2 && f.wt == 2) an = f.s;
    }
    if (an.n == 0 || ac.n == 0) { o->code = C_BAD_ETX; return; }
  }
  span ccpp = {0}, action = {0};
  int has_action = 0;
  {
    const uint8_t *p = act_pl.p, *e = act_pl.p + act_pl.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) ccpp = f.s;
      else if (f.num == 2 && f.wt == 2) action = f.s, has_action = 1;
    }
  }
  if (!has_action) { o->code = C_UNSUP; return; }
  span prp = {0};
  span ends[32];
  int nend = 0;
  {
    const uint8_t *p = action.p, *e = action.p + action.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) prp = f.s;
      else if (f.num == 2 && f.wt == 2) {
        if (nend == 32) { o->code = C_UNSUP; return; }
        ends[nend++] = f.s;
      }
    }
  }
  span prop_hash = {0}, cca = {0};
  {
    const uint8_t *p = prp.p, *e = prp.p + prp.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) prop_hash = f.s;
      else if (f.num == 2 && f.wt == 2) cca = f.s;
    }
  }
  if (ccpp.n == 0) { o->code = C_BAD_ETX; return; }
  {
    uint8_t *m = malloc(chb.n + act_hdr.n + ccpp.n + 1);
    memcpy(m, chb.p, chb.n);
    memcpy(m + chb.n, act_hdr.p, act_hdr.n);
    memcpy(m + chb.n + act_hdr.n, ccpp.p, ccpp.n);
    uint8_t dg[32];
    oracle_sha256(m, chb.n + act_hdr.n + ccpp.n, dg);
    free(m);
    if (prop_hash.n != 32 || memcmp(dg, prop_hash.p, 32) != 0) { o->code = C_BAD_ETX; return; }
  }
  o->reached = 1;
  /* Dispatch */
  span ccid = {0};
  int has_ccid = 0;
  {
    const uint8_t *p = ext.p, *e = ext.p + ext.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_HDR_EXT; return; }
      if (f.num == 2 && f.wt == 2) {
        has_ccid = 1;
        const uint8_t *q = f.s.p, *qe = f.s.p + f.s.n;
        field g;
        while (q < qe) {
          if (!next_field(&q, qe, &g)) { o->code = C_BAD_HDR_EXT; return; }
          if (g.num == 2 && g.wt == 2) ccid = g.s;
        }
      }
    }
  }
  if (prp.n == 0 || cca.n == 0) { o->code = C_BAD_RESP; return; }
  span results = {0}, events = {0}, acc_name = {0}, acc_ver = {0};
  int has_events = 0, has_accid = 0;
  {
    const uint8_t *p = cca.p, *e = cca.p + cca.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_RESP; return; }
      if (f.num == 1 && f.wt == 2) results = f.s;
      else if (f.num == 2 && f.wt == 2) events = f.s, has_events = 1;
      else if (f.num == 4 && f.wt == 2) {
        has_accid = 1;
        const uint8_t *q = f.s.p, *qe = f.s.p + f.s.n;
        field g;
        while (q < qe) {
          if (!next_field(&q, qe, &g)) { o->code = C_BAD_RESP; return; }
          if (g.num == 2 && g.wt == 2) acc_name = g.s;
          else if (g.num == 3 && g.wt == 2) acc_ver = g.s;
        }
      }
    }
  }
  /* the rwset: namespaces and their writes (collections: outside the subset) */
  span nss[16];
  int nns = 0, writes_cc = 0, other_writes = 0;
  {
    const uint8_t *p = results.p, *e = results.p + results.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_RWSET; return; }
      if (f.num == 2 && f.wt == 2) {
        span ns = {0}, kv = {0};
        const uint8_t *q = f.s.p, *qe = f.s.p + f.s.n;
        field g;
        while (q < qe) {
          if (!next_field(&q, qe, &g)) { o->code = C_BAD_RWSET; return; }
          if (g.num == 1 && g.wt == 2) ns = g.s;
          else if (g.num == 2 && g.wt == 2) kv = g.s;
          else if (g.num == 3) { o->code = C_UNSUP; return; }
        }
        int nw = 0;
        const uint8_t *r = kv.p, *re = kv.p + kv.n;
        while (r < re) {
          if (!next_field(&r, re, &g)) { o->code = C_BAD_RWSET; return; }
          if (g.num == 3) nw++;
          else if (g.num == 2 || g.num == 4) { o->code = C_UNSUP; return; } /* range queries, metadata */
        }
        if (nns == 16) { o->code = C_UNSUP; return; }
        nss[nns++] = ns;
        if (nw) {
          if (sp_eq(ns, M->ccname)) writes_cc = 1;
          else other_writes = 1;
        }
      }
    }
  }
  (void)writes_cc;
  if (!has_ccid || !has_accid) { o->code = C_OTHER; return; }
  if (ccid.n == 0 || !sp_eq(ccid, acc_name) || acc_ver.n == 0) { o->code = C_INVALID_CC; return; }
  if (has_events) {
    span evcc = {0};
    const uint8_t *p = events.p, *e = events.p + events.n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_OTHER; return; }
      if (f.num == 1 && f.wt == 2) evcc = f.s;
    }
    if (!sp_eq(evcc, ccid)) { o->code = C_OTHER; return; }
  }
  for (int a = 0; a < nns; a++)
    for (int b = a + 1; b < nns; b++)
      if (sp_eq(nss[a], nss[b])) { o->code = C_ILLEGAL_WS; return; }
  if (!sp_eq(ccid, M->ccname) || other_writes) { o->code = C_UNSUP; return; } /* one chaincode only */
  /* SignatureSetToValidIdentities: deserialize, dedup (Mspid + Id), verify, in order */
  int32_t ids[32];
  int nids = 0;
  for (int k = 0; k < nend; k++) {
    span endorser = {0}, sig = {0};
    const uint8_t *p = ends[k].p, *e = ends[k].p + ends[k].n;
    while (p < e) {
      if (!next_field(&p, e, &f)) { o->code = C_BAD_ETX; return; }
      if (f.num == 1 && f.wt == 2) endorser = f.s;
      else if (f.num == 2 && f.wt == 2) sig = f.s;
    }
    const int id = lookup(M->R, endorser);
    if (id < 0 || !M->R->ok[id]) continue;
    int dup = 0;
    for (int q = 0; q < nids; q++) dup |= M->R->canon[ids[q]] == M->R->canon[id];
    if (dup) continue;
    uint8_t *m = malloc(prp.n + endorser.n + 1);
    memcpy(m, prp.p, prp.n);
    memcpy(m + prp.n, endorser.p, endorser.n);
    const span msg = {m, prp.n + endorser.n};
    const int good = verify(M->R, id, msg, sig);
    free(m);
    if (good) ids[nids++] = id;
  }
  /* OutOf(k, [SignedBy(msp_i member)]): greedy, each principal takes the first unused signer */
  uint32_t used = 0;
  int sat = 0;
  for (int i = 0; i < M->pol_n; i++)
    for (int q = 0; q < nids; q++)
      if (!((used >> q) & 1u) && M->R->msp[ids[q]] == M->pol_msp[i]) {
        used |= 1u << q;
        sat++;
        break;
      }
  o->code = sat >= M->pol_k ? C_VALID : C_POLICY;
  return;
bad:
  o->code = C_OTHER;
}

/* Block data: repeated bytes data = 1 inside BlockData (Block field 2) */
static int block_envs(span blk, span **out, size_t *n) {
  field f;
  span data = {0};
  *out = NULL;
  *n = 0;
  FOR_FIELDS(blk, f) {
    if (f.num == 2 && f.wt == 2) data = f.s;
  }
  size_t cap = 0;
  FOR_FIELDS(data, f) {
    if (f.num == 1 && f.wt == 2) {
      if (*n == cap) {
        cap = cap ? 2 * cap : 512;
        *out = realloc(*out, cap * sizeof(span));
      }
      (*out)[(*n)++] = f.s;
    }
  }
  return 1;
bad:
  free(*out);
  *out = NULL;
  return 0;
}

typedef struct {
  const model *M;
  const uint8_t *const *blocks;
  const size_t *lens;
  size_t nblocks;
  txout **outs;
  size_t *ntx;
  int *bad;
  size_t next;
  pthread_mutex_t mu;
} pool_t;

static void *worker(void *arg) {
  pool_t *P = (pool_t *)arg;
  for (;;) {
    pthread_mutex_lock(&P->mu);
    const size_t b = P->next++;
    pthread_mutex_unlock(&P->mu);
    if (b >= P->nblocks) return NULL;
    span *envs;
    size_t n;
    const span blk = {P->blocks[b], P->lens[b]};
    if (!block_envs(blk, &envs, &n)) {
      P->bad[b] = 1;
      continue;
    }
    P->outs[b] = calloc(n ? n : 1, sizeof(txout));
    P->ntx[b] = n;
    for (size_t i = 0; i < n; i++) validate_tx(P->M, envs[i], &P->outs[b][i]);
    free(envs);
  }
}

/* Returns 0, or -1 for an unparsable block.  flags_out: the concatenated flags of all blocks
 * (caller-sized: the total transaction count), ntx_out[b] per block. */
int oracle_cpu_validate_blocks(const uint8_t *const *blocks, const size_t *lens, size_t nblocks,
                               const char *channel, const char *ccname, const int32_t *pol_msp, int pol_n,
                               int pol_k, const uint8_t *ser_buf, const uint64_t *ser_off,
                               const uint32_t *ser_len, const uint8_t *keys, const int32_t *msp,
                               const int32_t *canon, const uint8_t *ok, size_t nids, uint8_t *flags_out,
                               size_t flags_cap, size_t *ntx_out, int threads) {
  registry R = {ser_buf, ser_off, ser_len, keys, msp, canon, ok, nids, NULL, 0, calloc(nids ? nids : 1, sizeof(void *))};
  for (size_t i = 0; i < nids; i++)
    if (ok[i]) R.eckey[i] = oracle_p256_key_new(keys + 64 * i, keys + 64 * i + 32);
  size_t cap = 16;
  while (cap < 2 * nids) cap <<= 1;
  R.table = calloc(cap, sizeof(uint32_t));
  R.mask = cap - 1;
  for (size_t i = 0; i < nids; i++) {
    size_t pos = fnv(ser_buf + ser_off[i], ser_len[i]) & R.mask;
    while (R.table[pos]) pos = (pos + 1) & R.mask;
    R.table[pos] = (uint32_t)i + 1;
  }
  const model M = {&R, {(const uint8_t *)channel, strlen(channel)}, {(const uint8_t *)ccname, strlen(ccname)},
                   pol_msp, pol_k, pol_n};
  pool_t P = {&M, blocks, lens, nblocks, calloc(nblocks, sizeof(txout *)), ntx_out, calloc(nblocks, sizeof(int)), 0,
              PTHREAD_MUTEX_INITIALIZER};
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, worker, &P);
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  int rc = 0;
  size_t total = 0;
  for (size_t b = 0; b < nblocks; b++) {
    if (P.bad[b]) rc = -1;
    total += ntx_out[b];
  }
  if (!rc && total > flags_cap) rc = -1;
  if (!rc) {
    /* block order: txids indexed by earlier blocks (checkTxIdDupsLedger), then
     * markTXIdDuplicates among the VALID ones */
    size_t icap = 16, o = 0;
    while (icap < 2 * total + 2) icap <<= 1;
    char (*itab)[65] = calloc(icap, 65);
    for (size_t b = 0; b < nblocks; b++) {
      txout *T = P.outs[b];
      for (size_t i = 0; i < ntx_out[b]; i++) {
        if (!T[i].reached) continue;
        size_t pos = fnv((const uint8_t *)T[i].txid, 64) & (icap - 1);
        for (; itab[pos][64]; pos = (pos + 1) & (icap - 1))
          if (itab[pos][64] == 64 && memcmp(itab[pos], T[i].txid, 64) == 0) {
            T[i].code = C_DUP_TXID;
            break;
          }
      }
      {  /* markTXIdDuplicates: a VALID txid seen earlier in the block */
        size_t bcap = 16;
        while (bcap < 2 * ntx_out[b] + 2) bcap <<= 1;
        uint32_t *bt = calloc(bcap, sizeof(uint32_t));
        for (size_t i = 0; i < ntx_out[b]; i++) {
          if (T[i].code != C_VALID) continue;
          size_t pos = fnv((const uint8_t *)T[i].txid, 64) & (bcap - 1);
          for (; bt[pos]; pos = (pos + 1) & (bcap - 1))
            if (memcmp(T[bt[pos] - 1].txid, T[i].txid, 64) == 0) break;
          if (bt[pos]) T[i].code = C_DUP_TXID;
          else bt[pos] = (uint32_t)i + 1;
        }
        free(bt);
      }
      for (size_t i = 0; i < ntx_out[b]; i++) {
        if (!T[i].indexed) continue;
        size_t pos = fnv((const uint8_t *)T[i].index, T[i].index_len) & (icap - 1);
        for (; itab[pos][64]; pos = (pos + 1) & (icap - 1))
          if (itab[pos][64] == (char)T[i].index_len && memcmp(itab[pos], T[i].index, T[i].index_len) == 0) break;
        if (!itab[pos][64]) {
          memcpy(itab[pos], T[i].index, T[i].index_len);
          itab[pos][64] = (char)T[i].index_len;
        }
      }
      for (size_t i = 0; i < ntx_out[b]; i++) flags_out[o++] = T[i].code;
    }
    free(itab);
  }
  for (size_t b = 0; b < nblocks; b++) free(P.outs[b]);
  free(P.outs);
  free(P.bad);
  free(R.table);
  for (size_t i = 0; i < nids; i++) oracle_p256_key_free(R.eckey[i]);
  free(R.eckey);
  return rc;
}
