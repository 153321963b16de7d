// blockdev.h -- device-resident committer pipeline (blockdev.hip): layouts shared by the
// kernels and the host driver in fgv_block.cpp.  Not part of the C ABI.
//
// The block batch lives in HBM; the host only splits blocks into envelope spans (a tag/length
// walk) and launches.  Per transaction, on the device:
//   k_bd_parse  single-pass protobuf parse of the envelope (the rules of pbwire.h, restated for
//               device code with fixed capacities) -> DevTx: spans + structural codes
//   k_bd_ident  MSP identity resolution of the creator and every endorser: decode the
//               SerializedIdentity, hash, probe the HBM identity table, exact byte compare
//   k_bd_count  creator checks + device job counts, job slots claimed by wave-aggregated
//               atomics; k_bd_emit writes the SHA-256 jobs and the ECDSA verify jobs straight
//               into the job arrays
//   (k_sha256_jobs, k_der, k_inv, k_prep, k_point as for host-assembled batches)
//   k_bd_fold   code precedence, SignatureSetToValidIdentities, cauthdsl NOutOf fold, txid
//               index entries -> fgv_tx_result records in HBM (input of the device finalize)
// A transaction whose shape exceeds a fixed capacity below sets the overflow flag and the
// batch is redone by the host parser (same rules, unbounded containers).
#pragma once
#include <stdint.h>

#define BD_MAX_END 16      // endorsements per transaction
#define BD_MAX_NS 8        // namespaces per rwset
#define BD_MAX_POL 16      // policies to evaluate (chaincode / collection EPs of the written namespaces)
#define BD_MAX_MERGE 4     // occurrences of one singular message field (protobuf merge)
#define BD_MAX_GROUP 32    // nesting of unknown START_GROUP fields
#define BD_MAX_PNODE 64    // policy tree nodes evaluated per policy (stack depth 16)
#define BD_OCC (1 + BD_MAX_END)  // identity occurrences per tx: creator + endorsers
// k_bd_ident: 16-lane groups per tx (launch: ntx x 16 x BD_ID_PAR threads).  4 resolves a C2
// tx's occurrences at once, but its 4x waves slow k_bd_sha beside it more than they gain
// (MI355X, C2 step 0.79 -> 0.83-0.86 ms): 1
#define BD_ID_PAR 1u
// k_bd_sha digest slots per tx: payload, endorsements 0..BD_MAX_END-1, txid, proposal, index
#define BD_DIG_T (1 + BD_MAX_END)
#define BD_DIG_P (2 + BD_MAX_END)
#define BD_DIG_I (3 + BD_MAX_END)
#define BD_DIG_SLOTS (4 + BD_MAX_END)
#define SHA_GPW 21u     // k_bd_sha: transactions per 64-lane wave (3 lanes each)
// host -> device envelope table, per tx: block, envelope offset, length
#define BD_ENV_WORDS 3

struct DSpan {  // bytes [off, off+len) of block `DevTx::blk`; len 0 == nil
  uint32_t off, len;
};

enum : uint8_t { BDF_INDEX_OK = 1, BDF_INDEX_FROM_TXID = 2, BDF_IDX_SHDR = 4,
                 BDF_VW = 8,      // a vscc that runs reads a written key (GetValidationParameterForKey)
                 BDF_VANY = 16 }; // some vscc runs (PreValidate)
// per-block dependency-extraction hazards (validator_keylevel.go:184-222), after the head's
// counters: [2*blk] = 1 + the first batch tx index whose extraction fails, [2*blk+1] = the same
// for a panic; 0 = a transaction before the shard; UINT32_MAX = none.  k_bd_fold: a tx t of the
// block is past one iff the word <= t.

struct DevTx {
  uint32_t blk;
  uint8_t pre, etx, disp, flags;
  int32_t type;
  DSpan payload, env_sig, nonce, creator, chdr, act_hdr, ccpp, prop_hash, prp, txid;
  DSpan idx_nonce, idx_creator, index_txid;
  uint8_t npol, nend;
  uint8_t nwr;  // vscc namespaces of Dispatch (written namespaces + the invoked chaincode)
  uint8_t kln;  // k_bd_kl: earlier metadata writers of its written keys in its block (KlDev::dep)
  int16_t pol[BD_MAX_POL];
  DSpan end_ser[BD_MAX_END], end_sig[BD_MAX_END];
  DSpan results;  // ChaincodeAction.results when the whole TxReadWriteSet decodes (else nil)
};

// ---------------------------------------------------------------- key-level endorsement
// KeyLevelValidationParameterManagerImpl's per-block state (vpmanagerimpl.go:113-233) on the
// device.  k_bd_parse records every metadata write of every transaction whose rwset decodes
// (ExtractValidationParameterDependency, vpmanagerimpl.go:258-292) and every delete of a key that
// holds a committed VALIDATION_PARAMETER (tx_ops.go:17-51: it clears the parameter) in a
// chained hash table keyed by (namespace, collection, key); k_bd_kl then finds, per written key,
// the earlier metadata writers of the same block (the txs whose vscc result a
// GetValidationParameterForKey waits for) and the changes made by earlier blocks of the batch
// (outside the model: the reference commits block k before block k+1 reads the parameter).
// k_bd_fold folds every transaction against the committed parameters in parallel; the last
// transaction of a block to finish then walks the block's dependent transactions in order.
enum : uint32_t { KL_MD = 0, KL_DEL = 1 };
struct KlRec {
  uint64_t hash;
  uint32_t tx, blk, kind, next;  // next: record index + 1 in the bucket's chain (0: end)
  uint32_t ns_off, ns_len, coll_off, coll_len, key_off, key_len;  // spans of block `blk`
};
#define KL_DEPS 8      // earlier metadata writers of one transaction's keys
#define KL_MAXDEP 64   // dependent transactions per block
#define KL_BLK_WORDS 4 // per block: first tx, tx count, fold completions, dependents
struct KlDev {
  KlRec *rec;
  unsigned long long *head;  // bucket -> (seq << 32) | (record index + 1); other seqs read as empty
  uint32_t hmask, rcap, seq, on;  // on: whole batch (no shard ranges); the fold's walk needs the fused finalize
  uint32_t *cnt;       // records (the batch counters' word 11)
  uint32_t *blk;       // KL_BLK_WORDS per block (head region, reset per batch)
  uint32_t *deplist;   // KL_MAXDEP per block
  uint32_t *dep;       // KL_DEPS per transaction
};

// per-tx job bookkeeping written by k_bd_count / k_bd_emit
enum { BJ_C = 0, BJ_T, BJ_P, BJ_E, BJ_I, BJ_KINDS };
struct DevJobIdx {
  uint32_t cnt[BJ_KINDS];  // jobs of each kind (creator-payload, txid, proposal, endorsement, index)
  uint32_t base[BJ_KINDS]; // first job of each kind (slot within the kind's group)
};
// the verify job columns (fgv_block_jobs_reserve layout, stride = the batch's capacity):
// k_bd_count writes them when given (sig_ptr != null), else k_bd_emit
struct BdVerifyCols {
  uint64_t *sig_ptr;
  uint32_t *sig_len, *key_slot, *dig_idx;
};

// identity registry in HBM (built on the host from the channel model)
struct DevIdent {
  uint32_t msp_off, msp_len, idb_off, idb_len;  // into the identity byte arena
  int32_t key_slot;   // P-256 key table slot (vclass 0)
  int32_t msp;        // interned Mspid
  uint32_t canon;     // dedup id (Mspid + Id)
  uint32_t valid;
  uint32_t vclass;    // Verify: 0 on the GPU (SHA-256 or, hash3, SHA3-256 digests), 1 always fails, 2 outside
                      // the engine (P-384); 3 undeserializable
  uint32_t roles;     // SatisfiesPrincipal(ROLE r) bits
  uint32_t roles_known;
  uint32_t ous_known;        // GetOrganizationalUnits known: ident_ous[ou_off .. ou_off + ou_n)
  uint32_t ou_off, ou_n;
  uint32_t hash3;     // SHA3 MSP (vclass 0): its Verify digests are SHA3-256 (k_bd_sha3)
};
// one leaf principal (fgv_channel.h Prin; kinds DPR_* = PR_*)
enum : int32_t { DPR_ROLE = 0, DPR_IDENTITY = 1, DPR_OU = 2, DPR_NOMINAL = 3, DPR_NEVER = 4, DPR_UNRESOLVED = 5 };
struct DevPrin {
  int32_t kind, msp, role;
  uint32_t canon;
  int32_t ou;
  uint32_t pad;
};

struct DevPNode {
  int32_t type;       // 1 NOutOf, 2 SignedBy
  int32_t n;          // NOutOf threshold
  uint32_t p0, np;    // SignedBy: the principal's leaves prins[p0 .. p0+np), all must hold
  uint32_t kid0, nkids;  // NOutOf: kids[kid0 .. kid0+nkids) in the kid array
};
enum : uint32_t { DP_REJECT = 0, DP_SIG = 1, DP_IMPLICIT = 2, DP_UNSUP = 3 };
struct DevPolicy {
  uint32_t kind;      // DP_*
  uint32_t decode_ok, compile_ok, needs_roles;
  int32_t root;       // DP_SIG: node index
  int32_t threshold;  // DP_IMPLICIT
  uint32_t sub0, nsub;  // DP_IMPLICIT: policy indices subs[sub0 .. sub0+nsub)
};
// chaincode table entry: namespace bytes, compiled EP, status (0 ok, 1 INVALID_CHAINCODE, 2
// outside the model), collections known, its collections [coll0, coll0+ncoll) in the coll table,
// key-level validation parameters in the state (its keys are resolved one by one)
#define BD_CC_WORDS 8
// collection table entry: name bytes, EP (-1: the chaincode EP); implicit table: mspid bytes, EP
#define BD_COLL_WORDS 3

struct DevChannel {  // device pointers + sizes (passed by value to the kernels)
  const uint8_t *name;
  uint32_t name_len;
  uint32_t nident;
  const DevIdent *idents;
  const uint8_t *ident_bytes;
  const uint32_t *ident_table;  // open addressing: ident index + 1 (0 empty)
  const uint64_t *ident_hash;   // hash of each ident (same order as idents)
  uint32_t ident_mask;
  uint32_t ncc;
  const uint32_t *cc;           // ncc x BD_CC_WORDS
  const uint32_t *colls;        // BD_COLL_WORDS per collection
  uint32_t nimpl;
  const uint32_t *impl;         // nimpl x BD_COLL_WORDS (implicit org collections by mspid)
  uint32_t nmsp;
  const uint32_t *msps;         // nmsp x (off, len): the channel's MSP ids
  const uint8_t *cc_bytes;      // names of all the tables above
  const DevPolicy *policies;
  const DevPNode *nodes;
  const uint32_t *kids;
  const uint32_t *subs;
  const DevPrin *prins;
  const int32_t *ident_ous;     // interned (OU, certifier) ids of the identities
  // committed key-level validation parameters: open addressing, 8 words per slot (hash lo, hash
  // hi, arena offset of ns || coll || key, the three lengths, policy index or -3, used); null when
  // the state holds none
  const uint32_t *kvp;
  const uint8_t *kvp_bytes;
  uint32_t kvp_mask;
  uint32_t force_host;          // policy indices beyond int16 (DevTx::pol): the host parser
  const uint8_t *committed;     // committed ledger txids: open-addressing table of 32-byte keys
  uint32_t committed_mask;      // (all-zero key == empty; a zero txid is kept in committed_zero)
  uint32_t committed_zero;
};

// identity-index hash (host builds the table with it, device probes with it): Mspid bytes,
// id_bytes length, and the last <= 96 bytes of id_bytes as little-endian 32-bit words (a
// certificate ends in its signature, so the tail tells identities apart; the device reads it
// with 25 word loads instead of a byte walk).  Not cryptographic: every hit is confirmed by an
// exact compare of both fields.
#if defined(__HIPCC__)
#define BD_HD __host__ __device__
#else
#define BD_HD
#endif
#define BD_HASH_TAIL 96u
BD_HD inline uint64_t bd_mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0xC2B2AE3D27D4EB4Full;
  return h ^ (h >> 29);
}
BD_HD inline uint64_t bd_ident_hash_msp(const uint8_t *msp, uint32_t ml, uint32_t il) {
  uint64_t h = bd_mix(0x243F6A8885A308D3ull, ((uint64_t)ml << 32) | il);
  uint64_t w = 0;
  uint32_t k = 0;
  for (uint32_t i = 0; i < ml; i++) {
    w |= (uint64_t)msp[i] << (8 * (k++));
    if (k == 8) { h = bd_mix(h, w); w = 0; k = 0; }
  }
  return bd_mix(h, w ^ 0xA5);
}
// key-level state key (ns, coll, key): host form (byte loads); blockdev.hip kl_hash is the
// word-load form of the same function
inline uint64_t bd_kl_word(const uint8_t *p, uint32_t n, uint32_t j) {
  uint32_t w = 0;
  for (uint32_t b = 0; b < 4 && 4 * j + b < n; b++) w |= (uint32_t)p[4 * j + b] << (8 * b);
  return w;
}
inline uint64_t bd_kl_hash(const uint8_t *ns, uint32_t nl, const uint8_t *coll, uint32_t cl, const uint8_t *key,
                           uint32_t kl) {
  uint64_t h = bd_mix(0x6A09E667F3BCC908ull, ((uint64_t)nl << 32) | cl);
  h = bd_mix(h, kl);
  for (uint32_t j = 0; 4 * j < nl; j++) h = bd_mix(h, bd_kl_word(ns, nl, j));
  for (uint32_t j = 0; 4 * j < cl; j++) h = bd_mix(h, bd_kl_word(coll, cl, j));
  for (uint32_t j = 0; 4 * j < kl; j++) h = bd_mix(h, bd_kl_word(key, kl, j));
  return h;
}
// host form (byte loads); blockdev.hip has the word-load form of the same function
inline uint64_t bd_ident_hash(const uint8_t *msp, uint32_t ml, const uint8_t *idb, uint32_t il) {
  uint64_t h = bd_ident_hash_msp(msp, ml, il);
  const uint32_t T = il < BD_HASH_TAIL ? il : BD_HASH_TAIL, s = il - T;
  for (uint32_t j = 0; 4 * j < T; j++) {
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4 && 4 * j + b < T; b++) w |= (uint32_t)idb[s + 4 * j + b] << (8 * b);
    h = bd_mix(h, w);
  }
  return bd_mix(h, 0x5A);
}
