/*
 * fgv.h -- C ABI of the MI355X block-validation engine for Hyperledger Fabric's
 * committer hot path (libfgv.so).  Plain pointers and sizes only; no exceptions or
 * aborts cross this boundary.  Every entry point returns 0 on success or a negative
 * FGV_E* code; on a negative return the caller (the Go shim) falls back
 * to its own CPU path for that batch -- it never halts the channel.
 *
 * Each entry point names the reference interface it replaces (paths under the
 * PM-Master/fabric tree; fabric-lib-go is vendored at vendor/github.com/hyperledger/).
 */
#ifndef FGV_H
#define FGV_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
#define FGV_OK 0
#define FGV_EINVAL (-1)   /* bad argument (null pointer, size overflow)        */
#define FGV_EDEVICE (-2)  /* HIP runtime / kernel failure                      */
#define FGV_ENOMEM (-3)   /* device or host allocation failed                  */
#define FGV_ECOMM (-4)    /* RCCL / torch.distributed exchange failed          */
#define FGV_ESTATE (-5)   /* call out of order (e.g. not initialised)         */
#define FGV_EUNSUPPORTED (-6) /* block holds something outside the engine's model
                                 (config tx, key-level/collection endorsement policy,
                                 channel-reference policy, NodeOU roles, ...): validate it
                                 with the reference code instead                         */

/* ------------------------------------------------- per-signature status bytes
 * Only FGV_SIG_VALID means "valid"; the reference maps every other outcome to an
 * error (msp/identities.go:190-196), so the shim maps 0 -> (true,nil), else invalid. */
#define FGV_SIG_VALID 0     /* ecdsa.Verify returned true                          */
#define FGV_SIG_FALSE 1     /* equation false or R at infinity                     */
#define FGV_SIG_DER 2       /* Go encoding/asn1 decode error, or r<=0 / s<=0       */
#define FGV_SIG_HIGH_S 3    /* s > n>>1 (bccsp/utils/ecdsa.go:82-89)              */
#define FGV_SIG_RANGE 4     /* r >= n or s >= n                                    */
#define FGV_SIG_BADKEY 5    /* public key is not a P-256 point                     */
#define FGV_SIG_EMPTY 6     /* empty signature or digest (bccsp/sw/impl.go:253-259) */

typedef struct fgv_ctx fgv_ctx;

typedef struct fgv_config {
  int device;            /* HIP device ordinal (one process per GPU)                 */
  uint32_t key_slots;    /* comb-table cache: keys verified by the fixed-base key comb (0 = 256;
                            64 MiB of HBM per slot, 17-bit windows).  A key without a slot is
                            verified by the variable-base kernels instead -- same results, ~9x
                            the device work per verify -- so a full cache never fails a batch    */
  uint32_t host_threads; /* host worker threads for parsing / policy fold (0 = min(24,
                            the process's CPU share: affinity mask, OMP_NUM_THREADS)) */
  uint32_t key_ids;      /* distinct P-256 keys the context holds at once (0 = 1M): registered
                            keys for good, BCCSP-path keys until the id space is flushed.  HBM:
                            9 B per id up front (key map, use count, on-curve bit) plus 61,440 B
                            per id in use (the variable-base multiples 1..15 * 2^(4 w) Q of every
                            4-bit window w), grown by doubling as ids are taken -- 1M ids in use is
                            ~61.5 GB of the 288 GB.  FGV_ENOMEM:
                            a single call naming more distinct keys than key_ids, or a device
                            that cannot hold the multiples of the ids in use                      */
} fgv_config;

/* Replaces factory.GetDefault() / sw.NewDefaultSecurityLevel* for the verify + hash
 * capabilities (fabric-lib-go bccsp/factory/factory.go:42, bccsp/sw/new.go:29-80).
 * Builds the fixed-base generator table on the device. */
int fgv_init(const fgv_config *cfg, fgv_ctx **out);
void fgv_destroy(fgv_ctx *ctx);
const char *fgv_strerror(int code);
/* kernel-time accounting of the last call (ms, HIP events around each kernel) */
int fgv_last_timing(fgv_ctx *ctx, double *sha_ms, double *prep_ms, double *point_ms,
                    double *keytab_ms);
/* k_vb_mul's device time in the last timed verify call (0 when no item ran on the variable-base
 * kernels): it runs on its own stream beside the hashes, so point_ms above does not hold it. */
int fgv_last_vb_timing(fgv_ctx *ctx, double *vb_mul_ms);
/* host-side wall time of the last block call: parse, job assembly, device pass (incl.
 * transfers), fold (ms) */
int fgv_last_host_timing(fgv_ctx *ctx, double *parse_ms, double *assemble_ms, double *device_ms,
                         double *fold_ms);
/* work of the last block call: SHA-256 messages, 64-byte compressions, ECDSA verifies */
int fgv_last_counts(fgv_ctx *ctx, uint64_t *sha_jobs, uint64_t *sha_blocks, uint64_t *verifies);
/* per-kernel device time of the last device-parse block call (ms; HIP events recorded on each
 * kernel's own stream): out[0] k_bd_sha_payload, [1] k_bd_parse, [2] k_bd_sha, [3] k_bd_ident +
 * k_bd_count, [4] k_bd_emit, [5] k_der + k_inv, [6] k_prep, [7] k_point28 (+ k_point hand-overs),
 * [8] k_bd_fold, [9] the batch (first kernel to last); out[10] = SHA-256 compressions of the
 * payload hashes (k_bd_sha_payload's work); out[11] = host ms the pipelined call spent enqueueing
 * the next batch's front half (its framing walk's join included).  n entries are written. */
int fgv_last_kernel_times(fgv_ctx *ctx, double *out, size_t n);
/* Running sums over the block calls since the last reset (fgv_validate_blocks[_pipelined],
 * fgv_validate_shard_dev[_pipelined]) of the per-call diagnostics above, so that a benchmark reads
 * them once after its timed loop: out[0] calls, [1..12] fgv_last_kernel_times out[0..11] (ms; [10]
 * the payload compressions), [13] payload compressions, [14] SHA-256 compressions, [15] verifies,
 * [16..18] fgv_last_timing sha / prep / point ms, [19..22] fgv_last_host_timing parse / assemble /
 * device / fold ms, [23] host ms from the end of the previous call to the call's first back-half
 * kernel (the caller's work between calls included), [24] host ms of the call after its final
 * wait.  reset != 0 zeroes them after the read. */
int fgv_stats_sums(fgv_ctx *ctx, double *out, size_t n, int reset);
// Diagnostics: verifies of the last call that the fast point kernel (radix 2^28, incomplete
// formulas) handed to the exact kernel because an exceptional addition occurred (P = +-Q).
// Zero for honest inputs; reads one counter back from the device.
int fgv_last_point_handovers(fgv_ctx *ctx, uint64_t *handovers);

/* ---------------------------------------------------------- BCCSP Hash / Verify */

/* SHA-256 over n messages (msg i = buf[off[i] .. off[i]+len[i])), out = n*32 bytes.
 * Replaces CSP.Hash(msg, &SHA256Opts{}) -- bccsp/sw/impl.go:177-194, sw/hash.go:29-33. */
int fgv_sha256_batch(fgv_ctx *ctx, const uint8_t *buf, size_t buf_len, const uint64_t *off,
                     const uint32_t *len, size_t n, uint8_t *out);

/* ECDSA-P256 verify of n (key, DER signature, digest) triples; status = n bytes.
 * keys: n*64 bytes (X||Y big-endian affine); digests: n*32 bytes.
 * Replaces CSP.Verify(k, sig, digest, nil) for *ecdsaPublicKey keys:
 * bccsp/sw/impl.go:247-270 -> sw/ecdsa.go:71-75 -> verifyECDSA sw/ecdsa.go:41-57
 * (utils.UnmarshalECDSASignature utils/ecdsa.go:41-65, IsLowS :82-89, ecdsa.Verify). */
int fgv_p256_verify_batch(fgv_ctx *ctx, const uint8_t *keys, const uint8_t *sig_buf,
                          size_t sig_buf_len, const uint64_t *sig_off, const uint32_t *sig_len,
                          const uint8_t *digests, size_t n, uint8_t *status);

/* Fused identity.Verify(msg, sig): digest = SHA-256(msg) on the device, then verify.
 * Replaces msp/identities.go:170-199 (getHashOpt SHA2 + bccsp.Hash + bccsp.Verify). */
/* identity.Verify(msg, sig) for P-384 keys (replaces bccsp sw verifyECDSA for the P-384 curve,
 * fabric-lib-go bccsp/sw/ecdsa.go:41-57 with the P-384 half order of bccsp/utils/ecdsa.go:26-31):
 * keys n x 96 bytes (X || Y big-endian), digest = SHA-256(msg), Go-rule DER, low S, then the
 * equation on the GPU (per-key comb tables built once per context).  Same status bytes as P-256
 * (5: the key is not a P-384 point).  The committer verifies P-384 creators and endorsers the same
 * way when their identities are registered with pubkey_p384. */
int fgv_p384_verify_msgs(fgv_ctx *ctx, const uint8_t *keys, const uint8_t *msg_buf, size_t msg_buf_len,
                         const uint64_t *msg_off, const uint32_t *msg_len, const uint8_t *sig_buf, size_t sig_buf_len,
                         const uint64_t *sig_off, const uint32_t *sig_len, size_t n, uint8_t *status);
int fgv_p256_verify_msgs(fgv_ctx *ctx, const uint8_t *keys, const uint8_t *msg_buf,
                         size_t msg_buf_len, const uint64_t *msg_off, const uint32_t *msg_len,
                         const uint8_t *sig_buf, size_t sig_buf_len, const uint64_t *sig_off,
                         const uint32_t *sig_len, size_t n, uint8_t *status);

/* ------------------------------------------- key registry + HBM-resident batches */

/* Register public keys (n*64 bytes X||Y) with the context and return their key ids (the "slots"
 * fgv_p256_verify_msgs_dev takes).  The analogue of the MSP identity cache (msp/cache/cache.go:
 * 65-83): identities are deserialized once, and every later verify is an id lookup.
 * Key tiers: a key registered here takes a comb-table slot (the fast fixed-base
 * comb, built once per key) while one is free; otherwise -- and for identities registered with
 * only a CLIENT role, whose keys sign rarely -- it is verified by the variable-base kernels from
 * its coordinates alone, and promoted to a comb slot once it has signed FGV_PROMOTE_USES (64)
 * verifies.  The comb cache filling up changes speed, never results; FGV_ENOMEM only when the
 * id space (fgv_config.key_ids) is exhausted. */
int fgv_keys_register(fgv_ctx *ctx, const uint8_t *keys, size_t n, uint32_t *slots);
/* The same with a per-key tier hint: hot[i] != 0 asks for a comb slot now (as fgv_keys_register),
 * 0 starts the key on the variable-base kernels until it has signed FGV_PROMOTE_USES verifies --
 * for keys that will sign rarely (a client population, a churn of one-off signers).  hot may be
 * NULL (all hot).  Results never depend on the tier. */
int fgv_keys_register_tiered(fgv_ctx *ctx, const uint8_t *keys, size_t n, const uint8_t *hot, uint32_t *slots);
int fgv_keys_reset(fgv_ctx *ctx);
/* Key-tier statistics: ids in use, ids with a comb table, ids on the variable-base kernels, keys
 * promoted to a comb since fgv_init, and verifies of the last call that ran on the variable-base
 * kernels (reads one counter back from the device). */
int fgv_key_stats(fgv_ctx *ctx, uint64_t *ids, uint64_t *comb, uint64_t *vb, uint64_t *promoted,
                  uint64_t *vb_verifies_last);

/* identity.Verify over a batch already resident in device memory: every pointer below is a
 * DEVICE pointer (e.g. hipMalloc or a torch tensor's data_ptr on this device).  Message and
 * signature arenas must be readable 64 bytes past their last byte.  Runs k_sha256, k_der,
 * k_prep, k_point on the context's stream and returns when d_status is final. */
int fgv_p256_verify_msgs_dev(fgv_ctx *ctx, const uint8_t *d_msg_buf, const uint64_t *d_msg_off,
                             const uint32_t *d_msg_len, const uint8_t *d_sig_buf,
                             const uint64_t *d_sig_off, const uint32_t *d_sig_len,
                             const uint32_t *d_key_slot, size_t n, uint8_t *d_status);

/* ------------------------------------------------------------ committer: whole blocks */

/* Channel model the block validator runs against (what the peer's channel resources give
 * the reference validator):
 *   fgv_channel_init      -- channel name (chdr.ChannelId of valid txs; validator.go:155-158)
 *   fgv_channel_config    -- the channel's common.Config (configtx.pb.go Config: sequence +
 *                            channel_group): channel policies for channel_config_policy_reference
 *                            endorsement policies (core/policy/application.go:139-159; SIGNATURE
 *                            and IMPLICIT_META, common/policies/implicitmeta.go:27-104), the MSPs
 *                            of the channel and their SignatureHashFamily, the application orgs
 *                            (implicit-collection policies, deployedcc_infoprovider.go:270-305)
 *   fgv_msp_declare       -- an MSP of the channel without a config (identities of a declared
 *                            MSP that were never registered -> FGV_EUNSUPPORTED, not "unknown")
 *   fgv_msp_register_identity -- one MSP identity keyed by its exact SerializedIdentity
 *                            (mspid, id_bytes) pair, as the Go shim's MSP cache deserializes it
 *                            (msp/mspmgrimpl.go:75-100, msp/cache/cache.go:65-83)
 *   fgv_chaincode_define2 -- ValidationInfo of a namespace (dispatcher.go:237-275): plugin name
 *                            and ApplicationPolicy bytes; an empty plugin or policy means
 *                            INVALID_CHAINCODE, a plugin other than "vscc" FGV_EUNSUPPORTED
 *   fgv_collection_define -- a collection of a chaincode definition and its endorsement policy
 *                            (StaticCollectionConfig.endorsement_policy; len 0 = none: the
 *                            chaincode EP applies).  A defined chaincode whose collections were
 *                            never declared (no call, no FGV_CC_COLLECTIONS_KNOWN) makes hashed
 *                            writes to it FGV_EUNSUPPORTED; with them known, an undefined
 *                            collection is an ENDORSEMENT_POLICY_FAILURE (v20.go:84-100)
 *   fgv_ledger_add_txids  -- txids already in the block store (TxIDExists, kv_ledger.go:496)
 *   fgv_kvmeta_set        -- key-level (state-based) endorsement: the VALIDATION_PARAMETER metadata
 *                            value of one committed key (GetStateMetadata / GetPrivateDataMetadataByHash,
 *                            statebased/vpmanagerimpl.go:316-341); coll NULL or "" = a public key, a
 *                            private key is given by its key hash; vp NULL / len 0 = none.  The vscc
 *                            of a written key with one evaluates it (validator_keylevel.go:38-85,
 *                            translated as builtin/v20/validation_logic.go:50-66) instead of the
 *                            collection / chaincode EP; an earlier tx of the block that validly
 *                            wrote the key's metadata fails it (vpmanagerimpl.go:199-233).
 *                            fgv_mvcc_validate_block's commit keeps this state current; a block the
 *                            reference commits needs the caller's updates.  Blocks with metadata
 *                            writes or writes to keys with a parameter run the host parser.
 * Blocks the reference cannot validate are FGV_EUNSUPPORTED: a tx whose dependency extraction
 * (validator_keylevel.go:184-222) fails before a later tx's vscc reads a written key (the
 * reference waits forever, vpmanagerimpl.go:300-303) or panics (Actions[0] of none, a nil
 * ChaincodeEndorsedAction) before a later tx's vscc runs.
 * Identities a transaction names that the engine cannot judge exactly -- a certificate of a
 * channel MSP neither registered nor resolvable by the MSP cache-miss path below, a P-384 key, a
 * SHA3 MSP, a role principal for an identity registered without role bits, an ORGANIZATION_UNIT
 * principal of its MSP for a valid identity registered without its OUs -- make the batch
 * FGV_EUNSUPPORTED (the reference decides).
 * Principals (SatisfiesPrincipal, msp/mspimpl.go:425-660, MSP v1.4.3): ROLE (role bits), IDENTITY
 * (the same Mspid + Id, and valid; a principal naming a certificate of a channel MSP that was never
 * registered is resolved by the MSP cache miss like a batch's identities), ORGANIZATION_UNIT
 * (same MSP, valid, an (OU, certifier) pair of the identity), ANONYMITY (NOMINAL: any identity)
 * and COMBINED (every principal it collects, in order). */
#define FGV_KEY_P256 1             /* verified on the GPU                                      */
#define FGV_KEY_P384 2             /* P-384: verified per item on the GPU when pubkey_p384 is given
                                      (committer signatures; all zero: outside the engine)      */
#define FGV_KEY_OTHER 3            /* RSA etc.: Verify fails                        */
#define FGV_KEY_UNDESERIALIZABLE 4 /* DeserializeIdentity fails (Ed25519 under Fabric 2.x, F4)  */
#define FGV_HASH_SHA2 0
#define FGV_HASH_SHA3 1
#define FGV_ROLES_UNKNOWN 0x80000000u /* roles: only MEMBER (= valid) is known                 */
typedef struct fgv_identity_info {
  uint32_t key_type;      /* FGV_KEY_*                                                        */
  uint32_t hash_family;   /* the MSP's SignatureHashFamily: FGV_HASH_SHA2 / FGV_HASH_SHA3      */
  uint32_t valid;         /* msp.Validate(id) == nil                                          */
  uint32_t roles;         /* bit r <=> msp.SatisfiesPrincipal(id, ROLE{its mspid, r}) == nil,
                             r = MSPRole_MSPRoleType (MEMBER 0, ADMIN 1, CLIENT 2, PEER 3,
                             ORDERER 4): NodeOU classification / admin list (mspimpl.go:331-376,
                             477-660); or FGV_ROLES_UNKNOWN                                    */
  uint8_t pubkey[64];     /* P-256 X || Y (FGV_KEY_P256)                                      */
  uint8_t id_digest[32];  /* identity Id: SHA-256 of the certificate (common/policies/policy.go:375) */
  uint8_t pubkey_p384[96]; /* P-384 X || Y big-endian (FGV_KEY_P384); all zero: key not given  */
} fgv_identity_info;
#define FGV_CC_COLLECTIONS_KNOWN 1u /* the definition's collections are all declared           */
#define FGV_CC_KEY_LEVEL_EP 2u      /* the state holds key-level endorsement (SBE) metadata for
                                       this namespace that was NOT given by fgv_kvmeta_set: its
                                       validation is FGV_EUNSUPPORTED                            */
int fgv_channel_init(fgv_ctx *ctx, const char *channel_name);
int fgv_channel_config(fgv_ctx *ctx, const uint8_t *config, size_t len);
int fgv_msp_declare(fgv_ctx *ctx, const char *mspid);
int fgv_msp_register_identity(fgv_ctx *ctx, const uint8_t *serialized, size_t len, const fgv_identity_info *info);
/* identity.GetOrganizationalUnits() of a registered identity (msp/identities.go:121-145): n pairs
 * (OrganizationalUnitIdentifier, CertifiersIdentifier) for ORGANIZATION_UNIT principals
 * (msp/mspimpl.go:566-596).  Registering the identity again forgets them; the MSP cache miss sets
 * them itself.  FGV_ESTATE: the identity is not registered. */
int fgv_msp_identity_ous(fgv_ctx *ctx, const uint8_t *serialized, size_t len, size_t n, const char *const *ou,
                         const size_t *ou_lens, const uint8_t *const *certifiers, const size_t *certifier_lens);
int fgv_chaincode_define2(fgv_ctx *ctx, const char *ns, const char *plugin, const uint8_t *policy, size_t len,
                          uint32_t flags);
int fgv_collection_define(fgv_ctx *ctx, const char *ns, const char *collection, const uint8_t *policy,
                          size_t len);
int fgv_ledger_add_txids(fgv_ctx *ctx, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                         size_t n);
int fgv_kvmeta_set(fgv_ctx *ctx, const char *ns, const char *coll, const uint8_t *key, size_t key_len,
                   const uint8_t *vp, size_t vp_len);
size_t fgv_kvmeta_count(fgv_ctx *ctx);
/* the parameter held for (ns, coll, key): *len = its size (0: none); copies min(*len, cap) bytes */
int fgv_kvmeta_get(fgv_ctx *ctx, const char *ns, const char *coll, const uint8_t *key, size_t key_len, uint8_t *buf,
                   size_t cap, size_t *len);
/* The MSP cache miss (msp/cache/cache.go:65-83 -> the channel MSP's DeserializeIdentity,
 * Validate and SatisfiesPrincipal; msp/mspimpl.go:398-422, identities.go:48-84,
 * mspimpl.go:892-938, mspimplvalidate.go): identities of a channel MSP (from fgv_channel_config's
 * FabricMSPConfig: root CAs, OU identifiers, NodeOUs, admins) that were never registered are
 * deserialized here -- PEM, X.509 parse, the chain to a root (the CA signatures verified on the
 * GPU, one pass per call), sanitizeCert's low-S re-marshal, Id = SHA-256 of it, Validate's SKI /
 * OU rules and the role bits -- and registered like fgv_msp_register_identity (one that fails
 * DeserializeIdentity is registered as FGV_KEY_UNDESERIALIZABLE).  Modelled MSPs: root and
 * intermediate CAs (P-256, each a CA with a SubjectKeyIdentifier, unique issuer names), no CRLs,
 * OU certificates that are CAs of the MSP, ECDSA P-256 / Ed25519 leaf keys.
 *   fgv_msp_resolve        -- n SerializedIdentity bytes -> status[i] FGV_RESOLVE_*
 *   fgv_msp_resolve_blocks -- every creator / endorser of the blocks the registry lacks;
 *                             *registered = identities added (NULL allowed)
 *   fgv_set_auto_resolve   -- the validate calls (fgv_validate_blocks*, fgv_validate_shard*,
 *                             fgv_group_validate_blocks, fgv_blocks_verify_signed) resolve a
 *                             batch's misses and run it once more instead of returning
 *                             FGV_EUNSUPPORTED for them; on by default
 *   fgv_msp_identity       -- the registry's record of one identity (FGV_ESTATE: none) */
#define FGV_RESOLVE_KNOWN 0       /* registered already, or not an identity of a channel MSP    */
#define FGV_RESOLVE_OK 1          /* deserialized and registered (valid or not: see Validate)   */
#define FGV_RESOLVE_FAILED 2      /* DeserializeIdentity fails: registered as undeserializable  */
#define FGV_RESOLVE_UNSUPPORTED 3 /* outside the modelled MSP / certificate shapes: left out     */
#define FGV_RESOLVE_REPEAT 4      /* the same bytes earlier in this call                        */
int fgv_msp_resolve(fgv_ctx *ctx, size_t n, const uint8_t *const *serialized, const size_t *lens, int *status);
int fgv_msp_resolve_blocks(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                           size_t *registered);
int fgv_set_auto_resolve(fgv_ctx *ctx, int on);
int fgv_msp_identity(fgv_ctx *ctx, const uint8_t *serialized, size_t len, fgv_identity_info *out);
/* Round-1 forms: fgv_msp_add_identity = register with FGV_KEY_P256 (pubkey64 != NULL) or
 * FGV_KEY_OTHER, SHA2, FGV_ROLES_UNKNOWN; fgv_chaincode_define = fgv_chaincode_define2 with
 * plugin "vscc", flags 0. */
int fgv_msp_add_identity(fgv_ctx *ctx, const uint8_t *serialized, size_t len, const uint8_t *pubkey64,
                         int valid, const uint8_t *id_digest32);
int fgv_chaincode_define(fgv_ctx *ctx, const char *ns, const uint8_t *policy, size_t len);

/* TxValidator.Validate (core/committer/txvalidator/v20/validator.go:180-265) for `nblocks`
 * consecutive blocks (marshalled common.Block).  Writes one TxValidationCode byte per
 * transaction (blocks concatenated) into `flags` -- the TRANSACTIONS_FILTER metadata -- and
 * the transaction count of each block into ntx[b].  Block b sees the txids of blocks < b as
 * committed.  d_blocks: optional device copies of the same bytes (each readable 64 bytes
 * past its end); NULL -> the library uploads them.  Returns FGV_EUNSUPPORTED when a block
 * needs logic outside the engine's model (the caller validates that batch itself). */
int fgv_validate_blocks(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                        const size_t *lens, const uint8_t *const *d_blocks, uint8_t *flags,
                        size_t flags_cap, size_t *ntx);
/* fgv_validate_blocks that also prepares the NEXT batch while this one runs on the GPU (the
 * single-GPU committer pipeline): its envelope framing is walked on a host worker and, when both
 * batches are host-resident, its bytes are copied to the device on the copy stream
 * (next_d_blocks: its device copy, or NULL).  The next batch's buffers must stay valid and
 * unchanged until its call.  Results never depend on it. */
int fgv_validate_blocks_pipelined(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                                  const size_t *lens, const uint8_t *const *d_blocks, uint8_t *flags,
                                  size_t flags_cap, size_t *ntx, size_t next_nblocks,
                                  const uint8_t *const *next_blocks, const size_t *next_lens,
                                  const uint8_t *const *next_d_blocks);

/* Per-block outcomes (off by default: a batch holding anything outside the engine's model returns
 * FGV_EUNSUPPORTED as a whole, and the caller validates every block of it with the reference).
 * On, fgv_validate_blocks[_pipelined] return FGV_OK for such a batch, and fgv_last_block_status
 * reports for each block of the last call:
 *   FGV_OK           -- its flags are final;
 *   FGV_EUNSUPPORTED -- it holds something outside the model (a CONFIG transaction, a P-384
 *                       identity registered without its key, a SHA3 identity, a certificate no
 *                       channel MSP can judge, ...): validate this block with the reference; its
 *                       flag bytes are 0xFD where the engine could not decide a transaction;
 *   FGV_BLOCK_LATER  -- not decided: an earlier block of the call may change the key-level
 *                       VALIDATION_PARAMETER of a key this block writes, and the reference commits
 *                       that block before this one reads it (statebased/vpmanagerimpl.go:296-355);
 *                       or an earlier block holds a CONFIG transaction that reaches its apply step
 *                       (a config update changes the channel's MSPs and policies for every later
 *                       block).  Every block from the first such one (n_final) on is LATER: commit
 *                       blocks [0, n_final) and call again with the rest.
 * Blocks after an unsupported one stay final: a block reads the earlier blocks' txids (every one,
 * whatever its code: checkTxIdDupsLedger, validator.go:460-481) and, through the rule above,
 * never their codes.  Single-GPU calls; the group call with fgv_group_set_block_outcomes; the
 * shard calls (fgv_validate_shard_dev[_pipelined]) of the one-process-per-GPU protocol: the
 * rank's records keep 0xFD for undecided transactions and fgv_last_block_status reports this
 * rank's n_final (its key-level walk sees its own transactions; another rank's block whose bytes
 * are not in the call waits behind a change) with LATER from there on -- the caller takes the
 * minimum n_final over the ranks and marks the blocks whose final flags hold 0xFD unsupported
 * (fabric_amd/shard.py block_outcomes).  After a call that failed (returned anything but FGV_OK),
 * fgv_last_block_status fills every status with that return code, sets n_final = 0 and returns
 * the code: a failed call decided no block.  fgv_unsupported_stats: fallback counters since fgv_init -- calls that
 * returned FGV_EUNSUPPORTED, blocks handed to the reference (whole batches included), undecided
 * transactions of per-block calls. */
#define FGV_BLOCK_LATER 1
int fgv_set_block_outcomes(fgv_ctx *ctx, int on);
int fgv_last_block_status(fgv_ctx *ctx, int32_t *status, size_t n, size_t *n_final);
int fgv_unsupported_stats(fgv_ctx *ctx, uint64_t *batches, uint64_t *blocks, uint64_t *txs);

/* ----------------------------------------------- multi-GPU committer (one process per GPU)
 * fgv_validate_blocks = fgv_validate_shard over every transaction + fgv_finalize_flags.
 * With G GPUs each rank validates transactions [tx_lo[b], tx_hi[b]) of every block b (the
 * north-star sharding by transaction index), the ranks all-gather their fgv_tx_result
 * records (RCCL over xGMI), and fgv_finalize_flags applies the two cross-transaction steps
 * of the reference: the block-store txid index of earlier blocks of the batch
 * (checkTxIdDupsLedger, validator.go:460-481, which precedes Dispatch) and
 * markTXIdDuplicates (validator.go:279-295). */
#define FGV_TXR_REACHED 1u  /* tx reached the ledger duplicate check; txid = hex-decoded TxId */
#define FGV_TXR_INDEXED 2u  /* index_txid = the 64-hex txid this tx adds to the block index  */
typedef struct fgv_tx_result {
  uint8_t code;  /* code decided by the tx alone (initial ledger txids applied)           */
  uint8_t flags;
  uint8_t pad[2];
  uint8_t txid[32];
  uint8_t index_txid[32];
} fgv_tx_result; /* 68 bytes */

/* Where transactions are parsed: 0 (default) = on the GPU from the HBM-resident blocks
 * (parse, identity resolution, job assembly and policy fold as kernels; a transaction whose
 * shape exceeds a device capacity -- more than 16 endorsements, 8 namespaces, ... -- sends
 * its batch through the host parser), 1 = host parser (C++ threads).  Same results. */
int fgv_set_parse_mode(fgv_ctx *ctx, int mode);

/* tx_lo[b] == FGV_SHARD_SKIP: block b belongs to another rank -- it is not parsed, adds no
 * records, and ntx[b] comes back 0 (the block-granular plan of fabric_amd/shard.py). */
#define FGV_SHARD_SKIP 0xFFFFFFFFu
int fgv_validate_shard(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                       const uint8_t *const *d_blocks, const uint32_t *tx_lo, const uint32_t *tx_hi,
                       fgv_tx_result *results, size_t results_cap, size_t *ntx);
/* pure host function: results of ALL transactions, blocks concatenated in order */
int fgv_finalize_flags(size_t nblocks, const size_t *ntx, const fgv_tx_result *results,
                       uint8_t *flags);

/* Device-resident variants for the multi-GPU protocol (records stay in HBM between the
 * shard validation, the RCCL all-gather and the finalize):
 *   fgv_validate_shard_dev -- as fgv_validate_shard, records written to device memory
 *     `d_results` (4-byte aligned, results_cap records) in shard order;
 *   fgv_finalize_flags_dev -- fgv_finalize_flags over the all-gathered device buffer
 *     `d_gathered` = world x rows_per_rank records, rank r's rows holding its shard
 *     [floor(ntx_b*r/world), floor(ntx_b*(r+1)/world)) of every block b in block order
 *     (the layout all_gather produces from the per-rank fgv_validate_shard_dev buffers).
 *     Runs as device kernels (open-addressing txid table in HBM); flags -> host memory.
 * Same results as fgv_validate_shard + fgv_finalize_flags (validator.go:279-295, 460-481). */
int fgv_validate_shard_dev(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                           const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                           const uint32_t *tx_hi, void *d_results, size_t results_cap, size_t *ntx);
/* Several GPUs from one process (a peer that drives all its GPUs through this ABI): one
 * context per device; fgv_group_ctx(g, i) is device i's context, which the caller sets up
 * like any other (channel model, identities, chaincodes, ledger txids: the same calls on every
 * context).  fgv_group_validate_blocks = fgv_validate_blocks over all devices: the blocks are
 * split into contiguous ranges of about equal bytes, one per device (each device stages, splits
 * and parses only its own) -- or, with fewer blocks than devices (one block), the batch's
 * transactions into contiguous index ranges -- the devices validate in parallel (fgv_validate_shard_dev), their
 * records are gathered onto the first device by peer copies (xGMI), and the first device runs
 * the batch's cross-transaction steps (fgv_finalize_flags_dev_plan).  Same flags as one GPU.
 * host_threads 0 in cfg: the process's CPU share divided among the devices. */
typedef struct fgv_group fgv_group;
int fgv_group_init(const int *devices, size_t ndev, const fgv_config *cfg, fgv_group **out);
void fgv_group_destroy(fgv_group *g);
size_t fgv_group_size(const fgv_group *g);
fgv_ctx *fgv_group_ctx(fgv_group *g, size_t i);
int fgv_group_validate_blocks(fgv_group *g, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                              uint8_t *flags, size_t flags_cap, size_t *ntx);
/* Per-block outcomes of the group call (fgv_set_block_outcomes / fgv_last_block_status for one
 * context, same statuses and rules): on, fgv_group_validate_blocks returns FGV_OK for a batch
 * holding transactions outside the model -- each device marks them 0xFD in its records instead of
 * failing its range, and their blocks come back FGV_EUNSUPPORTED -- and a block whose keys'
 * key-level parameters an earlier block may change comes back FGV_BLOCK_LATER with every block
 * after it (n_final), whether the earlier block is on the same device or on another one (a device
 * whose blocks change key-level state: the whole batch is checked on the host). */
int fgv_group_set_block_outcomes(fgv_group *g, int on);
/* How the group's records meet:
 *   FGV_GROUP_COLL_PEER (default) -- gathered onto the first device with peer copies over xGMI,
 *     finalized there (works with a device listed twice);
 *   FGV_GROUP_COLL_RCCL -- one RCCL communicator over the group's devices (ncclCommInitAll; the
 *     devices must be distinct): ncclAllGather of the 68 B records into every device's HBM, each
 *     on its own stream, then the finalize on every device (the north star's collective; every
 *     device holds the final flags, the caller gets the first device's and the others are checked
 *     equal).  RCCL is loaded at run time (dlopen, RTLD_LOCAL).  FGV_EDEVICE when it is absent or
 *     the communicator cannot be created; FGV_EINVAL for repeated devices. */
#define FGV_GROUP_COLL_PEER 0
#define FGV_GROUP_COLL_RCCL 1
int fgv_group_set_collective(fgv_group *g, int mode);
/* (after a failed group call: every status = its return code, n_final = 0, returns the code) */
int fgv_group_last_block_status(fgv_group *g, int32_t *status, size_t n, size_t *n_final);
/* fgv_p256_verify_msgs over all devices of the group (config C4 through the C ABI): items
 * [n r / W, n (r+1) / W) on device r, each device verifying with its own key cache; same status
 * bytes as one device.  The devices read only the message / signature byte spans their items
 * reference. */
int fgv_group_p256_verify_msgs(fgv_group *g, const uint8_t *keys, const uint8_t *msg_buf, size_t msg_buf_len,
                               const uint64_t *msg_off, const uint32_t *msg_len, const uint8_t *sig_buf,
                               size_t sig_buf_len, const uint64_t *sig_off, const uint32_t *sig_len, size_t n,
                               uint8_t *status);

/* Deliver-side pre-split (no reference counterpart: the Go committer re-walks each block
 * inside TxValidator.Validate, validator.go:180-265).  Starts walking the block data framing
 * (the envelope spans) of a batch on a background host thread and returns at once; the next
 * fgv_validate_shard_dev whose batch has the same block addresses, lengths and tx_lo/tx_hi
 * uses that split instead of walking the blocks itself -- a peer splits block k+1 while
 * block k validates.  The block buffers must stay unchanged until that call.  The two most
 * recent requests are kept (a peer walks batches k+2 and k+3 while batch k validates: the
 * pipelined call before batch k+2 then finds its walk done and queues that batch's parse at
 * its own top); a validation call uses the request of its batch and discards the requests made
 * before it (all pending ones when none matches), and a third request discards the oldest.
 * Results never depend on whether a pre-split was used.  fgv_last_presplit: 1 if the last
 * device-parse validation used one (diagnostic). */
int fgv_presplit(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                 const uint32_t *tx_lo, const uint32_t *tx_hi);
int fgv_last_presplit(fgv_ctx *ctx);
/* Queue the H2D copy of a LATER host-resident batch now, on the engine's copy stream (a peer
 * calls it as soon as a batch of delivered blocks sits in its pinned receive buffer).  The
 * validation call whose batch has the same block addresses and lengths -- or a pipelined call
 * naming it as its next batch -- waits for that copy instead of copying.  The engine keeps three
 * staging arenas: the running call's batch and two staged ones (a further fgv_prefetch drops the
 * oldest staged batch, which its call then copies itself).  With the pipelined calls, staging
 * batch k+2 during batch k keeps the PCIe link busy back to back.  The buffers must stay valid
 * and unchanged until that call (or fgv_destroy); they should be pinned (fgv_host_alloc).  Results
 * never depend on it. */
int fgv_prefetch(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens);
/* fgv_validate_shard_dev of the current batch that also pre-splits the NEXT batch (next_*,
 * same meaning as fgv_presplit's arguments) as soon as the current batch's GPU work is
 * queued, so the walk overlaps the current validation instead of following it.  When the
 * current batch is host-resident (d_blocks NULL) the next batch's bytes are also copied to the
 * device now, on the engine's copy stream into a second staging arena, overlapping this
 * batch's kernels; the next call with those blocks waits for that copy instead of copying.
 * The next batch's buffers must then stay valid and unchanged until that call (or
 * fgv_destroy); for the copy to run asynchronously they should be pinned (fgv_host_alloc). */
int fgv_validate_shard_dev_next(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                                const size_t *lens, const uint8_t *const *d_blocks,
                                const uint32_t *tx_lo, const uint32_t *tx_hi, void *d_results,
                                size_t results_cap, size_t *ntx, size_t next_nblocks,
                                const uint8_t *const *next_blocks, const size_t *next_lens,
                                const uint32_t *next_lo, const uint32_t *next_hi);
/* The committer pipeline: fgv_validate_shard_dev of the current batch that also enqueues the
 * NEXT batch's front half -- envelope split, head upload, payload and message SHA-256, parse,
 * identity resolution, job counts -- on the engine's side streams while the current batch's
 * back half (verify jobs, ECDSA, policy fold) runs, so two batches are in flight on the GPU.
 * The next call whose batch (host and device block addresses, lengths, tx_lo/tx_hi) is that
 * one continues from it; any other call discards it.  next_d_blocks: the next batch's device
 * copy (NULL: host-resident -- copied on the copy stream when the current batch is
 * host-resident too, as fgv_validate_shard_dev_next does; else only pre-split).  The next
 * batch's host and device buffers must stay valid and unchanged until that call.  Channel-model
 * changes in between (identities, chaincodes, config) discard it; ledger txids added in between
 * (fgv_ledger_add_txids) do not -- only k_bd_fold, in the back half, reads them.  Results never
 * depend on whether a front half was enqueued ahead (fgv_last_ahead: it was, for the last call). */
int fgv_validate_shard_dev_pipelined(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks,
                                     const size_t *lens, const uint8_t *const *d_blocks,
                                     const uint32_t *tx_lo, const uint32_t *tx_hi, void *d_results,
                                     size_t results_cap, size_t *ntx, size_t next_nblocks,
                                     const uint8_t *const *next_blocks, const size_t *next_lens,
                                     const uint8_t *const *next_d_blocks, const uint32_t *next_lo,
                                     const uint32_t *next_hi);
int fgv_last_ahead(fgv_ctx *ctx);
/* Where the next batch's front half is enqueued by the pipelined calls (fgv_validate_shard_dev_
 * pipelined, fgv_validate_blocks_pipelined) when its device copy is known: 2 = at once, beside the
 * current batch's back half (the default; the environment variable FGV_AHEAD sets the initial
 * value; C2 on MI355X: 0.715-0.724 ms per step against 0.773-0.799 not ahead);
 * 0 = not ahead: one batch on the GPU at a time, the next one pre-split on the host; 1 = once the
 * current batch's ECDSA kernels are done; 3 = once its policy fold is done; 4 = once its k_prep
 * is done (beside its k_point28).  Results never depend on it. */
int fgv_set_ahead(fgv_ctx *ctx, int mode);
/* Per-kernel device times of the block committer (fgv_last_kernel_times, fgv_last_timing): on,
 * every kernel of the back half is bracketed by timestamp events -- each a packet on the
 * critical path (~5 us on MI355X) -- off (default; the environment variable FGV_TIMING sets the
 * initial value), only the events that order the streams are recorded, which time the payload
 * hashes, the parse, the other hashes and the identity/count kernels.  Results never depend on it. */
int fgv_set_timing(fgv_ctx *ctx, int on);
/* Page-locked host memory for block buffers (hipHostMalloc): H2D copies from it run on the copy
 * engine at PCIe rate, asynchronously.  fgv_last_h2d: bytes the last validation call copied
 * itself, and blocks it found already copied by the previous call's prefetch. */
int fgv_host_alloc(fgv_ctx *ctx, size_t bytes, void **out);
int fgv_host_free(fgv_ctx *ctx, void *p);
/* HBM of the context's device for blocks a caller keeps resident (the d_blocks of the validation
 * calls) -- a peer without another GPU runtime (a Go peer through cgo) allocates and fills it
 * through the engine: fgv_dev_alloc (hipMalloc), fgv_dev_upload (a synchronous copy from host
 * memory at `dst`), fgv_dev_free (waits for the context's streams first). */
/* The context's next device work waits for everything queued so far on `stream` (a HIP stream
 * of the context's device, e.g. the caller's RCCL stream after the all-gather of the shard
 * records that fgv_finalize_flags_dev reads; NULL = the null stream) -- an event, no host
 * synchronisation. */
int fgv_stream_wait_external(fgv_ctx *ctx, void *stream);
int fgv_dev_alloc(fgv_ctx *ctx, size_t bytes, void **out);
int fgv_dev_upload(fgv_ctx *ctx, void *dst, const void *src, size_t bytes);
int fgv_dev_free(fgv_ctx *ctx, void *p);
int fgv_last_h2d(fgv_ctx *ctx, uint64_t *copied_bytes, uint64_t *prefetched_blocks);
int fgv_finalize_flags_dev(fgv_ctx *ctx, size_t nblocks, const size_t *ntx, uint32_t world,
                           size_t rows_per_rank, const void *d_gathered, uint8_t *flags);
/* Any shard plan: rank r's rows hold transactions [rank_lo[r*nblocks+b], rank_hi[r*nblocks+b])
 * of every block b in block order (FGV_SHARD_SKIP = none of block b); the ranks' ranges of a
 * block must tile [0, ntx[b]). */
int fgv_finalize_flags_dev_plan(fgv_ctx *ctx, size_t nblocks, const size_t *ntx, uint32_t world,
                                size_t rows_per_rank, const uint32_t *rank_lo, const uint32_t *rank_hi,
                                const void *d_gathered, uint8_t *flags);

/* ------------------------------------------------------------------------------ MVCC */

/* Committed-state cache on the GPU (statedb GetVersion, stateleveldb.go:128-137): an
 * open-addressing table of (namespace, key) -> version Height{blockNum, txNum}, exact key
 * compare.  It is a cache of the state DB, loaded from it at start (fgv_statedb_load) and
 * kept current by fgv_mvcc_validate_block(..., commit=1) -- or, for a block the caller
 * committed through the reference path (e.g. after FGV_EUNSUPPORTED), by fgv_statedb_apply
 * with that block's update batch (the puts and deletes lockbased_txmgr.go:168-202 commits);
 * the DB stays authoritative.  Private-data key hashes live under the state DB's own
 * hashed-data namespace ns + "$$h" + collection (privacyenabledstate/db.go:355-357), key = the
 * key hash bytes.
 *   slots: table capacity (rounded up to a power of two, load factor kept <= 0.7)
 *   arena_bytes: capacity for namespace + key bytes (8-byte aligned entries; <= 32 GiB, else
 *                FGV_EINVAL) */
int fgv_statedb_init(fgv_ctx *ctx, uint64_t slots, uint64_t arena_bytes);
/* Keys of one call must be distinct (FGV_EINVAL otherwise); a key already in the table gets the
 * new version.  Namespace and key lengths <= 65535 bytes (else FGV_EUNSUPPORTED). */
int fgv_statedb_load(fgv_ctx *ctx, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                     const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn, size_t n);
/* The update batch of a block committed outside the engine, one namespace per call (distinct
 * keys): is_delete[i] != 0 removes the key, else key i gets version (blk[i], txn[i]). */
int fgv_statedb_apply(fgv_ctx *ctx, const char *ns, const uint8_t *key_buf, const uint64_t *key_off,
                      const uint32_t *key_len, const uint64_t *blk, const uint64_t *txn,
                      const uint8_t *is_delete, size_t n);
/* occupied table slots (keys ever inserted, deleted ones included), arena bytes used, capacities */
int fgv_statedb_stats(fgv_ctx *ctx, uint64_t *keys, uint64_t *arena_used, uint64_t *slots,
                      uint64_t *arena_cap);

/* MVCC validation of one block (txmgmt/validation/batch_preparer.go:72-119 +
 * validator.go:81-200): `flags` holds the committer's TxValidationFlags (ntx bytes) and is
 * updated in place -- committer-invalid txs are skipped, others become NIL_TXACTION(16),
 * INVALID_OTHER_REASON(255), MVCC_READ_CONFLICT(11) or stay VALID.  commit != 0 then applies
 * the valid write sets to the state cache at Height{block_num, txIdx}.  d_block: optional
 * device copy of the block bytes.  Hashed (private-data) reads are checked like public reads
 * against ns + "$$h" + coll (validator.go:246-293); writes are deletes by IsKVWriteDelete /
 * IsKVWriteHashDelete (rwset_proto_util.go:366-375).  The rwsets are extracted, checked and
 * committed on the device: one upload of the envelope table and the flags, one read-back of
 * the codes.  A block with range queries or metadata writes takes the host path instead
 * (validator.go:205-244 phantom checks -> PHANTOM_READ_CONFLICT(12), with the raw-reads and
 * merkle-summary validators; tx_ops.go:17-53 metadata-only writes re-put an existing key at the
 * writer's height): the device classifies the transactions and answers committed-version
 * lookups and range scans of the state table, the host runs the block in order.  A key written
 * twice (or given two metadata writes) by one transaction (txOps adds the operation flags,
 * tx_ops.go:183-203) returns FGV_EUNSUPPORTED, as does what the reference halts or panics on: a
 * committer-valid envelope it cannot parse, a merkle summary with maxDegree < 2, a versionless
 * raw range read it compares, a metadata write to a key deleted earlier in the block.  Nothing
 * is committed then, nor on FGV_ENOMEM (table / arena full). */
int fgv_mvcc_validate_block(fgv_ctx *ctx, const uint8_t *block, size_t len, const uint8_t *d_block,
                            uint64_t block_num, uint8_t *flags, size_t ntx, int commit);
/* fgv_mvcc_validate_block that also walks the NEXT block's framing (next, next_len; the
 * buffer must stay unchanged until that block's call) on the engine's host worker while this
 * block validates; that call then starts from the walked envelope spans (fgv_presplit of one
 * block does the same from outside).  Results never depend on it. */
int fgv_mvcc_validate_block_next(fgv_ctx *ctx, const uint8_t *block, size_t len, const uint8_t *d_block,
                                 uint64_t block_num, uint8_t *flags, size_t ntx, int commit,
                                 const uint8_t *next, size_t next_len);
/* n consecutive blocks of one channel, validated and (commit != 0) committed in order: the result
 * is exactly that of one fgv_mvcc_validate_block call per block (each block reads the state the
 * blocks before it committed, as the reference's committer does: kv_ledger.go CommitLegacy ->
 * txmgr.ValidateAndPrepare -> Commit per block, one block at a time).  The engine enqueues the
 * blocks as one device chain with one wait: block k+1's rwset extraction runs while block k is
 * checked and committed.  A block the device cannot finish on its own (range queries, metadata
 * writes, a long conflict chain) and the blocks after it continue through the single-block path.
 * Stops at the first block whose call would fail and returns that error; *n_done (optional) =
 * the blocks whose flags are final (and committed).  d_blocks may be NULL or hold NULLs.
 * HBM held by the context after such calls (kept for the next ones): up to 16 buffer sets (block k
 * of a call uses set k % 16), each sized for the largest block that used it -- per block byte
 * ~55 B of records and slots, plus ~0.8 KB per transaction of extraction scratch and a staging
 * copy of the block when it is host-resident; the batch pass (runs of blocks <= 4,096 tx) holds
 * the same for a whole run; the update-batch arenas (fgv_mvcc_set_update_bytes) 2 x 1.25 x the
 * call's block bytes in HBM and in pinned host memory. */
int fgv_mvcc_validate_blocks(fgv_ctx *ctx, size_t n, const uint8_t *const *blocks, const size_t *lens,
                             const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                             const size_t *ntx, int commit, size_t *n_done);
/* fgv_mvcc_validate_blocks that also walks the NEXT batch's framing (next_blocks / next_lens,
 * n_next blocks; the buffers must stay unchanged until that batch's call) on the engine's host
 * worker while this batch's chain runs; that call then starts from the walked envelope spans.
 * Results never depend on it. */
int fgv_mvcc_validate_blocks_next(fgv_ctx *ctx, size_t n, const uint8_t *const *blocks, const size_t *lens,
                                  const uint8_t *const *d_blocks, const uint64_t *block_nums, uint8_t *const *flags,
                                  const size_t *ntx, int commit, size_t *n_done, size_t n_next,
                                  const uint8_t *const *next_blocks, const size_t *next_lens);
int fgv_mvcc_last_stats(fgv_ctx *ctx, double *lookup_ms, double *total_ms, uint64_t *reads,
                        uint64_t *writes, uint32_t *rounds);

/* ------------------------------------------------- deliver-side block integrity (a20, f3)
 * BlockVerificationAssistant.VerifyBlock (common/deliverclient/block_verification.go:243-273):
 * fgv_blocks_verify without, fgv_blocks_verify_signed with the orderer-signature policy.
 * verifyHeader (:311-331), verifyMetadata (:303-309),
 * VerifyTransactionsAreWellFormed (protoutil/blockutils.go:310-350), Header.DataHash ==
 * ComputeBlockDataHash (blockutils.go:76-79).  The chain state is the last verified header
 * (number + BlockHeaderHash, blockutils.go:48-67); only a verified block advances it, as in
 * the reference.  The data hash is one sequential SHA-256 chain per block: blocks hash in
 * parallel on the context's host threads (SHA extensions when the CPU has them). */
#define FGV_BLK_OK 0
#define FGV_BLK_UNPARSABLE 1   /* proto.Unmarshal of the common.Block failed              */
#define FGV_BLK_NO_HEADER 2    /* "header must be different from nil"                     */
#define FGV_BLK_NUMBER 3       /* number != last verified + 1                              */
#define FGV_BLK_PREV_HASH 4    /* PreviousHash != hash of the last verified header         */
#define FGV_BLK_METADATA 5     /* fewer than 5 metadata entries                            */
#define FGV_BLK_EMPTY 6        /* no transactions ("empty block")                         */
#define FGV_BLK_TX_MALFORMED 7 /* envelope bad_tx is not well formed                      */
#define FGV_BLK_DATA_HASH 8    /* Header.DataHash != SHA-256(concat(Data.Data))            */
#define FGV_BLK_SIGNATURES 9   /* the orderer signatures do not satisfy the policy, or the
                                  signatures metadata / a signature header does not unmarshal */
#define FGV_BLK_SIG_UNSUPPORTED 10 /* signature check outside the engine's model (this block and
                                  every later one of the call; the call returns FGV_EUNSUPPORTED) */
typedef struct fgv_chain_state {
  uint64_t number;          /* last verified block number                     */
  uint8_t header_hash[32];  /* its BlockHeaderHash                             */
  uint8_t valid;            /* 0: no previous block (number/prev-hash unchecked) */
  uint8_t has_hash;         /* 0: previous hash unknown (not compared)         */
  uint8_t pad[6];
} fgv_chain_state;
typedef struct fgv_block_check {
  int32_t status;           /* FGV_BLK_*                                       */
  uint32_t bad_tx;          /* FGV_BLK_TX_MALFORMED: index of the envelope     */
  uint64_t number;          /* Header.Number                                   */
  uint8_t data_hash[32];    /* ComputeBlockDataHash(block.Data)                */
  uint8_t header_hash[32];  /* BlockHeaderHash(block.Header)                   */
} fgv_block_check;
int fgv_blocks_verify(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                      fgv_chain_state *chain, fgv_block_check *out);
/* VerifyBlock with sigVerifierFunc (:265-268): after the data-hash check, the block's orderer
 * signatures -- protoutil.BlockSignatureVerifier (protoutil/blockutils.go:245-290): Metadata at
 * metadata[SIGNATURES], per MetadataSignature the SignedData{creator of its SignatureHeader,
 * md.Value || signature_header || BlockHeaderBytes(header), signature} -- must satisfy the
 * channel policy `policy` (NULL: "/Channel/Orderer/BlockValidation", the policy
 * deliverclient/verifier_assembler.go:32-56 takes) of the context's channel model
 * (fgv_channel_config + the orderer identities registered like any other).  Signatures are
 * verified on the GPU in one pass for the whole call.  bft != 0: the channel runs BFT; a
 * signature that names its consenter by an identifier header is outside the model.
 * An orderer identity never registered is resolved through its channel MSP first (the MSP cache
 * miss, fgv_msp_resolve).  Outside the model: no channel config, an identity of a channel MSP the
 * cache-miss path cannot judge, a P-384 / SHA3 orderer identity -> FGV_BLK_SIG_UNSUPPORTED from
 * that block on, FGV_EUNSUPPORTED. */
int fgv_blocks_verify_signed(fgv_ctx *ctx, size_t nblocks, const uint8_t *const *blocks, const size_t *lens,
                             fgv_chain_state *chain, const char *policy, int bft, fgv_block_check *out);
/* ------------------------------------------------------------------- ledger commit hash (a21)
 * kvLedger.addBlockCommitHash (core/ledger/kvledger/kv_ledger.go:806-817):
 *   out = SHA-256(varint(ntx) || flags || updateBatchBytes || prev)
 * flags: the block's final TRANSACTIONS_FILTER (after MVCC); updateBatchBytes =
 * deterministicBytesForPubAndHashUpdates (txmgr/update_batch_bytes.go:29-105) of the puts and
 * deletes of its VALID endorser transactions at Height{block_num, tx}; prev: the previous
 * block's commit hash (prev_len 0 for block 1).  Host function (no context, no GPU).
 * FGV_EUNSUPPORTED for metadata writes (the batch merges them with state-DB values) or a key
 * written twice by one transaction; FGV_EINVAL if a VALID transaction does not parse. */
int fgv_commit_hash(const uint8_t *block, size_t len, const uint8_t *flags, size_t ntx, uint64_t block_num,
                    const uint8_t *prev, size_t prev_len, uint8_t out[32]);

/* fgv_commit_hash of n consecutive blocks (block b chained to block b-1's hash, block 0 to
 * prev): the update batches and everything before the previous hash are hashed on a
 * persistent pool of min(16, hardware threads) host threads in parallel (threads = 1: on the
 * caller's thread only; other values: the pool), then the chain.
 * out: n x 32 bytes.  Same per-block result as fgv_commit_hash (kv_ledger.go:806-817). */
int fgv_commit_hashes(size_t n, const uint8_t *const *blocks, const size_t *lens, const uint8_t *const *flags,
                      const size_t *ntx, const uint64_t *block_nums, const uint8_t *prev, size_t prev_len,
                      uint8_t *out, unsigned threads);

/* The update-batch bytes on the device (round 6).  With fgv_mvcc_set_update_bytes(ctx, 1), every
 * committing fgv_mvcc_validate_block[s][_next] call also serialises each committed block's
 * updateBatchBytes on the GPU from its MVCC write records (fabric_amd/csrc/mvcc_ub.hip: the valid
 * writes gathered, grouped, sorted and framed as txmgr.Updates, update_batch_bytes.go:29-105), so
 * only the serial SHA-256 stays on the host; the MVCC call itself does not wait for them.
 * fgv_mvcc_last_ticket names the last such call; fgv_mvcc_update_bytes_acquire(ticket) (from any
 * thread: the peer's hashing goroutine) waits for them, copies them back on the first acquire of
 * the ticket, and gives block b's bytes (bytes[b] = NULL: not produced on the device -- a
 * block on the host phantom path, more than 8,192 valid writes, ...); they stay valid until
 * fgv_mvcc_update_bytes_release(ticket).  Two calls are kept: the second committing call after
 * `ticket` waits for its release.  Only blocks [0, n_done) of a call are committed.
 * fgv_commit_hashes_ub: fgv_commit_hashes with ub[b] (ub_lens[b] bytes) used as block b's update
 * batch where given (ub NULL or ub[b] NULL: block b is decoded from blocks[b] as before) -- the
 * same 32 bytes per block. */
int fgv_mvcc_set_update_bytes(fgv_ctx *ctx, int on);
int fgv_mvcc_last_ticket(fgv_ctx *ctx, uint64_t *ticket);
int fgv_mvcc_update_bytes_acquire(fgv_ctx *ctx, uint64_t ticket, size_t n, const uint8_t **bytes, size_t *lens);
int fgv_mvcc_update_bytes_release(fgv_ctx *ctx, uint64_t ticket);
int fgv_commit_hashes_ub(size_t n, const uint8_t *const *ub, const size_t *ub_lens, const uint8_t *const *blocks,
                         const size_t *lens, const uint8_t *const *flags, const size_t *ntx,
                         const uint64_t *block_nums, const uint8_t *prev, size_t prev_len, uint8_t *out,
                         unsigned threads);

/* host SHA-256 of one buffer (the data-hash primitive); returns 1 when the SHA extensions
 * were used, 0 for the portable path */
int fgv_sha256_host(const uint8_t *buf, size_t n, uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif /* FGV_H */
