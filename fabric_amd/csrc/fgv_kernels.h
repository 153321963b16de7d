// fgv_kernels.h -- shared layout constants and kernel declarations (device + host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Key comb (u2 * Q): 16 windows of 17 bits with signed digits in [-65536, 65535] (16 x 17 = 272 bits:
// the top window, bits 255..271 of a scalar < 2^256, absorbs the final carry); 65536 entries
// (|d| = 1..65536) per window, 64 MiB per key, one copy in Montgomery-280 form (k_point28; the exact
// k_point converts an entry with one multiplication), built by k_keytab (KT_CHUNK entries per thread).
// 17-bit windows (round 6): 28 comb terms per verify instead of 32 with 13-bit windows (5.2 MB per
// key), -12.5 % of k_point28's additions for 12.8x the table (HBM holds 256 hot keys in 16 GiB).
#define WBITS 17
#define NWIN 16
#define TAB_K 65536
#define KT_CHUNK 32
#define KT_THREADS_PER_KEY (NWIN * (TAB_K / KT_CHUNK))  // 32,768
#define KT_BUILD_KEYS 2                                  // keys per k_keytab launch (scratch bound: 256 MiB)
#define KT_ENTRIES (NWIN * TAB_K)           // 1,048,576 affine points per table
#define KT_BYTES ((size_t)KT_ENTRIES * 64)  // 67,108,864 bytes per table
// Generator comb (u1 * G): 12 windows of 22 bits with signed digits in [-2^21, 2^21 - 1] (12 x 22
// = 264 bits: the top window, bits 242..263 of a scalar < 2^256, absorbs the final carry);
// 2^21 entries per window, 1.61 GB, one copy in Montgomery-280 form (the exact k_point converts
// an entry with one multiplication), HBM resident, built once per context by k_gtab (one launch
// per window).  12 G terms instead of 16.5 with 16-bit windows.
#define GWBITS 22
#define NGWIN 12
#define GT_K 2097152
#define GT_ENTRIES ((size_t)NGWIN * GT_K)
#define GT_BYTES ((size_t)GT_ENTRIES * 64)
#define GT_CHUNK 32                            // consecutive entries per k_gtab thread
#define GT_THREADS_PER_WIN (GT_K / GT_CHUNK)   // 65,536 threads per k_gtab launch (one window)
#define NTERMS (NGWIN + NWIN)         // comb terms per verify: 12 G + 20 Q
#define DIG_Q_OFF 48                  // digit array item: G digits int32 x 12 at 0, Q digits int32 x 16 here
#define PREP_B 2                            // items per lane in the batched inversion
#define POINT_THREADS 256   // 4 waves per workgroup, 2 x n_cu workgroups: 2 waves per SIMD, <= 256 VGPRs
#define POINT_LANES_MAX 8    // lanes cooperating on one verify in k_point (partial sums + tree)
#define POINT_EXACT_WGS 64   // k_point's grid behind k_point28 (the hand-overs: exceptional additions only)
#define DIG_STRIDE 112       // bytes per item of the digit array (G digits, then Q digits at DIG_Q_OFF)
#define ST_PENDING 0xFF
#define ST_VB 0xFE       // k_inv: pending on the variable-base kernels (k_vb_mul / k_vb_fin finish it)
#define ST_P384 0xFD     // k_der: a P-384 key (KEY_P384_FLAG in its key slot): k_p384_verify finishes it
#define KEY_P384_FLAG 0x40000000u  // key slot of a P-384 identity: the flag | its index in the P-384 key table

struct apoint_raw {  // affine point, Montgomery limbs (64 B, 16-B aligned)
  uint32_t x[8];
  uint32_t y[8];
};
struct jpoint_raw {  // key-table build scratch: Jacobian point + prefix product
  uint32_t x[8];
  uint32_t y[8];
  uint32_t z[8];
  uint32_t pref[8];
};

__global__ void k_keybase(const uint32_t *qxy, uint32_t nkeys, jpoint_raw *bases);
__global__ void k_keytab(const uint32_t *qxy, const uint32_t *slots, apoint_raw *tables, apoint_raw *tables28,
                         jpoint_raw *scratch, uint8_t *key_ok, uint32_t nkeys, const jpoint_raw *bases);
// Key tiers.  Every key has an id; kmap[id] is its comb slot (the 64 MiB table
// above) or KEY_NONE: the variable-base kernels verify it from a 60 KB per-key table
// (vbt[id][w][d-1] = d * 2^(4 w) Q, w < 64, d = 1..15, affine Montgomery-280: every 4-bit window
// of u2 has its own base, so u2 * Q is additions only -- no doublings).  k_keyprep checks
// new keys (on the curve) and writes vbt / key_ok; k_kmap_set points ids at their freshly built
// comb tables (after k_keytab).
#define KEY_NONE 0xFFFFFFFFu
#define VB_THREADS 256      // k_vb_mul workgroup (grid 2 x n_cu)
#define VB_LANES 8          // k_vb_mul lanes per item (32-bit slices of u2)
#define VB_WINS 64          // per-key table windows: W_w = 2^(4 w) Q, one per 4-bit window of u2 (round 6)
#define VB_TAB 15           // per window: 1 .. 15 times its base
#define VBT_WORDS (VB_WINS * VB_TAB * 16)  // per key id: 960 affine points, 61,440 B
#define VB_ACC_WORDS 24     // k_vb_mul -> k_vb_fin partial result: x, y, z (Montgomery-256)
// counters in the context's redo words: [0] k_point28 hand-overs, [1] k_point28 chunks, [2] k_point
// chunks, [3] items k_inv listed for the variable-base kernels, [4] taken by k_vb_mul, [5] taken
// by k_vb_fin, [6] finished k_vb_fin workgroups (the last one zeroes [3..6] for the next batch)
#define RD_VB_CNT 3
#define RD_VB_MUL 4
#define RD_VB_FIN 5
#define RD_VB_DONE 6
#define RD_VB2_CNT 9    // k_vb_mul28's hand-over list: items for the exact k_vb_mul
#define RD_VB2_MUL 10   // the exact hand-over pass's work counter
#define VB_HAND_WGS 16  // the exact hand-over pass's grid (empty for honest inputs)
#define RD_FIN_DONE 8     // finished k_fin_dups workgroups (the last one copies the counters out)
#define VB_FIN_WGS 32        // k_vb_fin workgroups (256 threads)
#define VB_BACKLOG_CAP 65536u  // host: promotion ids kept while the comb cache is full
#define VB_PROMO_CAP 1022   // promotion queue: [0] count, [1] the last batch's variable-base items,
                            // then ids whose use count reached the threshold
__global__ void k_keyprep(const uint32_t *qxy, const uint32_t *ids, uint32_t nkeys, uint32_t *vbt, uint8_t *key_ok);
__global__ void k_kmap_set(const uint32_t *ids, const uint32_t *slots, uint32_t n, uint32_t *kmap);
__global__ void k_vb_mul(uint32_t n, const uint32_t *key_slot, const uint32_t *vbt, const uint32_t *r_limbs,
                         const uint32_t *w_in, const uint32_t *ctr, uint32_t *take, const uint32_t *list, uint32_t *acc,
                         uint32_t *uses, uint32_t promote, uint32_t *promo, const uint32_t *remap);
__global__ void k_vb_mul_o4(uint32_t n, const uint32_t *key_slot, const uint32_t *vbt, const uint32_t *r_limbs,
                            const uint32_t *w_in, const uint32_t *ctr, uint32_t *take, const uint32_t *list,
                            uint32_t *acc, uint32_t *uses, uint32_t promote, uint32_t *promo, const uint32_t *remap);
__global__ void k_vb_mul28(uint32_t n, const uint32_t *key_slot, const uint32_t *vbt, const uint32_t *r_limbs,
                           const uint32_t *w_in, uint32_t *ctr, const uint32_t *list, uint32_t *acc, uint32_t *uses,
                           uint32_t promote, uint32_t *promo, uint32_t *hand);
// the same with 16 lanes per item (16-bit slices: half the doublings per lane; small batches)
__global__ void k_vb_mul28_16(uint32_t n, const uint32_t *key_slot, const uint32_t *vbt, const uint32_t *r_limbs,
                           const uint32_t *w_in, uint32_t *ctr, const uint32_t *list, uint32_t *acc, uint32_t *uses,
                           uint32_t promote, uint32_t *promo, uint32_t *hand);
__global__ void k_vb_fin(uint32_t n, uint8_t *status, const apoint_raw *gtab28, const int8_t *digits,
                         const uint32_t *r_limbs, uint32_t *ctr, const uint32_t *list, const uint32_t *acc);
__global__ void k_gtab(apoint_raw *tables28, jpoint_raw *scratch, uint32_t w);
// kmap (nullable: every key has a comb): items of keys without one go to vb_list (count at
// vb_cnt, one atomic per wave) for k_vb_mul / k_vb_fin
__global__ void k_inv(uint32_t n, const uint32_t *dn, uint8_t *status, const uint32_t *key_slot, const uint8_t *key_ok,
                      const uint32_t *r_limbs, const uint32_t *s_limbs, uint32_t *w_out, uint32_t *w_scratch,
                      const uint32_t *kmap, uint32_t *vb_list, uint32_t *vb_cnt);
__global__ void k_prep(uint32_t n, const uint32_t *dn, const uint8_t *status, const uint32_t *r_limbs, const uint32_t *w_in,
                       const uint8_t *digests, const uint32_t *dig_idx, int8_t *digits, uint32_t *redo);
__global__ void k_point(uint32_t n, const uint32_t *dn, uint32_t lanes_per_item, uint8_t *status, const uint32_t *key_slot, const apoint_raw *gtab,
                        const apoint_raw *ktab, const int8_t *digits, const uint32_t *r_limbs, uint32_t *redo,
                        const uint32_t *kmap);
__global__ void k_point28(uint32_t n, const uint32_t *dn, uint32_t lanes_per_item, uint8_t *status, const uint32_t *key_slot,
                          const apoint_raw *gtab28, const apoint_raw *ktab28, const int8_t *digits,
                          const uint32_t *r_limbs, uint32_t *redo, const uint32_t *kmap);
#define INV_THREADS 128
struct ShaJob {  // message = span0 || span1 || span2 (absolute device addresses)
  uint64_t p[3];
  uint32_t n[3];
  uint32_t pad;   // SHAJOB_SHA3: SHA3-256 instead (an identity of a SHA3 MSP, identities.go:219-227)
};
#define SHAJOB_SHA3 1u
__global__ void k_sha256_jobs(const ShaJob *jobs, uint32_t n, uint8_t *out);
__global__ void k_sha256(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint32_t n,
                         uint8_t *out);
// Verify stages: n is the batch capacity (the column stride of r / s / w); dn (optional) points
// to the item count in device memory, written by an earlier kernel on the stream (the block
// committer's job counts), so the stages are enqueued without the host knowing it.
// key_slot (optional): a slot with KEY_P384_FLAG marks a P-384 identity's signature -> ST_P384
__global__ void k_der(const uint8_t *sig_buf, const uint64_t *off, const uint32_t *len, uint32_t n,
                      const uint32_t *dn, uint8_t *status, uint32_t *r_limbs, uint32_t *s_limbs,
                      const uint32_t *key_slot);
// P-384 (p384.hip): the committer's P-384 identities, verified per item beside the P-256 chain
#define P384_WIN 48                                   // 8-bit windows of a scalar < 2^384
#define P384_TK 255                                   // entries d = 1..255 per window
#define P384_ENTRIES ((size_t)P384_WIN * P384_TK)     // 12,240 affine points per comb table
#define P384_ENTRY_WORDS 24                           // x || y, Montgomery, 12 limbs each
#define P384_LANES 4                                  // lanes per verify (windows split across them)
__global__ void k_p384_verify(uint32_t n, const uint32_t *dn, uint8_t *status, const uint64_t *sigp,
                              const uint32_t *sigl, const uint32_t *slot, const uint32_t *dig_idx,
                              const uint8_t *digests, const uint32_t *gtab, const uint32_t *ktab,
                              const uint8_t *key_ok, uint32_t nkeys);

// ---- MVCC (mvcc.hip)
#define MV_NIL 16       // NIL_TXACTION
#define MV_OTHER 255    // INVALID_OTHER_REASON
#define MV_UNSUP 0xFD   // outside the engine's model
#define MV_SKIP 0xFF    // committer-invalid: not validated
#define MVR_HASVER 1u   // read: has a version
#define MVR_DELETE 1u   // write: is a delete
#define MVR_HASHED 2u   // private-data key: namespace = ns + "$$h" + coll
#define MV_HOSTPATH 2u  // MvCounters.unsup bit: range queries / metadata writes -> the host path
#define MV_HALT 4u      // MvCounters.unsup bit: an earlier block of the batch was not finished on the device
#define MV_OVF 8u       // MvCounters.unsup bit: batch pass, a key with more than MB_WR writers (per-block chain)
#define MVRANGE_UNBOUNDED 1u  // MvRange.flags: end key "" (to the end of the namespace)
#define MV_TAG_OCC 1ull      // tag bit 0: slot occupied (tags are never 0)
#define MV_TAG_PRESENT 2ull  // committed-state tag bit 1: the key exists (clear = deleted)
struct MvRec {  // one read or write: spans into the block (or a host-supplied key arena)
  uint64_t tag;
  uint64_t blk, txn;  // reads: version (load/apply records: the version to store)
  uint32_t tx;
  uint32_t key_off, ns_off, coll_off;
  uint16_t key_len, ns_len, coll_len, flags;
};
static_assert(sizeof(MvRec) == 48, "MvRec: 3 x 16 B (k_mvx_extract copies it as uint4)");
struct MvTxInfo {  // per transaction
  uint32_t rbeg, rcnt, wbeg, wcnt;  // record ranges
  uint32_t rws_off, rws_len;        // TxReadWriteSet span in the block
  uint8_t code, pad[7];             // 0 participates; MV_NIL / MV_OTHER / MV_UNSUP / MV_SKIP
};
struct MvCounters {  // device-side counters of one block (zeroed by the head copy)
  unsigned long long wbytes;  // arena bytes the block's writes could need
  uint32_t nr, nw;            // records
  uint32_t unsup, done, rounds, nomem;
  uint32_t undec[4];          // undecided txs after round r (slot r & 3)
  uint32_t pad[2];
};
#define MV_INLINE 32  // flattened ns || key bytes a committed-state slot holds inline
struct __attribute__((aligned(64))) StateSlot {  // committed state: open addressing, one 64 B line;
  uint64_t tag;     // 0 = empty; bit 1 = present        the arena holds every flattened ns || key,
  uint64_t blk, txn;                                  // the slot a copy of a short one (ns_len +
  uint32_t off8;    // arena offset / 8 (arena up to 32 GiB)   key_len <= MV_INLINE), so a probe of
  uint16_t ns_len, key_len;                           // a short key reads this line only
  uint8_t ik[MV_INLINE];
};
static_assert(sizeof(StateSlot) == 64, "StateSlot: one 64 B line");
struct BlkSlot {    // keys written in the block
  uint64_t owner;   // (block epoch << 32) | (write index + 1); an older epoch = free
  // fixpoint first writers, double buffered by round parity: (global round << 32) |
  // (0xFFFFFFFF - tx) by atomicMax, so a value left by an earlier round reads as "none"
  uint64_t fw_cand[2], fw_valid[2];
  uint64_t last;    // (epoch << 32) | (tx + 1) of the last VALID writer
};
#define MB_WR 8  // batch pass: writers of one key a slot lists
struct __attribute__((aligned(64))) MbSlot {  // keys written in a batch of consecutive blocks
  uint64_t owner;   // (batch epoch << 32) | (write index + 1); an older epoch = free
  uint64_t last;    // (epoch << 32) | (global tx + 1) of the last VALID writer
  uint32_t nwr;     // writers listed (reset by the slot's claimer)
  uint32_t wr[MB_WR];  // their write-record indices, in no particular order
};
__global__ void k_mvb_prep(const uint8_t *base, const MvRec *reads, const MvRec *writes, MbSlot *btbl, uint32_t epoch,
                           uint32_t *wslot, const StateSlot *tbl, uint64_t mask, const uint8_t *arena, uint8_t *rstat,
                           MvCounters *c);
__global__ void k_mvb_find(uint32_t ntx, const uint8_t *base, const MvRec *reads, const MvRec *writes, MbSlot *btbl,
                           uint32_t epoch, const uint32_t *wslot, uint32_t *rslot, const MvTxInfo *info, uint8_t *st,
                           MvCounters *c);
__global__ void k_mvb_round(uint32_t ntx, uint32_t r, const MvTxInfo *info, const MvRec *reads, const MvRec *writes,
                            const uint32_t *rslot, const uint8_t *rstat, const MbSlot *btbl, uint8_t *st,
                            const uint32_t *bfirst, const uint64_t *bnums, uint32_t nb, MvCounters *c);
__global__ void k_mvb_last(uint32_t rlast, const MvRec *writes, const uint32_t *wslot, const uint8_t *st, MbSlot *btbl,
                           uint32_t epoch, MvCounters *c, const unsigned long long *top, uint64_t slots_cap,
                           uint64_t arena_cap);
__global__ void k_mvb_upsert_find(uint32_t rlast, const uint8_t *base, const MvRec *recs, const uint32_t *wslot,
                                  const uint8_t *st, const MbSlot *btbl, uint32_t epoch, StateSlot *tbl, uint64_t mask,
                                  const uint8_t *arena, const uint32_t *bfirst, const uint64_t *bnums, uint32_t nb,
                                  uint8_t *pend, const MvCounters *c);
void mvx_extract_launch(uint32_t tpw, hipStream_t st, uint32_t ntx, const uint8_t *base, const uint32_t *envtab,
                        const uint8_t *in_flags, MvTxInfo *info, MvRec *reads, MvRec *writes, MvCounters *c,
                        uint32_t touch, MvRec *scr, uint8_t *bad);
#define MVX_SCR 8    // k_mvx_extract scratch: records of each kind per tx
bool mvx_lds_scratch();  // the scratch is in LDS (FGV_MVX_LDSSCR=1, default): no global scratch bytes

__global__ void k_mvx_prep(const uint8_t *base, const MvRec *reads, const MvRec *writes, BlkSlot *btbl, uint32_t epoch,
                           uint32_t *wslot, const StateSlot *tbl, uint64_t mask, const uint8_t *arena, uint8_t *bad,
                           MvCounters *c, const MvCounters *prev);
__global__ void k_mvx_find(uint32_t ntx, const uint8_t *base, const MvRec *reads, const MvRec *writes,
                           const BlkSlot *btbl_r, BlkSlot *btbl, uint32_t epoch, const uint32_t *wslot, uint32_t *rslot,
                           const MvTxInfo *info, const uint8_t *bad, uint8_t *st, uint32_t rg1, const MvCounters *c);
__global__ void k_mvx_round(uint32_t ntx, uint32_t r, uint32_t rg, const MvTxInfo *info, const uint32_t *rslot,
                            const uint32_t *wslot, BlkSlot *btbl, uint8_t *st, MvCounters *c);
__global__ void k_mvx_flags(uint32_t ntx, uint32_t rlast, const uint8_t *in_flags, const MvTxInfo *info,
                            const uint8_t *st, uint8_t *out, MvCounters *c);
__global__ void k_mv_last(uint32_t rlast, const MvRec *writes, const uint32_t *wslot, const uint8_t *st, BlkSlot *btbl,
                          uint32_t epoch, MvCounters *c, const unsigned long long *top, uint64_t slots_cap,
                          uint64_t arena_cap);
__global__ void k_mv_upsert_find(uint32_t mode, uint32_t rlast, uint32_t n_host, const uint8_t *base, const MvRec *recs,
                                 const uint32_t *wslot, const uint8_t *st, const BlkSlot *btbl, uint32_t epoch,
                                 StateSlot *tbl, uint64_t mask, const uint8_t *arena, uint64_t block_num, uint8_t *pend,
                                 const MvCounters *c);
__global__ void k_mv_upsert_insert(uint32_t mode, uint32_t rlast, uint32_t n_host, const uint8_t *base,
                                   const MvRec *recs, const uint8_t *pend, StateSlot *tbl, uint64_t mask, uint8_t *arena,
                                   unsigned long long *top, uint64_t block_num, const MvCounters *c,
                                   const uint32_t *bfirst, const uint64_t *bnums, uint32_t nb);
__global__ void k_mv_tags(const uint8_t *base, MvRec *recs, uint32_t n);
__global__ void k_mv_tail(const MvCounters *c, const unsigned long long *top, uint32_t *hc, unsigned long long *htop);
// mvcc_ub.hip -- a committed block's update-batch bytes (the commit hash's input) on the device.
// Block write records carry their value span in blk (offset from the base) and txn (length)
// until the batch pass's commit stores versions there (k_mvb_upsert_find runs after k_ub_block).
#define UB_OK 0u
#define UB_NONE 1u  // not produced on the device (too many writes / groups, arena full, not decided)
#define UB_MAX 8192u  // valid writes of one block the device serialisation sorts (LDS)
struct UbMeta {  // per block of the call, pinned host memory (written by k_ub_sort)
  uint64_t off;  // in the call's arena
  uint32_t len, status;
};
struct UbBlk {  // per block of one launch, device memory: k_ub_sort -> k_ub_write
  uint64_t off;
  uint32_t len, nent, t0;
  uint64_t num;
};
#define UBE_LIVE 1u  // UbEnt.flags: a surviving write (the last of its key)
#define UBE_NS 2u    // carries the namespace field (first write of a namespace)
#define UBE_COLL 4u  // carries the collection field (first write of a collection)
struct UbEnt {   // one sorted position of a block: the record, its offset in the block's bytes
  uint32_t rec, off, flags;
};
void ub_block_launch(hipStream_t s, uint32_t nb, const uint8_t *base, const MvRec *writes, const MvTxInfo *info,
                     const uint8_t *st, const MvCounters *c, uint32_t rlast, const uint32_t *bfirst,
                     const uint64_t *bnums, uint32_t ntx0, uint64_t num0, uint8_t *out, uint64_t out_cap,
                     unsigned long long *used, UbMeta *meta, UbBlk *dmeta, UbEnt *ents);
struct MvRange {  // a range query's scan bounds (bytes in a host-built buffer)
  uint32_t ns_off, ns_len, s_off, s_len, e_off, e_len, flags, pad;
};
__global__ void k_mv_lookup(uint32_t n, const uint8_t *base, const MvRec *recs, const StateSlot *tbl, uint64_t mask,
                            const uint8_t *arena, uint64_t *ver, uint8_t *present);
__global__ void k_mv_range_scan(uint64_t cap, const StateSlot *tbl, const uint8_t *arena, uint32_t nranges,
                                const MvRange *ranges, const uint8_t *rbytes, uint8_t *out, uint64_t out_cap,
                                unsigned long long *used);

struct DevTx;
// finalize.hip -- batch txid index + markTXIdDuplicates over gathered fgv_tx_result records
__global__ void k_fin_rows(uint32_t P, const uint64_t *blk_start, uint32_t nb, uint32_t W, uint32_t rows,
                           const uint32_t *roff, const uint32_t *rlo, const uint32_t *rcnt, uint32_t *rowmap,
                           uint32_t *blkof, uint32_t cap, uint32_t *owner, int32_t *minblk, uint32_t *minvalid,
                           const DevTx *txs, const uint64_t *bases, const uint8_t *digests, uint8_t *keys,
                           uint32_t prio);
__global__ void k_fin_index(uint32_t P, const uint8_t *recs, const uint32_t *rowmap, const uint32_t *blkof,
                            uint32_t *owner, int32_t *minblk, uint32_t mask, uint64_t seed);
__global__ void k_fin_codes(uint32_t P, const uint8_t *recs, const uint32_t *rowmap, const uint32_t *blkof,
                            const uint32_t *owner, const int32_t *minblk, uint32_t *minvalid, uint32_t mask,
                            uint64_t seed, uint8_t *flags, uint32_t *pslot, const uint8_t *keys);
__global__ void k_fin_index_dev(uint32_t P, const DevTx *txs, const uint64_t *bases, const uint8_t *digests,
                                uint8_t *keys, uint32_t *owner, int32_t *minblk, uint32_t mask, uint64_t seed, uint32_t prio);
__global__ void k_fin_dups(uint32_t P, const uint32_t *pslot, const uint32_t *minvalid, uint8_t *flags, uint32_t *unsup,
                           uint8_t *out, const uint32_t *misc_src, uint32_t *misc_out, uint32_t *done);
