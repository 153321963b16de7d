// finalize.hip -- the cross-transaction steps of TxValidator.Validate on the device, over the
// all-gathered fgv_tx_result records of a block batch (libfgv.so):
//   * checkTxIdDupsLedger against the txid index of EARLIER blocks of the batch
//     (core/committer/txvalidator/v20/validator.go:460-481; it precedes Dispatch, so it
//     applies to every tx that reached it -- FGV_TXR_REACHED);
//   * markTXIdDuplicates (validator.go:279-295): among the VALID txs of a block, every
//     occurrence of a txid after the first becomes DUPLICATE_TXID (9).
// Layout: `recs` holds W ranks x `rows` padded records, rank r's rows = its shard
// [lo_rb, hi_rb) of every block b in block order, lo_rb = floor(ntx_b * r / W)
// (fabric_amd/shard.py).  Global position p enumerates transactions block-major.
//
// One open-addressing table keyed by the 32-byte txid (key bytes are never copied: a slot
// names its owner position, whose record holds the key).  Per slot: min block that indexes
// the txid, min position of a VALID tx carrying it.  Hash seeded per context.
//   k_fin_rows   p -> gathered row, block
//   k_fin_index  INDEXED txs: insert index_txid, atomicMin(min block)
//   k_fin_codes  REACHED txs: ledger-dup if min block < own block; VALID: atomicMin(position)
//   k_fin_dups   VALID txs whose txid has an earlier VALID position -> 9
// Every kernel is one lane per transaction, HBM/L2-latency bound (~70 B read per tx).
// Precondition (guaranteed by fgv_validate_shard[_dev], whose records these are): a VALID
// record is REACHED, and a REACHED record is INDEXED with index_txid == txid (its chdr.TxId
// equals hex(SHA-256(nonce||creator)), and that string is the index entry).
#include <hip/hip_runtime.h>

#include "../../include/fgv.h"
#include "blockdev.h"
#include "fin_dev.h"
#include "fgv_kernels.h"

namespace {

constexpr uint32_t REC = 68;
constexpr uint32_t OFF_TXID = 4, OFF_INDEX = 36;

__device__ inline void load_key(const uint8_t *recs, uint32_t row, uint32_t off, uint32_t k[8]) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(recs + (size_t)row * REC + off);
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = q[i];
}

// the owner's index key: its record's index_txid, or (keys != null) its entry of the early
// index's key array (k_fin_index_dev), indexed by position
__device__ inline bool key_eq(const uint32_t a[8], const uint8_t *recs, uint32_t row, const uint8_t *keys = nullptr,
                              uint32_t pos = 0) {
  const uint32_t *q = keys ? reinterpret_cast<const uint32_t *>(keys + (size_t)pos * 32)
                           : reinterpret_cast<const uint32_t *>(recs + (size_t)row * REC + OFF_INDEX);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; i++) eq &= q[i] == a[i];
  return eq;
}

// slot of key k, or -1 (owners' keys are their index_txid)
__device__ inline int64_t tab_find(const uint32_t k[8], uint64_t h, const uint32_t *owner, const uint32_t *rowmap,
                                   const uint8_t *recs, uint32_t mask, const uint8_t *keys) {
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint32_t s = (uint32_t)(h + probe) & mask;
    const uint32_t o = owner[s];
    if (o == 0) return -1;
    if (keys ? key_eq(k, recs, 0, keys, o - 1) : key_eq(k, recs, rowmap[o - 1])) return s;
  }
  return -1;
}
// index key of a transaction of the device-parsed batch, as k_bd_fold writes it into the record
// (blockdev.hip): the computed txid digest, or the hex-decoded chdr.TxId
__device__ inline bool dev_index_key(const DevTx &R, const uint64_t *bases, const uint8_t *digests, uint32_t ntx,
                                     uint32_t t, uint32_t k[8]) {
  if (!(R.flags & BDF_INDEX_OK)) return false;
  if (!(R.flags & BDF_INDEX_FROM_TXID)) {
    const uint32_t *d = reinterpret_cast<const uint32_t *>(digests + ((size_t)BD_DIG_I * ntx + t) * 32);
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = d[i];
    return true;
  }
  if (R.index_txid.len != 64) return false;
  // only lowercase hex can equal a VALID txid
  return hex64_words(reinterpret_cast<const uint8_t *>(bases[R.blk]) + R.index_txid.off, k);
}

}  // namespace

// rank r holds transactions [rlo[r][b], rlo[r][b] + rcnt[r][b]) of block b, at its rows from
// roff[r][b] (any shard plan whose ranges tile every block).  Also resets the txid table
// (slots [0, cap)): the grid covers max(P, cap).
// For a single-device batch (txs != null) it also writes every position's index key to `keys`:
// k_fin_index_dev compares other owners' keys with plain loads -- written by this earlier kernel,
// so no device-scope fence inside the insert (on MI355X an agent-scope release writes back the
// whole L2 of the XCD: it made the insert 60-240 us beside the verify chain).
__global__ void k_fin_rows(uint32_t P, const uint64_t *blk_start, uint32_t nb, uint32_t W, uint32_t rows,
                           const uint32_t *roff, const uint32_t *rlo, const uint32_t *rcnt, uint32_t *rowmap,
                           uint32_t *blkof, uint32_t cap, uint32_t *owner, int32_t *minblk, uint32_t *minvalid,
                           const DevTx *txs, const uint64_t *bases, const uint8_t *digests, uint8_t *keys,
                           uint32_t prio) {
  if (prio) __builtin_amdgcn_s_setprio(3);  // (beside k_point28: the fold waits for this index)
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < cap) {
    owner[p] = 0u;
    minblk[p] = 0x7F7F7F7F;
    minvalid[p] = 0xFFFFFFFFu;
  }
  if (p >= P) return;
  if (txs) {
    uint32_t k[8];
    if (dev_index_key(txs[p], bases, digests, P, p, k)) {
      uint32_t *kd = reinterpret_cast<uint32_t *>(keys + (size_t)p * 32);
#pragma unroll
      for (int i = 0; i < 8; i++) kd[i] = k[i];
    }
  }
  uint32_t lo = 0, hi = nb;  // last b with blk_start[b] <= p
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blk_start[mid] <= p) lo = mid;
    else hi = mid;
  }
  const uint32_t b = lo;
  const uint32_t i = (uint32_t)(p - blk_start[b]);
  uint32_t r = 0;
  for (; r + 1 < W; r++) {
    const size_t k = (size_t)r * nb + b;
    if (i >= rlo[k] && i < rlo[k] + rcnt[k]) break;
  }
  const size_t k = (size_t)r * nb + b;
  rowmap[p] = r * rows + roff[k] + (i - rlo[k]);
  blkof[p] = b;
}

__global__ void k_fin_index(uint32_t P, const uint8_t *recs, const uint32_t *rowmap, const uint32_t *blkof,
                            uint32_t *owner, int32_t *minblk, uint32_t mask, uint64_t seed) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const uint32_t row = rowmap[p];
  if (!(recs[(size_t)row * REC + 1] & FGV_TXR_INDEXED)) return;
  uint32_t k[8];
  load_key(recs, row, OFF_INDEX, k);
  const uint64_t h = fin_hash(k, seed);
  const int32_t b = (int32_t)blkof[p];
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint32_t s = (uint32_t)(h + probe) & mask;
    uint32_t o = owner[s];
    if (o == 0) {
      o = atomicCAS(&owner[s], 0u, p + 1);
      if (o == 0) {
        atomicMin(&minblk[s], b);
        return;
      }
    }
    if (key_eq(k, recs, rowmap[o - 1])) {
      atomicMin(&minblk[s], b);
      return;
    }
  }
}
// k_fin_index for a single-device batch straight from the parse and the digests (one rank,
// position p == tx t), so it runs beside the verify chain instead of after the fold: the
// owners' keys go to `keys` (32 B per position), which k_fin_codes then compares against
__global__ void k_fin_index_dev(uint32_t P, const DevTx *txs, const uint64_t *bases, const uint8_t *digests,
                                uint8_t *keys, uint32_t *owner, int32_t *minblk, uint32_t mask, uint64_t seed,
                                uint32_t prio) {
  if (prio) __builtin_amdgcn_s_setprio(3);
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const DevTx &R = txs[p];
  uint32_t k[8];
  if (!dev_index_key(R, bases, digests, P, p, k)) return;
  const uint64_t h = fin_hash(k, seed);  // (every key is in `keys` already: k_fin_rows)
  const int32_t b = (int32_t)R.blk;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint32_t s = (uint32_t)(h + probe) & mask;
    uint32_t o = owner[s];
    if (o == 0) {
      o = atomicCAS(&owner[s], 0u, p + 1);
      if (o == 0) {
        atomicMin(&minblk[s], b);
        return;
      }
    }
    const uint32_t *q = reinterpret_cast<const uint32_t *>(keys + (size_t)(o - 1) * 32);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; i++) eq &= q[i] == k[i];
    if (eq) {
      atomicMin(&minblk[s], b);
      return;
    }
  }
}

__global__ void k_fin_codes(uint32_t P, const uint8_t *recs, const uint32_t *rowmap, const uint32_t *blkof,
                            const uint32_t *owner, const int32_t *minblk, uint32_t *minvalid, uint32_t mask,
                            uint64_t seed, uint8_t *flags, uint32_t *pslot, const uint8_t *keys) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const uint32_t row = rowmap[p];
  const uint8_t *r = recs + (size_t)row * REC;
  uint8_t code = r[0];
  uint32_t slot = 0xFFFFFFFFu;
  if (r[1] & FGV_TXR_REACHED) {
    uint32_t k[8];
    load_key(recs, row, OFF_TXID, k);
    const int64_t s = tab_find(k, fin_hash(k, seed), owner, rowmap, recs, mask, keys);
    if (s >= 0) {
      if (minblk[s] < (int32_t)blkof[p]) code = 9;  // txid indexed by an earlier block of the batch
      slot = (uint32_t)s;
    }
  }
  if (code == 0 && slot != 0xFFFFFFFFu) atomicMin(&minvalid[slot], p);
  flags[p] = code;
  pslot[p] = slot;
}

// unsup (the fused single-device call: its batch counters' flag word): the first VALID position
// of a txid was later failed by the key-level walk (blockdev.hip kl_walk_block), so the txid's
// first VALID transaction is not known here -> the batch is unsupported (bit 2)
__global__ void k_fin_dups(uint32_t P, const uint32_t *pslot, const uint32_t *minvalid, uint8_t *flags,
                           uint32_t *unsup, uint8_t *out, const uint32_t *misc_src, uint32_t *misc_out,
                           uint32_t *done) {
  __builtin_amdgcn_s_setprio(3);  // the last kernel of the back half; the next front half runs beside it
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) {
    uint8_t f = flags[p];
    if (f == 0 && pslot[p] != 0xFFFFFFFFu) {
      const uint32_t m = minvalid[pslot[p]];
      if (m < p) {
        if (unsup && flags[m] != 0) {  // the first VALID position was failed by the key-level walk
          atomicOr(unsup, 2u);
          f = 0xFD;  // (undecided: the per-block outcomes mark its block unsupported)
        } else {
          f = 9;  // markTXIdDuplicates: an earlier VALID tx of this block
        }
        flags[p] = f;
      }
    }
    // (out: the caller's pinned flag buffer, mapped -- no copy kernel behind this one)
    if (out) out[p] = f;
  }
  if (!misc_out) return;
  // the batch counters (misc_src[5] may have just been set above) to the mapped host copy by the
  // last workgroup to finish
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const uint32_t t = atomicAdd(done, 1u);
    if (t == gridDim.x - 1) {
      __threadfence();
      for (int k = 0; k < 16; k++) misc_out[k] = __atomic_load_n(misc_src + k, __ATOMIC_RELAXED);
      __threadfence_system();
      atomicExch(done, 0u);
    }
  }
}
