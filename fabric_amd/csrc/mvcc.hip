// mvcc.hip -- MVCC validation of a block on the GPU (gfx950), HBM-bound integer work.
//
// Reference semantics (core/ledger/kvledger/txmgmt/validation/validator.go:81-200): in block
// order, a transaction is MVCC_READ_CONFLICT if one of its read keys was written by an
// EARLIER VALID transaction of the block, or if the committed version differs from the read
// version.  Validity is sequential, so the GPU decides it by a monotone fixpoint over the
// per-key first writers:
//   st[i] in {UNDECIDED, VALID, INVALID}; INVALID initially for committer-invalid txs and
//   for static version conflicts.  Each round:
//     fw_cand(k)  = min{ j : st[j] != INVALID, k in W_j }      (atomicMin)
//     fw_valid(k) = min{ j : st[j] == VALID,   k in W_j }
//     undecided i -> INVALID if some read key k has fw_valid(k) < i
//                 -> VALID   if every read key k has fw_cand(k) >= i (or is never written)
//   The lowest undecided tx is always decided, so it terminates; rounds = longest chain.
//
// Keys are (namespace id, key bytes).  Tables compare FULL key bytes (exact), with a 64-bit
// tag only as the probe start / fast reject.
#include "fgv_kernels.h"

#define MV_EMPTY 0ull
#define ST_UNDEC 0
#define ST_VALID 1
#define ST_INVALID 2
#define FW_INF 0xFFFFFFFFu

__device__ __forceinline__ uint64_t mv_tag(const uint8_t *p, uint32_t n, uint32_t ns) {
  uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)ns * 0x9E3779B97F4A7C15ull);
  for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h | 1ull;  // never MV_EMPTY
}

__device__ __forceinline__ bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

__global__ __launch_bounds__(256) void k_mv_tags(const MvKey *__restrict__ keys, uint32_t n,
                                                 uint64_t *__restrict__ tags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const MvKey k = keys[i];
  tags[i] = mv_tag(reinterpret_cast<const uint8_t *>(k.ptr), k.len, k.ns);
}

// reads and writes of a block in one launch
__global__ __launch_bounds__(256) void k_mv_tags2(const MvKey *__restrict__ reads, uint32_t nr,
                                                  uint64_t *__restrict__ rtags, const MvKey *__restrict__ writes,
                                                  uint32_t nw, uint64_t *__restrict__ wtags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr + nw) return;
  const MvKey k = i < nr ? reads[i] : writes[i - nr];
  (i < nr ? rtags[i] : wtags[i - nr]) = mv_tag(reinterpret_cast<const uint8_t *>(k.ptr), k.len, k.ns);
}

// ---- committed state lookups (reads): static version check
__device__ __forceinline__ int64_t state_find(const StateSlot *tbl, uint64_t mask, const uint8_t *arena,
                                              uint64_t tag, const uint8_t *key, uint32_t len, uint32_t ns) {
  uint64_t idx = tag & mask;
  for (uint64_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    const uint64_t t = tbl[idx].tag;
    if (t == MV_EMPTY) return -1;
    if (t == tag && tbl[idx].key_len == len && (tbl[idx].nsf & 0x7fff) == ns &&
        bytes_eq(arena + tbl[idx].key_off, key, len))
      return (int64_t)idx;
  }
  return -1;
}

__global__ __launch_bounds__(256) void k_mv_lookup(const MvKey *__restrict__ reads, const uint64_t *__restrict__ tags,
                                                   uint32_t n, const StateSlot *__restrict__ tbl, uint64_t mask,
                                                   const uint8_t *__restrict__ arena, uint8_t *__restrict__ bad_tx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const MvKey r = reads[i];
  const int64_t s = state_find(tbl, mask, arena, tags[i], reinterpret_cast<const uint8_t *>(r.ptr), r.len, r.ns);
  const bool committed = s >= 0 && (tbl[s].nsf & 0x8000);
  const bool has_ver = (r.flags & 1) != 0;
  bool same;
  if (!committed || !has_ver) same = committed == has_ver;  // version.AreSame with nil
  else same = tbl[s].blk == r.blk && tbl[s].txn == r.txn;
  if (!same) bad_tx[r.tx] = 1;
}

// ---- per-block table of written keys (claim = CAS owner := write index + 1)
__global__ __launch_bounds__(256) void k_mv_blk_insert(const MvKey *__restrict__ writes, const uint64_t *__restrict__ tags,
                                                       uint32_t n, BlkSlot *__restrict__ tbl, uint32_t mask,
                                                       uint32_t *__restrict__ wslot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const MvKey w = writes[i];
  const uint64_t tag = tags[i];
  uint32_t idx = (uint32_t)tag & mask;
  for (uint32_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    uint32_t owner = atomicCAS(&tbl[idx].owner, 0u, i + 1);
    if (owner == 0) owner = i + 1;
    const MvKey o = writes[owner - 1];
    if (tags[owner - 1] == tag && o.len == w.len && o.ns == w.ns &&
        bytes_eq(reinterpret_cast<const uint8_t *>(o.ptr), reinterpret_cast<const uint8_t *>(w.ptr), w.len)) {
      wslot[i] = idx;
      return;
    }
  }
  wslot[i] = FW_INF;  // table full: host sizes it at >= 2x the writes, unreachable
}

// ---- fixpoint
__device__ __forceinline__ uint64_t fw_enc(uint32_t round, uint32_t tx) {
  return ((uint64_t)round << 32) | (0xFFFFFFFFu - tx);
}
__device__ __forceinline__ uint32_t fw_dec(uint64_t v, uint32_t round) {  // FW_INF: no writer this round
  return (uint32_t)(v >> 32) == round ? 0xFFFFFFFFu - (uint32_t)v : FW_INF;
}

// read -> written-key slot for i < n (a probe of the block's write table; exact key compare),
// then the initial fixpoint state of
// transaction i - n (after k_mv_lookup's static version check)
__global__ __launch_bounds__(256) void k_mv_find_init(const MvKey *__restrict__ reads, const uint64_t *__restrict__ rtags,
                                                      uint32_t n, const BlkSlot *__restrict__ tbl, uint32_t mask,
                                                      const MvKey *__restrict__ writes,
                                                      const uint64_t *__restrict__ wtags, uint32_t *__restrict__ rslot,
                                                      uint32_t ntx, const uint8_t *__restrict__ part,
                                                      const uint8_t *__restrict__ bad_tx, uint8_t *__restrict__ st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) {
    const uint32_t t = i - n;
    if (t < ntx) st[t] = (part[t] && !bad_tx[t]) ? ST_UNDEC : ST_INVALID;
    return;
  }
  const MvKey r = reads[i];
  const uint64_t tag = rtags[i];
  uint32_t idx = (uint32_t)tag & mask;
  uint32_t out = FW_INF;
  for (uint32_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    const uint32_t owner = tbl[idx].owner;
    if (owner == 0) break;
    if (wtags[owner - 1] != tag) continue;
    const MvKey o = writes[owner - 1];
    if (o.len == r.len && o.ns == r.ns &&
        bytes_eq(reinterpret_cast<const uint8_t *>(o.ptr), reinterpret_cast<const uint8_t *>(r.ptr), r.len)) {
      out = idx;
      break;
    }
  }
  rslot[i] = out;
}

// round r (>= 1): first non-invalid and first valid writer of every written key; also zeroes
// the round's undecided count (k_mv_decide follows on the stream)
__global__ __launch_bounds__(256) void k_mv_min(const MvKey *__restrict__ writes, const uint32_t *__restrict__ wslot,
                                                uint32_t n, const uint8_t *__restrict__ st, BlkSlot *__restrict__ tbl,
                                                uint32_t round, uint32_t *__restrict__ undecided) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *undecided = 0u;
  if (i >= n) return;
  const uint32_t tx = writes[i].tx;
  const uint8_t s = st[tx];
  if (s == ST_INVALID) return;
  const uint32_t k = wslot[i];
  atomicMax(reinterpret_cast<unsigned long long *>(&tbl[k].fw_cand), (unsigned long long)fw_enc(round, tx));
  if (s == ST_VALID) atomicMax(reinterpret_cast<unsigned long long *>(&tbl[k].fw_valid), (unsigned long long)fw_enc(round, tx));
}

__global__ __launch_bounds__(256) void k_mv_decide(uint32_t ntx, const uint32_t *__restrict__ rbeg,
                                                   const uint32_t *__restrict__ rslot, const BlkSlot *__restrict__ tbl,
                                                   uint8_t *__restrict__ st, uint32_t round,
                                                   uint32_t *__restrict__ undecided) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ntx || st[i] != ST_UNDEC) return;
  bool all_clear = true, conflict = false;
  for (uint32_t r = rbeg[i]; r < rbeg[i + 1]; r++) {
    const uint32_t k = rslot[r];
    if (k == FW_INF) continue;  // key never written in this block
    if (fw_dec(tbl[k].fw_valid, round) < i) {
      conflict = true;
      break;
    }
    if (fw_dec(tbl[k].fw_cand, round) < i) all_clear = false;
  }
  if (conflict) st[i] = ST_INVALID;
  else if (all_clear) st[i] = ST_VALID;
  else atomicAdd(undecided, 1u);
}

// ---- commit: last valid writer per key (txops: later writes overwrite earlier ones)
__global__ __launch_bounds__(256) void k_mv_lastwriter(const MvKey *__restrict__ writes, const uint32_t *__restrict__ wslot,
                                                       uint32_t n, const uint8_t *__restrict__ st,
                                                       BlkSlot *__restrict__ tbl) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t tx = writes[i].tx;
  if (st[tx] != ST_VALID) return;
  atomicMax(reinterpret_cast<unsigned long long *>(&tbl[wslot[i]].last), ((unsigned long long)tx << 32) | (i + 1));
}

// apply (phase 1): update existing state entries in place, mark the rest for insertion
__global__ __launch_bounds__(256) void k_mv_apply_find(const BlkSlot *__restrict__ btbl, uint32_t bcap,
                                                       const MvKey *__restrict__ writes, const uint64_t *__restrict__ wtags,
                                                       StateSlot *__restrict__ tbl, uint64_t mask,
                                                       const uint8_t *__restrict__ arena, uint64_t block_num,
                                                       uint32_t *__restrict__ pend, uint32_t *__restrict__ npend) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bcap) return;
  const uint64_t last = btbl[b].last;
  if (last == 0) return;
  const uint32_t wi = (uint32_t)(last & 0xffffffffu) - 1, tx = (uint32_t)(last >> 32);
  const MvKey w = writes[wi];
  const int64_t s = state_find(tbl, mask, arena, wtags[wi], reinterpret_cast<const uint8_t *>(w.ptr), w.len, w.ns);
  const bool del = (w.flags & 1) != 0;
  if (s >= 0) {
    tbl[s].blk = block_num;
    tbl[s].txn = tx;
    tbl[s].nsf = (uint16_t)((tbl[s].nsf & 0x7fff) | (del ? 0 : 0x8000));
  } else if (!del) {
    pend[atomicAdd(npend, 1u)] = b;
  }
}

// apply (phase 2): claim empty slots for keys known to be absent (no byte compares needed:
// every key of this launch is distinct and absent from the table)
__global__ __launch_bounds__(256) void k_mv_apply_insert(const BlkSlot *__restrict__ btbl, const uint32_t *__restrict__ pend,
                                                         uint32_t np, const MvKey *__restrict__ writes,
                                                         const uint64_t *__restrict__ wtags, StateSlot *__restrict__ tbl,
                                                         uint64_t mask, uint8_t *__restrict__ arena,
                                                         unsigned long long *__restrict__ arena_top,
                                                         uint64_t block_num) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  const uint64_t last = btbl[pend[j]].last;
  const uint32_t wi = (uint32_t)(last & 0xffffffffu) - 1, tx = (uint32_t)(last >> 32);
  const MvKey w = writes[wi];
  const uint64_t tag = wtags[wi];
  const uint64_t off = atomicAdd(arena_top, (unsigned long long)w.len);
  for (uint32_t q = 0; q < w.len; q++) arena[off + q] = reinterpret_cast<const uint8_t *>(w.ptr)[q];
  uint64_t idx = tag & mask;
  for (uint64_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    if (atomicCAS(reinterpret_cast<unsigned long long *>(&tbl[idx].tag), MV_EMPTY, (unsigned long long)tag) == MV_EMPTY) {
      tbl[idx].key_off = (uint32_t)off;
      tbl[idx].key_len = (uint16_t)w.len;
      tbl[idx].nsf = (uint16_t)(w.ns | 0x8000);
      tbl[idx].blk = block_num;
      tbl[idx].txn = tx;
      return;
    }
  }
}

// bulk load: `keys` distinct, versions in blk/txn fields -> insert (same claim protocol)
__global__ __launch_bounds__(256) void k_mv_load(const MvKey *__restrict__ keys, const uint64_t *__restrict__ tags,
                                                 uint32_t n, StateSlot *__restrict__ tbl, uint64_t mask,
                                                 uint8_t *__restrict__ arena, unsigned long long *__restrict__ arena_top) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const MvKey k = keys[i];
  const uint64_t off = atomicAdd(arena_top, (unsigned long long)k.len);
  for (uint32_t q = 0; q < k.len; q++) arena[off + q] = reinterpret_cast<const uint8_t *>(k.ptr)[q];
  uint64_t idx = tags[i] & mask;
  for (uint64_t probe = 0; probe <= mask; probe++, idx = (idx + 1) & mask) {
    if (atomicCAS(reinterpret_cast<unsigned long long *>(&tbl[idx].tag), MV_EMPTY, (unsigned long long)tags[i]) ==
        MV_EMPTY) {
      tbl[idx].key_off = (uint32_t)off;
      tbl[idx].key_len = (uint16_t)k.len;
      tbl[idx].nsf = (uint16_t)(k.ns | 0x8000);
      tbl[idx].blk = k.blk;
      tbl[idx].txn = k.txn;
      return;
    }
  }
}

__global__ __launch_bounds__(256) void k_mv_flags(uint32_t ntx, const uint8_t *__restrict__ part,
                                                  const uint8_t *__restrict__ st, uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ntx) return;
  out[i] = (part[i] && st[i] == ST_INVALID) ? 11 : 0;
}
