// mvcc_multi.h -- one k_mvx_extract launch over several blocks of a chain (fgv_mvcc.cpp
// mvcc_chain): each block keeps its own buffer set, counters and record ranges, exactly as a
// launch per block would write them; the workgroups of block q are [wg0_q, wg0_{q+1}).
// A C3 block's extraction is a serial protobuf walk per transaction (one lane each): ~10k lanes
// leave most of the chip idle for ~0.1 ms, so the blocks after the first are walked together.
#pragma once
#include <hip/hip_runtime.h>

#include "fgv_kernels.h"

#define MVX_MULTI_MAX 16  // blocks per launch (kernel argument: 16 x 80 B)
struct MvxJob {
  const uint8_t *base;
  const uint32_t *envtab;
  const uint8_t *in_flags;
  MvTxInfo *info;
  MvRec *reads, *writes;
  MvCounters *c;
  MvRec *scr;
  uint8_t *bad;
  uint32_t ntx, wg0;  // transactions; the block's first workgroup
};
struct MvxJobs {
  uint32_t n, touch;
  MvxJob j[MVX_MULTI_MAX];
};
// grid = the workgroups of every block (wg0 of block q = sum of the earlier blocks')
void mvx_extract_multi_launch(uint32_t tpw, hipStream_t st, const MvxJobs &J, uint32_t wgs);

// k_mvx_flags and k_mv_last of one chain block in one launch (independent steps after the
// fixpoint; commit = 0: the codes only)
__global__ void k_mvx_flags_last(uint32_t ntx, uint32_t rlast, const uint8_t *in_flags, const MvTxInfo *info,
                                 const uint8_t *st, uint8_t *out, MvCounters *c, uint32_t commit, const MvRec *writes,
                                 const uint32_t *wslot, BlkSlot *btbl, uint32_t epoch, const unsigned long long *top,
                                 uint64_t slots_cap, uint64_t arena_cap);
// the tails of up to MVX_MULTI_MAX chain blocks at once (k_mv_tail's work; workgroup q = block q):
// their counters, and the arena top once, after the last block's commit
struct MvTails {
  uint32_t n;
  const MvCounters *c[MVX_MULTI_MAX];
  uint32_t *hc[MVX_MULTI_MAX];
};
__global__ void k_mv_tails(const MvTails T, const unsigned long long *top, unsigned long long *htop);
