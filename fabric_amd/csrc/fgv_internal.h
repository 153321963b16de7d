// fgv_internal.h -- host-internal interfaces between fgv_host.cpp (context, device buffers,
// kernels) and fgv_block.cpp (block parse / fold).  Not part of the C ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/fgv.h"
#include "fgv_kernels.h"

struct fgv_block_state;
fgv_block_state *fgv_block_state_new(unsigned threads);
void fgv_block_state_free(fgv_block_state *s);

int fgv_block_set_channel(fgv_block_state *S, const char *name);
int fgv_block_add_identity(fgv_block_state *S, const uint8_t *ser, size_t len, int32_t key_slot, int valid,
                           const uint8_t id_digest[32]);
int fgv_block_define_chaincode(fgv_block_state *S, const char *ns, const uint8_t *policy, size_t len);
int fgv_block_add_txids(fgv_block_state *S, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                        size_t n);
int fgv_block_validate_impl(fgv_ctx *c, fgv_block_state *S, size_t nblocks, const uint8_t *const *h_blocks,
                            const size_t *lens, const uint8_t *const *d_blocks, const uint32_t *tx_lo,
                            const uint32_t *tx_hi, fgv_tx_result *res_out, size_t res_cap, size_t *ntx_out);
long fgv_block_count_txs(const uint8_t *b, size_t n);
int fgv_finalize_impl(size_t nblocks, const size_t *ntx, const fgv_tx_result *res, uint8_t *flags);

// Device pass for one block batch: SHA-256 jobs -> digests (all), then ECDSA verify jobs whose
// digest is digests[dig_idx[i]] -> vstatus.  Implemented in fgv_host.cpp.
int fgv_run_block_jobs(fgv_ctx *c, const std::vector<ShaJob> &jobs, const std::vector<uint64_t> &sig_ptr,
                       const std::vector<uint32_t> &sig_len, const std::vector<uint32_t> &key_slot,
                       const std::vector<uint32_t> &dig_idx, std::vector<uint8_t> &digests,
                       std::vector<uint8_t> &vstatus);
