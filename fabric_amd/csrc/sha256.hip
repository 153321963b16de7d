// sha256.hip -- batched SHA-256 for gfx950: one message per lane, messages read in place
// from a byte arena (envelope bytes resident in HBM; no gather copy).
// Replaces bccsp/sw/hash.go:29-33 (Go crypto/sha256) for identity.Verify digests
// (msp/identities.go:179) and the TxID / proposal-hash checks (protoutil/proputils.go:354,
// protoutil/txutils.go:458).  Integer VALU only: ~2.7k 32-bit ops per 64-byte block.
#include "fgv_kernels.h"

#include "sha256_dev.h"
#include "sha3_dev.h"

__global__ __launch_bounds__(256) void k_sha256_jobs(const ShaJob *__restrict__ jobs, uint32_t n,
                                                     uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ShaJob j = jobs[i];
  if (j.pad == SHAJOB_SHA3) {  // a SHA3 MSP's identity.Verify digest (sha3_dev.h)
    const uint8_t *const p3[3] = {reinterpret_cast<const uint8_t *>(j.p[0]), reinterpret_cast<const uint8_t *>(j.p[1]),
                                  reinterpret_cast<const uint8_t *>(j.p[2])};
    fgvsha3::sha3_256_spans(p3, j.n, out + (size_t)i * 32);
    return;
  }
  JobView v;
  v.p[0] = reinterpret_cast<const uint8_t *>(j.p[0]);
  v.p[1] = reinterpret_cast<const uint8_t *>(j.p[1]);
  v.p[2] = reinterpret_cast<const uint8_t *>(j.p[2]);
  v.beg[0] = 0;
  v.beg[1] = j.n[0];
  v.beg[2] = j.n[0] + j.n[1];
  v.beg[3] = v.L = j.n[0] + j.n[1] + j.n[2];
  sha_view(v, out + (size_t)i * 32);
}

// one message per lane from a byte arena (BCCSP Hash batches, identity.Verify batches)
__global__ __launch_bounds__(256) void k_sha256(const uint8_t *__restrict__ buf,
                                                const uint64_t *__restrict__ off,
                                                const uint32_t *__restrict__ len, uint32_t n,
                                                uint8_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  JobView v;
  v.p[0] = v.p[1] = v.p[2] = buf + off[i];
  v.beg[0] = 0;
  v.beg[1] = v.beg[2] = v.beg[3] = v.L = len[i];
  sha_view(v, out + (size_t)i * 32);
}
