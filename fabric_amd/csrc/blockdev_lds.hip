// blockdev_lds.hip -- k_bd_parse_lds: the LDS-staged variant of the committer's protobuf walk
// (FGV_PARSE_LDS = 4 / 8 / 16 transactions per workgroup, an A/B mode), with
// the identity lookups of k_bd_ident folded into its idle lanes.
#include "blockdev_parse.h"

// LDS-staged walk: one 64-lane workgroup per TPW transactions.  The wave first copies the
// group's envelopes into LDS -- 16-byte loads of the aligned lines covering [off, off + len + 8)
// (the walk's over-read contract), every line in flight at once -- then lane j walks transaction
// j from LDS through a virtual base, so each of the walk's dependent loads is an LDS access
// instead of a cache round trip (the global walk pays ~0.5-1 us per field).  An envelope larger
// than CAP bytes is walked from global memory.
// ident (nullable): k_bd_ident's work in the same workgroup once the walks are done -- the
// creator and endorser SerializedIdentities of the group's transactions (bytes in LDS when
// staged) resolved against the HBM registry by four 16-lane groups at a time, the 56 lanes the
// walk leaves idle -- so the front half has one kernel fewer on its chain.
template <uint32_t TPW, uint32_t CAP>
__global__ __launch_bounds__(64) void k_bd_parse_lds(uint32_t ntx, const uint32_t *__restrict__ envtab,
                                                     const uint64_t *__restrict__ bases, DevChannel ch,
                                                     DevTx *__restrict__ out, uint32_t *__restrict__ flags,
                                                     uint32_t *__restrict__ xhaz, KlDev kl,
                                                     int32_t *__restrict__ ident) {
  __builtin_amdgcn_s_setprio(2);
  constexpr uint32_t C16 = CAP / 16;  // 16-byte lines per staged envelope
  __shared__ ParseLdsT<TPW> L;
  __shared__ uint4 env[TPW * C16];
  __shared__ uint32_t pre[TPW + 1];
  __shared__ uint64_t src[TPW];  // aligned source line of each staged envelope
  const uint32_t lane = threadIdx.x, t0 = blockIdx.x * TPW;
  uint32_t my = 0;
  if (lane < TPW && t0 + lane < ntx) {
    const uint32_t *et = envtab + BD_ENV_WORDS * (t0 + lane);
    const uint64_t a = bases[et[0]] + et[1];
    const uint64_t a0 = a & ~15ull, a1 = (a + et[2] + 8u + 15u) & ~15ull;
    if (a1 - a0 <= CAP) {
      my = (uint32_t)((a1 - a0) / 16u);
      src[lane] = a0;
    }
  }
  uint32_t v = my;  // inclusive prefix over the TPW lanes (wave scan)
  for (uint32_t dd = 1; dd < TPW; dd <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, dd);
    if (lane >= dd) v += o;
  }
  if (lane < TPW) pre[lane + 1] = v;
  if (lane == 0) pre[0] = 0;
  __syncthreads();
  const uint32_t total = pre[TPW];
  // 8 lines per lane per pass, all loads issued before the first LDS store
  constexpr uint32_t U = 8;
  for (uint32_t i0 = lane; i0 < total; i0 += 64 * U) {
    uint4 val[U];
    uint32_t dst[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t i = i0 + 64 * u;
      dst[u] = 0xFFFFFFFFu;
      if (i < total) {
        uint32_t j = 0;  // the envelope of line i: pre[j] <= i < pre[j + 1]
#pragma unroll
        for (uint32_t b = TPW / 2; b > 0; b >>= 1)
          if (pre[j + b] <= i) j += b;
        const uint32_t k = i - pre[j];
        val[u] = reinterpret_cast<const uint4 *>(src[j])[k];
        dst[u] = j * C16 + k;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (dst[u] != 0xFFFFFFFFu) env[dst[u]] = val[u];
  }
  __syncthreads();
  __shared__ const uint8_t *vbase[TPW];  // each transaction's walk base (LDS virtual base or block)
  __shared__ DSpan occ[TPW][BD_OCC];     // its creator and endorser SerializedIdentity spans
  __shared__ uint32_t nocc[TPW];         // 1 + endorsements (0: no transaction)
  __shared__ uint32_t want0[TPW];        // the creator is needed (the parse got past the channel check)
  const uint32_t t = t0 + lane;
  if (lane < TPW && t < ntx) {
    const uint32_t *et = envtab + BD_ENV_WORDS * t;
    const uint32_t blk = et[0];
    const uint8_t *base = reinterpret_cast<const uint8_t *>(bases[blk]);
    if (my) {  // the virtual base: block offset o -> env + (o - (a0 - block))
      const uint64_t a0 = src[lane];
      base = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(&env[lane * C16]) -
                                               (uintptr_t)(a0 - bases[blk]));
    } else {
      touch_lines(base + et[1], et[2]);
    }
    parse_one<TPW>(t, lane, blk, L, base, S{base + et[1], et[2]}, ch, out, flags, xhaz, kl);
    if (ident) {
      const DevTx &O = out[t];  // (written by this lane)
      const uint32_t ne = O.nend;
      vbase[lane] = base;
      nocc[lane] = 1 + ne;
      want0[lane] = O.pre == C_PENDING && O.creator.len != 0;
      occ[lane][0] = O.creator;
      for (uint32_t k = 0; k < ne; k++) occ[lane][1 + k] = O.end_ser[k];
    }
  } else if (ident && lane < TPW) {
    nocc[lane] = 0;
  }
  if (!ident) return;
  __syncthreads();
  // k_bd_ident's lookups: group g of 16 lanes takes (transaction, occurrence) pairs g, g + 4, ...
  const uint32_t g = lane / ID_LANES, l = lane % ID_LANES;
  for (uint32_t p = g; p < TPW * BD_OCC; p += 64u / ID_LANES) {
    const uint32_t j = p / BD_OCC, k = p % BD_OCC;
    if (k >= nocc[j]) continue;  // (uniform within the group)
    const bool want = k == 0 ? want0[j] != 0 : true;
    const int32_t res = want ? ident_lookup(absl(vbase[j], occ[j][k]), ch, l) : -1;
    if (l == 0) ident[(size_t)(t0 + j) * BD_OCC + k] = res;
  }
}

void bd_parse_lds_launch(uint32_t tpw, hipStream_t st, uint32_t ntx, const uint32_t *envtab, const uint64_t *bases,
                         const DevChannel &ch, DevTx *out, uint32_t *flags, uint32_t *xhaz, const KlDev &kl,
                         int32_t *ident) {
  if (tpw == 16)
    hipLaunchKernelGGL((k_bd_parse_lds<16, 4352>), dim3((ntx + 15) / 16), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
  else if (tpw == 4)
    hipLaunchKernelGGL((k_bd_parse_lds<4, 4352>), dim3((ntx + 3) / 4), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
  else
    hipLaunchKernelGGL((k_bd_parse_lds<8, 4352>), dim3((ntx + 7) / 8), dim3(64), 0, st, ntx, envtab, bases, ch, out,
                       flags, xhaz, kl, ident);
}
