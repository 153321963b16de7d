// lds_comb.hip -- micro-benchmark (profiling aid, not product code): the generator half of a
// verify, u1*G, as k_point28 computes it (radix-2^28 Montgomery, madd28 per comb term), with the
// fixed-base table of G either
//   global  the engine's comb: 17 windows of 16 bits, 32768 signed entries each (33.5 MB in HBM /
//           Infinity Cache), one 64-B gather per term, 17 terms per verify
//   lds w   a w-bit comb staged in LDS per workgroup (north_star's "generator tables in LDS"):
//           ceil(256/w) windows x 2^(w-1) entries x 64 B -- w = 7: 37 terms, 148 KB;
//           w = 6: 43 terms, 86 KB; w = 4: 64 terms, 32 KB
// Table contents and digits are random (the arithmetic's instruction stream and the access
// pattern are what is timed).  Prints ns per item for n items, one lane per item.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

#include "../../fabric_amd/csrc/p256_kernels.hip"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ inline void load_pt(const uint4 *p, f28 &px, f28 &py) {
  const uint4 n0 = p[0], n1 = p[1], n2 = p[2], n3 = p[3];
  const uint32_t wx[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
  const uint32_t wy[8] = {n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
  f28_from32(px, wx);
  f28_from32(py, wy);
}

__device__ inline uint32_t rnd(uint32_t &s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

// global comb: terms gathered from `tab` (windows x entries x 64 B), next term prefetched
__global__ __launch_bounds__(256, 2) void k_global(uint32_t n, const uint4 *tab, uint32_t windows, uint32_t entries,
                                                  uint32_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = 0x9E3779B9u ^ (i * 2654435761u);
  jp28 acc;
  load_pt(tab + ((size_t)(rnd(s) % entries)) * 4, acc.x, acc.y);
  f28_load_c(acc.z, ONE28);
  const uint4 *pn = tab + ((size_t)entries + rnd(s) % entries) * 4;
  uint4 n0 = pn[0], n1 = pn[1], n2 = pn[2], n3 = pn[3];
#pragma unroll 1
  for (uint32_t w = 1; w < windows; w++) {
    const uint32_t wx[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
    const uint32_t wy[8] = {n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
    if (w + 1 < windows) {
      pn = tab + ((size_t)(w + 1) * entries + rnd(s) % entries) * 4;
      n0 = pn[0];
      n1 = pn[1];
      n2 = pn[2];
      n3 = pn[3];
    }
    f28 px, py;
    f28_from32(px, wx);
    f28_from32(py, wy);
    madd28(acc, px, py);
  }
  out[i] = acc.x.v[0] ^ acc.y.v[1] ^ acc.z.v[2];
}

// LDS comb: the workgroup stages the whole table (windows x entries x 64 B) once, then every
// term is an LDS read
__global__ __launch_bounds__(256) void k_lds(uint32_t n, const uint4 *tab, uint32_t windows, uint32_t entries,
                                            uint32_t *out) {
  extern __shared__ uint4 lt[];
  const uint32_t words = windows * entries * 4;
  for (uint32_t k = threadIdx.x; k < words; k += blockDim.x) lt[k] = tab[k];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = 0x9E3779B9u ^ (i * 2654435761u);
  jp28 acc;
  load_pt(lt + (rnd(s) % entries) * 4, acc.x, acc.y);
  f28_load_c(acc.z, ONE28);
#pragma unroll 1
  for (uint32_t w = 1; w < windows; w++) {
    f28 px, py;
    load_pt(lt + (w * entries + rnd(s) % entries) * 4, px, py);
    madd28(acc, px, py);
  }
  out[i] = acc.x.v[0] ^ acc.y.v[1] ^ acc.z.v[2];
}

int main() {
  const uint32_t n = 131072;
  const size_t gbytes = (size_t)NGWIN * GT_K * 64;
  std::vector<uint32_t> h(gbytes / 4);
  uint32_t s = 12345;
  for (auto &x : h) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    x = s & 0x0FFFFFFFu;
  }
  uint4 *dtab;
  uint32_t *dout;
  CK(hipMalloc(&dtab, gbytes));
  CK(hipMalloc(&dout, n * 4));
  CK(hipMemcpy(dtab, h.data(), gbytes, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    const char *name;
    int lds;
    uint32_t windows, entries;
  } vs[] = {{"global 16-bit comb (17 terms, 33.5 MB)", 0, NGWIN, GT_K},
            {"lds 7-bit comb (37 terms, 148 KB)", 1, 37, 64},
            {"lds 6-bit comb (43 terms, 86 KB)", 1, 43, 32},
            {"lds 4-bit comb (64 terms, 32 KB)", 1, 64, 8}};
  for (const V &v : vs) {
    const size_t lb = (size_t)v.windows * v.entries * 64;
    if (v.lds) CK(hipFuncSetAttribute((const void *)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb));
    float best = 1e30f;
    for (int rep = 0; rep < 6; rep++) {
      CK(hipEventRecord(a));
      if (v.lds)
        hipLaunchKernelGGL(k_lds, dim3((n + 255) / 256), dim3(256), lb, 0, n, dtab, v.windows, v.entries, dout);
      else
        hipLaunchKernelGGL(k_global, dim3((n + 255) / 256), dim3(256), 0, 0, n, dtab, v.windows, v.entries, dout);
      CK(hipGetLastError());
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-42s %8.1f us per %u items  %6.2f ns/item\n", v.name, best * 1e3, n, best * 1e6 / n);
  }
  return 0;
}
