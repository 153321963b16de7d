// host_bench.cpp -- host-side profiling harness for the block path (tools only, not shipped).
// Links fgv_block.cpp with a stub device pass that computes the SHA-256 jobs with OpenSSL on
// the CPU and reports every signature valid; "device addresses" are the host addresses.
// Usage: host_bench batch.bin [iters] [threads]
#include <openssl/sha.h>

#include <chrono>
#include <cstdio>
#include <fstream>

#include "../fabric_amd/csrc/fgv_block.cpp"

static std::vector<ShaJob> g_jobs;
static std::vector<uint64_t> g_sigp;
static std::vector<uint32_t> g_sigl, g_slot, g_didx;
static std::vector<uint8_t> g_dig, g_vst;

int fgv_block_jobs_reserve(fgv_ctx *, size_t nj, size_t nv, BlockJobs *out) {
  g_jobs.resize(nj + 1);
  g_sigp.resize(nv + 1);
  g_sigl.resize(nv + 1);
  g_slot.resize(nv + 1);
  g_didx.resize(nv + 1);
  *out = BlockJobs{g_jobs.data(), g_sigp.data(), g_sigl.data(), g_slot.data(), g_didx.data()};
  return FGV_OK;
}

int fgv_run_block_jobs(fgv_ctx *c, size_t nj, size_t nv, uint64_t, const uint8_t **digests,
                       const uint8_t **vstatus) {
  g_dig.assign(nj * 32 + 32, 0);
  g_vst.assign(nv + 1, 0);
  fgv_parallel_for(c->blk, nj, [&](size_t i) {
    SHA256_CTX s;
    SHA256_Init(&s);
    for (int k = 0; k < 3; k++)
      if (g_jobs[i].n[k]) SHA256_Update(&s, (const void *)(uintptr_t)g_jobs[i].p[k], g_jobs[i].n[k]);
    SHA256_Final(&g_dig[i * 32], &s);
  });
  *digests = g_dig.data();
  *vstatus = g_vst.data();
  return FGV_OK;
}

static std::vector<std::string> section(const std::string &buf, size_t &o) {
  auto u32 = [&](size_t at) { uint32_t v; memcpy(&v, buf.data() + at, 4); return v; };
  uint32_t n = u32(o);
  o += 4;
  std::vector<std::string> out;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t l = u32(o);
    out.emplace_back(buf.substr(o + 4, l));
    o += 4 + l;
  }
  return out;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  std::ifstream f(argv[1], std::ios::binary);
  std::string buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  const unsigned threads = argc > 3 ? (unsigned)atoi(argv[3]) : 8;
  size_t o = 0;
  auto chn = section(buf, o), ids = section(buf, o), valid = section(buf, o), digs = section(buf, o),
       ccs = section(buf, o), pols = section(buf, o), blks = section(buf, o);
  fgv_ctx *c = new fgv_ctx();
  c->blk = fgv_block_state_new(threads);
  fgv_block_set_channel(c->blk, chn[0].c_str());
  for (size_t i = 0; i < ids.size(); i++)
    fgv_block_add_identity(c->blk, (const uint8_t *)ids[i].data(), ids[i].size(), (int32_t)i, valid[0][i],
                           (const uint8_t *)digs[i].data());
  for (size_t i = 0; i < ccs.size(); i++)
    fgv_block_define_chaincode(c->blk, ccs[i].c_str(), (const uint8_t *)pols[i].data(), pols[i].size());
  std::vector<const uint8_t *> bp;
  std::vector<size_t> bl;
  size_t total = 0;
  for (auto &b : blks) {
    bp.push_back((const uint8_t *)b.data());
    bl.push_back(b.size());
    total += fgv_block_count_txs(bp.back(), b.size());
  }
  std::vector<fgv_tx_result> res(total);
  std::vector<size_t> ntx(blks.size());
  double acc[5] = {};
  for (int it = 0; it < iters; it++) {
    auto t0 = std::chrono::steady_clock::now();
    int rc = fgv_block_validate_impl(c, c->blk, blks.size(), bp.data(), bl.data(), bp.data(), nullptr, nullptr,
                                     res.data(), res.size(), ntx.data());
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc) { fprintf(stderr, "rc %d\n", rc); return 1; }
    if (it == 0) continue;
    acc[0] += c->t_host_parse; acc[1] += c->t_host_assemble; acc[2] += c->t_host_device; acc[3] += c->t_host_fold;
    acc[4] += ms;
  }
  int hist[256] = {};
  for (auto &r : res) hist[r.code]++;
  const double k = iters > 1 ? iters - 1 : 1;
  printf("txs %zu threads %u: parse %.3f asm %.3f dev(cpu sha) %.3f fold %.3f total %.3f ms\n", total, threads,
         acc[0] / k, acc[1] / k, acc[2] / k, acc[3] / k, acc[4] / k);
  for (int i = 0; i < 256; i++)
    if (hist[i]) printf("  code %d: %d\n", i, hist[i]);
  return 0;
}
