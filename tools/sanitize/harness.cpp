// harness.cpp -- CPU sanitizer run of libfgv's host code on untrusted bytes (ASan + UBSan build,
// tools/sanitize/Makefile).  Reads a case file of records [u32 kind][u32 len][bytes] written by
// tests/test_sanitize.py and drives every host parser a block or rwset reaches without a GPU:
//   kind 1 block   fgv_blocks_verify (ctx NULL: header chain, metadata, envelope well-formedness,
//                  data hash), fgv_commit_hash (every tx taken as VALID: the rwset walk of the
//                  update batch), fgv_block_parse_probe (the committer's host parser + policy fold
//                  + orderer-signature metadata)
//   kind 2 serialized identity registered in the probe's channel
//   kind 3 chaincode policy bytes (ApplicationPolicy) of namespace "mycc"
//   kind 4 TxReadWriteSet bytes: fgv_mvcc_parse_probe (phantom-path decode + range validators)
//   kind 5 channel name
//   kind 6 PEM certificate: fgv_x509_probe (the MSP cache miss's PEM / X.509 / sanitizeCert)
//   kind 7 FabricMSPConfig bytes: fgv_msp_config_probe (the cache miss's MSP model parse)
//   kind 9 canary: reads one byte past its record (proves the sanitizer is live)
// Any sanitizer report aborts the process (halt_on_error); exit 0 = clean.
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

#include "../../fabric_amd/csrc/fgv_internal.h"

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s CASEFILE\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<std::pair<uint32_t, std::vector<uint8_t>>> recs;
  for (;;) {
    uint32_t hd[2];
    if (fread(hd, 4, 2, f) != 2) break;
    std::vector<uint8_t> b(hd[1]);
    if (hd[1] && fread(b.data(), 1, hd[1], f) != hd[1]) return 2;
    recs.emplace_back(hd[0], std::move(b));
  }
  fclose(f);
  std::string channel = "testchannel";
  std::vector<const uint8_t *> ids;
  std::vector<size_t> id_lens;
  std::vector<uint8_t> policy;
  for (auto &r : recs) {
    if (r.first == 2) ids.push_back(r.second.data()), id_lens.push_back(r.second.size());
    if (r.first == 3) policy = r.second;
    if (r.first == 5) channel.assign(r.second.begin(), r.second.end());
  }
  uint64_t acc = 0;
  size_t nblocks = 0, nrws = 0, ncerts = 0;
  for (auto &r : recs) {
    // an exact-size heap copy: ASan sees any read past the record
    std::vector<uint8_t> buf(r.second);
    const uint8_t *p = buf.empty() ? nullptr : buf.data();
    const size_t n = buf.size();
    if (r.first == 1) {
      nblocks++;
      fgv_chain_state chain{};
      fgv_block_check chk{};
      const uint8_t *const blocks[1] = {p ? p : reinterpret_cast<const uint8_t *>("")};
      const size_t lens[1] = {n};
      fgv_blocks_verify(nullptr, 1, blocks, lens, &chain, &chk);
      acc = acc * 31 + (uint64_t)chk.status;
      const long ntx = fgv_block_count_txs(blocks[0], n);
      if (ntx > 0) {
        std::vector<uint8_t> flags((size_t)ntx, 0);
        uint8_t out[32];
        acc = acc * 31 + (uint64_t)(fgv_commit_hash(blocks[0], n, flags.data(), flags.size(), 7, nullptr, 0, out) + 16);
      }
      acc = acc * 31 + fgv_block_parse_probe(channel.c_str(), ids.data(), id_lens.data(), ids.size(), "mycc",
                                             policy.data(), policy.size(), blocks[0], n);
    } else if (r.first == 9) {
      // canary (tests/test_sanitize.py): one byte read past the record -- the run must abort
      acc += buf.data()[buf.size()];
    } else if (r.first == 6) {
      ncerts++;
      static char out[1 << 16];
      acc = acc * 31 + (uint64_t)(fgv_x509_probe(p ? p : reinterpret_cast<const uint8_t *>(""), n, out, sizeof out) + 2);
    } else if (r.first == 7) {
      ncerts++;
      acc = acc * 31 + fgv_msp_config_probe(p ? p : reinterpret_cast<const uint8_t *>(""), n);
    } else if (r.first == 4) {
      nrws++;
      acc = acc * 31 + fgv_mvcc_parse_probe(p ? p : reinterpret_cast<const uint8_t *>(""), n);
    }
  }
  printf("sanitize harness: %zu blocks, %zu rwsets, %zu certs, digest %016llx\n", nblocks, nrws, ncerts,
         (unsigned long long)acc);
  return 0;
}
