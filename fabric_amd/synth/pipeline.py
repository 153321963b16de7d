"""Synthetic end-to-end commit pipeline (committer -> MVCC -> commit hash on the same blocks).

A peer takes each block through committer validation (core/committer/txvalidator/v20), then
MVCC validation and commit (core/ledger/kvledger/txmgmt/validation/validator.go:81-200,
kv_ledger.go:612-652), then the commit hash (kv_ledger.go:806-817).  These blocks are the C2
shape (500-tx endorser blocks, OutOf(2, Org1..3), real P-256 signatures, the C2 fault mix:
bad creator signature, one bad endorsement, policy unsatisfied, duplicate txid) whose rwsets
read-modify-write 4 keys of 200 B values in namespace "mycc" of a 1M-key state DB, with the C3
MVCC faults on top:
  stale    (1 %): one read carries a wrong version                         -> 11
  conflict (5 %): one read key was written by an earlier transaction of the block that ends
                  VALID (committer and MVCC)                                  -> 11
  shadow   (2 %): one read key was written by an earlier transaction the COMMITTER rejects
                  (its writes are never applied, so the read stands)          -> 0
Final code per transaction: the committer's code when it is not VALID, else the MVCC code.
After each block the generator applies the valid writes at Height{block, tx}, so the next
block's reads carry current versions (a cross-block read of a key the previous block wrote is
valid: the endorser simulated after that commit).
"""
import numpy as np

from . import blocks as B
from .blocks import kv_rwset, tx_rwset
from .mvcc import MvccState

NS = "mycc"


def _rwsets_fn(state, ntx, number, rng, out, stale, conflict, shadow, value_len, reads):
    def fn(labels):
        ccode = [B.EXPECTED[l] for l in labels]
        assert all(c is not None for c in ccode), "pipeline blocks need faults with known committer codes"
        keys = rng.choice(state.nkeys, size=ntx * reads, replace=False).reshape(ntx, reads)
        u = rng.random(ntx)
        read_keys = keys.copy()
        final = np.zeros(ntx, np.uint8)
        good, bad = [], []  # earlier txs: final VALID / committer-invalid
        kind = np.zeros(ntx, np.int8)
        for i in range(ntx):
            if ccode[i] != 0:
                final[i] = ccode[i]  # (its reads are never checked, its writes never applied)
                bad.append(i)
                continue
            if u[i] < stale:
                kind[i] = 1
                final[i] = 11
            elif u[i] < stale + conflict and good:
                j = good[rng.integers(len(good))]
                read_keys[i, 0] = keys[j, rng.integers(reads)]
                kind[i] = 2
                final[i] = 11
            elif u[i] < stale + conflict + shadow and bad:
                j = bad[rng.integers(len(bad))]
                read_keys[i, 0] = keys[j, rng.integers(reads)]
                kind[i] = 3
            if final[i] == 0:
                good.append(i)
        rws = []
        for i in range(ntx):
            rd = []
            for r in range(reads):
                k = int(read_keys[i, r])
                ver = state.version(k)
                if r == 1 and kind[i] == 1:
                    ver = (ver[0] + 1, ver[1]) if ver else (1, 1)
                rd.append((state.key(k), ver))
            val = rng.integers(0, 256, size=value_len, dtype=np.uint8).tobytes()
            wr = [(state.key(int(k)), val, False) for k in keys[i]]
            rws.append(tx_rwset([(NS, kv_rwset(rd, wr))]))
        for i in range(ntx):  # the expected commit: valid writes at Height{number, i}
            if final[i] == 0:
                for k in keys[i]:
                    state.blk[k] = number
                    state.txn[k] = i
                    state.present[k] = True
        out["final"] = final
        out["committer"] = np.array(ccode, np.uint8)
        return rws
    return fn


def make_blocks(net, state: MvccState, nblocks, ntx, first_number, seed=0, prev_hash=b"\x00" * 32, stale=0.01,
                conflict=0.05, shadow=0.02, value_len=200, reads=4, endorse_dist=((2, 0.6), (3, 0.4)), threads=8):
    """Consecutive pipeline blocks first_number, first_number + 1, ... (hash-chained).  Returns
    (list of block bytes, list of committer expected codes, list of final expected codes, the
    last header hash).  `state` advances by the blocks' expected commits."""
    out_b, out_c, out_f = [], [], []
    prev = prev_hash
    for i in range(nblocks):
        num = first_number + i
        rng = np.random.default_rng((seed << 20) ^ num)
        o = {}
        blk, lab, envs = B.make_block(net, ntx, number=num, seed=seed * 7919 + i, threads=threads, prev_hash=prev,
                                      endorse_dist=endorse_dist, value_len=value_len,
                                      rwsets=_rwsets_fn(state, ntx, num, rng, o, stale, conflict, shadow, value_len,
                                                        reads))
        out_b.append(blk)
        out_c.append(o["committer"])
        out_f.append(o["final"])
        prev = B.header_hash(num, prev, envs)
    return out_b, out_c, out_f, prev
