"""Synthetic MVCC workload (BASELINE configs[2], C3 shape).

State DB: N keys `k%07d` in namespace "mycc", committed versions uniform over blocks 1..1000,
tx 0..499 (seed 4).  Blocks of endorser transactions whose rwsets read 4 keys and write the
same 4 keys (read-modify-write); every tx of a block touches fresh keys (sampled without
replacement), then faults are injected with the generator's own label:
  stale    (1 %):   one read carries a wrong version              -> 11
  conflict (5 %):   one read key is written by an earlier clean tx -> 11
  chain    (0.5 %): one read key is written by an earlier STALE tx (invalid, so its write is
                    not in `updates`)                              -> 0
private_every=P > 0 makes every key index divisible by P a private-data key: it lives in the
hashed-data namespace "mycc$$hpvt" under SHA-256(key) and transactions read/write it through
the collection "pvt" hashed rwset (validator.go:246-293); the labels do not change.
Envelope signatures are not real (MVCC never checks them): the committer flags passed in say
which transactions are valid.  After each block the generator applies its own expectation of
the commit (valid writes at Height{block, tx}) so consecutive blocks read current versions.
"""
import hashlib

import numpy as np

from .blocks import f_bytes, f_msg, f_str, f_varint, hashed_rwset, kv_rwset, tx_rwset

NS = "mycc"
COLL = "pvt"
HASHED_NS = NS + "$$h" + COLL   # privacyenabledstate.deriveHashedDataNs


class MvccState:
    def __init__(self, nkeys=1_000_000, seed=4, private_every=0):
        rng = np.random.default_rng(seed)
        self.nkeys = nkeys
        self.private_every = private_every
        self.blk = rng.integers(1, 1001, size=nkeys, dtype=np.int64)
        self.txn = rng.integers(0, 500, size=nkeys, dtype=np.int64)
        self.present = np.ones(nkeys, dtype=bool)

    @staticmethod
    def key(i):
        return "k%07d" % i

    def is_private(self, i):
        return self.private_every > 0 and i % self.private_every == 0

    @staticmethod
    def key_hash(i):
        return hashlib.sha256(MvccState.key(i).encode()).digest()

    def items(self):
        """(keys list, blk, txn) of present public keys -- the bulk load of namespace NS"""
        idx = np.nonzero(self.present)[0]
        if self.private_every > 0:
            idx = idx[idx % self.private_every != 0]
        return [self.key(i) for i in idx], self.blk[idx], self.txn[idx]

    def items_hashed(self):
        """(key hashes, blk, txn) of present private keys -- the bulk load of HASHED_NS"""
        if self.private_every <= 0:
            return [], self.blk[:0], self.txn[:0]
        idx = np.nonzero(self.present)[0]
        idx = idx[idx % self.private_every == 0]
        return [self.key_hash(i) for i in idx], self.blk[idx], self.txn[idx]

    def version(self, i):
        return (int(self.blk[i]), int(self.txn[i])) if self.present[i] else None


def _envelope(rw_bytes, i, number):
    cca = f_bytes(1, rw_bytes) + f_msg(3, f_varint(1, 200)) + f_msg(4, f_str(2, NS) + f_str(3, "1.0"))
    prp = f_bytes(1, b"\x11" * 32) + f_bytes(2, cca)
    cap = f_bytes(1, b"ccpp") + f_msg(2, f_bytes(1, prp))
    shdr = f_bytes(1, b"creator") + f_bytes(2, b"n%08d" % i)
    tx = f_msg(1, f_bytes(1, shdr) + f_bytes(2, cap))
    chdr = f_varint(1, 3) + f_str(4, "testchannel") + f_str(5, "%064x" % (number * 1_000_000 + i))
    payload = f_msg(1, f_bytes(1, chdr) + f_bytes(2, shdr)) + f_bytes(2, tx)
    return f_bytes(1, payload) + f_bytes(2, b"\x30\x06\x02\x01\x01\x02\x01\x01")


def make_block(state: MvccState, ntx=10_000, number=1001, seed=0, stale=0.01, conflict=0.05, chain=0.005,
               reads=4, apply=True):
    """Returns (block_bytes, labels (0/11 per tx), committer_flags (all 0))."""
    rng = np.random.default_rng(seed)
    keys = rng.choice(state.nkeys, size=ntx * reads, replace=False).reshape(ntx, reads)
    u = rng.random(ntx)
    kind = np.zeros(ntx, np.int8)          # 0 clean, 1 stale, 2 conflict, 3 chain
    kind[u < stale] = 1
    kind[(u >= stale) & (u < stale + conflict)] = 2
    kind[(u >= stale + conflict) & (u < stale + conflict + chain)] = 3
    labels = np.zeros(ntx, np.uint8)
    read_keys = keys.copy()
    clean_seen, stale_seen = [], []
    for i in range(ntx):
        if kind[i] == 2 and clean_seen:
            j = clean_seen[rng.integers(len(clean_seen))]
            read_keys[i, 0] = keys[j, rng.integers(reads)]
            labels[i] = 11
        elif kind[i] == 3 and stale_seen:
            j = stale_seen[rng.integers(len(stale_seen))]
            read_keys[i, 0] = keys[j, rng.integers(reads)]
        elif kind[i] == 1:
            labels[i] = 11
        if kind[i] == 0:
            clean_seen.append(i)
        elif kind[i] == 1:
            stale_seen.append(i)
    envs = []
    vhash = hashlib.sha256(b"v" * 16).digest()
    for i in range(ntx):
        rd, hrd = [], []
        for r in range(reads):
            k = int(read_keys[i, r])
            ver = state.version(k)
            if r == 1 and kind[i] == 1:
                ver = (ver[0] + 1, ver[1]) if ver else (1, 1)
            if state.is_private(k):
                hrd.append((state.key_hash(k), ver))
            else:
                rd.append((state.key(k), ver))
        wr = [(state.key(int(k)), b"v" * 16, False) for k in keys[i] if not state.is_private(int(k))]
        hwr = [(state.key_hash(int(k)), vhash, False) for k in keys[i] if state.is_private(int(k))]
        ns_set = (NS, kv_rwset(rd, wr), [(COLL, hashed_rwset(hrd, hwr))]) if hrd or hwr else (NS, kv_rwset(rd, wr))
        envs.append(_envelope(tx_rwset([ns_set]), i, number))
    header = f_varint(1, number) + f_bytes(2, b"\x00" * 32) + f_bytes(3, b"\x00" * 32)
    block = f_msg(1, header) + f_msg(2, b"".join(f_msg(1, e) for e in envs)) + \
        f_msg(3, b"".join(f_msg(1, b"") for _ in range(5)))
    if apply:  # the generator's expected commit: valid txs' writes at Height{number, i}
        for i in range(ntx):
            if labels[i] == 0:
                for k in keys[i]:
                    state.blk[k] = number
                    state.txn[k] = i
                    state.present[k] = True
    return block, labels, np.zeros(ntx, np.uint8)
