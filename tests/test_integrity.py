"""Deliver-side block integrity (fgv_blocks_verify, host code of libfgv) against the restated
VerifyBlock (oracle/blockverify.py): header chain, metadata count, well-formed envelopes
(proto.Marshal round trip), block data hash.  Host-only: runs without a GPU (ctx = NULL)."""
import hashlib
import random

import pytest

from fabric_amd import _lib
from fabric_amd.synth import blocks as B
from oracle import blockverify as O
from tests.blockfix import corrupt_envelopes, network


def mk_block(envs, number, prev=b"", data_hash=None, nmeta=5, header=True, data=True, extra_header=b""):
    dh = hashlib.sha256(b"".join(envs)).digest() if data_hash is None else data_hash
    hdr = B.f_varint(1, number) + B.f_bytes(2, prev) + B.f_bytes(3, dh)
    out = B.f_msg(1, hdr) + extra_header if header else b""
    if data:
        out += B.f_msg(2, b"".join(B.f_msg(1, e) for e in envs))
    out += B.f_msg(3, b"".join(B.f_msg(1, b"") for _ in range(nmeta)))
    return out


def env(payload, sig, pre=b"", mid=b"", post=b""):
    return pre + B.f_bytes(1, payload) + mid + B.f_bytes(2, sig) + post


def check(blks, chain_py=None, chain_c=None):
    got = _lib.blocks_verify(blks, chain_c)
    exp = O.verify_blocks(blks, chain_py)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g[0] == e[0], (i, g[0], e[0])
        if e[0] == O.TX_MALFORMED:
            assert g[1] == e[1], (i, g[1], e[1])
        if e[2] is not None:
            assert g[3] == e[2], i
        if e[3] is not None:
            assert g[4] == e[3], i
    return [g[0] for g in got]


@pytest.fixture(scope="module")
def c2_envs():
    return B.make_block(network(), 40, number=1, seed=5)[2]


def test_chain_of_generated_blocks():
    net = network()
    prev, blks = b"\x00" * 32, []
    chain_py = dict(number=0, header_hash=None)
    for n in range(1, 5):
        blk, _, envs = B.make_block(net, 30, number=n, seed=n, prev_hash=prev)
        blks.append(blk)
        prev = O.block_header_hash(n, prev, hashlib.sha256(b"".join(envs)).digest())
    chain_c = _lib.ChainState(number=0, valid=1, has_hash=0)
    assert check(blks, chain_py, chain_c) == [0, 0, 0, 0]
    assert chain_c.number == 4 and bytes(chain_c.header_hash) == prev == chain_py["header_hash"]
    # the next block must follow: a replay of block 2 fails the number check, a forked block 5
    # fails the previous-hash check, and neither advances the chain
    fork = B.make_block(net, 5, number=5, seed=9, prev_hash=b"\x11" * 32)[0]
    good = B.make_block(net, 5, number=5, seed=9, prev_hash=prev)[0]
    assert check([blks[1], fork, good], chain_py, chain_c) == [O.NUMBER, O.PREV_HASH, O.OK]
    assert chain_c.number == 5


def test_header_metadata_and_data_hash_faults(c2_envs):
    e = c2_envs[:6]
    blks = [
        mk_block(e, 1),
        mk_block(e, 1, header=False),
        mk_block(e, 1, nmeta=4),
        mk_block(e, 1, data_hash=b"\x00" * 32),
        mk_block(e, 1, data_hash=b""),
        mk_block([], 1),
        mk_block(e, 1, data=False),
        b"\x0a\x05\x01",  # truncated
        mk_block(e, 1, extra_header=B.f_msg(1, B.f_varint(1, 7))),  # header merge: number -> 7
        mk_block(e, 300, prev=b"\x22" * 32),  # multi-byte ASN.1 INTEGER
        mk_block(e, 1 << 63, prev=b"\x22" * 200),  # leading 0x00 INTEGER, long-form length
    ]
    st = check(blks)
    assert st[:8] == [O.OK, O.NO_HEADER, O.METADATA, O.DATA_HASH, O.DATA_HASH, O.EMPTY, O.EMPTY, O.UNPARSABLE]
    assert st[8:] == [O.OK, O.OK, O.OK]


def test_well_formed_envelope_rules(c2_envs):
    p = c2_envs[0]
    e0 = B.f_bytes(1, b"") or b""
    raw = [
        env(b"payload", b"sig"),                               # canonical
        env(b"payload", b"sig", post=B.f_varint(9, 5)),        # unknown after: re-marshalled at the end
        env(b"payload", b"sig", pre=B.f_varint(9, 5)),         # unknown before: reordered -> mismatch
        env(b"payload", b"sig", mid=B.f_varint(9, 5)),         # unknown between
        env(b"payload", b"sig", pre=B.f_bytes(1, b"old")),     # duplicate payload: Marshal emits one
        env(b"payload", b"", post=e0),                         # no signature
        env(b"", b"sig"),                                      # no payload
        b"\x0a\x80\x07" + b"p" * 7 + b"\x12\x03sig",           # non-minimal length varint
        b"\x8a\x00\x07" + b"p" * 7 + b"\x12\x03sig",           # non-minimal tag varint
        b"\x08\x01" + env(b"payload", b"sig"),                 # field 1 as varint (unknown) first
        env(b"payload", b"sig", post=b"\x08\x01"),             # ... or last
        env(b"payload", b"sig", post=b"\x0b\x0c"),             # empty group after
        env(b"payload", b"sig")[:-1],                          # truncated
        env(b"payload", b"sig", post=b"\x00"),                 # field number 0 -> unmarshal error
        env(b"payload", b"sig", post=b"\xfa\xff\xff\xff\x0f\x00"),  # max field number, empty bytes
        env(b"payload", b"sig", post=b"\x12\x00"),             # trailing empty signature record
    ]
    for i, r in enumerate(raw):
        blk = mk_block([p, r], 1)
        exp = O.verify_blocks([blk])[0]
        got = _lib.blocks_verify([blk])[0]
        assert (got[0], got[1] if exp[0] == O.TX_MALFORMED else None) == (exp[0], exp[1]), (i, got, exp)
    st = [O.verify_blocks([mk_block([p, r], 1)])[0][0] for r in raw]
    assert st[:2] == [O.OK, O.OK] and st[2] == O.TX_MALFORMED and st[10] == O.OK


def test_config_block_skips_well_formedness():
    chdr = B.f_varint(1, 1) + B.f_str(4, "ch")
    payload = B.f_msg(1, B.f_bytes(1, chdr))
    cfg = env(payload, b"", pre=B.f_varint(9, 1))  # no signature, reordered unknown: still OK
    assert check([mk_block([cfg], 1)]) == [O.OK]
    assert check([mk_block([cfg, cfg], 1)]) == [O.TX_MALFORMED]


@pytest.mark.parametrize("seed", [1, 2])
def test_corrupted_envelopes_and_blocks(c2_envs, seed):
    rng = random.Random(seed)
    bad = corrupt_envelopes(c2_envs, seed, 120)
    blks = [mk_block([c2_envs[0], b], 1) for b in bad]
    good = mk_block(c2_envs[:5], 1)
    for _ in range(80):
        b = bytearray(good)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        blks.append(bytes(b))
    st = check(blks)
    assert len(set(st)) >= 3


def test_host_sha256_matches_hashlib():
    rng = random.Random(7)
    for n in list(range(0, 130)) + [4096, 100_001]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert _lib.sha256_host(b)[0] == hashlib.sha256(b).digest(), n
