"""CPU: SHA3 MSPs in the oracle (msp/identities.go:170-227: the digest follows the MSP's
SignatureHashFamily).  Blocks whose Org2 identities sign SHA3-256 digests validate as the
generator labels say under a config that declares Org2 SHA3; registered as SHA2, the same
signatures fail (the GPU parity of both is tests/test_gpu_channel.py::test_sha3_msp)."""
import dataclasses
import hashlib

from fabric_amd.synth import blocks, chanconfig
from oracle import v20


def test_sha3_known_answer():
    # FIPS 202 SHA3-256("abc") (the digest the synthetic SHA3 identities sign)
    assert hashlib.sha3_256(b"abc").hexdigest() == "3a985da74fe225b2045c172d6bd390bd855f086e3e9d525b46bfe24511431532"


def test_sha3_msp_oracle():
    fam = {"Org2MSP": "SHA3"}
    net = blocks.Network(seed=21, orgs=3, clients=30, hash_families=fam)
    cfg = chanconfig.make_config(net.mspids, hash_families=fam)
    ccs = {"mycc": blocks.out_of_policy(2, net.mspids)}
    blk, lab, _ = blocks.make_block(net, 120, number=1, seed=300)
    got = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), ccs, config=cfg), [blk])[0]
    assert all(e is None or c == e for c, e in zip(got, blocks.expected_codes(lab)))
    valid = sum(1 for c in got if c == 0)
    assert valid > 100
    ids2 = [(s, dataclasses.replace(i, hash_family="SHA2")) for s, i in net.identities()]
    got2 = v20.validate_blocks(v20.ChannelModel(net.channel, ids2, ccs, config=chanconfig.make_config(net.mspids)),
                               [blk])[0]
    assert sum(1 for c in got2 if c == 0) < valid
