"""CPU: the plain-C restated committer of the bench's CPU baseline (oracle/cpu_validator.c)
equals the Python oracle (oracle/v20.py) and the generator's labels on C2-shaped blocks with
every C2 fault class, in block order (txids of earlier blocks count as ledger duplicates)."""
import pytest

from fabric_amd.synth import blocks
from oracle import v20

import bench


@pytest.mark.parametrize("threads", [1, 3])
def test_c_baseline_equals_oracle(threads):
    net = blocks.Network(seed=3, orgs=3, clients=20)
    blks, labs, prev = [], [], b"\x00" * 32
    out = []
    for i in range(3):
        reuse = {5: (out[2].creator, out[2].nonce)} if i == 2 else None  # a txid of block 1 again
        b, lab, envs = blocks.make_block(net, 60, number=1 + i, seed=40 + i, endorse_dist=((2, 0.6), (3, 0.4)),
                                         prev_hash=prev, reuse=reuse, out_txs=out if i == 0 else None,
                                         faults=tuple((f, 4 * p) for f, p in blocks.FAULTS_C2))
        prev = blocks.header_hash(1 + i, prev, envs)
        blks.append(b)
        labs.append(lab)
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
    assert exp[2][5] == 9 and sum(c != 0 for f in exp for c in f) > 10
    rate, done, el, nb, parity = bench.cpu_c_validator(net, blks, labs, threads, 0.05, expected=exp)
    assert parity and done >= sum(len(f) for f in exp)
