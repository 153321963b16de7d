"""Quick GPU check of whole-block validation vs the oracle."""
import collections, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20

net = blocks.Network(seed=3, orgs=3, clients=100)
eng = _lib.Engine(0)
txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
force = ["bad_txid", "bad_proposal_hash", "bad_epoch", "unknown_cc", "two_actions", "rogue_creator", "high_s_creator",
         "dup_endorser", "forged_endorser", "event_other_cc", "bad_payload", "no_sig", "clean", "dup_txid"] + ["corrupt"] * 40
blks = [blocks.make_block(net, 500, number=1 + i, seed=i)[0] for i in range(3)]
blks.append(blocks.make_block(net, len(force), number=9, seed=9, faults=(), force=force)[0])
model = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
exp = v20.validate_blocks(model, blks)
t = time.time()
got = eng.validate_blocks(blks)
print("gpu wall", time.time() - t, eng.timing())
for b in range(len(blks)):
    mism = [(i, int(got[b][i]), exp[b][i]) for i in range(len(exp[b])) if got[b][i] != exp[b][i]]
    print("block", b, "n", len(exp[b]), "codes", dict(collections.Counter(exp[b])), "mismatches", mism[:10])
# throughput on 64 x 500-tx blocks
big = [blocks.make_block(net, 500, number=100 + i, seed=100 + i)[0] for i in range(64)]
eng.validate_blocks(big)
for _ in range(3):
    t = time.time(); eng.validate_blocks(big); el = time.time() - t
    print(f"64x500 tx: {el*1e3:.1f} ms -> {64*500/el:,.0f} tx/s", eng.timing())
