"""Throughput of key-level-endorsement batches (profiling aid, not the bench contract): 32
generated 500-tx blocks of namespace mycc with key-level parameters in state, metadata writes and
in-block dependencies (tests/sbe_cases.py; each block over its own key space, as a batch whose
blocks change each other's parameters is outside the model) -- on the device fold (DESIGN.md
s6a) and, for comparison, on the host parser's sequential fold (parse mode 1) -- against the same
blocks with no key-level state.  Blocks are host-resident (the call copies them H2D).  Parity with
the oracle is checked on each configuration; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fabric_amd import _lib, txvalidator
    from oracle import v20
    from tests import sbe_cases
    from tests.blockfix import network
    net = network()
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    nb, ntx, steps = 32, 500, 10
    made = [sbe_cases.make_sbe_block(net, ntx, 5000 + k, number=1 + k, nkeys=2000, vp_keys=400, prefix="b%dk" % k)
            for k in range(nb)]
    blks = [b for b, _ in made]
    kvmeta = {}
    for _, kv in made:
        kvmeta.update(kv)
    out, exps = {}, {}
    for name, kv, mode in (("key_level", kvmeta, 0), ("key_level_hostparse", kvmeta, 1), ("plain", {}, 0)):
        eng = _lib.Engine(0)
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), ccs, kvmeta=kv)
        key = "kl" if kv else "plain"
        if key not in exps:
            exps[key] = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=kv), blks)
        exp = exps[key]
        got = [list(f) for f in eng.validate_blocks(blks)]
        assert got == exp, name
        eng.validate_blocks(blks)
        t = time.perf_counter()
        for _ in range(steps):
            eng.validate_blocks(blks)
        el = (time.perf_counter() - t) / steps
        out[name] = dict(ms_per_batch=round(el * 1e3, 3), tx_per_s=round(nb * ntx / el, 1),
                         valid=sum(f.count(0) for f in exp), policy_failures=sum(f.count(10) for f in exp),
                         host_timing_ms=eng.host_timing())
        if mode == 0:
            # HBM-resident blocks through the pipelined call, as the headline bench runs C2: the next
            # call's front half enqueued ahead beside this one's back half
            import torch
            sizes = [(len(b) + 64 + 255) // 256 * 256 for b in blks]
            arena = torch.zeros(sum(sizes), dtype=torch.uint8, device="cuda:0")
            dptr, o = [], 0
            for b, sz in zip(blks, sizes):
                arena[o:o + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).to("cuda:0")
                dptr.append(arena.data_ptr() + o)
                o += sz
            torch.cuda.synchronize()
            bb = eng.block_batch(blks, dptr)
            got = eng.validate_blocks_pipelined(bb, bb)
            assert list(got) == [c for f in exp for c in f], name + " (HBM)"
            for _ in range(3):
                eng.validate_blocks_pipelined(bb, bb)
            t = time.perf_counter()
            for _ in range(4 * steps):
                eng.validate_blocks_pipelined(bb, bb)
            el = (time.perf_counter() - t) / (4 * steps)
            out[name + "_hbm_pipelined"] = dict(ms_per_batch=round(el * 1e3, 3), tx_per_s=round(nb * ntx / el, 1))
            del arena
        eng.close()
    print(json.dumps(dict(workload="32 x 500-tx key-level blocks (tools/bench_sbe.py)", parity=True, **out)))


if __name__ == "__main__":
    main()
