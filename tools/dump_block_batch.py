"""Dump a C2 block batch + channel config for tools/host_bench (host-side profiling only).

Format (little-endian): u32 count + (u32 len, bytes) records, in sections:
  channel name | identities (serialized) | valid flags (1 B each, one record) |
  id digests (32 B) | chaincode names | policies | blocks
"""
import struct
import sys

from fabric_amd.synth import blocks


def rec(b):
    return struct.pack("<I", len(b)) + b


def section(items):
    return struct.pack("<I", len(items)) + b"".join(rec(x) for x in items)


def main(path, nblocks=32, ntx=500):
    net = blocks.Network(seed=3, orgs=3, clients=100)
    blks = [blocks.make_block(net, ntx, number=1 + i, seed=i, threads=8)[0] for i in range(nblocks)]
    ids = net.identities()
    out = section([net.channel.encode()])
    out += section([i[0] for i in ids])
    out += section([bytes(1 if i[3] else 0 for i in ids)])
    out += section([i[4] for i in ids])
    out += section([k.encode() for k in net.chaincodes])
    out += section(list(net.chaincodes.values()))
    out += section(blks)
    open(path, "wb").write(out)


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
