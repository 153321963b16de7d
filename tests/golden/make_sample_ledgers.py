"""Extract the reference's sample-ledger blocks as golden fixtures (run in the build container;
the GPU box never reads /root/reference).

Source (reference test data, read as files):
  core/ledger/kvledger/tests/testdata/v20/sample_ledgers/ledgersData.zip
      chains/chains/testchannel/blockfile_000000      (20 blocks, a Fabric v2.0 network:
      channel config, _lifecycle approvals / commits, marbles + marbles-private txs)
  core/ledger/kvledger/tests/testdata/v11/sample_ledgers_with_commit_hashes/ledgersData.zip
      chains/chains/ledger{1,2}/blockfile_000000      (9 blocks each: lscc deploys, public and
      private writes, deletes, and an MVCC_READ_CONFLICT in block 8)

Blockfile format (common/ledger/blkstorage/block_serialization.go:28-140): per block a varint
length, then varint number, rawbytes data_hash, rawbytes previous_hash, varint #envelopes,
rawbytes each, varint #metadata, rawbytes each.  Each block is re-marshalled here as a
common.Block (field order and proto3 omission rules of Go's deterministic Marshal).

Output: tests/golden/sample_ledgers.bin (our own container: per block a 4-byte little-endian
length + the common.Block bytes) and sample_ledgers.json (ledger name -> list of
{number, offset, len, flags (TRANSACTIONS_FILTER as stored by the reference), commit_hash (hex of
Metadata[COMMIT_HASH].value or null)}).
"""
import json
import os
import struct
import zipfile

REF = "/root/reference/core/ledger/kvledger/tests/testdata"
SOURCES = [
    ("v20_testchannel", "v20/sample_ledgers/ledgersData.zip", "ledgersData/chains/chains/testchannel/blockfile_000000"),
    ("v11_ledger1", "v11/sample_ledgers_with_commit_hashes/ledgersData.zip", "ledgersData/chains/chains/ledger1/blockfile_000000"),
    ("v11_ledger2", "v11/sample_ledgers_with_commit_hashes/ledgersData.zip", "ledgersData/chains/chains/ledger2/blockfile_000000"),
]
HERE = os.path.dirname(os.path.abspath(__file__))


def uvarint(b, o):
    v, s = 0, 0
    while True:
        c = b[o]
        o += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, o


def pvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def fld(num, payload):
    return pvarint(num << 3 | 2) + pvarint(len(payload)) + payload


def rawbytes(b, o):
    n, o = uvarint(b, o)
    return b[o:o + n], o + n


def serialized_blocks(raw):
    o = 0
    while o < len(raw):
        n, o = uvarint(raw, o)
        sb, o = raw[o:o + n], o + n
        p = 0
        num, p = uvarint(sb, p)
        dh, p = rawbytes(sb, p)
        ph, p = rawbytes(sb, p)
        ntx, p = uvarint(sb, p)
        data = []
        for _ in range(ntx):
            d, p = rawbytes(sb, p)
            data.append(d)
        nm, p = uvarint(sb, p)
        md = []
        for _ in range(nm):
            m, p = rawbytes(sb, p)
            md.append(m)
        assert p == len(sb)
        yield num, dh, ph, data, md


def marshal_block(num, dh, ph, data, md):
    hdr = (pvarint(1 << 3) + pvarint(num) if num else b"") + (fld(2, ph) if ph else b"") + (fld(3, dh) if dh else b"")
    return fld(1, hdr) + fld(2, b"".join(fld(1, d) for d in data)) + fld(3, b"".join(fld(1, m) for m in md))


def main():
    blob, index = bytearray(), {}
    for name, zpath, member in SOURCES:
        raw = zipfile.ZipFile(os.path.join(REF, zpath)).read(member)
        out = []
        for num, dh, ph, data, md in serialized_blocks(raw):
            b = marshal_block(num, dh, ph, data, md)
            ch = md[4] if len(md) > 4 else b""
            # Metadata{value = 1}: 0x0a 0x20 + 32 bytes
            commit = ch[2:].hex() if len(ch) == 34 and ch[:2] == b"\x0a\x20" else None
            out.append(dict(number=num, offset=len(blob) + 4, len=len(b), flags=list(md[2]) if len(md) > 2 else [],
                            commit_hash=commit))
            blob += struct.pack("<I", len(b)) + b
        index[name] = out
    open(os.path.join(HERE, "sample_ledgers.bin"), "wb").write(bytes(blob))
    json.dump(index, open(os.path.join(HERE, "sample_ledgers.json"), "w"), indent=0)
    print({k: len(v) for k, v in index.items()}, len(blob), "bytes")


if __name__ == "__main__":
    main()
