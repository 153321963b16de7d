"""The ordering service of a synthetic network: orderer org MSPs, orderer identities, and the
block signatures an orderer writes (BlockWriter.addBlockSignature, orderer/common/
multichannel/blockwriter.go:206-227):

  metadata[SIGNATURES] = Metadata{value: OrdererBlockMetadata{last_config: LastConfig{index}},
                                  signatures: [MetadataSignature{signature_header:
                                      SignatureHeader{creator, nonce}, signature}]}
  signature = Sign(value || signature_header || BlockHeaderBytes(header))

Several signers model a multi-orderer quorum (BFT-style signature sets); faults corrupt one
signature, drop the set, or sign with an identity the policy does not admit."""
import hashlib

from . import Key, make_cert, sign
from .blocks import Identity, f_bytes, f_msg, f_varint

BLOCK_SIGNATURES = 0  # common.BlockMetadataIndex_SIGNATURES


class Orderers:
    """orgs: orderer org MSP ids (OrdererMSP, Orderer2MSP, ...); per_org orderer nodes each."""

    def __init__(self, seed=3, orgs=1, per_org=1):
        self.mspids = ["OrdererMSP" if i == 0 else "Orderer%dMSP" % (i + 1) for i in range(orgs)]
        self.cas = [Key(seed, 50_000 + o) for o in range(orgs)]
        self.nodes, self.org_nodes = [], [[] for _ in range(orgs)]
        for o, m in enumerate(self.mspids):
            for q in range(per_org):
                idx = o * per_org + q
                k = Key(seed, 51_000 + idx)
                pem = make_cert(k, self.cas[o], "orderer%d.ord%d" % (q, o + 1), m, "ca.ord%d" % (o + 1), False,
                                5000 + idx)
                ident = Identity(k, m, pem, "orderer")
                self.nodes.append(ident)
                self.org_nodes[o].append(ident)

    def identities(self):
        """(serialized, txvalidator.Identity) as the peer's MSP layer knows them: valid, MEMBER +
        ORDERER role bits (NodeOU orderer classification, msp/mspimpl.go:331-376)"""
        from ..txvalidator import Identity as TI
        return [(i.serialized, TI(i.mspid, i.key.pub, True, i.id_digest, roles=1 | 1 << 4)) for i in self.nodes]


def _fields(buf):
    """[(field number, payload bytes)] of a message whose fields are all length-delimited"""
    out, i = [], 0
    while i < len(buf):
        tag, i = _uv(buf, i)
        if tag & 7 != 2:
            raise ValueError("unexpected wire type")
        n, i = _uv(buf, i)
        out.append((tag >> 3, buf[i:i + n]))
        i += n
    return out


def _uv(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def header_der(number, prev, data_hash):
    """protoutil.BlockHeaderBytes: DER SEQUENCE{INTEGER number, OCTET STRING prev, OCTET STRING dh}"""
    def dlen(n):
        if n < 128:
            return bytes([n])
        b = n.to_bytes((n.bit_length() + 7) // 8, "big")
        return bytes([0x80 | len(b)]) + b
    nb = number.to_bytes(max(1, (number.bit_length() + 7) // 8), "big")
    if nb[0] & 0x80:
        nb = b"\x00" + nb
    body = b"\x02" + dlen(len(nb)) + nb + b"\x04" + dlen(len(prev)) + prev + b"\x04" + dlen(len(data_hash)) + data_hash
    return b"\x30" + dlen(len(body)) + body


def block_header(block):
    """(number, previous_hash, data_hash) of a generated block"""
    raw = [p for n, p in _fields(block) if n == 1][-1]
    number, prev, dh, i = 0, b"", b"", 0
    while i < len(raw):
        tag, i = _uv(raw, i)
        if tag & 7 == 0:
            number, i = _uv(raw, i)
            continue
        n, i = _uv(raw, i)
        if tag >> 3 == 2:
            prev = raw[i:i + n]
        elif tag >> 3 == 3:
            dh = raw[i:i + n]
        i += n
    return number, prev, dh


def signature_metadata(block, signers, last_config=0, nonce_seed=0, bad=(), value=None, header_override=None):
    """Metadata bytes for metadata[SIGNATURES] signed by `signers` (Identity list).  bad: indices
    whose signature is corrupted (a flipped bit of the message).  header_override: (number, prev,
    dh) to sign instead of the block's own header (a signature over another block)."""
    number, prev, dh = header_override or block_header(block)
    hb = header_der(number, prev, dh)
    if value is None:
        value = f_msg(1, f_varint(1, last_config))  # OrdererBlockMetadata{last_config: LastConfig{index}}
    sigs = b""
    for k, ident in enumerate(signers):
        nonce = hashlib.sha256(b"nonce-%d-%d-%d" % (nonce_seed, number, k)).digest()[:24]
        sh = f_bytes(1, ident.serialized) + f_bytes(2, nonce)
        msg = value + sh + hb
        if k in bad:
            msg = msg + b"\x00"
        sig = sign(ident.key, hashlib.sha256(msg).digest())
        sigs += f_msg(2, f_bytes(1, sh) + f_bytes(2, sig))
    return f_bytes(1, value) + sigs


def with_signatures(block, metadata0):
    """the block with metadata[SIGNATURES] replaced (other entries kept)"""
    parts = _fields(block)
    out = b""
    for n, p in parts:
        if n == 3:
            ents = [q for m, q in _fields(p) if m == 1] if p else []
            ents = ents + [b""] * max(0, 5 - len(ents))
            ents[BLOCK_SIGNATURES] = metadata0
            p = b"".join(f_msg(1, e) for e in ents)
        out += f_msg(n, p)
    return out


def sign_block(block, signers, **kw):
    return with_signatures(block, signature_metadata(block, signers, **kw))
