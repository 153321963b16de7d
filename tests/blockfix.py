"""Shared block fixtures for oracle and GPU block tests."""
import random

from fabric_amd.synth import blocks

# bad_payload last: its Payload does not unmarshal, so the key-level validator never signals its
# dependencies and the vscc of any later writer would wait for them forever (validator_keylevel.go:
# 184-222, vpmanagerimpl.go:300-303) -- a block the reference cannot validate
SPECIAL = ["bad_txid", "bad_proposal_hash", "bad_epoch", "unknown_cc", "two_actions", "rogue_creator",
           "high_s_creator", "dup_endorser", "forged_endorser", "event_other_cc", "no_sig",
           "clean", "dup_txid", "bad_payload"]

_NET = {}


def network(seed=3, orgs=3, clients=40, policy_n=2):
    k = (seed, orgs, clients, policy_n)
    if k not in _NET:
        _NET[k] = blocks.Network(seed=seed, orgs=orgs, clients=clients, policy_n=policy_n)
    return _NET[k]


def corrupt_envelopes(envs, seed, n):
    """n mutated copies of random envelopes: bit flips, truncation, byte insertion."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        e = bytearray(envs[rng.randrange(len(envs))])
        kind = rng.randrange(4)
        if kind == 0:
            for _ in range(rng.randint(1, 3)):
                e[rng.randrange(len(e))] ^= 1 << rng.randrange(8)
        elif kind == 1:
            del e[rng.randrange(len(e)):]
        elif kind == 2:
            pos = rng.randrange(len(e))
            e[pos:pos] = bytes([rng.randrange(256)])
        else:
            pos = rng.randrange(len(e))
            e[pos] = rng.choice([0x00, 0xff, 0x80, 0x7f, 0x0a, 0x12, 0x1a])
        out.append(bytes(e))
    return out


def block_from_envs(envs, number=1):
    f = blocks
    import hashlib
    header = f.f_varint(1, number) + f.f_bytes(2, b"\x00" * 32) + f.f_bytes(3, hashlib.sha256(b"".join(envs)).digest())
    data = b"".join(f.f_msg(1, e) for e in envs)
    return f.f_msg(1, header) + f.f_msg(2, data) + f.f_msg(3, b"".join(f.f_msg(1, b"") for _ in range(5)))


C5_NET = dict(seed=5, orgs=8, clients=60, policy_n=5, peers_per_org=2, ed25519_frac=0.1, ed25519_peers=1)
C5_ENDORSE = ((5, 0.5), (6, 0.5))


def network_c5():
    """C5-shaped network: 8 orgs x 2 peers, OutOf(5, 8 orgs), Ed25519 clients and one Ed25519
    peer (the reference rejects Ed25519 identities at DeserializeIdentity)."""
    k = tuple(sorted(C5_NET.items()))
    if k not in _NET:
        _NET[k] = blocks.Network(**C5_NET)
    return _NET[k]


def _varint_at(b, o):
    v = s = 0
    while True:
        c = b[o]
        o += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, o


def _venc(v):
    out = bytearray()
    while True:
        c = v & 0x7F
        v >>= 7
        out.append(c | (0x80 if v else 0))
        if not v:
            return bytes(out)


def replace_field(msg, path, new):
    """msg with the length-delimited field at path replaced by `new`; path: [(field number,
    occurrence)] from the outermost message inward (every enclosing length re-encoded)"""
    (num, occ), rest = path[0], path[1:]
    o, seen = 0, 0
    while o < len(msg):
        start = o
        key, o = _varint_at(msg, o)
        wt = key & 7
        if wt == 0:
            _, o = _varint_at(msg, o)
        elif wt == 1:
            o += 8
        elif wt == 5:
            o += 4
        elif wt == 2:
            ln, vs = _varint_at(msg, o)
            o = vs + ln
            if key >> 3 == num:
                if seen == occ:
                    inner = replace_field(msg[vs:o], rest, new) if rest else new
                    return msg[:start] + _venc(key) + _venc(len(inner)) + inner + msg[o:]
                seen += 1
        else:
            raise ValueError("wire type %d" % wt)
    raise KeyError(num)


# Block.data(2) -> BlockData.data(1)[tx] -> Envelope.payload(1) -> Payload.header(1) ->
# Header.signature_header(2) -> SignatureHeader.creator(1) -> SerializedIdentity.id_bytes(2)
def creator_idbytes_path(tx):
    return [(2, 0), (1, tx), (1, 0), (1, 0), (2, 0), (1, 0), (2, 0)]
