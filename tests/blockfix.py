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
