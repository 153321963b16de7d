"""Key-level endorsement cases: the reference-test known answers of tests/golden/
sbe_known_answers.json (see tests/golden/make_sbe_known_answers.py for the sources), and a
generator of synthetic blocks with key-level parameters, metadata writes and in-block
dependencies (expectations from the oracle)."""
import hashlib
import json
import os
import random

from fabric_amd.synth import blocks
from fabric_amd.synth.blocks import f_bytes, f_msg, f_str
from fabric_amd.txvalidator import Identity

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sbe_known_answers.json")


def load():
    d = json.load(open(GOLD))
    pool = d["identities"]
    out = []
    for c in d["cases"]:
        ids = []
        for k in c["identities"]:
            i = pool[k]
            ids.append((bytes.fromhex(i["ser"]), Identity(i["mspid"], bytes.fromhex(i["pub"]), True,
                                                          bytes.fromhex(i["id_digest"]), roles=i["roles"])))
        ccs = {}
        for ns, v in c["chaincodes"].items():
            colls = v["collections"]
            ccs[ns] = dict(policy=bytes.fromhex(v["policy"]),
                           collections=None if colls is None else
                           {k: (bytes.fromhex(x) if x else None) for k, x in colls.items()})
        kvmeta = {(ns, coll, bytes.fromhex(k)): bytes.fromhex(vp) for ns, coll, k, vp in c["kvmeta"]}
        out.append(dict(c, identities=ids, chaincodes=ccs, kvmeta=kvmeta, block=bytes.fromhex(c["block"])))
    return out


def matches(code, exp):
    return code != 0 if exp == "not_valid" else code == exp


# ------------------------------------------------------------------ synthetic blocks
VP = "VALIDATION_PARAMETER"


def _entries(md):
    return b"".join(f_msg(2, f_str(1, k) + f_bytes(2, v)) for k, v in md.items())


def _spe_any(mspids):
    return f_msg(2, blocks.n_out_of(1, [blocks.signed_by(i) for i in range(len(mspids))])) + \
        b"".join(f_msg(3, blocks.msp_role_principal(m)) for m in mspids)


def make_sbe_block(net, ntx, seed, number=1, coll="pvt1", nkeys=12, vp_keys=6, garbage_vp=False, prefix="k"):
    """A block of namespace mycc over a small key space (public keys k0.. and the same names in
    collection `coll`, by key hash): value writes, metadata writes setting or clearing a key's
    VALIDATION_PARAMETER (one org's members; with garbage_vp also bytes that do not unmarshal),
    endorser sets of 1-3 orgs so that the chaincode EP and the parameters hold or fail; and the
    committed state's parameters (one org / all orgs).  prefix: the key names' prefix (blocks of a
batch over disjoint key spaces).  Returns (block, kvmeta)."""
    rng = random.Random(seed)
    orgs = sorted({p.mspid for ps in net.org_peers for p in ps})
    all_orgs = f_msg(2, blocks.n_out_of(len(orgs), [blocks.signed_by(i) for i in range(len(orgs))])) + \
        b"".join(f_msg(3, blocks.msp_role_principal(m)) for m in orgs)
    kvmeta = {}
    for _ in range(vp_keys):
        k = ("%s%d" % (prefix, rng.randrange(nkeys))).encode()
        vp = _spe_any([rng.choice(orgs)]) if rng.random() < 0.8 else all_orgs
        kvmeta[("mycc", "", k) if rng.random() < 0.5 else ("mycc", coll, hashlib.sha256(k).digest())] = vp
    rws = []
    for _ in range(ntx):
        kind = rng.choice(["w", "w", "md", "pw", "pmd", "w2", "none"])
        keys = ["%s%d" % (prefix, rng.randrange(nkeys)) for _ in range(1 + (kind == "w2"))]
        r = rng.random()
        md = {} if r < 0.2 else {VP: _spe_any([rng.choice(orgs)])}
        if garbage_vp and r > 0.9:
            md = {VP: b"\xff\x01garbage"}
        kv, colls = b"", []
        if kind in ("w", "w2"):
            kv = blocks.kv_rwset([], [(k, b"v", False) for k in keys])
        elif kind == "md":
            kv = f_msg(4, f_str(1, keys[0]) + _entries(md))
        elif kind == "pw":
            colls = [(coll, blocks.hashed_rwset([], [(hashlib.sha256(keys[0].encode()).digest(), b"\x01" * 32, False)]))]
        elif kind == "pmd":
            colls = [(coll, f_msg(3, f_bytes(1, hashlib.sha256(keys[0].encode()).digest()) + _entries(md)))]
        rws.append(blocks.tx_rwset([("mycc", kv, colls)]))
    blk, _, _ = blocks.make_block(net, ntx, number=number, seed=seed, faults=(), rwsets=rws,
                                  endorse_dist=((1, 0.3), (2, 0.4), (3, 0.3)))
    return blk, kvmeta
