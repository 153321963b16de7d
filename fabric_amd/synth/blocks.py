"""Synthetic Fabric blocks (BASELINE configs C2 / C5 shapes).

A Network holds the MSPs (one CA per org, one endorsing peer per org, a pool of client
identities), the channel name and the chaincode definitions (ValidationInfo: plugin "vscc"
+ ApplicationPolicy bytes).  make_block() builds a common.Block of endorser transactions
exactly as a Fabric client/peer would (protoutil CreateSignedTx shape): every signature is an
OpenSSL ECDSA-P256 low-S signature over SHA-256 of the bytes Fabric signs.

Each transaction carries the generator's LABEL -- the validation code the injected fault must
produce in the reference (a generation-time fact, independent of the oracle):
  clean -> 0, bad creator sig -> 4, one bad endorsement of 3 -> 0, policy unsatisfied -> 10,
  duplicate txid -> 9, bad txid -> 8, bad proposal hash -> 5, epoch != 0 -> 3,
  unknown chaincode -> 25, two actions -> 5, unknown creator MSP -> 4, high-S creator -> 4,
  events with other chaincode id -> 255, corrupt envelope bytes -> None (oracle decides).

Wire encoding is hand-rolled proto3 (field numbers: SURVEY.md Appendix B, checked against
vendor/github.com/hyperledger/fabric-protos-go).
"""
import hashlib
import random

from . import EdKey, Key, Key384, ed25519_sign_batch, make_cert, make_cert_ed25519, make_cert_p384, sign384, sign_batch

# ------------------------------------------------------------------ proto3 encoding


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def f_bytes(num: int, b: bytes) -> bytes:
    """length-delimited field; proto3 omits empty bytes/strings/messages-by-bytes"""
    if not b:
        return b""
    return _varint(num << 3 | 2) + _varint(len(b)) + b


def f_msg(num: int, b: bytes) -> bytes:
    """embedded message: present even when empty"""
    return _varint(num << 3 | 2) + _varint(len(b)) + b


def f_str(num: int, s: str) -> bytes:
    return f_bytes(num, s.encode())


def f_varint(num: int, v: int) -> bytes:
    if v == 0:
        return b""
    return _varint(num << 3) + _varint(v)


# ------------------------------------------------------------------ messages

def serialized_identity(mspid: str, pem: bytes) -> bytes:
    return f_str(1, mspid) + f_bytes(2, pem)


def msp_role_principal(mspid: str, role: int = 0) -> bytes:
    role_bytes = f_str(1, mspid) + f_varint(2, role)
    return f_varint(1, 0) + f_bytes(2, role_bytes)  # classification ROLE = 0


def signed_by(i: int) -> bytes:
    return _varint(1 << 3) + _varint(i)  # oneof: encoded even when 0


def n_out_of(n: int, rules) -> bytes:
    return f_msg(2, f_varint(1, n) + b"".join(f_msg(2, r) for r in rules))


def out_of_policy(n: int, mspids) -> bytes:
    """ApplicationPolicy{signature_policy: OutOf(n, [m.member for m in mspids])}
    (common/policydsl/policydsl_builder.go SignedByNOutOfGivenRole shape)."""
    spe = f_varint(1, 0) + f_msg(2, n_out_of(n, [signed_by(i) for i in range(len(mspids))])) + \
        b"".join(f_msg(3, msp_role_principal(m)) for m in mspids)
    return f_msg(1, spe)


def _kvread(k, ver) -> bytes:
    v = b"" if ver is None else f_msg(2, f_varint(1, ver[0]) + f_varint(2, ver[1]))
    return f_str(1, k) + v


def range_query_info(start, end, exhausted, raw=None, merkle=None) -> bytes:
    """RangeQueryInfo{start_key, end_key, itr_exhausted, raw_reads: QueryReads{kv_reads} (raw:
    [(key, ver|None)]), reads_merkle_hashes: QueryReadsMerkleSummary (merkle: (max_degree,
    max_level, [hashes]))} -- rwsetutil.SetRawReads / SetMerkelSummary shapes"""
    out = f_str(1, start) + f_str(2, end) + f_varint(3, 1 if exhausted else 0)
    if raw is not None:
        out += f_msg(4, b"".join(f_msg(1, _kvread(k, v)) for k, v in raw))
    if merkle is not None:
        deg, lvl, hashes = merkle
        out += f_msg(5, f_varint(1, deg) + f_varint(2, lvl) + b"".join(f_msg(3, h) for h in hashes))
    return out


def _meta_entries() -> bytes:
    """KVMetadataEntry{name "VALIDATION_PARAMETER", value}: a key-level endorsement policy slot"""
    return f_msg(2, f_str(1, "VALIDATION_PARAMETER") + f_bytes(2, b"x"))


def kv_rwset(reads, writes, rqs=(), meta=()) -> bytes:
    """KVRWSet{reads 1, range_queries_info 2 (rqs: range_query_info bytes), writes 3,
    metadata_writes 4 (meta: keys)}"""
    out = b""
    for k, ver in reads:
        out += f_msg(1, _kvread(k, ver))
    for q in rqs:
        out += f_msg(2, q)
    for k, val, is_del in writes:
        out += f_msg(3, f_str(1, k) + f_varint(2, 1 if is_del else 0) + f_bytes(3, val))
    for k in meta:
        out += f_msg(4, f_str(1, k) + _meta_entries())
    return out


def hashed_rwset(reads, writes, meta=()) -> bytes:
    """HashedRWSet{hashed_reads: KVReadHash{key_hash, version}, hashed_writes: KVWriteHash{key_hash,
    is_delete, value_hash}}: reads [(key_hash, ver|None)], writes [(key_hash, value_hash, is_delete)]"""
    out = b""
    for k, ver in reads:
        v = b"" if ver is None else f_msg(2, f_varint(1, ver[0]) + f_varint(2, ver[1]))
        out += f_msg(1, f_bytes(1, k) + v)
    for k, vh, is_del in writes:
        out += f_msg(2, f_bytes(1, k) + f_varint(2, 1 if is_del else 0) + f_bytes(3, vh))
    for k in meta:
        out += f_msg(3, f_bytes(1, k) + _meta_entries())
    return out


def tx_rwset(ns_sets) -> bytes:
    """TxReadWriteSet{data_model KV, ns_rwset: [(ns, kvrwset_bytes[, [(collection, hashed_rwset_bytes)]])]}"""
    out = b""
    for ns_set in ns_sets:
        ns, rw = ns_set[0], ns_set[1]
        colls = b"".join(f_msg(3, f_str(1, c) + f_bytes(2, h)) for c, h in (ns_set[2] if len(ns_set) > 2 else ()))
        out += f_msg(2, f_str(1, ns) + f_bytes(2, rw) + colls)
    return out


def chaincode_id(name: str, version: str = "") -> bytes:
    return f_str(2, name) + f_str(3, version)


# ------------------------------------------------------------------ network

class Identity:
    """key: synth.Key (P-256) or synth.EdKey (Ed25519, config C5)."""

    def __init__(self, key, mspid: str, pem: bytes, role: str, hash_family: str = "SHA2"):
        self.key, self.mspid, self.pem, self.role = key, mspid, pem, role
        self.hash_family = hash_family  # the MSP's SignatureHashFamily (identities.go:219-227)
        self.kind = getattr(key, "kind", "p256")
        self.serialized = serialized_identity(mspid, pem)
        der = _pem_to_der(pem)
        self.id_digest = hashlib.sha256(der).digest()  # identity Id = hex(SHA-256(cert.Raw))


def verify_digest(ident, msg: bytes) -> bytes:
    """what identity.Verify hashes msg to: SHA3-256 for an MSP whose hash family is SHA3"""
    return hashlib.sha3_256(msg).digest() if ident.hash_family == "SHA3" else hashlib.sha256(msg).digest()


def _pem_to_der(pem: bytes) -> bytes:
    import base64
    body = pem.split(b"-----BEGIN CERTIFICATE-----")[1].split(b"-----END CERTIFICATE-----")[0]
    return base64.b64decode(b"".join(body.split()))


class Network:
    """orgs: number of MSPs; clients: client identities (spread over the orgs);
    peers_per_org: endorsing peers per org; ed25519_frac / ed25519_peers: share of the clients
    and number of the peers that hold Ed25519 keys (config C5, "Fabric v3" identities)."""

    def __init__(self, seed=3, orgs=3, clients=100, channel="testchannel", policy_n=2, pems=None,
                 peers_per_org=1, ed25519_frac=0.0, ed25519_peers=0, hash_families=None, p384_clients=0,
                 p384_peers=0):
        """pems: certificates exported by another process (Network.export_pems()) -- X.509
        signatures are randomised, so multi-process users share one set of certificates.
        hash_families: {mspid: "SHA3"} -- that MSP's identities sign SHA3-256 digests (its
        channel config must say so: chanconfig.make_config(hash_families=...))."""
        self.seed, self.channel, self.policy_n = seed, channel, policy_n
        self.hash_families = dict(hash_families or {})
        _pem_iter = iter(pems) if pems is not None else None
        sel = random.Random(seed * 7919 + 17)

        # which identities hold Ed25519 keys: ed25519_frac of the clients, ed25519_peers peers
        npeer = orgs * peers_per_org
        kc = int(round(ed25519_frac * clients))
        ed_clients = set(sel.sample(range(clients), kc)) if kc else set()
        ed_peers = set(sel.sample(range(npeer), min(ed25519_peers, npeer))) if ed25519_peers else set()
        # P-384 identities (round 6): the first p384_clients clients and p384_peers peers not drawn above
        p384_c = set([c for c in range(clients) if c not in ed_clients][:p384_clients])
        p384_p = set([q for q in range(npeer) if q not in ed_peers][:p384_peers])

        def cert(*a):  # reuse exported certificates in order
            return next(_pem_iter) if _pem_iter is not None else make_cert(*a)

        def ed_cert(*a):
            return next(_pem_iter) if _pem_iter is not None else make_cert_ed25519(*a)
        self.mspids = [f"Org{i + 1}MSP" for i in range(orgs)]
        self.cas, self.peers, self.clients = [], [], []
        self.org_peers = [[] for _ in range(orgs)]
        for o, m in enumerate(self.mspids):
            self.cas.append(Key(seed, 10_000 + o))
        for o, m in enumerate(self.mspids):
            for q in range(peers_per_org):
                idx = o * peers_per_org + q
                name = f"peer{q}.org{o + 1}"
                if idx in ed_peers:
                    pk = EdKey(seed, 20_000 + idx)
                    pem = ed_cert(pk, self.cas[o], name, m, f"ca.org{o + 1}", 100 + idx)
                elif idx in p384_p:
                    pk = Key384(seed, 20_000 + idx)
                    pem = next(_pem_iter) if _pem_iter is not None else make_cert_p384(
                        pk, self.cas[o], name, m, f"ca.org{o + 1}", 100 + idx)
                else:
                    pk = Key(seed, 20_000 + idx)
                    pem = cert(pk, self.cas[o], name, m, f"ca.org{o + 1}", False, 100 + idx)
                ident = Identity(pk, m, pem, "peer")
                self.peers.append(ident)
                self.org_peers[o].append(ident)
        for c in range(clients):
            o = c % orgs
            name = f"user{c}.org{o + 1}"
            if c in ed_clients:
                ck = EdKey(seed, 30_000 + c)
                pem = ed_cert(ck, self.cas[o], name, self.mspids[o], f"ca.org{o + 1}", 1000 + c)
            elif c in p384_c:
                ck = Key384(seed, 30_000 + c)
                pem = next(_pem_iter) if _pem_iter is not None else make_cert_p384(
                    ck, self.cas[o], name, self.mspids[o], f"ca.org{o + 1}", 1000 + c)
            else:
                ck = Key(seed, 30_000 + c)
                pem = cert(ck, self.cas[o], name, self.mspids[o], f"ca.org{o + 1}", False, 1000 + c)
            self.clients.append(Identity(ck, self.mspids[o], pem, "client"))
        # an identity from an MSP the channel does not know (deserialization fails)
        rk = Key(seed, 40_000)
        rogue_ca = Key(seed, 40_001)
        self.rogue = Identity(rk, "RogueMSP", cert(rk, rogue_ca, "rogue", "RogueMSP", "ca.rogue", False, 7),
                              "client")
        # an identity claiming Org1MSP but with a cert from a foreign CA: deserializes (known
        # MSP) but fails Validate (not issued by Org1's CA)
        fk = Key(seed, 40_002)
        self.forged = Identity(fk, self.mspids[0], cert(fk, rogue_ca, "forged", self.mspids[0], "ca.rogue",
                                                             False, 8), "peer")
        for ident in self.peers + self.clients + [self.forged]:
            ident.hash_family = self.hash_families.get(ident.mspid, "SHA2")
        self.chaincodes = {"mycc": out_of_policy(policy_n, self.mspids)}

    def export_pems(self):
        return [i.pem for i in self.peers + self.clients] + [self.rogue.pem, self.forged.pem]

    def identities(self):
        """What the MSP layer knows: (serialized, txvalidator.Identity).  RogueMSP is unknown to
        the channel, so it is NOT listed (deserialize error).  Ed25519 identities are listed as
        "undeserializable": the reference's BCCSP x509 key importer accepts only ECDSA/RSA keys
        (vendor/github.com/hyperledger/fabric-lib-go/bccsp/sw/keyimport.go:130-150),
        so DeserializeIdentity fails for them -- creator -> BAD_CREATOR_SIGNATURE, endorser ->
        skipped by SignatureSetToValidIdentities (common/policies/policy.go:363-395).  Role bits
        follow NodeOU classification (peers PEER, clients CLIENT; an invalid identity satisfies
        no role, msp/mspimpl.go:331-376)."""
        from ..txvalidator import Identity
        out = []
        for ident in self.peers + self.clients:
            role_bit = 1 << (3 if ident.role == "peer" else 2)
            if ident.kind == "p384":  # (round 6: verified per item on the GPU)
                out.append((ident.serialized, Identity(ident.mspid, ident.key.pub, True, ident.id_digest, key="p384",
                                                       roles=1 | role_bit, hash_family=ident.hash_family)))
                continue
            if ident.kind != "p256":
                out.append((ident.serialized, Identity(ident.mspid, None, True, ident.id_digest, key="undeserializable")))
                continue
            out.append((ident.serialized, Identity(ident.mspid, ident.key.pub, True, ident.id_digest, roles=1 | role_bit,
                                                   hash_family=ident.hash_family)))
        out.append((self.forged.serialized, Identity(self.forged.mspid, self.forged.key.pub, False,
                                                     self.forged.id_digest, roles=0,
                                                     hash_family=self.forged.hash_family)))
        return out

    def identities_legacy(self):
        """the round-1 registration: (serialized, mspid, pubkey64, valid, id_digest), P-256 only"""
        out = []
        for ident in self.peers + self.clients:
            if ident.kind == "p256":
                out.append((ident.serialized, ident.mspid, ident.key.pub, True, ident.id_digest))
        out.append((self.forged.serialized, self.forged.mspid, self.forged.key.pub, False, self.forged.id_digest))
        return out


# ------------------------------------------------------------------ blocks

FAULTS_C2 = (("bad_creator_sig", 0.02), ("one_bad_endorsement", 0.02), ("policy_unsatisfied", 0.02),
             ("dup_txid", 0.005))
EXPECTED = {"clean": 0, "bad_creator_sig": 4, "one_bad_endorsement": 0, "policy_unsatisfied": 10,
            "dup_txid": 9, "bad_txid": 8, "bad_proposal_hash": 5, "bad_epoch": 3, "unknown_cc": 25,
            "two_actions": 5, "rogue_creator": 4, "high_s_creator": 4, "dup_endorser": 10,
            "forged_endorser": 10, "event_other_cc": 255, "bad_payload": 2, "no_sig": 4,
            "corrupt": None, "dup_txid_prev": 9, "ed25519_creator": 4, "endorse_short": 10}
# labels whose code depends on the endorsement set (re-derived for C5-style networks)
_ENDORSE_LABELS = ("clean", "one_bad_endorsement", "dup_txid")


class _Tx:
    pass


def make_block(net: Network, ntx: int, number: int = 1, seed: int = 0, faults=FAULTS_C2, endorse_dist=((2, 0.6), (3, 0.4)),
               reads=4, writes=4, value_len=200, threads=8, prev_hash=b"\x00" * 32, force=None, ns="mycc",
               key_space=1_000_000, reuse=None, out_txs=None, collections=None, rwsets=None):
    """Returns (block_bytes, labels list, envelopes list).
    reuse: {tx index: (creator Identity, nonce)} -> that tx re-uses an earlier txid (label
    'dup_txid_prev'); out_txs: list that receives the generated tx objects; collections: names
    of private-data collections -- every tx then also writes one key hash into one of them
    (chosen per tx), so its namespace checks that collection's endorsement policy (the codes
    are then the oracle's to decide, labels stay as generated); rwsets: the TxReadWriteSet bytes
    of each tx instead of the generated ones (codes then the oracle's to decide), or a function
    of the drawn labels returning them."""
    rng = random.Random((net.seed << 20) ^ (number << 4) ^ seed)
    txs = []
    fault_names = [f for f, _ in faults]
    cum = []
    acc = 0.0
    for _, p in faults:
        acc += p
        cum.append(acc)
    for i in range(ntx):
        t = _Tx()
        t.index = i
        u = rng.random()
        t.label = "clean"
        for name, c in zip(fault_names, cum):
            if u < c:
                t.label = name
                break
        if force is not None and force[i] is not None:
            t.label = force[i]
        t.creator = net.rogue if t.label == "rogue_creator" else rng.choice(net.clients)
        if t.creator.kind not in ("p256", "p384") and t.label in ("clean", "one_bad_endorsement", "policy_unsatisfied",
                                                                   "bad_creator_sig", "high_s_creator"):
            t.label = "ed25519_creator"  # DeserializeIdentity fails
        t.nonce = bytes(rng.getrandbits(8) for _ in range(24))
        if reuse and i in reuse:
            t.creator, t.nonce = reuse[i]
            t.label = "dup_txid_prev"
        if t.label == "dup_txid":
            # (the first tx of a block has no earlier tx to repeat: it stays unique, so "clean" --
            # labelling it 9 made 2-rank bench runs report 3 parity mismatches per 32k tx)
            clean = [x for x in txs if x.label == "clean"] if i > 0 else []
            if clean:
                src = clean[rng.randrange(len(clean))]
                t.creator, t.nonce = src.creator, src.nonce
            else:
                # relabelled clean: the creator-kind rule above applies again (an Ed25519 creator
                # cannot be a clean transaction: DeserializeIdentity fails, code 4)
                t.label = "clean" if t.creator.kind in ("p256", "p384") else "ed25519_creator"
        r = rng.random()
        ne, accp = endorse_dist[-1][0], 0.0
        for e, p in endorse_dist:
            accp += p
            if r < accp:
                ne = e
                break
        norg = len(net.org_peers)

        def peer_of(o):
            ps = net.org_peers[o]
            return ps[0] if len(ps) == 1 else rng.choice(ps)
        orgs = rng.sample(range(norg), min(ne, norg))
        t.endorsers = [peer_of(o) for o in orgs]
        if t.label == "policy_unsatisfied":
            t.endorsers = t.endorsers[:1]
        if t.label == "dup_endorser":
            t.endorsers = [t.endorsers[0], t.endorsers[0]]
        if t.label == "forged_endorser":
            t.endorsers = [t.endorsers[0], net.forged]
        need = getattr(net, "policy_n", 2) + 1
        if t.label == "one_bad_endorsement" and len(t.endorsers) < need:
            orgs = rng.sample(range(norg), min(need, norg))
            t.endorsers = [peer_of(o) for o in orgs]
        t.bad_endorsement = rng.randrange(len(t.endorsers)) if t.label == "one_bad_endorsement" else -1
        if t.label in _ENDORSE_LABELS:
            # distinct orgs among the P-256 endorsers with a good signature (Ed25519 endorsers
            # fail DeserializeIdentity and are skipped) must satisfy OutOf(policy_n, orgs)
            good = {e.mspid for j, e in enumerate(t.endorsers) if e.kind in ("p256", "p384") and j != t.bad_endorsement}
            if len(good) < getattr(net, "policy_n", 2):
                t.label = "endorse_short"
        t.reads = [(f"k{rng.randrange(key_space):07d}", (rng.randrange(1, 1000), rng.randrange(500)))
                   for _ in range(reads)]
        t.writes = [(f"k{rng.randrange(key_space):07d}", bytes(rng.getrandbits(8) for _ in range(value_len)), False)
                    for _ in range(writes)]
        t.ccpp = f_bytes(1, bytes(rng.getrandbits(8) for _ in range(128)))  # ChaincodeProposalPayload{input}
        t.ts = (1_700_000_000 + number * 1000 + i, rng.randrange(10 ** 9))
        txs.append(t)

    # rwsets may be a function of the labels just drawn (the end-to-end pipeline generator
    # derives each transaction's MVCC reads from which earlier transactions will be valid)
    if callable(rwsets):
        rwsets = rwsets([t.label for t in txs])
    # pass 1: headers, proposal response payloads, endorsement digests
    e_privs, e_digests, e_refs = [], [], []
    p384_refs = []  # (tx, endorsement index, DER signature) of P-384 endorsers
    ed_privs, ed_msgs, ed_refs = [], [], []
    for t in txs:
        txid = hashlib.sha256(t.nonce + t.creator.serialized).hexdigest()
        if t.label == "bad_txid":
            txid = txid[:-1] + ("0" if txid[-1] != "0" else "1")
        ccname = "othercc" if t.label == "unknown_cc" else ns
        ext = f_msg(2, chaincode_id(ccname))  # ChaincodeHeaderExtension{chaincode_id}
        ts = f_msg(3, f_varint(1, t.ts[0]) + f_varint(2, t.ts[1]))
        t.chdr = f_varint(1, 3) + ts + f_str(4, net.channel) + f_str(5, txid) + \
            f_varint(6, 1 if t.label == "bad_epoch" else 0) + f_bytes(7, ext)
        t.shdr = f_bytes(1, t.creator.serialized) + f_bytes(2, t.nonce)
        ph = hashlib.sha256(t.chdr + t.shdr + t.ccpp).digest()
        if t.label == "bad_proposal_hash":
            ph = bytes([ph[0] ^ 1]) + ph[1:]
        if collections:
            t.coll = collections[rng.randrange(len(collections))]
            kh = hashlib.sha256(b"%d/%d/%s" % (number, len(e_refs) + len(ed_refs), t.nonce)).digest()
            rw = tx_rwset([(ccname, kv_rwset(t.reads, t.writes),
                            [(t.coll, hashed_rwset([], [(kh, hashlib.sha256(kh).digest(), False)]))])])
        else:
            rw = tx_rwset([(ccname, kv_rwset(t.reads, t.writes))])
        if rwsets is not None:
            rw = rwsets[t.index]
        events = b""
        if t.label == "event_other_cc":
            events = f_str(1, "someothercc") + f_str(3, "ev")
        cca = f_bytes(1, rw) + f_bytes(2, events) + f_msg(3, f_varint(1, 200)) + f_msg(4, chaincode_id(ccname, "1.0"))
        t.prp = f_bytes(1, ph) + f_bytes(2, cca)
        for j, e in enumerate(t.endorsers):
            if e.kind == "p384":
                p384_refs.append((t, j, sign384(e.key, verify_digest(e, t.prp + e.serialized))))
                continue
            if e.kind != "p256":
                ed_privs.append(e.key.priv)
                ed_msgs.append(t.prp + e.serialized)
                ed_refs.append((t, j))
                continue
            e_privs.append(e.key.priv)
            e_digests.append(verify_digest(e, t.prp + e.serialized))
            e_refs.append((t, j))
    esigs = sign_batch(b"".join(e_privs), b"".join(e_digests), len(e_privs), threads=threads) if e_privs else []
    for t in txs:
        t.esigs = [None] * len(t.endorsers)
    for (t, j), s in list(zip(e_refs, esigs)) + list(zip(ed_refs, ed25519_sign_batch(b"".join(ed_privs), ed_msgs))) + \
            [((t, j), s) for t, j, s in p384_refs]:
        if j == t.bad_endorsement:
            s = s[:10] + bytes([s[10] ^ 0x55]) + s[11:]
        t.esigs[j] = s

    # pass 2: assemble payloads; creator signatures
    c_privs, c_digests = [], []
    for t in txs:
        ends = b"".join(f_msg(2, f_bytes(1, e.serialized) + f_bytes(2, s)) for e, s in zip(t.endorsers, t.esigs))
        cea = f_bytes(1, t.prp) + ends
        cap = f_bytes(1, t.ccpp) + f_msg(2, cea)
        action = f_msg(1, f_bytes(1, t.shdr) + f_bytes(2, cap))
        if t.label == "two_actions":
            action = action + action
        hdr = f_bytes(1, t.chdr) + f_bytes(2, t.shdr)
        t.payload = f_msg(1, hdr) + f_bytes(2, action)
        if t.label == "bad_payload":
            t.payload = t.payload[:-3]  # truncated -> Payload unmarshal error
        if t.creator.kind == "p256":
            c_privs.append(t.creator.key.priv)
            c_digests.append(verify_digest(t.creator, t.payload))
    csigs = sign_batch(b"".join(c_privs), b"".join(c_digests), len(c_privs), threads=threads,
                       high_s=False) if c_privs else []
    ed_tx = [t for t in txs if t.creator.kind == "ed25519"]
    ed_sigs = iter(ed25519_sign_batch(b"".join(t.creator.key.priv for t in ed_tx), [t.payload for t in ed_tx]))
    p_sigs = iter(csigs)
    csigs = [next(p_sigs) if t.creator.kind == "p256" else
             sign384(t.creator.key, verify_digest(t.creator, t.payload)) if t.creator.kind == "p384" else next(ed_sigs)
             for t in txs]
    envs = []
    for t, s in zip(txs, csigs):
        if t.label == "bad_creator_sig":
            s = s[:12] + bytes([s[12] ^ 0x21]) + s[13:]
        if t.label == "high_s_creator":
            from .workloads import _der_int, _der_rs, N
            from . import N384, der_encode_int
            r_, s_ = _der_rs(s)
            if t.creator.kind == "p384":
                s = der_encode_int(r_, N384 - s_)
            else:
                body = _der_int(r_) + _der_int(N - s_)
                s = b"\x30" + bytes([len(body)]) + body
        if t.label == "no_sig":
            s = b""
        env = f_bytes(1, t.payload) + f_bytes(2, s)
        if t.label == "corrupt":
            b = bytearray(env)
            for _ in range(3):
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            env = bytes(b)
        envs.append(env)
    labels = [t.label for t in txs]
    if out_txs is not None:
        out_txs.extend(txs)
    data_hash = hashlib.sha256(b"".join(envs)).digest()
    header = f_varint(1, number) + f_bytes(2, prev_hash) + f_bytes(3, data_hash)
    data = b"".join(f_msg(1, e) for e in envs) if envs else b""
    metadata = b"".join(f_msg(1, b"") for _ in range(5))
    block = f_msg(1, header) + f_msg(2, data) + f_msg(3, metadata)
    return block, labels, envs


def config_block(net: Network, number: int, seed: int = 0, bad_sig=False, prev_hash=b"\x00" * 32):
    """A block holding one CONFIG transaction (HeaderType_CONFIG = 1), signed by a client of the
    network (orderers cut config transactions into blocks of their own): the envelope passes
    ValidateTransaction and reaches ChannelResources.Apply (validator.go:397-420) unless bad_sig.
    Payload.data is a stand-in ConfigEnvelope (the engine never decodes it)."""
    rng = random.Random((net.seed << 20) ^ (number << 4) ^ seed ^ 0xC0F)
    creator = next(c for c in net.clients if c.kind == "p256")
    nonce = bytes(rng.getrandbits(8) for _ in range(24))
    txid = hashlib.sha256(nonce + creator.serialized).hexdigest()
    chdr = f_varint(1, 1) + f_msg(3, f_varint(1, 1_700_000_000 + number)) + f_str(4, net.channel) + f_str(5, txid)
    shdr = f_bytes(1, creator.serialized) + f_bytes(2, nonce)
    payload = f_msg(1, f_bytes(1, chdr) + f_bytes(2, shdr)) + f_bytes(2, f_msg(1, f_msg(1, f_varint(1, number))))
    sig = sign_batch(creator.key.priv, verify_digest(creator, payload), 1, threads=1, high_s=False)[0]
    if bad_sig:
        sig = sig[:12] + bytes([sig[12] ^ 0x21]) + sig[13:]
    env = f_bytes(1, payload) + f_bytes(2, sig)
    data_hash = hashlib.sha256(env).digest()
    header = f_varint(1, number) + f_bytes(2, prev_hash) + f_bytes(3, data_hash)
    metadata = b"".join(f_msg(1, b"") for _ in range(5))
    return f_msg(1, header) + f_msg(2, f_msg(1, env)) + f_msg(3, metadata)


def header_hash(number: int, prev_hash: bytes, envs) -> bytes:
    """BlockHeaderHash of a generated block (protoutil/blockutils.go:48-67: SHA-256 of the DER
    SEQUENCE{INTEGER number, OCTET STRING previous_hash, OCTET STRING data_hash}), used to
    chain generated blocks through Header.PreviousHash."""
    def dlen(n):
        if n < 128:
            return bytes([n])
        b = n.to_bytes((n.bit_length() + 7) // 8, "big")
        return bytes([0x80 | len(b)]) + b
    nb = number.to_bytes(max(1, (number.bit_length() + 7) // 8), "big")
    if nb[0] & 0x80:
        nb = b"\x00" + nb
    dh = hashlib.sha256(b"".join(envs)).digest()
    body = b"\x02" + dlen(len(nb)) + nb + b"\x04" + dlen(len(prev_hash)) + prev_hash + b"\x04" + dlen(32) + dh
    return hashlib.sha256(b"\x30" + dlen(len(body)) + body).digest()


def expected_codes(labels):
    """Generator-side expectation (None where the fault's effect is left to the oracle).
    dup_txid: the later VALID duplicate gets 9 (validator.go:279-295)."""
    return [EXPECTED[l] for l in labels]
