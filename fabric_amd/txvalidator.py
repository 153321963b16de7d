"""Python mirror of the reference's committer interfaces over the HIP engine.

  TxValidator.validate(block)  ~ core/committer/txvalidator/v20/validator.go:180
                                 (TxValidator.Validate; returns TxValidationFlags)
  setup_channel(engine, ...)   ~ the channel resources the reference validator is wired with
                                 (MSP manager identities, lifecycle ValidationInfo, ledger)

There is no CPU fallback: FGV_EUNSUPPORTED / device errors propagate as exceptions so the
caller (a Go shim in production) runs the reference code for that batch.
"""
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import CC_COLLECTIONS_KNOWN, CC_KEY_LEVEL_EP, Engine, Unsupported  # noqa: F401


@dataclass
class Identity:
    """What the peer's MSP layer knows of one SerializedIdentity (fgv_identity_info):
    key "p256" | "p384" | "other" | "undeserializable"; hash_family of its MSP; roles: bit r set
    iff msp.SatisfiesPrincipal(id, ROLE{mspid, r}) (None = unknown); ous: GetOrganizationalUnits
    as [(OU identifier, certifiers identifier bytes)] (None = unknown)."""
    mspid: str
    pub: Optional[bytes]
    valid: bool
    id_digest: bytes
    key: str = "p256"
    hash_family: str = "SHA2"
    roles: Optional[int] = None
    ous: Optional[list] = None


def roles_want_comb(roles):
    """fgv_roles_want_comb (fgv_internal.h): anything but a definite client (CLIENT without
    ADMIN / PEER / ORDERER)"""
    return roles is None or not (roles & (1 << 2)) or bool(roles & ((1 << 1) | (1 << 3) | (1 << 4)))


def _as_identity(entry):
    """(serialized, Identity-like) or the round-1 (serialized, mspid, pub | None, valid, id_digest)"""
    if len(entry) == 2:
        return entry[0], entry[1]
    ser, mspid, pub, valid, dig = entry
    return ser, Identity(mspid, pub, valid, dig, key="p256" if pub is not None else "other")


def setup_channel(engine: Engine, channel: str, identities, chaincodes, committed_txids=(), config=None, msps=(),
                  kvmeta=None, hot_clients=False):
    """identities: iterable of (serialized, Identity) or (serialized, mspid, pubkey64 | None,
    valid, id_digest).  chaincodes: ns -> ApplicationPolicy bytes, or a dict {policy,
    plugin="vscc", collections=None | {name: EP bytes | None}, sbe=False}.  config: the channel's
    common.Config bytes (channel policies, MSPs, application orgs); msps: further MSP ids.
    kvmeta: {(ns, coll, key bytes): VALIDATION_PARAMETER bytes} of the committed state.
    hot_clients: register client keys with comb tables too (a peer whose clients are known to sign
    often: the steady state promotion by use reaches anyway)."""
    engine.channel_init(channel)
    if config is not None:
        engine.channel_config(config)
    for m in msps:
        engine.msp_declare(m)
    identities = [_as_identity(e) for e in identities]
    # every P-256 public key first, in one fgv_keys_register_tiered call: the keys that get comb
    # tables (fgv_roles_want_comb: peers, orderers, admins, unknown roles) are built by batched
    # k_keytab launches (up to KT_BUILD_KEYS keys each), the variable-base tables of the client
    # keys by one k_keyprep launch -- instead of one launch and one synchronisation per identity
    # below.  Client keys start on the variable-base kernels and are promoted by use.
    keyed = [i for _s, i in identities if i.key == "p256" and i.pub is not None]
    if keyed:
        engine.keys_register(np.frombuffer(b"".join(bytes(i.pub) for i in keyed), dtype=np.uint8),
                             hot=[hot_clients or roles_want_comb(i.roles) for i in keyed])
    for ser, i in identities:
        engine.msp_register_identity(ser, i.key, i.pub, i.valid, i.id_digest, roles=i.roles,
                                     hash_family=i.hash_family)
        if getattr(i, "ous", None) is not None:
            engine.msp_identity_ous(ser, i.ous)
    for ns, d in chaincodes.items():
        if not isinstance(d, dict):
            engine.chaincode_define(ns, d)
            continue
        colls = d.get("collections")
        flags = (CC_COLLECTIONS_KNOWN if colls is not None else 0) | (CC_KEY_LEVEL_EP if d.get("sbe") else 0)
        engine.chaincode_define(ns, d.get("policy") or b"", plugin=d.get("plugin", "vscc"), flags=flags)
        for name, ep in (colls or {}).items():
            engine.collection_define(ns, name, ep or b"")
    for (ns, coll, key), vp in (kvmeta or {}).items():
        engine.kvmeta_set(ns, coll, key, vp)
    if committed_txids:
        engine.ledger_add_txids(list(committed_txids))


class TxValidator:
    def __init__(self, engine: Engine):
        self.engine = engine

    def validate(self, block: bytes):
        return self.engine.validate_blocks([block])[0]

    def validate_many(self, blocks, d_blocks=None):
        return self.engine.validate_blocks(blocks, d_blocks)
