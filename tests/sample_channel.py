"""The channel model of the reference's v2.0 sample ledger (tests/golden/sample_ledgers.*,
ledger "v20_testchannel": 3 application orgs with NodeOUs, default v2 policies
/Channel/Application/Endorsement = MAJORITY Endorsement, org Endorsement = OR('OrgN.peer'),
_lifecycle approvals writing implicit collections, marbles / marbles-private).

What a peer's MSP layer and lifecycle cache would hand the engine, built from the blocks
themselves (test infrastructure):
  * channel config: the last config block's ConfigEnvelope.config (block 4);
  * identities: every creator / endorser certificate in the blocks, valid (the reference
    committed them), role bits from the MSP's NodeOU identifiers (msp/mspimpl.go:331-376,
    607-660 semantics: MEMBER = valid, CLIENT/PEER/ORDERER by OU, ADMIN by OU or admin list);
  * chaincode definitions as of each block: _lifecycle -> the LifecycleEndorsement reference
    (deployedcc_infoprovider.go:314-340), others from the ValidationInfo / Collections that
    earlier VALID _lifecycle transactions wrote (namespaces/fields/<cc>/...)."""
import hashlib

from oracle import v20
from oracle.protowire import decode
from tests.test_oracle_ledgers import ledgers
from tests.x509min import cert_info, pem_to_der

ROLE_MEMBER, ROLE_ADMIN, ROLE_CLIENT, ROLE_PEER, ROLE_ORDERER = range(5)
LIFECYCLE_POLICY = b"\x12" + bytes([len(b"/Channel/Application/LifecycleEndorsement")]) + \
    b"/Channel/Application/LifecycleEndorsement"  # ApplicationPolicy{channel_config_policy_reference}


def config_of(block):
    env = decode("Envelope", decode("Block", block)["data"]["data"][0])
    pl = decode("Payload", env["payload"])
    raw = pl.get("data")
    # ConfigEnvelope{config = 1}: the Config bytes themselves
    o, cfg = 0, None
    from oracle.protowire import _varint
    while o < len(raw):
        tag, o = _varint(raw, o)
        ln, o = _varint(raw, o)
        if tag == 0x0A:
            cfg = raw[o:o + ln]
        o += ln
    return cfg


def msp_nodeous(config):
    cfg = decode("Config", config)
    model = v20.ChannelModel("x", [], {}, config=config)
    out = {}
    for name, fc in model.config_msps.items():
        n = fc.get("fabric_node_ous") or {}
        ou = {r: (n.get(k) or {}).get("organizational_unit_identifier")
              for r, k in ((ROLE_CLIENT, "client_ou_identifier"), (ROLE_PEER, "peer_ou_identifier"),
                           (ROLE_ADMIN, "admin_ou_identifier"), (ROLE_ORDERER, "orderer_ou_identifier"))}
        out[name] = (bool(n.get("enable")), ou, [pem_to_der(a) if a.startswith(b"-----") else a for a in fc.get("admins", [])])
    del cfg
    return out


def identity_of(ser, nodeous):
    """(serialized, v20.Ident, key bytes) as the MSP layer would register it"""
    sid = decode("SerializedIdentity", ser)
    der = pem_to_der(sid["id_bytes"])
    info = cert_info(der)
    enabled, ou, admins = nodeous[sid["mspid"]]
    roles = 1 << ROLE_MEMBER
    if der in admins:
        roles |= 1 << ROLE_ADMIN
    if enabled:
        for r, name in ou.items():
            if name and name in info["ous"]:
                roles |= 1 << r
    key = {"p256": v20.KEY_P256, "p384": v20.KEY_P384}.get(info["key"], v20.KEY_OTHER)
    return ser, v20.Ident(sid["mspid"], info["pub"] if key == v20.KEY_P256 else None, True,
                          hashlib.sha256(der).digest(), key=key, hash_family="SHA2", roles=roles)


def tx_identities(env_bytes):
    env = decode("Envelope", env_bytes)
    pl = decode("Payload", env["payload"])
    sh = decode("SignatureHeader", pl["header"]["signature_header"])
    out = [sh["creator"]]
    ch = decode("ChannelHeader", pl["header"]["channel_header"])
    if ch.get("type", 0) == 3:
        _, cap = v20.get_action_from_envelope(env_bytes)
        out += [e["endorser"] for e in cap["action"].get("endorsements", [])]
    return out


def lifecycle_updates(env_bytes, defs):
    """apply a VALID _lifecycle transaction's namespaces/fields/<cc>/{ValidationInfo,Collections}"""
    cca, _ = v20.get_action_from_envelope(env_bytes)
    for ns in v20.parse_rwset(cca.get("results")):
        if ns["namespace"] != "_lifecycle":
            continue
        for w in ns["kv"].get("writes", []):
            parts = (w.get("key") or "").split("/")
            if len(parts) != 4 or parts[:2] != ["namespaces", "fields"]:
                continue
            sd = decode("StateData", w.get("value") or b"").get("Bytes") or b""
            d = defs.setdefault(parts[2], {"plugin": "vscc", "policy": b"", "collections": {}})
            if parts[3] == "ValidationInfo":
                vi = decode("ChaincodeValidationInfo", sd)
                d["plugin"] = vi.get("validation_plugin", "")
                d["policy"] = vi.get("validation_parameter") or b""
            elif parts[3] == "Collections":
                d["collections"] = {}
                for c in decode("CollectionConfigPackage", sd).get("config", []):
                    sc = c.get("static_collection_config") or {}
                    d["collections"][sc.get("name", "")] = sc.get("endorsement_policy")


def v20_channel():
    """-> (blocks, config bytes, [(ser, Ident)], defs_before[block number] = chaincode dict)"""
    blocks = ledgers()["v20_testchannel"]
    config = config_of(blocks[4]["block"])
    nodeous = msp_nodeous(config)
    idents, seen = [], set()
    defs_before, defs = {}, {"_lifecycle": {"plugin": "vscc", "policy": LIFECYCLE_POLICY, "collections": {}}}
    for b in blocks:
        data = decode("Block", b["block"])["data"].get("data", [])
        defs_before[b["number"]] = {k: dict(v, collections=dict(v["collections"])) for k, v in defs.items()}
        for i, d in enumerate(data):
            for ser in tx_identities(d):
                if ser not in seen:
                    seen.add(ser)
                    idents.append(identity_of(ser, nodeous))
            if b["number"] >= 5 and b["flags"][i] == 0:
                lifecycle_updates(d, defs)
    return blocks, config, idents, defs_before
