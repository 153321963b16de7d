"""The MSP cache-miss restatement (oracle/msp.py + oracle/x509.py) pinned by the reference's own
MSP test data and assertions (msp/nodeous_test.go, MSP version 1.4.3), and the engine's CPU-side
X.509 parser (fgv_x509_probe, no GPU) against the restatement on the same fixtures plus mutated
certificates.  Fixtures: tests/golden/msp_fixtures.json (tests/golden/make_msp_fixtures.py)."""
import hashlib
import json
import os
import random

import pytest

from oracle import x509 as X
from oracle.msp import MSP, ROLE_ADMIN, ROLE_CLIENT, ROLE_ORDERER, ROLE_PEER
from oracle.protowire import decode
from oracle.v20 import KEY_P256, Unsupported

HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, "golden", "msp_fixtures.json")))


def _msp(rel):
    return MSP(decode("FabricMSPConfig", bytes.fromhex(FX["msps"][rel]["config"])))


def _ident(rel, path):
    m = _msp("msp/testdata/" + rel)
    pem = FX["msps"]["msp/testdata/" + rel]["identities"][path].encode()
    return m.resolve(pem)


def _one(rel, folder):
    ids = FX["msps"]["msp/testdata/" + rel]["identities"]
    keys = [k for k in ids if k.startswith(folder + "/")]
    assert len(keys) == 1, keys
    return _ident(rel, keys[0])


def has(ident, role):
    return bool(ident.roles >> role & 1)


# ---- msp/nodeous_test.go
def test_signing_identity_without_node_ou_is_invalid():  # TestInvalidSigningIdentityNodeOU (v1.4.3)
    i = _one("nodeous2", "signcerts")
    assert i is not None and not i.valid and i.roles == 0


def test_valid_msp_with_node_ou_peer_and_client():  # TestValidMSPWithNodeOU, TestSatisfiesPrincipalPeer/Client
    peer = _one("nodeous3", "signcerts")
    assert peer.valid and has(peer, ROLE_PEER) and not has(peer, ROLE_CLIENT)
    admin = _one("nodeous3", "admincerts")
    assert admin.valid and has(admin, ROLE_CLIENT) and not has(admin, ROLE_PEER)
    assert has(admin, ROLE_ADMIN)  # (listed in admincerts)


def test_node_ou_with_organizational_units():  # TestValidMSPWithNodeOUAndOrganizationalUnits
    assert _one("nodeous6", "signcerts").valid


def test_node_ou_missing_common_ou():  # TestInvalidMSPWithNodeOUAndOrganizationalUnits
    assert not _one("nodeous7", "signcerts").valid
    assert not _one("nodeous7", "admincerts").valid


def test_admin_certifier_mismatch():  # TestInvalidAdminOU: certifiersIdentifier does not match
    assert not _one("nodeous4", "admincerts").valid


def test_admin_by_admin_ou():  # TestSatisfiesPrincipalAdmin
    i = _ident("nodeouadmin", "adm/testadmincert.pem")
    assert i.valid and has(i, ROLE_ADMIN)


@pytest.mark.parametrize("rel", ["nodeouadminclient", "nodeouadminclient2"])
def test_admin_listed_in_admincerts(rel):  # TestAdminInAdmincertsWith143MSP
    pem = FX["msps"]["msp/testdata/" + rel]["identities"]["admincerts/admin.pem"].encode()
    assert "admin" not in X.parse_certificate(X.pem_decode(pem))["ous"]
    assert has(_ident(rel, "admincerts/admin.pem"), ROLE_ADMIN)


def test_orderer_role():  # TestSatisfiesPrincipalOrderer / TestLoad142MSPWithInvalidOrdererConfiguration
    assert has(_one("nodeouorderer", "signcerts"), ROLE_ORDERER)
    for rel in ("nodeouorderer2", "nodeouorderer3"):
        assert not has(_one(rel, "signcerts"), ROLE_ORDERER)


def test_identity_id_is_sha256_of_sanitized_cert():
    """identities.go:48-84: Id = hex(SHA-256(sanitized cert.Raw)); a low-S cert is its own
    sanitization"""
    pem = FX["msps"]["msp/testdata/nodeous3"]["identities"]
    pem = pem[[k for k in pem if k.startswith("signcerts/")][0]].encode()
    c = X.parse_certificate(X.pem_decode(pem))
    i = _one("nodeous3", "signcerts")
    assert i.id_digest == hashlib.sha256(X.sanitized_raw(c)).digest()
    assert i.key == KEY_P256 and i.pub == c["pub"]


def test_ca_certificate_as_identity_is_outside_the_model():
    with pytest.raises(Unsupported):
        _one("nodeous3", "cacerts")


def test_msps_outside_the_model():
    for rel in ("msp/testdata/external",):  # CRL distribution points
        with pytest.raises(Unsupported):
            _msp(rel)


# ---- msp/revocation_test.go (CRLs: oracle/crl.py)
def test_revoked_identity_is_invalid():  # TestRevocation/ValidCRLSignature
    i = _one("revocation", "signcerts")
    assert i is not None and not i.valid and not has(i, 0)


def test_revoked_identity_fails_an_identity_principal():  # TestIdentityPolicyPrincipalAgainstRevokedIdentity
    assert not _one("revocation", "signcerts").valid  # (an IDENTITY principal validates first)


def test_crl_with_a_bad_signature_revokes_nothing():  # TestRevocation/InvalidCRLSignature
    i = _one("revocation2", "signcerts")
    assert i is not None and i.valid


def test_revoked_intermediate_ca_fails_setup():  # TestRevokedIntermediateCA: "CA Certificate is not valid"
    with pytest.raises(Unsupported):
        _msp("msp/testdata/revokedica")


def _der_tlv(tag, body):
    return bytes([tag]) + X._der_len(len(body)) + body


def test_crl_signature_with_a_trailing_integer_still_revokes():  # TestRevocation/MalformedCRLSignature
    """setupCRLs re-marshals (R, S): a signature SEQUENCE{R, S, T} still revokes"""
    import base64
    from oracle import crl as CRL
    conf = decode("FabricMSPConfig", bytes.fromhex(FX["msps"]["msp/testdata/revocation"]["config"]))
    raw = conf["revocation_list"][0]
    der = X.pem_decode(raw)
    t, s, e = X.tlv(der, 0)
    top = X.children(der, s, e)
    c = CRL.parse_crl(raw)
    sig = _der_tlv(0x30, X._der_intb(c["r"]) + X._der_intb(c["s"]) + X._der_intb(100))
    new = _der_tlv(0x30, der[top[0][3]:top[0][2]] + der[top[1][3]:top[1][2]] + _der_tlv(0x03, b"\x00" + sig))
    pem = b"-----BEGIN X509 CRL-----\n" + b"\n".join(
        base64.b64encode(new)[i:i + 64] for i in range(0, len(base64.b64encode(new)), 64)) + b"\n-----END X509 CRL-----\n"
    conf["revocation_list"] = [pem]
    m = MSP(conf)
    pem_id = FX["msps"]["msp/testdata/revocation"]["identities"]["signcerts/signcert-revoked.pem"].encode()
    assert not m.resolve(pem_id).valid


# ---- msp/mspwithintermediatecas_test.go
def test_intermediate_ca_identity_validates():  # TestMSPWithIntermediateCAs
    i = _one("intermediate", "signcerts")
    assert i is not None and i.valid


def test_identity_issued_by_an_internal_ca_is_invalid():  # TestMSPWithIntermediateCAs2
    assert _one("intermediate2", "signcerts").valid
    u = _ident("intermediate2", "users/user2-cert.pem")
    assert u is not None and not u.valid  # deserializes; "Parent certificate should be a leaf"


def test_intermediate_ca_as_identity():  # TestIntermediateCAIdentityValidity: CAs are no identities
    with pytest.raises(Unsupported):
        _one("intermediate", "intermediatecerts")


# ---- the engine's CPU X.509 parser against the restatement
def _oracle_view(pem):
    try:
        der = X.pem_decode(pem)
    except Unsupported:
        return {"stage": "pem", "status": 2}
    if der is None:
        return {"stage": "pem", "status": 1}
    try:
        c = X.parse_certificate(der)
    except X.ParseError:
        return {"stage": "parse", "status": 1}
    except Unsupported:
        return {"stage": "parse", "status": 2}
    h = lambda b: hashlib.sha256(b).hexdigest()
    v = {"stage": "ok", "status": 0, "key": {"p256": 1, "p384": 2, "other": 3, "undeserializable": 4}[c["key"]], "version": c["version"],
         "is_ca": int(c["is_ca"]), "bc_valid": int(c["bc_valid"]), "path_len": c["path_len"], "has_ski": int(c["ski"] is not None),
         "key_usage": c["key_usage"], "unhandled_critical": int(c["unhandled_critical"]),
         "not_before": c["not_before"], "not_after": c["not_after"],
         "pub": c["pub"].hex() if c["pub"] else "", "tbs": h(c["tbs"]), "issuer": h(c["issuer"]),
         "subject": h(c["subject"]), "sig": c["sig"].hex(), "ous": [o.encode().hex() for o in c["ous"]]}
    try:
        v["raw2"] = h(X.sanitized_raw(c))
        v["raw2_status"] = 0
    except Unsupported:
        v["raw2_status"] = 2
    return v


def _lib():
    from fabric_amd import _lib as L
    try:
        L.load()
    except L.FgvError as e:
        pytest.skip(str(e))
    return L


def test_engine_parser_matches_on_reference_certificates():
    L = _lib()
    for name, pem in sorted(FX["certs"].items()):
        assert L.x509_probe(pem.encode()) == _oracle_view(pem.encode()), name


def _mutants(pem, rng, n):
    der = X.pem_decode(pem)
    import base64
    for _ in range(n):
        d = bytearray(der)
        k = rng.randrange(4)
        if k == 0:  # flip bytes
            for _ in range(rng.randint(1, 3)):
                d[rng.randrange(len(d))] ^= 1 << rng.randrange(8)
        elif k == 1:  # set a byte
            d[rng.randrange(len(d))] = rng.choice((0x00, 0x01, 0x02, 0x04, 0x05, 0x06, 0x0C, 0x13, 0x16, 0x17,
                                                   0x18, 0x1E, 0x30, 0x31, 0x80, 0x81, 0x82, 0xA0, 0xA3, 0xFF))
        elif k == 2:  # truncate / extend
            d = d[:rng.randrange(len(d))] if rng.random() < 0.5 else d + bytes(rng.randrange(1, 4))
        else:  # splice a window from elsewhere
            a, b = sorted(rng.sample(range(len(d)), 2))
            w = d[a:b][:8]
            p = rng.randrange(len(d) - len(w) + 1)
            d[p:p + len(w)] = w
        body = base64.encodebytes(bytes(d))
        yield b"-----BEGIN CERTIFICATE-----\n" + body + b"-----END CERTIFICATE-----\n"


def test_engine_parser_matches_on_mutated_certificates():
    L = _lib()
    rng = random.Random(20261016)
    seeds = [p.encode() for _, p in sorted(FX["certs"].items())][:40]
    mism, total, ok = [], 0, 0
    for pem in seeds:
        for m in _mutants(pem, rng, 60):
            a, b = L.x509_probe(m), _oracle_view(m)
            total += 1
            ok += a.get("stage") == "ok"
            if a != b:
                mism.append((a, b))
    assert not mism, (len(mism), mism[:2])
    assert total == 2400 and ok > 100  # (a share of the mutants still parse: serial, times, names, keys)


def test_engine_pem_rules():
    L = _lib()
    der = X.pem_decode(next(iter(FX["certs"].values())).encode())
    import base64
    b64 = base64.b64encode(der)
    cases = [b"", b"no pem here", b"-----BEGIN CERTIFICATE-----\n" + b64 + b"\n-----END CERTIFICATE-----",
             b"junk\n-----BEGIN X-----\n" + b64 + b"\n-----END X-----\ntrailer",
             b"-----BEGIN CERTIFICATE-----\nProc-Type: 4,ENCRYPTED\n\n" + b64 + b"\n-----END CERTIFICATE-----",
             b"-----BEGIN CERTIFICATE-----\n" + b64[:-1] + b"\n-----END CERTIFICATE-----",
             b"-----BEGIN CERTIFICATE-----\n" + b64 + b"=\n-----END CERTIFICATE-----",
             b"-----BEGIN CERTIFICATE-----\n" + b64 + b"\n-----END OTHER-----",
             b"-----BEGIN CERTIFICATE-----\r\n" + b"\r\n".join(b64[i:i + 64] for i in range(0, len(b64), 64)) +
             b"\r\n-----END CERTIFICATE-----\r\n"]
    for c in cases:
        assert L.x509_probe(c) == _oracle_view(c), c[:60]


def test_synthetic_cases_oracle():
    """tests/msp_cases.py: the restatement gives the outcome each synthetic case is built for"""
    from oracle import v20
    from tests.msp_cases import FAILED, MSPID, OK, REPEAT, UNSUP, synthetic
    cfg, cases = synthetic()
    models = v20.ChannelModel("ch", [], {}, config=cfg).msp_models()
    assert not isinstance(models[MSPID], Exception), models[MSPID]
    for label, ser, st, valid, roles in cases:
        if st == REPEAT:
            continue
        sid = decode("SerializedIdentity", ser)
        m = models[sid.get("mspid", "")]
        if isinstance(m, Exception):
            assert st == UNSUP, label
            continue
        idb = sid.get("id_bytes") or b""
        try:
            got = m.resolve(idb)
        except Unsupported:
            assert st == UNSUP, label
            continue
        if got is None:
            assert st == FAILED, label
            continue
        assert st == OK and (got.valid, got.roles) == (valid, roles), (label, got.valid, got.roles)


def test_engine_parser_matches_on_synthetic_certificates():
    L = _lib()
    from tests.msp_cases import synthetic
    _, cases = synthetic()
    for label, ser, *_ in cases:
        pem = decode("SerializedIdentity", ser).get("id_bytes") or b""
        assert L.x509_probe(pem) == _oracle_view(pem), label


# ---- fork hazards: shapes Go's encoding/pem / crypto/x509 accept that the engine
# does not model come out Unsupported on both sides, never as an undeserializable identity
def test_reference_leaf_reframings_are_unsupported():
    from tests.msp_cases import fork_hazard_variants
    L = _lib()
    rel = "msp/testdata/nodeous3"
    m = _msp(rel)
    ids = FX["msps"][rel]["identities"]
    pem = ids[[k for k in ids if k.startswith("signcerts/")][0]].encode()
    assert m.resolve(pem).valid  # the leaf as issued
    for label, p in fork_hazard_variants(pem):
        want = "OK" if label == "short_line_wrap" else "UNSUP"
        try:
            got = m.resolve(p)
            got = "OK" if got is not None and got.valid else "FAILED"
        except Unsupported:
            got = "UNSUP"
        assert got == want, label
        v = L.x509_probe(p)
        assert v == _oracle_view(p), label
        assert (v["status"] == 2) == (want == "UNSUP"), (label, v)


def test_engine_parser_matches_on_mutated_pem_text():
    """byte-level mutations of the PEM text: the engine's framing decision equals the oracle's,
    and nothing that still holds a "-----BEGIN " is ever a PEM parse error"""
    L = _lib()
    rng = random.Random(7)
    seeds = [p.encode() for _, p in sorted(FX["certs"].items())][:30]
    n_unsup = 0
    for pem in seeds:
        for _ in range(40):
            d = bytearray(pem)
            k = rng.randrange(5)
            i = rng.randrange(len(d))
            if k == 0:
                d[i] = rng.choice(b" \t\r\n-=:A/+!\x00")
            elif k == 1:
                d.insert(i, rng.choice(b" \t\r\n-=:A"))
            elif k == 2:
                del d[i]
            elif k == 3:
                d = bytearray(rng.choice([b"x\n", b"\n", b" ", b"-----BEGIN X-----\n-----END X-----\n"])) + d
            else:
                d += rng.choice([b"x", b"\n\n", b"-----BEGIN CERTIFICATE-----\n"])
            m = bytes(d)
            a, b = L.x509_probe(m), _oracle_view(m)
            assert a == b, m[:80]
            if a["stage"] == "pem":
                assert a["status"] == 2 or b"-----BEGIN " not in m
                n_unsup += a["status"] == 2
    assert n_unsup > 100


# ---- the MSP's post-setup admin checks (mspimplsetup.go:612-624, 684-702)
@pytest.mark.parametrize("rel", ["nodeous1", "nodeous8", "badadmin"])
def test_msp_with_invalid_admin_does_not_set_up(rel):
    """TestInvalidAdminNodeOU (nodeous1, nodeous8: NodeOUs on, the admin carries no client / admin
    OU) and TestBadAdminIdentity (badadmin): Setup fails in the reference -> outside the model"""
    with pytest.raises(Unsupported):
        _msp("msp/testdata/" + rel)


def test_admin_setup_cases_oracle():
    from oracle import v20
    from tests.msp_cases import MSPID, admin_setup_cases
    for label, cfg, probe, sets_up in admin_setup_cases():
        m = v20.ChannelModel("ch", [], {}, config=cfg).msp_models()[MSPID]
        assert isinstance(m, Exception) != sets_up, (label, m)
        if sets_up:
            assert m.resolve(decode("SerializedIdentity", probe).get("id_bytes")) is not None, label
