"""Synthetic MSP cache-miss cases shared by tests/test_oracle_msp.py (the oracle against the
expected outcomes written here) and tests/test_gpu_msp.py (the engine against the oracle).

One channel MSP "Org1MSP" with three roots -- CA1 (SKI, keyCertSign), CA2 (no SKI), CA3 (key
usage without keyCertSign) -- NodeOUs client / peer / admin / orderer, one listed admin; and
leaves covering each rule of the miss path: role OUs, two role OUs, no OU, a listed admin, a
high-S CA signature, unknown issuer, wrong CA key, an unhandled critical extension, a CA as an
identity, SAN (DNS / URI), an empty validity window, Ed25519, a malformed IA5 OU, not PEM."""
from fabric_amd.synth import EdKey, Key, make_cert_ed25519
from fabric_amd.synth import x509gen as G
from fabric_amd.synth.blocks import serialized_identity
from fabric_amd.synth.chanconfig import fabric_msp_config, make_config

MSPID = "Org1MSP"
OK, FAILED, UNSUP, REPEAT = 1, 2, 3, 4  # FGV_RESOLVE_*
MEMBER, ADMIN, CLIENT, PEER, ORDERER = 0, 1, 2, 3, 4


def _roles(*rs):
    v = 0
    for r in rs:
        v |= 1 << r
    return v


def synthetic():
    """-> (config bytes, [(label, serialized, status, valid, roles)]) -- valid / roles only for OK"""
    ca1, ca2, ca3 = Key(77, 1), Key(77, 2), Key(77, 3)
    n1, n2, n3 = G.name("ca1.org1"), G.name("ca2.org1"), G.name("ca3.org1")
    r1 = G.ca_cert(ca1, "ca1.org1")
    r2 = G.ca_cert(ca2, "ca2.org1", with_ski=False)
    r3 = G.ca_cert(ca3, "ca3.org1", usage=(0,))
    k = [Key(77, 100 + i) for i in range(40)]

    def leaf(i, ous, issuer_key=ca1, issuer=n1, **kw):
        return G.cert(k[i], issuer_key, G.name("leaf%d" % i, ous=ous), issuer, serial=1000 + i, **kw)

    listed_admin = leaf(8, ["client"])
    out = []

    def add(label, pem, status, valid=None, roles=None):
        out.append((label, serialized_identity(MSPID, pem), status, valid, roles))

    add("peer", leaf(1, ["peer"]), OK, True, _roles(MEMBER, PEER))
    add("client", leaf(2, ["client"]), OK, True, _roles(MEMBER, CLIENT))
    add("admin_ou", leaf(3, ["admin"]), OK, True, _roles(MEMBER, ADMIN))
    add("orderer", leaf(4, ["orderer"]), OK, True, _roles(MEMBER, ORDERER))
    add("no_ou", leaf(5, []), OK, False, 0)
    add("two_role_ous", leaf(6, ["client", "peer"]), OK, False, 0)
    add("peer_plus_other_ou", leaf(7, ["dept1", "peer"]), OK, True, _roles(MEMBER, PEER))
    add("listed_admin", listed_admin, OK, True, _roles(MEMBER, ADMIN, CLIENT))
    add("high_s_ca_signature", leaf(9, ["peer"], high_s=True), OK, True, _roles(MEMBER, PEER))
    add("ca_without_ski", leaf(10, ["peer"], issuer_key=ca2, issuer=n2), OK, False, 0)
    add("unknown_issuer", leaf(11, ["peer"], issuer=G.name("ca.other")), FAILED)
    add("wrong_ca_key", leaf(12, ["peer"], issuer_key=ca2, issuer=n1), FAILED)
    add("unhandled_critical_ext", leaf(13, ["peer"], extensions=[G.ext("2a0304", b"\x05\x00", critical=True)]),
        FAILED)
    add("ca_as_identity", leaf(14, ["peer"], extensions=[G.basic_constraints(True)]), UNSUP)
    add("san_dns", leaf(15, ["peer"], extensions=[G.san_dns("peer0.org1.example.com")]), OK, True,
        _roles(MEMBER, PEER))
    add("san_uri", leaf(16, ["peer"], extensions=[G.ext("551d11", G.seq(G.tlv(0x86, b"https://x")))]), UNSUP)
    add("empty_validity", leaf(17, ["peer"], not_before="240101000000Z", not_after="240101000000Z"), FAILED)
    add("ca_without_cert_sign", leaf(18, ["peer"], issuer_key=ca3, issuer=n3), FAILED)
    add("ed25519", make_cert_ed25519(EdKey(77, 19), ca1, "leaf19", "Org1", "ca1.org1", 1019), FAILED)
    add("ia5_non_ascii_ou", G.cert(k[20], ca1, G.seq(G.tlv(0x31, G.seq(G.oid(G.OID_OU), G.tlv(0x16, b"p\xe9er")))), n1),
        FAILED)
    add("not_pem", b"definitely not a certificate", FAILED)
    add("key_usage_critical_ok", leaf(21, ["client"], extensions=[G.key_usage((0,))]), OK, True,
        _roles(MEMBER, CLIENT))
    out.append(("repeat", out[0][1], REPEAT, None, None))  # the same bytes again in one call
    fabric = fabric_msp_config(MSPID, root_certs=[r1, r2, r3], admins=[listed_admin])
    cfg = make_config([MSPID], msp_configs={MSPID: fabric})
    return cfg, out
