"""Synthetic MSP cache-miss cases shared by tests/test_oracle_msp.py (the oracle against the
expected outcomes written here) and tests/test_gpu_msp.py (the engine against the oracle).

Channel MSP "Org1MSP": roots CA1 (SKI, keyCertSign), CA3 (key usage without keyCertSign), CA4
(parent of intermediate INT1: an internal node of the certification tree), CA5 (pathLen 0, parent
of INT2); NodeOUs client / peer / admin / orderer; one listed admin.  "Org2MSP": a root without a
SubjectKeyIdentifier (the MSP would not set up: outside the model).  Leaves cover each rule of
the miss path: role OUs, two role OUs, no OU, a listed admin, a high-S CA signature, unknown
issuer, wrong CA key, an unhandled critical extension, a CA as an identity, SAN (DNS / URI), an
empty validity window, Ed25519, a malformed IA5 OU, not PEM, a chain through an intermediate, an
issuer that is an internal node, a path length exceeded, CRLs (a revoked leaf, a list signed by another key, a serial revoked
under another issuer).  Shapes Go's pem / x509 parsers may accept
and the restatement does not model (fork_hazard_variants) must come out Unsupported, never a code."""
import base64

from fabric_amd.synth import EdKey, Key, Key384, make_cert_ed25519
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


def _der(pem):
    return base64.b64decode(b"".join(pem.split(b"-----")[2].split()))


def _pem(der, typ=b"CERTIFICATE"):
    return b"-----BEGIN " + typ + b"-----\n" + base64.encodebytes(der) + b"-----END " + typ + b"-----\n"


def _outer_content(der):
    ln, o = der[1], 2
    if ln & 0x80:
        o = 2 + (ln & 0x7F)
        ln = int.from_bytes(der[2:o], "big")
    return der[o:o + ln]


def fork_hazard_variants(pem):
    """[(label, pem')]: a valid PEM certificate re-framed into shapes Go's encoding/pem and
    crypto/x509 accept (or may accept) and the engine does not model -> Unsupported"""
    der = _der(pem)
    b64 = base64.encodebytes(der)
    first = b64.index(b"\n")
    return [
        ("extra_outer_element", _pem(G.seq(_outer_content(der) + G.tlv(0x05, b"")))),
        ("junk_prefixed_pem", b"junk\n" + pem),
        ("begin_mid_line", b"junk " + pem),
        ("malformed_block_then_valid", b"-----BEGIN CERTIFICATE-----\n!!!!\n-----END CERTIFICATE-----\n" + pem),
        ("blank_in_base64", b"-----BEGIN CERTIFICATE-----\n" + b64[:10] + b" " + b64[10:] + b"-----END CERTIFICATE-----\n"),
        ("tab_after_type", b"-----BEGIN CERTIFICATE-----\t\n" + b64 + b"-----END CERTIFICATE-----\n"),
        ("text_after_end_line", pem.rstrip(b"\n") + b" trailing\n"),
        ("pem_header", b"-----BEGIN CERTIFICATE-----\nX-Note: hi\n" + b64 + b"-----END CERTIFICATE-----\n"),
        ("short_line_wrap", b"-----BEGIN CERTIFICATE-----\n" + b64[:first - 3] + b"\n" + b64[first - 3:] +
         b"-----END CERTIFICATE-----\n"),
    ]


def rsa_spki(n, e):
    """SubjectPublicKeyInfo{rsaEncryption, NULL, BIT STRING RSAPublicKey{modulus, exponent}}"""
    def sint(v):
        b = v.to_bytes((v.bit_length() + 8) // 8 or 1, "big", signed=True)
        return G.tlv(0x02, b)
    return G.seq(G.seq(G.oid("2a864886f70d010101"), G.tlv(0x05, b"")), G.tlv(0x03, b"\x00" + G.seq(sint(n), sint(e))))


def synthetic():
    """-> (config bytes, [(label, serialized, status, valid, roles)]) -- valid / roles only for OK"""
    ca1, ca2, ca3, ca4, ca5 = Key(77, 1), Key(77, 2), Key(77, 3), Key(77, 4), Key(77, 5)
    int1, int2 = Key(77, 6), Key(77, 7)
    n1, n3, n4 = G.name("ca1.org1"), G.name("ca3.org1"), G.name("ca4.org1")
    nI1, nI2 = G.name("int1.org1"), G.name("int2.org1")
    r1 = G.ca_cert(ca1, "ca1.org1")
    r3 = G.ca_cert(ca3, "ca3.org1", usage=(0,))
    r4 = G.ca_cert(ca4, "ca4.org1")                       # parent of int1: an internal node
    r5 = G.ca_cert(ca5, "ca5.org1", path_len=0)           # pathLen 0: no intermediate below int2
    i1 = G.ca_cert(int1, "int1.org1", issuer_key=ca4, issuer_cn="ca4.org1", serial=11)
    i2 = G.ca_cert(int2, "int2.org1", issuer_key=ca5, issuer_cn="ca5.org1", serial=12)
    r2 = G.ca_cert(ca2, "ca2.org2", org="Org2", with_ski=False)  # Org2MSP: a root without SKI
    k = [Key(77, 100 + i) for i in range(46)]

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
    add("via_intermediate", leaf(10, ["peer"], issuer_key=int1, issuer=nI1), OK, True, _roles(MEMBER, PEER))
    add("issued_by_internal_ca", leaf(22, ["peer"], issuer_key=ca4, issuer=n4), OK, False, 0)
    add("path_len_exceeded", leaf(23, ["peer"], issuer_key=int2, issuer=nI2), FAILED)
    add("intermediate_as_identity", i1, UNSUP)
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
    # P-384 leaves under a P-256 CA (round 6): resolved on a cache miss, verified on the GPU
    k384 = [Key384(77, 200 + i) for i in range(3)]

    def spki384(x, y):
        return G.seq(G.seq(G.oid(G.OID_EC), G.oid("2b81040022")), G.tlv(0x03, b"\x00\x04" + x + y))

    def leaf384(i, ous, x=None, y=None):
        kk = k384[i]
        return G.cert(k[0], ca1, G.name("p384leaf%d" % i, ous=ous), n1, serial=2000 + i,
                      spki=spki384(x or kk.qx, y or kk.qy))
    add("p384_peer", leaf384(0, ["peer"]), OK, True, _roles(MEMBER, PEER))
    add("p384_client", leaf384(1, ["client"]), OK, True, _roles(MEMBER, CLIENT))
    add("p384_off_curve", leaf384(2, ["peer"], y=bytes(47) + b"\x05"), FAILED)
    # re-framings of a valid peer certificate: Go's parsers may accept each (extra outer element,
    # PEM framing) -> Unsupported; a canonical CRLF / 64-column framing -> the same identity
    for j in range(9):
        lbl, p = fork_hazard_variants(leaf(25 + j, ["peer"]))[j]
        add(lbl, p, OK if lbl == "short_line_wrap" else UNSUP, *((True, _roles(MEMBER, PEER)) if lbl == "short_line_wrap" else ()))
    crlf = base64.b64encode(_der(leaf(35, ["peer"])))
    add("crlf_64_columns", b"-----BEGIN CERTIFICATE-----\r\n" + b"\r\n".join(crlf[i:i + 64] for i in range(0, len(crlf), 64))
        + b"\r\n-----END CERTIFICATE-----\r\n", OK, True, _roles(MEMBER, PEER))
    add("critical_ski", leaf(36, ["peer"], extensions=[G.ext("551d0e", G.tlv(0x04, b"\x01" * 20), critical=True)]), UNSUP)
    add("key_usage_trailing_bytes", leaf(37, ["peer"], extensions=[G.ext("551d0f", G.tlv(0x03, b"\x00\x80") + b"\x05\x00")]),
        UNSUP)
    add("basic_constraints_trailing_element",
        leaf(38, ["peer"], extensions=[G.ext("551d13", G.seq(G.tlv(0x01, b"\x00"), G.tlv(0x04, b"x")))]), UNSUP)
    add("no_begin_anywhere", b"-----END CERTIFICATE-----\n", FAILED)
    # RSA leaves (never pass identity.Verify): registered as keys that never verify,
    # with their validity and roles -- a 2048-bit modulus, and a key Go's PKCS#1 checks would
    # reject (negative modulus): the same verdict on every path
    add("rsa_leaf", leaf(39, ["peer"], spki=rsa_spki((1 << 2047) + 12345, 65537)), OK, True, _roles(MEMBER, PEER))
    add("rsa_leaf_bad_modulus", leaf(40, ["client"], spki=rsa_spki(-5, 3)), OK, True, _roles(MEMBER, CLIENT))
    # CRLs (mspimplvalidate.go:94-140): CA1's list revokes leaf 41 and leaf 43 under INT1 (another
    # issuer: its CRL would need INT1's SKI as AKI -- not revoked); a list carrying CA1's AKI but
    # signed with CA2's key (CheckCRLSignature fails: ignored) names leaf 42; CA1 signs its list
    # with a high-S signature, which Go's ecdsa accepts
    add("revoked_by_crl", leaf(41, ["peer"]), OK, False, 0)
    add("crl_signed_by_another_key", leaf(42, ["client"]), OK, True, _roles(MEMBER, CLIENT))
    add("serial_revoked_under_another_ca", leaf(43, ["peer"], issuer_key=int1, issuer=nI1), OK, True,
        _roles(MEMBER, PEER))
    crls = [G.crl(ca1, "ca1.org1", ca1, [1041, 1043, 99], high_s=True),
            G.crl(ca2, "ca1.org1", ca1, [1042])]
    out.append(("repeat", out[0][1], REPEAT, None, None))  # the same bytes again in one call
    out.append(("msp_root_without_ski", serialized_identity("Org2MSP", leaf(24, ["peer"], issuer_key=ca2,
                                                                           issuer=G.name("ca2.org2", "Org2"))),
                UNSUP, None, None))
    fabric = fabric_msp_config(MSPID, root_certs=[r1, r3, r4, r5], intermediate_certs=[i1, i2], admins=[listed_admin],
                               crls=crls)
    fabric2 = fabric_msp_config("Org2MSP", root_certs=[r2])
    cfg = make_config([MSPID, "Org2MSP"], msp_configs={MSPID: fabric, "Org2MSP": fabric2})
    return cfg, out


def admin_setup_cases():
    """the MSP's post-setup admin checks (mspimplsetup.go:612-624 postSetupV1 without
    NodeOUs -- every admin must Validate, CRLs included; :684-702 postSetupV142 with NodeOUs -- every
    admin carries the client or the admin OU).  -> [(label, config bytes, probe serialized identity,
    sets_up)]: when the MSP does not set up, the probe (an ordinary peer leaf) is Unsupported."""
    ca1, ca2 = Key(78, 1), Key(78, 2)
    n1 = G.name("ca1.org1")
    r1 = G.ca_cert(ca1, "ca1.org1")
    k = [Key(78, 100 + i) for i in range(12)]

    def leaf(i, ous, issuer_key=ca1, issuer=n1):
        return G.cert(k[i], issuer_key, G.name("adm%d" % i, ous=ous), issuer, serial=2000 + i)

    probe = serialized_identity(MSPID, leaf(0, ["peer", "dept1"]))
    out = []

    def case(label, admin, sets_up, node_ous=True, crls=(), ou_ids=()):
        fabric = fabric_msp_config(MSPID, root_certs=[r1], admins=[admin], crls=crls, ou_ids=ou_ids,
                                   node_ous=("client", "peer", "admin", "orderer") if node_ous else None)
        out.append((label, make_config([MSPID], msp_configs={MSPID: fabric}), probe, sets_up))

    case("admin_valid_no_nodeous", leaf(1, ["client"]), True, node_ous=False)
    case("admin_revoked_no_nodeous", leaf(2, ["client"]), False, node_ous=False,
         crls=[G.crl(ca1, "ca1.org1", ca1, [2002])])
    case("admin_revoked_with_nodeous", leaf(3, ["client"]), True, crls=[G.crl(ca1, "ca1.org1", ca1, [2003])])
    case("admin_ou_ids_mismatch_no_nodeous", leaf(4, ["dept2"]), False, node_ous=False, ou_ids=[(r1, "dept1")])
    case("admin_ou_ids_match_no_nodeous", leaf(5, ["dept1"]), True, node_ous=False, ou_ids=[(r1, "dept1")])
    case("admin_peer_ou_with_nodeous", leaf(6, ["peer"]), False)
    case("admin_admin_ou_with_nodeous", leaf(7, ["admin"]), True)
    case("admin_unknown_issuer", leaf(8, ["client"], issuer=G.name("ca.other")), False)
    case("admin_wrong_ca_key_no_nodeous", leaf(9, ["client"], issuer_key=ca2), False, node_ous=False)
    case("admin_wrong_ca_key_with_nodeous", leaf(10, ["client"], issuer_key=ca2), False)
    return out
