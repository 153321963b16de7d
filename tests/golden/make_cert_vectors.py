"""Generate tests/golden/msp_cert_sigs.json from the reference's own MSP fixtures.

Every X.509 certificate under /root/reference/msp/testdata and /root/reference/sampleconfig/msp
that is signed ecdsa-with-SHA256 by a P-256 issuer certificate present in the same MSP
directory yields one golden vector (issuer key, SHA-256(TBSCertificate), DER signature).

Expected outcomes are NOT computed by our oracle:
  * equation truth comes from OpenSSL 3.0.2 (`openssl verify`-equivalent X509_verify via the
    CLI), i.e. the CA really signed the certificate;
  * the low-S rule is a plain integer compare s <= n>>1 (bccsp/utils/ecdsa.go:82-89);
  * msp/testdata/mspid/signcerts/peer0-cert.pem must come out high-S, as asserted by the
    reference test msp/msp_test.go:1524-1535 (TestMSPIdentityIdentifier).
Derived vectors: the low-S twin (r, n-s) of every high-S signature (what sanitizeCert
produces, msp/mspimpl.go:892-938) -> valid; a one-bit digest flip of every vector -> invalid.

This script reads the reference tree as DATA and only runs here (not on the GPU box);
its output JSON is the committed fixture.
"""
import base64, glob, hashlib, json, os, subprocess, sys

REF = "/root/reference"
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
OID_ECDSA_SHA256 = bytes.fromhex("2a8648ce3d040302")
OID_EC_PUBKEY = bytes.fromhex("2a8648ce3d0201")
OID_P256 = bytes.fromhex("2a8648ce3d030107")


def tlv(b, o):
    tag = b[o]; o += 1
    l = b[o]; o += 1
    if l & 0x80:
        nb = l & 0x7F
        l = int.from_bytes(b[o:o + nb], "big"); o += nb
    return tag, o, l  # content at [o, o+l)


def children(b, o, l):
    end = o + l
    out = []
    while o < end:
        t, co, cl = tlv(b, o)
        out.append((t, o, co, cl))
        o = co + cl
    return out


def parse_cert(der):
    t, co, cl = tlv(der, 0)
    cert = children(der, co, cl)
    tbs_t, tbs_o, tbs_co, tbs_cl = cert[0]
    tbs_raw = der[tbs_o:tbs_co + tbs_cl]
    _, _, a_co, a_cl = cert[1]
    alg = children(der, a_co, a_cl)[0]
    alg_oid = der[alg[2]:alg[2] + alg[3]]
    _, _, s_co, s_cl = cert[2]
    sig = der[s_co + 1:s_co + s_cl]  # BIT STRING: skip unused-bits byte
    f = children(der, tbs_co, tbs_cl)
    i = 1 if f[0][0] == 0xA0 else 0
    issuer = der[f[i + 2][1]:f[i + 2][2] + f[i + 2][3]]
    subject = der[f[i + 4][1]:f[i + 4][2] + f[i + 4][3]]
    spki = f[i + 5]
    sp = children(der, spki[2], spki[3])
    algid = children(der, sp[0][2], sp[0][3])
    kalg = der[algid[0][2]:algid[0][2] + algid[0][3]]
    curve = der[algid[1][2]:algid[1][2] + algid[1][3]] if len(algid) > 1 else b""
    pub = der[sp[1][2] + 1:sp[1][2] + sp[1][3]]
    return dict(tbs=tbs_raw, alg=alg_oid, sig=sig, issuer=issuer, subject=subject,
                kalg=kalg, curve=curve, pub=pub)


def pem_certs(path):
    txt = open(path, "rb").read().decode(errors="ignore")
    out = []
    for blk in txt.split("-----BEGIN CERTIFICATE-----")[1:]:
        body = blk.split("-----END CERTIFICATE-----")[0]
        out.append(base64.b64decode("".join(body.split())))
    return out


def der_rs(sig):
    t, co, cl = tlv(sig, 0)
    ints = children(sig, co, cl)
    return (int.from_bytes(sig[ints[0][2]:ints[0][2] + ints[0][3]], "big"),
            int.from_bytes(sig[ints[1][2]:ints[1][2] + ints[1][3]], "big"))


def openssl_verifies(issuer_path, cert_path):
    # check only the signature (partial chain, no purpose/time checks)
    r = subprocess.run(["openssl", "verify", "-partial_chain", "-no_check_time", "-CAfile", issuer_path,
                        cert_path], capture_output=True, text=True)
    return r.returncode == 0


def main(out_path):
    dirs = sorted(glob.glob(f"{REF}/msp/testdata/*")) + [f"{REF}/sampleconfig/msp"]
    vecs = []
    tmp = "/tmp/fgv_golden"
    os.makedirs(tmp, exist_ok=True)
    for d in dirs:
        files = sorted(p for p in glob.glob(f"{d}/**/*", recursive=True)
                       if os.path.isfile(p) and (p.endswith(".pem") or "certs" in p))
        certs = []
        for p in files:
            try:
                for der in pem_certs(p):
                    certs.append((p, der, parse_cert(der)))
            except Exception:
                continue
        for p, der, c in certs:
            if c["alg"] != OID_ECDSA_SHA256:
                continue
            for ip, ider, ic in certs:
                if ic["subject"] != c["issuer"] or ic["kalg"] != OID_EC_PUBKEY or ic["curve"] != OID_P256:
                    continue
                if len(ic["pub"]) != 65 or ic["pub"][0] != 4:
                    continue
                a = os.path.join(tmp, "issuer.pem"); b = os.path.join(tmp, "cert.pem")
                open(a, "wb").write(b"-----BEGIN CERTIFICATE-----\n" + base64.encodebytes(ider) + b"-----END CERTIFICATE-----\n")
                open(b, "wb").write(b"-----BEGIN CERTIFICATE-----\n" + base64.encodebytes(der) + b"-----END CERTIFICATE-----\n")
                eq = openssl_verifies(a, b)
                if not eq:
                    continue  # different key with the same subject name
                r, s = der_rs(c["sig"])
                rel, irel = os.path.relpath(p, REF), os.path.relpath(ip, REF)
                digest = hashlib.sha256(c["tbs"]).digest()
                vecs.append(dict(source=rel, issuer=irel, qx=ic["pub"][1:33].hex(), qy=ic["pub"][33:].hex(),
                                 digest=digest.hex(), sig=c["sig"].hex(), high_s=s > N // 2,
                                 expected=3 if s > N // 2 else 0, kind="reference-cert"))
                break
    # de-duplicate identical (key, digest, sig)
    seen, uniq = {}, []
    for v in vecs:
        k = (v["qx"], v["digest"], v["sig"])
        if k not in seen:
            v["also"] = []
            seen[k] = v; uniq.append(v)
        else:
            seen[k]["also"].append(v["source"])
    derived = []
    for v in uniq:
        r, s = der_rs(bytes.fromhex(v["sig"]))
        if v["high_s"]:
            low = N - s
            import ctypes  # minimal DER re-encode (no synth dependency)
            def di(x):
                b = x.to_bytes((x.bit_length() + 7) // 8 or 1, "big")
                if b[0] & 0x80: b = b"\x00" + b
                return b"\x02" + bytes([len(b)]) + b
            body = di(r) + di(low)
            derived.append(dict(v, sig=(b"\x30" + bytes([len(body)]) + body).hex(), high_s=False, expected=0,
                                kind="low-s twin (sanitizeCert)"))
        dg = bytearray(bytes.fromhex(v["digest"])); dg[31] ^= 1
        derived.append(dict(v, digest=dg.hex(), expected=3 if v["high_s"] else 1, kind="digest bit flip"))
    mspid = [v for v in uniq if any(x.startswith("msp/testdata/mspid/signcerts") for x in [v["source"]] + v["also"])]
    assert mspid and all(v["high_s"] for v in mspid), "reference high-S fixture not found"
    json.dump(dict(generator="tests/golden/make_cert_vectors.py", n_reference=len(uniq),
                   vectors=uniq + derived), open(out_path, "w"), indent=1)
    print(f"{len(uniq)} reference vectors ({sum(v['high_s'] for v in uniq)} high-S), {len(derived)} derived")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "msp_cert_sigs.json"))
