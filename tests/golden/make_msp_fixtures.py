"""Generate tests/golden/msp_fixtures.json from the reference's own MSP test data (run here, in the
build container; the GPU box never reads /root/reference).

Data only: the certificate PEMs of msp/testdata/<dir>/{cacerts,admincerts,signcerts,adm,
intermediatecerts,crls} and sampleconfig/msp, and for each MSP directory the FabricMSPConfig a
peer builds from it -- restated from msp/configbuilder.go GetLocalMspConfig (files of a folder in
directory order, config.yaml OrganizationalUnitIdentifiers and NodeOUs with their certificate
files; a missing NodeOU certificate file is left out, configbuilder.go:365-380; crypto config
SHA2 / SHA256; MSP id "SampleOrg").  The expected outcomes are the reference's own test
assertions (msp/nodeous_test.go), written in tests/test_oracle_msp.py.

    python3 tests/golden/make_msp_fixtures.py
"""
import json
import os
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from fabric_amd.synth.blocks import f_bytes, f_msg, f_str, f_varint  # noqa: E402

REF = "/root/reference"
DIRS = ["msp/testdata/" + d for d in (
    "nodeous1", "nodeous2", "nodeous3", "nodeous4", "nodeous5", "nodeous6", "nodeous7", "nodeous8",
    "nodeouadmin", "nodeouadmin2", "nodeouadmin3", "nodeouadminclient", "nodeouadminclient2",
    "nodeouorderer", "nodeouorderer2", "nodeouorderer3", "nodeousbadconf2", "mspid", "expired",
    "badadmin", "badconfigou", "badconfigoucert", "intermediate", "intermediate2", "external", "revocation",
    "revocation2", "revokedica")] + \
    ["sampleconfig/msp"]
IDENTITY_FOLDERS = ("signcerts", "admincerts", "adm", "cacerts", "intermediatecerts", "users")


def pem_dir(path):
    """getPemMaterialFromDir: every regular file with a PEM block, in directory order"""
    if not os.path.isdir(path):
        return []
    out = []
    for name in sorted(os.listdir(path)):
        full = os.path.join(path, name)
        if os.path.isdir(full):
            continue
        raw = open(full, "rb").read()
        if b"-----BEGIN" in raw:
            out.append((name, raw))
    return out


def ou_ident(cert, ou):
    return (f_bytes(1, cert) if cert else b"") + (f_str(2, ou) if ou else b"")


def msp_config(d):
    cfg = {}
    p = os.path.join(d, "config.yaml")
    if os.path.exists(p):
        cfg = yaml.safe_load(open(p)) or {}
    out = f_str(1, "SampleOrg")
    for _, raw in pem_dir(os.path.join(d, "cacerts")):
        out += f_bytes(2, raw)
    for _, raw in pem_dir(os.path.join(d, "intermediatecerts")):
        out += f_bytes(3, raw)
    for _, raw in pem_dir(os.path.join(d, "admincerts")):
        out += f_bytes(4, raw)
    for _, raw in pem_dir(os.path.join(d, "crls")):
        out += f_bytes(5, raw)
    for o in cfg.get("OrganizationalUnitIdentifiers") or []:
        out += f_msg(7, ou_ident(open(os.path.join(d, o["Certificate"]), "rb").read(),
                                 o.get("OrganizationalUnitIdentifier") or ""))
    out += f_msg(8, f_str(1, "SHA2") + f_str(2, "SHA256"))
    n = cfg.get("NodeOUs")
    if n and n.get("Enable"):
        body = f_varint(1, 1)
        for field, key in ((2, "ClientOUIdentifier"), (3, "PeerOUIdentifier"), (4, "AdminOUIdentifier"),
                           (5, "OrdererOUIdentifier")):
            o = n.get(key)
            if not o or not o.get("OrganizationalUnitIdentifier"):
                continue
            cert = b""
            if o.get("Certificate"):
                f = os.path.join(d, o["Certificate"])
                cert = open(f, "rb").read() if os.path.exists(f) else b""
            body += f_msg(field, ou_ident(cert, o["OrganizationalUnitIdentifier"]))
        out += f_msg(11, body)
    return out


def main():
    fx = {"msps": {}, "certs": {}}
    for rel in DIRS:
        d = os.path.join(REF, rel)
        ids = {}
        for folder in IDENTITY_FOLDERS:
            for name, raw in pem_dir(os.path.join(d, folder)):
                ids[folder + "/" + name] = raw.decode()
        fx["msps"][rel] = {"config": msp_config(d).hex(), "identities": ids}
    for root, _, files in os.walk(os.path.join(REF, "msp/testdata")):
        for name in sorted(files):
            if not name.endswith(".pem") or "keystore" in root:
                continue
            raw = open(os.path.join(root, name), "rb").read()
            if b"CERTIFICATE-----" in raw:
                fx["certs"][os.path.relpath(os.path.join(root, name), REF)] = raw.decode()
    with open(os.path.join(HERE, "msp_fixtures.json"), "w") as f:
        json.dump(fx, f, indent=0, sort_keys=True)
    print("msps", len(fx["msps"]), "certs", len(fx["certs"]))


if __name__ == "__main__":
    main()
