"""Loader of tests/golden/committer_known_answers.json (reference-test known answers; see
tests/golden/make_committer_known_answers.py for the sources and the expected codes)."""
import json
import os

from fabric_amd.txvalidator import Identity

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "committer_known_answers.json")


def _env(payload, sig):
    from fabric_amd.synth.blocks import f_bytes
    return f_bytes(1, payload) + f_bytes(2, sig)


def bad_tx_envelopes(c):
    """TestBadTx (fullflow_test.go:213-247): every payload byte i -> (b + 1) % 255 with the
    original signature, then the original payload with a corrupted signature"""
    p, sig = bytes.fromhex(c["bad_tx_payload"]), bytes.fromhex(c["bad_tx_sig"])
    out = [_env(p[:i] + bytes([(p[i] + 1) % 255]) + p[i + 1:], sig) for i in range(len(p))]
    bad = bytearray(sig)
    bad[len(bad) // 2] = (bad[len(bad) // 2] - 1) % 256
    return out + [_env(p, bytes(bad))]


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
        ccs = {k: bytes.fromhex(v) for k, v in c["chaincodes"].items()}
        c = dict(c, identities=ids, chaincodes=ccs)
        if "block" in c:
            c["block"] = bytes.fromhex(c["block"])
        out.append(c)
    return d["vt_codes"], out


def matches(code, exp, vt_codes):
    if exp == "not_valid":
        return code != 0
    if exp == "passes_validate_transaction":
        return code not in vt_codes
    return code == exp
