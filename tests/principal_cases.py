"""Loader of tests/golden/principal_known_answers.json (reference msp_test.go SatisfiesPrincipal
assertions as endorsement policies; see tests/golden/make_principal_known_answers.py)."""
import json
import os

from fabric_amd.txvalidator import Identity

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "principal_known_answers.json")


def load():
    d = json.load(open(GOLD))
    s = d["signer"]
    ous = [(o, bytes.fromhex(c)) for o, c in s["ous"]]
    ser = bytes.fromhex(s["ser"])

    def ident(with_ous):
        return (ser, Identity(s["mspid"], bytes.fromhex(s["pub"]), True, bytes.fromhex(s["id_digest"]), roles=s["roles"],
                              ous=ous if with_ous else None))
    return dict(config=bytes.fromhex(d["config"]), block=bytes.fromhex(d["block"]),
                chaincodes={k: bytes.fromhex(v) for k, v in d["chaincodes"].items()}, expected=d["expected"],
                names=d["names"], ident=ident)


def single_blocks(block):
    """each transaction of the fixture block in a block of its own"""
    import hashlib

    from fabric_amd.synth.blocks import f_bytes, f_msg, f_varint
    from oracle.protowire import decode
    out = []
    for e in decode("Block", block)["data"]["data"]:
        header = f_varint(1, 2) + f_bytes(2, b"\0" * 32) + f_bytes(3, hashlib.sha256(e).digest())
        out.append(f_msg(1, header) + f_msg(2, f_msg(1, e)) + f_msg(3, b"".join(f_msg(1, b"") for _ in range(5))))
    return out
