"""Committer known answers ported from the reference's own tests (run in the build container;
the output JSON is the committed fixture, the GPU box never reads /root/reference).

The transactions are assembled the way protoutil builds them (CreateProposalFromCIS ->
CreateProposalResponse -> CreateSignedTx, protoutil/{proputils,txutils}.go) and signed with
the reference's own sample signer (sampleconfig/msp: SampleOrg, signcerts/peer.pem +
keystore/key.pem -- the identity `msptesttools.LoadMSPSetupForTesting` gives those tests).
The EXPECTED codes are the reference tests' assertions, not our oracle's output:

  core/committer/txvalidator/v20/validator_test.go
    :198 TestInvokeBadRWSet           results "barf"                      -> BAD_RWSET (22)
    :212 TestInvokeNoPolicy           chaincode with an empty policy      -> INVALID_CHAINCODE (25)
    :231 TestInvokeOK                 SignedByAnyMember([SampleOrg])      -> VALID
    :252 TestInvokeNOKDuplicateNs     two NsReadWriteSets for "mycc"       -> ILLEGAL_WRITESET (23)
    :1031 TestDuplicateTxId           TxIDExists -> true                  -> DUPLICATE_TXID (9)
    :1059 TestValidationInvalidEndorsing  the plugin rejects the endorsement -> ENDORSEMENT_POLICY_FAILURE (10)
          (modelled by a policy the endorser cannot satisfy: SignedByAnyMember([OtherOrg]))
  core/common/validation/fullflow_test.go  (ValidateTransaction level: "passes" = no code of
        msgvalidation.go -- BAD_PAYLOAD 2, BAD_COMMON_HEADER 3, BAD_CREATOR_SIGNATURE 4,
        INVALID_ENDORSER_TRANSACTION 5, BAD_PROPOSAL_TXID 8 -- is produced)
    :111 TestGoodPath                 "simulation_result" results, cc foo/v1 -> passes ValidateTransaction
    :162 TestTXWithTwoActionsRejected two TransactionActions              -> not VALID
    :213 TestBadTx                    every payload byte +1 (mod 255); a corrupted signature -> not VALID
    :272 Test2EndorsersAgree          two endorsements of the same response -> passes ValidateTransaction
  core/handlers/validation/builtin/v20/validation_logic_test.go:50-74 createTx(endorsedByDuplicatedIdentity)
        the same endorsement twice: the duplicated identity counts once (SignatureSetToValidIdentities)
        -> VALID under 1-of SampleOrg, ENDORSEMENT_POLICY_FAILURE under 2-of SampleOrg
  common/cauthdsl/cauthdsl_test.go:98-163 (signers = ["signer0", "signer1"]; each list element is a
        distinct identity of MSP "signer<i>" -- the mock principal match is on identity bytes, the
        evaluation sees the list as given)
    TestSimpleSignature  SignedBy(0): [s0] ok, [s1] fail
    TestMultipleSignature  And(0,1): [s0,s1] ok, [s0,s0] fail
    TestComplexNestedSignature  And(Or(And(0,1),And(0,0)),0): [s0,s1,s0] ok, [s0,s0,s0] ok, [s0,s1] fail,
        [s0,s1,s1] fail
    TestNegatively  And(SignedBy(-1), SignedBy(-2)) fails to compile -> evaluation error -> 10
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from fabric_amd import synth  # noqa: E402
from fabric_amd.synth.blocks import (f_bytes, f_msg, f_str, f_varint, kv_rwset, msp_role_principal,  # noqa: E402
                                     n_out_of, serialized_identity, signed_by, tx_rwset)
from tests.x509min import _kids, _tlv, cert_info, pem_to_der  # noqa: E402

REF = "/root/reference"
CHANNEL = "testchannelid"
VT_CODES = [2, 3, 4, 5, 8]


class Signer:
    def __init__(self, mspid, pem, priv):
        self.mspid, self.pem, self.priv = mspid, pem, priv
        self.ser = serialized_identity(mspid, pem)
        der = pem_to_der(pem)
        self.pub = cert_info(der)["pub"]
        self.id_digest = hashlib.sha256(der).digest()

    def sign(self, msg):
        return synth.sign(self, hashlib.sha256(msg).digest())


def sample_signer():
    """SampleOrg's signer: sampleconfig/msp signcerts/peer.pem + keystore/key.pem (PKCS#8)"""
    pem = open(f"{REF}/sampleconfig/msp/signcerts/peer.pem", "rb").read()
    kpem = open(f"{REF}/sampleconfig/msp/keystore/key.pem", "rb").read()
    import base64
    der = base64.b64decode(b"".join(kpem.split(b"-----")[2].split()))
    _, co, cl = _tlv(der, 0)
    pki = _kids(der, co, cl)                     # PrivateKeyInfo {version, algorithm, privateKey}
    inner = der[pki[2][1]:pki[2][1] + pki[2][2]]  # ECPrivateKey
    _, co, cl = _tlv(inner, 0)
    ec = _kids(inner, co, cl)
    d = inner[ec[1][1]:ec[1][1] + ec[1][2]]
    return Signer("SampleOrg", pem, d.rjust(32, b"\0"))


def synthetic_signer(mspid, idx):
    k = synth.Key(20231016, idx)
    ca = synth.Key(20231016, 1000 + idx)
    pem = synth.make_cert(k, ca, "signer%d" % idx, mspid, "ca." + mspid, False, 500 + idx)
    return Signer(mspid, pem, k.priv)


def signed_by_any_member(mspids):
    """policydsl.SignedByAnyMember -> ApplicationPolicy{signature_policy} bytes"""
    spe = f_msg(2, n_out_of(1, [signed_by(i) for i in range(len(mspids))])) + \
        b"".join(f_msg(3, msp_role_principal(m)) for m in mspids)
    return f_msg(1, spe)


def n_of_members(n, mspids):
    spe = f_msg(2, n_out_of(n, [signed_by(i) for i in range(len(mspids))])) + \
        b"".join(f_msg(3, msp_role_principal(m)) for m in mspids)
    return f_msg(1, spe)


def sig_rule(rule_bytes, mspids):
    """ApplicationPolicy from a SignaturePolicy rule (policydsl.And/Or/SignedBy shape)"""
    return f_msg(1, f_msg(2, rule_bytes) + b"".join(f_msg(3, msp_role_principal(m)) for m in mspids))


def AND(a, b):
    return n_out_of(2, [a, b])


def OR(a, b):
    return n_out_of(1, [a, b])


def SB(i):
    return signed_by(i) if i >= 0 else f_varint(1, i & 0xFFFFFFFFFFFFFFFF)


def make_tx(creator, endorsers, cc=("mycc", "1.0"), results=None, events=b"", two_actions=False, nonce=None,
            dup_endorsement=False):
    """CreateProposalFromCIS + CreateProposalResponse (one per endorser, same response) + CreateSignedTx"""
    name, version = cc
    nonce = nonce or hashlib.sha256(b"nonce" + creator.ser + name.encode()).digest()[:24]
    cis = f_msg(1, f_varint(1, 1) + f_msg(2, f_str(2, name) + f_str(3, version)) + f_msg(3, f_bytes(1, b"func")))
    ccpp = f_bytes(1, cis)                                     # ChaincodeProposalPayload{input}
    txid = hashlib.sha256(nonce + creator.ser).hexdigest()
    ext = f_msg(2, f_str(2, name) + f_str(3, version))         # ChaincodeHeaderExtension{chaincode_id}
    chdr = f_varint(1, 3) + f_msg(3, f_varint(1, 1_700_000_000)) + f_str(4, CHANNEL) + f_str(5, txid) + f_bytes(7, ext)
    shdr = f_bytes(1, creator.ser) + f_bytes(2, nonce)
    if results is None:
        results = tx_rwset([(name, kv_rwset([], [("key", b"value", False)]))])  # createRWset(ccID)
    cca = f_bytes(1, results) + f_bytes(2, events) + f_msg(3, f_varint(1, 200)) + f_msg(4, f_str(2, name) + f_str(3, version))
    prp = f_bytes(1, hashlib.sha256(chdr + shdr + ccpp).digest()) + f_bytes(2, cca)
    ends = b""
    for e in endorsers:
        end = f_msg(2, f_bytes(1, e.ser) + f_bytes(2, e.sign(prp + e.ser)))
        ends += end + (end if dup_endorsement else b"")
    action = f_msg(1, f_bytes(1, shdr) + f_bytes(2, f_bytes(1, ccpp) + f_msg(2, f_bytes(1, prp) + ends)))
    if two_actions:
        action = action + action
    payload = f_msg(1, f_bytes(1, chdr) + f_bytes(2, shdr)) + f_bytes(2, action)
    return dict(payload=payload, sig=creator.sign(payload), txid=txid)


def env(tx, payload=None, sig=None):
    return f_bytes(1, payload if payload is not None else tx["payload"]) + f_bytes(2, sig if sig is not None else tx["sig"])


def block(envs, number=2):
    header = f_varint(1, number) + f_bytes(2, b"\0" * 32) + f_bytes(3, hashlib.sha256(b"".join(envs)).digest())
    return f_msg(1, header) + f_msg(2, b"".join(f_msg(1, e) for e in envs)) + f_msg(3, b"".join(f_msg(1, b"") for _ in range(5)))


def ident_json(s, roles=None):
    return dict(ser=s.ser.hex(), mspid=s.mspid, pub=s.pub.hex(), id_digest=s.id_digest.hex(),
                roles=roles if roles is not None else 1)


def main():
    so = sample_signer()
    other = synthetic_signer("OtherOrg", 0)
    cases = []

    idpool = {}

    def case(name, source, txs, expected, chaincodes, committed=(), identities=None, mutate=None):
        ids = identities or [ident_json(so), ident_json(other)]
        for i in ids:
            idpool[i["id_digest"]] = i
        c = dict(name=name, source=source, channel=CHANNEL, expected=expected,
                 chaincodes={k: v.hex() for k, v in chaincodes.items()}, committed=list(committed),
                 identities=[i["id_digest"] for i in ids])
        if mutate is None:
            c["block"] = block([env(t) for t in txs]).hex()
        else:
            c.update(mutate)
        cases.append(c)

    any_so = signed_by_any_member(["SampleOrg"])
    cases_cc = {"mycc": any_so}
    case("TestInvokeBadRWSet", "core/committer/txvalidator/v20/validator_test.go:198",
         [make_tx(so, [so], results=b"barf")], [22], cases_cc)
    case("TestInvokeNoPolicy", "validator_test.go:212", [make_tx(so, [so])], [25], {"mycc": b""})
    case("TestInvokeOK", "validator_test.go:231", [make_tx(so, [so])], [0], cases_cc)
    dup_ns = tx_rwset([("mycc", kv_rwset([], [("foo", b"bar1", False)])), ("mycc", kv_rwset([], [("foo", b"bar2", False)]))])
    case("TestInvokeNOKDuplicateNs", "validator_test.go:252", [make_tx(so, [so], results=dup_ns)], [23], cases_cc)
    t = make_tx(so, [so])
    case("TestDuplicateTxId", "validator_test.go:1031", [t], [9], cases_cc, committed=[t["txid"]])
    case("TestValidationInvalidEndorsing", "validator_test.go:1059", [make_tx(so, [so])], [10],
         {"mycc": signed_by_any_member(["OtherOrg"])})
    # fullflow (ValidateTransaction level)
    foo = {"foo": any_so}
    case("TestGoodPath", "core/common/validation/fullflow_test.go:111",
         [make_tx(so, [so], cc=("foo", "v1"), results=b"simulation_result")], ["passes_validate_transaction"], foo)
    case("TestTXWithTwoActionsRejected", "fullflow_test.go:162",
         [make_tx(so, [so], cc=("somename", "someversion"), results=b"simulation_result", two_actions=True)],
         ["not_valid"], foo)
    case("Test2EndorsersAgree", "fullflow_test.go:272",
         [make_tx(so, [so, so], cc=("foo", "v1"), results=b"simulation_result")], ["passes_validate_transaction"], foo)
    # the loader expands: payload byte i -> (b + 1) % 255 for every i, and the signature with one
    # byte decremented (fullflow_test.go corrupt())
    base = make_tx(so, [so], cc=("foo", "v1"))
    case("TestBadTx", "fullflow_test.go:213", [], "not_valid_each", {"foo": any_so},
         mutate=dict(bad_tx_payload=base["payload"].hex(), bad_tx_sig=base["sig"].hex()))
    # builtin v20: an endorsement duplicated by the same identity counts once
    dup = make_tx(so, [so], cc=("foo", "v1"), dup_endorsement=True)
    case("DuplicatedIdentity_1of", "core/handlers/validation/builtin/v20/validation_logic_test.go:50-74", [dup], [0],
         {"foo": n_of_members(1, ["SampleOrg"])})
    case("DuplicatedIdentity_2of", "validation_logic_test.go:50-74", [dup], [10], {"foo": n_of_members(2, ["SampleOrg"])})
    # cauthdsl: signer<i> -> distinct identities of MSP "signer<i>"
    pool = {0: [synthetic_signer("signer0", 10 + j) for j in range(3)], 1: [synthetic_signer("signer1", 20 + j) for j in range(3)]}

    def cauth(name, rule, lists):
        for li, (seq, ok) in enumerate(lists):
            used = {0: 0, 1: 0}
            ends = []
            for s in seq:
                ends.append(pool[s][used[s]])
                used[s] += 1
            ids = [ident_json(so)] + [ident_json(x) for xs in pool.values() for x in xs]
            case("%s_%d" % (name, li), "common/cauthdsl/cauthdsl_test.go:%s" % {"TestSimpleSignature": 98,
                 "TestMultipleSignature": 114, "TestComplexNestedSignature": 130, "TestNegatively": 152}[name],
                 [make_tx(so, ends)], [0 if ok else 10], {"mycc": sig_rule(rule, ["signer0", "signer1"])}, identities=ids)
    cauth("TestSimpleSignature", SB(0), [([0], True), ([1], False)])
    cauth("TestMultipleSignature", AND(SB(0), SB(1)), [([0, 1], True), ([0, 0], False)])
    cauth("TestComplexNestedSignature", AND(OR(AND(SB(0), SB(1)), AND(SB(0), SB(0))), SB(0)),
          [([0, 1, 0], True), ([0, 0, 0], True), ([0, 1], False), ([0, 1, 1], False)])
    cauth("TestNegatively", AND(SB(-1), SB(-2)), [([0, 1], False)])
    out = os.path.join(HERE, "committer_known_answers.json")
    json.dump(dict(vt_codes=VT_CODES, identities=idpool, cases=cases), open(out, "w"), indent=0)
    print(len(cases), "cases ->", out)


if __name__ == "__main__":
    main()
