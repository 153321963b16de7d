"""Key-level (state-based) endorsement known answers ported from the reference's own tests (run
in the build container; the output JSON is the committed fixture, the GPU box never reads
/root/reference).  Transactions are built as in make_committer_known_answers.py (protoutil's
proposal -> response -> signed tx shapes); the EXPECTED outcomes are the reference tests'
assertions, not our oracle's output ("not_valid" where the test only asserts IsInvalid).

  core/committer/txvalidator/v20/validator_test.go
    :435 TestParallelValidation   100 txs over keys "0".."9" (public, then collection col1):
         value writes, metadata (VALIDATION_PARAMETER) writes by a signer that fails the
         chaincode EP (SignedByMspPeer(Org1)), value writes after them (valid: the metadata
         writer was invalid), valid metadata writes, value writes after those (invalid:
         ValidationParameterUpdatedError).  Decades 1, 4, 6, 9 invalid, the rest valid.
    :918 TestValidateTxWithStateBasedEndorsement  the key's VALIDATION_PARAMETER is a marshalled
         ApplicationPolicy{RejectAllPolicy} -- translated as a SignaturePolicyEnvelope it has no
         rule -> ENDORSEMENT_POLICY_FAILURE
    :689 TestInvokeOKMetaUpdateOnly     a metadata-only write, endorser fails the EP -> 10
    :718 TestInvokeOKPvtMetaUpdateOnly  a hashed metadata-only write in a collection -> 10
  core/common/validation/statebased/validator_keylevel_test.go (their two-tx blocks, at block
  level: tx 0 writes the key's metadata and its vscc fails (PostValidate with an error), tx 1's
  vscc then evaluates the key's parameter from state: passes (NoError) / fails (policy error))
    :82 TestKeylevelValidation, :123 TestKeylevelValidationPvtData, :161 ...MetaUpdate,
    :199 ...PvtMetaUpdate
  core/common/validation/statebased/vpmanager_test.go
    :267 TestDependencyNoConflict  the earlier metadata writer's validation failed -> no conflict
    :310 TestDependencyConflict    the earlier metadata writer validated -> the later tx fails
    :453 / :491 the same for a private key (by key hash)
    :664 TestWritesIntoDifferentNamespaces  a metadata write in another namespace is no conflict
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from fabric_amd.synth.blocks import f_bytes, f_msg, f_str, kv_rwset, msp_role_principal, n_out_of, signed_by  # noqa: E402
from make_committer_known_answers import (block, env, ident_json, make_tx, sample_signer,  # noqa: E402
                                          signed_by_any_member, synthetic_signer)

VP = "VALIDATION_PARAMETER"
PEER = 3


def spe(rule, principals):
    """SignaturePolicyEnvelope{version 0, rule, identities}"""
    return f_msg(2, rule) + b"".join(f_msg(3, p) for p in principals)


def app(spe_bytes):
    return f_msg(1, spe_bytes)


def signed_by_msp_peer(mspid):  # policydsl.SignedByMspPeer
    return spe(n_out_of(1, [signed_by(0)]), [msp_role_principal(mspid, PEER)])


def any_member_spe(mspids):  # policydsl.SignedByAnyMember
    return spe(n_out_of(1, [signed_by(i) for i in range(len(mspids))]), [msp_role_principal(m) for m in mspids])


REJECT_ALL = spe(n_out_of(1, []), [])  # policydsl.RejectAllPolicy


def entries(md):
    return b"".join(f_msg(2, f_str(1, k) + f_bytes(2, v)) for k, v in md.items())


def ns_rwset(writes=(), meta=(), pvt_writes=(), pvt_meta=(), coll=None):
    """KVRWSet with writes [(key, value)] and metadata writes [(key, {name: value})]; a collection's
    HashedRWSet with hashed writes [(key, value)] / metadata writes [(key, md)] (keys hashed)"""
    kv = kv_rwset([], [(k, v, False) for k, v in writes])
    for k, md in meta:
        kv += f_msg(4, f_str(1, k) + entries(md))
    colls = []
    if pvt_writes or pvt_meta:
        h = b""
        for k, v in pvt_writes:
            h += f_msg(2, f_bytes(1, hashlib.sha256(k.encode()).digest()) + f_bytes(3, hashlib.sha256(v).digest()))
        for k, md in pvt_meta:
            h += f_msg(3, f_bytes(1, hashlib.sha256(k.encode()).digest()) + entries(md))
        colls.append((coll, h))
    return kv, colls


def txrw(ns, kv, colls=()):
    return f_msg(2, f_str(1, ns) + f_bytes(2, kv) + b"".join(f_msg(3, f_str(1, c) + f_bytes(2, h)) for c, h in colls))


def main():
    cases, idpool = [], {}

    def case(name, source, txs, expected, chaincodes, identities, kvmeta=()):
        for i in identities:
            idpool[i["id_digest"]] = i
        cases.append(dict(
            name=name, source=source, expected=expected, identities=[i["id_digest"] for i in identities],
            chaincodes={ns: dict(policy=d["policy"].hex(),
                                 collections=None if d.get("collections") is None else
                                 {c: (ep.hex() if ep else None) for c, ep in d["collections"].items()})
                        for ns, d in chaincodes.items()},
            kvmeta=[[ns, coll, key.hex(), vp.hex()] for ns, coll, key, vp in kvmeta],
            block=block([env(t) for t in txs]).hex()))

    n = [0]

    def tx(creator, endorsers, rw, cc="mycc"):
        n[0] += 1
        return make_tx(creator, endorsers, cc=(cc, "1.0"), results=rw,
                       nonce=hashlib.sha256(b"sbe-%d" % n[0]).digest()[:24])

    # --- TestParallelValidation
    s0, s1 = synthetic_signer("Org1", 40), synthetic_signer("Org2", 41)
    ids01 = [ident_json(s0, roles=(1 << 0) | (1 << PEER)), ident_json(s1, roles=1)]
    ccs = {"mycc": dict(policy=app(signed_by_msp_peer("Org1")), collections={"col1": None})}
    txs, exp = [], []
    for t in range(100):
        key = str(t % 10)
        d = t // 10
        md_so = {VP: app(any_member_spe(["SampleOrg"]))}
        md_o2 = {VP: app(any_member_spe(["Org2"]))}
        if d == 0:
            kv, co = ns_rwset(writes=[(key, b"value1")]); sig = s0
        elif d == 1:
            kv, co = ns_rwset(meta=[(key, md_so)]); sig = s1
        elif d == 2:
            kv, co = ns_rwset(writes=[(key, b"value2")]); sig = s0
        elif d == 3:
            kv, co = ns_rwset(meta=[(key, md_o2)]); sig = s0
        elif d == 4:
            kv, co = ns_rwset(writes=[(key, b"value3")]); sig = s0
        elif d == 5:
            kv, co = ns_rwset(pvt_writes=[(key, b"value1")], coll="col1"); sig = s0
        elif d == 6:
            kv, co = ns_rwset(pvt_meta=[(key, md_so)], coll="col1"); sig = s1
        elif d == 7:
            kv, co = ns_rwset(pvt_writes=[(key, b"value2")], coll="col1"); sig = s0
        elif d == 8:
            kv, co = ns_rwset(pvt_meta=[(key, md_o2)], coll="col1"); sig = s0
        else:
            kv, co = ns_rwset(pvt_writes=[(key, b"value3")], coll="col1"); sig = s0
        txs.append(tx(sig, [sig], txrw("mycc", kv, co)))
        exp.append("not_valid" if d in (1, 4, 6, 9) else 0)
    case("TestParallelValidation", "core/committer/txvalidator/v20/validator_test.go:435", txs, exp, ccs, ids01)

    so, other = sample_signer(), synthetic_signer("OtherOrg", 0)
    ids_so = [ident_json(so), ident_json(other)]
    any_so = {"mycc": dict(policy=signed_by_any_member(["SampleOrg"]))}
    key_rw = txrw("mycc", kv_rwset([], [("key", b"value", False)]))
    case("TestValidateTxWithStateBasedEndorsement", "validator_test.go:918", [tx(so, [so], key_rw)], [10], any_so,
         ids_so, kvmeta=[("mycc", "", b"key", app(REJECT_ALL))])
    fail_ep = {"mycc": dict(policy=signed_by_any_member(["OtherOrg"]), collections={"mycollection": None})}
    kv, _ = ns_rwset(meta=[("somekey", {})])
    case("TestInvokeOKMetaUpdateOnly", "validator_test.go:689", [tx(so, [so], txrw("mycc", kv))], [10], fail_ep, ids_so)
    kv, co = ns_rwset(pvt_meta=[("somekey", {})], coll="mycollection")
    case("TestInvokeOKPvtMetaUpdateOnly", "validator_test.go:718", [tx(so, [so], txrw("mycc", kv, co))], [10], fail_ep,
         ids_so)

    # --- validator_keylevel_test.go, block level.  CC EP: SampleOrg member; `other` fails it.
    # The key's parameter in state: satisfied by `other` (EP) or by nobody (REJECT).
    ccs_k = {"cc": dict(policy=signed_by_any_member(["SampleOrg"]), collections={"coll": None})}
    kh = hashlib.sha256(b"key").digest()
    ep_other = any_member_spe(["OtherOrg"])
    md_write = txrw("cc", ns_rwset(meta=[("key", {VP: ep_other})])[0])
    for tname, line, (kv, co), pvt in [
            ("TestKeylevelValidation", 82, ns_rwset(writes=[("key", b"v")]), False),
            ("TestKeylevelValidationPvtData", 123, ns_rwset(pvt_writes=[("key", b"value")], coll="coll"), True),
            ("TestKeylevelValidationMetaUpdate", 161, ns_rwset(meta=[("key", {})]), False),
            ("TestKeylevelValidationPvtMetaUpdate", 199, ns_rwset(pvt_meta=[("key", {})], coll="coll"), True)]:
        coll, key = ("coll", kh) if pvt else ("", b"key")
        for vp, code, sfx in [(ep_other, 0, "ok"), (REJECT_ALL, 10, "policy_error")]:
            # tx 0: metadata write without endorsements -> its vscc fails (error result)
            t0 = tx(so, [], md_write, cc="cc")
            t1 = tx(so, [other], txrw("cc", kv, co), cc="cc")
            case("%s_%s" % (tname, sfx), "core/common/validation/statebased/validator_keylevel_test.go:%d" % line,
                 [t0, t1], [10, code], ccs_k, ids_so, kvmeta=[("cc", coll, key, vp)])

    # --- vpmanager_test.go dependencies (no parameters in state; CC EP = SampleOrg member)
    for tname, line, pvt in [("TestDependencyNoConflict", 267, False), ("TestDependencyConflict", 310, False),
                             ("TestPvtDependencyNoConflict", 453, True), ("TestPvtDependencyConflict", 491, True)]:
        conflict = "NoConflict" not in tname
        if pvt:
            mw = txrw("cc", *ns_rwset(pvt_meta=[("key", {VP: ep_other})], coll="coll"))
            w = txrw("cc", *ns_rwset(pvt_writes=[("key", b"v")], coll="coll"))
        else:
            mw = txrw("cc", ns_rwset(meta=[("key", {VP: ep_other})])[0])
            w = txrw("cc", ns_rwset(writes=[("key", b"v")])[0])
        t0 = tx(so, [so] if conflict else [other], mw, cc="cc")  # validates / fails
        t1 = tx(so, [so], w, cc="cc")
        case(tname, "core/common/validation/statebased/vpmanager_test.go:%d" % line, [t0, t1],
             [0, 10] if conflict else [10, 0], ccs_k, ids_so)
    # a metadata write of the same key in ANOTHER namespace is no dependency
    ccs_2 = dict(ccs_k, cc2=dict(policy=signed_by_any_member(["SampleOrg"])))
    t0 = tx(so, [so], txrw("cc2", ns_rwset(meta=[("key", {VP: ep_other})])[0]), cc="cc2")
    t1 = tx(so, [so], txrw("cc", ns_rwset(writes=[("key", b"v")])[0]), cc="cc")
    case("TestWritesIntoDifferentNamespaces", "core/common/validation/statebased/vpmanager_test.go:664", [t0, t1],
         [0, 0], ccs_2, ids_so)

    out = os.path.join(HERE, "sbe_known_answers.json")
    json.dump(dict(identities=idpool, cases=cases), open(out, "w"), indent=0)
    print(len(cases), "cases ->", out)


if __name__ == "__main__":
    main()
