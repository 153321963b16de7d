"""Restated committer validation of one block (TEST INFRASTRUCTURE ONLY -- the oracle).

Follows, line by line in behaviour (citations under /root/reference):
  core/committer/txvalidator/v20/validator.go:180-265   Validate: per-tx codes, halt on the
        lowest-index execution error, markTXIdDuplicates (:279-295, VALID txs only)
  validator.go:297-453                                    validateTx code precedence
  core/common/validation/msgvalidation.go:26-320          ValidateTransaction & helpers
  protoutil/proputils.go:351-370 (CheckTxID), protoutil/txutils.go:449-466 (GetProposalHash2),
  protoutil/proputils.go:198-223 + txutils.go:21-46 (GetActionFromEnvelope / GetPayloads)
  core/committer/txvalidator/v20/plugindispatcher/dispatcher.go:102-302  Dispatch
  core/handlers/validation/builtin/v20/validation_logic.go:109-217       builtin vscc v20
  core/common/validation/statebased/validator_keylevel.go:38-282, v20.go:105-167
        (no key-level validation parameters in the modelled state -> the chaincode EP is
         evaluated once per written namespace)
  core/policy/application.go:148-163, common/cauthdsl/cauthdsl.go:24-92, policy.go:86-108
  common/policies/policy.go:363-395   SignatureSetToValidIdentities (dedup before verify,
        insert after successful verify, order preserved)
  msp/identities.go:170-199           identity.Verify = SHA-256 + bccsp Verify (fgv_oracle.c)

Modelled environment (the same one the engine is configured with):
  * one channel; its MSP = a registry of identities keyed by the exact (mspid, id_bytes) pair
    of a SerializedIdentity, each with its P-256 key, Validate() result and identity digest
    (Id = hex SHA-256 of the certificate); unknown pairs fail DeserializeIdentity;
  * chaincode definitions: namespace -> ApplicationPolicy bytes (lifecycle ValidationInfo);
  * the ledger's committed txids (TxIDExists).
Anything outside that model raises Unsupported (the engine returns an error for such blocks).
"""
import hashlib

from . import sha256, verify_der
from .protowire import DecodeError, decode

VALID, NIL_ENVELOPE, BAD_PAYLOAD, BAD_COMMON_HEADER, BAD_CREATOR_SIGNATURE = 0, 1, 2, 3, 4
INVALID_ENDORSER_TRANSACTION, INVALID_CONFIG_TRANSACTION, UNSUPPORTED_TX_PAYLOAD = 5, 6, 7
BAD_PROPOSAL_TXID, DUPLICATE_TXID, ENDORSEMENT_POLICY_FAILURE = 8, 9, 10
UNKNOWN_TX_TYPE, TARGET_CHAIN_NOT_FOUND = 13, 14
BAD_HEADER_EXTENSION, BAD_CHANNEL_HEADER, BAD_RESPONSE_PAYLOAD, BAD_RWSET = 19, 20, 21, 22
ILLEGAL_WRITESET, INVALID_CHAINCODE, INVALID_OTHER_REASON = 23, 25, 255
ENDORSER_TRANSACTION, CONFIG, CONFIG_UPDATE = 3, 1, 2


class Unsupported(Exception):
    """Input outside the modelled environment (config tx, channel-reference policy, ...)."""


class Ident:
    def __init__(self, mspid, pub, valid, id_digest):
        self.mspid, self.pub, self.valid, self.id_digest = mspid, pub, valid, id_digest

    @property
    def dedup_key(self):  # identity.GetIdentifier().Mspid + .Id
        return self.mspid + self.id_digest.hex()


class ChannelModel:
    def __init__(self, channel, identities, chaincodes, committed_txids=()):
        """identities: iterable of (serialized, mspid, pub64, valid, id_digest)."""
        self.channel = channel
        self.msp = {}
        self.mspids = set()
        for ser, mspid, pub, valid, dig in identities:
            sid = decode("SerializedIdentity", ser)
            self.msp[(sid.get("mspid", ""), sid.get("id_bytes") or b"")] = Ident(mspid, pub, valid, dig)
            self.mspids.add(mspid)
        self.chaincodes = dict(chaincodes)
        self.committed = set(committed_txids)
        self.verify_calls = 0

    def deserialize(self, ser):
        """mspManagerImpl.DeserializeIdentity (msp/mspmgrimpl.go:75-100) over the registry."""
        try:
            sid = decode("SerializedIdentity", ser)
        except DecodeError:
            return None
        return self.msp.get((sid.get("mspid", ""), sid.get("id_bytes") or b""))

    def verify(self, ident, msg, sig):
        """identity.Verify: 0 iff valid (msp/identities.go:170-199)."""
        self.verify_calls += 1
        if not sig:
            return 6
        return verify_der(ident.pub[:32], ident.pub[32:], sig, sha256(msg))


# ----------------------------------------------------------------- policies

def _compile(rule, principals):
    """cauthdsl.compile (common/cauthdsl/cauthdsl.go:24-92); returns closure or raises ValueError."""
    if rule is None:
        raise ValueError("Empty policy element")
    if "n_out_of" in rule:
        noo = rule["n_out_of"]
        subs = [_compile(r, principals) for r in noo.get("rules", [])]
        n = noo.get("n", 0)

        def gate(ids, used):
            verified = 0
            for p in subs:
                _used = list(used)
                if p(ids, _used):
                    verified += 1
                    used[:] = _used
            return verified >= n
        return gate
    if "signed_by" in rule:
        idx = rule["signed_by"]
        if idx < 0 or idx >= len(principals):
            raise ValueError("identity index out of range")
        pr = principals[idx]

        def signed(ids, used):
            for i, ident in enumerate(ids):
                if used[i]:
                    continue
                if _satisfies(ident, pr):
                    used[i] = True
                    return True
            return False
        return signed
    raise ValueError("Unknown type")


def _principal(p):
    cls = p.get("principal_classification", 0)
    if cls != 0:
        raise Unsupported("principal classification %d" % cls)
    try:
        role = decode("MSPRole", p.get("principal") or b"")
    except DecodeError:
        return ("bad", None)
    if role.get("role", 0) != 0:
        raise Unsupported("MSP role %d needs NodeOU data" % role.get("role", 0))
    return ("member", role.get("msp_identifier", ""))


def _satisfies(ident, pr):
    """bccspmsp.satisfiesPrincipalInternal* for ROLE/MEMBER (msp/mspimpl.go:477-501)."""
    kind, mspid = pr
    if kind != "member":
        return False
    return ident.mspid == mspid and ident.valid


def signature_set_to_valid_identities(model, sigset):
    """common/policies/policy.go:363-395."""
    seen, out = set(), []
    for data, ident_bytes, sig in sigset:
        ident = model.deserialize(ident_bytes)
        if ident is None:
            continue
        if ident.dedup_key in seen:
            continue
        if model.verify(ident, data, sig) != 0:
            continue
        seen.add(ident.dedup_key)
        out.append(ident)
    return out


def evaluate_policy(model, policy_bytes, sigset):
    """ApplicationPolicyEvaluator.Evaluate (core/policy/application.go:148-163).  True iff ok."""
    try:
        ap = decode("ApplicationPolicy", policy_bytes)
    except DecodeError:
        return False
    if "signature_policy" in ap:
        spe = ap["signature_policy"]
        principals = [_principal(p) for p in spe.get("identities", [])]
        try:
            ev = _compile(spe.get("rule"), principals)
        except ValueError:
            return False
        ids = signature_set_to_valid_identities(model, sigset)
        return ev(ids, [False] * len(ids))
    if "channel_config_policy_reference" in ap:
        raise Unsupported("channel config policy reference")
    return False


# ----------------------------------------------------------------- msgvalidation

def _validate_endorser_transaction(data, hdr):
    """msgvalidation.go:165-245 -> True iff ok."""
    if not data or hdr is None:  # data nil (proto3 empty == nil)
        return False
    try:
        tx = decode("Transaction", data)
    except DecodeError:
        return False
    acts = tx.get("actions", [])
    if len(acts) != 1:
        return False
    act = acts[0]
    try:
        shdr = decode("SignatureHeader", act.get("header"))
    except DecodeError:
        return False
    if not shdr.get("nonce") or not shdr.get("creator"):
        return False
    try:
        cap = decode("ChaincodeActionPayload", act.get("payload"))
    except DecodeError:
        return False
    if "action" not in cap:
        raise Unsupported("nil ChaincodeEndorsedAction dereference (reference panics)")
    try:
        prp = decode("ProposalResponsePayload", cap["action"].get("proposal_response_payload"))
    except DecodeError:
        return False
    ch, sh, ccpp = hdr.get("channel_header"), act.get("header"), cap.get("chaincode_proposal_payload")
    if ch is None or sh is None or ccpp is None:
        return False
    ph = hashlib.sha256(ch + sh + ccpp).digest()
    return ph == (prp.get("proposal_hash") or b"")


def validate_transaction(model, env):
    """msgvalidation.go:248-320 -> (payload Msg or None, hdrs, code)."""
    try:
        payload = decode("Payload", env.get("payload"))
    except DecodeError:
        return None, None, BAD_PAYLOAD
    hdr = payload.get("header")
    if hdr is None:
        return None, None, BAD_COMMON_HEADER
    try:
        chdr = decode("ChannelHeader", hdr.get("channel_header"))
        shdr = decode("SignatureHeader", hdr.get("signature_header"))
    except DecodeError:
        return None, None, BAD_COMMON_HEADER
    if chdr.get("type", 0) not in (ENDORSER_TRANSACTION, CONFIG_UPDATE, CONFIG):
        return None, None, BAD_COMMON_HEADER
    if chdr.get("epoch", 0) != 0:
        return None, None, BAD_COMMON_HEADER
    if not shdr.get("nonce") or not shdr.get("creator"):
        return None, None, BAD_COMMON_HEADER
    # checkSignatureFromCreator (msgvalidation.go:26-64)
    creator, sig, msg = shdr["creator"], env.get("signature"), env.get("payload")
    if sig is None or msg is None:
        return None, None, BAD_CREATOR_SIGNATURE
    if chdr.get("channel_id", "") == "":
        raise Unsupported("empty channel id selects the peer's local MSP")
    ident = model.deserialize(creator) if chdr.get("channel_id", "") == model.channel else None
    if ident is None or not ident.valid:
        return None, None, BAD_CREATOR_SIGNATURE
    if model.verify(ident, msg, sig) != 0:
        return None, None, BAD_CREATOR_SIGNATURE
    t = chdr.get("type", 0)
    if t == ENDORSER_TRANSACTION:
        if chdr.get("tx_id", "") != hashlib.sha256(shdr["nonce"] + creator).hexdigest():
            return None, None, BAD_PROPOSAL_TXID
        if not _validate_endorser_transaction(payload.get("data"), hdr):
            return payload, (chdr, shdr), INVALID_ENDORSER_TRANSACTION
        return payload, (chdr, shdr), VALID
    if t == CONFIG:
        raise Unsupported("CONFIG transaction")
    return None, None, UNSUPPORTED_TX_PAYLOAD


# ----------------------------------------------------------------- dispatcher + vscc

def _writes_to_ns(ns):
    kv = ns.get("kv")
    if kv is not None and kv.get("writes"):
        return True
    for c in ns.get("coll", []):
        h = c.get("hashed")
        if h is not None and (h.get("hashed_writes") or h.get("metadata_writes")):
            return True
    return kv is not None and bool(kv.get("metadata_writes"))


def parse_rwset(results):
    """rwsetutil.TxRwSet.FromProtoBytes (core/ledger/kvledger/txmgmt/rwsetutil/rwset_proto_util.go:115-234)."""
    txrw = decode("TxReadWriteSet", results)
    out = []
    for ns in txrw.get("ns_rwset", []):
        kv = decode("KVRWSet", ns.get("rwset"))
        coll = []
        for c in ns.get("collection_hashed_rwset", []):
            coll.append({"name": c.get("collection_name", ""), "hashed": decode("HashedRWSet", c.get("hashed_rwset"))})
        out.append({"namespace": ns.get("namespace", ""), "kv": kv, "coll": coll})
    return out


def get_action_from_envelope(env_bytes):
    """protoutil.GetActionFromEnvelope -> ChaincodeAction Msg (raises DecodeError/ValueError)."""
    env = decode("Envelope", env_bytes)
    payl = decode("Payload", env.get("payload"))
    tx = decode("Transaction", payl.get("data"))
    if not tx.get("actions"):
        raise ValueError("at least one TransactionAction required")
    cap = decode("ChaincodeActionPayload", tx["actions"][0].get("payload"))
    if "action" not in cap or cap["action"].get("proposal_response_payload") is None:
        raise ValueError("no payload in ChaincodeActionPayload")
    prp = decode("ProposalResponsePayload", cap["action"]["proposal_response_payload"])
    if prp.get("extension") is None:
        raise ValueError("response payload is missing extension")
    return decode("ChaincodeAction", prp["extension"]), cap


def vscc_validate(model, env_bytes, ns, policy):
    """builtin v20 Validate (validation_logic.go:185-217) -> True iff endorsement policy holds."""
    try:
        env = decode("Envelope", env_bytes)
        payl = decode("Payload", env.get("payload"))
        chdr = decode("ChannelHeader", (payl.get("header") or {}).get("channel_header"))
        if chdr.get("type", 0) != ENDORSER_TRANSACTION:
            return False
        tx = decode("Transaction", payl.get("data"))
        cap = decode("ChaincodeActionPayload", tx["actions"][0].get("payload"))
        prp_bytes = cap["action"].get("proposal_response_payload")
        prp = decode("ProposalResponsePayload", prp_bytes)
        if prp.get("extension") is None:
            return False
        cca = decode("ChaincodeAction", prp["extension"])
    except (DecodeError, KeyError, IndexError):
        return False
    prp_bytes = prp_bytes or b""
    sigset = []
    for e in cap["action"].get("endorsements", []):
        endorser = e.get("endorser") or b""
        sigset.append((prp_bytes + endorser, endorser, e.get("signature")))
    try:
        rw = parse_rwset(cca.get("results"))
    except DecodeError:
        return False
    for nsrw in rw:
        if nsrw["namespace"] != ns:
            continue
        if nsrw["kv"].get("metadata_writes") or any(c["hashed"].get("metadata_writes") or c["hashed"].get("hashed_writes")
                                                   for c in nsrw["coll"]):
            raise Unsupported("key-level / collection endorsement policies")
    # without key-level validation parameters every write checks the chaincode EP once
    # (CheckCCEPIfNotChecked), and a namespace without writes checks it via
    # CheckCCEPIfNoEPChecked: one evaluation either way.
    return evaluate_policy(model, policy, sigset)


def dispatch(model, payload, env_bytes):
    """plugindispatcher.Dispatch (dispatcher.go:102-221) -> code."""
    chdr = decode("ChannelHeader", payload["header"].get("channel_header"))
    try:
        ext = decode("ChaincodeHeaderExtension", chdr.get("extension"))
    except DecodeError:
        return BAD_HEADER_EXTENSION
    try:
        cca, _ = get_action_from_envelope(env_bytes)
    except (DecodeError, ValueError):
        return BAD_RESPONSE_PAYLOAD
    try:
        rw = parse_rwset(cca.get("results"))
    except DecodeError:
        return BAD_RWSET
    if "chaincode_id" not in ext or "chaincode_id" not in cca:
        return INVALID_OTHER_REASON
    cc_id = ext["chaincode_id"].get("name", "")
    cc_ver = cca["chaincode_id"].get("version", "")
    if cc_id == "" or cc_id != cca["chaincode_id"].get("name", "") or cc_ver == "":
        return INVALID_CHAINCODE
    wr = [cc_id]
    if cca.get("events") is not None:
        try:
            ev = decode("ChaincodeEvent", cca["events"])
        except DecodeError:
            return INVALID_OTHER_REASON
        if ev.get("chaincode_id", "") != cc_id:
            return INVALID_OTHER_REASON
    seen = set()
    for nsrw in rw:
        if nsrw["namespace"] in seen:
            return ILLEGAL_WRITESET
        seen.add(nsrw["namespace"])
        if _writes_to_ns(nsrw) and nsrw["namespace"] not in wr:
            wr.append(nsrw["namespace"])
    # The reference iterates a Go map (random order).  Results only differ in the
    # reported code when namespaces fail with DIFFERENT codes; we report the first in
    # sorted order and flag multi-namespace disagreement as unsupported.
    for nsrw in rw:
        if nsrw["namespace"] in wr and (nsrw["kv"].get("metadata_writes") or any(
                c["hashed"].get("metadata_writes") or c["hashed"].get("hashed_writes") for c in nsrw["coll"])):
            raise Unsupported("key-level / collection endorsement policies")
    codes = set()
    for ns in sorted(wr):
        if ns not in model.chaincodes:
            codes.add(INVALID_CHAINCODE)
            continue
        if not vscc_validate(model, env_bytes, ns, model.chaincodes[ns]):
            codes.add(ENDORSEMENT_POLICY_FAILURE)
    if len(codes) > 1:
        raise Unsupported("namespaces fail with different codes (map-order dependent)")
    return codes.pop() if codes else VALID


# ----------------------------------------------------------------- block level

def validate_tx(model, d):
    """validator.go:297-453 -> (code, txid)."""
    try:
        env = decode("Envelope", d)
    except DecodeError:
        return INVALID_OTHER_REASON, ""
    payload, hdrs, code = validate_transaction(model, env)
    if code != VALID:
        return code, ""
    chdr, _ = hdrs
    # chainExists() is a stub returning true (validator.go:155-158)
    if chdr.get("type", 0) == ENDORSER_TRANSACTION:
        txid = chdr.get("tx_id", "")
        if txid in model.committed:
            return DUPLICATE_TXID, ""
        code = dispatch(model, payload, d)
        if code != VALID:
            return code, ""
        return VALID, txid
    return UNKNOWN_TX_TYPE, ""


def index_txid(d):
    """protoutil.GetOrComputeTxIDFromEnvelope (txutils.go:503-534); None on error."""
    try:
        env = decode("Envelope", d)
        payl = decode("Payload", env.get("payload"))
        if payl.get("header") is None:
            return None
        chdr = decode("ChannelHeader", payl["header"].get("channel_header"))
        if chdr.get("tx_id", ""):
            return chdr["tx_id"]
        shdr = decode("SignatureHeader", payl["header"].get("signature_header"))
        return hashlib.sha256((shdr.get("nonce") or b"") + (shdr.get("creator") or b"")).hexdigest()
    except DecodeError:
        return None


def validate_blocks(model, blocks):
    """Consecutive blocks: block k sees the txids indexed by blocks < k (blkstorage indexes
    every transaction's txid at commit, block_serialization.go:95-115)."""
    out = []
    for blk in blocks:
        out.append(validate_block(model, blk))
        data = (decode("Block", blk).get("data") or {}).get("data", [])
        for d in data:
            t = index_txid(d)
            if t:
                model.committed.add(t)
    return out


def validate_block(model, block_bytes):
    """TxValidator.Validate -> list of validation codes (TxValidationFlags)."""
    blk = decode("Block", block_bytes)
    data = (blk.get("data") or {}).get("data", [])
    flags, txids = [], []
    for d in data:
        code, txid = validate_tx(model, d)
        flags.append(code)
        txids.append(txid if code == VALID else "")
    seen = set()
    for i, t in enumerate(txids):  # markTXIdDuplicates
        if t == "":
            continue
        if t in seen:
            flags[i] = DUPLICATE_TXID
        else:
            seen.add(t)
    return flags
