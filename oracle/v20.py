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
  core/common/validation/statebased/validator_keylevel.go:38-282, v20.go:105-167,
        vpmanagerimpl.go:253-365  key-level (state-based) endorsement: each written key's
        VALIDATION_PARAMETER from committed state, the in-block dependency on an earlier tx's
        metadata write, the collection / chaincode EPs otherwise
  core/policy/application.go:148-163, common/cauthdsl/cauthdsl.go:24-92, policy.go:86-108
  common/policies/policy.go:363-395   SignatureSetToValidIdentities (dedup before verify,
        insert after successful verify, order preserved)
  msp/identities.go:170-199           identity.Verify = SHA-256 + bccsp Verify (fgv_oracle.c)

Modelled environment (the same one the engine is configured with):
  * one channel; its MSP = a registry of identities keyed by the exact (mspid, id_bytes) pair
    of a SerializedIdentity, each with its P-256 key, Validate() result and identity digest
    (Id = hex SHA-256 of the certificate); unknown pairs fail DeserializeIdentity;
  * chaincode definitions: namespace -> ApplicationPolicy bytes (lifecycle ValidationInfo);
  * the ledger's committed txids (TxIDExists);
  * the committed state's key-level validation parameters: (ns, coll, key bytes) -> the
    VALIDATION_PARAMETER metadata value (GetStateMetadata / GetPrivateDataMetadataByHash).
Anything outside that model raises Unsupported (the engine returns an error for such blocks).
"""
import hashlib

from . import sha256, verify_der, verify_der_p384
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


class ConfigTransaction(Unsupported):
    """A CONFIG transaction that reaches ChannelResources.Apply (validator.go:397-420): the
    channel's configuration (MSPs, policies) changes for every later block."""


KEY_P256, KEY_P384, KEY_OTHER, KEY_UNDESERIALIZABLE = "p256", "p384", "other", "undeserializable"
IMPLICIT_PREFIX = "_implicit_org_"  # core/chaincode/implicitcollection/name.go:24-29


class Ident:
    """An MSP identity as the peer's MSP layer knows it.
    key: KEY_P256 (verified on the GPU), KEY_P384 (pub = X || Y, 96 bytes: verified like P-256 with
    the P-384 constants; without pub, outside the engine -> Unsupported when a verify is needed), KEY_OTHER (RSA...: Verify fails),
    KEY_UNDESERIALIZABLE (e.g. Ed25519 under Fabric 2.x: DeserializeIdentity fails, F4).
    hash: the MSP's SignatureHashFamily (identities.go:219-227): SHA2 -> SHA-256, SHA3 -> SHA3-256.
    roles: bit r <=> msp.SatisfiesPrincipal(id, ROLE{mspid, r}) (MEMBER 0, ADMIN 1, CLIENT 2,
    PEER 3, ORDERER 4; msp/mspimpl.go:331-376, 477-660); None = unknown (legacy registration)."""

    def __init__(self, mspid, pub, valid, id_digest, key=KEY_P256, hash_family="SHA2", roles=None, ous=None):
        self.mspid, self.pub, self.valid, self.id_digest = mspid, pub, valid, id_digest
        self.key, self.hash_family, self.roles = key, hash_family, roles
        # GetOrganizationalUnits (msp/identities.go:121-145): [(OU identifier, certifiers
        # identifier bytes)], None = unknown (a registration without them)
        self.ous = None if ous is None else [(o, bytes(c)) for o, c in ous]

    @property
    def dedup_key(self):  # identity.GetIdentifier().Mspid + .Id
        return self.mspid + self.id_digest.hex()


class ChannelPolicy:
    """A policy of the channel configuration (common/policies/policy.go ManagerImpl)."""
    REJECT, SIGNATURE, IMPLICIT_META, UNSUPPORTED = range(4)

    def __init__(self, kind, spe=None, threshold=0, subs=()):
        self.kind, self.spe, self.threshold, self.subs = kind, spe, threshold, list(subs)


def _config_policies(group, path, out, msps, app_orgs, is_app=False):
    """Walk a ConfigGroup: flattened policies {"Application/org1/Endorsement": ChannelPolicy}
    (ManagerImpl folds sub-manager policies into its map under "group/name", policy.go), MSPs
    {name: FabricMSPConfig}, application orgs {mspid: org group name}."""
    children = [(e.get("key", ""), e.get("value") or {}) for e in group.get("groups", [])]
    for e in group.get("values", []):
        if e.get("key") == "MSP":
            mc = decode("MSPConfig", (e.get("value") or {}).get("value"))
            if mc.get("type", 0) != 0:
                raise Unsupported("non-X.509 MSP")
            fc = decode("FabricMSPConfig", mc.get("config"))
            msps[fc.get("name", "")] = fc
            if is_app:
                app_orgs[fc.get("name", "")] = path.rsplit("/", 1)[-1]
    for e in group.get("policies", []):
        name = e.get("key", "")
        pol = (e.get("value") or {}).get("policy") or {}
        t = pol.get("type", 0)
        key = (path + "/" + name) if path else name
        if t == 1:  # SIGNATURE: cauthdsl.NewPolicy (policy.go): version 0 only
            spe = decode("SignaturePolicyEnvelope", pol.get("value"))
            out[key] = ChannelPolicy(ChannelPolicy.SIGNATURE if spe.get("version", 0) == 0 else ChannelPolicy.UNSUPPORTED, spe=spe)
        elif t == 3:  # IMPLICIT_META (implicitmeta.go:27-60): one sub-policy per child group
            im = decode("ImplicitMetaPolicy", pol.get("value"))
            rule, sub = im.get("rule", 0), im.get("sub_policy", "")
            subs = [((path + "/" + c + "/" + sub) if path else (c + "/" + sub)) for c, _ in children]
            n = len(subs)
            thr = 1 if rule == 0 else n if rule == 1 else n // 2 + 1 if rule == 2 else 0
            out[key] = ChannelPolicy(ChannelPolicy.IMPLICIT_META, threshold=0 if n == 0 else thr, subs=subs)
        else:
            out[key] = ChannelPolicy(ChannelPolicy.UNSUPPORTED)
    for c, g in children:
        _config_policies(g, (path + "/" + c) if path else c, out, msps, app_orgs, is_app=(path == "Application"))


class ChannelModel:
    def __init__(self, channel, identities, chaincodes, committed_txids=(), config=None, msps=(), kvmeta=None):
        """identities: iterable of (serialized, mspid, pub64, valid, id_digest) or
        (serialized, Ident).  chaincodes: ns -> ApplicationPolicy bytes, or a dict
        {policy, plugin="vscc", collections=None | {name: EP bytes | None}, sbe=False}
        (collections None: not known -> hashed writes Unsupported).  config: common.Config bytes
        (channel policies, MSPs, application orgs).  msps: further MSP ids of the channel.
        kvmeta: {(ns, coll, key bytes): VALIDATION_PARAMETER bytes} of the committed state
        (coll "" = public key; a hashed key is its key hash)."""
        self.kvmeta = dict(kvmeta or {})
        self.channel = channel
        self.msp = {}
        self.mspids = set(msps)
        for entry in identities:
            if len(entry) == 2:
                ser, o = entry  # any object with the Ident fields (e.g. fabric_amd.txvalidator.Identity)
                ident = Ident(o.mspid, o.pub, o.valid, o.id_digest, key=o.key, hash_family=o.hash_family, roles=o.roles,
                              ous=getattr(o, "ous", None))
            else:
                ser, mspid, pub, valid, dig = entry
                ident = Ident(mspid, pub, valid, dig, key=KEY_P256 if pub else KEY_OTHER)
            sid = decode("SerializedIdentity", ser)
            self.msp[(sid.get("mspid", ""), sid.get("id_bytes") or b"")] = ident
            self.mspids.add(ident.mspid)
        self.chaincodes = {ns: (d if isinstance(d, dict) else dict(policy=d)) for ns, d in dict(chaincodes).items()}
        self.committed = set(committed_txids)
        self.verify_calls = 0
        self.policies, self.config_msps, self.app_orgs = None, {}, {}
        self.config_unsupported = False
        if config is not None:
            cfg = decode("Config", config)
            self.policies = {}
            _config_policies(cfg.get("channel_group") or {}, "", self.policies, self.config_msps, self.app_orgs)
            self.mspids |= set(self.config_msps)
            for name, fc in self.config_msps.items():
                fam = (fc.get("crypto_config") or {}).get("signature_hash_family", "")
                if fam not in ("SHA2", "SHA3"):
                    self.config_unsupported = True  # the peer would not have set this MSP up
                if fam == "SHA3":  # the MSP's identities hash with SHA3 (identities.go:219-227)
                    for ident in self.msp.values():
                        if ident.mspid == name:
                            ident.hash_family = "SHA3"

    def deserialize(self, ser):
        """mspManagerImpl.DeserializeIdentity (msp/mspmgrimpl.go:75-100) over the registry.  A
        certificate of a channel MSP that was never registered cannot be judged (x509 parse +
        Validate happen in the MSP layer) -> Unsupported; an unknown MSP -> deserialize error."""
        try:
            sid = decode("SerializedIdentity", ser)
        except DecodeError:
            return None
        key = (sid.get("mspid", ""), sid.get("id_bytes") or b"")
        ident = self.msp.get(key)
        if ident is None:
            if key[0] not in self.mspids:
                return None
            # a cache miss: the channel's MSP deserializes and validates the certificate
            # (oracle/msp.py); an MSP outside that model -> Unsupported
            m = self.msp_models().get(key[0])
            if m is None or isinstance(m, Unsupported):
                raise Unsupported("unregistered identity of channel MSP %s" % key[0])
            ident = m.resolve(key[1])
            if ident is None:
                ident = Ident(key[0], None, False, b"\0" * 32, key=KEY_UNDESERIALIZABLE)
            elif self.config_msps.get(key[0], {}).get("crypto_config", {}).get("signature_hash_family") == "SHA3":
                ident.hash_family = "SHA3"
            self.msp[key] = ident
        if ident.key == KEY_UNDESERIALIZABLE:
            return None
        return ident

    def msp_models(self):
        if getattr(self, "_msp_models", None) is None:
            from .msp import msps_of_config
            self._msp_models = msps_of_config(self.config_msps) if self.policies is not None else {}
        return self._msp_models

    # the engine digests SHA3 identities' messages for the committer's creator and endorsement
    # signatures only (its orderer-signature path keeps them outside the model):
    # blockverify.block_signatures_ok clears this while it evaluates
    sha3_verify = True

    def verify(self, ident, msg, sig):
        """identity.Verify: 0 iff valid (msp/identities.go:170-199): the digest follows the
        MSP's SignatureHashFamily (getHashOpt :219-227: SHA2 -> SHA-256, SHA3 -> SHA3-256)."""
        self.verify_calls += 1
        if ident.key == KEY_OTHER:
            return 5
        if ident.key == KEY_P384 and (ident.pub is None or len(ident.pub) != 96):
            raise Unsupported("P-384 key not known")  # (the engine: registered without pubkey_p384)
        if ident.key not in (KEY_P256, KEY_P384):
            raise Unsupported("key type %r" % ident.key)
        if ident.key == KEY_P384 and not self.sha3_verify:
            raise Unsupported("P-384 identity outside the committer's signatures")  # (the orderer path)
        if ident.hash_family == "SHA3" and not self.sha3_verify:
            raise Unsupported("SHA3 identity outside the committer's signatures")
        if ident.hash_family not in ("SHA2", "SHA3"):
            raise Unsupported("hash family %r" % ident.hash_family)
        if not sig:
            return 6
        digest = hashlib.sha3_256(msg).digest() if ident.hash_family == "SHA3" else sha256(msg)
        if ident.key == KEY_P384:
            return verify_der_p384(ident.pub, sig, digest)
        return verify_der(ident.pub[:32], ident.pub[32:], sig, digest)

    def channel_policy(self, ref):
        """ChannelPolicyReferenceProviderImpl -> ManagerImpl.GetPolicy (policy.go:330-358)"""
        if self.policies is None or self.config_unsupported:
            raise Unsupported("channel config policy reference without a (usable) channel config")
        if ref.startswith("/"):
            if not ref.startswith("/Channel/"):
                return ChannelPolicy(ChannelPolicy.REJECT)
            ref = ref[len("/Channel/"):]
        return self.policies.get(ref, ChannelPolicy(ChannelPolicy.REJECT)) if ref else ChannelPolicy(ChannelPolicy.REJECT)


# ----------------------------------------------------------------- policies

def _compile(rule, principals):
    """cauthdsl.compile (common/cauthdsl/cauthdsl.go:24-92); returns closure or raises ValueError.
    A SignedBy whose principal cannot be decided for an identity makes the evaluation Unsupported
    (the greedy choice depends on it)."""
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
                v = _satisfies(ident, pr)
                if v is None:
                    raise Unsupported("a principal the engine cannot decide for this identity")
                if v:
                    used[i] = True
                    return True
            return False
        return signed
    raise ValueError("Unknown type")


_NEVER_LEAF = ("never",)


def _leaves(model, cls, body, depth=0):
    """collectPrincipals (msp/mspimpl.go:440-471) + each leaf, for MSP v1.4.3: a COMBINED that
    does not decode or holds no principal is an error for every identity (a "never" leaf)."""
    if cls == 4:  # COMBINED
        if depth > 16:
            raise Unsupported("combined principals nested deeper than the engine's bound")
        try:
            cp = decode("CombinedPrincipal", body)
        except DecodeError:
            return [_NEVER_LEAF]
        prs = cp.get("principals", [])
        if not prs:
            return [_NEVER_LEAF]
        out = []
        for q in prs:
            out += _leaves(model, q.get("principal_classification", 0), q.get("principal") or b"", depth + 1)
        return out
    try:
        if cls == 0:  # ROLE
            role = decode("MSPRole", body)
            r = role.get("role", 0)
            if not 0 <= r <= 4:
                return [_NEVER_LEAF]  # "invalid MSP role type"
            return [("role", role.get("msp_identifier", ""), r)]
        if cls == 1:  # ORGANIZATION_UNIT
            ou = decode("OrganizationUnit", body)
            return [("ou", ou.get("msp_identifier", ""), ou.get("organizational_unit_identifier", ""),
                     ou.get("certifiers_identifier") or b"")]
        if cls == 2:  # IDENTITY: deserialized by the identity's MSP when a signer is checked
            return [("identity", body, model)]
        if cls == 3:  # ANONYMITY
            an = decode("MSPIdentityAnonymity", body)
            return [("nominal",)] if an.get("anonymity_type", 0) == 0 else [_NEVER_LEAF]
    except DecodeError:
        return [_NEVER_LEAF]
    return [_NEVER_LEAF]  # "invalid principal type"


def _principal(p, model=None):
    return _leaves(model, p.get("principal_classification", 0), p.get("principal") or b"")


def _leaf_sat(ident, leaf):
    """one leaf of SatisfiesPrincipal (mspimpl.go:477-660): True / False / None (undecided)"""
    kind = leaf[0]
    if kind == "role":  # same MSP; MEMBER = Validate, other roles from the role bits
        _, mspid, role = leaf
        if ident.mspid != mspid:
            return False
        if role == 0:
            return ident.valid
        if ident.roles is None:
            raise Unsupported("role principal %d needs the identity's role bits" % role)
        return bool((ident.roles >> role) & 1)
    if kind == "identity":  # the same sanitized certificate (Mspid + Id), then Validate
        _, body, model = leaf
        try:
            p = model.deserialize(body)
        except Unsupported:
            return None
        return p is not None and p.dedup_key == ident.dedup_key and ident.valid
    if kind == "ou":  # same MSP, Validate, then an (OU, certifier) pair of the identity
        _, mspid, ou, cert = leaf
        if ident.mspid != mspid or not ident.valid:
            return False
        if ident.ous is None:
            return None
        return (ou, cert) in ident.ous
    return kind == "nominal"


def _satisfies(ident, leaves):
    """SatisfiesPrincipal: the collected leaves in order, the first error decides; True / False /
    None (undecided: some leaf unknown and none failing)"""
    r = True
    for leaf in leaves:
        v = _leaf_sat(ident, leaf)
        if v is False:
            return False
        if v is None:
            r = None
    return r


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


def _eval_spe(model, spe, sigset):
    """cauthdsl policy.EvaluateSignedData (common/cauthdsl/policy.go:86-108)"""
    principals = [_principal(p, model) for p in spe.get("identities", [])]
    try:
        ev = _compile(spe.get("rule"), principals)
    except ValueError:
        return False
    ids = signature_set_to_valid_identities(model, sigset)
    # a role principal needs every candidate's role bits (the engine checks this up front)
    if any(lf[0] == "role" and lf[2] != 0 for pr in principals for lf in pr) and any(i.roles is None for i in ids):
        raise Unsupported("role principal needs the identities' role bits")
    return ev(ids, [False] * len(ids))


def _eval_channel_policy(model, pol, sigset, depth=0):
    """ImplicitMetaPolicy.EvaluateSignedData (implicitmeta.go:69-104): every sub-policy is
    evaluated (the reference stops early in Go map order; outcomes are pure, so the count decides).
    Threshold 0 (no sub-policies, or a rule outside ANY/ALL/MAJORITY, :45-58): `remaining`
    starts at 0 and each satisfied sub-policy takes it below 0, so only "none satisfied" passes."""
    if pol.kind == ChannelPolicy.REJECT:
        return False
    if pol.kind == ChannelPolicy.UNSUPPORTED or (pol.kind == ChannelPolicy.IMPLICIT_META and depth > 0):
        raise Unsupported("channel policy outside the model")
    if pol.kind == ChannelPolicy.SIGNATURE:
        return _eval_spe(model, pol.spe, sigset)
    ok = sum(1 for sub in pol.subs
             if _eval_channel_policy(model, model.policies.get(sub, ChannelPolicy(ChannelPolicy.REJECT)), sigset, depth + 1))
    return ok == 0 if pol.threshold == 0 else ok >= pol.threshold


def evaluate_policy(model, policy_bytes, sigset):
    """ApplicationPolicyEvaluator.Evaluate (core/policy/application.go:148-163).  True iff ok."""
    try:
        ap = decode("ApplicationPolicy", policy_bytes)
    except DecodeError:
        return False
    if "signature_policy" in ap:
        return _eval_spe(model, ap["signature_policy"], sigset)
    if "channel_config_policy_reference" in ap:
        return _eval_channel_policy(model, model.channel_policy(ap["channel_config_policy_reference"]), sigset)
    return False


def signed_by_any_member(mspid):
    """policydsl.SignedByAnyMember([mspid]) as ApplicationPolicy bytes"""
    def fb(num, b):
        return _pv(num << 3 | 2) + _pv(len(b)) + b
    role = fb(1, mspid.encode())  # MSPRole{msp_identifier, role MEMBER}
    spe = fb(2, fb(2, b"\x08\x01" + fb(2, b"\x08\x00"))) + fb(3, fb(2, role))
    return fb(1, spe)


def _pv(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def collection_policy(model, ns, coll):
    """ValidatorCommitter.CollectionValidationInfo (core/chaincode/lifecycle/
    deployedcc_infoprovider.go:343-382) -> ("app", bytes) | ("cc",) | ("reject",)"""
    if coll.startswith(IMPLICIT_PREFIX):
        mspid = coll[len(IMPLICIT_PREFIX):]
        if model.policies is None or model.config_unsupported or mspid not in model.app_orgs:
            raise Unsupported("implicit collection of an org outside the channel config")
        path = "Application/%s/Endorsement" % model.app_orgs[mspid]  # :277-300
        if path in model.policies:
            return ("ref", path)
        return ("app", signed_by_any_member(mspid))
    cc = model.chaincodes[ns]
    colls = cc.get("collections")
    if colls is None:
        raise Unsupported("collections of %s not known" % ns)
    if coll not in colls:
        return ("reject",)  # "no such collection" -> validation error -> policy failure
    return ("app", colls[coll]) if colls[coll] else ("cc",)


def _run(model, pol, cc_policy, sigset):
    if pol[0] == "cc":
        return evaluate_policy(model, cc_policy, sigset)
    if pol[0] == "app":
        return evaluate_policy(model, pol[1], sigset)
    if pol[0] == "ref":
        return _eval_channel_policy(model, model.policies[pol[1]], sigset)
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
        raise ConfigTransaction("CONFIG transaction")
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


EXTRACT_OK, EXTRACT_FAIL, EXTRACT_PANIC = 0, 1, 2
_NEVER, _INDET = "never", "indeterminate"


def extract_dependencies(d):
    """KeyLevelValidator.extractDependenciesForTx (validator_keylevel.go:184-222) and
    ExtractValidationParameterDependency (vpmanagerimpl.go:258-292) -> (status, keys).
    keys: (ns, coll, key bytes) of every metadata write of the tx, public and hashed, in any
    namespace (none when the rwset does not decode: the dependency is still signalled).
    EXTRACT_FAIL: an unmarshal error returns before ExtractValidationParameterDependency, so the
    tx's dependency is never signalled and a later GetValidationParameterForKey waits for it
    forever (vpmanagerimpl.go:300-303).  EXTRACT_PANIC: tx.Actions[0] of an empty list (:203) or
    cap.Action == nil (:209) panics the peer."""
    try:
        env = decode("Envelope", d)
        payl = decode("Payload", env.get("payload"))
        tx = decode("Transaction", payl.get("data"))
    except DecodeError:
        return EXTRACT_FAIL, []
    acts = tx.get("actions", [])
    if not acts:
        return EXTRACT_PANIC, []
    try:
        cap = decode("ChaincodeActionPayload", acts[0].get("payload"))
    except DecodeError:
        return EXTRACT_FAIL, []
    if "action" not in cap:
        return EXTRACT_PANIC, []
    try:
        prp = decode("ProposalResponsePayload", cap["action"].get("proposal_response_payload"))
        cca = decode("ChaincodeAction", prp.get("extension"))
    except DecodeError:
        return EXTRACT_FAIL, []
    try:
        rw = parse_rwset(cca.get("results"))
    except DecodeError:
        return EXTRACT_OK, []
    keys = []
    for nsrw in rw:
        for mw in nsrw["kv"].get("metadata_writes", []):
            keys.append((nsrw["namespace"], "", mw.get("key", "").encode()))
        for c in nsrw["coll"]:
            for mw in c["hashed"].get("metadata_writes", []):
                keys.append((nsrw["namespace"], c["name"], mw.get("key_hash") or b""))
    return EXTRACT_OK, keys


class BlockContext:
    """The per-block state of KeyLevelValidationParameterManagerImpl (vpmanagerimpl.go:113-233),
    restated sequentially: transactions are validated in block order, so every earlier tx's
    dependencies and vscc results are known when a later tx asks.  res[j][ns]: True (the vscc
    of ns returned nil), False (an error), _INDET (whether it runs depends on Go map order) or
    absent (it never runs: a GetValidationParameterForKey waiting on it blocks forever)."""

    def __init__(self, data):
        self.data, self.i = data, 0
        self.ext, self.deps, self.res = [], {}, []

    def _extract_upto(self, i):  # PreValidate(i): txDepOnce for every tx <= i
        while len(self.ext) <= i:
            j = len(self.ext)
            st, keys = extract_dependencies(self.data[j])
            self.ext.append(st)
            for k in keys:
                self.deps.setdefault(k, []).append(j)

    def pre_validate(self):
        self._extract_upto(self.i)
        if EXTRACT_PANIC in self.ext[:self.i]:
            raise Unsupported("the peer panics extracting an earlier tx's dependencies (validator_keylevel.go:203-209)")

    def validation_parameter_updated(self, ns, coll, key):
        """GetValidationParameterForKey's wait (vpmanagerimpl.go:296-311) -> True iff an earlier
        tx of the block validly (vscc nil for ns) wrote this key's metadata."""
        if EXTRACT_FAIL in self.ext[:self.i]:
            raise Unsupported("an earlier tx never signals its dependencies: the reference waits forever")
        rs = [self.res[j].get(ns, _NEVER) for j in self.deps.get((ns, coll, key), ()) if j < self.i]
        if any(r in (_NEVER, _INDET) for r in rs):
            raise Unsupported("the vscc result of an earlier metadata writer never arrives (or map order)")
        return any(r is True for r in rs)


def validation_parameter(model, ns, coll, key, ctx):
    """GetValidationParameterForKey (vpmanagerimpl.go:296-351) + toApplicationPolicyTranslator
    (builtin/v20/validation_logic.go:50-66) -> "updated", None (no key-level parameter) or the
    SignaturePolicyEnvelope."""
    if ctx is not None and ctx.validation_parameter_updated(ns, coll, key):
        return "updated"  # ValidationParameterUpdatedError -> policyErr
    vp = model.kvmeta.get((ns, coll, key), b"")
    if not vp:
        return None
    try:
        return decode("SignaturePolicyEnvelope", vp)
    except DecodeError:
        raise Unsupported("untranslatable validation parameter: VSCCExecutionFailureError halts the channel")


def vscc_validate(model, env_bytes, ns, ctx=None):
    """builtin v20 Validate (validation_logic.go:185-217) -> True iff it returns nil."""
    cc = model.chaincodes[ns]
    if cc.get("plugin", "vscc") != "vscc" or cc.get("sbe"):
        raise Unsupported("validation plugin other than the builtin vscc / undeclared key-level state")
    if ctx is not None:
        ctx.pre_validate()
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
    # baseEvaluator.Evaluate (validator_keylevel.go:87-143) over policyCheckerV20 (v20.go:105-167):
    # public writes, public metadata writes, hashed writes, hashed metadata writes; per key its
    # validation parameter, else CheckCCEPIfNotChecked (collection EP, else the chaincode EP
    # once).  The reference returns at the first error; every step's outcome is pure, so the
    # conjunction over ALL steps is the same verdict -- and a step outside the model anywhere
    # makes the tx Unsupported (never a guess, possibly where the reference had already stopped).
    ok, checked, some = True, set(), False
    for nsrw in rw:
        if nsrw["namespace"] != ns:
            continue
        keys = [("", w.get("key", "").encode()) for w in nsrw["kv"].get("writes", [])]
        keys += [("", w.get("key", "").encode()) for w in nsrw["kv"].get("metadata_writes", [])]
        keys += [(c["name"], w.get("key_hash") or b"") for c in nsrw["coll"] for w in c["hashed"].get("hashed_writes", [])]
        keys += [(c["name"], w.get("key_hash") or b"") for c in nsrw["coll"] for w in c["hashed"].get("metadata_writes", [])]
        for coll, key in keys:
            some = True
            vp = validation_parameter(model, ns, coll, key, ctx)
            if vp == "updated":
                ok = False
            elif vp is not None:
                ok &= _eval_spe(model, vp, sigset)
            elif coll and coll in checked:
                pass
            else:
                p = collection_policy(model, ns, coll) if coll else ("cc",)
                if p[0] == "reject":
                    ok = False
                elif p[0] != "cc":
                    ok &= _run(model, p, cc["policy"], sigset)
                    checked.add(coll)
                elif "" not in checked:
                    ok &= evaluate_policy(model, cc["policy"], sigset)
                    checked.add("")
    if not some:  # CheckCCEPIfNoEPChecked (FAB-9473)
        return evaluate_policy(model, cc["policy"], sigset)
    return ok


def dispatch(model, payload, env_bytes, ctx=None):
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
    # The reference iterates a Go map (random order) and stops at the first failing namespace.
    # Results only differ in the reported code when namespaces fail with DIFFERENT codes; we
    # report the first in sorted order and flag multi-namespace disagreement as unsupported.
    # A namespace's vscc result (read by later txs' key-level checks) is determined only when
    # it runs in every order: no OTHER namespace fails.
    codes, ran = {}, {}
    for ns in sorted(wr):
        cc = model.chaincodes.get(ns)
        # getCDataForCC (dispatcher.go:237-264): undefined chaincode, empty plugin or empty
        # validation parameter -> INVALID_CHAINCODE
        if cc is None or not cc.get("policy") or cc.get("plugin", "vscc") == "":
            codes[ns] = INVALID_CHAINCODE
            continue
        ok = vscc_validate(model, env_bytes, ns, ctx)
        ran[ns] = ok
        if not ok:
            codes[ns] = ENDORSEMENT_POLICY_FAILURE
    if ctx is not None:
        for ns, ok in ran.items():
            ctx.res[ctx.i][ns] = _INDET if any(n != ns for n in codes) else ok
    if len(set(codes.values())) > 1:
        raise Unsupported("namespaces fail with different codes (map-order dependent)")
    return next(iter(codes.values())) if codes else VALID


# ----------------------------------------------------------------- block level

def validate_tx(model, d, ctx=None):
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
        code = dispatch(model, payload, d, ctx)
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


def keylevel_writes(model, d):
    """-> (changed, touched): the (ns, coll, key) this tx may change the key-level state of --
    its metadata writes, and its deletes of keys holding a VALIDATION_PARAMETER in the committed
    state (tx_ops.go:17-51: a metadata write replaces the metadata, a delete drops it) -- and
    every key it writes or metadata-writes (what its vscc reads the parameter of)."""
    try:
        cca, _ = get_action_from_envelope(d)
        rw = parse_rwset(cca.get("results"))
    except (DecodeError, ValueError, KeyError, IndexError, TypeError):
        return set(), set()
    changed, touched = set(), set()
    for nsrw in rw:
        ns = nsrw["namespace"]
        sets = [("", nsrw["kv"].get("writes", []), "key", nsrw["kv"].get("metadata_writes", []), "key")]
        sets += [(c["name"], c["hashed"].get("hashed_writes", []), "key_hash", c["hashed"].get("metadata_writes", []),
                  "key_hash") for c in nsrw["coll"]]
        for coll, ws, wk, ms, mk in sets:
            for w in ws:
                k = w.get(wk) or (b"" if wk == "key_hash" else "")
                k = (ns, coll, k.encode() if isinstance(k, str) else k)
                touched.add(k)
                if w.get("is_delete") and model.kvmeta.get(k):
                    changed.add(k)
            for m in ms:
                k = m.get(mk) or (b"" if mk == "key_hash" else "")
                k = (ns, coll, k.encode() if isinstance(k, str) else k)
                touched.add(k)
                changed.add(k)
    return changed, touched


def check_keylevel_batch(model, blocks):
    """A batch validates every block against the key-level state committed before it; the
    reference commits block k (its valid metadata writes and deletes) before block k+1's vscc
    reads GetStateMetadata.  When a block other than the last may change the parameter of a key
    that a later block of the batch writes, the outcome depends on block k's validity and MVCC
    results: Unsupported (the caller validates the blocks one call at a time)."""
    if len(blocks) < 2:
        return
    seen_changed = set()
    for blk in blocks:
        data = (decode("Block", blk).get("data") or {}).get("data", [])
        ch_b, tc_b = set(), set()
        for d in data:
            c, t = keylevel_writes(model, d)
            ch_b |= c
            tc_b |= t
        if seen_changed & tc_b:
            raise Unsupported("a key-level parameter changed by an earlier block of the batch is written by a later one")
        seen_changed |= ch_b


def validate_blocks(model, blocks):
    """Consecutive blocks: block k sees the txids indexed by blocks < k (blkstorage indexes
    every transaction's txid at commit, block_serialization.go:95-115)."""
    check_keylevel_batch(model, blocks)
    out = []
    for blk in blocks:
        out.append(validate_block(model, blk))
        data = (decode("Block", blk).get("data") or {}).get("data", [])
        for d in data:
            t = index_txid(d)
            if t:
                model.committed.add(t)
    return out


def validate_blocks_outcomes(model, blocks):
    """The engine's per-block outcomes (fgv_set_block_outcomes, include/fgv.h) restated over the
    reference's rules: n_final = the first block writing a key whose key-level parameter an earlier
    block of the call may change (check_keylevel_batch's condition; the reference commits that
    block first); each block before it is validated (None when Unsupported), and every block's
    txids are indexed whatever its codes (blkstorage indexes every transaction,
    block_serialization.go:95-115), so a block after an unsupported one is still decided.
    -> (list of flags or None, n_final)"""
    n_final = len(blocks)
    seen_changed = set()
    for b, blk in enumerate(blocks):
        data = (decode("Block", blk).get("data") or {}).get("data", [])
        ch_b, tc_b = set(), set()
        for d in data:
            c, t = keylevel_writes(model, d)
            ch_b |= c
            tc_b |= t
        if seen_changed & tc_b:
            n_final = b
            break
        seen_changed |= ch_b
    out = []
    for b, blk in enumerate(blocks):
        if b >= n_final:
            out.append(None)
            continue
        try:
            out.append(validate_block(model, blk))
        except Unsupported:
            out.append(None)
        # a CONFIG transaction that reaches ChannelResources.Apply changes the configuration the
        # later blocks validate under: they wait for this block's commit (the caller re-applies
        # the channel config and calls again)
        if any(_reaches_config_apply(model, d) for d in (decode("Block", blk).get("data") or {}).get("data", [])):
            n_final = min(n_final, b + 1)
        for d in (decode("Block", blk).get("data") or {}).get("data", []):
            t = index_txid(d)
            if t:
                model.committed.add(t)
    return out, n_final


def _reaches_config_apply(model, d):
    try:
        validate_transaction(model, decode("Envelope", d))
    except ConfigTransaction:
        return True
    except (Unsupported, DecodeError):
        return False
    return False


def validate_block(model, block_bytes):
    """TxValidator.Validate -> list of validation codes (TxValidationFlags)."""
    blk = decode("Block", block_bytes)
    data = (blk.get("data") or {}).get("data", [])
    flags, txids = [], []
    ctx = BlockContext(data)
    for i, d in enumerate(data):
        ctx.i = i
        ctx.res.append({})
        code, txid = validate_tx(model, d, ctx)
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
