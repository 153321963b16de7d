"""Restated MSP identity path on a cache miss (TEST INFRASTRUCTURE ONLY -- the oracle).

An identity the peer's MSP cache has not seen (msp/cache/cache.go:65-83) is deserialized and
validated by the channel's MSP (bccspmsp, MSP version 1.4.3 -- Fabric v2 channels):
  mspimpl.go:398-422   deserializeIdentityInternal: pem.Decode, x509.ParseCertificate, bccsp
                       KeyImport (ECDSA / RSA keys; Ed25519 fails)
  identities.go:48-84  newIdentity: sanitizeCert, then Id = hex(SHA-256(sanitized cert.Raw))
  mspimpl.go:892-938   sanitizeCert: an ECDSA-signed certificate must chain to the MSP's roots
                       (getUniqueValidationChain: x509 Verify with CurrentTime = NotBefore + 1 s,
                       KeyUsages Any; exactly one chain) -- else DeserializeIdentity fails --
                       and is re-marshalled with a low-S signature
  mspimplvalidate.go   validateIdentity: the chain again, the signing CA's SubjectKeyIdentifier
                       must exist (validateCertAgainstChain), CRLs (oracle/crl.py),
                       validateIdentityOUsV142
                       (OrganizationalUnitIdentifiers intersection; NodeOU: exactly one of the
                       client / peer / admin / orderer OUs)
  mspimpl.go:607-680   satisfiesPrincipalInternalV142 / PreV13 for ROLE principals: MEMBER =
                       Validate; ADMIN = in the admins list or (valid and admin OU); CLIENT / PEER
                       / ORDERER = valid and that OU (NodeOUs required)
Intermediate CAs (mspimplsetup.go finalizeSetupCAs, mspimpl.go:835-858 getValidationChain):
every CA must be a CA with a SubjectKeyIdentifier (else the MSP does not set up); the parents of
intermediates are internal nodes of the certification tree, and an identity whose issuer is an
internal node is invalid; the certifier identifier of a chain is SHA-256 over its certificates
(getCertificationChainIdentifierFromChain).  x509 Verify (Go 1.21) per hop: CheckSignatureFrom,
validity at the leaf's NotBefore + 1 s, an intermediate needs basicConstraints CA, MaxPathLen.
Modelled MSP shapes: CRLs of the shape oracle/crl.py models, P-256 CAs, at most one candidate
parent per hop, OU certificates that are CAs of the MSP; anything else raises Unsupported.
"""
import hashlib

from . import verify_der
from . import crl as CRL
from . import x509 as X
from .protowire import decode
from .v20 import KEY_OTHER, KEY_P256, KEY_P384, Ident, Unsupported

ROLE_MEMBER, ROLE_ADMIN, ROLE_CLIENT, ROLE_PEER, ROLE_ORDERER = range(5)
MAX_CHAIN = 8


def _ca(pem, what):
    der = X.pem_decode(pem)
    if der is None:
        raise Unsupported(what + " PEM")
    try:
        c = X.parse_certificate(der)
    except X.ParseError:
        raise Unsupported(what + " does not parse")
    if c["key"] != "p256":
        raise Unsupported(what + " key")
    if not c["is_ca"] or c["ski"] is None:  # finalizeSetupCAs: the MSP would not set up
        raise Unsupported(what + " without the CA attribute or a SubjectKeyIdentifier")
    c["raw2"] = X.sanitized_raw(c)  # (setupCAs sanitizes the CAs)
    return c


class MSP:
    def __init__(self, fc):
        """fc: decoded FabricMSPConfig"""
        self.name = fc.get("name", "")
        # setupCRLs (mspimplsetup.go:215-245): a CRL x509.ParseCRL rejects fails the setup
        self.crls = []
        for raw in fc.get("revocation_list", []):
            try:
                self.crls.append(CRL.parse_crl(raw))
            except X.ParseError:
                raise Unsupported("a CRL the MSP does not set up with")
        cc = fc.get("crypto_config") or {}
        if cc.get("identity_identifier_hash_function", "SHA256") not in ("SHA256", ""):
            raise Unsupported("identity identifier hash")
        if not fc.get("root_certs"):
            raise Unsupported("MSP without root CAs")  # (setupCAs: "expected at least one CA certificate")
        self.roots = [_ca(pem, "root CA") for pem in fc.get("root_certs", [])]
        self.inters = [_ca(pem, "intermediate CA") for pem in fc.get("intermediate_certs", [])]
        for r in self.roots:  # a root verifies itself (validateCAIdentity: a chain of length 1)
            if r["issuer"] != r["subject"] or not X.ca_verifies(r, r, verify_der):
                raise Unsupported("root CA that is not self-signed")
        # the chains of the intermediates, checked at their own NotBefore + 1 s; their parents
        # are the internal nodes of the certification tree
        self.internal = set()
        self.inter_chain = {}
        for c in self.inters:
            ch = self._chain_of(c, c["not_before"] + 1)
            if ch is None or len(ch) < 2:
                raise Unsupported("intermediate CA without a validation chain")
            self.inter_chain[c["raw2"]] = ch
            for p in ch[1:]:
                self.internal.add(p["raw2"])
            # finalizeSetupCAs -> validateCAIdentity: a revoked intermediate fails the setup
            if CRL.revoked(c, ch, self.crls, verify_der):
                raise Unsupported("revoked intermediate CA: the MSP does not set up")

        # certifier identifiers: SHA-256 over the chain of the OU's certificate (a root: itself)
        def certifier(pem):
            if not pem:
                return None
            der = X.pem_decode(pem)
            for r in self.roots:
                if der == r["der"]:
                    return hashlib.sha256(r["raw2"]).digest()
            for c in self.inters:
                if der == c["der"]:
                    if c["raw2"] in self.internal:  # getValidationChain(cert, true): parent position 0
                        raise Unsupported("OU certificate that is an internal CA")
                    return hashlib.sha256(b"".join(x["raw2"] for x in self.inter_chain[c["raw2"]])).digest()
            raise Unsupported("OU certificate that is not a CA of the MSP")
        self.ou_ids = {}
        for ou in fc.get("organizational_unit_identifiers", []):
            if not ou.get("certificate"):
                raise Unsupported("OU identifier without a certificate")
            self.ou_ids.setdefault(ou.get("organizational_unit_identifier", ""), []).append(
                certifier(ou.get("certificate")))
        n = fc.get("fabric_node_ous") or {}
        self.node_ous = bool(n.get("enable"))
        self.role_ou = {}
        for role, key in ((ROLE_CLIENT, "client_ou_identifier"), (ROLE_PEER, "peer_ou_identifier"),
                          (ROLE_ADMIN, "admin_ou_identifier"), (ROLE_ORDERER, "orderer_ou_identifier")):
            o = n.get(key)
            if o is not None and self.node_ous:
                self.role_ou[role] = (o.get("organizational_unit_identifier", ""), certifier(o.get("certificate")))
        self.admins = []
        admin_certs = []
        for pem in fc.get("admins", []):
            der = X.pem_decode(pem)
            try:
                c = X.parse_certificate(der)
                self.admins.append(X.sanitized_raw(c))
            except (X.ParseError, TypeError):
                raise Unsupported("admin certificate")
            admin_certs.append(c)
        # postSetupV142 (mspimplsetup.go:684-702): without NodeOUs, postSetupV1 (:612-624) -- every
        # admin must Validate (its chain, the CRLs, the OU identifiers); with NodeOUs every admin
        # must carry the client or the admin OU (hasOURole over GetOrganizationalUnits, which is
        # empty when the admin has no certification chain).  Otherwise the MSP does not set up.
        for c in admin_certs:
            chain = self._chain(c)
            if chain is None:
                raise Unsupported("admin without a validation chain: the MSP does not set up")
            if not self.node_ous:
                if not self._valid(c, chain)[0]:
                    raise Unsupported("admin that does not validate: the MSP does not set up")
            elif not (self._has(ROLE_CLIENT, c) or self._has(ROLE_ADMIN, c)):
                raise Unsupported("admin without the client or admin OU: the MSP does not set up")

    def _parent_ok(self, parent, now, below):
        """x509 isValid for a CA at `below` intermediates under it + CheckSignatureFrom's rules"""
        if (parent["version"] == 3 and not parent["bc_valid"]) or (parent["bc_valid"] and not parent["is_ca"]):
            return False
        if parent["key_usage"] and not (parent["key_usage"] & (1 << 5)):
            return False
        if not (parent["not_before"] <= now <= parent["not_after"]):
            return False
        if parent["bc_valid"] and parent["path_len"] >= 0 and below > parent["path_len"]:
            return False  # TooManyIntermediates
        return True

    def _chain_of(self, c, now):
        """getUniqueValidationChain: [c, parent, ..., root] or None; Unsupported when a hop has
        several candidate parents (Go could build several chains)"""
        chain = [c]
        cur = c
        while not any(cur is r for r in self.roots):
            if len(chain) > MAX_CHAIN:
                raise Unsupported("certificate chain too long")
            cands = [x for x in self.roots + self.inters if x["subject"] == cur["issuer"] and x is not cur]
            if len(cands) > 1:
                raise Unsupported("several CAs with the issuer name")
            if not cands:
                return None
            p = cands[0]
            if p in chain:
                return None
            if not self._parent_ok(p, now, len(chain) - 1):
                return None
            if not X.ca_verifies(p, cur, verify_der):
                return None
            chain.append(p)
            cur = p
        return chain

    def _chain(self, c):
        """getUniqueValidationChain for a leaf: its chain to a root, or None"""
        if c["is_ca"]:
            raise Unsupported("CA certificate as an identity")
        if c["unhandled_critical"]:
            return None
        now = c["not_before"] + 1
        if not (c["not_before"] <= now <= c["not_after"]):
            return None
        return self._chain_of(c, now)

    def resolve(self, id_bytes):
        """-> v20.Ident, or None when DeserializeIdentity fails"""
        der = X.pem_decode(id_bytes)
        if der is None:
            return None
        try:
            c = X.parse_certificate(der)
        except X.ParseError:
            return None
        if c["key"] == "undeserializable":  # bccsp KeyImport fails (Ed25519)
            return None
        chain = self._chain(c)
        if chain is None:
            return None  # sanitizeCert: no validation chain -> newIdentity fails
        raw2 = X.sanitized_raw(c)
        digest = hashlib.sha256(raw2).digest()
        valid, ous = self._valid(c, chain)
        roles = 1 if valid else 0
        if raw2 in self.admins or (valid and self.node_ous and self._has(ROLE_ADMIN, c)):
            roles |= 1 << ROLE_ADMIN
        for role in (ROLE_CLIENT, ROLE_PEER, ROLE_ORDERER):
            if valid and self.node_ous and self._has(role, c):
                roles |= 1 << role
        key = {"p256": KEY_P256, "p384": KEY_P384}.get(c["key"], KEY_OTHER)
        return Ident(self.name, c["pub"] if key in (KEY_P256, KEY_P384) else None, valid, digest, key=key, roles=roles,
                     ous=ous)

    def _valid(self, c, chain):
        """validateIdentity of a leaf with its validation chain -> (valid, its OUs with certifier)"""
        # Validate: the issuer must be a leaf of the certification tree, its SKI must exist
        # (setup guarantees it), then the OUs; the certifier is the chain above the identity
        valid = chain[1]["raw2"] not in self.internal and chain[1]["ski"] is not None
        # validateCertAgainstChain: revoked by a CRL its issuing CA signed (mspimplvalidate.go:94-140)
        if valid and self.crls and CRL.revoked(c, chain, self.crls, verify_der):
            valid = False
        certifier = hashlib.sha256(b"".join(x["raw2"] for x in chain[1:])).digest()
        ous = [(o, certifier) for o in c["ous"]]
        if valid and self.ou_ids:
            valid = any(cid in self.ou_ids.get(o, []) for o, cid in ous)
        if valid and self.node_ous:
            cnt = 0
            for o, cid in ous:
                hit = [r for r, (name, _) in self.role_ou.items() if name == o]
                if not hit:
                    continue
                want = self.role_ou[hit[-1]][1]  # (validOUs map: a later role's identical OU overwrites)
                if want is not None and want != cid:
                    valid = False
                    break
                cnt += 1
                if cnt > 1:
                    break
            if cnt != 1:
                valid = False
        return valid, ous

    def _has(self, role, c):
        ou = self.role_ou.get(role)
        return ou is not None and ou[0] in c["ous"]


def msps_of_config(config_msps):
    """{mspid: MSP or the Unsupported it raised} for ChannelModel.config_msps"""
    out = {}
    for name, fc in config_msps.items():
        try:
            out[name] = MSP(fc)
        except Unsupported as e:
            out[name] = e
    return out


def decode_msp_value(value_bytes):
    mc = decode("MSPConfig", value_bytes)
    return decode("FabricMSPConfig", mc.get("config"))
