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
                       must exist (validateCertAgainstChain), CRLs, validateIdentityOUsV142
                       (OrganizationalUnitIdentifiers intersection; NodeOU: exactly one of the
                       client / peer / admin / orderer OUs)
  mspimpl.go:607-680   satisfiesPrincipalInternalV142 / PreV13 for ROLE principals: MEMBER =
                       Validate; ADMIN = in the admins list or (valid and admin OU); CLIENT / PEER
                       / ORDERER = valid and that OU (NodeOUs required)
Modelled MSP shapes: root CAs only (no intermediates), no CRLs, OU identifiers whose
certificate (if any) is one of the roots; anything else raises Unsupported.
"""
import hashlib

from . import verify_der
from . import x509 as X
from .protowire import decode
from .v20 import KEY_OTHER, KEY_P256, KEY_P384, Ident, Unsupported

ROLE_MEMBER, ROLE_ADMIN, ROLE_CLIENT, ROLE_PEER, ROLE_ORDERER = range(5)


class MSP:
    def __init__(self, fc):
        """fc: decoded FabricMSPConfig"""
        self.name = fc.get("name", "")
        if fc.get("intermediate_certs"):
            raise Unsupported("intermediate CAs")
        if fc.get("revocation_list"):
            raise Unsupported("CRLs")
        cc = fc.get("crypto_config") or {}
        if cc.get("identity_identifier_hash_function", "SHA256") not in ("SHA256", ""):
            raise Unsupported("identity identifier hash")
        self.roots = []
        if not fc.get("root_certs"):
            raise Unsupported("MSP without root CAs")  # (setupCAs: "expected at least one CA certificate")
        for pem in fc.get("root_certs", []):
            der = X.pem_decode(pem)
            if der is None:
                raise Unsupported("root CA PEM")
            try:
                c = X.parse_certificate(der)
            except X.ParseError:
                raise Unsupported("root CA does not parse")
            if c["key"] != "p256":
                raise Unsupported("root CA key")
            c["raw2"] = X.sanitized_raw(c)  # (setupCAs sanitizes the roots too)
            self.roots.append(c)
        # certifier identifiers: SHA-256 over the chain of the OU's certificate (a root: itself)
        def certifier(pem):
            if not pem:
                return None
            der = X.pem_decode(pem)
            for r in self.roots:
                if der == r["der"]:
                    return hashlib.sha256(r["raw2"]).digest()
            raise Unsupported("OU certificate that is not a root CA")
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
        for pem in fc.get("admins", []):
            der = X.pem_decode(pem)
            try:
                c = X.parse_certificate(der)
                self.admins.append(X.sanitized_raw(c))
            except (X.ParseError, TypeError):
                raise Unsupported("admin certificate")

    def _chain(self, c):
        """getUniqueValidationChain for a leaf: the one root that signed it, or None"""
        if c["is_ca"]:
            raise Unsupported("CA certificate as an identity")
        if c["unhandled_critical"]:
            return None
        now = c["not_before"] + 1
        if not (c["not_before"] <= now <= c["not_after"]):
            return None
        cands = [r for r in self.roots if r["subject"] == c["issuer"]]
        if len(cands) > 1:
            raise Unsupported("several roots with the leaf's issuer name")
        for r in cands:
            # CheckSignatureFrom: the parent must be allowed to sign certificates
            if (r["version"] == 3 and not r["bc_valid"]) or (r["bc_valid"] and not r["is_ca"]):
                return None
            if r["key_usage"] and not (r["key_usage"] & (1 << 5)):
                return None
            if not (r["not_before"] <= now <= r["not_after"]):
                return None
            if X.ca_verifies(r, c, verify_der):
                return r
        return None

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
        root = self._chain(c)
        if root is None:
            return None  # sanitizeCert: no validation chain -> newIdentity fails
        raw2 = X.sanitized_raw(c)
        digest = hashlib.sha256(raw2).digest()
        # Validate: the signing CA's SKI, then the OUs
        valid = root["ski"] is not None
        certifier = hashlib.sha256(root["raw2"]).digest()
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
        roles = 1 if valid else 0
        if raw2 in self.admins or (valid and self.node_ous and self._has(ROLE_ADMIN, c)):
            roles |= 1 << ROLE_ADMIN
        for role in (ROLE_CLIENT, ROLE_PEER, ROLE_ORDERER):
            if valid and self.node_ous and self._has(role, c):
                roles |= 1 << role
        key = {"p256": KEY_P256, "p384": KEY_P384}.get(c["key"], KEY_OTHER)
        return Ident(self.name, c["pub"] if key == KEY_P256 else None, valid, digest, key=key, roles=roles)

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
