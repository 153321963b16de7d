"""Synthetic channel configuration (common.Config) for the generated networks: the layout a
Fabric v2 `configtxgen` profile produces for an application channel (SURVEY s8(d) C2 variant):

  /Channel/Application/Endorsement           IMPLICIT_META MAJORITY Endorsement
  /Channel/Application/LifecycleEndorsement  IMPLICIT_META MAJORITY Endorsement
  /Channel/Application/<orgN>/Endorsement    SIGNATURE OR('OrgNMSP.peer')
  /Channel/Application/<orgN>/{Readers,Writers,Admins}
  /Channel/Application/<orgN> value MSP      FabricMSPConfig{name, crypto_config SHA2/SHA256,
                                             fabric_node_ous enabled}
and, with orderer orgs (the policies the deliver client verifies blocks with,
deliverclient/verifier_assembler.go:32-56):
  /Channel/Orderer/BlockValidation           IMPLICIT_META ANY Writers (configtxgen default)
  /Channel/Orderer/<ordN>/Writers            SIGNATURE OR('OrdererMSP.member')

Message layout: common/configtx.pb.go (Config, ConfigGroup with map<string, ...> entries),
common/policies.pb.go (Policy, ImplicitMetaPolicy), msp/msp_config.pb.go."""
from .blocks import f_bytes, f_msg, f_str, f_varint, msp_role_principal, n_out_of, signed_by

SIGNATURE, IMPLICIT_META = 1, 3
ANY, ALL, MAJORITY = 0, 1, 2
MEMBER, ADMIN, CLIENT, PEER, ORDERER = 0, 1, 2, 3, 4


def _entry(key, value_msg):
    return f_str(1, key) + f_msg(2, value_msg)


def signature_policy(n, principals):
    """SignaturePolicyEnvelope{rule: NOutOf(n, SignedBy(i)...), identities: ROLE principals}"""
    return f_msg(2, n_out_of(n, [signed_by(i) for i in range(len(principals))])) + \
        b"".join(f_msg(3, msp_role_principal(m, r)) for m, r in principals)


def config_policy(ptype, value):
    return f_msg(2, f_varint(1, ptype) + f_bytes(2, value))  # ConfigPolicy{policy: Policy{type, value}}


def implicit_meta(rule, sub):
    return config_policy(IMPLICIT_META, f_str(1, sub) + f_varint(2, rule))


def msp_value(mspid, hash_family="SHA2"):
    ou = lambda name: f_str(2, name)  # FabricOUIdentifier{organizational_unit_identifier}
    fabric = f_str(1, mspid) + f_msg(8, f_str(1, hash_family) + f_str(2, "SHA256")) + \
        f_msg(11, f_varint(1, 1) + f_msg(2, ou("client")) + f_msg(3, ou("peer")) + f_msg(4, ou("admin")) +
              f_msg(5, ou("orderer")))
    return f_bytes(2, f_varint(1, 0) + f_bytes(2, fabric))  # ConfigValue{value: MSPConfig{type 0, config}}


def fabric_msp_config(mspid, root_certs=(), admins=(), ou_ids=(), node_ous=("client", "peer", "admin", "orderer"),
                      node_ou_certs=None, hash_family="SHA2", intermediate_certs=(), crls=()):
    """FabricMSPConfig bytes: root CA PEMs, admin PEMs, OrganizationalUnitIdentifiers [(cert PEM,
    ou)], NodeOUs (client, peer, admin, orderer identifiers; None entries are left out; node_ous
    None = disabled; node_ou_certs: role index -> certificate PEM)"""
    out = f_str(1, mspid)
    for c in root_certs:
        out += f_bytes(2, c)
    for c in intermediate_certs:
        out += f_bytes(3, c)
    for c in admins:
        out += f_bytes(4, c)
    for c in crls:  # revocation_list
        out += f_bytes(5, c)
    for cert, ou in ou_ids:
        out += f_msg(7, f_bytes(1, cert) + f_str(2, ou))
    out += f_msg(8, f_str(1, hash_family) + f_str(2, "SHA256"))
    if node_ous is not None:
        body = f_varint(1, 1)
        for k, o in enumerate(node_ous):
            if o is not None:
                cert = (node_ou_certs or {}).get(k)
                body += f_msg(2 + k, (f_bytes(1, cert) if cert else b"") + f_str(2, o))
        out += f_msg(11, body)
    return out


def msp_value_raw(fabric):
    return f_bytes(2, f_varint(1, 0) + f_bytes(2, fabric))


def group(groups=(), values=(), policies=()):
    out = b""
    for k, g in groups:
        out += f_msg(2, _entry(k, g))
    for k, v in values:
        out += f_msg(3, _entry(k, v))
    for k, p in policies:
        out += f_msg(4, _entry(k, p))
    return out


def make_config(mspids, endorsement_rule=MAJORITY, org_endorsement_role=PEER, hash_families=None, orderer_mspids=(),
                block_validation=None, orderer_writers_role=MEMBER, msp_configs=None):
    """-> common.Config bytes; org group names org1..orgN (the MSP ids are separate names).
    orderer_mspids: orderer orgs (group names ord1..ordN) -> an Orderer group; block_validation:
    its BlockValidation policy bytes (ConfigPolicy), default IMPLICIT_META ANY Writers.
    msp_configs: mspid -> FabricMSPConfig bytes (fabric_msp_config) replacing the default MSP
    value (root CAs etc. for the MSP cache-miss path)."""
    def mspv(m, fam):
        raw = (msp_configs or {}).get(m)
        return msp_value_raw(raw) if raw is not None else msp_value(m, fam)
    orgs = []
    for i, m in enumerate(mspids):
        fam = (hash_families or {}).get(m, "SHA2")
        pols = [("Endorsement", config_policy(SIGNATURE, signature_policy(1, [(m, org_endorsement_role)]))),
                ("Readers", config_policy(SIGNATURE, signature_policy(1, [(m, ADMIN), (m, PEER), (m, CLIENT)]))),
                ("Writers", config_policy(SIGNATURE, signature_policy(1, [(m, ADMIN), (m, CLIENT)]))),
                ("Admins", config_policy(SIGNATURE, signature_policy(1, [(m, ADMIN)])))]
        orgs.append(("org%d" % (i + 1), group(values=[("MSP", mspv(m, fam))], policies=pols)))
    app = group(groups=orgs, policies=[("Endorsement", implicit_meta(endorsement_rule, "Endorsement")),
                                       ("LifecycleEndorsement", implicit_meta(MAJORITY, "Endorsement")),
                                       ("Readers", implicit_meta(ANY, "Readers")),
                                       ("Writers", implicit_meta(ANY, "Writers")),
                                       ("Admins", implicit_meta(MAJORITY, "Admins"))])
    groups = [("Application", app)]
    if orderer_mspids:
        ords = []
        for i, m in enumerate(orderer_mspids):
            fam = (hash_families or {}).get(m, "SHA2")
            pols = [("Readers", config_policy(SIGNATURE, signature_policy(1, [(m, MEMBER)]))),
                    ("Writers", config_policy(SIGNATURE, signature_policy(1, [(m, orderer_writers_role)]))),
                    ("Admins", config_policy(SIGNATURE, signature_policy(1, [(m, ADMIN)])))]
            ords.append(("ord%d" % (i + 1), group(values=[("MSP", mspv(m, fam))], policies=pols)))
        bv = block_validation if block_validation is not None else implicit_meta(ANY, "Writers")
        groups.append(("Orderer", group(groups=ords, policies=[("BlockValidation", bv),
                                                                ("Readers", implicit_meta(ANY, "Readers")),
                                                                ("Writers", implicit_meta(ANY, "Writers")),
                                                                ("Admins", implicit_meta(MAJORITY, "Admins"))])))
    root = group(groups=groups, policies=[("Readers", implicit_meta(ANY, "Readers")),
                                                          ("Writers", implicit_meta(ANY, "Writers")),
                                                          ("Admins", implicit_meta(MAJORITY, "Admins"))])
    return f_varint(1, 1) + f_msg(2, root)


def channel_ref(path):
    """ApplicationPolicy{channel_config_policy_reference: path}"""
    return f_str(2, path)
