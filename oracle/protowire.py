"""Go protobuf decoding semantics for the Fabric messages on the committer path.

TEST INFRASTRUCTURE ONLY (oracle).  Restates google.golang.org/protobuf v1.33.0 (vendored at
vendor/google.golang.org/protobuf; go.mod:42) as used by proto.Unmarshal:
  * tag = varint; field number outside [1, 2^29-1] -> error (impl/decode.go unmarshalPointer)
  * varints: at most 10 bytes, the 10th <= 1 (protowire.ConsumeVarint)
  * wire types 6/7 -> error; an END_GROUP at message level -> error; unknown START_GROUP is
    skipped to its matching END_GROUP (protowire.consumeFieldValueD)
  * a KNOWN field with the wrong wire type is skipped as an unknown field (errUnknown)
  * proto3 `string` fields must be valid UTF-8 (consumeStringValidateUTF8) -> error
  * proto3 `bytes`: last occurrence wins; an empty value decodes to nil (consumeBytesNoZero
    appends to a nil slice), so presence == non-empty
  * singular embedded message: present once seen (even empty); repeated occurrences MERGE
  * repeated fields append; oneof: the last member seen wins and clears the others
  * int32 = low 32 bits of the varint as signed; bool = varint != 0
"""


class DecodeError(Exception):
    pass


def _varint(b, o):
    v = 0
    for i in range(10):
        if o + i >= len(b):
            raise DecodeError("truncated varint")
        c = b[o + i]
        if i == 9 and c > 1:
            raise DecodeError("varint overflow")
        v |= (c & 0x7F) << (7 * i)
        if c < 0x80:
            return v, o + i + 1
    raise DecodeError("varint overflow")


def _skip(b, o, num, wt, depth=0):
    if wt == 0:
        return _varint(b, o)[1]
    if wt == 1:
        if o + 8 > len(b):
            raise DecodeError("truncated fixed64")
        return o + 8
    if wt == 5:
        if o + 4 > len(b):
            raise DecodeError("truncated fixed32")
        return o + 4
    if wt == 2:
        ln, o = _varint(b, o)
        if ln > len(b) - o:
            raise DecodeError("truncated bytes")
        return o + ln
    if wt == 3:
        if depth > 10000:
            raise DecodeError("recursion")
        while True:
            tag, o = _varint(b, o)
            n2, w2 = tag >> 3, tag & 7
            if n2 < 1 or n2 > (1 << 29) - 1:
                raise DecodeError("bad field number")
            if w2 == 4:
                if n2 != num:
                    raise DecodeError("end group mismatch")
                return o
            o = _skip(b, o, n2, w2, depth + 1)
    raise DecodeError("invalid wire type")


# name -> {num: (field, kind)}; kind: bytes | string | int32 | int64 | uint32 | uint64 | bool |
# enum | msg:Name | rep msg:Name | rep bytes.  ONEOF groups list fields that clear each other.
S = {
    "Block": {1: ("header", "msg:BlockHeader"), 2: ("data", "msg:BlockData"), 3: ("metadata", "msg:BlockMetadata")},
    "BlockHeader": {1: ("number", "uint64"), 2: ("previous_hash", "bytes"), 3: ("data_hash", "bytes")},
    "BlockData": {1: ("data", "rep bytes")},
    "BlockMetadata": {1: ("metadata", "rep bytes")},
    "Metadata": {1: ("value", "bytes"), 2: ("signatures", "rep msg:MetadataSignature")},
    "MetadataSignature": {1: ("signature_header", "bytes"), 2: ("signature", "bytes"),
                          3: ("identifier_header", "bytes")},
    "Envelope": {1: ("payload", "bytes"), 2: ("signature", "bytes")},
    "Payload": {1: ("header", "msg:Header"), 2: ("data", "bytes")},
    "Header": {1: ("channel_header", "bytes"), 2: ("signature_header", "bytes")},
    "ChannelHeader": {1: ("type", "int32"), 2: ("version", "int32"), 3: ("timestamp", "msg:Timestamp"),
                      4: ("channel_id", "string"), 5: ("tx_id", "string"), 6: ("epoch", "uint64"),
                      7: ("extension", "bytes"), 8: ("tls_cert_hash", "bytes")},
    "Timestamp": {1: ("seconds", "int64"), 2: ("nanos", "int32")},
    "SignatureHeader": {1: ("creator", "bytes"), 2: ("nonce", "bytes")},
    "Transaction": {1: ("actions", "rep msg:TransactionAction")},
    "TransactionAction": {1: ("header", "bytes"), 2: ("payload", "bytes")},
    "ChaincodeActionPayload": {1: ("chaincode_proposal_payload", "bytes"), 2: ("action", "msg:ChaincodeEndorsedAction")},
    "ChaincodeEndorsedAction": {1: ("proposal_response_payload", "bytes"), 2: ("endorsements", "rep msg:Endorsement")},
    "Endorsement": {1: ("endorser", "bytes"), 2: ("signature", "bytes")},
    "ProposalResponsePayload": {1: ("proposal_hash", "bytes"), 2: ("extension", "bytes")},
    "ChaincodeAction": {1: ("results", "bytes"), 2: ("events", "bytes"), 3: ("response", "msg:Response"),
                        4: ("chaincode_id", "msg:ChaincodeID")},
    "Response": {1: ("status", "int32"), 2: ("message", "string"), 3: ("payload", "bytes")},
    "ChaincodeID": {1: ("path", "string"), 2: ("name", "string"), 3: ("version", "string")},
    "ChaincodeHeaderExtension": {2: ("chaincode_id", "msg:ChaincodeID")},
    "ChaincodeEvent": {1: ("chaincode_id", "string"), 2: ("tx_id", "string"), 3: ("event_name", "string"),
                       4: ("payload", "bytes")},
    "TxReadWriteSet": {1: ("data_model", "enum"), 2: ("ns_rwset", "rep msg:NsReadWriteSet")},
    "NsReadWriteSet": {1: ("namespace", "string"), 2: ("rwset", "bytes"),
                       3: ("collection_hashed_rwset", "rep msg:CollectionHashedReadWriteSet")},
    "CollectionHashedReadWriteSet": {1: ("collection_name", "string"), 2: ("hashed_rwset", "bytes"),
                                     3: ("pvt_rwset_hash", "bytes")},
    "KVRWSet": {1: ("reads", "rep msg:KVRead"), 2: ("range_queries_info", "rep msg:RangeQueryInfo"),
                3: ("writes", "rep msg:KVWrite"), 4: ("metadata_writes", "rep msg:KVMetadataWrite")},
    "KVRead": {1: ("key", "string"), 2: ("version", "msg:Version")},
    "Version": {1: ("block_num", "uint64"), 2: ("tx_num", "uint64")},
    "KVWrite": {1: ("key", "string"), 2: ("is_delete", "bool"), 3: ("value", "bytes")},
    "KVMetadataWrite": {1: ("key", "string"), 2: ("entries", "rep msg:KVMetadataEntry")},
    "KVMetadataEntry": {1: ("name", "string"), 2: ("value", "bytes")},
    "RangeQueryInfo": {1: ("start_key", "string"), 2: ("end_key", "string"), 3: ("itr_exhausted", "bool"),
                       4: ("raw_reads", "msg:QueryReads"), 5: ("reads_merkle_hashes", "msg:QueryReadsMerkleSummary")},
    "QueryReads": {1: ("kv_reads", "rep msg:KVRead")},
    "QueryReadsMerkleSummary": {1: ("max_degree", "uint32"), 2: ("max_level", "uint32"),
                                3: ("max_level_hashes", "rep bytes")},
    "HashedRWSet": {1: ("hashed_reads", "rep msg:KVReadHash"), 2: ("hashed_writes", "rep msg:KVWriteHash"),
                    3: ("metadata_writes", "rep msg:KVMetadataWriteHash")},
    "KVReadHash": {1: ("key_hash", "bytes"), 2: ("version", "msg:Version")},
    "KVWriteHash": {1: ("key_hash", "bytes"), 2: ("is_delete", "bool"), 3: ("value_hash", "bytes"),
                    4: ("is_purge", "bool")},
    "KVMetadataWriteHash": {1: ("key_hash", "bytes"), 2: ("entries", "rep msg:KVMetadataEntry")},
    "SerializedIdentity": {1: ("mspid", "string"), 2: ("id_bytes", "bytes")},
    "ApplicationPolicy": {1: ("signature_policy", "msg:SignaturePolicyEnvelope"),
                          2: ("channel_config_policy_reference", "string")},
    "SignaturePolicyEnvelope": {1: ("version", "int32"), 2: ("rule", "msg:SignaturePolicy"),
                                3: ("identities", "rep msg:MSPPrincipal")},
    "SignaturePolicy": {1: ("signed_by", "int32"), 2: ("n_out_of", "msg:NOutOf")},
    "NOutOf": {1: ("n", "int32"), 2: ("rules", "rep msg:SignaturePolicy")},
    "MSPPrincipal": {1: ("principal_classification", "enum"), 2: ("principal", "bytes")},
    "MSPRole": {1: ("msp_identifier", "string"), 2: ("role", "enum")},
    "OrganizationUnit": {1: ("msp_identifier", "string"), 2: ("organizational_unit_identifier", "string"),
                         3: ("certifiers_identifier", "bytes")},
    "MSPIdentityAnonymity": {1: ("anonymity_type", "enum")},
    "CombinedPrincipal": {1: ("principals", "rep msg:MSPPrincipal")},
    # channel configuration (common/configtx.pb.go, common/policies.pb.go, msp/msp_config.pb.go);
    # map<string, V> fields are repeated {key = 1, value = 2} entries
    "Config": {1: ("sequence", "uint64"), 2: ("channel_group", "msg:ConfigGroup")},
    "ConfigEnvelope": {1: ("config", "msg:Config"), 2: ("last_update", "bytes")},
    "ConfigGroup": {1: ("version", "uint64"), 2: ("groups", "rep msg:ConfigGroupEntry"),
                    3: ("values", "rep msg:ConfigValueEntry"), 4: ("policies", "rep msg:ConfigPolicyEntry"),
                    5: ("mod_policy", "string")},
    "ConfigGroupEntry": {1: ("key", "string"), 2: ("value", "msg:ConfigGroup")},
    "ConfigValueEntry": {1: ("key", "string"), 2: ("value", "msg:ConfigValue")},
    "ConfigPolicyEntry": {1: ("key", "string"), 2: ("value", "msg:ConfigPolicy")},
    "ConfigValue": {1: ("version", "uint64"), 2: ("value", "bytes"), 3: ("mod_policy", "string")},
    "ConfigPolicy": {1: ("version", "uint64"), 2: ("policy", "msg:Policy"), 3: ("mod_policy", "string")},
    "Policy": {1: ("type", "int32"), 2: ("value", "bytes")},
    "ImplicitMetaPolicy": {1: ("sub_policy", "string"), 2: ("rule", "enum")},
    "MSPConfig": {1: ("type", "int32"), 2: ("config", "bytes")},
    "FabricMSPConfig": {1: ("name", "string"), 2: ("root_certs", "rep bytes"), 3: ("intermediate_certs", "rep bytes"),
                        4: ("admins", "rep bytes"), 5: ("revocation_list", "rep bytes"),
                        7: ("organizational_unit_identifiers", "rep msg:FabricOUIdentifier"),
                        8: ("crypto_config", "msg:FabricCryptoConfig"), 11: ("fabric_node_ous", "msg:FabricNodeOUs")},
    "FabricCryptoConfig": {1: ("signature_hash_family", "string"), 2: ("identity_identifier_hash_function", "string")},
    "FabricNodeOUs": {1: ("enable", "bool"), 2: ("client_ou_identifier", "msg:FabricOUIdentifier"),
                      3: ("peer_ou_identifier", "msg:FabricOUIdentifier"), 4: ("admin_ou_identifier", "msg:FabricOUIdentifier"),
                      5: ("orderer_ou_identifier", "msg:FabricOUIdentifier")},
    "FabricOUIdentifier": {1: ("certificate", "bytes"), 2: ("organizational_unit_identifier", "string")},
    # lifecycle state (peer/lifecycle/db.pb.go, chaincode_definition.pb.go, peer/collection.pb.go)
    "StateData": {1: ("Int64", "int64"), 2: ("Bytes", "bytes"), 3: ("String", "string")},
    "ChaincodeValidationInfo": {1: ("validation_plugin", "string"), 2: ("validation_parameter", "bytes")},
    "CollectionConfigPackage": {1: ("config", "rep msg:CollectionConfig")},
    "CollectionConfig": {1: ("static_collection_config", "msg:StaticCollectionConfig")},
    "StaticCollectionConfig": {1: ("name", "string"), 8: ("endorsement_policy", "bytes")},
}
ONEOF = {
    "RangeQueryInfo": ("raw_reads", "reads_merkle_hashes"),
    "ApplicationPolicy": ("signature_policy", "channel_config_policy_reference"),
    "SignaturePolicy": ("signed_by", "n_out_of"),
    "StateData": ("Int64", "Bytes", "String"),
}
# oneof members keep presence even for zero values (a "set" oneof field is present)
_ONEOF_MEMBERS = {f for v in ONEOF.values() for f in v}


class Msg(dict):
    """Decoded message: missing keys mean 'absent' (Go nil / zero value)."""

    def get(self, k, d=None):
        return dict.get(self, k, d)


def _signed32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def decode(name, b, into=None):
    """proto.Unmarshal(b, &name{}) -> Msg, or raise DecodeError."""
    if b is None:
        b = b""
    b = bytes(b)
    schema = S[name]
    m = Msg() if into is None else into
    oneof = ONEOF.get(name, ())
    o = 0
    n = len(b)
    while o < n:
        tag, o = _varint(b, o)
        num, wt = tag >> 3, tag & 7
        if num < 1 or num > (1 << 29) - 1:
            raise DecodeError("invalid field number")
        if wt == 4:
            raise DecodeError("unexpected end group")
        f = schema.get(num)
        kind = f[1] if f else None
        want = None
        if kind is not None:
            want = 2 if (kind in ("bytes", "string", "rep bytes") or "msg:" in kind) else 0
        if f is None or wt != want:
            o = _skip(b, o, num, wt)
            continue
        field = f[0]
        if want == 0:
            v, o = _varint(b, o)
            if kind == "int32" or kind == "enum":
                v = _signed32(v)
            elif kind == "int64":
                v = v - (1 << 64) if v >> 63 else v
            elif kind == "uint32":
                v &= 0xFFFFFFFF
            elif kind == "bool":
                v = v != 0
            val = v
        else:
            ln, o = _varint(b, o)
            if ln > n - o:
                raise DecodeError("truncated length-delimited field")
            raw = b[o:o + ln]
            o += ln
            if kind == "string":
                try:
                    val = raw.decode("utf-8")
                except UnicodeDecodeError:
                    raise DecodeError("invalid UTF-8")
            elif kind == "bytes":
                val = raw if raw else None  # consumeBytesNoZero: empty -> nil
            elif kind == "rep bytes":
                m.setdefault(field, []).append(raw)
                continue
            elif kind.startswith("rep msg:"):
                m.setdefault(field, []).append(decode(kind[8:], raw))
                continue
            else:  # singular message: merge into the existing one
                sub = m.get(field) if field in m and isinstance(m.get(field), Msg) else None
                val = decode(kind[4:], raw, into=sub)
        if field in oneof:
            for other in oneof:
                if other != field:
                    m.pop(other, None)
        if val is None:
            m.pop(field, None)
        elif kind in ("int32", "int64", "uint32", "uint64", "enum", "bool") and not val and field not in _ONEOF_MEMBERS:
            m.pop(field, None)  # proto3 zero scalar == absent
        elif kind == "string" and val == "" and field not in _ONEOF_MEMBERS:
            m.pop(field, None)
        else:
            m[field] = val
    return m
