"""Restated deliver-side block verification (TEST INFRASTRUCTURE ONLY -- the oracle).

BlockVerificationAssistant.VerifyBlock (common/deliverclient/block_verification.go:243-273),
with the orderer signature policy (sigVerifierFunc, :265-268) when a channel model is given:
  verifyHeader   :311-331  header != nil; Number == last.Number + 1; PreviousHash ==
                           lastBlockHeaderHash when that hash is non-empty
  verifyMetadata :303-309  len(Metadata.Metadata) >= len(BlockMetadataIndex_name) == 5
  protoutil.BlockDataHash (protoutil/blockutils.go:69-74):
      VerifyTransactionsAreWellFormed (:310-350) -- non-empty, HasConfigTx
      (protoutil/commonutils.go:198-230) skips the check, else every envelope unmarshals,
      has payload and signature, and proto.Marshal(env) == raw bytes
      ComputeBlockDataHash (:76-79) = SHA-256(bytes.Join(Data, nil))
  Header.DataHash == that hash (:258-263)
  sigVerifierFunc = protoutil.BlockSignatureVerifier(bft, consenters, policy) (blockutils.go:
      245-290) with policy = /Channel/Orderer/BlockValidation (verifier_assembler.go:32-56):
      Metadata at metadata[SIGNATURES] -> SignedData{creator of each SignatureHeader,
      md.Value || signature_header || BlockHeaderBytes(header), signature} ->
      policy.EvaluateSignedData (oracle/v20.py: SignatureSetToValidIdentities + cauthdsl /
      ImplicitMeta over the channel config); BFT identifier headers are outside the model
  then lastBlockHeader(Hash) advance (:268-270)
  BlockHeaderHash (:48-67) = SHA-256(asn1.Marshal{Number *big.Int, PreviousHash, DataHash})

proto.Marshal is restated from google.golang.org/protobuf v1.33.0 (vendored): known fields
in field-number order with minimal encodings, proto3 empty bytes omitted, then the unknown
fields' raw bytes in the order they were read (impl/encode.go appendUnknown).
"""
import hashlib

from .protowire import DecodeError, _skip, _varint, decode
from .v20 import Unsupported, _eval_channel_policy

OK, UNPARSABLE, NO_HEADER, NUMBER, PREV_HASH, METADATA, EMPTY, TX_MALFORMED, DATA_HASH, SIGNATURES, \
    SIG_UNSUPPORTED = range(11)
BLOCK_VALIDATION = "/Channel/Orderer/BlockValidation"  # common/policies/policy.go BlockValidation


def _enc_varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def marshal_envelope_roundtrip(raw):
    """proto.Unmarshal(raw, &Envelope{}) then proto.Marshal; returns (env dict, marshalled)
    or raises DecodeError."""
    raw = bytes(raw)
    env = decode("Envelope", raw)  # the decode rules (errors)
    unknown = []
    o = 0
    while o < len(raw):
        start = o
        tag, o = _varint(raw, o)
        num, wt = tag >> 3, tag & 7
        if num in (1, 2) and wt == 2:
            ln, o = _varint(raw, o)
            o += ln
            continue
        o = _skip(raw, o, num, wt)
        unknown.append(raw[start:o])
    out = b""
    for num, key in ((1, "payload"), (2, "signature")):
        v = env.get(key)
        if v:
            out += _enc_varint(num << 3 | 2) + _enc_varint(len(v)) + v
    return env, out + b"".join(unknown)


def _has_config_tx(data):
    if len(data) != 1:
        return False
    try:
        env = decode("Envelope", data[0])
        pl = decode("Payload", env.get("payload"))
        if pl.get("header") is None:
            return False
        ch = decode("ChannelHeader", pl["header"].get("channel_header"))
    except DecodeError:
        return False
    return ch.get("type", 0) == 1


def verify_transactions_well_formed(data):
    """None if well formed, else the index of the first bad envelope (-1: empty block)."""
    if not data:
        return -1
    if _has_config_tx(data):
        return None
    for i, raw in enumerate(data):
        try:
            env, expected = marshal_envelope_roundtrip(raw)
        except DecodeError:
            return i
        if not env.get("payload") or not env.get("signature"):
            return i
        if expected != bytes(raw):
            return i
    return None


def _der_len(n):
    if n < 128:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def block_header_bytes(number, prev, data_hash):
    nb = number.to_bytes(max(1, (number.bit_length() + 7) // 8), "big")
    if nb[0] & 0x80:
        nb = b"\x00" + nb
    body = b"\x02" + _der_len(len(nb)) + nb
    for x in (prev or b"", data_hash or b""):
        body += b"\x04" + _der_len(len(x)) + x
    return b"\x30" + _der_len(len(body)) + body


def block_header_hash(number, prev, data_hash):
    return hashlib.sha256(block_header_bytes(number, prev, data_hash)).digest()


def block_signature_set(blk, bft=False):
    """BlockSignatureVerifier up to EvaluateSignedData (blockutils.go:247-287): the SignedData
    set [(data, identity, signature)], or None when the verifier returns an error first
    (Metadata or a SignatureHeader does not unmarshal)."""
    md_raw = (blk["metadata"].get("metadata") or [b""])[0] or b""
    try:
        md = decode("Metadata", md_raw)
    except DecodeError:
        return None
    hdr = blk["header"]
    hb = block_header_bytes(hdr.get("number", 0), hdr.get("previous_hash"), hdr.get("data_hash"))
    out = []
    for ms in md.get("signatures", []):
        sh_raw = ms.get("signature_header") or b""
        if bft and not sh_raw and ms.get("identifier_header"):
            raise Unsupported("BFT identifier header (consenter lookup by id)")
        try:
            sh = decode("SignatureHeader", sh_raw)
        except DecodeError:
            return None
        out.append(((md.get("value") or b"") + sh_raw + hb, sh.get("creator") or b"", ms.get("signature") or b""))
    return out


def block_signatures_ok(model, blk, policy=BLOCK_VALIDATION, bft=False):
    """sigVerifierFunc(header, metadata) == nil; raises v20.Unsupported outside the model"""
    pol = model.channel_policy(policy)
    sigset = block_signature_set(blk, bft)
    if sigset is None:
        return False
    model.sha3_verify = False  # (the engine's orderer path: SHA3 identities are outside its model)
    try:
        return _eval_channel_policy(model, pol, sigset)
    finally:
        model.sha3_verify = True


def verify_blocks(blocks, chain=None, sig=None):
    """chain: None or dict(number=, header_hash=) (mutated).  sig: None, or dict(model=
    v20.ChannelModel, policy=, bft=) to check the orderer signatures.  Returns per block
    (status, bad_tx, data_hash, header_hash); a signature check outside the model gives
    SIG_UNSUPPORTED for that block and every later one (the reference decides them)."""
    out = []
    for k, raw in enumerate(blocks):
        try:
            blk = decode("Block", raw)
        except DecodeError:
            out.append((UNPARSABLE, None, None, None))
            continue
        hdr = blk.get("header")
        has_data = blk.get("data") is not None
        data = [d if d is not None else b"" for d in (blk["data"].get("data") or [])] if has_data else []
        dh = hashlib.sha256(b"".join(data)).digest() if has_data else None
        hh = block_header_hash(hdr.get("number", 0), hdr.get("previous_hash"), hdr.get("data_hash")) \
            if hdr is not None else None
        if hdr is None:
            out.append((NO_HEADER, None, dh, hh))
            continue
        if chain is not None:
            if hdr.get("number", 0) != chain["number"] + 1:
                out.append((NUMBER, None, dh, hh))
                continue
            if chain.get("header_hash") and (hdr.get("previous_hash") or b"") != chain["header_hash"]:
                out.append((PREV_HASH, None, dh, hh))
                continue
        meta = blk.get("metadata")
        if meta is None or len(meta.get("metadata") or []) < 5:
            out.append((METADATA, None, dh, hh))
            continue
        bad = verify_transactions_well_formed(data)
        if bad is not None:
            out.append((EMPTY, None, dh, hh) if bad < 0 else (TX_MALFORMED, bad, dh, hh))
            continue
        if (hdr.get("data_hash") or b"") != dh:
            out.append((DATA_HASH, None, dh, hh))
            continue
        if sig is not None:
            try:
                ok = block_signatures_ok(sig["model"], blk, sig.get("policy") or BLOCK_VALIDATION,
                                         sig.get("bft", False))
            except Unsupported:
                out.append((SIG_UNSUPPORTED, None, dh, hh))
                for rest in blocks[k + 1:]:
                    out.append((SIG_UNSUPPORTED, None, None, None))
                return out
            if not ok:
                out.append((SIGNATURES, None, dh, hh))
                continue
        out.append((OK, None, dh, hh))
        if chain is not None:
            chain["number"] = hdr.get("number", 0)
            chain["header_hash"] = hh
    return out
