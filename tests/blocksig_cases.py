"""Orderer-signature cases for VerifyBlock with sigVerifierFunc (oracle/blockverify.py and
fgv_blocks_verify_signed).  Each case: a channel setup (identities + config), a batch of
blocks, the chain state, the policy path, the BFT flag, and the statuses the reference gives --
written down from the reference's semantics (generation-time facts), not from the oracle:

  protoutil/blockutils.go:245-290  BlockSignatureVerifier: Metadata / SignatureHeader unmarshal
        errors fail the block; SignedData{creator, value||signature_header||BlockHeaderBytes,
        signature} per MetadataSignature, in order
  common/policies/policy.go:363-395  SignatureSetToValidIdentities: unknown MSP -> skipped,
        duplicate identity -> skipped before verify, failed verify -> skipped
  common/policies/implicitmeta.go:69-104  ANY / MAJORITY over the orderer orgs' Writers; an
        unknown rule gives threshold 0: only "no sub-policy satisfied" passes
  deliverclient/block_verification.go:243-273  the chain advances only past verified blocks

The reference's own orderer signatures are the pin: the v2.0 sample ledger's blocks 1..19 carry
metadata[SIGNATURES] written by its orderer (tests/test_oracle_blocksig.py, tests/test_gpu_blocksig.py)."""
import hashlib

from fabric_amd.synth import blocks as B
from fabric_amd.synth import chanconfig as CC
from fabric_amd.synth import orderer as OR

OK, NUMBER, PREV_HASH, DATA_HASH, SIGNATURES, UNSUP = 0, 3, 4, 8, 9, 10

_CACHE = {}


def world():
    """(net, orderers, identities, configs{name: bytes}) -- built once"""
    if "w" not in _CACHE:
        net = B.Network(seed=11, orgs=2, clients=8)
        ords = OR.Orderers(seed=11, orgs=2, per_org=2)
        ids = net.identities() + ords.identities()
        cfg = dict(
            any=CC.make_config(net.mspids, orderer_mspids=ords.mspids),
            majority=CC.make_config(net.mspids, orderer_mspids=ords.mspids,
                                    block_validation=CC.implicit_meta(CC.MAJORITY, "Writers")),
            rule7=CC.make_config(net.mspids, orderer_mspids=ords.mspids,
                                 block_validation=CC.implicit_meta(7, "Writers")),
            orderer_role=CC.make_config(net.mspids, orderer_mspids=ords.mspids, orderer_writers_role=CC.ORDERER),
            peer_role=CC.make_config(net.mspids, orderer_mspids=ords.mspids, orderer_writers_role=CC.PEER),
            direct=CC.make_config(net.mspids, orderer_mspids=ords.mspids,
                                  block_validation=CC.config_policy(CC.SIGNATURE, CC.signature_policy(
                                      2, [(ords.mspids[0], CC.MEMBER), (ords.mspids[1], CC.MEMBER)]))),
        )
        _CACHE["w"] = (net, ords, ids, cfg)
    return _CACHE["w"]


def chain_blocks(net, n, first=1, prev=b"\x00" * 32, ntx=4, seed=0):
    """n consecutive unsigned blocks; returns (blocks, header hash after each)"""
    out, hashes = [], []
    for k in range(n):
        num = first + k
        blk, _, envs = B.make_block(net, ntx, number=num, seed=1000 * seed + num, prev_hash=prev, threads=1)
        out.append(blk)
        prev = B.header_hash(num, prev, envs)
        hashes.append(prev)
    return out, hashes


def _raw_meta(block, meta0):
    return OR.with_signatures(block, meta0)


def cases():
    """[dict(name, config, drop, blocks, chain, policy, bft, expect)]; drop: serialized
    identities left out of the registration; chain: None or (number, header_hash | None)."""
    net, ords, ids, cfg = world()
    o1a, o1b, o2a, o2b = ords.nodes  # OrdererMSP x2, Orderer2MSP x2
    out = []

    def add(name, blks, expect, config="any", chain=None, policy=None, bft=False, drop=()):
        out.append(dict(name=name, config=config, drop=tuple(drop), blocks=blks, chain=chain, policy=policy,
                        bft=bft, expect=expect))

    raw, hh = chain_blocks(net, 6, seed=1)
    s = OR.sign_block
    # the chain of signed blocks: every block verifies and advances the chain
    add("good_chain", [s(b, [o1a], last_config=0, nonce_seed=i) for i, b in enumerate(raw)], [OK] * 6,
        chain=(0, None))
    # a bad signature fails its block, which does not advance the chain: the next block then fails
    # the number check (expected 2, got 3)
    add("bad_sig_stops_chain", [s(raw[0], [o1a]), s(raw[1], [o1a], bad=(0,)), s(raw[2], [o1a])],
        [OK, SIGNATURES, NUMBER], chain=(0, None))
    add("retry_after_bad_sig", [s(raw[0], [o1a], bad=(0,)), s(raw[0], [o1b])], [SIGNATURES, OK], chain=(0, None))
    b0 = raw[0]
    add("no_signatures", [_raw_meta(b0, b""), _raw_meta(b0, B.f_bytes(1, b"value-only"))], [SIGNATURES] * 2)
    add("peer_signer", [s(b0, [net.peers[0]])], [SIGNATURES])          # not a Writer of an orderer org
    add("rogue_signer", [s(b0, [net.rogue])], [SIGNATURES])            # unknown MSP: skipped
    add("one_of_two_bad_any", [s(b0, [o1a, o2a], bad=(0,)), s(b0, [o1a, o2a], bad=(1,)),
                               s(b0, [o1a, o2a], bad=(0, 1))], [OK, OK, SIGNATURES])
    # duplicate identity: the first copy fails to verify, so it is not yet "seen"; the second verifies
    add("duplicate_signer", [s(b0, [o1a, o1a], bad=(0,)), s(b0, [o1a, o1a], bad=(1,))], [OK, OK])
    # signature over another block's header (a replayed block signature)
    n1, p1, d1 = OR.block_header(raw[1])
    add("replayed_signature", [s(b0, [o1a], header_override=(n1, p1, d1))], [SIGNATURES])
    add("high_s", [_high_s(b0, o1a)], [SIGNATURES])
    # malformed metadata: a truncated Metadata, and a good signature followed by a malformed
    # signature header (the verifier errors out before any policy evaluation)
    good_md = OR.signature_metadata(b0, [o1a])
    bad_hdr = good_md + B.f_msg(2, B.f_bytes(1, b"\x0a\xff") + B.f_bytes(2, b"\x30\x00"))
    add("malformed_metadata", [_raw_meta(b0, good_md[:-3]), _raw_meta(b0, bad_hdr)], [SIGNATURES, SIGNATURES])
    # the metadata value is part of the signed message
    add("value_tampered", [_tamper_value(b0, o1a)], [SIGNATURES])
    # MAJORITY over two orderer orgs: both orgs must sign
    add("majority", [s(b0, [o1a]), s(b0, [o1a, o1b]), s(b0, [o1a, o2b]), s(b0, [o2a, o1b], bad=(0,))],
        [SIGNATURES, SIGNATURES, OK, SIGNATURES], config="majority")
    # a signature policy directly at BlockValidation: 2-of-(OrdererMSP.member, Orderer2MSP.member)
    add("direct_signature_policy", [s(b0, [o1a, o2a]), s(b0, [o1a, o1b])], [OK, SIGNATURES], config="direct")
    # NodeOU roles: Writers = OR('OrdererMSP.orderer') (role bit set) / OR('OrdererMSP.peer') (not)
    add("orderer_role", [s(b0, [o1a])], [OK], config="orderer_role")
    add("peer_role", [s(b0, [o1a])], [SIGNATURES], config="peer_role")
    # ImplicitMeta with an unknown rule: threshold 0 -> passes only when no sub-policy is satisfied
    add("rule7_threshold0", [s(b0, [o1a]), s(b0, [net.peers[0]]), _raw_meta(b0, b"")],
        [SIGNATURES, OK, OK], config="rule7")
    # policy paths: absent, outside /Channel/, relative
    add("absent_policy", [s(b0, [o1a])], [SIGNATURES], policy="/Channel/Orderer/Nope")
    add("foreign_root_policy", [s(b0, [o1a])], [SIGNATURES], policy="/Other/Orderer/BlockValidation")
    add("relative_policy", [s(b0, [o1a])], [OK], policy="Orderer/BlockValidation")
    # BFT: a signature that names its consenter by identifier header
    ident_sig = B.f_msg(2, B.f_bytes(2, b"\x30\x06\x02\x01\x01\x02\x01\x01") + B.f_bytes(3, B.f_varint(1, 2)))
    md_bft = good_md + ident_sig
    add("bft_identifier_header", [s(b0, [o1a]), _raw_meta(b0, md_bft), s(raw[1], [o1a])], [OK, UNSUP, UNSUP],
        bft=True)
    # ... without BFT the same signature is an empty creator: skipped, the good one satisfies
    add("identifier_header_not_bft", [_raw_meta(b0, md_bft)], [OK])
    # an unregistered certificate of a channel MSP: outside the model from that block on; blocks
    # before it are decided
    add("unregistered_orderer", [s(raw[0], [o1a]), s(raw[1], [o1b]), s(raw[2], [o1a])], [OK, UNSUP, UNSUP],
        chain=(0, None), drop=(o1b.serialized,))
    # ... but a block that fails earlier (data hash) never reaches the signature check
    add("unregistered_unreached", [_bad_data_hash(s(b0, [o1b]))], [DATA_HASH], drop=(o1b.serialized,))
    # no channel config: the policy cannot be resolved
    add("no_config", [s(b0, [o1a])], [UNSUP], config=None)
    return out


def _high_s(block, ident):
    """a valid signature made high-S (N - s): the BCCSP verifier rejects it (IsLowS)"""
    from fabric_amd.synth import sign_rs, der_encode
    N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    number, prev, dh = OR.block_header(block)
    value = B.f_msg(1, B.f_varint(1, 0))
    sh = B.f_bytes(1, ident.serialized) + B.f_bytes(2, b"n" * 24)
    r, s_ = sign_rs(ident.key, hashlib.sha256(value + sh + OR.header_der(number, prev, dh)).digest())
    sig = der_encode(r, N - s_)
    return OR.with_signatures(block, B.f_bytes(1, value) + B.f_msg(2, B.f_bytes(1, sh) + B.f_bytes(2, sig)))


def _tamper_value(block, ident):
    """signed over value LastConfig{0}, shipped with value LastConfig{1}"""
    md = OR.signature_metadata(block, [ident], last_config=0)
    v0, v1 = B.f_msg(1, B.f_varint(1, 0)), B.f_msg(1, B.f_varint(1, 1))
    assert md.startswith(B.f_bytes(1, v0))
    return OR.with_signatures(block, B.f_bytes(1, v1) + md[len(B.f_bytes(1, v0)):])


def _bad_data_hash(block):
    """the same block with a zeroed Header.DataHash (signatures left as they are)"""
    number, prev, dh = OR.block_header(block)
    parts = OR._fields(block)
    hdr = B.f_varint(1, number) + B.f_bytes(2, prev) + B.f_bytes(3, b"\x00" * 32)
    return b"".join(B.f_msg(n, hdr if n == 1 else p) for n, p in parts)


def identities_for(case):
    _, _, ids, _ = world()
    return [(ser, i) for ser, i in ids if ser not in case["drop"]]


def config_for(case):
    return None if case["config"] is None else world()[3][case["config"]]


def oracle_model(case):
    from oracle import v20
    net = world()[0]
    return v20.ChannelModel(net.channel, identities_for(case), {}, config=config_for(case),
                            msps=() if case["config"] is not None else tuple(world()[1].mspids))


def chain_dict(case):
    return None if case["chain"] is None else dict(number=case["chain"][0], header_hash=case["chain"][1])
