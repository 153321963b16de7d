"""CPU: key-level (state-based) endorsement in the restated committer (oracle/v20.py) against the
reference tests' known answers (tests/golden/sbe_known_answers.json), and the blocks the
reference cannot validate (dependency extraction failing or panicking before a later vscc)."""
import pytest

from fabric_amd.synth import blocks
from oracle import v20
from tests import sbe_cases
from tests.blockfix import block_from_envs, network

CASES = sbe_cases.load()


def model(case):
    return v20.ChannelModel("testchannelid", case["identities"], case["chaincodes"], kvmeta=case["kvmeta"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_known_answer(case):
    flags = v20.validate_block(model(case), case["block"])
    assert len(flags) == len(case["expected"])
    bad = [(i, f, e) for i, (f, e) in enumerate(zip(flags, case["expected"])) if not sbe_cases.matches(f, e)]
    assert not bad, bad


def test_parallel_validation_codes():
    """every invalid tx of TestParallelValidation fails its endorsement policy (10)"""
    c = next(c for c in CASES if c["name"] == "TestParallelValidation")
    flags = v20.validate_block(model(c), c["block"])
    assert {f for f, e in zip(flags, c["expected"]) if e == "not_valid"} == {10}


def _net_model(net, kvmeta=None):
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    return v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=kvmeta)


@pytest.mark.parametrize("seed", range(6))
def test_synthetic_blocks_decide(seed):
    """generated key-level blocks: the oracle decides (no Unsupported) and both outcomes occur"""
    net = network()
    blk, kvmeta = sbe_cases.make_sbe_block(net, 40, seed)
    flags = v20.validate_block(_net_model(net, kvmeta), blk)
    assert 0 in flags and 10 in flags


def test_untranslatable_parameter_halts():
    net = network()
    _, _, envs = blocks.make_block(net, 2, number=1, seed=3, faults=())
    m = _net_model(net, {("mycc", "", b"k%07d" % 0): b"\xff\x01"})
    # generated txs write 4 random keys: put the garbage parameter on one of them
    key = v20.parse_rwset(v20.get_action_from_envelope(envs[0])[0].get("results"))[0]["kv"]["writes"][0]["key"]
    m.kvmeta = {("mycc", "", key.encode()): b"\xff\x01"}
    with pytest.raises(v20.Unsupported):
        v20.validate_block(m, block_from_envs(envs))


def test_extraction_failure_before_a_writer():
    """a tx whose Payload does not unmarshal, then a valid writer: the reference waits forever"""
    net = network()
    _, _, envs = blocks.make_block(net, 3, number=1, seed=4, faults=())
    bad = blocks.f_bytes(1, b"\x0a\x05ab") + blocks.f_bytes(2, b"sig")  # Payload: truncated field
    assert v20.extract_dependencies(bad)[0] == v20.EXTRACT_FAIL
    m = _net_model(net)
    with pytest.raises(v20.Unsupported):
        v20.validate_block(m, block_from_envs([envs[0], bad, envs[1]]))
    alone = v20.validate_block(m, block_from_envs([bad]))[0]
    assert v20.validate_block(m, block_from_envs([envs[0], envs[1], bad])) == [0, 0, alone]


def test_extraction_panic_before_a_vscc():
    """a Transaction with no actions panics the extraction of any later tx's vscc"""
    net = network()
    _, _, envs = blocks.make_block(net, 2, number=1, seed=5, faults=())
    env = v20.decode("Envelope", envs[0])
    pl = v20.decode("Payload", env["payload"])
    hdr = blocks.f_msg(1, blocks.f_bytes(1, pl["header"]["channel_header"]) + blocks.f_bytes(2, pl["header"]["signature_header"]))
    noact = blocks.f_bytes(1, hdr) + blocks.f_bytes(2, env["signature"])  # Payload without data
    assert v20.extract_dependencies(noact)[0] == v20.EXTRACT_PANIC
    m = _net_model(net)
    with pytest.raises(v20.Unsupported):
        v20.validate_block(m, block_from_envs([noact, envs[1]]))
    assert v20.validate_block(m, block_from_envs([envs[1], noact]))[0] == 0
