"""GPU: libfgv reproduces the reference tests' own assertions (tests/golden/
committer_known_answers.json) in both parse modes, and equals the oracle code for code."""
import pytest

from fabric_amd import _lib, txvalidator
from oracle import v20
from tests.known_answers import load, matches

pytestmark = pytest.mark.gpu
VT, CASES = load()


def _engine(case, mode):
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, case["channel"], case["identities"], case["chaincodes"], case["committed"])
    return eng


@pytest.mark.parametrize("mode", [0, 1])
def test_bad_tx_never_valid(mode):
    """fullflow_test.go TestBadTx: every one-byte payload mutation and a corrupted signature are
    never VALID (engine == oracle); mutated channel certificates come out Unsupported."""
    from tests.blockfix import block_from_envs
    from tests.test_oracle_known_answers import split_bad_tx
    case = [c for c in CASES if c["name"] == "TestBadTx"][0]
    coded, unsup = split_bad_tx(case)
    eng = _engine(case, mode)
    blk = block_from_envs(coded, number=2)
    got = list(eng.validate_blocks([blk])[0])
    assert got == v20.validate_block(v20.ChannelModel(case["channel"], case["identities"], case["chaincodes"]), blk)
    assert 0 not in got
    for e in unsup[:10]:
        with pytest.raises(_lib.Unsupported):
            eng.validate_blocks([block_from_envs([e], number=2)])
    eng.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_known_answers(mode):
    for case in CASES:
        if "block" not in case:
            continue
        eng = _lib.Engine(0)
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, case["channel"], case["identities"], case["chaincodes"], case["committed"])
        got = list(eng.validate_blocks([case["block"]])[0])
        exp = v20.validate_block(v20.ChannelModel(case["channel"], case["identities"], case["chaincodes"],
                                                  case["committed"]), case["block"])
        assert got == exp, case["name"]
        assert all(matches(g, e, VT) for g, e in zip(got, case["expected"])), case["name"]
        eng.close()
