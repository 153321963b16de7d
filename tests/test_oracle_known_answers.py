"""CPU: the restated committer (oracle/v20.py) reproduces the reference tests' own assertions
(validator_test.go, fullflow_test.go, builtin v20 validation_logic_test.go, cauthdsl_test.go;
tests/golden/committer_known_answers.json)."""
import pytest

from oracle import v20
from tests.blockfix import block_from_envs
from tests.known_answers import bad_tx_envelopes, load, matches

VT, CASES = load()


def model(case):
    return v20.ChannelModel(case["channel"], case["identities"], case["chaincodes"], case["committed"])


@pytest.mark.parametrize("case", [c for c in CASES if "block" in c], ids=[c["name"] for c in CASES if "block" in c])
def test_known_answer(case):
    got = v20.validate_block(model(case), case["block"])
    assert len(got) == len(case["expected"])
    bad = [(i, g, e) for i, (g, e) in enumerate(zip(got, case["expected"])) if not matches(g, e, VT)]
    assert not bad, bad[:5]


def split_bad_tx(case):
    """TestBadTx mutations -> (envelopes the oracle codes, envelopes outside the model: a mutated
    certificate of the channel's MSP, which the MSP layer -- not the engine -- would reject)"""
    coded, unsup = [], []
    for e in bad_tx_envelopes(case):
        try:
            v20.validate_block(model(case), block_from_envs([e], number=2))
            coded.append(e)
        except v20.Unsupported:
            unsup.append(e)
    return coded, unsup


def test_bad_tx_never_valid():
    case = [c for c in CASES if c["name"] == "TestBadTx"][0]
    coded, unsup = split_bad_tx(case)
    got = v20.validate_block(model(case), block_from_envs(coded, number=2))
    assert 0 not in got and len(coded) > len(unsup)
