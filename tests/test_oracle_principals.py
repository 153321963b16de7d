"""The restated SatisfiesPrincipal (oracle/v20.py: ROLE, IDENTITY, ORGANIZATION_UNIT, ANONYMITY,
COMBINED, MSP v1.4.3) pinned by the reference's msp_test.go assertions
(tests/golden/principal_known_answers.json): the SampleOrg signer resolved through the channel's
FabricMSPConfig, or registered with its OUs; without its OUs an OU principal is undecidable."""
import pytest

from oracle import v20
from tests import principal_cases as PC

C = PC.load()


def _model(ids):
    return v20.ChannelModel("testchannelid", ids, C["chaincodes"], config=C["config"])


@pytest.mark.parametrize("mode", ["config", "registered"])
def test_principal_known_answers(mode):
    ids = [] if mode == "config" else [C["ident"](True)]
    got = v20.validate_block(_model(ids), C["block"])
    assert got == C["expected"], [(n, g, e) for n, g, e in zip(C["names"], got, C["expected"]) if g != e]


def test_ou_principal_without_ous_is_unsupported():
    ids = [C["ident"](False)]
    for name, blk, exp in zip(C["names"], PC.single_blocks(C["block"]), C["expected"]):
        ou_case = "OU" in name or "member+ou" in name or "2-of" in name or "1-of" in name
        try:
            got = v20.validate_block(_model(ids), blk)
        except v20.Unsupported:
            assert ou_case, name
            continue
        assert got == [exp], name
        # (an OU principal that fails before the OUs are read -- other MSP, bad bytes -- decides)
        assert not ou_case or exp == 10 or name.startswith("1-of"), name
