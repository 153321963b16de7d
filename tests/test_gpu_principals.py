"""GPU parity of the non-ROLE principals in the policy fold (ROLE, IDENTITY, ORGANIZATION_UNIT,
ANONYMITY, COMBINED; device fold and host fold): the reference's msp_test.go SatisfiesPrincipal
assertions as endorsement policies (tests/golden/principal_known_answers.json) come out with the
reference's codes, the signer resolved through the channel's FabricMSPConfig (MSP cache miss:
its OUs and certifier computed by the engine) or registered with fgv_msp_identity_ous; registered
without its OUs, a transaction that reaches an OU principal is Unsupported on both sides."""
import pytest

from fabric_amd import _lib, txvalidator
from oracle import v20
from tests import principal_cases as PC

pytestmark = pytest.mark.gpu
C = PC.load()
MODES = pytest.mark.parametrize("mode", [0, 1], ids=["devparse", "hostparse"])


def _eng(ids, mode):
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, "testchannelid", ids, C["chaincodes"], config=C["config"])
    return eng


@MODES
@pytest.mark.parametrize("reg", ["config", "registered"])
def test_principal_known_answers(mode, reg):
    ids = [] if reg == "config" else [C["ident"](True)]
    eng = _eng(ids, mode)
    got = list(eng.validate_blocks([C["block"]])[0])
    assert got == C["expected"], [(n, g, e) for n, g, e in zip(C["names"], got, C["expected"]) if g != e]
    if reg == "config":  # the cache miss registered the signer with its OUs
        rec = eng.msp_identity(ids[0][0] if ids else C["ident"](True)[0])
        assert rec["valid"] and rec["roles"] == 3
    eng.close()


@MODES
def test_ou_principal_without_ous(mode):
    ids = [C["ident"](False)]
    eng = _eng(ids, mode)
    for name, blk, exp in zip(C["names"], PC.single_blocks(C["block"]), C["expected"]):
        try:
            want = v20.validate_block(v20.ChannelModel("testchannelid", ids, C["chaincodes"], config=C["config"]), blk)
        except v20.Unsupported:
            with pytest.raises(_lib.Unsupported):
                eng.validate_blocks([blk])
            continue
        assert list(eng.validate_blocks([blk])[0]) == want == [exp], name
    # the OUs given afterwards: every case decides
    eng.msp_identity_ous(ids[0][0], C["ident"](True)[1].ous)
    assert list(eng.validate_blocks([C["block"]])[0]) == C["expected"]
    eng.close()
