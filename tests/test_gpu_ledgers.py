"""GPU replay of the reference's own sample ledgers (tests/golden/sample_ledgers.*): every
block's transactions enter fgv_mvcc_validate_block as committer-VALID, from an empty state,
committing as they go; the TRANSACTIONS_FILTER that comes out equals the one the reference
stored, and the commit hash computed from it (fgv_commit_hash) equals the stored
Metadata[COMMIT_HASH] -- a pin on the reference itself, not on our oracle.  The v2.0 ledger's
config blocks are outside the MVCC model (FGV_EUNSUPPORTED; they write only namespace "")."""
import pytest

from fabric_amd import _lib
from oracle.protowire import decode
from tests.test_oracle_ledgers import ledgers, tx_type

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["v11_ledger1", "v11_ledger2", "v20_testchannel"])
def test_replay_flags_and_commit_hashes(name):
    eng = _lib.Engine(0)
    eng.statedb_init(1 << 12, 1 << 20)
    prev, nvalidated = b"", 0
    for b in ledgers()[name]:
        data = decode("Block", b["block"])["data"].get("data", [])
        if all(tx_type(d) == 1 for d in data):
            if b["number"] > 0:
                with pytest.raises(_lib.Unsupported):
                    eng.mvcc_validate(b["block"], b["number"], [0] * len(data), commit=True)
            flags = b["flags"]
        else:
            flags = list(eng.mvcc_validate(b["block"], b["number"], [0] * len(data), commit=True))
            assert flags == b["flags"], b["number"]
            nvalidated += 1
        if b["commit_hash"] is not None:
            prev = _lib.commit_hash(b["block"], flags, b["number"], prev)
            assert prev.hex() == b["commit_hash"], b["number"]
    assert nvalidated >= 8
    eng.close()
