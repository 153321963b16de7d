"""Python mirror of the reference's committer interfaces over the HIP engine.

  TxValidator.validate(block)  ~ core/committer/txvalidator/v20/validator.go:180
                                 (TxValidator.Validate; returns TxValidationFlags)
  setup_channel(engine, ...)   ~ the channel resources the reference validator is wired with
                                 (MSP manager identities, lifecycle ValidationInfo, ledger)

There is no CPU fallback: FGV_EUNSUPPORTED / device errors propagate as exceptions so the
caller (a Go shim in production) runs the reference code for that batch.
"""
import numpy as np

from ._lib import Engine, Unsupported  # noqa: F401


def setup_channel(engine: Engine, channel: str, identities, chaincodes, committed_txids=()):
    """identities: iterable of (serialized, mspid, pubkey64 | None, valid, id_digest)."""
    engine.channel_init(channel)
    identities = list(identities)
    # all public keys first, in one fgv_keys_register call: their comb tables are then built by
    # batched k_keytab launches (up to KT_BUILD_KEYS keys each) instead of one launch per key,
    # and every msp_add_identity below finds its key cached (same slots, first-seen order)
    pubs = [pub for _ser, _mspid, pub, _valid, _dig in identities if pub is not None]
    if pubs:
        engine.keys_register(np.frombuffer(b"".join(bytes(p) for p in pubs), dtype=np.uint8))
    for ser, _mspid, pub, valid, dig in identities:
        engine.msp_add_identity(ser, pub, valid, dig)
    for ns, pol in chaincodes.items():
        engine.chaincode_define(ns, pol)
    if committed_txids:
        engine.ledger_add_txids(list(committed_txids))


class TxValidator:
    def __init__(self, engine: Engine):
        self.engine = engine

    def validate(self, block: bytes):
        return self.engine.validate_blocks([block])[0]

    def validate_many(self, blocks, d_blocks=None):
        return self.engine.validate_blocks(blocks, d_blocks)
