"""ctypes binding of libfgv.so (include/fgv.h).

The product path: every call goes to the HIP engine.  There is no CPU fallback here --
if the shared library or a GPU is missing, FgvError is raised (a Go shim would then use
its own sw BCCSP, which is the reference's behaviour, not ours).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfgv.so")

# status bytes (include/fgv.h)
SIG_VALID, SIG_FALSE, SIG_DER, SIG_HIGH_S, SIG_RANGE, SIG_BADKEY, SIG_EMPTY = range(7)

EXPORTED = [
    "fgv_init", "fgv_destroy", "fgv_strerror", "fgv_last_timing", "fgv_last_counts", "fgv_last_host_timing",
    "fgv_last_point_handovers", "fgv_last_kernel_times", "fgv_last_vb_timing",
    "fgv_sha256_batch",
    "fgv_p256_verify_batch", "fgv_p256_verify_msgs", "fgv_p384_verify_msgs", "fgv_keys_register", "fgv_keys_register_tiered", "fgv_keys_reset", "fgv_key_stats",
    "fgv_set_block_outcomes", "fgv_last_block_status", "fgv_unsupported_stats", "fgv_stats_sums",
    "fgv_p256_verify_msgs_dev", "fgv_channel_init", "fgv_msp_add_identity", "fgv_chaincode_define",
    "fgv_ledger_add_txids", "fgv_validate_blocks", "fgv_validate_shard", "fgv_finalize_flags",
    "fgv_validate_shard_dev", "fgv_finalize_flags_dev", "fgv_finalize_flags_dev_plan",
    "fgv_presplit", "fgv_prefetch", "fgv_last_presplit", "fgv_validate_shard_dev_next", "fgv_mvcc_validate_block_next",
    "fgv_statedb_init", "fgv_statedb_load", "fgv_statedb_apply", "fgv_statedb_stats", "fgv_mvcc_validate_block", "fgv_mvcc_validate_blocks", "fgv_mvcc_validate_blocks_next", "fgv_mvcc_last_stats",
    "fgv_blocks_verify", "fgv_sha256_host", "fgv_set_parse_mode", "fgv_commit_hash", "fgv_commit_hashes",
    "fgv_channel_config", "fgv_msp_declare", "fgv_msp_register_identity", "fgv_chaincode_define2",
    "fgv_collection_define", "fgv_host_alloc", "fgv_host_free", "fgv_last_h2d", "fgv_dev_alloc", "fgv_dev_upload",
    "fgv_dev_free", "fgv_stream_wait_external",
    "fgv_validate_shard_dev_pipelined", "fgv_last_ahead", "fgv_set_ahead", "fgv_blocks_verify_signed",
    "fgv_validate_blocks_pipelined", "fgv_set_timing",
    "fgv_group_init", "fgv_group_destroy", "fgv_group_size", "fgv_group_ctx", "fgv_group_validate_blocks",
    "fgv_group_set_block_outcomes", "fgv_group_last_block_status", "fgv_group_set_collective",
    "fgv_msp_resolve", "fgv_msp_resolve_blocks", "fgv_set_auto_resolve", "fgv_msp_identity",
    "fgv_kvmeta_set", "fgv_kvmeta_count", "fgv_kvmeta_get", "fgv_msp_identity_ous", "fgv_group_p256_verify_msgs",
    "fgv_mvcc_set_update_bytes", "fgv_mvcc_last_ticket", "fgv_mvcc_update_bytes_acquire",
    "fgv_mvcc_update_bytes_release", "fgv_commit_hashes_ub",
]
# fgv_msp_resolve status (include/fgv.h)
RESOLVE_KNOWN, RESOLVE_OK, RESOLVE_FAILED, RESOLVE_UNSUPPORTED, RESOLVE_REPEAT = range(5)
TX_RESULT_BYTES = 68
FGV_EUNSUPPORTED = -6
BLOCK_LATER = 1  # fgv_last_block_status: wait for the commit of the earlier blocks


class FgvError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class Unsupported(FgvError):
    """FGV_EUNSUPPORTED: the batch needs logic outside the engine's model."""


class ChainState(ctypes.Structure):
    """fgv_chain_state: the last verified block header (number + BlockHeaderHash)."""
    _fields_ = [("number", ctypes.c_uint64), ("header_hash", ctypes.c_uint8 * 32), ("valid", ctypes.c_uint8),
                ("has_hash", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 6)]


class BlockCheck(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("bad_tx", ctypes.c_uint32), ("number", ctypes.c_uint64),
                ("data_hash", ctypes.c_uint8 * 32), ("header_hash", ctypes.c_uint8 * 32)]


# fgv_block_check.status (include/fgv.h)
BLK_OK, BLK_UNPARSABLE, BLK_NO_HEADER, BLK_NUMBER, BLK_PREV_HASH, BLK_METADATA, BLK_EMPTY, BLK_TX_MALFORMED, \
    BLK_DATA_HASH, BLK_SIGNATURES, BLK_SIG_UNSUPPORTED = range(11)


KEY_TYPES = {"p256": 1, "p384": 2, "other": 3, "undeserializable": 4}
ROLES_UNKNOWN = 0x80000000
CC_COLLECTIONS_KNOWN, CC_KEY_LEVEL_EP = 1, 2


class IdentityInfo(ctypes.Structure):
    """fgv_identity_info (include/fgv.h)"""
    _fields_ = [("key_type", ctypes.c_uint32), ("hash_family", ctypes.c_uint32), ("valid", ctypes.c_uint32),
                ("roles", ctypes.c_uint32), ("pubkey", ctypes.c_uint8 * 64), ("id_digest", ctypes.c_uint8 * 32),
                ("pubkey_p384", ctypes.c_uint8 * 96)]


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("key_slots", ctypes.c_uint32),
                ("host_threads", ctypes.c_uint32), ("key_ids", ctypes.c_uint32)]


_L = None


def load():
    """Load libfgv.so (no GPU needed just to load and resolve symbols).

    torch (when installed) ships its own libamdhip64.so.7; libfgv.so links the same soname.
    Import torch first so the process holds ONE HIP runtime whichever module a caller
    touches first (a second copy makes torch report "No HIP GPUs are available")."""
    global _L
    if _L is None:
        if not os.environ.get("FGV_NO_TORCH"):  # (the torch-free harness: tools/bench_notorch.py)
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(LIB_PATH):
            raise FgvError(f"{LIB_PATH} not built -- run `make` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.fgv_init.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(vp)]
        L.fgv_destroy.argtypes = [vp]
        L.fgv_destroy.restype = None
        L.fgv_strerror.argtypes = [ctypes.c_int]
        L.fgv_strerror.restype = ctypes.c_char_p
        L.fgv_last_timing.argtypes = [vp] + [ctypes.POINTER(ctypes.c_double)] * 4
        L.fgv_last_vb_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.fgv_last_counts.argtypes = [vp] + [ctypes.POINTER(ctypes.c_uint64)] * 3
        L.fgv_last_point_handovers.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.fgv_last_kernel_times.argtypes = [vp, vp, sz]
        L.fgv_last_host_timing.argtypes = [vp] + [ctypes.POINTER(ctypes.c_double)] * 4
        L.fgv_sha256_batch.argtypes = [vp, vp, sz, vp, vp, sz, vp]
        L.fgv_p256_verify_batch.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, vp]
        L.fgv_p256_verify_msgs.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
        L.fgv_p384_verify_msgs.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
        L.fgv_keys_register.argtypes = [vp, vp, sz, vp]
        L.fgv_keys_register_tiered.argtypes = [vp, vp, sz, vp, vp]
        L.fgv_keys_reset.argtypes = [vp]
        L.fgv_key_stats.argtypes = [vp] + [ctypes.POINTER(ctypes.c_uint64)] * 5
        L.fgv_set_block_outcomes.argtypes = [vp, ctypes.c_int]
        L.fgv_stats_sums.argtypes = [vp, vp, sz, ctypes.c_int]
        L.fgv_last_block_status.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
        L.fgv_unsupported_stats.argtypes = [vp] + [ctypes.POINTER(ctypes.c_uint64)] * 3
        L.fgv_p256_verify_msgs_dev.argtypes = [vp] * 8 + [sz, vp]
        L.fgv_channel_init.argtypes = [vp, ctypes.c_char_p]
        L.fgv_msp_add_identity.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
        L.fgv_chaincode_define.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz]
        L.fgv_chaincode_define2.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_uint32]
        L.fgv_collection_define.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz]
        L.fgv_kvmeta_set.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        L.fgv_kvmeta_count.argtypes = [vp]
        L.fgv_kvmeta_count.restype = sz
        L.fgv_kvmeta_get.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz, vp, sz,
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.fgv_channel_config.argtypes = [vp, ctypes.c_char_p, sz]
        L.fgv_msp_declare.argtypes = [vp, ctypes.c_char_p]
        L.fgv_msp_register_identity.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(IdentityInfo)]
        L.fgv_group_p256_verify_msgs.argtypes = [vp, vp, vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
        L.fgv_msp_identity_ous.argtypes = [vp, ctypes.c_char_p, sz, sz, vp, vp, vp, vp]
        L.fgv_ledger_add_txids.argtypes = [vp, vp, vp, vp, sz]
        L.fgv_validate_blocks.argtypes = [vp, sz, vp, vp, vp, vp, sz, vp]
        L.fgv_validate_blocks_pipelined.argtypes = [vp, sz, vp, vp, vp, vp, sz, vp, sz, vp, vp, vp]
        L.fgv_validate_shard.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, sz, vp]
        L.fgv_finalize_flags.argtypes = [sz, vp, vp, vp]
        L.fgv_validate_shard_dev.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, sz, vp]
        L.fgv_finalize_flags_dev.argtypes = [vp, sz, vp, ctypes.c_uint32, sz, vp, vp]
        L.fgv_presplit.argtypes = [vp, sz, vp, vp, vp, vp]
        L.fgv_prefetch.argtypes = [vp, sz, vp, vp]
        L.fgv_validate_shard_dev_next.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, sz, vp, sz, vp, vp, vp, vp]
        L.fgv_last_presplit.argtypes = [vp]
        L.fgv_validate_shard_dev_pipelined.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, sz, vp, sz, vp, vp, vp, vp, vp]
        L.fgv_last_ahead.argtypes = [vp]
        L.fgv_set_ahead.argtypes = [vp, ctypes.c_int]
        L.fgv_set_timing.argtypes = [vp, ctypes.c_int]
        L.fgv_group_init.argtypes = [vp, sz, ctypes.POINTER(_Config), ctypes.POINTER(vp)]
        L.fgv_group_destroy.argtypes = [vp]
        L.fgv_group_destroy.restype = None
        L.fgv_group_size.argtypes = [vp]
        L.fgv_group_size.restype = sz
        L.fgv_group_ctx.argtypes = [vp, sz]
        L.fgv_group_ctx.restype = vp
        L.fgv_group_validate_blocks.argtypes = [vp, sz, vp, vp, vp, sz, vp]
        L.fgv_group_set_block_outcomes.argtypes = [vp, ctypes.c_int]
        L.fgv_group_set_collective.argtypes = [vp, ctypes.c_int]
        L.fgv_group_last_block_status.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
        L.fgv_finalize_flags_dev_plan.argtypes = [vp, sz, vp, ctypes.c_uint32, sz, vp, vp, vp, vp]
        L.fgv_statedb_init.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
        L.fgv_statedb_load.argtypes = [vp, ctypes.c_char_p, vp, vp, vp, vp, vp, sz]
        L.fgv_statedb_apply.argtypes = [vp, ctypes.c_char_p, vp, vp, vp, vp, vp, vp, sz]
        L.fgv_statedb_stats.argtypes = [vp] + [ctypes.POINTER(ctypes.c_uint64)] * 4
        L.fgv_mvcc_validate_block.argtypes = [vp, vp, sz, vp, ctypes.c_uint64, vp, sz, ctypes.c_int]
        L.fgv_mvcc_validate_block_next.argtypes = [vp, vp, sz, vp, ctypes.c_uint64, vp, sz, ctypes.c_int, vp, sz]
        L.fgv_mvcc_validate_blocks.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp]
        L.fgv_mvcc_validate_blocks_next.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp, sz, vp, vp]
        L.fgv_mvcc_last_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint32)]
        L.fgv_blocks_verify.argtypes = [vp, sz, vp, vp, vp, vp]
        L.fgv_blocks_verify_signed.argtypes = [vp, sz, vp, vp, vp, ctypes.c_char_p, ctypes.c_int, vp]
        L.fgv_set_parse_mode.argtypes = [vp, ctypes.c_int]
        L.fgv_sha256_host.argtypes = [vp, sz, vp]
        L.fgv_commit_hash.argtypes = [vp, sz, vp, sz, ctypes.c_uint64, vp, sz, vp]
        L.fgv_commit_hashes.argtypes = [sz, vp, vp, vp, vp, vp, vp, sz, vp, ctypes.c_uint]
        L.fgv_commit_hashes_ub.argtypes = [sz, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp, ctypes.c_uint]
        L.fgv_mvcc_set_update_bytes.argtypes = [vp, ctypes.c_int]
        L.fgv_mvcc_last_ticket.argtypes = [vp, vp]
        L.fgv_mvcc_update_bytes_acquire.argtypes = [vp, ctypes.c_uint64, sz, vp, vp]
        L.fgv_mvcc_update_bytes_release.argtypes = [vp, ctypes.c_uint64]
        L.fgv_host_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
        L.fgv_host_free.argtypes = [vp, vp]
        L.fgv_dev_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
        L.fgv_dev_upload.argtypes = [vp, vp, vp, sz]
        L.fgv_dev_free.argtypes = [vp, vp]
        L.fgv_stream_wait_external.argtypes = [vp, vp]
        L.fgv_last_h2d.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.fgv_msp_resolve.argtypes = [vp, sz, vp, vp, vp]
        L.fgv_msp_resolve_blocks.argtypes = [vp, sz, vp, vp, ctypes.POINTER(sz)]
        L.fgv_set_auto_resolve.argtypes = [vp, ctypes.c_int]
        L.fgv_msp_identity.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(IdentityInfo)]
        L.fgv_x509_probe.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz]
        _L = L
    return _L


def _check(rc):
    if rc == FGV_EUNSUPPORTED:
        raise Unsupported("libfgv: block outside the engine's model", rc)
    if rc != 0:
        raise FgvError(f"libfgv error {rc}: {load().fgv_strerror(rc).decode()}", rc)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


def pack(blobs):
    """List of bytes -> (arena uint8, offsets uint64, lengths uint32)."""
    lens = np.fromiter((len(b) for b in blobs), dtype=np.uint32, count=len(blobs))
    offs = np.zeros(len(blobs), dtype=np.uint64)
    if len(blobs) > 1:
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    arena = np.frombuffer(b"".join(blobs), dtype=np.uint8) if blobs else np.zeros(0, np.uint8)
    return np.ascontiguousarray(arena), offs, lens


class _BlockBatch:
    def __init__(self, blocks, d_blocks):
        """blocks: list of bytes / uint8 arrays (e.g. views into a PinnedBuffer)"""
        self.nb = len(blocks)
        self._bufs = [b if isinstance(b, np.ndarray) else np.frombuffer(b, dtype=np.uint8) for b in blocks]
        self.ptrs = (ctypes.c_void_p * self.nb)(*[b.ctypes.data for b in self._bufs])
        self.lens = (ctypes.c_size_t * self.nb)(*[b.size for b in self._bufs])
        self.dptr = (ctypes.c_void_p * self.nb)(*d_blocks) if d_blocks is not None else None
        self.ntx = (ctypes.c_size_t * self.nb)()


class MvccChainStep:
    """fgv_mvcc_validate_blocks[_next] over a fixed list of consecutive blocks with every ctypes
    argument bound once (the bench loop); run() restores the committer flags, makes the call and
    returns (flag arrays, rc, n_done).  Same C call as Engine.mvcc_validate_blocks."""

    def __init__(self, eng, blocks, block_nums, flags, commit=True, d_blocks=None, next_blocks=None):
        self._L, self._h = eng._L, eng._h
        n = len(blocks)
        self.n = n
        self._bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        self._flags0 = [np.array(f, dtype=np.uint8) for f in flags]
        self.flags = [f.copy() for f in self._flags0]
        self._bp = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in self._bufs])
        self._ln = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in blocks])
        self._nums = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in block_nums])
        self._fp = (ctypes.c_void_p * max(n, 1))(*[f.ctypes.data for f in self.flags])
        self._nt = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in self.flags])
        self._dp = None if d_blocks is None else (ctypes.c_void_p * max(n, 1))(*[d or None for d in d_blocks])
        self._commit = 1 if commit else 0
        self._done = ctypes.c_size_t(0)
        self._next = None
        if next_blocks:
            self._nbufs = [np.frombuffer(b, dtype=np.uint8) for b in next_blocks]
            self._next = (len(next_blocks), (ctypes.c_void_p * len(next_blocks))(*[b.ctypes.data for b in self._nbufs]),
                          (ctypes.c_size_t * len(next_blocks))(*[len(b) for b in next_blocks]))

    def set_flags(self, flags):
        """the committer flags the next run() starts from (one array per block)"""
        for f0, f in zip(self._flags0, flags):
            np.copyto(f0, f)

    def run(self):
        for f, f0 in zip(self.flags, self._flags0):
            np.copyto(f, f0)
        if self._next:
            rc = self._L.fgv_mvcc_validate_blocks_next(self._h, self.n, self._bp, self._ln, self._dp, self._nums,
                                                       self._fp, self._nt, self._commit, ctypes.byref(self._done),
                                                       *self._next)
        else:
            rc = self._L.fgv_mvcc_validate_blocks(self._h, self.n, self._bp, self._ln, self._dp, self._nums, self._fp,
                                                  self._nt, self._commit, ctypes.byref(self._done))
        return self.flags, rc, self._done.value


class BlockStep:
    """One committer pass over a resident batch with every ctypes argument bound once (the
    bench loop): fgv_validate_shard_dev -> [pre-split of the next batch] -> (caller's
    all-gather) -> fgv_finalize_flags_dev[_plan], plus the per-call diagnostics read into
    preallocated cells.  Same C calls as Engine.validate_shard_dev / presplit /
    finalize_flags_dev."""

    def __init__(self, eng, batch, tx_lo, tx_hi, d_send, rows, ntx, world, d_recv, flags_out, plan=None,
                 presplit=True, next_batch=None, fused=False):
        """fused (one GPU): fgv_validate_blocks_pipelined -- validation and finalize queued back to
        back, one synchronisation -- instead of the shard / all-gather / finalize protocol."""
        L, h = eng._L, eng._h
        self._L = L
        self._fused = None
        if fused:
            nb = next_batch or batch
            self._fused = (h, batch.nb, batch.ptrs, batch.lens, batch.dptr, flags_out.ctypes.data_as(ctypes.c_void_p),
                           flags_out.size, batch.ntx) + ((nb.nb, nb.ptrs, nb.lens, nb.dptr) if presplit else
                                                         (0, None, None, None))
        self._lo = np.ascontiguousarray(tx_lo, dtype=np.uint32)
        self._hi = np.ascontiguousarray(tx_hi, dtype=np.uint32)
        self._ntx = np.ascontiguousarray(ntx, dtype=np.uint64)
        self.flags = flags_out
        self._val = (h, batch.nb, batch.ptrs, batch.lens, batch.dptr, _ptr(self._lo), _ptr(self._hi),
                     ctypes.c_void_p(d_send), rows, batch.ntx)
        # presplit: the next batch (default: the same blocks) is split -- and, when host-resident,
        # copied to the device -- while this one's GPU work runs (fgv_validate_shard_dev_next)
        # (fgv_validate_shard_dev_pipelined: a device-resident next batch's front half is enqueued
        # ahead of its call)
        nb = next_batch or batch
        self._next = (nb.nb, nb.ptrs, nb.lens, nb.dptr, _ptr(self._lo), _ptr(self._hi)) if presplit else None
        if plan is None:
            self._fin_fn = L.fgv_finalize_flags_dev
            self._fin = (h, len(self._ntx), _ptr(self._ntx), world, rows, ctypes.c_void_p(d_recv), _ptr(flags_out))
        else:
            self._plo = np.ascontiguousarray(plan[0], dtype=np.uint32)
            self._phi = np.ascontiguousarray(plan[1], dtype=np.uint32)
            assert self._plo.shape == self._phi.shape == (world, len(self._ntx))
            self._fin_fn = L.fgv_finalize_flags_dev_plan
            self._fin = (h, len(self._ntx), _ptr(self._ntx), world, rows, _ptr(self._plo), _ptr(self._phi),
                         ctypes.c_void_p(d_recv), _ptr(flags_out))
        self._t = [ctypes.c_double() for _ in range(8)]
        self._c = [ctypes.c_uint64() for _ in range(3)]
        self._tr = (h,) + tuple(ctypes.byref(x) for x in self._t[:4])
        self._hr = (h,) + tuple(ctypes.byref(x) for x in self._t[4:])
        self._cr = (h,) + tuple(ctypes.byref(x) for x in self._c)

    def validate(self):
        if self._fused is not None:
            _check(self._L.fgv_validate_blocks_pipelined(*self._fused))
            return
        if self._next is None:
            _check(self._L.fgv_validate_shard_dev(*self._val))
        else:
            _check(self._L.fgv_validate_shard_dev_pipelined(*self._val, *self._next))

    def finalize(self):
        if self._fused is None:
            _check(self._fin_fn(*self._fin))
        return self.flags

    def stats(self):
        """(sha_ms, prep_ms, point_ms, keytab_ms, parse_ms, assemble_ms, device_ms, fold_ms),
        (sha_jobs, sha_blocks, verifies) of the last validation."""
        self._L.fgv_last_timing(*self._tr)
        self._L.fgv_last_host_timing(*self._hr)
        self._L.fgv_last_counts(*self._cr)
        return [x.value for x in self._t], [x.value for x in self._c]


class PinnedBuffer:
    """fgv_host_alloc'd page-locked bytes; .a is a uint8 numpy view, freed by close()."""

    def __init__(self, eng, nbytes):
        self._eng = eng
        p = ctypes.c_void_p()
        _check(eng._L.fgv_host_alloc(eng._h, nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.a = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.ptr))

    def close(self):
        if self.ptr and self._eng._h:
            self.a = None
            _check(self._eng._L.fgv_host_free(self._eng._h, ctypes.c_void_p(self.ptr)))
        self.ptr = None


class Group:
    """fgv_group: several GPUs driven from one process.  .engines[i] is device i's context
    (set each one up like an Engine: txvalidator.setup_channel(...) on every one)."""

    def __init__(self, devices, key_slots: int = 0, host_threads: int = 0, key_ids: int = 0):
        self._L = load()
        arr = (ctypes.c_int * len(devices))(*devices)
        cfg = _Config(devices[0], key_slots, host_threads, key_ids)
        h = ctypes.c_void_p()
        _check(self._L.fgv_group_init(arr, len(devices), ctypes.byref(cfg), ctypes.byref(h)))
        self._g = h
        self.engines = [Engine._borrow(self._L.fgv_group_ctx(h, i)) for i in range(self._L.fgv_group_size(h))]

    def validate_blocks(self, blocks):
        """fgv_group_validate_blocks: per-block flag arrays, as Engine.validate_blocks"""
        nb = len(blocks)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        ptrs = (ctypes.c_void_p * nb)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * nb)(*[len(b) for b in blocks])
        cap = sum(len(b) for b in blocks) // 16 + 1024
        flags = np.zeros(cap, dtype=np.uint8)
        ntx = (ctypes.c_size_t * nb)()
        _check(self._L.fgv_group_validate_blocks(self._g, nb, ptrs, lens, _ptr(flags), cap, ntx))
        out, o = [], 0
        for i in range(nb):
            out.append(flags[o:o + ntx[i]].copy())
            o += ntx[i]
        return out

    def set_block_outcomes(self, on=True):
        """fgv_group_set_block_outcomes: per-block results instead of a whole-batch Unsupported"""
        _check(self._L.fgv_group_set_block_outcomes(self._g, 1 if on else 0))

    COLL_PEER, COLL_RCCL = 0, 1

    def set_collective(self, mode):
        """fgv_group_set_collective: COLL_PEER (peer copies onto device 0) or COLL_RCCL (ncclAllGather
        of the records into every device + a finalize on each)"""
        _check(self._L.fgv_group_set_collective(self._g, mode))

    def last_block_status(self, nblocks):
        """fgv_group_last_block_status -> (per-block status list, n_final), as Engine.last_block_status"""
        st = np.zeros(nblocks, np.int32)
        nf = ctypes.c_size_t()
        _check(self._L.fgv_group_last_block_status(self._g, _ptr(st), nblocks, ctypes.byref(nf)))
        return st.tolist(), nf.value

    def verify_msgs(self, keys, msgs, sigs):
        """fgv_group_p256_verify_msgs: Engine.verify_msgs over the group's devices"""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        marena, moffs, mlens = pack(msgs) if isinstance(msgs, list) else msgs
        sarena, soffs, slens = pack(sigs) if isinstance(sigs, list) else sigs
        n = len(soffs)
        st = np.zeros(n, dtype=np.uint8)
        _check(self._L.fgv_group_p256_verify_msgs(self._g, _ptr(keys), _ptr(marena), marena.size, _ptr(moffs),
                                                  _ptr(mlens), _ptr(sarena), sarena.size, _ptr(soffs), _ptr(slens),
                                                  n, _ptr(st)))
        return st

    def close(self):
        if getattr(self, "_g", None):
            for e in self.engines:
                e._h = None
            self._L.fgv_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One libfgv context = one GPU (one process per GPU)."""

    def __init__(self, device: int = 0, key_slots: int = 0, host_threads: int = 0, key_ids: int = 0):
        """host_threads: fgv_config.host_threads (0 = the library default, 24); the
        FGV_HOST_THREADS environment variable sets it when the argument is 0.  key_slots: comb
        slots (0 = 2048); key_ids: distinct keys held at once (0 = 1M)"""
        self._L = load()
        host_threads = host_threads or int(os.environ.get("FGV_HOST_THREADS", "0"))
        cfg = _Config(device, key_slots, host_threads, key_ids)
        h = ctypes.c_void_p()
        _check(self._L.fgv_init(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._owned = True

    @classmethod
    def _borrow(cls, handle):
        """an Engine over a context owned by someone else (a Group's device context)"""
        e = cls.__new__(cls)
        e._L = load()
        e._h = ctypes.c_void_p(handle)
        e._owned = False
        return e

    def close(self):
        if getattr(self, "_h", None):
            if getattr(self, "_owned", True):
                self._L.fgv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def timing(self):
        v = [ctypes.c_double() for _ in range(4)]
        _check(self._L.fgv_last_timing(self._h, *[ctypes.byref(x) for x in v]))
        vb = ctypes.c_double()
        _check(self._L.fgv_last_vb_timing(self._h, ctypes.byref(vb)))
        return dict(zip(("sha_ms", "prep_ms", "point_ms", "keytab_ms", "vb_mul_ms"), [x.value for x in v] + [vb.value]))

    def host_timing(self):
        v = [ctypes.c_double() for _ in range(4)]
        _check(self._L.fgv_last_host_timing(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("parse_ms", "assemble_ms", "device_ms", "fold_ms"), (x.value for x in v)))

    def counts(self):
        v = [ctypes.c_uint64() for _ in range(3)]
        _check(self._L.fgv_last_counts(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("sha_jobs", "sha_blocks", "verifies"), (x.value for x in v)))

    def host_alloc(self, nbytes):
        """fgv_host_alloc: page-locked host memory as a PinnedBuffer (uint8 array in .a)"""
        return PinnedBuffer(self, nbytes)

    def dev_alloc(self, nbytes):
        """fgv_dev_alloc: HBM of the context's device (an int address); free with dev_free"""
        p = ctypes.c_void_p()
        _check(self._L.fgv_dev_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def dev_upload(self, dst, data: bytes, offset=0):
        """fgv_dev_upload: host bytes -> HBM at dst + offset (synchronous)"""
        buf = np.frombuffer(data, dtype=np.uint8)
        _check(self._L.fgv_dev_upload(self._h, dst + offset, buf.ctypes.data, buf.size))

    def wait_stream(self, stream_handle):
        """fgv_stream_wait_external: the engine's next work waits for `stream_handle` (a raw HIP
        stream, e.g. torch.cuda.current_stream().cuda_stream) -- no host synchronisation"""
        _check(self._L.fgv_stream_wait_external(self._h, ctypes.c_void_p(stream_handle)))

    def dev_free(self, p):
        _check(self._L.fgv_dev_free(self._h, p))

    def last_h2d(self):
        """fgv_last_h2d: (bytes the last call copied itself, blocks found prefetched)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.fgv_last_h2d(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    KERNELS = ("k_bd_sha_payload", "k_bd_parse", "k_bd_sha", "k_bd_ident+count", "k_bd_emit", "k_der+k_inv",
               "k_prep", "k_point28", "k_bd_fold", "batch")

    def kernel_times(self):
        """fgv_last_kernel_times: ({kernel: ms}, payload SHA-256 compressions)"""
        out = (ctypes.c_double * 11)()
        _check(self._L.fgv_last_kernel_times(self._h, out, 11))
        return dict(zip(self.KERNELS, out[:10])), int(out[10])

    def set_block_outcomes(self, on=True):
        """fgv_set_block_outcomes: per-block results instead of a whole-batch Unsupported"""
        _check(self._L.fgv_set_block_outcomes(self._h, 1 if on else 0))

    def last_block_status(self, nblocks):
        """fgv_last_block_status -> (per-block status list: 0 final, FGV_EUNSUPPORTED, BLOCK_LATER; n_final)"""
        st = np.zeros(nblocks, np.int32)
        nf = ctypes.c_size_t()
        _check(self._L.fgv_last_block_status(self._h, _ptr(st), nblocks, ctypes.byref(nf)))
        return st.tolist(), nf.value

    def unsupported_stats(self):
        v = [ctypes.c_uint64() for _ in range(3)]
        _check(self._L.fgv_unsupported_stats(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("batches", "blocks", "txs"), (x.value for x in v)))

    def stats_sums(self, reset=False):
        """fgv_stats_sums: running sums of the per-call diagnostics (include/fgv.h layout)"""
        out = (ctypes.c_double * 25)()
        _check(self._L.fgv_stats_sums(self._h, out, 25, 1 if reset else 0))
        v = list(out)
        return dict(calls=int(v[0]), kernel_ms=dict(zip(self.KERNELS, v[1:11])), front_ahead_ms=v[12],
                    pay_blocks=v[13], sha_blocks=v[14], verifies=v[15], sha_ms=v[16], prep_ms=v[17], point_ms=v[18],
                    parse_ms=v[19], assemble_ms=v[20], device_ms=v[21], fold_ms=v[22], gap_ms=v[23], finish_ms=v[24])

    def front_ahead_ms(self):
        """fgv_last_kernel_times out[11]: host ms spent enqueueing the next batch's front half"""
        out = (ctypes.c_double * 12)()
        _check(self._L.fgv_last_kernel_times(self._h, out, 12))
        return float(out[11])

    def point_handovers(self):
        v = ctypes.c_uint64()
        _check(self._L.fgv_last_point_handovers(self._h, ctypes.byref(v)))
        return v.value

    # --- BCCSP Hash
    def sha256_batch(self, msgs):
        arena, offs, lens = pack(msgs) if isinstance(msgs, list) else msgs
        n = len(offs)
        out = np.zeros((n, 32), dtype=np.uint8)
        _check(self._L.fgv_sha256_batch(self._h, _ptr(arena), arena.size, _ptr(offs), _ptr(lens), n,
                                        _ptr(out)))
        return out

    # --- BCCSP Verify (digest given)
    def verify_batch(self, keys, sigs, digests):
        """keys: (n,64) uint8 X||Y; sigs: list of DER bytes or packed triple; digests (n,32)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        digests = np.ascontiguousarray(digests, dtype=np.uint8)
        sarena, soffs, slens = pack(sigs) if isinstance(sigs, list) else sigs
        n = len(soffs)
        st = np.zeros(n, dtype=np.uint8)
        _check(self._L.fgv_p256_verify_batch(self._h, _ptr(keys), _ptr(sarena), sarena.size, _ptr(soffs),
                                             _ptr(slens), _ptr(digests), n, _ptr(st)))
        return st

    # --- identity.Verify(msg, sig), fused hash + verify
    def verify_msgs(self, keys, msgs, sigs):
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        marena, moffs, mlens = pack(msgs) if isinstance(msgs, list) else msgs
        sarena, soffs, slens = pack(sigs) if isinstance(sigs, list) else sigs
        n = len(soffs)
        st = np.zeros(n, dtype=np.uint8)
        _check(self._L.fgv_p256_verify_msgs(self._h, _ptr(keys), _ptr(marena), marena.size, _ptr(moffs),
                                            _ptr(mlens), _ptr(sarena), sarena.size, _ptr(soffs), _ptr(slens),
                                            n, _ptr(st)))
        return st

    def verify_msgs_p384(self, keys, msgs, sigs):
        """fgv_p384_verify_msgs: identity.Verify for P-384 keys (keys: n x 96 bytes X || Y)"""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        marena, moffs, mlens = pack(msgs) if isinstance(msgs, list) else msgs
        sarena, soffs, slens = pack(sigs) if isinstance(sigs, list) else sigs
        n = len(soffs)
        st = np.zeros(n, dtype=np.uint8)
        _check(self._L.fgv_p384_verify_msgs(self._h, _ptr(keys), _ptr(marena), marena.size, _ptr(moffs),
                                            _ptr(mlens), _ptr(sarena), sarena.size, _ptr(soffs), _ptr(slens),
                                            n, _ptr(st)))
        return st

    # --- key registry (MSP identity cache analogue)
    def keys_register(self, keys, hot=None):
        """hot: None (every key asks for a comb slot) or a per-key bool array (False: start on the
        variable-base kernels, fgv_keys_register_tiered)"""
        keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 64)
        slots = np.zeros(len(keys), dtype=np.uint32)
        if hot is None:
            _check(self._L.fgv_keys_register(self._h, _ptr(keys), len(keys), _ptr(slots)))
        else:
            h = np.ascontiguousarray(np.broadcast_to(np.asarray(hot, dtype=np.uint8), (len(keys),)))
            _check(self._L.fgv_keys_register_tiered(self._h, _ptr(keys), len(keys), _ptr(h), _ptr(slots)))
        return slots

    def keys_reset(self):
        _check(self._L.fgv_keys_reset(self._h))

    def key_stats(self):
        """fgv_key_stats: {ids, comb, vb, promoted, vb_verifies_last}"""
        v = [ctypes.c_uint64() for _ in range(5)]
        _check(self._L.fgv_key_stats(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("ids", "comb", "vb", "promoted", "vb_verifies_last"), (x.value for x in v)))

    # --- HBM-resident batch: arguments are device pointers (ints), e.g. tensor.data_ptr()
    def verify_msgs_dev(self, msg_buf, msg_off, msg_len, sig_buf, sig_off, sig_len, key_slot, n, status):
        _check(self._L.fgv_p256_verify_msgs_dev(self._h, msg_buf, msg_off, msg_len, sig_buf, sig_off, sig_len,
                                                key_slot, n, status))

    # --- committer: channel model + whole blocks
    def set_parse_mode(self, mode: int):
        """0: transactions parsed on the GPU (default); 1: host parser (same results)."""
        _check(self._L.fgv_set_parse_mode(self._h, mode))

    def channel_init(self, name: str):
        _check(self._L.fgv_channel_init(self._h, name.encode()))

    def msp_add_identity(self, serialized: bytes, pubkey64, valid: bool, id_digest: bytes):
        _check(self._L.fgv_msp_add_identity(self._h, serialized, len(serialized), pubkey64, 1 if valid else 0,
                                            id_digest))

    def chaincode_define(self, ns: str, policy: bytes, plugin: str = None, flags: int = 0):
        """fgv_chaincode_define (plugin None) / fgv_chaincode_define2"""
        if plugin is None and not flags:
            _check(self._L.fgv_chaincode_define(self._h, ns.encode(), policy, len(policy)))
        else:
            _check(self._L.fgv_chaincode_define2(self._h, ns.encode(), (plugin or "vscc").encode(), policy, len(policy),
                                                 flags))

    def collection_define(self, ns: str, coll: str, policy: bytes = b""):
        """fgv_collection_define: policy b"" = none (the chaincode EP applies)"""
        _check(self._L.fgv_collection_define(self._h, ns.encode(), coll.encode(), policy or None, len(policy or b"")))

    def kvmeta_set(self, ns: str, coll: str, key: bytes, vp: bytes = b""):
        """fgv_kvmeta_set: the committed VALIDATION_PARAMETER of (ns, coll, key) (coll "" = a
        public key, else the key hash); vp b"" removes it"""
        key = key.encode() if isinstance(key, str) else bytes(key)
        _check(self._L.fgv_kvmeta_set(self._h, ns.encode(), coll.encode(), key, len(key), vp or None, len(vp or b"")))

    def kvmeta_count(self) -> int:
        return int(self._L.fgv_kvmeta_count(self._h))

    def kvmeta_get(self, ns: str, coll: str, key: bytes):
        """the committed VALIDATION_PARAMETER the engine holds for (ns, coll, key), or None"""
        key = key.encode() if isinstance(key, str) else bytes(key)
        n = ctypes.c_size_t()
        _check(self._L.fgv_kvmeta_get(self._h, ns.encode(), coll.encode(), key, len(key), None, 0, ctypes.byref(n)))
        if n.value == 0:
            return None
        buf = ctypes.create_string_buffer(n.value)
        _check(self._L.fgv_kvmeta_get(self._h, ns.encode(), coll.encode(), key, len(key), buf, n.value,
                                      ctypes.byref(n)))
        return buf.raw[:n.value]

    def channel_config(self, config: bytes):
        """fgv_channel_config: the channel's common.Config bytes"""
        _check(self._L.fgv_channel_config(self._h, config, len(config)))

    def msp_declare(self, mspid: str):
        _check(self._L.fgv_msp_declare(self._h, mspid.encode()))

    def msp_register_identity(self, serialized: bytes, key: str, pub, valid: bool, id_digest: bytes, roles=None,
                              hash_family: str = "SHA2"):
        info = IdentityInfo()
        info.key_type = KEY_TYPES[key]
        info.hash_family = 1 if hash_family == "SHA3" else 0
        info.valid = 1 if valid else 0
        info.roles = ROLES_UNKNOWN if roles is None else int(roles)
        if pub is not None and key == "p384":
            if len(pub) == 96:  # (X || Y; anything else leaves the key unknown: outside the engine)
                ctypes.memmove(info.pubkey_p384, bytes(pub), 96)
        elif pub is not None:
            ctypes.memmove(info.pubkey, bytes(pub)[:64], min(64, len(pub)))
        ctypes.memmove(info.id_digest, bytes(id_digest), 32)
        _check(self._L.fgv_msp_register_identity(self._h, serialized, len(serialized), ctypes.byref(info)))

    def msp_identity_ous(self, serialized: bytes, ous):
        """fgv_msp_identity_ous: [(OrganizationalUnitIdentifier str, CertifiersIdentifier bytes)]"""
        n = len(ous)
        ob = [o.encode() for o, _ in ous]
        cb = [bytes(c) for _, c in ous]
        op = (ctypes.c_char_p * max(n, 1))(*ob)
        ol = (ctypes.c_size_t * max(n, 1))(*[len(o) for o in ob])
        cp = (ctypes.c_char_p * max(n, 1))(*cb)
        cl = (ctypes.c_size_t * max(n, 1))(*[len(c) for c in cb])
        _check(self._L.fgv_msp_identity_ous(self._h, serialized, len(serialized), n, op, ol, cp, cl))

    def msp_resolve(self, serialized):
        """fgv_msp_resolve: the MSP cache miss for a list of SerializedIdentity bytes ->
        list of RESOLVE_* statuses"""
        n = len(serialized)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in serialized]
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * n)(*[len(b) for b in serialized])
        st = (ctypes.c_int * n)()
        _check(self._L.fgv_msp_resolve(self._h, n, ptrs, lens, st))
        return list(st)

    def msp_resolve_blocks(self, blocks):
        """fgv_msp_resolve_blocks: the batch's unregistered creators / endorsers resolved ->
        the number registered"""
        nb = len(blocks)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        ptrs = (ctypes.c_void_p * nb)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * nb)(*[len(b) for b in blocks])
        reg = ctypes.c_size_t()
        _check(self._L.fgv_msp_resolve_blocks(self._h, nb, ptrs, lens, ctypes.byref(reg)))
        return reg.value

    def set_auto_resolve(self, on: bool):
        _check(self._L.fgv_set_auto_resolve(self._h, 1 if on else 0))

    def msp_identity(self, serialized: bytes):
        """fgv_msp_identity: the registry's record (dict) or None"""
        info = IdentityInfo()
        rc = self._L.fgv_msp_identity(self._h, serialized, len(serialized), ctypes.byref(info))
        if rc != 0:
            return None
        return dict(key=info.key_type, hash_family=info.hash_family, valid=bool(info.valid), roles=info.roles,
                    pub=bytes(info.pubkey_p384) if info.key_type == KEY_TYPES["p384"] else bytes(info.pubkey),
                    id_digest=bytes(info.id_digest))

    def ledger_add_txids(self, txids):
        arena, offs, lens = pack([t.encode() for t in txids])
        _check(self._L.fgv_ledger_add_txids(self._h, _ptr(arena), _ptr(offs), _ptr(lens), len(txids)))

    def validate_blocks(self, blocks, d_blocks=None):
        """blocks: list of bytes (host).  d_blocks: optional list of device addresses (ints).
        Returns a list of numpy uint8 flag arrays (TxValidationFlags), one per block."""
        nb = len(blocks)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        ptrs = (ctypes.c_void_p * nb)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * nb)(*[len(b) for b in blocks])
        dptr = (ctypes.c_void_p * nb)(*d_blocks) if d_blocks is not None else None
        cap = sum(len(b) for b in blocks) // 16 + 1024  # >= one byte per envelope
        flags = np.zeros(cap, dtype=np.uint8)
        ntx = (ctypes.c_size_t * nb)()
        _check(self._L.fgv_validate_blocks(self._h, nb, ptrs, lens, dptr, _ptr(flags), cap, ntx))
        out, o = [], 0
        for i in range(nb):
            out.append(flags[o:o + ntx[i]].copy())
            o += ntx[i]
        return out

    def validate_shard(self, blocks, tx_lo, tx_hi, d_blocks=None):
        """Validate transactions [tx_lo[b], tx_hi[b]) of each block.  Returns (results uint8
        array of shape (n, 68) = fgv_tx_result records, ntx per block)."""
        nb = len(blocks)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        ptrs = (ctypes.c_void_p * nb)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * nb)(*[len(b) for b in blocks])
        dptr = (ctypes.c_void_p * nb)(*d_blocks) if d_blocks is not None else None
        lo = np.ascontiguousarray(tx_lo, dtype=np.uint32)
        hi = np.ascontiguousarray(tx_hi, dtype=np.uint32)
        cap = int(np.maximum(hi.astype(np.int64) - lo, 0).sum())
        res = np.zeros((max(cap, 1), TX_RESULT_BYTES), dtype=np.uint8)
        ntx = (ctypes.c_size_t * nb)()
        _check(self._L.fgv_validate_shard(self._h, nb, ptrs, lens, dptr, _ptr(lo), _ptr(hi), _ptr(res), cap, ntx))
        return res[:cap], np.array(list(ntx), dtype=np.uint64)


    def validate_blocks_pipelined(self, batch, next_batch=None):
        """fgv_validate_blocks_pipelined over block_batch()es: validate `batch` (flags of every
        block, concatenated) while `next_batch` is pre-split (and, both host-resident, copied)."""
        cap = int(sum(batch.lens))
        flags = np.zeros(cap, dtype=np.uint8)
        nb = next_batch
        _check(self._L.fgv_validate_blocks_pipelined(self._h, batch.nb, batch.ptrs, batch.lens, batch.dptr,
                                                     _ptr(flags), cap, batch.ntx, nb.nb if nb else 0,
                                                     nb.ptrs if nb else None, nb.lens if nb else None,
                                                     nb.dptr if nb else None))
        return flags[:int(sum(batch.ntx))].copy()

    def block_batch(self, blocks, d_blocks=None):
        """Pre-packed ctypes arguments for a batch validated repeatedly (bench loop)."""
        return _BlockBatch(blocks, d_blocks)

    def validate_shard_dev(self, batch, tx_lo, tx_hi, d_results, cap):
        """fgv_validate_shard_dev: records (68 B each) written to device address d_results.
        batch: block_batch(...) or a list of blocks.  Returns ntx per block (uint64)."""
        if not isinstance(batch, _BlockBatch):
            batch = _BlockBatch(batch, None)
        lo = np.ascontiguousarray(tx_lo, dtype=np.uint32)
        hi = np.ascontiguousarray(tx_hi, dtype=np.uint32)
        _check(self._L.fgv_validate_shard_dev(self._h, batch.nb, batch.ptrs, batch.lens, batch.dptr, _ptr(lo),
                                              _ptr(hi), ctypes.c_void_p(d_results), cap, batch.ntx))
        return np.ctypeslib.as_array(batch.ntx).astype(np.uint64)

    def prefetch(self, batch):
        """fgv_prefetch: queue the H2D copy of a later host-resident batch (block_batch(...) of
        pinned blocks) on the engine's copy stream now; its validation call uses the staged copy."""
        assert isinstance(batch, _BlockBatch)
        _check(self._L.fgv_prefetch(self._h, batch.nb, batch.ptrs, batch.lens))

    def presplit(self, batch, tx_lo=None, tx_hi=None):
        """fgv_presplit: walk the batch's block framing on a background host thread for the
        next validate_shard_dev of the same batch (block_batch(...) keeps the buffers alive)."""
        assert isinstance(batch, _BlockBatch)
        lo = None if tx_lo is None else np.ascontiguousarray(tx_lo, dtype=np.uint32)
        hi = None if tx_hi is None else np.ascontiguousarray(tx_hi, dtype=np.uint32)
        _check(self._L.fgv_presplit(self._h, batch.nb, batch.ptrs, batch.lens, None if lo is None else _ptr(lo),
                                    None if hi is None else _ptr(hi)))

    def validate_shard_dev_next(self, batch, tx_lo, tx_hi, d_results, cap, next_batch, next_lo=None, next_hi=None):
        """fgv_validate_shard_dev_next: validate `batch`, pre-splitting `next_batch` while the
        GPU works.  Returns ntx per block of `batch`."""
        lo = np.ascontiguousarray(tx_lo, dtype=np.uint32)
        hi = np.ascontiguousarray(tx_hi, dtype=np.uint32)
        nlo = None if next_lo is None else np.ascontiguousarray(next_lo, dtype=np.uint32)
        nhi = None if next_hi is None else np.ascontiguousarray(next_hi, dtype=np.uint32)
        _check(self._L.fgv_validate_shard_dev_next(self._h, batch.nb, batch.ptrs, batch.lens, batch.dptr, _ptr(lo),
                                                   _ptr(hi), ctypes.c_void_p(d_results), cap, batch.ntx,
                                                   next_batch.nb, next_batch.ptrs, next_batch.lens, _ptr(nlo),
                                                   _ptr(nhi)))
        return np.ctypeslib.as_array(batch.ntx).astype(np.uint64)

    def last_presplit(self):
        return bool(self._L.fgv_last_presplit(self._h))

    def last_ahead(self):
        return bool(self._L.fgv_last_ahead(self._h))

    def set_timing(self, on: bool):
        """fgv_set_timing: per-kernel device times of the block committer (timestamp events)"""
        _check(self._L.fgv_set_timing(self._h, 1 if on else 0))

    def set_ahead(self, mode: int):
        """fgv_set_ahead: 0 off (default), 1 after ECDSA, 2 at once, 3 after the fold"""
        _check(self._L.fgv_set_ahead(self._h, mode))

    def validate_shard_dev_pipelined(self, batch, tx_lo, tx_hi, d_results, cap, next_batch, next_lo=None,
                                     next_hi=None):
        """fgv_validate_shard_dev_pipelined: validate `batch` and enqueue `next_batch`'s front half
        (its device copy: next_batch.dptr, or the copy stream's) ahead of its call."""
        lo = np.ascontiguousarray(tx_lo, dtype=np.uint32)
        hi = np.ascontiguousarray(tx_hi, dtype=np.uint32)
        nlo = None if next_lo is None else np.ascontiguousarray(next_lo, dtype=np.uint32)
        nhi = None if next_hi is None else np.ascontiguousarray(next_hi, dtype=np.uint32)
        _check(self._L.fgv_validate_shard_dev_pipelined(self._h, batch.nb, batch.ptrs, batch.lens, batch.dptr,
                                                        _ptr(lo), _ptr(hi), ctypes.c_void_p(d_results), cap,
                                                        batch.ntx, next_batch.nb, next_batch.ptrs, next_batch.lens,
                                                        next_batch.dptr, _ptr(nlo), _ptr(nhi)))
        return np.ctypeslib.as_array(batch.ntx).astype(np.uint64)

    def finalize_flags_dev(self, ntx, world, rows_per_rank, d_gathered, out=None, plan=None):
        """fgv_finalize_flags_dev over world x rows_per_rank gathered records at d_gathered;
        plan = (lo, hi) [world, nblocks] arrays of fabric_amd.shard.plan (default: the per-block
        transaction split)."""
        ntx = np.ascontiguousarray(ntx, dtype=np.uint64)
        flags = out if out is not None else np.empty(int(ntx.sum()), dtype=np.uint8)
        if plan is None:
            _check(self._L.fgv_finalize_flags_dev(self._h, len(ntx), _ptr(ntx), world, rows_per_rank,
                                                  ctypes.c_void_p(d_gathered), _ptr(flags)))
        else:
            lo = np.ascontiguousarray(plan[0], dtype=np.uint32)
            hi = np.ascontiguousarray(plan[1], dtype=np.uint32)
            assert lo.shape == hi.shape == (world, len(ntx))
            _check(self._L.fgv_finalize_flags_dev_plan(self._h, len(ntx), _ptr(ntx), world, rows_per_rank, _ptr(lo),
                                                       _ptr(hi), ctypes.c_void_p(d_gathered), _ptr(flags)))
        return flags

    # --- deliver-side block integrity (VerifyBlock; _signed: with the orderer signatures)
    def blocks_verify(self, blocks, chain=None):
        return blocks_verify(blocks, chain, ctx=self._h)

    def blocks_verify_signed(self, blocks, chain=None, policy=None, bft=False):
        """fgv_blocks_verify_signed -> (per-block tuples as blocks_verify, unsupported): when
        `unsupported`, the blocks from the first BLK_SIG_UNSUPPORTED on were not decided."""
        pol = policy.encode() if policy is not None else None
        rc, out = _verify_call(lambda *a: self._L.fgv_blocks_verify_signed(self._h, *a[:4], pol, 1 if bft else 0,
                                                                            a[4]), blocks, chain)
        if rc != FGV_EUNSUPPORTED:
            _check(rc)
        return out, rc == FGV_EUNSUPPORTED

    # --- MVCC
    def statedb_init(self, slots=1 << 22, arena_bytes=64 << 20):
        _check(self._L.fgv_statedb_init(self._h, slots, arena_bytes))

    def statedb_load(self, ns, keys, blk, txn):
        arena, offs, lens = pack([k.encode() if isinstance(k, str) else k for k in keys])
        blk = np.ascontiguousarray(blk, dtype=np.uint64)
        txn = np.ascontiguousarray(txn, dtype=np.uint64)
        _check(self._L.fgv_statedb_load(self._h, ns.encode(), _ptr(arena), _ptr(offs), _ptr(lens), _ptr(blk),
                                        _ptr(txn), len(keys)))

    def statedb_apply(self, ns, keys, blk, txn, is_delete):
        """fgv_statedb_apply: a block's update batch for namespace `ns` committed outside the
        engine (puts at their version, deletes)."""
        arena, offs, lens = pack([k.encode() if isinstance(k, str) else k for k in keys])
        blk = np.ascontiguousarray(blk, dtype=np.uint64)
        txn = np.ascontiguousarray(txn, dtype=np.uint64)
        dl = np.ascontiguousarray(is_delete, dtype=np.uint8)
        _check(self._L.fgv_statedb_apply(self._h, ns.encode(), _ptr(arena), _ptr(offs), _ptr(lens), _ptr(blk),
                                         _ptr(txn), _ptr(dl), len(keys)))

    def statedb_stats(self):
        v = [ctypes.c_uint64() for _ in range(4)]
        _check(self._L.fgv_statedb_stats(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("keys", "arena_used", "slots", "arena_cap"), (x.value for x in v)))

    def mvcc_validate(self, block: bytes, block_num: int, flags, commit=True, d_block=None, next_block=None):
        """flags: committer TxValidationFlags (updated copy returned).  next_block: bytes of the
        block validated next (its framing is walked meanwhile; keep the object alive)."""
        f = np.array(flags, dtype=np.uint8)
        buf = np.frombuffer(block, dtype=np.uint8)
        if next_block is None:
            _check(self._L.fgv_mvcc_validate_block(self._h, buf.ctypes.data, len(block), d_block, block_num, _ptr(f),
                                                   len(f), 1 if commit else 0))
        else:
            nb = np.frombuffer(next_block, dtype=np.uint8)
            _check(self._L.fgv_mvcc_validate_block_next(self._h, buf.ctypes.data, len(block), d_block, block_num,
                                                        _ptr(f), len(f), 1 if commit else 0, nb.ctypes.data,
                                                        len(next_block)))
        return f

    def mvcc_set_update_bytes(self, on=True):
        """fgv_mvcc_set_update_bytes: committing MVCC calls also build each block's update-batch
        bytes on the device (mvcc_ub.hip); fetch them with mvcc_update_bytes / commit_hashes_dev."""
        _check(self._L.fgv_mvcc_set_update_bytes(self._h, 1 if on else 0))

    def mvcc_last_ticket(self):
        t = ctypes.c_uint64(0)
        _check(self._L.fgv_mvcc_last_ticket(self._h, ctypes.byref(t)))
        return t.value

    def mvcc_update_bytes(self, ticket, n):
        """copies of the device-built update-batch bytes of the call `ticket` (None where a block's
        were not produced on the device)"""
        ptrs = (ctypes.c_void_p * max(n, 1))()
        lens = (ctypes.c_size_t * max(n, 1))()
        _check(self._L.fgv_mvcc_update_bytes_acquire(self._h, ticket, n, ptrs, lens))
        try:
            return [ctypes.string_at(ptrs[b], lens[b]) if ptrs[b] else None for b in range(n)]
        finally:
            self._L.fgv_mvcc_update_bytes_release(self._h, ticket)

    def mvcc_validate_blocks(self, blocks, block_nums, flags, commit=True, d_blocks=None, next_blocks=None):
        """fgv_mvcc_validate_blocks: consecutive blocks validated (and committed) in order as one
        device chain.  flags: one committer TxValidationFlags array per block.  next_blocks: the
        blocks of the next call (their framing is walked meanwhile; keep the objects alive).
        Returns (list of updated flag arrays, rc, n_done) -- rc != 0 is the error of block n_done."""
        n = len(blocks)
        bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        fl = [np.array(f, dtype=np.uint8) for f in flags]
        bp = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in bufs])
        ln = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in blocks])
        nums = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in block_nums])
        fp = (ctypes.c_void_p * max(n, 1))(*[f.ctypes.data for f in fl])
        nt = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in fl])
        dp = None if d_blocks is None else (ctypes.c_void_p * max(n, 1))(*[d or None for d in d_blocks])
        done = ctypes.c_size_t(0)
        if next_blocks:
            nbufs = [np.frombuffer(b, dtype=np.uint8) for b in next_blocks]
            nbp = (ctypes.c_void_p * len(nbufs))(*[b.ctypes.data for b in nbufs])
            nln = (ctypes.c_size_t * len(nbufs))(*[len(b) for b in next_blocks])
            rc = self._L.fgv_mvcc_validate_blocks_next(self._h, n, bp, ln, dp, nums, fp, nt, 1 if commit else 0,
                                                       ctypes.byref(done), len(nbufs), nbp, nln)
        else:
            rc = self._L.fgv_mvcc_validate_blocks(self._h, n, bp, ln, dp, nums, fp, nt, 1 if commit else 0,
                                                  ctypes.byref(done))
        return fl, rc, done.value

    def mvcc_stats(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        r, w = ctypes.c_uint64(), ctypes.c_uint64()
        rounds = ctypes.c_uint32()
        _check(self._L.fgv_mvcc_last_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(r), ctypes.byref(w),
                                           ctypes.byref(rounds)))
        return dict(lookup_ms=a.value, total_ms=b.value, reads=r.value, writes=w.value, rounds=rounds.value)


def finalize_flags(ntx, results):
    """fgv_finalize_flags over the results of ALL transactions (blocks concatenated)."""
    L = load()
    ntx = np.ascontiguousarray(ntx, dtype=np.uint64)
    results = np.ascontiguousarray(results, dtype=np.uint8)
    flags = np.zeros(int(ntx.sum()), dtype=np.uint8)
    _check(L.fgv_finalize_flags(len(ntx), _ptr(ntx), _ptr(results), _ptr(flags)))
    return flags


def blocks_verify(blocks, chain=None, ctx=None):
    """fgv_blocks_verify: per-block (status, bad_tx, number, data_hash, header_hash); `chain`
    (ChainState) is advanced past every verified block.  ctx None -> one host thread."""
    L = load()
    rc, out = _verify_call(lambda *a: L.fgv_blocks_verify(ctx, *a), blocks, chain)
    _check(rc)
    return out


def _verify_call(fn, blocks, chain, *extra):
    nb = len(blocks)
    bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
    ptrs = (ctypes.c_void_p * nb)(*[b.ctypes.data for b in bufs])
    lens = (ctypes.c_size_t * nb)(*[len(b) for b in blocks])
    out = (BlockCheck * nb)()
    rc = fn(nb, ptrs, lens, ctypes.byref(chain) if chain is not None else None, *extra, out)
    return rc, [(o.status, o.bad_tx, o.number, bytes(o.data_hash), bytes(o.header_hash)) for o in out]


def sha256_host(buf: bytes):
    """Host SHA-256 (the data-hash primitive).  Returns (digest, used_sha_extensions)."""
    L = load()
    out = ctypes.create_string_buffer(32)
    b = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, np.uint8)
    ni = L.fgv_sha256_host(b.ctypes.data, len(buf), out)
    return out.raw, bool(ni)


def commit_hash(block: bytes, flags, block_num: int, prev: bytes = b""):
    """fgv_commit_hash: the ledger commit hash of a block (kv_ledger.go:806-817)."""
    L = load()
    f = np.ascontiguousarray(flags, dtype=np.uint8)
    b = np.frombuffer(block, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    pv = np.frombuffer(prev, dtype=np.uint8) if prev else None
    _check(L.fgv_commit_hash(b.ctypes.data, len(block), _ptr(f), len(f), block_num,
                             pv.ctypes.data if pv is not None else None, len(prev), out))
    return out.raw


class CommitHashes:
    """fgv_commit_hashes over a fixed list of consecutive blocks with the ctypes arguments bound
    once (the pipeline bench): run(flags, prev) -> n x 32-byte commit hashes (bytes)."""

    def __init__(self, blocks, block_nums, threads=0):
        self._L = load()
        n = self.n = len(blocks)
        self._bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
        self._bp = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in self._bufs])
        self._ln = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in blocks])
        self._nums = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in block_nums])
        self._threads = threads
        self.out = ctypes.create_string_buffer(32 * max(n, 1))

    def run(self, flags, prev=b""):
        fl = [np.ascontiguousarray(f, dtype=np.uint8) for f in flags]
        fp = (ctypes.c_void_p * max(self.n, 1))(*[f.ctypes.data for f in fl])
        nt = (ctypes.c_size_t * max(self.n, 1))(*[len(f) for f in fl])
        pv = ctypes.create_string_buffer(prev, len(prev)) if prev else None
        _check(self._L.fgv_commit_hashes(self.n, self._bp, self._ln, fp, nt, self._nums, pv, len(prev), self.out,
                                         self._threads))
        return [self.out.raw[32 * b:32 * b + 32] for b in range(self.n)]


class CommitHashesDev(CommitHashes):
    """fgv_commit_hashes_ub with the device-built update-batch bytes of an MVCC call (its ticket):
    acquire -> hash -> release; a block without device bytes is decoded on the host."""

    def __init__(self, eng, blocks, block_nums, threads=0):
        super().__init__(blocks, block_nums, threads)
        self._eng = eng
        self._ub = (ctypes.c_void_p * max(self.n, 1))()
        self._ubl = (ctypes.c_size_t * max(self.n, 1))()

    def run(self, flags, prev=b"", ticket=0):
        fl = [np.ascontiguousarray(f, dtype=np.uint8) for f in flags]
        fp = (ctypes.c_void_p * max(self.n, 1))(*[f.ctypes.data for f in fl])
        nt = (ctypes.c_size_t * max(self.n, 1))(*[len(f) for f in fl])
        pv = ctypes.create_string_buffer(prev, len(prev)) if prev else None
        h = self._eng._h
        got = ticket and self._L.fgv_mvcc_update_bytes_acquire(h, ticket, self.n, self._ub, self._ubl) == 0
        try:
            _check(self._L.fgv_commit_hashes_ub(self.n, self._ub if got else None, self._ubl if got else None,
                                                self._bp, self._ln, fp, nt, self._nums, pv, len(prev), self.out,
                                                self._threads))
        finally:
            if got:
                self._L.fgv_mvcc_update_bytes_release(h, ticket)
        return [self.out.raw[32 * b:32 * b + 32] for b in range(self.n)]


def commit_hashes_ub(ub, blocks, flags, block_nums, prev: bytes = b"", threads=0):
    """fgv_commit_hashes_ub with the update-batch bytes given per block (None: decode the block)"""
    L = load()
    n = len(flags)
    ubb = [None if u is None else np.frombuffer(u, dtype=np.uint8) if len(u) else np.zeros(1, np.uint8) for u in ub]
    up = (ctypes.c_void_p * max(n, 1))(*[None if u is None else u.ctypes.data for u in ubb])
    ul = (ctypes.c_size_t * max(n, 1))(*[0 if u is None else len(u) for u in ub])
    bufs = [np.frombuffer(b, dtype=np.uint8) for b in blocks]
    bp = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in bufs])
    ln = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in blocks])
    nums = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in block_nums])
    fl = [np.ascontiguousarray(f, dtype=np.uint8) for f in flags]
    fp = (ctypes.c_void_p * max(n, 1))(*[f.ctypes.data for f in fl])
    nt = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in fl])
    pv = ctypes.create_string_buffer(prev, len(prev)) if prev else None
    out = ctypes.create_string_buffer(32 * max(n, 1))
    _check(L.fgv_commit_hashes_ub(n, up, ul, bp, ln, fp, nt, nums, pv, len(prev), out, threads))
    return [out.raw[32 * b:32 * b + 32] for b in range(n)]


def commit_hashes(blocks, flags, block_nums, prev: bytes = b"", threads=0):
    """fgv_commit_hashes: the chained commit hashes of consecutive blocks (kv_ledger.go:806-817)."""
    return CommitHashes(blocks, block_nums, threads).run(flags, prev)


def x509_probe(pem: bytes):
    """fgv_x509_probe (CPU, no GPU): the engine's PEM -> X.509 parse -> sanitizeCert of one
    certificate, as a dict (the parity tests compare it with oracle/x509.py)"""
    import json
    L = load()
    out = ctypes.create_string_buffer(1 << 16)
    n = L.fgv_x509_probe(pem, len(pem), out, len(out))
    if n < 0:
        raise FgvError("x509 probe output too large")
    return json.loads(out.raw[:n].decode())
