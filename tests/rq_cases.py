"""Range-query (phantom read) cases shared by the oracle tests and the GPU parity tests.

Known answers restate core/ledger/kvledger/txmgmt/validation/validator_test.go:240-345
(TestPhantomValidation, TestPhantomHashBasedValidation), rangequery_validator_test.go:20-55
(TestRangeQueryBoundaryConditions) and combined_iterator_test.go:17-83 as blocks validated
against a state DB; random_blocks() builds randomized blocks for engine-vs-oracle parity.
"""
import random

from fabric_amd.synth import blocks as B
from fabric_amd.synth import mvcc as M
from oracle.rangequery import ResultsHelper


def env(ns_sets, i=0, number=1):
    return M._envelope(B.tx_rwset(ns_sets), i, number)


def tx(reads=(), writes=(), rqs=(), ns="ns1"):
    return env([(ns, B.kv_rwset(reads, writes, rqs))])


def rqi(start, end, exhausted, raw=None, merkle=None):
    return B.range_query_info(start, end, exhausted, raw=raw, merkle=merkle)


def merkle_of(max_degree, kvs):
    """buildTestHashResults: RangeQueryResultsHelper(true, max_degree) over the results, Done()"""
    h = ResultsHelper(max_degree)
    for k, v in kvs:
        h.add((k.encode(), v))
    return h.done()


def _kv(i, v=None):
    return ("key%d" % i, v)


def phantom_db():
    """TestPhantomValidation: ns1 key1..key5 at Height{1, 0..4}"""
    return {("ns1", "key%d" % i): (1, i - 1) for i in range(1, 6)}


def hash_db():
    """TestPhantomHashBasedValidation: ns1 key1..key9 at Height{1, 0..8}"""
    return {("ns1", "key%d" % i): (1, i - 1) for i in range(1, 10)}


def known_answer_cases():
    """-> [(name, db, [envelopes], expected codes)]"""
    cases = []
    pdb = phantom_db()
    cases.append(("phantom_valid", pdb, [tx(rqs=[rqi("key2", "key4", True, raw=[("key2", (1, 1)), ("key3", (1, 2))])])], [0]))
    cases.append(("phantom_endkey_version", pdb, [tx(rqs=[rqi("key2", "key4", False, raw=[
        ("key2", (1, 1)), ("key3", (1, 2)), ("key4", (1, 2))])])], [12]))
    cases.append(("phantom_missing_key3", pdb, [tx(rqs=[rqi("key2", "key4", False, raw=[
        ("key2", (1, 1)), ("key4", (1, 3))])])], [12]))
    full = [("key2", (1, 1)), ("key3", (1, 2)), ("key4", (1, 3))]
    cases.append(("phantom_intrablock_delete", pdb, [tx(writes=[("key3", b"", False)]),
                                                     tx(rqs=[rqi("key2", "key4", False, raw=full)])], [0, 12]))
    cases.append(("phantom_intrablock_insert", pdb, [tx(writes=[("key2_1", b"value2_1", False)]),
                                                     tx(rqs=[rqi("key2", "key4", False, raw=full)])], [0, 12]))
    cases.append(("phantom_full_valid_after_unrelated_write", pdb, [tx(writes=[("key9", b"x", False)]),
                                                                    tx(rqs=[rqi("key2", "key4", False, raw=full)])], [0, 0]))
    hdb = hash_db()
    sim1 = [("key%d" % i, (1, i - 1)) for i in range(2, 9)]
    cases.append(("hash_valid", hdb, [tx(rqs=[rqi("key2", "key9", True, merkle=merkle_of(2, sim1))])], [0]))
    sim2 = [("key1", (1, 0)), ("key2", (1, 1)), ("key3", (1, 1))] + [("key%d" % i, (1, i - 1)) for i in range(4, 10)]
    cases.append(("hash_wrong_version", hdb, [tx(rqs=[rqi("key1", "key9", False, merkle=merkle_of(2, sim2))])], [12]))
    sim3 = [("key%d" % i, (1, i - 1)) for i in range(1, 10)]
    cases.append(("hash_full_valid", hdb, [tx(rqs=[rqi("key1", "key9", False, merkle=merkle_of(2, sim3))])], [0]))
    cases.append(("hash_degree3_valid", hdb, [tx(rqs=[rqi("", "", True, merkle=merkle_of(3, sim3))])], [0]))
    cases.append(("hash_small_summary_never_equal", hdb, [tx(rqs=[rqi("key1", "key3", True, merkle=(2, 1, [b"x"]))])], [12]))
    # TestRangeQueryBoundaryConditions (db key1..key5 at Height{1, 0..4})
    cases.append(("boundary_no_results", pdb, [tx(rqs=[rqi("key7", "key10", True, raw=[])])], [0]))
    cases.append(("boundary_no_results_during_validation", pdb,
                  [tx(rqs=[rqi("key7", "key10", True, raw=[("key8", (1, 8))])])], [12]))
    cases.append(("boundary_one_extra_tail", pdb, [tx(rqs=[rqi("key1", "key4", True, raw=[
        ("key1", (1, 0)), ("key2", (1, 1))])])], [12]))
    cases.append(("boundary_two_extra_tail", pdb, [tx(rqs=[rqi("key1", "key5", True, raw=[
        ("key1", (1, 0)), ("key2", (1, 1))])])], [12]))
    # combined_iterator_test.go: db key1,4,6,8 at {1,1}; earlier txs of the block put key3,
    # delete key5, put key6, put key7 (their heights are Height{blk, tx})
    cdb = {("ns", "key%d" % i): (1, 1) for i in (1, 4, 6, 8)}
    pre = [tx(writes=[("key3", b"value3", False)], ns="ns"), tx(writes=[("key5", b"", True)], ns="ns"),
           tx(writes=[("key6", b"value6_new", False)], ns="ns"), tx(writes=[("key7", b"value7", False)], ns="ns")]
    blk = 7
    ex = [("key3", (blk, 0)), ("key4", (1, 1)), ("key6", (blk, 2)), ("key7", (blk, 3))]
    cases.append(("combined_exclude_end", cdb, pre + [tx(rqs=[rqi("key2", "key8", True, raw=ex)], ns="ns")],
                  [0, 0, 0, 0, 0]))
    cases.append(("combined_include_end", cdb, pre + [tx(rqs=[rqi("key2", "key8", False, raw=ex + [("key8", (1, 1))])],
                                                         ns="ns")], [0, 0, 0, 0, 0]))
    cases.append(("combined_extra_range", cdb, pre + [tx(rqs=[rqi("key0", "key9", False, raw=[("key1", (1, 1))] + ex +
                                                                 [("key8", (1, 1))])], ns="ns")], [0, 0, 0, 0, 0]))
    cases.append(("combined_full_range", cdb, pre + [tx(rqs=[rqi("", "", True, raw=[("key1", (1, 1))] + ex +
                                                                [("key8", (1, 1))])], ns="ns")], [0, 0, 0, 0, 0]))
    cases.append(("combined_stale_view", cdb, pre + [tx(rqs=[rqi("key2", "key8", True, raw=[("key4", (1, 1)),
                                                                                          ("key6", (1, 1))])], ns="ns")],
                  [0, 0, 0, 0, 12]))
    # ordering: a stale public read in the same namespace wins over the phantom (11 before 12)
    cases.append(("read_before_range", pdb, [tx(reads=[("key1", (9, 9))], rqs=[rqi("key2", "key4", True, raw=[])])], [11]))
    return [(n, d, e, x, blk) for n, d, e, x in cases]


def random_blocks(seed, nblocks=4, ntx=120, nkeys=60):
    """-> (initial db {(ns, key): ver}, [(block bytes, committer flags)]): reads, range queries
    (raw or merkle, exhausted or not, perturbed at random), puts / deletes by earlier txs of the
    same block, a second namespace, a collection; simulation results come from the committed
    state as of the block's start, so intra-block writers decide most outcomes."""
    rnd = random.Random(seed)
    keys = ["k%03d" % i for i in range(nkeys)]
    db = {}
    for ns in ("ns1", "ns2"):
        for k in keys:
            if rnd.random() < 0.6:
                db[(ns, k)] = (rnd.randint(1, 5), rnd.randint(0, 9))
    state = dict(db)
    blocks = []
    for b in range(nblocks):
        number = 10 + b
        envs, flags = [], []
        for i in range(ntx):
            ns = rnd.choice(("ns1", "ns1", "ns2"))
            reads = []
            for _ in range(rnd.randint(0, 2)):
                k = rnd.choice(keys)
                v = state.get((ns, k))
                if rnd.random() < 0.1:
                    v = (99, 1)
                reads.append((k, v))
            rqs = []
            for _ in range(rnd.randint(0, 2)):
                a, c = sorted(rnd.sample(range(nkeys + 1), 2))
                start = keys[a] if rnd.random() < 0.9 else ""
                end = (keys[c] if c < nkeys else "k999") if rnd.random() < 0.85 else ""
                exhausted = rnd.random() < 0.5
                res = sorted((k, v) for (n, k), v in state.items()
                             if n == ns and k >= start and (end == "" or k < end))
                if not exhausted and end and (ns, end) in state:
                    res.append((end, state[(ns, end)]))
                r = rnd.random()
                if res and r < 0.15:
                    res.pop(rnd.randrange(len(res)))
                elif res and r < 0.25:
                    j = rnd.randrange(len(res))
                    res[j] = (res[j][0], (res[j][1][0] + 1, res[j][1][1]))
                elif r < 0.3:
                    res.append(("k998", (1, 1)))
                if rnd.random() < 0.35:
                    rqs.append(rqi(start, end, exhausted, merkle=merkle_of(rnd.choice((2, 3, 4)), res) or (2, 1, [])))
                else:
                    rqs.append(rqi(start, end, exhausted, raw=res))
            writes = []
            for k in rnd.sample(keys[10:], rnd.randint(0, 2)):  # (keys[:10] are never deleted)
                writes.append((k, b"" if rnd.random() < 0.25 else b"val", False))
            meta = rnd.sample(keys[:10], 1) if rnd.random() < 0.12 else []  # metadata-only writes
            ns_sets = [(ns, B.kv_rwset(reads, writes, rqs, meta))]
            if rnd.random() < 0.15:
                kh = bytes([rnd.randrange(256) for _ in range(32)])
                ns_sets = [(ns, B.kv_rwset(reads, writes, rqs, meta), [("coll", B.hashed_rwset([(kh, None)], [(kh, b"h" * 32, False)]))])]
            envs.append(env(ns_sets, i, number))
            flags.append(0 if rnd.random() < 0.95 else 10)
        from tests.blockfix import block_from_envs
        blk = block_from_envs(envs, number=number)
        blocks.append((blk, flags, number))
        # the generator's own view of the commit is not needed: the oracle commits
        from oracle import mvcc as OM
        sdb = OM.StateDB(state)
        OM.validate_block(sdb, blk, flags, number, commit=True)
        state = {(n, k.decode() if isinstance(k, bytes) and n in ("ns1", "ns2") else k): v for (n, k), v in sdb.v.items()}
    return db, blocks


def _hk(s):
    import hashlib
    return hashlib.sha256(s).digest()


def meta_db():
    return {("ns1", "key1"): (1, 0), ("ns1", "key2"): (1, 1), ("ns1$$hcoll1", _hk(b"k1")): (1, 2)}


def meta_cases():
    """metadata writes (tx_ops.go:17-53): -> [(name, [envelopes], committer flags, expected codes
    or "unsupported")], validated against meta_db() at block 5"""
    def mtx(reads=(), writes=(), meta=(), hreads=(), hwrites=(), hmeta=()):
        sets = [("ns1", B.kv_rwset(reads, writes, (), meta))]
        if hreads or hwrites or hmeta:
            sets = [("ns1", B.kv_rwset(reads, writes, (), meta), [("coll1", B.hashed_rwset(hreads, hwrites, hmeta))])]
        return env(sets)
    return [
        ("meta_existing_key_bumps_version", [mtx(meta=["key1"]), mtx(reads=[("key1", (1, 0))])], [0, 0], [0, 11]),
        ("meta_absent_key_is_noop", [mtx(meta=["key9"]), mtx(reads=[("key9", None)])], [0, 0], [0, 0]),
        ("meta_after_delete_panics", [mtx(writes=[("key2", b"", True)]), mtx(meta=["key2"])], [0, 0], "unsupported"),
        ("meta_on_key_put_earlier", [mtx(writes=[("key9", b"v", False)]), mtx(meta=["key9"]), mtx(reads=[("key9", None)])],
         [0, 0, 0], [0, 0, 11]),
        ("write_plus_meta_same_tx", [mtx(writes=[("key1", b"v", False)], meta=["key1"]), mtx(reads=[("key1", (1, 0))])],
         [0, 0], [0, 11]),
        ("hashed_meta_existing", [mtx(hmeta=[_hk(b"k1")]), mtx(hreads=[(_hk(b"k1"), (1, 2))])], [0, 0], [0, 11]),
        ("hashed_meta_absent_noop", [mtx(hmeta=[_hk(b"zz")]), mtx(hreads=[(_hk(b"zz"), None)])], [0, 0], [0, 0]),
        ("two_meta_writes_one_key", [mtx(meta=["key1", "key1"])], [0], "unsupported"),
        ("committer_invalid_meta_skipped", [mtx(reads=[("key1", (1, 0))]), mtx(meta=["key1"])], [0, 10], [0, 10]),
        ("invalid_tx_meta_not_applied", [mtx(reads=[("key1", (7, 7))], meta=["key2"]), mtx(reads=[("key2", (1, 1))])],
         [0, 0], [11, 0]),
    ]
