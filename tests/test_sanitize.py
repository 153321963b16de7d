"""CPU: the engine's host code on untrusted bytes under AddressSanitizer + UndefinedBehavior-
Sanitizer (tools/sanitize: libfgv's host sources built with -fsanitize=address,undefined on the
host side; no GPU call).  The harness drives every host parser a block reaches -- deliver-side
integrity (pbwire.h, envelope well-formedness, header DER), the commit-hash rwset walk
(fgv_commit.cpp), the committer's host parser + policy fold + orderer-signature metadata
(fgv_block.cpp, fgv_channel.cpp) and the MVCC phantom path's rwset decode and range-query
validators (fgv_mvcc.cpp) -- over generated blocks of every shape the tests use, the
reference's sample-ledger blocks, and thousands of mutations of them (bit flips, truncations,
insertions, corrupted envelopes and rwsets).  Any sanitizer report fails the run."""
import os
import random
import struct
import subprocess

import pytest

from fabric_amd.synth import blocks as B
from tests.blockfix import block_from_envs, corrupt_envelopes, network

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "build", "asan", "fgv_sanitize")


def _harness():
    if True:  # (make rebuilds it when a host source changed)
        subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "sanitize"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)
    return HARNESS


def _rec(kind, b):
    return struct.pack("<II", kind, len(b)) + b


def _mutate(rng, b, n):
    out = []
    for _ in range(n):
        x = bytearray(b)
        k = rng.randrange(4)
        if k == 0:
            for _ in range(rng.randint(1, 4)):
                x[rng.randrange(len(x))] ^= 1 << rng.randrange(8)
        elif k == 1:
            del x[rng.randrange(len(x)):]
        elif k == 2:
            p = rng.randrange(len(x))
            x[p:p] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 6)))
        else:
            p = rng.randrange(len(x))
            x[p] = rng.choice([0x00, 0xFF, 0x80, 0x7F, 0x0A, 0x12, 0x1A, 0x22, 0x0B, 0x0C])
        out.append(bytes(x))
    return out


def _rwsets(envs):
    from oracle import v20
    out = []
    for e in envs:
        try:
            cca, _ = v20.get_action_from_envelope(e)
        except Exception:  # not an endorser transaction that decodes: no rwset
            continue
        if cca.get("results"):
            out.append(cca["results"])
    return out


def _run(path):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:abort_on_error=0:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([_harness(), path], env=env, capture_output=True, text=True, timeout=600)
    report = r.stdout + r.stderr
    assert r.returncode == 0 and "Sanitizer" not in report and "runtime error" not in report, report[-4000:]
    return r.stdout


@pytest.fixture(scope="module")
def corpus():
    """(seed blocks, seed rwsets, identity records, policy) shared by the cases"""
    net = network()
    blks, rws = [], []
    blk, _, envs = B.make_block(net, 60, number=1, seed=11, threads=1)
    blks.append(blk)
    rws += _rwsets(envs)
    # hashed (private) rwsets and collections
    blk2, _, envs2 = B.make_block(net, 30, number=2, seed=12, threads=1, collections=("collA", "collB"))
    blks.append(blk2)
    rws += _rwsets(envs2)
    # range queries (raw and merkle) and metadata writes
    from tests import rq_cases as RQ
    for case in RQ.known_answer_cases()[:12]:
        case_envs = case[2]
        blks.append(block_from_envs(case_envs))
        rws += _rwsets(case_envs)
    # key-level endorsement known answers (metadata writes, hashed metadata writes, dependencies)
    from tests import sbe_cases
    for case in sbe_cases.load()[:8]:
        blks.append(case["block"])
    # orderer-signed blocks (metadata[SIGNATURES])
    from tests import blocksig_cases as BC
    for c in BC.cases()[:8]:
        blks += c["blocks"][:2]
    # the reference's sample-ledger blocks (config blocks, lifecycle, private data)
    from tests.test_oracle_ledgers import ledgers
    for b in ledgers()["v20_testchannel"][:12]:
        blks.append(b["block"])
    ids = [s for s, _ in net.identities()]
    return blks, rws, ids, net.chaincodes["mycc"], envs


def _write(tmp_path, name, blks, rws, ids, policy):
    body = _rec(5, b"testchannel") + _rec(3, policy) + b"".join(_rec(2, s) for s in ids)
    body += b"".join(_rec(1, b) for b in blks) + b"".join(_rec(4, r) for r in rws)
    p = tmp_path / name
    p.write_bytes(body)
    return str(p)


def test_harness_clean_on_valid_inputs(corpus, tmp_path):
    blks, rws, ids, policy, _ = corpus
    out = _run(_write(tmp_path, "valid.bin", blks, rws, ids, policy))
    assert "%d blocks" % len(blks) in out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_harness_clean_on_mutated_blocks(corpus, tmp_path, seed):
    blks, rws, ids, policy, envs = corpus
    rng = random.Random(seed)
    bad = []
    for b in blks:
        bad += _mutate(rng, b, 25)
    # blocks of corrupted envelopes (the envelope parser behind a well-formed block)
    for e in corrupt_envelopes(envs, seed, 200):
        bad.append(block_from_envs([envs[0], e]))
    bad_rws = []
    for r in rws:
        bad_rws += _mutate(rng, r, 6)
    out = _run(_write(tmp_path, "mut%d.bin" % seed, bad, bad_rws, ids, policy))
    assert "%d blocks" % len(bad) in out


def test_sanitizer_is_live(tmp_path):
    """a deliberate heap over-read (harness record kind 9) must abort with an ASan report"""
    p = tmp_path / "canary.bin"
    p.write_bytes(_rec(9, b"abcd"))
    r = subprocess.run([_harness(), str(p)], env=dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr


@pytest.mark.parametrize("seed", [1, 2])
def test_harness_clean_on_certificates_and_msp_configs(tmp_path, seed):
    """the MSP cache miss's host parsers: PEM / X.509 / sanitizeCert over the reference's MSP
    certificates, the synthetic cases and their mutations; FabricMSPConfig bytes and mutations"""
    import base64
    import json
    from oracle import x509 as X
    from oracle.protowire import decode
    from tests.msp_cases import synthetic
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "msp_fixtures.json")))
    pems = [p.encode() for p in fx["certs"].values()]
    pems += [decode("SerializedIdentity", c[1]).get("id_bytes") or b"" for c in synthetic()[1]]
    confs = [bytes.fromhex(m["config"]) for m in fx["msps"].values()]
    rng = random.Random(seed)
    recs = []
    from oracle.v20 import Unsupported
    from tests.msp_cases import fork_hazard_variants
    pems += [v for p in pems[:6] for _, v in fork_hazard_variants(p)]  # (the PEM / outer-shape branches)
    for p in pems[:60]:
        try:
            der = X.pem_decode(p)
        except Unsupported:
            continue
        if not der:
            continue
        for d in _mutate(rng, der, 25):
            recs.append(_rec(6, b"-----BEGIN CERTIFICATE-----\n" + base64.encodebytes(d) + b"-----END CERTIFICATE-----\n"))
        for m in _mutate(rng, p, 5):  # the PEM text itself
            recs.append(_rec(6, m))
    recs = [_rec(6, p) for p in pems] + [_rec(7, c) for c in confs] + recs
    for c in confs:
        recs += [_rec(7, m) for m in _mutate(rng, c, 20)]
    path = tmp_path / ("certs%d.bin" % seed)
    path.write_bytes(b"".join(recs))
    out = _run(str(path))
    assert "%d certs" % len(recs) in out
