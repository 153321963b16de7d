"""bench.py -- MI355X block-validation engine for Hyperledger Fabric's committer.

python bench.py --gpus N --steps K --warmup W [--workload block|c5|sig|mvcc]

block (default; BASELINE configs[1], C2 shape): 500-tx endorser blocks, 2-of-3 endorsement
  policy (OutOf(2, Org1..3.member)), 60 % of txs with 2 endorsements / 40 % with 3, 4 reads +
  4 writes of 200 B values, 100 client identities, injected faults (2 % bad creator sig, 2 %
  one bad endorsement of 3, 2 % policy unsatisfied, 0.5 % duplicate txid).  Weak scaling:
  every GPU owns --blocks-per-gpu blocks per step; a step is one committer pass over the
  world x B blocks: each rank validates its own blocks (fgv_validate_shard_dev_next: device
  parse + SHA-256 + ECDSA-P256 + policy fold), the ranks all-gather their 68-byte per-tx
  records over RCCL and finalize TxValidationFlags.  --batches distinct batches (default 6,
  ~366 MB per GPU, more than the 256 MiB Infinity Cache) are rotated through the timed loop.
  value = validated tx/s over all ranks with the blocks resident in HBM (max-over-ranks wall
  time of the timed steps).  Beside it: pcie_inclusive (the same rotation from page-locked
  host memory, each batch's H2D overlapped with the previous batch's validation),
  latency_1block_ms, per-kernel device times (kernel_ms), the roofline of the dominant kernel,
  and cpu_baseline = the restated full v20 validator (oracle/) on this host's CPU share and on
  one core, plus the identity.Verify-only bound.

c5 (configs[4]): 20k-tx blocks, 5-of-8 policy, P-256 + Ed25519, + deliver-side integrity.
sig (configs[3], C4 shape): 131,072 P-256 identity.Verify calls per GPU on 1.85 KB
  messages, inputs resident in HBM; value = verifies/s.
mvcc (configs[2], C3): 10k-tx blocks against a 1M-key state DB, validated and committed.
pipeline: the end-to-end commit path on the same C2-shaped blocks (committer -> MVCC with
  commit -> commit hash); value = committed tx/s; run with e.g. --steps 12 --warmup 2 (every
  batch is distinct and generated up front).
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np
import torch
import torch.distributed as dist

METRIC = "ECDSA-P256 verifies/sec + validated tx/sec per block at 1/2/4/8 MI355X"
STEPLOG = os.environ.get("BENCH_STEPLOG") == "1"  # per-step host timings of the timed loops (stderr)
# 32x32->64 multiply-add products per verify in the comb: 28 terms (12 signed
# 22-bit generator windows + 16 signed 17-bit key windows; round 5: 20 13-bit windows, 32 terms),
# the first one loaded, so 27 mixed additions x (8 field mults x 64 + 3 squarings x 36 products)
# + the projective x-check (3 x 64)
PRODUCTS_POINT = 27 * (8 * 64 + 3 * 36) + 3 * 64
# the same for one variable-base verify in k_vb_mul: 8 lanes, each 28 doublings
# (3 mults + 5 squarings), 7.5 expected mixed additions from the key's table (8 mults + 3
# squarings) and 3 butterfly additions (12 mults + 4 squarings), + u2 = r * s^-1 (sn_mul, 128)
VB_MUL_PRODUCTS = 8 * (28 * (3 * 64 + 5 * 36) + 7.5 * (8 * 64 + 3 * 36) + 3 * (12 * 64 + 4 * 36) + 128)
# chip-wide v_mad_u64_u32 issue rate measured by tools/valu_peak.hip (profiles/round1_valu_peak.json)
PEAK_MAD_PER_S = float(os.environ.get("FGV_PEAK_MAD", "3.106e13"))
# 256 CU x 4 SIMD x 32 lanes x 2.4 GHz simple int32 VALU lane-ops
PEAK_INT32_OPS = 78.6e12
SHA_OPS_PER_COMPRESSION = 2.7e3


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def pmc_traffic(workload):
    """HBM bytes per launch of the workload's dominant kernel from the committed rocprofv3 PMC
    passes (profiles/*_traffic.json, written by tools/summarize_profiles.py); None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        t = d["workloads"][workload]
        if "hbm_bytes" in t:
            return t["hbm_bytes"], (f"{os.path.basename(files[-1])}: {t['kernel']} fetch {t['fetch_bytes']} B + "
                                    f"write {t['write_bytes']} B")
        low = (f"; lower bound {t['hbm_bytes_per_block_low']} B with the gathers' FETCH_SIZE unscaled"
               if "hbm_bytes_per_block_low" in t else "")
        return t["hbm_bytes_per_block"], (f"{os.path.basename(files[-1])}: per block, {len(t['kernels'])} kernels, "
                                          f"fetch {t['fetch_bytes_per_block']} B + write {t['write_bytes_per_block']} B"
                                          + low)
    except (KeyError, ValueError, OSError):
        return None, None


def roofline(n_verifies, point_ms, workload):
    point_s = point_ms / 1e3
    achieved = n_verifies * PRODUCTS_POINT / point_s / 1e12 if point_s > 0 else 0.0
    traffic, src = pmc_traffic(workload)
    return dict(bound="valu", achieved=round(achieved, 3), peak=round(PEAK_MAD_PER_S / 1e12, 3),
                unit="Tops/s", frac=round(achieved * 1e12 / PEAK_MAD_PER_S, 4), traffic=traffic, traffic_source=src,
                kernel="k_point28 (+ k_point hand-overs)",
                kernel_avg_ms=round(point_ms, 4), per_launch_products=int(n_verifies * PRODUCTS_POINT),
                work_unit="v_mad_u64_u32 (32x32->64 multiply-add) products of the comb algorithm")


def roofline_vb(n_items, vb_ms):
    """k_vb_mul (the churn variants' dominant kernel) against the same v_mad_u64_u32 peak"""
    t = vb_ms / 1e3
    achieved = n_items * VB_MUL_PRODUCTS / t / 1e12 if t > 0 else 0.0
    return dict(bound="valu", achieved=round(achieved, 3), peak=round(PEAK_MAD_PER_S / 1e12, 3), unit="Tops/s",
                frac=round(achieved * 1e12 / PEAK_MAD_PER_S, 4), traffic=None, traffic_source=None,
                kernel="k_vb_mul", kernel_avg_ms=round(vb_ms, 4), per_launch_products=int(n_items * VB_MUL_PRODUCTS),
                work_unit="v_mad_u64_u32 products of the 8-lane variable-base multiplication u2 * Q")


def profiled_dominant(workload="block"):
    """the top row of the latest committed per-step kernel stats (profiles/round*_<workload>_
    kernel_stats.csv: rocprofv3 --kernel-trace --stats of 32-block steps, the one-time comb
    table builds and key preparations excluded) -> (kernel, avg us, file); (None, None, None) without one"""
    import csv
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", f"round*_{workload}_kernel_stats.csv"))
    if not files:
        return None, None, None
    f = max(files, key=lambda p: int(re.search(r"round(\d+)", os.path.basename(p)).group(1)))
    rows = [r for r in csv.DictReader(open(f)) if not r["Name"].startswith(("k_gtab", "k_keytab", "k_keybase", "k_keyprep", "k_kmap_set", "k_p384_tab", "k_p384_norm"))]
    if not rows:
        return None, None, None
    top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    return top["Name"].split("(")[0], float(top["AverageNs"]) / 1e3, os.path.basename(f)


def block_roofline(kavg, pay_blocks, verifies, batch_bytes, workload, sha_blocks=0.0):
    """roofline of the committer step's dominant kernel: the top row of the committed per-step
    kernel stats (profiled_dominant), timed live (HIP events on its stream) in this run, with
    frac_profiled = the same work / that row's average duration (recomputable from the file).
    Work models:
      k_point28         v_mad_u64_u32 products of the comb (PRODUCTS_POINT per verify) vs the
                        measured 31.06 T/s chip peak;
      k_bd_sha_payload  SHA-256 compressions x 2.7e3 int32 ops vs the 78.6 T
                        int32 lane-op peak;
      k_bd_sha          the same for the other messages' compressions (endorsement prp || endorser,
                        txid, proposal hash, index txid): sha_blocks = the step's compressions
                        minus the payloads' (not the call's total);
      k_bd_parse        the batch's block bytes (each envelope's lines are requested once) vs
                        8 TB/s HBM: a walk of dependent loads, so frac says how far from any
                        throughput bound it runs.
    The other two are `others`."""
    cands = {k: v for k, v in kavg.items() if k != "batch"}
    dom, dom_us, dom_src = profiled_dominant("block" if workload == "block" else workload)
    models = {}
    pt = roofline(verifies, kavg.get("k_point28", 0.0), workload + "_point")
    pt["per_launch_verifies"] = int(verifies)
    if dom_us and dom == "k_point28":
        pt["frac_profiled"] = round(verifies * PRODUCTS_POINT / (dom_us * 1e-6) / PEAK_MAD_PER_S, 4)
    models["k_point28"] = pt
    t_pay = kavg.get("k_bd_sha_payload", 0.0) / 1e3
    ach = pay_blocks * SHA_OPS_PER_COMPRESSION / t_pay / 1e12 if t_pay > 0 else 0.0
    traffic, src = pmc_traffic(workload)
    pay = dict(bound="valu", achieved=round(ach, 3), peak=round(PEAK_INT32_OPS / 1e12, 1), unit="Tops/s",
               frac=round(ach * 1e12 / PEAK_INT32_OPS, 4), traffic=traffic, traffic_source=src,
               kernel="k_bd_sha_payload", kernel_avg_ms=round(t_pay * 1e3, 4),
               per_launch_compressions=int(pay_blocks),
               work_unit="SHA-256 compressions x 2.7e3 simple int32 ops (SURVEY.md s8(d))")
    if dom_us and dom == "k_bd_sha_payload":
        pay["frac_profiled"] = round(pay_blocks * SHA_OPS_PER_COMPRESSION / (dom_us * 1e-6) / PEAK_INT32_OPS, 4)
    models["k_bd_sha_payload"] = pay
    t_sha = kavg.get("k_bd_sha", 0.0) / 1e3
    ach2 = sha_blocks * SHA_OPS_PER_COMPRESSION / t_sha / 1e12 if t_sha > 0 else 0.0
    sha = dict(bound="valu", achieved=round(ach2, 3), peak=round(PEAK_INT32_OPS / 1e12, 1), unit="Tops/s",
               frac=round(ach2 * 1e12 / PEAK_INT32_OPS, 4), traffic=None, traffic_source=None,
               kernel="k_bd_sha", kernel_avg_ms=round(t_sha * 1e3, 4), per_launch_compressions=int(sha_blocks),
               work_unit="SHA-256 compressions x 2.7e3 simple int32 ops (SURVEY.md s8(d))")
    if dom_us and dom == "k_bd_sha":
        sha["frac_profiled"] = round(sha_blocks * SHA_OPS_PER_COMPRESSION / (dom_us * 1e-6) / PEAK_INT32_OPS, 4)
    models["k_bd_sha"] = sha
    t_parse = kavg.get("k_bd_parse", 0.0) / 1e3
    gbs = batch_bytes / t_parse / 1e9 if t_parse > 0 else 0.0
    ptr, psrc = pmc_traffic(workload + "_parse")
    parse = dict(bound="hbm", achieved=round(gbs, 2), peak=8000.0, unit="GB/s", frac=round(gbs / 8000.0, 5),
                 traffic=ptr, traffic_source=psrc, kernel="k_bd_parse", kernel_avg_ms=round(t_parse * 1e3, 4),
                 per_launch_bytes=int(batch_bytes),
                 work_unit="block bytes of the batch (every envelope line requested once, touch_lines)")
    if dom_us and dom == "k_bd_parse":
        parse["frac_profiled"] = round(batch_bytes / (dom_us * 1e-6) / 8e12, 5)
    models["k_bd_parse"] = parse
    key = dom if dom in models else "k_point28"
    r = dict(models[key])
    r["others"] = {k: v for k, v in models.items() if k != key}
    r["dominant_kernel_profiled"] = dict(kernel=dom, avg_us=dom_us, source=dom_src)
    r["dominant_kernel_live"] = max(cands, key=cands.get) if cands else None
    return r


def cpu_verify_rate(keymat, msgs, sigs, threads, target_s=12.0):
    """Oracle (Go-rule DER + low-S + OpenSSL 3.0.2 P-256, SHA-256 of the message) on host
    threads; repeats the sample until ~target_s of CPU wall time."""
    import oracle
    from fabric_amd._lib import pack
    n = len(sigs)
    K = np.ascontiguousarray(keymat, dtype=np.uint8)
    ma, mo, ml = pack(msgs)
    sa, so, sl = pack(sigs)
    st = np.zeros(n, np.uint8)
    L = oracle.lib()
    done, t0 = 0, time.time()
    while time.time() - t0 < target_s:
        L.oracle_verify_msgs_batch(K.ctypes.data, ma.ctypes.data, mo.ctypes.data, ml.ctypes.data, sa.ctypes.data,
                                   so.ctypes.data, sl.ctypes.data, n, st.ctypes.data, threads, 1)
        done += n
    el = time.time() - t0
    return done / el, done, el


# ------------------------------------------------------------------ block workload
# C2 (configs[1], the headline) and C5 (configs[4]) share the block pipeline; C5 adds the
# deliver-side integrity pass (header chain + well-formedness + SHA-256 block data hash).
BLOCK_SPECS = {
    "block": dict(net=dict(seed=3, orgs=3, clients=100), endorse=((2, 0.6), (3, 0.4)), integrity=False,
                  desc="C2: {T}-tx endorser blocks, OutOf(2,[Org1..3.member]), 2-3 endorsements, "
                       "4R/4W x 200B, 100 clients, faults 2%/2%/2%/0.5%"),
    "c5": dict(net=dict(seed=5, orgs=8, clients=200, policy_n=5, peers_per_org=2, ed25519_frac=0.1,
                        ed25519_peers=1), endorse=((5, 0.5), (6, 0.5)), integrity=True,
               desc="C5: {T}-tx blocks, OutOf(5,[Org1..8.member]), 5-6 endorsements from 16 peers, 10% of "
                    "clients + 1 peer Ed25519 (rejected at DeserializeIdentity, SURVEY F4), faults "
                    "2%/2%/2%/0.5%, VerifyBlock integrity + SHA-256 block data hash"),
}


def _dist_info(world):
    """what the collective layer saw (the driver's scaling run checks that RCCL had N ranks)"""
    if world > 1 and dist.is_initialized():
        return dict(world_size=dist.get_world_size(), backend=str(dist.get_backend()),
                    same_device=bool(os.environ.get("FGV_BENCH_SAME_DEVICE")))
    return dict(world_size=1, backend=None)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """host threads this rank may use: the affinity mask, capped by OMP_NUM_THREADS (16 on a
    one-GPU lease, whose nproc shows the whole machine)"""
    n = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


_CPU_MODEL = None  # the forked full-validator workers' channel model


def _oracle_block(blk):
    from oracle import v20
    t = time.perf_counter()
    f = v20.validate_block(_CPU_MODEL, blk)
    return len(f), time.perf_counter() - t


def cpu_full_validator(net, blks, procs, target_s):
    """The restated v20 committer (oracle/v20.py: protobuf walk, MSP lookup, OpenSSL P-256
    identity.Verify through oracle/liboracle.so, policy evaluation, flag fold) on `procs`
    forked worker processes, one block per task, until ~target_s of wall time.  Runs before
    this process touches the GPU (fork)."""
    import multiprocessing as mp
    from oracle import v20
    global _CPU_MODEL
    _CPU_MODEL = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
    if procs == 1:
        done, t0 = 0, time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < target_s:
            done += _oracle_block(blks[i % len(blks)])[0]
            i += 1
        return done / (time.perf_counter() - t0), done, time.perf_counter() - t0, i
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        pool.map(int, range(procs))  # workers up
        per = _oracle_block(blks[0])[1]  # seconds per block on one core (sizes the sample)
        nblk = max(procs, int(round(target_s * procs / max(per, 1e-3) / procs)) * procs)
        t0 = time.perf_counter()
        res = pool.map(_oracle_block, [blks[i % len(blks)] for i in range(nblk)], chunksize=1)
        el = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    return done / el, done, el, nblk


def cpu_c_validator(net, blks, labels, threads, target_s, expected=None):
    """The plain-C restatement of the committer for this workload's shapes (oracle/
    cpu_validator.c: protobuf walk, registry lookup, SHA-256, Go-rule DER + low-S + OpenSSL 3
    P-256 Verify, OutOf(n, member) fold, txid duplicates) on `threads` host threads, whole
    blocks per thread, repeated until ~target_s of wall time.  Returns (tx/s, tx, seconds,
    blocks, parity with the generator's labels)."""
    import ctypes
    import oracle
    from fabric_amd.synth import blocks as B
    L = oracle.lib()
    ids = net.identities()
    msp_ix = {m: i for i, m in enumerate(net.mspids)}
    canon = {}
    ser = [s for s, _ in ids]
    soff = np.cumsum([0] + [len(x) for x in ser[:-1]]).astype(np.uint64)
    slen = np.array([len(x) for x in ser], np.uint32)
    sbuf = np.frombuffer(b"".join(ser), np.uint8)
    keys = np.zeros((len(ids), 64), np.uint8)
    msp = np.zeros(len(ids), np.int32)
    cano = np.zeros(len(ids), np.int32)
    ok = np.zeros(len(ids), np.uint8)
    for i, (_, I) in enumerate(ids):
        if I.pub is not None and I.key == "p256":
            keys[i] = np.frombuffer(I.pub, np.uint8)
            ok[i] = 1 if I.valid else 0
        msp[i] = msp_ix.get(I.mspid, -1)
        cano[i] = canon.setdefault((I.mspid, bytes(I.id_digest)), len(canon))
    pol = np.array([msp_ix[m] for m in net.mspids], np.int32)
    nb = len(blks)
    bptr = (ctypes.c_void_p * nb)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value for b in blks])
    lens = (ctypes.c_size_t * nb)(*[len(b) for b in blks])
    exp = [c for f in expected for c in f] if expected is not None else \
        [c for lab in labels for c in B.expected_codes(lab)]
    flags = np.zeros(len(exp) + 16, np.uint8)
    ntx = (ctypes.c_size_t * nb)()
    fn = L.oracle_cpu_validate_blocks
    fn.restype = ctypes.c_int
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    fn.argtypes = [vp, vp, sz, ctypes.c_char_p, ctypes.c_char_p, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp,
                   vp, vp, sz, vp, sz, vp, ctypes.c_int]

    def once():
        rc = fn(ctypes.cast(bptr, vp), ctypes.cast(lens, vp), nb, net.channel.encode(), b"mycc", pol.ctypes.data,
                len(pol), net.policy_n, sbuf.ctypes.data, soff.ctypes.data, slen.ctypes.data, keys.ctypes.data,
                msp.ctypes.data, cano.ctypes.data, ok.ctypes.data, len(ids), flags.ctypes.data, len(flags),
                ctypes.cast(ntx, vp), threads)
        assert rc == 0, rc
        return sum(ntx)
    n0 = once()
    parity = list(flags[:n0]) == exp
    done, rounds, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < target_s:
        done += once()
        rounds += 1
    el = time.perf_counter() - t0
    return done / el, done, el, rounds * nb, parity


def run_block(args, world, rank, local, dev_fn):

    from fabric_amd import _lib, shard, txvalidator
    from fabric_amd.synth import blocks

    spec = dict(BLOCK_SPECS[args.workload])
    if args.clients:  # identity churn: creators spread over this many client identities
        spec["net"] = dict(spec["net"], clients=args.clients)
        spec["desc"] = spec["desc"].replace("100 clients", f"{args.clients} clients (churn: client keys on the "
                                            f"variable-base kernels)")
    t0 = time.time()
    pems = None
    if world > 1:
        obj = [None]
        if rank == 0:
            obj[0] = blocks.Network(**spec["net"]).export_pems()
        dist.broadcast_object_list(obj, src=0)
        pems = obj[0]
    net = blocks.Network(pems=pems, **spec["net"])
    B, T, NB = args.blocks_per_gpu, args.tx_per_block, args.batches
    if args.workload == "c5":
        B, T, NB = args.c5_blocks_per_gpu, args.c5_tx_per_block, args.c5_batches
    # NB distinct batches per rank, rotated through the timed loop (their bytes together exceed
    # the 256 MiB Infinity Cache at the default sizes); each rank's blocks of a batch form a
    # hash chain numbered 1 + (k * world + rank) * B + i
    mine = []
    for k in range(NB):
        prev, cur = b"\x00" * 32, []
        for i in range(B):
            num = 1 + (k * world + rank) * B + i
            blk, lab, envs = blocks.make_block(net, T, number=num, seed=7919 * rank + 100003 * k + i, threads=8,
                                               endorse_dist=spec["endorse"], prev_hash=prev)
            cur.append((blk, lab))
            prev = blocks.header_hash(num, prev, envs)
        mine.append(cur)
    my_blocks = [[m[0] for m in cur] for cur in mine]
    log(f"[bench] rank {rank}: {NB} x {B} blocks x {T} tx ready in {time.time() - t0:.1f}s")

    cpu = None
    if rank == 0 and world == 1 and args.cpu_threads != 0:
        # CPU baselines first: the full-validator workers are forked before any GPU use
        procs = args.cpu_threads if args.cpu_threads > 0 else _cpu_share()
        sample = my_blocks[0][:max(1, min(B, 2 * procs))]
        labs = [m[1] for m in mine[0][:len(sample)]]
        c_n = cpu_c_validator(net, sample, labs, procs, args.cpu_seconds)
        c_1 = cpu_c_validator(net, sample[:2], labs[:2], 1, args.cpu_seconds / 2)
        log(f"[bench] cpu C validator: {c_n[0]:,.0f} tx/s on {procs} threads, {c_1[0]:,.0f} tx/s on 1, "
            f"parity {c_n[4] and c_1[4]}")
        full_n = cpu_full_validator(net, sample, procs, args.cpu_seconds / 3)
        full_1 = cpu_full_validator(net, sample[:1], 1, args.cpu_seconds / 4)
        cpu = dict(procs=procs, full=full_n, full1=full_1, c=c_n, c1=c_1)
        log(f"[bench] cpu full validator: {full_n[0]:,.0f} tx/s on {procs} procs, {full_1[0]:,.0f} tx/s on 1")
    dev = dev_fn()

    # Under the block plan a rank needs only its own blocks' bytes -- the others' results
    # arrive as all-gathered records -- so only the labels (for the parity check) travel.
    my_labels = [[m[1] for m in cur] for cur in mine]
    if world > 1:
        allb = [None] * world
        dist.all_gather_object(allb, my_labels)
        labels = [[l for r in range(world) for l in allb[r][k]] for k in range(NB)]
        blks = [[my_blocks[k][i] if r == rank else b"" for r in range(world) for i in range(B)] for k in range(NB)]
    else:
        labels, blks = my_labels, my_blocks

    eng = _lib.Engine(local, host_threads=args.host_threads or min(24, _cpu_share()))
    if args.host_parse:
        eng.set_parse_mode(1)
    # the headline's 100 clients sign ~160 times per step: registered with comb tables, the state
    # promotion by use reaches after the first call anyway -- so the untimed parity
    # and warmup calls run the same kernels as the timed steps (the profiled kernel averages agree
    # with the live ones); --clients (churn) keeps them on the variable-base kernels
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, hot_clients=not args.clients)
    ntx = np.array([T] * (world * B), dtype=np.int64)
    plan = shard.plan(ntx, world, "block")
    lo, hi = plan[0][rank], plan[1][rank]
    rows = shard.plan_rows(*plan)
    send = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
    recv = torch.zeros((world * rows, shard.REC), dtype=torch.uint8, device=dev) if world > 1 else send
    flags_out = np.empty(int(ntx.sum()), dtype=np.uint8)

    # (1) every batch resident in HBM (64 B tail padding per block): the headline `value`
    sizes = [(len(b) + 64 + 255) // 256 * 256 for bl in blks for b in bl]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptrs, o = [], 0
    for bl in blks:
        cur = []
        for b in bl:
            if len(b):  # (other ranks' blocks are empty placeholders)
                arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
            cur.append(arena.data_ptr() + o)
            o += (len(b) + 64 + 255) // 256 * 256
        dptrs.append(cur)
    hbm_batches = [eng.block_batch(blks[k], dptrs[k]) for k in range(NB)]
    torch.cuda.synchronize()

    def steps_for(batches):
        # batch k's call pre-splits (and, host-resident, pre-copies) batch k+1 of the rotation
        # one GPU: validation + finalize in one call (fgv_validate_blocks_pipelined); N > 1: each rank
        # validates its shard, the ranks all-gather the records, every rank finalizes
        st = [_lib.BlockStep(eng, batches[k], lo, hi, send.data_ptr(), rows, ntx, world, recv.data_ptr(), flags_out,
                             plan=plan, presplit=not args.no_presplit, next_batch=batches[(k + 1) % NB],
                             fused=world == 1 and not args.shard_protocol)
              for k in range(NB)]
        for k, s in enumerate(st):
            s.after_next = batches[(k + 2) % NB]
            s.after_next2 = batches[(k + 3) % NB]
        return st

    integ = dict(ms=0.0, ok=True)

    def verify_mine(k):  # deliver-side VerifyBlock of this rank's blocks of batch k (own host pool)
        first = 1 + (k * world + rank) * B
        chain = _lib.ChainState(number=first - 1, valid=1, has_hash=0)
        t = time.perf_counter()
        res = eng.blocks_verify(my_blocks[k], chain)
        integ["ms"] += (time.perf_counter() - t) * 1e3
        integ["ok"] &= all(r[0] == _lib.BLK_OK for r in res) and chain.number == first - 1 + B

    # C5: the deliver side verifies a batch (VerifyBlock: header chain, well-formedness, one
    # sequential SHA-256 data hash per block -- SURVEY H6) ahead of its validation: while the
    # committer validates batch k, VerifyBlock of batches k+1 .. k+INTEG_DEPTH runs on host threads
    # (one engine pool of FGV_HASH_THREADS per concurrent call); a step ends when its own batch
    # has been both verified and validated.  Consecutive calls take consecutive batches of the
    # rotation in every loop below.
    from concurrent.futures import ThreadPoolExecutor
    integ_ex = ThreadPoolExecutor(max_workers=args.integ_depth) if spec["integrity"] else None
    integ_fut, seq = {}, [0]

    def step(bs, k):
        s = None
        if spec["integrity"]:
            s = seq[0]
            seq[0] += 1
            for d in range(args.integ_depth + 1):
                if s + d not in integ_fut:
                    integ_fut[s + d] = integ_ex.submit(verify_mine, (k + d) % NB)
        t_a = time.perf_counter() if STEPLOG else 0.0
        bs.validate()
        if world > 1:
            shard.allgather_device(send, recv, eng=eng)
        t_b = time.perf_counter() if STEPLOG else 0.0
        f = bs.finalize()
        t_c = time.perf_counter() if STEPLOG else 0.0
        if args.presplit_early and world == 1 and not args.no_presplit:
            # a peer walks a batch's framing once its blocks are delivered (fgv_presplit keeps the
            # two latest requests): batches k+2 and k+3 after call k, so the call before each
            # batch finds its walk done at its top and queues the batch's parse there (front_early)
            eng.presplit(bs.after_next)
            eng.presplit(bs.after_next2)
        if STEPLOG:
            ht = eng.host_timing()
            steplog.append(dict(validate=(t_b - t_a) * 1e3, finalize=(t_c - t_b) * 1e3,
                                presplit=(time.perf_counter() - t_c) * 1e3, **{"lib_" + k: v for k, v in ht.items()}))
        if s is not None:
            integ_fut.pop(s).result()
        return f

    def parity(k, flags):
        exp = np.array([e if e is not None else 255 for bl in labels[k] for e in blocks.expected_codes(bl)], np.int64)
        known = np.array([e is not None for bl in labels[k] for e in blocks.expected_codes(bl)])
        bad = np.nonzero((flags.astype(np.int64) != exp) & known)[0]
        if len(bad):  # (diagnostic: which transactions, which codes)
            log(f"[bench] rank {rank}: batch {k}: {len(bad)} flags differ: "
                + ", ".join(f"tx {int(i)} (block {int(i) // T}) got {int(flags[i])} want {int(exp[i])}" for i in bad[:8]))
        return int(len(bad))

    steplog = []  # (BENCH_STEPLOG) per-step host phases

    def timed(steps_list, K, per_step=None, step_fn=None, start=0):
        # start: the rotation index the previous call announced as its next batch (its front
        # half and pre-split are already queued), so timed call 0 continues the pipeline
        fn = step_fn or step
        if world > 1:
            dist.barrier()
        # the interpreter's cyclic GC stays out of the timed loop (a generation-2 pass over the
        # bench's millions of label / block objects took ~6 ms inside one step of the PCIe pass)
        gc.collect()
        gc.disable()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        marks = []
        for s in range(start, start + K):
            fn(steps_list[s % NB], s % NB)
            if per_step is not None:
                per_step()
            if STEPLOG:
                marks.append(time.perf_counter())
        torch.cuda.synchronize()
        gc.enable()
        if STEPLOG and marks:  # (diagnostic: host-side per-step durations, BENCH_STEPLOG=1)
            d = [(b - a) * 1e3 for a, b in zip([t0] + marks[:-1], marks)]
            log("[bench] steps ms: " + " ".join("%.3f" % x for x in d))
            if len(steplog) >= K:
                j = max(range(K), key=lambda q: d[q])
                med = sorted(range(K), key=lambda q: d[q])[K // 2]
                log("[bench] slowest step %d: %s" % (j, {k: round(v, 3) for k, v in steplog[-K + j].items()}))
                log("[bench] median step %d: %s" % (med, {k: round(v, 3) for k, v in steplog[-K + med].items()}))
            steplog.clear()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    hsteps = steps_for(hbm_batches)
    mism = 0
    for k in range(NB):  # parity of every batch of the rotation (untimed)
        mism += parity(k, step(hsteps[k], k).copy())
    for s in range(args.warmup):
        step(hsteps[s % NB], s % NB)
    if not integ["ok"]:
        mism = max(mism, 1)
        log(f"[bench] rank {rank}: block integrity check failed")
    integ["ms"] = 0.0
    if mism:
        log(f"[bench] rank {rank}: {mism} flags differ from generator labels")

    # the last warmup call ran batch W-1 and announced batch W (mod NB): the timed loop starts there.
    # Per-call diagnostics are summed inside the library (fgv_stats_sums) and read once after the
    # loop: no library call per step besides the validation itself.
    start = args.warmup % NB
    eng.stats_sums(reset=True)
    el = timed(hsteps, args.steps, start=start)
    sums = eng.stats_sums()
    acc = dict(point=sums["point_ms"], prep=sums["prep_ms"], sha=sums["sha_ms"], verifies=sums["verifies"],
               sha_blocks=sums["sha_blocks"], pay_blocks=sums["pay_blocks"])
    kern = dict(sums["kernel_ms"])
    host = {k: sums[k] for k in ("parse_ms", "assemble_ms", "device_ms", "fold_ms", "front_ahead_ms", "gap_ms",
                                 "finish_ms")}
    kstats = eng.key_stats()  # (vb_verifies_last: the last timed step's variable-base verifies)
    # per-kernel times of the back half need the timestamp events fgv_set_timing adds (each a
    # packet on the critical path): read them from an instrumented, untimed pass
    kdiag = {n: 0.0 for n in _lib.Engine.KERNELS}
    eng.set_timing(True)
    for s in range(start + args.steps, start + args.steps + NB):
        step(hsteps[s % NB], s % NB)
        for key, v in eng.kernel_times()[0].items():
            kdiag[key] += v / NB
    eng.set_timing(False)
    # per-rank timing (the multi-rank rehearsal compares each rank's own device time with N=1's)
    print(f"[bench] rank {rank}/{world}: {el / args.steps * 1e3:.3f} ms per step, device batch "
          f"{kern.get('batch', 0.0) / max(1, args.steps):.3f} ms (first kernel to last), device pass "
          f"{host['device_ms'] / max(1, args.steps):.3f} ms (host wall of the device work), "
          f"{B * T} tx per rank-step", file=sys.stderr, flush=True)
    tot = torch.tensor([el, acc["verifies"], 1.0 if mism == 0 else 0.0], dtype=torch.float64, device=dev)
    if world > 1:
        mx = tot.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        mn = tot.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        el, all_verifies, ok = float(mx[0]), float(sm[1]), bool(mn[2] > 0)
    else:
        all_verifies, ok = float(acc["verifies"]), mism == 0
    K = args.steps
    total_tx = world * B * T * K
    batch_mb = sum(len(b) for b in my_blocks[0]) / 1e6

    # (2) PCIe-inclusive: the batches in page-locked host memory; each call copies nothing
    # itself -- the previous call queued its H2D on the copy stream (fgv_validate_shard_dev_next)
    pcie = None
    if not args.no_pcie:
        pins, pin_batches = [], []
        for k in range(NB):
            pb = eng.host_alloc(max(1, sum(len(b) for b in blks[k])))
            views, o = [], 0
            for b in blks[k]:
                pb.a[o:o + len(b)] = np.frombuffer(b, np.uint8)
                views.append(pb.a[o:o + len(b)])
                o += len(b)
            pins.append(pb)
            pin_batches.append(eng.block_batch(views))
        psteps = steps_for(pin_batches)

        # batch k stages batch k+2 (fgv_prefetch) besides its pipelined NEXT batch k+1: the copy
        # stream always holds the next copy, so the link runs back to back
        def pin_step(bs, k):
            t_p = time.perf_counter() if STEPLOG else 0.0
            eng.prefetch(pin_batches[(k + 2) % NB])
            f = step(bs, k)
            if STEPLOG and steplog:
                steplog[-1]["prefetch"] = (time.perf_counter() - t_p) * 1e3 - sum(
                    steplog[-1][q] for q in ("validate", "finalize", "presplit"))
            return f

        pm = 0
        for k in range(NB):  # parity of every batch (untimed)
            pm += parity(k, pin_step(psteps[k], k).copy())
        # warmup (untimed), continuing the rotation: the timed loop starts at the batch the last
        # call announced.  At least 32 steps: the first ~15-30 steps of sustained H2D traffic in a
        # process hold one ~7 ms stall of the whole device (compute and copy engine alike, link idle;
        # traced in r6i-r6p, DESIGN.md s5: absent with >= 30 warmup steps in every pass since, absent
        # from the HBM pass) -- a one-time transition, not the steady state a catching-up peer runs in
        PW = max(args.warmup, 32)
        for s in range(NB, NB + PW):
            pin_step(psteps[s % NB], s % NB)
        Kp = max(K, 2 * NB)
        pel = timed(psteps, Kp, step_fn=pin_step, start=(NB + PW) % NB)
        # raw H2D rate of one batch from pinned memory (the PCIe link's share of the step), after
        # the timed pass (torch's copies beside the engine's staged ones would skew neither)
        torch.cuda.synchronize()  # (device-wide: the engine's queued next-batch work too)
        hb = torch.from_numpy(pins[0].a)
        dbuf = torch.empty(hb.numel(), dtype=torch.uint8, device=dev)
        dbuf.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            dbuf.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        h2d = hb.numel() * 5 / (time.perf_counter() - t) / 1e9
        del dbuf
        if world > 1:
            t2 = torch.tensor([pel, float(pm)], dtype=torch.float64, device=dev)
            dist.all_reduce(t2, op=dist.ReduceOp.MAX)
            pel, pm = float(t2[0]), int(t2[1])
        pcie = dict(value=round(world * B * T * Kp / pel, 1), unit="validated tx/s", steps=Kp, warmup=PW,
                    ms_per_step=round(pel / Kp * 1e3, 3), parity_vs_labels=pm == 0,
                    h2d_GBps=round(h2d, 2), batch_MB=round(batch_mb, 2),
                    note="blocks in fgv_host_alloc'd host memory; during batch k's validation the copy stream "
                         "holds the H2D of batches k+1 and k+2 (fgv_prefetch), back to back")
        for pb in pins:
            pb.close()

    # (3) single-block latency (block in hand -> flags), no pre-split, HBM- and host-resident
    lat = None
    if world == 1 and not args.no_latency:
        lat = {}
        one = np.array([T], dtype=np.int64)
        f1 = np.empty(T, dtype=np.uint8)
        b0 = my_blocks[0][0]
        pb = eng.host_alloc(len(b0))
        pb.a[:] = np.frombuffer(b0, np.uint8)
        for name, bb in (("hbm", eng.block_batch([b0], [dptrs[0][0]])), ("host_pinned", eng.block_batch([pb.a]))):
            st1 = _lib.BlockStep(eng, bb, [0], [T], send.data_ptr(), T, one, 1, send.data_ptr(), f1, presplit=False,
                                 fused=not args.shard_protocol)
            ts = []
            for _ in range(args.latency_reps + 2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                st1.validate()
                st1.finalize()
                ts.append((time.perf_counter() - t) * 1e3)
            lat[name] = round(float(np.median(ts[2:])), 4)
        pb.close()

    # live (timed region): the kernels whose bracketing events order the streams anyway
    LIVE = ("k_bd_sha_payload", "k_bd_parse", "k_bd_sha", "k_bd_ident+count", "k_point28")
    kavg = {k: round(v / K, 4) if k in LIVE else round(kdiag[k], 4) for k, v in kern.items()}
    out = dict(metric=METRIC, value=round(total_tx / el, 1), unit="validated tx/s", n_gpus=world, steps=K,
               dist=_dist_info(world),
               warmup=args.warmup, ms_per_step=round(el / K * 1e3, 3), higher_is_better=True, scaling="weak",
               vs_baseline=None, dtype="u32", data="synthetic",
               config=dict(workload=spec["desc"].format(T=T),
                           blocks_per_step=world * B, tx_per_block=T, global_batch=world * B * T,
                           distinct_batches=NB, resident_MB=round(NB * batch_mb * world, 1),
                           parallelism=("single-gpu (fgv_validate_blocks_pipelined)" if world == 1 and not
                                        args.shard_protocol else f"block-range-shard{world}+allgather(68B/tx)"),
                           parse="host" if args.host_parse else "device",
                           block_split="serial" if args.no_presplit else "pipelined (next batch pre-split)"),
               value_basis=f"blocks resident in HBM, {NB} distinct batches rotated (PCIe-inclusive rate in "
                           f"pcie_inclusive)",
               verifies_per_s=round(all_verifies / el, 1), parity_vs_labels=ok,
               pcie_inclusive=pcie, latency_1block_ms=lat,
               kernel_ms=kavg,
               kernel_ms_source="HIP events: " + ", ".join(LIVE) + " live in the timed region; the rest from an "
                                "instrumented pass (fgv_set_timing) over the same batches",
               stage_ms=dict(sha=round(acc["sha"] / K, 4), prep=round(acc["prep"] / K, 4),
                             point=round(acc["point"] / K, 4)),
               sha256_compressions_per_step=int(acc["sha_blocks"] / K),
               host_ms=dict({k: round(v / K, 3) for k, v in host.items()},
                            **({"integrity_ms": round(integ["ms"] / K, 3)} if spec["integrity"] else {})),
               roofline=block_roofline(kavg, acc["pay_blocks"] / K, acc["verifies"] / K, batch_mb * 1e6,
                                       args.workload, (acc["sha_blocks"] - acc["pay_blocks"]) / K),
               key_tiers=dict(ids=kstats["ids"], comb=kstats["comb"], vb=kstats["vb"], promoted=kstats["promoted"],
                              vb_verifies_per_step=kstats["vb_verifies_last"]),
               cpu_baseline=None)
    if cpu is not None:
        rate, n, cel, nb = cpu["full"]
        r1, n1, c1, nb1 = cpu["full1"]
        crate, cn, ccel, cnb, cpar = cpu["c"]
        cr1, cn1, cc1, _, cpar1 = cpu["c1"]
        out["cpu_baseline"] = dict(
            value=round(crate, 1), unit="validated tx/s", cores=cpu["procs"], kind="port",
            sample=f"{cnb} blocks x {T} tx of this workload through the plain-C restated committer "
                   f"(oracle/cpu_validator.c: protobuf walk, registry lookup, SHA-256, Go DER + low-S + OpenSSL 3 "
                   f"P-256 Verify, OutOf fold, txid duplicates) on {cpu['procs']} threads in {ccel:.1f}s; 1 thread: "
                   f"{cr1:,.1f} tx/s ({cn1} tx in {cc1:.1f}s); flags equal to the generator's labels: {cpar and cpar1}; "
                   f"CPU {_cpu_model()}; a C restatement, not the Go peer (no Go toolchain on the box)",
            one_thread=round(cr1, 1), parity_vs_labels=bool(cpar and cpar1), cpu_model=_cpu_model())
        out["cpu_python_restatement"] = dict(
            value=round(rate, 1), unit="validated tx/s", cores=cpu["procs"], one_thread=round(r1, 1),
            sample=f"{nb} blocks through oracle/v20.py (the full restated v20 committer, the parity oracle) on "
                   f"{cpu['procs']} processes in {cel:.1f}s; 1 process: {n1} tx in {c1:.1f}s")
        vpt = acc["verifies"] / (B * T * K)
        from fabric_amd.synth.workloads import sig_pool
        pool = sig_pool(4096, seed=99, msg_len=1850)
        msgs = [m.tobytes() for m in pool["msgs"]]
        vr, vn, vel = cpu_verify_rate(pool["keymat"], msgs, pool["sigs"], cpu["procs"], args.cpu_seconds / 2)
        vr1, _, _ = cpu_verify_rate(pool["keymat"], msgs, pool["sigs"], 1, args.cpu_seconds / 4)
        out["cpu_crypto_bound"] = dict(
            value=round(vr / vpt, 1), unit="validated tx/s (identity.Verify only)", cores=cpu["procs"],
            one_thread=round(vr1 / vpt, 1),
            sample=f"{vn} identity.Verify (SHA-256 1.85KB + Go DER/low-S + OpenSSL P-256) in {vel:.1f}s = "
                   f"{vr:,.0f}/s on {cpu['procs']} threads, {vr1:,.0f}/s on 1, / {vpt:.2f} verifies per tx")
    if integ_ex is not None:
        for f in integ_fut.values():
            f.result()
        integ_ex.shutdown()
        out["integrity_pipeline"] = dict(depth=args.integ_depth, hash_threads_per_call=int(os.environ.get(
            "FGV_HASH_THREADS", "8")), note="VerifyBlock of the next batches runs on host threads while the "
                                             "committer validates this one; integrity_ms sums the calls' times")
    eng.close()
    return out


# ------------------------------------------------------------------ mvcc workload
# algorithmic HBM bytes per transaction: R x (16 B input + 64 B committed-
# table probe + 64 B write-table probe) + W x (8 B input + 64 B atomicMin line) + 2 B flags
MVCC_BYTES_PER_TX = 4 * (16 + 64 + 64) + 4 * (8 + 64) + 2


def run_mvcc(args, world, rank, local, dev):
    """C3: 10k-tx blocks against a 1M-key state DB, 5 % intra-block read->write conflicts,
    1 % stale reads, 0.5 % chains through invalid writers; blocks validated AND committed
    back to back (each block reads the state the previous one committed).  Replicas only:
    MVCC is sequential per channel, so every rank runs its own channel."""
    from fabric_amd import _lib
    from fabric_amd.synth import mvcc as M

    T, K, W = args.tx_per_mvcc_block, args.steps, args.warmup
    C = max(1, args.mvcc_chain)
    if C > 1:  # warm up with chain calls of the timed size (buffer sets of a C-block call allocated)
        W = max(W, C)
    t0 = time.time()
    st = M.MvccState(args.state_keys, seed=4 + rank, private_every=args.mvcc_private_every)
    keys, blk, txn = st.items()
    eng = _lib.Engine(local)
    eng.statedb_init(4 * args.state_keys, 64 << 20)
    eng.statedb_load("mycc", keys, blk, txn)
    if args.mvcc_private_every > 0:  # private-data keys: hashed namespace mycc$$hpvt
        hk, hb, ht = st.items_hashed()
        eng.statedb_load(M.HASHED_NS, hk, hb, ht)
    S = min(K, args.mvcc_single_steps) if C > 1 else 0  # the single-block pass after the chained one
    blocks = [M.make_block(st, T, number=1001 + i, seed=100 * rank + i) for i in range(W + K + S)]
    log(f"[bench] rank {rank}: {args.state_keys} keys + {W + K + S} x {T}-tx blocks ready in {time.time() - t0:.1f}s")
    sizes = [(len(b[0]) + 64 + 255) // 256 * 256 for b in blocks]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptr, o = [], 0
    for (b, _, _), sz in zip(blocks, sizes):
        arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        dptr.append(arena.data_ptr() + o)
        o += sz
    torch.cuda.synchronize()
    ok = True
    if C > 1:  # chain calls (the last one announces the first timed call's blocks for its pre-split)
        for i0 in range(0, W, C):
            i1 = min(i0 + C, W)
            nxt = [blocks[i][0] for i in range(i1, min(i1 + C, W + K))] if not args.no_presplit else None
            ws = _lib.MvccChainStep(eng, [blocks[i][0] for i in range(i0, i1)], range(1001 + i0, 1001 + i1),
                                    [blocks[i][2] for i in range(i0, i1)], commit=True, d_blocks=dptr[i0:i1],
                                    next_blocks=nxt)
            fl, rc, done = ws.run()
            _lib._check(rc)
            ok &= all(bool((f == blocks[i][1]).all()) for f, i in zip(fl, range(i0, i1)))
    else:
        for i in range(W):
            b, labels, flags = blocks[i]
            nb = blocks[i + 1][0] if not args.no_presplit else None
            ok &= bool((eng.mvcc_validate(b, 1001 + i, flags, commit=True, d_block=dptr[i], next_block=nb) == labels).all())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    lookup = total = 0.0
    rounds = []
    outs = []
    # C > 1: C consecutive blocks per fgv_mvcc_validate_blocks call (one device chain, block k+1's
    # extraction beside block k's checks and commit; a peer catching up holds many blocks);
    # C = 1: one fgv_mvcc_validate_block call per block, block i+1's framing walked on the engine's
    # host worker while block i validates (fgv_mvcc_validate_block_next)
    chains = []
    if C > 1:  # ctypes arguments bound once per call (as BlockStep does for the block workload)
        for i0 in range(W, W + K, C):
            i1 = min(i0 + C, W + K)
            # the next call's blocks are walked on the engine's host worker while this chain runs
            nxt = [blocks[i][0] for i in range(i1, min(i1 + C, W + K))] if not args.no_presplit else None
            chains.append((i1 - i0, _lib.MvccChainStep(eng, [blocks[i][0] for i in range(i0, i1)],
                                                       range(1001 + i0, 1001 + i1),
                                                       [blocks[i][2] for i in range(i0, i1)], commit=True,
                                                       d_blocks=dptr[i0:i1], next_blocks=nxt)))
    t0 = time.perf_counter()
    if C > 1:
        for nb, ch in chains:
            fl, rc, done = ch.run()
            _lib._check(rc)
            outs += fl  # (each chain object runs once)
            s = eng.mvcc_stats()
            total += s["total_ms"] * nb
            rounds.append(s["rounds"])
    else:
        for i in range(W, W + K):
            b, labels, flags = blocks[i]
            nb = blocks[i + 1][0] if i + 1 < W + K and not args.no_presplit else None
            outs.append(eng.mvcc_validate(b, 1001 + i, flags, commit=True, d_block=dptr[i], next_block=nb))
            s = eng.mvcc_stats()
            lookup += s["lookup_ms"]
            total += s["total_ms"]
            rounds.append(s["rounds"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    for i, f in zip(range(W, W + K), outs):
        ok &= bool((f == blocks[i][1]).all())
    single = None
    if S:  # per-block calls on the blocks that follow (latency of one block; untimed by the driver)
        t1 = time.perf_counter()
        for i in range(W + K, W + K + S):
            b, labels, flags = blocks[i]
            nb = blocks[i + 1][0] if i + 1 < W + K + S and not args.no_presplit else None
            ok &= bool((eng.mvcc_validate(b, 1001 + i, flags, commit=True, d_block=dptr[i], next_block=nb)
                        == labels).all())
        el1 = time.perf_counter() - t1
        single = dict(blocks=S, ms_per_block=round(el1 / S * 1e3, 3), tx_per_s=round(T * S / el1, 1))
    if world > 1:
        t = torch.tensor([el, 1.0 if ok else 0.0], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        mn = t.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        el, ok = float(mx[0]), bool(mn[1] > 0)
    per_block_ms = total / K
    mv_traffic, mv_src = pmc_traffic("mvcc")
    achieved = T * MVCC_BYTES_PER_TX / (per_block_ms / 1e3) / 1e9
    return dict(metric=METRIC, value=round(T * K * world / el, 1), unit="MVCC-validated tx/s", n_gpus=world, steps=K,
                dist=_dist_info(world),
                warmup=W, ms_per_step=round(el / K * 1e3, 3), higher_is_better=True, scaling="weak",
                vs_baseline=None, dtype="u64", data="synthetic",
                config=dict(workload=f"C3: {T}-tx blocks, {args.state_keys}-key state DB, 4R/4W, 5% intra-block "
                                     f"conflicts, 1% stale, 0.5% invalid-writer chains, commit per block"
                                     + (f", every {args.mvcc_private_every}th key private (hashed reads/writes)"
                                        if args.mvcc_private_every > 0 else "")
                                     + (f", {C} consecutive blocks per call (fgv_mvcc_validate_blocks)" if C > 1 else
                                        ", one call per block"),
                            parallelism=f"replicas{world} (sequential per channel)"),
                parity_vs_labels=ok, fixpoint_rounds=rounds, blocks_per_call=C, single_block_calls=single,
                stage_ms=dict(lookup=round(lookup / K, 4), gpu_total=round(per_block_ms, 4)),
                roofline=dict(bound="hbm", achieved=round(achieved, 2), peak=8000.0, unit="GB/s",
                              frac=round(achieved / 8000.0, 5), traffic=mv_traffic, traffic_source=mv_src,
                              kernel="MVCC GPU stages (per block)",
                              per_launch_bytes=T * MVCC_BYTES_PER_TX,
                              note="latency-bound: ~14 launches per 10k-tx block, one wait per call"),
                cpu_baseline=None)


# ------------------------------------------------------------------ sig workload
def run_sig(args, world, rank, local, dev):
    from fabric_amd import _lib
    from fabric_amd.synth.workloads import sig_pool

    n = args.per_gpu
    nkeys = args.sig_keys
    churn = nkeys > 16
    # churn: as many distinct messages as keys (every item its own key when --sig-keys >= per-gpu)
    uniq = min(n, max(16384, nkeys))
    pool = sig_pool(uniq, seed=1000 + rank, nkeys=min(nkeys, uniq))
    eng = _lib.Engine(local)
    # churn keys are registered cold (fgv_keys_register_tiered, hot=0): the variable-base kernels,
    # no 5.2 MB comb per key -- a signer population that each signs about once per batch
    slots_u = eng.keys_register(np.frombuffer(b"".join(k.pub for k in pool["keys"]), np.uint8).reshape(-1, 64),
                                hot=False if churn else None)
    kstats = eng.key_stats()
    idx = np.arange(n) % uniq
    msgs = np.ascontiguousarray(pool["msgs"][idx])
    msg_len = np.full(n, msgs.shape[1], np.uint32)
    msg_off = np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1])
    sa, so, sl = _lib.pack([pool["sigs"][i] for i in idx])
    slot = slots_u[pool["key_index"][idx]].astype(np.uint32)
    d_msg = torch.zeros(msgs.size + 64, dtype=torch.uint8, device=dev)
    d_msg[: msgs.size].copy_(torch.from_numpy(msgs.reshape(-1)))
    d_moff = torch.from_numpy(msg_off.view(np.int64).copy()).to(dev)
    d_mlen = torch.from_numpy(msg_len.view(np.int32).copy()).to(dev)
    d_sig = torch.zeros(sa.size + 64, dtype=torch.uint8, device=dev)
    d_sig[: sa.size].copy_(torch.from_numpy(sa.copy()))
    d_soff = torch.from_numpy(so.view(np.int64).copy()).to(dev)
    d_slen = torch.from_numpy(sl.view(np.int32).copy()).to(dev)
    d_slot = torch.from_numpy(slot.view(np.int32).copy()).to(dev)
    d_status = torch.zeros(n, dtype=torch.uint8, device=dev)
    gathered = torch.zeros(n * world, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def step():
        eng.verify_msgs_dev(d_msg.data_ptr(), d_moff.data_ptr(), d_mlen.data_ptr(), d_sig.data_ptr(),
                            d_soff.data_ptr(), d_slen.data_ptr(), d_slot.data_ptr(), n, d_status.data_ptr())
        if world > 1:
            dist.all_gather_into_tensor(gathered, d_status)
        return eng.timing()

    for _ in range(args.warmup):
        step()
    st = d_status.cpu().numpy()
    ok = bool(((st == 0) == pool["expect_valid"][idx]).all())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    acc = dict(point=0.0, prep=0.0, sha=0.0, vb=0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tm = step()
        acc["point"] += tm["point_ms"]
        acc["prep"] += tm["prep_ms"]
        acc["sha"] += tm["sha_ms"]
        acc["vb"] += tm["vb_mul_ms"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el, 1.0 if ok else 0.0], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        mn = t.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        el, ok = float(mx[0]), bool(mn[1] > 0)
    out = dict(metric=METRIC, value=round(n * world * args.steps / el, 1), unit="verifies/s", n_gpus=world,
               dist=_dist_info(world),
               steps=args.steps, warmup=args.warmup, ms_per_step=round(el / args.steps * 1e3, 3),
               higher_is_better=True, scaling="weak", vs_baseline=None, dtype="u32", data="synthetic",
               config=dict(workload=f"C4: P-256 SignedData batch, {n}/GPU, 1.85KB msgs, {min(nkeys, uniq)} keys"
                                    + (" (churn: registered cold, variable-base kernels)" if churn else "")
                                    + ", 1% tamper/0.5% high-S/0.5% bad DER/0.1% trailing",
                           global_batch=n * world, parallelism=f"shard{world}+allgather(1B/item)"),
               parity_vs_labels=ok,
               key_tiers=dict(comb=kstats["comb"], vb=kstats["vb"], promoted=eng.key_stats()["promoted"]),
               stage_ms=dict(sha=round(acc["sha"] / args.steps, 4), prep=round(acc["prep"] / args.steps, 4),
                             point=round(acc["point"] / args.steps, 4), vb_mul=round(acc["vb"] / args.steps, 4)),
               roofline=(roofline_vb(n, acc["vb"] / args.steps) if churn
                         else roofline(n, acc["point"] / args.steps, "sig")), cpu_baseline=None)
    if rank == 0 and world == 1 and args.cpu_threads > 0:
        rate, done, cel = cpu_verify_rate(pool["keymat"], [m.tobytes() for m in pool["msgs"]], pool["sigs"],
                                          args.cpu_threads)
        out["cpu_baseline"] = dict(value=round(rate, 1), unit="verifies/s", cores=args.cpu_threads, kind="port",
                                   sample=f"{done} C4-shaped identity.Verify (SHA-256 1.85KB + Go DER/low-S + "
                                          f"OpenSSL 3.0.2 P-256) in {cel:.1f}s on {args.cpu_threads} threads")
    eng.close()
    return out


# ------------------------------------------------------------------ end-to-end pipeline
def run_pipeline(args, world, rank, local, dev):
    """A peer's commit path on the same blocks, one step = one batch of B consecutive C2-shaped
    blocks (fabric_amd/synth/pipeline.py): committer validation (fgv_validate_blocks_pipelined,
    HBM-resident, the next batch pre-split) -> MVCC validation and commit of the B blocks in one
    device chain (fgv_mvcc_validate_blocks, the committer's flags in) -> the chained commit hashes
    (fgv_commit_hashes, host), the hashes of batch k computed on a host thread while batch k+1 is
    validated (they gate nothing: kv_ledger.go:806-817 chains them after the commit).  Reference:
    gossip/privdata/coordinator.go:152-184, core/ledger/kvledger/kv_ledger.go:612-652.  Every
    batch is distinct and processed once, in order, so each block reads the state the previous
    blocks committed.  Replicas for N > 1 (MVCC and the commit hash are sequential per channel)."""
    from concurrent.futures import ThreadPoolExecutor

    from fabric_amd import _lib, shard, txvalidator
    from fabric_amd.synth import blocks, pipeline
    from fabric_amd.synth.mvcc import MvccState

    B, T, W, K, L = args.blocks_per_gpu, args.tx_per_block, args.warmup, args.steps, args.pipeline_latency_blocks
    t0 = time.time()
    net = blocks.Network(seed=3, orgs=3, clients=100)
    st = MvccState(args.state_keys, seed=4 + rank)
    keys, kb, kt = st.items()
    batches, cexp, fexp, prev = [], [], [], b"\x00" * 32
    first = 1001
    for k in range(W + K):
        bl, c, f, prev = pipeline.make_blocks(net, st, B, T, first + k * B, seed=17 + k + 1000 * rank, prev_hash=prev)
        batches.append(bl), cexp.append(c), fexp.append(f)
    lat_blocks, lat_c, lat_f, _ = pipeline.make_blocks(net, st, L, T, first + (W + K) * B, seed=9999 + rank,
                                                       prev_hash=prev)
    log(f"[bench] rank {rank}: {args.state_keys} keys + {W + K} x {B} blocks x {T} tx (+{L} latency blocks) ready "
        f"in {time.time() - t0:.1f}s")
    eng = _lib.Engine(local, host_threads=args.host_threads or min(24, _cpu_share()))
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, hot_clients=True)
    eng.statedb_init(4 * args.state_keys, 256 << 20)
    eng.statedb_load("mycc", keys, kb, kt)
    dev_ub = not args.pipeline_host_hash
    eng.mvcc_set_update_bytes(dev_ub)
    allb = [bl for bl in batches] + [[b] for b in lat_blocks]
    sizes = [(len(b) + 64 + 255) // 256 * 256 for bl in allb for b in bl]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptrs, o = [], 0
    for bl in allb:
        cur = []
        for b in bl:
            arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
            cur.append(arena.data_ptr() + o)
            o += (len(b) + 64 + 255) // 256 * 256
        dptrs.append(cur)
    torch.cuda.synchronize()
    NBT = W + K
    hb = [eng.block_batch(batches[k], dptrs[k]) for k in range(NBT)]
    ntx = np.array([T] * B, dtype=np.int64)
    plan = shard.plan(ntx, 1, "block")
    rows = shard.plan_rows(*plan)
    send = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
    flags_out = np.empty(B * T, dtype=np.uint8)
    nums = [list(range(first + k * B, first + (k + 1) * B)) for k in range(NBT)]
    csteps = [_lib.BlockStep(eng, hb[k], plan[0][0], plan[1][0], send.data_ptr(), rows, ntx, 1, send.data_ptr(),
                             flags_out, plan=plan, presplit=True, next_batch=hb[(k + 1) % NBT], fused=True)
              for k in range(NBT)]
    msteps = [_lib.MvccChainStep(eng, batches[k], nums[k], [np.zeros(T, np.uint8)] * B, commit=True, d_blocks=dptrs[k],
                                 next_blocks=batches[k + 1] if k + 1 < NBT else None) for k in range(NBT)]
    hsteps = [_lib.CommitHashesDev(eng, batches[k], nums[k]) for k in range(NBT)]
    hash_ex = ThreadPoolExecutor(max_workers=1)
    state = dict(prev=b"", fut=None, mism=0, stage=np.zeros(3), futs={}, prevs={})

    def step(k, check):
        t = time.perf_counter()
        cf = csteps[k].validate() or csteps[k].finalize()
        t1 = time.perf_counter()
        msteps[k].set_flags([cf[b * T:(b + 1) * T] for b in range(B)])
        fl, rc, done = msteps[k].run()
        _lib._check(rc)
        ticket = eng.mvcc_last_ticket() if dev_ub else 0
        t2 = time.perf_counter()
        if state["fut"] is not None:
            state["prev"] = state["fut"].result()[-1]
        t3 = time.perf_counter()
        flc = [f.copy() for f in fl]
        state["fut"] = hash_ex.submit(hsteps[k].run, flc, state["prev"], ticket)
        state["futs"][k], state["prevs"][k] = state["fut"], state["prev"]
        state["stage"] += (t1 - t, t2 - t1, t3 - t2)
        if check:
            for b in range(B):
                state["mism"] += int((cf[b * T:(b + 1) * T] != cexp[k][b]).sum()) + int((fl[b] != fexp[k][b]).sum())

    for k in range(W):
        step(k, True)
    torch.cuda.synchronize()
    state["stage"][:] = 0
    t0 = time.perf_counter()
    for k in range(W, W + K):
        step(k, False)
    state["prev"] = state["fut"].result()[-1]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for k in range(W, W + K):  # parity of the timed batches after the clock: the final flags
        for b in range(B):     # (committer code, else MVCC code) of every block
            state["mism"] += int((msteps[k].flags[b] != fexp[k][b]).sum())
        # and the commit hashes against the host decode of the same blocks (fgv_commit_hashes)
        hh = _lib.commit_hashes(batches[k], fexp[k], nums[k], state["prevs"][k])
        state["mism"] += int(hh != state["futs"][k].result())
    stage = state["stage"] / K * 1e3
    # per-block latency: one block through all three stages, one call each (block in hand ->
    # final flags and commit hash), the state continuing from the timed batches
    lats = []
    prev = state["prev"]
    lat_h = [_lib.CommitHashesDev(eng, [b], [first + NBT * B + i], threads=1) for i, b in enumerate(lat_blocks)]
    for i, b in enumerate(lat_blocks):
        num = first + NBT * B + i
        torch.cuda.synchronize()
        t = time.perf_counter()
        cf = eng.validate_blocks([b], d_blocks=[dptrs[NBT + i][0]])[0]
        mf = eng.mvcc_validate(b, num, cf, commit=True, d_block=dptrs[NBT + i][0])
        prev = lat_h[i].run([mf], prev, eng.mvcc_last_ticket() if dev_ub else 0)[0]
        lats.append((time.perf_counter() - t) * 1e3)
        state["mism"] += int((cf != lat_c[i]).sum()) + int((mf != lat_f[i]).sum())
    hash_ex.shutdown()
    eng.close()
    ok = state["mism"] == 0
    if world > 1:
        tt = torch.tensor([el, 1.0 if ok else 0.0], dtype=torch.float64, device=dev)
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        mn = tt.clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        el, ok = float(mx[0]), bool(mn[1] > 0)
    return dict(metric=METRIC, value=round(world * B * T * K / el, 1), unit="committed tx/s (end to end)",
                n_gpus=world, steps=K, dist=_dist_info(world), warmup=W, ms_per_step=round(el / K * 1e3, 3),
                higher_is_better=True, scaling="weak", vs_baseline=None, dtype="u32", data="synthetic",
                config=dict(workload=f"commit pipeline: {B} x {T}-tx C2 blocks per step (OutOf(2,[Org1..3.member]), "
                                     f"C2 faults) -> MVCC of the same blocks against a {args.state_keys}-key state DB "
                                     f"(4R/4W x 200B read-modify-write, 1% stale, 5% conflicts, 2% reads of "
                                     f"committer-invalid writes) with commit -> chained commit hashes "
                                     f"({'host-built' if args.pipeline_host_hash else 'device-built'} update batches)",
                            blocks_per_step=B, tx_per_block=T, global_batch=world * B * T,
                            parallelism=f"replicas{world} (one channel per GPU)"),
                parity_vs_labels=ok,
                stage_ms_per_step=dict(committer=round(stage[0], 3), mvcc_chain=round(stage[1], 3),
                                       commit_hash_wait=round(stage[2], 3)),
                latency_1block_ms=dict(median=round(float(np.median(lats[2:])), 4) if len(lats) > 2 else None,
                                       p90=round(float(np.percentile(lats[2:], 90)), 4) if len(lats) > 2 else None,
                                       blocks=len(lats), note="one block in hand -> committer flags -> MVCC flags "
                                                              "and commit -> commit hash, one call each"),
                cpu_baseline=None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 40 timed steps: with 10 the pipeline's start-up was ~6 % of the C2 figure (MI355X, alternating:
    # 0.748 / 0.724 ms per step at 10 steps, 0.701 / 0.676 at 40; profiles/round3_ab/steps*)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="block", choices=["block", "c5", "sig", "mvcc", "pipeline"])
    ap.add_argument("--pipeline-latency-blocks", type=int, default=12,
                    help="pipeline: blocks taken one call per stage after the timed batches (latency)")
    ap.add_argument("--pipeline-host-hash", action="store_true",
                    help="pipeline: build the update batches on the host from the blocks (round 5) instead of "
                         "on the device (fgv_mvcc_set_update_bytes)")
    ap.add_argument("--c5-blocks-per-gpu", type=int, default=8)
    ap.add_argument("--c5-tx-per-block", type=int, default=20000)
    ap.add_argument("--tx-per-mvcc-block", type=int, default=10000)
    ap.add_argument("--state-keys", type=int, default=1_000_000)
    ap.add_argument("--mvcc-private-every", type=int, default=0,
                    help="C3 variant: every Nth key is private data (collection hashed rwsets)")
    ap.add_argument("--mvcc-chain", type=int, default=10,
                    help="C3: consecutive blocks per fgv_mvcc_validate_blocks call (1: one call per block)")
    ap.add_argument("--mvcc-single-steps", type=int, default=20,
                    help="C3 with --mvcc-chain > 1: blocks validated one call each after the timed pass (latency)")
    ap.add_argument("--blocks-per-gpu", type=int, default=32)
    ap.add_argument("--clients", type=int, default=0,
                    help="block workload: client identities (0: the workload's 100; e.g. 16000 = every creator "
                         "of a 16k-tx step about once: identity churn, client keys on the variable-base kernels)")
    ap.add_argument("--tx-per-block", type=int, default=500)
    ap.add_argument("--per-gpu", type=int, default=131072)
    ap.add_argument("--sig-keys", type=int, default=16,
                    help="C4: distinct signing keys (>16: churn, keys registered cold on the variable-base kernels)")
    ap.add_argument("--batches", type=int, default=6,
                    help="distinct blocks-per-gpu batches rotated through the timed loop (block workload)")
    ap.add_argument("--c5-batches", type=int, default=1)
    ap.add_argument("--integ-depth", type=int, default=2,
                    help="c5: batches whose VerifyBlock runs ahead of their validation (concurrent host calls)")
    ap.add_argument("--cpu-threads", type=int, default=-1,
                    help="CPU baseline processes/threads (-1: this rank's CPU share, 0: skip the baseline)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="wall time of each CPU baseline sample")
    ap.add_argument("--host-threads", type=int, default=0, help="fgv_config.host_threads (0: min(24, CPU share))")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host-resident) pass")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-block latency pass")
    ap.add_argument("--latency-reps", type=int, default=20)
    ap.add_argument("--host-parse", action="store_true", help="parse transactions on host threads (A/B)")
    ap.add_argument("--no-presplit", action="store_true", help="walk each batch's framing inside its validation call (A/B)")
    ap.add_argument("--presplit-early", dest="presplit_early", action="store_true", default=True,
                    help="pre-split batches k+2 and k+3 (fgv_presplit) when call k returns (default)")
    ap.add_argument("--no-presplit-early", dest="presplit_early", action="store_false",
                    help="only the pipelined call's own pre-split of its next batch (A/B)")
    ap.add_argument("--shard-protocol", action="store_true",
                    help="N=1 through the multi-GPU protocol (shard_dev + finalize_flags_dev) instead of the fused call")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (never set by the driver): several ranks on one GPU over gloo
    if os.environ.get("FGV_BENCH_SAME_DEVICE"):
        local = 0
    dev = torch.device("cuda", local)

    def dev_fn():  # the GPU is first touched here (the block workload forks CPU workers before)
        torch.cuda.set_device(local)
        return dev

    if world > 1:
        dev_fn()
        backend = os.environ.get("FGV_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if args.workload in ("block", "c5"):
        out = run_block(args, world, rank, local, dev_fn)
    else:
        if args.cpu_threads < 0:
            args.cpu_threads = _cpu_share()
        out = dict(sig=run_sig, mvcc=run_mvcc, pipeline=run_pipeline)[args.workload](args, world, rank, local, dev_fn())
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
