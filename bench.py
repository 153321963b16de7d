"""bench.py -- MI355X block-validation engine for Hyperledger Fabric's committer.

python bench.py --gpus N --steps K --warmup W [--workload block|sig]

block (default; BASELINE configs[1], C2 shape): 500-tx endorser blocks, 2-of-3 endorsement
  policy (OutOf(2, Org1..3.member)), 60 % of txs with 2 endorsements / 40 % with 3, 4 reads +
  4 writes of 200 B values, 100 client identities, injected faults (2 % bad creator sig, 2 %
  one bad endorsement of 3, 2 % policy unsatisfied, 0.5 % duplicate txid).  Weak scaling:
  every GPU owns --blocks-per-gpu blocks' worth of transactions; the batch of N x B blocks is
  resident in every GPU's HBM, each rank validates its transaction-index shard of every block
  (fgv_validate_shard: host parse + GPU SHA-256 + ECDSA-P256 + policy fold), the ranks
  all-gather their 68-byte per-tx records over RCCL and finalize TxValidationFlags.
  value = validated tx/s over all ranks (max-over-ranks wall time of the timed steps).

sig (configs[3], C4 shape): 131,072 P-256 identity.Verify calls per GPU on 1.85 KB
  messages, inputs resident in HBM; value = verifies/s.
"""
import argparse
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
# 32x32->64 multiply-add products per verify in the comb: ~42.5 terms (16 signed
# 16-bit generator windows + their carry window, nonzero about every other verify, + 26 signed
# 10-bit key windows), the first one loaded, so 41 mixed additions (rounded down) x (8 field
# mults x 64 + 3 squarings x 36 products) + the projective x-check (3 x 64)
PRODUCTS_POINT = 41 * (8 * 64 + 3 * 36) + 3 * 64
# chip-wide v_mad_u64_u32 issue rate measured by tools/valu_peak.hip (profiles/round1_valu_peak.json)
PEAK_MAD_PER_S = float(os.environ.get("FGV_PEAK_MAD", "3.106e13"))


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
        return t["hbm_bytes"], f"{os.path.basename(files[-1])}: {t['kernel']} fetch {t['fetch_bytes']} B + write {t['write_bytes']} B"
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


def run_block(args, world, rank, local, dev):
    import threading

    from fabric_amd import _lib, shard, txvalidator
    from fabric_amd.synth import blocks

    spec = BLOCK_SPECS[args.workload]
    t0 = time.time()
    pems = None
    if world > 1:
        obj = [None]
        if rank == 0:
            obj[0] = blocks.Network(**spec["net"]).export_pems()
        dist.broadcast_object_list(obj, src=0)
        pems = obj[0]
    net = blocks.Network(pems=pems, **spec["net"])
    B, T = args.blocks_per_gpu, args.tx_per_block
    if args.workload == "c5":
        B = args.c5_blocks_per_gpu
        T = args.c5_tx_per_block
    mine, prev = [], b"\x00" * 32
    for i in range(B):  # each rank's blocks form a hash chain (numbers 1 + rank*B + i)
        num = 1 + rank * B + i
        blk, lab, envs = blocks.make_block(net, T, number=num, seed=7919 * rank + i, threads=8,
                                           endorse_dist=spec["endorse"], prev_hash=prev)
        mine.append((blk, lab))
        prev = blocks.header_hash(num, prev, envs)
    my_blocks = [m[0] for m in mine]
    my_labels = [m[1] for m in mine]
    # The batch is every rank's blocks in rank order.  With at least one block per rank the
    # shard plan is block-granular (below): a rank needs only its own blocks' bytes -- the
    # others' results arrive as all-gathered records -- so only the labels (for the parity
    # check) are exchanged; the per-block transaction split needs every block everywhere.
    plan_mode = "block" if B >= 1 else "tx"
    if world > 1:
        allb = [None] * world
        dist.all_gather_object(allb, (my_blocks if plan_mode == "tx" else None, my_labels))
        labels = [l for r in range(world) for l in allb[r][1]]
        if plan_mode == "tx":
            blks = [b for r in range(world) for b in allb[r][0]]
        else:
            blks = [my_blocks[i] if r == rank else b"" for r in range(world) for i in range(B)]
    else:
        blks, labels = my_blocks, my_labels
    log(f"[bench] rank {rank}: {len(blks)} blocks x {T} tx ready in {time.time() - t0:.1f}s")

    eng = _lib.Engine(local)
    if args.host_parse:
        eng.set_parse_mode(1)
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
    # the batch resident in HBM (64 B tail padding per block)
    sizes = [(len(b) + 64 + 255) // 256 * 256 for b in blks]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptr, o = [], 0
    for b, sz in zip(blks, sizes):
        if len(b):  # (other ranks' blocks are empty placeholders under the block plan)
            arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        dptr.append(arena.data_ptr() + o)
        o += sz
    ntx = np.array([T] * len(blks), dtype=np.int64)
    # contiguous transaction ranges of the batch (fabric_amd/shard.py): on block boundaries, a
    # rank splits and parses only its own blocks
    plan = shard.plan(ntx, world, plan_mode)
    lo, hi = plan[0][rank], plan[1][rank]
    rows = shard.plan_rows(*plan)
    # records stay in HBM: shard validation -> all-gather (RCCL) -> device finalize
    send = torch.zeros((rows, shard.REC), dtype=torch.uint8, device=dev)
    recv = torch.zeros((world * rows, shard.REC), dtype=torch.uint8, device=dev) if world > 1 else send
    batch = eng.block_batch(blks, dptr)
    flags_out = np.empty(int(ntx.sum()), dtype=np.uint8)
    torch.cuda.synchronize()

    integ = dict(ms=0.0, ok=True)

    def verify_mine():  # deliver-side VerifyBlock of this rank's blocks (own host pool)
        chain = _lib.ChainState(number=rank * B, valid=1, has_hash=0)
        t = time.perf_counter()
        res = eng.blocks_verify(my_blocks, chain)
        integ["ms"] += (time.perf_counter() - t) * 1e3
        integ["ok"] &= all(r[0] == _lib.BLK_OK for r in res) and chain.number == rank * B + B

    # every ctypes argument bound once (fabric_amd._lib.BlockStep); the pre-split of the next
    # batch (here: the same blocks) overlaps this batch's all-gather + finalize, as a peer
    # splits block k+1 while block k commits
    bs = _lib.BlockStep(eng, batch, lo, hi, send.data_ptr(), rows, ntx, world, recv.data_ptr(), flags_out,
                        plan=plan, presplit=not args.no_presplit)

    def step():
        th = None
        if spec["integrity"]:  # concurrent with the committer pass, as in a pipelined peer
            th = threading.Thread(target=verify_mine)
            th.start()
        bs.validate()
        if world > 1:
            shard.allgather_device(send, recv)
        f = bs.finalize()
        if th is not None:
            th.join()
        return f

    flags = None
    for _ in range(args.warmup):
        flags = step()
    exp = np.array([e if e is not None else 255 for bl in labels for e in blocks.expected_codes(bl)], np.int64)
    known = np.array([e is not None for bl in labels for e in blocks.expected_codes(bl)])
    mism = int(((flags.astype(np.int64) != exp) & known).sum()) if flags is not None else -1
    if not integ["ok"]:
        mism = max(mism, 1)
        log(f"[bench] rank {rank}: block integrity check failed")
    integ["ms"] = 0.0
    if mism:
        log(f"[bench] rank {rank}: {mism} flags differ from generator labels")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    acc = dict(point=0.0, prep=0.0, sha=0.0, verifies=0, sha_blocks=0)
    host = dict(parse_ms=0.0, assemble_ms=0.0, device_ms=0.0, fold_ms=0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        tm, cn = bs.stats()
        for k, v in zip(("parse_ms", "assemble_ms", "device_ms", "fold_ms"), tm[4:]):
            host[k] += v
        acc["sha"] += tm[0]
        acc["prep"] += tm[1]
        acc["point"] += tm[2]
        acc["sha_blocks"] += cn[1]
        acc["verifies"] += cn[2]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
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
    total_tx = len(blks) * T * args.steps
    out = dict(metric=METRIC, value=round(total_tx / el, 1), unit="validated tx/s", n_gpus=world, steps=args.steps,
               warmup=args.warmup, ms_per_step=round(el / args.steps * 1e3, 3), higher_is_better=True, scaling="weak",
               vs_baseline=None, dtype="u32", data="synthetic",
               config=dict(workload=spec["desc"].format(T=T),
                           blocks_per_step=len(blks), tx_per_block=T, global_batch=len(blks) * T,
                           parallelism=f"{plan_mode}-range-shard{world}+allgather(68B/tx)",
                           parse="host" if args.host_parse else "device",
                           block_split="serial" if args.no_presplit else "pipelined (fgv_presplit)"),
               verifies_per_s=round(all_verifies / el, 1), parity_vs_labels=ok,
               stage_ms=dict(sha=round(acc["sha"] / args.steps, 4), prep=round(acc["prep"] / args.steps, 4),
                             point=round(acc["point"] / args.steps, 4)),
               sha256_compressions_per_step=int(acc["sha_blocks"] / args.steps),
               host_ms=dict({k: round(v / args.steps, 3) for k, v in host.items()},
                            **({"integrity_ms": round(integ["ms"] / args.steps, 3)} if spec["integrity"] else {})),
               roofline=roofline(acc["verifies"] / args.steps, acc["point"] / args.steps, args.workload), cpu_baseline=None)
    if rank == 0 and world == 1 and args.cpu_threads > 0:
        # crypto-bound upper bound of the reference's CPU committer on this host: every
        # verify is SHA-256(msg) + Go-rule DER + low-S + OpenSSL P-256 (what identity.Verify
        # costs), divided by the verifies per transaction of this workload
        from fabric_amd.synth.workloads import sig_pool
        pool = sig_pool(4096, seed=99, msg_len=1850)
        rate, n, cel = cpu_verify_rate(pool["keymat"], [m.tobytes() for m in pool["msgs"]], pool["sigs"],
                                       args.cpu_threads)
        vpt = acc["verifies"] / (len(blks) * T * args.steps)
        out["cpu_baseline"] = dict(value=round(rate / vpt, 1), unit="validated tx/s (crypto-bound upper bound)",
                                   cores=args.cpu_threads, kind="port",
                                   sample=f"{n} identity.Verify (SHA-256 1.85KB + Go DER/low-S + OpenSSL P-256) in "
                                          f"{cel:.1f}s on {args.cpu_threads} threads = {rate:,.0f} verifies/s, / "
                                          f"{vpt:.2f} verifies per tx; parse/policy cost not included")
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
    t0 = time.time()
    st = M.MvccState(args.state_keys, seed=4 + rank, private_every=args.mvcc_private_every)
    keys, blk, txn = st.items()
    eng = _lib.Engine(local)
    eng.statedb_init(4 * args.state_keys, 64 << 20)
    eng.statedb_load("mycc", keys, blk, txn)
    if args.mvcc_private_every > 0:  # private-data keys: hashed namespace mycc$$hpvt
        hk, hb, ht = st.items_hashed()
        eng.statedb_load(M.HASHED_NS, hk, hb, ht)
    blocks = [M.make_block(st, T, number=1001 + i, seed=100 * rank + i) for i in range(W + K)]
    log(f"[bench] rank {rank}: {args.state_keys} keys + {W + K} x {T}-tx blocks ready in {time.time() - t0:.1f}s")
    sizes = [(len(b[0]) + 64 + 255) // 256 * 256 for b in blocks]
    arena = torch.zeros(sum(sizes), dtype=torch.uint8, device=dev)
    dptr, o = [], 0
    for (b, _, _), sz in zip(blocks, sizes):
        arena[o:o + len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
        dptr.append(arena.data_ptr() + o)
        o += sz
    torch.cuda.synchronize()
    ok = True
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
    # block i+1's framing is walked on the engine's host worker while block i validates
    # (fgv_mvcc_validate_block_next; a peer has the next block in hand while it commits this one)
    t0 = time.perf_counter()
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
                warmup=W, ms_per_step=round(el / K * 1e3, 3), higher_is_better=True, scaling="weak",
                vs_baseline=None, dtype="u64", data="synthetic",
                config=dict(workload=f"C3: {T}-tx blocks, {args.state_keys}-key state DB, 4R/4W, 5% intra-block "
                                     f"conflicts, 1% stale, 0.5% invalid-writer chains, commit per block"
                                     + (f", every {args.mvcc_private_every}th key private (hashed reads/writes)"
                                        if args.mvcc_private_every > 0 else ""),
                            parallelism=f"replicas{world} (sequential per channel)"),
                parity_vs_labels=ok, fixpoint_rounds=rounds,
                stage_ms=dict(lookup=round(lookup / K, 4), gpu_total=round(per_block_ms, 4)),
                roofline=dict(bound="hbm", achieved=round(achieved, 2), peak=8000.0, unit="GB/s",
                              frac=round(achieved / 8000.0, 5), traffic=mv_traffic, traffic_source=mv_src,
                              kernel="MVCC GPU stages (per block)",
                              per_launch_bytes=T * MVCC_BYTES_PER_TX,
                              note="latency-bound: ~14 launches + 2 host syncs per 10k-tx block"),
                cpu_baseline=None)


# ------------------------------------------------------------------ sig workload
def run_sig(args, world, rank, local, dev):
    from fabric_amd import _lib
    from fabric_amd.synth.workloads import sig_pool

    n = args.per_gpu
    uniq = min(n, 16384)
    pool = sig_pool(uniq, seed=1000 + rank)
    eng = _lib.Engine(local)
    slots_u = eng.keys_register(np.frombuffer(b"".join(k.pub for k in pool["keys"]), np.uint8).reshape(-1, 64))
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
    acc = dict(point=0.0, prep=0.0, sha=0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tm = step()
        acc["point"] += tm["point_ms"]
        acc["prep"] += tm["prep_ms"]
        acc["sha"] += tm["sha_ms"]
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
               steps=args.steps, warmup=args.warmup, ms_per_step=round(el / args.steps * 1e3, 3),
               higher_is_better=True, scaling="weak", vs_baseline=None, dtype="u32", data="synthetic",
               config=dict(workload="C4: P-256 SignedData batch, 131072/GPU, 1.85KB msgs, 16 keys, "
                                    "1% tamper/0.5% high-S/0.5% bad DER/0.1% trailing",
                           global_batch=n * world, parallelism=f"shard{world}+allgather(1B/item)"),
               parity_vs_labels=ok,
               stage_ms=dict(sha=round(acc["sha"] / args.steps, 4), prep=round(acc["prep"] / args.steps, 4),
                             point=round(acc["point"] / args.steps, 4)),
               roofline=roofline(n, acc["point"] / args.steps, "sig"), cpu_baseline=None)
    if rank == 0 and world == 1 and args.cpu_threads > 0:
        rate, done, cel = cpu_verify_rate(pool["keymat"], [m.tobytes() for m in pool["msgs"]], pool["sigs"],
                                          args.cpu_threads)
        out["cpu_baseline"] = dict(value=round(rate, 1), unit="verifies/s", cores=args.cpu_threads, kind="port",
                                   sample=f"{done} C4-shaped identity.Verify (SHA-256 1.85KB + Go DER/low-S + "
                                          f"OpenSSL 3.0.2 P-256) in {cel:.1f}s on {args.cpu_threads} threads")
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="block", choices=["block", "c5", "sig", "mvcc"])
    ap.add_argument("--c5-blocks-per-gpu", type=int, default=8)
    ap.add_argument("--c5-tx-per-block", type=int, default=20000)
    ap.add_argument("--tx-per-mvcc-block", type=int, default=10000)
    ap.add_argument("--state-keys", type=int, default=1_000_000)
    ap.add_argument("--mvcc-private-every", type=int, default=0,
                    help="C3 variant: every Nth key is private data (collection hashed rwsets)")
    ap.add_argument("--blocks-per-gpu", type=int, default=32)
    ap.add_argument("--tx-per-block", type=int, default=500)
    ap.add_argument("--per-gpu", type=int, default=131072)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--host-parse", action="store_true", help="parse transactions on host threads (A/B)")
    ap.add_argument("--no-presplit", action="store_true", help="walk each batch's framing inside its validation call (A/B)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (never set by the driver): several ranks on one GPU over gloo
    if os.environ.get("FGV_BENCH_SAME_DEVICE"):
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("FGV_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    out = dict(block=run_block, c5=run_block, sig=run_sig, mvcc=run_mvcc)[args.workload](args, world, rank, local, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
