"""Summarise rocprofv3 CSVs (tools/profile_round.sh output) into profiles/<round>_*.

usage: python tools/summarize_profiles.py gpurun_out/prof round1
Writes profiles/<round>_{block,sig,mvcc}_kernel_stats.csv (copies) and
profiles/<round>_profile_summary.md (per-kernel durations, VALU counters, HBM bytes).
"""
import collections
import csv
import json
import os
import shutil
import sys

SIMDS = 256 * 4          # MI355X: 256 CUs x 4 SIMDs
XCDS = 8
PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9   # 78.6 T full-rate 32-bit lane-ops/s
HBM_PEAK = 8.0e12


def norm(name):
    """kernel name without arguments, a leading 'void ' or template arguments"""
    k = name.split("(")[0]
    if k.startswith("void "):
        k = k[5:]
    return k.split("<")[0]


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[norm(r["Name"])] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                                            pct=float(r["Percentage"]))
    return out


def pmc(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    dur = collections.defaultdict(float)
    grid = {}
    seen = set()
    for r in csv.DictReader(open(path)):
        k = norm(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
        if (k, r["Dispatch_Id"]) not in seen:
            seen.add((k, r["Dispatch_Id"]))
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
            grid[k] = int(r["Grid_Size"])
    res = {}
    for k, v in agg.items():
        d = len([1 for kk, _ in seen if kk == k])
        res[k] = dict(dispatches=d, avg_s=dur[k] / max(d, 1), grid=grid[k],
                      **{c: x / max(d, 1) for c, x in v.items()})
    return res


def main(src, rnd):
    os.makedirs("profiles", exist_ok=True)
    lines = [f"# rocprofv3 summary — {rnd}", "",
             "Collected by `tools/profile_round.sh` (kernel-trace/stats runs and separate `--pmc` runs, "
             "as MI355X_MICROARCH.md prescribes).  Profiled runs clock lower than un-profiled ones "
             "(DVFS), so durations here read a few % above the bench's live HIP-event numbers.", ""]
    for wl in ("block", "sig", "mvcc", "sigchurn"):
        p = os.path.join(src, wl, "run_kernel_stats.csv")
        if not os.path.exists(p):
            continue
        # the per-step kernels only: the one-time comb-table builds (k_gtab per context, k_keytab
        # per new key) and key preparations (k_keyprep, k_kmap_set) are dropped, so the top row is the step's dominant kernel
        with open(p) as fi, open(f"profiles/{rnd}_{wl}_kernel_stats.csv", "w", newline="") as fo:
            rd = csv.DictReader(fi)
            wr = csv.DictWriter(fo, fieldnames=rd.fieldnames)
            wr.writeheader()
            rows = [r for r in rd if not r["Name"].startswith(("k_gtab", "k_keytab", "k_keybase", "k_keyprep", "k_kmap_set", "k_p384_tab", "k_p384_norm"))]
            tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
            for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
                r["Percentage"] = f"{100 * float(r['TotalDurationNs']) / tot:.2f}"
                wr.writerow(r)
        p = f"profiles/{rnd}_{wl}_kernel_stats.csv"
        js = os.path.join(src, wl + ".json")
        bench = json.load(open(js)) if os.path.exists(js) and os.path.getsize(js) else {}
        lines += [f"## {wl} workload", "", f"bench line (profiled run): value={bench.get('value')} {bench.get('unit')}, "
                  f"stage_ms={bench.get('stage_ms')}", "", "| kernel | calls | avg µs | % of GPU time |", "|---|---|---|---|"]
        for k, v in sorted(kernel_stats(p).items(), key=lambda kv: -kv[1]["pct"]):
            lines.append(f"| {k[:60]} | {v['calls']} | {v['avg_us']:.1f} | {v['pct']:.1f} |")
        lines.append("")
    for vname, title in (("pmc_valu", "sig workload: 131,072 verifies per dispatch"),
                         ("pmc_blk_valu", "block workload: one C2 step of 16k transactions"),
                         ("pmc_sigchurn_valu", "sig churn: 131,072 verifies, every item its own key")):
      p = os.path.join(src, vname, "run_counter_collection.csv")
      if os.path.exists(p):
        lines += [f"## VALU counters ({title})", "",
                  "| kernel | avg µs | VALU wave-insts | INT32 | INT64 | lane-ops/s | % of 78.6 T full-rate peak | VALU busy % |",
                  "|---|---|---|---|---|---|---|---|"]
        for k, v in pmc(p).items():
            if not k.startswith("k_"):
                continue
            lane = v.get("SQ_INSTS_VALU", 0) * 64 / v["avg_s"] if v["avg_s"] else 0
            gui = v.get("GRBM_GUI_ACTIVE", 0) / XCDS
            busy = 100 * v.get("SQ_ACTIVE_INST_VALU", 0) * 4 / SIMDS / gui if gui else 0
            lines.append(f"| {k} | {v['avg_s'] * 1e6:.1f} | {v.get('SQ_INSTS_VALU', 0):.4g} | "
                         f"{v.get('SQ_INSTS_VALU_INT32', 0):.3g} | {v.get('SQ_INSTS_VALU_INT64', 0):.3g} | {lane:.3g} | "
                         f"{100 * lane / PEAK_LANE_OPS:.1f} | {busy:.0f} |")
        kp = pmc(p).get("k_point28") if vname == "pmc_valu" else None
        if kp:
            gui = kp.get("GRBM_GUI_ACTIVE", 0) / XCDS
            cpi = gui * SIMDS / kp["SQ_INSTS_VALU"] if kp.get("SQ_INSTS_VALU") else 0
            lines += ["", f"k_point28: {kp.get('SQ_INSTS_VALU', 0) / (131072 / 64):,.0f} VALU instructions per verify "
                          f"(L = 1 at this batch size: one lane = one verify); {cpi:.2f} SIMD cycles per "
                          f"wave-instruction (issue-bound near 4).", ""]
        lines += ["VALU busy % = 100·SQ_ACTIVE_INST_VALU·4 / SIMDs / (GRBM_GUI_ACTIVE/8) (gfx94x formula; "
                  "ROCm 7.2 ships no gfx950 derived-counter section).", ""]
    for name, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE"), ("pmc_blk_fetch", "FETCH_SIZE"),
                      ("pmc_blk_write", "WRITE_SIZE")):
        p = os.path.join(src, name, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        blk = name.startswith("pmc_blk")
        lines += [f"## {ctr} ({'block' if blk else 'mvcc'} workload, per dispatch)", "",
                  "| kernel | avg µs | KB | GB/s |", "|---|---|---|---|"]
        for k, v in pmc(p).items():
            if not (k.startswith("k_bd") or k.startswith("k_point") or k in ("k_inv", "k_prep", "k_der")
                    if blk else k.startswith("k_mv")):
                continue
            kb = v.get(ctr, 0) * (2 if ctr == "FETCH_SIZE" else 1)  # gfx950: FETCH_SIZE reads 1/2
            lines.append(f"| {k} | {v['avg_s'] * 1e6:.1f} | {kb:.1f} | {kb * 1024 / v['avg_s'] / 1e9 if v['avg_s'] else 0:.1f} |")
        lines += ["", "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports ½ of wide streaming reads); "
                  "small gathers are uncalibrated; the MVCC 1M-key table (32 MB) and the comb tables of the block "
                  "workload (~70 MB) are Infinity-Cache resident.", ""]
    # HBM traffic per launch of each workload's dominant kernel (bench.py roofline.traffic):
    # FETCH_SIZE (doubled, gfx950) + WRITE_SIZE from the separate --pmc passes, KB -> bytes
    traffic = {}
    for wl, fe, wr, kern in (("block", "pmc_blk_fetch", "pmc_blk_write", "k_bd_sha_payload"),
                             ("block_point", "pmc_blk_fetch", "pmc_blk_write", "k_point28"),
                             ("block_parse", "pmc_blk_fetch", "pmc_blk_write", "k_bd_parse"),
                             ("sig", "pmc_sig_fetch", "pmc_sig_write", "k_point28"),
                             ("mvcc", "pmc_fetch", "pmc_write", None)):
        pf = os.path.join(src, fe, "run_counter_collection.csv")
        pw = os.path.join(src, wr, "run_counter_collection.csv")
        if not (os.path.exists(pf) and os.path.exists(pw)):
            continue
        F, W = pmc(pf), pmc(pw)
        if kern:
            if kern in F and kern in W:
                fb, wb = F[kern]["FETCH_SIZE"] * 2 * 1024, W[kern]["WRITE_SIZE"] * 1024
                traffic[wl] = dict(kernel=kern, fetch_bytes=round(fb), write_bytes=round(wb), hbm_bytes=round(fb + wb),
                                   avg_us=round(F[kern]["avg_s"] * 1e6, 1))
        else:  # MVCC: every per-block kernel (the one-time state load k_mv_tags excluded), per block
            # blocks: one k_mvx_prep per block on every path (the chain's extractions are grouped
            # since round 5, k_mvx_extract_multi walking several blocks per launch)
            nblk = F.get("k_mvx_prep", {}).get("dispatches", 0)
            per_block = [k for k in F if k.startswith("k_mv") and k != "k_mv_tags"]
            if nblk:
                fb = sum(F[k]["FETCH_SIZE"] * 2 * 1024 * F[k]["dispatches"] for k in per_block) / nblk
                wb = sum(W[k]["WRITE_SIZE"] * 1024 * W[k]["dispatches"] for k in per_block if k in W) / nblk
                rounds = F.get("k_mvx_round", {}).get("dispatches", 0) / nblk
                traffic[wl] = dict(kernels=sorted(per_block), fetch_bytes_per_block=round(fb),
                                   write_bytes_per_block=round(wb), hbm_bytes_per_block=round(fb + wb),
                                   hbm_bytes_per_block_low=round(fb / 2 + wb),
                                   blocks=nblk,
                                   note=f"sum over one C3 block's MVCC kernels (k_mvx_round x{rounds:.1f}); "
                                        "FETCH_SIZE x2 per MI355X_MICROARCH.md (exact for streaming reads) gives "
                                        "hbm_bytes_per_block, an upper bound: random row gathers read 128 B per "
                                        "row at a counter ratio of 1.0 (tools/fetch_calib.py, "
                                        "profiles/round6_fetch_calibration.md), so the counter unscaled "
                                        "(hbm_bytes_per_block_low) is the lower bound; the block's envelope bytes "
                                        "read by k_mvx_extract and the 1M-key table probes are included; "
                                        "k_mv_tags = the one-time state load")
    if traffic:
        json.dump(dict(round=rnd, source="rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, separate passes "
                                        "(tools/profile_round.sh)", workloads=traffic),
                  open(f"profiles/{rnd}_traffic.json", "w"), indent=1)
        lines += ["## HBM traffic per launch (bench.py roofline.traffic)", "", "```", json.dumps(traffic, indent=1), "```", ""]
    open(f"profiles/{rnd}_profile_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
