#!/usr/bin/env python3
"""Assemble a round's profile evidence from gpurun_out/<dir> (made by
scripts/gpu_round_profiles.sh): per bench line, the rocprofv3 kernel-trace
stats (copied), the bench JSON line, and FETCH_SIZE/WRITE_SIZE PMC bytes per
launch of each kernel (gfx950 correction, MI355X_MICROARCH.md §HBM:
FETCH_SIZE x 2, both in KB) merged into profiles/traffic.json under the
line's workload; plus a markdown summary.
usage: python tools/round_profiles.py gpurun_out/r3prof profiles/round3"""
import csv
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

SRC, DST = sys.argv[1], sys.argv[2]
TRAFFIC = "profiles/traffic.json"
LINES = ("cfg2", "cfg4", "cfg5", "cfg5classic", "cfg5soa", "cfg2soa", "cfg3x", "halo")
# rocprof kernel short name -> bench profiler name
NAMES = {"bin_count_kernel": "bin_count", "pack_coop_kernel": "pack", "pack_img_kernel": "pack",
         "pack_kernel": "pack", "pack_ranked_kernel": "pack_fine", "pack_fine_kernel": "pack_fine",
         "rank_ids_kernel": "count_ids", "count_ids_kernel": "count_ids",
         "msel_pack_kernel": "halo_pack", "msel_count_kernel": "halo",
         "scan_onepass_kernel": "scan", "pack_fields_kernel": "pack",
         "pack_coop_fields_kernel": "pack", "pack_fields_tile_kernel": "pack",
         "onepass_partition_kernel": "onepass"}


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


os.makedirs(DST, exist_ok=True)
traffic = json.load(open(TRAFFIC)) if os.path.exists(TRAFFIC) else {}
md = ["| line | kernel | calls | rocprof avg ms | bench HIP-event avg ms | alg bytes / launch | "
      "PMC HBM bytes / launch (read + write) | PMC / alg |", "|---|---|---|---|---|---|---|---|"]
for ln in LINES:
    d = os.path.join(SRC, f"{ln}_trace")
    stats = os.path.join(d, "run_kernel_stats.csv")
    if not os.path.exists(stats):
        continue
    shutil.copy(stats, os.path.join(DST, f"{ln}_kernel_stats.csv"))
    b = bench_line(os.path.join(SRC, f"{ln}_trace.log"))
    json.dump(b, open(os.path.join(DST, f"{ln}_bench.json"), "w"), indent=1)
    wl = b["config"]["workload"]
    pmc = pmc_summary.load(os.path.join(SRC, f"{ln}_*_SIZE", "pmc_counter_collection.csv"))
    rocp = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            k = pmc_summary.short(row["Name"])
            c0, t0 = rocp.get(k, (0, 0.0))
            rocp[k] = (c0 + int(row["Calls"]), t0 + float(row["TotalDurationNs"]) / 1e6)
    rocp = {k: (c, t / c) for k, (c, t) in rocp.items()}
    w = traffic.setdefault(wl, {})
    for k, c in sorted(pmc.items()):
        if k not in NAMES or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        bn = NAMES[k]
        if bn == "bin_count" and ln == "cfg5":
            bn = "bin_fine"
        rd, wr = c["FETCH_SIZE"] * 1024 * 2, c["WRITE_SIZE"] * 1024
        if bn != "scan":
            w[bn] = {"hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
                     "kernel": k, "correction": "FETCH_SIZE*1024*2 + WRITE_SIZE*1024",
                     "source": f"{DST}/{ln}_*"}
        kb = b["kernels"].get(bn, {})
        alg = kb.get("alg_bytes_per_launch")
        calls, avg = rocp.get(k, (0, 0.0))
        md.append(f"| {ln} | {k} ({bn}) | {calls} | {avg:.3f} | "
                  f"{kb.get('avg_ms', float('nan')):.3f} | "
                  f"{'%.3g' % alg if alg else '-'} | {rd + wr:.3g} ({rd:.3g} + {wr:.3g}) | "
                  f"{'%.2f' % ((rd + wr) / alg) if alg else '-'} |")
json.dump(traffic, open(TRAFFIC, "w"), indent=1)
open(os.path.join(DST, "summary.md"), "w").write("\n".join(md) + "\n")
print("\n".join(md))
