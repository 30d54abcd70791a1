#!/usr/bin/env python3
"""SQ/TA/TCC counter summary of the bench lines (profiles/<round>/sq_summary.md).

Input: the rocprofv3 --pmc passes of scripts/gpu_pmc.sh (OUT=<line>
PASSES=sq: gpurun_out/pmc_<line>/pass*_counter_collection.csv)
and the bench JSON lines that tools/round_profiles.py copied next to the
output (<line>_bench.json: algorithmic bytes per launch of each kernel).
Per kernel and dispatch: wave cycles, the share of them spent waiting
(SQ_WAIT_ANY) and waiting for an instruction's operands (SQ_WAIT_INST_ANY),
VMEM instructions, algorithmic bytes per VMEM instruction (a full 64-lane
16-byte wave instruction moves 1024 B), LDS bank-conflict cycles over active
LDS cycles, VALU instructions.

usage: python tools/sq_summary.py gpurun_out profiles/round4
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

# rocprof kernel short name -> bench profiler name (as tools/round_profiles.py)
NAMES = {"bin_count_kernel": "bin_count", "pack_coop_kernel": "pack", "pack_img_kernel": "pack",
         "pack_kernel": "pack", "pack_ranked_kernel": "pack_fine", "rank_ids_kernel": "count_ids",
         "count_ids_kernel": "count_ids", "msel_pack_kernel": "halo_pack",
         "msel_count_kernel": "halo", "scan_onepass_kernel": "scan", "pack_fields_kernel": "pack",
         "pack_coop_fields_kernel": "pack", "pack_fields_tile_kernel": "pack",
         "onepass_partition_kernel": "onepass"}

SRC, DST = sys.argv[1], sys.argv[2]
# scripts/gpu_pmc.sh OUT=<line> PASSES=sq writes gpurun_out/pmc_<line>/
LINES = tuple((ln, f"pmc_{ln}") for ln in ("cfg2", "cfg5", "cfg5classic", "cfg5soa", "cfg2soa",
                                           "halo"))


def main():
    out = ["| line | kernel | wave cycles | SQ_WAIT_ANY / wave cycles | SQ_WAIT_INST_ANY / wave cycles "
           "| VMEM rd instr | VMEM wr instr | alg bytes per VMEM instr | LDS bank-conflict / active "
           "LDS cycles | VALU instr |", "|---|---|---|---|---|---|---|---|---|---|"]
    for line, sub in LINES:
        pattern = os.path.join(SRC, sub, "pass*_counter_collection.csv")
        d = pmc_summary.load(pattern)
        if not d:
            continue
        bench = {}
        bj = os.path.join(DST, f"{line}_bench.json")
        if os.path.exists(bj):
            bench = (json.load(open(bj)) or {}).get("kernels", {})
        for k, c in sorted(d.items()):
            if "SQ_WAVE_CYCLES" not in c or c.get("SQ_WAVES", 0) < 1 or k not in NAMES:
                continue   # this library's kernels only (not the input generators, torch, RCCL)
            wc = c["SQ_WAVE_CYCLES"]
            rd, wr = c.get("SQ_INSTS_VMEM_RD", 0.0), c.get("SQ_INSTS_VMEM_WR", 0.0)
            name = ("bin_fine" if line.startswith("cfg5") and k == "bin_count_kernel"
                    else NAMES.get(k, ""))
            alg = bench.get(name, {}).get("alg_bytes_per_launch")
            bpi = f"{alg / (rd + wr):.0f}" if alg and rd + wr else "--"
            lds = c.get("SQ_ACTIVE_INST_LDS", 0.0)
            conf = f"{c.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds:.2f}" if lds else "--"
            out.append(f"| {line} | {k} | {wc:.3g} | {c.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
                       f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {rd:.3g} | {wr:.3g} | {bpi} | "
                       f"{conf} | {c.get('SQ_INSTS_VALU', 0):.3g} |")
    os.makedirs(DST, exist_ok=True)
    with open(os.path.join(DST, "sq_summary.md"), "w") as f:
        f.write("# SQ counter summary (per dispatch, rocprofv3 --pmc, 3 passes per line; "
                "scripts/gpu_pmc.sh PASSES=sq)\n\n")
        f.write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
