"""Print one step's kernel sequence from a rocprofv3 kernel-trace CSV: start
offset, the idle gap before each kernel and its duration (us).  A step is the
span between two launches of the kernel named by --anchor (its last launch
of the step).  Builder's tool; reads only the CSV.

    python tools/step_timeline.py gpurun_out/r5prof/halo_trace/run_kernel_trace.csv --anchor msel_pack
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="pack_coop")
    ap.add_argument("--which", type=int, default=-2, help="step index among anchor launches")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit(f"fewer than two '{a.anchor}' launches")
    lo, hi = idx[a.which - 1], idx[a.which]
    t0 = int(rows[lo + 1]["Start_Timestamp"])
    prev = int(rows[lo]["End_Timestamp"])
    busy = 0
    for r in rows[lo + 1: hi + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0]
        print(f"{(s - t0) / 1e3:9.1f}  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  "
              f"{name[-70:]}")
        busy += e - s
        prev = e
    span = int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])
    print(f"step {span / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
