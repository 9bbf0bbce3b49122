#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV, so
each bench workload's kernel can be compared with bench.py's HIP-event
timing (the --stats table merges launches of one kernel across grid sizes).

    python tools/prof_summary.py <run_kernel_trace.csv> <out.csv>
"""
import csv
import statistics
import sys


def main(trace, out):
    rows = list(csv.DictReader(open(trace)))
    groups = {}
    for r in rows:
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]), r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"])
        groups.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_threads", "workgroup", "lds", "vgpr", "sgpr", "calls", "avg_us", "median_us",
                    "min_us", "max_us"])
        for (k, g, wg, lds, vg, sg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, g, wg, lds, vg, sg, len(d), round(statistics.mean(d) / 1e3, 2),
                        round(statistics.median(d) / 1e3, 2), round(min(d) / 1e3, 2), round(max(d) / 1e3, 2)])
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
