#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes of `bench.py --all-workloads` into HBM bytes per
launch for each bench workload (profiles/traffic.json).

Recipe (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
collected in SEPARATE --pmc passes (they do not fit one pass); both are in
KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B streaming stores.  hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
Dispatches are matched to workloads by kernel family and grid size, the grid
being the one mavg_plan() reports for that workload (no GPU needed here).

    python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json>
"""
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        fam = re.sub(r"^void mavg::(\w+)<.*", r"\1", r["Kernel_Name"])
        key = (fam, int(r["Grid_Size"]))
        out.setdefault(key, []).append(float(r["Counter_Value"]))
    return out


def main(fetch_csv, write_csv, out_json):
    import bench
    import digital_signal_processsing_amd as dsp
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    fam_of = {"tile_scan": "tile_scan_kernel", "segment_scan": "scan_kernel", "direct": "direct_kernel",
              "naive": "naive_kernel"}
    result = {}
    for name, (n, k, C, dt, algo) in bench.WORKLOADS.items():
        dtc = dsp.F32 if dt == "f32" else dsp.I16
        plan = dsp.plan(n, k, C, dtc, algo)
        grid = int(re.search(r"grid=(\d+)", plan).group(1)) * int(re.search(r"block=(\d+)", plan).group(1))
        fam = fam_of[plan.split("<")[0]]
        f, w = fetch.get((fam, grid)), write.get((fam, grid))
        if not f or not w:
            continue
        fetch_b = 2 * statistics.median(f) * 1024
        write_b = statistics.median(w) * 1024
        alg = 2 * (4 if dt == "f32" else 2) * n
        result[f"{name}:{dsp.resolve_algo(n, k, C, dtc, algo)}"] = {
            "kernel": plan,
            "fetch_size_kib_median": statistics.median(f),
            "write_size_kib_median": statistics.median(w),
            "hbm_read_bytes_per_launch": fetch_b,
            "hbm_write_bytes_per_launch": write_b,
            "hbm_bytes_per_launch": fetch_b + write_b,
            "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 4),
            "dispatches": [len(f), len(w)],
            "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), WRITE_SIZE x1, KiB -> bytes",
        }
    json.dump(result, open(out_json, "w"), indent=1, sort_keys=True)
    for k, v in sorted(result.items()):
        print(f"{k:32s} traffic/alg = {v['traffic_over_algorithmic']}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
