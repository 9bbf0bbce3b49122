#!/usr/bin/env python3
"""HBM traffic per launch of each tuner variant measured by
tools/gpu/r05_footprint_pmc.sh (one variant per process, FETCH_SIZE and
WRITE_SIZE in separate passes).  The variant's kernel is the one with the most
dispatches in its run among the library's kernels (1 + 10 launches; the
input fill runs once; the runtime's workspace memsets are not counted); bytes =
(2 x FETCH_SIZE + WRITE_SIZE) KiB, the gfx950 correction tools/pmc_traffic.py
applies, over the algorithmic 2 x 4 B per fp32 sample of 2^30 samples.

    python3 tools/tune/pmc_variants.py gpurun_out/<tag> [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

ALG = 2 * 4 * (1 << 30)


def counter(path_dir, name):
    files = glob.glob(os.path.join(path_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None, None
    by_kernel = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                by_kernel[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    ours = [kk for kk in by_kernel if kk.startswith("void mavg::") and "synth_kernel" not in kk]
    kern = max(ours, key=lambda kk: len(by_kernel[kk]))
    vals = [v for _, v in sorted(by_kernel[kern])]
    return kern, statistics.median(vals[1:] if len(vals) > 1 else vals)  # the first launch: cold


def main(root, out_json=None):
    rows = []
    for tsv in sorted(glob.glob(os.path.join(root, "k*_variants.tsv"))):
        k = int(re.search(r"k(\d+)_variants", tsv).group(1))
        for line in open(tsv):
            i, name = line.rstrip("\n").split("\t", 1)
            kf, fetch = counter(os.path.join(root, f"k{k}_v{i}_FETCH_SIZE"), "FETCH_SIZE")
            kw, write = counter(os.path.join(root, f"k{k}_v{i}_WRITE_SIZE"), "WRITE_SIZE")
            if fetch is None or write is None:
                continue
            assert kf == kw, (kf, kw)
            b = (2 * fetch + write) * 1024
            rows.append({"k": k, "variant": name, "kernel": kf.split("(")[0], "fetch_size_kib": fetch,
                         "write_size_kib": write, "hbm_bytes_per_launch": b,
                         "traffic_over_algorithmic": round(b / ALG, 4)})
    print("| k | variant | 2 x FETCH (GB) | WRITE (GB) | traffic / alg. |")
    print("|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['k']} | {r['variant']} | {2 * r['fetch_size_kib'] * 1024 / 1e9:.3f} | "
              f"{r['write_size_kib'] * 1024 / 1e9:.3f} | {r['traffic_over_algorithmic']} |")
    if out_json:
        json.dump(rows, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[2] if len(a) > 2 and a[1] == "--json" else None)
