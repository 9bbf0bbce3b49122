#!/usr/bin/env python3
"""Table of tools/gpu/r06_far_pmc.sh: per (k, variant) the medians over its
launches (the first, cold, dropped) of FETCH_SIZE, WRITE_SIZE, the L2's
memory-side read requests (TCC_EA0_RDREQ, and the ones destined for DRAM,
TCC_EA0_RDREQ_DRAM -- the Infinity Cache sits behind that path, so its hits
are inside this count too) and their sizes (32 / 64 / 128 B), as bytes per
launch over the algorithmic 8 B per fp32 sample of 2^30 samples.

    python3 tools/tune/pmc_far.py gpurun_out/<tag> [--json out.json]
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
GROUPS = [["FETCH_SIZE"], ["WRITE_SIZE"], ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum"],
          ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"]]


def counters(path_dir, names):
    """{counter: median over the variant's kernel launches (first dropped)}"""
    files = glob.glob(os.path.join(path_dir, "**", "*counter_collection.csv"), recursive=True)
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in names:
                by[r["Kernel_Name"]][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    ours = [kk for kk in by if kk.startswith("void mavg::") and "synth_kernel" not in kk]
    if not ours:
        return None, {}
    kern = max(ours, key=lambda kk: max(len(v) for v in by[kk].values()))
    out = {}
    for c, vals in by[kern].items():
        v = [x for _, x in sorted(vals)]
        out[c] = statistics.median(v[1:] if len(v) > 1 else v)
    return kern.split("(")[0], out


def main(root, out_json=None):
    rows = []
    for tsv in sorted(glob.glob(os.path.join(root, "k*_selected.tsv")), key=lambda p: int(re.search(r"k(\d+)_", p).group(1))):
        k = int(re.search(r"k(\d+)_selected", tsv).group(1))
        for line in open(tsv):
            i, name = line.rstrip("\n").split("\t", 1)
            vals, kern = {}, None
            for g, names in enumerate(GROUPS):
                kk, v = counters(os.path.join(root, f"k{k}_v{i}_g{g}"), names)
                kern = kern or kk
                vals.update(v)
            if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
                continue
            fetch_b = 2 * vals["FETCH_SIZE"] * 1024
            write_b = vals["WRITE_SIZE"] * 1024
            sized = sum(vals.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) * s for s in (32, 64, 128))
            rows.append({"k": k, "variant": name, "kernel": kern, "fetch_x2_bytes": fetch_b, "write_bytes": write_b,
                         "traffic_over_algorithmic": round((fetch_b + write_b) / ALG, 4),
                         "rdreq": vals.get("TCC_EA0_RDREQ_sum"), "rdreq_dram": vals.get("TCC_EA0_RDREQ_DRAM_sum"),
                         "rdreq_sized_bytes": sized,
                         "rdreq_32b": vals.get("TCC_EA0_RDREQ_32B_sum"), "rdreq_64b": vals.get("TCC_EA0_RDREQ_64B_sum"),
                         "rdreq_128b": vals.get("TCC_EA0_RDREQ_128B_sum")})
    print("| k | variant | 2 x FETCH (GB) | WRITE (GB) | traffic / alg. | RDREQ_DRAM / RDREQ | "
          "sized read bytes (GB) |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        ratio = (r["rdreq_dram"] / r["rdreq"]) if r["rdreq"] else float("nan")
        print(f"| {r['k']} | {r['variant']} | {r['fetch_x2_bytes'] / 1e9:.3f} | {r['write_bytes'] / 1e9:.3f} | "
              f"{r['traffic_over_algorithmic']} | {ratio:.4f} | {r['rdreq_sized_bytes'] / 1e9:.3f} |")
    if out_json:
        json.dump(rows, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[2] if len(a) > 2 and a[1] == "--json" else None)
