#!/usr/bin/env python3
"""Per-wave table of the PMC passes tools/pmc_long.sh collects (one directory
per <workload>_<group>, rocprofv3 CSV inside): counters of the scan kernels
only (the tuner's synth / copy kernels are skipped), averaged over dispatches.

    python tools/pmc_table.py gpurun_out/pmc_r02 [out.txt]
"""
import collections
import csv
import glob
import os
import sys

PER_WAVE = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
            "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
            "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_ANY"]


def load(root):
    res = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        tag = os.path.basename(os.path.dirname(f)).rsplit("_", 1)[0]
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if "ahead_scan" not in kn and "tile_scan" not in kn:
                continue
            res[tag]["kernel"] = kn.split("(")[0].replace("void mavg::", "")
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for c, v in agg.items():
            res[tag][c] = sum(v) / len(v)
    return res


def main(root, out=None):
    res = load(root)
    tags = sorted(res)
    lines = ["# per-dispatch means; per-wave rows divide by SQ_WAVES (rocprofv3 --pmc, tools/pmc_long.sh)"]
    for t in tags:
        lines.append(f"# {t}: {res[t].get('kernel')}")
    lines.append("%-28s" % "counter" + "".join("%14s" % t for t in tags))
    counters = sorted({c for t in tags for c in res[t] if c != "kernel"})
    for c in counters:
        lines.append("%-28s" % c + "".join("%14.4g" % res[t].get(c, float("nan")) for t in tags))
    lines.append("per wave:")
    for c in PER_WAVE:
        lines.append("%-28s" % c + "".join("%14.1f" % (res[t].get(c, float("nan")) / res[t].get("SQ_WAVES", 1))
                                           for t in tags))
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:3])
