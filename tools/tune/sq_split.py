#!/usr/bin/env python3
"""Wave-cycle split of the dominant kernel in each rocprofv3 SQ pass of
tools/gpu/r05_sq_pass.sh: per workload, the medians over its dispatches of
SQ_ACTIVE_INST_VALU / _LDS / _ANY, SQ_WAIT_ANY and SQ_WAIT_INST_ANY as
fractions of SQ_WAVE_CYCLES (all quad-cycle counts, MI355X_MICROARCH.md), and
VALU instructions per sample.

    python3 tools/tune/sq_split.py gpurun_out/<tag>
"""
import collections
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main(root):
    import bench
    print("| workload | kernel | VALU active | LDS active | any active | waiting | issue-stalled | VALU insts / sample |")
    print("|---|---|---|---|---|---|---|---|")
    for d in sorted(glob.glob(os.path.join(root, "sq_*/"))):
        name = os.path.basename(d.rstrip("/"))[3:]
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f[0])):
            if r["Kernel_Name"].startswith("void mavg::") and "synth" not in r["Kernel_Name"] and "copy" not in r["Kernel_Name"]:
                per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        kern = max(per, key=lambda kk: len(per[kk]["SQ_WAVE_CYCLES"]))
        m = {c: statistics.median(v) for c, v in per[kern].items()}
        wc = m["SQ_WAVE_CYCLES"]
        n = bench.WORKLOADS[name][0]
        print(f"| {name} | {kern.split('<')[0].replace('void mavg::', '')} | {m['SQ_ACTIVE_INST_VALU'] / wc:.3f} | "
              f"{m['SQ_ACTIVE_INST_LDS'] / wc:.3f} | {m['SQ_ACTIVE_INST_ANY'] / wc:.3f} | {m['SQ_WAIT_ANY'] / wc:.3f} | "
              f"{m['SQ_WAIT_INST_ANY'] / wc:.3f} | {m['SQ_INSTS_VALU'] * 64 / n:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
