#!/usr/bin/env python3
"""Reproduce bench.py's roofline fraction from a rocprofv3 kernel trace of the
SAME command.

bench.py times W warm-up + K measured launches of the workload's kernel with
HIP events and reports frac = algorithmic bytes / mean launch time / 8 TB/s.
This script takes the --kernel-trace CSV of that run, selects the dispatches
of exactly that kernel (full template signature + grid, rebuilt from the
mavg_plan() string in the bench line), drops the first W, keeps the next K
(the timed ones), and recomputes the same statistic from the profiler's own
timestamps.

    python tools/roofline_trace.py <kernel_trace.csv> <bench_line.json|log> <out.json> [--warmup W --steps K]
"""
import argparse
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from pmc_traffic import kernel_key, plan_key  # noqa: E402


def bench_line(path):
    """The headline JSON line of a bench log (first line starting with '{' whose metric is the headline)."""
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            if "roofline" in d:
                return d
    raise SystemExit(f"no bench JSON line in {path}")


def select(trace, plan, warmup, steps):
    key = plan_key(plan)
    grid = int(re.search(r"grid=(\d+)", plan).group(1)) * int(re.search(r"block=(\d+)", plan).group(1))
    rows = []
    for r in csv.DictReader(open(trace)):
        g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        if kernel_key(r["Kernel_Name"]) == key and g == grid:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    if len(rows) < warmup + steps:
        raise SystemExit(f"trace has {len(rows)} dispatches of {plan}, need warmup {warmup} + steps {steps}")
    return rows, rows[warmup:warmup + steps]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("out")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    a = ap.parse_args()
    b = bench_line(a.bench)
    roof = b["roofline"]
    warmup = b["warmup"] if a.warmup is None else a.warmup
    steps = b["steps"] if a.steps is None else a.steps
    allrows, timed = select(a.trace, roof["kernel"], warmup, steps)
    dur_ns = [e - s for s, e in timed]
    mean_ms = statistics.mean(dur_ns) / 1e6
    med_ms = statistics.median(dur_ns) / 1e6
    alg = roof["algorithmic_bytes_per_launch"]
    frac = alg / (mean_ms * 1e-3) / (roof["peak"] * 1e9)
    res = {
        "kernel": roof["kernel"],
        "dispatches_in_trace": len(allrows),
        "timed_dispatches": len(timed),
        "skipped_warmup": warmup,
        "durations_us": [round(d / 1e3, 2) for d in dur_ns],
        "mean_ms": round(mean_ms, 4),
        "median_ms": round(med_ms, 4),
        "min_ms": round(min(dur_ns) / 1e6, 4),
        "algorithmic_bytes_per_launch": alg,
        "peak_gbs": roof["peak"],
        "frac_from_trace_mean": round(frac, 4),
        "frac_from_trace_median": round(alg / (med_ms * 1e-3) / (roof["peak"] * 1e9), 4),
        "bench_frac": roof["frac"],
        "bench_kernel_avg_ms": roof["kernel_avg_ms"],
        "trace_over_bench_mean": round(mean_ms / roof["kernel_avg_ms"], 4),
        "bench_value": b["value"],
        "bench_cmd_steps_warmup": [b["steps"], b["warmup"]],
    }
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "durations_us"}, indent=1))


if __name__ == "__main__":
    main()
