#!/usr/bin/env python3
"""One table of several tools/tune/wide_ab logs: per log, each variant's
fraction of 8 TB/s (mean and median of its per-launch events) and its check.

    python3 tools/tune/wab_summary.py gpurun_out/<tag>/wab_*.log
"""
import re
import sys

ROW = re.compile(r"^(?P<name>.*?)\s+mean (?P<ms>[0-9.]+) ms\s+(?P<mean>[0-9.]+)\s+median (?P<med>[0-9.]+)")


def summarize(path):
    head, rows, bad = None, [], []
    with open(path) as f:
        for line in f:
            if line.startswith("n=2^"):
                head = line.split(" (")[0].strip()
            elif "check:" in line and " 0 bad" not in line or "skipped" in line:
                bad.append(line.strip())
            else:
                m = ROW.match(line.rstrip())
                if m and head is not None:
                    rows.append((m["name"][:70], float(m["mean"]), float(m["med"])))
    return head, rows, bad


def main(paths):
    for p in paths:
        head, rows, bad = summarize(p)
        print(f"## {p}: {head}")
        for name, mean, med in rows:
            print(f"  {name:<72} {mean:.4f} {med:.4f}")
        for b in bad:
            print(f"  ! {b}")


if __name__ == "__main__":
    main(sys.argv[1:])
