#!/usr/bin/env python3
"""Markdown table of a `bench.py --all-workloads` run: one row per JSON line
(stdout's headline and stderr's secondary lines, in one file), with the kernel
family, Gsamples/s, fraction of 8 TB/s, fraction of the same-box copy and the
PMC traffic ratio from a traffic.json (tools/pmc_traffic.py).

    python tools/bench_table.py <bench_all.log> [traffic.json]
"""
import json
import sys


def lines(path):
    out = []
    for ln in open(path, errors="replace"):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            out.append(json.loads(ln))
    return out


def main(path, traffic_path=None):
    traffic = json.load(open(traffic_path)) if traffic_path else {}
    print("| workload | kernel | Gsamples/s | of 8 TB/s | of same-box copy | traffic / alg. |")
    print("|---|---|---|---|---|---|")
    for d in lines(path):
        name = d["config"]["workload"].split(":")[0]
        r = d["roofline"]
        kern = r["kernel"].split(" grid")[0]
        fam = kern.split("<")[0]
        tags = [t for t in ("ch=1", "xg=1", "ip=1", "xl=1", "xl=2", "hillis", "self=1", "runs=1") if t in r["kernel"]]
        t = traffic.get(f"{name}:{d['config']['algo']}", {}).get("traffic_over_algorithmic")
        print(f"| {name} | {fam}{' ' + ','.join(tags) if tags else ''} | {d['value']:.0f} | {r['frac']:.3f} | "
              f"{r.get('frac_of_copy', float('nan')):.3f} | {t if t is not None else '—'} |")


if __name__ == "__main__":
    main(*sys.argv[1:3])
