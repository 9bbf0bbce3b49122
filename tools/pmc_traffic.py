#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes of `bench.py --all-workloads` into HBM bytes per
launch for each bench workload (profiles/traffic.json).

Recipe (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
collected in SEPARATE --pmc passes (they do not fit one pass); both are in
KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B streaming stores.  hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
Dispatches are matched to workloads by the kernel's full template signature
and grid size, both rebuilt from the plan string mavg_plan() reports for that
workload (no GPU needed here).  Several workloads share a grid (carry_2p30 and
both int16 lines launch 131072 workgroups), so the family and grid alone are
not enough.

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


TYPE = {"f32": "float", "f64": "double", "i16": "short", "i32": "int", "i64": "long"}
FAMILY = {"tile_scan": "tile_scan_kernel", "direct": "direct_kernel",
          "naive": "naive_kernel", "ahead_scan": "ahead_scan_kernel",
          "wide_tile": "wide_tile_kernel", "wide_ahead": "wide_ahead_kernel", "chan_tile": "chan_tile_kernel"}


def kernel_key(name):
    """'void mavg::tile_scan_kernel<float, double, 1, 4, 8, false, 0, false, 256>(...)'
    -> ('tile_scan_kernel', ('float', 'double', '1', ...))"""
    m = re.match(r"^void mavg::(\w+)<([^>]*)>", name)
    if not m:
        return None
    return m.group(1), tuple(a.strip() for a in m.group(2).split(","))


def plan_key(plan):
    """The kernel_key() a launch with this mavg_plan() string produces."""
    fam, rest = plan.split("<", 1)
    fields = rest.split(">", 1)[0].split(",")
    T, acc = TYPE[fields[0]], TYPE[fields[1].split("=")[1]]
    kv = dict(f.split("=") for f in fields[2:] if "=" in f)
    flavour = [f for f in fields[2:] if "=" not in f]
    hs = "true" if flavour and flavour[0] == "hillis" else "false"
    wg = re.search(r"block=(\d+)", plan).group(1)
    if fam == "tile_scan":
        args = (T, acc, kv["C"], kv["F"], kv["U"], hs, kv["nt"], wg, "true" if kv.get("rc", "1") == "1" else "false",
                kv.get("dv", "0"), "true" if kv.get("dma", "0") == "1" else "false")
    elif fam == "direct":
        args = (T, acc, kv["C"], kv["F"], kv["U"], wg, kv.get("nt", "0"))
    elif fam == "ahead_scan":
        b = {"0": "false", "1": "true"}
        args = (T, acc, kv["C"], kv["F"], kv["U"], kv["nt"], b[kv["rc"]], b[kv["dma"]], b[kv["wrec"]], kv["dv"], hs,
                "true" if " runs=1" in plan else "false", wg)
    elif fam == "wide_tile":
        args = (T, acc, kv["C"], kv["P"], kv["U"], wg, kv["nt"], kv.get("dv", "0"))
    elif fam == "chan_tile":
        args = (T, acc, kv["C"], kv["Q"], wg, kv["nt"], kv.get("dv", "0"), "true" if kv.get("xg", "0") == "1" else "false",
                "true" if kv.get("ip", "0") == "1" else "false", kv.get("xl", "0"))
    elif fam == "wide_ahead":
        args = (T, acc, kv["C"], kv["P"], kv["U"], wg, kv["nt"], kv.get("dv", "0"), kv["F"], kv["FU"],
                "true" if kv.get("ch", "0") == "1" else "false", "true" if kv.get("xg", "0") == "1" else "false",
                kv.get("mw", "0"), kv.get("xl", "0"))
    else:
        args = (T, acc)
    return FAMILY[fam], args


def per_kernel(path, counter):
    """(kernel key, grid) -> counter values in dispatch order."""
    out = {}
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        kk = kernel_key(r["Kernel_Name"])
        if kk is None:
            continue
        out.setdefault((kk, int(r["Grid_Size"])), []).append(float(r["Counter_Value"]))
    return out


def run_order(workloads, first="headline"):
    """bench.py --all-workloads runs `first`, then the others sorted by name."""
    return [first] + [w for w in sorted(workloads) if w != first]


def split_shared(values, names, name):
    """Workloads whose launches share a kernel signature and grid (e.g. long_1m
    and long_4m: the same 8192-frame look-ahead kernel) ran one after the other
    with the same number of launches: the name's own contiguous share."""
    if len(names) <= 1 or len(values) % len(names) != 0:
        return values
    m = len(values) // len(names)
    i = names.index(name)
    return values[i * m:(i + 1) * m]


def main(fetch_csv, write_csv, out_json):
    import bench
    import digital_signal_processsing_amd as dsp
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    result = {}
    keys = {}
    for name in run_order(bench.WORKLOADS):
        n, k, C, dt, algo = bench.WORKLOADS[name]
        plan = dsp.plan(n, k, C, dsp.F32 if dt == "f32" else dsp.I16, algo)
        grid = int(re.search(r"grid=(\d+)", plan).group(1)) * int(re.search(r"block=(\d+)", plan).group(1))
        keys[name] = (plan_key(plan), grid)
    for name, (n, k, C, dt, algo) in bench.WORKLOADS.items():
        dtc = dsp.F32 if dt == "f32" else dsp.I16
        plan = dsp.plan(n, k, C, dtc, algo)
        key = keys[name]
        sharing = [w for w in run_order(bench.WORKLOADS) if keys[w] == key]
        f, w = fetch.get(key), write.get(key)
        if not f or not w:
            continue
        f, w = split_shared(f, sharing, name), split_shared(w, sharing, name)
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
