#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / LDS / occupancy from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin or a file), one line per
kernel with the demangled name:

    hipcc ... -c --cuda-device-only -Rpass-analysis=kernel-resource-usage x.hip 2>&1 \\
        | python3 tools/resource_report.py [name-filter]
"""
import re
import subprocess
import sys


def parse(lines):
    out, cur = [], None
    for ln in lines:
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"\bSGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                         ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, ln)
            if m:
                cur[key] = int(m.group(1))
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def main():
    filt = sys.argv[1] if len(sys.argv) > 1 else ""
    ks = parse(sys.stdin)
    for k, dn in zip(ks, demangle([k["name"] for k in ks])):
        dn = re.sub(r"^void mavg::|\(mavg::\w+\)$", "", dn)
        if filt in dn:
            print(f"vgpr={k.get('vgpr', '?'):>3} scratch={k.get('scratch', '?'):>3} occ={k.get('occ', '?')}  {dn}")


if __name__ == "__main__":
    main()
