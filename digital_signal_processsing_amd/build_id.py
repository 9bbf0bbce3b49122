#!/usr/bin/env python3
"""Source id of libmavg: a SHA-256 over the sources the library is compiled
from (csrc/*.hip, csrc/*.hpp, csrc/Makefile, include/*.h), in name order.

csrc/Makefile runs this script and links the id into the library
(`mavg_build_id()`, include/mavg.h); `__graft_entry__.build()`, `smoke()` and
tests/test_abi.py compare the loaded library's id with the tree's, so a
prebuilt library linked from other sources is caught.  The Makefile also makes
every object depend on a stamp named after this id and a hash of the compile
flags, so objects are recompiled whenever either changes (stale objects with
newer mtimes are not relinked under a fresh id).  The id names the sources
only: the release, debug and hooks libraries share it and differ in flags.
Plain Python, no imports beyond the standard library (the Makefile runs it)."""
from __future__ import annotations

import glob
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)


def source_files(root: str = ROOT) -> list:
    csrc = os.path.join(root, "digital_signal_processsing_amd", "csrc")
    files = (glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))
             + [os.path.join(csrc, "Makefile")] + glob.glob(os.path.join(root, "include", "*.h")))
    return sorted(files, key=lambda p: os.path.relpath(p, root))


def source_id(root: str = ROOT) -> str:
    """16 hex digits of SHA-256(relative name, NUL, bytes, NUL for every source)."""
    h = hashlib.sha256()
    for p in source_files(root):
        h.update(os.path.relpath(p, root).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_id())
