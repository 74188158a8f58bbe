"""Build provenance: a hash of every source liblcv.so is compiled from — csrc/ (HIP kernels, driver,
host units; the generated lcv_sop_programs.inc is represented by its generator tools/gen_sop.py),
include/lcv.h and the package Makefile.  The Makefile compiles it into the library (lcv_build_id) and
__graft_entry__.smoke() recomputes it from the tree it runs in: a prebuilt library that does not match
the pushed sources fails the smoke test instead of being measured.

    python tools/build_id.py            # print the 16-hex-digit id
    python tools/build_id.py --header F # write F (#define LCV_BUILD_ID "...") only if it changed
"""
from __future__ import annotations

import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-client-consensus-specs_amd")
GENERATED = {"lcv_sop_programs.inc"}


def sources() -> list:
    csrc = os.path.join(PKG, "csrc")
    files = [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))
             if f.endswith((".hip", ".hpp", ".inc", ".cpp", ".h")) and f not in GENERATED]
    files += [os.path.join(ROOT, "include", "lcv.h"), os.path.join(ROOT, "tools", "gen_sop.py"),
              os.path.join(PKG, "Makefile")]
    return files


def build_id() -> str:
    h = hashlib.sha256()
    for path in sources():
        rel = os.path.relpath(path, ROOT).replace(os.sep, "/")
        with open(path, "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


def main(argv) -> int:
    bid = build_id()
    if len(argv) == 3 and argv[1] == "--header":
        text = f'#pragma once\n#define LCV_BUILD_ID "{bid}"\n'
        try:
            with open(argv[2]) as f:
                if f.read() == text:
                    return 0
        except FileNotFoundError:
            pass
        with open(argv[2], "w") as f:
            f.write(text)
        return 0
    print(bid)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
