"""The engine's source stamp: sha256 over csrc/*.hip, csrc/*.h and
include/lpg.h (sorted by file name; each file's base name, then its bytes),
first 16 hex digits.

The Makefile compiles this stamp into liblpg.so (``lpg_build_stamp()``);
``_lib.load()`` refuses a library whose stamp differs from the sources next to
it (a stale prebuilt binary must not run silently), and
bench.py attaches a PMC traffic file only at the same stamp.

    python3 linearprogramming_amd/_stamp.py [ROOT]   -> prints the stamp
"""
from __future__ import annotations

import glob
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root: str = ROOT) -> list:
    csrc = os.path.join(root, "linearprogramming_amd", "csrc")
    return sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")) +
                  [os.path.join(root, "include", "lpg.h")])


def source_stamp(root: str = ROOT) -> str:
    h = hashlib.sha256()
    for f in source_files(root):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_stamp(sys.argv[1] if len(sys.argv) > 1 else ROOT))
