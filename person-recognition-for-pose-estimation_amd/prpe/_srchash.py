"""Source hash of libprpe.so: sha256 over the files it is built from (csrc/*.hip, csrc/*.h,
include/prpe.h, in name order, each as name + bytes). build.py compiles it into the library
(``prpe_source_hash``); ``_lib.lib()`` recomputes it from the sources beside the library and
refuses a library built from other sources. No dependencies (build.py loads this file alone)."""
from __future__ import annotations

import glob
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
CSRC = os.path.join(PKG, "csrc")
HEADER = os.path.join(os.path.dirname(PKG), "include", "prpe.h")


def source_files() -> list[str]:
    fs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")))
    return fs + [HEADER]


def source_hash() -> str | None:
    """Hex sha256 of the library's sources, or None when they are not present."""
    files = source_files()
    if not os.path.isdir(CSRC) or not os.path.exists(HEADER):
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
