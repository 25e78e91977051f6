"""Hash of the sources that make the ICP path's kernels and their launches (bench.py, tools/pmc_traffic.py).

profiles/pmc_traffic.json is stamped with the sha256 of the profiled library AND with this hash: the
library hash changes with any source of the .so (GICP, the map, ego velocity), this one only with
the ICP kernels, their host-side launch code, the headers they include and the build flags — a PMC
row stays valid for a library rebuilt after a change elsewhere (bench.py names which hash matched).
"""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "icp-4dradar_amd")


def icp_source_files() -> list[str]:
    files = [os.path.join(PKG, "Makefile"), os.path.join(PKG, "csrc", "icp4r_kernels.hip"),
             os.path.join(PKG, "csrc", "icp4r_capi.cpp")]
    files += sorted(glob.glob(os.path.join(PKG, "csrc", "*.hpp")))
    files += sorted(glob.glob(os.path.join(ROOT, "include", "icp4r", "*.h")))
    return files


def icp_sources_sha256() -> str | None:
    h = hashlib.sha256()
    try:
        for p in icp_source_files():
            with open(p, "rb") as f:
                data = f.read()
            h.update(os.path.relpath(p, ROOT).encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    except OSError:
        return None
    return h.hexdigest()
