#!/usr/bin/env python3
"""Build ome_kernels with extra compiler flags into another directory, for same-box A/B runs
(load it with OME_LIB_DIR=<dir>).  Example:
    python scripts/build_variant.py ome_amd/_lib_noslp -fno-slp-vectorize
The default libraries in ome_amd/_lib are not touched."""
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import build as b  # noqa: E402


def main():
    out, extra = Path(sys.argv[1]).resolve(), sys.argv[2:]
    b.OBJDIR = out / "obj"
    b.LIBDIR = out
    kdir = b.CSRC / "kernels"
    lib = b._build_lib("ome_kernels", sorted(kdir.glob("*.hip")), sorted(kdir.glob("*.h")), b._hipcc(),
                       b.HIP_FLAGS + extra, [], True, min(8, os.cpu_count() or 4))
    print(lib, lib.stat().st_size)


if __name__ == "__main__":
    main()
