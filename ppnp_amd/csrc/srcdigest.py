#!/usr/bin/env python3
"""Digest of the HIP sources of libppnp_amd.so (*.hip and *.h in this directory, and the ABI
header include/ppnp_amd.h they compile against: basename and bytes, sorted by path).  The Makefile compiles it into the library (appnp_build_info), and
bench.py computes it from the tree it runs in: a library built from other sources shows as a
mismatch in the bench line, and the committed PMC traffic is keyed by it.  Standard library
only, so the build needs no package import."""

import glob
import hashlib
import os
import sys


def src_digest(directory: str = os.path.dirname(os.path.abspath(__file__))) -> str:
    h = hashlib.sha1()
    abi = os.path.join(directory, "..", "..", "include", "ppnp_amd.h")
    for p in sorted(glob.glob(os.path.join(directory, "*.hip"))
                    + glob.glob(os.path.join(directory, "*.h"))
                    + ([os.path.normpath(abi)] if os.path.exists(abi) else [])):
        with open(p, "rb") as fh:
            h.update(os.path.basename(p).encode() + fh.read())
    return h.hexdigest()[:12]


if __name__ == "__main__":
    sys.stdout.write(src_digest(*sys.argv[1:]) + "\n")
