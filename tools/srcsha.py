"""Fingerprint of the engine's sources (grapevine_amd/csrc/*, include/*.h).

A side figure that bench.py attaches to its line (PMC traffic per launch,
VALU instructions per launch, the sharded-step prediction) is recorded with
the fingerprint of the sources it was measured on; bench.py attaches it only
when the fingerprint equals the tree's ("What's weak" 4, 8).
"""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha(root=ROOT):
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(root, "grapevine_amd", "csrc", "*"))
                   + glob.glob(os.path.join(root, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
