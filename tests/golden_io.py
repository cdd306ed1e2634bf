"""Loader of the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py from the CPU restatement)."""
import json
import os

import numpy as np

from grapevine_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ("single_mixed", "single_full", "sharded4")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False
    kw = json.loads(str(z["config"]))
    n = kw.pop("msg_capacity")
    cfg = abi.make_config(n, **kw)
    sizes = [int(x) for x in z["sizes"]]
    reqs = z["requests"].view(abi.REQUEST_DTYPE)
    resps = z["responses"].view(abi.RESPONSE_DTYPE)
    counts = [tuple(int(v) for v in c) for c in z["counts"]]
    batches, o = [], 0
    for k, s in enumerate(sizes):
        batches.append((reqs[o:o + s], resps[o:o + s], counts[k]))
        o += s
    return cfg, batches
