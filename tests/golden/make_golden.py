#!/usr/bin/env python3
"""Generate the committed golden fixtures of the store path (test infrastructure).

There is no buildable or importable reference for this path (SURVEY.md §8(c):
mc-oblivious and the enclave handler are absent from /root/reference), so the
expected outputs come from this repo's own CPU restatement (oracle/, the
seqmodel and its cluster form).  The fixtures freeze that restatement: the
CPU suite checks the oracle still reproduces them byte for byte, and the GPU
suite checks the HIP engine against them without running the oracle.

Each fixture holds the config, the request batches (payloads cut to 8
random bytes so the files stay small), the expected response slabs and the
live message / mailbox counts after every batch.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from grapevine_amd import abi  # noqa: E402
from oracle import ffi  # noqa: E402

CASES = {
    # name: (config kwargs, seed, gen params kwargs, batch sizes)
    "single_mixed": (dict(msg_capacity=4096, mailbox_partitions=16, mailbox_partition_slots=32,
                          max_batch=1024), 0x67766f31,
                     dict(n_identities=120, hard_error=3, zero_recipient=3, hot=40),
                     [600, 600, 600, 600, 1]),
    "single_full": (dict(msg_capacity=256, mailbox_partitions=4, mailbox_partition_slots=16,
                         max_batch=1024), 0x67766f32,
                    dict(create=70, read=10, update=10, delete=10, n_identities=80),
                    [400, 400, 400]),
    "sharded4": (dict(msg_capacity=4096, mailbox_partitions=16, mailbox_partition_slots=32,
                      max_batch=1024, shard_count=4), 0x67766f33,
                 dict(n_identities=200, hard_error=2, zero_recipient=2),
                 [2000, 2000]),
}


def config_of(kw):
    kw = dict(kw)
    n = kw.pop("msg_capacity")
    return abi.make_config(n, **kw)


def trim(reqs):
    reqs = reqs.copy()
    reqs["payload"][:, 8:] = 0
    return reqs


def make(name):
    kw, seed, pkw, sizes = CASES[name]
    cfg = config_of(kw)
    model = ffi.Cluster(cfg) if kw.get("shard_count", 0) > 1 else ffi.Model(cfg)
    model.seed(seed)
    p = ffi.gen_params(**pkw)
    reqs, resps, counts = [], [], []
    for n in sizes:
        r = trim(model.gen_batch(n, p))
        o = model.process_batch(r)
        assert o is not None
        reqs.append(r)
        resps.append(o)
        counts.append((model.messages, model.mailboxes))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, config=json.dumps(kw), sizes=np.array(sizes),
                        requests=np.concatenate(reqs).view(np.uint8),
                        responses=np.concatenate(resps).view(np.uint8),
                        counts=np.array(counts, dtype=np.uint64))
    return path


def main():
    manifest = {}
    for name in CASES:
        path = make(name)
        manifest[os.path.basename(path)] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
