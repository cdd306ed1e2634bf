#!/usr/bin/env python3
"""Run a fixed schedule of batches with a chosen request mix (run under
rocprofv3 by tests/test_oblivious.py).  The prefill is identical for every
mix; only the last `--batches` batches differ.  Test infrastructure: the
oracle only generates realistic requests against the live state."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from grapevine_amd import abi  # noqa: E402
from grapevine_amd.store import ObliviousStore  # noqa: E402
from oracle import ffi  # noqa: E402

MIXES = {
    "main": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "all_create": dict(create=100, read=0, update=0, delete=0),
    "all_miss_read": dict(create=0, read=100, update=0, delete=0, nxt=0, miss=100),
    "hot_next": dict(create=30, read=35, update=0, delete=35, nxt=100, hot=100),
    "deletes": dict(create=0, read=0, update=0, delete=100, nxt=30),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("mix", choices=sorted(MIXES))
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--batches", type=int, default=3)
    p.add_argument("--auth", action="store_true", help="authenticated storage (DESIGN.md §8)")
    a = p.parse_args()
    cfg = abi.make_config(1 << a.log2n, max_batch=a.batch, auth_storage=a.auth)
    store = ObliviousStore(cfg)
    model = ffi.Model(cfg)
    model.seed(77)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=5000)
    for _ in range(4):
        reqs = model.gen_batch(a.batch, fill)
        model.process_batch(reqs)
        store.process_batch(reqs)
    model.seed(1234)  # same request-generator state for every mix
    params = ffi.gen_params(n_identities=5000, bad_auth=0, bad_recipient=0, hard_error=0,
                            zero_recipient=0, **{"miss": 0, **MIXES[a.mix]})
    for _ in range(a.batches):
        reqs = model.gen_batch(a.batch, params)
        want = model.process_batch(reqs)
        got = store.process_batch(reqs)
        assert got.tobytes() == want.tobytes(), "parity failure inside the probe"
    store.synchronize()
    print("probe ok", a.mix, store.stats()["messages"])


if __name__ == "__main__":
    main()
