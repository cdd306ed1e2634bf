#!/usr/bin/env python3
"""Run a fixed schedule of batches with a chosen request mix (run under
rocprofv3 by tests/test_oblivious.py and tests/test_timing.py).  The prefill is
identical for every mix; only the last `--batches` batches differ.  Test
infrastructure: the oracle only generates realistic requests against the live
state and checks the responses.

    python tools/oblivious_probe.py MIX [--log2n L] [--batch B] [--auth]
                                        [--shards S] [--fill-batches F]

--shards S > 1 runs the sharded store in its single-process form (S shards on
one device, the router kernels k_route_* and the padded all-to-all), against
the oracle's cluster model.
"""
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
    "rud": dict(create=0, read=34, update=33, delete=33, nxt=50),
    "all_create": dict(create=100, read=0, update=0, delete=0),
    "all_miss_read": dict(create=0, read=100, update=0, delete=0, nxt=0, miss=100),
    "hot_next": dict(create=30, read=35, update=0, delete=35, nxt=100, hot=100),
    "hot_next_rud": dict(create=0, read=50, update=0, delete=50, nxt=100, hot=100),
    "deletes": dict(create=0, read=0, update=0, delete=100, nxt=30),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("mix", choices=sorted(MIXES))
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--batches", type=int, default=3)
    p.add_argument("--fill-batches", type=int, default=4)
    p.add_argument("--shards", type=int, default=0)
    p.add_argument("--identities", type=int, default=5000)
    p.add_argument("--auth", action="store_true", help="authenticated storage (DESIGN.md §8)")
    a = p.parse_args()
    S = a.shards if a.shards > 1 else 0
    cfg = abi.make_config(1 << a.log2n, max_batch=a.batch, auth_storage=a.auth, shard_count=S)
    store = ObliviousStore(cfg)
    model = ffi.Cluster(cfg) if S else ffi.Model(cfg)
    n = a.batch * (S or 1)
    model.seed(77)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=a.identities)
    for _ in range(a.fill_batches):
        reqs = model.gen_batch(n, fill)
        want = model.process_batch(reqs)
        got = store.process_batch(reqs)
        assert got.tobytes() == want.tobytes(), "parity failure inside the probe (prefill)"
    model.seed(1234)  # same request-generator state for every mix
    params = ffi.gen_params(n_identities=a.identities, bad_auth=0, bad_recipient=0, hard_error=0,
                            zero_recipient=0, **{"miss": 0, **MIXES[a.mix]})
    for _ in range(a.batches):
        reqs = model.gen_batch(n, params)
        want = model.process_batch(reqs)
        got = store.process_batch(reqs)
        assert got.tobytes() == want.tobytes(), "parity failure inside the probe"
    store.synchronize()
    print("probe ok", a.mix, store.stats()["messages"])


if __name__ == "__main__":
    main()
