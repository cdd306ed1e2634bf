"""bench.py's response checks (check_batch) hold for the oracle's responses and
catch corrupted ones (CPU; torch on the host)."""
import numpy as np
import torch

import bench
from grapevine_amd import abi
from oracle import ffi


def as_t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(len(a), 1040).copy())


def test_oracle_responses_pass_and_corruption_is_caught():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)
    m = ffi.Model(cfg)
    m.seed(3)
    m.process_batch(m.gen_batch(1024, ffi.gen_params(create=100, read=0, update=0, delete=0,
                                                     n_identities=100)))
    reqs = m.gen_batch(1024, ffi.gen_params(n_identities=100))
    out = m.process_batch(reqs)
    r, o = as_t(reqs), as_t(out)
    viol, cre, dels = bench.check_batch(torch, r, o)
    assert viol == 0
    assert cre == int(((reqs["request_type"] == 1) & (out["status_code"] == 1)).sum())
    assert dels == int(((reqs["request_type"] == 4) & (out["status_code"] == 1)).sum())
    ok = np.nonzero((out["status_code"] == 1) & (reqs["request_type"] == 1))[0]
    fail = np.nonzero((out["status_code"] >= 2) & (out["status_code"] <= 7))[0]
    bad = o.clone()
    bad[ok[0], 100] ^= 1    # a payload byte of a successful CREATE's echo ...
    bad[fail[0], 200] ^= 1  # ... and of a failure record
    v2, _, _ = bench.check_batch(torch, r, bad)
    assert v2 == 2
