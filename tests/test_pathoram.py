"""BASELINE config 1: the Path ORAM restatement of the reference's CPU path
(oracle/gvs_pathoram.c) agrees bit-for-bit with the sequential model on a
seeded 10K-request create/read/delete mix at 2^16 capacity, and on the
targeted batch-interaction scenarios."""
import time

import pytest

from grapevine_amd import abi
from oracle import ffi

import targeted


def test_config1_10k_mix_bit_exact():
    cfg = abi.make_config(1 << 16, max_batch=4096)
    seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
    seq.seed(0x6772617065 + 1)
    p = ffi.gen_params(create=40, read=40, update=0, delete=20, n_identities=2000)
    t0 = time.perf_counter()
    for _ in range(5):  # 5 x 2000 = 10K requests
        reqs = seq.gen_batch(2000, p)
        want = seq.process_batch(reqs)
        got = oram.process_batch(reqs)
        assert got.tobytes() == want.tobytes()
    assert (oram.messages, oram.mailboxes) == (seq.messages, seq.mailboxes)
    assert oram.oram_accesses > 9_500 * 6  # 6 top-level accesses per request (hard errors: none)
    print(f"pathoram 10K ops in {time.perf_counter() - t0:.2f}s")


@pytest.mark.parametrize("name", sorted(targeted.SCENARIOS))
def test_targeted_scenarios(name):
    cfg, sc, reqs, expect = targeted.build(name)
    oram = ffi.PathOramModel(cfg)
    for h in sc.history:
        oram.process_batch(h)
    got = oram.process_batch(reqs)
    want = sc.model.process_batch(reqs)
    assert got.tobytes() == want.tobytes()
    assert list(got["status_code"]) == expect


def test_mixed_with_capacity_pressure():
    cfg = abi.make_config(4096, mailbox_partitions=4, mailbox_partition_slots=32, max_batch=1024)
    seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
    seq.seed(9)
    p = ffi.gen_params(n_identities=400, hot=15)
    for _ in range(8):
        reqs = seq.gen_batch(1024, p)
        assert oram.process_batch(reqs).tobytes() == seq.process_batch(reqs).tobytes()
