"""Targeted batch-interaction scenarios (tests/targeted.py): the oracle must
produce the statuses derived by hand from DESIGN.md §2 (CPU), and the HIP
engine must match the oracle bit-for-bit on the same batches (GPU)."""
import pytest

import targeted
from parity import diff_responses, diff_tables

NAMES = sorted(targeted.SCENARIOS)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_statuses(name):
    cfg, sc, reqs, expect = targeted.build(name)
    got = sc.model.process_batch(reqs)
    assert list(got["status_code"]) == expect


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_engine_matches_oracle(name):
    from grapevine_amd.store import ObliviousStore
    cfg, sc, reqs, expect = targeted.build(name)
    store = ObliviousStore(cfg)
    for h in sc.history:
        got = store.process_batch(h)
    want = sc.model.process_batch(reqs)
    got = store.process_batch(reqs)
    d = diff_responses(got, want, reqs)
    assert not d, "\n".join(d)
    assert list(got["status_code"]) == expect
    dt = diff_tables(store.dump_messages(), sc.model.dump_messages())
    assert not dt, "\n".join(dt)
    st = store.stats()
    assert (st["messages"], st["mailboxes"]) == (sc.model.messages, sc.model.mailboxes)
    store.close()
