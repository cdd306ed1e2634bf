"""Hand-built batches that hit the batch-interaction corners of DESIGN.md §2
(test infrastructure).  Each builder returns (setup_batches, test_batch,
expected_statuses); ids created inside the test batch are predicted with a
shadow oracle replaying the same history (ids are a deterministic PRP of
(slot, counter))."""
import numpy as np

from grapevine_amd import abi
from oracle import ffi

TS = 1_700_000_000


def ident(i):
    return ffi.identity(i)


def mk(t, auth, msg_id=bytes(16), recipient=bytes(32), payload=b"", ts=None):
    r = np.zeros(1, dtype=abi.REQUEST_DTYPE)[0]
    r["request_type"] = t
    r["auth_identity"] = np.frombuffer(auth, np.uint8)
    r["msg_id"] = np.frombuffer(msg_id, np.uint8)
    r["recipient"] = np.frombuffer(recipient, np.uint8)
    if payload:
        p = (payload * (936 // len(payload) + 1))[:936]
        r["payload"] = np.frombuffer(p, np.uint8)
    r["timestamp"] = ts if ts is not None else TS
    return r


def batch(reqs):
    out = np.zeros(len(reqs), dtype=abi.REQUEST_DTYPE)
    for i, r in enumerate(reqs):
        out[i] = r
        out[i]["timestamp"] = TS + i + 1
    return out


def ids_of(resps):
    return [bytes(r["record"]["msg_id"]) for r in resps]


class Scenario:
    """Runs setup batches on a model and lets a test predict ids via a shadow."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.model = ffi.Model(cfg)
        self.history = []

    def run(self, reqs):
        b = batch(reqs)
        self.history.append(b)
        return self.model.process_batch(b)

    def predict(self, reqs):
        """Responses the next batch would get, without applying it."""
        shadow = ffi.Model(self.cfg)
        for h in self.history:
            shadow.process_batch(h)
        return shadow.process_batch(batch(reqs))


def scenario_same_batch_interplay(cfg):
    """next-ops serialise before creates, creates before by-id ops."""
    X, A, Bq = ident(1), ident(2), ident(3)
    sc = Scenario(cfg)
    r = sc.run([mk(1, A, recipient=X, payload=b"m0"), mk(1, A, recipient=X, payload=b"m1")])
    m0, m1 = ids_of(r)
    # batch: create c2 for X; read-next X; delete-next X; read-next X; delete-next X; delete-next X;
    # read by id of the id c2 will get; update m0 (already popped -> NOT_FOUND); read m1 (popped)
    probe = [mk(1, Bq, recipient=X, payload=b"c2")]
    c2 = ids_of(sc.predict(probe))[0]
    reqs = [
        mk(1, Bq, recipient=X, payload=b"c2"),
        mk(2, X), mk(4, X), mk(2, X), mk(4, X), mk(4, X),
        mk(2, X, msg_id=c2),
        mk(3, A, msg_id=m0, recipient=X, payload=b"zz"),
        mk(2, A, msg_id=m1),
        mk(2, X),
    ]
    return sc, reqs, [1, 1, 1, 1, 1, 2, 1, 2, 2, 2]


def scenario_update_read_delete_same_id(cfg):
    X, A = ident(11), ident(12)
    sc = Scenario(cfg)
    (m,) = ids_of(sc.run([mk(1, A, recipient=X, payload=b"v0")]))
    reqs = [
        mk(2, A, msg_id=m),                                  # v0
        mk(3, A, msg_id=m, recipient=X, payload=b"v1"),      # ok
        mk(3, ident(99), msg_id=m, recipient=X, payload=b"bad"),  # NOT_FOUND (stranger)
        mk(3, X, msg_id=m, recipient=A, payload=b"bad"),     # INVALID_RECIPIENT
        mk(2, X, msg_id=m),                                  # v1
        mk(3, X, msg_id=m, recipient=X, payload=b"v2"),
        mk(4, A, msg_id=m, recipient=A),                     # INVALID_RECIPIENT
        mk(4, A, msg_id=m, recipient=X),                     # deleted (returns v2)
        mk(2, A, msg_id=m),                                  # NOT_FOUND
        mk(3, A, msg_id=m, recipient=X, payload=b"v3"),      # NOT_FOUND
        mk(4, X, msg_id=m, recipient=X),                     # NOT_FOUND
        mk(2, X),                                            # next: mailbox emptied by the by-id delete? no: next ops run first
    ]
    return sc, reqs, [1, 1, 2, 4, 1, 1, 4, 1, 2, 2, 2, 1]


def scenario_create_then_byid_same_batch(cfg):
    X, A = ident(21), ident(22)
    sc = Scenario(cfg)
    sc.run([mk(1, A, recipient=ident(23))])
    probe = [mk(1, A, recipient=X, payload=b"n0"), mk(1, A, recipient=X, payload=b"n1")]
    n0, n1 = ids_of(sc.predict(probe))
    reqs = probe + [
        mk(3, X, msg_id=n0, recipient=X, payload=b"u0"),
        mk(4, A, msg_id=n1, recipient=X),
        mk(2, A, msg_id=n1),
        mk(2, X, msg_id=n0),
        mk(2, X),  # next-op runs before the creates: X has no mailbox yet
    ]
    return sc, reqs, [1, 1, 1, 1, 2, 1, 2]


def scenario_62_limit_with_pop(cfg):
    X, A = ident(31), ident(32)
    sc = Scenario(cfg)
    st = sc.run([mk(1, A, recipient=X) for _ in range(62)])
    assert list(st["status_code"]) == [1] * 62
    reqs = [mk(1, A, recipient=X), mk(4, X), mk(1, A, recipient=X), mk(2, X)]
    # delete-next pops first, so the first create fits and the second hits 5
    return sc, reqs, [1, 1, 5, 1]


def scenario_empty_then_recreate(cfg):
    """A mailbox emptied by delete-next is freed and re-admitted in the same batch."""
    X, A = ident(41), ident(42)
    sc = Scenario(cfg)
    sc.run([mk(1, A, recipient=X)])
    reqs = [mk(1, A, recipient=X, payload=b"again"), mk(4, X), mk(2, X)]
    return sc, reqs, [1, 1, 2]


def scenario_recipient_partition_full(cfg):
    """Fill every mailbox row of the (single) partition, then pop one empty and
    admit new recipients in seq order of their first create."""
    A = ident(50)
    rows = cfg.mailbox_partition_slots * cfg.mailbox_partitions
    sc = Scenario(cfg)
    st = sc.run([mk(1, A, recipient=ident(1000 + k)) for k in range(rows)])
    assert list(st["status_code"]) == [1] * rows
    reqs = [
        mk(1, A, recipient=ident(5000)),      # new recipient: admitted into the row freed below
        mk(1, A, recipient=ident(5001)),      # new: no room -> 6
        mk(4, ident(1000)),                   # delete-next empties recipient 1000's mailbox
        mk(1, A, recipient=ident(5000)),      # same new recipient again -> ok
        mk(1, A, recipient=ident(1001)),      # existing -> ok
    ]
    return sc, reqs, [1, 6, 1, 1, 1]


def scenario_capacity_cutoff(cfg):
    """Message table one below full; a delete-next frees a slot inside the batch."""
    A = ident(60)
    n = cfg.msg_capacity
    sc = Scenario(cfg)
    per = 50
    k = 0
    while k < n - 1:
        m = min(1024, n - 1 - k)
        st = sc.run([mk(1, A, recipient=ident(2000 + (k + j) // per)) for j in range(m)])
        assert (st["status_code"] == 1).all()
        k += m
    reqs = [
        mk(1, A, recipient=ident(9000)),  # takes the last free slot
        mk(1, A, recipient=ident(9001)),  # slot freed by the delete-next below (next ops go first)
        mk(1, A, recipient=ident(9002)),  # TOO_MANY_MESSAGES
        mk(4, ident(2000)),               # pops a message -> frees a slot
        mk(1, A, recipient=bytes(32)),    # INVALID_RECIPIENT beats TOO_MANY_MESSAGES
    ]
    return sc, reqs, [1, 1, 7, 1, 4]


SCENARIOS = {
    "same_batch_interplay": (scenario_same_batch_interplay, dict(n=4096, Q=4, Sr=64)),
    "update_read_delete_same_id": (scenario_update_read_delete_same_id, dict(n=4096, Q=4, Sr=64)),
    "create_then_byid_same_batch": (scenario_create_then_byid_same_batch, dict(n=4096, Q=4, Sr=64)),
    "62_limit_with_pop": (scenario_62_limit_with_pop, dict(n=4096, Q=4, Sr=64)),
    "empty_then_recreate": (scenario_empty_then_recreate, dict(n=4096, Q=4, Sr=64)),
    "recipient_partition_full": (scenario_recipient_partition_full, dict(n=4096, Q=1, Sr=64)),
    "capacity_cutoff": (scenario_capacity_cutoff, dict(n=1024, Q=4, Sr=256)),
}


def build(name):
    fn, c = SCENARIOS[name]
    cfg = abi.make_config(c["n"], mailbox_partitions=c["Q"], mailbox_partition_slots=c["Sr"],
                          max_batch=1024)
    sc, reqs, expect = fn(cfg)
    return cfg, sc, batch(reqs), expect
