"""Shared helpers for GPU-vs-oracle parity tests (test infrastructure)."""
import numpy as np

from grapevine_amd import abi

KIND_NAMES = {1: "CREATE", 2: "READ", 3: "UPDATE", 4: "DELETE"}


def describe_request(r):
    t = int(r["request_type"])
    name = KIND_NAMES.get(t, f"type{t}")
    if t in (2, 4) and not r["msg_id"].any():
        name += "-next"
    return name


def diff_responses(got, want, reqs, limit=8):
    """Return a human-readable list of mismatching responses (empty if equal)."""
    n = len(want)
    if n == 0:
        return [] if len(got) == 0 else [f"{len(got)} responses for an empty batch"]
    g = got.view(np.uint8).reshape(n, -1)
    w = want.view(np.uint8).reshape(n, -1)
    bad = np.nonzero((g != w).any(axis=1))[0]
    out = []
    for i in bad[:limit]:
        fields = [f for f in ("msg_id", "sender", "recipient", "timestamp", "payload")
                  if not np.array_equal(got[i]["record"][f], want[i]["record"][f])]
        out.append(f"#{i} {describe_request(reqs[i])}: status got {got[i]['status_code']} "
                   f"want {want[i]['status_code']}; record fields differ: {fields}")
    if len(bad) > limit:
        out.append(f"... {len(bad)} mismatching responses in total")
    return out


def diff_tables(got, want, limit=5, chunk=1 << 18):
    g = got.view(np.uint8).reshape(len(got), -1)
    w = want.view(np.uint8).reshape(len(want), -1)
    # chunked: a C3 table is 16 GiB, a whole-array comparison would add 16 GiB
    bad = np.concatenate([np.nonzero((g[i:i + chunk] != w[i:i + chunk]).any(axis=1))[0] + i
                          for i in range(0, len(g), chunk)] or [np.zeros(0, dtype=np.int64)])
    out = [f"slot {s}: got id {bytes(got[s]['msg_id']).hex()} want {bytes(want[s]['msg_id']).hex()}"
           for s in bad[:limit]]
    if len(bad) > limit:
        out.append(f"... {len(bad)} mismatching slots")
    return out


def run_stream(store, model, params, batches, n, check_table=True, seen=None):
    """Drive `batches` seeded batches through both; assert bit-exact parity.
    Returns a Counter of the status codes seen (coverage evidence)."""
    from collections import Counter
    seen = Counter() if seen is None else seen
    for b in range(batches):
        reqs = model.gen_batch(n, params)
        want = model.process_batch(reqs)
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"batch {b}: " + "\n".join(d)
        st = store.stats()
        assert st["messages"] == model.messages, (b, st, model.messages)
        assert st["mailboxes"] == model.mailboxes, (b, st, model.mailboxes)
        assert st["creation_counter"] == model.creation_counter
        seen.update(int(x) for x in want["status_code"])
    if check_table:
        dt = diff_tables(store.dump_messages(), model.dump_messages())
        assert not dt, "\n".join(dt)
    return seen
