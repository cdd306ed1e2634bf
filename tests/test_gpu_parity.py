"""GPU parity: the HIP engine (libgvstore.so via the C ABI) against the CPU
oracle on identical seeded request streams.  Bit-exact responses (record bytes,
status codes), message-table bytes, live message / mailbox counts.

Store-level parity is against the repo's own restatement (oracle/); the
reference's hot path is absent, so it is "parity unpinned" w.r.t. upstream
(SURVEY.md §8(c)).
"""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import ObliviousStore
from oracle import ffi

from parity import diff_responses, run_stream

pytestmark = pytest.mark.gpu


def make_pair(n_msgs, Q, Sr, B, key=None):
    cfg = abi.make_config(n_msgs, mailbox_partitions=Q, mailbox_partition_slots=Sr,
                          max_batch=B, secret_key=key)
    return ObliviousStore(cfg), ffi.Model(cfg)


def test_library_is_native():
    import grapevine_amd.store as st
    lib = st.load_library()
    assert lib.gvs_version().decode().startswith("gvstore")


def test_mixed_stream_small():
    store, model = make_pair(4096, 16, 32, 1024)
    model.seed(11)
    seen = run_stream(store, model, ffi.gen_params(n_identities=300), batches=12, n=1024)
    assert {0, 1, 2, 4} <= set(seen), seen


def test_create_heavy_then_drain():
    store, model = make_pair(4096, 16, 32, 1024)
    model.seed(12)
    run_stream(store, model, ffi.gen_params(create=90, read=5, update=0, delete=5,
                                            n_identities=200), batches=4, n=1024)
    run_stream(store, model, ffi.gen_params(create=5, read=30, update=15, delete=50,
                                            nxt=70, n_identities=200), batches=6, n=1024)


def test_hot_recipient_62_limit():
    store, model = make_pair(8192, 16, 32, 1024)
    model.seed(13)
    seen = run_stream(store, model, ffi.gen_params(create=50, read=20, update=10, delete=20,
                                                   hot=40, n_identities=100), batches=8, n=1024)
    assert seen[5] > 0, seen


def test_message_capacity_exhaustion():
    # N = 256 slots, creates only: TOO_MANY_MESSAGES once full, then deletes free slots
    store, model = make_pair(256, 4, 64, 1024)
    model.seed(14)
    seen = run_stream(store, model, ffi.gen_params(create=100, read=0, update=0, delete=0,
                                                   n_identities=50), batches=2, n=300)
    assert seen[7] > 0, seen
    run_stream(store, model, ffi.gen_params(create=50, read=0, update=0, delete=50, nxt=50,
                                            n_identities=50), batches=4, n=500)


def test_recipient_capacity_exhaustion():
    # 4 partitions x 16 rows = 64 mailboxes for 2000 identities
    store, model = make_pair(4096, 4, 16, 1024)
    model.seed(15)
    seen = run_stream(store, model, ffi.gen_params(n_identities=2000), batches=6, n=1024)
    assert seen[6] > 0, seen


def test_partial_batches_and_single_access():
    store, model = make_pair(4096, 16, 32, 2048)
    model.seed(16)
    p = ffi.gen_params(n_identities=100)
    for n in (1, 7, 1000, 2048, 3):
        run_stream(store, model, p, batches=1, n=n, check_table=False)
    req = model.gen_batch(1, p)
    want = model.process_batch(req)
    got = store.access(req[0])
    assert bytes(got.tobytes()) == bytes(want[0].tobytes())


def test_c2_scale_stream():
    # BASELINE config 2: 2^20 messages, 4K-request batches
    store, model = make_pair(1 << 20, 256, 256, 4096)
    model.seed(0x6772617065 + 2)
    p = ffi.gen_params(create=60, read=15, update=10, delete=15, n_identities=20000)
    run_stream(store, model, p, batches=6, n=4096, check_table=False)
    p = ffi.gen_params(n_identities=20000)
    run_stream(store, model, p, batches=4, n=4096, check_table=True)


@pytest.mark.parametrize("name", ["single_mixed", "single_full", "sharded4"])
def test_golden_fixtures(name):
    """The HIP engine against the committed fixtures (tests/golden/), with no
    oracle in the loop."""
    from golden_io import load
    cfg, batches = load(name)
    store = ObliviousStore(cfg)
    for k, (reqs, want, (msgs, mboxes)) in enumerate(batches):
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"{name} batch {k}: " + "\n".join(d)
        st = store.stats()
        assert (st["messages"], st["mailboxes"]) == (msgs, mboxes), (name, k)
    store.close()
