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


def test_host_pipeline_matches_oracle():
    """gvs_process_batches: several host batches double-buffered (staging and
    PCIe of batch t+1 / t-1 behind batch t) equal the same batches one by one."""
    from parity import diff_tables
    store, model = make_pair(4096, 16, 32, 1024)
    model.seed(13)
    p = ffi.gen_params(n_identities=300)
    for sizes in ([1024, 1024, 1024, 1024, 1024], [1, 0, 700, 1024], [1024]):
        batches = [model.gen_batch(n, p) for n in sizes]
        want = [model.process_batch(b) for b in batches]
        got = store.process_batches(batches)
        for k, (g, w, b) in enumerate(zip(got, want, batches)):
            d = diff_responses(g, w, b)
            assert not d, f"{sizes} batch {k}: " + "\n".join(d)
        st = store.stats()
        assert (st["messages"], st["mailboxes"]) == (model.messages, model.mailboxes)
    assert not diff_tables(store.dump_messages(), model.dump_messages())


@pytest.mark.parametrize("pin", ["in", "out", "both"])
def test_host_pipeline_pinned_buffers(pin):
    """Caller buffers in pinned memory (gvs_host_alloc) skip the staging
    copies: same responses as the oracle, pageable and pinned mixed."""
    import ctypes
    store, model = make_pair(4096, 16, 32, 1024)
    model.seed(15)
    p = ffi.gen_params(n_identities=300)
    sizes = [1024, 600, 1024, 1]
    batches = [model.gen_batch(n, p) for n in sizes]
    want = np.concatenate([model.process_batch(b) for b in batches])
    total = sum(sizes)
    reqs = store.host_array(total, abi.REQUEST_DTYPE) if pin in ("in", "both") else \
        np.zeros(total, abi.REQUEST_DTYPE)
    out = store.host_array(total, abi.RESPONSE_DTYPE) if pin in ("out", "both") else \
        np.zeros(total, abi.RESPONSE_DTYPE)
    reqs[:] = np.concatenate(batches)
    counts = np.array(sizes, np.uint32)
    applied = ctypes.c_uint32(0)
    store._check(store.lib.gvs_process_batches(store.h, reqs.ctypes.data, counts.ctypes.data,
                                               len(sizes), out.ctypes.data, ctypes.byref(applied)))
    assert applied.value == len(sizes)
    d = diff_responses(np.array(out), want, reqs)
    assert not d, "\n".join(d)
    st = store.stats()
    assert (st["messages"], st["mailboxes"]) == (model.messages, model.mailboxes)
    store.close()


def test_host_pipeline_stops_at_failing_batch():
    """A batch that overflows a router bucket stops the pipeline there: the
    batches before it are applied, it and the later ones are not, and the
    store goes on from that state."""
    from grapevine_amd.store import GvsError
    S = 4
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          shard_count=S, route_capacity=320)
    store, cl = ObliviousStore(cfg), ffi.Cluster(cfg)
    cl.seed(14)
    p = ffi.gen_params(n_identities=300)
    hot = ffi.gen_params(create=100, read=0, update=0, delete=0, hot=60, n_identities=300)
    ok = [cl.gen_batch(S * 1024, p) for _ in range(2)]
    want = [cl.process_batch(b) for b in ok]
    bad = cl.gen_batch(S * 1024, hot)
    assert cl.process_batch(bad) is None
    later = cl.gen_batch(S * 1024, p)
    with pytest.raises(GvsError) as ei:
        store.process_batches(ok + [bad, later])
    assert ei.value.code == abi.GVS_ERR_BATCH_OVERFLOW and ei.value.applied == 2
    assert store.stats()["messages"] == cl.messages
    assert store.stats()["batches"] == 2 and store.stats()["epoch"] == 2
    # `later` was not applied: it runs now, as the oracle's next batch
    got = store.process_batches([later])
    d = diff_responses(got[0], cl.process_batch(later), later)
    assert not d, "\n".join(d)
    assert store.dump_messages().tobytes() == cl.dump_messages().tobytes()


def test_device_batches_match_oracle():
    """gvs_process_batches_device: several device-resident batches in one call
    (no host round trip between them) equal the oracle batch by batch."""
    torch = pytest.importorskip("torch")
    store, model = make_pair(4096, 16, 32, 1024)
    model.seed(16)
    p = ffi.gen_params(n_identities=300)
    sizes = [1024, 1, 0, 700, 1024, 1024]
    batches = [model.gen_batch(n, p) for n in sizes]
    want = np.concatenate([model.process_batch(b) for b in batches])
    reqs = np.concatenate(batches)
    d_in = torch.from_numpy(reqs.view(np.uint8).reshape(-1).copy()).cuda()
    d_out = torch.zeros(len(reqs) * 1040, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert store.process_batches_device(d_in.data_ptr(), sizes, d_out.data_ptr()) == len(sizes)
    got = d_out.cpu().numpy().view(abi.RESPONSE_DTYPE)
    d = diff_responses(got, want, reqs)
    assert not d, "\n".join(d)
    st = store.stats()
    assert (st["messages"], st["mailboxes"], st["batches"]) == (model.messages, model.mailboxes, len(sizes))
    store.close()


def test_device_batches_stop_at_failing_batch():
    """A batch that overflows a router bucket stops gvs_process_batches_device:
    the batches before it are applied, its and the later responses are zero,
    and the store goes on from that state."""
    torch = pytest.importorskip("torch")
    from grapevine_amd.store import GvsError
    S = 4
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          shard_count=S, route_capacity=320)
    store, cl = ObliviousStore(cfg), ffi.Cluster(cfg)
    cl.seed(17)
    p = ffi.gen_params(n_identities=300)
    hot = ffi.gen_params(create=100, read=0, update=0, delete=0, hot=60, n_identities=300)
    ok = [cl.gen_batch(S * 1024, p) for _ in range(2)]
    want = [cl.process_batch(b) for b in ok]
    bad = cl.gen_batch(S * 1024, hot)
    assert cl.process_batch(bad) is None
    later = cl.gen_batch(S * 1024, p)
    reqs = np.concatenate(ok + [bad, later])
    d_in = torch.from_numpy(reqs.view(np.uint8).reshape(-1).copy()).cuda()
    d_out = torch.full((len(reqs) * 1040,), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(GvsError) as ei:
        store.process_batches_device(d_in.data_ptr(), [S * 1024] * 4, d_out.data_ptr())
    assert ei.value.code == abi.GVS_ERR_BATCH_OVERFLOW and ei.value.applied == 2
    got = d_out.cpu().numpy().view(abi.RESPONSE_DTYPE)
    for k in range(2):
        d = diff_responses(got[k * S * 1024:(k + 1) * S * 1024], want[k], ok[k])
        assert not d, "\n".join(d)
    assert not got[2 * S * 1024:].view(np.uint8).any(), "unapplied responses must be zero"
    assert store.stats()["messages"] == cl.messages and store.stats()["batches"] == 2
    got_later = store.process_batches([later])
    d = diff_responses(got_later[0], cl.process_batch(later), later)
    assert not d, "\n".join(d)
