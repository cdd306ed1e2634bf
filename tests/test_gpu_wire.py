"""GPU parity of the device wire codec (SURVEY.md §8(f) rank 1;
include/gvstore.h gvs_process_wire_batch / gvs_wire_*_device).

  * decode: canonical and non-canonical QueryRequest encodings (reordered,
    repeated, merged records, unknown fields, non-minimal varints) and
    malformed ones -> the device's gvs_request slab, signatures and per-message
    status equal the host codec's prost-rule decoder (grapevine_amd/wire.py,
    pinned against google.protobuf in tests/test_wire.py), bit for bit;
  * encode: responses with and without timestamp, and hard errors -> the
    bytes prost writes (wire.encode_response), whole output slots checked;
  * end to end: wire requests through decode -> store -> encode on the GPU
    equal the CPU oracle's responses encoded on the host.
"""
import numpy as np
import pytest

from grapevine_amd import abi, wire
from grapevine_amd.store import ObliviousStore
from oracle import ffi

import wire_cases

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


def host(t, dtype, shape):
    return t.cpu().numpy().view(dtype).reshape(shape)


def small_store():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)
    return ObliviousStore(cfg), ffi.Model(cfg)


def slab(msgs, stride):
    s = np.zeros((len(msgs), stride), np.uint8)
    for k, m in enumerate(msgs):
        s[k, :len(m)] = np.frombuffer(m, np.uint8)
    return s, np.array([len(m) for m in msgs], np.uint32)


@pytest.mark.parametrize("stride", [1200, 2048])
def test_decode_matches_prost_rules(stride):
    store, _ = small_store()
    cases = [(n, m) for n, m in wire_cases.all_variants(21 + stride, 12) if len(m) <= stride]
    msgs = [m for _, m in cases]
    n = len(msgs)
    times = np.arange(1, n + 1, dtype=np.uint64) * 1_000_003
    s, lens = slab(msgs, stride)
    d_in, d_lens, d_t = dev(s), dev(lens), dev(times)
    d_req = torch.zeros(n * 1040, dtype=torch.uint8, device="cuda")
    d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n * 4,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # torch's fills/copies done before the engine stream runs
    rc = store.lib.gvs_wire_decode_device(store.h, d_in.data_ptr(), stride, d_lens.data_ptr(), n,
                                          d_t.data_ptr(), d_req.data_ptr(), d_sig.data_ptr(),
                                          d_st.data_ptr())
    assert rc == 0
    got_q = host(d_req, abi.REQUEST_DTYPE, (n,))
    got_sig = host(d_sig, np.uint8, (n, 64))
    got_st = host(d_st, np.uint32, (n,))
    want_q, want_sig, want_st = wire.decode_requests(msgs, timestamps=times, strict=False)
    for k, (name, _) in enumerate(cases):
        assert got_st[k] == want_st[k], (k, name, got_st[k], want_st[k])
        assert got_q[k].tobytes() == want_q[k].tobytes(), (k, name)
        assert got_sig[k].tobytes() == want_sig[k].tobytes(), (k, name)
    assert (got_st == 0).sum() > n // 4 and (got_st == 1).any() and (got_st == 2).any()
    store.close()


def test_length_beyond_stride_is_a_decode_error():
    store, _ = small_store()
    m = wire_cases.canonical(wire_cases.fields(__import__("random").Random(3)))
    s, lens = slab([m], 1100)
    lens[0] = 1101
    d_req = torch.zeros(1040, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(4, dtype=torch.uint8, device="cuda")
    keep = [dev(s), dev(lens), dev(np.array([7], np.uint64))]  # alive across the call
    torch.cuda.synchronize()
    assert store.lib.gvs_wire_decode_device(store.h, keep[0].data_ptr(), 1100, keep[1].data_ptr(), 1,
                                            keep[2].data_ptr(), d_req.data_ptr(), None,
                                            d_st.data_ptr()) == 0
    assert host(d_st, np.uint32, (1,))[0] == abi.WIRE_DECODE_ERROR
    assert not d_req.any().item()
    store.close()


@pytest.mark.parametrize("stride", [1042, 1100])
def test_encode_matches_prost(stride):
    store, _ = small_store()
    rng = np.random.default_rng(5)
    n = 301
    r = np.zeros(n, abi.RESPONSE_DTYPE)
    raw = r.view(np.uint8).reshape(n, 1040)
    raw[:, :1024] = rng.integers(0, 256, (n, 1024), dtype=np.uint8)
    r["record"]["timestamp"][::5] = 0
    r["status_code"] = rng.integers(1, 9, n)
    r["status_code"][3::7] = 0
    d_out = torch.full((n * stride,), 0xAB, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    d_r = dev(r)
    torch.cuda.synchronize()
    assert store.lib.gvs_wire_encode_device(store.h, d_r.data_ptr(), n, d_out.data_ptr(), stride,
                                            d_len.data_ptr()) == 0
    out = host(d_out, np.uint8, (n, stride))
    lens = host(d_len, np.uint32, (n,))
    for k in range(n):
        want = wire.encode_response(r[k])
        assert lens[k] == len(want), k
        assert out[k, :lens[k]].tobytes() == want, k
        assert not out[k, lens[k]:].any(), k  # the rest of the slot is zero-filled
    store.close()


def to_wire(reqs, rng):
    """The oracle's request stream as canonical wire messages, with a few
    replaced by non-canonical encodings of the same request or by malformed
    messages."""
    msgs = []
    for k, q in enumerate(reqs):
        f = dict(rt=int(q["request_type"]), auth=bytes(q["auth_identity"]), sig=rng.bytes(64),
                 id=bytes(q["msg_id"]), rc=bytes(q["recipient"]), pl=bytes(q["payload"]))
        m = wire_cases.canonical(f)
        pick = rng.random()
        if pick < 0.05:
            m = wire_cases.ld(4, wire_cases.record(f, (2, 3, 1))) + m[:105]
        elif pick < 0.08:
            m = m[:rng.integers(1, len(m))]
        msgs.append(m)
    return msgs


@pytest.mark.parametrize("host_api", [True, False])
def test_wire_batches_end_to_end(host_api):
    store, model = small_store()
    model.seed(31)
    params = ffi.gen_params(n_identities=200, hot=10)
    rng = np.random.default_rng(17)
    for b in range(4):
        reqs = model.gen_batch(1024, params)
        msgs = to_wire(reqs, rng)
        times = reqs["timestamp"].copy()
        q, sig, st = wire.decode_requests(msgs, timestamps=times, strict=False)
        want = [wire.encode_response(r) for r in model.process_batch(q)]
        if host_api:
            got, got_sig, got_st = store.process_wire_batch(msgs, times, in_stride=1104)
            assert (got_st == st).all()
            assert got_sig.tobytes() == sig.tobytes()
        else:
            s, lens = slab(msgs, 1104)
            n = len(msgs)
            d_out = torch.zeros(n * 1042, dtype=torch.uint8, device="cuda")
            d_len = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
            d_sig = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
            d_in, d_lens, d_t = dev(s), dev(lens), dev(times)  # alive across the call
            torch.cuda.synchronize()
            store._check(store.lib.gvs_process_wire_batch_device(
                store.h, d_in.data_ptr(), 1104, d_lens.data_ptr(), n, d_t.data_ptr(), None,
                d_out.data_ptr(), 1042, d_len.data_ptr(), d_sig.data_ptr(), None))
            out = host(d_out, np.uint8, (n, 1042))
            ol = host(d_len, np.uint32, (n,))
            got = [out[k, :ol[k]].tobytes() for k in range(n)]
            assert host(d_sig, np.uint8, (n, 64)).tobytes() == sig.tobytes()
        bad = [k for k in range(len(want)) if got[k] != want[k]]
        assert not bad, f"batch {b}: {len(bad)} responses differ (first {bad[:5]})"
        assert sum(1 for w in want if len(w) == 1042) > 900
        st_ = store.stats()
        assert (st_["messages"], st_["mailboxes"]) == (model.messages, model.mailboxes)
    store.close()


def test_wire_batches_pipelined():
    """gvs_process_wire_batches: several wire batches (one empty, ragged
    sizes) in one double-buffered call, equal to the oracle batch by batch;
    then a call with one batch carrying challenges, half signed correctly."""
    from oracle import sr25519 as sr
    import random
    store, model = small_store()
    model.seed(33)
    params = ffi.gen_params(n_identities=200, hot=10)
    rng = np.random.default_rng(19)
    sizes = [1024, 0, 517, 1024, 3, 40]
    batches, times, wants = [], [], []
    signer = random.Random(8)
    xs = {}
    chal = np.zeros((sum(sizes), 32), np.uint8)
    base = sum(sizes[:-1])
    for b, n in enumerate(sizes):
        reqs = model.gen_batch(n, params) if n else np.zeros(0, abi.REQUEST_DTYPE)
        msgs = to_wire(reqs, rng)
        t = reqs["timestamp"].copy()
        q, sig, st = wire.decode_requests(msgs, timestamps=t, strict=False)
        if b == len(sizes) - 1:  # signed batch: identities with known keys
            for k in range(n):
                x = xs.setdefault(k, signer.randrange(1, sr.L))
                pk = sr.public_key(x)
                c = rng.bytes(32)
                chal[base + k] = np.frombuffer(c, np.uint8)
                f = dict(rt=int(reqs[k]["request_type"]), auth=pk,
                         sig=sr.sign(x, c, signer.randrange(1, sr.L)) if k % 2 == 0 else rng.bytes(64),
                         id=bytes(reqs[k]["msg_id"]), rc=bytes(reqs[k]["recipient"]),
                         pl=bytes(reqs[k]["payload"]))
                msgs[k] = wire_cases.canonical(f)
            q, sig, st = wire.decode_requests(msgs, timestamps=t, strict=False)
            for k in range(n):
                if st[k] == 0 and not sr.verify(bytes(q[k]["auth_identity"]), bytes(chal[base + k]),
                                                bytes(sig[k])):
                    q[k]["request_type"] = 0
                    st[k] = abi.WIRE_BAD_SIGNATURE
        wants.append(([wire.encode_response(r) for r in model.process_batch(q)], st))
        batches.append(msgs)
        times.append(t)
    # challenges are all-or-none per call: the unsigned batches in one call,
    # the signed one in a second
    got = store.process_wire_batches(batches[:-1], np.concatenate(times[:-1]), in_stride=1104)
    got += store.process_wire_batches(batches[-1:], times[-1], in_stride=1104, challenges=chal[base:])
    assert len(got) == len(sizes)
    for b, ((g, gst), (w, wst)) in enumerate(zip(got, wants)):
        assert len(g) == sizes[b]
        assert (gst == wst).all(), b
        bad = [k for k in range(len(w)) if g[k] != w[k]]
        assert not bad, f"batch {b}: {len(bad)} responses differ (first {bad[:5]})"
    assert (wants[-1][1] == abi.WIRE_BAD_SIGNATURE).sum() >= 10
    st_ = store.stats()
    assert (st_["messages"], st_["mailboxes"]) == (model.messages, model.mailboxes)
    store.close()


def test_wire_pipeline_stops_at_failing_batch():
    """gvs_process_wire_batches on a 4-shard store: a batch that overflows a
    router bucket stops the pipeline there (the batches before it applied,
    it and the later one not), as gvs_process_batches does."""
    from grapevine_amd.store import GvsError
    S = 4
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          shard_count=S, route_capacity=320)
    store, cl = ObliviousStore(cfg), ffi.Cluster(cfg)
    cl.seed(15)
    p = ffi.gen_params(n_identities=300)
    hot = ffi.gen_params(create=100, read=0, update=0, delete=0, hot=60, n_identities=300)
    ok = [cl.gen_batch(S * 1024, p) for _ in range(2)]
    for b in ok:
        cl.process_batch(b)
    bad = cl.gen_batch(S * 1024, hot)
    assert cl.process_batch(bad) is None
    later = cl.gen_batch(S * 1024, p)

    def msgs(b):
        q = b.copy()
        q["request_type"][q["request_type"] == 0] = 0xFFFFFFFF  # still a hard error
        return [m.tobytes() for m in wire.encode_requests(q)]

    batches = ok + [bad, later]
    times = np.concatenate([b["timestamp"] for b in batches])
    with pytest.raises(GvsError) as ei:
        store.process_wire_batches([msgs(b) for b in batches], times, in_stride=1104)
    assert ei.value.code == abi.GVS_ERR_BATCH_OVERFLOW and ei.value.applied == 2
    assert store.stats()["messages"] == cl.messages
    assert store.stats()["batches"] == 2
    # `later` was not applied: it runs now, as the oracle's next batch
    got = store.process_wire_batches([msgs(later)], later["timestamp"], in_stride=1104)
    w = cl.process_batch(later)
    assert got[0][0] == [wire.encode_response(r) for r in w]
    assert store.dump_messages().tobytes() == cl.dump_messages().tobytes()
    store.close()


def test_wire_batches_pinned_slabs():
    """gvs_process_wire_batches with the message and response slabs in pinned
    memory (gvs_host_alloc: copied without staging) gives the same bytes as
    the oracle, batch by batch."""
    import ctypes
    store, model = small_store()
    model.seed(37)
    params = ffi.gen_params(n_identities=200, hot=10)
    rng = np.random.default_rng(23)
    sizes = [1024, 300, 1024]
    msgs, times, wants = [], [], []
    for n in sizes:
        reqs = model.gen_batch(n, params)
        m = to_wire(reqs, rng)
        t = reqs["timestamp"].copy()
        q, _, _ = wire.decode_requests(m, timestamps=t, strict=False)
        wants += [wire.encode_response(r) for r in model.process_batch(q)]
        msgs += m
        times.append(t)
    total, stride = len(msgs), 1104
    slab = store.host_array(total * stride, np.uint8).reshape(total, stride)
    out = store.host_array(total * 1042, np.uint8).reshape(total, 1042)
    slab[:] = 0
    for k, m in enumerate(msgs):
        slab[k, :len(m)] = np.frombuffer(m, np.uint8)
    lens = np.array([len(m) for m in msgs], np.uint32)
    t = np.concatenate(times)
    counts = np.array(sizes, np.uint32)
    olens = np.zeros(total, np.uint32)
    applied = ctypes.c_uint32(0)
    store._check(store.lib.gvs_process_wire_batches(
        store.h, slab.ctypes.data, stride, lens.ctypes.data, counts.ctypes.data, len(sizes),
        t.ctypes.data, None, out.ctypes.data, 1042, olens.ctypes.data, None, ctypes.byref(applied)))
    assert applied.value == len(sizes)
    got = [out[k, :olens[k]].tobytes() for k in range(total)]
    bad = [k for k in range(total) if got[k] != wants[k]]
    assert not bad, f"{len(bad)} responses differ (first {bad[:5]})"
    store.close()
