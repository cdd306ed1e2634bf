"""CPU tests of the sharded store's oracle: the routing rule,
the per-(source, shard) capacity, and that sharding preserves the semantics
of the unsharded store.  The GPU engine is checked against this cluster model
bit for bit in tests/test_gpu_sharded.py."""
import numpy as np
import pytest

from grapevine_amd import abi
from oracle import ffi

KEY = bytes((0x67 + 31 * i) & 0xFF for i in range(32))


def cluster_cfg(S, N=4096, B=1024, Q=16, Sr=32, C=0):
    return abi.make_config(N, mailbox_partitions=Q, mailbox_partition_slots=Sr, max_batch=B,
                           shard_count=S, route_capacity=C)


def test_shard_tagged_ids_round_trip_and_name_their_shard():
    for shard in (0, 1, 5, 63):
        for slot, ctr in ((0, 0), (4095, 7), (17, 1 << 40)):
            i = ffi.id_encode_shard(KEY[:16], shard, slot, ctr)
            assert ffi.id_decode_shard(KEY[:16], i, 4096, 64) == (shard, slot, ctr)
            if shard:
                assert ffi.id_decode_shard(KEY[:16], i, 4096, shard) is None  # shard out of range
    # shard 0 ids are exactly the unsharded store's ids
    assert ffi.id_encode_shard(KEY[:16], 0, 9, 3) == ffi.id_encode(KEY[:16], 9, 3)
    # another shard's id does not decode as an unsharded id
    assert ffi.id_decode(KEY[:16], ffi.id_encode_shard(KEY[:16], 1, 9, 3), 4096) is None


def test_default_route_capacity():
    assert ffi.route_capacity(65536, 1) == 65536
    c8 = ffi.route_capacity(65536, 8)
    assert c8 % 64 == 0 and 8192 + 8 * 90 < c8 <= 9216
    assert ffi.route_capacity(1024, 2) == 768
    assert ffi.route_capacity(1024, 64) <= 1024


def test_routing_rule_per_request_kind():
    S = 4
    cfg = cluster_cfg(S)
    cl = ffi.Cluster(cfg)
    cl.seed(3)
    p = ffi.gen_params(n_identities=200, hard_error=5, zero_recipient=5)
    for _ in range(3):  # populate so that by-id ops name real messages
        assert cl.process_batch(cl.gen_batch(1024, p)) is not None
    reqs = cl.gen_batch(1024, p)
    dest = ffi.route(cfg, reqs)
    for i, r in enumerate(reqs):
        t = int(r["request_type"])
        hard = t not in (1, 2, 3, 4) or not r["auth_identity"].any() or (t == 3 and not r["msg_id"].any())
        if hard:
            assert dest[i] == i % S
            continue
        if t == 1:
            if not r["recipient"].any():
                assert dest[i] == i % S
            else:
                _, lo = hash_of(r["recipient"])
                assert dest[i] == (lo & 0xFFFF) % S
        elif t in (2, 4) and not r["msg_id"].any():
            _, lo = hash_of(r["auth_identity"])
            assert dest[i] == (lo & 0xFFFF) % S
        else:
            dec = ffi.id_decode_shard(KEY[:16], bytes(r["msg_id"]), cfg.msg_capacity, S)
            assert dest[i] == (dec[0] if dec else i % S)


def hash_of(x):
    import ctypes
    hi, lo = ctypes.c_uint64(), ctypes.c_uint64()
    ffi.lib().gvo_recipient_hash(KEY[16:], bytes(x), ctypes.byref(hi), ctypes.byref(lo))
    return hi.value, lo.value


def test_messages_live_on_their_recipients_shard():
    S = 4
    cfg = cluster_cfg(S)
    cl = ffi.Cluster(cfg)
    cl.seed(5)
    p = ffi.gen_params(n_identities=300)
    for _ in range(6):
        assert cl.process_batch(cl.gen_batch(2048, p)) is not None
    total = 0
    for k in range(S):
        t = cl.shard(k).dump_messages()
        live = t[t["msg_id"].any(axis=1)]
        total += len(live)
        for rec in live:
            assert ffi.id_decode_shard(KEY[:16], bytes(rec["msg_id"]), cfg.msg_capacity, S)[0] == k
            assert (hash_of(rec["recipient"])[1] & 0xFFFF) % S == k
    assert total == cl.messages > 0


def test_single_shard_cluster_equals_plain_model():
    cfg1 = cluster_cfg(1)
    cl, m = ffi.Cluster(cfg1), ffi.Model(abi.make_config(4096, mailbox_partitions=16,
                                                         mailbox_partition_slots=32,
                                                         max_batch=1024))
    cl.seed(8)
    m.seed(8)
    p = ffi.gen_params(n_identities=250)
    for _ in range(5):
        r1, r2 = cl.gen_batch(1024, p), m.gen_batch(1024, p)
        assert r1.tobytes() == r2.tobytes()
        assert cl.process_batch(r1).tobytes() == m.process_batch(r2).tobytes()
    assert cl.messages == m.messages and cl.mailboxes == m.mailboxes


def shed_mask(cfg, reqs, B):
    return ffi.route_shed(cfg, reqs, B)


@pytest.mark.parametrize("S", [2, 4, 8])
def test_sharding_preserves_unsharded_semantics(S):
    """Same logical request stream into an unsharded model and an S-shard
    cluster (ample capacity everywhere): identical statuses and identical
    records except for the message ids, which name their shard.  Requests the
    router sheds (a source's ops past their routing key's cap; early batches
    hit few ids many times) go to the unsharded model as hard errors and come
    back from the cluster as INTERNAL_ERROR with their time."""
    rng = np.random.default_rng(100 + S)
    B = 1024
    single = ffi.Model(abi.make_config(1 << 16, mailbox_partitions=64, mailbox_partition_slots=64,
                                       max_batch=S * B))
    cl = ffi.Cluster(cluster_cfg(S, N=1 << 15, B=B, Q=32, Sr=64, C=B))
    ids_single, ids_cluster, owners = [], [], []
    n_shed = 0
    pool = [ffi.identity(i) for i in range(120)]
    for batch in range(8):
        n = S * B
        reqs = np.zeros(n, dtype=abi.REQUEST_DTYPE)
        refs = np.full(n, -1)
        kinds = rng.integers(1, 5, n)
        for i in range(n):
            r = reqs[i]
            r["timestamp"] = 1_000_000 + batch * n + i
            r["payload"][:8] = np.frombuffer(rng.bytes(8), np.uint8)
            r["request_type"] = kinds[i]
            a, b = rng.integers(0, len(pool), 2)
            r["auth_identity"] = np.frombuffer(pool[a], np.uint8)
            r["recipient"] = np.frombuffer(pool[b], np.uint8)
            if kinds[i] in (2, 4) and rng.random() < 0.5:
                continue  # next-message op, zero id
            if kinds[i] != 1 and ids_single:
                k = int(rng.integers(0, len(ids_single)))
                refs[i] = k
                snd, rcp = owners[k]
                r["auth_identity"] = np.frombuffer(snd if rng.random() < 0.5 else rcp, np.uint8)
                r["recipient"] = np.frombuffer(rcp, np.uint8)
            elif kinds[i] != 1:
                r["msg_id"][0] = 1
        r_single, r_cluster = reqs.copy(), reqs.copy()
        for i in np.nonzero(refs >= 0)[0]:
            r_single[i]["msg_id"] = np.frombuffer(ids_single[refs[i]], np.uint8)
            r_cluster[i]["msg_id"] = np.frombuffer(ids_cluster[refs[i]], np.uint8)
        shed = shed_mask(cl.config, r_cluster, B)
        n_shed += int(shed.sum())
        r_single["request_type"][shed] = 0
        o1 = single.process_batch(r_single)
        o2 = cl.process_batch(r_cluster)
        assert o2 is not None
        assert (o2["status_code"][shed] == abi.STATUS_CODE_INTERNAL_ERROR).all(), batch
        assert (o2["record"]["timestamp"][shed] == r_cluster["timestamp"][shed]).all(), batch
        o1["status_code"][shed] = abi.STATUS_CODE_INTERNAL_ERROR
        o1["record"]["timestamp"][shed] = r_cluster["timestamp"][shed]
        assert np.array_equal(o1["status_code"], o2["status_code"]), batch
        for f in ("sender", "recipient", "timestamp", "payload"):
            assert np.array_equal(o1["record"][f], o2["record"][f]), (batch, f)
        for i in np.nonzero((kinds == 1) & (o1["status_code"] == 1))[0]:
            ids_single.append(bytes(o1[i]["record"]["msg_id"]))
            ids_cluster.append(bytes(o2[i]["record"]["msg_id"]))
            owners.append((bytes(reqs[i]["auth_identity"]), bytes(reqs[i]["recipient"])))
    assert single.messages == cl.messages > 0
    assert single.mailboxes == cl.mailboxes
    assert n_shed > 0  # the cap was exercised


def test_bucket_overflow_rejects_whole_batch():
    """A source whose requests for one shard exceed C (many recipients, none
    past its cap) fails the whole batch: nothing is applied anywhere."""
    S = 4
    cfg = cluster_cfg(S, C=320)
    cl = ffi.Cluster(cfg)
    cl.seed(21)
    p = ffi.gen_params(n_identities=300)
    assert cl.process_batch(cl.gen_batch(S * 1024, p)) is not None
    before = [cl.shard(k).digest() for k in range(S)]
    msgs = cl.messages
    batch = cl.gen_batch(S * 1024, p)
    pool = cl.gen_batch(16 * 1024, ffi.gen_params(create=100, read=0, update=0, delete=0,
                                                  n_identities=4000))
    d0 = pool[ffi.route(cfg, pool) == 0]
    assert len(d0) >= 400
    batch[:400] = d0[:400]  # source 0: 400 creates for shard 0 > C = 320
    assert not shed_mask(cfg, batch, 1024)[:400].any()
    assert cl.process_batch(batch) is None
    assert [cl.shard(k).digest() for k in range(S)] == before and cl.messages == msgs


def test_hot_recipient_is_shed_not_rejected():
    """A source that sends 60 % of its window to one recipient no longer fails
    the batch for everyone (README.md:78-84; DESIGN.md §6 "Hot keys"): its
    first ROUTE_KEY_CAP creates for that recipient are routed, the rest are
    answered INTERNAL_ERROR with their time, and every other request is
    answered as the unsharded store answers it (with the shed ones turned into
    hard errors)."""
    S = 4
    cfg = cluster_cfg(S, C=320)
    cl = ffi.Cluster(cfg)
    cl.seed(21)
    p = ffi.gen_params(n_identities=300)
    assert cl.process_batch(cl.gen_batch(S * 1024, p)) is not None
    hot = cl.gen_batch(S * 1024, ffi.gen_params(create=100, read=0, update=0, delete=0, hot=60,
                                                n_identities=300))
    shed = shed_mask(cfg, hot, 1024)
    assert shed.sum() > S * 400
    msgs = cl.messages
    out = cl.process_batch(hot)
    assert out is not None
    assert (out["status_code"][shed] == abi.STATUS_CODE_INTERNAL_ERROR).all()
    assert (out["record"]["timestamp"][shed] == hot["timestamp"][shed]).all()
    assert not out["record"]["payload"][shed].any() and not out["record"]["sender"][shed].any()
    ok = out["status_code"] == 1
    assert ok[~shed].sum() > 0 and not ok[shed].any()
    assert cl.messages == msgs + int(ok.sum())

@pytest.mark.parametrize("S", [4, 8])
def test_realistic_traffic_is_never_shed(S):
    """The routing-key cap (DESIGN.md §6 "Hot keys") changes what a client
    sees only when one source window sends more than ROUTE_KEY_CAP requests to
    one mailbox or id: the unsharded store never sheds, so a shed request is a
    client-visible deviation (INTERNAL_ERROR where the reference would have
    processed it).  On realistic traffic (the bench's mix over many
    identities, BASELINE config 3's 64K-request windows split over the
    sources) nothing is shed, so sharded and unsharded stores answer alike."""
    B = 8192
    cl = ffi.Cluster(cluster_cfg(S, N=1 << 16, B=B, Q=64, Sr=64))
    cl.seed(40 + S)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=20000)
    mix = ffi.gen_params(n_identities=20000)
    for batch in range(5):
        reqs = cl.gen_batch(S * B, fill if batch < 2 else mix)
        assert not shed_mask(cl.config, reqs, B).any(), batch
        out = cl.process_batch(reqs)
        assert out is not None
        assert not (out["status_code"] == abi.STATUS_CODE_INTERNAL_ERROR).any(), batch


HOT_MIXES = {  # tools/oblivious_probe.py's hot mixes: every op on one recipient, no ids
    "hot_create": dict(create=100, read=0, update=0, delete=0, hot=100),
    "hot_next": dict(create=30, read=35, update=0, delete=35, nxt=100, hot=100),
    "hot_next_rud": dict(create=0, read=50, update=0, delete=50, nxt=100, hot=100),
}


@pytest.mark.parametrize("mix", sorted(HOT_MIXES))
def test_hot_window_deviation_is_confined_to_shed_keys(mix):
    """The sharded store's one semantic deviation from the unsharded store
    ("What's missing" 5; DESIGN.md §6 "Hot keys"), pinned
    against the unmodified unsharded model: the same hot window goes to both.
    Every shed request is answered differently (INTERNAL_ERROR), and every
    other answer that differs belongs to a later request with the same routing
    key as a shed one (it sees the store without the shed request's effect).
    A window of hot creates differs in exactly the shed requests: past the 62-
    message limit the unsharded store refuses them too."""
    S, B = 4, 1024
    single = ffi.Model(abi.make_config(1 << 16, mailbox_partitions=64, mailbox_partition_slots=64,
                                       max_batch=S * B))
    cl = ffi.Cluster(cluster_cfg(S, N=1 << 15, B=B, Q=32, Sr=64, C=B))
    single.seed(77)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=300)
    for _ in range(2):
        r = single.gen_batch(S * B, fill)
        single.process_batch(r)
        assert cl.process_batch(r) is not None
    p = ffi.gen_params(n_identities=300, bad_auth=0, bad_recipient=0, hard_error=0, zero_recipient=0,
                       **{"miss": 0, **HOT_MIXES[mix]})
    n_shed = n_confined = 0
    for _ in range(3):
        reqs = single.gen_batch(S * B, p)
        shed = ffi.route_shed(cl.config, reqs, B)
        key = ffi.route_key(cl.config, reqs)
        o1, o2 = single.process_batch(reqs), cl.process_batch(reqs)
        assert o2 is not None
        diff = o1["status_code"] != o2["status_code"]
        for f in ("sender", "recipient", "timestamp", "payload"):
            diff |= (o1["record"][f] != o2["record"][f]).reshape(len(reqs), -1).any(axis=1)
        assert (o2["status_code"][shed] == abi.STATUS_CODE_INTERNAL_ERROR).all()
        assert diff[shed].all()
        first_shed = {}
        for i in np.nonzero(shed)[0]:
            first_shed.setdefault(int(key[i]), int(i))
        for i in np.nonzero(diff & ~shed)[0]:
            k = int(key[i])
            assert k in first_shed and first_shed[k] < i, (mix, int(i))
            n_confined += 1
        if mix == "hot_create":
            assert np.array_equal(diff, shed)
        n_shed += int(shed.sum())
    assert n_shed > 0
    if mix == "hot_create":
        assert n_confined == 0
