"""GPU parity of the sharded store against the oracle's cluster
model (oracle/gvs_oracle.c gvo_cluster_*), bit for bit: responses, per-shard
message tables, live counts.

The single-GPU box runs the S-shard store in its single-process form (all
shards on one device, the all-to-all done with device copies), which drives
the same router, padded sub-batches and shard pipelines as the multi-process
form; the RCCL transport itself is exercised with one rank (send/recv to
self, error max-reduction)."""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import GvsError, ObliviousStore, comm_unique_id
from oracle import ffi

from parity import diff_responses, run_stream

pytestmark = pytest.mark.gpu


def sharded_pair(S, N=4096, B=1024, Q=16, Sr=32, C=0):
    cfg = abi.make_config(N, mailbox_partitions=Q, mailbox_partition_slots=Sr, max_batch=B,
                          shard_count=S, route_capacity=C)
    return ObliviousStore(cfg), ffi.Cluster(cfg)


@pytest.mark.parametrize("S", [2, 4])
def test_local_shards_mixed_stream(S):
    store, cl = sharded_pair(S)
    cl.seed(40 + S)
    st = store.stats()
    assert st["shards"] == S and st["route_capacity"] == cl.capacity
    seen = run_stream(store, cl, ffi.gen_params(n_identities=400, hard_error=2, zero_recipient=2),
                      batches=8, n=S * 1024)
    assert {0, 1, 2, 4} <= set(seen), seen


def test_local_shards_partial_batches():
    S = 4
    store, cl = sharded_pair(S)
    cl.seed(47)
    p = ffi.gen_params(n_identities=300)
    for n in (S * 1024, 1, 1500, 3 * 1024 + 5, 0, S * 1024):
        reqs = cl.gen_batch(n, p)
        want = cl.process_batch(reqs)
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"n={n}: " + "\n".join(d)
    assert store.stats()["messages"] == cl.messages


def test_local_shards_drain_and_capacity():
    S = 2
    store, cl = sharded_pair(S, N=1024, Q=4, Sr=64, C=1024)
    cl.seed(48)
    run_stream(store, cl, ffi.gen_params(create=95, read=5, update=0, delete=0, n_identities=150),
               batches=3, n=S * 1024)
    run_stream(store, cl, ffi.gen_params(create=5, read=30, update=15, delete=50, nxt=70,
                                         n_identities=150), batches=4, n=S * 1024)


def test_local_shards_bucket_overflow_applies_nothing():
    """One source sends more requests for one shard than C (many recipients,
    none past its routing key's cap): the whole batch fails on every shard."""
    S = 4
    store, cl = sharded_pair(S, C=320)
    cl.seed(49)
    run_stream(store, cl, ffi.gen_params(n_identities=300), batches=2, n=S * 1024)
    before = store.dump_messages()
    msgs = store.stats()["messages"]
    batch = cl.gen_batch(S * 1024, ffi.gen_params(n_identities=300))
    pool = cl.gen_batch(16 * 1024, ffi.gen_params(create=100, read=0, update=0, delete=0,
                                                  n_identities=4000))
    d0 = pool[ffi.route(cl.config, pool) == 0]
    batch[:400] = d0[:400]  # source 0: 400 creates for shard 0 > C = 320
    assert cl.process_batch(batch) is None
    with pytest.raises(GvsError) as ei:
        store.process_batch(batch)
    assert ei.value.code == abi.GVS_ERR_BATCH_OVERFLOW
    assert store.stats()["messages"] == msgs
    assert store.dump_messages().tobytes() == before.tobytes()
    # the store keeps working after a rejected batch
    run_stream(store, cl, ffi.gen_params(n_identities=300), batches=2, n=S * 1024)


@pytest.mark.parametrize("mix", ["hot_create", "hot_next", "hot_next_rud"])
def test_local_shards_hot_recipient_is_shed(mix):
    """A hot recipient (60-100 % of a source's window on one mailbox) no
    longer overflows its bucket: the requests past the routing key's cap are
    shed (spread to other shards as hard errors, answered INTERNAL_ERROR with
    their time) and the batch is applied, bit for bit as the cluster model
    says (DESIGN.md §6 "Hot keys")."""
    S = 4
    store, cl = sharded_pair(S)  # the default C: mean + 8 sigma + 64 covers the cap's 2 x 64
    cl.seed(53)
    run_stream(store, cl, ffi.gen_params(n_identities=300), batches=3, n=S * 1024)
    p = {"hot_create": ffi.gen_params(create=100, read=0, update=0, delete=0, hot=60, n_identities=300),
         "hot_next": ffi.gen_params(create=30, read=35, update=0, delete=35, nxt=100, hot=100,
                                    n_identities=300),
         "hot_next_rud": ffi.gen_params(create=0, read=50, update=0, delete=50, nxt=100, hot=100,
                                        n_identities=300)}[mix]
    for b in range(3):
        reqs = cl.gen_batch(S * 1024, p)
        want = cl.process_batch(reqs)
        assert want is not None
        assert (want["status_code"] == abi.STATUS_CODE_INTERNAL_ERROR).sum() > S * 100
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"batch {b}: " + "\n".join(d)
        assert store.stats()["messages"] == cl.messages
    assert store.dump_messages().shape[0] > 0


def test_rccl_single_rank_routed_path():
    """gvs_create_sharded with one rank: router, RCCL send/recv to self and the
    error all-reduce on the data path; must equal the unsharded oracle."""
    import os
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          shard_count=1, shard_index=0)
    store = ObliviousStore(cfg, comm_id=comm_unique_id())
    model = ffi.Model(abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32,
                                      max_batch=1024))
    model.seed(50)
    run_stream(store, model, ffi.gen_params(n_identities=300), batches=6, n=1024)
    store.close()


def test_local_shards_pipeline_not_a_power_of_two():
    """S*C = 2 x 9024 routed slots: the shard pipeline is 24576 ops (a multiple
    of the sort tiles, not the next power of two 32768), so the sorts run
    their non-power-of-two network and the table passes a ragged batch."""
    S, B = 2, 16384
    store, cl = sharded_pair(S, N=1 << 16, B=B, Q=64, Sr=64)
    st = store.stats()
    assert st["shard_batch"] == ffi.shard_batch(S * cl.capacity) == 24576
    cl.seed(51)
    run_stream(store, cl, ffi.gen_params(n_identities=3000), batches=4, n=S * B)
    run_stream(store, cl, ffi.gen_params(n_identities=3000), batches=1, n=S * B - 777)


def test_rccl_single_rank_with_expiry():
    """gvs_create_sharded with one rank and expiry: the X expiry slots sit after
    the routed ones (shard_batch(C + X)), never over a client's request."""
    import os
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    X, B = 128, 1024
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=B,
                          shard_count=1, shard_index=0, expiry_per_batch=X)
    store = ObliviousStore(cfg, comm_id=comm_unique_id())
    cl = ffi.Cluster(cfg)
    st = store.stats()
    assert st["shard_batch"] == ffi.shard_batch(cl.capacity + X) >= B + X
    cl.seed(52)
    p = ffi.gen_params(create=40, read=20, update=20, delete=20, n_identities=200)
    for b in range(8):
        cutoff = 1_700_000_000 + max(0, cl.ops - 1500) if b >= 2 else 0
        cl.set_expiry_cutoff(cutoff)
        store.set_expiry_cutoff(cutoff)
        reqs = cl.gen_batch(B, p)  # a full batch: expiry takes no client slot
        d = diff_responses(store.process_batch(reqs), cl.process_batch(reqs), reqs)
        assert not d, f"batch {b}: " + "\n".join(d)
        assert store.stats()["messages"] == cl.messages
    store.close()
