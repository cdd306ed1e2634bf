"""N>1 path on CPU (gloo, world size 2 and 4): the sharded store's protocol of
DESIGN.md §6 run as one process per rank, with the oracle standing in for
each rank's shard pipeline.

Each rank owns shard `rank`.  Every step, each rank takes its own batch and
places each request with the engine's own router (gvs_route_plan of the test
library: the device's route_dest run on the host) into S buckets of exactly
C slots padded with zero requests; the placement is cross-checked against the
oracle's restatement (gvo_route).  The ranks agree on overflow with a MAX
all-reduce (the engine's error agreement): if any rank's bucket overflows,
every rank rejects the batch and nothing is applied, as the cluster model
says.  Otherwise the buckets go all_to_all, each rank runs its shard on the
S*C received slots (a shard pipeline of gvs_route_plan's size), the responses
return with a second all_to_all and are put back in request order.  The
result must equal the single-process cluster model on the concatenated
batch, rank by rank and bit for bit, and every shard's state must equal the
cluster's shard.  Timing follows bench.py (barrier, max over ranks)."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys, time, json
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from grapevine_amd import abi, dist as gdist, store as gstore
    from oracle import ffi
    ri = gdist.init("gloo")
    S, r, B = ri.world, ri.rank, 1024
    base = dict(mailbox_partitions=8, mailbox_partition_slots=32, max_batch=B, shard_count=S)
    ccfg = abi.make_config(4096, **base)
    replica = ffi.Cluster(ccfg)              # whole-store oracle, identical on every rank
    _, C, be, _ = gstore.route_plan(ccfg, np.zeros(0, dtype=abi.REQUEST_DTYPE))
    assert C == replica.capacity and be == ffi.shard_batch(S * C)
    scfg = abi.make_config(4096, **dict(base, max_batch=be, shard_index=r))
    shard = ffi.Model(scfg)                  # this rank's shard
    replica.seed(1234)
    p = ffi.gen_params(n_identities=300, hard_error=2, zero_recipient=2)
    hot = ffi.gen_params(create=100, read=0, update=0, delete=0, hot=70, n_identities=300)
    cre = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=4000)
    rec = abi.REQUEST_DTYPE.itemsize
    gdist.barrier(ri)
    t0 = time.perf_counter()
    checked = rejected = shed_seen = 0
    for step in range(6):
        glob = replica.gen_batch(S * B, p)       # every source's batch, concatenated
        if step == 2:
            # one source's batch is hot on one recipient: the requests past the
            # routing key's cap are shed (spread, answered INTERNAL_ERROR), and
            # the batch is applied
            glob[:B] = replica.gen_batch(B, hot)
        if step == 4:
            # one source sends only creates for shard 0, to many recipients
            # (none past its cap): its bucket overflows and every rank rejects
            pool = replica.gen_batch(8 * S * B, cre)
            d0 = pool[ffi.route(ccfg, pool) == 0]
            assert len(d0) >= B
            glob[:B] = d0[:B]
        want = replica.process_batch(glob)       # None: the cluster rejects the batch
        mine = glob[r * B:(r + 1) * B]
        slot, _, _, over, shed = gstore.route_plan(ccfg, mine, with_shed=True)
        dest = ffi.route(ccfg, mine)             # the oracle's restatement agrees
        dest[shed] = (np.arange(B) % S)[shed]    # shed requests are spread
        key = ffi.route_key(ccfg, mine)          # and its routing keys give the same shed set
        rank = np.zeros(B, dtype=np.int64)
        seen = {{}}
        for i in range(B):
            k = int(key[i])
            rank[i] = seen.get(k, 0)
            seen[k] = rank[i] + 1
        assert (shed == ((key & 3) != 0) & (rank >= ffi.ROUTE_KEY_CAP)).all()
        placed = slot != 0xFFFFFFFF
        assert (slot[placed] // C == dest[placed]).all()
        flag = torch.tensor([1 if over else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item():
            assert want is None and step == 4
            rejected += 1
            continue
        assert want is not None
        send = np.zeros(S * C, dtype=abi.REQUEST_DTYPE)
        send[slot] = mine
        send["request_type"][slot[shed]] = 0     # shed requests travel as hard errors
        recv = torch.empty(S * C * rec, dtype=torch.uint8)
        dist.all_to_all_single(recv, torch.from_numpy(send.view(np.uint8).copy()))
        sub = recv.numpy().view(abi.REQUEST_DTYPE)
        out = shard.process_batch(sub)           # pads are type 0: hard errors
        back = torch.empty(S * C * rec, dtype=torch.uint8)
        dist.all_to_all_single(back, torch.from_numpy(out.view(np.uint8).copy()))
        got = back.numpy().view(abi.RESPONSE_DTYPE)[slot].copy()
        got[shed] = np.zeros(1, dtype=abi.RESPONSE_DTYPE)
        got["status_code"][shed] = abi.STATUS_CODE_INTERNAL_ERROR
        got["record"]["timestamp"][shed] = mine["timestamp"][shed]
        assert got.tobytes() == want[r * B:(r + 1) * B].tobytes(), step
        shed_seen += int(shed.sum())
        checked += B
    el = gdist.max_over_ranks(ri, time.perf_counter() - t0)
    total = gdist.sum_over_ranks(ri, checked)
    rs = replica.shard(r)
    with open(os.path.join({out!r}, "rank%d.json" % r), "w") as f:
        json.dump(dict(rank=r, world=S, elapsed=el, total=total, capacity=C, rejected=rejected,
                       shed=gdist.sum_over_ranks(ri, shed_seen),
                       digest_ok=shard.digest() == rs.digest(),
                       messages=shard.messages, replica_messages=rs.messages,
                       cluster_messages=replica.messages), f)
    gdist.finalize(ri)
""")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_protocol_gloo(tmp_path, world):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, out=str(tmp_path)))
    for attempt in range(3):  # a free port can be taken between probe and bind
        port = free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port",
               str(port), str(script)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
        busy = "address already in use" in (r.stdout + r.stderr).lower() or "EADDRINUSE" in r.stderr
        if r.returncode == 0 or not busy:
            break
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(world)]
    assert sorted(x["rank"] for x in rows) == list(range(world))
    assert len({x["elapsed"] for x in rows}) == 1          # max over ranks, same everywhere
    assert all(x["total"] == world * 5 * 1024 for x in rows)  # weak scaling: work adds up
    assert all(x["rejected"] == 1 for x in rows)            # overflow agreed by every rank
    assert all(x["shed"] > 400 for x in rows)               # the hot source's excess was shed
    assert all(x["digest_ok"] for x in rows)
    assert all(x["messages"] == x["replica_messages"] for x in rows)
    assert sum(x["messages"] for x in rows) == rows[0]["cluster_messages"] > 0
