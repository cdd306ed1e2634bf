"""N>1 path on CPU (gloo, world size 2): each rank owns an independent shard
and serves its own seeded stream; the job time is the max over ranks and the
aggregate is the sum (what bench.py does over RCCL on GPUs)."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys, time, json
    sys.path.insert(0, {root!r})
    from grapevine_amd import abi, dist as gdist
    from oracle import ffi
    ri = gdist.init("gloo")
    cfg = abi.make_config(4096, mailbox_partitions=8, mailbox_partition_slots=32, max_batch=1024)
    shard = ffi.Model(cfg)                       # this rank's shard (CPU stand-in)
    shard.seed(gdist.shard_seed(1234, ri.rank))
    p = ffi.gen_params(n_identities=300)
    gdist.barrier(ri)
    t0 = time.perf_counter()
    ok = 0
    for _ in range(3):
        out = shard.process_batch(shard.gen_batch(512, p))
        ok += int((out["status_code"] == 1).sum())
    el = gdist.max_over_ranks(ri, time.perf_counter() - t0 + 0.01 * ri.rank)
    total = gdist.sum_over_ranks(ri, 3 * 512)
    oks = gdist.sum_over_ranks(ri, ok)
    with open(os.path.join({out!r}, "rank%d.json" % ri.rank), "w") as f:
        json.dump(dict(rank=ri.rank, world=ri.world, elapsed=el, total=total, oks=oks,
                       digest=shard.digest(), local_ok=ok), f)
    gdist.finalize(ri)
""")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_gloo(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, out=str(tmp_path)))
    for attempt in range(3):  # a free port can be taken between probe and bind
        port = free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
        busy = "address already in use" in (r.stdout + r.stderr).lower() or "EADDRINUSE" in r.stderr
        if r.returncode == 0 or not busy:
            break
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    rows = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    assert sorted(x["rank"] for x in rows) == [0, 1]
    a, b = rows
    assert a["world"] == b["world"] == 2
    assert a["elapsed"] == b["elapsed"]              # max over ranks, same on both
    assert a["total"] == b["total"] == 2 * 3 * 512   # weak scaling: work adds up
    assert a["oks"] == a["local_ok"] + b["local_ok"]
    assert a["digest"] != b["digest"]                # independent shards, different streams
