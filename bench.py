#!/usr/bin/env python3
"""Benchmark: oblivious CRUD requests/s of the gvstore engine (BASELINE.json metric).

One "step" = one batch of B synthetic requests through the whole pipeline
(mailbox pass, allocation, message-table pass, mailbox write pass) with the
requests already resident in HBM.  Default workload = BASELINE config 3:
2^24 stored-message capacity prefilled to 75 %, 64K-request batches, a
25/25/25/25 CREATE/READ/UPDATE/DELETE mix with half of the READ/DELETE asking
for the next message (zero id), as SURVEY.md §8(d) specifies.

Multi-GPU (`torch.distributed.run`): one process per GPU, each owning one
shard of a single sharded store (gvs_create_sharded).  Every
rank submits its own 64K-request batch per step; the engine routes each
request to the shard that owns it inside fixed-size padded sub-batches over
RCCL send/recv (xGMI) and returns the responses to the submitting rank.
Per-GPU work is fixed as N grows (2^24 messages and 64K requests per GPU):
weak scaling.  Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from srcsha import source_sha  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md:36
# vector-ALU issue peak: 256 CUs x 4 SIMDs, one wave64 instruction per SIMD per
# 2 cycles (MI355X_MICROARCH.md:54), at the 2.4 GHz max clock (:34)
VALU_PEAK_GINST = 256 * 4 / 2 * 2.4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--log2n", type=int, default=24, help="log2 message capacity per GPU")
    p.add_argument("--batch", type=int, default=65536)
    p.add_argument("--fill", type=float, default=0.75)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline instances (host threads); 0 = this process's CPU share")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--host-steps", type=int, default=8,
                   help="batches timed through the host API (gvs_process_batches) after the device run")
    p.add_argument("--wire-steps", type=int, default=3,
                   help="batches through the device wire path (decode, store, encode); 0 = skip")
    p.add_argument("--routed", action="store_true",
                   help="N=1: use the sharded store's routed path (one shard over RCCL)")
    p.add_argument("--auth", action="store_true",
                   help="authenticated storage (AES-CTR sealed rows with a MAC per row, BASELINE config 5 mode)")
    p.add_argument("--sealed-waves", type=int, default=0, choices=(0, 4, 8, 12),
                   help="--auth: waves per workgroup of the sealed message pass (0: the store's choice)")
    p.add_argument("--mailbox-slots", type=int, default=256,
                   help="mailbox rows per partition (gvs_config.mailbox_partition_slots; R = N/16 either way)")
    p.add_argument("--expiry", type=int, default=0,
                   help="expiry sweep: X deletes per batch (DESIGN.md §9); each batch then carries "
                        "batch - X requests and every prefilled message is past the cutoff")
    p.add_argument("--predict-shards", type=int, default=0,
                   help="S > 1: time one GPU holding all S shards of a sharded store (in-process "
                        "transport, S x the per-GPU load) and print the predicted per-GPU step of an "
                        "S-GPU run instead of the normal line")
    p.add_argument("--xgmi-gbs", type=float, default=153.0,
                   help="--predict-shards: assumed xGMI rate per peer link and direction (GB/s); the "
                        "default is SURVEY.md §8(e)'s link budget (7 links x ~153 GB/s per GPU), not a "
                        "measured RCCL rate: no multi-GPU box has run here")
    p.add_argument("--prediction-json", default=os.path.join(ROOT, "profiles", "scale_prediction.json"))
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    p.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "valu_auth_latest.json"))
    p.add_argument("--valu-mix-json", default=os.path.join(ROOT, "profiles", "valu_mix_k_spass.json"))
    return p.parse_args()


def gen_batches(torch, dev, B, count, known, pool, g, ts0):
    """Synthetic request slabs (B x 1040 bytes, gvs_request layout) on `dev`."""
    out = []
    nk = known.shape[0]
    for b in range(count):
        r = torch.empty((B, 1040), dtype=torch.uint8, device=dev)
        r[:, :1024] = torch.randint(0, 256, (B, 1024), dtype=torch.uint8, device=dev, generator=g)
        r[:, 1024:] = 0
        roll = torch.randint(0, 100, (B,), device=dev, generator=g)
        typ = torch.where(roll < 25, 1, torch.where(roll < 50, 2, torch.where(roll < 75, 3, 4)))
        nxt = (torch.randint(0, 100, (B,), device=dev, generator=g) < 50) & ((typ == 2) | (typ == 4))
        byid = (typ != 1) & ~nxt
        k = torch.randint(0, nk, (B,), device=dev, generator=g)
        kn = known[k]  # (B, 80): id, sender, recipient
        coin = torch.randint(0, 2, (B, 1), device=dev, generator=g).bool()
        auth_byid = torch.where(coin, kn[:, 16:48], kn[:, 48:80])
        pi = torch.randint(0, pool.shape[0], (B, 2), device=dev, generator=g)
        auth = torch.where(byid[:, None], auth_byid, pool[pi[:, 0]])
        auth = torch.where(nxt[:, None], kn[:, 48:80], auth)
        rcpt = torch.where(byid[:, None], kn[:, 48:80], pool[pi[:, 1]])
        mid = torch.where(byid[:, None], kn[:, 0:16], r[:, 0:16])
        mid = torch.where(nxt[:, None], torch.zeros_like(mid), mid)
        r[:, 0:16] = mid
        r[:, 16:48] = auth
        r[:, 48:80] = rcpt
        ts = torch.arange(B, device=dev, dtype=torch.int64) + ts0 + b * B + 1
        r[:, 80:88] = ts.view(torch.uint8).reshape(B, 8)
        r[:, 1024:1028] = typ.to(torch.int32).view(torch.uint8).reshape(B, 4)
        out.append(r)
    return out


def prefill(torch, store, dev, B, target, pool, g, ts0, per_batch=None):
    """Fill the store with `target` creates through the normal pipeline; returns
    (id, sender, recipient) of every created message (device tensor n x 80)."""
    known = []
    done = 0
    d_out = torch.empty((B, 1040), dtype=torch.uint8, device=dev)
    while done < target:
        n = min(per_batch or B, target - done)
        r = torch.empty((n, 1040), dtype=torch.uint8, device=dev)
        r[:, :1024] = torch.randint(0, 256, (n, 1024), dtype=torch.uint8, device=dev, generator=g)
        r[:, 1024:] = 0
        pi = torch.randint(0, pool.shape[0], (n, 2), device=dev, generator=g)
        r[:, 16:48] = pool[pi[:, 0]]
        r[:, 48:80] = pool[pi[:, 1]]
        ts = torch.arange(n, device=dev, dtype=torch.int64) + ts0 + done + 1
        r[:, 80:88] = ts.view(torch.uint8).reshape(n, 8)
        r[:, 1024] = 1
        torch.cuda.synchronize(dev)
        store.process_batch_device(r.data_ptr(), n, d_out.data_ptr())
        ok = d_out[:n, 1024] == 1
        known.append(d_out[:n][ok][:, 0:80].clone())
        done += n
    return torch.cat(known)


def check_batch(torch, r, o):
    """Properties every response of one batch must have, checked
    on the device after the timed region: a successful CREATE echoes the
    request with a fresh nonzero id; a successful by-id op returns the record of
    the id it named, an UPDATE with the request's payload and time; every
    successful response names the caller as sender or recipient (the recipient,
    for next-message ops); a failure carries nothing but the request's time.
    Returns (violations, creates ok, deletes ok)."""
    typ = r[:, 1024:1028].contiguous().view(torch.int32).flatten()
    st = o[:, 1024:1028].contiguous().view(torch.int32).flatten()
    ok = st == 1
    mid_zero = (r[:, 0:16] == 0).all(1)
    auth, rrcpt = r[:, 16:48], r[:, 48:80]
    osnd, orcpt = o[:, 16:48], o[:, 48:80]
    eq = lambda a, b: (a == b).all(1)
    bad = torch.zeros_like(ok)
    cre = ok & (typ == 1)
    bad |= cre & ~(eq(osnd, auth) & eq(orcpt, rrcpt) & eq(o[:, 80:1024], r[:, 80:1024]) &
                   ~(o[:, 0:16] == 0).all(1))
    byid = ok & (typ != 1) & ~mid_zero
    bad |= byid & ~eq(o[:, 0:16], r[:, 0:16])
    bad |= byid & ~(eq(osnd, auth) | eq(orcpt, auth))
    upd = ok & (typ == 3)
    bad |= upd & ~eq(o[:, 80:1024], r[:, 80:1024])
    nxt = ok & ((typ == 2) | (typ == 4)) & mid_zero
    bad |= nxt & ~eq(orcpt, auth)
    fail = (st >= 2) & (st <= 7)
    bad |= fail & ~((o[:, 0:80] == 0).all(1) & eq(o[:, 80:88], r[:, 80:88]) & (o[:, 88:1024] == 0).all(1))
    bad |= (st < 0) | (st > 7)
    dels = ok & (typ == 4)
    return int(bad.sum()), int(cre.sum()), int(dels.sum())


def host_cpu():
    """CPU model, the machine's logical CPUs and this process's CPU share."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    # the GPU box runs one GPU's share of the host (OMP_NUM_THREADS = 16 there):
    # os.cpu_count() reports the whole machine, so the share caps the workers
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or affinity
    mem = None
    try:
        with open("/proc/meminfo") as f:
            mem = round(int(next(x for x in f if x.startswith("MemTotal")).split()[1]) / 2**20, 1)
    except (OSError, StopIteration, ValueError):
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "affinity": affinity,
            "share": min(share, affinity), "mem_gib": mem}


def c1_single_thread():
    """BASELINE config 1 as specified: the CPU reference path restated
    (oracle/gvs_pathoram.c), 2^16 message capacity, a seeded 10K
    create/read/delete mix (40/40/20, half of the reads and deletes by id, half
    next-message), on one thread.  Returns requests/s."""
    from grapevine_amd import abi
    from oracle import ffi
    cfg = abi.make_config(1 << 16)
    seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
    seq.seed(0x6772617065 + 1)
    mix = ffi.gen_params(create=40, read=40, update=0, delete=20, nxt=50, n_identities=1 << 12)
    left, ops, t = 10000, 0, 0.0
    while left:
        r = seq.gen_batch(min(left, cfg.max_batch), mix)
        t0 = time.perf_counter()
        oram.process_batch(r)
        t += time.perf_counter() - t0
        seq.process_batch(r)
        ops += len(r)
        left -= len(r)
    oram.close()
    seq.close()
    return ops / t


def c3_single_instance(budget_s):
    """One Path ORAM + cuckoo instance at the headline capacity, 2^24 messages
    (BASELINE config 3's table), on one thread, C3 mix: the restatement of
    cpu_baseline() without the reduced tree height.  Its tree arrays are lazy
    anonymous mappings (oracle/gvs_pathoram.c tree_zalloc), so host memory
    grows only with the paths the sample visits; the first touch of those
    pages (minor faults, counted) is inside the timed accesses.  The prefill
    is one 2048-create batch (the instance runs ~500 accesses/s)."""
    import resource
    from grapevine_amd import abi
    from oracle import ffi
    cfg = abi.make_config(1 << 24, max_batch=65536)
    mix = ffi.gen_params(create=25, read=25, update=25, delete=25, nxt=50, miss=0, bad_auth=0,
                         bad_recipient=0, hard_error=0, zero_recipient=0, n_identities=1 << 12)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=1 << 12)
    seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
    seq.seed(0x6772617065 + 24)
    r = seq.gen_batch(2048, fill)
    seq.process_batch(r)
    oram.process_batch(r)
    ops, t = 0, 0.0
    f0 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
    while t < budget_s:
        r = seq.gen_batch(512, mix)
        t0 = time.perf_counter()
        oram.process_batch(r)
        t += time.perf_counter() - t0
        seq.process_batch(r)
        ops += len(r)
    faults = resource.getrusage(resource.RUSAGE_SELF).ru_minflt - f0
    oram.close()
    seq.close()
    return {"value": ops / t, "unit": "req/s", "cores": 1, "capacity": 1 << 24, "requests": ops,
            "seconds": round(t, 2), "minor_faults_per_request": round(faults / max(ops, 1), 1),
            "peak_rss_gib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 1)}


def cpu_baseline(budget_s, threads):
    """The reference's CPU path, restated: the grapevine handler over Path ORAM
    (oracle/gvs_pathoram.c: CuckooHashTables over Path ORAM, Z = 4, recursive
    position map, 6 ORAM accesses per request, every block move an aligned cmov
    over every stash and branch slot, Circuit-ORAM style eviction along the
    accessed branch and one reverse-lexicographic path), cross-checked bit-for-bit against the sequential model in
    tests/test_pathoram.py.  One independent instance per host thread of this
    process's CPU share (the reference's maps are single-owner, &mut self);
    each is prefilled through its own accesses and then times the C3 mix for
    ~budget_s.  Also times BASELINE config 1 itself on one thread."""
    import threading
    from grapevine_amd import abi
    from oracle import ffi
    cpu = host_cpu()
    threads = threads or cpu["share"]
    c1 = c1_single_thread()
    c3 = c3_single_instance(budget_s)
    log2n = 18  # two cuckoo tables at 50 % load: ~2.7 GB per instance
    cfg = abi.make_config(1 << log2n, max_batch=65536)
    mix = ffi.gen_params(create=25, read=25, update=25, delete=25, nxt=50, miss=0, bad_auth=0,
                         bad_recipient=0, hard_error=0, zero_recipient=0, n_identities=1 << 14)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=1 << 14)
    res = [None] * threads

    def work(k):
        seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
        seq.seed(0x6772617065 + 3 + k)
        for _ in range(4):
            r = seq.gen_batch(4096, fill)
            seq.process_batch(r)
            oram.process_batch(r)
        ops, t = 0, 0.0
        while t < budget_s:
            r = seq.gen_batch(2048, mix)
            t0 = time.perf_counter()
            oram.process_batch(r)
            t += time.perf_counter() - t0
            seq.process_batch(r)
            ops += len(r)
        res[k] = (ops, t)
        oram.close()
        seq.close()

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ops = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": ops / wall, "unit": "req/s", "cores": threads, "kind": "port",
            "cpu_model": cpu["model"], "host_logical_cpus": cpu["logical_cpus"], "host_mem_gib": cpu["mem_gib"],
            "cpu_share": cpu["share"],
            "c1_single_thread_req_s": c1,
            "c3_capacity_single_thread": c3,
            "sample": f"PathORAM + CuckooHashTable restatement of the reference CPU path (oracle/gvs_pathoram.c; "
                      f"aligned-cmov block moves over every stash and branch slot, single-pass eviction), "
                      f"2^{log2n} capacity (tree height reduced from C3's 2^24 to bound memory), "
                      f"{threads} independent instances on {threads} host threads "
                      f"(this process's CPU share of {cpu['logical_cpus']} logical CPUs), C3 mix, "
                      f"{ops} requests in {wall:.1f}s; per-instance rate {ops / wall / threads:.0f} req/s; "
                      f"BASELINE config 1 (2^16, seeded 10K 40/40/20 create/read/delete) on one "
                      f"thread: {c1:.0f} req/s; one instance at the headline capacity 2^24 on one "
                      f"thread: {c3['value']:.0f} req/s ({c3['requests']} requests in {c3['seconds']} s, "
                      f"peak RSS {c3['peak_rss_gib']} GiB)"}


def front_end(torch, store, dev, batches, nreq, B):
    """The steps either side of the store on the device:
    wire QueryRequests -> decode -> store -> encode -> wire QueryResponses
    (gvs_process_wire_batch_device, no challenge check, so the store sees the
    same requests), and the batched schnorrkel check alone over B signatures
    (gvs_sr25519_verify_device).  The verifier runs the same instruction
    stream whatever its inputs, so random keys and signatures time it."""
    import numpy as np
    from grapevine_amd import abi, wire
    W_IN = 1104
    d_wires, d_lens, d_times = [], [], []
    for b in batches:
        q = b[:nreq].cpu().numpy().view(abi.REQUEST_DTYPE).reshape(-1).copy()
        q["request_type"][q["request_type"] == 0] = 0xFFFFFFFF  # still a hard error
        w = np.zeros((nreq, W_IN), np.uint8)
        w[:, :wire.REQUEST_WIRE_BYTES] = wire.encode_requests(q)
        d_wires.append(torch.from_numpy(w).to(dev))
        d_lens.append(torch.full((nreq,), wire.REQUEST_WIRE_BYTES, dtype=torch.int32, device=dev))
        d_times.append(torch.from_numpy(q["timestamp"].view(np.int64)).to(dev))
    d_out = torch.empty((nreq, wire.RESPONSE_WIRE_BYTES), dtype=torch.uint8, device=dev)
    d_olen = torch.empty((nreq,), dtype=torch.int32, device=dev)
    store.synchronize()
    torch.cuda.synchronize(dev)
    stage, lens = {}, None
    t0 = time.perf_counter()
    for i in range(len(batches)):
        store._check(store.lib.gvs_process_wire_batch_device(
            store.h, d_wires[i].data_ptr(), W_IN, d_lens[i].data_ptr(), nreq, d_times[i].data_ptr(),
            None, d_out.data_ptr(), wire.RESPONSE_WIRE_BYTES, d_olen.data_ptr(), None, None))
        for k, v in store.last_timings().items():
            stage[k] = stage.get(k, 0.0) + v
    store.synchronize()
    torch.cuda.synchronize(dev)
    t = time.perf_counter() - t0
    lens = torch.bincount(d_olen.to(torch.int64), minlength=1043)
    # the same path with the challenge check (random challenges: every signature
    # fails and every request becomes a hard error; the store does the same
    # fixed work for hard errors, so the timing stands for valid traffic)
    d_chal = torch.randint(0, 256, (nreq, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    stage_c = {}
    t0 = time.perf_counter()
    for i in range(len(batches)):
        store._check(store.lib.gvs_process_wire_batch_device(
            store.h, d_wires[i].data_ptr(), W_IN, d_lens[i].data_ptr(), nreq, d_times[i].data_ptr(),
            d_chal.data_ptr(), d_out.data_ptr(), wire.RESPONSE_WIRE_BYTES, d_olen.data_ptr(), None, None))
        for k, v in store.last_timings().items():
            stage_c[k] = stage_c.get(k, 0.0) + v
    store.synchronize()
    torch.cuda.synchronize(dev)
    t_c = time.perf_counter() - t0
    # the same requests from host memory, all batches in one double-buffered
    # call (gvs_process_wire_batches: uploads and downloads overlap the batches)
    import ctypes
    h_in = np.concatenate([w.cpu().numpy() for w in d_wires])
    h_lens = np.full(len(h_in), wire.REQUEST_WIRE_BYTES, np.uint32)
    h_times = np.concatenate([t.cpu().numpy() for t in d_times]).view(np.uint64)
    counts = np.full(len(batches), nreq, np.uint32)
    h_out = np.zeros((len(h_in), wire.RESPONSE_WIRE_BYTES), np.uint8)
    h_olen = np.zeros(len(h_in), np.uint32)
    applied = ctypes.c_uint32(0)

    h_chal = np.random.default_rng(7).integers(0, 256, (len(h_in), 32), dtype=np.uint8)

    def host_call(k, chal=None):
        store._check(store.lib.gvs_process_wire_batches(
            store.h, h_in.ctypes.data, W_IN, h_lens.ctypes.data, counts.ctypes.data, k,
            h_times.ctypes.data, None if chal is None else chal.ctypes.data, h_out.ctypes.data,
            wire.RESPONSE_WIRE_BYTES, h_olen.ctypes.data, None, ctypes.byref(applied)))
    host_call(1, h_chal)  # first use allocates the pipeline's buffers (and loads the verifier)
    store.synchronize()
    t0 = time.perf_counter()
    host_call(len(batches))
    store.synchronize()  # the last batch's deferred mailbox write pass, in the timed region
    t_h = time.perf_counter() - t0
    t0 = time.perf_counter()
    host_call(len(batches), h_chal)
    store.synchronize()
    t_hc = time.perf_counter() - t0
    # the same with the slabs in pinned memory (copied without staging)
    p_in = store.host_array(h_in.size, np.uint8).reshape(h_in.shape)
    p_out = store.host_array(h_out.size, np.uint8).reshape(h_out.shape)
    p_in[:] = h_in
    h_in, h_out = p_in, p_out
    host_call(1)
    store.synchronize()
    t0 = time.perf_counter()
    host_call(len(batches))
    store.synchronize()
    t_hp = time.perf_counter() - t0
    # batched signature check over B random (pk, 32-B challenge, signature)
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    pks = torch.randint(0, 256, (B, 32), dtype=torch.uint8, device=dev, generator=g)
    msgs = torch.randint(0, 256, (B, 32), dtype=torch.uint8, device=dev, generator=g)
    sigs = torch.randint(0, 256, (B, 64), dtype=torch.uint8, device=dev, generator=g)
    ok = torch.empty((B,), dtype=torch.int32, device=dev)
    ctx = b"grapevine-challenge"
    torch.cuda.synchronize(dev)
    ms = []
    for _ in range(3):
        store._check(store.lib.gvs_sr25519_verify_device(
            store.h, pks.data_ptr(), 32, msgs.data_ptr(), 32, 32, sigs.data_ptr(), 64, B, ctx, len(ctx),
            ok.data_ptr()))
        ms.append(store.last_timings().get("sr_verify", float("nan")))
    v_ms = min(ms)
    return {"wire_batch": {"value": nreq * len(batches) / t, "unit": "req/s",
                           "ms_per_batch": t / len(batches) * 1e3, "batches": len(batches),
                           "api": "gvs_process_wire_batch_device (1099-B QueryRequests in 1104-B slots, "
                                  "1042-B QueryResponses; no challenge check)",
                           "responses_1042B": int(lens[1042].item()), "responses_empty": int(lens[0].item()),
                           "stage_ms": {k: v / len(batches) for k, v in stage.items()}},
            "wire_batches_host": {"value": nreq * len(batches) / t_h, "unit": "req/s",
                                  "ms_per_batch": t_h / len(batches) * 1e3, "batches": len(batches),
                                  "api": "gvs_process_wire_batches (pageable host buffers, one call, "
                                         "double-buffered; PCIe-inclusive)",
                                  "responses_1042B": int((h_olen == 1042).sum()),
                                  "pinned_req_s": nreq * len(batches) / t_hp,
                                  "pinned_ms_per_batch": t_hp / len(batches) * 1e3},
            "wire_batches_host_checked": {"value": nreq * len(batches) / t_hc, "unit": "req/s",
                                          "ms_per_batch": t_hc / len(batches) * 1e3,
                                          "api": "gvs_process_wire_batches with per-request challenges "
                                                 "(decode, schnorrkel check, store, encode per batch)",
                                          "note": "random challenges: every signature fails (hard "
                                                  "errors); the store's work is fixed per batch"},
            "wire_batch_checked": {"value": nreq * len(batches) / t_c, "unit": "req/s",
                                   "ms_per_batch": t_c / len(batches) * 1e3,
                                   "api": "gvs_process_wire_batch_device with per-request challenges "
                                          "(decode, schnorrkel check, store, encode)",
                                   "note": "random challenges: every signature fails (hard errors); "
                                           "the store's work is fixed per batch",
                                   "stage_ms": {k: v / len(batches) for k, v in stage_c.items()}},
            "sr25519_verify": {"value": B / (v_ms * 1e-3), "unit": "signatures/s", "batch": B,
                               "ms": v_ms, "api": "gvs_sr25519_verify_device (context grapevine-challenge, "
                                                  "32-B messages; random inputs)"}}


def predict_shards(a, torch, dev, json_out):
    """Per-GPU step of an S-GPU run, measured on one GPU.  One process holds
    all S shards of a sharded store (gvs_create with shard_count = S: the same
    router, padded sub-batches and shard pipelines as the RCCL transport, the
    all-to-all done by device copies), each shard at the per-GPU size (2^log2n
    messages, 75 % full), and every call carries S x B requests, i.e. S sources
    of B each.  The GPU then does the work of all S ranks in series, so one
    rank's share is T / S; the xGMI exchange an S-GPU run adds is priced from
    its byte count at --xgmi-gbs per link and direction (the S - 1 peers in
    parallel, requests out and responses back)."""
    from grapevine_amd import abi
    from grapevine_amd.store import ObliviousStore
    S, N, B = a.predict_shards, 1 << a.log2n, a.batch
    cfg = abi.make_config(N, max_batch=B, device=0, shard_count=S)
    store = ObliviousStore(cfg)
    st0 = store.stats()
    C, SB = st0["route_capacity"], S * B
    g = torch.Generator(device=dev)
    g.manual_seed(0x6772617065 + 11)
    pool = torch.randint(0, 256, (S << 19, 32), dtype=torch.uint8, device=dev, generator=g)  # 2^19 per shard
    pool[:, 0] |= 1
    t0 = time.perf_counter()
    known = prefill(torch, store, dev, SB, int(N * a.fill) * S, pool, g, 1_700_000_000)
    t_fill = time.perf_counter() - t0
    batches = gen_batches(torch, dev, SB, a.warmup + a.steps, known, pool, g, 1_800_000_000)
    d_out = torch.empty((SB, 1040), dtype=torch.uint8, device=dev)
    for i in range(a.warmup):
        store.process_batch_device(batches[i].data_ptr(), SB, d_out.data_ptr())
    timed_in = torch.cat(batches[a.warmup:]).contiguous()
    timed_out = torch.empty((a.steps * SB, 1040), dtype=torch.uint8, device=dev)
    store.set_timing(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    store.process_batches_device(timed_in.data_ptr(), [SB] * a.steps, timed_out.data_ptr())
    torch.cuda.synchronize(dev)
    T = (time.perf_counter() - t0) / a.steps
    viol = sum(check_batch(torch, timed_in[i * SB:(i + 1) * SB], timed_out[i * SB:(i + 1) * SB])[0]
               for i in range(a.steps))
    slot = 1152
    xbytes = (S - 1) * C * slot  # per direction per rank: C slots to each of S - 1 peers
    x_ms = 2 * (C * slot) / (a.xgmi_gbs * 1e9) * 1e3  # peers in parallel, out and back
    st = store.stats()
    line = {"metric": "predicted per-GPU step of an S-GPU sharded run, measured on one GPU",
            "shards": S, "log2n_per_shard": a.log2n, "batch_per_source": B, "route_capacity": C,
            "source_sha": source_sha(),
            "shard_batch": st["shard_batch"], "steps": a.steps, "warmup": a.warmup,
            "inproc_ms_per_call": T * 1e3, "per_rank_compute_ms": T / S * 1e3,
            "xgmi_bytes_per_direction_per_rank": xbytes, "xgmi_gbs_assumed": a.xgmi_gbs,
            "xgmi_ms_out_and_back": x_ms,
            "predicted_per_gpu_step_ms": T / S * 1e3 + x_ms,
            "predicted_req_s_at_S": S * B / (T / S + x_ms * 1e-3),
            "predicted_req_s_per_gpu": B / (T / S + x_ms * 1e-3),
            "stage_ms_last_call": store.last_timings(), "violations": viol,
            "messages": st["messages"], "prefill_s": t_fill,
            "note": "the in-process call includes the router and the device-copy all-to-all of all S "
                    "sources; T / S is one rank's share"}
    json_out.write(json.dumps(line) + "\n")
    json_out.flush()
    store.close()


def main():
    a = parse()
    # RCCL prints a version banner on stdout at communicator creation; keep
    # stdout for the single JSON line and send everything else to stderr
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    from grapevine_amd import abi, dist as gdist
    from grapevine_amd.store import ObliviousStore

    from grapevine_amd.store import comm_unique_id

    ri = gdist.rank_info()
    world, rank, local = ri.world, ri.rank, ri.local
    if a.predict_shards > 1:
        return predict_shards(a, torch, torch.device("cuda", local), json_out)
    if world > 1:
        torch.cuda.set_device(local)
    gdist.init("nccl")  # torch's RCCL: comm-id broadcast, barriers, max-time reduction
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    N, B = 1 << a.log2n, a.batch
    if world > 1 or a.routed:
        # one shard per rank; the store's own RCCL communicator carries the data path
        cfg = abi.make_config(N, max_batch=B, device=local, shard_count=world, shard_index=rank,
                              auth_storage=a.auth, mailbox_partition_slots=a.mailbox_slots)
        cid = gdist.broadcast_bytes(ri, comm_unique_id() if rank == 0 else None, device=dev)
        store = ObliviousStore(cfg, comm_id=cid)
    else:
        cfg = abi.make_config(N, max_batch=B, device=local, auth_storage=a.auth,
                              expiry_per_batch=a.expiry, mailbox_partition_slots=a.mailbox_slots)
        store = ObliviousStore(cfg)
    shard_batch = store.stats()["shard_batch"]
    # what the data path spans, from the store's own RCCL communicator
    # (ncclCommCount / ncclCommUserRank; 0 / -1 without one), and every rank's
    # shard pipeline size and bucket capacity
    per_rank = gdist.gather_ints(ri, [store.get_option("rccl_ranks"), store.get_option("rccl_rank"),
                                      shard_batch, store.stats()["route_capacity"],
                                      store.get_option("txn_slots")], device=dev)
    if a.auth:
        store.set_option("sealed_pass_waves", a.sealed_waves)
    g = torch.Generator(device=dev)
    g.manual_seed(gdist.shard_seed(0x6772617065 + 3, rank))
    pool = torch.randint(0, 256, (1 << 19, 32), dtype=torch.uint8, device=dev, generator=g)
    pool[:, 0] |= 1
    known = prefill(torch, store, dev, B, int(N * a.fill), pool, g, 1_700_000_000,
                    per_batch=B - a.expiry)
    n_host = a.host_steps + (3 if a.host_steps else 0)  # pipelined, two one by one, one warm-up
    batches = gen_batches(torch, dev, B, a.warmup + a.steps + n_host + a.steps, known, pool, g,
                          1_800_000_000)
    one_by_one = batches[-a.steps:]  # the same API one call per batch, timed after the checks
    d_out = torch.empty((B, 1040), dtype=torch.uint8, device=dev)
    nreq = B - a.expiry  # requests per batch (the expiry deletes take the last X slots)
    # the timed batches back to back in one device array, submitted in one
    # call (gvs_process_batches_device: no host round trip between batches)
    timed_in = torch.cat([batches[a.warmup + i][:nreq] for i in range(a.steps)]).contiguous()
    timed_out = torch.empty((a.steps * nreq, 1040), dtype=torch.uint8, device=dev)
    d_outs = [timed_out[i * nreq:(i + 1) * nreq] for i in range(a.steps)]
    if a.expiry:
        store.set_expiry_cutoff(1_750_000_000)  # every prefilled message has expired
    store.set_timing(True)
    torch.cuda.synchronize(dev)
    for i in range(a.warmup):
        store.process_batch_device(batches[i].data_ptr(), nreq, d_out.data_ptr())
    torch.cuda.synchronize(dev)
    msgs_before = store.stats()["messages"]
    gdist.barrier(ri)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    store.process_batches_device(timed_in.data_ptr(), [nreq] * a.steps, timed_out.data_ptr())
    # the last batch's deferred mailbox write pass (gvs_synchronize): the timed
    # region holds exactly the K batches' work (stats() above ran the warm-up's)
    store.synchronize()
    torch.cuda.synchronize(dev)
    gdist.barrier(ri)
    torch.cuda.synchronize(dev)
    elapsed = gdist.max_over_ranks(ri, time.perf_counter() - t0, device=dev)
    # per-stage HIP-event times (and the message pass's, for the roofline):
    # the last timed batch's marks
    stage_ms = dict(store.last_timings())
    st = store.stats()
    d_out = d_outs[-1]
    statuses = torch.bincount(d_out[:, 1024].to(torch.int64), minlength=9)[:9].tolist()
    # response properties of every timed batch, and message conservation
    viol, n_cre, n_del = 0, 0, 0
    for i in range(a.steps):
        v, c, d = check_batch(torch, batches[a.warmup + i][:nreq], d_outs[i][:nreq])
        viol, n_cre, n_del = viol + v, n_cre + c, n_del + d
    expired = msgs_before + n_cre - n_del - st["messages"]
    checks = {"batches": a.steps, "violations": viol, "creates_ok": n_cre, "deletes_ok": n_del,
              "messages_before": msgs_before, "messages_after": st["messages"],
              "conserved": expired == 0 if not a.expiry else expired >= 0,
              "expired": expired}

    # for comparison: one gvs_process_batch_device call per batch (each call
    # waits for its batch's verdict before the next is enqueued)
    store.synchronize()
    gdist.barrier(ri)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for x in one_by_one:
        store.process_batch_device(x.data_ptr(), nreq, d_out.data_ptr())
    store.synchronize()
    torch.cuda.synchronize(dev)
    t_obo = gdist.max_over_ranks(ri, time.perf_counter() - t0, device=dev)
    per_batch_api = {"value": world * nreq * a.steps / t_obo, "unit": "req/s",
                     "ms_per_batch": t_obo / a.steps * 1e3,
                     "api": "gvs_process_batch_device, one call (and one host round trip) per batch"}

    host_path = None
    if a.host_steps:
        # the host API on batches in pageable host memory: gvs_process_batches
        # (pinned staging, copies on their own stream, double-buffered) and,
        # for comparison, gvs_process_batch one batch at a time
        import ctypes
        import numpy as np
        hb = [batches[a.warmup + a.steps + i][:nreq].cpu().numpy().view(abi.REQUEST_DTYPE).reshape(-1)
              for i in range(n_host)]
        # the caller's buffers exist (and are touched) before the call, as an
        # enclave's request/response arrays would: only the library call is timed
        reqs_all = np.ascontiguousarray(np.concatenate(hb[:a.host_steps]))
        out_all = np.ones(len(reqs_all), dtype=abi.RESPONSE_DTYPE)
        counts = np.full(a.host_steps, nreq, dtype=np.uint32)
        applied = ctypes.c_uint32(0)
        warm = np.ones(nreq, dtype=abi.RESPONSE_DTYPE)  # first call pins its staging buffers
        store._check(store.lib.gvs_process_batches(store.h, hb[-1].ctypes.data, counts.ctypes.data, 1,
                                                   warm.ctypes.data, ctypes.byref(applied)))
        store.synchronize()
        gdist.barrier(ri)
        t0 = time.perf_counter()
        store._check(store.lib.gvs_process_batches(store.h, reqs_all.ctypes.data, counts.ctypes.data,
                                                   a.host_steps, out_all.ctypes.data,
                                                   ctypes.byref(applied)))
        store.synchronize()
        t_pipe = gdist.max_over_ranks(ri, time.perf_counter() - t0, device=dev)
        one = [np.ones(nreq, dtype=abi.RESPONSE_DTYPE) for _ in hb[a.host_steps:-1]]
        gdist.barrier(ri)
        t0 = time.perf_counter()
        for x, o in zip(hb[a.host_steps:-1], one):
            store._check(store.lib.gvs_process_batch(store.h, x.ctypes.data, nreq, o.ctypes.data))
        store.synchronize()
        t_seq = gdist.max_over_ranks(ri, time.perf_counter() - t0, device=dev)
        # the same batches from caller buffers in pinned memory (gvs_host_alloc):
        # copied to and from the device directly, no staging
        pin_in = store.host_array(len(reqs_all), abi.REQUEST_DTYPE)
        pin_out = store.host_array(len(reqs_all), abi.RESPONSE_DTYPE)
        pin_in[:] = reqs_all
        pin_out[:] = out_all
        store.synchronize()
        gdist.barrier(ri)
        t0 = time.perf_counter()
        store._check(store.lib.gvs_process_batches(store.h, pin_in.ctypes.data, counts.ctypes.data,
                                                   a.host_steps, pin_out.ctypes.data,
                                                   ctypes.byref(applied)))
        store.synchronize()
        t_pin = gdist.max_over_ranks(ri, time.perf_counter() - t0, device=dev)
        host_path = {"value": world * nreq * a.host_steps / t_pipe, "unit": "req/s",
                     "batches": a.host_steps, "ms_per_batch": t_pipe / a.host_steps * 1e3,
                     "api": "gvs_process_batches (double-buffered, pinned staging)",
                     "one_by_one_req_s": world * nreq * 2 / t_seq,
                     "one_by_one_ms_per_batch": t_seq / 2 * 1e3,
                     "pinned_req_s": world * nreq * a.host_steps / t_pin,
                     "pinned_ms_per_batch": t_pin / a.host_steps * 1e3,
                     "note": "requests and responses in pageable host memory, PCIe and host copies included"}

    front = None
    if a.wire_steps and world == 1 and not a.routed:
        front = front_end(torch, store, dev,
                          gen_batches(torch, dev, B, a.wire_steps, known, pool, g, 1_900_000_000), nreq, B)

    if rank == 0:
        total = world * nreq * a.steps
        rpass_ms = stage_ms.get("rpass", float("nan"))
        # algorithmic bytes of one fixed-slot message-table pass:
        # every row read and written, and per transaction slot (W partitions x
        # c slots, whatever the batch holds) one 1 KiB final state read and one
        # 1 KiB snapshot written
        W = st["msg_partitions"]
        c = store.get_option("txn_slots")
        alg_bytes = 2 * N * 1024 + 2 * W * c * 1024
        # side figures from other runs are attached only when they were measured
        # on these kernel sources (tools/srcsha.py)
        src_sha = source_sha()
        achieved = alg_bytes / (rpass_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(a.traffic_json) as f:
                tj = json.load(f)
            # the pass's bytes depend on N, W and c only: attach
            # the file's figure when it was measured at the same N and slot
            # count, whatever the rank count
            if (tj.get("kernel") == "k_rpass2s" and tj.get("log2n") == a.log2n and not a.auth
                    and tj.get("expiry_per_batch", 0) == a.expiry and tj.get("source_sha") == src_sha
                    and tj.get("txn_slots", c if tj.get("batch") == B else None) == c):
                traffic = tj.get("rpass_bytes_per_launch")
        except (OSError, ValueError):
            pass
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "kernel": "k_rpass2s (fixed-schedule message-table pass)",
                    "txn_slots": c, "alg_bytes_per_launch": alg_bytes, "kernel_ms": rpass_ms}
        if a.auth:
            # sealed rows: the pass is bound by vector-ALU issue (AES + the row MAC),
            # DESIGN.md §8; SQ_INSTS_VALU per launch from a --pmc pass
            # (tools/valu_from_pmc.py) over the HIP-event kernel time
            insts = None
            try:
                with open(a.valu_json) as f:
                    vj = json.load(f)
                if (vj.get("log2n") == a.log2n and vj.get("batch") == B and vj.get("kernel") == "k_spass"
                        and vj.get("source_sha") == src_sha and not a.sealed_waves):
                    insts = vj.get("valu_insts_per_launch")
            except (OSError, ValueError):
                pass
            v_ach = insts / (rpass_ms * 1e-3) / 1e9 if insts else None
            # the ceiling of the pass's own instruction mix: three-source
            # operations issue 1.35-1.55x slower than the nominal rate
            # (tools/valu_mix_peak.py over tools/valu_rate_probe.hip)
            mix = None
            try:
                with open(a.valu_mix_json) as f:
                    mj = json.load(f)
                if mj.get("source_sha") == src_sha and not a.sealed_waves:
                    mix = {"ceiling": mj["ceiling_g_wave_instr_per_s"], "unit": "G wave-instr/s",
                           "frac": v_ach / mj["ceiling_g_wave_instr_per_s"] if v_ach else None,
                           "source": os.path.relpath(a.valu_mix_json, ROOT), "probe": mj.get("probe")}
            except (OSError, ValueError, KeyError):
                pass
            roofline = {"bound": "valu", "achieved": v_ach, "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                        "frac": v_ach / VALU_PEAK_GINST if v_ach else None, "traffic": None,
                        "mix_ceiling": mix,
                        "kernel": f"k_spass (fixed-schedule sealed message-table pass; "
                                  f"{a.sealed_waves or 'default'} waves per workgroup)",
                        "valu_insts_per_launch": insts, "kernel_ms": rpass_ms,
                        "hbm_achieved": achieved, "hbm_frac": achieved / HBM_PEAK_GBS,
                        "alg_bytes_per_launch": alg_bytes}
        cpu = None if a.no_cpu or world > 1 else cpu_baseline(a.cpu_seconds, a.cpu_threads)
        # the 8-GPU step as predicted from one GPU (bench.py --predict-shards 8,
        # profiles/scale_prediction.json), when measured at this size
        prediction = None
        try:
            with open(a.prediction_json) as f:
                pj = json.load(f)
            if (pj.get("log2n_per_shard") == a.log2n and pj.get("batch_per_source") == B
                    and pj.get("source_sha") == src_sha and not a.auth and not a.expiry):
                prediction = {k: pj[k] for k in ("shards", "predicted_per_gpu_step_ms", "predicted_req_s_at_S",
                                                 "per_rank_compute_ms", "xgmi_ms_out_and_back",
                                                 "xgmi_gbs_assumed", "route_capacity", "shard_batch")}
                prediction["source"] = os.path.relpath(a.prediction_json, ROOT)
        except (OSError, ValueError, KeyError):
            pass
        R = cfg.mailbox_partitions * cfg.mailbox_partition_slots
        batch_bytes = 2 * N * 1024 + 4 * R * 1024 + B * (1088 + 1088)
        batch_gbs = batch_bytes / (elapsed / a.steps) / 1e9
        line = {
            "metric": "oblivious CRUD req/s (node) at 2^24 msgs, 64K batch; % HBM peak",
            "value": total / elapsed,
            "unit": "req/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded on device): 75% prefill, 25/25/25/25 CRUD mix, 50% next-message reads/deletes",
            "config": {"workload": (f"C5 storage mode (AES-128-CTR sealed rows, AES + NH/UHASH-128 MAC on message rows, BLAKE2b on mailbox rows): " if a.auth else "C3: ")
                       + f"2^{a.log2n} message capacity per GPU, {B}-request batches",
                       "msg_capacity": N, "batch": B,
                       "mailboxes": cfg.mailbox_partitions * cfg.mailbox_partition_slots,
                       "mailbox_partition_slots": cfg.mailbox_partition_slots,
                       "parallelism": f"shards{world}",
                       "route_capacity": store.stats()["route_capacity"],
                       "shard_batch": shard_batch, "auth_storage": bool(a.auth),
                       "rccl_ranks": per_rank[0][0],
                       "per_rank": [{"rccl_rank": r[1], "rccl_ranks": r[0], "shard_batch": r[2],
                                     "route_capacity": r[3], "txn_slots": r[4]} for r in per_rank],
                       "expiry_per_batch": a.expiry,
                       "api": f"gvs_process_batches_device: the {a.steps} timed batches in one call"},
            "roofline": roofline,
            # SURVEY.md §8(d) whole-batch figure: message table and mailbox table
            # (read pass + write pass) read and written, requests in, responses out
            "batch_roofline": {"bytes": batch_bytes, "achieved": batch_gbs, "unit": "GB/s",
                               "frac": batch_gbs / HBM_PEAK_GBS,
                               "formula": "2*N*1024 + 4*R*1024 + B*(1088 + 1088), per ms_per_step"},
            "cpu_baseline": cpu,
            "per_batch_api": per_batch_api,
            "scaling_prediction": prediction,
            "host_path": host_path,
            "front_end": front,
            "checks": checks,
            "stage_ms": stage_ms,
            "store": {"messages": st["messages"], "mailboxes": st["mailboxes"],
                      "last_batch_status_hist": statuses},
        }
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    store.close()
    gdist.finalize(ri)


if __name__ == "__main__":
    main()
