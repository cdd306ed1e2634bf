#!/usr/bin/env python3
"""Run a fixed schedule of batches with a chosen request mix (run under
rocprofv3 by tests/test_oblivious.py and tests/test_timing.py).  The prefill is
identical for every mix; only the last `--batches` batches differ.  Test
infrastructure: the oracle only generates realistic requests against the live
state and checks the responses.

    python tools/oblivious_probe.py MIX [--log2n L] [--batch B] [--auth]
                                        [--shards S] [--fill-batches F]

MIX may name several message-store mixes joined by '+': they then run
interleaved in one process (schedule(); the timing test's in-process
comparison).

--shards S > 1 runs the sharded store in its single-process form (S shards on
one device, the router kernels k_route_* and the padded all-to-all), against
the oracle's cluster model.

--oram / --omap run the block store or the key-value map instead, with the
op mixes of KV_MIXES (2^log2n blocks or rows, --batch ops per batch).

--expiry X turns the expiry sweep on (X records per batch; the
caller submits batch - X requests).  Its mixes run the main request mix and
differ in what has expired: x_none (no message), x_all (every message: each
swept partition finds rows), x_few (the oldest 16 (k + 1) messages at measured
batch k, consecutive slots: expired rows in a few partitions only).  The
prefill runs without a cutoff.

--wire runs every batch (prefill included) through gvs_process_wire_batch:
protobuf requests in 1200-B slots, decoded, their schnorrkel signatures
checked against per-request challenges, the store, responses encoded.  The
wire_* mixes are the main mix with every signature forged, every message
malformed, or every message in a non-canonical encoding.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from grapevine_amd import abi  # noqa: E402
from grapevine_amd.store import ObliviousStore  # noqa: E402
from oracle import ffi  # noqa: E402

MIXES = {
    "main": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "rud": dict(create=0, read=34, update=33, delete=33, nxt=50),
    "all_create": dict(create=100, read=0, update=0, delete=0),
    "all_miss_read": dict(create=0, read=100, update=0, delete=0, nxt=0, miss=100),
    "hot_next": dict(create=30, read=35, update=0, delete=35, nxt=100, hot=100),
    "hot_next_rud": dict(create=0, read=50, update=0, delete=50, nxt=100, hot=100),
    "deletes": dict(create=0, read=0, update=0, delete=100, nxt=30),
    # --wire only: the main mix, mutated on the wire
    "wire_forged": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "wire_malformed": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "wire_noncanonical": dict(create=25, read=25, update=25, delete=25, nxt=50),
    # --expiry only: the main mix, with nothing / everything / a few old rows expired
    "x_none": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "x_all": dict(create=25, read=25, update=25, delete=25, nxt=50),
    "x_few": dict(create=25, read=25, update=25, delete=25, nxt=50),
}
TS0 = 1_700_000_000  # timestamp of the generator's first request (oracle gvo_gen_batch)


def expiry_cutoff(mix, k):
    """Cutoff before measured batch k of an --expiry mix."""
    if mix == "x_all":
        return 1 << 62
    if mix == "x_few":
        return TS0 + 1 + 16 * (k + 1)  # request j of the run has time TS0 + 1 + j
    return 0
WIRE_STRIDE = 1200

# --oram / --omap (the block store and the key-value map):
# op mixes as (pool, op probabilities); pool "uniform" = every block / the
# prefilled keys, "hot" = 64 of them, "one" = a single block, "fresh" = keys
# never inserted
KV_MIXES = {
    "oram": {
        "main": ("uniform", 0.5), "all_read": ("uniform", 0.0), "all_write": ("uniform", 1.0),
        "hot": ("hot", 0.5), "chain": ("one", 0.5),
    },
    "omap": {
        "main": ("uniform", (0.3, 0.3, 0.25, 0.15)), "all_read": ("uniform", (1, 0, 0, 0)),
        "all_insert": ("fresh", (0, 0, 1, 0)), "all_remove": ("uniform", (0, 0, 0, 1)),
        "hot": ("hot", (0.3, 0.3, 0.25, 0.15)), "miss": ("fresh", (1, 0, 0, 0)),
    },
}
KV_SECRET = bytes((0x51 + 11 * i) & 0xFF for i in range(32))


def run_kv(a, kind):
    """The block store or the key-value map: a prefill identical in every
    process, then --batches batches per seed of the chosen mix, each checked
    bit-exact against the sequential oracle (oracle/gvs_kv.c)."""
    import numpy as np
    from grapevine_amd.store import BlockStore, KeyValueMap
    assert a.mix in KV_MIXES[kind], f"{kind} mixes: {sorted(KV_MIXES[kind])}"
    cap, B = 1 << a.log2n, a.batch
    cfg = abi.make_oram_config(cap, max_batch=B, secret_key=KV_SECRET, auth_storage=a.auth)
    if kind == "oram":
        store, model = BlockStore(cfg), ffi.OramModel(cap)
    else:
        store, model = KeyValueMap(cfg), ffi.OmapModel(cap, KV_SECRET)
    keys = np.random.default_rng(5).integers(0, 256, (cap // 8, 16), dtype=np.uint8)
    keys[:, 0] |= 1  # no all-zero key

    def ops_of(rng, pool, p):
        if kind == "oram":
            ops = np.zeros(B, dtype=abi.BLOCK_OP_DTYPE)
            blocks = {"uniform": np.arange(cap), "hot": np.arange(64) * 4099 % cap,
                      "one": np.array([77])}[pool]
            ops["index"] = rng.choice(blocks, B)
            ops["op"] = (rng.random(B) < p).astype(np.uint32)
            ops["data"] = rng.integers(0, 256, (B, 1024), dtype=np.uint8)
            return ops
        ops = np.zeros(B, dtype=abi.OMAP_OP_DTYPE)
        if pool == "fresh":
            k = rng.integers(0, 256, (B, 16), dtype=np.uint8)
            k[:, 0] |= 1
        else:
            k = (keys if pool == "uniform" else keys[:64])[rng.integers(0, len(keys) if pool == "uniform"
                                                                        else 64, B)]
        ops["key"] = k
        ops["op"] = rng.choice(4, B, p=p)
        ops["value"] = rng.integers(0, 256, (B, 1024), dtype=np.uint8)
        return ops

    def check(ops, what):
        got, want = store.access(ops), model.access(ops)
        if not a.no_check:
            assert got.tobytes() == want.tobytes(), f"parity failure inside the probe ({what})"

    rng = np.random.default_rng(77)
    for _ in range(a.fill_batches):  # writes / inserts of the key pool
        check(ops_of(rng, "uniform", 1.0 if kind == "oram" else (0, 0, 1, 0)), "prefill")
    pool, p = KV_MIXES[kind][a.mix]
    seeds = [int(x) for x in a.seeds.split(",") if x] or [a.seed]
    for sd in seeds:
        rng = np.random.default_rng(sd)
        for _ in range(a.batches):
            check(ops_of(rng, pool, p), a.mix)
    store.close()
    model.close()
    print("probe ok", kind, a.mix)


class WirePath:
    """Requests as signed wire messages (test infrastructure: 64 ristretto keys,
    each with one pre-signed challenge; identities map to keys in order of
    first appearance, so every process maps them the same way)."""

    def __init__(self, store, model, n_keys):
        import random
        import numpy as np
        from oracle import sr25519 as sr
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import wire_cases
        self.store, self.model, self.wc = store, model, wire_cases
        # one key per identity; generated once per box (seeded), then cached
        cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gvs_probe_keys_{n_keys}.npy")
        if os.path.exists(cache):
            raw = np.load(cache)
        else:
            rng = random.Random(5)
            rows = []
            for _ in range(n_keys):
                x = rng.randrange(1, sr.L)
                chal = rng.randbytes(32)
                rows.append(sr.public_key(x) + chal + sr.sign(x, chal, rng.randrange(1, sr.L)))
            raw = np.frombuffer(b"".join(rows), np.uint8).reshape(n_keys, 128)
            np.save(cache + ".tmp.npy", raw)
            os.replace(cache + ".tmp.npy", cache)
        self.keys = [(bytes(r[:32]), bytes(r[32:64]), bytes(r[64:])) for r in raw]
        self.idmap = {}
        self.rng = random.Random(9)

    def key_of(self, v):
        if v not in self.idmap:
            self.idmap[v] = len(self.idmap) % len(self.keys)
        return self.idmap[v]

    def run(self, reqs, mix):
        import numpy as np
        from grapevine_amd import wire
        msgs, chal, valid = [], [], []
        for q in reqs:
            a0 = bytes(q["auth_identity"])
            k = self.key_of(a0) if any(a0) else None
            for f in ("recipient", "auth_identity"):
                v = bytes(q[f])
                if any(v):
                    q[f] = np.frombuffer(self.keys[self.key_of(v)][0], np.uint8)
            pk, c, sig = self.keys[k] if k is not None else (bytes(32), bytes(32), bytes(64))
            if mix == "wire_forged":
                sig = bytes([sig[0] ^ 1]) + sig[1:]
            f = dict(rt=int(q["request_type"]), auth=bytes(q["auth_identity"]), sig=sig,
                     id=bytes(q["msg_id"]), rc=bytes(q["recipient"]), pl=bytes(q["payload"]))
            m = self.wc.canonical(f)
            if mix == "wire_malformed":
                m = m[:self.rng.randrange(1, len(m))]
            elif mix == "wire_noncanonical":
                m = self.wc.ld(4, self.wc.record(f, (3, 1, 2))) + self.wc.fx64(10, 7) + m[:105]
            msgs.append(m)
            chal.append(c)
            valid.append(k is not None and mix != "wire_forged")
        times = reqs["timestamp"].copy()
        q, _, st = wire.decode_requests(msgs, timestamps=times, strict=False)
        for i in range(len(q)):
            if st[i] == 0 and not valid[i]:
                q[i]["request_type"] = 0
        want = [wire.encode_response(r) for r in self.model.process_batch(q)]
        got, _, _ = self.store.process_wire_batch(
            msgs, times, in_stride=WIRE_STRIDE,
            challenges=np.frombuffer(b"".join(chal), np.uint8).reshape(-1, 32))
        assert got == want, "parity failure inside the probe (wire path)"
        if mix == "main":
            assert sum(1 for r in got if r) > len(got) // 2, "wire prefill: most requests must verify"


def schedule(mix, seeds, per_seed, rotate=0):
    """The measured batches as (mix, seed, reseed before it, index of the batch
    among its mix's).  One mix: per_seed batches per seed.  An interleaved run
    (MIX = 'a+b+c', tests/test_timing.py) runs every mix in one process: for
    seed number s the mixes in the order rotated by s + rotate, per_seed batches
    each, the generator reseeded before each mix's batches, so every mix sees
    the same draws and the order of the mixes is balanced over the seeds."""
    mixes = mix.split("+")
    out, cnt = [], {m: 0 for m in mixes}
    for si, sd in enumerate(seeds):
        r = (si + rotate) % len(mixes)
        for m in mixes[r:] + mixes[:r]:
            for b in range(per_seed):
                out.append((m, sd, b == 0, cnt[m]))
                cnt[m] += 1
    return out


def mix_arg(v):
    names = set(MIXES) | set(KV_MIXES["oram"]) | set(KV_MIXES["omap"])
    if not v or any(m not in names for m in v.split("+")):
        raise argparse.ArgumentTypeError(f"a mix, or mixes joined by '+', of {sorted(names)}")
    return v


def main():
    p = argparse.ArgumentParser()
    p.add_argument("mix", type=mix_arg, help="a mix, or mixes joined by '+' (interleaved in one process)")
    p.add_argument("--rotate", type=int, default=0, help="interleaved runs: rotation of the mix order")
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--batches", type=int, default=3)
    p.add_argument("--fill-batches", type=int, default=4)
    p.add_argument("--shards", type=int, default=0)
    p.add_argument("--identities", type=int, default=5000)
    p.add_argument("--auth", action="store_true", help="authenticated storage (DESIGN.md §8)")
    p.add_argument("--wire", action="store_true", help="wire path with challenge check")
    p.add_argument("--expiry", type=int, default=0, help="expiry records per batch (x_* mixes)")
    p.add_argument("--pinned", action="store_true",
                   help="requests and responses in pinned host memory (gvs_host_alloc) through "
                        "gvs_process_batches: no pageable transfer between the batches' kernels")
    p.add_argument("--seed", type=int, default=1234, help="generator seed of the measured batches")
    p.add_argument("--seeds", default="",
                   help="comma-separated seeds: the measured batches are --batches per seed, the "
                        "generator reseeded before each seed's batches (seed-controlled runs)")
    p.add_argument("--no-check", action="store_true",
                   help="skip the parity asserts of the measured batches (GVS_DIAG variants)")
    p.add_argument("--oram", action="store_true", help="the block store (gvs_oram_*)")
    p.add_argument("--omap", action="store_true", help="the key-value map (gvs_omap_*)")
    a = p.parse_args()
    if a.oram or a.omap:
        assert "+" not in a.mix, "interleaved runs are for the message store"
        return run_kv(a, "oram" if a.oram else "omap")
    for m in a.mix.split("+"):
        assert a.wire or not m.startswith("wire_"), "wire_* mixes need --wire"
        assert bool(a.expiry) == m.startswith("x_") or (a.expiry and m == "main"), \
            "x_* mixes need --expiry (and --expiry takes x_* mixes or main)"
        assert m in MIXES, f"{m}: not a message-store mix"
    S = a.shards if a.shards > 1 else 0
    cfg = abi.make_config(1 << a.log2n, max_batch=a.batch, auth_storage=a.auth, shard_count=S,
                          expiry_per_batch=a.expiry)
    store = ObliviousStore(cfg)
    model = ffi.Cluster(cfg) if S else ffi.Model(cfg)
    n = a.batch * (S or 1) - (0 if S else a.expiry)
    model.seed(77)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=a.identities)
    wp = WirePath(store, model, a.identities) if a.wire else None
    if a.pinned:
        pin_in, pin_out = store.host_array(n, abi.REQUEST_DTYPE), store.host_array(n, abi.RESPONSE_DTYPE)

        def run(reqs):
            # one batch through gvs_process_batches from pinned buffers
            pin_in[:len(reqs)] = reqs
            counts = np.array([len(reqs)], np.uint32)
            applied = ctypes.c_uint32(0)
            store._check(store.lib.gvs_process_batches(store.h, pin_in.ctypes.data, counts.ctypes.data, 1,
                                                       pin_out.ctypes.data, ctypes.byref(applied)))
            return pin_out[:len(reqs)].copy()
    else:
        run = store.process_batch
    for _ in range(a.fill_batches):
        reqs = model.gen_batch(n, fill)
        if wp:
            wp.run(reqs, "main")
            continue
        want = model.process_batch(reqs)
        got = run(reqs)
        assert a.no_check or got.tobytes() == want.tobytes(), "parity failure inside the probe (prefill)"
    seeds = [int(x) for x in a.seeds.split(",") if x] or [a.seed]
    for k, (mix, sd, fresh, kx) in enumerate(schedule(a.mix, seeds, a.batches, a.rotate)):
        if fresh:
            model.seed(sd)  # same request-generator state for every mix
        if a.expiry:
            cut = expiry_cutoff(mix, kx)
            model.set_expiry_cutoff(cut)
            store.set_expiry_cutoff(cut)
        params = ffi.gen_params(n_identities=a.identities, bad_auth=0, bad_recipient=0, hard_error=0,
                                zero_recipient=0, **{"miss": 0, **MIXES[mix]})
        reqs = model.gen_batch(n, params)
        if wp:
            wp.run(reqs, mix)
            continue
        want = model.process_batch(reqs)
        got = run(reqs)
        assert a.no_check or got.tobytes() == want.tobytes(), f"parity failure inside the probe ({mix})"
    # no gvs_synchronize / gvs_get_stats here: they run the last batch's
    # deferred mailbox write pass (k_m2x), a launch after the last batch that
    # the traces would count in it; every batch was checked on return
    print("probe ok", a.mix, model.messages)


if __name__ == "__main__":
    main()
