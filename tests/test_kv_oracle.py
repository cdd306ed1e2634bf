"""CPU: the block-store oracle (oracle/gvs_kv.c) against a plain-Python
restatement of ORAM::access semantics (ops in order; each op sees the block
before its own write; an invalid op rejects the batch)."""
import numpy as np

from grapevine_amd import abi
from oracle import ffi


def random_ops(rng, n, capacity, hot=None, p_write=0.5):
    ops = np.zeros(n, dtype=abi.BLOCK_OP_DTYPE)
    pool = np.arange(capacity) if hot is None else rng.choice(capacity, hot, replace=False)
    ops["index"] = rng.choice(pool, n)
    ops["op"] = (rng.random(n) < p_write).astype(np.uint32)
    ops["data"] = rng.integers(0, 256, (n, 1024), dtype=np.uint8)
    return ops


def py_access(blocks, ops):
    out = []
    for o in ops:
        i = int(o["index"])
        out.append(blocks.get(i, bytes(1024)))
        if o["op"] == abi.ORAM_WRITE:
            blocks[i] = o["data"].tobytes()
    return out


def test_oram_oracle_matches_python_model():
    rng = np.random.default_rng(7)
    cap = 4096
    m = ffi.OramModel(cap)
    ref = {}
    for b in range(5):
        ops = random_ops(rng, 1024, cap, hot=300 if b % 2 else None)
        got = m.access(ops)
        want = py_access(ref, ops)
        assert got is not None
        assert [bytes(r) for r in got] == want, f"batch {b}"
    blocks = m.blocks()
    for i in range(cap):
        assert blocks[i].tobytes() == ref.get(i, bytes(1024))
    m.close()


def test_oram_oracle_rejects_invalid_batch_whole():
    rng = np.random.default_rng(8)
    m = ffi.OramModel(4096)
    ops = random_ops(rng, 64, 4096, p_write=1.0)
    before = m.blocks().copy()
    bad = ops.copy()
    bad[10]["index"] = 4096
    assert m.access(bad) is None
    bad = ops.copy()
    bad[3]["op"] = 2
    assert m.access(bad) is None
    assert (m.blocks() == before).all()
    assert m.access(ops) is not None
    m.close()


# ---------------------------------------------------------------- key-value map

SECRET = bytes((0x29 + 13 * i) & 0xFF for i in range(32))


def map_layout(capacity):
    S = min(max(capacity // 4096, 256), 4096, capacity)
    W = capacity // S
    return W, S, W.bit_length() - 1


def random_map_ops(rng, n, pool, p_ops=(0.3, 0.3, 0.25, 0.15), p_invalid=0.02):
    ops = np.zeros(n, dtype=abi.OMAP_OP_DTYPE)
    ops["key"] = pool[rng.integers(0, len(pool), n)]
    ops["key"][rng.random(n) < p_invalid] = 0
    ops["op"] = rng.choice(4, n, p=p_ops)
    ops["value"] = rng.integers(0, 256, (n, 1024), dtype=np.uint8)
    return ops


def key_pool(rng, k):
    pool = rng.integers(0, 256, (k, 16), dtype=np.uint8)
    pool[:, 0] |= 1
    return pool


class PyMap:
    """Plain-Python restatement of include/gvstore.h's map semantics."""

    def __init__(self, capacity, secret):
        self.W, self.S, self.logW = map_layout(capacity)
        self.secret = secret
        self.d = {}

    def part(self, key):
        hi, lo = ffi.omap_hash(self.secret, key)
        return (hi >> (64 - self.logW)) if self.logW else 0, (hi, lo & ~0xFFFFF)

    def access(self, ops):
        used = {}
        for k in self.d:
            q = self.part(k)[0]
            used[q] = used.get(q, 0) + 1
        new = {}
        for o in ops:
            k = o["key"].tobytes()
            if k == bytes(16) or k in self.d:
                continue
            if o["op"] in (abi.OMAP_WRITE, abi.OMAP_INSERT):
                new[k] = self.part(k)
        admitted = set()
        for q in set(v[0] for v in new.values()):
            ks = sorted((v[1], k) for k, v in new.items() if v[0] == q)
            free = self.S - used.get(q, 0)
            admitted |= {k for _, k in ks[:free]}
        out = []
        state = {}
        for o in ops:
            k = o["key"].tobytes()
            if k == bytes(16):
                out.append((abi.OMAP_INVALID_KEY, bytes(1024)))
                continue
            e, v = state.get(k, (k in self.d, self.d.get(k, bytes(1024))))
            op = int(o["op"])
            val = o["value"].tobytes()
            if e:
                out.append((abi.OMAP_FOUND, v))
                if op == abi.OMAP_WRITE:
                    v = val
                if op == abi.OMAP_REMOVE:
                    e, v = False, bytes(1024)
            elif op in (abi.OMAP_READ, abi.OMAP_REMOVE):
                out.append((abi.OMAP_NOT_FOUND, bytes(1024)))
            elif k not in admitted and k not in self.d:  # a present key keeps its row
                out.append((abi.OMAP_OVERFLOW, bytes(1024)))
            else:
                out.append((abi.OMAP_NOT_FOUND, val if op == abi.OMAP_INSERT else bytes(1024)))
                e, v = True, val
            state[k] = (e, v)
        for k, (e, v) in state.items():
            if e:
                self.d[k] = v
            else:
                self.d.pop(k, None)
        return out


def check_map(got, want):
    assert len(got) == len(want)
    for i, (st, v) in enumerate(want):
        assert int(got[i]["status"]) == st, (i, int(got[i]["status"]), st)
        assert got[i]["value"].tobytes() == v, i


def test_map_oracle_matches_python_model():
    rng = np.random.default_rng(21)
    cap = 4096
    m, ref = ffi.OmapModel(cap, SECRET), PyMap(cap, SECRET)
    pool = key_pool(rng, 600)
    for b in range(6):
        ops = random_map_ops(rng, 1024, pool)
        check_map(m.access(ops), ref.access(ops))
    assert m.size() == len(ref.d)
    m.close()


def test_map_oracle_overflow_admission():
    """One partition of 256 rows (capacity 4096 -> 16 partitions), far more new
    keys than rows: admission in hash order, the rest OMAP_OVERFLOW."""
    rng = np.random.default_rng(22)
    cap = 4096
    m, ref = ffi.OmapModel(cap, SECRET), PyMap(cap, SECRET)
    pool = key_pool(rng, 20000)
    for b in range(6):
        ops = random_map_ops(rng, 4096, pool, p_ops=(0.1, 0.4, 0.45, 0.05))
        got = m.access(ops)
        check_map(got, ref.access(ops))
    assert (got["status"] == abi.OMAP_OVERFLOW).sum() > 100
    assert m.size() == len(ref.d) <= cap
    m.close()


def test_map_oracle_rejects_unknown_op():
    rng = np.random.default_rng(23)
    m = ffi.OmapModel(4096, SECRET)
    ops = random_map_ops(rng, 10, key_pool(rng, 5))
    ops[3]["op"] = 9
    assert m.access(ops) is None
    assert m.size() == 0
