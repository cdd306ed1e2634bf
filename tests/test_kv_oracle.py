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
