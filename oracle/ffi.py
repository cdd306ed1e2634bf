"""ctypes binding of oracle/libgvs_oracle.so (test infrastructure only)."""
import ctypes
import os
import subprocess

import numpy as np

from grapevine_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class GenParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "pct_create", "pct_read", "pct_update", "pct_delete", "pct_next", "pct_miss",
        "pct_bad_auth", "pct_bad_recipient", "pct_hard_error", "pct_zero_recipient",
        "pct_hot", "n_identities")] + [("ts_base", ctypes.c_uint64)]


def gen_params(create=25, read=25, update=25, delete=25, nxt=50, miss=10, bad_auth=5,
               bad_recipient=5, hard_error=1, zero_recipient=1, hot=0, n_identities=1000,
               ts_base=1_700_000_000):
    return GenParams(create, read, update, delete, nxt, miss, bad_auth, bad_recipient,
                     hard_error, zero_recipient, hot, n_identities, ts_base)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libgvs_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.gvo_siphash24.argtypes = [u64, u64, ctypes.c_char_p, ctypes.c_size_t]
        L.gvo_siphash24.restype = u64
        L.gvo_id_encode.argtypes = [ctypes.c_char_p, u32, u64, ctypes.c_char_p]
        L.gvo_id_decode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, u64,
                                    ctypes.POINTER(u32), ctypes.POINTER(u64)]
        L.gvo_id_decode.restype = ctypes.c_int
        L.gvo_recipient_hash.argtypes = [ctypes.c_char_p, ctypes.c_char_p,
                                         ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.gvo_create.argtypes = [ctypes.POINTER(abi.GvsConfig)]
        L.gvo_create.restype = vp
        L.gvo_destroy.argtypes = [vp]
        L.gvo_process_batch.argtypes = [vp, vp, u32, vp]
        L.gvo_process_batch.restype = ctypes.c_int
        L.gvo_apply_one.argtypes = [vp, vp, vp]
        L.gvo_set_expiry_cutoff.argtypes = [vp, u64]
        for f in ("gvo_messages", "gvo_mailboxes", "gvo_creation_counter", "gvo_state_digest"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = u64
        L.gvo_dump_messages.argtypes = [vp, vp, u64]
        L.gvo_dump_messages.restype = ctypes.c_int
        L.gvo_live_message.argtypes = [vp, u64, vp]
        L.gvo_live_message.restype = ctypes.c_int
        L.gvo_identity.argtypes = [u32, ctypes.c_char_p]
        L.gvp_create.argtypes = [ctypes.POINTER(abi.GvsConfig)]
        L.gvp_create.restype = vp
        L.gvp_destroy.argtypes = [vp]
        L.gvp_process_batch.argtypes = [vp, vp, u32, vp]
        L.gvp_process_batch.restype = ctypes.c_int
        for f in ("gvp_messages", "gvp_mailboxes", "gvp_oram_accesses"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = u64
        L.gvo_gen_batch.argtypes = [vp, ctypes.POINTER(GenParams), ctypes.POINTER(u64), vp, u32, u64]
        cp = ctypes.c_char_p
        L.gvo_aes128_expand.argtypes = [cp, cp]
        L.gvo_aes128_encrypt.argtypes = [cp, cp, cp]
        L.gvo_blake2b.argtypes = [cp, ctypes.c_size_t, cp, cp, ctypes.c_size_t, cp, ctypes.c_size_t]
        L.gvo_storage_keys.argtypes = [cp, cp, cp]
        L.gvo_oram_create.argtypes = [u64]
        L.gvo_oram_create.restype = vp
        L.gvo_oram_destroy.argtypes = [vp]
        L.gvo_oram_access_batch.argtypes = [vp, vp, u32, vp]
        L.gvo_oram_access_batch.restype = ctypes.c_int
        L.gvo_oram_read_all.argtypes = [vp, vp]
        L.gvo_omap_create.argtypes = [u64, ctypes.c_char_p]
        L.gvo_omap_create.restype = vp
        L.gvo_omap_destroy.argtypes = [vp]
        L.gvo_omap_access_batch.argtypes = [vp, vp, u32, vp]
        L.gvo_omap_access_batch.restype = ctypes.c_int
        L.gvo_omap_size.argtypes = [vp]
        L.gvo_omap_size.restype = u64
        L.gvo_omap_hash.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.gvo_seal_row.argtypes = [cp, u32, u64, u32, cp, cp, cp, cp, cp]
        L.gvo_uhash_keys.argtypes = [cp, vp, vp, vp]
        L.gvo_row_hash.argtypes = [vp, vp, vp, cp, cp]
        L.gvo_id_encode_shard.argtypes = [ctypes.c_char_p, u32, u32, u64, ctypes.c_char_p]
        L.gvo_id_decode_shard.argtypes = [ctypes.c_char_p, ctypes.c_char_p, u64, u32,
                                          ctypes.POINTER(u32), ctypes.POINTER(u32),
                                          ctypes.POINTER(u64)]
        L.gvo_id_decode_shard.restype = ctypes.c_int
        L.gvo_route.argtypes = [ctypes.c_char_p, vp, u32, u32, u64]
        L.gvo_route.restype = u32
        L.gvo_route_key.argtypes = [ctypes.c_char_p, vp]
        L.gvo_route_key.restype = u32
        L.gvo_route_capacity.argtypes = [u32, u32]
        L.gvo_route_capacity.restype = u32
        L.gvo_cluster_create.argtypes = [ctypes.POINTER(abi.GvsConfig)]
        L.gvo_cluster_create.restype = vp
        L.gvo_cluster_destroy.argtypes = [vp]
        L.gvo_cluster_capacity.argtypes = [vp]
        L.gvo_cluster_capacity.restype = u32
        L.gvo_cluster_shard.argtypes = [vp, u32]
        L.gvo_cluster_shard.restype = vp
        L.gvo_cluster_process.argtypes = [vp, vp, u32, vp]
        L.gvo_cluster_process.restype = ctypes.c_int
        L.gvo_cluster_set_expiry_cutoff.argtypes = [vp, u64]
        L.gvo_shard_batch.argtypes = [u64]
        L.gvo_shard_batch.restype = u32
        for f in ("gvo_cluster_messages", "gvo_cluster_mailboxes"):
            getattr(L, f).argtypes = [vp]
            getattr(L, f).restype = u64
        L.gvo_cluster_gen_batch.argtypes = [vp, ctypes.POINTER(GenParams), ctypes.POINTER(u64),
                                            vp, u32, u64]
        _LIB = L
    return _LIB


def siphash24(key16: bytes, msg: bytes) -> int:
    k0 = int.from_bytes(key16[:8], "little")
    k1 = int.from_bytes(key16[8:16], "little")
    return lib().gvo_siphash24(k0, k1, msg, len(msg))


def id_encode(key16: bytes, slot: int, ctr: int) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().gvo_id_encode(key16, slot, ctr, out)
    return out.raw


def id_decode(key16: bytes, msg_id: bytes, n_slots: int):
    s, c = ctypes.c_uint32(), ctypes.c_uint64()
    ok = lib().gvo_id_decode(key16, msg_id, n_slots, ctypes.byref(s), ctypes.byref(c))
    return (s.value, c.value) if ok else None


def id_encode_shard(key16: bytes, shard: int, slot: int, ctr: int) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().gvo_id_encode_shard(key16, shard, slot, ctr, out)
    return out.raw


def id_decode_shard(key16: bytes, msg_id: bytes, n_slots: int, n_shards: int):
    sh, s, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    ok = lib().gvo_id_decode_shard(key16, msg_id, n_slots, n_shards, ctypes.byref(sh),
                                   ctypes.byref(s), ctypes.byref(c))
    return (sh.value, s.value, c.value) if ok else None


def route(config, reqs):
    """Owning shard of each request (index i = position in its source batch)."""
    reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
    key = bytes(config.secret_key)
    B = config.max_batch
    return np.array([lib().gvo_route(key, reqs[i:i + 1].ctypes.data, i % B, config.shard_count,
                                     config.msg_capacity) for i in range(len(reqs))],
                    dtype=np.uint32)


def route_key(config, reqs):
    """Routing key of each request (gvo_route_key; low 2 bits 0 = unkeyed)."""
    reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
    key = bytes(config.secret_key)
    return np.array([lib().gvo_route_key(key, reqs[i:i + 1].ctypes.data) for i in range(len(reqs))],
                    dtype=np.uint32)


ROUTE_KEY_CAP = 64  # gvo_oracle.h GVO_ROUTE_KEY_CAP


def route_shed(config, reqs, B=None):
    """The requests the router sheds (gvs_route.h, DESIGN.md §6 "Hot keys"):
    in each source window of B (default: the config's max_batch), those past
    the ROUTE_KEY_CAP-th of their routing key; unkeyed requests never."""
    B = B or config.max_batch
    key = route_key(config, reqs)
    shed = np.zeros(len(reqs), dtype=bool)
    for s0 in range(0, len(reqs), B):
        seen = {}
        for i in range(s0, min(len(reqs), s0 + B)):
            k = int(key[i])
            shed[i] = (k & 3) != 0 and seen.get(k, 0) >= ROUTE_KEY_CAP
            seen[k] = seen.get(k, 0) + 1
    return shed


def route_capacity(batch, n_shards):
    return lib().gvo_route_capacity(batch, n_shards)


def shard_batch(slots):
    """Ops per shard pipeline for `slots` routed slots plus expiry deletes."""
    return lib().gvo_shard_batch(slots)


def aes128_encrypt(key16: bytes, block16: bytes) -> bytes:
    rk = ctypes.create_string_buffer(176)
    lib().gvo_aes128_expand(key16, rk)
    out = ctypes.create_string_buffer(16)
    lib().gvo_aes128_encrypt(rk, block16, out)
    return out.raw


def blake2b(msg: bytes, digest_size=64, key=b"", person=None) -> bytes:
    out = ctypes.create_string_buffer(digest_size)
    lib().gvo_blake2b(key or None, len(key), person, msg, len(msg), out, digest_size)
    return out.raw


def storage_keys(secret32: bytes):
    a, m = ctypes.create_string_buffer(16), ctypes.create_string_buffer(32)
    lib().gvo_storage_keys(secret32, a, m)
    return a.raw, m.raw


def seal_row(secret32: bytes, table: int, row: int, epoch: int, pt: bytes, side_pt=None):
    """-> (ct 1024 B, side ct 16 B or None, tag 16 B)"""
    ct, sct, tag = (ctypes.create_string_buffer(1024), ctypes.create_string_buffer(16),
                    ctypes.create_string_buffer(16))
    lib().gvo_seal_row(secret32, table, row, epoch, pt, side_pt, ct, sct if side_pt else None, tag)
    return ct.raw, (sct.raw if side_pt else None), tag.raw


def uhash_keys(secret32: bytes):
    """-> (nh: 268 u32, l3k: 16 u64, l3p: 4 u32), the message tables' row-hash keys"""
    nh, l3k, l3p = np.zeros(268, np.uint32), np.zeros(16, np.uint64), np.zeros(4, np.uint32)
    lib().gvo_uhash_keys(secret32, nh.ctypes.data, l3k.ctypes.data, l3p.ctypes.data)
    return nh, l3k, l3p


def row_hash(keys, ct: bytes) -> bytes:
    nh, l3k, l3p = keys
    out = ctypes.create_string_buffer(16)
    lib().gvo_row_hash(nh.ctypes.data, l3k.ctypes.data, l3p.ctypes.data, ct, out)
    return out.raw


def identity(i: int) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().gvo_identity(i, out)
    return out.raw


class Model:
    """The sequential semantic model (seqmodel)."""

    def __init__(self, config):
        self.L = lib()
        self.config = config
        self.m = self.L.gvo_create(ctypes.byref(config))
        if not self.m:
            raise ValueError("invalid oracle config")
        self.rng = ctypes.c_uint64(0)
        self.ops = 0

    def close(self):
        if self.m:
            self.L.gvo_destroy(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_batch(self, reqs):
        reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
        out = np.zeros(len(reqs), dtype=abi.RESPONSE_DTYPE)
        rc = self.L.gvo_process_batch(self.m, reqs.ctypes.data, len(reqs), out.ctypes.data)
        if rc != 0:
            raise ValueError(f"oracle rejected batch: {rc}")
        return out

    def set_expiry_cutoff(self, cutoff):
        self.L.gvo_set_expiry_cutoff(self.m, int(cutoff))

    def apply_one(self, req):
        r = np.ascontiguousarray(np.asarray(req, dtype=abi.REQUEST_DTYPE).reshape(1))
        out = np.zeros(1, dtype=abi.RESPONSE_DTYPE)
        self.L.gvo_apply_one(self.m, r.ctypes.data, out.ctypes.data)
        return out[0]

    def seed(self, s):
        self.rng = ctypes.c_uint64(s)

    def gen_batch(self, n, params):
        reqs = np.zeros(n, dtype=abi.REQUEST_DTYPE)
        self.L.gvo_gen_batch(self.m, ctypes.byref(params), ctypes.byref(self.rng),
                             reqs.ctypes.data, n, self.ops)
        self.ops += n
        return reqs

    @property
    def messages(self):
        return self.L.gvo_messages(self.m)

    @property
    def mailboxes(self):
        return self.L.gvo_mailboxes(self.m)

    @property
    def creation_counter(self):
        return self.L.gvo_creation_counter(self.m)

    def digest(self):
        return self.L.gvo_state_digest(self.m)

    def dump_messages(self):
        n = self.config.msg_capacity
        out = np.zeros(n, dtype=abi.RECORD_DTYPE)
        assert self.L.gvo_dump_messages(self.m, out.ctypes.data, n) == 0
        return out

    def live_message(self, i):
        rec = np.zeros(1, dtype=abi.RECORD_DTYPE)
        if self.L.gvo_live_message(self.m, i, rec.ctypes.data) != 0:
            raise IndexError(i)
        return rec[0]


class _ShardView(Model):
    """A shard model owned by a Cluster (not freed on its own)."""

    def __init__(self, cluster, ptr, config):
        self.L = cluster.L
        self.config = config
        self.m = ptr
        self.rng = ctypes.c_uint64(0)
        self.ops = 0

    def close(self):
        self.m = None


class Cluster:
    """S shard seqmodels behind the engine's routing: the
    oracle of a sharded store.  A batch of n <= S*max_batch requests is the
    concatenation of the sources' batches (source k = [k*B, (k+1)*B))."""

    def __init__(self, config):
        self.L = lib()
        self.config = config
        self.c = self.L.gvo_cluster_create(ctypes.byref(config))
        if not self.c:
            raise ValueError("invalid oracle cluster config")
        self.S = config.shard_count
        self.capacity = self.L.gvo_cluster_capacity(self.c)
        self.rng = ctypes.c_uint64(0)
        self.ops = 0

    def close(self):
        if self.c:
            self.L.gvo_cluster_destroy(self.c)
            self.c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shard(self, k):
        return _ShardView(self, self.L.gvo_cluster_shard(self.c, k), self.config)

    def process_batch(self, reqs):
        """-> responses, or None when the batch overflows a (source, shard) bucket."""
        reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
        out = np.zeros(len(reqs), dtype=abi.RESPONSE_DTYPE)
        rc = self.L.gvo_cluster_process(self.c, reqs.ctypes.data, len(reqs), out.ctypes.data)
        if rc == abi.GVS_ERR_BATCH_OVERFLOW:
            return None
        if rc != 0:
            raise ValueError(f"oracle cluster rejected batch: {rc}")
        return out

    def set_expiry_cutoff(self, cutoff):
        self.L.gvo_cluster_set_expiry_cutoff(self.c, int(cutoff))

    def seed(self, s):
        self.rng = ctypes.c_uint64(s)

    def gen_batch(self, n, params):
        reqs = np.zeros(n, dtype=abi.REQUEST_DTYPE)
        self.L.gvo_cluster_gen_batch(self.c, ctypes.byref(params), ctypes.byref(self.rng),
                                     reqs.ctypes.data, n, self.ops)
        self.ops += n
        return reqs

    @property
    def messages(self):
        return self.L.gvo_cluster_messages(self.c)

    @property
    def mailboxes(self):
        return self.L.gvo_cluster_mailboxes(self.c)

    @property
    def creation_counter(self):
        return sum(self.shard(k).creation_counter for k in range(self.S))

    def dump_messages(self):
        return np.concatenate([self.shard(k).dump_messages() for k in range(self.S)])


class PathOramModel:
    """The Path ORAM restatement of the reference's CPU store path
    (oracle/gvs_pathoram.c): CPU baseline, cross-checked against Model."""

    def __init__(self, config):
        self.L = lib()
        self.config = config
        self.m = self.L.gvp_create(ctypes.byref(config))
        if not self.m:
            raise MemoryError("gvp_create failed")

    def close(self):
        if self.m:
            self.L.gvp_destroy(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_batch(self, reqs):
        reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
        out = np.zeros(len(reqs), dtype=abi.RESPONSE_DTYPE)
        rc = self.L.gvp_process_batch(self.m, reqs.ctypes.data, len(reqs), out.ctypes.data)
        if rc != 0:
            raise ValueError(f"pathoram rejected batch: {rc}")
        return out

    @property
    def messages(self):
        return self.L.gvp_messages(self.m)

    @property
    def mailboxes(self):
        return self.L.gvp_mailboxes(self.m)

    @property
    def oram_accesses(self):
        return self.L.gvp_oram_accesses(self.m)


class OramModel:
    """Sequential block store (oracle/gvs_kv.c): the ORAM::access semantics."""

    def __init__(self, capacity):
        self.L = lib()
        self.n = capacity
        self.o = self.L.gvo_oram_create(capacity)
        if not self.o:
            raise MemoryError("oracle block store")

    def access(self, ops):
        """ops: abi.BLOCK_OP_DTYPE array -> (n, 1024) uint8 blocks seen, or None
        when the batch is invalid (nothing applied)."""
        ops = np.ascontiguousarray(ops)
        out = np.zeros((len(ops), 1024), np.uint8)
        rc = self.L.gvo_oram_access_batch(self.o, ops.ctypes.data, len(ops), out.ctypes.data)
        return None if rc else out

    def blocks(self):
        out = np.zeros((self.n, 1024), np.uint8)
        self.L.gvo_oram_read_all(self.o, out.ctypes.data)
        return out

    def close(self):
        if self.o:
            self.L.gvo_oram_destroy(self.o)
            self.o = None

    def __del__(self):
        self.close()


class OmapModel:
    """Sequential key-value map (oracle/gvs_kv.c): ObliviousHashMap semantics
    with the batch admission rule of include/gvstore.h."""

    def __init__(self, capacity, secret):
        self.L = lib()
        self.o = self.L.gvo_omap_create(capacity, bytes(secret))
        if not self.o:
            raise MemoryError("oracle map")

    def access(self, ops):
        ops = np.ascontiguousarray(ops)
        out = np.zeros(len(ops), dtype=abi.OMAP_RESULT_DTYPE)
        rc = self.L.gvo_omap_access_batch(self.o, ops.ctypes.data, len(ops), out.ctypes.data)
        return None if rc else out

    def size(self):
        return self.L.gvo_omap_size(self.o)

    def close(self):
        if self.o:
            self.L.gvo_omap_destroy(self.o)
            self.o = None

    def __del__(self):
        self.close()


def omap_hash(secret, key):
    hi, lo = ctypes.c_uint64(), ctypes.c_uint64()
    lib().gvo_omap_hash(bytes(secret), bytes(key), ctypes.byref(hi), ctypes.byref(lo))
    return hi.value, lo.value
