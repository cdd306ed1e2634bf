"""Host-side mirror of the store surface over libgvstore.so (ctypes).

`ObliviousStore.process_batch` is the batched form of the enclave handler's
QueryRequest -> QueryResponse dispatch (types/src/lib.rs:27-120,
api/proto/grapevine.proto:57-122); `access` is the single-op shim in the shape
of mc-oblivious-traits' ObliviousHashMap::access_and_insert.
There is no CPU fallback: if the HIP library or a GPU is missing, construction
fails loudly.
"""
import ctypes
import os

import numpy as np

from . import abi

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))
# The production library exports include/gvstore.h only; the test build adds
# the hooks of include/gvstore_test.h (dumps, raw stores).  Tests select it
# with GVS_TEST_HOOKS=1 (tests/conftest.py).
_LIB_PATH = os.path.join(_HERE, "libgvstore.so")
_TEST_LIB_PATH = os.path.join(_HERE, "libgvstore_test.so")

EXPORTED = (
    "gvs_config_init", "gvs_create", "gvs_destroy", "gvs_process_batch", "gvs_process_batches",
    "gvs_process_batch_device", "gvs_process_batches_device", "gvs_access", "gvs_get_stats",
    "gvs_synchronize", "gvs_set_option", "gvs_get_option", "gvs_set_timing", "gvs_last_timings", "gvs_last_error", "gvs_version",
    "gvs_comm_unique_id", "gvs_create_sharded", "gvs_storage_seal_row", "gvs_set_expiry_cutoff",
    "gvs_oram_create", "gvs_oram_destroy", "gvs_oram_access_batch", "gvs_oram_access_batch_device",
    "gvs_oram_set_timing", "gvs_oram_last_timings", "gvs_oram_last_error",
    "gvs_omap_create", "gvs_omap_destroy", "gvs_omap_access_batch", "gvs_omap_access_batch_device",
    "gvs_omap_set_timing", "gvs_omap_last_timings", "gvs_omap_last_error",
    "gvs_process_wire_batch", "gvs_process_wire_batch_device", "gvs_wire_decode_device",
    "gvs_wire_encode_device", "gvs_sr25519_verify", "gvs_sr25519_verify_device",
    "gvs_host_alloc", "gvs_host_free", "gvs_process_wire_batches",
)
TEST_EXPORTED = ("gvs_dump_messages", "gvs_raw_size", "gvs_dump_raw", "gvs_store_raw",
                 "gvs_route_plan", "gvs_oram_test_handle", "gvs_omap_test_handle", "gvs_test_set_epoch")


def test_hooks_enabled():
    return os.environ.get("GVS_TEST_HOOKS") == "1"


class GvsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gvstore error {code}: {msg}")
        self.code = code


def load_library(path=None):
    """Load libgvstore.so and declare the C ABI signatures."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # GVS_LIB_OVERRIDE: a diagnostic build of the same engine (tools/, A/B runs)
    p = path or os.environ.get("GVS_LIB_OVERRIDE") or (_TEST_LIB_PATH if test_hooks_enabled() else _LIB_PATH)
    if not os.path.exists(p):
        raise RuntimeError(f"{os.path.basename(p)} not built at {p}; run `make` (HIP extension missing)")
    lib = ctypes.CDLL(p)
    hooks = hasattr(lib, "gvs_dump_raw")
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.gvs_config_init.argtypes = [ctypes.POINTER(abi.GvsConfig), ctypes.c_uint64]
    lib.gvs_create.argtypes = [ctypes.POINTER(abi.GvsConfig), ctypes.POINTER(vp)]
    lib.gvs_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.gvs_create_sharded.argtypes = [ctypes.POINTER(abi.GvsConfig), ctypes.c_char_p,
                                       ctypes.POINTER(vp)]
    lib.gvs_destroy.argtypes = [vp]
    lib.gvs_process_batch.argtypes = [vp, vp, u32, vp]
    lib.gvs_process_batch_device.argtypes = [vp, vp, u32, vp]
    lib.gvs_process_batches_device.argtypes = [vp, vp, vp, u32, vp, ctypes.POINTER(u32)]
    lib.gvs_process_wire_batch.argtypes = [vp, vp, u32, vp, u32, vp, vp, vp, u32, vp, vp, vp]
    lib.gvs_process_wire_batches.argtypes = [vp, vp, u32, vp, vp, u32, vp, vp, vp, u32, vp, vp,
                                             ctypes.POINTER(u32)]
    lib.gvs_process_wire_batch_device.argtypes = [vp, vp, u32, vp, u32, vp, vp, vp, u32, vp, vp, vp]
    lib.gvs_sr25519_verify.argtypes = [vp, vp, vp, u32, vp, u32, vp, u32, vp]
    lib.gvs_host_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    lib.gvs_host_free.argtypes = [vp, vp]
    lib.gvs_sr25519_verify_device.argtypes = [vp, vp, u32, vp, u32, u32, vp, u32, u32, vp, u32, vp]
    lib.gvs_wire_decode_device.argtypes = [vp, vp, u32, vp, u32, vp, vp, vp, vp]
    lib.gvs_wire_encode_device.argtypes = [vp, vp, u32, vp, u32, vp]
    lib.gvs_process_batches.argtypes = [vp, vp, vp, u32, vp, ctypes.POINTER(u32)]
    lib.gvs_access.argtypes = [vp, vp, vp]
    lib.gvs_get_stats.argtypes = [vp, ctypes.POINTER(abi.GvsStats)]
    lib.gvs_synchronize.argtypes = [vp]
    lib.gvs_set_timing.argtypes = [vp, i32]
    lib.gvs_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
    lib.gvs_get_option.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
    lib.gvs_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_float), i32]
    cp, u64 = ctypes.c_char_p, ctypes.c_uint64
    lib.gvs_storage_seal_row.argtypes = [cp, u32, u64, u32, cp, cp, cp, cp, cp]
    if hooks:
        lib.gvs_dump_messages.argtypes = [vp, vp, ctypes.c_uint64]
        lib.gvs_raw_size.argtypes = [vp, u32, u32, ctypes.POINTER(u64)]
        lib.gvs_dump_raw.argtypes = [vp, u32, u32, u64, vp, u64]
        lib.gvs_store_raw.argtypes = [vp, u32, u32, u64, vp, u64]
        P32 = ctypes.POINTER(u32)
        lib.gvs_route_plan.argtypes = [ctypes.POINTER(abi.GvsConfig), vp, u32, vp, P32, P32, vp]
        lib.gvs_oram_test_handle.argtypes = [vp]
        lib.gvs_oram_test_handle.restype = vp
        lib.gvs_omap_test_handle.argtypes = [vp]
        lib.gvs_omap_test_handle.restype = vp
        lib.gvs_test_set_epoch.argtypes = [vp, u32]
    lib.gvs_last_error.argtypes = [vp]
    lib.gvs_set_expiry_cutoff.argtypes = [vp, ctypes.c_uint64]
    lib.gvs_last_error.restype = ctypes.c_char_p
    lib.gvs_version.restype = ctypes.c_char_p
    lib.gvs_oram_create.argtypes = [ctypes.POINTER(abi.GvsOramConfig), ctypes.POINTER(vp)]
    lib.gvs_oram_destroy.argtypes = [vp]
    lib.gvs_oram_access_batch.argtypes = [vp, vp, u32, vp]
    lib.gvs_oram_access_batch_device.argtypes = [vp, vp, u32, vp]
    lib.gvs_oram_set_timing.argtypes = [vp, i32]
    lib.gvs_oram_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(ctypes.c_float), i32]
    lib.gvs_oram_last_error.argtypes = [vp]
    lib.gvs_oram_last_error.restype = ctypes.c_char_p
    lib.gvs_omap_create.argtypes = [ctypes.POINTER(abi.GvsOramConfig), ctypes.POINTER(vp)]
    lib.gvs_omap_destroy.argtypes = [vp]
    lib.gvs_omap_access_batch.argtypes = [vp, vp, u32, vp]
    lib.gvs_omap_access_batch_device.argtypes = [vp, vp, u32, vp]
    lib.gvs_omap_set_timing.argtypes = [vp, i32]
    lib.gvs_omap_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(ctypes.c_float), i32]
    lib.gvs_omap_last_error.argtypes = [vp]
    lib.gvs_omap_last_error.restype = ctypes.c_char_p
    for name in EXPORTED + (TEST_EXPORTED if hooks else ()):
        if name not in ("gvs_last_error", "gvs_version", "gvs_oram_last_error", "gvs_omap_last_error",
                        "gvs_oram_test_handle", "gvs_omap_test_handle"):
            getattr(lib, name).restype = i32
    if path is None:
        _LIB = lib
    return lib


def route_plan(config, reqs, with_shed=False):
    """The router's placement of one source's batch, on the host (test
    library, gvs_route_plan): -> (slot per request, C, shard pipeline size,
    overflowed[, shed flags])."""
    lib = load_library(_TEST_LIB_PATH)
    reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
    slot = np.zeros(len(reqs), dtype=np.uint32)
    shed = np.zeros(len(reqs), dtype=np.uint8)
    cap, be = ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib.gvs_route_plan(ctypes.byref(config), reqs.ctypes.data, len(reqs), slot.ctypes.data,
                            ctypes.byref(cap), ctypes.byref(be), shed.ctypes.data)
    if rc not in (0, abi.GVS_ERR_BATCH_OVERFLOW):
        raise GvsError(rc, "gvs_route_plan failed")
    out = (slot, cap.value, be.value, rc == abi.GVS_ERR_BATCH_OVERFLOW)
    return out + (shed.astype(bool),) if with_shed else out


def comm_unique_id():
    """RCCL unique id for gvs_create_sharded (call on one rank, share with all)."""
    buf = ctypes.create_string_buffer(abi.COMM_ID_BYTES)
    rc = load_library().gvs_comm_unique_id(buf)
    if rc != 0:
        raise GvsError(rc, "gvs_comm_unique_id failed")
    return buf.raw


class ObliviousStore:
    """One store handle (not thread-safe, like `&mut self`).

    - `comm_id=None`, `config.shard_count <= 1`: one shard on one GPU.
    - `comm_id=None`, `config.shard_count = S > 1`: all S shards on
      `config.device` in this process (single-GPU test form of the sharded
      store; a batch is the concatenation of S sources' batches).
    - `comm_id` given: this process's shard `config.shard_index` of an
      S-process store over RCCL; every call is collective.
    """

    def __init__(self, config, comm_id=None):
        self.lib = load_library()
        self.config = config
        self._pinned = []
        h = ctypes.c_void_p()
        if comm_id is None:
            rc = self.lib.gvs_create(ctypes.byref(config), ctypes.byref(h))
        else:
            rc = self.lib.gvs_create_sharded(ctypes.byref(config), comm_id, ctypes.byref(h))
        if rc != 0:
            raise GvsError(rc, "gvs_create failed (no GPU, bad config or out of memory)")
        self.h = h
        self.B = config.max_batch

    def close(self):
        if getattr(self, "h", None):
            for p in getattr(self, "_pinned", []):
                self.lib.gvs_host_free(self.h, p)
            self._pinned = []
            self.lib.gvs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise GvsError(rc, self.lib.gvs_last_error(self.h).decode())

    def process_batch(self, reqs):
        """reqs: np.ndarray of abi.REQUEST_DTYPE -> responses (abi.RESPONSE_DTYPE)."""
        reqs = np.ascontiguousarray(reqs, dtype=abi.REQUEST_DTYPE)
        out = np.zeros(len(reqs), dtype=abi.RESPONSE_DTYPE)
        self._check(self.lib.gvs_process_batch(self.h, reqs.ctypes.data, len(reqs), out.ctypes.data))
        return out

    def process_batches(self, batches):
        """Several batches from host memory, double-buffered (gvs_process_batches).
        -> list of response arrays.  On a failing batch raises GvsError with
        `.applied` = the number of batches applied before it."""
        counts = np.array([len(b) for b in batches], dtype=np.uint32)
        reqs = np.ascontiguousarray(np.concatenate(batches) if len(batches) else
                                    np.zeros(0, dtype=abi.REQUEST_DTYPE), dtype=abi.REQUEST_DTYPE)
        out = np.zeros(len(reqs), dtype=abi.RESPONSE_DTYPE)
        applied = ctypes.c_uint32(0)
        rc = self.lib.gvs_process_batches(self.h, reqs.ctypes.data, counts.ctypes.data, len(counts),
                                          out.ctypes.data, ctypes.byref(applied))
        if rc != 0:
            err = GvsError(rc, (self.lib.gvs_last_error(self.h) or b"").decode())
            err.applied = applied.value
            raise err
        return np.split(out, np.cumsum(counts)[:-1]) if len(counts) else []

    def process_batch_device(self, d_reqs_ptr, n, d_out_ptr):
        self._check(self.lib.gvs_process_batch_device(self.h, d_reqs_ptr, n, d_out_ptr))

    def process_batches_device(self, d_reqs_ptr, counts, d_out_ptr):
        """k batches from device memory in one call (gvs_process_batches_device):
        every batch enqueued before any result is awaited.  Returns the number
        applied; raises GvsError (with .applied) at the first failing batch."""
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        applied = ctypes.c_uint32(0)
        rc = self.lib.gvs_process_batches_device(self.h, d_reqs_ptr, c.ctypes.data, len(c), d_out_ptr,
                                                 ctypes.byref(applied))
        if rc != 0:
            err = GvsError(rc, self.lib.gvs_last_error(self.h).decode())
            err.applied = applied.value
            raise err
        return applied.value

    @staticmethod
    def _wire_slab(msgs, in_stride):
        if isinstance(msgs, np.ndarray):
            n, width = msgs.shape
            lens = np.full(n, width, np.uint32)
            stride = in_stride or width
            slab = np.zeros((n, stride), np.uint8)
            slab[:, :width] = msgs
        else:
            n = len(msgs)
            lens = np.array([len(m) for m in msgs], np.uint32)
            stride = in_stride or max(int(lens.max()) if n else 1, 1)
            slab = np.zeros((n, stride), np.uint8)
            for k, m in enumerate(msgs):
                slab[k, :len(m)] = np.frombuffer(bytes(m), np.uint8)
        return slab, lens, stride

    def process_wire_batches(self, batches, times, in_stride=None,
                             out_stride=abi.WIRE_RESPONSE_BYTES, challenges=None):
        """Several wire batches in one double-buffered call
        (gvs_process_wire_batches).  batches: list of lists of message bytes;
        times / challenges: per message over all batches (times may be a
        scalar).  -> list of (response bytes list, status array) per batch.
        On a failing batch raises GvsError with `.applied`."""
        counts = np.array([len(b) for b in batches], dtype=np.uint32)
        flat = [m for b in batches for m in b]
        n = len(flat)
        slab, lens, stride = self._wire_slab(flat, in_stride)
        times = np.ascontiguousarray(np.broadcast_to(np.asarray(times, np.uint64), (n,)))
        out = np.zeros((n, out_stride), np.uint8)
        out_lens = np.zeros(n, np.uint32)
        status = np.zeros(n, np.uint32)
        chal = None
        if challenges is not None:
            chal = np.ascontiguousarray(challenges, np.uint8).reshape(n, 32)
        applied = ctypes.c_uint32(0)
        rc = self.lib.gvs_process_wire_batches(
            self.h, slab.ctypes.data, stride, lens.ctypes.data, counts.ctypes.data, len(counts),
            times.ctypes.data, chal.ctypes.data if chal is not None else None, out.ctypes.data,
            out_stride, out_lens.ctypes.data, status.ctypes.data, ctypes.byref(applied))
        if rc != 0:
            err = GvsError(rc, (self.lib.gvs_last_error(self.h) or b"").decode())
            err.applied = applied.value
            raise err
        res, o = [], 0
        for c in counts:
            res.append(([out[k, :out_lens[k]].tobytes() for k in range(o, o + c)], status[o:o + c]))
            o += int(c)
        return res

    def process_wire_batch(self, msgs, times, in_stride=None, out_stride=abi.WIRE_RESPONSE_BYTES,
                           challenges=None):
        """Wire QueryRequests (list of bytes, or an (n, L) uint8 array of
        canonical messages) through the device codec and the store
        (gvs_process_wire_batch).  `challenges` ((n, 32) uint8, optional): the
        challenge each auth_signature must sign; failing requests become hard
        errors.  -> (list of response bytes, (n, 64) signatures, per-request
        GVS_WIRE_* status).  A hard error's response is b"" (the handler
        answers it with a gRPC error)."""
        slab, lens, stride = self._wire_slab(msgs, in_stride)
        n = len(lens)
        times = np.ascontiguousarray(np.broadcast_to(np.asarray(times, np.uint64), (n,)))
        out = np.zeros((n, out_stride), np.uint8)
        out_lens = np.zeros(n, np.uint32)
        sigs = np.zeros((n, 64), np.uint8)
        status = np.zeros(n, np.uint32)
        chal = None
        if challenges is not None:
            chal = np.ascontiguousarray(challenges, np.uint8).reshape(n, 32)
        self._check(self.lib.gvs_process_wire_batch(
            self.h, slab.ctypes.data, stride, lens.ctypes.data, n, times.ctypes.data,
            chal.ctypes.data if chal is not None else None, out.ctypes.data, out_stride,
            out_lens.ctypes.data, sigs.ctypes.data, status.ctypes.data))
        return [out[k, :out_lens[k]].tobytes() for k in range(n)], sigs, status

    def host_array(self, count, dtype):
        """A numpy array of `count` items in pinned host memory (gvs_host_alloc),
        which gvs_process_batches copies without staging.  Freed when the
        store closes."""
        dtype = np.dtype(dtype)
        p = ctypes.c_void_p()
        self._check(self.lib.gvs_host_alloc(self.h, max(1, count * dtype.itemsize), ctypes.byref(p)))
        self._pinned.append(p)
        buf = (ctypes.c_uint8 * (count * dtype.itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=dtype, count=count)

    def sr25519_verify(self, pks, msgs, sigs, context=b"grapevine-challenge"):
        """Batched schnorrkel verification on the device (gvs_sr25519_verify):
        pks (n, 32), msgs (n, L), sigs (n, 64) uint8 -> (n,) bool."""
        pks = np.ascontiguousarray(pks, np.uint8)
        msgs = np.ascontiguousarray(msgs, np.uint8)
        sigs = np.ascontiguousarray(sigs, np.uint8)
        n = len(pks)
        ok = np.zeros(n, np.uint32)
        self._check(self.lib.gvs_sr25519_verify(self.h, pks.ctypes.data, msgs.ctypes.data,
                                                msgs.shape[1] if msgs.ndim == 2 else 0,
                                                sigs.ctypes.data, n, context, len(context),
                                                ok.ctypes.data))
        return ok.astype(bool)

    def access(self, req):
        out = self.process_batch(np.asarray([req], dtype=abi.REQUEST_DTYPE) if not isinstance(req, np.ndarray) else req.reshape(1))
        return out[0]

    def stats(self):
        s = abi.GvsStats()
        self._check(self.lib.gvs_get_stats(self.h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in abi.GvsStats._fields_}

    def dump_messages(self):
        n = self.config.msg_capacity * self.stats()["shards"]
        out = np.zeros(n, dtype=abi.RECORD_DTYPE)
        self._check(self.lib.gvs_dump_messages(self.h, out.ctypes.data, n * 1024))
        return out

    def dump_raw_size(self, region, shard=0):
        """Size in bytes of one shard's raw region (abi.RAW_*).  Test use."""
        n = ctypes.c_uint64()
        self._check(self.lib.gvs_raw_size(self.h, shard, region, ctypes.byref(n)))
        return n.value

    def dump_raw(self, region, offset, nbytes, shard=0):
        """Raw device bytes of one shard's region (abi.RAW_*): ciphertext in
        authenticated mode.  Test use."""
        out = np.zeros(nbytes, dtype=np.uint8)
        self._check(self.lib.gvs_dump_raw(self.h, shard, region, offset, out.ctypes.data, nbytes))
        return out

    def store_raw(self, region, offset, data, shard=0):
        """Overwrite raw device bytes (tamper tests of the authenticated mode)."""
        buf = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
        self._check(self.lib.gvs_store_raw(self.h, shard, region, offset, buf.ctypes.data, len(buf)))

    def synchronize(self):
        self._check(self.lib.gvs_synchronize(self.h))

    def set_option(self, key, value):
        self._check(self.lib.gvs_set_option(self.h, key.encode(), int(value)))

    def get_option(self, key):
        v = ctypes.c_int64()
        self._check(self.lib.gvs_get_option(self.h, key.encode(), ctypes.byref(v)))
        return v.value

    def set_expiry_cutoff(self, cutoff):
        """Messages with timestamp < cutoff expire (gvs_set_expiry_cutoff)."""
        self._check(self.lib.gvs_set_expiry_cutoff(self.h, int(cutoff)))

    def set_timing(self, on=True):
        self._check(self.lib.gvs_set_timing(self.h, 1 if on else 0))

    def last_timings(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        c = self.lib.gvs_last_timings(self.h, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(max(c, 0))}


class BlockStore:
    """The block store (gvs_oram_*): mc-oblivious-traits ORAM::access, batched.
    `access(ops)` applies abi.BLOCK_OP_DTYPE ops in order and returns the
    (n, 1024) blocks they saw."""

    def __init__(self, config):
        self.lib = load_library()
        self.config = config
        h = ctypes.c_void_p()
        rc = self.lib.gvs_oram_create(ctypes.byref(config), ctypes.byref(h))
        if rc != 0:
            raise GvsError(rc, "gvs_oram_create failed (no GPU, bad config or out of memory)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.gvs_oram_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise GvsError(rc, self.lib.gvs_oram_last_error(self.h).decode())

    def access(self, ops):
        ops = np.ascontiguousarray(ops, dtype=abi.BLOCK_OP_DTYPE)
        out = np.zeros((len(ops), 1024), dtype=np.uint8)
        self._check(self.lib.gvs_oram_access_batch(self.h, ops.ctypes.data, len(ops), out.ctypes.data))
        return out

    def access_device(self, d_ops, n, d_out):
        """Device pointers (ints): n ops in, n x 1024 bytes out."""
        self._check(self.lib.gvs_oram_access_batch_device(self.h, d_ops, n, d_out))

    def _raw_handle(self):
        if not hasattr(self.lib, "gvs_oram_test_handle"):
            raise RuntimeError("raw regions need the test library (GVS_TEST_HOOKS=1)")
        return self.lib.gvs_oram_test_handle(self.h)

    def dump_raw(self, region, offset, nbytes):
        """Raw device bytes of the block table (abi.RAW_MESSAGES), its tags
        (RAW_MSG_TAGS) or its pending final states (RAW_PENDING*).  Test use."""
        out = np.zeros(nbytes, dtype=np.uint8)
        self._check(self.lib.gvs_dump_raw(self._raw_handle(), 0, region, offset, out.ctypes.data, nbytes))
        return out

    def store_raw(self, region, offset, data):
        """Overwrite raw device bytes (tamper tests of the sealed block store)."""
        buf = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
        self._check(self.lib.gvs_store_raw(self._raw_handle(), 0, region, offset, buf.ctypes.data, len(buf)))

    def set_timing(self, on=True):
        self._check(self.lib.gvs_oram_set_timing(self.h, 1 if on else 0))

    def last_timings(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        c = self.lib.gvs_oram_last_timings(self.h, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(max(c, 0))}


class KeyValueMap:
    """The key-value map (gvs_omap_*): mc-oblivious-traits ObliviousHashMap,
    batched.  `access(ops)` applies abi.OMAP_OP_DTYPE ops in order and returns
    abi.OMAP_RESULT_DTYPE results (status, the value each op saw)."""

    def __init__(self, config):
        self.lib = load_library()
        self.config = config
        h = ctypes.c_void_p()
        rc = self.lib.gvs_omap_create(ctypes.byref(config), ctypes.byref(h))
        if rc != 0:
            raise GvsError(rc, "gvs_omap_create failed (no GPU, bad config or out of memory)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.gvs_omap_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise GvsError(rc, self.lib.gvs_omap_last_error(self.h).decode())

    def access(self, ops):
        ops = np.ascontiguousarray(ops, dtype=abi.OMAP_OP_DTYPE)
        out = np.zeros(len(ops), dtype=abi.OMAP_RESULT_DTYPE)
        self._check(self.lib.gvs_omap_access_batch(self.h, ops.ctypes.data, len(ops), out.ctypes.data))
        return out

    def access_device(self, d_ops, n, d_out):
        self._check(self.lib.gvs_omap_access_batch_device(self.h, d_ops, n, d_out))

    def _raw_handle(self):
        if not hasattr(self.lib, "gvs_omap_test_handle"):
            raise RuntimeError("raw regions need the test library (GVS_TEST_HOOKS=1)")
        return self.lib.gvs_omap_test_handle(self.h)

    def dump_raw(self, region, offset, nbytes):
        """Raw device bytes of the value table and its regions (as BlockStore),
        the key directory (abi.RAW_KEY_DIR) or its tags (RAW_KEY_DIR_TAGS)."""
        out = np.zeros(nbytes, dtype=np.uint8)
        self._check(self.lib.gvs_dump_raw(self._raw_handle(), 0, region, offset, out.ctypes.data, nbytes))
        return out

    def store_raw(self, region, offset, data):
        """Overwrite raw device bytes (tamper tests of the sealed map)."""
        buf = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
        self._check(self.lib.gvs_store_raw(self._raw_handle(), 0, region, offset, buf.ctypes.data, len(buf)))

    def set_timing(self, on=True):
        self._check(self.lib.gvs_omap_set_timing(self.h, 1 if on else 0))

    def last_timings(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        c = self.lib.gvs_omap_last_timings(self.h, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(max(c, 0))}
