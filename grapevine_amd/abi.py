"""numpy / ctypes mirrors of the POD types in include/gvstore.h.

The request layout puts the Record a CREATE would store first (README.md:132-136:
16 B id, 32 B sender, 32 B recipient, 8 B timestamp, 936 B payload) with the
request's auth_identity in the sender position; see include/gvstore.h.
"""
import ctypes

import numpy as np

MSG_ID_BYTES = 16
KEY_BYTES = 32
PAYLOAD_BYTES = 936
RECORD_BYTES = 1024
MAILBOX_SLOTS = 62

# RequestType, types/src/lib.rs:16-22
REQUEST_TYPE_CREATE = 1
REQUEST_TYPE_READ = 2
REQUEST_TYPE_UPDATE = 3
REQUEST_TYPE_DELETE = 4

# StatusCode, types/src/lib.rs:122-137 (0 = hard error, see gvstore.h)
STATUS_HARD_ERROR = 0
STATUS_CODE_SUCCESS = 1
STATUS_CODE_NOT_FOUND = 2
STATUS_CODE_MESSAGE_ID_ALREADY_IN_USE = 3
STATUS_CODE_INVALID_RECIPIENT = 4
STATUS_CODE_TOO_MANY_MESSAGES_FOR_RECIPIENT = 5
STATUS_CODE_TOO_MANY_RECIPIENTS = 6
STATUS_CODE_TOO_MANY_MESSAGES = 7
STATUS_CODE_INTERNAL_ERROR = 8

GVS_OK = 0
GVS_ERR_INVALID_ARG = -1
GVS_ERR_DEVICE = -2
GVS_ERR_OUT_OF_MEMORY = -3
GVS_ERR_BATCH_OVERFLOW = -4
GVS_ERR_NO_DEVICE = -5
GVS_ERR_INTERNAL = -6
GVS_ERR_INTEGRITY = -7
GVS_ERR_EPOCH_EXHAUSTED = -8

RECORD_DTYPE = np.dtype([
    ("msg_id", "u1", 16),
    ("sender", "u1", 32),
    ("recipient", "u1", 32),
    ("timestamp", "<u8"),
    ("payload", "u1", PAYLOAD_BYTES),
])
REQUEST_DTYPE = np.dtype([
    ("msg_id", "u1", 16),
    ("auth_identity", "u1", 32),
    ("recipient", "u1", 32),
    ("timestamp", "<u8"),
    ("payload", "u1", PAYLOAD_BYTES),
    ("request_type", "<u4"),
    ("reserved", "<u4", 3),
])
RESPONSE_DTYPE = np.dtype([
    ("record", RECORD_DTYPE),
    ("status_code", "<u4"),
    ("reserved", "<u4", 3),
])
assert RECORD_DTYPE.itemsize == 1024
assert REQUEST_DTYPE.itemsize == 1040
assert RESPONSE_DTYPE.itemsize == 1040


class GvsConfig(ctypes.Structure):
    _fields_ = [
        ("msg_capacity", ctypes.c_uint64),
        ("mailbox_partitions", ctypes.c_uint32),
        ("mailbox_partition_slots", ctypes.c_uint32),
        ("max_batch", ctypes.c_uint32),
        ("device", ctypes.c_uint32),
        ("secret_key", ctypes.c_uint8 * 32),
        ("flags", ctypes.c_uint32),
        ("rows_per_partition", ctypes.c_uint32),
        ("shard_count", ctypes.c_uint32),
        ("shard_index", ctypes.c_uint32),
        ("route_capacity", ctypes.c_uint32),
        ("expiry_per_batch", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 2),
    ]


class GvsStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "messages", "mailboxes", "batches", "creation_counter", "free_ring_head",
        "free_ring_tail", "msg_partitions", "msg_partition_slots", "shards", "route_capacity",
        "shard_batch", "epoch")]

# wire codec (gvs_process_wire_batch, include/gvstore.h)
WIRE_REQUEST_BYTES, WIRE_RESPONSE_BYTES, WIRE_SLOT_MAX = 1099, 1042, 2048
WIRE_OK, WIRE_DECODE_ERROR, WIRE_BAD_FIELD, WIRE_BAD_SIGNATURE = 0, 1, 2, 3

COMM_ID_BYTES = 128
FLAG_AUTH_STORAGE = 1  # GVS_FLAG_AUTH_STORAGE: AES-CTR + BLAKE2b sealed tables
ERR_INTEGRITY = -7     # GVS_ERR_INTEGRITY

# gvs_dump_raw / gvs_store_raw regions
RAW_MESSAGES, RAW_MAILBOXES, RAW_SIDE, RAW_MSG_TAGS, RAW_MBOX_TAGS = range(5)
# the final row states the last batch left pending (by sorted position), their
# side entries and tags, and that batch's slot descriptors (include/gvstore_test.h)
RAW_PENDING, RAW_PENDING_SIDE, RAW_PENDING_TAGS, RAW_SLOTS = range(5, 9)
# the key-value map's key directory (N x 32 B: key, hash) and, sealed, its
# 1-KiB row tags (N/32 x 16 B)
RAW_KEY_DIR, RAW_KEY_DIR_TAGS = 9, 10
# header table field of a message row whose final state is pending in P
TABLE_PENDING_STATE, TABLE_PENDING_ROW = 2, 0x100


# block store (gvs_oram_*, include/gvstore.h)
ORAM_READ, ORAM_WRITE = 0, 1
BLOCK_OP_DTYPE = np.dtype([
    ("index", "<u8"),
    ("op", "<u4"),
    ("reserved", "<u4"),
    ("data", "u1", 1024),
])
assert BLOCK_OP_DTYPE.itemsize == 1040


class GvsOramConfig(ctypes.Structure):
    _fields_ = [
        ("capacity", ctypes.c_uint64),
        ("max_batch", ctypes.c_uint32),
        ("device", ctypes.c_uint32),
        ("secret_key", ctypes.c_uint8 * 32),
        ("flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32 * 3),
    ]


assert ctypes.sizeof(GvsOramConfig) == 64


# key-value map (gvs_omap_*, include/gvstore.h)
OMAP_READ, OMAP_WRITE, OMAP_INSERT, OMAP_REMOVE = 0, 1, 2, 3
OMAP_FOUND, OMAP_NOT_FOUND, OMAP_OVERFLOW, OMAP_INVALID_KEY = 0, 1, 2, 3
OMAP_OP_DTYPE = np.dtype([
    ("key", "u1", 16),
    ("op", "<u4"),
    ("reserved", "<u4", 3),
    ("value", "u1", 1024),
])
OMAP_RESULT_DTYPE = np.dtype([
    ("value", "u1", 1024),
    ("status", "<u4"),
    ("reserved", "<u4", 3),
])
assert OMAP_OP_DTYPE.itemsize == 1056 and OMAP_RESULT_DTYPE.itemsize == 1040


def make_oram_config(capacity, max_batch=4096, device=0, secret_key=None, auth_storage=False):
    cfg = GvsOramConfig()
    cfg.capacity = capacity
    cfg.max_batch = max_batch
    cfg.device = device
    cfg.flags = FLAG_AUTH_STORAGE if auth_storage else 0
    key = secret_key if secret_key is not None else bytes((0x67 + 31 * i) & 0xFF for i in range(32))
    for i in range(32):
        cfg.secret_key[i] = key[i]
    return cfg


def make_config(msg_capacity, mailbox_partitions=None, mailbox_partition_slots=256,
                max_batch=None, device=0, secret_key=None, shard_count=0, shard_index=0,
                route_capacity=0, rows_per_partition=0, auth_storage=False, expiry_per_batch=0):
    """Config mirroring gvs_config_init's defaults (R = N/16 mailboxes per shard)."""
    cfg = GvsConfig()
    cfg.shard_count = shard_count
    cfg.shard_index = shard_index
    cfg.route_capacity = route_capacity
    cfg.expiry_per_batch = expiry_per_batch
    cfg.rows_per_partition = rows_per_partition
    cfg.flags = FLAG_AUTH_STORAGE if auth_storage else 0
    cfg.msg_capacity = msg_capacity
    if mailbox_partitions is None:
        r = max(msg_capacity // 16, 256)
        mailbox_partitions = max(r // mailbox_partition_slots, 1)
    cfg.mailbox_partitions = mailbox_partitions
    cfg.mailbox_partition_slots = mailbox_partition_slots
    cfg.max_batch = max_batch if max_batch is not None else (4096 if msg_capacity < 65536 else 65536)
    cfg.device = device
    key = secret_key if secret_key is not None else bytes((0x67 + 31 * i) & 0xFF for i in range(32))
    for i in range(32):
        cfg.secret_key[i] = key[i]
    return cfg
