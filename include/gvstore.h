/*
 * gvstore.h — C ABI of the MI355X-native batched oblivious message store for
 * grapevine's CRUD path.
 *
 * This header is the single drop-in boundary between the (Rust) enclave request
 * handler and the HIP engine.  Every type is a plain-old-data struct; no torch,
 * HIP or C++ type appears here.  INTEGRATION.md shows the `extern "C"` Rust
 * binding (gvstore-sys) a maintainer would add next to the reference's
 * `types/` crate.
 *
 * What each entry point replaces in the reference (all hot-path code is absent
 * from the reference snapshot; the surface below follows the
 * types the reference does hold):
 *
 *   gvs_process_batch   the enclave handler's per-request dispatch over
 *                       QueryRequest -> QueryResponse
 *                       (types/src/lib.rs:27-59 request, :111-120 response,
 *                        semantics api/proto/grapevine.proto:57-122),
 *                       batched: B requests in, B responses out, request order.
 *   gvs_access          ObliviousHashMap::access_and_insert-style single-op
 *                       shim (mc-oblivious-traits, absent),
 *                       implemented as a batch of one.
 *   gvs_create/destroy  construction of the ORAM-backed maps (capacity fixed
 *                       at creation, README.md:73-80).
 *
 * Conventions: return 0 on success, a negative GVS_ERR_* on
 * API misuse or device failure.  Per-request outcomes are reported only in
 * gvs_response.status_code.  Nothing unwinds across this boundary.  A handle
 * is owned by one host thread at a time (the reference traits take &mut self);
 * calls are synchronous.  The caller owns request/response buffers; the library
 * owns all device memory.
 */
#ifndef GVSTORE_H
#define GVSTORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (types/src/lib.rs, README.md) ---------------------------- */

#define GVS_MSG_ID_BYTES 16    /* README.md:134 */
#define GVS_KEY_BYTES 32       /* ristretto public key, README.md:134,141 */
#define GVS_PAYLOAD_BYTES 936  /* README.md:134-136, 148 */
#define GVS_RECORD_BYTES 1024  /* README.md:132-136 */
#define GVS_MAILBOX_SLOTS 62   /* in-flight messages per recipient, README.md:78-80 */

/* RequestType, types/src/lib.rs:16-22 / api/proto/grapevine.proto:44-55 */
#define GVS_REQUEST_CREATE 1u
#define GVS_REQUEST_READ 2u
#define GVS_REQUEST_UPDATE 3u
#define GVS_REQUEST_DELETE 4u

/* StatusCode, types/src/lib.rs:122-137 / api/proto/grapevine.proto:178-197.
 * GVS_STATUS_HARD_ERROR (0, the proto's INVALID_STATUS) marks a request the
 * proto says must fail at the gRPC level instead of with a status
 * (grapevine.proto:57-64 fail-fast rules, :95 zero-id UPDATE). */
#define GVS_STATUS_HARD_ERROR 0u
#define GVS_STATUS_SUCCESS 1u
#define GVS_STATUS_NOT_FOUND 2u
#define GVS_STATUS_MESSAGE_ID_ALREADY_IN_USE 3u
#define GVS_STATUS_INVALID_RECIPIENT 4u
#define GVS_STATUS_TOO_MANY_MESSAGES_FOR_RECIPIENT 5u
#define GVS_STATUS_TOO_MANY_RECIPIENTS 6u
#define GVS_STATUS_TOO_MANY_MESSAGES 7u
#define GVS_STATUS_INTERNAL_ERROR 8u

/* return codes */
#define GVS_OK 0
#define GVS_ERR_INVALID_ARG (-1)
#define GVS_ERR_DEVICE (-2)      /* HIP / RCCL failure; see gvs_last_error */
#define GVS_ERR_OUT_OF_MEMORY (-3)
#define GVS_ERR_BATCH_OVERFLOW (-4) /* a fixed per-partition bound of the batch
                                       was exceeded; the batch was not applied.
                                       Sealed stores also bound the distinct rows
                                       of a message partition over this and the
                                       previous batch (86, the pass's LDS stages):
                                       that overflow depends on the previous batch,
                                       and the next batch may succeed */
#define GVS_ERR_NO_DEVICE (-5)
#define GVS_ERR_INTERNAL (-6)
#define GVS_ERR_INTEGRITY (-7) /* authenticated storage: a stored row failed
                                  its tag; the handle refuses further work */
#define GVS_ERR_EPOCH_EXHAUSTED (-8) /* authenticated storage: 2^32 - 256 batches
                                        applied; rows are bound to a 32-bit epoch,
                                        so the store must be rebuilt under a fresh
                                        secret_key before it could wrap */

/* gvs_config.flags */
#define GVS_FLAG_AUTH_STORAGE 1u /* AES-CTR sealed tables, a MAC per row */

/* ---- records ------------------------------------------------------------- */

/* Record, types/src/lib.rs:82-106; byte layout README.md:132-136.  This is
 * also the exact 1 KiB row stored in HBM. */
typedef struct gvs_record {
  uint8_t msg_id[GVS_MSG_ID_BYTES];
  uint8_t sender[GVS_KEY_BYTES];
  uint8_t recipient[GVS_KEY_BYTES];
  uint64_t timestamp;
  uint8_t payload[GVS_PAYLOAD_BYTES];
} gvs_record;

/* QueryRequest (types/src/lib.rs:27-59) with its RequestRecord (:63-78),
 * laid out so that its first 1024 bytes are the Record a CREATE would store:
 * `sender` is the request's auth_identity.  The 64-byte auth_signature is
 * verified by the caller before the store is reached (grapevine.proto:57-64,
 * README.md:187-200) and is not passed in.  `timestamp` is the server time the
 * caller assigns to this request (README.md:143-144: client timestamps are
 * ignored); it must be nonzero so responses stay constant-size on the wire
 * (SURVEY.md §4.1). */
typedef struct gvs_request {
  uint8_t msg_id[GVS_MSG_ID_BYTES];        /* RequestRecord.msg_id */
  uint8_t auth_identity[GVS_KEY_BYTES];    /* QueryRequest.auth_identity */
  uint8_t recipient[GVS_KEY_BYTES];        /* RequestRecord.recipient */
  uint64_t timestamp;                      /* server time for this request */
  uint8_t payload[GVS_PAYLOAD_BYTES];      /* RequestRecord.payload */
  uint32_t request_type;                   /* QueryRequest.request_type */
  uint32_t reserved[3];                    /* must be zero */
} gvs_request;

/* QueryResponse, types/src/lib.rs:111-120. */
typedef struct gvs_response {
  gvs_record record;
  uint32_t status_code;
  uint32_t reserved[3];
} gvs_response;

/* ---- configuration ------------------------------------------------------- */

typedef struct gvs_config {
  uint64_t msg_capacity;        /* N message slots per shard; power of two, >= 256 */
  uint32_t mailbox_partitions;  /* Q per shard; power of two */
  uint32_t mailbox_partition_slots; /* S_r mailboxes per partition; R = Q*S_r; a multiple of 16,
                                       at most 1024 (256 with GVS_FLAG_AUTH_STORAGE) */
  uint32_t max_batch;           /* B: requests per gvs_process_batch call (per rank
                                   when sharded); power of two, 1024 .. 2^19 */
  uint32_t device;              /* HIP device ordinal */
  uint8_t secret_key[32];       /* [0:16) id PRP key, [16:32) recipient PRF key;
                                   identical on every shard */
  uint32_t flags;               /* GVS_FLAG_* */
  uint32_t rows_per_partition;  /* message rows per table-pass workgroup (power of
                                   two 256..4096); 0 = automatic */
  uint32_t shard_count;         /* S shards of the store (0 or 1 = unsharded) */
  uint32_t shard_index;         /* this process's shard (gvs_create_sharded) */
  uint32_t route_capacity;      /* C: request slots per (source, shard) pair and
                                   batch; 0 = automatic */
  uint32_t expiry_per_batch;    /* X: expiry-sweep deletes per batch and shard
                                   (DESIGN.md §9); 0 = off, else a power of two
                                   <= max_batch / 2.  Unsharded callers then submit
                                   at most max_batch - X requests per batch; a
                                   sharded store gives the deletes slots of their
                                   own in each shard's pipeline. */
  uint32_t reserved[2];         /* must be 0 */
} gvs_config;

typedef struct gvs_stats {       /* summed over the handle's shards */
  uint64_t messages;            /* live messages */
  uint64_t mailboxes;           /* live mailboxes (recipients with messages) */
  uint64_t batches;             /* batches applied */
  uint64_t creation_counter;    /* next id generation number */
  uint64_t free_ring_head;
  uint64_t free_ring_tail;
  uint64_t msg_partitions;      /* W: workgroups of the message-table pass */
  uint64_t msg_partition_slots; /* N / W */
  uint64_t shards;              /* shards held by this handle */
  uint64_t route_capacity;      /* C (0 when unsharded) */
  uint64_t shard_batch;         /* requests each shard's pipeline processes per batch */
  uint64_t epoch;               /* batches applied to the tables (sealing epoch) */
} gvs_stats;

typedef struct gvs_handle gvs_handle;

/* Fill `cfg` with defaults for capacity N (R = N/16 mailboxes, B = 65536,
 * unsharded). */
int gvs_config_init(gvs_config *cfg, uint64_t msg_capacity);

/* Create a store.  With cfg->shard_count S > 1 the handle holds all S shards
 * on cfg->device in this process and routes every batch through the same
 * padded all-to-all as the multi-process form below, with device copies as
 * the transport (single-GPU test mode: n <= S * max_batch requests per call,
 * request k belongs to source rank k / max_batch). */
int gvs_create(const gvs_config *cfg, gvs_handle **out);
int gvs_destroy(gvs_handle *h);

/* Multi-GPU store, one process per GPU.  Every rank calls
 * gvs_create_sharded collectively with the same cfg except shard_index
 * (= its rank) and device, and the same `comm_id` (from gvs_comm_unique_id on
 * one rank, distributed by the caller).  Each gvs_process_batch call is then
 * collective: every rank submits its own n <= max_batch requests; each
 * request is routed to its owning shard inside fixed-size padded sub-batches
 * (C slots per rank pair) over RCCL, and its response comes back to the rank
 * that submitted it, in request order.  If any rank's requests for one shard
 * exceed C, every rank returns GVS_ERR_BATCH_OVERFLOW and nothing is applied. */
#define GVS_COMM_ID_BYTES 128
int gvs_comm_unique_id(uint8_t out[GVS_COMM_ID_BYTES]);
int gvs_create_sharded(const gvs_config *cfg, const uint8_t comm_id[GVS_COMM_ID_BYTES],
                       gvs_handle **out);

/* Process n <= max_batch requests (host memory) and write n responses in
 * request order.  Requests of one batch are linearised in the order defined
 * in DESIGN.md §2 (next-message reads/deletes, then creates, then by-id
 * operations, each in submission order). */
int gvs_process_batch(gvs_handle *h, const gvs_request *reqs, uint32_t n,
                      gvs_response *out);

/* k batches from host memory in one call, double-buffered: the requests of
 * batch t+1 are staged (pinned) and copied in, and the responses of batch t-1
 * copied out, while batch t runs, so PCIe and host copies hide behind the
 * table passes.  Batch t has counts[t] requests; the requests of all batches
 * are consecutive in `reqs` and their responses likewise in `out`.  Batches
 * apply in order, each with the semantics of gvs_process_batch; at the first
 * batch that fails, the call returns its error, that batch and the later
 * ones are not applied, and *applied (optional) holds the number applied.
 * The responses of the unapplied batches are zeroed in `out`. */
int gvs_process_batches(gvs_handle *h, const gvs_request *reqs, const uint32_t *counts,
                        uint32_t k, gvs_response *out, uint32_t *applied);

/* Pinned host memory for request / response arrays (hipHostMalloc on the
 * handle's device).  gvs_process_batches copies such buffers to and from the
 * device directly, without its pinned staging copies; any other host memory
 * works too, staged. */
int gvs_host_alloc(gvs_handle *h, size_t bytes, void **out);
int gvs_host_free(gvs_handle *h, void *p);

/* Same, with device-resident buffers (n * sizeof(gvs_request) and
 * n * sizeof(gvs_response) bytes on the handle's device).  Used by the
 * benchmark so that the timed region excludes PCIe. */
int gvs_process_batch_device(gvs_handle *h, const void *d_reqs, uint32_t n,
                             void *d_out);

/* k batches from device memory in one call: batch t has counts[t] requests;
 * the requests of all batches are consecutive in d_reqs and their responses
 * likewise in d_out.  Every batch is enqueued before any result is awaited
 * (no host round trip between batches).  At the first batch that fails, its
 * error is returned, it and the later ones are not applied, *applied
 * (optional) holds the number applied and the unapplied responses are zeroed. */
int gvs_process_batches_device(gvs_handle *h, const void *d_reqs, const uint32_t *counts,
                               uint32_t k, void *d_out, uint32_t *applied);

/* ---- wire codec ---------------------------------
 * The protobuf messages of api/proto/grapevine.proto:123-176 as the prost
 * structs of types/src/lib.rs:27-120 encode them.  A fully populated
 * QueryRequest is 1099 B; a QueryResponse with nonzero timestamp and status is
 * 1042 B (api/tests/grapevine_types.rs:22-31,46-55).
 *
 * Decoding follows prost: fields in any order, unknown fields skipped, the
 * last occurrence of a field wins, the embedded RequestRecord merged over its
 * occurrences; malformed varints, lengths past the message, a known field
 * with another wire type, field number 0 and groups are decode errors.  A
 * message that fails to decode, or whose auth_identity / auth_signature /
 * msg_id / recipient / payload are not 32 / 64 / 16 / 32 / 936 bytes, becomes
 * an all-zero request of type 0 (a hard error: grapevine.proto:57-64).
 * Encoding writes what prost writes: 1042 B (1033 B if the timestamp is 0),
 * or length 0 for a hard error (status 0), which the handler turns into a
 * gRPC error.  Message k occupies bytes [k*stride, k*stride + len_k) of its
 * slab; strides are at most GVS_WIRE_SLOT_MAX, output strides at least
 * GVS_WIRE_RESPONSE_BYTES.  Every slot is read, and every output slot
 * written, whole. */
#define GVS_WIRE_REQUEST_BYTES 1099
#define GVS_WIRE_RESPONSE_BYTES 1042
#define GVS_WIRE_SLOT_MAX 2048
#define GVS_WIRE_OK 0u            /* decode_status values */
#define GVS_WIRE_DECODE_ERROR 1u  /* prost would fail to decode the message */
#define GVS_WIRE_BAD_FIELD 2u     /* decoded, but a field has the wrong size */
#define GVS_WIRE_BAD_SIGNATURE 3u /* decoded, but the challenge signature does not verify */

/* n wire requests (host buffers) through decode -> [challenge check] ->
 * gvs_process_batch -> encode on the device.  times[k] is the server time of
 * request k (README.md:143-144).  challenges (optional, n x 32 B): the
 * challenge each request's auth_signature must sign (README.md:187-200); a
 * request whose signature does not verify as a schnorrkel signature by its
 * auth_identity under the context "grapevine-challenge" (types/src/lib.rs:13)
 * becomes a hard error (decode_status GVS_WIRE_BAD_SIGNATURE).  NULL: no
 * check (the caller verified).  sigs (optional) receives each request's 64-B
 * auth_signature (zero when it failed to decode); decode_status (optional)
 * one GVS_WIRE_* per request. */
int gvs_process_wire_batch(gvs_handle *h, const uint8_t *in, uint32_t in_stride,
                           const uint32_t *in_lens, uint32_t n, const uint64_t *times,
                           const uint8_t *challenges, uint8_t *out, uint32_t out_stride,
                           uint32_t *out_lens, uint8_t *sigs, uint32_t *decode_status);
/* k wire batches from host memory in one call, double-buffered like
 * gvs_process_batches (uploads of batch t+1 and downloads of batch t-1 run
 * while batch t is processed).  Batch t has counts[t] messages; the messages
 * of all batches are consecutive in `in` (and in in_lens, times, challenges),
 * their results likewise in out / out_lens / decode_status.  Stops at the
 * first failing batch: its error is returned, *applied = the batches before,
 * and the unapplied batches' out / out_lens / decode_status are zeroed.
 * `in` and `out` in pinned memory (gvs_host_alloc) are copied without
 * staging. */
int gvs_process_wire_batches(gvs_handle *h, const uint8_t *in, uint32_t in_stride,
                             const uint32_t *in_lens, const uint32_t *counts, uint32_t k,
                             const uint64_t *times, const uint8_t *challenges, uint8_t *out,
                             uint32_t out_stride, uint32_t *out_lens, uint32_t *decode_status,
                             uint32_t *applied);
/* The same with device buffers (in: n*in_stride B, in_lens: n u32, times: n
 * u64, challenges: optional n*32 B, out: n*out_stride B, out_lens: n u32,
 * sigs: optional n*64 B, decode_status: optional n u32). */
int gvs_process_wire_batch_device(gvs_handle *h, const void *d_in, uint32_t in_stride,
                                  const uint32_t *d_in_lens, uint32_t n, const uint64_t *d_times,
                                  const void *d_challenges, void *d_out, uint32_t out_stride,
                                  uint32_t *d_out_lens, void *d_sigs, uint32_t *d_decode_status);
/* The codec alone, device buffers: wire requests -> gvs_request[n] (+ sigs,
 * + per-request GVS_WIRE_* status, both optional); gvs_response[n] -> wire
 * responses.  Synchronous on the handle's stream. */
int gvs_wire_decode_device(gvs_handle *h, const void *d_wire, uint32_t stride,
                           const uint32_t *d_lens, uint32_t n, const uint64_t *d_times,
                           void *d_reqs, void *d_sigs, uint32_t *d_status);
int gvs_wire_encode_device(gvs_handle *h, const void *d_resps, uint32_t n, void *d_wire,
                           uint32_t stride, uint32_t *d_lens);

/* Schnorrkel signature check (README.md:187-200,
 * mc-crypto-keys' RistrettoPublic::verify_schnorrkel): ok[k] = 1 iff sigs[k]
 * (R || s, 64 B, schnorrkel's marker bit set) is a valid signature by the
 * ristretto255 public key pks[k] on msgs[k] under the signing context
 * `context` (<= 64 B; grapevine uses "grapevine-challenge"), else 0.  Batched
 * on the handle's device, one thread per signature, the same instruction
 * stream whatever the inputs.  Device form: pk k at d_pks + k*pk_stride, msg k
 * (msg_len bytes) at d_msgs + k*msg_stride, sig k at d_sigs + k*sig_stride. */
int gvs_sr25519_verify(gvs_handle *h, const uint8_t *pks, const uint8_t *msgs, uint32_t msg_len,
                       const uint8_t *sigs, uint32_t n, const uint8_t *context,
                       uint32_t context_len, uint32_t *ok);
int gvs_sr25519_verify_device(gvs_handle *h, const void *d_pks, uint32_t pk_stride,
                              const void *d_msgs, uint32_t msg_stride, uint32_t msg_len,
                              const void *d_sigs, uint32_t sig_stride, uint32_t n,
                              const uint8_t *context, uint32_t context_len, uint32_t *d_ok);

/* Message expiry (README.md:86-99: the untrusted host supplies the time and
 * the expiry period).  From the next batch on, messages whose timestamp is
 * < cutoff expire: each batch's message pass records up to X of them (fixed
 * per workgroup), and the following batch deletes them, if still
 * older than its cutoff, through X trailing delete slots: the message row, its
 * mailbox entry and its slot are freed as by a recipient's DELETE.  0 = none.
 * Requires gvs_config.expiry_per_batch > 0 for any effect.  Sharded: every
 * shard sweeps its own table; gvs_create_sharded ranks must all set the same
 * cutoff before the same batch. */
int gvs_set_expiry_cutoff(gvs_handle *h, uint64_t cutoff);

/* Single-request shim in the shape of ObliviousHashMap::access_and_insert. */
int gvs_access(gvs_handle *h, const gvs_request *req, gvs_response *out);

int gvs_get_stats(gvs_handle *h, gvs_stats *out);

/* Authenticated-storage format, host-side and device-free:
 * seal one 1024-B row (and for tables 1 and 2 its 16-B side entry; side_pt =
 * NULL otherwise) at `epoch` under the storage keys derived from `secret`
 * (gvs_config.secret_key).  table: 0 message row, 1 mailbox row, 2 a final
 * row state pending from the last batch (row = its position, side = the
 * physical row it replaces), 0x100 a message row whose final state is pending.
 * For offline verification of dumps and for tests. */
int gvs_storage_seal_row(const uint8_t secret[32], uint32_t table, uint64_t row, uint32_t epoch,
                         const uint8_t pt[1024], const uint8_t *side_pt, uint8_t ct[1024],
                         uint8_t *side_ct, uint8_t tag[16]);

/* Wait for all work on the handle's stream.  A plain single-GPU store runs
 * each batch's mailbox write pass together with the next batch's read pass
 * (one stream over the mailbox table, DESIGN.md §3 "Fused mailbox passes");
 * the last batch's write pass is still to run when a call returns (its
 * responses are final).  gvs_synchronize, gvs_get_stats and the test hooks
 * run it first.  Its one late check (the table's consistency, error bit 2)
 * then surfaces here or in the next batch, as GVS_ERR_INTERNAL with the
 * handle poisoned. */
int gvs_synchronize(gvs_handle *h);

/* Tuning knobs (engine-internal choices that never change results):
 * "sealed_pass_waves" = 0 (default: the authenticated message-table pass runs
 * 12 waves of 8-row chunks per workgroup, three per SIMD, when a partition has
 * at least 1024 rows, else 8), or 4, 8 or 12 to fix it.  Unknown keys or
 * values return GVS_ERR_INVALID_ARG. */
int gvs_set_option(gvs_handle *h, const char *key, int64_t value);

/* Read-only engine parameters of shard 0: "txn_slots" (transaction slots per
 * message partition, c), "group_slots" (recipient-group slots per mailbox
 * partition), "rccl_ranks" / "rccl_rank" (ncclCommCount / ncclCommUserRank of
 * the store's own RCCL communicator; 0 / -1 when the store has none),
 * "fixed_schedule_pass" (1 when the message-table pass stages every
 * transaction slot's line in LDS, so that its memory schedule is the same
 * whatever the batch holds; 0 when the store has more slots per partition
 * than the stages: c = B/W + 8 sqrt(B/W) + 16 rounded up to 8, W = N / rows
 * per partition, above 64, or a plain store whose partition rows are not a
 * multiple of 128; e.g. B = 131072 over 4096
 * partitions; the slot lines are then read inside the row stream, whose
 * traffic follows which rows the batch touches). */
int gvs_get_option(gvs_handle *h, const char *key, int64_t *value);

/* Enable (on != 0) per-stage HIP-event timing of subsequent batches. */
int gvs_set_timing(gvs_handle *h, int on);

/* Device timing of the last batch, per pipeline stage, from HIP events on the
 * handle's stream.  names[i] points at static strings. Returns the count. */
int gvs_last_timings(gvs_handle *h, const char **names, float *ms, int cap);

const char *gvs_last_error(gvs_handle *h);
const char *gvs_version(void);

/* ---------------------------------------------------------------------------
 * Block store: the mc-oblivious-traits ORAM<1024> surface, batched
 * (ORAM::access(index, f) with f: FnOnce(&mut A64Bytes<1024>)).
 *
 * `capacity` 1 KiB blocks, all zero initially, kept in the message table's
 * layout and updated by the same fixed-slot table pass.  One
 * call applies n <= max_batch ops in submission order: GVS_ORAM_READ returns
 * the block, GVS_ORAM_WRITE returns the block and then replaces it with
 * `data` (the callback's view before it writes).  The launch sequence, grids,
 * HBM bytes and kernel durations depend only on (capacity, max_batch, n).  An
 * index >= capacity or an unknown op fails the whole call with
 * GVS_ERR_INVALID_ARG and applies nothing.
 * ------------------------------------------------------------------------- */
typedef struct gvs_oram gvs_oram;

#define GVS_ORAM_READ 0u
#define GVS_ORAM_WRITE 1u

typedef struct gvs_oram_config {
  uint64_t capacity;       /* blocks: power of two in [4096, 2^32] */
  uint32_t max_batch;      /* power of two in [1024, 2^19] */
  uint32_t device;
  uint8_t secret_key[32];  /* storage keys when flags has GVS_FLAG_AUTH_STORAGE */
  uint32_t flags;
  uint32_t reserved[3];    /* zero */
} gvs_oram_config;         /* 64 B */

typedef struct gvs_block_op {
  uint64_t index;
  uint32_t op;             /* GVS_ORAM_READ / GVS_ORAM_WRITE */
  uint32_t reserved;
  uint8_t data[1024];      /* GVS_ORAM_WRITE: the new block */
} gvs_block_op;            /* 1040 B */

int gvs_oram_create(const gvs_oram_config *cfg, gvs_oram **out);
int gvs_oram_destroy(gvs_oram *o);
/* ops: n host gvs_block_op; out: n x 1024 bytes, the block each op saw. */
int gvs_oram_access_batch(gvs_oram *o, const gvs_block_op *ops, uint32_t n, uint8_t *out);
/* The same with device buffers. */
int gvs_oram_access_batch_device(gvs_oram *o, const void *d_ops, uint32_t n, void *d_out);
int gvs_oram_set_timing(gvs_oram *o, int on);
int gvs_oram_last_timings(gvs_oram *o, const char **names, float *ms, int cap);
const char *gvs_oram_last_error(gvs_oram *o);

/* ---------------------------------------------------------------------------
 * Key-value map: the mc-oblivious-traits ObliviousHashMap<16, 1024> surface,
 * batched (access_and_insert / read / remove with u32
 * OMAP_* statuses; the callback is a per-op choice of what to write).
 *
 * `capacity` rows of 1 KiB values; a 16-B key lives in the partition its
 * keyed hash selects (W partitions of S rows, the message table's layout,
 * DESIGN.md §10).  One call applies n <= max_batch ops in submission order:
 *   GVS_OMAP_READ    read(key): FOUND and the value, or NOT_FOUND
 *   GVS_OMAP_WRITE   access_and_insert with a callback that overwrites:
 *                    FOUND / NOT_FOUND, the value before, then `value` stored
 *   GVS_OMAP_INSERT  access_and_insert(key, default = `value`) with a callback
 *                    that keeps: FOUND and the value, or NOT_FOUND and the
 *                    default, which is inserted
 *   GVS_OMAP_REMOVE  remove(key): FOUND and the removed value, or NOT_FOUND
 * An all-zero key is OMAP_INVALID_KEY.  [D] New keys of a batch are admitted
 * into their partition's free rows (free when the batch starts) in keyed-hash
 * order; an INSERT / WRITE of a key that is not admitted gets OMAP_OVERFLOW
 * and changes nothing.  More distinct keys in one partition in one batch
 * than its group slots (mean + 8 sigma + 16 for uniformly hashed keys, at
 * most S) fails the batch with GVS_ERR_BATCH_OVERFLOW before any state
 * changes.  The launch sequence, grids, HBM bytes and kernel durations
 * depend only on (capacity, max_batch, n).  Plain storage only (flags 0).
 * ------------------------------------------------------------------------- */
typedef struct gvs_omap gvs_omap;
typedef gvs_oram_config gvs_omap_config;

#define GVS_OMAP_READ 0u
#define GVS_OMAP_WRITE 1u
#define GVS_OMAP_INSERT 2u
#define GVS_OMAP_REMOVE 3u

/* statuses (mc-oblivious-traits OMAP_* codes) */
#define GVS_OMAP_FOUND 0u
#define GVS_OMAP_NOT_FOUND 1u
#define GVS_OMAP_OVERFLOW 2u
#define GVS_OMAP_INVALID_KEY 3u

typedef struct gvs_omap_op {
  uint8_t key[16];
  uint32_t op;             /* GVS_OMAP_* */
  uint32_t reserved[3];
  uint8_t value[1024];     /* WRITE: the new value; INSERT: the default */
} gvs_omap_op;             /* 1056 B */

typedef struct gvs_omap_result {
  uint8_t value[1024];     /* the value the op saw (see above); zero if none */
  uint32_t status;         /* GVS_OMAP_FOUND .. GVS_OMAP_INVALID_KEY */
  uint32_t reserved[3];
} gvs_omap_result;         /* 1040 B */

int gvs_omap_create(const gvs_omap_config *cfg, gvs_omap **out);
int gvs_omap_destroy(gvs_omap *o);
int gvs_omap_access_batch(gvs_omap *o, const gvs_omap_op *ops, uint32_t n, gvs_omap_result *out);
int gvs_omap_access_batch_device(gvs_omap *o, const void *d_ops, uint32_t n, void *d_out);
int gvs_omap_set_timing(gvs_omap *o, int on);
int gvs_omap_last_timings(gvs_omap *o, const char **names, float *ms, int cap);
const char *gvs_omap_last_error(gvs_omap *o);

#ifdef __cplusplus
}
#endif

#endif /* GVSTORE_H */
