/*
 * gvs_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of grapevine's CRUD store semantics ("seqmodel"), used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product path (libgvstore.so) never links or calls this.
 *
 * Parity status: the hot-path code of the reference (mc-oblivious and the
 * grapevine enclave handler) is absent from /root/reference (SURVEY.md §0,
 * §8(c)); no store-level golden vectors exist.  Store-level parity is
 * therefore UNPINNED: this model follows the written spec
 * (api/proto/grapevine.proto:57-122, README.md:73-175, types/src/lib.rs:13-137)
 * and the precedence/batching decisions of DESIGN.md §2.  Its primitives are
 * pinned: SipHash-2-4 against the SipHash paper vectors and CPython's built-in
 * siphash24 (tests/test_oracle_primitives.py); the wire sizes against the
 * reference's own constant-size tests (api/tests/grapevine_types.rs:22-55).
 */
#ifndef GVS_ORACLE_H
#define GVS_ORACLE_H

#include "../include/gvstore.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gvo_model gvo_model;

typedef struct gvo_gen_params {
  uint32_t pct_create, pct_read, pct_update, pct_delete; /* sum to 100 */
  uint32_t pct_next;          /* % of READ/DELETE sent with a zero msg_id */
  uint32_t pct_miss;          /* % of by-id ops with a random (absent) id */
  uint32_t pct_bad_auth;      /* % of by-id ops authenticated by a stranger */
  uint32_t pct_bad_recipient; /* % of UPDATE/DELETE naming a wrong recipient */
  uint32_t pct_hard_error;    /* % malformed (zero auth / bad type / zero-id update) */
  uint32_t pct_zero_recipient;/* % of CREATE with an all-zero recipient */
  uint32_t pct_hot;           /* % of CREATE/next ops aimed at identity 0 */
  uint32_t n_identities;      /* size of the identity pool */
  uint64_t ts_base;           /* timestamps are ts_base + running op index */
} gvo_gen_params;

/* SipHash-2-4 (Aumasson & Bernstein 2012), 64-bit output. */
uint64_t gvo_siphash24(uint64_t k0, uint64_t k1, const uint8_t *m, size_t len);
/* 4-round Feistel PRP over 128 bits used for message ids. */
void gvo_id_encode(const uint8_t key[16], uint32_t slot, uint64_t ctr,
                   uint8_t out[16]);
/* The same for shard `shard` of a sharded store (tag ID_TAG ^ shard << 8). */
void gvo_id_encode_shard(const uint8_t key[16], uint32_t shard, uint32_t slot, uint64_t ctr,
                         uint8_t out[16]);
int gvo_id_decode_shard(const uint8_t key[16], const uint8_t id[16], uint64_t n_slots,
                        uint32_t n_shards, uint32_t *shard, uint32_t *slot, uint64_t *ctr);
/* returns 1 if the id decodes to (slot < n_slots, tag ok) */
int gvo_id_decode(const uint8_t key[16], const uint8_t id[16], uint64_t n_slots,
                  uint32_t *slot, uint64_t *ctr);
void gvo_recipient_hash(const uint8_t key[16], const uint8_t x[32],
                        uint64_t *h_hi, uint64_t *h_lo);

gvo_model *gvo_create(const gvs_config *cfg);
void gvo_destroy(gvo_model *m);
/* Apply a batch in the engine's linearisation order; responses in request order. */
int gvo_process_batch(gvo_model *m, const gvs_request *reqs, uint32_t n,
                      gvs_response *out);
/* Expiry sweep (gvs_set_expiry_cutoff). */
void gvo_set_expiry_cutoff(gvo_model *m, uint64_t cutoff);
/* The plain sequential handler on one request (no batch reordering). */
void gvo_apply_one(gvo_model *m, const gvs_request *req, gvs_response *out);

uint64_t gvo_messages(const gvo_model *m);
/* copy the slot-addressed message table (N records) */
int gvo_dump_messages(const gvo_model *m, gvs_record *dst, uint64_t n);
uint64_t gvo_mailboxes(const gvo_model *m);
uint64_t gvo_creation_counter(const gvo_model *m);
/* copy out a live message by index in the live list (0 <= i < messages) */
int gvo_live_message(const gvo_model *m, uint64_t i, gvs_record *out);
/* FNV-1a style digest over the whole logical state (ids, records, mailboxes) */
uint64_t gvo_state_digest(const gvo_model *m);

/* Seeded synthetic request stream, drawn against the model's current state
 * (live ids/recipients), SplitMix64 driven.  `rng` is updated in place. */
void gvo_identity(uint32_t i, uint8_t out[32]);
void gvo_gen_batch(const gvo_model *m, const gvo_gen_params *p, uint64_t *rng,
                   gvs_request *reqs, uint32_t n, uint64_t op_base);

/* Sharded store: S seqmodels behind the engine's routing rule
 * and its fixed per-(source, shard) capacity C.  `key` is the 32-byte secret
 * key of gvs_config. */
uint32_t gvo_route(const uint8_t key[32], const gvs_request *rq, uint32_t i, uint32_t n_shards,
                   uint64_t n_slots);
uint32_t gvo_route_capacity(uint32_t batch, uint32_t n_shards);
#define GVO_ROUTE_KEY_CAP 64u /* requests routed per routing key per source window */
uint32_t gvo_route_key(const uint8_t key[32], const gvs_request *rq);
typedef struct gvo_cluster gvo_cluster;
gvo_cluster *gvo_cluster_create(const gvs_config *cfg); /* cfg->shard_count shards */
void gvo_cluster_destroy(gvo_cluster *c);
uint32_t gvo_cluster_capacity(const gvo_cluster *c);
gvo_model *gvo_cluster_shard(gvo_cluster *c, uint32_t k);
/* n <= S * max_batch; source rank k submitted requests [k*B, (k+1)*B).
 * GVS_ERR_BATCH_OVERFLOW (nothing applied) if one source has more than C
 * requests for one shard. */
int gvo_cluster_process(gvo_cluster *c, const gvs_request *reqs, uint32_t n, gvs_response *out);
void gvo_cluster_set_expiry_cutoff(gvo_cluster *c, uint64_t cutoff);
uint32_t gvo_shard_batch(uint64_t m); /* ops per shard pipeline for m slots */
uint64_t gvo_cluster_messages(const gvo_cluster *c);
uint64_t gvo_cluster_mailboxes(const gvo_cluster *c);
void gvo_cluster_gen_batch(const gvo_cluster *c, const gvo_gen_params *p, uint64_t *rng,
                           gvs_request *reqs, uint32_t n, uint64_t op_base);

/* Authenticated-storage format (gvs_seal.c): AES-128 per
 * FIPS-197, BLAKE2b per RFC 7693, and the sealing of one stored row. */
void gvo_aes128_expand(const uint8_t key[16], uint8_t rk[176]);
void gvo_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]);
void gvo_blake2b(const uint8_t *key, size_t keylen, const uint8_t *person, const uint8_t *msg,
                 size_t len, uint8_t *out, size_t outlen);
void gvo_storage_keys(const uint8_t secret[32], uint8_t aes_key[16], uint8_t mac_key[32]);
void gvo_uhash_keys(const uint8_t secret[32], uint32_t nh[268], uint64_t l3k[16], uint32_t l3p[4]);
void gvo_row_hash(const uint32_t nh[268], const uint64_t l3k[16], const uint32_t l3p[4],
                  const uint8_t ct[1024], uint8_t out[16]);
void gvo_seal_row(const uint8_t secret[32], uint32_t table, uint64_t row, uint32_t epoch,
                  const uint8_t pt[1024], const uint8_t *side_pt, uint8_t ct[1024],
                  uint8_t *side_ct, uint8_t tag[16]);

/* Path ORAM restatement of the reference's CPU path (gvs_pathoram.c): the
 * same handler semantics over three Path ORAMs; the timed CPU baseline. */
typedef struct gvp_model gvp_model;
gvp_model *gvp_create(const gvs_config *cfg);
void gvp_destroy(gvp_model *m);
int gvp_process_batch(gvp_model *m, const gvs_request *reqs, uint32_t n, gvs_response *out);
void gvp_apply_one(gvp_model *m, const gvs_request *req, gvs_response *out);
uint64_t gvp_messages(const gvp_model *m);
uint64_t gvp_mailboxes(const gvp_model *m);
uint64_t gvp_oram_accesses(const gvp_model *m);

#ifdef __cplusplus
}
#endif
#endif
