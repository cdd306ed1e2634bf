/*
 * gvs_oracle.c — TEST INFRASTRUCTURE ONLY (see gvs_oracle.h for the parity
 * status).  A plain, non-oblivious, one-request-at-a-time restatement of the
 * grapevine enclave's CRUD handler over a slot-addressed message table and a
 * partitioned mailbox directory.  Every rule cites the reference text it
 * follows; decisions the reference leaves open are marked [D] and documented
 * in DESIGN.md §2.
 */
#include "gvs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ID_TAG 0x47565331u /* "GVS1": plaintext tag inside every message id [D] */

/* ---------------------------------------------------------------- SipHash */

static inline uint64_t rotl64(uint64_t x, int b) {
  return (x << b) | (x >> (64 - b));
}
static inline uint64_t ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
static inline void st64(uint8_t *p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

#define SIPROUND                                                              \
  do {                                                                        \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);             \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                                  \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                                  \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);             \
  } while (0)

uint64_t gvo_siphash24(uint64_t k0, uint64_t k1, const uint8_t *m, size_t len) {
  uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
  uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
  uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
  uint64_t v3 = 0x7465646279746573ULL ^ k1;
  size_t nb = len / 8;
  for (size_t i = 0; i < nb; ++i) {
    uint64_t mi = ld64(m + 8 * i);
    v3 ^= mi;
    SIPROUND;
    SIPROUND;
    v0 ^= mi;
  }
  uint64_t b = ((uint64_t)len) << 56;
  for (size_t j = 0; j < (len & 7); ++j) b |= ((uint64_t)m[8 * nb + j]) << (8 * j);
  v3 ^= b;
  SIPROUND;
  SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  SIPROUND;
  SIPROUND;
  SIPROUND;
  SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

/* ------------------------------------------------------------- id PRP [D] */
/* msg ids: CREATE "ignores the given id and chooses a random nonzero id"
 * (grapevine.proto:66-79).  [D] The id is a 128-bit keyed PRP (4-round
 * Luby-Rackoff Feistel, SipHash-2-4 round function) of (slot | TAG<<32, ctr):
 * pseudorandom to anyone without the key, unique by construction (so status 3
 * MESSAGE_ID_ALREADY_IN_USE cannot occur), and decodable to the slot. */

static uint64_t feistel_f(const uint8_t key[16], int r, uint64_t x) {
  uint8_t msg[16];
  st64(msg, x);
  st64(msg + 8, (uint64_t)r);
  return gvo_siphash24(ld64(key), ld64(key + 8), msg, 16);
}

/* [D] shard k of a sharded store issues ids with tag ID_TAG ^ k << 8, so an
 * id names its shard; shard 0 and the unsharded store use
 * ID_TAG itself. */
static uint32_t shard_tag(uint32_t shard) { return ID_TAG ^ (shard << 8); }

void gvo_id_encode_shard(const uint8_t key[16], uint32_t shard, uint32_t slot, uint64_t ctr,
                         uint8_t out[16]) {
  uint64_t L = (uint64_t)slot | ((uint64_t)shard_tag(shard) << 32), R = ctr;
  for (int r = 0; r < 4; ++r) {
    uint64_t nl = R, nr = L ^ feistel_f(key, r, R);
    L = nl;
    R = nr;
  }
  st64(out, L);
  st64(out + 8, R);
}

void gvo_id_encode(const uint8_t key[16], uint32_t slot, uint64_t ctr, uint8_t out[16]) {
  gvo_id_encode_shard(key, 0, slot, ctr, out);
}

static void id_plain(const uint8_t key[16], const uint8_t id[16], uint64_t *Lo, uint64_t *Ro) {
  uint64_t L = ld64(id), R = ld64(id + 8);
  for (int r = 3; r >= 0; --r) {
    uint64_t nl = R ^ feistel_f(key, r, L), nr = L;
    L = nl;
    R = nr;
  }
  *Lo = L;
  *Ro = R;
}

int gvo_id_decode_shard(const uint8_t key[16], const uint8_t id[16], uint64_t n_slots,
                        uint32_t n_shards, uint32_t *shard, uint32_t *slot, uint64_t *ctr) {
  uint64_t L, R;
  id_plain(key, id, &L, &R);
  uint32_t t = (uint32_t)(L >> 32) ^ ID_TAG;
  if ((t & 0xFF0000FFu) != 0) return 0;
  if ((t >> 8) >= (n_shards ? n_shards : 1u)) return 0;
  if ((uint64_t)(uint32_t)L >= n_slots) return 0;
  *shard = t >> 8;
  *slot = (uint32_t)L;
  *ctr = R;
  return 1;
}

int gvo_id_decode(const uint8_t key[16], const uint8_t id[16], uint64_t n_slots,
                  uint32_t *slot, uint64_t *ctr) {
  uint32_t shard;
  return gvo_id_decode_shard(key, id, n_slots, 1, &shard, slot, ctr);
}

/* recipient PRF: (h_hi, h_lo) = SipHash(X || 1), SipHash(X || 2); the
 * mailbox partition is the top log2(Q) bits of h_hi [D]. */
void gvo_recipient_hash(const uint8_t key[16], const uint8_t x[32],
                        uint64_t *h_hi, uint64_t *h_lo) {
  uint8_t msg[33];
  memcpy(msg, x, 32);
  msg[32] = 1;
  *h_hi = gvo_siphash24(ld64(key), ld64(key + 8), msg, 33);
  msg[32] = 2;
  *h_lo = gvo_siphash24(ld64(key), ld64(key + 8), msg, 33);
}

/* ------------------------------------------------------------------ model */

typedef struct mailbox {
  uint8_t x[32];
  uint32_t len;
  uint8_t ids[GVS_MAILBOX_SLOTS][16];
} mailbox;

struct gvo_model {
  gvs_config cfg;
  uint32_t shard;  /* index in a sharded store (tag of the ids it issues) */
  uint64_t N;
  uint32_t Q, Sr, B, logQ;
  uint8_t prp_key[16], hash_key[16];
  gvs_record *table;
  uint64_t count, ctr, n_mailboxes;
  uint32_t *ring;
  uint64_t ring_size, head, tail;
  mailbox *mb;     /* Q * Sr, partition q owns [q*Sr, q*Sr + pcount[q]) */
  uint32_t *pcount;
  uint32_t *live;  /* live slots */
  int64_t *live_pos;
  uint64_t n_live;
  /* expiry sweep */
  uint32_t X, W, S, xk, xep;
  uint64_t cutoff, batches;
  struct expiry_rec { uint8_t valid, id[16], rcpt[32]; } *xp, *xq; /* X pending deletes; next */
};

static int is_zero(const uint8_t *p, size_t n) {
  uint8_t acc = 0;
  for (size_t i = 0; i < n; ++i) acc |= p[i];
  return acc == 0;
}
static int is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

gvo_model *gvo_create(const gvs_config *cfg) {
  if (!cfg || !is_pow2(cfg->msg_capacity) || cfg->msg_capacity < 256 ||
      !is_pow2(cfg->mailbox_partitions) || cfg->mailbox_partition_slots == 0 ||
      cfg->max_batch < 1024 || cfg->max_batch % 1024) /* a shard pipeline: any multiple */
    return NULL;
  gvo_model *m = (gvo_model *)calloc(1, sizeof *m);
  if (!m) return NULL;
  m->cfg = *cfg;
  m->shard = cfg->shard_count > 1 ? cfg->shard_index : 0;
  m->N = cfg->msg_capacity;
  m->Q = cfg->mailbox_partitions;
  m->Sr = cfg->mailbox_partition_slots;
  m->B = cfg->max_batch;
  m->logQ = 0;
  while ((1u << m->logQ) < m->Q) m->logQ++;
  memcpy(m->prp_key, cfg->secret_key, 16);
  memcpy(m->hash_key, cfg->secret_key + 16, 16);
  m->table = (gvs_record *)calloc(m->N, sizeof(gvs_record));
  m->ring_size = m->N + m->B;
  m->ring = (uint32_t *)malloc(m->ring_size * sizeof(uint32_t));
  m->mb = (mailbox *)calloc((size_t)m->Q * m->Sr, sizeof(mailbox));
  m->pcount = (uint32_t *)calloc(m->Q, sizeof(uint32_t));
  m->live = (uint32_t *)malloc(m->N * sizeof(uint32_t));
  m->live_pos = (int64_t *)malloc(m->N * sizeof(int64_t));
  if (!m->table || !m->ring || !m->mb || !m->pcount || !m->live || !m->live_pos) {
    gvo_destroy(m);
    return NULL;
  }
  /* the free ring starts as slots 0..N-1 in order [D] */
  for (uint64_t s = 0; s < m->N; ++s) {
    m->ring[s] = (uint32_t)s;
    m->live_pos[s] = -1;
  }
  m->head = 0;
  m->tail = m->N;
  /* message-table partitions of the engine (gvs_engine.hip engine_init): the
   * expiry sweep's selection rule is defined over them [D] */
  uint64_t S = cfg->rows_per_partition ? cfg->rows_per_partition : m->N / 4096;
  if (S < 256) S = 256;
  if (S > 4096) S = 4096;
  if (S > m->N) S = m->N;
  m->S = (uint32_t)S;
  m->W = (uint32_t)(m->N / S);
  m->X = cfg->expiry_per_batch;
  if (m->X) {
    /* a shard model's B is its pipeline (gvo_shard_batch), X slots included */
    if (!is_pow2(m->X) || m->X > (cfg->shard_count > 1 ? m->B - 1 : m->B / 2)) {
      gvo_destroy(m);
      return NULL;
    }
    m->xep = m->X >= m->W ? m->X / m->W : 1;
    m->xk = m->X >= m->W ? 1 : m->W / m->X;
    m->xp = calloc(m->X, sizeof *m->xp);
    m->xq = calloc(m->X, sizeof *m->xq);
    if (!m->xp || !m->xq || m->xep > 8) { /* at most 8 records per partition and batch */
      gvo_destroy(m);
      return NULL;
    }
  }
  return m;
}

void gvo_destroy(gvo_model *m) {
  if (!m) return;
  free(m->table);
  free(m->ring);
  free(m->mb);
  free(m->pcount);
  free(m->live);
  free(m->live_pos);
  free(m->xp);
  free(m->xq);
  free(m);
}

static uint32_t partition_of(const gvo_model *m, const uint8_t x[32]) {
  uint64_t hi, lo;
  gvo_recipient_hash(m->hash_key, x, &hi, &lo);
  return m->logQ ? (uint32_t)(hi >> (64 - m->logQ)) : 0u;
}

static mailbox *find_mailbox(gvo_model *m, const uint8_t x[32], uint32_t *q_out) {
  uint32_t q = partition_of(m, x);
  if (q_out) *q_out = q;
  mailbox *base = m->mb + (size_t)q * m->Sr;
  for (uint32_t i = 0; i < m->pcount[q]; ++i)
    if (memcmp(base[i].x, x, 32) == 0) return &base[i];
  return NULL;
}

static void remove_mailbox(gvo_model *m, mailbox *mb) {
  uint32_t q = partition_of(m, mb->x);
  mailbox *base = m->mb + (size_t)q * m->Sr;
  uint32_t last = --m->pcount[q];
  if (mb != &base[last]) *mb = base[last];
  memset(&base[last], 0, sizeof(mailbox));
  m->n_mailboxes--;
}

static gvs_record *lookup(gvo_model *m, const uint8_t id[16], uint32_t *slot_out) {
  uint32_t slot, shard;
  uint64_t ctr;
  if (!gvo_id_decode_shard(m->prp_key, id, m->N, 1u << 16, &shard, &slot, &ctr)) return NULL;
  if (shard != m->shard) return NULL; /* issued by another shard */
  gvs_record *r = &m->table[slot];
  if (memcmp(r->msg_id, id, 16) != 0) return NULL;
  if (slot_out) *slot_out = slot;
  return r;
}

static int auth_ok(const gvs_record *r, const uint8_t a[32]) {
  return memcmp(a, r->sender, 32) == 0 || memcmp(a, r->recipient, 32) == 0;
}

static void live_add(gvo_model *m, uint32_t slot) {
  m->live_pos[slot] = (int64_t)m->n_live;
  m->live[m->n_live++] = slot;
}
static void live_remove(gvo_model *m, uint32_t slot) {
  int64_t p = m->live_pos[slot];
  uint32_t last = m->live[--m->n_live];
  m->live[p] = last;
  m->live_pos[last] = p;
  m->live_pos[slot] = -1;
}

/* free a slot: zero the row and append it to the free ring [D] */
static void free_slot(gvo_model *m, uint32_t slot) {
  memset(&m->table[slot], 0, sizeof(gvs_record));
  m->ring[m->tail % m->ring_size] = slot;
  m->tail++;
  m->count--;
  live_remove(m, slot);
}

static void resp_fail(gvs_response *o, uint32_t status, uint64_t ts) {
  memset(o, 0, sizeof *o);
  o->record.timestamp = ts; /* nonzero ts keeps QueryResponse at 1042 B [D] */
  o->status_code = status;
}
static void resp_hard(gvs_response *o) { memset(o, 0, sizeof *o); }
static void resp_ok(gvs_response *o, const gvs_record *r) {
  memset(o, 0, sizeof *o);
  o->record = *r;
  o->status_code = GVS_STATUS_SUCCESS;
}

/* CREATE, grapevine.proto:66-79, README.md:166-167.
 * [D] check order: INVALID_RECIPIENT(4), TOO_MANY_MESSAGES(7),
 * TOO_MANY_MESSAGES_FOR_RECIPIENT(5), TOO_MANY_RECIPIENTS(6). */
static void do_create(gvo_model *m, const gvs_request *rq, gvs_response *o) {
  if (is_zero(rq->recipient, 32)) {
    resp_fail(o, GVS_STATUS_INVALID_RECIPIENT, rq->timestamp);
    return;
  }
  if (m->count >= m->N) {
    resp_fail(o, GVS_STATUS_TOO_MANY_MESSAGES, rq->timestamp);
    return;
  }
  uint32_t q;
  mailbox *mb = find_mailbox(m, rq->recipient, &q);
  if (mb && mb->len >= GVS_MAILBOX_SLOTS) {
    resp_fail(o, GVS_STATUS_TOO_MANY_MESSAGES_FOR_RECIPIENT, rq->timestamp);
    return;
  }
  if (!mb && m->pcount[q] >= m->Sr) {
    resp_fail(o, GVS_STATUS_TOO_MANY_RECIPIENTS, rq->timestamp);
    return;
  }
  uint32_t slot = m->ring[m->head % m->ring_size];
  m->head++;
  uint64_t ctr = m->ctr++;
  gvs_record *r = &m->table[slot];
  gvo_id_encode_shard(m->prp_key, m->shard, slot, ctr, r->msg_id);
  memcpy(r->sender, rq->auth_identity, 32); /* sender = auth_identity */
  memcpy(r->recipient, rq->recipient, 32);
  r->timestamp = rq->timestamp; /* server time, README.md:143-144 */
  memcpy(r->payload, rq->payload, GVS_PAYLOAD_BYTES);
  m->count++;
  live_add(m, slot);
  if (!mb) {
    mb = m->mb + (size_t)q * m->Sr + m->pcount[q]++;
    memset(mb, 0, sizeof *mb);
    memcpy(mb->x, rq->recipient, 32);
    m->n_mailboxes++;
  }
  memcpy(mb->ids[mb->len++], r->msg_id, 16); /* FIFO per recipient [D] */
  resp_ok(o, r);
}

/* READ, grapevine.proto:81-90: by id (auth must be sender or recipient) or,
 * with a zero id, the next (oldest) message addressed to auth_identity. */
static void do_read(gvo_model *m, const gvs_request *rq, gvs_response *o) {
  if (is_zero(rq->msg_id, 16)) {
    mailbox *mb = find_mailbox(m, rq->auth_identity, NULL);
    if (!mb || mb->len == 0) {
      resp_fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
      return;
    }
    gvs_record *r = lookup(m, mb->ids[0], NULL);
    resp_ok(o, r);
    return;
  }
  gvs_record *r = lookup(m, rq->msg_id, NULL);
  if (!r || !auth_ok(r, rq->auth_identity)) {
    resp_fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
    return;
  }
  resp_ok(o, r);
}

/* UPDATE, grapevine.proto:92-102, README.md:170-172. */
static void do_update(gvo_model *m, const gvs_request *rq, gvs_response *o) {
  gvs_record *r = lookup(m, rq->msg_id, NULL);
  if (!r || !auth_ok(r, rq->auth_identity)) {
    resp_fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
    return;
  }
  if (memcmp(rq->recipient, r->recipient, 32) != 0) {
    resp_fail(o, GVS_STATUS_INVALID_RECIPIENT, rq->timestamp);
    return;
  }
  memcpy(r->payload, rq->payload, GVS_PAYLOAD_BYTES);
  r->timestamp = rq->timestamp;
  resp_ok(o, r);
}

static void mailbox_remove_id(mailbox *mb, const uint8_t id[16]) {
  for (uint32_t i = 0; i < mb->len; ++i) {
    if (memcmp(mb->ids[i], id, 16) == 0) {
      memmove(mb->ids[i], mb->ids[i + 1], (size_t)(mb->len - i - 1) * 16);
      mb->len--;
      memset(mb->ids[mb->len], 0, 16);
      return;
    }
  }
}

/* DELETE, grapevine.proto:104-118, README.md:173-175. */
static void do_delete(gvo_model *m, const gvs_request *rq, gvs_response *o) {
  if (is_zero(rq->msg_id, 16)) {
    mailbox *mb = find_mailbox(m, rq->auth_identity, NULL);
    if (!mb || mb->len == 0) {
      resp_fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
      return;
    }
    uint8_t id[16];
    memcpy(id, mb->ids[0], 16);
    mailbox_remove_id(mb, id);
    uint32_t slot;
    gvs_record *r = lookup(m, id, &slot);
    resp_ok(o, r);
    free_slot(m, slot);
    if (mb->len == 0) remove_mailbox(m, mb);
    return;
  }
  uint32_t slot;
  gvs_record *r = lookup(m, rq->msg_id, &slot);
  if (!r || !auth_ok(r, rq->auth_identity)) {
    resp_fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
    return;
  }
  if (memcmp(rq->recipient, r->recipient, 32) != 0) {
    resp_fail(o, GVS_STATUS_INVALID_RECIPIENT, rq->timestamp);
    return;
  }
  mailbox *mb = find_mailbox(m, r->recipient, NULL);
  resp_ok(o, r);
  if (mb) {
    mailbox_remove_id(mb, rq->msg_id);
    if (mb->len == 0) remove_mailbox(m, mb);
  }
  free_slot(m, slot);
}

/* fail-fast rules, grapevine.proto:57-64 and :95 */
static int is_hard_error(const gvs_request *rq) {
  uint32_t t = rq->request_type;
  if (t < GVS_REQUEST_CREATE || t > GVS_REQUEST_DELETE) return 1;
  if (is_zero(rq->auth_identity, 32)) return 1;
  if (t == GVS_REQUEST_UPDATE && is_zero(rq->msg_id, 16)) return 1;
  return 0;
}

void gvo_apply_one(gvo_model *m, const gvs_request *rq, gvs_response *o) {
  if (is_hard_error(rq)) {
    resp_hard(o);
    return;
  }
  switch (rq->request_type) {
    case GVS_REQUEST_CREATE: do_create(m, rq, o); break;
    case GVS_REQUEST_READ: do_read(m, rq, o); break;
    case GVS_REQUEST_UPDATE: do_update(m, rq, o); break;
    default: do_delete(m, rq, o); break;
  }
}

/* [D] batch linearisation: class 0 = READ/DELETE with zero id ("next"),
 * class 1 = CREATE, class 2 = everything else; submission order inside a
 * class.  Any order is a valid linearisation of concurrently pending
 * requests; this one lets the GPU resolve a batch in three table passes. */
static int batch_class(const gvs_request *rq) {
  if (is_hard_error(rq)) return 2;
  if (rq->request_type == GVS_REQUEST_CREATE) return 1;
  if ((rq->request_type == GVS_REQUEST_READ || rq->request_type == GVS_REQUEST_DELETE) &&
      is_zero(rq->msg_id, 16))
    return 0;
  return 2;
}

void gvo_set_expiry_cutoff(gvo_model *m, uint64_t cutoff) { m->cutoff = cutoff; }

/* Expiry delete k of a batch: the message recorded by the
 * previous batch's sweep is deleted as by its recipient, if it still exists
 * and its timestamp is still < cutoff (an UPDATE since then keeps it). */
static void do_expire(gvo_model *m, const struct expiry_rec *x) {
  if (!x->valid) return;
  gvs_record *r = lookup(m, x->id, NULL);
  if (!r || !(r->timestamp < m->cutoff)) return;
  gvs_request rq;
  gvs_response o;
  memset(&rq, 0, sizeof rq);
  memcpy(rq.msg_id, x->id, 16);
  memcpy(rq.auth_identity, x->rcpt, 32);
  memcpy(rq.recipient, x->rcpt, 32);
  rq.request_type = GVS_REQUEST_DELETE;
  do_delete(m, &rq, &o);
}

/* The sweep of batch b [D]: on the table as it stands before
 * the batch (the engine's table pass of batch b applies batch b-1's final row
 * states and reads every row), partitions w = b (mod xk) each record their
 * first xep messages with timestamp < cutoff that the batch does not already
 * delete (the records of batch b-1's sweep), in slot order within the
 * partition (slot s is in partition s mod W at offset s div W), at
 * xq[(w / xk) * xep ..]; unused entries are invalid.  Batch b+1 deletes them. */
static int pending_expiry(const gvo_model *m, const uint8_t id[16]) {
  for (uint32_t k = 0; k < m->X; ++k)
    if (m->xp[k].valid && memcmp(m->xp[k].id, id, 16) == 0) return 1;
  return 0;
}

static void expiry_sweep(gvo_model *m) {
  memset(m->xq, 0, m->X * sizeof *m->xq);
  for (uint32_t w = m->batches % m->xk; w < m->W; w += m->xk) {
    uint32_t c = 0;
    struct expiry_rec *dst = m->xq + (uint64_t)(w / m->xk) * m->xep;
    for (uint64_t o = 0; o < m->S && c < m->xep; ++o) {
      const gvs_record *r = &m->table[o * m->W + w];
      if (is_zero(r->msg_id, 16) || !(r->timestamp < m->cutoff)) continue;
      if (m->xk == 1 && pending_expiry(m, r->msg_id)) continue;
      dst[c].valid = 1;
      memcpy(dst[c].id, r->msg_id, 16);
      memcpy(dst[c].rcpt, r->recipient, 32);
      c++;
    }
  }
}

int gvo_process_batch(gvo_model *m, const gvs_request *reqs, uint32_t n,
                      gvs_response *out) {
  if (n > m->B - m->X) return GVS_ERR_INVALID_ARG;
  if (m->X) expiry_sweep(m);
  for (int cls = 0; cls < 3; ++cls)
    for (uint32_t i = 0; i < n; ++i)
      if (batch_class(&reqs[i]) == cls) gvo_apply_one(m, &reqs[i], &out[i]);
  if (m->X) {
    /* the expiry deletes occupy the batch's last X slots: by-id class, after
     * every request */
    for (uint32_t k = 0; k < m->X; ++k) do_expire(m, &m->xp[k]);
    struct expiry_rec *t = m->xp;
    m->xp = m->xq;
    m->xq = t;
  }
  m->batches++;
  return GVS_OK;
}

uint64_t gvo_messages(const gvo_model *m) { return m->count; }

int gvo_dump_messages(const gvo_model *m, gvs_record *dst, uint64_t n) {
  if (n < m->N) return -1;
  memcpy(dst, m->table, m->N * sizeof(gvs_record));
  return 0;
}
uint64_t gvo_mailboxes(const gvo_model *m) { return m->n_mailboxes; }
uint64_t gvo_creation_counter(const gvo_model *m) { return m->ctr; }

int gvo_live_message(const gvo_model *m, uint64_t i, gvs_record *out) {
  if (i >= m->n_live) return -1;
  *out = m->table[m->live[i]];
  return 0;
}

static uint64_t fnv(uint64_t h, const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ULL;
  }
  return h;
}

uint64_t gvo_state_digest(const gvo_model *m) {
  uint64_t h = 0xcbf29ce484222325ULL;
  for (uint64_t s = 0; s < m->N; ++s)
    if (!is_zero(m->table[s].msg_id, 16)) {
      h = fnv(h, (const uint8_t *)&s, 8);
      h = fnv(h, (const uint8_t *)&m->table[s], sizeof(gvs_record));
    }
  /* mailboxes: order-independent sum of per-mailbox digests */
  uint64_t acc = 0;
  for (uint32_t q = 0; q < m->Q; ++q)
    for (uint32_t i = 0; i < m->pcount[q]; ++i) {
      const mailbox *mb = m->mb + (size_t)q * m->Sr + i;
      uint64_t d = fnv(0xcbf29ce484222325ULL, mb->x, 32);
      d = fnv(d, (const uint8_t *)mb->ids, (size_t)mb->len * 16);
      acc += d;
    }
  return h ^ (acc * 0x9e3779b97f4a7c15ULL);
}

/* ------------------------------------------------------ stream generator */

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static uint32_t rnd_below(uint64_t *s, uint32_t n) {
  return n ? (uint32_t)(((unsigned __int128)splitmix64(s) * n) >> 64) : 0u;
}
static void rnd_bytes(uint64_t *s, uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; i += 8) {
    uint64_t v = splitmix64(s);
    for (size_t j = 0; j < 8 && i + j < n; ++j) p[i + j] = (uint8_t)(v >> (8 * j));
  }
}

void gvo_identity(uint32_t i, uint8_t out[32]) {
  uint64_t s = 0x6772617065766e65ULL ^ ((uint64_t)i * 0xd1342543de82ef95ULL);
  for (int j = 0; j < 4; ++j) st64(out + 8 * j, splitmix64(&s) | 1u);
}

/* a model to draw a live message from: the only one, or (sharded store) one
 * chosen uniformly; NULL when it holds no message */
static const gvo_model *pick_model(const gvo_model *const *ms, uint32_t nm, uint64_t *rng) {
  const gvo_model *m = nm > 1 ? ms[rnd_below(rng, nm)] : ms[0];
  return m->n_live ? m : NULL;
}
static const gvs_record *pick_live(const gvo_model *m, uint64_t *rng) {
  return &m->table[m->live[rnd_below(rng, (uint32_t)m->n_live)]];
}

static void gen_requests(const gvo_model *const *ms, uint32_t nm, const gvo_gen_params *p,
                         uint64_t *rng, gvs_request *reqs, uint32_t n, uint64_t op_base) {
  uint32_t nid = p->n_identities ? p->n_identities : 1;
  for (uint32_t i = 0; i < n; ++i) {
    gvs_request *rq = &reqs[i];
    memset(rq, 0, sizeof *rq);
    rq->timestamp = p->ts_base + op_base + i + 1;
    rnd_bytes(rng, rq->payload, GVS_PAYLOAD_BYTES);
    rnd_bytes(rng, rq->msg_id, 16);
    uint32_t r = rnd_below(rng, 100), t;
    if (r < p->pct_create) t = GVS_REQUEST_CREATE;
    else if (r < p->pct_create + p->pct_read) t = GVS_REQUEST_READ;
    else if (r < p->pct_create + p->pct_read + p->pct_update) t = GVS_REQUEST_UPDATE;
    else t = GVS_REQUEST_DELETE;
    rq->request_type = t;
    gvo_identity(rnd_below(rng, nid), rq->auth_identity);
    gvo_identity(rnd_below(rng, nid), rq->recipient);

    if (rnd_below(rng, 100) < p->pct_hard_error) {
      switch (rnd_below(rng, 3)) {
        case 0: memset(rq->auth_identity, 0, 32); break;
        case 1: rq->request_type = rnd_below(rng, 2) ? 0u : 5u + rnd_below(rng, 100); break;
        default: rq->request_type = GVS_REQUEST_UPDATE; memset(rq->msg_id, 0, 16); break;
      }
      continue;
    }
    int hot = rnd_below(rng, 100) < p->pct_hot;
    if (t == GVS_REQUEST_CREATE) {
      if (hot) gvo_identity(0, rq->recipient);
      if (rnd_below(rng, 100) < p->pct_zero_recipient) memset(rq->recipient, 0, 32);
      continue;
    }
    if (t != GVS_REQUEST_UPDATE && rnd_below(rng, 100) < p->pct_next) {
      memset(rq->msg_id, 0, 16);
      if (hot) {
        gvo_identity(0, rq->auth_identity);
      } else {
        const gvo_model *m = pick_model(ms, nm, rng);
        if (m && rnd_below(rng, 100) < 70) memcpy(rq->auth_identity, pick_live(m, rng)->recipient, 32);
      }
      continue;
    }
    /* by-id operation */
    const gvo_model *m = pick_model(ms, nm, rng);
    if (m && rnd_below(rng, 100) >= p->pct_miss) {
      const gvs_record *lr = pick_live(m, rng);
      memcpy(rq->msg_id, lr->msg_id, 16);
      if (rnd_below(rng, 100) >= p->pct_bad_auth)
        memcpy(rq->auth_identity, rnd_below(rng, 2) ? lr->sender : lr->recipient, 32);
      if (rnd_below(rng, 100) >= p->pct_bad_recipient)
        memcpy(rq->recipient, lr->recipient, 32);
    } else {
      rq->msg_id[0] |= 1; /* random, nonzero, almost surely absent */
    }
  }
}

void gvo_gen_batch(const gvo_model *m, const gvo_gen_params *p, uint64_t *rng,
                   gvs_request *reqs, uint32_t n, uint64_t op_base) {
  gen_requests(&m, 1, p, rng, reqs, n, op_base);
}

/* ------------------------------------------------------ sharded store [D] */
/* DESIGN.md §6.  A message lives on the shard that owns its recipient's
 * mailbox, so every request touches exactly one shard; the routing rule is
 * restated here from grapevine_amd/csrc/gvs_route.h (route_dest).  Requests
 * of one batch reach a shard in (source rank, submission index) order, which
 * is global submission order, and each shard linearises its sub-batch as
 * gvo_process_batch does.  Shards share no state, so the result is a valid
 * linearisation of the whole batch. */

uint32_t gvo_route(const uint8_t key[32], const gvs_request *rq, uint32_t i, uint32_t n_shards,
                   uint64_t n_slots) {
  const uint32_t S = n_shards ? n_shards : 1u;
  const uint32_t spread = i % S;
  const uint32_t t = rq->request_type;
  const int id_zero = is_zero(rq->msg_id, 16);
  if (is_hard_error(rq)) return spread;
  const int next = (t == GVS_REQUEST_READ || t == GVS_REQUEST_DELETE) && id_zero;
  uint64_t hi, lo;
  if (t == GVS_REQUEST_CREATE) {
    if (is_zero(rq->recipient, 32)) return spread;
    gvo_recipient_hash(key + 16, rq->recipient, &hi, &lo);
    return (uint32_t)(lo & 0xFFFFu) % S;
  }
  if (next) {
    gvo_recipient_hash(key + 16, rq->auth_identity, &hi, &lo);
    return (uint32_t)(lo & 0xFFFFu) % S;
  }
  uint32_t shard, slot;
  uint64_t ctr;
  if (gvo_id_decode_shard(key, rq->msg_id, n_slots, S, &shard, &slot, &ctr)) return shard;
  return spread;
}

/* The routing key of a request (gvs_route.h route_dest_key): low 2 bits 1 =
 * create (its recipient's mailbox), 2 = next-message op (the caller's
 * mailbox), 3 = by-id op (its id), 0 = unkeyed (hard errors, zero
 * recipients), which are never shed. */
uint32_t gvo_route_key(const uint8_t key[32], const gvs_request *rq) {
  const uint32_t t = rq->request_type;
  const int id_zero = is_zero(rq->msg_id, 16);
  if (is_hard_error(rq)) return 0;
  const int next = (t == GVS_REQUEST_READ || t == GVS_REQUEST_DELETE) && id_zero;
  uint64_t hi, lo;
  if (t == GVS_REQUEST_CREATE) {
    if (is_zero(rq->recipient, 32)) return 0;
    gvo_recipient_hash(key + 16, rq->recipient, &hi, &lo);
    return ((uint32_t)(lo >> 32) & ~3u) | 1u;
  }
  if (next) {
    gvo_recipient_hash(key + 16, rq->auth_identity, &hi, &lo);
    return ((uint32_t)(lo >> 32) & ~3u) | 2u;
  }
  uint8_t msg[17];  /* keyed: id || 0x03 */
  memcpy(msg, rq->msg_id, 16);
  msg[16] = 3;
  const uint64_t h = gvo_siphash24(ld64(key + 16), ld64(key + 24), msg, 17);
  return ((uint32_t)(h >> 32) & ~3u) | 3u;
}

uint32_t gvo_route_capacity(uint32_t batch, uint32_t n_shards) {
  if (n_shards <= 1) return batch;
  double mu = (double)((batch + n_shards - 1) / n_shards);
  uint64_t c = (uint64_t)ceil(mu + 8.0 * sqrt(mu) + 64.0);
  c = (c + 63) / 64 * 64;
  return (uint32_t)(c < batch ? c : batch);
}

struct gvo_cluster {
  gvs_config cfg;
  uint32_t S, C, B;
  gvo_model **shard;
  gvs_request *sub;
  gvs_response *subout;
  uint32_t *dest, *cnt;
  uint8_t *shed;
  uint64_t *keys;
};

/* Ops per shard pipeline for m routed slots plus expiry deletes: the smaller
 * of the next power of two and the next multiple of 8192, at least 1024
 * (gvs_engine.hip shard_batch). */
uint32_t gvo_shard_batch(uint64_t m) {
  uint64_t p2 = 1024;
  while (p2 < m) p2 <<= 1;
  const uint64_t r = (m + 8191) / 8192 * 8192;
  const uint64_t be = p2 < r ? p2 : r;
  return (uint32_t)(be < 1024 ? 1024 : be);
}

gvo_cluster *gvo_cluster_create(const gvs_config *cfg) {
  if (!cfg || cfg->shard_count < 1) return NULL;
  if (cfg->expiry_per_batch > cfg->max_batch / 2) return NULL;
  gvo_cluster *c = (gvo_cluster *)calloc(1, sizeof *c);
  if (!c) return NULL;
  c->cfg = *cfg;
  c->S = cfg->shard_count;
  c->B = cfg->max_batch;
  c->C = cfg->route_capacity ? cfg->route_capacity : gvo_route_capacity(c->B, c->S);
  c->shard = (gvo_model **)calloc(c->S, sizeof(gvo_model *));
  c->sub = (gvs_request *)malloc((size_t)c->S * c->C * sizeof(gvs_request));
  c->subout = (gvs_response *)malloc((size_t)c->S * c->C * sizeof(gvs_response));
  c->dest = (uint32_t *)malloc((size_t)c->S * c->B * sizeof(uint32_t));
  c->cnt = (uint32_t *)malloc((size_t)c->S * c->S * sizeof(uint32_t));
  c->shed = (uint8_t *)malloc((size_t)c->S * c->B);
  c->keys = (uint64_t *)malloc((size_t)c->B * sizeof(uint64_t));
  if (!c->shard || !c->sub || !c->subout || !c->dest || !c->cnt || !c->shed || !c->keys) {
    gvo_cluster_destroy(c);
    return NULL;
  }
  for (uint32_t k = 0; k < c->S; ++k) {
    gvs_config sc = *cfg;
    sc.shard_count = c->S;
    sc.shard_index = k;
    sc.max_batch = gvo_shard_batch((uint64_t)c->S * c->C + cfg->expiry_per_batch);
    c->shard[k] = gvo_create(&sc);
    if (!c->shard[k]) {
      gvo_cluster_destroy(c);
      return NULL;
    }
  }
  return c;
}

void gvo_cluster_destroy(gvo_cluster *c) {
  if (!c) return;
  if (c->shard)
    for (uint32_t k = 0; k < c->S; ++k) gvo_destroy(c->shard[k]);
  free(c->shard);
  free(c->sub);
  free(c->subout);
  free(c->dest);
  free(c->cnt);
  free(c->shed);
  free(c->keys);
  free(c);
}

uint32_t gvo_cluster_capacity(const gvo_cluster *c) { return c->C; }
gvo_model *gvo_cluster_shard(gvo_cluster *c, uint32_t k) { return k < c->S ? c->shard[k] : NULL; }

static int cmp_u64(const void *a, const void *b) {
  const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

/* n <= S*B requests; source rank k submitted [k*B, (k+1)*B).
 * Hot keys [D] (gvs_route.h): in each source's window, the requests of one
 * routing key after its GVO_ROUTE_KEY_CAP-th are shed: they go to shard
 * (index mod S) as hard errors (no state change) and are answered
 * INTERNAL_ERROR with the request's time. */
int gvo_cluster_process(gvo_cluster *c, const gvs_request *reqs, uint32_t n, gvs_response *out) {
  if (n > c->S * c->B) return GVS_ERR_INVALID_ARG;
  memset(c->cnt, 0, (size_t)c->S * c->S * sizeof(uint32_t));
  memset(c->shed, 0, n);
  for (uint32_t s0 = 0; s0 < n; s0 += c->B) {
    const uint32_t m = n - s0 < c->B ? n - s0 : c->B;
    for (uint32_t i = 0; i < m; ++i)
      c->keys[i] = ((uint64_t)gvo_route_key(c->cfg.secret_key, &reqs[s0 + i]) << 32) | i;
    qsort(c->keys, m, sizeof(uint64_t), cmp_u64);
    for (uint32_t j = GVO_ROUTE_KEY_CAP; j < m; ++j) {
      const uint32_t k = (uint32_t)(c->keys[j] >> 32);
      if ((k & 3u) && (uint32_t)(c->keys[j - GVO_ROUTE_KEY_CAP] >> 32) == k)
        c->shed[s0 + (uint32_t)c->keys[j]] = 1;
    }
  }
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t src = i / c->B, d = gvo_route(c->cfg.secret_key, &reqs[i], i % c->B, c->S,
                                           c->cfg.msg_capacity);
    if (c->shed[i]) d = (i % c->B) % c->S;
    c->dest[i] = d;
    if (++c->cnt[src * c->S + d] > c->C) return GVS_ERR_BATCH_OVERFLOW; /* nothing applied */
  }
  for (uint32_t d = 0; d < c->S; ++d) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
      if (c->dest[i] == d) {
        c->sub[m] = reqs[i];
        if (c->shed[i]) c->sub[m].request_type = 0; /* travels as a hard error */
        ++m;
      }
    int rc = gvo_process_batch(c->shard[d], c->sub, m, c->subout);
    if (rc) return rc;
    m = 0;
    for (uint32_t i = 0; i < n; ++i)
      if (c->dest[i] == d) {
        out[i] = c->subout[m++];
        if (c->shed[i]) resp_fail(&out[i], GVS_STATUS_INTERNAL_ERROR, reqs[i].timestamp);
      }
  }
  return GVS_OK;
}

void gvo_cluster_set_expiry_cutoff(gvo_cluster *c, uint64_t cutoff) {
  for (uint32_t k = 0; k < c->S; ++k) gvo_set_expiry_cutoff(c->shard[k], cutoff);
}

uint64_t gvo_cluster_messages(const gvo_cluster *c) {
  uint64_t t = 0;
  for (uint32_t k = 0; k < c->S; ++k) t += c->shard[k]->count;
  return t;
}
uint64_t gvo_cluster_mailboxes(const gvo_cluster *c) {
  uint64_t t = 0;
  for (uint32_t k = 0; k < c->S; ++k) t += c->shard[k]->n_mailboxes;
  return t;
}

void gvo_cluster_gen_batch(const gvo_cluster *c, const gvo_gen_params *p, uint64_t *rng,
                           gvs_request *reqs, uint32_t n, uint64_t op_base) {
  gen_requests((const gvo_model *const *)c->shard, c->S, p, rng, reqs, n, op_base);
}
