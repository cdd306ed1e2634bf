/*
 * gvs_pathoram.c — TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * A CPU restatement of the reference's store path: the grapevine handler
 * (DESIGN.md §2 semantics) over Path ORAM, the mc-oblivious design the
 * reference names (README.md:16,49-50; SURVEY.md §8(a) a10-a12, [U] recall:
 * Z = 4 blocks per bucket, recursive position map, greedy eviction, stash).
 * mc-oblivious itself is absent from /root/reference and not in Cargo.lock,
 * so this is a restatement of its published algorithm, not a build of it.
 *
 *   message store : ORAM of N blocks x 1 KiB (block index = slot)
 *   mailbox rows  : ORAM of R = Q*S_r blocks x 1 KiB (recipient + 62 ids)
 *   directory     : ORAM of Q blocks x (S_r x 16 B): per row the recipient PRF
 *
 * Every request costs exactly four top-level ORAM accesses (directory,
 * mailbox row, message, directory), real or dummy, so READ / UPDATE / DELETE
 * are indistinguishable by access count (grapevine.proto:120-122).  Data moves inside an access use
 * memcpy rather than constant-time cmov, so this is an optimistic (fast)
 * baseline for the reference's CPU path.
 *
 * It is an independent second implementation of the handler: tests check it
 * bit-for-bit against the seqmodel (gvs_oracle.c) on seeded streams, and
 * bench.py times it as the CPU baseline (BASELINE.json config 1).
 */
#include <stdlib.h>
#include <string.h>

#include "gvs_oracle.h"

#define Z 4

/* ------------------------------------------------------------------ ORAM */

typedef struct oram {
  uint64_t n;       /* logical blocks */
  uint32_t bsz;     /* block bytes */
  uint32_t L;       /* leaves = 1 << L */
  uint64_t leaves, nodes;
  uint8_t *data;    /* nodes * Z * bsz */
  uint64_t *meta;   /* nodes * Z: 0 = empty, else index + 1 */
  uint32_t *leaf;   /* nodes * Z */
  uint32_t scap, scount;
  uint8_t *sdata;
  uint64_t *smeta;
  uint32_t *sleaf;
  uint32_t *pm_plain; /* position map when small */
  struct oram *pm;    /* recursive position map */
  uint32_t pm_ent;    /* leaves per position-map block */
  uint64_t *rng;
  /* per-access scratch: path (L+1)*Z slots + stash */
  uint8_t *wdata;
  uint64_t *wmeta;
  uint32_t *wleaf;
  uint32_t wcap;
  uint64_t accesses;
} oram;

static uint64_t sm64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static void oram_free(oram *o) {
  if (!o) return;
  free(o->data);
  free(o->meta);
  free(o->leaf);
  free(o->sdata);
  free(o->smeta);
  free(o->sleaf);
  free(o->pm_plain);
  free(o->wdata);
  free(o->wmeta);
  free(o->wleaf);
  oram_free(o->pm);
  free(o);
}

static oram *oram_new(uint64_t n, uint32_t bsz, uint64_t *rng) {
  oram *o = (oram *)calloc(1, sizeof *o);
  if (!o) return NULL;
  o->n = n;
  o->bsz = bsz;
  o->rng = rng;
  uint64_t need = (n + 1) / 2; /* leaves ~ N/2: 4N slots, 25% utilisation */
  o->L = 0;
  while ((1ull << o->L) < need) o->L++;
  o->leaves = 1ull << o->L;
  o->nodes = 2 * o->leaves - 1;
  o->data = (uint8_t *)calloc(o->nodes * Z, bsz);
  o->meta = (uint64_t *)calloc(o->nodes * Z, sizeof(uint64_t));
  o->leaf = (uint32_t *)calloc(o->nodes * Z, sizeof(uint32_t));
  o->scap = 256;
  o->sdata = (uint8_t *)calloc(o->scap, bsz);
  o->smeta = (uint64_t *)calloc(o->scap, sizeof(uint64_t));
  o->sleaf = (uint32_t *)calloc(o->scap, sizeof(uint32_t));
  o->wcap = (o->L + 1) * Z + o->scap + 1;
  o->wdata = (uint8_t *)calloc(o->wcap, bsz);
  o->wmeta = (uint64_t *)calloc(o->wcap, sizeof(uint64_t));
  o->wleaf = (uint32_t *)calloc(o->wcap, sizeof(uint32_t));
  if (!o->data || !o->meta || !o->leaf || !o->sdata || !o->smeta || !o->sleaf || !o->wdata ||
      !o->wmeta || !o->wleaf) {
    oram_free(o);
    return NULL;
  }
  o->pm_ent = 1024 / 4; /* position map blocks are 1 KiB of u32 leaves */
  if (n <= 4096) {
    o->pm_plain = (uint32_t *)calloc(n, sizeof(uint32_t));
    if (!o->pm_plain) {
      oram_free(o);
      return NULL;
    }
  } else {
    o->pm = oram_new((n + o->pm_ent - 1) / o->pm_ent, 1024, rng);
    if (!o->pm) {
      oram_free(o);
      return NULL;
    }
  }
  return o;
}

typedef void (*access_fn)(void *ctx, uint8_t *block);
static void oram_access(oram *o, uint64_t idx, access_fn fn, void *ctx);

typedef struct {
  uint32_t off, newleaf, oldleaf;
} pm_ctx;
static void pm_fn(void *c, uint8_t *blk) {
  pm_ctx *p = (pm_ctx *)c;
  uint32_t *e = (uint32_t *)blk;
  p->oldleaf = e[p->off];
  e[p->off] = p->newleaf;
}

/* position-map entries hold leaf + 1; 0 = never assigned (the block has
 * never been written), which reads a uniformly random path */
static uint32_t pm_swap(oram *o, uint64_t idx, uint32_t newleaf) {
  uint32_t old;
  if (o->pm_plain) {
    old = o->pm_plain[idx];
    o->pm_plain[idx] = newleaf + 1;
  } else {
    pm_ctx c = {(uint32_t)(idx % o->pm_ent), newleaf + 1, 0};
    oram_access(o->pm, idx / o->pm_ent, pm_fn, &c);
    old = c.oldleaf;
  }
  return old ? old - 1 : (uint32_t)(sm64(o->rng) % o->leaves);
}

static inline uint64_t path_node(const oram *o, uint32_t leaf, uint32_t depth) {
  /* node at `depth` (0 = root) on the path to `leaf`, heap numbering */
  uint64_t x = o->leaves - 1 + leaf;
  for (uint32_t d = o->L; d > depth; --d) x = (x - 1) / 2;
  return x;
}

/* Path ORAM access: remap, read path + stash, apply fn, greedy evict. */
static void oram_access(oram *o, uint64_t idx, access_fn fn, void *ctx) {
  const uint32_t bsz = o->bsz;
  const uint32_t newleaf = (uint32_t)(sm64(o->rng) % o->leaves);
  const uint32_t old = pm_swap(o, idx, newleaf) % (uint32_t)o->leaves;
  o->accesses++;
  /* gather path (root..leaf) and stash into the work set */
  uint32_t w = 0;
  uint64_t nodes[64];
  /* the whole path is read, empty slots included (an oblivious ORAM reads and
     writes every bucket of the path whatever it holds) */
  for (uint32_t d = 0; d <= o->L; ++d) {
    nodes[d] = path_node(o, old, d);
    const uint64_t s = nodes[d] * Z;
    memcpy(o->wdata + (size_t)w * bsz, o->data + s * bsz, (size_t)Z * bsz);
    for (uint32_t z = 0; z < Z; ++z) {
      o->wmeta[w + z] = o->meta[s + z];
      o->wleaf[w + z] = o->leaf[s + z];
    }
    w += Z;
  }
  for (uint32_t i = 0; i < o->scount; ++i) {
    memcpy(o->wdata + (size_t)w * bsz, o->sdata + (size_t)i * bsz, bsz);
    o->wmeta[w] = o->smeta[i];
    o->wleaf[w] = o->sleaf[i];
    ++w;
  }
  /* locate (or create) the target block */
  uint32_t t = w;
  for (uint32_t i = 0; i < w; ++i)
    if (o->wmeta[i] == idx + 1) t = i;
  /* empty slots are never placed back */
  if (t == w) {
    memset(o->wdata + (size_t)w * bsz, 0, bsz);
    o->wmeta[w] = idx + 1;
    ++w;
  }
  o->wleaf[t] = newleaf;
  fn(ctx, o->wdata + (size_t)t * bsz);
  /* greedy eviction from the leaf up */
  uint8_t placed[1024];
  for (uint32_t i = 0; i < w; ++i) placed[i] = o->wmeta[i] == 0;
  for (int d = (int)o->L; d >= 0; --d) {
    uint32_t cnt = 0;
    const uint32_t shift = o->L - (uint32_t)d;
    const uint64_t base = nodes[d] * Z;
    for (uint32_t i = 0; i < w && cnt < Z; ++i) {
      if (placed[i] || (o->wleaf[i] >> shift) != (old >> shift)) continue;
      memcpy(o->data + (base + cnt) * bsz, o->wdata + (size_t)i * bsz, bsz);
      o->meta[base + cnt] = o->wmeta[i];
      o->leaf[base + cnt] = o->wleaf[i];
      placed[i] = 1;
      ++cnt;
    }
    for (; cnt < Z; ++cnt) {
      memset(o->data + (base + cnt) * bsz, 0, bsz);
      o->meta[base + cnt] = 0;
    }
  }
  uint32_t sc = 0;
  for (uint32_t i = 0; i < w; ++i) {
    if (placed[i]) continue;
    if (sc >= o->scap) abort(); /* stash overflow: negligible at Z = 4 */
    memcpy(o->sdata + (size_t)sc * bsz, o->wdata + (size_t)i * bsz, bsz);
    o->smeta[sc] = o->wmeta[i];
    o->sleaf[sc] = o->wleaf[i];
    ++sc;
  }
  o->scount = sc;
}

/* ------------------------------------------------------------- the model */

typedef struct dir_entry { /* 16 B per mailbox row: recipient PRF, 0 = free */
  uint64_t h_hi, h_lo;
} dir_entry;

struct gvp_model {
  gvs_config cfg;
  uint64_t N, R;
  uint32_t Q, Sr, B, logQ;
  uint8_t prp_key[16], hash_key[16];
  uint64_t count, ctr, n_mailboxes, head, tail, ring_size;
  uint32_t *ring;
  uint64_t rng;
  oram *msg, *rows, *dir;
};

static int zero(const uint8_t *p, size_t n) {
  uint8_t a = 0;
  for (size_t i = 0; i < n; ++i) a |= p[i];
  return a == 0;
}

gvp_model *gvp_create(const gvs_config *cfg) {
  gvp_model *m = (gvp_model *)calloc(1, sizeof *m);
  if (!m) return NULL;
  m->cfg = *cfg;
  m->N = cfg->msg_capacity;
  m->Q = cfg->mailbox_partitions;
  m->Sr = cfg->mailbox_partition_slots;
  m->R = (uint64_t)m->Q * m->Sr;
  m->B = cfg->max_batch;
  while ((1u << m->logQ) < m->Q) m->logQ++;
  memcpy(m->prp_key, cfg->secret_key, 16);
  memcpy(m->hash_key, cfg->secret_key + 16, 16);
  m->ring_size = m->N + m->B;
  m->ring = (uint32_t *)malloc(m->ring_size * sizeof(uint32_t));
  m->rng = 0x70617468u;
  m->msg = oram_new(m->N, 1024, &m->rng);
  m->rows = oram_new(m->R, 1024, &m->rng);
  m->dir = oram_new(m->Q, m->Sr * (uint32_t)sizeof(dir_entry), &m->rng);
  if (!m->ring || !m->msg || !m->rows || !m->dir) {
    gvp_destroy(m);
    return NULL;
  }
  for (uint64_t s = 0; s < m->N; ++s) m->ring[s] = (uint32_t)s;
  m->tail = m->N;
  return m;
}

void gvp_destroy(gvp_model *m) {
  if (!m) return;
  free(m->ring);
  oram_free(m->msg);
  oram_free(m->rows);
  oram_free(m->dir);
  free(m);
}

/* ---- directory access: lookup, lookup-or-allocate, free ---- */
typedef struct {
  uint64_t hi, lo;
  int op;        /* 0 lookup, 1 lookup or allocate, 2 free row `row`, 3 none (dummy) */
  uint32_t Sr;
  int32_t row;   /* out (op 0/1), in (op 2) */
  int fresh;     /* op 1: the row was allocated by this access */
} dir_ctx;
static void dir_fn(void *c, uint8_t *blk) {
  dir_ctx *x = (dir_ctx *)c;
  dir_entry *e = (dir_entry *)blk;
  if (x->op == 3) return;
  if (x->op == 2) {
    if (x->row >= 0) memset(&e[x->row], 0, sizeof(dir_entry));
    return;
  }
  int32_t found = -1, first_free = -1;
  for (uint32_t i = 0; i < x->Sr; ++i) {
    const int used = (e[i].h_hi | e[i].h_lo) != 0;
    if (used && e[i].h_hi == x->hi && e[i].h_lo == x->lo) found = (int32_t)i;
    if (!used && first_free < 0) first_free = (int32_t)i;
  }
  x->row = found;
  x->fresh = 0;
  if (found < 0 && x->op == 1 && first_free >= 0) {
    e[first_free].h_hi = x->hi;
    e[first_free].h_lo = x->lo;
    x->row = first_free;
    x->fresh = 1;
  }
}
static uint32_t part_of(const gvp_model *m, uint64_t hi) {
  return m->logQ ? (uint32_t)(hi >> (64 - m->logQ)) : 0u;
}
static void dir_do(gvp_model *m, uint32_t q, dir_ctx *c) {
  c->Sr = m->Sr;
  if (c->op == 3) q = (uint32_t)(sm64(&m->rng) % m->Q);
  oram_access(m->dir, q, dir_fn, c);
}

/* ---- mailbox row access ---- */
typedef struct {
  int op;        /* 0 read, 1 append-if-room, 2 pop head, 3 remove id, 4 fresh + append */
  uint8_t x[32], id[16];
  uint32_t len_before, len_after;
  int done;      /* append: there was room; pop: popped; remove: found */
  uint8_t head[16];
} row_ctx;
static void row_fn(void *c, uint8_t *blk) {
  row_ctx *x = (row_ctx *)c;
  uint8_t *ids = blk + 32;
  if (x->op == 4) memset(blk, 0, 1024), memcpy(blk, x->x, 32);
  uint32_t len = 0;
  while (len < GVS_MAILBOX_SLOTS && !zero(ids + 16 * len, 16)) ++len;
  x->len_before = len;
  memcpy(x->head, ids, 16);
  x->done = 0;
  if ((x->op == 1 || x->op == 4) && len < GVS_MAILBOX_SLOTS) {
    memcpy(ids + 16 * len, x->id, 16);
    ++len;
    x->done = 1;
  } else if (x->op == 2 && len) {
    memmove(ids, ids + 16, 16 * (GVS_MAILBOX_SLOTS - 1));
    memset(ids + 16 * (GVS_MAILBOX_SLOTS - 1), 0, 16);
    --len;
    x->done = 1;
  } else if (x->op == 3) {
    for (uint32_t i = 0; i < len; ++i)
      if (memcmp(ids + 16 * i, x->id, 16) == 0) {
        memmove(ids + 16 * i, ids + 16 * (i + 1), 16 * (GVS_MAILBOX_SLOTS - 1 - i));
        memset(ids + 16 * (GVS_MAILBOX_SLOTS - 1), 0, 16);
        --len;
        x->done = 1;
        break;
      }
  }
  if (len == 0 && x->op != 0) memset(blk, 0, 1024); /* an emptied row is cleared */
  x->len_after = len;
}
static void row_do(gvp_model *m, uint32_t q, int32_t row, row_ctx *c) {
  uint64_t idx;
  if (row >= 0) idx = (uint64_t)q * m->Sr + (uint32_t)row;
  else {
    idx = sm64(&m->rng) % m->R; /* dummy access: same cost */
    c->op = 0;
  }
  oram_access(m->rows, idx, row_fn, c);
}

/* ---- message access: read, or check-and-modify for by-id ops ---- */
typedef struct {
  int op;                 /* 0 read, 1 write rec, 2 clear, 3 by-id op of req */
  const gvs_request *rq;
  const uint8_t *want_id; /* op 0/2: expected id (may be NULL) */
  gvs_record rec, out;
  uint32_t status;
} msg_ctx;
static void msg_fn(void *c, uint8_t *blk) {
  msg_ctx *x = (msg_ctx *)c;
  gvs_record *r = (gvs_record *)blk;
  memcpy(&x->out, r, sizeof *r);
  if (x->op == 1) memcpy(r, &x->rec, sizeof *r);
  else if (x->op == 2) memset(r, 0, sizeof *r);
  else if (x->op == 3) {
    const gvs_request *q = x->rq;
    const uint32_t t = q->request_type;
    const int exists = memcmp(r->msg_id, q->msg_id, 16) == 0 && !zero(r->msg_id, 16);
    const int auth = exists && (memcmp(q->auth_identity, r->sender, 32) == 0 ||
                                memcmp(q->auth_identity, r->recipient, 32) == 0);
    x->status = GVS_STATUS_SUCCESS;
    if (!auth) x->status = GVS_STATUS_NOT_FOUND;
    else if (t != GVS_REQUEST_READ && memcmp(q->recipient, r->recipient, 32) != 0)
      x->status = GVS_STATUS_INVALID_RECIPIENT;
    if (x->status == GVS_STATUS_SUCCESS && t == GVS_REQUEST_UPDATE) {
      memcpy(r->payload, q->payload, GVS_PAYLOAD_BYTES);
      r->timestamp = q->timestamp;
      memcpy(&x->out, r, sizeof *r);
    } else if (x->status == GVS_STATUS_SUCCESS && t == GVS_REQUEST_DELETE) {
      memset(r, 0, sizeof *r);
    }
  }
}
static void msg_do(gvp_model *m, int64_t slot, msg_ctx *c) {
  uint64_t idx = slot >= 0 ? (uint64_t)slot : sm64(&m->rng) % m->N;
  if (slot < 0) c->op = 0;
  oram_access(m->msg, idx, msg_fn, c);
}

static void fail(gvs_response *o, uint32_t st, uint64_t ts) {
  memset(o, 0, sizeof *o);
  o->record.timestamp = ts;
  o->status_code = st;
}
static void ok(gvs_response *o, const gvs_record *r) {
  memset(o, 0, sizeof *o);
  o->record = *r;
  o->status_code = GVS_STATUS_SUCCESS;
}
static int hard(const gvs_request *rq) {
  uint32_t t = rq->request_type;
  return t < 1 || t > 4 || zero(rq->auth_identity, 32) || (t == 3 && zero(rq->msg_id, 16));
}
static void free_slot(gvp_model *m, uint32_t slot) {
  m->ring[m->tail % m->ring_size] = slot;
  m->tail++;
  m->count--;
}

/* Every request: four ORAM accesses (directory, row, message, directory),
 * real or dummy.  Order differs between creates/next ops and by-id ops. */

static void g_create(gvp_model *m, const gvs_request *rq, gvs_response *o) {
  const int bad = zero(rq->recipient, 32);
  uint64_t hi = 0, lo = 0;
  gvo_recipient_hash(m->hash_key, rq->recipient, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  const int full = m->count >= m->N;
  dir_ctx d = {hi, lo, (bad || full) ? 3 : 1, 0, -1, 0};
  dir_do(m, q, &d);
  row_ctx r;
  memset(&r, 0, sizeof r);
  gvs_record rec;
  memset(&rec, 0, sizeof rec);
  const uint32_t slot = m->ring[m->head % m->ring_size];  /* candidate */
  gvo_id_encode(m->prp_key, slot, m->ctr, rec.msg_id);
  r.op = d.fresh ? 4 : 1;
  memcpy(r.x, rq->recipient, 32);
  memcpy(r.id, rec.msg_id, 16);
  row_do(m, q, (bad || full) ? -1 : d.row, &r);
  uint32_t status = GVS_STATUS_SUCCESS;
  if (bad) status = GVS_STATUS_INVALID_RECIPIENT;
  else if (full) status = GVS_STATUS_TOO_MANY_MESSAGES;
  else if (d.row < 0) status = GVS_STATUS_TOO_MANY_RECIPIENTS;
  else if (!r.done) status = GVS_STATUS_TOO_MANY_MESSAGES_FOR_RECIPIENT;
  msg_ctx mc;
  memset(&mc, 0, sizeof mc);
  if (status == GVS_STATUS_SUCCESS) {
    m->head++;
    m->ctr++;
    memcpy(rec.sender, rq->auth_identity, 32);
    memcpy(rec.recipient, rq->recipient, 32);
    rec.timestamp = rq->timestamp;
    memcpy(rec.payload, rq->payload, GVS_PAYLOAD_BYTES);
    mc.op = 1;
    mc.rec = rec;
    msg_do(m, slot, &mc);
    m->count++;
    if (d.fresh) m->n_mailboxes++;
    ok(o, &rec);
  } else {
    msg_do(m, -1, &mc);
    fail(o, status, rq->timestamp);
  }
  dir_ctx d2 = {0, 0, 3, 0, -1, 0};
  dir_do(m, 0, &d2);
}

static void g_next(gvp_model *m, const gvs_request *rq, gvs_response *o, int del) {
  uint64_t hi, lo;
  gvo_recipient_hash(m->hash_key, rq->auth_identity, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  dir_ctx d = {hi, lo, 0, 0, -1, 0};
  dir_do(m, q, &d);
  row_ctx r;
  memset(&r, 0, sizeof r);
  r.op = del ? 2 : 0;
  row_do(m, q, d.row, &r);
  const int have = d.row >= 0 && r.len_before > 0;
  msg_ctx mc;
  memset(&mc, 0, sizeof mc);
  int64_t slot = -1;
  if (have) {
    uint32_t s;
    uint64_t ctr;
    gvo_id_decode(m->prp_key, r.head, m->N, &s, &ctr);
    slot = s;
    mc.op = del ? 2 : 0;
  }
  msg_do(m, slot, &mc);
  dir_ctx d2 = {hi, lo, (have && del && r.len_after == 0) ? 2 : 3, 0, d.row, 0};
  dir_do(m, q, &d2);
  if (!have) {
    fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
    return;
  }
  ok(o, &mc.out);
  if (del) {
    free_slot(m, (uint32_t)slot);
    if (r.len_after == 0) m->n_mailboxes--;
  }
}

static void g_byid(gvp_model *m, const gvs_request *rq, gvs_response *o) {
  uint32_t slot = 0;
  uint64_t ctr;
  const int valid = gvo_id_decode(m->prp_key, rq->msg_id, m->N, &slot, &ctr);
  msg_ctx mc;
  memset(&mc, 0, sizeof mc);
  mc.op = 3;
  mc.rq = rq;
  mc.status = GVS_STATUS_NOT_FOUND;
  msg_do(m, valid ? (int64_t)slot : -1, &mc);
  if (!valid) mc.status = GVS_STATUS_NOT_FOUND;
  const int del = mc.status == GVS_STATUS_SUCCESS && rq->request_type == GVS_REQUEST_DELETE;
  uint64_t hi, lo;
  gvo_recipient_hash(m->hash_key, rq->recipient, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  dir_ctx d = {hi, lo, del ? 0 : 3, 0, -1, 0};
  dir_do(m, q, &d);
  row_ctx r;
  memset(&r, 0, sizeof r);
  r.op = 3;
  memcpy(r.id, rq->msg_id, 16);
  row_do(m, q, del ? d.row : -1, &r);
  dir_ctx d2 = {hi, lo, (del && r.len_after == 0) ? 2 : 3, 0, d.row, 0};
  dir_do(m, q, &d2);
  if (mc.status != GVS_STATUS_SUCCESS) {
    fail(o, mc.status, rq->timestamp);
    return;
  }
  ok(o, &mc.out);
  if (del) {
    free_slot(m, slot);
    if (r.len_after == 0) m->n_mailboxes--;
  }
}

void gvp_apply_one(gvp_model *m, const gvs_request *rq, gvs_response *o) {
  if (hard(rq)) { /* fail fast at the gRPC level: no store access */
    memset(o, 0, sizeof *o);
    return;
  }
  switch (rq->request_type) {
    case GVS_REQUEST_CREATE: g_create(m, rq, o); break;
    case GVS_REQUEST_READ:
      if (zero(rq->msg_id, 16)) g_next(m, rq, o, 0);
      else g_byid(m, rq, o);
      break;
    case GVS_REQUEST_UPDATE: g_byid(m, rq, o); break;
    default:
      if (zero(rq->msg_id, 16)) g_next(m, rq, o, 1);
      else g_byid(m, rq, o);
      break;
  }
}

static int cls(const gvs_request *rq) {
  if (hard(rq)) return 2;
  if (rq->request_type == GVS_REQUEST_CREATE) return 1;
  if ((rq->request_type == 2 || rq->request_type == 4) && zero(rq->msg_id, 16)) return 0;
  return 2;
}

int gvp_process_batch(gvp_model *m, const gvs_request *reqs, uint32_t n, gvs_response *out) {
  if (n > m->B) return GVS_ERR_INVALID_ARG;
  for (int c = 0; c < 3; ++c)
    for (uint32_t i = 0; i < n; ++i)
      if (cls(&reqs[i]) == c) gvp_apply_one(m, &reqs[i], &out[i]);
  return GVS_OK;
}

uint64_t gvp_messages(const gvp_model *m) { return m->count; }
uint64_t gvp_mailboxes(const gvp_model *m) { return m->n_mailboxes; }
uint64_t gvp_oram_accesses(const gvp_model *m) {
  return m->msg->accesses + m->rows->accesses + m->dir->accesses;
}
