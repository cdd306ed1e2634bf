/* gvs_kv.c — sequential CPU restatement of the block store (gvs_oram_*) and
 * the key-value map (gvs_omap_*), TEST INFRASTRUCTURE ONLY: tests/ use it as
 * the checker of the HIP path; the product never links it.
 *
 * The surfaces follow mc-oblivious-traits (absent from the reference and from
 * Cargo.lock, version unpinned; SURVEY.md §8(b) restates the signatures):
 *   ORAM<1024>::access(index, f: FnOnce(&mut A64Bytes<1024>))     -> block store
 *   ObliviousHashMap<16, 1024>::access_and_insert / read / remove -> map
 * Parity against the reference is therefore unpinned; these
 * functions pin the GPU path to the sequential semantics of those traits.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gvstore.h"

/* ------------------------------------------------------------ block store */

typedef struct gvo_oram {
  uint64_t n;
  uint8_t *blocks; /* n x 1024, zero initially */
} gvo_oram;

gvo_oram *gvo_oram_create(uint64_t capacity) {
  gvo_oram *o = (gvo_oram *)calloc(1, sizeof *o);
  if (!o) return NULL;
  o->n = capacity;
  o->blocks = (uint8_t *)calloc(capacity, 1024);
  if (!o->blocks) {
    free(o);
    return NULL;
  }
  return o;
}

void gvo_oram_destroy(gvo_oram *o) {
  if (!o) return;
  free(o->blocks);
  free(o);
}

/* Apply n ops in order; out[i] = the block op i saw (before a write).  An
 * invalid op (index >= capacity, op > 1) rejects the whole batch: returns -1,
 * nothing applied, as gvs_oram_access_batch (GVS_ERR_INVALID_ARG). */
int gvo_oram_access_batch(gvo_oram *o, const gvs_block_op *ops, uint32_t n, uint8_t *out) {
  for (uint32_t i = 0; i < n; ++i)
    if (ops[i].index >= o->n || ops[i].op > GVS_ORAM_WRITE) return -1;
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t *b = o->blocks + ops[i].index * 1024;
    memcpy(out + (uint64_t)i * 1024, b, 1024);
    if (ops[i].op == GVS_ORAM_WRITE) memcpy(b, ops[i].data, 1024);
  }
  return 0;
}

void gvo_oram_read_all(const gvo_oram *o, uint8_t *dst) { memcpy(dst, o->blocks, o->n * 1024); }

/* ------------------------------------------------------------ key-value map
 *
 * ObliviousHashMap<16, 1024> semantics, batched (include/gvstore.h): ops in
 * submission order per key; [D] new keys of a batch are admitted into their
 * partition's rows that are free when the batch starts, in keyed-hash order
 * (hash hi, then hash lo without its low 20 bits), the r-th admitted key
 * taking the r-th free row; the others overflow.  Keys hash with SipHash-2-4
 * under secret_key[16..32) of key || 0x03 (hi) and key || 0x04 (lo); the
 * partition is the top log2(W) bits of hi.  Table layout as the engine's:
 * S = N / 4096 rows per partition clamped to [256, 4096], W = N / S. */

uint64_t gvo_siphash24(uint64_t k0, uint64_t k1, const uint8_t *m, size_t len);

static uint64_t kv_ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

void gvo_omap_hash(const uint8_t secret[32], const uint8_t key[16], uint64_t *hi, uint64_t *lo) {
  uint8_t msg[17];
  memcpy(msg, key, 16);
  msg[16] = 3;
  *hi = gvo_siphash24(kv_ld64(secret + 16), kv_ld64(secret + 24), msg, 17);
  msg[16] = 4;
  *lo = gvo_siphash24(kv_ld64(secret + 16), kv_ld64(secret + 24), msg, 17);
}

typedef struct gvo_omap {
  uint64_t n;
  uint32_t S, W, logW;
  uint8_t secret[32];
  uint8_t *keys; /* n x 16, zero = free */
  uint8_t *vals; /* n x 1024 */
} gvo_omap;

gvo_omap *gvo_omap_create(uint64_t capacity, const uint8_t secret[32]) {
  gvo_omap *m = (gvo_omap *)calloc(1, sizeof *m);
  if (!m) return NULL;
  uint64_t S = capacity / 4096;
  if (S < 256) S = 256;
  if (S > 4096) S = 4096;
  if (S > capacity) S = capacity;
  m->n = capacity;
  m->S = (uint32_t)S;
  m->W = (uint32_t)(capacity / S);
  while ((1u << m->logW) < m->W) ++m->logW;
  memcpy(m->secret, secret, 32);
  m->keys = (uint8_t *)calloc(capacity, 16);
  m->vals = (uint8_t *)calloc(capacity, 1024);
  if (!m->keys || !m->vals) {
    free(m->keys);
    free(m->vals);
    free(m);
    return NULL;
  }
  return m;
}

void gvo_omap_destroy(gvo_omap *m) {
  if (!m) return;
  free(m->keys);
  free(m->vals);
  free(m);
}

typedef struct kv_group {
  uint8_t key[16];
  uint64_t hi, lo; /* lo without its low 20 bits */
  uint32_t q;
  int64_t row;     /* physical row, -1: none */
  int exists, needs;
  uint8_t *value;  /* 1024 B working value */
} kv_group;

static int kv_group_cmp(const void *a, const void *b) {
  const kv_group *x = (const kv_group *)a, *y = (const kv_group *)b;
  if (x->hi != y->hi) return x->hi < y->hi ? -1 : 1;
  if (x->lo != y->lo) return x->lo < y->lo ? -1 : 1;
  return memcmp(x->key, y->key, 16);
}

static int key_zero(const uint8_t *k) {
  for (int i = 0; i < 16; ++i)
    if (k[i]) return 0;
  return 1;
}

/* returns -1 (nothing applied) if an op code is unknown */
int gvo_omap_access_batch(gvo_omap *m, const gvs_omap_op *ops, uint32_t n, gvs_omap_result *out) {
  for (uint32_t i = 0; i < n; ++i)
    if (ops[i].op > GVS_OMAP_REMOVE) return -1;
  kv_group *g = (kv_group *)calloc(n ? n : 1, sizeof *g);
  kv_group *t = (kv_group *)calloc(n ? n : 1, sizeof *t);
  uint32_t *gi = (uint32_t *)calloc(n ? n : 1, sizeof *gi);
  uint8_t *vals = (uint8_t *)calloc(n ? n : 1, 1024);
  uint32_t ng = 0, nt = 0;
  /* every valid op's key with its hash, sorted by hash: runs are the
   * distinct keys in admission order (t[].row carries the op index) */
  for (uint32_t i = 0; i < n; ++i) {
    if (key_zero(ops[i].key)) continue;
    kv_group *x = &t[nt++];
    memcpy(x->key, ops[i].key, 16);
    uint64_t hi, lo;
    gvo_omap_hash(m->secret, ops[i].key, &hi, &lo);
    x->hi = hi;
    x->lo = lo & ~(uint64_t)0xFFFFF;
    x->q = m->logW ? (uint32_t)(hi >> (64 - m->logW)) : 0u;
    x->row = i;
  }
  qsort(t, nt, sizeof *t, kv_group_cmp);
  for (uint32_t u = 0; u < nt; ++u) {
    if (u == 0 || kv_group_cmp(&t[u - 1], &t[u]) != 0) {
      g[ng] = t[u];
      g[ng].row = -1;
      g[ng].needs = 0;
      ++ng;
    }
    const uint32_t i = (uint32_t)t[u].row;
    gi[i] = ng - 1;
    if (ops[i].op == GVS_OMAP_WRITE || ops[i].op == GVS_OMAP_INSERT) g[ng - 1].needs = 1;
  }
  for (uint32_t k = 0; k < ng; ++k) {
    g[k].value = vals + (uint64_t)k * 1024;
    const uint64_t base = (uint64_t)g[k].q * m->S;
    for (uint32_t j = 0; j < m->S; ++j)
      if (memcmp(m->keys + (base + j) * 16, g[k].key, 16) == 0) {
        g[k].row = (int64_t)(base + j);
        g[k].exists = 1;
        memcpy(g[k].value, m->vals + (base + j) * 1024, 1024);
        break;
      }
    g[k].needs = g[k].needs && !g[k].exists;
  }
  /* admission per partition, in hash order, into the free rows in row order */
  uint32_t *cnt = (uint32_t *)calloc(m->W, sizeof *cnt);
  for (uint32_t k = 0; k < ng; ++k) {
    if (!g[k].needs) continue;
    const uint64_t base = (uint64_t)g[k].q * m->S;
    const uint32_t rank = cnt[g[k].q]++;
    uint32_t f = 0;
    for (uint32_t j = 0; j < m->S; ++j)
      if (key_zero(m->keys + (base + j) * 16)) {
        if (f == rank) {
          g[k].row = (int64_t)(base + j);
          break;
        }
        ++f;
      }
  }
  free(cnt);
  /* the ops, in order */
  for (uint32_t i = 0; i < n; ++i) {
    gvs_omap_result *r = &out[i];
    memset(r, 0, sizeof *r);
    if (key_zero(ops[i].key)) {
      r->status = GVS_OMAP_INVALID_KEY;
      continue;
    }
    kv_group *G = &g[gi[i]];
    const uint32_t op = ops[i].op;
    if (G->exists) {
      r->status = GVS_OMAP_FOUND;
      memcpy(r->value, G->value, 1024);
      if (op == GVS_OMAP_WRITE) memcpy(G->value, ops[i].value, 1024);
      if (op == GVS_OMAP_REMOVE) {
        G->exists = 0;
        memset(G->value, 0, 1024);
      }
    } else if (op == GVS_OMAP_READ || op == GVS_OMAP_REMOVE) {
      r->status = GVS_OMAP_NOT_FOUND;
    } else if (G->row < 0) {
      r->status = GVS_OMAP_OVERFLOW;
    } else {
      r->status = GVS_OMAP_NOT_FOUND;
      if (op == GVS_OMAP_INSERT) memcpy(r->value, ops[i].value, 1024);
      memcpy(G->value, ops[i].value, 1024);
      G->exists = 1;
    }
  }
  /* commit */
  for (uint32_t k = 0; k < ng; ++k) {
    if (g[k].row < 0) continue;
    uint8_t *key = m->keys + (uint64_t)g[k].row * 16, *val = m->vals + (uint64_t)g[k].row * 1024;
    if (g[k].exists) {
      memcpy(key, g[k].key, 16);
      memcpy(val, g[k].value, 1024);
    } else {
      memset(key, 0, 16);
      memset(val, 0, 1024);
    }
  }
  free(g);
  free(t);
  free(gi);
  free(vals);
  return 0;
}

uint64_t gvo_omap_size(const gvo_omap *m) {
  uint64_t c = 0;
  for (uint64_t r = 0; r < m->n; ++r) c += !key_zero(m->keys + r * 16);
  return c;
}
