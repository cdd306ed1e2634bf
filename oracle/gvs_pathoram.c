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
 *   messages  : CuckooHashTable msg_id (16 B) -> record (1 KiB)
 *   mailboxes : CuckooHashTable recipient PRF (16 B) -> row (recipient + 62 ids)
 *   occupancy : ORAM of ceil(Q / 256) blocks of u32: recipients per mailbox
 *               partition (the batched engine's capacity rule)
 *
 * A CuckooHashTable (mc-oblivious's design, restated: BASELINE.json config 1
 * "PathORAM + CuckooHashTable") is two Path ORAMs of buckets; a key has one
 * bucket in each, chosen by keyed SipHash, and every access reads and writes
 * both (two ORAM accesses, the second nested in the first so that both
 * buckets are modified together).  An insert into two full buckets displaces
 * a random item, which is re-placed by further single-bucket accesses (never
 * seen at the 50 % load used here).
 *
 * Every request costs exactly six top-level ORAM accesses (occupancy, two
 * per cuckoo access to the mailbox and the message tables, occupancy), real
 * or dummy, so READ / UPDATE / DELETE are indistinguishable by access count
 * (grapevine.proto:120-122).  Inside an access every block move is an
 * aligned cmov over every stash and branch slot (mc-oblivious's semantics,
 * README.md:49-50): the block is selected out of all slots and written back
 * into all of them under masks, and eviction is a Circuit-ORAM style single
 * pass with one held block (cmov over every slot of every level), along the
 * accessed branch and one deterministic reverse-lexicographic path.
 *
 * It is an independent second implementation of the handler: tests check it
 * bit-for-bit against the seqmodel (gvs_oracle.c) on seeded streams, and
 * bench.py times it as the CPU baseline (BASELINE.json config 1).
 */
#define _DEFAULT_SOURCE /* MAP_ANONYMOUS, MAP_NORESERVE */
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include "gvs_oracle.h"

#define Z 4
#define STASH 32 /* stash entries, every one scanned on every access */

/* ---------------------------------------------------- aligned cmov */

/* All-ones when c, else zero: the masks below select without a branch on
 * the secret (the C restatement of mc-oblivious's aligned cmov;
 * README.md:49-50). */
static inline uint64_t mask_of(int c) { return (uint64_t)0 - (uint64_t)(c != 0); }

/* dst <- src where mask, word by word (block sizes are multiples of 8) */
static inline void cmov_block(uint8_t *dst, const uint8_t *src, size_t n, uint64_t mask) {
  uint64_t *d = (uint64_t *)dst;
  const uint64_t *s = (const uint64_t *)src;
  for (size_t i = 0; i < n / 8; ++i) d[i] = (d[i] & ~mask) | (s[i] & mask);
}
static inline uint64_t cmov_u64(uint64_t a, uint64_t b, uint64_t mask) { return (a & ~mask) | (b & mask); }

/* ------------------------------------------------------------------ ORAM */

typedef struct oram {
  uint64_t n;       /* logical blocks */
  uint32_t bsz;     /* block bytes */
  uint32_t L;       /* leaves = 1 << L */
  uint64_t leaves, nodes;
  uint8_t *data;    /* nodes * Z * bsz */
  uint64_t *meta;   /* nodes * Z: 0 = empty, else index + 1 */
  uint32_t *leaf;   /* nodes * Z */
  uint8_t *sdata;   /* STASH entries */
  uint64_t *smeta;
  uint32_t *sleaf;
  uint32_t *pm_plain; /* position map when small */
  struct oram *pm;    /* recursive position map */
  uint32_t pm_ent;    /* leaves per position-map block */
  uint64_t *rng;
  /* the checked-out branch (root .. leaf, Z slots per level) and the block
     being accessed */
  uint8_t *wdata;
  uint64_t *wmeta;
  uint32_t *wleaf;
  uint8_t *tmp, *hold;
  uint64_t evictions;  /* deterministic eviction paths taken so far */
  uint64_t accesses;
} oram;

static uint64_t sm64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

/* Zeroed tree arrays.  Large ones are anonymous mappings without swap
 * reservation: at the headline capacity (2^24 messages) a cuckoo table's tree
 * is 64 GiB of address space, of which a timed sample touches only the paths
 * it visits (bench.py c3_single_instance); malloc's overcommit check would
 * refuse the whole allocation up front. */
#define BIG_ALLOC (1ull << 30)
static void *tree_zalloc(size_t bytes) {
  if (bytes < BIG_ALLOC) return calloc(1, bytes);
  void *p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  return p == MAP_FAILED ? NULL : p;
}
static void tree_free(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < BIG_ALLOC)
    free(p);
  else
    munmap(p, bytes);
}

static void oram_free(oram *o) {
  if (!o) return;
  tree_free(o->data, o->nodes * Z * (size_t)o->bsz);
  tree_free(o->meta, o->nodes * Z * sizeof(uint64_t));
  tree_free(o->leaf, o->nodes * Z * sizeof(uint32_t));
  free(o->sdata);
  free(o->smeta);
  free(o->sleaf);
  free(o->pm_plain);
  free(o->wdata);
  free(o->wmeta);
  free(o->wleaf);
  free(o->tmp);
  free(o->hold);
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
  o->data = (uint8_t *)tree_zalloc(o->nodes * Z * (size_t)bsz);
  o->meta = (uint64_t *)tree_zalloc(o->nodes * Z * sizeof(uint64_t));
  o->leaf = (uint32_t *)tree_zalloc(o->nodes * Z * sizeof(uint32_t));
  o->sdata = (uint8_t *)calloc(STASH, bsz);
  o->smeta = (uint64_t *)calloc(STASH, sizeof(uint64_t));
  o->sleaf = (uint32_t *)calloc(STASH, sizeof(uint32_t));
  o->wdata = (uint8_t *)calloc((size_t)(o->L + 1) * Z, bsz);
  o->wmeta = (uint64_t *)calloc((size_t)(o->L + 1) * Z, sizeof(uint64_t));
  o->wleaf = (uint32_t *)calloc((size_t)(o->L + 1) * Z, sizeof(uint32_t));
  o->tmp = (uint8_t *)calloc(1, bsz);
  o->hold = (uint8_t *)calloc(1, bsz);
  if (!o->data || !o->meta || !o->leaf || !o->sdata || !o->smeta || !o->sleaf || !o->wdata ||
      !o->wmeta || !o->wleaf || !o->tmp || !o->hold) {
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
  return ((o->leaves - 1 + leaf + 1) >> (o->L - depth)) - 1;
}

static void branch_io(oram *o, uint32_t leaf, int out) {
  const uint32_t bsz = o->bsz;
  for (uint32_t d = 0; d <= o->L; ++d) {
    const uint64_t s = path_node(o, leaf, d) * Z;
    uint8_t *t = o->data + s * bsz, *w = o->wdata + (size_t)d * Z * bsz;
    memcpy(out ? t : w, out ? w : t, (size_t)Z * bsz);
    memcpy(out ? o->meta + s : o->wmeta + d * Z, out ? o->wmeta + d * Z : o->meta + s, Z * sizeof(uint64_t));
    memcpy(out ? o->leaf + s : o->wleaf + d * Z, out ? o->wleaf + d * Z : o->leaf + s, Z * sizeof(uint32_t));
  }
}

/* deepest level (0 = root .. L) of branch `b` that a block of leaf `lf`
 * may live at; -1 for an empty slot */
static inline int32_t deepest_level(const oram *o, uint64_t meta, uint32_t lf, uint32_t b) {
  const uint32_t x = lf ^ b;
  const int32_t h = x ? 31 - __builtin_clz(x) : -1; /* highest set bit of x (lzcnt) */
  const int32_t d = (int32_t)o->L - h - 1;
  return meta ? d : -1;
}

/* Circuit-ORAM style single-pass eviction of the checked-out branch `b`
 * (Wang, Chan, Shi, CCS 2015: PrepareDeepest, PrepareTarget, EvictOnce):
 * the metadata passes choose at most one block to move down per level, then
 * one pass from the stash to the leaf carries it ("hold") with aligned cmov
 * over every slot of every level.  Level -1 is the stash.  The work done is
 * the same whatever the slots hold. */
static void evict_branch(oram *o, uint32_t b) {
  const uint32_t L = o->L, bsz = o->bsz;
  int32_t deepest[66], target[66]; /* index level + 1 */
  /* PrepareDeepest */
  int32_t src = -2, goal = -1;
  {
    int32_t g = -1;
    for (uint32_t s = 0; s < STASH; ++s) {
      const int32_t d = deepest_level(o, o->smeta[s], o->sleaf[s], b);
      g = d > g ? d : g;
    }
    src = g >= 0 ? -1 : -2;
    goal = g;
  }
  deepest[0] = -2;
  for (uint32_t i = 0; i <= L; ++i) {
    deepest[i + 1] = goal >= (int32_t)i ? src : -2;
    int32_t l = -1;
    for (uint32_t z = 0; z < Z; ++z) {
      const int32_t d = deepest_level(o, o->wmeta[i * Z + z], o->wleaf[i * Z + z], b);
      l = d > l ? d : l;
    }
    const int c = l > goal;
    goal = c ? l : goal;
    src = c ? (int32_t)i : src;
  }
  /* PrepareTarget */
  int32_t dest = -2;
  src = -2;
  for (int32_t i = (int32_t)L; i >= -1; --i) {
    target[i + 1] = -2;
    const int hit = i == src;
    target[i + 1] = hit ? dest : target[i + 1];
    dest = hit ? -2 : dest;
    src = hit ? -2 : src;
    int empty = 0;
    if (i >= 0)
      for (uint32_t z = 0; z < Z; ++z) empty |= o->wmeta[i * Z + z] == 0;
    const int take = ((dest == -2 && empty) || target[i + 1] != -2) && deepest[i + 1] != -2;
    src = take ? deepest[i + 1] : src;
    dest = take ? i : dest;
  }
  /* EvictOnce: level -1 (stash) .. L */
  uint64_t hmeta = 0;
  uint32_t hleaf = 0;
  int32_t hdest = -2;
  for (int32_t i = -1; i <= (int32_t)L; ++i) {
    const uint32_t nslot = i < 0 ? STASH : Z;
    uint8_t *bd = i < 0 ? o->sdata : o->wdata + (size_t)i * Z * bsz;
    uint64_t *bm = i < 0 ? o->smeta : o->wmeta + (size_t)i * Z;
    uint32_t *bl = i < 0 ? o->sleaf : o->wleaf + (size_t)i * Z;
    /* the held block drops here */
    const int drop = hmeta != 0 && i == hdest;
    uint8_t *tw = o->tmp; /* towrite */
    cmov_block(tw, o->hold, bsz, mask_of(drop));
    const uint64_t twm = drop ? hmeta : 0;
    const uint32_t twl = drop ? hleaf : 0;
    hmeta = drop ? 0 : hmeta;
    hdest = drop ? -2 : hdest;
    /* pick up the block of this level that goes deepest */
    const int pick = target[i + 1] != -2;
    int32_t best = -1, bz = -1;
    for (uint32_t z = 0; z < nslot; ++z) {
      const int32_t d = deepest_level(o, bm[z], bl[z], b);
      const int c = d > best;
      best = c ? d : best;
      bz = c ? (int32_t)z : bz;
    }
    for (uint32_t z = 0; z < nslot; ++z) {
      const uint64_t m = mask_of(pick && (int32_t)z == bz);
      cmov_block(o->hold, bd + (size_t)z * bsz, bsz, m);
      hmeta = cmov_u64(hmeta, bm[z], m);
      hleaf = (uint32_t)cmov_u64(hleaf, bl[z], m);
      bm[z] = cmov_u64(bm[z], 0, m);
    }
    hdest = pick ? target[i + 1] : hdest;
    /* the dropped block takes the first empty slot */
    int placed = !drop;
    for (uint32_t z = 0; z < nslot; ++z) {
      const int c = !placed && bm[z] == 0;
      const uint64_t m = mask_of(c);
      cmov_block(bd + (size_t)z * bsz, tw, bsz, m);
      bm[z] = cmov_u64(bm[z], twm, m);
      bl[z] = (uint32_t)cmov_u64(bl[z], twl, m);
      placed |= c;
    }
    if (!placed) abort(); /* the targets guarantee room */
  }
}

/* reverse-lexicographic eviction path g (Gentry et al.; Circuit ORAM) */
static uint32_t revlex(const oram *o, uint64_t g) {
  uint32_t r = 0;
  for (uint32_t k = 0; k < o->L; ++k) r |= (uint32_t)((g >> k) & 1u) << (o->L - 1 - k);
  return r;
}

/* Path ORAM access with aligned-cmov block moves: remap, check out the
 * branch, select the block out of every stash and branch slot, apply fn,
 * move it to the first free stash slot, evict along the branch and along one
 * deterministic path, check in. */
static void oram_access(oram *o, uint64_t idx, access_fn fn, void *ctx) {
  const uint32_t bsz = o->bsz, W = (o->L + 1) * Z;
  const uint32_t newleaf = (uint32_t)(sm64(o->rng) % o->leaves);
  const uint32_t old = pm_swap(o, idx, newleaf) % (uint32_t)o->leaves;
  o->accesses++;
  branch_io(o, old, 0);
  /* the block, out of every slot (zero if it is new) */
  uint8_t *t = o->hold; /* hold is free outside evict_branch */
  memset(t, 0, bsz);
  for (uint32_t s = 0; s < STASH; ++s)
    cmov_block(t, o->sdata + (size_t)s * bsz, bsz, mask_of(o->smeta[s] == idx + 1));
  for (uint32_t w = 0; w < W; ++w)
    cmov_block(t, o->wdata + (size_t)w * bsz, bsz, mask_of(o->wmeta[w] == idx + 1));
  fn(ctx, t);
  /* the block leaves its slot and goes to the first free stash slot with its
     new leaf (a block stays only on the path of its own leaf) */
  for (uint32_t s = 0; s < STASH; ++s) o->smeta[s] = cmov_u64(o->smeta[s], 0, mask_of(o->smeta[s] == idx + 1));
  for (uint32_t w = 0; w < W; ++w) o->wmeta[w] = cmov_u64(o->wmeta[w], 0, mask_of(o->wmeta[w] == idx + 1));
  uint64_t placed = 0;
  for (uint32_t s = 0; s < STASH; ++s) {
    const uint64_t m = ~placed & mask_of(o->smeta[s] == 0);
    cmov_block(o->sdata + (size_t)s * bsz, t, bsz, m);
    o->smeta[s] = cmov_u64(o->smeta[s], idx + 1, m);
    o->sleaf[s] = (uint32_t)cmov_u64(o->sleaf[s], newleaf, m);
    placed |= m;
  }
  if (!placed) abort(); /* stash overflow: negligible at Z = 4, 25 % load */
  evict_branch(o, old);
  branch_io(o, old, 1);
  const uint32_t e = revlex(o, o->evictions++);
  branch_io(o, e, 0);
  evict_branch(o, e);
  branch_io(o, e, 1);
}

/* ---------------------------------------------------- cuckoo hash table */

#define CK_PER 2        /* items per bucket */
#define CK_KICKS 64     /* displacement steps before giving up */
#define CK_VMAX 1024    /* value bytes at most */

typedef struct cuckoo {
  oram *t[2];
  uint64_t nb;        /* buckets per table */
  uint32_t vsz, isz;  /* value bytes; item bytes (16-byte key, value) */
  uint64_t hk[2][2];  /* SipHash keys of the two tables */
  uint64_t *rng;
  uint64_t kicks;
} cuckoo;

/* The op applied to a key's value (zeroed when absent): returns what becomes
 * of the item. */
enum { CK_LEAVE = 0, CK_KEEP = 1, CK_REMOVE = 2 };
typedef int (*ck_fn)(void *ctx, uint8_t *val, int present);

static int zero(const uint8_t *p, size_t n) {
  uint8_t a = 0;
  for (size_t i = 0; i < n; ++i) a |= p[i];
  return a == 0;
}

static void cuckoo_free(cuckoo *c) {
  if (!c) return;
  oram_free(c->t[0]);
  oram_free(c->t[1]);
  free(c);
}

/* room for `cap` items at 50 % load */
static cuckoo *cuckoo_new(uint64_t cap, uint32_t vsz, uint64_t *rng) {
  cuckoo *c = (cuckoo *)calloc(1, sizeof *c);
  if (!c) return NULL;
  c->nb = (cap + CK_PER - 1) / CK_PER;
  if (c->nb == 0) c->nb = 1;
  c->vsz = vsz;
  c->isz = 16 + vsz;
  c->rng = rng;
  for (int t = 0; t < 2; ++t) {
    c->hk[t][0] = sm64(rng);
    c->hk[t][1] = sm64(rng);
    c->t[t] = oram_new(c->nb, CK_PER * c->isz, rng);
    if (!c->t[t]) {
      cuckoo_free(c);
      return NULL;
    }
  }
  return c;
}

static uint64_t ck_bucket(const cuckoo *c, int t, const uint8_t *key) {
  return gvo_siphash24(c->hk[t][0], c->hk[t][1], key, 16) % c->nb;
}

typedef struct {
  cuckoo *c;
  const uint8_t *key;
  ck_fn fn;
  void *ctx;
  uint64_t b1;
  uint8_t *blk0;
  int present;
  int has_pend;           /* an item displaced from table 0 */
  uint8_t pend[16 + CK_VMAX];
} ck_acc;

static void ck_in1(void *p, uint8_t *blk1) {
  ck_acc *a = (ck_acc *)p;
  cuckoo *c = a->c;
  uint8_t *blk[2] = {a->blk0, blk1};
  uint8_t *hit = NULL, *fr = NULL;
  for (int t = 0; t < 2; ++t)
    for (uint32_t i = 0; i < CK_PER; ++i) {
      uint8_t *it = blk[t] + (size_t)i * c->isz;
      const int empty = zero(it, 16);
      if (!empty && memcmp(it, a->key, 16) == 0) hit = it;
      if (empty && !fr) fr = it;
    }
  uint8_t tmp[CK_VMAX];
  uint8_t *val = hit ? hit + 16 : tmp;
  if (!hit) memset(tmp, 0, c->vsz);
  a->present = hit != NULL;
  const int r = a->fn(a->ctx, val, hit != NULL);
  if (hit && r == CK_REMOVE) {
    memset(hit, 0, c->isz);
  } else if (!hit && r == CK_KEEP) {
    uint8_t *dst = fr;
    if (!dst) { /* both buckets full: displace a random item of table 0's */
      dst = blk[0] + (size_t)(sm64(c->rng) % CK_PER) * c->isz;
      memcpy(a->pend, dst, c->isz);
      a->has_pend = 1;
    }
    memcpy(dst, a->key, 16);
    memcpy(dst + 16, tmp, c->vsz);
  }
}

static void ck_in0(void *p, uint8_t *blk0) {
  ck_acc *a = (ck_acc *)p;
  a->blk0 = blk0;
  oram_access(a->c->t[1], a->b1, ck_in1, a);
}

typedef struct {
  cuckoo *c;
  uint8_t *item;  /* in: the item to place; out: the one it displaced */
  int placed;
} ck_kick;

static void ck_kick_fn(void *p, uint8_t *blk) {
  ck_kick *k = (ck_kick *)p;
  const cuckoo *c = k->c;
  uint8_t tmp[16 + CK_VMAX];
  for (uint32_t i = 0; i < CK_PER; ++i) {
    uint8_t *it = blk + (size_t)i * c->isz;
    if (zero(it, 16)) {
      memcpy(it, k->item, c->isz);
      k->placed = 1;
      return;
    }
  }
  uint8_t *v = blk + (size_t)(sm64(c->rng) % CK_PER) * c->isz;
  memcpy(tmp, v, c->isz);
  memcpy(v, k->item, c->isz);
  memcpy(k->item, tmp, c->isz);
}

/* One access to `key`: both buckets, fn applied to its value.  Returns
 * whether the key was present. */
static int cuckoo_access(cuckoo *c, const uint8_t key[16], ck_fn fn, void *ctx) {
  ck_acc a;
  a.c = c;
  a.key = key;
  a.fn = fn;
  a.ctx = ctx;
  a.b1 = ck_bucket(c, 1, key);
  a.has_pend = 0;
  a.present = 0;
  oram_access(c->t[0], ck_bucket(c, 0, key), ck_in0, &a);
  if (a.has_pend) { /* the displaced item goes to its other table, and so on */
    ck_kick k = {c, a.pend, 0};
    int t = 1;
    for (int step = 0; step < CK_KICKS && !k.placed; ++step, t ^= 1) {
      c->kicks++;
      oram_access(c->t[t], ck_bucket(c, t, k.item), ck_kick_fn, &k);
    }
    if (!k.placed) abort(); /* table overflow: not reached at 50 % load */
  }
  return a.present;
}

static int ck_leave(void *ctx, uint8_t *val, int present) {
  (void)ctx, (void)val, (void)present;
  return CK_LEAVE;
}

/* a dummy access: the buckets of a random key, nothing changed */
static void cuckoo_dummy(cuckoo *c) {
  uint8_t key[16];
  const uint64_t a = sm64(c->rng), b = sm64(c->rng);
  memcpy(key, &a, 8);
  memcpy(key + 8, &b, 8);
  cuckoo_access(c, key, ck_leave, NULL);
}

/* ------------------------------------------------------------- the model */

struct gvp_model {
  gvs_config cfg;
  uint64_t N, R;
  uint32_t Q, Sr, B, logQ;
  uint8_t prp_key[16], hash_key[16];
  uint64_t count, ctr, n_mailboxes, head, tail, ring_size;
  uint32_t *ring;
  uint64_t rng;
  cuckoo *msg, *mbox;
  oram *occ;
};

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
  m->msg = cuckoo_new(m->N, sizeof(gvs_record), &m->rng);
  m->mbox = cuckoo_new(m->R < m->N ? m->R : m->N, 1024, &m->rng);
  m->occ = oram_new((m->Q + 255) / 256, 1024, &m->rng);
  if (!m->ring || !m->msg || !m->mbox || !m->occ) {
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
  cuckoo_free(m->msg);
  cuckoo_free(m->mbox);
  oram_free(m->occ);
  free(m);
}

/* ---- partition occupancy: read, then add delta ---- */
typedef struct {
  uint32_t off;
  int32_t delta;
  uint32_t count; /* out: before the delta */
} occ_ctx;
static void occ_fn(void *c, uint8_t *blk) {
  occ_ctx *x = (occ_ctx *)c;
  uint32_t *e = (uint32_t *)blk;
  x->count = e[x->off];
  e[x->off] = (uint32_t)((int32_t)e[x->off] + x->delta);
}
/* q < 0: a dummy access (a random block, nothing changed) */
static uint32_t occ_do(gvp_model *m, int64_t q, int32_t delta) {
  const uint64_t nblk = (m->Q + 255) / 256;
  occ_ctx c = {0, 0, 0};
  uint64_t blk = sm64(&m->rng) % nblk;
  if (q >= 0) {
    blk = (uint64_t)q / 256;
    c.off = (uint32_t)q % 256;
    c.delta = delta;
  }
  oram_access(m->occ, blk, occ_fn, &c);
  return c.count;
}

static uint32_t part_of(const gvp_model *m, uint64_t hi) {
  return m->logQ ? (uint32_t)(hi >> (64 - m->logQ)) : 0u;
}
static void rkey(uint64_t hi, uint64_t lo, uint8_t key[16]) {
  memcpy(key, &hi, 8);
  memcpy(key + 8, &lo, 8);
}

/* ---- mailbox row access (the value: recipient + 62 ids) ---- */
typedef struct {
  int op;        /* 0 read, 1 append (create a fresh row if `room`), 2 pop head, 3 remove id */
  int room;      /* op 1: the partition can take a new recipient */
  uint8_t x[32], id[16];
  uint32_t len_before, len_after;
  int done;      /* append: appended; pop: popped; remove: found */
  int fresh;     /* op 1: a new row */
  uint8_t head[16];
} row_ctx;
static int row_fn(void *c, uint8_t *blk, int present) {
  row_ctx *x = (row_ctx *)c;
  uint8_t *ids = blk + 32;
  x->done = 0;
  x->fresh = 0;
  x->len_before = x->len_after = 0;
  if (!present) {
    if (x->op != 1 || !x->room) return CK_LEAVE;
    memcpy(blk, x->x, 32);
    memcpy(ids, x->id, 16);
    x->done = x->fresh = 1;
    x->len_after = 1;
    return CK_KEEP;
  }
  uint32_t len = 0;
  while (len < GVS_MAILBOX_SLOTS && !zero(ids + 16 * len, 16)) ++len;
  x->len_before = len;
  memcpy(x->head, ids, 16);
  if (x->op == 1 && len < GVS_MAILBOX_SLOTS) {
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
  x->len_after = len;
  if (x->op == 0) return CK_LEAVE;
  return len == 0 ? CK_REMOVE : CK_KEEP; /* an emptied row leaves the table */
}
/* key NULL: a dummy access */
static int row_do(gvp_model *m, const uint8_t *key, row_ctx *c) {
  if (!key) {
    cuckoo_dummy(m->mbox);
    return 0;
  }
  return cuckoo_access(m->mbox, key, row_fn, c);
}

/* ---- message access by id ---- */
typedef struct {
  int op;                 /* 0 read, 1 insert rec, 2 remove, 3 by-id op of req */
  const gvs_request *rq;
  gvs_record rec, out;
  uint32_t status;
} msg_ctx;
static int msg_fn(void *c, uint8_t *blk, int present) {
  msg_ctx *x = (msg_ctx *)c;
  gvs_record *r = (gvs_record *)blk;
  memcpy(&x->out, r, sizeof *r);
  if (x->op == 1) {
    memcpy(r, &x->rec, sizeof *r);
    return CK_KEEP;
  }
  if (x->op == 2) return present ? CK_REMOVE : CK_LEAVE;
  if (x->op != 3) return CK_LEAVE;
  const gvs_request *q = x->rq;
  const uint32_t t = q->request_type;
  const int auth = present && (memcmp(q->auth_identity, r->sender, 32) == 0 ||
                               memcmp(q->auth_identity, r->recipient, 32) == 0);
  x->status = GVS_STATUS_SUCCESS;
  if (!auth) x->status = GVS_STATUS_NOT_FOUND;
  else if (t != GVS_REQUEST_READ && memcmp(q->recipient, r->recipient, 32) != 0)
    x->status = GVS_STATUS_INVALID_RECIPIENT;
  if (x->status == GVS_STATUS_SUCCESS && t == GVS_REQUEST_UPDATE) {
    memcpy(r->payload, q->payload, GVS_PAYLOAD_BYTES);
    r->timestamp = q->timestamp;
    memcpy(&x->out, r, sizeof *r);
    return CK_KEEP;
  }
  if (x->status == GVS_STATUS_SUCCESS && t == GVS_REQUEST_DELETE) return CK_REMOVE;
  return CK_LEAVE;
}
/* id NULL: a dummy access */
static void msg_do(gvp_model *m, const uint8_t *id, msg_ctx *c) {
  if (!id) cuckoo_dummy(m->msg);
  else cuckoo_access(m->msg, id, msg_fn, c);
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

/* Every request: six ORAM accesses (occupancy, mailbox table x2, message
 * table x2, occupancy), real or dummy.  Order differs between creates/next
 * ops and by-id ops. */

static void g_create(gvp_model *m, const gvs_request *rq, gvs_response *o) {
  const int bad = zero(rq->recipient, 32);
  uint64_t hi = 0, lo = 0;
  gvo_recipient_hash(m->hash_key, rq->recipient, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  const int full = m->count >= m->N;
  const int skip = bad || full;
  const uint32_t used = occ_do(m, skip ? -1 : (int64_t)q, 0);
  gvs_record rec;
  memset(&rec, 0, sizeof rec);
  const uint32_t slot = m->ring[m->head % m->ring_size];  /* candidate */
  gvo_id_encode(m->prp_key, slot, m->ctr, rec.msg_id);
  row_ctx r;
  memset(&r, 0, sizeof r);
  r.op = 1;
  r.room = used < m->Sr;
  memcpy(r.x, rq->recipient, 32);
  memcpy(r.id, rec.msg_id, 16);
  uint8_t key[16];
  rkey(hi, lo, key);
  const int present = row_do(m, skip ? NULL : key, &r);
  uint32_t status = GVS_STATUS_SUCCESS;
  if (bad) status = GVS_STATUS_INVALID_RECIPIENT;
  else if (full) status = GVS_STATUS_TOO_MANY_MESSAGES;
  else if (!present && !r.room) status = GVS_STATUS_TOO_MANY_RECIPIENTS;
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
    msg_do(m, rec.msg_id, &mc);
    m->count++;
    if (r.fresh) m->n_mailboxes++;
    ok(o, &rec);
  } else {
    msg_do(m, NULL, &mc);
    fail(o, status, rq->timestamp);
  }
  occ_do(m, r.fresh ? (int64_t)q : -1, 1);
}

static void g_next(gvp_model *m, const gvs_request *rq, gvs_response *o, int del) {
  uint64_t hi, lo;
  gvo_recipient_hash(m->hash_key, rq->auth_identity, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  occ_do(m, -1, 0);
  row_ctx r;
  memset(&r, 0, sizeof r);
  r.op = del ? 2 : 0;
  uint8_t key[16];
  rkey(hi, lo, key);
  const int present = row_do(m, key, &r);
  const int have = present && r.len_before > 0;
  msg_ctx mc;
  memset(&mc, 0, sizeof mc);
  mc.op = del ? 2 : 0;
  msg_do(m, have ? r.head : NULL, &mc);
  const int emptied = have && del && r.len_after == 0;
  occ_do(m, emptied ? (int64_t)q : -1, -1);
  if (!have) {
    fail(o, GVS_STATUS_NOT_FOUND, rq->timestamp);
    return;
  }
  ok(o, &mc.out);
  if (del) {
    uint32_t s;
    uint64_t ctr;
    gvo_id_decode(m->prp_key, r.head, m->N, &s, &ctr);
    free_slot(m, s);
    if (emptied) m->n_mailboxes--;
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
  msg_do(m, valid ? rq->msg_id : NULL, &mc);
  const int del = mc.status == GVS_STATUS_SUCCESS && rq->request_type == GVS_REQUEST_DELETE;
  uint64_t hi, lo;
  gvo_recipient_hash(m->hash_key, rq->recipient, &hi, &lo);
  const uint32_t q = part_of(m, hi);
  occ_do(m, -1, 0);
  row_ctx r;
  memset(&r, 0, sizeof r);
  r.op = 3;
  memcpy(r.id, rq->msg_id, 16);
  uint8_t key[16];
  rkey(hi, lo, key);
  row_do(m, del ? key : NULL, &r);
  const int emptied = del && r.done && r.len_after == 0;
  occ_do(m, emptied ? (int64_t)q : -1, -1);
  if (mc.status != GVS_STATUS_SUCCESS) {
    fail(o, mc.status, rq->timestamp);
    return;
  }
  ok(o, &mc.out);
  if (del) {
    free_slot(m, slot);
    if (emptied) m->n_mailboxes--;
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
  return m->msg->t[0]->accesses + m->msg->t[1]->accesses + m->mbox->t[0]->accesses +
         m->mbox->t[1]->accesses + m->occ->accesses;
}
