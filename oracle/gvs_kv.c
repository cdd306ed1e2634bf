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
