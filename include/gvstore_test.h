/*
 * gvstore_test.h — test hooks of libgvstore_test.so (the same engine built
 * with -DGVS_TEST_HOOKS).  They read or overwrite a store's device state
 * (decrypting it in authenticated mode), so the production library
 * libgvstore.so does not export them: an enclave binds only include/gvstore.h.
 */
#ifndef GVSTORE_TEST_H
#define GVSTORE_TEST_H

#include "gvstore.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Copy the slot-addressed message table (N * 1024 bytes per shard, shards in
 * order) to host memory; test use. */
int gvs_dump_messages(gvs_handle *h, void *host_dst, uint64_t bytes);

/* Raw device regions of one shard, for tests of the storage format:
 * 0 message table (physical rows), 1 mailbox table, 2 mailbox side entries,
 * 3 message row tags, 4 mailbox row tags (3, 4: authenticated mode only),
 * 5 the final row states the last batch left pending (B x 1024, by sorted
 * position), 6 their side entries (B x 128: 16 used, target row, valid), 7 their tags
 * (authenticated mode), 8 the last batch's slot descriptors (W*c x 128). */
int gvs_raw_size(gvs_handle *h, uint32_t shard, uint32_t region, uint64_t *size);
int gvs_dump_raw(gvs_handle *h, uint32_t shard, uint32_t region, uint64_t offset, void *dst,
                 uint64_t bytes);
int gvs_store_raw(gvs_handle *h, uint32_t shard, uint32_t region, uint64_t offset,
                  const void *src, uint64_t bytes);

/* The engine handle under a block store (gvs_oram_*), so that the raw-region
 * hooks above reach its sealed block table (region 0), its tags (3) and its
 * pending final states (5, 6, 7): tamper tests of the sealed block store. */
gvs_handle *gvs_oram_test_handle(gvs_oram *o);

/* The engine handle under a key-value map (gvs_omap_*): its key directory
 * (region 9) and, sealed, the directory's row tags (10), besides the block
 * table's regions: tamper tests of the sealed map. */
gvs_handle *gvs_omap_test_handle(gvs_omap *m);

/* Set the storage epoch of every shard (authenticated mode only), without
 * re-sealing anything: tests that a store at the epoch limit refuses work
 * with GVS_ERR_EPOCH_EXHAUSTED on every entry point. */
int gvs_test_set_epoch(gvs_handle *h, uint32_t epoch);

/* The router's placement of one source's batch, computed on
 * the host by the device's own routing function: slot[i] = d * C + (rank of
 * request i among this batch's requests for shard d), or 0xFFFFFFFF when that
 * rank is >= C (the batch then overflows: GVS_ERR_BATCH_OVERFLOW).  shed[i]
 * (may be NULL) = 1 when request i is past its routing key's cap (it then
 * travels to shard i mod S as a hard error and is answered INTERNAL_ERROR).
 * Also reports C and the shard pipeline size.  No device is touched; the CPU
 * multi-process tests use it to run the real placement over gloo. */
int gvs_route_plan(const gvs_config *cfg, const gvs_request *reqs, uint32_t n, uint32_t *slot,
                   uint32_t *capacity, uint32_t *shard_batch, uint8_t *shed);

#ifdef __cplusplus
}
#endif

#endif /* GVSTORE_TEST_H */
