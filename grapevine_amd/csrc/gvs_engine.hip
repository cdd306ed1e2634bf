// gvs_engine.hip — host side of libgvstore.so: the C ABI of include/gvstore.h
// driving the gfx950 kernels of gvs_kernels.h / gvs_route.h on one HIP stream.
//
// A handle owns one or more shard engines (Engine: the tables and per-batch
// scratch of one shard) and, when sharded, the router buffers
// of DESIGN.md §6.  Three modes:
//   kSingle  one shard, no routing (gvs_create with shard_count <= 1)
//   kLocal   S shards on one device in this process; the all-to-all is a set
//            of device copies (gvs_create with shard_count > 1; tests)
//   kRccl    one shard per process; the all-to-all is RCCL send/recv over
//            xGMI, error words are max-reduced over ranks (gvs_create_sharded)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>

#include "../../include/gvstore.h"
#include "../../include/gvstore_test.h"
#include "gvs_kernels.h"
#include "gvs_route.h"
#include "gvs_mtx.h"
#include "gvs_kv.h"
#include "gvs_omap.h"
#include "gvs_wire.h"
#include "gvs_sr25519.h"
#include "gvs_spass.h"
#include "gvs_mauth.h"
#ifndef GVS_MA_EXTRA_LDS
#define GVS_MA_EXTRA_LDS 0  // A/B builds: extra dynamic LDS (one sealed mailbox workgroup per CU)
#endif

using namespace gvs;

static_assert(sizeof(gvs_record) == 1024, "record layout");
static_assert(sizeof(gvs_request) == 1040, "request layout");
static_assert(sizeof(gvs_response) == 1040, "response layout");
static_assert(sizeof(ncclUniqueId) == GVS_COMM_ID_BYTES, "comm id size");
static_assert(sizeof(gvs_oram_config) == 64, "oram config layout");
static_assert(sizeof(gvs_block_op) == 1040, "block op layout (kAbiU4 uint4)");
static_assert(sizeof(gvs_omap_op) == 1056, "map op layout (66 uint4)");
static_assert(sizeof(gvs_omap_result) == 1040, "map result layout (k_out)");

namespace {

constexpr int kMaxMarks = 24;
constexpr uint64_t kExtra = 64;   // per-op records after the B real ones (record B = dry dummy)
// Authenticated storage binds every sealed row to a 32-bit epoch (one per
// batch).  A store refuses work well before the epoch could wrap, since a
// wrapped epoch would reuse CTR keystream and accept replayed rows
// (gvs_crypto.h); the caller then rebuilds the store under a fresh key.
constexpr uint32_t kEpochLimit = 0xFFFFFF00u;

enum Mode { kSingle, kLocal, kRccl };

bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }
uint32_t log2u(uint64_t v) {
  uint32_t l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}
uint64_t ld64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

// One shard: persistent tables + per-batch scratch for a batch of B ops.
struct Engine {
  uint32_t shard = 0;
  uint64_t N = 0, R = 0, ring_size = 0;
  uint32_t Q = 0, Sr = 0, B = 0, W = 0, S = 0, logQ = 0, nblk = 0;
  KeyCtx kc{};
  uint4* table = nullptr;
  uint4* mbox = nullptr;
  uint4* side = nullptr;
  uint32_t* ring = nullptr;
  Scal* scal = nullptr;
  uint4* img = nullptr;
  uint32_t* types = nullptr;
  OpState* ops = nullptr;
  uint32_t* kinds = nullptr;
  Key128* s1keys = nullptr;
  M1Out* m1out = nullptr;
  uint32_t* pflag = nullptr;
  uint32_t* pslot = nullptr;
  uint32_t* bsum = nullptr;
  uint32_t* cslot = nullptr;
  ROp* rop = nullptr;
  uint64_t* rkeys = nullptr;
  RRes* rres = nullptr;
  uint4* resp = nullptr;     // (B + extra) internal response slots of kRespSlot bytes
  uint32_t* dflag = nullptr;
  uint32_t* dslot = nullptr;
  uint32_t* bsum2 = nullptr;
  uint4* recv = nullptr;     // routed modes: S*C incoming request slots
  uint4* mtag = nullptr;     // authenticated storage: N message-row tags
  uint4* btag = nullptr;     //                        R mailbox-row tags
  uint32_t epoch = 0;        // batches applied: rows are sealed at this epoch
  // expiry sweep: X = cfg.expiry_per_batch ops at [B - X, B)
  uint32_t X = 0, xk = 1, xep = 0;
  // fixed-slot message pass (gvs_txn.h)
  uint32_t c = 0;            // transaction slots per message partition
  uint32_t par = 0;          // flips with every applied batch (ping-pong buffers)
  uint32_t stamp_run = 0, stamp_prev = kNone, stamp_next = 1;
  uint4* tbuf[2] = {};       // (W*c + B) x 128-B slot descriptors
  uint4* xb2[2] = {};        // expiry records, written by one pass, read by the next batch
  uint4* rpos = nullptr;     // B sorted-position records
  uint4* rsb = nullptr;      // B x 128 B
  uint4* snap = nullptr;     // W*c x 1 KiB
  uint4* pbuf = nullptr;     // B x 1 KiB final row states, by sorted position
  uint4* psd = nullptr;      // B side entries of P (target row, valid), 128 B each
  uint4* ptag = nullptr;     // B tags of P (authenticated storage)
  uint4* ps = nullptr;       // W*c x 1 KiB final states by slot (AUTH: + W*c x 128 B side entries)
  uint4* snapp = nullptr;    // B x 1 KiB row snapshots at their first op's position
  uint4* dryb = nullptr;     // W x 4 KiB (k_rpass2: one 1 KiB per dry use)
  RtxV* rtx_agg = nullptr;
  RtxV* rtx_carry = nullptr;
  Rr1V* rr1_agg = nullptr;
  Rr1V* rr1_carry = nullptr;
  uint4* rr1g = nullptr;     // B x 256 B (gvs_txn.h Rr1Op::gathered)
  uint4* m2g = nullptr;      // B x 128 B (gvs_mtx.h k_m2g)
  uint4* idn = nullptr;      // B x 128 B request identity lines (k_meta -> k_rr1)
  uint4* snapid = nullptr;   // W*c x 128 B snapshot identity lines (k_rpass2 -> k_rr1)
  uint4* snapidp = nullptr;  // B x 128 B their identity lines (k_rpass2 -> k_rr1)
  uint4* vagg = nullptr, *vagg2 = nullptr, *vcarry2 = nullptr, *vcarry = nullptr;
  // fixed-slot mailbox passes (gvs_mtx.h)
  uint32_t cm = 0;           // group slots per mailbox partition
  uint4* mpos = nullptr;     // B
  uint4* gtx = nullptr;      // (Q*cm + B) x 128 B: this batch's (one of gtxb)
  uint4* gtxb[2] = {};       // ping-pong: a deferred write pass reads the previous batch's
  uint32_t gsel = 0;
  // Deferred mailbox write pass (plain single-GPU stores): a batch's k_m2x
  // runs fused with the next batch's read pass (k_m21x), or alone when the
  // table is needed first (flush_m2).  gscal->error: the next batch's
  // group-slot overflow while the write pass is still to run.
  bool m2_pending = false;
  MArgs m2_args{};
  Scal* gscal = nullptr;
  uint4* msnap = nullptr;    // Q*cm x 1 KiB
  uint4* msnapp = nullptr;   // B x 1 KiB (group snapshots by head position)
  uint4* mpid = nullptr;     // B x 16 B: each sorted position's message id (k_gtx, for k_m1r_c)
  uint4* mdry = nullptr;     // Q x 8 KiB (k_m1x / k_m2x: one 1 KiB per dry use)
  uint4* m2tx = nullptr;     // (Q*cm + B) x 1152 B
  GtxV* gtx_agg = nullptr;
  GtxV* gtx_carry = nullptr;
  // block / key-value stores (gvs_kv.h, gvs_omap.h)
  uint4* kvmeta = nullptr;   // B x 128-B op lines
  uint4* kvdummy = nullptr;  // B x 1 KiB
  uint4* kdir = nullptr;     // N x 32 B key directory (key, hash)
  uint4* ktag = nullptr;     // sealed map: N/32 directory row tags
  Key128* okeys = nullptr;   // B (hash, seq) sort keys
  uint4* opr = nullptr;      // B x 128 B position records
  uint4* opos = nullptr;     // B
  uint4* ogt = nullptr;      // (W*c + B) x 128 B group records
  uint4* ogp = nullptr;      // (B + W*c) x 128 B group results by head position
  OgtV* ogt_agg = nullptr;
  OgtV* ogt_carry = nullptr;
  OrowV* orow_agg = nullptr;
  OrowV* orow_carry = nullptr;
};

// Router state of one source rank (kLocal: one per virtual rank).
struct Router {
  uint32_t* dest = nullptr;
  uint64_t* rkey = nullptr;  // routing keys, sorted per window (hot-key cap)
  uint64_t* marks = nullptr; // shed marks by sorted position, then sorted back to request order
  uint32_t* shed = nullptr;
  uint32_t* bcnt = nullptr;
  uint32_t* pos = nullptr;
  uint32_t* tot = nullptr;
  uint4* send = nullptr;     // S*C outgoing request slots
  uint4* back = nullptr;     // S*C returning response slots
};

}  // namespace

// Double-buffered host path (gvs_process_batches): pinned host staging, two
// device staging pairs, a copy stream and per-slot events.
struct HostPipe {
  bool ready = false;
  uint4* din[2] = {};
  uint4* dout[2] = {};
  uint8_t* hin[2] = {};
  uint8_t* hout[2] = {};
  uint32_t* herr = nullptr;  // pinned: the agreed error word of the batch in each slot
  uint32_t* errs = nullptr;  // pinned: one error word per batch of gvs_process_batches_device
  uint32_t nerr = 0;
  hipStream_t copy = nullptr;      // host -> device
  hipStream_t copy_out = nullptr;  // device -> host (its own queue: an H2D of batch t+1
                                   // must not wait behind the D2H of batch t)
  hipEvent_t h2d[2] = {}, done[2] = {}, d2h[2] = {};
};

// Device staging of the host wire path (gvs_process_wire_batch), allocated on
// first use for max_submit messages of kWireSlotMax bytes each way.
struct WireStage {
  uint8_t* in = nullptr;
  uint8_t* out = nullptr;
  uint32_t* in_lens = nullptr;
  uint32_t* out_lens = nullptr;
  uint64_t* times = nullptr;
  uint4* sigs = nullptr;
  uint32_t* status = nullptr;
  uint4* chal = nullptr;     // n x 32-B challenges
};

// Double-buffered wire path (gvs_process_wire_batches): per slot, the device
// and pinned host buffers of one batch's wire messages and results, allocated
// on first use for max_submit messages of kWireSlotMax bytes each way.
struct WirePipe {
  bool ready = false;
  uint8_t *din[2] = {}, *dout[2] = {};
  uint32_t *dlens[2] = {}, *dolens[2] = {}, *dstat[2] = {};
  uint64_t* dtimes[2] = {};
  uint4* dchal[2] = {};
  uint8_t *hin[2] = {}, *hout[2] = {}, *hchal[2] = {};
  uint32_t *hlens[2] = {}, *holens[2] = {}, *hstat[2] = {};
  uint64_t* htimes[2] = {};
  hipEvent_t h2d[2] = {}, done[2] = {}, d2h[2] = {};
};

// Pinned bounce buffers of the single-call host APIs (gvs_process_batch, the
// wire batch, the block store and the map).  A hipMemcpy from or to pageable
// memory pins the caller's pages in place and unpins them afterwards; the
// unmapping invalidates the device's TLB, so every kernel of the next batch
// re-walks the page tables of the buffers it touches, a number of walks (L2
// uncached reads, counted in FETCH_SIZE) that follows the batch's data
// (DESIGN.md §3 "Counters").  Pageable caller memory is therefore copied by
// the host into grow-only pinned buffers and moved by DMA from there.
struct Bounce {
  static constexpr int kSlots = 8;  // 0..3 in, 4..7 out
  void* buf[kSlots] = {};
  size_t cap[kSlots] = {};
  struct Out {
    void* dst;
    int slot;
    size_t bytes;
  };
  std::vector<Out> pend;  // device -> pinned copies enqueued, to hand to the caller after the sync
  // a DMA from or into a slot may still be in flight: a call that failed after
  // enqueuing returns without the stream sync of finish()
  bool inflight = false;
};

struct gvs_handle {
  gvs_config cfg{};
  Mode mode = kSingle;
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t S = 1;       // shards in the store
  uint32_t C = 0;       // routed slots per (source, shard)
  uint32_t Bsub = 0;    // requests per source per call (cfg.max_batch)
  uint32_t Be = 0;      // ops per shard pipeline (Bsub, or shard_batch(S*C + X))
  std::vector<Engine> eng;
  std::vector<Router> rt;
  ncclComm_t comm = nullptr;
  uint4* in_stage = nullptr;   // host API staging (caller layout)
  uint4* out_stage = nullptr;
  hipEvent_t ev[kMaxMarks] = {};
  const char* mark_name[kMaxMarks] = {};
  int n_marks = 0;
  bool timed = false;
  bool auth = false;         // GVS_FLAG_AUTH_STORAGE
  bool poisoned = false;     // an integrity failure was seen
  SealCtx sc{};              // storage keys (epoch filled per engine)
  uint32_t* te = nullptr;    // AES table on the device
  uint32_t* nhk = nullptr;   // message row hash's NH key on the device (sc.nhk)
  uint64_t cutoff = 0;       // expiry sweep: rows with timestamp < cutoff expire
  int kind = 0;              // 0 message store, 1 block store (gvs_oram_*), 2 key-value map (gvs_omap_*)
  int sealed_nw = 0;         // waves per workgroup of the sealed message pass (4, 8, 12; 0: by S)
  HostPipe pipe;
  WireStage wire;
  WirePipe wpipe;
  Bounce bounce;
  uint8_t* sr_dev = nullptr;  // gvs_sr25519_verify's device staging (grow-only)
  size_t sr_cap = 0;
  uint32_t* err_pin = nullptr;  // finish(): the error word's pinned landing place
  std::vector<void*> allocs;
  std::string err;
};

#define GVS_HIP(h, call)                                                        \
  do {                                                                          \
    hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess) {                                                     \
      if (h) (h)->err = std::string(#call) + ": " + hipGetErrorString(e_);      \
      return GVS_ERR_DEVICE;                                                    \
    }                                                                           \
  } while (0)

#define GVS_NCCL(h, call)                                                       \
  do {                                                                          \
    ncclResult_t r_ = (call);                                                   \
    if (r_ != ncclSuccess) {                                                    \
      if (h) (h)->err = std::string(#call) + ": " + ncclGetErrorString(r_);     \
      return GVS_ERR_DEVICE;                                                    \
    }                                                                           \
  } while (0)

static int dalloc(gvs_handle* h, void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    h->err = std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? GVS_ERR_OUT_OF_MEMORY : GVS_ERR_DEVICE;
  }
  h->allocs.push_back(*p);
  return GVS_OK;
}

template <typename T>
static int dalloc_t(gvs_handle* h, T** p, size_t count) {
  return dalloc(h, reinterpret_cast<void**>(p), count * sizeof(T));
}

static void mark(gvs_handle* h, const char* name) {
  if (!h->timed || h->n_marks >= kMaxMarks) return;
  (void)hipEventRecord(h->ev[h->n_marks], h->stream);
  h->mark_name[h->n_marks++] = name;
}

// ------------------------------------------------------------------ creation

static int validate(const gvs_config* c) {
  if (!c) return GVS_ERR_INVALID_ARG;
  if (!is_pow2(c->msg_capacity) || c->msg_capacity < 256 || c->msg_capacity > (1ull << 32))
    return GVS_ERR_INVALID_ARG;
  if (!is_pow2(c->mailbox_partitions) || c->mailbox_partitions + 1 > (uint32_t)kBinsMax)
    return GVS_ERR_INVALID_ARG;
  if (c->mailbox_partition_slots == 0 || c->mailbox_partition_slots > (uint32_t)kSrMax ||
      (c->mailbox_partition_slots % 16) != 0)
    return GVS_ERR_INVALID_ARG;
  if (!is_pow2(c->max_batch) || c->max_batch < 1024 || c->max_batch > (1u << (kSeqBits - 1)))
    return GVS_ERR_INVALID_ARG;
  if (c->flags & ~GVS_FLAG_AUTH_STORAGE) return GVS_ERR_INVALID_ARG;
  // sealed mailbox partitions: the per-row values of k_m1a / k_m2a live in the
  // AES window's holes (gvs_mauth.h)
  if ((c->flags & GVS_FLAG_AUTH_STORAGE) && c->mailbox_partition_slots > kSrAuth) return GVS_ERR_INVALID_ARG;
  if (c->rows_per_partition && (!is_pow2(c->rows_per_partition) ||
                                c->rows_per_partition < (uint32_t)kTile ||
                                c->rows_per_partition > (uint32_t)kRowsMax))
    return GVS_ERR_INVALID_ARG;
  if (c->shard_count > kShardsMax) return GVS_ERR_INVALID_ARG;
  if (c->route_capacity > c->max_batch) return GVS_ERR_INVALID_ARG;
  for (int i = 0; i < 2; ++i)
    if (c->reserved[i] != 0) return GVS_ERR_INVALID_ARG;
  if (c->expiry_per_batch &&
      (!is_pow2(c->expiry_per_batch) || c->expiry_per_batch > c->max_batch / 2))
    return GVS_ERR_INVALID_ARG;
  return GVS_OK;
}

// Default C: mean load B/S plus 8 standard deviations of a binomial bucket
// and a constant, rounded to 64.  Uniformly keyed traffic then overflows with
// probability far below 1e-12 per batch; skewed traffic (one recipient taking
// more than C of a source's requests) fails the batch as a whole.
static uint32_t auto_capacity(uint32_t B, uint32_t S) {
  if (S <= 1) return B;
  const double mu = std::ceil((double)B / S);
  uint64_t c = (uint64_t)std::ceil(mu + 8.0 * std::sqrt(mu) + 64.0);
  c = (c + 63) / 64 * 64;
  return (uint32_t)(c < B ? c : B);
}

// Ops per shard pipeline for m routed slots plus expiry deletes (0: too many).
// The oracle's cluster model (oracle/gvs_oracle.c gvo_shard_batch) agrees.
static uint32_t shard_batch(uint64_t m) {
  uint64_t p2 = 1024;
  while (p2 < m) p2 <<= 1;
  const uint64_t r = (m + 8191) / 8192 * 8192;
  const uint64_t be = std::max<uint64_t>(1024, std::min(p2, r));
  return be > (1u << (kSeqBits - 1)) ? 0u : (uint32_t)be;
}

// Transaction slots per message partition (gvs_txn.h): the distinct rows a
// batch's B ops touch in one of W partitions are at most binomial(B, 1/W) for
// uniformly spread slots; mean + 8 standard deviations + 16, rounded to 8,
// overflows with probability far below 1e-12 per batch.  At most S (a
// partition's rows) and B.
static uint32_t txn_slots(uint32_t B, uint32_t W, uint32_t S) {
  const double mu = (double)B / W;
  uint64_t c = (uint64_t)std::ceil(mu + 8.0 * std::sqrt(mu) + 16.0);
  c = (c + 7) / 8 * 8;
  if (c > S) c = S;
  if (c > B) c = B;
  if (c > kSlotMax) c = kSlotMax;
  return (uint32_t)c;
}

// The X expiry deletes of one batch are by-id deletes of X recorded messages;
// each distinct recipient among them takes one group slot of its mailbox
// partition.  Their load per partition must fit the partition's group slots
// on its own, by the same binomial bound the slots are sized with (recipients
// are spread by the keyed PRF): otherwise a batch could overflow on its expiry
// deletes alone, and since a failed batch keeps its records for the next one,
// every later batch (even an empty one) would fail the same way.  This rules
// out configurations whose group slots are capped (kGroupMax) below the
// deletes' own bound, e.g. few mailbox partitions and a large X.
static bool expiry_fits(const gvs_config* c, bool sharded) {
  if (!c->expiry_per_batch) return true;
  uint32_t Be = c->max_batch;
  if (sharded) {
    const uint32_t S = c->shard_count ? c->shard_count : 1;
    const uint32_t C = c->route_capacity ? c->route_capacity : auto_capacity(c->max_batch, S);
    Be = shard_batch((uint64_t)S * C + c->expiry_per_batch);
    if (!Be) return false;
  }
  const uint32_t need = txn_slots(c->expiry_per_batch, c->mailbox_partitions, ~0u);
  return need <= txn_slots(Be, c->mailbox_partitions, kGroupMax);
}

// ------------------------------------------------- authenticated storage (host)

static uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) p ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return p;
}

// AES S-box from log/antilog tables of the generator 3 plus the affine map
static void aes_sbox(uint8_t sb[256]) {
  uint8_t lg[256] = {}, alg[256] = {};
  uint8_t x = 1;
  for (int i = 0; i < 255; ++i) {
    alg[i] = x;
    lg[x] = (uint8_t)i;
    x = gf_mul(x, 3);
  }
  for (int v = 0; v < 256; ++v) {
    uint8_t inv = v ? alg[(255 - lg[v]) % 255] : 0;
    uint8_t s = inv, r = inv;
    for (int k = 0; k < 4; ++k) {
      r = (uint8_t)((r << 1) | (r >> 7));
      s ^= r;
    }
    sb[v] = (uint8_t)(s ^ 0x63);
  }
}

static void aes_tables(const uint8_t sb[256], uint32_t te0[256]) {
  for (int v = 0; v < 256; ++v) {
    const uint8_t s1 = sb[v], s2 = gf_mul(s1, 2), s3 = (uint8_t)(s2 ^ s1);
    te0[v] = ((uint32_t)s2 << 24) | ((uint32_t)s1 << 16) | ((uint32_t)s1 << 8) | s3;
  }
}

static void aes_expand(const uint8_t sb[256], const uint8_t key[16], AesRk& rk) {
  for (int i = 0; i < 4; ++i)
    rk.w[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
              ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
  uint32_t rcon = 0x01000000u;
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk.w[i - 1];
    if (i % 4 == 0) {
      t = ((uint32_t)sb[(t >> 16) & 0xff] << 24) | ((uint32_t)sb[(t >> 8) & 0xff] << 16) |
          ((uint32_t)sb[t & 0xff] << 8) | sb[t >> 24];
      t ^= rcon;
      rcon = (uint32_t)gf_mul((uint8_t)(rcon >> 24), 2) << 24;
    }
    rk.w[i] = rk.w[i - 4] ^ t;
  }
}

static void b2_block(const uint8_t* p, size_t n, uint64_t m[16]) {
  uint8_t b[128] = {};
  std::memcpy(b, p, n);
  for (int i = 0; i < 16; ++i) m[i] = ld64(b + 8 * i);
}

// keyed BLAKE2b (32-byte key) of a message shorter than one block
static void b2_keyed_short(const uint8_t key[32], const char* msg, uint32_t nn, uint8_t* out) {
  B2State s = b2_init(nn, 32, 0, 0);
  uint64_t m[16];
  b2_block(key, 32, m);
  b2_compress(s, m, 128, false);
  const size_t len = std::strlen(msg);
  b2_block((const uint8_t*)msg, len, m);
  b2_compress(s, m, 128 + len, true);
  for (uint32_t i = 0; i < nn; ++i) out[i] = (uint8_t)(s.h[i / 8] >> (8 * (i % 8)));
}

// storage keys from the config secret: AES key, MAC key
// states, the message row hash's keys (nh: kNhWords words on the host; the
// caller puts them in device memory for sc.nhk)
static void storage_ctx(const uint8_t secret[32], SealCtx& sc, uint32_t te0[256], uint32_t nh[kNhWords]) {
  uint8_t sb[256], ak[16], mk[32];
  aes_sbox(sb);
  aes_tables(sb, te0);
  b2_keyed_short(secret, "gvs storage aes", 16, ak);
  b2_keyed_short(secret, "gvs storage mac", 32, mk);
  aes_expand(sb, ak, sc.rk);
  uint8_t kh[16];
  b2_keyed_short(secret, "gvs storage head", 16, kh);
  aes_expand(sb, kh, sc.rkh);
  for (uint32_t i = 0; i < 4; ++i)  // mailbox table: 4 leaves of 256 B
    sc.leafk1[i] = b2_keyed_state(mk, kLeafPerson0, (uint64_t)i | (1ull << 32));
  sc.headk = b2_keyed_state(mk, kHeadPerson0, 0);
  // row hash keys: BLAKE2b-512(key = mac_key, "gvs-uhash-" | byte j), j < 19
  uint8_t kb[19 * 64];
  for (uint32_t j = 0; j < 19; ++j) {
    const uint8_t msg[11] = {'g', 'v', 's', '-', 'u', 'h', 'a', 's', 'h', '-', (uint8_t)j};
    B2State st = b2_init(64, 32, 0, 0);
    uint64_t m[16];
    b2_block(mk, 32, m);
    b2_compress(st, m, 128, false);
    b2_block(msg, sizeof msg, m);
    b2_compress(st, m, 128 + sizeof msg, true);
    for (uint32_t i = 0; i < 64; ++i) kb[64 * j + i] = (uint8_t)(st.h[i / 8] >> (8 * (i % 8)));
  }
  auto ld32 = [](const uint8_t* q) {
    return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
  };
  for (uint32_t w = 0; w < kNhWords; ++w) nh[w] = ld32(kb + 4 * w);
  for (uint32_t i = 0; i < 16; ++i) {
    const uint64_t k = ld64(kb + 1072 + 8 * i) & ((1ull << 36) - 1);
    sc.l3k[i] = k >= kP36 ? k - kP36 : k;
  }
  for (uint32_t t = 0; t < 4; ++t) sc.l3p[t] = ld32(kb + 1200 + 4 * t);
  sc.nhk = nullptr;
  sc.epoch = 0;
  sc.on = 1;
}

static SealCtx seal_of(const gvs_handle* h, const Engine& e) {
  SealCtx c = h->sc;
  c.epoch = e.epoch;
  return c;
}

static int engine_init(gvs_handle* h, Engine& e, uint32_t shard, uint32_t B) {
  const gvs_config* cfg = &h->cfg;
  e.shard = shard;
  e.N = cfg->msg_capacity;
  e.Q = cfg->mailbox_partitions;
  e.Sr = cfg->mailbox_partition_slots;
  e.R = (uint64_t)e.Q * e.Sr;
  e.B = B;
  e.logQ = log2u(e.Q);
  // rows per message-table partition (one workgroup each): the config value
  // if set, else N/4096 clamped to [256, 4096] (C3: 4096 rows -> 4096
  // workgroups, 16 times the chip's resident capacity; few partitions keep
  // the fixed transaction slots W*c small, gvs_txn.h)
  uint64_t S = cfg->rows_per_partition ? cfg->rows_per_partition : e.N / 4096;
  if (S < (uint64_t)kTile) S = kTile;
  if (S > (uint64_t)kRowsMax) S = kRowsMax;
  if (S > e.N) S = e.N;
  if (!is_pow2(S)) return GVS_ERR_INVALID_ARG;
  e.S = (uint32_t)S;
  e.W = (uint32_t)(e.N / S);
  e.nblk = B / 1024;
  e.ring_size = e.N + B;
  if (e.W + 1 > (uint32_t)kBinsMax) return GVS_ERR_INVALID_ARG;
  e.c = txn_slots(B, e.W, e.S);
  e.cm = txn_slots(B, e.Q, kGroupMax);  // recipient groups per mailbox partition
  // expiry sweep: X records per batch; workgroups w = epoch (mod xk) record
  // xep each (X >= W: every workgroup, X / W each; X < W: one each, a rotating
  // 1/xk of the workgroups)
  e.X = cfg->expiry_per_batch;
  if (e.X) {
    e.xep = e.X >= e.W ? e.X / e.W : 1u;
    e.xk = e.X >= e.W ? 1u : e.W / e.X;
    if (e.xep > kXepMax) return GVS_ERR_INVALID_ARG;
  }
  e.kc.pk0 = ld64(cfg->secret_key);
  e.kc.pk1 = ld64(cfg->secret_key + 8);
  e.kc.hk0 = ld64(cfg->secret_key + 16);
  e.kc.hk1 = ld64(cfg->secret_key + 24);
  e.kc.tag = shard_tag(shard);
  e.kc.nshards = h->S;

#define A(ptr, n)                                \
  do {                                           \
    if (int r_ = dalloc_t(h, &e.ptr, (n))) return r_; \
  } while (0)
  const uint64_t E = kExtra;
  A(table, e.N * 64);
  A(mbox, e.R * 64);
  A(side, e.R);
  A(ring, e.ring_size);
  A(scal, 1);
  A(img, (B + E) * 64);
  A(types, B);
  A(ops, B);
  A(kinds, B);
  A(s1keys, B);
  A(m1out, B + E);
  A(pflag, B);
  A(pslot, B);
  A(bsum, 2 * e.nblk);
  A(cslot, B);
  A(rop, B + E);
  A(rkeys, B);
  A(rres, B + E);
  A(resp, (B + E) * kSlotU4);
  A(dflag, B);
  A(dslot, B);
  A(bsum2, e.nblk);
  if (h->mode != kSingle) A(recv, (uint64_t)h->S * h->C * kSlotU4);
  if (h->auth) {
    A(mtag, e.N);
    A(btag, e.R);
  }
  {  // fixed-slot message pass
    const uint64_t WC = (uint64_t)e.W * e.c;
    for (int k = 0; k < 2; ++k) {
      A(tbuf[k], (WC + B) * 8);
      if (e.X) A(xb2[k], (uint64_t)e.X * 8);
    }
    A(rpos, B);
    A(rsb, (uint64_t)B * 8);
    A(snap, WC * 64);
    if (h->auth) A(pbuf, (uint64_t)B * 64);  // sealed P (plain final states go to PS)
    A(psd, (uint64_t)B * 8);
    if (h->auth) A(ptag, B);
    A(ps, (WC + B) * (h->auth ? 72 : 64));  // W*c slots + B sink lines (AUTH: then their side-entry lines)
    A(snapp, (uint64_t)B * 64);
    A(dryb, (uint64_t)e.W * 256);
    A(rtx_agg, B / kScanT);
    A(rtx_carry, B / kScanT);
    A(rr1_agg, B / kScanT);
    A(rr1_carry, B / kScanT);
    A(rr1g, (uint64_t)B * 16);
    A(m2g, (uint64_t)B * 8);
    A(idn, (uint64_t)B * 8);
    A(snapid, WC * 8);
    A(snapidp, (uint64_t)B * 8);
    const uint64_t nvb = B / kVBlk, nvb2 = (nvb + 63) / 64;
    A(vagg, nvb * kVLineU4);
    A(vcarry, nvb * kVLineU4);
    A(vagg2, nvb2 * kVLineU4);
    A(vcarry2, nvb2 * kVLineU4);
    const uint64_t QC = (uint64_t)e.Q * e.cm;
    A(mpos, B);
    A(gtxb[0], (QC + B) * 8);
    A(gtxb[1], (QC + B) * 8);
    e.gtx = e.gtxb[0];
    A(gscal, 1);
    A(msnap, QC * 64);
    A(msnapp, (uint64_t)B * 64);
    A(mpid, B);
    A(mdry, (uint64_t)e.Q * kMDryU4);
    A(m2tx, (QC + B) * kVLineU4);
    A(gtx_agg, B / kScanT);
    A(gtx_carry, B / kScanT);
  }
#undef A
  hipStream_t s = h->stream;
  GVS_HIP(h, hipMemsetAsync(e.img + (uint64_t)B * 64, 0, E * 1024, s));
  GVS_HIP(h, hipMemsetAsync(e.rop + B, 0, E * sizeof(ROp), s));
  GVS_HIP(h, hipMemsetAsync(e.table, 0, e.N * 1024, s));
  GVS_HIP(h, hipMemsetAsync(e.mbox, 0, e.R * 1024, s));
  GVS_HIP(h, hipMemsetAsync(e.side, 0, e.R * 16, s));
  for (int k = 0; k < 2; ++k) GVS_HIP(h, hipMemsetAsync(e.gtxb[k], 0, ((uint64_t)e.Q * e.cm + B) * 128, s));
  GVS_HIP(h, hipMemsetAsync(e.gscal, 0, sizeof(Scal), s));
  GVS_HIP(h, hipMemsetAsync(e.rkeys, 0xFF, (uint64_t)B * 8, s));  // null rows until written
  for (int k = 0; k < 2; ++k) {
    GVS_HIP(h, hipMemsetAsync(e.tbuf[k], 0, ((uint64_t)e.W * e.c + B) * 128, s));
    if (e.X) GVS_HIP(h, hipMemsetAsync(e.xb2[k], 0, (uint64_t)e.X * 128, s));
  }
  // free ring = slots 0..N-1 in order; scalars
  std::vector<uint32_t> ring(e.ring_size, kNone);
  for (uint64_t i = 0; i < e.N; ++i) ring[i] = (uint32_t)i;
  Scal sc{};
  sc.head = 0;
  sc.tail = e.N;
  GVS_HIP(h, hipMemcpyAsync(e.ring, ring.data(), ring.size() * 4, hipMemcpyHostToDevice, s));
  GVS_HIP(h, hipMemcpyAsync(e.scal, &sc, sizeof sc, hipMemcpyHostToDevice, s));
  if (h->auth) {  // every row starts as a sealed all-zero row at epoch 0
    e.epoch = 0;
    const SealCtx c = seal_of(h, e);
    hipLaunchKernelGGL(k_seal_init, dim3(1024), dim3(256), 0, s, c, (const uint32_t*)h->te,
                       e.table, e.mtag, (uint4*)nullptr, 0u, e.N);
    hipLaunchKernelGGL(k_seal_init, dim3(256), dim3(256), 0, s, c, (const uint32_t*)h->te,
                       e.mbox, e.btag, e.side, 1u, e.R);
    GVS_HIP(h, hipGetLastError());
  }
  GVS_HIP(h, hipStreamSynchronize(s));
  return GVS_OK;
}

static int router_init(gvs_handle* h, Router& r) {
  const uint64_t B = h->Bsub, SC = (uint64_t)h->S * h->C;
  if (int rc = dalloc_t(h, &r.dest, B)) return rc;
  if (int rc = dalloc_t(h, &r.rkey, B)) return rc;
  if (int rc = dalloc_t(h, &r.marks, B)) return rc;
  if (int rc = dalloc_t(h, &r.shed, B)) return rc;
  if (int rc = dalloc_t(h, &r.bcnt, (B / 1024) * h->S)) return rc;
  if (int rc = dalloc_t(h, &r.pos, B)) return rc;
  if (int rc = dalloc_t(h, &r.tot, h->S)) return rc;
  if (int rc = dalloc_t(h, &r.send, SC * kSlotU4)) return rc;
  if (int rc = dalloc_t(h, &r.back, SC * kSlotU4)) return rc;
  return GVS_OK;
}

extern "C" int gvs_destroy(gvs_handle* h);

static int create_common(const gvs_config* cfg, Mode mode, const uint8_t* comm_id,
                         gvs_handle** out) {
  if (!out) return GVS_ERR_INVALID_ARG;
  *out = nullptr;
  if (int rc = validate(cfg)) return rc;
  if (!expiry_fits(cfg, mode != kSingle)) return GVS_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GVS_ERR_NO_DEVICE;
  if ((int)cfg->device >= ndev) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = new (std::nothrow) gvs_handle();
  if (!h) return GVS_ERR_OUT_OF_MEMORY;
  h->cfg = *cfg;
  h->mode = mode;
  h->device = (int)cfg->device;
  h->auth = (cfg->flags & GVS_FLAG_AUTH_STORAGE) != 0;
  h->S = cfg->shard_count ? cfg->shard_count : 1;
  h->Bsub = cfg->max_batch;
  if (mode == kRccl && cfg->shard_index >= h->S) {
    delete h;
    return GVS_ERR_INVALID_ARG;
  }
  if (mode == kSingle) {
    h->C = 0;
    h->Be = h->Bsub;
  } else {
    // a shard pipeline: the S*C routed slots, then the expiry sweep's X
    // deletes; the smaller of the next power of two and the next multiple of
    // 8192 (the sorts take any multiple of their tile, gvs_kernels.h)
    h->C = cfg->route_capacity ? cfg->route_capacity : auto_capacity(h->Bsub, h->S);
    h->Be = shard_batch((uint64_t)h->S * h->C + cfg->expiry_per_batch);
    if (h->Be == 0) {
      delete h;
      return GVS_ERR_INVALID_ARG;
    }
  }
  auto fail = [&](int code) {
    std::string e = h->err;
    gvs_destroy(h);
    (void)e;
    return code;
  };
  if (hipSetDevice(h->device) != hipSuccess) return fail(GVS_ERR_DEVICE);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(GVS_ERR_DEVICE);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(GVS_ERR_DEVICE);
  if (h->auth) {
    uint32_t te0[256], nh[kNhWords];
    storage_ctx(cfg->secret_key, h->sc, te0, nh);
    if (int rc = dalloc_t(h, &h->te, 256)) return fail(rc);
    if (hipMemcpy(h->te, te0, sizeof te0, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GVS_ERR_DEVICE);
    if (int rc = dalloc_t(h, &h->nhk, kNhWords)) return fail(rc);
    if (hipMemcpy(h->nhk, nh, sizeof nh, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GVS_ERR_DEVICE);
    h->sc.nhk = h->nhk;
  }

  const uint32_t n_eng = mode == kLocal ? h->S : 1u;
  const uint32_t n_src = mode == kSingle ? 0u : (mode == kLocal ? h->S : 1u);
  h->eng.resize(n_eng);
  h->rt.resize(n_src);
  for (uint32_t k = 0; k < n_eng; ++k) {
    const uint32_t shard = mode == kRccl ? cfg->shard_index : k;
    if (int rc = engine_init(h, h->eng[k], shard, h->Be)) return fail(rc);
  }
  for (uint32_t k = 0; k < n_src; ++k)
    if (int rc = router_init(h, h->rt[k])) return fail(rc);
  const uint64_t stage = (uint64_t)h->Bsub * (mode == kLocal ? h->S : 1u);
  if (int rc = dalloc_t(h, &h->in_stage, stage * kAbiU4)) return fail(rc);
  if (int rc = dalloc_t(h, &h->out_stage, stage * kAbiU4)) return fail(rc);
  if (mode == kRccl) {
    ncclUniqueId id;
    std::memcpy(&id, comm_id, sizeof id);
    ncclResult_t r = ncclCommInitRank(&h->comm, (int)h->S, id, (int)cfg->shard_index);
    if (r != ncclSuccess) {
      h->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      h->comm = nullptr;
      return fail(GVS_ERR_DEVICE);
    }
  }
  *out = h;
  return GVS_OK;
}

// ------------------------------------------------------------------ pipeline

// Bitonic sort of n keys (n a multiple of L = 1024 E, gvs_kernels.h): tiles
// sorted in registers/LDS, then for each merge level k up to the power of two
// >= n the global steps (two per launch) and the tile-local finish.
static uint32_t lower_count(uint32_t n, uint32_t blk, uint32_t half) {
  return (n / blk) * half + std::min(n % blk, half);  // indices b*blk + o < n, o < half
}

template <typename K, int E>
static void sort_tiles(hipStream_t s, K* d, uint32_t n) {
  constexpr uint32_t L = 1024u * E;
  hipLaunchKernelGGL((k_bitonic_tile<K, E>), dim3(n / L), dim3(1024), 0, s, d, 0u, 1);
  for (uint32_t k = 2 * L; (k >> 1) < n; k <<= 1) {
    uint32_t j = k >> 1;
    for (; j >= 8 * L; j >>= 4) {  // four steps per launch while all are global
      const uint32_t nq = lower_count(n, 2 * j, j >> 3);
      hipLaunchKernelGGL(k_bitonic_global4<K>, dim3((nq + 255) / 256), dim3(256), 0, s, d, n, k, j, nq);
    }
    for (; j >= 2 * L; j >>= 2) {  // two steps per launch while both are global
      const uint32_t nq = lower_count(n, 2 * j, j >> 1);
      hipLaunchKernelGGL(k_bitonic_global2<K>, dim3((nq + 255) / 256), dim3(256), 0, s, d, n, k, j, nq);
    }
    if (j >= L) {
      const uint32_t np = lower_count(n, 2 * j, j);
      hipLaunchKernelGGL(k_bitonic_global<K>, dim3((np + 255) / 256), dim3(256), 0, s, d, n, k, j, np);
    }
    hipLaunchKernelGGL((k_bitonic_tile<K, E>), dim3(n / L), dim3(1024), 0, s, d, k, 0);
  }
}

// Tiles of 1024 keys (EMAX = 1) at every call: 64 workgroups per tile launch
// for a 64K batch instead of 8-16, which outweighs the extra global steps
// (C3: both sorts 0.23 -> 0.145 ms per batch, profiles/r03n_pass_ab.txt)
template <typename K, int EMAX>
static int sort_keys(gvs_handle* h, K* d, uint32_t n) {
  if (n < 1024 || n % 1024) return GVS_ERR_INTERNAL;
  uint32_t e = EMAX;  // the largest tile that divides n
  while ((n / 1024) % e) e >>= 1;
  switch (e) {
    case 1: sort_tiles<K, 1>(h->stream, d, n); break;
    case 2: sort_tiles<K, 2>(h->stream, d, n); break;
    case 4: sort_tiles<K, (EMAX < 4 ? EMAX : 4)>(h->stream, d, n); break;
    default: sort_tiles<K, EMAX>(h->stream, d, n); break;
  }
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

static MArgs margs(const gvs_handle* h, const Engine& e) {
  MArgs a{};
  a.sc = seal_of(h, e);
  a.te = h->te;
  a.btag = e.btag;
  a.keys = e.s1keys;
  a.mbox = e.mbox;
  a.side = e.side;
  a.m1out = e.m1out;
  a.rop = e.rop;
  a.rres = e.rres;
  a.scal = e.scal;
  a.Q = e.Q;
  a.Sr = e.Sr;
  a.B = e.B;
  a.N = e.N;
  a.kc = e.kc;
  return a;
}

static AllocArgs aargs(const Engine& e) {
  AllocArgs a{};
  a.kinds = e.kinds;
  a.m1out = e.m1out;
  a.ops = e.ops;
  a.pflag = e.pflag;
  a.pslot = e.pslot;
  a.bsum = e.bsum;
  a.cslot = e.cslot;
  a.ring = e.ring;
  a.rop = e.rop;
  a.rkeys = e.rkeys;
  a.scal = e.scal;
  a.B = e.B;
  a.nblk = e.nblk;
  a.W = e.W;
  a.S = e.S;
  a.N = e.N;
  a.ring_size = e.ring_size;
  a.kc = e.kc;
  return a;
}

// ------------------------------------------- pipeline 2: fixed-slot transactions

// a prime not dividing n (so x -> x * m mod n is a permutation) with n * m
// below 2^32 (the kernels compute x * m in 32 bits): the largest such prime
// of the list, 1 when none is
static uint32_t scatter_mul(uint64_t n) {
  for (uint32_t m : {4093u, 4091u, 4079u, 2039u, 2029u, 1021u, 1019u, 509u, 503u, 251u, 241u, 127u, 113u,
                     61u, 59u, 31u, 29u, 13u, 11u, 7u, 5u, 3u})
    if (n % m != 0u && n * m < (1ull << 32)) return m;
  return 1u;
}

static MArgs margs2(const gvs_handle* h, const Engine& e) {
  MArgs a = margs(h, e);
  a.gtx = e.gtx;
  a.m2tx = e.m2tx;
  a.msnap = e.msnap;
  a.msnapp = e.msnapp;
  a.mdry = e.mdry;
  a.stamp = e.stamp_run;
  a.cm = e.cm;
  a.sink_mul = scatter_mul((uint64_t)e.Q * e.cm);
  return a;
}

template <class A>
static void vscan_fields(A& a, const Engine& e) {
  a.vagg = e.vagg;
  a.vagg2 = e.vagg2;
  a.vcarry2 = e.vcarry2;
  a.vcarry = e.vcarry;
  a.scal = e.scal;
  a.nvb = e.B / kVBlk;
  a.nvb2 = (a.nvb + 63) / 64;
}

// the four scan kernels of a 1 KiB copy-forward (phase C is op-specific)
template <class Op>
static void vscan_abc(hipStream_t s, const typename Op::Args& a) {
  hipLaunchKernelGGL(k_vscan_a<Op>, dim3((a.nvb + 3) / 4), dim3(256), 0, s, a);  // a block per wave
  hipLaunchKernelGGL(k_vscan_b1<Op>, dim3(a.nvb2), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_vscan_b2<Op>, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_vscan_b3<Op>, dim3(a.nvb2), dim3(256), 0, s, a);
}

static PsealArgs pargs(const gvs_handle* h, const Engine& e, uint32_t ep) {
  return PsealArgs{e.pbuf, e.psd, e.ptag, seal_of(h, e), h->te, e.scal, ep,
                   e.ps, e.ps + ((uint64_t)e.W * e.c + e.B) * 64, e.W * e.c};
}

// Sealed stores stage every slot line of a partition in LDS when c fits
// (gvs_spass.h); the two batches' slots then share kSpBufs buffers, which
// k_sjoint checks before any state changes.
static bool sealed_staged(const Engine& e) { return e.c <= kSpSlots; }

static void launch_sjoint(gvs_handle* h, Engine& e) {
  if (!h->auth || !sealed_staged(e)) return;
  hipLaunchKernelGGL(k_sjoint, dim3((e.W + 3) / 4), dim3(256), 0, h->stream, (const uint4*)e.tbuf[e.par ^ 1],
                     (const uint4*)e.tbuf[e.par], e.stamp_prev, e.stamp_run, e.W, e.S, e.c, kSpBufs, e.scal);
}

// Phase A of pipeline 2: phase_a's kernels, then allocation, the message-pass
// sort and the transaction slots (k_rtx), so that every fixed-capacity check
// (mailbox groups, transaction slots) is decided before any state changes.
static int phase_a2(gvs_handle* h, Engine& e, const uint4* d_in, uint32_t stride, uint32_t n) {
  hipStream_t s = h->stream;
  const uint32_t B = e.B, nblk = e.nblk;
  e.stamp_run = e.stamp_next++;
  if (e.stamp_next == kNone) e.stamp_next = 1;
  const uint32_t xbase = B - e.X;
  // this batch's group descriptors; a deferred write pass of the previous
  // batch still reads the other buffer
  e.gtx = e.gtxb[e.gsel];
  e.gsel ^= 1u;
  const bool fuse = e.m2_pending;
  hipLaunchKernelGGL(k_copy, dim3(B / (4 * kCopyPerWave)), dim3(256), 0, s, d_in, stride, n, B, e.img, e.types,
                     (const uint4*)(e.X ? e.xb2[e.par ^ 1] : nullptr), xbase);
  mark(h, "copy");
  {
    MetaArgs a{e.img, e.types, e.ops, e.kinds, e.s1keys, n, B, e.Q, e.logQ, e.N, e.kc, xbase, e.idn};
    // one op per thread, no block-level work: 256-thread workgroups spread
    // the batch over every CU (1024-thread ones filled a quarter of them)
    hipLaunchKernelGGL(k_meta, dim3(B / 256), dim3(256), 0, s, a);
  }
  mark(h, "meta");
  if (int r = sort_keys<Key128, 1>(h, e.s1keys, B)) return r;
  mark(h, "sort_s1");
  {
    GtxArgs a{e.s1keys, e.ops, e.mpos, e.gtx, e.gtx_agg, e.gtx_carry, fuse ? e.gscal : e.scal,
              B,        e.Q,   e.logQ, e.cm,  B / kScanT, e.stamp_run};
    a.mpid = e.mpid;
    hipLaunchKernelGGL(k_scan_a<GtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<GtxOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<GtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  mark(h, "gtx");
  if (h->auth) {
    hipLaunchKernelGGL(k_m1a, dim3(e.Q), dim3(256), (e.cm + 1) * sizeof(GroupM) + GVS_MA_EXTRA_LDS, s, margs2(h, e));
  } else if (fuse) {
    // the previous batch's write pass and this batch's read pass in one
    // stream over the mailbox table; then this batch's group-slot overflow
    // (held apart so that it could not stop the previous batch's write)
    // joins its error word
    M21Args fa{e.m2_args, margs2(h, e), &e.gscal->error};
    hipLaunchKernelGGL(k_m21x, dim3(e.Q), dim3(256), e.Sr * sizeof(uint4) + 2 * (e.cm + 1) * sizeof(GroupM), s,
                       fa);
    hipLaunchKernelGGL(k_err_fold, dim3(1), dim3(64), 0, s, e.scal, &e.gscal->error);
    e.m2_pending = false;
  } else {
    hipLaunchKernelGGL(k_m1x<false>, dim3(e.Q), dim3(256), (e.cm + 1) * sizeof(GroupM), s, margs2(h, e));
  }
  {
    M1rArgs a{};
    vscan_fields(a, e);
    a.mpos = e.mpos;
    a.ops = e.ops;
    a.msnapp = e.msnapp;
    a.mpid = e.mpid;
    a.m1out = e.m1out;
    a.N = e.N;
    a.kc = e.kc;
    vscan_abc<M1rOp>(s, a);
    hipLaunchKernelGGL(k_m1r_c, dim3(a.nvb), dim3(256), 0, s, a);
  }
  mark(h, "m1");
  {
    AllocArgs a = aargs(e);
    hipLaunchKernelGGL(k_alloc_sum, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_alloc_ring, dim3(1), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_alloc_b, dim3(nblk * 4), dim3(256), 0, s, a);
  }
  mark(h, "alloc");
  if (int r = sort_keys<uint64_t, 1>(h, e.rkeys, B)) return r;
  mark(h, "sort_r");
  {
    RtxArgs a{e.rkeys, e.rpos, e.tbuf[e.par], e.rtx_agg, e.rtx_carry, e.scal,
              B,       e.W,    e.S,           e.c,       B / kScanT,  e.stamp_run};
    hipLaunchKernelGGL(k_scan_a<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<RtxOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  launch_sjoint(h, e);
  mark(h, "rtx");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

// The message-table pass of the fixed-slot pipeline (also the block and
// key-value stores' table pass): previous batch's P unsealed first (AUTH).
static void launch_rpass2(gvs_handle* h, Engine& e) {
  hipStream_t s = h->stream;
  const uint32_t B = e.B;
  R2Args a{};
  a.table = e.table;
  a.tcur = e.tbuf[e.par];
  a.tprev = e.tbuf[e.par ^ 1];
  a.stamp_cur = e.stamp_run;
  a.stamp_prev = e.stamp_prev;
  a.ps = e.ps;
  a.psds = h->auth ? e.ps + ((uint64_t)e.W * e.c + B) * 64 : nullptr;
  a.snap = e.snap;
  a.snapid = e.snapid;
  a.snapp = e.snapp;
  a.snapidp = e.snapidp;
  a.dry = e.dryb;
  a.scal = e.scal;
  a.W = e.W;
  a.S = e.S;
  a.c = e.c;
  a.xon = e.X ? 1u : 0u;
  a.xk = e.xk;
  a.xrot = e.epoch % e.xk;
  a.xep = e.xep;
  a.xexcl = e.xk == 1 ? 1u : 0u;
  a.cutoff = h->cutoff;
  a.xbuf = e.X ? e.xb2[e.par] : nullptr;
  a.xprev = e.X ? e.xb2[e.par ^ 1] : nullptr;
  if (h->auth) {
    a.sc = seal_of(h, e);
    a.te = h->te;
    a.mtag = e.mtag;
    // the previous batch's P (sealed at this epoch, by position) is unsealed
    // first, each row's final state to its slot's line of PS
    if (e.stamp_prev != kNone)
      hipLaunchKernelGGL(k_pseal<false>, dim3(B / 64), dim3(256), 0, s, pargs(h, e, e.epoch));
    mark(h, "punseal");
    // waves per workgroup: 12 (three per SIMD) once a partition has rounds
    // enough to keep them busy (S >= 1024: 32 groups of 32 rows), else 8
    const int nw = h->sealed_nw ? h->sealed_nw : (e.S >= 1024 ? 12 : 8);
    if (!sealed_staged(e))  // more slots than LDS stages: slot lines in the stream
      hipLaunchKernelGGL((k_spass<8, false>), dim3(e.W), dim3(512), 0, s, a);
    else if (nw == 12)
      hipLaunchKernelGGL((k_spass<12, true>), dim3(e.W), dim3(768), 0, s, a);
    else if (nw == 4)
      hipLaunchKernelGGL((k_spass<4, true>), dim3(e.W), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((k_spass<8, true>), dim3(e.W), dim3(512), 0, s, a);
  } else if (e.c <= kStageSlots && e.S % (16 * 8) == 0) {
    // the fixed-schedule pass: slot lines staged in LDS (gvs_txn.h k_rpass2s)
    hipLaunchKernelGGL((k_rpass2s<16, 8>), dim3(e.W), dim3(512), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_rpass2<16, true, true, 2>), dim3(e.W), dim3(256), 0, s, a);
  }
}

// The plain single-GPU message store defers each batch's mailbox write pass
// (DESIGN.md §3 "Fused mailbox passes"); sealed stores (k_m2a) and sharded
// stores run it at the end of the batch.
static bool defer_m2(const gvs_handle* h) { return h->mode == kSingle && !h->auth && h->kind == 0; }

static int phase_b2(gvs_handle* h, Engine& e, uint32_t n, uint4* d_out) {
  hipStream_t s = h->stream;
  const uint32_t B = e.B, nblk = e.nblk;
  launch_rpass2(h, e);
  mark(h, "rpass");
  {
    Rr1Args a{e.rpos, e.rop, e.rsb, e.rr1_agg, e.rr1_carry, e.scal, B, B / kScanT, B - e.X, e.S,
              e.rr1g, 0u, e.idn, e.snapidp};
    hipLaunchKernelGGL(k_scan_a<Rr1Op>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<Rr1Op>, dim3(1), dim3(kScanT), 0, s, a);
    a.pass = 1;
    hipLaunchKernelGGL(k_scan_c<Rr1Op>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  mark(h, "rr1");
  {
    Rr2Args a{};
    vscan_fields(a, e);
    a.rs = e.rsb;
    a.img = e.img;
    a.snapp = e.snapp;
    a.pbuf = e.pbuf;
    a.psd = e.psd;
    a.ps = h->auth ? nullptr : e.ps;  // AUTH: all by position, sealed, scattered by the unseal
    a.psink = h->auth ? e.pbuf : e.ps + (uint64_t)e.W * e.c * 64;  // non-last states (plain: PS's sink lines)
    a.resp = e.resp;
    a.rres = e.rres;
    a.B = B;
    a.cutoff = h->cutoff;
    vscan_abc<Rr2Op>(s, a);
    hipLaunchKernelGGL(k_rr2_c, dim3(a.nvb), dim3(256), 0, s, a);
  }
  if (h->auth)  // P at the epoch the pass wrote the rows at
    hipLaunchKernelGGL(k_pseal<true>, dim3(B / 64), dim3(256), 0, s, pargs(h, e, e.epoch + 1));
  mark(h, "rr2");
  {
    PostArgs a{e.kinds, e.rres, e.rop, e.dflag, e.dslot, e.bsum2, e.ring, e.scal, B, nblk,
               e.ring_size};
    hipLaunchKernelGGL(k_post_sum, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_post_ring, dim3(1), dim3(1024), 0, s, a);
  }
  mark(h, "post");
  {
    M2rArgs a{};
    vscan_fields(a, e);
    a.mpos = e.mpos;
    a.ops = e.ops;
    a.rop = e.rop;
    a.rres = e.rres;
    a.m1out = e.m1out;
    a.m2tx = e.m2tx;
    a.Q = e.Q;
    a.cm = e.cm;
    a.stamp = e.stamp_run;
    a.m2g = e.m2g;
    hipLaunchKernelGGL(k_m2g, dim3(B / 256), dim3(256), 0, s, a);
    vscan_abc<M2rOp>(s, a);
    hipLaunchKernelGGL(k_m2r_c, dim3(a.nvb), dim3(256), 0, s, a);
  }
  mark(h, "m2r");
  if (h->auth)
    hipLaunchKernelGGL(k_m2a, dim3(e.Q), dim3(256), (e.cm + 1) * sizeof(GroupM) + GVS_MA_EXTRA_LDS, s, margs2(h, e));
  else if (defer_m2(h))  // runs with the next batch's read pass (k_m21x) or alone in flush_m2
    e.m2_pending = true, e.m2_args = margs2(h, e);
  else
    hipLaunchKernelGGL(k_m2x<false>, dim3(e.Q), dim3(256), (e.cm + 1) * sizeof(GroupM) + e.Sr * sizeof(uint4), s,
                       margs2(h, e));
  if (d_out && n)
    hipLaunchKernelGGL(k_out, dim3((n + 4 * kCopyPerWave - 1) / (4 * kCopyPerWave)), dim3(256), 0, s,
                       (const uint4*)e.resp, n, d_out);
  mark(h, "m2");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}



static RouteArgs rargs(gvs_handle* h, const Router& r, const Engine& e, const uint4* in,
                       uint32_t n) {
  RouteArgs a{};
  a.in = in;
  a.n = n;
  a.B = h->Bsub;
  a.S = h->S;
  a.C = h->C;
  a.dest = r.dest;
  a.rkey = r.rkey;
  a.shed = r.shed;
  a.bcnt = r.bcnt;
  a.pos = r.pos;
  a.tot = r.tot;
  a.send = r.send;
  a.err = &e.scal->error;
  a.N = e.N;
  a.kc = e.kc;
  return a;
}

static int route(gvs_handle* h, const Router& r, const Engine& e, const uint4* in, uint32_t n) {
  hipStream_t s = h->stream;
  const RouteArgs a = rargs(h, r, e, in, n);
  const uint32_t nblk = h->Bsub / 1024;
  hipLaunchKernelGGL(k_route_dest, dim3(nblk), dim3(1024), 0, s, a);
  if (int rc = sort_keys<uint64_t, 1>(h, r.rkey, h->Bsub)) return rc;  // by (routing key, index)
  hipLaunchKernelGGL(k_route_mark, dim3(nblk), dim3(1024), 0, s, a, r.marks);
  if (int rc = sort_keys<uint64_t, 1>(h, r.marks, h->Bsub)) return rc;  // back to request order
  hipLaunchKernelGGL(k_route_apply, dim3(nblk), dim3(1024), 0, s, a, (const uint64_t*)r.marks);
  hipLaunchKernelGGL(k_route_hist, dim3(nblk), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_route_pos, dim3(nblk), dim3(1024), 0, s, a);
  if (n) hipLaunchKernelGGL(k_route_copy, dim3((n + 3) / 4), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_route_fill, dim3((h->S * h->C + 3) / 4), dim3(256), 0, s, a);
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

static int reset_errors(gvs_handle* h) {
  for (auto& e : h->eng)
    GVS_HIP(h, hipMemsetAsync(&e.scal->error, 0, sizeof(uint32_t), h->stream));
  return GVS_OK;
}

// all-to-all of S buckets of C slots: src_buf(k) bucket d -> dst_buf(d) bucket k
static int exchange(gvs_handle* h, bool forward) {
  const size_t bytes = (size_t)h->C * kRespSlot;
  const uint64_t span = (uint64_t)h->C * kSlotU4;
  if (h->mode == kLocal) {
    for (uint32_t src = 0; src < h->S; ++src)
      for (uint32_t dst = 0; dst < h->S; ++dst) {
        // forward: router src, bucket dst -> engine dst, bucket src
        // back:    engine src, bucket dst -> router dst, bucket src
        const uint4* from = forward ? h->rt[src].send + dst * span : h->eng[src].resp + dst * span;
        uint4* to = forward ? h->eng[dst].recv + src * span : h->rt[dst].back + src * span;
        GVS_HIP(h, hipMemcpyAsync(to, from, bytes, hipMemcpyDeviceToDevice, h->stream));
      }
    return GVS_OK;
  }
  const uint4* sendbuf = forward ? h->rt[0].send : h->eng[0].resp;
  uint4* recvbuf = forward ? h->eng[0].recv : h->rt[0].back;
  GVS_NCCL(h, ncclGroupStart());
  for (uint32_t p = 0; p < h->S; ++p) {
    GVS_NCCL(h, ncclSend(sendbuf + p * span, bytes, ncclUint8, (int)p, h->comm, h->stream));
    GVS_NCCL(h, ncclRecv(recvbuf + p * span, bytes, ncclUint8, (int)p, h->comm, h->stream));
  }
  GVS_NCCL(h, ncclGroupEnd());
  return GVS_OK;
}

// Make every shard see the OR (kLocal) / max (kRccl) of all error words, so
// that all shards apply a batch or none does.
static int agree_errors(gvs_handle* h) {
  if (h->mode == kLocal) {
    ErrSet es{};
    es.n = h->S;
    for (uint32_t k = 0; k < h->S; ++k) es.e[k] = &h->eng[k].scal->error;
    hipLaunchKernelGGL(k_err_or, dim3(1), dim3(64), 0, h->stream, es);
    GVS_HIP(h, hipGetLastError());
  } else if (h->mode == kRccl) {
    uint32_t* e = &h->eng[0].scal->error;
    GVS_NCCL(h, ncclAllReduce(e, e, 1, ncclUint32, ncclMax, h->comm, h->stream));
  }
  return GVS_OK;
}

// Enqueue one batch: n requests in the caller layout at d_in, responses in the
// caller layout to d_out (kLocal: n <= S*Bsub, source k = requests
// [k*Bsub, (k+1)*Bsub)).
static int run_batch_body(gvs_handle* h, const uint4* d_in, uint32_t n, uint4* d_out);

static int run_batch(gvs_handle* h, const uint4* d_in, uint32_t n, uint4* d_out,
                     bool reset = true) {
  h->n_marks = 0;
  mark(h, "start");
  if (reset)
    if (int r = reset_errors(h)) return r;
  return run_batch_body(h, d_in, n, d_out);
}

static int run_batch_body(gvs_handle* h, const uint4* d_in, uint32_t n, uint4* d_out) {
  if (h->mode == kSingle) {
    Engine& e = h->eng[0];
    if (int r = phase_a2(h, e, d_in, kAbiU4, n)) return r;
    return phase_b2(h, e, n, d_out);
  }
  const uint32_t n_src = (uint32_t)h->rt.size();
  for (uint32_t k = 0; k < n_src; ++k) {
    const uint64_t off = (uint64_t)k * h->Bsub;
    const uint32_t nk = n > off ? (uint32_t)std::min<uint64_t>(n - off, h->Bsub) : 0u;
    if (int r = route(h, h->rt[k], h->eng[k], d_in + off * kAbiU4, nk)) return r;
  }
  mark(h, "route");
  if (int r = exchange(h, true)) return r;
  mark(h, "xchg");
  const uint32_t SC = h->S * h->C;
  for (auto& e : h->eng)
    if (int r = phase_a2(h, e, e.recv, kSlotU4, SC)) return r;
  if (int r = agree_errors(h)) return r;
  mark(h, "agree");
  for (auto& e : h->eng)
    if (int r = phase_b2(h, e, SC, nullptr)) return r;
  if (int r = exchange(h, false)) return r;
  mark(h, "xchg_back");
  for (uint32_t k = 0; k < n_src; ++k) {
    const uint64_t off = (uint64_t)k * h->Bsub;
    const uint32_t nk = n > off ? (uint32_t)std::min<uint64_t>(n - off, h->Bsub) : 0u;
    if (nk)
      hipLaunchKernelGGL(k_route_gather, dim3((nk + 4 * kGatherPerWave - 1) / (4 * kGatherPerWave)),
                         dim3(256), 0, h->stream,
                         (const uint32_t*)h->rt[k].pos, (const uint32_t*)h->rt[k].shed,
                         d_in + off * kAbiU4, (const uint4*)h->rt[k].back, nk, d_out + off * kAbiU4);
  }
  mark(h, "gather");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

// The status of a batch from its (agreed) error word; records the handle's
// state (poisoned, message).  0: applied.
static int decode_error(gvs_handle* h, uint32_t e) {
  // a failed batch leaves no write pass behind: the one it inherited ran in
  // its k_m21x (the error word was clear then), its own is not to run
  if (e)
    for (auto& en : h->eng) en.m2_pending = false;
  if (e & 8u) {
    h->poisoned = true;
    h->err = "integrity failure: a stored row does not match its tag (authenticated storage)";
    return GVS_ERR_INTEGRITY;
  }
  if (e & 2u) h->poisoned = true;  // M2 stopped half-way: tables inconsistent
  if (e & 4u) {
    h->err = "batch overflow: more than route_capacity requests of one source for one shard";
    return GVS_ERR_BATCH_OVERFLOW;
  }
  if (e & 1u) {
    h->err = h->kind == 2 ? "batch overflow: more distinct keys in one partition than its group slots"
                          : "batch overflow: more recipients in one mailbox partition than its group slots";
    return GVS_ERR_BATCH_OVERFLOW;
  }
  if (e & kRErr) {
    h->err = "batch overflow: more distinct rows of one message partition than its transaction slots";
    return GVS_ERR_BATCH_OVERFLOW;
  }
  if (e & kJErr) {
    h->err = "batch overflow: the distinct rows of one message partition in this and the previous batch "
             "exceed the sealed pass's LDS staging buffers (" + std::to_string(kSpBufs) + ")";
    return GVS_ERR_BATCH_OVERFLOW;
  }
  if (e & kKvErr) {
    h->err = "invalid op: block index >= capacity or unknown op code";
    return GVS_ERR_INVALID_ARG;
  }
  if (e) {
    h->err = "internal error flag " + std::to_string(e);
    return GVS_ERR_INTERNAL;
  }
  return GVS_OK;
}

// host-side state an applied batch advances
struct HostState {
  uint32_t epoch[kShardsMax], par[kShardsMax], stamp_prev[kShardsMax];
};
static HostState save_state(const gvs_handle* h) {
  HostState st{};
  for (size_t k = 0; k < h->eng.size(); ++k) {
    st.epoch[k] = h->eng[k].epoch;
    st.par[k] = h->eng[k].par;
    st.stamp_prev[k] = h->eng[k].stamp_prev;
  }
  return st;
}
static void restore_state(gvs_handle* h, const HostState& st) {
  for (size_t k = 0; k < h->eng.size(); ++k) {
    h->eng[k].epoch = st.epoch[k];
    h->eng[k].par = st.par[k];
    h->eng[k].stamp_prev = st.stamp_prev[k];
  }
}
static void advance(gvs_handle* h) {
  for (auto& en : h->eng) {
    en.epoch += 1;  // every row was rewritten at epoch + 1
    // this batch's slots now hold the pending final states
    en.par ^= 1u;
    en.stamp_prev = en.stamp_run;
  }
}

static int finish(gvs_handle* h) {
  if (h->mode != kSingle)
    if (int r = agree_errors(h)) return r;  // late flags (M2) too: same verdict on every shard
  // read back into pinned memory: a copy to the stack goes through the
  // runtime's pageable path (bounce buffers above)
  if (!h->err_pin) GVS_HIP(h, hipHostMalloc((void**)&h->err_pin, sizeof(uint32_t), hipHostMallocDefault));
  GVS_HIP(h, hipMemcpyAsync(h->err_pin, &h->eng[0].scal->error, sizeof(uint32_t), hipMemcpyDeviceToHost,
                            h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  if (int r = decode_error(h, *h->err_pin)) return r;
  advance(h);
  return GVS_OK;
}

// Run a deferred mailbox write pass on its own (k_m2x), before anything reads
// the mailbox table or its counters from the host: stats, the raw-region
// hooks.  Its only late flag is the write pass's own consistency check (error
// bit 2: the handle is poisoned).
static int flush_m2(gvs_handle* h) {
  bool any = false;
  for (auto& e : h->eng) {
    if (!e.m2_pending) continue;
    hipLaunchKernelGGL(k_m2x<false>, dim3(e.Q), dim3(256), (e.cm + 1) * sizeof(GroupM) + e.Sr * sizeof(uint4),
                       h->stream, e.m2_args);
    e.m2_pending = false;
    any = true;
  }
  if (!any) return GVS_OK;
  GVS_HIP(h, hipGetLastError());
  if (!h->err_pin) GVS_HIP(h, hipHostMalloc((void**)&h->err_pin, sizeof(uint32_t), hipHostMallocDefault));
  GVS_HIP(h, hipMemcpyAsync(h->err_pin, &h->eng[0].scal->error, sizeof(uint32_t), hipMemcpyDeviceToHost,
                            h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return decode_error(h, *h->err_pin);
}

static int check_epoch(gvs_handle* h) {
  if (h->auth && h->eng[0].epoch >= kEpochLimit) {
    h->err = "storage epoch exhausted: rebuild the store under a fresh secret_key";
    return GVS_ERR_EPOCH_EXHAUSTED;
  }
  return GVS_OK;
}

static uint32_t max_submit(const gvs_handle* h) {
  // sharded: the expiry deletes have their own slots past the routed ones
  return h->mode == kSingle ? h->Bsub - h->eng[0].X : h->Bsub * (h->mode == kLocal ? h->S : 1u);
}


// ------------------------------------------- block store (gvs_oram_*, gvs_kv.h)

// A table of N 1 KiB blocks with the message table's layout and pass; no
// mailboxes, free ring or expiry.
static int kv_engine_init(gvs_handle* h, Engine& e, uint64_t N, uint32_t B) {
  e.N = N;
  e.B = B;
  e.nblk = B / 1024;
  uint64_t S = N / 4096;
  if (S < (uint64_t)kTile) S = kTile;
  if (S > (uint64_t)kRowsMax) S = kRowsMax;
  if (S > N) S = N;
  e.S = (uint32_t)S;
  e.W = (uint32_t)(N / S);
  e.c = txn_slots(B, e.W, e.S);
  // the sealed map's key pass holds the AES tables in LDS and a partition's
  // directory entries in registers: fewer group slots and rows (gvs_omap.h)
  if (h->kind == 2 && h->auth && (e.c > kOkeySealedSlots || e.S > kOkeySealedRows)) return GVS_ERR_INVALID_ARG;
  const uint64_t WC = (uint64_t)e.W * e.c;
#define A(ptr, n)                                     \
  do {                                                \
    if (int r_ = dalloc_t(h, &e.ptr, (n))) return r_; \
  } while (0)
  A(table, N * 64);
  A(scal, 1);
  A(img, (uint64_t)B * 64);
  A(kvmeta, (uint64_t)B * 8);
  A(kvdummy, (uint64_t)B * 64);
  A(rkeys, B);
  A(rpos, B);
  for (int k = 0; k < 2; ++k) A(tbuf[k], (WC + B) * 8);
  A(snap, WC * 64);
  A(snapp, (uint64_t)B * 64);
  if (h->auth) A(pbuf, (uint64_t)B * 64);  // sealed P (plain final states go to PS)
  A(psd, (uint64_t)B * 8);
  A(ps, (WC + B) * (h->auth ? 72 : 64));  // W*c slots + B sink lines (AUTH: then their side-entry lines)
  A(snapid, WC * 8);
  A(snapidp, (uint64_t)B * 8);
  A(dryb, (uint64_t)e.W * 256);
  A(rtx_agg, B / kScanT);
  A(rtx_carry, B / kScanT);
  const uint64_t nvb = B / kVBlk, nvb2 = (nvb + 63) / 64;
  A(vagg, nvb * kVLineU4);
  A(vcarry, nvb * kVLineU4);
  A(vagg2, nvb2 * kVLineU4);
  A(vcarry2, nvb2 * kVLineU4);
  if (h->auth) {
    A(mtag, N);
    A(ptag, B);
  }
  if (h->kind == 2) {  // key-value map: key directory, key sort, group slots
    A(kdir, N * 2);
    if (h->auth) A(ktag, N / 32);
    A(okeys, B);
    A(opr, (uint64_t)B * 8);
    A(opos, B);
    A(ogt, (WC + B) * 8);
    A(ogp, ((uint64_t)B + WC) * 8);
    A(ogt_agg, B / kScanT);
    A(ogt_carry, B / kScanT);
    A(orow_agg, B / kScanT);
    A(orow_carry, B / kScanT);
    A(resp, (uint64_t)B * kSlotU4);
  }
#undef A
  hipStream_t s = h->stream;
  GVS_HIP(h, hipMemsetAsync(e.table, 0, N * 1024, s));
  if (h->kind == 2) {
    GVS_HIP(h, hipMemsetAsync(e.kdir, 0, N * 32, s));
    GVS_HIP(h, hipMemsetAsync(e.ogt, 0, (WC + B) * 128, s));
  }
  for (int k = 0; k < 2; ++k) GVS_HIP(h, hipMemsetAsync(e.tbuf[k], 0, (WC + B) * 128, s));
  GVS_HIP(h, hipMemsetAsync(e.scal, 0, sizeof(Scal), s));
  GVS_HIP(h, hipMemsetAsync(e.rkeys, 0xFF, (uint64_t)B * 8, s));  // null rows until written
  if (h->auth) {  // every block starts as a sealed all-zero row at epoch 0
    e.epoch = 0;
    hipLaunchKernelGGL(k_seal_init, dim3(1024), dim3(256), 0, s, seal_of(h, e), (const uint32_t*)h->te,
                       e.table, e.mtag, (uint4*)nullptr, 0u, N);
    if (h->kind == 2)  // the map's key directory: sealed rows of 32 entries
      hipLaunchKernelGGL(k_kdir_seal_init, dim3(1024), dim3(256), 0, s, seal_of(h, e), (const uint32_t*)h->te,
                         e.kdir, e.ktag, N / 32);
    GVS_HIP(h, hipGetLastError());
  }
  GVS_HIP(h, hipStreamSynchronize(s));
  return GVS_OK;
}

// One block-store batch: n ops (gvs_block_op) at d_in, the blocks they saw
// (n x 1 KiB) to d_out.
static int oram_batch(gvs_handle* h, Engine& e, const uint4* d_in, uint32_t n, uint4* d_out) {
  hipStream_t s = h->stream;
  const uint32_t B = e.B;
  h->n_marks = 0;
  mark(h, "start");
  if (int r = reset_errors(h)) return r;
  e.stamp_run = e.stamp_next++;
  if (e.stamp_next == kNone) e.stamp_next = 1;
  {
    BcopyArgs a{d_in, e.img, e.kvmeta, e.rkeys, e.scal, e.N, n, B, e.W, e.S};
    hipLaunchKernelGGL(k_bcopy, dim3(B / 256), dim3(256), 0, s, a);
  }
  mark(h, "copy");
  if (int r = sort_keys<uint64_t, 1>(h, e.rkeys, B)) return r;
  mark(h, "sort_r");
  {
    RtxArgs a{e.rkeys, e.rpos, e.tbuf[e.par], e.rtx_agg, e.rtx_carry, e.scal,
              B,       e.W,    e.S,           e.c,       B / kScanT,  e.stamp_run};
    hipLaunchKernelGGL(k_scan_a<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<RtxOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  launch_sjoint(h, e);
  mark(h, "rtx");
  launch_rpass2(h, e);
  mark(h, "rpass");
  {
    KvArgs a{};
    vscan_fields(a, e);
    a.rpos = e.rpos;
    a.meta = e.kvmeta;
    a.img = e.img;
    a.snapp = e.snapp;
    a.pbuf = e.pbuf;
    a.psd = e.psd;
    a.ps = h->auth ? nullptr : e.ps;
    a.psink = h->auth ? e.pbuf : e.ps + (uint64_t)e.W * e.c * 64;  // non-last states (plain: PS's sink lines)
    a.out = d_out;
    a.outdummy = e.kvdummy;
    a.n = n;
    a.S = e.S;
    a.omap = 0;
    vscan_abc<KvOp>(s, a);
    hipLaunchKernelGGL(k_kv_c, dim3(a.nvb), dim3(256), 0, s, a);
  }
  if (h->auth)  // P at the epoch the pass wrote the rows at
    hipLaunchKernelGGL(k_pseal<true>, dim3(B / 64), dim3(256), 0, s, pargs(h, e, e.epoch + 1));
  mark(h, "kv");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

struct gvs_oram {
  gvs_handle* h = nullptr;
};

// One key-value batch: n ops (gvs_omap_op) at d_in, results (gvs_omap_result)
// to d_out (gvs_omap.h).
static int omap_batch(gvs_handle* h, Engine& e, const uint4* d_in, uint32_t n, uint4* d_out) {
  hipStream_t s = h->stream;
  const uint32_t B = e.B;
  h->n_marks = 0;
  mark(h, "start");
  if (int r = reset_errors(h)) return r;
  e.stamp_run = e.stamp_next++;
  if (e.stamp_next == kNone) e.stamp_next = 1;
  {
    OcopyArgs a{d_in, e.img, e.kvmeta, e.okeys, e.scal, e.kc, n, B};
    hipLaunchKernelGGL(k_ocopy, dim3(B / 256), dim3(256), 0, s, a);
  }
  mark(h, "copy");
  if (int r = sort_keys<Key128, 1>(h, e.okeys, B)) return r;
  hipLaunchKernelGGL(k_ogather, dim3(B / 256), dim3(256), 0, s, OposArgs{e.okeys, e.kvmeta, e.opr, B});
  mark(h, "sort_k");
  {
    OgtArgs a{e.opr, e.opos, e.ogt, e.ogt_agg, e.ogt_carry, e.scal, B, e.W, log2u(e.W), e.c,
              B / kScanT, e.stamp_run};
    hipLaunchKernelGGL(k_scan_a<OgtOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<OgtOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<OgtOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  mark(h, "groups");
  {
    OkeyArgs a{e.ogt, e.kdir, e.ogp, e.scal, e.W, e.S, e.c, B, e.stamp_run};
    if (h->auth) {
      a.sc = seal_of(h, e);
      a.te = h->te;
      a.ktag = e.ktag;
      hipLaunchKernelGGL(k_okey<true>, dim3(e.W), dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL(k_okey<false>, dim3(e.W), dim3(256), 0, s, a);
    }
  }
  mark(h, "keys");
  {
    OrowArgs a{e.opos, e.opr, e.ogp, e.rkeys, e.kvmeta, e.orow_agg, e.orow_carry, e.scal, B, B / kScanT};
    hipLaunchKernelGGL(k_scan_a<OrowOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<OrowOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<OrowOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  mark(h, "rows");
  if (int r = sort_keys<uint64_t, 1>(h, e.rkeys, B)) return r;
  mark(h, "sort_r");
  {
    RtxArgs a{e.rkeys, e.rpos, e.tbuf[e.par], e.rtx_agg, e.rtx_carry, e.scal,
              B,       e.W,    e.S,           e.c,       B / kScanT,  e.stamp_run};
    hipLaunchKernelGGL(k_scan_a<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_b<RtxOp>, dim3(1), dim3(kScanT), 0, s, a);
    hipLaunchKernelGGL(k_scan_c<RtxOp>, dim3(B / kScanT), dim3(kScanT), 0, s, a);
  }
  launch_sjoint(h, e);
  mark(h, "rtx");
  launch_rpass2(h, e);
  mark(h, "rpass");
  {
    KvArgs a{};
    vscan_fields(a, e);
    a.rpos = e.rpos;
    a.meta = e.kvmeta;
    a.img = e.img;
    a.snapp = e.snapp;
    a.pbuf = e.pbuf;
    a.psd = e.psd;
    a.ps = h->auth ? nullptr : e.ps;
    a.psink = h->auth ? e.pbuf : e.ps + (uint64_t)e.W * e.c * 64;  // non-last states (plain: PS's sink lines)
    a.out = e.resp;
    a.outdummy = e.kvdummy;
    a.n = n;
    a.S = e.S;
    a.omap = 1;
    vscan_abc<KvOp>(s, a);
    hipLaunchKernelGGL(k_kv_c, dim3(a.nvb), dim3(256), 0, s, a);
  }
  if (h->auth)  // P at the epoch the pass wrote the rows at
    hipLaunchKernelGGL(k_pseal<true>, dim3(B / 64), dim3(256), 0, s, pargs(h, e, e.epoch + 1));
  if (d_out && n)
    hipLaunchKernelGGL(k_out, dim3((n + 4 * kCopyPerWave - 1) / (4 * kCopyPerWave)), dim3(256), 0, s,
                       (const uint4*)e.resp, n, d_out);
  mark(h, "kv");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

struct gvs_omap {
  gvs_handle* h = nullptr;
};

// ------------------------------------------------------------------ C ABI

extern "C" {

const char* gvs_version(void) { return "gvstore 0.2.0 (gfx950)"; }

int gvs_config_init(gvs_config* cfg, uint64_t msg_capacity) {
  if (!cfg || !is_pow2(msg_capacity) || msg_capacity < 256) return GVS_ERR_INVALID_ARG;
  std::memset(cfg, 0, sizeof *cfg);
  cfg->msg_capacity = msg_capacity;
  uint64_t R = msg_capacity / 16 < 256 ? 256 : msg_capacity / 16;  // R = N/16
  cfg->mailbox_partition_slots = 256;
  cfg->mailbox_partitions = (uint32_t)(R / 256);
  cfg->max_batch = msg_capacity < 65536 ? 4096 : 65536;
  for (int i = 0; i < 32; ++i) cfg->secret_key[i] = (uint8_t)(0x67 + 31 * i);
  return GVS_OK;
}

int gvs_destroy(gvs_handle* h) {
  if (!h) return GVS_ERR_INVALID_ARG;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  HostPipe& hp = h->pipe;
  if (hp.copy) (void)hipStreamSynchronize(hp.copy);
  if (hp.copy_out) (void)hipStreamSynchronize(hp.copy_out);
  for (int b = 0; b < 2; ++b) {
    if (hp.hin[b]) (void)hipHostFree(hp.hin[b]);
    if (hp.hout[b]) (void)hipHostFree(hp.hout[b]);
    for (hipEvent_t ev : {hp.h2d[b], hp.done[b], hp.d2h[b]})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (hp.herr) (void)hipHostFree(hp.herr);
  if (hp.errs) (void)hipHostFree(hp.errs);
  for (void* q : h->bounce.buf)
    if (q) (void)hipHostFree(q);
  if (h->sr_dev) (void)hipFree(h->sr_dev);
  if (h->err_pin) (void)hipHostFree(h->err_pin);
  WirePipe& wp = h->wpipe;
  for (int b = 0; b < 2; ++b) {
    for (void* q : {(void*)wp.hin[b], (void*)wp.hout[b], (void*)wp.hchal[b], (void*)wp.hlens[b],
                    (void*)wp.holens[b], (void*)wp.hstat[b], (void*)wp.htimes[b]})
      if (q) (void)hipHostFree(q);
    for (hipEvent_t ev : {wp.h2d[b], wp.done[b], wp.d2h[b]})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (hp.copy) (void)hipStreamDestroy(hp.copy);
  if (hp.copy_out) (void)hipStreamDestroy(hp.copy_out);
  for (void* p : h->allocs) (void)hipFree(p);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return GVS_OK;
}

int gvs_create(const gvs_config* cfg, gvs_handle** out) {
  if (!cfg) return GVS_ERR_INVALID_ARG;
  return create_common(cfg, cfg->shard_count > 1 ? kLocal : kSingle, nullptr, out);
}

int gvs_comm_unique_id(uint8_t out[GVS_COMM_ID_BYTES]) {
  if (!out) return GVS_ERR_INVALID_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return GVS_ERR_DEVICE;
  std::memcpy(out, &id, sizeof id);
  return GVS_OK;
}

int gvs_create_sharded(const gvs_config* cfg, const uint8_t comm_id[GVS_COMM_ID_BYTES],
                       gvs_handle** out) {
  if (!cfg || !comm_id || cfg->shard_count < 1) return GVS_ERR_INVALID_ARG;
  return create_common(cfg, kRccl, comm_id, out);
}

static int h2d(gvs_handle* h, int slot, void* dst, const void* src, size_t bytes);
static int d2h(gvs_handle* h, int slot, void* dst, const void* src, size_t bytes);
static int bounce_done(gvs_handle* h, int rc);
static int bounce_begin(gvs_handle* h);

int gvs_process_batch(gvs_handle* h, const gvs_request* reqs, uint32_t n, gvs_response* out) {
  if (!h || (!reqs && n) || (!out && n) || n > max_submit(h)) return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = bounce_begin(h)) return r;
  if (int r = h2d(h, 0, h->in_stage, reqs, (size_t)n * sizeof(gvs_request))) return r;
  if (int r = run_batch(h, h->in_stage, n, h->out_stage)) return r;
  if (int r = d2h(h, 4, out, h->out_stage, (size_t)n * sizeof(gvs_response))) return r;
  return bounce_done(h, finish(h));
}

// memcpy over up to 8 host threads (pinned staging of 64K-request batches:
// one thread moves ~10 GB/s, too slow to hide behind a ~7 ms batch)
static void par_memcpy(void* dst, const void* src, size_t bytes) {
  const size_t kMin = 4u << 20;
  unsigned nt = std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency()));
  if (bytes < 2 * kMin || nt < 2) {
    std::memcpy(dst, src, bytes);
    return;
  }
  nt = (unsigned)std::min<size_t>(nt, bytes / kMin);
  const size_t chunk = (bytes + nt - 1) / nt;
  std::vector<std::thread> th;
  for (unsigned k = 1; k < nt; ++k) {
    const size_t o = k * chunk, len = std::min(chunk, bytes - std::min(bytes, o));
    if (len)
      th.emplace_back([=] { std::memcpy((uint8_t*)dst + o, (const uint8_t*)src + o, len); });
  }
  std::memcpy(dst, src, std::min(chunk, bytes));
  for (auto& t : th) t.join();
}

// host memory the device can copy from directly (hipHostMalloc'd, e.g. by
// gvs_host_alloc, or registered)
static bool is_pinned(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error for the caller
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

// at the entry of a call that uses the bounce slots: wait for the copies of an
// earlier call that ended on an error path (its slots may still be read or
// written by the stream) before any slot is rewritten or freed.  Within one
// call every slot is used once, so a call's own copies never wait here.
static int bounce_begin(gvs_handle* h) {
  h->bounce.pend.clear();
  if (!h->bounce.inflight) return GVS_OK;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  h->bounce.inflight = false;
  return GVS_OK;
}

static int bounce_grow(gvs_handle* h, int slot, size_t bytes) {
  Bounce& b = h->bounce;
  if (b.cap[slot] >= bytes) return GVS_OK;
  if (b.buf[slot]) GVS_HIP(h, hipHostFree(b.buf[slot]));
  b.buf[slot] = nullptr;
  b.cap[slot] = 0;
  const size_t cap = std::max<size_t>(bytes, 1u << 20);
  GVS_HIP(h, hipHostMalloc(&b.buf[slot], cap, hipHostMallocDefault));
  b.cap[slot] = cap;
  return GVS_OK;
}

// host -> device from caller memory `src`: pinned memory is copied from
// directly, pageable memory through bounce slot `slot` (0..3)
static int h2d(gvs_handle* h, int slot, void* dst, const void* src, size_t bytes) {
  if (!bytes) return GVS_OK;
  if (!is_pinned(src)) {
    if (int r = bounce_grow(h, slot, bytes)) return r;
    par_memcpy(h->bounce.buf[slot], src, bytes);
    src = h->bounce.buf[slot];
    h->bounce.inflight = true;
  }
  GVS_HIP(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, h->stream));
  return GVS_OK;
}

// device -> host into caller memory `dst`: pageable memory through bounce
// slot `slot` (4..7), handed over by bounce_done after the stream's sync
static int d2h(gvs_handle* h, int slot, void* dst, const void* src, size_t bytes) {
  if (!bytes) return GVS_OK;
  if (is_pinned(dst)) {
    GVS_HIP(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
    return GVS_OK;
  }
  if (int r = bounce_grow(h, slot, bytes)) return r;
  GVS_HIP(h, hipMemcpyAsync(h->bounce.buf[slot], src, bytes, hipMemcpyDeviceToHost, h->stream));
  h->bounce.inflight = true;
  h->bounce.pend.push_back(Bounce::Out{dst, slot, bytes});
  return GVS_OK;
}

// after the call's stream sync (finish): the pageable outputs, on success
static int bounce_done(gvs_handle* h, int rc) {
  if (rc == GVS_OK) h->bounce.inflight = false;  // finish() synchronised the stream
  if (rc == GVS_OK)
    for (const auto& o : h->bounce.pend) par_memcpy(o.dst, h->bounce.buf[o.slot], o.bytes);
  h->bounce.pend.clear();
  return rc;
}

int gvs_host_alloc(gvs_handle* h, size_t bytes, void** out) {
  if (!h || !out || !bytes) return GVS_ERR_INVALID_ARG;
  *out = nullptr;
  GVS_HIP(h, hipSetDevice(h->device));
  GVS_HIP(h, hipHostMalloc(out, bytes, hipHostMallocDefault));
  return GVS_OK;
}

int gvs_host_free(gvs_handle* h, void* p) {
  if (!h) return GVS_ERR_INVALID_ARG;
  if (p) GVS_HIP(h, hipHostFree(p));
  return GVS_OK;
}

static int pipe_init(gvs_handle* h) {
  HostPipe& p = h->pipe;
  if (p.ready) return GVS_OK;
  const uint64_t cap = (uint64_t)h->Bsub * (h->mode == kLocal ? h->S : 1u);
  for (int b = 0; b < 2; ++b) {
    if (int rc = dalloc_t(h, &p.din[b], cap * kAbiU4)) return rc;
    if (int rc = dalloc_t(h, &p.dout[b], cap * kAbiU4)) return rc;
    GVS_HIP(h, hipHostMalloc((void**)&p.hin[b], cap * sizeof(gvs_request), hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.hout[b], cap * sizeof(gvs_response), hipHostMallocDefault));
    GVS_HIP(h, hipEventCreateWithFlags(&p.h2d[b], hipEventDisableTiming));
    GVS_HIP(h, hipEventCreateWithFlags(&p.done[b], hipEventDisableTiming));
    GVS_HIP(h, hipEventCreateWithFlags(&p.d2h[b], hipEventDisableTiming));
  }
  GVS_HIP(h, hipHostMalloc((void**)&p.herr, 2 * sizeof(uint32_t), hipHostMallocDefault));
  GVS_HIP(h, hipStreamCreateWithFlags(&p.copy, hipStreamNonBlocking));
  GVS_HIP(h, hipStreamCreateWithFlags(&p.copy_out, hipStreamNonBlocking));
  p.ready = true;
  return GVS_OK;
}

// k batches from host memory, double-buffered: batch t+1's requests are
// staged and copied in, and batch t-1's responses copied out, while batch t
// runs.  Batches apply in order; the error word is not reset between them,
// so after a failed batch the following ones enqueued behind it do nothing,
// and the host state is rolled back to the failed batch.
int gvs_process_batches(gvs_handle* h, const gvs_request* reqs, const uint32_t* counts,
                        uint32_t k, gvs_response* out, uint32_t* applied) {
  if (applied) *applied = 0;
  if (!h || h->kind != 0 || (k && (!counts || !reqs || !out))) return GVS_ERR_INVALID_ARG;
  for (uint32_t t = 0; t < k; ++t)
    if (counts[t] > max_submit(h)) return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (k == 0) return GVS_OK;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = pipe_init(h)) return r;
  HostPipe& p = h->pipe;
  hipStream_t s = h->stream;
  if (int r = reset_errors(h)) return r;
  // Caller buffers in pinned memory (gvs_host_alloc) are copied to and from
  // directly; pageable ones go through the pinned staging pair.
  const bool pin_in = is_pinned(reqs), pin_out = is_pinned(out);
  HostState snap[2];
  uint64_t off[2] = {0, 0};
  uint64_t next_off = 0;
  uint32_t enq = 0;  // batches enqueued
  int stop = GVS_OK;
  for (uint32_t t = 0;; ++t) {
    bool more = t < k && stop == GVS_OK;
    if (more)
      if (int r = check_epoch(h)) {
        stop = r;
        more = false;
      }
    if (more) {  // enqueue batch t in slot b
      const uint32_t b = t & 1u, n = counts[t];
      const void* src = reqs + next_off;
      if (!pin_in) {
        if (t >= 2) GVS_HIP(h, hipEventSynchronize(p.h2d[b]));  // hin[b] free again
        par_memcpy(p.hin[b], reqs + next_off, (size_t)n * sizeof(gvs_request));
        src = p.hin[b];
      }
      if (t >= 2) GVS_HIP(h, hipStreamWaitEvent(p.copy, p.done[b], 0));  // din[b] consumed
      if (n)
        GVS_HIP(h, hipMemcpyAsync(p.din[b], src, (size_t)n * sizeof(gvs_request),
                                  hipMemcpyHostToDevice, p.copy));
      GVS_HIP(h, hipEventRecord(p.h2d[b], p.copy));
      GVS_HIP(h, hipStreamWaitEvent(s, p.h2d[b], 0));
      if (t >= 2) GVS_HIP(h, hipStreamWaitEvent(s, p.d2h[b], 0));  // dout[b] copied out
      snap[b] = save_state(h);
      int rr = run_batch(h, p.din[b], n, p.dout[b], false);
      if (!rr && h->mode != kSingle) rr = agree_errors(h);
      if (rr) {  // batch t was not (wholly) enqueued: the ones before it are still collected
        restore_state(h, snap[b]);
        stop = rr;
        more = false;
      }
    }
    if (more) {
      const uint32_t b = t & 1u, n = counts[t];
      GVS_HIP(h, hipMemcpyAsync(&p.herr[b], &h->eng[0].scal->error, sizeof(uint32_t),
                                hipMemcpyDeviceToHost, s));
      GVS_HIP(h, hipEventRecord(p.done[b], s));
      GVS_HIP(h, hipStreamWaitEvent(p.copy_out, p.done[b], 0));
      if (n)
        GVS_HIP(h, hipMemcpyAsync(pin_out ? (void*)(out + next_off) : (void*)p.hout[b], p.dout[b],
                                  (size_t)n * sizeof(gvs_response), hipMemcpyDeviceToHost, p.copy_out));
      GVS_HIP(h, hipEventRecord(p.d2h[b], p.copy_out));
      advance(h);  // as if applied; rolled back below if it was not
      off[b] = next_off;
      next_off += n;
      enq = t + 1;
    }
    if (t >= 1 && t - 1 < enq) {  // collect batch t-1
      const uint32_t pb = (t - 1) & 1u;
      GVS_HIP(h, hipEventSynchronize(p.d2h[pb]));
      if (const uint32_t e = p.herr[pb]) {
        restore_state(h, snap[pb]);
        GVS_HIP(h, hipStreamSynchronize(s));  // batch t, if enqueued, did nothing
        GVS_HIP(h, hipStreamSynchronize(p.copy));
        GVS_HIP(h, hipStreamSynchronize(p.copy_out));
        // the batches from the failed one on were not applied: their range of
        // `out` (which a pinned caller buffer may have received stale device
        // responses into) is zeroed, never left holding other batches' data
        uint64_t total = 0;
        for (uint32_t i = 0; i < k; ++i) total += counts[i];
        std::memset(out + off[pb], 0, (size_t)(total - off[pb]) * sizeof(gvs_response));
        return decode_error(h, e);
      }
      if (!pin_out)
        par_memcpy(out + off[pb], p.hout[pb], (size_t)counts[t - 1] * sizeof(gvs_response));
      if (applied) *applied = t;
    }
    if (!more && t >= enq) break;
  }
  if (stop != GVS_OK) {  // the batches not applied answer nothing
    uint64_t total = 0;
    for (uint32_t i = 0; i < k; ++i) total += counts[i];
    GVS_HIP(h, hipStreamSynchronize(p.copy_out));
    std::memset(out + next_off, 0, (size_t)(total - next_off) * sizeof(gvs_response));
  }
  return stop;
}

int gvs_process_batches_device(gvs_handle* h, const void* d_reqs, const uint32_t* counts, uint32_t k,
                               void* d_out, uint32_t* applied) {
  if (applied) *applied = 0;
  if (!h || h->kind != 0 || (k && (!counts || !d_reqs || !d_out))) return GVS_ERR_INVALID_ARG;
  for (uint32_t t = 0; t < k; ++t)
    if (counts[t] > max_submit(h)) return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (k == 0) return GVS_OK;
  GVS_HIP(h, hipSetDevice(h->device));
  HostPipe& p = h->pipe;  // pinned error words, one per batch
  if (k > p.nerr) {
    if (p.errs) (void)hipHostFree(p.errs);
    p.errs = nullptr;
    p.nerr = 0;
    GVS_HIP(h, hipHostMalloc((void**)&p.errs, (size_t)k * sizeof(uint32_t), hipHostMallocDefault));
    p.nerr = k;
  }
  if (int r = reset_errors(h)) return r;
  const uint4* in = (const uint4*)d_reqs;
  uint4* out = (uint4*)d_out;
  std::vector<HostState> snap(k);
  uint64_t off = 0, total = 0;
  for (uint32_t t = 0; t < k; ++t) total += counts[t];
  uint32_t enq = 0;
  int stop = GVS_OK;
  // every batch enqueued back to back; the error word is not reset between
  // them, so the batches behind a failing one do nothing
  for (uint32_t t = 0; t < k; ++t) {
    if (int r = check_epoch(h)) {
      stop = r;
      break;
    }
    snap[t] = save_state(h);
    int r = run_batch(h, in + off * kAbiU4, counts[t], out + off * kAbiU4, false);
    if (!r && h->mode != kSingle) r = agree_errors(h);
    if (r) {  // batch t was not (wholly) enqueued: the ones before it still count
      restore_state(h, snap[t]);
      stop = r;
      break;
    }
    GVS_HIP(h, hipMemcpyAsync(&p.errs[t], &h->eng[0].scal->error, sizeof(uint32_t),
                              hipMemcpyDeviceToHost, h->stream));
    advance(h);  // as if applied; rolled back below if it was not
    off += counts[t];
    enq = t + 1;
  }
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  off = 0;
  for (uint32_t t = 0; t < enq; ++t) {
    if (const uint32_t e = p.errs[t]) {
      restore_state(h, snap[t]);
      GVS_HIP(h, hipMemsetAsync(out + off * kAbiU4, 0, (size_t)(total - off) * sizeof(gvs_response),
                                h->stream));
      GVS_HIP(h, hipStreamSynchronize(h->stream));
      return decode_error(h, e);
    }
    off += counts[t];
    if (applied) *applied = t + 1;
  }
  if (stop != GVS_OK && off < total) {  // the batches not applied answer nothing
    GVS_HIP(h, hipMemsetAsync(out + off * kAbiU4, 0, (size_t)(total - off) * sizeof(gvs_response), h->stream));
    GVS_HIP(h, hipStreamSynchronize(h->stream));
  }
  return stop;
}

int gvs_process_batch_device(gvs_handle* h, const void* d_reqs, uint32_t n, void* d_out) {
  if (!h || (!d_reqs && n) || (!d_out && n) || n > max_submit(h)) return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = run_batch(h, (const uint4*)d_reqs, n, (uint4*)d_out)) return r;
  return finish(h);
}

// ------------------------------------------------------------ wire codec

static bool wire_strides_ok(uint32_t in_stride, uint32_t out_stride) {
  return in_stride >= 1 && in_stride <= kWireSlotMax && out_stride >= kWireResp &&
         out_stride <= kWireSlotMax;
}

static void enqueue_wire_decode(gvs_handle* h, const void* d_wire, uint32_t stride,
                                const uint32_t* d_lens, uint32_t n, const uint64_t* d_times,
                                void* d_reqs, void* d_sigs, uint32_t* d_status) {
  if (!n) return;
  WireDecArgs a{(const uint8_t*)d_wire, stride, n, d_lens, d_times, (uint4*)d_reqs,
                (uint4*)d_sigs, d_status};
  const uint32_t lds = wire_decode_lds(stride);
  if (lds > 65536u)  // past the default dynamic-LDS limit (kWireSlotMax strides)
    (void)hipFuncSetAttribute((const void*)k_wire_decode, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)wire_decode_lds(kWireSlotMax));
  hipLaunchKernelGGL(k_wire_decode, dim3((n + kWireMsgs - 1) / kWireMsgs), dim3(64), lds, h->stream, a);
}

static void enqueue_wire_encode(gvs_handle* h, const void* d_resps, uint32_t n, void* d_wire,
                                uint32_t stride, uint32_t* d_lens) {
  if (!n) return;
  WireEncArgs a{(const uint4*)d_resps, n, stride, (uint8_t*)d_wire, d_lens};
  hipLaunchKernelGGL(k_wire_encode, dim3((n + 3) / 4), dim3(256), 0, h->stream, a);
}

int gvs_wire_decode_device(gvs_handle* h, const void* d_wire, uint32_t stride,
                           const uint32_t* d_lens, uint32_t n, const uint64_t* d_times,
                           void* d_reqs, void* d_sigs, uint32_t* d_status) {
  if (!h || stride < 1 || stride > kWireSlotMax ||
      (n && (!d_wire || !d_lens || !d_times || !d_reqs)))
    return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipSetDevice(h->device));
  enqueue_wire_decode(h, d_wire, stride, d_lens, n, d_times, d_reqs, d_sigs, d_status);
  GVS_HIP(h, hipGetLastError());
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

int gvs_wire_encode_device(gvs_handle* h, const void* d_resps, uint32_t n, void* d_wire,
                           uint32_t stride, uint32_t* d_lens) {
  if (!h || stride < kWireResp || stride > kWireSlotMax || (n && (!d_resps || !d_wire || !d_lens)))
    return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipSetDevice(h->device));
  enqueue_wire_encode(h, d_resps, n, d_wire, stride, d_lens);
  GVS_HIP(h, hipGetLastError());
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

// grapevine's challenge signing context (types/src/lib.rs:13)
static const char kChallengeContext[] = "grapevine-challenge";

static int sr_args(const uint8_t* context, uint32_t context_len, sr::SrArgs& a) {
  if (context_len > sizeof a.ctx || (context_len && !context)) return GVS_ERR_INVALID_ARG;
  std::memset(&a, 0, sizeof a);
  if (context_len) std::memcpy(a.ctx, context, context_len);
  a.ctx_len = context_len;
  return GVS_OK;
}

static void enqueue_sr_verify(gvs_handle* h, const sr::SrArgs& a) {
  if (!a.n) return;
  hipLaunchKernelGGL(sr::k_sr_verify, dim3((a.n + sr::kSrThreads - 1) / sr::kSrThreads),
                     dim3(sr::kSrThreads), 0, h->stream, a);
}

// Handle-owned wire staging: signatures and statuses always (the device path
// may not pass them), the host-side slabs only for gvs_process_wire_batch.
static int wire_stage_init(gvs_handle* h, bool io) {
  WireStage& w = h->wire;
  const uint64_t cap = max_submit(h);
  if (!w.sigs) {
    if (int rc = dalloc_t(h, &w.sigs, cap * 4)) return rc;
    if (int rc = dalloc_t(h, &w.status, cap)) return rc;
  }
  if (io && !w.in) {
    if (int rc = dalloc_t(h, &w.in, cap * kWireSlotMax)) return rc;
    if (int rc = dalloc_t(h, &w.out, cap * kWireSlotMax)) return rc;
    if (int rc = dalloc_t(h, &w.in_lens, cap)) return rc;
    if (int rc = dalloc_t(h, &w.out_lens, cap)) return rc;
    if (int rc = dalloc_t(h, &w.times, cap)) return rc;
    if (int rc = dalloc_t(h, &w.chal, cap * 2)) return rc;
  }
  return GVS_OK;
}

// decode -> (challenge check) -> the batch -> encode, all on the engine
// stream; the request and response slabs live in the handle's host-API
// staging.  d_chal: n x 32-B challenges, or null (signatures not checked).
static int wire_batch(gvs_handle* h, const void* d_in, uint32_t in_stride, const uint32_t* d_in_lens,
                      uint32_t n, const uint64_t* d_times, const void* d_chal, void* d_out,
                      uint32_t out_stride, uint32_t* d_out_lens, void* d_sigs, uint32_t* d_status) {
  if (int rc = wire_stage_init(h, false)) return rc;
  h->n_marks = 0;
  mark(h, "start");
  uint4* sigs = d_sigs ? (uint4*)d_sigs : h->wire.sigs;
  uint32_t* status = d_status ? d_status : h->wire.status;
  enqueue_wire_decode(h, d_in, in_stride, d_in_lens, n, d_times, h->in_stage, sigs, status);
  mark(h, "wire_decode");
  if (d_chal) {
    sr::SrArgs a;
    (void)sr_args((const uint8_t*)kChallengeContext, sizeof kChallengeContext - 1, a);
    a.pk = (const uint8_t*)h->in_stage + 16;  // gvs_request.auth_identity
    a.pk_stride = sizeof(gvs_request);
    a.msg = (const uint8_t*)d_chal;
    a.msg_stride = 32;
    a.msg_len = 32;
    a.sig = (const uint8_t*)sigs;
    a.sig_stride = 64;
    a.n = n;
    a.reqs = h->in_stage;
    a.status = status;
    enqueue_sr_verify(h, a);
    mark(h, "sr_verify");
  }
  if (int r = run_batch_body(h, h->in_stage, n, h->out_stage)) return r;
  enqueue_wire_encode(h, h->out_stage, n, d_out, out_stride, d_out_lens);
  mark(h, "wire_encode");
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

int gvs_process_wire_batch_device(gvs_handle* h, const void* d_in, uint32_t in_stride,
                                  const uint32_t* d_in_lens, uint32_t n, const uint64_t* d_times,
                                  const void* d_challenges, void* d_out, uint32_t out_stride,
                                  uint32_t* d_out_lens, void* d_sigs, uint32_t* d_status) {
  if (!h || h->kind != 0 || !wire_strides_ok(in_stride, out_stride) || n > max_submit(h) ||
      (n && (!d_in || !d_in_lens || !d_times || !d_out || !d_out_lens)))
    return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = reset_errors(h)) return r;
  if (int r = wire_batch(h, d_in, in_stride, d_in_lens, n, d_times, d_challenges, d_out,
                         out_stride, d_out_lens, d_sigs, d_status))
    return r;
  return finish(h);
}

int gvs_process_wire_batch(gvs_handle* h, const uint8_t* in, uint32_t in_stride,
                           const uint32_t* in_lens, uint32_t n, const uint64_t* times,
                           const uint8_t* challenges, uint8_t* out, uint32_t out_stride,
                           uint32_t* out_lens, uint8_t* sigs, uint32_t* decode_status) {
  if (!h || h->kind != 0 || !wire_strides_ok(in_stride, out_stride) || n > max_submit(h) ||
      (n && (!in || !in_lens || !times || !out || !out_lens)))
    return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int rc = wire_stage_init(h, true)) return rc;
  WireStage& w = h->wire;
  if (int r = bounce_begin(h)) return r;
  if (n) {
    if (int r = h2d(h, 0, w.in, in, (size_t)n * in_stride)) return r;
    if (int r = h2d(h, 1, w.in_lens, in_lens, (size_t)n * 4)) return r;
    if (int r = h2d(h, 2, w.times, times, (size_t)n * 8)) return r;
    if (challenges)
      if (int r = h2d(h, 3, w.chal, challenges, (size_t)n * 32)) return r;
  }
  if (int r = reset_errors(h)) return r;
  if (int r = wire_batch(h, w.in, in_stride, w.in_lens, n, w.times, challenges ? w.chal : nullptr,
                         w.out, out_stride, w.out_lens, w.sigs, w.status))
    return r;
  if (n) {
    if (int r = d2h(h, 4, out, w.out, (size_t)n * out_stride)) return r;
    if (int r = d2h(h, 5, out_lens, w.out_lens, (size_t)n * 4)) return r;
    if (sigs)
      if (int r = d2h(h, 6, sigs, w.sigs, (size_t)n * 64)) return r;
    if (decode_status)
      if (int r = d2h(h, 7, decode_status, w.status, (size_t)n * 4)) return r;
  }
  return bounce_done(h, finish(h));
}

static int wire_pipe_init(gvs_handle* h) {
  WirePipe& p = h->wpipe;
  if (p.ready) return GVS_OK;
  if (int r = pipe_init(h)) return r;  // the copy streams and the host pipeline's pinned words
  const uint64_t cap = max_submit(h), big = cap * kWireSlotMax;
  for (int b = 0; b < 2; ++b) {
    if (int rc = dalloc_t(h, &p.din[b], big)) return rc;
    if (int rc = dalloc_t(h, &p.dout[b], big)) return rc;
    if (int rc = dalloc_t(h, &p.dlens[b], cap)) return rc;
    if (int rc = dalloc_t(h, &p.dolens[b], cap)) return rc;
    if (int rc = dalloc_t(h, &p.dstat[b], cap)) return rc;
    if (int rc = dalloc_t(h, &p.dtimes[b], cap)) return rc;
    if (int rc = dalloc_t(h, &p.dchal[b], cap * 2)) return rc;
    GVS_HIP(h, hipHostMalloc((void**)&p.hin[b], big, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.hout[b], big, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.hchal[b], cap * 32, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.hlens[b], cap * 4, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.holens[b], cap * 4, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.hstat[b], cap * 4, hipHostMallocDefault));
    GVS_HIP(h, hipHostMalloc((void**)&p.htimes[b], cap * 8, hipHostMallocDefault));
    GVS_HIP(h, hipEventCreateWithFlags(&p.h2d[b], hipEventDisableTiming));
    GVS_HIP(h, hipEventCreateWithFlags(&p.done[b], hipEventDisableTiming));
    GVS_HIP(h, hipEventCreateWithFlags(&p.d2h[b], hipEventDisableTiming));
  }
  p.ready = true;
  return GVS_OK;
}

// k wire batches from host memory, double-buffered like gvs_process_batches:
// batch t+1's messages go up on the copy stream and batch t-1's results come
// down on the other while batch t runs (decode, challenge check, the store,
// encode).  At the first batch that fails, its error is returned and it and
// the later batches are not applied.
int gvs_process_wire_batches(gvs_handle* h, const uint8_t* in, uint32_t in_stride,
                             const uint32_t* in_lens, const uint32_t* counts, uint32_t k,
                             const uint64_t* times, const uint8_t* challenges, uint8_t* out,
                             uint32_t out_stride, uint32_t* out_lens, uint32_t* decode_status,
                             uint32_t* applied) {
  if (applied) *applied = 0;
  if (!h || h->kind != 0 || !wire_strides_ok(in_stride, out_stride) ||
      (k && (!counts || !in || !in_lens || !times || !out || !out_lens)))
    return GVS_ERR_INVALID_ARG;
  for (uint32_t t = 0; t < k; ++t)
    if (counts[t] > max_submit(h)) return GVS_ERR_INVALID_ARG;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (k == 0) return GVS_OK;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = wire_pipe_init(h)) return r;
  if (int r = wire_stage_init(h, false)) return r;
  WirePipe& p = h->wpipe;
  HostPipe& hp = h->pipe;
  hipStream_t s = h->stream;
  if (int r = reset_errors(h)) return r;
  // message and response slabs in pinned memory (gvs_host_alloc) are copied
  // to and from directly; pageable ones go through the pinned staging pair
  const bool pin_in = is_pinned(in), pin_out = is_pinned(out);
  HostState snap[2];
  uint64_t off[2] = {0, 0}, next_off = 0;
  uint32_t enq = 0;
  int stop = GVS_OK;
  for (uint32_t t = 0;; ++t) {
    bool more = t < k && stop == GVS_OK;
    if (more)
      if (int r = check_epoch(h)) {
        stop = r;
        more = false;
      }
    if (more) {  // enqueue batch t in slot b
      const uint32_t b = t & 1u, n = counts[t];
      if (t >= 2) GVS_HIP(h, hipEventSynchronize(p.h2d[b]));  // staging b free again
      const uint8_t* src = pin_in ? in + next_off * in_stride : p.hin[b];
      if (!pin_in) par_memcpy(p.hin[b], in + next_off * in_stride, (size_t)n * in_stride);
      std::memcpy(p.hlens[b], in_lens + next_off, (size_t)n * 4);
      std::memcpy(p.htimes[b], times + next_off, (size_t)n * 8);
      if (challenges) std::memcpy(p.hchal[b], challenges + next_off * 32, (size_t)n * 32);
      if (t >= 2) GVS_HIP(h, hipStreamWaitEvent(hp.copy, p.done[b], 0));  // device slot b consumed
      if (n) {
        GVS_HIP(h, hipMemcpyAsync(p.din[b], src, (size_t)n * in_stride, hipMemcpyHostToDevice, hp.copy));
        GVS_HIP(h, hipMemcpyAsync(p.dlens[b], p.hlens[b], (size_t)n * 4, hipMemcpyHostToDevice, hp.copy));
        GVS_HIP(h, hipMemcpyAsync(p.dtimes[b], p.htimes[b], (size_t)n * 8, hipMemcpyHostToDevice, hp.copy));
        if (challenges)
          GVS_HIP(h, hipMemcpyAsync(p.dchal[b], p.hchal[b], (size_t)n * 32, hipMemcpyHostToDevice, hp.copy));
      }
      GVS_HIP(h, hipEventRecord(p.h2d[b], hp.copy));
      GVS_HIP(h, hipStreamWaitEvent(s, p.h2d[b], 0));
      if (t >= 2) GVS_HIP(h, hipStreamWaitEvent(s, p.d2h[b], 0));  // results b copied out
      snap[b] = save_state(h);
      if (int r = wire_batch(h, p.din[b], in_stride, p.dlens[b], n, p.dtimes[b],
                             challenges ? p.dchal[b] : nullptr, p.dout[b], out_stride, p.dolens[b],
                             nullptr, p.dstat[b]))
        return r;
      if (h->mode != kSingle)
        if (int r = agree_errors(h)) return r;
      GVS_HIP(h, hipMemcpyAsync(&hp.herr[b], &h->eng[0].scal->error, sizeof(uint32_t),
                                hipMemcpyDeviceToHost, s));
      GVS_HIP(h, hipEventRecord(p.done[b], s));
      GVS_HIP(h, hipStreamWaitEvent(hp.copy_out, p.done[b], 0));
      if (n) {
        GVS_HIP(h, hipMemcpyAsync(pin_out ? out + next_off * out_stride : p.hout[b], p.dout[b],
                                  (size_t)n * out_stride, hipMemcpyDeviceToHost, hp.copy_out));
        GVS_HIP(h, hipMemcpyAsync(p.holens[b], p.dolens[b], (size_t)n * 4, hipMemcpyDeviceToHost, hp.copy_out));
        GVS_HIP(h, hipMemcpyAsync(p.hstat[b], p.dstat[b], (size_t)n * 4, hipMemcpyDeviceToHost, hp.copy_out));
      }
      GVS_HIP(h, hipEventRecord(p.d2h[b], hp.copy_out));
      advance(h);  // as if applied; rolled back below if it was not
      off[b] = next_off;
      next_off += n;
      enq = t + 1;
    }
    if (t >= 1 && t - 1 < enq) {  // collect batch t-1
      const uint32_t pb = (t - 1) & 1u, n = counts[t - 1];
      GVS_HIP(h, hipEventSynchronize(p.d2h[pb]));
      if (const uint32_t e = hp.herr[pb]) {
        restore_state(h, snap[pb]);
        GVS_HIP(h, hipStreamSynchronize(s));
        GVS_HIP(h, hipStreamSynchronize(hp.copy));
        GVS_HIP(h, hipStreamSynchronize(hp.copy_out));
        // unapplied batches: zero their range of `out` and their lengths (a
        // pinned `out` may have received stale device responses)
        uint64_t total = 0;
        for (uint32_t i = 0; i < k; ++i) total += counts[i];
        std::memset(out + off[pb] * out_stride, 0, (size_t)(total - off[pb]) * out_stride);
        std::memset(out_lens + off[pb], 0, (size_t)(total - off[pb]) * 4);
        if (decode_status) std::memset(decode_status + off[pb], 0, (size_t)(total - off[pb]) * 4);
        return decode_error(h, e);
      }
      if (!pin_out) par_memcpy(out + off[pb] * out_stride, p.hout[pb], (size_t)n * out_stride);
      std::memcpy(out_lens + off[pb], p.holens[pb], (size_t)n * 4);
      if (decode_status) std::memcpy(decode_status + off[pb], p.hstat[pb], (size_t)n * 4);
      if (applied) *applied = t;
    }
    if (!more && t >= enq) break;
  }
  return stop;
}

int gvs_sr25519_verify_device(gvs_handle* h, const void* d_pks, uint32_t pk_stride,
                              const void* d_msgs, uint32_t msg_stride, uint32_t msg_len,
                              const void* d_sigs, uint32_t sig_stride, uint32_t n,
                              const uint8_t* context, uint32_t context_len, uint32_t* d_ok) {
  sr::SrArgs a;
  if (!h || sr_args(context, context_len, a) || pk_stride < 32 || sig_stride < 64 ||
      msg_stride < msg_len || msg_len > 4096 || (n && (!d_pks || (msg_len && !d_msgs) || !d_sigs || !d_ok)))
    return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipSetDevice(h->device));
  a.pk = (const uint8_t*)d_pks;
  a.pk_stride = pk_stride;
  a.msg = (const uint8_t*)d_msgs;
  a.msg_stride = msg_stride;
  a.msg_len = msg_len;
  a.sig = (const uint8_t*)d_sigs;
  a.sig_stride = sig_stride;
  a.n = n;
  a.ok = d_ok;
  h->n_marks = 0;
  mark(h, "start");
  enqueue_sr_verify(h, a);
  mark(h, "sr_verify");
  GVS_HIP(h, hipGetLastError());
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

int gvs_sr25519_verify(gvs_handle* h, const uint8_t* pks, const uint8_t* msgs, uint32_t msg_len,
                       const uint8_t* sigs, uint32_t n, const uint8_t* context,
                       uint32_t context_len, uint32_t* ok) {
  if (!h || (n && (!pks || (msg_len && !msgs) || !sigs || !ok)) || msg_len > 4096)
    return GVS_ERR_INVALID_ARG;
  if (!n) return GVS_OK;
  GVS_HIP(h, hipSetDevice(h->device));
  const size_t b_pk = (size_t)n * 32, b_msg = (size_t)n * msg_len, b_sig = (size_t)n * 64,
               b_ok = (size_t)n * 4;
  const size_t need = b_pk + b_msg + b_sig + b_ok + 64;
  // grow-only device staging: a hipMalloc / hipFree per call would change the
  // page tables (and invalidate the TLB) between batches
  if (h->sr_cap < need) {
    if (h->sr_dev) GVS_HIP(h, hipFree(h->sr_dev));
    h->sr_dev = nullptr;
    h->sr_cap = 0;
    GVS_HIP(h, hipMalloc((void**)&h->sr_dev, need));
    h->sr_cap = need;
  }
  uint8_t* d = h->sr_dev;
  if (int r = bounce_begin(h)) return r;
  if (int r = h2d(h, 0, d, pks, b_pk)) return r;
  if (int r = h2d(h, 1, d + b_pk, msgs, b_msg)) return r;
  if (int r = h2d(h, 2, d + b_pk + b_msg, sigs, b_sig)) return r;
  uint32_t* d_ok = (uint32_t*)(d + ((b_pk + b_msg + b_sig + 3) & ~(size_t)3));
  if (int r = gvs_sr25519_verify_device(h, d, 32, d + b_pk, msg_len ? msg_len : 1, msg_len,
                                        d + b_pk + b_msg, 64, n, context, context_len, d_ok))
    return bounce_done(h, r);
  if (int r = d2h(h, 4, ok, d_ok, b_ok)) return r;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return bounce_done(h, GVS_OK);
}

int gvs_set_expiry_cutoff(gvs_handle* h, uint64_t cutoff) {
  if (!h) return GVS_ERR_INVALID_ARG;
  h->cutoff = cutoff;
  return GVS_OK;
}

int gvs_access(gvs_handle* h, const gvs_request* req, gvs_response* out) {
  return gvs_process_batch(h, req, 1, out);
}

int gvs_get_stats(gvs_handle* h, gvs_stats* out) {
  if (!h || !out) return GVS_ERR_INVALID_ARG;
  if (int r = flush_m2(h)) return r;
  std::memset(out, 0, sizeof *out);
  for (auto& e : h->eng) {
    Scal sc{};
    GVS_HIP(h, hipMemcpyAsync(&sc, e.scal, sizeof sc, hipMemcpyDeviceToHost, h->stream));
    GVS_HIP(h, hipStreamSynchronize(h->stream));
    out->messages += sc.count;
    out->mailboxes += sc.n_mailboxes;
    out->batches = sc.batches;
    out->creation_counter += sc.ctr;
    out->free_ring_head += sc.head;
    out->free_ring_tail += sc.tail;
  }
  out->msg_partitions = h->eng[0].W;
  out->msg_partition_slots = h->eng[0].S;
  out->shards = h->eng.size();
  out->route_capacity = h->C;
  out->shard_batch = h->Be;
  out->epoch = h->eng[0].epoch;
  return GVS_OK;
}

int gvs_synchronize(gvs_handle* h) {
  if (!h) return GVS_ERR_INVALID_ARG;
  if (int r = flush_m2(h)) return r;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

int gvs_set_timing(gvs_handle* h, int on) {
  if (!h) return GVS_ERR_INVALID_ARG;
  h->timed = on != 0;
  return GVS_OK;
}

int gvs_get_option(gvs_handle* h, const char* key, int64_t* value) {
  if (!h || !key || !value) return GVS_ERR_INVALID_ARG;
  const Engine& e = h->eng[0];
  if (std::strcmp(key, "txn_slots") == 0) *value = e.c;
  else if (std::strcmp(key, "group_slots") == 0) *value = e.cm;
  else if (std::strcmp(key, "fixed_schedule_pass") == 0)
    // 1: the message-table pass stages every slot line in LDS and runs the same
    // memory schedule whatever the batch holds (k_rpass2s, or k_spass<NW, true>
    // sealed); 0: more transaction slots than LDS stages (c above kStageSlots /
    // kSpSlots, i.e. B / W large), and the slot lines are read in the stream
    *value = h->auth ? (sealed_staged(e) ? 1 : 0) : ((e.c <= kStageSlots && e.S % (16 * 8) == 0) ? 1 : 0);
  else if (std::strcmp(key, "rccl_ranks") == 0) {
    // the store's own communicator (0 without one): what the data path spans
    int n = 0;
    if (h->comm && ncclCommCount(h->comm, &n) != ncclSuccess) return GVS_ERR_DEVICE;
    *value = n;
  } else if (std::strcmp(key, "rccl_rank") == 0) {
    int r = -1;
    if (h->comm && ncclCommUserRank(h->comm, &r) != ncclSuccess) return GVS_ERR_DEVICE;
    *value = r;
  } else return GVS_ERR_INVALID_ARG;
  return GVS_OK;
}

int gvs_set_option(gvs_handle* h, const char* key, int64_t value) {
  if (!h || !key) return GVS_ERR_INVALID_ARG;
  if (std::strcmp(key, "sealed_pass_waves") == 0 && (value == 0 || value == 4 || value == 8 || value == 12)) {
    h->sealed_nw = (int)value;
    return GVS_OK;
  }
  return GVS_ERR_INVALID_ARG;
}

// stage i = time from mark i to mark i+1; names are the later mark's
int gvs_last_timings(gvs_handle* h, const char** names, float* ms, int cap) {
  if (!h) return GVS_ERR_INVALID_ARG;
  if (!h->timed) return 0;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  int c = 0;
  for (int i = 0; i + 1 < h->n_marks && c < cap; ++i, ++c) {
    float t = 0.f;
    (void)hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]);
    if (names) names[c] = h->mark_name[i + 1];
    if (ms) ms[c] = t;
  }
  return c;
}

const char* gvs_last_error(gvs_handle* h) { return h ? h->err.c_str() : "null handle"; }

int gvs_storage_seal_row(const uint8_t secret[32], uint32_t table, uint64_t row, uint32_t epoch,
                         const uint8_t pt[1024], const uint8_t* side_pt, uint8_t ct[1024],
                         uint8_t* side_ct, uint8_t tag[16]) {
  const bool known = table <= 2 || table == kPendTable;
  if (!secret || !pt || !ct || !tag || !known || (side_pt && !side_ct)) return GVS_ERR_INVALID_ARG;
  SealCtx sc{};
  uint32_t te0[256], nh[kNhWords];
  storage_ctx(secret, sc, te0, nh);
  auto xor_block = [&](const uint8_t* src, uint8_t* dst, uint32_t j) {
    const uint4 k = ctr_keystream(sc.rk, te0, table, row, epoch, j);
    const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
    for (int b = 0; b < 16; ++b) dst[b] = (uint8_t)(src[b] ^ (kw[b / 4] >> (8 * (b % 4))));
  };
  for (uint32_t j = 0; j < 64; ++j) xor_block(pt + 16 * j, ct + 16 * j, j);
  uint64_t sd[2] = {0, 0};
  if (side_pt) {
    xor_block(side_pt, side_ct, 64);
    sd[0] = ld64(side_ct);
    sd[1] = ld64(side_ct + 8);
  }
  uint64_t t[2];
  head_aes(sc.rkh, te0, row, epoch, table, side_pt ? sd : nullptr, t);
  {  // the row hash (every table this function seals), leaf by leaf as the kernels do
    uint64_t sum[4] = {0, 0, 0, 0}, g[2];
    for (uint32_t i = 0; i < 8; ++i) {
      uint32_t w[32];
      for (uint32_t k = 0; k < 32; ++k) {
        const uint8_t* q = ct + 128 * i + 4 * k;
        w[k] = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
      }
      nh_words(nh, 32 * i, w, sum);
    }
    row_hash_fin(sum, sc.l3k, sc.l3p, g);
    t[0] ^= g[0];
    t[1] ^= g[1];
  }
  for (int b = 0; b < 16; ++b) tag[b] = (uint8_t)(t[b / 8] >> (8 * (b % 8)));
  return GVS_OK;
}

#ifdef GVS_TEST_HOOKS
int gvs_dump_messages(gvs_handle* h, void* host_dst, uint64_t bytes) {
  if (!h || !host_dst) return GVS_ERR_INVALID_ARG;
  const uint64_t N = h->eng[0].N;
  if (bytes < N * 1024 * h->eng.size()) return GVS_ERR_INVALID_ARG;
  std::vector<uint8_t> phys(N * 1024);
  uint8_t* dst = (uint8_t*)host_dst;
  std::vector<uint32_t> te0(256);
  SealCtx sc{};
  uint32_t nh_unused[kNhWords];
  if (h->auth) storage_ctx(h->cfg.secret_key, sc, te0.data(), nh_unused);
  for (const auto& e : h->eng) {
    GVS_HIP(h, hipMemcpyAsync(phys.data(), e.table, phys.size(), hipMemcpyDeviceToHost, h->stream));
    GVS_HIP(h, hipStreamSynchronize(h->stream));
    auto unseal = [&](uint8_t* d, uint32_t table, uint64_t row) {  // decrypt at the current epoch
      for (uint32_t j = 0; j < 64; ++j) {
        const uint4 k = ctr_keystream(sc.rk, te0.data(), table, row, e.epoch, j);
        const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
        for (int b = 0; b < 16; ++b) d[16 * j + b] ^= (uint8_t)(kw[b / 4] >> (8 * (b % 4)));
      }
    };
    if (h->auth) {  // sealed rows in the tile layout (gvs_seal_dev.h tile_unit)
      std::vector<uint8_t> t(phys);
      for (uint64_t row = 0; row < N; ++row)
        for (uint32_t b = 0; b < 64; ++b) std::memcpy(&phys[row * 1024 + b * 16], &t[tile_unit(row, b) * 16], 16);
      for (uint64_t row = 0; row < N; ++row) unseal(phys.data() + row * 1024, 0u, row);
    }
    if (e.stamp_prev != kNone) {
      // rows the last batch changed are pending in P (applied by the next pass):
      // slot descriptor {row in partition, stamp, P position, first position};
      // plain stores keep the final state at the slot (PS), AUTH stores by
      // position, sealed (P)
      const uint64_t WC = (uint64_t)e.W * e.c;
      std::vector<uint4> td(WC * 8);
      std::vector<uint8_t> pv(h->auth ? (uint64_t)e.B * 1024 : WC * 1024);
      GVS_HIP(h, hipMemcpy(td.data(), e.tbuf[e.par ^ 1], WC * 128, hipMemcpyDeviceToHost));
      GVS_HIP(h, hipMemcpy(pv.data(), h->auth ? e.pbuf : e.ps, pv.size(), hipMemcpyDeviceToHost));
      for (uint64_t k = 0; k < WC; ++k) {
        const uint4 d = td[k * 8];
        if (d.y != e.stamp_prev || d.x >= e.S || d.z >= e.B) continue;
        uint8_t* src = pv.data() + (h->auth ? (uint64_t)d.z : k) * 1024;
        if (h->auth) unseal(src, 2u, d.z);
        std::memcpy(phys.data() + ((k / e.c) * e.S + d.x) * 1024, src, 1024);
      }
    }
    for (uint64_t sl = 0; sl < N; ++sl) {
      const uint64_t row = (sl % e.W) * e.S + sl / e.W;
      std::memcpy(dst + sl * 1024, phys.data() + row * 1024, 1024);
    }
    dst += N * 1024;
  }
  return GVS_OK;
}

static int raw_region(gvs_handle* h, uint32_t shard, uint32_t region, void** base,
                      uint64_t* size) {
  if (shard >= h->eng.size()) return GVS_ERR_INVALID_ARG;
  Engine& e = h->eng[shard];
  switch (region) {
    case 0: *base = e.table; *size = e.N * 1024; break;
    case 1: *base = e.mbox; *size = e.R * 1024; break;
    case 2: *base = e.side; *size = e.R * 16; break;
    case 3: *base = e.mtag; *size = e.mtag ? e.N * 16 : 0; break;
    case 4: *base = e.btag; *size = e.btag ? e.R * 16 : 0; break;
    // pipeline 2: the final states pending from the last batch, their side
    // entries and tags, and that batch's slot descriptors
    case 5: *base = e.pbuf; *size = (uint64_t)e.B * 1024; break;
    case 6: *base = e.psd; *size = (uint64_t)e.B * 128; break;
    case 7: *base = e.ptag; *size = e.ptag ? (uint64_t)e.B * 16 : 0; break;
    case 8: *base = e.tbuf[e.par ^ 1]; *size = (uint64_t)e.W * e.c * 128; break;
    // the key-value map's key directory and, sealed, its row tags
    case 9: *base = e.kdir; *size = e.kdir ? e.N * 32 : 0; break;
    case 10: *base = e.ktag; *size = e.ktag ? e.N / 32 * 16 : 0; break;
    default: return GVS_ERR_INVALID_ARG;
  }
  return *base ? GVS_OK : GVS_ERR_INVALID_ARG;
}

int gvs_raw_size(gvs_handle* h, uint32_t shard, uint32_t region, uint64_t* size) {
  if (!h || !size) return GVS_ERR_INVALID_ARG;
  void* base;
  return raw_region(h, shard, region, &base, size);
}

// A sealed message / block table is stored in 8-row tiles (gvs_seal_dev.h
// tile_unit), a sealed mailbox table in 16-row tiles (mtile_unit); the raw
// hooks show and take them as rows (row r at r * 1024), the layout of the
// storage format (oracle/gvs_seal.c), converting the tiles the byte range
// covers.  Rows per tile, 0 for a region stored as rows.
static uint32_t tiled(const gvs_handle* h, uint32_t region) {
  return !h->auth ? 0u : region == 0 ? 8u : region == 1 && h->kind == 0 ? 16u : 0u;
}
static uint64_t tile_u(uint32_t tr, uint64_t r, uint32_t b) { return tr == 8 ? tile_unit(r, b) : mtile_unit(r, b); }

static int tiles_in(gvs_handle* h, const void* base, uint32_t tr, uint64_t t0, uint64_t nt, std::vector<uint8_t>& rows) {
  const uint64_t tb = (uint64_t)tr * 1024;
  std::vector<uint8_t> t(nt * tb);
  GVS_HIP(h, hipMemcpyAsync(t.data(), (const uint8_t*)base + t0 * tb, t.size(), hipMemcpyDeviceToHost, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  rows.resize(t.size());
  for (uint64_t r = 0; r < nt * tr; ++r)
    for (uint32_t b = 0; b < 64; ++b) std::memcpy(&rows[r * 1024 + b * 16], &t[tile_u(tr, r, b) * 16], 16);
  return GVS_OK;
}

int gvs_dump_raw(gvs_handle* h, uint32_t shard, uint32_t region, uint64_t offset, void* dst,
                 uint64_t bytes) {
  if (!h || !dst) return GVS_ERR_INVALID_ARG;
  if (int r = flush_m2(h)) return r;
  void* base;
  uint64_t size;
  if (int r = raw_region(h, shard, region, &base, &size)) return r;
  if (offset > size || bytes > size - offset) return GVS_ERR_INVALID_ARG;
  if (const uint32_t tr = tiled(h, region); tr && bytes) {
    const uint64_t tb = (uint64_t)tr * 1024, t0 = offset / tb, t1 = (offset + bytes + tb - 1) / tb;
    std::vector<uint8_t> rows;
    if (int r = tiles_in(h, base, tr, t0, t1 - t0, rows)) return r;
    std::memcpy(dst, &rows[offset - t0 * tb], bytes);
    return GVS_OK;
  }
  GVS_HIP(h, hipMemcpyAsync(dst, (uint8_t*)base + offset, bytes, hipMemcpyDeviceToHost, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

int gvs_store_raw(gvs_handle* h, uint32_t shard, uint32_t region, uint64_t offset,
                  const void* src, uint64_t bytes) {
  if (!h || !src) return GVS_ERR_INVALID_ARG;
  if (int r = flush_m2(h)) return r;
  void* base;
  uint64_t size;
  if (int r = raw_region(h, shard, region, &base, &size)) return r;
  if (offset > size || bytes > size - offset) return GVS_ERR_INVALID_ARG;
  if (const uint32_t tr = tiled(h, region); tr && bytes) {
    const uint64_t tb = (uint64_t)tr * 1024, t0 = offset / tb, t1 = (offset + bytes + tb - 1) / tb;
    std::vector<uint8_t> rows;
    if (int r = tiles_in(h, base, tr, t0, t1 - t0, rows)) return r;
    std::memcpy(&rows[offset - t0 * tb], src, bytes);
    std::vector<uint8_t> t(rows.size());
    for (uint64_t r = 0; r < (t1 - t0) * tr; ++r)
      for (uint32_t b = 0; b < 64; ++b) std::memcpy(&t[tile_u(tr, r, b) * 16], &rows[r * 1024 + b * 16], 16);
    GVS_HIP(h, hipMemcpyAsync((uint8_t*)base + t0 * tb, t.data(), t.size(), hipMemcpyHostToDevice, h->stream));
    GVS_HIP(h, hipStreamSynchronize(h->stream));
    return GVS_OK;
  }
  GVS_HIP(h, hipMemcpyAsync((uint8_t*)base + offset, src, bytes, hipMemcpyHostToDevice, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}


// Set every shard's epoch (authenticated mode): tests of the epoch limit.  No
// row is re-sealed, so a batch at the new epoch fails its tags, unless the
// call is refused first (GVS_ERR_EPOCH_EXHAUSTED) as it must be at the limit.
int gvs_test_set_epoch(gvs_handle* h, uint32_t epoch) {
  if (!h || !h->auth) return GVS_ERR_INVALID_ARG;
  for (auto& e : h->eng) e.epoch = epoch;
  return GVS_OK;
}

// the block store's and the map's engine handles, for the raw-region hooks above
gvs_handle* gvs_oram_test_handle(gvs_oram* o) { return o ? o->h : nullptr; }
gvs_handle* gvs_omap_test_handle(gvs_omap* m) { return m ? m->h : nullptr; }

// The router's placement on the host, with the device's route_dest (see
// include/gvstore_test.h): slot[i] = d * C + rank of request i among this
// source's requests for shard d, or 0xFFFFFFFF past C.
int gvs_route_plan(const gvs_config* cfg, const gvs_request* reqs, uint32_t n, uint32_t* slot,
                   uint32_t* capacity, uint32_t* shard_batch_out, uint8_t* shed) {
  if (!cfg || (n && (!reqs || !slot))) return GVS_ERR_INVALID_ARG;
  if (int rc = validate(cfg)) return rc;
  const uint32_t S = cfg->shard_count ? cfg->shard_count : 1u, B = cfg->max_batch;
  if (n > B) return GVS_ERR_INVALID_ARG;
  const uint32_t C = cfg->route_capacity ? cfg->route_capacity : auto_capacity(B, S);
  RouteArgs a{};
  a.in = reinterpret_cast<const uint4*>(reqs);
  a.n = n;
  a.B = B;
  a.S = S;
  a.C = C;
  a.N = cfg->msg_capacity;
  a.kc.pk0 = ld64(cfg->secret_key);
  a.kc.pk1 = ld64(cfg->secret_key + 8);
  a.kc.hk0 = ld64(cfg->secret_key + 16);
  a.kc.hk1 = ld64(cfg->secret_key + 24);
  a.kc.nshards = S;
  std::vector<uint32_t> cnt(S, 0);
  std::vector<uint64_t> keys(n);
  std::vector<uint32_t> dest(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t k;
    dest[i] = route_dest_key(a, i, k);
    keys[i] = ((uint64_t)k << 32) | i;
  }
  std::sort(keys.begin(), keys.end());  // the hot-key cap, as k_route_mark / k_route_apply
  if (shed) std::fill(shed, shed + n, (uint8_t)0);
  for (uint32_t j = kRouteKeyCap; j < n; ++j) {
    const uint32_t k = (uint32_t)(keys[j] >> 32), i = (uint32_t)keys[j];
    if ((k & 3u) != kKeyNone && (uint32_t)(keys[j - kRouteKeyCap] >> 32) == k) {
      dest[i] = i % S;
      if (shed) shed[i] = 1;
    }
  }
  bool over = false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t d = dest[i];
    const uint32_t r = cnt[d]++;
    over |= r >= C;
    slot[i] = r < C ? d * C + r : kNone;
  }
  if (capacity) *capacity = C;
  if (shard_batch_out) *shard_batch_out = S > 1 ? shard_batch((uint64_t)S * C + cfg->expiry_per_batch) : B;
  return over ? GVS_ERR_BATCH_OVERFLOW : GVS_OK;
}
#endif  // GVS_TEST_HOOKS


// ---- block store: mc-oblivious-traits ORAM::access, batched

// a block store (kind 1) or key-value map (kind 2) handle
static int kv_create(const gvs_oram_config* cfg, int kind, gvs_handle** out) {
  *out = nullptr;
  if (!is_pow2(cfg->capacity) || cfg->capacity < 4096 || cfg->capacity > (1ull << 32))
    return GVS_ERR_INVALID_ARG;
  if (!is_pow2(cfg->max_batch) || cfg->max_batch < 1024 || cfg->max_batch > (1u << (kSeqBits - 1)))
    return GVS_ERR_INVALID_ARG;
  if (cfg->flags & ~GVS_FLAG_AUTH_STORAGE) return GVS_ERR_INVALID_ARG;
  for (int i = 0; i < 3; ++i)
    if (cfg->reserved[i]) return GVS_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GVS_ERR_NO_DEVICE;
  if ((int)cfg->device >= ndev) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = new (std::nothrow) gvs_handle();
  if (!h) return GVS_ERR_OUT_OF_MEMORY;
  h->kind = kind;
  h->mode = kSingle;
  h->device = (int)cfg->device;
  h->auth = (cfg->flags & GVS_FLAG_AUTH_STORAGE) != 0;
  h->cfg.msg_capacity = cfg->capacity;
  h->cfg.max_batch = cfg->max_batch;
  h->cfg.device = cfg->device;
  h->cfg.flags = cfg->flags;
  std::memcpy(h->cfg.secret_key, cfg->secret_key, 32);
  h->Bsub = h->Be = cfg->max_batch;
  auto fail = [&](int code) {
    gvs_destroy(h);
    return code;
  };
  if (hipSetDevice(h->device) != hipSuccess) return fail(GVS_ERR_DEVICE);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(GVS_ERR_DEVICE);
  for (auto& ev : h->ev)
    if (hipEventCreate(&ev) != hipSuccess) return fail(GVS_ERR_DEVICE);
  if (h->auth) {
    uint32_t te0[256], nh[kNhWords];
    storage_ctx(cfg->secret_key, h->sc, te0, nh);
    if (int rc = dalloc_t(h, &h->te, 256)) return fail(rc);
    if (hipMemcpy(h->te, te0, sizeof te0, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GVS_ERR_DEVICE);
    if (int rc = dalloc_t(h, &h->nhk, kNhWords)) return fail(rc);
    if (hipMemcpy(h->nhk, nh, sizeof nh, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GVS_ERR_DEVICE);
    h->sc.nhk = h->nhk;
  }
  h->eng.resize(1);
  Engine& e = h->eng[0];
  e.kc.hk0 = ld64(cfg->secret_key + 16);
  e.kc.hk1 = ld64(cfg->secret_key + 24);
  if (int rc = kv_engine_init(h, e, cfg->capacity, cfg->max_batch)) return fail(rc);
  const uint64_t in_u4 = kind == 2 ? 66 : kAbiU4, out_u4 = kind == 2 ? kAbiU4 : 64;
  if (int rc = dalloc_t(h, &h->in_stage, (uint64_t)cfg->max_batch * in_u4)) return fail(rc);
  if (int rc = dalloc_t(h, &h->out_stage, (uint64_t)cfg->max_batch * out_u4)) return fail(rc);
  *out = h;
  return GVS_OK;
}

int gvs_oram_create(const gvs_oram_config* cfg, gvs_oram** out) {
  if (!cfg || !out) return GVS_ERR_INVALID_ARG;
  *out = nullptr;
  gvs_handle* h;
  if (int rc = kv_create(cfg, 1, &h)) return rc;
  gvs_oram* o = new (std::nothrow) gvs_oram();
  if (!o) {
    gvs_destroy(h);
    return GVS_ERR_OUT_OF_MEMORY;
  }
  o->h = h;
  *out = o;
  return GVS_OK;
}

int gvs_oram_destroy(gvs_oram* o) {
  if (!o) return GVS_ERR_INVALID_ARG;
  if (o->h) gvs_destroy(o->h);
  delete o;
  return GVS_OK;
}

int gvs_oram_access_batch(gvs_oram* o, const gvs_block_op* ops, uint32_t n, uint8_t* out) {
  if (!o || (!ops && n) || (!out && n) || n > o->h->Bsub) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = o->h;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = bounce_begin(h)) return r;
  if (int r = h2d(h, 0, h->in_stage, ops, (size_t)n * sizeof(gvs_block_op))) return r;
  if (int r = oram_batch(h, h->eng[0], h->in_stage, n, h->out_stage)) return r;
  if (int r = d2h(h, 4, out, h->out_stage, (size_t)n * 1024)) return r;
  return bounce_done(h, finish(h));
}

int gvs_oram_access_batch_device(gvs_oram* o, const void* d_ops, uint32_t n, void* d_out) {
  if (!o || (!d_ops && n) || (!d_out && n) || n > o->h->Bsub) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = o->h;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  const uint4* in = n ? (const uint4*)d_ops : h->in_stage;
  if (int r = oram_batch(h, h->eng[0], in, n, n ? (uint4*)d_out : h->out_stage)) return r;
  return finish(h);
}

int gvs_oram_set_timing(gvs_oram* o, int on) { return o ? gvs_set_timing(o->h, on) : GVS_ERR_INVALID_ARG; }

int gvs_oram_last_timings(gvs_oram* o, const char** names, float* ms, int cap) {
  return o ? gvs_last_timings(o->h, names, ms, cap) : GVS_ERR_INVALID_ARG;
}

const char* gvs_oram_last_error(gvs_oram* o) { return o ? o->h->err.c_str() : "null handle"; }

// ---- key-value map: mc-oblivious-traits ObliviousHashMap, batched

int gvs_omap_create(const gvs_omap_config* cfg, gvs_omap** out) {
  if (!cfg || !out) return GVS_ERR_INVALID_ARG;
  *out = nullptr;
  gvs_handle* h;
  if (int rc = kv_create(reinterpret_cast<const gvs_oram_config*>(cfg), 2, &h)) return rc;
  gvs_omap* o = new (std::nothrow) gvs_omap();
  if (!o) {
    gvs_destroy(h);
    return GVS_ERR_OUT_OF_MEMORY;
  }
  o->h = h;
  *out = o;
  return GVS_OK;
}

int gvs_omap_destroy(gvs_omap* o) {
  if (!o) return GVS_ERR_INVALID_ARG;
  if (o->h) gvs_destroy(o->h);
  delete o;
  return GVS_OK;
}

int gvs_omap_access_batch(gvs_omap* o, const gvs_omap_op* ops, uint32_t n, gvs_omap_result* out) {
  if (!o || (!ops && n) || (!out && n) || n > o->h->Bsub) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = o->h;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = bounce_begin(h)) return r;
  if (int r = h2d(h, 0, h->in_stage, ops, (size_t)n * sizeof(gvs_omap_op))) return r;
  if (int r = omap_batch(h, h->eng[0], h->in_stage, n, h->out_stage)) return r;
  if (int r = d2h(h, 4, out, h->out_stage, (size_t)n * sizeof(gvs_omap_result))) return r;
  return bounce_done(h, finish(h));
}

int gvs_omap_access_batch_device(gvs_omap* o, const void* d_ops, uint32_t n, void* d_out) {
  if (!o || (!d_ops && n) || (!d_out && n) || n > o->h->Bsub) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = o->h;
  if (h->poisoned) return GVS_ERR_INTEGRITY;
  if (int r = check_epoch(h)) return r;
  GVS_HIP(h, hipSetDevice(h->device));
  const uint4* in = n ? (const uint4*)d_ops : h->in_stage;
  if (int r = omap_batch(h, h->eng[0], in, n, (uint4*)d_out)) return r;
  return finish(h);
}

int gvs_omap_set_timing(gvs_omap* o, int on) { return o ? gvs_set_timing(o->h, on) : GVS_ERR_INVALID_ARG; }

int gvs_omap_last_timings(gvs_omap* o, const char** names, float* ms, int cap) {
  return o ? gvs_last_timings(o->h, names, ms, cap) : GVS_ERR_INVALID_ARG;
}

const char* gvs_omap_last_error(gvs_omap* o) { return o ? o->h->err.c_str() : "null handle"; }

}  // extern "C"
