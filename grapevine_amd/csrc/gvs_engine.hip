// gvs_engine.hip — host side of libgvstore.so: the C ABI of include/gvstore.h
// driving the gfx950 kernels of gvs_kernels.h on one HIP stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/gvstore.h"
#include "gvs_kernels.h"

using namespace gvs;

static_assert(sizeof(gvs_record) == 1024, "record layout");
static_assert(sizeof(gvs_request) == 1040, "request layout");
static_assert(sizeof(gvs_response) == 1040, "response layout");

namespace {

constexpr int kNullBlocks = 32;   // R-pass blocks for ops that touch no row
constexpr int kDummyBlocks = 32;  // M-pass blocks for ops that touch no mailbox
constexpr int kMaxStages = 16;

const char* kStageNames[] = {"copy", "meta", "sort_s1", "m1", "alloc", "sort_r",
                             "rpass", "post", "m2"};
constexpr int kNumStages = 9;

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

}  // namespace

struct gvs_handle {
  gvs_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t N = 0, R = 0, ring_size = 0;
  uint32_t Q = 0, Sr = 0, B = 0, W = 0, S = 0, NT = 0, logQ = 0;
  KeyCtx kc{};
  // persistent state
  uint4* table = nullptr;
  uint4* mbox = nullptr;
  uint4* side = nullptr;
  uint32_t* ring = nullptr;
  Scal* scal = nullptr;
  // per-batch scratch
  uint32_t nblk = 0;
  uint64_t extra = 0;
  uint4* img = nullptr;
  uint32_t* types = nullptr;
  OpState* ops = nullptr;
  uint32_t* kinds = nullptr;
  Key128* s1keys = nullptr;
  uint32_t* qcount = nullptr;
  uint32_t* qstart = nullptr;
  M1Out* m1out = nullptr;
  uint32_t* pflag = nullptr;
  uint32_t* pslot = nullptr;
  uint32_t* bsum = nullptr;
  uint32_t* cslot = nullptr;
  ROp* rop = nullptr;
  uint64_t* rkeys = nullptr;
  uint32_t* pcount = nullptr;
  uint32_t* pstart = nullptr;
  RRes* rres = nullptr;
  uint4* resp = nullptr;
  uint32_t* dflag = nullptr;
  uint32_t* dslot = nullptr;
  uint32_t* bsum2 = nullptr;
  uint4* in_stage = nullptr;
  uint4* out_stage = nullptr;
  hipEvent_t ev[kMaxStages + 1] = {};
  bool timed = false;
  int rpass_variant = 6;
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

extern "C" {

const char* gvs_version(void) { return "gvstore 0.1.0 (gfx950)"; }

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
  if (c->flags != 0) return GVS_ERR_INVALID_ARG;
  for (int i = 1; i < 7; ++i)
    if (c->reserved[i] != 0) return GVS_ERR_INVALID_ARG;
  return GVS_OK;
}

int gvs_destroy(gvs_handle* h) {
  if (!h) return GVS_ERR_INVALID_ARG;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : h->allocs) (void)hipFree(p);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return GVS_OK;
}

int gvs_create(const gvs_config* cfg, gvs_handle** out) {
  if (!out) return GVS_ERR_INVALID_ARG;
  *out = nullptr;
  int rc = validate(cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GVS_ERR_NO_DEVICE;
  if ((int)cfg->device >= ndev) return GVS_ERR_INVALID_ARG;
  gvs_handle* h = new (std::nothrow) gvs_handle();
  if (!h) return GVS_ERR_OUT_OF_MEMORY;
  h->cfg = *cfg;
  h->device = (int)cfg->device;
  h->N = cfg->msg_capacity;
  h->Q = cfg->mailbox_partitions;
  h->Sr = cfg->mailbox_partition_slots;
  h->R = (uint64_t)h->Q * h->Sr;
  h->B = cfg->max_batch;
  h->logQ = log2u(h->Q);
  // rows per message-table partition (one workgroup each): reserved[0] if set,
  // else N/16384 clamped to [256, 4096] (C3: 1024 rows -> 16384 workgroups, so
  // the grid is many times the resident capacity and its tail is short)
  uint64_t S = cfg->reserved[0] ? cfg->reserved[0] : h->N / 16384;
  if (S < (uint64_t)kTile) S = kTile;
  if (S > (uint64_t)kRowsMax) S = kRowsMax;
  if (S > h->N) S = h->N;
  if (!is_pow2(S)) {
    delete h;
    return GVS_ERR_INVALID_ARG;
  }
  h->S = (uint32_t)S;
  h->W = (uint32_t)(h->N / S);
  h->NT = (uint32_t)(h->N / kTile);
  h->nblk = h->B / 1024;
  h->ring_size = h->N + h->B;
  if (h->W + 1 > (uint32_t)kBinsMax || h->S > (uint32_t)kRowsMax) {
    delete h;
    return GVS_ERR_INVALID_ARG;
  }
  h->kc.pk0 = ld64(cfg->secret_key);
  h->kc.pk1 = ld64(cfg->secret_key + 8);
  h->kc.hk0 = ld64(cfg->secret_key + 16);
  h->kc.hk1 = ld64(cfg->secret_key + 24);

  auto fail = [&](int code) {
    gvs_destroy(h);
    return code;
  };
  if (hipSetDevice(h->device) != hipSuccess) return fail(GVS_ERR_DEVICE);
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(GVS_ERR_DEVICE);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(GVS_ERR_DEVICE);

  const uint64_t B = h->B;
#define A(ptr, n)                            \
  do {                                       \
    int r_ = dalloc_t(h, &h->ptr, (n));      \
    if (r_) {                                \
      std::string e_ = h->err;               \
      gvs_destroy(h);                        \
      (void)e_;                              \
      return r_;                             \
    }                                        \
  } while (0)
  A(table, h->N * 64);
  A(mbox, h->R * 64);
  A(side, h->R);
  A(ring, h->ring_size);
  A(scal, 1);
  // per-op arrays carry E extra records after the B real ones; record B is the
  // shared dummy of the dry-run ops (fixed instruction footprint)
  const uint64_t E = 64;
  h->extra = E;
  A(img, (B + E) * 64);
  A(types, B);
  A(ops, B);
  A(kinds, B);
  A(s1keys, B);
  A(qcount, h->Q + 1);
  A(qstart, h->Q + 2);
  A(m1out, B + E);
  A(pflag, B);
  A(pslot, B);
  A(bsum, 2 * h->nblk);
  A(cslot, B);
  A(rop, B + E);
  A(rkeys, B);
  A(pcount, h->W + 1);
  A(pstart, h->W + 2);
  A(rres, B + E);
  A(resp, (B + E) * (kRespSlot / 16));
  A(dflag, B);
  A(dslot, B);
  A(bsum2, h->nblk);
  A(in_stage, B * 65);
  A(out_stage, B * 65);
#undef A
  hipStream_t s = h->stream;
  if (hipMemsetAsync(h->img + B * 64, 0, E * 1024, s) != hipSuccess ||
      hipMemsetAsync(h->rop + B, 0, E * sizeof(ROp), s) != hipSuccess ||
      hipMemsetAsync(h->table, 0, h->N * 1024, s) != hipSuccess ||
      hipMemsetAsync(h->mbox, 0, h->R * 1024, s) != hipSuccess ||
      hipMemsetAsync(h->side, 0, h->R * 16, s) != hipSuccess)
    return fail(GVS_ERR_DEVICE);
  // free ring = slots 0..N-1 in order; scalars
  {
    std::vector<uint32_t> ring(h->ring_size, kNone);
    for (uint64_t i = 0; i < h->N; ++i) ring[i] = (uint32_t)i;
    Scal sc{};
    sc.head = 0;
    sc.tail = h->N;
    if (hipMemcpyAsync(h->ring, ring.data(), ring.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(h->scal, &sc, sizeof sc, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return fail(GVS_ERR_DEVICE);
  }
  *out = h;
  return GVS_OK;
}

}  // extern "C"

template <typename K, int LMAX>
static int sort_keys(gvs_handle* h, K* d, uint32_t n) {
  const uint32_t L = n < (uint32_t)LMAX ? n : (uint32_t)LMAX;
  hipStream_t s = h->stream;
  hipLaunchKernelGGL((k_bitonic_local<K, LMAX>), dim3(n / L), dim3(1024), 0, s, d, L, 0u, 1);
  for (uint32_t k = 2 * L; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j >= L; j >>= 1)
      hipLaunchKernelGGL(k_bitonic_global<K>, dim3((n / 2 + 255) / 256), dim3(256), 0, s, d, n, k, j);
    hipLaunchKernelGGL((k_bitonic_local<K, LMAX>), dim3(n / L), dim3(1024), 0, s, d, L, k, 0);
  }
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

static MArgs margs(gvs_handle* h) {
  MArgs a{};
  a.keys = h->s1keys;
  a.qstart = h->qstart;
  a.mbox = h->mbox;
  a.side = h->side;
  a.m1out = h->m1out;
  a.rop = h->rop;
  a.rres = h->rres;
  a.scal = h->scal;
  a.Q = h->Q;
  a.Sr = h->Sr;
  a.B = h->B;
  a.dummy_blocks = kDummyBlocks;
  a.N = h->N;
  a.kc = h->kc;
  return a;
}

static AllocArgs aargs(gvs_handle* h) {
  AllocArgs a{};
  a.kinds = h->kinds;
  a.m1out = h->m1out;
  a.ops = h->ops;
  a.pflag = h->pflag;
  a.pslot = h->pslot;
  a.bsum = h->bsum;
  a.cslot = h->cslot;
  a.ring = h->ring;
  a.rop = h->rop;
  a.rkeys = h->rkeys;
  a.pcount = h->pcount;
  a.scal = h->scal;
  a.B = h->B;
  a.nblk = h->nblk;
  a.W = h->W;
  a.S = h->S;
  a.N = h->N;
  a.ring_size = h->ring_size;
  a.kc = h->kc;
  return a;
}

// Enqueue the whole pipeline for one batch on h->stream; responses for the
// first n requests are written to d_out (caller layout).
static int run_pipeline(gvs_handle* h, const uint4* d_in, uint32_t n, uint4* d_out) {
  hipStream_t s = h->stream;
  const uint32_t B = h->B, nblk = h->nblk;
  int st = 0;
  auto mark = [&](int i) {
    if (h->timed) (void)hipEventRecord(h->ev[i], s);
  };
  GVS_HIP(h, hipMemsetAsync(&h->scal->error, 0, sizeof(uint32_t), s));
  GVS_HIP(h, hipMemsetAsync(h->qcount, 0, (h->Q + 1) * sizeof(uint32_t), s));
  GVS_HIP(h, hipMemsetAsync(h->pcount, 0, (h->W + 1) * sizeof(uint32_t), s));
  mark(st++);
  hipLaunchKernelGGL(k_copy, dim3(B / 4), dim3(256), 0, s, d_in, n, B, h->img, h->types);
  mark(st++);
  {
    MetaArgs a{h->img, h->types, h->ops, h->kinds, h->s1keys, h->qcount,
               n, B, h->Q, h->logQ, h->N, h->kc};
    hipLaunchKernelGGL(k_meta, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, s, h->qcount, h->qstart, h->Q + 1);
  }
  mark(st++);
  if (int r = sort_keys<Key128, 4096>(h, h->s1keys, B)) return r;
  mark(st++);
  hipLaunchKernelGGL(k_m1, dim3(h->Q + kDummyBlocks), dim3(256), 0, s, margs(h));
  mark(st++);
  {
    AllocArgs a = aargs(h);
    hipLaunchKernelGGL(k_alloc_sum, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_alloc_ring, dim3(1), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_alloc_b, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, s, h->pcount, h->pstart, h->W + 1);
  }
  mark(st++);
  if (int r = sort_keys<uint64_t, 8192>(h, h->rkeys, B)) return r;
  mark(st++);
  {
    RArgs a{};
    a.table = h->table;
    a.rkeys = h->rkeys;
    a.pstart = h->pstart;
    a.rop = h->rop;
    a.img = h->img;
    a.resp = h->resp;
    a.rres = h->rres;
    a.scal = h->scal;
    a.n = n;
    a.B = B;
    a.W = h->W;
    a.S = h->S;
    a.null_blocks = kNullBlocks;
    const dim3 g(h->W + kNullBlocks), b(256);
    switch (h->rpass_variant) {
      case 0: hipLaunchKernelGGL((k_rpass<4, false, false, 1>), g, b, 0, s, a); break;
      case 1: hipLaunchKernelGGL((k_rpass<4, true, true, 1>), g, b, 0, s, a); break;
      case 3: hipLaunchKernelGGL((k_rpass<8, true, false, 4>), g, b, 0, s, a); break;
      case 4: hipLaunchKernelGGL((k_rpass<8, false, true, 4>), g, b, 0, s, a); break;
      case 5: hipLaunchKernelGGL((k_rpass<2, true, true, 8>), g, b, 0, s, a); break;
      case 6: hipLaunchKernelGGL((k_rpass<16, true, true, 2>), g, b, 0, s, a); break;
      case 7: hipLaunchKernelGGL((k_rpass<32, true, true, 1>), g, b, 0, s, a); break;
      case 8: hipLaunchKernelGGL((k_rpass<16, true, true, 1>), g, b, 0, s, a); break;
      case 9: hipLaunchKernelGGL((k_rpass<8, true, true, 2>), g, b, 0, s, a); break;
      case 10: hipLaunchKernelGGL((k_rpass<16, false, true, 2>), g, b, 0, s, a); break;
      default: hipLaunchKernelGGL((k_rpass<8, true, true, 4>), g, b, 0, s, a); break;
    }
  }
  mark(st++);
  {
    PostArgs a{h->kinds, h->rres, h->rop, h->dflag, h->dslot, h->bsum2, h->ring, h->scal,
               B, nblk, h->ring_size};
    hipLaunchKernelGGL(k_post_sum, dim3(nblk), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_post_ring, dim3(1), dim3(1024), 0, s, a);
  }
  mark(st++);
  hipLaunchKernelGGL(k_m2, dim3(h->Q + kDummyBlocks), dim3(256), 0, s, margs(h));
  if (n) hipLaunchKernelGGL(k_out, dim3((n + 3) / 4), dim3(256), 0, s, (const uint4*)h->resp, n, d_out);
  mark(st++);
  GVS_HIP(h, hipGetLastError());
  return GVS_OK;
}

static int finish(gvs_handle* h) {
  uint32_t e = 0;
  GVS_HIP(h, hipMemcpyAsync(&e, &h->scal->error, sizeof e, hipMemcpyDeviceToHost, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  if (e & 1u) {
    h->err = "batch overflow: more than 512 distinct recipients in one mailbox partition";
    return GVS_ERR_BATCH_OVERFLOW;
  }
  if (e) {
    h->err = "internal error flag " + std::to_string(e);
    return GVS_ERR_INTERNAL;
  }
  return GVS_OK;
}

extern "C" {

int gvs_process_batch(gvs_handle* h, const gvs_request* reqs, uint32_t n, gvs_response* out) {
  if (!h || (!reqs && n) || (!out && n) || n > h->B) return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipSetDevice(h->device));
  if (n)
    GVS_HIP(h, hipMemcpyAsync(h->in_stage, reqs, (size_t)n * sizeof(gvs_request),
                              hipMemcpyHostToDevice, h->stream));
  if (int r = run_pipeline(h, h->in_stage, n, h->out_stage)) return r;
  if (n)
    GVS_HIP(h, hipMemcpyAsync(out, h->out_stage, (size_t)n * sizeof(gvs_response),
                              hipMemcpyDeviceToHost, h->stream));
  return finish(h);
}

int gvs_process_batch_device(gvs_handle* h, const void* d_reqs, uint32_t n, void* d_out) {
  if (!h || (!d_reqs && n) || (!d_out && n) || n > h->B) return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipSetDevice(h->device));
  if (int r = run_pipeline(h, (const uint4*)d_reqs, n, (uint4*)d_out)) return r;
  return finish(h);
}

int gvs_access(gvs_handle* h, const gvs_request* req, gvs_response* out) {
  return gvs_process_batch(h, req, 1, out);
}

int gvs_get_stats(gvs_handle* h, gvs_stats* out) {
  if (!h || !out) return GVS_ERR_INVALID_ARG;
  Scal sc{};
  GVS_HIP(h, hipMemcpyAsync(&sc, h->scal, sizeof sc, hipMemcpyDeviceToHost, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  out->messages = sc.count;
  out->mailboxes = sc.n_mailboxes;
  out->batches = sc.batches;
  out->creation_counter = sc.ctr;
  out->free_ring_head = sc.head;
  out->free_ring_tail = sc.tail;
  out->msg_partitions = h->W;
  out->msg_partition_slots = h->S;
  return GVS_OK;
}

int gvs_dump_messages(gvs_handle* h, void* host_dst, uint64_t bytes) {
  if (!h || !host_dst || bytes < h->N * 1024) return GVS_ERR_INVALID_ARG;
  std::vector<uint8_t> phys(h->N * 1024);
  GVS_HIP(h, hipMemcpyAsync(phys.data(), h->table, phys.size(), hipMemcpyDeviceToHost, h->stream));
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  uint8_t* dst = (uint8_t*)host_dst;
  for (uint64_t sl = 0; sl < h->N; ++sl) {
    uint64_t row = (sl % h->W) * h->S + sl / h->W;
    std::memcpy(dst + sl * 1024, phys.data() + row * 1024, 1024);
  }
  return GVS_OK;
}

int gvs_synchronize(gvs_handle* h) {
  if (!h) return GVS_ERR_INVALID_ARG;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  return GVS_OK;
}

int gvs_set_timing(gvs_handle* h, int on) {
  if (!h) return GVS_ERR_INVALID_ARG;
  h->timed = on != 0;
  return GVS_OK;
}

int gvs_set_option(gvs_handle* h, const char* key, int64_t value) {
  if (!h || !key) return GVS_ERR_INVALID_ARG;
  if (std::strcmp(key, "rpass_variant") == 0 && value >= 0 && value <= 10) {
    h->rpass_variant = (int)value;
    return GVS_OK;
  }
  return GVS_ERR_INVALID_ARG;
}

int gvs_last_timings(gvs_handle* h, const char** names, float* ms, int cap) {
  if (!h) return GVS_ERR_INVALID_ARG;
  if (!h->timed) return 0;
  GVS_HIP(h, hipStreamSynchronize(h->stream));
  int c = 0;
  for (int i = 0; i < kNumStages && c < cap; ++i, ++c) {
    float t = 0.f;
    (void)hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]);
    if (names) names[c] = kStageNames[i];
    if (ms) ms[c] = t;
  }
  return c;
}

const char* gvs_last_error(gvs_handle* h) { return h ? h->err.c_str() : "null handle"; }

}  // extern "C"
