// ce_ctx.cpp -- context, device batch engine (open / seal) and the Cryptor C ABI.
//
// Cryptor trait: crdt-enc/src/cryptor.rs:11-27.  EncHandler (XChaCha20-Poly1305):
// crdt-enc-xchacha20poly1305/src/lib.rs:28-101.  Every AEAD in this library runs on the GPU;
// there is no CPU implementation of the cipher in the product.
#include <sys/random.h>

#include <algorithm>
#include <cstdio>

#include "ce_internal.h"

namespace ce {

hipError_t DevBuf::reserve(size_t bytes) {
  if (bytes <= cap) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  size_t want = std::max<size_t>(bytes, 256);
  want = (want + 4095) & ~size_t(4095);
  hipError_t e = hipMalloc(&p, want);
  if (e == hipSuccess) cap = want;
  return e;
}
DevBuf::~DevBuf() {
  if (p) (void)hipFree(p);
}
hipError_t HostBuf::reserve(size_t bytes) {
  if (bytes <= cap) return hipSuccess;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  size_t want = std::max<size_t>(bytes, 256);
  want = (want + 4095) & ~size_t(4095);
  hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
  if (e == hipSuccess) cap = want;
  return e;
}
HostBuf::~HostBuf() {
  if (p) (void)hipHostFree(p);
}

void os_random(uint8_t* out, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = getrandom(out + got, n - got, 0);
    if (r > 0) got += (size_t)r;
  }
}

int32_t key_status(const KeyRef& k) {
  // xchacha lib.rs:74-78: key.ensure_version(KEY_VERSION), key.len() == KEY_LEN
  if (std::memcmp(k.version, kKeyVersion, 16) != 0) return CE_ERR_KEY_VERSION;
  if (k.len != 32) return CE_ERR_KEY_LEN;
  return CE_OK;
}

DevKey dev_key(const KeyRef& k) {
  DevKey d{};
  if (k.len == 32) std::memcpy(d.k, k.key, 32);
  return d;
}

uint32_t grid_waves_for(uint32_t work) {
  // 256 CUs x 32 resident waves (segment kernel: <= 64 VGPRs -> 8 waves / SIMD)
  const uint32_t full = 256u * 32u;
  return std::max<uint32_t>(1, std::min<uint32_t>(work, full));
}

static int reserve_batch(ce_ctx* ctx, uint32_t n, uint64_t blob_len, uint32_t* extra_cap,
                         uint32_t seg_blocks = kSegBlocks) {
  const uint64_t ec = blob_len / (seg_blocks * 16) + 16;
  if (ec > 0xffffffffull) return ctx->fail(CE_ERR_INVALID_ARG, "batch too large");
  *extra_cap = (uint32_t)ec;
  hipError_t e;
  if ((e = ctx->params.reserve((size_t)n * sizeof(FileParams))) != hipSuccess ||
      (e = ctx->status.reserve((size_t)n * 4 + 64)) != hipSuccess ||
      (e = ctx->counters.reserve(256)) != hipSuccess ||
      (e = ctx->extra.reserve(ec * 8)) != hipSuccess ||
      (e = ctx->multi.reserve(ec * 4)) != hipSuccess ||
      (e = ctx->partials.reserve(ec * 2 * 5 * 4)) != hipSuccess ||
      (e = ctx->large.reserve((size_t)n * 4 + 64)) != hipSuccess ||
      (e = ctx->h_counters.reserve(256)) != hipSuccess)
    return ctx->hip_fail(e, "reserve batch scratch");
  return CE_OK;
}

SegScratch segscratch(ce_ctx* ctx, uint32_t extra_cap) {
  SegScratch sc;
  sc.counters = ctx->counters.as<uint32_t>();
  sc.extra_list = ctx->extra.as<uint2>();
  sc.extra_cap = extra_cap;
  sc.multi_files = ctx->multi.as<uint32_t>();
  sc.partials = ctx->partials.as<uint32_t>();
  sc.large_list = ctx->large.as<uint32_t>();
  sc.seg_blocks = kSegBlocks;
  return sc;
}

// the counter block: [5] (first failing index, atomicMin) and [13] (the gate's first gap) start at
// UINT32_MAX, the rest at 0 -- one k_fill launch (two runtime fills were two blit dispatches)
static hipError_t reset_counters(ce_ctx* ctx) {
  FillArgs fl{};
  fl.n = 0;
  fl.counters = ctx->counters.as<uint32_t>();
  return launch_fill(ctx->stream, fl);
}

int device_open_setup(ce_ctx* ctx, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                      uint64_t blob_len, bool outer, const KeyRef& key, int32_t* d_status,
                      uint32_t* extra_cap, FillArgs* fills, const std::function<int()>* after_fill) {
  int rc = reserve_batch(ctx, n, blob_len, extra_cap);
  if (rc) return rc;
  hipError_t e;
  if (fills) {  // the caller's scratch and the counter block in one launch
    fills->counters = ctx->counters.as<uint32_t>();
    if ((e = launch_fill(ctx->stream, *fills)) != hipSuccess) return ctx->hip_fail(e, "fill");
  } else if ((e = reset_counters(ctx)) != hipSuccess) {
    return ctx->hip_fail(e, "memset counters");
  }
  // the caller's launches that need the filled scratch but not the setup (the version gate):
  // the setup then runs straight into the kernel that consumes it
  if (after_fill && (rc = (*after_fill)())) return rc;
  SegScratch sc = segscratch(ctx, *extra_cap);
  if ((e = ctx->poly_aux.reserve((size_t)n * sizeof(PolyAux))) != hipSuccess)
    return ctx->hip_fail(e, "reserve poly aux");
  const int t = ctx->tbegin("open_setup");
  if ((e = launch_open_setup(ctx->stream, d_blob, d_offs, n, outer, dev_key(key), key_status(key),
                             ctx->params.as<FileParams>(), d_status, sc,
                             ctx->poly_aux.as<PolyAux>())) != hipSuccess)
    return ctx->hip_fail(e, "open setup");
  ctx->tend(t);
  return CE_OK;
}

// small_lanes: single-page files opened by k_open_fold_v2's open-only form (16 lanes per file,
// lane-owned ChaCha20 blocks) and the segment pass left with the larger ones -- a wave per
// single-page file idles half its lanes on a 2 KiB file (C3's op files)
int device_open(ce_ctx* ctx, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                uint64_t blob_len, bool outer, const KeyRef& key, uint8_t* d_out,
                int32_t* d_status, bool sync_counters, bool small_lanes, const DecodeArgs* ds) {
  uint32_t ec;
  int rc = reserve_batch(ctx, n, blob_len, &ec);
  if (rc) return rc;
  hipError_t e;
  if ((e = reset_counters(ctx)) != hipSuccess) return ctx->hip_fail(e, "memset counters");
  SegScratch sc = segscratch(ctx, ec);
  FileParams* P = ctx->params.as<FileParams>();
  // the DS form's 8-lane kernel reads the setup's PolyAux rows (k_open_ds8)
  static const bool ds8_on = !(getenv("CE_DS8") && atoi(getenv("CE_DS8")) == 0);  // (ce_fused.hip)
  const bool want_aux = small_lanes && ds && ds->ds.on && ds->ds.big && ds8_on;
  if (want_aux && (e = ctx->poly_aux.reserve((size_t)n * sizeof(PolyAux))) != hipSuccess)
    return ctx->hip_fail(e, "reserve poly aux");
  int t = ctx->tbegin("open_setup");
  if ((e = launch_open_setup(ctx->stream, d_blob, d_offs, n, outer, dev_key(key), key_status(key),
                             P, d_status, sc, want_aux ? ctx->poly_aux.as<PolyAux>() : nullptr)) != hipSuccess)
    return ctx->hip_fail(e, "open setup");
  ctx->tend(t);
  if (small_lanes) {
    DecodeArgs da{};
    da.pt = d_out;
    da.blob = d_blob;
    da.params = P;
    da.status = d_status;
    da.n = n;
    da.counters = ctx->counters.as<uint32_t>();
    if (ds) {
      da.ds = ds->ds;
      da.aux = want_aux ? ctx->poly_aux.as<PolyAux>() : nullptr;
      da.supported = ds->supported;
      da.n_supported = ds->n_supported;
      da.table = ds->table;
      da.mask = ds->mask;
    }
    t = ctx->tbegin("open_small");
    if ((e = launch_open_small_v2(ctx->stream, da)) != hipSuccess) return ctx->hip_fail(e, "open small");
    ctx->tend(t);
  }
  t = ctx->tbegin("segments_open");
  if ((e = launch_segments(ctx->stream, false, d_blob, d_out, P, n, d_status, sc,
                           grid_waves_for(n + ec), small_lanes)) != hipSuccess)
    return ctx->hip_fail(e, "open segments");
  ctx->tend(t);
  t = ctx->tbegin("finalize_open");
  if ((e = launch_finalize_multi(ctx->stream, false, d_out, P, d_status, sc, n)) != hipSuccess)
    return ctx->hip_fail(e, "open finalize");
  ctx->tend(t);
  if (sync_counters) {
    if ((e = hipMemcpyAsync(ctx->h_counters.p, ctx->counters.p, 64, hipMemcpyDeviceToHost,
                            ctx->stream)) != hipSuccess ||
        (e = stream_wait(ctx->stream)) != hipSuccess)
      return ctx->hip_fail(e, "open sync");
  }
  return CE_OK;
}

uint32_t* ctx_counters(ce_ctx* ctx) {
  return ctx->counters.reserve(256) == hipSuccess ? ctx->counters.as<uint32_t>() : nullptr;
}

int device_seal(ce_ctx* ctx, const uint8_t* d_clear, const uint64_t* d_offs, uint32_t n,
                uint64_t clear_len_total, const uint8_t* d_outer_version, const uint8_t* d_nonces,
                uint8_t* d_out, const uint64_t* d_out_offs, const KeyRef& key, bool counters_ready) {
  if (int32_t ks = key_status(key)) return ctx->fail(ks, "key rejected");
  // a compaction's single state file of up to 1 MiB: one-page segments, so its keystream is 4x
  // the waves (the segment kernel's four dependent pages per wave were most of its time)
  const uint32_t seg_blocks = n <= 4 && clear_len_total <= (1u << 20) ? kPageBytes / 16 : kSegBlocks;
  uint32_t ec;
  int rc = reserve_batch(ctx, n, clear_len_total + 16ull * n, &ec, seg_blocks);
  if (rc) return rc;
  hipError_t e;
  if (!counters_ready && (e = reset_counters(ctx)) != hipSuccess) return ctx->hip_fail(e, "memset counters");
  SegScratch sc = segscratch(ctx, ec);
  sc.seg_blocks = seg_blocks;
  FileParams* P = ctx->params.as<FileParams>();
  int t = ctx->tbegin("seal_setup");
  if ((e = launch_seal_setup(ctx->stream, d_clear, d_offs, n, d_outer_version, d_nonces, d_out,
                             d_out_offs, dev_key(key), P, sc)) != hipSuccess)
    return ctx->hip_fail(e, "seal setup");
  ctx->tend(t);
  t = ctx->tbegin("segments_seal");
  // one wave per segment: a single large state file still fills the chip
  if ((e = launch_segments(ctx->stream, true, d_clear, d_out, P, n, ctx->status.as<int32_t>(), sc,
                           grid_waves_for(n + ec))) != hipSuccess)
    return ctx->hip_fail(e, "seal segments");
  ctx->tend(t);
  t = ctx->tbegin("finalize_seal");
  if ((e = launch_finalize_multi(ctx->stream, true, d_out, P, ctx->status.as<int32_t>(), sc, n)) !=
      hipSuccess)
    return ctx->hip_fail(e, "seal finalize");
  ctx->tend(t);
  return CE_OK;
}

int seal_one(ce_ctx* ctx, const KeyRef& key, const uint8_t* outer_version, const uint8_t* nonce,
             const uint8_t* clear_in, size_t clear_in_len, std::vector<uint8_t>* file,
             const uint8_t* prefix16) {
  if (int32_t ks = key_status(key)) return ctx->fail(ks, "key rejected");
  const size_t pl = prefix16 ? 16 : 0;
  const size_t clear_len = pl + clear_in_len;
  const uint64_t pre = outer_version ? 16 : 0;
  const uint64_t total = pre + sealed_len(clear_len);
  uint8_t nb[24];
  if (nonce) std::memcpy(nb, nonce, 24);
  else os_random(nb, 24);
  hipError_t e;
  // one pinned upload: clear text, then at A = align256(clear_len) the small arguments
  // [offs(2) | out_offs(1) | nonce(24 B) | outer version(16 B)]
  const uint64_t A = (clear_len + 255) & ~255ull;
  if ((e = ctx->blob.reserve(A + 128)) != hipSuccess ||
      (e = ctx->out.reserve(total + 64)) != hipSuccess ||
      (e = ctx->h_stage.reserve(std::max<uint64_t>(A + 128, total) + 256)) != hipSuccess)
    return ctx->hip_fail(e, "seal_one reserve");
  uint8_t* hs = ctx->h_stage.as<uint8_t>();
  const uint64_t args[3] = {0, clear_len, 0};
  if (pl) std::memcpy(hs, prefix16, 16);
  std::memcpy(hs + pl, clear_in, clear_in_len);
  std::memcpy(hs + A, args, 24);
  std::memcpy(hs + A + 24, nb, 24);
  if (outer_version) std::memcpy(hs + A + 48, outer_version, 16);
  if ((e = hipMemcpyAsync(ctx->blob.p, hs, A + 64, hipMemcpyHostToDevice, ctx->stream)))
    return ctx->hip_fail(e, "seal_one upload");
  uint8_t* db = ctx->blob.as<uint8_t>();
  int rc = device_seal(ctx, db, reinterpret_cast<const uint64_t*>(db + A), 1, clear_len,
                       outer_version ? db + A + 48 : nullptr, db + A + 24, ctx->out.as<uint8_t>(),
                       reinterpret_cast<const uint64_t*>(db + A + 16), key);
  if (rc) return rc;
  if ((e = hipMemcpyAsync(hs, ctx->out.p, total, hipMemcpyDeviceToHost, ctx->stream)) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "seal_one download");
  file->resize(total);
  std::memcpy(file->data(), hs, total);
  return CE_OK;
}

}  // namespace ce

using namespace ce;

extern "C" {

const char* ce_status_str(int s) {
  switch (s) {
    case CE_OK: return "ok";
    case CE_ERR_OUTER_LEN: return "invalid length";
    case CE_ERR_OUTER_VERSION: return "version check failed";
    case CE_ERR_KEY_VERSION: return "not matching key version";
    case CE_ERR_KEY_LEN: return "Invalid key length";
    case CE_ERR_PARSE_VBOX: return "failed to parse version box";
    case CE_ERR_DATA_VERSION: return "not matching version of encryption box";
    case CE_ERR_PARSE_ENCBOX: return "failed to parse encryption box";
    case CE_ERR_NONCE_LEN: return "Invalid nonce length";
    case CE_ERR_AUTH: return "Decryption failed";
    case CE_ERR_PT_LEN: return "invalid length";
    case CE_ERR_PT_VERSION: return "version check failed";
    case CE_ERR_DECODE: return "failed to decode msgpack";
    case CE_ERR_OP_VERSION: return "Unexpected op version. Got ops in the wrong order? Bug in storage?";
    case CE_ERR_INVALID_ARG: return "invalid argument";
    case CE_ERR_DEVICE: return "HIP device error";
    case CE_ERR_NO_KEY: return "no latest key";
    case CE_ERR_IO: return "io error";
    case CE_ERR_NO_LOCAL_META: return "local meta does not exist, and `create` option is not set";
    case CE_ERR_SHARD: return "sharded ingest: partition contract broken or next_op_versions differ";
    default: return "unknown";
  }
}

void ce_buf_free(ce_buf* b) {
  if (b && b->data) free(b->data);
  if (b) { b->data = nullptr; b->len = 0; }
}

static int buf_set(ce_buf* out, const uint8_t* d, size_t n) {
  out->data = (uint8_t*)malloc(n ? n : 1);
  if (!out->data) return CE_ERR_INVALID_ARG;
  if (n) std::memcpy(out->data, d, n);
  out->len = n;
  return CE_OK;
}

int ce_ctx_create(int device, ce_ctx** out) {
  if (!out) return CE_ERR_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0)
    return CE_ERR_DEVICE;  // no GPU: the product has no CPU path
  if (hipSetDevice(device) != hipSuccess) return CE_ERR_DEVICE;
  // CE_SPIN=1 (diagnostics): host waits spin instead of yielding (wake-up latency of the
  // per-step synchronisations)
  if (const char* sp = getenv("CE_SPIN")) {
    if (atoi(sp)) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  }
  ce_ctx* c = new ce_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return CE_ERR_DEVICE;
  }
  c->own_stream = true;
  // the counter block is addressed by every batch path (gate flags live in it): allocate it
  // with the context, not on first use
  if (c->counters.reserve(256) != hipSuccess || c->h_counters.reserve(256) != hipSuccess ||
      hipMemset(c->counters.p, 0, 256) != hipSuccess) {
    ce_ctx_destroy(c);
    return CE_ERR_DEVICE;
  }
  *out = c;
  return CE_OK;
}

void ce_ctx_destroy(ce_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& t : c->timed) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->setup_ev) (void)hipEventDestroy(c->setup_ev);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  if (c->side_ev) (void)hipEventDestroy(c->side_ev);
  if (c->up_ev) (void)hipEventDestroy(c->up_ev);
  if (c->spin_ev) (void)hipEventDestroy(c->spin_ev);
  destroy_uploader(c);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int ce_ctx_set_stream(ce_ctx* c, void* s) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipStreamSynchronize(c->stream);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  if (s) {
    c->stream = (hipStream_t)s;
    c->own_stream = false;
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return CE_ERR_DEVICE;
    c->own_stream = true;
  }
  return CE_OK;
}

void ce_ctx_synchronize(ce_ctx* c) {
  if (c) (void)hipStreamSynchronize(c->stream);
}

const char* ce_ctx_last_error(ce_ctx* c) { return c ? c->last_error.c_str() : ""; }

int ce_ctx_set_timing(ce_ctx* c, int enable) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->timing = enable != 0;
  return CE_OK;
}

int ce_ctx_set_timing_only(ce_ctx* c, const char* kernel) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->timing_only = kernel ? kernel : "";
  return CE_OK;
}

int ce_ctx_clock_probe(ce_ctx* c, void* hip_stream, uint64_t* d_out, uint32_t blocks,
                       uint32_t samples, uint32_t ticks) {
  if (!c || !d_out || blocks == 0 || blocks > 4096 || samples == 0 || ticks == 0 ||
      (uint64_t)samples * ticks > 100000000ull)
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  const hipError_t e = launch_clock_probe(hip_stream ? (hipStream_t)hip_stream : c->stream,
                                          reinterpret_cast<unsigned long long*>(d_out), blocks,
                                          samples, ticks);
  return e == hipSuccess ? CE_OK : c->hip_fail(e, "clock probe");
}

int ce_ctx_timing_read(ce_ctx* c, const char* kernel, double* total_ms, uint64_t* launches) {
  if (!c || !kernel || !total_ms || !launches) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipStreamSynchronize(c->stream);
  double tot = 0;
  uint64_t cnt = 0;
  for (auto& t : c->timed) {
    if (std::strcmp(t.name, kernel) != 0) continue;
    float ms = 0;
    if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) { tot += ms; cnt++; }
  }
  *total_ms = tot;
  *launches = cnt;
  return CE_OK;
}

void ce_ctx_timing_reset(ce_ctx* c) {
  if (!c) return;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipStreamSynchronize(c->stream);
  for (auto& t : c->timed) { c->event_pool.push_back(t.a); c->event_pool.push_back(t.b); }
  c->timed.clear();
}

size_t ce_cryptor_sealed_len(size_t clear_len) { return (size_t)sealed_len(clear_len); }

int ce_cryptor_gen_key(ce_ctx* c, ce_buf* out) {
  (void)c;
  if (!out) return CE_ERR_INVALID_ARG;
  uint8_t vb[48];
  std::memcpy(vb, kKeyVersion, 16);
  os_random(vb + 16, 32);  // xchacha lib.rs:29-38 (rand::rng)
  return buf_set(out, vb, 48);
}

int ce_cryptor_encrypt(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                       size_t key_len, const uint8_t* nonce, const uint8_t* clear,
                       size_t clear_len, ce_buf* out) {
  if (!c || !key_version || !out || (clear_len && !clear)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  KeyRef k{key_version, key, key_len};
  std::vector<uint8_t> file;
  int rc = seal_one(c, k, nullptr, nonce, clear, clear_len, &file);
  if (rc) return rc;
  return buf_set(out, file.data(), file.size());
}

int ce_cryptor_decrypt_batch(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                             size_t key_len, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                             uint8_t* out_blob, uint64_t* out_offs, uint64_t* out_lens,
                             int32_t* status) {
  if (!c || !key_version || !offs || !out_blob || !out_offs || !out_lens || !status)
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  KeyRef k{key_version, key, key_len};
  // Cryptor::decrypt checks the key before anything else (xchacha lib.rs:74-78)
  if (int32_t ks = key_status(k)) {
    for (uint32_t i = 0; i < n; i++) { status[i] = ks; out_lens[i] = 0; out_offs[i] = 0; }
    return n ? ks : CE_OK;
  }
  if (n == 0) return CE_OK;
  const uint64_t blen = offs[n];
  hipError_t e;
  if ((e = c->blob.reserve(blen + 64)) || (e = c->offs.reserve((n + 1) * 8ull)) ||
      (e = c->out.reserve(blen + 16ull * n + 128)))
    return c->hip_fail(e, "decrypt_batch reserve");
  if ((e = hipMemcpyAsync(c->blob.p, blob, blen, hipMemcpyHostToDevice, c->stream)) ||
      (e = hipMemcpyAsync(c->offs.p, offs, (n + 1) * 8ull, hipMemcpyHostToDevice, c->stream)))
    return c->hip_fail(e, "decrypt_batch upload");
  int rc = device_open(c, c->blob.as<uint8_t>(), c->offs.as<uint64_t>(), n, blen, false, k,
                       c->out.as<uint8_t>(), c->status.as<int32_t>(), false);
  if (rc) return rc;
  std::vector<FileParams> P(n);
  if ((e = hipMemcpyAsync(status, c->status.p, n * 4ull, hipMemcpyDeviceToHost, c->stream)) ||
      (e = hipMemcpyAsync(P.data(), c->params.p, n * sizeof(FileParams), hipMemcpyDeviceToHost,
                          c->stream)) ||
      (e = hipMemcpyAsync(out_blob, c->out.p, blen + 16ull * n, hipMemcpyDeviceToHost, c->stream)) ||
      (e = stream_wait(c->stream)))
    return c->hip_fail(e, "decrypt_batch download");
  int first = CE_OK;
  for (uint32_t i = 0; i < n; i++) {
    out_offs[i] = P[i].out_off;
    out_lens[i] = status[i] == CE_OK ? P[i].len : 0;
    if (status[i] == kStatusHostParse) {
      // exotic byte-string encoding: not decoded in place on the device
      status[i] = CE_ERR_PARSE_ENCBOX;
    }
    if (status[i] != CE_OK && first == CE_OK) first = status[i];
  }
  return first;
}

int ce_cryptor_decrypt(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                       size_t key_len, const uint8_t* enc, size_t enc_len, ce_buf* out) {
  if (!c || !out || (enc_len && !enc)) return CE_ERR_INVALID_ARG;
  const uint64_t offs[2] = {0, enc_len};
  std::vector<uint8_t> ob(enc_len + 16 + 64);
  uint64_t oo = 0, ol = 0;
  int32_t st = 0;
  int rc = ce_cryptor_decrypt_batch(c, key_version, key, key_len, enc, offs, 1, ob.data(), &oo,
                                    &ol, &st);
  if (rc) return rc;
  return buf_set(out, ob.data() + oo, ol);
}

int ce_cryptor_encrypt_batch(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                             size_t key_len, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                             const uint8_t* nonces, uint8_t* out_blob, size_t out_cap,
                             uint64_t* out_offs) {
  if (!c || !key_version || !offs || !out_offs) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  KeyRef k{key_version, key, key_len};
  if (int32_t ks = key_status(k)) return ks;
  out_offs[0] = 0;
  for (uint32_t i = 0; i < n; i++) out_offs[i + 1] = out_offs[i] + sealed_len(offs[i + 1] - offs[i]);
  if (n == 0) return CE_OK;
  if (out_offs[n] > out_cap || !out_blob) return CE_ERR_INVALID_ARG;
  const uint64_t blen = offs[n];
  std::vector<uint8_t> nb;
  if (!nonces) {
    nb.resize(24ull * n);
    os_random(nb.data(), nb.size());
    nonces = nb.data();
  }
  hipError_t e;
  if ((e = c->blob.reserve(blen + 64)) || (e = c->offs.reserve((n + 1) * 8ull)) ||
      (e = c->out_offs.reserve((n + 1) * 8ull)) || (e = c->nonces.reserve(24ull * n)) ||
      (e = c->out.reserve(out_offs[n] + 64)))
    return c->hip_fail(e, "encrypt_batch reserve");
  if ((e = hipMemcpyAsync(c->blob.p, blob, blen, hipMemcpyHostToDevice, c->stream)) ||
      (e = hipMemcpyAsync(c->offs.p, offs, (n + 1) * 8ull, hipMemcpyHostToDevice, c->stream)) ||
      (e = hipMemcpyAsync(c->out_offs.p, out_offs, (n + 1) * 8ull, hipMemcpyHostToDevice, c->stream)) ||
      (e = hipMemcpyAsync(c->nonces.p, nonces, 24ull * n, hipMemcpyHostToDevice, c->stream)))
    return c->hip_fail(e, "encrypt_batch upload");
  int rc = device_seal(c, c->blob.as<uint8_t>(), c->offs.as<uint64_t>(), n, blen, nullptr,
                       c->nonces.as<uint8_t>(), c->out.as<uint8_t>(), c->out_offs.as<uint64_t>(), k);
  if (rc) return rc;
  if ((e = hipMemcpyAsync(out_blob, c->out.p, out_offs[n], hipMemcpyDeviceToHost, c->stream)) ||
      (e = stream_wait(c->stream)))
    return c->hip_fail(e, "encrypt_batch download");
  return CE_OK;
}

int ce_cryptor_decrypt_batch_device(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                                    size_t key_len, const uint8_t* d_blob, const uint64_t* d_offs,
                                    uint32_t n, uint8_t* d_out, int32_t* d_status,
                                    uint32_t* n_failed) {
  if (!c || !key_version || !d_blob || !d_offs || !d_out) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  KeyRef k{key_version, key, key_len};
  uint64_t blen = 0;
  hipError_t e;
  if (n && ((e = hipMemcpyAsync(&blen, d_offs + n, 8, hipMemcpyDeviceToHost, c->stream)) ||
            (e = stream_wait(c->stream))))
    return c->hip_fail(e, "decrypt_batch_device offs");
  int32_t* st = d_status;
  if (!st) {
    if ((e = c->status.reserve(n * 4ull + 64))) return c->hip_fail(e, "status");
    st = c->status.as<int32_t>();
  }
  int rc = device_open(c, d_blob, d_offs, n, blen, false, k, d_out, st, n_failed != nullptr);
  if (rc) return rc;
  if (n_failed) {
    const uint32_t* hc = c->h_counters.as<uint32_t>();
    *n_failed = hc[2];
  }
  return CE_OK;
}

int ce_cryptor_encrypt_batch_device(ce_ctx* c, const uint8_t key_version[16], const uint8_t* key,
                                    size_t key_len, const uint8_t* outer_version,
                                    const uint8_t* d_clear, const uint64_t* d_offs, uint32_t n,
                                    const uint8_t* d_nonces, uint8_t* d_out,
                                    const uint64_t* d_out_offs) {
  if (!c || !key_version || !d_clear || !d_offs || !d_nonces || !d_out || !d_out_offs)
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  KeyRef k{key_version, key, key_len};
  uint64_t blen = 0;
  hipError_t e;
  if (n && ((e = hipMemcpyAsync(&blen, d_offs + n, 8, hipMemcpyDeviceToHost, c->stream)) ||
            (e = stream_wait(c->stream))))
    return c->hip_fail(e, "encrypt_batch_device offs");
  const uint8_t* dov = nullptr;
  if (outer_version) {
    if ((e = c->outer_ver.reserve(64)) ||
        (e = hipMemcpyAsync(c->outer_ver.p, outer_version, 16, hipMemcpyHostToDevice, c->stream)))
      return c->hip_fail(e, "outer version");
    dov = c->outer_ver.as<uint8_t>();
  }
  return device_seal(c, d_clear, d_offs, n, blen, dov, d_nonces, d_out, d_out_offs, k);
}

}  // extern "C"
