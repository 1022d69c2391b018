// ce_internal.h -- host-side internals shared by ce_ctx.cpp, ce_storage.cpp, ce_core.cpp.
#pragma once
#include <utility>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <sched.h>

#include <array>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <functional>
#include <vector>

#include "ce_common.h"
#include "ce_kernels.h"
#include "crdtenc.h"

namespace ce {

using Uuid = std::array<uint8_t, 16>;

struct UuidHash {
  size_t operator()(const Uuid& u) const {
    uint32_t w[4];
    std::memcpy(w, u.data(), 16);
    return actor_hash(w[0], w[1], w[2], w[3]);
  }
};

std::string uuid_to_string(const Uuid& u);              // lowercase hyphenated
bool uuid_parse(const std::string& s, Uuid* out);       // Uuid::from_str formats
void os_random(uint8_t* out, size_t n);                 // getrandom(2)
Uuid uuid_v4();
void sha3_256(const uint8_t* msg, size_t len, uint8_t out[32]);
std::string base32_nopad(const uint8_t* in, size_t len);

// growable device buffer
// Owning buffers are move-only: a copy would free the same allocation twice (a vector of them
// that grows moves its elements).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
    return *this;
  }
  hipError_t reserve(size_t bytes);
  ~DevBuf();
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// growable pinned host buffer
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  HostBuf(HostBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
  HostBuf& operator=(HostBuf&& o) noexcept {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
    return *this;
  }
  hipError_t reserve(size_t bytes);
  ~HostBuf();
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Wait for everything queued on `s` by polling an event (the blocking wait's wake-up costs tens
// of microseconds on the box; the dot-set paths wait many times per step), yielding the core
// between polls after the first few.  CE_SYNC_YIELD=1: hipStreamSynchronize.
inline hipError_t stream_wait(hipStream_t s) {
  static const bool yield = getenv("CE_SYNC_YIELD") != nullptr;
  if (yield) return hipStreamSynchronize(s);
  thread_local hipEvent_t evs[64] = {};  // per device: an event belongs to the device it was made on
  int dev = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev))) return e;
  if (dev < 0 || dev >= 64) return hipStreamSynchronize(s);
  hipEvent_t& ev = evs[dev];
  if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return e;
  if ((e = hipEventRecord(ev, s))) return e;
  for (unsigned i = 0; (e = hipEventQuery(ev)) == hipErrorNotReady; i++)
    if (i >= 32) sched_yield();
  return e;
}

// A point on `s` to wait for later while the work queued after it keeps running (stream_mark),
// and the wait (mark_wait: the same polling as stream_wait).  One mark per thread and device is
// live at a time.
inline hipError_t stream_mark(hipStream_t s, hipEvent_t* out) {
  thread_local hipEvent_t evs[64] = {};
  int dev = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev))) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  hipEvent_t& ev = evs[dev];
  if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return e;
  *out = ev;
  return hipEventRecord(ev, s);
}

inline hipError_t mark_wait(hipEvent_t ev) {
  hipError_t e;
  for (unsigned i = 0; (e = hipEventQuery(ev)) == hipErrorNotReady; i++)
    if (i >= 32) sched_yield();
  return e;
}

struct KeyRef {
  const uint8_t* version;  // 16
  const uint8_t* key;
  size_t len;
};

// Result of a device open pass.
struct OpenResult {
  uint32_t auth_failed = 0;
  uint32_t first_fail = 0xffffffffu;
};

}  // namespace ce

namespace ce {
struct Uploader;  // ce_upload.cpp: pinned staging ring + copy stream
struct HostPool;  // ce_upload.cpp: host worker threads (gather copies, per-file host parsing)
}

struct ce_storage {
  std::string local, remote;  // crdt-enc-tokio Storage{local_path, remote_path} (lib.rs:22-26)
};

struct ce_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::recursive_mutex mu;
  std::string last_error;
  // batch scratch (device)
  ce::DevBuf params, status, counters, extra, multi, partials, large, out, apply, refold, miss,
      supported, blob, offs, nonces, out_offs, outer_ver, batch_counters, split, segrec, redo, heads,
      poly_aux;  // PolyAux rows of the fused open (device_open_setup)
  ce::HostBuf h_counters, h_apply, h_stage, h_stage2, h_heads;
  uint32_t publish_gen = 0;  // k_publish_words generations (the setup's counters, C2 path)
  // marks the setup kernel's counter snapshot (h_counters + 128) as landed on the host
  hipEvent_t setup_ev = nullptr;
  // a side stream for readbacks that must not sit between the main stream's kernels (the setup
  // counters), and the event it waits on
  hipStream_t side = nullptr;
  hipEvent_t side_ev = nullptr;
  hipEvent_t up_ev = nullptr;  // the side stream's uploads (the main stream waits on it)
  ce::Uploader* up = nullptr;  // host-buffer entry points (created on first use)
  ce::HostPool* pool = nullptr;  // created on first use
  // kernel timing (ce_ctx_set_timing)
  bool timing = false;
  struct TimedLaunch {
    const char* name;
    hipEvent_t a, b;
  };
  std::vector<TimedLaunch> timed;
  std::vector<hipEvent_t> event_pool;
  hipEvent_t take_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  // brackets one launch: t0 = begin(name) ... end(t0)
  std::string timing_only;  // ce_ctx_set_timing_only: time one kernel name ("" = all)
  int tbegin(const char* name) {
    if (!timing || (!timing_only.empty() && timing_only != name)) return -1;
    TimedLaunch t{name, take_event(), take_event()};
    (void)hipEventRecord(t.a, stream);
    timed.push_back(t);
    return (int)timed.size() - 1;
  }
  void tend(int idx) {
    if (idx >= 0) (void)hipEventRecord(timed[idx].b, stream);
  }
  // a timed launch whose dispatch records the two events itself (hipExtLaunchKernel): *a / *b
  // stay null when the name is not timed
  int tlaunch(const char* name, hipEvent_t* a, hipEvent_t* b) {
    *a = *b = nullptr;
    if (!timing || (!timing_only.empty() && timing_only != name)) return -1;
    TimedLaunch t{name, take_event(), take_event()};
    *a = t.a;
    *b = t.b;
    timed.push_back(t);
    return (int)timed.size() - 1;
  }

  // stream synchronise by polling an event (CE_SYNC_YIELD=1: hipStreamSynchronize).  The
  // blocking wait's wake-up costs tens of microseconds per step on the box; a step waits once.
  // The poll yields the core between queries after the first few, so the library does not hold a
  // host core against the upload pool or other ranks' threads for a whole kernel.
  hipEvent_t spin_ev = nullptr;
  hipError_t sync_spin() {
    static const bool yield = getenv("CE_SYNC_YIELD") != nullptr;
    if (yield) return hipStreamSynchronize(stream);
    hipError_t e;
    if (!spin_ev && (e = hipEventCreateWithFlags(&spin_ev, hipEventDisableTiming))) return e;
    if ((e = hipEventRecord(spin_ev, stream))) return e;
    for (unsigned i = 0; (e = hipEventQuery(spin_ev)) == hipErrorNotReady; i++)
      if (i >= 32) sched_yield();
    return e;
  }

  int fail(int code, const std::string& msg) {
    last_error = msg;
    return code;
  }
  int hip_fail(hipError_t e, const char* where) {
    last_error = std::string(where) + ": " + hipGetErrorString(e);
    return CE_ERR_DEVICE;
  }
};

namespace ce {

int32_t key_status(const KeyRef& k);
DevKey dev_key(const KeyRef& k);

// Open n files resident in HBM (d_blob/d_offs) on ctx's stream; plaintexts land in ctx->out.
// outer: files carry the core's 16-byte version prefix.  After the call ctx->status holds the
// per-file statuses and ctx->params the FileParams; counters are copied to h_counters.
int device_open_setup(ce_ctx* ctx, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                      uint64_t blob_len, bool outer, const KeyRef& key, int32_t* d_status,
                      uint32_t* extra_cap, FillArgs* fills = nullptr,
                      const std::function<int()>* after_fill = nullptr);
SegScratch segscratch(ce_ctx* ctx, uint32_t extra_cap);
int device_open(ce_ctx* ctx, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                uint64_t blob_len, bool outer, const KeyRef& key, uint8_t* d_out,
                int32_t* d_status, bool sync_counters, bool small_lanes = false,
                const DecodeArgs* ds = nullptr);
// (ds: small_lanes only -- Orswot op files decoded in the open: ds->ds, supported / n_supported,
// table / mask are taken from it; ce_fused.hip ds_fused_decode)

// Seal n clear texts resident in HBM.  d_out_offs[i] = output start of file i.
// counters_ready: the caller's kernel already reset ctx's counter block (k_compact_prologue)
int device_seal(ce_ctx* ctx, const uint8_t* d_clear, const uint64_t* d_offs, uint32_t n,
                uint64_t clear_len_total, const uint8_t* d_outer_version, const uint8_t* d_nonces,
                uint8_t* d_out, const uint64_t* d_out_offs, const KeyRef& key, bool counters_ready = false);
// ctx's counter block (device), allocated on first use
uint32_t* ctx_counters(ce_ctx* ctx);

// Seal one host clear text into a host file: [outer(16)] || Cryptor::encrypt([prefix16] ||
// clear).  `file` keeps its capacity across calls (the pinned staging buffer is the only copy
// of the clear text the seal makes).
int seal_one(ce_ctx* ctx, const KeyRef& key, const uint8_t* outer_version, const uint8_t* nonce,
             const uint8_t* clear, size_t clear_len, std::vector<uint8_t>* file,
             const uint8_t* prefix16 = nullptr);

uint32_t grid_waves_for(uint32_t work);

// ce_dma.cpp: device -> host copies on an SDMA engine (HSA), completion on a signal
struct DmaD2H {
  bool ok = false;
  hsa_agent_t gpu{0}, cpu{0};
  uint32_t engine = 0;  // hsa_amd_sdma_engine_id_t bit, 0: the runtime's choice
};
bool dma_init(int device, DmaD2H* out);
bool dma_d2h(const DmaD2H& d, void* dst, const void* src, size_t n, hsa_signal_t sig);  // false: not issued
void dma_wait(hsa_signal_t sig);
bool dma_signal(hsa_signal_t* sig);
void dma_signal_destroy(hsa_signal_t sig);

// ce_upload.cpp: host files -> ctx->blob / ctx->offs through the pinned staging ring (ordered
// before later work on ctx->stream, no host synchronise)
int stage_host_batch(ce_ctx* ctx, const uint8_t* const* files, const uint64_t* offs, uint32_t n);
void destroy_uploader(ce_ctx* ctx);
// fn(i) for i in [0, n) on the context's host threads (inline when n < 2); fn must not touch
// HIP streams or shared mutable state
void host_parallel_for(ce_ctx* ctx, uint32_t n, const std::function<void(uint32_t)>& fn);

}  // namespace ce
