// ce_upload.cpp -- host buffers -> HBM for the host-buffer entry points (what a Rust caller has
// after Storage::load_ops: one Vec<u8> per file, crdt-enc/src/lib.rs:495 and
// crdt-enc-tokio/src/lib.rs:222-278).
//
// The files are gathered, chunk by chunk, into a ring of four pinned 32 MiB staging buffers by a
// pool of host threads (pinned to the GPU's NUMA node when it has room for them), and each filled
// chunk is DMA'd to its place in the device blob on the context's copy stream while the threads
// fill the next ones.  Measured on the box (tools/h2d_probe.py):
// host memcpy reaches ~120 GB/s on 8-16 threads, H2D DMA ~57 GB/s, so the pipeline runs at the
// PCIe rate.  The compute stream waits for the last chunk with an event (no host synchronise);
// the kernels then run on the whole batch.
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <fstream>
#include <functional>
#include <sstream>
#include <thread>

#include "ce_core.h"

namespace ce {

// The CPUs of the GPU's NUMA node that this process may run on (empty: unknown, or none
// allowed): the gather threads copy into pinned staging the GPU's DMA engine reads, so on a
// multi-socket host they run next to it.  CE_UPLOAD_NUMA=0 disables the pinning.
static std::vector<int> gpu_node_cpus(int device) {
  std::vector<int> out;
  const char* env = getenv("CE_UPLOAD_NUMA");
  if (env && env[0] == '0') return out;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return out;
  std::string id(bus);
  for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
  int node = -1;
  {
    std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
    if (!(f >> node) || node < 0) return out;
  }
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!std::getline(f, list)) return out;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
  std::stringstream ss(list);
  std::string part;
  while (std::getline(ss, part, ',')) {
    int a = -1, b = -1;
    if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
    } else if (sscanf(part.c_str(), "%d", &a) == 1) {
      b = a;
    } else {
      continue;
    }
    for (int c = a; c <= b && c < CPU_SETSIZE; c++)
      if (c >= 0 && CPU_ISSET(c, &allowed)) out.push_back(c);
  }
  return out;
}

// A fixed pool of host threads for parallel_for (gather copies).
struct HostPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::function<void(int)> job;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
  int numa_cpus = 0;  // CPUs of the GPU's node the threads were pinned to (0: not pinned)

  explicit HostPool(int n, int device = -1) {
    const std::vector<int> cpus = device >= 0 ? gpu_node_cpus(device) : std::vector<int>{};
    // pin only when the node has room for the whole pool (else the threads would share cores)
    const bool pin = (int)cpus.size() >= n;
    if (pin) numa_cpus = (int)cpus.size();
    for (int i = 0; i < n; i++)
      th.emplace_back([this, i, pin, cpus] {
        if (pin) {
          cpu_set_t set;
          CPU_ZERO(&set);
          for (int c : cpus) CPU_SET(c, &set);
          (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
        }
        uint64_t seen = 0;
        for (;;) {
          std::function<void(int)> f;
          {
            std::unique_lock<std::mutex> l(mu);
            cv.wait(l, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            f = job;
          }
          f(i);
          std::lock_guard<std::mutex> l(mu);
          if (--pending == 0) done_cv.notify_all();
        }
      });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  int size() const { return (int)th.size(); }
  void run(const std::function<void(int)>& f) {
    std::unique_lock<std::mutex> l(mu);
    job = f;
    pending = (int)th.size();
    gen++;
    cv.notify_all();
    done_cv.wait(l, [&] { return pending == 0; });
  }
};

// A ring of kRing pinned chunks: the threads fill chunk k + 1.. while the DMAs of the earlier
// ones run back to back on the copy stream; a chunk is refilled once its DMA is done.
static constexpr int kRing = 4;
struct Uploader {
  size_t chunk = 32ull << 20;  // CE_UPLOAD_CHUNK (bytes) overrides: tests force many chunks
  hipStream_t copy = nullptr;
  HostBuf stage[kRing];
  hipEvent_t ev[kRing] = {}, t0 = nullptr, t1 = nullptr, order = nullptr;
  bool used[kRing] = {};
  ~Uploader() {
    if (copy) (void)hipStreamSynchronize(copy);
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : {t0, t1, order})
      if (e) (void)hipEventDestroy(e);
    if (copy) (void)hipStreamDestroy(copy);
  }
};

static int pool_threads() {
  // the job's CPU share (OMP_NUM_THREADS is 16 on the GPU box), at most 16
  int n = (int)std::thread::hardware_concurrency();
  if (const char* e = getenv("OMP_NUM_THREADS")) n = std::min(n, std::max(1, atoi(e)));
  if (const char* e = getenv("CE_UPLOAD_THREADS")) n = std::max(1, atoi(e));
  return std::max(1, std::min(n, 16));
}

static int get_uploader(ce_ctx* ctx, Uploader** out) {
  if (!ctx->up) {
    auto* u = new Uploader();
    if (const char* c = getenv("CE_UPLOAD_CHUNK")) u->chunk = std::max<size_t>(4096, strtoull(c, nullptr, 10));
    hipError_t e = hipStreamCreateWithFlags(&u->copy, hipStreamNonBlocking);
    for (int k = 0; k < kRing && e == hipSuccess; k++)
      if ((e = hipEventCreateWithFlags(&u->ev[k], hipEventDisableTiming)) == hipSuccess) e = u->stage[k].reserve(u->chunk);
    if (e || (e = hipEventCreate(&u->t0)) || (e = hipEventCreate(&u->t1)) ||
        (e = hipEventCreateWithFlags(&u->order, hipEventDisableTiming))) {
      delete u;
      return ctx->hip_fail(e, "uploader");
    }
    ctx->up = u;
  }
  *out = ctx->up;
  return CE_OK;
}

static HostPool* get_pool(ce_ctx* ctx) {
  if (!ctx->pool) ctx->pool = new HostPool(pool_threads(), ctx->device);
  return ctx->pool;
}

void destroy_uploader(ce_ctx* ctx) {
  delete ctx->up;
  ctx->up = nullptr;
  delete ctx->pool;
  ctx->pool = nullptr;
}

void host_parallel_for(ce_ctx* ctx, uint32_t n, const std::function<void(uint32_t)>& fn) {
  if (n < 2) {
    for (uint32_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<uint32_t> next{0};
  get_pool(ctx)->run([&](int) {
    for (uint32_t i; (i = next.fetch_add(1)) < n;) fn(i);
  });
}

// Logical blob = files[0] || files[1] || ... (offs: n+1 prefix sums).  Upload it into d_dst on
// the copy stream through the pinned ring; ctx->stream waits for the last chunk.
int upload_iov(ce_ctx* ctx, const uint8_t* const* files, const uint64_t* offs, uint32_t n,
               uint8_t* d_dst) {
  Uploader* u;
  int rc = get_uploader(ctx, &u);
  if (rc) return rc;
  const uint64_t total = offs[n];
  hipError_t e;
  // d_dst may still be read by work queued on the compute stream: the copies wait for it
  if ((e = hipEventRecord(u->order, ctx->stream)) || (e = hipStreamWaitEvent(u->copy, u->order, 0)))
    return ctx->hip_fail(e, "upload order");
  if ((e = hipEventRecord(u->t0, u->copy))) return ctx->hip_fail(e, "upload");
  int tl = -1;  // ce_ctx_set_timing: "upload" spans the DMA on the copy stream
  if (ctx->timing) {
    ce_ctx::TimedLaunch t{"upload", ctx->take_event(), ctx->take_event()};
    (void)hipEventRecord(t.a, u->copy);
    ctx->timed.push_back(t);
    tl = (int)ctx->timed.size() - 1;
  }
  HostPool* pool = get_pool(ctx);
  const int T = pool->size();
  for (uint64_t c0 = 0, k = 0; c0 < total; c0 += u->chunk, k = (k + 1) % kRing) {
    const uint64_t len = std::min<uint64_t>(u->chunk, total - c0);
    if (u->used[k] && (e = hipEventSynchronize(u->ev[k]))) return ctx->hip_fail(e, "upload ring");
    uint8_t* st = u->stage[k].as<uint8_t>();
    pool->run([&](int t) {
      uint64_t lo = c0 + len * t / T, hi = c0 + len * (t + 1) / T;
      if (lo >= hi) return;
      // first file overlapping lo
      uint32_t f = (uint32_t)(std::upper_bound(offs, offs + n + 1, lo) - offs) - 1;
      while (lo < hi && f < n) {
        const uint64_t fe = std::min<uint64_t>(offs[f + 1], hi);
        if (fe > lo) std::memcpy(st + (lo - c0), files[f] + (lo - offs[f]), fe - lo);
        lo = std::max(lo, fe);
        f++;
      }
    });
    if ((e = hipMemcpyAsync(d_dst + c0, st, len, hipMemcpyHostToDevice, u->copy)) ||
        (e = hipEventRecord(u->ev[k], u->copy)))
      return ctx->hip_fail(e, "upload chunk");
    u->used[k] = true;
  }
  if ((e = hipEventRecord(u->t1, u->copy)) || (e = hipStreamWaitEvent(ctx->stream, u->t1, 0)))
    return ctx->hip_fail(e, "upload join");
  if (tl >= 0) (void)hipEventRecord(ctx->timed[tl].b, u->copy);
  return CE_OK;
}

// Host files -> ctx->blob / ctx->offs (device) for a host-buffer entry point.  files[i] holds
// offs[i+1] - offs[i] bytes (offs: n+1 host prefix sums).
int stage_host_batch(ce_ctx* ctx, const uint8_t* const* files, const uint64_t* offs, uint32_t n) {
  hipError_t e;
  const uint64_t blen = offs[n];
  if ((e = ctx->blob.reserve(blen + 64)) || (e = ctx->offs.reserve((n + 1) * 8ull)))
    return ctx->hip_fail(e, "ingest reserve");
  // pageable source: staged by the runtime before the call returns (offs may be a temporary)
  if ((e = hipMemcpyAsync(ctx->offs.p, offs, (n + 1) * 8ull, hipMemcpyHostToDevice, ctx->stream)))
    return ctx->hip_fail(e, "ingest offsets");
  return upload_iov(ctx, files, offs, n, ctx->blob.as<uint8_t>());
}

}  // namespace ce
