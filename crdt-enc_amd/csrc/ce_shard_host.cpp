// ce_shard_host.cpp -- multi-GPU partition of VClock / GCounter op files by address, and the
// cross-rank version gate (crdt-enc/src/lib.rs:516-544) that keeps the fold identical to the
// reference's single loop over the whole batch.  Layout and semantics: ce_common.h (ShardStats,
// shard_hi); kernels: ce_shard.hip.
//
// Batch order.  The reference folds Storage::load_ops's result: each writer's files in version
// order (storage.rs:36-40), writers in whatever order the tokio listing yields them
// (crdt-enc-tokio/src/lib.rs:204-278, buffer_unordered).  Across ranks the batch order is fixed
// as the shared writer list's order -- one of the orders the reference itself may take -- which
// only matters when a gap stops the fold (the writers after it fold nothing).
//
// Per step (crdtenc shard.ingest_sharded):
//   ce_core_shard_stats -> all_reduce(MAX) -> ce_core_shard_window -> ce_core_ingest_ops_device_
//   sharded (folded, pending) -> pending batch all_reduce(MAX) with the failure flags ->
//   ce_core_pending_commit on every rank (or none: all-or-nothing across ranks, lib.rs:497-514).
#include <algorithm>
#include <cstring>
#include <numeric>

#include "ce_core.h"
#include "ce_shard.h"

using namespace ce;

namespace {

uint32_t owner_bytes(const uint8_t* actor16, uint64_t v, uint32_t world) {
  uint32_t w[4];
  std::memcpy(w, actor16, 16);
  return shard_owner(w[0], w[1], w[2], w[3], v, world);
}

// host twin of walk_owned (ce_shard.hip)
uint64_t walk_owned_host(const uint8_t* actor16, uint64_t lo, uint64_t end, uint32_t rank, uint32_t world,
                         bool* over) {
  uint64_t steps = 0;
  for (uint64_t u = lo; u < end; u++) {
    if (owner_bytes(actor16, u, world) == rank) return u;
    if (++steps >= kShardWalkLimit) { *over = true; return ~0ull; }
    if (u == ~0ull - 1) break;
  }
  return ~0ull;
}

inline long long enc(uint64_t u) { return (long long)(u ^ kShardFlip); }
inline uint64_t dec(long long x) { return (uint64_t)x ^ kShardFlip; }

// the writers' expected versions (next_op_versions.get, lib.rs:519) and UUID words -> device
int stage_writers(ce_core* c, const uint8_t* actors, uint32_t m, std::vector<uint64_t>* e0) {
  ce_ctx* ctx = c->ctx;
  e0->assign(m, 0);
  for (uint32_t a = 0; a < m; a++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * a, 16);
    auto it = c->slot_of.find(u);
    if (it != c->slot_of.end()) (*e0)[a] = c->nov[it->second];
  }
  // d_shard: writers [16m] | e0 [8m] | cand [8m] | vmaxp1 [8m] | run_count [4m] | has_ge [4m] | bad
  hipError_t e;
  if ((e = c->d_shard.reserve(48ull * m + 64))) return ctx->hip_fail(e, "shard scratch");
  uint8_t* b = c->d_shard.as<uint8_t>();
  const bool new_writers =
      c->shard_writers.size() != 16ull * m || std::memcmp(c->shard_writers.data(), actors, 16ull * m) != 0;
  if (new_writers) {
    c->shard_writers.assign(actors, actors + 16ull * m);
    if ((e = hipMemcpyAsync(b, c->shard_writers.data(), 16ull * m, hipMemcpyHostToDevice, ctx->stream)))
      return ctx->hip_fail(e, "shard writers");
  }
  if (!new_writers && c->shard_e0 == *e0) return CE_OK;  // d_shard already holds them
  c->shard_e0 = *e0;
  // staged through the pinned buffer so the copy is asynchronous
  if ((e = c->h_shard.reserve(8ull * m + 64))) return ctx->hip_fail(e, "shard e0");
  // the previous upload from this buffer has been consumed (ce_core_shard_stats waits at its end;
  // a window call's copy is ordered before anything later on the stream that could rewrite it)
  if ((e = stream_wait(ctx->stream))) return ctx->hip_fail(e, "shard e0");
  std::memcpy(c->h_shard.p, e0->data(), 8ull * m);
  if ((e = hipMemcpyAsync(b + 16ull * m, c->h_shard.p, 8ull * m, hipMemcpyHostToDevice, ctx->stream)))
    return ctx->hip_fail(e, "shard e0");
  return CE_OK;
}

}  // namespace

extern "C" {

uint32_t ce_shard_owner(const uint8_t actor[16], uint64_t version, uint32_t world) {
  if (!actor || world == 0) return 0;
  return owner_bytes(actor, version, world);
}

int ce_shard_owners(const uint8_t* actors, uint32_t m, const uint32_t* file_actor,
                    const uint64_t* file_version, uint64_t n, uint32_t world, uint32_t* owner_out) {
  if ((n && (!actors || !file_actor || !file_version || !owner_out)) || world == 0) return CE_ERR_INVALID_ARG;
  for (uint64_t i = 0; i < n; i++) {
    if (file_actor[i] >= m) return CE_ERR_INVALID_ARG;
    owner_out[i] = owner_bytes(actors + 16ull * file_actor[i], file_version[i], world);
  }
  return CE_OK;
}

uint32_t ce_shard_stats_len(uint32_t m) { return 2 * m + 3; }

int ce_shard_stats_host(const uint8_t* actors, uint32_t m, const uint64_t* e0, const uint32_t* fa,
                        const uint64_t* fv, uint64_t n, uint32_t rank, uint32_t world, int64_t* stats) {
  if ((m && (!actors || !e0)) || (n && (!fa || !fv)) || !stats || world == 0 || rank >= world)
    return CE_ERR_INVALID_ARG;
  std::vector<uint64_t> cand(m, ~0ull), vmaxp1(m, 0);
  std::vector<uint32_t> runs(m, 0);
  std::vector<uint8_t> has_ge(m, 0);
  bool bad = false;
  for (uint64_t i = 0; i < n; i++) {  // k_shard_files
    const uint32_t a = fa[i];
    if (a >= m) { bad = true; continue; }
    const uint8_t* act = actors + 16ull * a;
    const uint64_t v = fv[i];
    const bool prev = i > 0 && fa[i - 1] == a;
    const bool next = i + 1 < n && fa[i + 1] == a;
    const uint64_t pv = prev ? fv[i - 1] : 0;
    if (!prev && runs[a]++ != 0) bad = true;
    if (prev && pv > v) bad = true;
    if (owner_bytes(act, v, world) != rank) bad = true;
    if (v >= e0[a]) {
      has_ge[a] = 1;
      if (!next) vmaxp1[a] = std::max(vmaxp1[a], v + 1);
      bool over = false;
      uint64_t cc = ~0ull;
      if (!prev || pv < e0[a]) cc = walk_owned_host(act, e0[a], v, rank, world, &over);
      if (cc == ~0ull && !over && v != ~0ull)
        cc = walk_owned_host(act, v + 1, next ? fv[i + 1] : ~0ull, rank, world, &over);
      if (over) bad = true;
      cand[a] = std::min(cand[a], cc);
    }
  }
  for (uint32_t a = 0; a < m; a++) {  // k_shard_writers
    if (!has_ge[a]) {
      bool over = false;
      cand[a] = walk_owned_host(actors + 16ull * a, e0[a], ~0ull, rank, world, &over);
      if (over) bad = true;
    }
    stats[a] = enc(~cand[a]);
    stats[(uint64_t)m + a] = enc(vmaxp1[a]);
  }
  const uint64_t h = shard_e0_hash(e0, m);
  stats[2ull * m] = enc(bad ? 1 : 0);
  stats[2ull * m + 1] = enc(h);
  stats[2ull * m + 2] = enc(~h);
  return CE_OK;
}

int ce_shard_window_host(uint32_t m, const uint64_t* e0, const int64_t* stats, uint64_t* hi) {
  if ((m && !e0) || !stats || !hi) return CE_ERR_INVALID_ARG;
  const uint32_t as = shard_first_gap(m, [&](uint32_t a, uint64_t* cand, uint64_t* vmaxp1) {
    *cand = ~dec(stats[a]);
    *vmaxp1 = dec(stats[(uint64_t)m + a]);
  });
  for (uint32_t a = 0; a < m; a++)
    hi[a] = shard_hi(a, as, e0[a], ~dec(stats[a]), dec(stats[(uint64_t)m + a]));
  const uint64_t h = dec(stats[2ull * m + 1]), nh = dec(stats[2ull * m + 2]);
  hi[m] = (dec(stats[2ull * m]) ? kShardBad : 0) | (as < m ? kShardGap : 0) | (h != ~nh ? kShardE0Mismatch : 0);
  return CE_OK;
}

// The windows straight from every rank's (writer, version) metadata, gathered: the reference's
// loop (lib.rs:516-544) over the whole batch in (writer, version) order.  Used when a rank's batch
// breaks the partition contract (stats flag kShardBad), and as the checker of the stats path.
int ce_shard_window_exact(uint32_t m, const uint64_t* e0, const uint32_t* fa, const uint64_t* fv,
                          uint64_t n, uint64_t* hi) {
  if ((m && !e0) || (n && (!fa || !fv)) || !hi) return CE_ERR_INVALID_ARG;
  std::vector<uint64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  for (uint64_t i = 0; i < n; i++)
    if (fa[i] >= m) return CE_ERR_INVALID_ARG;
  std::sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) {
    return fa[x] != fa[y] ? fa[x] < fa[y] : fv[x] < fv[y];
  });
  std::vector<uint64_t> expect(e0, e0 + m);
  uint64_t flags = 0;
  uint32_t stop = m;
  for (uint64_t j = 0; j < n; j++) {
    const uint32_t a = fa[idx[j]];
    const uint64_t v = fv[idx[j]];
    if (v < expect[a]) continue;                       // already read (lib.rs:521-525)
    if (v > expect[a]) { flags |= kShardGap; stop = a; break; }  // lib.rs:527-531
    expect[a] = v + 1;                                 // applied (lib.rs:533-538)
  }
  for (uint32_t a = 0; a < m; a++) hi[a] = a > stop ? e0[a] : expect[a];
  hi[m] = flags;
  return CE_OK;
}

int ce_core_writer_versions(ce_core* c, const uint8_t* actors, uint32_t m, uint64_t* e0_out) {
  if (!c || (m && (!actors || !e0_out))) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  for (uint32_t a = 0; a < m; a++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * a, 16);
    auto it = c->slot_of.find(u);
    e0_out[a] = it == c->slot_of.end() ? 0 : c->nov[it->second];
  }
  return CE_OK;
}

int ce_core_shard_stats(ce_core* c, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                        const uint64_t* d_fv, uint32_t n, uint32_t rank, uint32_t world, int64_t* d_stats) {
  if (!c || (m && !actors) || (n && (!d_fa || !d_fv)) || !d_stats || world == 0 || rank >= world ||
      is_dotset_kind(c->kind))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  ce_ctx* ctx = c->ctx;
  std::vector<uint64_t> e0;
  int rc = stage_writers(c, actors, m, &e0);
  if (rc) return rc;
  uint8_t* b = c->d_shard.as<uint8_t>();
  ShardArgs s{};
  s.fa = d_fa;
  s.fv = d_fv;
  s.n = n;
  s.m = m;
  s.rank = rank;
  s.world = world;
  s.writers = reinterpret_cast<const uint32_t*>(b);
  s.e0 = reinterpret_cast<const uint64_t*>(b + 16ull * m);
  s.cand = reinterpret_cast<unsigned long long*>(b + 24ull * m);
  s.vmaxp1 = reinterpret_cast<unsigned long long*>(b + 32ull * m);
  s.run_count = reinterpret_cast<uint32_t*>(b + 40ull * m);
  s.has_ge = reinterpret_cast<uint32_t*>(b + 44ull * m);
  s.bad = reinterpret_cast<uint32_t*>(b + 48ull * m);
  s.stats = reinterpret_cast<long long*>(d_stats);
  FillArgs fl{};
  fl.r[0] = {reinterpret_cast<uint32_t*>(s.cand), 2ull * m, 0xffffffffu};
  fl.r[1] = {reinterpret_cast<uint32_t*>(s.vmaxp1), 4ull * m + 1, 0u};  // vmaxp1, runs, has_ge, bad
  fl.n = 2;
  hipError_t e;
  if ((e = launch_fill(ctx->stream, fl)) || (e = launch_shard_stats(ctx->stream, s, shard_e0_hash(e0.data(), m))))
    return ctx->hip_fail(e, "shard stats");
  // the caller's collective may run on another stream: the stats are complete on return
  if ((e = ctx->sync_spin())) return ctx->hip_fail(e, "shard stats");
  return CE_OK;
}

int ce_core_shard_window(ce_core* c, const uint8_t* actors, uint32_t m, const int64_t* d_stats, uint64_t* d_hi) {
  if (!c || (m && !actors) || !d_stats || !d_hi || is_dotset_kind(c->kind)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  std::vector<uint64_t> e0;
  int rc = stage_writers(c, actors, m, &e0);
  if (rc) return rc;
  const hipError_t e = launch_shard_window(c->ctx->stream, reinterpret_cast<const long long*>(d_stats),
                                           reinterpret_cast<const uint64_t*>(c->d_shard.as<uint8_t>() + 16ull * m),
                                           m, d_hi);
  return e ? c->ctx->hip_fail(e, "shard window") : CE_OK;
}

int ce_core_ingest_ops_device_sharded(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                                      uint64_t blob_len, const uint8_t* actors, uint32_t m,
                                      const uint32_t* d_fa, const uint64_t* d_fv, const uint64_t* d_hi,
                                      int32_t* status) {
  if (!c || (n && (!d_blob || !d_offs || !d_fa || !d_fv)) || (m && !actors) || !d_hi || is_dotset_kind(c->kind))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  ce_ctx* ctx = c->ctx;
  if (n) return ingest_ops_dev_sharded(c, d_blob, d_offs, n, blob_len, actors, m, d_fa, d_fv, d_hi, status);
  // no file on this rank: the windows still set next_op_versions, and the pending batch is empty
  c->pending = false;
  std::vector<uint64_t> hi(m + 1);
  hipError_t e;
  if ((e = hipMemsetAsync(c->d_batch.p, 0, c->cap * 8ull, ctx->stream)) ||
      (e = hipMemcpyAsync(hi.data(), d_hi, (m + 1) * 8ull, hipMemcpyDeviceToHost, ctx->stream)) ||
      (e = hipStreamSynchronize(ctx->stream)))
    return ctx->hip_fail(e, "sharded ingest");
  if (hi[m] & (kShardBad | kShardE0Mismatch)) return ctx->fail(CE_ERR_SHARD, "partition contract / e0");
  c->pending_nov.clear();
  for (uint32_t a = 0; a < m; a++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * a, 16);
    auto it = c->slot_of.find(u);
    const uint64_t e0 = it == c->slot_of.end() ? 0 : c->nov[it->second];
    c->pending_nov.push_back({u, std::max(e0, hi[a])});
  }
  c->pending = true;
  c->pending_gen = c->table_gen;
  return (hi[m] & kShardGap) ? CE_ERR_OP_VERSION : CE_OK;
}

int ce_core_pending_export(ce_core* c, uint64_t* d_batch, uint64_t cap_words, int* ready) {
  if (!c || !d_batch || !ready || is_dotset_kind(c->kind)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  if (!c->pending || c->pending_gen != c->table_gen) return c->ctx->fail(CE_ERR_INVALID_ARG, "no pending batch");
  // an actor outside the registered slots (the ingest inserted it, and may have grown the table
  // past the caller's buffer): not exportable, and nothing is written
  *ready = c->registered == c->size && c->cap <= cap_words ? 1 : 0;
  if (!*ready) return CE_OK;
  hipError_t e;
  if ((e = hipMemcpyAsync(d_batch, c->d_batch.p, c->cap * 8ull, hipMemcpyDeviceToDevice, c->ctx->stream)) ||
      (e = c->ctx->sync_spin()))
    return c->ctx->hip_fail(e, "pending export");
  return CE_OK;
}

int ce_core_pending_commit(ce_core* c, int accept, const uint64_t* d_import, uint64_t import_words) {
  if (!c || is_dotset_kind(c->kind)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (!c->pending) return c->ctx->fail(CE_ERR_INVALID_ARG, "no pending batch");
  c->pending = false;
  if (!accept) return CE_OK;  // another rank's batch failed: the state stays unchanged
  if (c->pending_gen != c->table_gen) return c->ctx->fail(CE_ERR_INVALID_ARG, "actor table changed since the ingest");
  if (d_import && import_words < c->cap)
    return c->ctx->fail(CE_ERR_INVALID_ARG, "reduced batch shorter than the dense capacity");
  const hipError_t e = launch_merge_max(c->ctx->stream, c->d_state.as<unsigned long long>(),
                                        d_import ? reinterpret_cast<const unsigned long long*>(d_import)
                                                 : c->d_batch.as<unsigned long long>(),
                                        c->cap);
  if (e) return c->ctx->hip_fail(e, "pending commit");
  for (auto& p : c->pending_nov) {  // next_op_versions.inc per applied file (lib.rs:537-538)
    if (p.second == 0) continue;   // nothing applied and nothing known: no entry (VClock::get = 0)
    uint32_t s;
    int rc = insert_actor(c, p.first, &s);
    if (rc) return rc;
    c->nov[s] = std::max(c->nov[s], p.second);
  }
  return table_upload(c);
}

}  // extern "C"
