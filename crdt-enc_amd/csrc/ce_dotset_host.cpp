// ce_dotset_host.cpp -- Core<S> for the dot-set kinds S = Orswot<u64, Uuid> and MVReg<u64, Uuid>
// (crdts 7), driving the kernels of ce_dotset.hip.
//
//   read_remote_ops   (crdt-enc/src/lib.rs:471-547)  GPU open -> version gate -> device decode of
//                     Vec<S::Op> into columnar arrays -> data-parallel fold (Orswot: applied
//                     flags by a stable sort + segmented max scan, pair-table max-insert,
//                     removal thresholds; MVReg: maximal-clock rounds)
//   read_remote_states (lib.rs:401-469)  GPU open -> host flatten of StateWrapper<S> -> per-pair
//                     Orswot::merge kernel (MVReg: survivor rounds with earlier-wins ties)
//   apply_ops         (lib.rs:666-722)   host parse of the local ops -> the same GPU fold
//
// The deferred removals of an Orswot and the values of an MVReg are small and live on the host;
// the entries (member -> VClock) live in HBM in the member / pair tables of ce_dotset.h.
#include <algorithm>
#include <cstdio>
#include <map>
#include <set>
#include <thread>

#include <memory>
#include <optional>

#include "ce_core.h"
#include "ce_dotset.h"
#include "ce_dotset_codec.h"
#include "ce_dotset_io.h"

namespace ce {

using IdDots = std::vector<std::pair<uint32_t, uint64_t>>;  // (actor id, counter), ids ascending

struct DsState {
  int kind = CE_STATE_ORSWOT;
  // Orswot
  DevBuf clock;  // u64[clock_cap] by actor id
  uint32_t clock_cap = 0;
  DevBuf mkey, pkey, cur, add, kill, oth, live, hold;  // hold: k-way merge holder bits (zero between merges)
  // a fold / k-way merge whose closing counts (live[0..3] -> pinned h_cnt[56..60)) and deferred
  // flags have not been read yet: ds_settle reads them at the next host wait
  bool settle_pending = false, settle_fold = false;
  bool settle_delta = false;  // live[0..1] are changes (the partitioned fold), not totals
  // a fold / merge overflowed a table: the tables and the deferred set no longer describe the
  // state, so every later operation fails until ce_core_reset (sticky: the overflow is only seen
  // at the settle after the call that caused it returned)
  bool poisoned = false;
  uint32_t settle_nr = 0;
  uint64_t settle_rmc = 0, settle_rmm = 0;
  std::vector<std::pair<IdDots, std::vector<uint64_t>>> settle_d0;
  uint32_t pcap = 0;  // pair table (and member overflow table: members <= pairs) capacity
  uint32_t mcap_s = 4096;     // primary member table slots (ensure_pairs grows it past half full)
  uint64_t used_members = 0;  // used primary member slots at the last fold / k-way merge
  bool settle_members = false;
  bool primary_fixed = false;  // CE_DS_PRIMARY_SLOTS: never grown (the overflow path under test)
  uint64_t head_hint = 1u << 18;  // state head prefix to download (ds_merge_states_device)
  // add / kill / oth / hold hold values between a launch that sets them and the one that clears
  // them (finalize, merge_finalize, kfinal): only then does tables_alloc need to clear them
  bool scratch_dirty = true;
  uint64_t used_pairs = 0, live_pairs = 0;
  std::map<IdDots, std::set<uint64_t>> deferred;  // removal clock -> members (HashMap in crdts)
  // MVReg
  std::vector<std::pair<IdDots, uint64_t>> vals;
  std::vector<std::vector<uint8_t>> ser_parts;  // per-thread entry writer output (reused)
  // scratch
  DevBuf cnt, ops[10], applied, sort_keys, sort_perm, sort_keys2, sort_perm2, ctr_sorted, excl,
      cub_tmp, deferred_flags, d0[5], col[6], mv[6], other[4], oclock;
  DevBuf misses;
  DevBuf part_akey, part_hk[2], part_items, part_ovf[2];  // the partitioned fold (DsPartArgs)
  DevBuf part_cnt;              // pcnt[2 parts] + ovf_n[4]: zero between folds (each apply zeroes them)
  uint32_t part_cnt_parts = 0;  // partitions part_cnt was zeroed for (0: zero it again)
  uint32_t part_gen = 0;        // partitioned folds so far (the parity of ovf_n)
  uint32_t part_factor = 3;     // run length = the expected share x part_factor / 2 (+64)
  HostBuf h_cnt;
  // run-contiguity marks of the adds' actors (k_ds_contig: a generation per check, no clearing)
  DevBuf contig_marks;
  uint32_t contig_cap = 0, contig_gen = 0;
  bool adds_contig = false;  // this batch's adds: every actor's adds one contiguous run
  bool adds_mono = false;    // ... and each run's counters strictly increase: k_ds_contig wrote the
                             // applied flags and exclusive maxima (applied, excl) of adds_mono_n adds
  uint32_t adds_mono_n = 0;
  DevBuf seal_out;           // the compaction's sealed file (ds_compact_device)
  DevBuf tile_col[9];        // the tiled emit's file-minor scratch rows (k_ds_emit<true>)
  // Orswot op files decoded in the open (k_open_fold_v2's DS form): raw counts, done flags and
  // the file-major rows (add actor / counter / member, removal actor / counter / member)
  DevBuf fz_cnt, fz_done, fz_col[6], fz_why, fz_big;
  DevBuf ser_sort;               // the serializer's radix-sort state (ce_ser_sort.hip), zeroed once
  size_t ser_sort_words = 0;
  uint32_t ser_sort_gen = 0;     // sorts so far (the state's histogram parity)
  // the multi-GPU column exchange (ds_export_columns_device / ds_merge_columns_device)
  HostBuf cx_host, cx_heads, cx_map, cx_dheads;
  DevBuf cx_mapd, cx_ids, cx_slot, cx_defact, cx_defflag;
  std::vector<uint32_t> cx_idslot;  // actor id -> table slot, as of table_gen cx_idslot_gen
  uint64_t cx_idslot_gen = ~0ull;
  void* col5_zeroed = nullptr;  // col[5] (the collect counter) was cleared at this address
  // device state reader (per state file: candidates, sorted heads, entry ends, Dot counts and
  // bases, members, sorted members [0..6]
  // and emitted (member, actor id, value) columns [7..9]), pinned staging for its downloads
  std::vector<std::array<DevBuf, 10>> rd;
  DevBuf cnt_part;  // the count pass's per-block maxima / decoded-file counts (DsDecodeArgs::bpart)
  DevBuf rd_tmp, rd_misc, ser[17], uuid_of_id, rank_of_id, id_of_rank, rd_oclocks, cnt_tot, rd_args_d, rd_chunks;
  HostBuf rd_host, rd_small, rd_clock, rd_args_h, h_clock, rd_tailh;
  uint64_t uuid_ids = ~0ull;  // id count uuid_of_id / rank_of_id (and id_rank / rank_id) were built for
  std::vector<uint32_t> id_rank, rank_id;  // UUID-order rank of each stable id, and its inverse
};

void ds_free(DsState* d) { delete d; }

namespace {

constexpr uint32_t kMissCap = 65536;

uint32_t pow2_at_least(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)p;
}

int bits_for(uint32_t v) {
  int b = 1;
  while (b < 32 && (1ull << b) <= v) b++;
  return b;
}

DsTables tables(DsState* d) {
  DsTables t;
  t.mkey = d->mkey.as<unsigned long long>();
  t.smask = d->mcap_s - 1;
  t.mmask = d->pcap - 1;
  t.pkey = d->pkey.as<unsigned long long>();
  t.cur = d->cur.as<unsigned long long>();
  t.add = d->add.as<unsigned long long>();
  t.kill = d->kill.as<unsigned long long>();
  t.oth = d->oth.as<unsigned long long>();
  t.pmask = d->pcap - 1;
  t.live = d->live.as<uint32_t>();
  return t;
}

int tables_alloc(ce_core* c, uint32_t cap, const FillRange* extra = nullptr) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  const uint64_t mslots = (uint64_t)d->mcap_s + cap + 1;
  void* const was[4] = {d->add.p, d->kill.p, d->oth.p, d->hold.p};
  if ((e = d->mkey.reserve(mslots * 8)) || (e = d->pkey.reserve(cap * 8ull)) ||
      (e = d->cur.reserve(cap * 8ull)) || (e = d->add.reserve(cap * 8ull)) ||
      (e = d->kill.reserve(cap * 8ull)) || (e = d->oth.reserve(cap * 8ull)) ||
      (e = d->hold.reserve(cap * 8ull)) || (e = d->live.reserve(64 + 64 * 16)))  // (+ the k-way merge's count replicas)
    return ctx->hip_fail(e, "dot-set tables");
  d->pcap = cap;
  // every table cleared by one launch (eight blit fills cost a dispatch gap each)
  FillArgs fl{};
  fl.r[0] = {d->mkey.as<uint32_t>(), mslots * 2, 0xffffffffu};
  fl.r[1] = {d->pkey.as<uint32_t>(), cap * 2ull, 0xffffffffu};
  fl.r[2] = {d->cur.as<uint32_t>(), cap * 2ull, 0u};
  fl.r[3] = {d->live.as<uint32_t>(), 16, 0u};
  fl.n = 4;
  // the scratch columns are zero after every completed fold / merge: cleared only when new or
  // when an operation stopped between setting and clearing them (~128 MB of fill at C3)
  const bool moved = was[0] != d->add.p || was[1] != d->kill.p || was[2] != d->oth.p || was[3] != d->hold.p;
  if (moved || d->scratch_dirty || getenv("CE_DS_CLEAR_ALL")) {
    fl.r[fl.n++] = {d->add.as<uint32_t>(), cap * 2ull, 0u};
    fl.r[fl.n++] = {d->kill.as<uint32_t>(), cap * 2ull, 0u};
    fl.r[fl.n++] = {d->oth.as<uint32_t>(), cap * 2ull, 0u};
    fl.r[fl.n++] = {d->hold.as<uint32_t>(), cap * 2ull, 0u};
    c->path_counts["ds_clear_scratch"]++;
  }
  if (extra) fl.r[fl.n++] = *extra;
  if ((e = launch_fill(ctx->stream, fl))) return ctx->hip_fail(e, "dot-set tables");
  d->scratch_dirty = false;
  d->used_pairs = 0;
  d->live_pairs = 0;
  d->used_members = 0;
  return CE_OK;
}

int ensure_clock(ce_core* c) {
  DsState* d = c->ds;
  const uint32_t need = std::max<uint32_t>(1024, (uint32_t)c->id_actor.size());
  if (need <= d->clock_cap) return CE_OK;
  const uint32_t cap = pow2_at_least(need);
  DevBuf nb;
  hipError_t e;
  if ((e = nb.reserve(cap * 8ull)) || (e = hipMemsetAsync(nb.p, 0, cap * 8ull, c->ctx->stream)) ||
      (d->clock_cap && (e = hipMemcpyAsync(nb.p, d->clock.p, d->clock_cap * 8ull,
                                           hipMemcpyDeviceToDevice, c->ctx->stream))) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "clock");
  std::swap(d->clock.p, nb.p);
  std::swap(d->clock.cap, nb.cap);
  d->clock_cap = cap;
  if ((e = d->oclock.reserve(cap * 8ull))) return c->ctx->hip_fail(e, "clock");
  return CE_OK;
}

// the device address of pinned host memory (kernels write their small results straight into it:
// no runtime copy, which the HIP runtime issues as a blit dispatch)
void* host_dev_ptr(void* h) {
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess || !dp) {
    (void)hipGetLastError();
    return h;
  }
  return dp;
}

// live entries -> (member, actor id, value) columns in d->col[0..2]; returns the count and
// (max_member) the largest live member.  extra_dl: one more download (dst, src, bytes) queued
// before the one wait (the compaction's clock)
int collect(ce_core* c, uint32_t* n_live, unsigned long long* max_member = nullptr,
            void* extra_dst = nullptr, const void* extra_src = nullptr, size_t extra_bytes = 0) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  const uint64_t cap = d->pcap;
  hipError_t e;
  if ((e = d->col[0].reserve(cap * 8 + 64)) || (e = d->col[1].reserve(cap * 4 + 64)) ||
      (e = d->col[2].reserve(cap * 8 + 64)) || (e = d->col[5].reserve(64 + 8ull * kCollectBlocks)) ||
      (e = d->h_cnt.reserve(512)))
    return ctx->hip_fail(e, "collect");
  uint32_t* cnt = d->col[5].as<uint32_t>();
  uint32_t* hc = d->h_cnt.as<uint32_t>() + 48;  // pinned: [0] count, [2..3] max member
  // the output counter is zero between collects (k_ds_collect_max resets it): cleared only when new
  if (d->col5_zeroed != d->col[5].p) {
    if ((e = hipMemsetAsync(cnt, 0, 16, ctx->stream))) return ctx->hip_fail(e, "collect");
    d->col5_zeroed = d->col[5].p;
  }
  // the count, largest member and the extra range (8-byte words) land in pinned memory from the
  // collect's last kernel
  if ((e = launch_ds_collect(ctx->stream, tables(d), d->col[0].as<unsigned long long>(),
                             d->col[1].as<uint32_t>(), d->col[2].as<unsigned long long>(), cnt,
                             reinterpret_cast<unsigned long long*>(d->col[5].as<uint8_t>() + 64),
                             static_cast<uint32_t*>(host_dev_ptr(hc)),
                             extra_bytes ? static_cast<unsigned long long*>(host_dev_ptr(extra_dst)) : nullptr,
                             static_cast<const unsigned long long*>(extra_src), (uint32_t)(extra_bytes / 8))) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "collect");
  *n_live = hc[0];
  if (max_member) *max_member = ((unsigned long long)hc[3] << 32) | hc[2];
  return CE_OK;
}

// make room for `extra` new pairs at <= 50% load: rebuild from the live entries when needed
// (or the primary member table past half full: rebuilt with 2.5x the members it holds)
int ensure_pairs(ce_core* c, uint64_t extra) {
  DsState* d = c->ds;
  const bool grow_members = d->used_members * 2 > d->mcap_s && d->mcap_s < (1u << 27) && !d->primary_fixed;
  if ((d->used_pairs + extra) * 2 <= d->pcap && !grow_members) return CE_OK;
  int rc;
  if (grow_members) {  // size the primary table for every member held, the overflow's too
    hipError_t e;
    if ((e = d->h_cnt.reserve(512))) return c->ctx->hip_fail(e, "members");
    uint32_t* hm = d->h_cnt.as<uint32_t>() + 40;
    if ((e = d->col[5].reserve(64 + 8ull * kCollectBlocks)) ||
        // (word 4: words 0..3 are the collect's counters, kept zero between collects)
        (e = hipMemsetAsync(d->col[5].as<uint32_t>() + 4, 0, 4, c->ctx->stream)) ||
        (e = launch_ds_count_members(c->ctx->stream, tables(d), d->col[5].as<uint32_t>() + 4)) ||
        (e = hipMemcpyAsync(hm, d->col[5].as<uint32_t>() + 4, 4, hipMemcpyDeviceToHost, c->ctx->stream)) ||
        (e = stream_wait(c->ctx->stream)))
      return c->ctx->hip_fail(e, "members");
    d->mcap_s = pow2_at_least(std::max<uint64_t>(4096, std::min<uint64_t>(1u << 27, hm[0] * 5ull / 2)));
  }
  uint32_t n_live = 0;
  if ((rc = collect(c, &n_live))) return rc;
  uint32_t cap = pow2_at_least(std::max<uint64_t>(4096, 2 * (n_live + extra) + 1));
  // test knob: a pair table that cannot grow past n slots, so an ingest overflows it
  const uint32_t cap_max = getenv("CE_DS_TEST_PAIR_CAP") ? pow2_at_least(std::max(4096, atoi(getenv("CE_DS_TEST_PAIR_CAP")))) : 0;
  if (cap_max && cap > cap_max) cap = std::max(cap_max, d->pcap);
  // the collected columns survive the reallocation of the tables
  if ((rc = tables_alloc(c, cap))) return rc;
  hipError_t e;
  if ((e = launch_ds_reinsert(c->ctx->stream, tables(d), d->col[0].as<unsigned long long>(),
                              d->col[1].as<uint32_t>(), d->col[2].as<unsigned long long>(), n_live)))
    return c->ctx->hip_fail(e, "rebuild");
  d->used_pairs = n_live;
  d->live_pairs = n_live;
  return CE_OK;
}

// ---------------------------------------------------------------------------------------
// host-side op decoding (local apply_ops, and op vectors the device defers to the host:
// unsorted clocks, nesting beyond the device parser's stack)
// ---------------------------------------------------------------------------------------
struct HostOp {
  int type = 0;             // 0 Add / Put, 1 Rm
  Uuid dot_actor{};
  uint64_t dot_ctr = 0;
  Dots clock;               // Rm / Put clock, BTreeMap semantics (sorted, later duplicate wins)
  std::vector<uint64_t> members;
  uint64_t val = 0;
};

// externally tagged enum: map(1) {name | index: body}
bool read_variant(Rd& r, const std::vector<const char*>& names, int* v) {
  uint64_t cnt;
  if (r.i >= r.n || !is_map_marker(r.p[r.i]) || !rd_map_hdr(r, &cnt) || cnt != 1) return false;
  if (r.i >= r.n) return false;
  if (is_binstr_marker(r.p[r.i])) {
    int kind;
    uint64_t off, l;
    if (!rd_binstr(r, &kind, &off, &l)) return false;
    for (size_t j = 0; j < names.size(); j++)
      if (std::strlen(names[j]) == l && std::memcmp(names[j], r.p + off, l) == 0) { *v = (int)j; return true; }
    return false;
  }
  uint64_t x;
  if (!rd_u64(r, &x) || x >= names.size()) return false;
  *v = (int)x;
  return true;
}

bool read_members(Rd& r, std::vector<uint64_t>* out) {
  uint64_t cnt, m;
  if (r.i >= r.n || !is_array_marker(r.p[r.i]) || !rd_array_hdr(r, &cnt) || cnt > r.n - r.i) return false;
  for (uint64_t k = 0; k < cnt; k++) {
    if (!rd_u64(r, &m)) return false;
    out->push_back(m);
  }
  return true;
}

void sort_dots(Dots* d) {
  std::sort(d->begin(), d->end(), [](const std::pair<Uuid, uint64_t>& a, const std::pair<Uuid, uint64_t>& b) {
    return a.first < b.first;
  });
}

bool parse_ops_host(int kind, const uint8_t* p, size_t n, std::vector<HostOp>* out) {
  Rd r{p, n, 0};
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(r.p[0]) || !rd_array_hdr(r, &cnt) || cnt > r.n) return false;
  for (uint64_t k = 0; k < cnt; k++) {
    HostOp op;
    int v;
    if (kind == CE_STATE_ORSWOT) {
      if (!read_variant(r, {"Add", "Rm"}, &v)) return false;
      op.type = v;
      bool ok;
      if (v == 0) {
        ok = read_struct(r, {"dot", "members"}, [&](int f, Rd& q) {
          if (f == 1) return read_members(q, &op.members);
          return read_struct(q, {"actor", "counter"}, [&](int g, Rd& s) {
            if (g == 1) return rd_u64(s, &op.dot_ctr);
            uint64_t off;
            if (!rd_uuid(s, &off)) return false;
            std::memcpy(op.dot_actor.data(), s.p + off, 16);
            return true;
          });
        });
      } else {
        ok = read_struct(r, {"clock", "members"}, [&](int f, Rd& q) {
          if (f == 1) return read_members(q, &op.members);
          return read_vclock(q, &op.clock);
        });
      }
      if (!ok) return false;
    } else {
      if (!read_variant(r, {"Put"}, &v)) return false;
      if (!read_struct(r, {"clock", "val"}, [&](int f, Rd& q) {
            if (f == 0) return read_vclock(q, &op.clock);
            return rd_u64(q, &op.val);
          }))
        return false;
    }
    sort_dots(&op.clock);
    out->push_back(std::move(op));
  }
  return true;
}

// compact canonical re-encoding (structs as arrays, variants as indices, minimal integers,
// sorted clocks): never longer than any accepted input form of the same ops
void encode_ops_compact(int kind, const std::vector<HostOp>& ops, Wr* w) {
  w->arr(ops.size());
  auto vclock = [&](const Dots& d) {
    w->arr(1);
    w->map(d.size());
    for (auto& x : d) { w->bin(x.first.data(), 16); w->uint(x.second); }
  };
  auto members = [&](const std::vector<uint64_t>& m) {
    w->arr(m.size());
    for (uint64_t x : m) w->uint(x);
  };
  for (auto& op : ops) {
    w->map(1);
    w->uint(kind == CE_STATE_ORSWOT ? (uint64_t)op.type : 0);
    w->arr(2);
    if (kind == CE_STATE_ORSWOT && op.type == 0) {
      w->arr(2);
      w->bin(op.dot_actor.data(), 16);
      w->uint(op.dot_ctr);
      members(op.members);
    } else if (kind == CE_STATE_ORSWOT) {
      vclock(op.clock);
      members(op.members);
    } else {
      vclock(op.clock);
      w->uint(op.val);
    }
  }
}

// ---------------------------------------------------------------------------------------
// columnar batches
// ---------------------------------------------------------------------------------------
struct Counts {
  uint64_t v[kCntN] = {0, 0, 0, 0, 0};
};

int reserve_ops(ce_core* c, const Counts& k) {
  DsState* d = c->ds;
  hipError_t e;
  const uint64_t na = k.v[kCntAdd] + 1, nam = k.v[kCntAddM] + 1, nr = k.v[kCntRm] + 1,
                 nrc = k.v[kCntRmC] + 1, nrm = k.v[kCntRmM] + 1;
  if ((e = d->ops[0].reserve(na * 4)) || (e = d->ops[1].reserve(na * 8)) ||
      (e = d->ops[2].reserve(na * 4)) || (e = d->ops[3].reserve(nam * 8)) ||
      (e = d->ops[4].reserve(nr * 4)) || (e = d->ops[5].reserve(nr * 4)) ||
      (e = d->ops[6].reserve(nrc * 4)) || (e = d->ops[7].reserve(nrc * 8)) ||
      (e = d->ops[8].reserve(nrm * 8)) || (e = d->ops[9].reserve(nr * 8)))
    return c->ctx->hip_fail(e, "ops reserve");
  return CE_OK;
}

DsOps ops_view(DsState* d) {
  DsOps o;
  o.add_actor = d->ops[0].as<uint32_t>();
  o.add_ctr = d->ops[1].as<unsigned long long>();
  o.add_mbeg = d->ops[2].as<uint32_t>();
  o.add_mem = d->ops[3].as<unsigned long long>();
  o.rm_cbeg = d->ops[4].as<uint32_t>();
  o.rm_mbeg = d->ops[5].as<uint32_t>();
  o.rmc_actor = d->ops[6].as<uint32_t>();
  o.rmc_ctr = d->ops[7].as<unsigned long long>();
  o.rm_mem = d->ops[8].as<unsigned long long>();
  o.put_val = d->ops[9].as<unsigned long long>();
  return o;
}

// write the CSR end sentinels: add_mbeg[n_add], rm_cbeg[n_rm], rm_mbeg[n_rm]
int write_sentinels(ce_core* c, const Counts& k) {
  DsState* d = c->ds;
  DsOps o = ops_view(d);
  hipError_t e;
  if ((e = launch_ds_set3(c->ctx->stream, o.add_mbeg + k.v[kCntAdd], (uint32_t)k.v[kCntAddM],
                          o.rm_cbeg + k.v[kCntRm], (uint32_t)k.v[kCntRmC], o.rm_mbeg + k.v[kCntRm],
                          (uint32_t)k.v[kCntRmM])))
    return c->ctx->hip_fail(e, "sentinels");
  return CE_OK;
}

// host ops -> columnar arrays at the given offsets (ids must exist).  Orswot adds/removals or
// MVReg puts.
struct HostCols {
  std::vector<uint32_t> add_actor, add_mbeg, rm_cbeg, rm_mbeg, rmc_actor;
  std::vector<unsigned long long> add_ctr, add_mem, rmc_ctr, rm_mem, put_val;
};

int host_cols(ce_core* c, const std::vector<HostOp>& ops, const Counts& base, HostCols* hc) {
  for (auto& op : ops) {
    if (c->kind == CE_STATE_ORSWOT && op.type == 0) {
      uint32_t s;
      int rc = insert_actor(c, op.dot_actor, &s);
      if (rc) return rc;
      hc->add_mbeg.push_back((uint32_t)(base.v[kCntAddM] + hc->add_mem.size()));
      hc->add_actor.push_back(actor_id_of_slot(c, s));
      hc->add_ctr.push_back(op.dot_ctr);
      for (uint64_t m : op.members) hc->add_mem.push_back(m);
    } else {
      hc->rm_cbeg.push_back((uint32_t)(base.v[kCntRmC] + hc->rmc_actor.size()));
      hc->rm_mbeg.push_back((uint32_t)(base.v[kCntRmM] + hc->rm_mem.size()));
      for (auto& x : op.clock) {
        uint32_t s;
        int rc = insert_actor(c, x.first, &s);
        if (rc) return rc;
        hc->rmc_actor.push_back(actor_id_of_slot(c, s));
        hc->rmc_ctr.push_back(x.second);
      }
      for (uint64_t m : op.members) hc->rm_mem.push_back(m);
      hc->put_val.push_back(op.val);
    }
  }
  return CE_OK;
}

template <typename T>
hipError_t up(T* dst, const std::vector<T>& v, hipStream_t s) {
  if (v.empty()) return hipSuccess;
  return hipMemcpyAsync(dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
}

int upload_cols(ce_core* c, const HostCols& hc, const Counts& base) {
  DsOps o = ops_view(c->ds);
  hipStream_t s = c->ctx->stream;
  hipError_t e;
  if ((e = up(o.add_actor + base.v[kCntAdd], hc.add_actor, s)) ||
      (e = up(o.add_ctr + base.v[kCntAdd], hc.add_ctr, s)) ||
      (e = up(o.add_mbeg + base.v[kCntAdd], hc.add_mbeg, s)) ||
      (e = up(o.add_mem + base.v[kCntAddM], hc.add_mem, s)) ||
      (e = up(o.rm_cbeg + base.v[kCntRm], hc.rm_cbeg, s)) ||
      (e = up(o.rm_mbeg + base.v[kCntRm], hc.rm_mbeg, s)) ||
      (e = up(o.rmc_actor + base.v[kCntRmC], hc.rmc_actor, s)) ||
      (e = up(o.rmc_ctr + base.v[kCntRmC], hc.rmc_ctr, s)) ||
      (e = up(o.rm_mem + base.v[kCntRmM], hc.rm_mem, s)) ||
      (e = up(o.put_val + base.v[kCntRm], hc.put_val, s)) || (e = stream_wait(s)))
    return c->ctx->hip_fail(e, "ops upload");
  return CE_OK;
}

// deferred removals (host) -> CSR removal arrays in d->d0 (cbeg, mbeg, actor, ctr, members)
int upload_removals(ce_core* c, const std::vector<std::pair<IdDots, std::vector<uint64_t>>>& rms) {
  DsState* d = c->ds;
  std::vector<uint32_t> cbeg{0}, mbeg{0}, act;
  std::vector<unsigned long long> ctr, mem;
  for (auto& r : rms) {
    for (auto& x : r.first) { act.push_back(x.first); ctr.push_back(x.second); }
    for (uint64_t m : r.second) mem.push_back(m);
    cbeg.push_back((uint32_t)act.size());
    mbeg.push_back((uint32_t)mem.size());
  }
  hipError_t e;
  if ((e = d->d0[0].reserve(cbeg.size() * 4)) || (e = d->d0[1].reserve(mbeg.size() * 4)) ||
      (e = d->d0[2].reserve(act.size() * 4 + 4)) || (e = d->d0[3].reserve(ctr.size() * 8 + 8)) ||
      (e = d->d0[4].reserve(mem.size() * 8 + 8)))
    return c->ctx->hip_fail(e, "removals");
  hipStream_t s = c->ctx->stream;
  if ((e = up(d->d0[0].as<uint32_t>(), cbeg, s)) || (e = up(d->d0[1].as<uint32_t>(), mbeg, s)) ||
      (e = up(d->d0[2].as<uint32_t>(), act, s)) || (e = up(d->d0[3].as<unsigned long long>(), ctr, s)) ||
      (e = up(d->d0[4].as<unsigned long long>(), mem, s)) || (e = stream_wait(s)))
    return c->ctx->hip_fail(e, "removals");
  return CE_OK;
}

// removals as CSR arrays on the host (the column merge's: hundreds of thousands of deferred
// removals at N = 8 with read-context clocks, without a heap object per removal)
struct RmCsr {
  std::vector<uint32_t> cbeg{0}, mbeg{0}, act;
  std::vector<unsigned long long> ctr, mem;
  uint32_t size() const { return (uint32_t)cbeg.size() - 1; }
  void close() {
    cbeg.push_back((uint32_t)act.size());
    mbeg.push_back((uint32_t)mem.size());
  }
};

int upload_removals_csr(ce_core* c, const RmCsr& r) {
  DsState* d = c->ds;
  hipError_t e;
  if ((e = d->d0[0].reserve(r.cbeg.size() * 4)) || (e = d->d0[1].reserve(r.mbeg.size() * 4)) ||
      (e = d->d0[2].reserve(r.act.size() * 4 + 4)) || (e = d->d0[3].reserve(r.ctr.size() * 8 + 8)) ||
      (e = d->d0[4].reserve(r.mem.size() * 8 + 8)))
    return c->ctx->hip_fail(e, "removals");
  hipStream_t s = c->ctx->stream;
  if ((e = up(d->d0[0].as<uint32_t>(), r.cbeg, s)) || (e = up(d->d0[1].as<uint32_t>(), r.mbeg, s)) ||
      (e = up(d->d0[2].as<uint32_t>(), r.act, s)) || (e = up(d->d0[3].as<unsigned long long>(), r.ctr, s)) ||
      (e = up(d->d0[4].as<unsigned long long>(), r.mem, s)) || (e = stream_wait(s)))
    return c->ctx->hip_fail(e, "removals");
  return CE_OK;
}

std::vector<std::pair<IdDots, std::vector<uint64_t>>> deferred_list(DsState* d) {
  std::vector<std::pair<IdDots, std::vector<uint64_t>>> v;
  for (auto& x : d->deferred) v.push_back({x.first, std::vector<uint64_t>(x.second.begin(), x.second.end())});
  return v;
}

int flags_for(ce_core* c, const uint32_t* cbeg, const uint32_t* act, const unsigned long long* ctr,
              uint32_t n_rm, std::vector<uint8_t>* flags) {
  DsState* d = c->ds;
  flags->assign(n_rm, 0);
  if (!n_rm) return CE_OK;
  hipError_t e;
  if ((e = d->deferred_flags.reserve(n_rm + 64)) ||
      (e = launch_ds_deferred(c->ctx->stream, cbeg, act, ctr, d->clock.as<unsigned long long>(),
                              d->deferred_flags.as<uint8_t>(), n_rm)) ||
      (e = hipMemcpyAsync(flags->data(), d->deferred_flags.p, n_rm, hipMemcpyDeviceToHost, c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "deferred");
  return CE_OK;
}

int finalize(ce_core* c) {
  DsState* d = c->ds;
  uint32_t h[4];
  hipError_t e;
  if ((e = hipMemsetAsync(d->live.p, 0, 8, c->ctx->stream))) return c->ctx->hip_fail(e, "finalize");
  const int t = c->ctx->tbegin("ds_finalize");
  if ((e = launch_ds_finalize(c->ctx->stream, tables(d)))) return c->ctx->hip_fail(e, "finalize");
  c->ctx->tend(t);
  if (
      (e = hipMemcpyAsync(h, d->live.p, 16, hipMemcpyDeviceToHost, c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "finalize");
  if (h[2]) {
    d->poisoned = true;
    return c->ctx->fail(CE_ERR_DEVICE, "dot-set table overflow");
  }
  d->live_pairs = h[0];
  d->used_pairs = h[1];
  return CE_OK;
}

// Orswot fold of a columnar batch in application order (k = counts); the removals of the
// batch plus the current deferred set (re-applied by apply_deferred) set the thresholds.
// kill_bound: an upper bound on the batch's removal items (sum over removals of members x clock
// entries; ~0 = unknown: the global kernels).  adds_contig: the emit that produced THESE columns
// proved every actor's adds one contiguous run (only ds_ingest_ops can say so; any other caller
// passes false, and the sorted path is always correct)
int orswot_fold(ce_core* c, const Counts& k, uint64_t kill_bound, bool adds_contig) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  DsOps o = ops_view(d);
  hipError_t e;
  int rc;
  if ((rc = ensure_clock(c))) return rc;
  const uint32_t na = (uint32_t)k.v[kCntAdd], nr = (uint32_t)k.v[kCntRm];
  // 1) applied flags: stable sort of the adds by actor, segmented exclusive max of counters
  if ((e = d->applied.reserve(na + 64))) return ctx->hip_fail(e, "applied");
  // the clock update's keys / counters: sorted copies, or the columns themselves when every
  // actor's adds already form one contiguous run (the scan by key then needs no sort)
  // (set after the reserves below: a reserve may move the buffer)
  const uint32_t* clock_keys = nullptr;
  const unsigned long long* clock_ctr = nullptr;
  if (na && adds_contig && d->adds_mono && d->adds_mono_n == na) {
    // k_ds_contig already wrote the applied flags and exclusive maxima (strictly increasing runs)
    clock_keys = o.add_actor;
    clock_ctr = o.add_ctr;
    c->path_counts["ds_adds_monotone"]++;
  } else if (na && adds_contig) {
    if ((e = d->excl.reserve(na * 8ull))) return ctx->hip_fail(e, "applied");
    unsigned long long* ex = d->excl.as<unsigned long long>();
    size_t t2 = 0;
    if ((e = ds_excl_max_by_key(nullptr, t2, o.add_actor, o.add_ctr, ex, na, s)) ||
        (e = d->cub_tmp.reserve(t2 + 256)))
      return ctx->hip_fail(e, "applied");
    t2 = d->cub_tmp.cap;
    const int ta = ctx->tbegin("ds_applied");
    if ((e = ds_excl_max_by_key(d->cub_tmp.p, t2, o.add_actor, o.add_ctr, ex, na, s)) ||
        (e = launch_ds_applied(s, o.add_actor, nullptr, o.add_ctr, ex, d->clock.as<unsigned long long>(),
                               d->applied.as<uint8_t>(), na)))
      return ctx->hip_fail(e, "applied");
    ctx->tend(ta);
    c->path_counts["ds_adds_contiguous"]++;
    clock_keys = o.add_actor;
    clock_ctr = o.add_ctr;
  } else if (na) {
    if ((e = d->sort_keys.reserve(na * 4ull)) || (e = d->sort_perm.reserve(na * 4ull)) ||
        (e = d->sort_keys2.reserve(na * 4ull)) || (e = d->sort_perm2.reserve(na * 4ull)) ||
        (e = d->ctr_sorted.reserve(na * 8ull)) || (e = d->excl.reserve(na * 8ull)))
      return ctx->hip_fail(e, "applied");
    clock_keys = d->sort_keys2.as<uint32_t>();
    clock_ctr = d->ctr_sorted.as<unsigned long long>();
    const int bits = bits_for((uint32_t)c->id_actor.size());
    size_t t1 = 0, t2 = 0;
    uint32_t* keys2 = d->sort_keys2.as<uint32_t>();
    uint32_t* perm = d->sort_perm.as<uint32_t>();
    uint32_t* perm2 = d->sort_perm2.as<uint32_t>();
    unsigned long long* cs = d->ctr_sorted.as<unsigned long long>();
    unsigned long long* ex = d->excl.as<unsigned long long>();
    if ((e = ds_sort_pairs_u32(nullptr, t1, o.add_actor, keys2, perm, perm2, na, bits, s)) ||
        (e = ds_excl_max_by_key(nullptr, t2, keys2, cs, ex, na, s)))
      return ctx->hip_fail(e, "applied");
    if ((e = d->cub_tmp.reserve(std::max(t1, t2) + 256))) return ctx->hip_fail(e, "applied");
    t1 = t2 = d->cub_tmp.cap;
    const int ta = ctx->tbegin("ds_applied");
    if ((e = launch_ds_iota(s, perm, na)) ||
        (e = ds_sort_pairs_u32(d->cub_tmp.p, t1, o.add_actor, keys2, perm, perm2, na, bits, s)) ||
        (e = launch_ds_gather_ctr(s, perm2, o.add_ctr, cs, na)) ||
        (e = ds_excl_max_by_key(d->cub_tmp.p, t2, keys2, cs, ex, na, s)) ||
        (e = launch_ds_applied(s, keys2, perm2, cs, ex, d->clock.as<unsigned long long>(),
                               d->applied.as<uint8_t>(), na)))
      return ctx->hip_fail(e, "applied");
    ctx->tend(ta);
  }
  // 2) entries: max-insert the applied adds (capacity for every add member), 3) removal
  //    thresholds: the batch's removals and the deferred set (uploaded only when there is one:
  //    the upload waits for its pageable sources), then finalize -- partitioned (DsPartArgs) when
  //    the batch fits its limits, else the global kernels
  if ((rc = ensure_pairs(c, k.v[kCntAddM]))) return rc;
  auto d0 = deferred_list(d);
  const uint32_t n0 = (uint32_t)d0.size();
  if (n0 && (rc = upload_removals(c, d0))) return rc;
  uint64_t m0 = 0, kb0 = 0;  // the deferred set's members and items
  for (auto& x : d0) {
    m0 += x.second.size();
    kb0 += (uint64_t)x.second.size() * x.first.size();
  }
  uint32_t* live = d->live.as<uint32_t>();
  DsPartArgs pa{};
  pa.parts = d->pcap >> kDsPartBits;
  // K1 block size (CE_DS_PART_THREADS: 1024, 512 or 256; CE_PART_BATCH items per thread): 512 by
  // default -- with 8 items per thread C3's 1.7M adds were ~415 blocks, every CU busy (1024: ~207
  // blocks on 256 CUs; same box k_ds_part_adds 80 -> 62 us), with 4 ~830 blocks (49.7 us)
  static const uint32_t k1_threads = [] {
    const char* v = getenv("CE_DS_PART_THREADS");
    const uint32_t t = v ? (uint32_t)atoi(v) : (getenv("CE_DS_PART_SMALL") && atoi(getenv("CE_DS_PART_SMALL")) == 0 ? 1024u : 512u);
    return t == 1024u || t == 256u ? t : 512u;
  }();
  pa.chunk = k1_threads == 1024u ? kDsPartChunk : k1_threads == 512u ? kDsPartChunkSmall : 256u * CE_PART_BATCH;
  pa.kchunk = pa.chunk / 4;  // removals are ~1/4 of C3's ops: as many blocks
  pa.ba = (uint32_t)((na + pa.chunk - 1) / pa.chunk);
  pa.bk0 = (uint32_t)((nr + pa.kchunk - 1) / pa.kchunk);
  pa.bk = pa.bk0 + (uint32_t)((n0 + pa.kchunk - 1) / pa.kchunk);
  const uint64_t kill_items = kill_bound == ~0ull ? ~0ull : kill_bound + kb0;
  // runs: the expected share of a partition x part_factor / 2, + 64 (C3: ~12 sigma of slack);
  // what passes it goes to the overflow lists (sized for the whole batch)
  const uint64_t sub = (uint64_t)pa.parts * kDsPartReps;  // sub-runs per side
  const uint64_t cap_a = pa.parts ? k.v[kCntAddM] / sub * d->part_factor / 2 + 32 : 0,
                 cap_k = pa.parts && kill_items != ~0ull ? kill_items / sub * d->part_factor / 2 + 32 : 0;
  // (the removal-item bound is loose for multi-entry clocks -- members x the largest file's clock
  // entries: C3 read-context 23.6M for 2.1M actual items -- so it only caps the scratch: up to 64M
  // items, ~1 GB of runs and overflow list, the partitioned fold takes it)
  const bool part = !getenv("CE_DS_FOLD_GLOBAL") && pa.parts >= 1 && pa.parts <= kDsPartMaxParts &&
                    (kill_items <= 4 * (k.v[kCntRmM] + k.v[kCntRmC] + kb0) + (1ull << 20) || kill_items <= (1ull << 26)) &&
                    k.v[kCntAddM] + kill_items < (1ull << 31) && sub * (cap_a + cap_k) < (1ull << 31);
  if (part) {
    pa.cap[0] = (uint32_t)cap_a;
    pa.cap[1] = (uint32_t)cap_k;
    pa.ovf_cap[0] = (uint32_t)k.v[kCntAddM];
    pa.ovf_cap[1] = (uint32_t)kill_items;
    if ((e = d->part_akey.reserve(8 * k.v[kCntAddM] + 64)) || (e = d->part_hk[0].reserve(8 * k.v[kCntRmM] + 64)) ||
        (e = d->part_hk[1].reserve(8 * m0 + 64)) ||
        (e = d->part_items.reserve(16ull * sub * (cap_a + cap_k) + 64)) ||
        (e = d->part_ovf[0].reserve(16 * k.v[kCntAddM] + 64)) || (e = d->part_ovf[1].reserve(16 * kill_items + 64)))
      return ctx->hip_fail(e, "fold");
    if (d->part_cnt_parts < pa.parts) {  // new (or larger) counters: zeroed once, then by the applies
      if ((e = d->part_cnt.reserve(8ull * kDsPartReps * pa.parts + 64)) ||
          (e = hipMemsetAsync(d->part_cnt.p, 0, 8ull * kDsPartReps * pa.parts + 64, s)))
        return ctx->hip_fail(e, "fold");
      d->part_cnt_parts = pa.parts;
    }
    pa.t = tables(d);
    pa.o = o;
    pa.applied = d->applied.as<uint8_t>();
    pa.n_add = na;
    pa.akey = d->part_akey.as<unsigned long long>();
    pa.ks[0] = {o.rm_cbeg, o.rm_mbeg, o.rmc_actor, o.rmc_ctr, o.rm_mem, d->part_hk[0].as<unsigned long long>(), nr};
    pa.ks[1] = {d->d0[0].as<uint32_t>(), d->d0[1].as<uint32_t>(), d->d0[2].as<uint32_t>(),
                d->d0[3].as<unsigned long long>(), d->d0[4].as<unsigned long long>(),
                d->part_hk[1].as<unsigned long long>(), n0};
    pa.pcnt = d->part_cnt.as<uint32_t>();
    pa.ovf_n = pa.pcnt + 2ull * kDsPartReps * d->part_cnt_parts;
    pa.items = d->part_items.as<unsigned long long>();
    pa.ovf[0] = d->part_ovf[0].as<unsigned long long>();
    pa.ovf[1] = d->part_ovf[1].as<unsigned long long>();
    pa.par = d->part_gen++ & 1u;
    const int tp = ctx->tbegin("ds_part_fold");
    if ((e = launch_ds_part_count(s, pa)) || (e = launch_ds_part_apply(s, pa)) ||
        (e = launch_ds_clock(s, clock_keys, clock_ctr, d->excl.as<unsigned long long>(),
                             d->clock.as<unsigned long long>(), na)))
      return ctx->hip_fail(e, "fold");
    ctx->tend(tp);
    c->path_counts["ds_fold_partitioned"]++;
    if ((e = d->deferred_flags.reserve(nr + n0 + 64))) return ctx->hip_fail(e, "finalize");
  } else {
    const int tp = ctx->tbegin("ds_add_pairs");
    d->scratch_dirty = true;
    if ((e = launch_ds_add_pairs(s, tables(d), o, d->applied.as<uint8_t>(), na)) ||
        (e = launch_ds_clock(s, clock_keys, clock_ctr, d->excl.as<unsigned long long>(),
                             d->clock.as<unsigned long long>(), na)))
      return ctx->hip_fail(e, "add");
    ctx->tend(tp);
    const int tk = ctx->tbegin("ds_kill");
    if ((e = launch_ds_kill(s, tables(d), o.rm_cbeg, o.rm_mbeg, o.rmc_actor, o.rmc_ctr, o.rm_mem, nr)) ||
        (n0 && (e = launch_ds_kill(s, tables(d), d->d0[0].as<uint32_t>(), d->d0[1].as<uint32_t>(),
                                   d->d0[2].as<uint32_t>(), d->d0[3].as<unsigned long long>(),
                                   d->d0[4].as<unsigned long long>(), n0))))
      return ctx->hip_fail(e, "kill");
    ctx->tend(tk);
    // finalize and the deferred flags without a host wait: live / used pairs, the overflow flag and
    // whether any removal stays deferred land in pinned memory; ds_settle reads them at the
    // caller's next host wait (the removal columns stay intact until then)
    if ((e = d->deferred_flags.reserve(nr + n0 + 64)) || (e = launch_ds_set3(s, live, 0u, live + 1, 0u, live + 3, 0u)))
      return ctx->hip_fail(e, "finalize");
    const int t = ctx->tbegin("ds_finalize");
    if ((e = launch_ds_finalize(s, tables(d)))) return ctx->hip_fail(e, "finalize");
    d->scratch_dirty = false;
    ctx->tend(t);
    c->path_counts["ds_fold_global"]++;
  }
  // the last deferred-flags launch publishes live[0..6) into the pinned h_cnt[56..62) (ds_settle)
  uint8_t* fl = d->deferred_flags.as<uint8_t>();
  uint32_t* pub = static_cast<uint32_t*>(host_dev_ptr(d->h_cnt.as<uint32_t>() + 56));
  if ((e = launch_ds_deferred(s, o.rm_cbeg, o.rmc_actor, o.rmc_ctr, d->clock.as<unsigned long long>(), fl, nr, live + 3,
                              live, n0 ? nullptr : pub, 6)) ||
      (n0 && (e = launch_ds_deferred(s, d->d0[0].as<uint32_t>(), d->d0[2].as<uint32_t>(),
                                     d->d0[3].as<unsigned long long>(), d->clock.as<unsigned long long>(), fl + nr,
                                     n0, live + 3, live, pub, 6))))
    return ctx->hip_fail(e, "finalize");
  d->settle_pending = true;
  d->settle_fold = true;
  d->settle_delta = part;
  d->settle_members = part;
  d->settle_nr = nr;
  d->settle_rmc = k.v[kCntRmC];
  d->settle_rmm = k.v[kCntRmM];
  d->settle_d0 = std::move(d0);
  return CE_OK;
}

}  // namespace

// A fold's or k-way merge's closing counts and the new deferred set, once the stream has
// drained (usually it has: callers settle right after a host wait of their own)
int ds_settle(ce_core* c) {
  DsState* d = c->ds;
  if (!d) return CE_OK;
  ce_ctx* ctx = c->ctx;
  if (d->poisoned) return ctx->fail(CE_ERR_DEVICE, "dot-set table overflow in an earlier operation (reset the core)");
  if (!d->settle_pending) return CE_OK;
  hipStream_t s = ctx->stream;
  hipError_t e;
  if ((e = stream_wait(s))) return ctx->hip_fail(e, "settle");
  d->settle_pending = false;
  const uint32_t* hl = d->h_cnt.as<uint32_t>() + 56;
  if (hl[2]) {
    d->poisoned = true;
    d->settle_d0.clear();
    return ctx->fail(CE_ERR_DEVICE, "dot-set table overflow");
  }
  if (d->settle_delta) {
    // (k_ds_part_apply adds both words as one 64-bit value: a negative live change borrowed one
    // from the used count's word)
    d->live_pairs += (int64_t)(int32_t)hl[0];
    d->used_pairs += hl[1] + ((int32_t)hl[0] < 0 ? 1u : 0u);
    // items past their partition's run (folded from the overflow lists): longer runs next time
    if (d->settle_fold && hl[5]) {
      d->part_factor = std::min<uint32_t>(64, std::max<uint32_t>(1, d->part_factor) * 2);
      c->path_counts["ds_fold_run_overflow"]++;
    }
  } else {
    d->live_pairs = hl[0];
    d->used_pairs = hl[1];
  }
  if (d->settle_members) d->used_members = hl[4];
  if (!d->settle_fold) return CE_OK;
  // 4) deferred = removals whose clock is not covered by the new clock (none: the usual case)
  std::map<IdDots, std::set<uint64_t>> nd;
  auto d0 = std::move(d->settle_d0);
  d->settle_d0.clear();
  if (hl[3]) {
    const uint32_t nr = d->settle_nr, n0 = (uint32_t)d0.size();
    DsOps o = ops_view(d);
    std::vector<uint8_t> f(nr + n0);
    std::vector<uint32_t> cb(nr + 1), mb(nr + 1), act(d->settle_rmc);
    std::vector<unsigned long long> ctr(d->settle_rmc), mem(d->settle_rmm);
    if ((!f.empty() && (e = hipMemcpyAsync(f.data(), d->deferred_flags.p, f.size(), hipMemcpyDeviceToHost, s))) ||
        (nr && (e = hipMemcpyAsync(cb.data(), o.rm_cbeg, (nr + 1) * 4ull, hipMemcpyDeviceToHost, s))) ||
        (nr && (e = hipMemcpyAsync(mb.data(), o.rm_mbeg, (nr + 1) * 4ull, hipMemcpyDeviceToHost, s))) ||
        (!act.empty() && (e = hipMemcpyAsync(act.data(), o.rmc_actor, act.size() * 4, hipMemcpyDeviceToHost, s))) ||
        (!ctr.empty() && (e = hipMemcpyAsync(ctr.data(), o.rmc_ctr, ctr.size() * 8, hipMemcpyDeviceToHost, s))) ||
        (!mem.empty() && (e = hipMemcpyAsync(mem.data(), o.rm_mem, mem.size() * 8, hipMemcpyDeviceToHost, s))) ||
        (e = stream_wait(s)))
      return ctx->hip_fail(e, "deferred download");
    for (uint32_t i = 0; i < n0; i++)
      if (f[nr + i]) nd[d0[i].first].insert(d0[i].second.begin(), d0[i].second.end());
    for (uint32_t r = 0; r < nr; r++) {
      if (!f[r]) continue;
      IdDots key;
      for (uint32_t j = cb[r]; j < cb[r + 1]; j++) key.push_back({act[j], ctr[j]});
      std::sort(key.begin(), key.end());
      auto& set = nd[key];
      for (uint32_t j = mb[r]; j < mb[r + 1]; j++) set.insert(mem[j]);
    }
  }
  d->deferred = std::move(nd);
  return CE_OK;
}

namespace {

// MVReg survivors among n candidates already in ops rm_cbeg/rmc_*/put_val; returns indices in
// ascending (insertion) order
int mvreg_survivors(ce_core* c, uint32_t n, bool later_wins, std::vector<uint32_t>* out) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  out->clear();
  if (n == 0) return CE_OK;
  int rc;
  if ((rc = ensure_clock(c))) return rc;
  DsOps o = ops_view(d);
  MvArgs a{};
  a.cbeg = o.rm_cbeg;
  a.c_actor = o.rmc_actor;
  a.c_ctr = o.rmc_ctr;
  a.n = n;
  a.later_wins = later_wins ? 1 : 0;
  a.n_blk = std::min<uint32_t>(1024, (n + 255) / 256);
  hipError_t e;
  if ((e = d->mv[0].reserve(n + 64)) || (e = d->mv[1].reserve(n * 8ull)) || (e = d->mv[2].reserve(n * 8ull)) ||
      (e = d->mv[3].reserve(a.n_blk * 32ull)) || (e = d->mv[4].reserve(64)) ||
      (e = d->mv[5].reserve(d->clock_cap * 8ull)))
    return ctx->hip_fail(e, "mvreg");
  if (d->mv[5].cap < d->clock_cap * 8ull) return ctx->fail(CE_ERR_DEVICE, "mvreg scratch");
  a.alive = d->mv[0].as<uint8_t>();
  a.sum_hi = d->mv[1].as<unsigned long long>();
  a.sum_lo = d->mv[2].as<unsigned long long>();
  a.blk = d->mv[3].as<unsigned long long>();
  a.win = d->mv[4].as<uint32_t>();
  a.wclock = d->mv[5].as<unsigned long long>();
  if ((e = hipMemsetAsync(a.wclock, 0, d->clock_cap * 8ull, s)) || (e = launch_mv_prep(s, a)))
    return ctx->hip_fail(e, "mvreg");
  for (uint32_t round = 0; round <= n; round++) {
    uint32_t w;
    if ((e = launch_mv_round(s, a)) || (e = hipMemcpyAsync(&w, a.win, 4, hipMemcpyDeviceToHost, s)) ||
        (e = stream_wait(s)))
      return ctx->hip_fail(e, "mvreg round");
    if (w == 0xffffffffu) break;
    if (w >= n) return ctx->fail(CE_ERR_DEVICE, "mvreg winner out of range");
    out->push_back(w);
  }
  std::sort(out->begin(), out->end());
  return CE_OK;
}

// candidate i's clock and value (device) -> host
int fetch_candidate(ce_core* c, uint32_t i, std::pair<IdDots, uint64_t>* v) {
  DsOps o = ops_view(c->ds);
  hipStream_t s = c->ctx->stream;
  uint32_t cb[2];
  hipError_t e;
  if ((e = hipMemcpyAsync(cb, o.rm_cbeg + i, 8, hipMemcpyDeviceToHost, s)) ||
      (e = hipMemcpyAsync(&v->second, o.put_val + i, 8, hipMemcpyDeviceToHost, s)) ||
      (e = stream_wait(s)))
    return c->ctx->hip_fail(e, "candidate");
  const uint32_t k = cb[1] - cb[0];
  std::vector<uint32_t> act(k);
  std::vector<unsigned long long> ctr(k);
  if (k && ((e = hipMemcpyAsync(act.data(), o.rmc_actor + cb[0], k * 4ull, hipMemcpyDeviceToHost, s)) ||
            (e = hipMemcpyAsync(ctr.data(), o.rmc_ctr + cb[0], k * 8ull, hipMemcpyDeviceToHost, s)) ||
            (e = stream_wait(s))))
    return c->ctx->hip_fail(e, "candidate");
  v->first.clear();
  for (uint32_t j = 0; j < k; j++) v->first.push_back({act[j], ctr[j]});
  std::sort(v->first.begin(), v->first.end());
  return CE_OK;
}

// current MVReg values -> host columns (prefix of the candidate list)
void vals_cols(DsState* d, HostCols* hc) {
  for (auto& v : d->vals) {
    hc->rm_cbeg.push_back((uint32_t)hc->rmc_actor.size());
    hc->rm_mbeg.push_back(0);
    for (auto& x : v.first) { hc->rmc_actor.push_back(x.first); hc->rmc_ctr.push_back(x.second); }
    hc->put_val.push_back(v.second);
  }
}

// MVReg: candidates = the K current values (prefix) then n_new more; survivors -> vals
int mvreg_commit(ce_core* c, uint32_t K, uint32_t total, bool later_wins) {
  DsState* d = c->ds;
  std::vector<uint32_t> surv;
  int rc = mvreg_survivors(c, total, later_wins, &surv);
  if (rc) return rc;
  std::vector<std::pair<IdDots, uint64_t>> nv;
  for (uint32_t i : surv) {
    if (i < K) { nv.push_back(d->vals[i]); continue; }
    std::pair<IdDots, uint64_t> v;
    if ((rc = fetch_candidate(c, i, &v))) return rc;
    nv.push_back(std::move(v));
  }
  d->vals = std::move(nv);
  return CE_OK;
}

// ---------------------------------------------------------------------------------------
// version gate (lib.rs:519-538), device first, host for batches outside load_ops order
// ---------------------------------------------------------------------------------------
// The version gate in two halves, so its host round trip can share another's: gate_enqueue
// uploads the expected versions and queues the gate kernels and the download of their flags and
// next versions (pinned); gate_finish reads them after the caller's wait (the host gate when the
// batch is not in load_ops shape).
struct GateJob {
  uint32_t* hf = nullptr;            // pinned: [0] not grouped, [1] first gap
  unsigned long long* hnn = nullptr; // pinned: next versions per writer
  GateArgs ga{};
};

int gate_enqueue(ce_core* c, const uint32_t* d_fa, const uint64_t* d_fv, uint32_t n, uint32_t m,
                 const std::vector<uint32_t>& wslot, std::vector<uint64_t>* expect, GateJob* job,
                 const FillRange* extra = nullptr) {
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  if ((e = ctx->apply.reserve(n + 64)) || (e = c->d_gate.reserve(m * 24ull + 64)) ||
      (e = ctx->h_stage2.reserve(m * 16ull + 128)))
    return ctx->hip_fail(e, "gate reserve");
  uint64_t* he0 = ctx->h_stage2.as<uint64_t>();
  for (uint32_t a = 0; a < m; a++) he0[a] = c->nov[wslot[a]];
  expect->assign(he0, he0 + m);
  job->hnn = reinterpret_cast<unsigned long long*>(he0 + m);
  job->hf = reinterpret_cast<uint32_t*>(he0 + 2ull * m);
  GateArgs& ga = job->ga;
  ga = GateArgs{};
  ga.fa = d_fa;
  ga.fv = d_fv;
  ga.n = n;
  ga.m = m;
  uint8_t* gbase = c->d_gate.as<uint8_t>();
  ga.e0 = reinterpret_cast<const uint64_t*>(gbase);
  ga.newnov = reinterpret_cast<unsigned long long*>(gbase + 8ull * m);
  ga.run_count = reinterpret_cast<uint32_t*>(gbase + 16ull * m);
  ga.run_first = reinterpret_cast<uint32_t*>(gbase + 20ull * m);
  ga.flags = ctx->counters.as<uint32_t>() + 12;
  ga.apply = ctx->apply.as<uint8_t>();
  // one launch: e0 copied from the mapped pinned stage, the gate's scratch and flags set, and the
  // caller's extra range (the count pass's counters)
  void* he0_dev = nullptr;
  if (hipHostGetDevicePointer(&he0_dev, he0, 0) != hipSuccess) {
    (void)hipGetLastError();
    he0_dev = nullptr;
  }
  FillArgs fl{};
  if (he0_dev) fl.r[fl.n++] = {reinterpret_cast<uint32_t*>(gbase), 2ull * m, 0u, static_cast<const uint32_t*>(he0_dev)};
  else if ((e = hipMemcpyAsync(gbase, he0, m * 8ull, hipMemcpyHostToDevice, ctx->stream))) return ctx->hip_fail(e, "gate");
  fl.r[fl.n++] = {reinterpret_cast<uint32_t*>(gbase + 8ull * m), 4ull * m, 0u};
  fl.r[fl.n++] = {ga.flags, 1, 0u};
  fl.r[fl.n++] = {ga.flags + 1, 1, 0xffffffffu};
  if (extra) {
    fl.r[fl.n++] = *extra;
    // the next versions straight into the pinned words the host reads (no copy after the count)
    std::memset(job->hnn, 0, 8ull * m);
    ga.newnov_host = static_cast<unsigned long long*>(host_dev_ptr(job->hnn));
  }
  if ((e = launch_fill(ctx->stream, fl))) return ctx->hip_fail(e, "gate");
  const int t = ctx->tbegin("gate");
  if ((e = launch_gate(ctx->stream, ga))) return ctx->hip_fail(e, "gate");
  ctx->tend(t);
  // the flags come back with the caller's next download when it passes `extra` (k_ds_col_totals
  // copies them), else here
  // (with `extra`, k_gate_apply writes the next versions into job->hnn itself)
  if (!extra && ((e = hipMemcpyAsync(job->hf, ga.flags, 8, hipMemcpyDeviceToHost, ctx->stream)) ||
                 (e = hipMemcpyAsync(job->hnn, ga.newnov, m * 8ull, hipMemcpyDeviceToHost, ctx->stream))))
    return ctx->hip_fail(e, "gate");
  return CE_OK;
}

int gate_finish(ce_core* c, const uint32_t* d_fa, const uint64_t* d_fv, uint32_t n, uint32_t m,
                const GateJob& job, uint32_t* first_gap, std::vector<uint64_t>* expect) {
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  if (job.hf[0]) {
    std::vector<uint32_t> fa(n);
    std::vector<uint64_t> fv(n);
    std::vector<uint8_t> ap(n);
    if ((e = hipMemcpyAsync(fa.data(), d_fa, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = hipMemcpyAsync(fv.data(), d_fv, n * 8ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "host gate");
    for (uint32_t i = 0; i < n; i++)
      if (fa[i] >= m) return ctx->fail(CE_ERR_INVALID_ARG, "file_actor out of range");
    *first_gap = host_gate(fa.data(), fv.data(), n, expect, ap.data());
    if ((e = hipMemcpyAsync(ctx->apply.p, ap.data(), n, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "host gate");
    return CE_OK;
  }
  *first_gap = job.hf[1] == 0xffffffffu ? n : job.hf[1];
  for (uint32_t a = 0; a < m; a++) (*expect)[a] = std::max<uint64_t>((*expect)[a], job.hnn[a]);
  return CE_OK;
}

// files the device parser left to the host: re-encode compactly in place, patch the length
int resolve_host_decode(ce_core* c, uint32_t n, std::vector<int32_t>* st) {
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  for (uint32_t i = 0; i < n; i++) {
    if ((*st)[i] != kStatusHostDecode) continue;
    FileParams P;
    if ((e = hipMemcpy(&P, ctx->params.as<FileParams>() + i, sizeof P, hipMemcpyDeviceToHost)))
      return ctx->hip_fail(e, "host decode");
    std::vector<uint8_t> pt(P.len);
    if ((e = hipMemcpy(pt.data(), ctx->out.as<uint8_t>() + P.out_off, P.len, hipMemcpyDeviceToHost)))
      return ctx->hip_fail(e, "host decode");
    std::vector<HostOp> ops;
    int32_t s = CE_OK;
    if (!parse_ops_host(c->kind, pt.data() + 16, pt.size() - 16, &ops)) {
      s = CE_ERR_DECODE;
    } else {
      Wr w;
      w.b.assign(pt.begin(), pt.begin() + 16);
      encode_ops_compact(c->kind, ops, &w);
      if (w.b.size() > pt.size()) return ctx->fail(CE_ERR_DEVICE, "compact op encoding grew");
      FileParams NP = P;
      NP.len = (uint32_t)w.b.size();
      if ((e = hipMemcpy(ctx->out.as<uint8_t>() + P.out_off, w.b.data(), w.b.size(), hipMemcpyHostToDevice)) ||
          (e = hipMemcpy(ctx->params.as<FileParams>() + i, &NP, sizeof NP, hipMemcpyHostToDevice)))
        return ctx->hip_fail(e, "host decode");
    }
    (*st)[i] = s;
    if ((e = hipMemcpy(ctx->status.as<int32_t>() + i, &s, 4, hipMemcpyHostToDevice)))
      return ctx->hip_fail(e, "host decode");
  }
  return CE_OK;
}

DsDecodeArgs decode_args(ce_core* c, uint32_t n) {
  ce_ctx* ctx = c->ctx;
  DsState* d = c->ds;
  DsDecodeArgs a{};
  a.kind = c->kind == CE_STATE_ORSWOT ? kDsOrswot : kDsMVReg;
  a.pt = ctx->out.as<uint8_t>();
  a.params = ctx->params.as<FileParams>();
  a.status = ctx->status.as<int32_t>();
  a.n = n;
  a.supported = c->d_supported.as<uint8_t>();
  a.n_supported = (uint32_t)c->supported.size();
  a.apply = ctx->apply.as<uint8_t>();
  a.cnt = d->cnt.as<uint32_t>();
  a.table = c->d_table.as<ActorSlot>();
  a.mask = c->cap - 1;
  a.ops = ops_view(d);
  a.counters = d->misses.as<uint32_t>();
  a.miss_list = reinterpret_cast<uint4*>(d->misses.as<uint8_t>() + 64);
  a.miss_cap = kMissCap;
  return a;
}

int fail_first(ce_core* c, const std::vector<int32_t>& st, int32_t* status_out, uint32_t n) {
  if (status_out) std::memcpy(status_out, st.data(), n * 4ull);
  for (uint32_t i = 0; i < n; i++)
    if (st[i] != CE_OK) return st[i];
  (void)c;
  return CE_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// entry points (ce_core.h)
// ---------------------------------------------------------------------------------------
int ds_init(ce_core* c) {
  c->ds = new DsState();
  if (const char* ps = getenv("CE_DS_PRIMARY_SLOTS")) {  // tests: a fixed (tiny) primary member table
    c->ds->mcap_s = pow2_at_least(std::max(32, atoi(ps)));
    c->ds->primary_fixed = true;
  }
  if (const char* pf = getenv("CE_DS_PART_FACTOR"))  // tests: short partition runs (overflow lists)
    c->ds->part_factor = (uint32_t)std::max(0, atoi(pf));
  c->ds->kind = c->kind;
  hipError_t e;
  if ((e = c->ds->misses.reserve(64 + kMissCap * 16ull)) || (e = c->ds->h_cnt.reserve(512)))
    return c->ctx->hip_fail(e, "dot-set init");
  int rc = ensure_clock(c);
  if (rc) return rc;
  return c->kind == CE_STATE_ORSWOT ? tables_alloc(c, 4096) : CE_OK;
}

int ds_reset(ce_core* c) {
  DsState* d = c->ds;
  // an overflow poisons the core until here: the reset rebuilds every table from empty
  if (int rs = ds_settle(c); rs && !d->poisoned) return rs;
  d->poisoned = false;
  d->settle_pending = false;
  d->settle_d0.clear();
  d->deferred.clear();
  d->vals.clear();
  hipError_t e;
  const FillRange clock_zero{d->clock.as<uint32_t>(), 2ull * d->clock_cap, 0u};
  if (c->kind == CE_STATE_ORSWOT)  // the clock cleared by the tables' fill launch
    return tables_alloc(c, std::max<uint32_t>(4096, d->pcap), d->clock_cap ? &clock_zero : nullptr);
  if (d->clock_cap && (e = hipMemsetAsync(d->clock.p, 0, d->clock_cap * 8ull, c->ctx->stream)))
    return c->ctx->hip_fail(e, "reset");
  return CE_OK;
}

int ds_ingest_ops(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                  uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                  const uint64_t* d_fv, int32_t* status_out) {
  ce_ctx* ctx = c->ctx;
  DsState* d = c->ds;
  hipError_t e;
  int rc;
  if ((rc = ds_async_kick(c, false))) return rc;  // a previous compaction's download, when its seal is done
  // writers get actor ids first (the gate is keyed by them)
  std::vector<uint32_t> wslot(m);
  const uint64_t gen0 = c->table_gen;
  for (uint32_t a = 0; a < m; a++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * a, 16);
    if ((rc = insert_actor(c, u, &wslot[a]))) return rc;
  }
  if (c->table_gen != gen0) refresh_slots(c, actors, m, &wslot);  // a growth moved them
  const uint64_t gen1 = c->table_gen;
  if ((rc = table_upload(c)) || (rc = ensure_supported(c))) return rc;
  if ((e = ctx->out.reserve(blob_len + 16ull * n + 128)) || (e = ctx->status.reserve(n * 4ull + 64)) ||
      (e = d->cnt.reserve(2ull * kCntN * n * 4 + 64)))
    return ctx->hip_fail(e, "ingest reserve");
  // 1) open every file (lib.rs:501-502), plaintext -> HBM; Orswot op files of at most
  //    kDsFuseRegion bytes are decoded inside the open instead (their plaintext stays in LDS:
  //    ce_fused.hip ds_fused_decode; CE_DS_FUSED_DECODE=0 turns it off)
  HostPhase hpo("ops: open+gate+count");
  const bool fused_off = getenv("CE_DS_FUSED_DECODE") && atoi(getenv("CE_DS_FUSED_DECODE")) == 0;  // (tests flip it)
  const bool fused = c->kind == CE_STATE_ORSWOT && n > 0 && !fused_off;
  DecodeArgs fz{};
  if (fused) {
    constexpr uint32_t kRows = 64;  // ops per file the rows hold (more: the lane-per-file decode)
    static const uint32_t kEl[6] = {4, 8, 8, 4, 8, 8};
    if ((e = d->fz_cnt.reserve(4ull * kCntN * n + 64)) || (e = d->fz_done.reserve(n + 64)) ||
        (e = d->fz_big.reserve(n + 64)))
      return ctx->hip_fail(e, "fused decode");
    for (int j = 0; j < 6; j++)
      if ((e = d->fz_col[j].reserve((uint64_t)kRows * n * kEl[j] + 64))) return ctx->hip_fail(e, "fused decode");
    fz.ds.on = 1;
    fz.ds.rows = kRows;
    fz.ds.rawcnt = d->fz_cnt.as<uint32_t>();
    fz.ds.done = d->fz_done.as<uint8_t>();
    fz.ds.big = d->fz_big.as<uint8_t>();
    fz.ds.add_actor = d->fz_col[0].as<uint32_t>();
    fz.ds.add_ctr = d->fz_col[1].as<unsigned long long>();
    fz.ds.add_mem = d->fz_col[2].as<unsigned long long>();
    fz.ds.rm_actor = d->fz_col[3].as<uint32_t>();
    fz.ds.rm_ctr = d->fz_col[4].as<unsigned long long>();
    fz.ds.rm_mem = d->fz_col[5].as<unsigned long long>();
    fz.supported = c->d_supported.as<uint8_t>();
    fz.n_supported = (uint32_t)c->supported.size();
    fz.table = c->d_table.as<ActorSlot>();
    fz.mask = c->cap - 1;
    if (getenv("CE_DS_FUSE_DEBUG")) {
      if ((e = d->fz_why.reserve(4ull * n + 64)) || (e = hipMemsetAsync(d->fz_why.p, 0xff, 4ull * n + 4, ctx->stream)))
        return ctx->hip_fail(e, "fused decode");
      fz.ds.why = d->fz_why.as<uint32_t>();
    }
  }
  if ((rc = device_open(ctx, d_blob, d_offs, n, blob_len, true, key_of(c), ctx->out.as<uint8_t>(),
                        ctx->status.as<int32_t>(), false, true, fused ? &fz : nullptr)))
    return rc;
  // 2) version gate -> apply flags (decode errors reject the batch whatever the gate says),
  // 3) data version + Vec<S::Op> decode, count pass, 4) bases: one exclusive scan over the kCntN
  // count columns back to back (the emit subtracts each column's first base), then one block for
  // the column totals, maxima and a status summary.  The gate's flags and next versions and that
  // block come back in ONE wait; the statuses themselves only when a file is not OK.  Files left
  // to the host (envelope or op decoder) or a batch outside the device gate's shape: resolve on
  // the host, then the count pass again.
  uint32_t first_gap = n;
  std::vector<uint64_t> expect;
  GateJob gj;
  const FillRange count_counters{d->misses.as<uint32_t>(), 16, 0u};  // the count pass's counters
  if ((rc = gate_enqueue(c, d_fa, d_fv, n, m, wslot, &expect, &gj, &count_counters))) return rc;
  DsDecodeArgs a = decode_args(c, n);
  if (fused) {
    a.fdone = fz.ds.done;
    a.fuse = fz.ds;
  }
  const uint32_t cnt_nb = ds_count_blocks(n);
  if ((e = d->cnt_part.reserve(4ull * kDsCountPart * cnt_nb + 64))) return ctx->hip_fail(e, "count");
  a.bpart = d->cnt_part.as<uint32_t>();
  if ((uint64_t)kCntN * n > 0x7fffffffull) return ctx->fail(CE_ERR_INVALID_ARG, "batch too large for one scan");
  uint32_t* cnt = d->cnt.as<uint32_t>();
  uint32_t* bases = cnt + (size_t)kCntN * n;
  {
    size_t tb = 0;
    if ((e = d->cnt_tot.reserve(128)) || (e = ds_excl_sum_u32(nullptr, tb, cnt, bases, kCntN * n, ctx->stream)) ||
        (e = d->cub_tmp.reserve(tb + 256)))
      return ctx->hip_fail(e, "scan");
  }
  uint32_t* hsum = d->h_cnt.as<uint32_t>() + 64;  // pinned: the col_totals block (17 words)
  bool counters_clear = true;  // the gate's fill cleared them for the first pass
  auto count_pass = [&]() -> int {
    if (n == 0) {
      std::memset(hsum, 0, 20 * 4);
      hsum[18] = 0xffffffffu;
      std::memset(gj.hnn, 0, 8ull * m);  // (the gate's fill zeroed the device copy)
      return CE_OK;
    }
    size_t t = d->cub_tmp.cap;
    if (!counters_clear && (e = hipMemsetAsync(d->misses.p, 0, 64, ctx->stream))) return ctx->hip_fail(e, "count");
    counters_clear = false;
    const int tc = ctx->tbegin("ds_count");
    if ((e = launch_ds_count(ctx->stream, a))) return ctx->hip_fail(e, "count");
    ctx->tend(tc);
    if ((e = ds_excl_sum_u32(d->cub_tmp.p, t, cnt, bases, kCntN * n, ctx->stream)) ||
        (e = launch_ds_col_totals(ctx->stream, cnt, bases, n, d->misses.as<uint32_t>() + 8, a.bpart, cnt_nb,
                                  ctx->status.as<int32_t>(),
                                  ctx->counters.as<uint32_t>() + 12, d->misses.as<uint32_t>(),
                                  static_cast<uint32_t*>(host_dev_ptr(hsum)), nullptr, 0, nullptr)))
      return ctx->hip_fail(e, "count");
    return CE_OK;
  };
  auto wait = [&](const char* what) { return (e = stream_wait(ctx->stream)) ? ctx->hip_fail(e, what) : CE_OK; };
  if ((rc = count_pass()) || (rc = wait("count"))) return rc;
  gj.hf = hsum + 17;  // the gate's flags, copied by k_ds_col_totals
  if ((rc = ds_settle(c))) return rc;  // the previous fold / merge (drained by the wait above)
  bool recount = false;
  if (hsum[14]) {  // envelopes left to the host: normalize + open there, patch the batch
    if ((rc = resolve_host_parse(c, d_blob, d_offs, n, true))) return rc;
    recount = true;
  }
  recount = recount || gj.hf[0];  // not in load_ops shape: the host gate rewrites the apply flags
  if ((rc = gate_finish(c, d_fa, d_fv, n, m, gj, &first_gap, &expect))) return rc;
  if (recount && ((rc = count_pass()) || (rc = wait("count")))) return rc;
  if (hsum[15]) {  // op vectors left to the host decoder: re-encode compactly, count again
    std::vector<int32_t> st(n);
    if ((e = hipMemcpyAsync(st.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (rc = wait("count")) || (rc = resolve_host_decode(c, n, &st)) || (rc = count_pass()) || (rc = wait("count")))
      return rc ? rc : ctx->hip_fail(e, "count");
  }
  if (hsum[13] || status_out) {  // a file not OK (all-or-nothing, lib.rs:497-514), or asked for
    std::vector<int32_t> st(n);
    if ((e = hipMemcpyAsync(st.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (rc = wait("status")))
      return rc ? rc : ctx->hip_fail(e, "status");
    if ((rc = fail_first(c, st, status_out, n))) return rc;
  }
  hpo.~HostPhase();
  hpo.name = "";
  HostPhase hps("ops: scan+emit");
  Counts k, kmax;
  for (int j = 0; j < kCntN; j++) {
    k.v[j] = hsum[j];
    kmax.v[j] = hsum[8 + j];
  }
  // MVReg: the current values come first in the candidate list
  HostCols vc;
  Counts base;
  if (c->kind == CE_STATE_MVREG) {
    vals_cols(d, &vc);
    base.v[kCntRm] = vc.rm_cbeg.size();
    base.v[kCntRmC] = vc.rmc_actor.size();
  }
  Counts tot;
  for (int j = 0; j < kCntN; j++) tot.v[j] = k.v[j] + base.v[j];
  if (tot.v[kCntRmC] >= (1ull << 32) || tot.v[kCntAddM] >= (1ull << 32) || tot.v[kCntRmM] >= (1ull << 32))
    return ctx->fail(CE_ERR_INVALID_ARG, "batch too large for 32-bit op offsets");
  if ((rc = reserve_ops(c, tot))) return rc;
  if (c->kind == CE_STATE_MVREG && (rc = upload_cols(c, vc, Counts{}))) return rc;
  // 5) emit (actor ids from the device table; unknown actors -> insert and emit again)
  a = decode_args(c, n);
  a.cnt = d->cnt.as<uint32_t>() + (size_t)kCntN * n;  // bases
  const uint32_t n_fused = fused ? hsum[19] : 0;  // files the open decoded
  if (fz.ds.why) {
    std::vector<uint32_t> w(n + 1);
    if (hipMemcpy(w.data(), fz.ds.why, 4ull * (n + 1), hipMemcpyDeviceToHost) == hipSuccess) {
      std::map<uint32_t, uint32_t> h;
      for (uint32_t i = 0; i < n; i++) h[w[i] & 0xffff]++;
      fprintf(stderr, "[ds fused decode] n=%u fused=%u file0: cnt %u p0 %u nc %u; why:", n, n_fused, w[n] >> 16,
              (w[n] >> 8) & 0xff, w[n] & 0xff);
      for (auto& x : h) fprintf(stderr, " %x:%u", x.first, x.second);
      fprintf(stderr, " (file 0 %08x)\n", w[0]);
    }
  }
  if (n_fused) {
    a.fdone = fz.ds.done;
    a.fuse = fz.ds;
    for (int j = 0; j < kCntN; j++) {  // the untile's last-tile bound and LDS rows
      a.tile.total[j] = (uint32_t)k.v[j];
      a.tile.max_rows = std::max<uint32_t>(a.tile.max_rows, (uint32_t)kmax.v[j]);
    }
    c->path_counts["ds_fused_decode"]++;
    c->path_counts["ds_fused_files"] += n_fused;
  }
  for (int j = 0; j < kCntN; j++) a.base_off[j] = (uint32_t)base.v[j];
  // Orswot: the tiled emit (file-minor scratch rows, then k_ds_untile) when every file's counts
  // fit its LDS tile and the rows cost at most ~2x the columns (files of similar shape, as op
  // files in load_ops order are); the direct per-lane stores otherwise
  {
    static const int kGroup[9] = {kCntAdd, kCntAdd, kCntAdd, kCntAddM, kCntRm, kCntRm, kCntRmC, kCntRmC, kCntRmM};
    static const uint32_t kElem[9] = {4, 8, 4, 8, 4, 4, 4, 8, 8};
    const uint64_t npad = (n + 63ull) & ~63ull;
    bool tile = c->kind == CE_STATE_ORSWOT && !getenv("CE_DS_EMIT_DIRECT");
    uint64_t rows_bytes = 0, cols_bytes = 0;
    for (int cc = 0; cc < 9 && tile; cc++) {
      const uint64_t mx = kmax.v[kGroup[cc]];
      if (mx > kTileMaxRows || mx * npad >= (1ull << 32)) tile = false;
      rows_bytes += mx * npad * kElem[cc];
      cols_bytes += k.v[kGroup[cc]] * kElem[cc];
    }
    if (tile && rows_bytes > 2 * cols_bytes + (1ull << 20)) tile = false;
    if (tile) {
      for (int cc = 0; cc < 9; cc++) {
        if ((e = d->tile_col[cc].reserve(kmax.v[kGroup[cc]] * npad * kElem[cc] + 64))) return ctx->hip_fail(e, "emit tile");
        a.tile.col[cc] = d->tile_col[cc].p;
      }
      a.tile.npad = npad;
      a.tile.max_rows = 1;
      for (int j = 0; j < kCntN; j++) {
        a.tile.total[j] = (uint32_t)k.v[j];
        a.tile.max_rows = std::max<uint32_t>(a.tile.max_rows, (uint32_t)kmax.v[j]);
      }
      c->path_counts["ds_emit_tiled"]++;
    }
  }
  for (int round = 0;; round++) {
    uint32_t hm[4];
    // round 0: k_ds_col_totals (the last kernel of the count pass) cleared misses[0..8)
    if (round > 0 && (e = hipMemsetAsync(d->misses.p, 0, 64, ctx->stream))) return ctx->hip_fail(e, "emit");
    const int te = ctx->tbegin("ds_emit");
    if ((e = launch_ds_emit(ctx->stream, a, n_fused < n))) return ctx->hip_fail(e, "emit");
    ctx->tend(te);
    // are every actor's adds one contiguous run (load_ops order, each writer adding its own
    // dots)?  Then the fold's applied flags need no sort (orswot_fold); the flag rides in
    // misses[3] with the miss count
    const uint32_t n_add = (uint32_t)tot.v[kCntAdd];
    const bool check = c->kind == CE_STATE_ORSWOT && n_add > 0;
    if (check) {
      const uint32_t need = std::max<uint32_t>(1024, (uint32_t)c->id_actor.size());
      if (need > d->contig_cap) {
        const uint32_t cap = pow2_at_least(need);
        if ((e = d->contig_marks.reserve(4ull * cap)) || (e = hipMemsetAsync(d->contig_marks.p, 0, 4ull * cap, ctx->stream)))
          return ctx->hip_fail(e, "contig");
        d->contig_cap = cap;
        d->contig_gen = 0;
      }
      if (++d->contig_gen == 0) {  // wrapped: marks from 2^32 checks ago could collide
        if ((e = hipMemsetAsync(d->contig_marks.p, 0, 4ull * d->contig_cap, ctx->stream))) return ctx->hip_fail(e, "contig");
        d->contig_gen = 1;
      }
      // the miss count and the flags come back in pinned h_cnt[88..91), written by the contig
      // launch, which also computes the fold's applied flags when the runs strictly increase
      uint32_t* hp = d->h_cnt.as<uint32_t>() + 88;
      hp[0] = hp[1] = hp[2] = 0;
      DsMono mono{};
      if (!getenv("CE_DS_SORT_ADDS") && !getenv("CE_DS_NO_MONO")) {
        if ((e = d->applied.reserve(n_add + 64)) || (e = d->excl.reserve(n_add * 8ull)))
          return ctx->hip_fail(e, "applied");
        mono = DsMono{a.ops.add_ctr, d->clock.as<unsigned long long>(), d->clock_cap, d->applied.as<uint8_t>(),
                      d->excl.as<unsigned long long>()};
      }
      const int tc = ctx->tbegin("ds_contig");  // (with mono: the fold's applied flags)
      if ((e = launch_ds_contig(ctx->stream, a.ops.add_actor, n_add, d->contig_marks.as<uint32_t>(), d->contig_cap,
                                d->contig_gen, a.counters + 3, d->misses.as<uint32_t>() + 2,
                                static_cast<uint32_t*>(host_dev_ptr(hp)), mono)))
        return ctx->hip_fail(e, "contig");
      ctx->tend(tc);
      if ((e = stream_wait(ctx->stream))) return ctx->hip_fail(e, "emit");
      hm[2] = hp[0];
      hm[3] = hp[1];
      d->adds_mono = mono.ctr && hp[2] == 0;
      d->adds_mono_n = n_add;
    } else if ((e = hipMemcpyAsync(hm, d->misses.p, 16, hipMemcpyDeviceToHost, ctx->stream)) ||
               (e = stream_wait(ctx->stream))) {
      return ctx->hip_fail(e, "emit");
    }
    d->adds_contig = check && hm[3] == 0 && !getenv("CE_DS_SORT_ADDS");
    if (!check) d->adds_mono = false;
    if (hm[2] == 0) break;
    if (round > 64) return ctx->fail(CE_ERR_DEVICE, "actor table did not converge");
    const uint32_t nm = std::min<uint32_t>(hm[2], kMissCap);
    std::vector<uint4> ml(nm);
    if ((e = hipMemcpy(ml.data(), d->misses.as<uint8_t>() + 64, nm * 16ull, hipMemcpyDeviceToHost)))
      return ctx->hip_fail(e, "misses");
    for (auto& x : ml) {
      Uuid u;
      std::memcpy(u.data(), &x, 16);
      uint32_t s;
      if ((rc = insert_actor(c, u, &s))) return rc;
    }
    if ((rc = table_upload(c))) return rc;
    a.table = c->d_table.as<ActorSlot>();
    a.mask = c->cap - 1;
  }
  if ((rc = write_sentinels(c, tot))) return rc;
  hps.~HostPhase();
  hps.name = "";
  HostPhase hpf("ops: fold");
  // 6) fold (lib.rs:534-535 `state.apply(op)` for every op of every applied file, in order)
  if (c->kind == CE_STATE_ORSWOT) {
    // removal items <= members x the largest per-file clock-entry count (a removal's clock is
    // part of one file)
    rc = orswot_fold(c, tot, tot.v[kCntRmM] * std::max<uint64_t>(1, kmax.v[kCntRmC]), d->adds_contig);
    d->adds_contig = false;  // describes this batch's columns only
  } else {
    rc = mvreg_commit(c, (uint32_t)base.v[kCntRm], (uint32_t)tot.v[kCntRm], true);
  }
  if (rc) return rc;
  // 7) next_op_versions (lib.rs:537-538) and the gap error (lib.rs:527-531).  The decode's misses
  //    (actors the ops name that the table did not hold: removal clocks naming other writers)
  //    may have grown the table since the writers got their slots: refreshed first
  if (c->table_gen != gen1) refresh_slots(c, actors, m, &wslot);
  for (uint32_t w = 0; w < m; w++) c->nov[wslot[w]] = std::max(c->nov[wslot[w]], expect[w]);
  if (first_gap < n) {
    if (status_out) status_out[first_gap] = CE_ERR_OP_VERSION;
    return CE_ERR_OP_VERSION;
  }
  return CE_OK;
}

namespace {

// StateWrapper<Orswot<u64, Uuid>> / StateWrapper<MVReg<u64, Uuid>> (host flatten)
struct HostState {
  Dots nov;
  Dots clock;
  // entries flattened: member e_member[i] has dots e_dots[e_beg[i] .. e_beg[i + 1])
  std::vector<uint64_t> e_member;
  std::vector<uint32_t> e_beg{0};
  Dots e_dots;
  std::vector<std::pair<Dots, std::vector<uint64_t>>> deferred;
  std::vector<std::pair<Dots, uint64_t>> vals;
};

bool read_state(int kind, const uint8_t* p, size_t n, HostState* hs) {
  Rd r{p, n, 0};
  return read_struct(r, {"next_op_versions", "state"}, [&](int f, Rd& q) {
    if (f == 0) return read_vclock(q, &hs->nov);
    if (kind == CE_STATE_ORSWOT)
      return read_struct(q, {"clock", "entries", "deferred"}, [&](int g, Rd& s) {
        uint64_t cnt;
        if (g == 0) return read_vclock(s, &hs->clock);
        if (!rd_map_hdr(s, &cnt) || cnt > s.n) return false;
        bool ascending = true;
        for (uint64_t k = 0; k < cnt; k++) {
          if (g == 1) {
            uint64_t m;
            if (!rd_u64(s, &m) || !read_vclock(s, &hs->e_dots)) return false;
            if (k && m <= hs->e_member.back()) ascending = false;
            hs->e_member.push_back(m);
            hs->e_beg.push_back((uint32_t)hs->e_dots.size());
          } else {
            Dots key;
            std::vector<uint64_t> ms;
            if (!read_vclock(s, &key) || !read_members(s, &ms)) return false;
            hs->deferred.push_back({key, ms});
          }
        }
        if (g == 1 && !ascending) {
          // HashMap<M, VClock>: a repeated member keeps its later clock
          std::unordered_map<uint64_t, size_t> last;
          for (size_t i = 0; i < hs->e_member.size(); i++) last[hs->e_member[i]] = i;
          std::vector<uint64_t> mem;
          std::vector<uint32_t> beg{0};
          Dots dd;
          for (size_t i = 0; i < hs->e_member.size(); i++) {
            if (last[hs->e_member[i]] != i) continue;
            mem.push_back(hs->e_member[i]);
            dd.insert(dd.end(), hs->e_dots.begin() + hs->e_beg[i], hs->e_dots.begin() + hs->e_beg[i + 1]);
            beg.push_back((uint32_t)dd.size());
          }
          hs->e_member.swap(mem);
          hs->e_beg.swap(beg);
          hs->e_dots.swap(dd);
        }
        return true;
      });
    return read_struct(q, {"vals"}, [&](int, Rd& s) {
      uint64_t cnt;
      if (!rd_array_hdr(s, &cnt) || cnt > s.n) return false;
      for (uint64_t k = 0; k < cnt; k++) {
        uint64_t two, v;
        Dots dv;
        if (!rd_array_hdr(s, &two) || two != 2 || !read_vclock(s, &dv) || !rd_u64(s, &v)) return false;
        hs->vals.push_back({dv, v});
      }
      return true;
    });
  });
}

// id_dots without inserting: false when an actor is not in the table (safe on several threads)
bool id_dots_lookup(const ce_core* c, const Dots& d, IdDots* out) {
  out->clear();
  out->reserve(d.size());
  for (auto& x : d) {
    auto it = c->slot_of.find(x.first);
    if (it == c->slot_of.end()) return false;
    out->push_back({actor_id_of_slot(c, it->second), x.second});
  }
  return true;  // (in the clock's order: its users scatter it by id)
}

int id_dots(ce_core* c, Dots d, IdDots* out) {
  sort_dots(&d);
  out->clear();
  for (auto& x : d) {
    uint32_t s;
    int rc = insert_actor(c, x.first, &s);
    if (rc) return rc;
    out->push_back({actor_id_of_slot(c, s), x.second});
  }
  std::sort(out->begin(), out->end());
  return CE_OK;
}

struct OtherCols {  // the other state's (member, actor id, value) columns in HBM
  const unsigned long long* member;
  const uint32_t* actor;
  const unsigned long long* value;
  const unsigned long long* clock_host = nullptr;  // pinned dense clock by actor id, or null
  uint32_t clock_cap = 0;
  const unsigned long long* clock_dev = nullptr;   // the same dense clock already in HBM, or null
};
int orswot_merge_cols(ce_core* c, const IdDots& oclock,
                      const std::vector<std::pair<IdDots, std::vector<uint64_t>>>& od,
                      const OtherCols& oc, uint32_t n, uint32_t* live_async, bool* queued = nullptr,
                      bool want_live = true);

// Orswot::merge(other) on the device (entries) and host (deferred)
int orswot_merge_one(ce_core* c, const HostState& hs) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  int rc;
  IdDots oclock;
  if ((rc = id_dots(c, hs.clock, &oclock))) return rc;
  std::vector<unsigned long long> mem, val;
  std::vector<uint32_t> act;
  mem.reserve(hs.e_dots.size());
  act.reserve(hs.e_dots.size());
  val.reserve(hs.e_dots.size());
  {
    // actor id lookups: the state's clock names (almost) every actor of its entries
    std::unordered_map<Uuid, uint32_t, UuidHash> ids;
    ids.reserve(hs.clock.size() * 2 + 16);
    for (size_t i = 0; i < hs.e_member.size(); i++)
      for (uint32_t j = hs.e_beg[i]; j < hs.e_beg[i + 1]; j++) {
        const auto& x = hs.e_dots[j];
        if (x.second == 0) continue;  // a zero counter is no dot (absent)
        auto it = ids.find(x.first);
        uint32_t id;
        if (it != ids.end()) id = it->second;
        else {
          uint32_t sl;
          if ((rc = insert_actor(c, x.first, &sl))) return rc;
          id = actor_id_of_slot(c, sl);
          ids.emplace(x.first, id);
        }
        mem.push_back(hs.e_member[i]);
        act.push_back(id);
        val.push_back(x.second);
      }
  }
  std::vector<std::pair<IdDots, std::vector<uint64_t>>> od;
  for (auto& x : hs.deferred) {
    IdDots k;
    if ((rc = id_dots(c, x.first, &k))) return rc;
    od.push_back({k, x.second});
  }
  if ((rc = table_upload(c)) || (rc = ensure_clock(c)) || (rc = ensure_pairs(c, mem.size()))) return rc;
  hipError_t e;
  if ((e = d->other[0].reserve(mem.size() * 8 + 8)) || (e = d->other[1].reserve(act.size() * 4 + 4)) ||
      (e = d->other[2].reserve(val.size() * 8 + 8)))
    return ctx->hip_fail(e, "merge");
  if ((e = up(d->other[0].as<unsigned long long>(), mem, s)) || (e = up(d->other[1].as<uint32_t>(), act, s)) ||
      (e = up(d->other[2].as<unsigned long long>(), val, s)))
    return ctx->hip_fail(e, "merge");
  return orswot_merge_cols(c, oclock, od,
                           {d->other[0].as<unsigned long long>(), d->other[1].as<uint32_t>(),
                            d->other[2].as<unsigned long long>()},
                           (uint32_t)mem.size(), nullptr);
}

// Orswot::merge(other) with other's entries already in d->other[0..2] as (member, actor id,
// counter) columns of n pairs, its clock and deferred removals by actor id
// Orswot::merge(other) for other's columns in HBM.  With live_async set and no deferred
// removals on either side the merge is queued without a host round trip: finalize's counts are
// copied to live_async (pinned, 4 words) for the caller to read after its own synchronise, and
// used_pairs grows by the upper bound n meanwhile.
int orswot_merge_cols(ce_core* c, const IdDots& oclock,
                      const std::vector<std::pair<IdDots, std::vector<uint64_t>>>& od,
                      const OtherCols& ocols, uint32_t n, uint32_t* live_async, bool* queued,
                      bool want_live) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  int rc;
  if ((rc = ensure_clock(c))) return rc;
  hipError_t e;
  const uint32_t cap = d->clock_cap;
  // other.deferred applied, clocks merged, apply_deferred: thresholds from both deferred sets
  auto rms = deferred_list(d);
  rms.insert(rms.end(), od.begin(), od.end());
  const bool queue = live_async && rms.empty();
  const unsigned long long* oclk = d->oclock.as<unsigned long long>();
  if (queue && ocols.clock_dev && ocols.clock_cap == cap) {  // already in HBM
    oclk = ocols.clock_dev;
  } else if (queue && ocols.clock_host && ocols.clock_cap == cap) {  // pinned: no host wait
    if ((e = hipMemcpyAsync(d->oclock.p, ocols.clock_host, cap * 8ull, hipMemcpyHostToDevice, s)))
      return ctx->hip_fail(e, "merge");
  } else {
    std::vector<unsigned long long> oc(cap, 0);
    for (auto& x : oclock) oc[x.first] = x.second;
    if ((e = up(d->oclock.as<unsigned long long>(), oc, s))) return ctx->hip_fail(e, "merge");
  }
  if (queue) {
    // no deferred removals on either side: merge + finalize in one pass over the pairs, then
    // the clock; the counts come back only for the merge the caller reads them after
    const int tm = ctx->tbegin("ds_merge");
    d->scratch_dirty = true;
    if ((e = launch_ds_put_other(s, tables(d), ocols.member, ocols.actor, ocols.value, n, true)) ||
        (e = launch_ds_merge_finalize(s, tables(d), d->clock.as<unsigned long long>(), oclk)) ||
        (e = launch_merge_max(s, d->clock.as<unsigned long long>(), oclk, cap)))
      return ctx->hip_fail(e, "merge");
    d->scratch_dirty = false;  // merge_finalize cleared oth / add / kill
    ctx->tend(tm);
    if (want_live && (e = hipMemcpyAsync(live_async, d->live.p, 16, hipMemcpyDeviceToHost, s)))
      return ctx->hip_fail(e, "finalize");
    d->used_pairs += n;
    if (queued) *queued = true;
    return CE_OK;
  }
  const int tm = ctx->tbegin("ds_merge");
  d->scratch_dirty = true;
  if ((e = launch_ds_put_other(s, tables(d), ocols.member, ocols.actor, ocols.value, n)) ||
      (e = launch_ds_merge(s, tables(d), d->clock.as<unsigned long long>(), d->oclock.as<unsigned long long>())))
    return ctx->hip_fail(e, "merge");
  ctx->tend(tm);
  {
  }
  if ((rc = upload_removals(c, rms))) return rc;
  const uint32_t nr = (uint32_t)rms.size();
  if ((e = launch_ds_kill(s, tables(d), d->d0[0].as<uint32_t>(), d->d0[1].as<uint32_t>(), d->d0[2].as<uint32_t>(),
                          d->d0[3].as<unsigned long long>(), d->d0[4].as<unsigned long long>(), nr)) ||
      (e = launch_merge_max(s, d->clock.as<unsigned long long>(), d->oclock.as<unsigned long long>(), cap)))
    return ctx->hip_fail(e, "merge");
  if ((rc = finalize(c))) return rc;
  d->scratch_dirty = false;  // merge cleared oth, finalize add / kill
  std::vector<uint8_t> fl;
  if ((rc = flags_for(c, d->d0[0].as<uint32_t>(), d->d0[2].as<uint32_t>(), d->d0[3].as<unsigned long long>(), nr, &fl)))
    return rc;
  std::map<IdDots, std::set<uint64_t>> nd;
  for (uint32_t i = 0; i < nr; i++)
    if (fl[i]) nd[rms[i].first].insert(rms[i].second.begin(), rms[i].second.end());
  d->deferred = std::move(nd);
  return CE_OK;
}

int mvreg_merge_one(ce_core* c, const HostState& hs) {
  DsState* d = c->ds;
  int rc;
  HostCols hc;
  vals_cols(d, &hc);
  const uint32_t K = (uint32_t)d->vals.size();
  for (auto& v : hs.vals) {
    IdDots id;
    if ((rc = id_dots(c, v.first, &id))) return rc;
    hc.rm_cbeg.push_back((uint32_t)hc.rmc_actor.size());
    hc.rm_mbeg.push_back(0);
    for (auto& x : id) { hc.rmc_actor.push_back(x.first); hc.rmc_ctr.push_back(x.second); }
    hc.put_val.push_back(v.second);
  }
  Counts tot;
  tot.v[kCntRm] = hc.rm_cbeg.size();
  tot.v[kCntRmC] = hc.rmc_actor.size();
  if ((rc = ensure_clock(c)) || (rc = reserve_ops(c, tot)) || (rc = upload_cols(c, hc, Counts{})) ||
      (rc = write_sentinels(c, tot)))
    return rc;
  return mvreg_commit(c, K, (uint32_t)tot.v[kCntRm], false);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// read_remote_states for Orswot with the plaintexts left in HBM (ce_dotset_io.hip reader)
// ---------------------------------------------------------------------------------------
namespace {

bool key_is(Rd& r, const char* name) {
  int kind;
  uint64_t off, len;
  if (r.i >= r.n || !is_binstr_marker(r.p[r.i]) || !rd_binstr(r, &kind, &off, &len)) return false;
  return len == std::strlen(name) && std::memcmp(r.p + off, name, len) == 0;
}

// canonical StateWrapper<Orswot> head: map(2) "next_op_versions" VClock "state" map(3) "clock"
// VClock "entries" map(N) -> body offset.  0 = parsed, 1 = not the canonical layout (host
// parser), 2 = ran out of bytes (fetch a longer prefix)
int parse_state_prefix(const uint8_t* p, size_t n, bool whole, HostState* hs, uint64_t* body,
                       uint64_t* n_entries) {
  Rd r{p, n, 0};
  uint64_t cnt;
  auto fail = [&]() { return whole ? 1 : 2; };
  hs->nov.clear();
  hs->clock.clear();
  if (!rd_map_hdr(r, &cnt)) return fail();
  if (cnt != 2) return 1;
  if (!key_is(r, "next_op_versions")) return r.i >= r.n ? fail() : 1;
  if (!read_vclock(r, &hs->nov)) return fail();
  if (!key_is(r, "state")) return r.i >= r.n ? fail() : 1;
  if (!rd_map_hdr(r, &cnt)) return fail();
  if (cnt != 3) return 1;
  if (!key_is(r, "clock")) return r.i >= r.n ? fail() : 1;
  if (!read_vclock(r, &hs->clock)) return fail();
  if (!key_is(r, "entries")) return r.i >= r.n ? fail() : 1;
  if (r.i >= r.n) return fail();
  if (!rd_map_hdr(r, n_entries)) return fail();
  *body = r.i;
  return 0;
}

// "deferred" map(k) { VClock: [members] } after the entries
bool parse_state_tail(const uint8_t* p, size_t n, HostState* hs) {
  Rd r{p, n, 0};
  uint64_t cnt;
  if (!key_is(r, "deferred") || !rd_map_hdr(r, &cnt) || cnt > r.n) return false;
  hs->deferred.clear();
  for (uint64_t k = 0; k < cnt; k++) {
    Dots key;
    std::vector<uint64_t> ms;
    if (!read_vclock(r, &key) || !read_members(r, &ms)) return false;
    hs->deferred.push_back({key, ms});
  }
  return true;
}

struct DevState {
  bool device = false;
  uint64_t pt = 0;      // plaintext offset (past the 16-byte data version) in ctx->out
  uint64_t len = 0;
  uint64_t body = 0;
  uint32_t n_entries = 0, n_dots = 0, cap = 0;
  HostState hs;
  IdDots oclock;
  std::vector<std::pair<IdDots, std::vector<uint64_t>>> od;
};

hipError_t dl(void* dst, const void* src, size_t n, hipStream_t s) {
  hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
  return e ? e : stream_wait(s);
}

// per-file byte ranges of device memory -> the pinned host buffer `hb` at hoff[i], in one
// download: packed on the device first (launch_gather_ranges), since every hipMemcpyAsync is
// its own blit dispatch with its own gap on the box.  Not synchronised.
hipError_t gather_download(DsState* d, hipStream_t s, uint8_t* hb, const std::vector<GatherRange>& r,
                           uint64_t total) {
  // hb is pinned (a HostBuf): the gather kernel writes it through its device address, no staging
  // copy and no runtime copy launch
  (void)d;
  if (total == 0) return hipSuccess;
  return launch_gather_ranges(s, static_cast<uint8_t*>(host_dev_ptr(hb)), r.data(), (uint32_t)r.size());
}

// the repeat-check set of a file with n entries: a power of two >= 2 n words (mask = size - 1)
uint32_t dset_mask_for(uint64_t n) {
  uint64_t p = 64;
  while (p < 2 * n) p <<= 1;
  return (uint32_t)(p - 1);
}

OrswotReadArgs read_args(ce_core* c, DsState* d, size_t f, const DevState& ds, const uint8_t* out,
                         uint32_t cap) {
  OrswotReadArgs a{};
  a.s = out + ds.pt;
  a.lo = ds.body;
  a.hi = ds.len;
  auto& b = d->rd[f];
  // (the count straight into the pinned small words the host reads after stage 0)
  a.n_cand_dev = static_cast<uint32_t*>(host_dev_ptr(d->rd_small.as<uint32_t>())) + 2 * f;
  a.flags = d->rd_misc.as<uint32_t>() + 2 * f + 1;
  a.skip = d->rd_misc.as<uint32_t>() + 2 * f;
  a.cap = cap;
  a.n_cand = ds.n_entries;
  a.cand = b[1].as<uint32_t>();
  a.end = b[2].as<uint32_t>();
  a.ndots = b[3].as<uint32_t>();
  a.dbase = b[4].as<uint32_t>();
  a.member = b[5].as<unsigned long long>();
  a.msort = b[6].as<unsigned long long>();
  a.dset_mask = dset_mask_for(ds.n_entries);
  a.table = c->d_table.as<ActorSlot>();
  a.mask = c->cap - 1;
  return a;
}

}  // namespace

// files i = plaintexts at out + off[i] (after the 16-byte data version), len[i] bytes, st[i] =
// status so far.  Canonical Orswot states are decoded on the device; others go to read_state.
// Every stage runs over all files before its one host round trip (heads, entry counts, entry
// ends, tails, emitted columns); the merges are then queued back to back and synchronised once.
int ds_merge_states_device(ce_core* c, const uint8_t* out, const std::vector<uint64_t>& off,
                           const std::vector<uint64_t>& len, int32_t* st, int32_t* status_out) {
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  const size_t n = off.size();
  // the head prefix per file: sized from the heads the last merge met (x 1.25, 16 KiB .. 256 KiB);
  // a longer head is fetched file by file below, so the hint only saves bytes (C3: 8 x 256 KiB
  // was a 51 us blit to host memory for ~20 KiB heads)
  const uint64_t kPrefix = d->head_hint;
  if (int rs = ds_settle(c)) return rs;
  std::vector<DevState> ds(n);
  std::vector<std::vector<uint8_t>> host_pt(n);
  hipError_t e;
  int rc;
  if (d->rd.size() < n) d->rd.resize(n);
  // pinned words: [0, 2n) candidate counts / flags, [2n, 6n) entry tails, [6n, 10n) live counts
  // device words: [0, 2n) candidate counts / flags, [2n, 6n) entry tails (k_rd_tail)
  // (rd_misc's candidate counts are cleared with the reader's chunk counter, one fill launch)
  if ((e = d->rd_misc.reserve(24ull * n + 64)) || (e = d->rd_small.reserve(40ull * n + 64)))
    return ctx->hip_fail(e, "state reader");
  uint32_t* small = d->rd_small.as<uint32_t>();
  static const bool rd_debug = getenv("CE_RD_DEBUG") != nullptr;  // which stage declined a file
  int decline_stage = 0;
  auto host_parse = [&](size_t i) -> int {  // the whole plaintext through read_state
    if (rd_debug)
      fprintf(stderr, "CE_RD_DEBUG file %zu declined at stage %d (entries %u, found %u, tail %u %u %u %u, flags %u)\n", i,
              decline_stage, ds[i].n_entries, small[2 * i], small[2 * n + 4 * i], small[2 * n + 4 * i + 1],
              small[2 * n + 4 * i + 2], small[2 * n + 4 * i + 3], small[2 * i + 1]);
    ds[i].device = false;
    c->path_counts["states_host_parse"]++;
    host_pt[i].resize(len[i]);
    if (len[i] && (e = dl(host_pt[i].data(), out + off[i], len[i], s))) return ctx->hip_fail(e, "state download");
    ds[i].hs = HostState();
    if (!read_state(c->kind, host_pt[i].data(), len[i], &ds[i].hs)) st[i] = CE_ERR_DECODE;
    return CE_OK;
  };
  auto sync = [&](const char* what) { return (e = stream_wait(s)) ? ctx->hip_fail(e, what) : CE_OK; };
  int first = CE_OK;
  // dense other-clocks in pinned memory, so the queued merges never wait on a pageable copy:
  // actor-major at stride ostride for the k-way merge, file-major for the merges one by one;
  // every file's in HBM with one copy
  const uint32_t ostride = ds_oclock_stride((uint32_t)n);
  unsigned long long* hclk = nullptr;
  bool oclk_pre = false, spec = false;
  uint32_t oclk_cap = 0;
  hipEvent_t pre_ev = nullptr;  // (set: the upload goes on the side stream, after this point of s)
  auto upload_oclocks = [&](bool kway) -> int {
    const uint32_t ccap = oclk_cap = d->clock_cap;
    const size_t oc_words = kway ? (size_t)ccap * ostride : (size_t)ccap * n;
    if ((e = d->rd_clock.reserve(8ull * oc_words + 64))) return ctx->hip_fail(e, "merge");
    hclk = d->rd_clock.as<unsigned long long>();
    if (kway) {
      std::memset(hclk, 0, 8ull * oc_words);
      for (size_t i = 0; i < n; i++)
        for (auto& y : ds[i].oclock) hclk[(size_t)y.first * ostride + i] = y.second;
    } else {
      for (size_t i = 0; i < n; i++)
        if (ds[i].device) {
          std::memset(hclk + (size_t)ccap * i, 0, 8ull * ccap);
          for (auto& y : ds[i].oclock) hclk[(size_t)ccap * i + y.first] = y.second;
        }
    }
    if ((e = d->rd_oclocks.reserve(8ull * oc_words + 64))) return ctx->hip_fail(e, "merge");
    if (pre_ev) {  // beside the reader's stages (an SDMA copy); s waits for it before the merge
      if ((e = hipStreamWaitEvent(ctx->side, pre_ev, 0)) ||
          (e = hipMemcpyAsync(d->rd_oclocks.p, hclk, 8ull * oc_words, hipMemcpyHostToDevice, ctx->side)) ||
          (e = hipEventRecord(ctx->up_ev, ctx->side)) || (e = hipStreamWaitEvent(s, ctx->up_ev, 0)))
        return ctx->hip_fail(e, "merge");
      pre_ev = nullptr;
      return CE_OK;
    }
    if ((e = hipMemcpyAsync(d->rd_oclocks.p, hclk, 8ull * oc_words, hipMemcpyHostToDevice, s)))
      return ctx->hip_fail(e, "merge");
    return CE_OK;
  };
  {
    HostPhase hp("states: device read");
    // 1) the heads on the host: a prefix of every file long enough for next_op_versions and
    //    the clock (a longer one, file by file, when it is not)
    std::vector<uint64_t> poff(n + 1, 0);
    for (size_t i = 0; i < n; i++)
      poff[i + 1] = poff[i] + (st[i] == CE_OK ? std::min<uint64_t>(len[i], kPrefix) : 0);
    auto ph = std::make_unique<HostPhase>("  rd: heads download");
    if ((e = d->rd_host.reserve(poff[n] + 64))) return ctx->hip_fail(e, "state head");
    uint8_t* hb = d->rd_host.as<uint8_t>();
    {
      std::vector<GatherRange> gr;
      for (size_t i = 0; i < n; i++)
        if (poff[i + 1] > poff[i]) gr.push_back({out + off[i], poff[i], poff[i + 1] - poff[i]});
      if ((e = gather_download(d, s, hb, gr, poff[n]))) return ctx->hip_fail(e, "state head");
    }
    hipEvent_t heads_ev = nullptr;
    if ((e = stream_mark(s, &heads_ev))) return ctx->hip_fail(e, "state head");
    // 1b) queued behind the heads, stage 0 over each whole file -- the entry-head candidates in
    //     position order (count, scan, write) -- runs while the host parses the heads; the
    //     candidates before the entries (the clocks' own "dots" maps) are skipped on the device
    //     once the host knows where the entries start (k_rdm_skip)
    auto h2 = std::make_unique<HostPhase>("   rd.b stage 0");
    constexpr uint32_t kTailWin = 4096;
    std::vector<size_t> dev0;
    std::vector<OrswotReadArgs> A0;
    std::vector<int32_t> k0_of(n, -1);
    uint32_t nch = 0;
    for (size_t i = 0; i < n; i++) {
      if (st[i] != CE_OK || len[i] < 8 || len[i] > 0xffffffffull) continue;
      DevState& x = ds[i];
      x.pt = off[i];
      x.len = len[i];
      x.body = 0;
      x.n_entries = 0;
      x.cap = (uint32_t)(len[i] / 7 + 1);  // (a head takes >= 7 bytes)
      if ((e = d->rd[i][1].reserve(4ull * x.cap + 64))) return ctx->hip_fail(e, "state reader");
      OrswotReadArgs a = read_args(c, d, i, x, out, x.cap);
      a.chunk0 = nch;
      a.nchunks = orswot_read_chunks(a.lo, a.hi);
      nch += a.nchunks;
      k0_of[i] = (int32_t)A0.size();
      A0.push_back(a);
      dev0.push_back(i);
    }
    if ((e = d->rd_chunks.reserve(8ull * (nch + 1) + 64)) ||
        (e = d->rd_tmp.reserve(orswot_read_multi_tmp_bytes(nch))))
      return ctx->hip_fail(e, "state reader");
    uint32_t* chunk_cnt = d->rd_chunks.as<uint32_t>();
    uint32_t* chunk_scan = chunk_cnt + nch + 1;
    if (!A0.empty() &&
        ((e = launch_fill(s, FillArgs{{FillRange{chunk_cnt + nch, 1, 0u}, FillRange{d->rd_misc.as<uint32_t>(), 6ull * n + 1, 0u}},
                                      2, nullptr})) ||
         (e = launch_orswot_read_multi(s, nullptr, A0.data(), (uint32_t)A0.size(), 0, chunk_cnt, chunk_scan, d->rd_tmp.p,
                                       d->rd_tmp.cap))))
      return ctx->hip_fail(e, "state reader");
    h2.reset();
    if ((e = mark_wait(heads_ev))) return ctx->hip_fail(e, "state head");
    // the heads parsed and their clocks' actors looked up (read-only) on the host threads, a file
    // per task; a head longer than its prefix, a declined file and actors outside the table are
    // then handled in file order (the order the ids are handed out in)
    ph = std::make_unique<HostPhase>("  rd: heads parse + lookups");
    std::vector<int> pres(n, -1);
    std::vector<uint64_t> pbody(n, 0), pne(n, 0);
    std::vector<uint8_t> need_insert(n, 0);
    std::vector<uint32_t> todo;
    for (size_t i = 0; i < n; i++)
      if (st[i] == CE_OK) todo.push_back((uint32_t)i);
    host_parallel_for(ctx, (uint32_t)todo.size(), [&](uint32_t k) {
      const size_t i = todo[k];
      DevState& x = ds[i];
      const uint64_t want = poff[i + 1] - poff[i];
      pres[i] = parse_state_prefix(hb + poff[i], want, want == len[i], &x.hs, &pbody[i], &pne[i]);
      if (pres[i] == 0 && !id_dots_lookup(c, x.hs.clock, &x.oclock)) need_insert[i] = 1;
    });
    std::vector<size_t> dev;
    uint64_t head_max = 0;
    for (size_t i : todo) {
      DevState& x = ds[i];
      x.pt = off[i];
      x.len = len[i];
      uint64_t want = poff[i + 1] - poff[i], body = pbody[i], ne = pne[i];
      int pr = pres[i];
      std::vector<uint8_t> pre;
      const bool longer = pr == 2;
      while (pr == 2) {
        want = std::min<uint64_t>(len[i], want * 4);
        pre.resize(want);
        if ((e = dl(pre.data(), out + off[i], want, s))) return ctx->hip_fail(e, "state head");
        pr = parse_state_prefix(pre.data(), want, want == len[i], &x.hs, &body, &ne);
      }
      if (pr != 0 || ne == 0 || ne > (1ull << 30) || k0_of[i] < 0) {  // (the repeat-check set needs 2 ne < 2^32)
        decline_stage = 1;
        if ((rc = host_parse(i))) return rc;
        continue;
      }
      if (longer && !id_dots_lookup(c, x.hs.clock, &x.oclock)) need_insert[i] = 1;
      x.body = body;
      head_max = std::max<uint64_t>(head_max, body);
      x.n_entries = (uint32_t)ne;
      dev.push_back(i);
    }
    if (head_max) {
      uint64_t h = 16384;
      while (h < head_max + head_max / 4 + 1024 && h < (1u << 18)) h <<= 1;
      d->head_hint = h;
    }
    // 2) the states' actors into the table (the emitted columns carry their ids)
    ph = std::make_unique<HostPhase>("  rd: actors");
    for (size_t i : dev)
      if (need_insert[i] && (rc = id_dots(c, ds[i].hs.clock, &ds[i].oclock))) return rc;
    h2 = std::make_unique<HostPhase>("   rd.b reserve");
    // stages 1 and 2 are one launch per kind for all device files (launch_orswot_read_multi:
    // descriptors as launch arguments, gridDim.y = file), queued back to back behind stage 0 (a
    // file failing a stage is skipped by the later ones on the device), so the reader waits once
    // more: head counts, tail words, the deferred maps' bytes and the flags come back in pinned
    // memory together.  The columns are sized for the most Dots the entries' bytes can hold (a
    // non-zero Dot takes >= 19 of them).
    if ((e = d->rd_tailh.reserve((uint64_t)kTailWin * n + 64))) return ctx->hip_fail(e, "state reader");
    uint8_t* tailh = d->rd_tailh.as<uint8_t>();
    // every file still on the device path, no deferred removal held: the k-way merge is queued
    // behind stage 2 before the host wait, on the reader's device words (pair counts, a go flag
    // that is 1 only when every file was read without a flag and with an empty deferred map --
    // otherwise its kernels do nothing and the host merges below as before)
    spec = n >= 2 && n <= kRdInline && dev.size() == n && d->deferred.empty() && !getenv("CE_NO_KMERGE") &&
           !getenv("CE_NO_KMERGE_EARLY");
    uint32_t* misc = d->rd_misc.as<uint32_t>();
    std::vector<OrswotReadArgs> hA(dev.size());
    std::vector<uint64_t> dmax(n, 0);
    for (size_t k = 0; k < dev.size(); k++) {
      const size_t i = dev[k];
      DevState& x = ds[i];
      const uint64_t ne = x.n_entries;
      const uint64_t dots_max = (x.len - std::min<uint64_t>(x.len, x.body)) / 19 + 1;
      dmax[i] = dots_max;
      auto& b = d->rd[i];
      if ((e = b[2].reserve(4ull * ne + 64)) || (e = b[3].reserve(4ull * ne + 64)) ||
          (e = b[4].reserve(4ull * ne + 64)) || (e = b[5].reserve(8ull * ne + 64)) ||
          (e = b[6].reserve(8ull * (dset_mask_for(ne) + 2) + 64)) || (e = b[7].reserve(8ull * dots_max + 8)) ||
          (e = b[8].reserve(4ull * dots_max + 4)) || (e = b[9].reserve(8ull * dots_max + 8)))
        return ctx->hip_fail(e, "state reader");
      OrswotReadArgs a = read_args(c, d, i, x, out, x.cap);
      a.tail_out = static_cast<uint32_t*>(host_dev_ptr(small)) + 2 * n + 4 * i;  // pinned: no download
      a.tail_host = static_cast<uint8_t*>(host_dev_ptr(tailh)) + (uint64_t)kTailWin * i;
      a.tail_cap = kTailWin;
      a.col_member = b[7].as<unsigned long long>();
      a.col_actor = b[8].as<uint32_t>();
      a.col_value = b[9].as<unsigned long long>();
      a.tail_dev = misc + 2 * n + 4 * i;
      if (spec && k == 0) {
        a.go = misc + 6 * n;
        a.go_host = static_cast<uint32_t*>(host_dev_ptr(small)) + 10 * n;
      }
      hA[k] = a;
    }
    if ((rc = table_upload(c)) || (rc = ensure_clock(c))) return rc;
    for (auto& a : hA) {  // (the upload may have moved the table)
      a.table = c->d_table.as<ActorSlot>();
      a.mask = c->cap - 1;
    }
    h2 = std::make_unique<HostPhase>("   rd.c launch");
    const uint32_t nd = (uint32_t)dev.size();
    if (nd == n && n >= 2 && n <= 64 && d->deferred.empty()) {  // (the other-clocks' upload, below)
      if ((!ctx->side && (e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking))) ||
          (!ctx->up_ev && (e = hipEventCreateWithFlags(&ctx->up_ev, hipEventDisableTiming))) ||
          (!ctx->side_ev && (e = hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming))) ||
          (e = hipEventRecord(ctx->side_ev, s)))
        return ctx->hip_fail(e, "state reader");
      pre_ev = ctx->side_ev;
    }
    if (nd && ((e = launch_orswot_read_multi(s, nullptr, hA.data(), nd, 1, nullptr, nullptr, nullptr, 0)) ||
               (e = launch_orswot_read_multi(s, nullptr, hA.data(), nd, 2, nullptr, nullptr, nullptr, 0))))
      return ctx->hip_fail(e, "state reader");
    // the k-way merge's dense other-clocks (below), built and uploaded while stages 1-2 run when
    // every file is still on the device path (else they are rebuilt for the merges one by one)
    oclk_pre = n >= 2 && n <= 64 && dev.size() == n && d->deferred.empty() && !getenv("CE_NO_KMERGE");
    if (oclk_pre && (rc = upload_oclocks(true))) return rc;
    // the reader's wait is for the stages only, not for the merge queued behind them
    hipEvent_t stages_ev = nullptr;
    if (!A0.empty() && (e = stream_mark(s, &stages_ev))) return ctx->hip_fail(e, "state reader");
    if (spec) {
      uint64_t bound = 0;
      for (size_t i = 0; i < n; i++) bound += dmax[i];
      if ((rc = ensure_pairs(c, bound))) return rc;
      if ((e = d->cx_slot.reserve(4 * bound + 64))) return ctx->hip_fail(e, "merge");
      std::vector<DsMergeSrc> hs(n);
      for (size_t i = 0, q = 0; i < n; q += dmax[i], i++) {
        auto& b = d->rd[i];
        hs[i] = DsMergeSrc{b[7].as<unsigned long long>(), b[8].as<uint32_t>(), b[9].as<unsigned long long>(),
                           (uint32_t)dmax[i], d->cx_slot.as<uint32_t>() + q, misc + 2 * n + 4 * i};
      }
      // no pair in the table yet (read_remote after a reset: C3's state files): the merge reads no
      // current values
      const bool fresh = d->used_pairs == 0 && !d->settle_pending;
      d->scratch_dirty = true;
      if ((e = launch_ds_kmerge(s, tables(d), nullptr, hs.data(), (uint32_t)n, d->clock.as<unsigned long long>(),
                                d->rd_oclocks.as<unsigned long long>(), d->clock_cap, ostride,
                                d->hold.as<unsigned long long>(),
                                static_cast<uint32_t*>(host_dev_ptr(d->h_cnt.as<uint32_t>() + 56)), misc + 6 * n,
                                fresh)))
        return ctx->hip_fail(e, "merge");
      d->scratch_dirty = false;  // (k_ds_kfinal cleared oth / hold, or nothing ran)
    }
    h2 = std::make_unique<HostPhase>("   rd.d sync");
    // (also when no file is left for stage 1: stage 0 may still be running over the candidates)
    if (!A0.empty() && (e = mark_wait(stages_ev))) return ctx->hip_fail(e, "state reader");
    h2.reset();
    // 3) the first N heads in position order are the entries (count in small[2i]); the tail words
    //    (end, dbase, Dots of the last entry, flags after stage 1) in small[2n + 4i]
    ph = std::make_unique<HostPhase>("  rd: entries");
    std::vector<uint64_t> toff(n + 1, 0), eend(n, 0);
    std::vector<size_t> dev3;
    for (size_t k = 0; k < dev.size(); k++) {
      const size_t i = dev[k];
      const uint32_t found = small[2 * i];
      DevState& x = ds[i];
      if (found < x.n_entries || found > x.cap) {  // fewer heads than entries, or overflow
        decline_stage = 2;
        if ((rc = host_parse(i))) return rc;
        continue;
      }
      const uint32_t* tail = small + 2 * n + 4 * i;
      eend[i] = x.body + (uint64_t)tail[0];
      if (tail[3] == 0 && tail[0] != 0xffffffffu && eend[i] <= len[i]) {
        x.n_dots = tail[1] + tail[2];
        dev3.push_back(i);
      } else if ((decline_stage = 3) && (rc = host_parse(i))) {
        return rc;
      }
    }
    // 4) the deferred maps after the entries, on the host: from the pinned window (k_rdm_tail),
    //    or downloaded when longer
    ph = std::make_unique<HostPhase>("  rd: tails");
    uint64_t ttot = 0;
    for (size_t i : dev3)
      if (len[i] - eend[i] > kTailWin) { toff[i] = ttot; ttot += len[i] - eend[i]; }
    if (ttot) {
      if ((e = d->rd_host.reserve(ttot + 64))) return ctx->hip_fail(e, "state tail");
      hb = d->rd_host.as<uint8_t>();
      std::vector<GatherRange> gr;
      for (size_t i : dev3)
        if (len[i] - eend[i] > kTailWin) gr.push_back({out + off[i] + eend[i], toff[i], len[i] - eend[i]});
      if ((e = gather_download(d, s, hb, gr, ttot))) return ctx->hip_fail(e, "state tail");
      if ((rc = sync("state tail"))) return rc;
    }
    std::vector<size_t> dev4;
    for (size_t i : dev3) {
      const uint64_t tl = len[i] - eend[i];
      const uint8_t* tp = tl > kTailWin ? hb + toff[i] : tailh + (uint64_t)kTailWin * i;
      if (parse_state_tail(tp, tl, &ds[i].hs)) {
        DevState& x = ds[i];
        x.od.clear();
        for (auto& y : x.hs.deferred) {
          IdDots k;
          if ((rc = id_dots(c, y.first, &k))) return rc;
          x.od.push_back({k, y.second});
        }
        dev4.push_back(i);
      } else if ((decline_stage = 4) && (rc = host_parse(i))) {
        return rc;
      }
    }
    // 5) the emitted (member, actor id, value) columns of every entry Dot; an actor outside the
    //    table (not in the state's clock) flagged the file for the host parser (small[2i + 1])
    ph = std::make_unique<HostPhase>("  rd: emit");
    if ((rc = table_upload(c))) return rc;  // (the deferred maps' actors)
    for (size_t i : dev4) {
      if (small[2 * i + 1] == 0) {
        ds[i].device = true;
        c->path_counts["states_device_read"]++;
      } else if ((decline_stage = 5) && (rc = host_parse(i))) {
        return rc;
      }
    }
    for (size_t i = 0; i < n; i++)
      if (st[i] != CE_OK && first == CE_OK) first = st[i];
  }
  if (status_out) std::memcpy(status_out, st, n * 4);
  if (first != CE_OK) return first;  // nothing merged (lib.rs:431-456)
  HostPhase hp("states: merge");
  // every file read on the device and no deferred removal anywhere: all merges in one pass
  // (launch_ds_kmerge; the order-free form of the merges below)
  bool kway = n >= 2 && n <= 64 && d->deferred.empty() && !getenv("CE_NO_KMERGE");
  for (size_t i = 0; i < n && kway; i++) kway = ds[i].device && ds[i].od.empty();
  const bool early = spec && small[10 * n] != 0;  // the k-way merge queued before the wait ran
  if (early && !kway) {
    // the early merge already changed the pair table and the clock: later calls must fail until
    // ce_core_reset (all-or-nothing, lib.rs:431-456), as after a table overflow
    d->poisoned = true;
    return ctx->fail(CE_ERR_DEVICE, "state reader: early merge for a declined file");
  }
  uint64_t dev_dots = 0;
  for (size_t i = 0; i < n; i++)
    if (ds[i].device) dev_dots += ds[i].n_dots;
  if (!early && (rc = ensure_pairs(c, dev_dots))) return rc;
  uint32_t* live = small + 6 * n;
  const uint32_t ccap = d->clock_cap;
  if (!early && !(kway && oclk_pre && oclk_cap == ccap) && (rc = upload_oclocks(kway))) return rc;
  if (early) c->path_counts["states_kway_early"]++;
  if (kway) {
    HostPhase hk("  merge: k-way");
    if (!early) {  // (else queued before the reader's wait, on its device words)
      if ((e = d->rd_args_h.reserve(n * sizeof(DsMergeSrc) + 64)) || (e = d->rd_args_d.reserve(n * sizeof(DsMergeSrc) + 64)))
        return ctx->hip_fail(e, "merge");
      uint64_t dots = 0;
      for (size_t i = 0; i < n; i++) dots += ds[i].n_dots;
      if ((e = d->cx_slot.reserve(4 * dots + 64))) return ctx->hip_fail(e, "merge");
      auto* hs = d->rd_args_h.as<DsMergeSrc>();
      for (size_t i = 0, q = 0; i < n; q += ds[i].n_dots, i++) {
        auto& b = d->rd[i];
        hs[i] = DsMergeSrc{b[7].as<unsigned long long>(), b[8].as<uint32_t>(), b[9].as<unsigned long long>(), ds[i].n_dots,
                           d->cx_slot.as<uint32_t>() + q};
      }
      // no host wait: the merged counts land in pinned memory for ds_settle (the next ingest's
      // first wait), like a fold's
      const bool fresh = d->used_pairs == 0 && !d->settle_pending;
      d->scratch_dirty = true;
      if ((e = launch_ds_kmerge(s, tables(d), nullptr, hs, (uint32_t)n,
                                d->clock.as<unsigned long long>(), d->rd_oclocks.as<unsigned long long>(), ccap, ostride,
                                d->hold.as<unsigned long long>(),
                                static_cast<uint32_t*>(host_dev_ptr(d->h_cnt.as<uint32_t>() + 56)), nullptr, fresh)))
        return ctx->hip_fail(e, "merge");
    }
    c->path_counts["states_kway_merge"]++;
    d->scratch_dirty = false;  // k_ds_kfinal cleared oth / hold
    d->settle_pending = true;
    d->settle_fold = false;
    d->settle_delta = false;
    d->settle_members = true;
    for (size_t i = 0; i < n; i++)
      for (auto& y : ds[i].hs.nov) {
        uint32_t sl;
        if ((rc = insert_actor(c, y.first, &sl))) return rc;
        c->nov[sl] = std::max(c->nov[sl], y.second);
      }
    return table_upload(c);
  }
  size_t last_dev = n;
  for (size_t i = 0; i < n; i++)
    if (ds[i].device) last_dev = i;
  std::vector<uint8_t> queued(n, 0);
  bool last_queued = false;
  for (size_t i = 0; i < n; i++) {  // lib.rs:458-466, in order
    DevState& x = ds[i];
    if (x.device) {
      auto& b = d->rd[i];
      bool q = false;
      OtherCols oc{b[7].as<unsigned long long>(), b[8].as<uint32_t>(), b[9].as<unsigned long long>(),
                   hclk + (size_t)ccap * i, ccap, d->rd_oclocks.as<unsigned long long>() + (size_t)ccap * i};
      if ((rc = ensure_pairs(c, x.n_dots)) ||
          (rc = orswot_merge_cols(c, x.oclock, x.od, oc, x.n_dots, live + 4 * i, &q, i == last_dev)))
        return rc;
      queued[i] = q;
      last_queued = q;
    } else {
      if ((rc = orswot_merge_one(c, x.hs))) return rc;
      last_queued = false;
    }
    for (auto& y : x.hs.nov) {
      uint32_t sl;
      if ((rc = insert_actor(c, y.first, &sl))) return rc;
      c->nov[sl] = std::max(c->nov[sl], y.second);
    }
  }
  {
    HostPhase hs("  merge: wait");
    if ((rc = sync("merge"))) return rc;
  }
  // the overflow flag (live[2]) is sticky on the device: the last merge's download carries it
  if (last_dev < n && queued[last_dev] && live[4 * last_dev + 2])
    return ctx->fail(CE_ERR_DEVICE, "dot-set table overflow");
  for (size_t i = n; i-- > 0;)
    if (queued[i]) {
      if (last_queued) {
        d->live_pairs = live[4 * i];
        d->used_pairs = live[4 * i + 1];
      }
      break;
    }
  return table_upload(c);
}

int ds_merge_states(ce_core* c, const std::vector<std::pair<const uint8_t*, size_t>>& sws,
                    int32_t* st, int32_t* status_out) {
  if (int rs = ds_settle(c)) return rs;
  const size_t n = sws.size();
  std::vector<HostState> hs(n);
  int first = CE_OK;
  {
    HostPhase hp("states: host parse");
    // one host thread per state file (files are independent; the merge below stays in order)
    auto parse = [&](size_t i) {
      if (st[i] == CE_OK && !read_state(c->kind, sws[i].first, sws[i].second, &hs[i])) st[i] = CE_ERR_DECODE;
    };
    size_t big = 0;
    for (size_t i = 0; i < n; i++) big += sws[i].second >= (1u << 16);
    if (n > 1 && big > 1) {
      std::vector<std::thread> th;
      const size_t T = std::min<size_t>(16, n);
      for (size_t t = 0; t < T; t++)
        th.emplace_back([&, t] {
          for (size_t i = t; i < n; i += T) parse(i);
        });
      for (auto& x : th) x.join();
    } else {
      for (size_t i = 0; i < n; i++) parse(i);
    }
    for (size_t i = 0; i < n; i++)
      if (st[i] != CE_OK && first == CE_OK) first = st[i];
  }
  if (status_out) std::memcpy(status_out, st, n * 4);
  if (first != CE_OK) return first;  // nothing merged (lib.rs:431-456)
  HostPhase hp("states: merge");
  for (size_t i = 0; i < n; i++) {   // lib.rs:458-466
    int rc = c->kind == CE_STATE_ORSWOT ? orswot_merge_one(c, hs[i]) : mvreg_merge_one(c, hs[i]);
    if (rc) return rc;
    for (auto& x : hs[i].nov) {
      uint32_t s;
      if ((rc = insert_actor(c, x.first, &s))) return rc;
      c->nov[s] = std::max(c->nov[s], x.second);
    }
  }
  return table_upload(c);
}

int ds_check_ops(ce_core* c, const uint8_t* ops, size_t len) {
  if (int rs = ds_settle(c)) return rs;
  std::vector<HostOp> v;
  if (!parse_ops_host(c->kind, ops, len, &v))
    return c->ctx->fail(CE_ERR_DECODE, c->kind == CE_STATE_ORSWOT ? "ops are not a Vec<orswot::Op<u64, Uuid>>"
                                                                 : "ops are not a Vec<mvreg::Op<u64, Uuid>>");
  return CE_OK;
}

int ds_apply_local_ops(ce_core* c, const uint8_t* ops, size_t len) {
  if (int rs = ds_settle(c)) return rs;
  DsState* d = c->ds;
  std::vector<HostOp> v;
  if (!parse_ops_host(c->kind, ops, len, &v)) return c->ctx->fail(CE_ERR_DECODE, "ops");
  HostCols hc;
  Counts base;
  if (c->kind == CE_STATE_MVREG) {
    vals_cols(d, &hc);
    base.v[kCntRm] = hc.rm_cbeg.size();
    base.v[kCntRmC] = hc.rmc_actor.size();
  }
  int rc = host_cols(c, v, Counts{}, &hc);  // offsets continue after the current values in hc
  if (rc) return rc;
  Counts tot;
  tot.v[kCntAdd] = hc.add_actor.size();
  tot.v[kCntAddM] = hc.add_mem.size();
  tot.v[kCntRm] = hc.rm_cbeg.size();
  tot.v[kCntRmC] = hc.rmc_actor.size();
  tot.v[kCntRmM] = hc.rm_mem.size();
  if ((rc = table_upload(c)) || (rc = ensure_clock(c)) || (rc = reserve_ops(c, tot)) ||
      (rc = upload_cols(c, hc, Counts{})) || (rc = write_sentinels(c, tot)))
    return rc;
  if (c->kind == CE_STATE_ORSWOT) {
    uint64_t items = 0;  // removal items, exactly
    const size_t nr = hc.rm_cbeg.size();
    for (size_t r = 0; r < nr; r++) {
      const uint64_t ce = r + 1 < nr ? hc.rm_cbeg[r + 1] : hc.rmc_actor.size();
      const uint64_t me = r + 1 < nr ? hc.rm_mbeg[r + 1] : hc.rm_mem.size();
      items += (ce - hc.rm_cbeg[r]) * (me - hc.rm_mbeg[r]);
    }
    return orswot_fold(c, tot, items, false);
  }
  return mvreg_commit(c, (uint32_t)base.v[kCntRm], (uint32_t)tot.v[kCntRm], true);
}

// Compaction of an Orswot state without bringing the entries to the host: the clear text
// (prefix16 || to_vec_named(StateWrapper), the same bytes as ds_serialize) is written into
// x->blob by the device writer (ce_dotset_io.hip) around a host-built head (next_op_versions,
// clock) and tail (deferred), sealed on the device and downloaded once.
// The device writer itself: prefix16 || to_vec_named(StateWrapper) into `dst` when dst_cap covers
// the bound U, else into x->blob (*clear = where it went), with the seal's staging words
// (offsets [0, clear len, out offset], stats, nonce, outer version) at x->blob + *A.  Queued on
// x->stream; the clear length lands in the second offset word.
static int ds_serialize_dev(ce_core* c, ce_ctx* x, const uint8_t* outer, const uint8_t* prefix16,
                            const uint8_t* nonce, uint8_t* dst, uint64_t dst_cap, uint64_t* A_out,
                            uint64_t* U_out, uint8_t** clear) {
  DsState* d = c->ds;
  hipStream_t s = x->stream;
  hipError_t e;
  int rc;
  auto uuid_dots = [&](const IdDots& v) {
    Dots o;
    for (auto& y : v) o.push_back({c->id_actor[y.first], y.second});
    sort_dots(&o);
    return o;
  };
  auto put_vclock = [](Wr& w, const Dots& v) {
    w.map(1);
    w.str("dots");
    w.map(v.size());
    for (auto& y : v) { w.bin(y.first.data(), 16); w.uint(y.second); }
  };
  // actor UUIDs and UUID-order ranks by stable id (host copies kept: nov and the clock are
  // written in UUID order by walking the ranks -- no per-step sort)
  auto cph = std::make_unique<HostPhase>("  cd: actor order");
  const uint32_t na = (uint32_t)c->id_actor.size();
  if (d->uuid_ids != na) {
    std::vector<uint8_t> u(16ull * na + 16);
    d->rank_id.resize(na);
    d->id_rank.assign(na + 1, 0);
    for (uint32_t i = 0; i < na; i++) {
      std::memcpy(u.data() + 16ull * i, c->id_actor[i].data(), 16);
      d->rank_id[i] = i;
    }
    std::sort(d->rank_id.begin(), d->rank_id.end(), [&](uint32_t a, uint32_t b) { return c->id_actor[a] < c->id_actor[b]; });
    for (uint32_t i = 0; i < na; i++) d->id_rank[d->rank_id[i]] = i;
    if ((e = d->uuid_of_id.reserve(u.size())) || (e = d->rank_of_id.reserve(4ull * d->id_rank.size())) ||
        (e = d->id_of_rank.reserve(4ull * d->rank_id.size() + 64)) ||
        (e = hipMemcpyAsync(d->uuid_of_id.p, u.data(), u.size(), hipMemcpyHostToDevice, s)) ||
        (e = hipMemcpyAsync(d->rank_of_id.p, d->id_rank.data(), 4ull * d->id_rank.size(), hipMemcpyHostToDevice, s)) ||
        (na && (e = hipMemcpyAsync(d->id_of_rank.p, d->rank_id.data(), 4ull * na, hipMemcpyHostToDevice, s))) ||
        (e = stream_wait(s)))
      return x->hip_fail(e, "actor ranks");
    d->uuid_ids = na;
  }
  // head: [prefix16] map(2) "next_op_versions" nov "state" map(3) "clock" clock "entries"
  cph = std::make_unique<HostPhase>("  cd: nov");
  std::vector<uint64_t> by_rank(na, 0);
  for (uint32_t sl = 0; sl < c->cap; sl++)
    if (c->h_table[sl].used && c->nov[sl]) by_rank[d->id_rank[actor_id_of_slot(c, sl)]] = c->nov[sl];
  Dots nov;
  for (uint32_t r = 0; r < na; r++)
    if (by_rank[r]) nov.push_back({c->id_actor[d->rank_id[r]], by_rank[r]});
  if ((rc = ensure_clock(c))) return rc;
  cph = std::make_unique<HostPhase>("  cd: collect + clock");
  if ((e = d->h_clock.reserve(8ull * na + 64))) return x->hip_fail(e, "clock download");
  // live pairs -> columns, their count and largest member, and the clock: one wait
  uint32_t nl = 0;
  unsigned long long max_member = 0;
  if ((rc = collect(c, &nl, &max_member, d->h_clock.p, d->clock.p, 8ull * na)) || (rc = ds_settle(c))) return rc;
  // the sorts and scans over the collected pairs first (they need nothing from the host): the
  // head and tail bytes below are built while they run
  cph = std::make_unique<HostPhase>("  cd: sort enqueue");
  for (int k = 0; k < 17; k++) {
    // 0-3 u32 sort keys / perms, 4-6 u64 keys / sorted members / values, 7-10 actors, heads,
    // ranks, lengths, 11 entry CSR (n + 1), 12 byte offsets, 13-14 u64 values and 16 u64 keys
    // (the radix sort's ping-pong), 15 the scans' scratch (below)
    if (k == 15) continue;
    const size_t sz = (k >= 4 && k <= 6) || k >= 13 ? 8ull * nl + 64 : 4ull * nl + 68;
    if ((e = d->ser[k].reserve(sz))) return x->hip_fail(e, "ds compact reserve");
  }
  if ((e = d->ser[15].reserve(orswot_ser_tmp_bytes(std::max<uint32_t>(nl, 1))))) return x->hip_fail(e, "ds compact reserve");
  if (ser_sort_state_words(nl) > d->ser_sort_words) {  // (zero once; the sorts keep it so)
    const size_t w = ser_sort_state_words(std::max<uint32_t>(nl, 1u << 20));
    if ((e = d->ser_sort.reserve(4 * w + 64)) || (e = hipMemsetAsync(d->ser_sort.p, 0, 4 * w + 64, s)))
      return x->hip_fail(e, "ds compact reserve");
    d->ser_sort_words = w;
    d->ser_sort_gen = 0;
  }
  OrswotSerScratch sc{};
  sc.member_in = d->col[0].as<unsigned long long>();
  sc.actor_in = d->col[1].as<uint32_t>();
  sc.value_in = d->col[2].as<unsigned long long>();
  sc.rank_of_id = d->rank_of_id.as<uint32_t>();
  sc.id_of_rank = d->id_of_rank.as<uint32_t>();
  sc.rank_bits = bits_for(na);
  sc.member_bits = max_member ? 64 - __builtin_clzll(max_member) : 1;  // radix passes over those bits only
  sc.k32a = d->ser[0].as<uint32_t>();
  sc.k32b = d->ser[1].as<uint32_t>();
  sc.p32a = d->ser[2].as<uint32_t>();
  sc.p32b = d->ser[3].as<uint32_t>();
  sc.k64a = d->ser[4].as<unsigned long long>();
  sc.member_sorted = d->ser[5].as<unsigned long long>();
  sc.value_sorted = d->ser[6].as<unsigned long long>();
  sc.actor_sorted = d->ser[7].as<uint32_t>();
  sc.head = d->ser[8].as<uint32_t>();
  sc.hrank = d->ser[9].as<uint32_t>();
  sc.len = d->ser[10].as<uint32_t>();
  sc.seg = d->ser[11].as<uint32_t>();
  sc.pos = d->ser[12].as<uint32_t>();
  sc.tmp = d->ser[15].p;
  sc.tmp_bytes = d->ser[15].cap;
  sc.sort_state = d->ser_sort.as<uint32_t>();
  sc.sort_gen = &d->ser_sort_gen;
  sc.v64a = d->ser[13].as<unsigned long long>();
  sc.v64b = d->ser[14].as<unsigned long long>();
  sc.k64b = d->ser[16].as<unsigned long long>();
  const int t = x->tbegin("ds_serialize");
  if ((e = launch_orswot_ser_sort(s, sc, nl))) return x->hip_fail(e, "ds serialize");
  const unsigned long long* ck = d->h_clock.as<unsigned long long>();
  cph = std::make_unique<HostPhase>("  cd: head + tail bytes");
  Dots clock;
  for (uint32_t r = 0; r < na; r++) {
    const uint32_t id = d->rank_id[r];
    if (ck[id]) clock.push_back({c->id_actor[id], ck[id]});
  }
  Wr hw;
  if (prefix16) hw.b.insert(hw.b.end(), prefix16, prefix16 + 16);
  hw.map(2);
  hw.str("next_op_versions");
  put_vclock(hw, nov);
  hw.str("state");
  hw.map(3);
  hw.str("clock");
  put_vclock(hw, clock);
  hw.str("entries");
  // tail: "deferred" map {VClock bytes: [members]} sorted by the clock's bytes
  Wr tw;
  tw.str("deferred");
  std::vector<std::pair<std::vector<uint8_t>, const std::set<uint64_t>*>> df;
  for (auto& y : d->deferred) {
    Wr kw;
    put_vclock(kw, uuid_dots(y.first));
    df.push_back({kw.b, &y.second});
  }
  std::sort(df.begin(), df.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  tw.map(df.size());
  for (auto& y : df) {
    tw.b.insert(tw.b.end(), y.first.begin(), y.first.end());
    tw.arr(y.second->size());
    for (uint64_t m : *y.second) tw.uint(m);
  }
  cph = std::make_unique<HostPhase>("  cd: serialize + seal enqueue");
  // clear text bound: head + map header + entries (member <= 9 + 6 + 5, Dot <= 18 + 9) + tail
  const uint64_t U = hw.b.size() + 5 + 20ull * nl + 27ull * nl + tw.b.size();
  const uint64_t A = (U + 255) & ~255ull;  // [offs(2) | out_offs(1) | stats | nonce | outer] after it
  const uint64_t total_max = 16 + sealed_len(U);
  if ((e = x->blob.reserve(A + 256 + hw.b.size() + tw.b.size())) ||
      (e = x->h_stage.reserve(std::max<uint64_t>(total_max + 64, 256 + hw.b.size() + tw.b.size()))))
    return x->hip_fail(e, "ds compact reserve");
  uint8_t* db = x->blob.as<uint8_t>();
  uint8_t* hs = x->h_stage.as<uint8_t>();
  std::memset(hs, 0, 128);
  if (nonce) std::memcpy(hs + 32, nonce, 24);
  else if (outer) os_random(hs + 32, 24);
  if (outer) std::memcpy(hs + 56, outer, 16);
  std::memcpy(hs + 128, hw.b.data(), hw.b.size());
  std::memcpy(hs + 128 + hw.b.size(), tw.b.data(), tw.b.size());
  if ((e = hipMemcpyAsync(db + A, hs, 128 + hw.b.size() + tw.b.size(), hipMemcpyHostToDevice, s)))
    return x->hip_fail(e, "ds compact upload");
  OrswotSerArgs a{};
  a.out = dst && dst_cap >= U ? dst : db;
  a.prefix = db + A + 128;
  a.prefix_len = hw.b.size();
  a.suffix = db + A + 128 + hw.b.size();
  a.suffix_len = tw.b.size();
  a.uuid_of_id = d->uuid_of_id.as<uint8_t>();
  a.n = nl;
  auto* offs = reinterpret_cast<unsigned long long*>(db + A);  // [0] 0, [1] clear len, [2] out_offs
  a.seal_offs = offs;
  a.stats = reinterpret_cast<uint32_t*>(db + A + 24);
  if ((e = launch_orswot_ser_write(s, sc, a))) return x->hip_fail(e, "ds serialize");
  x->tend(t);
  *A_out = A;
  *U_out = U;
  *clear = a.out;
  return CE_OK;
}

int ds_async_kick(ce_core* c, bool force) {
  if (!c->pend) return CE_OK;
  hipError_t e = force ? hipEventSynchronize(c->seal_ev) : hipEventQuery(c->seal_ev);
  if (e == hipErrorNotReady) return CE_OK;
  if (e) return c->ctx->hip_fail(e, "compact download");
  const uint32_t slot = c->pend_slot;
  const uint64_t n = c->copy_len.as<volatile uint64_t>()[slot];
  if (!c->dma_tried) {
    c->dma_tried = true;
    (void)dma_init(c->ctx->device, &c->dma);
  }
  // an SDMA engine when the HSA runtime gives one (the compute units and their memory path stay
  // with the next batch), else the HIP runtime's copy on the copy stream
  c->copy_dma[slot] = false;
  if (n < ~1ull && c->dma.ok && (c->copy_sig[slot].handle || dma_signal(&c->copy_sig[slot])) &&
      dma_d2h(c->dma, c->pend_dst, c->ds->seal_out.p, n, c->copy_sig[slot])) {
    c->copy_dma[slot] = true;
    c->path_counts["compact_download_sdma"]++;
  } else {
    if (n < ~1ull && (e = hipMemcpyAsync(c->pend_dst, c->ds->seal_out.p, n, hipMemcpyDeviceToHost, c->copy_stream)))
      return c->ctx->hip_fail(e, "compact download");
    if ((e = hipEventRecord(c->copy_ev[slot], c->copy_stream))) return c->ctx->hip_fail(e, "compact download");
  }
  c->copy_last_slot = (int)slot;
  c->pend = false;
  return CE_OK;
}

// wait for the newest download (it reads seal_out): on the host (device = false) or, for a
// runtime copy, ordered before the next work on stream s
int ds_download_fence(ce_core* c, hipStream_t s, bool device) {
  if (c->copy_last_slot < 0) return CE_OK;
  const int k = c->copy_last_slot;
  if (c->copy_dma[k]) {
    dma_wait(c->copy_sig[k]);
    return CE_OK;
  }
  hipError_t e = device ? hipStreamWaitEvent(s, c->copy_ev[k], 0) : hipEventSynchronize(c->copy_ev[k]);
  return e ? c->ctx->hip_fail(e, "compact download") : CE_OK;
}

int ds_compact_device(ce_core* c, ce_ctx* x, const uint8_t* outer, const uint8_t* prefix16,
                      const uint8_t* nonce, const KeyRef& key, std::vector<uint8_t>* file) {
  HostPhase hp("ds compact (device writer)");
  c->path_counts["compact_device_writer"]++;
  // a previous compact_into_async's download reads seal_out: enqueue it before this seal
  if (int rk = ds_async_kick(c, true)) return rk;
  hipStream_t s = x->stream;
  hipError_t e;
  int rc;
  uint64_t A = 0, U = 0;
  uint8_t* clear = nullptr;
  if ((rc = ds_serialize_dev(c, x, outer, prefix16, nonce, nullptr, 0, &A, &U, &clear))) return rc;
  uint8_t* db = x->blob.as<uint8_t>();
  auto* offs = reinterpret_cast<unsigned long long*>(db + A);
  auto cph = std::make_unique<HostPhase>("  cd: seal enqueue");
  // the sealed file in its own buffer (the next ingest reuses the context's plaintext buffer
  // while an async download of this file may still run); a previous compaction's download may
  // still read it: the seal waits for it on the device, a reallocation on the host
  DsState* d = c->ds;
  const uint64_t total_max = 16 + sealed_len(U);
  if (total_max + 64 > d->seal_out.cap && (rc = ds_download_fence(c, s, false))) return rc;
  if ((e = d->seal_out.reserve(total_max + 64))) return x->hip_fail(e, "ds compact reserve");
  if ((rc = ds_download_fence(c, s, true))) return rc;
  rc = device_seal(x, db, reinterpret_cast<const uint64_t*>(offs), 1, U, db + A + 56, db + A + 32,
                   d->seal_out.as<uint8_t>(), reinterpret_cast<const uint64_t*>(db + A + 16), key);
  if (rc) return rc;
  // compact_into_async: no host round trip.  A one-lane kernel behind the seal writes the file's
  // length into a pinned slot; the download (the runtime's DMA engine copy, which leaves the
  // CUs and HBM to the next batch) is enqueued on the copy stream by ds_async_kick once the
  // seal is done -- at the next batch's first host wait, or at ce_core_compact_wait.
  bool pinned = false;
  if (c->sink_async && c->sink) {
    hipPointerAttribute_t pa{};
    pinned = hipPointerGetAttributes(&pa, c->sink) == hipSuccess && pa.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // an unregistered pointer leaves an error behind
  }
  if (pinned && !getenv("CE_ASYNC_OFF")) {
    cph = std::make_unique<HostPhase>("  cd: async download");
    if ((!c->copy_stream && (e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking))) ||
        (!c->seal_ev && (e = hipEventCreateWithFlags(&c->seal_ev, hipEventDisableTiming))))
      return x->hip_fail(e, "ds compact download");
    if (!c->copy_len_dev) {
      void* dp = nullptr;
      if ((e = c->copy_len.reserve(8ull * ce_core::kAsyncSlots)) || (e = hipHostGetDevicePointer(&dp, c->copy_len.p, 0)))
        return x->hip_fail(e, "ds compact download");
      c->copy_len_dev = static_cast<uint64_t*>(dp);
    }
    const uint64_t t = ++c->copy_next;
    const uint32_t slot = (uint32_t)(t % ce_core::kAsyncSlots);
    hipEvent_t& ev = c->copy_ev[slot];
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return x->hip_fail(e, "ds compact download");
    if (c->copy_slot_ticket[slot]) {  // the slot's previous copy
      if (c->copy_dma[slot]) dma_wait(c->copy_sig[slot]);
      else if ((e = hipEventSynchronize(ev))) return x->hip_fail(e, "ds compact download");
    }
    if ((e = launch_publish_sealed_len(s, reinterpret_cast<const uint64_t*>(db + A + 8), U, c->sink_cap,
                                       c->copy_len_dev + slot)) ||
        (e = hipEventRecord(c->seal_ev, s)))
      return x->hip_fail(e, "ds compact download");
    c->pend = true;
    c->pend_slot = slot;
    c->pend_dst = c->sink;
    c->path_counts["compact_async"]++;
    c->copy_slot_ticket[slot] = t;
    c->sink_ticket = t;
    c->sink_len = 0;  // known when the ticket completes
    file->clear();
    return CE_OK;
  }
  cph = std::make_unique<HostPhase>("  cd: length wait");
  uint64_t clear_len = 0;
  if ((e = hipMemcpyAsync(&clear_len, db + A + 8, 8, hipMemcpyDeviceToHost, s)) || (e = stream_wait(s)))
    return x->hip_fail(e, "ds compact");
  if (clear_len > U) return x->fail(CE_ERR_DEVICE, "serializer overran its bound");
  const uint64_t total = 16 + sealed_len(clear_len);
  uint8_t* to = nullptr;
  if (c->sink && total <= c->sink_cap) {  // compact_into: straight into the caller's buffer
    file->clear();
    c->sink_len = total;
    to = c->sink;
  } else {
    file->resize(total);
    to = file->data();
  }
  cph = std::make_unique<HostPhase>("  cd: download");
  if ((e = hipMemcpyAsync(to, d->seal_out.p, total, hipMemcpyDeviceToHost, s)) || (e = stream_wait(s)))
    return x->hip_fail(e, "ds compact download");
  return CE_OK;
}

// to_vec_named(StateWrapper<Orswot>) into device memory (the dot-set exchange between GPUs,
// crdtenc shard.reduce_dotset): the device writer straight into dst when cap covers its bound,
// else through x->blob.  *len = the length; CE_ERR_INVALID_ARG (nothing written) when cap < *len.
int ds_state_bytes_device(ce_core* c, ce_ctx* x, uint8_t* dst, uint64_t cap, uint64_t* len) {
  hipStream_t s = x->stream;
  hipError_t e;
  int rc;
  uint64_t A = 0, U = 0;
  uint8_t* clear = nullptr;
  if ((rc = ds_serialize_dev(c, x, nullptr, nullptr, nullptr, dst, cap, &A, &U, &clear))) return rc;
  const uint8_t* db = x->blob.as<uint8_t>();
  uint64_t n = 0;
  if ((e = hipMemcpyAsync(&n, db + A + 8, 8, hipMemcpyDeviceToHost, s)) || (e = stream_wait(s)))
    return x->hip_fail(e, "state bytes");
  if (n > U) return x->fail(CE_ERR_DEVICE, "serializer overran its bound");
  *len = n;
  if (clear == dst) return CE_OK;
  if (n > cap) return x->fail(CE_ERR_INVALID_ARG, "device buffer too small for the state");
  // complete on return, like the direct write: the caller's collective runs on another stream
  if (n && ((e = hipMemcpyAsync(dst, clear, n, hipMemcpyDeviceToDevice, s)) || (e = stream_wait(s))))
    return x->hip_fail(e, "state bytes");
  return CE_OK;
}

// ---- the multi-GPU exchange as columns (include/crdtenc.h ce_core_export_columns_device) ----
// A rank's partial Orswot goes to the compacting rank as columns -- the live (member, actor,
// counter) pairs straight from the collect, its clock and next_op_versions, its actor UUIDs --
// instead of a serialized StateWrapper that the receiver parses back (read_remote_states' merge,
// crdt-enc/src/lib.rs:458-466, of every rank's partial).  Layout (byte offsets, 8-aligned):
//   0 u32 magic 'CECL' | u32 version 1 | u64 pairs np | u32 actors na | u32 flags | u64 dlen
//   32 uuid[16 na] | clock u64[na] | nov u64[na] | member u64[np] | value u64[np] | actor u32[np]
//   then, when flags bit 0 (the partial holds deferred removals), at the next 8-byte boundary the
//   deferred map as dlen bytes of CSR arrays (what the kill / deferred-flag kernels read in place):
//   u64 n_rm, n_ent, n_mem, 0 | cbeg u32[n_rm + 1] | mbeg u32[n_rm + 1] | pad8 | actor u32[n_ent] |
//   pad8 | counter u64[n_ent] | member u64[n_mem]
// (actor = an index into the partial's own UUID list).
namespace {
constexpr uint32_t kColsMagic = 0x4c434543u;  // "CECL"
constexpr uint32_t kColsDeferred = 1u;        // flags: a deferred section follows the columns
struct ColsHeader {
  uint32_t magic, version;
  uint64_t np;
  uint32_t na, flags;
  uint64_t dlen;  // bytes of the deferred section (0 without one)
};
static_assert(sizeof(ColsHeader) == 32, "column partial header");
uint64_t cols_len(uint64_t na, uint64_t np) { return 32 + 32 * na + 20 * np; }
uint64_t cols_def_off(uint64_t na, uint64_t np) { return (cols_len(na, np) + 7) & ~7ull; }
uint64_t al8(uint64_t x) { return (x + 7) & ~7ull; }
// byte offsets inside a deferred section (from its start)
struct DefLayout {
  uint64_t cbeg, mbeg, act, ctr, mem, len;
  DefLayout(uint64_t n_rm, uint64_t n_ent, uint64_t n_mem) {
    cbeg = 32;
    mbeg = cbeg + 4 * (n_rm + 1);
    act = al8(mbeg + 4 * (n_rm + 1));
    ctr = al8(act + 4 * n_ent);
    mem = ctr + 8 * n_ent;
    len = mem + 8 * n_mem;
  }
};
}  // namespace

int ds_export_columns_device(ce_core* c, uint8_t* dst, uint64_t cap, uint64_t* len) {
  if (int rs = ds_settle(c)) return rs;
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  *len = 0;
  if (c->kind != CE_STATE_ORSWOT)
    return ctx->fail(CE_ERR_INVALID_ARG, "no column form (not an Orswot): use the state bytes");
  if (!dst && cap == 0) {  // the query form: *len = 1, the state has a column form
    *len = 1;
    return CE_ERR_INVALID_ARG;
  }
  int rc;
  hipError_t e;
  if ((rc = ensure_clock(c))) return rc;
  uint32_t nl = 0;
  if ((rc = collect(c, &nl))) return rc;
  const uint32_t na = (uint32_t)c->id_actor.size();
  // the deferred map (on the host) as CSR arrays by this core's actor ids
  std::vector<uint8_t> dw;
  if (!d->deferred.empty()) {
    uint64_t ne = 0, nm = 0;
    for (auto& x : d->deferred) {
      ne += x.first.size();
      nm += x.second.size();
    }
    const uint64_t nr = d->deferred.size();
    const DefLayout L(nr, ne, nm);
    dw.assign(L.len, 0);
    uint64_t* hdr = reinterpret_cast<uint64_t*>(dw.data());
    hdr[0] = nr;
    hdr[1] = ne;
    hdr[2] = nm;
    uint32_t* cb = reinterpret_cast<uint32_t*>(dw.data() + L.cbeg);
    uint32_t* mb = reinterpret_cast<uint32_t*>(dw.data() + L.mbeg);
    uint32_t* ac = reinterpret_cast<uint32_t*>(dw.data() + L.act);
    uint64_t* ct = reinterpret_cast<uint64_t*>(dw.data() + L.ctr);
    uint64_t* me = reinterpret_cast<uint64_t*>(dw.data() + L.mem);
    uint32_t r = 0, e = 0, q = 0;
    cb[0] = mb[0] = 0;
    for (auto& x : d->deferred) {
      for (auto& y : x.first) {
        ac[e] = y.first;
        ct[e++] = y.second;
      }
      for (uint64_t m : x.second) me[q++] = m;
      cb[++r] = e;
      mb[r] = q;
    }
  }
  const uint64_t o_def = cols_def_off(na, nl), dlen = dw.size();
  const uint64_t need = dw.empty() ? cols_len(na, nl) : o_def + dlen;
  *len = need;
  if (need > cap) return ctx->fail(CE_ERR_INVALID_ARG, "device buffer too small for the columns");
  // header, UUIDs, next versions by id and the deferred words: built in pinned memory, read by
  // the copy launch
  if ((e = d->cx_host.reserve(32 + 24ull * na + dlen + 64))) return ctx->hip_fail(e, "columns");
  uint8_t* h = d->cx_host.as<uint8_t>();
  const ColsHeader hd{kColsMagic, 1u, nl, na, dw.empty() ? 0u : kColsDeferred, dlen};
  std::memcpy(h, &hd, 32);
  for (uint32_t i = 0; i < na; i++) std::memcpy(h + 32 + 16ull * i, c->id_actor[i].data(), 16);
  uint64_t* hn = reinterpret_cast<uint64_t*>(h + 32 + 16ull * na);
  std::fill(hn, hn + na, 0ull);
  for (uint32_t sl = 0; sl < c->cap; sl++)
    if (c->h_table[sl].used && c->nov[sl]) hn[actor_id_of_slot(c, sl)] = c->nov[sl];
  const uint32_t* hdev = static_cast<const uint32_t*>(host_dev_ptr(h));
  const uint64_t o_clock = 32 + 16ull * na, o_nov = o_clock + 8ull * na, o_mem = o_nov + 8ull * na,
                 o_val = o_mem + 8ull * nl, o_act = o_val + 8ull * nl;
  auto w = [&](uint64_t o) { return reinterpret_cast<uint32_t*>(dst + o); };
  FillArgs fl{};
  fl.r[fl.n++] = {w(0), (32 + 16ull * na) / 4, 0u, hdev};
  fl.r[fl.n++] = {w(o_clock), 2ull * na, 0u, d->clock.as<uint32_t>()};
  fl.r[fl.n++] = {w(o_nov), 2ull * na, 0u, hdev + (32 + 16ull * na) / 4};
  fl.r[fl.n++] = {w(o_mem), 2ull * nl, 0u, d->col[0].as<uint32_t>()};
  fl.r[fl.n++] = {w(o_val), 2ull * nl, 0u, d->col[2].as<uint32_t>()};
  fl.r[fl.n++] = {w(o_act), nl, 0u, d->col[1].as<uint32_t>()};
  if (!dw.empty()) {
    std::memcpy(h + 32 + 24ull * na, dw.data(), dlen);  // (32 + 24 na: 8-aligned)
    fl.r[fl.n++] = {w(o_def), dlen / 4, 0u, hdev + (32 + 24ull * na) / 4};
  }
  // complete on return, as the state-bytes export: the caller's collective runs on another stream
  const int tx = ctx->tbegin("cols_export");
  if ((e = launch_fill(s, fl))) return ctx->hip_fail(e, "columns");
  ctx->tend(tx);
  if ((e = stream_wait(s))) return ctx->hip_fail(e, "columns");
  c->path_counts["columns_export"]++;
  return CE_OK;
}

int ds_merge_columns_device(ce_core* c, const uint8_t* const* parts, const uint64_t* lens, uint32_t k) {
  if (int rs = ds_settle(c)) return rs;
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  if (c->kind != CE_STATE_ORSWOT)
    return ctx->fail(CE_ERR_INVALID_ARG, "no column merge (not an Orswot): use the state bytes");
  if (k == 0) return CE_OK;
  if (k > 64) return ctx->fail(CE_ERR_INVALID_ARG, "at most 64 column partials per merge");
  hipError_t e;
  int rc;
  std::optional<HostPhase> ph;  // CE_HOST_PROF
  ph.emplace("  cols: download");
  // 1) every part's header, UUIDs, clock and next versions in one gathered download, sized for
  //    as many actors as this core knows (a second one only for parts naming more)
  const uint64_t guess = 32 + 32ull * std::max<uint64_t>(c->id_actor.size(), 64);
  std::vector<uint64_t> pre(k), poff(k);
  uint64_t tot = 0;
  for (uint32_t f = 0; f < k; f++) {
    if (lens[f] < 32) return ctx->fail(CE_ERR_DECODE, "not a column partial");
    pre[f] = std::min<uint64_t>(lens[f], guess) & ~7ull;
    poff[f] = tot;
    tot += pre[f];
  }
  if ((e = d->cx_host.reserve(tot + 64))) return ctx->hip_fail(e, "columns");
  {
    std::vector<GatherRange> gr;
    for (uint32_t f = 0; f < k; f++) gr.push_back({parts[f], poff[f], pre[f]});
    if ((e = gather_download(d, s, d->cx_host.as<uint8_t>(), gr, tot)) || (e = stream_wait(s)))
      return ctx->hip_fail(e, "columns");
  }
  std::vector<ColsHeader> hd(k);
  std::vector<const uint8_t*> base(k);
  uint64_t np_tot = 0, more = 0;
  for (uint32_t f = 0; f < k; f++) {
    base[f] = d->cx_host.as<uint8_t>() + poff[f];
    std::memcpy(&hd[f], base[f], 32);
    const bool hasdef = hd[f].flags == kColsDeferred;
    const uint64_t want = hasdef ? cols_def_off(hd[f].na, hd[f].np) + hd[f].dlen : cols_len(hd[f].na, hd[f].np);
    if (hd[f].magic != kColsMagic || hd[f].version != 1 || (hd[f].flags & ~kColsDeferred) ||
        (hasdef ? (hd[f].dlen < 40 || (hd[f].dlen & 7)) : hd[f].dlen != 0) || want != lens[f] ||
        hd[f].np >= (1ull << 31))
      return ctx->fail(CE_ERR_DECODE, "not a column partial");
    np_tot += hd[f].np;
    if (32 + 32ull * hd[f].na > pre[f]) more += 32 + 32ull * hd[f].na;
  }
  if (more) {
    if ((e = d->cx_heads.reserve(more + 64))) return ctx->hip_fail(e, "columns");
    std::vector<GatherRange> gr;
    uint64_t o = 0;
    for (uint32_t f = 0; f < k; f++)
      if (32 + 32ull * hd[f].na > pre[f]) {
        gr.push_back({parts[f], o, 32 + 32ull * hd[f].na});
        base[f] = d->cx_heads.as<uint8_t>() + o;
        o += 32 + 32ull * hd[f].na;
      }
    if ((e = gather_download(d, s, d->cx_heads.as<uint8_t>(), gr, more)) || (e = stream_wait(s)))
      return ctx->hip_fail(e, "columns");
  }
  // the parts' deferred maps (Orswot::merge merges other.deferred, lib.rs:458-466): only their
  // 32-byte heads come to the host; the CSR arrays are read in place by the kill and deferred-flag
  // kernels after the k-way merge below, their actors mapped to this core's ids on the device
  struct PartDef {
    uint32_t f;
    uint64_t n_rm, n_ent, n_mem, ent0, rm0;
    const uint8_t* base;
    DefLayout L{0, 0, 0};
  };
  std::vector<PartDef> pdef;
  uint64_t def_ent = 0, def_rm = 0;
  {
    std::vector<GatherRange> gr;
    uint64_t o = 0;
    for (uint32_t f = 0; f < k; f++)
      if (hd[f].flags & kColsDeferred) {
        gr.push_back({parts[f] + cols_def_off(hd[f].na, hd[f].np), o, 32});
        o += 32;
      }
    if (o) {
      ph.emplace("  cols: deferred heads");
      if ((e = d->cx_dheads.reserve(o + 64))) return ctx->hip_fail(e, "columns");
      if ((e = gather_download(d, s, d->cx_dheads.as<uint8_t>(), gr, o)) || (e = stream_wait(s)))
        return ctx->hip_fail(e, "columns");
      const uint64_t* q = d->cx_dheads.as<uint64_t>();
      uint32_t qi = 0;
      for (uint32_t f = 0; f < k; f++) {
        if (!(hd[f].flags & kColsDeferred)) continue;
        PartDef x;
        x.f = f;
        x.n_rm = q[4 * qi];
        x.n_ent = q[4 * qi + 1];
        x.n_mem = q[4 * qi + 2];
        qi++;
        if (x.n_rm > hd[f].dlen || x.n_ent > hd[f].dlen || x.n_mem > hd[f].dlen || x.n_rm >= (1ull << 31) ||
            x.n_ent >= (1ull << 31) || x.n_mem >= (1ull << 31))  // (the kernels index them in 32 bits)
          return ctx->fail(CE_ERR_DECODE, "column partial: deferred map");
        x.L = DefLayout(x.n_rm, x.n_ent, x.n_mem);
        if (x.L.len != hd[f].dlen) return ctx->fail(CE_ERR_DECODE, "column partial: deferred map");
        x.base = parts[f] + cols_def_off(hd[f].na, hd[f].np);
        x.ent0 = def_ent;
        x.rm0 = def_rm;
        def_ent += x.n_ent;
        def_rm += x.n_rm;
        pdef.push_back(x);
      }
    }
  }
  // every deferred section checked on the device (offsets ordered and in range, actor indices in
  // the part's list) before this core's state or the remap and kill kernels touch anything
  if (!pdef.empty()) {
    if ((e = d->cx_defact.reserve(4 * def_ent + 64)) || (e = d->cx_defflag.reserve(def_rm + 64 + 4 * (uint64_t)k)))
      return ctx->hip_fail(e, "columns");
    uint32_t* bad = reinterpret_cast<uint32_t*>(d->cx_defflag.as<uint8_t>() + ((def_rm + 3) & ~3ull));
    std::vector<uint32_t> hb(pdef.size());
    if ((e = hipMemsetAsync(bad, 0, 4 * hb.size(), s))) return ctx->hip_fail(e, "columns");
    for (size_t i = 0; i < pdef.size(); i++) {
      const PartDef& x = pdef[i];
      if ((e = launch_ds_csr_check(s, reinterpret_cast<const uint32_t*>(x.base + x.L.cbeg),
                                   reinterpret_cast<const uint32_t*>(x.base + x.L.mbeg),
                                   reinterpret_cast<const uint32_t*>(x.base + x.L.act), (uint32_t)x.n_rm,
                                   (uint32_t)x.n_ent, (uint32_t)x.n_mem, hd[x.f].na, bad + i)))
        return ctx->hip_fail(e, "columns");
    }
    if ((e = hipMemcpyAsync(hb.data(), bad, 4 * hb.size(), hipMemcpyDeviceToHost, s)) || (e = stream_wait(s)))
      return ctx->hip_fail(e, "columns");
    for (uint32_t b : hb)
      if (b) return ctx->fail(CE_ERR_DECODE, "column partial: deferred map");
  }
  ph.emplace("  cols: actors");
  // 2) every part's actors in this core's table (ids), next_op_versions merged (VClock::merge).
  //    A part whose UUID list is this core's id order (every rank registered the same actors)
  //    maps by identity, its next versions through the cached id -> slot list.
  auto idslot = [&]() {
    if (d->cx_idslot_gen != c->table_gen || d->cx_idslot.size() != c->id_actor.size()) {
      d->cx_idslot.assign(c->id_actor.size(), 0u);
      for (uint32_t sl = 0; sl < c->cap; sl++)
        if (c->h_table[sl].used) d->cx_idslot[actor_id_of_slot(c, sl)] = sl;
      d->cx_idslot_gen = c->table_gen;
    }
  };
  uint64_t maps = 0;
  for (uint32_t f = 0; f < k; f++) maps += hd[f].na;
  if ((e = d->cx_map.reserve(4 * maps + 64)) || (e = d->cx_mapd.reserve(4 * maps + 64)) ||
      (e = d->cx_ids.reserve(4 * np_tot + 64)) || (e = d->cx_slot.reserve(4 * np_tot + 64)))
    return ctx->hip_fail(e, "columns");
  uint32_t* hmap = d->cx_map.as<uint32_t>();
  {
    uint64_t m = 0;
    for (uint32_t f = 0; f < k; f++) {
      const uint32_t na = hd[f].na;
      const uint8_t* u = base[f] + 32;
      const uint64_t* nv = reinterpret_cast<const uint64_t*>(u + 24ull * na);
      const bool ident = na <= c->id_actor.size() && (na == 0 || std::memcmp(u, c->id_actor.data(), 16ull * na) == 0);
      if (ident) {
        idslot();  // (an earlier part's new actors may have moved the slots)
        for (uint32_t i = 0; i < na; i++) {
          hmap[m + i] = i;
          if (nv[i]) {
            uint64_t& x = c->nov[d->cx_idslot[i]];
            x = std::max(x, nv[i]);
          }
        }
      } else {
        for (uint32_t i = 0; i < na; i++) {
          Uuid id;
          std::memcpy(id.data(), u + 16ull * i, 16);
          uint32_t sl;
          if ((rc = insert_actor(c, id, &sl))) return rc;
          hmap[m + i] = actor_id_of_slot(c, sl);
          if (nv[i]) c->nov[sl] = std::max(c->nov[sl], nv[i]);
        }
      }
      m += na;
    }
  }
  ph.emplace("  cols: tables");
  if ((rc = table_upload(c)) || (rc = ensure_clock(c)) || (rc = ensure_pairs(c, np_tot))) return rc;
  ph.emplace("  cols: launch");
  // 3) maps uploaded and the dense other-clocks zeroed in one launch, then the remap
  const uint32_t ccap = d->clock_cap, ostride = ds_oclock_stride(k);
  if ((e = d->rd_oclocks.reserve(8ull * ccap * ostride + 64))) return ctx->hip_fail(e, "columns");
  FillArgs fl{};
  fl.r[fl.n++] = {d->cx_mapd.as<uint32_t>(), maps, 0u, static_cast<const uint32_t*>(host_dev_ptr(hmap))};
  fl.r[fl.n++] = {d->rd_oclocks.as<uint32_t>(), 2ull * ccap * ostride, 0u};
  std::vector<DsColsRemap> rm(k);
  std::vector<DsMergeSrc> src(k);
  {
    uint64_t m = 0, q = 0;
    for (uint32_t f = 0; f < k; f++) {
      const uint64_t na = hd[f].na, np = hd[f].np;
      const uint8_t* b = parts[f];
      const uint64_t o_clock = 32 + 16 * na, o_mem = o_clock + 16 * na, o_val = o_mem + 8 * np, o_act = o_val + 8 * np;
      rm[f] = DsColsRemap{reinterpret_cast<const uint32_t*>(b + o_act), d->cx_ids.as<uint32_t>() + q,
                          d->cx_mapd.as<uint32_t>() + m, reinterpret_cast<const unsigned long long*>(b + o_clock),
                          d->rd_oclocks.as<unsigned long long>() + f, (uint32_t)np, (uint32_t)na, ostride};
      src[f] = DsMergeSrc{reinterpret_cast<const unsigned long long*>(b + o_mem), d->cx_ids.as<uint32_t>() + q,
                          reinterpret_cast<const unsigned long long*>(b + o_val), (uint32_t)np,
                          d->cx_slot.as<uint32_t>() + q};
      m += na;
      q += np;
    }
  }
  // the deferred sections' actors: part-local -> this core's ids (k_cols_remap, no clock), and a
  // check of their CSR bounds on the device before any kernel walks them
  if (!pdef.empty()) {
    uint64_t mo = 0;
    std::vector<uint64_t> moff(k);
    for (uint32_t f = 0; f < k; f++) {
      moff[f] = mo;
      mo += hd[f].na;
    }
    for (size_t i = 0; i < pdef.size(); i++) {
      const PartDef& x = pdef[i];
      rm.push_back(DsColsRemap{reinterpret_cast<const uint32_t*>(x.base + x.L.act), d->cx_defact.as<uint32_t>() + x.ent0,
                               d->cx_mapd.as<uint32_t>() + moff[x.f], nullptr, nullptr, (uint32_t)x.n_ent, 0u, 0u});
    }
  }
  // 4) one k-way merge of every part into the state (launch_ds_kmerge; the live counts land in
  //    pinned memory for ds_settle, like the state files' merge)
  d->scratch_dirty = true;
  const int tm = ctx->tbegin("cols_merge");
  if ((fl.n && (e = launch_fill(s, fl))) || (e = launch_cols_remap(s, rm.data(), (uint32_t)rm.size())) ||
      (e = launch_ds_kmerge(s, tables(d), nullptr, src.data(), k, d->clock.as<unsigned long long>(),
                            d->rd_oclocks.as<unsigned long long>(), ccap, ostride, d->hold.as<unsigned long long>(),
                            static_cast<uint32_t*>(host_dev_ptr(d->h_cnt.as<uint32_t>() + 56)))))
    return ctx->hip_fail(e, "columns");
  ctx->tend(tm);
  d->scratch_dirty = false;
  d->settle_pending = true;
  d->settle_fold = false;
  d->settle_delta = false;
  d->settle_members = true;
  c->path_counts["columns_merge"]++;
  // the parts may be reused by the caller after the return: the merge reads them
  ph.emplace("  cols: settle");
  if ((rc = ds_settle(c))) return rc;
  // 5) deferred removals (ours and the parts'): every removal's thresholds over the merged pairs
  //    (apply_rm's reset_remove), finalize, and the removals the merged clock does not cover stay
  //    deferred (apply_deferred) -- order-free, as the merge rule above
  if (!pdef.empty() || !d->deferred.empty()) {
    ph.emplace("  cols: apply deferred");
    RmCsr own;  // this core's deferred removals (uploaded), then the parts' in place
    std::vector<const std::pair<const IdDots, std::set<uint64_t>>*> ownp;
    for (auto& x : d->deferred) {
      for (auto& y : x.first) {
        own.act.push_back(y.first);
        own.ctr.push_back(y.second);
      }
      for (uint64_t mv : x.second) own.mem.push_back(mv);
      own.close();
      ownp.push_back(&x);
    }
    const uint32_t no = own.size();
    if (no && (rc = upload_removals_csr(c, own))) return rc;
    if (no && (e = launch_ds_kill(s, tables(d), d->d0[0].as<uint32_t>(), d->d0[1].as<uint32_t>(), d->d0[2].as<uint32_t>(),
                                  d->d0[3].as<unsigned long long>(), d->d0[4].as<unsigned long long>(), no)))
      return ctx->hip_fail(e, "columns");
    for (auto& x : pdef) {
      if ((e = launch_ds_kill(s, tables(d), reinterpret_cast<const uint32_t*>(x.base + x.L.cbeg),
                              reinterpret_cast<const uint32_t*>(x.base + x.L.mbeg), d->cx_defact.as<uint32_t>() + x.ent0,
                              reinterpret_cast<const unsigned long long*>(x.base + x.L.ctr),
                              reinterpret_cast<const unsigned long long*>(x.base + x.L.mem), (uint32_t)x.n_rm)))
        return ctx->hip_fail(e, "columns");
    }
    d->scratch_dirty = true;
    if ((rc = finalize(c))) return rc;
    d->scratch_dirty = false;
    // which removals the merged clock does not cover (they stay deferred): the parts' flags on the
    // device, one download
    std::vector<uint8_t> fo, fp(def_rm);
    if ((rc = flags_for(c, d->d0[0].as<uint32_t>(), d->d0[2].as<uint32_t>(), d->d0[3].as<unsigned long long>(), no, &fo)))
      return rc;
    for (auto& x : pdef)
      if (x.n_rm && (e = launch_ds_deferred(s, reinterpret_cast<const uint32_t*>(x.base + x.L.cbeg),
                                            d->cx_defact.as<uint32_t>() + x.ent0,
                                            reinterpret_cast<const unsigned long long*>(x.base + x.L.ctr),
                                            d->clock.as<unsigned long long>(), d->cx_defflag.as<uint8_t>() + x.rm0,
                                            (uint32_t)x.n_rm)))
        return ctx->hip_fail(e, "columns");
    if (def_rm && ((e = hipMemcpyAsync(fp.data(), d->cx_defflag.p, def_rm, hipMemcpyDeviceToHost, s)) || (e = stream_wait(s))))
      return ctx->hip_fail(e, "columns");
    std::map<IdDots, std::set<uint64_t>> nd;
    for (uint32_t i = 0; i < no; i++)
      if (fo[i]) nd[ownp[i]->first].insert(ownp[i]->second.begin(), ownp[i]->second.end());
    for (auto& x : pdef) {  // (usually none: the merged clock covers what the partials deferred)
      bool any = false;
      for (uint64_t i = 0; i < x.n_rm && !any; i++) any = fp[x.rm0 + i] != 0;
      if (!any) continue;
      std::vector<uint8_t> sec(x.L.len);
      std::vector<uint32_t> ids(x.n_ent);
      if ((e = hipMemcpyAsync(sec.data(), x.base, x.L.len, hipMemcpyDeviceToHost, s)) ||
          (x.n_ent && (e = hipMemcpyAsync(ids.data(), d->cx_defact.as<uint32_t>() + x.ent0, 4 * x.n_ent,
                                          hipMemcpyDeviceToHost, s))) ||
          (e = stream_wait(s)))
        return ctx->hip_fail(e, "columns");
      const uint32_t* cb = reinterpret_cast<const uint32_t*>(sec.data() + x.L.cbeg);
      const uint32_t* mb = reinterpret_cast<const uint32_t*>(sec.data() + x.L.mbeg);
      const uint64_t* ct = reinterpret_cast<const uint64_t*>(sec.data() + x.L.ctr);
      const uint64_t* me = reinterpret_cast<const uint64_t*>(sec.data() + x.L.mem);
      for (uint64_t i = 0; i < x.n_rm; i++) {
        if (!fp[x.rm0 + i]) continue;
        IdDots kk;
        for (uint32_t j = cb[i]; j < cb[i + 1]; j++)
          if (ct[j]) kk.push_back({ids[j], ct[j]});
        std::sort(kk.begin(), kk.end());
        nd[kk].insert(me + mb[i], me + mb[i + 1]);
      }
    }
    d->deferred = std::move(nd);
    c->path_counts["columns_merge_deferred"]++;
  }
  return CE_OK;
}

// canonical to_vec_named(StateWrapper<S>) (lib.rs:336, 739-743); HashMap / HashSet contents
// sorted (members ascending, deferred clocks by their msgpack bytes) -- SURVEY.md F9
int ds_serialize(ce_core* c, std::vector<uint8_t>* out) {
  if (int rs = ds_settle(c)) return rs;
  HostPhase hp("serialize");
  DsState* d = c->ds;
  ce_ctx* ctx = c->ctx;
  hipStream_t s = ctx->stream;
  hipError_t e;
  auto uuid_dots = [&](const IdDots& v) {
    Dots o;
    for (auto& x : v) o.push_back({c->id_actor[x.first], x.second});
    sort_dots(&o);
    return o;
  };
  auto put_vclock = [](Wr& w, const Dots& v) {
    w.map(1);
    w.str("dots");
    w.map(v.size());
    for (auto& x : v) { w.bin(x.first.data(), 16); w.uint(x.second); }
  };
  Dots nov;
  for (uint32_t sl = 0; sl < c->cap; sl++)
    if (c->h_table[sl].used && c->nov[sl]) nov.push_back({c->slot_actor[sl], c->nov[sl]});
  sort_dots(&nov);
  Wr w;
  w.b.swap(*out);  // reuse the caller's capacity
  w.b.clear();
  w.map(2);
  w.str("next_op_versions");
  put_vclock(w, nov);
  w.str("state");
  if (c->kind == CE_STATE_MVREG) {
    w.map(1);
    w.str("vals");
    w.arr(d->vals.size());
    for (auto& v : d->vals) {
      w.arr(2);
      put_vclock(w, uuid_dots(v.first));
      w.uint(v.second);
    }
    out->swap(w.b);
    return CE_OK;
  }
  // clock
  const uint32_t na = (uint32_t)c->id_actor.size();
  std::vector<unsigned long long> ck(na);
  if (na && ((e = hipMemcpyAsync(ck.data(), d->clock.p, na * 8ull, hipMemcpyDeviceToHost, s)) ||
             (e = stream_wait(s))))
    return ctx->hip_fail(e, "clock download");
  IdDots clock;
  for (uint32_t i = 0; i < na; i++)
    if (ck[i]) clock.push_back({i, ck[i]});
  // entries: collect live pairs, sort by member on the device
  uint32_t nl = 0;
  HostPhase hp1("ser: collect/sort/download");
  int rc = collect(c, &nl);
  if (rc) return rc;
  std::vector<unsigned long long> mem(nl), val(nl);
  std::vector<uint32_t> act(nl);
  if (nl) {
    if ((e = d->col[3].reserve(nl * 8ull)) || (e = d->col[4].reserve(nl * 4ull)) ||
        (e = d->sort_perm.reserve(nl * 4ull)) || (e = d->sort_perm2.reserve(nl * 4ull)) ||
        (e = d->ctr_sorted.reserve(nl * 8ull)))
      return ctx->hip_fail(e, "serialize");
    size_t tb = 0;
    unsigned long long* k0 = d->col[0].as<unsigned long long>();
    unsigned long long* k1 = d->col[3].as<unsigned long long>();
    uint32_t* p0 = d->sort_perm.as<uint32_t>();
    uint32_t* p1 = d->sort_perm2.as<uint32_t>();
    if ((e = ds_sort_pairs_u64(nullptr, tb, k0, k1, p0, p1, nl, s)) || (e = d->cub_tmp.reserve(tb + 256)))
      return ctx->hip_fail(e, "serialize");
    tb = d->cub_tmp.cap;
    if ((e = launch_ds_iota(s, p0, nl)) || (e = ds_sort_pairs_u64(d->cub_tmp.p, tb, k0, k1, p0, p1, nl, s)) ||
        (e = launch_ds_gather_entries(s, d->sort_perm2.as<uint32_t>(), d->col[1].as<uint32_t>(),
                                      d->col[2].as<unsigned long long>(), d->col[4].as<uint32_t>(),
                                      d->ctr_sorted.as<unsigned long long>(), nl)) ||
        (e = hipMemcpyAsync(mem.data(), d->col[3].p, nl * 8ull, hipMemcpyDeviceToHost, s)) ||
        (e = hipMemcpyAsync(act.data(), d->col[4].p, nl * 4ull, hipMemcpyDeviceToHost, s)) ||
        (e = hipMemcpyAsync(val.data(), d->ctr_sorted.p, nl * 8ull, hipMemcpyDeviceToHost, s)) ||
        (e = stream_wait(s)))
      return ctx->hip_fail(e, "serialize");
  }
  hp1.~HostPhase();
  hp1.name = "";
  HostPhase hp2("ser: host write");
  size_t n_members = 0;
  for (uint32_t i = 0; i < nl; i++) n_members += i == 0 || mem[i] != mem[i - 1];
  // actor id -> rank in UUID byte order (BTreeMap order of a VClock)
  std::vector<uint32_t> order(na), rank(na);
  for (uint32_t i = 0; i < na; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return c->id_actor[a] < c->id_actor[b]; });
  for (uint32_t i = 0; i < na; i++) rank[order[i]] = i;
  w.b.reserve(w.b.size() + 64 + (size_t)n_members * 16 + (size_t)nl * 28 + clock.size() * 28);
  w.map(3);
  w.str("clock");
  put_vclock(w, uuid_dots(clock));
  w.str("entries");
  w.map(n_members);
  // members are written in parallel: the sorted pairs are cut at member boundaries into one
  // chunk per host thread, each chunk written with raw-pointer stores into its own buffer
  // (sized for the worst case, trimmed), and the chunks appended in order
  auto write_members = [&](uint32_t i0, uint32_t i1, std::vector<uint8_t>* ob) {
    std::vector<std::pair<uint32_t, uint64_t>> g;  // (rank, counter) of one member
    ob->resize((size_t)(i1 - i0) * 47 + 64);
    uint8_t* o = ob->data();
    size_t pos = 0;
    auto put_uint = [&](uint64_t v) {
      if (v <= 0x7f) { o[pos++] = (uint8_t)v; return; }
      int k;
      if (v <= 0xff) { o[pos++] = 0xcc; k = 1; }
      else if (v <= 0xffff) { o[pos++] = 0xcd; k = 2; }
      else if (v <= 0xffffffffull) { o[pos++] = 0xce; k = 4; }
      else { o[pos++] = 0xcf; k = 8; }
      for (int b = k - 1; b >= 0; b--) o[pos++] = (uint8_t)(v >> (8 * b));
    };
    for (uint32_t i = i0; i < i1;) {
      uint32_t j = i;
      g.clear();
      while (j < i1 && mem[j] == mem[i]) { g.push_back({rank[act[j]], val[j]}); j++; }
      if (g.size() > 1) std::sort(g.begin(), g.end());
      put_uint(mem[i]);
      std::memcpy(o + pos, "\x81\xa4" "dots", 6);  // VClock {dots: ..}
      pos += 6;
      const size_t k = g.size();
      if (k <= 15) o[pos++] = (uint8_t)(0x80 | k);
      else if (k <= 0xffff) { o[pos++] = 0xde; o[pos++] = (uint8_t)(k >> 8); o[pos++] = (uint8_t)k; }
      else { o[pos++] = 0xdf; for (int b = 3; b >= 0; b--) o[pos++] = (uint8_t)(k >> (8 * b)); }
      for (auto& x : g) {
        o[pos++] = 0xc4;
        o[pos++] = 16;
        std::memcpy(o + pos, c->id_actor[order[x.first]].data(), 16);
        pos += 16;
        put_uint(x.second);
      }
      i = j;
    }
    ob->resize(pos);
  };
  const uint32_t T = nl < (1u << 16) ? 1u : std::min<uint32_t>(16, std::max(1u, std::thread::hardware_concurrency()));
  std::vector<uint32_t> cut(T + 1, nl);
  cut[0] = 0;
  for (uint32_t t = 1; t < T; t++) {
    uint32_t x = std::max<uint32_t>(cut[t - 1], (uint32_t)((uint64_t)nl * t / T));
    while (x < nl && x > 0 && mem[x] == mem[x - 1]) x++;
    cut[t] = x;
  }
  std::vector<std::vector<uint8_t>>& parts = d->ser_parts;  // reused across compactions
  if (parts.size() < T) parts.resize(T);
  if (T == 1) {
    write_members(0, nl, &parts[0]);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; t++) th.emplace_back(write_members, cut[t], cut[t + 1], &parts[t]);
    for (auto& x : th) x.join();
  }
  for (uint32_t t = 0; t < T; t++) w.b.insert(w.b.end(), parts[t].begin(), parts[t].end());
  w.str("deferred");
  std::vector<std::pair<std::vector<uint8_t>, const std::set<uint64_t>*>> df;
  for (auto& x : d->deferred) {
    Wr kw;
    put_vclock(kw, uuid_dots(x.first));
    df.push_back({kw.b, &x.second});
  }
  std::sort(df.begin(), df.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  w.map(df.size());
  for (auto& x : df) {
    w.b.insert(w.b.end(), x.first.begin(), x.first.end());
    w.arr(x.second->size());
    for (uint64_t m : *x.second) w.uint(m);
  }
  out->swap(w.b);
  return CE_OK;
}

}  // namespace ce
