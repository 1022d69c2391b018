// ce_core.h -- the Core object (crdt-enc/src/lib.rs:188-207 Core / CoreMutData) and the host
// helpers shared by ce_core.cpp (VClock / GCounter state) and ce_dotset_host.cpp (Orswot / MVReg).
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "ce_internal.h"

namespace ce {
int storage_load_ops_vec(ce_storage* s, const std::vector<Uuid>& actors,
                         const std::vector<uint64_t>& first, std::vector<uint8_t>* blob,
                         std::vector<uint64_t>* offs, std::vector<uint32_t>* aidx,
                         std::vector<uint64_t>* vers);
int storage_list_op_actors_vec(ce_storage* s, std::vector<Uuid>* out);
int storage_list_states_vec(ce_storage* s, std::vector<std::string>* out);
int storage_read_state(ce_storage* s, const std::string& name, std::vector<uint8_t>* out);
int storage_store_content(ce_storage* s, const char* sub, const uint8_t* d, size_t n,
                          std::string* name);
int storage_remove_state(ce_storage* s, const std::string& name);
int storage_store_op(ce_storage* s, const Uuid& actor, uint64_t version, const uint8_t* d,
                     size_t n);
int storage_remove_op(ce_storage* s, const Uuid& actor, uint64_t version);
int storage_load_local_meta(ce_storage* s, std::vector<uint8_t>* out, bool* missing);
int storage_store_local_meta(ce_storage* s, const uint8_t* d, size_t n);
ce_storage* storage_new(const std::string& local, const std::string& remote);

struct DsState;  // Orswot / MVReg state (ce_dotset_host.cpp)
void ds_free(DsState* d);

inline bool is_dotset_kind(int kind) { return kind == CE_STATE_ORSWOT || kind == CE_STATE_MVREG; }
}  // namespace ce

namespace ce {
struct AltKey {  // a key of the set besides the latest (ce_core_set_keys, CE_OPEN_MULTI_KEY)
  uint8_t version[16];
  std::vector<uint8_t> key;
};
}  // namespace ce

struct ce_core {
  ce_ctx* ctx = nullptr;
  int kind = CE_STATE_GCOUNTER;
  std::vector<ce::Uuid> supported;  // sorted (lib.rs:227-228)
  ce::Uuid current_data_version{};
  ce_storage* storage = nullptr;
  uint32_t flags = 0;
  ce::Uuid local_actor{};
  bool has_key = false;
  uint8_t key_version[16] = {0};
  std::vector<uint8_t> key;
  std::vector<ce::AltKey> alt_keys;  // tried in id order on AUTH failures (CE_OPEN_MULTI_KEY)
  std::map<std::string, uint64_t> path_counts;  // which code path ran (ce_core_path_count)
  // actor table: UUID -> hash slot; ActorSlot.pad[0] holds the actor's stable id (insertion
  // order, survives table growth) used by the dot-set kinds' device arrays.
  uint32_t cap = 0, size = 0, registered = 0;
  std::vector<ce::ActorSlot> h_table;
  std::vector<ce::Uuid> slot_actor;
  std::vector<ce::Uuid> id_actor;   // stable id -> UUID
  std::vector<uint64_t> nov;  // next_op_versions by slot
  std::unordered_map<ce::Uuid, uint32_t, ce::UuidHash> slot_of;
  bool table_dirty = true;
  uint64_t table_gen = 0;               // bumped whenever an actor gets a slot or slots move
  std::vector<uint8_t> ser_buf, file_buf;  // compaction: serialized state, sealed file (reused)
  // compact_into: the caller's buffer; a compaction that fits writes the file there directly
  // (sink_len = its length) instead of into file_buf
  uint8_t* sink = nullptr;
  size_t sink_cap = 0, sink_len = 0;
  // ce_core_compact_into_async: the sealed file's download into the sink is left in flight on
  // copy_stream (ticket -> copy_ev[ticket % kAsyncSlots]); the next compaction's seal waits for
  // the last one on the device before it rewrites the sealed output
  static constexpr uint32_t kAsyncSlots = 16;
  bool sink_async = false;
  uint64_t sink_ticket = 0;               // set by the device writer when it left a copy in flight
  hipStream_t copy_stream = nullptr;
  hipEvent_t copy_ev[kAsyncSlots] = {};
  uint64_t copy_slot_ticket[kAsyncSlots] = {};
  uint64_t copy_next = 0;                 // last ticket handed out
  // pinned, mapped: per slot, the sealed file's length the device wrote behind the seal
  // (ce_core_compact_wait); the download itself is enqueued by ds_async_kick once the seal is
  // done (the runtime's DMA copy needs the exact length on the host), at most one pending
  ce::HostBuf copy_len;
  uint64_t* copy_len_dev = nullptr;
  hipEvent_t seal_ev = nullptr;
  // the download on an SDMA engine when the HSA runtime offers one (copy_sig per slot), else the
  // HIP runtime's copy on copy_stream (copy_ev); copy_last_slot: the newest download's slot
  ce::DmaD2H dma;
  bool dma_tried = false;
  hsa_signal_t copy_sig[kAsyncSlots] = {};
  bool copy_dma[kAsyncSlots] = {};
  int copy_last_slot = -1;
  bool pend = false;
  uint32_t pend_slot = 0;
  uint8_t* pend_dst = nullptr;
  std::vector<uint32_t> sorted_slots;   // used slots in UUID byte order (BTreeMap order)
  uint64_t sorted_gen = ~0ull;
  std::vector<uint8_t> last_writers;    // writer list of the previous ingest and its slots
  std::vector<uint32_t> last_wslot;
  uint64_t last_writers_gen = ~0ull;
  ce::DevBuf d_table, d_state, d_batch, d_supported, d_refold2, d_tmp, d_gate, d_meta;
  ce::DevBuf d_sorted, d_wslot;                  // sorted_slots on the device (compaction serializer)
  uint64_t d_sorted_gen = ~0ull;
  int files_per_wave = 4;  // fused kernel geometry (CE_FILES_PER_WAVE overrides)
  bool supported_on_device = false;
  bool host_compact = false;  // CE_HOST_COMPACT=1: serialize on the host (reference check)
  int fused = 2;           // fused kernel: 1 keystream staged in LDS, 2 block-owning lanes (CE_FUSED)
  std::set<std::string> read_states;  // lib.rs:205
  ce_ctx* aux = nullptr;              // single-file work during a batch (exotic envelopes)
  ce::DsState* ds = nullptr;          // Orswot / MVReg state (dot-set kinds only)
  // sharded ingest (ce_core_ingest_ops_device_sharded): the batch is folded into d_batch and
  // held there with its next_op_versions until ce_core_pending_commit
  bool pending = false;
  uint64_t pending_gen = 0;                                  // table_gen of the pending batch
  std::vector<std::pair<ce::Uuid, uint64_t>> pending_nov;    // (writer, next_op_version)
  ce::DevBuf d_shard;                  // writer UUIDs | e0 | stats scratch (ce_core_shard_*)
  ce::HostBuf h_shard;                 // pinned staging of the e0 upload (its own: the copy is async)
  std::vector<uint64_t> shard_e0;      // the e0 d_shard holds
  std::vector<uint8_t> shard_writers;  // the writer list d_shard holds
};

namespace ce {

// msgpack writer (rmp-serde to_vec_named)
struct Wr {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void be(uint64_t v, int k) {
    for (int j = k - 1; j >= 0; j--) b.push_back((uint8_t)(v >> (8 * j)));
  }
  void uint(uint64_t v) {
    if (v <= 0x7f) u8((uint8_t)v);
    else if (v <= 0xff) { u8(0xcc); be(v, 1); }
    else if (v <= 0xffff) { u8(0xcd); be(v, 2); }
    else if (v <= 0xffffffffull) { u8(0xce); be(v, 4); }
    else { u8(0xcf); be(v, 8); }
  }
  void str(const char* s) {
    const size_t l = std::strlen(s);
    u8((uint8_t)(0xa0 | l));
    b.insert(b.end(), s, s + l);
  }
  void bin(const uint8_t* d, size_t l) {
    if (l <= 0xff) { u8(0xc4); be(l, 1); }
    else if (l <= 0xffff) { u8(0xc5); be(l, 2); }
    else { u8(0xc6); be(l, 4); }
    b.insert(b.end(), d, d + l);
  }
  void map(size_t n) {
    if (n <= 15) u8((uint8_t)(0x80 | n));
    else if (n <= 0xffff) { u8(0xde); be(n, 2); }
    else { u8(0xdf); be(n, 4); }
  }
  void arr(size_t n) {
    if (n <= 15) u8((uint8_t)(0x90 | n));
    else if (n <= 0xffff) { u8(0xdc); be(n, 2); }
    else { u8(0xdd); be(n, 4); }
  }
};

using Dots = std::vector<std::pair<Uuid, uint64_t>>;

// CE_HOST_PROF=1: wall time of host phases to stderr (diagnostics only)
struct HostPhase {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit HostPhase(const char* n) : name(n) {}
  ~HostPhase() {
    static const bool on = std::getenv("CE_HOST_PROF") != nullptr;
    if (!on || !name || !*name) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "CE_HOST_PROF %-24s %9.3f ms\n", name, ms);
  }
};

// next_op_versions of an ingest whose device commit is still in flight (compact_enqueue)
struct NovApply {
  const uint32_t* wslot;                 // device: slot of each writer
  const unsigned long long* newnov;      // device: the gate's next_op_versions per writer
  uint32_t m;
  const uint32_t* counters;              // device: the ingest's counter block
  unsigned long long* nov_dev = nullptr; // device: the pre-ingest next_op_versions (cap words),
                                         // uploaded with the gate block; the compaction applies
                                         // newnov to it in place
  const uint8_t* host_tail = nullptr;    // out (set by the compaction): pinned host copy of
                                         // [clear length | the counters | newnov[m]] after sync
  // the ingest's commit (k_merge_max_if: state = max(state, batch) over merge_n words), left to
  // the compaction's first kernel when set: one launch and one dependency gap fewer
  unsigned long long* merge_dst = nullptr;
  const unsigned long long* merge_src = nullptr;
  uint32_t merge_n = 0;
};

bool skip_any(Rd& r, int depth = 0);
bool bytes_any(Rd& r, std::vector<uint8_t>* out);
bool read_struct(Rd& r, const std::vector<const char*>& names,
                 const std::function<bool(int, Rd&)>& cb);
bool read_vclock(Rd& r, Dots* out);
int insert_actor(ce_core* c, const Uuid& u, uint32_t* slot);
// slots of m actors (16 bytes each) after a table growth moved the ones handed out before it
void refresh_slots(ce_core* c, const uint8_t* actors, uint32_t m, std::vector<uint32_t>* slots);
inline uint32_t actor_id_of_slot(const ce_core* c, uint32_t slot) { return c->h_table[slot].pad[0]; }
int table_upload(ce_core* c);
KeyRef key_of(ce_core* c);
int ensure_supported(ce_core* c);
int resolve_host_parse(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                       bool outer);
uint32_t host_gate(const uint32_t* fa, const uint64_t* fv, uint32_t n, std::vector<uint64_t>* expect,
                   uint8_t* apply);
int merge_dots_host(ce_core* c, const Dots& dots);
// read_remote_ops over a batch resident in HBM (ce_core.cpp).  shard_hi (device, m + 1 words):
// the sharded gate's windows and flags (ce_shard.hip) instead of the local gate; the batch is
// then left pending (not committed) for ce_core_pending_commit.
int ingest_ops_dev_sharded(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                           uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                           const uint64_t* d_fv, const uint64_t* shard_hi, int32_t* status_out);

// dot-set kinds (ce_dotset_host.cpp): same contracts as the VClock/GCounter paths in ce_core.cpp
int ds_init(ce_core* c);
int ds_reset(ce_core* c);
int ds_ingest_ops(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                  uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                  const uint64_t* d_fv, int32_t* status_out);
// read_remote_states after load_states; plaintext StateWrappers (after the data version)
// sws[i] = {nullptr, 0} for files whose status st[i] is already a failure.
int ds_compact_device(ce_core* c, ce_ctx* x, const uint8_t* outer, const uint8_t* prefix16,
                      const uint8_t* nonce, const KeyRef& key, std::vector<uint8_t>* file);
int ds_merge_states_device(ce_core* c, const uint8_t* out, const std::vector<uint64_t>& off,
                           const std::vector<uint64_t>& len, int32_t* st, int32_t* status_out);
int ds_merge_states(ce_core* c, const std::vector<std::pair<const uint8_t*, size_t>>& sws,
                    int32_t* st, int32_t* status_out);
int ds_serialize(ce_core* c, std::vector<uint8_t>* out);
// Orswot: the same bytes written on the device into dst (cap bytes); *len = their length
// compact_into_async: enqueue the pending download once its seal is done (force: wait for it)
int ds_async_kick(ce_core* c, bool force);
// the newest compaction download done reading seal_out (host wait, or ordered on s)
int ds_download_fence(ce_core* c, hipStream_t s, bool device);
// the last fold's / k-way merge's closing counts and deferred set (waits for the stream)
int ds_settle(ce_core* c);
int ds_state_bytes_device(ce_core* c, ce_ctx* x, uint8_t* dst, uint64_t cap, uint64_t* len);
int ds_export_columns_device(ce_core* c, uint8_t* dst, uint64_t cap, uint64_t* len);
int ds_merge_columns_device(ce_core* c, const uint8_t* const* parts, const uint64_t* lens, uint32_t k);
// Core::apply_ops for a local Vec<S::Op> (already validated by ds_check_ops)
int ds_check_ops(ce_core* c, const uint8_t* ops, size_t len);
int ds_apply_local_ops(ce_core* c, const uint8_t* ops, size_t len);

}  // namespace ce
