// ce_dotset.h -- launch interface of the dot-set fold kernels (ce_dotset.hip): decode of
// Vec<orswot::Op> / Vec<mvreg::Op> op files into columnar arrays, and the data-parallel
// Orswot / MVReg fold (the formulation is stated, and checked against the sequential oracle, in
// tests/dotset_model.py).
//
// HBM layout (all arrays device-resident, one set per Core):
//   actors        stable actor id (ActorSlot.pad[0]) indexes every dense per-actor array
//   clock         u64[n_actors]          Orswot.clock (VClock::dots by id)
//   member table  u64 mkey[ms + pcap + 1] open addressing on the u64 member: a primary table of ms
//                                        slots (L2-sized, grown with the members present), an
//                                        overflow table of pcap slots for members whose primary
//                                        window is full, the last slot reserved for the member ~0
//                                        (the empty-key sentinel); the slot index is the handle
//   pair table    u64 pkey[pcap]         (member handle << 24 | actor id), EMPTY = ~0
//                 u64 cur/add/kill/oth[pcap]  entry value (Orswot.entries[m][a]), the batch's
//                                        applied-add max, removal threshold, merged state's value
//   ops (CSR)     adds: actor u32, counter u64, mbeg u32 -> add members u64
//                 removals / puts: cbeg u32 -> clock (actor u32, counter u64), mbeg u32 ->
//                 members u64 (removals), val u64 (puts)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ce_common.h"
#include "ce_kernels.h"

namespace ce {

static constexpr unsigned long long kDsEmpty = ~0ull;
static constexpr uint32_t kDsNoActor = 0xffffffffu;
static constexpr int32_t kStatusHostDecode = 101;  // op vector the device leaves to the host
static constexpr int kDsActorBits = 24;            // actor ids < 2^24 in a pair key
static constexpr int kDsPartBits = 11;             // pair-table partition: 2048 slots (k_ds_part_apply)
static constexpr uint32_t kDsPartSlots = 1u << kDsPartBits;

enum DsKind { kDsOrswot = 0, kDsMVReg = 1 };

// per-file counts (count pass) / bases (after the exclusive scan), 5 arrays of n
enum { kCntAdd = 0, kCntAddM = 1, kCntRm = 2, kCntRmC = 3, kCntRmM = 4, kCntN = 5 };

struct DsOps {
  uint32_t* add_actor;
  unsigned long long* add_ctr;
  uint32_t* add_mbeg;          // [n_add + 1]
  unsigned long long* add_mem;
  uint32_t* rm_cbeg;           // [n_rm + 1]  (MVReg: puts)
  uint32_t* rm_mbeg;           // [n_rm + 1]
  uint32_t* rmc_actor;
  unsigned long long* rmc_ctr;
  unsigned long long* rm_mem;
  unsigned long long* put_val; // MVReg
};

// The tiled emit (Orswot): file-minor scratch rows per op column (column c = add_actor,
// add_ctr, add_mbeg, add_mem, rm_cbeg, rm_mbeg, rmc_actor, rmc_ctr, rm_mem), entry k of file i at
// col[c][k * npad + i]; npad = 0 disables it.  total[g] = the count column totals (the last
// file's end).  Every per-file count must be <= kTileMaxRows.
static constexpr uint32_t kTileMaxRows = 96;
struct DsTile {
  void* col[9];
  uint64_t npad;
  uint32_t total[5];
  uint32_t max_rows;  // the largest per-file count of any column group (<= kTileMaxRows): LDS rows
};

struct DsDecodeArgs {
  int kind;                     // DsKind
  const uint8_t* pt;            // plaintext blob (FileParams.out_off / len)
  const FileParams* params;
  int32_t* status;
  uint32_t n;
  const uint8_t* supported;     // n_supported * 16 bytes
  uint32_t n_supported;
  const uint8_t* apply;         // version gate: 1 = fold this file
  uint32_t* cnt;                // [kCntN][n] counts (count pass) / bases (emit pass)
  uint32_t base_off[kCntN];     // emit: added to every base (MVReg: current values first)
  const ActorSlot* table;
  uint32_t mask;
  DsOps ops;
  uint32_t* counters;           // [0] decode failures, [1] host-decode files, [2] misses,
                                // [3] adds not run-contiguous, [8 + k] largest count of column k
  uint4* miss_list;
  uint32_t miss_cap;
  DsTile tile;                  // emit: the tiled layout (npad 0: direct CSR stores)
  // Orswot files the open already decoded (k_open_fold_v2's DS form): done[i] = 1 -> the count
  // pass takes fuse.rawcnt, the emit skips the file, k_ds_untile reads its file-major rows
  // (fuse.*) and writes the offsets columns as op index + base.  null: none.
  const uint8_t* fdone;
  DsFuse fuse;
  // count pass: per block [8 words]: the largest count of each column and the files the open
  // decoded, reduced by k_ds_col_totals (same-address atomics from every block serialised across
  // the XCDs, ~60 ns each).  null: the atomics into counters[5] / counters[8 + k]
  uint32_t* bpart;
};
// k_ds_count's grid for n files (its bpart rows: kDsCountPart words each -- [0, 5) column
// maxima, [5] files the open decoded, [8] files not OK, [9] left to the host envelope parser,
// [10] left to the host op decoder, [11] the first not OK)
uint32_t ds_count_blocks(uint32_t n);
static constexpr uint32_t kDsCountPart = 16;
hipError_t launch_ds_count(hipStream_t s, const DsDecodeArgs& a);
hipError_t launch_ds_emit(hipStream_t s, const DsDecodeArgs& a, bool emit_legacy = true);

struct DsTables {
  unsigned long long* mkey;      // [smask + 1] primary, [mmask + 1] overflow, 1 reserved (member ~0)
  uint32_t smask;               // primary slots - 1 (power of two, sized for the members present)
  uint32_t mmask;               // overflow slots - 1 (= pmask: members <= pairs)
  unsigned long long* pkey;
  unsigned long long* cur;
  unsigned long long* add;
  unsigned long long* kill;
  unsigned long long* oth;
  uint32_t pmask;
  uint32_t* live;               // [0] live pairs after finalize, [1] used pairs, [2] probe overflow,
                                // [3] a removal deferred, [4] used primary member slots (part fold, k-way merge)
};

// applied flags of the adds: keys = add_actor sorted stably, perm = add index per position
hipError_t launch_ds_iota(hipStream_t s, uint32_t* v, uint32_t n);
hipError_t launch_ds_gather_ctr(hipStream_t s, const uint32_t* perm, const unsigned long long* ctr,
                                unsigned long long* out, uint32_t n);
hipError_t launch_ds_applied(hipStream_t s, const uint32_t* keys_sorted, const uint32_t* perm,
                             const unsigned long long* ctr_sorted,
                             const unsigned long long* excl_max, const unsigned long long* clock,
                             uint8_t* applied, uint32_t n);
// flag |= 1 unless every actor's adds are one contiguous run (marks: u32[n_marks] holding older
// generations only; gen = a fresh nonzero value per check)
// the contiguity check's optional second job (k_ds_contig): applied flags and exclusive maxima of
// strictly increasing runs (ctr null: off)
struct DsMono {
  const unsigned long long* ctr;
  const unsigned long long* clock;
  uint32_t ccap;
  uint8_t* applied;
  unsigned long long* excl;
};
hipError_t launch_ds_contig(hipStream_t s, const uint32_t* actor, uint32_t n, uint32_t* marks, uint32_t n_marks,
                            uint32_t gen, uint32_t* flag, const uint32_t* miss_src = nullptr, uint32_t* pub = nullptr,
                            DsMono mono = DsMono{});
// clock[a] = max(clock[a], counter) for every add
hipError_t launch_ds_clock(hipStream_t s, const uint32_t* keys_sorted, const unsigned long long* ctr_sorted,
                           const unsigned long long* excl_max, unsigned long long* clock, uint32_t n_add);
// insert (member, actor) of every applied add, add[pair] = max counter
hipError_t launch_ds_add_pairs(hipStream_t s, DsTables t, DsOps o, const uint8_t* applied,
                               uint32_t n_add);
// removal thresholds: kill[(m, a)] = max R[a] over removals listing m (existing pairs only)
hipError_t launch_ds_kill(hipStream_t s, DsTables t, const uint32_t* cbeg, const uint32_t* mbeg,
                          const uint32_t* c_actor, const unsigned long long* c_ctr,
                          const unsigned long long* mem, uint32_t n_rm);
// v = max(cur, add); v <= kill -> 0; cur = v; add = kill = 0; live/used counts
hipError_t launch_ds_finalize(hipStream_t s, DsTables t);

// The partitioned fold (adds + removals + finalize of one Orswot batch; the global kernels above
// remain for batches outside its limits).  Every (pair key, value) item goes to its pair-table
// partition's run, then one workgroup per partition loads the partition's keys into LDS, inserts
// the adds / max-merges their counters and the removal thresholds there, and writes back only the
// slots that changed:
//   launch_ds_part_count   K1: adds (member insert, pair key per add member), then removals
//                          (member lookup) -- two launches, so a removal's lookup sees every member
//                          the batch's adds inserted.  Each block counts its items per partition in
//                          LDS, reserves its share of every partition's run with one returning add
//                          per partition on pcnt (contiguous counters: 256 B per wave instruction),
//                          and writes its items there: no histogram, scan or scatter pass
//   launch_ds_part_apply   K4 one workgroup per partition over its runs
// A partition's run holds cap items (the batch's expected share x the host's factor); the items of
// a block whose reservation passes it go to the overflow list, which every apply workgroup then
// filters for its partition (correct at any skew; the host widens the runs after one).  pcnt is
// zeroed by the apply that reads it; ovf_n by parity (the apply of fold g zeroes fold g + 1's).
// live[0] += change of the live-pair count (two's complement), live[1] += pairs inserted, live[5]
// = items that overflowed; K1 zeroes live[0], live[1], live[3] and live[4].
#ifndef CE_PART_BATCH
#define CE_PART_BATCH 4  // K1 items per lane whose loads are issued before any is used (same box
                         // at C3: 8 -> 4 k_ds_part_adds 62.7 -> 49.7 us, more lanes in flight; 2: 48.8
                         // but the rest of the fold slower)
#endif
static constexpr uint32_t kDsPartChunk = 1024 * CE_PART_BATCH;  // adds / removals per 1024-thread K1 block
static constexpr uint32_t kDsPartThreadsSmall = 512;  // the half-size K1 blocks (CE_DS_PART_SMALL)
static constexpr uint32_t kDsPartChunkSmall = 512 * CE_PART_BATCH;
static constexpr uint32_t kDsPartReps = 8;          // sub-runs per partition and side (K1 block % 8)
static constexpr uint32_t kDsPartMaxParts = 16384;  // LDS histogram bound (64 KB)
struct DsKillSrc {
  const uint32_t* cbeg;
  const uint32_t* mbeg;
  const uint32_t* c_actor;
  const unsigned long long* c_ctr;
  const unsigned long long* mem;
  unsigned long long* hk;       // K1: member handle per removal member of a removal with several items
  uint32_t n;
};
struct DsPartArgs {
  DsTables t;
  DsOps o;
  const uint8_t* applied;
  uint32_t n_add;
  unsigned long long* akey;     // K1: pair key per member of an add with several members
  DsKillSrc ks[2];              // the batch's removals, the deferred set
  uint32_t ba, bk0, bk;         // add blocks, blocks of ks[0], all removal blocks
  uint32_t parts;               // (pmask + 1) >> kDsPartBits
  uint32_t chunk;               // adds per K1 block (kDsPartChunk)
  uint32_t kchunk;              // removals per K1 block (fewer items: smaller blocks' worth)
  uint32_t cap[2];              // sub-run length: adds, removals
  uint32_t* pcnt;               // [2][kDsPartReps][parts]: items reserved per sub-run (adds, removals)
  unsigned long long* items;    // (key, value) pairs: [parts][kDsPartReps][cap[0]] adds, then the removals
  unsigned long long* ovf[2];   // overflow lists (key, value): adds, removals
  uint32_t ovf_cap[2];
  uint32_t* ovf_n;              // [4]: [2 par + 0 / 1] overflow counts of adds / removals
  uint32_t par;                 // this fold's parity
};
hipError_t launch_ds_part_count(hipStream_t s, const DsPartArgs& a);
// out[0] += members held (primary + overflow); out zeroed beforehand
hipError_t launch_ds_count_members(hipStream_t s, DsTables t, uint32_t* out);
hipError_t launch_ds_part_apply(hipStream_t s, const DsPartArgs& a);
// deferred[r] = !(R <= clock)
// deferred[r] = removal r's clock is not covered by `clock`; any (may be null): set to 1 when
// some removal is deferred
hipError_t launch_ds_deferred(hipStream_t s, const uint32_t* cbeg, const uint32_t* c_actor,
                              const unsigned long long* c_ctr, const unsigned long long* clock,
                              uint8_t* deferred, uint32_t n_rm, uint32_t* any = nullptr,
                              const uint32_t* pub_src = nullptr, uint32_t* pub_dst = nullptr, uint32_t pub_words = 0);
// (pub_dst: the grid's last block copies pub_src[0..pub_words) -- the fold's live counters, pub_src
// = DsTables.live, live[7] counting the blocks -- into the caller's pinned memory)
// state merge: insert the other state's entries with oth = value, then the per-pair merge rule
hipError_t launch_ds_put_other(hipStream_t s, DsTables t, const unsigned long long* member,
                               const uint32_t* actor, const unsigned long long* value, uint32_t n,
                               bool zero_counts = false);
hipError_t launch_ds_merge(hipStream_t s, DsTables t, const unsigned long long* clock,
                           const unsigned long long* oclock);
// k_ds_merge + k_ds_finalize in one pass (counts into live[0..1], zeroed by put_other with
// zero_counts)
// one state file's entry columns (member, actor id, value) for the k-way merge
struct DsMergeSrc {
  const unsigned long long* member;
  const uint32_t* actor;
  const unsigned long long* value;
  uint32_t n;
  uint32_t* slot;  // optional, n words: k_ds_kput records each pair's slot for k_ds_khold
  const uint32_t* n_dev;  // optional: the pair count is n_dev[1] + n_dev[2] (the reader's device
                          // tail words), n only sizes the grid
};
// Orswot::merge of nf state files at once (no deferred removals on any side): d_src / h_src the
// same descriptors in HBM and on the host, oclocks = the files' dense clocks actor-major
// (oclocks[a * ostride + f], ostride = ds_oclock_stride(nf), the padding zero),
// hold = a zeroed u64 per pair slot (left zeroed); live[0..1] = live / used pairs after
hipError_t launch_ds_kmerge(hipStream_t s, DsTables t, const DsMergeSrc* d_src, const DsMergeSrc* h_src, uint32_t nf,
                            unsigned long long* clock, const unsigned long long* oclocks, uint32_t ccap, uint32_t ostride,
                            unsigned long long* hold, uint32_t* pub_dst = nullptr,  // pub_dst: live[0..5) -> pinned
                            const uint32_t* go = nullptr,  // go: every kernel does nothing unless *go
                            bool fresh = false);  // the table holds no pair: the current values are not read
// one column partial of the multi-GPU exchange (ds_merge_columns_device): its actor column and
// clock remapped to the receiving core's ids
struct DsColsRemap {
  const uint32_t* actor;          // np partial-local actor indices
  uint32_t* ids;                  // np receiver ids (out)
  const uint32_t* map;            // na: partial-local index -> receiver id (device)
  const unsigned long long* clock;  // na: the partial's clock by its indices
  unsigned long long* oclock;     // dense by receiver id at stride ostride (zeroed; out)
  uint32_t np, na, ostride;
};
// the actor-major stride of nf files' dense clocks (launch_ds_kmerge): a multiple of 8, >= nf
inline uint32_t ds_oclock_stride(uint32_t nf) { return nf <= 8 ? 8u : (nf + 7u) & ~7u; }
static constexpr uint32_t kColsInline = 16;
struct DsColsRemaps {
  DsColsRemap f[kColsInline];
};
hipError_t launch_cols_remap(hipStream_t s, const DsColsRemap* parts, uint32_t k);
// a column partial's deferred CSR section checked in place (offsets ordered and in range, actor
// indices < na): *bad (zeroed beforehand) = 1 when it is not
hipError_t launch_ds_csr_check(hipStream_t s, const uint32_t* cbeg, const uint32_t* mbeg, const uint32_t* act,
                               uint32_t n_rm, uint32_t n_ent, uint32_t n_mem, uint32_t na, uint32_t* bad);
hipError_t launch_ds_merge_finalize(hipStream_t s, DsTables t, const unsigned long long* clock,
                                   const unsigned long long* oclock);
// live pairs -> (member, actor, value) columns (any order); n_out[0] (zeroed beforehand) = their
// count, n_out[2..3] = the largest member; bmax: kCollectBlocks words of scratch
static constexpr uint32_t kCollectBlocks = 2048;
hipError_t launch_ds_collect(hipStream_t s, DsTables t, unsigned long long* member, uint32_t* actor,
                             unsigned long long* value, uint32_t* n_out, unsigned long long* bmax, uint32_t* host_out,
                             unsigned long long* extra_dst = nullptr, const unsigned long long* extra_src = nullptr,
                             uint32_t extra_words = 0);
// rebuild: insert (member, actor, value) into fresh (cleared) tables as cur
hipError_t launch_ds_reinsert(hipStream_t s, DsTables t, const unsigned long long* member,
                              const uint32_t* actor, const unsigned long long* value, uint32_t n);
hipError_t launch_ds_gather_entries(hipStream_t s, const uint32_t* perm, const uint32_t* actor_in,
                                    const unsigned long long* value_in, uint32_t* actor_out,
                                    unsigned long long* value_out, uint32_t n);

// device-wide primitives (sorts: hipCUB; scans: ce_scan.hip): tmp = nullptr queries the temp
// size into tb
hipError_t ds_sort_pairs_u32(void* tmp, size_t& tb, const uint32_t* kin, uint32_t* kout,
                             const uint32_t* vin, uint32_t* vout, uint32_t n, int bits, hipStream_t s);
hipError_t ds_sort_pairs_u64(void* tmp, size_t& tb, const unsigned long long* kin,
                             unsigned long long* kout, const uint32_t* vin, uint32_t* vout,
                             uint32_t n, hipStream_t s);
// out[i] = max(vals[j] : j < i, keys[j] == keys[i]) (0 for a segment's first element)
hipError_t ds_excl_max_by_key(void* tmp, size_t& tb, const uint32_t* keys,
                              const unsigned long long* vals, unsigned long long* out, uint32_t n,
                              hipStream_t s);
hipError_t ds_excl_sum_u32(void* tmp, size_t& tb, const uint32_t* in, uint32_t* out, uint32_t n,
                           hipStream_t s);
// totals of the kCntN columns of one back-to-back exclusive scan (out[kCntN], device)
// out (19 words): column totals [0..kCntN), column maxima [8..8+kCntN), status summary [13..17),
// the gate's two flags [17..19) (gate_flags may be null); then clear8[0..8) = 0 (may be null)
hipError_t launch_ds_col_totals(hipStream_t s, const uint32_t* cnt, const uint32_t* bases, uint32_t n,
                                const uint32_t* maxima, const uint32_t* bpart, uint32_t nb,
                                const int32_t* status, const uint32_t* gate_flags,
                                uint32_t* clear8, uint32_t* out, const unsigned long long* nn_src = nullptr,
                                uint32_t nn_m = 0, unsigned long long* nn_dst = nullptr);
hipError_t launch_ds_set3(hipStream_t s, uint32_t* p0, uint32_t v0, uint32_t* p1, uint32_t v1, uint32_t* p2,
                          uint32_t v2);

// MVReg survivors: candidates = CSR clocks (cbeg, actor, ctr) with priorities (index order)
struct MvArgs {
  const uint32_t* cbeg;
  const uint32_t* c_actor;
  const unsigned long long* c_ctr;
  uint32_t n;
  int later_wins;                 // ties (equal clocks): 1 = highest index wins, 0 = lowest
  uint8_t* alive;
  unsigned long long* sum_hi;     // 128-bit counter sums
  unsigned long long* sum_lo;
  unsigned long long* blk;        // per-block best: 4 words (hi, lo, prio, idx)
  uint32_t n_blk;
  uint32_t* win;                  // [0] winner index or ~0, [1] alive count
  unsigned long long* wclock;     // dense winner clock by actor id (kept zero between rounds)
};
hipError_t launch_mv_prep(hipStream_t s, const MvArgs& a);
hipError_t launch_mv_round(hipStream_t s, const MvArgs& a);  // argmax + scatter + kill + clear

}  // namespace ce
