// ce_dotset_io.h -- launch interface of ce_dotset_io.hip: StateWrapper<Orswot<u64, Uuid>> bytes
// written from / read into the device entry columns.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ce_common.h"
#include "ce_kernels.h"

namespace ce {

// writer: out = prefix || map header(n_members) || entries || suffix (prefix = the host-built
// bytes up to and including the "entries" key; suffix = "deferred" and its map)
struct OrswotSerArgs {
  uint8_t* out;
  const uint8_t* prefix;
  uint64_t prefix_len;
  const uint8_t* suffix;
  uint64_t suffix_len;
  const uint8_t* uuid_of_id;       // 16 bytes per stable actor id
  uint32_t n;                      // live pairs
  unsigned long long* seal_offs;   // [0] = 0, [1] = clear length, [2] = 0 (the seal's out_offs)
  uint32_t* stats;                 // [0] = members written
  // filled by launch_orswot_ser (sorted columns and scans)
  const unsigned long long* member;
  const uint32_t* actor;
  const unsigned long long* value;
  const uint32_t* head;
  const uint32_t* hrank;
  const uint32_t* seg;
  const uint32_t* pos;
  const uint32_t* len;
};

struct OrswotSerScratch {
  const unsigned long long* member_in;   // collect order
  const uint32_t* actor_in;
  const unsigned long long* value_in;
  const uint32_t* rank_of_id;            // UUID byte order rank of each stable actor id
  const uint32_t* id_of_rank;            // its inverse
  int rank_bits;
  int member_bits;                       // significant bits of the largest member (<= 64)
  uint32_t *k32a, *k32b, *p32a, *p32b;   // n each
  unsigned long long *k64a, *member_sorted, *value_sorted;
  uint32_t* actor_sorted;
  uint32_t *head, *hrank, *len, *pos;    // n each
  uint32_t* seg;                         // n + 1
  void* tmp;
  size_t tmp_bytes;
  // the radix sort (launch_ser_sort): its state words and parity, and the ping-pong key / value
  // buffers of its passes (n each; k64b / v64a / v64b u64)
  uint32_t* sort_state;
  uint32_t* sort_gen;                    // sorts so far (host): the state's histogram parity
  unsigned long long *k64b, *v64a, *v64b;
};

// the serializer's LSD radix sort (ce_ser_sort.hip): pairs (member_in, actor_in, value_in) in
// collect order -> member_out / actor_out / value_out ordered by key = member << rank_bits | rank
// (key_bits <= 64).  State (u32 words, zero before the first sort; the sorts keep it so):
// hist [2][8 replicas][kSortMaxPlaces][256] | ticket [kSortMaxPlaces] | pad, then from word
// kSortStateHead: look [places][tiles][256]
static constexpr uint32_t kSortMaxPlaces = 8;
static constexpr uint32_t kSortStateHead = 2 * 8 * kSortMaxPlaces * 256 + 64;
struct SerSortArgs {
  const unsigned long long* member_in;
  const uint32_t* actor_in;
  const unsigned long long* value_in;
  const uint32_t* rank_of_id;
  const uint32_t* id_of_rank;
  int rank_bits, key_bits;
  uint32_t n, tiles, places, par;
  uint32_t ticketed;  // tiles ordered by an atomic ticket (when they do not all fit on the GPU at
                      // once), else by blockIdx
  uint32_t *hist, *ticket, *look;
  const void* keys_in;
  void* keys_out;
  const unsigned long long* vals_in;
  unsigned long long* vals_out;
  unsigned long long* member_out;
  uint32_t* actor_out;
  unsigned long long* value_out;
  // generic (sort_pairs_*): the first pass reads keys gk_in / u32 values gv_in, the last writes
  // gk_out / gv_out (the serializer's key build and column unpack are off)
  int generic;
  const void* gk_in;
  void* gk_out;
  const uint32_t* gv_in;
  uint32_t* gv_out;
};
uint32_t ser_sort_tiles(uint32_t n);
inline size_t ser_sort_state_words(uint32_t n) {
  return kSortStateHead + (size_t)kSortMaxPlaces * ser_sort_tiles(n) * 256;
}
// kbuf: two key buffers of n (u32 when key_bits <= 32, else u64), vbuf: two u64 buffers of n
hipError_t launch_ser_sort(hipStream_t s, const SerSortArgs& a, void* const kbuf[2], unsigned long long* const vbuf[2]);
// Stable LSD radix sort of (key, u32 value) pairs over the key's low `bits` bits (the same
// kernels as the serializer's sort; hipCUB's DeviceRadixSort::SortPairs interface: tmp == null ->
// *tb = the scratch bytes needed).  kin / vin are not modified; kout / vout may not alias them.
hipError_t sort_pairs_u32(void* tmp, size_t& tb, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                          uint32_t* vout, uint32_t n, int bits, hipStream_t s);
hipError_t sort_pairs_u64(void* tmp, size_t& tb, const unsigned long long* kin, unsigned long long* kout,
                          const uint32_t* vin, uint32_t* vout, uint32_t n, int bits, hipStream_t s);
hipError_t launch_orswot_ser(hipStream_t s, OrswotSerScratch& sc, const OrswotSerArgs& a);
// the same in two halves: the sorts and scans over the n collected pairs (no host input), then the
// writer (needs the host-built prefix / suffix) -- the host builds them while the sorts run
hipError_t launch_orswot_ser_sort(hipStream_t s, OrswotSerScratch& sc, uint32_t n);
hipError_t launch_orswot_ser_write(hipStream_t s, const OrswotSerScratch& sc, const OrswotSerArgs& a);
size_t orswot_ser_tmp_bytes(uint32_t n);

// reader over the bytes [lo, hi) of state plaintext s that follow the entries map header
struct OrswotReadArgs {
  const uint8_t* s;
  uint64_t lo, hi;
  uint32_t* n_cand_dev;  // stage 0: entry heads found (pinned; stage 1: those from lo on)
  uint32_t* skip;        // device word: stage 0 the heads found, stage 1 (k_rdm_skip) the heads
                         // before lo (stage 0 runs with lo = 0, before the host knows lo)
  uint32_t cap;          // room in cand
  uint32_t n_cand;       // stage >= 1: the entries (the first n_cand heads; host-checked)
  uint32_t* cand;        // entry heads in position order (positions from the file's start)
  uint32_t* end;        // entry end (relative to lo), n_cand
  uint32_t* ndots;      // non-zero Dots per entry
  uint32_t* dbase;      // exclusive scan of ndots
  unsigned long long* member;  // per entry
  unsigned long long* msort;   // repeat check: open-addressing set of the members, dset_mask + 2
                               // words (all ones = empty; the last word counts all-ones members)
  uint32_t dset_mask;          // power of two minus one, >= 2 n_cand - 1
  uint32_t* tail_out;          // stage 1: end, dbase, ndots of the last entry and the flags word
  uint32_t* tail_dev;          // optional device words: end, dbase, ndots of the last entry (as
                               // tail_out) and [3] = 1 when the tail is exactly an empty deferred
                               // map (k_rdm_tail) -- what a merge queued before the host wait reads
  uint32_t* go;                // optional (stage 2, one launch): device word and go[1] pinned --
  uint32_t* go_host;           //   1 when every file of the launch is flag-free with an empty map
  uint8_t* tail_host;          // stage 1: the bytes after the entries (the deferred map) when they
  uint32_t tail_cap;           //   fit tail_cap (pinned; else the host downloads them)
  uint32_t* flags;      // 1 non-canonical entry, 2 broken chain, 4 unknown actor, 8 repeated member,
                        // 16 heads found outside [n_cand, cap] (stages 1-2 skip the file)
  const ActorSlot* table;
  uint32_t mask;
  unsigned long long* col_member;
  uint32_t* col_actor;
  unsigned long long* col_value;
  uint32_t chunk0, nchunks;    // multi-file reader: this file's 4 KiB chunks in the count array
};
// kRdInline descriptors per launch, passed by value (launch_orswot_read_multi)
static constexpr uint32_t kRdInline = 16;
struct RdFiles {
  OrswotReadArgs f[kRdInline];
};
// the reader over nf files at once (d_args / h_args: the same descriptors in HBM and on the
// host): stage 0 = entry heads in position order into `cand` and their count into *n_cand_dev
// (chunk_cnt / chunk_scan: sum of nchunks + 1 words); 1 = entry parse, chain check, repeated
// members, Dot scan, tail words and tail bytes; 2 = emit columns, then each file's flags word into
// n_cand_dev[1].  The stages are queued back to back: a file whose earlier stage failed is skipped
// by the later ones (its flags word), so one host wait covers all three
hipError_t launch_orswot_read_multi(hipStream_t s, const OrswotReadArgs* d_args, const OrswotReadArgs* h_args,
                                    uint32_t nf, int stage, uint32_t* chunk_cnt, uint32_t* chunk_scan,
                                    void* tmp, size_t tmp_bytes);
size_t orswot_read_multi_tmp_bytes(uint32_t nchunks);
uint32_t orswot_read_chunks(uint64_t lo, uint64_t hi);

}  // namespace ce
