// ce_kernels.h -- host-side launch interface of the gfx950 kernels (ce_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ce_common.h"

namespace ce {

// Segment = up to kSegPages pages of 4 KiB of ciphertext processed by one wavefront.
static constexpr uint32_t kPageBytes = 4096;
static constexpr uint32_t kSegPages = 4;
static constexpr uint32_t kSegBlocks = kSegPages * kPageBytes / 16;  // Poly1305 blocks
// files with at most one page of ciphertext are opened, decoded and folded in one kernel
static constexpr uint32_t kSmallMax = kPageBytes;

// Per-file AEAD parameters written by the setup kernels (256 B, read with scalar loads).
struct alignas(16) FileParams {
  uint32_t subkey[8];    // HChaCha20(key, nonce[0:16])
  uint32_t n2[2];        // nonce[16:24] (ChaCha20 nonce words 14, 15; word 13 = 0)
  uint32_t pad0[2];
  uint32_t s[4];         // Poly1305 s
  uint32_t tag[4];       // expected tag (open)
  uint32_t rpow[7][5];   // r^(2^k), k = 0..6, radix-2^26 limbs
  uint32_t pad1;
  uint64_t in_off;       // open: ciphertext offset in the input blob; seal: clear text offset
  uint64_t out_off;      // open: plaintext offset in the output; seal: ciphertext offset
  uint32_t len;          // ciphertext length without tag (== plaintext length)
  int32_t status;
  uint32_t nseg;
  uint32_t extra_base;   // first entry of this file's extra segments (nseg > 1)
};
static_assert(sizeof(FileParams) == 256, "FileParams layout");

// Per-file constants of the single-page fused open (k_open_fold_v3), written by the open setup
// (lane per file) so the kernel's 16-lane groups do not each recompute them.  With delta =
// 4 ceil(len / 64) - ceil(len / 16) pieces missing from the last ChaCha20 block, the tag
// polynomial is T = U r^(6 - delta) + G' r^2 + L r (U: the lanes' chains, G': the last block's
// pieces, L: the length block le64(0) || le64(len) + 2^128).
struct alignas(16) PolyAux {
  uint32_t r3[5];   // r^3 (the full blocks' four-product step)
  uint32_t r12[5];  // r^12, r^48: the chains' weights r^(4q) = r^(4 (q & 3)) r^(16 (q >> 2))
  uint32_t r48[5];
  uint32_t e6[5];   // r^(6 - delta)
  uint32_t lr[5];   // L r mod p
  uint32_t ts[4];   // (tag - s) mod 2^128: T mod p must equal it (xchacha lib.rs:92-97)
  uint32_t pad[3];
};
static_assert(sizeof(PolyAux) == 128, "PolyAux layout");

struct DevKey {
  uint32_t k[8];
};

// device scratch shared by one batch
struct SegScratch {
  uint32_t* counters;     // [0] extra segments, [1] multi-segment files, [2] auth failures,
                          // [3] decode failures, [4] misses, [5] first failing index (min),
                          // [6] partial slots, [7] host-parse envelopes, [8] setup failures,
                          // [9] large files, [11] / [14] multi-segment files folded from
                          // segment records / decoded whole (k_segdec_apply),
                          // [12] gate: batch not in load_ops shape,
                          // [13] gate: first gap
  uint2* extra_list;      // (file, seg) for segments j >= 1
  uint32_t extra_cap;
  uint32_t* multi_files;  // files with nseg > 1
  uint32_t* partials;     // 5 limbs per segment: [file-major] base = extra index
  uint32_t* large_list;   // files with more than one page (counters[9] entries)
  uint32_t seg_blocks;    // Poly1305 blocks per segment: kSegBlocks; a seal of a few small files
                          // (a compaction's state) uses one page, 4x the waves in flight
};

// One launch for an ingest's scratch initialisation (each hipMemsetAsync is its own blit
// dispatch with its own gap): ranges of u32 words set to a value, and the 16-word counter block
// zeroed with [5] (first failing index) and [13] (the gate's first gap) = UINT32_MAX.
static constexpr int kMaxFill = 10;
struct FillRange {
  uint32_t* p;
  uint64_t words;
  uint32_t value;
  const uint32_t* src = nullptr;  // non-null: copy `words` words from src (e.g. mapped pinned host memory)
};
struct FillArgs {
  FillRange r[kMaxFill];
  int n;
  uint32_t* counters;  // or null
};
hipError_t launch_fill(hipStream_t s, const FillArgs& a);
// src[0..n) -> dst[0..n) (mapped pinned memory), then dst[n] = gen once they are visible (n <= 64)
hipError_t launch_publish_words(hipStream_t s, const uint32_t* src, uint32_t n, uint32_t* dst, uint32_t gen);
// a compaction's sealed-file length (clear length read on the device at clear_len_at, <= bound;
// ~0 when over cap, ~1 when over bound) -> len_out (mapped pinned memory)
hipError_t launch_publish_sealed_len(hipStream_t s, const uint64_t* clear_len_at, uint64_t bound, uint64_t cap,
                                     uint64_t* len_out);

// file-level open: outer version check (when outer), envelope parse, key schedule.
hipError_t launch_open_setup(hipStream_t s, const uint8_t* blob, const uint64_t* offs,
                             uint32_t n, bool outer, DevKey key, int32_t key_status,
                             FileParams* params, int32_t* status, SegScratch sc,
                             PolyAux* aux = nullptr);
// seal setup: header write + key schedule; out_offs[i] = start of output i.
hipError_t launch_seal_setup(hipStream_t s, const uint8_t* clear, const uint64_t* offs,
                             uint32_t n, const uint8_t* outer_version /* device, or null */,
                             const uint8_t* nonces, uint8_t* out, const uint64_t* out_offs,
                             DevKey key, FileParams* params, SegScratch sc);
// one wavefront per segment (grid-stride); seal selects encrypt.
hipError_t launch_segments(hipStream_t s, bool seal, const uint8_t* in, uint8_t* out,
                           const FileParams* params, uint32_t n, int32_t* status, SegScratch sc,
                           uint32_t grid_waves, bool skip_small = false);
// multi-segment files: combine partial Poly1305 sums, emit/compare tag (one wave per file);
// n = files in the batch (bounds the multi-segment count, sizes the grid)
hipError_t launch_finalize_multi(hipStream_t s, bool seal, uint8_t* out, const FileParams* params,
                                 int32_t* status, SegScratch sc, uint32_t n);

// decode Vec<Dot<Uuid>> of every opened file and max-fold the dots of applied files into
// batch_counters (dense by actor slot).  One wavefront per file.
// Orswot op files decoded inside the open (k_open_fold_v2's DS form; ce_fused.hip
// ds_fused_decode): a file of at most kDsFuseRegion plaintext bytes whose ops are all the
// canonical one-member Add / one-entry-clock Rm forms has its op columns written as file-major
// rows (op k of file f at col[f * rows + k]) and its counts into rawcnt; any other file has its
// plaintext stored to HBM for the lane-per-file decode (done[f] = 0).
static constexpr uint32_t kDsFuseRegion = 2048;
struct DsFuse {
  int on;
  uint32_t rows;                 // rows per file (<= 96)
  uint32_t* rawcnt;              // [5][n]: adds, add members, removals, removal clock entries, removal members
  uint8_t* done;                 // [n]
  uint32_t* add_actor;           // dot-set actor ids (ActorSlot.pad[0])
  unsigned long long* add_ctr;
  unsigned long long* add_mem;
  uint32_t* rm_actor;
  unsigned long long* rm_ctr;
  unsigned long long* rm_mem;
  uint32_t* why;                 // diagnostics (CE_DS_FUSE_DEBUG=1): per file, the step that declined it
  uint8_t* big;                  // [n] k_open_ds8: 1 = a single-page file past kDsFuseRegion, left
                                 // to the 16-lane DS kernel's pass over that mask (a.only)
};

struct DecodeArgs {
  const uint8_t* pt;            // plaintext blob (FileParams.out_off / len)
  const FileParams* params;
  int32_t* status;
  uint32_t n;
  const uint8_t* supported;     // n_supported * 16 bytes (device)
  uint32_t n_supported;
  const uint8_t* apply;         // 1 = fold this file (version gate), null = all
  const ActorSlot* table;       // open addressing, capacity = mask + 1
  uint32_t mask;
  unsigned long long* batch;    // [capacity] max counters
  uint32_t* counters;           // SegScratch counters
  uint4* miss_list;             // actors not in the table
  uint32_t miss_cap;
  uint8_t* refold;              // per file: had a miss
  const uint8_t* only;          // null, or per-file: process only files with only[i] != 0
  int large_only;               // skip files the fused kernel handles (iterate large_list)
  int ablate;                   // diagnostics only (CE_ABLATE): 1 no decode, 2 no Poly1305,
                                // 4 no ChaCha20, 8 no ciphertext loads -- results invalid
  unsigned long long* prof;     // diagnostics only (CE_PROF): per-wave phase cycles, 8 per wave
  const uint32_t* large_list;
  const uint8_t* blob;          // fused kernel: input files (ciphertext at FileParams.in_off)
  uint8_t* redo;                // k_segdec_apply: files left to the whole-file decode
  int nil_actor;                // the nil UUID is in the actor table: lookups take the two-load
                                // probe (lookup_slot1)
  DsFuse ds;                    // launch_open_small_v2: Orswot ops decoded in the open (ds.on)
  const PolyAux* aux;           // fused open (k_open_fold_v3): the setup's per-file constants
};
hipError_t launch_decode_dots(hipStream_t s, const DecodeArgs& a, uint32_t grid_waves);
// diagnostics: shader clock vs the reference clock (ce_ctx_clock_probe)
hipError_t launch_clock_probe(hipStream_t s, unsigned long long* out, uint32_t blocks,
                              uint32_t samples, uint32_t ticks);

// multi-page Vec<Dot> decode split over kSplitParts waves per file (large_list order); files
// with fewer than kSplitMinDots Dots, or whose parts do not all verify, take the one-wave path
static constexpr uint32_t kSplitParts = 16;
static constexpr uint32_t kSplitMinDots = 2048;
static constexpr uint32_t kSplitDone = 0xfffffffeu;  // record 0: file decoded in one wave
struct SplitScratch {
  uint4* part;     // [n_large * kSplitParts] (slot + 1 | 0 none | ~0 failed, 0, max lo, max hi)
};
hipError_t launch_decode_split(hipStream_t s, const DecodeArgs& a, SplitScratch sp, uint32_t n_large);
// C4 fused decode: open segments of large files with the decode in the same pass (one-segment
// files folded there; longer files leave per-segment records, 2 uint4 per Poly1305 partial
// slot), then k_segdec_apply after launch_finalize_multi checks the records and folds
hipError_t launch_segments_decode(hipStream_t s, const uint8_t* in, uint8_t* out, const DecodeArgs& da,
                                  SegScratch sc, uint32_t grid_waves, uint4* rec);
hipError_t launch_segdec_apply(hipStream_t s, const DecodeArgs& a, SegScratch sc, const uint4* rec,
                               uint32_t n_large);

// fused open + decode + fold of single-page files (ce_fused.hip); files_per_wave in {1, 2, 4}
hipError_t launch_open_fold_small(hipStream_t s, const DecodeArgs& a, int files_per_wave);
// the same with whole ChaCha20 blocks per lane (keystream XOR in registers; ce_fused.hip
// k_open_fold_v2); files_per_wave in {2, 4}
// t0 / t1: timing events recorded by the dispatch itself (hipExtLaunchKernel), or none
hipError_t launch_open_fold_v2(hipStream_t s, const DecodeArgs& a, int files_per_wave,
                               hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// open only: single-page files (<= kSmallMax) into a.pt at their out_off, 16 lanes per file
// (k_open_fold_v2<..., DEC = false>); statuses and the failure counters as the segment pass sets them
hipError_t launch_open_small_v2(hipStream_t s, const DecodeArgs& a);

// version gate on the device (ce_fused.hip): files grouped by actor with consecutive versions
// (Storage::load_ops order, storage.rs:36-40) -> apply flags, first gap, next versions.
struct GateArgs {
  const uint32_t* fa;      // file -> local actor index
  const uint64_t* fv;      // file version
  uint32_t n, m;
  const uint64_t* e0;      // expected version per local actor (next_op_versions.get)
  uint32_t* run_count;     // [m]
  uint32_t* run_first;     // [m]
  uint32_t* flags;         // [0] not grouped/consecutive, [1] first gap (min file index)
  unsigned long long* newnov;  // [m] max(v + 1) over applied files
  uint8_t* apply;          // [n]
  unsigned long long* newnov_host;  // optional mapped pinned copy of newnov (zeroed by the host;
                                    // exact when flags[0] stays 0: one run per actor)
};
hipError_t launch_gate(hipStream_t s, const GateArgs& g);

// dst[i] = max(dst[i], src[i])
hipError_t launch_merge_max(hipStream_t s, unsigned long long* dst,
                            const unsigned long long* src, uint32_t n);
// launch_merge_max unless the counter block flags a batch that cannot commit as folded
hipError_t launch_merge_max_if(hipStream_t s, unsigned long long* dst, const unsigned long long* src,
                               uint32_t n, const uint32_t* counters);
// nov[wslot[a]] = max(nov[wslot[a]], newnov[a]) unless the counters flag (as launch_merge_max_if)
hipError_t launch_nov_apply(hipStream_t s, unsigned long long* nov, const uint32_t* wslot,
                            const unsigned long long* newnov, uint32_t m, const uint32_t* counters);
// to_vec_named(StateWrapper<VClock|GCounter>) from the dense nov / state arrays (k sorted slots);
// clear length -> offs[1] (offs[0] = 0).  Upper bound of the output: vclock_ser_bound(k)
hipError_t launch_serialize_vclock(hipStream_t s, const unsigned long long* nov,
                                  const unsigned long long* st, const uint32_t* sorted, uint32_t k,
                                  const ActorSlot* table, bool gcounter, const uint8_t* prefix16,
                                  uint8_t* out, unsigned long long* offs);
inline uint64_t vclock_ser_bound(uint64_t k) { return 16 + 24 + 5 + 27 * k + 19 + 5 + 27 * k; }

// The compaction's prologue as one launch (instead of an 80-byte upload, two counter fills and
// k_nov_apply): the seal's small arguments at `args` -- offs[2] = {0, (serializer)}, out_offs[1]
// = {0}, nonce (24 B), outer version (16 B), data-version prefix (16 B) --, the seal context's
// counter block reset (as reset_counters: zero, [5] = [13] = UINT32_MAX), and, with m > 0,
// nov[wslot[a]] = max(nov[wslot[a]], newnov[a]) unless the ingest's counters flag (k_nov_apply).
struct CompactArgs {
  uint8_t nonce[24];
  uint8_t outer[16];
  uint8_t prefix[16];
};
// with merge_n > 0 also the ingest's commit, as k_merge_max_if (same skip condition)
hipError_t launch_compact_prologue(hipStream_t s, uint8_t* args, const CompactArgs& ca, uint32_t* seal_counters,
                                   unsigned long long* nov, const uint32_t* wslot,
                                   const unsigned long long* newnov, uint32_t m, const uint32_t* counters,
                                   unsigned long long* merge_dst = nullptr,
                                   const unsigned long long* merge_src = nullptr, uint32_t merge_n = 0);
// The compaction's epilogue readback in one place: dst = [clear length u64 (from src_len) |
// the ingest's counter block (16 u32) | newnov u64[m]], so one download carries what the host
// reads after the step.
hipError_t launch_tail_pack(hipStream_t s, uint8_t* dst, const unsigned long long* src_len,
                            const uint32_t* counters, const unsigned long long* newnov, uint32_t m);

// Byte ranges of device memory packed into one device buffer (dst + dst_off), so that a batch
// of per-file pieces comes back in ONE download (each hipMemcpyAsync is its own blit dispatch
// with its own gap on the box).  Any alignment.
struct GatherRange {
  const uint8_t* src;
  uint64_t dst_off, len;
};
hipError_t launch_gather_ranges(hipStream_t s, uint8_t* dst, const GatherRange* r, uint32_t n);

// Per opened state file, 32 bytes: status (i32) | clear length (u32) | plaintext offset (u64) |
// the plaintext's first 16 bytes (the data version) when the status is CE_OK and len >= 16
hipError_t launch_state_heads(hipStream_t s, const FileParams* params, const int32_t* status,
                              const uint8_t* out, uint32_t n, uint8_t* dst);

}  // namespace ce
