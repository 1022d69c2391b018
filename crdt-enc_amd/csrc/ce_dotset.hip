// ce_dotset.hip -- gfx950 kernels of the Orswot / MVReg fold (crdts 7 semantics, see
// ce_dotset.h for the HBM layout and tests/dotset_model.py for the formulation).
//
// Everything here is integer / pointer-chasing work bounded by HBM latency and atomics, so the
// kernels are grid-stride loops of 256-thread blocks, one lane per file / op / pair bucket;
// block-level LDS counters keep the global atomics to one per block.  No MFMA: nothing here is a
// contraction.
#include <hip/hip_runtime.h>

#include <cstdlib>


#include "ce_dotset.h"
#include "ce_dotset_codec.h"
#include "ce_dotset_io.h"

namespace ce {
namespace {

constexpr int kBlock = 256;

inline uint32_t blocks_for(uint64_t n, uint32_t cap = 8192) {
  uint64_t b = (n + kBlock - 1) / kBlock;
  if (b == 0) b = 1;
  return (uint32_t)(b < cap ? b : cap);
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ unsigned long long ld_volatile(const unsigned long long* p) {
  return __atomic_load_n(p, __ATOMIC_RELAXED);
}

// member handle (index into mkey) or kDsEmpty when absent (insert = false).  A member lives in
// the primary table (smask + 1 slots, sized for the members actually present: small enough to stay
// in L2) unless the kMemberWindow slots of its probe sequence there were all taken by other members
// when it was inserted; then it lives in the overflow table (as large as the pair table, so it
// never fills).  Slots never empty again, so a lookup that meets an empty slot in the window knows
// the member is in neither table, and every thread inserting one member takes the same branch.
constexpr uint32_t kMemberWindow = 32;

__device__ __forceinline__ unsigned long long member_reserved(const DsTables& t) {
  return (unsigned long long)t.smask + 1 + t.mmask + 1;
}

__device__ unsigned long long member_find(const DsTables& t, unsigned long long m, bool insert) {
  if (m == kDsEmpty) return member_reserved(t);  // reserved bucket
  const unsigned long long x = mix64(m);
  uint32_t h = (uint32_t)x & t.smask;
  for (uint32_t probe = 0; probe < kMemberWindow; probe++) {
    const unsigned long long k = ld_volatile(t.mkey + h);
    if (k == m) return h;
    if (k == kDsEmpty) {
      if (!insert) return kDsEmpty;
      const unsigned long long prev = atomicCAS(t.mkey + h, kDsEmpty, m);
      if (prev == kDsEmpty || prev == m) return h;
    }
    h = (h + 1) & t.smask;
  }
  const unsigned long long base = (unsigned long long)t.smask + 1;
  unsigned long long* ov = t.mkey + base;
  h = (uint32_t)(x >> 32) & t.mmask;
  for (uint32_t probe = 0; probe <= t.mmask; probe++) {
    const unsigned long long k = ld_volatile(ov + h);
    if (k == m) return base + h;
    if (k == kDsEmpty) {
      if (!insert) return kDsEmpty;
      const unsigned long long prev = atomicCAS(ov + h, kDsEmpty, m);
      if (prev == kDsEmpty || prev == m) return base + h;
    }
    h = (h + 1) & t.mmask;
  }
  atomicAdd(t.live + 2, 1u);  // table full (host sizes it to <= 50% load)
  return kDsEmpty;
}

// used primary member slots among [b * per, (b + 1) * per) for block b of nb (live[4] after a
// fold / k-way merge: ensure_pairs grows the primary table past half full)
__device__ __forceinline__ uint32_t primary_used(const DsTables& t, uint32_t b, uint32_t nb) {
  const uint32_t ms = t.smask + 1, per = (ms + nb - 1) / nb;
  const uint32_t i0 = min(ms, b * per), i1 = min(ms, i0 + per);
  uint32_t n = 0;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) n += t.mkey[i] != kDsEmpty;
  return n;
}

// The pair table is cut into partitions of kDsPartSlots consecutive slots: a key's probe sequence
// starts at mix64(key) & pmask and wraps inside that slot's partition, so one partition holds every
// pair whose hash lands in it (k_ds_part_apply folds a partition in LDS).  The tables are always
// at least one partition (tables_alloc: >= 4096 slots).
__device__ __forceinline__ uint32_t pair_part(const DsTables& t, unsigned long long key) {
  return ((uint32_t)mix64(key) & t.pmask) >> kDsPartBits;
}

__device__ unsigned long long pair_find(const DsTables& t, unsigned long long key, bool insert) {
  uint32_t h = (uint32_t)mix64(key) & t.pmask;
  const uint32_t lo = h & ~(kDsPartSlots - 1);
  for (uint32_t probe = 0; probe < kDsPartSlots; probe++) {
    const unsigned long long k = ld_volatile(t.pkey + h);
    if (k == key) return h;
    if (k == kDsEmpty) {
      if (!insert) return kDsEmpty;
      const unsigned long long prev = atomicCAS(t.pkey + h, kDsEmpty, key);
      if (prev == kDsEmpty || prev == key) return h;
    }
    h = lo | ((h + 1) & (kDsPartSlots - 1));
  }
  atomicAdd(t.live + 2, 1u);
  return kDsEmpty;
}

// pair_find(insert = true) that also says whether this call inserted the key (its compare-and-swap
// won): exactly one caller per new pair does
__device__ unsigned long long pair_find_ins(const DsTables& t, unsigned long long key, bool* ins) {
  uint32_t h = (uint32_t)mix64(key) & t.pmask;
  const uint32_t lo = h & ~(kDsPartSlots - 1);
  *ins = false;
  for (uint32_t probe = 0; probe < kDsPartSlots; probe++) {
    const unsigned long long k = ld_volatile(t.pkey + h);
    if (k == key) return h;
    if (k == kDsEmpty) {
      const unsigned long long prev = atomicCAS(t.pkey + h, kDsEmpty, key);
      if (prev == kDsEmpty) {
        *ins = true;
        return h;
      }
      if (prev == key) return h;
    }
    h = lo | ((h + 1) & (kDsPartSlots - 1));
  }
  atomicAdd(t.live + 2, 1u);
  return kDsEmpty;
}

__device__ __forceinline__ unsigned long long pair_key(unsigned long long handle, uint32_t aid) {
  return (handle << kDsActorBits) | aid;
}

__device__ __forceinline__ unsigned long long member_of(const DsTables& t, unsigned long long h) {
  return h == member_reserved(t) ? kDsEmpty : t.mkey[h];
}

// block-aggregated counter increment: returns this lane's index among all incrementing lanes
__device__ __forceinline__ unsigned long long wave_max64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = ((unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o) << 32) |
                                 (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    v = y > v ? y : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t block_count(uint32_t* global, bool pred, uint32_t* lds) {
  if (threadIdx.x == 0) *lds = 0;
  __syncthreads();
  uint32_t mine = 0;
  if (pred) mine = atomicAdd(lds, 1u);
  __syncthreads();
  if (threadIdx.x == 0 && *lds) lds[1] = atomicAdd(global, *lds);
  __syncthreads();
  return lds[1] + mine;
}

// ---------------------------------------------------------------------------------------
// decode: one lane per file
// ---------------------------------------------------------------------------------------
// the last actor a lane resolved (a file's ops are mostly its writer's)
struct ActorCache {
  uint4 k = make_uint4(0, 0, 0, 0);
  uint32_t id = kDsNoActor;
};

// ST (staged): the file's bytes sit in LDS (k_ds_count / k_ds_emit stage a wave's files); every
// LDS access stays dword-aligned -- aligned dword loads, bytes shifted into place with alignbyte
template <bool ST>
__device__ __forceinline__ uint4 load16(const uint8_t* q) {
  if (!ST) return *reinterpret_cast<const uint4*>(q);  // unaligned 16 B inside the plaintext
  const uintptr_t x = reinterpret_cast<uintptr_t>(q);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(x & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(x & 3);
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = b[k];
  return make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], sh), __builtin_amdgcn_alignbyte(d[2], d[1], sh),
                    __builtin_amdgcn_alignbyte(d[3], d[2], sh), __builtin_amdgcn_alignbyte(d[4], d[3], sh));
}

template <bool ST = false>
__device__ __forceinline__ uint32_t lookup_actor(const DsDecodeArgs& a, const uint8_t* u,
                                                 ActorCache* cache = nullptr) {
  const uint4 k = load16<ST>(u);
  if (cache && cache->id != kDsNoActor && k.x == cache->k.x && k.y == cache->k.y &&
      k.z == cache->k.z && k.w == cache->k.w)
    return cache->id;
  const uint32_t w[4] = {k.x, k.y, k.z, k.w};
  uint32_t h = actor_hash(w[0], w[1], w[2], w[3]) & a.mask;
  for (uint32_t probe = 0; probe <= a.mask; probe++) {
    const ActorSlot& s = a.table[h];
    if (!s.used) break;
    if (s.k[0] == w[0] && s.k[1] == w[1] && s.k[2] == w[2] && s.k[3] == w[3]) {
      if (cache) { cache->k = k; cache->id = s.pad[0]; }
      return s.pad[0];
    }
    h = (h + 1) & a.mask;
  }
  const uint32_t i = atomicAdd(a.counters + 2, 1u);
  if (i < a.miss_cap) a.miss_list[i] = make_uint4(w[0], w[1], w[2], w[3]);
  return kDsNoActor;
}

template <bool ST = false>
struct CountSinkT {
  static constexpr bool kStaged = ST;
  uint32_t c[kCntN] = {0, 0, 0, 0, 0};
  __device__ void add_begin() { c[kCntAdd]++; }
  __device__ void add_dot(uint64_t, uint64_t) {}
  __device__ void add_member(uint64_t) { c[kCntAddM]++; }
  __device__ void add_end() {}
  __device__ void rm_begin() { c[kCntRm]++; }
  __device__ void rm_dot(uint64_t, uint64_t) { c[kCntRmC]++; }
  __device__ void rm_member(uint64_t) { c[kCntRmM]++; }
  __device__ void rm_end() {}
  __device__ void put_begin() { c[kCntRm]++; }
  __device__ void put_dot(uint64_t, uint64_t) { c[kCntRmC]++; }
  __device__ void put_val(uint64_t) {}
  __device__ void put_end() {}
};

// TILE (Orswot, DsDecodeArgs.tile): every column entry goes to its file-minor scratch row
// instead -- entry k of file i at tile.col[c][k * npad + i] -- so a wave's 64 files write 64
// consecutive words per store when their files share a layout (k_ds_untile then writes the CSR
// columns in order); the values (ids, counters, CSR offsets) are the same.
template <bool TILE, bool ST = false>
struct EmitSinkT {
  static constexpr bool kStaged = ST;
  const DsDecodeArgs* a;
  const uint8_t* p;
  uint32_t ia, iam, ir, irc, irm;
  uint32_t ia0, iam0, ir0, irc0, irm0, file;  // TILE: the file's bases and index
  ActorCache cache;
  template <typename T>
  __device__ __forceinline__ void put(T* col, int c, uint32_t idx, uint32_t base, T v) {
    if (TILE) reinterpret_cast<T*>(a->tile.col[c])[(size_t)(idx - base) * a->tile.npad + file] = v;
    else col[idx] = v;
  }
  __device__ void add_begin() { put(a->ops.add_mbeg, 2, ia, ia0, iam); }
  __device__ void add_dot(uint64_t off, uint64_t c) {
    put(a->ops.add_actor, 0, ia, ia0, lookup_actor<ST>(*a, p + off, &cache));
    put(a->ops.add_ctr, 1, ia, ia0, (unsigned long long)c);
  }
  __device__ void add_member(uint64_t m) { put(a->ops.add_mem, 3, iam, iam0, (unsigned long long)m); iam++; }
  __device__ void add_end() { ia++; }
  __device__ void rm_begin() {
    put(a->ops.rm_cbeg, 4, ir, ir0, irc);
    put(a->ops.rm_mbeg, 5, ir, ir0, irm);
  }
  __device__ void rm_dot(uint64_t off, uint64_t c) {
    put(a->ops.rmc_actor, 6, irc, irc0, lookup_actor<ST>(*a, p + off, &cache));
    put(a->ops.rmc_ctr, 7, irc, irc0, (unsigned long long)c);
    irc++;
  }
  __device__ void rm_member(uint64_t m) { put(a->ops.rm_mem, 8, irm, irm0, (unsigned long long)m); irm++; }
  __device__ void rm_end() { ir++; }
  __device__ void put_begin() { a->ops.rm_cbeg[ir] = irc; }
  __device__ void put_dot(uint64_t off, uint64_t c) {
    a->ops.rmc_actor[irc] = lookup_actor<ST>(*a, p + off, &cache);
    a->ops.rmc_ctr[irc] = c;
    irc++;
  }
  __device__ void put_val(uint64_t v) { a->ops.put_val[ir] = v; }
  __device__ void put_end() { ir++; }
};

// ---- canonical-op fast path of the lane-per-file Orswot op decode --------------------------
// The grammar (ce_dotset_codec.h) walks a file byte by byte, one dependent global load per byte.
// The forms rmp-serde's to_vec_named writes for the common ops are checked instead from 64-byte
// register windows (unaligned 16-byte loads; every plaintext buffer has >= 64 bytes of slack
// past its last file):
//   Add: 81 a3"Add" 82 a3"dot" 82 a5"actor" c4 10 <uuid> a7"counter" <uint> a7"members" 91 <uint>
//   Rm:  81 a2"Rm" 82 a5"clock" 81 a4"dots" 81 c4 10 <uuid> <uint> a7"members" 91 <uint>
// (one member; a one-entry clock), <uint> = positive fixint / cc / cd / ce / cf.  Anything else
// -- other widths, more members or clock entries, reordered or extra fields -- is parsed by the
// grammar from the same op on (no sink call is made before an op is fully proven), so the sink
// sees exactly the calls ds_parse_orswot_ops would make.
template <bool ST = false>
struct Win64 {
  uint32_t w[16];
  __device__ __forceinline__ explicit Win64(const uint8_t* q) {
    if (ST) {  // staged in LDS: 17 aligned dwords, shifted (load16)
      const uintptr_t x = reinterpret_cast<uintptr_t>(q);
      const uint32_t* b = reinterpret_cast<const uint32_t*>(x & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(x & 3);
      uint32_t d[17];
#pragma unroll
      for (int k = 0; k < 17; k++) d[k] = b[k];
#pragma unroll
      for (int k = 0; k < 16; k++) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 v = *reinterpret_cast<const uint4*>(q + 16 * k);  // unaligned
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  }
  // LE word at byte b (b compile-time, b + 4 <= 64)
  __device__ __forceinline__ uint32_t word(int b) const {
    return (b & 3) ? __builtin_amdgcn_alignbyte(w[(b >> 2) + 1], w[b >> 2], b & 3) : w[b >> 2];
  }
  __device__ __forceinline__ uint32_t byte(int b) const { return (w[b >> 2] >> (8 * (b & 3))) & 0xffu; }
  // msgpack uint at byte b (positive fixint, cc, cd, ce, cf); *len = its size, 0 if another form
  __device__ __forceinline__ uint64_t uint_at(int b, uint32_t* len) const {
    const uint32_t m = byte(b);
    const uint32_t x0 = __builtin_bswap32(word(b + 1)), x1 = __builtin_bswap32(word(b + 5));
    if (m < 0x80u) { *len = 1; return m; }
    if (m == 0xccu) { *len = 2; return x0 >> 24; }
    if (m == 0xcdu) { *len = 3; return x0 >> 16; }
    if (m == 0xceu) { *len = 5; return x0; }
    if (m == 0xcfu) { *len = 9; return ((uint64_t)x0 << 32) | x1; }
    *len = 0;
    return 0;
  }
};

// "a7 members 91 <uint>" at q: the one-member array; returns bytes consumed, 0 if not that form
template <bool ST>
__device__ __forceinline__ uint32_t fast_members1(const uint8_t* q, uint64_t* m) {
  const Win64<ST> v(q);
  if (v.word(0) != 0x6d656da7u || v.word(4) != 0x73726562u || v.byte(8) != 0x91u) return 0;
  uint32_t l;
  *m = v.uint_at(9, &l);
  return l ? 9 + l : 0;
}

template <typename S>
__device__ __forceinline__ bool fast_orswot_op(const uint8_t* p, uint64_t n, uint64_t& i, S& sink) {
  constexpr bool ST = S::kStaged;
  if (n - i < 32) return false;
  const uint8_t* q = p + i;
  const Win64<ST> v(q);
  uint32_t l, lm;
  uint64_t ctr, mem;
  if (v.w[0] == 0x6441a381u && v.w[1] == 0x64a38264u && v.w[2] == 0xa582746fu &&
      v.w[3] == 0x6f746361u && (v.w[4] & 0xffffffu) == 0x10c472u && v.word(35) == 0x756f63a7u &&
      v.word(39) == 0x7265746eu) {  // Add
    ctr = v.uint_at(43, &l);
    if (!l) return false;
    lm = fast_members1<ST>(q + 43 + l, &mem);
    if (!lm || 43ull + l + lm > n - i) return false;
    sink.add_begin();
    sink.add_dot(i + 19, ctr);
    sink.add_member(mem);
    sink.add_end();
    i += 43 + l + lm;
    return true;
  }
  if (v.w[0] == 0x6d52a281u && v.w[1] == 0x6c63a582u && v.w[2] == 0x816b636fu && v.w[3] == 0x746f64a4u &&
      (v.w[4] & 0xf0ffu) == 0x8073u && (v.w[4] & 0x0f00u) >= 0x0200u) {
    // Rm whose clock has 2..15 entries (fixmap; crdts rm(member, read_ctx) carries the member's
    // whole read context): each entry "c4 10 <uuid> <uint>" from its own 64-byte window, the
    // entries' actors strictly ascending as ds_vclock requires (else the grammar takes the op and
    // reports it for the host parse).  Proven in full first, then the sink calls ds_orswot_op
    // would make, in the same order.
    const uint32_t ne = (v.w[4] >> 8) & 15u;
    uint64_t off = 18;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;  // the previous actor, big-endian words
    for (uint32_t e = 0; e < ne; e++) {
      if (off + 27 > n - i + 64) return false;  // (the window stays inside the buffer's slack)
      const Win64<ST> w(q + off);
      if (w.byte(0) != 0xc4u || w.byte(1) != 0x10u) return false;
      const uint32_t u0 = __builtin_bswap32(w.word(2)), u1 = __builtin_bswap32(w.word(6)),
                     u2 = __builtin_bswap32(w.word(10)), u3 = __builtin_bswap32(w.word(14));
      if (e && !(u0 > p0 || (u0 == p0 && (u1 > p1 || (u1 == p1 && (u2 > p2 || (u2 == p2 && u3 > p3)))))))
        return false;
      p0 = u0; p1 = u1; p2 = u2; p3 = u3;
      w.uint_at(18, &l);
      if (!l) return false;
      off += 18 + l;
      if (off > n - i) return false;
    }
    lm = fast_members1<ST>(q + off, &mem);
    if (!lm || off + lm > n - i) return false;
    sink.rm_begin();
    off = 18;
    for (uint32_t e = 0; e < ne; e++) {
      const Win64<ST> w(q + off);
      ctr = w.uint_at(18, &l);
      sink.rm_dot(i + off + 2, ctr);
      off += 18 + l;
    }
    sink.rm_member(mem);
    sink.rm_end();
    i += off + lm;
    return true;
  }
  if (v.w[0] == 0x6d52a281u && v.w[1] == 0x6c63a582u && v.w[2] == 0x816b636fu &&
      v.w[3] == 0x746f64a4u && v.w[4] == 0x10c48173u) {  // Rm with a one-entry clock
    ctr = v.uint_at(36, &l);
    if (!l) return false;
    lm = fast_members1<ST>(q + 36 + l, &mem);
    if (!lm || 36ull + l + lm > n - i) return false;
    sink.rm_begin();
    sink.rm_dot(i + 20, ctr);
    sink.rm_member(mem);
    sink.rm_end();
    i += 36 + l + lm;
    return true;
  }
  return false;
}

template <typename S>
__device__ int parse_orswot_fast(const uint8_t* p, uint64_t n, S& sink) {
  Rd r{p, n, 0};
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(p[0]) || !rd_array_hdr(r, &cnt) || cnt > r.n) return kDsErr;
  for (uint64_t k = 0; k < cnt; k++) {
    if (fast_orswot_op(p, n, r.i, sink)) continue;
    const int s = ds_orswot_op(r, sink);
    if (s != kDsOk) return s;
  }
  return kDsOk;
}

template <typename S>
__device__ int parse_file(int kind, const uint8_t* p, uint64_t n, S& sink) {
  return kind == kDsOrswot ? parse_orswot_fast(p, n, sink) : ds_parse_mvreg_ops(p, n, sink);
}

// ---- staged decode: a wave's 64 files copied into LDS first ---------------------------------
// A lane parses its file op by op, each op's window load waiting on the previous op's length: a
// chain of ~32 dependent loads per file.  From HBM / L2 each link costs a round trip (and the
// lanes' scattered 64-byte windows re-fetched every line ~5x at C3); staged, a wave copies its
// files' byte range [lo, hi) with coalesced 16-byte loads (eight per lane in flight) and the chain
// runs on LDS.  A wave whose range exceeds kStageWave, or a lane whose file lies outside it,
// reads HBM as before.
constexpr uint32_t kStageWave = 39 * 1024;               // bytes per wave (4 waves: 156 KB per CU)
constexpr uint32_t kStageLds = (kBlock / 64) * kStageWave;

__device__ __forceinline__ unsigned long long wave_min64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = ((unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o) << 32) |
                                 (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    v = y < v ? y : v;
  }
  return v;
}

// this lane's file bytes in the wave's LDS region, or nullptr (read from HBM).  Every lane of the
// block calls it (the copy is followed by a block barrier).
__device__ const uint8_t* stage_files(const DsDecodeArgs& a, uint32_t i, bool act, uint8_t* lds) {
  const uint64_t off = act ? a.params[i].out_off : ~0ull;
  const uint64_t end = act ? off + a.params[i].len : 0ull;
  const uint64_t lo = wave_min64(off) & ~15ull, hi = wave_max64(end);
  uint8_t* region = lds + (threadIdx.x >> 6) * kStageWave;
  // the windows read up to 64 bytes past a file's end (the buffer's slack) plus the aligned
  // loads' 4: the region holds hi - lo + 64 + 16 bytes; the copy stops inside the slack (whole
  // 16-byte vectors only: the last few slack bytes' values are never used)
  const bool ok = hi > lo && hi - lo + 64 + 16 <= kStageWave;
  if (ok) {
    const uint4* src = reinterpret_cast<const uint4*>(a.pt + lo);
    uint4* dst = reinterpret_cast<uint4*>(region);
    const uint32_t nv = (uint32_t)((hi + 64 - lo) >> 4), lane = threadIdx.x & 63;
    for (uint32_t v0 = lane; v0 < nv; v0 += 64 * 8) {
      uint4 t[8];
#pragma unroll
      for (int q = 0; q < 8; q++) t[q] = v0 + 64 * q < nv ? src[v0 + 64 * q] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (v0 + 64 * q < nv) dst[v0 + 64 * q] = t[q];
    }
  }
  __syncthreads();
  return ok && act ? region + (off - lo) : nullptr;
}

template <bool ST>
__device__ __forceinline__ int32_t count_file(const DsDecodeArgs& a, const uint8_t* p, uint32_t len,
                                              CountSinkT<ST>& cs) {
  if (len < 16) return CE_ERR_PT_LEN;  // VersionBytesRef::deserialize (lib.rs:504)
  bool ok = false;
  for (uint32_t v = 0; v < a.n_supported && !ok; v++) {
    bool eq = true;
    for (int b = 0; b < 16; b++) eq = eq && p[b] == a.supported[16 * v + b];
    ok = eq;
  }
  if (!ok) return CE_ERR_PT_VERSION;  // ensure_versions (lib.rs:505)
  const int r = parse_file(a.kind, p + 16, len - 16, cs);  // from_slice (lib.rs:507)
  if (r == kDsErr) {
    atomicAdd(a.counters + 0, 1u);
    return CE_ERR_DECODE;
  }
  if (r == kDsHost) {
    atomicAdd(a.counters + 1, 1u);
    return kStatusHostDecode;
  }
  return CE_OK;
}

template <bool STAGE>
__global__ void __launch_bounds__(kBlock) k_ds_count(DsDecodeArgs a) {
  extern __shared__ uint8_t stage_lds[];
  __shared__ uint32_t smax[kCntN], sfused, sst[4];
  if (threadIdx.x < kCntN) smax[threadIdx.x] = 0;
  if (threadIdx.x == 0) sfused = 0;
  if (threadIdx.x < 4) sst[threadIdx.x] = threadIdx.x == 3 ? 0xffffffffu : 0u;
  __syncthreads();
  uint32_t mx[kCntN];
#pragma unroll
  for (int k = 0; k < kCntN; k++) mx[k] = 0;
  uint32_t nbad = 0, nhp = 0, nhd = 0, first_bad = 0xffffffffu;
  // (STAGE: the trip count is uniform over the block -- every lane reaches the barriers)
  for (uint32_t i0 = blockIdx.x * kBlock; i0 < a.n; i0 += gridDim.x * kBlock) {
    const uint32_t i = i0 + threadIdx.x;
    const bool in = i < a.n;
    int32_t st = in ? a.status[i] : CE_ERR_DECODE;
    // decoded in the open (its tag verified): the counts it left, no parse
    const bool fd = in && a.fdone && a.fdone[i];
    const uint8_t* sp = STAGE ? stage_files(a, i, in && st == CE_OK && !fd, stage_lds) : nullptr;
    uint32_t c[kCntN] = {0, 0, 0, 0, 0};
    if (fd) {
#pragma unroll
      for (int k = 0; k < kCntN; k++) c[k] = a.fuse.rawcnt[(size_t)k * a.n + i];
    }
    if (a.fdone) {  // files the open decoded (the host reads the count with the totals)
      const unsigned long long b = __ballot(fd);
      if (b && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(b)) {
        if (a.bpart) atomicAdd(&sfused, (uint32_t)__popcll(b));
        else atomicAdd(a.counters + 5, (uint32_t)__popcll(b));
      }
    }
    if (in && st == CE_OK && !fd) {
      const uint32_t len = a.params[i].len;
      if (STAGE && sp) {
        CountSinkT<true> cs;
        st = count_file(a, sp, len, cs);
#pragma unroll
        for (int k = 0; k < kCntN; k++) c[k] = cs.c[k];
      } else {
        CountSinkT<false> cs;
        st = count_file(a, a.pt + a.params[i].out_off, len, cs);
#pragma unroll
        for (int k = 0; k < kCntN; k++) c[k] = cs.c[k];
      }
      if (st != CE_OK) a.status[i] = st;
    }
    if (in) {
      const bool keep = st == CE_OK && a.apply[i];
      for (int k = 0; k < kCntN; k++) a.cnt[(size_t)k * a.n + i] = keep ? c[k] : 0u;
#pragma unroll
      for (int k = 0; k < kCntN; k++) mx[k] = max(mx[k], keep ? c[k] : 0u);
      if (st != CE_OK) {  // the status summary (final statuses: the parse above may have failed)
        nbad++;
        nhp += st == kStatusHostParse;
        nhd += st == kStatusHostDecode;
        first_bad = min(first_bad, i);
      }
    }
    if (STAGE) __syncthreads();  // the next trip's staging overwrites the region
  }
  // the largest per-file count of each column (counters[8 + k]): the tiled emit's row count;
  // reduced per wave, then per block in LDS, so each block adds one global atomic per column
#pragma unroll
  for (int k = 0; k < kCntN; k++) {
    uint32_t m = mx[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(&smax[k], m);
  }
  if (nbad) {
    atomicAdd(&sst[0], nbad);
    if (nhp) atomicAdd(&sst[1], nhp);
    if (nhd) atomicAdd(&sst[2], nhd);
    atomicMin(&sst[3], first_bad);
  }
  __syncthreads();
  if (a.bpart) {
    if (threadIdx.x < kCntN) a.bpart[kDsCountPart * blockIdx.x + threadIdx.x] = smax[threadIdx.x];
    if (threadIdx.x == kCntN) a.bpart[kDsCountPart * blockIdx.x + 5] = sfused;
    if (threadIdx.x >= 8 && threadIdx.x < 12) a.bpart[kDsCountPart * blockIdx.x + threadIdx.x] = sst[threadIdx.x - 8];
  } else if (threadIdx.x < kCntN && smax[threadIdx.x]) {
    atomicMax(a.counters + 8 + threadIdx.x, smax[threadIdx.x]);
  }
}

template <bool TILE, bool ST>
__device__ __forceinline__ void emit_file(const DsDecodeArgs& a, uint32_t i, const uint8_t* p) {
  const uint32_t len = a.params[i].len;
  EmitSinkT<TILE, ST> es;
  es.a = &a;
  es.p = p;
  // the bases are one exclusive scan over all kCntN columns back to back: column k's base is
  // its entry minus the column's first (u32 arithmetic: exact while a column's total < 2^32)
  auto base = [&](int k) { return a.cnt[(size_t)k * a.n + i] - a.cnt[(size_t)k * a.n]; };
  es.ia = es.ia0 = a.base_off[kCntAdd] + base(kCntAdd);
  es.iam = es.iam0 = a.base_off[kCntAddM] + base(kCntAddM);
  es.ir = es.ir0 = a.base_off[kCntRm] + base(kCntRm);
  es.irc = es.irc0 = a.base_off[kCntRmC] + base(kCntRmC);
  es.irm = es.irm0 = a.base_off[kCntRmM] + base(kCntRmM);
  es.file = i;
  parse_file(a.kind, p, len - 16, es);
}

template <bool TILE, bool STAGE>
__global__ void __launch_bounds__(kBlock) k_ds_emit(DsDecodeArgs a) {
  extern __shared__ uint8_t stage_lds[];
  for (uint32_t i0 = blockIdx.x * kBlock; i0 < a.n; i0 += gridDim.x * kBlock) {
    const uint32_t i = i0 + threadIdx.x;
    const bool act = i < a.n && a.status[i] == CE_OK && a.apply[i] && !(a.fdone && a.fdone[i]);
    const uint8_t* sp = STAGE ? stage_files(a, i, act, stage_lds) : nullptr;
    if (act) {
      if (STAGE && sp) emit_file<TILE, true>(a, i, sp + 16);
      else emit_file<TILE, false>(a, i, a.pt + a.params[i].out_off + 16);
    }
    if (STAGE) __syncthreads();
  }
}

// The tiled emit's scratch rows -> the CSR columns, in order: block (x = 64-file tile, y =
// column) stages the tile's rows (k < the tile's largest count) in LDS with coalesced reads, then
// writes the tile's contiguous output range with coalesced stores (each output index finds its
// file among the tile's 65 bases by binary search in LDS).
// Files the open decoded (a.fdone) come from its file-major rows instead (a.fuse: op k of file f at
// [f * rows + k]); their offsets columns are the op index plus the file's base in the member /
// clock-entry column (one member, one clock entry per op).  Without the tiled emit (tile.npad 0:
// the other files were stored directly) only the open's files are written.
__global__ void __launch_bounds__(kBlock) k_ds_untile(DsDecodeArgs a) {
  extern __shared__ unsigned long long tile[];  // [tile.max_rows * 64]: sized at launch
  __shared__ uint32_t sb[65];
  __shared__ uint32_t ob[64];     // fused files: the offsets column's base (add_mbeg / rm_cbeg / rm_mbeg)
  __shared__ uint8_t sdone[64];
  __shared__ uint32_t tmax;
  const int c = blockIdx.y;
  const int g = c == 0 || c == 1 || c == 2 ? kCntAdd : c == 3 ? kCntAddM : c == 4 || c == 5 ? kCntRm
                : c == 6 || c == 7 ? kCntRmC : kCntRmM;
  const bool wide = c == 1 || c == 3 || c == 7 || c == 8;
  void* const dst[9] = {a.ops.add_actor, a.ops.add_ctr, a.ops.add_mbeg, a.ops.add_mem, a.ops.rm_cbeg,
                        a.ops.rm_mbeg, a.ops.rmc_actor, a.ops.rmc_ctr, a.ops.rm_mem};
  const uint32_t i0 = blockIdx.x * 64;
  // the offsets columns' base groups: add_mbeg -> add members, rm_cbeg -> clock entries, rm_mbeg
  // -> removal members
  const int og = c == 2 ? kCntAddM : c == 4 ? kCntRmC : kCntRmM;
  const bool synth = c == 2 || c == 4 || c == 5;
  if (threadIdx.x == 0) tmax = 0;
  if (threadIdx.x <= 64) {
    const uint32_t i = i0 + threadIdx.x;
    sb[threadIdx.x] = i < a.n ? a.cnt[(size_t)g * a.n + i] - a.cnt[(size_t)g * a.n] + a.base_off[g]
                              : a.tile.total[g] + a.base_off[g];
    if (threadIdx.x < 64) {
      sdone[threadIdx.x] = i < a.n && a.fdone && a.fdone[i];
      ob[threadIdx.x] = i < a.n ? a.cnt[(size_t)og * a.n + i] - a.cnt[(size_t)og * a.n] + a.base_off[og] : 0u;
    }
  }
  // every file of the tile decoded in the open (the usual case when any was): each output entry
  // reads its file's row directly -- a file's entries are contiguous there -- no staging
  const bool alldone = __syncthreads_and(threadIdx.x >= 64 || i0 + threadIdx.x >= a.n || sdone[threadIdx.x]);
  const void* fsrc = c == 0 ? (const void*)a.fuse.add_actor : c == 1 ? (const void*)a.fuse.add_ctr
                     : c == 3 ? (const void*)a.fuse.add_mem : c == 6 ? (const void*)a.fuse.rm_actor
                     : c == 7 ? (const void*)a.fuse.rm_ctr : (const void*)a.fuse.rm_mem;
  const uint32_t R = a.fuse.rows;
  if (a.fdone && alldone) {
    const uint32_t lo = sb[0], hi = sb[64];
    for (uint32_t j = lo + threadIdx.x; j < hi; j += kBlock) {
      uint32_t l = 0;  // last file whose base <= j
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1)
        if (sb[l + step] <= j) l += step;
      const uint32_t k = j - sb[l];
      const size_t idx = (size_t)(i0 + l) * R + k;
      if (synth) reinterpret_cast<uint32_t*>(dst[c])[j] = ob[l] + k;
      else if (wide) reinterpret_cast<unsigned long long*>(dst[c])[j] = reinterpret_cast<const unsigned long long*>(fsrc)[idx];
      else reinterpret_cast<uint32_t*>(dst[c])[j] = reinterpret_cast<const uint32_t*>(fsrc)[idx];
    }
    return;
  }
  if (threadIdx.x < 64) atomicMax(&tmax, sb[threadIdx.x + 1] - sb[threadIdx.x]);
  __syncthreads();
  const uint32_t rows = tmax;  // <= kTileMaxRows (the host checked every column's largest count)
  const size_t npad = a.tile.npad;
  const bool legacy = npad != 0;  // the other files' rows are in tile.col (else: stored directly)
  if (legacy) {
    for (uint32_t x = threadIdx.x; x < rows * 64; x += kBlock) {
      const size_t idx = (size_t)(x >> 6) * npad + i0 + (x & 63);
      if (sdone[x & 63]) continue;
      tile[x] = wide ? reinterpret_cast<const unsigned long long*>(a.tile.col[c])[idx]
                     : reinterpret_cast<const uint32_t*>(a.tile.col[c])[idx];
    }
  }
  if (a.fdone && rows) {
    // file-major rows: a file's ops are contiguous (x -> file x / rows, op x % rows)
    for (uint32_t x = threadIdx.x; x < rows * 64; x += kBlock) {
      const uint32_t l = x / rows, k = x - l * rows;
      if (!sdone[l] || k >= R) continue;
      const size_t idx = (size_t)(i0 + l) * R + k;
      tile[k * 64 + l] = synth ? (unsigned long long)(ob[l] + k)
                         : wide ? reinterpret_cast<const unsigned long long*>(fsrc)[idx]
                                : reinterpret_cast<const uint32_t*>(fsrc)[idx];
    }
  }
  __syncthreads();
  const uint32_t lo = sb[0], hi = sb[64];
  for (uint32_t j = lo + threadIdx.x; j < hi; j += kBlock) {
    uint32_t l = 0;  // last file whose base <= j
#pragma unroll
    for (uint32_t step = 32; step > 0; step >>= 1)
      if (sb[l + step] <= j) l += step;
    if (!legacy && !sdone[l]) continue;  // stored by the direct emit
    const unsigned long long v = tile[(j - sb[l]) * 64 + l];
    if (wide) reinterpret_cast<unsigned long long*>(dst[c])[j] = v;
    else reinterpret_cast<uint32_t*>(dst[c])[j] = (uint32_t)v;
  }
}

// ---------------------------------------------------------------------------------------
// Orswot fold
// ---------------------------------------------------------------------------------------
__global__ void k_ds_iota(uint32_t* v, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) v[i] = i;
}

__global__ void k_ds_gather_ctr(const uint32_t* perm, const unsigned long long* ctr,
                                unsigned long long* out, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) out[i] = ctr[perm[i]];
}

// applied(add k) = c_k > max(C0[a_k], max{c_j : j < k, a_j = a_k})  (crdts Orswot::apply:
// "if self.clock.get(&dot.actor) >= dot.counter { return }")
// perm null: the adds in their own order (run-contiguous actors, no sort)
__global__ void k_ds_applied(const uint32_t* keys, const uint32_t* perm,
                             const unsigned long long* ctr, const unsigned long long* excl,
                             const unsigned long long* clock, uint8_t* applied, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const unsigned long long c0 = clock[keys[i]];
    const unsigned long long prev = excl[i] > c0 ? excl[i] : c0;
    applied[perm ? perm[i] : i] = ctr[i] > prev;
  }
}

// flag |= 1 unless every actor's adds form one contiguous run: a run head stamps its actor's
// mark with this check's generation; a second head of the same actor finds the stamp.
// With mono (the pinned form): also the applied flags and exclusive maxima of runs whose counters
// strictly increase (load_ops order of a writer's own op files): the exclusive max of add i is
// then its predecessor's counter, so add i applies iff ctr > max(ctr[i - 1], C0[a]) (C0 = clock
// before the batch; ids past ccap are new actors, C0 = 0).  pub: pinned words -- [0] the emit's
// miss count copied from miss_src, [1] the contiguity flag, [2] set when a run does not
// strictly increase (then the fold takes the segmented scan); plain stores, zeroed by the host.
__global__ void k_ds_contig(const uint32_t* actor, uint32_t n, uint32_t* marks, uint32_t n_marks, uint32_t gen,
                            uint32_t* flag, const uint32_t* miss_src, uint32_t* pub, DsMono mono) {
  if (pub && blockIdx.x == 0 && threadIdx.x == 0) pub[0] = *miss_src;  // (the emit is done)
  bool bad = false, rise = true;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t a = actor[i];
    const bool head = i == 0 || actor[i - 1] != a;
    if (mono.ctr) {
      const unsigned long long c = mono.ctr[i], prev = head ? 0ull : mono.ctr[i - 1];
      if (!head && c <= prev) rise = false;
      const unsigned long long c0 = a < mono.ccap ? mono.clock[a] : 0ull;
      mono.excl[i] = prev;
      mono.applied[i] = c > (prev > c0 ? prev : c0);
    }
    if (!head) continue;
    if (a >= n_marks) { bad = true; continue; }
    bad |= atomicExch(marks + a, gen) == gen;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) {
    if (pub) pub[1] = 1u;
    else atomicOr(flag, 1u);
  }
  if (pub && __any(!rise) && (threadIdx.x & 63) == 0) pub[2] = 1u;
}

// clock[a] = max(clock[a], every counter of actor a in the batch), from the actor-sorted adds:
// the last add of each actor's run holds the run's max (exclusive max + its own), and writes it
// with a plain store (one writer per actor).  Per-add atomicMax on 4096 clock words serialised.
__global__ void k_ds_clock(const uint32_t* keys_sorted, const unsigned long long* ctr_sorted,
                           const unsigned long long* excl_max, unsigned long long* clock, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t a = keys_sorted[i];
    if (i + 1 < n && keys_sorted[i + 1] == a) continue;
    const unsigned long long m = ctr_sorted[i] > excl_max[i] ? ctr_sorted[i] : excl_max[i];
    if (m > clock[a]) clock[a] = m;
  }
}

__global__ void __launch_bounds__(kBlock) k_ds_add_pairs(DsTables t, DsOps o, const uint8_t* applied,
                                                         uint32_t n) {
  for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < n; k += gridDim.x * kBlock) {
    if (!applied[k]) continue;
    const uint32_t aid = o.add_actor[k];
    const unsigned long long c = o.add_ctr[k];
    for (uint32_t j = o.add_mbeg[k]; j < o.add_mbeg[k + 1]; j++) {
      const unsigned long long h = member_find(t, o.add_mem[j], true);
      if (h == kDsEmpty) continue;
      const unsigned long long b = pair_find(t, pair_key(h, aid), true);
      if (b != kDsEmpty) atomicMax(t.add + b, c);
    }
  }
}

// crdts Orswot::apply_rm: entry.reset_remove(clock) drops actor a when R[a] >= entry[a]
__global__ void __launch_bounds__(kBlock) k_ds_kill(DsTables t, const uint32_t* cbeg, const uint32_t* mbeg,
                                                    const uint32_t* c_actor,
                                                    const unsigned long long* c_ctr,
                                                    const unsigned long long* mem, uint32_t n) {
  for (uint32_t r = blockIdx.x * kBlock + threadIdx.x; r < n; r += gridDim.x * kBlock) {
    const uint32_t c0 = cbeg[r], c1 = cbeg[r + 1];
    if (c0 == c1) continue;
    for (uint32_t j = mbeg[r]; j < mbeg[r + 1]; j++) {
      const unsigned long long h = member_find(t, mem[j], false);
      if (h == kDsEmpty) continue;
      for (uint32_t e = c0; e < c1; e++) {
        const unsigned long long b = pair_find(t, pair_key(h, c_actor[e]), false);
        if (b != kDsEmpty) atomicMax(t.kill + b, c_ctr[e]);
      }
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_ds_finalize(DsTables t) {
  // per-lane counts over the grid-stride loop, summed per block at the end: two atomics per
  // block (same-address atomics serialise in L2, ~10 ns each; per-wave ones cost 0.2 ms at C3)
  const uint32_t cap = t.pmask + 1;
  uint32_t n_used = 0, n_live = 0;
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < cap; b += gridDim.x * kBlock) {
    if (t.pkey[b] == kDsEmpty) continue;
    n_used++;
    const unsigned long long c = t.cur[b], ad = t.add[b], kl = t.kill[b];
    unsigned long long v = c > ad ? c : ad;
    if (v != 0 && v <= kl) v = 0;
    if (v != c) t.cur[b] = v;
    if (ad) t.add[b] = 0;
    if (kl) t.kill[b] = 0;
    n_live += v != 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n_used += __shfl_xor(n_used, o);
    n_live += __shfl_xor(n_live, o);
  }
  __shared__ uint32_t part[2][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = n_live;
    part[1][threadIdx.x >> 6] = n_used;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t l = 0, u = 0;
    for (int w = 0; w < kBlock / 64; w++) {
      l += part[0][w];
      u += part[1][w];
    }
    // live[0] (live pairs) and live[1] (used slots) in one 64-bit add: same-address atomics
    // serialise in L2 (~60 ns each across XCDs), one per block instead of two
    if (l | u) atomicAdd(reinterpret_cast<unsigned long long*>(t.live), ((unsigned long long)u << 32) | l);
  }
}

// ---- partitioned fold (ce_dotset.h: DsPartArgs) ----------------------------------------
// The global kernels above cost ~3 random line touches per add (member probe, pair probe, the
// add slot's atomic) plus two full passes over the 4M-slot table (finalize); here the items are
// bucketed by partition first (two streaming passes), then each partition's 2048 keys and the
// counters / thresholds of its items meet in LDS, and only changed slots go back to HBM.
constexpr int kPartThreads = 1024;     // K1 (the 512-thread form: kDsPartThreadsSmall)
constexpr int kApplyThreads = 512;     // K4

// member handle of m when its first probe holds it (g = mkey[that bucket], read ahead of time
// for several items at once), else member_find
__device__ __forceinline__ unsigned long long member_handle(const DsTables& t, unsigned long long m,
                                                            unsigned long long g, bool insert) {
  if (g == m && m != kDsEmpty) return (uint32_t)mix64(m) & t.smask;
  return member_find(t, m, insert);
}

constexpr int kPartBatch = CE_PART_BATCH;  // items per lane whose loads are issued before any is used
static_assert(kDsPartChunk == kPartThreads * kPartBatch, "K1 walks its chunk in one trip");
static_assert(kDsPartChunkSmall == kDsPartThreadsSmall * kPartBatch, "K1 walks its chunk in one trip");

// K1 after its count: lh[p] (this block's items of partition p) -> the base of its reservation in
// p's run, one returning add per partition with items (64 contiguous counters per wave instruction)
// (block b reserves in sub-run b % kDsPartReps of every partition: a counter then takes
// ~blocks / 8 same-address adds -- one counter per partition took ~200, ~60 ns each across XCDs)
template <int T>
__device__ __forceinline__ void part_reserve(uint32_t* lh, uint32_t parts, uint32_t* pcnt) {
  __syncthreads();
  uint32_t* c = pcnt + (size_t)(blockIdx.x % kDsPartReps) * parts;
  for (uint32_t p = threadIdx.x; p < parts; p += T) {
    const uint32_t n = lh[p];
    if (n) lh[p] = atomicAdd(c + p, n);
  }
  __syncthreads();
}

// one item to its place in partition p's run (pos from the block's LDS cursor), or to the overflow
// list past the run's end
__device__ __forceinline__ void part_put(const DsPartArgs& a, int side, uint32_t p, uint32_t pos,
                                         unsigned long long key, unsigned long long v) {
  unsigned long long* dst;
  if (pos < a.cap[side]) {
    const uint32_t r = blockIdx.x % kDsPartReps;
    dst = a.items + 2ull * ((size_t)side * a.parts * kDsPartReps * a.cap[0] +
                            ((size_t)p * kDsPartReps + r) * a.cap[side] + pos);
  } else {
    const uint32_t o = atomicAdd(a.ovf_n + 2 * a.par + side, 1u);
    if (o >= a.ovf_cap[side]) {  // (sized for every item of the batch: not reached)
      atomicAdd(a.t.live + 2, 1u);
      return;
    }
    dst = a.ovf[side] + 2ull * o;
  }
  *reinterpret_cast<ulonglong2*>(dst) = make_ulonglong2(key, v);
}

template <int T>
__global__ void __launch_bounds__(T) k_ds_part_adds(DsPartArgs a) {
  extern __shared__ uint32_t lh[];  // [parts]: counts, then the block's cursors in every run
  for (uint32_t p = threadIdx.x; p < a.parts; p += T) lh[p] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.t.live[0] = 0;
    a.t.live[1] = 0;
    a.t.live[3] = 0;
    a.t.live[4] = 0;
  }
  __syncthreads();
  const uint32_t k1 = min(a.n_add, blockIdx.x * a.chunk + a.chunk);
  // an add with one member keeps its pair key and counter in registers; one with several leaves
  // its members' keys in akey for the write below
  uint32_t j0[kPartBatch], j1[kPartBatch], aid[kPartBatch];
  unsigned long long m[kPartBatch], g[kPartBatch], c[kPartBatch], key[kPartBatch];
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    const uint32_t k = blockIdx.x * a.chunk + threadIdx.x + q * T;
    j0[q] = j1[q] = 0;
    m[q] = g[q] = c[q] = 0;
    if (k < k1 && a.applied[k]) {
      j0[q] = a.o.add_mbeg[k];
      j1[q] = a.o.add_mbeg[k + 1];
      aid[q] = a.o.add_actor[k];
      c[q] = a.o.add_ctr[k];
      if (j1[q] == j0[q] + 1) {
        m[q] = a.o.add_mem[j0[q]];
        g[q] = a.t.mkey[(uint32_t)mix64(m[q]) & a.t.smask];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    key[q] = kDsEmpty;
    if (j1[q] == j0[q] + 1) {
      const unsigned long long h = member_handle(a.t, m[q], g[q], true);
      if (h != kDsEmpty) {
        key[q] = pair_key(h, aid[q]);
        atomicAdd(&lh[pair_part(a.t, key[q])], 1u);
      }
    } else {
      for (uint32_t j = j0[q]; j < j1[q]; j++) {
        const unsigned long long h = member_find(a.t, a.o.add_mem[j], true);
        const unsigned long long kj = h == kDsEmpty ? kDsEmpty : pair_key(h, aid[q]);
        a.akey[j] = kj;
        if (kj != kDsEmpty) atomicAdd(&lh[pair_part(a.t, kj)], 1u);
      }
    }
  }
  part_reserve<T>(lh, a.parts, a.pcnt);
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    if (j1[q] == j0[q] + 1) {
      if (key[q] == kDsEmpty) continue;
      const uint32_t p = pair_part(a.t, key[q]);
      part_put(a, 0, p, atomicAdd(&lh[p], 1u), key[q], c[q]);
    } else {
      for (uint32_t j = j0[q]; j < j1[q]; j++) {
        const unsigned long long kj = a.akey[j];
        if (kj == kDsEmpty) continue;
        const uint32_t p = pair_part(a.t, kj);
        part_put(a, 0, p, atomicAdd(&lh[p], 1u), kj, c[q]);
      }
    }
  }
}

// removal r kills (m, a_e) for every member m and clock entry e (k_ds_kill); a member absent after
// the adds has no pair to kill.  A removal with one member and one clock entry (one item) keeps it
// in registers; others leave their member handles in hk for the write below.
template <int T>
__global__ void __launch_bounds__(T) k_ds_part_kills(DsPartArgs a) {
  extern __shared__ uint32_t lh[];
  for (uint32_t p = threadIdx.x; p < a.parts; p += T) lh[p] = 0;
  __syncthreads();
  const uint32_t b = blockIdx.x;
  const DsKillSrc& x = a.ks[b < a.bk0 ? 0 : 1];
  const uint32_t r0 = (b < a.bk0 ? b : b - a.bk0) * a.kchunk;
  const uint32_t r1 = min(x.n, r0 + a.kchunk);
  uint32_t c0[kPartBatch], c1[kPartBatch], j0[kPartBatch], j1[kPartBatch];
  unsigned long long m[kPartBatch], g[kPartBatch], key[kPartBatch], v[kPartBatch];
  uint32_t ca[kPartBatch];
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    const uint32_t r = r0 + threadIdx.x + q * T;
    c0[q] = c1[q] = j0[q] = j1[q] = 0;
    m[q] = g[q] = v[q] = 0;
    ca[q] = 0;
    if (r < r1) {
      c0[q] = x.cbeg[r];
      c1[q] = x.cbeg[r + 1];
      j0[q] = x.mbeg[r];
      j1[q] = x.mbeg[r + 1];
      if (c0[q] == c1[q]) {  // an empty clock kills nothing
        j1[q] = j0[q];
      } else if (j1[q] == j0[q] + 1 && c1[q] == c0[q] + 1) {
        m[q] = x.mem[j0[q]];
        g[q] = a.t.mkey[(uint32_t)mix64(m[q]) & a.t.smask];
        ca[q] = x.c_actor[c0[q]];
        v[q] = x.c_ctr[c0[q]];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    key[q] = kDsEmpty;
    if (j1[q] == j0[q] + 1 && c1[q] == c0[q] + 1) {
      const unsigned long long h = member_handle(a.t, m[q], g[q], false);
      if (h != kDsEmpty) {
        key[q] = pair_key(h, ca[q]);
        atomicAdd(&lh[pair_part(a.t, key[q])], 1u);
      }
    } else {
      for (uint32_t j = j0[q]; j < j1[q]; j++) {
        const unsigned long long h = member_find(a.t, x.mem[j], false);
        x.hk[j] = h;
        if (h == kDsEmpty) continue;
        for (uint32_t e = c0[q]; e < c1[q]; e++) atomicAdd(&lh[pair_part(a.t, pair_key(h, x.c_actor[e]))], 1u);
      }
    }
  }
  part_reserve<T>(lh, a.parts, a.pcnt + (size_t)kDsPartReps * a.parts);
#pragma unroll
  for (int q = 0; q < kPartBatch; q++) {
    if (j1[q] == j0[q] + 1 && c1[q] == c0[q] + 1) {
      if (key[q] == kDsEmpty) continue;
      const uint32_t p = pair_part(a.t, key[q]);
      part_put(a, 1, p, atomicAdd(&lh[p], 1u), key[q], v[q]);
    } else {
      for (uint32_t j = j0[q]; j < j1[q]; j++) {
        const unsigned long long h = x.hk[j];
        if (h == kDsEmpty) continue;
        for (uint32_t e = c0[q]; e < c1[q]; e++) {
          const unsigned long long kj = pair_key(h, x.c_actor[e]);
          const uint32_t p = pair_part(a.t, kj);
          part_put(a, 1, p, atomicAdd(&lh[p], 1u), kj, x.c_ctr[e]);
        }
      }
    }
  }
}

// K4: partition p = blockIdx.x (+ k * gridDim.x).  Keys in LDS follow pair_find's probe order
// (start at mix64(key) mod the partition, wrap inside it), so a key inserted here sits where the
// global kernels look for it.  Then finalize (k_ds_finalize) of the touched slots only: an
// untouched slot's value is unchanged by it.  Every phase issues all of a lane's global loads
// before using any (the compiler does not overlap the trips of a loop: one round trip each).
constexpr int kApplySlotsPerLane = kDsPartSlots / kApplyThreads;
constexpr int kApplyItemBatch = 4;

__device__ __forceinline__ uint32_t lds_insert(unsigned long long* key, unsigned long long k) {
  constexpr uint32_t M = kDsPartSlots - 1;
  uint32_t h = (uint32_t)mix64(k) & M;
  for (uint32_t probe = 0; probe < kDsPartSlots; probe++) {
    const unsigned long long c = key[h];
    if (c == k) return h;
    if (c == kDsEmpty) {
      const unsigned long long prev = atomicCAS(&key[h], kDsEmpty, k);
      if (prev == kDsEmpty || prev == k) return h;
    }
    h = (h + 1) & M;
  }
  return ~0u;
}

__device__ __forceinline__ uint32_t lds_lookup(const unsigned long long* key, unsigned long long k) {
  constexpr uint32_t M = kDsPartSlots - 1;
  uint32_t h = (uint32_t)mix64(k) & M;
  for (uint32_t probe = 0; probe < kDsPartSlots; probe++) {
    const unsigned long long c = key[h];
    if (c == k) return h;
    if (c == kDsEmpty) return ~0u;
    h = (h + 1) & M;
  }
  return ~0u;
}

__global__ void __launch_bounds__(kApplyThreads) k_ds_part_apply(DsPartArgs a) {
  __shared__ unsigned long long key[kDsPartSlots], add[kDsPartSlots], kill[kDsPartSlots];
  __shared__ int part[3][kApplyThreads / 64];
  int dl = 0, du = 0, dm = 0;
  const uint32_t tid = threadIdx.x;
  // this fold's overflow counts (usually 0); the next fold's zeroed; live[5] = the items that
  // overflowed, for the host's run sizing
  const uint32_t no_a = min(a.ovf_n[2 * a.par], a.ovf_cap[0]), no_k = min(a.ovf_n[2 * a.par + 1], a.ovf_cap[1]);
  if (blockIdx.x == 0 && tid == 0) {
    a.ovf_n[2 * (a.par ^ 1)] = 0;
    a.ovf_n[2 * (a.par ^ 1) + 1] = 0;
    a.t.live[5] = no_a + no_k;
  }
  // a grid of a few workgroups per CU walks the partitions
  for (uint32_t p = blockIdx.x; p < a.parts; p += gridDim.x) {
    const size_t base = (size_t)p << kDsPartBits;
    unsigned long long k0[kApplySlotsPerLane];
#pragma unroll
    for (int q = 0; q < kApplySlotsPerLane; q++) k0[q] = a.t.pkey[base + tid + q * kApplyThreads];
#pragma unroll
    for (int q = 0; q < kApplySlotsPerLane; q++) {
      const uint32_t i = tid + q * kApplyThreads;
      key[i] = k0[q];
      add[i] = 0;
      kill[i] = 0;
    }
    __syncthreads();
    // adds: insert, max-merge the counter (the partition's run, then its overflowed items)
    // the partition's kDsPartReps sub-runs of each side, as one index space
    uint32_t pa_[kDsPartReps + 1], pk_[kDsPartReps + 1];
    pa_[0] = pk_[0] = 0;
#pragma unroll
    for (int r = 0; r < (int)kDsPartReps; r++) {
      pa_[r + 1] = pa_[r] + min(a.pcnt[(size_t)r * a.parts + p], a.cap[0]);
      pk_[r + 1] = pk_[r] + min(a.pcnt[(size_t)(kDsPartReps + r) * a.parts + p], a.cap[1]);
    }
    const uint32_t na_p = pa_[kDsPartReps], nk_p = pk_[kDsPartReps];
    const unsigned long long* ra = a.items + 2ull * ((size_t)p * kDsPartReps * a.cap[0]);
    auto at = [](const uint32_t* pre, uint32_t cap, uint32_t i) {  // item i's slot in the sub-runs
      uint32_t r = 0;
#pragma unroll
      for (int q = 1; q < (int)kDsPartReps; q++) r += i >= pre[q];
      return r * cap + (i - pre[r]);
    };
    for (uint32_t i0 = 0; i0 < na_p; i0 += kApplyThreads * kApplyItemBatch) {
      ulonglong2 it[kApplyItemBatch];
#pragma unroll
      for (int b = 0; b < kApplyItemBatch; b++) {
        const uint32_t i = i0 + tid + b * kApplyThreads;
        it[b] = i < na_p ? *reinterpret_cast<const ulonglong2*>(ra + 2ull * at(pa_, a.cap[0], i))
                         : make_ulonglong2(kDsEmpty, 0);
      }
#pragma unroll
      for (int b = 0; b < kApplyItemBatch; b++) {
        if (it[b].x == kDsEmpty) continue;
        const uint32_t h = lds_insert(key, it[b].x);
        if (h != ~0u) atomicMax(&add[h], it[b].y);
        else atomicAdd(a.t.live + 2, 1u);  // partition full (tables sized to <= 50% load)
      }
    }
    for (uint32_t i = tid; i < no_a; i += kApplyThreads) {
      const ulonglong2 it = *reinterpret_cast<const ulonglong2*>(a.ovf[0] + 2ull * i);
      if (pair_part(a.t, it.x) != p) continue;
      const uint32_t h = lds_insert(key, it.x);
      if (h != ~0u) atomicMax(&add[h], it.y);
      else atomicAdd(a.t.live + 2, 1u);
    }
    __syncthreads();
    // removals: thresholds of existing pairs
    const unsigned long long* rk =
        a.items + 2ull * ((size_t)a.parts * kDsPartReps * a.cap[0] + (size_t)p * kDsPartReps * a.cap[1]);
    for (uint32_t i0 = 0; i0 < nk_p; i0 += kApplyThreads * kApplyItemBatch) {
      ulonglong2 it[kApplyItemBatch];
#pragma unroll
      for (int b = 0; b < kApplyItemBatch; b++) {
        const uint32_t i = i0 + tid + b * kApplyThreads;
        it[b] = i < nk_p ? *reinterpret_cast<const ulonglong2*>(rk + 2ull * at(pk_, a.cap[1], i))
                         : make_ulonglong2(kDsEmpty, 0);
      }
#pragma unroll
      for (int b = 0; b < kApplyItemBatch; b++) {
        if (it[b].x == kDsEmpty) continue;
        const uint32_t h = lds_lookup(key, it[b].x);
        if (h != ~0u) atomicMax(&kill[h], it[b].y);
      }
    }
    for (uint32_t i = tid; i < no_k; i += kApplyThreads) {
      const ulonglong2 it = *reinterpret_cast<const ulonglong2*>(a.ovf[1] + 2ull * i);
      if (pair_part(a.t, it.x) != p) continue;
      const uint32_t h = lds_lookup(key, it.x);
      if (h != ~0u) atomicMax(&kill[h], it.y);
    }
    dm += (int)primary_used(a.t, p, a.parts);
    __syncthreads();
    if (tid < 2 * kDsPartReps)  // every lane has read the counts (barriers above): the next fold's are zero
      a.pcnt[(size_t)tid * a.parts + p] = 0;
    // finalize the touched slots: the current values they need, all loads first
    unsigned long long ad[kApplySlotsPerLane], kl[kApplySlotsPerLane], c[kApplySlotsPerLane];
    bool fresh[kApplySlotsPerLane];
#pragma unroll
    for (int q = 0; q < kApplySlotsPerLane; q++) {
      const uint32_t i = tid + q * kApplyThreads;
      ad[q] = add[i];
      kl[q] = kill[i];
      fresh[q] = k0[q] == kDsEmpty && key[i] != kDsEmpty;
      c[q] = 0;
      if (!fresh[q] && (ad[q] | kl[q])) c[q] = a.t.cur[base + i];
    }
#pragma unroll
    for (int q = 0; q < kApplySlotsPerLane; q++) {
      const uint32_t i = tid + q * kApplyThreads;
      if (fresh[q]) {
        a.t.pkey[base + i] = key[i];
        du++;
      }
      if (!(ad[q] | kl[q])) continue;
      unsigned long long v = c[q] > ad[q] ? c[q] : ad[q];
      if (v != 0 && v <= kl[q]) v = 0;
      if (v != c[q]) a.t.cur[base + i] = v;
      dl += (int)(v != 0) - (int)(c[q] != 0);
    }
    __syncthreads();  // the next partition reuses the LDS tables
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dl += __shfl_xor(dl, o);
    du += __shfl_xor(du, o);
    dm += __shfl_xor(dm, o);
  }
  if ((tid & 63) == 0) {
    part[0][tid >> 6] = dl;
    part[1][tid >> 6] = du;
    part[2][tid >> 6] = dm;
  }
  __syncthreads();
  if (tid == 0) {
    int l = 0, u = 0, mm = 0;
    for (int w = 0; w < kApplyThreads / 64; w++) {
      l += part[0][w];
      u += part[1][w];
      mm += part[2][w];
    }
    // live[0] (signed change of the live pairs) and live[1] (slots used) in one 64-bit add of
    // u 2^32 + l: the sum is exact whatever the order, so the words hold U 2^32 + L with L signed
    // -- read back as L = (int32) live[0], U = live[1] + (L < 0) (ds_settle)
    if (l | u)
      atomicAdd(reinterpret_cast<unsigned long long*>(a.t.live),
                ((unsigned long long)(uint32_t)u << 32) + (unsigned long long)(long long)l);
    if (mm) atomicAdd(a.t.live + 4, (uint32_t)mm);
  }
}

// the last block of a grid to finish copies words [0, pub.words) of pub.src (device counters the
// grid and the kernels before it produced) into pub.dst (the caller's pinned memory), so the host
// reads them after its next wait without a runtime copy; pub.done (zero between uses) counts blocks
struct DsPublish {
  const uint32_t* src;
  uint32_t* dst;
  uint32_t words;
  uint32_t* done;
};

// The last block of the grid copies pub.src[0..words) (counters earlier kernels produced) into
// pub.dst, with word any_word (>= 0) OR'ed with "some block of this grid had `some`".  Found in
// two levels: block b adds 1 (+ 1 << 16 when `some`) into done[1 + b % 8], the block completing
// its replica adds its replica's verdict into done[0] -- ~blocks / 8 same-address adds per word,
// ~60 ns each across XCDs, and the flag travels in the same atomics, so no block needs a fence
// (an agent-scope fence per block writes back its XCD's L2: ~20 us over 128 blocks).
// done[0..8] are zero between uses.
__device__ __forceinline__ void publish_last(const DsPublish& pub, bool some, int any_word) {
  if (!pub.dst) return;
  __shared__ bool last;
  __shared__ uint32_t any_all;
  const bool bsome = __syncthreads_or(some) != 0;
  if (threadIdx.x == 0) {
    const uint32_t r = blockIdx.x & 7u, reps = min(gridDim.x, 8u);
    const uint32_t in_r = (gridDim.x - r + 7u) / 8u;  // blocks counting into replica r
    last = false;
    const uint32_t o = atomicAdd(pub.done + 1 + r, 1u + (bsome ? 0x10000u : 0u));
    if ((o & 0xffffu) == in_r - 1) {
      pub.done[1 + r] = 0;
      const bool rsome = (o >> 16) != 0 || bsome;
      const uint32_t o2 = atomicAdd(pub.done, 1u + (rsome ? 0x10000u : 0u));
      last = (o2 & 0xffffu) == reps - 1;
      any_all = ((o2 >> 16) != 0 || rsome) ? 1u : 0u;
    }
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < pub.words) {
    uint32_t v = __hip_atomic_load(pub.src + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)threadIdx.x == any_word) v |= any_all;
    pub.dst[threadIdx.x] = v;
  }
  if (threadIdx.x == 0) *pub.done = 0;
}

__global__ void k_ds_deferred(const uint32_t* cbeg, const uint32_t* c_actor,
                              const unsigned long long* c_ctr, const unsigned long long* clock,
                              uint8_t* deferred, uint32_t n, uint32_t* any, DsPublish pub) {
  bool some = false;
  // four removals per lane and trip, their loads issued together (one-entry clocks: C3's); longer
  // clocks walk the rest
  constexpr int kQ = 4;
  for (uint32_t r0 = blockIdx.x * kBlock + threadIdx.x; r0 < n; r0 += gridDim.x * kBlock * kQ) {
    uint32_t e0[kQ], e1[kQ], ca[kQ];
    unsigned long long cc[kQ];
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      const uint32_t r = r0 + q * gridDim.x * kBlock;
      e0[q] = r < n ? cbeg[r] : 0u;
      e1[q] = r < n ? cbeg[r + 1] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      ca[q] = e0[q] < e1[q] ? c_actor[e0[q]] : 0u;
      cc[q] = e0[q] < e1[q] ? c_ctr[e0[q]] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < kQ; q++) {
      const uint32_t r = r0 + q * gridDim.x * kBlock;
      if (r >= n) continue;
      bool d = e0[q] < e1[q] && cc[q] > clock[ca[q]];
      for (uint32_t e = e0[q] + 1; e < e1[q] && !d; e++) d = c_ctr[e] > clock[c_actor[e]];
      deferred[r] = d;  // !(clock <= self.clock)
      some = some || d;
    }
  }
  // any[0] = 1 when some removal is deferred (one atomic per wave that has one; rare); a
  // publishing launch carries it in its last-block count instead (publish_last)
  if (any && !pub.dst) {
    const unsigned long long b = __ballot(some);
    if (b && (threadIdx.x & 63) == (uint32_t)(__ffsll(b) - 1)) atomicOr(any, 1u);
  }
  publish_last(pub, some, any && pub.dst ? (int)(any - pub.src) : -1);
}

__global__ void __launch_bounds__(kBlock) k_ds_put_other(DsTables t, const unsigned long long* member,
                                                         const uint32_t* actor,
                                                         const unsigned long long* value, uint32_t n,
                                                         int zero_counts) {
  // k_ds_merge_finalize (next on the stream) counts into live[0..1]
  if (zero_counts && blockIdx.x == 0 && threadIdx.x < 2) t.live[threadIdx.x] = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const unsigned long long h = member_find(t, member[i], true);
    if (h == kDsEmpty) continue;
    const unsigned long long b = pair_find(t, pair_key(h, actor[i]), true);
    if (b != kDsEmpty) t.oth[b] = value[i];
  }
}

// Orswot::merge per (member, actor): keep ours if equal to theirs (VClock::intersection) or
// newer than their clock (clone_without(other.clock)); take theirs if newer than our clock.
__global__ void k_ds_merge(DsTables t, const unsigned long long* clock, const unsigned long long* oclock) {
  const uint32_t cap = t.pmask + 1;
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < cap; b += gridDim.x * kBlock) {
    const unsigned long long key = t.pkey[b];
    if (key == kDsEmpty) continue;
    const uint32_t a = (uint32_t)(key & ((1u << kDsActorBits) - 1));
    const unsigned long long s = t.cur[b], o = t.oth[b];
    unsigned long long r = 0;
    if (s == o) r = s;
    if (s > oclock[a] && s > r) r = s;
    if (o > clock[a] && o > r) r = o;
    t.cur[b] = r;
    t.oth[b] = 0;
  }
}

// k_ds_merge then k_ds_finalize in one pass over the pair table (a state merge queued without a
// host round trip): the merged value goes through finalize's add / kill thresholds, the pair
// scratch is cleared, and live / used pairs are counted (live[0..1], zeroed by k_ds_put_other).
__global__ void __launch_bounds__(kBlock) k_ds_merge_finalize(DsTables t, const unsigned long long* clock,
                                                              const unsigned long long* oclock) {
  const uint32_t cap = t.pmask + 1;
  uint32_t n_used = 0, n_live = 0;
  for (uint32_t b = blockIdx.x * kBlock + threadIdx.x; b < cap; b += gridDim.x * kBlock) {
    const unsigned long long key = t.pkey[b];
    if (key == kDsEmpty) continue;
    n_used++;
    const uint32_t a = (uint32_t)(key & ((1u << kDsActorBits) - 1));
    const unsigned long long s = t.cur[b], o = t.oth[b], ad = t.add[b], kl = t.kill[b];
    unsigned long long r = 0;
    if (s == o) r = s;
    if (s > oclock[a] && s > r) r = s;
    if (o > clock[a] && o > r) r = o;
    unsigned long long v = r > ad ? r : ad;
    if (v != 0 && v <= kl) v = 0;
    if (v != s) t.cur[b] = v;
    if (o) t.oth[b] = 0;
    if (ad) t.add[b] = 0;
    if (kl) t.kill[b] = 0;
    n_live += v != 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n_used += __shfl_xor(n_used, o);
    n_live += __shfl_xor(n_live, o);
  }
  __shared__ uint32_t part[2][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = n_live;
    part[1][threadIdx.x >> 6] = n_used;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t l = 0, u = 0;
    for (int w = 0; w < kBlock / 64; w++) {
      l += part[0][w];
      u += part[1][w];
    }
    // live[0] (live pairs) and live[1] (used slots) in one 64-bit add: same-address atomics
    // serialise in L2 (~60 ns each across XCDs), one per block instead of two
    if (l | u) atomicAdd(reinterpret_cast<unsigned long long*>(t.live), ((unsigned long long)u << 32) | l);
  }
}

// k-way Orswot::merge of nf state files (read on the device) into the current state when no
// deferred removal exists on any side: one pass over the pair table instead of one per file.
// Per (member, actor) Orswot::merge keeps our value if theirs is equal (VClock::intersection) or
// their clock is below it (clone_without), and theirs if our clock is below it (crdts Orswot::merge).
// Every state's entry values are <= its own clock, so of two different values at most the larger
// can survive a merge (the smaller is covered by the larger's clock); folding the merges in file
// order therefore keeps M = the largest value among ours and the files' iff every source that does
// not hold exactly M has a clock below it: M > C_Y[a] -- a condition independent of the order.
// k_ds_kput: pairs inserted, oth = max over the files; k_ds_khold: bit f of hold = file f holds
// that max; k_ds_kfinal: the test above, then finalize's add / kill as k_ds_merge_finalize.
// (sources by value, kMergeInline files per launch: an uploaded descriptor array was a runtime copy)
constexpr uint32_t kMergeInline = 16;
constexpr uint32_t kSlotOwner = 0x80000000u;  // DsMergeSrc.slot: this row inserted the pair
// the k-way merge's live / used / member counts: each block of its final pass adds into one of
// kLiveReps replicas (t.live[16 + 16 r ..], 64 B apart: same-address atomics serialise in L2, one
// chain per replica instead of one for the grid), k_ds_kclock sums them into live[0], [1], [4]
constexpr uint32_t kLiveReps = 16;
__device__ __forceinline__ void kmerge_count(const DsTables& t, uint32_t block, uint32_t l, uint32_t u, uint32_t mm) {
  uint32_t* r = t.live + 16 + 16 * (block % kLiveReps);
  if (l | u) atomicAdd(reinterpret_cast<unsigned long long*>(r), ((unsigned long long)u << 32) | l);
  if (mm) atomicAdd(r + 2, mm);
}
struct DsMergeSrcs {
  DsMergeSrc f[kMergeInline];
  uint32_t f0;  // the first file's index in the merge (its hold bit)
  uint32_t fresh;  // the table held no pair before the merge: every cur is 0 (not read)
  const uint32_t* go;  // optional: nothing happens unless *go (a merge queued before the host
                       // knows that every file was read on the device, ds_merge_states_device)
};

__device__ __forceinline__ bool kmerge_off(const uint32_t* go) {
  return go && *reinterpret_cast<volatile const uint32_t*>(go) == 0;
}
__device__ __forceinline__ uint32_t kmerge_n(const DsMergeSrc& x) {
  return x.n_dev ? x.n_dev[1] + x.n_dev[2] : x.n;
}

__global__ void __launch_bounds__(kBlock) k_ds_kput(DsTables t, DsMergeSrcs src) {
  if (kmerge_off(src.go)) return;
  const DsMergeSrc x = src.f[blockIdx.y];
  if (src.f0 == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2) t.live[threadIdx.x] = 0;  // k_ds_kfinal counts
  if (src.f0 == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 2) t.live[4] = 0;
  if (src.f0 == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 16 * kLiveReps) t.live[16 + threadIdx.x] = 0;
  const uint32_t n = kmerge_n(x);
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const unsigned long long h = member_find(t, x.member[i], true);
    bool ins = false;
    const unsigned long long b = h == kDsEmpty ? kDsEmpty : pair_find_ins(t, pair_key(h, x.actor[i]), &ins);
    if (b != kDsEmpty) atomicMax(&t.oth[b], x.value[i]);
    // the slot, bit 31 = this row inserted the pair (its owner for k_ds_kfinal_rows)
    if (x.slot) x.slot[i] = b == kDsEmpty ? ~0u : (uint32_t)b | (ins ? kSlotOwner : 0u);
  }
}

// H: the hold word (u32 when the merge has at most 32 sources: half the bytes of k_ds_kfinal's read)
template <typename H>
__global__ void __launch_bounds__(kBlock) k_ds_khold(DsTables t, DsMergeSrcs src, H* hold) {
  if (kmerge_off(src.go)) return;
  const DsMergeSrc x = src.f[blockIdx.y];
  const uint32_t fb = src.f0 + blockIdx.y;
  const uint32_t n = kmerge_n(x);
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    unsigned long long b;
    if (x.slot) {  // recorded by k_ds_kput: no second probe of the member and pair tables
      const uint32_t r = x.slot[i];
      if (r == ~0u) continue;
      b = r & ~kSlotOwner;
    } else {
      const unsigned long long h = member_find(t, x.member[i], false);
      if (h == kDsEmpty) continue;
      b = pair_find(t, pair_key(h, x.actor[i]), false);
      if (b == kDsEmpty) continue;
    }
    const unsigned long long c = src.fresh ? 0ull : t.cur[b], o = t.oth[b];
    if (x.value[i] == (c > o ? c : o)) atomicOr(&hold[b], (H)1 << fb);
  }
}

// oclocks: the files' dense clocks actor-major, oclocks[a * ostride + f] (ostride a multiple of 8
// >= nf, the padding zero): a slot's first eight files' clocks are one 64-byte line, four 16-byte
// loads (file-major, eight gathers from lines 32 KiB apart took ~70 us at C3's 8 state files)
template <typename H>
__global__ void __launch_bounds__(kBlock) k_ds_kfinal(DsTables t, const unsigned long long* clock,
                                                      const unsigned long long* oclocks, uint32_t ostride,
                                                      uint32_t nf, H* hold, const uint32_t* go, uint32_t fresh) {
  if (kmerge_off(go)) return;
  const uint32_t cap = t.pmask + 1;
  uint32_t n_used = 0, n_live = 0, n_mem = primary_used(t, blockIdx.x, gridDim.x);
  // kKQ slots per lane and trip, every load of a trip issued before any is used
  constexpr int kKQ = 4;
  for (uint32_t b0 = blockIdx.x * kBlock * kKQ + threadIdx.x; b0 < cap; b0 += gridDim.x * kBlock * kKQ) {
    unsigned long long key[kKQ], s[kKQ], o[kKQ], hm[kKQ];
#pragma unroll
    for (int q = 0; q < kKQ; q++) key[q] = b0 + q * kBlock < cap ? t.pkey[b0 + q * kBlock] : kDsEmpty;
#pragma unroll
    for (int q = 0; q < kKQ; q++) {
      s[q] = o[q] = hm[q] = 0;
      if (key[q] == kDsEmpty) continue;
      // (add / kill are zero here: every fold's finalize clears what it set, so a state merge never
      // meets a batch's scratch -- not read, 64 MB less per pass at C3)
      s[q] = fresh ? 0ull : t.cur[b0 + q * kBlock];
      o[q] = t.oth[b0 + q * kBlock];
      hm[q] = hold[b0 + q * kBlock];
    }
    // the clocks the rule reads: ours and those of the first kKF files not holding the max, one
    // batch of loads for every slot of the trip (a loop over the files waits on each in turn)
    constexpr int kKF = 8;
    unsigned long long ck[kKQ], oc[kKQ][kKF];
#pragma unroll
    for (int q = 0; q < kKQ; q++) {
      const uint32_t a = (uint32_t)(key[q] & ((1u << kDsActorBits) - 1));
      ck[q] = key[q] != kDsEmpty ? clock[a] : 0ull;
      const uint4* op = reinterpret_cast<const uint4*>(oclocks + (size_t)a * ostride);
#pragma unroll
      for (int i = 0; i < kKF / 2; i++) {
        const uint4 w = key[q] != kDsEmpty && (uint32_t)(2 * i) < nf ? op[i] : make_uint4(0, 0, 0, 0);
        oc[q][2 * i] = ((unsigned long long)w.y << 32) | w.x;
        oc[q][2 * i + 1] = ((unsigned long long)w.w << 32) | w.z;
      }
#pragma unroll
      for (int f = 0; f < kKF; f++)
        if ((hm[q] >> f) & 1ull) oc[q][f] = 0ull;  // a holder does not kill (m > 0)
    }
#pragma unroll
    for (int q = 0; q < kKQ; q++) {
      if (key[q] == kDsEmpty) continue;
      const uint32_t b = b0 + q * kBlock;
      n_used++;
      const uint32_t a = (uint32_t)(key[q] & ((1u << kDsActorBits) - 1));
      const unsigned long long m = s[q] > o[q] ? s[q] : o[q];
      bool keep = m != 0 && (s[q] == m || m > ck[q]);
#pragma unroll
      for (int f = 0; f < kKF; f++) keep = keep && m > oc[q][f];  // (0 for a holder: m > 0)
      for (uint32_t f = kKF; f < nf && keep; f++)
        if (!((hm[q] >> f) & 1ull)) keep = m > oclocks[(size_t)a * ostride + f];
      const unsigned long long v = keep ? m : 0ull;
      if (v != s[q]) t.cur[b] = v;
      if (o[q]) t.oth[b] = 0;
      if (hm[q]) hold[b] = 0;
      n_live += v != 0;
    }
  }
#pragma unroll
  for (int q = 32; q > 0; q >>= 1) {
    n_used += __shfl_xor(n_used, q);
    n_live += __shfl_xor(n_live, q);
    n_mem += __shfl_xor(n_mem, q);
  }
  __shared__ uint32_t part[3][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = n_live;
    part[1][threadIdx.x >> 6] = n_used;
    part[2][threadIdx.x >> 6] = n_mem;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t l = 0, u = 0, mm = 0;
    for (int w = 0; w < kBlock / 64; w++) {
      l += part[0][w];
      u += part[1][w];
      mm += part[2][w];
    }
    // live[0] (live pairs) and live[1] (used slots) in one 64-bit add: same-address atomics
    // serialise in L2 (~60 ns each across XCDs), one per block instead of two
    kmerge_count(t, blockIdx.x, l, u, mm);  // (replicas zeroed by k_ds_kput)
  }
}

// k_ds_kfinal over the merge's rows instead of the table's slots, for a merge into an empty table
// (fresh: every used slot was inserted by exactly one row, its owner -- k_ds_kput's slot bit 31):
// the owner row applies the rule to its slot (the current value is 0), so the pass reads the rows'
// slots and the touched slots' words, not the whole table's keys (C3: 0.41M rows, 4M slots).
// Grid (x, y) as k_ds_kput's, sources y of this launch (f0 + y); the primary member table's used
// slots are counted in slices over every block of every launch (live[4]).
template <typename H>
__global__ void __launch_bounds__(kBlock) k_ds_kfinal_rows(DsTables t, DsMergeSrcs src, const unsigned long long* clock,
                                                           const unsigned long long* oclocks, uint32_t ostride,
                                                           uint32_t nf, H* hold, uint32_t blocks_total) {
  if (kmerge_off(src.go)) return;
  const DsMergeSrc x = src.f[blockIdx.y];
  const uint32_t n = kmerge_n(x);
  const uint32_t bl = (src.f0 + blockIdx.y) * gridDim.x + blockIdx.x;  // this block among all
  uint32_t n_used = 0, n_live = 0, n_mem = primary_used(t, bl, blocks_total);
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t r = x.slot[i];
    if (r == ~0u || !(r & kSlotOwner)) continue;
    const uint32_t b = r & ~kSlotOwner;
    const unsigned long long key = t.pkey[b], m = t.oth[b], hm = hold[b];
    const uint32_t a = (uint32_t)(key & ((1u << kDsActorBits) - 1));
    const unsigned long long ck = clock[a];
    const uint4* op = reinterpret_cast<const uint4*>(oclocks + (size_t)a * ostride);
    constexpr int kKF = 8;
    unsigned long long oc[kKF];
#pragma unroll
    for (int q = 0; q < kKF / 2; q++) {
      const uint4 w = (uint32_t)(2 * q) < nf ? op[q] : make_uint4(0, 0, 0, 0);
      oc[2 * q] = ((unsigned long long)w.y << 32) | w.x;
      oc[2 * q + 1] = ((unsigned long long)w.w << 32) | w.z;
    }
    n_used++;
    bool keep = m != 0 && m > ck;  // (the current value is 0: "ours" is never the max)
#pragma unroll
    for (int f = 0; f < kKF; f++) keep = keep && (((hm >> f) & 1ull) || m > oc[f]);
    for (uint32_t f = kKF; f < nf && keep; f++)
      if (!((hm >> f) & 1ull)) keep = m > oclocks[(size_t)a * ostride + f];
    if (keep) t.cur[b] = m;
    t.oth[b] = 0;
    if (hm) hold[b] = 0;
    n_live += keep;
  }
#pragma unroll
  for (int q = 32; q > 0; q >>= 1) {
    n_used += __shfl_xor(n_used, q);
    n_live += __shfl_xor(n_live, q);
    n_mem += __shfl_xor(n_mem, q);
  }
  __shared__ uint32_t part[3][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = n_live;
    part[1][threadIdx.x >> 6] = n_used;
    part[2][threadIdx.x >> 6] = n_mem;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t l = 0, u = 0, mm = 0;
    for (int w = 0; w < kBlock / 64; w++) {
      l += part[0][w];
      u += part[1][w];
      mm += part[2][w];
    }
    kmerge_count(t, bl, l, u, mm);
  }
}

// clock = max(clock, every file's clock)
// (pub_dst: the k-way merge's live counters, final since k_ds_kfinal, into the caller's pinned memory)
__global__ void k_ds_kclock(unsigned long long* clock, const unsigned long long* oclocks, uint32_t ccap,
                            uint32_t ostride, uint32_t nf, const uint32_t* pub_src, uint32_t* pub_dst,
                            uint32_t pub_words, const uint32_t* go) {
  if (kmerge_off(go)) return;
  if (blockIdx.x == 0) {
    // the final pass's replicated counts summed into live[0], [1], [4] (pub_src = t.live), then
    // live[0..pub_words) into the caller's pinned memory
    uint32_t* live = const_cast<uint32_t*>(pub_src);
    const uint32_t w = threadIdx.x;
    if (w == 0 || w == 1 || w == 4) {  // replica words 0, 1, 2
      uint32_t v = 0;
      for (uint32_t r = 0; r < kLiveReps; r++) v += live[16 + 16 * r + (w == 4 ? 2u : w)];
      live[w] = v;
      if (pub_dst && w < pub_words) pub_dst[w] = v;
    } else if (pub_dst && w < pub_words) {
      pub_dst[w] = pub_src[w];
    }
  }
  for (uint32_t a = blockIdx.x * kBlock + threadIdx.x; a < ccap; a += gridDim.x * kBlock) {
    unsigned long long v = clock[a];
    for (uint32_t f = 0; f < nf; f++) {
      const unsigned long long w = oclocks[(size_t)a * ostride + f];
      v = w > v ? w : v;
    }
    clock[a] = v;
  }
}

// live pairs -> (member, actor id, value) columns, in no particular order (the writer sorts).
// A block owns a contiguous run of slots and walks it in 2048-slot sub-ranges, one reservation
// (a same-address atomic) per sub-range: 2048 over C3's 4M-slot table (16K reservations, one per
// 256 slots, cost ~0.2 ms: same-address atomics serialise in L2).  n_out[2..3]:
// the largest live member (the writer sorts only its significant bits), per-block maxima through
// bmax and k_ds_collect_max.
__global__ void __launch_bounds__(kBlock) k_ds_collect(DsTables t, unsigned long long* member, uint32_t* actor,
                                                       unsigned long long* value, uint32_t* n_out,
                                                       unsigned long long* bmax) {
  // one pass: a sub-range's live pairs are staged in LDS (kCQ slots per lane, every load of the
  // trip issued first), the sub-range reserves its output slice with one atomic, then the staged
  // columns go out with coalesced stores
  constexpr int kCQ = 8;
  constexpr uint32_t kSub = kBlock * kCQ;
  __shared__ unsigned long long sm[kSub], sv[kSub];
  __shared__ uint32_t sa[kSub];
  __shared__ uint32_t lcount, base;
  __shared__ unsigned long long lmax[kBlock / 64];
  const uint32_t cap = t.pmask + 1;
  const uint32_t per = (cap + gridDim.x - 1) / gridDim.x;
  const uint32_t r0 = min(cap, blockIdx.x * per), r1 = min(cap, r0 + per);
  unsigned long long mx = 0;
  for (uint32_t s0 = r0; s0 < r1; s0 += kSub) {
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    const uint32_t b0 = s0 + threadIdx.x;
    unsigned long long key[kCQ], v[kCQ], m[kCQ];
#pragma unroll
    for (int q = 0; q < kCQ; q++) key[q] = b0 + q * kBlock < r1 ? t.pkey[b0 + q * kBlock] : kDsEmpty;
#pragma unroll
    for (int q = 0; q < kCQ; q++) v[q] = key[q] != kDsEmpty ? t.cur[b0 + q * kBlock] : 0ull;
#pragma unroll
    for (int q = 0; q < kCQ; q++) m[q] = v[q] ? member_of(t, key[q] >> kDsActorBits) : 0ull;
#pragma unroll
    for (int q = 0; q < kCQ; q++) {
      if (v[q] == 0) continue;
      const uint32_t idx = atomicAdd(&lcount, 1u);
      sm[idx] = m[q];
      sa[idx] = (uint32_t)(key[q] & ((1u << kDsActorBits) - 1));
      sv[idx] = v[q];
      mx = m[q] > mx ? m[q] : mx;
    }
    __syncthreads();
    const uint32_t nl = lcount;
    if (threadIdx.x == 0) base = nl ? atomicAdd(n_out, nl) : 0u;
    __syncthreads();
    const uint32_t o = base;
    for (uint32_t i = threadIdx.x; i < nl; i += kBlock) {
      member[o + i] = sm[i];
      actor[o + i] = sa[i];
      value[o + i] = sv[i];
    }
    __syncthreads();  // the staging is reused by the next sub-range
  }
  mx = wave_max64(mx);
  if ((threadIdx.x & 63) == 0) lmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long mm = 0;
    for (int w = 0; w < kBlock / 64; w++) mm = lmax[w] > mm ? lmax[w] : mm;
    bmax[blockIdx.x] = mm;
  }
}

// ... and the results straight into the caller's pinned memory (host_out: [0] count, [2..3] the
// largest member; extra: one more device range copied alongside, the compaction's clock), then the
// output counter back to zero for the next collect: no runtime fill or copy around the pair
__global__ void __launch_bounds__(kBlock) k_ds_collect_max(const unsigned long long* bmax, uint32_t nb, uint32_t* n_out,
                                                           uint32_t* host_out, unsigned long long* extra_dst,
                                                           const unsigned long long* extra_src, uint32_t extra_words) {
  __shared__ unsigned long long lmax[kBlock / 64];
  unsigned long long mx = 0;
  for (uint32_t i = threadIdx.x; i < nb; i += kBlock) mx = bmax[i] > mx ? bmax[i] : mx;
  mx = wave_max64(mx);
  if ((threadIdx.x & 63) == 0) lmax[threadIdx.x >> 6] = mx;
  for (uint32_t i = threadIdx.x; i < extra_words; i += kBlock) extra_dst[i] = extra_src[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int w = 0; w < kBlock / 64; w++) m = lmax[w] > m ? lmax[w] : m;
    n_out[2] = (uint32_t)m;
    n_out[3] = (uint32_t)(m >> 32);
    if (host_out) {
      host_out[0] = n_out[0];
      host_out[2] = (uint32_t)m;
      host_out[3] = (uint32_t)(m >> 32);
      n_out[0] = 0;
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_ds_reinsert(DsTables t, const unsigned long long* member,
                                                        const uint32_t* actor,
                                                        const unsigned long long* value, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const unsigned long long h = member_find(t, member[i], true);
    if (h == kDsEmpty) continue;
    const unsigned long long b = pair_find(t, pair_key(h, actor[i]), true);
    if (b != kDsEmpty) t.cur[b] = value[i];
  }
}

__global__ void k_ds_gather_entries(const uint32_t* perm, const uint32_t* actor_in,
                                    const unsigned long long* value_in, uint32_t* actor_out,
                                    unsigned long long* value_out, uint32_t n) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    actor_out[i] = actor_in[perm[i]];
    value_out[i] = value_in[perm[i]];
  }
}

// ---------------------------------------------------------------------------------------
// MVReg: survivors = maximal clocks, one round per survivor
// ---------------------------------------------------------------------------------------
__global__ void k_mv_prep(MvArgs a) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += gridDim.x * kBlock) {
    unsigned long long hi = 0, lo = 0;
    for (uint32_t e = a.cbeg[i]; e < a.cbeg[i + 1]; e++) {
      const unsigned long long c = a.c_ctr[e];
      lo += c;
      hi += lo < c;
    }
    a.sum_hi[i] = hi;
    a.sum_lo[i] = lo;
    a.alive[i] = a.cbeg[i + 1] > a.cbeg[i];  // MVReg::apply ignores an empty clock
  }
}

struct MvKey {
  unsigned long long hi, lo, prio;
  uint32_t idx;
};

__device__ __forceinline__ bool mv_better(const MvKey& x, const MvKey& y) {
  if (x.idx == 0xffffffffu) return false;
  if (y.idx == 0xffffffffu) return true;
  if (x.hi != y.hi) return x.hi > y.hi;
  if (x.lo != y.lo) return x.lo > y.lo;
  return x.prio > y.prio;
}

__device__ MvKey mv_block_reduce(MvKey k) {
  __shared__ unsigned long long sh[kBlock], sl[kBlock], sp[kBlock];
  __shared__ uint32_t si[kBlock];
  sh[threadIdx.x] = k.hi;
  sl[threadIdx.x] = k.lo;
  sp[threadIdx.x] = k.prio;
  si[threadIdx.x] = k.idx;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      MvKey x{sh[threadIdx.x], sl[threadIdx.x], sp[threadIdx.x], si[threadIdx.x]};
      MvKey y{sh[threadIdx.x + w], sl[threadIdx.x + w], sp[threadIdx.x + w], si[threadIdx.x + w]};
      if (mv_better(y, x)) {
        sh[threadIdx.x] = y.hi;
        sl[threadIdx.x] = y.lo;
        sp[threadIdx.x] = y.prio;
        si[threadIdx.x] = y.idx;
      }
    }
    __syncthreads();
  }
  return MvKey{sh[0], sl[0], sp[0], si[0]};
}

__global__ void __launch_bounds__(kBlock) k_mv_argmax(MvArgs a) {
  MvKey best{0, 0, 0, 0xffffffffu};
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += gridDim.x * kBlock) {
    if (!a.alive[i]) continue;
    MvKey k{a.sum_hi[i], a.sum_lo[i], a.later_wins ? i : (unsigned long long)(a.n - 1 - i), i};
    if (mv_better(k, best)) best = k;
  }
  best = mv_block_reduce(best);
  if (threadIdx.x == 0) {
    a.blk[4 * blockIdx.x + 0] = best.hi;
    a.blk[4 * blockIdx.x + 1] = best.lo;
    a.blk[4 * blockIdx.x + 2] = best.prio;
    a.blk[4 * blockIdx.x + 3] = best.idx;
  }
}

__global__ void __launch_bounds__(kBlock) k_mv_final(MvArgs a) {
  MvKey best{0, 0, 0, 0xffffffffu};
  for (uint32_t b = threadIdx.x; b < a.n_blk; b += kBlock) {
    MvKey k{a.blk[4 * b], a.blk[4 * b + 1], a.blk[4 * b + 2], (uint32_t)a.blk[4 * b + 3]};
    if (mv_better(k, best)) best = k;
  }
  best = mv_block_reduce(best);
  if (threadIdx.x == 0) a.win[0] = best.idx;
  if (best.idx == 0xffffffffu) return;
  // winner clock -> dense
  for (uint32_t e = a.cbeg[best.idx] + threadIdx.x; e < a.cbeg[best.idx + 1]; e += kBlock)
    a.wclock[a.c_actor[e]] = a.c_ctr[e];
}

// candidates whose clock is <= the winner's (equal included) are dominated
__global__ void k_mv_kill(MvArgs a) {
  const uint32_t w = a.win[0];
  if (w == 0xffffffffu) return;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < a.n; i += gridDim.x * kBlock) {
    if (!a.alive[i]) continue;
    bool le = true;
    for (uint32_t e = a.cbeg[i]; e < a.cbeg[i + 1] && le; e++) le = a.c_ctr[e] <= a.wclock[a.c_actor[e]];
    if (le) a.alive[i] = 0;
  }
}

__global__ void k_mv_clear(MvArgs a) {
  const uint32_t w = a.win[0];
  if (w == 0xffffffffu) return;
  for (uint32_t e = a.cbeg[w] + threadIdx.x; e < a.cbeg[w + 1]; e += kBlock) a.wclock[a.c_actor[e]] = 0;
}

}  // namespace

namespace {
struct MaxOp {
  __host__ __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a > b ? a : b;
  }
};
}  // namespace

// the stable pair sorts: the hand-written LSD radix sort of ce_ser_sort.hip (no hipCUB)
hipError_t ds_sort_pairs_u32(void* tmp, size_t& tb, const uint32_t* kin, uint32_t* kout,
                             const uint32_t* vin, uint32_t* vout, uint32_t n, int bits, hipStream_t s) {
  return sort_pairs_u32(tmp, tb, kin, kout, vin, vout, n, bits, s);
}

hipError_t ds_sort_pairs_u64(void* tmp, size_t& tb, const unsigned long long* kin,
                             unsigned long long* kout, const uint32_t* vin, uint32_t* vout,
                             uint32_t n, hipStream_t s) {
  return sort_pairs_u64(tmp, tb, kin, kout, vin, vout, n, 64, s);
}

// ds_excl_max_by_key / ds_excl_sum_u32: ce_scan.hip (no hipCUB: its scans query the device
// properties on the host at every call)

// One block after the count pass and its scan, so the host reads everything the emit's sizing
// needs in one download: out[0..kCntN) column totals (last base + last count - first base),
// out[8..8+kCntN) the largest per-file count of each column (k_ds_count's counters[8..]),
// out[13..16) the status summary: files not OK, files left to the host envelope parser, files
// left to the host op decoder; out[16] the first file not OK (0xffffffff: none); out[17..19) the
// version gate's flags (gate_flags, when given); then clear8[0..8) = 0 (the emit's counters)
__global__ void __launch_bounds__(1024) k_ds_col_totals(const uint32_t* cnt, const uint32_t* bases, uint32_t n,
                                                        const uint32_t* maxima, const uint32_t* bpart, uint32_t nb,
                                                        const int32_t* status,
                                                        const uint32_t* gate_flags, uint32_t* clear8, uint32_t* out,
                                                        const unsigned long long* nn_src, uint32_t nn_m,
                                                        unsigned long long* nn_dst) {
  // the version gate's next versions per writer too (out and nn_dst: the caller's pinned memory)
  for (uint32_t i = threadIdx.x; nn_dst && i < nn_m; i += blockDim.x) nn_dst[i] = nn_src[i];
  __shared__ uint32_t acc[4], pmax[kCntN + 1];
  const uint32_t k = threadIdx.x;
  if (k < 3) acc[k] = 0;
  if (k == 3) acc[3] = 0xffffffffu;
  if (k <= kCntN) pmax[k] = 0;
  __syncthreads();
  if (bpart) {  // the count pass's per-block maxima, decoded-file counts and status summaries
    uint32_t m[kCntN + 1] = {0, 0, 0, 0, 0, 0};
    uint32_t bad = 0, hp = 0, hd = 0, first = 0xffffffffu;
    for (uint32_t b = k; b < nb; b += blockDim.x) {
      const uint32_t* r = bpart + kDsCountPart * b;
#pragma unroll
      for (int j = 0; j < kCntN; j++) m[j] = max(m[j], r[j]);
      m[kCntN] += r[5];
      bad += r[8];
      hp += r[9];
      hd += r[10];
      first = min(first, r[11]);
    }
#pragma unroll
    for (int j = 0; j < kCntN; j++)
      if (m[j]) atomicMax(&pmax[j], m[j]);
    if (m[kCntN]) atomicAdd(&pmax[kCntN], m[kCntN]);
    if (bad) {
      atomicAdd(&acc[0], bad);
      if (hp) atomicAdd(&acc[1], hp);
      if (hd) atomicAdd(&acc[2], hd);
      atomicMin(&acc[3], first);
    }
  }
  __syncthreads();
  if (k < kCntN) {
    const size_t c0 = (size_t)k * n, cl = c0 + n - 1;
    out[k] = bases[cl] + cnt[cl] - bases[c0];
    out[8 + k] = bpart ? pmax[k] : maxima[k];
  }
  if (k == 5) out[19] = bpart ? pmax[kCntN] : clear8 ? clear8[5] : 0u;  // files the open decoded
  if (gate_flags && k < 2) out[17 + k] = gate_flags[k];
  __syncthreads();
  if (clear8 && k < 8) clear8[k] = 0;  // the emit's counters (after the maxima above were read)
  uint32_t bad = 0, hp = 0, hd = 0, first = 0xffffffffu;
  // (without bpart) 16 statuses per lane in flight per trip
  constexpr int kSt = 16;
  for (uint32_t i0 = k; !bpart && i0 < n; i0 += kSt * blockDim.x) {
    int32_t v[kSt];
#pragma unroll
    for (int q = 0; q < kSt; q++) {
      const uint32_t i = i0 + q * blockDim.x;
      v[q] = i < n ? status[i] : CE_OK;
    }
#pragma unroll
    for (int q = 0; q < kSt; q++) {
      const int32_t st = v[q];
      if (st != CE_OK) {
        bad++;
        hp += st == kStatusHostParse;
        hd += st == kStatusHostDecode;
        first = min(first, i0 + q * blockDim.x);
      }
    }
  }
  if (bad) {
    atomicAdd(&acc[0], bad);
    if (hp) atomicAdd(&acc[1], hp);
    if (hd) atomicAdd(&acc[2], hd);
    atomicMin(&acc[3], first);
  }
  __syncthreads();
  if (k < 4) out[13 + k] = acc[k];
}

hipError_t launch_ds_col_totals(hipStream_t s, const uint32_t* cnt, const uint32_t* bases, uint32_t n,
                                const uint32_t* maxima, const uint32_t* bpart, uint32_t nb,
                                const int32_t* status, const uint32_t* gate_flags,
                                uint32_t* clear8, uint32_t* out, const unsigned long long* nn_src, uint32_t nn_m,
                                unsigned long long* nn_dst) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_col_totals, dim3(1), dim3(1024), 0, s, cnt, bases, n, maxima, bpart, nb, status, gate_flags,
                     clear8, out, nn_src, nn_m, nn_dst);
  return hipGetLastError();
}

// up to three u32 stores with by-value data (small patches without a host staging buffer)
__global__ void k_ds_set3(uint32_t* p0, uint32_t v0, uint32_t* p1, uint32_t v1, uint32_t* p2, uint32_t v2) {
  if (threadIdx.x == 0 && p0) *p0 = v0;
  if (threadIdx.x == 1 && p1) *p1 = v1;
  if (threadIdx.x == 2 && p2) *p2 = v2;
}

hipError_t launch_ds_set3(hipStream_t s, uint32_t* p0, uint32_t v0, uint32_t* p1, uint32_t v1, uint32_t* p2,
                          uint32_t v2) {
  hipLaunchKernelGGL(k_ds_set3, dim3(1), dim3(64), 0, s, p0, v0, p1, v1, p2, v2);
  return hipGetLastError();
}

// CE_DS_DECODE_STAGE=1: the staged decode (a wave's files in LDS)
static bool decode_stage() {
  const char* v = getenv("CE_DS_DECODE_STAGE");  // (read per launch: the tests flip it)
  return v && atoi(v) != 0;
}

uint32_t ds_count_blocks(uint32_t n) { return blocks_for(n); }

hipError_t launch_ds_count(hipStream_t s, const DsDecodeArgs& a) {
  if (a.n == 0) return hipSuccess;
  if (decode_stage()) hipLaunchKernelGGL(k_ds_count<true>, dim3(ds_count_blocks(a.n)), dim3(kBlock), kStageLds, s, a);
  else hipLaunchKernelGGL(k_ds_count<false>, dim3(ds_count_blocks(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// emit_legacy: some file is left to the lane-per-file emit (false: the open decoded every applied
// file, only the untile runs)
hipError_t launch_ds_emit(hipStream_t s, const DsDecodeArgs& a, bool emit_legacy) {
  if (a.n == 0) return hipSuccess;
  if (a.tile.npad) {
    if (!emit_legacy) {
    } else if (decode_stage()) {
      hipLaunchKernelGGL((k_ds_emit<true, true>), dim3(blocks_for(a.n)), dim3(kBlock), kStageLds, s, a);
    } else {
      hipLaunchKernelGGL((k_ds_emit<true, false>), dim3(blocks_for(a.n)), dim3(kBlock), 0, s, a);
    }
  } else if (emit_legacy) {
    if (decode_stage()) hipLaunchKernelGGL((k_ds_emit<false, true>), dim3(blocks_for(a.n)), dim3(kBlock), kStageLds, s, a);
    else hipLaunchKernelGGL((k_ds_emit<false, false>), dim3(blocks_for(a.n)), dim3(kBlock), 0, s, a);
  }
  if (a.tile.npad || a.fdone) {
    // LDS for the batch's largest per-file count, not kTileMaxRows: more blocks per CU
    const uint32_t rows = a.tile.max_rows ? std::min<uint32_t>(a.tile.max_rows, kTileMaxRows) : kTileMaxRows;
    hipLaunchKernelGGL(k_ds_untile, dim3((a.n + 63) / 64, 9), dim3(kBlock), (size_t)rows * 64 * 8, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_ds_iota(hipStream_t s, uint32_t* v, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_iota, dim3(blocks_for(n)), dim3(kBlock), 0, s, v, n);
  return hipGetLastError();
}

hipError_t launch_ds_gather_ctr(hipStream_t s, const uint32_t* perm, const unsigned long long* ctr,
                                unsigned long long* out, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_gather_ctr, dim3(blocks_for(n)), dim3(kBlock), 0, s, perm, ctr, out, n);
  return hipGetLastError();
}

hipError_t launch_ds_applied(hipStream_t s, const uint32_t* keys_sorted, const uint32_t* perm,
                             const unsigned long long* ctr_sorted,
                             const unsigned long long* excl_max, const unsigned long long* clock,
                             uint8_t* applied, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_applied, dim3(blocks_for(n)), dim3(kBlock), 0, s, keys_sorted, perm,
                     ctr_sorted, excl_max, clock, applied, n);
  return hipGetLastError();
}

hipError_t launch_ds_contig(hipStream_t s, const uint32_t* actor, uint32_t n, uint32_t* marks, uint32_t n_marks,
                            uint32_t gen, uint32_t* flag, const uint32_t* miss_src, uint32_t* pub, DsMono mono) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_contig, dim3(blocks_for(n)), dim3(kBlock), 0, s, actor, n, marks, n_marks, gen, flag,
                     miss_src, pub, mono);
  return hipGetLastError();
}

hipError_t launch_ds_clock(hipStream_t s, const uint32_t* keys_sorted, const unsigned long long* ctr_sorted,
                           const unsigned long long* excl_max, unsigned long long* clock, uint32_t n_add) {
  if (n_add == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_clock, dim3(blocks_for(n_add)), dim3(kBlock), 0, s, keys_sorted, ctr_sorted,
                     excl_max, clock, n_add);
  return hipGetLastError();
}

hipError_t launch_ds_add_pairs(hipStream_t s, DsTables t, DsOps o, const uint8_t* applied,
                               uint32_t n_add) {
  if (n_add == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_add_pairs, dim3(blocks_for(n_add)), dim3(kBlock), 0, s, t, o, applied, n_add);
  return hipGetLastError();
}

hipError_t launch_ds_kill(hipStream_t s, DsTables t, const uint32_t* cbeg, const uint32_t* mbeg,
                          const uint32_t* c_actor, const unsigned long long* c_ctr,
                          const unsigned long long* mem, uint32_t n_rm) {
  if (n_rm == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_kill, dim3(blocks_for(n_rm)), dim3(kBlock), 0, s, t, cbeg, mbeg, c_actor,
                     c_ctr, mem, n_rm);
  return hipGetLastError();
}

hipError_t launch_ds_finalize(hipStream_t s, DsTables t) {
  hipLaunchKernelGGL(k_ds_finalize, dim3(blocks_for((uint64_t)t.pmask + 1, 1024)), dim3(kBlock), 0, s, t);
  return hipGetLastError();
}

__global__ void __launch_bounds__(kBlock) k_ds_count_members(DsTables t, uint32_t* out) {
  const uint64_t n = (uint64_t)t.smask + 1 + t.mmask + 1;
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) c += t.mkey[i] != kDsEmpty;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

hipError_t launch_ds_count_members(hipStream_t s, DsTables t, uint32_t* out) {
  hipLaunchKernelGGL(k_ds_count_members, dim3(blocks_for((uint64_t)t.smask + t.mmask + 2, 1024)), dim3(kBlock), 0, s, t, out);
  return hipGetLastError();
}

hipError_t launch_ds_part_count(hipStream_t s, const DsPartArgs& a) {
  const size_t lds = (size_t)a.parts * 4;
  if (a.chunk == 256 * kPartBatch) {
    hipLaunchKernelGGL(k_ds_part_adds<256>, dim3(a.ba ? a.ba : 1), dim3(256), lds, s, a);
    if (a.bk) hipLaunchKernelGGL(k_ds_part_kills<256>, dim3(a.bk), dim3(256), lds, s, a);
  } else if (a.chunk == kDsPartChunkSmall) {
    hipLaunchKernelGGL(k_ds_part_adds<kDsPartThreadsSmall>, dim3(a.ba ? a.ba : 1), dim3(kDsPartThreadsSmall), lds, s, a);
    if (a.bk) hipLaunchKernelGGL(k_ds_part_kills<kDsPartThreadsSmall>, dim3(a.bk), dim3(kDsPartThreadsSmall), lds, s, a);
  } else {
    hipLaunchKernelGGL(k_ds_part_adds<kPartThreads>, dim3(a.ba ? a.ba : 1), dim3(kPartThreads), lds, s, a);
    if (a.bk) hipLaunchKernelGGL(k_ds_part_kills<kPartThreads>, dim3(a.bk), dim3(kPartThreads), lds, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_ds_part_apply(hipStream_t s, const DsPartArgs& a) {
  static const uint32_t grid = getenv("CE_DS_APPLY_GRID") ? (uint32_t)atoi(getenv("CE_DS_APPLY_GRID")) : 768u;
  hipLaunchKernelGGL(k_ds_part_apply, dim3(grid && grid < a.parts ? grid : a.parts), dim3(kApplyThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ds_deferred(hipStream_t s, const uint32_t* cbeg, const uint32_t* c_actor,
                              const unsigned long long* c_ctr, const unsigned long long* clock,
                              uint8_t* deferred, uint32_t n_rm, uint32_t* any, const uint32_t* pub_src,
                              uint32_t* pub_dst, uint32_t pub_words) {
  if (n_rm == 0 && !pub_dst) return hipSuccess;
  // (publishing: live[7..16) count the blocks in two levels, zero between uses)
  const DsPublish pub{pub_src, pub_dst, pub_words, pub_dst ? const_cast<uint32_t*>(pub_src) + 7 : nullptr};
  // publishing: at most 512 blocks (grid-stride, four removals per lane and trip): the two-level
  // count is then ~64 same-address atomics per word (one word for 1600 blocks took 95 us)
  const uint32_t nb = std::max<uint32_t>(1, std::min<uint32_t>(pub_dst ? 512 : 8192, blocks_for((n_rm + 3) / 4)));
  if (nb > 0xffffu * 8u) return hipErrorInvalidValue;  // (the 16-bit block counts)
  hipLaunchKernelGGL(k_ds_deferred, dim3(nb), dim3(kBlock), 0, s, cbeg, c_actor, c_ctr, clock, deferred, n_rm, any, pub);
  return hipGetLastError();
}

hipError_t launch_ds_put_other(hipStream_t s, DsTables t, const unsigned long long* member,
                               const uint32_t* actor, const unsigned long long* value, uint32_t n,
                               bool zero_counts) {
  if (n == 0 && !zero_counts) return hipSuccess;
  hipLaunchKernelGGL(k_ds_put_other, dim3(n ? blocks_for(n) : 1), dim3(kBlock), 0, s, t, member, actor, value, n,
                     zero_counts ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_ds_merge_finalize(hipStream_t s, DsTables t, const unsigned long long* clock,
                                   const unsigned long long* oclock) {
  hipLaunchKernelGGL(k_ds_merge_finalize, dim3(blocks_for((uint64_t)t.pmask + 1, 1024)), dim3(kBlock), 0, s, t,
                     clock, oclock);
  return hipGetLastError();
}

hipError_t launch_ds_kmerge(hipStream_t s, DsTables t, const DsMergeSrc* d_src, const DsMergeSrc* h_src, uint32_t nf,
                            unsigned long long* clock, const unsigned long long* oclocks, uint32_t ccap, uint32_t ostride,
                            unsigned long long* hold, uint32_t* pub_dst, const uint32_t* go, bool fresh) {
  (void)d_src;
  uint32_t nmax = 0;
  for (uint32_t f = 0; f < nf; f++) nmax = h_src[f].n > nmax ? h_src[f].n : nmax;
  const uint32_t gx = nmax ? blocks_for(nmax) : 1;
  auto srcs = [&](uint32_t c0) {
    DsMergeSrcs m{};
    m.f0 = c0;
    m.go = go;
    m.fresh = fresh ? 1u : 0u;
    for (uint32_t i = 0; i < kMergeInline && c0 + i < nf; i++) m.f[i] = h_src[c0 + i];
    return m;
  };
  for (uint32_t c0 = 0; c0 < nf; c0 += kMergeInline)
    hipLaunchKernelGGL(k_ds_kput, dim3(gx, std::min(kMergeInline, nf - c0)), dim3(kBlock), 0, s, t, srcs(c0));
  // 512 blocks (2 per CU, 8 trips each): fewer blocks' end-of-grid atomics (same box: 1024 65.0 us,
  // 512 60.5, 256 73.1, 4096 148)
  static const uint32_t kf_cap = getenv("CE_KFINAL_BLOCKS") ? (uint32_t)atoi(getenv("CE_KFINAL_BLOCKS")) : 512u;
  const dim3 gf(blocks_for((uint64_t)t.pmask + 1, kf_cap));
  // CE_KFINAL_ROWS=1: into an empty table with every row's slot recorded, the final rule over the
  // rows' owners (k_ds_kfinal_rows) instead of a scan of the whole table.  Measured at C3 (same
  // box): 48.7 vs 49.3 us, but 139 MB fetched against the scan's 79 (the rows' random slot
  // accesses each pull a sector for 8 bytes), so the scan stays the default
  static const bool rows_env = getenv("CE_KFINAL_ROWS") && atoi(getenv("CE_KFINAL_ROWS")) != 0;
  bool rows = rows_env && fresh && t.pmask < kSlotOwner;
  for (uint32_t f = 0; f < nf && rows; f++) rows = h_src[f].slot != nullptr;
  uint32_t nlaunch = 0;
  for (uint32_t c0 = 0; c0 < nf; c0 += kMergeInline) nlaunch += std::min(kMergeInline, nf - c0);
  const uint32_t blocks_total = gx * nlaunch;
  auto go_hold = [&](auto* hp) {
    using H = std::remove_pointer_t<decltype(hp)>;
    for (uint32_t c0 = 0; c0 < nf; c0 += kMergeInline)
      hipLaunchKernelGGL(k_ds_khold<H>, dim3(gx, std::min(kMergeInline, nf - c0)), dim3(kBlock), 0, s, t, srcs(c0), hp);
    if (rows) {
      for (uint32_t c0 = 0; c0 < nf; c0 += kMergeInline)
        hipLaunchKernelGGL(k_ds_kfinal_rows<H>, dim3(gx, std::min(kMergeInline, nf - c0)), dim3(kBlock), 0, s, t,
                           srcs(c0), clock, oclocks, ostride, nf, hp, blocks_total);
    } else {
      hipLaunchKernelGGL(k_ds_kfinal<H>, gf, dim3(kBlock), 0, s, t, clock, oclocks, ostride, nf, hp, go, fresh ? 1u : 0u);
    }
  };
  if (nf <= 32) go_hold(reinterpret_cast<uint32_t*>(hold));  // (the buffer is zero as u64 words: its u32 view too)
  else go_hold(hold);
  hipLaunchKernelGGL(k_ds_kclock, dim3(std::max<uint32_t>(1, blocks_for(ccap))), dim3(kBlock), 0, s, clock, oclocks,
                     ccap, ostride, nf, t.live, pub_dst, 5u, go);
  return hipGetLastError();
}

// Column partials (ds_merge_columns_device): each part's actor column holds indices into its own
// actor list; map[i] is that actor's id in the receiving core.  ids[j] = map[actor[j]] and the
// part's clock scattered densely by receiver id into oclock (zeroed beforehand by the caller's fill).
__global__ void __launch_bounds__(kBlock) k_cols_remap(DsColsRemaps r) {
  const DsColsRemap x = r.f[blockIdx.y];
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < x.np; j += gridDim.x * kBlock) x.ids[j] = x.map[x.actor[j]];
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < x.na; i += gridDim.x * kBlock)
    x.oclock[(size_t)x.map[i] * x.ostride] = x.clock[i];
}

// a column partial's deferred section (CSR: cbeg / mbeg n_rm + 1 offsets, act n_ent indices into
// the partial's na actors) checked before the remap and the kill kernels walk it: *bad = 1 on any
// offset out of order or past its array, or an actor index >= na
__global__ void __launch_bounds__(kBlock) k_ds_csr_check(const uint32_t* cbeg, const uint32_t* mbeg, const uint32_t* act,
                                                         uint32_t n_rm, uint32_t n_ent, uint32_t n_mem, uint32_t na,
                                                         uint32_t* bad) {
  const uint32_t nt = gridDim.x * kBlock;
  bool b = false;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i <= n_rm; i += nt) {
    const uint32_t c = cbeg[i], m = mbeg[i];
    if (i == 0) b |= c != 0 || m != 0;
    else b |= c < cbeg[i - 1] || m < mbeg[i - 1];
    if (i == n_rm) b |= c != n_ent || m != n_mem;
    b |= c > n_ent || m > n_mem;
  }
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < n_ent; j += nt) b |= act[j] >= na;
  if (b) *bad = 1u;
}

hipError_t launch_ds_csr_check(hipStream_t s, const uint32_t* cbeg, const uint32_t* mbeg, const uint32_t* act,
                               uint32_t n_rm, uint32_t n_ent, uint32_t n_mem, uint32_t na, uint32_t* bad) {
  const uint32_t mx = std::max(n_rm + 1, n_ent);
  hipLaunchKernelGGL(k_ds_csr_check, dim3(std::min<uint32_t>(blocks_for(mx), 1024)), dim3(kBlock), 0, s, cbeg, mbeg, act,
                     n_rm, n_ent, n_mem, na, bad);
  return hipGetLastError();
}

hipError_t launch_cols_remap(hipStream_t s, const DsColsRemap* parts, uint32_t k) {
  for (uint32_t c0 = 0; c0 < k; c0 += kColsInline) {
    DsColsRemaps r{};
    uint32_t mx = 1;
    const uint32_t kk = std::min(kColsInline, k - c0);
    for (uint32_t i = 0; i < kk; i++) {
      r.f[i] = parts[c0 + i];
      mx = std::max(mx, std::max(r.f[i].np, r.f[i].na));
    }
    hipLaunchKernelGGL(k_cols_remap, dim3(std::min<uint32_t>(blocks_for(mx), 2048), kk), dim3(kBlock), 0, s, r);
  }
  return hipGetLastError();
}

hipError_t launch_ds_merge(hipStream_t s, DsTables t, const unsigned long long* clock,
                           const unsigned long long* oclock) {
  hipLaunchKernelGGL(k_ds_merge, dim3(blocks_for((uint64_t)t.pmask + 1)), dim3(kBlock), 0, s, t, clock, oclock);
  return hipGetLastError();
}

hipError_t launch_ds_collect(hipStream_t s, DsTables t, unsigned long long* member, uint32_t* actor,
                             unsigned long long* value, uint32_t* n_out, unsigned long long* bmax, uint32_t* host_out,
                             unsigned long long* extra_dst, const unsigned long long* extra_src, uint32_t extra_words) {
  const uint32_t nb = blocks_for((uint64_t)t.pmask + 1, kCollectBlocks);
  hipLaunchKernelGGL(k_ds_collect, dim3(nb), dim3(kBlock), 0, s, t, member, actor, value, n_out, bmax);
  hipLaunchKernelGGL(k_ds_collect_max, dim3(1), dim3(kBlock), 0, s, bmax, nb, n_out, host_out, extra_dst, extra_src,
                     extra_words);
  return hipGetLastError();
}

hipError_t launch_ds_reinsert(hipStream_t s, DsTables t, const unsigned long long* member,
                              const uint32_t* actor, const unsigned long long* value, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_reinsert, dim3(blocks_for(n)), dim3(kBlock), 0, s, t, member, actor, value, n);
  return hipGetLastError();
}

hipError_t launch_ds_gather_entries(hipStream_t s, const uint32_t* perm, const uint32_t* actor_in,
                                    const unsigned long long* value_in, uint32_t* actor_out,
                                    unsigned long long* value_out, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ds_gather_entries, dim3(blocks_for(n)), dim3(kBlock), 0, s, perm, actor_in,
                     value_in, actor_out, value_out, n);
  return hipGetLastError();
}

hipError_t launch_mv_prep(hipStream_t s, const MvArgs& a) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_mv_prep, dim3(blocks_for(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_mv_round(hipStream_t s, const MvArgs& a) {
  hipLaunchKernelGGL(k_mv_argmax, dim3(a.n_blk), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(k_mv_final, dim3(1), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(k_mv_kill, dim3(blocks_for(a.n)), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(k_mv_clear, dim3(1), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace ce
