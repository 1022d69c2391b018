// ce_dotset_io.hip -- StateWrapper<Orswot<u64, Uuid>> bytes on the device, both directions:
//
//   writer  the compaction's clear text (crdt-enc/src/lib.rs:336, to_vec_named) from the live
//           (member, actor, counter) pairs of the entry tables: pairs sorted by (member, actor
//           UUID rank), one lane per pair computing its byte length, two exclusive scans
//           (entry heads, byte offsets), one lane per pair writing its Dot (and its member's
//           entry head).  Host-built prefix (next_op_versions, clock) and suffix (deferred)
//           are placed around it on the device, so the clear text goes straight into the seal.
//   reader  the `entries` map of a state file (read_remote_states, lib.rs:447) into columns:
//           the canonical VClock head `81 a4 "dots"` is searched in parallel, one lane per
//           candidate parses its entry's Dots, and the chain of entries is validated end to
//           end (each member key exactly fills the gap left by the previous entry), so a
//           spurious pattern inside a UUID or counter can only make the reader decline, never
//           misread.  Anything outside the canonical form is declined to the host parser.
//
// Integer / byte work bounded by HBM latency; no MFMA.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#if CE_FUSED_DIAG  // hipCUB only for the diagnostics build's A/B (CE_SER_CUB)
#include <hipcub/hipcub.hpp>
#endif
#include <map>
#include <mutex>

#include "ce_device.h"
#include "ce_dotset.h"
#include "ce_dotset_io.h"

namespace ce {
namespace {

constexpr int kB = 256;

inline uint32_t nblk(uint64_t n, uint32_t cap = 8192) {
  uint64_t b = (n + kB - 1) / kB;
  if (b == 0) b = 1;
  return (uint32_t)(b < cap ? b : cap);
}

// rmp-serde's smallest encodings
__device__ __forceinline__ uint32_t ulen(unsigned long long v) {
  return v <= 0x7full ? 1u : v <= 0xffull ? 2u : v <= 0xffffull ? 3u : v <= 0xffffffffull ? 5u : 9u;
}
__device__ __forceinline__ uint32_t maplen(uint32_t k) { return k <= 15u ? 1u : k <= 0xffffu ? 3u : 5u; }
__device__ __forceinline__ uint32_t put_uint(uint8_t* o, unsigned long long v) {
  if (v <= 0x7full) { o[0] = (uint8_t)v; return 1; }
  int k;
  if (v <= 0xffull) { o[0] = 0xcc; k = 1; }
  else if (v <= 0xffffull) { o[0] = 0xcd; k = 2; }
  else if (v <= 0xffffffffull) { o[0] = 0xce; k = 4; }
  else { o[0] = 0xcf; k = 8; }
  for (int b = 0; b < k; b++) o[1 + b] = (uint8_t)(v >> (8 * (k - 1 - b)));
  return 1u + (uint32_t)k;
}
__device__ __forceinline__ uint32_t put_map(uint8_t* o, uint32_t k) {
  if (k <= 15u) { o[0] = (uint8_t)(0x80 | k); return 1; }
  if (k <= 0xffffu) { o[0] = 0xde; o[1] = (uint8_t)(k >> 8); o[2] = (uint8_t)k; return 3; }
  o[0] = 0xdf; o[1] = (uint8_t)(k >> 24); o[2] = (uint8_t)(k >> 16); o[3] = (uint8_t)(k >> 8); o[4] = (uint8_t)k;
  return 5;
}

// ---------------------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------------------
__global__ void k_ser_rank(const uint32_t* actor, const uint32_t* rank_of_id, uint32_t* key, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) key[i] = rank_of_id[actor[i]];
}

__global__ void k_ser_iota(uint32_t* v, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) v[i] = i;
}

__global__ void k_ser_gather2(const uint32_t* perm, const uint32_t* actor_in, const unsigned long long* value_in,
                              uint32_t* actor_out, unsigned long long* value_out, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
    actor_out[i] = actor_in[perm[i]];
    value_out[i] = value_in[perm[i]];
  }
}

__global__ void k_ser_gather_member(const uint32_t* perm, const unsigned long long* member_in,
                                    unsigned long long* member_out, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) member_out[i] = member_in[perm[i]];
}

// one sort when (member, rank) packs into K: key = member << rank_bits | rank ((member, actor)
// pairs are unique, so no two keys tie); the values ride through the sort itself
template <typename K>
__global__ void k_ser_key(const uint32_t* actor, const uint32_t* rank_of_id, const unsigned long long* member,
                          int rank_bits, K* key, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB)
    key[i] = ((K)member[i] << rank_bits) | (K)rank_of_id[actor[i]];
}

// member and actor id back out of the sorted key (member_out may alias key): no gather
template <typename K>
__global__ void k_ser_unpack(const K* key, int rank_bits, const uint32_t* id_of_rank, unsigned long long* member_out,
                             uint32_t* actor_out, uint32_t n) {
  const K mask = ((K)1 << rank_bits) - 1;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
    const K k = key[i];
    actor_out[i] = id_of_rank[(uint32_t)(k & mask)];
    member_out[i] = (unsigned long long)(k >> rank_bits);
  }
}

// head[i] = pair i starts a member's entry
__global__ void k_ser_head(const unsigned long long* member, uint32_t* head, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB)
    head[i] = i == 0 || member[i] != member[i - 1];
}

// entry e = hrank of its head: seg[e] = head position, seg[e + 1] written by the entry's last
// pair (so seg[] is the CSR of entries over pairs, seg[n_members] = n)
__global__ void k_ser_seg(const unsigned long long* member, const uint32_t* head, const uint32_t* hrank,
                          uint32_t* seg, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
    const uint32_t e = hrank[i] + head[i] - 1;  // entry of pair i
    if (head[i]) seg[e] = i;
    if (i + 1 == n || member[i + 1] != member[i]) seg[e + 1] = i + 1;
  }
}

// bytes of pair i: its Dot (c4 10 uuid16 uint) and, at a head, the entry head
// (member uint, 81 a4 "dots", map header of the entry's Dot count)
__global__ void k_ser_len(const unsigned long long* member, const unsigned long long* value,
                          const uint32_t* head, const uint32_t* hrank, const uint32_t* seg,
                          uint32_t* len, uint32_t n) {
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
    uint32_t l = 18u + ulen(value[i]);
    if (head[i]) {
      const uint32_t e = hrank[i];
      l += ulen(member[i]) + 6u + maplen(seg[e + 1] - seg[e]);
    }
    len[i] = l;
  }
}

// The entry bookkeeping over the sorted pairs in two scans of 2048-pair tiles, each a tile-sums
// launch and an apply launch that sums the tiles before its own (no separate scan of the sums):
//   k_ser_head_tiles / k_ser_head_apply: head[i] (pair i starts a member's entry), hrank = its
//     exclusive scan, seg[] = the entries' CSR over pairs (seg[e] = head position, seg[e + 1]
//     written by the entry's last pair, seg[n_members] = n)
//   k_ser_len_tiles / k_ser_len_apply: len[i] = bytes of pair i (its Dot, plus at a head the entry
//     head: member uint, 81 a4 "dots", map header of the entry's Dot count) and pos = its scan
// (four launches where head, scan, seg, len, scan were seven)
constexpr uint32_t kSerItems = 8, kSerTile = kB * kSerItems;

__device__ __forceinline__ uint32_t ser_block_incl(uint32_t v, uint32_t* lds) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o);
    if (lane >= (uint32_t)o) v += y;
  }
  if (lane == 63) lds[w] = v;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t k = 0; k < w; k++) add += lds[k];
  __syncthreads();
  return v + add;
}

// the sum of tile_sum[0 .. blockIdx.x), every lane
__device__ __forceinline__ uint32_t ser_tiles_before(const uint32_t* tile_sum, uint32_t* lds, uint32_t* off) {
  uint32_t b = 0;
  for (uint32_t x = threadIdx.x; x < blockIdx.x; x += kB) b += tile_sum[x];
  b = ser_block_incl(b, lds);
  if (threadIdx.x == kB - 1) *off = b;
  __syncthreads();
  return *off;
}

__global__ void __launch_bounds__(kB) k_ser_head_tiles(const unsigned long long* member, uint32_t n, uint32_t* tile_sum) {
  __shared__ uint32_t lds[kB / 64];
  const uint32_t i0 = blockIdx.x * kSerTile + threadIdx.x * kSerItems;
  uint32_t s = 0;
  unsigned long long prev = i0 > 0 && i0 < n ? member[i0 - 1] : 0ull;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++) {
    const uint32_t i = i0 + k;
    if (i < n) {
      const unsigned long long m = member[i];
      s += i == 0 || m != prev;
      prev = m;
    }
  }
  s = ser_block_incl(s, lds);
  if (threadIdx.x == kB - 1) tile_sum[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kB) k_ser_head_apply(const unsigned long long* member, uint32_t n, const uint32_t* tile_sum,
                                                       uint32_t* head, uint32_t* hrank, uint32_t* seg) {
  __shared__ uint32_t lds[kB / 64];
  __shared__ uint32_t off;
  const uint32_t base = ser_tiles_before(tile_sum, lds, &off);
  const uint32_t i0 = blockIdx.x * kSerTile + threadIdx.x * kSerItems;
  unsigned long long m[kSerItems + 2];
  m[0] = i0 > 0 && i0 <= n ? member[i0 - 1] : 0ull;
#pragma unroll
  for (int k = 0; k <= (int)kSerItems; k++) m[k + 1] = i0 + k < n ? member[i0 + k] : 0ull;
  uint32_t h[kSerItems], s = 0;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++) {
    h[k] = i0 + k < n && (i0 + k == 0 || m[k + 1] != m[k]);
    s += h[k];
  }
  uint32_t run = ser_block_incl(s, lds) - s + base;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++) {
    const uint32_t i = i0 + k;
    if (i < n) {
      head[i] = h[k];
      hrank[i] = run;
      const uint32_t e = run + h[k] - 1;  // entry of pair i
      if (h[k]) seg[e] = i;
      if (i + 1 == n || m[k + 2] != m[k + 1]) seg[e + 1] = i + 1;
    }
    run += h[k];
  }
}

__device__ __forceinline__ uint32_t ser_len_of(const unsigned long long* member, const unsigned long long* value,
                                               const uint32_t* head, const uint32_t* hrank, const uint32_t* seg,
                                               uint32_t i) {
  uint32_t l = 18u + ulen(value[i]);
  if (head[i]) {
    const uint32_t e = hrank[i];
    l += ulen(member[i]) + 6u + maplen(seg[e + 1] - seg[e]);
  }
  return l;
}

__global__ void __launch_bounds__(kB) k_ser_len_tiles(const unsigned long long* member, const unsigned long long* value,
                                                      const uint32_t* head, const uint32_t* hrank, const uint32_t* seg,
                                                      uint32_t n, uint32_t* tile_sum) {
  __shared__ uint32_t lds[kB / 64];
  const uint32_t i0 = blockIdx.x * kSerTile + threadIdx.x * kSerItems;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++)
    if (i0 + k < n) s += ser_len_of(member, value, head, hrank, seg, i0 + k);
  s = ser_block_incl(s, lds);
  if (threadIdx.x == kB - 1) tile_sum[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kB) k_ser_len_apply(const unsigned long long* member, const unsigned long long* value,
                                                      const uint32_t* head, const uint32_t* hrank, const uint32_t* seg,
                                                      uint32_t n, const uint32_t* tile_sum, uint32_t* len, uint32_t* pos) {
  __shared__ uint32_t lds[kB / 64];
  __shared__ uint32_t off;
  const uint32_t base = ser_tiles_before(tile_sum, lds, &off);
  const uint32_t i0 = blockIdx.x * kSerTile + threadIdx.x * kSerItems;
  uint32_t l[kSerItems], s = 0;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++) {
    l[k] = i0 + k < n ? ser_len_of(member, value, head, hrank, seg, i0 + k) : 0u;
    s += l[k];
  }
  uint32_t run = ser_block_incl(s, lds) - s + base;
#pragma unroll
  for (int k = 0; k < (int)kSerItems; k++) {
    if (i0 + k < n) {
      len[i0 + k] = l[k];
      pos[i0 + k] = run;
    }
    run += l[k];
  }
}

// A block's 256 Dots are one contiguous output range (pos is the scan of their lengths, member
// headers included): the bytes are assembled in LDS with byte stores, then go out as aligned
// 16-byte stores (byte stores at the range's two unaligned ends).  Byte stores straight to HBM
// put ~25 scattered one-byte writes per lane through the memory pipeline (~110 us at C3).
constexpr uint32_t kSerMaxDot = 47;  // member uint 9 + "dots" 6 + map header 5 + bin16 18 + uint 9
__global__ void __launch_bounds__(kB) k_ser_write(OrswotSerArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kB * kSerMaxDot + 32];
  const uint32_t nm = a.hrank[a.n - 1] + a.head[a.n - 1];
  const uint64_t base = a.prefix_len + maplen(nm);
  for (uint32_t i0 = blockIdx.x * kB; i0 < a.n; i0 += gridDim.x * kB) {  // block-uniform trips
    const uint32_t i1 = min(a.n, i0 + kB);
    const uint64_t lo = base + a.pos[i0], hi = base + a.pos[i1 - 1] + a.len[i1 - 1];
    const uint64_t lo16 = lo & ~15ull;
    const uint32_t i = i0 + threadIdx.x;
    if (i < i1) {
      uint8_t* o = buf + (base + a.pos[i] - lo16);
      if (a.head[i]) {
        const uint32_t e = a.hrank[i];
        o += put_uint(o, a.member[i]);
        o[0] = 0x81; o[1] = 0xa4; o[2] = 'd'; o[3] = 'o'; o[4] = 't'; o[5] = 's';
        o += 6;
        o += put_map(o, a.seg[e + 1] - a.seg[e]);
      }
      o[0] = 0xc4;
      o[1] = 16;
      const uint4 u = *reinterpret_cast<const uint4*>(a.uuid_of_id + 16ull * a.actor[i]);
      const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int b = 0; b < 16; b++) o[2 + b] = (uint8_t)(uw[b >> 2] >> (8 * (b & 3)));
      put_uint(o + 18, a.value[i]);
    }
    __syncthreads();
    // [lo, hi) out: aligned 16-byte stores over [a0, a1), bytes at the ends
    const uint64_t a0 = (lo + 15) & ~15ull, a1 = hi & ~15ull;
    const bool al = (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;  // (a caller's buffer may not be)
    if (al && a0 < a1) {
      for (uint64_t x = a0 + 16ull * threadIdx.x; x < a1; x += 16ull * kB)
        *reinterpret_cast<uint4*>(a.out + x) = *reinterpret_cast<const uint4*>(buf + (x - lo16));
      if (threadIdx.x < a0 - lo) a.out[lo + threadIdx.x] = buf[lo - lo16 + threadIdx.x];
      if (threadIdx.x < hi - a1) a.out[a1 + threadIdx.x] = buf[a1 - lo16 + threadIdx.x];
    } else {
      for (uint64_t x = lo + threadIdx.x; x < hi; x += kB) a.out[x] = buf[x - lo16];
    }
    __syncthreads();  // the next trip reuses buf
  }
}

// the prefix and the entries map header, the suffix after the entries, the clear length into
// the seal's offsets (offs[0] = 0, offs[1] = clear length, out_offs[0] = 0)
__global__ void k_ser_tail(OrswotSerArgs a) {
  const uint32_t nm = a.n ? a.hrank[a.n - 1] + a.head[a.n - 1] : 0u;
  const uint64_t body = a.n ? (uint64_t)a.pos[a.n - 1] + a.len[a.n - 1] : 0ull;
  const uint64_t hl = maplen(nm);
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
  // the prefix (next_op_versions and the clock: ~200 KB at 4096 actors) in 16-byte pieces when
  // both ends allow it -- one block copying bytes took ~0.2 ms
  if (((reinterpret_cast<uintptr_t>(a.out) | reinterpret_cast<uintptr_t>(a.prefix)) & 15) == 0) {
    const uint64_t n16 = a.prefix_len / 16;
    for (uint64_t j = gt; j < n16; j += gs)
      reinterpret_cast<uint4*>(a.out)[j] = reinterpret_cast<const uint4*>(a.prefix)[j];
    for (uint64_t j = 16 * n16 + gt; j < a.prefix_len; j += gs) a.out[j] = a.prefix[j];
  } else {
    for (uint64_t j = gt; j < a.prefix_len; j += gs) a.out[j] = a.prefix[j];
  }
  const uint64_t s0 = a.prefix_len + hl + body;
  for (uint64_t j = gt; j < a.suffix_len; j += gs) a.out[s0 + j] = a.suffix[j];
  if (gt == 0) put_map(a.out + a.prefix_len, nm);
  if (gt == 0) {
    a.seal_offs[0] = 0;
    a.seal_offs[1] = s0 + a.suffix_len;
    a.seal_offs[2] = 0;  // out_offs[0]
    a.stats[0] = nm;
  }
}

// ---------------------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// canonical msgpack uint at p (bounded by end): value, length (0 = not a canonical uint)
__device__ __forceinline__ uint32_t rd_uint(const uint8_t* p, const uint8_t* end, unsigned long long* v) {
  if (p >= end) return 0;
  const uint8_t m = p[0];
  if (m < 0x80) { *v = m; return 1; }
  uint32_t k = m == 0xcc ? 1 : m == 0xcd ? 2 : m == 0xce ? 4 : m == 0xcf ? 8 : 0;
  if (!k || p + 1 + k > end) return 0;
  unsigned long long x = 0;
  for (uint32_t b = 0; b < k; b++) x = (x << 8) | p[1 + b];
  // rmp-serde writes the smallest form; a longer one would still decode, but the chain check
  // below relies on the canonical length, so anything else goes to the host parser
  if (ulen(x) != 1 + k) return 0;
  *v = x;
  return 1 + k;
}

// candidate entry heads: 81 a4 'd' 'o' 't' 's' at p, followed by a map header.  A block takes
// kFindChunk consecutive positions (k_rdm_count / k_rdm_write)
static constexpr uint32_t kFindPer = 16, kFindChunk = kFindPer * kB;
__device__ __forceinline__ bool entry_head_at(const uint8_t* s, uint64_t p) {
  if (s[p] != 0x81 || s[p + 1] != 0xa4 || s[p + 2] != 'd' || s[p + 3] != 'o' || s[p + 4] != 't' ||
      s[p + 5] != 's')
    return false;
  const uint8_t m = s[p + 6];
  return (m & 0xf0) == 0x80 || m == 0xde || m == 0xdf;
}

// HashMap<M, VClock> keeps a repeated member's later clock: a file with repeated members goes to
// the host parser (flag 8).  Found by inserting every member into an open-addressing set
// (atomicCAS on the all-ones empty word; all-ones members are counted in the word after the
// set, k_rdm_dups): one launch where a 64-bit radix sort + neighbour compare took a dozen.
__device__ __forceinline__ uint32_t mix_member(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// ---------------------------------------------------------------------------------------
// reader over many state files at once (gridDim.y = file): every stage is one launch for all
// files instead of one (or, with the candidate sort, eight) per file -- at C3's 8 state files the
// per-file launches were host-bound (~110 launches, 0.5 ms).  The entry heads come out in
// position order without a sort: a count pass per 4 KiB chunk, one exclusive scan over all
// files' chunks, a write pass that ranks each chunk's heads in order.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* part) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kB / 64; w++) t += part[w];
  return t;
}

__global__ void __launch_bounds__(kB) k_rdm_count(RdFiles fa, uint32_t* cnt) {
  __shared__ uint32_t part[kB / 64];
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (blockIdx.x >= a.nchunks) return;
  const uint64_t c0 = a.lo + (uint64_t)blockIdx.x * kFindChunk;
  uint32_t n = 0;
#pragma unroll 4
  for (uint32_t k = 0; k < kFindPer; k++) {
    const uint64_t p = c0 + k * kB + threadIdx.x;
    n += (p + 7 <= a.hi && entry_head_at(a.s, p)) ? 1u : 0u;
  }
  const uint32_t t = block_sum(n, part);
  if (threadIdx.x == 0) cnt[a.chunk0 + blockIdx.x] = t;
}

// chunk heads in position order: cand[scan(chunk) - scan(file's first chunk) + rank]
__global__ void __launch_bounds__(kB) k_rdm_write(RdFiles fa, const uint32_t* scan) {
  __shared__ uint32_t part[kB / 64];
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (blockIdx.x >= a.nchunks) return;
  const uint64_t c0 = a.lo + (uint64_t)blockIdx.x * kFindChunk;
  uint32_t at = scan[a.chunk0 + blockIdx.x] - scan[a.chunk0];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t k = 0; k < kFindPer; k++) {
    const uint64_t p = c0 + k * kB + threadIdx.x;
    const bool hit = p + 7 <= a.hi && entry_head_at(a.s, p);
    const unsigned long long bm = __ballot(hit);
    __syncthreads();
    if (lane == 0) part[w] = (uint32_t)__builtin_popcountll(bm);
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < kB / 64; j++) {
      before += (uint32_t)j < w ? part[j] : 0u;
      tot += part[j];
    }
    if (hit) {
      const uint32_t r = at + before + (uint32_t)__builtin_popcountll(bm & ((1ull << lane) - 1ull));
      if (r < a.cap) a.cand[r] = (uint32_t)(p - a.lo);
    }
    at += tot;
  }
}

// the heads found; a count outside [n_cand, cap] (fewer heads than entries, or cand overflowed)
// flags the file so that stages 1 and 2, queued behind without a host wait, skip it
__global__ void k_rdm_found(RdFiles fa, const uint32_t* scan, uint32_t nf) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nf) return;
  const OrswotReadArgs& a = fa.f[f];
  const uint32_t found = scan[a.chunk0 + a.nchunks] - scan[a.chunk0];
  *a.n_cand_dev = found;
  *a.skip = found;
}

// stage 1's first launch, block per file, once the host knows where the entries start (lo): the
// heads before lo (the clocks' own "dots" maps: a couple) are skipped, the count from lo on goes
// to the host, and a count outside [n_cand, cap] flags the file for the later stages to skip
__global__ void __launch_bounds__(256) k_rdm_skip(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.x];
  const uint32_t found = *reinterpret_cast<volatile const uint32_t*>(a.skip);
  const uint32_t m = min(found, a.cap);
  const uint32_t t = threadIdx.x;
  const int before = __syncthreads_count(t < m && (uint64_t)a.cand[t] < a.lo);
  if (t != 0) return;
  uint32_t k = (uint32_t)before;
  if (k == 256u && m > 256u) {  // (many heads before lo: binary search the rest)
    uint32_t l = 256u, h = m;
    while (l < h) {
      const uint32_t mid = (l + h) / 2;
      if ((uint64_t)a.cand[mid] < a.lo) l = mid + 1;
      else h = mid;
    }
    k = l;
  }
  *a.skip = k;
  *a.n_cand_dev = found - k;
  if (found - k < a.n_cand || found > a.cap) atomicOr(a.flags, 16u);
}

__device__ __forceinline__ bool rdm_skip(const OrswotReadArgs& a) {
  return (*reinterpret_cast<volatile const uint32_t*>(a.flags) & 16u) != 0;
}

// entry i's head, relative to lo (stage 1 on: the heads before lo skipped)
__device__ __forceinline__ uint32_t rdm_head(const OrswotReadArgs& a, uint32_t sk, uint32_t i) {
  return a.cand[sk + i] - (uint32_t)a.lo;
}

__global__ void k_rdm_entry(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (rdm_skip(a)) return;
  const uint32_t sk = *a.skip;
  const uint8_t* base = a.s + a.lo;
  const uint8_t* end = a.s + a.hi;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint8_t* p = base + rdm_head(a, sk, i) + 6;
    uint32_t k;
    bool ok = true;
    if ((p[0] & 0xf0) == 0x80) { k = p[0] & 15u; p += 1; }
    else if (p[0] == 0xde) { if (p + 3 > end) ok = false; k = ((uint32_t)p[1] << 8) | p[2]; p += 3; }
    else { if (p + 5 > end) ok = false; k = rd_be32(p + 1); p += 5; }
    uint32_t nz = 0;
    uint32_t prev[4] = {0, 0, 0, 0};
    for (uint32_t d = 0; d < k && ok; d++) {
      if (p + 18 > end || p[0] != 0xc4 || p[1] != 16) { ok = false; break; }
      const uint32_t w0 = rd_be32(p + 2), w1 = rd_be32(p + 6), w2 = rd_be32(p + 10), w3 = rd_be32(p + 14);
      if (d > 0) {
        const bool gt = w0 != prev[0] ? w0 > prev[0] : w1 != prev[1] ? w1 > prev[1]
                      : w2 != prev[2] ? w2 > prev[2] : w3 > prev[3];
        if (!gt) { ok = false; break; }
      }
      prev[0] = w0; prev[1] = w1; prev[2] = w2; prev[3] = w3;
      unsigned long long c;
      const uint32_t ul = rd_uint(p + 18, end, &c);
      if (!ul) { ok = false; break; }
      nz += c != 0;
      p += 18 + ul;
    }
    a.end[i] = ok ? (uint32_t)(p - base) : 0xffffffffu;
    a.ndots[i] = ok ? nz : 0u;
    if (!ok) atomicOr(a.flags, 1u);
  }
}

// the chain check (k_rd_chain) and the repeat set's clearing in one pass: the set is cleared
// here and filled by k_rdm_dups, the next launch
__global__ void k_rdm_chain(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (rdm_skip(a)) return;
  const uint32_t sk = *a.skip;
  const uint8_t* base = a.s + a.lo;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint32_t start = i == 0 ? 0u : a.end[i - 1];
    const uint32_t head = rdm_head(a, sk, i);
    unsigned long long m = 0;
    const uint32_t ul = start <= head ? rd_uint(base + start, base + head, &m) : 0u;
    if (!ul || start + ul != head || a.end[i] == 0xffffffffu) atomicOr(a.flags, 2u);
    a.member[i] = m;
  }
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.dset_mask + 2u; i += gridDim.x * kB) a.msort[i] = ~0ull;
}

__global__ void k_rdm_dups(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (rdm_skip(a)) return;
  constexpr unsigned long long kEmpty = ~0ull;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const unsigned long long m = a.member[i];
    if (m == kEmpty) {
      if (atomicAdd(&a.msort[(size_t)a.dset_mask + 1], 1ull) != kEmpty) atomicOr(a.flags, 8u);
      continue;
    }
    uint32_t h = mix_member(m) & a.dset_mask;
    for (uint32_t probe = 0; probe <= a.dset_mask; probe++) {
      const unsigned long long old = atomicCAS(&a.msort[h], kEmpty, m);
      if (old == kEmpty) break;
      if (old == m) { atomicOr(a.flags, 8u); break; }
      h = (h + 1) & a.dset_mask;
    }
  }
}

// exclusive scan of ndots -> dbase over 2048-entry tiles, then the tail words (k_rd_tail) for
// the file's one download.  k_rdm_tile_sums: tile totals into the repeat-check set's words (free
// once k_rdm_dups is done); k_rdm_tile_scan: a tile's base from the totals before it, the tile
// scanned in LDS, dbase written coalesced.  (One 1024-thread block per file walking contiguous
// per-thread runs -- a load and a store per entry, each instruction touching 64 lines -- took
// ~50 us at C3's 8 x 100k entries.)
constexpr uint32_t kScanTile = kB * 8;

__global__ void __launch_bounds__(kB) k_rdm_tile_sums(RdFiles fa) {
  __shared__ uint32_t part[kB / 64];
  const OrswotReadArgs a = fa.f[blockIdx.y];
  const uint32_t t0 = blockIdx.x * kScanTile;
  if (t0 >= a.n_cand || rdm_skip(a)) return;
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t i = t0 + q * kB + threadIdx.x;
    v += i < a.n_cand ? a.ndots[i] : 0u;
  }
  const uint32_t tot = block_sum(v, part);
  if (threadIdx.x == 0) reinterpret_cast<uint32_t*>(a.msort)[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kB) k_rdm_tile_scan(RdFiles fa) {
  __shared__ uint32_t part[kB / 64];
  __shared__ uint32_t run[kB];
  const OrswotReadArgs a = fa.f[blockIdx.y];
  const uint32_t t0 = blockIdx.x * kScanTile;
  if (t0 >= a.n_cand || rdm_skip(a)) return;
  // the tile's base: the totals of the tiles before it
  const uint32_t* tsum = reinterpret_cast<const uint32_t*>(a.msort);
  uint32_t b = 0;
  for (uint32_t x = threadIdx.x; x < blockIdx.x; x += kB) b += tsum[x];
  const uint32_t base = block_sum(b, part);
  // lane l owns entries t0 + 8 l .. + 7 (two 16-byte loads), a block scan of the lanes' sums
  uint32_t v[8];
  const uint32_t i0 = t0 + 8 * threadIdx.x;
#pragma unroll
  for (int q = 0; q < 8; q++) v[q] = i0 + q < a.n_cand ? a.ndots[i0 + q] : 0u;
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) s += v[q];
  uint32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
    if ((int)(threadIdx.x & 63) >= o) incl += y;
  }
  if ((threadIdx.x & 63) == 63) run[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) wbase += run[w];
  uint32_t r = base + wbase + incl - s;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (i0 + q < a.n_cand) {
      a.dbase[i0 + q] = r;
      if (i0 + q == a.n_cand - 1 && a.tail_out) {
        a.tail_out[0] = a.end[i0 + q];
        a.tail_out[1] = r;  // dbase of the last entry
        a.tail_out[2] = v[q];
        a.tail_out[3] = *a.flags;
        if (a.tail_dev) {
          a.tail_dev[0] = a.end[i0 + q];
          a.tail_dev[1] = r;
          a.tail_dev[2] = v[q];
        }
      }
    }
    r += v[q];
  }
}

// the bytes after the last entry (the deferred map) into pinned memory, block per file, when the
// entries parsed and the tail fits the window
__global__ void __launch_bounds__(kB) k_rdm_tail(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.x];
  if (!a.tail_host || *reinterpret_cast<volatile const uint32_t*>(a.flags)) return;
  const uint32_t e = a.end[a.n_cand - 1];
  if (e == 0xffffffffu || a.lo + e > a.hi || a.hi - (a.lo + e) > a.tail_cap) return;
  const uint8_t* src = a.s + a.lo + e;
  const uint32_t n = (uint32_t)(a.hi - (a.lo + e));
  for (uint32_t j = threadIdx.x; j < n; j += kB) a.tail_host[j] = src[j];
  // "deferred" -> {} in its one canonical form: what lets a merge run before the host parses it
  if (threadIdx.x == 0 && a.tail_dev) {
    const uint8_t k[10] = {0xa8, 'd', 'e', 'f', 'e', 'r', 'r', 'e', 'd', 0x80};
    bool empty = n == 10;
    for (int j = 0; j < 10 && empty; j++) empty = src[j] == k[j];
    a.tail_dev[3] = empty ? 1u : 0u;
  }
}

// emit: only files whose entries all parsed (flags 0 after stage 1; the host checks the rest)
__global__ void k_rdm_emit(RdFiles fa) {
  const OrswotReadArgs a = fa.f[blockIdx.y];
  if (*reinterpret_cast<volatile const uint32_t*>(a.flags)) return;
  const uint32_t sk = *a.skip;
  const uint8_t* base = a.s + a.lo;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint8_t* p = base + rdm_head(a, sk, i) + 6;
    uint32_t k;
    if ((p[0] & 0xf0) == 0x80) { k = p[0] & 15u; p += 1; }
    else if (p[0] == 0xde) { k = ((uint32_t)p[1] << 8) | p[2]; p += 3; }
    else { k = rd_be32(p + 1); p += 5; }
    uint32_t o = a.dbase[i];
    for (uint32_t d = 0; d < k; d++) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; j++)
        w[j] = (uint32_t)p[2 + 4 * j] | ((uint32_t)p[3 + 4 * j] << 8) | ((uint32_t)p[4 + 4 * j] << 16) |
               ((uint32_t)p[5 + 4 * j] << 24);
      unsigned long long c;
      const uint32_t ul = rd_uint(p + 18, a.s + a.hi, &c);
      if (c) {
        const uint32_t sl = lookup_slot(a.table, a.mask, w[0], w[1], w[2], w[3]);
        if (sl == 0xffffffffu) atomicOr(a.flags, 4u);
        a.col_member[o] = a.member[i];
        a.col_actor[o] = sl == 0xffffffffu ? 0u : a.table[sl].pad[0];
        a.col_value[o] = c;
        o++;
      }
      p += 18 + ul;
    }
  }
}

// each file's flags word next to its head count in pinned memory (after the emit)
__global__ void k_rdm_flags(RdFiles fa, uint32_t nf) {
  const uint32_t f = threadIdx.x;
  bool ok = true;
  if (f < nf) {
    const uint32_t fl = *fa.f[f].flags;
    fa.f[f].n_cand_dev[1] = fl;
    ok = fl == 0 && fa.f[f].tail_dev && fa.f[f].tail_dev[3] == 1u;
  }
  const bool all = __all(ok);
  if (f == 0 && fa.f[0].go) {
    *fa.f[0].go = all ? 1u : 0u;
    *fa.f[0].go_host = all ? 1u : 0u;
  }
}

}  // namespace

// The descriptors go to the kernels as launch arguments, kRdInline files per launch (a
// descriptor array uploaded with hipMemcpyAsync was a runtime copy -- a blit dispatch -- per stage).
hipError_t launch_orswot_read_multi(hipStream_t s, const OrswotReadArgs* /*d_args*/, const OrswotReadArgs* h_args,
                                    uint32_t nf, int stage, uint32_t* chunk_cnt, uint32_t* chunk_scan,
                                    void* tmp, size_t tmp_bytes) {
  if (nf == 0) return hipSuccess;
  auto files = [&](uint32_t c0) {
    RdFiles r{};
    for (uint32_t i = 0; i < kRdInline && c0 + i < nf; i++) r.f[i] = h_args[c0 + i];
    return r;
  };
  auto part = [&](uint32_t c0) { return std::min<uint32_t>(kRdInline, nf - c0); };
  if (stage == 0) {
    uint32_t nchunks = 0;
    for (uint32_t f = 0; f < nf; f++) nchunks = std::max(nchunks, h_args[f].chunk0 + h_args[f].nchunks);
    auto gx_of = [&](uint32_t c0) {
      uint32_t g = 1;
      for (uint32_t f = c0; f < c0 + part(c0); f++) g = std::max(g, h_args[f].nchunks);
      return g;
    };
    for (uint32_t c0 = 0; c0 < nf; c0 += kRdInline)
      hipLaunchKernelGGL(k_rdm_count, dim3(gx_of(c0), part(c0)), dim3(kB), 0, s, files(c0), chunk_cnt);
    size_t tb = tmp_bytes;
    hipError_t e = ds_excl_sum_u32(tmp, tb, chunk_cnt, chunk_scan, nchunks + 1, s);
    if (e) return e;
    for (uint32_t c0 = 0; c0 < nf; c0 += kRdInline) {
      const RdFiles r = files(c0);
      hipLaunchKernelGGL(k_rdm_write, dim3(gx_of(c0), part(c0)), dim3(kB), 0, s, r, chunk_scan);
      hipLaunchKernelGGL(k_rdm_found, dim3(1), dim3(64), 0, s, r, chunk_scan, part(c0));
    }
    return hipGetLastError();
  }
  for (uint32_t c0 = 0; c0 < nf; c0 += kRdInline) {
    const RdFiles r = files(c0);
    const uint32_t k = part(c0);
    uint32_t gx = 1;
    for (uint32_t f = c0; f < c0 + k; f++) gx = std::max(gx, nblk(std::max<uint64_t>(h_args[f].n_cand, h_args[f].dset_mask + 2ull)));
    if (stage == 1) {
      hipLaunchKernelGGL(k_rdm_skip, dim3(k), dim3(256), 0, s, r);
      hipLaunchKernelGGL(k_rdm_entry, dim3(gx, k), dim3(kB), 0, s, r);
      hipLaunchKernelGGL(k_rdm_chain, dim3(gx, k), dim3(kB), 0, s, r);
      hipLaunchKernelGGL(k_rdm_dups, dim3(gx, k), dim3(kB), 0, s, r);
      uint32_t gt = 1;
      for (uint32_t f = c0; f < c0 + k; f++) gt = std::max(gt, (h_args[f].n_cand + kScanTile - 1) / kScanTile);
      hipLaunchKernelGGL(k_rdm_tile_sums, dim3(gt, k), dim3(kB), 0, s, r);
      hipLaunchKernelGGL(k_rdm_tile_scan, dim3(gt, k), dim3(kB), 0, s, r);
      hipLaunchKernelGGL(k_rdm_tail, dim3(k), dim3(kB), 0, s, r);
    } else {
      hipLaunchKernelGGL(k_rdm_emit, dim3(gx, k), dim3(kB), 0, s, r);
      hipLaunchKernelGGL(k_rdm_flags, dim3(1), dim3(64), 0, s, r, k);
    }
  }
  return hipGetLastError();
}

size_t orswot_read_multi_tmp_bytes(uint32_t nchunks) {
  size_t b = 0;
  (void)ds_excl_sum_u32(nullptr, b, nullptr, nullptr, nchunks + 1, nullptr);
  return b + 256;
}

uint32_t orswot_read_chunks(uint64_t lo, uint64_t hi) {
  return hi > lo ? (uint32_t)((hi - lo + kFindChunk - 1) / kFindChunk) : 0u;
}

hipError_t launch_orswot_ser(hipStream_t s, OrswotSerScratch& sc, const OrswotSerArgs& in) {
  hipError_t e = launch_orswot_ser_sort(s, sc, in.n);
  return e ? e : launch_orswot_ser_write(s, sc, in);
}

hipError_t launch_orswot_ser_sort(hipStream_t s, OrswotSerScratch& sc, uint32_t n) {
  // pairs (member, actor id, value) in collect order -> sorted by (member, rank): the hand-written
  // radix sort of the packed (member, rank) key when it fits 64 bits (ce_ser_sort.hip; CE_SER_CUB=1:
  // hipCUB's sort of the same key, for A/B), else (or CE_SER_TWO_SORTS=1) the general form -- sort
  // by rank, then stably by member, LSD order -- and a gather
  hipError_t e;
  const int kb = sc.member_bits + sc.rank_bits;
#if CE_FUSED_DIAG
  static const bool cub = getenv("CE_SER_CUB") != nullptr;  // diagnostics build: hipCUB's sort, A/B
#else
  constexpr bool cub = false;
#endif
  const bool two = getenv("CE_SER_TWO_SORTS") != nullptr;  // (the tests flip it)
  if (n && kb <= 64 && !two && !cub && n < (1u << 30)) {
    SerSortArgs a{};
    a.member_in = sc.member_in;
    a.actor_in = sc.actor_in;
    a.value_in = sc.value_in;
    a.rank_of_id = sc.rank_of_id;
    a.id_of_rank = sc.id_of_rank;
    a.rank_bits = sc.rank_bits;
    a.key_bits = kb;
    a.n = n;
    a.par = (*sc.sort_gen)++ & 1u;
    a.hist = sc.sort_state;
    a.ticket = a.hist + 2 * 8 * kSortMaxPlaces * 256;
    a.look = a.hist + kSortStateHead;
    a.member_out = sc.member_sorted;
    a.actor_out = sc.actor_sorted;
    a.value_out = sc.value_sorted;
    void* kbuf[2] = {kb <= 32 ? (void*)sc.k32a : (void*)sc.k64a, kb <= 32 ? (void*)sc.k32b : (void*)sc.k64b};
    unsigned long long* vbuf[2] = {sc.v64a, sc.v64b};
    if ((e = launch_ser_sort(s, a, kbuf, vbuf))) return e;
#if CE_FUSED_DIAG
  } else if (n && kb <= 64 && !two) {
    // (member, rank) in one key: hipCUB's radix sort over member_bits + rank_bits
    size_t tb = sc.tmp_bytes;
    if (kb <= 32) {
      hipLaunchKernelGGL(k_ser_key<uint32_t>, dim3(nblk(n)), dim3(kB), 0, s, sc.actor_in, sc.rank_of_id, sc.member_in,
                         sc.rank_bits, sc.k32a, n);
      if ((e = hipcub::DeviceRadixSort::SortPairs(sc.tmp, tb, sc.k32a, sc.k32b, sc.value_in, sc.value_sorted, (int)n,
                                                   0, kb, s)))
        return e;
      hipLaunchKernelGGL(k_ser_unpack<uint32_t>, dim3(nblk(n)), dim3(kB), 0, s, sc.k32b, sc.rank_bits, sc.id_of_rank,
                         sc.member_sorted, sc.actor_sorted, n);
    } else {
      hipLaunchKernelGGL(k_ser_key<unsigned long long>, dim3(nblk(n)), dim3(kB), 0, s, sc.actor_in, sc.rank_of_id,
                         sc.member_in, sc.rank_bits, sc.k64a, n);
      if ((e = hipcub::DeviceRadixSort::SortPairs(sc.tmp, tb, sc.k64a, sc.member_sorted, sc.value_in, sc.value_sorted,
                                                   (int)n, 0, kb, s)))
        return e;
      hipLaunchKernelGGL(k_ser_unpack<unsigned long long>, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted,
                         sc.rank_bits, sc.id_of_rank, sc.member_sorted, sc.actor_sorted, n);
    }
#endif
  } else if (n) {
    // the general form (keys past 64 bits, CE_SER_TWO_SORTS): two stable pair sorts of the
    // hand-written radix sort (ce_ser_sort.hip), by rank, then by member
    size_t tb = sc.tmp_bytes;
    hipLaunchKernelGGL(k_ser_rank, dim3(nblk(n)), dim3(kB), 0, s, sc.actor_in, sc.rank_of_id, sc.k32a, n);
    hipLaunchKernelGGL(k_ser_iota, dim3(nblk(n)), dim3(kB), 0, s, sc.p32a, n);
    if ((e = sort_pairs_u32(sc.tmp, tb, sc.k32a, sc.k32b, sc.p32a, sc.p32b, n, sc.rank_bits, s)))
      return e;
    hipLaunchKernelGGL(k_ser_gather_member, dim3(nblk(n)), dim3(kB), 0, s, sc.p32b, sc.member_in, sc.k64a, n);
    tb = sc.tmp_bytes;
    if ((e = sort_pairs_u64(sc.tmp, tb, sc.k64a, sc.member_sorted, sc.p32b, sc.p32a, n,
                            sc.member_bits > 0 && sc.member_bits <= 64 ? sc.member_bits : 64, s)))
      return e;
    hipLaunchKernelGGL(k_ser_gather2, dim3(nblk(n)), dim3(kB), 0, s, sc.p32a, sc.actor_in, sc.value_in,
                       sc.actor_sorted, sc.value_sorted, n);
  }
  const uint32_t nt = (n + kSerTile - 1) / kSerTile;
  if (n && nt <= 4096 && 8ull * nt <= sc.tmp_bytes) {
    // (an apply block sums the tile totals before it: up to 4096 tiles, 8M pairs)
    uint32_t* ts = static_cast<uint32_t*>(sc.tmp);
    hipLaunchKernelGGL(k_ser_head_tiles, dim3(nt), dim3(kB), 0, s, sc.member_sorted, n, ts);
    hipLaunchKernelGGL(k_ser_head_apply, dim3(nt), dim3(kB), 0, s, sc.member_sorted, n, ts, sc.head, sc.hrank, sc.seg);
    hipLaunchKernelGGL(k_ser_len_tiles, dim3(nt), dim3(kB), 0, s, sc.member_sorted, sc.value_sorted, sc.head, sc.hrank,
                       sc.seg, n, ts + nt);
    hipLaunchKernelGGL(k_ser_len_apply, dim3(nt), dim3(kB), 0, s, sc.member_sorted, sc.value_sorted, sc.head, sc.hrank,
                       sc.seg, n, ts + nt, sc.len, sc.pos);
  } else if (n) {
    size_t tb = sc.tmp_bytes;
    hipLaunchKernelGGL(k_ser_head, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.head, n);
    tb = sc.tmp_bytes;
    if ((e = ds_excl_sum_u32(sc.tmp, tb, sc.head, sc.hrank, n, s))) return e;
    hipLaunchKernelGGL(k_ser_seg, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.head, sc.hrank, sc.seg, n);
    hipLaunchKernelGGL(k_ser_len, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.value_sorted, sc.head,
                       sc.hrank, sc.seg, sc.len, n);
    tb = sc.tmp_bytes;
    if ((e = ds_excl_sum_u32(sc.tmp, tb, sc.len, sc.pos, n, s))) return e;
  }
  return hipGetLastError();
}

hipError_t launch_orswot_ser_write(hipStream_t s, const OrswotSerScratch& sc, const OrswotSerArgs& in) {
  OrswotSerArgs a = in;
  const uint32_t n = a.n;
  if (n) {
    a.member = sc.member_sorted;
    a.actor = sc.actor_sorted;
    a.value = sc.value_sorted;
    a.head = sc.head;
    a.hrank = sc.hrank;
    a.seg = sc.seg;
    a.pos = sc.pos;
    a.len = sc.len;
    hipLaunchKernelGGL(k_ser_write, dim3(nblk(n)), dim3(kB), 0, s, a);
  }
  hipLaunchKernelGGL(k_ser_tail, dim3(64), dim3(kB), 0, s, a);
  return hipGetLastError();
}

static size_t cached_tmp_bytes(uint32_t n, size_t (*raw)(uint32_t), std::map<uint32_t, size_t>& cache) {
  static std::mutex mu;
  uint32_t p = 1;
  while (p < n && p < 0x80000000u) p <<= 1;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(p);
  if (it != cache.end()) return it->second;
  const size_t v = raw(p);
  cache[p] = v;
  return v;
}

static size_t ser_tmp_bytes_raw(uint32_t n) {
  size_t a = 0, b = 0, c = 0;
  (void)sort_pairs_u32(nullptr, a, nullptr, nullptr, nullptr, nullptr, n, 32, nullptr);
  (void)sort_pairs_u64(nullptr, b, nullptr, nullptr, nullptr, nullptr, n, 64, nullptr);
  (void)ds_excl_sum_u32(nullptr, c, nullptr, nullptr, n, nullptr);
  size_t d = 0, e = 0;
#if CE_FUSED_DIAG  // CE_SER_CUB: the packed-key sorts through hipCUB, u64 values
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, d, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (unsigned long long*)nullptr, (unsigned long long*)nullptr, (int)n, 0, 32);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, e, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (unsigned long long*)nullptr, (int)n, 0, 64);
#endif
  return std::max(std::max(a, b), std::max(c, std::max(d, e))) + 256;
}

size_t orswot_ser_tmp_bytes(uint32_t n) {
  static std::map<uint32_t, size_t> cache;
  return cached_tmp_bytes(n, ser_tmp_bytes_raw, cache);
}

}  // namespace ce
