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

#include <hipcub/hipcub.hpp>
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

__global__ void k_ser_write(OrswotSerArgs a) {
  const uint32_t nm = a.hrank[a.n - 1] + a.head[a.n - 1];
  const uint64_t base = a.prefix_len + maplen(nm);
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n; i += gridDim.x * kB) {
    uint8_t* o = a.out + base + a.pos[i];
    if (a.head[i]) {
      const uint32_t e = a.hrank[i];
      o += put_uint(o, a.member[i]);
      o[0] = 0x81; o[1] = 0xa4; o[2] = 'd'; o[3] = 'o'; o[4] = 't'; o[5] = 's';
      o += 6;
      o += put_map(o, a.seg[e + 1] - a.seg[e]);
    }
    o[0] = 0xc4;
    o[1] = 16;
    const uint8_t* u = a.uuid_of_id + 16ull * a.actor[i];
#pragma unroll
    for (int b = 0; b < 16; b++) o[2 + b] = u[b];
    put_uint(o + 18, a.value[i]);
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
// kFindChunk consecutive positions and collects its heads in LDS; one global atomicAdd per block
// reserves their slice of the list (one head every ~50 bytes: per-wave or per-lane atomics on
// the one counter serialised in L2 at ~10 ns each, 217 us per C3 state file)
static constexpr uint32_t kFindPer = 16, kFindChunk = kFindPer * kB, kFindLds = 1024;
__device__ __forceinline__ bool entry_head_at(const uint8_t* s, uint64_t p) {
  if (s[p] != 0x81 || s[p + 1] != 0xa4 || s[p + 2] != 'd' || s[p + 3] != 'o' || s[p + 4] != 't' ||
      s[p + 5] != 's')
    return false;
  const uint8_t m = s[p + 6];
  return (m & 0xf0) == 0x80 || m == 0xde || m == 0xdf;
}

__global__ void __launch_bounds__(kB) k_rd_find(const uint8_t* s, uint64_t lo, uint64_t hi, uint32_t* cand,
                                                uint32_t* n_cand, uint32_t cap) {
  __shared__ uint32_t lcount, lbase;
  __shared__ uint32_t lst[kFindLds];
  for (uint64_t c0 = lo + (uint64_t)blockIdx.x * kFindChunk; c0 < hi; c0 += (uint64_t)gridDim.x * kFindChunk) {
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
#pragma unroll 4
    for (uint32_t k = 0; k < kFindPer; k++) {
      const uint64_t p = c0 + k * kB + threadIdx.x;
      if (p + 7 <= hi && entry_head_at(s, p)) {
        const uint32_t i = atomicAdd(&lcount, 1u);
        if (i < kFindLds) {
          lst[i] = (uint32_t)(p - lo);
        } else {  // more heads than the LDS list holds (adversarial bytes): one by one
          const uint32_t g = atomicAdd(n_cand, 1u);
          if (g < cap) cand[g] = (uint32_t)(p - lo);
        }
      }
    }
    __syncthreads();
    const uint32_t m = lcount < kFindLds ? lcount : kFindLds;
    if (threadIdx.x == 0 && m) lbase = atomicAdd(n_cand, m);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += kB) {
      const uint32_t g = lbase + i;
      if (g < cap) cand[g] = lst[i];
    }
    __syncthreads();
  }
}

// lane per candidate (sorted): parse the entry's VClock from its head; end[i] = byte after it,
// ndots[i] = its non-zero Dots, ok[i] = canonical (UUIDs strictly ascending, uints canonical)
__global__ void k_rd_entry(OrswotReadArgs a) {
  const uint8_t* base = a.s + a.lo;
  const uint8_t* end = a.s + a.hi;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint8_t* p = base + a.cand[i] + 6;
    uint32_t k;
    bool ok = true;
    if ((p[0] & 0xf0) == 0x80) { k = p[0] & 15u; p += 1; }
    else if (p[0] == 0xde) { if (p + 3 > end) ok = false; k = ((uint32_t)p[1] << 8) | p[2]; p += 3; }
    else { if (p + 5 > end) ok = false; k = rd_be32(p + 1); p += 5; }
    uint32_t nz = 0;
    uint32_t prev[4] = {0, 0, 0, 0};
    for (uint32_t d = 0; d < k && ok; d++) {
      if (p + 18 > end || p[0] != 0xc4 || p[1] != 16) { ok = false; break; }
      // big-endian words: byte order = numeric order for the ascending check
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

// lane per entry: its member key must exactly fill [end of the previous entry, its head)
__global__ void k_rd_chain(OrswotReadArgs a) {
  const uint8_t* base = a.s + a.lo;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint32_t start = i == 0 ? 0u : a.end[i - 1];
    const uint32_t head = a.cand[i];
    unsigned long long m = 0;
    const uint32_t ul = start <= head ? rd_uint(base + start, base + head, &m) : 0u;
    if (!ul || start + ul != head || a.end[i] == 0xffffffffu) atomicOr(a.flags, 2u);
    a.member[i] = m;
  }
}

// HashMap<M, VClock> keeps a repeated member's later clock: a file with repeated members goes to
// the host parser (flag 8).  Found by inserting every member into an open-addressing set
// (atomicCAS on the all-ones empty word; all-ones members are counted in the word after the
// set): one launch where a 64-bit radix sort + neighbour compare took a dozen.
__device__ __forceinline__ uint32_t mix_member(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void k_rd_dups_hash(const unsigned long long* member, unsigned long long* set, uint32_t mask,
                               uint32_t* flags, uint32_t n) {
  constexpr unsigned long long kEmpty = ~0ull;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
    const unsigned long long m = member[i];
    if (m == kEmpty) {
      if (atomicAdd(&set[(size_t)mask + 1], 1ull) != kEmpty) atomicOr(flags, 8u);  // second one
      continue;
    }
    uint32_t h = mix_member(m) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
      const unsigned long long old = atomicCAS(&set[h], kEmpty, m);
      if (old == kEmpty) break;
      if (old == m) { atomicOr(flags, 8u); break; }
      h = (h + 1) & mask;
    }
  }
}

// the last entry's end / Dot base / Dot count and the flags word, for one download of all files
__global__ void k_rd_tail(OrswotReadArgs a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const uint32_t l = a.n_cand - 1;
    a.tail_out[0] = a.end[l];
    a.tail_out[1] = a.dbase[l];
    a.tail_out[2] = a.ndots[l];
    a.tail_out[3] = *a.flags;
  }
}

// lane per entry: its non-zero Dots -> (member, actor id, counter) at its exclusive-scan base;
// actor ids from the device actor table (a miss declines the file to the host)
__global__ void k_rd_emit(OrswotReadArgs a) {
  const uint8_t* base = a.s + a.lo;
  for (uint32_t i = blockIdx.x * kB + threadIdx.x; i < a.n_cand; i += gridDim.x * kB) {
    const uint8_t* p = base + a.cand[i] + 6;
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

}  // namespace

hipError_t launch_orswot_ser(hipStream_t s, OrswotSerScratch& sc, const OrswotSerArgs& in) {
  // pairs (member, actor id, value) in collect order -> sorted by (member, rank): sort by rank,
  // then stably by member (LSD order), gather
  OrswotSerArgs a = in;
  const uint32_t n = a.n;
  hipError_t e;
  if (n) {
    size_t tb = sc.tmp_bytes;
    hipLaunchKernelGGL(k_ser_rank, dim3(nblk(n)), dim3(kB), 0, s, sc.actor_in, sc.rank_of_id, sc.k32a, n);
    hipLaunchKernelGGL(k_ser_iota, dim3(nblk(n)), dim3(kB), 0, s, sc.p32a, n);
    if ((e = hipcub::DeviceRadixSort::SortPairs(sc.tmp, tb, sc.k32a, sc.k32b, sc.p32a, sc.p32b, (int)n, 0,
                                                 sc.rank_bits, s)))
      return e;
    hipLaunchKernelGGL(k_ser_gather_member, dim3(nblk(n)), dim3(kB), 0, s, sc.p32b, sc.member_in, sc.k64a, n);
    tb = sc.tmp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(sc.tmp, tb, sc.k64a, sc.member_sorted, sc.p32b, sc.p32a,
                                                 (int)n, 0, 64, s)))
      return e;
    hipLaunchKernelGGL(k_ser_gather2, dim3(nblk(n)), dim3(kB), 0, s, sc.p32a, sc.actor_in, sc.value_in,
                       sc.actor_sorted, sc.value_sorted, n);
    hipLaunchKernelGGL(k_ser_head, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.head, n);
    tb = sc.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(sc.tmp, tb, sc.head, sc.hrank, (int)n, s))) return e;
    hipLaunchKernelGGL(k_ser_seg, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.head, sc.hrank, sc.seg, n);
    hipLaunchKernelGGL(k_ser_len, dim3(nblk(n)), dim3(kB), 0, s, sc.member_sorted, sc.value_sorted, sc.head,
                       sc.hrank, sc.seg, sc.len, n);
    tb = sc.tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(sc.tmp, tb, sc.len, sc.pos, (int)n, s))) return e;
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
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (unsigned long long*)nullptr,
                                           (unsigned long long*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)n, 0, 64);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return std::max(a, std::max(b, c)) + 256;
}

size_t orswot_ser_tmp_bytes(uint32_t n) {
  static std::map<uint32_t, size_t> cache;
  return cached_tmp_bytes(n, ser_tmp_bytes_raw, cache);
}

hipError_t launch_orswot_read(hipStream_t s, OrswotReadArgs a, void* tmp, size_t tmp_bytes, int stage) {
  hipError_t e;
  if (stage == 0) {  // candidates, then sorted by position
    hipLaunchKernelGGL(k_rd_find, dim3(nblk((a.hi - a.lo + kFindPer - 1) / kFindPer)), dim3(kB), 0, s, a.s, a.lo,
                       a.hi, a.cand_raw,
                       a.n_cand_dev, a.cap);
    return hipGetLastError();
  }
  if (stage == 1) {
    size_t tb = tmp_bytes;
    if (a.n_cand) {
      hipLaunchKernelGGL(k_rd_entry, dim3(nblk(a.n_cand)), dim3(kB), 0, s, a);
      hipLaunchKernelGGL(k_rd_chain, dim3(nblk(a.n_cand)), dim3(kB), 0, s, a);
      if ((e = hipMemsetAsync(a.msort, 0xff, 8ull * ((size_t)a.dset_mask + 2), s))) return e;
      hipLaunchKernelGGL(k_rd_dups_hash, dim3(nblk(a.n_cand)), dim3(kB), 0, s, a.member, a.msort, a.dset_mask,
                         a.flags, a.n_cand);
      tb = tmp_bytes;
      if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, a.ndots, a.dbase, (int)a.n_cand, s))) return e;
      if (a.tail_out) hipLaunchKernelGGL(k_rd_tail, dim3(1), dim3(64), 0, s, a);
    }
    return hipGetLastError();
  }
  if (a.n_cand) hipLaunchKernelGGL(k_rd_emit, dim3(nblk(a.n_cand)), dim3(kB), 0, s, a);
  return hipGetLastError();
}

hipError_t hipcub_sort_u32(void* tmp, size_t& tb, const uint32_t* kin, uint32_t* kout, uint32_t n, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(tmp, tb, kin, kout, (int)n, 0, 32, s);
}

// hipCUB's temp-storage queries cost tens of microseconds each on the host; the sizes only
// grow with n, so they are taken once per power of two and cached
static size_t read_tmp_bytes_raw(uint32_t n) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, c, (unsigned long long*)nullptr,
                                          (unsigned long long*)nullptr, (int)n, 0, 64);
  return std::max(a, std::max(b, c)) + 256;
}


size_t orswot_read_tmp_bytes(uint32_t n) {
  static std::map<uint32_t, size_t> cache;
  return cached_tmp_bytes(n, read_tmp_bytes_raw, cache);
}

}  // namespace ce
