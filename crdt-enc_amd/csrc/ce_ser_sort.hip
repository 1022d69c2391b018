// ce_ser_sort.hip -- the Orswot serializer's sort: the live (member, actor, counter) pairs of a
// collect ordered by (member, actor UUID rank), as the StateWrapper's entries map is written
// (crdts Orswot's BTreeMap<M, VClock> -> rmp-serde; crdt-enc/src/lib.rs:332-380).
//
// An LSD radix sort over the packed key member << rank_bits | rank (unique per pair), 8-bit
// digits, one kernel per digit place and one histogram kernel before them -- no runtime fills:
//   k_sort_hist   every place's digit counts (LDS per block, then one no-return add per digit
//                 into hist[par]); zeroes what the passes need zero: their lookback words and tile
//                 tickets, and the other parity's histogram (the next sort's)
//   k_sort_pass   one 4096-item tile per workgroup, tiles in ticket order: the tile's items
//                 ranked stably per digit (per-wave match on the digit bits, wave counters in
//                 LDS), the tile's digit counts published for the tiles after it and its prefix
//                 found by looking back over the tiles before it (decoupled look-back; the words
//                 are agent-scope atomics), then the tile reordered in LDS and written out as
//                 contiguous digit runs.  The first pass builds the key from the collect columns
//                 (member, actor id -> rank); the last writes the serializer's sorted member /
//                 actor id / counter columns directly.
// Stability: a wave owns 1024 consecutive items and walks them 64 at a time in order, the waves'
// counts are prefixed in wave order and the tiles' in ticket order, so equal digits keep their
// input order, as LSD needs.
#include "ce_dotset_io.h"

namespace ce {
namespace {

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / 64;
constexpr int kSortPerLane = 16;
constexpr uint32_t kSortTile = kSortThreads * kSortPerLane;  // 4096
constexpr int kDigitBits = 8;
constexpr uint32_t kDigits = 1u << kDigitBits;
constexpr uint32_t kFlagAgg = 1u << 30, kFlagInc = 2u << 30, kCountMask = (1u << 30) - 1;
static_assert(kDigits == kSortThreads, "one lane per digit in the tile bookkeeping");
constexpr int kLookWindow = 16;
// the histogram in kHistReps replicas (block b adds into replica b % kHistReps, ~ its XCD): a
// digit's count is then ~tiles / 8 same-address adds per replica (~60 ns each across XCDs: one
// copy took ~24 us at C3's 406 tiles); the passes sum the replicas
constexpr uint32_t kHistReps = 8;
static_assert(kHistReps * kSortMaxPlaces * kDigits * 2 + kSortMaxPlaces <= kSortStateHead, "state layout");

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename K>
__device__ __forceinline__ K pair_key(const SerSortArgs& a, uint32_t i) {
  if (a.generic) return reinterpret_cast<const K*>(a.gk_in)[i];
  return ((K)a.member_in[i] << a.rank_bits) | (K)a.rank_of_id[a.actor_in[i]];
}

// block-wide exclusive scan of one value per lane (256 lanes); returns the lane's prefix and
// *total the sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < kSortWaves; k++) {
    before += (uint32_t)k < w ? wsum[k] : 0u;
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

template <typename K>
__global__ void __launch_bounds__(kSortThreads) k_sort_hist(SerSortArgs a) {
  __shared__ uint32_t lh[kSortMaxPlaces][kDigits];
  const uint32_t t = threadIdx.x;
  // zero what this sort's passes need zero, and the next sort's histogram
  const uint32_t nz = a.places * a.tiles * kDigits;
  for (uint32_t i = blockIdx.x * kSortThreads + t; i < nz; i += gridDim.x * kSortThreads) a.look[i] = 0;
  if (blockIdx.x == 0) {
    if (t < kSortMaxPlaces) a.ticket[t] = 0;
    for (uint32_t i = t; i < kHistReps * kSortMaxPlaces * kDigits; i += kSortThreads)
      a.hist[(size_t)(a.par ^ 1) * kHistReps * kSortMaxPlaces * kDigits + i] = 0;
  }
  for (uint32_t p = 0; p < a.places; p++) lh[p][t] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * kSortTile + t; i < min(a.n, (blockIdx.x + 1) * kSortTile); i += kSortThreads) {
    const K key = pair_key<K>(a, i);
    for (uint32_t p = 0; p < a.places; p++) atomicAdd(&lh[p][(uint32_t)(key >> (p * kDigitBits)) & (kDigits - 1)], 1u);
  }
  __syncthreads();
  uint32_t* h = a.hist + ((size_t)a.par * kHistReps + blockIdx.x % kHistReps) * kSortMaxPlaces * kDigits;
  for (uint32_t p = 0; p < a.places; p++)
    if (lh[p][t]) atomicAdd(h + p * kDigits + t, lh[p][t]);
}

template <typename K, bool FIRST, bool LAST>
__global__ void __launch_bounds__(kSortThreads) k_sort_pass(SerSortArgs a, uint32_t place) {
  __shared__ K lkey[kSortTile];
  __shared__ unsigned long long lval[kSortTile];
  __shared__ uint32_t wcnt[kSortWaves][kDigits];  // per wave: items of each digit so far
  __shared__ uint32_t tstart[kDigits], gofs[kDigits], wsum[kSortWaves], tile_s;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  // the look-back waits only on earlier tiles: in dispatch order (an atomic ticket) when the tiles
  // do not all fit on the GPU at once, else by blockIdx -- every tile is resident, so each one's
  // predecessors run; the ticket is a same-address atomic per tile, ~60 ns each across XCDs
  // (~25 us per pass at C3's 415 tiles)
  if (t == 0) tile_s = a.ticketed ? atomicAdd(a.ticket + place, 1u) : blockIdx.x;
#pragma unroll
  for (int k = 0; k < kSortWaves; k++) wcnt[k][t] = 0;
  __syncthreads();
  const uint32_t tile = tile_s, base = tile * kSortTile;
  const uint32_t shift = place * kDigitBits;
  // wave w's items: base + 1024 w + 64 k + lane, k = 0..15 (in input order)
  K key[kSortPerLane];
  unsigned long long val[kSortPerLane];
  uint32_t rk[kSortPerLane];
#pragma unroll
  for (int k = 0; k < kSortPerLane; k++) {
    const uint32_t i = base + w * (64 * kSortPerLane) + k * 64 + lane;
    key[k] = 0;
    val[k] = 0;
    if (i < a.n) {
      if (FIRST) {
        key[k] = pair_key<K>(a, i);
        val[k] = a.generic ? (unsigned long long)a.gv_in[i] : a.value_in[i];
      } else {
        key[k] = reinterpret_cast<const K*>(a.keys_in)[i];
        val[k] = a.vals_in[i];
      }
    }
  }
  const unsigned long long lt = (1ull << lane) - 1;
#pragma unroll
  for (int k = 0; k < kSortPerLane; k++) {
    const uint32_t i = base + w * (64 * kSortPerLane) + k * 64 + lane;
    const bool ok = i < a.n;
    const uint32_t d = (uint32_t)(key[k] >> shift) & (kDigits - 1);
    // lanes holding the same digit: the digit's bits matched by ballots
    unsigned long long peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < kDigitBits; b++) {
      const unsigned long long m = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const uint32_t before = wcnt[w][d];  // every peer reads the count before the leader adds
    rk[k] = before + (uint32_t)__popcll(peers & lt);
    if (ok && (peers & lt) == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // digit t: the tile's count, the waves' bases inside it, the tile-local start of the digit
  uint32_t tot = 0, wb[kSortWaves];
#pragma unroll
  for (int k = 0; k < kSortWaves; k++) {
    wb[k] = tot;
    tot += wcnt[k][t];
  }
  // publish the tile's count of digit t, then its prefix over the tiles before (look-back)
  uint32_t* look = a.look + ((size_t)place * a.tiles) * kDigits;
  uint32_t prefix = 0;
  if (tile == 0) {
    st_agent(look + t, tot | kFlagInc);
  } else {
    st_agent(look + (size_t)tile * kDigits + t, tot | kFlagAgg);
    // kLookWindow predecessors' words per round, their loads in flight together (a cross-XCD
    // load is ~1 us: one at a time, a walk over a few dozen aggregates cost tens of us)
    for (int32_t j = (int32_t)tile - 1; j >= 0;) {
      uint32_t v[kLookWindow];
#pragma unroll
      for (int q = 0; q < kLookWindow; q++) v[q] = j - q >= 0 ? ld_agent(look + (size_t)(j - q) * kDigits + t) : kFlagInc;
      int q = 0;
      bool found = false;
      for (; q < kLookWindow; q++) {
        if (v[q] == 0) break;  // not published yet: poll again from there
        prefix += v[q] & kCountMask;
        if (v[q] & kFlagInc) {
          found = true;
          break;
        }
      }
      if (found) break;
      j -= q;
      if (q < kLookWindow) __builtin_amdgcn_s_sleep(1);
    }
    st_agent(look + (size_t)tile * kDigits + t, (prefix + tot) | kFlagInc);
  }
  const uint32_t* h = a.hist + (size_t)a.par * kHistReps * kSortMaxPlaces * kDigits + place * kDigits;
  uint32_t hv = 0;
#pragma unroll
  for (uint32_t r = 0; r < kHistReps; r++) hv += h[(size_t)r * kSortMaxPlaces * kDigits + t];
  uint32_t all;
  const uint32_t hx = block_excl_scan(hv, wsum, &all);
  gofs[t] = hx + prefix;
  const uint32_t ts = block_excl_scan(tot, wsum, &all);
  tstart[t] = ts;
#pragma unroll
  for (int k = 0; k < kSortWaves; k++) wcnt[k][t] = wb[k] + ts;  // tile-local base of (wave k, digit t)
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSortPerLane; k++) {
    const uint32_t i = base + w * (64 * kSortPerLane) + k * 64 + lane;
    if (i >= a.n) continue;
    const uint32_t d = (uint32_t)(key[k] >> shift) & (kDigits - 1);
    const uint32_t lp = wcnt[w][d] + rk[k];
    lkey[lp] = key[k];
    lval[lp] = val[k];
  }
  __syncthreads();
  // the tile in digit order: consecutive lanes write consecutive places of a digit's run
  const uint32_t tn = min(kSortTile, a.n - base);
  for (uint32_t lp = t; lp < tn; lp += kSortThreads) {
    const K kk = lkey[lp];
    const uint32_t d = (uint32_t)(kk >> shift) & (kDigits - 1);
    const uint32_t g = gofs[d] + (lp - tstart[d]);
    if (LAST && a.generic) {
      reinterpret_cast<K*>(a.gk_out)[g] = kk;
      a.gv_out[g] = (uint32_t)lval[lp];
    } else if (LAST) {
      a.member_out[g] = (unsigned long long)(kk >> a.rank_bits);
      a.actor_out[g] = a.id_of_rank[(uint32_t)kk & ((1u << a.rank_bits) - 1)];
      a.value_out[g] = lval[lp];
    } else {
      reinterpret_cast<K*>(a.keys_out)[g] = kk;
      a.vals_out[g] = lval[lp];
    }
  }
}

template <typename K, bool FIRST, bool LAST>
void pass_launch(hipStream_t s, SerSortArgs a, uint32_t p) {
  // resident workgroups of this pass on the whole GPU (the occupancy calculator: LDS-bound)
  static const uint32_t res = [] {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_pass<K, FIRST, LAST>, kSortThreads, 0) != hipSuccess)
      return 0u;
    return (uint32_t)(per_cu > 0 ? per_cu : 0) * (uint32_t)(cus > 0 ? cus : 0);
  }();
  // Without the ticket the look-back relies on in-order workgroup dispatch: the command processor
  // hands out a grid's workgroups in blockIdx order, so every tile a tile waits on was dispatched
  // before it and holds a CU -- even when other streams' kernels (RCCL, the side stream) occupy
  // part of the GPU and not every tile is resident at once.  CE_SORT_TICKET=1 takes the ticket
  // (dispatch order made explicit) on any grid.
  static const bool force_ticket = getenv("CE_SORT_TICKET") != nullptr;  // (tests / A/B)
  a.ticketed = force_ticket || a.tiles > res ? 1u : 0u;
  hipLaunchKernelGGL((k_sort_pass<K, FIRST, LAST>), dim3(a.tiles), dim3(kSortThreads), 0, s, a, p);
}

template <typename K>
hipError_t sort_typed(hipStream_t s, SerSortArgs a, void* const kbuf[2], unsigned long long* const vbuf[2]) {
  hipLaunchKernelGGL(k_sort_hist<K>, dim3(a.tiles), dim3(kSortThreads), 0, s, a);
  for (uint32_t p = 0; p < a.places; p++) {
    const bool first = p == 0, last = p + 1 == a.places;
    a.keys_in = kbuf[(p + 1) & 1];
    a.vals_in = vbuf[(p + 1) & 1];
    a.keys_out = kbuf[p & 1];
    a.vals_out = vbuf[p & 1];
    if (first && last) pass_launch<K, true, true>(s, a, p);
    else if (first) pass_launch<K, true, false>(s, a, p);
    else if (last) pass_launch<K, false, true>(s, a, p);
    else pass_launch<K, false, false>(s, a, p);
  }
  return hipGetLastError();
}

// the generic sorts' state is scratch, not kept across sorts: this sort's histogram and tickets
// start at zero (the serializer's persistent state has k_sort_hist zero the next sort's instead)
__global__ void __launch_bounds__(kSortThreads) k_sort_zero(uint32_t* hist) {
  for (uint32_t i = blockIdx.x * kSortThreads + threadIdx.x; i < kSortStateHead; i += gridDim.x * kSortThreads) hist[i] = 0;
}

template <typename K>
hipError_t sort_pairs_t(void* tmp, size_t& tb, const K* kin, K* kout, const uint32_t* vin, uint32_t* vout,
                        uint32_t n, int bits, hipStream_t s) {
  // scratch: sort state | keys x 2 | u64 values x 2 (the passes' ping-pong buffers)
  const uint32_t tiles = (n + kSortTile - 1) / kSortTile;
  const size_t sw = ((size_t)kSortStateHead + (size_t)kSortMaxPlaces * tiles * kDigits) * 4;
  const size_t a0 = (sw + 255) & ~(size_t)255, kb = ((size_t)n * sizeof(K) + 255) & ~(size_t)255,
               vb = ((size_t)n * 8 + 255) & ~(size_t)255;
  const size_t need = a0 + 2 * kb + 2 * vb + 256;
  if (!tmp) {
    tb = need;
    return hipSuccess;
  }
  if (tb < need) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  uint8_t* base = static_cast<uint8_t*>(tmp);
  SerSortArgs a{};
  a.generic = 1;
  a.gk_in = kin;
  a.gk_out = kout;
  a.gv_in = vin;
  a.gv_out = vout;
  a.n = n;
  a.key_bits = bits > 0 ? bits : (int)(8 * sizeof(K));
  a.par = 0;
  a.hist = reinterpret_cast<uint32_t*>(base);
  a.ticket = a.hist + 2 * 8 * kSortMaxPlaces * 256;
  a.look = a.hist + kSortStateHead;
  a.tiles = tiles;
  a.places = (uint32_t)((a.key_bits + kDigitBits - 1) / kDigitBits);
  if (a.places == 0) a.places = 1;
  void* kbuf[2] = {base + a0, base + a0 + kb};
  unsigned long long* vbuf[2] = {reinterpret_cast<unsigned long long*>(base + a0 + 2 * kb),
                                 reinterpret_cast<unsigned long long*>(base + a0 + 2 * kb + vb)};
  hipLaunchKernelGGL(k_sort_zero, dim3(16), dim3(kSortThreads), 0, s, a.hist);
  return sort_typed<K>(s, a, kbuf, vbuf);
}

}  // namespace

hipError_t sort_pairs_u32(void* tmp, size_t& tb, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                          uint32_t* vout, uint32_t n, int bits, hipStream_t s) {
  return sort_pairs_t<uint32_t>(tmp, tb, kin, kout, vin, vout, n, bits > 32 ? 32 : bits, s);
}

hipError_t sort_pairs_u64(void* tmp, size_t& tb, const unsigned long long* kin, unsigned long long* kout,
                          const uint32_t* vin, uint32_t* vout, uint32_t n, int bits, hipStream_t s) {
  return sort_pairs_t<unsigned long long>(tmp, tb, kin, kout, vin, vout, n, bits > 64 ? 64 : bits, s);
}

uint32_t ser_sort_tiles(uint32_t n) { return (n + kSortTile - 1) / kSortTile; }

hipError_t launch_ser_sort(hipStream_t s, const SerSortArgs& in, void* const kbuf[2],
                           unsigned long long* const vbuf[2]) {
  SerSortArgs a = in;
  if (a.n == 0) return hipSuccess;
  a.tiles = ser_sort_tiles(a.n);
  a.places = (uint32_t)((a.key_bits + kDigitBits - 1) / kDigitBits);
  if (a.places == 0) a.places = 1;
  return a.key_bits <= 32 ? sort_typed<uint32_t>(s, a, kbuf, vbuf) : sort_typed<unsigned long long>(s, a, kbuf, vbuf);
}

}  // namespace ce
