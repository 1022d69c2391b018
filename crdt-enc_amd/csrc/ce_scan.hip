// ce_scan.hip -- device-wide exclusive scans for the dot-set path, in place of hipCUB's.
//
// hipCUB's DeviceScan (rocPRIM's look-back scan) queries the device properties on the host at
// every call (to pick a sleep variant of its look-back state for one older chip); in the HIP
// runtime torch loads that query costs tens of microseconds, which a C3 step paid ~5 times while
// the GPU waited for the next launch (profiles/r04_c3_step.txt).  These scans are plain launches
// over 2048-item tiles: tile totals, then the tiles rescanned with their offsets (each block
// sums the totals before its tile; past 4096 tiles one block scans the totals first).  Sizes
// come from the launch, nothing is read back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#if CE_FUSED_DIAG  // hipCUB only for the diagnostics build's A/B (CE_HIPCUB_SCAN)
#include <hipcub/hipcub.hpp>
#endif

#include <algorithm>
#include <cstdlib>

#include "ce_dotset.h"

namespace ce {
namespace {

constexpr int kB = 256;
constexpr int kItems = 8;
constexpr uint32_t kTile = kB * kItems;

uint32_t tiles_for(uint64_t n) { return (uint32_t)((n + kTile - 1) / kTile); }

// block-wide inclusive sum of one value per thread (kB threads, 4 waves)
__device__ uint32_t block_incl_sum(uint32_t v, uint32_t* lds) {
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

__global__ void __launch_bounds__(kB) k_sum_tiles(const uint32_t* in, uint64_t n, uint32_t* tile_sum) {
  __shared__ uint32_t lds[kB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++)
    if (i0 + k < n) s += in[i0 + k];
  s = block_incl_sum(s, lds);
  if (threadIdx.x == kB - 1) tile_sum[blockIdx.x] = s;
}

// one block: tile_sum[0..nt) -> exclusive offsets, in place
__global__ void __launch_bounds__(kB) k_scan_tile_sums(uint32_t* tile_sum, uint32_t nt) {
  __shared__ uint32_t lds[kB / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nt; base += kB) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nt ? tile_sum[i] : 0u;
    const uint32_t inc = block_incl_sum(v, lds);
    const uint32_t c = carry;
    if (i < nt) tile_sum[i] = c + inc - v;
    __syncthreads();
    if (threadIdx.x == kB - 1) carry = c + inc;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kB) k_sum_apply(const uint32_t* in, uint32_t* out, uint64_t n,
                                                  const uint32_t* tile_off) {
  __shared__ uint32_t lds[kB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  uint32_t v[kItems];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : 0u;
    s += v[k];
  }
  uint32_t run = block_incl_sum(s, lds) - s + tile_off[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
}

// k_sum_apply with the tile's offset summed from the totals before it (no separate scan of the
// totals: one launch less per scan; the reads grow as tiles^2 / 2, so only up to kApplyScanTiles)
constexpr uint32_t kApplyScanTiles = 4096;
__global__ void __launch_bounds__(kB) k_sum_apply_direct(const uint32_t* in, uint32_t* out, uint64_t n,
                                                         const uint32_t* tile_sum) {
  __shared__ uint32_t lds[kB / 64];
  __shared__ uint32_t off;
  uint32_t b = 0;
  for (uint32_t x = threadIdx.x; x < blockIdx.x; x += kB) b += tile_sum[x];
  b = block_incl_sum(b, lds);
  if (threadIdx.x == kB - 1) off = b;
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  uint32_t v[kItems];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    v[k] = i0 + k < n ? in[i0 + k] : 0u;
    s += v[k];
  }
  uint32_t run = block_incl_sum(s, lds) - s + off;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
}

// ---- segmented exclusive max of u64 values over runs of equal u32 keys ----
struct Seg {
  uint32_t kf, kl;         // first / last key
  unsigned long long mx;   // max over the final run (key kl)
  uint32_t uni, empty;     // one run throughout / no items
};

__device__ Seg seg_combine(const Seg& a, const Seg& b) {
  if (a.empty) return b;
  if (b.empty) return a;
  Seg r;
  r.kf = a.kf;
  r.kl = b.kl;
  r.uni = a.uni && b.uni && a.kl == b.kf;
  r.mx = (b.uni && b.kf == a.kl) ? (a.mx > b.mx ? a.mx : b.mx) : b.mx;
  r.empty = 0;
  return r;
}

__device__ Seg seg_shfl_up(const Seg& s, int o) {
  Seg r;
  r.kf = __shfl_up(s.kf, o);
  r.kl = __shfl_up(s.kl, o);
  r.mx = ((unsigned long long)(uint32_t)__shfl_up((int)(uint32_t)(s.mx >> 32), o) << 32) |
         (uint32_t)__shfl_up((int)(uint32_t)s.mx, o);
  r.uni = __shfl_up(s.uni, o);
  r.empty = __shfl_up(s.empty, o);
  return r;
}

// block-wide EXCLUSIVE segmented scan of the threads' summaries (the identity for thread 0)
__device__ Seg block_excl_seg(Seg s, Seg* lds) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  Seg inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Seg y = seg_shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc = seg_combine(y, inc);
  }
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  Seg pre;
  pre.empty = 1;
  pre.kf = pre.kl = 0;
  pre.mx = 0;
  pre.uni = 1;
  for (uint32_t k = 0; k < w; k++) pre = seg_combine(pre, lds[k]);
  __syncthreads();
  // exclusive within the wave: the previous lane's inclusive value
  Seg prev = seg_shfl_up(inc, 1);
  if (lane == 0) {
    prev.empty = 1;
    prev.kf = prev.kl = 0;
    prev.mx = 0;
    prev.uni = 1;
  }
  return seg_combine(pre, prev);
}

__device__ Seg thread_seg(const uint32_t* keys, const unsigned long long* vals, uint64_t i0, uint64_t n) {
  Seg s;
  s.empty = i0 >= n;
  s.kf = s.kl = 0;
  s.mx = 0;
  s.uni = 1;
  if (s.empty) return s;
  s.kf = s.kl = keys[i0];
  s.mx = vals[i0];
#pragma unroll
  for (int k = 1; k < kItems; k++) {
    if (i0 + k >= n) break;
    const uint32_t kk = keys[i0 + k];
    const unsigned long long v = vals[i0 + k];
    if (kk == s.kl) {
      s.mx = v > s.mx ? v : s.mx;
    } else {
      s.kl = kk;
      s.mx = v;
      s.uni = 0;
    }
  }
  return s;
}

__global__ void __launch_bounds__(kB) k_seg_tiles(const uint32_t* keys, const unsigned long long* vals, uint64_t n,
                                                  Seg* tile_seg) {
  __shared__ Seg lds[kB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  const Seg s = thread_seg(keys, vals, i0, n);
  const Seg ex = block_excl_seg(s, lds);
  if (threadIdx.x == kB - 1) tile_seg[blockIdx.x] = seg_combine(ex, s);
}

// one block: tile summaries -> the carry INTO each tile, in place (kB tiles per trip)
__global__ void __launch_bounds__(kB) k_seg_carry(Seg* tile_seg, uint32_t nt) {
  __shared__ Seg lds[kB / 64];
  __shared__ Seg carry;
  if (threadIdx.x == 0) {
    carry.empty = 1;
    carry.kf = carry.kl = 0;
    carry.mx = 0;
    carry.uni = 1;
  }
  __syncthreads();
  for (uint32_t base = 0; base < nt; base += kB) {
    const uint32_t i = base + threadIdx.x;
    Seg x;
    x.empty = 1;
    x.kf = x.kl = 0;
    x.mx = 0;
    x.uni = 1;
    if (i < nt) x = tile_seg[i];
    const Seg ex = block_excl_seg(x, lds);
    const Seg c = carry;
    if (i < nt) tile_seg[i] = seg_combine(c, ex);
    __syncthreads();
    if (threadIdx.x == kB - 1) carry = seg_combine(c, seg_combine(ex, x));
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kB) k_seg_apply(const uint32_t* keys, const unsigned long long* vals,
                                                  unsigned long long* out, uint64_t n, const Seg* tile_in) {
  __shared__ Seg lds[kB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  const Seg s = thread_seg(keys, vals, i0, n);
  const Seg c = seg_combine(tile_in[blockIdx.x], block_excl_seg(s, lds));
  if (s.empty) return;
  uint32_t rk = c.kl;
  unsigned long long rm = c.empty ? 0ull : c.mx;
  if (c.empty) rk = ~keys[i0];  // forces a new run at the first item
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    if (i0 + k >= n) break;
    const uint32_t kk = keys[i0 + k];
    const unsigned long long v = vals[i0 + k];
    if (kk != rk) {
      rk = kk;
      rm = 0;
    }
    out[i0 + k] = rm;
    rm = v > rm ? v : rm;
  }
}

// k_seg_apply with the carry into the tile combined from the tile summaries before it (a lane
// folds a contiguous run of them in order, a block scan orders the lanes): no k_seg_carry launch
// up to kApplyScanTiles tiles
__global__ void __launch_bounds__(kB) k_seg_apply_direct(const uint32_t* keys, const unsigned long long* vals,
                                                         unsigned long long* out, uint64_t n, const Seg* tile_seg) {
  __shared__ Seg lds[kB / 64];
  __shared__ Seg carry;
  const uint32_t nb = blockIdx.x, per = (nb + kB - 1) / kB;
  Seg agg;
  agg.empty = 1;
  agg.kf = agg.kl = 0;
  agg.mx = 0;
  agg.uni = 1;
  for (uint32_t j = threadIdx.x * per; j < min(nb, (threadIdx.x + 1) * per); j++) agg = seg_combine(agg, tile_seg[j]);
  const Seg ea = block_excl_seg(agg, lds);
  if (threadIdx.x == kB - 1) carry = seg_combine(ea, agg);
  __syncthreads();
  const Seg tile_in = carry;
  const uint64_t i0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kItems;
  const Seg s = thread_seg(keys, vals, i0, n);
  const Seg c = seg_combine(tile_in, block_excl_seg(s, lds));
  if (s.empty) return;
  uint32_t rk = c.kl;
  unsigned long long rm = c.empty ? 0ull : c.mx;
  if (c.empty) rk = ~keys[i0];  // forces a new run at the first item
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    if (i0 + k >= n) break;
    const uint32_t kk = keys[i0 + k];
    const unsigned long long v = vals[i0 + k];
    if (kk != rk) {
      rk = kk;
      rm = 0;
    }
    out[i0 + k] = rm;
    rm = v > rm ? v : rm;
  }
}

}  // namespace

namespace {
struct MaxOp {
  __device__ __host__ unsigned long long operator()(unsigned long long a, unsigned long long b) const { return a > b ? a : b; }
};
// CE_HIPCUB_SCAN=1 (diagnostics build only): hipCUB's scans instead, for same-box A/B
bool use_hipcub() {
#if CE_FUSED_DIAG
  static const bool v = getenv("CE_HIPCUB_SCAN") != nullptr;
  return v;
#else
  return false;
#endif
}
// CE_SCAN_3PASS=1 (tests): the three-launch form (tile sums, one carry block, apply) at any size;
// by default it only runs past kApplyScanTiles tiles
bool three_pass() {
  static const bool v = getenv("CE_SCAN_3PASS") != nullptr;
  return v;
}
}  // namespace

hipError_t ds_excl_sum_u32(void* tmp, size_t& tb, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
#if CE_FUSED_DIAG
  if (use_hipcub()) {
    size_t need = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (int)n, s);
    if (!tmp) { tb = std::max<size_t>(need, 4ull * (tiles_for(n) + 1) + 64); return e; }
    return hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, (int)n, s);
  }
#endif
  const uint32_t nt = tiles_for(n);
  const size_t need = 4ull * (nt + 1) + 64;
  if (!tmp) {
    tb = need;
    return hipSuccess;
  }
  if (tb < need) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  uint32_t* ts = static_cast<uint32_t*>(tmp);
  hipLaunchKernelGGL(k_sum_tiles, dim3(nt), dim3(kB), 0, s, in, (uint64_t)n, ts);
  if (nt <= kApplyScanTiles && !three_pass()) {
    hipLaunchKernelGGL(k_sum_apply_direct, dim3(nt), dim3(kB), 0, s, in, out, (uint64_t)n, ts);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_scan_tile_sums, dim3(1), dim3(kB), 0, s, ts, nt);
  hipLaunchKernelGGL(k_sum_apply, dim3(nt), dim3(kB), 0, s, in, out, (uint64_t)n, ts);
  return hipGetLastError();
}

hipError_t ds_excl_max_by_key(void* tmp, size_t& tb, const uint32_t* keys, const unsigned long long* vals,
                              unsigned long long* out, uint32_t n, hipStream_t s) {
#if CE_FUSED_DIAG
  if (use_hipcub()) {
    size_t need = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveScanByKey(nullptr, need, keys, vals, out, MaxOp(), 0ull, (int)n,
                                                          hipcub::Equality(), s);
    if (!tmp) { tb = std::max<size_t>(need, sizeof(Seg) * (tiles_for(n) + 1) + 64); return e; }
    return hipcub::DeviceScan::ExclusiveScanByKey(tmp, tb, keys, vals, out, MaxOp(), 0ull, (int)n,
                                                  hipcub::Equality(), s);
  }
#endif
  const uint32_t nt = tiles_for(n);
  const size_t need = sizeof(Seg) * (nt + 1) + 64;
  if (!tmp) {
    tb = need;
    return hipSuccess;
  }
  if (tb < need) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  Seg* ts = static_cast<Seg*>(tmp);
  hipLaunchKernelGGL(k_seg_tiles, dim3(nt), dim3(kB), 0, s, keys, vals, (uint64_t)n, ts);
  if (nt <= kApplyScanTiles && !three_pass()) {
    hipLaunchKernelGGL(k_seg_apply_direct, dim3(nt), dim3(kB), 0, s, keys, vals, out, (uint64_t)n, ts);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_seg_carry, dim3(1), dim3(kB), 0, s, ts, nt);
  hipLaunchKernelGGL(k_seg_apply, dim3(nt), dim3(kB), 0, s, keys, vals, out, (uint64_t)n, ts);
  return hipGetLastError();
}

}  // namespace ce
