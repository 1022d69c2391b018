// ce_shard.hip -- the version gate of read_remote_ops (crdt-enc/src/lib.rs:516-544) when a
// VClock / GCounter batch is partitioned across ranks by op-file address (ce_common.h
// shard_owner): each rank's files of one writer are a subset of that writer's run, so the gate
// is agreed through per-writer statistics reduced over the ranks (ShardStats, ce_common.h).
//
//   k_shard_files   thread per file: contract checks (one run per writer, versions ascending,
//                   the partition owns the file here), the largest held version >= e0, and the
//                   first owned-but-absent version in the gap after the file (or in [e0, v)
//                   before the run's first file >= e0)
//   k_shard_writers thread per writer: the writers without a held version >= e0 walk from e0,
//                   then every word is encoded for all_reduce(MAX) (k_shard_tail: the flags)
//   k_shard_window  one block: the windows [e0, hi) from the reduced stats
//   k_gate_window   thread per file / writer: the gate of the sharded ingest (apply iff
//                   e0 <= v < hi), next_op_versions = hi
#include "ce_kernels.h"
#include "ce_shard.h"

namespace ce {

__device__ __forceinline__ uint32_t owner_of(const uint32_t* wk, uint32_t a, uint64_t v, uint32_t world) {
  const uint4 k = *reinterpret_cast<const uint4*>(wk + 4ull * a);
  return shard_owner(k.x, k.y, k.z, k.w, v, world);
}

// first version u in [lo, end) owned by `rank` (end = ~0: unbounded); ~0 if none, *over when the
// walk passed kShardWalkLimit versions without deciding
__device__ __forceinline__ uint64_t walk_owned(const uint32_t* wk, uint32_t a, uint64_t lo, uint64_t end,
                                               uint32_t rank, uint32_t world, bool* over) {
  uint64_t steps = 0;
  for (uint64_t u = lo; u < end; u++) {
    if (owner_of(wk, a, u, world) == rank) return u;
    if (++steps >= kShardWalkLimit) { *over = true; return ~0ull; }
    if (u == ~0ull - 1) break;
  }
  return ~0ull;
}

__global__ void k_shard_files(ShardArgs s) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s.n) return;
  const uint32_t a = s.fa[i];
  if (a >= s.m) { atomicOr(s.bad, 1u); return; }
  const uint64_t v = s.fv[i];
  const uint64_t e0 = s.e0[a];
  const bool prev = i > 0 && s.fa[i - 1] == a;
  const bool next = i + 1 < s.n && s.fa[i + 1] == a;
  const uint64_t pv = prev ? s.fv[i - 1] : 0;
  bool bad = false;
  if (!prev && atomicAdd(&s.run_count[a], 1u) != 0) bad = true;  // writer split into runs
  if (prev && pv > v) bad = true;                                 // descending inside the run
  if (owner_of(s.writers, a, v, s.world) != s.rank) bad = true;   // another rank's file
  if (v >= e0) {
    s.has_ge[a] = 1;
    if (!next) atomicMax(&s.vmaxp1[a], (unsigned long long)(v + 1));
    bool over = false;
    uint64_t c = ~0ull;
    if (!prev || pv < e0) c = walk_owned(s.writers, a, e0, v, s.rank, s.world, &over);  // [e0, v)
    if (c == ~0ull && !over) {
      const uint64_t nv = next ? s.fv[i + 1] : ~0ull;  // the gap (v, next) of this rank's run
      if (v != ~0ull) c = walk_owned(s.writers, a, v + 1, nv, s.rank, s.world, &over);
    }
    if (over) bad = true;
    if (c != ~0ull) atomicMin(&s.cand[a], (unsigned long long)c);
  }
  if (bad) atomicOr(s.bad, 1u);
}

__global__ void k_shard_writers(ShardArgs s) {
  const uint32_t a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.m) return;
  uint64_t c = s.cand[a];
  if (!s.has_ge[a]) {  // nothing held at or above e0: the first owned version from e0 is absent
    bool over = false;
    c = walk_owned(s.writers, a, s.e0[a], ~0ull, s.rank, s.world, &over);
    if (over) atomicOr(s.bad, 1u);
  }
  s.stats[a] = (long long)(~c ^ kShardFlip);
  s.stats[(uint64_t)s.m + a] = (long long)(s.vmaxp1[a] ^ kShardFlip);
}

__global__ void k_shard_tail(ShardArgs s, uint64_t e0_hash) {
  s.stats[2ull * s.m] = (long long)((uint64_t)(*s.bad ? 1 : 0) ^ kShardFlip);
  s.stats[2ull * s.m + 1] = (long long)(e0_hash ^ kShardFlip);
  s.stats[2ull * s.m + 2] = (long long)(~e0_hash ^ kShardFlip);
}

hipError_t launch_shard_stats(hipStream_t st, const ShardArgs& s, uint64_t e0_hash) {
  if (s.n) hipLaunchKernelGGL(k_shard_files, dim3((s.n + 255) / 256), dim3(256), 0, st, s);
  if (s.m) hipLaunchKernelGGL(k_shard_writers, dim3((s.m + 255) / 256), dim3(256), 0, st, s);
  hipLaunchKernelGGL(k_shard_tail, dim3(1), dim3(1), 0, st, s, e0_hash);
  return hipGetLastError();
}

// One block: the first gapped writer by a block-wide min, then every writer's window.
__global__ __launch_bounds__(1024) void k_shard_window(const long long* stats, const uint64_t* e0,
                                                       uint32_t m, uint64_t* hi) {
  __shared__ uint32_t astar;
  if (threadIdx.x == 0) astar = m;
  __syncthreads();
  for (uint32_t a = threadIdx.x; a < m; a += blockDim.x) {
    const uint64_t cand = ~((uint64_t)stats[a] ^ kShardFlip);
    const uint64_t vmaxp1 = (uint64_t)stats[(uint64_t)m + a] ^ kShardFlip;
    if (vmaxp1 != 0 && cand < vmaxp1) atomicMin(&astar, a);
  }
  __syncthreads();
  const uint32_t as = astar;
  for (uint32_t a = threadIdx.x; a < m; a += blockDim.x) {
    const uint64_t cand = ~((uint64_t)stats[a] ^ kShardFlip);
    const uint64_t vmaxp1 = (uint64_t)stats[(uint64_t)m + a] ^ kShardFlip;
    hi[a] = shard_hi(a, as, e0[a], cand, vmaxp1);
  }
  if (threadIdx.x == 0) {
    const uint64_t bad = (uint64_t)stats[2ull * m] ^ kShardFlip;
    const uint64_t h = (uint64_t)stats[2ull * m + 1] ^ kShardFlip;
    const uint64_t nh = (uint64_t)stats[2ull * m + 2] ^ kShardFlip;
    hi[m] = (bad ? kShardBad : 0) | (as < m ? kShardGap : 0) | (h != ~nh ? kShardE0Mismatch : 0);
  }
}

hipError_t launch_shard_window(hipStream_t st, const long long* stats, const uint64_t* e0, uint32_t m,
                               uint64_t* hi) {
  hipLaunchKernelGGL(k_shard_window, dim3(1), dim3(1024), 0, st, stats, e0, m, hi);
  return hipGetLastError();
}

__global__ void k_gate_window(GateArgs g, const uint64_t* hi, uint32_t* counters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t flags = hi[g.m];
  const bool none = (flags & (kShardBad | kShardE0Mismatch)) != 0;
  if (i == 0) counters[10] = (uint32_t)flags;
  if (i < g.m) g.newnov[i] = none ? 0ull : (unsigned long long)hi[i];
  if (i < g.n) {
    const uint32_t a = g.fa[i];
    const uint64_t v = g.fv[i];
    g.apply[i] = !none && a < g.m && v >= g.e0[a] && v < hi[a] ? 1 : 0;
  }
}

hipError_t launch_gate_window(hipStream_t st, const GateArgs& g, const uint64_t* hi, uint32_t* counters) {
  const uint32_t t = g.n > g.m ? g.n : g.m;
  hipLaunchKernelGGL(k_gate_window, dim3((t + 255) / 256 + (t == 0)), dim3(256), 0, st, g, hi, counters);
  return hipGetLastError();
}

}  // namespace ce
