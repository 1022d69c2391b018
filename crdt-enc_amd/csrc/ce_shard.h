// ce_shard.h -- launch interface of ce_shard.hip (the cross-rank version gate of a batch
// partitioned by op-file address; layout of ShardStats and the windows in ce_common.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ce_common.h"
#include "ce_kernels.h"

namespace ce {

struct ShardArgs {
  const uint32_t* fa;          // [n] file -> writer index (the writer list shared by every rank)
  const uint64_t* fv;          // [n] file version
  uint32_t n, m, rank, world;
  const uint32_t* writers;     // [4m] writer UUID words
  const uint64_t* e0;          // [m] next_op_versions.get(writer)
  // scratch, initialised by the caller: cand = ~0, vmaxp1 = run_count = has_ge = bad = 0
  unsigned long long* cand;    // [m]
  unsigned long long* vmaxp1;  // [m]
  uint32_t* run_count;         // [m]
  uint32_t* has_ge;            // [m]
  uint32_t* bad;               // [1]
  long long* stats;            // [2m + 3] out (ShardStats)
};
hipError_t launch_shard_stats(hipStream_t s, const ShardArgs& a, uint64_t e0_hash);
// hi[0..m) = window ends, hi[m] = flags (kShardBad | kShardGap | kShardE0Mismatch)
hipError_t launch_shard_window(hipStream_t s, const long long* stats, const uint64_t* e0, uint32_t m,
                               uint64_t* hi);
// the sharded ingest's gate: apply[i] = e0 <= v < hi[writer]; newnov = hi; counters[10] = flags
hipError_t launch_gate_window(hipStream_t s, const GateArgs& g, const uint64_t* hi, uint32_t* counters);

}  // namespace ce
