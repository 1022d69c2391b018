#!/usr/bin/env python3
"""Per-rank byte imbalance of the C4 workload (bench_configs.py run_c4: 1024 writers x 32
versions, plaintexts log-uniform on [256 B, 1 MiB], same seed) under the two multi-GPU
partitions of VClock / GCounter op files:

  actor    whole writers per rank, contiguous ranges (shard.actor_range)
  address  each op file by a hash of its address ops/<actor>/<version> (crdtenc.shard_owners)

and the same for a writer-skewed C2-sized batch (Zipf version counts per writer).
For N = 2, 4, 8: bytes per rank, max / mean (the step waits for the slowest rank, so this is
the weak-scaling efficiency bound from imbalance alone), files per rank.  CPU only.

    python tools/partition_balance.py > profiles/r03_c4_partition_balance.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "crdt-enc_amd"))
sys.path.insert(0, REPO)
import crdtenc  # noqa: E402
import shard  # noqa: E402


def c4_sizes():
    """The C4 generator's file sizes (bench_configs.run_c4, same seeds), (m, V) int64."""
    import bench
    actors = bench.actors_table()[::4]
    m, V = actors.shape[0], 32
    rng = np.random.default_rng(404)
    size = np.exp(rng.uniform(np.log(256), np.log(1 << 20), size=(m, V))).astype(np.int64)
    kd = np.maximum(1, (size - 19) // 38)
    pt = 16 + np.where(kd <= 15, 1, np.where(kd <= 0xffff, 3, 5)) + 38 * kd
    f_len = np.vectorize(lambda x: 16 + crdtenc.sealed_len(int(x)))(pt)
    return actors, f_len


def main():
    actors, f_len = c4_sizes()
    m, V = f_len.shape
    fa = np.repeat(np.arange(m, dtype=np.uint32), V)
    fv = np.tile(np.arange(V, dtype=np.uint64), m)
    flat = f_len.ravel()
    out = {"workload": "C4 (bench_configs.run_c4): %d writers x %d versions, %.3f GB of op files" % (m, V, flat.sum() / 1e9),
           "rows": []}
    for world in (2, 4, 8):
        for part in ("actor", "address"):
            if part == "actor":
                rank = np.array([shard.file_rank(int(a), m, world) for a in fa])
            else:
                rank = crdtenc.shard_owners([bytes(a) for a in actors], fa, fv, world)
            b = np.bincount(rank, weights=flat, minlength=world)
            f = np.bincount(rank, minlength=world)
            out["rows"].append({"n_gpus": world, "partition": part,
                                "bytes_per_rank_GB": [round(x / 1e9, 4) for x in b],
                                "max_over_mean": round(float(b.max() / b.mean()), 4),
                                "files_per_rank": [int(x) for x in f]})
    # writer skew: 4096 writers whose version counts follow Zipf(1.1) (a few busy writers, a
    # long tail), 1M x 4 KiB op files in total -- C2's volume with C4-style skew across writers
    import bench
    acts = bench.actors_table()
    w = 1.0 / np.arange(1, 4097) ** 1.1
    cnt = np.maximum(1, np.round(w / w.sum() * (1 << 20))).astype(np.int64)
    np.random.default_rng(5).shuffle(cnt)
    fa2 = np.repeat(np.arange(4096, dtype=np.uint32), cnt)
    fv2 = np.concatenate([np.arange(c, dtype=np.uint64) for c in cnt])
    out["writer_skew"] = {"workload": "4096 writers, version counts Zipf(1.1) (max %d, median %d), "
                                      "%d x 4195 B op files" % (cnt.max(), int(np.median(cnt)), cnt.sum()),
                          "rows": []}
    for world in (2, 4, 8):
        for part in ("actor", "address"):
            if part == "actor":
                rank = np.array([shard.file_rank(a, 4096, world) for a in range(4096)])[fa2]
            else:
                rank = crdtenc.shard_owners([bytes(a) for a in acts], fa2, fv2, world)
            f = np.bincount(rank, minlength=world)
            out["writer_skew"]["rows"].append({"n_gpus": world, "partition": part,
                                               "max_over_mean": round(float(f.max() / f.mean()), 4),
                                               "files_per_rank": [int(x) for x in f]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
