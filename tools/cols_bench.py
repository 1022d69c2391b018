"""The column exchange of C3 at N = parts + 1 in one process (for rocprofv3 --kernel-trace): ranks
1..N-1's partials (writers [r 4096/N, (r+1) 4096/N) with their state files and `--versions` op-file
versions) are exported once as columns (ce_core_export_columns_device); each step rebuilds rank 0's
partial and merges all N - 1 column partials into it in one call (ce_core_merge_columns_device),
the receiver's side of shard.gather_dotset_columns.  --parts 7: rank 0's merge at N = 8.  Prints
the host times of export and merge and the check against the state-bytes merges one by one."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "crdt-enc_amd"))

import torch  # noqa: E402

import bench_configs as B  # noqa: E402
import crdtenc  # noqa: E402


def partial(ctx, dev, actors, lo, hi, V0, V, rank, rm_ctx="own"):
    per = B.N_ACTORS // 8
    mine = [j for j in range(8) if lo <= j * per < hi]
    states = B._state_files_c3(ctx, B.KEY, actors, V0, dev, mine)
    sdev, soffs, sblob = B.device_blob([states[j] for j in mine], dev)
    files, offs, n, blob_len, fa, fv = B.seal_op_files(ctx, B.KEY, actors, lo, hi, V0, V0 + V, dev, 1234 + rank,
                                                       rm_ctx=rm_ctx, V0=V0)
    writers = b"".join(bytes(a) for a in actors[lo:hi])
    core = B.new_core(ctx, B.KEY)
    core.register_actors([bytes(a) for a in actors])

    def fold():
        core.reset()
        for rc in (core.ingest_states_device(sdev.data_ptr(), soffs.data_ptr(), len(mine), sblob),
                   core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, writers,
                                          fa.data_ptr(), fv.data_ptr()),
                   core.settle()):
            if rc:
                raise crdtenc.CeError(rc, ctx.last_error())
    keep = (sdev, soffs, files, offs, fa, fv)
    return core, fold, keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--versions", type=int, default=16)
    ap.add_argument("--state-versions", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--parts", type=int, default=1, help="partials merged into rank 0's (N - 1; 1 or 7)")
    ap.add_argument("--rm-ctx", default="own", choices=["own", "read"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = crdtenc.Context(0)
    actors = B.actors_table()
    N = args.parts + 1
    cs = [partial(ctx, dev, actors, r * B.N_ACTORS // N, (r + 1) * B.N_ACTORS // N, args.state_versions,
                  args.versions, r, args.rm_ctx) for r in range(N)]
    c0, fold0, k0 = cs[0]
    bufs, ns, ex = [], [], []
    for r in range(1, N):
        c1, fold1, _ = cs[r]
        fold1()
        rc, need = c1.export_columns_device(0, 0)
        assert rc == 64 and need == 1, (rc, need)
        buf = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        for _ in range(args.steps if r == 1 else 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc, n = c1.export_columns_device(buf.data_ptr(), buf.numel())
            if r == 1:
                ex.append((time.perf_counter() - t0) * 1e3)
            assert rc == 0, (rc, ctx.last_error())
        bufs.append(buf)
        ns.append(n)
    mg = []
    for i in range(args.steps + 2):
        fold0()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = c0.merge_columns_device([b.data_ptr() for b in bufs], ns)
        if i >= 2:
            mg.append((time.perf_counter() - t0) * 1e3)
        assert rc == 0, (rc, ctx.last_error())
    got = c0.state_bytes()
    fold0()
    for r in range(1, N):
        assert c0.merge_state(cs[r][0].state_bytes()) == 0
    ok = got == c0.state_bytes()
    n = sum(ns)
    med = lambda v: sorted(v)[len(v) // 2]
    print(json.dumps({"partials": N - 1, "rm_ctx": args.rm_ctx, "column_bytes": n, "export_ms_median": round(med(ex), 4),
                      "merge_ms_median": round(med(mg), 4), "deferred_merges": c0.path_count("columns_merge_deferred"),
                      "equals_state_bytes_merge": ok}), flush=True)
    for c in cs:
        c[0].close()
    ctx.close()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
