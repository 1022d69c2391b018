#!/usr/bin/env python3
"""bench.py -- crdt-enc compaction/ingest hot path on MI355X (BASELINE.json configs[1] = C2).

One step = Core::compact over one batch resident in HBM (crdt-enc/src/lib.rs:332-380 minus
disk I/O): XChaCha20-Poly1305 open of every op file + version gate + Vec<Dot> decode + GCounter
max-fold (read_remote_ops, lib.rs:471-547), StateWrapper serialization, GPU seal of the new
state and its SHA3-256/BASE32 content name.  The core is reset to the empty state before each
step so every step folds all files.

Workload per GPU (weak scaling): 1,048,576 op files from this rank's actor shard; plaintext =
APP_VERSION(16) || msgpack(Vec<Dot>) with 107 Dots (4085 B, "4 KiB"); actor a's file v holds
its own increments (variant A).  The global job at N GPUs has 4096 actors x 256*N versions,
sharded by actor (all versions of an actor on one rank, as the version gate needs); the per-rank
partial GCounters meet in one RCCL all_reduce(MAX) over the dense actor-indexed state.

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "crdt-enc_amd"))
import crdtenc  # noqa: E402
import shard  # noqa: E402

METRIC = ("op files compacted/sec + AEAD-open GB/s, 1M×4KiB ops/4096 actors, 1–8 GPUs")
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")      # examples/test/src/main.rs:7
CORE = crdtenc.CORE_VERSION
N_ACTORS = 4096
K_DOTS = 107                       # 16 + 3 + 107 * 38 = 4085 B of plaintext
PT_LEN = 16 + 3 + 38 * K_DOTS
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 256 CU x 4 SIMD32 x 2.4 GHz = 78.6 T int32 lane-ops/s
# measured ceiling of the int32 ARX stream itself: tools/ubench_chacha (pure ChaCha20 blocks,
# 8 waves/SIMD) reaches 2.55 TB/s of keystream = 39.8 G blocks/s x 976 ops = 38.9 T lane-ops/s,
# i.e. wave64 int32 VALU instructions issue once per ~4 cycles per SIMD, not every 2
# (profiles/r01_ubench_chacha.txt)
VALU_INT32_MEASURED_TOPS = 38.9
DEFAULT_FUSED = 2                  # ce_core.h `fused` default (CE_FUSED overrides it in both)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def actors_table(seed=0xC0FFEE):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, size=(N_ACTORS, 16), dtype=np.uint8)
    a[:, 6] = (a[:, 6] & 0x0F) | 0x40       # UUIDv4-shaped
    a[:, 8] = (a[:, 8] & 0x3F) | 0x80
    order = sorted(range(N_ACTORS), key=lambda i: a[i].tobytes())
    return a[order]


def build_files(ctx, key, actors_local, versions, dev, seed):
    """Seal n = len(actors_local) * versions op files on the GPU; returns (files, offs, n, len)."""
    m_act = actors_local.shape[0]
    n = m_act * versions
    file_len = 16 + crdtenc.sealed_len(PT_LEN)
    files = torch.empty(n * file_len + 64, dtype=torch.uint8, device=dev)
    offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * file_len
    act = torch.from_numpy(actors_local).to(dev)
    pre1 = torch.tensor(list(b"\x82\xa5actor\xc4\x10"), dtype=torch.uint8, device=dev)
    pre2 = torch.tensor(list(b"\xa7counter"), dtype=torch.uint8, device=dev)
    app = torch.tensor(list(APP), dtype=torch.uint8, device=dev)
    hdr = torch.tensor([0xdc, K_DOTS >> 8, K_DOTS & 255], dtype=torch.uint8, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    kk = torch.arange(K_DOTS, dtype=torch.int64, device=dev)
    chunk = 1 << 16
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        idx = torch.arange(c0, c0 + m, dtype=torch.int64, device=dev)
        a_loc, v = idx // versions, idx % versions
        clear = torch.empty((m, PT_LEN), dtype=torch.uint8, device=dev)
        clear[:, :16] = app
        clear[:, 16:19] = hdr
        dots = clear[:, 19:].view(m, K_DOTS, 38)
        dots[:, :, 0:9] = pre1
        dots[:, :, 9:25] = act[a_loc][:, None, :]
        dots[:, :, 25:33] = pre2
        dots[:, :, 33] = 0xce                                  # uint32, big endian
        cval = 65536 + v[:, None] * K_DOTS + kk[None, :] + 1   # actor's own increments
        for b in range(4):
            dots[:, :, 34 + b] = ((cval >> (8 * (3 - b))) & 255).to(torch.uint8)
        coffs = torch.arange(m + 1, dtype=torch.int64, device=dev) * PT_LEN
        nonces = torch.randint(0, 256, (m, 24), dtype=torch.uint8, device=dev, generator=gen)
        ooffs = (idx * file_len).contiguous()
        torch.cuda.current_stream().synchronize()
        ctx.encrypt_batch_device(key, clear.data_ptr(), coffs.data_ptr(), m, nonces.data_ptr(),
                                 files.data_ptr(), ooffs.data_ptr(), outer_version=CORE)
        ctx.synchronize()
    return files, offs, n, n * file_len


def expected_state(actors_all, versions_global):
    """Closed form of the merged StateWrapper<GCounter> (size-independent check)."""
    import msgpack
    top = 65536 + versions_global * K_DOTS
    nov = {bytes(a): versions_global for a in actors_all}
    st = {bytes(a): top for a in actors_all}
    return msgpack.packb({"next_op_versions": {"dots": nov}, "state": {"inner": {"dots": st}}},
                         use_bin_type=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--versions", type=int, default=256, help="versions per actor per GPU")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="files in the CPU baseline sample (0 = the whole per-GPU workload, "
                         "~5-10 s of CPU work at 16 threads)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if N_ACTORS % world:
        raise SystemExit("world size must divide 4096")

    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = crdtenc.Context(local)
    ctx.set_stream(stream.cuda_stream)

    actors_all = actors_table()
    lo, hi = shard.actor_range(N_ACTORS, world, rank)
    per = hi - lo
    actors_local = actors_all[lo:hi]
    versions = args.versions * world                    # weak scaling: 1M files per GPU
    key = bytes(np.random.default_rng(7).integers(0, 256, 32, dtype=np.uint8))

    t0 = time.time()
    files, offs, n, blob_len = build_files(ctx, key, actors_local, versions, dev, seed=1234 + rank)
    log("rank %d: sealed %d op files (%.2f GB) in %.1f s" % (rank, n, blob_len / 1e9, time.time() - t0))

    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    core.register_actors([bytes(a) for a in actors_all])   # same dense slots on every rank
    cap = core.dense_capacity()
    # state and next_op_versions side by side: one all_reduce(MAX) per step (latency-bound)
    dense = torch.zeros(2 * cap, dtype=torch.int64, device=dev)
    st_t, nov_t = dense[:cap], dense[cap:]
    local_actor_bytes = b"".join(bytes(a) for a in actors_local)
    fa = np.repeat(np.arange(per, dtype=np.uint32), versions)
    fv = np.tile(np.arange(versions, dtype=np.uint64), per)
    # per-file metadata lives in HBM with the files (what Storage::load_ops hands over)
    fa_d = torch.from_numpy(fa.astype(np.int32)).to(dev)
    fv_d = torch.from_numpy(fv.astype(np.int64)).to(dev)

    out = {}
    # The SHA3-256 content name of step i's state file (host, ~0.2 MB) is computed on a host
    # thread while step i+1's kernels run; every name is done before the timed region ends.
    from concurrent.futures import ThreadPoolExecutor
    namer = ThreadPoolExecutor(1)
    names = []

    def step():
        core.reset()
        if world == 1:
            # Core::compact (lib.rs:332-380): read_remote_ops + the compaction output in one call
            rc, f, _ = core.compact_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len,
                                               local_actor_bytes, fa_d.data_ptr(), fv_d.data_ptr(),
                                               name=False)
            if rc:
                raise crdtenc.CeError(rc, ctx.last_error())
            out["file"] = f
            names.append(namer.submit(crdtenc.content_name, f))
            return
        rc = core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len,
                                    local_actor_bytes, fa_d.data_ptr(), fv_d.data_ptr())
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        if world > 1:
            core.export_dense(st_t.data_ptr(), nov_t.data_ptr())
            shard.merge_dense(dense)           # all_reduce(MAX) over u64
            core.import_dense(st_t.data_ptr(), nov_t.data_ptr())
        if rank == 0:
            f, _ = core.compact_to_buffer(name=False)
            out["file"] = f
            names.append(namer.submit(crdtenc.content_name, f))

    for _ in range(args.warmup):
        step()
    for fu in names:
        fu.result()
    names.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    for fu in names:
        out["name"] = fu.result()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.set_timing(False)
    ms = (t1 - t0) * 1e3 / args.steps
    ms_t = torch.tensor([ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ms_t, op=dist.ReduceOp.MAX)
    ms_max = float(ms_t.item())

    kern = {k: ctx.timing(k) for k in ("open_setup", "gate", "open_fold_small", "segments_open",
                                       "finalize_open", "decode", "merge", "seal_setup",
                                       "segments_seal", "finalize_seal")}

    # size-independent correctness check of the last step's result
    ok = True
    if rank == 0:
        sb = core.state_bytes()
        ok = sb == expected_state(actors_all if world > 1 else actors_local, versions)
        if not ok:
            log("STATE MISMATCH vs closed form")

    # CPU baseline: the oracle (C restatement of the reference path), reference-shaped:
    # cpu_threads AEAD workers, decode + ordered fold on one thread (lib.rs:497-544)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, REPO)
        import oracle
        s = min(args.cpu_sample, n) if args.cpu_sample > 0 else n
        s -= s % versions
        file_len = blob_len // n
        host = files[: s * file_len].cpu().numpy()
        h_offs = (np.arange(s + 1, dtype=np.uint64) * file_len)
        h_act = np.ascontiguousarray(actors_local[fa[:s]])
        h_ver = np.ascontiguousarray(fv[:s])
        threads = min(args.cpu_threads, os.cpu_count() or 1)
        t = time.perf_counter()
        err, ser = oracle.compact_ops_baseline(
            oracle.STATE_GCOUNTER, key, APP, host.ctypes.data_as(ctypes.c_void_p),
            h_offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            h_act.ctypes.data_as(ctypes.c_void_p),
            h_ver.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), s, threads)
        dt = time.perf_counter() - t
        # the same sample through the GPU path must serialize to the same bytes
        core.reset()
        rc = core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), s, s * file_len,
                                    b"".join(bytes(a) for a in actors_local[: s // versions]),
                                    fa_d.data_ptr(), fv_d.data_ptr())
        same = rc == 0 and err == 0 and core.state_bytes() == ser
        cpu = {"value": round(s / dt, 1), "unit": "op files/s", "cores": threads, "kind": "port",
               "sample": "%d files (%d actors x %d versions) of this workload, oracle/ce_oracle.c "
                         "reference-shaped: %d AEAD threads, decode+fold on one thread; "
                         "serialized state == GPU path: %s" % (s, s // versions, versions, threads, same),
               "seconds": round(dt, 3)}

    if rank == 0:
        # dominant kernel: the fused open+decode+fold of the 4 KiB op files
        seg_ms, seg_n = kern["open_fold_small"]
        avg_s = seg_ms / max(seg_n, 1) / 1e3
        ct_bytes = n * PT_LEN
        bytes_per_launch = n * (PT_LEN + 16)              # read ct + tag; plaintext stays in LDS
        ops_per_file = 992 * -(-PT_LEN // 64) + 48 * (-(-PT_LEN // 16) + 1)
        achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
        valu = n * ops_per_file / avg_s / 1e12 if avg_s > 0 else 0.0
        fused = os.environ.get("CE_FUSED", str(DEFAULT_FUSED))
        lpf = 64 // int(os.environ.get("CE_FILES_PER_WAVE", "4"))
        kname = ("k_open_fold_v2<%d> (XChaCha20-Poly1305 open + Vec<Dot> decode + fold, "
                 "lane-owned ChaCha20 blocks)" % lpf if fused == "2" and lpf != 64 else
                 "k_open_fold_small<%d> (XChaCha20-Poly1305 open + Vec<Dot> decode + fold)" % lpf)
        traffic = None
        tf = os.path.join(REPO, "profiles", "traffic_open_fold_small.json")
        if os.path.exists(tf):
            with open(tf) as f:
                rec = json.load(f)
            # only a measurement of the kernel this run used (and of the same 1M-file launch)
            if kname.split(" (")[0].rstrip(">") in rec.get("kernel", "") and \
                    rec.get("files_per_launch") == n:
                traffic = rec.get("bytes_per_launch")
        # VALU issue from the PMC record of this kernel (SQ_INSTS_VALU x 64 lanes per file,
        # tools/pmc_valu.sh) at this run's launch time: the kernel's binding roofline
        valu_pmc = None
        vf = os.path.join(REPO, "profiles", "r01_valu_pmc.json")
        if os.path.exists(vf) and avg_s > 0 and fused == "2" and lpf == 16:
            with open(vf) as f:
                rec = json.load(f).get("fused", {})
            ipf = rec.get("valu_instr_per_file_per_lane")
            if ipf:
                t = n * ipf / avg_s / 1e12
                valu_pmc = {"instr_per_file": ipf, "achieved_tops": round(t, 2),
                            "frac_of_measured": round(t / VALU_INT32_MEASURED_TOPS, 4),
                            "frac_of_peak": round(t / VALU_PEAK_TOPS, 4),
                            "source": "profiles/r01_valu_pmc.json (rocprofv3 SQ_INSTS_VALU x 64 "
                                      "per file, same kernel and workload)"}
        line = {
            "metric": METRIC,
            "value": round(n * world / (ms_max / 1e3), 1),
            "unit": "op files/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_max, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (GPU-sealed op files, seeded)",
            "config": {
                "workload": "C2: 1,048,576 x 4 KiB encrypted GCounter op files per GPU "
                            "(4096 actors x %d versions at N=%d, actor-sharded), decrypt + "
                            "max-join + compact" % (versions, world),
                "files_per_gpu": n, "plaintext_bytes": PT_LEN, "file_bytes": blob_len // n,
                "dots_per_file": K_DOTS, "actors": N_ACTORS,
                "parallelism": "actor-sharded files, RCCL all_reduce(MAX) of dense state"
                               if world > 1 else "single GPU",
            },
            "aead_open_GBps": round(ct_bytes / avg_s / 1e9, 1) if avg_s > 0 else None,
            "roofline": {
                "kernel": kname,
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": bytes_per_launch, "avg_launch_ms": round(avg_s * 1e3, 4),
                "valu": {"achieved_tops": round(valu, 2), "peak_tops": round(VALU_PEAK_TOPS, 1),
                         "frac": round(valu / VALU_PEAK_TOPS, 4),
                         "int32_measured_peak_tops": VALU_INT32_MEASURED_TOPS,
                         "frac_of_measured": round(valu / VALU_INT32_MEASURED_TOPS, 4),
                         "ops_per_file": ops_per_file, "pmc_instructions": valu_pmc},
            },
            "kernels_ms_per_step": {k: round(v[0] / max(v[1], 1), 4) for k, v in kern.items() if v[1]},
            "state_check": "closed-form StateWrapper bytes: %s" % ("ok" if ok else "MISMATCH"),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    core.close()
    ctx.close()


if __name__ == "__main__":
    main()
