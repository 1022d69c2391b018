#!/usr/bin/env python3
"""bench_configs.py -- the other BASELINE.json configs on one MI355X (bench.py measures C2).

  --config c3   Orswot<u64, Uuid>, 100k members, 4096 actors, mixed state + op files:
                8 state files (each the compaction of 512 actors' first V0 versions) then
                4096 x V op files of 32 ops (26 Add + 6 Rm, 1961 B plaintext); one step =
                reset + read_remote_states + read_remote_ops + compact (crdt-enc/src/lib.rs:
                332-547) with the op and state files resident in HBM (the line's
                `states_from_host` times the state files staged from host buffers instead).

  --config c4   skewed sizes: 1024 actors x 32 versions of GCounter op files whose plaintexts are
                log-uniform on [256 B, 1 MiB] (~4 GB, the C2 byte volume): single-page files take
                the fused kernel, larger ones the 16 KiB-segment open + the wave-per-file decode.
                One step = reset + Core::compact over the batch in HBM (compact_ops_device).
                Check: the StateWrapper equals its closed form.
  --config c5   key-rotation mix: the C2 batch (1M x 4 KiB, 4096 actors) with the odd actors'
                files sealed under a second data key and 0.1% of all files with one flipped tag
                bit.  One step = reset + read_remote_ops with per-file statuses under the latest
                key (key_cryptor.rs:59-70): every second-key and tampered file must be rejected
                (CE_ERR_AUTH), every other file accepted, and nothing folded (lib.rs:497-516).

With N > 1 ranks (bench.py --gpus N) every config runs strong-scaled over the ranks
(run_config -> run_c*_multi below).

Prints one JSON line per run.  Checks (size-independent): the merged clock equals its closed
form (actor a's adds count 26 per version), and an actor-sharded fold of the same files merged
with merge_state (the multi-GPU exchange) serializes to the same bytes.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "crdt-enc_amd"))
import crdtenc  # noqa: E402

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = crdtenc.CORE_VERSION
N_ACTORS = 4096
N_MEMBERS = 100_000
N_ADD, N_RM = 26, 6
# one Add / Rm op in rmp-serde's to_vec_named form with fixed-width (uint32) integers
ADD_T = (b"\x81\xa3Add\x82\xa3dot\x82\xa5actor\xc4\x10" + bytes(16) + b"\xa7counter\xce" + bytes(4) +
         b"\xa7members\x91\xce" + bytes(4))
RM_T = (b"\x81\xa2Rm\x82\xa5clock\x81\xa4dots\x81\xc4\x10" + bytes(16) + b"\xce" + bytes(4) +
        b"\xa7members\x91\xce" + bytes(4))
ADD_UUID, ADD_CTR, ADD_MEM = 19, 44, 58
RM_UUID, RM_CTR, RM_MEM = 20, 37, 51
HDR = APP + b"\xdc" + (N_ADD + N_RM).to_bytes(2, "big")
PT_LEN = len(HDR) + N_ADD * len(ADD_T) + N_RM * len(RM_T)
assert (len(ADD_T), len(RM_T), PT_LEN) == (62, 55, 1961)


HOST_PROF = bool(os.environ.get("CE_HOST_PROF"))
NO_NAMES = bool(os.environ.get("CE_C3_NO_NAMES"))


class _StepMarks:
    """CE_ROCTX=1: each timed step as a ROCTx range "c3_step" (rocprofv3 --marker-trace), so the
    trace tools (tools/c3_step_breakdown.py, c3_host_trace.py) cut exactly the timed steps"""

    def __init__(self):
        self.lib = None
        if os.environ.get("CE_ROCTX"):
            import ctypes
            for name in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
                try:
                    self.lib = ctypes.CDLL(name)   # the ROCTx rocprofv3 --marker-trace intercepts
                    break
                except OSError:
                    pass
            self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]

    def push(self):
        if self.lib:
            self.lib.roctxRangePushA(b"c3_step")

    def pop(self):
        if self.lib:
            self.lib.roctxRangePop()


MARKS = _StepMarks()
KEY = bytes(np.random.default_rng(7).integers(0, 256, 32, dtype=np.uint8))  # latest data key


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def actors_table(seed=0xC0FFEE):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, size=(N_ACTORS, 16), dtype=np.uint8)
    a[:, 6] = (a[:, 6] & 0x0F) | 0x40
    a[:, 8] = (a[:, 8] & 0x3F) | 0x80
    order = sorted(range(N_ACTORS), key=lambda i: a[i].tobytes())
    return a[order]


def member_of(a, v, j):
    """deterministic member of actor a's add j in version v (int64 tensors)"""
    h = (a * 1000003 + v * 7919 + j * 104729) * 2654435761
    return (h ^ (h >> 13)) % N_MEMBERS


def _be32(x, out):
    for b in range(4):
        out[..., b] = ((x >> (8 * (3 - b))) & 255).to(torch.uint8)


def orswot_clears(actors, a_idx, v, dev):
    """plaintexts [m, PT_LEN] of op files (actor a_idx[i], version v[i]): adds with dots
    (a, 26 v + j + 1); removals of the actor's own earlier adds (previous version, or this one)"""
    m = a_idx.shape[0]
    out = torch.empty((m, PT_LEN), dtype=torch.uint8, device=dev)
    out[:, :len(HDR)] = torch.tensor(list(HDR), dtype=torch.uint8, device=dev)
    act = torch.from_numpy(actors).to(dev)[a_idx]
    adds = out[:, len(HDR):len(HDR) + N_ADD * 62].view(m, N_ADD, 62)
    adds[:] = torch.tensor(list(ADD_T), dtype=torch.uint8, device=dev)
    adds[:, :, ADD_UUID:ADD_UUID + 16] = act[:, None, :]
    j = torch.arange(N_ADD, dtype=torch.int64, device=dev)[None, :]
    _be32(v[:, None] * N_ADD + j + 1, adds[:, :, ADD_CTR:ADD_CTR + 4])
    _be32(member_of(a_idx[:, None], v[:, None], j), adds[:, :, ADD_MEM:ADD_MEM + 4])
    rms = out[:, len(HDR) + N_ADD * 62:].view(m, N_RM, 55)
    rms[:] = torch.tensor(list(RM_T), dtype=torch.uint8, device=dev)
    rms[:, :, RM_UUID:RM_UUID + 16] = act[:, None, :]
    k = torch.arange(N_RM, dtype=torch.int64, device=dev)[None, :]
    jv = (k * 5 + 3) % N_ADD
    vv = torch.where(v[:, None] > 0, v[:, None] - 1, v[:, None])
    _be32(vv * N_ADD + jv + 1, rms[:, :, RM_CTR:RM_CTR + 4])
    _be32(member_of(a_idx[:, None], vv, jv), rms[:, :, RM_MEM:RM_MEM + 4])
    return out


_READ_CTX = {}
READ_CTX_STATS = {}  # the last read-ctx batch: plaintext bytes, removal clock entries


def read_ctx_table(V0):
    """What every writer has read from the state files when its op versions start: per member, the
    (actor, largest counter) of the adds of versions [0, V0) listing it, actors ascending (a
    VClock's BTreeMap order; the actor table is sorted by UUID bytes) -- CSR by member."""
    if V0 in _READ_CTX:
        return _READ_CTX[V0]
    a = torch.arange(N_ACTORS, dtype=torch.int64).repeat_interleave(V0 * N_ADD)
    v = torch.arange(V0, dtype=torch.int64).repeat_interleave(N_ADD).repeat(N_ACTORS)
    j = torch.arange(N_ADD, dtype=torch.int64).repeat(N_ACTORS * V0)
    m = member_of(a, v, j).numpy()
    a, ctr = a.numpy(), (v * N_ADD + j + 1).numpy()
    o = np.lexsort((ctr, a, m))
    m, a, ctr = m[o], a[o], ctr[o]
    last = np.ones(len(m), bool)  # the last (largest counter) of each (member, actor) run
    last[:-1] = (m[1:] != m[:-1]) | (a[1:] != a[:-1])
    m, a, ctr = m[last], a[last], ctr[last]
    beg = np.searchsorted(m, np.arange(N_MEMBERS + 1))
    _READ_CTX[V0] = (beg, a, ctr)
    return _READ_CTX[V0]


def orswot_clears_read_ctx(actors, a_idx, v, V0):
    """orswot_clears with every Rm carrying the removed member's read context in place of the
    one-entry clock {writer: its own earlier counter}: Rm{clock: the member's entry clock as writer
    a reads it -- the state files' adds of m (read_ctx_table) and a's own removed add --, members:
    [m]}, crdts' rm(member, read_ctx), fixed-width uints.  Clocks name other writers' dots, so a
    writer shard defers them ("Rm ops with read-ctx clocks").  -> plaintexts"""
    base = orswot_clears(actors, a_idx.cpu(), v.cpu(), "cpu").numpy()
    beg, ta, tc = read_ctx_table(V0)
    beg, ta, tc = beg.tolist(), ta.tolist(), tc.tolist()
    ent_b = [b"\xc4\x10" + actors[x].tobytes() + b"\xce" for x in range(N_ACTORS)]
    cut = len(HDR) + N_ADD * len(ADD_T)
    vv = torch.where(v > 0, v - 1, v).cpu()
    k = torch.arange(N_RM, dtype=torch.int64)
    jv = (k * 5 + 3) % N_ADD
    mm = member_of(a_idx.cpu()[:, None], vv[:, None], jv[None, :]).tolist()
    own = (vv[:, None] * N_ADD + jv[None, :] + 1).tolist()
    out = []
    n_ent = 0
    for i, ai in enumerate(a_idx.tolist()):
        parts = [base[i, :cut].tobytes()]
        for r in range(N_RM):
            m = mm[i][r]
            b0, b1 = beg[m], beg[m + 1]
            ent = dict(zip(ta[b0:b1], tc[b0:b1]))
            oc = own[i][r]
            if ent.get(ai, 0) < oc:
                ent[ai] = oc
            e = len(ent)
            n_ent += e
            parts.append(b"\x81\xa2Rm\x82\xa5clock\x81\xa4dots")
            parts.append(bytes([0x80 | e]) if e <= 15 else b"\xde" + e.to_bytes(2, "big"))
            for x in sorted(ent):
                parts.append(ent_b[x] + ent[x].to_bytes(4, "big"))
            parts.append(b"\xa7members\x91\xce" + m.to_bytes(4, "big"))
        out.append(b"".join(parts))
    READ_CTX_STATS["clock_entries"] = n_ent
    return out


def seal_op_files(ctx, key, actors, a_lo, a_hi, v_lo, v_hi, dev, seed, rm_ctx="own", V0=None):
    """op files of actors [a_lo, a_hi) x versions [v_lo, v_hi), actor-major (load_ops order).
    rm_ctx "read": removals carry read contexts (orswot_clears_read_ctx; variable file lengths)"""
    if rm_ctx == "read":
        return _seal_op_files_read_ctx(ctx, key, actors, a_lo, a_hi, v_lo, v_hi, dev, seed, V0)
    na, nv = a_hi - a_lo, v_hi - v_lo
    n = na * nv
    flen = 16 + crdtenc.sealed_len(PT_LEN)
    files = torch.empty(n * flen + 64, dtype=torch.uint8, device=dev)
    offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * flen
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    chunk = 1 << 15
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        idx = torch.arange(c0, c0 + m, dtype=torch.int64, device=dev)
        a_idx, v = a_lo + idx // nv, v_lo + idx % nv
        clear = orswot_clears(actors, a_idx, v, dev)
        coffs = torch.arange(m + 1, dtype=torch.int64, device=dev) * PT_LEN
        nonces = torch.randint(0, 256, (m, 24), dtype=torch.uint8, device=dev, generator=gen)
        ooffs = (idx * flen).contiguous()
        torch.cuda.current_stream().synchronize()
        ctx.encrypt_batch_device(key, clear.data_ptr(), coffs.data_ptr(), m, nonces.data_ptr(),
                                 files.data_ptr(), ooffs.data_ptr(), outer_version=CORE)
        ctx.synchronize()
    fa = torch.arange(na, dtype=torch.int32, device=dev).repeat_interleave(nv)
    fv = torch.arange(v_lo, v_hi, dtype=torch.int64, device=dev).repeat(na)
    return files, offs, n, n * flen, fa, fv


def _seal_op_files_read_ctx(ctx, key, actors, a_lo, a_hi, v_lo, v_hi, dev, seed, V0):
    na, nv = a_hi - a_lo, v_hi - v_lo
    n = na * nv
    idx = torch.arange(n, dtype=torch.int64)
    a_idx, v = a_lo + idx // nv, v_lo + idx % nv
    clears = orswot_clears_read_ctx(actors, a_idx, v, V0 if V0 is not None else v_lo)
    clen = np.array([len(c) for c in clears], np.int64)
    READ_CTX_STATS.update(plaintext_bytes=int(clen.sum()), files=n, mean_file_plaintext=round(float(clen.mean()), 1),
                          max_file_plaintext=int(clen.max()))
    flen = np.array([16 + crdtenc.sealed_len(int(x)) for x in clen], np.int64)
    fo = np.zeros(n + 1, np.int64)
    fo[1:] = np.cumsum(flen)
    co = np.zeros(n + 1, np.int64)
    co[1:] = np.cumsum(clen)
    clear = torch.from_numpy(np.frombuffer(b"".join(clears), np.uint8).copy()).to(dev)
    files = torch.empty(int(fo[-1]) + 64, dtype=torch.uint8, device=dev)
    coffs = torch.from_numpy(co).to(dev)
    ooffs = torch.from_numpy(fo[:-1].copy()).to(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    nonces = torch.randint(0, 256, (n, 24), dtype=torch.uint8, device=dev, generator=gen)
    torch.cuda.current_stream().synchronize()
    ctx.encrypt_batch_device(key, clear.data_ptr(), coffs.data_ptr(), n, nonces.data_ptr(),
                             files.data_ptr(), ooffs.data_ptr(), outer_version=CORE)
    ctx.synchronize()
    offs = torch.from_numpy(fo).to(dev)
    fa = torch.arange(na, dtype=torch.int32, device=dev).repeat_interleave(nv)
    fv = torch.arange(v_lo, v_hi, dtype=torch.int64, device=dev).repeat(na)
    return files, offs, n, int(fo[-1]), fa, fv


def name_threads():
    """SHA3 name threads for the pipelined compactions: the job's CPU share less four (the
    launching thread, the runtime's and the download waits: at share - 2 the cgroup quota was
    exceeded and throttled, C3 3.27-3.39 ms/step against 2.58-2.67 at share - 4 on one box,
    tools/c3_names_ab.sh), at least 4; CE_NAME_THREADS overrides"""
    if os.environ.get("CE_NAME_THREADS"):
        return max(1, int(os.environ["CE_NAME_THREADS"]))
    import bench
    return max(4, bench.host_cpu()[2] - 4)


def _lower_priority():
    try:
        import threading
        os.setpriority(os.PRIO_PROCESS, threading.get_native_id(), 10)
    except (AttributeError, OSError):
        pass


class BatchNamer:
    """Content names on `threads` host threads, each taking up to `kmax` pending files at once
    (crdtenc.content_names: eight SHA3-256 sponges per AVX-512 step, ~2.7x one core's rate at
    eight, ~2x at four) -- submit() returns a Future of the name"""

    def __init__(self, threads, kmax):
        import collections
        import threading
        self.q = collections.deque()
        self.cv = threading.Condition()
        self.kmax, self.stop = kmax, False
        self.th = [threading.Thread(target=self._run, daemon=True) for _ in range(threads)]
        for t in self.th:
            t.start()

    def submit(self, buf):
        from concurrent.futures import Future
        f = Future()
        with self.cv:
            self.q.append((buf, f))
            self.cv.notify()
        return f

    def _run(self):
        _lower_priority()
        while True:
            with self.cv:
                while not self.q and not self.stop:
                    self.cv.wait()
                if not self.q:
                    return
                batch = [self.q.popleft() for _ in range(min(self.kmax, len(self.q)))]
            try:
                for (_, f), nm in zip(batch, crdtenc.content_names([b for b, _ in batch])):
                    f.set_result(nm)
            except Exception as e:  # noqa: BLE001 -- every waiter sees the failure
                for _, f in batch:
                    f.set_exception(e)

    def shutdown(self):
        with self.cv:
            self.stop = True
            self.cv.notify_all()
        for t in self.th:
            t.join()


class CompactPipe:
    """Pipelined Core::compact outputs (C3): NB pinned buffers; each file's download is left in
    flight (ce_core_compact_into_async: an SDMA engine copy) while the next step runs on the
    device, then its SHA3-256 name (crdt-enc-tokio/src/lib.rs:403-432, a sequential sponge, ~48 ms
    for 35 MB on one core) is hashed on the host threads, up to four pending files per
    multi-buffer batch.  flush() completes every download, drain() every name; a buffer is reused
    only after its name is done."""

    def __init__(self, core, nb=None, use_async=True):
        from concurrent.futures import ThreadPoolExecutor
        if nb is None:
            nb = name_threads() + 1
        self.core, self.nb, self.use_async = core, nb, use_async
        # the hashing threads below the launching thread's priority: the device pipeline's
        # host waits and launches are never queued behind a name (the names catch up in the gaps)
        # the names in multi-buffer batches of up to four pending files (crdtenc.content_names;
        # same box, 120 steps: 3.10-3.47 ms/step against 3.76-3.78 one file per thread, 3.35 at
        # three, 4.0 at eight -- a batch's latency is the drain); CE_NAME_BATCH=1: one per thread
        kmax = int(os.environ.get("CE_NAME_BATCH", "4"))
        if kmax > 1:   # more buffers in flight: a batch holds its files for its whole hash
            nb = max(nb, int(os.environ.get("CE_NAME_BUFFERS", "32")))
            self.nb = nb
            self.namer = BatchNamer(name_threads(), kmax)
        else:
            self.namer = ThreadPoolExecutor(nb - 1, initializer=_lower_priority)
        self.obuf = [crdtenc.host_buffer(1 << 26) for _ in range(nb)]   # pinned: DMA-engine downloads
        self.fut = [None] * nb
        self.inflight = []      # (buffer, length, ticket) of downloads not yet waited for
        self.order = []         # name futures in step order
        self.i = 0
        self.last_file = None
        self.names = not NO_NAMES

    def _name(self, k, ln, tk):
        ln = self.core.compact_wait(tk) if tk else ln
        self.last_file = self.obuf[k][:ln]
        if not self.names:    # diagnostics only: the step without the host's SHA3 load beside it
            return
        self.fut[k] = (self.namer.submit(self.last_file) if isinstance(self.namer, BatchNamer)
                       else self.namer.submit(crdtenc.content_name, self.last_file))
        self.order.append(self.fut[k])

    def compact(self):
        k = self.i % self.nb
        self.i += 1
        if self.fut[k] is not None:
            self.fut[k].result()
            self.fut[k] = None
        if self.use_async:
            ln, tk = self.core.compact_into_async(self.obuf[k])
        else:
            self.obuf[k], ln, _ = self.core.compact_into(self.obuf[k], name=False)
            tk = 0
        self.inflight.append((k, ln, tk))
        while len(self.inflight) > 1:       # the previous step's download overlapped this step
            self._name(*self.inflight.pop(0))

    def flush(self):
        while self.inflight:
            self._name(*self.inflight.pop(0))

    def drain(self):
        self.flush()
        name = None
        for fu in self.order:
            name = fu.result()
        self.order.clear()
        return name

    def close(self):
        self.drain()
        self.namer.shutdown()


def device_blob(files, dev):
    """files (bytes) back to back in HBM: (u8 tensor with 64 bytes of slack, i64 offsets, length)"""
    offs = np.zeros(len(files) + 1, np.int64)
    offs[1:] = np.cumsum([len(f) for f in files])
    blob = torch.zeros(int(offs[-1]) + 64, dtype=torch.uint8, device=dev)
    if len(files):
        blob[: int(offs[-1])] = torch.from_numpy(np.frombuffer(b"".join(files), np.uint8).copy()).to(dev)
    return blob, torch.from_numpy(offs).to(dev), int(offs[-1])


def new_core(ctx, key, flags=0):
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP,
                        flags=flags)
    core.set_latest_key(key)
    return core


def gcounter_cpu_baseline(key, host_blob, h_offs, h_act, h_ver, check, what):
    """oracle/ce_oracle.c on this host over a bounded sample of the workload, both modes
    (bench.py's cpu_baseline legs); check(err, serialized) compares with the GPU path."""
    import ctypes
    sys.path.insert(0, REPO)
    import bench
    import oracle
    model, avail, threads, why = bench.host_cpu()
    s = len(h_offs) - 1
    res = {}
    for mode, best, th in (("best", True, threads), ("reference_shaped", False, min(16, threads))):
        t = time.perf_counter()
        err, ser = oracle.compact_ops_baseline(
            oracle.STATE_GCOUNTER, key, APP, host_blob.ctypes.data_as(ctypes.c_void_p),
            h_offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), h_act.ctypes.data_as(ctypes.c_void_p),
            h_ver.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), s, th, best=best)
        dt = time.perf_counter() - t
        res[mode] = {"value": round(s / dt, 1), "cores": th, "seconds": round(dt, 3),
                     "same_result_as_gpu": bool(check(err, ser))}
    res["best"]["mode"] = "open + decode parallel over files, fold parallel over actors"
    res["reference_shaped"]["mode"] = ("%d AEAD threads (buffered(16), lib.rs:497-514), decode + "
                                       "fold on one thread" % res["reference_shaped"]["cores"])
    # the headline is the faster mode (on a reject-path batch the reference-shaped one stops
    # after the opens, while the best mode also runs its parallel decode check)
    top = max(res, key=lambda k: res[k]["value"])
    t = res[top]
    return {"value": t["value"], "unit": "files/s", "cores": t["cores"], "kind": "port",
            "sample": "%s; oracle/ce_oracle.c, %s mode (%s) on %d threads" % (what, top, t["mode"], t["cores"]),
            "seconds": t["seconds"], "same_result_as_gpu": all(v["same_result_as_gpu"] for v in res.values()),
            "host_cpu": model, "nproc": os.cpu_count(), "usable_cpus": avail, "cores_rule": why,
            "modes": {k: dict(v, unit="files/s") for k, v in res.items()}}


def orswot_cpu_baseline(key, state_files, blob, offs, file_actor, file_version, gpu_state, what):
    """oracle/ce_oracle.c oc_compact_orswot_best (the C restatement of oracle/crdts.py) on this
    host: every file opened + decoded on T threads, the state merges and the op fold in file
    order on one thread (order-dependent: removals defer), then the canonical StateWrapper
    serialized, sealed and named as Core::compact does.  Two thread counts: the host's CPU
    share ('best') and 16 ('reference_shaped': load_ops' buffered(16), lib.rs:497-514)."""
    sys.path.insert(0, REPO)
    import bench
    import oracle
    model, avail, threads, why = bench.host_cpu()
    nf = len(state_files) + len(offs) - 1
    res = {}
    for mode, th in (("best", threads), ("reference_shaped", min(16, threads))):
        err, ser, dt, ph = oracle.compact_orswot_best(key, APP, state_files, blob, offs, file_actor,
                                                      file_version, th, seal=True)
        res[mode] = {"value": round(nf / dt, 1), "cores": th, "seconds": round(dt, 3),
                     "phases_s": {k: round(v, 4) for k, v in
                                  zip(("open_decode", "state_merges", "op_fold", "serialize_seal"), ph)},
                     "same_result_as_gpu": err == 0 and ser == gpu_state}
    top = max(res, key=lambda k: res[k]["value"])
    t = res[top]
    return {"value": t["value"], "unit": "files/s", "cores": t["cores"], "kind": "port",
            "sample": "%s; oracle/ce_oracle.c oc_compact_orswot_best, %s mode (open + decode on %d "
                      "threads, merges + fold on one)" % (what, top, t["cores"]),
            "seconds": t["seconds"], "same_result_as_gpu": all(v["same_result_as_gpu"] for v in res.values()),
            "host_cpu": model, "nproc": os.cpu_count(), "usable_cpus": avail, "cores_rule": why,
            "modes": {k: dict(v, unit="files/s") for k, v in res.items()}}


def run_c3(args, ctx, dev):
    actors = actors_table()
    key = bytes(np.random.default_rng(7).integers(0, 256, 32, dtype=np.uint8))
    V0, V = args.state_versions, args.versions
    rm_ctx = getattr(args, "rm_ctx", "own")
    t0 = time.time()
    # state files: compaction (ingest-readable format) of 512 actors' versions [0, V0) each
    states = []
    per = N_ACTORS // 8
    for j in range(8):
        f, o, n, bl, fa, fv = seal_op_files(ctx, key, actors, j * per, (j + 1) * per, 0, V0, dev, 99 + j)
        sc = new_core(ctx, key, flags=crdtenc.COMPACT_INGEST_FORMAT)
        rc = sc.ingest_ops_device(f.data_ptr(), o.data_ptr(), n, bl,
                                  b"".join(bytes(a) for a in actors[j * per:(j + 1) * per]),
                                  fa.data_ptr(), fv.data_ptr())
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        states.append(sc.compact_to_buffer(nonce=bytes(24))[0])
        sc.close()
        del f, o
    files, offs, n, blob_len, fa, fv = seal_op_files(ctx, key, actors, 0, N_ACTORS, V0, V0 + V, dev, 1234,
                                                     rm_ctx=rm_ctx, V0=V0)
    rc_stats = dict(READ_CTX_STATS) if rm_ctx == "read" else None
    all_actors = b"".join(bytes(a) for a in actors)
    log("c3: %d state files (%.1f MB), %d op files (%.2f GB) in %.1f s" % (
        len(states), sum(map(len, states)) / 1e6, n, blob_len / 1e9, time.time() - t0))

    core = new_core(ctx, key)
    core.register_actors([bytes(a) for a in actors])
    out = {}
    # the state files resident in HBM like the op files (load_states' result; the bench's inputs
    # are resident when the timed region starts); `states_from_host` below times them staged
    # from per-file host buffers instead
    sdev, soffs, sblob = device_blob(states, dev)
    host_states = [False]

    phase = {"reset": 0.0, "states": 0.0, "ops": 0.0, "compact": 0.0}
    # step i's sealed file comes down while step i+1 runs on the device, and its SHA3-256 content
    # name is computed on host threads (CompactPipe); every download and name is done before the
    # timed region ends
    pipe = CompactPipe(core, use_async=not os.environ.get("CE_C3_SYNC_COMPACT"))
    NB = pipe.nb
    obuf = pipe.obuf

    def step():
        t = time.perf_counter()
        core.reset()
        t1 = time.perf_counter()
        if host_states[0]:
            rc, st = core.ingest_states_iov(states)   # load_states' per-file host buffers, no join
        else:
            rc = core.ingest_states_device(sdev.data_ptr(), soffs.data_ptr(), len(states), sblob)
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        t2 = time.perf_counter()
        rc = core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, all_actors,
                                    fa.data_ptr(), fv.data_ptr())
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        t3 = time.perf_counter()
        pipe.compact()
        t4 = time.perf_counter()
        for k, a, b in (("reset", t, t1), ("states", t1, t2), ("ops", t2, t3), ("compact", t3, t4)):
            phase[k] += (b - a) * 1e3

    for _ in range(args.warmup):
        step()
    pipe.drain()
    torch.cuda.synchronize()
    for k in phase:
        phase[k] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        MARKS.push()
        step()
        MARKS.pop()
    pipe.flush()                 # every sealed file downloaded
    t_loop = time.perf_counter()
    out["name"] = pipe.drain()   # and named
    out["file"] = pipe.last_file
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    ms = (t_end - t0) * 1e3 / args.steps
    # the same loop without its tail: the names still being hashed when the last step returns
    # (one 35 MB SHA3-256 is ~48 ms on one host thread, spread over the steps the timed region holds)
    ms_loop = (t_loop - t0) * 1e3 / args.steps
    drain_ms = (t_end - t_loop) * 1e3
    phase_timed = dict(phase)
    # the per-kernel breakdown from a few more steps with the event timers on (two event records
    # per timed launch: host time the timed loop above does not pay)
    ctx.timing_reset()
    ctx.set_timing(True)
    for _ in range(min(10, args.steps)):
        step()
    pipe.flush()
    pipe.drain()
    ctx.set_timing(False)
    # the same steps with the state files staged from host buffers (PCIe-inclusive; never value)
    host_states[0] = True
    step()
    pipe.drain()
    torch.cuda.synchronize()
    th0 = time.perf_counter()
    nh = max(4, args.steps // 4)
    for _ in range(nh):
        step()
    pipe.flush()
    th1 = time.perf_counter()
    pipe.drain()
    host_states[0] = False
    # diagnostic leg: the same pipelined step with the content names off (the host's SHA3 load
    # beside the device pipeline removed; never the line's value)
    pipe.names = False
    step()
    pipe.flush()
    torch.cuda.synchronize()
    tn0 = time.perf_counter()
    nn = max(10, args.steps // 2)
    for _ in range(nn):
        step()
    pipe.flush()
    torch.cuda.synchronize()
    no_names = {"ms_per_step": round((time.perf_counter() - tn0) * 1e3 / nn, 3), "steps": nn,
                "what": "diagnostic: the same pipelined step (downloads included) without the SHA3-256 "
                        "content names, i.e. without the host hashing load beside the device pipeline"}
    pipe.names = not NO_NAMES
    states_from_host = {"pipelined_ms_per_step": round((th1 - th0) * 1e3 / nh, 3), "steps": nh,
                        "what": "the same step with the 8 state files uploaded from per-file host "
                                "buffers each step (ce_core_ingest_states_iov: pinned staging + DMA)"}
    names = ("open_setup", "open_small", "segments_open", "finalize_open", "gate", "ds_count", "ds_emit",
             "ds_contig", "ds_applied", "ds_add_pairs", "ds_kill", "ds_finalize", "ds_part_fold", "ds_merge",
             "seal_setup", "segments_seal")
    kern = {k: ctx.timing(k) for k in names}
    sb = core.state_bytes()
    t_n = time.perf_counter()
    crdtenc.content_name(out["file"])     # one SHA3-256 name, timed alone (untimed region)
    name_ms = round((time.perf_counter() - t_n) * 1e3, 3)
    # one Core::compact as a caller sees it (crdt-enc/src/lib.rs:332-363): nothing pipelined --
    # reset, read_remote_states, read_remote_ops, serialize + seal + download, then the content
    # name store_state needs before compact returns (crdt-enc-tokio/src/lib.rs:403-432)
    single = []
    for _ in range(3):
        torch.cuda.synchronize()
        t_s = time.perf_counter()
        core.reset()
        assert core.ingest_states_device(sdev.data_ptr(), soffs.data_ptr(), len(states), sblob) == 0
        assert core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, all_actors,
                                      fa.data_ptr(), fv.data_ptr()) == 0
        t_c = time.perf_counter()
        obuf[0], ln, _ = core.compact_into(obuf[0], name=False)
        t_h = time.perf_counter()
        crdtenc.content_name(obuf[0][:ln])
        t_e = time.perf_counter()
        single.append(((t_e - t_s) * 1e3, (t_c - t_s) * 1e3, (t_h - t_c) * 1e3, (t_e - t_h) * 1e3))
    best = min(single)
    single_call = {"ms": round(best[0], 3), "read_remote_ms": round(best[1], 3),
                   "serialize_seal_download_ms": round(best[2], 3), "content_name_ms": round(best[3], 3),
                   "what": "one Core::compact, nothing pipelined (best of 3): read_remote (states + "
                           "ops) -> serialize + seal + download -> SHA3-256/BASE32 name of the "
                           "state file on one host thread (a sequential sponge)"}

    # checks: closed-form clock; sharded fold + merge_state == whole fold
    import msgpack
    d = msgpack.unpackb(sb, raw=True, strict_map_key=False)
    clock = d[b"state"][b"clock"][b"dots"]
    want = N_ADD * (V0 + V)
    clock_ok = len(clock) == N_ACTORS and all(c == want for c in clock.values())
    entries = len(d[b"state"][b"entries"])
    parts = []
    for r in range(2):
        p = new_core(ctx, key)
        lo, hi = r * N_ACTORS // 2, (r + 1) * N_ACTORS // 2
        for sw_i in range(8 * r // 2, 8 * (r + 1) // 2):
            assert p.ingest_states([states[sw_i]])[0] == 0
        f0, f1 = lo * V, hi * V
        b0, b1 = int(offs[f0]), int(offs[f1])
        sub = files[b0:b1]
        so = (offs[f0:f1 + 1] - b0).contiguous()
        rc = p.ingest_ops_device(sub.data_ptr(), so.data_ptr(), f1 - f0, b1 - b0,
                                 b"".join(bytes(a) for a in actors[lo:hi]),
                                 (fa[f0:f1] - lo).contiguous().data_ptr(), fv[f0:f1].contiguous().data_ptr())
        assert rc == 0, rc
        parts.append(p)
    parts[0].merge_state(parts[1].state_bytes())
    shard_ok = parts[0].state_bytes() == sb
    for p in parts:
        p.close()

    # CPU baseline: the whole step's workload (every state and op file), state bytes vs the GPU's
    cpu = None
    if not args.no_cpu:
        hb = files[:blob_len].cpu().numpy()
        ho = offs.cpu().numpy().astype(np.uint64)
        ha = actors[fa.cpu().numpy()]
        hv = fv.cpu().numpy().astype(np.uint64)
        cpu = orswot_cpu_baseline(key, states, hb, ho, ha, hv, sb,
                                  "the whole step: %d state files + %d op files, sealed + named"
                                  % (len(states), n))
        del hb

    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in kern.items() if v[1]}
    n_state = len(states)
    pt_ops = rc_stats["plaintext_bytes"] if rc_stats else n * PT_LEN
    ct = pt_ops + sum(len(s) for s in states)
    open_ms = sum(k_ms.get(x, 0) for x in ("open_setup", "open_small", "segments_open", "finalize_open"))
    # fold roofline: algorithmic bytes of the columnar fold per step -- adds: actor 4 + counter 8
    # + mbeg 4 + member 8 + pair key/value RMW 32; removals: cbeg/mbeg 8 + clock entry 12 +
    # member 8 + pair key/kill 24
    n_add, n_rm = n * N_ADD, n * N_RM
    n_rmc = rc_stats["clock_entries"] if rc_stats else n_rm   # removal clock entries
    fold_bytes = n_add * (4 + 8 + 4 + 8 + 32) + n_rm * (8 + 8) + n_rmc * (12 + 24)
    # (the partitioned fold: applied flags + ds_part_fold = member probes, bucketing, the LDS fold
    # with finalize, the clock; the global kernels: applied + add_pairs + kill, finalize apart)
    # (ds_contig: the contiguity check, which also writes the applied flags of increasing runs)
    fold_ms = sum(k_ms.get(x, 0) for x in ("ds_applied", "ds_contig", "ds_add_pairs", "ds_kill", "ds_part_fold"))
    # the op open's VALU roofline: SURVEY §8(d)'s int32 lane-ops per file at the op files' mean
    # plaintext length, over the open kernels' time (setup + the fused DS open) against the
    # 78.6 T lane-op/s slot peak (bench.py roofline)
    mean_pt = pt_ops / n
    ops_file = 992 * math.ceil(mean_pt / 64) + 992 + 960 + 48 * (math.ceil(mean_pt / 16) + 1)
    op_open_ms = sum(k_ms.get(x, 0) for x in ("open_setup", "open_small"))
    open_roofline = None
    if op_open_ms:
        ach = ops_file * n / (op_open_ms / 1e3) / 1e12
        open_roofline = {"bound": "valu", "ops_per_file": ops_file, "files": n,
                         "ms": round(op_open_ms, 4), "achieved": round(ach, 2), "peak": 78.6,
                         "unit": "T int32 lane-ops/s", "frac": round(ach / 78.6, 4),
                         "note": "ops at the op files' mean plaintext (%.0f B); open_setup covers the state "
                                 "files' setup as well" % mean_pt}
    shape = ("26 Add + 6 Rm, %d B" % PT_LEN if not rc_stats else
             "26 Add + 6 Rm whose clocks are the removed member's read context (the state files' adds "
             "of it + the writer's own: %.2f entries per clock), %.0f B mean, %d B max"
             % (n_rmc / n_rm, rc_stats["mean_file_plaintext"], rc_stats["max_file_plaintext"]))
    line = {
        "metric": "C3 op+state files compacted/sec (Orswot<u64,Uuid>)" + (
            ", read-context removals" if rc_stats else ""),
        "value": round((n + n_state) / (ms / 1e3), 1), "unit": "files/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32/u64", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C3: Orswot, %d members, %d actors; %d state files (512 actors x %d "
                               "versions each) + %d op files (4096 x %d versions, %s), "
                               "all resident in HBM" % (N_MEMBERS, N_ACTORS, n_state, V0, n, V, shape),
                   "rm_ctx": rm_ctx, "removal_clock_entries": n_rmc,
                   "ops": n * (N_ADD + N_RM), "entries": entries,
                   "state_file_bytes": int(len(out["file"])), "name_ms": name_ms},
        "single_compact_latency": single_call,
        "states_from_host": states_from_host,
        "pipelined": {"ms_per_step": round(ms_loop, 3), "name_drain_ms": round(drain_ms, 3),
                      "download_overlap": pipe.use_async,
                      "download_engine": "sdma" if core.path_count("compact_download_sdma") else "runtime copy",
                      "name_threads": name_threads(),
                      "name_batch": int(os.environ.get("CE_NAME_BATCH", "4")),
                      "what": "steps back to back, each sealed file's download overlapping the next "
                              "step on the device (ce_core_compact_into_async) and its content name "
                              "hashed on %d host threads; timed up to the last download; ms_per_step "
                              "above adds the names still being hashed then (drain / steps)" % name_threads()},
        "no_names": no_names,
        "aead_open_GBps": round(ct / (open_ms / 1e3) / 1e9, 1) if open_ms else None,
        "open_roofline": open_roofline,
        "fold": {"kernels": "applied flags (ds_contig for increasing runs, else ds_applied) + ds_part_fold (member "
                            "probes, items into per-partition runs, LDS fold + finalize, clock)" if "ds_part_fold" in k_ms
                 else "ds_applied + ds_add_pairs + ds_kill",
                 "ms": round(fold_ms, 4),
                 "algorithmic_bytes": fold_bytes,
                 "achieved_GBps": round(fold_bytes / (fold_ms / 1e3) / 1e9, 1) if fold_ms else None,
                 "peak_GBps": 8000.0},
        "kernels_ms_per_step": k_ms,
        "phases_ms_per_step": {k: round(v / args.steps, 3) for k, v in phase_timed.items()},
        "cpu_baseline": cpu,
        "checks": {"closed_form_clock": clock_ok, "sharded_merge_equals_whole": shard_ok},
    }
    pipe.close()
    core.close()
    return line



def dots_plaintext(uuid, k, ctr0):
    """APP || msgpack([Dot{actor, counter}] * k), counters ctr0+1 .. ctr0+k as uint32 (38 B per
    Dot, rmp-serde's smallest array header)."""
    hdr = bytes([0x90 | k]) if k <= 15 else (b"\xdc" + k.to_bytes(2, "big") if k <= 0xffff
                                             else b"\xdd" + k.to_bytes(4, "big"))
    d = np.empty((k, 38), np.uint8)
    d[:, 0:9] = np.frombuffer(b"\x82\xa5actor\xc4\x10", np.uint8)
    d[:, 9:25] = uuid
    d[:, 25:33] = np.frombuffer(b"\xa7counter", np.uint8)
    d[:, 33] = 0xce
    c = np.arange(ctr0 + 1, ctr0 + k + 1, dtype=np.uint64)
    for b in range(4):
        d[:, 34 + b] = (c >> np.uint64(8 * (3 - b))) & np.uint64(255)
    return APP + hdr + d.tobytes()


def c4_roofline(pt_len, f_len, k_ms):
    """C4's segment pass (multi-page files: open + Vec<Dot> decode + fold in k_segments) against
    the VALU slot peak, like C2's line: ops = 992 * ceil(ct / 64) + 48 * (ceil(ct / 16) + 1) per file
    (ct = plaintext length), summed over the files the pass takes, / its average launch"""
    def ops(x):
        return 992 * -(-x // 64) + 48 * (-(-x // 16) + 1)
    big = [i for i, x in enumerate(pt_len) if x > 4096]
    seg_ms = k_ms.get("segments_open")
    if not big or not seg_ms:
        return None
    o = sum(ops(pt_len[i]) for i in big)
    b = sum(f_len[i] + pt_len[i] for i in big)     # ciphertext read + plaintext written
    achieved = o / (seg_ms / 1e3) / 1e12
    return {"kernel": "k_segments<false,true> (multi-page open + decode + fold)", "bound": "valu",
            "files": len(big), "ops_per_launch": o, "avg_launch_ms": seg_ms,
            "achieved": round(achieved, 2), "peak": 78.6, "unit": "T int32 lane-ops/s",
            "frac": round(achieved / 78.6, 4),
            "hbm": {"bytes_per_launch": b, "achieved_GBps": round(b / (seg_ms / 1e3) / 1e9, 1), "peak_GBps": 8000.0},
            "ops_formula": "992*ceil(ct/64) + 48*(ceil(ct/16)+1) per multi-page file / avg launch of segments_open"}


def run_c4(args, ctx, dev):
    import msgpack
    actors = actors_table()[::4]                      # 1024 actors, UUID order
    m, V = actors.shape[0], args.c4_versions
    rng = np.random.default_rng(404)
    size = np.exp(rng.uniform(np.log(256), np.log(1 << 20), size=(m, V))).astype(np.int64)
    kd = np.maximum(1, (size - 19) // 38)             # dots per file
    n = m * V
    pt_len = [16 + (1 if k <= 15 else 3 if k <= 0xffff else 5) + 38 * int(k) for k in kd.ravel()]
    f_len = [16 + crdtenc.sealed_len(x) for x in pt_len]
    offs_h = np.zeros(n + 1, np.int64)
    offs_h[1:] = np.cumsum(f_len)
    blob_len = int(offs_h[-1])
    files = torch.empty(blob_len + 64, dtype=torch.uint8, device=dev)
    t0 = time.time()
    # seal in chunks of ~256 MB of plaintext on the GPU (seeded nonces)
    gen = np.random.default_rng(405)
    i = 0
    cum = np.zeros(m, np.int64)
    while i < n:
        j, tot = i, 0
        while j < n and (j == i or tot + pt_len[j] <= 1 << 28):
            tot += pt_len[j]
            j += 1
        parts, coffs = [], [0]
        for f in range(i, j):
            a, v = divmod(f, V)
            parts.append(dots_plaintext(actors[a], int(kd[a, v]), 65536 + int(cum[a])))
            cum[a] += kd[a, v]
            coffs.append(coffs[-1] + len(parts[-1]))
        clear = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
        co = torch.tensor(coffs, dtype=torch.int64, device=dev)
        nonces = torch.from_numpy(gen.integers(0, 256, (j - i, 24), dtype=np.uint8)).to(dev)
        oo = torch.from_numpy(offs_h[i:j].copy()).to(dev)
        torch.cuda.current_stream().synchronize()
        ctx.encrypt_batch_device(KEY, clear.data_ptr(), co.data_ptr(), j - i, nonces.data_ptr(),
                                 files.data_ptr(), oo.data_ptr(), outer_version=CORE)
        ctx.synchronize()
        i = j
    offs = torch.from_numpy(offs_h).to(dev)
    fa = torch.from_numpy(np.repeat(np.arange(m, dtype=np.int32), V)).to(dev)
    fv = torch.from_numpy(np.tile(np.arange(V, dtype=np.int64), m)).to(dev)
    log("c4: sealed %d files (%.2f GB, %d > 4 KiB) in %.1f s" % (n, blob_len / 1e9,
                                                                int((np.array(pt_len) > 4096).sum()), time.time() - t0))
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(KEY)
    wr = b"".join(bytes(a) for a in actors)

    def step():
        core.reset()
        rc, f, _ = core.compact_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, wr,
                                           fa.data_ptr(), fv.data_ptr(), name=False)
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        return f

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    t = time.perf_counter()
    for _ in range(args.steps):
        f = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / args.steps
    ctx.set_timing(False)
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in
            ((k, ctx.timing(k)) for k in ("open_setup", "gate", "open_fold_small", "segments_open",
                                         "finalize_open", "decode", "merge")) if v[1]}
    want = msgpack.packb({"next_op_versions": {"dots": {bytes(a): V for a in actors}},
                          "state": {"inner": {"dots": {bytes(actors[a]): 65536 + int(kd[a].sum())
                                                       for a in range(m)}}}}, use_bin_type=True)
    ok = core.state_bytes() == want
    sys.path.insert(0, REPO)
    import bench
    clock = None if args.no_clock else bench.probe_clock(ctx, step, dev)
    ct = sum(pt_len)
    cpu = None
    if not args.no_cpu:  # the first A actors' files through the GPU path and the oracle
        A = min(args.c4_cpu_actors, m)
        sn = A * V
        core.reset()
        rc = core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), sn, int(offs_h[sn]), wr[: 16 * A],
                                    fa.data_ptr(), fv.data_ptr())
        gpu_sample = core.state_bytes() if rc == 0 else None
        hb = files[: int(offs_h[sn])].cpu().numpy()
        h_act = np.ascontiguousarray(actors[np.repeat(np.arange(A), V)])
        cpu = gcounter_cpu_baseline(KEY, hb, np.ascontiguousarray(offs_h[: sn + 1].astype(np.uint64)), h_act,
                                    np.tile(np.arange(V, dtype=np.uint64), A), lambda e, ser: e == 0 and ser == gpu_sample,
                                    "%d files (%d actors x %d versions, %.2f GB) of this workload"
                                    % (sn, A, V, offs_h[sn] / 1e9))
    line = {
        "metric": "C4 skewed-size op files compacted/sec + AEAD GB/s (GCounter, 256 B-1 MiB)",
        "value": round(n / (ms / 1e3), 1), "unit": "files/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C4: %d GCounter op files (%d actors x %d versions), plaintext "
                               "log-uniform on [256 B, 1 MiB], %.2f GB" % (n, m, V, ct / 1e9),
                   "files_single_page": int((np.array(pt_len) <= 4096).sum()),
                   "dots": int(kd.sum())},
        "aead_GBps_end_to_end": round(ct / (ms / 1e3) / 1e9, 1),
        "kernels_ms_per_step": k_ms,
        "roofline": c4_roofline(pt_len, f_len, k_ms),
        "clock": clock,
        # multi-segment files folded from the segment pass's records vs decoded whole, over
        # every ingest of the run (warmup + steps)
        "cpu_baseline": cpu,
        "decode_paths": {"ingests": args.warmup + args.steps,
                         "segdec_records": core.path_count("segdec_records"),
                         "segdec_fallback": core.path_count("segdec_fallback")},
        "checks": {"closed_form_state": ok},
    }
    core.close()
    return line


def run_c5(args, ctx, dev):
    sys.path.insert(0, REPO)
    import bench
    actors = bench.actors_table()
    key1 = bytes(np.random.default_rng(8).integers(0, 256, 32, dtype=np.uint8))
    V = args.c5_versions
    ev, od = np.ascontiguousarray(actors[0::2]), np.ascontiguousarray(actors[1::2])
    t0 = time.time()
    f0, o0, n0, l0, _ = bench.build_files(ctx, KEY, ev, actors, V, dev, seed=1234)
    f1, o1, n1, l1, _ = bench.build_files(ctx, KEY if args.c5_clean else key1, od, actors, V, dev, seed=1235)
    n = n0 + n1
    files = torch.cat([f0[:l0], f1[:l1], torch.zeros(64, dtype=torch.uint8, device=dev)])
    del f0, f1
    offs = torch.cat([o0[:n0], o1 + l0])
    blob_len = l0 + l1
    flen = l0 // n0
    # 0.1% of all files (either key) get one flipped tag bit
    rng = np.random.default_rng(506)
    tam = np.sort(rng.choice(n, size=0 if args.c5_clean else n // 1000, replace=False))
    pos = torch.from_numpy((tam + 1) * flen - 1).to(dev)
    files[pos] ^= 1
    writers = np.concatenate([ev, od])
    m = writers.shape[0]
    fa = torch.from_numpy(np.repeat(np.arange(m, dtype=np.int32), V)).to(dev)
    fv = torch.from_numpy(np.tile(np.arange(V, dtype=np.int64), m)).to(dev)
    want = np.zeros(n, np.int32)
    want[n0:] = 0 if args.c5_clean else 9
    want[tam] = 9
    log("c5: %d files (%d under the second key, %d tampered) in %.1f s" % (n, n1, len(tam), time.time() - t0))
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(KEY)
    wr = b"".join(bytes(a) for a in writers)
    empty = core.state_bytes()

    def step(status=False):
        core.reset()
        return core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, wr,
                                      fa.data_ptr(), fv.data_ptr(), want_status=status)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    t = time.perf_counter()
    for _ in range(args.steps):
        rc = step()   # the batch verdict; the per-file statuses are fetched either way
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / args.steps
    ctx.set_timing(False)
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in
            ((k, ctx.timing(k)) for k in ("open_setup", "gate", "open_fold_small")) if v[1]}
    rc2, st = step(status=True)  # untimed: the statuses as a Python list for the check
    st = np.array(st, np.int32)
    cpu = None
    if not args.no_cpu:  # the first A actors under each key, GPU verdict vs the oracle's
        A = min(args.c5_cpu_actors, ev.shape[0])
        sn = A * V
        sub = torch.cat([files[: sn * flen], files[l0: l0 + sn * flen], torch.zeros(64, dtype=torch.uint8, device=dev)])
        so = torch.arange(2 * sn + 1, dtype=torch.int64, device=dev) * flen
        sw = np.concatenate([ev[:A], od[:A]])
        sfa = torch.from_numpy(np.repeat(np.arange(2 * A, dtype=np.int32), V)).to(dev)
        sfv = torch.from_numpy(np.tile(np.arange(V, dtype=np.int64), 2 * A)).to(dev)
        core.reset()
        g_rc = core.ingest_ops_device(sub.data_ptr(), so.data_ptr(), 2 * sn, 2 * sn * flen,
                                      b"".join(bytes(a) for a in sw), sfa.data_ptr(), sfv.data_ptr())
        hb = sub[: 2 * sn * flen].cpu().numpy()
        cpu = gcounter_cpu_baseline(KEY, hb, (np.arange(2 * sn + 1, dtype=np.uint64) * flen),
                                    np.ascontiguousarray(sw[np.repeat(np.arange(2 * A), V)]),
                                    np.tile(np.arange(V, dtype=np.uint64), 2 * A),
                                    lambda e, ser: e == g_rc,
                                    "%d files (%d actors under each key x %d versions; all opened, the batch rejected) "
                                    "of this workload" % (2 * sn, A, V))
    checks = {"batch_rejected": (rc == 9 and rc2 == 9) != args.c5_clean, "statuses_match": bool((st == want).all()),
              "state_unchanged": (core.state_bytes() == empty) != args.c5_clean}
    line = {
        "metric": "C5 key-rotation mix: op files verified/sec on the reject path",
        "value": round(n / (ms / 1e3), 1), "unit": "files/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C5: %d x 4 KiB GCounter op files, 4096 actors; odd actors' files under "
                               "a second data key, %d files with a flipped tag bit; latest key only"
                               % (n, len(tam)),
                   "rejected": int((want != 0).sum())},
        "aead_open_GBps": round(n * bench.pt_len("a") / (k_ms["open_fold_small"] / 1e3) / 1e9, 1)
        if k_ms.get("open_fold_small") else None,
        "kernels_ms_per_step": k_ms,
        "cpu_baseline": cpu,
        "checks": checks,
    }
    core.close()
    return line


# ---------------------------------------------------------------------------------------------
# N > 1 ranks (one process per GPU, torch.distributed; bench.py --gpus N runs these under its
# `configs` key).  Strong scaling: the config's whole workload is split across the ranks, and
# value = the job's files / the max-over-ranks step time.
# ---------------------------------------------------------------------------------------------

def _dist():
    import torch.distributed as dist
    import shard
    return dist, shard


def _comm_device(dev):
    dist, _ = _dist()
    return "cpu" if dist.get_backend() == "gloo" else dev


def _max_over_ranks(x, dev):
    dist, shard = _dist()
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    shard.all_reduce_(t, dist.ReduceOp.MAX)
    return float(t.item())


def _all_true(ok, dev):
    dist, shard = _dist()
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
    shard.all_reduce_(t, dist.ReduceOp.MIN)
    return int(t.item()) == 1


def _timed_steps(step, steps, warmup, dev, drain=None):
    """warmup, then `steps` steps bracketed by barrier + synchronize; the max over ranks (ms)"""
    dist, _ = _dist()
    for _ in range(warmup):
        step()
    if drain:
        drain()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if drain:
        drain()
    torch.cuda.synchronize()
    dist.barrier()
    return _max_over_ranks((time.perf_counter() - t0) * 1e3 / steps, dev)


def _state_files_c3(ctx, key, actors, V0, dev, which):
    """C3's state files j in `which`: the ingest-readable compaction of writers [512 j, 512 (j+1))'s
    versions [0, V0) (as run_c3 builds them)"""
    per = N_ACTORS // 8
    out = {}
    for j in which:
        f, o, n, bl, fa, fv = seal_op_files(ctx, key, actors, j * per, (j + 1) * per, 0, V0, dev, 99 + j)
        sc = new_core(ctx, key, flags=crdtenc.COMPACT_INGEST_FORMAT)
        rc = sc.ingest_ops_device(f.data_ptr(), o.data_ptr(), n, bl,
                                  b"".join(bytes(a) for a in actors[j * per:(j + 1) * per]),
                                  fa.data_ptr(), fv.data_ptr())
        if rc:
            raise crdtenc.CeError(rc, ctx.last_error())
        out[j] = sc.compact_to_buffer(nonce=bytes(24))[0]
        sc.close()
    return out


def run_c3_multi(args, ctx, dev, world, rank):
    """C3 over N ranks: rank r holds the writers shard.actor_range(4096, N, r) -- their op files
    and the state files of their 512-writer groups -- and folds them (read_remote_states, then
    read_remote_ops; crdt-enc/src/lib.rs:401-547); the partial StateWrappers then meet along the
    binomial tree of shard.reduce_dotset, in HBM end to end (device writer -> send/recv -> device
    state reader + merge, lib.rs:446-466), and rank 0 compacts (lib.rs:332-380).  Checks: rank 0's
    state == the single-core fold of every file (built on rank 0 after the timed steps) and the
    closed-form clock."""
    dist, shard = _dist()
    if 8 % world:
        return {"skipped": "C3's 8 state files are 512-writer groups: N must divide 8", "n_gpus": world}
    actors = actors_table()
    key = KEY
    V0, V = args.state_versions, args.versions
    lo, hi = shard.actor_range(N_ACTORS, world, rank)
    per = N_ACTORS // 8
    t0 = time.time()
    mine = [j for j in range(8) if lo <= j * per < hi]
    states = _state_files_c3(ctx, key, actors, V0, dev, mine)
    my_states = [states[j] for j in mine]
    rm_ctx = getattr(args, "rm_ctx", "own")
    files, offs, n, blob_len, fa, fv = seal_op_files(ctx, key, actors, lo, hi, V0, V0 + V, dev, 1234 + rank,
                                                     rm_ctx=rm_ctx, V0=V0)
    writers = b"".join(bytes(a) for a in actors[lo:hi])
    log("c3 rank %d: writers [%d, %d), %d state files, %d op files in %.1f s" % (
        rank, lo, hi, len(my_states), n, time.time() - t0))
    core = new_core(ctx, key)
    core.register_actors([bytes(a) for a in actors])
    sdev, soffs, sblob = device_blob(my_states, dev)
    comm = _comm_device(dev)
    buf = shard.StateBuffer(dev)
    hops, timing_on = [], [False]
    pipe = CompactPipe(core, use_async=not os.environ.get("CE_C3_SYNC_COMPACT")) if rank == 0 else None
    out = {}
    phase = {"states": 0.0, "ops": 0.0, "reduce": 0.0, "compact": 0.0}

    def step():
        t_a = time.perf_counter()
        core.reset()
        if my_states:
            rc = core.ingest_states_device(sdev.data_ptr(), soffs.data_ptr(), len(my_states), sblob)
            if rc:
                raise crdtenc.CeError(rc, ctx.last_error())
        t_b = time.perf_counter()

        def ingest():
            return core.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, writers,
                                          fa.data_ptr(), fv.data_ptr())
        t_c = [0.0]

        def ingest_timed():
            r = ingest()
            t_c[0] = time.perf_counter()
            return r
        rc, _ = shard.ingest_dotset_sharded(core, ingest_timed, device=comm, snapshot=False, buf=buf,
                                            timing=hops if timing_on[0] else None)
        if rc:
            raise crdtenc.CeError(rc, "sharded C3 ingest")
        t_d = time.perf_counter()
        if rank == 0:
            pipe.compact()
        t_e = time.perf_counter()
        if timing_on[0]:
            for key_, a_, b_ in (("states", t_a, t_b), ("ops", t_b, t_c[0]), ("reduce", t_c[0], t_d),
                                 ("compact", t_d, t_e)):
                phase[key_] += (b_ - a_) * 1e3

    def drain():
        if pipe is not None:
            out["name"] = pipe.drain()

    for _ in range(args.warmup):
        step()
    drain()
    timing_on[0] = True
    ctx.timing_reset()
    ctx.set_timing(True)
    ms = _timed_steps(step, args.steps, 0, dev, drain=drain)
    ctx.set_timing(False)
    timing_on[0] = False
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in
            ((k, ctx.timing(k)) for k in ("open_setup", "open_small", "segments_open", "gate", "ds_count",
                                         "ds_emit", "ds_applied", "ds_add_pairs", "ds_kill", "ds_finalize",
                                         "ds_merge", "cols_export", "cols_merge", "seal_setup",
                                         "segments_seal")) if v[1]}
    # per-hop exchange figures: mean over the timed steps on each rank, max over ranks
    def mean(key_):
        v = [h[key_] for h in hops if key_ in h]
        return sum(v) / len(v) if v else 0.0
    hop = {k: round(_max_over_ranks(mean(k), dev), 3)
           for k in ("serialize_ms", "export_ms", "send_ms", "recv_ms", "merge_ms")}
    hop["exchange"] = "columns" if core.path_count("columns_merge") or core.path_count("columns_export") else "state bytes"
    hop_bytes = int(_max_over_ranks(max([h["bytes"] for h in hops] or [0]), dev))
    tot = torch.tensor([n + len(my_states)], dtype=torch.int64, device=dev)
    shard.all_reduce_(tot, dist.ReduceOp.SUM)
    n_total = int(tot.item())
    ok_clock = ok_whole = True
    entries = None
    if rank == 0:
        import msgpack
        sb = core.state_bytes()
        d = msgpack.unpackb(sb, raw=True, strict_map_key=False)
        clock = d[b"state"][b"clock"][b"dots"]
        ok_clock = len(clock) == N_ACTORS and all(c == N_ADD * (V0 + V) for c in clock.values())
        entries = len(d[b"state"][b"entries"])
        # the single-core fold of every file, untimed
        all_states = _state_files_c3(ctx, key, actors, V0, dev, range(8))
        fw, ow, nw, bw, faw, fvw = seal_op_files(ctx, key, actors, 0, N_ACTORS, V0, V0 + V, dev, 4321,
                                                 rm_ctx=rm_ctx, V0=V0)
        whole = new_core(ctx, key)
        assert whole.ingest_states([all_states[j] for j in range(8)])[0] == 0
        rc = whole.ingest_ops_device(fw.data_ptr(), ow.data_ptr(), nw, bw, b"".join(bytes(a) for a in actors),
                                     faw.data_ptr(), fvw.data_ptr())
        ok_whole = rc == 0 and whole.state_bytes() == sb
        whole.close()
        del fw
        pipe.close()
    ok_clock, ok_whole = _all_true(ok_clock, dev), _all_true(ok_whole, dev)
    line = {
        "metric": "C3 op+state files compacted/sec (Orswot<u64,Uuid>)" + (
            ", read-context removals" if rm_ctx == "read" else ""),
        "value": round(n_total / (ms / 1e3), 1), "unit": "files/s", "n_gpus": world, "scaling": "strong",
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32/u64", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C3: Orswot, %d members, %d actors; 8 state files (512 actors x %d versions "
                               "each) + %d op files (4096 x %d versions, 26 Add + 6 Rm, %d B), split over %d "
                               "ranks by writer" % (N_MEMBERS, N_ACTORS, V0, N_ACTORS * V, V, PT_LEN, world),
                   "files_total": n_total, "entries": entries, "rm_ctx": rm_ctx,
                   "parallelism": "writer shards (shard.actor_range) with their 512-writer state groups; "
                                  "statuses all_reduce(MAX); %s; compaction + content name on rank 0"
                                  % (("partial Orswots as columns gathered to rank 0 in HBM "
                                      "(ce_core_export_columns_device -> %s send/recv -> one "
                                      "ce_core_merge_columns_device)" if hop["exchange"] == "columns" else
                                      "partial StateWrappers reduced along a binomial tree to rank 0 in HBM "
                                      "(ce_core_state_bytes_device -> %s send/recv -> ce_core_merge_state_device)")
                                     % ("RCCL" if comm != "cpu" else "gloo (host-staged)"))},
        "exchange": {"hops_per_step": world - 1,
                     "tree_depth": 1 if hop["exchange"] == "columns" else (world - 1).bit_length(),
                     "max_state_bytes_per_hop": hop_bytes, "per_hop_ms_max_over_ranks": hop},
        "kernels_ms_per_step_rank0": k_ms,
        "phases_ms_per_step_rank0": {k: round(v / args.steps, 3) for k, v in phase.items()},
        "checks": {"closed_form_clock": ok_clock, "equals_single_core_fold": ok_whole},
    }
    core.close()
    return line


def _c4_sizes(args):
    """C4's file table (run_c4): per (actor, version) Dot counts, plaintext and file lengths, and
    each file's first counter (65536 + the actor's Dots in earlier versions)"""
    rng = np.random.default_rng(404)
    m, V = N_ACTORS // 4, args.c4_versions
    size = np.exp(rng.uniform(np.log(256), np.log(1 << 20), size=(m, V))).astype(np.int64)
    kd = np.maximum(1, (size - 19) // 38)
    ctr0 = 65536 + np.cumsum(kd, axis=1) - kd
    pt = np.array([16 + (1 if k <= 15 else 3 if k <= 0xffff else 5) + 38 * int(k) for k in kd.ravel()], np.int64)
    fl = np.array([16 + crdtenc.sealed_len(int(x)) for x in pt], np.int64)
    return kd, ctr0, pt, fl


def _seal_selected(ctx, key, sel, make_clear, f_len, dev, seed):
    """Seal the files `sel` (global indices, ascending) back to back: make_clear(i) -> plaintext,
    f_len[i] = its sealed size.  Returns (files, offs i64[n+1] on dev, n, blob_len)."""
    n = len(sel)
    offs_h = np.zeros(n + 1, np.int64)
    offs_h[1:] = np.cumsum(f_len[sel]) if n else []
    blob_len = int(offs_h[-1])
    files = torch.empty(blob_len + 64, dtype=torch.uint8, device=dev)
    gen = np.random.default_rng(seed)
    i = 0
    while i < n:
        j, tot, parts, coffs = i, 0, [], [0]
        while j < n and (j == i or tot <= (1 << 28)):   # ~256 MB of plaintext per launch
            c = make_clear(int(sel[j]))
            parts.append(c)
            coffs.append(coffs[-1] + len(c))
            tot += len(c)
            j += 1
        clear = torch.from_numpy(np.frombuffer(b"".join(parts), np.uint8).copy()).to(dev)
        co = torch.tensor(coffs, dtype=torch.int64, device=dev)
        nonces = torch.from_numpy(gen.integers(0, 256, (j - i, 24), dtype=np.uint8)).to(dev)
        oo = torch.from_numpy(offs_h[i:j].copy()).to(dev)
        torch.cuda.current_stream().synchronize()
        ctx.encrypt_batch_device(key, clear.data_ptr(), co.data_ptr(), j - i, nonces.data_ptr(),
                                 files.data_ptr(), oo.data_ptr(), outer_version=CORE)
        ctx.synchronize()
        i = j
    return files, torch.from_numpy(offs_h).to(dev), n, blob_len


def run_c4_multi(args, ctx, dev, world, rank):
    """C4 over N ranks: the skewed-size op files partitioned by address (shard.ingest_sharded:
    cross-rank version gate, pending fold, one all_reduce(MAX) of the dense batch; lib.rs:516-544),
    rank 0 compacts.  Check: every rank's StateWrapper == the closed form."""
    import msgpack
    dist, shard = _dist()
    actors = actors_table()[::4]
    m, V = actors.shape[0], args.c4_versions
    kd, ctr0, pt, fl = _c4_sizes(args)
    fa_all = np.repeat(np.arange(m, dtype=np.uint32), V)
    fv_all = np.tile(np.arange(V, dtype=np.uint64), m)
    own = crdtenc.shard_owners([bytes(a) for a in actors], fa_all, fv_all, world)
    sel = np.nonzero(own == rank)[0]
    t0 = time.time()
    files, offs, n, blob_len = _seal_selected(
        ctx, KEY, sel, lambda f: dots_plaintext(actors[f // V], int(kd.ravel()[f]), int(ctr0.ravel()[f])),
        fl, dev, 405 + rank)
    fa = torch.from_numpy(fa_all[sel].astype(np.int32)).to(dev)
    fv = torch.from_numpy(fv_all[sel].astype(np.int64)).to(dev)
    log("c4 rank %d: %d of %d files (%.2f GB) in %.1f s" % (rank, n, m * V, blob_len / 1e9, time.time() - t0))
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(KEY)
    core.register_actors([bytes(a) for a in actors])
    ops = shard.DeviceShardOps(core, b"".join(bytes(a) for a in actors), files, offs, n, blob_len, fa, fv)
    paths = set()

    def step():
        core.reset()
        rc, path = shard.ingest_sharded(ops)
        if rc:
            raise crdtenc.CeError(rc, "sharded C4 ingest " + ctx.last_error())
        paths.add(path)
        if rank == 0:
            core.compact_to_buffer(name=False)

    ctx.timing_reset()
    ctx.set_timing(True)
    ms = _timed_steps(step, args.steps, args.warmup, dev)
    ctx.set_timing(False)
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in
            ((k, ctx.timing(k)) for k in ("open_setup", "gate", "open_fold_small", "segments_open",
                                         "finalize_open", "decode")) if v[1]}
    want = msgpack.packb({"next_op_versions": {"dots": {bytes(a): V for a in actors}},
                          "state": {"inner": {"dots": {bytes(actors[a]): 65536 + int(kd[a].sum())
                                                       for a in range(m)}}}}, use_bin_type=True)
    ok = _all_true(core.state_bytes() == want, dev)
    ct = int(pt.sum())
    line = {
        "metric": "C4 skewed-size op files compacted/sec + AEAD GB/s (GCounter, 256 B-1 MiB)",
        "value": round(m * V / (ms / 1e3), 1), "unit": "files/s", "n_gpus": world, "scaling": "strong",
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C4: %d GCounter op files (%d actors x %d versions), plaintext log-uniform on "
                               "[256 B, 1 MiB], %.2f GB, partitioned by address over %d ranks"
                               % (m * V, m, V, ct / 1e9, world),
                   "files_this_rank0": n if rank == 0 else None,
                   "parallelism": "op files by address hash (ce_shard_owner), cross-rank version gate "
                                  "(stats all_reduce MAX), pending batch + flags all_reduce(MAX), exchange "
                                  "path %s; compaction on rank 0" % "/".join(sorted(paths))},
        "aead_GBps_end_to_end": round(ct / (ms / 1e3) / 1e9, 1),
        "kernels_ms_per_step_rank0": k_ms,
        "checks": {"closed_form_state_every_rank": ok},
    }
    core.close()
    return line


def run_c5_multi(args, ctx, dev, world, rank):
    """C5 over N ranks: the key-rotation batch partitioned by address; one tampered or second-key
    file anywhere rejects the whole batch on every rank (lib.rs:497-516) and no state changes.
    Checks: every rank returns AUTH, every rank's per-file statuses == expected, state unchanged."""
    dist, shard = _dist()
    sys.path.insert(0, REPO)
    import bench
    actors = bench.actors_table()
    key1 = bytes(np.random.default_rng(8).integers(0, 256, 32, dtype=np.uint8))
    V = args.c5_versions
    ev, od = np.ascontiguousarray(actors[0::2]), np.ascontiguousarray(actors[1::2])
    writers = np.concatenate([ev, od])
    mw = writers.shape[0]
    fa_all = np.repeat(np.arange(mw, dtype=np.int64), V)
    fv_all = np.tile(np.arange(V, dtype=np.int64), mw)
    n_all = mw * V
    own = crdtenc.shard_owners([bytes(a) for a in writers], fa_all.astype(np.uint32), fv_all.astype(np.uint64), world)
    sel = np.nonzero(own == rank)[0]
    half = mw // 2
    se, so = sel[fa_all[sel] < half], sel[fa_all[sel] >= half]
    t0 = time.time()
    f0, o0, n0, l0, _ = bench.build_files(ctx, KEY, ev, actors, V, dev, seed=1234 + rank,
                                          fa=fa_all[se], fv=fv_all[se])
    f1, o1, n1, l1, _ = bench.build_files(ctx, KEY if args.c5_clean else key1, od, actors, V, dev,
                                          seed=5678 + rank, fa=fa_all[so] - half, fv=fv_all[so])
    n = n0 + n1
    files = torch.cat([f0[:l0], f1[:l1], torch.zeros(64, dtype=torch.uint8, device=dev)])
    del f0, f1
    offs = torch.cat([o0[:n0], o1 + l0])
    blob_len = l0 + l1
    flen = l0 // max(n0, 1) if n0 else l1 // max(n1, 1)
    rng = np.random.default_rng(506)
    tam = np.sort(rng.choice(n_all, size=0 if args.c5_clean else n_all // 1000, replace=False))
    loc = np.concatenate([se, so])               # global index of each local file
    hit = np.nonzero(np.isin(loc, tam))[0]
    if len(hit):
        files[torch.from_numpy((hit + 1) * flen - 1).to(dev)] ^= 1
    want = np.zeros(n, np.int32)
    if not args.c5_clean:
        want[n0:] = 9
    want[hit] = 9
    fa = torch.from_numpy(fa_all[loc].astype(np.int32)).to(dev)
    fv = torch.from_numpy(fv_all[loc]).to(dev)
    log("c5 rank %d: %d of %d files (%d second-key, %d tampered) in %.1f s" % (
        rank, n, n_all, n1, len(hit), time.time() - t0))
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(KEY)
    core.register_actors([bytes(a) for a in writers])
    empty = core.state_bytes()
    ops = shard.DeviceShardOps(core, b"".join(bytes(a) for a in writers), files, offs, n, blob_len, fa, fv)
    res = {}

    def step():
        core.reset()
        res["rc"], res["path"] = shard.ingest_sharded(ops)

    ctx.timing_reset()
    ctx.set_timing(True)
    ms = _timed_steps(step, args.steps, args.warmup, dev)
    ctx.set_timing(False)
    k_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in
            ((k, ctx.timing(k)) for k in ("open_setup", "gate", "open_fold_small")) if v[1]}
    ops.want_status = True      # untimed: the statuses of this rank's files
    core.reset()
    rc2, path2 = shard.ingest_sharded(ops)
    ops.want_status = False
    st = np.array(ops.status, np.int32) if ops.status is not None else np.zeros(0, np.int32)
    exp_rc = 0 if args.c5_clean else 9
    checks = {"batch_rejected_every_rank": _all_true(res["rc"] == exp_rc and rc2 == exp_rc, dev),
              "statuses_match_every_rank": _all_true(len(st) == n and bool((st == want).all()), dev),
              "state_unchanged_every_rank": _all_true((core.state_bytes() == empty) != args.c5_clean, dev)}
    line = {
        "metric": "C5 key-rotation mix: op files verified/sec on the reject path",
        "value": round(n_all / (ms / 1e3), 1), "unit": "files/s", "n_gpus": world, "scaling": "strong",
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "dtype": "u32", "data": "synthetic (GPU-sealed, seeded)",
        "config": {"workload": "C5: %d x 4 KiB GCounter op files, 4096 actors; odd actors' files under a second "
                               "data key, %d files with a flipped tag bit; latest key only; partitioned by "
                               "address over %d ranks" % (n_all, len(tam), world),
                   "path": res.get("path"),
                   "parallelism": "op files by address hash; each rank opens its share; the failure status "
                                  "meets in the dense batch's all_reduce(MAX), so every rank rejects"},
        "kernels_ms_per_step_rank0": k_ms,
        "checks": checks,
    }
    core.close()
    return line


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c3r", "c4", "c5"])
    ap.add_argument("--rm-ctx", default="own", choices=["own", "read"],
                    help="C3 removals: 'own' = one-entry clock {writer: its own earlier counter}; 'read' = "
                         "the removed member's read context (config c3r)")
    ap.add_argument("--c4-versions", type=int, default=32, help="C4 versions per actor (1024 actors)")
    ap.add_argument("--c5-versions", type=int, default=256, help="C5 versions per actor (4096 actors)")
    ap.add_argument("--c5-clean", action="store_true",
                    help="C5 control: every file under the latest key, none tampered (accept path)")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 20; 40 for c3, whose last names are hashed after its last step)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-clock", action="store_true", help="skip the shader-clock probe (C4)")
    ap.add_argument("--c4-cpu-actors", type=int, default=256, help="C4 CPU sample: files of this many actors")
    ap.add_argument("--c5-cpu-actors", type=int, default=128, help="C5 CPU sample: actors per key")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--versions", type=int, default=16, help="op-file versions per actor")
    ap.add_argument("--state-versions", type=int, default=4, help="versions folded into states")
    return ap


def _read_ctx(run):
    """config c3r: C3 with read-context removals (SURVEY.md §8d's op shape)"""
    def go(args, *a):
        args.rm_ctx = "read"
        return run(args, *a)
    return go


RUNNERS = {"c3": run_c3, "c3r": _read_ctx(run_c3), "c4": run_c4, "c5": run_c5}
RUNNERS_MULTI = {"c3": run_c3_multi, "c3r": _read_ctx(run_c3_multi), "c4": run_c4_multi, "c5": run_c5_multi}


def run_config(name, args, ctx, dev, world=1, rank=0):
    """One config on this rank: the single-GPU runner at N = 1, the strong-scaling one at N > 1
    (every rank calls it; the line is complete on rank 0)."""
    if world == 1:
        return RUNNERS[name](args, ctx, dev)
    return RUNNERS_MULTI[name](args, ctx, dev, world, rank)


def main():
    args = make_parser().parse_args()
    if args.steps is None:
        args.steps = 120 if args.config == "c3" else 40 if args.config == "c3r" else 20
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = crdtenc.Context(0)
    ctx.set_stream(stream.cuda_stream)
    # every host thread on the GPU's NUMA node (bench.py does the same): the names' SHA3 threads
    # 3.42 -> 2.60 ms/step with the names on one box (tools/c3_names_ab.sh, CE_BENCH_NUMA_PIN=0: off)
    if os.environ.get("CE_BENCH_NUMA_PIN", "1") == "1":
        sys.path.insert(0, REPO)
        import bench
        cpus = bench.gpu_node_cpus(dev)
        if cpus:
            os.sched_setaffinity(0, cpus)
    line = RUNNERS[args.config](args, ctx, dev)
    print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
