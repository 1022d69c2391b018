"""Multi-GPU layout of the ingest path (one process per GPU, torch.distributed).

VClock / GCounter: files are partitioned by ADDRESS (north star: "sharded by content hash").  An
op file is addressed by its path ops/<actor>/<version> (crdt-enc-tokio/src/lib.rs:280-293; op
files are not content-named), and its owner rank is a hash of that address
(crdtenc.shard_owners / ce_shard_owner), so one writer's run is spread over every rank and the
bytes balance however skewed the writers are.  The version gate (crdt-enc/src/lib.rs:519-531)
is then agreed across ranks before the fold (ingest_sharded): each rank's per-writer statistics
-- the first version >= e0 it owns but does not hold, the largest version it holds -- meet in
one all_reduce(MAX), every rank derives the same windows [e0, hi) from them, and folds exactly
the files the reference's single loop would.  The folded batch stays pending until a second
all_reduce(MAX) of the dense batch carries every rank's failure status too: any failure leaves
every rank's state unchanged (lib.rs:497-514), otherwise each rank commits the reduced batch.
A Dot naming an actor outside the registered slots sends every rank to the all-gather of
serialized states instead.

Writer sharding (actor_range / file_rank) is kept for the dot-set kinds (below) and as the
previous layout of the VClock path (exchange_vclock after a local ingest).

Counters are u64 but the collective's MAX is signed int64: the sign bit is flipped before and
after the reduce, which maps u64 order onto i64 order (values >= 2^63 stay correctly ordered).

Orswot / MVReg (dot sets) do not reduce pointwise: each rank serializes its partial
StateWrapper and the partial states are merged with Core.merge_state -- the CvRDT merge
read_remote_states applies to state files (crdt-enc/src/lib.rs:458-466), run by the GPU merge
kernel -- along a binomial tree to the compacting rank (reduce_dotset: at most ceil(log2 N)
merges per rank; exchange_dotset, the all-gather to every rank, is kept for callers that need
the merged state everywhere).  Sharding by writer keeps every actor's ops on one rank, so each
partial state is an op-based replica of that shard and the merge equals one fold over all files
(SURVEY.md §8e).
"""
import os

import torch
import torch.distributed as dist

_FLIP = torch.iinfo(torch.int64).min


def actor_range(n_actors, world, rank):
    """[start, end) of the writer actors this rank ingests (contiguous, balanced)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    return rank * n_actors // world, (rank + 1) * n_actors // world


def file_rank(actor_index, n_actors, world):
    """Rank that owns the files of global writer actor `actor_index`."""
    r = actor_index * world // n_actors
    while actor_range(n_actors, world, r)[0] > actor_index:
        r -= 1
    while actor_range(n_actors, world, r)[1] <= actor_index:
        r += 1
    return r


def _host_staged(t, group=None):
    """gloo reduces host tensors: device tensors are staged through host memory for it (the
    CPU tests and the one-GPU multi-rank rehearsal); RCCL ("nccl") reduces them in place."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce_(t, op, group=None):
    if _host_staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def merge_dense(*tensors, group=None):
    """In place: every tensor (int64 views of u64 arrays) becomes the elementwise u64 max over
    all ranks."""
    for t in tensors:
        if t.dtype != torch.int64:
            raise TypeError("dense arrays are int64 views of u64")
        t.bitwise_xor_(_FLIP)
        all_reduce_(t, dist.ReduceOp.MAX, group=group)
        t.bitwise_xor_(_FLIP)
    return tensors


def exchange_vclock(core, dense, group=None):
    """Merge the partial VClock / GCounter states of all ranks into every rank's `core`.

    Fast path: the dense actor-indexed arrays (state ‖ next_op_versions, `dense` = int64[2 cap]
    on the rank's device) are exported, all_reduce(MAX)ed once and imported.  A Dot may name an
    actor outside the registered set (VClock::apply takes any actor, crdt-enc/src/lib.rs:
    533-535); when any rank holds one, every rank falls back to the all-gather of serialized
    StateWrappers + merge_state (the exchange the dot-set kinds use).  The decision is itself
    one all_reduce(MAX) of a flag, so all ranks take the same path.  Returns "dense" or "bytes".
    """
    flag = torch.tensor([0 if core.dense_ready() else 1], dtype=torch.int64, device=dense.device)
    all_reduce_(flag, dist.ReduceOp.MAX, group=group)
    if int(flag.item()) == 0:
        cap = dense.numel() // 2
        st, nov = dense[:cap], dense[cap:]
        core.export_dense(st.data_ptr(), nov.data_ptr())
        merge_dense(dense, group=group)
        core.import_dense(st.data_ptr(), nov.data_ptr())
        return "dense"
    exchange_dotset(core, group=group,
                    device="cpu" if dist.get_backend(group) == "gloo" else dense.device)
    return "bytes"


def max_u64_(dst, src):
    """In place dst = u64 max(dst, src) for int64 views (the local form of merge_dense)."""
    a = dst.bitwise_xor(_FLIP)
    b = src.bitwise_xor(_FLIP)
    torch.maximum(a, b, out=a)
    dst.copy_(a.bitwise_xor_(_FLIP))
    return dst


def all_gather_bytes(data, group=None, device="cpu"):
    """Every rank's byte string, in rank order (variable lengths: padded to the longest)."""
    world = dist.get_world_size(group)
    n = torch.tensor([len(data)], dtype=torch.int64, device=device)
    lens = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(lens, n, group=group)
    lens = [int(x.item()) for x in lens]
    width = max(max(lens), 1)
    buf = torch.zeros(width, dtype=torch.uint8, device=device)
    if data:
        buf[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device)
    parts = [torch.empty(width, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return [bytes(p[:k].cpu().numpy().tobytes()) for p, k in zip(parts, lens)]


def _send_bytes(data, dst, group=None, device="cpu"):
    n = torch.tensor([len(data)], dtype=torch.int64, device=device)
    dist.send(n, dst, group=group)
    if data:
        dist.send(torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device), dst, group=group)


def _recv_bytes(src, group=None, device="cpu"):
    n = torch.zeros(1, dtype=torch.int64, device=device)
    dist.recv(n, src, group=group)
    k = int(n.item())
    if not k:
        return b""
    buf = torch.empty(k, dtype=torch.uint8, device=device)
    dist.recv(buf, src, group=group)
    return bytes(buf.cpu().numpy().tobytes())


def _global(group, r):
    """dist.send / recv take global ranks"""
    return r if group is None else dist.get_global_rank(group, r)


class StateBuffer:
    """A growable byte buffer in HBM for partial StateWrappers (one per rank, reused across
    steps): the dot-set exchange sends and receives it without a host copy."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.t = None

    def ensure(self, n):
        if self.t is None or self.t.numel() < n:
            self.t = torch.empty(max(n + (n >> 3), 1 << 20), dtype=torch.uint8, device=self.device)
        return self.t


_ERR_INVALID_ARG = 64


def _on_comm_device(t, comm_device):
    """t already lives where the collectives run (a plain "cuda" means the current device)"""
    d = torch.device(comm_device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return t.device == d


def _send_state_device(core, buf, dst, group, comm_device, timing):
    """core's StateWrapper serialized into HBM (ce_core_state_bytes_device: the device writer,
    complete on return) -> dist.send.  With RCCL the bytes go GPU to GPU; gloo stages them
    through the host (the CPU / one-GPU rehearsal)."""
    import time
    t0 = time.perf_counter()
    t = buf.ensure(1 << 20)
    rc, n = core.state_bytes_device(t.data_ptr(), t.numel())
    if rc == _ERR_INVALID_ARG and n > t.numel():
        t = buf.ensure(n)
        rc, n = core.state_bytes_device(t.data_ptr(), t.numel())
    if rc:
        raise RuntimeError("state_bytes_device failed: %d" % rc)
    t1 = time.perf_counter()
    dist.send(torch.tensor([n], dtype=torch.int64, device=comm_device), dst, group=group)
    if n:
        dist.send(t[:n] if _on_comm_device(t, comm_device) else t[:n].to(comm_device), dst, group=group)
        # the buffer is written again by the next export on the core's stream: the send (queued on
        # torch's stream under RCCL) must have read it first
        torch.cuda.current_stream(t.device).synchronize()
    if timing is not None:
        timing.append({"send": True, "bytes": n, "serialize_ms": round((t1 - t0) * 1e3, 3),
                       "send_ms": round((time.perf_counter() - t1) * 1e3, 3)})


def _recv_merge_device(core, buf, src, group, comm_device, timing):
    """dist.recv of a partial StateWrapper into HBM -> ce_core_merge_state_device (the device
    state reader and merge; only the state's head and deferred tail reach the host)."""
    import time
    t0 = time.perf_counter()
    hdr = torch.zeros(1, dtype=torch.int64, device=comm_device)
    dist.recv(hdr, src, group=group)
    n = int(hdr.item())
    if not n:
        raise RuntimeError("rank %d sent an empty state" % src)
    t = buf.ensure(n)
    if _on_comm_device(t, comm_device):
        dist.recv(t[:n], src, group=group)
        # the receive completes on torch's stream; the core reads on its own stream
        torch.cuda.current_stream(t.device).synchronize()
    else:
        h = torch.empty(n, dtype=torch.uint8, device=comm_device)
        dist.recv(h, src, group=group)
        t[:n].copy_(h)
        torch.cuda.current_stream(t.device).synchronize()
    t1 = time.perf_counter()
    rc = core.merge_state_device(t.data_ptr(), n)
    if rc:
        raise RuntimeError("merge_state_device from rank %d failed: %d" % (src, rc))
    if timing is not None:
        timing.append({"recv": True, "bytes": n, "recv_ms": round((t1 - t0) * 1e3, 3),
                       "merge_ms": round((time.perf_counter() - t1) * 1e3, 3)})


_MAX_COLUMN_PARTS = 64  # ce_core_merge_columns_device merges at most 64 partials per call


def _columns_ok(core, group, device):
    """every rank can exchange its partial as columns (an Orswot core; deferred removals travel in
    the columns' deferred section) and the receiver can merge all of them in one call: one
    all_reduce(MAX) of a refusal flag, so all ranks take the same path"""
    if dist.get_world_size(group) - 1 > _MAX_COLUMN_PARTS:
        return False
    flag = torch.tensor([0 if core.columns_ready() else 1], dtype=torch.int64, device=device)
    all_reduce_(flag, dist.ReduceOp.MAX, group=group)
    return int(flag.item()) == 0


def gather_dotset_columns(core, group=None, device="cpu", dst=0, buf=None, timing=None):
    """Merge the partial Orswots of all ranks into rank `dst`'s `core` in ONE k-way merge: every
    other rank exports its state as columns (ce_core_export_columns_device: the live pairs, clock,
    next versions and actor UUIDs straight from the device, no msgpack) and sends them to `dst`,
    which merges all N - 1 partials at once (ce_core_merge_columns_device; read_remote_states'
    merge, crdt-enc/src/lib.rs:458-466, of every partial, in one pass).  RCCL moves device tensors
    GPU to GPU; gloo stages them through the host.  Returns the merges this rank ran (1 on dst)."""
    import time
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if buf is None:
        buf = StateBuffer(torch.device("cuda", core.ctx.device))
    t0 = time.perf_counter()
    n, err = 0, 0
    if rank != dst:
        t = buf.ensure(1 << 20)
        rc, n = core.export_columns_device(t.data_ptr(), t.numel())
        if rc == _ERR_INVALID_ARG and n > t.numel():
            t = buf.ensure(n)
            rc, n = core.export_columns_device(t.data_ptr(), t.numel())
        if rc:
            # the failure goes into the length exchange below (n = -rc), so every rank raises
            # together instead of the others waiting in the collectives for this one
            n, err = -abs(rc), rc
    t1 = time.perf_counter()
    # every partial's length in one all_gather, then every transfer posted at once: each peer's
    # partial comes over its own xGMI link instead of one after another
    got = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(got, torch.tensor([n], dtype=torch.int64, device=device), group=group)
    lens_all = [int(x.item()) for x in got]
    bad = [(r, -x) for r, x in enumerate(lens_all) if x < 0]
    if bad:
        raise RuntimeError("export_columns_device failed on rank(s) %s" % ", ".join("%d (%d)" % b for b in bad))
    if rank != dst:
        peer = _global(group, dst)
        src = t[:n] if _on_comm_device(t, device) else t[:n].to(device)
        dist.isend(src, peer, group=group).wait()
        torch.cuda.current_stream(t.device).synchronize()  # the next export rewrites the buffer
        if timing is not None:
            timing.append({"send": True, "bytes": n, "export_ms": round((t1 - t0) * 1e3, 3),
                           "send_ms": round((time.perf_counter() - t1) * 1e3, 3)})
        return 0
    parts = getattr(buf, "parts", None)
    if parts is None:
        parts = buf.parts = {}
    ptrs, lens, reqs, staged = [], [], [], []
    for r in range(world):
        if r == dst:
            continue
        n = lens_all[r]
        pb = parts.setdefault(r, StateBuffer(buf.device))
        t = pb.ensure(n)
        if _on_comm_device(t, device):
            reqs.append(dist.irecv(t[:n], _global(group, r), group=group))
        else:
            h = torch.empty(n, dtype=torch.uint8, device=device)
            reqs.append(dist.irecv(h, _global(group, r), group=group))
            staged.append((t, h, n))
        ptrs.append(t.data_ptr())
        lens.append(n)
    for q in reqs:
        q.wait()
    for t, h, n in staged:
        t[:n].copy_(h)
    torch.cuda.current_stream(buf.device).synchronize()  # the receives land on torch's stream
    t2 = time.perf_counter()
    rc = core.merge_columns_device(ptrs, lens)
    if rc:
        raise RuntimeError("merge_columns_device failed: %d" % rc)
    if timing is not None:
        timing.append({"recv": True, "parts": len(lens), "bytes": sum(lens), "recv_ms": round((t2 - t1) * 1e3, 3),
                       "merge_ms": round((time.perf_counter() - t2) * 1e3, 3)})
    return 1


def reduce_dotset(core, group=None, device="cpu", dst=0, buf=None, timing=None):
    """Merge the partial Orswot / MVReg states of all ranks into rank `dst`'s `core` along a
    binomial tree: in round k (k = 0, 1, ...) the rank at distance 2^k above a multiple of
    2^(k+1) sends its (already merged) StateWrapper to that multiple, which merges it (the
    CvRDT merge of read_remote_states, crdt-enc/src/lib.rs:446-466, on the GPU).  Only the
    compacting rank ends with the whole state; every rank does at most ceil(log2 N) merges and
    each state crosses the fabric once (exchange_dotset: N - 1 merges on every rank).

    With a crdtenc.Core the state stays in HBM end to end: serialized by the device writer into
    `buf` (a StateBuffer; made here when None), sent / received as a device tensor (RCCL: GPU to
    GPU over xGMI; gloo stages it through the host), merged by the device state reader.  Other
    cores (the CPU tests' twins) exchange host bytes.  `device` is the collectives' device
    ("cpu" for gloo).  `timing` (a list) receives one record per hop.  Returns the number of
    merges this rank ran."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    rel = (rank - dst) % world
    on_device = hasattr(core, "state_bytes_device")
    # device Orswot cores: the partials as columns, one k-way merge on dst (CE_DS_EXCHANGE=tree:
    # the binomial tree of serialized partials below, for A/B)
    if (on_device and world > 1 and hasattr(core, "export_columns_device") and getattr(core, "kind", None) == 2
            and os.environ.get("CE_DS_EXCHANGE") != "tree" and _columns_ok(core, group, device)):
        return gather_dotset_columns(core, group=group, device=device, dst=dst, buf=buf, timing=timing)
    if on_device and buf is None:
        buf = StateBuffer(torch.device("cuda", core.ctx.device))
    merges, step = 0, 1
    while step < world:
        if rel % (2 * step) == step:          # send to the partner below, then done
            peer = _global(group, (rank - step) % world)
            if on_device:
                _send_state_device(core, buf, peer, group, device, timing)
            else:
                _send_bytes(core.state_bytes(), peer, group=group, device=device)
            break
        if rel % (2 * step) == 0 and rel + step < world:
            peer = _global(group, (rank + step) % world)
            if on_device:
                _recv_merge_device(core, buf, peer, group, device, timing)
            else:
                sw = _recv_bytes(peer, group=group, device=device)
                rc = core.merge_state(sw)
                if rc:
                    raise RuntimeError("merge_state from rank %d failed: %d" % (peer, rc))
            merges += 1
        step *= 2
    return merges


def ingest_dotset_sharded(core, ingest, group=None, device="cpu", snapshot=True, buf=None, timing=None):
    """read_remote_ops of the dot-set kinds over writer shards (actor_range), then the tree
    reduce to rank 0 (reduce_dotset; buf / timing passed through).  `ingest()` folds this rank's
    files into `core` and returns its status.
    All-or-nothing across ranks (lib.rs:497-514): the statuses meet in one all_reduce(MAX) before
    any state moves; on a failure anywhere, every rank that folded its shard goes back to the
    StateWrapper it held before (reset + merge_state of the snapshot) and the failing status is
    returned on every rank.  snapshot=False: the caller knows the state before the ingest (e.g.
    empty after a reset) and restores it itself; a failure then raises.  Returns (rc, merges)."""
    s0 = core.state_bytes() if snapshot else None
    rc = ingest()
    if rc == 0 and hasattr(core, "settle"):
        rc = core.settle()  # a device table overflow is only seen once the fold has run
    code = torch.tensor([rc], dtype=torch.int64, device=device)
    all_reduce_(code, dist.ReduceOp.MAX, group=group)
    code = int(code.item())
    if code:
        if rc == 0:
            if s0 is None:
                raise RuntimeError("a rank failed and no snapshot was kept")
            core.reset()
            if core.merge_state(s0):
                raise RuntimeError("restoring the snapshot failed")
        return code, 0
    return 0, reduce_dotset(core, group=group, device=device, buf=buf, timing=timing)


def exchange_dotset(core, group=None, device="cpu"):
    """Merge the partial Orswot / MVReg states of all ranks into `core` (a crdtenc.Core or any
    object with state_bytes() / merge_state(bytes) -> status)."""
    rank = dist.get_rank(group)
    states = all_gather_bytes(core.state_bytes(), group=group, device=device)
    for r, sw in enumerate(states):
        if r != rank:
            rc = core.merge_state(sw)
            if rc:
                raise RuntimeError("merge_state of rank %d failed: %d" % (r, rc))
    return core


# ---------------------------------------------------------------------------------------------
# VClock / GCounter partitioned by op-file address: the cross-rank version gate
# ---------------------------------------------------------------------------------------------
ERR_OP_VERSION, ERR_SHARD = 13, 69
SHARD_BAD, SHARD_GAP, SHARD_E0_MISMATCH = 1, 2, 4


class DeviceShardOps:
    """The sharded-ingest steps of a crdtenc.Core over this rank's batch resident in HBM
    (torch tensors: files u8, offs i64[n+1], fa i32[n] into the shared writer list, fv i64[n])."""

    def __init__(self, core, actors, files, offs, n, blob_len, fa, fv):
        self.core, self.actors = core, actors
        self.files, self.offs, self.n, self.blob_len, self.fa, self.fv = files, offs, n, blob_len, fa, fv
        self.want_status = False   # True: ingest() keeps the per-file statuses in self.status
        self.status = None
        self.m = len(actors) // 16
        self.device = fa.device
        self.stats = torch.empty(2 * self.m + 3, dtype=torch.int64, device=self.device)
        self.hi = torch.empty(self.m + 1, dtype=torch.int64, device=self.device)
        self.dense = torch.empty(core.dense_capacity() + 2, dtype=torch.int64, device=self.device)

    def _ordered(self):
        """The core runs on its context's stream: when that is not torch's current stream, what
        torch (or a collective) wrote must be complete before the core reads it."""
        cur = torch.cuda.current_stream(self.device)
        if getattr(self.core.ctx, "stream_ptr", None) != cur.cuda_stream:
            cur.synchronize()

    def compute_stats(self, rank, world):
        self.core.shard_stats(self.actors, self.fa.data_ptr(), self.fv.data_ptr(), self.n, rank, world,
                              self.stats.data_ptr())
        return self.stats

    def window(self):
        self._ordered()
        self.core.shard_window(self.actors, self.stats.data_ptr(), self.hi.data_ptr())
        return self.hi

    def set_window(self, hi, flags):
        import numpy as np
        h = np.append(np.asarray(hi, np.uint64), np.uint64(flags)).view(np.int64)
        self.hi.copy_(torch.from_numpy(h))
        self._ordered()

    def metadata(self):
        return self.fa[: self.n].cpu().numpy().astype("uint32"), self.fv[: self.n].cpu().numpy().astype("uint64")

    def writer_versions(self):
        return self.core.writer_versions(self.actors)

    def ingest(self):
        r = self.core.ingest_ops_device_sharded(self.files.data_ptr(), self.offs.data_ptr(), self.n,
                                                self.blob_len, self.actors, self.fa.data_ptr(),
                                                self.fv.data_ptr(), self.hi.data_ptr(),
                                                want_status=self.want_status)
        if self.want_status:
            r, self.status = r
        return r

    def dense_buffer(self):
        self.dense.zero_()
        return self.dense

    def export_pending(self, dense):
        """False (nothing written) when the batch cannot go through the dense reduce: an actor
        outside the registered slots, or a table grown past `dense` during the ingest."""
        if dense.dtype != torch.int64:
            raise TypeError("dense is an int64 view of u64")
        self._ordered()
        return self.core.pending_export(dense.data_ptr(), dense.numel())

    def commit(self, accept, reduced=None):
        self._ordered()
        if reduced is None:
            self.core.pending_commit(accept)
        else:
            self.core.pending_commit(accept, reduced.data_ptr(), reduced.numel())


def contract_flags(stats):
    """SHARD_BAD | SHARD_E0_MISMATCH from reduced ShardStats (int64[2m + 3], the last three words
    flipped-u64: contract flag, h(e0), ~h(e0); layout ce_common.h) -- the flags word the window
    kernel derives, read on the host so every rank branches on the same value."""
    import numpy as np
    t = stats[-3:].cpu().numpy().view(np.uint64) ^ np.uint64(1 << 63)
    bad, h, nh = (int(x) for x in t)
    return (SHARD_BAD if bad else 0) | (SHARD_E0_MISMATCH if h != (~nh & 0xFFFFFFFFFFFFFFFF) else 0)


def _gather_metadata(fa, fv, group=None):
    """Every rank's (writer, version) metadata, concatenated (the exact fallback's input)."""
    import numpy as np
    blob = np.concatenate([np.asarray(fa, np.uint32).view(np.uint8),
                           np.asarray(fv, np.uint64).view(np.uint8)]).tobytes()
    parts = all_gather_bytes(blob, group=group)
    fas, fvs = [], []
    for p in parts:
        k = len(p) // 12
        fas.append(np.frombuffer(p[: 4 * k], np.uint32))
        fvs.append(np.frombuffer(p[4 * k:], np.uint64))
    return np.concatenate(fas), np.concatenate(fvs)


def ingest_sharded(ops, group=None, exchange_bytes=None):
    """read_remote_ops (crdt-enc/src/lib.rs:471-547) over a batch partitioned across the ranks by
    op-file address.  `ops`: a DeviceShardOps (or the CPU test's twin).  Every rank ends with the
    state the reference reaches folding the whole batch in (shared writer order, version) order.
    Returns (rc, path): rc 0, CE_ERR_OP_VERSION (the fold stopped at a gap; the files before it
    are folded on every rank) or the failing status (every rank's state unchanged); path
    "dense" | "bytes" (state all-gather) | "rejected", plus "+exact" when the windows came from
    the gathered metadata."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    # 1) the gate: per-writer stats, one all_reduce(MAX), identical windows on every rank
    stats = ops.compute_stats(rank, world)
    all_reduce_(stats, dist.ReduceOp.MAX, group=group)
    # The path is chosen from the reduced stats' flag words, identical on every rank, never from
    # one rank's ingest status: a rank failing early (no key, a bad file) must still take the
    # same collectives as the others.
    flags = contract_flags(stats)
    if flags & SHARD_E0_MISMATCH:
        # the ranks started from different next_op_versions: no window is right for all of them
        # (the exact fallback would compute each rank's from its own e0); refused, nothing folded
        return ERR_SHARD, "refused"
    exact = ""
    if flags & SHARD_BAD:
        # a rank's batch breaks the partition contract: the windows from everyone's metadata,
        # the reference loop on the host (one gather, every rank)
        import crdtenc
        e0 = ops.writer_versions()
        fa, fv = ops.metadata()
        fa_all, fv_all = _gather_metadata(fa, fv, group=group)
        hi, wflags = crdtenc.shard_window_exact(e0, fa_all, fv_all)
        ops.set_window(hi, wflags)
        exact = "+exact"
    else:
        ops.window()
    # any failure here, including a rank-local early return, reaches every rank through the
    # reduce below, and every rank keeps its state
    rc = ops.ingest()
    # 2) all-or-nothing + exchange: the pending batch and the failure flags in one all_reduce
    failed = rc not in (0, ERR_OP_VERSION)
    dense = ops.dense_buffer()
    cap = dense.numel() - 2
    ready = ops.export_pending(dense[:cap]) if not failed else True
    flags = torch.tensor([rc if failed else 0, 0 if ready else 1], dtype=torch.int64)
    dense[cap:].copy_(flags.to(dense.device))
    merge_dense(dense, group=group)
    code, not_ready = (int(x) for x in dense[cap:].cpu().tolist())
    if code:
        if not failed:
            ops.commit(False)
        return code, "rejected" + exact
    if not_ready:
        ops.commit(True)
        (exchange_bytes or exchange_dotset)(ops.core, group=group,
                                            device="cpu" if dist.get_backend(group) == "gloo" else dense.device)
        return rc, "bytes" + exact
    ops.commit(True, dense[:cap])
    return rc, "dense" + exact

