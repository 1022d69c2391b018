"""Multi-GPU layout of the ingest path (one process per GPU, torch.distributed).

Files are sharded by writer actor: every version of an actor goes to one rank, in order.  The
version gate (crdt-enc/src/lib.rs:519-531) then only needs rank-local state.  After each rank has
folded its shard, the partial states meet in ONE exchange: VClock/GCounter merge is a pointwise
max (crdts VClock::merge; GCounter::merge delegates to it), so the dense actor-indexed arrays
(batch state and next_op_versions, exported with Core.export_dense over slots registered
identically on every rank) are combined with all_reduce(MAX).  Over RCCL that is one 64 KiB
latency-bound message per array on xGMI; with gloo it runs the same code on CPU tensors.  A
Dot naming an actor outside the registered slots sends every rank to the all-gather of
serialized partial states instead (exchange_vclock).

Counters are u64 but the collective's MAX is signed int64: the sign bit is flipped before and
after the reduce, which maps u64 order onto i64 order (values >= 2^63 stay correctly ordered).

Orswot / MVReg (dot sets) do not reduce pointwise: each rank serializes its partial
StateWrapper, the byte strings are all-gathered (one length exchange + one padded all_gather),
and every rank merges the others' partial states with Core.merge_state -- the CvRDT merge
read_remote_states applies to state files (crdt-enc/src/lib.rs:458-466), run by the GPU merge
kernel.  Sharding by writer keeps every actor's ops on one rank, so each partial state is an
op-based replica of that shard and the merge equals one fold over all files.
"""
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
