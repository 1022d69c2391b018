"""Multi-GPU layout of the ingest path (one process per GPU, torch.distributed).

Files are sharded by writer actor: every version of an actor goes to one rank, in order.  The
version gate (crdt-enc/src/lib.rs:519-531) then only needs rank-local state.  After each rank has
folded its shard, the partial states meet in ONE exchange: VClock/GCounter merge is a pointwise
max (crdts VClock::merge; GCounter::merge delegates to it), so the dense actor-indexed arrays
(batch state and next_op_versions, exported with Core.export_dense over slots registered
identically on every rank) are combined with all_reduce(MAX).  Over RCCL that is one 64 KiB
latency-bound message per array on xGMI; with gloo it runs the same code on CPU tensors.

Counters are u64 but the collective's MAX is signed int64: the sign bit is flipped before and
after the reduce, which maps u64 order onto i64 order (values >= 2^63 stay correctly ordered).
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


def merge_dense(*tensors, group=None):
    """In place: every tensor (int64 views of u64 arrays) becomes the elementwise u64 max over
    all ranks."""
    for t in tensors:
        if t.dtype != torch.int64:
            raise TypeError("dense arrays are int64 views of u64")
        t.bitwise_xor_(_FLIP)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        t.bitwise_xor_(_FLIP)
    return tensors


def max_u64_(dst, src):
    """In place dst = u64 max(dst, src) for int64 views (the local form of merge_dense)."""
    a = dst.bitwise_xor(_FLIP)
    b = src.bitwise_xor(_FLIP)
    torch.maximum(a, b, out=a)
    dst.copy_(a.bitwise_xor_(_FLIP))
    return dst
