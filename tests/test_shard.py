"""Multi-GPU partition of VClock / GCounter op files by address (shard.ingest_sharded,
include/crdtenc.h ce_shard_*), on CPU:

  * the product's host twins of the gate (ce_shard_stats_host over each rank's share ->
    all_reduce(MAX) -> ce_shard_window_host) give the same windows as the reference's loop over
    the whole batch in (writer, version) order (ce_shard_window_exact, crdt-enc/src/lib.rs:
    516-544), on randomized batches with holes, old versions, duplicates and replicated e0;
  * world-2 gloo runs of shard.ingest_sharded itself (tests/shard_twin.py: the oracle opens and
    folds, the product's host twins gate) where one writer's run is split across both ranks,
    with a gap, skipped old versions, a tampered file, a partition-contract break (the exact
    fallback) and an unregistered Dot actor (the bytes exchange): every rank's state == the
    oracle's single fold.
"""
import os
import random
import socket
import sys

import msgpack
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "crdt-enc_amd"), REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import crdtenc  # noqa: E402
import shard  # noqa: E402

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
FLIP = np.uint64(1 << 63)


def _reduce_max(stats_list):
    """all_reduce(MAX) of int64 stats (the flipped-u64 encoding makes it the u64 max)."""
    return np.maximum.reduce(stats_list)


def test_owner_is_deterministic_and_balanced():
    rng = random.Random(3)
    actors = [rng.randbytes(16) for _ in range(64)]
    fa = np.repeat(np.arange(64, dtype=np.uint32), 512)
    fv = np.tile(np.arange(512, dtype=np.uint64), 64)
    for world in (1, 2, 3, 8):
        own = crdtenc.shard_owners(actors, fa, fv, world)
        assert own.max() < world
        cnt = np.bincount(own, minlength=world)
        assert cnt.min() > 0.9 * len(fa) / world, cnt
        one = [crdtenc.lib().ce_shard_owner(actors[int(fa[i])], int(fv[i]), world) for i in range(0, len(fa), 997)]
        assert one == list(own[::997])
    # a writer's run is spread over every rank (the property writer sharding lacks)
    own = crdtenc.shard_owners(actors, fa, fv, 8)
    for a in range(64):
        assert len(set(own[fa == a])) == 8


def _random_batch(rng, m, world):
    """Writers with random version sets (holes, old versions, duplicates) and a replicated e0."""
    e0 = np.array([rng.choice([0, 0, 1, 5, 17]) for _ in range(m)], np.uint64)
    fa, fv = [], []
    for a in range(m):
        kind = rng.random()
        top = int(e0[a]) + rng.randint(0, 40)
        vs = list(range(0, top))
        if kind < 0.3:           # a hole somewhere
            if vs:
                del vs[rng.randrange(len(vs))]
        elif kind < 0.4:         # several holes
            vs = [v for v in vs if rng.random() < 0.8]
        elif kind < 0.5:         # run starts above e0
            vs = [v for v in vs if v >= int(e0[a]) + 1]
        elif kind < 0.55:        # no file at all
            vs = []
        if rng.random() < 0.1 and vs:   # a duplicate (same address twice)
            vs.append(rng.choice(vs))
        vs.sort()
        fa += [a] * len(vs)
        fv += vs
    return e0, np.array(fa, np.uint32), np.array(fv, np.uint64)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_stats_windows_equal_reference_loop(world):
    """The fast path's windows == the reference loop's (ce_shard_window_exact), for every rank
    count, on 40 random batches each; a rank holding another rank's file flags the contract."""
    rng = random.Random(world)
    for trial in range(40):
        m = rng.randint(1, 24)
        writers = [rng.randbytes(16) for _ in range(m)]
        e0, fa, fv = _random_batch(rng, m, world)
        own = crdtenc.shard_owners(writers, fa, fv, world) if len(fa) else np.zeros(0, np.uint32)
        stats = [crdtenc.shard_stats_host(writers, e0, fa[own == r], fv[own == r], r, world) for r in range(world)]
        hi, flags = crdtenc.shard_window_host(e0, _reduce_max(stats))
        want_hi, want_flags = crdtenc.shard_window_exact(e0, fa, fv)
        assert flags & (shard.SHARD_BAD | shard.SHARD_E0_MISMATCH) == 0, (trial, flags)
        assert (hi == want_hi).all() and flags == want_flags, (trial, hi, want_hi, flags, want_flags)
    # contract breaks: a file on the wrong rank; a writer's files out of order; e0 not replicated
    writers = [rng.randbytes(16) for _ in range(4)]
    fa = np.repeat(np.arange(4, dtype=np.uint32), 10)
    fv = np.tile(np.arange(10, dtype=np.uint64), 4)
    e0 = np.zeros(4, np.uint64)
    if world > 1:
        own = crdtenc.shard_owners(writers, fa, fv, world)
        moved = own.copy()
        moved[7] = (moved[7] + 1) % world
        stats = [crdtenc.shard_stats_host(writers, e0, fa[moved == r], fv[moved == r], r, world) for r in range(world)]
        assert crdtenc.shard_window_host(e0, _reduce_max(stats))[1] & shard.SHARD_BAD
        e1 = e0.copy()
        e1[2] = 3
        stats = [crdtenc.shard_stats_host(writers, e1 if r == 1 else e0, fa[own == r], fv[own == r], r, world)
                 for r in range(world)]
        assert crdtenc.shard_window_host(e0, _reduce_max(stats))[1] & shard.SHARD_E0_MISMATCH
    st = crdtenc.shard_stats_host(writers, e0, fa[::-1].copy(), fv[::-1].copy(), 0, 1)
    assert crdtenc.shard_window_host(e0, st)[1] & shard.SHARD_BAD


def test_window_exact_is_the_reference_loop():
    """ce_shard_window_exact against a direct restatement of lib.rs:516-544 in Python."""
    rng = random.Random(11)
    for _ in range(200):
        m = rng.randint(1, 6)
        e0, fa, fv = _random_batch(rng, m, 1)
        order = sorted(range(len(fa)), key=lambda i: (fa[i], fv[i]))
        exp = [int(x) for x in e0]
        stop, gap = m, False
        for i in order:
            a, v = int(fa[i]), int(fv[i])
            if v < exp[a]:
                continue
            if v > exp[a]:
                stop, gap = a, True
                break
            exp[a] = v + 1
        want = [int(e0[a]) if a > stop else exp[a] for a in range(m)]
        hi, flags = crdtenc.shard_window_exact(e0, fa, fv)
        assert list(hi) == want and bool(flags & shard.SHARD_GAP) == gap


# ---- world-2 gloo runs of shard.ingest_sharded ----------------------------------------------

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scenario(name, seed=9, m=6, versions=9):
    """(key, writers, registered, files, fa, fv, pre): files sealed with the oracle, in
    (writer, version) order; pre = how many leading versions of each writer both the ranks and
    the oracle fold first (the replicated starting state)."""
    import oracle
    rng = random.Random(seed)
    key = rng.randbytes(32)
    writers = sorted(rng.randbytes(16) for _ in range(m))
    stranger = rng.randbytes(16)
    files, fa, fv = [], [], []
    for a in range(m):
        for v in range(versions):
            if name == "gap" and a == 2 and v == 4:
                continue
            dots = [{"actor": writers[a] if rng.random() < 0.7 else rng.choice(writers),
                     "counter": max(1, rng.getrandbits(rng.choice([8, 20, 40, 64])))}
                    for _ in range(rng.randint(1, 8))]
            if name == "unregistered" and a == 4 and v == 6:
                dots.append({"actor": stranger, "counter": 12345})
            if name == "grow" and a == 4 and v == 6:
                # more new actors than the initial table holds (1/4 of 8192 slots): the ingest grows
                # the actor table past the dense buffer the exchange was sized with
                dots += [{"actor": rng.randbytes(16), "counter": rng.randint(1, 1 << 30)} for _ in range(2100)]
            st, enc = oracle.cryptor_encrypt(key, rng.randbytes(24), APP + msgpack.packb(dots, use_bin_type=True))
            assert st == 0
            if name == "tamper" and a == 3 and v == 5:
                enc = enc[:-1] + bytes([enc[-1] ^ 1])
            files.append(crdtenc.CORE_VERSION + enc)
            fa.append(a)
            fv.append(v)
    pre = {a: (3 if name == "old_versions" and a % 2 == 0 else 0) for a in range(m)}
    return key, writers, list(writers), files, fa, fv, pre


def _oracle_fold(key, writers, files, fa, fv, pre):
    import oracle
    oc = oracle.Core(oracle.STATE_GCOUNTER)
    first = [i for i in range(len(files)) if fv[i] < pre[fa[i]]]
    if first:
        assert oc.read_remote_ops(key, [APP], [files[i] for i in first], [writers[fa[i]] for i in first],
                                  [fv[i] for i in first])[0] == 0
    rc, _ = oc.read_remote_ops(key, [APP], files, [writers[x] for x in fa], fv)   # (writer, version) order
    return rc, oc.serialize()


def _rank_main(rank, world, port, name, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shard_twin import HostShardOps, TwinCore
        key, writers, registered, files, fa, fv, pre = _scenario(name)
        own = crdtenc.shard_owners(writers, fa, fv, world)
        if name == "contract":         # one file handed to the other rank
            own[11] = (own[11] + 1) % world
        core = TwinCore()
        pre = _rank_pre(name, pre, rank)
        if any(pre.values()):          # the starting state (replicated, except for e0_mismatch)
            _, ser = _oracle_fold(key, writers, [files[i] for i in range(len(files)) if fv[i] < pre[fa[i]]],
                                  [fa[i] for i in range(len(files)) if fv[i] < pre[fa[i]]],
                                  [fv[i] for i in range(len(files)) if fv[i] < pre[fa[i]]], {a: 0 for a in pre})
            core.fold_bytes(ser)
        start = core.state_bytes()
        sel = [i for i in range(len(files)) if own[i] == rank]
        split = sorted(set(fa[i] for i in sel))
        ops = HostShardOps(core, key, writers, registered, [files[i] for i in sel], [fa[i] for i in sel],
                           [fv[i] for i in sel])
        rc, path = shard.ingest_sharded(ops)
        with open("%s.%d" % (out_path, rank), "wb") as f:
            f.write(msgpack.packb([rc, path, len(sel), split, core.state_bytes(), start], use_bin_type=True))
    finally:
        dist.destroy_process_group()


def _rank_pre(name, pre, rank):
    """Versions of each writer folded before the sharded ingest on `rank`: the scenario's
    replicated start, except e0_mismatch, where rank 1 alone has also folded writer 1's version 0
    (the ranks start from different next_op_versions)."""
    if name == "e0_mismatch" and rank == 1:
        return {**pre, 1: 1}
    return pre


def _expected(name, key, writers, files, fa, fv, pre):
    """(rc, state) every rank must end with; None for the state when it is the rank's own start."""
    orc, want = _oracle_fold(key, writers, files, fa, fv, pre)
    if name == "tamper":   # the reference panics (lib.rs:502): nothing folded, the state unchanged
        first = [i for i in range(len(files)) if fv[i] < pre[fa[i]]]
        return 9, _oracle_fold(key, writers, [files[i] for i in first], [fa[i] for i in first],
                               [fv[i] for i in first], {a: 0 for a in pre})[1]
    if name == "e0_mismatch":  # refused before any fold: each rank keeps its own start
        return shard.ERR_SHARD, None
    return orc, want


@pytest.mark.parametrize("name,want_rc,want_path", [
    ("clean", 0, "dense"),
    ("old_versions", 0, "dense"),
    ("gap", 13, "dense"),
    ("tamper", 9, "rejected"),
    ("contract", 0, "dense+exact"),
    ("unregistered", 0, "bytes"),
    ("grow", 0, "bytes"),
    ("e0_mismatch", 69, "refused"),
])
def test_two_rank_sharded_ingest_equals_single_fold(tmp_path, name, want_rc, want_path):
    key, writers, _, files, fa, fv, pre = _scenario(name)
    orc, want = _expected(name, key, writers, files, fa, fv, pre)
    assert orc == want_rc
    out = str(tmp_path / "r")
    mp.spawn(_rank_main, args=(2, _free_port(), name, out), nprocs=2, join=True)
    starts = set()
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            rc, path, n, split, state, start = msgpack.unpackb(f.read(), raw=False)
        assert (rc, path) == (want_rc, want_path), (r, rc, path)
        assert 0 < n < len(files) and len(split) == len(writers)   # every writer split across ranks
        assert state == (start if want is None else want), r
        starts.add(start)
    if name == "e0_mismatch":
        assert len(starts) == 2
