"""N>1 path on CPU: world_size-2 gloo ranks, files sharded by writer actor (shard.actor_range),
partial StateWrapper<GCounter|VClock> folded per rank, exchanged once with
shard.merge_dense (all_reduce MAX over u64 with the sign flip), and the merged state must
serialize to the bytes of a single-process fold over all files (crdt-enc/src/lib.rs:471-547,
739-743).  The per-rank fold here is the oracle (no GPU in this container); on the GPU box the
same exchange runs over Core.export_dense / import_dense (test_gpu_parity)."""
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
for p in (os.path.join(REPO, "crdt-enc_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import shard  # noqa: E402

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = bytes.fromhex("e834d789101b463498239de990a9051f")


def _workload(seed=5, n_actors=6, versions=5):
    import oracle
    rng = random.Random(seed)
    key = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(n_actors))
    files, fa, fv = [], [], []
    for a in range(n_actors):
        for v in range(versions):
            dots = []
            for _ in range(rng.randint(1, 12)):
                big = rng.random() < 0.15
                ctr = rng.getrandbits(64) | (1 << 63) if big else rng.getrandbits(rng.choice([5, 14, 30]))
                dots.append({"actor": actors[a] if rng.random() < 0.7 else rng.choice(actors),
                             "counter": max(ctr, 1)})
            clear = APP + msgpack.packb(dots, use_bin_type=True)
            st, enc = oracle.cryptor_encrypt(key, rng.randbytes(24), clear)
            assert st == 0
            files.append(CORE + enc)
            fa.append(a)
            fv.append(v)
    return key, actors, files, fa, fv


def _fold(kind, key, actors, files, fa, fv):
    import oracle
    oc = oracle.Core(kind)
    rc, _ = oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)
    assert rc == 0
    return oc.serialize()


def _dense(kind, ser, actors):
    import oracle
    d = msgpack.unpackb(ser, raw=True, strict_map_key=False)
    nov = d[b"next_op_versions"][b"dots"]
    st = d[b"state"][b"inner"][b"dots"] if kind == oracle.STATE_GCOUNTER else d[b"state"][b"dots"]
    idx = {a: i for i, a in enumerate(actors)}
    s = np.zeros(len(actors), dtype=np.uint64)
    n = np.zeros(len(actors), dtype=np.uint64)
    for a, c in st.items():
        s[idx[a]] = c
    for a, c in nov.items():
        n[idx[a]] = c
    return torch.from_numpy(s.view(np.int64).copy()), torch.from_numpy(n.view(np.int64).copy())


def _serialize_dense(kind, actors, s, n):
    import oracle
    su, nu = s.numpy().view(np.uint64), n.numpy().view(np.uint64)
    nov = {a: int(nu[i]) for i, a in enumerate(actors) if nu[i]}
    st = {a: int(su[i]) for i, a in enumerate(actors) if su[i]}
    state = {"inner": {"dots": st}} if kind == oracle.STATE_GCOUNTER else {"dots": st}
    return msgpack.packb({"next_op_versions": {"dots": nov}, "state": state}, use_bin_type=True)


def _rank_main(rank, world, port, kind, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, actors, files, fa, fv = _workload()
        lo, hi = shard.actor_range(len(actors), world, rank)
        sel = [i for i in range(len(files)) if lo <= fa[i] < hi]
        ser = _fold(kind, key, actors, [files[i] for i in sel], [fa[i] for i in sel], [fv[i] for i in sel])
        s, n = _dense(kind, ser, actors)
        shard.merge_dense(s, n)
        if rank == 0:
            with open(out_path, "wb") as f:
                f.write(_serialize_dense(kind, actors, s, n))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_actor_range_partitions():
    for n in (1, 5, 4096):
        for w in (1, 2, 3, 8):
            ranges = [shard.actor_range(n, w, r) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))
            for a in range(n):
                r = shard.file_rank(a, n, w)
                assert ranges[r][0] <= a < ranges[r][1]


def test_merge_dense_is_u64_max():
    # single-rank gloo group: the flip must leave values intact and order u64 correctly
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        v = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1], dtype=np.uint64)
        t = torch.from_numpy(v.view(np.int64).copy())
        shard.merge_dense(t)
        assert (t.numpy().view(np.uint64) == v).all()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", [0, 1], ids=["vclock", "gcounter"])
def test_two_rank_exchange_equals_single_fold(kind, tmp_path):
    key, actors, files, fa, fv = _workload()
    want = _fold(kind, key, actors, files, fa, fv)
    out = str(tmp_path / "merged.bin")
    mp.spawn(_rank_main, args=(2, _free_port(), kind, out), nprocs=2, join=True)
    with open(out, "rb") as f:
        got = f.read()
    assert got == want


class _OracleDotCore:
    """state_bytes / merge_state over the sequential oracle (oracle/crdts.py)"""

    def __init__(self, kind):
        from oracle import crdts as C
        self.C = C
        self.core = C.Core(kind)

    def state_bytes(self):
        return self.core.serialize()

    def merge_state(self, sw):
        nov, st = self.C.dec_state(self.core.kind, sw)
        self.core.state.merge(st)
        self.core.nov.merge(nov)
        return 0

    def reset(self):
        self.core = self.C.Core(self.core.kind)


def _dot_workload(kind):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import dotset_gen as G
    rng = random.Random(21)
    actors = G.actors_for(rng, 6)
    if kind == "orswot":
        files = G.well_formed_orswot(rng, actors, 4, 5, 25)[0]
    else:
        files = G.well_formed_mvreg(rng, actors, 4, 3)
    return G.batch(files, kind, APP)


def _dot_fold(kind, actors, clears, fa, fv, sel):
    import oracle
    key = bytes(range(32))
    core = _OracleDotCore(kind)
    files = [CORE + oracle.cryptor_encrypt(key, bytes(24), clears[i])[1] for i in sel]
    rc, _ = core.core.read_remote_ops(key, [APP], files, [actors[fa[i]] for i in sel], [fv[i] for i in sel])
    assert rc == 0
    return core


def _dot_rank_main(rank, world, port, kind, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        actors, clears, fa, fv = _dot_workload(kind)
        lo, hi = shard.actor_range(len(actors), world, rank)
        core = _dot_fold(kind, actors, clears, fa, fv, [i for i in range(len(fa)) if lo <= fa[i] < hi])
        shard.exchange_dotset(core)
        with open("%s.%d" % (out_path, rank), "wb") as f:
            f.write(core.state_bytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
def test_two_rank_dotset_exchange_equals_single_fold(kind, tmp_path):
    actors, clears, fa, fv = _dot_workload(kind)
    want = _dot_fold(kind, actors, clears, fa, fv, range(len(fa))).state_bytes()
    out = str(tmp_path / "merged")
    mp.spawn(_dot_rank_main, args=(2, _free_port(), kind, out), nprocs=2, join=True)
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            assert f.read() == want


class _DenseCore:
    """Host stand-in for crdtenc.Core's exchange surface (dense_ready, export/import_dense,
    state_bytes, merge_state) over the product's StateWrapper<GCounter> bytes: registered actors
    own dense slots in registration order; a Dot on any other actor makes dense_ready() False."""

    def __init__(self, kind, registered):
        self.kind, self.reg = kind, list(registered)
        self.slot = {a: i for i, a in enumerate(self.reg)}
        self.state, self.nov = {}, {}

    def fold(self, ser):
        import msgpack
        d = msgpack.unpackb(ser, raw=True, strict_map_key=False)
        nov = d[b"next_op_versions"][b"dots"]
        st = d[b"state"][b"inner"][b"dots"] if self.kind == 1 else d[b"state"][b"dots"]
        for a, c in st.items():
            self.state[a] = max(self.state.get(a, 0), c)
        for a, c in nov.items():
            self.nov[a] = max(self.nov.get(a, 0), c)

    def dense_ready(self):
        return all(a in self.slot for a in list(self.state) + list(self.nov))

    def export_dense(self, p_state, p_nov):
        self._dense[: len(self.reg)] = torch.from_numpy(np.array(
            [self.state.get(a, 0) for a in self.reg], dtype=np.uint64).view(np.int64))
        cap = self._dense.numel() // 2
        self._dense[cap: cap + len(self.reg)] = torch.from_numpy(np.array(
            [self.nov.get(a, 0) for a in self.reg], dtype=np.uint64).view(np.int64))

    def import_dense(self, p_state, p_nov):
        cap = self._dense.numel() // 2
        s = self._dense[: len(self.reg)].numpy().view(np.uint64)
        n = self._dense[cap: cap + len(self.reg)].numpy().view(np.uint64)
        for i, a in enumerate(self.reg):
            if s[i]:
                self.state[a] = max(self.state.get(a, 0), int(s[i]))
            if n[i]:
                self.nov[a] = max(self.nov.get(a, 0), int(n[i]))

    def state_bytes(self):
        import msgpack
        st = dict(sorted(self.state.items()))
        body = {"inner": {"dots": st}} if self.kind == 1 else {"dots": st}
        return msgpack.packb({"next_op_versions": {"dots": dict(sorted(self.nov.items()))},
                              "state": body}, use_bin_type=True)

    def merge_state(self, sw):
        self.fold(sw)
        return 0


def _vclock_rank_main(rank, world, port, kind, n_reg, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, actors, files, fa, fv = _workload()
        lo, hi = shard.actor_range(len(actors), world, rank)
        sel = [i for i in range(len(files)) if lo <= fa[i] < hi]
        core = _DenseCore(kind, actors[:n_reg])
        core.fold(_fold(kind, key, actors, [files[i] for i in sel], [fa[i] for i in sel],
                        [fv[i] for i in sel]))
        core._dense = dense = torch.zeros(2 * 16, dtype=torch.int64)
        path = shard.exchange_vclock(core, dense)
        with open("%s.%d" % (out_path, rank), "wb") as f:
            f.write(path.encode() + b"\n" + core.state_bytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_reg,path", [(6, "dense"), (4, "bytes")], ids=["all_registered", "unregistered_actor"])
def test_exchange_vclock_paths(tmp_path, n_reg, path):
    """shard.exchange_vclock under a real world-2 gloo group: every actor registered -> one
    dense all_reduce(MAX); an actor outside the registered slots on either rank -> both ranks
    take the state all-gather + merge_state path.  Either way == the single fold."""
    kind = 1
    key, actors, files, fa, fv = _workload()
    want = _fold(kind, key, actors, files, fa, fv)
    out = str(tmp_path / "v")
    mp.spawn(_vclock_rank_main, args=(2, _free_port(), kind, n_reg, out), nprocs=2, join=True)
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            got_path, state = f.read().split(b"\n", 1)
        assert got_path.decode() == path
        assert state == want


def _c3_medium(tamper_rank=None, world=2):
    """test_c3_shaped_medium's generator (tests/test_gpu_dotset.py): 256 writers, members from
    10k, 4 versions x 12 ops per writer, sealed with the oracle; tamper_rank: one file of that
    rank's writer shard gets a flipped tag bit."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import dotset_gen as G
    import oracle
    rng = random.Random(3)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 256)
    files = G.well_formed_orswot(rng, actors, 4, 12, 10000, max_members=1)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = [CORE + oracle.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
    if tamper_rank is not None:
        lo, hi = shard.actor_range(len(acts), world, tamper_rank)
        i = next(i for i in range(len(fa)) if lo <= fa[i] < hi)
        sealed[i] = sealed[i][:-1] + bytes([sealed[i][-1] ^ 1])
    return key, acts, sealed, fa, fv


def _tree_rank_main(rank, world, port, tamper_rank, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key, acts, files, fa, fv = _c3_medium(tamper_rank, world)
        lo, hi = shard.actor_range(len(acts), world, rank)
        sel = [i for i in range(len(fa)) if lo <= fa[i] < hi]
        core = _OracleDotCore("orswot")

        def ingest():
            return core.core.read_remote_ops(key, [APP], [files[i] for i in sel], [acts[fa[i]] for i in sel],
                                             [fv[i] for i in sel])[0]

        rc, merges = shard.ingest_dotset_sharded(core, ingest)
        with open("%s.%d" % (out_path, rank), "wb") as f:
            f.write(msgpack.packb([rc, merges, core.state_bytes()], use_bin_type=True))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tamper", [(2, None), (4, None), (3, None), (4, 2)])
def test_dotset_tree_reduce_c3_medium(tmp_path, world, tamper):
    """shard.ingest_dotset_sharded at C3's shape (256 writers, 10k members, 1024 op files):
    writer shards folded per rank, then the binomial-tree reduce -- rank 0 ends with the oracle's
    single fold and runs ceil(log2 N) merges, no rank more; with a tampered file on one rank every
    rank returns AUTH with its state unchanged (lib.rs:497-514)."""
    from oracle import crdts as C
    key, acts, files, fa, fv = _c3_medium(tamper, world)
    oc = C.Core("orswot")
    orc = oc.read_remote_ops(key, [APP], files, [acts[i] for i in fa], fv)[0]
    out = str(tmp_path / "t")
    mp.spawn(_tree_rank_main, args=(world, _free_port(), tamper, out), nprocs=world, join=True)
    empty = C.Core("orswot").serialize()
    log = []
    for r in range(world):
        with open("%s.%d" % (out, r), "rb") as f:
            rc, merges, state = msgpack.unpackb(f.read(), raw=False)
        log.append(merges)
        if tamper is None:
            assert rc == 0 and orc == 0
            if r == 0:
                assert state == oc.serialize()
        else:
            assert rc == orc == 9 and state == empty and merges == 0
    if tamper is None:
        depth = (world - 1).bit_length()
        assert log[0] == depth and max(log) <= depth and sum(log) == world - 1, log
    print("merges per rank:", log)

