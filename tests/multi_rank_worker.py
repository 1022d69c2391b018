"""One rank of the multi-process product exchange tests (tests/test_gpu_multi.py): a real
torch.distributed group (gloo, every rank on GPU 0 of the box), the HIP ingest through the C ABI
on this rank's actor shard, then shard.exchange_vclock -- the dense all_reduce(MAX) when every
Dot names a registered actor, else the all-gather of serialized StateWrappers + merge_state.
Writes the merged StateWrapper bytes and the path taken to <out>.<rank>.

  python tests/multi_rank_worker.py RANK WORLD PORT MODE OUT
    MODE: registered | unregistered (GCounter, exchange_vclock) | orswot (Orswot<u64, Uuid>,
    shard.exchange_dotset: the all-gather of partial StateWrappers + the GPU Orswot::merge) |
    sharded:<scenario> (GCounter partitioned by address, shard.ingest_sharded; scenarios of
    tests/test_shard.py)
"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "crdt-enc_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")


def workload(mode, seed=77, n_actors=6, versions=5):
    """Seeded op files (sealed with the oracle): writer actors `actors`; with mode
    'unregistered' some Dots name `strangers`, actors no rank registers."""
    import msgpack
    import oracle
    import crdtenc
    rng = random.Random(seed)
    key = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(n_actors))
    strangers = sorted(rng.randbytes(16) for _ in range(3))
    files, fa, fv = [], [], []
    for a in range(n_actors):
        for v in range(versions):
            dots = []
            for _ in range(rng.randint(1, 9)):
                r = rng.random()
                who = actors[a] if r < 0.6 else rng.choice(actors)
                if mode == "unregistered" and a % 3 == 2 and r > 0.85:
                    who = rng.choice(strangers)
                ctr = rng.getrandbits(64) | (1 << 63) if rng.random() < 0.2 else rng.getrandbits(20)
                dots.append({"actor": who, "counter": max(ctr, 1)})
            clear = APP + msgpack.packb(dots, use_bin_type=True)
            st, enc = oracle.cryptor_encrypt(key, rng.randbytes(24), clear)
            assert st == 0
            files.append(crdtenc.CORE_VERSION + enc)
            fa.append(a)
            fv.append(v)
    return key, actors, files, fa, fv


def workload_orswot(seed=88, n_actors=8, versions=4, p_rm=0.2):
    """Seeded well-formed Orswot op files (tests/dotset_gen.py), sealed with the oracle, in
    load_ops order: removals may name other writers' adds, so a rank's partial state carries
    deferred removals the exchange has to resolve."""
    import crdtenc
    import dotset_gen as G
    import oracle
    rng = random.Random(seed)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, n_actors)
    files = G.well_formed_orswot(rng, actors, versions, 6, 30, p_rm=p_rm)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = []
    for c in clears:
        st, enc = oracle.cryptor_encrypt(key, rng.randbytes(24), c)
        assert st == 0
        sealed.append(crdtenc.CORE_VERSION + enc)
    return key, acts, sealed, fa, fv


def main_orswot(rank, world, out, tree=False, p_rm=0.2, device="cpu"):
    import crdtenc
    import shard
    key, actors, files, fa, fv = workload_orswot(p_rm=p_rm)
    ctx = crdtenc.Context(0)
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    lo, hi = shard.actor_range(len(actors), world, rank)
    sel = [i for i in range(len(files)) if lo <= fa[i] < hi]

    def ingest():
        return core.ingest_ops([files[i] for i in sel], actors[lo:hi], [fa[i] - lo for i in sel],
                               [fv[i] for i in sel])[0]

    if tree:   # the binomial-tree reduce to rank 0 (shard.ingest_dotset_sharded)
        rc, merges = shard.ingest_dotset_sharded(core, ingest, device=device)
        assert rc == 0, rc
        tag = b"tree %d %d" % (merges, core.path_count("columns_merge"))
    else:
        rc = ingest()
        assert rc == 0, rc
        shard.exchange_dotset(core, device="cpu")
        tag = b"dotset"
    with open("%s.%d" % (out, rank), "wb") as f:
        f.write(tag + b"\n" + core.state_bytes())
    core.close()
    ctx.close()


def main_sharded(rank, world, name, out):
    """shard.ingest_sharded through the C ABI: this rank's share (by address) of the scenario's
    op files resident in HBM, the device gate kernels, the pending fold, the dense exchange."""
    import msgpack
    import numpy as np
    import torch
    import crdtenc
    import shard
    from test_shard import _scenario, _rank_pre
    key, writers, registered, files, fa, fv, pre = _scenario(name)
    pre = _rank_pre(name, pre, rank)
    own = crdtenc.shard_owners(writers, fa, fv, world)
    if name == "contract":
        own[11] = (own[11] + 1) % world
    ctx = crdtenc.Context(0)
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    core.register_actors(registered)
    first = [i for i in range(len(files)) if fv[i] < pre[fa[i]]]
    if first:  # the starting state (replicated, except for e0_mismatch)
        rc, _ = core.ingest_ops([files[i] for i in first], writers, [fa[i] for i in first], [fv[i] for i in first])
        assert rc == 0, rc
    start = core.state_bytes()
    sel = [i for i in range(len(files)) if own[i] == rank]
    blob = b"".join(files[i] for i in sel)
    offs = np.zeros(len(sel) + 1, np.int64)
    offs[1:] = np.cumsum([len(files[i]) for i in sel])
    dev = torch.device("cuda", 0)
    d_files = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    d_fa = torch.tensor([fa[i] for i in sel], dtype=torch.int32, device=dev)
    d_fv = torch.tensor([fv[i] for i in sel], dtype=torch.int64, device=dev)
    ops = shard.DeviceShardOps(core, b"".join(writers), d_files, d_offs, len(sel), len(blob), d_fa, d_fv)
    rc, path = shard.ingest_sharded(ops)
    with open("%s.%d" % (out, rank), "wb") as f:
        f.write(msgpack.packb([rc, path, len(sel), core.state_bytes(), start], use_bin_type=True))
    core.close()
    ctx.close()


def main():
    rank, world, port, mode, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    if mode.startswith("orswot") or mode.startswith("sharded:"):
        sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch
    import torch.distributed as dist
    import crdtenc
    import shard
    # CE_TEST_BACKEND=nccl: RCCL (one rank per device; the one-GPU box runs world 1), the
    # collectives on device tensors
    backend = os.environ.get("CE_TEST_BACKEND", "gloo")
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    cdev = "cuda:0" if backend == "nccl" else "cpu"
    try:
        if mode in ("orswot", "orswot_tree", "orswot_adds"):
            # orswot_adds: adds only, no deferred removal -- the column exchange
            main_orswot(rank, world, out, tree=mode != "orswot", p_rm=0.0 if mode == "orswot_adds" else 0.2,
                        device=cdev)
            return
        if mode.startswith("sharded:"):
            main_sharded(rank, world, mode.split(":", 1)[1], out)
            return
        key, actors, files, fa, fv = workload(mode)
        ctx = crdtenc.Context(0)
        core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
        core.set_latest_key(key)
        core.register_actors(actors)
        lo, hi = shard.actor_range(len(actors), world, rank)
        sel = [i for i in range(len(files)) if lo <= fa[i] < hi]
        rc, _ = core.ingest_ops([files[i] for i in sel], actors[lo:hi], [fa[i] - lo for i in sel],
                                [fv[i] for i in sel])
        assert rc == 0, rc
        dense = torch.zeros(2 * core.dense_capacity(), dtype=torch.int64, device="cuda")
        path = shard.exchange_vclock(core, dense)
        with open("%s.%d" % (out, rank), "wb") as f:
            f.write(path.encode() + b"\n" + core.state_bytes())
        core.close()
        ctx.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
