"""GPU parity on scaled-down versions of BASELINE.json's configs C4 (skewed file sizes) and C5
(key-rotation mix with tampered tags), against the C oracle.

C5 semantics: the reference decrypts every file with Keys::latest_key only
(crdt-enc/src/lib.rs:484-490), so files sealed under the other data key fail authentication like
tampered ones; any failure rejects the whole batch before the fold (lib.rs:497-514).  Parity =
identical per-file statuses and an unchanged state.
"""
import math
import random

import msgpack
import numpy as np
import pytest
import torch

import crdtenc

pytestmark = pytest.mark.gpu
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = crdtenc.CORE_VERSION


@pytest.fixture(scope="module")
def ctx():
    c = crdtenc.Context(0)
    yield c
    c.close()


def _dots_clear(rng, actors, a, target):
    """Vec<Dot> plaintext of about `target` bytes, mostly the writer's own dots"""
    n = max(1, (target - 16) // 30)
    dots = [{"actor": actors[a] if rng.random() < 0.8 else rng.choice(actors),
             "counter": rng.getrandbits(rng.choice([7, 20, 40]))} for _ in range(n)]
    return APP + msgpack.packb(dots, use_bin_type=True)


def _core(ctx, key, kind=crdtenc.STATE_GCOUNTER):
    core = crdtenc.Core(ctx, kind=kind, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    return core


def test_c4_skewed_sizes_log_uniform(ctx, oracle):
    """C4: plaintexts log-uniform on [256 B, 1 MiB], 8 writers, host and device entry points"""
    rng = random.Random(404)
    key = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(8))
    clears, fa, fv = [], [], []
    for a in range(8):
        for v in range(12):
            size = int(math.exp(rng.uniform(math.log(256), math.log(1 << 20))))
            clears.append(_dots_clear(rng, actors, a, size))
            fa.append(a)
            fv.append(v)
    files = [CORE + e for e in ctx.encrypt_batch(key, clears)]
    oc = oracle.Core()
    orc, ost = oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)
    assert orc == 0
    core = _core(ctx, key)
    rc, st = core.ingest_ops(files, actors, fa, fv)
    assert (rc, st) == (orc, ost)
    assert core.state_bytes() == oc.serialize()
    # device-resident entry point over the same batch
    blob = b"".join(files)
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(f) for f in files])
    d_blob = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_fa = torch.tensor(fa, dtype=torch.int32).cuda()
    d_fv = torch.tensor(fv, dtype=torch.int64).cuda()
    torch.cuda.synchronize()
    core2 = _core(ctx, key)
    rc2, st2 = core2.ingest_ops_device(d_blob.data_ptr(), d_offs.data_ptr(), len(files), len(blob),
                                       b"".join(actors), d_fa.data_ptr(), d_fv.data_ptr(),
                                       want_status=True)
    assert rc2 == 0 and st2 == ost
    assert core2.state_bytes() == oc.serialize()
    core.close()
    core2.close()


@pytest.mark.parametrize("tamper", [0, 3], ids=["rotation", "rotation+tamper"])
def test_c5_key_rotation_mix(ctx, oracle, tamper):
    """C5: half the files under the other data key (+ a few flipped tag bits): every reject
    status matches the reference's latest-key-only decrypt and nothing is folded"""
    rng = random.Random(505 + tamper)
    key0, key1 = rng.randbytes(32), rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(16))
    clears, fa, fv, which = [], [], [], []
    for a in range(16):
        for v in range(64):
            clears.append(_dots_clear(rng, actors, a, rng.choice([600, 4000, 9000])))
            fa.append(a)
            fv.append(v)
            which.append(rng.random() < 0.5)
    sealed0 = ctx.encrypt_batch(key0, clears)
    sealed1 = ctx.encrypt_batch(key1, clears)
    files = [CORE + (s1 if w else s0) for s0, s1, w in zip(sealed0, sealed1, which)]
    tampered = set(rng.sample(range(len(files)), tamper))
    for i in tampered:
        b = bytearray(files[i])
        b[-1 - rng.randrange(16)] ^= 1 << rng.randrange(8)
        files[i] = bytes(b)
    for latest in (key0, key1):
        oc = oracle.Core()
        empty = oc.serialize()
        orc, ost = oc.read_remote_ops(latest, [APP], files, [actors[i] for i in fa], fv)
        core = _core(ctx, latest)
        rc, st = core.ingest_ops(files, actors, fa, fv)
        assert rc == orc == 9
        assert st == ost
        assert core.state_bytes() == oc.serialize() == empty
        core.close()
    # the files of the latest key alone fold (and match the oracle)
    keep = [i for i in range(len(files)) if not which[i] and i not in tampered]
    sel = lambda xs: [xs[i] for i in keep]
    # keep each actor's versions contiguous from 0: re-number them
    nv, seen = [], {}
    for i in keep:
        nv.append(seen.get(fa[i], 0))
        seen[fa[i]] = nv[-1] + 1
    files0 = [CORE + sealed0[i] for i in keep]
    oc = oracle.Core()
    orc, ost = oc.read_remote_ops(key0, [APP], files0, [actors[i] for i in sel(fa)], nv)
    core = _core(ctx, key0)
    rc, st = core.ingest_ops(files0, actors, sel(fa), nv)
    assert (rc, st) == (orc, ost) and rc == 0
    assert core.state_bytes() == oc.serialize()
    core.close()


@pytest.mark.parametrize("tamper", [0, 2])
def test_multi_key_opt_in(ctx, oracle, tamper):
    """Keys with a rotated data key (ce_keys from the wire form, latest = Keys::latest_key).
    Default (reference): files under the older key fail like tampered ones, the batch
    is rejected and nothing folds.  CE_OPEN_MULTI_KEY: those files open under the older key (in
    id order), so the batch folds to the state of all plaintexts; a tampered file still fails
    under every key and rejects the batch.  Files of the older key also carry Dots on actors the
    table has never seen (the retry path's miss resolution)."""
    from oracle import keys as K
    rng = random.Random(911 + tamper)
    writer = rng.randbytes(16)
    ks = K.Keys()
    old_id, new_id = rng.randbytes(16), rng.randbytes(16)
    k_old, k_new = rng.randbytes(32), rng.randbytes(32)
    ks.insert_latest_key(writer, old_id, k_old)
    ks.insert_latest_key(writer, new_id, k_new)
    keys = crdtenc.Keys.decode(ks.to_bytes())
    assert keys.latest()[2] == k_new and len(keys) == 2
    actors = sorted(rng.randbytes(16) for _ in range(12))
    strangers = [rng.randbytes(16) for _ in range(5)]
    clears, fa, fv, old = [], [], [], []
    for a in range(12):
        for v in range(24):
            o = rng.random() < 0.5
            c = _dots_clear(rng, actors, a, rng.choice([600, 4000, 9000]))
            if o and rng.random() < 0.3:
                dots = msgpack.unpackb(c[16:])
                dots.append({"actor": rng.choice(strangers), "counter": rng.getrandbits(30)})
                c = APP + msgpack.packb(dots, use_bin_type=True)
            clears.append(c)
            fa.append(a)
            fv.append(v)
            old.append(o)
    s_old, s_new = ctx.encrypt_batch(k_old, clears), ctx.encrypt_batch(k_new, clears)
    files = [CORE + (so if o else sn) for so, sn, o in zip(s_old, s_new, old)]
    tampered = set(rng.sample(range(len(files)), tamper))
    for i in tampered:
        b = bytearray(files[i])
        b[-1 - rng.randrange(16)] ^= 1 << rng.randrange(8)
        files[i] = bytes(b)
    # reference behaviour (flag off): latest key only
    oc = oracle.Core()
    empty = oc.serialize()
    orc, ost = oc.read_remote_ops(k_new, [APP], files, [actors[i] for i in fa], fv)
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_keys(keys)
    rc, st = core.ingest_ops(files, actors, fa, fv)
    assert rc == orc == 9 and st == ost
    assert core.state_bytes() == empty
    core.close()
    # opt-in
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP,
                        flags=crdtenc.OPEN_MULTI_KEY)
    core.set_keys(keys)
    rc, st = core.ingest_ops(files, actors, fa, fv)
    if tamper:
        assert rc == 9 and sorted(i for i, s in enumerate(st) if s) == sorted(tampered)
        assert core.state_bytes() == empty
    else:
        assert rc == 0 and all(s == 0 for s in st)
        ref = oracle.Core()
        assert ref.read_remote_ops(k_new, [APP], [CORE + s for s in s_new],
                                   [actors[i] for i in fa], fv)[0] == 0
        assert core.state_bytes() == ref.serialize()
    core.close()


def test_c3_read_context_removals(ctx):
    """C3 with SURVEY.md §8d's removal shape (bench config c3r): every Rm carries the removed
    member's read context -- the state files' adds of it and the writer's own (crdts'
    rm(member, read_ctx)), so op files pass the 2 KiB fused-decode region and removals name
    other writers' dots.  At a small size, through bench_configs' own runner: the closed-form
    clock, the writer-sharded fold + merge_state == the whole fold, and the C restatement's state
    bytes over the same files == the GPU's (crdt-enc/src/lib.rs:457-465, 533-535)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench_configs as B
    ns = B.make_parser().parse_args(["--config", "c3r", "--steps", "2", "--warmup", "1", "--versions", "2",
                                     "--state-versions", "1"])
    line = B.RUNNERS["c3r"](ns, ctx, torch.device("cuda", 0))
    assert line["config"]["rm_ctx"] == "read"
    assert line["config"]["removal_clock_entries"] > 2 * 4096 * 2 * B.N_RM   # multi-entry clocks
    assert all(line["checks"].values()), line["checks"]
    assert line["cpu_baseline"]["same_result_as_gpu"], line["cpu_baseline"]
