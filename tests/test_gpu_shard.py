"""The address-partitioned VClock / GCounter ingest on the GPU (ce_shard.hip, ce_shard_host.cpp,
shard.ingest_sharded):

  * the device gate kernels == the host twins (ShardStats of every rank's share, the windows of
    the reduced stats) on randomized batches with holes, old versions and duplicates;
  * the whole protocol for three ranks inside one process through the C ABI (the collectives
    done by numpy max): the GPU fold of each share, pending until the reduced batch is committed,
    every core's state == the oracle's single fold over all files in (writer, version) order;
  * two processes (gloo, one GPU) running shard.ingest_sharded on the scenarios of
    tests/test_shard.py: a writer split across ranks, a gap, skipped old versions, a tampered
    file (every rank unchanged), a contract break (exact windows), an unregistered Dot actor.
"""
import os
import random
import socket
import subprocess
import sys

import msgpack
import numpy as np
import pytest
import torch

import crdtenc
import shard

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_shard import _random_batch, _scenario, _oracle_fold, _expected  # noqa: E402

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")


@pytest.fixture(scope="module")
def ctx():
    c = crdtenc.Context(0)
    yield c
    c.close()


def _core(ctx, e0=None, writers=None, key=None):
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(key or bytes(32))
    if e0 is not None and any(int(x) for x in e0):   # next_op_versions = e0 (a merged state)
        sw = {"next_op_versions": {"dots": dict(sorted((writers[a], int(e0[a])) for a in range(len(writers)) if e0[a]))},
              "state": {"inner": {"dots": {}}}}
        assert core.merge_state(msgpack.packb(sw, use_bin_type=True)) == 0
    return core


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_device_stats_and_window_equal_host(ctx, world):
    rng = random.Random(100 + world)
    dev = torch.device("cuda", 0)
    for trial in range(12):
        m = rng.randint(1, 40)
        writers = [rng.randbytes(16) for _ in range(m)]
        e0, fa, fv = _random_batch(rng, m, world)
        core = _core(ctx, e0, writers)
        assert list(core.writer_versions(b"".join(writers))) == [int(x) for x in e0]
        own = crdtenc.shard_owners(writers, fa, fv, world) if len(fa) else np.zeros(0, np.uint32)
        dstats = []
        for r in range(world):
            sel = own == r
            d_fa = torch.from_numpy(fa[sel].astype(np.int32)).to(dev)
            d_fv = torch.from_numpy(fv[sel].astype(np.int64)).to(dev)
            st = torch.empty(2 * m + 3, dtype=torch.int64, device=dev)
            core.shard_stats(b"".join(writers), d_fa.data_ptr(), d_fv.data_ptr(), int(sel.sum()), r, world,
                             st.data_ptr())
            want = crdtenc.shard_stats_host(writers, e0, fa[sel], fv[sel], r, world)
            got = st.cpu().numpy()
            assert (got == want).all(), (trial, r)
            dstats.append(got)
        red = torch.from_numpy(np.maximum.reduce(dstats)).to(dev)
        torch.cuda.synchronize()
        hi = torch.empty(m + 1, dtype=torch.int64, device=dev)
        core.shard_window(b"".join(writers), red.data_ptr(), hi.data_ptr())
        ctx.synchronize()
        h, flags = crdtenc.shard_window_host(e0, red.cpu().numpy())
        got = hi.cpu().numpy().view(np.uint64)
        assert (got[:m] == h).all() and int(got[m]) == flags
        assert (h == crdtenc.shard_window_exact(e0, fa, fv)[0]).all()
        core.close()


@pytest.mark.parametrize("name,want_rc", [("clean", 0), ("gap", 13), ("old_versions", 0), ("tamper", 9),
                                          ("unregistered", 0)])
def test_three_shares_one_process(ctx, oracle, name, want_rc):
    """Three cores on one GPU play three ranks (collectives = numpy max): stats -> max ->
    windows -> sharded ingest (pending) -> dense max -> commit; == the oracle's single fold."""
    key, writers, registered, files, fa, fv, pre = _scenario(name)
    world = 3
    own = crdtenc.shard_owners(writers, fa, fv, world)
    dev = torch.device("cuda", 0)
    W = b"".join(writers)
    cores, shares = [], []
    first = [i for i in range(len(files)) if fv[i] < pre[fa[i]]]
    for r in range(world):
        core = _core(ctx, key=key)
        core.register_actors(registered)
        if first:
            rc, _ = core.ingest_ops([files[i] for i in first], writers, [fa[i] for i in first], [fv[i] for i in first])
            assert rc == 0
        sel = [i for i in range(len(files)) if own[i] == r]
        blob = b"".join(files[i] for i in sel)
        offs = np.zeros(len(sel) + 1, np.int64)
        offs[1:] = np.cumsum([len(files[i]) for i in sel])
        d = dict(files=torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to(dev),
                 offs=torch.from_numpy(offs).to(dev), n=len(sel), blob_len=len(blob),
                 fa=torch.tensor([fa[i] for i in sel], dtype=torch.int32, device=dev),
                 fv=torch.tensor([fv[i] for i in sel], dtype=torch.int64, device=dev))
        cores.append(core)
        shares.append(d)
    m = len(writers)
    stats = []
    for r, (core, d) in enumerate(zip(cores, shares)):
        st = torch.empty(2 * m + 3, dtype=torch.int64, device=dev)
        core.shard_stats(W, d["fa"].data_ptr(), d["fv"].data_ptr(), d["n"], r, world, st.data_ptr())
        stats.append(st.cpu().numpy())
    red = torch.from_numpy(np.maximum.reduce(stats)).to(dev)
    torch.cuda.synchronize()
    rcs, batches, ready = [], [], []
    for core, d in zip(cores, shares):
        hi = torch.empty(m + 1, dtype=torch.int64, device=dev)
        core.shard_window(W, red.data_ptr(), hi.data_ptr())
        rc = core.ingest_ops_device_sharded(d["files"].data_ptr(), d["offs"].data_ptr(), d["n"], d["blob_len"],
                                            W, d["fa"].data_ptr(), d["fv"].data_ptr(), hi.data_ptr())
        rcs.append(rc)
        b = torch.zeros(core.dense_capacity(), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()   # the core's own stream reads / writes it next
        if rc in (0, 13):
            ready.append(core.pending_export(b.data_ptr(), b.numel()))
        batches.append(b.cpu().numpy().view(np.uint64))
    failed = [rc for rc in rcs if rc not in (0, 13)]
    if failed:
        assert failed == [want_rc]
        for core, rc in zip(cores, rcs):
            if rc in (0, 13):
                core.pending_commit(False)
        want = _oracle_fold(key, writers, [files[i] for i in first], [fa[i] for i in first],
                            [fv[i] for i in first], {a: 0 for a in pre})[1]
    else:
        assert set(rcs) == {want_rc}
        orc, want = _oracle_fold(key, writers, files, fa, fv, pre)
        assert orc == want_rc
        if all(ready):
            red_b = torch.from_numpy(np.maximum.reduce(batches).view(np.int64).copy()).to(dev)
            torch.cuda.synchronize()
            for core in cores:
                core.pending_commit(True, red_b.data_ptr(), red_b.numel())
        else:   # a Dot on an unregistered actor: commit locally, then merge serialized states
            assert name == "unregistered"
            for core in cores:
                core.pending_commit(True)
            parts = [c.state_bytes() for c in cores]
            for r, core in enumerate(cores):
                for q, p in enumerate(parts):
                    if q != r:
                        assert core.merge_state(p) == 0
    for core in cores:
        assert core.state_bytes() == want
        core.close()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name,want_rc,want_path", [
    ("clean", 0, "dense"), ("gap", 13, "dense"), ("old_versions", 0, "dense"),
    ("tamper", 9, "rejected"), ("contract", 0, "dense+exact"), ("unregistered", 0, "bytes"),
    ("grow", 0, "bytes"), ("e0_mismatch", 69, "refused"),
])
def test_two_process_sharded_ingest(tmp_path, name, want_rc, want_path):
    """'grow': one rank's Dots name 2100 new actors, so its ingest grows the actor table past the
    dense buffer sized before it -- the export must decline (no write past the buffer) and every
    rank take the state all-gather; 'e0_mismatch': the ranks start from different
    next_op_versions -- refused on every rank, each state unchanged."""
    key, writers, _, files, fa, fv, pre = _scenario(name)
    want_rc2, want = _expected(name, key, writers, files, fa, fv, pre)
    assert want_rc2 == want_rc
    out = str(tmp_path / "s")
    port = str(_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"),
                               str(r), "2", port, "sharded:" + name, out]) for r in range(2)]
    rcs = [p.wait(timeout=180) for p in procs]
    assert rcs == [0, 0]
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            rc, path, n, state, start = msgpack.unpackb(f.read(), raw=False)
        assert (rc, path) == (want_rc, want_path), r
        assert 0 < n < len(files)
        assert state == (start if want is None else want), r
