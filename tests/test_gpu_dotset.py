"""GPU parity of the dot-set kinds (Orswot<u64, Uuid>, MVReg<u64, Uuid>) through the C ABI,
against the sequential crdts restatement (oracle/crdts.py).

Compared bit-exactly: per-file statuses, return codes and the canonical serialized StateWrapper
(the reference's HashMap order is random; both sides sort).  Parity with crdts 7
itself is unpinned: the oracle restates its published source.
"""
import os
import random
import struct

import msgpack
import numpy as np
import pytest

import crdtenc
import dotset_gen as G
from oracle import crdts as C

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = crdtenc.CORE_VERSION
KIND = {"orswot": crdtenc.STATE_ORSWOT, "mvreg": crdtenc.STATE_MVREG}


@pytest.fixture(scope="module")
def ctx():
    c = crdtenc.Context(0)
    yield c
    c.close()


def seal_files(ctx, key, clears):
    return [CORE + e for e in ctx.encrypt_batch(key, clears)]


def new_core(ctx, kind, key):
    core = crdtenc.Core(ctx, kind=KIND[kind], supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    return core


def check_ops(ctx, kind, key, core, oc, actors, clears, fa, fv):
    files = seal_files(ctx, key, clears)
    rc, st = core.ingest_ops(files, actors, fa, fv)
    orc, ost = oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)
    assert (rc, st) == (orc, ost)
    assert core.state_bytes() == oc.serialize()
    return rc


def gen(kind, rng, actors, versions, ops, members, adversarial):
    if kind == "orswot":
        if adversarial:
            return G.adversarial_orswot(rng, actors, versions, ops, members)
        return G.well_formed_orswot(rng, actors, versions, ops, members)[0]
    if adversarial:
        return G.adversarial_mvreg(rng, actors, versions, ops)
    return G.well_formed_mvreg(rng, actors, versions, ops)


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
@pytest.mark.parametrize("seed", range(6))
def test_ops_parity(ctx, kind, seed):
    rng = random.Random(1000 + seed)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, rng.randint(2, 9))
    core, oc = new_core(ctx, kind, key), C.Core(kind)
    adversarial = seed % 2 == 1
    files = gen(kind, rng, actors, 6, rng.randint(1, 8), 40, adversarial)
    # two batches: versions 0..2 then 3..5 (state and deferred removals carried over)
    first = {a: [ops for ops in files[a][:3]] for a in files}
    acts, clears, fa, fv = G.batch(first, kind, APP)
    assert check_ops(ctx, kind, key, core, oc, acts, clears, fa, fv) == 0
    acts, clears, fa, fv = G.batch(files, kind, APP, start={a: 3 for a in files})
    assert check_ops(ctx, kind, key, core, oc, acts, clears, fa, fv) == 0
    core.close()


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
def test_ops_parity_larger(ctx, kind):
    """table growth / rebuild, many actors, thousands of ops"""
    rng = random.Random(77)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 64)
    core, oc = new_core(ctx, kind, key), C.Core(kind)
    files = gen(kind, rng, actors, 8, 12, 3000, False)
    for lo in range(0, 8, 2):
        part = {a: files[a][: lo + 2] for a in files}
        acts, clears, fa, fv = G.batch(part, kind, APP, start={a: lo for a in files})
        assert check_ops(ctx, kind, key, core, oc, acts, clears, fa, fv) == 0
    core.close()


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
def test_reject_and_gap(ctx, kind):
    rng = random.Random(5)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 3)
    core, oc = new_core(ctx, kind, key), C.Core(kind)
    files = gen(kind, rng, actors, 4, 3, 10, False)
    acts, clears, fa, fv = G.batch(files, kind, APP)
    sealed = seal_files(ctx, key, clears)
    # a tampered tag anywhere: nothing folded (lib.rs:497-514)
    bad = list(sealed)
    b = bytearray(bad[5])
    b[-1] ^= 1
    bad[5] = bytes(b)
    rc, st = core.ingest_ops(bad, acts, fa, fv)
    orc, ost = oc.read_remote_ops(key, [APP], bad, [acts[i] for i in fa], fv)
    assert rc == orc == 9 and st == ost
    # a decode error (not a Vec<Op>) rejects too
    bad = list(clears)
    bad[2] = APP + msgpack.packb({"x": 1})
    rc2 = check_ops(ctx, kind, key, core, oc, acts, bad, fa, fv)
    assert rc2 == 12
    assert core.state_bytes() == oc.serialize() == C.Core(kind).serialize()
    # a version gap for actor 1: earlier files stay folded, error at the gap (lib.rs:527-531)
    keep = [i for i in range(len(fa)) if not (fa[i] == 1 and fv[i] == 1)]
    rc3 = check_ops(ctx, kind, key, core, oc, acts, [clears[i] for i in keep], [fa[i] for i in keep],
                    [fv[i] for i in keep])
    assert rc3 == 13
    core.close()


def _noncanonical_orswot(ops, rng):
    """same ops, other accepted encodings: struct arrays, variant indices, field maps in a
    different order with unknown keys, unsorted removal clocks"""
    out = []
    for op in ops:
        if op[0] == "Add":
            _, (a, c), ms = op
            form = rng.randrange(3)
            if form == 0:
                out.append({0: [[a, c], ms]})
            elif form == 1:
                out.append({"Add": {"zz": [1, {"q": None}], "members": ms, "dot": {"counter": c, "actor": a}}})
            else:
                out.append({"Add": [{"actor": a, "counter": c}, ms]})
        else:
            _, clock, ms = op
            dots = list(clock.dots.items())
            rng.shuffle(dots)
            out.append({1: {"members": ms, "clock": [dict(dots)]}})
    return msgpack.packb(out, use_bin_type=True)


def test_orswot_accepts_rmp_forms(ctx):
    rng = random.Random(9)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 4)
    files = G.adversarial_orswot(rng, actors, 3, 6, 12)
    acts = sorted(files)
    clears, fa, fv = [], [], []
    for i, a in enumerate(acts):
        for v, ops in enumerate(files[a]):
            clears.append(APP + _noncanonical_orswot(ops, rng))
            fa.append(i)
            fv.append(v)
    core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
    assert check_ops(ctx, "orswot", key, core, oc, acts, clears, fa, fv) == 0
    core.close()


def seal_states(ctx, key, sws):
    """state files in the format read_remote_states reads (lib.rs:435-447)"""
    return seal_files(ctx, key, [APP + sw for sw in sws])


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
@pytest.mark.parametrize("seed", range(4))
def test_states_then_ops(ctx, kind, seed):
    rng = random.Random(300 + seed)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 5)
    adversarial = seed % 2 == 1
    # partial replicas -> state files
    sws = []
    for _ in range(3):
        part = C.Core(kind)
        files = gen(kind, rng, actors, 2, 5, 20, adversarial)
        acts, clears, fa, fv = G.batch(files, kind, APP)
        f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
        assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
        sws.append(part.serialize())
    core, oc = new_core(ctx, kind, key), C.Core(kind)
    sf = seal_states(ctx, key, sws)
    rc, st = core.ingest_states(sf)
    orc, ost = oc.read_remote_states(key, [APP], sf)
    assert (rc, st) == (orc, ost) == (0, [0, 0, 0])
    assert core.state_bytes() == oc.serialize()
    # then ops on top (read_remote: states, then ops), from writers the states have not seen
    files = gen(kind, rng, actors[:2] + G.actors_for(rng, 3), 3, 4, 20, adversarial)
    acts, clears, fa, fv = G.batch(files, kind, APP)
    check_ops(ctx, kind, key, core, oc, acts, clears, fa, fv)
    # and another state merged into a non-empty state
    sf = seal_states(ctx, key, [sws[0]])
    assert core.ingest_states(sf)[0] == oc.read_remote_states(key, [APP], sf)[0] == 0
    assert core.state_bytes() == oc.serialize()
    core.close()


@pytest.mark.parametrize("primary", [None, "32"])
@pytest.mark.parametrize("p_rm", [0.0, 0.25])
def test_orswot_kway_state_merge(ctx, p_rm, primary):
    """Many state files merged at once (launch_ds_kmerge, taken when no state and no current
    deferred set holds a removal) == the oracle's merges one by one, in two file orders, into an
    empty and into a non-empty state, and == the sequential device merges (CE_NO_KMERGE=1).
    States are version prefixes and writer subsets of one history: the same (member, actor) at
    different counters, values covered by another file's clock, entries only some files hold.
    primary "32": a 32-slot primary member table that is never grown (CE_DS_PRIMARY_SLOTS), so
    most members live in the overflow table."""
    if primary:
        os.environ["CE_DS_PRIMARY_SLOTS"] = primary
    try:
        _kway_state_merge(ctx, p_rm)
    finally:
        os.environ.pop("CE_DS_PRIMARY_SLOTS", None)


def test_orswot_kway_final_rows_form():
    """The k-way merge's opt-in final pass over the rows' pair owners (CE_KFINAL_ROWS=1,
    k_ds_kfinal_rows: taken for merges into an empty table) == the oracle, through the same
    k-way test in a child process (the switch is read once per process)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CE_KFINAL_ROWS="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        "tests/test_gpu_dotset.py::test_orswot_kway_state_merge"], cwd=repo, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "passed" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def _kway_state_merge(ctx, p_rm):
    rng = random.Random(91 + int(p_rm * 100))
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 6)
    files = G.well_formed_orswot(rng, actors, 6, 6, 40, p_rm=p_rm)[0]
    sws = []
    for v in range(1, 7):
        for sub in (actors, actors[::2], actors[1:4]):
            part = C.Core("orswot")
            hist = {a: files[a][:v] for a in sub}
            acts, clears, fa, fv = G.batch(hist, "orswot", APP)
            f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
            assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
            sws.append(part.serialize())
    rng.shuffle(sws)
    kway_runs = 0
    # (into an empty state: the k-way merge reads no current values; 40 files: 64-bit hold words)
    wide = (sws * 3)[:40]
    for batch, first in ((sws[:9], True), (sws[9:], True), (list(reversed(sws)), True), (sws[:9], False),
                         (wide, False), (wide, True)):
        got = []
        for env in (None, "1"):
            if env:
                os.environ["CE_NO_KMERGE"] = env
            try:
                core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
                if first:
                    pre = seal_states(ctx, key, [sws[0]])          # a non-empty state first
                    assert core.ingest_states(pre)[0] == oc.read_remote_states(key, [APP], pre)[0] == 0
                sf = seal_states(ctx, key, batch)
                rc, st = core.ingest_states(sf)
                orc, ost = oc.read_remote_states(key, [APP], sf)
                assert (rc, st) == (orc, ost) and rc == 0
                assert core.state_bytes() == oc.serialize()
                got.append(core.state_bytes())
                if not env:
                    kway_runs += core.path_count("states_kway_merge")
                core.close()
            finally:
                os.environ.pop("CE_NO_KMERGE", None)
        assert got[0] == got[1]
    if p_rm == 0.0:
        assert kway_runs >= 2   # adds only: no deferred removal anywhere


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
def test_local_apply_ops(ctx, kind):
    rng = random.Random(44)
    key = rng.randbytes(32)
    core = new_core(ctx, kind, key)
    me = core.info_actor()
    actors = G.actors_for(rng, 3)
    files = gen(kind, rng, actors, 2, 4, 10, True)
    oc = C.Core(kind)
    enc = C.enc_orswot_ops if kind == "orswot" else C.enc_mvreg_ops
    for a in sorted(files):
        for ops in files[a]:
            assert core.apply_ops(enc(ops)) == 0
            for op in ops:
                oc.state.apply(op)
            oc.nov.apply(me, oc.nov.get(me) + 1)
    assert core.state_bytes() == oc.serialize()
    assert core.apply_ops(msgpack.packb([{"Nope": 1}])) == 12
    core.close()


def test_orswot_sharded_merge_equals_single(ctx):
    """multi-GPU exchange step: actor shards fold independently, then each merges the other's
    partial StateWrapper (all-gather + local merge) == one core over everything"""
    rng = random.Random(8)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 8)
    files = G.well_formed_orswot(rng, actors, 4, 6, 30)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    whole = new_core(ctx, "orswot", key)
    assert whole.ingest_ops(sealed, acts, fa, fv)[0] == 0
    parts = []
    for r in range(2):
        idx = [i for i in range(len(fa)) if fa[i] % 2 == r]
        core = new_core(ctx, "orswot", key)
        assert core.ingest_ops([sealed[i] for i in idx], acts, [fa[i] for i in idx],
                               [fv[i] for i in idx])[0] == 0
        parts.append(core)
    sw = [p.state_bytes() for p in parts]
    assert parts[0].merge_state(sw[1]) == 0 and parts[1].merge_state(sw[0]) == 0
    assert parts[0].state_bytes() == parts[1].state_bytes() == whole.state_bytes()
    for p in parts + [whole]:
        p.close()


def test_compact_roundtrip(ctx):
    rng = random.Random(12)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 3)
    files = G.well_formed_orswot(rng, actors, 3, 5, 15)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP,
                        flags=crdtenc.COMPACT_INGEST_FORMAT)
    core.set_latest_key(key)
    assert core.ingest_ops(seal_files(ctx, key, clears), acts, fa, fv)[0] == 0
    f, name = core.compact_to_buffer(nonce=bytes(24))
    buf, n, name2 = core.compact_into(np.zeros(1, np.uint8), nonce=bytes(24))
    assert bytes(buf[:n]) == f and name2 == name
    other = new_core(ctx, "orswot", key)
    assert other.ingest_states([f])[0] == 0
    assert other.state_bytes() == core.state_bytes()
    core.close()
    other.close()


def _orswot_state_forms(sw, rng):
    """Re-encodings of one canonical StateWrapper<Orswot> (oracle bytes) that
    read_remote_states accepts: (name, bytes, device-reader eligible)."""
    d = msgpack.unpackb(sw, raw=True, strict_map_key=False, object_pairs_hook=list)
    dd = dict(d)
    nov, st = dd[b"next_op_versions"], dict(dd[b"state"])
    entries = st[b"entries"]

    def enc(entries_pairs, member_enc=None, vclock_enc=None):
        w = C.Wr()
        w.map(2)
        w.str("next_op_versions")
        w.b += msgpack.packb(dict(nov), use_bin_type=True) if False else _vclock_bytes(nov)
        w.str("state")
        w.map(3)
        w.str("clock")
        w.b += _vclock_bytes(st[b"clock"])
        w.str("entries")
        w.map(len(entries_pairs))
        for m, vc in entries_pairs:
            w.b += member_enc(m) if member_enc else msgpack.packb(m)
            w.b += vclock_enc(vc) if vclock_enc else _vclock_bytes(vc)
        w.str("deferred")
        w.b += msgpack.packb(st[b"deferred"], use_bin_type=True) if False else _raw_deferred(sw)
        return bytes(w.b)

    out = [("canonical", sw, True)]
    shuffled = list(entries)
    rng.shuffle(shuffled)
    out.append(("hashmap_order", enc(shuffled), True))
    if len(entries) >= 2:
        dup = list(entries) + [(entries[0][0], entries[1][1])]   # repeated member: later clock wins
        out.append(("repeated_member", enc(dup), False))
        out.append(("long_uint_member", enc(list(entries), member_enc=lambda m: b"\xcf" + m.to_bytes(8, "big")), False))
        out.append(("descending_dots", enc(list(entries), vclock_enc=lambda vc: _vclock_bytes(vc, reverse=True)), False))
        # the all-ones member is the repeat check's empty word: once (device) and repeated (host)
        top = (1 << 64) - 1
        out.append(("all_ones_member", enc([(top, entries[0][1])] + list(entries[1:])), True))
        out.append(("repeated_all_ones_member", enc([(top, entries[0][1]), (top, entries[1][1])] + list(entries[2:])), False))
    return out


def _vclock_bytes(vc, reverse=False):
    pairs = dict(vc)[b"dots"] if isinstance(vc, list) else vc[b"dots"]
    w = C.Wr()
    w.map(1)
    w.str("dots")
    items = sorted(pairs, key=lambda p: p[0], reverse=reverse)
    w.map(len(items))
    for a, c in items:
        w.bin(a)
        w.uint(c)
    return bytes(w.b)


def _raw_deferred(sw):
    """the canonical deferred map's bytes (everything after the "deferred" key)"""
    i = sw.rindex(b"\xa8deferred")
    return sw[i + 9:]


@pytest.mark.parametrize("seed", range(3))
def test_orswot_state_reader_forms(ctx, seed):
    """read_remote_states for Orswot decodes canonical state files on the device
    (ce_dotset_io.hip: parallel entry-head search + chained per-entry parse) and declines every
    other accepted form to the host parser; both give the oracle's state.  CE_HOST_STATES=1
    (the host parser for everything) is compared too."""
    import os
    rng = random.Random(900 + seed)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 6)
    part = C.Core("orswot")
    files = gen("orswot", rng, actors, 3, 6, 40, seed == 2)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
    assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
    sw = part.serialize()
    for name, body, eligible in _orswot_state_forms(sw, rng):
        sf = seal_files(ctx, key, [APP + body])
        oc = C.Core("orswot")
        orc, ost = oc.read_remote_states(key, [APP], sf)
        assert orc == 0, name
        for host in (False, True):
            if host:
                os.environ["CE_HOST_STATES"] = "1"
            try:
                core = new_core(ctx, "orswot", key)
                rc, st = core.ingest_states(sf)
                assert (rc, st) == (orc, ost), (name, host)
                assert core.state_bytes() == oc.serialize(), (name, host)
                dev = core.path_count("states_device_read")
                assert dev == (1 if (eligible and not host) else 0), (name, host, dev)
                if not host:
                    assert core.path_count("states_host_parse") == 1 - dev
                core.close()
            finally:
                os.environ.pop("CE_HOST_STATES", None)


def test_orswot_state_reader_long_deferred(ctx):
    """A state whose deferred map is longer than the reader's 4 KiB pinned tail window
    (k_rdm_tail) is read on the device with the map downloaded instead; beside it a state with
    an empty map takes the window.  Both give the oracle's state."""
    rng = random.Random(77)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 24)
    part = C.Core("orswot")
    files = G.adversarial_orswot(rng, actors, 2, 40, 60)
    # removals far past every add: each stays deferred under its own clock (~9 KiB of map)
    files[actors[0]].append([("Rm", C.VClock({actors[j % 24]: 1000 + j}), [j % 60, (7 * j) % 60])
                             for j in range(300)])
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
    assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
    big = part.serialize()
    assert len(_raw_deferred(big)) > 4096
    small_part = C.Core("orswot")
    wf = G.well_formed_orswot(rng, actors[:4], 2, 6, 30)[0]
    acts, clears, fa, fv = G.batch(wf, "orswot", APP)
    f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
    assert small_part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
    for bodies in ([big], [small_part.serialize(), big]):
        sf = seal_files(ctx, key, [APP + b for b in bodies])
        oc = C.Core("orswot")
        assert oc.read_remote_states(key, [APP], sf)[0] == 0
        core = new_core(ctx, "orswot", key)
        rc, st = core.ingest_states(sf)
        assert rc == 0 and list(st) == [0] * len(bodies)
        assert core.state_bytes() == oc.serialize()
        assert core.path_count("states_device_read") == len(bodies)
        core.close()


@pytest.mark.parametrize("form", ["canonical", "map16_empty_deferred", "no_early"])
def test_orswot_kway_merge_queued_early(ctx, form):
    """With several state files and no deferred removal held, the k-way merge is queued behind
    the reader before the host wait and runs only if every file read cleanly with its deferred
    map in the one canonical empty form (k_rdm_flags' go word); a map16 {} -- accepted, but not
    that form -- leaves the early merge idle and the host queues the same merge after the wait.
    CE_NO_KMERGE_EARLY=1 turns the early merge off.  All three equal the oracle."""
    import os
    rng = random.Random(4242)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 8)
    bodies = []
    for k in range(3):
        part = C.Core("orswot")
        wf = G.well_formed_orswot(rng, actors, 2, 5, 50)[0]
        acts, clears, fa, fv = G.batch(wf, "orswot", APP)
        f = [CORE + C._oc.cryptor_encrypt(key, bytes(24), c)[1] for c in clears]
        assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
        sw = part.serialize()
        assert sw.endswith(b"\xa8deferred\x80")
        bodies.append(sw)
    if form == "map16_empty_deferred":
        bodies[1] = bodies[1][:-1] + b"\xde\x00\x00"
    sf = seal_files(ctx, key, [APP + b for b in bodies])
    oc = C.Core("orswot")
    assert oc.read_remote_states(key, [APP], sf)[0] == 0
    if form == "no_early":
        os.environ["CE_NO_KMERGE_EARLY"] = "1"
    try:
        core = new_core(ctx, "orswot", key)
        rc, st = core.ingest_states(sf)
        assert rc == 0 and list(st) == [0, 0, 0]
        assert core.state_bytes() == oc.serialize()
        assert core.path_count("states_device_read") == 3
        assert core.path_count("states_kway_merge") == 1
        assert core.path_count("states_kway_early") == (1 if form == "canonical" else 0)
        core.close()
    finally:
        os.environ.pop("CE_NO_KMERGE_EARLY", None)


def test_orswot_device_compaction_bytes(ctx):
    """Core::compact for Orswot writes the clear text on the device (ce_dotset_io.hip writer):
    the sealed file opens to exactly data_version || the canonical StateWrapper (host writer ==
    oracle bytes), in both output formats."""
    rng = random.Random(77)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 7)
    files = G.well_formed_orswot(rng, actors, 5, 8, 300)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    oc = C.Core("orswot")
    sealed = seal_files(ctx, key, clears)
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    for flags, outer, pre in ((crdtenc.COMPACT_INGEST_FORMAT, CORE, APP), (0, APP, b"")):
        core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP,
                            flags=flags)
        core.set_latest_key(key)
        assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
        assert core.state_bytes() == oc.serialize()
        f, _ = core.compact_to_buffer(nonce=bytes(24))
        assert f[:16] == outer
        st, pt = ctx.decrypt(key, f[16:])
        assert st == 0 and pt == pre + oc.serialize()
        assert core.path_count("compact_device_writer") == 1
        core.close()


def test_c3_shaped_medium(ctx):
    """C3's shape at a size the Python oracle folds in a few seconds: 256 actors, 10k members,
    four state files (each a quarter of the actors' first two versions) decoded on the device,
    then two more versions of op files from every actor (12 ops each, single-member Adds and
    Rms whose clocks span the actors), then the compaction through the device writer.  State
    bytes == oracle at every stage."""
    rng = random.Random(3)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 256)
    files = G.well_formed_orswot(rng, actors, 4, 12, 10000, max_members=1)[0]
    sws = []
    for q in range(4):
        part = C.Core("orswot")
        sub = {a: files[a][:2] for a in actors[q * 64:(q + 1) * 64]}
        acts, clears, fa, fv = G.batch(sub, "orswot", APP)
        f = seal_files(ctx, key, clears)
        assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
        sws.append(part.serialize())
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    oc = C.Core("orswot")
    sf = seal_states(ctx, key, sws)
    rc, st = core.ingest_states(sf)
    assert (rc, st) == oc.read_remote_states(key, [APP], sf) == (0, [0] * 4)
    assert core.state_bytes() == oc.serialize()
    assert core.path_count("states_device_read") == 4
    acts, clears, fa, fv = G.batch(files, "orswot", APP, start={a: 2 for a in actors})
    assert check_ops(ctx, "orswot", key, core, oc, acts, clears, fa, fv) == 0
    f, _ = core.compact_to_buffer(nonce=bytes(24))
    st, pt = ctx.decrypt(key, f[16:])
    assert st == 0 and pt == oc.serialize()
    assert core.path_count("compact_device_writer") == 1
    core.close()


def _c_fold(key, states, files, acts, fa, fv):
    """oracle/ce_oracle.c oc_compact_orswot_best (the C restatement, pinned to oracle/crdts.py by
    tests/test_oracle_orswot_c.py): states merged, then the op files folded in load_ops order"""
    import oracle
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(f) for f in files])
    actor = np.frombuffer(b"".join(acts[i] for i in fa) or bytes(16), np.uint8).reshape(-1, 16)
    err, sw, _, _ = oracle.compact_orswot_best(key, APP, states, b"".join(files) or b"\0", offs,
                                               actor, np.array(list(fv) or [0], np.uint64), 16)
    return err, sw


def test_c3_full_size_adversarial(ctx):
    """C3 at full size: 4096 actors, members drawn from 100k, four state files (a quarter of the
    writers' version 0 each) read on the device, then versions 1-2 of every writer: Adds naming
    other writers' dots, multi-actor removal clocks that defer -- ~98k ops in 12k op files --
    then the compaction through the device writer.  The Python oracle is too slow at this size;
    the checker is its C restatement."""
    rng = random.Random(4096)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 4096)
    hist = G.adversarial_orswot(rng, actors, 3, 8, 100_000)
    sws = []
    for q in range(4):
        sub = {a: hist[a][:1] for a in actors[q * 1024:(q + 1) * 1024]}
        acts, clears, fa, fv = G.batch(sub, "orswot", APP)
        err, sw = _c_fold(key, [], seal_files(ctx, key, clears), acts, fa, fv)
        assert err == 0
        sws.append(sw)
    sf = seal_states(ctx, key, sws)
    acts, clears, fa, fv = G.batch(hist, "orswot", APP, start={a: 1 for a in actors})
    files = seal_files(ctx, key, clears)
    err, want = _c_fold(key, sf, files, acts, fa, fv)
    assert err == 0 and b"deferred" in want
    core = new_core(ctx, "orswot", key)
    assert core.ingest_states(sf) == (0, [0] * 4)
    assert core.path_count("states_device_read") == 4
    rc, st = core.ingest_ops(files, acts, fa, fv)
    assert rc == 0 and st == [0] * len(files)
    got = core.state_bytes()
    assert len(got) == len(want) and got == want
    f, _ = core.compact_to_buffer(nonce=bytes(24))
    st, pt = ctx.decrypt(key, f[16:])
    assert st == 0 and pt == want
    assert core.path_count("compact_device_writer") == 1
    core.close()


def test_ingest_states_iov_matches_blob(ctx):
    """ce_core_ingest_states_iov (per-file host buffers through the pinned staging ring) ==
    ce_core_ingest_states (one blob): statuses and state bytes, a tampered file included."""
    rng = random.Random(11)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 6)
    sws = []
    for _ in range(3):
        part = C.Core("orswot")
        files = gen("orswot", rng, actors, 2, 6, 50, False)
        acts, clears, fa, fv = G.batch(files, "orswot", APP)
        f = seal_files(ctx, key, clears)
        assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
        sws.append(part.serialize())
    sf = seal_states(ctx, key, sws)
    a, b = new_core(ctx, "orswot", key), new_core(ctx, "orswot", key)
    assert a.ingest_states(sf) == b.ingest_states_iov(sf) == (0, [0, 0, 0])
    assert a.state_bytes() == b.state_bytes()
    bad = list(sf)
    t = bytearray(bad[1])
    t[-3] ^= 1
    bad[1] = bytes(t)
    ra, rb = a.ingest_states(bad), b.ingest_states_iov(bad)
    assert ra == rb and ra[0] == 9
    assert a.state_bytes() == b.state_bytes()
    a.close()
    b.close()


def _u(x, w):
    """msgpack uint in a chosen width (rmp-serde's reader accepts every one of them)"""
    if w == "fix":
        return bytes([x])
    if w == "d2":  # signed int32 marker, non-negative value (the serde u64 visitor accepts it)
        return b"\xd2" + x.to_bytes(4, "big", signed=True)
    n = {"cc": 1, "cd": 2, "ce": 4, "cf": 8}[w]
    return bytes([{"cc": 0xcc, "cd": 0xcd, "ce": 0xce, "cf": 0xcf}[w]]) + x.to_bytes(n, "big")


def _arr(n):
    return bytes([0x90 | n]) if n < 16 else b"\xdc" + n.to_bytes(2, "big")


def _add(actor, ctr, members, cw, mw):
    return (b"\x81\xa3Add\x82\xa3dot\x82\xa5actor\xc4\x10" + actor + b"\xa7counter" + _u(ctr, cw) +
            b"\xa7members" + _arr(len(members)) + b"".join(_u(m, mw) for m in members))


def _rm(clock, members, cw, mw):
    return (b"\x81\xa2Rm\x82\xa5clock\x81\xa4dots" + bytes([0x80 | len(clock)]) +
            b"".join(b"\xc4\x10" + a + _u(c, cw) for a, c in clock) +
            b"\xa7members" + _arr(len(members)) + b"".join(_u(m, mw) for m in members))


@pytest.mark.parametrize("case", ["widths", "mixed_fallback", "truncated_tail", "near_template"])
def test_orswot_op_fast_path_boundaries(ctx, case):
    """The device op decode proves canonical one-member Add / one-entry-clock Rm ops from register
    windows (ce_dotset.hip fast_orswot_op) and hands every other form to the grammar from the
    same op on: each uint width, multi-member / multi-entry ops between fast ones, a signed
    marker, a field-name near miss and a file cut inside its last op -- all == oracle."""
    rng = random.Random(sum(map(ord, case)))
    key = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(3))
    widths = ["fix", "cc", "cd", "ce", "cf"]
    clears, fa, fv = [], [], []
    for a in range(3):
        for v in range(4):
            ops = []
            base = 64 * v + 1
            for j in range(10):
                cw, mw = widths[(j + v) % 5], widths[(j + a) % 5]
                ctr = base + j if cw != "fix" else min(base + j, 127)
                lim = {"fix": 128, "cc": 256, "cd": 65536, "ce": 1 << 32, "cf": 1 << 64}
                mem = rng.randrange(0, lim[mw])
                if case == "widths" or j % 3:
                    ops.append(_add(actors[a], ctr, [mem], cw, mw))
                elif case == "mixed_fallback":
                    ops.append(_add(actors[a], ctr, [1, 2, 3], cw, "cd") if j % 2 else
                               _rm([(actors[0], 5), (actors[2], 9)], [4], "cc", "fix"))
                    ops.append(_add(actors[a], 2000 + ctr, [7], "d2", "cc"))
                else:
                    ops.append(_rm([(actors[(a + j) % 3], base)], [mem % 50], "cc" if cw == "fix" else cw, "cd"))
            if case == "near_template" and v == 2:
                ops[4] = ops[4].replace(b"members", b"membres", 1)  # unknown field -> members missing
            body = _arr(len(ops)) + b"".join(ops)
            if case == "truncated_tail" and a == 1 and v == 3:
                body = body[:-3]
            clears.append(APP + body)
            fa.append(a)
            fv.append(v)
    core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
    check_ops(ctx, "orswot", key, core, oc, actors, clears, fa, fv)
    core.close()


@pytest.mark.parametrize("case", ["ascending", "unordered", "repeated", "cut", "signed"])
def test_orswot_multi_entry_clock_fast_path(ctx, case):
    """Removals whose clock carries the member's read context (2..15 entries, crdts
    rm(member, read_ctx)) are proven by the lane decode's window path (fast_orswot_op) -- every
    uint width, entry counts 2..15 -- and anything it must not take goes to the grammar from the
    same op: actors out of order or repeated (ds_vclock reports those for the host parse), a file
    cut inside an entry, a signed counter marker.  All == the oracle."""
    rng = random.Random(sum(map(ord, case)) + 77)
    key = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(16))
    widths = ["fix", "cc", "cd", "ce", "cf"]
    lim = {"fix": 128, "cc": 256, "cd": 65536, "ce": 1 << 32, "cf": 1 << 64}
    clears, fa, fv = [], [], []
    for a in range(4):
        for v in range(4):
            ops = []
            for j in range(12):
                cw = widths[(j + v + a) % 5]
                if j % 3 == 0:
                    ops.append(_add(actors[a], 64 * v + j + 1, [rng.randrange(0, 40)], "cc", "fix"))
                    continue
                ne = 2 + (j * 5 + v + a) % 14
                sel = sorted(rng.sample(range(16), ne))
                clock = [(actors[k], rng.randrange(1, lim[cw])) for k in sel]
                if case == "unordered" and j == 4 and v % 2 == 0:
                    clock[0], clock[-1] = clock[-1], clock[0]
                if case == "repeated" and j == 5 and v % 2 == 1:
                    clock[1] = (clock[0][0], clock[1][1])
                op = _rm(clock, [rng.randrange(0, 40)], cw, "fix")
                if case == "signed" and j == 7:
                    op = op.replace(b"\xc4\x10" + clock[1][0] + _u(clock[1][1], cw),
                                    b"\xc4\x10" + clock[1][0] + b"\xd2" + (5).to_bytes(4, "big"), 1)
                ops.append(op)
            body = _arr(len(ops)) + b"".join(ops)
            if case == "cut" and a == 2 and v == 1:
                body = body[:-25]
            clears.append(APP + body)
            fa.append(a)
            fv.append(v)
    core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
    check_ops(ctx, "orswot", key, core, oc, actors[:4], clears, fa, fv)
    core.close()


@pytest.mark.parametrize("kind", ["orswot", "mvreg", "gcounter"])
def test_state_bytes_and_merge_device(ctx, kind):
    """The dot-set exchange without a host hop (shard.reduce_dotset): ce_core_state_bytes_device
    writes exactly ce_core_state_bytes into HBM (straight from the device writer, and through the
    grow-and-retry path when the buffer is short), and ce_core_merge_state_device of those bytes
    == ce_core_merge_state of the host copy == the oracle's merge, deferred removals included."""
    import torch
    rng = random.Random(31 if kind != "mvreg" else 32)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 12)
    dev = torch.device("cuda", 0)
    okind = "orswot" if kind == "gcounter" else kind
    hist = gen(okind, rng, actors, 3, 8, 400, True)
    halves = [{a: hist[a] for a in actors[:6]}, {a: hist[a] for a in actors[6:]}]
    parts = []
    for h in halves:
        if kind == "gcounter":
            core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
            core.set_latest_key(key)
            acts = list(h)
            clears, fa, fv = [], [], []
            for i, a in enumerate(acts):
                for v in range(3):
                    dots = [{"actor": rng.choice(actors), "counter": rng.getrandbits(40) + 1} for _ in range(9)]
                    clears.append(APP + msgpack.packb(dots, use_bin_type=True))
                    fa.append(i)
                    fv.append(v)
            assert core.ingest_ops(seal_files(ctx, key, clears), acts, fa, fv)[0] == 0
        else:
            core = new_core(ctx, okind, key)
            acts, clears, fa, fv = G.batch(h, okind, APP)
            assert core.ingest_ops(seal_files(ctx, key, clears), acts, fa, fv)[0] == 0
        parts.append(core)
    a, b = parts
    want_b = b.state_bytes()
    buf = torch.zeros(len(want_b) + 4096, dtype=torch.uint8, device=dev)
    rc, n = b.state_bytes_device(buf.data_ptr(), buf.numel())
    assert rc == 0 and n == len(want_b)
    torch.cuda.synchronize()
    assert bytes(buf[:n].cpu().numpy().tobytes()) == want_b
    small = torch.zeros(16, dtype=torch.uint8, device=dev)
    rc, n2 = b.state_bytes_device(small.data_ptr(), small.numel())
    assert rc == 64 and n2 == len(want_b)
    # the host merge on a copy of a's state, then the device merge into a
    ref = crdtenc.Core(ctx, kind=a_kind(kind), supported=[APP], current_data_version=APP)
    assert ref.merge_state(a.state_bytes()) == 0 and ref.merge_state(want_b) == 0
    assert a.merge_state_device(buf.data_ptr(), n) == 0
    assert a.state_bytes() == ref.state_bytes()
    if kind != "gcounter":
        oc = C.Core(okind)
        oc2 = C.Core(okind)
        for h, o in zip(halves, (oc, oc2)):
            acts, clears, fa, fv = G.batch(h, okind, APP)
            assert o.read_remote_ops(key, [APP], seal_files(ctx, key, clears), [acts[i] for i in fa], fv)[0] == 0
        assert oc2.serialize() == want_b
        sf = seal_states(ctx, key, [oc2.serialize()])
        assert oc.read_remote_states(key, [APP], sf)[0] == 0
        assert a.state_bytes() == oc.serialize()
    if kind == "orswot":
        assert a.path_count("states_device_read") == 1
    for x in (a, b, ref):
        x.close()


def a_kind(kind):
    return {"orswot": crdtenc.STATE_ORSWOT, "mvreg": crdtenc.STATE_MVREG, "gcounter": crdtenc.STATE_GCOUNTER}[kind]


def test_ingest_states_device_matches_host(ctx):
    """ce_core_ingest_states_device (state files resident in HBM) == ce_core_ingest_states (host
    blob): statuses and state bytes, for Orswot (device state reader) and GCounter (host parse of
    the device-opened plaintexts), a tampered file included."""
    import torch
    rng = random.Random(12)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 6)
    sws = []
    for _ in range(3):
        part = C.Core("orswot")
        files = gen("orswot", rng, actors, 2, 6, 50, False)
        acts, clears, fa, fv = G.batch(files, "orswot", APP)
        f = seal_files(ctx, key, clears)
        assert part.read_remote_ops(key, [APP], f, [acts[i] for i in fa], fv)[0] == 0
        sws.append(part.serialize())
    dev = torch.device("cuda", 0)

    def on_device(fs):
        offs = np.zeros(len(fs) + 1, np.int64)
        offs[1:] = np.cumsum([len(x) for x in fs])
        blob = torch.from_numpy(np.frombuffer(b"".join(fs) + bytes(64), np.uint8).copy()).to(dev)
        return blob, torch.from_numpy(offs).to(dev), int(offs[-1])
    for fs in (seal_states(ctx, key, sws), None):
        if fs is None:   # one tampered file: nothing merged, same statuses
            fs = seal_states(ctx, key, sws)
            t = bytearray(fs[1])
            t[-3] ^= 1
            fs[1] = bytes(t)
        a, b = new_core(ctx, "orswot", key), new_core(ctx, "orswot", key)
        blob, offs, ln = on_device(fs)
        torch.cuda.synchronize()
        ra = a.ingest_states(fs)
        rb = b.ingest_states_device(blob.data_ptr(), offs.data_ptr(), len(fs), ln, want_status=True)
        assert ra == rb and (ra[0] in (0, 9))
        assert a.state_bytes() == b.state_bytes()
        a.close()
        b.close()


@pytest.mark.parametrize("adversarial", [False, True])
def test_orswot_adds_without_sort(ctx, adversarial):
    """The fold's applied flags skip the stable sort by actor when every actor's adds form one
    contiguous run (k_ds_contig): the well-formed history (each writer adding its own dots, in
    load_ops order) takes that path, the adversarial one (adds naming other writers' dots) the
    sort; both == the oracle, and == the sort path forced with CE_DS_SORT_ADDS=1."""
    rng = random.Random(515 + adversarial)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 9)
    files = gen("orswot", rng, actors, 4, 10, 200, adversarial)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    got = {}
    for mode in (None, "CE_DS_NO_MONO", "CE_DS_SORT_ADDS"):
        if mode:
            os.environ[mode] = "1"
        try:
            core = new_core(ctx, "orswot", key)
            assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
            got[mode] = (core.state_bytes(), core.path_count("ds_adds_contiguous"), core.path_count("ds_adds_monotone"))
            core.close()
        finally:
            if mode:
                os.environ.pop(mode, None)
    assert got[None][0] == got["CE_DS_NO_MONO"][0] == got["CE_DS_SORT_ADDS"][0] == oc.serialize()
    assert got["CE_DS_SORT_ADDS"][1:] == (0, 0)
    # well-formed: contiguous, strictly increasing runs -> the applied flags from k_ds_contig
    assert got[None][1:] == ((0, 0) if adversarial else (0, 1))
    assert got["CE_DS_NO_MONO"][1:] == ((0, 0) if adversarial else (1, 0))


def test_orswot_adds_contiguous_not_increasing(ctx):
    """A writer's adds contiguous (its own dots) but their counters not strictly increasing: a
    repeated and a lower counter inside the run.  k_ds_contig flags the run, the fold takes the
    segmented max scan (ds_adds_contiguous, not ds_adds_monotone), and the state == the oracle's
    (the lower / repeated counters do not apply)."""
    rng = random.Random(5151)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 3)
    files = {actors[0]: [[("Add", (actors[0], 5), [1]), ("Add", (actors[0], 3), [2]), ("Add", (actors[0], 5), [3]),
                          ("Add", (actors[0], 9), [4])]],
             actors[1]: [[("Add", (actors[1], 2), [1]), ("Add", (actors[1], 4), [5])]],
             actors[2]: [[("Add", (actors[2], 7), [6]), ("Add", (actors[2], 7), [7])]]}
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    core = new_core(ctx, "orswot", key)
    assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
    assert core.state_bytes() == oc.serialize()
    assert core.path_count("ds_adds_contiguous") == 1 and core.path_count("ds_adds_monotone") == 0
    core.close()


def test_compact_into_async_overlaps_next_ingest(ctx):
    """ce_core_compact_into_async leaves the sealed file's download in flight: the next batch's
    reset, ingest and compaction are queued before the first download is waited for, and both
    files still open to exactly the StateWrappers they were compacted from (the seal has its own
    output buffer; the second seal waits for the first download on the device)."""
    import torch
    rng = random.Random(808)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 8)
    core = new_core(ctx, "orswot", key)
    bufs = [crdtenc.host_buffer(1 << 22) for _ in range(2)]
    want, tickets = [], []
    for r in range(2):
        files = gen("orswot", rng, actors, 3, 8, 500 + 100 * r, False)
        acts, clears, fa, fv = G.batch(files, "orswot", APP)
        core.reset()
        assert core.ingest_ops(seal_files(ctx, key, clears), acts, fa, fv)[0] == 0
        want.append(core.state_bytes())
        tickets.append(core.compact_into_async(bufs[r], nonce=bytes(24)))
    assert tickets[0][1] != 0 and tickets[1][1] > tickets[0][1]
    assert tickets[0][0] == tickets[1][0] == 0      # lengths come with the wait
    lens = {}
    for r in (1, 0):
        _, t = tickets[r]
        lens[r] = ln = core.compact_wait(t)
        f = bytes(bufs[r][:ln])
        assert f[:16] == APP
        st, pt = ctx.decrypt(key, f[16:])
        assert st == 0 and pt == want[r]
    assert core.compact_wait(tickets[0][1]) == lens[0]   # waiting twice is fine
    assert core.path_count("compact_async") == 2
    # a pinned buffer too small: the wait reports it; a pageable buffer: the synchronous path
    small = crdtenc.host_buffer(64)
    ln, t = core.compact_into_async(small, nonce=bytes(24))
    with pytest.raises(Exception):
        core.compact_wait(t)
    import numpy as np
    pageable = np.zeros(1 << 22, np.uint8)
    ln, t = core.compact_into_async(pageable, nonce=bytes(24))
    assert t == 0 and ln > 0 and bytes(pageable[:16]) == APP
    core.close()


@pytest.mark.parametrize("adversarial", [False, True])
def test_orswot_tiled_emit_equals_direct(ctx, adversarial):
    """The op decode's tiled emit (file-minor scratch rows, then k_ds_untile into the CSR
    columns) == the direct per-lane stores (CE_DS_EMIT_DIRECT=1) == the oracle, on uniform and on
    ragged files (op counts 1-10 per file, empty member lists, multi-entry removal clocks)."""
    rng = random.Random(616 + adversarial)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 11)
    files = gen("orswot", rng, actors, 5, 10, 300, adversarial)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    got = {}
    for direct in (False, True):
        if direct:
            os.environ["CE_DS_EMIT_DIRECT"] = "1"
        try:
            core = new_core(ctx, "orswot", key)
            assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
            got[direct] = (core.state_bytes(), core.path_count("ds_emit_tiled"))
            core.close()
        finally:
            os.environ.pop("CE_DS_EMIT_DIRECT", None)
    assert got[False][0] == got[True][0] == oc.serialize()
    assert got[False][1] == 1 and got[True][1] == 0


@pytest.mark.parametrize("adversarial", [False, True])
def test_orswot_partitioned_fold_equals_global(ctx, adversarial):
    """The partitioned fold (items reserved into per-partition runs, each partition folded in LDS:
    k_ds_part_*; with 64-item runs most items go through the overflow lists) == the global kernels (k_ds_add_pairs / k_ds_kill / k_ds_finalize, forced with
    CE_DS_FOLD_GLOBAL=1) == the oracle, over four batches that grow the tables past one partition
    and carry deferred removals from batch to batch (adversarial: removals naming other writers'
    dots, multi-entry clocks and several members per removal)."""
    rng = random.Random(717 + adversarial)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 24)
    files = gen("orswot", rng, actors, 8, 14, 2500, adversarial)
    batches = []
    for lo in range(0, 8, 2):
        part = {a: files[a][: lo + 2] for a in files}
        acts, clears, fa, fv = G.batch(part, "orswot", APP, start={a: lo for a in files})
        batches.append((acts, seal_files(ctx, key, clears), fa, fv))
    oc = C.Core("orswot")
    want = []
    for acts, sealed, fa, fv in batches:
        rc = oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0]
        want.append((rc, oc.serialize()))
    got = {}
    modes = {"partitioned": {}, "global": {"CE_DS_FOLD_GLOBAL": "1"},
             "member_overflow": {"CE_DS_PRIMARY_SLOTS": "64"},   # most members in the overflow table
             "run_overflow": {"CE_DS_PART_FACTOR": "0"}}          # 64-item runs: the overflow lists
    for mode, env in modes.items():
        os.environ.update(env)
        try:
            core = new_core(ctx, "orswot", key)
            out = []
            for acts, sealed, fa, fv in batches:
                out.append((core.ingest_ops(sealed, acts, fa, fv)[0], core.state_bytes()))
            got[mode] = (out, core.path_count("ds_fold_partitioned"), core.path_count("ds_fold_global"),
                         core.path_count("ds_fold_run_overflow"))
            core.close()
        finally:
            for k in env:
                os.environ.pop(k, None)
    for mode in modes:
        assert got[mode][0] == want, mode
    assert got["partitioned"][1:3] == (len(batches), 0)
    assert got["member_overflow"][1:3] == (len(batches), 0)
    assert got["run_overflow"][1:3] == (len(batches), 0)
    if not adversarial:   # (the adversarial batches apply few adds: their runs may not fill)
        assert got["run_overflow"][3] >= 1
    assert got["global"][1:3] == (0, len(batches))


@pytest.mark.parametrize("n_members", [300, 1 << 20, 1 << 40, (1 << 64) - 1, "shared"])
def test_orswot_serializer_one_sort_equals_two(ctx, n_members):
    """The device serializer orders the live (member, actor) pairs by (member, actor UUID rank):
    by the hand-written radix sort of the packed key when member bits + actor-rank bits fit 64
    (ce_ser_sort.hip), else by rank then stably by member (two pair sorts of the same kernels).
    Each form (default, CE_SER_TWO_SORTS=1) and the host serializer (state_bytes, its own
    pair sort) == the oracle's bytes, for small,
    20-bit, 40-bit (64-bit keys) and full 64-bit members (the two sorts), and for members every
    one of 300 actors adds (slices of 300 pairs)."""
    rng = random.Random(929 + (n_members % 1000 if isinstance(n_members, int) else 7))
    key = rng.randbytes(32)
    if n_members == "shared":
        actors = G.actors_for(rng, 300)
        files = {a: [[("Add", (a, 1), [5, 77, 1000 + i % 3])]] for i, a in enumerate(actors)}
    else:
        actors = G.actors_for(rng, 7)
        files = G.well_formed_orswot(rng, actors, 3, 8, n_members)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    import torch
    want = oc.serialize()
    got = []
    for mode in (None, "CE_SER_TWO_SORTS"):
        if mode:
            os.environ[mode] = "1"
        try:
            core = new_core(ctx, "orswot", key)
            assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
            buf = torch.zeros(len(want) + 4096, dtype=torch.uint8, device="cuda:0")
            rc, n = core.state_bytes_device(buf.data_ptr(), buf.numel())   # the device serializer
            assert rc == 0
            torch.cuda.synchronize()
            got.append(bytes(buf[:n].cpu().numpy().tobytes()))
            got.append(core.state_bytes())
            core.close()
        finally:
            if mode:
                os.environ.pop(mode, None)
    assert got[0] == got[1] == got[2] == got[3] == want


@pytest.mark.parametrize("member_bits", [18, 36])
def test_orswot_serializer_sort_many_tiles(ctx, member_bits):
    """The hand-written sort over many 4096-pair tiles (the look-back between tiles, every digit
    place, 32- and 64-bit keys): ~300 K live pairs from 256 writers, serialized on the device ==
    the same state serialized with the tiles ordered by an atomic ticket (CE_SORT_TICKET=1; by
    blockIdx otherwise, when every tile is resident; separate processes: the choices are read
    once), with the two-sort form and by the host serializer, and == the C restatement's bytes
    over the same files (oracle/ce_oracle.c)."""
    import subprocess
    import sys
    code = (
        "import os, sys, hashlib, random\n"
        "sys.path.insert(0, %r); sys.path.insert(0, %r); sys.path.insert(0, os.path.dirname(sys.path[0]))\n"
        "import crdtenc, torch\n"
        "import dotset_gen as G\n"
        "from oracle import crdts as C\n"
        "rng = random.Random(4242)\n"
        "key = rng.randbytes(32)\n"
        "actors = G.actors_for(rng, 256)\n"
        "files = {a: [[('Add', (a, v * 400 + j + 1), [(rng.getrandbits(%d) | 1) for _ in range(3)]) "
        "for j in range(400)] for v in range(1)] for a in actors}\n"
        "acts, clears, fa, fv = G.batch(files, 'orswot', bytes.fromhex(%r))\n"
        "ctx = crdtenc.Context(0)\n"
        "sealed = [bytes.fromhex(%r) + e for e in ctx.encrypt_batch(key, clears)]\n"
        "core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[bytes.fromhex(%r)], current_data_version=bytes.fromhex(%r))\n"
        "core.set_latest_key(key)\n"
        "assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0\n"
        "buf = torch.zeros(64 << 20, dtype=torch.uint8, device='cuda:0')\n"
        "rc, n = core.state_bytes_device(buf.data_ptr(), buf.numel())\n"
        "assert rc == 0, rc\n"
        "torch.cuda.synchronize()\n"
        "b = bytes(buf[:n].cpu().numpy().tobytes())\n"
        "assert core.state_bytes() == b\n"
        "if os.environ.get('CE_T_ORACLE'):\n"
        "    import numpy as np, oracle\n"
        "    offs = np.zeros(len(sealed) + 1, np.uint64); offs[1:] = np.cumsum([len(x) for x in sealed])\n"
        "    err, ser, _, _ = oracle.compact_orswot_best(key, bytes.fromhex(%r), [], b''.join(sealed), offs,\n"
        "        np.frombuffer(b''.join(acts[i] for i in fa), np.uint8).reshape(-1, 16), np.array(fv, np.uint64), 8, seal=False)\n"
        "    assert err == 0 and ser == b, 'C oracle differs'\n"
        "print(hashlib.sha256(b).hexdigest(), n)\n"
        % (os.path.join(REPO, "crdt-enc_amd"), os.path.join(REPO, "tests"), member_bits, APP.hex(),
           CORE.hex(), APP.hex(), APP.hex(), APP.hex()))
    outs = []
    for env in ({"CE_T_ORACLE": "1"}, {"CE_SORT_TICKET": "1"}, {"CE_SER_TWO_SORTS": "1"}):
        p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True,
                           timeout=300, cwd=REPO)
        assert p.returncode == 0, p.stderr.decode()[-2000:]
        outs.append(p.stdout.decode().split()[-2:])
    assert outs[0] == outs[1] == outs[2], outs
    assert int(outs[0][1]) > 300000 * 20


@pytest.mark.parametrize("kind", ["orswot", "mvreg"])
@pytest.mark.parametrize("adversarial", [False, True])
def test_staged_decode_equals_global(ctx, kind, adversarial):
    """The staged op decode (CE_DS_DECODE_STAGE=1: a wave's files copied into LDS, the parse
    reading dword-aligned LDS words) == the HBM-reading decode == the oracle: statuses and state,
    on canonical and adversarial files (ragged sizes, non-canonical forms, multi-entry clocks)."""
    rng = random.Random(1313 + adversarial + (kind == "mvreg") * 7)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 9)
    files = gen(kind, rng, actors, 5, 12, 300, adversarial)
    acts, clears, fa, fv = G.batch(files, kind, APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core(kind)
    want = oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)
    got = {}
    for staged in (False, True):
        os.environ["CE_DS_DECODE_STAGE"] = "1" if staged else "0"
        try:
            core = new_core(ctx, kind, key)
            got[staged] = (core.ingest_ops(sealed, acts, fa, fv), core.state_bytes())
            core.close()
        finally:
            os.environ.pop("CE_DS_DECODE_STAGE", None)
    assert got[False] == got[True]
    assert got[True][0] == want and got[True][1] == oc.serialize()


def test_local_apply_after_contiguous_ingest(ctx):
    """a load_ops-ordered ingest whose adds are one run per actor takes the
    sort-free applied flags; a later local apply_ops with interleaved actors (Add(A), Add(B),
    Add(A)) must not inherit that flag -- it takes the sorted path and equals the oracle."""
    rng = random.Random(2024)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 6)
    files, truth = G.well_formed_orswot(rng, actors, 3, 8, 200)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
    assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    # (contiguous, strictly increasing runs: the applied flags come from k_ds_contig)
    assert core.path_count("ds_adds_monotone") == 1 and core.path_count("ds_adds_contiguous") == 0
    me = core.info_actor()
    a, b = acts[0], acts[1]
    ca, cb = oc.state.clock.get(a), oc.state.clock.get(b)
    for rnd in range(3):
        ops = [("Add", (a, ca + 1), [1000 + rnd]), ("Add", (b, cb + 1), [2000 + rnd]),
               ("Add", (a, ca + 2), [3000 + rnd]), ("Add", (b, cb + 2), [1000 + rnd])]
        ca, cb = ca + 2, cb + 2
        assert core.apply_ops(C.enc_orswot_ops(ops)) == 0
        for op in ops:
            oc.state.apply(op)
        oc.nov.apply(me, oc.nov.get(me) + 1)
        assert core.state_bytes() == oc.serialize(), rnd
    # the local applies took the sort
    assert core.path_count("ds_adds_monotone") == 1 and core.path_count("ds_adds_contiguous") == 0
    core.close()


def test_table_overflow_is_sticky_until_reset(ctx):
    """a pair-table overflow is found on the device after the ingest
    returned; it must not be lost.  With the pair table pinned at 4096 slots
    (CE_DS_TEST_PAIR_CAP) an ingest of ~9k distinct (member, actor) pairs overflows: settle
    reports CE_ERR_DEVICE, every later call fails the same way, and reset brings the core back
    (a small batch then equals the oracle)."""
    rng = random.Random(4242)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 9)
    big = {a: [[("Add", (a, v * 500 + i + 1), [v * 500 + i]) for i in range(500)] for v in range(2)]
           for a in actors}
    acts, clears, fa, fv = G.batch(big, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    os.environ["CE_DS_TEST_PAIR_CAP"] = "4096"
    try:
        core = new_core(ctx, "orswot", key)
        rc = core.ingest_ops(sealed, acts, fa, fv)[0]
        assert rc in (0, 65), rc        # 0: found later (the fold closes without a wait)
        assert core.settle() == 65      # CE_ERR_DEVICE
        assert core.settle() == 65      # sticky
        with pytest.raises(Exception):
            core.state_bytes()
        assert core.ingest_ops(sealed[:1], acts, fa[:1], fv[:1])[0] == 65
    finally:
        os.environ.pop("CE_DS_TEST_PAIR_CAP", None)
    core.reset()
    assert core.settle() == 0
    small = {a: [[("Add", (a, 1), [7])]] for a in actors[:3]}
    acts, clears, fa, fv = G.batch(small, "orswot", APP)
    oc = C.Core("orswot")
    assert check_ops(ctx, "orswot", key, core, oc, acts, clears, fa, fv) == 0
    core.close()


def test_scan_forms_equal(ctx):
    """the dot-set scans (ce_scan.hip) in their default two-launch form, the
    three-launch form (CE_SCAN_3PASS=1, otherwise only past 4096 tiles) give identical state
    bytes == the oracle, on an adversarial batch (the
    sorted adds' segmented max scan, ragged actor runs across 2048-item tiles; the per-file
    count scans over 4096 files).  The forms are chosen once per process, so each runs in its own
    child process (tests/scan_modes_worker.py)."""
    import hashlib
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    rng = random.Random(31337)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 256)
    files = G.adversarial_orswot(rng, actors, 16, 6, 5000)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    orc = oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0]
    want = "%d %s" % (orc, hashlib.sha256(oc.serialize()).hexdigest())
    outs = {}
    for mode, env in {"two": {}, "three": {"CE_SCAN_3PASS": "1"}}.items():
        e = dict(os.environ)
        e.pop("CE_SCAN_3PASS", None)
        e.pop("CE_HIPCUB_SCAN", None)
        e.update(env)
        r = subprocess.run([sys.executable, os.path.join(here, "scan_modes_worker.py")], env=e,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[mode] = r.stdout.strip().splitlines()[-1]
    assert outs["two"] == outs["three"] == want, outs


def _canonical_orswot(rng, actors, n_versions, ops_per_file, members, widths=(1, 2, 3, 5, 9), p_rm=0.2):
    """Op files whose ops are all the forms the open's decode proves: one-member Adds of the
    writer's own dots, removals with a one-entry clock {writer: an earlier counter}; counters and
    members drawn from every msgpack uint width (fixint, cc, cd, ce, cf)."""
    lim = {1: (0, 127), 2: (128, 255), 3: (256, 65535), 5: (65536, (1 << 32) - 1), 9: (1 << 32, (1 << 64) - 1)}
    files = {a: [] for a in actors}
    ctr = {a: 0 for a in actors}
    for _ in range(n_versions):
        for a in actors:
            ops = []
            for _ in range(ops_per_file):
                w = rng.choice(widths)
                lo, hi = lim[w]
                if ctr[a] and rng.random() < p_rm:
                    ops.append(("Rm", C.VClock({a: rng.randint(1, ctr[a])}), [rng.randrange(members)]))
                else:
                    ctr[a] = max(ctr[a] + 1, rng.randint(lo, hi))
                    mem = rng.randrange(members) if rng.random() < 0.5 else rng.randint(*lim[rng.choice(widths)])
                    ops.append(("Add", (a, ctr[a]), [mem]))
            files[a].append(ops)
    return files


@pytest.mark.parametrize("case", ["canonical", "well_formed", "adversarial", "large_files", "spurious_magic",
                                  "foreign_actor", "trailing", "bad_version", "tampered"])
def test_orswot_fused_decode_equals_lane_decode(ctx, case):
    """Orswot op files decoded inside the open (k_open_fold_v2's DS form: the plaintext stays in
    LDS, 16 lanes per file prove the canonical ops and write their rows) == the lane-per-file
    decode from HBM (CE_DS_FUSED_DECODE=0) == the oracle: statuses, return code and state bytes.
    The cases mix files the open proves with files it must hand to the lane decode: removals
    with several clock entries and several members (well_formed / adversarial), files past
    kDsFuseRegion (large_files), member values whose bytes spell an op's first word (a candidate
    the decode must drop), ops naming actors outside the table (foreign_actor: the emit's miss
    rounds), bytes after the Vec (ignored by from_slice), an unsupported data version and a
    flipped tag bit."""
    rng = random.Random(sum(map(ord, case)))
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 12)
    if case == "canonical":
        files = _canonical_orswot(rng, actors, 6, 24, 300)
    elif case == "well_formed":
        files = G.well_formed_orswot(rng, actors, 5, 20, 200, max_members=1)[0]
    elif case == "adversarial":
        files = gen("orswot", rng, actors, 5, 12, 200, True)
    elif case == "large_files":
        files = _canonical_orswot(rng, actors, 3, 60, 300)          # ~3.5 KiB: past the LDS region
        files.update(_canonical_orswot(rng, actors[:4], 3, 20, 300))
    elif case == "spurious_magic":
        files = _canonical_orswot(rng, actors, 4, 16, 300)
        a = actors[0]
        # ce members 0x81a34164 / 0x81a2526d: bytes 81 a3 41 64 / 81 a2 52 6d inside an op
        files[a][1][2] = ("Add", (a, 10 ** 9), [0x81A34164])
        files[a][2][3] = ("Add", (a, 10 ** 9 + 1), [0x81A2526D])
        files[a][3] = [op if op[0] == "Rm" else ("Add", op[1], [0x81A34164A3646F74]) for op in files[a][3]]
        # members ending in 81 a2 / 81 a3 right before the next op: two prefixes in one dword
        b = actors[1]
        files[b][0] = [op if op[0] == "Rm" else ("Add", op[1], [rng.choice([0x123481A2, 0x81A3, 0x81A2])])
                       for op in files[b][0]]
    elif case == "foreign_actor":
        files = _canonical_orswot(rng, actors, 4, 16, 300)
        stranger = rng.randbytes(16)
        files[actors[2]][1][0] = ("Add", (stranger, 5), [42])
        files[actors[3]][2][1] = ("Rm", C.VClock({stranger: 3}), [42])
    else:
        files = _canonical_orswot(rng, actors, 4, 16, 300)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    if case == "trailing":
        clears = [c + rng.randbytes(rng.randint(1, 90)) if i % 3 == 0 else c for i, c in enumerate(clears)]
    if case == "bad_version":
        clears[7] = bytes(16) + clears[7][16:]
    sealed = seal_files(ctx, key, clears)
    if case == "tampered":
        b = bytearray(sealed[5])
        b[-1] ^= 1
        sealed[5] = bytes(b)
    oc = C.Core("orswot")
    want = oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)
    got = {}
    for fused in (True, False):
        os.environ["CE_DS_FUSED_DECODE"] = "1" if fused else "0"
        try:
            core = new_core(ctx, "orswot", key)
            got[fused] = (core.ingest_ops(sealed, acts, fa, fv), core.state_bytes(), core.path_count("ds_fused_files"))
            core.close()
        finally:
            os.environ.pop("CE_DS_FUSED_DECODE", None)
    assert got[True][:2] == got[False][:2]
    assert got[True][0] == want and got[True][1] == oc.serialize()
    assert got[False][2] == 0
    n = len(sealed)
    if case in ("canonical", "trailing", "spurious_magic"):
        assert got[True][2] == n          # every file proven in the open
    elif case in ("bad_version", "tampered"):
        assert want[0] != 0
    elif case == "large_files":
        assert 0 < got[True][2] < n
    elif case in ("well_formed", "foreign_actor"):
        assert 0 < got[True][2] < n


def test_orswot_member_table_growth_then_compaction(ctx):
    """The primary member table grows past half full (ensure_pairs counts the members, rebuilds the
    tables from a collect of the live pairs) batch after batch; the collect's output counter stays
    zero between collects (k_ds_collect_max resets it; the member count uses another word), so
    every rebuild and the device serializer see exactly the live pairs == the oracle."""
    rng = random.Random(5150)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 16)
    files = G.well_formed_orswot(rng, actors, 6, 60, 40000, p_rm=0.1, max_members=3)[0]
    core, oc = new_core(ctx, "orswot", key), C.Core("orswot")
    import torch
    for lo in range(0, 6, 2):
        part = {a: files[a][: lo + 2] for a in files}
        acts, clears, fa, fv = G.batch(part, "orswot", APP, start={a: lo for a in files})
        assert check_ops(ctx, "orswot", key, core, oc, acts, clears, fa, fv) == 0
        want = oc.serialize()
        buf = torch.zeros(len(want) + 4096, dtype=torch.uint8, device="cuda:0")
        rc, n = core.state_bytes_device(buf.data_ptr(), buf.numel())
        assert rc == 0
        torch.cuda.synchronize()
        assert bytes(buf[:n].cpu().numpy().tobytes()) == want
    core.close()


def test_columns_export_merge_equals_state_merge(ctx):
    """The column form of the multi-GPU exchange through the C ABI: writer shards folded on
    separate cores, the others' states exported as columns into HBM and merged into the first in
    one k-way merge == merging their StateWrappers one by one == one core over every file == the
    oracle; a state with a deferred removal exports its deferred map with the columns."""
    import torch
    rng = random.Random(6060)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 12)
    files = G.well_formed_orswot(rng, actors, 4, 10, 500, p_rm=0.0)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    shards = []
    for r in range(4):
        idx = [i for i in range(len(fa)) if fa[i] % 4 == r]
        core = new_core(ctx, "orswot", key)
        assert core.ingest_ops([sealed[i] for i in idx], acts, [fa[i] for i in idx], [fv[i] for i in idx])[0] == 0
        shards.append(core)
    bufs, lens = [], []
    for core in shards[1:]:
        assert core.columns_ready()
        rc, n = core.export_columns_device(0, 0)
        assert rc == 64 and n == 1                  # the query form
        t = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
        rc, n = core.export_columns_device(t.data_ptr(), 64)
        assert rc == 64 and n > 64                  # too small: the needed length
        t = torch.zeros(n + 128, dtype=torch.uint8, device="cuda:0")
        rc, n2 = core.export_columns_device(t.data_ptr(), t.numel())
        assert rc == 0 and n2 == n
        bufs.append(t)
        lens.append(n)
    seq = new_core(ctx, "orswot", key)
    assert seq.merge_state(shards[0].state_bytes()) == 0
    for core in shards[1:]:
        assert seq.merge_state(core.state_bytes()) == 0
    assert shards[0].merge_columns_device([t.data_ptr() for t in bufs], lens) == 0
    assert shards[0].state_bytes() == seq.state_bytes() == oc.serialize()
    assert shards[0].path_count("columns_merge") == 1
    # not a column partial: refused, state unchanged
    bad = torch.zeros(256, dtype=torch.uint8, device="cuda:0")
    assert shards[1].merge_columns_device([bad.data_ptr()], [256]) == 12
    # a deferred removal travels in the columns' deferred section: either side may hold one
    dfiles = {acts[0]: [[("Rm", C.VClock({acts[1]: 99}), [7])]]}
    dacts, dclears, dfa, dfv = G.batch(dfiles, "orswot", APP, start={acts[0]: 0})
    d = new_core(ctx, "orswot", key)
    assert d.ingest_ops(seal_files(ctx, key, dclears), dacts, dfa, dfv)[0] == 0
    assert d.columns_ready()
    rc, n = d.export_columns_device(bufs[0].data_ptr(), bufs[0].numel())
    assert rc == 0 and n > 0
    dbuf = bufs[0][:n].clone()
    # a deferred section the device check refuses (an actor index past the partial's actors, then
    # removal offsets out of order): CE_ERR_DECODE, the receiver's state unchanged
    hb = dbuf.cpu().numpy().tobytes()
    np_, na_ = struct.unpack_from("<QI", hb, 8)
    dof = (32 + 32 * na_ + 20 * np_ + 7) & ~7
    n_rm, n_ent, n_mem = struct.unpack_from("<QQQ", hb, dof)
    assert (n_rm, n_ent, n_mem) == (1, 1, 1)
    act_off = dof + ((32 + 8 * (n_rm + 1) + 7) & ~7)
    before = shards[1].state_bytes()
    for off, val in ((act_off, na_ + 3), (dof + 36, 5)):
        bad = bytearray(hb)
        struct.pack_into("<I", bad, off, val)
        tb = torch.frombuffer(bytes(bad), dtype=torch.uint8).to("cuda:0")
        assert shards[1].merge_columns_device([tb.data_ptr()], [n]) == 12
        assert shards[1].state_bytes() == before
    seq2 = new_core(ctx, "orswot", key)
    assert seq2.merge_state(shards[1].state_bytes()) == 0 and seq2.merge_state(d.state_bytes()) == 0
    assert shards[1].merge_columns_device([dbuf.data_ptr()], [n]) == 0       # theirs deferred
    assert shards[1].state_bytes() == seq2.state_bytes()
    assert shards[1].path_count("columns_merge_deferred") == 1
    seq3 = new_core(ctx, "orswot", key)
    assert seq3.merge_state(d.state_bytes()) == 0 and seq3.merge_state(shards[2].state_bytes()) == 0
    assert d.merge_columns_device([bufs[1].data_ptr()], [lens[1]]) == 0       # ours deferred
    assert d.state_bytes() == seq3.state_bytes()
    for core in shards + [seq, seq2, seq3, d]:
        core.close()


@pytest.mark.parametrize("shape", ["writers", "overlap"])
def test_columns_merge_deferred_and_covered_removals(ctx, shape):
    """Column partials that hold deferred removals and removals covering each other's dots:
    well-formed histories whose removals carry the member's whole read context (crdts
    rm(member, read_ctx)).  "writers": writer shards, so a shard defers a removal that names
    another writer's dots; "overlap": every shard folds three consecutive writers, so the
    partials' clocks overlap and one partial's removals cover pairs another still holds (the
    kill side of the merge rule through k_cols_remap's remapped clocks).  One k-way merge of the
    exported columns == merging the StateWrappers one by one == one core over every file == the
    oracle (crdt-enc/src/lib.rs:457-465, Orswot::merge with other.deferred)."""
    import torch
    rng = random.Random(7171 if shape == "writers" else 7272)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 9)
    files = G.well_formed_orswot(rng, actors, 5, 8, 60, p_rm=0.35)[0]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    ns = 3
    shards = []
    for r in range(ns):
        if shape == "writers":
            ws = {a for a in range(len(acts)) if a % ns == r}
        else:
            ws = {(3 * r + j) % len(acts) for j in range(5)}
        idx = [i for i in range(len(fa)) if fa[i] in ws]
        core = new_core(ctx, "orswot", key)
        assert core.ingest_ops([sealed[i] for i in idx], acts, [fa[i] for i in idx], [fv[i] for i in idx])[0] == 0
        shards.append(core)
    seq = new_core(ctx, "orswot", key)
    for core in shards:
        assert seq.merge_state(core.state_bytes()) == 0
    bufs, lens = [], []
    for core in shards[1:]:
        rc, n = core.export_columns_device(0, 0)
        assert rc == 64 and n == 1
        t = torch.zeros(1 << 21, dtype=torch.uint8, device="cuda:0")
        rc, n = core.export_columns_device(t.data_ptr(), t.numel())
        assert rc == 0 and n > 0
        bufs.append(t)
        lens.append(n)
    assert shards[0].merge_columns_device([t.data_ptr() for t in bufs], lens) == 0
    got = shards[0].state_bytes()
    assert got == seq.state_bytes() == oc.serialize()
    assert shards[0].path_count("columns_merge") == 1
    # the workload exercises what it says: some partial held a deferred removal
    assert shards[0].path_count("columns_merge_deferred") == 1
    for core in shards + [seq]:
        core.close()


def test_orswot_writer_versions_after_table_growth(ctx):
    """Removal clocks naming more actors than the actor table holds (2,100 strangers, the writer
    shard of C3 with read-context removals): the decode's misses grow the table inside the
    ingest, and every writer's next_op_versions must still land on its own slot afterwards
    (lib.rs:537-538) -- the state, next versions included, == the oracle's."""
    rng = random.Random(8080)
    key = rng.randbytes(32)
    writers = G.actors_for(rng, 3)
    strangers = G.actors_for(rng, 2100)
    files = {}
    for i, w in enumerate(writers):
        files[w] = [[("Add", (w, v + 1), [100 * i + v]),
                     ("Rm", C.VClock({s: 5 for s in strangers[700 * i:700 * (i + 1)]}), [7])] for v in range(3)]
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    sealed = seal_files(ctx, key, clears)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], sealed, [acts[i] for i in fa], fv)[0] == 0
    core = new_core(ctx, "orswot", key)
    assert core.ingest_ops(sealed, acts, fa, fv)[0] == 0
    assert core.state_bytes() == oc.serialize()
    core.close()
