"""The C Orswot restatement (oracle/ce_oracle.c oc_compact_orswot_best, the C3 CPU baseline)
against the Python restatement (oracle/crdts.py Core) on the dot-set histories the GPU parity
tests use: state files (with deferred removals) merged, then op files folded, canonical bytes
compared; plus the reject paths (tampered tag, decode error, version gap, bad state).

Both are restatements of crdts 7 (parity with crdts itself is unpinned); this test
pins the C one to the Python one, which the GPU suite pins the product to.
"""
import random

import msgpack
import numpy as np
import pytest

import dotset_gen as G
import oracle
from oracle import crdts as C

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = C.CORE_VERSION


def seal(key, clears):
    return [CORE + oracle.cryptor_encrypt(key, random.Random(len(c)).randbytes(24), c)[1] for c in clears]


def run_c(key, states, files, acts, fa, fv, threads=4):
    blob = b"".join(files) or b"\0"
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    for i, f in enumerate(files):
        offs[i + 1] = offs[i] + len(f)
    actor = np.frombuffer(b"".join(acts[i] for i in fa) or bytes(16), dtype=np.uint8).reshape(-1, 16)
    ver = np.array(list(fv) or [0], dtype=np.uint64)
    err, sw, _, _ = oracle.compact_orswot_best(key, APP, states, blob, offs, actor, ver, threads)
    return err, sw


def run_py(key, states, files, acts, fa, fv):
    oc = C.Core("orswot")
    rc = oc.read_remote_states(key, [APP], states)[0] if states else 0
    if rc:
        return rc, None
    rc = oc.read_remote_ops(key, [APP], files, [acts[i] for i in fa], fv)[0]
    return rc, oc.serialize()


def replica_states(rng, key, actors, n, adversarial):
    out = []
    for _ in range(n):
        part = C.Core("orswot")
        if adversarial:
            hist = G.adversarial_orswot(rng, actors, 2, 5, 20)
        else:
            hist = G.well_formed_orswot(rng, actors, 2, 5, 20)[0]
        acts, clears, fa, fv = G.batch(hist, "orswot", APP)
        assert part.read_remote_ops(key, [APP], seal(key, clears), [acts[i] for i in fa], fv)[0] == 0
        out.append(part.serialize())
    return seal(key, [APP + s for s in out])


@pytest.mark.parametrize("seed", range(8))
def test_states_and_ops_match_python(seed):
    rng = random.Random(900 + seed)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, rng.randint(2, 7))
    adversarial = seed % 2 == 1
    states = replica_states(rng, key, actors, rng.randint(0, 3), adversarial)
    hist = (G.adversarial_orswot(rng, actors, 4, 6, 30) if adversarial
            else G.well_formed_orswot(rng, actors, 4, 6, 30)[0])
    acts, clears, fa, fv = G.batch(hist, "orswot", APP)
    files = seal(key, clears)
    want = run_py(key, states, files, acts, fa, fv)
    assert want[0] == 0
    assert run_c(key, states, files, acts, fa, fv) == want
    assert run_c(key, states, files, acts, fa, fv, threads=1) == want


def test_larger_history_matches_python():
    """table growth (entries, actors), thousands of ops, many deferred removals"""
    rng = random.Random(31)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 40)
    states = replica_states(rng, key, actors, 2, True)
    hist = G.adversarial_orswot(rng, actors, 6, 10, 2000)
    acts, clears, fa, fv = G.batch(hist, "orswot", APP)
    files = seal(key, clears)
    want = run_py(key, states, files, acts, fa, fv)
    assert want[0] == 0 and b"deferred" in want[1]
    assert run_c(key, states, files, acts, fa, fv, threads=8) == want


def _noncanonical(ops, rng):
    out = []
    for op in ops:
        if op[0] == "Add":
            _, (a, c), ms = op
            out.append(rng.choice([{0: [[a, c], ms]},
                                   {"Add": {"zz": [1], "members": ms, "dot": {"counter": c, "actor": a}}}]))
        else:
            _, clock, ms = op
            dots = list(clock.dots.items())
            rng.shuffle(dots)
            out.append({1: {"members": ms, "clock": [dict(dots)]}})
    return msgpack.packb(out, use_bin_type=True)


def test_accepts_rmp_forms():
    rng = random.Random(12)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 4)
    hist = G.adversarial_orswot(rng, actors, 3, 6, 12)
    acts = sorted(hist)
    clears, fa, fv = [], [], []
    for i, a in enumerate(acts):
        for v, ops in enumerate(hist[a]):
            clears.append(APP + _noncanonical(ops, rng))
            fa.append(i)
            fv.append(v)
    files = seal(key, clears)
    want = run_py(key, [], files, acts, fa, fv)
    assert want[0] == 0
    assert run_c(key, [], files, acts, fa, fv) == want


def test_reject_paths():
    rng = random.Random(4)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 3)
    hist = G.well_formed_orswot(rng, actors, 4, 3, 10)[0]
    acts, clears, fa, fv = G.batch(hist, "orswot", APP)
    files = seal(key, clears)
    bad = list(files)
    b = bytearray(bad[5])
    b[-1] ^= 1
    bad[5] = bytes(b)
    assert run_c(key, [], bad, acts, fa, fv)[0] == run_py(key, [], bad, acts, fa, fv)[0] == 9
    bad = list(clears)
    bad[2] = APP + msgpack.packb({"x": 1})
    bad = seal(key, bad)
    assert run_c(key, [], bad, acts, fa, fv)[0] == run_py(key, [], bad, acts, fa, fv)[0] == 12
    keep = [i for i in range(len(fa)) if not (fa[i] == 1 and fv[i] == 1)]
    args = ([files[i] for i in keep], acts, [fa[i] for i in keep], [fv[i] for i in keep])
    assert run_c(key, [], *args)[0] == run_py(key, [], *args)[0] == 13
    st = seal(key, [APP + msgpack.packb({"next_op_versions": {"dots": {}}})])
    assert run_c(key, st, files, acts, fa, fv)[0] == run_py(key, st, files, acts, fa, fv)[0] == 12
    # empty batch: the empty StateWrapper
    assert run_c(key, [], [], [], [], []) == (0, C.Core("orswot").serialize())
