"""The columnar (data-parallel) formulation of the Orswot/MVReg fold that the GPU kernels use
(tests/dotset_model.py) equals the sequential crdts restatement (oracle/crdts.py) -- CPU only."""
import random

import pytest

from oracle import crdts as C
import dotset_gen as G
import dotset_model as M


def _seq_apply(kind, files):
    s = C.Orswot() if kind == "orswot" else C.MVReg()
    for a in sorted(files):
        for ops in files[a]:
            for op in ops:
                s.apply(op)
    return s


def _ops(files):
    return [op for a in sorted(files) for ops in files[a] for op in ops]


@pytest.mark.parametrize("seed", range(12))
def test_orswot_ingest_model(seed):
    rng = random.Random(seed)
    actors = G.actors_for(rng, 5)
    gen = G.adversarial_orswot if seed % 2 else (lambda *a: G.well_formed_orswot(*a)[0])
    f0 = gen(rng, actors, 3, 5, 12)
    f1 = gen(rng, actors, 3, 5, 12)
    seq = _seq_apply("orswot", f0)
    clock, cur, d = M.orswot_to_cols(seq)
    for a in sorted(f1):
        for ops in f1[a]:
            for op in ops:
                seq.apply(op)
    clock, cur, d = M.orswot_ingest(clock, cur, d, _ops(f1))
    got = M.cols_to_orswot(clock, cur, d)
    nov = C.VClock()
    assert C.serialize("orswot", nov, got) == C.serialize("orswot", nov, seq)


@pytest.mark.parametrize("seed", range(12))
def test_orswot_merge_model(seed):
    rng = random.Random(100 + seed)
    actors = G.actors_for(rng, 5)
    gen = G.adversarial_orswot if seed % 2 else (lambda *a: G.well_formed_orswot(*a)[0])
    parts = [_seq_apply("orswot", gen(rng, actors, 2, 5, 10)) for _ in range(3)]
    seq = C.Orswot()
    cols = ({}, {}, [])
    for p in parts:
        seq.merge(p)
        cols = M.orswot_merge(*cols, *M.orswot_to_cols(p))
    nov = C.VClock()
    assert C.serialize("orswot", nov, M.cols_to_orswot(*cols)) == C.serialize("orswot", nov, seq)


@pytest.mark.parametrize("seed", range(12))
def test_mvreg_model(seed):
    rng = random.Random(200 + seed)
    actors = G.actors_for(rng, 4)
    gen = G.adversarial_mvreg if seed % 2 else G.well_formed_mvreg
    f0, f1 = gen(rng, actors, 3, 4), gen(rng, actors, 3, 4)
    seq = _seq_apply("mvreg", f0)
    base = list(seq.vals)
    for op in _ops(f1):
        seq.apply(op)
    got = M.mvreg_survivors(base + [(op[1], op[2]) for op in _ops(f1)], later_wins=True)
    assert [(c.dots, v) for c, v in got] == [(c.dots, v) for c, v in seq.vals]
    # merge: ties go to self (the earlier value)
    other = _seq_apply("mvreg", gen(rng, actors, 2, 4))
    m = C.MVReg()
    m.vals = list(seq.vals)
    m.merge(other)
    got = M.mvreg_survivors(list(seq.vals) + list(other.vals), later_wins=False)
    assert [(c.dots, v) for c, v in got] == [(c.dots, v) for c, v in m.vals]
