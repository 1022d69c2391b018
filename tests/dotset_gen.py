"""Synthetic Orswot<u64, Uuid> / MVReg<u64, Uuid> op histories for the dot-set parity tests.

well_formed_*: every actor writes its own dots (Dot{actor, counter} with counter = previous + 1,
crdts' `inc`), removals carry the read context of the member at generation time (crdts'
`Orswot::rm(member, ctx)`), so the result does not depend on how actors interleave -- the
property read_remote_ops's `buffered(16)` ordering relies on (crdt-enc/src/lib.rs:497-544).
adversarial_*: foreign-actor dots, repeated / decreasing counters, random removal clocks --
exercises the exact sequential semantics (skipped adds, deferred removals).
"""
import random

from oracle import crdts as C


def actors_for(rng, n):
    return sorted(rng.randbytes(16) for _ in range(n))


def well_formed_orswot(rng, actors, n_versions, ops_per_file, n_members, p_rm=0.2,
                       max_members=2):
    """-> {actor: [ops of version 0, ops of version 1, ...]} plus the generating replica."""
    truth = C.Orswot()
    files = {a: [] for a in actors}
    counters = {a: 0 for a in actors}
    live = []
    for _ in range(n_versions):
        order = list(actors)
        rng.shuffle(order)
        for a in order:
            ops = []
            for _ in range(ops_per_file):
                if live and rng.random() < p_rm:
                    m = live[rng.randrange(len(live))]
                    e = truth.entries.get(m)
                    if e is None:
                        continue
                    op = ("Rm", e.clone(), [m])
                else:
                    counters[a] += 1
                    k = rng.randint(0, max_members) if max_members > 1 else 1
                    ms = [rng.randrange(n_members) for _ in range(k)]
                    op = ("Add", (a, counters[a]), ms)
                    live.extend(ms)
                truth.apply(op)
                ops.append(op)
            files[a].append(ops)
    return files, truth


def adversarial_orswot(rng, actors, n_versions, ops_per_file, n_members):
    files = {a: [] for a in actors}
    for a in actors:
        for _ in range(n_versions):
            ops = []
            for _ in range(ops_per_file):
                r = rng.random()
                if r < 0.6:
                    act = a if rng.random() < 0.7 else rng.choice(actors)
                    ops.append(("Add", (act, rng.randint(1, 12)),
                                [rng.randrange(n_members) for _ in range(rng.randint(0, 3))]))
                else:
                    clock = C.VClock({rng.choice(actors): rng.randint(1, 12)
                                      for _ in range(rng.randint(0, 3))})
                    ops.append(("Rm", clock, [rng.randrange(n_members) for _ in range(rng.randint(0, 3))]))
            files[a].append(ops)
    return files


def well_formed_mvreg(rng, actors, n_versions, ops_per_file, p_stale=0.6):
    """Puts whose clocks are the writer's view (the shared clock, sometimes a stale copy) + inc."""
    seen = C.VClock()
    stale = []
    files = {a: [] for a in actors}
    for _ in range(n_versions):
        order = list(actors)
        rng.shuffle(order)
        for a in order:
            ops = []
            for _ in range(ops_per_file):
                base = rng.choice(stale) if stale and rng.random() < p_stale else seen
                clock = base.clone()
                clock.dots[a] = seen.get(a) + 1
                seen.merge(clock)
                stale.append(clock.clone())
                if len(stale) > 16:
                    stale.pop(0)
                ops.append(("Put", clock, rng.getrandbits(rng.choice([7, 16, 40, 64]))))
            files[a].append(ops)
    return files


def adversarial_mvreg(rng, actors, n_versions, ops_per_file):
    files = {a: [] for a in actors}
    for a in actors:
        for _ in range(n_versions):
            ops = []
            for _ in range(ops_per_file):
                clock = C.VClock({rng.choice(actors): rng.randint(1, 4) for _ in range(rng.randint(0, 3))})
                ops.append(("Put", clock, rng.randrange(1000)))
            files[a].append(ops)
    return files


def batch(files, kind, data_version, start=None):
    """load_ops order: per actor (sorted), versions ascending from start[a] (default 0)."""
    enc = C.enc_orswot_ops if kind == "orswot" else C.enc_mvreg_ops
    clears, fa, fv, actors = [], [], [], sorted(files)
    for i, a in enumerate(actors):
        s = (start or {}).get(a, 0)
        for v, ops in enumerate(files[a]):
            if v < s:
                continue
            clears.append(data_version + enc(ops))
            fa.append(i)
            fv.append(v)
    return actors, clears, fa, fv
