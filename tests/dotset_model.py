"""Columnar model of the GPU dot-set fold (crdt-enc_amd/csrc/ce_dotset.hip), in plain Python.

TEST INFRASTRUCTURE: it states the data-parallel formulation the kernels implement, so that
tests/test_dotset_model.py can check it against the sequential oracle (oracle/crdts.py) on
adversarial op streams, independently of the GPU.

Orswot state = clock C[a], entry values cur[(m, a)] (absent = 0), deferred removals D.
Ingesting ops (batch order = application order, lib.rs:516-544):
  applied(add k)  = c_k > max(C0[a_k], max{c_j : j < k, a_j = a_k})      (segmented prefix max)
  add[(m, a)]     = max c_k over applied adds k of actor a that list m
  kill[(m, a)]    = max R[a] over removals (D0 and the batch) that list m
  cur'            = v = max(cur, add); 0 if v <= kill
  C1              = max(C0, every add dot);  D1 = {R in D0 + batch : not R <= C1} (members unioned)
Merging a state O (Orswot::merge): per (m, a) with s = cur, t = O's value,
  r = max(s if s == t, s if s > O.C[a], t if t > C[a]); then kills by D + O.D; C = max; D filtered.
MVReg: survivors = maximal put clocks; among equal clocks the latest applied op (merge: the
earliest value) wins; survivors keep their insertion order.
"""
from oracle import crdts as C


def orswot_to_cols(o):
    cur = {}
    for m, vc in o.entries.items():
        for a, c in vc.dots.items():
            cur[(m, a)] = c
    d = [(dict(k), set(ms)) for k, ms in o.deferred.items()]
    return dict(o.clock.dots), cur, d


def cols_to_orswot(clock, cur, d):
    o = C.Orswot()
    o.clock = C.VClock(clock)
    for (m, a), v in cur.items():
        if v:
            o.entries.setdefault(m, C.VClock()).dots[a] = v
    for r, ms in d:
        o.deferred.setdefault(C.VClock(r).key(), set()).update(ms)
    return o


def _le(r, clock):
    return all(clock.get(a, 0) >= c for a, c in r.items())


def _kill(cur, rms):
    kill = {}
    for r, ms in rms:
        for m in ms:
            for a, c in r.items():
                if (m, a) in cur:
                    kill[(m, a)] = max(kill.get((m, a), 0), c)
    return {k: (0 if v <= kill.get(k, 0) else v) for k, v in cur.items()}


def _defer(rms, clock):
    out = {}
    for r, ms in rms:
        if not _le(r, clock):
            out.setdefault(tuple(sorted(r.items())), set()).update(ms)
    return [(dict(k), ms) for k, ms in out.items()]


def orswot_ingest(clock, cur, d, ops):
    clock1 = dict(clock)
    pm = {}
    add = {}
    rms = list(d)
    for op in ops:
        if op[0] == "Add":
            _, (a, c), ms = op
            prev = max(clock.get(a, 0), pm.get(a, 0))
            pm[a] = max(pm.get(a, 0), c)
            clock1[a] = max(clock1.get(a, 0), c)
            if c > prev:
                for m in ms:
                    add[(m, a)] = max(add.get((m, a), 0), c)
        else:
            rms.append((dict(op[1].dots), set(op[2])))
    merged = dict(cur)
    for k, v in add.items():
        merged[k] = max(merged.get(k, 0), v)
    return clock1, _kill(merged, rms), _defer(rms, clock1)


def orswot_merge(clock, cur, d, oclock, ocur, od):
    keys = set(cur) | set(ocur)
    r = {}
    for k in keys:
        s, t = cur.get(k, 0), ocur.get(k, 0)
        a = k[1]
        v = max(s if s == t else 0, s if s > oclock.get(a, 0) else 0, t if t > clock.get(a, 0) else 0)
        r[k] = v
    rms = list(d) + list(od)
    c = dict(clock)
    for a, x in oclock.items():
        c[a] = max(c.get(a, 0), x)
    return c, _kill(r, rms), _defer(rms, c)


def mvreg_survivors(cands, later_wins):
    """cands: list of (VClock, val) in insertion order -> survivors in insertion order."""
    alive = [i for i, (c, _) in enumerate(cands) if not c.is_empty()]
    out = []
    while alive:
        def key(i):
            return (sum(cands[i][0].dots.values()), i if later_wins else -i)
        w = max(alive, key=key)
        out.append(w)
        wc = cands[w][0]
        alive = [i for i in alive if not cands[i][0].le(wc)]
    return [cands[i] for i in sorted(out)]
