"""Sequential CPU restatement of the dot-set CRDTs on crdt-enc's fold path (Orswot, MVReg) and of
`read_remote_states` / `read_remote_ops` for them.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and never by crdt-enc_amd/), as the checker of the
GPU fold in crdt-enc_amd/csrc/ce_dotset.{cpp,hip}.

What it follows
  * crdt-enc/src/lib.rs:401-469 read_remote_states: open every state file, then
    `state.merge(sw.state)` + `next_op_versions.merge(..)` per file (lib.rs:458-466); any failure
    rejects the batch before the fold.
  * crdt-enc/src/lib.rs:471-547 read_remote_ops: open + decode every file first (lib.rs:497-514,
    `.buffered(16)` keeps load_ops order), then per file the version gate (lib.rs:519-531),
    `state.apply(op)` for each op (lib.rs:534-535) and next_op_versions.inc/apply (lib.rs:537-538).
  * crdts = "7" (crdt-enc/Cargo.toml; third-party, not vendored here, patch version unpinned:
    SURVEY.md F2): VClock, Orswot<M, A>, MVReg<V, A> restated from their published source
    (SURVEY.md Appendix B).  The methods below keep crdts' names (apply, apply_rm,
    apply_deferred, merge, reset_remove, intersection, clone_without) and statement order.

Parity status: the reference's own tests pin nothing about these types, so the
Orswot/MVReg semantics and the enum wire form ({"Add": {..}} externally tagged, SURVEY.md
Appendix A) are *parity unpinned*.  Orswot/MVReg hold HashMaps/HashSets whose iteration order is
random in the reference, so states are compared in the canonical serialization
written here: entries sorted by member, deferred sorted by the msgpack bytes of the clock, members
sorted.
"""
import msgpack

import oracle as _oc

CORE_VERSION = bytes.fromhex("e834d789101b463498239de990a9051f")  # crdt-enc/src/lib.rs:26


# ------------------------------------------------------------------------------------------
# VClock<A> (crdts 7 vclock.rs); dots: actor(bytes16) -> counter(u64 > 0)
# ------------------------------------------------------------------------------------------
class VClock:
    __slots__ = ("dots",)

    def __init__(self, dots=None):
        self.dots = dict(dots or {})

    def get(self, a):
        return self.dots.get(a, 0)

    def apply(self, actor, counter):
        if self.get(actor) < counter:
            self.dots[actor] = counter

    def merge(self, other):
        for a, c in other.dots.items():
            self.apply(a, c)

    def reset_remove(self, other):
        for a, c in other.dots.items():
            if c >= self.get(a):
                self.dots.pop(a, None)

    def clone_without(self, base):
        v = VClock(self.dots)
        v.reset_remove(base)
        return v

    @staticmethod
    def intersection(left, right):
        return VClock({a: c for a, c in left.dots.items() if right.get(a) == c})

    def is_empty(self):
        return not self.dots

    def le(self, other):  # self <= other (PartialOrd: every dot of self is covered)
        return all(other.get(a) >= c for a, c in self.dots.items())

    def ge(self, other):
        return other.le(self)

    def key(self):
        return tuple(sorted(self.dots.items()))

    def __eq__(self, other):
        return self.dots == other.dots

    def lt(self, other):
        return self != other and self.le(other)

    def clone(self):
        return VClock(self.dots)


# ------------------------------------------------------------------------------------------
# Orswot<M, A> (crdts 7 orswot.rs)
# ------------------------------------------------------------------------------------------
class Orswot:
    def __init__(self):
        self.clock = VClock()
        self.entries = {}     # member -> VClock
        self.deferred = {}    # VClock.key() -> set(members)

    # CmRDT::apply
    def apply(self, op):
        kind = op[0]
        if kind == "Add":
            _, (actor, counter), members = op
            if self.clock.get(actor) >= counter:
                return  # already seen
            for m in members:
                self.entries.setdefault(m, VClock()).apply(actor, counter)
            self.clock.apply(actor, counter)
            self.apply_deferred()
        else:
            _, clock, members = op
            self.apply_rm(set(members), clock)

    def apply_rm(self, members, clock):
        for m in members:
            e = self.entries.get(m)
            if e is not None:
                e.reset_remove(clock)
                if e.is_empty():
                    del self.entries[m]
        if not clock.le(self.clock):
            self.deferred.setdefault(clock.key(), set()).update(members)

    def apply_deferred(self):
        deferred, self.deferred = self.deferred, {}
        for k, members in deferred.items():
            self.apply_rm(members, VClock(dict(k)))

    # CvRDT::merge
    def merge(self, other):
        kept = {}
        for m, clock in self.entries.items():
            if m not in other.entries:
                if other.clock.ge(clock):
                    continue  # other has seen it and dropped it
                clock = clock.clone()
                clock.reset_remove(other.clock)
                kept[m] = clock
            else:
                kept[m] = clock
        self.entries = kept
        for m, clock in other.entries.items():
            ours = self.entries.get(m)
            if ours is not None:
                common = VClock.intersection(clock, ours)
                common.merge(clock.clone_without(self.clock))
                common.merge(ours.clone_without(other.clock))
                if common.is_empty():
                    del self.entries[m]
                else:
                    self.entries[m] = common
            else:
                if self.clock.ge(clock):
                    continue  # seen and dropped
                c = clock.clone()
                c.reset_remove(self.clock)
                self.entries[m] = c
        for k, members in other.deferred.items():
            self.apply_rm(set(members), VClock(dict(k)))
        self.clock.merge(other.clock)
        self.apply_deferred()


# ------------------------------------------------------------------------------------------
# MVReg<V, A> (crdts 7 mvreg.rs); vals: list of (VClock, V) in Vec order
# ------------------------------------------------------------------------------------------
class MVReg:
    def __init__(self):
        self.vals = []

    def apply(self, op):
        _, clock, val = op
        if clock.is_empty():
            return
        # retain values concurrent with or greater than the op clock
        self.vals = [(c, v) for (c, v) in self.vals if not c.le(clock)]
        if any(clock.lt(c) for (c, _) in self.vals):
            return  # already seen
        self.vals.append((clock, val))

    def merge(self, other):
        self.vals = [(c, v) for (c, v) in self.vals if not any(c.lt(oc) for (oc, _) in other.vals)]
        add = [(c, v) for (c, v) in other.vals
               if not any(c.lt(sc) for (sc, _) in self.vals) and all(c != sc for (sc, _) in self.vals)]
        self.vals.extend(add)


# ------------------------------------------------------------------------------------------
# msgpack: decode (rmp-serde from_slice forms used by the tests) and canonical encode
# ------------------------------------------------------------------------------------------
class DecodeError(Exception):
    pass


class _Map(list):
    """A msgpack map as its list of (key, value) pairs (keys may be maps: Orswot.deferred)."""


def _unpack(b):
    """first value of b; bytes after it are ignored (rmp_serde::from_slice reads one value)"""
    try:
        u = msgpack.Unpacker(raw=False, strict_map_key=False, use_list=True,
                             object_pairs_hook=_Map, max_buffer_size=max(len(b), 1 << 20))
        u.feed(b)
        return u.unpack()
    except Exception as e:  # noqa: BLE001 -- any msgpack error is a decode error
        raise DecodeError(str(e))


def _struct(obj, names):
    """derive(Deserialize) struct: map keyed by field name or index (unknown keys ignored,
    duplicates rejected) or an array of exactly len(names)."""
    if isinstance(obj, _Map):
        out = [None] * len(names)
        seen = set()
        for k, v in obj:
            if isinstance(k, (bytes, str)):
                k = k.decode("latin-1") if isinstance(k, bytes) else k
                f = names.index(k) if k in names else None
            elif isinstance(k, int) and not isinstance(k, bool) and k >= 0:
                f = k if k < len(names) else None
            else:
                raise DecodeError("field key")
            if f is None:
                continue
            if f in seen:
                raise DecodeError("duplicate field")
            seen.add(f)
            out[f] = v
        if len(seen) != len(names):
            raise DecodeError("missing field")
        return out
    if isinstance(obj, list):
        if len(obj) != len(names):
            raise DecodeError("struct arity")
        return list(obj)
    raise DecodeError("struct form")


def _uuid(x):
    if not isinstance(x, (bytes, bytearray)) or len(x) != 16:
        raise DecodeError("uuid")
    return bytes(x)


def _u64(x):
    if not isinstance(x, int) or isinstance(x, bool) or x < 0 or x >= 1 << 64:
        raise DecodeError("u64")
    return x


def _pairs(x):
    if not isinstance(x, _Map):
        raise DecodeError("map")
    return list(x)


def _seq(x):
    if not isinstance(x, list) or isinstance(x, _Map):
        raise DecodeError("seq")
    return x


def dec_vclock(obj):
    """VClock {dots: BTreeMap<Uuid, u64>}: a later duplicate key overwrites an earlier one."""
    (dots,) = _struct(obj, ["dots"])
    v = VClock()
    for a, c in _pairs(dots):
        v.dots[_uuid(a)] = _u64(c)
    return v


def _enum(obj, variants):
    """externally tagged enum: map of one entry {variant name | index: body}"""
    p = _pairs(obj)
    if len(p) != 1:
        raise DecodeError("enum")
    k, body = p[0]
    if isinstance(k, bytes):
        k = k.decode("latin-1")
    if isinstance(k, int) and not isinstance(k, bool) and 0 <= k < len(variants):
        k = variants[k]
    if k not in variants:
        raise DecodeError("variant")
    return k, body


def dec_orswot_op(obj):
    k, body = _enum(obj, ["Add", "Rm"])
    if k == "Add":
        dot, members = _struct(body, ["dot", "members"])
        actor, counter = _struct(dot, ["actor", "counter"])
        return ("Add", (_uuid(actor), _u64(counter)), [_u64(m) for m in _seq(members)])
    clock, members = _struct(body, ["clock", "members"])
    return ("Rm", dec_vclock(clock), [_u64(m) for m in _seq(members)])


def dec_mvreg_op(obj):
    k, body = _enum(obj, ["Put"])
    clock, val = _struct(body, ["clock", "val"])
    return ("Put", dec_vclock(clock), _u64(val))


def dec_ops(kind, b):
    obj = _seq(_unpack(b))
    f = dec_orswot_op if kind == "orswot" else dec_mvreg_op
    return [f(o) for o in obj]


def dec_state(kind, b):
    """StateWrapper<S> {next_op_versions, state} -> (VClock, S)"""
    nov, st = _struct(_unpack(b), ["next_op_versions", "state"])
    nov = dec_vclock(nov)
    if kind == "orswot":
        o = Orswot()
        clock, entries, deferred = _struct(st, ["clock", "entries", "deferred"])
        o.clock = dec_vclock(clock)
        for m, c in _pairs(entries):
            o.entries[_u64(m)] = dec_vclock(c)
        for k, ms in _pairs(deferred):
            o.deferred.setdefault(dec_vclock(k).key(), set()).update(_u64(m) for m in _seq(ms))
        return nov, o
    r = MVReg()
    (vals,) = _struct(st, ["vals"])
    for pair in _seq(vals):
        c, v = _seq(pair)
        r.vals.append((dec_vclock(c), _u64(v)))
    return nov, r


class Wr:
    def __init__(self):
        self.b = bytearray()

    def uint(self, v):
        b = self.b
        if v <= 0x7f:
            b.append(v)
        elif v <= 0xff:
            b += bytes([0xcc, v])
        elif v <= 0xffff:
            b += b"\xcd" + v.to_bytes(2, "big")
        elif v <= 0xffffffff:
            b += b"\xce" + v.to_bytes(4, "big")
        else:
            b += b"\xcf" + v.to_bytes(8, "big")

    def str(self, s):
        s = s.encode()
        self.b += bytes([0xa0 | len(s)]) + s

    def bin(self, d):
        self.b += bytes([0xc4, len(d)]) + d

    def hdr(self, n, fix, m16, m32):
        if n <= 15:
            self.b.append(fix | n)
        elif n <= 0xffff:
            self.b += bytes([m16]) + n.to_bytes(2, "big")
        else:
            self.b += bytes([m32]) + n.to_bytes(4, "big")

    def map(self, n):
        self.hdr(n, 0x80, 0xde, 0xdf)

    def arr(self, n):
        self.hdr(n, 0x90, 0xdc, 0xdd)

    def vclock(self, v):
        self.map(1)
        self.str("dots")
        self.map(len(v.dots))
        for a in sorted(v.dots):
            self.bin(a)
            self.uint(v.dots[a])


def vclock_bytes(v):
    w = Wr()
    w.vclock(v)
    return bytes(w.b)


def serialize(kind, nov, st):
    """Canonical to_vec_named(StateWrapper<S>) (lib.rs:336, 739-743)."""
    w = Wr()
    w.map(2)
    w.str("next_op_versions")
    w.vclock(nov)
    w.str("state")
    if kind == "orswot":
        w.map(3)
        w.str("clock")
        w.vclock(st.clock)
        w.str("entries")
        w.map(len(st.entries))
        for m in sorted(st.entries):
            w.uint(m)
            w.vclock(st.entries[m])
        w.str("deferred")
        items = sorted(((vclock_bytes(VClock(dict(k))), sorted(ms)) for k, ms in st.deferred.items()))
        w.map(len(items))
        for kb, ms in items:
            w.b += kb
            w.arr(len(ms))
            for m in ms:
                w.uint(m)
    else:
        w.map(1)
        w.str("vals")
        w.arr(len(st.vals))
        for c, v in st.vals:
            w.arr(2)
            w.vclock(c)
            w.uint(v)
    return bytes(w.b)


def enc_orswot_ops(ops):
    """rmp-serde to_vec_named(Vec<orswot::Op<u64, Uuid>>), enums externally tagged."""
    w = Wr()
    w.arr(len(ops))
    for op in ops:
        w.map(1)
        if op[0] == "Add":
            _, (a, c), members = op
            w.str("Add")
            w.map(2)
            w.str("dot")
            w.map(2)
            w.str("actor")
            w.bin(a)
            w.str("counter")
            w.uint(c)
        else:
            _, clock, members = op
            w.str("Rm")
            w.map(2)
            w.str("clock")
            w.vclock(clock)
        w.str("members")
        w.arr(len(members))
        for m in members:
            w.uint(m)
    return bytes(w.b)


def enc_mvreg_ops(ops):
    w = Wr()
    w.arr(len(ops))
    for _, clock, val in ops:
        w.map(1)
        w.str("Put")
        w.map(2)
        w.str("clock")
        w.vclock(clock)
        w.str("val")
        w.uint(val)
    return bytes(w.b)


# ------------------------------------------------------------------------------------------
# Core restatement (StateWrapper<S> fold) for S in {Orswot<u64, Uuid>, MVReg<u64, Uuid>}
# ------------------------------------------------------------------------------------------
def open_file(key, supported, f):
    """lib.rs:435-447 / 501-507 check order -> (status, clear text after the data version)."""
    if len(f) < 16:
        return 1, None
    if f[:16] != CORE_VERSION:
        return 2, None
    st, pt = _oc.cryptor_decrypt(key, f[16:])
    if st:
        return st, None
    if len(pt) < 16:
        return 10, None
    if pt[:16] not in supported:
        return 11, None
    return 0, pt[16:]


class Core:
    def __init__(self, kind):
        assert kind in ("orswot", "mvreg")
        self.kind = kind
        self.nov = VClock()
        self.state = Orswot() if kind == "orswot" else MVReg()

    def serialize(self):
        return serialize(self.kind, self.nov, self.state)

    def read_remote_ops(self, key, supported, files, actors, versions):
        status, decoded, first = [], [], 0
        for f in files:
            st, pt = open_file(key, supported, f)
            ops = None
            if st == 0:
                try:
                    ops = dec_ops(self.kind, pt)
                except DecodeError:
                    st = 12
            status.append(st)
            decoded.append(ops)
            if st and not first:
                first = st
        if first:
            return first, status
        for i, ops in enumerate(decoded):
            a, v = actors[i], versions[i]
            expected = self.nov.get(a)
            if v < expected:
                continue
            if expected < v:
                status[i] = 13
                return 13, status
            for op in ops:
                self.state.apply(op)
            self.nov.apply(a, expected + 1)
        return 0, status

    def read_remote_states(self, key, supported, files):
        status, decoded, first = [], [], 0
        for f in files:
            st, pt = open_file(key, supported, f)
            sw = None
            if st == 0:
                try:
                    sw = dec_state(self.kind, pt)
                except (DecodeError, ValueError, TypeError):
                    st = 12
            status.append(st)
            decoded.append(sw)
            if st and not first:
                first = st
        if first:
            return first, status
        for nov, s in decoded:
            self.state.merge(s)
            self.nov.merge(nov)
        return 0, status
