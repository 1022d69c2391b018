"""CPU restatement of the key path in front of the hot path: remote meta -> the key cryptor's
register -> Keys -> Keys::latest_key.

TEST INFRASTRUCTURE ONLY (tests/ and tests/golden/make_keys_golden.py import it; the product's
counterpart is crdt-enc_amd/csrc/ce_keys.cpp).

What it follows
  * crdt-enc/src/key_cryptor.rs:35-52 Keys { latest_key_id: MVReg<Uuid, Uuid>,
    keys: Orswot<Key, Uuid> }, Keys::merge; :59-70 latest_key (min id among the register's
    values, panic when an id has no key); :72-82 insert_latest_key; :85-139 Key (Eq/Hash/Ord
    by id only).
  * crdt-enc/src/lib.rs:553-612 read_remote_meta_ (RemoteMeta files merged), :647-664
    store_remote_meta (VersionBytes(CURRENT_VERSION, to_vec_named(RemoteMeta))), :752-764
    RemoteMeta { storage, cryptor, key_cryptor: MVReg<VersionBytes, Uuid> }.
  * crdt-enc-gpgme/src/lib.rs:79-105 set_remote_meta -> decode_version_bytes_mvreg_custom_phf
    (crdt-enc/src/utils/mod.rs:94-126): every register value is VersionBytes(gpgme version,
    to_vec_named(Keys)) (the key encryption is a TODO pass-through), Keys merged.
  * crdts 7 MVReg / Orswot from oracle/crdts.py (same restatement as the dot-set fold).

Parity unpinned: the reference's tests cover none of this, crdts and rmp-serde are not in the
container; the wire forms follow SURVEY.md Appendix A.
"""
from . import crdts as C

CORE_VERSION = bytes.fromhex("e834d789101b463498239de990a9051f")    # crdt-enc/src/lib.rs:26
GPGME_VERSION = bytes.fromhex("e69cb68e7fbb41aa8d2287eace7a04c9")   # crdt-enc-gpgme/src/lib.rs:16
KEY_VERSION = bytes.fromhex("5df28591439a4cef8ca68433276cc9ed")     # xchacha lib.rs:13


class Keys:
    """Keys with Orswot members identified by key id; key material kept beside them."""

    def __init__(self):
        self.latest = C.MVReg()          # vals: (VClock, id)
        self.keys = C.Orswot()           # entries: id -> VClock
        self.material = {}               # id -> (version16, key bytes)

    def merge(self, other):              # key_cryptor.rs:42-50
        self.latest.merge(other.latest)
        ours = dict(self.material)
        self.keys.merge(other.keys)
        # HashMap insert of the other side's Key for common / other-only entries
        self.material = {m: other.material.get(m, ours.get(m)) for m in self.keys.entries}

    def insert_latest_key(self, actor, key_id, key):  # key_cryptor.rs:72-82
        add_dot = (actor, self.keys.clock.get(actor) + 1)     # read_ctx().derive_add_ctx(actor)
        self.keys.apply(("Add", add_dot, [key_id]))
        self.material[key_id] = (KEY_VERSION, key)
        clock = C.VClock()                                    # MVReg read ctx: add clock of vals
        for c, _ in self.latest.vals:
            clock.merge(c)
        clock.apply(actor, clock.get(actor) + 1)
        self.latest.apply(("Put", clock, key_id))

    def latest_key(self):                # key_cryptor.rs:59-70
        ids = [v for _, v in self.latest.vals]
        taken = set()
        for i in ids:
            # keys.take(&id) removes the key, so a second value naming the same id finds nothing
            if i not in self.keys.entries or i in taken:
                raise KeyError("Could not find key for latest key id")   # the reference panics
            taken.add(i)
        if not ids:
            return None
        i = min(ids)
        return i, self.material[i]

    # ---- wire form: to_vec_named(Keys) ----
    def to_bytes(self):
        w = C.Wr()
        w.map(2)
        w.str("latest_key_id")
        w.map(1)
        w.str("vals")
        w.arr(len(self.latest.vals))
        for c, v in self.latest.vals:
            w.arr(2)
            w.vclock(c)
            w.bin(v)
        w.str("keys")
        w.map(3)
        w.str("clock")
        w.vclock(self.keys.clock)
        w.str("entries")
        w.map(len(self.keys.entries))
        for m in sorted(self.keys.entries):
            _key(w, m, self.material[m])
            w.vclock(self.keys.entries[m])
        w.str("deferred")
        items = sorted((C.vclock_bytes(C.VClock(dict(k))), sorted(ms)) for k, ms in self.keys.deferred.items())
        w.map(len(items))
        for kb, ms in items:
            w.b += kb
            w.arr(len(ms))
            for m in ms:
                _key(w, m, self.material.get(m, (KEY_VERSION, bytes(32))))
        return bytes(w.b)


def _key(w, key_id, mat):
    """Key { id: Uuid, key: VersionBytes(Uuid, serde_bytes) } (key_cryptor.rs:85-89)"""
    w.map(2)
    w.str("id")
    w.bin(key_id)
    w.str("key")
    w.arr(2)
    w.bin(mat[0])
    w.bin(mat[1])


def _version_bytes(obj):
    v = C._seq(obj)
    if len(v) != 2:
        raise C.DecodeError("VersionBytes arity")
    return C._uuid(v[0]), bytes(v[1]) if isinstance(v[1], (bytes, bytearray)) else bytes(C._seq(v[1]))


def _dec_mvreg(obj, dec_v):
    (vals,) = C._struct(obj, ["vals"])
    r = C.MVReg()
    for pair in C._seq(vals):
        c, v = C._seq(pair)
        r.vals.append((C.dec_vclock(c), dec_v(v)))
    return r


def _dec_key(obj):
    kid, kv = C._struct(obj, ["id", "key"])
    return C._uuid(kid), _version_bytes(kv)


def decode_keys(b):
    """rmp_serde::from_slice::<Keys>"""
    latest, keys = C._struct(C._unpack(b), ["latest_key_id", "keys"])
    k = Keys()
    k.latest = _dec_mvreg(latest, C._uuid)
    clock, entries, deferred = C._struct(keys, ["clock", "entries", "deferred"])
    k.keys.clock = C.dec_vclock(clock)
    for m, c in C._pairs(entries):
        kid, mat = _dec_key(m)
        k.keys.entries[kid] = C.dec_vclock(c)
        k.material[kid] = mat
    for kc, ms in C._pairs(deferred):
        k.keys.deferred.setdefault(C.dec_vclock(kc).key(), set()).update(_dec_key(m)[0] for m in C._seq(ms))
    return k


def remote_meta_bytes(key_cryptor_reg):
    """VersionBytes(CURRENT_VERSION, to_vec_named(RemoteMeta)) with empty storage / cryptor
    registers and the given key_cryptor register (list of (VClock, (version, bytes)))."""
    w = C.Wr()
    w.map(3)
    for name, vals in (("storage", []), ("cryptor", []), ("key_cryptor", key_cryptor_reg)):
        w.str(name)
        w.map(1)
        w.str("vals")
        w.arr(len(vals))
        for c, (ver, data) in vals:
            w.arr(2)
            w.vclock(c)
            w.arr(2)
            w.bin(ver)
            if len(data) < 256:
                w.bin(data)
            else:
                w.b += (b"\xc5" + len(data).to_bytes(2, "big") if len(data) < 65536
                        else b"\xc6" + len(data).to_bytes(4, "big")) + data
    return CORE_VERSION + bytes(w.b)


def keys_from_remote_metas(files):
    """read_remote_meta_ + KeyHandler::set_remote_meta: merged Keys."""
    reg = C.MVReg()
    for f in files:
        if len(f) < 16:
            raise C.DecodeError("outer length")
        if f[:16] != CORE_VERSION:
            raise C.DecodeError("outer version")
        _, _, kc = C._struct(C._unpack(f[16:]), ["storage", "cryptor", "key_cryptor"])
        reg.merge(_dec_mvreg(kc, _version_bytes))
    out = Keys()
    for _, (ver, data) in reg.vals:
        if ver != GPGME_VERSION:
            raise C.DecodeError("key cryptor version")
        out.merge(decode_keys(data))
    return out
