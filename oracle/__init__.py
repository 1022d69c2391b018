"""ctypes binding of the C oracle (oracle/ce_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  Never imported by the product (crdt-enc_amd/).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libce_oracle.so")

STATUS = {
    0: "OK", 1: "OUTER_LEN", 2: "OUTER_VERSION", 3: "KEY_VERSION", 4: "KEY_LEN",
    5: "PARSE_VBOX", 6: "DATA_VERSION", 7: "PARSE_ENCBOX", 8: "NONCE_LEN", 9: "AUTH",
    10: "PT_LEN", 11: "PT_VERSION", 12: "DECODE", 13: "OP_VERSION",
}

KEY_VERSION = bytes.fromhex("5df28591439a4cef8ca68433276cc9ed")
STATE_VCLOCK, STATE_GCOUNTER = 0, 1

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C %s oracle`" % os.path.dirname(HERE))
        L = ctypes.CDLL(LIB_PATH)
        P, S, U8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p
        L.oc_cryptor_sealed_len.restype = S
        L.oc_cryptor_sealed_len.argtypes = [S]
        L.oc_core_serialize.restype = S
        L.oc_base32_nopad.restype = S
        L.oc_open_batch_mt.restype = S
        L.oc_compact_ops_baseline.restype = S
        L.oc_compact_ops_best.restype = S
        L.oc_compact_orswot_best.restype = S
        L.oc_compact_orswot_best.argtypes = [P, P, P, P, S, P, P, P, P, S, ctypes.c_int,
                                             ctypes.c_int, P, S, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_double)]
        L.oc_vclock_get.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), len(b) or 1)


def chacha20_block(key, counter, nonce12):
    out = ctypes.create_string_buffer(64)
    lib().oc_chacha20_block(_buf(key), ctypes.c_uint32(counter), _buf(nonce12), out)
    return out.raw


def hchacha20(key, n16):
    out = ctypes.create_string_buffer(32)
    lib().oc_hchacha20(_buf(key), _buf(n16), out)
    return out.raw


def poly1305(key, msg):
    out = ctypes.create_string_buffer(16)
    lib().oc_poly1305(_buf(key), _buf(msg), ctypes.c_size_t(len(msg)), out)
    return out.raw


def xchacha_seal(key, nonce, pt, aad=b""):
    out = ctypes.create_string_buffer(len(pt) + 16)
    if aad:
        lib().oc_xchacha_seal_aad(_buf(key), _buf(nonce), _buf(aad), ctypes.c_size_t(len(aad)),
                                  _buf(pt), ctypes.c_size_t(len(pt)), out)
    else:
        lib().oc_xchacha_seal(_buf(key), _buf(nonce), _buf(pt), ctypes.c_size_t(len(pt)), out)
    return out.raw


def xchacha_open(key, nonce, ct):
    out = ctypes.create_string_buffer(max(len(ct), 1))
    st = lib().oc_xchacha_open(_buf(key), _buf(nonce), _buf(ct), ctypes.c_size_t(len(ct)), out)
    return st, (out.raw[:len(ct) - 16] if st == 0 else None)


def sha3_256(msg):
    out = ctypes.create_string_buffer(32)
    lib().oc_sha3_256(_buf(msg), ctypes.c_size_t(len(msg)), out)
    return out.raw


def base32_nopad(b):
    out = ctypes.create_string_buffer(len(b) * 2 + 8)
    n = lib().oc_base32_nopad(_buf(b), ctypes.c_size_t(len(b)), out)
    return out.raw[:n].decode()


def cryptor_encrypt(key, nonce, clear, key_version=KEY_VERSION):
    cap = lib().oc_cryptor_sealed_len(len(clear))
    out = ctypes.create_string_buffer(cap)
    ol = ctypes.c_size_t(0)
    st = lib().oc_cryptor_encrypt(_buf(key_version), _buf(key), ctypes.c_size_t(len(key)),
                                  _buf(nonce), _buf(clear), ctypes.c_size_t(len(clear)), out,
                                  ctypes.byref(ol))
    return st, (out.raw[:ol.value] if st == 0 else None)


def cryptor_decrypt(key, enc, key_version=KEY_VERSION):
    out = ctypes.create_string_buffer(max(len(enc), 1))
    ol = ctypes.c_size_t(0)
    st = lib().oc_cryptor_decrypt(_buf(key_version), _buf(key), ctypes.c_size_t(len(key)),
                                  _buf(enc), ctypes.c_size_t(len(enc)), out, ctypes.byref(ol))
    return st, (out.raw[:ol.value] if st == 0 else None)


class OracleCore(ctypes.Structure):
    pass


class _VClock(ctypes.Structure):
    _fields_ = [("actor", ctypes.c_void_p), ("counter", ctypes.c_void_p),
                ("n", ctypes.c_size_t), ("cap", ctypes.c_size_t)]


class _Core(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("next_op_versions", _VClock), ("state", _VClock)]


def _pack_batch(files):
    blob = b"".join(files)
    offs = [0]
    for f in files:
        offs.append(offs[-1] + len(f))
    return blob, (ctypes.c_uint64 * len(offs))(*offs)


class Core:
    """Oracle StateWrapper<S> for S in {VClock, GCounter}."""

    def __init__(self, kind=STATE_GCOUNTER):
        self.c = _Core()
        lib().oc_core_init(ctypes.byref(self.c), kind)

    def __del__(self):
        try:
            lib().oc_core_free(ctypes.byref(self.c))
        except Exception:
            pass

    def serialize(self):
        n = lib().oc_core_serialize(ctypes.byref(self.c), None, ctypes.c_size_t(0))
        out = ctypes.create_string_buffer(max(n, 1))
        lib().oc_core_serialize(ctypes.byref(self.c), out, ctypes.c_size_t(n))
        return out.raw[:n]

    def read_remote_ops(self, key, supported, files, actors, versions, key_version=KEY_VERSION):
        blob, offs = _pack_batch(files)
        n = len(files)
        sup = b"".join(supported)
        st = (ctypes.c_int32 * max(n, 1))()
        act = b"".join(actors)
        ver = (ctypes.c_uint64 * max(n, 1))(*versions)
        rc = lib().oc_read_remote_ops(ctypes.byref(self.c), _buf(key_version), _buf(key),
                                      ctypes.c_size_t(len(key)), _buf(sup),
                                      ctypes.c_size_t(len(supported)), _buf(blob), offs,
                                      _buf(act), ver, ctypes.c_size_t(n), st)
        return rc, list(st)[:n]

    def read_remote_states(self, key, supported, files, key_version=KEY_VERSION):
        blob, offs = _pack_batch(files)
        n = len(files)
        sup = b"".join(supported)
        st = (ctypes.c_int32 * max(n, 1))()
        rc = lib().oc_read_remote_states(ctypes.byref(self.c), _buf(key_version), _buf(key),
                                         ctypes.c_size_t(len(key)), _buf(sup),
                                         ctypes.c_size_t(len(supported)), _buf(blob), offs,
                                         ctypes.c_size_t(n), st)
        return rc, list(st)[:n]


_out_buf = None


def compact_ops_baseline(kind, key, data_version, blob, offs, file_actor, file_version,
                         n_files, n_threads, best=False):
    """CPU baseline over numpy/ctypes buffers (blob: bytes-like, offs: uint64[n+1]).
    best=False: reference-shaped (n_threads AEAD workers, decode + fold on one thread);
    best=True: every stage on n_threads threads (fold sharded by actor)."""
    global _out_buf
    cap = 8 << 20
    if _out_buf is None:
        _out_buf = ctypes.create_string_buffer(cap)
    out = _out_buf
    err = ctypes.c_int(0)
    fn = lib().oc_compact_ops_best if best else lib().oc_compact_ops_baseline
    n = fn(kind, _buf(key), _buf(data_version), blob, offs, file_actor, file_version,
           ctypes.c_size_t(n_files), n_threads, out, ctypes.c_size_t(cap), ctypes.byref(err))
    return err.value, out.raw[:n]


def _addr(x):
    """address of a bytes-like / numpy buffer (kept alive by the caller)"""
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return ctypes.cast(ctypes.c_char_p(x), ctypes.c_void_p).value


def compact_orswot_best(key, data_version, state_files, blob, offs, file_actor, file_version,
                        n_threads, seal=True, cap=1 << 27):
    """Orswot CPU baseline (oc_compact_orswot_best).  state_files: list of bytes; blob: op files
    back to back (bytes or uint8 numpy), offs: uint64 numpy [n+1], file_actor: uint8 numpy
    [n, 16], file_version: uint64 numpy [n].  Returns (err, StateWrapper bytes, seconds of the
    C call, phase seconds [open+decode, state merges, op fold, serialize+seal])."""
    import time
    import numpy as np
    sblob = b"".join(state_files) or b"\0"
    soffs = np.zeros(len(state_files) + 1, dtype=np.uint64)
    for i, f in enumerate(state_files):
        soffs[i + 1] = soffs[i] + len(f)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    fa = np.ascontiguousarray(file_actor, dtype=np.uint8).reshape(-1, 16)
    fv = np.ascontiguousarray(file_version, dtype=np.uint64)
    n = len(offs) - 1
    assert fa.shape[0] >= n and fv.shape[0] >= n
    kb, dv = _buf(key), _buf(data_version)
    while True:
        out = ctypes.create_string_buffer(cap)
        err = ctypes.c_int(0)
        ph = (ctypes.c_double * 4)()
        t = time.perf_counter()
        ln = lib().oc_compact_orswot_best(
            ctypes.addressof(kb), ctypes.addressof(dv), _addr(sblob), soffs.ctypes.data,
            len(state_files), _addr(blob), offs.ctypes.data, fa.ctypes.data, fv.ctypes.data, n,
            n_threads, 1 if seal else 0, ctypes.addressof(out), cap, ctypes.byref(err), ph)
        dt = time.perf_counter() - t
        if ln <= cap:
            return err.value, out.raw[:ln], dt, list(ph)
        cap = ln
