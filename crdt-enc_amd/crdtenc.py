"""ctypes binding of libcrdtenc.so (include/crdtenc.h) -- the MI355X hot path of crdt-enc.

Mirrors the reference's plugin/Core interface (Rust, chpio/crdt-enc):
  Cryptor  crdt-enc/src/cryptor.rs:11-27, EncHandler crdt-enc-xchacha20poly1305/src/lib.rs
  Storage  crdt-enc/src/storage.rs:8-43,  tokio local dir crdt-enc-tokio/src/lib.rs
  Core     crdt-enc/src/lib.rs (open, read_remote, compact, apply_ops, state bytes)

There is no CPU fallback: loading fails loudly when the library is missing, and every
cipher/fold call runs the gfx950 kernels (CE_ERR_DEVICE without a GPU).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CRDTENC_LIB selects another in-tree build (e.g. libcrdtenc_prof.so, the diagnostics build)
LIB_PATH = os.environ.get("CRDTENC_LIB") or os.path.join(HERE, "libcrdtenc.so")

OK = 0
STATUS_NAMES = {
    0: "OK", 1: "OUTER_LEN", 2: "OUTER_VERSION", 3: "KEY_VERSION", 4: "KEY_LEN",
    5: "PARSE_VBOX", 6: "DATA_VERSION", 7: "PARSE_ENCBOX", 8: "NONCE_LEN", 9: "AUTH",
    10: "PT_LEN", 11: "PT_VERSION", 12: "DECODE", 13: "OP_VERSION", 64: "INVALID_ARG",
    65: "DEVICE", 66: "NO_KEY", 67: "IO", 68: "NO_LOCAL_META", 69: "SHARD",
}
ERR_OP_VERSION, ERR_SHARD = 13, 69
# window flags word (hi[m], include/crdtenc.h ce_core_shard_window)
SHARD_BAD, SHARD_GAP, SHARD_E0_MISMATCH = 1, 2, 4
STATE_VCLOCK, STATE_GCOUNTER, STATE_ORSWOT, STATE_MVREG = 0, 1, 2, 3
OPEN_CREATE, COMPACT_INGEST_FORMAT, OPEN_MULTI_KEY = 1, 2, 4

CORE_VERSION = bytes.fromhex("e834d789101b463498239de990a9051f")   # crdt-enc/src/lib.rs:26
KEY_VERSION = bytes.fromhex("5df28591439a4cef8ca68433276cc9ed")    # xchacha lib.rs:13

# symbols declared in include/crdtenc.h (checked by tests/test_abi.py)
EXPORTS = [
    "ce_buf_free", "ce_status_str", "ce_ctx_create", "ce_ctx_destroy", "ce_ctx_set_stream",
    "ce_ctx_synchronize", "ce_ctx_last_error", "ce_cryptor_gen_key", "ce_cryptor_encrypt",
    "ce_cryptor_decrypt", "ce_cryptor_sealed_len", "ce_cryptor_decrypt_batch",
    "ce_cryptor_encrypt_batch", "ce_cryptor_decrypt_batch_device",
    "ce_cryptor_encrypt_batch_device", "ce_storage_open", "ce_storage_close",
    "ce_storage_list_op_actors", "ce_storage_load_ops", "ce_storage_store_ops",
    "ce_storage_remove_ops", "ce_storage_list_state_names", "ce_storage_store_state",
    "ce_storage_load_state", "ce_storage_remove_state", "ce_content_name", "ce_content_name_async",
    "ce_content_name_wait", "ce_core_open",
    "ce_core_close", "ce_core_set_latest_key", "ce_core_info_actor", "ce_core_read_remote",
    "ce_core_compact", "ce_core_apply_ops", "ce_core_state_bytes", "ce_core_ingest_ops",
    "ce_core_ingest_ops_device", "ce_core_ingest_states", "ce_core_compact_to_buffer",
    "ce_core_compact_into", "ce_core_compact_ops_device",
    "ce_core_register_actors", "ce_core_dense_capacity", "ce_core_export_dense",
    "ce_core_import_dense", "ce_vbuf_init", "ce_vbuf_remaining", "ce_vbuf_chunk",
    "ce_vbuf_advance", "ce_vbuf_chunks_vectored", "ce_ctx_set_timing", "ce_ctx_timing_read",
    "ce_ctx_timing_reset", "ce_ctx_set_timing_only", "ce_core_reset", "ce_core_settle", "ce_core_merge_state", "ce_core_dense_ready",
    "ce_keys_decode", "ce_keys_from_remote_metas", "ce_keys_merge", "ce_keys_free",
    "ce_keys_count", "ce_keys_latest", "ce_keys_get", "ce_keys_at", "ce_core_set_keys",
    "ce_core_apply_ops_batch", "ce_core_ingest_ops_iov", "ce_core_ingest_states_iov", "ce_core_compact_ops_iov",
    "ce_core_path_count", "ce_ctx_clock_probe",
    "ce_shard_owner", "ce_shard_owners", "ce_shard_stats_len", "ce_core_shard_stats",
    "ce_core_shard_window", "ce_core_ingest_ops_device_sharded", "ce_core_pending_export",
    "ce_core_pending_commit", "ce_core_writer_versions", "ce_shard_stats_host",
    "ce_shard_window_host", "ce_shard_window_exact", "ce_core_compact_ops_device_into",
    "ce_core_state_bytes_device", "ce_core_merge_state_device", "ce_core_export_columns_device",
    "ce_core_merge_columns_device", "ce_core_ingest_states_device",
    "ce_core_compact_into_async", "ce_core_compact_wait", "ce_host_alloc", "ce_host_free", "ce_content_names",
]


class _HostMem:
    """ce_host_alloc'd memory, freed with the last array viewing it"""

    def __init__(self, n):
        self.p = lib().ce_host_alloc(n)
        if not self.p:
            raise MemoryError("ce_host_alloc(%d)" % n)

    def __del__(self):
        try:
            if getattr(self, "p", None):
                lib().ce_host_free(self.p)
        except Exception:       # interpreter teardown
            pass
        self.p = None


def host_buffer(nbytes):
    """A u8 numpy array over pinned host memory (ce_host_alloc): the destination for
    Core.compact_into_async, whose download then runs on the device's DMA engines."""
    import numpy as np
    m = _HostMem(nbytes)
    c = (ctypes.c_uint8 * nbytes).from_address(m.p)
    c._ce_mem = m            # the array's base (c) keeps the allocation alive
    return np.frombuffer(c, dtype=np.uint8)


def _np_ptr(a, dtype):
    import numpy as np
    a = np.ascontiguousarray(a, dtype=dtype)
    return a, ctypes.c_void_p(a.ctypes.data)


def shard_owners(actors, file_actor, file_version, world):
    """Owner rank of every op file ops/<actors[file_actor[i]]>/<file_version[i]> (numpy u32)."""
    import numpy as np
    n = len(file_actor)
    acts = b"".join(bytes(a) for a in actors)
    fa, fap = _np_ptr(file_actor, np.uint32)
    fv, fvp = _np_ptr(file_version, np.uint64)
    out = np.empty(max(n, 1), np.uint32)
    rc = lib().ce_shard_owners(_cbuf(acts), ctypes.c_uint32(len(actors)), fap, fvp, ctypes.c_uint64(n),
                               ctypes.c_uint32(world), ctypes.c_void_p(out.ctypes.data))
    if rc:
        raise CeError(rc, "ce_shard_owners")
    return out[:n]


def shard_stats_host(actors, e0, file_actor, file_version, rank, world):
    """ShardStats (int64[2m + 3]) of one rank's host metadata (the CPU twin of the device pass)."""
    import numpy as np
    m = len(actors)
    st = np.empty(lib().ce_shard_stats_len(m), np.int64)
    e, ep = _np_ptr(e0, np.uint64)
    fa, fap = _np_ptr(file_actor, np.uint32)
    fv, fvp = _np_ptr(file_version, np.uint64)
    rc = lib().ce_shard_stats_host(_cbuf(b"".join(bytes(a) for a in actors)), ctypes.c_uint32(m), ep, fap, fvp,
                                   ctypes.c_uint64(len(fa)), ctypes.c_uint32(rank), ctypes.c_uint32(world),
                                   ctypes.c_void_p(st.ctypes.data))
    if rc:
        raise CeError(rc, "ce_shard_stats_host")
    return st


def shard_window_host(e0, stats):
    """(hi u64[m], flags) from reduced stats."""
    import numpy as np
    m = len(e0)
    hi = np.empty(m + 1, np.uint64)
    e, ep = _np_ptr(e0, np.uint64)
    s, sp = _np_ptr(stats, np.int64)
    rc = lib().ce_shard_window_host(ctypes.c_uint32(m), ep, sp, ctypes.c_void_p(hi.ctypes.data))
    if rc:
        raise CeError(rc, "ce_shard_window_host")
    return hi[:m], int(hi[m])


def shard_window_exact(e0, file_actor, file_version):
    """(hi u64[m], flags) from every rank's gathered (writer, version) metadata."""
    import numpy as np
    m = len(e0)
    hi = np.empty(m + 1, np.uint64)
    e, ep = _np_ptr(e0, np.uint64)
    fa, fap = _np_ptr(file_actor, np.uint32)
    fv, fvp = _np_ptr(file_version, np.uint64)
    rc = lib().ce_shard_window_exact(ctypes.c_uint32(m), ep, fap, fvp, ctypes.c_uint64(len(fa)),
                                     ctypes.c_void_p(hi.ctypes.data))
    if rc:
        raise CeError(rc, "ce_shard_window_exact")
    return hi[:m], int(hi[m])


class CeError(RuntimeError):
    def __init__(self, code, detail=""):
        self.code = code
        super().__init__("%s (%d)%s" % (STATUS_NAMES.get(code, "?"), code,
                                        (": " + detail) if detail else ""))


class Buf(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class OpenOptions(ctypes.Structure):
    _fields_ = [("state_kind", ctypes.c_int), ("supported_data_versions", ctypes.c_char_p),
                ("n_supported", ctypes.c_size_t), ("current_data_version", ctypes.c_char_p),
                ("local_path", ctypes.c_char_p), ("remote_path", ctypes.c_char_p),
                ("flags", ctypes.c_uint32)]


class VBuf(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_size_t), ("version", ctypes.c_uint8 * 16),
                ("content", ctypes.c_void_p), ("content_len", ctypes.c_size_t)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libcrdtenc.so not built (run `make -C %s product`); the product "
                               "has no CPU fallback" % os.path.dirname(HERE))
        # One HIP runtime per process: torch bundles libamdhip64 with the same SONAME
        # (libamdhip64.so.7) but is linked by file name, so it must be loaded first; our
        # DT_NEEDED then binds to it and torch tensors / streams and our kernels share it.
        if not os.environ.get("CRDTENC_NO_TORCH"):
            try:
                import torch  # noqa: F401
            except Exception:
                pass
        L = ctypes.CDLL(LIB_PATH)
        L.ce_status_str.restype = ctypes.c_char_p
        L.ce_ctx_last_error.restype = ctypes.c_char_p
        L.ce_cryptor_sealed_len.restype = ctypes.c_size_t
        L.ce_cryptor_sealed_len.argtypes = [ctypes.c_size_t]
        L.ce_core_dense_capacity.restype = ctypes.c_uint32
        L.ce_keys_count.restype = ctypes.c_uint32
        L.ce_core_path_count.restype = ctypes.c_uint64
        L.ce_shard_owner.restype = ctypes.c_uint32
        L.ce_shard_owner.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32]
        L.ce_shard_stats_len.restype = ctypes.c_uint32
        L.ce_vbuf_remaining.restype = ctypes.c_size_t
        L.ce_vbuf_chunk.restype = ctypes.c_size_t
        L.ce_vbuf_chunks_vectored.restype = ctypes.c_size_t
        L.ce_host_alloc.restype = ctypes.c_void_p
        L.ce_host_alloc.argtypes = [ctypes.c_size_t]
        L.ce_host_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def _take(b):
    data = ctypes.string_at(b.data, b.len) if b.len else b""
    lib().ce_buf_free(ctypes.byref(b))
    return data


def _cbuf(b):
    return ctypes.create_string_buffer(bytes(b), max(len(b), 1))


def sealed_len(n):
    return lib().ce_cryptor_sealed_len(n)


def _ptr(data):
    """(pointer, length) of bytes / bytearray / a contiguous uint8 numpy array, without a copy
    (the object must outlive the call)."""
    if isinstance(data, bytes):
        return ctypes.c_char_p(data), len(data)
    mv = memoryview(data).cast("B")
    if mv.readonly:
        return _cbuf(data), mv.nbytes
    return (ctypes.c_char * mv.nbytes).from_buffer(mv), mv.nbytes


def content_name(data):
    out = ctypes.create_string_buffer(64)
    p, n = _ptr(data)
    rc = lib().ce_content_name(p, ctypes.c_size_t(n), out)
    if rc:
        raise CeError(rc)
    return out.value.decode()


def content_names(bufs):
    """content_name of every buffer, eight SHA3-256 sponges per AVX-512 step (ce_content_names)"""
    n = len(bufs)
    if n == 0:
        return []
    held = [_ptr(b) for b in bufs]
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(p, ctypes.c_void_p) for p, _ in held])
    lens = (ctypes.c_size_t * n)(*[k for _, k in held])
    out = (ctypes.c_char * (64 * n))()
    rc = lib().ce_content_names(ptrs, lens, ctypes.c_uint32(n), out)
    if rc:
        raise CeError(rc)
    raw = bytes(out)
    return [raw[64 * i: 64 * (i + 1)].split(b"\0", 1)[0].decode() for i in range(n)]


class NameJob:
    """ce_content_name_async: the name of `data` computed on the library's host thread; the
    buffer must stay alive (and unchanged) until result() returns."""

    def __init__(self, data):
        p, n = _ptr(data)
        self._keep = (data, p)
        t = ctypes.c_uint64(0)
        rc = lib().ce_content_name_async(p, ctypes.c_size_t(n), ctypes.byref(t))
        if rc:
            raise CeError(rc)
        self.ticket = t.value
        self._name = None

    def result(self):
        if self._name is None:
            out = ctypes.create_string_buffer(64)
            rc = lib().ce_content_name_wait(ctypes.c_uint64(self.ticket), out)
            if rc:
                raise CeError(rc)
            self._name = out.value.decode()
            self._keep = None
        return self._name

    def __del__(self):
        # a job dropped unwaited (e.g. an exception between steps): the worker still reads the
        # buffer through a raw pointer, so wait for it before the buffer can be freed (this also
        # retires the ticket's entry in the library's done table)
        try:
            if self._name is None and getattr(self, "_keep", None) is not None:
                out = ctypes.create_string_buffer(64)
                lib().ce_content_name_wait(ctypes.c_uint64(self.ticket), out)
                self._keep = None
        except Exception:
            pass


def content_name_async(data):
    return NameJob(data)


class Context:
    """One per GPU (one process per GPU)."""

    def __init__(self, device=0):
        import weakref
        self.p = ctypes.c_void_p()
        self.device = device
        self._cores = weakref.WeakSet()  # cores hold the context: close them first
        rc = lib().ce_ctx_create(device, ctypes.byref(self.p))
        if rc:
            raise CeError(rc, "ce_ctx_create(device=%d)" % device)

    def close(self):
        if self.p:
            for c in list(self._cores):
                c.close()
            lib().ce_ctx_destroy(self.p)
            self.p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self):
        return lib().ce_ctx_last_error(self.p).decode(errors="replace")

    def check(self, rc, what=""):
        if rc:
            raise CeError(rc, "%s %s" % (what, self.last_error()))

    def set_stream(self, stream_ptr):
        self.check(lib().ce_ctx_set_stream(self.p, ctypes.c_void_p(stream_ptr)), "set_stream")
        self.stream_ptr = stream_ptr

    def synchronize(self):
        lib().ce_ctx_synchronize(self.p)

    def set_timing(self, enable=True):
        self.check(lib().ce_ctx_set_timing(self.p, 1 if enable else 0), "set_timing")

    def set_timing_only(self, kernel=None):
        """Time only launches named `kernel` (None: every launch)."""
        self.check(lib().ce_ctx_set_timing_only(self.p, kernel.encode() if kernel else None),
                   "set_timing_only")

    def timing(self, kernel):
        """(total_ms, launches) of one kernel since the last reset (HIP events on our stream)."""
        ms = ctypes.c_double(0)
        cnt = ctypes.c_uint64(0)
        self.check(lib().ce_ctx_timing_read(self.p, kernel.encode(), ctypes.byref(ms),
                                            ctypes.byref(cnt)), "timing")
        return ms.value, cnt.value

    def timing_reset(self):
        lib().ce_ctx_timing_reset(self.p)

    def clock_probe(self, out_ptr, blocks, samples, ticks, stream_ptr=None):
        """Diagnostics: launch the shader-clock probe (ce_ctx_clock_probe) on stream_ptr (None:
        the context stream); out_ptr = device uint64[blocks * samples * 2] (cycles, ticks)."""
        self.check(lib().ce_ctx_clock_probe(self.p, ctypes.c_void_p(stream_ptr), ctypes.c_void_p(out_ptr),
                                            ctypes.c_uint32(blocks), ctypes.c_uint32(samples),
                                            ctypes.c_uint32(ticks)), "clock_probe")

    # ---- Cryptor ----
    def gen_key(self):
        b = Buf()
        self.check(lib().ce_cryptor_gen_key(self.p, ctypes.byref(b)), "gen_key")
        vb = _take(b)
        return vb[:16], vb[16:]

    def encrypt(self, key, clear, nonce=None, key_version=KEY_VERSION):
        b = Buf()
        rc = lib().ce_cryptor_encrypt(self.p, _cbuf(key_version), _cbuf(key),
                                      ctypes.c_size_t(len(key)),
                                      _cbuf(nonce) if nonce is not None else None,
                                      _cbuf(clear), ctypes.c_size_t(len(clear)), ctypes.byref(b))
        self.check(rc, "encrypt")
        return _take(b)

    def decrypt(self, key, enc, key_version=KEY_VERSION):
        """Returns (status, plaintext or None)."""
        b = Buf()
        rc = lib().ce_cryptor_decrypt(self.p, _cbuf(key_version), _cbuf(key),
                                      ctypes.c_size_t(len(key)), _cbuf(enc),
                                      ctypes.c_size_t(len(enc)), ctypes.byref(b))
        if rc:
            return rc, None
        return 0, _take(b)

    def decrypt_batch(self, key, items, key_version=KEY_VERSION):
        """items: list of enc boxes.  Returns (rc, [status], [plaintext or None], out_blob)."""
        n = len(items)
        blob = b"".join(items)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, it in enumerate(items):
            offs[i] = o
            o += len(it)
        offs[n] = o
        out = ctypes.create_string_buffer(o + 16 * n + 64)
        oo = (ctypes.c_uint64 * max(n, 1))()
        ol = (ctypes.c_uint64 * max(n, 1))()
        st = (ctypes.c_int32 * max(n, 1))()
        rc = lib().ce_cryptor_decrypt_batch(self.p, _cbuf(key_version), _cbuf(key),
                                            ctypes.c_size_t(len(key)), _cbuf(blob), offs,
                                            ctypes.c_uint32(n), out, oo, ol, st)
        raw = out.raw
        pts = [raw[oo[i]:oo[i] + ol[i]] if st[i] == 0 else None for i in range(n)]
        return rc, list(st)[:n], pts, raw, [oo[i] for i in range(n)]

    def encrypt_batch(self, key, clears, nonces=None, key_version=KEY_VERSION):
        n = len(clears)
        blob = b"".join(clears)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, c in enumerate(clears):
            offs[i] = o
            o += len(c)
        offs[n] = o
        cap = sum(sealed_len(len(c)) for c in clears)
        out = ctypes.create_string_buffer(max(cap, 1))
        oo = (ctypes.c_uint64 * (n + 1))()
        nb = _cbuf(b"".join(nonces)) if nonces is not None else None
        rc = lib().ce_cryptor_encrypt_batch(self.p, _cbuf(key_version), _cbuf(key),
                                            ctypes.c_size_t(len(key)), _cbuf(blob), offs,
                                            ctypes.c_uint32(n), nb, out, ctypes.c_size_t(cap), oo)
        self.check(rc, "encrypt_batch")
        raw = out.raw
        return [raw[oo[i]:oo[i + 1]] for i in range(n)]

    def decrypt_batch_device(self, key, d_blob, d_offs, n, d_out, d_status=0,
                             key_version=KEY_VERSION):
        nf = ctypes.c_uint32(0)
        rc = lib().ce_cryptor_decrypt_batch_device(
            self.p, _cbuf(key_version), _cbuf(key), ctypes.c_size_t(len(key)),
            ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_void_p(d_out), ctypes.c_void_p(d_status or None), ctypes.byref(nf))
        self.check(rc, "decrypt_batch_device")
        return nf.value

    def encrypt_batch_device(self, key, d_clear, d_offs, n, d_nonces, d_out, d_out_offs,
                             outer_version=None, key_version=KEY_VERSION):
        rc = lib().ce_cryptor_encrypt_batch_device(
            self.p, _cbuf(key_version), _cbuf(key), ctypes.c_size_t(len(key)),
            _cbuf(outer_version) if outer_version is not None else None,
            ctypes.c_void_p(d_clear), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_void_p(d_nonces), ctypes.c_void_p(d_out), ctypes.c_void_p(d_out_offs))
        self.check(rc, "encrypt_batch_device")


class Storage:
    """crdt-enc-tokio Storage (local dir)."""

    def __init__(self, local_path, remote_path):
        self.p = ctypes.c_void_p()
        rc = lib().ce_storage_open(local_path.encode(), remote_path.encode(), ctypes.byref(self.p))
        if rc:
            raise CeError(rc, "ce_storage_open")

    def __del__(self):
        try:
            lib().ce_storage_close(self.p)
        except Exception:
            pass

    def list_op_actors(self):
        b = Buf()
        rc = lib().ce_storage_list_op_actors(self.p, ctypes.byref(b))
        if rc:
            raise CeError(rc)
        d = _take(b)
        return [d[i:i + 16] for i in range(0, len(d), 16)]

    def load_ops(self, actor_first):
        actors = b"".join(a for a, _ in actor_first)
        m = len(actor_first)
        first = (ctypes.c_uint64 * max(m, 1))(*[f for _, f in actor_first])
        bufs = [Buf() for _ in range(4)]
        rc = lib().ce_storage_load_ops(self.p, _cbuf(actors), first, ctypes.c_uint32(m),
                                       *[ctypes.byref(x) for x in bufs])
        if rc:
            raise CeError(rc)
        blob, offs, aidx, vers = [_take(x) for x in bufs]
        import struct
        o = struct.unpack("<%dQ" % (len(offs) // 8), offs)
        ai = struct.unpack("<%dI" % (len(aidx) // 4), aidx)
        vv = struct.unpack("<%dQ" % (len(vers) // 8), vers)
        return [(actor_first[ai[i]][0], vv[i], blob[o[i]:o[i + 1]]) for i in range(len(ai))]

    def store_ops(self, actor, version, data):
        rc = lib().ce_storage_store_ops(self.p, _cbuf(actor), ctypes.c_uint64(version),
                                        _cbuf(data), ctypes.c_size_t(len(data)))
        if rc:
            raise CeError(rc)

    def list_state_names(self):
        b = Buf()
        rc = lib().ce_storage_list_state_names(self.p, ctypes.byref(b))
        if rc:
            raise CeError(rc)
        d = _take(b)
        return [x.decode() for x in d.split(b"\0") if x]

    def store_state(self, data):
        out = ctypes.create_string_buffer(64)
        rc = lib().ce_storage_store_state(self.p, _cbuf(data), ctypes.c_size_t(len(data)), out)
        if rc:
            raise CeError(rc)
        return out.value.decode()

    def load_state(self, name):
        b = Buf()
        rc = lib().ce_storage_load_state(self.p, name.encode(), ctypes.byref(b))
        if rc:
            raise CeError(rc)
        return _take(b)


class Keys:
    """Keys { latest_key_id: MVReg<Uuid, Uuid>, keys: Orswot<Key, Uuid> }
    (crdt-enc/src/key_cryptor.rs:35-82), decoded and merged on the host by the product."""

    def __init__(self, p):
        self.p = p

    @classmethod
    def decode(cls, msgpack_bytes):
        p = ctypes.c_void_p()
        rc = lib().ce_keys_decode(_cbuf(msgpack_bytes), ctypes.c_size_t(len(msgpack_bytes)),
                                  ctypes.byref(p))
        if rc:
            raise CeError(rc, "ce_keys_decode")
        return cls(p)

    @classmethod
    def from_remote_metas(cls, files):
        """Core::read_remote_meta_ + the gpgme KeyHandler's decode of the key register."""
        n = len(files)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, f in enumerate(files):
            offs[i] = o
            o += len(f)
        offs[n] = o
        p = ctypes.c_void_p()
        rc = lib().ce_keys_from_remote_metas(_cbuf(b"".join(files)), offs, ctypes.c_uint32(n),
                                             ctypes.byref(p))
        if rc:
            raise CeError(rc, "ce_keys_from_remote_metas")
        return cls(p)

    def close(self):
        if self.p:
            lib().ce_keys_free(self.p)
            self.p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def merge(self, other):
        rc = lib().ce_keys_merge(self.p, other.p)
        if rc:
            raise CeError(rc, "ce_keys_merge")

    def __len__(self):
        return lib().ce_keys_count(self.p)

    def _get(self, fn, *args):
        n = ctypes.c_size_t(0)
        ver = ctypes.create_string_buffer(16)
        ident = ctypes.create_string_buffer(16)
        rc = fn(self.p, *args, ident, ver, None, ctypes.c_size_t(0), ctypes.byref(n)) if fn is not \
            lib().ce_keys_get else fn(self.p, *args, ver, None, ctypes.c_size_t(0), ctypes.byref(n))
        if rc:
            raise CeError(rc)
        key = ctypes.create_string_buffer(max(n.value, 1))
        if fn is lib().ce_keys_get:
            rc = fn(self.p, *args, ver, key, ctypes.c_size_t(n.value), ctypes.byref(n))
        else:
            rc = fn(self.p, *args, ident, ver, key, ctypes.c_size_t(n.value), ctypes.byref(n))
        if rc:
            raise CeError(rc)
        return ident.raw, ver.raw, key.raw[:n.value]

    def latest(self):
        """Keys::latest_key -> (id, key version, key); CeError NO_KEY / DECODE otherwise."""
        return self._get(lib().ce_keys_latest)

    def get(self, key_id):
        _, ver, key = self._get(lib().ce_keys_get, _cbuf(key_id))
        return ver, key

    def items(self):
        return [self._get(lib().ce_keys_at, ctypes.c_uint32(i)) for i in range(len(self))]


class Core:
    """Core<S> for S in {VClock<Uuid>, GCounter<Uuid>, Orswot<u64, Uuid>, MVReg<u64, Uuid>}
    (crdt-enc/src/lib.rs)."""

    def __init__(self, ctx, kind=STATE_GCOUNTER, supported=(), current_data_version=None,
                 local_path=None, remote_path=None, flags=0):
        self.ctx = ctx
        self.kind = kind
        sup = b"".join(supported)
        cdv = current_data_version or (supported[0] if supported else bytes(16))
        self._keep = [sup, cdv]
        o = OpenOptions(kind, sup, len(supported), cdv,
                        local_path.encode() if local_path else None,
                        remote_path.encode() if remote_path else None, flags)
        self.p = ctypes.c_void_p()
        rc = lib().ce_core_open(ctx.p, ctypes.byref(o), ctypes.byref(self.p))
        if rc:
            raise CeError(rc, "ce_core_open " + ctx.last_error())
        ctx._cores.add(self)

    def close(self):
        if self.p:
            lib().ce_core_close(self.p)
            self.p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_latest_key(self, key, key_version=KEY_VERSION):
        self.ctx.check(lib().ce_core_set_latest_key(self.p, _cbuf(key_version), _cbuf(key),
                                                    ctypes.c_size_t(len(key))), "set_latest_key")

    def set_keys(self, keys):
        """CoreSubHandle::set_keys (lib.rs:382-388): Keys::latest_key for reads and writes; the
        other keys are tried on AUTH failures only with OPEN_MULTI_KEY."""
        self.ctx.check(lib().ce_core_set_keys(self.p, keys.p), "set_keys")

    def info_actor(self):
        out = ctypes.create_string_buffer(16)
        self.ctx.check(lib().ce_core_info_actor(self.p, out), "info")
        return out.raw

    def state_bytes(self):
        b = Buf()
        self.ctx.check(lib().ce_core_state_bytes(self.p, ctypes.byref(b)), "state_bytes")
        return _take(b)

    def ingest_ops(self, files, actors, file_actor, versions, want_status=True):
        n = len(files)
        blob = b"".join(files)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, f in enumerate(files):
            offs[i] = o
            o += len(f)
        offs[n] = o
        st = (ctypes.c_int32 * max(n, 1))() if want_status else None
        fa = (ctypes.c_uint32 * max(n, 1))(*file_actor)
        fv = (ctypes.c_uint64 * max(n, 1))(*versions)
        rc = lib().ce_core_ingest_ops(self.p, _cbuf(blob), offs, ctypes.c_uint32(n),
                                      _cbuf(b"".join(actors)), ctypes.c_uint32(len(actors)), fa,
                                      fv, st)
        return rc, (list(st)[:n] if want_status else None)

    def ingest_ops_device(self, d_blob, d_offs, n, blob_len, actors, d_file_actor,
                          d_file_version, want_status=False):
        """Batch resident in HBM: d_* are device pointers (u8 files, u64 offs[n+1],
        u32 file_actor[n], u64 file_version[n]); actors = host bytes (16 per writer)."""
        st = (ctypes.c_int32 * max(n, 1))() if want_status else None
        rc = lib().ce_core_ingest_ops_device(
            self.p, ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_uint64(blob_len), _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
            ctypes.c_void_p(d_file_actor), ctypes.c_void_p(d_file_version), st)
        return (rc, list(st)[:n]) if want_status else rc

    def compact_ops_device(self, d_blob, d_offs, n, blob_len, actors, d_file_actor,
                           d_file_version, nonce=None, name=True):
        """Core::compact over a batch resident in HBM (read_remote_ops + compaction output in
        one call): returns (rc, file, name); file/name are None when rc != 0."""
        b = Buf()
        nm = ctypes.create_string_buffer(64) if name else None
        rc = lib().ce_core_compact_ops_device(
            self.p, ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_uint64(blob_len), _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
            ctypes.c_void_p(d_file_actor), ctypes.c_void_p(d_file_version),
            _cbuf(nonce) if nonce is not None else None, ctypes.byref(b), nm)
        if rc:
            return rc, None, None
        return rc, _take(b), (nm.value.decode() if name else None)

    def compact_ops_device_into(self, buf, d_blob, d_offs, n, blob_len, actors, d_file_actor,
                                d_file_version, nonce=None, name=False):
        """compact_ops_device with the sealed file downloaded straight into the uint8 numpy
        array `buf` (pinned, e.g. torch.empty(..., pin_memory=True).numpy()): (rc, length,
        name or None)."""
        ln = ctypes.c_size_t(0)
        nm = ctypes.create_string_buffer(64) if name else None
        rc = lib().ce_core_compact_ops_device_into(
            self.p, ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_uint64(blob_len), _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
            ctypes.c_void_p(d_file_actor), ctypes.c_void_p(d_file_version),
            _cbuf(nonce) if nonce is not None else None, ctypes.c_void_p(buf.ctypes.data),
            ctypes.c_size_t(buf.nbytes), ctypes.byref(ln), nm)
        return rc, ln.value, (nm.value.decode() if (name and rc == 0) else None)

    def ingest_ops_iov(self, files, actors, file_actor, versions, want_status=True):
        """Per-file host buffers (Storage::load_ops's Vec<u8>s): no concatenation."""
        n = len(files)
        bufs = [_cbuf(f) for f in files]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
        st = (ctypes.c_int32 * max(n, 1))() if want_status else None
        fa = (ctypes.c_uint32 * max(n, 1))(*file_actor)
        fv = (ctypes.c_uint64 * max(n, 1))(*versions)
        rc = lib().ce_core_ingest_ops_iov(self.p, ptrs, lens, ctypes.c_uint32(n),
                                          _cbuf(b"".join(actors)), ctypes.c_uint32(len(actors)), fa,
                                          fv, st)
        return rc, (list(st)[:n] if want_status else None)

    def compact_ops_iov(self, ptrs, lens, n, actors, file_actor, file_version, nonce=None,
                        name=True):
        """Core::compact over per-file host buffers: ptrs / lens = ctypes arrays (n entries) of
        file addresses and sizes, file_actor (u32) / file_version (u64) host arrays (ctypes or
        numpy .ctypes pointers).  Returns (rc, file, name)."""
        b = Buf()
        nm = ctypes.create_string_buffer(64) if name else None
        rc = lib().ce_core_compact_ops_iov(
            self.p, ptrs, lens, ctypes.c_uint32(n), _ptr(actors)[0],
            ctypes.c_uint32(len(actors) // 16), file_actor, file_version,
            _cbuf(nonce) if nonce is not None else None, ctypes.byref(b), nm)
        if rc:
            return rc, None, None
        return rc, _take(b), (nm.value.decode() if name else None)

    def ingest_states(self, files):
        n = len(files)
        blob = b"".join(files)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, f in enumerate(files):
            offs[i] = o
            o += len(f)
        offs[n] = o
        st = (ctypes.c_int32 * max(n, 1))()
        rc = lib().ce_core_ingest_states(self.p, _cbuf(blob), offs, ctypes.c_uint32(n), st)
        return rc, list(st)[:n]

    def ingest_states_iov(self, files):
        """ingest_states over per-file host buffers (no concatenation, no copy)."""
        n = len(files)
        bufs = [_ptr(f)[0] for f in files]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
        st = (ctypes.c_int32 * max(n, 1))()
        rc = lib().ce_core_ingest_states_iov(self.p, ptrs, lens, ctypes.c_uint32(n), st)
        return rc, list(st)[:n]

    def ingest_states_device(self, d_blob, d_offs, n, blob_len, want_status=False):
        """ingest_states over state files resident in HBM (device pointers)."""
        st = (ctypes.c_int32 * max(n, 1))() if want_status else None
        rc = lib().ce_core_ingest_states_device(self.p, ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs),
                                                ctypes.c_uint32(n), ctypes.c_uint64(blob_len), st)
        return (rc, list(st)[:n]) if want_status else rc

    def read_remote(self):
        return lib().ce_core_read_remote(self.p)

    def compact(self):
        name = ctypes.create_string_buffer(64)
        rc = lib().ce_core_compact(self.p, name)
        return rc, name.value.decode()

    def compact_to_buffer(self, nonce=None, name=True):
        """(file, content name); name=False skips the SHA3-256 name (None): content_name(file)
        gives it later, e.g. on another thread."""
        b = Buf()
        nm = ctypes.create_string_buffer(64) if name else None
        rc = lib().ce_core_compact_to_buffer(self.p, _cbuf(nonce) if nonce is not None else None,
                                             ctypes.byref(b), nm)
        self.ctx.check(rc, "compact_to_buffer")
        return _take(b), (nm.value.decode() if name else None)

    def compact_into(self, buf, nonce=None, name=True):
        """compact_to_buffer into a caller-owned uint8 numpy array `buf` (grown when too small,
        so pass the returned array back next time): (array, length, content name or None)."""
        import numpy as np
        n = ctypes.c_size_t(0)
        nm = ctypes.create_string_buffer(64) if name else None
        nc = _cbuf(nonce) if nonce is not None else None
        for _ in range(2):
            rc = lib().ce_core_compact_into(self.p, nc, ctypes.c_void_p(buf.ctypes.data),
                                            ctypes.c_size_t(buf.nbytes), ctypes.byref(n), nm)
            if rc == 64 and n.value > buf.nbytes:
                buf = np.empty(n.value + (n.value >> 3), np.uint8)
                continue
            break
        self.ctx.check(rc, "compact_into")
        return buf, n.value, (nm.value.decode() if name else None)

    def compact_into_async(self, buf, nonce=None):
        """compact_into with the download left in flight: (length, ticket).  ticket 0: the file
        is already in buf[:length]; else length is 0 and compact_wait(ticket) returns it once the
        file is in buf (pinned buf; raises then when the file did not fit)."""
        n = ctypes.c_size_t(0)
        t = ctypes.c_uint64(0)
        rc = lib().ce_core_compact_into_async(self.p, _cbuf(nonce) if nonce is not None else None,
                                              ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes),
                                              ctypes.byref(n), ctypes.byref(t))
        self.ctx.check(rc, "compact_into_async")
        return n.value, t.value

    def compact_wait(self, ticket):
        """the length of the file compact_into_async(ticket) left in flight, once it is complete"""
        n = ctypes.c_uint64(0)
        self.ctx.check(lib().ce_core_compact_wait(self.p, ctypes.c_uint64(ticket), ctypes.byref(n)), "compact_wait")
        return n.value

    def apply_ops(self, ops_msgpack):
        return lib().ce_core_apply_ops(self.p, _cbuf(ops_msgpack), ctypes.c_size_t(len(ops_msgpack)))

    def apply_ops_batch(self, ops_list, nonces=None):
        """n Core::apply_ops calls in one GPU seal: returns (rc, [op file bytes])."""
        n = len(ops_list)
        offs = (ctypes.c_uint64 * (n + 1))()
        o = 0
        for i, x in enumerate(ops_list):
            offs[i] = o
            o += len(x)
        offs[n] = o
        fb, fo = Buf(), Buf()
        rc = lib().ce_core_apply_ops_batch(self.p, _cbuf(b"".join(ops_list)), offs, ctypes.c_uint32(n),
                                           _cbuf(b"".join(nonces)) if nonces is not None else None,
                                           ctypes.byref(fb), ctypes.byref(fo))
        if rc:
            return rc, None
        blob, fofs = _take(fb), _take(fo)
        import struct
        o = struct.unpack("<%dQ" % (n + 1), fofs)
        return 0, [blob[o[i]:o[i + 1]] for i in range(n)]

    def reset(self):
        self.ctx.check(lib().ce_core_reset(self.p), "reset")

    def settle(self):
        """Wait for the queued device work; the status a fold / merge found after its call
        returned (a dot-set table overflow, sticky until reset)."""
        return lib().ce_core_settle(self.p)

    def merge_state(self, state_wrapper_msgpack):
        """read_remote_states' merge of one decrypted StateWrapper (lib.rs:447, 458-466)."""
        return lib().ce_core_merge_state(self.p, _cbuf(state_wrapper_msgpack),
                                         ctypes.c_size_t(len(state_wrapper_msgpack)))

    def export_columns_device(self, d_dst, cap):
        """The column form of an Orswot for the multi-GPU exchange, into device memory d_dst (cap
        bytes), deferred removals as its final section: (rc, length); rc INVALID_ARG with the
        needed length when cap is too small, with length 0 when the state has no column form
        (not an Orswot: use state_bytes_device)."""
        n = ctypes.c_uint64(0)
        rc = lib().ce_core_export_columns_device(self.p, ctypes.c_void_p(d_dst), ctypes.c_uint64(cap), ctypes.byref(n))
        return rc, n.value

    def columns_ready(self):
        """the state has a column form (an Orswot, deferred removals included)"""
        n = ctypes.c_uint64(0)
        lib().ce_core_export_columns_device(self.p, None, ctypes.c_uint64(0), ctypes.byref(n))
        return n.value != 0

    def merge_columns_device(self, d_parts, lens):
        """Merge column partials (device pointers, byte lengths; at most 64) into the state at once,
        their deferred removals and this state's applied after the k-way merge."""
        k = len(d_parts)
        ptrs = (ctypes.c_void_p * max(k, 1))(*d_parts)
        ls = (ctypes.c_uint64 * max(k, 1))(*lens)
        return lib().ce_core_merge_columns_device(self.p, ptrs, ls, ctypes.c_uint32(k))

    def state_bytes_device(self, d_dst, cap):
        """StateWrapper bytes written into device memory d_dst (cap bytes): (rc, length); rc
        INVALID_ARG with the needed length when cap is too small."""
        n = ctypes.c_uint64(0)
        rc = lib().ce_core_state_bytes_device(self.p, ctypes.c_void_p(d_dst), ctypes.c_uint64(cap), ctypes.byref(n))
        return rc, n.value

    def merge_state_device(self, d_sw, length):
        """merge_state of a StateWrapper resident in HBM (device pointer, length bytes)."""
        return lib().ce_core_merge_state_device(self.p, ctypes.c_void_p(d_sw), ctypes.c_uint64(length))

    def register_actors(self, actors):
        self.ctx.check(lib().ce_core_register_actors(self.p, _cbuf(b"".join(actors)),
                                                     ctypes.c_uint32(len(actors))), "register")

    def dense_capacity(self):
        return lib().ce_core_dense_capacity(self.p)

    def path_count(self, path):
        return lib().ce_core_path_count(self.p, path.encode())

    def dense_ready(self):
        """True when export/import_dense can carry the whole state (no unregistered actor)."""
        return lib().ce_core_dense_ready(self.p) == 1

    def export_dense(self, d_state, d_nov):
        self.ctx.check(lib().ce_core_export_dense(self.p, ctypes.c_void_p(d_state),
                                                  ctypes.c_void_p(d_nov)), "export_dense")

    # ---- multi-GPU partition by op-file address (include/crdtenc.h, shard.ingest_sharded) ----
    def shard_stats(self, actors, d_fa, d_fv, n, rank, world, d_stats):
        self.ctx.check(lib().ce_core_shard_stats(self.p, _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
                                                 ctypes.c_void_p(d_fa), ctypes.c_void_p(d_fv),
                                                 ctypes.c_uint32(n), ctypes.c_uint32(rank),
                                                 ctypes.c_uint32(world), ctypes.c_void_p(d_stats)),
                       "shard_stats")

    def shard_window(self, actors, d_stats, d_hi):
        self.ctx.check(lib().ce_core_shard_window(self.p, _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
                                                  ctypes.c_void_p(d_stats), ctypes.c_void_p(d_hi)),
                       "shard_window")

    def ingest_ops_device_sharded(self, d_blob, d_offs, n, blob_len, actors, d_fa, d_fv, d_hi,
                                  want_status=False):
        st = (ctypes.c_int32 * max(n, 1))() if want_status else None
        rc = lib().ce_core_ingest_ops_device_sharded(
            self.p, ctypes.c_void_p(d_blob), ctypes.c_void_p(d_offs), ctypes.c_uint32(n),
            ctypes.c_uint64(blob_len), _ptr(actors)[0], ctypes.c_uint32(len(actors) // 16),
            ctypes.c_void_p(d_fa), ctypes.c_void_p(d_fv), ctypes.c_void_p(d_hi), st)
        return (rc, list(st)[:n]) if want_status else rc

    def pending_export(self, d_batch, cap_words):
        """The pending batch into d_batch (u64[cap_words]); False (nothing written) when it names
        an unregistered actor or the table outgrew cap_words."""
        ready = ctypes.c_int(0)
        self.ctx.check(lib().ce_core_pending_export(self.p, ctypes.c_void_p(d_batch), ctypes.c_uint64(cap_words),
                                                    ctypes.byref(ready)), "pending_export")
        return ready.value == 1

    def pending_commit(self, accept, d_import=None, import_words=0):
        self.ctx.check(lib().ce_core_pending_commit(self.p, 1 if accept else 0,
                                                    ctypes.c_void_p(d_import) if d_import else None,
                                                    ctypes.c_uint64(import_words)),
                       "pending_commit")

    def writer_versions(self, actors):
        import numpy as np
        m = len(actors) // 16
        out = np.zeros(max(m, 1), np.uint64)
        self.ctx.check(lib().ce_core_writer_versions(self.p, _ptr(actors)[0], ctypes.c_uint32(m),
                                                     ctypes.c_void_p(out.ctypes.data)), "writer_versions")
        return out[:m]

    def import_dense(self, d_state, d_nov):
        self.ctx.check(lib().ce_core_import_dense(self.p, ctypes.c_void_p(d_state),
                                                  ctypes.c_void_p(d_nov)), "import_dense")
