"""CPU-side checks of the C ABI: the library loads, exports every symbol include/crdtenc.h
declares, and its host-only pieces (framing, naming, storage layout) match the reference.
No compute calls here -- cipher/fold calls need the GPU (tests/test_gpu_*.py)."""
import ctypes
import hashlib
import os
import re
import struct
import base64

import pytest

import crdtenc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = bytes.fromhex


def header_functions():
    src = open(os.path.join(REPO, "include", "crdtenc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ce_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = crdtenc.lib()
    declared = header_functions()
    assert len(declared) >= 40
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(crdtenc.EXPORTS) == declared


def test_status_strings_follow_reference_messages():
    lib = crdtenc.lib()
    assert lib.ce_status_str(9) == b"Decryption failed"             # xchacha lib.rs:97
    assert lib.ce_status_str(8) == b"Invalid nonce length"          # xchacha lib.rs:90
    assert lib.ce_status_str(66) == b"no latest key"                # lib.rs:420


def test_sealed_len_matches_box_layout(oracle):
    for n in [0, 1, 100, 200, 4096 - 99, 4096, 65535, 1 << 20]:
        assert crdtenc.sealed_len(n) == oracle.lib().oc_cryptor_sealed_len(n)
    # 200 B -> 282 B box (298 B file), 4096 -> 4179 (+16)
    assert crdtenc.sealed_len(200) + 16 == 298
    assert crdtenc.sealed_len(4096) + 16 == 4195
    assert crdtenc.sealed_len(1 << 20) + 16 == (1 << 20) + 103


def test_content_name_matches_fixture(repo_fx):
    for kind in ("gcounter", "vclock"):
        c = repo_fx["compact"][kind]
        assert crdtenc.content_name(H(c["file"])) == c["name"]
    for n in [0, 1, 135, 136, 137, 5000]:
        d = os.urandom(n)
        want = base64.b32encode(hashlib.sha3_256(d).digest()).decode().rstrip("=")
        assert crdtenc.content_name(d) == want


def test_content_name_async_matches_hashlib():
    """ce_content_name_async / _wait (the library's host-thread name, what bench.py overlaps
    with the next step) == BASE32_NOPAD(SHA3-256) for jobs queued together and waited out of
    order; a ticket cannot be waited twice."""
    import numpy as np
    data = np.frombuffer(os.urandom(300000), dtype=np.uint8).copy()
    sizes = [0, 1, 135, 136, 137, 4095, 4096, 221184, 300000]
    jobs = [crdtenc.content_name_async(data[:n]) for n in sizes]
    for n, j in reversed(list(zip(sizes, jobs))):
        want = base64.b32encode(hashlib.sha3_256(data[:n].tobytes()).digest()).decode().rstrip("=")
        assert j.result() == want, n
    out = ctypes.create_string_buffer(64)
    assert crdtenc.lib().ce_content_name_wait(ctypes.c_uint64(jobs[0].ticket), out) != 0


@pytest.mark.parametrize("no_openssl", [False, True])
def test_content_name_large_inputs(no_openssl):
    """BASE32_NOPAD(SHA3-256(bytes)) (crdt-enc-tokio/src/lib.rs:407-417) at and past the 4 KiB
    cut-over to dlopen'd OpenSSL and up to 3 MiB, against hashlib: in-process (OpenSSL present),
    and in a child process with CE_NO_OPENSSL=1 (read once, when the first name is taken), which
    pins the portable Keccak-f[1600] sponge on large inputs."""
    import subprocess
    import sys
    sizes = [4095, 4096, 4097, (1 << 20) + 7, 3 << 20]
    code = ("import os, sys, hashlib, base64; sys.path.insert(0, %r); import crdtenc\n"
            "for n in %r:\n"
            "    d = bytes((i * 2654435761 >> 13) & 255 for i in range(n))\n"
            "    want = base64.b32encode(hashlib.sha3_256(d).digest()).decode().rstrip('=')\n"
            "    assert crdtenc.content_name(d) == want, n\n"
            "print('ok')\n") % (os.path.join(REPO, "crdt-enc_amd"), sizes)
    env = dict(os.environ)
    env.pop("CE_NO_OPENSSL", None)
    if no_openssl:
        env["CE_NO_OPENSSL"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


def test_product_library_has_no_diagnostic_kernel_variants():
    """The product libcrdtenc.so carries only the measured default instantiations of
    k_open_fold_v2 (OPT 1 at 4 files per wave, OPT 3 at 2, and the open-only form at 16 lanes
    per file and 3 blocks per lane, which decodes nothing): the diagnostics variants -- some
    give wrong results on purpose (OPT 129/385 skip the actor lookups, 513/1025 may write
    status 77) -- live only in libcrdtenc_prof.so (CE_FUSED_DIAG), so no environment variable
    can select them from the product."""
    raw = open(os.path.join(REPO, "crdt-enc_amd", "libcrdtenc.so"), "rb").read()
    found = set(re.findall(rb"k_open_fold_v2ILi(\d+)ELi(\d+)ELb([01])ELi(\d+)ELb([01])ELb([01])E", raw))
    assert found, "no k_open_fold_v2 instantiation found in the product library"
    opts = {tuple(int(x) for x in t) for t in found}
    # (LPF, waves, JIT, OPT, DEC, DS): the C2 kernel, its 2-files-per-wave form, the open-only
    # form and the open-only form with the Orswot op decode (DS)
    assert opts <= {(16, 2, 0, 1, 1, 0), (32, 3, 0, 3, 1, 0), (16, 3, 0, 1, 0, 0), (16, 3, 0, 1, 0, 1)}, sorted(opts)
    assert not re.search(rb"decode_foldILi\d+ELi[1-9]", raw)


# ---- VersionBytesBuf: port of crdt-enc/tests/version_box_buf.rs ----
UUID = H("d8d2cf50a5c6433b98e68c268fd84fa0")


def vbuf(content):
    b = crdtenc.VBuf()
    keep = ctypes.create_string_buffer(bytes(content), max(len(content), 1))
    crdtenc.lib().ce_vbuf_init(ctypes.byref(b), UUID, keep, ctypes.c_size_t(len(content)))
    b._keep = keep
    return b


def chunk(b):
    p = ctypes.c_void_p()
    n = crdtenc.lib().ce_vbuf_chunk(ctypes.byref(b), ctypes.byref(p))
    return ctypes.string_at(p.value, n) if n else b""


def remaining(b):
    return crdtenc.lib().ce_vbuf_remaining(ctypes.byref(b))


def advance(b, n):
    return crdtenc.lib().ce_vbuf_advance(ctypes.byref(b), ctypes.c_size_t(n))


def vectored(b, k):
    ptrs = (ctypes.c_void_p * max(k, 1))()
    lens = (ctypes.c_size_t * max(k, 1))()
    n = crdtenc.lib().ce_vbuf_chunks_vectored(ctypes.byref(b), ptrs, lens, ctypes.c_size_t(k))
    return [ctypes.string_at(ptrs[i], lens[i]) if lens[i] else b"" for i in range(n)]


def test_vbuf_simple():                                     # version_box_buf.rs:8-33
    b = vbuf(b"\x01\x02\x03")
    assert remaining(b) == 19
    assert chunk(b) == UUID
    advance(b, 16)
    assert remaining(b) == 3 and chunk(b) == b"\x01\x02\x03"
    advance(b, 3)
    assert remaining(b) == 0
    assert advance(b, 0) == 0 and remaining(b) == 0


def test_vbuf_unaligned_advance():                          # version_box_buf.rs:35-63
    b = vbuf(b"\x01\x02\x03")
    advance(b, 4)
    assert remaining(b) == 15 and chunk(b) == UUID[4:]
    advance(b, 13)
    assert remaining(b) == 2 and chunk(b) == b"\x02\x03"
    advance(b, 2)
    assert remaining(b) == 0 and advance(b, 0) == 0


def test_vbuf_out_of_bounds_advance():                      # version_box_buf.rs:65-70
    b = vbuf(b"\x01\x02\x03")
    assert advance(b, 16 + 3 + 1) == -1                     # the reference panics


def test_vbuf_vectored():                                   # version_box_buf.rs:72-140
    b = vbuf(b"\x01\x02\x03")
    assert vectored(b, 0) == []
    assert vectored(b, 1) == [UUID]
    assert vectored(b, 2) == [UUID, b"\x01\x02\x03"]
    assert vectored(b, 3) == [UUID, b"\x01\x02\x03"]
    advance(b, 5)
    assert vectored(b, 1) == [UUID[5:]]
    assert vectored(b, 2) == [UUID[5:], b"\x01\x02\x03"]
    advance(b, 12)
    assert vectored(b, 1) == [b"\x02\x03"]
    assert vectored(b, 2) == [b"\x02\x03"]
    advance(b, 2)
    assert vectored(b, 1) == [] and vectored(b, 2) == []


# ---- Storage: crdt-enc-tokio layout (host only) ----
def uuid_str(u):
    h = u.hex()
    return "%s-%s-%s-%s-%s" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:])


def test_storage_layout(tmp_path):
    local, remote = str(tmp_path / "local"), str(tmp_path / "remote")
    st = crdtenc.Storage(local, remote)
    a, b = H("00112233445566778899aabbccddeeff"), H("ffeeddccbbaa99887766554433221100")
    for v in range(3):
        st.store_ops(a, v, b"A%d" % v)
    st.store_ops(b, 0, b"B0")
    st.store_ops(b, 2, b"B2")            # gap: load_ops stops at the first missing version
    assert os.path.exists(os.path.join(remote, "ops", uuid_str(a), "2"))
    assert sorted(st.list_op_actors()) == sorted([a, b])
    got = st.load_ops([(a, 1), (b, 0)])
    assert [(x[0], x[1], x[2]) for x in got] == [(a, 1, b"A1"), (a, 2, b"A2"), (b, 0, b"B0")]
    with pytest.raises(crdtenc.CeError):   # create_new: never overwrite an op file
        st.store_ops(a, 0, b"again")
    name = st.store_state(b"state-bytes")
    assert name == base64.b32encode(hashlib.sha3_256(b"state-bytes").digest()).decode().rstrip("=")
    assert st.list_state_names() == [name]
    assert st.load_state(name) == b"state-bytes"


def test_storage_requires_absolute_paths():
    with pytest.raises(crdtenc.CeError):
        crdtenc.Storage("relative/local", "/abs/remote")


def test_no_gpu_means_no_compute():
    """The product has no CPU path: without a GPU the context refuses to open."""
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(crdtenc.CeError) as e:
        crdtenc.Context(0)
    assert e.value.code == 65


def test_content_names_multi_buffer_matches_hashlib():
    """ce_content_names (eight SHA3-256 sponges per AVX-512 step, message tails on their own
    sponge) == BASE32_NOPAD(SHA3-256) per buffer, for batches of 1-17 with equal and mixed
    lengths around the 136-byte rate, empty buffers included (and the scalar fallback when the CPU
    has no AVX-512F: the same answers)."""
    import random
    import numpy as np
    rng = random.Random(11)
    for n in (1, 2, 3, 7, 8, 9, 16, 17):
        for mixed in (False, True):
            lens = ([rng.choice([0, 1, 135, 136, 137, 271, 272, 1000, 5000, 136 * 50]) for _ in range(n)]
                    if mixed else [rng.randint(0, 20000)] * n)
            bufs = [np.frombuffer(os.urandom(k), np.uint8) if k else np.zeros(0, np.uint8) for k in lens]
            want = [base64.b32encode(hashlib.sha3_256(b.tobytes()).digest()).decode().rstrip("=") for b in bufs]
            assert crdtenc.content_names(bufs) == want, (n, lens)
