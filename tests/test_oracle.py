"""Pin the C oracle against the golden fixtures (CPU only).

The fixtures come from OpenSSL / Python msgpack / hashlib (tests/golden/make_golden.py), i.e.
from implementations independent of both the oracle and the HIP product.
"""
import hashlib

import pytest

H = bytes.fromhex


def test_chacha20_block_rfc8439(oracle, kats):
    for v in kats["chacha20_block"]:
        assert oracle.chacha20_block(H(v["key"]), v["counter"], H(v["nonce"])).hex() == v["out"]


def test_hchacha20(oracle, kats):
    for v in kats["hchacha20"]:
        assert oracle.hchacha20(H(v["key"]), H(v["nonce16"])).hex() == v["out"]


def test_poly1305_rfc8439(oracle, kats):
    for v in kats["poly1305"]:
        assert oracle.poly1305(H(v["key"]), H(v["msg"])).hex() == v["tag"]


def test_xchacha_aad_kat(oracle, kats):
    for v in kats["xchacha_aad"]:
        ct = oracle.xchacha_seal(H(v["key"]), H(v["nonce"]), H(v["pt"]), H(v["aad"]))
        assert ct.hex() == v["ct"]


def test_xchacha_vectors(oracle, kats):
    for v in kats["xchacha"]:
        key, nonce = H(v["key"]), H(v["nonce"])
        ct = oracle.xchacha_seal(key, nonce, v["pt_bytes"])
        assert ct == v["ct_bytes"], v["len"]
        assert hashlib.sha256(ct).hexdigest() == v["ct_sha256"]
        st, pt = oracle.xchacha_open(key, nonce, ct)
        assert st == 0 and pt == v["pt_bytes"]
        bad = bytearray(ct)
        bad[len(bad) // 2] ^= 4
        st, pt = oracle.xchacha_open(key, nonce, bytes(bad))
        assert st == 9 and pt is None


def test_sha3_base32(oracle, kats):
    for v in kats["sha3_256"]:
        assert oracle.sha3_256(H(v["msg"])).hex() == v["out"]
    for v in kats["base32_nopad"]:
        assert oracle.base32_nopad(H(v["in"])) == v["out"]


def test_cryptor_roundtrip_layout(oracle, repo_fx):
    """EncHandler::encrypt box layout (xchacha lib.rs:59-67) == the msgpack fixture bytes."""
    key = H(repo_fx["key"])
    c = repo_fx["compact"]["gcounter"]
    clear = H(repo_fx["expected_state"]["gcounter"])
    st, enc = oracle.cryptor_encrypt(key, H(c["nonce"]), clear)
    assert st == 0
    sealed = H(repo_fx["data_version"]) + enc
    assert sealed.hex() == c["file"]
    assert oracle.base32_nopad(oracle.sha3_256(sealed)) == c["name"]
    st, pt = oracle.cryptor_decrypt(key, enc)
    assert st == 0 and pt == clear


@pytest.mark.parametrize("kind", ["gcounter", "vclock"])
def test_read_remote_ops_fixture(oracle, repo_fx, kind):
    key = H(repo_fx["key"])
    files = [H(f["file"]) for f in repo_fx["files"]]
    actors = [H(f["actor"]) for f in repo_fx["files"]]
    versions = [f["version"] for f in repo_fx["files"]]
    core = oracle.Core(oracle.STATE_GCOUNTER if kind == "gcounter" else oracle.STATE_VCLOCK)
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], files, actors, versions)
    assert rc == 0 and all(s == 0 for s in st)
    assert core.serialize().hex() == repo_fx["expected_state"][kind]
    # idempotence: re-reading the same batch skips every file (version < expected)
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], files, actors, versions)
    assert rc == 0
    assert core.serialize().hex() == repo_fx["expected_state"][kind]


@pytest.mark.parametrize("kind", ["gcounter", "vclock"])
def test_read_remote_states_then_ops(oracle, repo_fx, kind):
    key = H(repo_fx["key"])
    core = oracle.Core(oracle.STATE_GCOUNTER if kind == "gcounter" else oracle.STATE_VCLOCK)
    rc, st = core.read_remote_states(key, [H(repo_fx["data_version"])], [H(repo_fx["state_files"][kind])])
    assert rc == 0, st
    files = [H(f["file"]) for f in repo_fx["files"]]
    actors = [H(f["actor"]) for f in repo_fx["files"]]
    versions = [f["version"] for f in repo_fx["files"]]
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], files, actors, versions)
    # the state file claims next_op_versions[actor0] = 30 and [actor3] = 2: those files skip
    assert rc == 0 and all(s == 0 for s in st)
    assert core.serialize().hex() == repo_fx["expected_after_state_then_ops"][kind]


def test_negatives(oracle, repo_fx):
    key = H(repo_fx["key"])
    sup = [H(repo_fx["data_version"])]
    for case in repo_fx["negatives"]:
        core = oracle.Core()
        f = H(case["file"])
        rc, st = core.read_remote_ops(key, sup, [f], [bytes(16)], [0])
        assert st[0] == case["status"], (case["name"], st[0], case["status"])
        if case["status"] != 0:
            # all-or-nothing: nothing folded
            assert core.serialize() == oracle.Core().serialize()


def test_batch_reject_leaves_state(oracle, repo_fx):
    key = H(repo_fx["key"])
    files = [H(f["file"]) for f in repo_fx["files"]]
    bad = bytearray(files[7])
    bad[-3] ^= 1
    files[7] = bytes(bad)
    actors = [H(f["actor"]) for f in repo_fx["files"]]
    versions = [f["version"] for f in repo_fx["files"]]
    core = oracle.Core()
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], files, actors, versions)
    assert rc == 9 and st[7] == 9 and sum(s != 0 for s in st) == 1
    assert core.serialize() == oracle.Core().serialize()


def test_wrong_key_version(oracle, repo_fx):
    key = H(repo_fx["key"])
    f = H(repo_fx["files"][0]["file"])
    core = oracle.Core()
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], [f], [bytes(16)], [0],
                                  key_version=bytes(16))
    assert st == [3]
    rc, st = core.read_remote_ops(key[:31], [H(repo_fx["data_version"])], [f], [bytes(16)], [0])
    assert st == [4]
    # outer version is checked by the core before the cryptor sees the key
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], [bytes(16) + f[16:]],
                                  [bytes(16)], [0], key_version=bytes(16))
    assert st == [2]


def test_version_gate(oracle, repo_fx):
    key = H(repo_fx["key"])
    fx = [f for f in repo_fx["files"] if f["actor"] == repo_fx["actors"][1]]
    files = [H(f["file"]) for f in fx]
    actors = [H(f["actor"]) for f in fx]
    versions = [f["version"] for f in fx]
    # drop version 3 -> gap: versions 0..2 applied, then "Unexpected op version"
    core = oracle.Core()
    rc, st = core.read_remote_ops(key, [H(repo_fx["data_version"])], files[:3] + files[4:],
                                  actors[:3] + actors[4:], versions[:3] + versions[4:])
    assert rc == 13
    assert st[:3] == [0, 0, 0] and st[3] == 13
    # the fold keeps versions 0..2 (applied before the error), nothing after the gap
    assert core.serialize() != oracle.Core().serialize()
    ref = oracle.Core()
    rc, _ = ref.read_remote_ops(key, [H(repo_fx["data_version"])], files[:3], actors[:3], versions[:3])
    assert rc == 0 and ref.serialize() == core.serialize()


@pytest.mark.parametrize("best", [False, True], ids=["reference_shaped", "best_cpu"])
@pytest.mark.parametrize("kind", ["gcounter", "vclock"])
def test_cpu_baselines_match_sequential_fold(oracle, repo_fx, kind, best):
    """Both CPU baseline modes (bench.py cpu_baseline) serialize what the sequential
    read_remote_ops oracle serializes: fixture files, then a version gap (fold stops there)."""
    import ctypes
    import numpy as np
    key = H(repo_fx["key"])
    dv = H(repo_fx["data_version"])
    k = oracle.STATE_GCOUNTER if kind == "gcounter" else oracle.STATE_VCLOCK
    fx = repo_fx["files"]
    for drop in (None, 5):
        sel = [i for i in range(len(fx)) if i != drop]
        files = [H(fx[i]["file"]) for i in sel]
        actors = [H(fx[i]["actor"]) for i in sel]
        versions = [fx[i]["version"] for i in sel]
        ref = oracle.Core(k)
        rc_ref, _ = ref.read_remote_ops(key, [dv], files, actors, versions)
        blob = np.frombuffer(b"".join(files), dtype=np.uint8).copy()
        offs = np.cumsum([0] + [len(f) for f in files]).astype(np.uint64)
        act = np.frombuffer(b"".join(actors), dtype=np.uint8).copy()
        ver = np.array(versions, dtype=np.uint64)
        for threads in (1, 3, 8):
            err, ser = oracle.compact_ops_baseline(
                k, key, dv, blob.ctypes.data_as(ctypes.c_void_p),
                offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                act.ctypes.data_as(ctypes.c_void_p),
                ver.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(files), threads, best=best)
            assert err == rc_ref, (drop, threads)
            if err == 0:
                assert ser == ref.serialize(), (drop, threads)
