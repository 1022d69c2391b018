#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run once, in the build container).

Independent of both the C oracle and the HIP product: the AEAD comes from OpenSSL 3
(libcrypto via ctypes), msgpack from the Python `msgpack` package (use_bin_type=True,
which matches rmp-serde 1.x `to_vec_named`), SHA3 from hashlib and
BASE32 from base64.  The reference itself (Rust) cannot be built or run here (SURVEY.md
§8c), so these fixtures are how the oracle is pinned.

Layouts mirrored:
  op file   = CURRENT_VERSION(16) || msgpack([bin16 DATA_VERSION, bin(EncBox)])
              (crdt-enc/src/lib.rs:695, crdt-enc-xchacha20poly1305/src/lib.rs:59-67)
  EncBox    = {"nonce": bin24, "enc_data": bin(ct || tag16)}  (xchacha lib.rs:104-113)
  plaintext = app data version(16) || msgpack(Vec<Dot>)       (crdt-enc/src/lib.rs:670-671)
  Dot       = {"actor": bin16, "counter": uint}                 (crdts 7, derive Serialize)
  state     = {"next_op_versions": VClock, "state": S}          (crdt-enc/src/lib.rs:739-743)
"""
import base64
import ctypes
import hashlib
import json
import os
import random
import struct

import msgpack

HERE = os.path.dirname(os.path.abspath(__file__))

CORE_VERSION = bytes.fromhex("e834d789101b463498239de990a9051f")   # lib.rs:26
BOX_VERSION = bytes.fromhex("c7f269be0ff54a7799c37c23c96d5cb4")    # xchacha lib.rs:11
KEY_VERSION = bytes.fromhex("5df28591439a4cef8ca68433276cc9ed")    # xchacha lib.rs:13
APP_VERSION = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")    # examples/test/src/main.rs:7

# ----------------------------------------------------------------------------------------
# OpenSSL via ctypes
# ----------------------------------------------------------------------------------------
_c = ctypes.CDLL("libcrypto.so.3")
_c.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_c.EVP_chacha20.restype = ctypes.c_void_p
_c.EVP_chacha20_poly1305.restype = ctypes.c_void_p
for fn in ("EVP_EncryptInit_ex", "EVP_EncryptUpdate", "EVP_EncryptFinal_ex",
           "EVP_CIPHER_CTX_ctrl", "EVP_CIPHER_CTX_free"):
    getattr(_c, fn).argtypes = None
EVP_CTRL_AEAD_SET_IVLEN = 0x9
EVP_CTRL_AEAD_GET_TAG = 0x10


def _chacha20_stream(key, iv16, data):
    ctx = ctypes.c_void_p(_c.EVP_CIPHER_CTX_new())
    assert _c.EVP_EncryptInit_ex(ctx, ctypes.c_void_p(_c.EVP_chacha20()), None, key, iv16) == 1
    out = ctypes.create_string_buffer(len(data) + 64)
    ol = ctypes.c_int(0)
    assert _c.EVP_EncryptUpdate(ctx, out, ctypes.byref(ol), data, ctypes.c_int(len(data))) == 1
    _c.EVP_CIPHER_CTX_free(ctx)
    return out.raw[:ol.value]


def hchacha20(key, n16):
    """HChaCha20 from OpenSSL's ChaCha20 block: block(counter=n16[0:4], nonce=n16[4:16])
    minus the initial state, words 0-3 and 12-15 (draft-irtf-cfrg-xchacha-03 §2.2)."""
    ks = _chacha20_stream(key, n16, b"\0" * 64)
    w = struct.unpack("<16I", ks)
    init = struct.unpack("<4I", b"expand 32-byte k") + struct.unpack("<8I", key) + \
        struct.unpack("<4I", n16)
    raw = [(w[i] - init[i]) & 0xffffffff for i in range(16)]
    return struct.pack("<8I", *(raw[0:4] + raw[12:16]))


def chacha20poly1305_seal(key, n12, pt, aad=b""):
    ctx = ctypes.c_void_p(_c.EVP_CIPHER_CTX_new())
    assert _c.EVP_EncryptInit_ex(ctx, ctypes.c_void_p(_c.EVP_chacha20_poly1305()), None, None, None) == 1
    assert _c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, 12, None) == 1
    assert _c.EVP_EncryptInit_ex(ctx, None, None, key, n12) == 1
    ol = ctypes.c_int(0)
    if aad:
        assert _c.EVP_EncryptUpdate(ctx, None, ctypes.byref(ol), aad, ctypes.c_int(len(aad))) == 1
    out = ctypes.create_string_buffer(len(pt) + 32)
    assert _c.EVP_EncryptUpdate(ctx, out, ctypes.byref(ol), pt, ctypes.c_int(len(pt))) == 1
    n = ol.value
    fin = ctypes.create_string_buffer(32)
    assert _c.EVP_EncryptFinal_ex(ctx, fin, ctypes.byref(ol)) == 1
    tag = ctypes.create_string_buffer(16)
    assert _c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
    _c.EVP_CIPHER_CTX_free(ctx)
    return out.raw[:n] + tag.raw


def xchacha_seal(key, nonce24, pt, aad=b""):
    sub = hchacha20(key, nonce24[:16])
    return chacha20poly1305_seal(sub, b"\0\0\0\0" + nonce24[16:], pt, aad)


# ----------------------------------------------------------------------------------------
# reference boxes
# ----------------------------------------------------------------------------------------
def enc_box(nonce, ct):
    return msgpack.packb({"nonce": nonce, "enc_data": ct}, use_bin_type=True)


def cryptor_encrypt(key, nonce, clear):
    """EncHandler::encrypt (xchacha lib.rs:40-71) with a fixed nonce."""
    ct = xchacha_seal(key, nonce, clear)
    return msgpack.packb([BOX_VERSION, enc_box(nonce, ct)], use_bin_type=True)


def op_file(key, nonce, dots, data_version=APP_VERSION):
    clear = data_version + msgpack.packb(
        [{"actor": a, "counter": c} for a, c in dots], use_bin_type=True)
    return CORE_VERSION + cryptor_encrypt(key, nonce, clear), clear


def vclock_obj(d):
    return {"dots": {k: d[k] for k in sorted(d)}}


def state_wrapper_bytes(kind, nov, st):
    s = vclock_obj(st)
    if kind == "gcounter":
        s = {"inner": s}
    return msgpack.packb({"next_op_versions": vclock_obj(nov), "state": s}, use_bin_type=True)


def b32(b):
    return base64.b32encode(b).decode().rstrip("=")


def hx(b):
    return b.hex()


# ----------------------------------------------------------------------------------------
def make_kats(rng):
    k = {}
    # draft-irtf-cfrg-xchacha-03 §2.2.1
    key = bytes(range(32))
    n16 = bytes.fromhex("000000090000004a0000000031415927")
    sub = hchacha20(key, n16)
    assert sub.hex() == "82413b4227b27bfed30e42508a877d73a0f9e4d58a74a853c12ec41326d3ecdc"
    k["hchacha20"] = [{"key": hx(key), "nonce16": hx(n16), "out": hx(sub)}]
    for _ in range(4):
        key = rng.randbytes(32); n16 = rng.randbytes(16)
        k["hchacha20"].append({"key": hx(key), "nonce16": hx(n16), "out": hx(hchacha20(key, n16))})
    # draft-irtf-cfrg-xchacha-03 §A.3.1
    key = bytes(range(0x80, 0xa0))
    nonce = bytes(range(0x40, 0x58))
    aad = bytes.fromhex("50515253c0c1c2c3c4c5c6c7")
    pt = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for "
          b"the future, sunscreen would be it.")
    ct = xchacha_seal(key, nonce, pt, aad)
    assert ct[:16].hex() == "bd6d179d3e83d43b9576579493c0e939"
    assert ct[-16:].hex() == "c0875924c1c7987947deafd8780acf49"
    k["xchacha_aad"] = [{"key": hx(key), "nonce": hx(nonce), "aad": hx(aad), "pt": hx(pt), "ct": hx(ct)}]
    # no-AAD vectors over the lengths that exercise every tail case of the device kernels
    k["xchacha"] = []
    side = bytearray()
    for n in [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 255, 256, 1000, 1023, 1024, 1025, 4079,
              4080, 4096, 4097, 8191, 16384, 65536 + 17]:
        key = rng.randbytes(32); nonce = rng.randbytes(24); pt = rng.randbytes(n)
        ct = xchacha_seal(key, nonce, pt)
        e = {"key": hx(key), "nonce": hx(nonce), "len": n, "bin_off": len(side),
             "tag": hx(ct[-16:]), "ct_sha256": hashlib.sha256(ct).hexdigest()}
        side.extend(pt + ct)   # kat_xchacha.bin: pt || ct||tag per vector
        k["xchacha"].append(e)
    with open(os.path.join(HERE, "kat_xchacha.bin"), "wb") as f:
        f.write(bytes(side))
    # RFC 8439 §2.5.2 Poly1305
    k["poly1305"] = [{"key": "85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b",
                      "msg": hx(b"Cryptographic Forum Research Group"),
                      "tag": "a8061dc1305136c6c22b8baf0c0127a9"}]
    # RFC 8439 §2.3.2 ChaCha20 block
    k["chacha20_block"] = [{"key": hx(bytes(range(32))), "counter": 1,
                            "nonce": "000000090000004a00000000",
                            "out": "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                                   "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e"}]
    k["sha3_256"] = [{"msg": "", "out": "a7ffc6f8bf1ed76651c14756a061d662f580ff4de43b49fa82d80a4b80f8434a"},
                     {"msg": hx(b"abc"), "out": "3a985da74fe225b2045c172d6bd390bd855f086e3e9d525b46bfe24511431532"}]
    for n in [1, 135, 136, 137, 271, 272, 1000]:
        m = rng.randbytes(n)
        k["sha3_256"].append({"msg": hx(m), "out": hashlib.sha3_256(m).hexdigest()})
    k["base32_nopad"] = [{"in": hx(s.encode()), "out": b32(s.encode())}
                         for s in ["", "f", "fo", "foo", "foob", "fooba", "foobar"]]
    k["base32_nopad"].append({"in": hx(bytes(range(32))), "out": b32(bytes(range(32)))})
    return k


def make_repo(rng):
    """A 4-actor GCounter op repository (16 versions per actor) + a state file."""
    key = rng.randbytes(32)
    key1 = rng.randbytes(32)
    actors = sorted(rng.randbytes(16) for _ in range(4))
    files = []
    nov = {}
    st = {}
    plains = []
    file_dots = []
    for ai, a in enumerate(actors):
        ctr = 0
        for v in range(16):
            ndots = rng.choice([0, 1, 2, 5, 17, 40])
            dots = []
            for _ in range(ndots):
                if rng.random() < 0.8:
                    ctr += rng.choice([1, 1, 2, 100, 70000, 1 << 33])
                    dots.append((a, ctr))
                else:
                    dots.append((rng.choice(actors), rng.randrange(0, 1 << 20)))
            f, clear = op_file(key, rng.randbytes(24), dots)
            files.append({"actor": hx(a), "version": v, "file": hx(f),
                          "clear_sha256": hashlib.sha256(clear).hexdigest()})
            plains.append(clear)
            file_dots.append(dots)
            for da, dc in dots:
                if st.get(da, 0) < dc:
                    st[da] = dc
            nov[a] = v + 1
    expected = {kind: hx(state_wrapper_bytes(kind, nov, st)) for kind in ("gcounter", "vclock")}

    # a state file in the ingest format (outer CURRENT_VERSION, inner data-version prefix)
    st2 = {actors[0]: 5, actors[1]: (1 << 40) + 3, rng.randbytes(16): 9}
    nov2 = {actors[0]: 30, actors[3]: 2}
    state_files = {}
    merged = {}
    for kind in ("gcounter", "vclock"):
        sw = state_wrapper_bytes(kind, nov2, st2)
        sf = CORE_VERSION + cryptor_encrypt(key, rng.randbytes(24), APP_VERSION + sw)
        state_files[kind] = hx(sf)
        # read_remote_states (lib.rs:458-466) then read_remote_ops with the version gate
        # (lib.rs:519-538): files with version < next_op_versions[actor] are skipped.
        m_st = dict(st2); m_nov = dict(nov2)
        for f, dots in zip(files, file_dots):
            a = bytes.fromhex(f["actor"])
            if f["version"] < m_nov.get(a, 0):
                continue
            assert f["version"] == m_nov.get(a, 0)
            for da, dc in dots:
                if m_st.get(da, 0) < dc:
                    m_st[da] = dc
            m_nov[a] = m_nov.get(a, 0) + 1
        merged[kind] = hx(state_wrapper_bytes(kind, m_nov, m_st))

    # compact output: cryptor.encrypt(msgpack(StateWrapper)) tagged with current_data_version
    # (lib.rs:336,358,360) and named BASE32_NOPAD(SHA3-256(file)) (tokio lib.rs:403-432)
    cnonce = rng.randbytes(24)
    comp = {}
    for kind in ("gcounter", "vclock"):
        clear = bytes.fromhex(expected[kind])
        sealed = APP_VERSION + cryptor_encrypt(key, cnonce, clear)
        comp[kind] = {"nonce": hx(cnonce), "file": hx(sealed),
                      "name": b32(hashlib.sha3_256(sealed).digest())}
    return {"key": hx(key), "key1": hx(key1), "data_version": hx(APP_VERSION),
            "actors": [hx(a) for a in actors], "files": files, "expected_state": expected,
            "state_files": state_files, "expected_after_state_then_ops": merged,
            "compact": comp}


def make_negatives(rng, key):
    """Per-file status cases in the reference's check order (include/crdtenc.h codes).
    'pinned' = the expected status follows from byte-level facts checked in this container;
    unpinned cases follow the recalled rmp-serde/serde acceptance rules."""
    A = rng.randbytes(16)
    dots = [(A, 1), (A, 2), (A, 300)]
    clear = APP_VERSION + msgpack.packb([{"actor": a, "counter": c} for a, c in dots], use_bin_type=True)
    nonce = rng.randbytes(24)
    ct = xchacha_seal(key, nonce, clear)
    good = CORE_VERSION + msgpack.packb([BOX_VERSION, enc_box(nonce, ct)], use_bin_type=True)
    cases = [("good", good, 0, True)]

    def box(vbox_obj):
        return CORE_VERSION + msgpack.packb(vbox_obj, use_bin_type=True)

    t = bytearray(good); t[-1] ^= 1
    cases.append(("tampered_tag", bytes(t), 9, True))
    t = bytearray(good); t[-40] ^= 0x80
    cases.append(("tampered_ct", bytes(t), 9, True))
    key1 = rng.randbytes(32)
    cases.append(("wrong_key", CORE_VERSION + cryptor_encrypt(key1, nonce, clear), 9, True))
    cases.append(("short_file", CORE_VERSION[:15], 1, True))
    cases.append(("outer_version", bytes(16) + good[16:], 2, True))
    cases.append(("vbox_not_array", CORE_VERSION + b"\xc0", 5, True))
    cases.append(("vbox_map", box({"0": BOX_VERSION, "1": enc_box(nonce, ct)}), 5, False))
    cases.append(("vbox_3_elems", box([BOX_VERSION, enc_box(nonce, ct), 1]), 5, False))
    cases.append(("vbox_truncated", good[:40], 5, True))
    cases.append(("box_version", box([bytes(16), enc_box(nonce, ct)]), 6, True))
    cases.append(("encbox_garbage", box([BOX_VERSION, b"\x01\x02"]), 7, True))
    cases.append(("encbox_missing_nonce",
                  box([BOX_VERSION, msgpack.packb({"enc_data": ct}, use_bin_type=True)]), 7, True))
    dup = (b"\x83" + msgpack.packb("nonce") + msgpack.packb(nonce, use_bin_type=True)
           + msgpack.packb("nonce") + msgpack.packb(nonce, use_bin_type=True)
           + msgpack.packb("enc_data") + msgpack.packb(ct, use_bin_type=True))
    cases.append(("encbox_dup_field", box([BOX_VERSION, dup]), 7, False))
    cases.append(("encbox_array_form",
                  box([BOX_VERSION, msgpack.packb([nonce, ct], use_bin_type=True)]), 0, False))
    cases.append(("encbox_reordered",
                  box([BOX_VERSION, msgpack.packb({"enc_data": ct, "nonce": nonce}, use_bin_type=True)]), 0, False))
    cases.append(("encbox_extra_field",
                  box([BOX_VERSION, msgpack.packb({"x": [1, {"y": None}], "nonce": nonce, "enc_data": ct},
                                                  use_bin_type=True)]), 0, False))
    cases.append(("encbox_str_fields",
                  box([BOX_VERSION, msgpack.packb({"nonce": nonce, "enc_data": ct}, use_bin_type=False)]), 0, False))
    n23 = nonce[:23]
    cases.append(("nonce_23", box([BOX_VERSION, enc_box(n23, ct)]), 8, True))
    cases.append(("ct_too_short", box([BOX_VERSION, enc_box(nonce, ct[:15])]), 9, True))
    cases.append(("trailing_bytes", good + b"\x00\xff", 0, False))

    def sealed(cl):
        return CORE_VERSION + cryptor_encrypt(key, rng.randbytes(24), cl)
    cases.append(("pt_short", sealed(APP_VERSION[:15]), 10, True))
    cases.append(("pt_version", sealed(bytes(16) + clear[16:]), 11, True))
    cases.append(("pt_garbage", sealed(APP_VERSION + b"\xc1"), 12, True))
    cases.append(("pt_empty_vec", sealed(APP_VERSION + b"\x90"), 0, True))
    cases.append(("dot_array_form", sealed(APP_VERSION + msgpack.packb([[A, 7]], use_bin_type=True)), 0, False))
    cases.append(("dot_negative", sealed(APP_VERSION + msgpack.packb([{"actor": A, "counter": -1}], use_bin_type=True)), 12, False))
    cases.append(("dot_int_keys", sealed(APP_VERSION + msgpack.packb([{0: A, 1: 5}], use_bin_type=True)), 0, False))
    cases.append(("dot_uuid_str", sealed(APP_VERSION + msgpack.packb([{"actor": "a" * 16, "counter": 5}], use_bin_type=True)), 12, False))
    cases.append(("dot_uuid_15", sealed(APP_VERSION + msgpack.packb([{"actor": A[:15], "counter": 5}], use_bin_type=True)), 12, True))
    cases.append(("dot_missing_counter", sealed(APP_VERSION + msgpack.packb([{"actor": A}], use_bin_type=True)), 12, False))
    cases.append(("dot_u64_max", sealed(APP_VERSION + msgpack.packb([{"actor": A, "counter": (1 << 64) - 1}], use_bin_type=True)), 0, True))
    cases.append(("dot_float", sealed(APP_VERSION + msgpack.packb([{"actor": A, "counter": 1.0}], use_bin_type=True)), 12, False))
    cases.append(("vec_is_map", sealed(APP_VERSION + msgpack.packb({"a": 1}, use_bin_type=True)), 12, False))
    cases.append(("pt_trailing", sealed(clear + b"\xc1\xc1"), 0, False))
    return [{"name": n, "file": hx(f), "status": s, "pinned": p} for n, f, s, p in cases]


def main():
    rng = random.Random(0xC0FFEE)
    kats = make_kats(rng)
    repo = make_repo(rng)
    negs = make_negatives(rng, bytes.fromhex(repo["key"]))
    repo["negatives"] = negs
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kats, f, indent=1)
    with open(os.path.join(HERE, "repo_gcounter.json"), "w") as f:
        json.dump(repo, f, indent=1)
    print("wrote kat.json, repo_gcounter.json")


if __name__ == "__main__":
    main()
