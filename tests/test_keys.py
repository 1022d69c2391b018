"""The key path (crdt-enc/src/key_cryptor.rs:35-82, lib.rs:553-612, crdt-enc-gpgme/src/lib.rs:
79-129) through the product's C ABI (host code: no GPU needed) and the oracle restatement,
against tests/golden/keys.json (tests/golden/make_keys_golden.py; parity unpinned -- the wire
forms and crdts 7 semantics are restated)."""
import json
import os

import pytest

import crdtenc

H = bytes.fromhex
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def keys_fx():
    with open(os.path.join(REPO, "tests", "golden", "keys.json")) as f:
        return json.load(f)


def test_oracle_reproduces_fixture(keys_fx):
    from oracle import keys as K
    for c in keys_fx["cases"]:
        k = K.decode_keys(H(c["keys"]))
        assert len(k.keys.entries) == c["count"], c["name"]
        if c["error"] == "missing":
            with pytest.raises(KeyError):
                k.latest_key()
        elif c["error"] == "no_key":
            assert k.latest_key() is None
        else:
            i, (ver, key) = k.latest_key()
            assert (i.hex(), ver.hex(), key.hex()) == (c["latest"]["id"], c["latest"]["version"],
                                                     c["latest"]["key"]), c["name"]
        assert k.to_bytes().hex() == c["keys"]          # canonical re-encode round trip
    m = keys_fx["remote_metas"]
    k = K.keys_from_remote_metas([H(f) for f in m["files"]])
    assert k.latest_key()[0].hex() == m["latest"]["id"] and len(k.keys.entries) == m["count"]


@pytest.mark.parametrize("i", range(7))
def test_product_latest_key(keys_fx, i):
    c = keys_fx["cases"][i]
    k = crdtenc.Keys.decode(H(c["keys"]))
    assert len(k) == c["count"]
    if c["error"] == "missing":
        with pytest.raises(crdtenc.CeError) as e:
            k.latest()
        assert e.value.args[0] == 12 or "DECODE" in str(e.value)
    elif c["error"] == "no_key":
        with pytest.raises(crdtenc.CeError) as e:
            k.latest()
        assert "NO_KEY" in str(e.value) or e.value.args[0] == 66
    else:
        kid, ver, key = k.latest()
        assert (kid.hex(), ver.hex(), key.hex()) == (c["latest"]["id"], c["latest"]["version"],
                                                     c["latest"]["key"])
        assert k.get(kid) == (ver, key)


def test_product_merge_equals_fixture(keys_fx):
    cases = {c["name"]: c for c in keys_fx["cases"]}
    a = crdtenc.Keys.decode(H(cases["rotated"]["keys"]))
    b = crdtenc.Keys.decode(H(cases["replica_b"]["keys"]))
    a.merge(b)
    want = cases["concurrent_merged"]
    assert len(a) == want["count"]
    assert a.latest()[0].hex() == want["latest"]["id"]
    ids = [kid for kid, _, _ in a.items()]
    assert ids == sorted(ids)


def test_product_remote_metas(keys_fx):
    m = keys_fx["remote_metas"]
    k = crdtenc.Keys.from_remote_metas([H(f) for f in m["files"]])
    kid, ver, key = k.latest()
    assert (kid.hex(), ver.hex(), key.hex()) == (m["latest"]["id"], m["latest"]["version"], m["latest"]["key"])
    assert len(k) == m["count"]
    assert crdtenc.Keys.from_remote_metas([H(m["files"][0])]).latest()[0].hex() == m["single_file_latest"]
    with pytest.raises(crdtenc.CeError):
        crdtenc.Keys.from_remote_metas([H(m["bad_version_file"])])
    with pytest.raises(crdtenc.CeError):
        crdtenc.Keys.from_remote_metas([bytes(16) + H(m["files"][0])[16:]])
