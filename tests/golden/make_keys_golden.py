#!/usr/bin/env python3
"""Generate tests/golden/keys.json: Keys / remote-meta wire bytes and the key Keys::latest_key
picks (crdt-enc/src/key_cryptor.rs:35-82; crdt-enc/src/lib.rs:553-612,647-664;
crdt-enc-gpgme/src/lib.rs:79-129).  Run once in the build container:

    python tests/golden/make_keys_golden.py

The Keys histories are simulated with oracle/keys.py (insert_latest_key as the reference
applies it: an Orswot Add under the replica's next dot and an MVReg Put under the register's
read clock incremented for the replica), written in the rmp-serde to_vec_named forms of
SURVEY.md Appendix A.  The reference cannot be built here and its tests cover
none of this, so these vectors are parity-unpinned restatements: they pin the product
(crdt-enc_amd/csrc/ce_keys.cpp) to oracle/keys.py, not to crdts 7 itself."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import crdts as C  # noqa: E402
from oracle import keys as K  # noqa: E402


def main():
    rng = random.Random(0x4B455953)
    A, B = sorted(rng.randbytes(16) for _ in range(2))
    ids = [rng.randbytes(16) for _ in range(4)]
    mats = [rng.randbytes(32) for _ in range(4)]
    cases = []

    def add(name, keys, note):
        lk = None
        try:
            r = keys.latest_key()
            lk = None if r is None else {"id": r[0].hex(), "version": r[1][0].hex(), "key": r[1][1].hex()}
            err = None if r is not None else "no_key"
        except KeyError:
            err = "missing"
        cases.append({"name": name, "note": note, "keys": keys.to_bytes().hex(), "latest": lk,
                      "error": err, "count": len(keys.keys.entries)})

    k = K.Keys()
    k.insert_latest_key(A, ids[0], mats[0])
    add("single", k, "one insert_latest_key by replica A")
    base = K.decode_keys(k.to_bytes())

    k.insert_latest_key(A, ids[1], mats[1])
    add("rotated", k, "A inserts a second key: its Put clock {A:2} dominates {A:1}")
    ka = K.decode_keys(k.to_bytes())

    kb = K.decode_keys(base.to_bytes())
    kb.insert_latest_key(B, ids[2], mats[2])
    add("replica_b", kb, "B inserts its own key on the state after A's first insert")

    m = K.decode_keys(ka.to_bytes())
    m.merge(K.decode_keys(kb.to_bytes()))
    add("concurrent_merged", m, "A's rotation merged with B's concurrent insert: two latest ids, "
                                "latest_key = the smaller id")

    miss = K.decode_keys(base.to_bytes())
    miss.latest.vals.append((C.VClock({B: 5}), ids[3]))
    add("latest_without_key", miss, "a latest id no key carries: the reference panics "
                                   "(key_cryptor.rs:67)")
    add("empty", K.Keys(), "no key at all: latest_key() is None (lib.rs:420 'no latest key')")
    rep = K.decode_keys(base.to_bytes())
    rep.latest.vals.append((C.VClock({B: 5}), rep.latest.vals[0][1]))
    add("repeated_latest_id", rep, "two concurrent register values name the same key id: "
                                   "keys.take(&id) removed it on the first, so the reference "
                                   "panics on the second (key_cryptor.rs:60-67)")

    # remote metas: two files whose key_cryptor registers hold concurrent Keys values
    reg_a = [(C.VClock({A: 1}), (K.GPGME_VERSION, ka.to_bytes()))]
    reg_b = [(C.VClock({B: 1}), (K.GPGME_VERSION, kb.to_bytes()))]
    f1, f2 = K.remote_meta_bytes(reg_a), K.remote_meta_bytes(reg_b)
    merged = K.keys_from_remote_metas([f1, f2])
    r = merged.latest_key()
    bad = K.remote_meta_bytes([(C.VClock({A: 2}), (bytes(16), ka.to_bytes()))])
    metas = {"files": [f1.hex(), f2.hex()], "latest": {"id": r[0].hex(), "version": r[1][0].hex(),
                                                       "key": r[1][1].hex()},
             "count": len(merged.keys.entries), "bad_version_file": bad.hex(),
             "single_file_latest": K.keys_from_remote_metas([f1]).latest_key()[0].hex()}
    out = {"generator": "tests/golden/make_keys_golden.py (oracle/keys.py restatement; parity "
                        "unpinned)", "cases": cases, "remote_metas": metas}
    with open(os.path.join(HERE, "keys.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
