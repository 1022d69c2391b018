"""GPU parity of C4's fused decode (k_segments<false, true> + k_segdec_apply, ce_kernels.hip):
multi-page GCounter op files decoded inside the segment pass, against the oracle
(oracle/ce_oracle.c oc_read_remote_ops, crdt-enc/src/lib.rs:480-540) and against the separate
decode kernel (CE_SEGDEC=0).  Every case the records cannot prove -- another Dot length, a
second actor, a miss, a non-canonical Dot, a Dots past the array's count --
must fall back to the whole-file decode with the same result; state bytes are compared
bit-exactly.
"""
import os
import random

import msgpack
import pytest

import crdtenc

pytestmark = pytest.mark.gpu
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
CORE = crdtenc.CORE_VERSION
SEG = 16384  # plaintext bytes per segment (kSegBlocks * 16)


@pytest.fixture(scope="module")
def ctx():
    c = crdtenc.Context(0)
    yield c
    c.close()


def dot(actor, ctr):
    return msgpack.packb({"actor": actor, "counter": ctr}, use_bin_type=True)


def body(parts, count=None, hdr32=False):
    """VersionBytes(APP, Vec<Dot>) from pre-packed Dots (array header of `count`)."""
    n = len(parts) if count is None else count
    h = b"\xdd" + n.to_bytes(4, "big") if hdr32 else _arr_hdr(n)
    return APP + h + b"".join(parts)


def _arr_hdr(n):
    if n <= 15:
        return bytes([0x90 | n])
    if n < 65536:
        return b"\xdc" + n.to_bytes(2, "big")
    return b"\xdd" + n.to_bytes(4, "big")


def cases():
    rng = random.Random(77)
    writer, other, stranger = rng.randbytes(16), rng.randbytes(16), rng.randbytes(16)
    big = 1 << 20  # ce counters: 38-byte Dots
    uni = [dot(writer, big + 3 * i) for i in range(20000)]                 # ~760 KB, 47 segments
    out = {"uniform": body(uni)}
    # 35-byte Dots (cc counters) behind an array32 header: base 21, and 21 + k * 35 lands exactly
    # on segment 14's start (the Dot starting at a boundary belongs to the next segment)
    d35 = [dot(writer, 128 + (i * 7) % 128) for i in range(10000)]
    out["exact_boundary"] = body(d35, hdr32=True)
    assert (14 * SEG - 21) % 35 == 0
    # a second registered actor inside segment 5
    x = list(uni)
    x[5 * SEG // 38] = dot(other, big + 999999)
    out["second_actor_inside"] = body(x)
    # a second registered actor on the Dot crossing segment 1's end
    base = 16 + 3
    ks = (SEG - base) // 38
    x = list(uni)
    x[ks] = dot(other, big + 5)
    out["second_actor_straddler"] = body(x)
    # an unregistered actor (miss) in segment 20
    x = list(uni)
    x[20 * SEG // 38] = dot(stranger, big + 7)
    out["miss"] = body(x)
    # a shorter Dot (fixint counter) in the last segment
    x = list(uni)
    x[-3] = dot(writer, 5)
    out["length_change"] = body(x)
    # a non-canonical Dot (keys reordered) in segment 9
    x = list(uni)
    x[9 * SEG // 38] = msgpack.packb({"counter": big + 1, "actor": writer}, use_bin_type=True)
    out["non_canonical"] = body(x)
    # the first Dot non-canonical: no grid from the header
    x = list(uni)
    x[0] = msgpack.packb({"counter": big, "actor": writer}, use_bin_type=True)
    out["first_non_canonical"] = body(x)
    # Dots past the array's count (trailing canonical bytes)
    out["trailing_dots"] = body(uni, count=19000)
    # one segment, more than a page: decoded inside the segment kernel
    out["one_segment"] = body([dot(writer, big + i) for i in range(300)])
    # many actors throughout
    acts = [writer, other]
    out["two_actors_alternating"] = body([dot(acts[i % 2], big + i) for i in range(9000)])
    return writer, other, out


# (files folded from segment records, files decoded whole) per case
EXPECT = {
    "uniform": (1, 0), "exact_boundary": (1, 0), "second_actor_inside": (0, 1),
    "second_actor_straddler": (0, 1), "miss": (0, 1), "length_change": (0, 1),
    "non_canonical": (0, 1), "first_non_canonical": (0, 1), "trailing_dots": (0, 1),
    "one_segment": (0, 0), "two_actors_alternating": (0, 1),
}


@pytest.mark.parametrize("segdec", ["1", "0"])
def test_segment_decode_cases(ctx, monkeypatch, segdec):
    from oracle import Core as OCore
    monkeypatch.setenv("CE_SEGDEC", segdec)
    writer, other, cs = cases()
    names = list(cs)
    clears = [cs[k] for k in names]
    key = os.urandom(32)
    files = [CORE + e for e in ctx.encrypt_batch(key, clears)]
    n = len(files)
    for i, name in enumerate(names):  # each case alone: its own state vs the oracle's
        core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
        core.set_latest_key(key)
        rc, st = core.ingest_ops([files[i]], [writer, other], [0], [0])
        oc = OCore()
        orc, ost = oc.read_remote_ops(key, [APP], [files[i]], [writer], [0])
        assert (rc, st) == (orc, ost), name
        assert core.state_bytes() == oc.serialize(), name
        if segdec == "1":  # which path the file took (ce_core_path_count)
            rec, fb = core.path_count("segdec_records"), core.path_count("segdec_fallback")
            assert (rec, fb) == EXPECT[name], (name, rec, fb)
    # all together, then a tampered big file, then the batch again (every file gated off) + one more
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    rc, st = core.ingest_ops(files, [writer, other], [0] * n, list(range(n)))
    oc = OCore()
    orc, ost = oc.read_remote_ops(key, [APP], files, [writer] * n, list(range(n)))
    assert (rc, st) == (orc, ost)
    assert core.state_bytes() == oc.serialize()
    bad = bytearray(files[0])
    bad[len(bad) // 3] ^= 4
    rc, st = core.ingest_ops(files[:-1] + [bytes(bad)], [writer, other], [0] * n, list(range(n, 2 * n)))
    orc, ost = oc.read_remote_ops(key, [APP], files[:-1] + [bytes(bad)], [writer] * n, list(range(n, 2 * n)))
    assert (rc, st) == (orc, ost) and rc != 0
    assert core.state_bytes() == oc.serialize()
    extra = [CORE + e for e in ctx.encrypt_batch(key, [body([dot(writer, (1 << 40) + i) for i in range(2000)])])]
    rc, st = core.ingest_ops(files + extra, [writer, other], [0] * (n + 1), list(range(n + 1)))
    orc, ost = oc.read_remote_ops(key, [APP], files + extra, [writer] * (n + 1), list(range(n + 1)))
    assert (rc, st) == (orc, ost)
    assert core.state_bytes() == oc.serialize()
