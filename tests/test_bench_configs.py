"""The C3 generator of bench_configs.py writes valid Vec<orswot::Op<u64, Uuid>> plaintexts with
the intended dots/members (checked with the oracle's decoder, CPU only)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench_configs as B  # noqa: E402
from oracle import crdts as C  # noqa: E402


def test_c3_plaintexts_decode():
    actors = B.actors_table()
    a = torch.tensor([0, 5, 4095], dtype=torch.int64)
    v = torch.tensor([0, 3, 17], dtype=torch.int64)
    pts = B.orswot_clears(actors, a, v, "cpu")
    assert pts.shape == (3, B.PT_LEN)
    for i in range(3):
        b = bytes(pts[i].numpy())
        assert b[:16] == B.APP
        ops = C.dec_ops("orswot", b[16:])
        assert len(ops) == B.N_ADD + B.N_RM
        ai, vi = int(a[i]), int(v[i])
        for j in range(B.N_ADD):
            kind, (act, ctr), ms = ops[j]
            assert kind == "Add" and act == bytes(actors[ai]) and ctr == vi * B.N_ADD + j + 1
            assert ms == [int(B.member_of(torch.tensor(ai), torch.tensor(vi), torch.tensor(j)))]
        for k in range(B.N_RM):
            kind, clock, ms = ops[B.N_ADD + k]
            jv = (k * 5 + 3) % B.N_ADD
            vv = vi - 1 if vi else vi
            assert kind == "Rm" and clock.dots == {bytes(actors[ai]): vv * B.N_ADD + jv + 1}
            assert ms == [int(B.member_of(torch.tensor(ai), torch.tensor(vv), torch.tensor(jv)))]


def test_c4_plaintexts_decode():
    """C4's Vec<Dot> plaintexts: rmp-serde's smallest array header at every size class, the
    actor's UUID and consecutive counters (checked with msgpack, CPU only)."""
    import msgpack
    import numpy as np
    u = np.arange(16, dtype=np.uint8)
    for k in (1, 15, 16, 300, 65535, 65536):
        pt = B.dots_plaintext(u, k, 65536 + 7)
        assert pt[:16] == B.APP
        want = [{"actor": bytes(range(16)), "counter": 65536 + 7 + i + 1} for i in range(k)]
        assert msgpack.packb(want, use_bin_type=True) == pt[16:]
