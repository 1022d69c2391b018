"""The multi-rank code paths under RCCL ("nccl" is RCCL on ROCm): a one-rank process group on
the box's one GPU, so shard.ingest_sharded (the gate statistics' all_reduce(MAX) of flipped-sign
u64 words, the dense batch's all_reduce, the state all-gather of the "bytes" path) and
shard.ingest_dotset_sharded (the status all_reduce, the column path's length all_gather) run on
device tensors through RCCL and its stream handling, with the results the gloo tests check
(the 8-GPU node runs the same code with N ranks)."""
import os
import socket
import subprocess
import sys

import msgpack
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, mode):
    out = str(tmp_path / "n")
    env = dict(os.environ, CE_TEST_BACKEND="nccl")
    p = subprocess.run([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"), "0", "1",
                        str(_port()), mode, out], env=env, capture_output=True, timeout=240)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    with open(out + ".0", "rb") as f:
        return f.read()


@pytest.mark.parametrize("name,want_rc,want_path", [
    ("clean", 0, "dense"), ("gap", 13, "dense"), ("tamper", 9, "rejected"), ("unregistered", 0, "bytes"),
])
def test_one_rank_rccl_sharded_ingest(tmp_path, name, want_rc, want_path):
    from test_shard import _scenario, _expected
    key, writers, _, files, fa, fv, pre = _scenario(name)
    want_rc2, want = _expected(name, key, writers, files, fa, fv, pre)
    assert want_rc2 == want_rc
    rc, path, n, state, start = msgpack.unpackb(_run(tmp_path, "sharded:" + name), raw=False)
    assert (rc, path, n) == (want_rc, want_path, len(files))
    assert state == (start if want is None else want)


def test_one_rank_rccl_dotset(tmp_path):
    import multi_rank_worker as W
    from oracle import crdts as C
    APP = W.APP
    key, actors, files, fa, fv = W.workload_orswot()
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)[0] == 0
    tag, state = _run(tmp_path, "orswot_tree").split(b"\n", 1)
    assert tag == b"tree 0 0" and state == oc.serialize()
