"""Multi-rank runs of the product on the one GPU of the box (gloo group, every rank on
device 0; RCCL refuses two ranks on one device, and the driver's 8-GPU node runs the same code
over RCCL).  Covers the N>1 path end to end through the C ABI:
  * bench.py --gpus 2 launching its own ranks (CE_BENCH_SHARE_GPU=1, CE_DIST_BACKEND=gloo);
  * shard.exchange_vclock with every Dot on a registered actor (dense all_reduce(MAX) path) and
    with Dots on actors no rank registered (state all-gather + merge_state path), each merged
    state == the oracle's single fold over all files (crdt-enc/src/lib.rs:471-547)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_share_gpu():
    """bench.py --gpus 2 as the driver's scaling run would start it (here: gloo, both ranks on
    the one GPU): the weak C2 line, the strong C2 leg, and C3 / C3r / C4 / C5 at N = 2 under `configs`,
    each with every check true (small sizes: --quick)."""
    env = dict(os.environ, CE_BENCH_SHARE_GPU="1", CE_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--versions",
                        "2", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-variant-b", "--quick"],
                       env=env, capture_output=True, timeout=400)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    line = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["state_check"].endswith("ok")
    assert line["config"]["files_per_gpu"] == 4096 * 2
    assert "dense" in line["config"]["parallelism"]
    st = line["strong"]
    assert st["scaling"] == "strong" and st["state_check"].endswith("ok") and st["files_total"] == 4096 * 2
    for c in ("c3", "c3r", "c4", "c5"):
        cl = line["configs"][c]
        assert cl["n_gpus"] == 2 and cl["scaling"] == "strong", (c, cl)
        assert cl["checks"] and all(cl["checks"].values()), (c, cl["checks"])
    assert line["configs"]["c3"]["exchange"]["hops_per_step"] == 1
    assert line["configs"]["c3"]["exchange"]["max_state_bytes_per_hop"] > 0
    # C3's removals name the writer's own adds: no deferred removal, the partials go as columns
    assert line["configs"]["c3"]["exchange"]["per_hop_ms_max_over_ranks"]["exchange"] == "columns"
    assert line["configs"]["c5"]["config"]["path"] == "rejected"
    # read-context removals (c3r): writer shards defer removals naming the other shard's dots;
    # they travel in the columns' deferred section, still one merge on rank 0
    assert line["configs"]["c3r"]["exchange"]["per_hop_ms_max_over_ranks"]["exchange"] == "columns"


@pytest.mark.parametrize("mode,path", [("registered", "dense"), ("unregistered", "bytes")])
def test_exchange_vclock_two_processes(tmp_path, oracle, mode, path):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import multi_rank_worker as W
    key, actors, files, fa, fv = W.workload(mode)
    oc = oracle.Core(oracle.STATE_GCOUNTER)
    assert oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)[0] == 0
    want = oc.serialize()
    out = str(tmp_path / "m")
    port = str(_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"),
                               str(r), "2", port, mode, out]) for r in range(2)]
    rcs = [p.wait(timeout=180) for p in procs]
    assert rcs == [0, 0]
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            got_path, state = f.read().split(b"\n", 1)
        assert got_path.decode() == path
        assert state == want


def test_exchange_dotset_two_processes(tmp_path):
    """§8(e) for the dot sets: two ranks fold their writer shards of Orswot op files on the GPU,
    then shard.exchange_dotset all-gathers the partial StateWrappers over a real (gloo) group and
    each rank merges the other's with the GPU Orswot::merge (crdt-enc/src/lib.rs:458-466).  Both
    end with the oracle's single fold over every file."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import multi_rank_worker as W
    from oracle import crdts as C
    key, actors, files, fa, fv = W.workload_orswot()
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)[0] == 0
    want = oc.serialize()
    out = str(tmp_path / "d")
    port = str(_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"),
                               str(r), "2", port, "orswot", out]) for r in range(2)]
    rcs = [p.wait(timeout=180) for p in procs]
    assert rcs == [0, 0]
    for r in range(2):
        with open("%s.%d" % (out, r), "rb") as f:
            tag, state = f.read().split(b"\n", 1)
        assert tag == b"dotset" and state == want


def test_reduce_dotset_two_processes(tmp_path):
    """shard.ingest_dotset_sharded on the GPU: writer shards folded per rank, then the tree
    reduce -- rank 1 sends its StateWrapper, rank 0 merges it once (GPU Orswot::merge) and holds
    the oracle's single fold."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import multi_rank_worker as W
    from oracle import crdts as C
    key, actors, files, fa, fv = W.workload_orswot()
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)[0] == 0
    out = str(tmp_path / "t")
    port = str(_port())
    env = dict(os.environ, CE_DS_EXCHANGE="tree")
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"),
                               str(r), "2", port, "orswot_tree", out], env=env) for r in range(2)]
    assert [p.wait(timeout=180) for p in procs] == [0, 0]
    with open(out + ".0", "rb") as f:
        tag, state = f.read().split(b"\n", 1)
    # (CE_DS_EXCHANGE=tree: the serialized tree for partials with deferred removals)
    assert tag == b"tree 1 0" and state == oc.serialize()
    with open(out + ".1", "rb") as f:
        assert f.read().split(b"\n", 1)[0] == b"tree 0 0"


@pytest.mark.parametrize("world,exchange,p_rm", [(3, "columns", 0.0), (3, "tree", 0.0), (3, "columns", 0.2)])
def test_reduce_dotset_columns_three_processes(tmp_path, world, exchange, p_rm):
    """The column exchange: ranks 1..N-1 export their partial Orswot as columns
    (ce_core_export_columns_device), rank 0 merges all of them in one k-way merge
    (ce_core_merge_columns_device) and holds the oracle's single fold; CE_DS_EXCHANGE=tree takes
    the serialized binomial tree for the same files, with the same result.  p_rm 0.2: removals
    with the member's read context, so ranks hold deferred removals (the columns' deferred
    section)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import multi_rank_worker as W
    from oracle import crdts as C
    key, actors, files, fa, fv = W.workload_orswot(p_rm=p_rm)
    oc = C.Core("orswot")
    assert oc.read_remote_ops(key, [APP], files, [actors[i] for i in fa], fv)[0] == 0
    out = str(tmp_path / "t")
    port = str(_port())
    env = dict(os.environ)
    if exchange == "tree":
        env["CE_DS_EXCHANGE"] = "tree"
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "multi_rank_worker.py"),
                               str(r), str(world), port, "orswot_adds" if p_rm == 0.0 else "orswot_tree", out],
                              env=env) for r in range(world)]
    assert [p.wait(timeout=180) for p in procs] == [0] * world
    with open(out + ".0", "rb") as f:
        tag, state = f.read().split(b"\n", 1)
    assert state == oc.serialize()
    if exchange == "columns":
        assert tag == b"tree 1 1"          # one merge, the column form
        for r in range(1, world):
            with open("%s.%d" % (out, r), "rb") as f:
                assert f.read().split(b"\n", 1)[0] == b"tree 0 0"
    else:
        assert tag == b"tree 2 0"          # ceil(log2 3) serialized merges

