"""C3 read-context removals at a small size: where do the writer-sharded fold + merge and the
whole fold part?  GPU whole vs the C restatement over every file; GPU shard states vs the C
restatement over each shard; the GPU merge of the two shards vs the Python restatement's
Orswot::merge of the C shard states (oracle/crdts.py)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "crdt-enc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench_configs as B  # noqa: E402
import crdtenc  # noqa: E402
import oracle  # noqa: E402
from oracle import crdts as C  # noqa: E402


def main():
    V0, V = int(os.environ.get("V0", "1")), int(os.environ.get("V", "2"))
    dev = torch.device("cuda", 0)
    ctx = crdtenc.Context(0)
    actors = B.actors_table()
    key = bytes(np.random.default_rng(7).integers(0, 256, 32, dtype=np.uint8))
    N, per = B.N_ACTORS, B.N_ACTORS // 8
    states = []
    for j in range(8):
        f, o, n, bl, fa, fv = B.seal_op_files(ctx, key, actors, j * per, (j + 1) * per, 0, V0, dev, 99 + j)
        sc = B.new_core(ctx, key, flags=crdtenc.COMPACT_INGEST_FORMAT)
        assert sc.ingest_ops_device(f.data_ptr(), o.data_ptr(), n, bl, b"".join(bytes(a) for a in actors[j * per:(j + 1) * per]),
                                    fa.data_ptr(), fv.data_ptr()) == 0
        states.append(sc.compact_to_buffer(nonce=bytes(24))[0])
        sc.close()
    files, offs, n, blob_len, fa, fv = B.seal_op_files(ctx, key, actors, 0, N, V0, V0 + V, dev, 1234, rm_ctx="read", V0=V0)
    hb = files[:blob_len].cpu().numpy()
    ho = offs.cpu().numpy().astype(np.uint64)
    ha = actors[fa.cpu().numpy()]
    hv = fv.cpu().numpy().astype(np.uint64)
    print("built", n, blob_len, flush=True)
    out = {}
    err, cw, _, _ = oracle.compact_orswot_best(key, B.APP, states, hb, ho, ha, hv, 8, seal=False)
    print("c whole", err, len(cw), flush=True)
    whole = B.new_core(ctx, key)
    if os.environ.get("REGISTER", "1") == "1":
        whole.register_actors([bytes(a) for a in actors])
    assert whole.ingest_states(states)[0] == 0
    print("whole states", flush=True)
    assert whole.ingest_ops_device(files.data_ptr(), offs.data_ptr(), n, blob_len, b"".join(bytes(a) for a in actors),
                                   fa.data_ptr(), fv.data_ptr()) == 0
    print("whole ops", flush=True)
    gw = whole.state_bytes()
    print("whole bytes", len(gw), flush=True)
    out["gpu_whole_eq_c_whole"] = err == 0 and cw == gw
    parts, cparts = [], []
    for r in range(2):
        lo, hi = r * N // 2, (r + 1) * N // 2
        f0, f1 = lo * V, hi * V
        b0, b1 = int(offs[f0]), int(offs[f1])
        p = B.new_core(ctx, key)
        assert p.ingest_states(states[4 * r:4 * r + 4])[0] == 0
        so = (offs[f0:f1 + 1] - b0).contiguous()
        assert p.ingest_ops_device(files[b0:b1].data_ptr(), so.data_ptr(), f1 - f0, b1 - b0,
                                   b"".join(bytes(a) for a in actors[lo:hi]),
                                   (fa[f0:f1] - lo).contiguous().data_ptr(), fv[f0:f1].contiguous().data_ptr()) == 0
        parts.append(p)
        print("part", r, flush=True)
    out["gpu_whole_eq_c_whole"] = gw == cw
    # the C restatement's merge of the GPU's two shard states (sealed as state files: CORE ||
    # encrypt(APP || state)); the C fold of a shard is slow (its deferred removals)
    gparts = [p.state_bytes() for p in parts]
    sfs = [crdtenc.CORE_VERSION + e for e in ctx.encrypt_batch(key, [B.APP + c for c in gparts])]
    empty = np.zeros(1, np.uint64)
    err, cmerged, _, _ = oracle.compact_orswot_best(key, B.APP, sfs, b"\0", empty, np.zeros((0, 16), np.uint8),
                                                    np.zeros(0, np.uint64), 8, seal=False)
    out["c_merge_of_gpu_parts_eq_c_whole"] = err == 0 and cmerged == cw
    print("c merge", out, flush=True)
    g1 = parts[1].state_bytes()
    assert parts[0].merge_state(g1) == 0
    gm = parts[0].state_bytes()
    out["gpu_merge_eq_c_merge"] = gm == cmerged
    out["gpu_merge_eq_gpu_whole"] = gm == gw
    seq = B.new_core(ctx, key)
    assert seq.merge_state(gparts[0]) == 0 and seq.merge_state(gparts[1]) == 0
    out["gpu_seq_merge_eq_c_merge"] = seq.state_bytes() == cmerged
    if cmerged != cw:  # where: the members whose entries differ (merge of the shards vs the whole)
        gm = cmerged
        cmerged = cw
        import msgpack
        a = msgpack.unpackb(cmerged, raw=True, strict_map_key=False)[b"state"]
        b = msgpack.unpackb(gm, raw=True, strict_map_key=False)[b"state"]
        ea, eb = a[b"entries"], b[b"entries"]
        diff = [m for m in set(ea) | set(eb) if ea.get(m) != eb.get(m)]
        out["entries_whole_merged"] = [len(ea), len(eb)]
        out["n_diff_members"] = len(diff)
        out["clock_eq"] = a[b"clock"] == b[b"clock"]
        out["deferred_whole_merged"] = [len(a[b"deferred"]), len(b[b"deferred"])]
        ta = msgpack.unpackb(cmerged, raw=True, strict_map_key=False)
        tb = msgpack.unpackb(gm, raw=True, strict_map_key=False)
        out["nov_eq"] = ta[b"next_op_versions"] == tb[b"next_op_versions"]
        na_, nb_ = ta[b"next_op_versions"][b"dots"], tb[b"next_op_versions"][b"dots"]
        dn = [k for k in set(na_) | set(nb_) if na_.get(k) != nb_.get(k)]
        out["nov_diff"] = [(na_.get(k), nb_.get(k)) for k in dn[:5]]
        out["nov_len"] = [len(na_), len(nb_)]
        i = next((i for i in range(min(len(cmerged), len(gm))) if cmerged[i] != gm[i]), None)
        out["first_diff_byte"] = i
        if i is not None:
            out["ctx_whole"] = cmerged[max(0, i - 24):i + 24].hex()
            out["ctx_merged"] = gm[max(0, i - 24):i + 24].hex()
        act_ix = {bytes(x): i for i, x in enumerate(actors)}
        for m in diff[:4]:
            fmt = lambda e: None if e is None else {act_ix.get(k, -1): v for k, v in e[b"dots"].items()}
            print("member", m, "whole:", fmt(ea.get(m)), "merged:", fmt(eb.get(m)), flush=True)
        print(out, flush=True)
    os.environ["CE_NO_KMERGE"] = "1"
    print(out, flush=True)


if __name__ == "__main__":
    main()
