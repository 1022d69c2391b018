"""C2 at its full size through the GPU path (missing 4).

1,048,576 x 4 KiB op files from 4096 actors sealed on the GPU (bench.build_files, the bench's
own generator): a 4.39 GB blob, so the files of the last ~190 actors start past 2^32 and every
offset / in_off of theirs needs its high word.  Core::compact runs through
ce_core_compact_ops_device_into (read_remote_ops + compaction output, crdt-enc/src/lib.rs:
332-380, 471-547).  Checked:
  - the sealed compaction opens under the oracle's AEAD (xchacha lib.rs:73-101) to exactly the
    StateWrapper<GCounter> the closed form gives (every actor at 65536 + 256 * 107, next op
    version 256), and its content name is the oracle's SHA3-256/BASE32 of the file;
  - the oracle folds a sample of whole actors spread over the blob -- the first, one in the
    middle, and the last two, whose files lie past 4 GiB -- and their counters and next op
    versions equal the GPU state's.
"""
import os
import sys

import msgpack
import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import crdtenc  # noqa: E402
import oracle  # noqa: E402

pytestmark = pytest.mark.gpu
VERSIONS = 256
SAMPLE = (0, 1, 2048, 4094, 4095)


def test_c2_full_size_past_4gib():
    dev = torch.device("cuda:0")
    ctx = crdtenc.Context(0)
    actors = bench.actors_table()
    key = bytes(np.random.default_rng(7).integers(0, 256, 32, dtype=np.uint8))
    files, offs, n, blob_len, _ = bench.build_files(ctx, key, actors, actors, VERSIONS, dev, seed=1234)
    assert n == 1 << 20 and blob_len > (1 << 32) + (64 << 20)
    flen = blob_len // n
    assert flen * bench.N_ACTORS * VERSIONS == blob_len
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_GCOUNTER, supported=[bench.APP], current_data_version=bench.APP)
    core.set_latest_key(key)
    fa = np.repeat(np.arange(bench.N_ACTORS, dtype=np.int32), VERSIONS)
    fv = np.tile(np.arange(VERSIONS, dtype=np.int64), bench.N_ACTORS)
    fa_d, fv_d = torch.from_numpy(fa).to(dev), torch.from_numpy(fv).to(dev)
    act_bytes = b"".join(bytes(a) for a in actors)
    bound = 16 + crdtenc.sealed_len(69 + 54 * 8192)
    out = torch.empty(bound, dtype=torch.uint8, pin_memory=True).numpy()
    rc, ln, name = core.compact_ops_device_into(out, files.data_ptr(), offs.data_ptr(), n, blob_len,
                                                act_bytes, fa_d.data_ptr(), fv_d.data_ptr(),
                                                nonce=bytes(24), name=True)
    assert rc == 0, core.ctx.last_error()
    f = bytes(out[:ln])
    want = bench.expected_state(actors, VERSIONS)
    assert f[:16] == bench.APP
    st, pt = oracle.cryptor_decrypt(key, f[16:])
    assert st == 0 and pt == want
    assert name == oracle.base32_nopad(oracle.sha3_256(f))
    gpu = msgpack.unpackb(core.state_bytes(), raw=False)
    # the oracle over whole actors, the last two past 4 GiB
    sample_files, sample_act, sample_ver = [], [], []
    for a in SAMPLE:
        lo = a * VERSIONS * flen
        if a >= 4094:
            assert lo > (1 << 32)
        host = files[lo: lo + VERSIONS * flen].cpu().numpy().tobytes()
        for v in range(VERSIONS):
            sample_files.append(host[v * flen:(v + 1) * flen])
            sample_act.append(bytes(actors[a]))
            sample_ver.append(v)
    oc = oracle.Core()
    orc, ost = oc.read_remote_ops(key, [bench.APP], sample_files, sample_act, sample_ver)
    assert orc == 0 and set(ost) == {0}
    osw = msgpack.unpackb(oc.serialize(), raw=False)
    assert sorted(osw["state"]["inner"]["dots"]) == sorted(bytes(actors[a]) for a in SAMPLE)
    for a in SAMPLE:
        u = bytes(actors[a])
        assert osw["state"]["inner"]["dots"][u] == gpu["state"]["inner"]["dots"][u] == 65536 + VERSIONS * 107
        assert osw["next_op_versions"]["dots"][u] == gpu["next_op_versions"]["dots"][u] == VERSIONS
    core.close()
    ctx.close()
    del files, offs, fa_d, fv_d
    torch.cuda.empty_cache()
