import os, random, sys
sys.path.insert(0, "crdt-enc_amd"); sys.path.insert(0, ".")
import msgpack, crdtenc, oracle
APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")
ctx = crdtenc.Context(0)
key = os.urandom(32)
rng = random.Random(3)
writers = [rng.randbytes(16) for _ in range(3)]
for n_others, ndots in [(50, 400), (3000, 400), (9000, 10), (9000, 400)]:
    others = [rng.randbytes(16) for _ in range(n_others)]
    clears = []
    for i in range(30):
        dots = [{"actor": rng.choice(others), "counter": rng.getrandbits(20)} for _ in range(ndots)]
        clears.append(APP + msgpack.packb(dots, use_bin_type=True))
    files = [crdtenc.CORE_VERSION + e for e in ctx.encrypt_batch(key, clears)]
    fa = [i % 3 for i in range(30)]
    order = sorted(range(30), key=lambda i: (fa[i], i))
    files = [files[i] for i in order]; fa = [fa[i] for i in order]
    vers, cnt = [], {}
    for a in fa:
        vers.append(cnt.get(a, 0)); cnt[a] = cnt.get(a, 0) + 1
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_VCLOCK, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    rc, st = core.ingest_ops(files, writers, fa, vers)
    oc = oracle.Core(oracle.STATE_VCLOCK)
    orc, ost = oc.read_remote_ops(key, [APP], files, [writers[i] for i in fa], vers)
    same = rc == 0 and core.state_bytes() == oc.serialize()
    print(n_others, ndots, "rc", rc, "oracle", orc, "statuses", st, "same", same, flush=True)
    # plain decrypt check of every file
    r2, st2, pts, raw, offs = ctx.decrypt_batch(key, [f[16:] for f in files])
    bad = [i for i in range(30) if pts[i] != clears[order[i]]]
    print("  decrypt mismatches:", bad, flush=True)
    core.close()
ctx.close()
