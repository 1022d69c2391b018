"""Child process of tests/test_gpu_dotset.py::test_scan_forms_equal: the same adversarial Orswot
batch as the parent (seed 31337), ingested on cuda:0 under whatever scan form the environment
selects; prints "<rc> <sha256 of the state bytes>"."""
import hashlib
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "crdt-enc_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)

import crdtenc  # noqa: E402
import dotset_gen as G  # noqa: E402

APP = bytes.fromhex("aadfd5a66e194b24a8024fa27c72f20c")


def main():
    rng = random.Random(31337)
    key = rng.randbytes(32)
    actors = G.actors_for(rng, 256)
    files = G.adversarial_orswot(rng, actors, 16, 6, 5000)
    acts, clears, fa, fv = G.batch(files, "orswot", APP)
    ctx = crdtenc.Context(0)
    sealed = [crdtenc.CORE_VERSION + e for e in ctx.encrypt_batch(key, clears)]
    core = crdtenc.Core(ctx, kind=crdtenc.STATE_ORSWOT, supported=[APP], current_data_version=APP)
    core.set_latest_key(key)
    rc = core.ingest_ops(sealed, acts, fa, fv)[0]
    print("%d %s" % (rc, hashlib.sha256(core.state_bytes()).hexdigest()))
    core.close()
    ctx.close()


if __name__ == "__main__":
    main()
