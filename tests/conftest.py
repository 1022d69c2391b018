import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "crdt-enc_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        k = json.load(f)
    with open(os.path.join(GOLDEN, "kat_xchacha.bin"), "rb") as f:
        side = f.read()
    for e in k["xchacha"]:
        o, n = e["bin_off"], e["len"]
        e["pt_bytes"] = side[o:o + n]
        e["ct_bytes"] = side[o + n:o + 2 * n + 16]
    return k


@pytest.fixture(scope="session")
def repo_fx():
    with open(os.path.join(GOLDEN, "repo_gcounter.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o
