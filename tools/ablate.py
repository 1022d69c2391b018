"""Diagnostics: time k_open_fold_small with phases switched off (CE_ABLATE bits).  Results are
invalid by construction; only the kernel time matters.  Run: python tools/ablate.py BITS"""
import os, sys, time
sys.argv = [sys.argv[0]] + ["--versions", "64", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-variant-b",
                           "--no-host-buffers", "--configs", ""]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench, crdtenc, torch
orig = crdtenc.Core.ingest_ops_device
def patched(self, *a, **k):
    orig(self, *a, **k)
    return 0
crdtenc.Core.ingest_ops_device = patched
orig_c = crdtenc.Core.compact_ops_device
def patched_c(self, *a, **k):
    orig_c(self, *a, **k)
    return 0, b"", None
crdtenc.Core.compact_ops_device = patched_c
crdtenc.Core.state_bytes = lambda self: b""
bench.main()
