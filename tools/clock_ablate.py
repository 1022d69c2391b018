"""Diagnostics: C2 (1M files) with phases of the fused kernel switched off (CE_ABLATE bits of
the diagnostics build) and the shader clock probed beside it.  Results are invalid by
construction (return codes and the state are ignored); only the kernel time and the clock
matter."""
import os
import sys
sys.argv = [sys.argv[0]] + ["--steps", "10", "--warmup", "1", "--no-cpu", "--no-variant-b",
                            "--no-host-buffers"]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import crdtenc  # noqa: E402
orig_c = crdtenc.Core.compact_ops_device


def patched_c(self, *a, **k):
    orig_c(self, *a, **k)
    return 0, b"", None


crdtenc.Core.compact_ops_device = patched_c
crdtenc.Core.state_bytes = lambda self: b""
bench.main()
