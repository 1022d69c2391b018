"""Which engine the HIP runtime in a torch process uses for a 35 MB device -> pinned host copy,
and how it slows a 512 MB fill beside it (env knobs A/B; run once per setting)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "crdt-enc_amd"))
import crdtenc  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
N = 35 << 20
src = torch.full((N,), 7, dtype=torch.uint8, device="cuda")
big = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
dst = crdtenc.host_buffer(N)
s2 = torch.cuda.Stream()
s1 = torch.cuda.current_stream()


def copy():
    rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(N),
                            2, ctypes.c_void_p(s2.cuda_stream))
    assert rc == 0, rc


def timed(fn, stream):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    fn()
    b.record(stream)
    return a, b


for rep in range(3):
    torch.cuda.synchronize()
    fa, fb = timed(lambda: big.fill_(1), s1)
    torch.cuda.synchronize()
    ca, cb = timed(copy, s2)
    torch.cuda.synchronize()
    alone_fill, alone_copy = fa.elapsed_time(fb), ca.elapsed_time(cb)
    ca, cb = timed(copy, s2)
    fa, fb = timed(lambda: big.fill_(2), s1)
    torch.cuda.synchronize()
    print("%s rep %d: copy alone %.0f us, fill alone %.0f us | together: copy %.0f us, fill %.0f us; ok %s" % (
        os.environ.get("PROBE_TAG", "default"), rep, alone_copy * 1e3, alone_fill * 1e3,
        ca.elapsed_time(cb) * 1e3, fa.elapsed_time(fb) * 1e3, bool(dst[12345] == 7)))
