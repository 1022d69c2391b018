"""Pinned host -> device copy rate in a torch process (the HIP runtime torch loads): 32 MiB chunks
back to back on one stream, on two streams alternating, and 128 MiB chunks; GB/s each."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "crdt-enc_amd"))
import crdtenc  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
TOT = 2 << 30
dev = torch.empty(TOT, dtype=torch.uint8, device="cuda")
src = crdtenc.host_buffer(128 << 20)
src[:] = 3
streams = [torch.cuda.Stream() for _ in range(2)]


def run(chunk, nstreams):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k, off in enumerate(range(0, TOT, chunk)):
        s = streams[k % nstreams]
        rc = hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr() + off), ctypes.c_void_p(src.ctypes.data),
                                ctypes.c_size_t(chunk), 1, ctypes.c_void_p(s.cuda_stream))
        assert rc == 0
    torch.cuda.synchronize()
    return TOT / (time.perf_counter() - t) / 1e9


for rep in range(2):
    print("chunk 32 MiB 1 stream %.1f GB/s | 2 streams %.1f | chunk 128 MiB 1 stream %.1f" % (
        run(32 << 20, 1), run(32 << 20, 2), run(128 << 20, 1)))
