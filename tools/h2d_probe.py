"""H2D transfer rates on the box: pageable vs pinned host memory (torch), and host memcpy
rates (1 and 8 threads) -- sizing the pipelined host-buffer ingest."""
import time, threading, ctypes
import numpy as np
import torch

N = 1 << 30
dev = torch.device("cuda", 0)
d = torch.empty(N, dtype=torch.uint8, device=dev)
pag = torch.from_numpy(np.random.default_rng(0).integers(0, 255, N, dtype=np.uint8))
pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
pin.copy_(pag)
for name, src in (("pageable", pag), ("pinned", pin)):
    for _ in range(2):
        torch.cuda.synchronize(); t = time.perf_counter()
        d.copy_(src, non_blocking=True); torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print("H2D %s: %.1f GB/s" % (name, N / dt / 1e9), flush=True)
dst = np.empty(N, dtype=np.uint8)
src = pag.numpy()
for th in (1, 4, 8, 16):
    def part(i):
        lo, hi = i * N // th, (i + 1) * N // th
        ctypes.memmove(dst.ctypes.data + lo, src.ctypes.data + lo, hi - lo)
    for _ in range(2):
        t = time.perf_counter()
        ts = [threading.Thread(target=part, args=(i,)) for i in range(th)]
        [x.start() for x in ts]; [x.join() for x in ts]
        dt = time.perf_counter() - t
    print("host memcpy %d threads: %.1f GB/s" % (th, N / dt / 1e9), flush=True)
