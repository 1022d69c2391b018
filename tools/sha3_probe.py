"""Host SHA3-256 rates on this machine: one 35 MB buffer through ce_content_name (OpenSSL when
present), and k buffers at once through ce_content_names (AVX-512 multi-buffer)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "crdt-enc_amd"))
import crdtenc  # noqa: E402

big = [np.frombuffer(os.urandom(35 << 20), np.uint8) for _ in range(8)]
for rep in range(2):
    t = time.perf_counter(); crdtenc.content_name(big[0]); t1 = time.perf_counter() - t
    res = []
    for k in (1, 2, 4, 8):
        t = time.perf_counter(); crdtenc.content_names(big[:k]); res.append((k, time.perf_counter() - t))
    print("one via content_name %.1f ms | " % (t1 * 1e3) +
          " ".join("x%d %.1f ms (%.1f ms/file)" % (k, s * 1e3, s * 1e3 / k) for k, s in res))
