"""Host-buffer encode (salz_gpu_encode_host: H2D + encode + D2H) timed per call, for A/B of the
pinned staging (SALZ_PIN_STAGE). python tools/pin_bench.py [size]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import salz_amd  # noqa: E402
from tests.helpers import gen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
src = gen("text", n, 1)
ctx = salz_amd.Context(0, n)
ctx.encode(src)
ts = []
for _ in range(4):
    t0 = time.perf_counter()
    ctx.encode(src)
    ts.append(time.perf_counter() - t0)
print(os.environ.get("SALZ_PIN_STAGE", "1"), "ms", [round(t * 1e3, 2) for t in ts])
