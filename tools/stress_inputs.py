#!/usr/bin/env python3
"""Pathological inputs at large sizes: time one GPU encode, round-trip it, and (with --parity)
compare with the CPU port.  python tools/stress_inputs.py [--size N] [--parity]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=64 << 20)
ap.add_argument("--parity", action="store_true")
ap.add_argument("--cases", default="", help="comma-separated subset of the cases (default: all)")
ap.add_argument("--stages", action="store_true", help="a second encode with stage timing: ms per stage")
a = ap.parse_args()
n = a.size
cases = {
    "zeros": lambda: np.zeros(n, np.uint8),
    "period3": lambda: np.resize(np.frombuffer(b"abc", np.uint8), n),
    "period1000": lambda: np.resize(gen("smx", 1000, 7, 256), n),
    "random": lambda: gen("smx", n, 3, 256),
    "binary2": lambda: gen("smx", n, 5, 2),
    "fib": lambda: gen("fib", n),
    "sawtooth": lambda: np.resize(np.arange(256, dtype=np.uint8), n),
    "halves": lambda: np.resize(gen("text", n // 2 + 1, 11), n),  # one repeat at distance n/2
    "runs": lambda: np.repeat(gen("smx", n // 64 + 1, 13, 256), 64)[:n],
    "mixed": lambda: gen("mixed", n, 17),
}
ctx = salz_amd.Context(0, n)
# one output buffer, touched once: the timed encode is H2D, encode and D2H, not the host's page
# faults on a fresh 300 MB array or a copy into Python bytes (as bench.py's e2e step)
obuf = np.zeros(salz_amd.encoded_len_max(n), np.uint8)
want = [c for c in a.cases.split(",") if c]
for name, make in cases.items():
    if want and name not in want:
        continue
    src = make()
    ctx.encode(src[: 1 << 20])  # warm
    t0 = time.perf_counter()
    olen = ctx.encode_into(src, obuf)
    t1 = time.perf_counter()
    out = obuf[:olen].tobytes()
    ok = salz_amd.decode_safe(out, n, frame=True) == src.tobytes()
    st = ctx.stats()
    algo = f"dc3 {st['sa_dc3_levels']} levels" if st["sa_dc3_levels"] else f"doubling {st['sa_rounds']} rounds"
    line = (f"{name:11s} {n} B -> {len(out)} B  {(t1 - t0) * 1e3:8.1f} ms  {n / (t1 - t0) / 1e6:8.1f} MB/s  "
            f"roundtrip {ok}  sa: {algo}")
    if a.parity:
        rc, ref = oracle_encode(src)
        line += f"  parity {rc == 0 and ref == out}"
    if a.stages:  # (timed stages synchronise between stages: a separate encode)
        ctx.set_timing(True)
        ctx.encode_into(src, obuf)
        ctx.set_timing(False)
        st = ctx.stats()
        line += "  |" + " ".join(f"{k[3:]} {st[k]:.1f}" for k in ("ms_upload", "ms_sa", "ms_lcp", "ms_ansv",
                                                                    "ms_parse", "ms_emit", "ms_total"))
        line += f" parse_iters {st['parse_iters']}"
    print(line, flush=True)
