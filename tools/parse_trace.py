"""Per-pass parse log (SALZ_DEBUG=parse) of one encode per case: changed decisions, dirty waves and
lazy-cost counters of every fixed-point pass, for reading where a block's parse passes go.

    SALZ_DEBUG=parse python tools/parse_trace.py mixed:100000000 mixed:16777216 text:100000000
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import salz_amd  # noqa: E402
from tests.helpers import gen  # noqa: E402


def main():
    cases = sys.argv[1:] or ["mixed:16777216"]
    for case in cases:
        kind, n = case.split(":")
        n = int(n)
        src = gen(kind, n, 1, 16 if kind == "smx" else 256)
        ctx = salz_amd.Context(0, max(n, 1 << 20))
        ctx.encode(src)  # warm
        print(f"== {kind} {n}", file=sys.stderr, flush=True)
        t = time.perf_counter()
        out = ctx.encode(src)
        print(f"== {kind} {n}: {len(out)} B, {(time.perf_counter() - t) * 1e3:.2f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
