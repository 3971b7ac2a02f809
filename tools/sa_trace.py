"""Per-round suffix-sort log (SALZ_DEBUG=sa) of one encode per case: the round kind, depth, active
suffixes, large groups, survivors and the round's wall time, for reading where the rounds go.

    SALZ_DEBUG=sa python tools/sa_trace.py text:100000000 mixed:100000000
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import salz_amd  # noqa: E402
from tests.helpers import gen  # noqa: E402


def main():
    for case in sys.argv[1:] or ["text:16777216"]:
        kind, n = case.split(":")
        n = int(n)
        src = gen(kind, n, 1, 16 if kind == "smx" else 256)
        ctx = salz_amd.Context(0, max(n, 1 << 20))
        ctx.encode(src)  # warm
        print(f"== {kind} {n}", file=sys.stderr, flush=True)
        ctx.encode(src)


if __name__ == "__main__":
    main()
