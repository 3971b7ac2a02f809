#!/usr/bin/env python3
"""Diagnostics: repeat encodes of one input, print per-call stats and output hash.

  python tools/diag.py --kind text --size 20000000 --reps 3 [--oracle]
"""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="text")
ap.add_argument("--size", type=int, default=20_000_000)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--alpha", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--oracle", action="store_true")
ap.add_argument("--tag", default="")
a = ap.parse_args()

src = gen(a.kind, a.size, a.seed, a.alpha)
ctx = salz_amd.Context(0, a.size)
ctx.set_timing(True)
ref = None
if a.oracle:
    t = time.time()
    rc, ref = oracle_encode(src)
    print(f"{a.tag} oracle {time.time() - t:.2f}s len={len(ref)}", flush=True)
for r in range(a.reps):
    t = time.time()
    try:
        out = ctx.encode(src)
        ok = None if ref is None else (out == ref)
        st = ctx.stats()
        print(f"{a.tag} rep{r} {time.time() - t:.3f}s len={len(out)} sha={hashlib.sha256(out).hexdigest()[:16]} "
              f"match={ok} {json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()})}",
              flush=True)
    except salz_amd.SalzError as e:
        print(f"{a.tag} rep{r} FAILED {e}", flush=True)
