#!/usr/bin/env python3
"""Determinism check: encode every block of a workload P times with one context, device-resident
buffers (as bench.py), and report any block whose stream differs between passes or whose encode
fails; with --stages, recheck a bad block's stage arrays against the oracle.
  python tools/diag_repeat.py [--kind mixed] [--size N] [--block B] [--passes P]"""
import argparse
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode, oracle_stages  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mixed")
ap.add_argument("--size", type=int, default=211_957_760)
ap.add_argument("--block", type=int, default=16 << 20)
ap.add_argument("--passes", type=int, default=6)
ap.add_argument("--timing-pass", type=int, default=-1, help="turn per-stage timing on for this pass")
a = ap.parse_args()
src = gen(a.kind, a.size, 1)
nb = (a.size + a.block - 1) // a.block
spans = [(b * a.block, min(a.size, (b + 1) * a.block)) for b in range(nb)]
ctx = salz_amd.Context(0, a.block)
cap = salz_amd.encoded_len_max(a.block) + 4096
d_src = [salz_amd.DeviceBuffer(e - s).upload(src[s:e]) for s, e in spans]
d_dst = [salz_amd.DeviceBuffer(cap) for _ in spans]
ref = {}
bad = set()
for p in range(a.passes):
    ctx.set_timing(p == a.timing_pass)
    for b, ((s, e), di, do) in enumerate(zip(spans, d_src, d_dst)):
        try:
            n = ctx.encode_device(di.ptr, e - s, do.ptr, cap)
        except salz_amd.SalzError as ex:
            print(f"pass {p} block {b}: FAILED {ex}", flush=True)
            bad.add(b)
            continue
        h = hashlib.sha256(do.download(n)).hexdigest()[:16]
        if b not in ref:
            ref[b] = h
        elif ref[b] != h:
            print(f"pass {p} block {b}: stream differs from pass 0 ({h} vs {ref[b]})", flush=True)
            bad.add(b)
print("passes done; bad blocks:", sorted(bad), flush=True)
for b in sorted(bad)[:2]:
    s, e = spans[b]
    blk = src[s:e]
    o = oracle_stages(blk)
    for t in range(3):
        try:
            out, d = ctx.encode_dump(blk)
        except salz_amd.SalzError as ex:
            print(f"block {b} dump try {t}: FAILED {ex}", flush=True)
            continue
        diff = {k: int(np.nonzero(d[k] != o[k])[0][0]) for k in ("sa", "lp", "ln", "dlen") if (d[k] != o[k]).any()}
        print(f"block {b} dump try {t}: first diffs {diff}", flush=True)
