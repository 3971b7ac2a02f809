#!/usr/bin/env python3
"""Diagnostics: encode consecutive blocks of one input with ONE context (workspace reuse, as
bench.py's sharded workloads do) and compare each block's suffix array / stream with the
oracle.   python tools/diag_blocks.py [--kind mixed] [--size N] [--block B] [--blocks K]"""
import argparse
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
ap.add_argument("--blocks", default="")
ap.add_argument("--device", action="store_true", help="encode through salz_gpu_encode_device")
a = ap.parse_args()
src = gen(a.kind, a.size, 1)
nb = (a.size + a.block - 1) // a.block
which = [int(x) for x in a.blocks.split(",")] if a.blocks else list(range(nb))
ctx = salz_amd.Context(0, a.block)
for b in which:
    blk = src[b * a.block:(b + 1) * a.block]
    try:
        if a.device:
            db = salz_amd.DeviceBuffer(len(blk)).upload(blk)
            cap = salz_amd.encoded_len_max(a.block) + 4096
            dd = salz_amd.DeviceBuffer(cap)
            nout = ctx.encode_device(db.ptr, len(blk), dd.ptr, cap)
            rc, ref = oracle_encode(blk)
            print(f"block {b}: device path stream_ok={dd.download(nout) == ref}", flush=True)
            continue
        out, d = ctx.encode_dump(blk)
    except salz_amd.SalzError as e:
        print(f"block {b}: FAILED {e}", flush=True)
        fresh = salz_amd.Context(0, len(blk))
        try:
            out2 = fresh.encode(blk)
            rc, ref = oracle_encode(blk)
            print(f"block {b}: fresh context ok={out2 == ref}", flush=True)
        except salz_amd.SalzError as e2:
            print(f"block {b}: fresh context FAILED too: {e2}", flush=True)
        fresh.close()
        continue
    o = oracle_stages(blk)
    bad = {k: int(np.nonzero(d[k] != o[k])[0][0]) for k in ("sa", "lp", "ln", "dlen") if (d[k] != o[k]).any()}
    rc, ref = oracle_encode(blk)
    print(f"block {b}: n={len(blk)} stream_ok={out == ref} first_diff={bad}", flush=True)
