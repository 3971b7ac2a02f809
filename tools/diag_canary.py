#!/usr/bin/env python3
"""Out-of-bounds write detector: canary device buffers filled with a pattern are allocated
around a context; after repeated encodes, any changed canary byte means some kernel wrote
outside its own buffers.   python tools/diag_canary.py [--mb 512] [--iters 10]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mb", type=int, default=256)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--size", type=int, default=1048575)
a = ap.parse_args()
pat = np.full(a.mb << 20, 0xA5, np.uint8)
canaries = [salz_amd.DeviceBuffer(len(pat)).upload(pat)]
ctx = salz_amd.Context(0, a.size)
canaries.append(salz_amd.DeviceBuffer(len(pat)).upload(pat))
src = gen("text", a.size, 3)
rc, ref = oracle_encode(src)
d_src = salz_amd.DeviceBuffer(len(src)).upload(src)
canaries.append(salz_amd.DeviceBuffer(len(pat)).upload(pat))
cap = salz_amd.encoded_len_max(len(src)) + 4096
d_dst = salz_amd.DeviceBuffer(cap)
canaries.append(salz_amd.DeviceBuffer(len(pat)).upload(pat))
bad = 0
for _ in range(a.iters):
    n = ctx.encode_device(d_src.ptr, len(src), d_dst.ptr, cap)
    bad += d_dst.download(n) != ref
for k, c in enumerate(canaries):
    got = np.frombuffer(c.download(len(pat)), np.uint8)
    diff = np.nonzero(got != 0xA5)[0]
    print(f"canary {k} at {c.ptr:#x}: {len(diff)} bytes changed" + (f", first at +{diff[0]}" if len(diff) else ""), flush=True)
print("stream mismatches:", bad, "ctx", hex(ctx.handle), flush=True)
