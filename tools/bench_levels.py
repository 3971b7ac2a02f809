#!/usr/bin/env python3
"""Level sweep with round-trip check: the scripts/bench.sh harness of the reference
(/root/reference/scripts/bench.sh:42-61: for each level 0..9, compress, decompress, diff),
on the MI355X build and without sudo / git checkouts.

Each level L encodes the input as the CLI container with blocks of 1 << (15 + L) bytes
(programs/salzcli.c:109) through salz_encode_blocks (all visible GPUs), decodes it with the
threaded host decoder, compares, and prints one JSON line per level.

  python tools/bench_levels.py [--file PATH | --kind text --size N] [--levels 0-9] [--gpus N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--file")
    ap.add_argument("--kind", default="text")
    ap.add_argument("--size", type=int, default=50_000_003)
    ap.add_argument("--levels", default="0-9")
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    if a.file:
        src = np.fromfile(a.file, dtype=np.uint8)
        name = os.path.basename(a.file)
    else:
        from tests.helpers import gen

        src = gen(a.kind, a.size, 1)
        name = f"{a.kind}-{a.size}"
    lo, hi = (int(x) for x in a.levels.split("-"))
    for level in range(lo, hi + 1):
        block = 1 << (15 + level)
        line = {"input": name, "bytes": len(src), "level": level, "block": block}
        if len(src) % block <= 8:
            # the reference CLI fails when the trailing fread() chunk has 0..8 bytes
            line["skipped"] = "trailing block of 0..8 bytes (reference CLI fails too)"
            print(json.dumps(line), flush=True)
            continue
        packed = salz_amd.encode_blocks(src, block, a.gpus)  # warm (contexts, code objects)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            packed = salz_amd.encode_blocks(src, block, a.gpus)
        t1 = time.perf_counter()
        back = salz_amd.decode_blocks(packed, len(src))
        t2 = time.perf_counter()
        line.update({
            "compressed": len(packed),
            "ratio": round(len(src) / len(packed), 4),
            "compress_MBps": round(len(src) * a.reps / (t1 - t0) / 1e6, 1),
            "decompress_MBps": round(len(src) / (t2 - t1) / 1e6, 1),
            "roundtrip_ok": back == src.tobytes(),
            "note": "host buffers: includes H2D/D2H and per-call context setup",
        })
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
