#!/usr/bin/env python3
"""Golden vectors for the int32 cost-wrap regime of the reference parse (lib/salz.c:621-661).

The reference DP keeps bit costs in int32: `9 + aux[...]` and the factor sum (size_t arithmetic
truncated to int32) wrap once the cost of the rest of the block passes 2^31 - 1, i.e. once the
encoded suffix exceeds 256 MiB of output (9 n > 2^31 - 1 for incompressible data). Two inputs
(tests/helpers.py wrap_input):
  smx256   268,435,456 splitmix64 bytes: costs wrap, every decision is still a literal or a
           short factor, and the block falls back to PLAIN;
  wrap400  400,000,000 bytes of splitmix64 data where the last 4 MiB of every 16 MiB repeat an
           earlier 4 MiB run (seeded offsets): ~0.84 of the input's size comes out, so the cost
           from position 0 is ~2.7e9 bits and about the first fifth of the parse runs on wrapped
           costs, yet the stream is SALZ (not PLAIN) and its header length field is truncated.
The expected bytes come from the CPU oracle (oracle/liboracle.so, the clean-room restatement of
lib/salz.c whose DP uses the same two's-complement int32 arithmetic, salz_oracle.c:359-382),
so the GPU test on the box compares hashes instead of re-running the 4-minute oracle.

  python tools/make_wrap_golden.py > tests/golden/cost_wrap.json
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.helpers import oracle_encode, wrap_input  # noqa: E402


def main():
    vecs = []
    for name, n in (("smx256", 1 << 28), ("wrap400", 400_000_000)):
        src = wrap_input(name, n)
        t = time.time()
        rc, out = oracle_encode(src)
        assert rc == 0
        hdr = int.from_bytes(out[:4], "little")
        vecs.append({"name": name, "n": n, "in_sha256": hashlib.sha256(src.tobytes()).hexdigest(),
                     "out_len": len(out), "out_type": hdr >> 24, "out_hdr_len": hdr & 0xFFFFFF,
                     "out_sha256": hashlib.sha256(out).hexdigest(), "oracle_s": round(time.time() - t, 1)})
        print(name, vecs[-1], file=sys.stderr, flush=True)
    json.dump({"source": "tools/make_wrap_golden.py: oracle/liboracle.so (CPU restatement of lib/salz.c, "
                         "int32 wrapping DP) on tests/helpers.py wrap_input(name, n) as ONE block",
               "vectors": vecs}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
