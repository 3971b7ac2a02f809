"""Parse time by chunk length on large single blocks of small alphabets (diagnostic):
    SALZ_PARSE=klog=7 python tools/klog_probe.py
prints, per input, the stage times of one encode (after a warm-up) and the round trip."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen  # noqa: E402

n = 256 << 20
cases = {
    "fib": lambda: gen("fib", n),
    "binary2": lambda: gen("smx", n, 5, 2),
    "dna4": lambda: gen("smx", n, 6, 4),
    "smx16": lambda: gen("smx", n, 7, 16),
    "period1000": lambda: np.resize(gen("smx", 1000, 7, 256), n),
}
ctx = salz_amd.Context(0, n)
for name, make in cases.items():
    src = make()
    ctx.encode(src)
    out = ctx.encode(src)
    st = ctx.stats()
    ok = salz_amd.decode_safe(out, n, frame=True) == src.tobytes()
    print(f"{os.environ.get('SALZ_PARSE', 'default'):8s} {name:10s} {len(out):10d} B parse {st['ms_parse']:.3f} ms "
          f"total {st['ms_total']:.3f} ms iters {st.get('parse_iters')} roundtrip {ok}", flush=True)
