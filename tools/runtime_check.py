#!/usr/bin/env python3
"""Which HIP runtime does libsalz run on when torch is in the same process, and does it work?

  python tools/runtime_check.py torch-first|salz-first|salz-only

torch ships its own libamdhip64.so (same SONAME as /opt/rocm's). Imported first, torch's copy
serves libsalz too (one runtime); imported after libsalz, torch loads its copy by RPATH next
to /opt/rocm's (two runtimes in one process). bench.py at N > 1 imports torch (gloo), so this
checks parity and speed of a 20 MB encode under each order, plus a torch device tensor used
as libsalz's output buffer.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
order = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
if order == "torch-first":
    import torch  # noqa: F401
    import salz_amd
elif order == "salz-first":
    import salz_amd
    import torch  # noqa: F401
else:
    import salz_amd
from tests.helpers import gen, oracle_encode  # noqa: E402

maps = open(f"/proc/{os.getpid()}/maps").read()
libs = sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip64" in l))
print(order, "runtimes:", libs, flush=True)
src = gen("text", 20_000_000, 2)
rc, ref = oracle_encode(src)
ctx = salz_amd.Context(0, len(src))
out = ctx.encode(src)
t = time.perf_counter()
for _ in range(3):
    out = ctx.encode(src)
dt = (time.perf_counter() - t) / 3
print(order, "parity:", out == ref, f"{len(src) / dt / 1e6:.1f} MB/s (host buffers)", flush=True)
if order != "salz-only":
    import torch
    if torch.cuda.is_available():
        d_src = torch.from_numpy(src.copy()).cuda()
        d_dst = torch.empty(salz_amd.encoded_len_max(len(src)), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        n = ctx.encode_device(d_src.data_ptr(), len(src), d_dst.data_ptr(), d_dst.numel())
        got = d_dst[:n].cpu().numpy().tobytes()
        print(order, "torch tensors as device buffers, parity:", got == ref, flush=True)
ctx.close()
