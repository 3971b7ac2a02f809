#!/usr/bin/env python3
"""Device-resident radix sort self-test in T concurrent host threads (own workspace/stream each)."""
import ctypes
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
m = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
bits = int(sys.argv[3]) if len(sys.argv) > 3 else 40
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 50
f = salz_amd.lib.salz_debug_radix_selftest
f.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
f.restype = ctypes.c_long
res = {}


def work(t):
    res[t] = f(0, m, bits, iters, 1000 * t + 1)


ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
for th in ths:
    th.start()
for th in ths:
    th.join()
print(f"radix selftest T={T} m={m} bits={bits} iters={iters}: failures per thread {res}", flush=True)
