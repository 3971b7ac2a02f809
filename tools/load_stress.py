#!/usr/bin/env python3
"""python tools/load_stress.py N ITERS EXTRA_BYTES -> mismatches of k_sa_init's loads"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd
f = salz_amd.lib.salz_debug_load_selftest
f.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32]
f.restype = ctypes.c_long
n, iters, extra, pre, seed = (int(x) for x in sys.argv[1:6])
print("load selftest mismatches:", f(0, n, iters, extra, pre, seed), flush=True)
