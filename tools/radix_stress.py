#!/usr/bin/env python3
"""Device-side radix sort self-test: python tools/radix_stress.py M BITS ITERS SEED"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd
f = salz_amd.lib.salz_debug_radix_selftest
f.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
f.restype = ctypes.c_long
m, bits, iters, seed = (int(x) for x in sys.argv[1:5])
print("radix selftest failures:", f(0, m, bits, iters, seed), flush=True)
