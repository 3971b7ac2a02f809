#!/usr/bin/env python3
"""Encode repeatedly; after each encode compare the GPU SA snapshot with the oracle SA and
write a compact report of the differences (needs SALZ_DEBUG_SAROUND=1)."""
import ctypes, os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd
from tests.helpers import gen, oracle, oracle_encode
size, reps, tag = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
src = gen("text", size, 1)
n = size - 8
ref = np.zeros(n, np.int32)
oracle().oracle_suffix_array(src.ctypes.data, ref.ctypes.data, n)
ctx = salz_amd.Context(0, size)
f = salz_amd.lib.salz_debug_fetch
f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
sa = np.zeros(n, np.uint32); rnd = np.zeros(n, np.uint32)
for r in range(reps):
    try:
        ctx.encode(src)
        st = "ok"
    except salz_amd.SalzError as e:
        st = "fail"
    f(ctx.handle, 0, sa.ctypes.data, n); f(ctx.handle, 1, rnd.ctypes.data, n)
    bad = np.nonzero(sa != ref.astype(np.uint32))[0]
    rep = {"tag": tag, "rep": r, "status": st, "nbad": int(len(bad))}
    if len(bad):
        rep["first"] = int(bad[0]); rep["last"] = int(bad[-1])
        rep["rounds_of_bad"] = {int(k): int(v) for k, v in zip(*np.unique(rnd[bad], return_counts=True))}
        rep["rounds_all"] = {int(k): int(v) for k, v in zip(*np.unique(rnd, return_counts=True))}
        # contiguous runs of bad ranks
        runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
        rep["nruns"] = len(runs)
        rep["runs"] = [[int(x[0]), int(len(x))] for x in runs[:20]]
        rep["sample"] = [[int(b), int(sa[b]), int(ref[b]), int(rnd[b])] for b in bad[:10]]
        np.save(f"gpurun_out/sa_bad_{tag}_{r}.npy", np.stack([bad.astype(np.uint32), sa[bad], ref[bad].astype(np.uint32), rnd[bad]]))
    print(json.dumps(rep), flush=True)
