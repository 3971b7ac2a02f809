#!/usr/bin/env python3
"""Concurrency check: T host threads, each with its own context (own HIP stream and
workspace) on device 0, encode the same blocks repeatedly; every stream is compared with the
oracle. Control: the same with T = 1.
  python tools/diag_concurrency.py --threads 2 --iters 20 [--kind text --size 1048575]"""
import argparse
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=2)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--kind", default="text")
ap.add_argument("--size", type=int, default=1048575)
ap.add_argument("--device", action="store_true", help="device-resident input (salz_gpu_encode_device)")
ap.add_argument("--procs", action="store_true", help="one process per worker instead of threads")
a = ap.parse_args()
src = gen(a.kind, a.size, 3)
rc, ref = oracle_encode(src)
assert rc == 0
stats = {}


def work(t):
    ctx = salz_amd.Context(0, a.size)
    bad = fail = 0
    if a.device:
        d_src = salz_amd.DeviceBuffer(len(src)).upload(src)
        cap = salz_amd.encoded_len_max(len(src)) + 4096
        d_dst = salz_amd.DeviceBuffer(cap)
    for _ in range(a.iters):
        try:
            if a.device:
                nout = ctx.encode_device(d_src.ptr, len(src), d_dst.ptr, cap)
                if d_dst.download(nout) != ref:
                    bad += 1
            elif ctx.encode(src) != ref:
                bad += 1
        except salz_amd.SalzError as e:
            fail += 1
            if fail <= 3:
                print(f"thread {t}: {e}", flush=True)
    stats[t] = (bad, fail)
    ctx.close()


def proc_main(t, q):
    work(t)
    q.put((t, stats[t]))


if __name__ == "__main__":
    if a.procs:
        import multiprocessing as mp

        mpc = mp.get_context("spawn")
        q = mpc.Queue()
        ps = [mpc.Process(target=proc_main, args=(t, q)) for t in range(a.threads)]
        for p in ps:
            p.start()
        for _ in ps:
            t, v = q.get(timeout=300)
            stats[t] = v
        for p in ps:
            p.join()
    else:
        ths = [threading.Thread(target=work, args=(t,)) for t in range(a.threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    print(f"threads={a.threads} iters={a.iters} {a.kind} {a.size}: (mismatch, failed) per thread {stats}", flush=True)
