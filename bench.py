#!/usr/bin/env python3
"""bench.py - compress MB/s of the MI355X SA-LZ encoder on an enwik8-sized block.

Workload (BASELINE.json configs[1], "enwik8 (100 MB) single block, SA+PLCP+LZ on one MI355X"):
one 100,000,000-byte block of the deterministic wiki-text surrogate (tools/datagen.c; the real
enwik8 is not available offline) per GPU, resident in HBM before timing. A step is one full
salz_gpu_encode_device call: suffix array, LCP, PSV/NSV candidates, optimal parse and emission of
the bit-exact reference stream into HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: launched by torch.distributed.run, one rank per GPU; each rank encodes its own block:
   weak scaling over independent blocks, no data-path collective.)

Prints ONE JSON line (rank 0). `roofline` prices the dominant kernel (the radix-sort scatter of
the suffix sorter) by algorithmic bytes / HIP-event-measured launch time; `cpu_baseline` times the
CPU port of the reference (oracle/liboracle.so, 1 thread) on the same block, which also serves as a
bit-exact parity check of the GPU stream at full size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
RADIX_BYTES_PER_ELEM = 24  # scatter: read 8 B key + 4 B value, write 8 B key + 4 B value


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kind", default="text", help="text | fib | smx | mixed")
    ap.add_argument("--size", type=int, default=100_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="bytes of the block timed on the CPU port (0 = whole block)")
    ap.add_argument("--profile-steps", action="store_true",
                    help="per-stage HIP-event timing on every timed step (adds small overhead)")
    return ap.parse_args()


def main():
    args = parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo on CPU tensors: no GPU runtime of torch's own

        dist.init_process_group("gloo")

    import numpy as np

    import salz_amd
    from tests.helpers import gen  # workload generator (tools/libdatagen.so)

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allsum(x: float) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    ndev = salz_amd.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    device = local % ndev
    N = args.size
    src = gen(args.kind, N, 1, 16 if args.kind == "smx" else 256)
    ctx = salz_amd.Context(device, N)
    d_src = salz_amd.DeviceBuffer(N, device).upload(src)
    cap = salz_amd.encoded_len_max(N) + 4096
    d_dst = salz_amd.DeviceBuffer(cap, device)

    # Warmup (untimed), then one instrumented pass for the kernel-level numbers.
    out_len = 0
    for _ in range(args.warmup):
        out_len = ctx.encode_device(d_src.ptr, N, d_dst.ptr, cap)
    ctx.set_timing(True)
    out_len = ctx.encode_device(d_src.ptr, N, d_dst.ptr, cap)
    st = ctx.stats()
    ctx.set_timing(bool(args.profile_steps))

    # Timed region: exactly K steps bracketed by barrier + device sync on both sides.
    barrier()
    salz_amd.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_len = ctx.encode_device(d_src.ptr, N, d_dst.ptr, cap)
    salz_amd.synchronize(device)
    t1 = time.perf_counter()
    barrier()
    dt = allmax(t1 - t0)
    if args.profile_steps:
        st = ctx.stats()

    stream = d_dst.download(out_len)
    # Exchange step of the block queue: every rank's encoded length -> container offsets.
    total_out = allsum(float(out_len + 4))

    # Round trip through the product decoder (frame rule for > 16 MiB streams).
    back = salz_amd.decode_safe(stream, N, frame=True)
    roundtrip_ok = back == src.tobytes()

    value = world * N * args.steps / dt / 1e6
    ms_step = dt / args.steps * 1e3

    # Roofline of the dominant kernel (radix scatter): algorithmic bytes / event-timed duration.
    launches = max(int(st["radix_scatter_launches"]), 1)
    ms_rx = float(st["ms_radix_scatter"])
    bytes_rx = RADIX_BYTES_PER_ELEM * float(st["radix_scatter_elems"])
    achieved = bytes_rx / (ms_rx * 1e-3) / 1e9 if ms_rx > 0 else 0.0
    roofline = {
        "kernel": "k_radix_scatter",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "launches": launches,
        "avg_launch_us": round(ms_rx * 1e3 / launches, 2),
        "alg_bytes_per_launch": int(bytes_rx / launches),
    }

    cpu = None
    parity_full = None
    if rank == 0 and not args.no_cpu_baseline:
        from tests.helpers import oracle_encode  # CPU port of the reference (baseline + checker)

        sample = N if args.cpu_sample <= 0 else min(args.cpu_sample, N)
        c0 = time.perf_counter()
        rc, ref = oracle_encode(src[:sample])
        c1 = time.perf_counter()
        cpu = {
            "value": round(sample / (c1 - c0) / 1e6, 3),
            "unit": "MB/s",
            "cores": 1,
            "kind": "port",
            "sample": f"one {sample:,}-byte block of the same {args.kind} input, oracle/liboracle.so "
                      f"(clean-room C restatement of lib/salz.c + own SA-IS), 1 thread, "
                      f"{c1 - c0:.2f} s",
        }
        if sample == N:
            parity_full = bool(rc == 0 and ref == stream)

    if rank == 0:
        line = {
            "metric": "compress MB/s + achieved HBM GB/s, enwik8 block, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic ({args.kind} surrogate, tools/datagen.c; enwik8 not available offline)",
            "config": {
                "workload": "enwik8-sized single block per GPU (BASELINE configs[1])",
                "block_bytes": N,
                "blocks_per_gpu": 1,
                "input": args.kind,
                "parallelism": f"independent blocks x{world}",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "encoded_bytes": out_len,
            "ratio": round(N / out_len, 4),
            "container_bytes_all_ranks": int(total_out),
            "roundtrip_ok": roundtrip_ok,
            "parity_vs_cpu_port": parity_full,
            "stages_ms": {k: round(st[k], 3) for k in
                          ("ms_sa", "ms_lcp", "ms_ansv", "ms_parse", "ms_emit", "ms_total")},
            "sa_rounds": st["sa_rounds"],
            "parse_iters": st["parse_iters"],
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
