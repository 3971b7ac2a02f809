#!/usr/bin/env python3
"""bench.py - compress MB/s of the MI355X SA-LZ encoder (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "enwik8 (100 MB) single block, SA+PLCP+LZ on one
MI355X"): one 100,000,000-byte block of the deterministic wiki-text surrogate per GPU
(tools/datagen.c; the real enwik8 is not available offline), resident in HBM before timing.
A step is one full salz_gpu_encode_device call per block: suffix array, LCP, PSV/NSV
candidates, optimal parse and emission of the bit-exact reference stream into HBM.

Other BASELINE configs (--workload):
  enwik9   configs[3]: 10^9 bytes of the text surrogate in 64 MiB blocks, contiguous block
           ranges sharded over the ranks (salz_amd/dist.py); a step encodes every block once
  silesia  configs[2]: 211,957,760 bytes of the mixed surrogate in 16 MiB blocks, sharded
  fib256   configs[4]: the 268,435,456-byte Fibonacci word as one block per GPU

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload enwik8|enwik9|silesia|fib256]
                  [--dist-backend nccl|gloo] [--launch] [--no-pmc]
  N > 1: one rank per GPU. Under an outside launcher (torch.distributed.run sets WORLD_SIZE)
  this process is one rank; otherwise it starts `python -m torch.distributed.run
  --nproc-per-node N bench.py ...` as a child process (before it touches any GPU), relays rank
  0's JSON line and exits non-zero when the line's n_gpus differs from N. Weak scaling for the
  one-block workloads, strong for the sharded ones. A step is encode + the exchange step of
  salz_amd/dist.py: RCCL all-gather of each rank's packed frame bytes, then every rank's run of
  frames straight into rank 0's container in HBM over xGMI (point-to-point). No collective
  touches the encode itself. --dist-backend gloo runs the same launch, shard and exchange code
  with the payload staged through host memory, so several ranks can share one GPU (rehearsal on
  a one-GPU box); --launch goes through the launcher at N = 1 too (the RCCL path at world 1).

Prints ONE JSON line (rank 0). `roofline` prices the dominant kernel (the suffix sorter's
radix scatter) by algorithmic bytes / HIP-event-measured launch time on the library's own
stream; its `traffic` (HBM bytes per launch) comes from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) of one encode of the same input, run as child processes of this run before it
touches the GPU (`traffic_source` says so, or names the file it fell back to).
`cpu_baseline` times the CPU port of the reference (oracle/liboracle.so, 1 thread) on one block
of the same input after the timed region, which also checks full-block parity of the GPU stream.
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

WORKLOADS = {
    # name: (config, kind, total bytes, block bytes or None = one block per rank)
    "enwik8": ("enwik8-sized single block per GPU (BASELINE configs[1])", "text", 100_000_000, None),
    "enwik9": ("enwik9-sized input, 64 MiB blocks sharded over GPUs (BASELINE configs[3])", "text",
               1_000_000_000, 64 << 20),
    "silesia": ("Silesia-sized mixed input, 16 MiB blocks sharded over GPUs (BASELINE configs[2])",
                "mixed", 211_957_760, 16 << 20),
    "fib256": ("256 MiB Fibonacci word, single block per GPU (BASELINE configs[4])", "fib", 1 << 28, None),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="enwik8", choices=sorted(WORKLOADS))
    ap.add_argument("--kind", default=None, help="override the input generator (text|fib|smx|mixed)")
    ap.add_argument("--size", type=int, default=0, help="override the total input bytes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="bytes of one block timed on the CPU port (0 = the whole first block)")
    ap.add_argument("--profile-steps", action="store_true",
                    help="per-stage HIP-event timing on every timed step (adds small overhead)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-buffer (salz_encode_safe-style) end-to-end timing")
    ap.add_argument("--cpu-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 PMC passes that measure roofline.traffic in this run")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="N > 1 exchange backend: nccl (RCCL over xGMI, one GPU per rank) or gloo "
                         "(payload staged through host memory; ranks may share a GPU)")
    ap.add_argument("--launch", action="store_true",
                    help="go through torch.distributed.run even at --gpus 1 (world-1 RCCL path)")
    ap.add_argument("--ctx-streams", action="store_true",
                    help="tuning: each slot encodes on its context's own HIP stream instead of a torch stream")
    ap.add_argument("--slots", type=int, default=0,
                    help="concurrent encoder contexts per GPU for the sharded workloads "
                         "(0 = auto: 4; one block per GPU: 1)")
    ap.add_argument("--batch-bytes", type=int, default=8 << 20,
                    help="sharded workloads with blocks of at most 4 MiB: consecutive blocks "
                         "encoded per pipeline pass (salz_gpu_encode_batch_device; 0 = one block "
                         "per pass; larger blocks always go one per pass)")
    return ap.parse_args()


def cpu_child(spec: str) -> None:
    """CPU baseline in a process of its own, pinned to one core before it touches anything:
    the CPU port of the reference (oracle/liboracle.so) on `sample` bytes of the workload's
    first block. Prints one JSON line; the parent compares the stream hash with the GPU's."""
    import ctypes
    import hashlib

    import numpy as np

    kind, total, start, sample, core = spec.split(",")
    total, start, sample, core = int(total), int(start), int(sample), int(core)
    os.sched_setaffinity(0, {core})
    from tests.helpers import gen, oracle, oracle_encode  # CPU port of the reference (baseline + checker)

    src = gen(kind, total, 1, 16 if kind == "smx" else 256)
    blk = np.ascontiguousarray(src[start:start + sample])
    del src
    # Wait for the parent's go (sent after its timed region), so the CPU work never overlaps
    # the GPU measurement; an empty read means the parent is gone.
    if sys.stdin.readline().strip() != "go":
        return
    c0 = time.perf_counter()
    rc, ref = oracle_encode(blk)
    c1 = time.perf_counter()
    sa_buf = np.empty(max(sample - 8, 1), np.int32)
    c2 = time.perf_counter()
    oracle().oracle_suffix_array(blk.ctypes.data, sa_buf.ctypes.data, ctypes.c_int32(max(sample - 8, 0)))
    c3 = time.perf_counter()
    print(json.dumps({"rc": rc, "enc_s": c1 - c0, "sa_s": c3 - c2, "core": core,
                      "affinity": sorted(os.sched_getaffinity(0)),
                      "sha256": hashlib.sha256(ref).hexdigest() if rc == 0 else None}), flush=True)


def start_cpu_child(kind, total, start, sample):
    """Start the pinned CPU-baseline child before this process makes any GPU call. It prepares
    its input, then blocks until the parent writes "go" (after the timed region and the e2e
    timing), so the baseline's CPU work never overlaps a GPU measurement."""
    import subprocess

    cores = sorted(os.sched_getaffinity(0))
    core = cores[-1]
    spec = f"{kind},{total},{start},{sample},{core}"
    return subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-child", spec],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True), core


def launch_ranks(args) -> int:
    """--gpus N without an outside launcher: one rank per GPU through torch.distributed.run,
    started as a CHILD process before this process touches any GPU (never an exec). Relays rank
    0's JSON line; fails when the ranks' world differs from N."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    env.setdefault("OMP_NUM_THREADS", "4")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        sys.stdout.write(p.stdout)
        print(f"bench.py: torch.distributed.run exited with {p.returncode}", file=sys.stderr)
        return p.returncode or 1
    line = json.loads(lines[-1])
    if line.get("n_gpus") != args.gpus:
        print(f"bench.py: the ranks reported n_gpus={line.get('n_gpus')}, expected {args.gpus}",
              file=sys.stderr)
        return 3
    print(lines[-1], flush=True)
    return 0


def pmc_child(args) -> None:
    """One encode of the workload's first block with the library's launch timing on, for the
    rocprofv3 --pmc passes (no torch, no extra encodes: the counters cover exactly one encode).
    Prints the kernel-level statistics as one JSON line."""
    import salz_amd
    from tests.helpers import gen

    config, kind, total, block = WORKLOADS[args.workload]
    kind = args.kind or kind
    total = args.size or total
    n = min(block, total) if block else total
    src = gen(kind, total, 1, 16 if kind == "smx" else 256)[:n]
    ctx = salz_amd.Context(0, n)
    ctx.set_timing(True)
    ctx.encode(src)
    st = ctx.stats()
    print(json.dumps({"radix_scatter_launches": st["radix_scatter_launches"],
                      "radix_scatter_bytes": st["radix_scatter_bytes"]}), flush=True)


def measure_traffic(args):
    """roofline.traffic measured in this run: two rocprofv3 --pmc passes (FETCH_SIZE, then
    WRITE_SIZE; one pass cannot hold both on gfx950) over `bench.py --pmc-child`, corrected as
    /opt/skills/guides/MI355X_MICROARCH.md prescribes (tools/pmc_traffic.py). Runs BEFORE this
    process makes any GPU call (the profiler children start from a process without GPU state).
    Returns (per-launch traffic dict, error string)."""
    import shutil
    import subprocess
    import tempfile

    # Under a profiler already (this bench is the program of an outer rocprofv3 run), its library
    # is preloaded into every child: a nested rocprofv3 would start with the GPU initialised and
    # then exec the program, which is never done. Those runs measure the counters themselves.
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None, "not measured: this run is itself under rocprofv3"
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import load  # noqa: E402

    tmp = tempfile.mkdtemp(prefix="salz_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    child_args = ["--pmc-child", "--workload", args.workload]
    if args.kind:
        child_args += ["--kind", args.kind]
    if args.size:
        child_args += ["--size", str(args.size)]
    res, stats = {}, None
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(tmp, counter)
        cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), *child_args]
        try:
            p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                               env=env, cwd="/tmp", timeout=150)
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 --pmc {counter} timed out"
        if p.returncode != 0:
            return None, f"rocprofv3 --pmc {counter} exited with {p.returncode}"
        js = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        stats = json.loads(js[-1]) if js else stats
        csvp = os.path.join(d, "pmc_counter_collection.csv")
        if not os.path.exists(csvp):
            return None, f"no counter file from the {counter} pass"
        rows = load(csvp).get("k_radix_scatter", [])
        if not rows:
            return None, f"no k_radix_scatter dispatches in the {counter} pass"
        res[counter] = (sum(v for _, v, _ in rows), len(rows))
    shutil.rmtree(tmp, ignore_errors=True)
    fetch = 2 * res["FETCH_SIZE"][0] * 1024 / res["FETCH_SIZE"][1]
    write = res["WRITE_SIZE"][0] * 1024 / res["WRITE_SIZE"][1]
    out = {"traffic_per_launch": round(fetch + write), "fetch_bytes_per_launch": round(fetch),
           "write_bytes_per_launch": round(write), "pmc_launches": res["FETCH_SIZE"][1]}
    if stats and stats.get("radix_scatter_launches"):
        out["pmc_alg_bytes_per_launch"] = round(stats["radix_scatter_bytes"] / stats["radix_scatter_launches"])
        out["pmc_timed_launches"] = stats["radix_scatter_launches"]
    return out, None


def link_rates(torch, dev, host_block, d_stream, stream_len) -> dict:
    """Host link rates of one block and one stream, so the e2e figure can be read against them:
    H2D of the block and D2H of its stream from pinned host memory (the DMA engines alone) and
    from pageable memory (what a salz_encode_safe caller hands over), best of 3, CUDA events."""
    n = len(host_block)
    pin_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pin_in.numpy()[:] = host_block
    pin_out = torch.empty(stream_len, dtype=torch.uint8, pin_memory=True)
    page_in = torch.from_numpy(host_block.copy())
    page_out = torch.empty(stream_len, dtype=torch.uint8)
    d_in = torch.empty(n, dtype=torch.uint8, device=dev)

    def best(fn, nbytes):
        ms = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            fn()
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return round(nbytes / (min(ms) * 1e-3) / 1e9, 2)

    src_stream = d_stream[:stream_len]
    return {
        "h2d_gbs": best(lambda: d_in.copy_(pin_in, non_blocking=True), n),
        "d2h_gbs": best(lambda: pin_out.copy_(src_stream, non_blocking=True), stream_len),
        "h2d_pageable_gbs": best(lambda: d_in.copy_(page_in), n),
        "d2h_pageable_gbs": best(lambda: page_out.copy_(src_stream), stream_len),
        "link_what": f"one {n:,}-byte block H2D and its {stream_len:,}-byte stream D2H, pinned "
                     "(h2d_gbs, d2h_gbs) and pageable host memory, best of 3",
    }


def git_head() -> str:
    try:
        import subprocess

        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or "unknown"
    except Exception:
        return "unknown"


def main():
    args = parse_args()
    if args.cpu_child:
        cpu_child(args.cpu_child)
        return
    if args.pmc_child:
        pmc_child(args)
        return
    launched = "WORLD_SIZE" in os.environ  # a rank of torch.distributed.run (ours or the driver's)
    if not launched and (args.gpus > 1 or args.launch):
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if launched and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")

    config, kind, total, block = WORKLOADS[args.workload]
    kind = args.kind or kind
    total = args.size or total
    sharded = block is not None
    child = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU baseline is an N=1 figure
        first = min(block, total) if sharded else total
        sample = first if args.cpu_sample <= 0 else min(args.cpu_sample, first)
        child, _ = start_cpu_child(kind, total, 0, sample)
    # roofline.traffic of this run: PMC passes in profiler children, before any GPU call here
    traffic_meas, traffic_err = None, "not measured (--no-pmc, N > 1 or a sharded workload)"
    if rank == 0 and world == 1 and not sharded and not args.no_pmc:
        traffic_meas, traffic_err = measure_traffic(args)

    # torch first: libsalz then shares torch's HIP runtime (one runtime per process), and
    # torch owns the HBM buffers the encoder reads and writes and RCCL moves.
    import torch

    dist = None
    cpu_group = None
    if launched:
        import torch.distributed as dist

        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        # gloo prints its mesh-connection notice on fd 1; keep stdout to the one JSON line
        sys.stdout.flush()
        saved, null = os.dup(1), os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)
        try:
            if args.dist_backend == "nccl":
                # nccl = RCCL over xGMI for the exchange step (lengths + payload runs, HBM to
                # HBM); a gloo side group carries the host-side barrier and timing reductions.
                dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
                cpu_group = dist.new_group(backend="gloo")
            else:  # rehearsal: everything over gloo, payload staged through host memory
                dist.init_process_group("gloo")
                cpu_group = dist.group.WORLD
            dist.barrier(group=cpu_group)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(null)

    import salz_amd
    from salz_amd.dist import block_count, gather_container, my_blocks, pack_frames, packed_len
    from tests.helpers import gen  # workload generator (tools/libdatagen.so)

    def barrier():
        if dist is not None:
            dist.barrier(group=cpu_group)

    def allreduce(vals, op):
        if dist is None:
            return vals
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=op, group=cpu_group)
        return t.tolist()

    SUM = dist.ReduceOp.SUM if dist else None
    MAX = dist.ReduceOp.MAX if dist else None

    ndev = salz_amd.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    device = local % ndev
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)

    src = gen(kind, total, 1, 16 if kind == "smx" else 256)
    if sharded:
        if total % block == 0:
            raise SystemExit("bench.py: total must not be a multiple of the block size (reference CLI)")
        nblocks = block_count(total, block)
        spans = [(b * block, min(total, (b + 1) * block)) for b in my_blocks(nblocks, rank, world)]
    else:
        nblocks = world
        spans = [(0, total)]
    block_field = block or total
    # Units of work: the single-block workloads encode their block per pass (the
    # salz_encode_safe path); the sharded ones encode consecutive blocks of the rank's range
    # batch_bytes at a time in one pipeline pass each (salz_gpu_encode_batch_device, blocks of at
    # most 4 MiB, as salz_encode_blocks does), whose
    # output is already the frames (u32 length + stream per block).
    use_batch = sharded and block % 512 == 0 and block <= (4 << 20) and args.batch_bytes > 0
    bpb = max(1, args.batch_bytes // block) if use_batch else 1
    units = [(spans[i][0], spans[min(i + bpb, len(spans)) - 1][1], min(bpb, len(spans) - i))
             for i in range(0, len(spans), bpb)]
    max_unit = max([e - s for s, e, _ in units] + [9])
    # Several units per GPU: independent encoder contexts (own stream + workspace each) on host
    # threads, so one unit's host round trips overlap another's kernels.
    nslots = args.slots or (1 if not sharded else 4)
    nslots = max(1, min(nslots, max(len(units), 1)))
    ctxs = [salz_amd.Context(device, max_unit) for _ in range(nslots)]
    ctx = ctxs[0]
    streams_t = [torch.cuda.Stream(device=dev) for _ in range(nslots)]
    blk_cap = salz_amd.encoded_len_max(block or total) + 4096
    caps = [k * (blk_cap + 4) + 64 for _, _, k in units]
    d_src = [torch.from_numpy(src[s:e].copy()).to(dev) for s, e, _ in units]
    d_dst = [torch.empty(c, dtype=torch.uint8, device=dev) for c in caps]
    d_packed = torch.empty(max(sum(caps), 1), dtype=torch.uint8, device=dev)
    d_container = torch.empty(8 + nblocks * (blk_cap + 4), dtype=torch.uint8, device=dev) if rank == 0 else None
    torch.cuda.synchronize()
    pool = None
    if nslots > 1:
        from concurrent.futures import ThreadPoolExecutor

        pool = ThreadPoolExecutor(nslots)

    def enc(k, j):
        s, e, _ = units[j]
        if use_batch:
            return ctxs[k].encode_batch_device(d_src[j].data_ptr(), e - s, block, d_dst[j].data_ptr(),
                                               caps[j], None if args.ctx_streams else streams_t[k].cuda_stream)
        return ctxs[k].encode_device(d_src[j].data_ptr(), e - s, d_dst[j].data_ptr(), caps[j],
                                     None if args.ctx_streams else streams_t[k].cuda_stream)

    # Units are handed out largest first to whichever slot is free (the last block of a sharded
    # input is the short one: it no longer runs alone at the end of the step).
    order = sorted(range(len(units)), key=lambda j: units[j][0] - units[j][1])
    import threading

    take_lock = threading.Lock()
    take_next = [0]

    def take():
        with take_lock:
            i = take_next[0]
            take_next[0] += 1
        return order[i] if i < len(order) else None

    def run_slot(k):  # slot k encodes units until none is left (ctypes drops the GIL)
        done = []
        while (j := take()) is not None:
            done.append((j, enc(k, j)))
        return done

    def step():
        """One step: encode this rank's blocks into HBM, their frames packed in block order,
        and the exchange step that assembles the whole container in rank 0's HBM (RCCL for
        N > 1)."""
        if pool is None:
            lens = [enc(0, j) for j in range(len(units))]
        else:
            lens = [0] * len(units)
            take_next[0] = 0
            for part in pool.map(run_slot, range(nslots)):
                for j, v in part:
                    lens[j] = v
        if use_batch:  # the units' frames, one after another
            nb, o = 0, 0
            for d, n in zip(d_dst, lens):
                d_packed[o:o + n].copy_(d[:n])
                o += n
            nb = o
        else:
            nb = pack_frames(d_dst, lens, d_packed)
        cont = gather_container(d_packed, nb, block_field, rank, world, None, d_container)
        torch.cuda.synchronize()
        return lens, cont

    # Warmup (untimed), then one instrumented pass for the kernel-level numbers (slot 0 alone,
    # so the HIP-event launch times are not inflated by a concurrent slot).
    for _ in range(args.warmup):
        step()
    ctx.set_timing(True)
    if units:
        enc(0, len(units) - 1)
    st = ctx.stats()  # stats of the last unit of this rank (zeros for a rank without blocks)
    ctx.set_timing(bool(args.profile_steps))
    lens, cont = step()

    # Timed region: exactly K steps bracketed by barrier + device sync on both sides.
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lens, cont = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt = allreduce([t1 - t0], MAX)[0]
    if args.profile_steps:
        st = ctx.stats()

    if use_batch:  # split every unit's frames into its blocks' streams
        streams = []
        for d, n in zip(d_dst, lens):
            data, pos = d.narrow(0, 0, n).cpu().numpy().tobytes(), 0
            while pos < len(data):
                L = int.from_bytes(data[pos:pos + 4], "little")
                streams.append(data[pos + 4:pos + 4 + L])
                pos += 4 + L
    else:
        streams = [d.narrow(0, 0, n).cpu().numpy().tobytes() for d, n in zip(d_dst, lens)]
    in_bytes, out_bytes = allreduce([float(sum(e - s for s, e in spans)),
                                     float(sum(len(x) for x in streams))], SUM)

    # Round trip of every local block through the product decoder (frame rule > 16 MiB), and on
    # rank 0 the assembled container (every rank's blocks) through the threaded decoder.
    ok = all(salz_amd.decode_safe(s_, e - s, frame=True) == src[s:e].tobytes()
             for s_, (s, e) in zip(streams, spans))
    container_ok, container_sha = None, None
    if rank == 0:
        cbytes = cont.cpu().numpy().tobytes()
        want_len = total * world if not sharded else total
        back = salz_amd.decode_blocks(cbytes, want_len)
        container_ok = back == (src.tobytes() * world if not sharded else src.tobytes())
        import hashlib

        container_sha = hashlib.sha256(cbytes).hexdigest()
    roundtrip_ok = allreduce([0.0 if ok else 1.0], SUM)[0] == 0

    value = in_bytes * args.steps / dt / 1e6
    ms_step = dt / args.steps * 1e3

    # Roofline of the dominant kernel (radix scatter): algorithmic bytes / event-timed duration.
    launches = max(int(st["radix_scatter_launches"]), 1)
    ms_rx = float(st["ms_radix_scatter"])
    # (24 B per element, + 1 B where a pass also writes the next pass's digit byte, radix.hip)
    bytes_rx = float(st.get("radix_scatter_bytes") or RADIX_BYTES_PER_ELEM * float(st["radix_scatter_elems"]))
    achieved = bytes_rx / (ms_rx * 1e-3) / 1e9 if ms_rx > 0 else 0.0
    # HBM traffic of the same kernel: the rocprofv3 --pmc passes of this run (measure_traffic),
    # per launch, against the same algorithmic-byte definition as alg_bytes_per_launch (the PMC
    # child's own launch statistics of the same encode). Without them, the last committed
    # measurement (bench_traffic.json), labelled with its file, build and date.
    alg_per_launch = bytes_rx / launches
    traffic, traffic_info = None, {"traffic_source": traffic_err}
    if traffic_meas is not None:
        traffic = traffic_meas["traffic_per_launch"]
        basis = traffic_meas.get("pmc_alg_bytes_per_launch") or alg_per_launch
        traffic_info = {
            "traffic_source": "measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                              "passes over one encode of the same input (bench.py --pmc-child), "
                              "before the timed region",
            "traffic_fetch_per_launch": traffic_meas["fetch_bytes_per_launch"],
            "traffic_write_per_launch": traffic_meas["write_bytes_per_launch"],
            "traffic_launches": traffic_meas["pmc_launches"],
            "traffic_alg_basis_per_launch": int(basis),
            "traffic_over_alg": round(traffic / basis, 3),
        }
    else:
        tpath = os.path.join(ROOT, "bench_traffic.json")
        if os.path.exists(tpath) and not sharded:
            t = json.load(open(tpath))
            if t.get("kernel") == "k_radix_scatter" and t.get("kind") == kind and t.get("size") == total:
                traffic = t["traffic_per_launch"]
                basis = t.get("alg_bytes_per_launch") or alg_per_launch
                traffic_info = {
                    "traffic_source": f"bench_traffic.json (build {t.get('head', 'unknown')}, "
                                      f"{t.get('date', 'undated')}; not this run: {traffic_err})",
                    "traffic_alg_basis_per_launch": int(basis),
                    "traffic_over_alg": round(traffic / basis, 3),
                }
    roofline = {
        "kernel": "k_radix_scatter",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_unit": "bytes/launch (2*FETCH_SIZE*1024 + WRITE_SIZE*1024, rocprofv3 PMC)",
        **traffic_info,
        "launches": launches,
        "avg_launch_us": round(ms_rx * 1e3 / launches, 2),
        "alg_bytes_per_launch": int(alg_per_launch),
        "alg_bytes_definition": "24 B per element (8 B key + 4 B value read and written) + 1 B per "
                                "element where the pass also writes the next pass's digit byte",
    }

    # Whole-pipeline roofline: A(N) = 66 n + m compulsory bytes per block
    # (each stage's int32 arrays written once and read once), over the measured block time.
    n_pos = in_bytes - 8 * nblocks
    alg_pipeline = 66.0 * n_pos + out_bytes
    pipe_gbs = alg_pipeline * args.steps / dt / 1e9
    roofline_pipeline = {"alg_bytes_per_step": int(alg_pipeline), "achieved": round(pipe_gbs, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(pipe_gbs / HBM_PEAK_GBS, 4),
                         "definition": "A(N) = 66 n + m per block (SURVEY.md §8 d3)"}

    # End to end from host buffers (the salz_encode_safe path: H2D, encode, D2H of the
    # stream), same blocks and slots; never `value`.
    e2e = None
    if not args.no_e2e:
        import numpy as np

        host_units = [src[s:e] for s, e, _ in units]
        # the caller's output buffers, allocated and touched once (the reference CLI reuses its
        # buffers too, programs/salzcli.c)
        host_out = [np.ones(c, np.uint8) for c in caps] if not use_batch else None

        def enc_host(k, j):
            if use_batch:
                return ctxs[k].encode_batch(host_units[j], block)
            return ctxs[k].encode_into(host_units[j], host_out[j])

        def run_slot_host(k):
            done = []
            while (j := take()) is not None:
                done.append(enc_host(k, j))
            return done

        def step_host():
            if pool is None:
                return [enc_host(0, j) for j in range(len(units))]
            take_next[0] = 0
            return list(pool.map(run_slot_host, range(nslots)))

        step_host()
        barrier()
        h0 = time.perf_counter()
        for _ in range(args.steps):
            step_host()
        h1 = time.perf_counter()
        barrier()
        dth = allreduce([h1 - h0], MAX)[0]
        e2e = {"value": round(in_bytes * args.steps / dth / 1e6, 3), "unit": "MB/s",
               "ms_per_step": round(dth / args.steps * 1e3, 3),
               "what": "host buffers in and out (pageable numpy memory, the output buffers "
                       "allocated once): H2D of each block, encode, D2H of each stream; same "
                       "blocks and slots as value, no exchange",
               **link_rates(torch, dev, src[units[0][0]:units[0][1]], d_dst[0], lens[0])}

    cpu = None
    parity_full = None
    if child is not None:
        import hashlib

        # the CPU baseline runs now, after every GPU measurement of this run
        out_txt, _ = child.communicate("go\n", timeout=900)
        r = json.loads(out_txt.strip().splitlines()[-1])
        first = spans[0][1] - spans[0][0]
        sample = first if args.cpu_sample <= 0 else min(args.cpu_sample, first)
        model = ""
        try:
            model = next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
        except (OSError, StopIteration):
            pass
        cpu = {
            "value": round(sample / r["enc_s"] / 1e6, 3),
            "unit": "MB/s",
            "cores": 1,
            "kind": "port",
            "sample": f"one {sample:,}-byte block of the same {kind} input, oracle/liboracle.so "
                      f"(clean-room C restatement of lib/salz.c + own SA-IS), 1 thread pinned to "
                      f"core {r['core']} (sched_setaffinity in a child started before any GPU call, "
                      f"run after the GPU timing), "
                      f"{r['enc_s']:.2f} s",
            "pinned_core": r["core"],
            "sa_s": round(r["sa_s"], 3),
            "post_sa_s": round(r["enc_s"] - r["sa_s"], 3),
            "cpu_model": model,
        }
        if sample == first and r["sha256"] is not None:
            parity_full = r["sha256"] == hashlib.sha256(streams[0]).hexdigest()

    if dist is None:
        exchange_desc = "local"
    elif args.dist_backend == "nccl":
        exchange_desc = (f"RCCL all-gather of run lengths + xGMI point-to-point payload runs, "
                         f"world {world}")
    else:
        exchange_desc = f"gloo all-gather + point-to-point runs staged through host memory, world {world}"
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
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic ({kind} surrogate, tools/datagen.c; the corpus is not available offline)",
            "config": {
                "workload": config,
                "input_bytes_total": int(in_bytes),
                "block_bytes": block_field,
                "blocks": nblocks,
                "input": kind,
                "parallelism": f"independent blocks over {world} GPU(s), {nslots} encoder slot(s) per GPU"
                               f"{f', {bpb} blocks per pipeline pass' if use_batch else ''}; "
                               f"step = encode + frame packing + exchange ("
                               f"{exchange_desc}"
                               f") + container assembly in rank 0's HBM",
            },
            "roofline": roofline,
            "roofline_pipeline": roofline_pipeline,
            "cpu_baseline": cpu,
            "value_e2e": e2e["value"] if e2e else None,
            "e2e": e2e,
            "encoded_bytes": int(out_bytes),
            "container_bytes": int(cont.numel()),
            "container_sha256": container_sha,
            "ratio": round(in_bytes / out_bytes, 4),
            "roundtrip_ok": bool(roundtrip_ok),
            "container_roundtrip_ok": container_ok,
            "parity_vs_cpu_port": parity_full,
            "stages_ms_last_block": {k: round(st[k], 3) for k in
                                     ("ms_sa", "ms_lcp", "ms_ansv", "ms_parse", "ms_emit", "ms_total")},
            "sa_rounds": st["sa_rounds"],
            "sa_dc3_levels": st["sa_dc3_levels"],
            "parse_iters": st["parse_iters"],
        }
        print(json.dumps(line), flush=True)
    if pool is not None:
        pool.shutdown()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
