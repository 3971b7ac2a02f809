"""Time one block encoded with its suffix array split over the ranks (salz_amd.dist.encode_block_split,
SURVEY.md §8 f3). One process per GPU, launched like bench.py:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_split.py \
        [--kind text|fib|mixed] [--size BYTES] [--steps K]

Each rank uses cuda:LOCAL_RANK and the nccl backend when it has a GPU of its own: the per-round
exchange then runs through the library's own RCCL communicator (salz_gpu_dist_comm, over xGMI), or
through torch.distributed callbacks with --callbacks; gloo with host staging when several ranks share
one GPU (--gloo; a correctness rehearsal only). The block is resident in HBM before timing. One rank
reads rank[i + h] locally and runs no collective; SALZ_SA=xchg forces the exchange there.
Rank 0 prints one JSON line: MB/s of the whole block (strong scaling: one block whatever N) and
whether the stream equals the single-GPU salz_gpu_encode_device stream.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="text")
    ap.add_argument("--size", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gloo", action="store_true")
    ap.add_argument("--callbacks", action="store_true",
                    help="nccl: exchange through torch.distributed callbacks instead of the library's RCCL comm")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    import salz_amd
    from salz_amd.dist import DistComm, encode_block_split
    from tests.helpers import gen

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = 0 if args.gloo else local
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if args.gloo else "nccl",
                            **({} if args.gloo else {"device_id": torch.device("cuda", dev)}))
    rank, world = dist.get_rank(), dist.get_world_size()
    src = gen(args.kind, args.size, 1)
    ctx = salz_amd.Context(dev, len(src))
    comm = None if args.gloo or args.callbacks else DistComm(dev)
    d_src = torch.from_numpy(src.copy()).to(torch.device("cuda", dev))  # resident, like bench.py's blocks
    cache = {}
    out = None
    for _ in range(args.warmup):
        out = encode_block_split(d_src, dev, ctx=ctx, comm=comm, cache=cache)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):  # (the stream stays in HBM, as bench.py's value counts it)
        out = encode_block_split(d_src, dev, ctx=ctx, comm=comm, cache=cache, as_tensor=True)
    torch.cuda.synchronize()
    dist.barrier()
    dt = (time.perf_counter() - t0) / args.steps
    if rank == 0:
        out = out.cpu().numpy().tobytes()
        ref = ctx.encode(src)
        print(json.dumps({"metric": "split-block compress MB/s", "value": round(len(src) / dt / 1e6, 1),
                          "unit": "MB/s", "n_ranks": world, "backend": "gloo" if args.gloo else "nccl",
                          "ms_per_block": round(dt * 1e3, 2), "input": args.kind, "bytes": len(src),
                          "scaling": "strong", "identical_to_single_gpu": out == ref,
                          "exchange": "gloo callbacks" if args.gloo else "torch.distributed callbacks"
                          if args.callbacks else "RCCL in the library",
                          "xchg_forced": "xchg" in os.environ.get("SALZ_SA", "")}), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
