"""One rank of a split-suffix-array encode (salz_amd.dist.encode_block_split), for
tests/test_dist_split.py: every rank encodes the same blocks over gloo on one GPU; rank 0 writes
the streams.

  python tests/split_worker.py RANK WORLD PORT IN.npz OUT.npz [perblock|nccl]

perblock: every block gets a context of its own, sized to that block (encode_block_split
without ctx), instead of one context sized to the largest block.
nccl: the nccl backend with the library's own RCCL communicator (salz_amd.dist.DistComm) for the
exchange (one rank per GPU: world 1 on the test box).
"""
import os
import sys

import numpy as np


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    src_path, out_path = sys.argv[4], sys.argv[5]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist

    import salz_amd
    from salz_amd.dist import encode_block_split

    opt = sys.argv[6] if len(sys.argv) > 6 else ""
    comm = None
    if opt == "nccl":
        import torch
        from salz_amd.dist import DistComm

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
        comm = DistComm(0)
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    data = np.load(src_path)
    names = sorted(data.files)
    perblock = opt == "perblock"
    ctx = None if perblock else salz_amd.Context(0, max(len(data[k]) for k in names))
    out = {}
    info = []  # per block (rank 0): split or not, and the DC3 levels of the encode
    cache = {}
    for k in names:
        s = encode_block_split(data[k], 0, ctx=ctx, comm=comm, cache=cache)
        if rank == 0:
            out[k] = np.frombuffer(s, np.uint8)
            lv = ctx.stats()["sa_dc3_levels"] if ctx is not None else -1
            info.append((k, int(cache["split"]), lv))
    if rank == 0:
        out["__info__"] = np.array(repr(info))
    if ctx is not None:
        ctx.close()
    if comm is not None:
        comm.close()
    if rank == 0:
        np.savez(out_path, **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
