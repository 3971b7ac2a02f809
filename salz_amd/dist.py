"""Block-sharded container encode over processes, one per GPU.

The reference CLI encodes a file as consecutive independent blocks and frames them as
"ZLAS" + u32 block size, then u32 length + stream per block (programs/salzcli.c:102-185).
Blocks share nothing (lib/salz.c:777-823), so the path shards by block:

  1. rank r encodes blocks b with b % world == r on its own GPU (no data-path collective);
  2. ranks exchange the per-block encoded lengths: an all-reduce of a zero-filled length
     vector, which is an all-gather for disjoint block sets (the one exchange step);
  3. every rank derives the container offsets from the lengths (exclusive scan in block
     order), and rank 0 gathers the payloads and writes them at those offsets.

The exchange runs on a torch.distributed process group (gloo: lengths are a few hundred
bytes, payloads are at most the input size). `encode_block` is the per-block encoder: the
GPU path (`gpu_block_encoder`) in production, the CPU oracle in the gloo tests.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

MAGIC = 0x53414C5A  # "ZLAS" little-endian (programs/salzcli.c:115-121)


def block_count(src_len: int, block_size: int) -> int:
    """Blocks the reference CLI loop produces: it always encodes the trailing fread() chunk,
    an empty one when src_len is a multiple of block_size (programs/salzcli.c:143-179)."""
    return src_len // block_size + 1


def my_blocks(nblocks: int, rank: int, world: int) -> list[int]:
    return list(range(rank, nblocks, world))


def container_offsets(lengths: Sequence[int]) -> tuple[np.ndarray, int]:
    """Byte offset of each block's u32 length field, and the container size."""
    frame = np.asarray(lengths, dtype=np.int64) + 4
    offs = 8 + np.concatenate([[0], np.cumsum(frame)[:-1]]) if len(frame) else np.zeros(0, np.int64)
    return offs.astype(np.int64), int(8 + frame.sum())


def assemble(block_size: int, streams: Sequence[bytes]) -> bytes:
    offs, total = container_offsets([len(s) for s in streams])
    out = bytearray(total)
    out[0:4] = MAGIC.to_bytes(4, "little")
    out[4:8] = int(block_size).to_bytes(4, "little")
    for o, s in zip(offs, streams):
        out[o:o + 4] = len(s).to_bytes(4, "little")
        out[o + 4:o + 4 + len(s)] = s
    return bytes(out)


def gpu_block_encoder(device: int, max_block: int) -> Callable[[np.ndarray], bytes]:
    """Per-block encoder on one GPU (a cached salz_gpu_ctx; fails loudly without a GPU)."""
    import salz_amd

    ctx = salz_amd.Context(device, max_block)
    return ctx.encode


def encode_container(src: np.ndarray, block_size: int, encode_block: Callable[[np.ndarray], bytes],
                     rank: int = 0, world: int = 1, group=None) -> Optional[bytes]:
    """Encode src as the reference container with blocks sharded over `world` ranks.
    Returns the container on rank 0, None elsewhere. Raises on any block failure (the
    reference CLI aborts the whole file, programs/salzcli.c:156-161)."""
    import torch
    import torch.distributed as dist

    nblocks = block_count(len(src), block_size)
    mine = my_blocks(nblocks, rank, world)
    streams = {b: encode_block(src[b * block_size:(b + 1) * block_size]) for b in mine}

    lengths = torch.zeros(nblocks, dtype=torch.int64)
    for b, s in streams.items():
        lengths[b] = len(s)
    if world > 1:
        dist.all_reduce(lengths, op=dist.ReduceOp.SUM, group=group)
    lens = lengths.tolist()

    if world == 1:
        return assemble(block_size, [streams[b] for b in range(nblocks)])
    if rank != 0:
        if mine:
            payload = torch.from_numpy(np.frombuffer(b"".join(streams[b] for b in mine), np.uint8).copy())
            dist.send(payload, dst=0, group=group)
        return None
    got = dict(streams)
    for r in range(1, world):
        theirs = my_blocks(nblocks, r, world)
        if not theirs:
            continue
        buf = torch.empty(sum(lens[b] for b in theirs), dtype=torch.uint8)
        dist.recv(buf, src=r, group=group)
        data = buf.numpy().tobytes()
        o = 0
        for b in theirs:
            got[b] = data[o:o + lens[b]]
            o += lens[b]
    return assemble(block_size, [got[b] for b in range(nblocks)])
