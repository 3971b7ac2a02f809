"""Block-sharded container encode over processes, one per GPU.

The reference CLI encodes a file as consecutive independent blocks and frames them as
"ZLAS" + u32 block size, then u32 length + stream per block (programs/salzcli.c:102-185,
the loop at :143-179). Blocks share nothing (lib/salz.c:777-823), so the path shards by block:

  1. rank r encodes a CONTIGUOUS range of blocks on its own GPU (no data-path collective);
     its frames (u32 length + stream, in block order) are packed into one byte buffer, so in
     the container they form one contiguous run;
  2. the one exchange step: an all-gather of each rank's packed byte count, from which every
     rank knows where its run starts in the container (exclusive scan in rank order);
  3. rank 0 receives every other rank's run straight into its place in the container
     (point-to-point, all receives in flight together), after the 8-byte header and its own run.

With the nccl backend (RCCL on ROCm) the buffers are HBM tensors: the lengths are all-gathered
and the payload runs travel GPU to GPU over xGMI, and the container is assembled in rank 0's
HBM. The same code runs on gloo with CPU tensors (tests/test_dist.py, world 2 and 3).
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional, Sequence

import numpy as np

MAGIC = 0x53414C5A  # "ZLAS" little-endian (programs/salzcli.c:115-121)


def block_count(src_len: int, block_size: int) -> int:
    """Blocks the reference CLI loop produces: it always encodes the trailing fread() chunk,
    an empty one when src_len is a multiple of block_size (programs/salzcli.c:143-179)."""
    return src_len // block_size + 1


def my_blocks(nblocks: int, rank: int, world: int) -> list[int]:
    """Rank r's blocks: a contiguous range, sizes differing by at most one across ranks."""
    base, extra = divmod(nblocks, world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


def container_offsets(lengths: Sequence[int]) -> tuple[np.ndarray, int]:
    """Byte offset of each block's u32 length field, and the container size."""
    frame = np.asarray(lengths, dtype=np.int64) + 4
    offs = 8 + np.concatenate([[0], np.cumsum(frame)[:-1]]) if len(frame) else np.zeros(0, np.int64)
    return offs.astype(np.int64), int(8 + frame.sum())


def header(block_size: int) -> bytes:
    return MAGIC.to_bytes(4, "little") + int(block_size).to_bytes(4, "little")


def assemble(block_size: int, streams: Sequence[bytes]) -> bytes:
    offs, total = container_offsets([len(s) for s in streams])
    out = bytearray(total)
    out[0:8] = header(block_size)
    for o, s in zip(offs, streams):
        out[o:o + 4] = len(s).to_bytes(4, "little")
        out[o + 4:o + 4 + len(s)] = s
    return bytes(out)


def packed_len(lengths: Sequence[int]) -> int:
    return int(sum(int(L) + 4 for L in lengths))


def pack_frames(streams, lengths: Sequence[int], out):
    """Write u32 length + stream for each block into the byte tensor `out` (same device as the
    streams: HBM for the GPU path). Returns the number of bytes written."""
    import torch

    lens = [int(L) for L in lengths]
    hdr = torch.tensor(np.frombuffer(np.asarray(lens, dtype="<u4").tobytes(), np.uint8).copy())
    hdr = hdr.to(out.device, non_blocking=False)
    o = 0
    for k, (s, L) in enumerate(zip(streams, lens)):
        out[o:o + 4].copy_(hdr[4 * k:4 * k + 4])
        out[o + 4:o + 4 + L].copy_(s[:L])
        o += 4 + L
    return o


def gather_container(packed, nbytes: int, block_size: int, rank: int = 0, world: int = 1,
                     group=None, out=None):
    """The exchange step. `packed` holds this rank's `nbytes` of frames. Returns the container
    tensor on rank 0 (on packed's device; `out` may supply its storage), None elsewhere.

    Whenever a process group is initialised (world 1 included, so a one-rank launch runs the
    same collectives), the counts are all-gathered and the runs travel point to point. With
    nccl (RCCL) the HBM tensors go straight through; with gloo, device tensors are staged
    through host memory (several ranks may then share one GPU)."""
    import torch

    dev = packed.device
    dist = None
    try:
        import torch.distributed as _d

        if _d.is_available() and _d.is_initialized():
            dist = _d
    except ImportError:
        pass
    if dist is None and world > 1:
        raise RuntimeError("gather_container: world > 1 needs an initialised process group")
    if dist is not None and dist.get_world_size(group) != world:
        # (a local container inside a larger job would wait on peers that never join)
        raise RuntimeError(f"gather_container: world={world} but the process group has "
                           f"{dist.get_world_size(group)} ranks")
    host = dist is not None and dist.get_backend(group) == "gloo" and packed.is_cuda
    cdev = torch.device("cpu") if host else dev
    if dist is not None:
        cnt = torch.tensor([nbytes], dtype=torch.int64, device=cdev)
        allc = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(allc, cnt, group=group)
        counts = [int(c.item()) for c in allc]
    else:
        counts = [nbytes]
    total = 8 + sum(counts)
    if rank != 0:
        if nbytes:
            src = packed[:nbytes].cpu() if host else packed[:nbytes]
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, src, 0, group=group)]):
                req.wait()
        return None
    if out is None or out.numel() < total:
        out = torch.empty(total, dtype=torch.uint8, device=dev)
    out[:8].copy_(torch.tensor(list(header(block_size)), dtype=torch.uint8).to(dev))
    out[8:8 + counts[0]].copy_(packed[:counts[0]])
    if dist is not None:
        ops, bufs, off = [], [], 8 + counts[0]
        for r in range(1, world):
            if counts[r]:
                dstv = out[off:off + counts[r]]
                buf = torch.empty(counts[r], dtype=torch.uint8) if host else dstv
                bufs.append((dstv, buf))
                ops.append(dist.P2POp(dist.irecv, buf, r, group=group))
            off += counts[r]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if host:
            for dstv, buf in bufs:
                dstv.copy_(buf)
    return out[:total]


def gpu_block_encoder(device: int, max_block: int) -> Callable[[np.ndarray], bytes]:
    """Per-block encoder on one GPU (a cached salz_gpu_ctx; fails loudly without a GPU)."""
    import salz_amd

    ctx = salz_amd.Context(device, max_block)
    return ctx.encode


def encode_container(src: np.ndarray, block_size: int, encode_block: Callable[[np.ndarray], bytes],
                     rank: int = 0, world: int = 1, group=None) -> Optional[bytes]:
    """Encode src as the reference container with blocks sharded over `world` ranks (host
    buffers; gloo or any backend that moves CPU tensors). Returns the container on rank 0,
    None elsewhere. Raises on any block failure (the reference CLI aborts the whole file,
    programs/salzcli.c:156-161)."""
    import torch

    nblocks = block_count(len(src), block_size)
    mine = my_blocks(nblocks, rank, world)
    streams = [encode_block(src[b * block_size:(b + 1) * block_size]) for b in mine]
    lens = [len(s) for s in streams]
    packed = torch.empty(max(packed_len(lens), 1), dtype=torch.uint8)
    n = pack_frames([torch.frombuffer(bytearray(s), dtype=torch.uint8) if s else torch.empty(0, dtype=torch.uint8)
                     for s in streams], lens, packed)
    out = gather_container(packed, n, block_size, rank, world, group)
    return None if out is None else out.numpy().tobytes()


# ---- one block's suffix array split over the ranks (dsa.hip) -------------------

class _Collectives:
    """The all-to-all and allreduce the library's split suffix sort calls back (salz_dist_ops),
    over torch.distributed: device tensors straight through RCCL (nccl backend, xGMI), or staged
    through host memory for gloo (the tests: several ranks on one GPU)."""

    def __init__(self, xsend, xrecv, world: int, group=None):
        import torch
        import torch.distributed as dist

        import salz_amd

        self.xsend, self.xrecv, self.world, self.group = xsend, xrecv, world, group
        self.host = dist.get_backend(group) == "gloo"
        self.cdev = torch.device("cpu") if self.host else xsend.device
        self.error = None
        self._a2a = salz_amd.DIST_ALLTOALL(self._alltoall)
        self._ar = salz_amd.DIST_ALLREDUCE(self._allreduce)
        self.ops = salz_amd.DistOps(None, self._a2a, self._ar)

    def _alltoall(self, _user, send_counts, recv_counts):
        import torch
        import torch.distributed as dist

        try:
            sc = [int(send_counts[i]) for i in range(self.world)]
            t = torch.tensor(sc, dtype=torch.int64, device=self.cdev)
            r = torch.empty_like(t)
            dist.all_to_all_single(r, t, group=self.group)
            rc = [int(v) for v in r.tolist()]
            for i, v in enumerate(rc):
                recv_counts[i] = v
            ns, nr = sum(sc), sum(rc)
            if self.host:
                recv = torch.empty(nr, dtype=torch.int32)
                dist.all_to_all_single(recv, self.xsend[:ns].cpu(), rc, sc, group=self.group)
                self.xrecv[:nr].copy_(recv)
            else:
                dist.all_to_all_single(self.xrecv[:nr], self.xsend[:ns], rc, sc, group=self.group)
            if self.xsend.is_cuda:
                torch.cuda.synchronize(self.xsend.device)
            return 0
        except Exception as e:  # reported by the caller; the library fails the call
            self.error = e
            return -1

    def _allreduce(self, _user, value):
        import torch
        import torch.distributed as dist

        try:
            t = torch.tensor([int(value[0])], dtype=torch.int64, device=self.cdev)
            dist.all_reduce(t, group=self.group)
            value[0] = int(t.item())
            return 0
        except Exception as e:
            self.error = e
            return -1


def _gather_pieces(piece, offsets, rank: int, world: int, full, group=None, host: bool = False):
    """Rank r's piece (int32 tensor, offsets[r+1] - offsets[r] entries) into full[offsets[r]:...]
    on rank 0, point to point."""
    import torch
    import torch.distributed as dist

    lens = [offsets[r + 1] - offsets[r] for r in range(world)]
    if rank != 0:
        if lens[rank]:
            src = piece[:lens[rank]].cpu() if host else piece[:lens[rank]]
            dist.send(src, 0, group=group)
        return
    full[:lens[0]].copy_(piece[:lens[0]])
    for r in range(1, world):
        if lens[r]:
            if host:
                buf = torch.empty(lens[r], dtype=torch.int32)
                dist.recv(buf, r, group=group)
                full[offsets[r]:offsets[r + 1]].copy_(buf)
            else:
                dist.recv(full[offsets[r]:offsets[r + 1]], r, group=group)


class DistComm:
    """The library's own RCCL communicator for the split suffix sort (salz_gpu_dist_comm): rank 0
    makes the 128-byte id, the group broadcasts it, every rank joins. The per-round all-to-all
    and allreduce then run inside the library on its stream, with no callback into Python."""

    def __init__(self, device: int, group=None):
        import torch
        import torch.distributed as dist

        import salz_amd

        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        idb = (ctypes.c_uint8 * 128)()
        if self.rank == 0 and salz_amd.lib.salz_gpu_dist_comm_id(idb) != 0:
            raise salz_amd.SalzError(f"RCCL unique id: {salz_amd.last_error()}")
        obj = [bytes(idb) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group, device=torch.device("cuda", device))
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        self.handle = salz_amd.lib.salz_gpu_dist_comm_create(device, self.world, self.rank, idb)
        if not self.handle:
            raise salz_amd.SalzError(f"RCCL communicator: {salz_amd.last_error()}")

    def close(self):
        import salz_amd

        if self.handle:
            salz_amd.lib.salz_gpu_dist_comm_destroy(self.handle)
            self.handle = None


def encode_block_split(src, device: int = 0, group=None, ctx=None, comm: Optional[DistComm] = None,
                       cache: Optional[dict] = None, as_tensor: bool = False):
    """One block encoded with its suffix array split over the ranks of `group` (every rank
    passes the same block: a host array, or a uint8 tensor on this rank's GPU). Each rank sorts
    its two-byte-prefix bucket on its GPU, exchanging only rank[i + h] requests per doubling
    round: through the library's own RCCL communicator when `comm` is given (DistComm, nccl
    groups), else through torch.distributed callbacks (any backend; gloo stages through host
    memory). Rank 0 gathers the pieces (and their LCPs) and runs the rest of the pipeline.
    A block of 2^20 suffixes or more that the repetition probe sends to DC3 is not split (the
    split sorter is prefix doubling only, dsa.hip): rank 0 encodes it whole on its GPU instead, and
    cache["split"] says which way the last block went.
    `cache` (a dict kept by the caller) holds the device buffers across calls. Returns the stream
    on rank 0 (bit-identical to salz_encode_safe; with as_tensor, the uint8 tensor of it in HBM,
    a view of the cached output buffer), None elsewhere."""
    import torch
    import torch.distributed as dist

    import salz_amd

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", device)
    if isinstance(src, torch.Tensor):
        if src.dtype != torch.uint8:
            raise TypeError(f"encode_block_split: a uint8 tensor is required, not {src.dtype}")
        text = (src if src.device == dev else src.to(dev)).reshape(-1).contiguous()
    else:
        s = np.ascontiguousarray(np.asarray(src, dtype=np.uint8).reshape(-1))
        text = torch.from_numpy(s.copy()).to(dev)
    N = int(text.numel())
    n = N - 8
    own = ctx is None
    if own:
        ctx = salz_amd.Context(device, N)
    bufs = cache if cache is not None else {}
    try:
        key = (N, dev.index, rank)  # (device buffers: one set per block size, device and rank)
        if bufs.get("key") != key:
            xcap = N + 64
            bufs.clear()
            bufs.update(key=key, xcap=xcap,
                        xsend=torch.empty(xcap, dtype=torch.int32, device=dev),
                        xrecv=torch.empty(xcap, dtype=torch.int32, device=dev),
                        sa_piece=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                        lcp_piece=torch.empty(max(n, 1), dtype=torch.int32, device=dev))
            if rank == 0:
                bufs.update(full_sa=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                            full_lcp=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                            out=torch.empty(salz_amd.encoded_len_max(N), dtype=torch.uint8, device=dev))
        xsend, xrecv, sa_piece, lcp_piece = bufs["xsend"], bufs["xrecv"], bufs["sa_piece"], bufs["lcp_piece"]
        torch.cuda.synchronize(dev)
        offs = (ctypes.c_uint64 * (world + 1))()
        lcp_ok = ctypes.c_int(0)
        host = dist.get_backend(group) == "gloo"
        if comm is not None:
            rc = salz_amd.lib.salz_gpu_dist_suffix_array_comm(
                ctx.handle, text.data_ptr(), N, comm.handle, xsend.data_ptr(), xrecv.data_ptr(), bufs["xcap"],
                sa_piece.data_ptr(), lcp_piece.data_ptr(), offs, ctypes.byref(lcp_ok))
            err = ""
        else:
            coll = _Collectives(xsend, xrecv, world, group)
            rc = salz_amd.lib.salz_gpu_dist_suffix_array(
                ctx.handle, text.data_ptr(), N, world, rank, ctypes.byref(coll.ops), xsend.data_ptr(),
                xrecv.data_ptr(), bufs["xcap"], sa_piece.data_ptr(), lcp_piece.data_ptr(), offs, ctypes.byref(lcp_ok))
            err = coll.error or ""
        if rc == 1:  # not split (a repetitive block, every rank alike): rank 0 encodes it whole (DC3)
            bufs["split"] = False
            if rank != 0:
                return None
            out = bufs["out"]
            olen = ctx.encode_device(text.data_ptr(), N, out.data_ptr(), out.numel())
            return out[:olen] if as_tensor else out[:olen].cpu().numpy().tobytes()
        if rc != 0:
            raise salz_amd.SalzError(f"split suffix sort failed: {salz_amd.last_error()} {err}")
        bufs["split"] = True
        offsets = [int(offs[i]) for i in range(world + 1)]
        if world > 1:
            ok = torch.tensor([lcp_ok.value], dtype=torch.int64, device="cpu" if host else dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
            with_lcp = bool(ok.item())
        else:
            with_lcp = bool(lcp_ok.value)
        full_sa = bufs.get("full_sa") if rank == 0 else None
        full_lcp = bufs.get("full_lcp") if rank == 0 and with_lcp else None
        if world > 1:
            _gather_pieces(sa_piece, offsets, rank, world, full_sa, group, host)
            if with_lcp:
                _gather_pieces(lcp_piece, offsets, rank, world, full_lcp, group, host)
        else:  # one rank: its piece is the whole array
            full_sa, full_lcp = sa_piece, (lcp_piece if with_lcp else None)
        if rank != 0:
            return None
        fix = [o for o in offsets[:world] if o < n]  # every piece's first entry
        fixa = (ctypes.c_uint64 * max(len(fix), 1))(*fix)
        out = bufs["out"]
        olen = ctypes.c_size_t(0)
        torch.cuda.synchronize(dev)
        if salz_amd.lib.salz_gpu_encode_from_sa(ctx.handle, text.data_ptr(), N, full_sa.data_ptr(),
                                                full_lcp.data_ptr() if with_lcp else None, fixa,
                                                len(fix) if with_lcp else 0, out.data_ptr(), out.numel(),
                                                ctypes.byref(olen)) != 0:
            raise salz_amd.SalzError(f"encode from suffix array failed: {salz_amd.last_error()}")
        if as_tensor:
            return out[:olen.value]
        return out[:olen.value].cpu().numpy().tobytes()
    finally:
        if own:
            ctx.close()
