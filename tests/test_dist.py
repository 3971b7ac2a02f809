"""Multi-process block sharding on CPU: gloo process groups, world 2 and 3.

The per-block encoder is the CPU oracle here (test infrastructure), so these tests cover the
sharding, the length exchange, the container offsets and the payload gather; the GPU
encoder behind the same interface is covered by tests/test_gpu_parity.py.
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

from tests.helpers import gen, oracle_encode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_block(b: np.ndarray) -> bytes:
    rc, out = oracle_encode(b)
    if rc != 0:
        raise RuntimeError(f"block of {len(b)} bytes failed")
    return out


def _worker(rank, world, port, kind, size, block, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from salz_amd.dist import encode_container

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        src = gen(kind, size, 3)
        out = encode_container(src, block, _oracle_block, rank, world)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _run(world, kind, size, block):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kind, size, block, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world,kind,size,block", [(2, "text", 300_000 + 123, 65536),
                                                   (3, "mixed", 250_000 + 77, 32768),
                                                   (2, "fib", 40_000, 65536),
                                                   (3, "text", 40_000, 32768)])
def test_sharded_container_matches_single_process(world, kind, size, block):
    from salz_amd.dist import assemble, block_count

    got = _run(world, kind, size, block)
    src = gen(kind, size, 3)
    streams = [_oracle_block(src[b * block:(b + 1) * block]) for b in range(block_count(size, block))]
    assert got == assemble(block, streams)
    # the container decodes back with the product's threaded host decoder
    import salz_amd

    assert salz_amd.decode_blocks(got, size) == src.tobytes()


def test_container_layout_matches_reference_cli():
    from salz_amd.dist import assemble, container_offsets

    offs, total = container_offsets([5, 7, 1])
    assert offs.tolist() == [8, 17, 28] and total == 33
    c = assemble(1 << 20, [b"abcde", b"x" * 7, b"y"])
    assert c[:8] == bytes.fromhex("5a4c415300001000")  # "ZLAS", u32 block size
    assert c[8:12] == (5).to_bytes(4, "little") and c[12:17] == b"abcde"


def test_shards_cover_every_block_once():
    from salz_amd.dist import my_blocks

    for world in (1, 2, 3, 8):
        for nb in (1, 7, 15, 16):
            seen = sorted(b for r in range(world) for b in my_blocks(nb, r, world))
            assert seen == list(range(nb))


def _world1_worker(port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from salz_amd.dist import gather_container, header

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        packed = torch.arange(40, dtype=torch.uint8)
        out = gather_container(packed, 37, 1 << 20, 0, 1)
        q.put(bytes(out.numpy().tobytes()) == header(1 << 20) + bytes(range(37)))
    finally:
        dist.destroy_process_group()


def test_gather_container_world1_process_group():
    """With a process group initialised at world 1 (bench.py --launch), the exchange step runs
    its collectives (all-gather of the run length) and still yields header + the rank's run."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_worker, args=(_free_port(), q))
    p.start()
    ok = q.get(timeout=120)
    p.join(timeout=60)
    assert ok and p.exitcode == 0


def _xchg_worker(rank, world, port, q):
    """One exchange of the split suffix sort both ways: torch's all_to_all_single with split sizes
    (the gloo callbacks' path, salz_amd/dist.py) and the grouped point-to-point sends and receives
    of the in-library RCCL path (dsa.hip RcclXchg) at the offsets the library computes."""
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import salz_amd

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(100 + rank)
        sc = [int(x) for x in rng.integers(0, 40, world)]
        sc[(rank + 1) % world] = 0  # a peer that gets nothing
        rc_t = torch.zeros(world, dtype=torch.int64)
        dist.all_to_all_single(rc_t, torch.tensor(sc, dtype=torch.int64))
        rc = [int(x) for x in rc_t]
        xsend = torch.tensor([rank * 1_000_000 + d * 1000 + k for d in range(world) for k in range(sc[d])],
                             dtype=torch.int64)
        want = torch.zeros(sum(rc), dtype=torch.int64)
        dist.all_to_all_single(want, xsend, rc, sc)
        so, ro = salz_amd.xchg_offsets(sc, rc)
        got = torch.full((sum(rc),), -1, dtype=torch.int64)
        reqs = []
        for r in range(world):
            if r == rank:
                got[ro[r]:ro[r] + rc[r]] = xsend[so[r]:so[r] + sc[r]]
                continue
            if sc[r]:
                reqs.append(dist.isend(xsend[so[r]:so[r] + sc[r]].clone(), r))
            if rc[r]:
                buf = torch.empty(rc[r], dtype=torch.int64)
                reqs.append((dist.irecv(buf, r), buf, ro[r]))
        for x in reqs:
            if isinstance(x, tuple):
                x[0].wait()
                got[x[2]:x[2] + len(x[1])] = x[1]
            else:
                x.wait()
        q.put((rank, bool(torch.equal(got, want)), sc, rc))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_exchange_offsets_match_all_to_all(world):
    """The in-library RCCL exchange's packing: the per-peer send and receive offsets
    it uses for its grouped ncclSend / ncclRecv give, rank by rank, exactly what all_to_all_single
    with split sizes (the gloo callbacks' path) delivers, with empty runs among them. The RCCL calls
    themselves run only at world 1 on the one-GPU box (tests/test_dist_split.py); a multi-rank RCCL
    exchange is not covered by this suite."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_xchg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
