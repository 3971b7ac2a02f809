"""salz_encode_safe from several threads (VERDICT r02 missing #2).

The reference encoder keeps no globals and allocates per call (lib/salz.c:175-256, :777-823),
so T threads calling salz_encode_safe have T blocks in flight. Here the calls go through the C
ABI (ctypes into libsalz.so: salz_encode_safe, plain pointers and sizes; ctypes releases the
GIL) and the library's context pool hands each call an idle context (own HIP stream and
workspace), preferring the caller's current device (pipeline.hip, salz_gpu_encode_default).
Every output must equal the CPU port's stream; four threads must beat one thread's aggregate
MB/s by 1.3x on 1 MiB and 16 MiB blocks.
"""
import ctypes
import threading
import time

import numpy as np
import pytest

from tests.helpers import enc_max, gen, golden, oracle_encode, sha256

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    import salz_amd

    if salz_amd.device_count() == 0:
        pytest.fail("no HIP device visible: GPU tests need an MI355X")
    return salz_amd.lib


def _encode_safe(lib, blk: np.ndarray) -> bytes:
    cap = enc_max(len(blk))
    out = np.empty(cap, np.uint8)
    n = ctypes.c_size_t(cap)
    rc = lib.salz_encode_safe(blk.ctypes.data, len(blk), out.ctypes.data, ctypes.byref(n))
    assert rc == 0
    return out[: n.value].tobytes()


def _run(lib, blocks, threads):
    """Encode every block once, `threads` callers pulling block indices; returns (outputs, s)."""
    outs = [None] * len(blocks)
    nxt = [0]
    mu = threading.Lock()

    def work():
        while True:
            with mu:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(blocks):
                return
            outs[i] = _encode_safe(lib, blocks[i])

    ths = [threading.Thread(target=work) for _ in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return outs, time.perf_counter() - t0


def _blocks(kind, size, count):
    src = gen(kind, size * count + 1, 11)
    return [np.ascontiguousarray(src[i * size:(i + 1) * size]) for i in range(count)]


def test_safe_four_threads_match_oracle(lib):
    blocks = (_blocks("text", 1 << 20, 6) + _blocks("mixed", 700_001, 4) + [gen("fib", 500_000)]
              + [gen("smx", 400_000, 2, 4)] + _blocks("text", 9_000, 8))
    refs = [oracle_encode(b)[1] for b in blocks]
    for rep in range(2):
        outs, _ = _run(lib, blocks, 4)
        bad = [i for i, (o, r) in enumerate(zip(outs, refs)) if o != r]
        assert bad == [], f"pass {rep}: blocks {bad} differ from the oracle"


@pytest.mark.parametrize("size,count", [(1 << 20, 48), (16 << 20, 8)])
def test_safe_four_threads_scale(lib, size, count):
    blocks = _blocks("text", size, count)
    _run(lib, blocks[:4], 4)  # warm every pool context up to this block size
    one = min(_run(lib, blocks, 1)[1] for _ in range(3))
    outs, four = min((_run(lib, blocks, 4) for _ in range(3)), key=lambda r: r[1])
    mbs1 = size * count / one / 1e6
    mbs4 = size * count / four / 1e6
    print(f"salz_encode_safe {size} B blocks: 1 thread {mbs1:.0f} MB/s, 4 threads {mbs4:.0f} MB/s "
          f"({mbs4 / mbs1:.2f}x)")
    rc, ref = oracle_encode(blocks[0])
    assert outs[0] == ref
    # (round 3: 1.63x on 16 MiB blocks; round 4: 1.46x, one thread faster while four saturate
    # the GPU at about the C3 rate)
    assert mbs4 >= 1.3 * mbs1, f"4 threads {mbs4:.0f} MB/s vs 1 thread {mbs1:.0f} MB/s"


def test_safe_pool_cache_cap(lib):
    """The pool caps what idle workspaces hold per device: after one
    256 MiB call (about 30 GB of workspace) the device's pool falls back under the cap, and
    1 MiB calls that follow keep it there; every stream still equals the reference's."""
    cap = 8 << 30
    lib.salz_gpu_pool_config(0, cap, -1)
    try:
        vec = next(v for v in golden("appendix_c.json")["vectors"] if v["n"] == 1 << 28)
        out = _encode_safe(lib, gen("fib", vec["n"]))
        assert sha256(out) == vec["out_sha256"]
        held = lib.salz_gpu_pool_bytes(0)
        assert held <= cap, f"{held} bytes held after the 256 MiB call"
        blocks = _blocks("text", 1 << 20, 8)
        outs, _ = _run(lib, blocks, 4)
        assert outs == [oracle_encode(b)[1] for b in blocks]
        held = lib.salz_gpu_pool_bytes(0)
        assert 0 < held <= cap, f"{held} bytes held after the 1 MiB calls"
    finally:
        lib.salz_gpu_pool_config(0, 32 << 30, -1)


def test_safe_pool_concurrent_large_blocks_keep_workspaces(lib):
    """Two threads encoding large blocks at once, their two workspaces together over the cache cap
    but each under it: a busy context's workspace does not count against the cap, so
    neither caller frees its own workspace after every call and reallocates it on the next."""
    blocks = _blocks("text", 24 << 20, 2)
    refs = [oracle_encode(b)[1] for b in blocks]
    try:
        lib.salz_gpu_pool_config(0, 1, -1)  # release every idle workspace after this call
        _encode_safe(lib, blocks[0][:100_000])
        assert lib.salz_gpu_pool_bytes(0) == 0
        lib.salz_gpu_pool_config(0, 64 << 30, -1)
        _encode_safe(lib, blocks[0])  # one context, sized for these blocks
        one = lib.salz_gpu_pool_bytes(0)
        lib.salz_gpu_pool_config(0, one * 3 // 2, -1)  # cap between one workspace and two
        allocs0 = lib.salz_gpu_workspace_allocs()
        outs = [None] * 2

        def work(k):
            for _ in range(5):
                outs[k] = _encode_safe(lib, blocks[k])

        ths = [threading.Thread(target=work, args=(k,)) for k in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        grown = lib.salz_gpu_workspace_allocs() - allocs0
    finally:
        lib.salz_gpu_pool_config(0, 32 << 30, -1)
    assert outs == refs
    # (the second context's first workspace, plus at most one call end that meets its neighbour
    # idle between two calls, which the cap then releases by design; before the r04 fix about one
    # reallocation per call: ~10)
    assert grown <= 2, f"{grown} workspace allocations in 10 concurrent calls"


def test_safe_keeps_caller_device(lib):
    """salz_encode_safe leaves the calling thread's current HIP device as it found it (ADVICE r03:
    the pool may run or create a context elsewhere), also under concurrent calls."""
    hip = ctypes.CDLL("libamdhip64.so")
    ndev = ctypes.c_int(0)
    assert hip.hipGetDeviceCount(ctypes.byref(ndev)) == 0
    blocks = _blocks("text", 300_000, 8)
    bad = []

    def work(dev):
        assert hip.hipSetDevice(dev) == 0
        for b in blocks:
            _encode_safe(lib, b)
            cur = ctypes.c_int(-1)
            hip.hipGetDevice(ctypes.byref(cur))
            if cur.value != dev:
                bad.append((dev, cur.value))

    lib.salz_gpu_pool_config(0, 0, 1)  # borrowing across devices on: the harder case
    try:
        ths = [threading.Thread(target=work, args=(k % ndev.value,)) for k in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    finally:
        lib.salz_gpu_pool_config(0, 0, 0)
    assert bad == []
