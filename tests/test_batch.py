"""Batches: several independent blocks encoded by ONE pass of the GPU pipeline
(salz_gpu_encode_batch; the container encoders salz_encode_blocks / salz_encode_stream use it
for block sizes that are multiples of 512).

Every block's stream must equal the oracle's stream of that block alone (lib/salz.c:777-823 on
the block), whatever shares the batch with it: the suffix sort keys carry the block, candidates
never cross a block, the parse restarts at each block and emission writes one stream per block.
Cases cover ragged last blocks (down to 9 bytes), PLAIN blocks next to compressible ones, long
repeats (the Phi/PLCP path), both doubling-round sorts, every parse chunk length, and batches
of hundreds of blocks.
"""
import numpy as np
import pytest

from tests.helpers import enc_max, gen, oracle_encode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def salz():
    import salz_amd

    if salz_amd.device_count() == 0:
        pytest.fail("no HIP device visible: GPU tests need an MI355X")
    return salz_amd


@pytest.fixture(scope="module")
def ctx(salz):
    c = salz.Context(0, 8 << 20)
    yield c
    c.close()


def _src(kind, n, seed):
    if kind == "patch":  # text, random bytes (PLAIN blocks) and runs, side by side
        rng = np.random.default_rng(seed)
        parts, size = [], 0
        while size < n:
            k = int(rng.integers(0, 3))
            m = int(rng.integers(500, 20000))
            if k == 0:
                parts.append(gen("text", m, seed + size))
            elif k == 1:
                parts.append(rng.integers(0, 256, m, dtype=np.uint8))
            else:
                parts.append(np.full(m, rng.integers(0, 256), np.uint8))
            size += m
        return np.concatenate(parts)[:n].copy()
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "smx4":
        return gen("smx", n, seed, 4)
    return gen(kind, n, seed)


def _check(ctx, src, block):
    """Every stream equals the oracle's for its block with the reference CLI's output capacity
    salz_encoded_len_max(block) (programs/salzcli.c:130); if the oracle fails a block at that
    capacity (an incompressible block whose SALZ form runs past it before the PLAIN fallback),
    the batch must fail too."""
    import salz_amd

    nb = max(1, -(-len(src) // block))
    refs = [oracle_encode(src[b * block:(b + 1) * block], enc_max(block)) for b in range(nb)]
    if any(rc != 0 for rc, _ in refs):
        with pytest.raises(salz_amd.SalzError):
            ctx.encode_batch(src, block)
        return
    streams = ctx.encode_batch(src, block)
    assert len(streams) == nb
    for b, (s, (rc, ref)) in enumerate(zip(streams, refs)):
        assert s == ref, f"block {b} of {nb} ({len(src[b * block:(b + 1) * block])} bytes) differs"


@pytest.mark.parametrize("kind,size,block", [
    ("text", 512 * 9 + 100, 512),
    ("text", 4096 * 20 + 9, 4096),          # 9-byte last block
    ("text", 4096 * 20 + 15, 4096),         # last block with 7 suffixes
    ("mixed", 32768 * 40 + 12345, 32768),
    ("fib", 65536 * 6 + 777, 65536),        # long repeats: Phi / PLCP path
    ("smx4", 16384 * 30 + 999, 16384),
    ("zeros", 8192 * 12 + 33, 8192),
    ("patch", 4096 * 64 + 300, 4096),       # PLAIN blocks among compressible ones
    ("text", 512 * 700 + 50, 512),          # 701 blocks in one batch
    ("mixed", (1 << 20) * 3 + 4097, 1 << 20),
    ("text", 3000, 1 << 20),                # one block (batch of 1)
])
def test_batch_matches_per_block_oracle(ctx, kind, size, block):
    _check(ctx, _src(kind, size, 3), block)


@pytest.mark.parametrize("env", [("SALZ_SA", "plcp"), ("SALZ_SA", "global"), ("SALZ_SA", "segmented"),
                                 ("SALZ_PARSE", "klog=6"), ("SALZ_PARSE", "klog=9"),
                                 ("SALZ_PARSE", "noskip")])
@pytest.mark.parametrize("kind,size,block", [("mixed", 16384 * 25 + 4321, 16384),
                                             ("patch", 8192 * 30 + 100, 8192)])
def test_batch_equivalent_paths(ctx, monkeypatch, env, kind, size, block):
    monkeypatch.setenv(*env)
    _check(ctx, _src(kind, size, 5), block)


def test_batch_plain_blocks(ctx):
    """Incompressible blocks fall back to PLAIN (lib/salz.c:755-767) next to compressible ones
    in the same batch."""
    rnd = np.random.default_rng(1).integers(0, 256, 4096, dtype=np.uint8)
    parts = [gen("text", 4096, 1), rnd, gen("text", 4096, 2), np.zeros(4096, np.uint8), rnd,
             gen("mixed", 1000, 3)]
    src = np.concatenate(parts)
    streams = ctx.encode_batch(src, 4096)
    for b, s in enumerate(streams):
        rc, ref = oracle_encode(src[b * 4096:(b + 1) * 4096], enc_max(4096))
        assert rc == 0 and s == ref
    assert [s[3] for s in streams] == [1, 0, 1, 1, 0, 1]  # header types: SALZ / PLAIN


def test_batch_rejects_short_last_block(ctx, salz):
    """A last block of 1..8 bytes fails, as the reference does for such a block; through the
    container encoders an exact multiple of the block size fails too (the reference CLI always
    encodes the trailing fread() chunk, here empty, programs/salzcli.c:143-179)."""
    for tail in (1, 8):
        with pytest.raises(salz.SalzError):
            ctx.encode_batch(gen("text", 4096 * 3 + tail, 1), 4096)
    assert len(ctx.encode_batch(gen("text", 4096 * 3, 1), 4096)) == 3
    for tail in (0, 5):
        with pytest.raises(salz.SalzError):
            salz.encode_blocks(gen("text", 4096 * 3 + tail, 1), 4096)


@pytest.mark.parametrize("batch_bytes", ["65536", "1048576"])
def test_encode_blocks_batched_container(salz, monkeypatch, batch_bytes):
    """salz_encode_blocks in batches (SALZ_BATCH_BYTES sets the batch size) gives the container
    of the per-block oracle streams, several batches per call."""
    monkeypatch.setenv("SALZ_BATCH_BYTES", batch_bytes)
    src = _src("patch", 32768 * 50 + 1234, 7)
    block = 32768
    got = salz.encode_blocks(src, block)
    want = bytearray(b"ZLAS" + block.to_bytes(4, "little"))
    for off in range(0, len(src), block):
        rc, s = oracle_encode(src[off:off + block])
        assert rc == 0
        want += len(s).to_bytes(4, "little") + s
    assert got == bytes(want)
