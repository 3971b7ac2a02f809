"""BASELINE.json configs at their full sizes on the GPU, each against the CPU oracle.

  C2  configs[1]: one 100,000,000-byte text block (salz_encode_safe path). Its stream is
      longer than 16 MiB - 1, so the header's 24-bit length field is truncated exactly as the
      reference does (lib/salz.c:760-772); the frame-length rule decodes it.
      Exercises K = 512 parse chunks and the split rank scatter (m >= 32M, sa.hip).
  C4  configs[3]: 64 MiB text blocks through salz_encode_blocks (two full blocks + a tail),
      every frame equal to the oracle's stream of that block (programs/salzcli.c:143-179).
  C3  configs[2]: mixed input in 16 MiB blocks, 4 full blocks + a tail, so that
      salz_encode_blocks runs its 4 concurrent encoder slots on one GPU.
  C5  configs[4] (the 256 MiB Fibonacci word) is pinned by its golden hash in
      test_gpu_parity.py::test_fib_256mib_golden.
Plus a 40 MiB mixed block with the default (size-chosen) parse chunk length.

The oracle needs ~15 s of host CPU for the 100 MB block and ~30 s for all of C4; every test
here fits the 900 s GPU step.
"""
import numpy as np
import pytest

from tests.helpers import gen, oracle_encode

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(scope="module")
def salz():
    import salz_amd

    if salz_amd.device_count() == 0:
        pytest.fail("no HIP device visible: GPU tests need an MI355X")
    return salz_amd


def _hdr(stream: bytes):
    h = int.from_bytes(stream[:4], "little")
    return h >> 24, h & 0xFFFFFF


def _frames(container: bytes):
    assert container[:4] == b"ZLAS"
    pos, out = 8, []
    while pos < len(container):
        L = int.from_bytes(container[pos:pos + 4], "little")
        out.append(container[pos + 4:pos + 4 + L])
        pos += 4 + L
    assert pos == len(container)
    return out


def test_c2_enwik8_block_100mb(salz):
    N = 100_000_000
    src = gen("text", N, 1)
    c = salz.Context(0, N)
    out = c.encode(src)
    c.close()
    rc, ref = oracle_encode(src)
    assert rc == 0
    assert len(out) == len(ref)
    assert out == ref
    typ, field = _hdr(out)
    assert typ == 1 and len(out) - 4 > 0xFFFFFF
    assert field == (len(out) - 4) & 0xFFFFFF  # truncated exactly like the reference
    assert salz.decode_safe(out, N, frame=True) == src.tobytes()


def _blocks_vs_oracle(salz, src: np.ndarray, block: int):
    got = salz.encode_blocks(src, block)
    frames = _frames(got)
    assert len(frames) == len(src) // block + 1
    for b, fr in enumerate(frames):
        rc, ref = oracle_encode(src[b * block:(b + 1) * block])
        assert rc == 0
        assert fr == ref, f"block {b} differs from the oracle"
        typ, field = _hdr(fr)
        assert field == ((len(fr) - 4) & 0xFFFFFF if typ == 1 else min(block, len(src) - b * block) & 0xFFFFFF)
    assert salz.decode_blocks(got, len(src)) == src.tobytes()
    return frames


def test_c4_enwik9_64mib_blocks(salz):
    src = gen("text", 2 * 64 * MiB + 5_000_017, 2)
    frames = _blocks_vs_oracle(salz, src, 64 * MiB)
    assert any(len(f) - 4 > 0xFFFFFF for f in frames[:2])  # the >16 MiB header rule is hit


def test_c3_silesia_16mib_blocks_four_slots(salz):
    src = gen("mixed", 4 * 16 * MiB + 3_000_001, 3)
    _blocks_vs_oracle(salz, src, 16 * MiB)


def test_mixed_40mib_default_chunk_length(salz, monkeypatch):
    monkeypatch.delenv("SALZ_PARSE", raising=False)
    N = 40 * MiB + 3
    assert salz.lib.salz_gpu_parse_chunk_log(N) == 9
    src = gen("mixed", N, 8)
    c = salz.Context(0, N)
    out = c.encode(src)
    c.close()
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("name,n", [("smx256", 1 << 28), ("wrap400", 400_000_000)])
def test_int32_cost_wrap_regime(salz, name, n):
    """Blocks whose parse runs on wrapped int32 costs (9 n > 2^31 - 1; lib/salz.c:621-661 keeps
    the costs in int32 and its factor sums are truncated to int32, SURVEY §7 hard part 5):
    smx256 (256 MiB of splitmix bytes) comes out PLAIN; wrap400 (400 MB, a quarter repeated)
    comes out as a SALZ stream whose cost from position 0 is ~2.7e9 bits, so the first fifth of
    its parse decides on wrapped costs. Both must equal the oracle's bytes, pinned as golden
    hashes by tools/make_wrap_golden.py (the oracle takes 2-4 minutes per input), and decode
    back through the frame-length rule."""
    import hashlib
    import json
    import os

    from tests.helpers import GOLDEN_DIR, wrap_input

    vec = {v["name"]: v for v in json.load(open(os.path.join(GOLDEN_DIR, "cost_wrap.json")))["vectors"]}[name]
    src = wrap_input(name, n)
    assert hashlib.sha256(src.tobytes()).hexdigest() == vec["in_sha256"]
    out = salz.encode_safe(src)
    assert len(out) == vec["out_len"]
    h = int.from_bytes(out[:4], "little")
    assert (h >> 24, h & 0xFFFFFF) == (vec["out_type"], vec["out_hdr_len"])
    assert hashlib.sha256(out).hexdigest() == vec["out_sha256"]
    assert salz.decode_safe(out, n, frame=True) == src.tobytes()
