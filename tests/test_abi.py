"""CPU tests of the drop-in boundary: libsalz.so loads, exports every symbol the public headers
declare, its host-side pieces (vnibble helpers, decoder, container decode) agree with the oracle,
and encoding fails loudly when no GPU is present (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests.helpers import ROOT, gen, oracle, oracle_encode


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"typedef\s+struct[^{;]*\{.*?\}\s*\w+\s*;", "", txt, flags=re.S)  # struct members
    txt = re.sub(r"typedef[^;]*;", "", txt)  # function-pointer typedefs are not exports
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", txt)
    return sorted(set(n for n in names if n not in ("if", "return", "sizeof")))


def test_headers_declare_reference_api():
    assert set(_declared("salz.h")) >= {"salz_encode_safe", "salz_decode_safe", "encode_vnibble_le",
                                        "vnibble_size"}
    txt = open(os.path.join(ROOT, "include", "salz.h")).read()
    assert "static inline int salz_encoded_len_max(size_t plain_len)" in txt


@pytest.mark.parametrize("header", ["salz.h", "salz_gpu.h"])
def test_library_exports_declared_symbols(header):
    import salz_amd

    for name in _declared(header):
        assert hasattr(salz_amd.lib, name), f"libsalz.so does not export {name}"


def test_no_torch_or_oracle_in_product_library():
    import subprocess

    out = subprocess.run(["ldd", os.path.join(ROOT, "salz_amd", "libsalz.so")], capture_output=True,
                         text=True).stdout
    assert "oracle" not in out and "torch" not in out
    syms = subprocess.run(["nm", "-D", os.path.join(ROOT, "salz_amd", "libsalz.so")],
                          capture_output=True, text=True).stdout
    assert "oracle_" not in syms


def test_encoded_len_max_formula():
    import salz_amd

    for n in [0, 1, 8, 9, 63, 64, 65, 1048575, 1 << 24, 100_000_000]:
        assert salz_amd.encoded_len_max(n) == 4 + n + ((n + 63) // 64 * 64) // 8


def test_vnibble_closed_form_matches_reference_restatement():
    """encode_vnibble_le / vnibble_size (lib/salz.c:352-445, :565-588): the product's
    closed form equals the oracle's byte-packing restatement (low 4k bits), and like the
    reference it stores only the ceil(k / 2) bytes that hold the nibbles (:354-444): the bytes
    of *res beyond them keep what the caller had there."""
    import salz_amd

    o = oracle()
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    rng = np.random.default_rng(1)
    vals = list(range(0, 70000)) + [int(x) for x in rng.integers(0, 2**32, 20000, dtype=np.uint64)]
    vals += [8, 72, 584, 4680, 37448, 299592, 2396744, 19173960, 153391688, 1227133512]
    vals += [v - 1 for v in vals[-10:]] + [0xFFFFFFFF]
    fill = 0xA5A5A5A5A5A5A5A5
    for v in vals:
        a.value = fill
        k1 = salz_amd.lib.encode_vnibble_le(v, ctypes.byref(a))
        nb = (k1 + 1) // 2
        assert a.value >> (8 * nb) == fill >> (8 * nb), v
        k2 = o.oracle_encode_vnibble_le(v, ctypes.byref(b))
        assert k1 == k2 == salz_amd.lib.vnibble_size(v) == o.oracle_vnibble_size(v)
        m = (1 << (4 * k1)) - 1
        assert a.value & m == b.value & m, v


@pytest.mark.parametrize("kind,n,alpha", [("text", 400000, 256), ("fib", 100000, 0), ("smx", 50000, 4),
                                         ("smx", 30000, 256), ("mixed", 600000, 256)])
def test_product_decoder_on_reference_streams(kind, n, alpha):
    import salz_amd

    src = gen(kind, n, 5, alpha)
    rc, stream = oracle_encode(src)
    assert rc == 0
    assert salz_amd.decode_safe(stream, n) == src.tobytes()
    assert salz_amd.decode_safe(stream, n, frame=True) == src.tobytes()
    with pytest.raises(salz_amd.SalzError):
        salz_amd.decode_safe(stream, n - 1)
    with pytest.raises(salz_amd.SalzError):
        salz_amd.decode_safe(stream[:-3], n)


def test_decoder_rejects_bad_headers():
    import salz_amd

    for bad in [b"", b"\x00\x00", b"\x05\x00\x00\x02abcde", b"\x10\x00\x00\x01\x00"]:
        with pytest.raises(salz_amd.SalzError):
            salz_amd.decode_safe(bad, 100)


def test_frame_rule_for_truncated_header():
    """> 16 MiB streams: header length field is (len & 0xffffff) (lib/salz.c:770); the frame
    decoder recovers it from the container length. Simulated with a PLAIN stream."""
    import salz_amd

    n = (1 << 24) + 1000
    body = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8).tobytes()
    hdr = (0 << 24) | (n & 0xFFFFFF)
    stream = hdr.to_bytes(4, "little") + body
    # like the reference, the plain decoder trusts the truncated field (1000 bytes)
    assert salz_amd.decode_safe(stream, n) == body[:1000]
    assert salz_amd.decode_safe(stream, n, frame=True) == body


def test_container_decode_matches_reference_cli_layout():
    import salz_amd

    src = gen("text", 3 * 65536 + 777, 9)
    bs = 65536
    frames = []
    for off in range(0, len(src) + 1, bs):
        blk = src[off:off + bs]
        if len(blk) == 0:
            break
        rc, s = oracle_encode(blk)
        assert rc == 0
        frames.append(len(s).to_bytes(4, "little") + s)
    cont = (0x53414C5A).to_bytes(4, "little") + bs.to_bytes(4, "little") + b"".join(frames)
    assert salz_amd.decode_blocks(cont, len(src), threads=3) == src.tobytes()


def test_encode_fails_loudly_without_gpu():
    import salz_amd

    if salz_amd.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(salz_amd.SalzError, match="no usable HIP device"):
        salz_amd.encode_safe(gen("text", 10000, 1))


def test_parse_chunk_log_boundaries(monkeypatch):
    """Parse chunk length K = 2^klog per block length (parse.hip parse_chunk_log): more than
    2^17 chunks up to 32 MiB, more than 2^16 above. Pins the boundaries the bench configs sit
    on (C1/C3: K = 64, C2/C4/C5: K = 512) and the 32 MiB edge."""
    import salz_amd

    monkeypatch.delenv("SALZ_PARSE", raising=False)
    f = salz_amd.lib.salz_gpu_parse_chunk_log
    MiB = 1 << 20
    want = {9: 6, 1 * MiB - 1: 6, 16 * MiB: 6, 16 * MiB + 1: 6, 24_000_000: 7, 32 * MiB: 7,
            32 * MiB + 8: 8, 40 * MiB: 9, 64 * MiB: 9, 100_000_000: 9, 256 * MiB: 9}
    for N, k in want.items():
        assert f(N) == k, (N, f(N), k)
    monkeypatch.setenv("SALZ_PARSE", "klog=8")
    assert f(16 * MiB) == 8


@pytest.mark.parametrize("size,block", [(100, 1000), (9, 9), (15, 15), (5000, 512), (512 * 7 + 9, 512),
                                        (512 * 3 + 15, 512), (512 * 4 + 100, 512), (32768 * 5 + 300, 32768)])
def test_batch_round0_order(size, block):
    """Round 0 of a batch (common.hpp init_suffix): every live suffix exactly once (dead
    positions: the 8 bytes after each block's suffix text), the suffixes with fewer than 8
    bytes left first, shortest first within each block, then the rest in text order."""
    import salz_amd

    nb = 1 if block >= size else -(-size // block)
    out = np.zeros(size, np.uint32)
    m = salz_amd.lib.salz_debug_init_order(size, block, out.ctypes.data)
    order = out[:m].tolist()
    starts = [b * block for b in range(nb)]
    ends = [min(s + block, size) - 8 for s in starts] if nb > 1 else [size - 8]
    live = sorted(p for s, e in zip(starts, ends) for p in range(s, e))
    assert sorted(order) == live and m == len(live)
    blk = (lambda p: 0) if nb == 1 else (lambda p: p // block)
    left = [ends[blk(p)] - p for p in order]
    nshort = sum(1 for x in left if x < 8)
    assert all(x < 8 for x in left[:nshort]) and all(x >= 8 for x in left[nshort:])
    for b in range(nb):  # shortest first within a block
        mine = [x for p, x in zip(order[:nshort], left[:nshort]) if blk(p) == b]
        assert mine == sorted(mine)
    assert order[nshort:] == sorted(order[nshort:])
