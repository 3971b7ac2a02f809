"""The drop-in boundary seen from C, the reference's own language.

Two kinds of C callers, both built by __graft_entry__.build() against include/salz.h (which
pulls in include/common.h like lib/salz.h:16 does) with the reference's -Werror -pedantic flags:

  tests/c/abi_caller[_static]          our plain C caller of salz_encode_safe / salz_decode_safe,
                                       linked against libsalz.so and against libsalz.a
  oracle/_ref/salzcli_mi355x[_static]  the reference's programs/salzcli.c compiled UNCHANGED
                                       against include/ + libsalz (oracle/Makefile `ref`)

GPU tests: the C callers reproduce the reference's golden hashes through the
header alone, and the reference CLI writes, through our library, exactly the container the
oracle's per-block streams make (BASELINE configs[0]: 1,048,575 bytes of text at the default
level 5; multi-block at level 0), and decodes it back.
CPU tests: the binaries exist, link the product library, and fail loudly without a GPU.
"""
import os
import subprocess

import numpy as np
import pytest

from tests.helpers import ROOT, gen, golden, oracle_encode, sha256

CALLERS = {
    "shared": os.path.join(ROOT, "tests", "c", "abi_caller"),
    "static": os.path.join(ROOT, "tests", "c", "abi_caller_static"),
}
REF_CLI = {
    "shared": os.path.join(ROOT, "oracle", "_ref", "salzcli_mi355x"),
    "static": os.path.join(ROOT, "oracle", "_ref", "salzcli_mi355x_static"),
}
HAVE_REF_CLI = all(os.path.exists(p) for p in REF_CLI.values())


def _run(cmd, **kw):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, **kw)


@pytest.mark.parametrize("link", sorted(CALLERS))
def test_c_caller_links_product_library(link):
    path = CALLERS[link]
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    ldd = _run(["ldd", path]).stdout
    if link == "shared":
        assert "libsalz.so" in ldd
    else:
        assert "libsalz.so" not in ldd and "libamdhip64" in ldd
        syms = _run(["nm", path]).stdout
        assert " T salz_encode_safe" in syms and "oracle_" not in syms


@pytest.mark.skipif(not HAVE_REF_CLI, reason="oracle/_ref not built (needs /root/reference at build time)")
@pytest.mark.parametrize("link", sorted(REF_CLI))
def test_reference_cli_links_product_library(link):
    ldd = _run(["ldd", REF_CLI[link]]).stdout
    assert ("libsalz.so" in ldd) == (link == "shared")
    assert "liboracle" not in ldd


def test_c_caller_fails_loudly_without_gpu():
    """No GPU (this container): salz_encode_safe returns -1 and says why; no CPU fallback."""
    import salz_amd

    if salz_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = _run([CALLERS["shared"], "--errors"])
    assert r.returncode == 1
    assert "no usable HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("link", sorted(CALLERS))
def test_c_caller_error_conventions(link):
    r = _run([CALLERS[link], "--errors"])
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok errors")


@pytest.mark.gpu
@pytest.mark.parametrize("link", sorted(CALLERS))
@pytest.mark.parametrize("vec", [v for v in golden("appendix_c.json")["vectors"] if v["n"] <= 1 << 24],
                         ids=lambda v: f"{v['kind']}{v['n']}-{v['alphabet']}")
def test_c_caller_reproduces_golden_hashes(tmp_path, link, vec):
    src = gen(vec["kind"], vec["n"], vec["seed"], vec["alphabet"])
    assert sha256(src) == vec["in_sha256"]
    fin, fout = tmp_path / "in.bin", tmp_path / "out.salz"
    fin.write_bytes(src.tobytes())
    r = _run([CALLERS[link], str(fin), str(fout)])
    assert r.returncode == 0, r.stderr
    out = fout.read_bytes()
    assert len(out) == vec["out_len"]
    assert sha256(out) == vec["out_sha256"]


def _want_container(src: np.ndarray, block: int) -> bytes:
    want = bytearray(b"ZLAS" + block.to_bytes(4, "little"))
    for off in range(0, len(src), block):
        rc, s = oracle_encode(src[off:off + block])
        assert rc == 0
        want += len(s).to_bytes(4, "little") + s
    return bytes(want)


@pytest.mark.gpu
@pytest.mark.skipif(not HAVE_REF_CLI, reason="oracle/_ref not built (needs /root/reference at build time)")
@pytest.mark.parametrize("link", sorted(REF_CLI))
@pytest.mark.parametrize("level,size", [(5, 1_048_575), (0, 200_003)])
def test_reference_cli_on_product_library(tmp_path, link, level, size):
    """programs/salzcli.c, unchanged, compresses through libsalz (salz_encode_safe per block,
    programs/salzcli.c:143-179) to the container of the oracle's streams, and restores the
    file through salz_decode_safe. Level 5 on 1,048,575 bytes is BASELINE configs[0]."""
    src = gen("text", size, 12)
    f = tmp_path / "doc.txt"
    f.write_bytes(src.tobytes())
    r = _run([REF_CLI[link], f"-{level}", "-k", "-q", str(f)])
    assert r.returncode == 0, r.stderr
    packed = (tmp_path / "doc.txt.salz").read_bytes()
    assert packed == _want_container(src, 1 << (15 + level))
    f.unlink()
    r = _run([REF_CLI[link], "-d", "-q", str(tmp_path / "doc.txt.salz")])
    assert r.returncode == 0, r.stderr
    assert f.read_bytes() == src.tobytes()
