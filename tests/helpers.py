"""Shared test helpers: the CPU oracle (test infrastructure), the data generators and the
golden vectors. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
the oracle."""
from __future__ import annotations

import ctypes
import hashlib
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")

_oracle = None
_datagen = None


def oracle() -> ctypes.CDLL:
    global _oracle
    if _oracle is None:
        path = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.oracle_encode.argtypes = [vp, sz, vp, ctypes.POINTER(sz)]
        lib.oracle_decode.argtypes = [vp, sz, vp, ctypes.POINTER(sz)]
        lib.oracle_stages.argtypes = [vp, sz] + [vp] * 8
        lib.oracle_suffix_array.argtypes = [vp, vp, ctypes.c_int32]
        lib.oracle_encode_vnibble_le.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
        lib.oracle_encode_vnibble_le.restype = sz
        lib.oracle_vnibble_size.argtypes = [ctypes.c_uint32]
        lib.oracle_vnibble_size.restype = sz
        _oracle = lib
    return _oracle


def datagen() -> ctypes.CDLL:
    global _datagen
    if _datagen is None:
        path = os.path.join(ROOT, "tools", "libdatagen.so")
        if not os.path.exists(path):
            raise RuntimeError("tools/libdatagen.so missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.datagen_fib.argtypes = [vp, sz]
        lib.datagen_smx.argtypes = [vp, sz, ctypes.c_uint64, ctypes.c_uint32]
        lib.datagen_text.argtypes = [vp, sz, ctypes.c_uint64]
        lib.datagen_mixed.argtypes = [vp, sz, ctypes.c_uint64]
        _datagen = lib
    return _datagen


def gen(kind: str, n: int, seed: int = 1, alphabet: int = 256) -> np.ndarray:
    """fib | smx | text | mixed, deterministic (tools/datagen.c)."""
    b = np.zeros(max(n, 1), np.uint8)
    p = b.ctypes.data
    g = datagen()
    if kind == "fib":
        g.datagen_fib(p, n)
    elif kind == "smx":
        g.datagen_smx(p, n, seed, alphabet)
    elif kind == "text":
        g.datagen_text(p, n, seed)
    elif kind == "mixed":
        g.datagen_mixed(p, n, seed)
    else:
        raise ValueError(kind)
    return b[:n]


def enc_max(n: int) -> int:
    return 4 + n + ((n + 63) // 64 * 64) // 8


def oracle_encode(src: np.ndarray, cap: int | None = None):
    s = np.ascontiguousarray(src, dtype=np.uint8)
    cap = enc_max(len(s)) if cap is None else cap
    out = np.zeros(max(cap, 1), np.uint8)
    n = ctypes.c_size_t(cap)
    rc = oracle().oracle_encode(s.ctypes.data if len(s) else None, len(s), out.ctypes.data,
                                ctypes.byref(n))
    return rc, out[: n.value].tobytes() if rc == 0 else None


def oracle_decode(src: bytes, cap: int):
    s = np.frombuffer(src, np.uint8)
    out = np.zeros(max(cap, 1), np.uint8)
    n = ctypes.c_size_t(cap)
    rc = oracle().oracle_decode(s.ctypes.data, len(s), out.ctypes.data, ctypes.byref(n))
    return rc, out[: n.value].tobytes() if rc == 0 else None


def oracle_stages(src: np.ndarray) -> dict:
    s = np.ascontiguousarray(src, dtype=np.uint8)
    n = len(s) - 8
    arrs = {k: np.zeros(n + (1 if k == "cost" else 0), np.int32)
            for k in ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff", "cost")}
    rc = oracle().oracle_stages(s.ctypes.data, len(s),
                                *[arrs[k].ctypes.data for k in
                                  ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff", "cost")])
    assert rc == 0
    return arrs


def sha256(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def golden(name: str):
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return json.load(f)


def wrap_input(name: str, n: int) -> np.ndarray:
    """Inputs of the int32 cost-wrap regime (tools/make_wrap_golden.py): "smx256" = splitmix64
    bytes (seed 5); "wrap400" = the same bytes with the last 4 MiB of every 16 MiB replaced by a
    copy of an earlier 4 MiB run at a seeded offset."""
    src = gen("smx", n, 5, 256).copy()
    if name == "smx256":
        return src
    assert name == "wrap400"
    rng = np.random.default_rng(5)
    seg, rep = 16 << 20, 4 << 20
    for b in range(seg, n + 1, seg):
        lo = b - rep
        s = int(rng.integers(0, lo - rep))
        src[lo:b] = src[s:s + rep]
    return src
