"""CPU tests: the oracle (test infrastructure) against the reference's golden vectors, plus
structural properties of each stage. No GPU needed."""
import ctypes
import json
import os

import numpy as np
import pytest

from tests.helpers import enc_max, gen, golden, oracle, oracle_decode, oracle_encode, oracle_stages, sha256


VECTORS = golden("appendix_c.json")["vectors"]


@pytest.mark.parametrize("vec", [v for v in VECTORS if v["n"] <= 1 << 24],
                         ids=lambda v: f"{v['kind']}{v['n']}-{v['alphabet']}")
def test_oracle_matches_reference_golden(vec):
    src = gen(vec["kind"], vec["n"], vec["seed"], vec["alphabet"])
    assert sha256(src) == vec["in_sha256"], "generator drifted from Appendix C"
    rc, out = oracle_encode(src)
    assert rc == 0
    assert len(out) == vec["out_len"]
    assert sha256(out) == vec["out_sha256"]


@pytest.mark.slow
def test_oracle_fib_256mib_golden():
    vec = [v for v in VECTORS if v["n"] == 268435456][0]
    src = gen("fib", vec["n"])
    rc, out = oracle_encode(src)
    assert rc == 0 and sha256(out) == vec["out_sha256"]


def _naive_sa(t: bytes):
    return sorted(range(len(t)), key=lambda i: t[i:])


@pytest.mark.parametrize("seed", range(40))
def test_oracle_sais_matches_naive(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 300))
    alpha = int(rng.choice([1, 2, 3, 4, 256]))
    t = rng.integers(0, alpha, n, dtype=np.uint8)
    if seed % 5 == 0:
        t = np.tile(t[: max(1, n // 7)], 8)[:n].copy()
    sa = np.zeros(len(t), np.int32)
    assert oracle().oracle_suffix_array(t.ctypes.data, sa.ctypes.data, len(t)) == 0
    assert list(sa) == _naive_sa(t.tobytes())


def test_oracle_stages_properties():
    src = gen("text", 200000, 4)
    n = len(src) - 8
    st = oracle_stages(src)
    t = src[:n].tobytes()
    # PSV/NSV are nearest smaller positions in rank order (lib/salz.c:471-490)
    rank = np.empty(n, np.int64)
    rank[st["sa"]] = np.arange(n)
    rng = np.random.default_rng(0)
    for p in rng.integers(1, n, 300):
        r = rank[p]
        left = [st["sa"][q] for q in range(r - 1, -1, -1) if st["sa"][q] < p][:1]
        right = [st["sa"][q] for q in range(r + 1, n) if st["sa"][q] < p][:1]
        assert st["psv"][p] == (left[0] if left else -1)
        assert st["nsv"][p] == (right[0] if right else -1)

        def lcp(a, b):
            k = 0
            while b + k < n and t[a + k] == t[b + k]:
                k += 1
            return k

        if st["psv"][p] >= 0:
            assert st["lp"][p] == lcp(st["psv"][p], p)
        if st["nsv"][p] >= 0:
            assert st["ln"][p] == lcp(st["nsv"][p], p)
    # the parse path covers [0, n) with valid tokens
    p = 0
    while p < n:
        assert st["dlen"][p] == 1 or st["dlen"][p] >= 3
        p += st["dlen"][p]
    assert p == n


@pytest.mark.parametrize("kind,n", [("text", 300000), ("fib", 65536), ("smx", 100000), ("mixed", 500000)])
def test_oracle_roundtrip(kind, n):
    src = gen(kind, n, 3, 4)
    rc, out = oracle_encode(src)
    assert rc == 0
    rc, back = oracle_decode(out, n)
    assert rc == 0 and back == src.tobytes()


def test_oracle_short_blocks_fail():
    for N in range(0, 9):
        rc, _ = oracle_encode(np.zeros(N, np.uint8), cap=enc_max(max(N, 1)) + 8)
        assert rc == -1


def test_oracle_capacity_semantics():
    src = gen("text", 40000, 2)
    rc, ref = oracle_encode(src)
    assert rc == 0
    rc2, out = oracle_encode(src, cap=len(ref))
    assert rc2 == 0 and out == ref
    rc3, _ = oracle_encode(src, cap=len(ref) - 1)
    assert rc3 == -1


def test_vnibble_restatement_small_exhaustive():
    o = oracle()
    x = ctypes.c_uint64()
    prev_k = 1
    for v in list(range(0, 5000)) + [37447, 37448, 299591, 299592, 2396743, 2396744, 19173959,
                                     19173960, 153391687, 153391688, 1227133511, 1227133512,
                                     0xFFFFFFFF]:
        k = o.oracle_encode_vnibble_le(v, ctypes.byref(x))
        assert k == o.oracle_vnibble_size(v)
        assert k >= prev_k or v < 5000
        low = x.value & ((1 << (4 * k)) - 1)
        assert low & 0x8, "terminator bit on the last nibble"
        for j in range(1, k):
            assert not (low >> (4 * j)) & 0x8
        prev_k = k


@pytest.mark.slow
@pytest.mark.skipif(not os.environ.get("SALZ_SLOW"), reason="2-4 min of oracle each: set SALZ_SLOW=1")
@pytest.mark.parametrize("name,n", [("smx256", 1 << 28), ("wrap400", 400_000_000)])
def test_oracle_cost_wrap_golden(name, n):
    """The cost-wrap golden vectors (tools/make_wrap_golden.py) against a fresh oracle run:
    2-4 minutes each (SALZ_SLOW=1); the GPU side checks the same hashes every round."""
    import hashlib

    from tests.helpers import GOLDEN_DIR, wrap_input

    vec = {v["name"]: v for v in json.load(open(os.path.join(GOLDEN_DIR, "cost_wrap.json")))["vectors"]}[name]
    src = wrap_input(name, n)
    assert hashlib.sha256(src.tobytes()).hexdigest() == vec["in_sha256"]
    rc, out = oracle_encode(src)
    assert rc == 0 and hashlib.sha256(out).hexdigest() == vec["out_sha256"]


def test_cost_wrap_inputs_are_in_the_wrap_regime():
    """wrap400's stream (342 MB) means a parse cost from position 0 above 2^31 - 1 bits."""
    from tests.helpers import GOLDEN_DIR

    vec = {v["name"]: v for v in json.load(open(os.path.join(GOLDEN_DIR, "cost_wrap.json")))["vectors"]}
    assert vec["wrap400"]["out_type"] == 1 and 8 * (vec["wrap400"]["out_len"] - 4) > 2**31
    assert 9 * (vec["smx256"]["n"] - 8) > 2**31 and vec["smx256"]["out_type"] == 0
