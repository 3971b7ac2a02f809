"""GPU parity: the HIP pipeline against the CPU oracle and the reference's golden vectors.

Every comparison is bit-exact (integer / byte work). Stage arrays are compared one by one
so a mismatch names the stage (SA, PSV/NSV, lengths, decisions, costs, bytes).
"""
import os

import numpy as np
import pytest

from tests.helpers import ROOT, enc_max, gen, golden, oracle_decode, oracle_encode, oracle_stages, sha256

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def salz():
    import salz_amd

    if salz_amd.device_count() == 0:
        pytest.fail("no HIP device visible: GPU tests need an MI355X")
    return salz_amd


@pytest.fixture(scope="module")
def ctx(salz):
    c = salz.Context(0, 1 << 25)
    yield c
    c.close()


def _first_diff(a, b):
    idx = np.nonzero(a != b)[0]
    return int(idx[0]) if len(idx) else -1


def _special(kind, n):
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "period3":
        return np.frombuffer((b"abc" * (n // 3 + 1))[:n], np.uint8).copy()
    if kind == "runs":
        rng = np.random.default_rng(5)
        return np.repeat(rng.integers(0, 3, n // 50 + 1, dtype=np.uint8), 50)[:n].copy()
    if kind == "runs40":  # runs of 40 equal bytes, 64 byte values
        rng = np.random.default_rng(6)
        return np.repeat(rng.integers(0, 64, n // 40 + 1, dtype=np.uint8), 40)[:n].copy()
    if kind == "halves":  # a text repeated once at distance ~n / 2
        return np.resize(gen("text", n // 2 + 1, 11), n)
    if kind == "halves_edit":  # the same with 24 bytes of the copy changed (mismatches on the diagonal)
        src = np.resize(gen("text", n // 2 + 3, 12), n)
        rng = np.random.default_rng(7)
        for p in rng.integers(n // 2 + 3, n, 24):
            src[p] = (int(src[p]) + int(rng.integers(1, 40))) % 95 + 32
        return src
    if kind == "thirds":  # a text repeated twice more (three copies: no twins)
        return np.resize(gen("text", n // 3 + 5, 13), n)
    raise ValueError(kind)


STAGE_CASES = [
    ("fib", 10007, 0, 0),
    ("smx", 20011, 3, 4),
    ("smx", 70000, 9, 2),
    ("smx", 50000, 5, 256),
    ("text", 100003, 1, 0),
    ("mixed", 300000, 2, 0),
    ("zeros", 5000, 0, 0),
    ("period3", 9001, 0, 0),
    ("runs", 40000, 0, 0),
]


def _make(kind, n, seed, alpha):
    if kind in ("zeros", "period3", "runs", "runs40", "halves", "halves_edit", "thirds"):
        return _special(kind, n)
    return gen(kind, n, seed, alpha)


@pytest.mark.parametrize("kind,n,seed,alpha", STAGE_CASES)
def test_stages_match_oracle(ctx, kind, n, seed, alpha):
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    for k in ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"{k} differs at {i}: gpu {d[k][i]} oracle {o[k][i]}"
    i = _first_diff(d["cost"][1:], o["cost"][1:])
    assert i < 0, f"cost differs at {i + 1}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("kind,n,seed,alpha", [("mixed", 3000000, 4, 0), ("text", 1500000, 8, 0)])
def test_scan_launch_shapes(ctx, kind, n, seed, alpha):
    """Scans of 2..1024 tiles, each tile reducing its own carry from the tile totals before it,
    give the oracle's stream."""
    src = _make(kind, n, seed, alpha)
    rc, ref = oracle_encode(src)
    assert rc == 0 and ctx.encode(src) == ref


@pytest.mark.parametrize("vec", [v for v in golden("appendix_c.json")["vectors"] if v["n"] <= 1 << 24],
                         ids=lambda v: f"{v['kind']}{v['n']}-{v['alphabet']}")
def test_appendix_c_golden(ctx, vec):
    src = gen(vec["kind"], vec["n"], vec["seed"], vec["alphabet"])
    assert sha256(src) == vec["in_sha256"]
    out = ctx.encode(src)
    assert len(out) == vec["out_len"]
    assert sha256(out) == vec["out_sha256"]


def test_edge_sizes(ctx, salz):
    rng = np.random.default_rng(11)
    for N in list(range(9, 81)) + [127, 128, 129, 4095, 4096, 4097, 65536 + 9]:
        for kind in ("rand4", "zeros", "rand256"):
            if kind == "rand4":
                src = rng.integers(97, 101, N, dtype=np.uint8)
            elif kind == "zeros":
                src = np.zeros(N, np.uint8)
            else:
                src = rng.integers(0, 256, N, dtype=np.uint8)
            rc, ref = oracle_encode(src)
            out = ctx.encode(src)
            assert rc == 0 and out == ref, (N, kind)


def test_short_blocks_fail_like_reference(ctx, salz):
    for N in range(0, 9):
        with pytest.raises(salz.SalzError):
            ctx.encode(np.zeros(N, np.uint8))


def test_capacity_failure(ctx, salz):
    src = gen("text", 50000, 3)
    rc, ref = oracle_encode(src)
    assert rc == 0
    assert ctx.encode(src, dst_capacity=len(ref)) == ref
    with pytest.raises(salz.SalzError):
        ctx.encode(src, dst_capacity=len(ref) - 1)


def test_encode_safe_default_context_and_roundtrip(salz):
    src = gen("text", 1048575, 7)
    out = salz.encode_safe(src)
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref
    assert salz.decode_safe(out, len(src)) == src.tobytes()
    rc, back = oracle_decode(out, len(src))
    assert rc == 0 and back == src.tobytes()


def test_plain_fallback(ctx):
    src = gen("smx", 300000, 4, 256)
    out = ctx.encode(src)
    assert out[3] == 0 and len(out) == len(src) + 4
    assert out[4:] == src.tobytes()


def test_text_4mib_matches_oracle(ctx):
    src = gen("text", 4 << 20, 3)
    rc, ref = oracle_encode(src)
    assert rc == 0 and ctx.encode(src) == ref


def test_device_resident_api(salz):
    src = gen("text", 2 << 20, 5)
    rc, ref = oracle_encode(src)
    ctx = salz.Context(0, len(src))
    d_src = salz.DeviceBuffer(len(src)).upload(src)
    d_dst = salz.DeviceBuffer(enc_max(len(src)))
    n = ctx.encode_device(d_src.ptr, len(src), d_dst.ptr, d_dst.nbytes)
    assert d_dst.download(n) == ref
    # same context, second block of a different size: workspace reuse is exact
    src2 = gen("fib", 1 << 20)
    d_src.upload(src2)
    n2 = ctx.encode_device(d_src.ptr, len(src2), d_dst.ptr, d_dst.nbytes)
    rc, ref2 = oracle_encode(src2)
    assert d_dst.download(n2) == ref2
    d_src.free()
    d_dst.free()
    ctx.close()


@pytest.fixture
def klog(request, monkeypatch):
    """Force the parse chunk length (2^klog positions per lane) through SALZ_PARSE=klog=N."""
    monkeypatch.setenv("SALZ_PARSE", f"klog={request.param}")
    return request.param


@pytest.mark.parametrize("klog", [6, 7, 8, 9], indirect=True)
@pytest.mark.parametrize("kind,n,seed,alpha", [("text", 300007, 2, 0), ("mixed", 400000, 3, 0),
                                               ("fib", 70001, 0, 0), ("smx", 100000, 1, 4)])
def test_stages_every_chunk_length(ctx, klog, kind, n, seed, alpha):
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    for k in ("dlen", "doff"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"K=2^{klog}: {k} differs at {i}: gpu {d[k][i]} oracle {o[k][i]}"
    i = _first_diff(d["cost"][1:], o["cost"][1:])
    assert i < 0, f"K=2^{klog}: cost differs at {i + 1}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("kind,n", [("text", 12_000_000), ("text", 20_000_000), ("mixed", 24_000_000),
                                    ("mixed", 40_000_017)])
def test_large_blocks_match_oracle(salz, kind, n):
    """Blocks large enough for the default chunk lengths 2^7 / 2^8 (parse_chunk_log); a 12 MB text
    block, which the 8-16 MiB rule moves from K = 2^6 to 2^7; and a mixed block over 32 MiB: more
    than 127 distinct bytes, so it parses with K = 2^7 (pipeline.hip)."""
    src = gen(kind, n, 4)
    rc, ref = oracle_encode(src)
    c = salz.Context(0, n)
    assert rc == 0 and c.encode(src) == ref
    c.close()


@pytest.mark.parametrize("alpha,n", [(2, 16_777_216), (4, 9_000_001)])
def test_large_exit_set_matches_oracle(salz, alpha, n):
    """Short factors in short chunks: the exit set E outgrows the space for every pointer-
    jumping level (|E| ~ 2 M at 16 MiB of a binary alphabet), so the parse keeps level 0
    only and emission recomputes the levels (parse.hip, emit.hip)."""
    src = gen("smx", n, 5, alpha)
    rc, ref = oracle_encode(src)
    c = salz.Context(0, n)
    assert rc == 0 and c.encode(src) == ref
    c.close()


def test_fib_256mib_golden(salz):
    """SURVEY App. C / BASELINE configs[4]: 256 MiB Fibonacci word, one block, against the
    reference's golden output hash (the oracle would take minutes at this size)."""
    vec = next(v for v in golden("appendix_c.json")["vectors"] if v["n"] == 1 << 28)
    src = gen("fib", vec["n"])
    c = salz.Context(0, vec["n"])
    out = c.encode(src)
    c.close()
    assert len(out) == vec["out_len"]
    assert sha256(out) == vec["out_sha256"]
    assert salz.decode_safe(out, len(src)) == src.tobytes()


@pytest.mark.parametrize("block,size", [(1 << 20, 5 * (1 << 20) + 12345), (1 << 16, (1 << 18) + 777)])
def test_encode_blocks_container(salz, block, size):
    """The CLI container (programs/salzcli.c:102-185) from the multi-block queue equals the
    per-block oracle streams framed in block order; decodes back (host threads)."""
    src = gen("mixed", size, 9)
    got = salz.encode_blocks(src, block)
    want = bytearray(b"ZLAS" + block.to_bytes(4, "little"))
    for off in range(0, size, block):
        rc, s = oracle_encode(src[off:off + block])
        assert rc == 0
        want += len(s).to_bytes(4, "little") + s
    assert got == bytes(want)
    assert salz.decode_blocks(got, size) == src.tobytes()


@pytest.mark.parametrize("cap,block,size", [(1 << 20, 1 << 20, 5 * (1 << 20) + 12345),
                                            (1 << 16, 1 << 20, 3 * (1 << 20) + 4097)])
def test_encode_batch_grows_workspace(salz, cap, block, size):
    """A fresh context smaller than the batch grows its workspace so every block, a short last
    one included, gets its own output slot (ensure_batch_room in pipeline.hip); the streams
    equal the per-block oracle's."""
    src = gen("mixed", size, 11)
    c = salz.Context(0, cap)
    got = c.encode_batch(src, block)
    c.close()
    assert len(got) == -(-size // block)
    for k, off in enumerate(range(0, size, block)):
        rc, s = oracle_encode(src[off:off + block])
        assert rc == 0 and got[k] == s, k


@pytest.mark.parametrize("mode", ["global", "segmented"])
@pytest.mark.parametrize("kind,n,seed,alpha", [("text", 600000, 5, 0), ("mixed", 500000, 6, 0),
                                               ("fib", 300000, 0, 0), ("smx", 200000, 2, 2),
                                               ("smx", 150000, 3, 20), ("runs", 120000, 0, 0),
                                               ("zeros", 70000, 0, 0), ("smx", 300000, 4, 100),
                                               ("runs40", 700001, 0, 0), ("smx", 250000, 8, 200)])
def test_suffix_sort_modes(ctx, monkeypatch, mode, kind, n, seed, alpha):
    """Both doubling-round sorts (global radix on (group, rank); LDS sort of small groups +
    extracted large groups; SALZ_SA=global / segmented) give the unique suffix array, with round-0
    keys from the compacted alphabet (texts of <= 127 distinct bytes: 2 to 32 symbols per key,
    round 1 keyed by the text at i + h0) or raw 8-byte keys (more than 127 distinct bytes, round 1
    on ranks); groups of up to 128 members (rank rounds) or 256 (the text round) placed by counting
    and larger ones by LSD passes in LDS; the large groups of a rank round in whole radix tiles
    sorted each on its rank bits, or in one list on (large group, rank) where there is one."""
    monkeypatch.setenv("SALZ_SA", mode)
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    i = _first_diff(d["sa"], o["sa"])
    assert i < 0, f"{mode}: sa differs at rank {i}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


DC3_CASES = STAGE_CASES + [("text", 300001, 4, 0), ("smx", 40000, 7, 200), ("mixed", 200003, 8, 0),
                           ("fib", 65537, 0, 0), ("zeros", 3000, 0, 0)]


@pytest.mark.parametrize("kind,n,seed,alpha", DC3_CASES)
def test_dc3_matches_oracle(ctx, monkeypatch, kind, n, seed, alpha):
    """The DC3 suffix sorter (dc3.hip, forced with SALZ_SA=dc3) gives the unique suffix array on
    every input kind, from the block's byte codes (at most 255 distinct bytes) or raw bytes + 1 (all
    256), with the levels of small triples named from their presence bitmap and the others by
    sorting."""
    monkeypatch.setenv("SALZ_SA", "dc3")
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    assert ctx.stats()["sa_dc3_levels"] > 0
    o = oracle_stages(src)
    i = _first_diff(d["sa"], o["sa"])
    assert i < 0, f"sa differs at rank {i}: gpu {d['sa'][i]} oracle {o['sa'][i]}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("kind,n,seed,alpha", [("fib", 400_000, 0, 0), ("text", 300_001, 4, 0),
                                               ("zeros", 70_000, 0, 0), ("smx", 200_000, 2, 4)])
def test_staged_scatters(ctx, monkeypatch, kind, n, seed, alpha):
    """The staged scatters (scatter.hpp: Phi of the PLCP stage, the DC3 levels' rank and name
    arrays), forced on with SALZ_SA=stage=1 (by default only past 256 MB), give the same
    suffix array, LCPs and stream."""
    monkeypatch.setenv("SALZ_SA", "stage=1,dc3,plcp")
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    for k in ("sa", "lp", "ln"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"{k} differs at {i}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("kind,n", [("fib", 6_000_001), ("period3", 4_000_000), ("runs", 5_000_000),
                                    ("smx4", 3_000_000)])
def test_dc3_large_blocks_match_oracle(ctx, monkeypatch, kind, n):
    """DC3 at a few MB (several levels with staged-size arrays, forced on for the random
    4-letter text) against the CPU port's suffix array and stream."""
    monkeypatch.setenv("SALZ_SA", "dc3")
    src = gen("smx", n, 9, 4) if kind == "smx4" else _make(kind, n, 0, 0)
    out, d = ctx.encode_dump(src)
    assert ctx.stats()["sa_dc3_levels"] > 0
    o = oracle_stages(src)
    i = _first_diff(d["sa"], o["sa"])
    assert i < 0, f"sa differs at rank {i}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


def test_dc3_presence_27bit_level(salz, monkeypatch):
    """A 64 MiB block of runs over all 256 byte values: DC3 level 0 has 9-bit symbols, so its
    triples are 27-bit keys, named from the 2^27-bit presence bitmap (dc3.hip kLutMaxBits; the
    block's radix counts, 512 words a tile, hold the bitmap and its prefix from 2^26 bytes up),
    and the stream equals the oracle's."""
    monkeypatch.setenv("SALZ_SA", "dc3")
    rng = np.random.default_rng(27)
    n = (64 << 20) + 1001
    k = n // 40 + 2
    src = np.repeat(rng.integers(0, 256, k).astype(np.uint8), rng.integers(20, 61, k))[:n]
    assert len(np.unique(src)) == 256
    big = salz.Context(0, n)
    try:
        out = big.encode(src)
        assert big.stats()["sa_dc3_levels"] > 0
    finally:
        big.close()
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


def test_dc3_edge_sizes(ctx, monkeypatch):
    """DC3 at every suffix count 1..200 (each n mod 3, the dummy sample, one-level and
    recursing strings) and around powers of two."""
    monkeypatch.setenv("SALZ_SA", "dc3")
    rng = np.random.default_rng(13)
    sizes = list(range(9, 209)) + [4096 + 8 + d for d in (-1, 0, 1, 2)] + [65536 + 8 + d for d in (0, 1, 2)]
    for N in sizes:
        for kind in ("rand2", "zeros", "rand256"):
            if kind == "rand2":
                src = rng.integers(97, 99, N, dtype=np.uint8)
            elif kind == "zeros":
                src = np.zeros(N, np.uint8)
            else:
                src = rng.integers(0, 256, N, dtype=np.uint8)
            rc, ref = oracle_encode(src)
            out = ctx.encode(src)
            assert rc == 0 and out == ref, (N, kind)


@pytest.mark.parametrize("kind,n,seed", [("text", 6_000_007, 8), ("mixed", 5_000_001, 9)])
def test_ansv_staging_levels(ctx, kind, n, seed):
    """Candidates of blocks past 2^22 positions, staged by text range with the suffix's position
    bits packed into the answer: psv/nsv and their lengths equal the oracle's."""
    src = gen(kind, n, seed)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    for k in ("psv", "nsv", "lp", "ln"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"{k} differs at {i}: gpu {d[k][i]} oracle {o[k][i]}"
    assert out == oracle_encode(src)[1]


def test_suffix_sort_round_checks():
    """SALZ_CHECK=rounds,sa (the suffix sorter's per-round invariants, the text round's keys and
    order included, and the final permutation check) pass, and the streams equal the oracle's;
    the halves blocks run with twin pairs.
    The switch is read once per process, so the encodes run in a child process."""
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import salz_amd\n"
        "from tests.test_gpu_parity import _make\n"
        "from tests.helpers import oracle_encode\n"
        "ctx = salz_amd.Context(0, 1 << 21)\n"
        "for kind, n, seed, alpha in (('text', 600000, 5, 0), ('mixed', 300000, 6, 0), ('smx', 200000, 2, 20),\n"
        "                             ('fib', 100000, 0, 0), ('runs40', 400001, 0, 0), ('mixed', 2000000, 7, 0),\n"
        "                             ('text', 2000000, 9, 0), ('halves', 2000003, 0, 0),\n"
        "                             ('halves_edit', 1500001, 0, 0)):\n"
        "    src = _make(kind, n, seed, alpha)\n"
        "    assert ctx.encode(src) == oracle_encode(src)[1], kind\n"
        "print('round checks ok')\n" % ROOT)
    env = dict(os.environ, SALZ_CHECK="rounds,sa")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0 and "round checks ok" in r.stdout, (r.stdout + r.stderr)[-3000:]


@pytest.mark.parametrize("algo", ["", "doubling"])
def test_dc3_auto_switch(ctx, monkeypatch, algo):
    """A repetitive block of >= 1 MiB goes to DC3 by default, before round 0: when the repetition
    probe finds its evenly spaced 32-gram samples repeated among themselves (Fibonacci, period 3),
    or finds three quarters of them occurring elsewhere in the block by scanning every position
    (runs of 40 equal bytes, a text three times: the samples rarely meet there); a text repeated
    once at distance d (three quarters of the points with one copy at d) stays with doubling and
    splits its twin pairs; text does not go; SALZ_SA=doubling keeps prefix doubling. All give the
    reference stream."""
    monkeypatch.setenv("SALZ_SA", algo)
    for kind, n in (("fib", 3 << 20), ("period3", 2 << 20), ("text", 2 << 20), ("halves", (2 << 20) + 4321),
                    ("runs40", (3 << 20) + 77), ("thirds", (3 << 20) + 11)):
        src = _make(kind, n, 1, 0)
        out = ctx.encode(src)
        rep = kind not in ("text", "halves") and algo != "doubling"
        st = ctx.stats()
        assert (st["sa_dc3_levels"] > 0) == rep, kind
        if rep:  # the probe skips round 0 of doubling
            assert st["sa_rounds"] == 0, (kind, st["sa_rounds"])
        if kind == "halves" and algo == "":  # twin pairs: as many rounds as text (doubling alone: ~18)
            assert 0 < st["sa_rounds"] <= 13, st["sa_rounds"]
        rc, ref = oracle_encode(src)
        assert rc == 0 and out == ref, kind


@pytest.mark.parametrize("lcp_sa", ["", "plcp"])
@pytest.mark.parametrize("kind,n", [("halves", (2 << 20) + 4321), ("halves", (5 << 20) + 6),
                                    ("halves_edit", (3 << 20) + 5)])
def test_twin_pairs_match_oracle(ctx, monkeypatch, lcp_sa, kind, n):
    """Twin pairs (sa.hip k_twin_pairs): two-member groups {x, x + d} ordered and split by the first
    mismatch on diagonal d (the copy running to the end of the block, or edited bytes in it): the
    suffix array, the LCPs from the sort (and from the PLCP stage), the candidates and the stream
    equal the oracle's."""
    monkeypatch.setenv("SALZ_SA", lcp_sa)
    src = _make(kind, n, 0, 0)
    out, d = ctx.encode_dump(src)
    st = ctx.stats()
    assert st["sa_dc3_levels"] == 0 and 0 < st["sa_rounds"] <= 13, st
    o = oracle_stages(src)
    for k in ("sa", "psv", "nsv", "lp", "ln"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"{k} differs at {i}: gpu {d[k][i]} oracle {o[k][i]}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("lcp_sa", ["1", "0"])
@pytest.mark.parametrize("kind,n,seed,alpha", [("text", 400000, 1, 0), ("mixed", 500000, 3, 0),
                                               ("fib", 200000, 0, 0), ("smx", 300000, 2, 4),
                                               ("runs", 150000, 0, 0), ("zeros", 60000, 0, 0),
                                               ("smx", 100000, 5, 256)])
def test_lcp_paths(ctx, monkeypatch, lcp_sa, kind, n, seed, alpha):
    """Both LCP sources give the reference stream: the LCP left behind by the suffix sort
    (sa.hip k_heads_lcp, the default) and the Phi/PLCP stage (lcp.hip, SALZ_SA=plcp)."""
    monkeypatch.setenv("SALZ_SA", "" if lcp_sa == "1" else "plcp")
    src = _make(kind, n, seed, alpha)
    out = ctx.encode(src)
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


@pytest.mark.parametrize("skip", ["1", "0"])
@pytest.mark.parametrize("kind,n,seed,alpha,klog", [("mixed", 3_000_000, 3, 0, "6"),
                                                    ("mixed", 2_000_001, 7, 0, "9"),
                                                    ("text", 1_500_000, 2, 0, "7"),
                                                    ("smx", 1_000_000, 4, 4, "6"),
                                                    ("runs", 400_000, 0, 0, "6")])
def test_parse_wave_skip(ctx, monkeypatch, skip, kind, n, seed, alpha, klog):
    """From the third pass on, waves of chunks whose decisions would repeat skip the pass
    (parse.hip k_parse_mark: the chunk range test, then a wave per listed chunk; lazy per-chunk
    cost offsets; exit set re-packed only in the tiles the walk touched) and without
    (SALZ_PARSE=noskip): decisions, the exact suffix costs and the stream match the oracle."""
    flags = {"0": "noskip"}.get(skip)
    monkeypatch.setenv("SALZ_PARSE", f"klog={klog}" + (f",{flags}" if flags else ""))
    src = _make(kind, n, seed, alpha)
    out, d = ctx.encode_dump(src)
    o = oracle_stages(src)
    for k in ("dlen", "doff"):
        i = _first_diff(d[k], o[k])
        assert i < 0, f"{k} differs at {i}: gpu {d[k][i]} oracle {o[k][i]}"
    i = _first_diff(d["cost"][1:], o["cost"][1:])
    assert i < 0, f"cost differs at {i + 1}"
    rc, ref = oracle_encode(src)
    assert rc == 0 and out == ref


def test_concurrent_contexts_match_oracle(salz):
    """Four contexts encoding at once on one GPU (threads, own streams): every stream must
    equal the CPU port's. Concurrent kernels once exposed a load-ordering hazard in the
    suffix sorter's key kernel ("Concurrent encodes")."""
    import threading

    cases = [gen("text", 1_048_575, 3), gen("mixed", 700_001, 4), gen("fib", 500_000), gen("smx", 400_000, 2, 4)]
    refs = [oracle_encode(c)[1] for c in cases]
    bad = []

    def work(t):
        ctx = salz.Context(0, 1_048_575)
        for it in range(6):
            k = (t + it) % len(cases)
            if ctx.encode(cases[k]) != refs[k]:
                bad.append((t, it, k))
        ctx.close()

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert bad == []


def test_cli_roundtrip_matches_reference_container(salz, tmp_path):
    """salz_amd/salz (programs/salzcli.c mirror): -3 compresses to the reference container
    (blocks of 1 << 18, each the oracle's stream), -d restores the file, -k keeps the input."""
    import subprocess

    cli = os.path.join(ROOT, "salz_amd", "salz")
    src = gen("text", 700_001, 6)
    f = tmp_path / "doc.txt"
    f.write_bytes(src.tobytes())
    subprocess.run([cli, "-3", "-k", "-q", str(f)], check=True, timeout=120)
    packed = (tmp_path / "doc.txt.salz").read_bytes()
    block = 1 << 18
    want = bytearray(b"ZLAS" + block.to_bytes(4, "little"))
    for off in range(0, len(src), block):
        rc, s = oracle_encode(src[off:off + block])
        assert rc == 0
        want += len(s).to_bytes(4, "little") + s
    assert packed == bytes(want)
    f.unlink()
    subprocess.run([cli, "-d", "-q", str(tmp_path / "doc.txt.salz")], check=True, timeout=120)
    assert f.read_bytes() == src.tobytes()


def _run_rss(cmd, timeout=600):
    """Run cmd as the only child of a fresh Python process; returns (rc, peak RSS in MiB)."""
    import subprocess
    import sys

    probe = ("import resource, subprocess, sys; r = subprocess.run(sys.argv[1:]); "
             "print(r.returncode, resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss)")
    out = subprocess.run([sys.executable, "-c", probe, *cmd], capture_output=True, text=True,
                         timeout=timeout, check=True).stdout.split()
    return int(out[-2]), int(out[-1]) / 1024.0


def test_cli_streams_gigabyte_file_with_bounded_memory(salz, tmp_path):
    """The CLI streams (salz_encode_stream / salz_decode_stream, programs/salzcli.c:102-270):
    an enwik9-sized file (10^9 + 7 bytes, level 9 = 16 MiB blocks, 60 blocks) compresses with
    the same peak host RSS as a 9-block file that already fills every encoder slot and the
    block ring (contexts and ring buffers are created as the input needs them) to exactly the
    container salz_encode_blocks makes in memory, whose first and last frames equal the
    oracle's streams, and decompresses back with bounded RSS too."""
    cli = os.path.join(ROOT, "salz_amd", "salz")
    N, block = 1_000_000_007, 16 << 20
    # the reference point: a file just long enough to fill every encoder slot and the whole
    # block ring (contexts and ring buffers are created lazily, so a one-block file uses less)
    small = tmp_path / "small.txt"
    gen("text", 8 * block + 1003, 21).tofile(small)  # (a trailing block of <= 8 bytes fails)
    rc, rss0 = _run_rss([cli, "-9", "-k", "-q", str(small)])
    assert rc == 0
    rc, rss0_d = _run_rss([cli, "-d", "-q", "-f", str(tmp_path / "small.txt.salz")])
    assert rc == 0
    src = gen("text", N, 21)
    f = tmp_path / "big.txt"
    src.tofile(f)
    rc, rss = _run_rss([cli, "-9", "-k", "-q", str(f)])
    assert rc == 0
    assert rss - rss0 < 256, f"peak RSS {rss:.0f} MiB vs {rss0:.0f} MiB for 9 blocks"
    packed = (tmp_path / "big.txt.salz").read_bytes()
    want = salz.encode_blocks(src, block)
    assert packed == want
    pos, frames = 8, []
    while pos < len(packed):
        L = int.from_bytes(packed[pos:pos + 4], "little")
        frames.append((pos + 4, L))
        pos += 4 + L
    assert len(frames) == N // block + 1
    for b in (0, len(frames) - 1):
        o, L = frames[b]
        rc_o, ref = oracle_encode(src[b * block:(b + 1) * block])
        assert rc_o == 0 and packed[o:o + L] == ref
    del want, packed
    f.unlink()
    rc, rss_d = _run_rss([cli, "-d", "-q", str(tmp_path / "big.txt.salz")])
    assert rc == 0 and rss_d - rss0_d < 384, f"decode peak RSS {rss_d:.0f} MiB vs {rss0_d:.0f} MiB"
    back = np.fromfile(f, np.uint8)
    assert back.size == N and np.array_equal(back, src)


def test_cli_multi_batch_ring_and_exact_multiple(salz, tmp_path):
    """The streaming CLI at level 5 (1 MiB blocks, 8 blocks per ring batch): 2 * 8 MiB + 100
    bytes spans three batches and must equal salz_encode_blocks' container; an input of exactly
    16 MiB ends in an empty trailing block, which fails like the reference CLI
    (programs/salzcli.c:143-179, lib/salz.c:197) and leaves no output file (:350-353)."""
    import subprocess

    cli = os.path.join(ROOT, "salz_amd", "salz")
    src = gen("text", 2 * (8 << 20) + 100, 31)
    f = tmp_path / "three.txt"
    src.tofile(f)
    subprocess.run([cli, "-5", "-k", "-q", str(f)], check=True, timeout=300)
    packed = (tmp_path / "three.txt.salz").read_bytes()
    assert packed == salz.encode_blocks(src, 1 << 20)
    rc, ref = oracle_encode(src[(16 << 20):])  # the 100-byte trailing block
    assert rc == 0 and packed.endswith(len(ref).to_bytes(4, "little") + ref)
    g = tmp_path / "exact.txt"
    src[: 16 << 20].tofile(g)
    r = subprocess.run([cli, "-5", "-k", "-q", str(g)], timeout=300)
    assert r.returncode != 0
    assert not (tmp_path / "exact.txt.salz").exists()


@pytest.mark.parametrize("m,bits", [(1, 64), (4095, 17), (4097, 64), (13 * 4096 + 5, 40), (100_003, 63),
                                    (4096 * 4096, 24), (4096 * 4096 + 1, 64), (8192 * 4096 + 3000, 33),
                                    (24576 * 4096 + 4097, 40), (100_003, 9), (200_001, 45),
                                    (24576 * 4096 + 4097, 63)])
@pytest.mark.parametrize("nine", [False, True])
def test_radix_sort_selftest(salz, m, bits, nine):
    """The LSD radix sort (radix.hip) on random keys, and on keys with few distinct values for
    stability: sorted, stable and a permutation of its input, at tile counts that are and are not
    multiples of the 8 XCDs (the scatter's XCD-contiguous tile order) and across the row scan's
    shapes (256-thread rows up to 4096 tiles, 512 up to 8192, 1024 beyond, looping past 24576);
    digit plans of 8-bit passes (the default; 24, 40, 64 bits), 9-bit passes (9, 45, 63 bits: one pass fewer)
    and both (17, 33 bits) with 9-bit digits allowed (the rank rounds' plan)."""
    assert salz.radix_selftest(m, bits, iters=2, seed=7, nine=nine) == 0
