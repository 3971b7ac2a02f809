"""One block's suffix array split over several ranks (dsa.hip,
salz_amd.dist.encode_block_split): each rank sorts its two-byte-prefix bucket on the GPU and
exchanges rank requests per doubling round; rank 0 gathers the pieces and encodes. The stream
must equal the CPU port's. The ranks run gloo with host-staged buffers, all on the box's one
GPU (RCCL refuses two ranks on one device); the library's own RCCL communicator runs at one rank."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.helpers import ROOT, gen, oracle_encode

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs():
    rng = np.random.default_rng(3)
    return {
        "text": gen("text", 2_000_003, 5),
        "mixed": gen("mixed", 1_500_000, 6),
        "fib": gen("fib", 1_048_575),  # long repeats: LCPs from the PLCP stage
        "small": gen("text", 1000, 2),
        "zeros": np.zeros(50_000, np.uint8),  # one class: every other bucket is empty
        "rand": rng.integers(0, 256, 100_000, dtype=np.uint8),  # PLAIN
        "smx4": gen("smx", 300_000, 2, 4),
    }


def _rep_inputs():
    """Blocks of 2^20 suffixes or more that the repetition probe sends to DC3: not split."""
    runs = np.repeat(np.random.default_rng(5).integers(0, 3, (3 << 20) // 50 + 1, dtype=np.uint8), 50)[:3 << 20]
    return {"fib3m": gen("fib", 3 << 20), "runs3m": runs.copy()}


def _run_split(tmp_path, world, inputs, *extra, sa_env=""):
    src = tmp_path / "in.npz"
    out = tmp_path / "out.npz"
    np.savez(src, **inputs)
    port = _port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", SALZ_SA=sa_env)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "split_worker.py"), str(r), str(world),
                               str(port), str(src), str(out), *extra], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("split workers timed out")
        logs.append(o.decode(errors="replace"))
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    got = np.load(out)
    for k, s in inputs.items():
        rc, ref = oracle_encode(s)
        assert rc == 0
        assert got[k].tobytes() == ref, k
    import ast

    return {k: (split, lv) for k, split, lv in ast.literal_eval(str(got["__info__"]))}


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_suffix_array_matches_oracle(tmp_path, world):
    """World 1 reads rank[i + h] locally (no collective); the others exchange requests every
    doubling round but round 1 of text blocks, which is keyed by the text every rank holds."""
    info = _run_split(tmp_path, world, _inputs())
    assert all(split for split, _ in info.values()), info


@pytest.mark.parametrize("world", [1, 2, 3])
def test_split_repetitive_blocks_encode_whole(tmp_path, world):
    """A 3 MiB Fibonacci block and runs of 50 equal bytes (the repetition probe's DC3 blocks) are
    not split into ~log2(max LCP) exchanged doubling rounds: every rank takes the probe's decision
    and rank 0 encodes the block whole with DC3; the streams equal the CPU
    port's."""
    info = _run_split(tmp_path, world, _rep_inputs())
    for k, (split, levels) in info.items():
        assert not split and levels > 0, (k, split, levels)


@pytest.mark.parametrize("world,sa_env", [(1, "xchg"), (3, "xchg")])
def test_split_exchange_variants(tmp_path, world, sa_env):
    """The exchange forced at one rank (SALZ_SA=xchg: requests to itself through the collectives)
    and at three (where it runs anyway; round 1 of the mixed block is on ranks, one exchange more
    than the text blocks', so the idle ranks' sequences differ by block)."""
    _run_split(tmp_path, world, _inputs(), sa_env=sa_env)


@pytest.mark.parametrize("sa_env", ["", "xchg"])
def test_split_rccl_comm_one_rank(tmp_path, sa_env):
    """The library's own RCCL communicator (salz_gpu_dist_comm: nccl backend, one rank on the
    box's GPU): the collectives run inside the library, forced through the exchange with xchg."""
    _run_split(tmp_path, 1, _inputs(), "nccl", sa_env=sa_env)


def test_split_small_blocks_own_context(tmp_path):
    """Blocks under 32 KiB, each with a context sized to it: the 65536-class histogram must not
    live in a per-slot array (it overran ws.u0 for such contexts)."""
    inputs = {"t20k": gen("text", 20_000, 7), "t32775": gen("text", 32_775, 8), "m1k": gen("mixed", 1_000, 9),
              "fib5k": gen("fib", 5_000)}
    _run_split(tmp_path, 2, inputs, "perblock")
