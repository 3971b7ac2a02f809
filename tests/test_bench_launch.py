"""bench.py's own multi-rank launch (the sharded loop is programs/salzcli.c:143-179).

`bench.py --gpus N` without an outside launcher starts `torch.distributed.run` with N ranks as a
child process and relays rank 0's line. On the one-GPU box the two-rank run uses
`--dist-backend gloo` (RCCL refuses two ranks on one device), so the same launch, block sharding
and exchange code runs with the payload staged through host memory; its container must be
byte-identical to the one-rank container. `--launch` at N = 1 runs the RCCL (nccl) path at
world 1: RCCL init, the HBM all-gather of the run lengths and the container assembly.
"""
import json
import os
import subprocess
import sys

import pytest

from tests.helpers import ROOT


def _bench(*args, timeout=300):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-e2e", "--no-pmc",
           "--steps", "1", "--warmup", "0", *args]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_gloo_equals_one_rank():
    sharded = ["--workload", "enwik9", "--size", "300000017"]
    two = _bench("--gpus", "2", "--dist-backend", "gloo", *sharded)
    one = _bench("--gpus", "1", *sharded)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["roundtrip_ok"] and two["container_roundtrip_ok"] is True
    assert one["container_roundtrip_ok"] is True
    assert two["container_sha256"] == one["container_sha256"]
    assert two["container_bytes"] == one["container_bytes"]
    assert "gloo" in two["config"]["parallelism"]


@pytest.mark.gpu
def test_bench_world1_through_rccl():
    line = _bench("--gpus", "1", "--launch")
    assert line["n_gpus"] == 1
    assert line["config"]["workload"].startswith("enwik8-sized single block")
    assert line["config"]["input_bytes_total"] == 100_000_000
    assert "RCCL" in line["config"]["parallelism"]
    assert line["roundtrip_ok"] and line["container_roundtrip_ok"] is True


def test_bench_rejects_world_mismatch():
    """An outside launcher whose world differs from --gpus is an error, not a silent N."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29555")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-pmc",
                        "--no-cpu-baseline"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=120, env=env)
    assert p.returncode != 0 and "launcher started 1 ranks" in (p.stderr + p.stdout)


def test_bench_skips_its_pmc_passes_under_a_profiler(monkeypatch):
    """Under an outer rocprofv3 (its library preloaded, ROCPROF_* set) bench.py must not start its
    own rocprofv3 children: the preloaded profiler would initialise the GPU in the nested
    wrapper, which then execs the program."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setenv("ROCPROF_COUNTERS", "FETCH_SIZE")
    traffic, why = bench.measure_traffic(None)
    assert traffic is None and "under rocprofv3" in why
    monkeypatch.delenv("ROCPROF_COUNTERS")
    monkeypatch.setenv("LD_PRELOAD", "/opt/rocm/lib/librocprofiler-sdk-tool.so")
    traffic, why = bench.measure_traffic(None)
    assert traffic is None and "under rocprofv3" in why
