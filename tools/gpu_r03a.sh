# round 3: the new tests (pool, launcher, split small blocks, CLI ring, cost wrap), then the bench
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_safe_pool.py tests/test_bench_launch.py "tests/test_dist_split.py::test_split_small_blocks_own_context" "tests/test_gpu_parity.py::test_cli_multi_batch_ring_and_exact_multiple" "tests/test_configs.py::test_int32_cost_wrap_regime" -s > $out/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -5 $out/pytest.log; cat $out/bench.json
exit $rc
