set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03a
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_safe_pool.py tests/test_bench_launch.py "tests/test_dist_split.py::test_split_small_blocks_own_context" "tests/test_gpu_parity.py::test_cli_multi_batch_ring_and_exact_multiple" -s > $out/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -5 $out/pytest.log; cat $out/bench.json
exit $rc
