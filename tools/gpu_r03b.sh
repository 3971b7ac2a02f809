# round 3: the tests after the streaming CLI test, smoke, the default bench and its kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03b}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s "tests/test_gpu_parity.py::test_cli_streams_gigabyte_file_with_bounded_memory" "tests/test_gpu_parity.py::test_cli_multi_batch_ring_and_exact_multiple" tests/test_safe_pool.py > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_prof.json 2> $out/prof.err
rc=$?
grep -E "passed|failed|error|salz_encode_safe" $out/pytest.log | tail -5; cat $out/smoke.log $out/bench.json 2>/dev/null
exit $rc
