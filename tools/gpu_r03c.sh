# round 3: suffix-sort parity (pair finishing), the pending tests, bench + per-round trace + kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03c}
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "suffix_sort_modes or stages_match or appendix_c or lcp_paths or edge_sizes or large_blocks or staged_scatters" > $out/pytest_sa.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_batch.py tests/test_dist_split.py tests/test_safe_pool.py "tests/test_gpu_parity.py::test_cli_streams_gigabyte_file_with_bounded_memory" "tests/test_gpu_parity.py::test_cli_multi_batch_ring_and_exact_multiple" tests/test_configs.py > $out/pytest.log 2>&1 &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 2 --warmup 1 > $out/text_sa.json 2> $out/text_sa.log &&
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_prof.json 2> $out/prof.err
rc=$?
tail -2 $out/pytest_sa.log; grep -E "passed|failed|salz_encode_safe" $out/pytest.log | tail -4; cat $out/bench.json 2>/dev/null
exit $rc
