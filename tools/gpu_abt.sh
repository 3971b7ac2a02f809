# stage parity tests, then A/B of the in-tree build against ab/base.so (tools/ab.sh)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-abt}
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_batch.py -k "${TESTS:-stages_match or appendix_c or edge_sizes or large_blocks or batch or suffix_sort_modes}" > $out/pytest.log 2>&1 &&
timeout -k 10 600 bash tools/ab.sh ${R:-3} --no-pmc ${BENCH_ARGS:-} > $out/ab.txt 2>&1
rc=$?
tail -2 $out/pytest.log; cat $out/ab.txt
exit $rc
