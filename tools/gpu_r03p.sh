# Parse parity subset, then A/B against ab/base.so (previous commit): C3 (4 slots and 1), mixed 100 MB, C2.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03p}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs.py -k "stages_every_chunk or stages_match or large_exit_set or large_blocks or batch or appendix or c3_ or c2_ or mixed or edge or fib or dc3_large or lcp_paths" > $out/pytest.log 2>&1 &&
for w in "" "--kind mixed" "--workload silesia" "--workload fib256 --steps 2"; do for r in 1 2; do for v in base new; do
  if [ $v = base ]; then export SALZ_LIB_PATH=/root/repo/ab/base.so; else unset SALZ_LIB_PATH; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 3 $w > $out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/ab.json'));print('$w', '$v', d['value'], d['stages_ms_last_block'])"
done; done; done > $out/ab.txt
rc=$?
tail -2 $out/pytest.log; cat $out/ab.txt
exit $rc
