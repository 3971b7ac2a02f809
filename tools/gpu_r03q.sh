# Deep-prefetch late walk: parse parity subset, env A/B on mixed 100 MB, C3 and C2, and a mixed trace.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03q}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "parse_wave_skip or stages_every_chunk or stages_match or large_exit_set or large_blocks or batch or appendix" > $out/pytest.log 2>&1 &&
for w in "--kind mixed" "--workload silesia" ""; do for r in 1 2; do for v in 0 1; do
  SALZ_PARSE_DEEP=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 3 $w > $out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/ab.json'));print('$w deep=$v', d['value'], d['stages_ms_last_block'])"
done; done; done > $out/ab.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_mixed -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed_prof.json 2> $out/mixed_prof.err
rc=$?
tail -2 $out/pytest.log; cat $out/ab.txt
exit $rc
