# Lazy parse costs: parse parity subset, then A/B of the lazy passes on mixed 100 MB, C3 and C2.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03l}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "parse_wave_skip or stages_every_chunk or stages_match or large_exit_set or large_blocks or batch or appendix" > $out/pytest.log 2>&1 &&
ARGS="--no-pmc --kind mixed" KTOP=16 timeout -k 10 300 bash tools/gpu_prof_ab.sh "SALZ_PARSE_LAZY=0" "-" > $out/prof_mixed.txt 2>&1 &&
cp gpurun_out/prof_ab/2/prof_kernel_trace.csv $out/mixed_lazy_trace.csv &&
timeout -k 10 600 bash tools/gpu_envab.sh $out/ab "SALZ_PARSE_LAZY=0" "SALZ_PARSE_LAZY=1" > $out/ab.txt 2>&1 &&
for w in silesia; do for v in 0 1; do SALZ_PARSE_LAZY=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload $w --steps 2 --warmup 1 > $out/$w.$v.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('$out/$w.$v.json'));print('$w lazy=$v', d['value'], d['stages_ms_last_block'])"; done; done > $out/ab_c3.txt
rc=$?
tail -3 $out/pytest.log; grep -E "^==|parse|cost_rest|lazy" $out/prof_mixed.txt; cat $out/ab.txt $out/ab_c3.txt
exit $rc
