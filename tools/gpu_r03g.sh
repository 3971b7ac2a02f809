set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03g}
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_batch.py -k "suffix_sort_modes or stages_match or appendix_c or lcp_paths or edge_sizes or large_blocks or staged_scatters or batch" > $out/pytest_sa.log 2>&1 &&
timeout -k 10 600 bash tools/gpu_envab.sh $out/ab "SALZ_ALPHA_K8=1" "SALZ_ALPHA_K8=0" > $out/ab.txt 2>&1 &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 1 --warmup 0 --no-e2e > $out/text_sa.json 2> $out/text_sa.log
rc=$?
tail -2 $out/pytest_sa.log; cat $out/ab.txt; grep "sa round" $out/text_sa.log | head -11
exit $rc
