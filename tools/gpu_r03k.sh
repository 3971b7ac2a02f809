# A/B: ANSV blocks per workgroup, 512-thread text-sourced radix pass; parity subset with both on.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03k}
mkdir -p $out
SALZ_ANSV_SUB=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs.py -k "stages_match or appendix_c or edge_sizes or c2_ or large_blocks or batch" > $out/pytest.log 2>&1 &&
timeout -k 10 600 bash tools/gpu_envab.sh $out/ab "SALZ_ANSV_SUB=1" "SALZ_ANSV_SUB=2" "SALZ_ANSV_SUB=4" "SALZ_ANSV_SUB=8" > $out/ab.txt 2>&1
rc=$?
tail -2 $out/pytest.log; cat $out/ab.txt
exit $rc
