# K = 128 for every single block of 8-16 MiB: parity subset, then C3 text and C3.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03x}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs.py tests/test_batch.py -k "c3_ or large_blocks or mixed or batch or blocks or stream or cli or chunk or grows" > $out/pytest.log 2>&1 &&
for k in text mixed; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --kind $k --steps 2 > $out/s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/s.json'));print('silesia $k', d['value'], d['stages_ms_last_block'])"
done > $out/c3.txt
rc=$?
tail -2 $out/pytest.log; cat $out/c3.txt
exit $rc
