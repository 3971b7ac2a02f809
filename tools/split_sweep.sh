timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -2 gpurun_out/pt.log
timeout -k 10 200 python bench.py --no-cpu-baseline --workload fib256 --steps 1 --warmup 1 > gpurun_out/fr.json 2> gpurun_out/fr.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/fr.json'));s=d['stages_ms_last_block'];print('fib', d['value'], s, d['roundtrip_ok'])"
bash tools/ab.sh 1
