timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -2 gpurun_out/pt.log
for r in 4 1; do
SALZ_SPLIT_RATIO=$r timeout -k 10 200 python bench.py --no-cpu-baseline --workload fib256 --steps 1 --warmup 1 > gpurun_out/fr.json 2> gpurun_out/fr.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/fr.json'));s=d['stages_ms_last_block'];print('fib ratio $r', d['value'], s['ms_sa'], d['roundtrip_ok'])"
done
bash tools/ab.sh 1
for r in 4 1; do
SALZ_SPLIT_RATIO=$r timeout -k 10 200 python bench.py --no-cpu-baseline --kind mixed --steps 2 > gpurun_out/fr.json 2> gpurun_out/fr.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/fr.json'));s=d['stages_ms_last_block'];print('mixed ratio $r', d['value'], s['ms_sa'], d['roundtrip_ok'])"
done
