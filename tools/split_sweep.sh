for kind in text mixed; do for r in 1 4 1000; do
SALZ_SPLIT_RATIO=$r timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --kind $kind > gpurun_out/sr.json 2> gpurun_out/sr.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/sr.json'));s=d['stages_ms_last_block'];print('$kind ratio $r', d['value'], s['ms_sa'], d['roundtrip_ok'])"
done; done
