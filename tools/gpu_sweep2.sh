set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r02i; mkdir -p $out
for sl in 2 4; do
  SALZ_SLOTS=$sl timeout -k 10 300 python tools/bench_levels.py --size 50000003 --levels 0-9 --reps 2 > $out/levels_s$sl.jsonl 2> $out/levels_s$sl.err || exit 1
done
SALZ_SLOTS=4 SALZ_BATCH_BYTES=8388608 timeout -k 10 300 python tools/bench_levels.py --size 50000003 --levels 0-7 --reps 2 > $out/levels_s4_8m.jsonl 2> $out/levels_s4_8m.err || exit 1
timeout -k 10 200 python bench.py --workload silesia --steps 2 --no-cpu-baseline --no-e2e > $out/silesia.json 2> $out/silesia.err || exit 1
timeout -k 10 200 python bench.py --workload silesia --kind text --size 50000003 --steps 2 --no-cpu-baseline --no-e2e > $out/text50.json 2> $out/text50.err || exit 1
python -c "import json; d=json.load(open('$out/silesia.json')); print('silesia', d['value'])"
for f in $out/levels_*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['level'], d.get('compress_MBps'), end='; ')
print()"; done
