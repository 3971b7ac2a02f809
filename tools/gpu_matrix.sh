# Every BASELINE workload on one box (bench.py lines) + the level sweep; per-kernel stats of C5.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03m}
mkdir -p $out
timeout -k 10 200 python bench.py --no-pmc --workload fib256 --steps 2 --warmup 1 --no-cpu-baseline > $out/fib.json 2> $out/fib.err &&
timeout -k 10 200 python bench.py --no-pmc --kind mixed --steps 2 --warmup 1 --no-cpu-baseline > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 200 python bench.py --no-pmc --workload silesia --steps 2 --warmup 1 > $out/silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --no-pmc --workload enwik9 --steps 1 --warmup 1 > $out/enwik9.json 2> $out/enwik9.err &&
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fib -o prof --output-format csv -- python3 bench.py --no-pmc --no-cpu-baseline --no-e2e --workload fib256 --steps 2 --warmup 1 > $out/fib_prof.json 2> $out/fib_prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_mixed -o prof --output-format csv -- python3 bench.py --no-pmc --no-cpu-baseline --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed_prof.json 2> $out/mixed_prof.err
rc=$?
for f in fib mixed silesia enwik9; do python -c "import json;d=json.load(open('$out/$f.json'));print('$f', d['value'], d.get('value_e2e'), d['stages_ms_last_block'], d['roundtrip_ok'], d.get('parity_vs_cpu_port'))"; done
cat $out/levels.jsonl | python -c "import sys,json;[print(json.loads(l).get('level'), json.loads(l).get('compress_MBps') or json.loads(l)) for l in sys.stdin]" 2>/dev/null | head -12
exit $rc
