#!/bin/bash
# Throughput of every BASELINE config plus the level sweep (one GPU call; each step time-boxed).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-perf}
mkdir -p $out
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $out/bench.json 2> $out/bench.err &&
timeout -k 10 200 python bench.py --workload silesia --steps 3 --no-cpu-baseline > $out/silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --workload enwik9 --steps 2 --no-cpu-baseline --no-e2e > $out/enwik9.json 2> $out/enwik9.err &&
timeout -k 10 200 python bench.py --workload fib256 --steps 2 --no-cpu-baseline --no-e2e > $out/fib.json 2> $out/fib.err &&
timeout -k 10 200 python bench.py --kind mixed --steps 2 --no-cpu-baseline --no-e2e > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err
rc=$?
for f in bench silesia enwik9 fib mixed; do python -c "
import json,sys
try:
    d=json.load(open('$out/$f.json'))
    print('$f', d['value'], 'e2e', d.get('value_e2e'), 'ms', d['ms_per_step'], d['stages_ms_last_block'], 'rt', d['roundtrip_ok'], d.get('container_roundtrip_ok'), 'par', d['parity_vs_cpu_port'])
except Exception as e: print('$f', 'missing', e)
"; done
cut -c1-200 $out/levels.jsonl
exit $rc
