#!/bin/bash
# Suffix-sort change check: the large-block parity tests, then text / Fibonacci / mixed benches
# with per-round SA timing and a kernel trace of the text bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-sa}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "large or fib or c2 or c4 or c3 or stages_match or suffix_sort or lcp_paths or batch_matches" > $out/pytest.log 2>&1 &&
SALZ_DEBUG_SA=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --steps 1 --warmup 1 > $out/text_sa.json 2> $out/text_sa.log &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload fib256 --steps 1 --warmup 1 > $out/fib_sa.json 2> $out/fib_sa.log &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 > $out/text.json 2> $out/text.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload fib256 --steps 2 > $out/fib.json 2> $out/fib.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --kind mixed --steps 3 > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_text -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --steps 2 --warmup 0 > $out/prof_text.json 2> $out/prof_text.err
rc=$?
tail -3 $out/pytest.log
for f in text fib mixed; do python -c "
import json
try:
    d=json.load(open('$out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['stages_ms_last_block'], d['roundtrip_ok'])
except Exception as e: print('$f missing', e)"; done
exit $rc
