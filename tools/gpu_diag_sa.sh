#!/bin/bash
# Per-round suffix-sort diagnostics (SALZ_DEBUG_SA=1: m, groups and wall time per doubling
# round) for the text, Fibonacci and mixed workloads, plus a kernel-trace profile of each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-diag}
mkdir -p $out
SALZ_DEBUG_SA=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --steps 1 --warmup 1 > $out/text.json 2> $out/text_sa.log &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload fib256 --steps 1 --warmup 1 > $out/fib.json 2> $out/fib_sa.log &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --kind mixed --steps 1 --warmup 1 > $out/mixed.json 2> $out/mixed_sa.log &&
for WL in enwik8 fib256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$WL -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --workload $WL --steps 2 --warmup 0 > $out/prof_$WL.json 2> $out/prof_$WL.err || exit 1
done
rc=$?
cat $out/text.json $out/fib.json $out/mixed.json | cut -c1-300
exit $rc
