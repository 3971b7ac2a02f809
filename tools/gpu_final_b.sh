#!/bin/bash
# Round-end set, part B (one GPU call): every workload's bench line, a kernel-trace profile of C5,
# the mixed 100 MB block, the level sweep, the pathological inputs at 256 MiB and the split
# suffix array at one rank.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-final}
mkdir -p $out
timeout -k 10 200 python bench.py --workload fib256 --steps 3 --warmup 1 > $out/bench_fib.json 2> $out/fib.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --kind mixed --steps 3 --warmup 1 > $out/bench_mixed.json 2> $out/mixed.err &&
timeout -k 10 200 python bench.py --workload silesia --steps 3 --warmup 1 > $out/bench_silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --workload enwik9 --steps 2 --warmup 1 > $out/bench_enwik9.json 2> $out/enwik9.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fib -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload fib256 --steps 2 --warmup 1 > $out/fib_prof.json 2> $out/fib_prof.err &&
python tools/prof_summary.py $out/prof_fib/prof_kernel_stats.csv > $out/fib256_kernel_stats.txt &&
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err &&
timeout -k 10 500 python tools/stress_inputs.py --size 268435456 --stages > $out/stress256M.txt 2> $out/stress.err
rc=$?
for f in $out/bench_*.json; do echo $f; cut -c1-300 $f; done
exit $rc
