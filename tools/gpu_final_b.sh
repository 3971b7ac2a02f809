# Round-end check, part B: the other workloads, their traces, per-kernel PMC traffic of C2 and the
# level sweep. Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03z}
mkdir -p $out
timeout -k 10 200 python bench.py --workload silesia --steps 2 --warmup 1 > $out/silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --workload enwik9 --steps 1 --warmup 1 > $out/enwik9.json 2> $out/enwik9.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --kind mixed --steps 2 --warmup 1 > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fib -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload fib256 --steps 2 --warmup 1 > $out/fib.json 2> $out/fib.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_mixed -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed_prof.json 2> $out/mixed_prof.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_fetch.json 2> $out/pmc_fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_write.json 2> $out/pmc_write.err &&
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err
rc=$?
for f in silesia enwik9 mixed fib; do cut -c1-300 $out/$f.json; done
exit $rc
