# C5 (256 MiB Fibonacci, DC3) kernel trace of the current build.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03s}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fib -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload fib256 --steps 1 --warmup 1 > $out/fib.json 2> $out/fib.err
rc=$?
cut -c1-600 $out/fib.json
exit $rc
