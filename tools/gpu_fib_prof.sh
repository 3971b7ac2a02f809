#!/bin/bash
# One GPU call: kernel stats and trace of the C5 Fibonacci workload (DC3 path).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-fibp}; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --workload fib256 --steps 1 --warmup 0 > $out/fib.json 2> $out/fib.err
