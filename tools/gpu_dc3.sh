#!/bin/bash
# One GPU call: the DC3 parity tests, then the Fibonacci 256 MiB bench (BASELINE configs[4]).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-dc3}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "dc3 or fib_256" > $out/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --workload fib256 --steps 3 --warmup 1 > $out/fib.json 2> $out/fib.err
rc=$?
grep -E "passed|failed|error|Error" $out/pytest.log | tail -5; cat $out/fib.json
exit $rc
