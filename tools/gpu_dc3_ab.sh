#!/bin/bash
# One GPU call: DC3 parity tests, then the in-tree build against ab/base.so on C5 Fibonacci.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-dc3ab}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "dc3 or staged or fib_256" > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $out/pytest.log | head; exit $rc; }
R=2 ARGS="--workload fib256 --steps 2" bash tools/ab_env.sh "SALZ_LIB_PATH=$PWD/ab/base.so" "-"
