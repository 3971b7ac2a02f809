#!/bin/bash
# One GPU call: staged-scatter and DC3 parity tests, then A/B of SALZ_SCATTER_STAGE on C5.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-stage}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "staged or dc3 or fib_256 or lcp_paths" > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $out/pytest.log | head; exit $rc; }
R=2 ARGS="--workload fib256 --steps 2" bash tools/ab_env.sh "SALZ_SCATTER_STAGE=0" "-"
