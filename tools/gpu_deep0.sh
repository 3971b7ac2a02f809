#!/bin/bash
# One GPU call: suffix-sort parity tests with the depth-16 round 0, then A/B (SALZ_DEEP0) on text.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-deep0}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_batch.py -x -q --timeout 300 --timeout-method thread -k "stages_match or suffix_sort or appendix or lcp_paths or batch or edge or concurrent or c2 or c4" > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $out/pytest.log | head -20; exit $rc; }
R=2 bash tools/ab_env.sh "SALZ_DEEP0=0" "-" &&
R=1 ARGS="--workload enwik9 --steps 1" bash tools/ab_env.sh "SALZ_DEEP0=0" "-"
