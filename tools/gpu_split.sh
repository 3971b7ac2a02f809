#!/bin/bash
# One GPU call: the split-suffix-array tests (ranks over gloo on the box's GPU) and the suffix
# sorter's single-GPU parity tests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-split}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_dist_split.py -x -v --timeout 300 --timeout-method thread > $out/split.log 2>&1
rc=$?
grep -E "passed|failed|Error|error" $out/split.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "stages_match or suffix_sort or appendix or lcp_paths" > $out/parity.log 2>&1
rc=$?
tail -3 $out/parity.log
exit $rc
