#!/bin/bash
# One GPU call: the GPU parity suite (or the tests matching $TESTS), then tools/ab.sh (baseline
# ab/base.so vs the in-tree build) on text 100 MB, mixed 100 MB and the Silesia-sized workload.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} \
  > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
bash tools/ab.sh ${R:-2} &&
bash tools/ab.sh ${R:-2} --kind mixed &&
bash tools/ab.sh ${R:-2} --workload silesia --steps 2 --warmup 1
