#!/bin/bash
# One GPU call: parse parity tests, then A/B of the in-tree build against ab/base.so on mixed
# 100 MB, Silesia-sized blocks and text.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-parse}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "parse_wave_skip or stages_match or large or dc3_auto" > $out/pytest.log 2>&1 || { grep -E "passed|failed|Error" $out/pytest.log | tail; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -1
B=SALZ_LIB_PATH=$PWD/ab/base.so
R=2 ARGS="--kind mixed" bash tools/ab_env.sh "$B" "-" &&
R=2 ARGS="--workload silesia" bash tools/ab_env.sh "$B" "-" &&
R=2 bash tools/ab_env.sh "$B" "-"
