#!/bin/bash
# Parity tests + the level sweep (multi-block container path).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-quick}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err
rc=$?
tail -2 $out/pytest.log; cat $out/levels.jsonl | cut -c1-220
exit $rc
