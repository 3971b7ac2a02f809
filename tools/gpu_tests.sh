#!/bin/bash
# One GPU call: the -m gpu suite (optionally a -k filter in $K), smoke(), then the default bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-tests}
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $out/bench.json 2> $out/bench.err
rc=$?
grep -E "passed|failed|error" $out/pytest.log | tail -3; cat $out/smoke.log $out/bench.json 2>/dev/null
exit $rc
