#!/bin/bash
# One GPU call: parity tests, smoke, bench (default config) and a kernel-trace profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-run}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline > $out/bench_prof.json 2> $out/prof.err
rc=$?
tail -3 $out/pytest.log; cat $out/smoke.log $out/bench.json 2>/dev/null
exit $rc
