# round 3 GPU check: full -m gpu suite, smoke, default bench (with its PMC passes) and a kernel
# trace of the bench. Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_prof.json 2> $out/prof.err
rc=$?
tail -3 $out/pytest.log; cat $out/smoke.log $out/bench.json 2>/dev/null
exit $rc
