# Round-end check, part A: the full -m gpu suite, smoke, the default bench (PMC passes and CPU
# baseline in the run) and a kernel trace of the bench. Every GPU step has its own limit.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03z}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_prof.json 2> $out/prof.err
rc=$?
tail -3 $out/pytest.log; cat $out/smoke.log; cut -c1-400 $out/bench.json
exit $rc
