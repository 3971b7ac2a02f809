#!/bin/bash
# One GPU call, parameterised (replaces the per-experiment gpu_r03*.sh scripts). Every GPU step
# runs under its own time limit and the chain stops at the first failure.
#   TAG=r04a TESTS="tests/test_gpu_parity.py -k sort" BENCH="--no-cpu-baseline" PROF=1 tools/gpu_run.sh
#   TESTS    pytest arguments (default: the whole -m gpu suite; "none" skips the tests)
#   SMOKE=1  __graft_entry__.smoke()
#   BENCH    bench.py arguments for one bench line (default none)
#   PROF=1   rocprofv3 kernel-trace summary of the bench command (tools/prof_summary.py)
#   ROUNDS=1 per-round suffix-sort trace of that profile (tools/trace_rounds.py)
#   EXTRA    further shell commands, run last under a 600 s limit
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-run}
mkdir -p "$out"
rc=0
if [ "${TESTS:-}" != "none" ]; then
  eval "timeout -k 10 900 python -u -m pytest ${TESTS:--m gpu tests} -x -q --timeout 300 --timeout-method thread" \
    > "$out/pytest.log" 2>&1 || rc=$?
  tail -3 "$out/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 180 python -c 'import __graft_entry__ as g; g.smoke()' > "$out/smoke.log" 2>&1 || exit $?
  cat "$out/smoke.log"
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 500 python bench.py $BENCH > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
  cut -c1-600 "$out/bench.json"
fi
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/prof" -o prof --output-format csv -- \
    python3 bench.py ${PBENCH:---no-cpu-baseline --no-pmc --no-e2e} > "$out/bench_prof.json" 2> "$out/prof.err" || exit $?
  python tools/prof_summary.py "$out/prof/prof_kernel_stats.csv" > "$out/kernel_stats.txt" 2>&1 && head -30 "$out/kernel_stats.txt"
  if [ -n "${ROUNDS:-}" ]; then
    python tools/trace_rounds.py "$out/prof/prof_kernel_trace.csv" 2 > "$out/rounds.txt" 2>&1 && cat "$out/rounds.txt"
  fi
fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > "$out/extra.log" 2>&1 || { tail -20 "$out/extra.log"; exit 1; }
  tail -40 "$out/extra.log"
fi
exit 0
