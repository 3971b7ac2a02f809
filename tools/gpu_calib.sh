#!/bin/bash
# PMC calibration of FETCH_SIZE / WRITE_SIZE per access pattern (tools/gather_bench calib): one
# rocprofv3 pass per counter group, then a kernel trace for the durations. Every step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-calib}
mkdir -p "$out"
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
grep -E "TCC_EA0?_(RD|WR)REQ|TCC_BUBBLE|TCC_REQ" "$out/counters.txt" | head -40 > "$out/tcc_ea_counters.txt" || true
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o pmc -- tools/gather_bench calib > "$out/calib.txt" 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o pmc -- tools/gather_bench calib > /dev/null 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d "$out/trace" -o tr -- tools/gather_bench calib > /dev/null 2>&1 || exit 1
if [ -n "${EXTRA_PMC:-}" ]; then
  timeout -s KILL 60 rocprofv3 --pmc $EXTRA_PMC --output-format csv -d "$out/extra" -o pmc -- tools/gather_bench calib > /dev/null 2>&1 || exit 1
fi
cat "$out/calib.txt" "$out/tcc_ea_counters.txt"
