#!/bin/bash
# Kernel-trace profiles of the 256 MiB pathological inputs (tools/stress_inputs.py), one case per
# rocprofv3 run:  TAG=r06c CASES="runs halves" bash tools/gpu_stress_prof.sh
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-stressprof}
mkdir -p "$out"
for c in ${CASES:-runs halves}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_$c" -o prof --output-format csv -- \
    python3 tools/stress_inputs.py --size ${SIZE:-268435456} --cases "$c" > "$out/stress_$c.txt" 2>&1 || exit $?
  python tools/prof_summary.py "$out/prof_$c/prof_kernel_stats.csv" > "$out/${c}_kernel_stats.txt" 2>&1 || exit $?
  cat "$out/stress_$c.txt"; head -40 "$out/${c}_kernel_stats.txt"
done
