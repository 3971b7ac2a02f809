#!/bin/bash
# Per-kernel A/B of environment settings on one GPU box: a rocprofv3 kernel-trace of the bench per
# setting ("-" for none), summarised with tools/prof_summary.py (top KTOP kernels).
#   ARGS="--kind mixed" bash tools/gpu_prof_ab.sh "SALZ_SEG_TINY=0" "-"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_ab
k=0
for setting in "$@"; do
  k=$((k + 1))
  d=gpurun_out/prof_ab/$k
  (
    [ "$setting" != "-" ] && export $setting
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o prof --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-e2e --steps 3 $ARGS > $d.json 2> $d.err
  ) || { tail -5 $d.err; exit 1; }
  echo "== $setting: $(python3 -c "import json;d=json.load(open('$d.json'));print(d['value'], d['stages_ms_last_block'])")"
  python3 tools/prof_summary.py $d/prof_kernel_stats.csv > $d.txt && head -${KTOP:-14} $d.txt
done
