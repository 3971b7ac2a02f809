#!/bin/bash
# Kernel-trace profile of one bench workload: WL=<workload> TAG=<tag> tools/gpu_prof.sh [extra bench args]
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-prof}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_${WL} -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --workload ${WL:-enwik8} --steps 1 --warmup 0 "$@" > $out/${WL}.json 2> $out/${WL}.err
