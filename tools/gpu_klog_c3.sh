#!/bin/bash
# One GPU call: parse chunk length on the Silesia-sized workload (16 MiB blocks, 4 slots).
set -o pipefail
export TMPDIR=/tmp
R=2 ARGS="--workload silesia" bash tools/ab_env.sh "-" "SALZ_PARSE_KLOG=7" "SALZ_PARSE_KLOG=8" "SALZ_PARSE_KLOG=9"
