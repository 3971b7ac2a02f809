#!/bin/bash
# One GPU call: parse chunk length on 64 MiB mixed blocks: the default rule
# (K = 512 from 32 MiB + 8) against K = 256 and 128.
set -o pipefail
export TMPDIR=/tmp
R=2 ARGS="--kind mixed --size 67108864" bash tools/ab_env.sh "SALZ_PARSE_KLOG=7" "SALZ_PARSE_KLOG=8" "-"

