#!/bin/bash
# Concurrency regression check (DESIGN.md "Concurrent encodes and the unaligned text load"):
# several contexts encode on one GPU at once, every stream compared with the CPU port, with
# the stage invariant checks on. One GPU call:
#   gpurun -- 'bash tools/diag_blocks.sh'
set -o pipefail
mkdir -p gpurun_out/dg
export SALZ_CHECK_STAGES=1
timeout -k 10 200 python tools/diag_concurrency.py --threads 4 --iters 20 --device > gpurun_out/dg/text.log 2>&1 &&
timeout -k 10 200 python tools/diag_concurrency.py --threads 4 --iters 20 --device --kind mixed --size 2000001 > gpurun_out/dg/mixed.log 2>&1 &&
timeout -k 10 200 python tools/diag_concurrency.py --threads 2 --iters 10 --device --procs > gpurun_out/dg/procs.log 2>&1
rc=$?
for f in text mixed procs; do tail -1 gpurun_out/dg/$f.log; done
exit $rc
