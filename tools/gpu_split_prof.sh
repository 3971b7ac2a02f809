#!/bin/bash
# One GPU call: kernel trace of the split-block path on one rank (RCCL).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-splitp}; mkdir -p $out
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 tools/bench_split.py --kind text --steps 2 > $out/text1.json 2> $out/text1.err
rc=$?
cat $out/text1.json
exit $rc
