#!/bin/bash
# One GPU call: the split-suffix-array tests (ranks over gloo on the box's one GPU), then
# tools/bench_split.py on one rank over RCCL and on 2 / 4 gloo ranks sharing the GPU.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-split}; mkdir -p $out
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 python -u -m pytest tests/test_dist_split.py -x -v --timeout 300 --timeout-method thread > $out/split.log 2>&1 &&
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29511 tools/bench_split.py --kind text > $out/text1.json 2> $out/text1.err &&
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29512 tools/bench_split.py --kind text --size 20000000 --gloo > $out/text2g.json 2> $out/text2g.err &&
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29513 tools/bench_split.py --kind mixed --size 20000000 --gloo > $out/mixed4g.json 2> $out/mixed4g.err
rc=$?
grep -E "passed|failed" $out/split.log | tail -1; cat $out/*.json
exit $rc
