#!/bin/bash
# One GPU call: the split-block path on one rank (RCCL) against the single-GPU path, and a
# two-rank gloo rehearsal on the same GPU.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-splitb}; mkdir -p $out
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29511 tools/bench_split.py --kind text > $out/text1.json 2> $out/text1.err &&
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29512 tools/bench_split.py --kind text --size 20000000 --gloo > $out/text2g.json 2> $out/text2g.err &&
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29513 tools/bench_split.py --kind mixed --size 20000000 --gloo > $out/mixed4g.json 2> $out/mixed4g.err
rc=$?
cat $out/*.json; tail -3 $out/*.err | head -30
exit $rc
