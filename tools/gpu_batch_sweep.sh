#!/bin/bash
# Batch-size sweep: C3 (silesia-sized mixed, 16 MiB blocks), C4 (enwik9-sized, 64 MiB blocks)
# and the level sweep through salz_encode_blocks, at several SALZ_BATCH_BYTES.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-sweep}
mkdir -p $out
for bb in ${BATCHES:-16777216 33554432 67108864 134217728}; do
  timeout -k 10 200 python bench.py --workload silesia --steps 2 --no-cpu-baseline --no-e2e --batch-bytes $bb > $out/silesia_$bb.json 2> $out/silesia_$bb.err || exit 1
  SALZ_BATCH_BYTES=$bb timeout -k 10 300 python tools/bench_levels.py --size 50000003 --levels 0-9 --reps 2 > $out/levels_$bb.jsonl 2> $out/levels_$bb.err || exit 1
done
for sl in 1 2 4; do
  timeout -k 10 300 python bench.py --workload enwik9 --steps 1 --no-cpu-baseline --no-e2e --slots $sl > $out/enwik9_s$sl.json 2> $out/enwik9_s$sl.err || exit 1
done
for f in $out/silesia_*.json $out/enwik9_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['parallelism'][-60:])"; done
for f in $out/levels_*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['level'], d.get('compress_MBps'), end='; ')
print()"; done
