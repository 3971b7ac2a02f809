#!/bin/bash
# Run two concurrent diag processes on the one GPU; $1 = tag, rest = env assignments.
tag=$1; shift
( env "$@" timeout -k 10 200 python tools/diag.py --size 20000000 --reps ${REPS:-4} --tag ${tag}A > gpurun_out/${tag}A.log 2>&1 &
  env "$@" timeout -k 10 200 python tools/diag.py --size 20000000 --reps ${REPS:-4} --tag ${tag}B > gpurun_out/${tag}B.log 2>&1; wait )
for f in gpurun_out/${tag}A.log gpurun_out/${tag}B.log; do
  echo "== $f ok=$(grep -c 'len=' $f) failed=$(grep -c FAILED $f)"; grep "^check" $f | head -12
done
