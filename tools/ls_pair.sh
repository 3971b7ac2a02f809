#!/bin/bash
# two concurrent load-stress processes: $1 = tag, $2/$3 = "N ITERS EXTRA PRE SEED" for A / B
( timeout -k 10 200 python tools/load_stress.py $2 > gpurun_out/$1a.log 2>&1 &
  timeout -k 10 200 python tools/load_stress.py $3 > gpurun_out/$1b.log 2>&1; wait )
echo "$1: A[$2] $(grep -h mismatches gpurun_out/$1a.log) $(grep -h -o 'T=0x[0-9a-f]*' gpurun_out/$1a.log) | B[$3] $(grep -h mismatches gpurun_out/$1b.log) $(grep -h -o 'T=0x[0-9a-f]*' gpurun_out/$1b.log)"
