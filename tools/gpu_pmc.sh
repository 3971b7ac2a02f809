#!/bin/bash
# PMC passes (one counter group per run, per the MI355X guide) over one bench step, plus
# per-round SA diagnostics for the text and Fibonacci configs.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-pmc}
mkdir -p $out
SALZ_DEBUG_SA=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $out/text.json 2> $out/text_sa.log &&
SALZ_DEBUG_SA=1 SALZ_DEBUG_PARSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --kind fib --size 268435456 --steps 1 --warmup 1 > $out/fib.json 2> $out/fib_sa.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $out/pmc_fetch.json 2> $out/pmc_fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o pmc -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $out/pmc_write.json 2> $out/pmc_write.err
rc=$?
cat $out/text.json $out/fib.json
exit $rc
