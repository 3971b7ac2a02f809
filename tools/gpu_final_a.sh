#!/bin/bash
# Round-end set, part A (one GPU call): the -m gpu suite, smoke, the default bench line (CPU
# baseline and PMC traffic measured in the same run), a kernel-trace profile of C2 with the
# per-round suffix sort, and per-kernel PMC traffic / SQ counters of C2.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-final}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e > $out/bench_prof.json 2> $out/prof.err &&
python tools/prof_summary.py $out/prof/prof_kernel_stats.csv > $out/text100M_kernel_stats.txt &&
python tools/trace_rounds.py $out/prof/prof_kernel_trace.csv 2 > $out/text100M_rounds.txt &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_fetch.json 2> $out/pmc_fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_write.json 2> $out/pmc_write.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $out/pmc_sq -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_sq.json 2> $out/pmc_sq.err
rc=$?
python tools/pmc_traffic.py $out/pmc_fetch/pmc_counter_collection.csv $out/pmc_write/pmc_counter_collection.csv --summary $out/pmc_traffic.txt > /dev/null 2>&1
python tools/sq_summary.py $out/pmc_sq/pmc_counter_collection.csv > $out/sq_counters.txt 2>&1
tail -2 $out/pytest.log; cat $out/smoke.log; cut -c1-400 $out/bench.json
exit $rc
