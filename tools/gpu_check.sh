#!/bin/bash
# One GPU call: parity tests, smoke, bench (default config) and a kernel-trace profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r02w}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_prof.json 2> $out/prof.err
rc=$?
tail -3 $out/pytest.log; cat $out/smoke.log $out/bench.json 2>/dev/null

[ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --steps 1 --warmup 0 > $out/pmc_fetch.json 2> $out/pmc_fetch.err &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --steps 1 --warmup 0 > $out/pmc_write.json 2> $out/pmc_write.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $out/pmc_sq -o pmc -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 0 > $out/pmc_sq.json 2> $out/pmc_sq.err &&
SALZ_DEBUG=sa timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > $out/text_sa.json 2> $out/text_sa.log &&
SALZ_DEBUG=sa timeout -k 10 200 python bench.py --no-cpu-baseline --workload fib256 --steps 2 --warmup 1 > $out/fib.json 2> $out/fib_sa.log &&
timeout -k 10 200 python bench.py --no-cpu-baseline --kind mixed --steps 2 --warmup 1 > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 200 python bench.py --workload silesia --steps 2 --warmup 1 > $out/silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --workload enwik9 --steps 1 --warmup 1 > $out/enwik9.json 2> $out/enwik9.err
timeout -k 10 300 python tools/bench_levels.py --size 50000003 > $out/levels.jsonl 2> $out/levels.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fib -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload fib256 --steps 2 --warmup 1 > $out/fib_prof.json 2> $out/fib_prof.err
SALZ_SA=dc3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 2 --warmup 1 > $out/text_dc3.json 2> $out/text_dc3.err
SALZ_SA=dc3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed_dc3.json 2> $out/mixed_dc3.err
