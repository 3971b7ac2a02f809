# Parse study: kernel traces of the mixed 100 MB block and the Silesia-sized workload, with the
# per-pass debug lines. Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03j}
mkdir -p $out
SALZ_DEBUG_PARSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed.json 2> $out/mixed_parse.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_mixed -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 2 --warmup 1 > $out/mixed_prof.json 2> $out/mixed_prof.err &&
SALZ_DEBUG_PARSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --steps 2 --warmup 1 > $out/silesia.json 2> $out/silesia_parse.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_silesia -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --steps 2 --warmup 1 > $out/silesia_prof.json 2> $out/silesia_prof.err
rc=$?
cat $out/mixed.json $out/silesia.json
exit $rc
