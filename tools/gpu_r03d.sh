# A/B of the in-tree build against ab/base.so (tools/ab.sh), then the in-tree build's per-round
# trace and kernel stats
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03d}
mkdir -p $out
timeout -k 10 600 bash tools/ab.sh 3 --no-pmc > $out/ab.txt 2>&1 &&
SALZ_DEBUG_SA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 2 --warmup 1 > $out/text_sa.json 2> $out/text_sa.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e > $out/bench_prof.json 2> $out/prof.err
rc=$?
cat $out/ab.txt
exit $rc
