set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03m}
mkdir -p $out
SALZ_DEBUG_PARSE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 1 --warmup 0 > $out/mixed.json 2> $out/mixed_parse.log
rc=$?
grep "parse it" $out/mixed_parse.log | tail -30
exit $rc
