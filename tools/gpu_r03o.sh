# C3 (Silesia-sized, 16 MiB blocks) with one encoder slot: kernel trace for the per-block breakdown.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03o}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c3s1 -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --slots 1 --steps 1 --warmup 1 > $out/c3s1.json 2> $out/c3s1.err &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --slots 1 --steps 2 --warmup 1 > $out/c3s1_noprof.json 2>/dev/null
rc=$?
[ $rc -eq 0 ] && for r in 1 2; do for kl in 9 8 7 6; do
  SALZ_PARSE_KLOG=$kl timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 3 > $out/kl.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/kl.json'));print('mixed klog $kl', d['value'], d['parse_iters'], d['stages_ms_last_block'])"
done; done > $out/klog_ab.txt
rc=$?
cat $out/klog_ab.txt
cat $out/c3s1.json $out/c3s1_noprof.json | cut -c1-900
exit $rc
