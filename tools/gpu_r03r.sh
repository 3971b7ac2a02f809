# Parse chunk length on large blocks: mixed and text 100 MB, enwik9-sized 64 MiB text blocks.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03r}
mkdir -p $out
for w in "--kind mixed" "" "--workload enwik9 --steps 1"; do for r in 1 2; do for kl in 9 8 7; do
  SALZ_PARSE_KLOG=$kl timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 3 $w > $out/kl.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/kl.json'));print('$w klog $kl', d['value'], d['parse_iters'], d['stages_ms_last_block'])"
done; done; done > $out/klog_ab.txt
rc=$?
cat $out/klog_ab.txt
exit $rc
