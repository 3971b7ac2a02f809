# C3 chunk length with the round-3 parse (16 MiB mixed blocks: K = 64 by default).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03v}
mkdir -p $out
for r in 1 2; do for kl in 6 7 8; do
  SALZ_PARSE_KLOG=$kl timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --steps 2 > $out/kl.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/kl.json'));print('silesia klog $kl', d['value'], d['parse_iters'], d['stages_ms_last_block'])"
done; done > $out/klog.txt
rc=$?
cat $out/klog.txt
exit $rc
