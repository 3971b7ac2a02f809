# C3 and C4 throughput against the number of encoder slots.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03u}
mkdir -p $out
for r in 1 2; do for sl in 3 4 6 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --slots $sl --steps 2 > $out/s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/s.json'));print('silesia slots $sl', d['value'])"
done; done > $out/slots.txt &&
for sl in 2 4 6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload enwik9 --slots $sl --steps 1 > $out/s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$out/s.json'));print('enwik9 slots $sl', d['value'])"
done >> $out/slots.txt
rc=$?
cat $out/slots.txt
exit $rc
