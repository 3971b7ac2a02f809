#!/bin/bash
# Staged scatter A/B (round 6): parity of the staged paths, then fib256, C2 and the 256 MiB halves
# block over the libraries (ab/<name>.so, "tree" = in-tree build).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r06s}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "staged or dc3 or lcp or fib or ansv" > $out/pytest.log 2>&1 &&
LIBS="${FIBLIBS:-base tree}" bash tools/ab_libs.sh 2 --workload fib256 --no-pmc --no-e2e > $out/ab_fib.txt 2>&1 &&
LIBS="${C2LIBS:-base tree}" bash tools/ab_libs.sh 2 --no-pmc --no-e2e > $out/ab_c2.txt 2>&1 &&
for v in ${HALVESLIBS:-base tree}; do
  if [ $v = tree ]; then unset SALZ_LIB_PATH; else export SALZ_LIB_PATH=$PWD/ab/$v.so; fi
  echo "== $v" >> $out/halves.txt
  timeout -k 10 200 python tools/stress_inputs.py --size 268435456 --cases halves --stages >> $out/halves.txt 2>&1 || exit 1
done
rc=$?
tail -3 $out/pytest.log; cat $out/ab_fib.txt $out/ab_c2.txt; cut -c1-300 $out/halves.txt
exit $rc
