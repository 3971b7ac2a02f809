#!/bin/bash
# A/B/C... timing on one GPU box: alternate the default bench over several library builds.
#   bash tools/ab_multi.sh R lib1.so lib2.so ... [-- extra bench.py args]
R=$1; shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out/abm
for r in $(seq 1 $R); do
  for lib in "${libs[@]}"; do
    v=$(basename $lib .so)
    SALZ_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 3 "$@" > gpurun_out/abm/$v$r.json 2> gpurun_out/abm/$v$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abm/$v$r.json'));s=d['stages_ms_last_block'];print('$v', d['value'], ' '.join(f'{k[3:]}={v:.2f}' for k,v in s.items()), d['roundtrip_ok'])"
  done
done
