#!/bin/bash
# A/B/... timing on one GPU box over several libraries (ab/<name>.so; "tree" = the in-tree build),
# R rounds each, alternating:  LIBS="base tree stage" bash tools/ab_libs.sh [R] [bench.py args...]
R=${1:-3}; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in ${LIBS:-base tree}; do
    if [ $v = tree ]; then unset SALZ_LIB_PATH; else export SALZ_LIB_PATH=$PWD/ab/$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 "$@" > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab/$v$r.json'));s=d['stages_ms_last_block'];print('$v', d['value'], ' '.join(f'{k[3:]}={v:.2f}' for k,v in s.items()), d['roundtrip_ok'])"
  done
done
