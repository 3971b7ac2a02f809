#!/bin/bash
# A/B timing of environment settings on one GPU box: R rounds, each running the bench once per
# setting (a setting is a space-separated list of VAR=value, "-" for none).
#   R=3 ARGS="--kind mixed" bash tools/ab_env.sh "SALZ_SA=global" -
R=${R:-3}
mkdir -p gpurun_out/ab_env
for r in $(seq 1 $R); do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    envs=""; [ "$setting" != "-" ] && envs="$setting"
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 3 $ARGS > gpurun_out/ab_env/$k.$r.json 2> gpurun_out/ab_env/$k.$r.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_env/$k.$r.json'));s=d['stages_ms_last_block'];print('$setting', d['value'], ' '.join(f'{k[3:]}={v:.2f}' for k,v in s.items()), d['roundtrip_ok'])"
  done
done
